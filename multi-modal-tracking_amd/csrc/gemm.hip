// MFMA GEMM / implicit-GEMM convolution for gfx950 with fused epilogues.
//
// Replaces every eager Linear / conv of the hot path (mixformer.py:26-76,137-138;
// fusion_utils.py:252-278; deformable_encoder_lnspecific.py:131-158; head.py:7-20,159-198;
// score_decoder.py:19-66).  One kernel body serves:
//   - plain / segmented-row / K-split GEMMs (qkv, proj, fc1, fc2, fusion 1x1 convs, [q_v|q_i] ...),
//   - NHWC implicit-GEMM 3x3 and 1x1 convolutions whose input is read through a nearest-upsample
//     index map (the pyramid head's F.interpolate + conv, never materialised),
//   - up to two independent "groups" (modalities / corner branches) per launch (blockIdx.z).
// Tiling: BMxBN output tile per 256-thread workgroup (4 waves, 2x2; 128x128 for large M, 64x64
// when the grid would not fill the 256 CUs, which is the batch-1 tracking case), K staged 128
// bytes per row per step (64 bf16 / 32 fp32) through a double-buffered XOR-swizzled LDS image.
// Global->LDS staging goes through a ring of DEPTH register sets: DEPTH K-steps of loads are in
// flight while the matrix cores work on the current one (the batch-1 GEMMs are latency-bound, not
// bandwidth-bound).  bf16 uses v_mfma_f32_16x16x32_bf16, fp32 the exact-f32 v_mfma_f32_16x16x4_f32.
// Epilogue: bias, GELU(erf)/ReLU, residual with a row map (identity, modulo, or down-sampled conv
// map; fp32 or compute dtype), optional second output (C2 = C + R).
#include "common.hpp"

namespace {

constexpr int NCH = 8, NT = 256, DEPTH = 3;

template <typename T, bool CONV, int BM, int BN>
__global__ __launch_bounds__(NT) void gemm_kernel(const mmt_gemm_params p) {
    constexpr int EPC = 16 / (int)sizeof(T);
    constexpr int KT = NCH * EPC;
    constexpr int AR = BM / 32, BR = BN / 32;  // staged 16-B chunks per thread per K-step
    constexpr int WM = BM / 2, WN = BN / 2, MT = WM / 16, NTL = WN / 16;
    __shared__ uint4 lds[2][(BM + BN) * NCH];

    const int g = blockIdx.z;
    const int tiles_m = (p.M + BM - 1) / BM;
    const int tm = blockIdx.x % tiles_m, tn = blockIdx.x / tiles_m;
    const int m0 = tm * BM, n0 = tn * BN;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wr = wid >> 1, wc = wid & 1;
    const int l16 = lane & 15, lg = lane >> 4;
    const int c = tid & 7;

    const T* A0 = (const T*)p.a[g];
    const T* A1 = (const T*)p.a1[g];
    const T* W = (const T*)p.w[g];
    const int M = p.M, N = p.N, K = p.K;

    int64_t aoff[AR], boff[BR];
    bool aval[AR], bval[BR];
    int ay[AR], ax[AR];
    const int ch = p.conv_h, cup = p.conv_up > 0 ? p.conv_up : 1, hi = CONV ? p.conv_h / cup : 0;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
        const int m = m0 + (tid >> 3) + 32 * i;
        aval[i] = m < M;
        if (!CONV) {
            const int64_t seg = m / p.a_seg_rows;
            aoff[i] = (seg % p.a_segs_a) * p.a_stride_a + (seg / p.a_segs_a) * p.a_stride_b + (m % p.a_seg_rows) * p.lda;
            ay[i] = ax[i] = 0;
        } else {
            const int hw = ch * ch;
            const int b = m / hw, rem = m - b * hw;
            ay[i] = rem / ch;
            ax[i] = rem - ay[i] * ch;
            aoff[i] = (int64_t)b * hi * hi;
        }
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
        const int n = n0 + (tid >> 3) + 32 * i;
        bval[i] = n < N;
        boff[i] = (int64_t)n * K;
    }

    struct Stage {
        uint4 a[AR], b[BR];
    };
    auto load_tile = [&](int kt, Stage& s) {
        const int k = kt * KT + c * EPC;
        const bool kin = k < K;
        int iy_d = 0, ix_d = 0, ci = k;
        if (CONV && p.conv_k3) {
            const int tap = k / p.conv_cin;
            ci = k - tap * p.conv_cin;
            iy_d = tap / 3 - 1;
            ix_d = tap % 3 - 1;
        }
#pragma unroll
        for (int i = 0; i < AR; ++i) {
            uint4 v = make_uint4(0, 0, 0, 0);
            if (aval[i] && kin) {
                if (!CONV) {
                    const T* src = (p.k_split > 0 && k >= p.k_split) ? A1 + aoff[i] + (k - p.k_split) : A0 + aoff[i] + k;
                    v = *(const uint4*)src;
                } else {
                    const int iy = ay[i] + iy_d, ix = ax[i] + ix_d;
                    if (iy >= 0 && ix >= 0 && iy < ch && ix < ch) {
                        const int64_t pix = aoff[i] + (int64_t)(iy / cup) * hi + (ix / cup);
                        v = *(const uint4*)(A0 + pix * p.lda + ci);
                    }
                }
            }
            s.a[i] = v;
        }
#pragma unroll
        for (int i = 0; i < BR; ++i) {
            uint4 w = make_uint4(0, 0, 0, 0);
            if (bval[i] && kin) w = *(const uint4*)(W + boff[i] + k);
            s.b[i] = w;
        }
    };
    auto store_tile = [&](int buf, const Stage& s) {
#pragma unroll
        for (int i = 0; i < AR; ++i) {
            const int row = (tid >> 3) + 32 * i;
            lds[buf][row * NCH + (c ^ (row & 7))] = s.a[i];
        }
#pragma unroll
        for (int i = 0; i < BR; ++i) {
            const int row = (tid >> 3) + 32 * i;
            lds[buf][(BM + row) * NCH + (c ^ (row & 7))] = s.b[i];
        }
    };

    f32x4 acc[MT][NTL];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NTL; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto compute = [&](int buf) {
        const uint4* L = lds[buf];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int sw = (4 * t + lg) ^ (lane & 7);
            uint4 af[MT], bfr[NTL];
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) af[mt] = L[(wr * WM + mt * 16 + l16) * NCH + sw];
#pragma unroll
            for (int nt = 0; nt < NTL; ++nt) bfr[nt] = L[(BM + wc * WN + nt * 16 + l16) * NCH + sw];
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int nt = 0; nt < NTL; ++nt) {
                    if constexpr (sizeof(T) == 2) {
                        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                            __builtin_bit_cast(bf16x8, af[mt]), __builtin_bit_cast(bf16x8, bfr[nt]), acc[mt][nt], 0, 0, 0);
                    } else {
                        const f32x4 a4 = __builtin_bit_cast(f32x4, af[mt]);
                        const f32x4 b4 = __builtin_bit_cast(f32x4, bfr[nt]);
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[j], b4[j], acc[mt][nt], 0, 0, 0);
                    }
                }
        }
    };

    // ---- K loop: ring of DEPTH register stages, double-buffered LDS, one barrier per K-step
    const int nk = (K + KT - 1) / KT;
    Stage st[DEPTH];
#pragma unroll
    for (int j = 0; j < DEPTH; ++j)
        if (j < nk) load_tile(j, st[j]);
    for (int k0 = 0; k0 < nk; k0 += DEPTH) {
#pragma unroll
        for (int j = 0; j < DEPTH; ++j) {
            const int kt = k0 + j;
            if (kt < nk) {
                store_tile(kt & 1, st[j]);
                __syncthreads();
                if (kt + DEPTH < nk) load_tile(kt + DEPTH, st[j]);
                compute(kt & 1);
            }
        }
    }

    // ---- epilogue
    const float* bias = p.bias[g];
    const float* R = p.r[g];
    char* C = (char*)p.c[g];
    char* C2 = (char*)p.c2[g];
    const int osz = p.c_f32 ? 4 : (int)sizeof(T);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NTL; ++nt) {
            const int n = n0 + wc * WN + nt * 16 + l16;
            if (n >= N) continue;
            const float bn = bias ? bias[n] : 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wr * WM + mt * 16 + lg * 4 + r;
                if (m >= M) continue;
                float v = acc[mt][nt][r] + bn;
                if (p.act == 1) v = gelu_erf(v);
                else if (p.act == 2) v = fmaxf(v, 0.f);
                float rv = 0.f;
                if (R) {
                    int64_t rr = m;
                    if (p.r_mode == 1) rr = m % p.r_p0;
                    else if (p.r_mode == 2) {
                        const int hw = p.r_p0 * p.r_p0, b = m / hw, rem = m - b * hw;
                        const int y = rem / p.r_p0, x = rem - y * p.r_p0, hs = p.r_p0 / p.r_p1;
                        rr = (int64_t)b * hs * hs + (int64_t)(y / p.r_p1) * hs + (x / p.r_p1);
                    }
                    rv = p.r_t ? to_f<T>(((const T*)R)[rr * p.ldr + n]) : R[rr * p.ldr + n];
                }
                const int64_t off = ((int64_t)m * p.ldc + n) * osz;
                const float out1 = C2 ? v : v + rv;
                if (p.c_f32) *(float*)(C + off) = out1;
                else *(T*)(C + off) = from_f<T>(out1);
                if (C2) {
                    if (p.c_f32) *(float*)(C2 + off) = v + rv;
                    else *(T*)(C2 + off) = from_f<T>(v + rv);
                }
            }
        }
}

template <typename T, bool CONV>
void launch_tiles(const mmt_gemm_params& p, hipStream_t st) {
    auto blocks = [&](int bm, int bn) { return (int64_t)((p.M + bm - 1) / bm) * ((p.N + bn - 1) / bn) * p.groups; };
    // Large problems: 128x128 (best MFMA:LDS ratio).  Otherwise 64x64 to put work on every CU.
    if (blocks(128, 128) >= 512) {
        dim3 grid((unsigned)(blocks(128, 128) / p.groups), 1, p.groups);
        hipLaunchKernelGGL((gemm_kernel<T, CONV, 128, 128>), grid, dim3(NT), 0, st, p);
    } else {
        dim3 grid((unsigned)(blocks(64, 64) / p.groups), 1, p.groups);
        hipLaunchKernelGGL((gemm_kernel<T, CONV, 64, 64>), grid, dim3(NT), 0, st, p);
    }
}

template <typename T>
int launch_gemm(const mmt_gemm_params& p, hipStream_t st) {
    const int EPC = 16 / (int)sizeof(T);
    if (p.M <= 0 || p.N <= 0 || p.K <= 0 || p.groups < 1 || p.groups > MMT_MAX_GROUPS) return MMT_EBADARG;
    if (p.K % EPC || p.lda % EPC) return MMT_EBADARG;
    if (p.conv_h > 0) {
        if (p.conv_cin % EPC || p.conv_up < 1 || p.conv_h % p.conv_up) return MMT_EBADARG;
        if (p.K != (p.conv_k3 ? 9 : 1) * p.conv_cin) return MMT_EBADARG;
        if (p.M % (p.conv_h * p.conv_h)) return MMT_EBADARG;
    } else {
        if (p.a_seg_rows <= 0 || p.a_segs_a <= 0) return MMT_EBADARG;
        if (p.k_split % EPC || p.a_stride_a % EPC || p.a_stride_b % EPC) return MMT_EBADARG;
    }
    if (p.r_mode == 2 && (p.r_p1 < 1 || p.r_p0 % p.r_p1)) return MMT_EBADARG;
    if (p.r_mode == 1 && p.r_p0 < 1) return MMT_EBADARG;
    for (int g = 0; g < p.groups; ++g) {
        if (!p.a[g] || !p.w[g] || !p.c[g]) return MMT_EBADARG;
        if (((uintptr_t)p.a[g] | (uintptr_t)p.w[g]) & 15) return MMT_EBADARG;
        if (p.k_split > 0 && p.conv_h == 0 && (!p.a1[g] || ((uintptr_t)p.a1[g] & 15))) return MMT_EBADARG;
        if (p.c2[g] && !p.r[g]) return MMT_EBADARG;
    }
    if (p.conv_h > 0) launch_tiles<T, true>(p, st);
    else launch_tiles<T, false>(p, st);
    return launch_status();
}

}  // namespace

extern "C" int mmt_gemm(const mmt_gemm_params* p, int dtype, void* stream) {
    if (!p) return MMT_EBADARG;
    if (dtype == MMT_BF16) return launch_gemm<bf16_t>(*p, (hipStream_t)stream);
    if (dtype == MMT_F32) return launch_gemm<float>(*p, (hipStream_t)stream);
    return MMT_EBADARG;
}
