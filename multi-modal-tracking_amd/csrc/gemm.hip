// MFMA GEMM / implicit-GEMM convolution for gfx950 with fused epilogues.
//
// Replaces every eager Linear / conv of the hot path (mixformer.py:26-76,137-138;
// fusion_utils.py:252-278; deformable_encoder_lnspecific.py:131-158; head.py:7-20,159-198;
// score_decoder.py:19-66).  One kernel body serves:
//   - plain / segmented-row / K-split GEMMs (qkv, proj, fc1, fc2, fusion 1x1 convs, [q_v|q_i] ...),
//   - NHWC implicit-GEMM 3x3 and 1x1 convolutions whose input is read through a nearest-upsample
//     index map (the pyramid head's F.interpolate + conv, never materialised),
//   - up to two independent "groups" (modalities / corner branches) per launch (blockIdx.z).
// Tiling: 128x128 output tile per 256-thread workgroup (4 waves, 2x2, 64x64 per wave as 4x4
// 16x16 MFMA tiles), K staged 128 bytes per row per step (64 bf16 / 32 fp32) through a
// double-buffered, XOR-swizzled LDS image (register staging: global loads for step k+1 are in
// flight while step k runs on the matrix cores).  bf16 uses v_mfma_f32_16x16x32_bf16, fp32 uses
// the exact-f32 v_mfma_f32_16x16x4_f32.  Epilogue: bias, GELU(erf)/ReLU, fp32 residual with a
// row map (identity, modulo, or down-sampled conv map), optional second output.
#include "common.hpp"

namespace {

constexpr int BM = 128, BN = 128, NCH = 8, NT = 256;

struct ConvGeom {
    int h, up, cin, k3;
};

template <typename T, bool CONV>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(const mmt_gemm_params p) {
    constexpr int EPC = 16 / (int)sizeof(T);
    constexpr int KT = NCH * EPC;
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

    int64_t aoff[4], boff[4];
    bool aval[4], bval[4];
    int ay[4], ax[4];
    const int ch = p.conv_h, cup = p.conv_up > 0 ? p.conv_up : 1, hi = CONV ? p.conv_h / cup : 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = (tid >> 3) + 32 * i;
        const int m = m0 + row;
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
        const int n = n0 + row;
        bval[i] = n < N;
        boff[i] = (int64_t)n * K;
    }

    uint4 ra[4], rb[4];
    auto load_tile = [&](int kt) {
        const int k = kt * KT + c * EPC;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint4 v = make_uint4(0, 0, 0, 0);
            if (aval[i] && k < K) {
                if (!CONV) {
                    const T* src = (p.k_split > 0 && k >= p.k_split) ? A1 + aoff[i] + (k - p.k_split) : A0 + aoff[i] + k;
                    v = *(const uint4*)src;
                } else {
                    int iy = ay[i], ix = ax[i], ci = k;
                    if (p.conv_k3) {
                        const int tap = k / p.conv_cin;
                        ci = k - tap * p.conv_cin;
                        iy += tap / 3 - 1;
                        ix += tap % 3 - 1;
                    }
                    if (iy >= 0 && ix >= 0 && iy < ch && ix < ch) {
                        const int64_t pix = aoff[i] + (int64_t)(iy / cup) * hi + (ix / cup);
                        v = *(const uint4*)(A0 + pix * p.lda + ci);
                    }
                }
            }
            ra[i] = v;
            uint4 w = make_uint4(0, 0, 0, 0);
            if (bval[i] && k < K) w = *(const uint4*)(W + boff[i] + k);
            rb[i] = w;
        }
    };
    auto store_tile = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = (tid >> 3) + 32 * i;
            lds[buf][row * NCH + (c ^ (row & 7))] = ra[i];
            lds[buf][(BM + row) * NCH + (c ^ (row & 7))] = rb[i];
        }
    };

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = (K + KT - 1) / KT;
    load_tile(0);
    store_tile(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) load_tile(kt + 1);
        const uint4* L = lds[cur];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int sw = (4 * t + lg) ^ (lane & 7);
            uint4 af[4], bfr[4];
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) af[mt] = L[(wr * 64 + mt * 16 + l16) * NCH + sw];
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) bfr[nt] = L[(BM + wc * 64 + nt * 16 + l16) * NCH + sw];
#pragma unroll
            for (int mt = 0; mt < 4; ++mt)
#pragma unroll
                for (int nt = 0; nt < 4; ++nt) {
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
        if (kt + 1 < nk) store_tile(cur ^ 1);
        __syncthreads();
    }

    // ---- epilogue
    const float* bias = p.bias[g];
    const float* R = p.r[g];
    char* C = (char*)p.c[g];
    char* C2 = (char*)p.c2[g];
    const int osz = p.c_f32 ? 4 : (int)sizeof(T);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
            const int n = n0 + wc * 64 + nt * 16 + l16;
            if (n >= N) continue;
            const float bn = bias ? bias[n] : 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wr * 64 + mt * 16 + lg * 4 + r;
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
    const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
    dim3 grid(tiles, 1, p.groups);
    if (p.conv_h > 0) hipLaunchKernelGGL((gemm_kernel<T, true>), grid, dim3(NT), 0, st, p);
    else hipLaunchKernelGGL((gemm_kernel<T, false>), grid, dim3(NT), 0, st, p);
    return launch_status();
}

}  // namespace

extern "C" int mmt_gemm(const mmt_gemm_params* p, int dtype, void* stream) {
    if (!p) return MMT_EBADARG;
    if (dtype == MMT_BF16) return launch_gemm<bf16_t>(*p, (hipStream_t)stream);
    if (dtype == MMT_F32) return launch_gemm<float>(*p, (hipStream_t)stream);
    return MMT_EBADARG;
}
