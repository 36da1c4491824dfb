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
#include "gemm_internal.hpp"

namespace {

constexpr int NCH = 8, DEPTH = 3;

// KS = wave groups splitting the K-steps inside the workgroup (4 waves each): group kg takes
// K-steps kg, kg+KS, ...; the partial accumulators are summed through LDS at the end.  KS = 2
// doubles the waves per SIMD for the small-M (batch-1) GEMMs without any global reduction.
template <typename T, bool CONV, int BM, int BN, int KS>
__global__ __launch_bounds__(256 * KS) void gemm_kernel(const mmt_gemm_params p) {
    constexpr int EPC = 16 / (int)sizeof(T);
    constexpr int KT = NCH * EPC;
    constexpr int AR = BM / 32, BR = BN / 32;  // staged 16-B chunks per thread per K-step
    constexpr int WM = BM / 2, WN = BN / 2, MT = WM / 16, NTL = WN / 16;
    __shared__ u32x4 lds[2][KS][(BM + BN) * NCH];

    // XCD-aware bijective remap (workgroups are dealt round-robin over the 8 XCDs): give each XCD
    // a contiguous run of (tile, group) ids, tm fastest, so the W column-slices and A rows a run
    // re-reads stay in that XCD's L2.  Placement only changes speed, never results.
    const int nwg = gridDim.x * gridDim.z;
    const int orig = blockIdx.x + gridDim.x * blockIdx.z;
    const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
    const int g = lin / gridDim.x, tile = lin - g * gridDim.x;
    const int tiles_m = (p.M + BM - 1) / BM;
    const int tm = tile % tiles_m, tn = tile / tiles_m;
    const int m0 = tm * BM, n0 = tn * BN;
    const int lane = threadIdx.x & 63, kg = threadIdx.x >> 8;
    const int tid = threadIdx.x & 255, wid = tid >> 6;  // thread / wave within the k-group
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
        const int mr = m0 + (tid >> 3) + 32 * i;
        aval[i] = mr < M;
        const int m = aval[i] ? mr : M - 1;  // clamped: always a valid address
        if (!CONV) {
            const int64_t seg = m / p.a_seg_rows;
            aoff[i] = (seg % p.a_segs_a) * p.a_stride_a + (seg / p.a_segs_a) * p.a_stride_b + (m % p.a_seg_rows) * p.lda;
            ay[i] = ax[i] = 0;
        } else {
            const int hw = ch * ch;
            const int b = m / hw, rem = m - b * hw;
            ay[i] = rem / ch;
            ax[i] = rem - ay[i] * ch;
            aoff[i] = (int64_t)b * (p.a_stride_a > 0 ? p.a_stride_a : (int64_t)hi * hi);  // image pitch (pixels)
        }
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
        const int n = n0 + (tid >> 3) + 32 * i;
        bval[i] = n < N;
        boff[i] = (int64_t)(bval[i] ? n : N - 1) * K;
    }

    // Loads are never predicated: out-of-range rows / K-columns / padding taps read a clamped,
    // in-bounds address and are zeroed when written to LDS.  (A guarded load becomes an
    // s_and_saveexec branch and hipcc then drains vmcnt(0) before every barrier, which serialises
    // the whole prefetch ring.)  The ring's three stages are plain named register arrays: a stage
    // struct passed by reference is demoted to scratch by hipcc.
#define MMT_LOAD_TILE(KTV, SA, SB, SOK)                                                                  \
    {                                                                                                    \
        const int kraw_ = (KTV) * KT + c * EPC;                                                          \
        const bool kin_ = kraw_ < K;                                                                     \
        const int k_ = kin_ ? kraw_ : 0;                                                                 \
        int iyd_ = 0, ixd_ = 0, ci_ = k_;                                                                \
        if (CONV && p.conv_k3) {                                                                         \
            int tap_ = k_ / p.conv_cin;                                                                  \
            ci_ = k_ - tap_ * p.conv_cin;                                                                \
            if (p.conv_k3 == 2) tap_ = 8 - tap_; /* flipped taps */                                      \
            iyd_ = tap_ / 3 - 1;                                                                         \
            ixd_ = tap_ % 3 - 1;                                                                         \
        }                                                                                                \
        uint32_t ok_ = 0;                                                                                \
        _Pragma("unroll") for (int i = 0; i < AR; ++i) {                                                 \
            bool v_ = aval[i] && kin_;                                                                   \
            const T* src_;                                                                               \
            if (!CONV) {                                                                                 \
                const bool hp_ = p.k_split > 0 && k_ >= p.k_split;                                      \
                src_ = (hp_ ? A1 : A0) + aoff[i] + (hp_ ? k_ - p.k_split : k_);                          \
            } else {                                                                                     \
                int iy_ = ay[i] + iyd_, ix_ = ax[i] + ixd_;                                              \
                v_ = v_ && iy_ >= 0 && ix_ >= 0 && iy_ < ch && ix_ < ch;                                 \
                iy_ = min(max(iy_, 0), ch - 1);                                                          \
                ix_ = min(max(ix_, 0), ch - 1);                                                          \
                src_ = A0 + (aoff[i] + (int64_t)(iy_ / cup) * hi + (ix_ / cup)) * p.lda + ci_;            \
            }                                                                                            \
            SA[i] = *(const u32x4*)src_;                                                                 \
            ok_ |= (uint32_t)v_ << i;                                                                    \
        }                                                                                                \
        _Pragma("unroll") for (int i = 0; i < BR; ++i) {                                                 \
            SB[i] = *(const u32x4*)(W + boff[i] + k_);                                                   \
            ok_ |= (uint32_t)(bval[i] && kin_) << (AR + i);                                              \
        }                                                                                                \
        SOK = ok_;                                                                                       \
    }
#define MMT_STORE_TILE(BUF, SA, SB, SOK)                                                                 \
    {                                                                                                    \
        const u32x4 z_ = {0u, 0u, 0u, 0u};                                                               \
        _Pragma("unroll") for (int i = 0; i < AR; ++i) {                                                 \
            const int row_ = (tid >> 3) + 32 * i;                                                        \
            lds[BUF][kg][row_ * NCH + (c ^ (row_ & 7))] = (((SOK) >> i) & 1) ? SA[i] : z_;               \
        }                                                                                                \
        _Pragma("unroll") for (int i = 0; i < BR; ++i) {                                                 \
            const int row_ = (tid >> 3) + 32 * i;                                                        \
            lds[BUF][kg][(BM + row_) * NCH + (c ^ (row_ & 7))] = (((SOK) >> (AR + i)) & 1) ? SB[i] : z_; \
        }                                                                                                \
    }

    f32x4 acc[MT][NTL];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NTL; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto compute = [&](int buf) {
        const u32x4* L = lds[buf][kg];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int sw = (4 * t + lg) ^ (lane & 7);
            u32x4 af[MT], bfr[NTL];
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) af[mt] = L[(wr * WM + mt * 16 + l16) * NCH + sw];
#pragma unroll
            for (int nt = 0; nt < NTL; ++nt) bfr[nt] = L[(BM + wc * WN + nt * 16 + l16) * NCH + sw];
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int nt = 0; nt < NTL; ++nt) {
                    if constexpr (sizeof(T) == 2) {
                        acc[mt][nt] = mfma16x16x32<T>(af[mt], bfr[nt], acc[mt][nt]);
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
    // Three named stages; the tail issues clamped re-loads of the last K-step instead of branching
    // around the loads.
    // Step s covers K-steps s*KS .. s*KS+KS-1 (one per k-group); K-steps past the end load a
    // clamped address and are masked to zero.
    const int nk = (K + KT - 1) / KT;
    const int ns = (nk + KS - 1) / KS;
    static_assert(DEPTH == 3, "ring is written out for three stages");
    u32x4 sa0[AR], sb0[BR], sa1[AR], sb1[BR], sa2[AR], sb2[BR];
    uint32_t ok0, ok1, ok2;
    MMT_LOAD_TILE(kg, sa0, sb0, ok0);
    MMT_LOAD_TILE(min(1, ns - 1) * KS + kg, sa1, sb1, ok1);
    MMT_LOAD_TILE(min(2, ns - 1) * KS + kg, sa2, sb2, ok2);
#define MMT_STEP(SV, SA, SB, SOK)                                        \
    {                                                                    \
        MMT_STORE_TILE((SV) & 1, SA, SB, SOK);                           \
        lds_barrier();                                                   \
        MMT_LOAD_TILE(min((SV) + DEPTH, ns - 1) * KS + kg, SA, SB, SOK); \
        compute((SV) & 1);                                               \
    }
    int st = 0;
    for (; st + DEPTH <= ns; st += DEPTH) {
        MMT_STEP(st, sa0, sb0, ok0);
        MMT_STEP(st + 1, sa1, sb1, ok1);
        MMT_STEP(st + 2, sa2, sb2, ok2);
    }
    if (st < ns) MMT_STEP(st, sa0, sb0, ok0);
    if (st + 1 < ns) MMT_STEP(st + 1, sa1, sb1, ok1);
#undef MMT_STEP
#undef MMT_LOAD_TILE
#undef MMT_STORE_TILE

    if constexpr (KS > 1) {  // sum the k-groups' partial tiles through LDS
        static_assert(KS == 2, "k-group reduction written for two groups");
        static_assert((size_t)4 * MT * NTL * 64 * 16 <= sizeof(lds), "reduction buffer");
        __syncthreads();
        f32x4* red = (f32x4*)&lds[0][0][0];
        if (kg == 1) {
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int nt = 0; nt < NTL; ++nt) red[((wid * MT + mt) * NTL + nt) * 64 + lane] = acc[mt][nt];
        }
        __syncthreads();
        if (kg == 1) return;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int nt = 0; nt < NTL; ++nt) acc[mt][nt] += red[((wid * MT + mt) * NTL + nt) * 64 + lane];
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
                const int64_t cm = p.c_seg_rows > 0 ? (m / p.c_seg_rows) * p.c_seg_pitch + m % p.c_seg_rows : m;
                if (R) {
                    int64_t rr = cm;
                    if (p.r_mode == 1) rr = m % p.r_p0;
                    else if (p.r_mode == 2) {
                        const int hw = p.r_p0 * p.r_p0, b = m / hw, rem = m - b * hw;
                        const int y = rem / p.r_p0, x = rem - y * p.r_p0, hs = p.r_p0 / p.r_p1;
                        rr = (int64_t)b * hs * hs + (int64_t)(y / p.r_p1) * hs + (x / p.r_p1);
                    }
                    rv = p.r_t ? to_f<T>(((const T*)R)[rr * p.ldr + n]) : R[rr * p.ldr + n];
                }
                const int64_t off = (cm * p.ldc + n) * osz;
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
    const int nk64 = (p.K + 16 / (int)sizeof(T) * NCH - 1) / (16 / (int)sizeof(T) * NCH);
    // Large problems: 128x128 (best MFMA:LDS ratio).  Otherwise 64x64 to put work on every CU,
    // with two k-groups per tile when there are enough K-steps to share.
    if (blocks(128, 128) >= 512) {
        dim3 grid((unsigned)(blocks(128, 128) / p.groups), 1, p.groups);
        hipLaunchKernelGGL((gemm_kernel<T, CONV, 128, 128, 1>), grid, dim3(256), 0, st, p);
    } else if (nk64 >= 8) {
        dim3 grid((unsigned)(blocks(64, 64) / p.groups), 1, p.groups);
        hipLaunchKernelGGL((gemm_kernel<T, CONV, 64, 64, 2>), grid, dim3(512), 0, st, p);
    } else {
        dim3 grid((unsigned)(blocks(64, 64) / p.groups), 1, p.groups);
        hipLaunchKernelGGL((gemm_kernel<T, CONV, 64, 64, 1>), grid, dim3(256), 0, st, p);
    }
}

// GEMV path for a handful of rows (the score head's single-token Linears, M = batch; its 16 ROI tokens): one wave per
// output column n, lanes stride K with 16-B loads of the W row and the M activation rows, wave-sum,
// + bias, activation.  The tiled kernels would stream W through one K loop per 64-column tile (a few
// workgroups for the whole launch).  Plain fp32 GEMMs only: no residual / row maps / conv / split.
constexpr int GEMV_MAXM = 16;
__global__ __launch_bounds__(256) void gemv_f32_kernel(const float* __restrict__ a, const float* __restrict__ w,
                                                       const float* __restrict__ bias, float* __restrict__ c, int M,
                                                       int N, int K, int64_t lda, int64_t ldc, int act) {
    const int n = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (n >= N) return;  // wave-uniform
    const float* wr = w + (int64_t)n * K;
    float acc[GEMV_MAXM];
#pragma unroll
    for (int m = 0; m < GEMV_MAXM; ++m) acc[m] = 0.f;
    for (int k = lane * 4; k < K; k += 256) {
        const float4 wv = *(const float4*)(wr + k);
#pragma unroll
        for (int m = 0; m < GEMV_MAXM; ++m) {
            if (m < M) {
                const float4 av = *(const float4*)(a + m * lda + k);
                acc[m] = fmaf(wv.x, av.x, fmaf(wv.y, av.y, fmaf(wv.z, av.z, fmaf(wv.w, av.w, acc[m]))));
            }
        }
    }
#pragma unroll
    for (int m = 0; m < GEMV_MAXM; ++m) {
        if (m < M) {
            float v = wave_sum(acc[m]);
            if (lane == 0) {
                if (bias) v += bias[n];
                if (act == 1) v = gelu_erf(v);
                else if (act == 2) v = fmaxf(v, 0.f);
                c[m * ldc + n] = v;
            }
        }
    }
}

// Argument checks shared by mmt_gemm and mmt_gemm_multi: 0 or MMT_EBADARG.
template <typename T>
int check_gemm(const mmt_gemm_params& p) {
    const int EPC = 16 / (int)sizeof(T);
    if (p.M <= 0 || p.N <= 0 || p.K <= 0 || p.groups < 1 || p.groups > MMT_MAX_GROUPS) return MMT_EBADARG;
    if (p.impl < -1 || p.impl > 9) return MMT_EBADARG;
    if (p.act < 0 || (p.act > 2 && p.act != 5) || p.c2_copy < 0 || p.c2_copy > 4) return MMT_EBADARG;
    if (p.c2_copy == 4 && !p.c_f32) return MMT_EBADARG;
    if (p.K % EPC || p.lda % EPC) return MMT_EBADARG;
    if (p.conv_h > 0) {
        if (p.conv_cin % EPC || p.conv_up < 1 || p.conv_h % p.conv_up) return MMT_EBADARG;
        if (p.conv_k3 < 0 || p.conv_k3 > 2 || p.K != (p.conv_k3 ? 9 : 1) * p.conv_cin) return MMT_EBADARG;
        if (p.M % (p.conv_h * p.conv_h)) return MMT_EBADARG;
    } else {
        if (p.a_seg_rows <= 0 || p.a_segs_a <= 0) return MMT_EBADARG;
        if (p.k_split % EPC || p.a_stride_a % EPC || p.a_stride_b % EPC) return MMT_EBADARG;
    }
    // MN-major operands (16-bit LDS-DMA kernels): W alone (w_t 1 / 2) or A and W (a_t 1), plain GEMM mode
    if (p.a_t < 0 || p.a_t > 1 || p.w_t < 0 || p.w_t > 2 || (p.a_t && !p.w_t)) return MMT_EBADARG;
    if (p.w_t) {
        if (sizeof(T) != 2 || p.conv_h > 0 || p.ln_fold || p.k_split || p.a_seg_rows < p.M) return MMT_EBADARG;
        if (p.N % 8 || p.ldw % EPC || p.ldw < (p.w_t == 2 ? p.N - 8 : p.N)) return MMT_EBADARG;
        if (p.a_t && (p.M % 8 || p.lda < p.M)) return MMT_EBADARG;
    }
    if (p.row_scale && p.row_scale_div < 1) return MMT_EBADARG;
    if (p.r_mode == 2 && (p.r_p1 < 1 || p.r_p0 % p.r_p1)) return MMT_EBADARG;
    if (p.r_mode == 1 && p.r_p0 < 1) return MMT_EBADARG;
    if (p.c_seg_rows < 0 || (p.c_seg_rows > 0 && (p.conv_h > 0 || p.c_seg_pitch < p.c_seg_rows))) return MMT_EBADARG;
    for (int g = 0; g < p.groups; ++g) {
        if (!p.a[g] || !p.w[g] || !p.c[g]) return MMT_EBADARG;
        if (((uintptr_t)p.a[g] | (uintptr_t)p.w[g]) & 15) return MMT_EBADARG;
        if (p.k_split > 0 && p.conv_h == 0 && (!p.a1[g] || ((uintptr_t)p.a1[g] & 15))) return MMT_EBADARG;
        if (p.c2[g] && !p.r[g] && p.c2_copy < 2) return MMT_EBADARG;
        if ((p.act == 5 && !p.r[g]) || (p.c2_copy >= 2 && !p.c2[g])) return MMT_EBADARG;
        if (p.c2_copy >= 3 && (p.N % 8 || p.ldc < p.N - 8)) return MMT_EBADARG;
        if (p.w_t && (((uintptr_t)p.w[g] & 15) || (p.a_t && ((uintptr_t)p.a[g] & 15)))) return MMT_EBADARG;
    }
    return 0;
}

template <typename T>
int launch_gemm(const mmt_gemm_params& p, hipStream_t st) {
    if (const int e = check_gemm<T>(p)) return e;
    if (sizeof(T) == 4 && p.M <= GEMV_MAXM && p.groups == 1 && p.conv_h == 0 && !p.r[0] && !p.c2[0] && p.c_f32 &&
        p.k_split == 0 && !p.ln_fold && p.splitk == 0 && p.c_seg_rows == 0 && p.a_seg_rows >= p.M && p.K % 4 == 0 &&
        p.lda % 4 == 0 && p.impl <= 0) {
        hipLaunchKernelGGL(gemv_f32_kernel, dim3((unsigned)((p.N + 3) / 4)), dim3(256), 0, st, (const float*)p.a[0],
                           (const float*)p.w[0], (const float*)p.bias[0], (float*)p.c[0], p.M, p.N, p.K, p.lda, p.ldc,
                           p.act);
        return launch_status();
    }
    if constexpr (sizeof(T) == 2)
        if (mmt_gemm_glds<T>(p, st, p.impl) == 0) return launch_status();
    if (p.ln_fold || p.c2_copy || p.act == 5 || p.w_t || p.row_scale) return MMT_EBADARG;  // LDS-DMA kernel features only
    if (p.conv_h > 0) launch_tiles<T, true>(p, st);
    else launch_tiles<T, false>(p, st);
    return launch_status();
}

// Independent problems in one launch when the LDS-DMA kernel takes them all in one configuration,
// else one launch each (same results up to the fp32 summation order of the chosen tile shapes).
template <typename T>
int launch_gemm_multi(const mmt_gemm_params* ps, int n, hipStream_t st) {
    if (n < 1 || n > 4) return MMT_EBADARG;
    for (int i = 0; i < n; ++i)
        if (const int e = check_gemm<T>(ps[i])) return e;
    if constexpr (sizeof(T) == 2)
        if (mmt_gemm_glds_multi<T>(ps, n, st) == 0) return launch_status();
    for (int i = 0; i < n; ++i)
        if (const int e = launch_gemm<T>(ps[i], st)) return e;
    return 0;
}

}  // namespace

extern "C" int mmt_gemm_multi(const mmt_gemm_params* ps, int n, int dtype, void* stream) {
    if (!ps) return MMT_EBADARG;
    if (dtype == MMT_BF16) return launch_gemm_multi<bf16_t>(ps, n, (hipStream_t)stream);
    if (dtype == MMT_F16) return launch_gemm_multi<f16_t>(ps, n, (hipStream_t)stream);
    if (dtype == MMT_F32) return launch_gemm_multi<float>(ps, n, (hipStream_t)stream);
    return MMT_EBADARG;
}

extern "C" int mmt_gemm(const mmt_gemm_params* p, int dtype, void* stream) {
    if (!p) return MMT_EBADARG;
    if (dtype == MMT_BF16) return launch_gemm<bf16_t>(*p, (hipStream_t)stream);
    if (dtype == MMT_F16) return launch_gemm<f16_t>(*p, (hipStream_t)stream);
    if (dtype == MMT_F32) return launch_gemm<float>(*p, (hipStream_t)stream);
    return MMT_EBADARG;
}
