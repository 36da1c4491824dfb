// Large-tile bf16 GEMM for gfx950 with LDS-DMA staging (global_load_lds_dwordx4).
//
// The batch-1 ViT GEMMs of the hot path (qkv / proj / fc1 / fc2 of mixformer.py:26-76, M = 2x528
// rows) were bound by per-CU tile traffic and staging instructions in the register-staged 64x64
// kernel (gemm.hip): PMC showed ~90 % L2 hits, 7x fewer HBM bytes than tile bytes, MFMA busy
// ~15 % of the wave lifetime and VALU (clamped-load address math + selects) 22x the MFMA count.
// This kernel cuts both:
//   - 128x128 (or 128x64 with two K-split wave groups) output tiles per workgroup: 2-4x fewer
//     L2->CU bytes per FLOP than 64x64, one workgroup per CU, 4 waves as 2x2 with 64x64 / 64x32
//     wave tiles (the LDS-read : MFMA ratio of ds_read_b128 at 256 B/clk stays below 1);
//   - staging by global_load_lds_dwordx4: every wave-instruction lands one 1-KiB piece (8 rows x
//     128 B of the K-step) in LDS with no VGPR round trip.  The LDS image is lane-linear, so the
//     XOR swizzle that makes the fragment reads conflict-free (chunk c of row r at c ^ (r & 7)) is
//     applied on the per-lane SOURCE address and again on the read;
//   - an ST-deep ring of stage images with counted `s_waitcnt vmcnt` and a raw s_barrier, so up
//     to ST-1 K-steps stay in flight across the barrier (__syncthreads would drain vmcnt(0)).
// The MFMA is issued with the operands swapped (C^T = W A^T): each lane then holds 4 consecutive
// output columns of one row, so the epilogue stores 8-B (bf16) / 16-B (fp32) vectors and reads
// bias / residual as vectors.  Epilogue semantics are those of gemm.hip (include/mmt_hip.h).
// Rows past M / columns past N load clamped in-bounds rows (they only feed discarded outputs);
// K must be a multiple of 64, which holds for every GEMM this path routes here.
#include "common.hpp"
#include "gemm_internal.hpp"

// MMT_GEMM_ABLATE (measurement builds only, tools/build_ablate.sh): 1 = no DMA after the prologue
// (MFMA + LDS reads + barriers alone), 2 = no MFMA work (DMA pipeline alone).
#ifndef MMT_GEMM_ABLATE
#define MMT_GEMM_ABLATE 0
#endif

// MMT_GEMM_STAMP (measurement builds only, tools/build_ablate.sh): workgroup-leader timestamps
// per phase, read back with mmt_gemm_stamps() (tools/gemm_stamps.py).
#ifndef MMT_GEMM_STAMP
#define MMT_GEMM_STAMP 0
#endif
#if MMT_GEMM_STAMP
__device__ unsigned long long g_mmt_stamps[16384 * 6];
#define MMT_STAMP(I, INSN)                                                                          \
    if (threadIdx.x == 0) {                                                                        \
        unsigned long long t_;                                                                     \
        asm volatile(INSN " %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                      \
        g_mmt_stamps[(blockIdx.x + gridDim.x * blockIdx.z) * 6 + (I)] = t_;                        \
    }
extern "C" int mmt_gemm_stamps(unsigned long long* host, int n) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_mmt_stamps), sizeof(unsigned long long) * n);
}
#else
#define MMT_STAMP(I, INSN)
#endif

namespace {

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

template <int N>
MMT_DEV void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

MMT_DEV void glds16(const void* src, unsigned char* dst) {
    __builtin_amdgcn_global_load_lds((glb_void*)src, (lds_void*)dst, 16, 0, 0);
}

// Wait until at most `ahead` stages of this wave's DMA are still outstanding (L per stage).
template <int L, int ST>
MMT_DEV void wait_stages(int ahead) {
    static_assert(ST <= 4, "wait table written for ST <= 4");
    if (ahead <= 0) wait_vm<0>();
    else if (ahead == 1) wait_vm<L>();
    else if (ahead == 2 || ST < 4) wait_vm<(ST >= 3 ? 2 * L : L)>();
    else wait_vm<(ST >= 4 ? 3 * L : L)>();
}

template <int BM, int BN, int KS, int ST>
__global__ __launch_bounds__(256 * KS) __attribute__((amdgpu_waves_per_eu(KS, KS))) void gemm_glds_kernel(const mmt_gemm_params p) {
    constexpr int KT = 64;                    // bf16 elements of K per step: 128-B rows
    constexpr int STAGE = (BM + BN) * 128;    // bytes of one stage image (A rows, then W rows)
    constexpr int PA = BM / 32, PB = BN / 32; // 1-KiB pieces per wave per stage (4 waves)
    constexpr int L = PA + PB;                // DMA instructions per wave per stage
    constexpr int WM = BM / 2, WN = BN / 2, MT = WM / 16, NT = WN / 16;
    static_assert(KS * ST * STAGE <= 160 * 1024, "LDS budget");
    static_assert(KS == 1 || BM * BN * 4 <= KS * ST * STAGE, "k-group reduction buffer");
    __shared__ __attribute__((aligned(1024))) unsigned char lds[KS * ST * STAGE];
    MMT_STAMP(0, "s_memrealtime");
    MMT_STAMP(1, "s_memtime");

    // XCD-aware bijective remap (see gemm.hip): each XCD gets a contiguous run of (group, tile)
    // ids, tm fastest, so a run's W column slices and A rows stay in that XCD's L2.
    const int nwg = gridDim.x * gridDim.z;
    const int orig = blockIdx.x + gridDim.x * blockIdx.z;
    const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
    const int g = lin / gridDim.x, tile = lin - g * gridDim.x;
    const int tiles_m = (p.M + BM - 1) / BM;
    const int tm = tile % tiles_m, tn = tile / tiles_m;
    const int m0 = tm * BM, n0 = tn * BN;
    const int lane = threadIdx.x & 63, kg = threadIdx.x >> 8;
    const int wid = (threadIdx.x & 255) >> 6, wr = wid >> 1, wc = wid & 1;
    const int l16 = lane & 15, lg = lane >> 4;
    const int M = p.M, N = p.N, K = p.K;

    const bf16_t* A0 = (const bf16_t*)p.a[g];
    const bf16_t* A1 = (const bf16_t*)p.a1[g];
    const bf16_t* W = (const bf16_t*)p.w[g];

    // This lane stages row (piece*8 + prow), logical chunk pch, into byte 16*lane of the piece:
    // position (lane & 7) of row prow holds chunk (lane & 7) ^ prow  (the read-side XOR).
    const int prow = lane >> 3, pch = (lane & 7) ^ prow;
    int64_t aoff[PA], boff[PB];
    const int segr = (int)p.a_seg_rows, sega = (int)p.a_segs_a;
#pragma unroll
    for (int i = 0; i < PA; ++i) {
        const int m = min(m0 + (wid * PA + i) * 8 + prow, M - 1);
        const int seg = m / segr, sa = seg % sega;  // 32-bit: the launcher checks the ranges
        aoff[i] = sa * p.a_stride_a + (int64_t)((seg - sa) / sega) * p.a_stride_b + (int64_t)(m - seg * segr) * p.lda +
                  pch * 8;
    }
#pragma unroll
    for (int i = 0; i < PB; ++i) boff[i] = (int64_t)min(n0 + (wid * PB + i) * 8 + prow, N - 1) * K + pch * 8;
    const int ks = p.k_split;

    unsigned char* ring = lds + kg * ST * STAGE;
    const int nk = K / KT, ns = (nk + KS - 1) / KS;

    auto issue = [&](int s) {  // this k-group's step s -> ring slot s % ST
        const int k0 = min(s * KS + kg, nk - 1) * KT;
        unsigned char* base = ring + (s % ST) * STAGE;
        const bool hp = ks > 0 && k0 + pch * 8 >= ks;
        const bf16_t* ab = hp ? A1 - ks : A0;
#pragma unroll
        for (int i = 0; i < PA; ++i) glds16(ab + aoff[i] + k0, base + (wid * PA + i) * 1024);
#pragma unroll
        for (int i = 0; i < PB; ++i) glds16(W + boff[i] + k0, base + BM * 128 + (wid * PB + i) * 1024);
    };

    f32x4 acc[NT][MT];  // acc[nt][mt] = (C^T) fragment: rows n, columns m
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int j = 0; j < MT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // Fragments of one K-step: [t][*] = the two 32-deep halves of the 64-deep step.
#define MMT_READ(BUF, AF, BF)                                                                                    \
    {                                                                                                            \
        const unsigned char* b_ = (BUF);                                                                         \
        _Pragma("unroll") for (int t = 0; t < 2; ++t) {                                                          \
            const int sw_ = (4 * t + lg) ^ (lane & 7);                                                           \
            _Pragma("unroll") for (int mt = 0; mt < MT; ++mt) AF[t][mt] =                                        \
                *(const u32x4*)(b_ + ((wr * WM + mt * 16 + l16) * 8 + sw_) * 16);                                \
            _Pragma("unroll") for (int nt = 0; nt < NT; ++nt) BF[t][nt] =                                        \
                *(const u32x4*)(b_ + BM * 128 + ((wc * WN + nt * 16 + l16) * 8 + sw_) * 16);                     \
        }                                                                                                        \
        __builtin_amdgcn_sched_barrier(0); /* all reads issue before the MFMAs that hide them */                 \
    }
#define MMT_MMA(AF, BF)                                                                                          \
    {                                                                                                            \
        if (MMT_GEMM_ABLATE == 2) {                                                                              \
            acc[0][0] += __builtin_bit_cast(f32x4, AF[0][0]) + __builtin_bit_cast(f32x4, BF[1][NT - 1]);         \
        } else {                                                                                                 \
            _Pragma("unroll") for (int t = 0; t < 2; ++t)                                                        \
            _Pragma("unroll") for (int nt = 0; nt < NT; ++nt)                                                    \
            _Pragma("unroll") for (int mt = 0; mt < MT; ++mt) acc[nt][mt] =                                      \
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, BF[t][nt]),                   \
                                                        __builtin_bit_cast(bf16x8, AF[t][mt]), acc[nt][mt], 0, 0, 0); \
        }                                                                                                        \
    }

    // ---- K loop.  Step j's fragments are read into registers right after the barrier that
    // publishes step j, and step j-1's MFMAs run while those reads are in flight (two register
    // sets, loop unrolled by 2 so both are statically named).  The barrier also proves every wave
    // has finished reading slot (j-1) % ST, which the DMA of step j+ST-1 then refills: ST-1
    // K-steps of DMA stay in flight behind the one being multiplied.
    auto sync_for = [&](int j) {
        // stages issued after j that may stay in flight while j is consumed
        if (MMT_GEMM_ABLATE != 1) wait_stages<L, ST>(min(ns - 1, j + ST - 2) - j);
        lds_barrier();
        if (MMT_GEMM_ABLATE != 1 && j + ST - 1 < ns) issue(j + ST - 1);
    };
    u32x4 fa0[2][MT], fb0[2][NT], fa1[2][MT], fb1[2][NT];
    for (int j = 0; j < ST - 1 && j < ns; ++j) issue(j);
    if (MMT_GEMM_ABLATE == 1) wait_vm<0>();
    sync_for(0);
    MMT_STAMP(2, "s_memtime");
    MMT_READ(ring, fa0, fb0);
    // Every k-group has a real K-step at j < ns-1; only the last can be empty (KS = 2 with an odd
    // step count).  Keeping that test out of the loop keeps the accumulators in place (a
    // conditional MFMA block inside the loop made hipcc shuttle them through VGPRs every step).
    int s = 0;
    for (; s + 2 < ns; s += 2) {
        sync_for(s + 1);
        MMT_READ(ring + ((s + 1) % ST) * STAGE, fa1, fb1);
        MMT_MMA(fa0, fb0);
        sync_for(s + 2);
        MMT_READ(ring + ((s + 2) % ST) * STAGE, fa0, fb0);
        MMT_MMA(fa1, fb1);
    }
    const bool last_ok = KS == 1 || (ns - 1) * KS + kg < nk;
    if (s + 1 < ns) {
        sync_for(s + 1);
        MMT_READ(ring + ((s + 1) % ST) * STAGE, fa1, fb1);
        MMT_MMA(fa0, fb0);
        if (last_ok) MMT_MMA(fa1, fb1);
    } else if (last_ok) {
        MMT_MMA(fa0, fb0);
    }
#undef MMT_READ
#undef MMT_MMA
    MMT_STAMP(3, "s_memtime");

    if constexpr (KS > 1) {  // sum the k-groups' partial tiles through LDS
        static_assert(KS == 2, "k-group reduction written for two groups");
        lds_barrier();
        f32x4* red = (f32x4*)lds;
        if (kg == 1) {
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) red[((wid * NT + nt) * MT + mt) * 64 + lane] = acc[nt][mt];
        }
        lds_barrier();
        if (kg == 1) return;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) acc[nt][mt] += red[((wid * NT + nt) * MT + mt) * 64 + lane];
    }

    // ---- epilogue: 4 consecutive columns per lane.  Bias / residual loads are issued first and
    // unconditionally (clamped row / column); only the stores are predicated.  (Loads inside a
    // lane-divergent guard make hipcc wait vmcnt(0) per fragment: MT*NT serial round trips.)
    const float* bias = p.bias[g];
    const float* R = p.r[g];
    char* C = (char*)p.c[g];
    char* C2 = (char*)p.c2[g];
    int nc[NT];
    f32x4 bn[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        nc[nt] = min(n0 + wc * WN + nt * 16 + lg * 4, N - 4);
        bn[nt] = bias ? *(const f32x4*)(bias + nc[nt]) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    int64_t rbase[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int m = min(m0 + wr * WM + mt * 16 + l16, M - 1);
        int64_t rr = m;
        if (p.r_mode == 1) rr = m % p.r_p0;
        else if (p.r_mode == 2) {
            const int hw = p.r_p0 * p.r_p0, b = m / hw, rem = m - b * hw;
            const int y = rem / p.r_p0, x = rem - y * p.r_p0, hs = p.r_p0 / p.r_p1;
            rr = (int64_t)b * hs * hs + (int64_t)(y / p.r_p1) * hs + (x / p.r_p1);
        }
        rbase[mt] = rr * p.ldr;
    }
    f32x4 rv[NT][MT];  // every residual load in flight at once: one round trip, not NT
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            rv[nt][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (R) {  // wave-uniform
                if (p.r_t) {
                    const uint2 u = *(const uint2*)((const bf16_t*)R + rbase[mt] + nc[nt]);
                    rv[nt][mt] = f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                                       __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u)};
                } else {
                    rv[nt][mt] = *(const f32x4*)(R + rbase[mt] + nc[nt]);
                }
            }
        }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int n = n0 + wc * WN + nt * 16 + lg * 4;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            const int m = m0 + wr * WM + mt * 16 + l16;
            f32x4 v = acc[nt][mt] + bn[nt];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (p.act == 1) v[j] = gelu_erf(v[j]);
                else if (p.act == 2) v[j] = fmaxf(v[j], 0.f);
            }
            const f32x4 o1 = C2 ? v : v + rv[nt][mt];
            const f32x4 o2 = v + rv[nt][mt];
            if (m < M && n < N) {
                const int64_t e = (int64_t)m * p.ldc + n;
                if (p.c_f32) {
                    *(f32x4*)((float*)C + e) = o1;
                    if (C2) *(f32x4*)((float*)C2 + e) = o2;
                } else {
                    *(uint2*)((bf16_t*)C + e) = make_uint2(pack_bf16x2(o1[0], o1[1]), pack_bf16x2(o1[2], o1[3]));
                    if (C2) *(uint2*)((bf16_t*)C2 + e) = make_uint2(pack_bf16x2(o2[0], o2[1]), pack_bf16x2(o2[2], o2[3]));
                }
            }
        }
    }
#if MMT_GEMM_STAMP
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    MMT_STAMP(4, "s_memtime");
    MMT_STAMP(5, "s_memrealtime");
}

template <int BM, int BN, int KS, int ST>
void launch(const mmt_gemm_params& p, hipStream_t st) {
    const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
    hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, KS, ST>), dim3(tiles, 1, p.groups), dim3(256 * KS), 0, st, p);
}

bool aligned(const void* ptr, int bytes) { return ((uintptr_t)ptr & (uintptr_t)(bytes - 1)) == 0; }

}  // namespace

// Returns 1 when the shape / layout is not one this kernel takes (caller uses gemm.hip's kernel).
int mmt_gemm_glds_bf16(const mmt_gemm_params& p, hipStream_t st, int force) {
    if (force < 0) return 1;
    if (p.conv_h > 0 || p.K % 64 || p.N % 4 || p.ldc % 4 || (p.r[0] && p.ldr % 4)) return 1;
    if (p.lda % 8 || p.a_stride_a % 8 || p.a_stride_b % 8 || p.k_split % 8) return 1;
    if (p.a_seg_rows > INT32_MAX || p.a_segs_a > INT32_MAX) return 1;
    for (int g = 0; g < p.groups; ++g) {
        const int cb = p.c_f32 ? 16 : 8;
        if (!aligned(p.c[g], cb) || (p.c2[g] && !aligned(p.c2[g], cb))) return 1;
        if (p.bias[g] && !aligned(p.bias[g], 16)) return 1;
        if (p.r[g] && !aligned(p.r[g], p.r_t ? 8 : 16)) return 1;
    }
    auto blocks = [&](int bm, int bn) { return (int64_t)((p.M + bm - 1) / bm) * ((p.N + bn - 1) / bn) * p.groups; };
    const int nk = p.K / 64;
    int cfg = force;
    if (cfg == 0) {
        if (blocks(128, 128) >= 128) cfg = 1;
        else if (blocks(128, 64) >= 64 && nk >= 4) cfg = 2;
        else if (nk >= 4) cfg = 3;
        else return 1;
    }
    switch (cfg) {
        case 1: launch<128, 128, 1, 4>(p, st); break;
        case 2: launch<128, 64, 2, 3>(p, st); break;
        case 3: launch<64, 64, 2, 4>(p, st); break;
        default: return 1;
    }
    return 0;
}
