// Large-tile bf16 / fp16 GEMM for gfx950 with LDS-DMA staging (global_load_lds_dwordx4).
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

#include <algorithm>

// MMT_GEMM_ABLATE (measurement builds only, tools/build_ablate.sh): 3 = no epilogue C / C2 stores,
// 4 = no epilogue tile reads (constants instead); 1 = no DMA after the prologue
// (MFMA + LDS reads + barriers alone), 2 = no MFMA work (DMA pipeline alone).
#ifndef MMT_GEMM_ABLATE
#define MMT_GEMM_ABLATE 0
#endif
// A/B build knob: row tiles per row group of the large-grid tile order (below)
#ifndef MMT_GEMM_GM
#define MMT_GEMM_GM 8
#endif
// A/B build (tools/build_ablate.sh ab): 1 = also compile impl 9 (the 256x256 one-wave-per-SIMD tile; measured
// slower than the product's tiles with the fused epilogues)
#ifndef MMT_GEMM_AB
#define MMT_GEMM_AB 0
#endif
// A/B build knob (tools/build_ablate.sh occ2nores): 0 = the residual producers that hand LayerNorm statistics
// on (inference proj / fc2 with ln_stats_out) stay off impl 8, as before round 5
#ifndef MMT_GEMM_OCC2_RES
#define MMT_GEMM_OCC2_RES 1
#endif
// A/B build knob (tools/build_ablate.sh skticket): 1 = the ticket-first split-K hand-off (round 5, first half)
#ifndef MMT_GEMM_SK_TICKET_FIRST
#define MMT_GEMM_SK_TICKET_FIRST 0
#endif
// A/B build knob: the smallest weight-gradient grid (tiles x groups) that takes impl 8 with a K split (round 6);
// a large value restores the round-5 choice (impl 1 below 257 tiles, impl 8 unsplit above)
#ifndef MMT_GEMM_SK8_MIN
#define MMT_GEMM_SK8_MIN 64
#endif
// A/B build knob (tools/build_ablate.sh noocc2): 1 = the cost model never switches to impl 8
#ifndef MMT_GEMM_NO_OCC2
#define MMT_GEMM_NO_OCC2 0
#endif

// Stamp build (MMT_STAMP_BUILD): per-phase workgroup timestamps, read with mmt_gemm_stamps().
#if MMT_STAMP_BUILD
__device__ unsigned long long g_mmt_stamps[16384 * 8];
extern "C" int mmt_gemm_stamps(unsigned long long* host, int n) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_mmt_stamps), sizeof(unsigned long long) * n);
}
#endif
#define MMT_STAMP(I, INSN) MMT_STAMP_AT(g_mmt_stamps, I, INSN)

namespace {

template <int N>
struct gemm_ic {
    static constexpr int value = N;
};

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

// Zero source for A chunks outside the operand: conv padding taps and the K tail past K (a glds
// lane cannot zero its LDS bytes, so it loads zeros instead).
__device__ __attribute__((aligned(64))) const uint32_t g_zero_chunk[16] = {0};
// Ones column of the MN-major W operand (w_t 2): the chunk of columns N-8 .. N-1 is (1, 0, ..., 0) in
// every contraction row (bf16 / fp16 one in the low half of the first dword).
__device__ __attribute__((aligned(64))) const uint32_t g_one_chunk_bf16[4] = {0x3F80u, 0u, 0u, 0u};
__device__ __attribute__((aligned(64))) const uint32_t g_one_chunk_f16[4] = {0x3C00u, 0u, 0u, 0u};

// ds_read_b64_tr_b16 as inline asm (the builtin makes hipcc drain vmcnt(0), i.e. the whole DMA ring,
// before each read); the K loop orders the reads against their MFMAs itself (lds_barrier's lgkmcnt(0)
// or an explicit wait, then a register pin).
template <int OFF>
MMT_DEV uint2 gemm_tr16(const unsigned char* p) {
    uint2 r;
    const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) unsigned char*)p;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "n"(OFF));
    return r;
}

// MN-major operand images (mmt_gemm_params.a_t / w_t, LNM 3 / 4): the 64 contraction rows of a K-step
// as 256-B rows of 128 M (or N) elements; 16-B chunk c of row k stored at c ^ gemm_trsw(k), which
// makes the transposed fragment reads below conflict-free (the 8 rows a 32-lane half reads, k & 3 and
// bit 3 distinct, land on 8 disjoint 32-B bank groups).
MMT_DEV int gemm_trsw(int k) { return 2 * ((k & 3) | (((k >> 3) & 1) << 2)); }

// WGM x WGN waves per k-group own WM x WN sub-tiles; KS k-groups split the K-steps.  CONV: A is
// the implicit im2col of an NHWC 3x3/pad-1 (conv_k3) or 1x1 convolution, input read through the
// nearest-upsample index map (gemm.hip's conv mode).  LNF: LayerNorm folded into the GEMM
// (mmt_gemm_params.ln_fold): the row statistics of A are accumulated from the A fragments the
// waves already hold for the MFMAs (wave column wc sums fragment rows mt = wc, wc + WGN, ...), so
// the normalised operand never exists in memory and the LayerNorm launch disappears.
// EPI 1: the compact epilogue of a 16-bit C with bias / LayerNorm fold / ReLU or GELU only (no residual, C2,
// statistics, row map or row scale; the launcher checks): the general epilogue's branches for every other mode
// made the strip passes ~44 KiB of code per kernel, fetched cold by every workgroup (per-phase stamps: qkv
// passes 1.96 -> 0.68 us, fc1 2.90 -> 1.63 us with this form, profiles/r04_gemm_epilogue_stamps.jsonl).
// EPI 2: the compact epilogue of the residual producers (fp32 C = acc + bias + R, its 16-bit copy C2, the next
// LayerNorm's row statistics).
template <typename T, int BM, int BN, int WGM, int WGN, int KS, int ST, bool CONV, int LNM, int OCC = 1, bool RS = false,
          int EPI = 0>
MMT_DEV void gemm_glds_tile(const mmt_gemm_params& p, const int g, const int tile, const int slice, const int nsk,
                            const int ntiles) {
    constexpr int NW = WGM * WGN, TPG = 64 * NW;  // waves / threads per k-group
    constexpr int KT = 64;                        // bf16 elements of K per step: 128-B rows
    constexpr int STAGE = (BM + BN) * 128;        // bytes of one stage image (A rows, then W rows)
    constexpr int PA = BM / 8 / NW, PB = BN / 8 / NW;  // 1-KiB pieces per wave per stage
    static_assert(PA * 8 * NW == BM && PB * 8 * NW == BN, "pieces divide evenly over the waves");
    constexpr int L = PA + PB;  // DMA instructions per wave per stage
    constexpr int WM = BM / WGM, WN = BN / WGN, MT = WM / 16, NT = WN / 16;
    static_assert(KS * ST * STAGE <= 160 * 1024, "LDS budget");
    constexpr bool SB = BM * BN >= 256 * 256 || OCC > 1;  // single-buffered fragments (impl 7's 256x256; impl 8)
    // impl 9: 256x256 at ONE wave per SIMD (4 waves of 128x128, the 256 accumulators pinned to AGPRs by
    // inline-asm MFMAs), 2-slot ring of 64-deep stages; LayerNorm fold with handed-in statistics allowed
    constexpr bool W4 = BM == 256 && BN == 256 && NW == 4;
    static_assert(!W4 || (KS == 1 && ST == 2 && OCC == 1 && !CONV && (LNM == 0 || LNM == 2)), "impl 9 geometry");
    static_assert(!SB || (KS == 1 && (LNM == 0 || LNM >= 2) && !CONV), "impl 7 / 8 / 9: plain GEMM (or handed-in LN statistics)");
    // LNM 3: W given MN-major (W^T [K][ldw], the Linear backward's dX); 4: A and W MN-major (dW)
    constexpr bool TA = LNM == 4, TB = LNM == 3 || LNM == 4;
    static_assert(!TB || (BM == 128 && BN == 128 && !CONV), "MN-major operands: 128x128 tiles");
    static_assert(KS == 1 || BM * BN * 4 <= KS * ST * STAGE, "k-group reduction buffer");
    // impl 9: its half-tile fp32 image (128 x 260 floats) and the row statistics exceed the 128 KiB ring
    constexpr int LDS_BYTES = W4 ? (BM / 2) * (BN + 4) * 4 + BM * 8 + 64 : KS * ST * STAGE;
    static_assert(LDS_BYTES >= KS * ST * STAGE && LDS_BYTES <= 160 * 1024, "LDS budget");
    __shared__ __attribute__((aligned(1024))) unsigned char lds[LDS_BYTES];
    MMT_STAMP(0, "s_memrealtime");
    MMT_STAMP(1, "s_memtime");

    const int tiles_m = (p.M + BM - 1) / BM;
    // Tile order.  Grids of one or two rounds (batch 1): row tiles fastest, so the workgroups of one
    // XCD share its W column slice.  Larger grids (impl 5 / 6): row groups of GM tiles, column tiles next, so
    // the ~32 workgroups an XCD holds at a time cover GM row panels x every column tile and each A
    // panel / W slice is fetched into that XCD's L2 once and re-read from it (instead of the A
    // panels streaming in again from the Infinity Cache for every column tile).
    // (compiled into the large-M tiles only: in the batch-1 tile shapes the extra prologue code cost
    // ~1 % of the frame, interleaved bench A/B 953.5 vs 944.5 frames/s).  Round 5: also for the two-per-CU
    // 128x128 tiles (impl 8), which ran row-fastest over grids of thousands of tiles, so every XCD streamed
    // all of A from the Infinity Cache: fc1 at 16 pairs 149.0 -> 128.2 us, the training step 470-471 ->
    // 484 samples/s interleaved (profiles/r05_gemm_occ2_rowgroup_ab.txt)
    constexpr int GM = MMT_GEMM_GM;
    int tm, tn;
    if ((BM * BN >= 256 * 128 || OCC > 1) && gridDim.x * gridDim.y * gridDim.z > 512 && tiles_m > GM) {
        const int tiles_n = ntiles / tiles_m, grp = tile / (GM * tiles_n), first = grp * GM;
        const int gsz = min(tiles_m - first, GM), r = tile - grp * GM * tiles_n;
        tm = first + r % gsz;
        tn = r / gsz;
    } else {
        tm = tile % tiles_m;
        tn = tile / tiles_m;
    }
    constexpr bool LNF = LNM == 1 || LNM == 2;  // LayerNorm folded: 1 = row statistics from the A fragments, 2 = handed in
    const int m0_tile = tm * BM, n0 = tn * BN;
    const int lane = threadIdx.x & 63, kg = threadIdx.x / TPG;
    const int wid = (threadIdx.x % TPG) >> 6, wr = wid / WGN, wc = wid % WGN;
    const int l16 = lane & 15, lg = lane >> 4;
    const int M = p.M, N = p.N, K = p.K;

    const T* A0 = (const T*)p.a[g];
    const T* A1 = (const T*)p.a1[g];
    const T* W = (const T*)p.w[g];

    // This lane stages row (piece*8 + prow), logical chunk pch, into byte 16*lane of the piece:
    // position (lane & 7) of row prow holds chunk (lane & 7) ^ prow  (the read-side XOR).
    const int prow = lane >> 3, pch = (lane & 7) ^ prow;
    int64_t aoff[PA], boff[PB];  // GEMM: row offset of A; conv: input-image base pixel
    int ay[PA], ax[PA];           // conv: output pixel of the row
    const int ch = p.conv_h, cup = CONV ? p.conv_up : 1, hi = CONV ? p.conv_h / cup : 0;
    if constexpr (!CONV) {
        const int segr = (int)p.a_seg_rows, sega = (int)p.a_segs_a;
        const bool plain = segr >= M;  // one segment (wave-uniform): no divisions ahead of the first DMA
#pragma unroll
        for (int i = 0; i < PA; ++i) {
            const int m = min(m0_tile + (wid * PA + i) * 8 + prow, M - 1);
            if (plain) {
                aoff[i] = (int64_t)m * p.lda;
            } else {
                const int seg = m / segr, sa = seg % sega;  // 32-bit: the launcher checks the ranges
                aoff[i] = sa * p.a_stride_a + (int64_t)((seg - sa) / sega) * p.a_stride_b + (int64_t)(m - seg * segr) * p.lda;
            }
            ay[i] = ax[i] = 0;
        }
    } else {
#pragma unroll
        for (int i = 0; i < PA; ++i) {
            const int m = min(m0_tile + (wid * PA + i) * 8 + prow, M - 1);
            const int b = m / (ch * ch), rem = m - b * ch * ch;
            ay[i] = rem / ch;
            ax[i] = rem - ay[i] * ch;
            aoff[i] = (int64_t)b * (p.a_stride_a > 0 ? p.a_stride_a : (int64_t)hi * hi);  // image pitch (pixels)
        }
    }
#pragma unroll
    for (int i = 0; i < PB; ++i) boff[i] = (int64_t)min(n0 + (wid * PB + i) * 8 + prow, N - 1) * K;
    const int ks = p.k_split, cin = p.conv_cin, k3 = p.conv_k3;
    const float inv_cin = CONV && k3 ? 1.f / (float)cin : 0.f;
    const int cup_sh = CONV ? 31 - __builtin_clz(cup) : 0;

    unsigned char* ring = lds + kg * ST * STAGE;
    // this slice's K-steps [kb0, kb0 + nk) of the nk_all 64-deep steps (the launcher keeps nk >= KS)
    const int nk_all = (K + KT - 1) / KT, kb0 = slice * nk_all / nsk;
    const int nk = (slice + 1) * nk_all / nsk - kb0, ns = (nk + KS - 1) / KS;

    auto issue = [&](int s) {  // this k-group's step s -> ring slot s % ST
        const int k = (min(s * KS + kg, nk - 1) + kb0) * KT + pch * 8;  // this lane's 8-element chunk
        const bool kin = k < K;
        unsigned char* base = ring + (s % ST) * STAGE;
        // MN-major images: lane -> row (lane >> 4) of its 4-row piece, physical chunk lane & 15
        const int kst = (min(s * KS + kg, nk - 1) + kb0) * KT, trq = lane >> 4, trc = lane & 15;
        if constexpr (TA) {
#pragma unroll
            for (int i = 0; i < PA; ++i) {
                const int kr = (wid * PA + i) * 4 + trq, kk = kst + kr, m = m0_tile + (trc ^ gemm_trsw(kr)) * 8;
                glds16(kk < K && m < M ? (const void*)(A0 + (int64_t)kk * p.lda + m) : (const void*)g_zero_chunk,
                       base + (wid * PA + i) * 1024);
            }
        } else if constexpr (!CONV) {
            const bool hp = ks > 0 && k >= ks;
            const T* ab = (hp ? A1 - ks : A0) + k;
#pragma unroll
            for (int i = 0; i < PA; ++i)
                glds16(kin ? (const void*)(ab + aoff[i]) : (const void*)g_zero_chunk, base + (wid * PA + i) * 1024);
        } else {
            // Per-step address math stays off the integer-division path (a runtime-divisor division
            // is ~35 VALU; at 9 per step it held the DMA issue back by ~0.3 us per K-step): the tap
            // comes from a float reciprocal (exact: k < 2^24 and (k + 0.5) / cin sits >= 0.5 / cin
            // from an integer), the upsample factor is a power of two (shift), and the element
            // offset fits 32 bits (both checked by the launcher).
            int dy = 0, dx = 0, ci = k;
            if (k3) {  // k = (ky*3 + kx)*cin + ci; k3 == 2: the taps in reverse order (the flipped kernel)
                const uint32_t tap = (uint32_t)(((float)k + 0.5f) * inv_cin);
                ci = k - (int)tap * cin;
                const uint32_t tf = k3 == 2 ? 8u - tap : tap;
                const int ty = (int)(tf / 3u);
                dy = ty - 1;
                dx = (int)tf - ty * 3 - 1;
            }
#pragma unroll
            for (int i = 0; i < PA; ++i) {
                const int iy = ay[i] + dy, ix = ax[i] + dx;
                const bool ok = kin && iy >= 0 && ix >= 0 && iy < ch && ix < ch;
                const uint32_t pix = (uint32_t)aoff[i] + (uint32_t)((iy >> cup_sh) * hi + (ix >> cup_sh));
                const T* src = A0 + (pix * (uint32_t)p.lda + (uint32_t)ci);
                glds16(ok ? (const void*)src : (const void*)g_zero_chunk, base + (wid * PA + i) * 1024);
            }
        }
        if constexpr (TB) {
            const void* one = __is_same(T, bf16_t) ? (const void*)g_one_chunk_bf16 : (const void*)g_one_chunk_f16;
#pragma unroll
            for (int i = 0; i < PB; ++i) {
                const int kr = (wid * PB + i) * 4 + trq, kk = kst + kr, n = n0 + (trc ^ gemm_trsw(kr)) * 8;
                const void* src = kk >= K || n >= N ? (const void*)g_zero_chunk
                                  : p.w_t == 2 && n == N - 8 ? one
                                                             : (const void*)(W + (int64_t)kk * p.ldw + n);
                glds16(src, base + BM * 128 + (wid * PB + i) * 1024);
            }
        } else {
            const int kw = kin ? k : 0;  // past K: any in-bounds W bytes (they meet zero A chunks)
#pragma unroll
            for (int i = 0; i < PB; ++i) glds16(W + boff[i] + kw, base + BM * 128 + (wid * PB + i) * 1024);
        }
    };

    constexpr int MTW = (MT + WGN - 1) / WGN;  // LNF: fragment rows whose statistics this wave sums
    const int wc_u = __builtin_amdgcn_readfirstlane(wc);  // (v_dot2_f32_bf16 was tried for these sums: inexact)
    float lsx[MTW], lsxx[MTW];
#pragma unroll
    for (int j = 0; j < MTW; ++j) lsx[j] = lsxx[j] = 0.f;
    f32x4 acc[NT][MT];  // acc[nt][mt] = (C^T) fragment: rows n, columns m
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int j = 0; j < MT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // MN-major image: the 16 x 32 fragment of rows c0 .. c0+15, K-half t, as two transposed 4 x 16 reads
    // (lane l16 gets row c0 + l16, contraction 32t + 8lg + 4h .. +3 in read h)
    const int trl = 2 * (lg & 1) * 4, trq4 = l16 >> 2, trp = l16 & 3;
    auto tr_frag = [&](const unsigned char* img, int t, int c0) -> u32x4 {
        const int sw = 2 * trq4 + trl;  // gemm_trsw of rows 32t + 8lg + 4h + trq4
        const unsigned char* a = img + (32 * t + 8 * lg + trq4) * 256 + ((((c0 >> 3) + (trp >> 1)) ^ sw) * 16) + 8 * (trp & 1);
        const uint2 lo = gemm_tr16<0>(a), hi = gemm_tr16<1024>(a);
        return u32x4{lo.x, lo.y, hi.x, hi.y};
    };
    auto frag_a = [&](const unsigned char* b_, int t, int sw_, int mt) -> u32x4 {
        if constexpr (TA) return tr_frag(b_, t, wr * WM + mt * 16);
        else return *(const u32x4*)(b_ + ((wr * WM + mt * 16 + l16) * 8 + sw_) * 16);
    };
    auto frag_b = [&](const unsigned char* b_, int t, int sw_, int nt) -> u32x4 {
        if constexpr (TB) return tr_frag(b_ + BM * 128, t, wc * WN + nt * 16);
        else return *(const u32x4*)(b_ + BM * 128 + ((wc * WN + nt * 16 + l16) * 8 + sw_) * 16);
    };
    // Fragments of one K-step: [t][*] = the two 32-deep halves of the 64-deep step.
#define MMT_READ(BUF, AF, BF, MTV)                                                                               \
    {                                                                                                            \
        const unsigned char* b_ = (BUF);                                                                         \
        _Pragma("unroll") for (int t = 0; t < 2; ++t) {                                                          \
            const int sw_ = (4 * t + lg) ^ (lane & 7);                                                           \
            _Pragma("unroll") for (int mt = 0; mt < MTV; ++mt) AF[t][mt] = frag_a(b_, t, sw_, mt);               \
            _Pragma("unroll") for (int nt = 0; nt < NT; ++nt) BF[t][nt] = frag_b(b_, t, sw_, nt);                \
        }                                                                                                        \
        __builtin_amdgcn_sched_barrier(0); /* all reads issue before the MFMAs that hide them */                 \
    }
    // asm (transposed) reads: after the wait that completed them, the registers pass through an empty asm
    // so that no MFMA reading them is scheduled above it (no-op for the plain reads)
#define MMT_PIN(AF, BF, MTV)                                                                                     \
    if constexpr (TB) {                                                                                          \
        _Pragma("unroll") for (int t = 0; t < 2; ++t) {                                                          \
            _Pragma("unroll") for (int mt = 0; mt < MTV; ++mt) asm volatile("" : "+v"(AF[t][mt]));               \
            _Pragma("unroll") for (int nt = 0; nt < NT; ++nt) asm volatile("" : "+v"(BF[t][nt]));                \
        }                                                                                                        \
    }
#define MMT_WAIT_PIN(AF, BF, MTV)                                                                                \
    if constexpr (TB) {                                                                                          \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                       \
        MMT_PIN(AF, BF, MTV)                                                                                     \
    }
#define MMT_MMA(AF, BF, MTV)                                                                                     \
    {                                                                                                            \
        if (MMT_GEMM_ABLATE == 2) {                                                                              \
            acc[0][0] += __builtin_bit_cast(f32x4, AF[0][0]) + __builtin_bit_cast(f32x4, BF[1][NT - 1]);         \
        } else {                                                                                                 \
            _Pragma("unroll") for (int t = 0; t < 2; ++t)                                                        \
            _Pragma("unroll") for (int nt = 0; nt < NT; ++nt)                                                    \
            _Pragma("unroll") for (int mt = 0; mt < MTV; ++mt) acc[nt][mt] =                                     \
                mfma16x16x32<T>(BF[t][nt], AF[t][mt], acc[nt][mt]);                                              \
        }                                                                                                        \
        if constexpr (LNM == 1) { /* compile-time fragment index, scalar (wave-uniform) wave-column test; */     \
            /* packed fp32 sums (v_pk_add / v_pk_fma on the {lo, hi} bf16 pair), issued after the MFMAs */       \
            _Pragma("unroll") for (int mt_ = 0; mt_ < MTV; ++mt_) {                                              \
                if (mt_ % WGN == wc_u) {                                                                         \
                    f32x2 sx_ = {0.f, 0.f}, sxx_ = {0.f, 0.f};                                                   \
                    _Pragma("unroll") for (int t = 0; t < 2; ++t)                                                \
                    _Pragma("unroll") for (int e = 0; e < 4; ++e) {                                              \
                        const f32x2 v_ = unpack2<T>(AF[t][mt_][e]);                                              \
                        sx_ += v_;                                                                               \
                        sxx_ = __builtin_elementwise_fma(v_, v_, sxx_);                                          \
                    }                                                                                            \
                    lsx[mt_ / WGN] += sx_[0] + sx_[1];                                                           \
                    lsxx[mt_ / WGN] += sxx_[0] + sxx_[1];                                                        \
                }                                                                                                \
            }                                                                                                    \
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
    for (int j = 0; j < ST - 1 && j < ns; ++j) issue(j);
    if (MMT_GEMM_ABLATE == 1) wait_vm<0>();
    sync_for(0);
    MMT_STAMP(2, "s_memtime");
    // MTV = this wave's 16-row fragments that hold rows < M.  The K loop is instantiated per MTV
    // (all, 1, none: the row tails of the 528-row groups, M % 16 == 0) and chosen once, outside
    // the loop, so the fragment reads and MFMAs of padding rows are never issued; the DMA and
    // barriers are the same in every copy.
    auto kloop = [&](auto MTVc) {
        constexpr int MTV = decltype(MTVc)::value;
        if constexpr (SB) {
            // 256x256 tile (2 waves per SIMD, 128 accumulator registers each): one fragment set, read
            // and multiplied per 32-deep half; the SIMD's other wave covers the read latency
            u32x4 ha[1][MT], hb[1][NT];
            for (int s = 0; s < ns; ++s) {
                if (s > 0) sync_for(s);
                const unsigned char* b_ = ring + (s % ST) * STAGE;
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const int sw_ = (4 * t + lg) ^ (lane & 7);
#pragma unroll
                    for (int mt = 0; mt < MTV; ++mt) ha[0][mt] = frag_a(b_, t, sw_, mt);
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt) hb[0][nt] = frag_b(b_, t, sw_, nt);
                    if constexpr (TB) {
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
                        for (int mt = 0; mt < MTV; ++mt) asm volatile("" : "+v"(ha[0][mt]));
#pragma unroll
                        for (int nt = 0; nt < NT; ++nt) asm volatile("" : "+v"(hb[0][nt]));
                    }
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                        for (int mt = 0; mt < MTV; ++mt) acc[nt][mt] = mfma16x16x32<T>(hb[0][nt], ha[0][mt], acc[nt][mt]);
                }
            }
            return;
        }
        u32x4 fa0[2][MT], fb0[2][NT], fa1[2][MT], fb1[2][NT];
        MMT_READ(ring, fa0, fb0, MTV);
        // Every k-group has a real K-step at j < ns-1; only the last can be empty (KS = 2 with an odd
        // step count).  Keeping that test out of the loop keeps the accumulators in place (a
        // conditional MFMA block inside the loop made hipcc shuttle them through VGPRs every step).
        int s = 0;
        for (; s + 2 < ns; s += 2) {
            sync_for(s + 1);  // (its lds_barrier waits lgkmcnt(0): fa0 / fb0 are complete)
            MMT_PIN(fa0, fb0, MTV);
            MMT_READ(ring + ((s + 1) % ST) * STAGE, fa1, fb1, MTV);
            MMT_MMA(fa0, fb0, MTV);
            sync_for(s + 2);
            MMT_PIN(fa1, fb1, MTV);
            MMT_READ(ring + ((s + 2) % ST) * STAGE, fa0, fb0, MTV);
            MMT_MMA(fa1, fb1, MTV);
        }
        const bool last_ok = KS == 1 || (ns - 1) * KS + kg < nk;
        if (s + 1 < ns) {
            sync_for(s + 1);
            MMT_PIN(fa0, fb0, MTV);
            MMT_READ(ring + ((s + 1) % ST) * STAGE, fa1, fb1, MTV);
            MMT_MMA(fa0, fb0, MTV);
            MMT_WAIT_PIN(fa1, fb1, MTV);
            if (last_ok) MMT_MMA(fa1, fb1, MTV);
        } else if (last_ok) {
            MMT_WAIT_PIN(fa0, fb0, MTV);
            MMT_MMA(fa0, fb0, MTV);
        }
    };
    if constexpr (W4) {
        // impl 9: one wave per SIMD, each a 128x128 wave tile = 64 v_mfma_f32_16x16x32 per 32-deep half.  The
        // accumulators are inline-asm operands with the "a" constraint (all 256 AGPRs: through the builtin hipcc
        // shuttled them through VGPRs every step and spilled).  Half t+1's fragments are read beside half t's 64
        // MFMAs (two statically named fragment sets); one K-step of DMA is in flight behind the one multiplied
        // (2-slot ring of 64 KiB stages: a 4-slot ring of 32-deep stages measured the same,
        // profiles/r05_gemm256_proto.jsonl).  Rows past M (last row tile) are computed from clamped rows and not
        // stored.  No MFMA sits under a branch (hipcc then keeps the accumulators in place).
        u32x4 fa[2][MT], fb[2][NT];
        auto rd = [&](int s, int t, u32x4 (&af)[MT], u32x4 (&bf)[NT]) {
            const unsigned char* b_ = ring + (s % ST) * STAGE;
            const int sw_ = (4 * t + lg) ^ (lane & 7);
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) af[mt] = frag_a(b_, t, sw_, mt);
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) bf[nt] = frag_b(b_, t, sw_, nt);
        };
        auto mma = [&](const u32x4 (&af)[MT], const u32x4 (&bf)[NT]) {
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) {
                    // s_nop 1: covers a VALU write of a fragment register hipcc might place just before (it does
                    // not see the MFMA inside the asm)
                    if constexpr (__is_same(T, bf16_t))
                        asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                                     : "+a"(acc[nt][mt]) : "v"(bf[nt]), "v"(af[mt]));
                    else
                        asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_f16 %0, %1, %2, %0"
                                     : "+a"(acc[nt][mt]) : "v"(bf[nt]), "v"(af[mt]));
                }
        };
        issue(0);
        if (ns > 1) {
            issue(1);
            wait_vm<L>();  // step 0 landed (step 1's L pieces may stay in flight)
        } else {
            wait_vm<0>();
        }
        lds_barrier();
        rd(0, 0, fa[0], fb[0]);
        for (int s = 0; s + 1 < ns; ++s) {
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0) as a builtin: hipcc then knows fa[0] / fb[0] are in
            __builtin_amdgcn_sched_barrier(0);
            rd(s, 1, fa[1], fb[1]);
            __builtin_amdgcn_sched_barrier(0);
            mma(fa[0], fb[0]);
            __builtin_amdgcn_sched_barrier(0);
            wait_vm<0>();   // step s+1 landed (nothing newer in flight)
            lds_barrier();  // every wave is past its reads of slot s % 2
            if (s + 2 < ns) issue(s + 2);
            rd(s + 1, 0, fa[0], fb[0]);
            __builtin_amdgcn_sched_barrier(0);
            mma(fa[1], fb[1]);
            __builtin_amdgcn_sched_barrier(0);
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_sched_barrier(0);
        rd(ns - 1, 1, fa[1], fb[1]);
        __builtin_amdgcn_sched_barrier(0);
        mma(fa[0], fb[0]);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_sched_barrier(0);
        mma(fa[1], fb[1]);
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4" ::: "memory");  // last MFMA results -> accvgpr reads
    } else {
        const int mtv = __builtin_amdgcn_readfirstlane(min(max((M - m0_tile - wr * WM + 15) / 16, 0), MT));
        if (mtv == 0) kloop(gemm_ic<0>{});
        else if (mtv == 1 && MT > 1) kloop(gemm_ic<1>{});
        else kloop(gemm_ic<MT>{});  // whole fragments (other partial counts: padding computed, not stored)
    }
#undef MMT_READ
#undef MMT_MMA
#undef MMT_PIN
#undef MMT_WAIT_PIN
    MMT_STAMP(3, "s_memtime");

    // ---- split-K hand-off of the two-per-CU MN-major tiles (impl 8 with a_t / w_t: the training step's dW / dX
    // GEMMs; round 6).  Their grids are 0.6-1.6 rounds of the 512 two-per-CU slots (dW of fc1: 336 tiles of 132
    // K-steps), so a K split evens the CUs' work out.  The one-per-CU tiles hand off through the assembled tile
    // image (below); this tile's fp32 image does not fit its 64 KiB ring in one piece, so the hand-off runs on the
    // accumulator registers instead, before the epilogue: every slice stores its fragments lane-linear (one 1-KiB
    // wave-instruction per 16x16 fragment, so the slab layout is [wave][fragment][lane]), drains them and takes an
    // agent-scope arrival ticket (the store-first form of the one-per-CU tiles, no waiting anywhere); the
    // workgroup that draws the last ticket resets it, sums the nsk slabs in SLICE order (its own read back too,
    // which frees its accumulators for the sum) and alone runs the epilogue.  The sum's order is fixed, so the
    // result does not depend on arrival order; the same K ranges and fragment order as impl 1's split give
    // bit-identical partials.
    constexpr bool SK2 = OCC > 1 && TB && !W4;
    if constexpr (SK2) {
        if (nsk > 1) {
            constexpr int FR = NT * MT, SLAB = BM * BN * 4;
            static_assert(NW * FR * 64 * 16 == SLAB, "register slab covers the tile");
            const int64_t tix = (int64_t)g * ntiles + tile;
            const __amdgpu_buffer_rsrc_t slabs = __builtin_amdgcn_make_buffer_rsrc(
                p.sk_ws + tix * nsk * (BM * BN), (short)0, nsk * SLAB, 0x00020000);
            const int woff = (wid * FR * 64 + lane) * 16;
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[nt][mt]), slabs,
                                                           slice * SLAB + woff + (nt * MT + mt) * 1024, 0, 16);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
            __syncthreads();
            int* flag = (int*)lds;  // every wave is past its fragment reads (barrier above)
            if (threadIdx.x == 0) {
                const uint32_t old = __hip_atomic_fetch_add(p.sk_cnt + tix, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const int last = old == (uint32_t)(nsk - 1);
                if (last) __hip_atomic_store(p.sk_cnt + tix, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                *flag = last;
            }
            __syncthreads();
            if (!*flag) return;
            __syncthreads();  // every wave has read the flag before the epilogue reuses the LDS
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) acc[nt][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
            for (int q = 0; q < nsk; ++q) {  // slice order
                u32x4 v[NT][MT];
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt)
                        v[nt][mt] = __builtin_amdgcn_raw_buffer_load_b128(slabs, q * SLAB + woff + (nt * MT + mt) * 1024, 0, 16);
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt) acc[nt][mt] += __builtin_bit_cast(f32x4, v[nt][mt]);
            }
        }
    }

    // ---- epilogue through LDS.  Fragment-shaped stores (16 rows x 32 B per wave-instruction) ran
    // at a fraction of the store path's rate (5-8 us of a 15-19 us launch, per in-kernel stamps),
    // so the fp32 tile is first assembled in LDS (summing the two k-groups when KS = 2) and then
    // every thread owns 8 consecutive columns of RPP-row strips: bias / residual loads and C / C2
    // stores are whole 256-512-B row segments per wave-instruction.
    constexpr int TP = BN + 4;  // tile row pitch (floats); +4 keeps the fragment writes 2-way
    // EPASS: a tile whose fp32 image does not fit the stage ring (256x256) is assembled and written
    // out in WGM passes of one wave row (WM rows) each
    constexpr int EPASS = BM * TP * 4 + KS * BM * 8 + 16 <= KS * ST * STAGE ? 1 : WGM, EB = BM / EPASS;
    static_assert(EPASS == 1 || (EB == WM && KS == 1 && (LNM == 0 || LNM >= 2)),
                  "multi-pass epilogue: plain GEMM tiles (also with handed-in LayerNorm statistics)");
    static_assert(EB * TP * 4 + KS * BM * 8 + 4 <= LDS_BYTES, "epilogue pass fits in LDS");
    constexpr int FLAG_OFF = EB * TP * 4 + KS * BM * 8;  // split-K "this workgroup sums" word
    float* ctile = (float*)lds;
    float* rstat = ctile + EB * TP;  // LNF: [KS][BM][2] partial (sum x, sum x^2) per k-group (all BM tile rows)
    // LNM 2: the handed-in row statistics (K/64 partial (sum, sum of squares) pairs per A row), read
    // now so that their latency overlaps the tile's LDS assembly: TPRW threads per tile row, each
    // loading every TPRW-th pair of its row (at most 8: K <= 64 * 8 * TPRW), summed below
    constexpr int NTH_E = TPG * KS, TPRW = NTH_E / BM;
    static_assert(TPRW >= 1 && (TPRW & (TPRW - 1)) == 0 && TPRW <= 64, "statistics reduction geometry");
    constexpr int NSP = TPRW >= 2 ? 8 : 16;  // pairs per thread (K <= 64 * 16, glds_takes)
    f32x2 stp[NSP];
    const int kp = K / 64, srow = threadIdx.x / TPRW, spart = threadIdx.x % TPRW;
    if constexpr (LNM == 2) {
        const f32x2* st = (const f32x2*)p.ln_stats_in[g] + (int64_t)min(m0_tile + srow, M - 1) * kp;
#pragma unroll
        for (int i = 0; i < NSP; ++i) {
            const int j = spart + i * TPRW;
            stp[i] = j < kp ? st[j] : f32x2{0.f, 0.f};
        }
    }
    // Residual rows of a single-pass, unsplit epilogue, loaded before the tile assembly: their L2 /
    // Infinity Cache latency then overlaps the fragment writes and barriers below instead of being
    // exposed once per group of four strip passes (proj / fc2 / encoder Linears: fp32 residual stream).
    constexpr int TPR0 = BN / 8, RPP0 = TPG * KS / TPR0, NPASS0 = EB / RPP0;
    constexpr bool RPRE = EPASS == 1 && NPASS0 <= 8 && BM * BN <= 128 * 128 && OCC == 1;  // batch-1 tiles (large
                                                                                          // ones / OCC 2 spill)
    const int tc0 = (threadIdx.x % TPR0) * 8, tr0 = threadIdx.x / TPR0, nc0 = min(n0 + tc0, N - 8);
    auto rload = [&](int m, int nc, f32x4& ra, f32x4& rb) {  // residual row of output row m, columns nc..nc+7
        const float* R = p.r[g];
        const int64_t csr = p.c_seg_rows > 0 ? p.c_seg_rows : INT64_MAX, csp = p.c_seg_pitch;
        int64_t rr = csr == INT64_MAX ? (int64_t)m : (m / csr) * csp + m % csr;
        if (p.r_mode == 1) rr = m % p.r_p0;
        else if (p.r_mode == 2) {
            const int hw = p.r_p0 * p.r_p0, b = m / hw, rem = m - b * hw;
            const int y = rem / p.r_p0, x = rem - y * p.r_p0, hs = p.r_p0 / p.r_p1;
            rr = (int64_t)b * hs * hs + (int64_t)(y / p.r_p1) * hs + (x / p.r_p1);
        }
        if (p.r_t) {
            const u32x4 u = *(const u32x4*)((const T*)R + rr * p.ldr + nc);
            const f32x2 u0 = unpack2<T>(u[0]), u1 = unpack2<T>(u[1]), u2 = unpack2<T>(u[2]), u3 = unpack2<T>(u[3]);
            ra = f32x4{u0[0], u0[1], u1[0], u1[1]};
            rb = f32x4{u2[0], u2[1], u3[0], u3[1]};
        } else {
            ra = *(const f32x4*)(R + rr * p.ldr + nc);
            rb = *(const f32x4*)(R + rr * p.ldr + nc + 4);
        }
    };
    f32x4 rpa[RPRE ? NPASS0 : 1], rpb[RPRE ? NPASS0 : 1];
    const bool rpre = RPRE && p.r[g] != nullptr && nsk == 1;  // wave-uniform
    if constexpr (RPRE) {
        if (rpre) {
#pragma unroll
            for (int i = 0; i < NPASS0; ++i) rload(min(m0_tile + tr0 + i * RPP0, M - 1), nc0, rpa[i], rpb[i]);
        }
    }
    lds_barrier();  // every wave is past its last fragment read (the DMA ring is drained: vmcnt(0))
    if constexpr (LNM == 2) {  // (sum, sum of squares) of the row, in pair order within each thread
        float sx = 0.f, sxx = 0.f;
#pragma unroll
        for (int i = 0; i < NSP; ++i) {
            sx += stp[i][0];
            sxx += stp[i][1];
        }
#pragma unroll
        for (int o = 1; o < TPRW; o <<= 1) {  // the row's TPRW threads are consecutive lanes
            sx += __shfl_xor(sx, o, 64);
            sxx += __shfl_xor(sxx, o, 64);
        }
        if (spart == 0) {
            rstat[srow * 2] = sx;
            rstat[srow * 2 + 1] = sxx;
        }
    }
    if constexpr (LNM == 1) {
#pragma unroll
        for (int j = 0; j < MTW; ++j) {
            const int mt = wc + j * WGN;
            const float sx = lanegroup_sum(lsx[j]), sxx = lanegroup_sum(lsxx[j]);
            if (mt < MT && lg == 0) {
                rstat[(kg * BM + wr * WM + mt * 16 + l16) * 2] = sx;
                rstat[(kg * BM + wr * WM + mt * 16 + l16) * 2 + 1] = sxx;
            }
        }
    }
    if ((KS == 1 || kg == 1) && (EPASS == 1 || wr == 0)) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
                *(f32x4*)(ctile + ((EPASS == 1 ? wr * WM : 0) + mt * 16 + l16) * TP + wc * WN + nt * 16 + lg * 4) =
                    acc[nt][mt];
    }
    if constexpr (KS == 2) {
        lds_barrier();
        if (kg == 0) {
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) {
                    f32x4* t4 = (f32x4*)(ctile + (wr * WM + mt * 16 + l16) * TP + wc * WN + nt * 16 + lg * 4);
                    *t4 = *t4 + acc[nt][mt];
                }
        }
    }
    static_assert(KS <= 2, "k-group reduction written for up to two groups");
    lds_barrier();
    MMT_STAMP(4, "s_memtime");

    // 8-column strips: one 16-B store per lane for a bf16 C (two for fp32); dwordx2 stores were
    // store-issue-bound.
    constexpr int NTHR = TPG * KS, TPR = BN / 8, RPP = NTHR / TPR, NPASS = EB / RPP;
    static_assert(NTHR % TPR == 0 && EB % RPP == 0, "strip geometry");
    const float* bias = p.bias[g];
    const float* R = p.r[g];
    char* C = (char*)p.c[g];
    char* C2 = (char*)p.c2[g];
    const int tc = (threadIdx.x % TPR) * 8, tr = threadIdx.x / TPR;

#if MMT_GEMM_SK_TICKET_FIRST
    // ---- split-K hand-off (cdna_hip_programming.md Guideline 16, form R1 in its counter variant), ticket
    // first: lane 0 draws an agent-scope arrival ticket BEFORE any partial is stored, so the slice that draws the
    // last one keeps its partial in LDS and never writes it (nsk - 1 slabs cross memory instead of nsk; round 5,
    // VERDICT r4 item 7).  Every other slice stores its fp32 partial tile WRITE-THROUGH (buffer_store ... sc1, no
    // release fence), every wave drains its stores, and after a workgroup barrier lane 0 adds to the tile's
    // "published" counter.  The last slice's lane 0 polls that counter (relaxed agent loads = sc1, s_sleep between
    // polls, bounded) until the nsk - 1 others have published -- they all hold tickets already, i.e. are past
    // their K loops, so the wait is their store drain -- resets both counters for the next launch, and after a
    // workgroup barrier every wave reads the other partials with sc1 loads only (no acquire either), summing the
    // nsk partials in SLICE order (its own from LDS): the result does not depend on which slice arrives last.  It
    // alone runs the epilogue.  Tickets [0, sk_cnt_n / 2), published counts [sk_cnt_n / 2, sk_cnt_n).
    // (compiled only into the tiles the launcher may split: the two-per-CU and 256x256 tiles never are, and the
    // hand-off's registers made their epilogues spill, round 5)
    constexpr bool CAN_SPLIT = OCC == 1 && BM * BN < 256 * 256;
    if (CAN_SPLIT && nsk > 1) {
        const int64_t tix = (int64_t)g * ntiles + tile;
        constexpr int SLAB = BM * BN * 4;  // bytes of one partial tile
        const __amdgpu_buffer_rsrc_t slabs = __builtin_amdgcn_make_buffer_rsrc(
            p.sk_ws + tix * nsk * (BM * BN), (short)0, nsk * SLAB, 0x00020000);
        uint32_t* ticket = p.sk_cnt + tix;
        uint32_t* published = p.sk_cnt + p.sk_cnt_n / 2 + tix;
        int* flag = (int*)(lds + FLAG_OFF);
        if (threadIdx.x == 0) *flag = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                                      (uint32_t)(nsk - 1);
        __syncthreads();
        if (!*flag) {
#pragma unroll
            for (int ps = 0; ps < NPASS; ++ps) {
                const int r = tr + ps * RPP, off = slice * SLAB + (r * BN + tc) * 4;
                __builtin_amdgcn_raw_buffer_store_b128(*(const u32x4*)(ctile + r * TP + tc), slabs, off, 0, 16);
                __builtin_amdgcn_raw_buffer_store_b128(*(const u32x4*)(ctile + r * TP + tc + 4), slabs, off + 16, 0, 16);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
            __syncthreads();
            if (threadIdx.x == 0) __hip_atomic_fetch_add(published, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        if (threadIdx.x == 0) {
            for (int spin = 0; spin < (1 << 22); ++spin) {  // bounded: the others only have stores left
                if (__hip_atomic_load(published, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (uint32_t)(nsk - 1)) break;
                __builtin_amdgcn_s_sleep(1);
            }
            __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(published, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below
#pragma unroll
        for (int ps = 0; ps < NPASS; ++ps) {
            const int r = tr + ps * RPP, off = (r * BN + tc) * 4;
            f32x4 sa = {0.f, 0.f, 0.f, 0.f}, sb = sa;
#pragma unroll
            for (int q0 = 0; q0 < 8; q0 += 4) {  // 4 slices' loads in flight together, summed in order
                u32x4 pa[4], pb[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int q = q0 + j;
                    if (q < nsk && q != slice) {
                        pa[j] = __builtin_amdgcn_raw_buffer_load_b128(slabs, q * SLAB + off, 0, 16);
                        pb[j] = __builtin_amdgcn_raw_buffer_load_b128(slabs, q * SLAB + off + 16, 0, 16);
                    }
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int q = q0 + j;
                    if (q < nsk) {
                        if (q == slice) {
                            sa += *(const f32x4*)(ctile + r * TP + tc);
                            sb += *(const f32x4*)(ctile + r * TP + tc + 4);
                        } else {
                            sa += __builtin_bit_cast(f32x4, pa[j]);
                            sb += __builtin_bit_cast(f32x4, pb[j]);
                        }
                    }
                }
            }
            *(f32x4*)(ctile + r * TP + tc) = sa;  // this thread's own strip: no barrier needed
            *(f32x4*)(ctile + r * TP + tc + 4) = sb;
        }
    }
#else
    // ---- split-K hand-off, store first (round 4; the product form again since round 5's end): every slice stores its
    // fp32 partial tile WRITE-THROUGH (buffer_store ... sc1, so no release fence), every wave drains its stores, and
    // after a workgroup barrier lane 0 takes an agent-scope arrival ticket.  The workgroup that draws the last ticket
    // resets it and reads the other slices' partials with sc1 loads only (so no acquire either), summing the nsk
    // partials in SLICE order (its own from LDS): the result does not depend on which slice arrives last.  It alone
    // runs the epilogue.  (The ticket-first form above writes one partial less per tile -- head conv1 17.6 -> 12.1 MB
    // -- but its last slice waits on the others' store drain: head conv1 27.8 -> 30.6 us and conv2 14.5 -> 17.1 us in
    // the batch-1 frame, profiles/r05_splitk_form_ab.txt.)
    constexpr bool CAN_SPLIT = OCC == 1 && BM * BN < 256 * 256;
    if (CAN_SPLIT && nsk > 1) {
        const int64_t tix = (int64_t)g * ntiles + tile;
        constexpr int SLAB = BM * BN * 4;  // bytes of one partial tile
        const __amdgpu_buffer_rsrc_t slabs = __builtin_amdgcn_make_buffer_rsrc(
            p.sk_ws + tix * nsk * (BM * BN), (short)0, nsk * SLAB, 0x00020000);
#pragma unroll
        for (int ps = 0; ps < NPASS; ++ps) {
            const int r = tr + ps * RPP, off = slice * SLAB + (r * BN + tc) * 4;
            __builtin_amdgcn_raw_buffer_store_b128(*(const u32x4*)(ctile + r * TP + tc), slabs, off, 0, 16);
            __builtin_amdgcn_raw_buffer_store_b128(*(const u32x4*)(ctile + r * TP + tc + 4), slabs, off + 16, 0, 16);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
        __syncthreads();
        int* flag = (int*)(lds + FLAG_OFF);
        if (threadIdx.x == 0) {
            const uint32_t old = __hip_atomic_fetch_add(p.sk_cnt + tix, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int last = old == (uint32_t)(nsk - 1);
            if (last) __hip_atomic_store(p.sk_cnt + tix, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            *flag = last;
        }
        __syncthreads();
        if (!*flag) return;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below
#pragma unroll
        for (int ps = 0; ps < NPASS; ++ps) {
            const int r = tr + ps * RPP, off = (r * BN + tc) * 4;
            f32x4 sa = {0.f, 0.f, 0.f, 0.f}, sb = sa;
#pragma unroll
            for (int q0 = 0; q0 < 8; q0 += 4) {  // 4 slices' loads in flight together, summed in order
                u32x4 pa[4], pb[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int q = q0 + j;
                    if (q < nsk && q != slice) {
                        pa[j] = __builtin_amdgcn_raw_buffer_load_b128(slabs, q * SLAB + off, 0, 16);
                        pb[j] = __builtin_amdgcn_raw_buffer_load_b128(slabs, q * SLAB + off + 16, 0, 16);
                    }
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int q = q0 + j;
                    if (q < nsk) {
                        if (q == slice) {
                            sa += *(const f32x4*)(ctile + r * TP + tc);
                            sb += *(const f32x4*)(ctile + r * TP + tc + 4);
                        } else {
                            sa += __builtin_bit_cast(f32x4, pa[j]);
                            sb += __builtin_bit_cast(f32x4, pb[j]);
                        }
                    }
                }
            }
            *(f32x4*)(ctile + r * TP + tc) = sa;  // this thread's own strip: no barrier needed
            *(f32x4*)(ctile + r * TP + tc + 4) = sb;
        }
    }
#endif
    const int n = n0 + tc, nc = min(n, N - 8);
    const bool csplit = p.c2_copy == 3 || p.c2_copy == 4;
    float* stats_out = p.c2_copy && !csplit && C2 ? p.ln_stats_out[g] : nullptr;
    // c2_copy 3: the last 8 output columns go to C2 (row pitch 8), the others to C (pitch ldc >= N - 8);
    // c2_copy 4: of those 8 only column N - 8, to C2 as one contiguous vector (row pitch 1: the training dW
    // GEMM's bias gradient, handed to autograd as it is)
    const bool colsplit = csplit && n >= N - 8;
    char* Cs = colsplit ? C2 : C;
    if (csplit) C2 = nullptr;
    f32x4 bn0 = {0.f, 0.f, 0.f, 0.f}, bn1 = bn0, cs0 = bn0, cs1 = bn0;
    if (bias) {
        bn0 = *(const f32x4*)(bias + nc);
        bn1 = *(const f32x4*)(bias + nc + 4);
    }
    if constexpr (LNF) {
        cs0 = *(const f32x4*)(p.ln_colsum[g] + nc);
        cs1 = *(const f32x4*)(p.ln_colsum[g] + nc + 4);
    }
    const float inv_k = 1.f / (float)K;
    // output row map (template K/V cache: search rows of a [S][ntok] stream); identity if c_seg_rows == 0
    // (32-bit unsigned division: M and the segment rows are < 2^31; a 64-bit one is a long software sequence)
    const int64_t csr = p.c_seg_rows > 0 ? p.c_seg_rows : INT64_MAX, csp = p.c_seg_pitch;
    const uint32_t csr32 = (uint32_t)min(csr, (int64_t)INT32_MAX);
    auto crow = [&](int m) -> int64_t {
        if (csr == INT64_MAX) return (int64_t)m;
        const uint32_t qd = (uint32_t)m / csr32;
        return (int64_t)qd * csp + (int64_t)((uint32_t)m - qd * csr32);
    };
    constexpr int PG = NPASS < 4 ? NPASS : 4;  // passes whose residual loads are in flight together
    for (int ep = 0; ep < EPASS; ++ep) {
    if (ep > 0) {  // the next wave row's accumulators into the (re-used) tile image
        lds_barrier();
        if (wr == ep) {
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
                    *(f32x4*)(ctile + (mt * 16 + l16) * TP + wc * WN + nt * 16 + lg * 4) = acc[nt][mt];
        }
        lds_barrier();
    }
    const int m0 = m0_tile + ep * EB;  // first tile row of this pass
    if constexpr (EPI == 1) {
        static_assert(!RS, "compact epilogue: no row scale");
#pragma unroll
        for (int i = 0; i < NPASS; ++i) {
            const int r = tr + i * RPP, m = m0 + r;
            f32x4 va = *(const f32x4*)(ctile + r * TP + tc);
            f32x4 vb = *(const f32x4*)(ctile + r * TP + tc + 4);
            if constexpr (LNF) {  // as the general path
                float sx = 0.f, sxx = 0.f;
                constexpr int NQ = LNM == 1 ? KS : 1;
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    sx += rstat[(q * BM + ep * EB + r) * 2];
                    sxx += rstat[(q * BM + ep * EB + r) * 2 + 1];
                }
                const float mu = sx * inv_k, var = fmaxf(sxx * inv_k - mu * mu, 0.f);
                const float rstd = rsqrtf(var + p.ln_eps);
                va = (va - mu * cs0) * rstd;
                vb = (vb - mu * cs1) * rstd;
            }
            va += bn0;
            vb += bn1;
            if (C2 && m < M && n < N)  // c2_copy 2: the pre-activation in the compute dtype (training fc1)
                *(u32x4*)((T*)C2 + (int64_t)m * p.ldc + n) = u32x4{pack2<T>(va[0], va[1]), pack2<T>(va[2], va[3]),
                                                                pack2<T>(vb[0], vb[1]), pack2<T>(vb[2], vb[3])};
            if (p.act == 1) {
                va.xy = gelu_erf2(va.xy);
                va.zw = gelu_erf2(va.zw);
                vb.xy = gelu_erf2(vb.xy);
                vb.zw = gelu_erf2(vb.zw);
            } else if (p.act == 2) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    va[j] = fmaxf(va[j], 0.f);
                    vb[j] = fmaxf(vb[j], 0.f);
                }
            }
            if (m < M && n < N)
                *(u32x4*)((T*)C + crow(m) * p.ldc + n) = u32x4{pack2<T>(va[0], va[1]), pack2<T>(va[2], va[3]),
                                                               pack2<T>(vb[0], vb[1]), pack2<T>(vb[2], vb[3])};
        }
    } else if constexpr (EPI == 2) {  // compact residual producer: fp32 C = acc + bias + R, C2 its 16-bit copy,
                                      // the next LayerNorm's row statistics (proj / fc2 of the ViT blocks)
        static_assert(!LNF, "compact residual epilogue: plain tiles");
#pragma unroll
        for (int p0 = 0; p0 < NPASS; p0 += PG) {
            f32x4 ra[PG], rb[PG];
#pragma unroll
            for (int i = 0; i < PG; ++i) {
                ra[i] = rb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
                if constexpr (RPRE) {
                    if (rpre) {
                        ra[i] = rpa[p0 + i];
                        rb[i] = rpb[p0 + i];
                        continue;
                    }
                }
                if (R) {  // plain rows (the launcher checks r_mode / r_t / c_seg_rows)
                    const float* rr = R + (int64_t)min(m0 + tr + (p0 + i) * RPP, M - 1) * p.ldr + nc;
                    ra[i] = *(const f32x4*)rr;
                    rb[i] = *(const f32x4*)(rr + 4);
                }
            }
#pragma unroll
            for (int i = 0; i < PG; ++i) {
                const int r = tr + (p0 + i) * RPP, m = m0 + r;
                f32x4 va = *(const f32x4*)(ctile + r * TP + tc) + bn0;
                f32x4 vb = *(const f32x4*)(ctile + r * TP + tc + 4) + bn1;
                if constexpr (RS) {  // the residual branch's per-sample stochastic-depth scale (training)
                    const float sc = p.row_scale[min(m, M - 1) / p.row_scale_div];
                    va *= sc;
                    vb *= sc;
                }
                const f32x4 sa = va + ra[i], sb = vb + rb[i];
                if (stats_out) {  // as the general path
                    float ps = 0.f, pq = 0.f;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const f32x2 u = unpack2<T>(pack2<T>(j < 2 ? sa[2 * j] : sb[2 * j - 4], j < 2 ? sa[2 * j + 1] : sb[2 * j - 3]));
                        ps += u[0] + u[1];
                        pq = fmaf(u[0], u[0], fmaf(u[1], u[1], pq));
                    }
                    ps = sum8_lanes(ps);
                    pq = sum8_lanes(pq);
                    if ((tc & 63) == 0 && m < M && n < N)
                        *(f32x2*)(stats_out + ((int64_t)m * (N / 64) + n / 64) * 2) = f32x2{ps, pq};
                }
                if (m < M && n < N) {
                    const int64_t e = (int64_t)m * p.ldc + n;
                    *(f32x4*)((float*)C + e) = sa;
                    *(f32x4*)((float*)C + e + 4) = sb;
                    if (C2)
                        *(u32x4*)((T*)C2 + e) = u32x4{pack2<T>(sa[0], sa[1]), pack2<T>(sa[2], sa[3]),
                                                      pack2<T>(sb[0], sb[1]), pack2<T>(sb[2], sb[3])};
                }
            }
        }
    } else {
#pragma unroll
    for (int p0 = 0; p0 < NPASS; p0 += PG) {
        f32x4 ra[PG], rb[PG];
#pragma unroll
        for (int i = 0; i < PG; ++i) {
            ra[i] = rb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
            if constexpr (RPRE) {
                if (rpre) {
                    ra[i] = rpa[p0 + i];
                    rb[i] = rpb[p0 + i];
                    continue;
                }
            }
            if (R) rload(min(m0 + tr + (p0 + i) * RPP, M - 1), nc, ra[i], rb[i]);  // wave-uniform test; clamped row
        }
#pragma unroll
        for (int i = 0; i < PG; ++i) {
            const int r = tr + (p0 + i) * RPP, m = m0 + r;
            f32x4 va = *(const f32x4*)(ctile + r * TP + tc);
            f32x4 vb = *(const f32x4*)(ctile + r * TP + tc + 4);
            if (MMT_GEMM_ABLATE == 4) va = vb = f32x4{(float)r, (float)tc, 0.f, 1.f};  // measurement: no tile reads
            if constexpr (LNF) {  // Linear(LayerNorm(x)) = rstd * (x.W' - mu * colsum(W')) + b'
                float sx = 0.f, sxx = 0.f;
                constexpr int NQ = LNM == 1 ? KS : 1;  // LNM 2: one (sum, sum x^2) pair per row
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    sx += rstat[(q * BM + ep * EB + r) * 2];
                    sxx += rstat[(q * BM + ep * EB + r) * 2 + 1];
                }
                const float mu = sx * inv_k, var = fmaxf(sxx * inv_k - mu * mu, 0.f);
                const float rstd = rsqrtf(var + p.ln_eps);
                va = (va - mu * cs0) * rstd;
                vb = (vb - mu * cs1) * rstd;
            }
            va += bn0;
            vb += bn1;
            const f32x4 prea = va, preb = vb;  // pre-activation (c2_copy 2)
            if (p.act == 5) {  // GELU backward: (acc + bias) * GELU'(R), R not added
                const f32x2 g0 = gelu_erf_grad2(ra[i].xy), g1 = gelu_erf_grad2(ra[i].zw);
                const f32x2 g2 = gelu_erf_grad2(rb[i].xy), g3 = gelu_erf_grad2(rb[i].zw);
                va = f32x4{va[0] * g0[0], va[1] * g0[1], va[2] * g1[0], va[3] * g1[1]};
                vb = f32x4{vb[0] * g2[0], vb[1] * g2[1], vb[2] * g3[0], vb[3] * g3[1]};
                ra[i] = rb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
            if (p.act == 1) {
                va.xy = gelu_erf2(va.xy);
                va.zw = gelu_erf2(va.zw);
                vb.xy = gelu_erf2(vb.xy);
                vb.zw = gelu_erf2(vb.zw);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (p.act == 2) {
                    va[j] = fmaxf(va[j], 0.f);
                    vb[j] = fmaxf(vb[j], 0.f);
                }
            }
            if constexpr (RS) {  // per-sample stochastic depth of a residual branch (row_scale; training only:
                                 // a run-time test here cost the inference frame ~1 %)
                const float sc = p.row_scale[min(m, M - 1) / p.row_scale_div];
                va *= sc;
                vb *= sc;
            }
            const f32x4 sa = va + ra[i], sb = vb + rb[i];  // + residual
            const bool split_c2 = C2 && !p.c2_copy;           // C = v, C2 = v + R
            const f32x4 oa = split_c2 ? va : sa, ob = split_c2 ? vb : sb;
            if (stats_out) {  // the next LayerNorm's row statistics over this 64-column group, taken
                              // on the 16-bit values C2 holds (what the consumer's A fragments hold)
                float ps = 0.f, pq = 0.f;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const f32x2 u = unpack2<T>(pack2<T>(j < 2 ? sa[2 * j] : sb[2 * j - 4], j < 2 ? sa[2 * j + 1] : sb[2 * j - 3]));
                    ps += u[0] + u[1];
                    pq = fmaf(u[0], u[0], fmaf(u[1], u[1], pq));
                }
                ps = sum8_lanes(ps);  // the group's 8 threads are 8 consecutive lanes
                pq = sum8_lanes(pq);
                if ((tc & 63) == 0 && m < M && n < N)
                    *(f32x2*)(stats_out + (crow(m) * (N / 64) + n / 64) * 2) = f32x2{ps, pq};
            }
            if (m < M && n < N && (MMT_GEMM_ABLATE != 3 || oa[0] == -1.2345e30f)) {  // (3: measurement, no stores)
                const int64_t e = crow(m) * p.ldc + n, es = colsplit ? crow(m) * 8 : e;
                if (colsplit && p.c2_copy == 4) {
                    ((float*)Cs)[crow(m)] = oa[0];  // (fp32 outputs: the launcher checks)
                } else if (p.c_f32) {
                    *(f32x4*)((float*)Cs + es) = oa;
                    *(f32x4*)((float*)Cs + es + 4) = ob;
                    if (C2 && p.c2_copy == 2) {  // the pre-activation in the compute dtype
                        *(u32x4*)((T*)C2 + e) = u32x4{pack2<T>(prea[0], prea[1]), pack2<T>(prea[2], prea[3]),
                                                      pack2<T>(preb[0], preb[1]), pack2<T>(preb[2], preb[3])};
                    } else if (C2 && p.c2_copy) {  // compute-dtype copy of C (the next LayerNorm-folded GEMM's A)
                        *(u32x4*)((T*)C2 + e) = u32x4{pack2<T>(sa[0], sa[1]), pack2<T>(sa[2], sa[3]),
                                                      pack2<T>(sb[0], sb[1]), pack2<T>(sb[2], sb[3])};
                    } else if (C2) {
                        *(f32x4*)((float*)C2 + e) = sa;
                        *(f32x4*)((float*)C2 + e + 4) = sb;
                    }
                } else {
                    *(u32x4*)((T*)Cs + es) = u32x4{pack2<T>(oa[0], oa[1]), pack2<T>(oa[2], oa[3]),
                                                 pack2<T>(ob[0], ob[1]), pack2<T>(ob[2], ob[3])};
                    if (C2 && p.c2_copy == 2)
                        *(u32x4*)((T*)C2 + e) = u32x4{pack2<T>(prea[0], prea[1]), pack2<T>(prea[2], prea[3]),
                                                      pack2<T>(preb[0], preb[1]), pack2<T>(preb[2], preb[3])};
                    else if (C2)
                        *(u32x4*)((T*)C2 + e) = u32x4{pack2<T>(sa[0], sa[1]), pack2<T>(sa[2], sa[3]),
                                                      pack2<T>(sb[0], sb[1]), pack2<T>(sb[2], sb[3])};
                }
            }
        }
    }
    }
    }  // epilogue passes
    MMT_STAMP(5, "s_memtime");
#if MMT_STAMP_BUILD
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    MMT_STAMP(6, "s_memtime");
    MMT_STAMP(7, "s_memrealtime");
}

// XCD-aware bijective remap of the launch's workgroup ids (see gemm.hip): each XCD gets a contiguous
// run of the linear ids, so a run's W column slices and A rows stay in that XCD's L2 and a tile's
// split-K partials are mostly written and summed on one XCD (speed only: the hand-off is correct
// for any placement).
MMT_DEV int gemm_xcd_lin() {
    const int nwg = gridDim.x * gridDim.y * gridDim.z;
    const int orig = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
    return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
}

// One GEMM: grid (tiles, split-K slices, groups); linear ids (group, tile, slice), slice fastest.
template <typename T, int BM, int BN, int WGM, int WGN, int KS, int ST, bool CONV, int LNM, int EPI = 0>
__global__ __launch_bounds__(64 * WGM * WGN * KS)
    __attribute__((amdgpu_waves_per_eu(WGM * WGN * KS / 4, WGM * WGN * KS / 4))) void gemm_glds_kernel(
        const mmt_gemm_params p) {
    const int nsk = gridDim.y;  // split-K slices per tile
    const int lin = gemm_xcd_lin();
    const int per_g = gridDim.x * nsk;
    const int g = lin / per_g, rem_t = lin - g * per_g;
    const int tile = rem_t / nsk, slice = rem_t - tile * nsk;
    gemm_glds_tile<T, BM, BN, WGM, WGN, KS, ST, CONV, LNM, 1, false, EPI>(p, g, tile, slice, nsk, gridDim.x);
}

// The same tile at two workgroups per CU (impl 8: 128x128, 8 waves, 2-slot ring = 64 KiB of LDS, <= 128
// VGPRs): one workgroup's prologue / epilogue runs beside the other's K loop on the CU, which the one-
// workgroup-per-CU tiles cannot overlap (large-M grids of short K: the training step's K = 768 GEMMs).
// (LNM 2: the LayerNorm fold on handed-in statistics, round 5 -- the inference qkv / fc1 of config 3)
template <typename T, int BM, int BN, int WGM, int WGN, int KS, int ST, bool RS = false, int EPI = 0, int LNM = 0>
__global__ __launch_bounds__(64 * WGM * WGN * KS)
    __attribute__((amdgpu_waves_per_eu(WGM * WGN * KS / 2, WGM * WGN * KS / 2))) void gemm_glds_kernel_occ2(
        const mmt_gemm_params p) {
    const int nsk = gridDim.y;
    const int lin = gemm_xcd_lin();
    const int per_g = gridDim.x * nsk;
    const int g = lin / per_g, rem_t = lin - g * per_g;
    const int tile = rem_t / nsk, slice = rem_t - tile * nsk;
    gemm_glds_tile<T, BM, BN, WGM, WGN, KS, ST, false, LNM, 2, RS, EPI>(p, g, tile, slice, nsk, gridDim.x);
}

// impl 8's tile with MN-major operands (LNM 3: W; 4: A and W)
template <typename T, int LNM, int EPI = 0>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 4))) void gemm_glds_kernel_occ2_t(
    const mmt_gemm_params p) {
    const int nsk = gridDim.y;
    const int lin = gemm_xcd_lin();
    const int per_g = gridDim.x * nsk;
    const int g = lin / per_g, rem_t = lin - g * per_g;
    const int tile = rem_t / nsk, slice = rem_t - tile * nsk;
    gemm_glds_tile<T, 128, 128, 2, 4, 1, 2, false, LNM, 2, false, EPI>(p, g, tile, slice, nsk, gridDim.x);
}

// impl 9: the 256x256 tile at one wave per SIMD (4 waves of 128x128, accumulators in AGPRs), one workgroup per
// CU; plain GEMM mode, optionally with the LayerNorm fold on handed-in statistics (LNM 2) or the row scale (RS)
#if MMT_GEMM_AB
template <typename T, int LNM, bool RS = false, int EPI = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_glds_kernel_w4(
    const mmt_gemm_params p) {
    const int lin = gemm_xcd_lin();
    const int g = lin / gridDim.x, tile = lin - g * gridDim.x;
    gemm_glds_tile<T, 256, 256, 2, 2, 1, 2, false, LNM, 1, RS, EPI>(p, g, tile, 0, 1, gridDim.x);
}
#endif

// Several independent GEMMs of one kernel configuration in one launch (mmt_gemm_multi): problem i
// owns the remapped linear ids [wg0[i], wg0[i + 1]), (group, tile) with the tile fastest, no split-K.
// The head's parallel conv chains and the fusion encoder's value / offset Linears are each a
// handful of workgroups, so side by side they share one launch's latency instead of paying it twice.
constexpr int GEMM_MULTI = 4;
struct gemm_multi_args {
    mmt_gemm_params p[GEMM_MULTI];
    int32_t wg0[GEMM_MULTI + 1];
    int32_t tiles[GEMM_MULTI];
    int32_t n;
};

template <typename T, int BM, int BN, int WGM, int WGN, int KS, int ST, bool CONV>
__global__ __launch_bounds__(64 * WGM * WGN * KS)
    __attribute__((amdgpu_waves_per_eu(WGM * WGN * KS / 4, WGM * WGN * KS / 4))) void gemm_glds_multi_kernel(
        const gemm_multi_args a) {
    const int lin = gemm_xcd_lin();
    int i = 0;
    while (i + 1 < a.n && lin >= a.wg0[i + 1]) ++i;  // wave-uniform (scalar)
    const int loc = lin - a.wg0[i], nt = a.tiles[i];
    const int g = loc / nt;
    gemm_glds_tile<T, BM, BN, WGM, WGN, KS, ST, CONV, 0>(a.p[i], g, loc - g * nt, 0, 1, nt);
}

// Whether the compact 16-bit epilogue (EPI 1) covers the GEMM's epilogue (bias, folded LayerNorm, ReLU / GELU,
// the pre-activation copy of c2_copy 2).
bool compact_epilogue(const mmt_gemm_params& p) {
    // an output row map (the template K/V cache passes' qkv rows into the [S][ntok] cache) is fine; not with
    // c2_copy 2's pre-activation copy, which is stored at the plain row
    if (p.c_f32 || (p.c2_copy != 0 && p.c2_copy != 2) || (p.c_seg_rows && p.c2_copy == 2) || p.row_scale ||
        p.act < 0 || p.act > 2)
        return false;
    for (int g = 0; g < p.groups; ++g)  // C2 only as c2_copy 2's pre-activation copy
        if (p.r[g] || p.ln_stats_out[g] || (p.c2[g] != nullptr) != (p.c2_copy == 2)) return false;
    return true;
}

// Whether the compact residual-producer epilogue (EPI 2) covers it: fp32 C = acc + bias (+ R, plain rows),
// C2 (if any) its 16-bit copy (c2_copy 1), LayerNorm statistics out (with C2) -- no activation, row map or scale.
bool residual_epilogue(const mmt_gemm_params& p, bool rs = false) {  // rs: a row-scale (RS) kernel
    if (!p.c_f32 || p.act || p.c_seg_rows || (p.row_scale != nullptr) != rs || p.r_mode || p.r_t || p.ln_fold) return false;
    for (int g = 0; g < p.groups; ++g) {
        if (p.c2[g] && p.c2_copy != 1) return false;
        if (!p.c2[g] && (p.c2_copy || p.ln_stats_out[g])) return false;
    }
    return true;
}

template <typename T, int BM, int BN, int WGM, int WGN, int KS, int ST>
void launch(const mmt_gemm_params& p, int nsk, hipStream_t st) {
    const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
    const dim3 grid(tiles, nsk, p.groups), block(64 * WGM * WGN * KS);
    if (p.conv_h == 0 && p.ln_fold != 1 && compact_epilogue(p)) {  // (LayerNorm folded with handed-in statistics or none)
        if (p.ln_fold == 2)
            hipLaunchKernelGGL((gemm_glds_kernel<T, BM, BN, WGM, WGN, KS, ST, false, 2, 1>), grid, block, 0, st, p);
        else
            hipLaunchKernelGGL((gemm_glds_kernel<T, BM, BN, WGM, WGN, KS, ST, false, 0, 1>), grid, block, 0, st, p);
        return;
    }
    if (p.conv_h == 0 && residual_epilogue(p)) {
        hipLaunchKernelGGL((gemm_glds_kernel<T, BM, BN, WGM, WGN, KS, ST, false, 0, 2>), grid, block, 0, st, p);
        return;
    }
    if (p.conv_h > 0 && compact_epilogue(p))  // the corner head's plain conv + ReLU layers
        hipLaunchKernelGGL((gemm_glds_kernel<T, BM, BN, WGM, WGN, KS, ST, true, 0, 1>), grid, block, 0, st, p);
    else if (p.conv_h > 0)
        hipLaunchKernelGGL((gemm_glds_kernel<T, BM, BN, WGM, WGN, KS, ST, true, 0>), grid, block, 0, st, p);
    else if (p.ln_fold == 2)
        hipLaunchKernelGGL((gemm_glds_kernel<T, BM, BN, WGM, WGN, KS, ST, false, 2>), grid, block, 0, st, p);
    else if (p.ln_fold)
        hipLaunchKernelGGL((gemm_glds_kernel<T, BM, BN, WGM, WGN, KS, ST, false, 1>), grid, block, 0, st, p);
    else
        hipLaunchKernelGGL((gemm_glds_kernel<T, BM, BN, WGM, WGN, KS, ST, false, 0>), grid, block, 0, st, p);
}

// impl 9's launch: 1 when the mode is not one it takes (LayerNorm summed in the K loop, conv, MN-major operands)
template <typename T>
int launch_w4(const mmt_gemm_params& p, hipStream_t st) {
#if !MMT_GEMM_AB
    return 1;  // A/B build only
#else
    if ((p.ln_fold != 0 && p.ln_fold != 2) || p.conv_h > 0 || p.a_t || p.w_t) return 1;
    const dim3 grid((unsigned)(((p.M + 255) / 256) * ((p.N + 255) / 256)), 1, p.groups), block(256);
    if (p.row_scale) {
        if (p.ln_fold) return 1;
        if (residual_epilogue(p, true)) hipLaunchKernelGGL((gemm_glds_kernel_w4<T, 0, true, 2>), grid, block, 0, st, p);
        else hipLaunchKernelGGL((gemm_glds_kernel_w4<T, 0, true>), grid, block, 0, st, p);
    } else if (p.ln_fold == 2) {
        if (compact_epilogue(p)) hipLaunchKernelGGL((gemm_glds_kernel_w4<T, 2, false, 1>), grid, block, 0, st, p);
        else hipLaunchKernelGGL((gemm_glds_kernel_w4<T, 2>), grid, block, 0, st, p);
    } else if (compact_epilogue(p)) {
        hipLaunchKernelGGL((gemm_glds_kernel_w4<T, 0, false, 1>), grid, block, 0, st, p);
    } else if (residual_epilogue(p)) {
        hipLaunchKernelGGL((gemm_glds_kernel_w4<T, 0, false, 2>), grid, block, 0, st, p);
    } else {
        hipLaunchKernelGGL((gemm_glds_kernel_w4<T, 0>), grid, block, 0, st, p);
    }
    return 0;
#endif
}

bool aligned(const void* ptr, int bytes) { return ((uintptr_t)ptr & (uintptr_t)(bytes - 1)) == 0; }

// Whether the shape / layout is one the LDS-DMA kernel takes.
bool glds_takes(const mmt_gemm_params& p) {
    if (p.K % 8 || p.N % 8 || p.ldc % 8 || (p.r[0] && p.ldr % 8)) return false;
    if (p.ln_fold && p.conv_h > 0) return false;
    if (p.ln_fold == 2 && (p.a_seg_rows < p.M || p.k_split || p.K % 64 || p.K > 64 * 8 * 2)) return false;  // identity A map
    for (int g = 0; g < p.groups; ++g) {
        if (p.ln_fold == 2 && (!p.ln_stats_in[g] || !aligned(p.ln_stats_in[g], 8))) return false;
        if (p.ln_stats_out[g] && (!p.c2_copy || !p.c2[g] || p.N % 64 || !aligned(p.ln_stats_out[g], 8))) return false;
    }
    if (p.conv_h > 0) {  // the kernel's conv addressing: power-of-two upsample, 32-bit element offsets
        const int cup = p.conv_up, hi = p.conv_up > 0 ? p.conv_h / p.conv_up : 0;
        if (cup <= 0 || (cup & (cup - 1)) || hi * cup != p.conv_h) return false;
        const int64_t imgs = (p.M + (int64_t)p.conv_h * p.conv_h - 1) / ((int64_t)p.conv_h * p.conv_h);
        const int64_t pitch = p.a_stride_a > 0 ? p.a_stride_a : (int64_t)hi * hi;
        if ((imgs * pitch * (int64_t)p.lda + p.K) >= ((int64_t)1 << 32) || p.K >= (1 << 24)) return false;
    }
    if (p.lda % 8 || p.a_stride_a % 8 || p.a_stride_b % 8 || p.k_split % 8) return false;
    if (p.a_seg_rows > INT32_MAX || p.a_segs_a > INT32_MAX) return false;
    for (int g = 0; g < p.groups; ++g) {
        if (!aligned(p.c[g], 16) || (p.c2[g] && !aligned(p.c2[g], 16))) return false;
        if (p.bias[g] && !aligned(p.bias[g], 16)) return false;
        if (p.r[g] && !aligned(p.r[g], 16)) return false;
        if (p.ln_fold && (!p.ln_colsum[g] || !aligned(p.ln_colsum[g], 16))) return false;
    }
    return true;
}

// Cost model fitted to in-kernel stamps at batch 1 (tools/gemm_stamps.py): one workgroup per
// CU (>= 128 KiB of LDS each), so time ~ rounds of 256 workgroups x (fixed prologue +
// epilogue + K-steps per workgroup x time per step).  Per-step times are per-CU LDS-fill
// bound: 128x128 (32 KiB/step) ~0.52 us, 128x64 with 2 k-groups ~0.52 us per pair of
// steps, 64x64 with 2 k-groups ~0.33 us per pair.  A K split into n slices adds the partial
// tile round trip of the last-arriving slice (~0.8 us + 0.5 us per 64 KiB slab it reads).
// Large-M tiles (impl 5 / 6: 256x128 / 128x256, 8 waves with 64x64 wave tiles, 3-slot ring of
// 48 KiB stages): 1.5x the MFMA work per byte of LDS fill of 128x128, for grids of many rounds.
struct Cand { int cfg, bm, bn, ks; float fixed_us, step_us; };
constexpr Cand kCands[7] = {{1, 128, 128, 1, 6.0f, 0.52f}, {2, 128, 64, 2, 5.0f, 0.52f}, {3, 64, 64, 2, 3.2f, 0.33f},
                            {4, 128, 128, 1, 6.0f, 0.60f}, {5, 256, 128, 1, 7.0f, 0.70f}, {6, 128, 256, 1, 7.0f, 0.70f},
                            {7, 256, 256, 1, 9.0f, 1.33f}};
int64_t tiles_of(const mmt_gemm_params& p, int bm, int bn) {
    return (int64_t)((p.M + bm - 1) / bm) * ((p.N + bn - 1) / bn);
}

}  // namespace

// Returns 1 when the shape / layout is not one this kernel takes (caller uses gemm.hip's kernel).
template <typename T>
int mmt_gemm_glds(const mmt_gemm_params& p, hipStream_t st, int force) {
    if (force < 0 || !glds_takes(p)) return 1;
    const int nk = (p.K + 63) / 64;
    const Cand* cands = kCands;
    // largest split the workspace allows for a candidate (each slice keeps >= ks K-steps)
    auto max_split = [&](const Cand& c) -> int {
        if (p.ln_fold || !p.sk_ws || !p.sk_cnt) return 1;
        const int64_t t = tiles_of(p, c.bm, c.bn) * p.groups;
        if (2 * t > p.sk_cnt_n) return 1;  // a ticket and a published count per tile
        int n = 8;
        while (n > 1 && ((int64_t)n * c.ks > nk || t * n * c.bm * c.bn > p.sk_ws_floats)) --n;
        return n;
    };
    auto cost = [&](const Cand& c, int n) {
        const int64_t wg = tiles_of(p, c.bm, c.bn) * p.groups * n;
        const int steps = (nk + n - 1) / n;
        const float red = n > 1 ? 0.8f + 0.5f * (float)(n - 1) * (float)(c.bm * c.bn) / 16384.f : 0.f;
        return (float)((wg + 255) / 256) * (c.fixed_us + (float)((steps + c.ks - 1) / c.ks) * c.step_us) + red;
    };
    int cfg = force, nsk = 1;
    if (p.row_scale) {  // the training step's residual branches: impl 8's tile with the row-scale epilogue
        if (force == 9) return launch_w4<T>(p, st);
        if ((force != 0 && force != 8) || p.ln_fold || p.conv_h > 0 || p.a_t || p.w_t) return 1;
        const dim3 grid((unsigned)tiles_of(p, 128, 128), 1, p.groups);
        if (residual_epilogue(p, true))
            hipLaunchKernelGGL((gemm_glds_kernel_occ2<T, 128, 128, 2, 4, 1, 2, true, 2>), grid, dim3(512), 0, st, p);
        else
            hipLaunchKernelGGL((gemm_glds_kernel_occ2<T, 128, 128, 2, 4, 1, 2, true>), grid, dim3(512), 0, st, p);
        return 0;
    }
    if (p.a_t || p.w_t) {  // MN-major operands: the 128x128 tiles (impl 1, or impl 8 on big unsplit grids)
        if (force != 0 && force != 1 && force != 8) return 1;
        const int64_t t8 = tiles_of(p, 128, 128) * p.groups;
        const bool big = t8 > 256;
        const Cand& c = cands[0];
        // Round 6: the weight gradients (A and W MN-major) of >= MMT_GEMM_SK8_MIN tiles on impl 8 with the K split
        // that fills ~480 of the 512 two-per-CU slots (the register hand-off above).  Isolated, two groups of 8448
        // tokens (profiles/r06_sk8_gemm_ab.jsonl): dW of qkv 104.1 -> 100.3 us (impl 1 unsplit -> 2 slices), proj
        // 49.7 -> 43.7 (impl 1 / 3 slices -> 6), fc1 144.6 -> 136.5 and fc2 134.8 -> 131.8 (impl 8 unsplit -> 2).
        // The input gradients (W only MN-major) stay unsplit: every split measured slower (dX of fc1 108.7 -> 133).
        if (force == 0 && p.a_t && t8 >= MMT_GEMM_SK8_MIN && p.splitk == 0 && max_split(c) > 1) {
            cfg = 8;
            nsk = (int)std::min<int64_t>(max_split(c), (480 + t8 - 1) / t8);
        } else if (force == 1 || (force == 0 && !big)) {
            cfg = 1;
            const int nmax = p.splitk >= 1 ? std::min(p.splitk, max_split(c)) : max_split(c);
            float best = 1e30f;
            for (int n = (p.splitk >= 2 ? nmax : 1); n <= nmax; ++n) {
                const float t = cost(c, n) * (n > 1 && p.splitk == 0 ? 1.15f : 1.f);
                if (t < best) best = t, nsk = n;
            }
        } else {
            cfg = 8;
            if (p.splitk >= 2) nsk = std::min(p.splitk, max_split(c));  // forced slice count (A/B tools)
        }
        const int lnm = p.a_t ? 4 : 3;
        const dim3 grid((unsigned)tiles_of(p, 128, 128), nsk, p.groups);
        if (cfg == 8) {
            if (lnm == 4) hipLaunchKernelGGL((gemm_glds_kernel_occ2_t<T, 4>), grid, dim3(512), 0, st, p);
            else if (compact_epilogue(p)) hipLaunchKernelGGL((gemm_glds_kernel_occ2_t<T, 3, 1>), grid, dim3(512), 0, st, p);
            else hipLaunchKernelGGL((gemm_glds_kernel_occ2_t<T, 3>), grid, dim3(512), 0, st, p);
        } else {
            if (lnm == 4) hipLaunchKernelGGL((gemm_glds_kernel<T, 128, 128, 2, 4, 1, 4, false, 4>), grid, dim3(512), 0, st, p);
            else hipLaunchKernelGGL((gemm_glds_kernel<T, 128, 128, 2, 4, 1, 4, false, 3>), grid, dim3(512), 0, st, p);
        }
        return 0;
    }
    if (cfg == 0) {
        float best = 1e30f;
        // 128x256 (impl 6) only for grids of more than one round of 128x128 tiles: the batch-1 grids
        // (<= 240 tiles) keep their shapes; the large-M ones gain (gemm_ab.py: training dW 481-554 ->
        // 635-640 TFLOP/s, batch-8 fc2 571 -> 680; profiles/r03_gemm_large_vs_hipblaslt.jsonl)
        const bool big = tiles_of(p, 128, 128) * p.groups > 256;
        // 256x256 (impl 7): plain GEMMs only (no folded LayerNorm, no conv, no split-K), and not under a
        // GELU epilogue, whose four-pass form measured slower (fc1 at 16 pairs: 515 vs 565 TFLOP/s)
        const bool big7 = big && !p.ln_fold && p.conv_h == 0 && p.act != 1;
        for (int ci = 0; ci < (big7 ? 7 : big ? 6 : 3); ++ci) {
            if (ci == 3 || ci == 4) continue;  // impl 4 / 5: A/B only
            if (ci == 6) {  // impl 7: no split-K
                const float t = cost(cands[ci], 1);
                if (t < best) best = t, cfg = 7, nsk = 1;
                continue;
            }
            const Cand& c = cands[ci];
            const int nmax = p.splitk >= 1 ? std::min(p.splitk, max_split(c)) : max_split(c);
            for (int n = (p.splitk >= 2 ? nmax : 1); n <= nmax; ++n) {
                // a split must win clearly: the model prices the partial round trip loosely
                const float t = cost(c, n) * (n > 1 && p.splitk == 0 ? 1.15f : 1.f);
                if (t < best) best = t, cfg = c.cfg, nsk = n;
            }
        }
        // 128x128 at two workgroups per CU (impl 8) instead of a one-per-CU 128x128 / 256x128 / 128x256 tile
        // on big unsplit plain grids: 1.14-1.25x impl 1 and 1.02-1.16x the model's pick on the training
        // step's forward / dX shapes and batch-8 fc1 / fc2 (profiles/r03_gemm_occ2_ab.jsonl); the
        // 256x256 tile (impl 7) keeps its shapes (dX of fc2: 597 vs 525 TFLOP/s)
        // Not for the inference residual producers (C2 copy + LayerNorm statistics out: config 3 at 64
        // sequences 2650 -> 2541 frames/s with them on impl 8, interleaved, profiles/r03_gemm_occ2_ab.jsonl)
        // Round 5: also instead of impl 7, since impl 8's row-group tile order (above) it is faster on every
        // shape impl 7 took (two groups of 8448 rows: qkv 102.0 -> 81.5 us, the dX-like N 3072 / K 768 129.1 ->
        // 104.3 us; profiles/r05_gemm_w4_ab.jsonl)
        // Round 5: and for the residual producers with the LayerNorm-statistics hand-off (round 3 kept them off: config 3
        // at 64 sequences 2650 -> 2541 frames/s; with the row-group order the proj entry of that plan runs 211.5 ->
        // 180.4 us, fc2 444.0 -> 445.0, profiles/r05_c3_entry_ab.jsonl)
        // and (round 5) for the LayerNorm fold on handed-in statistics, whatever tile the model picked (config 3's qkv /
        // fc1 in the plan at 64 / 8 sequences: qkv 332.4 -> 321.8 / 51.9 -> 48.2 us, fc1 486.7 -> 484.2 / 69.6 -> 67.8,
        // profiles/r05_c3_ln2_ab.jsonl)
        if (!MMT_GEMM_NO_OCC2 && big && nsk == 1 && p.ln_fold != 1 && p.conv_h == 0 &&
            (MMT_GEMM_OCC2_RES || !p.ln_stats_out[0]) &&
            (cfg == 1 || cfg == 5 || cfg == 6 || cfg == 7 || (p.ln_fold == 2 && (cfg == 2 || cfg == 3))))
            cfg = 8;
    } else if (cfg == 8) {
        nsk = 1;  // impl 8: no split-K
    } else if (cfg >= 1 && cfg <= 7) {
        const Cand& c = cands[cfg - 1];
        if (p.splitk >= 2) {
            nsk = std::min(p.splitk, max_split(c));
        } else if (p.splitk == 0) {
            float best = 1e30f;
            for (int n = 1; n <= max_split(c); ++n) {
                const float t = cost(c, n) * (n > 1 ? 1.15f : 1.f);
                if (t < best) best = t, nsk = n;
            }
        }
    }
    switch (cfg) {
        case 1: launch<T, 128, 128, 2, 4, 1, 4>(p, nsk, st); break;
        case 2: launch<T, 128, 64, 2, 2, 2, 3>(p, nsk, st); break;
        case 3: launch<T, 64, 64, 2, 2, 2, 4>(p, nsk, st); break;
        case 4: launch<T, 128, 128, 2, 2, 1, 4>(p, nsk, st); break;
        case 5: launch<T, 256, 128, 4, 2, 1, 3>(p, nsk, st); break;
        case 6: launch<T, 128, 256, 2, 4, 1, 3>(p, nsk, st); break;
        case 7:
            if (p.ln_fold || p.conv_h > 0 || nsk > 1) return 1;
            hipLaunchKernelGGL((gemm_glds_kernel<T, 256, 256, 4, 2, 1, 2, false, 0>),
                               dim3((unsigned)tiles_of(p, 256, 256), 1, p.groups), dim3(512), 0, st, p);
            break;
        case 8:  // 128x128 at two workgroups per CU: plain GEMM mode (LayerNorm fold only with handed-in statistics, no
                 // conv), and no split-K: its 64 KiB ring holds the fp32 tile image only in two passes (as impl 7)
            if (p.ln_fold == 1 || p.conv_h > 0 || nsk > 1) return 1;
            {
                const dim3 grid((unsigned)tiles_of(p, 128, 128), nsk, p.groups);
                if (p.ln_fold == 2) {
                    if (compact_epilogue(p))
                        hipLaunchKernelGGL((gemm_glds_kernel_occ2<T, 128, 128, 2, 4, 1, 2, false, 1, 2>), grid, dim3(512), 0, st, p);
                    else
                        hipLaunchKernelGGL((gemm_glds_kernel_occ2<T, 128, 128, 2, 4, 1, 2, false, 0, 2>), grid, dim3(512), 0, st, p);
                } else if (compact_epilogue(p))
                    hipLaunchKernelGGL((gemm_glds_kernel_occ2<T, 128, 128, 2, 4, 1, 2, false, 1>), grid, dim3(512), 0, st, p);
                else if (residual_epilogue(p))
                    hipLaunchKernelGGL((gemm_glds_kernel_occ2<T, 128, 128, 2, 4, 1, 2, false, 2>), grid, dim3(512), 0, st, p);
                else
                    hipLaunchKernelGGL((gemm_glds_kernel_occ2<T, 128, 128, 2, 4, 1, 2>), grid, dim3(512), 0, st, p);
            }
            break;
        case 9: return launch_w4<T>(p, st);
        default: return 1;
    }
    return 0;
}

namespace {
template <typename T, int BM, int BN, int WGM, int WGN, int KS, int ST>
void launch_multi(const mmt_gemm_params* ps, int n, bool conv, hipStream_t st) {
    gemm_multi_args a{};
    a.n = n;
    a.wg0[0] = 0;
    for (int i = 0; i < n; ++i) {
        a.p[i] = ps[i];
        a.tiles[i] = (int32_t)tiles_of(ps[i], BM, BN);
        a.wg0[i + 1] = a.wg0[i] + a.tiles[i] * ps[i].groups;
    }
    const dim3 grid(a.wg0[n]), block(64 * WGM * WGN * KS);
    if (conv) hipLaunchKernelGGL((gemm_glds_multi_kernel<T, BM, BN, WGM, WGN, KS, ST, true>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((gemm_glds_multi_kernel<T, BM, BN, WGM, WGN, KS, ST, false>), grid, block, 0, st, a);
}
}  // namespace

// n independent GEMMs in one launch; returns 1 when some problem is not one the LDS-DMA kernel
// takes in this mode (all GEMM or all conv, no folded LayerNorm, no split-K, one forced impl).  The
// configuration is chosen once for the union: rounds of 256 workgroups over all problems times the
// slowest problem's per-workgroup time (the cost model above).
template <typename T>
int mmt_gemm_glds_multi(const mmt_gemm_params* ps, int n, hipStream_t st) {
    if (n < 1 || n > GEMM_MULTI) return 1;
    const bool conv = ps[0].conv_h > 0;
    const int force = ps[0].impl;
    for (int i = 0; i < n; ++i) {
        const mmt_gemm_params& p = ps[i];
        if (!glds_takes(p) || (p.conv_h > 0) != conv || p.ln_fold || p.impl != force || force < 0 || force > 4 ||
            p.a_t || p.w_t)
            return 1;
    }
    int cfg = force;
    if (cfg == 0) {
        float best = 1e30f;
        for (int ci = 0; ci < 3; ++ci) {
            const Cand& c = kCands[ci];
            int64_t wg = 0;
            float slowest = 0.f;
            for (int i = 0; i < n; ++i) {
                wg += tiles_of(ps[i], c.bm, c.bn) * ps[i].groups;
                const int steps = (ps[i].K + 63) / 64;
                slowest = std::max(slowest, c.fixed_us + (float)((steps + c.ks - 1) / c.ks) * c.step_us);
            }
            const float t = (float)((wg + 255) / 256) * slowest;
            if (t < best) best = t, cfg = c.cfg;
        }
    }
    int64_t wg_total = 0;
    for (int i = 0; i < n; ++i) wg_total += tiles_of(ps[i], kCands[cfg - 1].bm, kCands[cfg - 1].bn) * ps[i].groups;
    if (wg_total > INT32_MAX) return 1;
    switch (cfg) {
        case 1: launch_multi<T, 128, 128, 2, 4, 1, 4>(ps, n, conv, st); break;
        case 2: launch_multi<T, 128, 64, 2, 2, 2, 3>(ps, n, conv, st); break;
        case 3: launch_multi<T, 64, 64, 2, 2, 2, 4>(ps, n, conv, st); break;
        case 4: launch_multi<T, 128, 128, 2, 2, 1, 4>(ps, n, conv, st); break;
        default: return 1;
    }
    return 0;
}

template int mmt_gemm_glds<bf16_t>(const mmt_gemm_params&, hipStream_t, int);
template int mmt_gemm_glds<f16_t>(const mmt_gemm_params&, hipStream_t, int);
template int mmt_gemm_glds_multi<bf16_t>(const mmt_gemm_params*, int, hipStream_t);
template int mmt_gemm_glds_multi<f16_t>(const mmt_gemm_params*, int, hipStream_t);
