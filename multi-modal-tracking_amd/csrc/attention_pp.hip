// MAM attention, impl 24: the range-checked exponent kernel (impl 22's math: P = exp2(S) with no
// reference point, row sums on the matrix pipe, epilogue range check with the exact two-pass fallback)
// re-built for ONE wave per SIMD with an explicit software pipeline over 32-key blocks.
//
// Reference: Attention.forward, lib/models/mixformer_vit_rgbt/mixformer.py:52-78 and the cross-modal
// form asymmetric_shared.py:55-104 (template queries -> own template keys; search queries -> all keys,
// or [template_V | template_I | own search]).  Layouts as attention.hip: qkv [seq][token][3][head][64]
// read in place, out [seq][token][head * 64].
//
// Why a second structure.  At d = 64 a score carries 256 MFMA FLOPs against one v_exp_f32 (8 issue
// cycles per 64 scores) and half a v_cvt_pk_bf16_f32, so the vector issue of the softmax is ~90 % of the
// matrix-pipe time and the two have to overlap almost perfectly.  impl 22 leaves that overlap to two
// co-resident waves per SIMD (each with its own score -> exp -> PV chain per 64-key tile); PMC at B = 32
// shows the matrix pipe 29 % busy with each wave stalled on its own chain most of the time.  Here each
// SIMD runs one wave that owns the whole register file, and the chain is pipelined across blocks inside
// the wave.  Iteration i (32-key block i, the wave's 64 queries as two 32-query blocks):
//   phase 1:  PV(i - 1) MFMAs (8 x 32x32x16 + 4 row-sum 16x16x32)  beside  exp2 + pack of S(i), query
//             block 0, and the K fragment reads of block i + 1
//   phase 2:  QK^T(i + 1) MFMAs (8 x 32x32x16)                     beside  exp2 + pack of S(i), query
//             block 1, and the V^T fragment reads of block i
// so every exponential reads scores whose MFMAs were issued one phase earlier, every MFMA reads
// fragments read one phase earlier, and the phase's MFMAs are independent of its vector work.
// MFMA-pipe cycles per iteration 8 x 32 + 4 x 16 + 8 x 32 = 576 against ~550 issue cycles (32 v_exp,
// 16 v_cvt_pk, 20 MFMA issue slots, 12 LDS reads), i.e. the loop is designed to be matrix-bound.
//
// Geometry: 2 waves (128 queries of one (sequence, head)) per workgroup, two workgroups per CU (one
// wave per SIMD: the kernel's registers exceed the 256 a second wave could have).  K / V tiles of 64
// keys stream through a 4-slot LDS-DMA ring (wave 0 DMAs the K pieces, wave 1 the V pieces, images and
// swizzles of attention.hip), two tiles in flight; one barrier per tile, at the phase-1 start of the
// iteration whose K reads enter a new tile.  Q comes straight from global memory into registers.
// Counted-wait rule of attention.hip: no global store inside the loop (outputs after the last wait).
// Results are bit-identical to impl 22 (same MFMA order per accumulator, same exponentials).
#include "attn_common.hpp"

#ifndef MMT_ATTN_AB
#define MMT_ATTN_AB 0
#endif
#if MMT_ATTN_AB  // A/B build only (tools/build_ablate.sh ab): not faster than impl 22 / 4 anywhere

namespace {

// MMT_ATTN_ABLATE (measurement builds only, tools/build_ablate.sh; results are wrong): 1 = no K / V DMA
// after the prologue, 3 = no exponentials, 5 = free-running (no per-tile wait / barrier / refill), 7 = no
// K / V fragment reads in the steady-state loop, 8 = no s_nop before the PV MFMAs, 9 = no packs (P = S
// bits), 10 = no PV MFMAs in the steady-state loop, 11 = no QK^T MFMAs in the steady-state loop
#ifndef MMT_ATTN_ABLATE
#define MMT_ATTN_ABLATE 0
#endif

// LDS fragment reads as inline asm (invisible to hipcc's wait-count tracking, which would otherwise
// drain the LDS-DMA ring before each read); the waits are explicit (wait_k / wait_v below).
MMT_DEV u32x4 pp_b128(const char* p) {
    u32x4 r;
    const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
    asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(a));
    return r;
}

#if MMT_STAMP_BUILD
// measurement build (tools/build_ablate.sh stamp): per workgroup, wave 0: [0] realtime / [1] memtime at
// entry, [2] loop start, [3] loop end (before the last block), [4] end, [5] realtime end, [6] blocks, [7] nqa
__device__ unsigned long long g_mmt_attn_pp_stamps[16384 * 8];
extern "C" int mmt_attn_pp_stamps(unsigned long long* host, int n) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_mmt_attn_pp_stamps), sizeof(unsigned long long) * n);
}
#endif
#define MMT_PPSTAMP(I, INSN) MMT_STAMP_AT(g_mmt_attn_pp_stamps, I, INSN)

template <int NQ>
struct PPState {
    f32x16 o[NQ][2];  // O^T accumulators [query block][32-dim half]
    f32x4 lacc[NQ];   // row sums (every element = this lane's query)
};

// KS = key halves per workgroup: 1 (impl 24: 2 waves = 128 queries over all keys, two workgroups per CU)
// or 2 (impl 25, small grids such as batch-1 tracking: 4 waves, waves 2-3 take the second half of the
// 32-key blocks of the same 128 queries with their own K / V ring; without a reference point the halves'
// O and row sums simply add, through LDS at the end).
template <int KS>
__global__ __launch_bounds__(128 * KS) __attribute__((amdgpu_waves_per_eu(1, 1))) void mam_attention_pp_kernel(
    const mmt_attn_params p) {
    // K / V tile slots per key half: R - 2 tiles in flight ahead of the one being read (4: two workgroups
    // per CU; a 5-slot ring measured slower, B = 32 84.7 -> 92.0 us, profiles/r04_attn_pp_ab.jsonl)
    constexpr int PP_R = 4;
    __shared__ __attribute__((aligned(1024))) char lds_all[KS * PP_R * FTILE];
    MMT_PPSTAMP(0, "s_memrealtime");
    MMT_PPSTAMP(1, "s_memtime");
    int bx, h, s;
    attn_block_ids_xcd(bx, h, s);

    const int n_t = p.n_t, ntok = p.ntok, C = p.C;
    const int64_t pitch = p.tok_pitch > 0 ? p.tok_pitch : ntok;
    const int nqb_t = (n_t + FQ - 1) / FQ;
    const int qb0 = bx + (p.q_part == 2 ? nqb_t : 0);
    const bool tmpl = qb0 < nqb_t;
    const int q0 = tmpl ? qb0 * FQ : n_t + (qb0 - nqb_t) * FQ;
    const int qend = tmpl ? n_t : ntok;
    const int Lk = tmpl ? n_t : (p.asym ? ntok + n_t : ntok);
    const bool cross = p.asym && !tmpl;
    const int64_t rs = 3 * (int64_t)C;
    const bf16_t* qkv = (const bf16_t*)p.qkv;
    const int sV = s % p.Bm, sI = sV + p.Bm;

    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int l32 = lane & 31, hf = lane >> 5;
    const int prow = lane >> 3, pcol = lane & 7;
    const int wq = w & 1;                     // query wave: queries q0 + 64 wq + [0, 64)
    const int half = KS == 2 ? (w >> 1) : 0;  // key half
    char* lds = lds_all + half * PP_R * FTILE;
    // this half's 32-key blocks [kb0, kb0 + nb) of the nb_all blocks: keys k0 .. k0 + Lh - 1
    const int nb_all = (Lk + 31) / 32;
    const int nb_h0 = KS == 2 ? (nb_all + 1) / 2 : nb_all;
    const int kb0 = half ? nb_h0 : 0;
    const int nb = half ? nb_all - nb_h0 : nb_h0;
    const int k0 = 32 * kb0;
    const int Lh = min(Lk, 32 * (kb0 + nb)) - k0;

    // ---- K / V tiles of the half: wave 0 of the pair DMAs the 8 K pieces of a tile, wave 1 the 8 V pieces
    const int isv = wq;
    const int64_t col = (isv ? 2 * C : C) + h * D + (isv ? (pcol ^ attn_vswz(prow)) : (pcol ^ prow)) * 8;
    auto key_row = [&](int kk) -> const bf16_t* {
        int seq = s, row = kk;
        if (cross) {
            if (kk < n_t) seq = sV;
            else if (kk < 2 * n_t) { seq = sI; row = kk - n_t; }
            else row = kk - n_t;
        }
        return qkv + ((int64_t)seq * pitch + row) * rs;
    };
    const bool aligned = n_t % KB == 0 && k0 % KB == 0;
    const int nkt = nb > 0 ? (Lh + KB - 1) / KB : 0;  // tiles of this half
    // Full tiles inside one key segment (all but a tail) are DMA'd by buffer_load ... lds: the lane's
    // offset inside a piece (row prow, swizzled chunk) is a constant VGPR, the piece's row base a scalar
    // soffset, so a tile costs no vector instructions (a flat global_load_lds needs a 64-bit address
    // per piece: ~60 VALU per tile, a quarter of the kernel's vector issue at B = 32).
    const __amdgpu_buffer_rsrc_t qrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)qkv, 0, (int)min((int64_t)0x7fffffff, (int64_t)p.S * pitch * rs * 2), 0x00020000);
    const int lane_voff = (int)((prow * rs + col) * 2);
    typedef __attribute__((address_space(3))) void lds_void_t;
    auto issue_tile = [&](int t) {
        MMT_ATTN_ASSERT(t >= 0 && t < nkt);
        char* slot = lds + (t % PP_R) * FTILE + isv * KB * 128;
        if (aligned && t * KB + KB <= Lh) {
            const int kk = k0 + t * KB;  // wave-uniform: the tile's first key, its (sequence, row)
            int seq = s, row = kk;
            if (cross) {
                if (kk < n_t) seq = sV;
                else if (kk < 2 * n_t) { seq = sI; row = kk - n_t; }
                else row = kk - n_t;
            }
            const int soff = __builtin_amdgcn_readfirstlane((int)(((int64_t)seq * pitch + row) * rs * 2));
#pragma unroll
            for (int pk = 0; pk < 8; ++pk)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(qrs, (lds_void_t*)(slot + pk * 1024), 16, lane_voff,
                                                         soff + pk * 8 * (int)rs * 2, 0, 0);
        } else {
#pragma unroll
            for (int pk = 0; pk < 8; ++pk)
                attn_glds16(key_row(min(k0 + t * KB + pk * 8 + prow, Lk - 1)) + col, slot + pk * 1024);
        }
    };
    // barriers: each half syncs once per tile after its first; the halves' counts are evened out before
    // the merge (s_barrier is a workgroup-wide rendezvous)
    const int nkt_max = KS == 2 ? (min(Lk, 32 * nb_h0) + KB - 1) / KB : nkt;
    auto pad_barriers = [&]() {
        for (int t = max(nkt, 1); t < nkt_max; ++t) lds_barrier();
    };

    // ---- Q fragments straight from global memory (B operand of S^T = K Q^T: query l32 of the block,
    // d = 16 ks + 8 hf .. + 7); rows past the block's end re-read the last query.  Issued before the
    // first tiles, so the counted waits below cover them.
    const int qbase = q0 + 64 * wq;  // query blocks qbase + 32 qb + [0, 32)
    const int nqa = (qbase < qend ? 1 : 0) + (qbase + 32 < qend ? 1 : 0);
    u32x4 qf[2][4];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
        const bf16_t* qp = qkv + ((int64_t)s * pitch + min(qbase + 32 * qb + l32, qend - 1)) * rs + h * D;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) qf[qb][ks] = *(const u32x4*)(qp + (2 * ks + hf) * 8);
    }
    // prologue DMA: tiles 0 .. R - 2 (sync point t issues tile t + R - 2)
    for (int t = 0; t < PP_R - 1 && t < nkt; ++t) issue_tile(t);

    const float cexp = p.scale * 1.4426950408889634f;
    if (fabsf(cexp - 1.f) > 1e-6f) {  // natural-scale q: to log2 units
#pragma unroll
        for (int qb = 0; qb < 2; ++qb)
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                u32x4 v = qf[qb][ks];
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    v[e] = pack_bf16x2(__uint_as_float(v[e] << 16) * cexp, __uint_as_float(v[e] & 0xffff0000u) * cexp);
                qf[qb][ks] = v;
            }
    }

    // sync point of tile t (t >= 1): this wave's pieces of tile t landed (the R - 3 tiles after it may
    // still be in flight), every wave's (the barrier), and every wave is past the V reads of tile t - 2,
    // whose slot then takes tile t + R - 2.  Tile 0: the prologue wait.
    auto sync_tile = [&](int t) {
        if (MMT_ATTN_ABLATE == 5) return;
        attn_wait_dyn(8 * (min(nkt - 1, t + PP_R - 3) - t));
        lds_barrier();
        if (MMT_ATTN_ABLATE != 1 && t + PP_R - 2 < nkt) issue_tile(t + PP_R - 2);
    };
    attn_wait_dyn(8 * (max(0, min(nkt - 1, PP_R - 2))));
    lds_barrier();

    const int nvl = Lh - 32 * (nb - 1);  // keys of this half's last block
    // the halves' merge (KS = 2): half 1 leaves O and the row sums of its query wave in LDS (its own
    // ring, done with), half 0 adds them before its epilogue
    float* mrg = (float*)(lds_all + PP_R * FTILE) + wq * (4 * 16 * 64 + 2 * 64);
    if (nqa == 0 || nb == 0) {  // no queries / no keys: keep the workgroup's DMA / barrier schedule
        for (int t = 1; t < nkt; ++t) sync_tile(t);
        pad_barriers();
        if (KS == 2) lds_barrier();  // the merge (half 0 always has keys: it takes the longer half)
        return;
    }

    const float one_or_zero = (((lane & 15) >> 2) & 1) == ((lane >> 4) & 1) ? 1.f : 0.f;
    const uint32_t sel_w = pack_bf16x2(one_or_zero, one_or_zero);
    u32x4 sel_u = u32x4{sel_w, sel_w, sel_w, sel_w};
    const int kpos = (l32 & 7) * 16;
    const int li = lane & 15, qr = li >> 2, pc = li & 3, dsub = (lane >> 4) & 1;

    auto kimg_of = [&](int b) { return lds + ((b >> 1) % PP_R) * FTILE + (b & 1) * 32 * 128; };
    auto kread = [&](int b, u32x4 (&kf)[4]) {
        const char* krow = kimg_of(b) + l32 * 128;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) kf[ks] = pp_b128(krow + ((((2 * ks + hf) * 16) ^ kpos)));
    };
    auto vread = [&](int b, uint2 (&vt)[2][2][2]) {
        const char* vimg = lds + ((b >> 1) % PP_R) * FTILE + KB * 128;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int row = 32 * (b & 1) + 16 * j + 4 * hf + qr;
#pragma unroll
            for (int db = 0; db < 2; ++db) {
                const char* b1 = vimg + row * 128 + (((4 * db + 2 * dsub + (pc >> 1)) ^ attn_vswz(row)) * 16) + (pc & 1) * 8;
                vt[j][db][0] = attn_tr16<0>(b1);
                vt[j][db][1] = attn_tr16<8 * 128>(b1);
            }
        }
    };

    auto run = [&](auto NQc) {
        constexpr int NQ = decltype(NQc)::value;
        PPState<NQ> st;
#pragma unroll
        for (int qb = 0; qb < NQ; ++qb) {
#pragma unroll
            for (int r = 0; r < 16; ++r) { st.o[qb][0][r] = 0.f; st.o[qb][1][r] = 0.f; }
            st.lacc[qb] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        u32x4 kf[4];
        uint2 vt[2][2][2];
        // two score sets and two packed-P sets, their roles alternating with the block parity (named
        // registers: no copies between iterations)
        f32x16 sA[NQ], sB[NQ];
        u32x4 pA[NQ][2], pB[NQ][2];

        auto qk = [&](f32x16 (&dst)[NQ]) {
#pragma unroll
            for (int qb = 0; qb < NQ; ++qb) dst[qb] = f32x16{};
#pragma unroll
            for (int ks = 0; ks < 4; ++ks)
#pragma unroll
                for (int qb = 0; qb < NQ; ++qb)
                    dst[qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kf[ks]),
                                                                      __builtin_bit_cast(bf16x8, qf[qb][ks]), dst[qb], 0, 0, 0);
        };
        // O^T += V^T P^T and the row sums, on the accumulator registers (inline asm: the "a" constraint is
        // the only way to keep O out of the 256 architectural VGPRs, which the scores, P, Q and the
        // fragments need).  Hazards the compiler does not see through the asm, covered here: a VALU write
        // of an operand (the P pack, a tuple copy) needs 2 wait states before the MFMA reads it (s_nop 1);
        // the epilogue waits out the last MFMAs before reading O (pv_drain).  Back-to-back accumulation
        // into the same registers needs none.
        auto pv = [&](int qb, const u32x4 (&pb)[2]) {
            const u32x4 su = sel_u;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
#pragma unroll
                for (int db = 0; db < 2; ++db) {
                    const uint2 ua = vt[j][db][0], ub = vt[j][db][1];
                    const u32x4 vf = u32x4{ua.x, ua.y, ub.x, ub.y};
                    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0"
                                 : "+a"(st.o[qb][db]) : "v"(vf), "v"(pb[j]));
                }
                asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                             : "+a"(st.lacc[qb]) : "v"(su), "v"(pb[j]));
            }
        };
        auto pv_drain = [&]() {  // the last MFMAs' results (16 passes) before any VALU reads them
#pragma unroll
            for (int qb = 0; qb < NQ; ++qb)
                asm volatile("s_nop 15\n\ts_nop 15" : "+a"(st.o[qb][0]), "+a"(st.o[qb][1]), "+a"(st.lacc[qb]));
        };
        // P = exp2(S) of query block qb (scores in place; MASK: keys >= Lk of block b give 0), packed
        auto softmax = [&](f32x16& sv, int b, auto MASKc, u32x4 (&dst)[2]) {
            constexpr bool MASK = decltype(MASKc)::value;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float e = __builtin_amdgcn_exp2f(sv[r]);
                sv[r] = (!MASK || 32 * (kb0 + b) + 8 * (r >> 2) + 4 * hf + (r & 3) < Lk) ? e : 0.f;
            }
#pragma unroll
            for (int j = 0; j < 2; ++j)
                dst[j] = u32x4{pack_bf16x2(sv[8 * j], sv[8 * j + 1]), pack_bf16x2(sv[8 * j + 2], sv[8 * j + 3]),
                               pack_bf16x2(sv[8 * j + 4], sv[8 * j + 5]), pack_bf16x2(sv[8 * j + 6], sv[8 * j + 7])};
        };
        auto wait_v = [&]() {  // V(i - 1) fragments (read in the previous phase 2): the only LDS reads in flight
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vt[0][0][0]), "+v"(vt[0][0][1]), "+v"(vt[0][1][0]),
                         "+v"(vt[0][1][1]), "+v"(vt[1][0][0]), "+v"(vt[1][0][1]), "+v"(vt[1][1][0]), "+v"(vt[1][1][1]));
        };
        auto wait_k = [&]() { asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(kf[0]), "+v"(kf[1]), "+v"(kf[2]), "+v"(kf[3])); };

        // iteration i (not the last block): phase 1 = PV(i - 1) | softmax(i, query block 0) | K(i + 1)
        // reads; phase 2 = QK^T(i + 1) | softmax(i, query block 1) | V(i) reads.  S(i) in sc, S(i + 1)
        // into sn, P(i - 1) in pp, P(i) into pc.
        auto iter = [&](int i, f32x16 (&sc)[NQ], f32x16 (&sn)[NQ], u32x4 (&pp)[NQ][2], u32x4 (&pc)[NQ][2],
                        auto FIRSTc) {
            constexpr bool FIRST = decltype(FIRSTc)::value;
            if (i & 1) sync_tile((i + 1) >> 1);  // K(i + 1) opens tile (i + 1) / 2
            if constexpr (!FIRST) wait_v();
            kread(i + 1, kf);
            if constexpr (!FIRST) {
#pragma unroll
                for (int qb = 0; qb < NQ; ++qb) pv(qb, pp[qb]);
            }
            softmax(sc[0], i, attn_ic<0>{}, pc[0]);
            __builtin_amdgcn_sched_barrier(0);
            wait_k();
            vread(i, vt);
            qk(sn);
            if constexpr (NQ == 2) softmax(sc[1], i, attn_ic<0>{}, pc[1]);
            __builtin_amdgcn_sched_barrier(0);
        };
        // The steady-state iteration of a wave with two query blocks, hand-placed: each MFMA followed by
        // the vector work that fits its gap (MI355X_MICROARCH.md: a 32x32x16 gap hides ~24 issue cycles,
        // i.e. two v_exp_f32 and one v_cvt_pk; a 16x16x32 row-sum gap ~8, one v_cvt_pk), fenced by
        // sched_barrier so that hipcc keeps the grouping:
        //   phase 1: 12 PV(i - 1) MFMAs; 16 exp2 + 8 packs of S(i) query block 0; K(i + 1) in the first two gaps
        //   phase 2: 8 QK^T(i + 1) MFMAs; 16 exp2 + 8 packs of S(i) query block 1; V(i) in the first four gaps
        auto mf_o = [&](int qb, int j, int db, const u32x4& pb) {
            const uint2 ua = vt[j][db][0], ub = vt[j][db][1];
            const u32x4 vf = u32x4{ua.x, ua.y, ub.x, ub.y};
            if (MMT_ATTN_ABLATE == 10) return;
            if (MMT_ATTN_ABLATE == 8)
                asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(st.o[qb][db]) : "v"(vf), "v"(pb));
            else
                asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(st.o[qb][db]) : "v"(vf), "v"(pb));
        };
        auto mf_l = [&](int qb, const u32x4& pb) {
            const u32x4 su = sel_u;
            if (MMT_ATTN_ABLATE == 10) return;
            if (MMT_ATTN_ABLATE == 8)
                asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(st.lacc[qb]) : "v"(su), "v"(pb));
            else
                asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(st.lacc[qb]) : "v"(su), "v"(pb));
        };
        auto ex2 = [&](f32x16& sv, int r) {
            if (MMT_ATTN_ABLATE == 3) return;
            sv[r] = __builtin_amdgcn_exp2f(sv[r]);
            sv[r + 1] = __builtin_amdgcn_exp2f(sv[r + 1]);
        };
        auto cv = [&](const f32x16& sv, u32x4 (&dst)[2], int r) {
            dst[r >> 3][(r & 7) >> 1] = MMT_ATTN_ABLATE == 9 ? __float_as_uint(sv[r]) : pack_bf16x2(sv[r], sv[r + 1]);
        };
        auto kr = [&](int b, int ks) {
            if (MMT_ATTN_ABLATE == 7) return;
            kf[ks] = pp_b128(kimg_of(b) + l32 * 128 + ((((2 * ks + hf) * 16) ^ kpos)));
        };
        auto vr = [&](int b, int j, int db) {
            if (MMT_ATTN_ABLATE == 7) return;
            const char* vimg = lds + ((b >> 1) % PP_R) * FTILE + KB * 128;
            const int row = 32 * (b & 1) + 16 * j + 4 * hf + qr;
            const char* b1 = vimg + row * 128 + (((4 * db + 2 * dsub + (pc >> 1)) ^ attn_vswz(row)) * 16) + (pc & 1) * 8;
            vt[j][db][0] = attn_tr16<0>(b1);
            vt[j][db][1] = attn_tr16<8 * 128>(b1);
        };
        auto qk1 = [&](f32x16& dst, int qb, int ks) {
            if (MMT_ATTN_ABLATE == 11) return;
            dst = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kf[ks]), __builtin_bit_cast(bf16x8, qf[qb][ks]),
                                                          ks ? dst : f32x16{}, 0, 0, 0);
        };
        auto iter2 = [&](int i, f32x16 (&sc)[NQ], f32x16 (&sn)[NQ], u32x4 (&pp)[NQ][2], u32x4 (&pc)[NQ][2]) {
          if constexpr (NQ == 2) {
            if (i & 1) sync_tile((i + 1) >> 1);
            wait_v();
            __builtin_amdgcn_sched_barrier(0);
            // phase 1
            mf_o(0, 0, 0, pp[0][0]); kr(i + 1, 0); kr(i + 1, 1); ex2(sc[0], 0); __builtin_amdgcn_sched_barrier(0);
            mf_o(0, 0, 1, pp[0][0]); kr(i + 1, 2); kr(i + 1, 3); ex2(sc[0], 2); __builtin_amdgcn_sched_barrier(0);
            mf_l(0, pp[0][0]); cv(sc[0], pc[0], 0); __builtin_amdgcn_sched_barrier(0);
            mf_o(0, 1, 0, pp[0][1]); ex2(sc[0], 4); cv(sc[0], pc[0], 2); __builtin_amdgcn_sched_barrier(0);
            mf_o(0, 1, 1, pp[0][1]); ex2(sc[0], 6); __builtin_amdgcn_sched_barrier(0);
            mf_l(0, pp[0][1]); cv(sc[0], pc[0], 4); __builtin_amdgcn_sched_barrier(0);
            mf_o(1, 0, 0, pp[1][0]); ex2(sc[0], 8); cv(sc[0], pc[0], 6); __builtin_amdgcn_sched_barrier(0);
            mf_o(1, 0, 1, pp[1][0]); ex2(sc[0], 10); __builtin_amdgcn_sched_barrier(0);
            mf_l(1, pp[1][0]); cv(sc[0], pc[0], 8); __builtin_amdgcn_sched_barrier(0);
            mf_o(1, 1, 0, pp[1][1]); ex2(sc[0], 12); cv(sc[0], pc[0], 10); __builtin_amdgcn_sched_barrier(0);
            mf_o(1, 1, 1, pp[1][1]); ex2(sc[0], 14); __builtin_amdgcn_sched_barrier(0);
            mf_l(1, pp[1][1]); cv(sc[0], pc[0], 12); __builtin_amdgcn_sched_barrier(0);
            cv(sc[0], pc[0], 14);
            wait_k();
            __builtin_amdgcn_sched_barrier(0);
            // phase 2
            qk1(sn[0], 0, 0); vr(i, 0, 0); ex2(sc[1], 0); __builtin_amdgcn_sched_barrier(0);
            qk1(sn[1], 1, 0); vr(i, 0, 1); ex2(sc[1], 2); cv(sc[1], pc[1], 0); __builtin_amdgcn_sched_barrier(0);
            qk1(sn[0], 0, 1); vr(i, 1, 0); ex2(sc[1], 4); cv(sc[1], pc[1], 2); __builtin_amdgcn_sched_barrier(0);
            qk1(sn[1], 1, 1); vr(i, 1, 1); ex2(sc[1], 6); cv(sc[1], pc[1], 4); __builtin_amdgcn_sched_barrier(0);
            qk1(sn[0], 0, 2); ex2(sc[1], 8); cv(sc[1], pc[1], 6); __builtin_amdgcn_sched_barrier(0);
            qk1(sn[1], 1, 2); ex2(sc[1], 10); cv(sc[1], pc[1], 8); __builtin_amdgcn_sched_barrier(0);
            qk1(sn[0], 0, 3); ex2(sc[1], 12); cv(sc[1], pc[1], 10); __builtin_amdgcn_sched_barrier(0);
            qk1(sn[1], 1, 3); ex2(sc[1], 14); cv(sc[1], pc[1], 12); __builtin_amdgcn_sched_barrier(0);
            cv(sc[1], pc[1], 14);
            __builtin_amdgcn_sched_barrier(0);
          }
        };
        // the last block i = nb - 1: PV(i - 1) | softmax(i) (masked past Lk) | V(i) reads; then PV(i)
        auto last = [&](int i, f32x16 (&sc)[NQ], u32x4 (&pp)[NQ][2], u32x4 (&pc)[NQ][2], auto FIRSTc) {
            constexpr bool FIRST = decltype(FIRSTc)::value;
            if constexpr (!FIRST) {
                wait_v();
#pragma unroll
                for (int qb = 0; qb < NQ; ++qb) pv(qb, pp[qb]);
            }
            vread(i, vt);
            if (nvl < 32) {
#pragma unroll
                for (int qb = 0; qb < NQ; ++qb) softmax(sc[qb], i, attn_ic<1>{}, pc[qb]);
            } else {
#pragma unroll
                for (int qb = 0; qb < NQ; ++qb) softmax(sc[qb], i, attn_ic<0>{}, pc[qb]);
            }
            wait_v();
#pragma unroll
            for (int qb = 0; qb < NQ; ++qb) pv(qb, pc[qb]);
            pv_drain();
        };

        // prologue: K(0) -> S(0)
        MMT_PPSTAMP(2, "s_memtime");
        kread(0, kf);
        wait_k();
        qk(sA);
        if (nb == 1) {
            last(0, sA, pB, pA, attn_ic<1>{});
        } else {
            iter(0, sA, sB, pB, pA, attn_ic<1>{});  // even blocks: S in sA, P into pA
            int i = 1;
            for (; i + 1 < nb - 1; i += 2) {
                if constexpr (NQ == 2) {
                    iter2(i, sB, sA, pA, pB);
                    iter2(i + 1, sA, sB, pB, pA);
                } else {
                    iter(i, sB, sA, pA, pB, attn_ic<0>{});
                    iter(i + 1, sA, sB, pB, pA, attn_ic<0>{});
                }
            }
            if (i < nb - 1) {  // one odd block before the last
                if constexpr (NQ == 2) iter2(i, sB, sA, pA, pB);
                else iter(i, sB, sA, pA, pB, attn_ic<0>{});
                ++i;
            }
            MMT_PPSTAMP(3, "s_memtime");
            if (i & 1) last(i, sB, pA, pB, attn_ic<0>{});
            else last(i, sA, pB, pA, attn_ic<0>{});
        }

        if constexpr (KS == 2) {
            pad_barriers();
            if (half == 1) {
#pragma unroll
                for (int qb = 0; qb < NQ; ++qb) {
#pragma unroll
                    for (int db = 0; db < 2; ++db)
#pragma unroll
                        for (int r4 = 0; r4 < 4; ++r4)
                            *(f32x4*)(mrg + (((qb * 2 + db) * 4 + r4) * 64 + lane) * 4) =
                                f32x4{st.o[qb][db][4 * r4], st.o[qb][db][4 * r4 + 1], st.o[qb][db][4 * r4 + 2],
                                      st.o[qb][db][4 * r4 + 3]};
                    mrg[4 * 16 * 64 + qb * 64 + lane] = st.lacc[qb][0];
                }
                lds_barrier();
                return;
            }
            lds_barrier();
            if (nb_all - nb_h0 > 0) {  // half 1 had keys
#pragma unroll
                for (int qb = 0; qb < NQ; ++qb) {
#pragma unroll
                    for (int db = 0; db < 2; ++db)
#pragma unroll
                        for (int r4 = 0; r4 < 4; ++r4) {
                            const f32x4 v = *(const f32x4*)(mrg + (((qb * 2 + db) * 4 + r4) * 64 + lane) * 4);
#pragma unroll
                            for (int e = 0; e < 4; ++e) st.o[qb][db][4 * r4 + e] += v[e];
                        }
                    st.lacc[qb][0] += mrg[4 * 16 * 64 + qb * 64 + lane];
                }
            }
        }
        // per query block: range check, normalise and store, or the exact fallback (impl 22's)
#pragma unroll
        for (int qb = 0; qb < NQ; ++qb) {
            const float l = st.lacc[qb][0];
            float chk = 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) chk += st.o[qb][0][r] * 0.f + st.o[qb][1][r] * 0.f;
            const bool ok = (l >= LZ_LO && l <= LZ_HI && chk == 0.f) || MMT_ATTN_ABLATE != 0;
            const int q = qbase + 32 * qb + l32;
            bf16_t* op = (bf16_t*)p.out + attn_out_row(p, s, q, pitch) * C + h * D;
            if (__builtin_expect(__all(ok), 1)) {
                const float inv = 1.f / l;
                if (q < qend) {
#pragma unroll
                    for (int db = 0; db < 2; ++db)
#pragma unroll
                        for (int g = 0; g < 4; ++g)
                            *(uint2*)(op + 32 * db + 8 * g + 4 * hf) =
                                make_uint2(pack_bf16x2(st.o[qb][db][4 * g] * inv, st.o[qb][db][4 * g + 1] * inv),
                                           pack_bf16x2(st.o[qb][db][4 * g + 2] * inv, st.o[qb][db][4 * g + 3] * inv));
                }
                continue;
            }
            float qv[32], acc[32];
            const int qc = min(q, qend - 1);
            {
                const bf16_t* qp = qkv + ((int64_t)s * pitch + qc) * rs + h * D + 32 * hf;
#pragma unroll
                for (int i = 0; i < 32; ++i) qv[i] = bf2f(qp[i]) * cexp;
            }
            auto score = [&](int kk) {
                const bf16_t* kp = key_row(kk) + C + h * D + 32 * hf;
                float d0 = 0.f;
#pragma unroll
                for (int i = 0; i < 32; ++i) d0 += qv[i] * bf2f(kp[i]);
                return d0 + __shfl_xor(d0, 32, 64);
            };
            float m = -INFINITY;
            for (int kk = 0; kk < Lk; ++kk) m = fmaxf(m, score(kk));
            float lf = 0.f;
#pragma unroll
            for (int i = 0; i < 32; ++i) acc[i] = 0.f;
            for (int kk = 0; kk < Lk; ++kk) {
                const float e = __builtin_amdgcn_exp2f(score(kk) - m);
                lf += e;
                const bf16_t* vp = key_row(kk) + 2 * C + h * D + 32 * hf;
#pragma unroll
                for (int i = 0; i < 32; ++i) acc[i] += e * bf2f(vp[i]);
            }
            if (q < qend) {
                const float inv = 1.f / lf;
#pragma unroll
                for (int i = 0; i < 32; i += 8)
                    *(u32x4*)(op + 32 * hf + i) = u32x4{pack_bf16x2(acc[i] * inv, acc[i + 1] * inv), pack_bf16x2(acc[i + 2] * inv, acc[i + 3] * inv),
                                                        pack_bf16x2(acc[i + 4] * inv, acc[i + 5] * inv), pack_bf16x2(acc[i + 6] * inv, acc[i + 7] * inv)};
            }
        }
    };
    if (nqa == 2) run(attn_ic<2>{});
    else run(attn_ic<1>{});
    MMT_PPSTAMP(4, "s_memtime");
    MMT_PPSTAMP(5, "s_memrealtime");
#if MMT_STAMP_BUILD
    if (threadIdx.x == 0) {
        const int wg = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
        g_mmt_attn_pp_stamps[wg * 8 + 6] = nb;
        g_mmt_attn_pp_stamps[wg * 8 + 7] = nqa;
    }
#endif
}

}  // namespace

// launched by attention.hip's dispatcher (impl 24: ks 1, impl 25: ks 2): grid (128-query blocks, heads,
// sequences), 128 x ks threads
int mmt_attn_launch_pp(const mmt_attn_params& p, int ks, hipStream_t st) {
    const int t = (p.n_t + FQ - 1) / FQ, sr = (p.ntok - p.n_t + FQ - 1) / FQ;
    const int nqb = p.q_part == 1 ? t : p.q_part == 2 ? sr : t + sr;
    if (ks == 2) hipLaunchKernelGGL(mam_attention_pp_kernel<2>, dim3(nqb, p.H, p.S), dim3(256), 0, st, p);
    else hipLaunchKernelGGL(mam_attention_pp_kernel<1>, dim3(nqb, p.H, p.S), dim3(128), 0, st, p);
    return 0;
}
#endif  // MMT_ATTN_AB
