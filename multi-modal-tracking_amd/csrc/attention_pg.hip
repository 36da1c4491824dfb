// MAM attention, impl 28 (A/B build only): impl 22's math (P = exp2(S) with no reference point, row sums on the matrix
// pipe, epilogue range check with the exact two-pass fallback) in the "ping-pong" schedule of two waves
// per SIMD (MI355X_MICROARCH.md, "Two waves per SIMD", items 1-6).
//
// Reference: Attention.forward, lib/models/mixformer_vit_rgbt/mixformer.py:52-78 and the cross-modal
// form asymmetric_shared.py:55-104 (template queries -> own template keys; search queries -> all keys,
// or [template_V | template_I | own search]).  Layouts as attention.hip: qkv [seq][token][3][head][64]
// read in place, out [seq][token][head * 64].
//
// Why.  At d = 64 a 32-query x 32-key block costs 8 MFMA pipe slots of 32 cycles (4 QK^T + 4 PV 32x32x16,
// plus 2 row-sum 16x16x32) against 16 v_exp_f32 (8 issue cycles each) and 8 v_cvt_pk per wave, i.e.
// the vector issue of the softmax is ~90 % of the matrix-pipe time.  impl 22 leaves the overlap of the
// two to whatever phase two unrelated co-resident waves happen to be in (PMC at B = 32: MFMA pipe busy
// 28 %).  Here the two waves of a SIMD belong to one 512-thread workgroup and are held half a block
// apart by the workgroup barrier, so one wave's MFMA segment always runs beside its partner's softmax:
//   per wave and 32-key block k:  X_k = exp2 + pack of S(k) -> P(k); LDS reads of V(k), K(k + 1)
//                                 Y_k = QK^T(k + 1) -> S(k + 1); O += V(k)^T P(k), row sums
//   waves 0-3 (group 0):  Y_-1 | X_0 | Y_0 | X_1 | Y_1 | ...        (one s_barrier between segments)
//   waves 4-7 (group 1):   --  | Y_-1 | X_0 | Y_0 | X_1 | ...       (one extra barrier at the start)
// so in every interval one wave of each SIMD issues only MFMAs (20 per interval) and its partner only
// vector / LDS / DMA work.  Group 1 runs at s_setprio 1 (the arbitration loser otherwise, item 4).
//
// Work items.  A search item = the (up to 512) search queries of one (sequence, head): waves w = 0..7
// take queries 64 w .. 64 w + 63 (two 32-query blocks), one K / V stream.  Template items (n_t <= 128:
// 4 per workgroup, n_t <= 256: 2) share a workgroup, each with its own stream and the same block count;
// the item's waves are (j, j + 4), (2j, 2j+1, 2j+4, 2j+5) or all eight.  Search workgroups come first
// in the grid and the short template workgroups fill the tail.  One workgroup per CU (8 waves x 256
// registers fill the register file).
//
// K / V stream.  64-key tiles (K image + V image, attention.hip's swizzles) in a 3-slot LDS ring per
// item (2 for 4-item template workgroups, whose two tiles are all DMA'd up front), filled by
// buffer_load ... lds from the group-0 waves of the item.  Tile t is read by X_{2t-1} .. X_{2t+1}, i.e.
// by group 1 last in interval 4t + 4, so tile t + 3 is issued into its slot in group 0's X_{2t+2}
// (interval 4t + 5) and waited for (counted vmcnt, then the barrier) at the end of group 0's Y_{4t+8}:
// five intervals of flight.  No global store inside the loop (attention.hip's counted-wait rule).
//
// Results are bit-identical to impl 22 (same MFMAs per accumulator in the same order, same
// exponentials, same normalisation); the output rows leave as 16-B stores after a permlane32 swap.
#include "attn_common.hpp"

#ifndef MMT_ATTN_AB
#define MMT_ATTN_AB 0
#endif
#if MMT_ATTN_AB  // A/B build only (tools/build_ablate.sh ab): not faster than impl 22 / 4 anywhere

// MMT_ATTN_ABLATE (measurement builds only, tools/build_ablate.sh; results are wrong): 31 = no exponentials /
// packs in X, 32 = no MFMAs in Y, 33 = no barriers inside the block loop (free-running waves), 34 = no K / V
// fragment reads in X
#ifndef MMT_ATTN_ABLATE
#define MMT_ATTN_ABLATE 0
#endif

namespace {

constexpr int PG_LDS = 8 * FTILE;  // 128 KiB: 4 template items x 2 slots, 2 x 3, or one search item x 3
constexpr int PG_QCH = 512;        // queries per item (8 waves x 64)

struct PgCfg {
    int32_t nsw;           // search workgroups (one item each): blocks [0, nsw); template workgroups after
    int32_t G;             // template items per template workgroup (4 / 2 / 1)
    int32_t nch_s, nch_t;  // 512-query chunks of the search / template queries
};

MMT_DEV u32x4 pg_b128(const char* p) {
    u32x4 r;
    const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
    asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(a));
    return r;
}

// one segment boundary: nothing moves across it
MMT_DEV void pg_barrier() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}
// a barrier inside the block loop (measurement build 33: none)
MMT_DEV void pg_loop_barrier() {
    if (MMT_ATTN_ABLATE != 33) pg_barrier();
    else __builtin_amdgcn_sched_barrier(0);
}

#if MMT_STAMP_BUILD
// measurement build: per workgroup [0] realtime at entry, [1] memtime at entry, [2] after the prologue
// barrier, [3] loop end, [4] end (wave 0), [5] realtime at the end, [6] blocks + 1000 x template, [7] loop
// end of wave 4
__device__ unsigned long long g_mmt_attn_pg_stamps[16384 * 8];
extern "C" int mmt_attn_pg_stamps(unsigned long long* host, int n) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_mmt_attn_pg_stamps), sizeof(unsigned long long) * n);
}
// segment stamps of blocks 6 and 7 (waves 0 and 4): X start, X end, Y start, Y end; kept in registers and
// written after the loop (no store inside it)
__device__ unsigned long long g_mmt_attn_pg_seg[16384 * 16];
extern "C" int mmt_attn_pg_seg(unsigned long long* host, int n) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_mmt_attn_pg_seg), sizeof(unsigned long long) * n);
}
#define PG_SEG(K, I)                                                                               \
    if ((K) == 6 || (K) == 7) {                                                                    \
        unsigned long long t_;                                                                     \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                 \
        seg[((K) - 6) * 4 + (I)] = t_;                                                             \
    }
#define PG_STAMP(W, I, INSN)                                                            \
    if (threadIdx.x == 64 * (W)) {                                                      \
        unsigned long long t_;                                                          \
        asm volatile(INSN " %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");          \
        g_mmt_attn_pg_stamps[blockIdx.x * 8 + (I)] = t_;                                \
    }
#else
#define PG_STAMP(W, I, INSN)
#define PG_SEG(K, I)
#endif

__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void mam_attention_pg_kernel(
    const mmt_attn_params p, const PgCfg cfg) {
    __shared__ __attribute__((aligned(1024))) char lds_all[PG_LDS];
    PG_STAMP(0, 0, "s_memrealtime");
    PG_STAMP(0, 1, "s_memtime");
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = w >> 2, wA = w & 3;  // grp 1: the younger half, one interval behind
    const int wg = blockIdx.x;
    const bool tmpl = wg >= cfg.nsw;
    const int G = tmpl ? cfg.G : 1;
    const int per = 4 / G;                 // waves of one group per item
    const int j = wA / per;                // item slot of this wave in the workgroup
    const int iw = wA % per + per * grp;   // wave within its item: queries 64 iw .. 64 iw + 63
    const int spi = G == 4 ? 2 : 3;        // LDS tile slots per item
    char* lds = lds_all + j * spi * FTILE;
    const int nch = tmpl ? cfg.nch_t : cfg.nch_s;
    const int nitems = p.S * p.H * nch;
    int item = tmpl ? (wg - cfg.nsw) * G + j : wg;
    const bool valid = item < nitems;      // false: an empty template slot (barriers only)
    item = valid ? item : nitems - 1;
    const int c = item % nch, h = (item / nch) % p.H, s = item / (nch * p.H);

    const int n_t = p.n_t, ntok = p.ntok, C = p.C;
    const int64_t pitch = p.tok_pitch > 0 ? p.tok_pitch : ntok;
    const int q0 = (tmpl ? 0 : n_t) + c * PG_QCH;
    const int qend = min(tmpl ? n_t : ntok, q0 + PG_QCH);
    const bool cross = p.asym && !tmpl;
    const int Lk = tmpl ? n_t : (p.asym ? ntok + n_t : ntok);
    const int nb = (Lk + 31) >> 5, nt = (Lk + KB - 1) / KB;
    const int64_t rs = 3 * (int64_t)C;
    const bf16_t* qkv = (const bf16_t*)p.qkv;
    const int sV = p.asym ? s % p.Bm : s, sI = sV + p.Bm;

    const int l32 = lane & 31, hf = lane >> 5, prow = lane >> 3, pcol = lane & 7;
    const int qbase = q0 + 64 * iw;  // query blocks qbase + 32 qb + [0, 32)
    const int nqa = valid ? (qbase < qend ? 1 : 0) + (qbase + 32 < qend ? 1 : 0) : 0;

    // ---- K / V tiles: the group-0 waves of the item issue ppw of the 16 pieces (8 rows x 128 B) of a tile
    const bool issuer = grp == 0 && valid;
    const int ppw = 16 / per, pk0 = (wA % per) * ppw;
    auto key_seq_row = [&](int kk, int& seq, int& row) {
        seq = s;
        row = kk;
        if (cross) {
            if (kk < n_t) seq = sV;
            else if (kk < 2 * n_t) { seq = sI; row = kk - n_t; }
            else row = kk - n_t;
        }
    };
    auto key_row = [&](int kk) -> const bf16_t* {
        int seq, row;
        key_seq_row(kk, seq, row);
        return qkv + ((int64_t)seq * pitch + row) * rs;
    };
    const __amdgpu_buffer_rsrc_t qrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)qkv, 0, (int)min((int64_t)0x7fffffff, (int64_t)p.S * pitch * rs * 2), 0x00020000);
    const int voffK = (int)((prow * rs + C + h * D + (pcol ^ prow) * 8) * 2);
    const int voffV = (int)((prow * rs + 2 * C + h * D + (pcol ^ attn_vswz(prow)) * 8) * 2);
    typedef __attribute__((address_space(3))) void lds_void_t;
    const bool aligned = n_t % KB == 0;
    auto issue_tile = [&](int t) {
        MMT_ATTN_ASSERT(t >= 0 && t < nt);
        char* slot = lds + (t % spi) * FTILE;
        if (aligned && t * KB + KB <= Lk) {  // one key segment: a scalar row base, no vector work per piece
            int seq, row;
            key_seq_row(t * KB, seq, row);
            const int soff = __builtin_amdgcn_readfirstlane((int)(((int64_t)seq * pitch + row) * rs * 2));
            for (int i = 0; i < ppw; ++i) {
                const int pk = pk0 + i, isv = pk >> 3;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(qrs, (lds_void_t*)(slot + isv * KB * 128 + (pk & 7) * 1024), 16,
                                                         isv ? voffV : voffK, soff + (pk & 7) * 8 * (int)rs * 2, 0, 0);
            }
        } else {  // the tail tile (rows past Lk re-read the last key) or a tile across key segments
            for (int i = 0; i < ppw; ++i) {
                const int pk = pk0 + i, isv = pk >> 3;
                const int kk = min(t * KB + (pk & 7) * 8 + prow, Lk - 1);
                const int64_t col = (isv ? 2 * C : C) + h * D + (isv ? (pcol ^ attn_vswz(prow)) : (pcol ^ prow)) * 8;
                attn_glds16(key_row(kk) + col, slot + isv * KB * 128 + (pk & 7) * 1024);
            }
        }
    };

    // ---- prologue: Q straight into registers (B operand of S^T = K Q^T: query l32 of the block, d =
    // 16 ks + 8 hf .. + 7; rows past the block's end re-read the last query), then the first tiles
    u32x4 qf[2][4];
    if (nqa > 0) {
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
            const bf16_t* qp = qkv + ((int64_t)s * pitch + min(qbase + 32 * qb + l32, qend - 1)) * rs + h * D;
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) qf[qb][ks] = *(const u32x4*)(qp + (2 * ks + hf) * 8);
        }
    }
    const int npro = min(spi, nt);
    if (issuer)
        for (int t = 0; t < npro; ++t) issue_tile(t);
    if (issuer) attn_wait_dyn(ppw * (npro - 1));  // Q and tile 0 (Q loads are older than every piece)
    else attn_wait_vm<0>();
    const float cexp = p.scale * 1.4426950408889634f;
    if (nqa > 0 && fabsf(cexp - 1.f) > 1e-6f) {  // natural-scale q (tests / A/B callers): to log2 units
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
#ifndef MMT_PG_PRIO
#define MMT_PG_PRIO 2  // 0: none, 1: static s_setprio 1 for group 1, 2: s_setprio 1 around each MFMA segment
#endif
    if (MMT_PG_PRIO == 1 && grp == 1) __builtin_amdgcn_s_setprio(1);  // wave-uniform branch (w is readfirstlane'd)
    pg_barrier();
    PG_STAMP(0, 2, "s_memtime");

    const float one_or_zero = (((lane & 15) >> 2) & 1) == ((lane >> 4) & 1) ? 1.f : 0.f;
    const uint32_t sel_w = pack_bf16x2(one_or_zero, one_or_zero);
    const u32x4 sel_u = u32x4{sel_w, sel_w, sel_w, sel_w};
    const int kpos = (l32 & 7) * 16;
    const int li = lane & 15, qr = li >> 2, pc = li & 3, dsub = (lane >> 4) & 1;
    const int nvl = Lk - 32 * (nb - 1);  // keys of the last block

    auto run = [&](auto NQc) {
        constexpr int NQ = decltype(NQc)::value;  // active 32-query blocks (0: the skeleton only)
        constexpr int NA = NQ > 0 ? NQ : 1;
        f32x16 o[NA][2];
        f32x4 lacc[NA];
        f32x16 sv[NA];
        u32x4 pf[NA][2];
        u32x4 kf[4];
        uint2 vt[2][2][2];
#pragma unroll
        for (int qb = 0; qb < NA; ++qb) {
            o[qb][0] = f32x16{};
            o[qb][1] = f32x16{};
            lacc[qb] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        auto kread = [&](int b) {
            const char* krow = lds + ((b >> 1) % spi) * FTILE + (32 * (b & 1) + l32) * 128;
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) kf[ks] = pg_b128(krow + ((((2 * ks + hf) * 16) ^ kpos)));
        };
        auto vread = [&](int b) {
            const char* vimg = lds + ((b >> 1) % spi) * FTILE + KB * 128;
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) {
                const int row = 32 * (b & 1) + 16 * jj + 4 * hf + qr;
#pragma unroll
                for (int db = 0; db < 2; ++db) {
                    const char* b1 = vimg + row * 128 + (((4 * db + 2 * dsub + (pc >> 1)) ^ attn_vswz(row)) * 16) + (pc & 1) * 8;
                    vt[jj][db][0] = attn_tr16<0>(b1);
                    vt[jj][db][1] = attn_tr16<8 * 128>(b1);
                }
            }
        };
        // the asm reads landed; the wait redefines their registers, so nothing reads them earlier
        auto wait_k = [&]() { asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(kf[0]), "+v"(kf[1]), "+v"(kf[2]), "+v"(kf[3])); };
        auto wait_kv = [&]() {
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(kf[0]), "+v"(kf[1]), "+v"(kf[2]), "+v"(kf[3]), "+v"(vt[0][0][0]), "+v"(vt[0][0][1]),
                           "+v"(vt[0][1][0]), "+v"(vt[0][1][1]), "+v"(vt[1][0][0]), "+v"(vt[1][0][1]), "+v"(vt[1][1][0]),
                           "+v"(vt[1][1][1]));
        };
        // Every MFMA of a segment is in ONE asm statement that opens with 2 wait states (a VALU write of an
        // operand, e.g. a register copy the compiler placed before it) and closes with 21 (the 16-pass results
        // before any vector instruction -- the next segment's exponentials, or a copy of an accumulator the
        // compiler places after it -- reads them): hipcc cannot see the hazards inside asm, and it does move
        // accumulators between asm statements.  The trailing wait states run while the pipe is still busy
        // with the segment's last MFMA.
        // S^T(b) = K Q^T (the scores are in log2 units), each accumulator from zero, ks in order; Q lives in
        // accumulator registers (MFMA A / B operands may be AGPRs), so that the architectural VGPRs hold only
        // the scores, P and the fragments and nothing is spilled (a reload's vmcnt(0) would drain the ring).
        auto qk = [&]() {
            if constexpr (NQ == 2) {
                asm volatile(
                    "s_nop 1\n\t"
                    "v_mfma_f32_32x32x16_bf16 %0, %2, %6, 0\n\t"
                    "v_mfma_f32_32x32x16_bf16 %1, %2, %10, 0\n\t"
                    "v_mfma_f32_32x32x16_bf16 %0, %3, %7, %0\n\t"
                    "v_mfma_f32_32x32x16_bf16 %1, %3, %11, %1\n\t"
                    "v_mfma_f32_32x32x16_bf16 %0, %4, %8, %0\n\t"
                    "v_mfma_f32_32x32x16_bf16 %1, %4, %12, %1\n\t"
                    "v_mfma_f32_32x32x16_bf16 %0, %5, %9, %0\n\t"
                    "v_mfma_f32_32x32x16_bf16 %1, %5, %13, %1\n\t"
                    "s_nop 7\n\ts_nop 7\n\ts_nop 4"
                    : "=&v"(sv[0]), "=&v"(sv[1])
                    : "v"(kf[0]), "v"(kf[1]), "v"(kf[2]), "v"(kf[3]), "a"(qf[0][0]), "a"(qf[0][1]), "a"(qf[0][2]),
                      "a"(qf[0][3]), "a"(qf[1][0]), "a"(qf[1][1]), "a"(qf[1][2]), "a"(qf[1][3]));
            } else if constexpr (NQ == 1) {
                asm volatile(
                    "s_nop 1\n\t"
                    "v_mfma_f32_32x32x16_bf16 %0, %1, %5, 0\n\t"
                    "v_mfma_f32_32x32x16_bf16 %0, %2, %6, %0\n\t"
                    "v_mfma_f32_32x32x16_bf16 %0, %3, %7, %0\n\t"
                    "v_mfma_f32_32x32x16_bf16 %0, %4, %8, %0\n\t"
                    "s_nop 7\n\ts_nop 7\n\ts_nop 4"
                    : "=&v"(sv[0])
                    : "v"(kf[0]), "v"(kf[1]), "v"(kf[2]), "v"(kf[3]), "a"(qf[0][0]), "a"(qf[0][1]), "a"(qf[0][2]),
                      "a"(qf[0][3]));
            }
        };
        // P(b) = exp2(S(b)) (MASK: keys >= Lk give 0), packed as the B operand of the PV MFMA
        auto softmax = [&](int b, auto MASKc) {
            constexpr bool MASK = decltype(MASKc)::value;
#pragma unroll
            for (int qb = 0; qb < NQ; ++qb) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float e = __builtin_amdgcn_exp2f(sv[qb][r]);
                    sv[qb][r] = (!MASK || 32 * b + 8 * (r >> 2) + 4 * hf + (r & 3) < Lk) ? e : 0.f;
                }
#pragma unroll
                for (int jj = 0; jj < 2; ++jj)
                    pf[qb][jj] = u32x4{pack_bf16x2(sv[qb][8 * jj], sv[qb][8 * jj + 1]), pack_bf16x2(sv[qb][8 * jj + 2], sv[qb][8 * jj + 3]),
                                       pack_bf16x2(sv[qb][8 * jj + 4], sv[qb][8 * jj + 5]), pack_bf16x2(sv[qb][8 * jj + 6], sv[qb][8 * jj + 7])};
            }
        };
        // O^T += V^T P^T (per 16-key step jj, query block qb, 32-dim half db) and the row sums, on accumulator
        // registers; same order per accumulator as impl 22
        auto pv = [&]() {
            u32x4 vf[2][2];
#pragma unroll
            for (int jj = 0; jj < 2; ++jj)
#pragma unroll
                for (int db = 0; db < 2; ++db) {
                    const uint2 ua = vt[jj][db][0], ub = vt[jj][db][1];
                    vf[jj][db] = u32x4{ua.x, ua.y, ub.x, ub.y};
                }
            if constexpr (NQ == 2) {
                asm volatile(
                    "s_nop 1\n\t"
                    "v_mfma_f32_32x32x16_bf16 %0, %6, %10, %0\n\t"
                    "v_mfma_f32_32x32x16_bf16 %1, %7, %10, %1\n\t"
                    "v_mfma_f32_16x16x32_bf16 %4, %14, %10, %4\n\t"
                    "v_mfma_f32_32x32x16_bf16 %2, %6, %12, %2\n\t"
                    "v_mfma_f32_32x32x16_bf16 %3, %7, %12, %3\n\t"
                    "v_mfma_f32_16x16x32_bf16 %5, %14, %12, %5\n\t"
                    "v_mfma_f32_32x32x16_bf16 %0, %8, %11, %0\n\t"
                    "v_mfma_f32_32x32x16_bf16 %1, %9, %11, %1\n\t"
                    "v_mfma_f32_16x16x32_bf16 %4, %14, %11, %4\n\t"
                    "v_mfma_f32_32x32x16_bf16 %2, %8, %13, %2\n\t"
                    "v_mfma_f32_32x32x16_bf16 %3, %9, %13, %3\n\t"
                    "v_mfma_f32_16x16x32_bf16 %5, %14, %13, %5\n\t"
                    "s_nop 7\n\ts_nop 7\n\ts_nop 4"
                    : "+a"(o[0][0]), "+a"(o[0][1]), "+a"(o[1][0]), "+a"(o[1][1]), "+a"(lacc[0]), "+a"(lacc[1])
                    : "v"(vf[0][0]), "v"(vf[0][1]), "v"(vf[1][0]), "v"(vf[1][1]), "v"(pf[0][0]), "v"(pf[0][1]),
                      "v"(pf[1][0]), "v"(pf[1][1]), "v"(sel_u));
            } else if constexpr (NQ == 1) {
                asm volatile(
                    "s_nop 1\n\t"
                    "v_mfma_f32_32x32x16_bf16 %0, %3, %7, %0\n\t"
                    "v_mfma_f32_32x32x16_bf16 %1, %4, %7, %1\n\t"
                    "v_mfma_f32_16x16x32_bf16 %2, %9, %7, %2\n\t"
                    "v_mfma_f32_32x32x16_bf16 %0, %5, %8, %0\n\t"
                    "v_mfma_f32_32x32x16_bf16 %1, %6, %8, %1\n\t"
                    "v_mfma_f32_16x16x32_bf16 %2, %9, %8, %2\n\t"
                    "s_nop 7\n\ts_nop 7\n\ts_nop 4"
                    : "+a"(o[0][0]), "+a"(o[0][1]), "+a"(lacc[0])
                    : "v"(vf[0][0]), "v"(vf[0][1]), "v"(vf[1][0]), "v"(vf[1][1]), "v"(pf[0][0]), "v"(pf[0][1]),
                      "v"(sel_u));
            }
        };

        if constexpr (NQ > 0) {
            kread(0);
            wait_k();
        }
        if (grp == 1) pg_barrier();  // the stagger: group 1 one interval behind
        if (MMT_PG_PRIO == 2) __builtin_amdgcn_s_setprio(1);
        if constexpr (NQ > 0) qk();  // Y_-1
        if (MMT_PG_PRIO == 2) __builtin_amdgcn_s_setprio(0);
        pg_barrier();
#if MMT_STAMP_BUILD
        unsigned long long seg[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
        // one 32-key block: X_k then Y_k (LAST: no K(k + 1) / QK^T(k + 1); MASK: keys >= Lk give P = 0)
        auto step = [&](int k, auto MASKc, auto LASTc) {
            PG_SEG(k, 0);
            constexpr bool LAST = decltype(LASTc)::value;
            // X_k: tile (k / 2 - 1) + spi into the slot group 1 finished reading in the last interval
            if (issuer && k >= 2 && !(k & 1)) {
                const int t = (k >> 1) - 1 + spi;
                if (t < nt) issue_tile(t);
            }
            if constexpr (NQ > 0) {
                if (MMT_ATTN_ABLATE != 31) softmax(k, MASKc);
                if (MMT_ATTN_ABLATE != 34) {
                    vread(k);
                    if constexpr (!LAST) kread(k + 1);
                }
                wait_kv();
            }
            PG_SEG(k, 1);
            pg_loop_barrier();
            PG_SEG(k, 2);
            // Y_k
            if (MMT_PG_PRIO == 2) __builtin_amdgcn_s_setprio(1);
            if constexpr (NQ > 0) {
                if constexpr (!LAST) {
                    if (MMT_ATTN_ABLATE != 32) qk();
                }
                if (MMT_ATTN_ABLATE != 32) pv();
            }
            if (MMT_PG_PRIO == 2) __builtin_amdgcn_s_setprio(0);
            PG_SEG(k, 3);
            if (issuer && !(k & 1)) {  // tile k / 2 + 1 landed (its first reader is the next X segment)
                const int u = (k >> 1) + 1;
                if (u < nt) attn_wait_dyn(ppw * min(nt - 1 - u, spi - 2));
            }
            if (!(LAST && grp == 1)) pg_loop_barrier();
        };
        for (int k = 0; k < nb - 1; ++k) step(k, attn_ic<0>{}, attn_ic<0>{});
        if (nvl < 32) step(nb - 1, attn_ic<1>{}, attn_ic<1>{});
        else step(nb - 1, attn_ic<0>{}, attn_ic<1>{});
        PG_STAMP(0, 3, "s_memtime");
        PG_STAMP(4, 7, "s_memtime");
#if MMT_STAMP_BUILD
        if (lane == 0 && (w == 0 || w == 4))
            for (int i = 0; i < 8; ++i) g_mmt_attn_pg_seg[blockIdx.x * 16 + (w == 4 ? 8 : 0) + i] = seg[i];
#endif
        if constexpr (NQ > 0) {
            // the last MFMAs' results (16 passes) before any vector instruction reads O
#pragma unroll
            for (int qb = 0; qb < NQ; ++qb) asm volatile("s_nop 15\n\ts_nop 15" : "+a"(o[qb][0]), "+a"(o[qb][1]), "+a"(lacc[qb]));
            // per query block: range check, normalise and store, or the exact fallback (impl 22's)
#pragma unroll
            for (int qb = 0; qb < NQ; ++qb) {
                const float l = lacc[qb][0];
                float chk = 0.f;
#pragma unroll
                for (int r = 0; r < 16; ++r) chk += o[qb][0][r] * 0.f + o[qb][1][r] * 0.f;
                const bool ok = l >= LZ_LO && l <= LZ_HI && chk == 0.f;
                const int q = qbase + 32 * qb + l32;
                bf16_t* op = (bf16_t*)p.out + attn_out_row(p, s, q, pitch) * C + h * D;
                if (__builtin_expect(__all(ok), 1)) {
                    const float inv = 1.f / l;
                    // lane (q, hf) holds d = 32 db + 8 g + 4 hf + [0, 4); a permlane32 swap of the column
                    // groups g, g + 1 gives each lane 16 contiguous bytes of its row (guide T21)
#pragma unroll
                    for (int db = 0; db < 2; ++db)
#pragma unroll
                        for (int g = 0; g < 4; g += 2) {
                            const f32x16& ov = o[qb][db];
                            const uint32_t a0 = pack_bf16x2(ov[4 * g] * inv, ov[4 * g + 1] * inv);
                            const uint32_t a1 = pack_bf16x2(ov[4 * g + 2] * inv, ov[4 * g + 3] * inv);
                            const uint32_t b0 = pack_bf16x2(ov[4 * g + 4] * inv, ov[4 * g + 5] * inv);
                            const uint32_t b1 = pack_bf16x2(ov[4 * g + 6] * inv, ov[4 * g + 7] * inv);
                            const auto x0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
                            const auto x1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
                            if (q < qend) *(u32x4*)(op + 32 * db + 8 * g + 8 * hf) = u32x4{x0[0], x1[0], x0[1], x1[1]};
                        }
                    continue;
                }
                // exact fallback (scores outside the fp32-safe range): two-pass fp32 softmax per query,
                // lane (query l32, half hf) owns d = 32 hf .. 32 hf + 31; rows straight from global memory
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
        }
    };
    if (nqa == 2) run(attn_ic<2>{});
    else if (nqa == 1) run(attn_ic<1>{});
    else run(attn_ic<0>{});
    PG_STAMP(0, 4, "s_memtime");
    PG_STAMP(0, 5, "s_memrealtime");
#if MMT_STAMP_BUILD
    if (threadIdx.x == 0) g_mmt_attn_pg_stamps[blockIdx.x * 8 + 6] = nb + (tmpl ? 1000 : 0);
#endif
}

}  // namespace

// launched by attention.hip's dispatcher (impl 28): search workgroups, then template workgroups
int mmt_attn_launch_pg(const mmt_attn_params& p, hipStream_t st) {
    PgCfg cfg;
    const int ns = p.ntok - p.n_t;
    cfg.G = p.n_t <= 128 ? 4 : p.n_t <= 256 ? 2 : 1;
    cfg.nch_s = (ns + PG_QCH - 1) / PG_QCH;
    cfg.nch_t = cfg.G == 1 ? (p.n_t + PG_QCH - 1) / PG_QCH : 1;
    const int64_t sh = (int64_t)p.S * p.H;
    cfg.nsw = p.q_part == 1 ? 0 : (int)(sh * cfg.nch_s);
    const int ntw = p.q_part == 2 ? 0 : (int)((sh * cfg.nch_t + cfg.G - 1) / cfg.G);
    if ((int64_t)cfg.nsw + ntw <= 0) return 0;
    hipLaunchKernelGGL(mam_attention_pg_kernel, dim3(cfg.nsw + ntw), dim3(512), 0, st, p, cfg);
    return 0;
}
#endif  // MMT_ATTN_AB
