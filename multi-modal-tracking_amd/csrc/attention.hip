// Mixed Attention Module (MAM) — asymmetric template/search softmax attention for gfx950.
//
// Reference: Attention.forward, lib/models/mixformer_vit_rgbt/mixformer.py:52-78 (template
// queries -> template keys; search queries -> all keys) and the cross-modal variant
// asymmetric_shared.py:55-104 (search_m -> [template_V | template_I | search_m]).
// The qkv Linear output is consumed in place ([seq][token][3][head][64], no permute) and the
// result is written as [seq][token][head*64], i.e. exactly the proj GEMM's A operand.
//
// Kernels (mmt_attn_params.impl; 0 = the library's choice, launch_attn at the end of this file):
//   fp32 (parity path)  mam_attention_kernel: register-staged K/V ring, v_mfma_f32_16x16x4_f32
//   impl 4   bf16/fp16 latency kernel (batch-1 tracking): 64 queries x 4 key groups per workgroup,
//            online softmax with a running maximum, key groups merged through LDS
//   impl 8   bf16/fp16 throughput kernel with a running maximum (training forward with log-sum-exp,
//            fp16 batched)
//   impl 17 / 21 / 22  bf16 range-checked exponent kernels (no reference point, exact fallback):
//            32 (17 / 21) or 64 (22, the batched default) queries per wave; 21 = 17 with the two key
//            blocks of a tile software-pipelined
//   impl 23  (A/B build only, MMT_ATTN_AB) the 64-queries-per-wave kernel as a two-stage pipeline
//            over (key block, query block) units with a sched_group_barrier issue pattern and
//            256-query workgroups: bit-identical to 22, measured 6-10 % slower
// Scores are computed transposed (S^T = K Q^T) so that each lane owns one query column: the softmax
// statistics need no cross-lane reduction and the exponentiated scores are already laid out as the B
// operand of O^T = V^T P^T (no LDS round trip for P).  V^T fragments come from ds_read_b64_tr_b16 on
// a swizzled V image.  Softmax statistics are fp32 (exp2 with the scale folded in).
//
// Counted-wait rule (the round-2 impl 20-25 illegal-address fault): on gfx9-class
// hardware vmcnt counts vector-memory STORES as well as loads, so no kernel below issues a global
// store between an LDS-DMA issue and the counted s_waitcnt vmcnt(n) that covers it (outputs are
// written after the key loop's last counted wait).  Every DMA'd key tile index is in [0, nkt);
// building with -DMMT_ATTN_CHECK=1 turns that into a device assert (MMT_ATTN_ASSERT).
#include "attn_common.hpp"


namespace {


// XCD-aware bijective block remap (as gemm.hip): workgroups are dealt round-robin over the 8 XCDs,
// so consecutive (query block, head, sequence) ids would put the query blocks of one (sequence,
// head) on different XCDs, each fetching the same K / V rows into its own L2.  Giving each XCD a
// contiguous run of ids (query block fastest) keeps those re-reads in one L2.  Speed only; applied
// to grids larger than the chip (batched inference: B = 8 / 32 throughput kernel 33 -> 29 / 90 ->
// 84 us), not to the single-wave batch-1 grid.
MMT_DEV void attn_block_ids(int& bx, int& by, int& bz) {
    const int nbx = gridDim.x, nby = gridDim.y, nwg = nbx * nby * gridDim.z;
    if (nwg <= 256) {
        bx = blockIdx.x;
        by = blockIdx.y;
        bz = blockIdx.z;
        return;
    }
    const int orig = blockIdx.x + nbx * (blockIdx.y + nby * blockIdx.z);
    const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
    bx = lin % nbx;
    by = (lin / nbx) % nby;
    bz = lin / (nbx * nby);
}


template <typename T>
struct AttnCfg {
    static constexpr bool BF = sizeof(T) == 2;
    static constexpr int KCH = D * (int)sizeof(T) / 16;  // 16-B chunks per K/V row (8 / 16)
    static constexpr int QCH = KCH / 4;                  // chunk steps per lane over d (2 / 4)
    static constexpr int VROW = BF ? 160 : 272;          // padded V row (bytes)
};

// QT = 16-query MFMA tiles per wave (1: 4 waves x 16 queries, for small grids; 2: 2 waves x 32).
template <typename T, int QT>
__global__ __launch_bounds__(256 / QT) void mam_attention_kernel(const mmt_attn_params p) {
    constexpr int NTH = 256 / QT;
    using Cfg = AttnCfg<T>;
    constexpr int KCH = Cfg::KCH, QCH = Cfg::QCH, VROW = Cfg::VROW;
    __shared__ u32x4 kl[2][KB * KCH];
    __shared__ __attribute__((aligned(16))) char vl[2][KB * VROW];

    const int n_t = p.n_t, ntok = p.ntok, C = p.C;
    const int64_t pitch = p.tok_pitch > 0 ? p.tok_pitch : ntok;  // rows between sequences
    const int nqb_t = (n_t + 63) / 64;
    int bx, h, s;
    attn_block_ids(bx, h, s);
    const int qb = bx + (p.q_part == 2 ? nqb_t : 0);
    const bool tmpl = qb < nqb_t;
    const int q0 = tmpl ? qb * 64 : n_t + (qb - nqb_t) * 64;
    const int qend = tmpl ? n_t : ntok;
    const int Lk = tmpl ? n_t : (p.asym ? ntok + n_t : ntok);
    const bool cross = p.asym && !tmpl;
    const int64_t rs = 3 * (int64_t)C;
    const T* qkv = (const T*)p.qkv;
    const int sV = s % p.Bm, sI = sV + p.Bm;

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int l16 = lane & 15, lg = lane >> 4;

    // ---- Q fragments (B operand of S^T = K Q^T)
    u32x4 qf[QT][QCH];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
        const int q = q0 + 16 * QT * w + 16 * qt + l16;
        const T* qp = qkv + ((int64_t)s * pitch + min(q, qend - 1)) * rs + h * D;  // clamped, never stored
#pragma unroll
        for (int t = 0; t < QCH; ++t) qf[qt][t] = *(const u32x4*)(qp + (4 * t + lg) * (16 / (int)sizeof(T)));
    }

    // ---- K/V staging
    constexpr int PER = KB * KCH / NTH;  // chunks per thread per tile (4 / 8)
    const int ch = tid % KCH;
    auto key_ptr = [&](int kk) -> const T* {
        int seq = s, row = kk;
        if (cross) {
            if (kk < n_t) seq = sV;
            else if (kk < 2 * n_t) { seq = sI; row = kk - n_t; }
            else row = kk - n_t;
        }
        return qkv + ((int64_t)seq * pitch + row) * rs + h * D;
    };
    // K/V loads are unconditional (rows past Lk re-read key Lk-1 and are masked in the scores;
    // their V rows are multiplied by p = 0): a guarded load would make hipcc drain vmcnt(0).
    u32x4 rk[PER], rv[PER];
    auto load_kv = [&](int kt) {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int row = (tid + NTH * i) / KCH;
            const int kk = min(kt * KB + row, Lk - 1);
            const T* kp = key_ptr(kk) + ch * (16 / (int)sizeof(T));
            rk[i] = *(const u32x4*)(kp + C);
            rv[i] = *(const u32x4*)(kp + 2 * C);
        }
    };
    auto store_kv = [&](int buf) {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int row = (tid + NTH * i) / KCH;
            kl[buf][row * KCH + (ch ^ (row & 7))] = rk[i];
            *(u32x4*)(vl[buf] + row * VROW + ch * 16) = rv[i];
        }
    };

    const float cexp = p.scale * 1.4426950408889634f;
    float m_run[QT], l_run[QT];
    f32x4 o[4][QT];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
        m_run[qt] = -1e30f;
        l_run[qt] = 0.f;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[dt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

    const int nkt = (Lk + KB - 1) / KB;
    load_kv(0);
    store_kv(0);
    lds_barrier();
    for (int kt = 0; kt < nkt; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nkt) load_kv(kt + 1);

        // S^T tiles: sacc[kt16][qt], lane: query l16, keys 16*kt16 + 4*lg + r
        f32x4 sacc[4][QT];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) sacc[a][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kt16 = 0; kt16 < 4; ++kt16) {
#pragma unroll
            for (int t = 0; t < QCH; ++t) {
                const u32x4 kf = kl[cur][(kt16 * 16 + l16) * KCH + ((4 * t + lg) ^ (l16 & 7))];
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) {
                    if constexpr (Cfg::BF) {
                        sacc[kt16][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                            __builtin_bit_cast(bf16x8, kf), __builtin_bit_cast(bf16x8, qf[qt][t]), sacc[kt16][qt], 0, 0, 0);
                    } else {
                        const f32x4 ka = __builtin_bit_cast(f32x4, kf), qa = __builtin_bit_cast(f32x4, qf[qt][t]);
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            sacc[kt16][qt] = __builtin_amdgcn_mfma_f32_16x16x4f32(ka[j], qa[j], sacc[kt16][qt], 0, 0, 0);
                    }
                }
            }
        }
        // mask the tail of the key range
        if (kt * KB + KB > Lk) {
#pragma unroll
            for (int kt16 = 0; kt16 < 4; ++kt16)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (kt * KB + kt16 * 16 + 4 * lg + r >= Lk)
#pragma unroll
                        for (int qt = 0; qt < QT; ++qt) sacc[kt16][qt][r] = -1e30f;
        }
        // online softmax (per query column)
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            float mx = -1e30f;
#pragma unroll
            for (int kt16 = 0; kt16 < 4; ++kt16)
#pragma unroll
                for (int r = 0; r < 4; ++r) mx = fmaxf(mx, sacc[kt16][qt][r]);
            mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
            mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
            const float mnew = fmaxf(m_run[qt], mx);
            const float alpha = exp2f((m_run[qt] - mnew) * cexp);
            m_run[qt] = mnew;
            const float mc = mnew * cexp;
            float ls = 0.f;
#pragma unroll
            for (int kt16 = 0; kt16 < 4; ++kt16)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float e = exp2f(sacc[kt16][qt][r] * cexp - mc);
                    sacc[kt16][qt][r] = e;
                    ls += e;
                }
            l_run[qt] = l_run[qt] * alpha + ls;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) o[dt][qt] *= alpha;
        }
        // O^T += V^T P^T
        if constexpr (Cfg::BF) {
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                bf16x8 pf[QT];
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        pf[qt][j] = (__bf16)sacc[2 * kk][qt][j];
                        pf[qt][4 + j] = (__bf16)sacc[2 * kk + 1][qt][j];
                    }
                }
                const int qr = l16 >> 2, pc = l16 & 3;
#pragma unroll
                for (int dt = 0; dt < 4; ++dt) {
                    const char* b1 = vl[cur] + (32 * kk + 4 * lg + qr) * VROW + (dt * 16 + 4 * pc) * 2;
                    const s16x4 va = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)b1);
                    const s16x4 vb = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (__attribute__((address_space(3))) s16x4*)(b1 + 16 * VROW));
                    // whole-vector casts: per-element short->__bf16 casts miscompile (ROCm 7.2)
                    const uint2 ua = __builtin_bit_cast(uint2, va), ub = __builtin_bit_cast(uint2, vb);
                    const bf16x8 vf = __builtin_bit_cast(bf16x8, make_uint4(ua.x, ua.y, ub.x, ub.y));
#pragma unroll
                    for (int qt = 0; qt < QT; ++qt)
                        o[dt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[qt], o[dt][qt], 0, 0, 0);
                }
            }
        } else {
            const float* vf = (const float*)vl[cur];
#pragma unroll
            for (int kt16 = 0; kt16 < 4; ++kt16)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int key = kt16 * 16 + 4 * lg + r;
#pragma unroll
                    for (int dt = 0; dt < 4; ++dt) {
                        const float va = vf[key * (VROW / 4) + dt * 16 + l16];
#pragma unroll
                        for (int qt = 0; qt < QT; ++qt)
                            o[dt][qt] = __builtin_amdgcn_mfma_f32_16x16x4f32(va, sacc[kt16][qt][r], o[dt][qt], 0, 0, 0);
                    }
                }
        }
        if (kt + 1 < nkt) store_kv(cur ^ 1);
        lds_barrier();
    }

    // ---- normalise and store: lane holds O[q = l16][d = dt*16 + 4*lg + r]
    T* out = (T*)p.out;
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
        float l = l_run[qt];
        l += __shfl_xor(l, 16, 64);
        l += __shfl_xor(l, 32, 64);
        const float inv = 1.f / l;
        const int q = q0 + 16 * QT * w + 16 * qt + l16;
        if (q >= qend) continue;
        T* op = out + attn_out_row(p, s, q, pitch) * C + h * D;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
            if constexpr (Cfg::BF) {
                uint2 pk;
                pk.x = (uint32_t)f2bf(o[dt][qt][0] * inv) | ((uint32_t)f2bf(o[dt][qt][1] * inv) << 16);
                pk.y = (uint32_t)f2bf(o[dt][qt][2] * inv) | ((uint32_t)f2bf(o[dt][qt][3] * inv) << 16);
                *(uint2*)(op + dt * 16 + 4 * lg) = pk;
            } else {
                *(f32x4*)(op + dt * 16 + 4 * lg) = o[dt][qt] * inv;
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// bf16 kernel with LDS-DMA staging.  The register-staged kernel above prefetches one 64-key tile
// ahead, so each of the 9-11 key tiles of a search block exposes most of an L2/HBM round trip
// (batch-1: ~13 us per launch, ~4 % of MFMA peak).  Here every wave-instruction of
// global_load_lds_dwordx4 lands one 1-KiB piece (8 key rows x 128 B) of a K or V tile in LDS, and
// a ring of NS tile slots is filled up front: up to NS-1 tiles (448 keys) are in flight before the
// first score is computed, and the rest stream in behind the matrix work (counted vmcnt + raw
// barrier, as in gemm_glds.hip).  Q arrives the same way (its own 8-KiB image).
// LDS images are lane-linear, so conflict-free reads come from XOR swizzles applied on the
// per-lane source address and again on the read: K / Q rows (read by ds_read_b128) hold chunk c at
// c ^ (row & 7); V rows (read transposed by ds_read_b64_tr_b16: 8 rows x 2 adjacent chunks per
// 32-lane group) hold chunk c at c ^ (row & 6).
#if MMT_STAMP_BUILD
__device__ unsigned long long g_mmt_attn_stamps[16384 * 8];
extern "C" int mmt_attn_stamps(unsigned long long* host, int n) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_mmt_attn_stamps), sizeof(unsigned long long) * n);
}
#endif
#define MMT_ASTAMP(I, INSN) MMT_STAMP_AT(g_mmt_attn_stamps, I, INSN)

constexpr int ANS = 8;              // K/V tile slots in the ring
constexpr int ATILE = 2 * KB * 128; // bytes of one slot: K image then V image


// KG key groups of 4 waves: the WG's 64 queries (16 per wave) are shared, the key tiles are dealt
// round-robin over the groups (tile t -> group t % KG), each group keeps its own online-softmax
// state, and the states are merged through LDS at the end.  At batch 1 the grid is ~216 WGs, one
// per CU: splitting the keys puts 4*KG waves on the CU to hide the per-tile dependency chain
// (LDS read -> MFMA -> max -> exp -> MFMA) that one wave per SIMD exposed in full.
// NS = ring slots (tiles held).  (KG 3 with 9 slots, the whole 528-key stream issued in the prologue
// and three full rounds, measured no faster: 9.64 vs 9.49 us at B = 1 -- the per-CU fill of the
// 136 KiB of K / V, not the DMA rounds, bounds this kernel.)
template <typename T, int KG, int NS = ANS>
__global__ __launch_bounds__(256 * KG) __attribute__((amdgpu_waves_per_eu(KG, KG))) void mam_attention_glds_kernel(
    const mmt_attn_params p) {
    constexpr int NWV = 4 * KG;  // waves; a tile's 16 K/V pieces go to waves piece % NWV
    constexpr int R = NS / KG;   // rounds (KG tiles each) held by the ring
    static_assert(R >= 2 && NWV <= 16 && NWV >= 8 && R * KG == NS, "ring geometry");
    __shared__ __attribute__((aligned(1024))) char lds[NS * ATILE + 64 * 128];
    char* qimg = lds + NS * ATILE;
    MMT_ASTAMP(0, "s_memrealtime");
    MMT_ASTAMP(1, "s_memtime");

    const int n_t = p.n_t, ntok = p.ntok, C = p.C;
    const int64_t pitch = p.tok_pitch > 0 ? p.tok_pitch : ntok;  // rows between sequences
    const int nqb_t = (n_t + 63) / 64;
    int bx, h, s;
    attn_block_ids(bx, h, s);  // (grouping a (sequence, head)'s query blocks on one XCD measured
                               // slower at batch 1: 8.94 vs 8.47 us in the frame)
    const int qb = bx + (p.q_part == 2 ? nqb_t : 0);
    const bool tmpl = qb < nqb_t;
    const int q0 = tmpl ? qb * 64 : n_t + (qb - nqb_t) * 64;
    const int qend = tmpl ? n_t : ntok;
    const int Lk = tmpl ? n_t : (p.asym ? ntok + n_t : ntok);
    const bool cross = p.asym && !tmpl;
    const int64_t rs = 3 * (int64_t)C;
    const T* qkv = (const T*)p.qkv;
    const int sV = s % p.Bm, sI = sV + p.Bm;

    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int kg = w >> 2, qw = w & 3;  // key group, 16-query sub-block
    const int ppw = (15 - w) / NWV + 1;  // this wave's K/V pieces per tile (16 over NWV waves)
    const int l16 = lane & 15, lg = lane >> 4;
    const int prow = lane >> 3, pcol = lane & 7;  // this lane's row / position in a 1-KiB piece

    auto key_row = [&](int kk) -> const T* {
        int seq = s, row = kk;
        if (cross) {
            if (kk < n_t) seq = sV;
            else if (kk < 2 * n_t) { seq = sI; row = kk - n_t; }
            else row = kk - n_t;
        }
        return qkv + ((int64_t)seq * pitch + row) * rs + h * D;
    };
    const int nkt = (Lk + KB - 1) / KB, nr = (nkt + KG - 1) / KG;
    // Tile t into slot t % NS: its 16 pieces (8 K, 8 V) are dealt over the waves (piece w + i*NWV).
    auto issue_tile = [&](int t) {
        MMT_ATTN_ASSERT(t >= 0 && t < nkt);
        char* slot = lds + (t % NS) * ATILE;
#pragma unroll
        for (int i = 0; i < (16 + NWV - 1) / NWV; ++i) {
            const int piece = w + i * NWV, isv = piece >> 3, pk = piece & 7, r = pk * 8 + prow;
            if (piece >= 16) break;  // wave-uniform
            const T* src = key_row(min(t * KB + r, Lk - 1)) + (isv ? 2 * C : C);
            const int sw = isv ? (pcol ^ (prow & 6)) : (pcol ^ prow);
            attn_glds16(src + sw * 8, slot + isv * KB * 128 + pk * 1024);
        }
    };
    auto tiles_in = [&](int r) { return min(KG, nkt - r * KG); };  // valid tiles of round r
    auto issue_round = [&](int r) {
        for (int j = 0; j < tiles_in(r); ++j) issue_tile(r * KG + j);
    };
    // Q image: 8 pieces over the first 8 waves (rows past the block's end re-read the last query)
    if (w < 8) {
#pragma unroll
        for (int i = 0; i < (NWV >= 8 ? 1 : 8 / NWV); ++i) {
            const int piece = NWV >= 8 ? w : w * (8 / NWV) + i, r = piece * 8 + prow;
            const T* src = qkv + ((int64_t)s * pitch + min(q0 + r, qend - 1)) * rs + h * D;
            attn_glds16(src + ((pcol ^ prow) * 8), qimg + piece * 1024);
        }
    }
    // the whole stream when it fits the ring (no slot reuse), else R - 1 rounds ahead of the consumer
    const int pro = nr <= R ? nr : R - 1;
    for (int r = 0; r < pro; ++r) issue_round(r);

    const float cexp = p.scale * 1.4426950408889634f;
    float m_run = -1e30f, l_run = 0.f;
    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    u32x4 qf[2];
    const int qr = l16 >> 2, pc = l16 & 3;

    for (int r = 0; r < nr; ++r) {
        // this wave's DMA of round r (and of Q, issued first) has landed once at most the pieces
        // of the rounds issued after it are outstanding
        int after = 0;
        for (int r2 = r + 1; r2 <= (nr <= R ? nr - 1 : min(nr - 1, r + R - 2)); ++r2) after += ppw * tiles_in(r2);
        attn_wait_dyn(after);
        lds_barrier();  // every wave's pieces of round r landed; every wave is done with round r-1
        if (nr > R && r + R - 1 < nr) issue_round(r + R - 1);  // refills the slots of round r-1
        if (r == 0) {
            MMT_ASTAMP(2, "s_memtime");
#pragma unroll
            for (int t = 0; t < 2; ++t)
                qf[t] = *(const u32x4*)(qimg + ((16 * qw + l16) * 8 + ((4 * t + lg) ^ (l16 & 7))) * 16);
        }
        const int kt = r * KG + kg;
        if (kt >= nkt) continue;  // wave-uniform: this group has no tile in the last round
        const char* kimg = lds + (kt % NS) * ATILE;
        const char* vimg = kimg + KB * 128;
        // V^T fragments for the PV product, issued first so they land behind the QK^T work:
        // vt[kk][dt] = keys 32kk + 4lg + qr (+16), d = dt*16 + 4pc..+3
        uint2 vt[2][4][2];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int row = 32 * kk + 4 * lg + qr;  // and row + 16: same (row & 6)
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                const char* b1 = vimg + row * 128 + (((2 * dt + (pc >> 1)) ^ (row & 6)) * 16) + (pc & 1) * 8;
                vt[kk][dt][0] = attn_tr16<0>(b1);
                vt[kk][dt][1] = attn_tr16<16 * 128>(b1);
            }
        }
        // S^T tiles: sacc[kt16], lane: query l16, keys 16*kt16 + 4*lg + r
        u32x4 kf[4][2];
#pragma unroll
        for (int kt16 = 0; kt16 < 4; ++kt16)
#pragma unroll
            for (int t = 0; t < 2; ++t)
                kf[kt16][t] = *(const u32x4*)(kimg + ((kt16 * 16 + l16) * 8 + ((4 * t + lg) ^ (l16 & 7))) * 16);
        f32x4 sacc[4];
#pragma unroll
        for (int kt16 = 0; kt16 < 4; ++kt16) {
            sacc[kt16] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int t = 0; t < 2; ++t)
                sacc[kt16] = mfma16x16x32<T>(kf[kt16][t], qf[t], sacc[kt16]);
        }
        if (kt * KB + KB > Lk) {  // mask the tail of the key range (clamped rows)
#pragma unroll
            for (int kt16 = 0; kt16 < 4; ++kt16)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (kt * KB + kt16 * 16 + 4 * lg + j >= Lk) sacc[kt16][j] = -1e30f;
        }
        // online softmax (per query column)
        float mx = -1e30f;
#pragma unroll
        for (int kt16 = 0; kt16 < 4; ++kt16)
#pragma unroll
            for (int j = 0; j < 4; ++j) mx = fmaxf(mx, sacc[kt16][j]);
        mx = lanegroup_max(mx);
        const float mnew = fmaxf(m_run, mx);
        const float alpha = __builtin_amdgcn_exp2f((m_run - mnew) * cexp);
        m_run = mnew;
        const float mc = mnew * cexp;
        float ls = 0.f;
#pragma unroll
        for (int kt16 = 0; kt16 < 4; ++kt16)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float e = __builtin_amdgcn_exp2f(sacc[kt16][j] * cexp - mc);
                sacc[kt16][j] = e;
                ls += e;
            }
        l_run = l_run * alpha + ls;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
        // O^T += V^T P^T
        attn_lds_wait();
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const u32x4 pf = u32x4{pack2<T>(sacc[2 * kk][0], sacc[2 * kk][1]), pack2<T>(sacc[2 * kk][2], sacc[2 * kk][3]),
                                   pack2<T>(sacc[2 * kk + 1][0], sacc[2 * kk + 1][1]),
                                   pack2<T>(sacc[2 * kk + 1][2], sacc[2 * kk + 1][3])};
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                const uint2 ua = vt[kk][dt][0], ub = vt[kk][dt][1];
                o[dt] = mfma16x16x32<T>(u32x4{ua.x, ua.y, ub.x, ub.y}, pf, o[dt]);
            }
        }
    }
    MMT_ASTAMP(3, "s_memtime");

    // ---- merge the key groups' states (m, partial l, O) through LDS, group 0 finishes
    if constexpr (KG > 1) {
        float* mg = (float*)lds;  // [KG][4 waves][64 lanes][20]: m, l, -, -, O (16-B aligned)
        constexpr int ST = 20;
        lds_barrier();                           // ring no longer read by anyone
        float* mine = mg + ((kg * 4 + qw) * 64 + lane) * ST;
        if (kg > 0) {
            mine[0] = m_run;
            mine[1] = l_run;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) *(f32x4*)(mine + 4 + 4 * dt) = o[dt];
        }
        lds_barrier();
        if (kg > 0) return;
        float mall = m_run;
#pragma unroll
        for (int g2 = 1; g2 < KG; ++g2) mall = fmaxf(mall, mg[((g2 * 4 + qw) * 64 + lane) * ST]);
        const float a0 = __builtin_amdgcn_exp2f((m_run - mall) * cexp);
        l_run *= a0;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[dt] *= a0;
#pragma unroll
        for (int g2 = 1; g2 < KG; ++g2) {
            const float* src = mg + ((g2 * 4 + qw) * 64 + lane) * ST;
            const float ag = __builtin_amdgcn_exp2f((src[0] - mall) * cexp);
            l_run += src[1] * ag;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int j = 0; j < 4; ++j) o[dt][j] += src[4 + 4 * dt + j] * ag;
        }
    }

    // ---- normalise and store: lane holds O[q = l16][d = dt*16 + 4*lg + r]
    const float inv = 1.f / lanegroup_sum(l_run);
    const int q = q0 + 16 * qw + l16;
    if (q < qend) {
        T* op = (T*)p.out + attn_out_row(p, s, q, pitch) * C + h * D;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
            *(uint2*)(op + dt * 16 + 4 * lg) =
                make_uint2(pack2<T>(o[dt][0] * inv, o[dt][1] * inv), pack2<T>(o[dt][2] * inv, o[dt][3] * inv));
    }
#if MMT_STAMP_BUILD
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    MMT_ASTAMP(4, "s_memtime");
    MMT_ASTAMP(5, "s_memrealtime");
}


// ---------------------------------------------------------------------------------------------
// Throughput kernel for large grids (batched inference): one workgroup = 4 waves x 32 queries =
// 128 queries of one (sequence, head), OCC workgroups per CU.  Each K / V fragment read from LDS
// feeds two 16-query MFMA tiles (half the LDS traffic per FLOP of the latency kernel), and the
// softmax is trimmed to one transcendental + ~1 other VALU op per score, since at d = 64 the VALU
// work per score is as long as its 256 MFMA FLOPs:
//   - Q arrives pre-multiplied by scale*log2(e) (folded into the qkv weights by the runtime, or
//     applied here once if scale*log2(e) != 1), and the QK^T accumulators start at -m (the running
//     maximum) instead of 0, so exp2 of the accumulator IS the unnormalised probability;
//   - the running maximum is the first key tile's maximum and is raised only when a later tile's
//     scores exceed it by more than FA_THR (log2 units; then that tile rescales O and l), so most
//     tiles skip the rescale entirely (a wave-uniform branch);
//   - the row sums l come from one extra MFMA per 32 keys against an all-ones operand (the same
//     bf16 P that multiplies V), not from per-score adds.
// K / V tiles stream through an FNS-deep LDS-DMA ring (counted vmcnt + raw barrier, one barrier
// per tile).  The MFMA / VALU overlap comes from the OCC co-resident workgroups (a software-
// pipelined variant with one workgroup per CU measured 2.6x slower).  When the key segments are
// 64-aligned (n_t % 64 == 0) a tile never straddles a segment and its DMA source is one
// wave-uniform row base plus per-lane constant offsets.
#ifndef MMT_ATTN_FA_MIN_WG
#define MMT_ATTN_FA_MIN_WG 200  // workgroups of the throughput kernel from which it is chosen
#endif
#ifndef MMT_ATTN_LZ2_MIN_WG
// from this many 128-query workgroups (B >= 8 at ViT-B) the 64-queries-per-wave kernel (impl 22) is
// the default: 2-wave workgroups underfill the SIMDs below it (B = 6: 21.5 vs 20.3 us; B = 8: 25.0
// vs 27.0, B = 32: 78.6 vs 85.4 against impl 21, profiles/r02_lz2_ab.jsonl)
#define MMT_ATTN_LZ2_MIN_WG 900
#endif
constexpr float FA_THR = 8.f;

template <typename T, int FNS, int OCC>  // storage type, ring depth, workgroups per CU
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, OCC))) void mam_attention_fa_kernel(
    const mmt_attn_params p) {
    __shared__ __attribute__((aligned(1024))) char lds[FNS * FTILE + FQ * 128];
    char* qimg = lds + FNS * FTILE;

    const int n_t = p.n_t, ntok = p.ntok, C = p.C;
    const int64_t pitch = p.tok_pitch > 0 ? p.tok_pitch : ntok;  // rows between sequences
    const int nqb_t = (n_t + FQ - 1) / FQ;
    int bx, h, s;
    attn_block_ids(bx, h, s);
    const int qb = bx + (p.q_part == 2 ? nqb_t : 0);
    const bool tmpl = qb < nqb_t;
    const int q0 = tmpl ? qb * FQ : n_t + (qb - nqb_t) * FQ;
    const int qend = tmpl ? n_t : ntok;
    const int Lk = tmpl ? n_t : (p.asym ? ntok + n_t : ntok);
    const bool cross = p.asym && !tmpl;
    const int64_t rs = 3 * (int64_t)C;
    const T* qkv = (const T*)p.qkv;
    const int sV = s % p.Bm, sI = sV + p.Bm;

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int l16 = lane & 15, lg = lane >> 4;
    const int prow = lane >> 3, pcol = lane & 7;
    const int qr = l16 >> 2, pc = l16 & 3;

    // ---- K / V DMA.  This wave's 4 pieces of a tile: piece w*4+i (waves 0-1: K, 2-3: V), rows
    // pk*8 + prow of the tile, this lane's swizzled 16-B chunk.
    const int isv = w >> 1;
    const int64_t col = (isv ? 2 * C : C) + h * D + (isv ? (pcol ^ (prow & 6)) : (pcol ^ prow)) * 8;
    auto key_row = [&](int kk) -> const T* {
        int seq = s, row = kk;
        if (cross) {
            if (kk < n_t) seq = sV;
            else if (kk < 2 * n_t) { seq = sI; row = kk - n_t; }
            else row = kk - n_t;
        }
        return qkv + ((int64_t)seq * pitch + row) * rs;
    };
    const bool aligned = n_t % KB == 0;  // every tile lies in one key segment
    const int nkt = (Lk + KB - 1) / KB;
    auto issue_tile = [&](int t) {
        MMT_ATTN_ASSERT(t >= 0 && t < nkt);
        char* slot = lds + (t % FNS) * FTILE + isv * KB * 128;
        if (aligned && t * KB + KB <= Lk) {
            const T* base = key_row(t * KB);  // wave-uniform
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int pk = (w & 1) * 4 + i;
                attn_glds16(base + (int64_t)(pk * 8 + prow) * rs + col, slot + pk * 1024);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int pk = (w & 1) * 4 + i;
                attn_glds16(key_row(min(t * KB + pk * 8 + prow, Lk - 1)) + col, slot + pk * 1024);
            }
        }
    };
    // Q image: 128 rows (16 pieces, 4 per wave); rows past the block's end re-read the last query
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int piece = w * 4 + i, r = piece * 8 + prow;
        const T* src = qkv + ((int64_t)s * pitch + min(q0 + r, qend - 1)) * rs + h * D;
        attn_glds16(src + ((pcol ^ prow) * 8), qimg + piece * 1024);
    }
    for (int t = 0; t < FNS - 1 && t < nkt; ++t) issue_tile(t);

    const bool active = q0 + 32 * w < qend;  // wave-uniform: this wave has queries
    const float cexp = p.scale * 1.4426950408889634f;
    const bool prescale = fabsf(cexp - 1.f) > 1e-6f;
    float mr[2] = {0.f, 0.f};
    f32x4 o[4][2], lsum[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
        lsum[qt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[dt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const u32x4 ones = u32x4{one2<T>(), one2<T>(), one2<T>(), one2<T>()};
    u32x4 qf[2][2];

    for (int kt = 0; kt < nkt; ++kt) {
        attn_wait_dyn(4 * (min(nkt - 1, kt + FNS - 2) - kt));
        lds_barrier();  // every wave's pieces of tile kt landed; every wave is done with tile kt-1
        if (kt + FNS - 1 < nkt) issue_tile(kt + FNS - 1);
        if (kt == 0) {
#pragma unroll
            for (int qt = 0; qt < 2; ++qt)
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int row = 32 * w + 16 * qt + l16;
                    qf[qt][u] = *(const u32x4*)(qimg + (row * 8 + ((4 * u + lg) ^ (l16 & 7))) * 16);
                    if (prescale) {
                        u32x4 v = qf[qt][u];
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            v[e] = pack2<T>(unpack2<T>(v[e])[0] * cexp, unpack2<T>(v[e])[1] * cexp);
                        qf[qt][u] = v;
                    }
                }
        }
        if (!active) continue;
        const char* kimg = lds + (kt % FNS) * FTILE;
        const char* vimg = kimg + KB * 128;
        uint2 vt[2][4][2];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int row = 32 * kk + 4 * lg + qr;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                const char* b1 = vimg + row * 128 + (((2 * dt + (pc >> 1)) ^ (row & 6)) * 16) + (pc & 1) * 8;
                vt[kk][dt][0] = attn_tr16<0>(b1);
                vt[kk][dt][1] = attn_tr16<16 * 128>(b1);
            }
        }
        u32x4 kf[4][2];
#pragma unroll
        for (int kt16 = 0; kt16 < 4; ++kt16)
#pragma unroll
            for (int u = 0; u < 2; ++u)
                kf[kt16][u] = *(const u32x4*)(kimg + ((kt16 * 16 + l16) * 8 + ((4 * u + lg) ^ (l16 & 7))) * 16);
        // S^T - m: the accumulators start at -m (per query column = per lane)
        f32x4 sacc[4][2];
#pragma unroll
        for (int kt16 = 0; kt16 < 4; ++kt16)
#pragma unroll
            for (int qt = 0; qt < 2; ++qt) {
                sacc[kt16][qt] = f32x4{-mr[qt], -mr[qt], -mr[qt], -mr[qt]};
#pragma unroll
                for (int u = 0; u < 2; ++u)
                    sacc[kt16][qt] = mfma16x16x32<T>(kf[kt16][u], qf[qt][u], sacc[kt16][qt]);
            }
        if (kt * KB + KB > Lk) {
#pragma unroll
            for (int kt16 = 0; kt16 < 4; ++kt16)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (kt * KB + kt16 * 16 + 4 * lg + j >= Lk) sacc[kt16][0][j] = sacc[kt16][1][j] = -1e30f;
        }
        float mx[2];
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
            float m = sacc[0][qt][0];
#pragma unroll
            for (int kt16 = 0; kt16 < 4; ++kt16)
#pragma unroll
                for (int j = 0; j < 4; ++j) m = fmaxf(m, sacc[kt16][qt][j]);
            mx[qt] = lanegroup_max(m);
        }
        if (kt == 0 || __any(mx[0] > FA_THR || mx[1] > FA_THR)) {  // (re)base the running maximum
#pragma unroll
            for (int qt = 0; qt < 2; ++qt) {
                const float d = kt == 0 ? mx[qt] : fmaxf(mx[qt], 0.f);
                mr[qt] += d;
                const float alpha = __builtin_amdgcn_exp2f(-d);
#pragma unroll
                for (int kt16 = 0; kt16 < 4; ++kt16) sacc[kt16][qt] -= d;
#pragma unroll
                for (int dt = 0; dt < 4; ++dt) o[dt][qt] *= alpha;
                lsum[qt] *= alpha;
            }
        }
#pragma unroll
        for (int kt16 = 0; kt16 < 4; ++kt16)
#pragma unroll
            for (int qt = 0; qt < 2; ++qt)
#pragma unroll
                for (int j = 0; j < 4; ++j) sacc[kt16][qt][j] = __builtin_amdgcn_exp2f(sacc[kt16][qt][j]);
        attn_lds_wait();
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            u32x4 pf[2];
#pragma unroll
            for (int qt = 0; qt < 2; ++qt)
                pf[qt] = u32x4{pack2<T>(sacc[2 * kk][qt][0], sacc[2 * kk][qt][1]),
                               pack2<T>(sacc[2 * kk][qt][2], sacc[2 * kk][qt][3]),
                               pack2<T>(sacc[2 * kk + 1][qt][0], sacc[2 * kk + 1][qt][1]),
                               pack2<T>(sacc[2 * kk + 1][qt][2], sacc[2 * kk + 1][qt][3])};
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                const uint2 ua = vt[kk][dt][0], ub = vt[kk][dt][1];
                const u32x4 vf = u32x4{ua.x, ua.y, ub.x, ub.y};
#pragma unroll
                for (int qt = 0; qt < 2; ++qt) o[dt][qt] = mfma16x16x32<T>(vf, pf[qt], o[dt][qt]);
            }
#pragma unroll
            for (int qt = 0; qt < 2; ++qt) lsum[qt] = mfma16x16x32<T>(ones, pf[qt], lsum[qt]);
        }
    }

    // ---- normalise and store: lane holds O[q = l16][d = dt*16 + 4*lg + r]; every row of lsum = l
    if (!active) return;
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
        const float inv = 1.f / lsum[qt][0];
        const int q = q0 + 32 * w + 16 * qt + l16;
        if (q < qend && p.lse && lg == 0)  // training: log2-sum-exp2 of the pre-scaled scores
            p.lse[((int64_t)s * p.H + h) * ntok + q] = mr[qt] + __builtin_amdgcn_logf(lsum[qt][0]);
        if (q < qend) {
            T* op = (T*)p.out + attn_out_row(p, s, q, pitch) * C + h * D;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
                *(uint2*)(op + dt * 16 + 4 * lg) = make_uint2(pack2<T>(o[dt][qt][0] * inv, o[dt][qt][1] * inv),
                                                              pack2<T>(o[dt][qt][2] * inv, o[dt][qt][3] * inv));
        }
    }
}



// ---------------------------------------------------------------------------------------------
// Range-checked exponent kernel (impl 17 / 21; 22 below is its 64-queries-per-wave form).  At d = 64 a score
// carries only 256 MFMA FLOPs, so the softmax's per-score VALU work decides the rate.  This
// kernel removes all of it except the exponential and the bf16 pack:
//   - no running maximum.  softmax(s) = exp2(s) / sum exp2(s) for any common reference point,
//     so with the scores already in log2 units (q pre-multiplied by scale*log2(e)) the kernel
//     uses 0 as the reference: P = exp2(S) straight off the QK^T accumulators.  This is exact
//     (bf16 rounds relative to the value) as long as nothing leaves fp32 range; the epilogue
//     checks exactly that (row sum l in [2^-100, 2^100], O finite) and a wave whose check fails
//     recomputes its 32 queries with an exact two-pass fp32 softmax (fallback below), so extreme
//     scores cost time, never accuracy;
//   - the row sums come out of the matrix pipe: one v_mfma_f32_16x16x32_bf16 per 16 keys against
//     a constant 0/1 selector operand (A[m][k] = 1 iff bit 2 of m == bit 3 of k) sums the same
//     bf16 P fragment that multiplies V, and lands lane l's sum for its own query l%32 in every
//     element of its accumulator (no cross-lane step) (SUM_MFMA = false: VALU adds, A/B only);
//   - 32x32x16 MFMAs throughout (an MFMA holds the SIMD's vector issue for 8 of its 32 cycles,
//     against 8 of 16 for the 16x16x32 form), so at most 1/4 of the issue slots go to the matrix
//     instructions and the rest stay free for v_exp / v_cvt_pk of the co-resident waves.
// Geometry: one workgroup = 4 waves x 32 queries of one (sequence, head); key tiles of 64 stream
// through an FNS-deep LDS-DMA ring (the K / V images and swizzles of the 32x32x16 kernel above);
// OCC workgroups per CU.  S^T = K Q^T puts query l%32 on lane l (keys 8(r/4) + 4(l/32) + r%4 in
// accumulator element r), and P^T feeds O^T = V^T P^T as the B operand directly, with V^T read in
// the matching key order by ds_read_b64_tr_b16.  The last tile computes only the 16-key steps
// that hold valid keys (528 = 8 x 64 + 16).  The block -> tile map is XCD-aware at every grid size
// (the query blocks of one (sequence, head) share one XCD's L2 for their K / V re-reads).
// MMT_ATTN_ABLATE (measurement builds only, tools/build_ablate.sh; results are wrong): 1 = no K/V
// DMA after the prologue, 2 = no matrix / softmax work, 3 = no exponentials (P = S)
#ifndef MMT_ATTN_ABLATE
#define MMT_ATTN_ABLATE 0
#endif



// PIPE: the two 32-key blocks of a full tile software-pipelined inside the wave (impl 21, the
// large-grid default): both blocks' scores are computed before either block's exponentials, so
// block 1's QK^T MFMAs run beside block 0's v_exp / packs and block 0's PV MFMAs beside block 1's,
// and one wave's dependency chain (scores -> exp -> PV) stops idling the matrix pipe on its own
// VALU.  B = 32: 78.9 vs 83.8 us, asym 88.5 vs 93.2; B = 8: 27.2 vs 29.8 (same run, bit-identical
// output).  Measured and dropped: sched_group_barrier interleave hints (79.3), the block-1 PV moved
// past the next tile's barrier (79.6), 2 workgroups per CU (85.3).
template <int FNS, int OCC, bool SUM_MFMA, bool PIPE = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, OCC))) void mam_attention_lz_kernel(
    const mmt_attn_params p) {
    __shared__ __attribute__((aligned(1024))) char lds[FNS * FTILE];

    const int n_t = p.n_t, ntok = p.ntok, C = p.C;
    const int64_t pitch = p.tok_pitch > 0 ? p.tok_pitch : ntok;  // rows between sequences
    const int nqb_t = (n_t + FQ - 1) / FQ;
    int bx, h, s;
    attn_block_ids_xcd(bx, h, s);
    const int qb = bx + (p.q_part == 2 ? nqb_t : 0);
    const bool tmpl = qb < nqb_t;
    const int q0 = tmpl ? qb * FQ : n_t + (qb - nqb_t) * FQ;
    const int qend = tmpl ? n_t : ntok;
    const int Lk = tmpl ? n_t : (p.asym ? ntok + n_t : ntok);
    const bool cross = p.asym && !tmpl;
    const int64_t rs = 3 * (int64_t)C;
    const bf16_t* qkv = (const bf16_t*)p.qkv;
    const int sV = s % p.Bm, sI = sV + p.Bm;

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int l32 = lane & 31, hf = lane >> 5;
    const int prow = lane >> 3, pcol = lane & 7;

    // ---- K / V DMA (waves 0-1: K, 2-3: V), 4 pieces of 8 rows x 128 B per wave per tile
    const int isv = w >> 1;
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
    const bool aligned = n_t % KB == 0;  // every full tile lies in one key segment
    const int nkt = (Lk + KB - 1) / KB;
    auto issue_tile = [&](int t) {
        MMT_ATTN_ASSERT(t >= 0 && t < nkt);
        char* slot = lds + (t % FNS) * FTILE + isv * KB * 128;
        if (aligned && t * KB + KB <= Lk) {
            const bf16_t* base = key_row(t * KB);  // wave-uniform
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int pk = (w & 1) * 4 + i;
                attn_glds16(base + (int64_t)(pk * 8 + prow) * rs + col, slot + pk * 1024);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int pk = (w & 1) * 4 + i;
                attn_glds16(key_row(min(t * KB + pk * 8 + prow, Lk - 1)) + col, slot + pk * 1024);
            }
        }
    };
    // Q image (128 rows x 128 B, rows past the block's end re-read the last query) in the last ring
    // slot: read into registers at the first tile, before that slot's first refill
    char* qimg = lds + (FNS - 1) * FTILE;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int piece = w * 4 + i, r = piece * 8 + prow;
        const bf16_t* src = qkv + ((int64_t)s * pitch + min(q0 + r, qend - 1)) * rs + h * D;
        attn_glds16(src + ((pcol ^ prow) * 8), qimg + piece * 1024);
    }
    for (int t = 0; t < FNS - 1 && t < nkt; ++t) issue_tile(t);

    const bool active = q0 + 32 * w < qend;  // wave-uniform: this wave has queries
    const int q = q0 + 32 * w + l32;
    const int qc = min(q, qend - 1);
    const float cexp = p.scale * 1.4426950408889634f;
    const bool prescale = fabsf(cexp - 1.f) > 1e-6f;
    u32x4 qf[4];  // B operand of S^T = K Q^T: query q, d = 16ks + 8hf .. +7

    f32x16 o[2];
#pragma unroll
    for (int r = 0; r < 16; ++r) { o[0][r] = 0.f; o[1][r] = 0.f; }
    f32x4 lacc = f32x4{0.f, 0.f, 0.f, 0.f};  // SUM_MFMA: row sums (every element = this lane's query)
    float lsum0 = 0.f, lsum1 = 0.f;          // VALU row sums (half of this lane's query's keys)
    // selector operand of the row-sum MFMA: lane l holds A[l%16][8(l/16) .. +7]
    const float one_or_zero = (((lane & 15) >> 2) & 1) == ((lane >> 4) & 1) ? 1.f : 0.f;
    const uint32_t sel_w = pack_bf16x2(one_or_zero, one_or_zero);
    const bf16x8 sel = __builtin_bit_cast(bf16x8, u32x4{sel_w, sel_w, sel_w, sel_w});

    const int kpos = (l32 & 7) * 16;
    const int li = lane & 15, qr = li >> 2, pc = li & 3, dsub = (lane >> 4) & 1;

    // one 32-key block kb of a tile: NJ 16-key steps (2 = the whole block), MASK = zero P past Lk
    auto block = [&](const char* kimg, int kb, int nv, auto NJc, auto MASKc) {
        constexpr int NJ = decltype(NJc)::value;
        constexpr bool MASK = decltype(MASKc)::value;
        const char* vimg = kimg + KB * 128;
        const char* krow = kimg + (32 * kb + l32) * 128;
        u32x4 kf[4];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) kf[ks] = *(const u32x4*)(krow + ((((2 * ks + hf) * 16) ^ kpos)));
        f32x16 sacc;
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[r] = 0.f;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
            sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kf[ks]),
                                                           __builtin_bit_cast(bf16x8, qf[ks]), sacc, 0, 0, 0);
        // V^T fragments of the block's 16-key steps, issued behind the QK^T MFMAs
        uint2 vt[NJ][2][2];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int row = 32 * kb + 16 * j + 4 * hf + qr;
#pragma unroll
            for (int db = 0; db < 2; ++db) {
                const char* b1 = vimg + row * 128 + (((4 * db + 2 * dsub + (pc >> 1)) ^ attn_vswz(row)) * 16) + (pc & 1) * 8;
                vt[j][db][0] = attn_tr16<0>(b1);
                vt[j][db][1] = attn_tr16<8 * 128>(b1);
            }
        }
        // P = exp2(S) (the scores are in log2 units; no reference point, see above)
#pragma unroll
        for (int r = 0; r < 8 * NJ; ++r) {
            float e = (MMT_ATTN_ABLATE == 3 || MMT_ATTN_ABLATE == 6) ? sacc[r] : __builtin_amdgcn_exp2f(sacc[r]);
            if constexpr (MASK) {
                if (32 * kb + 8 * (r >> 2) + 4 * hf + (r & 3) >= nv) e = 0.f;
            }
            sacc[r] = e;
            if constexpr (!SUM_MFMA) {
                if (r & 1) lsum1 += e;  // single v_add_f32: this file builds with -fno-slp-vectorize
                else lsum0 += e;
            }
        }
        attn_lds_wait();
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int rb = 8 * j;
            const bf16x8 pf = __builtin_bit_cast(
                bf16x8, u32x4{pack_bf16x2(sacc[rb], sacc[rb + 1]), pack_bf16x2(sacc[rb + 2], sacc[rb + 3]),
                              pack_bf16x2(sacc[rb + 4], sacc[rb + 5]), pack_bf16x2(sacc[rb + 6], sacc[rb + 7])});
#pragma unroll
            for (int db = 0; db < 2; ++db) {
                const uint2 ua = vt[j][db][0], ub = vt[j][db][1];
                const bf16x8 vf = __builtin_bit_cast(bf16x8, make_uint4(ua.x, ua.y, ub.x, ub.y));
                o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, o[db], 0, 0, 0);
            }
            if constexpr (SUM_MFMA) lacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel, pf, lacc, 0, 0, 0);
        }
    };

    // tile kt's pieces landed (this wave: counted vmcnt; every wave: the barrier) and every wave is
    // done with tile kt-1, whose slot then takes tile kt + FNS - 1
    auto next_tile = [&](int kt) {
        attn_wait_dyn(4 * (min(nkt - 1, kt + FNS - 2) - kt));
        lds_barrier();
        if (MMT_ATTN_ABLATE != 1 && kt + FNS - 1 < nkt) issue_tile(kt + FNS - 1);
    };
    {  // tile 0 and Q: Q into registers, then its slot is free for tile FNS - 1
        attn_wait_dyn(4 * (min(nkt - 1, FNS - 2)));
        lds_barrier();
        const int row = 32 * w + l32;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            qf[ks] = *(const u32x4*)(qimg + row * 128 + (((2 * ks + hf) ^ (row & 7)) * 16));
            if (prescale) {  // natural-scale q (training / A/B callers): to log2 units
                u32x4 v = qf[ks];
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    v[e] = pack_bf16x2(__uint_as_float(v[e] << 16) * cexp, __uint_as_float(v[e] & 0xffff0000u) * cexp);
                qf[ks] = v;
            }
        }
        lds_barrier();
        if (MMT_ATTN_ABLATE != 1 && FNS - 1 < nkt) issue_tile(FNS - 1);
    }
    // a full tile, both blocks software-pipelined (PIPE; row sums on the matrix pipe)
    auto tile_pipe = [&](const char* kimg) {
        const char* vimg = kimg + KB * 128;
        auto vfrags = [&](int kb, uint2 (&vt)[2][2][2]) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int row = 32 * kb + 16 * j + 4 * hf + qr;
#pragma unroll
                for (int db = 0; db < 2; ++db) {
                    const char* b1 = vimg + row * 128 + (((4 * db + 2 * dsub + (pc >> 1)) ^ attn_vswz(row)) * 16) + (pc & 1) * 8;
                    vt[j][db][0] = attn_tr16<0>(b1);
                    vt[j][db][1] = attn_tr16<8 * 128>(b1);
                }
            }
        };
        auto pv = [&](const uint2 (&vt)[2][2][2], const f32x16& s) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int rb = 8 * j;
                const bf16x8 pf = __builtin_bit_cast(
                    bf16x8, u32x4{pack_bf16x2(s[rb], s[rb + 1]), pack_bf16x2(s[rb + 2], s[rb + 3]),
                                  pack_bf16x2(s[rb + 4], s[rb + 5]), pack_bf16x2(s[rb + 6], s[rb + 7])});
#pragma unroll
                for (int db = 0; db < 2; ++db) {
                    const uint2 ua = vt[j][db][0], ub = vt[j][db][1];
                    o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, make_uint4(ua.x, ua.y, ub.x, ub.y)),
                                                                    pf, o[db], 0, 0, 0);
                }
                lacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel, pf, lacc, 0, 0, 0);
            }
        };
        f32x16 s0, s1;
#pragma unroll
        for (int r = 0; r < 16; ++r) { s0[r] = 0.f; s1[r] = 0.f; }
        u32x4 k0[4], k1[4];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) k0[ks] = *(const u32x4*)(kimg + l32 * 128 + ((((2 * ks + hf) * 16) ^ kpos)));
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) k1[ks] = *(const u32x4*)(kimg + (32 + l32) * 128 + ((((2 * ks + hf) * 16) ^ kpos)));
        uint2 v0[2][2][2], v1[2][2][2];
        vfrags(0, v0);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
            s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, k0[ks]), __builtin_bit_cast(bf16x8, qf[ks]), s0, 0, 0, 0);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
            s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, k1[ks]), __builtin_bit_cast(bf16x8, qf[ks]), s1, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 16; ++r) s0[r] = (MMT_ATTN_ABLATE == 3 || MMT_ATTN_ABLATE == 6) ? s0[r] : __builtin_amdgcn_exp2f(s0[r]);
        vfrags(1, v1);
        // block 0's V^T reads (the 8 oldest of the 16 asm reads) landed; the wait redefines them
        asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(v0[0][0][0]), "+v"(v0[0][0][1]), "+v"(v0[0][1][0]), "+v"(v0[0][1][1]),
                     "+v"(v0[1][0][0]), "+v"(v0[1][0][1]), "+v"(v0[1][1][0]), "+v"(v0[1][1][1]));
        pv(v0, s0);
#pragma unroll
        for (int r = 0; r < 16; ++r) s1[r] = (MMT_ATTN_ABLATE == 3 || MMT_ATTN_ABLATE == 6) ? s1[r] : __builtin_amdgcn_exp2f(s1[r]);
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v1[0][0][0]), "+v"(v1[0][0][1]), "+v"(v1[0][1][0]), "+v"(v1[0][1][1]),
                     "+v"(v1[1][0][0]), "+v"(v1[1][0][1]), "+v"(v1[1][1][0]), "+v"(v1[1][1][1]));
        pv(v1, s1);
    };
    const int nfull = Lk / KB;  // full 64-key tiles; Lk % KB keys remain for a tail tile
    const bool compute = active && MMT_ATTN_ABLATE != 2;
    for (int kt = 0; kt < nfull; ++kt) {
        if (compute) {
            const char* kimg = lds + (kt % FNS) * FTILE;
            if constexpr (PIPE && SUM_MFMA) {
                tile_pipe(kimg);
            } else {
                block(kimg, 0, KB, attn_ic<2>{}, attn_ic<0>{});
                block(kimg, 1, KB, attn_ic<2>{}, attn_ic<0>{});
            }
        }
        if (kt + 1 < nkt) next_tile(kt + 1);
    }
    if (nfull < nkt && compute) {  // the tail tile: only the 16-key steps that hold valid keys
        const char* kimg = lds + (nfull % FNS) * FTILE;
        const int nv = Lk - nfull * KB;
        if (nv > 16) block(kimg, 0, nv, attn_ic<2>{}, attn_ic<1>{});
        else block(kimg, 0, nv, attn_ic<1>{}, attn_ic<1>{});
        if (nv > 48) block(kimg, 1, nv, attn_ic<2>{}, attn_ic<1>{});
        else if (nv > 32) block(kimg, 1, nv, attn_ic<1>{}, attn_ic<1>{});
    }
    if (!active) return;

    float l;
    if constexpr (SUM_MFMA) {
        l = lacc[0];
    } else {
        l = lsum0 + lsum1;
        auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(l), __float_as_uint(l), false, false);
        l = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    }
    float chk = 0.f;  // NaN iff some O element is not finite
#pragma unroll
    for (int r = 0; r < 16; ++r) chk += o[0][r] * 0.f + o[1][r] * 0.f;
    const bool ok = (l >= LZ_LO && l <= LZ_HI && chk == 0.f) || MMT_ATTN_ABLATE != 0;
    bf16_t* op = (bf16_t*)p.out + attn_out_row(p, s, q, pitch) * C + h * D;
    if (__builtin_expect(__all(ok), 1)) {
        const float inv = 1.f / l;
        if (q < qend) {
            if (p.lse && hf == 0) p.lse[((int64_t)s * p.H + h) * ntok + q] = __builtin_amdgcn_logf(l);
#pragma unroll
            for (int db = 0; db < 2; ++db)
#pragma unroll
                for (int g = 0; g < 4; ++g)
                    *(uint2*)(op + 32 * db + 8 * g + 4 * hf) =
                        make_uint2(pack_bf16x2(o[db][4 * g] * inv, o[db][4 * g + 1] * inv),
                                   pack_bf16x2(o[db][4 * g + 2] * inv, o[db][4 * g + 3] * inv));
        }
        return;
    }
    // ---- exact fallback (scores outside the fp32-safe range): two-pass fp32 softmax per query,
    // lane (query l32, half hf) owns d = 32hf .. 32hf+31 of the dot products and of O; K / V rows
    // come straight from global memory.  Rare by construction (|log2-scores| ~ 100).
    float qv[32], acc[32];
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
        if (p.lse && hf == 0) p.lse[((int64_t)s * p.H + h) * ntok + q] = m + __builtin_amdgcn_logf(lf);
#pragma unroll
        for (int i = 0; i < 32; i += 8)
            *(u32x4*)(op + 32 * hf + i) = u32x4{pack_bf16x2(acc[i] * inv, acc[i + 1] * inv), pack_bf16x2(acc[i + 2] * inv, acc[i + 3] * inv),
                                                pack_bf16x2(acc[i + 4] * inv, acc[i + 5] * inv), pack_bf16x2(acc[i + 6] * inv, acc[i + 7] * inv)};
    }
}

// ---- impl 22: the range-checked kernel with 64 queries per wave (large-grid default) ---------------
// Two 32-query blocks per wave share every K / V fragment the wave reads from LDS (half the LDS
// reads per FLOP of impl 17 / 21), and each wave carries two independent score -> exp -> PV chains;
// 2 waves x 64 queries = 128 queries per workgroup as before, 2 waves per SIMD (up to 256 registers),
// four workgroups per CU.  Wave 0 streams the tile's 8 K pieces, wave 1 its 8 V pieces.  The tile
// loop is instantiated per count of the wave's active query blocks (2 / 1), chosen once.
// SPLIT: block 1's exponentials after the V^T wait, below its scheduling barrier, so they interleave
// with block 0's PV MFMAs (B = 8 / 16 / 32: 26.6 / 47.2 / 78.8 -> 25.6 / 44.3 / 76.9 us, bit-identical)
// PIPE2: on full tiles both key blocks' scores (both query blocks) come before any exponential, so
// the second key block's QK^T MFMAs run beside the first block's softmax (B = 8 / 16 / 32: 27.2 /
// 47.1 / 75.2 -> 24.9 / 43.5 / 72.1 us, bit-identical; 243 VGPRs)
// One work item of impl 22 (query block bx of 128 queries, head h, sequence s); lds = FNS tile slots.
// Every LDS-DMA it issues has landed when it returns (the last tile's wait is vmcnt(0)); its output
// stores may still be in flight.  (A persistent form that looped over these items in a longest-first
// static order measured no faster: profiles/r03_attn_persistent_ab.jsonl.)
template <int FNS, bool SPLIT = true, bool PIPE2 = true>
MMT_DEV void mam_lz2_item(const mmt_attn_params& p, char* lds, const int bx, const int h, const int s) {
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

    const int isv = w;  // wave 0: K pieces, wave 1: V pieces
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
    const bool aligned = n_t % KB == 0;
    const int nkt = (Lk + KB - 1) / KB;
    auto issue_tile = [&](int t) {
        MMT_ATTN_ASSERT(t >= 0 && t < nkt);
        char* slot = lds + (t % FNS) * FTILE + isv * KB * 128;
        if (aligned && t * KB + KB <= Lk) {
            const bf16_t* base = key_row(t * KB);
#pragma unroll
            for (int pk = 0; pk < 8; ++pk) attn_glds16(base + (int64_t)(pk * 8 + prow) * rs + col, slot + pk * 1024);
        } else {
#pragma unroll
            for (int pk = 0; pk < 8; ++pk) attn_glds16(key_row(min(t * KB + pk * 8 + prow, Lk - 1)) + col, slot + pk * 1024);
        }
    };
    char* qimg = lds + (FNS - 1) * FTILE;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int piece = w * 8 + i, r = piece * 8 + prow;
        const bf16_t* src = qkv + ((int64_t)s * pitch + min(q0 + r, qend - 1)) * rs + h * D;
        attn_glds16(src + ((pcol ^ prow) * 8), qimg + piece * 1024);
    }
    for (int t = 0; t < FNS - 1 && t < nkt; ++t) issue_tile(t);

    const int qbase = q0 + 64 * w;  // query blocks qbase + 32 qb + [0, 32)
    const int nqa = (qbase < qend ? 1 : 0) + (qbase + 32 < qend ? 1 : 0);
    const float cexp = p.scale * 1.4426950408889634f;
    const bool prescale = fabsf(cexp - 1.f) > 1e-6f;
    const float one_or_zero = (((lane & 15) >> 2) & 1) == ((lane >> 4) & 1) ? 1.f : 0.f;
    const uint32_t sel_w = pack_bf16x2(one_or_zero, one_or_zero);
    const bf16x8 sel = __builtin_bit_cast(bf16x8, u32x4{sel_w, sel_w, sel_w, sel_w});
    const int kpos = (l32 & 7) * 16;
    const int li = lane & 15, qr = li >> 2, pc = li & 3, dsub = (lane >> 4) & 1;

    auto next_tile = [&](int kt) {
        if (MMT_ATTN_ABLATE == 5 || MMT_ATTN_ABLATE == 6) return;  // measurement builds: free-running waves (no waits / barriers / refills; 6: no exponentials either)
        attn_wait_dyn(8 * (min(nkt - 1, kt + FNS - 2) - kt));
        lds_barrier();
        if (MMT_ATTN_ABLATE != 1 && kt + FNS - 1 < nkt) issue_tile(kt + FNS - 1);
    };
    u32x4 qf[2][4];
    {  // tile 0 and Q landed; Q into registers, then its slot takes tile FNS - 1
        attn_wait_dyn(8 * (min(nkt - 1, FNS - 2)));
        lds_barrier();
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
            const int row = 64 * w + 32 * qb + l32;
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                qf[qb][ks] = *(const u32x4*)(qimg + row * 128 + (((2 * ks + hf) ^ (row & 7)) * 16));
                if (prescale) {
                    u32x4 v = qf[qb][ks];
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        v[e] = pack_bf16x2(__uint_as_float(v[e] << 16) * cexp, __uint_as_float(v[e] & 0xffff0000u) * cexp);
                    qf[qb][ks] = v;
                }
            }
        }
        lds_barrier();
        if (FNS - 1 < nkt) issue_tile(FNS - 1);
    }
    const int nfull = Lk / KB;

    auto run = [&](auto NQc) {
        constexpr int NQ = decltype(NQc)::value;
        f32x16 o[NQ][2];
        f32x4 lacc[NQ];
#pragma unroll
        for (int qb = 0; qb < NQ; ++qb) {
#pragma unroll
            for (int r = 0; r < 16; ++r) { o[qb][0][r] = 0.f; o[qb][1][r] = 0.f; }
            lacc[qb] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        auto block = [&](const char* kimg, int kb, int nv, auto NJc, auto MASKc) {
            constexpr int NJ = decltype(NJc)::value;
            constexpr bool MASK = decltype(MASKc)::value;
            const char* vimg = kimg + KB * 128;
            const char* krow = kimg + (32 * kb + l32) * 128;
            u32x4 kf[4];
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) kf[ks] = *(const u32x4*)(krow + ((((2 * ks + hf) * 16) ^ kpos)));
            f32x16 sacc[NQ];
#pragma unroll
            for (int qb = 0; qb < NQ; ++qb) {
#pragma unroll
                for (int r = 0; r < 16; ++r) sacc[qb][r] = 0.f;
#pragma unroll
                for (int ks = 0; ks < 4; ++ks)
                    sacc[qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kf[ks]),
                                                                       __builtin_bit_cast(bf16x8, qf[qb][ks]), sacc[qb], 0, 0, 0);
            }
            uint2 vt[NJ][2][2];
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int row = 32 * kb + 16 * j + 4 * hf + qr;
#pragma unroll
                for (int db = 0; db < 2; ++db) {
                    const char* b1 = vimg + row * 128 + (((4 * db + 2 * dsub + (pc >> 1)) ^ attn_vswz(row)) * 16) + (pc & 1) * 8;
                    vt[j][db][0] = attn_tr16<0>(b1);
                    vt[j][db][1] = attn_tr16<8 * 128>(b1);
                }
            }
            auto expo = [&](int qb) {
#pragma unroll
                for (int r = 0; r < 8 * NJ; ++r) {
                    float e = (MMT_ATTN_ABLATE == 3 || MMT_ATTN_ABLATE == 6) ? sacc[qb][r] : __builtin_amdgcn_exp2f(sacc[qb][r]);
                    if constexpr (MASK) {
                        if (32 * kb + 8 * (r >> 2) + 4 * hf + (r & 3) >= nv) e = 0.f;
                    }
                    sacc[qb][r] = e;
                }
            };
            if constexpr (SPLIT && NQ == 2) {
                expo(0);
                attn_lds_wait();
                expo(1);  // below the wait's scheduling barrier: free to interleave with block 0's PV
            } else {
#pragma unroll
                for (int qb = 0; qb < NQ; ++qb) expo(qb);
                attn_lds_wait();
            }
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int rb = 8 * j;
                bf16x8 vf[2];
#pragma unroll
                for (int db = 0; db < 2; ++db) {
                    const uint2 ua = vt[j][db][0], ub = vt[j][db][1];
                    vf[db] = __builtin_bit_cast(bf16x8, make_uint4(ua.x, ua.y, ub.x, ub.y));
                }
#pragma unroll
                for (int qb = 0; qb < NQ; ++qb) {
                    const bf16x8 pf = __builtin_bit_cast(
                        bf16x8, u32x4{pack_bf16x2(sacc[qb][rb], sacc[qb][rb + 1]), pack_bf16x2(sacc[qb][rb + 2], sacc[qb][rb + 3]),
                                      pack_bf16x2(sacc[qb][rb + 4], sacc[qb][rb + 5]), pack_bf16x2(sacc[qb][rb + 6], sacc[qb][rb + 7])});
#pragma unroll
                    for (int db = 0; db < 2; ++db) o[qb][db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[db], pf, o[qb][db], 0, 0, 0);
                    lacc[qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel, pf, lacc[qb], 0, 0, 0);
                }
            }
        };
        // a full tile with both key blocks' scores computed before any exponential (PIPE2)
        auto tile2 = [&](const char* kimg) {
            const char* vimg = kimg + KB * 128;
            f32x16 sa[2][NQ];
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {
                const char* krow = kimg + (32 * kb + l32) * 128;
                u32x4 kf[4];
#pragma unroll
                for (int ks = 0; ks < 4; ++ks) kf[ks] = *(const u32x4*)(krow + ((((2 * ks + hf) * 16) ^ kpos)));
#pragma unroll
                for (int qb = 0; qb < NQ; ++qb) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) sa[kb][qb][r] = 0.f;
#pragma unroll
                    for (int ks = 0; ks < 4; ++ks)
                        sa[kb][qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kf[ks]),
                                                                             __builtin_bit_cast(bf16x8, qf[qb][ks]), sa[kb][qb], 0, 0, 0);
                }
            }
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {
                uint2 vt[2][2][2];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int row = 32 * kb + 16 * j + 4 * hf + qr;
#pragma unroll
                    for (int db = 0; db < 2; ++db) {
                        const char* b1 = vimg + row * 128 + (((4 * db + 2 * dsub + (pc >> 1)) ^ attn_vswz(row)) * 16) + (pc & 1) * 8;
                        vt[j][db][0] = attn_tr16<0>(b1);
                        vt[j][db][1] = attn_tr16<8 * 128>(b1);
                    }
                }
#pragma unroll
                for (int r = 0; r < 16; ++r) sa[kb][0][r] = (MMT_ATTN_ABLATE == 3 || MMT_ATTN_ABLATE == 6) ? sa[kb][0][r] : __builtin_amdgcn_exp2f(sa[kb][0][r]);
                attn_lds_wait();
                if constexpr (NQ == 2) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) sa[kb][1][r] = (MMT_ATTN_ABLATE == 3 || MMT_ATTN_ABLATE == 6) ? sa[kb][1][r] : __builtin_amdgcn_exp2f(sa[kb][1][r]);
                }
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int rb = 8 * j;
                    bf16x8 vf[2];
#pragma unroll
                    for (int db = 0; db < 2; ++db) {
                        const uint2 ua = vt[j][db][0], ub = vt[j][db][1];
                        vf[db] = __builtin_bit_cast(bf16x8, make_uint4(ua.x, ua.y, ub.x, ub.y));
                    }
#pragma unroll
                    for (int qb = 0; qb < NQ; ++qb) {
                        const f32x16& sv = sa[kb][qb];
                        const bf16x8 pf = __builtin_bit_cast(
                            bf16x8, u32x4{pack_bf16x2(sv[rb], sv[rb + 1]), pack_bf16x2(sv[rb + 2], sv[rb + 3]),
                                          pack_bf16x2(sv[rb + 4], sv[rb + 5]), pack_bf16x2(sv[rb + 6], sv[rb + 7])});
#pragma unroll
                        for (int db = 0; db < 2; ++db) o[qb][db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[db], pf, o[qb][db], 0, 0, 0);
                        lacc[qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel, pf, lacc[qb], 0, 0, 0);
                    }
                }
            }
        };
        for (int kt = 0; kt < nfull; ++kt) {
            const char* kimg = lds + (kt % FNS) * FTILE;
            if constexpr (PIPE2) {
                tile2(kimg);
            } else {
                block(kimg, 0, KB, attn_ic<2>{}, attn_ic<0>{});
                block(kimg, 1, KB, attn_ic<2>{}, attn_ic<0>{});
            }
            if (kt + 1 < nkt) next_tile(kt + 1);
        }
        if (nfull < nkt) {
            const char* kimg = lds + (nfull % FNS) * FTILE;
            const int nv = Lk - nfull * KB;
            if (nv > 16) block(kimg, 0, nv, attn_ic<2>{}, attn_ic<1>{});
            else block(kimg, 0, nv, attn_ic<1>{}, attn_ic<1>{});
            if (nv > 48) block(kimg, 1, nv, attn_ic<2>{}, attn_ic<1>{});
            else if (nv > 32) block(kimg, 1, nv, attn_ic<1>{}, attn_ic<1>{});
        }
        // per query block: range check, normalise and store, or the exact fallback
#pragma unroll
        for (int qb = 0; qb < NQ; ++qb) {
            const float l = lacc[qb][0];
            float chk = 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) chk += o[qb][0][r] * 0.f + o[qb][1][r] * 0.f;
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
                                make_uint2(pack_bf16x2(o[qb][db][4 * g] * inv, o[qb][db][4 * g + 1] * inv),
                                           pack_bf16x2(o[qb][db][4 * g + 2] * inv, o[qb][db][4 * g + 3] * inv));
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
    if (MMT_ATTN_ABLATE == 2) {  // measurement build: the DMA / barrier skeleton alone
        for (int kt = 0; kt < nfull; ++kt)
            if (kt + 1 < nkt) next_tile(kt + 1);
    } else if (nqa == 2) {
        run(attn_ic<2>{});
    } else if (nqa == 1) {
        run(attn_ic<1>{});
    } else {  // no queries: keep the DMA and barrier schedule of the workgroup
        for (int kt = 0; kt < nfull; ++kt)
            if (kt + 1 < nkt) next_tile(kt + 1);
    }
}

template <int FNS>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2, 2))) void mam_attention_lz2_kernel(
    const mmt_attn_params p) {
    __shared__ __attribute__((aligned(1024))) char lds[FNS * FTILE];
    int bx, h, s;
    attn_block_ids_xcd(bx, h, s);
    mam_lz2_item<FNS>(p, lds, bx, h, s);
}

#ifndef MMT_ATTN_AB
#define MMT_ATTN_AB 0  // A/B build only (tools/build_ablate.sh ab): impl 23
#endif
#if MMT_ATTN_AB
// ---- impl 23: block-pipelined range-checked kernel with a hand-placed issue order ---------------------
// The same math per 32-key block as impl 17 / 22 (P = exp2(S) with no reference point, row sums on the
// matrix pipe, epilogue range check with the exact fallback), re-timed so that one wave carries two
// independent instruction streams at every point of its loop:
//   slot b, phase 1:  QK^T MFMAs of block b+1 (8)       beside the 32 v_exp_f32 of block b's scores
//                     and the V^T fragment reads of block b
//   slot b, phase 2:  PV + row-sum MFMAs of block b (12)  beside the 16 v_cvt_pk of block b and the K
//                     fragment reads of block b+2
// i.e. a two-stage software pipeline over 32-key blocks (scores of one block in flight while the
// previous block is exponentiated and multiplied into O), with sched_group_barrier placing about two
// exponentials / one pack per MFMA gap (the guide's "<= 24 cycles of issue per 32x32x16 gap").  64
// queries per wave (two 32-query blocks share every K / V fragment), NW waves per workgroup sharing one
// K / V stream (NW = 4: 256 queries, half the L2 -> LDS fill of 128-query workgroups), 2 waves per SIMD.
// K / V tiles: a 4-slot LDS-DMA ring, one barrier per 64-key tile placed inside the slot that first
// reads the tile; tile t + 2 is issued there into the slot of tile t - 2, which every wave has finished
// reading (the fragment reads run one block ahead of the math).  Loop: global memory sees only the
// LDS-DMA pieces, so the counted vmcnt waits never include a store (stores start in the epilogue).
template <int NW, int WPE = 2>  // waves per workgroup, waves per SIMD (1: the whole 512-register file)
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void mam_attention_hs_kernel(
    const mmt_attn_params p) {
    constexpr int R = 4;          // K / V tile slots
    constexpr int QWG = 64 * NW;  // queries per workgroup
    constexpr int NP = 16 / NW;   // 1-KiB DMA pieces per wave per tile (8 K + 8 V pieces)
    static_assert(QWG * 128 <= 2 * FTILE, "the Q image fits the last two ring slots");
    __shared__ __attribute__((aligned(1024))) char lds[R * FTILE];

    const int n_t = p.n_t, ntok = p.ntok, C = p.C;
    const int64_t pitch = p.tok_pitch > 0 ? p.tok_pitch : ntok;
    const int nqb_t = (n_t + QWG - 1) / QWG;
    int bx, h, s;
    attn_block_ids_xcd(bx, h, s);
    const int qbk = bx + (p.q_part == 2 ? nqb_t : 0);
    const bool tmpl = qbk < nqb_t;
    const int q0 = tmpl ? qbk * QWG : n_t + (qbk - nqb_t) * QWG;
    const int qend = tmpl ? n_t : ntok;
    const int Lk = tmpl ? n_t : (p.asym ? ntok + n_t : ntok);
    const bool cross = p.asym && !tmpl;
    const int64_t rs = 3 * (int64_t)C;
    const bf16_t* qkv = (const bf16_t*)p.qkv;
    const int sV = s % p.Bm, sI = sV + p.Bm;

    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int l32 = lane & 31, hf = lane >> 5;
    const int prow = lane >> 3, pcol = lane & 7;

    auto key_row = [&](int kk) -> const bf16_t* {
        int seq = s, row = kk;
        if (cross) {
            if (kk < n_t) seq = sV;
            else if (kk < 2 * n_t) { seq = sI; row = kk - n_t; }
            else row = kk - n_t;
        }
        return qkv + ((int64_t)seq * pitch + row) * rs;
    };
    const bool aligned = n_t % KB == 0;
    const int nkt = (Lk + KB - 1) / KB;
    // wave w DMAs pieces w*NP .. w*NP+NP-1 of a tile: pieces 0-7 = K rows 8i..8i+7, 8-15 = V rows
    const int isv = (w * NP) >> 3;  // wave-uniform: a wave's pieces are all K or all V
    const int64_t col = (isv ? 2 * C : C) + h * D + (isv ? (pcol ^ attn_vswz(prow)) : (pcol ^ prow)) * 8;
    auto issue_tile = [&](int t) {
        MMT_ATTN_ASSERT(t >= 0 && t < nkt);
        char* slot = lds + (t % R) * FTILE + isv * KB * 128;
        if (aligned && t * KB + KB <= Lk) {
            const bf16_t* base = key_row(t * KB);  // wave-uniform
#pragma unroll
            for (int i = 0; i < NP; ++i) {
                const int r8 = (w * NP + i) & 7;
                attn_glds16(base + (int64_t)(r8 * 8 + prow) * rs + col, slot + r8 * 1024);
            }
        } else {
#pragma unroll
            for (int i = 0; i < NP; ++i) {
                const int r8 = (w * NP + i) & 7;
                attn_glds16(key_row(min(t * KB + r8 * 8 + prow, Lk - 1)) + col, slot + r8 * 1024);
            }
        }
    };
    // Q image (QWG rows x 128 B, rows past the block's end re-read the last query) in the last two
    // slots, read into registers before those slots take tiles 2 and 3
    char* qimg = lds + (R - 2) * FTILE;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int r = 64 * w + 8 * i + prow;
        const bf16_t* src = qkv + ((int64_t)s * pitch + min(q0 + r, qend - 1)) * rs + h * D;
        attn_glds16(src + ((pcol ^ prow) * 8), qimg + (8 * w + i) * 1024);
    }
    for (int t = 0; t < 2 && t < nkt; ++t) issue_tile(t);

    const int qbase = q0 + 64 * w;  // query blocks qbase + 32 qb + [0, 32)
    const bool active = qbase < qend;
    const float cexp = p.scale * 1.4426950408889634f;
    const bool prescale = fabsf(cexp - 1.f) > 1e-6f;
    const float one_or_zero = (((lane & 15) >> 2) & 1) == ((lane >> 4) & 1) ? 1.f : 0.f;
    const uint32_t sel_w = pack_bf16x2(one_or_zero, one_or_zero);
    const bf16x8 sel = __builtin_bit_cast(bf16x8, u32x4{sel_w, sel_w, sel_w, sel_w});
    const int kpos = (l32 & 7) * 16;
    const int li = lane & 15, qr = li >> 2, pc = li & 3, dsub = (lane >> 4) & 1;

    u32x4 qf[2][4];
    attn_wait_vm<0>();
    lds_barrier();
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
        const int row = 64 * w + 32 * qb + l32;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            qf[qb][ks] = *(const u32x4*)(qimg + row * 128 + (((2 * ks + hf) ^ (row & 7)) * 16));
            if (prescale) {
                u32x4 v = qf[qb][ks];
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    v[e] = pack_bf16x2(__uint_as_float(v[e] << 16) * cexp, __uint_as_float(v[e] & 0xffff0000u) * cexp);
                qf[qb][ks] = v;
            }
        }
    }
    lds_barrier();
    for (int t = 2; t < R && t < nkt; ++t) issue_tile(t);

    const int nb = (Lk + 31) / 32;       // 32-key blocks; the last holds Lk - 32 (nb - 1) keys
    const int nvl = Lk - 32 * (nb - 1);  // valid keys of the last block
    // LDS fragment reads (inline asm: invisible to hipcc's wait-count tracking, so that it does not
    // drain the LDS-DMA ring before them; the waits below are explicit)
    auto kread = [&](int b, u32x4 (&kf)[4]) {
        const char* krow = lds + ((b >> 1) % R) * FTILE + (32 * (b & 1) + l32) * 128;
        const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)krow;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const uint32_t ak = a + ((((2 * ks + hf) * 16) ^ kpos));
            asm volatile("ds_read_b128 %0, %1" : "=v"(kf[ks]) : "v"(ak));
        }
    };
    auto vread = [&](int b, uint2 (&vt)[2][2][2]) {
        const char* vimg = lds + ((b >> 1) % R) * FTILE + KB * 128;
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
    // tile sync point X_t, in step (2t - 1, 0) before the first reads of tile t (K of block 2t): its
    // pieces landed (own: counted vmcnt; every wave's: the barrier), and every wave is past step
    // (2t - 2, 1), i.e. past the last reads of tile t - 2 (V^T of block 2t - 3, step (2t - 3, 0)), whose
    // slot then takes tile t + 2
    auto sync_tile = [&](int t) {
        if (t < 2 || t >= nkt) return;  // tiles 0 / 1 landed in the prologue
        attn_wait_dyn(t + 1 < nkt ? NP : 0);
        lds_barrier();
        if (t + 2 < nkt) issue_tile(t + 2);
    };

    f32x16 o[2][2];
    f32x4 lacc[2];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
#pragma unroll
        for (int r = 0; r < 16; ++r) { o[qb][0][r] = 0.f; o[qb][1][r] = 0.f; }
        lacc[qb] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // Pipeline unit u = (32-key block b, query block qb), in the order (0,0), (0,1), (1,0), ...; step u
    // issues the MFMAs of PV(u - 1) (4 + 2 row-sum) and QK^T(u + 1) (4) beside the 16 exponentials
    // and 8 packs of unit u: 288 matrix-pipe cycles against ~240 issue cycles, with two score and two
    // P buffers live (S(u), S(u + 1); P(u - 1), P(u)).  K fragments change every second step (read
    // after the QK^T MFMAs of step (b, 0) that last use K(b)), V^T fragments likewise (read after
    // the PV MFMAs of step (b, 0) that last use V(b - 1)).
    f32x16 sc[2];    // raw scores / exponentials of the two query blocks
    u32x4 pf[2][2];  // packed P of the two query blocks, [qb][16-key half]
    u32x4 kf[4];
    uint2 vt[2][2][2];
    auto qk = [&](int qb) {  // scores of query block qb against the block whose K fragments are in kf
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
            sc[qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kf[ks]),
                                                             __builtin_bit_cast(bf16x8, qf[qb][ks]),
                                                             ks ? sc[qb] : f32x16{}, 0, 0, 0);
    };
    auto pv = [&](int qb) {  // O += V^T P^T and the row sums, query block qb, block in vt / pf[qb]
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const bf16x8 pb = __builtin_bit_cast(bf16x8, pf[qb][j]);
#pragma unroll
            for (int db = 0; db < 2; ++db) {
                const uint2 ua = vt[j][db][0], ub = vt[j][db][1];
                o[qb][db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                    __builtin_bit_cast(bf16x8, make_uint4(ua.x, ua.y, ub.x, ub.y)), pb, o[qb][db], 0, 0, 0);
            }
            lacc[qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel, pb, lacc[qb], 0, 0, 0);
        }
        if constexpr (WPE == 1) {  // O and the row sums live in the accumulator registers
            asm volatile("" : "+a"(o[qb][0]), "+a"(o[qb][1]), "+a"(lacc[qb]));
        }
    };
    // P = exp2(S) (keys past Lk: 0) of accumulator elements [r0, r1) of query block qb, packed to bf16
    // (r0, r1 multiples of 2: whole packed pairs)
    auto softmax = [&](int qb, bool mask, int r0, int r1) {
        for (int r = r0; r < r1; ++r) {
            const float e = __builtin_amdgcn_exp2f(sc[qb][r]);
            sc[qb][r] = !mask || 8 * (r >> 2) + 4 * hf + (r & 3) < nvl ? e : 0.f;
        }
        for (int r = r0; r < r1; r += 2) pf[qb][r >> 3][(r & 7) >> 1] = pack_bf16x2(sc[qb][r], sc[qb][r + 1]);
    };
    // the issue pattern of one step: MFMAs each followed by 2 exponentials and 1 pack / select, the
    // last ones bare (the ~24 issue cycles per 32x32x16 gap of MI355X_MICROARCH.md)
    auto interleave = [&](int nmfma) {
        for (int i = 0; i < nmfma; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
            if (i < 8) {
                __builtin_amdgcn_sched_group_barrier(0x400, 2, 0);  // 2 transcendental (v_exp)
                __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);  // 1 VALU (pack / select)
            }
        }
    };
    // an empty asm that takes query block qb's packed P: its exponentials and packs are computed inside
    // the step's scheduling region (hipcc otherwise sinks them into the next basic block, out of reach
    // of the region's sched_group_barrier pattern)
    auto pin = [&](int qb) { asm volatile("" : "+v"(pf[qb][0]), "+v"(pf[qb][1])); };
    // step (b, 0): PV(b - 1, 1), QK^T(b, 1), softmax(b, 0); reads V(b)
    auto step0 = [&](int b, auto FIRSTc, auto MASKc) {
        constexpr bool FIRST = decltype(FIRSTc)::value, MASK = decltype(MASKc)::value;
        attn_lds_wait();  // V(b - 1) fragments (the sched barrier keeps their consumers below)
        if constexpr (!FIRST) pv(1);
        vread(b, vt);  // the previous V^T fragments are consumed by the MFMAs above
        qk(1);
        softmax(0, MASK, 0, 16);
        interleave(FIRST ? 4 : 10);
        pin(0);
        __builtin_amdgcn_sched_barrier(0);
    };
    // step (b, 1): PV(b, 0), QK^T(b + 1, 0), softmax(b, 1); reads K(b + 1) at its start (after the
    // sync point of a new tile), waited for just before the QK^T MFMAs that need them (the six PV /
    // row-sum MFMAs cover the read latency)
    auto step1 = [&](int b, auto LASTc, auto MASKc) {
        constexpr bool LAST = decltype(LASTc)::value, MASK = decltype(MASKc)::value;
        if constexpr (!LAST) {
            if (b & 1) sync_tile((b + 1) / 2);  // first reads of tile (b + 1) / 2
            kread(b + 1, kf);
        }
        // V(b) (read in step (b, 0)): every LDS read but the four K reads just issued (LDS reads
        // return in order)
        if constexpr (!LAST) asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        pv(0);
        softmax(1, MASK, 0, 12);
        interleave(6);
        pin(1);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!LAST) attn_lds_wait();  // K(b + 1)
        if constexpr (!LAST) qk(0);
        softmax(1, MASK, 12, 16);
        if constexpr (!LAST) interleave(4);
        pin(1);
        __builtin_amdgcn_sched_barrier(0);
    };
    using I0 = attn_ic<0>;
    using I1 = attn_ic<1>;

    if (active) {
        kread(0, kf);
        attn_lds_wait();
        qk(0);
        const bool mask = nvl < 32;  // the last block holds keys past Lk
        if (nb == 1) {
            step0(0, I1{}, I1{});
            step1(0, I1{}, I1{});
        } else {
            step0(0, I1{}, I0{});
            step1(0, I0{}, I0{});
            for (int b = 1; b < nb - 1; ++b) {
                step0(b, I0{}, I0{});
                step1(b, I0{}, I0{});
            }
            if (mask) {
                step0(nb - 1, I0{}, I1{});
                step1(nb - 1, I1{}, I1{});
            } else {
                step0(nb - 1, I0{}, I0{});
                step1(nb - 1, I1{}, I0{});
            }
        }
        pv(1);  // the last unit's PV
    } else {  // no queries: keep the DMA and barrier schedule of the workgroup
        for (int b = 1; b < nb; b += 2) sync_tile((b + 1) / 2);
        return;
    }

    // per query block: range check, normalise and store, or the exact fallback (as impl 22)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
        const float l = lacc[qb][0];
        float chk = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) chk += o[qb][0][r] * 0.f + o[qb][1][r] * 0.f;
        const bool ok = l >= LZ_LO && l <= LZ_HI && chk == 0.f;
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
                            make_uint2(pack_bf16x2(o[qb][db][4 * g] * inv, o[qb][db][4 * g + 1] * inv),
                                       pack_bf16x2(o[qb][db][4 * g + 2] * inv, o[qb][db][4 * g + 3] * inv));
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
}
#endif  // MMT_ATTN_AB

}  // namespace

int mmt_attn_launch_ps(const mmt_attn_params& p, hipStream_t st);  // attention_ps.hip: impl 29 (persistent)
#if MMT_ATTN_AB
int mmt_attn_launch_pp(const mmt_attn_params& p, int ks, hipStream_t st);  // attention_pp.hip: impl 24 / 25
int mmt_attn_launch_pg(const mmt_attn_params& p, hipStream_t st);          // attention_pg.hip: impl 28
#endif

namespace {

template <typename T>
int launch_attn(const mmt_attn_params& p, hipStream_t st) {
    // impl: 0 = the library's choice by dtype and grid size; forced (A/B and tests): 4 = latency kernel,
    // 8 = running-maximum throughput kernel, 17 / 21 / 22 = range-checked exponent kernels (22 = 64
    // queries per wave); A/B build: 23 = the block-pipelined form of 22 with 256-query workgroups
    if (p.impl != 0 && p.impl != 4 && p.impl != 8 && p.impl != 17 && p.impl != 21 && p.impl != 22 && p.impl != 29 &&
        !(MMT_ATTN_AB && (p.impl == 23 || p.impl == 24 || p.impl == 25 || p.impl == 26 || p.impl == 27 || p.impl == 28)))
        return MMT_EBADARG;
    // lse (training forward) is written by impls 0 / 4 / 8 / 17 / 21 only: impls 22 / 23 never write it
    if (p.lse && (sizeof(T) != 2 || p.impl >= 22)) return MMT_EBADARG;
    // fp16: the kernels with a running maximum (latency kernel, throughput kernel); the range-checked
    // exponent kernels are bf16, and the training forward (lse) is bf16
    if (__is_same(T, f16_t) && (p.lse || p.impl >= 17)) return MMT_EBADARG;
    if (!p.qkv || !p.out || p.H <= 0 || p.C != p.H * D || p.S <= 0 || p.ntok <= p.n_t || p.n_t <= 0) return MMT_EBADARG;
    if (p.tok_pitch != 0 && (p.tok_pitch < p.ntok || p.lse)) return MMT_EBADARG;
    if (p.asym && (p.Bm <= 0 || p.S != 2 * p.Bm)) return MMT_EBADARG;
    if (((uintptr_t)p.qkv | (uintptr_t)p.out) & 15) return MMT_EBADARG;
    if (p.q_part < 0 || p.q_part > 2) return MMT_EBADARG;
    {  // compact out rows: every stored query lands in [0, out_pitch) of its sequence
        const int qa = p.q_part == 2 ? p.n_t : 0, qb = p.q_part == 1 ? p.n_t : p.ntok;
        if (p.out_pitch < 0 || p.out_q0 < 0 || p.out_q0 > qa || ((p.out_pitch || p.out_q0) && p.lse) ||
            (p.out_pitch > 0 && p.out_pitch < qb - p.out_q0))
            return MMT_EBADARG;
    }
    // q_part: 0 all queries, 1 template queries only, 2 search queries only (template K/V cache)
    auto qblocks = [&](int qt) {
        const int t = (p.n_t + qt - 1) / qt, sr = (p.ntok - p.n_t + qt - 1) / qt;
        return p.q_part == 1 ? t : p.q_part == 2 ? sr : t + sr;
    };
    const int nqb = qblocks(64);
    dim3 grid(nqb, p.H, p.S);
    if constexpr (sizeof(T) == 2) {
        const int nfa = qblocks(FQ);
        const dim3 fgrid(nfa, p.H, p.S);
        const bool bf = __is_same(T, bf16_t);
        int impl = p.impl;
        if (impl == 0) {
            // large grids, bf16 inference: the range-checked exponent kernel, 64 queries per wave from
            // MMT_ATTN_LZ2_MIN_WG workgroups (impl 22), else with its two blocks per tile software-
            // pipelined (impl 21; B = 8 / 32: 27.2 / 78.9 us against 29.8 / 83.8 for impl 17 and 30-34 /
            // 84-93 for impl 8, profiles/r02_attn_ab.jsonl, r02_pipe_ab.jsonl); the training forward
            // (lse) takes impl 21 too (round 6: 46.9 vs 56.2 us for impl 8 at the training shape, 32 sequences,
            // tools/attn_fwd_lse_ab.py, profiles/r06_attn_fwd_lse_ab.txt; impl 22 writes no lse); fp16 keeps the
            // running-maximum throughput kernel; small grids (batch-1 tracking): the latency kernel (64 queries x 4
            // key groups)
            const int64_t wg = (int64_t)nfa * p.H * p.S;
            if (bf && !p.lse && wg >= MMT_ATTN_LZ2_MIN_WG) impl = 22;
            else if (bf && wg >= MMT_ATTN_FA_MIN_WG) impl = 21;
            else if (p.lse || wg >= MMT_ATTN_FA_MIN_WG) impl = 8;
            else impl = 4;
        }
        if (impl == 17) hipLaunchKernelGGL((mam_attention_lz_kernel<3, 3, true>), fgrid, dim3(256), 0, st, p);
        else if (impl == 21) hipLaunchKernelGGL((mam_attention_lz_kernel<3, 3, true, true>), fgrid, dim3(256), 0, st, p);
        else if (impl == 22) hipLaunchKernelGGL((mam_attention_lz2_kernel<2>), fgrid, dim3(128), 0, st, p);
        else if (impl == 29) {  // persistent kernel: bf16 only, its own shape check
            if (!bf) return MMT_EBADARG;
            const int rc = mmt_attn_launch_ps(p, st);
            if (rc) return rc;
        }
#if MMT_ATTN_AB
        else if (impl == 24 || impl == 25) mmt_attn_launch_pp(p, impl == 25 ? 2 : 1, st);
        else if (impl == 28) mmt_attn_launch_pg(p, st);
        else if (impl == 23) {  // block-pipelined kernel, 4 waves (256 queries) per workgroup
            const int nt = (p.n_t + 255) / 256, ns = (p.ntok - p.n_t + 255) / 256;
            const dim3 hgrid(p.q_part == 1 ? nt : p.q_part == 2 ? ns : nt + ns, p.H, p.S);
            hipLaunchKernelGGL((mam_attention_hs_kernel<4>), hgrid, dim3(256), 0, st, p);
        } else if (impl == 26) {  // the same at one wave per SIMD (one 256-query workgroup per CU)
            const int nt = (p.n_t + 255) / 256, ns = (p.ntok - p.n_t + 255) / 256;
            const dim3 hgrid(p.q_part == 1 ? nt : p.q_part == 2 ? ns : nt + ns, p.H, p.S);
            hipLaunchKernelGGL((mam_attention_hs_kernel<4, 1>), hgrid, dim3(256), 0, st, p);
        } else if (impl == 27) {  // 2-wave (128-query) workgroups at one wave per SIMD (two per CU)
            hipLaunchKernelGGL((mam_attention_hs_kernel<2, 1>), fgrid, dim3(128), 0, st, p);
        }
#endif
        else if (impl == 8 || p.lse) hipLaunchKernelGGL((mam_attention_fa_kernel<T, 2, 3>), fgrid, dim3(256), 0, st, p);
        else hipLaunchKernelGGL((mam_attention_glds_kernel<T, 4>), grid, dim3(1024), 0, st, p);
    } else {  // fp32 (parity path); small grids: 4 waves x 16 queries to occupy more SIMDs
        if ((int64_t)nqb * p.H * p.S < 1024) hipLaunchKernelGGL((mam_attention_kernel<T, 1>), grid, dim3(256), 0, st, p);
        else hipLaunchKernelGGL((mam_attention_kernel<T, 2>), grid, dim3(128), 0, st, p);
    }
    return launch_status();
}

}  // namespace

extern "C" int mmt_mam_attention(const mmt_attn_params* p, int dtype, void* stream) {
    if (!p) return MMT_EBADARG;
    if (dtype == MMT_BF16) return launch_attn<bf16_t>(*p, (hipStream_t)stream);
    if (dtype == MMT_F16) return launch_attn<f16_t>(*p, (hipStream_t)stream);
    if (dtype == MMT_F32) return launch_attn<float>(*p, (hipStream_t)stream);
    return MMT_EBADARG;
}
