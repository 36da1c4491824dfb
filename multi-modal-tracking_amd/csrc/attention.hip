// Mixed Attention Module (MAM) — asymmetric template/search softmax attention for gfx950.
//
// Reference: Attention.forward, lib/models/mixformer_vit_rgbt/mixformer.py:52-78 (template
// queries -> template keys; search queries -> all keys) and the cross-modal variant
// asymmetric_shared.py:55-104 (search_m -> [template_V | template_I | search_m]).
// The qkv Linear output is consumed in place ([seq][token][3][head][64], no permute) and the
// result is written as [seq][token][head*64], i.e. exactly the proj GEMM's A operand.
//
// One workgroup = 64 queries of one (sequence, head): 2 waves x 32 queries (two 16-query MFMA
// tiles sharing every K/V fragment read) for large grids, or 4 waves x 16 queries when the grid
// is small (batch-1 tracking) so that more SIMDs get a wave.  Keys stream through a double-buffered
// LDS ring in 64-key tiles (register-staged: the next tile's global loads are in flight during
// the current tile's matrix work).  Scores are computed transposed (S^T = K Q^T) so that each
// lane owns one query column: the online-softmax max/sum/rescale need only two cross-lane
// shuffles, and the exponentiated scores are already laid out as the B operand of O^T = V^T P^T
// (no LDS round trip for P).  V^T fragments come from ds_read_b64_tr_b16 on a 160-byte-row V
// image (bank-conflict-free).  bf16: v_mfma_f32_16x16x32_bf16; fp32: v_mfma_f32_16x16x4_f32.
// Softmax statistics are fp32 (exp2 with the scale folded in).
#include "common.hpp"

namespace {

constexpr int D = 64, KB = 64;

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

    const int qb = blockIdx.x, h = blockIdx.y, s = blockIdx.z;
    const int n_t = p.n_t, ntok = p.ntok, C = p.C;
    const int nqb_t = (n_t + 63) / 64;
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
        const T* qp = qkv + ((int64_t)s * ntok + min(q, qend - 1)) * rs + h * D;  // clamped, never stored
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
        return qkv + ((int64_t)seq * ntok + row) * rs + h * D;
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
        T* op = out + ((int64_t)s * ntok + q) * C + h * D;
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
template <int N>
MMT_DEV void attn_wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
typedef __attribute__((address_space(3))) void attn_lds_void;
typedef __attribute__((address_space(1))) void attn_glb_void;
MMT_DEV void attn_glds16(const void* src, char* dst) {
    __builtin_amdgcn_global_load_lds((attn_glb_void*)src, (attn_lds_void*)dst, 16, 0, 0);
}
// ds_read_b64_tr_b16 as inline asm: through the builtin, hipcc cannot tell the read from the
// in-flight LDS-DMA writes and drains vmcnt(0) before it (i.e. waits for the whole prefetch ring).
// Inline asm is invisible to its wait-count tracking, so the caller waits with attn_lds_wait().
template <int OFF>
MMT_DEV uint2 attn_tr16(const char* p) {
    uint2 r;
    const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "n"(OFF));
    return r;
}
MMT_DEV void attn_lds_wait() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);  // keep the MFMAs that consume the asm reads below the wait
}

constexpr int ANS = 8;              // K/V tile slots in the ring
constexpr int ATILE = 2 * KB * 128; // bytes of one slot: K image then V image

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void mam_attention_glds_kernel(
    const mmt_attn_params p) {
    __shared__ __attribute__((aligned(1024))) char lds[ANS * ATILE + 64 * 128];
    char* qimg = lds + ANS * ATILE;

    const int qb = blockIdx.x, h = blockIdx.y, s = blockIdx.z;
    const int n_t = p.n_t, ntok = p.ntok, C = p.C;
    const int nqb_t = (n_t + 63) / 64;
    const bool tmpl = qb < nqb_t;
    const int q0 = tmpl ? qb * 64 : n_t + (qb - nqb_t) * 64;
    const int qend = tmpl ? n_t : ntok;
    const int Lk = tmpl ? n_t : (p.asym ? ntok + n_t : ntok);
    const bool cross = p.asym && !tmpl;
    const int64_t rs = 3 * (int64_t)C;
    const bf16_t* qkv = (const bf16_t*)p.qkv;
    const int sV = s % p.Bm, sI = sV + p.Bm;

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int l16 = lane & 15, lg = lane >> 4;
    const int prow = lane >> 3, pcol = lane & 7;  // this lane's row / position in a 1-KiB piece

    auto key_row = [&](int kk) -> const bf16_t* {
        int seq = s, row = kk;
        if (cross) {
            if (kk < n_t) seq = sV;
            else if (kk < 2 * n_t) { seq = sI; row = kk - n_t; }
            else row = kk - n_t;
        }
        return qkv + ((int64_t)seq * ntok + row) * rs + h * D;
    };
    // Tile kt into slot kt % ANS: wave w stages K pieces 2w, 2w+1 and V pieces 2w, 2w+1.
    const int nkt = (Lk + KB - 1) / KB;
    auto issue = [&](int kt) {
        char* slot = lds + (kt % ANS) * ATILE;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int piece = 2 * w + i, r = piece * 8 + prow;  // r & 7 == prow
            const bf16_t* src = key_row(min(kt * KB + r, Lk - 1));
            attn_glds16(src + C + ((pcol ^ prow) * 8), slot + piece * 1024);
            attn_glds16(src + 2 * C + ((pcol ^ (prow & 6)) * 8), slot + KB * 128 + piece * 1024);
        }
    };
    // Q image: wave w stages pieces 2w, 2w+1 (rows past the block's end re-read the last query)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int piece = 2 * w + i, r = piece * 8 + prow;
        const bf16_t* src = qkv + ((int64_t)s * ntok + min(q0 + r, qend - 1)) * rs + h * D;
        attn_glds16(src + ((pcol ^ prow) * 8), qimg + piece * 1024);
    }
    for (int kt = 0; kt < ANS - 1 && kt < nkt; ++kt) issue(kt);

    const float cexp = p.scale * 1.4426950408889634f;
    float m_run = -1e30f, l_run = 0.f;
    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    u32x4 qf[2];

    for (int kt = 0; kt < nkt; ++kt) {
        // this wave's DMA of tile kt (and of Q, issued first) has landed once at most `ahead`
        // later tiles (4 instructions each) are outstanding
        const int ahead = min(nkt - 1, kt + ANS - 2) - kt;
        switch (ahead) {
            case 0: attn_wait_vm<0>(); break;
            case 1: attn_wait_vm<4>(); break;
            case 2: attn_wait_vm<8>(); break;
            case 3: attn_wait_vm<12>(); break;
            case 4: attn_wait_vm<16>(); break;
            case 5: attn_wait_vm<20>(); break;
            default: attn_wait_vm<24>(); break;
        }
        lds_barrier();  // every wave's pieces of tile kt landed; every wave is done with tile kt-1
        if (kt + ANS - 1 < nkt) issue(kt + ANS - 1);  // refills the slot tile kt-1 used
        if (kt == 0) {
#pragma unroll
            for (int t = 0; t < 2; ++t)
                qf[t] = *(const u32x4*)(qimg + ((16 * w + l16) * 8 + ((4 * t + lg) ^ (l16 & 7))) * 16);
        }
        const char* kimg = lds + (kt % ANS) * ATILE;
        const char* vimg = kimg + KB * 128;
        // V^T fragments for the PV product, issued first so they land behind the QK^T work:
        // vt[kk][dt] = keys 32kk + 4lg + qr (+16), d = dt*16 + 4pc..+3
        const int qr = l16 >> 2, pc = l16 & 3;
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
        f32x4 sacc[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) sacc[a] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kt16 = 0; kt16 < 4; ++kt16)
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const u32x4 kf = *(const u32x4*)(kimg + ((kt16 * 16 + l16) * 8 + ((4 * t + lg) ^ (l16 & 7))) * 16);
                sacc[kt16] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kf),
                                                                     __builtin_bit_cast(bf16x8, qf[t]), sacc[kt16], 0, 0, 0);
            }
        if (kt * KB + KB > Lk) {  // mask the tail of the key range (clamped rows)
#pragma unroll
            for (int kt16 = 0; kt16 < 4; ++kt16)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (kt * KB + kt16 * 16 + 4 * lg + r >= Lk) sacc[kt16][r] = -1e30f;
        }
        // online softmax (per query column)
        float mx = -1e30f;
#pragma unroll
        for (int kt16 = 0; kt16 < 4; ++kt16)
#pragma unroll
            for (int r = 0; r < 4; ++r) mx = fmaxf(mx, sacc[kt16][r]);
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float mnew = fmaxf(m_run, mx);
        const float alpha = exp2f((m_run - mnew) * cexp);
        m_run = mnew;
        const float mc = mnew * cexp;
        float ls = 0.f;
#pragma unroll
        for (int kt16 = 0; kt16 < 4; ++kt16)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float e = exp2f(sacc[kt16][r] * cexp - mc);
                sacc[kt16][r] = e;
                ls += e;
            }
        l_run = l_run * alpha + ls;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
        // O^T += V^T P^T
        attn_lds_wait();
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            bf16x8 pf;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                pf[j] = (__bf16)sacc[2 * kk][j];
                pf[4 + j] = (__bf16)sacc[2 * kk + 1][j];
            }
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                const uint2 ua = vt[kk][dt][0], ub = vt[kk][dt][1];
                const bf16x8 vf = __builtin_bit_cast(bf16x8, make_uint4(ua.x, ua.y, ub.x, ub.y));
                o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf, o[dt], 0, 0, 0);
            }
        }
    }

    // ---- normalise and store: lane holds O[q = l16][d = dt*16 + 4*lg + r]
    float l = l_run;
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    const float inv = 1.f / l;
    const int q = q0 + 16 * w + l16;
    if (q < qend) {
        bf16_t* op = (bf16_t*)p.out + ((int64_t)s * ntok + q) * C + h * D;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
            *(uint2*)(op + dt * 16 + 4 * lg) =
                make_uint2(pack_bf16x2(o[dt][0] * inv, o[dt][1] * inv), pack_bf16x2(o[dt][2] * inv, o[dt][3] * inv));
    }
}

template <typename T>
int launch_attn(const mmt_attn_params& p, hipStream_t st) {
    if (!p.qkv || !p.out || p.H <= 0 || p.C != p.H * D || p.S <= 0 || p.ntok <= p.n_t || p.n_t <= 0) return MMT_EBADARG;
    if (p.asym && (p.Bm <= 0 || p.S != 2 * p.Bm)) return MMT_EBADARG;
    if (((uintptr_t)p.qkv | (uintptr_t)p.out) & 15) return MMT_EBADARG;
    const int nqb = (p.n_t + 63) / 64 + (p.ntok - p.n_t + 63) / 64;
    dim3 grid(nqb, p.H, p.S);
    if constexpr (sizeof(T) == 2) {  // bf16: LDS-DMA kernel, 4 waves x 16 queries per workgroup
        hipLaunchKernelGGL(mam_attention_glds_kernel, grid, dim3(256), 0, st, p);
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
    if (dtype == MMT_F32) return launch_attn<float>(*p, (hipStream_t)stream);
    return MMT_EBADARG;
}
