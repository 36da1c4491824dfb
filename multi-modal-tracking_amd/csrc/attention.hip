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

template <typename T>
int launch_attn(const mmt_attn_params& p, hipStream_t st) {
    if (!p.qkv || !p.out || p.H <= 0 || p.C != p.H * D || p.S <= 0 || p.ntok <= p.n_t || p.n_t <= 0) return MMT_EBADARG;
    if (p.asym && (p.Bm <= 0 || p.S != 2 * p.Bm)) return MMT_EBADARG;
    if (((uintptr_t)p.qkv | (uintptr_t)p.out) & 15) return MMT_EBADARG;
    const int nqb = (p.n_t + 63) / 64 + (p.ntok - p.n_t + 63) / 64;
    dim3 grid(nqb, p.H, p.S);
    // small grids (batch-1 tracking): 4 waves x 16 queries per workgroup to occupy more SIMDs
    if ((int64_t)nqb * p.H * p.S < 1024) hipLaunchKernelGGL((mam_attention_kernel<T, 1>), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((mam_attention_kernel<T, 2>), grid, dim3(128), 0, st, p);
    return launch_status();
}

}  // namespace

extern "C" int mmt_mam_attention(const mmt_attn_params* p, int dtype, void* stream) {
    if (!p) return MMT_EBADARG;
    if (dtype == MMT_BF16) return launch_attn<bf16_t>(*p, (hipStream_t)stream);
    if (dtype == MMT_F32) return launch_attn<float>(*p, (hipStream_t)stream);
    return MMT_EBADARG;
}
