// MAM attention backward for gfx950 (training step).
//
// Reference: the autograd of Attention.forward, lib/models/mixformer_vit_rgbt/mixformer.py:52-78
// (template queries -> template keys; search queries -> all keys of their sequence), as
// train_script_mixformer*.py trains it.  Inputs are the forward's qkv buffer ([seq][token][3][head]
// [64], bf16), its output O, the output gradient dO and the per-query log-sum-exp the throughput
// forward kernel leaves (lse, log2 domain of the pre-scaled scores: P = exp2(q'.k - lse) with
// q' = bf16(q * scale * log2 e), exactly the forward's operand).  The result is dQKV in the qkv
// layout, i.e. directly the dY of the qkv Linear's backward.
//
// Two deterministic kernels (no atomics; every gradient element is summed by one wave in a fixed
// order), recomputing the scores instead of storing them:
//   mam_bwd_dq_kernel   one workgroup = 4 waves x 16 queries of one (sequence, head); per 64-key
//                       tile: S^T = K q'^T, P, dP^T = V dO^T, dS = P (dP - delta),
//                       dQ^T += K^T dS^T; delta = rowsum(dO o O) is computed here and stored.
//   mam_bwd_dkv_kernel  one workgroup = 4 waves x 16 keys; per 64-query tile of the queries that
//                       attend those keys: S = q' K^T, P, dP = dO V^T, dS,
//                       dV^T += dO^T P, dK^T += q'^T dS.
// Operand tiles are staged through LDS with a 160-byte row pitch (conflict-free for both the
// ds_read_b128 row reads and the ds_read_b64_tr_b16 transposed reads each tile gets).
#include "common.hpp"

namespace {

constexpr int D = 64, TP = 160;  // head dim, LDS row pitch (bytes)

// Register budgets (A/B knobs; 0 = the compiler's choice): the dkv kernel at >= 3 waves per SIMD (147 registers, no
// spills) instead of the compiler's 182 (2 waves): 252 -> 215 us for the training shape's backward, the same results
// (tools/attn_bwd_ab.py, profiles/r06_attn_bwd_ab.txt).  4 waves spills.
#ifndef MMT_BWD_DKV_WAVES
#define MMT_BWD_DKV_WAVES 3
#endif
#ifndef MMT_BWD_DQ_WAVES
#define MMT_BWD_DQ_WAVES 0
#endif
#if MMT_BWD_DKV_WAVES > 0
#define MMT_BWD_DKV_ATTR __attribute__((amdgpu_waves_per_eu(MMT_BWD_DKV_WAVES)))
#else
#define MMT_BWD_DKV_ATTR
#endif
#if MMT_BWD_DQ_WAVES > 0
#define MMT_BWD_DQ_ATTR __attribute__((amdgpu_waves_per_eu(MMT_BWD_DQ_WAVES)))
#else
#define MMT_BWD_DQ_ATTR
#endif

MMT_DEV bf16x8 tr_frag(const char* tile, int kk, int dt, int lg, int l16) {
    // A operand [16 rows of d][32 k] read transposed from a row-major [k][d] tile: rows
    // 32kk + 4lg + qr and +16 (the same permuted k order as pack_p below), d = dt*16 + 4pc..+3
    const int qr = l16 >> 2, pc = l16 & 3;
    const char* b1 = tile + (32 * kk + 4 * lg + qr) * TP + (dt * 16 + 4 * pc) * 2;
    const s16x4 va = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)b1);
    const s16x4 vb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(b1 + 16 * TP));
    const uint2 ua = __builtin_bit_cast(uint2, va), ub = __builtin_bit_cast(uint2, vb);
    return __builtin_bit_cast(bf16x8, make_uint4(ua.x, ua.y, ub.x, ub.y));
}

MMT_DEV u32x4 row_frag(const char* tile, int row, int chunk) {
    return *(const u32x4*)(tile + row * TP + chunk * 16);
}

// B operand [32 k][16 cols] from four 16x16 accumulator tiles laid out [k = 16*i + 4lg + r][col]
MMT_DEV bf16x8 pack_p(const f32x4 (&a)[4], int kk) {
    return __builtin_bit_cast(bf16x8, u32x4{pack_bf16x2(a[2 * kk][0], a[2 * kk][1]), pack_bf16x2(a[2 * kk][2], a[2 * kk][3]),
                                            pack_bf16x2(a[2 * kk + 1][0], a[2 * kk + 1][1]),
                                            pack_bf16x2(a[2 * kk + 1][2], a[2 * kk + 1][3])});
}

MMT_DEV u32x4 scale_bf16x8(u32x4 u, float c) {
#pragma unroll
    for (int e = 0; e < 4; ++e) u[e] = pack_bf16x2(__uint_as_float(u[e] << 16) * c, __uint_as_float(u[e] & 0xffff0000u) * c);
    return u;
}

MMT_DEV f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }
MMT_DEV f32x4 mfma(u32x4 a, u32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// 64 rows x 128 B of a [row][rs] bf16 buffer into a TP-pitch LDS tile, in two halves: load_tile fetches
// this thread's two 16-B chunks into registers (rows past `rows` re-read row rows-1), store_tile writes them
// (scaled by c if c != 1: q' = bf16(q * c)).  The K loops fetch tile t+1 into registers before they multiply
// tile t, so its global latency hides behind the MFMAs (round 5: the tile was loaded and stored between the
// two barriers, every wave waiting on it).
MMT_DEV void load_tile(u32x4 (&v)[2], const bf16_t* base, int64_t rs, int r0, int rows) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int idx = threadIdx.x + 256 * i, r = idx >> 3, ch = idx & 7;
        v[i] = *(const u32x4*)(base + (int64_t)min(r0 + r, rows - 1) * rs + ch * 8);
    }
}
MMT_DEV void store_tile(char* tile, const u32x4 (&v)[2], float c) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int idx = threadIdx.x + 256 * i, r = idx >> 3, ch = idx & 7;
        *(u32x4*)(tile + r * TP + ch * 16) = c != 1.f ? scale_bf16x8(v[i], c) : v[i];
    }
}

__global__ __launch_bounds__(256) MMT_BWD_DQ_ATTR void mam_bwd_dq_kernel(const mmt_attn_bwd_params p) {
    __shared__ __attribute__((aligned(16))) char kt_l[64 * TP];
    __shared__ __attribute__((aligned(16))) char vt_l[64 * TP];
    const int qb = blockIdx.x, h = blockIdx.y, s = blockIdx.z;
    const int n_t = p.n_t, ntok = p.ntok, C = p.C, H = p.H;
    const int nqb_t = (n_t + 63) / 64;
    const bool tmpl = qb < nqb_t;
    const int q0 = tmpl ? qb * 64 : n_t + (qb - nqb_t) * 64;
    const int qend = tmpl ? n_t : ntok;
    const int Lk = tmpl ? n_t : ntok;
    const int64_t rs = 3 * (int64_t)C;
    const bf16_t* qkv = (const bf16_t*)p.qkv + (int64_t)s * ntok * rs + h * D;
    const bf16_t* O = (const bf16_t*)p.out + (int64_t)s * ntok * C + h * D;
    const bf16_t* dO = (const bf16_t*)p.dout + (int64_t)s * ntok * C + h * D;
    const float c = p.scale * 1.4426950408889634f;

    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, l16 = lane & 15, lg = lane >> 4;
    const int q = q0 + 16 * w + l16, qc = min(q, qend - 1);
    u32x4 qf[2], dof[2];
    float delta = 0.f;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        qf[u] = scale_bf16x8(*(const u32x4*)(qkv + (int64_t)qc * rs + 32 * u + 8 * lg), c);
        dof[u] = *(const u32x4*)(dO + (int64_t)qc * C + 32 * u + 8 * lg);
        const u32x4 ov = *(const u32x4*)(O + (int64_t)qc * C + 32 * u + 8 * lg);
#pragma unroll
        for (int e = 0; e < 4; ++e)
            delta += __uint_as_float(dof[u][e] << 16) * __uint_as_float(ov[e] << 16) +
                     __uint_as_float(dof[u][e] & 0xffff0000u) * __uint_as_float(ov[e] & 0xffff0000u);
    }
    delta = lanegroup_sum(delta);
    const float lse = p.lse[((int64_t)s * H + h) * ntok + qc];

    f32x4 dq[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dq[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nkt = (Lk + 63) / 64;
    u32x4 kr[2], vr[2];
    load_tile(kr, qkv + C, rs, 0, Lk);
    load_tile(vr, qkv + 2 * C, rs, 0, Lk);
    for (int kt = 0; kt < nkt; ++kt) {
        __syncthreads();  // every wave is past its reads of tile kt-1
        store_tile(kt_l, kr, 1.f);
        store_tile(vt_l, vr, 1.f);
        __syncthreads();
        if (kt + 1 < nkt) {  // tile kt+1 in flight while tile kt is multiplied
            load_tile(kr, qkv + C, rs, (kt + 1) * 64, Lk);
            load_tile(vr, qkv + 2 * C, rs, (kt + 1) * 64, Lk);
        }
        f32x4 sp[4], dp[4];
#pragma unroll
        for (int kt16 = 0; kt16 < 4; ++kt16) {
            sp[kt16] = dp[kt16] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                sp[kt16] = mfma(row_frag(kt_l, kt16 * 16 + l16, 4 * u + lg), qf[u], sp[kt16]);
                dp[kt16] = mfma(row_frag(vt_l, kt16 * 16 + l16, 4 * u + lg), dof[u], dp[kt16]);
            }
        }
        // lane: query l16, keys kt*64 + 16*kt16 + 4*lg + r
#pragma unroll
        for (int kt16 = 0; kt16 < 4; ++kt16)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const bool ok = kt * 64 + kt16 * 16 + 4 * lg + r < Lk;
                const float pr = ok ? __builtin_amdgcn_exp2f(sp[kt16][r] - lse) : 0.f;
                sp[kt16][r] = pr * (dp[kt16][r] - delta);  // dS
            }
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const bf16x8 dsf = pack_p(sp, kk);
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) dq[dt] = mfma(tr_frag(kt_l, kk, dt, lg, l16), dsf, dq[dt]);
        }
    }
    if (q < qend) {
        bf16_t* dst = (bf16_t*)p.dqkv + ((int64_t)s * ntok + q) * rs + h * D;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
            *(uint2*)(dst + dt * 16 + 4 * lg) = make_uint2(pack_bf16x2(dq[dt][0] * p.scale, dq[dt][1] * p.scale),
                                                           pack_bf16x2(dq[dt][2] * p.scale, dq[dt][3] * p.scale));
        if (lg == 0) p.delta[((int64_t)s * H + h) * ntok + q] = delta;
    }
}

__global__ __launch_bounds__(256) MMT_BWD_DKV_ATTR void mam_bwd_dkv_kernel(const mmt_attn_bwd_params p) {
    __shared__ __attribute__((aligned(16))) char q_l[64 * TP];
    __shared__ __attribute__((aligned(16))) char do_l[64 * TP];
    __shared__ float lse_l[64], del_l[64];
    const int kt = blockIdx.x, h = blockIdx.y, s = blockIdx.z;
    const int n_t = p.n_t, ntok = p.ntok, C = p.C, H = p.H;
    const int64_t rs = 3 * (int64_t)C;
    const bf16_t* qkv = (const bf16_t*)p.qkv + (int64_t)s * ntok * rs + h * D;
    const bf16_t* dO = (const bf16_t*)p.dout + (int64_t)s * ntok * C + h * D;
    const float* lse = p.lse + ((int64_t)s * H + h) * ntok;
    const float* del = p.delta + ((int64_t)s * H + h) * ntok;
    const float c = p.scale * 1.4426950408889634f;

    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, l16 = lane & 15, lg = lane >> 4;
    const int key = kt * 64 + 16 * w + l16, kc = min(key, ntok - 1);
    u32x4 kb[2], vb[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        kb[u] = *(const u32x4*)(qkv + (int64_t)kc * rs + C + 32 * u + 8 * lg);
        vb[u] = *(const u32x4*)(qkv + (int64_t)kc * rs + 2 * C + 32 * u + 8 * lg);
    }
    // queries attending this key tile: template keys -> every query; search keys -> search queries
    const int q_lo = kt * 64 < n_t ? 0 : n_t;
    f32x4 dk[4], dv[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dk[dt] = dv[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    u32x4 qr[2], dr[2];
    float lr = 0.f, dl = 0.f;
    auto fetch = [&](int t0) {  // the query tile at t0 into registers
        load_tile(qr, qkv, rs, t0, ntok);
        load_tile(dr, dO, C, t0, ntok);
        if (threadIdx.x < 64) {
            lr = lse[min(t0 + (int)threadIdx.x, ntok - 1)];
            dl = del[min(t0 + (int)threadIdx.x, ntok - 1)];
        }
    };
    fetch(q_lo);
    for (int qt0 = q_lo; qt0 < ntok; qt0 += 64) {
        __syncthreads();  // every wave is past its reads of the previous tile
        store_tile(q_l, qr, c);
        store_tile(do_l, dr, 1.f);
        if (threadIdx.x < 64) {
            lse_l[threadIdx.x] = lr;
            del_l[threadIdx.x] = dl;
        }
        __syncthreads();
        if (qt0 + 64 < ntok) fetch(qt0 + 64);  // the next tile in flight while this one is multiplied
        f32x4 sp[4], dp[4];
#pragma unroll
        for (int qt16 = 0; qt16 < 4; ++qt16) {
            sp[qt16] = dp[qt16] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                sp[qt16] = mfma(row_frag(q_l, qt16 * 16 + l16, 4 * u + lg), kb[u], sp[qt16]);
                dp[qt16] = mfma(row_frag(do_l, qt16 * 16 + l16, 4 * u + lg), vb[u], dp[qt16]);
            }
        }
        // lane: key l16, queries qt0 + 16*qt16 + 4*lg + r
#pragma unroll
        for (int qt16 = 0; qt16 < 4; ++qt16)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int qi = 16 * qt16 + 4 * lg + r, qq = qt0 + qi;
                const bool ok = qq < ntok && key < ntok && (qq >= n_t || key < n_t);
                const float pr = ok ? __builtin_amdgcn_exp2f(sp[qt16][r] - lse_l[qi]) : 0.f;
                sp[qt16][r] = pr;
                dp[qt16][r] = pr * (dp[qt16][r] - del_l[qi]);  // dS
            }
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const bf16x8 pf = pack_p(sp, kk), dsf = pack_p(dp, kk);
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                dv[dt] = mfma(tr_frag(do_l, kk, dt, lg, l16), pf, dv[dt]);
                dk[dt] = mfma(tr_frag(q_l, kk, dt, lg, l16), dsf, dk[dt]);
            }
        }
    }
    if (key < ntok) {
        const float ks = 1.f / 1.4426950408889634f;  // q' = q * scale * log2 e  ->  dK = scale * dS^T q
        bf16_t* dst = (bf16_t*)p.dqkv + ((int64_t)s * ntok + key) * rs + h * D;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
            *(uint2*)(dst + C + dt * 16 + 4 * lg) = make_uint2(pack_bf16x2(dk[dt][0] * ks, dk[dt][1] * ks),
                                                               pack_bf16x2(dk[dt][2] * ks, dk[dt][3] * ks));
            *(uint2*)(dst + 2 * C + dt * 16 + 4 * lg) =
                make_uint2(pack_bf16x2(dv[dt][0], dv[dt][1]), pack_bf16x2(dv[dt][2], dv[dt][3]));
        }
    }
}

}  // namespace

extern "C" int mmt_mam_attention_bwd(const mmt_attn_bwd_params* p, int dtype, void* stream) {
    if (!p || dtype != MMT_BF16) return MMT_EBADARG;
    if (!p->qkv || !p->out || !p->dout || !p->lse || !p->delta || !p->dqkv) return MMT_EBADARG;
    if (p->asym || p->H <= 0 || p->C != p->H * D || p->S <= 0 || p->ntok <= p->n_t || p->n_t <= 0) return MMT_EBADARG;
    if (((uintptr_t)p->qkv | (uintptr_t)p->out | (uintptr_t)p->dout | (uintptr_t)p->dqkv) & 15) return MMT_EBADARG;
    hipStream_t st = (hipStream_t)stream;
    const int nqb = (p->n_t + 63) / 64 + (p->ntok - p->n_t + 63) / 64;
    hipLaunchKernelGGL(mam_bwd_dq_kernel, dim3(nqb, p->H, p->S), dim3(256), 0, st, *p);
    hipLaunchKernelGGL(mam_bwd_dkv_kernel, dim3((p->ntok + 63) / 64, p->H, p->S), dim3(256), 0, st, *p);
    return launch_status();
}
