// Candidate elimination (CE) of the asymmetric shared backbone for gfx950.
//
// Reference: lib/models/mixformer_vit_rgbt/asymmetric_shared_ce.py
//   Asym_Attention.forward(return_attention=True) :198-202  attn_t2s = softmax over the 2k search keys
//       [k_s_V | k_s_I] of the 2 n_t template queries [q_mt_V ; q_mt_I] (per head)
//   candidate_elimination :52-102: mean over the template queries (all of them when ce_template_mask is
//       None, as the tracker calls it; else the masked ones, :81-89, e.g. generate_mask_cond's CTR_POINT
//       mask, lib/utils/ce_utils.py:14-38, which the training actor passes) and heads, split into the
//       RGB / TIR halves, and per modality
//   get_token_from_attn :22-46: sort descending, keep the first ceil(keep_ratio * k) search tokens in
//       that order after the template tokens, global_index gathered alongside
//   VisionTransformer._recover_search :426-447: after the last block, the surviving tokens go back to
//       their original search positions, pruned positions become zero tokens.
//
// The token rows stay in the [S][pitch][C] streams at the original pitch (ntok); a stage only
// rewrites the first n_t + keep rows of every sequence, and the following blocks' GEMMs and
// attention run on those rows (row maps / mmt_attn_params.tok_pitch).
//
//   mmt_ce_t2s_attention  partial column sums of attn_t2s: one workgroup per (16 template queries
//                         (bf16, MFMA scores) or 8 (fp32, VALU), head, frame), scores from the qkv rows
//                         in place, softmax per query row in LDS, the rows summed per key ->
//                         partial[b][h][qblock][2k]; with a template mask ([b][2 n_t] bytes, query
//                         order [q_mt_V ; q_mt_I]) a row enters the sum times its 0 / 1 mask value, and
//                         a workgroup whose queries are all masked out writes zeros without scoring
//   mmt_ce_select         the partial sums added in a fixed order (deterministic) into each
//                         frame's first partial row, then one workgroup per (modality, frame): the
//                         rank of every token by (attention desc, index asc) -> the kept tokens in
//                         sorted order and their original positions
//   mmt_ce_gather         rows of the next stage: template rows copied, kept search rows gathered in
//                         rank order, from X into a second fp32 stream (+ the bf16 copy the folded
//                         LayerNorm GEMMs read)
//   mmt_ce_recover        the backbone output's search rows at their original positions (zeros
//                         where pruned), in the dtype the fusion reads
#include "common.hpp"

namespace {

constexpr int CE_QB = 8;        // template queries per t2s workgroup
constexpr int CE_MAXK = 1024;   // search tokens per modality (select workgroup size)

// One key row (64 values) held as loaded (16-B vectors), read as fp32 element by element.
template <typename T> struct CeRow;
template <> struct CeRow<bf16_t> {
    u32x4 c[8];
    MMT_DEV void load(const bf16_t* p) {
#pragma unroll
        for (int i = 0; i < 8; ++i) c[i] = *(const u32x4*)(p + 8 * i);
    }
    MMT_DEV float get(int d) const {
        const uint32_t u = c[d >> 3][(d & 7) >> 1];
        return __uint_as_float((d & 1) ? (u & 0xffff0000u) : (u << 16));
    }
};
template <> struct CeRow<float> {
    float4 c[16];
    MMT_DEV void load(const float* p) {
#pragma unroll
        for (int i = 0; i < 16; ++i) c[i] = *(const float4*)(p + 4 * i);
    }
    MMT_DEV float get(int d) const {
        const float4 v = c[d >> 2];
        return (d & 3) == 0 ? v.x : (d & 3) == 1 ? v.y : (d & 3) == 2 ? v.z : v.w;
    }
};

// One workgroup per (8 template queries, head, frame).  Scores go to LDS ([8][2k], 2k padded to a
// multiple of 4): per key a thread loads the row with 16-B vectors and takes the 8 dot products
// against the queries read as 16-B LDS broadcasts; each wave then normalises 2 query rows with
// 16-B LDS accesses, and the column sums over the 8 rows are written as this block's partial row.
template <typename T>
__global__ __launch_bounds__(256) void ce_t2s_kernel(const T* __restrict__ qkv, float* __restrict__ part,
                                                     const unsigned char* __restrict__ tmask, int Bm, int pitch,
                                                     int n_t, int k, int C, float scale) {
    extern __shared__ __attribute__((aligned(16))) float sm[];  // q [CE_QB][64] then scores [CE_QB][nkp]
    float* qs = sm;
    float* sc = sm + CE_QB * 64;
    const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z, nqb = gridDim.x, H = gridDim.y;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int nk = 2 * k, nkp = (nk + 3) & ~3;
    const int64_t rs = 3 * (int64_t)C;
    float* dst = part + (((int64_t)b * H + h) * nqb + qb) * nk;
    float mq[CE_QB];  // template-mask weight of each query row (1 without a mask)
    bool any = false;
#pragma unroll
    for (int qi = 0; qi < CE_QB; ++qi) {
        mq[qi] = tmask ? (tmask[(int64_t)b * 2 * n_t + qb * CE_QB + qi] ? 1.f : 0.f) : 1.f;
        any |= mq[qi] != 0.f;
    }
    if (!any) {  // block-uniform: no query of this block counts
        for (int key = tid; key < nk; key += 256) dst[key] = 0.f;
        return;
    }
    for (int e = tid; e < CE_QB * 64; e += 256) {  // [q_mt_V ; q_mt_I]: query gq < n_t from frame b's RGB rows
        const int gq = qb * CE_QB + (e >> 6);
        const int seq = gq < n_t ? b : b + Bm, row = gq < n_t ? gq : gq - n_t;
        qs[e] = to_f<T>(qkv[((int64_t)seq * pitch + row) * rs + h * 64 + (e & 63)]);
    }
    for (int e = nk + tid; e < nkp; e += 256)
        for (int qi = 0; qi < CE_QB; ++qi) sc[qi * nkp + e] = -INFINITY;  // padding keys: exp -> 0
    __syncthreads();
    for (int key = tid; key < nk; key += 256) {  // [k_s_V | k_s_I]
        const int seq = key < k ? b : b + Bm, row = n_t + (key < k ? key : key - k);
        CeRow<T> r;
        r.load(qkv + ((int64_t)seq * pitch + row) * rs + C + h * 64);
#pragma unroll 2
        for (int qi = 0; qi < CE_QB; ++qi) {
            float acc = 0.f;
#pragma unroll
            for (int d = 0; d < 64; d += 4) {
                const float4 q4 = *(const float4*)(qs + qi * 64 + d);  // LDS broadcast
                acc = fmaf(q4.x, r.get(d), acc);
                acc = fmaf(q4.y, r.get(d + 1), acc);
                acc = fmaf(q4.z, r.get(d + 2), acc);
                acc = fmaf(q4.w, r.get(d + 3), acc);
            }
            sc[qi * nkp + key] = acc * scale;
        }
    }
    __syncthreads();
    for (int qi = w; qi < CE_QB; qi += 4) {  // softmax of each query row (fp32, max-subtracted)
        float4* r4 = (float4*)(sc + qi * nkp);
        const int n4 = nkp >> 2;
        float mx = -INFINITY;
        for (int j = lane; j < n4; j += 64) {
            const float4 v = r4[j];
            mx = fmaxf(mx, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
        }
        mx = wave_max(mx);
        float se = 0.f;
        for (int j = lane; j < n4; j += 64) {
            float4 v = r4[j];
            v.x = expf(v.x - mx);
            v.y = expf(v.y - mx);
            v.z = expf(v.z - mx);
            v.w = expf(v.w - mx);
            se += (v.x + v.y) + (v.z + v.w);
            r4[j] = v;
        }
        const float inv = 1.f / wave_sum(se);
        for (int j = lane; j < n4; j += 64) {
            float4 v = r4[j];
            v.x *= inv;
            v.y *= inv;
            v.z *= inv;
            v.w *= inv;
            r4[j] = v;
        }
    }
    __syncthreads();
    for (int key = tid; key < nk; key += 256) {
        float s2 = 0.f;
#pragma unroll
        for (int qi = 0; qi < CE_QB; ++qi) s2 += sc[qi * nkp + key] * mq[qi];
        dst[key] = s2;
    }
}

// bf16 path: the scores of 16 template queries by MFMA, kept in registers.  S^T [16 keys][16
// queries] blocks = K Q^T with v_mfma_f32_16x16x32_bf16 (A = key rows, B = query rows, 16-B
// fragments read straight from the qkv rows, all of a wave's key blocks loaded up front); lane l
// holds query l%16 against keys 4*(l/16)..+3 of each block.  Row max / sum: over the lane's values,
// the 4 lanes of the query (permlane swaps) and the 4 waves (LDS); column sums over the 16 queries:
// DPP row scans inside each 16-lane group.  No score matrix in LDS.
// inclusive sum over the 16 lanes of a DPP row (row_shr 1, 2, 4, 8; lanes shifted in from outside the
// row add 0): lane 15 of each row holds the row's total
MMT_DEV float ce_row16_sum(float v) {
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x111, 0xf, 0xf, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x112, 0xf, 0xf, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x114, 0xf, 0xf, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x118, 0xf, 0xf, false));
    return v;
}
constexpr int CE_QBM = 16, CE_MAXI = 18;  // key blocks per wave: 2k <= 4 * 18 * 16 = 1152 (ViT-L 384 px)
__global__ __launch_bounds__(256) void ce_t2s_mfma_kernel(const bf16_t* __restrict__ qkv, float* __restrict__ part,
                                                          const unsigned char* __restrict__ tmask, int Bm, int pitch,
                                                          int n_t, int k, int C, float scale) {
    __shared__ float red[2][4][16];
    const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z, nqb = gridDim.x, H = gridDim.y;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l16 = lane & 15, lg = lane >> 4;
    const int nk = 2 * k, nkb = (nk + 15) / 16;
    const int64_t rs = 3 * (int64_t)C;
    const int gq = qb * CE_QBM + l16;  // query of [q_mt_V ; q_mt_I]
    float* dst = part + (((int64_t)b * H + h) * nqb + qb) * nk;
    // template-mask weight of this lane's query (1 without a mask); every wave holds the same 16
    // queries, so a block with none of them counted is skipped by all four waves alike
    const float mq = tmask ? (tmask[(int64_t)b * 2 * n_t + gq] ? 1.f : 0.f) : 1.f;
    if (__all(mq == 0.f)) {
        for (int key = tid; key < nk; key += 256) dst[key] = 0.f;
        return;
    }
    const int qseq = gq < n_t ? b : b + Bm, qrow = gq < n_t ? gq : gq - n_t;
    const bf16_t* qp = qkv + ((int64_t)qseq * pitch + qrow) * rs + h * 64 + 8 * lg;
    const u32x4 q0 = *(const u32x4*)qp, q1 = *(const u32x4*)(qp + 32);
    u32x4 kf[CE_MAXI][2];
#pragma unroll
    for (int i = 0; i < CE_MAXI; ++i) {
        const int kb = w + 4 * i;
        if (kb < nkb) {
            const int key = min(kb * 16 + l16, nk - 1);  // clamped; masked below
            const int seq = key < k ? b : b + Bm, row = n_t + (key < k ? key : key - k);
            const bf16_t* kp = qkv + ((int64_t)seq * pitch + row) * rs + C + h * 64 + 8 * lg;
            kf[i][0] = *(const u32x4*)kp;
            kf[i][1] = *(const u32x4*)(kp + 32);
        }
    }
    f32x4 sc[CE_MAXI];
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < CE_MAXI; ++i) {
        const int kb = w + 4 * i;
        if (kb < nkb) {
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kf[i][0]),
                                                          __builtin_bit_cast(bf16x8, q0), acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kf[i][1]),
                                                          __builtin_bit_cast(bf16x8, q1), acc, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                acc[r] = kb * 16 + 4 * lg + r < nk ? acc[r] * scale : -INFINITY;
                mx = fmaxf(mx, acc[r]);
            }
            sc[i] = acc;
        }
    }
    mx = lanegroup_max(mx);  // the 4 lanes of the query (l, l^16, l^32, l^48)
    if (lg == 0) red[0][w][l16] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(red[0][0][l16], red[0][1][l16]), fmaxf(red[0][2][l16], red[0][3][l16]));
    float se = 0.f;
#pragma unroll
    for (int i = 0; i < CE_MAXI; ++i) {
        if (w + 4 * i < nkb) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                sc[i][r] = expf(sc[i][r] - mx);
                se += sc[i][r];
            }
        }
    }
    se = lanegroup_sum(se);
    if (lg == 0) red[1][w][l16] = se;
    __syncthreads();
    const float inv = 1.f / ((red[1][0][l16] + red[1][1][l16]) + (red[1][2][l16] + red[1][3][l16]));
#pragma unroll
    for (int i = 0; i < CE_MAXI; ++i) {
        const int kb = w + 4 * i;
        if (kb < nkb) {
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = ce_row16_sum(sc[i][r] * inv * mq);  // sum over the 16 queries
            if (l16 == 15) {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (kb * 16 + 4 * lg + r < nk) dst[kb * 16 + 4 * lg + r] = v[r];
            }
        }
    }
}

// Sum of the nparts partial rows of frame b into row 0, for 64 keys per workgroup: the 16 waves
// take interleaved parts, lanes take keys (coalesced), and the 16 wave sums are added in wave order
// (a fixed order: the selection is deterministic).
__global__ __launch_bounds__(1024) void ce_reduce_kernel(float* __restrict__ part, int nparts, int nk) {
    __shared__ float red[16][64];
    const int b = blockIdx.y, key = blockIdx.x * 64 + (threadIdx.x & 63), w = threadIdx.x >> 6;
    float* pb = part + (int64_t)b * nparts * nk;
    float v = 0.f;
    if (key < nk) {
        for (int q0 = w; q0 < nparts; q0 += 16 * 16) {  // 16 loads in flight per lane, added in order
            float t[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) t[i] = q0 + 16 * i < nparts ? pb[(int64_t)(q0 + 16 * i) * nk + key] : 0.f;
#pragma unroll
            for (int i = 0; i < 16; ++i) v += t[i];
        }
    }
    red[w][threadIdx.x & 63] = v;
    __syncthreads();
    if (w == 0 && key < nk) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) s += red[i][threadIdx.x];
        pb[key] = s;
    }
}

// One workgroup per (64 tokens, modality, frame): lane = token, the 16 waves count over 16 slices
// of the k sums in LDS (a single wave's compare chain over all k was latency-bound), partial ranks
// added through LDS; rank = #(sum greater) + #(equal sum at a lower index).
__global__ __launch_bounds__(1024) void ce_select_kernel(const float* __restrict__ part, int nparts, int Bm, int k,
                                                         int keep, int ns_full, const int* __restrict__ gidx_in,
                                                         int* __restrict__ gidx_out, int* __restrict__ order,
                                                         float* __restrict__ mean_out, float mean_scale) {
    __shared__ __attribute__((aligned(16))) float a[CE_MAXK + 64];
    __shared__ int pr[16][64];
    const int s = blockIdx.y, m = s / Bm, b = s % Bm, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int nk = 2 * k, sl = ((k + 63) / 64) * 4, kp = 16 * sl;  // slice length: a multiple of 4
    const float* sum = part + (int64_t)b * nparts * nk + m * k;    // row 0 = the sum (ce_reduce_kernel)
    for (int j = tid; j < kp; j += 1024) a[j] = j < k ? sum[j] : -INFINITY;  // padding never counts
    __syncthreads();
    const int i = blockIdx.x * 64 + lane;
    const float ai = a[min(i, k - 1)];
    int rank = 0;
    for (int j0 = w * sl; j0 < w * sl + sl; j0 += 4) {
        const float4 v = *(const float4*)(a + j0);
        rank += (v.x > ai) || (v.x == ai && j0 < i);
        rank += (v.y > ai) || (v.y == ai && j0 + 1 < i);
        rank += (v.z > ai) || (v.z == ai && j0 + 2 < i);
        rank += (v.w > ai) || (v.w == ai && j0 + 3 < i);
    }
    pr[w][lane] = rank;
    __syncthreads();
    if (w != 0 || i >= k) return;
#pragma unroll
    for (int u = 1; u < 16; ++u) rank += pr[u][lane];
    if (mean_out) mean_out[(int64_t)b * nk + m * k + i] = ai * mean_scale;
    if (rank < keep) {
        order[(int64_t)s * ns_full + rank] = i;
        gidx_out[(int64_t)s * ns_full + rank] = gidx_in ? gidx_in[(int64_t)s * ns_full + i] : i;
    }
}

template <typename TO>
__global__ __launch_bounds__(256) void ce_gather_kernel(const float* __restrict__ x, float* __restrict__ xc,
                                                        TO* __restrict__ xn, const int* __restrict__ order, int pitch,
                                                        int n_t, int ns_full, int C) {
    const int r = blockIdx.x, s = blockIdx.y;
    const int src = r < n_t ? r : n_t + order[(int64_t)s * ns_full + (r - n_t)];
    const float* xs = x + ((int64_t)s * pitch + src) * C;
    const int64_t dro = ((int64_t)s * pitch + r) * C;
    for (int c = threadIdx.x * 4; c < C; c += 1024) {
        const float4 v = *(const float4*)(xs + c);
        *(float4*)(xc + dro + c) = v;
        if (xn) {
            xn[dro + c] = from_f<TO>(v.x);
            xn[dro + c + 1] = from_f<TO>(v.y);
            xn[dro + c + 2] = from_f<TO>(v.z);
            xn[dro + c + 3] = from_f<TO>(v.w);
        }
    }
}

// One workgroup per (original search position, sequence): its slot among the survivors (a scan
// of the final gidx, at most ns_full entries) -> that row, or a zero row.
template <typename TO>
__global__ __launch_bounds__(256) void ce_recover_kernel(const float* __restrict__ x, const int* __restrict__ gidx,
                                                         int keep, TO* __restrict__ out, int pitch, int n_t,
                                                         int ns_full, int C) {
    __shared__ int slot;
    const int pos = blockIdx.x, s = blockIdx.y;
    if (threadIdx.x == 0) slot = -1;
    __syncthreads();
    for (int j = threadIdx.x; j < keep; j += 256)
        if (gidx[(int64_t)s * ns_full + j] == pos) slot = j;  // at most one match
    __syncthreads();
    TO* o = out + ((int64_t)s * pitch + n_t + pos) * C;
    const float* xs = x + ((int64_t)s * pitch + n_t + (slot < 0 ? 0 : slot)) * C;
    for (int c = threadIdx.x * 4; c < C; c += 1024) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (slot >= 0) v = *(const float4*)(xs + c);
        o[c] = from_f<TO>(v.x);
        o[c + 1] = from_f<TO>(v.y);
        o[c + 2] = from_f<TO>(v.z);
        o[c + 3] = from_f<TO>(v.w);
    }
}

}  // namespace

extern "C" int mmt_ce_t2s_attention_masked(const void* qkv, float* partial, const unsigned char* template_mask, int Bm,
                                           int tok_pitch, int n_t, int n_s, int C, int H, float scale, int dtype,
                                           void* stream) {
    if (!qkv || !partial || Bm <= 0 || n_t <= 0 || n_s <= 0 || C != 64 * H || H <= 0 || (2 * n_t) % CE_QBM ||
        tok_pitch < n_t + n_s || n_s > CE_MAXK)
        return MMT_EBADARG;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == MMT_BF16) {
        if (2 * n_s > 4 * CE_MAXI * 16) return MMT_EBADARG;
        hipLaunchKernelGGL(ce_t2s_mfma_kernel, dim3((unsigned)(2 * n_t / CE_QBM), (unsigned)H, (unsigned)Bm), dim3(256),
                           0, st, (const bf16_t*)qkv, partial, template_mask, Bm, tok_pitch, n_t, n_s, C, scale);
    } else if (dtype == MMT_F32) {
        const size_t shm = sizeof(float) * (CE_QB * 64 + CE_QB * (size_t)((2 * n_s + 3) & ~3));
        hipLaunchKernelGGL(ce_t2s_kernel<float>, dim3((unsigned)(2 * n_t / CE_QB), (unsigned)H, (unsigned)Bm),
                           dim3(256), shm, st, (const float*)qkv, partial, template_mask, Bm, tok_pitch, n_t, n_s, C,
                           scale);
    } else return MMT_EBADARG;
    return launch_status();
}

extern "C" int mmt_ce_t2s_attention(const void* qkv, float* partial, int Bm, int tok_pitch, int n_t, int n_s, int C,
                                    int H, float scale, int dtype, void* stream) {
    return mmt_ce_t2s_attention_masked(qkv, partial, nullptr, Bm, tok_pitch, n_t, n_s, C, H, scale, dtype, stream);
}

extern "C" int mmt_ce_select(float* partial, int nparts, int Bm, int n_s, int keep, int ns_full, const int* gidx_in,
                             int* gidx_out, int* order, float* attn_mean, float mean_scale, void* stream) {
    if (!partial || !gidx_out || !order || nparts <= 0 || Bm <= 0 || n_s <= 0 || n_s > ns_full || ns_full > CE_MAXK ||
        keep <= 0 || keep > n_s || gidx_in == gidx_out)
        return MMT_EBADARG;
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(ce_reduce_kernel, dim3((unsigned)((2 * n_s + 63) / 64), (unsigned)Bm), dim3(1024), 0, st,
                       partial, nparts, 2 * n_s);
    hipLaunchKernelGGL(ce_select_kernel, dim3((unsigned)((n_s + 63) / 64), (unsigned)(2 * Bm)), dim3(1024), 0, st,
                       partial, nparts, Bm, n_s, keep, ns_full, gidx_in, gidx_out, order, attn_mean, mean_scale);
    return launch_status();
}

extern "C" int mmt_ce_gather(const float* x, float* xc, void* xn, const int* order, int S, int tok_pitch, int n_t,
                             int keep, int ns_full, int C, int xn_dtype, void* stream) {
    if (!x || !xc || !order || x == xc || S <= 0 || n_t <= 0 || keep <= 0 || keep > ns_full ||
        tok_pitch < n_t + ns_full || C <= 0 || C % 4 || C > 1024)
        return MMT_EBADARG;
    dim3 grid((unsigned)(n_t + keep), (unsigned)S);
    hipStream_t st = (hipStream_t)stream;
    if (!xn || xn_dtype == MMT_BF16)
        hipLaunchKernelGGL(ce_gather_kernel<bf16_t>, grid, dim3(256), 0, st, x, xc, (bf16_t*)xn, order, tok_pitch, n_t,
                           ns_full, C);
    else if (xn_dtype == MMT_F32)
        hipLaunchKernelGGL(ce_gather_kernel<float>, grid, dim3(256), 0, st, x, xc, (float*)xn, order, tok_pitch, n_t,
                           ns_full, C);
    else return MMT_EBADARG;
    return launch_status();
}

extern "C" int mmt_ce_recover(const float* x, const int* gidx, int keep, void* out, int S, int tok_pitch, int n_t,
                              int ns_full, int C, int dtype, void* stream) {
    if (!x || !gidx || !out || S <= 0 || n_t <= 0 || ns_full <= 0 || keep <= 0 || keep > ns_full ||
        tok_pitch < n_t + ns_full || C <= 0 || C % 4 || C > 1024 || (const void*)x == out)
        return MMT_EBADARG;
    dim3 grid((unsigned)ns_full, (unsigned)S);
    hipStream_t st = (hipStream_t)stream;
    if (dtype == MMT_BF16)
        hipLaunchKernelGGL(ce_recover_kernel<bf16_t>, grid, dim3(256), 0, st, x, gidx, keep, (bf16_t*)out, tok_pitch, n_t,
                           ns_full, C);
    else if (dtype == MMT_F32)
        hipLaunchKernelGGL(ce_recover_kernel<float>, grid, dim3(256), 0, st, x, gidx, keep, (float*)out, tok_pitch, n_t,
                           ns_full, C);
    else return MMT_EBADARG;
    return launch_status();
}
