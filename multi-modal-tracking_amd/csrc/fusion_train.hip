// The training step's deformable-encoder glue (deformable_encoder_lnspecific.py:131-160 with
// ms_deform_attn_bimodal.py:97-128, as mmt_amd.train.fusion_forward runs it), fused into one pass each:
//
//   mmt_ft_query_prep      query = src + lpos (fp32), the bimodal query [q_v | q_i] in bf16 (the offsets /
//                          weights Linear's operand) and src in bf16 (value_proj's operand) from one read of src;
//                          backward: d src = d pass-through + unshuffle(d q_bi) + d src_bf16, d lpos = the batch
//                          sum of unshuffle(d q_bi) (fixed order)
//   mmt_ft_drop_residual   x + dropout(y) (fp32 stream x, bf16 branch y), with `dup`: y holds the nq unique
//                          query rows of each half (the output_proj of the bimodal query, repeated on both
//                          halves, cat([y, y], 1)); backward: d y = the dropout backward (bf16), the halves' sum
//   mmt_ft_relu_drop       dropout(relu(h)) on the FFN's hidden activations (relu already applied by the GEMM
//                          epilogue); backward: the dropout and ReLU backward in one pass
//
// Dropout (nn.Dropout in training): keep with probability 1 - p, survivors scaled by 1 / (1 - p) in fp32 and
// rounded to bf16, as torch's fused dropout kernel computes them.  The keep draws come from a counter-based hash
// of (seed, step counter, call-site salt, element index) -- 16 bits per element, keep iff r16 < round((1 - p) 2^16)
// -- instead of torch's Philox stream: the same distribution, regenerated in the backward from the same key (no
// mask tensor), and graph-capturable: seed and counter live in device memory ({seed, counter} int64), and the
// step advances the counter with one captured add.  p = 0 or eval: plain adds / copies, no draws.
#include "common.hpp"

namespace {

struct FtDrop {
    const int64_t* state;  // {seed, counter}
    uint32_t salt;
    uint32_t thr;  // keep iff r16 < thr (0..65536)
    float scale;   // 1 / (1 - p)
    int on;
};

MMT_DEV uint64_t ft_mix(uint64_t x) {  // splitmix64 finaliser
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}

// keep factors (scale or 0) of the 8 elements 8 * c .. 8 * c + 7 of the call site's tensor
MMT_DEV void ft_keep8(const FtDrop& d, uint64_t key, int64_t c, float* k) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint64_t r = ft_mix(key ^ ((uint64_t)(2 * c + h) * 0xD1B54A32D192ED03ull));
#pragma unroll
        for (int j = 0; j < 4; ++j) k[4 * h + j] = ((uint32_t)(r >> (16 * j)) & 0xffffu) < d.thr ? d.scale : 0.f;
    }
}

MMT_DEV uint64_t ft_key(const FtDrop& d) {
    const uint64_t seed = (uint64_t)d.state[0], ctr = (uint64_t)d.state[1];
    return ft_mix(seed ^ ft_mix(ctr * 0x9E3779B97F4A7C15ull + d.salt));
}

MMT_DEV void ld8_f32(const float* p, float* v) {
    const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = a[j], v[4 + j] = b[j];
}
MMT_DEV void st8_f32(float* p, const float* v) {
    *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]};
    *(f32x4*)(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
}
MMT_DEV void ld8_bf16(const bf16_t* p, float* v) {
    const u32x4 u = *(const u32x4*)p;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        v[2 * j] = __uint_as_float(u[j] << 16);
        v[2 * j + 1] = __uint_as_float(u[j] & 0xffff0000u);
    }
}
MMT_DEV void st8_bf16(bf16_t* p, const float* v) {
    *(u32x4*)p = u32x4{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7])};
}
MMT_DEV float rbf(float x) { return bf2f(f2bf(x)); }  // round to bf16 and back

// src [B][2][nq][d] fp32, lpos [2][nq][d] fp32 -> qbi [B][nq][2d] bf16 = bf16(src + lpos) of the two halves side by
// side, srcb [B][2][nq][d] bf16 = bf16(src); one thread per 8 elements of src
__global__ __launch_bounds__(256) void ft_query_prep_kernel(const float* __restrict__ src, const float* __restrict__ lpos,
                                                            bf16_t* __restrict__ qbi, bf16_t* __restrict__ srcb, int nq,
                                                            int d8, int64_t total) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= total) return;
    const int c8 = (int)(i % d8);
    const int64_t rowi = i / d8;  // b * 2 nq + n
    const int n = (int)(rowi % (2 * nq));
    const int64_t b = rowi / (2 * nq);
    const int h = n / nq, q = n % nq;
    float s[8], l[8], o[8];
    ld8_f32(src + i * 8, s);
    ld8_f32(lpos + ((int64_t)n * d8 + c8) * 8, l);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = s[j] + l[j];
    st8_bf16(qbi + (((b * nq + q) * 2 + h) * d8 + c8) * 8, o);
    st8_bf16(srcb + i * 8, s);
}

// d src = dthrough (optional) + unshuffle(dqbi) + dsrcb (fp32), dlpos [2 nq][d] = sum over b of unshuffle(dqbi) in
// batch order; one thread per 8 elements of lpos, looping over the batch
__global__ __launch_bounds__(256) void ft_query_prep_bwd_kernel(const bf16_t* __restrict__ dqbi,
                                                                const bf16_t* __restrict__ dsrcb,
                                                                const float* __restrict__ dthrough,
                                                                float* __restrict__ dsrc, float* __restrict__ dlpos, int B,
                                                                int nq, int d8) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // n * d8 + c8
    if (i >= (int64_t)2 * nq * d8) return;
    const int c8 = (int)(i % d8), n = (int)(i / d8);
    const int h = n / nq, q = n % nq;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int b = 0; b < B; ++b) {
        const int64_t e = ((int64_t)b * 2 * nq * d8 + i) * 8;
        float dq[8], ds[8], dt[8];
        ld8_bf16(dqbi + ((((int64_t)b * nq + q) * 2 + h) * d8 + c8) * 8, dq);
        ld8_bf16(dsrcb + e, ds);
        if (dthrough) ld8_f32(dthrough + e, dt);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            acc[j] += dq[j];
            ds[j] = (dthrough ? dt[j] + dq[j] : dq[j]) + ds[j];
        }
        st8_f32(dsrc + e, ds);
    }
    st8_f32(dlpos + i * 8, acc);
}

// out [B][rows][d] fp32 = x + bf16(keep * y) (fp32 math, the branch rounded to bf16 as torch's dropout output);
// dup: y [B][rows / 2][d] repeated on both halves of the rows
__global__ __launch_bounds__(256) void ft_drop_residual_kernel(const float* __restrict__ x, const bf16_t* __restrict__ y,
                                                               float* __restrict__ out, FtDrop dr, int rows, int dup,
                                                               int d8, int64_t total) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= total) return;
    int64_t yi = i;
    if (dup) {
        const int c8 = (int)(i % d8);
        const int64_t rowi = i / d8;
        const int n = (int)(rowi % rows);
        const int64_t b = rowi / rows;
        yi = (b * (rows / 2) + n % (rows / 2)) * d8 + c8;
    }
    float xv[8], yv[8], k[8];
    ld8_f32(x + i * 8, xv);
    ld8_bf16(y + yi * 8, yv);
    if (dr.on) {
        ft_keep8(dr, ft_key(dr), i, k);
#pragma unroll
        for (int j = 0; j < 8; ++j) yv[j] = rbf(yv[j] * k[j]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[j] += yv[j];
    st8_f32(out + i * 8, xv);
}

// d y = bf16(keep * bf16(dout)) (torch: the add's gradient cast to the branch's dtype, then the dropout backward);
// dup: the two halves' results summed (bf16 + bf16 -> bf16, autograd's accumulation of the cat's slices)
__global__ __launch_bounds__(256) void ft_drop_residual_bwd_kernel(const float* __restrict__ dout, bf16_t* __restrict__ dy,
                                                                   FtDrop dr, int rows, int dup, int d8, int64_t total) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // chunk of dy
    if (i >= total) return;
    const uint64_t key = dr.on ? ft_key(dr) : 0;
    float acc[8];
    const int nh = dup ? 2 : 1;
    for (int hh = 0; hh < nh; ++hh) {
        int64_t oi = i;
        if (dup) {
            const int c8 = (int)(i % d8);
            const int64_t rowi = i / d8;
            const int q = (int)(rowi % (rows / 2));
            const int64_t b = rowi / (rows / 2);
            oi = (b * rows + hh * (rows / 2) + q) * d8 + c8;
        }
        float g[8], k[8];
        ld8_f32(dout + oi * 8, g);
        if (dr.on) ft_keep8(dr, key, oi, k);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            g[j] = rbf(g[j]);
            if (dr.on) g[j] = rbf(g[j] * k[j]);
            acc[j] = hh == 0 ? g[j] : acc[j] + g[j];
        }
    }
    st8_bf16(dy + i * 8, acc);
}

// out = bf16(keep * h) over n elements (h = relu(.) from the GEMM epilogue)
__global__ __launch_bounds__(256) void ft_relu_drop_kernel(const bf16_t* __restrict__ h, bf16_t* __restrict__ out,
                                                           FtDrop dr, int64_t total) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= total) return;
    float v[8], k[8];
    ld8_bf16(h + i * 8, v);
    ft_keep8(dr, ft_key(dr), i, k);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= k[j];
    st8_bf16(out + i * 8, v);
}

// dh = (h > 0) ? bf16(keep * dy) : 0 (the dropout backward, then ReLU's threshold_backward on its output)
__global__ __launch_bounds__(256) void ft_relu_drop_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ h,
                                                               bf16_t* __restrict__ dh, FtDrop dr, int64_t total) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= total) return;
    float g[8], hv[8], k[8];
    ld8_bf16(dy + i * 8, g);
    ld8_bf16(h + i * 8, hv);
    if (dr.on) ft_keep8(dr, ft_key(dr), i, k);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if (dr.on) g[j] = g[j] * k[j];
        g[j] = hv[j] > 0.f ? g[j] : 0.f;
    }
    st8_bf16(dh + i * 8, g);
}

// out [S][nrows][C] bf16 = bf16(x[s][row0 + r][c]) of x [S][rows][C] fp32 (the backbones' search tokens for the
// fusion's adjust Linears); backward: dx [S][rows][C] fp32 = float(dout) on those rows, 0 on the others
__global__ __launch_bounds__(256) void ft_rows_cast_kernel(const float* __restrict__ x, bf16_t* __restrict__ out,
                                                           int rows, int row0, int nrows, int c8, int64_t total) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // chunk of out
    if (i >= total) return;
    const int c = (int)(i % c8);
    const int64_t sr = i / c8;
    const int r = (int)(sr % nrows);
    const int64_t sq = sr / nrows;
    float v[8];
    ld8_f32(x + ((sq * rows + row0 + r) * c8 + c) * 8, v);
    st8_bf16(out + i * 8, v);
}

__global__ __launch_bounds__(256) void ft_rows_cast_bwd_kernel(const bf16_t* __restrict__ dout, float* __restrict__ dx,
                                                               int rows, int row0, int nrows, int c8, int64_t total) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // chunk of dx
    if (i >= total) return;
    const int c = (int)(i % c8);
    const int64_t sr = i / c8;
    const int r = (int)(sr % rows) - row0;
    const int64_t sq = sr / rows;
    float v[8];
    if (r >= 0 && r < nrows) {
        ld8_bf16(dout + ((sq * nrows + r) * c8 + c) * 8, v);
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = 0.f;
    }
    st8_f32(dx + i * 8, v);
}

FtDrop make_drop(const int64_t* state, int salt, float p) {
    FtDrop d;
    d.state = state;
    d.salt = (uint32_t)salt;
    d.on = state != nullptr && p > 0.f;
    const double keep = 1.0 - (double)p;
    d.thr = (uint32_t)(keep * 65536.0 + 0.5);
    d.scale = d.on ? (float)(1.0 / keep) : 1.f;
    return d;
}

unsigned grid_of(int64_t chunks) { return (unsigned)((chunks + 255) / 256); }

}  // namespace

extern "C" int mmt_ft_query_prep(const float* src, const float* lpos, void* qbi, void* srcb, int B, int nq, int d,
                                 void* stream) {
    if (!src || !lpos || !qbi || !srcb || B <= 0 || nq <= 0 || d <= 0 || d % 8) return MMT_EBADARG;
    if (((uintptr_t)src | (uintptr_t)lpos | (uintptr_t)qbi | (uintptr_t)srcb) & 15) return MMT_EBADARG;
    const int64_t total = (int64_t)B * 2 * nq * (d / 8);
    hipLaunchKernelGGL(ft_query_prep_kernel, dim3(grid_of(total)), dim3(256), 0, (hipStream_t)stream, src, lpos,
                       (bf16_t*)qbi, (bf16_t*)srcb, nq, d / 8, total);
    return launch_status();
}

extern "C" int mmt_ft_query_prep_bwd(const void* dqbi, const void* dsrcb, const float* dthrough, float* dsrc,
                                     float* dlpos, int B, int nq, int d, void* stream) {
    if (!dqbi || !dsrcb || !dsrc || !dlpos || B <= 0 || nq <= 0 || d <= 0 || d % 8) return MMT_EBADARG;
    if (((uintptr_t)dqbi | (uintptr_t)dsrcb | (uintptr_t)dthrough | (uintptr_t)dsrc | (uintptr_t)dlpos) & 15)
        return MMT_EBADARG;
    hipLaunchKernelGGL(ft_query_prep_bwd_kernel, dim3(grid_of((int64_t)2 * nq * (d / 8))), dim3(256), 0,
                       (hipStream_t)stream, (const bf16_t*)dqbi, (const bf16_t*)dsrcb, dthrough, dsrc, dlpos, B, nq,
                       d / 8);
    return launch_status();
}

extern "C" int mmt_ft_drop_residual(const float* x, const void* y, float* out, const int64_t* rng, int salt, float p,
                                    int B, int rows, int d, int dup, void* stream) {
    if (!x || !y || !out || B <= 0 || rows <= 0 || d <= 0 || d % 8 || (dup && rows % 2) || p < 0.f || p >= 1.f)
        return MMT_EBADARG;
    if (((uintptr_t)x | (uintptr_t)y | (uintptr_t)out) & 15) return MMT_EBADARG;
    const int64_t total = (int64_t)B * rows * (d / 8);
    hipLaunchKernelGGL(ft_drop_residual_kernel, dim3(grid_of(total)), dim3(256), 0, (hipStream_t)stream, x,
                       (const bf16_t*)y, out, make_drop(rng, salt, p), rows, dup, d / 8, total);
    return launch_status();
}

extern "C" int mmt_ft_drop_residual_bwd(const float* dout, void* dy, const int64_t* rng, int salt, float p, int B,
                                        int rows, int d, int dup, void* stream) {
    if (!dout || !dy || B <= 0 || rows <= 0 || d <= 0 || d % 8 || (dup && rows % 2) || p < 0.f || p >= 1.f)
        return MMT_EBADARG;
    if (((uintptr_t)dout | (uintptr_t)dy) & 15) return MMT_EBADARG;
    const int64_t total = (int64_t)B * (dup ? rows / 2 : rows) * (d / 8);
    hipLaunchKernelGGL(ft_drop_residual_bwd_kernel, dim3(grid_of(total)), dim3(256), 0, (hipStream_t)stream, dout,
                       (bf16_t*)dy, make_drop(rng, salt, p), rows, dup, d / 8, total);
    return launch_status();
}

extern "C" int mmt_ft_relu_drop(const void* h, void* out, const int64_t* rng, int salt, float p, int64_t n,
                                void* stream) {
    if (!h || !out || !rng || n <= 0 || n % 8 || p <= 0.f || p >= 1.f) return MMT_EBADARG;
    if (((uintptr_t)h | (uintptr_t)out) & 15) return MMT_EBADARG;
    hipLaunchKernelGGL(ft_relu_drop_kernel, dim3(grid_of(n / 8)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)h,
                       (bf16_t*)out, make_drop(rng, salt, p), n / 8);
    return launch_status();
}

extern "C" int mmt_ft_relu_drop_bwd(const void* dy, const void* h, void* dh, const int64_t* rng, int salt, float p,
                                    int64_t n, void* stream) {
    if (!dy || !h || !dh || n <= 0 || n % 8 || p < 0.f || p >= 1.f) return MMT_EBADARG;
    if (((uintptr_t)dy | (uintptr_t)h | (uintptr_t)dh) & 15) return MMT_EBADARG;
    hipLaunchKernelGGL(ft_relu_drop_bwd_kernel, dim3(grid_of(n / 8)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)dy, (const bf16_t*)h, (bf16_t*)dh, make_drop(rng, salt, p), n / 8);
    return launch_status();
}

extern "C" int mmt_ft_rows_cast(const float* x, void* out, int S, int rows, int row0, int nrows, int C, void* stream) {
    if (!x || !out || S <= 0 || rows <= 0 || row0 < 0 || nrows <= 0 || row0 + nrows > rows || C <= 0 || C % 8)
        return MMT_EBADARG;
    if (((uintptr_t)x | (uintptr_t)out) & 15) return MMT_EBADARG;
    const int64_t total = (int64_t)S * nrows * (C / 8);
    hipLaunchKernelGGL(ft_rows_cast_kernel, dim3(grid_of(total)), dim3(256), 0, (hipStream_t)stream, x, (bf16_t*)out,
                       rows, row0, nrows, C / 8, total);
    return launch_status();
}

extern "C" int mmt_ft_rows_cast_bwd(const void* dout, float* dx, int S, int rows, int row0, int nrows, int C,
                                    void* stream) {
    if (!dout || !dx || S <= 0 || rows <= 0 || row0 < 0 || nrows <= 0 || row0 + nrows > rows || C <= 0 || C % 8)
        return MMT_EBADARG;
    if (((uintptr_t)dout | (uintptr_t)dx) & 15) return MMT_EBADARG;
    const int64_t total = (int64_t)S * rows * (C / 8);
    hipLaunchKernelGGL(ft_rows_cast_bwd_kernel, dim3(grid_of(total)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)dout, dx, rows, row0, nrows, C / 8, total);
    return launch_status();
}
