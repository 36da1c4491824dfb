// AdamW update of the training step as three launches over every parameter:
// gradient-norm partials, the clip factor (+ the step counter and bias corrections, kept on the
// device so that the step can be captured in a hipGraph), and one fused update pass.
//
// Reference semantics: torch.nn.utils.clip_grad_norm_(params, max_norm) (ltr_trainer.py: TRAIN.
// GRAD_CLIP_NORM; total L2 norm, factor min(1, max_norm / (norm + 1e-6))) followed by
// torch.optim.AdamW(param_groups, weight_decay) (train_script_mixformer.py:105-140; per-group lr of
// base_functions.py:362-400) in PyTorch's fused form:
//   p *= 1 - lr * wd;  m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g^2;
//   p -= (lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps).
// The update pass is HBM-bound: 16 B read (p, g, m, v) and 12 B written (p, m, v) per parameter,
// plus the optional bf16 shadow copy of p (2 B) that the next forward's GEMMs read instead of a
// per-weight cast launch, and the optional gradient zeroing (4 B) that replaces zero_grad.
// Parameters are addressed through a device table of tensors and a list of fixed-size chunks
// (one workgroup each), so one launch covers the ~200 tensors of the model; the chunk order makes
// the norm's summation order fixed (the factor is bitwise reproducible).
#include "common.hpp"

#include <cmath>

namespace {

constexpr int CHUNK = 1 << 16;  // elements per chunk (one workgroup of 256 threads, 16 float4 each)

__global__ __launch_bounds__(256) void adamw_sqnorm_kernel(const mmt_adamw_tensor* __restrict__ tens,
                                                           const mmt_adamw_chunk* __restrict__ chunks,
                                                           float* __restrict__ partial) {
    const mmt_adamw_chunk c = chunks[blockIdx.x];
    const mmt_adamw_tensor t = tens[c.tensor];
    const int64_t n = min((int64_t)CHUNK, t.n - c.offset);
    const float* g = t.g + c.offset;
    float s = 0.f;
    if ((((uintptr_t)g) & 15) == 0) {
        const int64_t n4 = n >> 2;
        for (int64_t i = threadIdx.x; i < n4; i += 256) {
            const float4 v = ((const float4*)g)[i];
            s = fmaf(v.x, v.x, s);
            s = fmaf(v.y, v.y, s);
            s = fmaf(v.z, v.z, s);
            s = fmaf(v.w, v.w, s);
        }
        for (int64_t i = (n4 << 2) + threadIdx.x; i < n; i += 256) s = fmaf(g[i], g[i], s);
    } else {
        for (int64_t i = threadIdx.x; i < n; i += 256) s = fmaf(g[i], g[i], s);
    }
    __shared__ float red[256];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

// One workgroup: the clip factor and this step's bias corrections, into the device state
// st[0] = total norm (partials summed in fixed order), st[1] = min(1, max_norm / (norm + 1e-6)) (1
// without clipping), st[2] = 1 - b1^t, st[3] = sqrt(1 - b2^t) for t = ++step (st[4], an int32), so
// a captured hipGraph replays correct steps.
__global__ __launch_bounds__(256) void adamw_finalize_kernel(const float* __restrict__ partial, int n, float max_norm,
                                                             double b1, double b2, float* __restrict__ st) {
    double s = 0.0;
    for (int i = threadIdx.x; i < n; i += 256) s += (double)partial[i];
    __shared__ double red[256];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const float norm = (float)sqrt(red[0]);
        const int t = ((int*)st)[4] + 1;
        st[0] = norm;
        st[1] = max_norm > 0.f ? fminf(1.f, max_norm / (norm + 1e-6f)) : 1.f;
        st[2] = (float)(1.0 - pow(b1, (double)t));
        st[3] = (float)sqrt(1.0 - pow(b2, (double)t));
        ((int*)st)[4] = t;
    }
}

struct adamw_hp {
    float lr[MMT_ADAMW_MAX_GROUPS], wd[MMT_ADAMW_MAX_GROUPS];
    float b1, b2, omb1, omb2, eps;  // omb = 1 - b from the double values (as torch's scalars)
    int zero_grad;
};

MMT_DEV float adamw_one(float p, float& m, float& v, float g, float lr, float wd, float bc1, float bc2_sqrt,
                        const adamw_hp& h) {
    p *= 1.f - lr * wd;
    m = h.b1 * m + h.omb1 * g;
    v = h.b2 * v + h.omb2 * g * g;
    const float denom = sqrtf(v) / bc2_sqrt + h.eps;
    return p - (lr / bc1) * m / denom;
}

__global__ __launch_bounds__(256) void adamw_step_kernel(const mmt_adamw_tensor* __restrict__ tens,
                                                         const mmt_adamw_chunk* __restrict__ chunks,
                                                         const float* __restrict__ st, const adamw_hp h) {
    const mmt_adamw_chunk c = chunks[blockIdx.x];
    const mmt_adamw_tensor t = tens[c.tensor];
    const int64_t n = min((int64_t)CHUNK, t.n - c.offset);
    const float scale = st[1], bc1 = st[2], bc2s = st[3];
    const float lr = h.lr[t.group], wd = h.wd[t.group];
    float* p = t.p + c.offset;
    float* g = t.g + c.offset;
    float* m = t.m + c.offset;
    float* v = t.v + c.offset;
    uint16_t* sh = t.shadow ? t.shadow + c.offset : nullptr;
    const bool vec = ((((uintptr_t)p) | ((uintptr_t)g) | ((uintptr_t)m) | ((uintptr_t)v)) & 15) == 0 &&
                     (!sh || (((uintptr_t)sh) & 7) == 0);
    int64_t done = 0;
    if (vec) {
        const int64_t n4 = n >> 2;
        for (int64_t i = threadIdx.x; i < n4; i += 256) {
            float4 pp = ((const float4*)p)[i], gg = ((const float4*)g)[i];
            float4 mm = ((const float4*)m)[i], vv = ((const float4*)v)[i];
            pp.x = adamw_one(pp.x, mm.x, vv.x, gg.x * scale, lr, wd, bc1, bc2s, h);
            pp.y = adamw_one(pp.y, mm.y, vv.y, gg.y * scale, lr, wd, bc1, bc2s, h);
            pp.z = adamw_one(pp.z, mm.z, vv.z, gg.z * scale, lr, wd, bc1, bc2s, h);
            pp.w = adamw_one(pp.w, mm.w, vv.w, gg.w * scale, lr, wd, bc1, bc2s, h);
            ((float4*)p)[i] = pp;
            ((float4*)m)[i] = mm;
            ((float4*)v)[i] = vv;
            if (h.zero_grad) ((float4*)g)[i] = float4{0.f, 0.f, 0.f, 0.f};
            if (sh) {
                uint2 u;
                u.x = pack_bf16x2(pp.x, pp.y);
                u.y = pack_bf16x2(pp.z, pp.w);
                ((uint2*)sh)[i] = u;
            }
        }
        done = n4 << 2;
    }
    for (int64_t i = done + threadIdx.x; i < n; i += 256) {
        float mm = m[i], vv = v[i];
        const float pp = adamw_one(p[i], mm, vv, g[i] * scale, lr, wd, bc1, bc2s, h);
        p[i] = pp;
        m[i] = mm;
        v[i] = vv;
        if (h.zero_grad) g[i] = 0.f;
        if (sh) sh[i] = (uint16_t)(pack_bf16x2(pp, 0.f) & 0xffffu);
    }
}

}  // namespace

extern "C" int mmt_adamw_step(const mmt_adamw_tensor* tensors, const mmt_adamw_chunk* chunks, int nchunks,
                              float* partial, float* state, const float* lr, const float* weight_decay, int ngroups,
                              double beta1, double beta2, double eps, float max_norm, int zero_grad, void* stream) {
    if (!tensors || !chunks || nchunks <= 0 || !partial || !state || !lr || !weight_decay || ngroups < 1 ||
        ngroups > MMT_ADAMW_MAX_GROUPS)
        return MMT_EBADARG;
    hipStream_t st = (hipStream_t)stream;
    if (max_norm > 0.f)
        hipLaunchKernelGGL(adamw_sqnorm_kernel, dim3(nchunks), dim3(256), 0, st, tensors, chunks, partial);
    hipLaunchKernelGGL(adamw_finalize_kernel, dim3(1), dim3(256), 0, st, partial, max_norm > 0.f ? nchunks : 0,
                       max_norm, beta1, beta2, state);
    adamw_hp h{};
    for (int i = 0; i < ngroups; ++i) {
        h.lr[i] = lr[i];
        h.wd[i] = weight_decay[i];
    }
    h.b1 = (float)beta1;
    h.b2 = (float)beta2;
    h.omb1 = (float)(1.0 - beta1);
    h.omb2 = (float)(1.0 - beta2);
    h.eps = (float)eps;
    h.zero_grad = zero_grad;
    hipLaunchKernelGGL(adamw_step_kernel, dim3(nchunks), dim3(256), 0, st, tensors, chunks, (const float*)state, h);
    return launch_status();
}

extern "C" int mmt_adamw_chunk_elems(void) { return CHUNK; }
