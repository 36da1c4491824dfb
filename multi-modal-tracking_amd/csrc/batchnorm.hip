// BatchNorm2d + ReLU of the corner head's conv() blocks (lib/models/mixformer_cvt/head.py:7-20) in the
// training step, on NHWC bf16 maps [M = B*H*W][C]: per-channel batch statistics (training) or running
// statistics (eval), the affine and the ReLU in one elementwise pass, and the backward through the ReLU
// mask.  Replaces MIOpen's batch-norm kernels and the NCHW <-> NHWC copies around them.
//
// Statistics are sums in a fixed order (rows of a workgroup, then workgroups in index order, in double
// at the end), so the results are bitwise reproducible; the sums are taken about a per-channel pivot (the
// first row's value) so that E[x^2] - E[x]^2 does not cancel for channels with a large mean.
#include "common.hpp"

namespace {

constexpr int BN_THREADS = 256;

// rows [r0, r1) of this workgroup: the grid splits M into gridDim.x nearly equal runs
MMT_DEV void bn_rows(int64_t M, int64_t& r0, int64_t& r1) {
    r0 = M * blockIdx.x / gridDim.x;
    r1 = M * (blockIdx.x + 1) / gridDim.x;
}

MMT_DEV void unpack8(const u32x4 u, float* f) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const f32x2 v = unpack2<bf16_t>(u[j]);
        f[2 * j] = v.x;
        f[2 * j + 1] = v.y;
    }
}

// Per-workgroup (sum, sum of squares) of x - pivot over its rows: part[blk][2][C].  Rows are `pitch`
// channels apart (pitch >= C, a multiple of 8: the 1-channel maps live in 8-channel rows); thread t owns
// channel chunk t % C8 (8 channels, one 16-B load per row) and rows t / C8 + k * R of the run (R = 256 / C8);
// the R row lanes are summed through LDS in lane order, channels >= C are never stored.
__global__ __launch_bounds__(BN_THREADS) void bn_stats_kernel(const u32x4* __restrict__ x, int64_t M, int C, int pitch,
                                                              float* __restrict__ part) {
    __shared__ float red[BN_THREADS * 16];
    const int C8 = pitch / 8, R = BN_THREADS / C8, t = threadIdx.x;
    const int ck = t % C8, rl = t / C8;
    int64_t r0, r1;
    bn_rows(M, r0, r1);
    float s[8], q[8], piv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
    unpack8(x[ck], piv);
    if (rl < R) {
#pragma unroll 4
        for (int64_t r = r0 + rl; r < r1; r += R) {
            float v[8];
            unpack8(x[r * C8 + ck], v);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float d = v[j] - piv[j];
                s[j] += d;
                q[j] += d * d;
            }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            red[(rl * C8 + ck) * 16 + j] = s[j];
            red[(rl * C8 + ck) * 16 + 8 + j] = q[j];
        }
    }
    __syncthreads();
    for (int c = t; c < 2 * C; c += BN_THREADS) {  // (kind, channel): lanes summed in order
        const int kind = c / C, ch = c % C;
        float acc = 0.f;
        for (int l = 0; l < R; ++l) acc += red[(l * C8 + ch / 8) * 16 + kind * 8 + ch % 8];
        part[((int64_t)blockIdx.x * 2 + kind) * C + ch] = acc;
    }
}

// The batch mean / variance from the partials, the running statistics update (momentum, unbiased variance
// as nn.BatchNorm2d), and the per-channel coefficients save[4][C] = (mean, invstd, scale = gamma * invstd,
// shift = beta - mean * scale); eval (training = 0): the running statistics give mean / invstd.  A
// workgroup serves 32 channels: lane l of channel c sums the workgroup partials l, l + 8, ... in double,
// then the 8 lanes are added in order (fixed order: bitwise reproducible).
constexpr int BN_FCH = 32, BN_FLANES = BN_THREADS / BN_FCH;

MMT_DEV void bn_lane_sums(const float* __restrict__ part, int nblk, int C, int c, int lane, double* red, double& a,
                          double& b) {
    double s = 0.0, q = 0.0;
    if (c < C) {
        // eight partials' loads in flight, then summed in k order (round 6: one load per iteration serialised the
        // loop on its latency, ~9 us per finalize launch)
        int k = lane;
        for (; k + 7 * BN_FLANES < nblk; k += 8 * BN_FLANES) {
            float a[8], b[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                a[j] = part[((int64_t)(k + j * BN_FLANES) * 2) * C + c];
                b[j] = part[((int64_t)(k + j * BN_FLANES) * 2 + 1) * C + c];
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                s += (double)a[j];
                q += (double)b[j];
            }
        }
        for (; k < nblk; k += BN_FLANES) {
            s += (double)part[((int64_t)k * 2) * C + c];
            q += (double)part[((int64_t)k * 2 + 1) * C + c];
        }
    }
    const int t = threadIdx.x;
    red[t] = s;
    red[BN_THREADS + t] = q;
    __syncthreads();
    a = b = 0.0;
    if (lane == 0) {
        for (int l = 0; l < BN_FLANES; ++l) {
            a += red[l * BN_FCH + t];
            b += red[BN_THREADS + l * BN_FCH + t];
        }
    }
}

__global__ __launch_bounds__(BN_THREADS) void bn_finalize_kernel(const u32x4* __restrict__ x, const float* __restrict__ part,
                                                                 int nblk, int64_t M, int C, const float* __restrict__ gamma,
                                                                 const float* __restrict__ beta, float* running_mean,
                                                                 float* running_var, float momentum, float eps,
                                                                 int training, float* __restrict__ save) {
    __shared__ double red[2 * BN_THREADS];
    const int lane = threadIdx.x / BN_FCH, c = blockIdx.x * BN_FCH + threadIdx.x % BN_FCH;
    double s = 0.0, q = 0.0;
    if (training) bn_lane_sums(part, nblk, C, c, lane, red, s, q);
    if (lane != 0 || c >= C) return;
    float mean, var;
    if (training) {
        const bf16_t* xb = (const bf16_t*)x;  // pivot: row 0
        const double ms = s / (double)M;
        const double vb = fmax(q / (double)M - ms * ms, 0.0);  // biased (normalisation)
        mean = (float)((double)bf2f(xb[c]) + ms);
        var = (float)vb;
        if (running_mean) {
            running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
            const double vu = M > 1 ? vb * (double)M / (double)(M - 1) : vb;  // unbiased (running)
            running_var[c] = (1.f - momentum) * running_var[c] + momentum * (float)vu;
        }
    } else {
        mean = running_mean[c];
        var = running_var[c];
    }
    const float inv = 1.f / sqrtf(var + eps);
    const float sc = (gamma ? gamma[c] : 1.f) * inv;
    save[c] = mean;
    save[C + c] = inv;
    save[2 * C + c] = sc;
    save[3 * C + c] = (beta ? beta[c] : 0.f) - mean * sc;
}

// y = relu(x * scale + shift) (bf16 out, padding channels 0), 8 channels per thread
__global__ __launch_bounds__(BN_THREADS) void bn_apply_kernel(const u32x4* __restrict__ x, u32x4* __restrict__ y, int64_t n8,
                                                              int C, int pitch, const float* __restrict__ save, int relu) {
    const int64_t i = (int64_t)blockIdx.x * BN_THREADS + threadIdx.x;
    if (i >= n8) return;
    const int c0 = (int)(i % (pitch / 8)) * 8;
    float v[8], r[8];
    unpack8(x[i], v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int c = c0 + j;
        float a = c < C ? v[j] * save[2 * C + c] + save[3 * C + c] : 0.f;  // padding channels: 0
        r[j] = relu ? fmaxf(a, 0.f) : a;
    }
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = pack_bf16x2(r[2 * j], r[2 * j + 1]);
    y[i] = o;
}

// Backward partials: g = dy * [x * scale + shift > 0] (the forward's pre-activation, same arithmetic), per
// workgroup (sum g * xhat, sum g) -> part[blk][2][C] (dgamma, dbeta order)
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_stats_kernel(const u32x4* __restrict__ x, const u32x4* __restrict__ dy,
                                                                  int64_t M, int C, int pitch, const float* __restrict__ save,
                                                                  int relu, float* __restrict__ part) {
    __shared__ float red[BN_THREADS * 16];
    const int C8 = pitch / 8, R = BN_THREADS / C8, t = threadIdx.x;
    const int ck = t % C8, rl = t / C8, c0 = ck * 8;
    int64_t r0, r1;
    bn_rows(M, r0, r1);
    float sgx[8], sg[8], mean[8], inv[8], sc[8], sh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {  // padding channels (c >= C): zero coefficients, never stored
        const bool in = c0 + j < C;
        sgx[j] = sg[j] = 0.f;
        mean[j] = in ? save[c0 + j] : 0.f;
        inv[j] = in ? save[C + c0 + j] : 0.f;
        sc[j] = in ? save[2 * C + c0 + j] : 0.f;
        sh[j] = in ? save[3 * C + c0 + j] : 0.f;
    }
    if (rl < R) {
#pragma unroll 4
        for (int64_t r = r0 + rl; r < r1; r += R) {
            float v[8], d[8];
            unpack8(x[r * C8 + ck], v);
            unpack8(dy[r * C8 + ck], d);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float g = (!relu || v[j] * sc[j] + sh[j] > 0.f) ? d[j] : 0.f;
                sg[j] += g;
                sgx[j] += g * ((v[j] - mean[j]) * inv[j]);
            }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            red[(rl * C8 + ck) * 16 + j] = sgx[j];
            red[(rl * C8 + ck) * 16 + 8 + j] = sg[j];
        }
    }
    __syncthreads();
    for (int c = t; c < 2 * C; c += BN_THREADS) {
        const int kind = c / C, ch = c % C;
        float acc = 0.f;
        for (int l = 0; l < R; ++l) acc += red[(l * C8 + ch / 8) * 16 + kind * 8 + ch % 8];
        part[((int64_t)blockIdx.x * 2 + kind) * C + ch] = acc;
    }
}

// dgb[2][C] = (dgamma, dbeta) summed over the workgroups (bn_lane_sums order), and the dx coefficients
// coef[3][C] = (gamma * invstd, dbeta / M, dgamma / M) (training) or (gamma * invstd, 0, 0) (eval)
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_finalize_kernel(const float* __restrict__ part, int nblk, int64_t M,
                                                                     int C, const float* __restrict__ gamma,
                                                                     const float* __restrict__ save, int training,
                                                                     float* __restrict__ dgb, float* __restrict__ coef) {
    __shared__ double red[2 * BN_THREADS];
    const int lane = threadIdx.x / BN_FCH, c = blockIdx.x * BN_FCH + threadIdx.x % BN_FCH;
    double a, b;
    bn_lane_sums(part, nblk, C, c, lane, red, a, b);
    if (lane != 0 || c >= C) return;
    dgb[c] = (float)a;
    dgb[C + c] = (float)b;
    coef[c] = (gamma ? gamma[c] : 1.f) * save[C + c];
    coef[C + c] = training ? (float)(b / (double)M) : 0.f;
    coef[2 * C + c] = training ? (float)(a / (double)M) : 0.f;
}

// dx = gamma * invstd * (g - mean(g) - xhat * mean(g * xhat)) (training) or gamma * invstd * g (eval), bf16
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_dx_kernel(const u32x4* __restrict__ x, const u32x4* __restrict__ dy,
                                                               u32x4* __restrict__ dx, int64_t n8, int C, int pitch,
                                                               const float* __restrict__ save, const float* __restrict__ coef,
                                                               int relu) {
    const int64_t i = (int64_t)blockIdx.x * BN_THREADS + threadIdx.x;
    if (i >= n8) return;
    const int c0 = (int)(i % (pitch / 8)) * 8;
    float v[8], d[8], r[8];
    unpack8(x[i], v);
    unpack8(dy[i], d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int c = c0 + j;
        if (c >= C) {
            r[j] = 0.f;
            continue;
        }
        const float g = (!relu || v[j] * save[2 * C + c] + save[3 * C + c] > 0.f) ? d[j] : 0.f;
        const float xh = (v[j] - save[c]) * save[C + c];
        r[j] = coef[c] * (g - coef[C + c] - xh * coef[2 * C + c]);
    }
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = pack_bf16x2(r[2 * j], r[2 * j + 1]);
    dx[i] = o;
}

int bn_blocks(int64_t M) {  // ~32+ rows per workgroup, at most 256 workgroups (one per CU)
    const int64_t nb = (M + 31) / 32;
    return (int)(nb < 256 ? nb : 256);
}

bool bn_args_ok(const void* x, int64_t M, int C, int pitch) {
    return x && M > 0 && C > 0 && pitch >= C && pitch % 8 == 0 && pitch / 8 <= BN_THREADS && ((uintptr_t)x & 15) == 0;
}

}  // namespace

extern "C" int64_t mmt_batchnorm_ws_floats(int64_t M, int C) { return (int64_t)bn_blocks(M) * 2 * C + 3 * (int64_t)C; }

extern "C" int mmt_batchnorm_relu(const void* x, void* y, int64_t M, int C, int pitch, const float* gamma, const float* beta,
                                  float* running_mean, float* running_var, float momentum, float eps, int training,
                                  int relu, float* save, float* ws, int64_t ws_floats, void* stream) {
    if (!bn_args_ok(x, M, C, pitch) || !y || ((uintptr_t)y & 15) || !save) return MMT_EBADARG;
    if (!training && (!running_mean || !running_var)) return MMT_EBADARG;
    if ((running_mean == nullptr) != (running_var == nullptr)) return MMT_EBADARG;
    const int nb = bn_blocks(M);
    if (training && (!ws || ws_floats < (int64_t)nb * 2 * C)) return MMT_EBADARG;
    hipStream_t st = (hipStream_t)stream;
    if (training)
        hipLaunchKernelGGL(bn_stats_kernel, dim3(nb), dim3(BN_THREADS), 0, st, (const u32x4*)x, M, C, pitch, ws);
    hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + BN_FCH - 1) / BN_FCH), dim3(BN_THREADS), 0, st, (const u32x4*)x, (const float*)ws, nb, M, C,
                       gamma, beta, running_mean, running_var, momentum, eps, training, save);
    const int64_t n8 = M * (pitch / 8);
    hipLaunchKernelGGL(bn_apply_kernel, dim3((unsigned)((n8 + BN_THREADS - 1) / BN_THREADS)), dim3(BN_THREADS), 0, st,
                       (const u32x4*)x, (u32x4*)y, n8, C, pitch, (const float*)save, relu);
    return launch_status();
}

extern "C" int mmt_batchnorm_relu_bwd(const void* x, const void* dy, void* dx, int64_t M, int C, int pitch, const float* gamma,
                                      const float* save, int training, int relu, float* dgb, float* ws, int64_t ws_floats,
                                      void* stream) {
    if (!bn_args_ok(x, M, C, pitch) || !dy || !dx || ((uintptr_t)dy & 15) || ((uintptr_t)dx & 15) || !save || !dgb) return MMT_EBADARG;
    const int nb = bn_blocks(M);
    if (!ws || ws_floats < mmt_batchnorm_ws_floats(M, C)) return MMT_EBADARG;
    hipStream_t st = (hipStream_t)stream;
    float* coef = ws + (int64_t)nb * 2 * C;
    hipLaunchKernelGGL(bn_bwd_stats_kernel, dim3(nb), dim3(BN_THREADS), 0, st, (const u32x4*)x, (const u32x4*)dy, M, C,
                       pitch, save, relu, ws);
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + BN_FCH - 1) / BN_FCH), dim3(BN_THREADS), 0, st, (const float*)ws, nb, M, C, gamma, save,
                       training, dgb, coef);
    const int64_t n8 = M * (pitch / 8);
    hipLaunchKernelGGL(bn_bwd_dx_kernel, dim3((unsigned)((n8 + BN_THREADS - 1) / BN_THREADS)), dim3(BN_THREADS), 0, st,
                       (const u32x4*)x, (const u32x4*)dy, (u32x4*)dx, n8, C, pitch, save, (const float*)coef, relu);
    return launch_status();
}
