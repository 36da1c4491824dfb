// Corner-head tail, PrRoIPool and score-decoder attention for gfx950.
//   mmt_conv3x3_c1         the Cout=1 conv-BN-ReLU closing adjust3_* / adjust4_* (head.py:115-120),
//                          BN folded into (w, bias) on the host
//   mmt_corner_softargmax  conv5_* (1x1, 48->1) + F.interpolate(adjust3, x4) + F.interpolate(adjust4,
//                          x2) (head.py:191-192), softmax over the 80x80 map and the expectation of the
//                          coordinate grids (head.py:138-145, 200-212), /img_sz, box_xyxy_to_cxcywh
//                          (lib/utils/box_ops.py:27-32); one workgroup per frame, both corners
//   mmt_corner_score_train / _bwd  the training step's conv5 + pyramid adds of one branch and their backward
//   mmt_prroi_pool_forward PrRoIPoolingForward (prroi_pooling_gpu_impl.cu:149-212) with explicit
//                          feature strides so the channels-last fusion output is pooled in place
//   mmt_spm_attention      ScoreDecoder single-query multi-head attention (score_decoder.py:55-61)
#include "common.hpp"

namespace {

// 8 lanes per output pixel, each summing a strided slice of the 9*cin/EPC 16-byte chunks.
// (the body of one 32-pixel block bx; the pair kernel runs two convolutions' blocks in one grid)
template <typename T>
MMT_DEV void conv3x3_c1_block(const T* __restrict__ in, const T* __restrict__ w, const float* __restrict__ bias,
                              float* __restrict__ out, int B, int h, int cin, int64_t in_stride, int bx) {
    constexpr int EPC = 16 / (int)sizeof(T);
    const int g = blockIdx.y;
    const int64_t npx = (int64_t)B * h * h;
    const int64_t idx = (int64_t)bx * 32 + (threadIdx.x >> 3);
    const int sl = threadIdx.x & 7;
    const int nch = cin / EPC;
    float acc = 0.f;
    if (idx < npx) {
        const int b = idx / (h * h), rem = idx % (h * h), y = rem / h, x = rem % h;
        const T* ib = in + (int64_t)g * npx * in_stride + (int64_t)b * h * h * in_stride;
        const T* wg = w + (int64_t)g * 9 * cin;
        // (tap, chunk) advance incrementally (no per-iteration division) and the body is branch-free
        // (clamped pixel, zeroed value) so the unrolled iterations' loads issue together
        int tap = sl / nch, cc = sl - tap * nch;
#pragma unroll 4
        for (int u = sl; u < 9 * nch; u += 8) {
            const int ty = (tap * 11) >> 5;  // tap / 3 for tap < 9
            const int iy = y + ty - 1, ix = x + (tap - 3 * ty) - 1;
            const bool ok = iy >= 0 && iy < h && ix >= 0 && ix < h;
            const int cy = min(max(iy, 0), h - 1), cx = min(max(ix, 0), h - 1);
            uint4 xv = *(const uint4*)(ib + ((int64_t)cy * h + cx) * in_stride + cc * EPC);
            const uint4 wv = *(const uint4*)(wg + tap * cin + cc * EPC);
            if (!ok) xv = uint4{0u, 0u, 0u, 0u};
            for (cc += 8; cc >= nch; cc -= nch) ++tap;
            if constexpr (sizeof(T) == 2) {
                const uint32_t xa[4] = {xv.x, xv.y, xv.z, xv.w}, wa[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const f32x2 xj = unpack2<T>(xa[j]), wj = unpack2<T>(wa[j]);
                    acc += xj[0] * wj[0];
                    acc += xj[1] * wj[1];
                }
            } else {
                const f32x4 xf = __builtin_bit_cast(f32x4, xv), wf = __builtin_bit_cast(f32x4, wv);
                acc += xf[0] * wf[0] + xf[1] * wf[1] + xf[2] * wf[2] + xf[3] * wf[3];
            }
        }
    }
    acc += __shfl_xor(acc, 1, 64);
    acc += __shfl_xor(acc, 2, 64);
    acc += __shfl_xor(acc, 4, 64);
    if (idx < npx && sl == 0) out[(int64_t)g * npx + idx] = fmaxf(acc + bias[g], 0.f);
}

template <typename T>
__global__ __launch_bounds__(256) void conv3x3_c1_kernel(const T* __restrict__ in, const T* __restrict__ w,
                                                         const float* __restrict__ bias, float* __restrict__ out, int B,
                                                         int h, int cin, int64_t in_stride) {
    conv3x3_c1_block<T>(in, w, bias, out, B, h, cin, in_stride, blockIdx.x);
}

// Two independent Cout=1 convolutions (adjust3[2] and adjust4[1], head.py:115-120) in one launch:
// blocks [0, nb0) take the first, the rest the second.
template <typename T>
__global__ __launch_bounds__(256) void conv3x3_c1_pair_kernel(const T* __restrict__ in0, const T* __restrict__ w0,
                                                              const float* __restrict__ b0, float* __restrict__ out0,
                                                              int h0, int64_t st0, const T* __restrict__ in1,
                                                              const T* __restrict__ w1, const float* __restrict__ b1,
                                                              float* __restrict__ out1, int h1, int64_t st1, int B,
                                                              int cin, int nb0) {
    if ((int)blockIdx.x < nb0) conv3x3_c1_block<T>(in0, w0, b0, out0, B, h0, cin, st0, blockIdx.x);
    else conv3x3_c1_block<T>(in1, w1, b1, out1, B, h1, cin, st1, blockIdx.x - nb0);
}

// score(p) for both corners: conv5 (1x1, c4 -> 1) + up4(adjust3) + up2(adjust4); one thread per pixel.
template <typename T>
__global__ __launch_bounds__(256) void corner_score_kernel(const T* __restrict__ x4, const float* __restrict__ w5,
                                                           const float* __restrict__ b5, const float* __restrict__ a3,
                                                           const float* __restrict__ a4, float* __restrict__ maps, int B,
                                                           int fh, int c4) {
    constexpr int EPC = 16 / (int)sizeof(T);
    const int g = blockIdx.y;
    const int np = fh * fh, f4 = fh / 4, f2 = fh / 2;
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (int64_t)B * np) return;
    const int b = idx / np, p = idx % np, y = p / fh, x = p % fh;
    const T* px = x4 + ((int64_t)g * B * np + idx) * c4;
    const float* wg = w5 + g * c4;
    float s = 0.f;
    for (int cc = 0; cc < c4; cc += EPC) {
        const uint4 v = *(const uint4*)(px + cc);
        if constexpr (sizeof(T) == 2) {
            const uint32_t va[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const f32x2 vj = unpack2<T>(va[j]);
                s += vj[0] * wg[cc + 2 * j];
                s += vj[1] * wg[cc + 2 * j + 1];
            }
        } else {
            const f32x4 f = __builtin_bit_cast(f32x4, v);
            s += f[0] * wg[cc] + f[1] * wg[cc + 1] + f[2] * wg[cc + 2] + f[3] * wg[cc + 3];
        }
    }
    s = (s + b5[g]) + a3[((int64_t)g * B + b) * f4 * f4 + (y / 4) * f4 + x / 4] +
        a4[((int64_t)g * B + b) * f2 * f2 + (y / 2) * f2 + x / 2];
    maps[((int64_t)g * B + b) * np + p] = s;
}

// ---- training (train.py _HipCornerScore): one corner branch's score map with autograd's backward.
// sm[b][p] = (x4[b][p] . w5 + b5) + a3[b][up4(p)] + a4[b][up2(p)]  (head.py:191-192: conv5 1x1 48 -> 1 in fp32,
// nearest-upsampled adjust3 / adjust4 maps); x4 bf16 NHWC rows [B][fh*fh][c4]; a3 / a4 bf16 1-channel maps at
// pixel strides s3 / s4 (the 8-channel rows the HIP BatchNorm writes).  Replaces aten's fp32 F.linear through
// hipBLASLt (~175 us a launch for 10 MFLOP), two nearest upsamplings and two adds, and their backward.
__global__ __launch_bounds__(256) void corner_score_train_kernel(const bf16_t* __restrict__ x4, const float* __restrict__ w5,
                                                                 const float* __restrict__ b5, const bf16_t* __restrict__ a3,
                                                                 int64_t s3, const bf16_t* __restrict__ a4, int64_t s4,
                                                                 float* __restrict__ out, int B, int fh, int c4) {
    const int np = fh * fh, f4 = fh / 4, f2 = fh / 2;
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (int64_t)B * np) return;
    const int b = idx / np, p = idx % np, y = p / fh, x = p % fh;
    const bf16_t* px = x4 + idx * c4;
    float s = 0.f;
    for (int cc = 0; cc < c4; cc += 8) {
        const uint4 v = *(const uint4*)(px + cc);
        const uint32_t va[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const f32x2 vj = unpack2<bf16_t>(va[j]);
            s += vj[0] * w5[cc + 2 * j];
            s += vj[1] * w5[cc + 2 * j + 1];
        }
    }
    s = (s + b5[0]) + bf2f(a3[((int64_t)b * f4 * f4 + (y / 4) * f4 + x / 4) * s3]) +
        bf2f(a4[((int64_t)b * f2 * f2 + (y / 2) * f2 + x / 2) * s4]);
    out[idx] = s;
}

// Backward of one branch: one workgroup per 4-row band of one map (fh threads per row, 4 rows): dx4[p][c] =
// bf16(dsm[p] w5[c]); da3 (the band's fh/4 outputs, each the sum of its 4x4 dsm block) and da4 (2 rows of fh/2,
// each a 2x2 sum), bf16 like the maps (contiguous [..][1]); the band's dw5 / db5 partial sums, in a fixed order
// (pixels of the band in 6 interleaved groups per channel, then the groups in order) into part[band][c4 + 1]:
// deterministic, no atomics.  corner_score_train_fin_kernel sums the bands in order.
__global__ __launch_bounds__(512) void corner_score_train_bwd_kernel(const float* __restrict__ dsm, const bf16_t* __restrict__ x4,
                                                                     const float* __restrict__ w5, bf16_t* __restrict__ dx4,
                                                                     bf16_t* __restrict__ da3, int p3, bf16_t* __restrict__ da4,
                                                                     int p4, float* __restrict__ part, int B, int fh, int c4) {
    __shared__ float sd[4 * 128];       // the band's dsm (fh <= 128)
    __shared__ float red[8][64 + 1];    // per-group partial sums of each channel (c4 <= 64) and the bias
    const int np = fh * fh, bands = fh / 4, band = blockIdx.x;
    const int b = band / bands, r0 = (band % bands) * 4;
    const int nbp = 4 * fh;  // pixels of the band
    const int64_t p0 = (int64_t)b * np + (int64_t)r0 * fh;
    for (int t = threadIdx.x; t < nbp; t += blockDim.x) sd[t] = dsm[p0 + t];
    __syncthreads();
    // dx4: thread per (pixel, 8-channel chunk)
    const int nchunk = c4 / 8;
    for (int t = threadIdx.x; t < nbp * nchunk; t += blockDim.x) {
        const int pp = t / nchunk, ck = t - pp * nchunk;
        const float d = sd[pp];
        uint32_t o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = pack_bf16x2(d * w5[ck * 8 + 2 * j], d * w5[ck * 8 + 2 * j + 1]);
        *(uint4*)(dx4 + (p0 + pp) * c4 + ck * 8) = uint4{o[0], o[1], o[2], o[3]};
    }
    // dw5 / db5 partials: channel c (c < c4) or the bias (c == c4) over pixel group gi (pixels gi, gi + 8, ...)
    for (int t = threadIdx.x; t < 8 * (c4 + 1); t += blockDim.x) {
        const int c = t % (c4 + 1), gi = t / (c4 + 1);
        float acc = 0.f;
        for (int pp = gi; pp < nbp; pp += 8) acc += c < c4 ? sd[pp] * bf2f(x4[(p0 + pp) * c4 + c]) : sd[pp];
        red[gi][c] = acc;
    }
    // da3: fh / 4 outputs of this band; da4: 2 rows of fh / 2
    const int f4 = fh / 4, f2 = fh / 2;
    for (int t = threadIdx.x; t < f4 + 2 * f2; t += blockDim.x) {
        if (t < f4) {
            float acc = 0.f;
#pragma unroll
            for (int dy = 0; dy < 4; ++dy)
#pragma unroll
                for (int dx = 0; dx < 4; ++dx) acc += sd[dy * fh + 4 * t + dx];
            bf16_t* o = da3 + ((int64_t)b * f4 * f4 + (r0 / 4) * f4 + t) * p3;  // channel 0, padding channels 0
            o[0] = f2bf(acc);
            for (int j = 1; j < p3; ++j) o[j] = 0;
        } else {
            const int u = t - f4, ry = u / f2, cx = u - ry * f2;
            float acc = 0.f;
#pragma unroll
            for (int dy = 0; dy < 2; ++dy)
#pragma unroll
                for (int dx = 0; dx < 2; ++dx) acc += sd[(2 * ry + dy) * fh + 2 * cx + dx];
            bf16_t* o = da4 + ((int64_t)b * f2 * f2 + (r0 / 2 + ry) * f2 + cx) * p4;
            o[0] = f2bf(acc);
            for (int j = 1; j < p4; ++j) o[j] = 0;
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c <= c4; c += blockDim.x) {
        float acc = 0.f;
#pragma unroll
        for (int gi = 0; gi < 8; ++gi) acc += red[gi][c];
        part[(int64_t)band * (c4 + 1) + c] = acc;
    }
}

// dw5[c] = sum over the bands of part[band][c]; db5 = the same for column c4.  16 band groups (bands g, g + 16, ...)
// summed in parallel, then the groups in order: a fixed order (round 6: one thread per channel walked all bands,
// 75 us at 16 pairs)
__global__ __launch_bounds__(1024) void corner_score_train_fin_kernel(const float* __restrict__ part, float* __restrict__ dw5,
                                                                     float* __restrict__ db5, int nbands, int c4) {
    __shared__ float red[16][65];
    const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
    float acc = 0.f;
    if (c <= c4)
        for (int i = g; i < nbands; i += 16) acc += part[(int64_t)i * (c4 + 1) + c];
    red[g][c] = acc;
    __syncthreads();
    if (g == 0 && c <= c4) {
        float t = 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) t += red[j][c];
        if (c < c4) dw5[c] = t;
        else db5[0] = t;
    }
}

// softmax over each fh x fh map + expectation of the coordinate grids; one workgroup per frame.
// One 1024-thread block per frame handles both corner maps.  All map reads are issued up front
// (independent, unrolled: SA_PER per thread per map) so the kernel pays one memory round trip, not
// one per strided-loop iteration (the 256-thread loop version took ~20 us at batch 1).
constexpr int SA_NT = 1024;  // fh*fh <= SA_NT*SA_PER: SA_PER 8 for 80x80 (320/4), 16 for 96x96 (384/4)
template <int SA_PER>
__global__ __launch_bounds__(SA_NT) void softargmax_kernel(const float* __restrict__ maps, float* __restrict__ cxcywh,
                                                           float* __restrict__ xyxy, float* __restrict__ rois,
                                                           float roi_scale, int B, int fh, int stride) {
    __shared__ float red[2][3][SA_NT / 64];
    __shared__ float mred[2][SA_NT / 64];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int np = fh * fh;
    float v[2][SA_PER];
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        const float* m = maps + ((int64_t)g * B + b) * np;
#pragma unroll
        for (int i = 0; i < SA_PER; ++i) {
            const int p = tid + SA_NT * i;
            v[g][i] = m[min(p, np - 1)];  // clamped read, masked below
        }
    }
    float mx[2];
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        float t = -INFINITY;
#pragma unroll
        for (int i = 0; i < SA_PER; ++i)
            if (tid + SA_NT * i < np) t = fmaxf(t, v[g][i]);
        t = wave_max(t);
        if (lane == 0) mred[g][w] = t;
    }
    __syncthreads();
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        float t = mred[g][0];
#pragma unroll
        for (int i = 1; i < SA_NT / 64; ++i) t = fmaxf(t, mred[g][i]);
        mx[g] = t;
    }
    // grid coordinates of this thread's pixels, stepped by SA_NT without a division per pixel
    int px[SA_PER], py[SA_PER];
    {
        const int dq = SA_NT / fh, dr = SA_NT - dq * fh;
        int y = tid / fh, x = tid - y * fh;
#pragma unroll
        for (int i = 0; i < SA_PER; ++i) {
            px[i] = x;
            py[i] = y;
            x += dr;
            y += dq;
            if (x >= fh) x -= fh, ++y;
        }
    }
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        float se = 0.f, sx = 0.f, sy = 0.f;
#pragma unroll
        for (int i = 0; i < SA_PER; ++i) {
            const int p = tid + SA_NT * i;
            if (p < np) {
                const float e = expf(v[g][i] - mx[g]);
                se += e;
                sx += e * (float)(stride * px[i]);
                sy += e * (float)(stride * py[i]);
            }
        }
        se = wave_sum(se);
        sx = wave_sum(sx);
        sy = wave_sum(sy);
        if (lane == 0) {
            red[g][0][w] = se;
            red[g][1][w] = sx;
            red[g][2][w] = sy;
        }
    }
    __syncthreads();
    if (tid == 0) {
        float res[4];
        const float img = (float)(fh * stride);
        for (int g = 0; g < 2; ++g) {
            float se = 0.f, sx = 0.f, sy = 0.f;
            for (int i = 0; i < SA_NT / 64; ++i) {
                se += red[g][0][i];
                sx += red[g][1][i];
                sy += red[g][2][i];
            }
            res[2 * g] = (sx / se) / img;
            res[2 * g + 1] = (sy / se) / img;
        }
        if (xyxy) {
            xyxy[b * 4 + 0] = res[0]; xyxy[b * 4 + 1] = res[1];
            xyxy[b * 4 + 2] = res[2]; xyxy[b * 4 + 3] = res[3];
        }
        const float cx = (res[0] + res[2]) / 2, cy = (res[1] + res[3]) / 2;
        const float w = res[2] - res[0], h = res[3] - res[1];
        cxcywh[b * 4 + 0] = cx;
        cxcywh[b * 4 + 1] = cy;
        cxcywh[b * 4 + 2] = w;
        cxcywh[b * 4 + 3] = h;
        if (rois) {  // box_cxcywh_to_xyxy(coord) * feature size, with the batch index
            rois[b * 5 + 0] = (float)b;
            rois[b * 5 + 1] = (cx - 0.5f * w) * roi_scale;
            rois[b * 5 + 2] = (cy - 0.5f * h) * roi_scale;
            rois[b * 5 + 3] = (cx + 0.5f * w) * roi_scale;
            rois[b * 5 + 4] = (cy + 0.5f * h) * roi_scale;
        }
    }
}

MMT_DEV float prroi_get(const float* d, int h, int w, int H, int W, int64_t sh, int64_t sw) {
    return (h < 0 || w < 0 || h >= H || w >= W) ? 0.f : d[h * sh + w * sw];
}
MMT_DEV float prroi_term(float a, float b, float la, float lb) {
    return (la - 0.5f * la * la - a + 0.5f * a * a) * (lb - 0.5f * lb * lb - b + 0.5f * b * b);
}
// PrRoIPoolingMatCalculation, prroi_pooling_gpu_impl.cu:71-106
MMT_DEV float prroi_mat(const float* d, int s_h, int s_w, int e_h, int e_w, float y0, float x0, float y1, float x1,
                        int H, int W, int64_t sh, int64_t sw) {
    float sum = 0.f;
    float alpha = x0 - (float)s_w, beta = y0 - (float)s_h, la = x1 - (float)s_w, lb = y1 - (float)s_h;
    sum += prroi_get(d, s_h, s_w, H, W, sh, sw) * prroi_term(alpha, beta, la, lb);
    alpha = (float)e_w - x1;
    la = (float)e_w - x0;
    sum += prroi_get(d, s_h, e_w, H, W, sh, sw) * prroi_term(alpha, beta, la, lb);
    alpha = x0 - (float)s_w;
    beta = (float)e_h - y1;
    la = x1 - (float)s_w;
    lb = (float)e_h - y0;
    sum += prroi_get(d, e_h, s_w, H, W, sh, sw) * prroi_term(alpha, beta, la, lb);
    alpha = (float)e_w - x1;
    la = (float)e_w - x0;
    sum += prroi_get(d, e_h, e_w, H, W, sh, sw) * prroi_term(alpha, beta, la, lb);
    return sum;
}

__global__ __launch_bounds__(256) void prroi_kernel(const float* __restrict__ feat, const float* __restrict__ rois,
                                                    float* __restrict__ out, int R, int C, int H, int W, int64_t s_b,
                                                    int64_t s_c, int64_t s_h, int64_t s_w, int PH, int PW, float scale,
                                                    int64_t o_r, int64_t o_c, int64_t o_p) {
    const int64_t total = (int64_t)R * C * PH * PW;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const int pw = idx % PW, ph = (idx / PW) % PH;
    const int c = (idx / PW / PH) % C;
    const int n = idx / PW / PH / C;
    const float* roi = rois + n * 5;
    const int bi = (int)roi[0];
    const float x0 = roi[1] * scale, y0 = roi[2] * scale, x1 = roi[3] * scale, y1 = roi[4] * scale;
    const float rw = fmaxf(x1 - x0, 0.f), rh = fmaxf(y1 - y0, 0.f);
    const float bh = rh / (float)PH, bw = rw / (float)PW;
    const float* d = feat + bi * s_b + c * s_c;
    const float ws = x0 + bw * pw, hs = y0 + bh * ph;
    const float we = ws + bw, he = hs + bh;
    const float win = fmaxf(0.f, bw * bh);
    float* dst = out + (int64_t)n * o_r + (int64_t)c * o_c + (int64_t)(ph * PW + pw) * o_p;
    if (win == 0.f) {
        *dst = 0.f;
        return;
    }
    const int sw_ = (int)floorf(ws), ew = (int)ceilf(we), sh_ = (int)floorf(hs), eh = (int)ceilf(he);
    float sum = 0.f;
    for (int wi = sw_; wi < ew; ++wi)
        for (int hi = sh_; hi < eh; ++hi)
            sum += prroi_mat(d, hi, wi, hi + 1, wi + 1, fmaxf(hs, (float)hi), fmaxf(ws, (float)wi),
                             fminf(he, (float)hi + 1.f), fminf(we, (float)(wi + 1)), H, W, s_h, s_w);
    *dst = sum / win;
}

// ---- PrRoIPool backward (prroi_pooling_gpu_impl.cu:214-378), contiguous NCHW features, (R,5) rois.
// PrRoIPoolingDistributeDiff / MatDistributeDiff (:108-147): the four corner terms of one cell,
// each an atomic add of top_diff * coeff where the tap lies inside the map.
MMT_DEV void prroi_dist(float* g, float v, int h, int w, int H, int W) {
    if (h >= 0 && w >= 0 && h < H && w < W) atomicAdd(g + (int64_t)h * W + w, v);
}
MMT_DEV void prroi_mat_dist(float* g, float top, int s_h, int s_w, int e_h, int e_w, float y0, float x0, float y1,
                            float x1, int H, int W) {
    float alpha = x0 - (float)s_w, beta = y0 - (float)s_h, la = x1 - (float)s_w, lb = y1 - (float)s_h;
    prroi_dist(g, top * prroi_term(alpha, beta, la, lb), s_h, s_w, H, W);
    alpha = (float)e_w - x1;
    la = (float)e_w - x0;
    prroi_dist(g, top * prroi_term(alpha, beta, la, lb), s_h, e_w, H, W);
    alpha = x0 - (float)s_w;
    beta = (float)e_h - y1;
    la = x1 - (float)s_w;
    lb = (float)e_h - y0;
    prroi_dist(g, top * prroi_term(alpha, beta, la, lb), e_h, s_w, H, W);
    alpha = (float)e_w - x1;
    la = (float)e_w - x0;
    prroi_dist(g, top * prroi_term(alpha, beta, la, lb), e_h, e_w, H, W);
}

// PrRoIPoolingBackward (:214-270): one thread per pooled element (n, c, ph, pw)
__global__ __launch_bounds__(256) void prroi_bwd_kernel(const float* __restrict__ rois, const float* __restrict__ gout,
                                                        float* __restrict__ gfeat, int R, int C, int H, int W, int PH,
                                                        int PW, float scale) {
    const int64_t total = (int64_t)R * C * PH * PW;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const int pw = idx % PW, ph = (idx / PW) % PH;
    const int c = (idx / PW / PH) % C;
    const int n = idx / PW / PH / C;
    const float* roi = rois + n * 5;
    const int bi = (int)roi[0];
    const float x0 = roi[1] * scale, y0 = roi[2] * scale, x1 = roi[3] * scale, y1 = roi[4] * scale;
    const float bh = fmaxf(y1 - y0, 0.f) / (float)PH, bw = fmaxf(x1 - x0, 0.f) / (float)PW;
    const float ws = x0 + bw * pw, hs = y0 + bh * ph, we = ws + bw, he = hs + bh;
    const float win = fmaxf(0.f, bw * bh);
    const float top = win == 0.f ? 0.f : gout[idx] / win;
    float* g = gfeat + ((int64_t)bi * C + c) * H * W;
    const int sw_ = (int)floorf(ws), ew = (int)ceilf(we), sh_ = (int)floorf(hs), eh = (int)ceilf(he);
    for (int wi = sw_; wi < ew; ++wi)
        for (int hi = sh_; hi < eh; ++hi)
            prroi_mat_dist(g, top, hi, wi, hi + 1, wi + 1, fmaxf(hs, (float)hi), fmaxf(ws, (float)wi),
                           fminf(he, (float)hi + 1.f), fminf(we, (float)(wi + 1)), H, W);
}

// PrRoIPoolingInterpolation / SingleCoorIntegral (:44-69)
MMT_DEV float prroi_interp(const float* d, float h, float w, int H, int W) {
    const int h1 = (int)floorf(h), w1 = (int)floorf(w);
    float r = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int hh = h1 + (k & 1), ww = w1 + (k >> 1);
        const float v = (hh < 0 || ww < 0 || hh >= H || ww >= W) ? 0.f : d[(int64_t)hh * W + ww];
        r += v * (1.f - fabsf(h - (float)hh)) * (1.f - fabsf(w - (float)ww));
    }
    return r;
}
MMT_DEV float prroi_coor_int(float s, float t, float c1, float c2) {
    return 0.5f * (t * t - s * s) * c2 + (t - 0.5f * t * t - s + 0.5f * s * s) * c1;
}

// PrRoIPoolingCoorBackward (:272-378): one workgroup per ROI sums the (c, ph, pw) contributions
// in registers + LDS and stores the 5 coordinate gradients once (the reference adds them with
// 4 atomics per pooled element into the same 4 words).
__global__ __launch_bounds__(256) void prroi_coor_bwd_kernel(const float* __restrict__ feat, const float* __restrict__ rois,
                                                             const float* __restrict__ out, const float* __restrict__ gout,
                                                             float* __restrict__ groi, int C, int H, int W, int PH, int PW,
                                                             float scale) {
    __shared__ float red[4][4];
    const int n = blockIdx.x, tid = threadIdx.x;
    const float* roi = rois + n * 5;
    const int bi = (int)roi[0];
    const float x0 = roi[1] * scale, y0 = roi[2] * scale, x1 = roi[3] * scale, y1 = roi[4] * scale;
    const float bh = fmaxf(y1 - y0, 0.f) / (float)PH, bw = fmaxf(x1 - x0, 0.f) / (float)PW;
    const float win = fmaxf(0.f, bw * bh);
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    const int per = C * PH * PW;
    for (int e = tid; e < per; e += 256) {
        const int pw = e % PW, ph = (e / PW) % PH, c = e / (PW * PH);
        const int64_t idx = (int64_t)n * per + e;
        const float go = gout[idx];
        const float sum_out = win == 0.f ? 0.f : go / win;
        if (sum_out == 0.f) continue;  // the reference's early return (:318)
        const float ws = x0 + bw * pw, hs = y0 + bh * ph, we = ws + bw, he = hs + bh;
        const float* d = feat + ((int64_t)bi * C + c) * H * W;
        const int sw_ = (int)floorf(ws), ew = (int)ceilf(we), sh_ = (int)floorf(hs), eh = (int)ceilf(he);
        float gx1 = 0.f, gx2 = 0.f, gy1 = 0.f, gy2 = 0.f;
        for (int hi = sh_; hi < eh; ++hi) {
            const float a = fmaxf(hs, (float)hi) - hi, b = fminf(he, (float)(hi + 1)) - hi;
            gx1 += prroi_coor_int(a, b, prroi_interp(d, hi, ws, H, W), prroi_interp(d, hi + 1, ws, H, W));
            gx2 += prroi_coor_int(a, b, prroi_interp(d, hi, we, H, W), prroi_interp(d, hi + 1, we, H, W));
        }
        for (int wi = sw_; wi < ew; ++wi) {
            const float a = fmaxf(ws, (float)wi) - wi, b = fminf(we, (float)(wi + 1)) - wi;
            gy1 += prroi_coor_int(a, b, prroi_interp(d, hs, wi, H, W), prroi_interp(d, hs, wi + 1, H, W));
            gy2 += prroi_coor_int(a, b, prroi_interp(d, he, wi, H, W), prroi_interp(d, he, wi + 1, H, W));
        }
        const float top = out[idx];
        const float px1 = (-gx1 + (he - hs) * top) / win * scale, py1 = (-gy1 + (we - ws) * top) / win * scale;
        const float px2 = (gx2 - (he - hs) * top) / win * scale, py2 = (gy2 - (we - ws) * top) / win * scale;
        acc[0] += (px1 * (1.f - (float)pw / PW) + px2 * (1.f - (float)(pw + 1) / PW)) * go;
        acc[1] += (py1 * (1.f - (float)ph / PH) + py2 * (1.f - (float)(ph + 1) / PH)) * go;
        acc[2] += (px2 * (float)(pw + 1) / PW + px1 * (float)pw / PW) * go;
        acc[3] += (py2 * (float)(ph + 1) / PH + py1 * (float)ph / PH) * go;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float v = wave_sum(acc[k]);
        if ((tid & 63) == 0) red[k][tid >> 6] = v;
    }
    __syncthreads();
    if (tid == 0) {
        groi[n * 5] = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) groi[n * 5 + 1 + k] = red[k][0] + red[k][1] + red[k][2] + red[k][3];
    }
}

// ScoreDecoder single-query attention (score_decoder.py:55-61): one 256-thread workgroup per (batch,
// head).  Scores: thread t takes keys t, t+256, .. (64-wide dot with the query in LDS, the key row by
// 16-B loads); softmax statistics by block reduction; output: lane = channel, the 4 waves take
// interleaved keys, partial sums combined through LDS.
constexpr int SPM_MAXK = 2048;  // keys (16 ROI tokens; 2 x 64 / 2 x 144 template tokens)
__global__ __launch_bounds__(256) void spm_attention_kernel(const float* __restrict__ q, int64_t q_stride,
                                                            const float* __restrict__ kv, float* __restrict__ out,
                                                            int Lk, int C, float scale) {
    __shared__ float sc[SPM_MAXK];  // Lk scores
    __shared__ __attribute__((aligned(16))) float qs[64];
    __shared__ float red[4];
    __shared__ float part[4][64];
    const int h = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid < 64) qs[tid] = q[b * q_stride + h * 64 + tid];
    __syncthreads();
    const float* kb = kv + (int64_t)b * Lk * 2 * C + h * 64;
    float mx = -INFINITY;
    for (int t = tid; t < Lk; t += 256) {
        const float* kr = kb + (int64_t)t * 2 * C;
        float acc = 0.f;
#pragma unroll
        for (int d = 0; d < 64; d += 4) {
            const float4 kv4 = *(const float4*)(kr + d);
            const float4 q4 = *(const float4*)(qs + d);
            acc = fmaf(q4.x, kv4.x, fmaf(q4.y, kv4.y, fmaf(q4.z, kv4.z, fmaf(q4.w, kv4.w, acc))));
        }
        acc *= scale;
        sc[t] = acc;
        mx = fmaxf(mx, acc);
    }
    mx = wave_max(mx);
    if (lane == 0) red[w] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    __syncthreads();
    float se = 0.f;
    for (int t = tid; t < Lk; t += 256) {
        const float e = expf(sc[t] - mx);
        sc[t] = e;
        se += e;
    }
    se = wave_sum(se);
    if (lane == 0) red[w] = se;
    __syncthreads();
    const float inv = 1.f / (red[0] + red[1] + red[2] + red[3]);
    float acc = 0.f;
    for (int t = w; t < Lk; t += 4) acc = fmaf(sc[t], kb[(int64_t)t * 2 * C + C + lane], acc);
    part[w][lane] = acc;
    __syncthreads();
    if (w == 0) out[(int64_t)b * C + h * 64 + lane] = (part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane]) * inv;
}

}  // namespace

extern "C" int mmt_conv3x3_c1(const void* in, const void* w, const float* bias, float* out, int G, int B, int h, int cin,
                              int64_t in_stride, int dtype, void* stream) {
    const int epc = dtype == MMT_BF16 || dtype == MMT_F16 ? 8 : 4;
    if (!in || !w || !bias || !out || G <= 0 || B <= 0 || h <= 0 || cin <= 0 || cin % epc || in_stride % epc)
        return MMT_EBADARG;
    const int64_t npx = (int64_t)B * h * h;
    dim3 grid((unsigned)((npx + 31) / 32), G);
    hipStream_t st = (hipStream_t)stream;
    if (dtype == MMT_BF16)
        hipLaunchKernelGGL(conv3x3_c1_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)in, (const bf16_t*)w, bias,
                           out, B, h, cin, in_stride);
    else if (dtype == MMT_F16)
        hipLaunchKernelGGL(conv3x3_c1_kernel<f16_t>, grid, dim3(256), 0, st, (const f16_t*)in, (const f16_t*)w, bias,
                           out, B, h, cin, in_stride);
    else if (dtype == MMT_F32)
        hipLaunchKernelGGL(conv3x3_c1_kernel<float>, grid, dim3(256), 0, st, (const float*)in, (const float*)w, bias,
                           out, B, h, cin, in_stride);
    else return MMT_EBADARG;
    return launch_status();
}

extern "C" int mmt_conv3x3_c1_pair(const void* in0, const void* w0, const float* b0, float* out0, int h0,
                                   int64_t in_stride0, const void* in1, const void* w1, const float* b1, float* out1,
                                   int h1, int64_t in_stride1, int G, int B, int cin, int dtype, void* stream) {
    const int epc = dtype == MMT_BF16 || dtype == MMT_F16 ? 8 : 4;
    if (!in0 || !w0 || !b0 || !out0 || !in1 || !w1 || !b1 || !out1 || G <= 0 || B <= 0 || h0 <= 0 || h1 <= 0 ||
        cin <= 0 || cin % epc || in_stride0 % epc || in_stride1 % epc)
        return MMT_EBADARG;
    const int64_t nb0 = ((int64_t)B * h0 * h0 + 31) / 32, nb1 = ((int64_t)B * h1 * h1 + 31) / 32;
    if (nb0 + nb1 > INT32_MAX) return MMT_EBADARG;
    const dim3 grid((unsigned)(nb0 + nb1), G);
    hipStream_t st = (hipStream_t)stream;
#define MMT_C1_PAIR(T)                                                                                          \
    hipLaunchKernelGGL(conv3x3_c1_pair_kernel<T>, grid, dim3(256), 0, st, (const T*)in0, (const T*)w0, b0, out0, h0, \
                       in_stride0, (const T*)in1, (const T*)w1, b1, out1, h1, in_stride1, B, cin, (int)nb0)
    if (dtype == MMT_BF16) MMT_C1_PAIR(bf16_t);
    else if (dtype == MMT_F16) MMT_C1_PAIR(f16_t);
    else if (dtype == MMT_F32) MMT_C1_PAIR(float);
    else return MMT_EBADARG;
#undef MMT_C1_PAIR
    return launch_status();
}

extern "C" int mmt_corner_softargmax(const void* x4, const float* w5, const float* b5, const float* a3, const float* a4,
                                     float* score_maps, float* boxes_cxcywh, float* boxes_xyxy, float* rois,
                                     float roi_scale, int B, int fh, int c4, int stride, int dtype, void* stream) {
    const int epc = dtype == MMT_BF16 || dtype == MMT_F16 ? 8 : 4;
    if (!x4 || !w5 || !b5 || !a3 || !a4 || !score_maps || !boxes_cxcywh || B <= 0 || fh <= 0 || fh % 4 || c4 <= 0 ||
        c4 % epc || fh * fh > SA_NT * 16)
        return MMT_EBADARG;
    hipStream_t st = (hipStream_t)stream;
    dim3 grid((unsigned)(((int64_t)B * fh * fh + 255) / 256), 2);
    if (dtype == MMT_BF16)
        hipLaunchKernelGGL(corner_score_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)x4, w5, b5, a3, a4,
                           score_maps, B, fh, c4);
    else if (dtype == MMT_F16)
        hipLaunchKernelGGL(corner_score_kernel<f16_t>, grid, dim3(256), 0, st, (const f16_t*)x4, w5, b5, a3, a4,
                           score_maps, B, fh, c4);
    else if (dtype == MMT_F32)
        hipLaunchKernelGGL(corner_score_kernel<float>, grid, dim3(256), 0, st, (const float*)x4, w5, b5, a3, a4,
                           score_maps, B, fh, c4);
    else return MMT_EBADARG;
    if (fh * fh <= SA_NT * 8)
        hipLaunchKernelGGL(softargmax_kernel<8>, dim3(B), dim3(SA_NT), 0, st, score_maps, boxes_cxcywh, boxes_xyxy,
                           rois, roi_scale, B, fh, stride);
    else
        hipLaunchKernelGGL(softargmax_kernel<16>, dim3(B), dim3(SA_NT), 0, st, score_maps, boxes_cxcywh, boxes_xyxy,
                           rois, roi_scale, B, fh, stride);
    return launch_status();
}

extern "C" int mmt_corner_score_train(const void* x4, const float* w5, const float* b5, const void* a3, int64_t s3,
                                      const void* a4, int64_t s4, float* score_map, int B, int fh, int c4, void* stream) {
    if (!x4 || !w5 || !b5 || !a3 || !a4 || !score_map || B <= 0 || fh <= 0 || fh % 4 || c4 <= 0 || c4 % 8 || s3 <= 0 ||
        s4 <= 0)
        return MMT_EBADARG;
    hipLaunchKernelGGL(corner_score_train_kernel, dim3((unsigned)(((int64_t)B * fh * fh + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, (const bf16_t*)x4, w5, b5, (const bf16_t*)a3, s3, (const bf16_t*)a4, s4,
                       score_map, B, fh, c4);
    return launch_status();
}

extern "C" int64_t mmt_corner_score_train_ws_floats(int B, int fh, int c4) {
    return (int64_t)B * (fh / 4) * (c4 + 1);
}

extern "C" int mmt_corner_score_train_bwd(const float* dsm, const void* x4, const float* w5, void* dx4, void* da3, int p3,
                                          void* da4, int p4, float* dw5, float* db5, float* ws, int B, int fh, int c4,
                                          void* stream) {
    if (!dsm || !x4 || !w5 || !dx4 || !da3 || !da4 || !dw5 || !db5 || !ws || B <= 0 || fh <= 0 || fh % 4 || fh > 128 ||
        c4 <= 0 || c4 % 8 || c4 > 63 || p3 < 1 || p3 > 8 || p4 < 1 || p4 > 8)
        return MMT_EBADARG;
    hipStream_t st = (hipStream_t)stream;
    const int nb = B * (fh / 4);
    hipLaunchKernelGGL(corner_score_train_bwd_kernel, dim3(nb), dim3(512), 0, st, dsm, (const bf16_t*)x4, w5, (bf16_t*)dx4,
                       (bf16_t*)da3, p3, (bf16_t*)da4, p4, ws, B, fh, c4);
    hipLaunchKernelGGL(corner_score_train_fin_kernel, dim3(1), dim3(1024), 0, st, ws, dw5, db5, nb, c4);
    return launch_status();
}

extern "C" int mmt_prroi_pool_forward(const float* features, const float* rois, float* out, int R, int C, int H, int W,
                                      int64_t s_b, int64_t s_c, int64_t s_h, int64_t s_w, int ph, int pw,
                                      float spatial_scale, int64_t o_r, int64_t o_c, int64_t o_p, void* stream) {
    if (!features || !rois || !out || R < 0 || C <= 0 || H <= 0 || W <= 0 || ph <= 0 || pw <= 0) return MMT_EBADARG;
    if (R == 0) return 0;
    const int64_t total = (int64_t)R * C * ph * pw;
    hipLaunchKernelGGL(prroi_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, features,
                       rois, out, R, C, H, W, s_b, s_c, s_h, s_w, ph, pw, spatial_scale, o_r, o_c, o_p);
    return launch_status();
}

extern "C" int mmt_prroi_pool_backward(const float* rois, const float* grad_out, float* grad_features, int B, int R,
                                       int C, int H, int W, int ph, int pw, float spatial_scale, void* stream) {
    if (!rois || !grad_out || !grad_features || B <= 0 || R < 0 || C <= 0 || H <= 0 || W <= 0 || ph <= 0 || pw <= 0)
        return MMT_EBADARG;
    hipStream_t st = (hipStream_t)stream;
    if (const int e = zero_fill_async(grad_features, sizeof(float) * (size_t)B * C * H * W, st)) return e;
    if (R == 0) return 0;
    const int64_t total = (int64_t)R * C * ph * pw;
    hipLaunchKernelGGL(prroi_bwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, rois, grad_out,
                       grad_features, R, C, H, W, ph, pw, spatial_scale);
    return launch_status();
}

extern "C" int mmt_prroi_pool_coor_backward(const float* features, const float* rois, const float* out,
                                            const float* grad_out, float* grad_rois, int R, int C, int H, int W, int ph,
                                            int pw, float spatial_scale, void* stream) {
    if (!features || !rois || !out || !grad_out || !grad_rois || R < 0 || C <= 0 || H <= 0 || W <= 0 || ph <= 0 ||
        pw <= 0)
        return MMT_EBADARG;
    if (R == 0) return 0;
    hipLaunchKernelGGL(prroi_coor_bwd_kernel, dim3((unsigned)R), dim3(256), 0, (hipStream_t)stream, features, rois, out,
                       grad_out, grad_rois, C, H, W, ph, pw, spatial_scale);
    return launch_status();
}

extern "C" int mmt_spm_attention(const float* q, int64_t q_stride, const float* kv, float* out, int B, int Lk, int C,
                                 int H, float scale, void* stream) {
    if (!q || !kv || !out || B <= 0 || Lk <= 0 || Lk > SPM_MAXK || C != H * 64) return MMT_EBADARG;
    if (((uintptr_t)kv & 15) || (C & 3) || ((uintptr_t)q & 3)) return MMT_EBADARG;
    hipLaunchKernelGGL(spm_attention_kernel, dim3(H, B), dim3(256), 0, (hipStream_t)stream, q, q_stride,
                       kv, out, Lk, C, scale);
    return launch_status();
}

extern "C" const char* mmt_version(void) { return "libmmt_hip 0.1 gfx950"; }
