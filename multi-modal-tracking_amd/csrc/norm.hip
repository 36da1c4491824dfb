// Normalisation / staging kernels (HBM-bound, one pass, vectorised 16-B accesses).
//   mmt_layernorm    nn.LayerNorm of the ViT blocks (eps 1e-6, mixformer.py:137-138; shared/asym
//                    per-modality norm1_v/_i, norm2_v/_i, mixformer_shared.py:149-157) and of the
//                    fusion encoder (eps 1e-5, deformable_encoder_lnspecific.py:153-155 with the
//                    src + output_proj residual fused in via a broadcast row map)
//   mmt_layernorm_bwd  its backward for the training step (dx, per-group dgamma / dbeta); _add: plus the
//                      input's second gradient (the block's residual add) in the same pass
//   mmt_groupnorm    nn.GroupNorm(32) after the fusion 1x1 convs (fusion_utils.py:252-268)
//   mmt_groupnorm_bwd  its backward for the training step (dx, dgamma / dbeta; channels-last)
//   mmt_add_cast     src + pos -> bf16 query staging (ms_deform_attn_bimodal.py:93-95)
//   mmt_patch_im2col PatchEmbed input staging for the patch GEMM (mixformer.py:29-34, :237-247)
#include "common.hpp"

namespace {

// One wave per row; C = 64 * 4 * V floats (V float4 per lane).
template <typename T, int V>
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ in, const float* __restrict__ add,
                                                        int64_t add_rows, float* out_f32, T* out_t, const float* g0,
                                                        const float* b0, const float* g1, const float* b1,
                                                        int64_t rows, int64_t rpg, float eps) {
    constexpr int C = 256 * V;
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const float4* x4 = (const float4*)(in + row * C);
    const float4* a4 = add ? (const float4*)(add + (row % add_rows) * C) : nullptr;
    // gamma / beta issued with the row (not after the two reductions: one memory round trip fewer)
    const bool second = g1 && ((row / rpg) & 1);  // groups alternate every rpg rows
    const float4* gg = (const float4*)(second ? g1 : g0);
    const float4* bb = (const float4*)(second ? b1 : b0);
    float4 ga[V], be[V];
#pragma unroll
    for (int i = 0; i < V; ++i) {
        ga[i] = gg[lane + 64 * i];
        be[i] = bb[lane + 64 * i];
    }
    float4 v[V];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < V; ++i) {
        v[i] = x4[lane + 64 * i];
        if (a4) {
            const float4 a = a4[lane + 64 * i];
            v[i].x += a.x; v[i].y += a.y; v[i].z += a.z; v[i].w += a.w;
        }
        s += v[i].x + v[i].y + v[i].z + v[i].w;
    }
    const float mean = wave_sum(s) * (1.f / C);
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < V; ++i) {
        const float dx = v[i].x - mean, dy = v[i].y - mean, dz = v[i].z - mean, dw = v[i].w - mean;
        q += dx * dx + dy * dy + dz * dz + dw * dw;
    }
    const float rstd = rsqrtf(wave_sum(q) * (1.f / C) + eps);
#pragma unroll
    for (int i = 0; i < V; ++i) {
        const int idx = lane + 64 * i;
        float4 y;
        y.x = (v[i].x - mean) * rstd * ga[i].x + be[i].x;
        y.y = (v[i].y - mean) * rstd * ga[i].y + be[i].y;
        y.z = (v[i].z - mean) * rstd * ga[i].z + be[i].z;
        y.w = (v[i].w - mean) * rstd * ga[i].w + be[i].w;
        if (out_f32) ((float4*)(out_f32 + row * C))[idx] = y;
        if (out_t) {
            if constexpr (sizeof(T) == 2) {
                uint2 pk;
                pk.x = pack2<T>(y.x, y.y);
                pk.y = pack2<T>(y.z, y.w);
                ((uint2*)(out_t + row * C))[idx] = pk;
            } else {
                ((float4*)(out_t + row * C))[idx] = y;
            }
        }
    }
}

// GroupNorm: one 512-thread workgroup per (instance, group); the group's values (P positions x cg
// channels, float4 granules) stay in registers, so the input is read once; two-pass statistics
// (mean, then mean of squared deviations) as torch computes them.
constexpr int GN_THREADS = 512, GN_VMAX = 12;

template <typename T>
__global__ __launch_bounds__(GN_THREADS) void groupnorm_kernel(const float* __restrict__ in, float* out_f32, T* out_t,
                                                               const float* g0, const float* b0, const float* g1,
                                                               const float* b1, int inst_per_set, int P, int Ctot,
                                                               int groups, float eps) {
    __shared__ float red[GN_THREADS / 64];
    __shared__ float gbs[2 * GN_THREADS];  // this group's gamma, beta (cg <= 512), read behind the reductions
    const int inst = blockIdx.y, grp = blockIdx.x;
    const int cg = Ctot / groups, q = cg / 4, items = P * q;
    const int64_t base = (int64_t)inst * P * Ctot + grp * cg;
    {  // issued before the input loads; block_sum's barriers publish them
        const bool second = g1 && inst >= inst_per_set;
        if ((int)threadIdx.x < cg) {
            gbs[threadIdx.x] = (second ? g1 : g0)[grp * cg + threadIdx.x];
            gbs[GN_THREADS + threadIdx.x] = (second ? b1 : b0)[grp * cg + threadIdx.x];
        }
    }
    // item -> (pixel, 4-channel chunk) without a runtime-divisor division per item: the float
    // quotient is exact (items < 2^24; (it + 0.5) / q sits >= 0.5 / q from an integer)
    const float inv_q = 1.f / (float)q;
    int pix[GN_VMAX], c4s[GN_VMAX];
#pragma unroll
    for (int i = 0; i < GN_VMAX; ++i) {
        const int it = threadIdx.x + GN_THREADS * i;
        pix[i] = (int)(((float)it + 0.5f) * inv_q);
        c4s[i] = 4 * (it - pix[i] * q);
    }
    float4 v[GN_VMAX];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < GN_VMAX; ++i) {
        const int it = threadIdx.x + GN_THREADS * i;
        if (it < items) {
            v[i] = *(const float4*)(in + base + (int64_t)pix[i] * Ctot + c4s[i]);
            s += v[i].x + v[i].y + v[i].z + v[i].w;
        }
    }
    const float n = (float)(P * cg);
    const float mean = block_sum<GN_THREADS>(s, red) / n;
    float sq = 0.f;
#pragma unroll
    for (int i = 0; i < GN_VMAX; ++i) {
        const int it = threadIdx.x + GN_THREADS * i;
        if (it < items) {
            const float dx = v[i].x - mean, dy = v[i].y - mean, dz = v[i].z - mean, dw = v[i].w - mean;
            sq += dx * dx + dy * dy + dz * dz + dw * dw;
        }
    }
    const float rstd = rsqrtf(block_sum<GN_THREADS>(sq, red) / n + eps);
    const float* gg = gbs;
    const float* bb = gbs + GN_THREADS;
#pragma unroll
    for (int i = 0; i < GN_VMAX; ++i) {
        const int it = threadIdx.x + GN_THREADS * i;
        if (it < items) {
            const int c4 = c4s[i];
            const int64_t off = base + (int64_t)pix[i] * Ctot + c4;
            float4 y;
            y.x = (v[i].x - mean) * rstd * gg[c4 + 0] + bb[c4 + 0];
            y.y = (v[i].y - mean) * rstd * gg[c4 + 1] + bb[c4 + 1];
            y.z = (v[i].z - mean) * rstd * gg[c4 + 2] + bb[c4 + 2];
            y.w = (v[i].w - mean) * rstd * gg[c4 + 3] + bb[c4 + 3];
            if (out_f32) *(float4*)(out_f32 + off) = y;
            if (out_t) {
                if constexpr (sizeof(T) == 2) {
                    uint2 pk;
                    pk.x = pack2<T>(y.x, y.y);
                    pk.y = pack2<T>(y.z, y.w);
                    *(uint2*)(out_t + off) = pk;
                } else {
                    *(float4*)(out_t + off) = y;
                }
            }
        }
    }
}

// LayerNorm backward (training step): one wave per row, LNB_RPW rows per 256-thread workgroup.
// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dy * gamma, xhat = (x - mean) * rstd with the
// row statistics recomputed from x (two-pass, as the forward).  The affine gradients are per-lane
// column partial sums over the workgroup's rows (one set per row group), reduced across the 4 waves
// in LDS and stored per workgroup; layernorm_bwd_reduce_kernel then sums the workgroups' partials in
// workgroup order (deterministic, no atomics) into dgb.
constexpr int LNB_RPW = 32;

// dres != NULL: dx += dres (the input's second gradient, the residual add of a pre-LN block; may alias dx).
template <typename TD, int V>
__global__ __launch_bounds__(256) void layernorm_bwd_kernel(const float* __restrict__ x, const TD* __restrict__ dy,
                                                            const float* g0, const float* g1, const float* dres,
                                                            float* dx, float* __restrict__ part, int64_t rows,
                                                            int64_t rpg, float eps) {
    constexpr int C = 256 * V;
    __shared__ float4 red[4][4][V][64];  // [wave][group x (dgamma, dbeta)][V][lane]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float4 pg[2][V], pb[2][V];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < V; ++i) pg[h][i] = pb[h][i] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int r = w; r < LNB_RPW; r += 4) {
        const int64_t row = (int64_t)blockIdx.x * LNB_RPW + r;
        if (row >= rows) break;
        const int h = (g1 && ((row / rpg) & 1)) ? 1 : 0;  // wave-uniform; groups alternate every rpg rows
        const float4* gam = (const float4*)(h ? g1 : g0);
        float4 v[V], d[V], ga[V];
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < V; ++i) {
            const int idx = lane + 64 * i;
            v[i] = ((const float4*)(x + row * C))[idx];
            ga[i] = gam[idx];
            if constexpr (sizeof(TD) == 2) {
                const uint2 u = ((const uint2*)(dy + row * C))[idx];
                const f32x2 a = unpack2<TD>(u.x), b = unpack2<TD>(u.y);
                d[i] = make_float4(a[0], a[1], b[0], b[1]);
            } else {
                d[i] = ((const float4*)(dy + row * C))[idx];
            }
            s += v[i].x + v[i].y + v[i].z + v[i].w;
        }
        const float mean = wave_sum(s) * (1.f / C);
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < V; ++i) {
            v[i].x -= mean; v[i].y -= mean; v[i].z -= mean; v[i].w -= mean;
            q += v[i].x * v[i].x + v[i].y * v[i].y + v[i].z * v[i].z + v[i].w * v[i].w;
        }
        const float rstd = rsqrtf(wave_sum(q) * (1.f / C) + eps);
        float sg = 0.f, sgx = 0.f;
#pragma unroll
        for (int i = 0; i < V; ++i) {
            v[i].x *= rstd; v[i].y *= rstd; v[i].z *= rstd; v[i].w *= rstd;  // xhat
            const float4 g = make_float4(d[i].x * ga[i].x, d[i].y * ga[i].y, d[i].z * ga[i].z, d[i].w * ga[i].w);
            sg += g.x + g.y + g.z + g.w;
            sgx += g.x * v[i].x + g.y * v[i].y + g.z * v[i].z + g.w * v[i].w;
            float4& acg = pg[h][i];
            float4& acb = pb[h][i];
            acg.x += d[i].x * v[i].x; acg.y += d[i].y * v[i].y; acg.z += d[i].z * v[i].z; acg.w += d[i].w * v[i].w;
            acb.x += d[i].x; acb.y += d[i].y; acb.z += d[i].z; acb.w += d[i].w;
            d[i] = g;
        }
        const float mg = wave_sum(sg) * (1.f / C), mgx = wave_sum(sgx) * (1.f / C);
#pragma unroll
        for (int i = 0; i < V; ++i) {
            float4 o;
            o.x = rstd * (d[i].x - mg - v[i].x * mgx);
            o.y = rstd * (d[i].y - mg - v[i].y * mgx);
            o.z = rstd * (d[i].z - mg - v[i].z * mgx);
            o.w = rstd * (d[i].w - mg - v[i].w * mgx);
            if (dres) {  // wave-uniform
                const float4 r = ((const float4*)(dres + row * C))[lane + 64 * i];
                o.x += r.x; o.y += r.y; o.z += r.z; o.w += r.w;
            }
            ((float4*)(dx + row * C))[lane + 64 * i] = o;
        }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < V; ++i) {
            red[w][2 * h][i][lane] = pg[h][i];
            red[w][2 * h + 1][i][lane] = pb[h][i];
        }
    __syncthreads();
    // thread t sums the 4 waves for (set j = t / 64, every V column chunk of lane t % 64), in wave order
    const int j = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < V; ++i) {
        float4 a = red[0][j][i][lane];
#pragma unroll
        for (int ww = 1; ww < 4; ++ww) {
            const float4 b = red[ww][j][i][lane];
            a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
        }
        ((float4*)(part + ((int64_t)blockIdx.x * 4 + j) * C))[lane + 64 * i] = a;
    }
}

// dgb[j][c] += sum over workgroups b of part[b][j][c]; j = group * 2 + (0 gamma, 1 beta).
// 64 (j, c) columns per 256-thread workgroup, each column's partials cut into 4 contiguous runs of workgroups,
// one wave per run: every thread adds its run in workgroup order (16 loads in flight), then the 4 run sums are
// added in run order, so the sum is the same on every launch (round 5: one thread per column walked all of a
// column's ~530 partials alone, 14 us per launch at 16 training pairs).
__global__ __launch_bounds__(256) void layernorm_bwd_reduce_kernel(const float* __restrict__ part, float* dgb, int nwg,
                                                                   int C, int sets, int accumulate) {
    __shared__ float red[4][64];
    const int lane = threadIdx.x & 63, run = threadIdx.x >> 6;
    const int i = blockIdx.x * 64 + lane;
    const int ic = min(i, sets * C - 1);
    const float* col = part + ic;
    const int64_t st = (int64_t)4 * C;
    const int b1 = (int)((int64_t)(run + 1) * nwg / 4);
    float s = 0.f;
    int b = (int)((int64_t)run * nwg / 4);
    for (; b + 16 <= b1; b += 16) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = col[(b + u) * st];
#pragma unroll
        for (int u = 0; u < 16; ++u) s += v[u];
    }
    for (; b < b1; ++b) s += col[b * st];
    red[run][lane] = s;
    __syncthreads();
    if (run == 0 && i < sets * C) {
        const float t = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
        dgb[i] = accumulate ? dgb[i] + t : t;
    }
}

// GroupNorm backward (training step): one 512-thread workgroup per (instance, group) as the forward, the
// group's x and dy in registers.  dx = rstd * (g - mean(g) - xhat * mean(g * xhat)) with g = dy * gamma_c;
// the per-channel (sum dy * xhat, sum dy) of the workgroup go through LDS as [PC][cg] products, in chunks of
// PC = GNB_LDS / (2 cg) positions, and are summed over P in position order by one thread per channel (the
// accumulator carried across chunks), into part[instance][2][Ctot]; a second launch sums the instances in
// order (deterministic, no atomics).  ViT-B at 320 (P 400, cg 24) is one chunk; ViT-L at 384 (P 576, cg 32)
// two.
constexpr int GNB_LDS = 2 * 9600;  // floats: PC * cg products of each kind (one chunk covers P 400 x cg 24)

__global__ __launch_bounds__(GN_THREADS) void groupnorm_bwd_kernel(const float* __restrict__ in,
                                                                   const float* __restrict__ dy, const float* gamma,
                                                                   float* __restrict__ dx, float* __restrict__ part,
                                                                   int P, int Ctot, int groups, float eps) {
    __shared__ float red[GN_THREADS / 64];
    __shared__ float prod[GNB_LDS];  // [P][cg] dy * xhat, then [P][cg] dy
    const int inst = blockIdx.y, grp = blockIdx.x;
    const int cg = Ctot / groups, q = cg / 4, items = P * q;
    const int64_t base = (int64_t)inst * P * Ctot + grp * cg;
    const float inv_q = 1.f / (float)q;
    int pix[GN_VMAX], c4s[GN_VMAX];
#pragma unroll
    for (int i = 0; i < GN_VMAX; ++i) {
        const int it = threadIdx.x + GN_THREADS * i;
        pix[i] = (int)(((float)it + 0.5f) * inv_q);
        c4s[i] = 4 * (it - pix[i] * q);
    }
    float4 v[GN_VMAX], d[GN_VMAX];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < GN_VMAX; ++i) {
        const int it = threadIdx.x + GN_THREADS * i;
        if (it < items) {
            const int64_t off = base + (int64_t)pix[i] * Ctot + c4s[i];
            v[i] = *(const float4*)(in + off);
            d[i] = *(const float4*)(dy + off);
            s += v[i].x + v[i].y + v[i].z + v[i].w;
        }
    }
    const float n = (float)(P * cg);
    const float mean = block_sum<GN_THREADS>(s, red) / n;
    float sq = 0.f;
#pragma unroll
    for (int i = 0; i < GN_VMAX; ++i) {
        const int it = threadIdx.x + GN_THREADS * i;
        if (it < items) {
            v[i].x -= mean; v[i].y -= mean; v[i].z -= mean; v[i].w -= mean;
            sq += v[i].x * v[i].x + v[i].y * v[i].y + v[i].z * v[i].z + v[i].w * v[i].w;
        }
    }
    const float rstd = rsqrtf(block_sum<GN_THREADS>(sq, red) / n + eps);
    float sg = 0.f, sgx = 0.f;
    const int PC = GNB_LDS / (2 * cg);  // positions per LDS chunk
    float4 dd[GN_VMAX];                 // dy kept for the later chunks' products
#pragma unroll
    for (int i = 0; i < GN_VMAX; ++i) {
        const int it = threadIdx.x + GN_THREADS * i;
        if (it < items) {
            const int c = grp * cg + c4s[i];
            const float4 ga = *(const float4*)(gamma + c);
            v[i].x *= rstd; v[i].y *= rstd; v[i].z *= rstd; v[i].w *= rstd;  // xhat
            if (pix[i] < PC) {  // first chunk's products now; later chunks after the dx pass
                float* pp = prod + pix[i] * cg + c4s[i];
                pp[0] = d[i].x * v[i].x; pp[1] = d[i].y * v[i].y; pp[2] = d[i].z * v[i].z; pp[3] = d[i].w * v[i].w;
                float* pb = prod + PC * cg + pix[i] * cg + c4s[i];
                pb[0] = d[i].x; pb[1] = d[i].y; pb[2] = d[i].z; pb[3] = d[i].w;
            }
            dd[i] = d[i];
            d[i] = make_float4(d[i].x * ga.x, d[i].y * ga.y, d[i].z * ga.z, d[i].w * ga.w);  // g
            sg += d[i].x + d[i].y + d[i].z + d[i].w;
            sgx += d[i].x * v[i].x + d[i].y * v[i].y + d[i].z * v[i].z + d[i].w * v[i].w;
        }
    }
    const float mg = block_sum<GN_THREADS>(sg, red) / n;  // (its barriers also publish the LDS products)
    const float mgx = block_sum<GN_THREADS>(sgx, red) / n;
#pragma unroll
    for (int i = 0; i < GN_VMAX; ++i) {
        const int it = threadIdx.x + GN_THREADS * i;
        if (it < items) {
            float4 o;
            o.x = rstd * (d[i].x - mg - v[i].x * mgx);
            o.y = rstd * (d[i].y - mg - v[i].y * mgx);
            o.z = rstd * (d[i].z - mg - v[i].z * mgx);
            o.w = rstd * (d[i].w - mg - v[i].w * mgx);
            *(float4*)(dx + base + (int64_t)pix[i] * Ctot + c4s[i]) = o;
        }
    }
    // thread -> (kind, channel): sum over positions in order, chunk by chunk
    const int kind = (int)threadIdx.x / cg, ch = (int)threadIdx.x % cg;
    float acc = 0.f;
    for (int p0 = 0; p0 < P; p0 += PC) {
        if (p0) {  // refill the LDS image with this chunk's products (the first chunk was written above)
            __syncthreads();
#pragma unroll
            for (int i = 0; i < GN_VMAX; ++i) {
                const int it = threadIdx.x + GN_THREADS * i;
                const int r = pix[i] - p0;
                if (it < items && r >= 0 && r < PC) {
                    float* pp = prod + r * cg + c4s[i];
                    pp[0] = dd[i].x * v[i].x; pp[1] = dd[i].y * v[i].y; pp[2] = dd[i].z * v[i].z;
                    pp[3] = dd[i].w * v[i].w;
                    float* pb = prod + PC * cg + r * cg + c4s[i];
                    pb[0] = dd[i].x; pb[1] = dd[i].y; pb[2] = dd[i].z; pb[3] = dd[i].w;
                }
            }
            __syncthreads();
        }
        if ((int)threadIdx.x < 2 * cg) {
            const float* col = prod + kind * PC * cg + ch;
            const int np = min(PC, P - p0);
            for (int pp = 0; pp < np; ++pp) acc += col[pp * cg];
        }
    }
    if ((int)threadIdx.x < 2 * cg) part[((int64_t)inst * 2 + kind) * Ctot + grp * cg + ch] = acc;
}

// dgb[j][c] (+)= sum over instances (in order) of part[inst][j][c]
__global__ __launch_bounds__(256) void groupnorm_bwd_reduce_kernel(const float* __restrict__ part, float* dgb, int n_inst,
                                                                   int Ctot, int accumulate) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= 2 * Ctot) return;
    float s = 0.f;
    for (int b = 0; b < n_inst; ++b) s += part[(int64_t)b * 2 * Ctot + i];
    dgb[i] = accumulate ? dgb[i] + s : s;
}

template <typename T>
__global__ void add_cast_kernel(const float* __restrict__ in, const float* __restrict__ add, int64_t add_n,
                                float* out_f32, T* out_t, int64_t n4) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n4) return;
    float4 v = ((const float4*)in)[i];
    if (add) {
        const float4 a = ((const float4*)add)[i % (add_n / 4)];
        v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    }
    if (out_f32) ((float4*)out_f32)[i] = v;
    if (out_t) {
        if constexpr (sizeof(T) == 2) {
            uint2 pk;
            pk.x = pack2<T>(v.x, v.y);
            pk.y = pack2<T>(v.z, v.w);
            ((uint2*)out_t)[i] = pk;
        } else {
            ((float4*)out_t)[i] = v;
        }
    }
}

// out[r][c] = (T)(in[r][c] * scale[r / rows_per]), 8 elements per thread (two 16-B loads, one 16-B store)
template <typename T>
__global__ __launch_bounds__(256) void scale_rows_cast_kernel(const float4* __restrict__ in, const float* __restrict__ scale,
                                                              int64_t rows_per, int64_t cols8, uint4* __restrict__ out,
                                                              int64_t n8) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n8) return;
    const float sc = scale[(i / cols8) / rows_per];
    const float4 a = in[2 * i], b = in[2 * i + 1];
    out[i] = uint4{pack2<T>(a.x * sc, a.y * sc), pack2<T>(a.z * sc, a.w * sc), pack2<T>(b.x * sc, b.y * sc),
                   pack2<T>(b.z * sc, b.w * sc)};
}

// One thread per (sequence-row token, channel, ky): 16 contiguous kx pixels -> 16 outputs.
template <typename T>
__global__ void patch_im2col_kernel(const float* t0, const float* t1, const float* o0, const float* o1, const float* s0,
                                    const float* s1, T* out, int Bm, int ht, int hs, int P, int64_t total) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const int gt = ht / P, gs = hs / P;
    const int nt = gt * gt, ntok = 2 * nt + gs * gs;
    const int ky = idx % P;
    const int c = (idx / P) % 3;
    const int64_t row = idx / (3 * P);
    const int tok = row % ntok;
    const int64_t seq = row / ntok;
    const int m = (int)(seq / Bm), b = (int)(seq % Bm);
    const float* img;
    int hw, g, t;
    if (tok < nt) { img = m ? t1 : t0; hw = ht; g = gt; t = tok; }
    else if (tok < 2 * nt) { img = m ? o1 : o0; hw = ht; g = gt; t = tok - nt; }
    else { img = m ? s1 : s0; hw = hs; g = gs; t = tok - 2 * nt; }
    const int py = t / g, px = t % g;
    const float* src = img + (((int64_t)b * 3 + c) * hw + (py * P + ky)) * hw + px * P;
    T* dst = out + row * (3 * P * P) + (c * P + ky) * P;
    for (int kx = 0; kx < P; kx += 4) {
        const float4 v = *(const float4*)(src + kx);
        dst[kx + 0] = from_f<T>(v.x);
        dst[kx + 1] = from_f<T>(v.y);
        dst[kx + 2] = from_f<T>(v.z);
        dst[kx + 3] = from_f<T>(v.w);
    }
}

}  // namespace

extern "C" int mmt_layernorm(const float* in, const float* add, int64_t add_rows, float* out_f32, void* out_t,
                             const float* gamma0, const float* beta0, const float* gamma1, const float* beta1,
                             int64_t rows, int64_t rows_per_group, int C, float eps, int dtype, void* stream) {
    if (!in || !gamma0 || !beta0 || rows <= 0 || (C % 256) || C < 256 || C > 1024) return MMT_EBADARG;
    if (add && add_rows <= 0) return MMT_EBADARG;
    if (gamma1 && (rows_per_group <= 0 || !beta1)) return MMT_EBADARG;
    if (rows_per_group <= 0) rows_per_group = rows;
    hipStream_t st = (hipStream_t)stream;
    dim3 grid((unsigned)((rows + 3) / 4));
#define LN_CASE(T, V)                                                                                              \
    hipLaunchKernelGGL((layernorm_kernel<T, V>), grid, dim3(256), 0, st, in, add, add_rows, out_f32, (T*)out_t,  \
                       gamma0, beta0, gamma1, beta1, rows, rows_per_group, eps)
    const int V = C / 256;  // 1..4 (the checks above): one instantiation each
    if (dtype == MMT_BF16) {
        if (V == 1) LN_CASE(bf16_t, 1); else if (V == 2) LN_CASE(bf16_t, 2); else if (V == 3) LN_CASE(bf16_t, 3); else LN_CASE(bf16_t, 4);
    } else if (dtype == MMT_F16) {
        if (V == 1) LN_CASE(f16_t, 1); else if (V == 2) LN_CASE(f16_t, 2); else if (V == 3) LN_CASE(f16_t, 3); else LN_CASE(f16_t, 4);
    } else if (dtype == MMT_F32) {
        if (V == 1) LN_CASE(float, 1); else if (V == 2) LN_CASE(float, 2); else if (V == 3) LN_CASE(float, 3); else LN_CASE(float, 4);
    } else return MMT_EBADARG;
#undef LN_CASE
    return launch_status();
}

extern "C" int mmt_layernorm_bwd_add(const float* x, const void* dy, int dy_dtype, const float* gamma0,
                                     const float* gamma1, const float* dres, float* dx, float* dgb, int dgb_accumulate,
                                     float* ws, int64_t ws_floats, int64_t rows, int64_t rows_per_group, int C,
                                     float eps, void* stream) {
    if (!x || !dy || !gamma0 || !dx || !dgb || !ws || rows <= 0 || (C % 256) || C < 256 || C > 1024) return MMT_EBADARG;
    if (gamma1 && rows_per_group <= 0) return MMT_EBADARG;
    if (!gamma1) rows_per_group = rows;
    if (((uintptr_t)x | (uintptr_t)dy | (uintptr_t)gamma0 | (uintptr_t)gamma1 | (uintptr_t)dx | (uintptr_t)ws |
         (uintptr_t)dres) & 15)
        return MMT_EBADARG;
    const int64_t nwg = (rows + LNB_RPW - 1) / LNB_RPW;
    if (nwg > INT32_MAX || ws_floats < nwg * 4 * C) return MMT_EBADARG;
    hipStream_t st = (hipStream_t)stream;
    const int V = C / 256;
#define LNB_CASE(TD, VV)                                                                                           \
    hipLaunchKernelGGL((layernorm_bwd_kernel<TD, VV>), dim3((unsigned)nwg), dim3(256), 0, st, x, (const TD*)dy,    \
                       gamma0, gamma1, dres, dx, ws, rows, rows_per_group, eps)
#define LNB_V(TD)                                                                                                  \
    if (V == 1) LNB_CASE(TD, 1); else if (V == 2) LNB_CASE(TD, 2); else if (V == 3) LNB_CASE(TD, 3); else LNB_CASE(TD, 4)
    if (dy_dtype == MMT_BF16) { LNB_V(bf16_t); }
    else if (dy_dtype == MMT_F16) { LNB_V(f16_t); }
    else if (dy_dtype == MMT_F32) { LNB_V(float); }
    else return MMT_EBADARG;
#undef LNB_V
#undef LNB_CASE
    const int sets = gamma1 ? 4 : 2;
    hipLaunchKernelGGL(layernorm_bwd_reduce_kernel, dim3((unsigned)((sets * C + 63) / 64)), dim3(256), 0, st, ws, dgb,
                       (int)nwg, C, sets, dgb_accumulate);
    return launch_status();
}

extern "C" int mmt_layernorm_bwd(const float* x, const void* dy, int dy_dtype, const float* gamma0,
                                 const float* gamma1, float* dx, float* dgb, int dgb_accumulate, float* ws,
                                 int64_t ws_floats, int64_t rows, int64_t rows_per_group, int C, float eps,
                                 void* stream) {
    return mmt_layernorm_bwd_add(x, dy, dy_dtype, gamma0, gamma1, nullptr, dx, dgb, dgb_accumulate, ws, ws_floats,
                                 rows, rows_per_group, C, eps, stream);
}

extern "C" int mmt_groupnorm(const float* in, float* out_f32, void* out_t, const float* gamma0, const float* beta0,
                             const float* gamma1, const float* beta1, int n_inst, int inst_per_set, int P, int Ctot,
                             int groups, float eps, int dtype, void* stream) {
    if (!in || !gamma0 || !beta0 || n_inst <= 0 || P <= 0 || groups <= 0 || Ctot % groups) return MMT_EBADARG;
    if ((Ctot / groups) % 4 || Ctot / groups > GN_THREADS || (int64_t)P * (Ctot / groups / 4) > (int64_t)GN_THREADS * GN_VMAX)
        return MMT_EBADARG;
    if (inst_per_set <= 0) inst_per_set = n_inst;
    dim3 grid(groups, n_inst);
    hipStream_t st = (hipStream_t)stream;
    if (dtype == MMT_BF16)
        hipLaunchKernelGGL((groupnorm_kernel<bf16_t>), grid, dim3(GN_THREADS), 0, st, in, out_f32, (bf16_t*)out_t, gamma0,
                           beta0, gamma1, beta1, inst_per_set, P, Ctot, groups, eps);
    else if (dtype == MMT_F16)
        hipLaunchKernelGGL((groupnorm_kernel<f16_t>), grid, dim3(GN_THREADS), 0, st, in, out_f32, (f16_t*)out_t, gamma0,
                           beta0, gamma1, beta1, inst_per_set, P, Ctot, groups, eps);
    else if (dtype == MMT_F32)
        hipLaunchKernelGGL((groupnorm_kernel<float>), grid, dim3(GN_THREADS), 0, st, in, out_f32, (float*)out_t, gamma0,
                           beta0, gamma1, beta1, inst_per_set, P, Ctot, groups, eps);
    else return MMT_EBADARG;
    return launch_status();
}

extern "C" int mmt_groupnorm_bwd(const float* x, const float* dy, const float* gamma, float* dx, float* dgb,
                                 int dgb_accumulate, float* ws, int64_t ws_floats, int n_inst, int P, int Ctot,
                                 int groups, float eps, void* stream) {
    if (!x || !dy || !gamma || !dx || !dgb || !ws || n_inst <= 0 || P <= 0 || groups <= 0 || Ctot % groups)
        return MMT_EBADARG;
    const int cg = Ctot / groups;
    if (cg % 4 || 2 * cg > GN_THREADS || (int64_t)P * (cg / 4) > (int64_t)GN_THREADS * GN_VMAX ||
        ws_floats < (int64_t)n_inst * 2 * Ctot)
        return MMT_EBADARG;
    if (((uintptr_t)x | (uintptr_t)dy | (uintptr_t)gamma | (uintptr_t)dx) & 15) return MMT_EBADARG;
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(groupnorm_bwd_kernel, dim3(groups, n_inst), dim3(GN_THREADS), 0, st, x, dy, gamma, dx, ws, P, Ctot,
                       groups, eps);
    hipLaunchKernelGGL(groupnorm_bwd_reduce_kernel, dim3((unsigned)((2 * Ctot + 255) / 256)), dim3(256), 0, st, ws, dgb,
                       n_inst, Ctot, dgb_accumulate);
    return launch_status();
}

extern "C" int mmt_add_cast(const float* in, const float* add, int64_t add_n, float* out_f32, void* out_t, int64_t n,
                            int dtype, void* stream) {
    if (!in || n <= 0 || (n % 4) || (add && (add_n <= 0 || add_n % 4))) return MMT_EBADARG;
    const int64_t n4 = n / 4;
    dim3 grid((unsigned)((n4 + 255) / 256));
    hipStream_t st = (hipStream_t)stream;
    if (dtype == MMT_BF16)
        hipLaunchKernelGGL((add_cast_kernel<bf16_t>), grid, dim3(256), 0, st, in, add, add_n, out_f32, (bf16_t*)out_t, n4);
    else if (dtype == MMT_F16)
        hipLaunchKernelGGL((add_cast_kernel<f16_t>), grid, dim3(256), 0, st, in, add, add_n, out_f32, (f16_t*)out_t, n4);
    else if (dtype == MMT_F32)
        hipLaunchKernelGGL((add_cast_kernel<float>), grid, dim3(256), 0, st, in, add, add_n, out_f32, (float*)out_t, n4);
    else return MMT_EBADARG;
    return launch_status();
}

extern "C" int mmt_scale_rows_cast(const float* in, const float* scale, int64_t rows_per, void* out, int64_t rows,
                                   int64_t cols, int dtype, void* stream) {
    if (!in || !scale || !out || rows <= 0 || cols <= 0 || cols % 8 || rows_per <= 0) return MMT_EBADARG;
    if (((uintptr_t)in | (uintptr_t)out) & 15) return MMT_EBADARG;
    const int64_t n8 = rows * cols / 8;
    const dim3 grid((unsigned)((n8 + 255) / 256));
    hipStream_t st = (hipStream_t)stream;
    if (dtype == MMT_BF16)
        hipLaunchKernelGGL((scale_rows_cast_kernel<bf16_t>), grid, dim3(256), 0, st, (const float4*)in, scale, rows_per,
                           cols / 8, (uint4*)out, n8);
    else if (dtype == MMT_F16)
        hipLaunchKernelGGL((scale_rows_cast_kernel<f16_t>), grid, dim3(256), 0, st, (const float4*)in, scale, rows_per,
                           cols / 8, (uint4*)out, n8);
    else return MMT_EBADARG;
    return launch_status();
}

extern "C" int mmt_patch_im2col(const float* img_t0, const float* img_t1, const float* img_o0, const float* img_o1,
                                const float* img_s0, const float* img_s1, void* out, int Bm, int ht, int hs, int patch,
                                int dtype, void* stream) {
    // one modality (the RGB-only MixFormer, lib/models/mixformer_vit): img_t1 = img_o1 = img_s1 = NULL
    const int nmod = (!img_t1 && !img_o1 && !img_s1) ? 1 : 2;
    if (!img_t0 || !img_o0 || !img_s0 || !out || Bm <= 0) return MMT_EBADARG;
    if (nmod == 2 && (!img_t1 || !img_o1 || !img_s1)) return MMT_EBADARG;
    if (patch % 4 || ht % patch || hs % patch) return MMT_EBADARG;
    const int gt = ht / patch, gs = hs / patch;
    const int64_t rows = (int64_t)nmod * Bm * (2 * gt * gt + gs * gs);
    const int64_t total = rows * 3 * patch;
    dim3 grid((unsigned)((total + 255) / 256));
    hipStream_t st = (hipStream_t)stream;
    if (dtype == MMT_BF16)
        hipLaunchKernelGGL((patch_im2col_kernel<bf16_t>), grid, dim3(256), 0, st, img_t0, img_t1, img_o0, img_o1,
                           img_s0, img_s1, (bf16_t*)out, Bm, ht, hs, patch, total);
    else if (dtype == MMT_F16)
        hipLaunchKernelGGL((patch_im2col_kernel<f16_t>), grid, dim3(256), 0, st, img_t0, img_t1, img_o0, img_o1,
                           img_s0, img_s1, (f16_t*)out, Bm, ht, hs, patch, total);
    else if (dtype == MMT_F32)
        hipLaunchKernelGGL((patch_im2col_kernel<float>), grid, dim3(256), 0, st, img_t0, img_t1, img_o0, img_o1,
                           img_s0, img_s1, (float*)out, Bm, ht, hs, patch, total);
    else return MMT_EBADARG;
    return launch_status();
}
