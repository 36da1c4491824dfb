// Multi-scale deformable attention (MSDA) for gfx950.
//
// mmt_ms_deform_attn_forward — drop-in for the reference op `ms_deform_attn_forward`
//   (ops/src/vision.cpp:13-16 -> ms_deform_attn_cuda.cu:20-80 -> ms_deform_im2col_cuda.cuh:237-299):
//   out[n,q,m*D+c] = sum_l sum_p w[n,q,m,l,p] * bilinear(V_l[n,:,:,m,c], loc*(W_l,H_l) - 0.5),
//   taps outside the map read 0 and a sample is skipped unless -1 < h < H and -1 < w < W
//   (cuh:55-78, :285-291).  fp64 / fp32 / bf16 (the reference dispatches fp32/fp64 only).
//   One thread per output channel with the channel index fastest: a wave reads whole value rows.
//
// mmt_msda_bimodal — the fused middle of MSDeformAttn_Bimodal.forward
//   (ms_deform_attn_bimodal.py:97-128): softmax of the 8 (level, point) logits per head, sampling
//   location = reference point of the query's own cell + offset / (W, H), and the bimodal gather
//   (level 0 = RGB map, level 1 = TIR map).  The reference duplicates the offsets/weights of its
//   400 bimodal queries onto both 400-query halves and its reference points are per cell, so both
//   halves produce identical rows; this kernel computes them once (B*nq rows, not 2*B*nq).
//   Layout: one 512-thread workgroup per (batch, query) = 8 waves = 8 heads, lane = channel.
//
// mmt_ms_deform_attn_backward — drop-in for `ms_deform_attn_backward` (vision.cpp:13-16 ->
//   ms_deform_attn_cuda.cu:83-153 -> ms_deformable_col2im kernels, ms_deform_im2col_cuda.cuh:86-235
//   for the per-tap arithmetic): grad_value = sum over the four taps of every sample of w_k * g * a,
//   gathered per pixel in a fixed order (msda_bwd_value_kernel: deterministic, no atomics; heads wider than
//   64 channels fall back to the reference's float atomics),
//   grad_attn = sum_c g * bilinear, grad_loc = (W * dbil/dw, H * dbil/dh) * g * a summed over the
//   channels.  One wave per (n, q, m) sample row, lanes over channels: the channel sums of
//   grad_loc / grad_attn are wave reductions with one plain store each (the reference's
//   blocksize-aware shared-memory reductions and their atomics are not needed), and samples the
//   forward skipped (outside (-1, H) x (-1, W)) keep zero gradients, as the reference's zeros_like.
#include "common.hpp"

namespace {

template <typename T> struct Acc { using type = float; };
template <> struct Acc<double> { using type = double; };

template <typename T> MMT_DEV typename Acc<T>::type ld(const T* p) { return to_f<T>(*p); }
template <> MMT_DEV double ld<double>(const double* p) { return *p; }
template <typename T> MMT_DEV void st(T* p, typename Acc<T>::type v) { *p = from_f<T>(v); }
template <> MMT_DEV void st<double>(double* p, double v) { *p = v; }

// ms_deform_attn_im2col_bilinear (cuh:33-84): v points at (0,0) of this (head, channel) plane,
// `stride` elements between consecutive pixels.
template <typename T, typename A>
MMT_DEV A bilinear(const T* v, int H, int W, int64_t stride, A h, A w) {
    const int hl = (int)floor(h), wl = (int)floor(w);
    const int hh_ = hl + 1, wh_ = wl + 1;
    const A lh = h - (A)hl, lw = w - (A)wl;
    const A hh = (A)1 - lh, hw = (A)1 - lw;
    A v1 = 0, v2 = 0, v3 = 0, v4 = 0;
    if (hl >= 0 && wl >= 0) v1 = ld<T>(v + ((int64_t)hl * W + wl) * stride);
    if (hl >= 0 && wh_ <= W - 1) v2 = ld<T>(v + ((int64_t)hl * W + wh_) * stride);
    if (hh_ <= H - 1 && wl >= 0) v3 = ld<T>(v + ((int64_t)hh_ * W + wl) * stride);
    if (hh_ <= H - 1 && wh_ <= W - 1) v4 = ld<T>(v + ((int64_t)hh_ * W + wh_) * stride);
    const A w1 = hh * hw, w2 = hh * lw, w3 = lh * hw, w4 = lh * lw;
    return w1 * v1 + w2 * v2 + w3 * v3 + w4 * v4;
}

template <typename T>
__global__ __launch_bounds__(256) void msda_generic_kernel(const T* __restrict__ value, const int64_t* __restrict__ shapes,
                                                           const int64_t* __restrict__ lstart, const T* __restrict__ loc,
                                                           const T* __restrict__ aw, T* __restrict__ out, int N, int S,
                                                           int M, int D, int Lq, int L, int P, int64_t total) {
    using A = typename Acc<T>::type;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * blockDim.x) {
        const int c = idx % D;
        const int64_t samp = idx / D;  // (n, q, m)
        const int m = samp % M;
        const int n = (int)(samp / ((int64_t)M * Lq));
        int64_t wi = samp * L * P;
        A col = 0;
        for (int l = 0; l < L; ++l) {
            const int H = (int)shapes[2 * l], W = (int)shapes[2 * l + 1];
            const T* vbase = value + (((int64_t)n * S + lstart[l]) * M + m) * D + c;
            for (int p = 0; p < P; ++p, ++wi) {
                const A lx = ld<T>(loc + 2 * wi), ly = ld<T>(loc + 2 * wi + 1), w = ld<T>(aw + wi);
                const A h_im = ly * (A)H - (A)0.5, w_im = lx * (A)W - (A)0.5;
                if (h_im > (A)-1 && w_im > (A)-1 && h_im < (A)H && w_im < (A)W)
                    col += bilinear<T, A>(vbase, H, W, (int64_t)M * D, h_im, w_im) * w;
            }
        }
        st<T>(out + idx, col);
    }
}

// 8 heads x 2 levels x 4 points, 64 channels per head.  Each lane owns 16 bytes of channels (8 bf16 /
// 4 fp32) of one head, so one wave (bf16) or two (fp32) cover a query (one query per workgroup) and
// every corner gather is a 16-byte load.  A level's 16 corner loads are issued before any is used:
// out-of-map corners and samples read a clamped in-map pixel with weight 0, which leaves each
// channel's sum exactly as the reference's skip / zero-corner form (cuh:33-84) computes it.
template <typename T>
__global__ __launch_bounds__(64 * (int)sizeof(T) / 2) void msda_bimodal_kernel(const float* __restrict__ offw,
                                                                              const T* __restrict__ value,
                                                                              T* __restrict__ out, int B, int hw) {
    constexpr int NH = 8, NL = 2, NP = 4, DH = 64, CM = NH * DH;
    constexpr int EPL = 16 / (int)sizeof(T), LPH = DH / EPL;  // one query per workgroup: 8 * LPH threads
    const int nq = hw * hw;
    const int64_t row = blockIdx.x;  // b * nq + q
    const int t = threadIdx.x, m = t / LPH, c0 = (t % LPH) * EPL;
    const int b = (int)(row / nq), q = (int)(row % nq);
    const float* ow = offw + row * (NH * NL * NP * 3);
    // softmax over the 8 logits of this head (fp32, max-subtracted)
    float lg[NL * NP];
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < NL * NP; ++i) {
        lg[i] = ow[NH * NL * NP * 2 + m * NL * NP + i];
        mx = fmaxf(mx, lg[i]);
    }
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < NL * NP; ++i) {
        lg[i] = expf(lg[i] - mx);
        sum += lg[i];
    }
    const float inv = 1.f / sum;
    const float rx = ((float)(q % hw) + 0.5f) / (float)hw;
    const float ry = ((float)(q / hw) + 0.5f) / (float)hw;
    float col[EPL];
#pragma unroll
    for (int j = 0; j < EPL; ++j) col[j] = 0.f;
#pragma unroll
    for (int l = 0; l < NL; ++l) {  // per level: 16 corner loads in flight, then their math
        uint4 raw[NP][4];
        float wt[NP][4], at[NP];
        const T* vb = value + ((int64_t)(l * B + b) * nq) * CM + m * DH + c0;
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            const int oi = ((m * NL + l) * NP + p) * 2;
            const float lx = rx + ow[oi] / (float)hw;
            const float ly = ry + ow[oi + 1] / (float)hw;
            const float h_im = ly * (float)hw - 0.5f, w_im = lx * (float)hw - 0.5f;
            const bool in = h_im > -1.f && w_im > -1.f && h_im < (float)hw && w_im < (float)hw;
            const float hf = floorf(h_im), wf = floorf(w_im);
            const int hl = (int)hf, wl = (int)wf, hh_ = hl + 1, wh_ = wl + 1;
            const float lh = h_im - hf, lw = w_im - wf, hh = 1.f - lh, hwt = 1.f - lw;
            const bool y0 = hl >= 0, y1 = hh_ <= hw - 1, x0 = wl >= 0, x1 = wh_ <= hw - 1;
            wt[p][0] = in && y0 && x0 ? hh * hwt : 0.f;
            wt[p][1] = in && y0 && x1 ? hh * lw : 0.f;
            wt[p][2] = in && y1 && x0 ? lh * hwt : 0.f;
            wt[p][3] = in && y1 && x1 ? lh * lw : 0.f;
            at[p] = in ? lg[l * NP + p] * inv : 0.f;
            const int ya = min(max(hl, 0), hw - 1), yb = min(max(hh_, 0), hw - 1);
            const int xa = min(max(wl, 0), hw - 1), xb = min(max(wh_, 0), hw - 1);
            raw[p][0] = *(const uint4*)(vb + (ya * hw + xa) * CM);
            raw[p][1] = *(const uint4*)(vb + (ya * hw + xb) * CM);
            raw[p][2] = *(const uint4*)(vb + (yb * hw + xa) * CM);
            raw[p][3] = *(const uint4*)(vb + (yb * hw + xb) * CM);
        }
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            float v[4][EPL];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t w4[4] = {raw[p][k].x, raw[p][k].y, raw[p][k].z, raw[p][k].w};
#pragma unroll
                for (int j = 0; j < EPL; ++j) {
                    if constexpr (sizeof(T) == 2)
                        v[k][j] = unpack2<T>(w4[j >> 1])[j & 1];
                    else
                        v[k][j] = __uint_as_float(w4[j]);
                }
            }
#pragma unroll
            for (int j = 0; j < EPL; ++j)
                col[j] += (wt[p][0] * v[0][j] + wt[p][1] * v[1][j] + wt[p][2] * v[2][j] + wt[p][3] * v[3][j]) * at[p];
        }
    }
    T* o = out + row * CM + m * DH + c0;
    if constexpr (sizeof(T) == 2) {
        *(uint4*)o = uint4{pack2<T>(col[0], col[1]), pack2<T>(col[2], col[3]), pack2<T>(col[4], col[5]),
                           pack2<T>(col[6], col[7])};
    } else {
        *(f32x4*)o = f32x4{col[0], col[1], col[2], col[3]};
    }
}

template <typename A> MMT_DEV A wave_sum_t(A v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// ATOMIC: grad_value by float atomics here (the general fallback); else msda_bwd_value_kernel gathers it
template <typename T, bool ATOMIC>
__global__ __launch_bounds__(256) void msda_bwd_kernel(const T* __restrict__ value, const int64_t* __restrict__ shapes,
                                                       const int64_t* __restrict__ lstart, const T* __restrict__ loc,
                                                       const T* __restrict__ aw, const T* __restrict__ gout,
                                                       T* __restrict__ gvalue, T* __restrict__ gloc, T* __restrict__ gaw,
                                                       int S, int M, int D, int Lq, int L, int P, int64_t nsamp) {
    using A = T;  // fp32 / fp64 only, as the reference's dispatch
    const int64_t samp = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // (n, q, m)
    if (samp >= nsamp) return;                                           // wave-uniform
    const int lane = threadIdx.x & 63;
    const int m = samp % M;
    const int n = (int)(samp / ((int64_t)M * Lq));
    const T* g = gout + samp * D;
    int64_t wi = samp * L * P;
    for (int l = 0; l < L; ++l) {
        const int H = (int)shapes[2 * l], W = (int)shapes[2 * l + 1];
        const int64_t base = (((int64_t)n * S + lstart[l]) * M + m) * D;
        const int64_t ws = (int64_t)M * D, hs = (int64_t)W * ws;
        for (int p = 0; p < P; ++p, ++wi) {
            const A lx = loc[2 * wi], ly = loc[2 * wi + 1], a = aw[wi];
            const A h = ly * (A)H - (A)0.5, w = lx * (A)W - (A)0.5;
            A sx = 0, sy = 0, sa = 0;
            if (h > (A)-1 && w > (A)-1 && h < (A)H && w < (A)W) {  // sample-uniform, so wave-uniform
                const int hl = (int)floor(h), wl = (int)floor(w), hh_ = hl + 1, wh_ = wl + 1;
                const A lh = h - (A)hl, lw = w - (A)wl, hh = (A)1 - lh, hw = (A)1 - lw;
                const A w1 = hh * hw, w2 = hh * lw, w3 = lh * hw, w4 = lh * lw;
                const bool k1 = hl >= 0 && wl >= 0, k2 = hl >= 0 && wh_ <= W - 1;
                const bool k3 = hh_ <= H - 1 && wl >= 0, k4 = hh_ <= H - 1 && wh_ <= W - 1;
                const int64_t o1 = hl * hs + wl * ws, o2 = o1 + ws, o3 = o1 + hs, o4 = o3 + ws;
                for (int c = lane; c < D; c += 64) {
                    const A tg = g[c], tgv = tg * a;
                    const T* v = value + base + c;
                    T* gv = gvalue + base + c;
                    A gh = 0, gw = 0, v1 = 0, v2 = 0, v3 = 0, v4 = 0;
                    if (k1) { v1 = v[o1]; gh -= hw * v1; gw -= hh * v1; if (ATOMIC) atomicAdd(gv + o1, w1 * tgv); }
                    if (k2) { v2 = v[o2]; gh -= lw * v2; gw += hh * v2; if (ATOMIC) atomicAdd(gv + o2, w2 * tgv); }
                    if (k3) { v3 = v[o3]; gh += hw * v3; gw -= lh * v3; if (ATOMIC) atomicAdd(gv + o3, w3 * tgv); }
                    if (k4) { v4 = v[o4]; gh += lw * v4; gw += lh * v4; if (ATOMIC) atomicAdd(gv + o4, w4 * tgv); }
                    sa += tg * (w1 * v1 + w2 * v2 + w3 * v3 + w4 * v4);
                    sx += (A)W * gw * tgv;
                    sy += (A)H * gh * tgv;
                }
                sa = wave_sum_t<A>(sa);
                sx = wave_sum_t<A>(sx);
                sy = wave_sum_t<A>(sy);
            }
            if (lane == 0) {
                gaw[wi] = sa;
                gloc[2 * wi] = sx;
                gloc[2 * wi + 1] = sy;
            }
        }
    }
}

MMT_DEV float fma_(float a, float b, float c) { return fmaf(a, b, c); }
MMT_DEV double fma_(double a, double b, double c) { return fma(a, b, c); }

// A bucket's ordered sum, acc = fma(w_e, x_e, acc) for e = e0 .. e1 - 1, with the loads of U entries issued before
// their adds: the gathers take it for buckets longer than BUCKET_LONG (collapsed sampling locations: one chain of
// thousands of entries would otherwise wait out a load latency per entry).  Same order, same bits as the
// one-entry-per-step loops.
constexpr int BUCKET_LONG = 24;
template <int U, typename A, typename Wt, typename Val>
MMT_DEV A bucket_sum(int e0, int e1, A acc, Wt&& wt, Val&& val) {
    for (int e = e0; e < e1; e += U) {
        A w[U], x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int ec = min(e + u, e1 - 1);
            w[u] = wt(ec);
            x[u] = val(ec);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (e + u < e1) acc = fma_(w[u], x[u], acc);
    }
    return acc;
}

// grad_value without atomics (deterministic): one workgroup per (n, m, level, chunk of 64 consecutive pixels of
// the level in raster order).  Every sample of (n, m, level) -- Lq x P of them, in batches of MSDA_SB -- is expanded
// into its four bilinear taps (the forward's validity rules, cuh:55-84); the taps that land in the chunk are counted
// per pixel, bucketed (LDS) in (sample, tap) order (bucket_pass), and each pixel's channels summed in that fixed
// order: grad_value[pixel, c] = sum w_k * (g[q, c] * a), written once.  Taps are the reference's atomics
// (ms_deform_im2col_cuda.cuh:86-235, ms_deformable_col2im_*) re-ordered; thread (c, pixel group) owns 16 pixels.
constexpr int MSDA_PIX = 64, MSDA_SB = 1024;

// Stable bucket placement (replaces the per-bucket one-thread insertion sort, whose cost grew with the square of a
// bucket's length when sampling locations collapse onto a pixel).  A sample contributes at most one tap to a pixel,
// so (sample, tap) order within a bucket is the order of the items i = 4 j + k.  The workgroup's NW waves own
// contiguous runs of items; a wave walks its run 64 items at a time in order, finds the lanes whose taps land on the
// same pixel by a bitwise ballot match over the NB bits of the pixel index, and places lane L at
//   bucket start + earlier waves' items on the pixel + this wave's earlier items on it + #peers below L.
// Counts live in tbl: NW rows of packed 16-bit (wave, pixel) counters, ceil(np / 2) words per row (a pixel's
// items <= the samples, < 65536).  Same order as the sort, so the same sums bit for bit.
template <int NB>
MMT_DEV uint64_t bucket_peers(int r) {  // lanes whose pixel equals this lane's (r < 0: no tap, no peers)
    uint64_t pe = __ballot(r >= 0);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const uint64_t m = __ballot((r >> b) & 1);
        pe &= ((r >> b) & 1) ? m : ~m;
    }
    return r >= 0 ? pe : 0ull;
}

// One pass over this wave's items [i0, i1): item(i, r, w) sets the pixel r (< 0: no tap) and the weight.
// place = false: add the counts into tbl_w.  place = true: tbl_w holds this wave's starting offsets (after
// bucket_wave_offsets); put(pos, i, w) stores the entry.
template <int NB, typename A, typename Item, typename Put>
MMT_DEV void bucket_pass(uint32_t* tbl_w, const int* start, int i0, int i1, bool place, Item&& item, Put&& put) {
    const int lane = threadIdx.x & 63;
    for (int b = i0; b < i1; b += 64) {  // wave-uniform
        const int i = b + lane;
        int r = -1;
        A wk = (A)0;
        if (i < i1) item(i, r, wk);
        const uint64_t pe = bucket_peers<NB>(r);
        const uint64_t below = pe & ((1ull << lane) - 1ull);
        const bool lead = r >= 0 && below == 0ull;
        const uint32_t sh = 16u * (uint32_t)(r & 1);
        uint32_t old = 0;
        if (lead) old = atomicAdd(&tbl_w[r >> 1], (uint32_t)__popcll(pe) << sh);
        if (place) {
            const int leader = r >= 0 ? __ffsll((unsigned long long)pe) - 1 : lane;
            old = __shfl(old, leader, 64);
            if (r >= 0) put(start[r] + (int)((old >> sh) & 0xffffu) + __popcll(below), i, wk);
        }
    }
}

// After the counting pass: every (wave, pixel) counter becomes the items of earlier waves on that pixel, and
// total[r] the pixel's count, for r < 2 * words (total holds that many).  Threads stride over the words.
template <int NW>
MMT_DEV void bucket_wave_offsets(uint32_t* tbl, int words, int* total, int nthreads) {
    for (int x = threadIdx.x; x < words; x += nthreads) {
        uint32_t run = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const uint32_t v = tbl[w * words + x];
            tbl[w * words + x] = run;
            run += v;
        }
        total[2 * x] = (int)(run & 0xffffu);
        total[2 * x + 1] = (int)(run >> 16);
    }
}

template <typename T>
__global__ __launch_bounds__(256) void msda_bwd_value_kernel(const T* __restrict__ loc, const T* __restrict__ aw,
                                                             const T* __restrict__ gout, T* __restrict__ gvalue,
                                                             const int64_t* __restrict__ shapes,
                                                             const int64_t* __restrict__ lstart, int S, int M, int D,
                                                             int Lq, int L, int P) {
    using A = T;
    __shared__ int cnt[MSDA_PIX + 1];
    __shared__ uint32_t tbl[4 * (MSDA_PIX / 2)];  // the 4 waves' packed (wave, pixel) counters
    __shared__ int ekey[4 * MSDA_SB];
    __shared__ A ew[4 * MSDA_SB];
    __shared__ A sa[MSDA_SB];
    __shared__ int sq[MSDA_SB];
    const int t = threadIdx.x;
    // (level, chunk) of this workgroup: chunks of every level back to back
    int l = 0, chunk = blockIdx.x, H = 0, W = 0;
    for (; l < L; ++l) {
        H = (int)shapes[2 * l];
        W = (int)shapes[2 * l + 1];
        const int nc = (H * W + MSDA_PIX - 1) / MSDA_PIX;
        if (chunk < nc) break;
        chunk -= nc;
    }
    if (l >= L) return;  // past the last level's chunks (the grid is an upper bound): uniform
    const int m = blockIdx.y, n = blockIdx.z;
    const int p0 = chunk * MSDA_PIX, np = min(MSDA_PIX, H * W - p0);
    const int c = t & 63, pg = t >> 6;  // channel, pixel group (pixels pg, pg + 4, ...)
    A acc[MSDA_PIX / 4];
#pragma unroll
    for (int i = 0; i < MSDA_PIX / 4; ++i) acc[i] = 0;
    const int ns = Lq * P;
    // the taps of sample j (of this (n, m, l)) inside the chunk: f(k, pixel - p0, w_k)
    auto taps = [&](int j, auto&& f) {
        const int q = j / P, p = j - q * P;
        const int64_t wi = (((int64_t)n * Lq + q) * M + m) * L * P + (int64_t)l * P + p;
        const A lx = loc[2 * wi], ly = loc[2 * wi + 1];
        const A h = ly * (A)H - (A)0.5, w = lx * (A)W - (A)0.5;
        if (!(h > (A)-1 && w > (A)-1 && h < (A)H && w < (A)W)) return;
        const int hl = (int)floor(h), wl = (int)floor(w), hh_ = hl + 1, wh_ = wl + 1;
        const A lh = h - (A)hl, lw = w - (A)wl, hh = (A)1 - lh, hw = (A)1 - lw;
        const int r1 = hl * W + wl - p0;
        if (hl >= 0 && wl >= 0 && (unsigned)r1 < (unsigned)np) f(0, r1, hh * hw);
        if (hl >= 0 && wh_ <= W - 1 && (unsigned)(r1 + 1) < (unsigned)np) f(1, r1 + 1, hh * lw);
        if (hh_ <= H - 1 && wl >= 0 && (unsigned)(r1 + W) < (unsigned)np) f(2, r1 + W, lh * hw);
        if (hh_ <= H - 1 && wh_ <= W - 1 && (unsigned)(r1 + W + 1) < (unsigned)np) f(3, r1 + W + 1, lh * lw);
    };
    const int wv = t >> 6;
    for (int b0 = 0; b0 < ns; b0 += MSDA_SB) {
        const int nb = min(MSDA_SB, ns - b0);
        if (t < 4 * (MSDA_PIX / 2)) tbl[t] = 0;
        for (int j = t; j < nb; j += 256) {  // the samples' q and a
            const int jj = b0 + j, q = jj / P, p = jj - q * P;
            sq[j] = q;
            sa[j] = aw[(((int64_t)n * Lq + q) * M + m) * L * P + (int64_t)l * P + p];
        }
        __syncthreads();
        // items i = 4 j + k of this batch, a contiguous run per wave; the chunk's taps counted, then placed stably
        const int items = 4 * nb, per = (items + 4 * 64 - 1) / (4 * 64) * 64;
        const int i0 = min(wv * per, items), i1 = min(i0 + per, items);
        auto item = [&](int i, int& r, A& wk) {
            const int k = i & 3;
            taps(b0 + (i >> 2), [&](int kk, int rr, A ww) {
                if (kk == k) r = rr, wk = ww;
            });
        };
        uint32_t* tw = tbl + wv * (MSDA_PIX / 2);
        bucket_pass<6, A>(tw, cnt, i0, i1, false, item, [](int, int, A) {});
        __syncthreads();
        bucket_wave_offsets<4>(tbl, MSDA_PIX / 2, cnt, 256);
        __syncthreads();
        if (t < 64) {  // exclusive scan of the 64 counts (one wave), in place: bucket starts, cnt[64] = total
            const int v = cnt[t];
            int x = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int y = __shfl_up(x, o, 64);
                if (t >= o) x += y;
            }
            cnt[t] = x - v;
            if (t == 63) cnt[MSDA_PIX] = x;
        }
        __syncthreads();
        bucket_pass<6, A>(tw, cnt, i0, i1, true, item, [&](int pos, int i, A wk) {
            ekey[pos] = i;
            ew[pos] = wk;
        });
        __syncthreads();
        {  // the wave's 16 pixels advance together (pixels are wave-uniform): 16 independent gathers in flight
            int e0[MSDA_PIX / 4], e1[MSDA_PIX / 4], len = 0;
#pragma unroll
            for (int i = 0; i < MSDA_PIX / 4; ++i) {
                const int r = min(pg + 4 * i, np);  // past the chunk: an empty range
                e0[i] = cnt[r];
                e1[i] = r < np ? cnt[r + 1] : cnt[r];
                len = max(len, e1[i] - e0[i]);
            }
            const int64_t gq = (int64_t)M * D, g0 = ((int64_t)n * Lq * M + m) * D + min(c, D - 1);
            if (len > BUCKET_LONG) {  // wave-uniform: pixel by pixel, 8 entries' loads in flight
#pragma unroll
                for (int i = 0; i < MSDA_PIX / 4; ++i)
                    acc[i] = bucket_sum<8>(e0[i], e1[i], acc[i], [&](int e) { return ew[e]; },
                                           [&](int e) { const int j = ekey[e] >> 2; return gout[g0 + sq[j] * gq] * sa[j]; });
            } else {
                for (int k = 0; k < len; ++k) {
#pragma unroll
                    for (int i = 0; i < MSDA_PIX / 4; ++i) {
                        const int e = e0[i] + k;
                        if (e < e1[i]) {
                            const int j = ekey[e] >> 2;
                            acc[i] = fma_(ew[e], gout[g0 + sq[j] * gq] * sa[j], acc[i]);
                        }
                    }
                }
            }
        }
        __syncthreads();
    }
    if (c < D) {
        T* gv = gvalue + (((int64_t)n * S + lstart[l] + p0) * M + m) * D + c;
#pragma unroll
        for (int i = 0; i < MSDA_PIX / 4; ++i) {
            const int r = pg + 4 * i;
            if (r < np) gv[(int64_t)r * M * D] = acc[i];
        }
    }
}

// grad_value, one workgroup per (n, m, level) (round 6): the level's Lq x P samples expanded
// into their taps ONCE (msda_bwd_value_kernel re-expanded them in every 64-pixel chunk workgroup), counted per pixel
// of the whole level, bucketed in (sample, tap) order -- the same summation order as
// msda_bwd_value_kernel, so the same sums bit for bit -- then each pixel's channels summed, 16 waves over the
// pixels with four independent sums in flight per wave.  Taken when a level's samples and pixels fit the LDS
// lists (Lq P <= NML_S, H W <= NML_PIX) and D <= 64.
constexpr int NML_T = 1024, NML_S = 2048, NML_PIX = 1024;
template <typename T>
__global__ __launch_bounds__(NML_T) void msda_bwd_value_nml_kernel(const T* __restrict__ loc, const T* __restrict__ aw,
                                                                   const T* __restrict__ gout, T* __restrict__ gvalue,
                                                                   const int64_t* __restrict__ shapes,
                                                                   const int64_t* __restrict__ lstart, int S, int M,
                                                                   int D, int Lq, int L, int P) {
    using A = T;
    __shared__ int cnt[NML_PIX + 2];
    __shared__ uint32_t tbl[(NML_T / 64) * (NML_PIX / 2)];  // the 16 waves' packed (wave, pixel) counters
    __shared__ int ekey[4 * NML_S];
    __shared__ A ew[4 * NML_S];
    __shared__ A sa[NML_S];
    const int t = threadIdx.x;
    const int l = blockIdx.x, m = blockIdx.y, n = blockIdx.z;
    const int H = (int)shapes[2 * l], W = (int)shapes[2 * l + 1], np = H * W, ns = Lq * P;
    const int words = (np + 1) / 2;
    for (int x = t; x < (NML_T / 64) * words; x += NML_T) tbl[x] = 0;
    for (int j = t; j < ns; j += NML_T) {
        const int q = j / P, p = j - q * P;
        sa[j] = aw[(((int64_t)n * Lq + q) * M + m) * L * P + (int64_t)l * P + p];
    }
    __syncthreads();
    auto taps = [&](int j, auto&& f) {  // msda_bwd_value_kernel's tap rules, pixels of the whole level
        const int q = j / P, p = j - q * P;
        const int64_t wi = (((int64_t)n * Lq + q) * M + m) * L * P + (int64_t)l * P + p;
        const A lx = loc[2 * wi], ly = loc[2 * wi + 1];
        const A h = ly * (A)H - (A)0.5, w = lx * (A)W - (A)0.5;
        if (!(h > (A)-1 && w > (A)-1 && h < (A)H && w < (A)W)) return;
        const int hl = (int)floor(h), wl = (int)floor(w), hh_ = hl + 1, wh_ = wl + 1;
        const A lh = h - (A)hl, lw = w - (A)wl, hh = (A)1 - lh, hw = (A)1 - lw;
        const int r1 = hl * W + wl;
        if (hl >= 0 && wl >= 0) f(0, r1, hh * hw);
        if (hl >= 0 && wh_ <= W - 1) f(1, r1 + 1, hh * lw);
        if (hh_ <= H - 1 && wl >= 0) f(2, r1 + W, lh * hw);
        if (hh_ <= H - 1 && wh_ <= W - 1) f(3, r1 + W + 1, lh * lw);
    };
    // items i = 4 j + k, a contiguous run per wave: counted, offsets, scanned, placed stably (no sort)
    const int wv = t >> 6, items = 4 * ns, per = (items + NML_T - 1) / NML_T * 64;
    const int i0 = min(wv * per, items), i1 = min(i0 + per, items);
    auto item = [&](int i, int& r, A& wk) {
        const int k = i & 3;
        taps(i >> 2, [&](int kk, int rr, A ww) {
            if (kk == k) r = rr, wk = ww;
        });
    };
    uint32_t* tw = tbl + wv * words;
    bucket_pass<10, A>(tw, cnt, i0, i1, false, item, [](int, int, A) {});
    __syncthreads();
    bucket_wave_offsets<NML_T / 64>(tbl, words, cnt, NML_T);
    __syncthreads();
    if (t < 64) {  // exclusive scan of the np counts in place: lane t owns a run of ceil(np / 64)
        const int per_l = (np + 63) / 64, r0 = min(t * per_l, np), r1 = min(r0 + per_l, np);
        int sum = 0;
        for (int r = r0; r < r1; ++r) sum += cnt[r];
        int x = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (t >= o) x += y;
        }
        int run = x - sum;
        for (int r = r0; r < r1; ++r) {
            const int v = cnt[r];
            cnt[r] = run;
            run += v;
        }
        if (t == 63) cnt[np] = x;
    }
    __syncthreads();
    bucket_pass<10, A>(tw, cnt, i0, i1, true, item, [&](int pos, int i, A wk) {
        ekey[pos] = i;
        ew[pos] = wk;
    });
    __syncthreads();
    const int wave = t >> 6, c = t & 63;
    constexpr int NW = NML_T / 64, PS = 4;
    const int64_t gq = (int64_t)M * D, g0 = ((int64_t)n * Lq * M + m) * D + min(c, D - 1);
    for (int r0 = wave; r0 < np; r0 += NW * PS) {
        int e0[PS], e1[PS], len = 0;
        A acc[PS];
#pragma unroll
        for (int i = 0; i < PS; ++i) {
            const int r = r0 + i * NW;
            e0[i] = r < np ? cnt[r] : 0;
            e1[i] = r < np ? cnt[r + 1] : 0;
            len = max(len, e1[i] - e0[i]);
            acc[i] = 0;
        }
        if (len > BUCKET_LONG) {  // wave-uniform: pixel by pixel, 8 entries' loads in flight
#pragma unroll
            for (int i = 0; i < PS; ++i)
                acc[i] = bucket_sum<8>(e0[i], e1[i], acc[i], [&](int e) { return ew[e]; },
                                       [&](int e) { const int j = ekey[e] >> 2; return gout[g0 + (j / P) * gq] * sa[j]; });
        } else {
            for (int k = 0; k < len; ++k) {
#pragma unroll
                for (int i = 0; i < PS; ++i) {
                    const int e = e0[i] + k;
                    if (e < e1[i]) {
                        const int j = ekey[e] >> 2;
                        acc[i] = fma_(ew[e], gout[g0 + (j / P) * gq] * sa[j], acc[i]);
                    }
                }
            }
        }
        if (c < D) {
            T* gv = gvalue + (((int64_t)n * S + lstart[l]) * M + m) * D + c;
#pragma unroll
            for (int i = 0; i < PS; ++i) {
                const int r = r0 + i * NW;
                if (r < np) gv[(int64_t)r * M * D] = acc[i];
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------------------------
// Training form of MSDeformAttn_Bimodal's middle (ms_deform_attn_bimodal.py:97-128 as the training step runs it,
// mmt_amd.train.fusion_forward): from the bf16 outputs of value_proj / sampling_offsets / attention_weights to the
// bf16 input of output_proj, forward and backward, with the reference's arithmetic:
//   a[q,m,:]  = softmax(float(awl[q, m*8 : m*8+8]))             (F.softmax(aw.float(), -1): torch's warp
//               softmax order for 8 logits -- butterfly max / sum over lanes i^4, i^2, i^1, then e_i / sum)
//   loc       = ref[q] + float(off[q,m,l,p,:]) / (hw, hw)        (ref: the device-computed reference points)
//   out[q, m*64 + c] = bf16(sum_l sum_p a * bilinear(V_l[:, :, m, c], loc * hw - 0.5))   (msda_generic_kernel)
// Backward: grad_value (bf16) = the deterministic per-pixel gather of msda_bwd_value_kernel (same (sample, tap)
// summation order, so the same fp32 sums); grad_awl = bf16(a * (gaw - sum_j a_j gaw_j)) (softmax backward);
// grad_off = bf16(gloc / hw) (the division's backward), gaw / gloc per sample as msda_bwd_kernel, summed over the
// 64 channels in 8-lane groups.  Replaces the generic fp32 kernels plus the step's softmax, location, cast and
// backward glue (round 6).  Layouts: value / grad_value [B][2][nq][8][64], off / grad_off [B][nq][8][2][4][2],
// awl / grad_awl [B][nq][8][8], ref fp32 [nq][2] (x, y), out / grad_out [B][nq][512]; nq = hw * hw.
constexpr int MT_NH = 8, MT_NL = 2, MT_NP = 4, MT_DH = 64, MT_CM = MT_NH * MT_DH, MT_NQ_MAX = 484;

// torch's softmax of 8 logits (persistent warp softmax, 8 lanes): butterfly max and sum, e_i / sum
MMT_DEV void mt_softmax8(const float* lg, float* a) {
    float e[8];
    float mx = lg[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) mx = fmaxf(mx, lg[i]);
#pragma unroll
    for (int i = 0; i < 8; ++i) e[i] = expf(lg[i] - mx);
    const float s = ((e[0] + e[4]) + (e[2] + e[6])) + ((e[1] + e[5]) + (e[3] + e[7]));
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = e[i] / s;
}

MMT_DEV void mt_load_logits(const bf16_t* awl, float* lg) {  // 8 consecutive bf16 (16 B)
    const uint4 u = *(const uint4*)awl;
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        lg[2 * j] = __uint_as_float(w[j] << 16);
        lg[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
    }
}

// sample geometry (msda_generic_kernel / msda_bwd_kernel): h_im / w_im, the in-range flag, the taps' corner
struct MtGeom {
    float h, w;
    bool in;
};
MMT_DEV MtGeom mt_geom(float rx, float ry, float ox, float oy, int hw) {
    const float lx = rx + ox / (float)hw, ly = ry + oy / (float)hw;
    MtGeom g;
    g.h = ly * (float)hw - 0.5f;
    g.w = lx * (float)hw - 0.5f;
    g.in = g.h > -1.f && g.w > -1.f && g.h < (float)hw && g.w < (float)hw;
    return g;
}

MMT_DEV uint4 mt_ld(bool k, const bf16_t* p) {  // a valid tap's 16 B, else zeros (no select of addresses)
    uint4 r = uint4{0u, 0u, 0u, 0u};
    if (k) r = *(const uint4*)p;
    return r;
}

MMT_DEV void mt_unpack8(uint4 u, float* v) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        v[2 * j] = __uint_as_float(w[j] << 16);
        v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
    }
}

// forward: one wave per (b, q); lane = (head m, 8-channel group)
__global__ __launch_bounds__(64) void msda_train_fwd_kernel(const bf16_t* __restrict__ value, const bf16_t* __restrict__ off,
                                                            const bf16_t* __restrict__ awl, const float* __restrict__ ref,
                                                            bf16_t* __restrict__ out, int hw, int op, int ap) {
    const int nq = hw * hw;
    const int64_t row = blockIdx.x;  // b * nq + q
    const int b = (int)(row / nq), q = (int)(row % nq);
    const int t = threadIdx.x, m = t >> 3, c0 = (t & 7) * 8;
    float lg[8], a[8];
    mt_load_logits(awl + row * ap + m * 8, lg);
    mt_softmax8(lg, a);
    const float rx = ref[2 * q], ry = ref[2 * q + 1];
    const bf16_t* ob = off + row * op + m * (MT_NL * MT_NP * 2);
    float col[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) col[j] = 0.f;
#pragma unroll
    for (int l = 0; l < MT_NL; ++l) {
        const bf16_t* vb = value + ((int64_t)(b * MT_NL + l) * nq) * MT_CM + m * MT_DH + c0;
#pragma unroll
        for (int p = 0; p < MT_NP; ++p) {
            const int i = l * MT_NP + p;
            const MtGeom g = mt_geom(rx, ry, bf2f(ob[2 * i]), bf2f(ob[2 * i + 1]), hw);
            if (!g.in) continue;  // lane-group uniform
            const int hl = (int)floorf(g.h), wl = (int)floorf(g.w), hh_ = hl + 1, wh_ = wl + 1;
            const float lh = g.h - (float)hl, lw = g.w - (float)wl, hh = 1.f - lh, hwt = 1.f - lw;
            const bool k1 = hl >= 0 && wl >= 0, k2 = hl >= 0 && wh_ <= hw - 1;
            const bool k3 = hh_ <= hw - 1 && wl >= 0, k4 = hh_ <= hw - 1 && wh_ <= hw - 1;
            float v1[8], v2[8], v3[8], v4[8];
            mt_unpack8(mt_ld(k1, vb + (hl * hw + wl) * MT_CM), v1);
            mt_unpack8(mt_ld(k2, vb + (hl * hw + wh_) * MT_CM), v2);
            mt_unpack8(mt_ld(k3, vb + (hh_ * hw + wl) * MT_CM), v3);
            mt_unpack8(mt_ld(k4, vb + (hh_ * hw + wh_) * MT_CM), v4);
            const float w1 = hh * hwt, w2 = hh * lw, w3 = lh * hwt, w4 = lh * lw;
#pragma unroll
            for (int j = 0; j < 8; ++j) col[j] += (w1 * v1[j] + w2 * v2[j] + w3 * v3[j] + w4 * v4[j]) * a[i];
        }
    }
    bf16_t* o = out + row * MT_CM + m * MT_DH + c0;
    *(uint4*)o = uint4{pack_bf16x2(col[0], col[1]), pack_bf16x2(col[2], col[3]), pack_bf16x2(col[4], col[5]),
                       pack_bf16x2(col[6], col[7])};
}

// backward, per sample: gaw / gloc (msda_bwd_kernel's per-channel arithmetic, channel sums over the lane's 8
// channels then the 8 lanes of the head), the softmax backward over the head's 8 samples, grad_off = gloc / hw
__global__ __launch_bounds__(64) void msda_train_bwd_samp_kernel(const bf16_t* __restrict__ value,
                                                                 const bf16_t* __restrict__ off,
                                                                 const bf16_t* __restrict__ awl,
                                                                 const float* __restrict__ ref,
                                                                 const bf16_t* __restrict__ gout,
                                                                 bf16_t* __restrict__ goff, bf16_t* __restrict__ gawl,
                                                                 int hw, int op, int ap) {
    const int nq = hw * hw;
    const int64_t row = blockIdx.x;
    const int b = (int)(row / nq), q = (int)(row % nq);
    const int t = threadIdx.x, m = t >> 3, cg = t & 7, c0 = cg * 8;
    float lg[8], a[8];
    mt_load_logits(awl + row * ap + m * 8, lg);
    mt_softmax8(lg, a);
    const float rx = ref[2 * q], ry = ref[2 * q + 1];
    const bf16_t* ob = off + row * op + m * (MT_NL * MT_NP * 2);
    float g[8];
    mt_unpack8(*(const uint4*)(gout + row * MT_CM + m * MT_DH + c0), g);
    float gaw[8], gx[8], gy[8];
#pragma unroll
    for (int l = 0; l < MT_NL; ++l) {
        const bf16_t* vb = value + ((int64_t)(b * MT_NL + l) * nq) * MT_CM + m * MT_DH + c0;
#pragma unroll
        for (int p = 0; p < MT_NP; ++p) {
            const int i = l * MT_NP + p;
            const MtGeom ge = mt_geom(rx, ry, bf2f(ob[2 * i]), bf2f(ob[2 * i + 1]), hw);
            float sa = 0.f, sx = 0.f, sy = 0.f;
            if (ge.in) {
                const int hl = (int)floorf(ge.h), wl = (int)floorf(ge.w), hh_ = hl + 1, wh_ = wl + 1;
                const float lh = ge.h - (float)hl, lw = ge.w - (float)wl, hh = 1.f - lh, hwt = 1.f - lw;
                const float w1 = hh * hwt, w2 = hh * lw, w3 = lh * hwt, w4 = lh * lw;
                const bool k1 = hl >= 0 && wl >= 0, k2 = hl >= 0 && wh_ <= hw - 1;
                const bool k3 = hh_ <= hw - 1 && wl >= 0, k4 = hh_ <= hw - 1 && wh_ <= hw - 1;
                float v1[8], v2[8], v3[8], v4[8];
                mt_unpack8(mt_ld(k1, vb + (hl * hw + wl) * MT_CM), v1);
                mt_unpack8(mt_ld(k2, vb + (hl * hw + wh_) * MT_CM), v2);
                mt_unpack8(mt_ld(k3, vb + (hh_ * hw + wl) * MT_CM), v3);
                mt_unpack8(mt_ld(k4, vb + (hh_ * hw + wh_) * MT_CM), v4);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float tg = g[j], tgv = tg * a[i];
                    float gh = 0.f, gw = 0.f;
                    if (k1) { gh -= hwt * v1[j]; gw -= hh * v1[j]; }
                    if (k2) { gh -= lw * v2[j]; gw += hh * v2[j]; }
                    if (k3) { gh += hwt * v3[j]; gw -= lh * v3[j]; }
                    if (k4) { gh += lw * v4[j]; gw += lh * v4[j]; }
                    sa += tg * (w1 * v1[j] + w2 * v2[j] + w3 * v3[j] + w4 * v4[j]);
                    sx += (float)hw * gw * tgv;
                    sy += (float)hw * gh * tgv;
                }
            }
            // the head's 8 lanes: xor 1, 2, 4 (every lane ends with the head's channel sum)
#pragma unroll
            for (int o = 1; o < 8; o <<= 1) {
                sa += __shfl_xor(sa, o, 64);
                sx += __shfl_xor(sx, o, 64);
                sy += __shfl_xor(sy, o, 64);
            }
            gaw[i] = sa;
            gx[i] = sx;
            gy[i] = sy;
        }
    }
    // softmax backward (torch: a * (grad - sum(grad * a)), the sum in the warp butterfly order)
    float ga[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) ga[i] = gaw[i] * a[i];
    const float s = ((ga[0] + ga[4]) + (ga[2] + ga[6])) + ((ga[1] + ga[5]) + (ga[3] + ga[7]));
    // lane cg of the head stores sample i = cg: its logit gradient and its two offset gradients
    float dl = 0.f, dx = 0.f, dy = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
        if (i == cg) dl = a[i] * (gaw[i] - s), dx = gx[i] / (float)hw, dy = gy[i] / (float)hw;
    gawl[row * ap + m * 8 + cg] = f2bf(dl);
    *(uint32_t*)(goff + row * op + (m * 8 + cg) * 2) = pack_bf16x2(dx, dy);
}

// backward, grad_value: one workgroup per (b, m, level) -- every sample of the level's nq queries expanded into its
// taps (counted per pixel, bucketed in (sample, tap) order), then per pixel and channel
// sum w_k * (g[q, c] * a) in that order: msda_bwd_value_kernel's order with the grad_out rows and the level's
// attention weights staged in LDS.  16 waves; lane = channel in the gather.
constexpr int MT_VT = 1024;
__global__ __launch_bounds__(MT_VT) void msda_train_bwd_value_kernel(const bf16_t* __restrict__ off,
                                                                     const bf16_t* __restrict__ awl,
                                                                     const float* __restrict__ ref,
                                                                     const bf16_t* __restrict__ gout,
                                                                     bf16_t* __restrict__ gvalue, int hw, int op, int ap) {
    __shared__ __attribute__((aligned(16))) bf16_t gl[MT_NQ_MAX * MT_DH];  // grad_out rows of head m
    __shared__ float al[MT_NQ_MAX * MT_NP];                                  // a of this level's points
    __shared__ int ekey[MT_NQ_MAX * MT_NP * 4];
    __shared__ float ew[MT_NQ_MAX * MT_NP * 4];
    __shared__ int cnt[MT_NQ_MAX + 2];
    __shared__ uint32_t tbl[(MT_VT / 64) * (MT_NQ_MAX / 2)];  // the 16 waves' packed (wave, pixel) counters
    const int nq = hw * hw, t = threadIdx.x;
    const int l = blockIdx.x, m = blockIdx.y, b = blockIdx.z;
    const int64_t row0 = (int64_t)b * nq;
    for (int i = t; i < nq * (MT_DH / 8); i += MT_VT) {  // 16-B pieces of the grad_out rows
        const int q = i >> 3, k = i & 7;
        *(uint4*)&gl[q * MT_DH + k * 8] = *(const uint4*)(gout + (row0 + q) * MT_CM + m * MT_DH + k * 8);
    }
    for (int q = t; q < nq; q += MT_VT) {
        float lg[8], a[8];
        mt_load_logits(awl + (row0 + q) * ap + m * 8, lg);
        mt_softmax8(lg, a);
#pragma unroll
        for (int p = 0; p < MT_NP; ++p) al[q * MT_NP + p] = a[l * MT_NP + p];
    }
    const int words = (nq + 1) / 2;
    for (int x = t; x < (MT_VT / 64) * words; x += MT_VT) tbl[x] = 0;
    __syncthreads();
    const int ns = nq * MT_NP;
    // the taps of sample j = q * 4 + p: f(k, pixel, w_k) for the valid ones (msda_bwd_value_kernel's rules)
    auto taps = [&](int j, auto&& f) {
        const int q = j >> 2, p = j & 3;
        const bf16_t* o = off + (row0 + q) * op + ((m * MT_NL + l) * MT_NP + p) * 2;
        const MtGeom g = mt_geom(ref[2 * q], ref[2 * q + 1], bf2f(o[0]), bf2f(o[1]), hw);
        if (!g.in) return;
        const int hl = (int)floorf(g.h), wl = (int)floorf(g.w), hh_ = hl + 1, wh_ = wl + 1;
        const float lh = g.h - (float)hl, lw = g.w - (float)wl, hh = 1.f - lh, hwt = 1.f - lw;
        const int r1 = hl * hw + wl;
        if (hl >= 0 && wl >= 0) f(0, r1, hh * hwt);
        if (hl >= 0 && wh_ <= hw - 1) f(1, r1 + 1, hh * lw);
        if (hh_ <= hw - 1 && wl >= 0) f(2, r1 + hw, lh * hwt);
        if (hh_ <= hw - 1 && wh_ <= hw - 1) f(3, r1 + hw + 1, lh * lw);
    };
    // items i = 4 j + k, a contiguous run per wave: counted, offsets, scanned, placed stably (no sort)
    const int wv = t >> 6, items = 4 * ns, per = (items + MT_VT - 1) / MT_VT * 64;
    const int i0 = min(wv * per, items), i1 = min(i0 + per, items);
    auto item = [&](int i, int& r, float& wk) {
        const int k = i & 3;
        taps(i >> 2, [&](int kk, int rr, float ww) {
            if (kk == k) r = rr, wk = ww;
        });
    };
    uint32_t* tw = tbl + wv * words;
    bucket_pass<9, float>(tw, cnt, i0, i1, false, item, [](int, int, float) {});
    __syncthreads();
    bucket_wave_offsets<MT_VT / 64>(tbl, words, cnt, MT_VT);
    __syncthreads();
    if (t < 64) {  // exclusive scan of the nq counts in place: lane t owns a run of ceil(nq / 64)
        const int per_l = (nq + 63) / 64, r0 = min(t * per_l, nq), r1 = min(r0 + per_l, nq);
        int sum = 0;
        for (int r = r0; r < r1; ++r) sum += cnt[r];
        int x = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (t >= o) x += y;
        }
        int run = x - sum;
        for (int r = r0; r < r1; ++r) {
            const int v = cnt[r];
            cnt[r] = run;
            run += v;
        }
        if (t == 63) cnt[nq] = x;
    }
    __syncthreads();
    bucket_pass<9, float>(tw, cnt, i0, i1, true, item, [&](int pos, int i, float wk) {
        ekey[pos] = i;
        ew[pos] = wk;
    });
    __syncthreads();
    // gather: wave w takes pixels w, w + 16, ... four at a time (independent sums in flight); lane = channel
    const int wave = t >> 6, c = t & 63;
    constexpr int NW = MT_VT / 64, PS = 4;
    bf16_t* gv = gvalue + ((int64_t)(b * MT_NL + l) * nq) * MT_CM + m * MT_DH + c;
    for (int r0 = wave; r0 < nq; r0 += NW * PS) {
        int e0[PS], e1[PS], len = 0;
        float acc[PS];
#pragma unroll
        for (int i = 0; i < PS; ++i) {
            const int r = r0 + i * NW;
            e0[i] = r < nq ? cnt[r] : 0;
            e1[i] = r < nq ? cnt[r + 1] : 0;
            len = max(len, e1[i] - e0[i]);
            acc[i] = 0.f;
        }
        if (len > BUCKET_LONG) {  // wave-uniform: pixel by pixel, 8 entries' loads in flight
#pragma unroll
            for (int i = 0; i < PS; ++i)
                acc[i] = bucket_sum<8>(e0[i], e1[i], acc[i], [&](int e) { return ew[e]; },
                                       [&](int e) { const int j = ekey[e] >> 2; return bf2f(gl[(j >> 2) * MT_DH + c]) * al[j]; });
        } else {
            for (int k = 0; k < len; ++k) {
#pragma unroll
                for (int i = 0; i < PS; ++i) {
                    const int e = e0[i] + k;
                    if (e < e1[i]) {
                        const int j = ekey[e] >> 2;
                        acc[i] = fma_(ew[e], bf2f(gl[(j >> 2) * MT_DH + c]) * al[j], acc[i]);
                    }
                }
            }
        }
#pragma unroll
        for (int i = 0; i < PS; ++i) {
            const int r = r0 + i * NW;
            if (r < nq) gv[(int64_t)r * MT_CM] = f2bf(acc[i]);
        }
    }
}

}  // namespace

extern "C" int mmt_msda_bimodal_train_fwd(const void* value, const void* off, int off_pitch, const void* awl,
                                          int awl_pitch, const float* ref, void* out, int B, int hw, void* stream) {
    if (!value || !off || !awl || !ref || !out || B <= 0 || hw <= 0 || hw * hw > MT_NQ_MAX) return MMT_EBADARG;
    if (off_pitch < 128 || off_pitch % 2 || awl_pitch < 64 || awl_pitch % 8) return MMT_EBADARG;
    if (((uintptr_t)value | (uintptr_t)awl | (uintptr_t)out) & 15 || (uintptr_t)off & 3) return MMT_EBADARG;
    hipLaunchKernelGGL(msda_train_fwd_kernel, dim3((unsigned)(B * hw * hw)), dim3(64), 0, (hipStream_t)stream,
                       (const bf16_t*)value, (const bf16_t*)off, (const bf16_t*)awl, ref, (bf16_t*)out, hw, off_pitch,
                       awl_pitch);
    return launch_status();
}

extern "C" int mmt_msda_bimodal_train_bwd(const void* value, const void* off, int off_pitch, const void* awl,
                                          int awl_pitch, const float* ref, const void* grad_out, void* grad_value,
                                          void* grad_off, void* grad_awl, int B, int hw, void* stream) {
    if (!value || !off || !awl || !ref || !grad_out || !grad_value || !grad_off || !grad_awl || B <= 0 || hw <= 0 ||
        hw * hw > MT_NQ_MAX)
        return MMT_EBADARG;
    if (off_pitch < 128 || off_pitch % 2 || awl_pitch < 64 || awl_pitch % 8) return MMT_EBADARG;
    if (((uintptr_t)value | (uintptr_t)awl | (uintptr_t)grad_out | (uintptr_t)grad_awl) & 15 ||
        ((uintptr_t)off | (uintptr_t)grad_off) & 3)
        return MMT_EBADARG;
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(msda_train_bwd_samp_kernel, dim3((unsigned)(B * hw * hw)), dim3(64), 0, st, (const bf16_t*)value,
                       (const bf16_t*)off, (const bf16_t*)awl, ref, (const bf16_t*)grad_out, (bf16_t*)grad_off,
                       (bf16_t*)grad_awl, hw, off_pitch, awl_pitch);
    hipLaunchKernelGGL(msda_train_bwd_value_kernel, dim3(MT_NL, MT_NH, (unsigned)B), dim3(MT_VT), 0, st,
                       (const bf16_t*)off, (const bf16_t*)awl, ref, (const bf16_t*)grad_out, (bf16_t*)grad_value, hw,
                       off_pitch, awl_pitch);
    return launch_status();
}

extern "C" int mmt_ms_deform_attn_backward_impl(const void* value, const int64_t* spatial_shapes,
                                                const int64_t* level_start, const void* sampling_loc,
                                                const void* attn_weight, const void* grad_output, void* grad_value,
                                                void* grad_loc, void* grad_attn, int N, int S, int M, int D, int Lq,
                                                int L, int P, int max_hw, int value_impl, int dtype, void* stream);

extern "C" int mmt_ms_deform_attn_backward(const void* value, const int64_t* spatial_shapes, const int64_t* level_start,
                                           const void* sampling_loc, const void* attn_weight, const void* grad_output,
                                           void* grad_value, void* grad_loc, void* grad_attn, int N, int S, int M, int D,
                                           int Lq, int L, int P, int dtype, void* stream) {
    // without the level sizes on the host, the per-level gather is taken when every level fits whatever its shape:
    // S (the pixels of all levels) bounds each level's
    return mmt_ms_deform_attn_backward_impl(value, spatial_shapes, level_start, sampling_loc, attn_weight, grad_output,
                                            grad_value, grad_loc, grad_attn, N, S, M, D, Lq, L, P, S, 0, dtype, stream);
}

extern "C" int mmt_ms_deform_attn_backward_impl(const void* value, const int64_t* spatial_shapes,
                                                const int64_t* level_start, const void* sampling_loc,
                                                const void* attn_weight, const void* grad_output, void* grad_value,
                                                void* grad_loc, void* grad_attn, int N, int S, int M, int D, int Lq,
                                                int L, int P, int max_hw, int value_impl, int dtype, void* stream) {
    if (!value || !spatial_shapes || !level_start || !sampling_loc || !attn_weight || !grad_output || !grad_value ||
        !grad_loc || !grad_attn)
        return MMT_EBADARG;
    if (N <= 0 || S <= 0 || M <= 0 || D <= 0 || Lq <= 0 || L <= 0 || P <= 0) return MMT_EBADARG;
    const size_t esz = dtype == MMT_F64 ? 8 : dtype == MMT_F32 ? 4 : 0;
    if (!esz) return MMT_EBADARG;
    hipStream_t st = (hipStream_t)stream;
    const int64_t nsamp = (int64_t)N * Lq * M;
    dim3 grid((unsigned)((nsamp + 3) / 4));
    // grad_value: the deterministic gather (msda_bwd_value_kernel) for up to 64 channels per head; wider heads
    // accumulate by float atomics inside msda_bwd_kernel.  grad_loc / grad_attn are fully written either way.
    const bool gather = D <= 64;
    if (!gather)
        if (const int e = zero_fill_async(grad_value, (size_t)N * S * M * D * esz, st)) return e;
    // the gather's grid: (chunks of MSDA_PIX pixels over the levels, heads, batch); the sum over levels of
    // ceil(HW_l / 64) is at most S / 64 + L (the shapes stay on the device: the kernel skips past the last)
    const dim3 vgrid((unsigned)(S / MSDA_PIX + L), (unsigned)M, (unsigned)N);
    // the per-(n, m, level) gather when the lists fit (value_impl 0 auto / 2 forced; 1 = the 64-pixel chunks)
    const bool nml_fits = (int64_t)Lq * P <= NML_S && max_hw <= NML_PIX && max_hw > 0;
    if (value_impl == 2 && !nml_fits) return MMT_EBADARG;
    const bool nml = gather && value_impl != 1 && nml_fits;
#define MSDA_BWD_CASE(T)                                                                                           \
    if (gather) {                                                                                                  \
        hipLaunchKernelGGL((msda_bwd_kernel<T, false>), grid, dim3(256), 0, st, (const T*)value, spatial_shapes,  \
                           level_start, (const T*)sampling_loc, (const T*)attn_weight, (const T*)grad_output,       \
                           (T*)grad_value, (T*)grad_loc, (T*)grad_attn, S, M, D, Lq, L, P, nsamp);                  \
        if (nml)                                                                                                   \
            hipLaunchKernelGGL((msda_bwd_value_nml_kernel<T>), dim3((unsigned)L, (unsigned)M, (unsigned)N),         \
                               dim3(NML_T), 0, st, (const T*)sampling_loc, (const T*)attn_weight,                   \
                               (const T*)grad_output, (T*)grad_value, spatial_shapes, level_start, S, M, D, Lq, L,  \
                               P);                                                                                  \
        else                                                                                                       \
            hipLaunchKernelGGL((msda_bwd_value_kernel<T>), vgrid, dim3(256), 0, st, (const T*)sampling_loc,       \
                               (const T*)attn_weight, (const T*)grad_output, (T*)grad_value, spatial_shapes,        \
                               level_start, S, M, D, Lq, L, P);                                                     \
    } else {                                                                                                       \
        hipLaunchKernelGGL((msda_bwd_kernel<T, true>), grid, dim3(256), 0, st, (const T*)value, spatial_shapes,   \
                           level_start, (const T*)sampling_loc, (const T*)attn_weight, (const T*)grad_output,       \
                           (T*)grad_value, (T*)grad_loc, (T*)grad_attn, S, M, D, Lq, L, P, nsamp);                  \
    }
    if (dtype == MMT_F32) { MSDA_BWD_CASE(float) }
    else { MSDA_BWD_CASE(double) }
#undef MSDA_BWD_CASE
    return launch_status();
}

extern "C" int mmt_ms_deform_attn_forward(const void* value, const int64_t* spatial_shapes, const int64_t* level_start,
                                          const void* sampling_loc, const void* attn_weight, void* out, int N, int S,
                                          int M, int D, int Lq, int L, int P, int dtype, void* stream) {
    if (!value || !spatial_shapes || !level_start || !sampling_loc || !attn_weight || !out) return MMT_EBADARG;
    if (N <= 0 || S <= 0 || M <= 0 || D <= 0 || Lq <= 0 || L <= 0 || P <= 0) return MMT_EBADARG;
    const int64_t total = (int64_t)N * Lq * M * D;
    const int64_t want = (total + 255) / 256;
    dim3 grid((unsigned)(want < 65536 ? want : 65536));
    hipStream_t st = (hipStream_t)stream;
#define MSDA_CASE(T)                                                                                            \
    hipLaunchKernelGGL((msda_generic_kernel<T>), grid, dim3(256), 0, st, (const T*)value, spatial_shapes,     \
                       level_start, (const T*)sampling_loc, (const T*)attn_weight, (T*)out, N, S, M, D, Lq, L, P, \
                       total)
    if (dtype == MMT_F32) MSDA_CASE(float);
    else if (dtype == MMT_F64) MSDA_CASE(double);
    else if (dtype == MMT_BF16) MSDA_CASE(bf16_t);
    else return MMT_EBADARG;
#undef MSDA_CASE
    return launch_status();
}

extern "C" int mmt_msda_bimodal(const float* offw, const void* value, void* out, int B, int hw, int dtype,
                                void* stream) {
    if (!offw || !value || !out || B <= 0 || hw <= 0) return MMT_EBADARG;
    if (((uintptr_t)value | (uintptr_t)out) & 15) return MMT_EBADARG;  // 16-byte channel vectors
    const int64_t rows = (int64_t)B * hw * hw;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == MMT_BF16)  // one query per workgroup: one wave (bf16) / two (fp32)
        hipLaunchKernelGGL((msda_bimodal_kernel<bf16_t>), dim3((unsigned)rows), dim3(64), 0, st, offw,
                           (const bf16_t*)value, (bf16_t*)out, B, hw);
    else if (dtype == MMT_F16)
        hipLaunchKernelGGL((msda_bimodal_kernel<f16_t>), dim3((unsigned)rows), dim3(64), 0, st, offw,
                           (const f16_t*)value, (f16_t*)out, B, hw);
    else if (dtype == MMT_F32)
        hipLaunchKernelGGL((msda_bimodal_kernel<float>), dim3((unsigned)rows), dim3(128), 0, st, offw,
                           (const float*)value, (float*)out, B, hw);
    else return MMT_EBADARG;
    return launch_status();
}
