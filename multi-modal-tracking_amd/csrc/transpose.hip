// bf16 matrix transpose for the training step's weight-gradient GEMMs.
//
// The LDS-DMA GEMM contracts over the contiguous dimension of both operands (C = A W^T, A [M][K],
// W [N][K]).  A Linear's backward needs dX = dY W (contract over N) and dW = dY^T X (contract over
// the token dimension M), so W, dY and X are transposed first: out[c][r] = in[r][c] for a
// rows x cols bf16 matrix with leading dimensions ld_in / ld_out (elements), `batch` matrices
// stride_in / stride_out apart.  64 x 64 tiles through LDS: 16-B loads along the input rows and
// 16-B stores along the output rows, both coalesced; HBM-bound (2 bytes read + 2 written per
// element).
#include "common.hpp"

namespace {

constexpr int TT = 64, PITCH = TT + 2;  // tile edge, LDS row pitch (u16): odd word stride

// fill (mmt_transpose_bf16): 0 only out[c][r] for r < rows; 1 also the padding columns r in [rows, ld_out)
// as zeros; 2 also 8 appended output rows: row `cols` = 1 for r < rows (else 0), rows cols+1.. zero
// (the ones row that gives a GEMM against the result the row sums of its other operand).  Out-of-range
// input is read as those values, so the whole padded output is written in one pass.
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16_t* __restrict__ in, bf16_t* __restrict__ out,
                                                             int rows, int cols, int64_t ld_in, int64_t ld_out,
                                                             int64_t stride_in, int64_t stride_out, int fill) {
    __shared__ uint16_t tile[TT * PITCH];
    const int r0 = blockIdx.y * TT, c0 = blockIdx.x * TT;
    const int ocols = cols + (fill == 2 ? 8 : 0);                // output rows written
    const int orows = fill >= 1 ? (int)ld_out : rows;             // output columns written
    in += blockIdx.z * stride_in;
    out += blockIdx.z * stride_out;
    const bool vec_in = (cols & 7) == 0 && (ld_in & 7) == 0;
    const bool vec_out = ((fill >= 1 ? (int)ld_out : rows) & 7) == 0 && (ld_out & 7) == 0;
#pragma unroll
    for (int i = 0; i < 2; ++i) {  // 512 chunks of 8 elements: tile row r, columns 8ch..8ch+7
        const int idx = threadIdx.x + 256 * i, r = idx >> 3, ch = idx & 7;
        const int gr = r0 + r, gc = c0 + 8 * ch;
        uint16_t v[8];
        if (gr < rows && vec_in && gc + 8 <= cols) {
            const u32x4 u = *(const u32x4*)(in + (int64_t)gr * ld_in + gc);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[2 * e] = (uint16_t)(u[e] & 0xffffu), v[2 * e + 1] = (uint16_t)(u[e] >> 16);
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e)
                v[e] = (gr < rows && gc + e < cols) ? in[(int64_t)gr * ld_in + gc + e]
                       : (fill == 2 && gr < rows && gc + e == cols) ? (uint16_t)0x3f80u  // bf16 1.0
                                                                   : (uint16_t)0;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) tile[r * PITCH + 8 * ch + e] = v[e];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 2; ++i) {  // output row = input column c, elements = input rows 8ch..8ch+7
        const int idx = threadIdx.x + 256 * i, c = idx >> 3, ch = idx & 7;
        const int oc = c0 + c, orow = r0 + 8 * ch;
        if (oc >= ocols) continue;
        uint16_t v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = tile[(8 * ch + e) * PITCH + c];
        if (vec_out && orow + 8 <= orows) {
            u32x4 u;
#pragma unroll
            for (int e = 0; e < 4; ++e) u[e] = (uint32_t)v[2 * e] | ((uint32_t)v[2 * e + 1] << 16);
            *(u32x4*)(out + (int64_t)oc * ld_out + orow) = u;
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e)
                if (orow + e < orows) out[(int64_t)oc * ld_out + orow + e] = v[e];
        }
    }
}

}  // namespace

extern "C" int mmt_transpose_bf16(const void* in, void* out, int rows, int cols, int64_t ld_in, int64_t ld_out,
                                  int batch, int64_t stride_in, int64_t stride_out, int fill, void* stream) {
    if (!in || !out || rows <= 0 || cols <= 0 || batch <= 0 || ld_in < cols || ld_out < rows) return MMT_EBADARG;
    if (fill < 0 || fill > 2 || ld_out > INT32_MAX || (fill == 2 && batch != 1)) return MMT_EBADARG;
    if (((uintptr_t)in | (uintptr_t)out) & 15) return MMT_EBADARG;
    const int ocols = cols + (fill == 2 ? 8 : 0);
    const int64_t orows = fill >= 1 ? ld_out : rows;
    const dim3 grid((ocols + TT - 1) / TT, (unsigned)((orows + TT - 1) / TT), batch);
    hipLaunchKernelGGL(transpose_bf16_kernel, grid, dim3(256), 0, (hipStream_t)stream, (const bf16_t*)in, (bf16_t*)out,
                       rows, cols, ld_in, ld_out, stride_in, stride_out, fill);
    return launch_status();
}

// 3x3 / pad-1 im2col of an NHWC bf16 map for the corner head's weight-gradient GEMMs (training step):
// out[(b, y, x)][(ky * 3 + kx) * C + c] = in[b][y + ky - 1][x + kx - 1][c], 0 outside the map -- the A
// operand layout of the implicit-GEMM conv (k = (ky * 3 + kx) * C + ci), materialised so that
// dW = dY^T im2col(X) is one GEMM contracting over pixels.  One thread per 16 B (8 channels): coalesced
// 16-B loads and stores, HBM-bound (9 x the map written, the map read ~9 x from L2).  UP: the conv's input is
// the nearest-upsampled (x UP, a power of two) map of in [B][H/UP][W/UP][C] -- H, W are the upsampled sizes:
// the pixel (yy, xx) reads in[yy / UP][xx / UP] (round 6: the head's upsampling folded into the convs).
namespace {
__global__ __launch_bounds__(256) void im2col3x3_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out, int H,
                                                         int W, int c8, int64_t total, int up_sh) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (pixel, tap, chunk)
    if (i >= total) return;
    const int ch = (int)(i % c8);
    const int64_t pt = i / c8;
    const int tap = (int)(pt % 9);
    const int64_t pix = pt / 9;
    const int x = (int)(pix % W), y = (int)((pix / W) % H);
    const int64_t b = pix / ((int64_t)W * H);
    const int yy = y + tap / 3 - 1, xx = x + tap % 3 - 1;
    const int hi = H >> up_sh, wi = W >> up_sh;
    u32x4 v = u32x4{0u, 0u, 0u, 0u};
    if (yy >= 0 && yy < H && xx >= 0 && xx < W) v = in[((b * hi + (yy >> up_sh)) * wi + (xx >> up_sh)) * c8 + ch];
    out[i] = v;
}

// Backward of nearest upsampling x UP on NHWC bf16: out[b][y][x][c] = bf16(sum over the UP x UP block of
// in[b][UP y + dy][UP x + dx][c]) (fp32 sums, rows then columns: a fixed order); one thread per 8 channels
__global__ __launch_bounds__(256) void upsample_sum_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out, int Hi,
                                                            int Wi, int c8, int up, int64_t total) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (low-res pixel, chunk)
    if (i >= total) return;
    const int ch = (int)(i % c8);
    const int64_t pix = i / c8;
    const int x = (int)(pix % Wi), y = (int)((pix / Wi) % Hi);
    const int64_t b = pix / ((int64_t)Wi * Hi);
    const int W = Wi * up, H = Hi * up;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int dy = 0; dy < up; ++dy)
        for (int dx = 0; dx < up; ++dx) {
            const u32x4 v = in[((b * H + (int64_t)y * up + dy) * W + (int64_t)x * up + dx) * c8 + ch];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc[2 * j] += __uint_as_float(v[j] << 16);
                acc[2 * j + 1] += __uint_as_float(v[j] & 0xffff0000u);
            }
        }
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = pack_bf16x2(acc[2 * j], acc[2 * j + 1]);
    out[i] = o;
}

// out = bf16(up(a) + b) on NHWC bf16 maps: a [B][H/UP][W/UP][C], b / out [B][H][W][C] (fp32 add): the corner
// head's pyramid input x4 = up2(adjust2) + x3 (head.py:189), before the conv that upsamples it once more
__global__ __launch_bounds__(256) void add_up_kernel(const u32x4* __restrict__ a, const u32x4* __restrict__ bm,
                                                      u32x4* __restrict__ out, int H, int W, int c8, int up_sh,
                                                      int64_t total) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (pixel, chunk)
    if (i >= total) return;
    const int ch = (int)(i % c8);
    const int64_t pix = i / c8;
    const int x = (int)(pix % W), y = (int)((pix / W) % H);
    const int64_t b = pix / ((int64_t)W * H);
    const u32x4 va = a[((b * (H >> up_sh) + (y >> up_sh)) * (W >> up_sh) + (x >> up_sh)) * c8 + ch], vb = bm[i];
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        o[j] = pack_bf16x2(__uint_as_float(va[j] << 16) + __uint_as_float(vb[j] << 16),
                           __uint_as_float(va[j] & 0xffff0000u) + __uint_as_float(vb[j] & 0xffff0000u));
    out[i] = o;
}

// The same im2col with channel-major columns: out[pix][c * 9 + ky * 3 + kx] -- PyTorch's Conv2d weight order
// [Cout][Cin][3][3], so the dW GEMM against it writes the parameter's gradient in place (no permute pass).
// One thread per (pixel, 8 channels): nine 16-B tap loads (as im2col3x3_kernel), the 8 x 9 transpose in
// registers -> its 144 contiguous output bytes; the wave's 64 x 144 B (contiguous: items are consecutive) go
// out through LDS so that every 16-B store instruction covers 1 KiB of consecutive bytes.
__global__ __launch_bounds__(256) void im2col3x3_cm_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out, int H,
                                                            int W, int c8, int64_t total, int up_sh) {
    __shared__ u32x4 stage[4][64 * 9];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (pixel, chunk)
    uint16_t e[72];                                               // e[c * 9 + tap]
    if (i < total) {
        const int ch = (int)(i % c8);
        const int64_t pix = i / c8;
        const int x = (int)(pix % W), y = (int)((pix / W) % H);
        const int64_t b = pix / ((int64_t)W * H);
        const int hi = H >> up_sh, wi = W >> up_sh;
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const int yy = y + tap / 3 - 1, xx = x + tap % 3 - 1;
            u32x4 v = u32x4{0u, 0u, 0u, 0u};
            if (yy >= 0 && yy < H && xx >= 0 && xx < W) v = in[((b * hi + (yy >> up_sh)) * wi + (xx >> up_sh)) * c8 + ch];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                e[(2 * j) * 9 + tap] = (uint16_t)(v[j] & 0xffffu);
                e[(2 * j + 1) * 9 + tap] = (uint16_t)(v[j] >> 16);
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < 72; ++k) e[k] = 0;
    }
#pragma unroll
    for (int q = 0; q < 9; ++q)
        stage[wave][lane * 9 + q] =
            u32x4{(uint32_t)e[8 * q] | ((uint32_t)e[8 * q + 1] << 16), (uint32_t)e[8 * q + 2] | ((uint32_t)e[8 * q + 3] << 16),
                  (uint32_t)e[8 * q + 4] | ((uint32_t)e[8 * q + 5] << 16), (uint32_t)e[8 * q + 6] | ((uint32_t)e[8 * q + 7] << 16)};
    __syncthreads();
    const int64_t base = ((int64_t)blockIdx.x * 256 + wave * 64) * 9, end = total * 9;
#pragma unroll
    for (int s = 0; s < 9; ++s) {
        const int g = 64 * s + lane;
        if (base + g < end) out[base + g] = stage[wave][g];
    }
}

// The corner head's 3x3 conv weights, fp32 [Cout][Cin][3][3], to the two bf16 operand layouts of the training
// convs, for up to MMT_WPREP_MAX convs in one launch: wf [Cp][ky][kx][Cin] (forward: the implicit-GEMM conv's W)
// and wb [Cin][ky][kx][Cp] (dX: the flipped-tap conv's W), rows / columns co in [Cout, Cp) zero, and bp [Cp]
// fp32 = the bias padded with zeros (when given).  Workgroups [blk0[i], blk0[i+1]) serve conv i: the first half
// one thread per (co, ci) of the forward layout (adjacent threads: adjacent ci), the second per (ci, co) of the
// backward layout (adjacent co), so both stores are coalesced; the reads (9 contiguous floats) go through L2.
constexpr int WP_CO = 64, WP_CI = 16;  // the backward layout's LDS tile: 64 output x 16 input channels x 9 taps
__global__ __launch_bounds__(256) void conv_wprep_kernel(mmt_conv_wprep_batch bt) {
    __shared__ float tile[WP_CO * WP_CI * 9];
    int i = 0;
    while (i + 1 < bt.n && (int)blockIdx.x >= bt.blk0[i + 1]) ++i;
    const mmt_conv_wprep& c = bt.item[i];
    const int64_t half = (int64_t)c.cp * c.cin;
    const int64_t nb = (half + 255) / 256;
    const int64_t blk = (int64_t)blockIdx.x - bt.blk0[i];
    bf16_t* wf = (bf16_t*)c.wf;
    bf16_t* wb = (bf16_t*)c.wb;
    if (blk < nb) {  // forward layout: thread per (co, ci), 9 contiguous floats in, 9 column stores (adjacent ci)
        // (an LDS-staged row-piece form measured slower: 83 vs 68 us for the head's 22 convs, r06af / r06ae)
        const int64_t t = blk * 256 + threadIdx.x;
        if (t >= half) return;
        const int co = (int)(t / c.cin), ci = (int)(t % c.cin);
        float v[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) v[k] = co < c.cout ? c.w[((int64_t)co * c.cin + ci) * 9 + k] : 0.f;
#pragma unroll
        for (int k = 0; k < 9; ++k) wf[((int64_t)co * 9 + k) * c.cin + ci] = f2bf(v[k]);
        if (ci == 0 && c.bp) c.bp[co] = (co < c.cout && c.b) ? c.b[co] : 0.f;
        return;
    }
    // backward layout, one (64 co x 16 ci) tile: each co's 16 x 9 contiguous floats read row by row into LDS,
    // then wb[ci][k][co0 .. co0 + 64) stored as 128-B runs (round 6: one thread per (ci, co) read 9 floats from a
    // different row per lane, ~1 TB/s)
    const int ntc = (c.cp + WP_CO - 1) / WP_CO;
    const int tb = (int)(blk - nb), co0 = (tb % ntc) * WP_CO, ci0 = (tb / ntc) * WP_CI;
    const int nci = min(WP_CI, c.cin - ci0);
    for (int e = threadIdx.x; e < WP_CO * WP_CI * 9; e += 256) {
        const int r = e / (WP_CI * 9), q = e % (WP_CI * 9), co = co0 + r;  // q = ci_local * 9 + k
        tile[e] = (co < c.cout && q < nci * 9) ? c.w[((int64_t)co * c.cin + ci0) * 9 + q] : 0.f;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < WP_CI * 9 * (WP_CO / 2); e += 256) {
        const int j = e % (WP_CO / 2), q = e / (WP_CO / 2);  // q = ci_local * 9 + k; co pair j
        const int co = co0 + 2 * j;
        if (q >= nci * 9 || co >= c.cp) continue;
        const int cl = q / 9, k = q % 9;
        const uint32_t u = pack_bf16x2(tile[(2 * j) * WP_CI * 9 + q], tile[(2 * j + 1) * WP_CI * 9 + q]);
        *(uint32_t*)(wb + ((int64_t)(ci0 + cl) * 9 + k) * c.cp + co) = u;
    }
}
}  // namespace

static int up_shift(int up) {
    return up == 1 ? 0 : up == 2 ? 1 : up == 4 ? 2 : up == 8 ? 3 : -1;
}

extern "C" int mmt_im2col3x3_up_bf16(const void* in, void* out, int B, int H, int W, int C, int up, void* stream) {
    const int sh = up_shift(up);
    if (!in || !out || B <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 8 || sh < 0 || H % up || W % up) return MMT_EBADARG;
    if (((uintptr_t)in | (uintptr_t)out) & 15) return MMT_EBADARG;
    const int c8 = C / 8;
    const int64_t total = (int64_t)B * H * W * 9 * c8;
    hipLaunchKernelGGL(im2col3x3_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       (const u32x4*)in, (u32x4*)out, H, W, c8, total, sh);
    return launch_status();
}

extern "C" int mmt_upsample_sum_bf16(const void* in, void* out, int B, int Hi, int Wi, int C, int up, void* stream) {
    if (!in || !out || B <= 0 || Hi <= 0 || Wi <= 0 || C <= 0 || C % 8 || up_shift(up) < 0) return MMT_EBADARG;
    if (((uintptr_t)in | (uintptr_t)out) & 15) return MMT_EBADARG;
    const int c8 = C / 8;
    const int64_t total = (int64_t)B * Hi * Wi * c8;
    hipLaunchKernelGGL(upsample_sum_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       (const u32x4*)in, (u32x4*)out, Hi, Wi, c8, up, total);
    return launch_status();
}

extern "C" int mmt_add_up_bf16(const void* a, const void* b, void* out, int B, int H, int W, int C, int up, void* stream) {
    const int sh = up_shift(up);
    if (!a || !b || !out || B <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 8 || sh < 0 || H % up || W % up) return MMT_EBADARG;
    if (((uintptr_t)a | (uintptr_t)b | (uintptr_t)out) & 15) return MMT_EBADARG;
    const int c8 = C / 8;
    const int64_t total = (int64_t)B * H * W * c8;
    hipLaunchKernelGGL(add_up_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       (const u32x4*)a, (const u32x4*)b, (u32x4*)out, H, W, c8, sh, total);
    return launch_status();
}

extern "C" int mmt_im2col3x3_bf16(const void* in, void* out, int B, int H, int W, int C, void* stream) {
    if (!in || !out || B <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 8) return MMT_EBADARG;
    if (((uintptr_t)in | (uintptr_t)out) & 15) return MMT_EBADARG;
    const int c8 = C / 8;
    const int64_t total = (int64_t)B * H * W * 9 * c8;
    hipLaunchKernelGGL(im2col3x3_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       (const u32x4*)in, (u32x4*)out, H, W, c8, total, 0);
    return launch_status();
}

extern "C" int mmt_im2col3x3_cm_bf16(const void* in, void* out, int B, int H, int W, int C, int up, void* stream) {
    const int sh = up_shift(up);
    if (!in || !out || B <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 8 || sh < 0 || H % up || W % up) return MMT_EBADARG;
    if (((uintptr_t)in | (uintptr_t)out) & 15) return MMT_EBADARG;
    const int c8 = C / 8;
    const int64_t total = (int64_t)B * H * W * c8;
    hipLaunchKernelGGL(im2col3x3_cm_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       (const u32x4*)in, (u32x4*)out, H, W, c8, total, sh);
    return launch_status();
}

extern "C" int mmt_conv3x3_wprep(const mmt_conv_wprep* items, int n, void* stream) {
    if (!items || n <= 0 || n > MMT_WPREP_MAX) return MMT_EBADARG;
    mmt_conv_wprep_batch bt;
    bt.n = n;
    int64_t blocks = 0;
    for (int i = 0; i < n; ++i) {
        const mmt_conv_wprep& c = items[i];
        if (!c.w || !c.wf || !c.wb || c.cout <= 0 || c.cin <= 0 || c.cp < c.cout || c.cp % 2) return MMT_EBADARG;
        bt.item[i] = c;
        bt.blk0[i] = (int)blocks;
        blocks += ((int64_t)c.cp * c.cin + 255) / 256 + (int64_t)((c.cp + WP_CO - 1) / WP_CO) * ((c.cin + WP_CI - 1) / WP_CI);
        if (blocks > INT32_MAX) return MMT_EBADARG;
    }
    hipLaunchKernelGGL(conv_wprep_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, bt);
    return launch_status();
}
