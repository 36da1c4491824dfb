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
