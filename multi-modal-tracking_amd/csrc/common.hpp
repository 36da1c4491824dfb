// Shared device helpers for the gfx950 (CDNA4) kernels of libmmt_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mmt_hip.h"

typedef uint16_t bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

#define MMT_DEV __device__ __forceinline__

MMT_DEV float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
MMT_DEV bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }

template <typename T> MMT_DEV float to_f(T v);
template <> MMT_DEV float to_f<float>(float v) { return v; }
template <> MMT_DEV float to_f<bf16_t>(bf16_t v) { return bf2f(v); }
template <typename T> MMT_DEV T from_f(float v);
template <> MMT_DEV float from_f<float>(float v) { return v; }
template <> MMT_DEV bf16_t from_f<bf16_t>(float v) { return f2bf(v); }

// Two floats -> packed bf16 pair (RNE), lo in bits 0-15.  Whole-vector conversion: a per-element
// bit_cast between 16-bit types has been seen to miscompile.
MMT_DEV uint32_t pack_bf16x2(float lo, float hi) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{lo, hi}, bf16x2));
}

// fp16 storage (MMT_F16; BASELINE config 5): the same 2-byte layouts and MFMA shapes as bf16
// (v_mfma_f32_*_f16 issue at the bf16 rate), 11-bit significand, range +-65504.  Kernels that
// take either 16-bit type are templated on the storage type T (bf16_t or f16_t) and reach the
// type through the helpers below.
typedef _Float16 f16_t;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
template <> MMT_DEV float to_f<f16_t>(f16_t v) { return (float)v; }
template <> MMT_DEV f16_t from_f<f16_t>(float v) { return (f16_t)v; }
MMT_DEV uint32_t pack_f16x2(float lo, float hi) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{lo, hi}, f16x2));
}
template <typename T> MMT_DEV uint32_t pack2(float lo, float hi);
template <> MMT_DEV uint32_t pack2<bf16_t>(float lo, float hi) { return pack_bf16x2(lo, hi); }
template <> MMT_DEV uint32_t pack2<f16_t>(float lo, float hi) { return pack_f16x2(lo, hi); }
// the two 16-bit values of a dword (lo = bits 0-15) as floats
template <typename T> MMT_DEV f32x2 unpack2(uint32_t u);
template <> MMT_DEV f32x2 unpack2<bf16_t>(uint32_t u) { return f32x2{__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)}; }
template <> MMT_DEV f32x2 unpack2<f16_t>(uint32_t u) {
    return __builtin_convertvector(__builtin_bit_cast(f16x2, u), f32x2);
}
// MFMA on 8 packed 16-bit values per lane (operand order as the builtins)
template <typename T> MMT_DEV f32x4 mfma16x16x32(u32x4 a, u32x4 b, f32x4 c);
template <> MMT_DEV f32x4 mfma16x16x32<bf16_t>(u32x4 a, u32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
template <> MMT_DEV f32x4 mfma16x16x32<f16_t>(u32x4 a, u32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}
// 1.0 in both halves of a dword
template <typename T> constexpr uint32_t one2() { return sizeof(T) == 2 && __is_same(T, f16_t) ? 0x3c003c00u : 0x3f803f80u; }

// GELU(x) = x/2 (1 + erf(x/sqrt2)) with a branch-free erf (Abramowitz-Stegun 7.1.26, |error| <=
// 1.5e-7): libm erff branches on |x|, which in a 64-value epilogue means 64 divergent regions.
// t comes from v_rcp_f32 (1 ulp): an IEEE division is a 10-instruction sequence per element.
MMT_DEV float erf_fast(float x) {
    const float a = fabsf(x), t = __builtin_amdgcn_rcpf(1.0f + 0.3275911f * a);
    const float y = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
    return copysignf(1.0f - y * __expf(-a * a), x);
}
MMT_DEV float gelu_erf(float x) { return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752440f)); }

// gelu_erf on two values at once: the same approximation with the polynomial, the exponent
// argument and the final scale as packed fp32 ops (v_pk_fma_f32 / v_pk_mul_f32 issue two lanes'
// worth of fp32 per slot), leaving only v_rcp / v_exp per element.  The GEMM epilogue evaluates 64
// of these per thread with one wave per SIMD, so its VALU issue count is what the fc1 tail costs.
MMT_DEV f32x2 gelu_erf2(f32x2 x) {
    const f32x2 z = x * 0.70710678118654752440f;
    const f32x2 a = __builtin_elementwise_abs(z);
    const f32x2 d = __builtin_elementwise_fma(a, f32x2(0.3275911f), f32x2(1.0f));
    const f32x2 t = {__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
    f32x2 y = __builtin_elementwise_fma(t, f32x2(1.061405429f), f32x2(-1.453152027f));
    y = __builtin_elementwise_fma(y, t, f32x2(1.421413741f));
    y = __builtin_elementwise_fma(y, t, f32x2(-0.284496736f));
    y = __builtin_elementwise_fma(y, t, f32x2(0.254829592f));
    y = y * t;
    const f32x2 q = a * (a * -1.44269504088896340736f);  // -a^2 log2(e)
    const f32x2 e = {__builtin_amdgcn_exp2f(q[0]), __builtin_amdgcn_exp2f(q[1])};
    const f32x2 r = __builtin_elementwise_fma(-y, e, f32x2(1.0f));  // erf(|z|)
    const f32x2 h = x * 0.5f;
    // GELU = h (1 + sign(z) erf|z|); sign(z) = sign(x)
    const f32x2 s = {copysignf(r[0], x[0]), copysignf(r[1], x[1])};
    return __builtin_elementwise_fma(h, s, h);
}

// d GELU(x) / dx = Phi(x) + x phi(x) for two values, with gelu_erf2's erf approximation:
// Phi(x) = 0.5 (1 + sign(x) erf(|x| / sqrt 2)), phi(x) = exp(-x^2 / 2) / sqrt(2 pi) (the same exponential)
MMT_DEV f32x2 gelu_erf_grad2(f32x2 x) {
    const f32x2 z = x * 0.70710678118654752440f;
    const f32x2 a = __builtin_elementwise_abs(z);
    const f32x2 d = __builtin_elementwise_fma(a, f32x2(0.3275911f), f32x2(1.0f));
    const f32x2 t = {__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
    f32x2 y = __builtin_elementwise_fma(t, f32x2(1.061405429f), f32x2(-1.453152027f));
    y = __builtin_elementwise_fma(y, t, f32x2(1.421413741f));
    y = __builtin_elementwise_fma(y, t, f32x2(-0.284496736f));
    y = __builtin_elementwise_fma(y, t, f32x2(0.254829592f));
    y = y * t;
    const f32x2 q = a * (a * -1.44269504088896340736f);
    const f32x2 e = {__builtin_amdgcn_exp2f(q[0]), __builtin_amdgcn_exp2f(q[1])};  // exp(-x^2 / 2)
    const f32x2 r = __builtin_elementwise_fma(-y, e, f32x2(1.0f));                  // erf(|z|)
    const f32x2 s = {copysignf(r[0], x[0]), copysignf(r[1], x[1])};
    const f32x2 phi = __builtin_elementwise_fma(s, f32x2(0.5f), f32x2(0.5f));        // Phi(x)
    return __builtin_elementwise_fma(x * 0.39894228040143267794f, e, phi);
}

MMT_DEV float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
MMT_DEV float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Reductions over the 4 lane groups (lanes l, l^16, l^32, l^48) of an MFMA 16x16 fragment layout:
// gfx950 v_permlane32_swap / v_permlane16_swap (VALU) instead of ds_bpermute round trips through
// the LDS pipe.
MMT_DEV float lanegroup_max(float v) {
    auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
MMT_DEV float lanegroup_sum(float v) {
    auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// Sum over each aligned group of 8 consecutive lanes, every lane receiving its group's sum: DPP
// (VALU) row moves -- quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror -- instead of
// ds_bpermute round trips.
template <int CTRL>
MMT_DEV float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
MMT_DEV float sum8_lanes(float v) {
    v += dpp_f<0xB1>(v);
    v += dpp_f<0x4E>(v);
    return v + dpp_f<0x141>(v);
}

// Block-wide sum for blockDim.x == NT (multiple of 64); `red` needs NT/64 floats of LDS.
template <int NT>
MMT_DEV float block_sum(float v, float* red) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) t += red[i];
    return t;
}
template <int NT>
MMT_DEV float block_max(float v, float* red) {
    v = wave_max(v);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    float t = -INFINITY;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) t = fmaxf(t, red[i]);
    return t;
}

// Workgroup barrier for LDS hand-offs that leaves global loads in flight: waits only for this
// wave's LDS operations (lgkmcnt), unlike __syncthreads(), whose fence makes hipcc drain vmcnt(0)
// and so serialises any register prefetch ring.  The "memory" clobber keeps LDS accesses on
// their side of the barrier.
// The wait is the s_waitcnt builtin (gfx9 encoding: lgkmcnt 0, vmcnt / expcnt at their maximum)
// rather than inline asm so that hipcc's wait-count tracking knows the LDS reads are retired (it
// otherwise re-waits for them later, and with >15 newer LDS reads outstanding it can only
// express that as lgkmcnt(0)).
MMT_DEV void lds_barrier() {
    __builtin_amdgcn_s_waitcnt(0xc07f);
    asm volatile("s_barrier" ::: "memory");
}

// Measurement builds only (tools/build_ablate.sh, MMT_STAMP_BUILD=1): the leader thread of each
// workgroup records clock stamps into a per-kernel __device__ array, read back by an exported
// mmt_*_stamps() (tools/gemm_stamps.py, tools/attn_stamps.py).  Compiled out of the product.
#ifndef MMT_STAMP_BUILD
#define MMT_STAMP_BUILD 0
#endif
#if MMT_STAMP_BUILD
#define MMT_STAMP_AT(BUF, I, INSN)                                                                  \
    if (threadIdx.x == 0) {                                                                        \
        unsigned long long t_;                                                                     \
        asm volatile(INSN " %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                      \
        BUF[(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) * 8 + (I)] = t_;       \
    }
#else
#define MMT_STAMP_AT(BUF, I, INSN)
#endif

static inline int hip_status(hipError_t e) { return e == hipSuccess ? 0 : -(int)e; }
static inline int launch_status() { return hip_status(hipGetLastError()); }

// Zero a device buffer with a kernel instead of hipMemsetAsync: a memset captured into a hipGraph
// was not re-applied on replay for the MSDA gradient buffer (ROCm 7.2; replay 0 exact, later replays
// accumulated onto the previous replay's sums: tools/graph_replay_debug.py), a kernel is.
static __global__ __launch_bounds__(256) void mmt_zero_fill_kernel(uint32_t* __restrict__ p, int64_t n, int vec) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (vec) {
        const int64_t n4 = n / 4;
        if (i < n4) ((uint4*)p)[i] = uint4{0u, 0u, 0u, 0u};
        if (i < n - 4 * n4) p[4 * n4 + i] = 0u;  // the < 4 tail words, block 0
    } else if (i < n) {
        p[i] = 0u;
    }
}
// bytes: a multiple of 4
static inline int zero_fill_async(void* p, size_t bytes, hipStream_t st) {
    const int64_t n = (int64_t)(bytes / 4);
    if (n <= 0) return 0;
    const int vec = (((uintptr_t)p) & 15) == 0;
    const int64_t items = vec ? (n / 4 > 4 ? n / 4 : 4) : n;
    hipLaunchKernelGGL(mmt_zero_fill_kernel, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, st, (uint32_t*)p, n, vec);
    return launch_status();
}
