// Prototype (tools only): the 256x256 four-wave bf16 tile of gemm256.hip with REGISTER-STAGED operand loads
// instead of LDS-DMA: per 64-deep K-step every thread loads 16 x 16 B (buffer_load_dwordx4, SGPR base + a
// loop-invariant VGPR offset + the step's scalar offset) into 64 staging VGPRs, writes them to the LDS stage
// image with ds_write_b128 one step later (XOR swizzle chunk c of row r at c ^ (r & 7), as gemm256_k64.hip),
// and the fragments of the next 32-deep half are read beside the MFMAs of the current one.  The LDS-DMA form
// pays ~60-185 issue cycles per 1-KiB piece beside MFMAs (MI355X_MICROARCH.md, LDS-DMA piece issue cost):
// 16 pieces per wave per 2048 MFMA cycles at this tile.
//
// Per step j (one barrier):  read F1 = step j half 1  |  MFMA(F0)  |  wait vmcnt(0): R = step j+1
//   | ds_write R -> slot (j+1)&1  |  loads of step j+2 -> R  |  lgkmcnt(0) + barrier  |  read F0 = step j+1
//   half 0  |  MFMA(F1).
// C = A W^T in fp32: M, N multiples of 256, K of 64 (the launcher checks).
#include "../../multi-modal-tracking_amd/csrc/common.hpp"

namespace {
struct g256_args {
    const bf16_t* a;
    const bf16_t* w;
    float* c;
    int64_t sa, sw, sc;  // group strides (elements)
    int M, N, K, tiles_m, tiles_n, groups;
};

constexpr int BM = 256, BN = 256, STAGE = (BM + BN) * 128;

#ifndef G256_GM
#define G256_GM 8
#endif

__global__ __launch_bounds__(256) void gemm256_rs_kernel(g256_args p) {
    __shared__ __attribute__((aligned(1024))) unsigned char lds[2 * STAGE];
    const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
    const int per_g = p.tiles_m * p.tiles_n, g = lin / per_g, t = lin - g * per_g;
    const int grp = t / (G256_GM * p.tiles_n), first = grp * G256_GM, gsz = min(p.tiles_m - first, G256_GM);
    const int r = t - grp * G256_GM * p.tiles_n, tm = first + r % gsz, tn = r / gsz;
    const int m0 = tm * BM, n0 = tn * BN;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, wr = wid >> 1, wc = wid & 1;
    const int l16 = lane & 15, lg = lane >> 4;
    const int K = p.K, nk = K / 64;
    // buffer resources over this tile's A rows and W rows (byte offsets fit 32 bits: checked by the launcher)
    const __amdgpu_buffer_rsrc_t ars = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.a + g * p.sa + (int64_t)m0 * K), (short)0, BM * K * 2, 0x00020000);
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.w + g * p.sw + (int64_t)n0 * K), (short)0, BN * K * 2, 0x00020000);
    // thread -> (row t/8 + 32 i, chunk t%8) of the step, i = 0..7 for A and for W
    const int srow = threadIdx.x >> 3, sch = threadIdx.x & 7;
    const int voff = srow * K * 2 + sch * 16;  // + i * 32 * K * 2 (immediate-free: a VGPR per i below)
    const int woff = (srow * 8 + (sch ^ (srow & 7))) * 16;  // LDS byte offset of row srow's chunk (rows + 32 i keep r & 7)
    u32x4 ra[8], rb[8];
    auto gload = [&](int s) {
        const int ko = s * 128;  // bytes of K before step s
#pragma unroll
        for (int i = 0; i < 8; ++i)
            ra[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ars, voff + i * 32 * K * 2, ko, 0));
#pragma unroll
        for (int i = 0; i < 8; ++i)
            rb[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wrs, voff + i * 32 * K * 2, ko, 0));
    };
    auto swrite = [&](int s) {
        unsigned char* base = lds + (s & 1) * STAGE + woff;
#pragma unroll
        for (int i = 0; i < 8; ++i) *(u32x4*)(base + i * 32 * 128) = ra[i];
#pragma unroll
        for (int i = 0; i < 8; ++i) *(u32x4*)(base + BM * 128 + i * 32 * 128) = rb[i];
    };

    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    u32x4 fa[2][8], fb[2][8];
    auto read = [&](int s, int h, u32x4 (&af)[8], u32x4 (&bf)[8]) {
        const unsigned char* b_ = lds + (s & 1) * STAGE;
        const int sw_ = (4 * h + lg) ^ (lane & 7);
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) af[mt] = *(const u32x4*)(b_ + ((wr * 128 + mt * 16 + l16) * 8 + sw_) * 16);
#pragma unroll
        for (int nt = 0; nt < 8; ++nt) bf[nt] = *(const u32x4*)(b_ + BM * 128 + ((wc * 128 + nt * 16 + l16) * 8 + sw_) * 16);
    };
    auto mma = [&](const u32x4 (&af)[8], const u32x4 (&bf)[8]) {
#pragma unroll
        for (int nt = 0; nt < 8; ++nt)
#pragma unroll
            for (int mt = 0; mt < 8; ++mt)
                asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                             : "+a"(acc[nt][mt])
                             : "v"(bf[nt]), "v"(af[mt]));
    };

    gload(0);
    swrite(0);  // (hipcc waits for the loads)
    gload(1);   // nk >= 2: K % 128 == 0 is not required; the launcher checks nk >= 2
    lds_barrier();
    read(0, 0, fa[0], fb[0]);
    for (int j = 0; j + 1 < nk; ++j) {
        __builtin_amdgcn_s_waitcnt(0xc07f);  // F0 (read beside the last MFMA block) is in: hipcc, knowing it,
        __builtin_amdgcn_sched_barrier(0);   // then needs no lgkmcnt wait among the 16 new reads below
        read(j, 1, fa[1], fb[1]);
        __builtin_amdgcn_sched_barrier(0);
        mma(fa[0], fb[0]);
        __builtin_amdgcn_sched_barrier(0);
        swrite(j + 1);  // hipcc waits vmcnt for ra / rb
        gload(min(j + 2, nk - 1));  // past the end: re-loads the last step (discarded), constant vmcnt
        lds_barrier();
        read(j + 1, 0, fa[0], fb[0]);
        __builtin_amdgcn_sched_barrier(0);
        mma(fa[1], fb[1]);
        __builtin_amdgcn_sched_barrier(0);
    }
    read(nk - 1, 1, fa[1], fb[1]);
    __builtin_amdgcn_sched_barrier(0);
    mma(fa[0], fb[0]);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_sched_barrier(0);
    mma(fa[1], fb[1]);
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0);  // the discarded tail loads

    lds_barrier();
    constexpr int TP = BN + 4;
    float* img = (float*)lds;
    float* C = p.c + g * p.sc;
#pragma unroll
    for (int ps = 0; ps < 4; ++ps) {
        if (wr == (ps >> 1)) {
#pragma unroll
            for (int nt = 0; nt < 8; ++nt)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int mt = (ps & 1) * 4 + q;
                    *(f32x4*)(img + (q * 16 + l16) * TP + wc * 128 + nt * 16 + lg * 4) = acc[nt][mt];
                }
        }
        lds_barrier();
        const int c4 = (threadIdx.x & 63) * 4, r0 = threadIdx.x >> 6;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int rr = r0 + i * 4;
            *(f32x4*)(C + (int64_t)(m0 + ps * 64 + rr) * p.N + n0 + c4) = *(const f32x4*)(img + rr * TP + c4);
        }
        lds_barrier();
    }
}
}  // namespace

extern "C" int proto_gemm256(const void* a, const void* w, void* c, int groups, int M, int N, int K, void* stream) {
    if (M % 256 || N % 256 || K % 64 || K < 128 || groups < 1 || (int64_t)256 * K * 2 >= (1ll << 31)) return -22;
    g256_args p;
    p.a = (const bf16_t*)a;
    p.w = (const bf16_t*)w;
    p.c = (float*)c;
    p.sa = (int64_t)M * K;
    p.sw = (int64_t)N * K;
    p.sc = (int64_t)M * N;
    p.M = M, p.N = N, p.K = K, p.tiles_m = M / 256, p.tiles_n = N / 256, p.groups = groups;
    hipLaunchKernelGGL(gemm256_rs_kernel, dim3(p.tiles_m * p.tiles_n * groups), dim3(256), 0, (hipStream_t)stream, p);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
