// Prototype (tools only, not in the product library): a 256x256 bf16 GEMM tile at one workgroup of
// 4 waves per CU, each wave a 128x128 output tile (8 x 8 blocks of v_mfma_f32_16x16x32_bf16), the shape
// hipBLASLt picks for the training step's large-M GEMMs (kernel name MT256x256x64 / MIWT8_8 / WG32_8_1,
// profiles/r05_hipblaslt_kernels.jsonl).  Measures the K loop's speed before the product kernel takes it:
//   - 32-deep K-steps staged by global_load_lds_dwordx4 into a 4-slot ring of 32 KiB stage images
//     (A rows then W rows, 64-B rows; 16-B chunk c of row r stored at c ^ (2 * ((r >> 2) & 1)), which
//     makes the ds_read_b128 fragment reads conflict-free: the 16 lanes an LDS cycle serves hit 16
//     distinct (row mod 4, chunk) bank groups);
//   - the next step's fragments are read beside the current step's 64 MFMAs (one wave per SIMD never
//     waits on its own LDS reads);
//   - the DMA of step j+4 is issued at the top of step j into the slot step j's fragments just left:
//     three steps (~1.3 us) of cover for the L2 / HBM latency, 96 KiB in flight per CU (a 2-slot ring of
//     64-deep steps, one step in flight, ran at ~32 GB/s per CU: latency-bound, gemm256_k64.hip).
// C = A W^T in fp32 (no epilogue modes): M, N multiples of 256, K of 64 (the launcher checks).
#include "../../multi-modal-tracking_amd/csrc/common.hpp"

namespace {
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

MMT_DEV void glds16(const void* src, unsigned char* dst) {
    __builtin_amdgcn_global_load_lds((glb_void*)src, (lds_void*)dst, 16, 0, 0);
}
template <int N>
MMT_DEV void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

struct g256_args {
    const bf16_t* a;
    const bf16_t* w;
    float* c;
    int64_t sa, sw, sc;  // group strides (elements)
    int M, N, K, tiles_m, tiles_n, groups;
};

constexpr int BM = 256, BN = 256, STAGE = (BM + BN) * 64, ST = 4;

// measurement ablations (results wrong): 1 = no DMA after the prologue, 2 = no MFMAs, 3 = no fragment reads
#ifndef G256_ABL
#define G256_ABL 0
#endif
#ifndef G256_GM
#define G256_GM 8
#endif

__global__ __launch_bounds__(256) void gemm256_kernel(g256_args p) {
    __shared__ __attribute__((aligned(1024))) unsigned char lds[ST * STAGE];
    // XCD-aware linear id: consecutive ids on one XCD; then GM row tiles x all column tiles per group
    const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
    const int per_g = p.tiles_m * p.tiles_n, g = lin / per_g, t = lin - g * per_g;
    const int grp = t / (G256_GM * p.tiles_n), first = grp * G256_GM, gsz = min(p.tiles_m - first, G256_GM);
    const int r = t - grp * G256_GM * p.tiles_n, tm = first + r % gsz, tn = r / gsz;
    const int m0 = tm * BM, n0 = tn * BN;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, wr = wid >> 1, wc = wid & 1;
    const int l16 = lane & 15, lg = lane >> 4;
    const bf16_t* A = p.a + g * p.sa;
    const bf16_t* W = p.w + g * p.sw;
    const int K = p.K, nk = K / 32;

    // DMA: this wave's 4 A pieces and 4 W pieces (1 KiB = 16 rows x 64 B each) per stage; lane l writes
    // row l >> 2, physical chunk l & 3, i.e. logical chunk (l & 3) ^ swz(row)
    const int prow = lane >> 2, pch = (lane & 3) ^ (2 * ((prow >> 2) & 1));
    const bf16_t* asrc = A + (int64_t)(m0 + wid * 64 + prow) * K + pch * 8;
    const bf16_t* wsrc = W + (int64_t)(n0 + wid * 64 + prow) * K + pch * 8;
    auto issue = [&](int s) {
        if (G256_ABL == 1 && s >= 4) return;
        unsigned char* base = lds + (s & 3) * STAGE + wid * 4 * 1024;
        const int k = s * 32;
#pragma unroll
        for (int i = 0; i < 4; ++i) glds16(asrc + (int64_t)i * 16 * K + k, base + i * 1024);
#pragma unroll
        for (int i = 0; i < 4; ++i) glds16(wsrc + (int64_t)i * 16 * K + k, base + BM * 64 + i * 1024);
    };

    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    u32x4 fa[2][8], fb[2][8];
    const int rsw = (lg ^ (2 * ((l16 >> 2) & 1))) * 16;  // this lane's physical chunk (fragment rows are 16-aligned)
    auto read = [&](int s, u32x4 (&af)[8], u32x4 (&bf)[8]) {
        if (G256_ABL == 3 && s > 0) {
#pragma unroll
            for (int i = 0; i < 8; ++i) asm volatile("" : "+v"(af[i]), "+v"(bf[i]));
            return;
        }
        const unsigned char* b_ = lds + (s & 3) * STAGE + rsw;
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) af[mt] = *(const u32x4*)(b_ + (wr * 128 + mt * 16 + l16) * 64);
#pragma unroll
        for (int nt = 0; nt < 8; ++nt) bf[nt] = *(const u32x4*)(b_ + BM * 64 + (wc * 128 + nt * 16 + l16) * 64);
    };
    auto mma = [&](const u32x4 (&af)[8], const u32x4 (&bf)[8]) {
        if (G256_ABL == 2) {
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[0][0]) : "v"(bf[7]), "v"(af[7]));
            return;
        }
#pragma unroll
        for (int nt = 0; nt < 8; ++nt)
#pragma unroll
            for (int mt = 0; mt < 8; ++mt)
                // inline asm with the accumulator pinned to AGPRs ("+a": the 64 tiles fill all 256, so hipcc
                // cannot shuttle them through VGPRs as it does for the builtin here).  No s_nop pad: the
                // fragment registers are written only by ds_read (an s_nop costs 4 issue cycles per step of
                // its count beside a 16-cycle MFMA, which holds the SIMD's issue for 8)
                asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                             : "+a"(acc[nt][mt])
                             : "v"(bf[nt]), "v"(af[mt]));
    };
    // wait until step j's DMA (this wave's part) has landed, given the steps issued after it
    // (past the last step the ring re-issues the last step's DMA into the freed slot, so three newer
    // steps are always in flight and the count is constant)
    auto wait_step = [&](int) {
        if (G256_ABL == 1) wait_vm<0>();
        else wait_vm<24>();
    };

    for (int s = 0; s < 4; ++s) issue(min(s, nk - 1));
    wait_step(0);
    lds_barrier();
    read(0, fa[0], fb[0]);
    // two steps per iteration (statically named fragment sets); no MFMA under a branch
    int j = 0;
    for (; j + 2 < nk; j += 2) {
        wait_step(j + 1);
        lds_barrier();  // step j+1 landed for every wave; every wave is past its reads of slot j & 3
        issue(min(j + 4, nk - 1));
        read(j + 1, fa[1], fb[1]);
        __builtin_amdgcn_sched_barrier(0);
        mma(fa[0], fb[0]);
        __builtin_amdgcn_sched_barrier(0);
        wait_step(j + 2);
        lds_barrier();
        issue(min(j + 5, nk - 1));
        read(j + 2, fa[0], fb[0]);
        __builtin_amdgcn_sched_barrier(0);
        mma(fa[1], fb[1]);
        __builtin_amdgcn_sched_barrier(0);
    }
    {  // the last two steps (nk is even: K % 64 == 0; no MFMA under a branch)
        wait_step(j + 1);
        lds_barrier();
        read(j + 1, fa[1], fb[1]);
        __builtin_amdgcn_sched_barrier(0);
        mma(fa[0], fb[0]);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_sched_barrier(0);
        mma(fa[1], fb[1]);
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4" ::: "memory");  // last MFMA results -> accvgpr reads

    // epilogue: four passes of 64 tile rows through an fp32 LDS image, then 16-B row stores
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
        // 64 rows x 256 floats: thread -> 4 consecutive floats of a row, 4 rows per 256 threads
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
    if (M % 256 || N % 256 || K % 64 || K < 64 || groups < 1) return -22;
    g256_args p;
    p.a = (const bf16_t*)a;
    p.w = (const bf16_t*)w;
    p.c = (float*)c;
    p.sa = (int64_t)M * K;
    p.sw = (int64_t)N * K;
    p.sc = (int64_t)M * N;
    p.M = M, p.N = N, p.K = K, p.tiles_m = M / 256, p.tiles_n = N / 256, p.groups = groups;
    hipLaunchKernelGGL(gemm256_kernel, dim3(p.tiles_m * p.tiles_n * groups), dim3(256), 0, (hipStream_t)stream, p);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
