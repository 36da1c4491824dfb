// Helpers shared by the MAM attention translation units (attention.hip, attention_pp.hip): tile
// geometry, the XCD-aware block map, LDS-DMA issue / counted waits, and the LDS fragment reads.
#pragma once
#include "common.hpp"

// MMT_ATTN_CHECK=1 builds turn the key-tile index checks into device asserts
#ifndef MMT_ATTN_CHECK
#define MMT_ATTN_CHECK 0
#endif
#if MMT_ATTN_CHECK
#include <cassert>
#define MMT_ATTN_ASSERT(c) assert(c)
#else
#define MMT_ATTN_ASSERT(c) ((void)0)
#endif

namespace {

constexpr int D = 64, KB = 64;                 // head dim, keys per K / V tile
constexpr int FQ = 128, FTILE = 2 * KB * 128;  // queries per throughput workgroup; bytes of a K + V tile slot
constexpr float LZ_LO = 0x1p-100f, LZ_HI = 0x1p100f;  // range of the row sums without a reference point

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int N>
struct attn_ic {
    static constexpr int value = N;
};

// XCD-aware bijective block remap at every grid size: each XCD gets a contiguous run of (query
// block, head, sequence) ids, query block fastest, so the query blocks of one (sequence, head)
// re-read its K / V rows from one L2.
MMT_DEV void attn_block_ids_xcd(int& bx, int& by, int& bz) {
    const int nbx = gridDim.x, nby = gridDim.y, nwg = nbx * nby * gridDim.z;
    const int orig = blockIdx.x + nbx * (blockIdx.y + nby * blockIdx.z);
    const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
    bx = lin % nbx;
    by = (lin / nbx) % nby;
    bz = lin / (nbx * nby);
}

template <int N>
MMT_DEV void attn_wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
typedef __attribute__((address_space(3))) void attn_lds_void;
typedef __attribute__((address_space(1))) void attn_glb_void;
MMT_DEV void attn_glds16(const void* src, char* dst) {
    __builtin_amdgcn_global_load_lds((attn_glb_void*)src, (attn_lds_void*)dst, 16, 0, 0);
}
// ds_read_b64_tr_b16 as inline asm: through the builtin, hipcc cannot tell the read from the
// in-flight LDS-DMA writes and drains vmcnt(0) before it (i.e. waits for the whole prefetch ring).
// Inline asm is invisible to its wait-count tracking, so the caller waits with attn_lds_wait().
template <int OFF>
MMT_DEV uint2 attn_tr16(const char* p) {
    uint2 r;
    const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "n"(OFF));
    return r;
}
MMT_DEV void attn_lds_wait() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);  // keep the MFMAs that consume the asm reads below the wait
}

MMT_DEV void attn_wait_dyn(int n) {
    switch (n) {
        case 0: attn_wait_vm<0>(); break;
        case 1: attn_wait_vm<1>(); break;
        case 2: attn_wait_vm<2>(); break;
        case 3: attn_wait_vm<3>(); break;
        case 4: attn_wait_vm<4>(); break;
        case 5: attn_wait_vm<5>(); break;
        case 6: attn_wait_vm<6>(); break;
        case 7: attn_wait_vm<7>(); break;
        case 8: attn_wait_vm<8>(); break;
        case 9: attn_wait_vm<9>(); break;
        case 10: attn_wait_vm<10>(); break;
        case 11: attn_wait_vm<11>(); break;
        case 12: attn_wait_vm<12>(); break;
        case 13: attn_wait_vm<13>(); break;
        case 14: attn_wait_vm<14>(); break;
        case 15: attn_wait_vm<15>(); break;
        case 16: attn_wait_vm<16>(); break;
        case 17: attn_wait_vm<17>(); break;
        default: attn_wait_vm<18>(); break;
    }
}

// first out row of query q of sequence s (mmt_attn_params.out_pitch / out_q0: compact activations of the
// template K/V cache passes; identity layout by default)
MMT_DEV int64_t attn_out_row(const mmt_attn_params& p, int s, int q, int64_t pitch) {
    return (int64_t)s * (p.out_pitch > 0 ? p.out_pitch : pitch) + q - p.out_q0;
}

// V image swizzle: chunk c of row r at c ^ (r & 6) ^ ((r & 2) << 1): the 4 rows x 4 chunks a
// half-wave reads per tr instruction then cover all 64 banks once.
MMT_DEV int attn_vswz(int row) { return (row & 6) ^ ((row & 2) << 1); }

}  // namespace
