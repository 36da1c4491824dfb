// MAM attention, impl 29: the persistent one-wave-per-SIMD kernel.
//
// Reference: Attention.forward, lib/models/mixformer_vit_rgbt/mixformer.py:52-78 and the cross-modal
// form asymmetric_shared.py:55-104 (template queries -> own template keys; search queries -> all keys,
// or [template_V | template_I | own search]).  Layouts as attention.hip: qkv [seq][token][3][head][64]
// read in place, out [seq][token][head * 64].
//
// Math per 32-key block: impl 24's (= impl 22's): P = exp2(S) with no reference point, row sums on the
// matrix pipe, epilogue range check with the exact two-pass fallback.  Same MFMA order per accumulator and
// the same exponentials, so the output is bit-identical to impl 22.
//
// What is new is the structure around the block loop ("impl 29"):
//  * one 4-wave workgroup per CU (each wave owns the 512-register file: O in AGPRs), launched once per
//    CU and walking a static list of ITEMS.  An item is one (sequence, head) key stream shared by the
//    four waves through one LDS ring; per (sequence, head) there are na all-search items (4 x 64 search
//    queries, one task per wave) and one mixed item: three search waves (the remaining 64 / 64 / 16 search
//    queries) and the template wave, which takes all 128 template queries (four 32-query blocks) in one
//    pass over the stream's own-template tiles (tiles 0-1, or 2-3 for a cross-modal TIR sequence).
//  * the K / V tile stream is continuous across items: the sync point of stream tile T waits for this
//    wave's pieces of T, takes one barrier and issues tile T + PF, whatever item that tile belongs to;
//    an item's Q rides with its first tile into the wave's Q image in LDS.  No item pays a cold prologue.
//  * a task's output is normalised into a ring slot no wave reads until the next sync point refills it,
//    and leaves as whole 128-B rows (raw buffer stores; rows past the queries get an out-of-bounds offset,
//    so every store issues and the wave's vector-memory count stays exact for the counted waits).
// Ring: PF = 3 tiles issued ahead of the sync point, LAG = 4 slots kept behind it (the template wave reads
// its second tile until its task ends), R = 7 slots of 16 KiB + 5 Q images of 8 KiB.
// Counted waits: vmcnt counts loads and stores of a wave in issue order (GFX9 memory model), so the wait
// for tile T is vmcnt(ops this wave issued after T's last piece), tracked as a wave-uniform count.
// Shape (checked by the launcher): bf16, all queries (q_part 0), n_t = 128 (two tiles), the search tasks
// leave three for the mixed item (400 search tokens: 13 query blocks of 32), an even last 32-key block of
// the search stream, >= 8 tiles per stream.
#include "attn_common.hpp"

namespace {

// MMT_ATTN_ABLATE (measurement builds, tools/build_ps_variant.sh; results wrong): 3 = no exponentials,
// 5 = free-running (no per-tile wait / barrier), 20 = no O staging writes, 21 = every output store dropped
#ifndef MMT_ATTN_ABLATE
#define MMT_ATTN_ABLATE 0
#endif

constexpr int PS_PF = 3, PS_LAG = 4, PS_R = PS_PF + PS_LAG;
constexpr int PS_QIMG = 64 * 128;                   // one 64-query Q image
constexpr int PS_LDS = PS_R * FTILE + 5 * PS_QIMG;  // 112 KiB ring + 40 KiB Q images
constexpr uint32_t PS_OOB = 0x80000000u;            // buffer offset past any num_records: store dropped

typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));

MMT_DEV u32x4 ps_b128(const char* p) {
    u32x4 r;
    const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
    asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(a));
    return r;
}
MMT_DEV void ps_w64(char* p, uint32_t x, uint32_t y) {
    const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)p;
    const u32x2v v = {x, y};
    asm volatile("ds_write_b64 %0, %1" ::"v"(a), "v"(v) : "memory");
}

template <int N>
MMT_DEV void ps_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// vmcnt(n) for a wave-uniform n, rounded down to a multiple of 4 (every count the stream produces is one:
// 4 pieces per tile, 8 / 16 Q pieces, 4 / 8 / 16 row stores); rounding down only waits longer
MMT_DEV void ps_wait(int n) {
    if (n == 8) { ps_vm<8>(); return; }  // the steady state: two tiles issued after the awaited one
    switch (n >> 2) {
        case 0: ps_vm<0>(); break;
        case 1: ps_vm<4>(); break;
        case 2: ps_vm<8>(); break;
        case 3: ps_vm<12>(); break;
        case 4: ps_vm<16>(); break;
        case 5: ps_vm<20>(); break;
        case 6: ps_vm<24>(); break;
        case 7: ps_vm<28>(); break;
        case 8: ps_vm<32>(); break;
        case 9: ps_vm<36>(); break;
        default: ps_vm<40>(); break;
    }
}

#if MMT_STAMP_BUILD
// measurement build (tools/build_ps_variant.sh stamp): an event log per workgroup for wave 0 and wave 3
// (lane 0), kept in the 8 KiB of LDS past the kernel's own and copied out at the end: entry = s_memtime in
// bits 0-47, the event's argument in bits 48-55, its code (PS_EV_*) in bits 56-63; word 0 of each log =
// the number of events.  (A global store per event would enter the counted waits.)
#define PS_NEV 512
__device__ unsigned long long g_mmt_attn_ps_stamps[1024 * 2 * PS_NEV];
extern "C" int mmt_attn_ps_stamps(unsigned long long* host, int n) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_mmt_attn_ps_stamps), sizeof(unsigned long long) * n);
}
enum { PS_EV_SYNC = 1, PS_EV_WAITED = 2, PS_EV_BARRIER = 3, PS_EV_TASK_START = 4, PS_EV_LOOP_END = 5, PS_EV_STORED = 6,
       PS_EV_END = 7, PS_EV_STAGED = 8, PS_EV_READ = 9 };
#define PS_EV(CODE, ARG)                                                                                          \
    if ((threadIdx.x == 0 || threadIdx.x == 192) && ev_n < PS_NEV / 2 - 1) {                                      \
        unsigned long long t_;                                                                                    \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                                 \
        const unsigned long long e_ =                                                                             \
            (t_ & 0xffffffffffffull) | ((unsigned long long)((ARG) & 255) << 48) | ((unsigned long long)(CODE) << 56); \
        const uint32_t a_ = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)(                      \
            ev_log + (threadIdx.x ? PS_NEV / 2 : 0) + 1 + ev_n);                                                  \
        asm volatile("ds_write_b64 %0, %1" ::"v"(a_), "v"(e_) : "memory"); /* asm: no vmcnt(0) from hipcc */      \
        ++ev_n;                                                                                                   \
    }
#else
#define PS_EV(CODE, ARG)
#endif

template <int NQ>
struct PSState {
    f32x16 o[NQ][2];  // O^T accumulators [query block][32-dim half]
    f32x4 lacc[NQ];   // row sums (every element = this lane's query)
};

// (sequence, head, kind) of item ids id0, id0 + step, id0 + 2 step, ...: advanced without divisions
struct PSItem {
    int s, h, kind;
};

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void mam_attention_ps_kernel(
    const mmt_attn_params p) {
#if MMT_STAMP_BUILD
    __shared__ __attribute__((aligned(1024))) char lds[PS_LDS + 8192];
    unsigned long long* ev_log = (unsigned long long*)(lds + PS_LDS);
    int ev_n = 0;
#else
    __shared__ __attribute__((aligned(1024))) char lds[PS_LDS];
#endif
    const int n_t = p.n_t, ntok = p.ntok, C = p.C, H = p.H;
    const int64_t pitch = p.tok_pitch > 0 ? p.tok_pitch : ntok;
    const int64_t rs = 3 * (int64_t)C;
    const bf16_t* qkv = (const bf16_t*)p.qkv;
    const int Lk = p.asym ? ntok + n_t : ntok;  // the search key stream (every item streams it)
    const int nkt = (Lk + KB - 1) / KB;
    const int nst = ((ntok - n_t + 31) / 32 + 1) / 2;  // 64-query search tasks per (sequence, head)
    const int na = nst / 4, ipp = na + 1;              // items per (sequence, head): na all-search + mixed
    const int NI = p.S * H * ipp;
    // static walk: workgroup g runs on XCD g % 8; XCD x takes a contiguous run of the items (the items
    // of one (sequence, head) adjacent, so they read its K / V through one L2), its workgroups stride it
    const int G = gridDim.x, g = blockIdx.x, xcd = g & 7, gi = g >> 3, gper = G >> 3;
    const int q8 = NI >> 3, r8 = NI & 7;
    const int icnt = q8 + (xcd < r8 ? 1 : 0), ibase = xcd * q8 + min(xcd, r8);
    const int nitem = gi < icnt ? (icnt - gi + gper - 1) / gper : 0;
    const int Ttot = nitem * nkt;
    // item cursor steps: id + gper = (pair + dpr) * ipp + kind + dk, pair = s * H + h
    const int it0 = ibase + gi, pr0 = it0 / ipp, dpr = gper / ipp, dk = gper - dpr * ipp;
    const int ds = dpr / H, dh = dpr - ds * H;
    const PSItem item0 = PSItem{pr0 / H, pr0 % H, it0 - pr0 * ipp};
    auto advance = [&](PSItem& it) __attribute__((always_inline)) {
        it.kind += dk;
        const int c1 = it.kind >= ipp ? 1 : 0;
        it.kind -= c1 * ipp;
        it.h += dh + c1;
        const int c2 = it.h >= H ? 1 : 0;
        it.h -= c2 * H;
        it.s += ds + c2;
    };

    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int l32 = lane & 31, hf = lane >> 5;
    const int prow = lane >> 3, pcol = lane & 7;
    const __amdgpu_buffer_rsrc_t qrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)qkv, 0, (int)min((int64_t)0x7fffffff, (int64_t)p.S * pitch * rs * 2), 0x00020000);
    const int64_t opitch = p.out_pitch > 0 ? p.out_pitch : pitch;
    const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
        p.out, 0, (int)min((int64_t)0x7fffffff, (int64_t)p.S * opitch * C * 2), 0x00020000);
    typedef __attribute__((address_space(3))) void lds_void_t;
    char* const qimg_base = lds + PS_R * FTILE;

    // ---- the tile stream: issue cursor (item ik, tile itl, ring slot islot); vector-memory ops issued by
    // this wave (vm); in-flight tiles form a queue of at most PF = 3 marks (the count right after each
    // tile's last piece): ma (the oldest, next to sync), mb, mc
    int ik = 0, itl = 0, islot = 0, nq = 0, vm = 0;
    int ma = 0, mb = 0, mc = 0;
    PSItem iid = item0;
    auto issue = [&]() __attribute__((always_inline)) {
        const int s = iid.s, h = iid.h;
        if (itl == 0) {  // this wave's Q rows of item ik ride with its first tile (template wave: all 128)
            const bool tmpl = iid.kind == na && w == 3;
            const int q0 = tmpl ? 0 : n_t + 64 * (4 * iid.kind + w), qe = tmpl ? n_t : ntok;
            char* qdst = qimg_base + w * PS_QIMG;
            const int np = tmpl ? 16 : 8;
            for (int pk = 0; pk < np; ++pk) {
                const bf16_t* src = qkv + ((int64_t)s * pitch + min(q0 + pk * 8 + prow, qe - 1)) * rs + h * D;
                attn_glds16(src + ((pcol ^ prow) * 8), qdst + pk * 1024);
            }
            vm += np;
        }
        const int kk = itl * KB;  // the tile's first key; tiles never straddle a key segment (n_t % 64 == 0)
        int seq = s, row = kk;
        if (p.asym) {
            const int sV = s % p.Bm;
            if (kk < n_t) seq = sV;
            else if (kk < 2 * n_t) { seq = sV + p.Bm; row = kk - n_t; }
            else row = kk - n_t;
        }
        char* slot = lds + islot * FTILE;
        const int64_t colk = C + h * D + (pcol ^ prow) * 8, colv = 2 * C + h * D + (pcol ^ attn_vswz(prow)) * 8;
        if (kk + KB <= Lk) {
            const int soff = __builtin_amdgcn_readfirstlane((int)(((int64_t)seq * pitch + row) * rs * 2));
            const int vk = (int)((prow * rs + colk) * 2), vv = (int)((prow * rs + colv) * 2);
#pragma unroll
            for (int pp = 0; pp < 2; ++pp) {
                const int pk = 2 * w + pp;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(qrs, (lds_void_t*)(slot + pk * 1024), 16, vk,
                                                         soff + pk * 8 * (int)rs * 2, 0, 0);
                __builtin_amdgcn_raw_ptr_buffer_load_lds(qrs, (lds_void_t*)(slot + KB * 128 + pk * 1024), 16, vv,
                                                         soff + pk * 8 * (int)rs * 2, 0, 0);
            }
        } else {  // the stream's tail tile: rows past the last key re-read the last key
            const int last = Lk - 1 - kk;
#pragma unroll
            for (int pp = 0; pp < 2; ++pp) {
                const int pk = 2 * w + pp;
                const bf16_t* rp = qkv + ((int64_t)seq * pitch + row + min(pk * 8 + prow, last)) * rs;
                attn_glds16(rp + colk, slot + pk * 1024);
                attn_glds16(rp + colv, slot + KB * 128 + pk * 1024);
            }
        }
        vm += 4;
        ma = nq == 0 ? vm : ma;  // (selects, not a conditional store: that became a store through a
        mb = nq == 1 ? vm : mb;  // selected stack address, i.e. scratch plus a vmcnt(0) per sync)
        mc = nq == 2 ? vm : mc;
        ++nq;
        if (++islot == PS_R) islot = 0;
        if (++itl == nkt) {
            itl = 0;
            ++ik;
            advance(iid);
        }
    };
    int sT = 0;  // next stream tile to sync
    auto sync_one = [&]() __attribute__((always_inline)) {
        PS_EV(PS_EV_SYNC, sT);
        if (MMT_ATTN_ABLATE != 5) {
            ps_wait(__builtin_amdgcn_readfirstlane(vm - ma));  // this wave's pieces of tile sT landed
            PS_EV(PS_EV_WAITED, sT);
            lds_barrier();                                      // ... and every wave's; all past tile sT - LAG
            PS_EV(PS_EV_BARRIER, sT);
        }
        ma = mb;
        mb = mc;
        --nq;
        if (sT + PS_PF < Ttot) issue();
        ++sT;
    };
    auto sync_to = [&](int T) __attribute__((always_inline)) {
        while (sT <= T) sync_one();
    };

    // prologue: the first PF tiles of the stream
    for (int t = 0; t < PS_PF && t < Ttot; ++t) issue();

    const float cexp = p.scale * 1.4426950408889634f;
    const bool prescale = fabsf(cexp - 1.f) > 1e-6f;
    const float one_or_zero = (((lane & 15) >> 2) & 1) == ((lane >> 4) & 1) ? 1.f : 0.f;
    const uint32_t sel_w = pack_bf16x2(one_or_zero, one_or_zero);
    const int kpos = (l32 & 7) * 16;
    const int li = lane & 15, qr = li >> 2, pc = li & 3, dsub = (lane >> 4) & 1;

    // ---- pieces shared by both task kinds ---------------------------------------------------------------
    // Q fragments of query blocks [0, NQ) from a Q image (B operand of S^T = K Q^T), pre-scaled if needed
    auto load_q = [&](auto NQc, u32x4 (&qf)[decltype(NQc)::value][4], const char* qimg) __attribute__((always_inline)) {
        constexpr int NQ = decltype(NQc)::value;
#pragma unroll
        for (int qb = 0; qb < NQ; ++qb) {
            const int row = 32 * qb + l32;
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) qf[qb][ks] = ps_b128(qimg + row * 128 + (((2 * ks + hf) ^ (row & 7)) * 16));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (prescale) {
#pragma unroll
            for (int qb = 0; qb < NQ; ++qb)
#pragma unroll
                for (int ks = 0; ks < 4; ++ks) {
                    u32x4 v = qf[qb][ks];
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        v[e] = pack_bf16x2(__uint_as_float(v[e] << 16) * cexp, __uint_as_float(v[e] & 0xffff0000u) * cexp);
                    qf[qb][ks] = v;
                }
        }
    };
    // O^T += V^T P^T for query block qb and its row sums, on the accumulator registers (inline asm, "a"
    // constraint; a VALU write of an operand needs 2 wait states before the MFMA reads it: s_nop 1).  ZC: the
    // accumulators' first product (source C = 0: no zero fill of the accumulators)
    auto mfma_o = [&](f32x16& acc, const u32x4& vf, const u32x4& pb, auto ZCc) __attribute__((always_inline)) {
        if constexpr (decltype(ZCc)::value)
            asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(vf), "v"(pb));
        else
            asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(vf), "v"(pb));
    };
    auto mfma_l = [&](f32x4& acc, const u32x4& pb, auto ZCc) __attribute__((always_inline)) {
        const u32x4 su = u32x4{sel_w, sel_w, sel_w, sel_w};
        if constexpr (decltype(ZCc)::value)
            asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(su), "v"(pb));
        else
            asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(su), "v"(pb));
    };
    // P = exp2(S) of one query block (MASK: keys >= Lkt of block b give 0), packed to bf16 pairs
    auto softmax = [&](f32x16& sv, int b, int Lkt, auto MASKc, u32x4 (&dst)[2]) __attribute__((always_inline)) {
        constexpr bool MASK = decltype(MASKc)::value;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float e = MMT_ATTN_ABLATE == 3 ? sv[r] : __builtin_amdgcn_exp2f(sv[r]);
            sv[r] = (!MASK || 32 * b + 8 * (r >> 2) + 4 * hf + (r & 3) < Lkt) ? e : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
            dst[j] = u32x4{pack_bf16x2(sv[8 * j], sv[8 * j + 1]), pack_bf16x2(sv[8 * j + 2], sv[8 * j + 3]),
                           pack_bf16x2(sv[8 * j + 4], sv[8 * j + 5]), pack_bf16x2(sv[8 * j + 6], sv[8 * j + 7])};
    };
    auto kread_at = [&](const char* kimg, u32x4 (&kf)[4]) __attribute__((always_inline)) {
        const char* krow = kimg + l32 * 128;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) kf[ks] = ps_b128(krow + ((((2 * ks + hf) * 16) ^ kpos)));
    };
    auto vread_at = [&](const char* vimg, int b, uint2 (&vt)[2][2][2]) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int row = 32 * (b & 1) + 16 * j + 4 * hf + qr;
#pragma unroll
            for (int db = 0; db < 2; ++db) {
                const char* b1 = vimg + row * 128 + (((4 * db + 2 * dsub + (pc >> 1)) ^ attn_vswz(row)) * 16) + (pc & 1) * 8;
                vt[j][db][0] = attn_tr16<0>(b1);
                vt[j][db][1] = attn_tr16<8 * 128>(b1);
            }
        }
    };
    auto slot_ptr = [&](int T) __attribute__((always_inline)) {  // ring slot of stream tile T (T > -R)
        return lds + ((T + PS_R) % PS_R) * FTILE;
    };

    // epilogue of a task: per query block the range check; normalised O rows go through LDS (oimg: a ring
    // region no wave reads until a later sync point refills it) and out as whole 128-B rows; a block that
    // fails the check takes the exact fallback, stored here, and its staged rows are not stored
    auto epilogue = [&](auto NQc, auto QB0c, auto QB1c, PSState<decltype(NQc)::value>& st, char* oimg, const int s,
                        const int h, const int qbase, const int qend, const int Lkt) __attribute__((always_inline)) {
        constexpr int NQ = decltype(NQc)::value, QB0 = decltype(QB0c)::value, QB1 = decltype(QB1c)::value;
        constexpr int NS = QB1 - QB0;  // query blocks staged and stored by this call
        // the last MFMAs' results (16 passes) before any VALU reads them (the MFMAs are asm: no hazard tracking)
        if constexpr (QB0 == 0) {
            asm volatile("s_nop 15\n\ts_nop 15" : "+a"(st.o[0][0]), "+a"(st.o[0][1]), "+a"(st.lacc[0]));
#pragma unroll
            for (int qb = 1; qb < NQ; ++qb) asm volatile("" : "+a"(st.o[qb][0]), "+a"(st.o[qb][1]), "+a"(st.lacc[qb]));
        }
        int fail = 0;  // wave-uniform bit mask of query blocks that took the fallback
#pragma unroll
        for (int qb = QB0; qb < QB1; ++qb) {
            const float l = st.lacc[qb][0];
            // chk = 0 iff every O value is finite (x * 0 is 0 or NaN): summed as a tree of packed pairs, not
            // impl 22's serial chain (48 dependent adds per query block at the seam)
            f32x2 c2[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) c2[r] = f32x2{st.o[qb][0][r], st.o[qb][1][r]} * 0.f;
#pragma unroll
            for (int w2 = 8; w2 >= 1; w2 >>= 1)
#pragma unroll
                for (int r = 0; r < w2; ++r) c2[r] = c2[r] + c2[r + w2];
            const float chk = c2[0][0] + c2[0][1];
            const bool ok = (l >= LZ_LO && l <= LZ_HI && chk == 0.f) || MMT_ATTN_ABLATE != 0;
            const int q = qbase + 32 * qb + l32;
            if (__builtin_expect(__all(ok), 1)) {
                const float inv = 1.f / l;
                const int row = 32 * (qb - QB0) + l32;
                char* orow_p = oimg + row * 128 + hf * 8;
                if (MMT_ATTN_ABLATE == 20) continue;  // measurement build: no staging writes
#pragma unroll
                for (int db = 0; db < 2; ++db)
#pragma unroll
                    for (int gg = 0; gg < 4; ++gg)
                        ps_w64(orow_p + (((4 * db + gg) ^ (row & 7)) * 16),
                               pack_bf16x2(st.o[qb][db][4 * gg] * inv, st.o[qb][db][4 * gg + 1] * inv),
                               pack_bf16x2(st.o[qb][db][4 * gg + 2] * inv, st.o[qb][db][4 * gg + 3] * inv));
                continue;
            }
            fail |= 1 << (qb - QB0);
        }
        // query blocks that failed the check: the exact two-pass fallback from global memory, stored here (one
        // runtime loop: rare, and kept out of the unrolled code)
#pragma unroll 1
        for (int fb = 0; fb < NS; ++fb) {
            if (!((fail >> fb) & 1)) continue;
            const int q = qbase + 32 * (QB0 + fb) + l32;
            bf16_t* op = (bf16_t*)p.out + attn_out_row(p, s, q, pitch) * C + h * D;
            auto key_row = [&](int kk) -> const bf16_t* {  // key kk of this task's key range
                int seq = s, row = kk;
                if (p.asym && Lkt != n_t) {  // (template tasks: own template keys)
                    const int sV = s % p.Bm;
                    if (kk < n_t) seq = sV;
                    else if (kk < 2 * n_t) { seq = sV + p.Bm; row = kk - n_t; }
                    else row = kk - n_t;
                }
                return qkv + ((int64_t)seq * pitch + row) * rs;
            };
            float qv[32], acc[32];
            const int qc = min(q, qend - 1);
            {
                const bf16_t* qp = qkv + ((int64_t)s * pitch + qc) * rs + h * D + 32 * hf;
#pragma unroll
                for (int i = 0; i < 32; ++i) qv[i] = bf2f(qp[i]) * cexp;
            }
            auto score = [&](int kk) {
                const bf16_t* kp = key_row(kk) + C + h * D + 32 * hf;
                float d0 = 0.f;
#pragma unroll
                for (int i = 0; i < 32; ++i) d0 += qv[i] * bf2f(kp[i]);
                return d0 + __shfl_xor(d0, 32, 64);
            };
            float m = -INFINITY;
            for (int kk = 0; kk < Lkt; ++kk) m = fmaxf(m, score(kk));
            float lf = 0.f;
#pragma unroll
            for (int i = 0; i < 32; ++i) acc[i] = 0.f;
            for (int kk = 0; kk < Lkt; ++kk) {
                const float e = __builtin_amdgcn_exp2f(score(kk) - m);
                lf += e;
                const bf16_t* vp = key_row(kk) + 2 * C + h * D + 32 * hf;
#pragma unroll
                for (int i = 0; i < 32; ++i) acc[i] += e * bf2f(vp[i]);
            }
            if (q < qend) {
                const float inv = 1.f / lf;
#pragma unroll
                for (int i = 0; i < 32; i += 8)
                    *(u32x4*)(op + 32 * hf + i) = u32x4{pack_bf16x2(acc[i] * inv, acc[i + 1] * inv), pack_bf16x2(acc[i + 2] * inv, acc[i + 3] * inv),
                                                        pack_bf16x2(acc[i + 4] * inv, acc[i + 5] * inv), pack_bf16x2(acc[i + 6] * inv, acc[i + 7] * inv)};
            }
        }
        // whole rows back from LDS (piece pk = rows 8 pk .. 8 pk + 7, a lane per 16-B chunk) and out (LDS is in
        // order per wave, so the reads see the writes)
        PS_EV(PS_EV_STAGED, 0);
        u32x4 ov[4 * NS];
#pragma unroll
        for (int pk = 0; pk < 4 * NS; ++pk) ov[pk] = ps_b128(oimg + (8 * pk + prow) * 128 + ((pcol ^ prow) * 16));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        PS_EV(PS_EV_READ, 0);
        const int q0 = qbase + 32 * QB0;
        const int obase = __builtin_amdgcn_readfirstlane((int)((((int64_t)s * opitch + q0 - p.out_q0) * C + h * D) * 2));
#pragma unroll
        for (int pk = 0; pk < 4 * NS; ++pk) {
            const int row = 8 * pk + prow;
            const bool bad = q0 + row >= qend || ((fail >> (pk >> 2)) & 1);
            const int off = (bad || MMT_ATTN_ABLATE == 21) ? (int)PS_OOB : obase + row * C * 2 + pcol * 16;
            __builtin_amdgcn_raw_buffer_store_b128(ov[pk], ors, off, 0, 0);
        }
        vm += 4 * NS;
        PS_EV(PS_EV_STORED, 0);
    };

    // ---- search task: NQ (2 or 1) query blocks over the whole key stream of the item (tile slots from the
    // item's first stream tile Tb), software-pipelined over 32-key blocks (impl 24's iteration); its sync
    // points are the stream's: iteration i = 2 t - 1 opens tile t
    auto run_search = [&](auto NQc, const int s, const int h, const int qbase, const int Tb) __attribute__((always_inline)) {
        constexpr int NQ = decltype(NQc)::value;
        const int qend = ntok, Lkt = Lk;
        u32x4 qf[NQ][4];
        load_q(NQc, qf, qimg_base + w * PS_QIMG);
        PS_EV(PS_EV_TASK_START, qbase >> 5);
        const int nb = (Lkt + 31) / 32;
        const int nvl = Lkt - 32 * (nb - 1);  // keys of the last block
        PSState<NQ> st;
        auto kimg_of = [&](int b) { return slot_ptr(Tb + (b >> 1)) + (b & 1) * 32 * 128; };
        auto vimg_of = [&](int b) { return slot_ptr(Tb + (b >> 1)) + KB * 128; };
        u32x4 kf[4];
        uint2 vt[2][2][2];
        f32x16 sA[NQ], sB[NQ];
        u32x4 pA[NQ][2], pB[NQ][2];

        auto qk = [&](f32x16 (&dst)[NQ]) {
#pragma unroll
            for (int qb = 0; qb < NQ; ++qb) dst[qb] = f32x16{};
#pragma unroll
            for (int ks = 0; ks < 4; ++ks)
#pragma unroll
                for (int qb = 0; qb < NQ; ++qb)
                    dst[qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kf[ks]),
                                                                      __builtin_bit_cast(bf16x8, qf[qb][ks]), dst[qb], 0, 0, 0);
        };
        auto vfrag = [&](int j, int db) {
            const uint2 ua = vt[j][db][0], ub = vt[j][db][1];
            return u32x4{ua.x, ua.y, ub.x, ub.y};
        };
        auto pv = [&](int qb, const u32x4 (&pb)[2], auto ZCc) {
            constexpr bool ZC = decltype(ZCc)::value;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
#pragma unroll
                for (int db = 0; db < 2; ++db) {
                    if (ZC && j == 0) mfma_o(st.o[qb][db], vfrag(j, db), pb[j], attn_ic<1>{});
                    else mfma_o(st.o[qb][db], vfrag(j, db), pb[j], attn_ic<0>{});
                }
                if (ZC && j == 0) mfma_l(st.lacc[qb], pb[j], attn_ic<1>{});
                else mfma_l(st.lacc[qb], pb[j], attn_ic<0>{});
            }
        };
        auto wait_v = [&]() {
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vt[0][0][0]), "+v"(vt[0][0][1]), "+v"(vt[0][1][0]),
                         "+v"(vt[0][1][1]), "+v"(vt[1][0][0]), "+v"(vt[1][0][1]), "+v"(vt[1][1][0]), "+v"(vt[1][1][1]));
        };
        auto wait_k = [&]() { asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(kf[0]), "+v"(kf[1]), "+v"(kf[2]), "+v"(kf[3])); };
        auto tsync = [&](int i) {  // K(i + 1) opens tile (i + 1) / 2: exactly the stream's next sync point
            MMT_ATTN_ASSERT(sT == Tb + ((i + 1) >> 1));
            sync_one();
        };

        // generic iteration (first block, and NQ = 1): phase 1 = PV(i - 1) | softmax(i, query block 0) |
        // K(i + 1) reads; phase 2 = QK^T(i + 1) | softmax(i, query block 1) | V(i) reads
        auto iter = [&](int i, f32x16 (&sc)[NQ], f32x16 (&sn)[NQ], u32x4 (&pp)[NQ][2], u32x4 (&pcur)[NQ][2],
                        auto FIRSTc, auto SYNCc, auto ZCc) {
            constexpr bool FIRST = decltype(FIRSTc)::value;
            if constexpr (decltype(SYNCc)::value) tsync(i);
            if constexpr (!FIRST) wait_v();
            kread_at(kimg_of(i + 1), kf);
            if constexpr (!FIRST) {
#pragma unroll
                for (int qb = 0; qb < NQ; ++qb) pv(qb, pp[qb], ZCc);
            }
            softmax(sc[0], i, Lkt, attn_ic<0>{}, pcur[0]);
            __builtin_amdgcn_sched_barrier(0);
            wait_k();
            vread_at(vimg_of(i), i, vt);
            qk(sn);
            if constexpr (NQ == 2) softmax(sc[1], i, Lkt, attn_ic<0>{}, pcur[1]);
            __builtin_amdgcn_sched_barrier(0);
        };
        // the hand-placed steady-state iteration of impl 24 (two query blocks)
        auto mf_o = [&](int qb, int j, int db, const u32x4& pb, auto ZCc) {
            if (decltype(ZCc)::value && j == 0) mfma_o(st.o[qb][db], vfrag(j, db), pb, attn_ic<1>{});
            else mfma_o(st.o[qb][db], vfrag(j, db), pb, attn_ic<0>{});
        };
        auto mf_l = [&](int qb, int j, const u32x4& pb, auto ZCc) {
            if (decltype(ZCc)::value && j == 0) mfma_l(st.lacc[qb], pb, attn_ic<1>{});
            else mfma_l(st.lacc[qb], pb, attn_ic<0>{});
        };
        auto ex2 = [&](f32x16& sv, int r) {
            if (MMT_ATTN_ABLATE == 3) return;
            sv[r] = __builtin_amdgcn_exp2f(sv[r]);
            sv[r + 1] = __builtin_amdgcn_exp2f(sv[r + 1]);
        };
        auto cv = [&](const f32x16& sv, u32x4 (&dst)[2], int r) { dst[r >> 3][(r & 7) >> 1] = pack_bf16x2(sv[r], sv[r + 1]); };
        auto kr = [&](int b, int ks) { kf[ks] = ps_b128(kimg_of(b) + l32 * 128 + ((((2 * ks + hf) * 16) ^ kpos))); };
        auto vr = [&](int b, int j, int db) {
            const char* vimg = vimg_of(b);
            const int row = 32 * (b & 1) + 16 * j + 4 * hf + qr;
            const char* b1 = vimg + row * 128 + (((4 * db + 2 * dsub + (pc >> 1)) ^ attn_vswz(row)) * 16) + (pc & 1) * 8;
            vt[j][db][0] = attn_tr16<0>(b1);
            vt[j][db][1] = attn_tr16<8 * 128>(b1);
        };
        auto qk1 = [&](f32x16& dst, int qb, int ks) {
            dst = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kf[ks]), __builtin_bit_cast(bf16x8, qf[qb][ks]),
                                                          ks ? dst : f32x16{}, 0, 0, 0);
        };
        auto iter2 = [&](int i, f32x16 (&sc)[NQ], f32x16 (&sn)[NQ], u32x4 (&pp)[NQ][2], u32x4 (&pcur)[NQ][2],
                         auto SYNCc, auto ZCc) {
            if constexpr (NQ == 2) {
                constexpr auto Z = ZCc;
                if constexpr (decltype(SYNCc)::value) tsync(i);
                wait_v();
                __builtin_amdgcn_sched_barrier(0);
                // phase 1
                mf_o(0, 0, 0, pp[0][0], Z); kr(i + 1, 0); kr(i + 1, 1); ex2(sc[0], 0); __builtin_amdgcn_sched_barrier(0);
                mf_o(0, 0, 1, pp[0][0], Z); kr(i + 1, 2); kr(i + 1, 3); ex2(sc[0], 2); __builtin_amdgcn_sched_barrier(0);
                mf_l(0, 0, pp[0][0], Z); cv(sc[0], pcur[0], 0); __builtin_amdgcn_sched_barrier(0);
                mf_o(0, 1, 0, pp[0][1], Z); ex2(sc[0], 4); cv(sc[0], pcur[0], 2); __builtin_amdgcn_sched_barrier(0);
                mf_o(0, 1, 1, pp[0][1], Z); ex2(sc[0], 6); __builtin_amdgcn_sched_barrier(0);
                mf_l(0, 1, pp[0][1], Z); cv(sc[0], pcur[0], 4); __builtin_amdgcn_sched_barrier(0);
                mf_o(1, 0, 0, pp[1][0], Z); ex2(sc[0], 8); cv(sc[0], pcur[0], 6); __builtin_amdgcn_sched_barrier(0);
                mf_o(1, 0, 1, pp[1][0], Z); ex2(sc[0], 10); __builtin_amdgcn_sched_barrier(0);
                mf_l(1, 0, pp[1][0], Z); cv(sc[0], pcur[0], 8); __builtin_amdgcn_sched_barrier(0);
                mf_o(1, 1, 0, pp[1][1], Z); ex2(sc[0], 12); cv(sc[0], pcur[0], 10); __builtin_amdgcn_sched_barrier(0);
                mf_o(1, 1, 1, pp[1][1], Z); ex2(sc[0], 14); __builtin_amdgcn_sched_barrier(0);
                mf_l(1, 1, pp[1][1], Z); cv(sc[0], pcur[0], 12); __builtin_amdgcn_sched_barrier(0);
                cv(sc[0], pcur[0], 14);
                wait_k();
                __builtin_amdgcn_sched_barrier(0);
                // phase 2
                qk1(sn[0], 0, 0); vr(i, 0, 0); ex2(sc[1], 0); __builtin_amdgcn_sched_barrier(0);
                qk1(sn[1], 1, 0); vr(i, 0, 1); ex2(sc[1], 2); cv(sc[1], pcur[1], 0); __builtin_amdgcn_sched_barrier(0);
                qk1(sn[0], 0, 1); vr(i, 1, 0); ex2(sc[1], 4); cv(sc[1], pcur[1], 2); __builtin_amdgcn_sched_barrier(0);
                qk1(sn[1], 1, 1); vr(i, 1, 1); ex2(sc[1], 6); cv(sc[1], pcur[1], 4); __builtin_amdgcn_sched_barrier(0);
                qk1(sn[0], 0, 2); ex2(sc[1], 8); cv(sc[1], pcur[1], 6); __builtin_amdgcn_sched_barrier(0);
                qk1(sn[1], 1, 2); ex2(sc[1], 10); cv(sc[1], pcur[1], 8); __builtin_amdgcn_sched_barrier(0);
                qk1(sn[0], 0, 3); ex2(sc[1], 12); cv(sc[1], pcur[1], 10); __builtin_amdgcn_sched_barrier(0);
                qk1(sn[1], 1, 3); ex2(sc[1], 14); cv(sc[1], pcur[1], 12); __builtin_amdgcn_sched_barrier(0);
                cv(sc[1], pcur[1], 14);
                __builtin_amdgcn_sched_barrier(0);
            }
        };
        // the last block i = nb - 1 (even: launcher check): PV(i - 1) | softmax(i) (masked past Lkt) | V(i)
        // reads; then PV(i)
        auto last = [&](int i, f32x16 (&sc)[NQ], u32x4 (&pp)[NQ][2], u32x4 (&pcur)[NQ][2]) {
            wait_v();
#pragma unroll
            for (int qb = 0; qb < NQ; ++qb) pv(qb, pp[qb], attn_ic<0>{});
            vread_at(vimg_of(i), i, vt);
            if (nvl < 32) {
#pragma unroll
                for (int qb = 0; qb < NQ; ++qb) softmax(sc[qb], i, Lkt, attn_ic<1>{}, pcur[qb]);
            } else {
#pragma unroll
                for (int qb = 0; qb < NQ; ++qb) softmax(sc[qb], i, Lkt, attn_ic<0>{}, pcur[qb]);
            }
            wait_v();
#pragma unroll
            for (int qb = 0; qb < NQ; ++qb) pv(qb, pcur[qb], attn_ic<0>{});
        };

        // blocks: 0 (prologue QK^T + iteration 0), 1 (the accumulators' first PV), 2, then pairs (odd, even),
        // then the last (even) block; nb >= 15 and odd (launcher)
        kread_at(kimg_of(0), kf);
        wait_k();
        qk(sA);
        iter(0, sA, sB, pB, pA, attn_ic<1>{}, attn_ic<0>{}, attn_ic<0>{});
        if constexpr (NQ == 2) {
            iter2(1, sB, sA, pA, pB, attn_ic<1>{}, attn_ic<1>{});
            iter2(2, sA, sB, pB, pA, attn_ic<0>{}, attn_ic<0>{});
        } else {
            iter(1, sB, sA, pA, pB, attn_ic<0>{}, attn_ic<1>{}, attn_ic<1>{});
            iter(2, sA, sB, pB, pA, attn_ic<0>{}, attn_ic<0>{}, attn_ic<0>{});
        }
        int i = 3;
        for (; i + 1 < nb - 1; i += 2) {
            if constexpr (NQ == 2) {
                iter2(i, sB, sA, pA, pB, attn_ic<1>{}, attn_ic<0>{});
                iter2(i + 1, sA, sB, pB, pA, attn_ic<0>{}, attn_ic<0>{});
            } else {
                iter(i, sB, sA, pA, pB, attn_ic<0>{}, attn_ic<1>{}, attn_ic<0>{});
                iter(i + 1, sA, sB, pB, pA, attn_ic<0>{}, attn_ic<0>{}, attn_ic<0>{});
            }
        }
        // one more odd block (nb odd: the loop leaves i = nb - 2), then the last (even) block
        if constexpr (NQ == 2) iter2(i, sB, sA, pA, pB, attn_ic<1>{}, attn_ic<0>{});
        else iter(i, sB, sA, pA, pB, attn_ic<0>{}, attn_ic<1>{}, attn_ic<0>{});
        ++i;
        last(i, sA, pB, pA);  // i = nb - 1 even: S(i) in sA, P(i - 1) in pB
        PS_EV(PS_EV_LOOP_END, 0);
        // staging: stream tile sT - LAG (waves 0 / 1) or sT - LAG + 1 (waves 2 / 3), i.e. the slots the next
        // two sync points refill: every wave is done with them, their last DMAs have landed
        char* oimg = slot_ptr(sT - PS_LAG + (w >> 1)) + (w & 1) * PS_QIMG;
        epilogue(NQc, attn_ic<0>{}, NQc, st, oimg, s, h, qbase, qend, Lkt);
    };

    // ---- template task: the 128 template queries (four 32-query blocks) over the item's own-template tiles
    // tt, tt + 1 (stream tiles Tb + tt ...).  Not software-pipelined: the template wave has the slack (its
    // four blocks are ~8 two-query-block blocks of work against the search waves' 16.5).  It starts after
    // sync point tt + 1 (both tiles landed) and takes tt + 2 .. tt + 4 after its blocks 0 .. 2, where the
    // search waves take them if a block here costs at most two of theirs; LAG 4 keeps tile tt until sync
    // point tt + 4 (after its block 2) and tile tt + 1 until tt + 5 (after its block 3).
    auto run_tmpl = [&](const int s, const int h, const int Tb, const int tt) __attribute__((always_inline)) {
        constexpr int NQ = 4;
        u32x4 qf[NQ][4];
        load_q(attn_ic<4>{}, qf, qimg_base + 3 * PS_QIMG);  // images 3 and 4: rows 0 .. 127
        PS_EV(PS_EV_TASK_START, 0);
        PSState<NQ> st;
        u32x4 kf[4];
        uint2 vt[2][2][2];
        auto block = [&](int b, auto ZCc) {
            const char* tbase = slot_ptr(Tb + tt + (b >> 1));
            kread_at(tbase + (b & 1) * 32 * 128, kf);
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(kf[0]), "+v"(kf[1]), "+v"(kf[2]), "+v"(kf[3]));
            f32x16 sc[NQ];
#pragma unroll
            for (int qb = 0; qb < NQ; ++qb) sc[qb] = f32x16{};
#pragma unroll
            for (int ks = 0; ks < 4; ++ks)
#pragma unroll
                for (int qb = 0; qb < NQ; ++qb)
                    sc[qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kf[ks]),
                                                                     __builtin_bit_cast(bf16x8, qf[qb][ks]), sc[qb], 0, 0, 0);
            vread_at(tbase + KB * 128, b, vt);
            u32x4 pcur[NQ][2];
#pragma unroll
            for (int qb = 0; qb < NQ; ++qb) softmax(sc[qb], b, n_t, attn_ic<0>{}, pcur[qb]);
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vt[0][0][0]), "+v"(vt[0][0][1]), "+v"(vt[0][1][0]),
                         "+v"(vt[0][1][1]), "+v"(vt[1][0][0]), "+v"(vt[1][0][1]), "+v"(vt[1][1][0]), "+v"(vt[1][1][1]));
#pragma unroll
            for (int qb = 0; qb < NQ; ++qb) {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
#pragma unroll
                    for (int db = 0; db < 2; ++db) {
                        const uint2 ua = vt[j][db][0], ub = vt[j][db][1];
                        const u32x4 vf = u32x4{ua.x, ua.y, ub.x, ub.y};
                        if (decltype(ZCc)::value && j == 0) mfma_o(st.o[qb][db], vf, pcur[qb][j], attn_ic<1>{});
                        else mfma_o(st.o[qb][db], vf, pcur[qb][j], attn_ic<0>{});
                    }
                    if (decltype(ZCc)::value && j == 0) mfma_l(st.lacc[qb], pcur[qb][j], attn_ic<1>{});
                    else mfma_l(st.lacc[qb], pcur[qb][j], attn_ic<0>{});
                }
            }
        };
        block(0, attn_ic<1>{});
        sync_one();  // tt + 2
        block(1, attn_ic<0>{});
        sync_one();  // tt + 3
        block(2, attn_ic<0>{});
        sync_one();  // tt + 4: tile tt refilled, read by blocks 0 and 1 only
        block(3, attn_ic<0>{});
        PS_EV(PS_EV_LOOP_END, 0);
        // output in two halves, each in the two-block window between sync points: tt + 5 (tile tt + 1 done,
        // refilled) then query blocks 0-1 staged in tile tt + 2 (= sT - LAG: refilled at tt + 6, no wave reads
        // it any more), then tt + 6 and blocks 2-3 in tile tt + 3
        sync_one();
        epilogue(attn_ic<4>{}, attn_ic<0>{}, attn_ic<2>{}, st, slot_ptr(sT - PS_LAG), s, h, 0, n_t, n_t);
        sync_one();
        epilogue(attn_ic<4>{}, attn_ic<2>{}, attn_ic<4>{}, st, slot_ptr(sT - PS_LAG), s, h, 0, n_t, n_t);
    };

    // ---- the wave's walk over its items
    PSItem id = item0;
    for (int k = 0; k < nitem; ++k) {
        const int Tb = k * nkt;
        if (id.kind == na && w == 3) {
            const int tt = (p.asym && id.s >= p.Bm) ? 2 : 0;  // own template keys in the stream: [tmpl V | tmpl I | ...]
            sync_to(Tb + tt + 1);
            run_tmpl(id.s, id.h, Tb, tt);
        } else {
            sync_to(Tb);  // (the previous item's remaining sync points first)
            // every search task runs two query blocks (the mixed item's last one, 16 queries, pads the second:
            // it shares its item with full tasks, so the padding costs no time, and one copy of the pipelined
            // loop keeps the kernel's code small)
            run_search(attn_ic<2>{}, id.s, id.h, n_t + 64 * (4 * id.kind + w), Tb);
        }
        advance(id);
    }
    sync_to(Ttot - 1);  // the last item's remaining sync points (every wave takes every barrier)
    PS_EV(PS_EV_END, 0);
#if MMT_STAMP_BUILD
    if (threadIdx.x == 0 || threadIdx.x == 192) {
        const int wl = threadIdx.x ? 1 : 0;
        unsigned long long* dst = g_mmt_attn_ps_stamps + (blockIdx.x * 2 + wl) * PS_NEV;
        dst[0] = ev_n;
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        for (int i = 0; i < ev_n; ++i) dst[1 + i] = ev_log[wl * (PS_NEV / 2) + 1 + i];
    }
#endif
}

}  // namespace

// launched by attention.hip's dispatcher (impl 29); returns MMT_EBADARG for shapes it does not take
int mmt_attn_launch_ps(const mmt_attn_params& p, hipStream_t st) {
    const int ns = p.ntok - p.n_t, nsb = (ns + 31) / 32, nst = (nsb + 1) / 2;
    const int Lk = p.asym ? p.ntok + p.n_t : p.ntok, nkt = (Lk + KB - 1) / KB;
    const int64_t pitch = p.tok_pitch > 0 ? p.tok_pitch : p.ntok;
    // n_t = 128: the template task's two tiles; nst % 4 == 3: the mixed item's three search tasks (the
    // last with 16 queries at most 32); the search stream's last 32-key block even (Lk % 64 in (0, 32]);
    // nkt >= 8: the next item's Q images are refilled (sync point nkt - PF) after the template wave read its,
    // and the template task's last sync point (tt + 6) lies inside its item
    if (p.q_part != 0 || p.lse || p.n_t != 128 || nst % 4 != 3 || nkt < 8 || nkt > 64 || Lk % 64 == 0 || Lk % 64 > 32)
        return MMT_EBADARG;
    if ((int64_t)p.S * pitch * 3 * p.C * 2 > 0x7fffffffLL) return MMT_EBADARG;
    const int64_t opitch = p.out_pitch > 0 ? p.out_pitch : pitch;
    if ((int64_t)p.S * opitch * p.C * 2 > 0x7fffffffLL) return MMT_EBADARG;
    static int ncu = 0;
    if (ncu == 0) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
            ncu = n;
        else
            ncu = 256;
    }
    const int64_t items = (int64_t)p.S * p.H * (nst / 4 + 1);
    int G = (int)(((items < ncu ? items : ncu) + 7) / 8 * 8);  // a multiple of 8 (the XCD walk)
    if (G > 1024) G = 1024;
    hipLaunchKernelGGL(mam_attention_ps_kernel, dim3(G), dim3(256), 0, st, p);
    return 0;
}
