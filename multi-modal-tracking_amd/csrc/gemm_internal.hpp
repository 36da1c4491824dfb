// Internal (non-ABI) entry points shared between the GEMM translation units.
#pragma once
#include "common.hpp"

// LDS-DMA large-tile 16-bit GEMM (gemm_glds.hip), T = bf16_t or f16_t.  force = mmt_gemm_params.impl: -1 never, 0 pick a
// tile shape, 1..4 force a tile shape (include/mmt_hip.h).  Returns 0 when launched, 1 when the shape or
// layout is not one it takes (the caller then runs gemm.hip's kernel).
template <typename T>
int mmt_gemm_glds(const mmt_gemm_params& p, hipStream_t st, int force);

// n (1..4) independent problems of one LDS-DMA configuration in one launch (mmt_gemm_multi).
// Returns 0 when launched, 1 when some problem does not qualify (the caller launches them one by one).
template <typename T>
int mmt_gemm_glds_multi(const mmt_gemm_params* ps, int n, hipStream_t st);
