// Internal (non-ABI) entry points shared between the GEMM translation units.
#pragma once
#include "common.hpp"

// LDS-DMA large-tile 16-bit GEMM (gemm_glds.hip), T = bf16_t or f16_t.  force = mmt_gemm_params.impl: -1 never, 0 pick a
// tile shape, 1..4 force a tile shape (include/mmt_hip.h).  Returns 0 when launched, 1 when the shape or
// layout is not one it takes (the caller then runs gemm.hip's kernel).
template <typename T>
int mmt_gemm_glds(const mmt_gemm_params& p, hipStream_t st, int force);
