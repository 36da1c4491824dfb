#!/bin/bash
# Measurement-only variants of libmmt_hip.so (never the product):
#   ablate1: LDS-DMA GEMM K loop without DMA after the prologue (MMT_GEMM_ABLATE=1)
#   ablate2: LDS-DMA GEMM K loop without MFMA work          (MMT_GEMM_ABLATE=2)
#   aab1/2/3: range-checked MAM attention without K/V DMA after the prologue / without matrix and
#            softmax work / without exponentials / without exponentials and bf16 packing
#            (MMT_ATTN_ABLATE=1/2/3/4); aab5: impl 22 free-running (no per-tile wait / barrier / refill); aab6: aab5 without exponentials
#   stamp:   per-phase workgroup timestamps in the GEMM / attention kernels (MMT_STAMP_BUILD=1)
#   stamp_e3 / stamp_e4: stamp builds of the GEMM without epilogue stores / tile reads (MMT_GEMM_ABLATE=3 / 4)
#   ab:      the product plus the A/B-only attention kernels impl 23-28 (MMT_ATTN_AB=1) and GEMM impl 9 (MMT_GEMM_AB=1)
#   noocc2:  the product without the cost model's switch to the two-per-CU 128x128 GEMM tile (impl 8)
#   occ2nores: the product with the inference residual producers (LayerNorm statistics out) kept off impl 8
#   skticket: the product with the ticket-first split-K hand-off (MMT_GEMM_SK_TICKET_FIRST=1)
#   gm4 / gm16: the large-grid GEMM tile order with 4 / 16 row tiles per row group (MMT_GEMM_GM; product 8)
# Use with MMT_HIP_LIB=multi-modal-tracking_amd/mmt_amd/_lib/<variant>/libmmt_hip.so.
set -e
ONLY=${1:-}
cd "$(dirname "$0")/../multi-modal-tracking_amd/csrc"
build() {
  if [ -n "$ONLY" ] && [ "$ONLY" != "$1" ]; then return; fi
  make -s OUT=../mmt_amd/_lib/$1 OBJDIR=../mmt_amd/_lib/$1/obj \
       CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 $2"
}
build ablate1 -DMMT_GEMM_ABLATE=1
build ablate2 -DMMT_GEMM_ABLATE=2
build stamp -DMMT_STAMP_BUILD=1
build stamp_e3 "-DMMT_STAMP_BUILD=1 -DMMT_GEMM_ABLATE=3"
build stamp_e4 "-DMMT_STAMP_BUILD=1 -DMMT_GEMM_ABLATE=4"
build aab1 -DMMT_ATTN_ABLATE=1
build aab2 -DMMT_ATTN_ABLATE=2
build aab3 -DMMT_ATTN_ABLATE=3
build aab4 -DMMT_ATTN_ABLATE=4
build aab5 -DMMT_ATTN_ABLATE=5
build aab6 -DMMT_ATTN_ABLATE=6
build ab "-DMMT_ATTN_AB=1 -DMMT_GEMM_AB=1"
# impl 28 (the A/B-only ping-pong MAM kernel) stamp / ablation builds: tools/build_pg_variant.sh
build noocc2 -DMMT_GEMM_NO_OCC2=1
build occ2nores -DMMT_GEMM_OCC2_RES=0
build skticket -DMMT_GEMM_SK_TICKET_FIRST=1
build gm4 -DMMT_GEMM_GM=4
build gm16 -DMMT_GEMM_GM=16
