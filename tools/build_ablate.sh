#!/bin/bash
# Measurement-only variants of libmmt_hip.so (never the product):
#   ablate1: LDS-DMA GEMM K loop without DMA after the prologue (MMT_GEMM_ABLATE=1)
#   ablate2: LDS-DMA GEMM K loop without MFMA work          (MMT_GEMM_ABLATE=2)
#   stamp:   per-phase workgroup timestamps in the GEMM / attention kernels (MMT_STAMP_BUILD=1)
# Use with MMT_HIP_LIB=multi-modal-tracking_amd/mmt_amd/_lib/<variant>/libmmt_hip.so.
set -e
cd "$(dirname "$0")/../multi-modal-tracking_amd/csrc"
build() {
  make -s OUT=../mmt_amd/_lib/$1 OBJDIR=../mmt_amd/_lib/$1/obj \
       CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 $2"
}
build ablate1 -DMMT_GEMM_ABLATE=1
build ablate2 -DMMT_GEMM_ABLATE=2
build stamp -DMMT_STAMP_BUILD=1
