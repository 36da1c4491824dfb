#!/bin/bash
# Builds measurement-only variants of libmmt_hip.so with the LDS-DMA GEMM's K loop ablated
# (MMT_GEMM_ABLATE=1: no DMA after the prologue; 2: no MFMA).  Results are wrong by design; use
# with MMT_HIP_LIB=... python tools/gemm_ab.py --no-check.
set -e
cd "$(dirname "$0")/../multi-modal-tracking_amd/csrc"
for a in 1 2; do
  make -s OUT=../mmt_amd/_lib/ablate$a OBJDIR=../mmt_amd/_lib/ablate$a/obj \
       CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 -DMMT_GEMM_ABLATE=$a"
done
