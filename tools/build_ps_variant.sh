#!/bin/bash
# Measurement-only variants of libmmt_hip.so that differ in attention_ps.hip (impl 29) alone: that file is
# compiled with the given flags and linked with the product's other objects (run `make` first).
#   stamp:  per-sync-point s_memtime stamps (MMT_STAMP_BUILD=1; tools/attn_ps_stamps.py)
#   free:   free-running waves: no per-tile wait / barrier (MMT_ATTN_ABLATE=5; results wrong)
#   noexp:  no exponentials (MMT_ATTN_ABLATE=3; results wrong)
# usage: tools/build_ps_variant.sh NAME "FLAGS"; then MMT_HIP_LIB=multi-modal-tracking_amd/mmt_amd/_lib/NAME/libmmt_hip.so
set -e
NAME=$1; FLAGS=$2
cd "$(dirname "$0")/../multi-modal-tracking_amd/csrc"
OUT=../mmt_amd/_lib/$NAME; mkdir -p $OUT
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 -fno-slp-vectorize \
  -mllvm -amdgpu-mfma-vgpr-form $FLAGS -c attention_ps.hip -o $OUT/attention_ps.o
OBJS=$(ls ../mmt_amd/_lib/obj/*.o | grep -v attention_ps.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -mcode-object-version=5 $OBJS $OUT/attention_ps.o -o $OUT/libmmt_hip.so
rm -f $OUT/attention_ps.o
