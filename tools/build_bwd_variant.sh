#!/bin/bash
# Measurement-only variants of libmmt_hip.so that differ in attention_bwd.hip (the MAM backward) alone: that file is
# compiled with the given flags and linked with the product's other objects (run `make` first).
# usage: tools/build_bwd_variant.sh NAME "FLAGS"; then MMT_HIP_LIB=multi-modal-tracking_amd/mmt_amd/_lib/NAME/libmmt_hip.so
set -e
NAME=$1; FLAGS=$2
cd "$(dirname "$0")/../multi-modal-tracking_amd/csrc"
OUT=../mmt_amd/_lib/$NAME; mkdir -p $OUT
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 $FLAGS -c attention_bwd.hip \
  -o $OUT/attention_bwd.o
OBJS=$(ls ../mmt_amd/_lib/obj/*.o | grep -v attention_bwd.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -mcode-object-version=5 $OBJS $OUT/attention_bwd.o -o $OUT/libmmt_hip.so
rm -f $OUT/attention_bwd.o
