#!/bin/bash
# Measurement-only variant of libmmt_hip.so with ONE source file replaced: SRC (e.g. an older revision of
# csrc/norm.hip, `git show HEAD:multi-modal-tracking_amd/csrc/norm.hip > /tmp/norm.hip`) compiled with FLAGS in place
# of the product object of the same name, linked with the product's other objects (run `make` first).
# usage: tools/build_file_variant.sh NAME SRC.hip ["FLAGS"]; then MMT_HIP_LIB=multi-modal-tracking_amd/mmt_amd/_lib/NAME/libmmt_hip.so
set -e
NAME=$1; SRC=$(readlink -f "$2"); FLAGS=${3:-}
BASE=$(basename "$SRC" .hip)
cd "$(dirname "$0")/../multi-modal-tracking_amd/csrc"
OUT=../mmt_amd/_lib/$NAME; mkdir -p $OUT
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 -I. $FLAGS -c "$SRC" -o $OUT/$BASE.o
OBJS=$(ls ../mmt_amd/_lib/obj/*.o | grep -v "/$BASE.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -mcode-object-version=5 $OBJS $OUT/$BASE.o -o $OUT/libmmt_hip.so
rm -f $OUT/$BASE.o
