#!/bin/bash
# Fast measurement variants of libmmt_hip.so with the A/B-only ping-pong MAM kernel (impl 28, attention_pg.hip):
# the product's objects are reused, attention_pg.o is rebuilt with the given defines, and the library is
# relinked under _lib/<name>/.  usage: tools/build_pg_variant.sh <name> "<defines>"
set -e
NAME=$1; DEFS=$2
cd "$(dirname "$0")/../multi-modal-tracking_amd/csrc"
OUT=../mmt_amd/_lib/$NAME; mkdir -p $OUT/obj
for o in ../mmt_amd/_lib/obj/*.o; do case "$(basename $o)" in attention.o|attention_pg.o) ;; *) cp -p $o $OUT/obj/;; esac; done
# impl 28 lives in the A/B build: the dispatcher (attention.o) and attention_pg.o with MMT_ATTN_AB=1
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 -fno-slp-vectorize \
    -DMMT_ATTN_AB=1 -c attention.hip -o $OUT/obj/attention.o &
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 -fno-slp-vectorize \
    -mllvm -amdgpu-mfma-vgpr-form -DMMT_ATTN_AB=1 $DEFS -c attention_pg.hip -o $OUT/obj/attention_pg.o
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -mcode-object-version=5 $OUT/obj/*.o -o $OUT/libmmt_hip.so
