#!/bin/bash
# Stamp builds of attention_pp.hip with one MMT_ATTN_ABLATE switch each (measurement only): copies the
# stamp build's objects and recompiles the attention objects.  Usage: tools/build_pp_ablate.sh 3 7 8 ...
set -e
cd "$(dirname "$0")/../multi-modal-tracking_amd/csrc"
L=../mmt_amd/_lib
for a in "$@"; do
  rm -rf $L/stamp_a$a; mkdir -p $L/stamp_a$a; cp -r $L/stamp/obj $L/stamp_a$a/obj
  rm -f $L/stamp_a$a/obj/attention_pp.o
  make -s OUT=$L/stamp_a$a OBJDIR=$L/stamp_a$a/obj ATTN_EXTRA="-DMMT_ATTN_ABLATE=$a" \
       CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 -DMMT_STAMP_BUILD=1" 2>&1 | grep -v warning || true
done
