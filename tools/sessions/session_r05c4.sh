#!/bin/bash
# batch-1 split-K entries under the store-first hand-off: forced tile:split choices in place
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/r05c4; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 500 python -u tools/plan_entry_ab.py --names head_conv1_adj12,head_conv2,enc_linear2,enc_linear1,enc_value_offw,enc_outproj,fc2,patch_gemm,fusion_adjust,fusion_adjust_cat \
    --cfgs 0:0,1:1,1:2,1:3,1:4,1:5,1:6,2:1,2:2,2:3,2:4,3:1,3:2,3:3,3:4 > $OUT/entry_ab.jsonl 2> $OUT/entry_ab.err
rc=$?; cat $OUT/entry_ab.jsonl | cut -c1-400; tail -2 $OUT/entry_ab.err; exit $rc
