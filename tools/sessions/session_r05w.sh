#!/bin/bash
# batch-1 ViT GEMM entries: tile / split-K choices after the ticket-first split-K hand-off
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05w; mkdir -p $OUT
timeout -k 10 400 python -u tools/plan_entry_ab.py --names qkv,proj,fc1,fc2 --cfgs 0:0,1:1,1:2,1:3,1:4,2:1,2:2,2:3,3:1,3:2 > $OUT/entry_ab.jsonl 2> $OUT/entry_ab.err
rc=$?; echo "rc=$rc"; cat $OUT/entry_ab.jsonl; tail -3 $OUT/entry_ab.err; exit $rc
