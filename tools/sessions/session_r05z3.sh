#!/bin/bash
# config 3 (shared, 64 sequences): the ViT GEMM entries of the real plan under forced tiles
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05z; mkdir -p $OUT; cd $ROOT
timeout -k 10 300 python -u tools/plan_entry_ab.py --variant shared --batch 64 --names proj,fc2 --cfgs 0:0,8:1,6:1,5:1,1:1 > $OUT/c3_entry_ab.jsonl 2> $OUT/c3_entry_ab.err
rc=$?; echo "rc=$rc"; [ $rc -ne 0 ] && { tail -3 $OUT/c3_entry_ab.err; exit $rc; }
timeout -k 10 300 python -u tools/plan_entry_ab.py --variant shared --batch 64 --names qkv,fc1 --cfgs 0:0,6:1,5:1,1:1 >> $OUT/c3_entry_ab.jsonl 2>> $OUT/c3_entry_ab.err
rc=$?; echo "rc=$rc"; cat $OUT/c3_entry_ab.jsonl; tail -2 $OUT/c3_entry_ab.err; exit $rc
