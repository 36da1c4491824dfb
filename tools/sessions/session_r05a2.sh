#!/bin/bash
# round 5, session 2: GEMM auto rule (impl 8 over 7), fused LayerNorm backward + residual gradient
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05a2; mkdir -p $OUT; cd $ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_train_ops.py -m gpu -x -q --timeout 200 \
    --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --train --steps 20 --warmup 5 --no-cpu-baseline > $OUT/train_bench.log 2>&1
rc=$?; echo "train rc=$rc"; grep -o '"value": [0-9.]*' $OUT/train_bench.log | head -2; [ $rc -ne 0 ] && { tail -5 $OUT/train_bench.log; exit $rc; }
timeout -k 10 300 python -u tools/plan_entry_ab.py --variant shared --batch 64 --names proj,fc2 --cfgs 0:0,8:1,6:1,5:1,1:1 > $OUT/c3_entry_ab.jsonl 2> $OUT/c3_entry_ab.err
rc=$?; echo "rc=$rc"; [ $rc -ne 0 ] && { tail -3 $OUT/c3_entry_ab.err; exit $rc; }
timeout -k 10 300 python -u tools/plan_entry_ab.py --variant shared --batch 64 --names qkv,fc1 --cfgs 0:0,6:1,5:1,1:1 >> $OUT/c3_entry_ab.jsonl 2>> $OUT/c3_entry_ab.err
rc=$?; echo "rc=$rc"; cat $OUT/c3_entry_ab.jsonl; exit $rc
