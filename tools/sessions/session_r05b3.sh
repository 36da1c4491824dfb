#!/bin/bash
# impl 8 with the LayerNorm fold on handed-in statistics as the auto choice: GEMM / model parity, config 3 bench
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/r05b3; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/plan_entry_ab.py --variant shared --batch 64 --names qkv,fc1 --cfgs 0:0,8:1,6:1 > $OUT/c3_ln2_ab.jsonl 2> $OUT/c3_ln2_ab.err
rc=$?; cat $OUT/c3_ln2_ab.jsonl; [ $rc -ne 0 ] && { tail -3 $OUT/c3_ln2_ab.err; exit $rc; }
timeout -k 10 300 python -u bench.py --variant shared --total-seqs 64 --no-cpu-baseline --no-kv-cache --no-train-line --no-mam-batched --no-fp16-line --no-kernel-profile --steps 30 --warmup 5 > $OUT/c3.log 2>&1
rc=$?; echo "c3 rc=$rc $(grep -o '"value": [0-9.]*' $OUT/c3.log | head -1)"
