#!/bin/bash
# training forward attention with log-sum-exp on impl 21 (range-checked) instead of impl 8: parity, interleaved A/B
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/r05c3; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_ops.py tests/test_gpu_ops_registry.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_lib_trainonly.sh r05c3 attn8 3
