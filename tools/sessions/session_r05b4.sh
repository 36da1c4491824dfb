#!/bin/bash
# split-K hand-off compiled only into splittable tiles (impl 8 epilogues without scratch spills): parity, then
# interleaved training / config-3 A/B against the spilling build
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/r05b4; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_train_ops.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_lib_train.sh r05b4 spill 2
