#!/bin/bash
# MN-major GEMMs on impl 8 from 192 tiles: gradient-GEMM parity, interleaved training A/B against the 256 threshold
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/r05b5; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_train_ops.py -m gpu -x -q --timeout 200 --timeout-method thread -k "mn_major or column_split or train or module or grad" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_lib_trainonly.sh r05b5 mn256 3
