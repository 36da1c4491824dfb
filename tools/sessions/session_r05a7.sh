#!/bin/bash
# dK / dV kernel at 32 keys per wave: backward parity, then interleaved training A/B against 16 keys per wave
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05a7; mkdir -p $OUT; cd $ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_ops.py tests/test_gpu_ops_registry.py -m gpu -x -q --timeout 200 \
    --timeout-method thread -k "attention or mam or graph_replay or module" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_lib_trainonly.sh r05a7 dkv16 3
