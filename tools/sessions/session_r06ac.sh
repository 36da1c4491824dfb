#!/bin/bash
# round 6: search tokens as bf16 rows from the backbones to the fusion: tests, then the training session
set -u
T=${1:-r06ac}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train_ops.py -m gpu \
  -k "token_rows or groupnorm or encoder_layers" > $OUT/tok_tests.log 2>&1
rc=$?; tail -3 $OUT/tok_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|err" $OUT/tok_tests.log | head -30; exit $rc; }
bash tools/sessions/session_r06t.sh ${T}_s
