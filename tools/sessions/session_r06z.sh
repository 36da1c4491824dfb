#!/bin/bash
# round 6: corner boxes + box loss on HIP: tests, then the training session
set -u
T=${1:-r06z}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train_ops.py -m gpu \
  -k "corner_boxes or box_loss" > $OUT/loss_tests.log 2>&1
rc=$?; tail -3 $OUT/loss_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|err" $OUT/loss_tests.log | head -30; exit $rc; }
bash tools/sessions/session_r06t.sh ${T}_s
