#!/bin/bash
# round 6: head conv weight prep in one launch + channel-major im2col (dW in the parameter's layout): tests, then
# bench --train, aten call sites (with the backward nodes' forward sites), one-step rocprof breakdown
set -u
T=${1:-r06t}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train_ops.py -m gpu \
  -k "conv3x3 or head or corner or add_up or batchnorm or module_forward or graph_replay or train_step" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --train > $OUT/train.json 2> $OUT/train.err
rc=$?; echo "train rc=$rc"; cut -c1-300 $OUT/train.json; [ $rc -ne 0 ] && { tail -5 $OUT/train.err; exit $rc; }
timeout -k 10 300 python -u tools/train_aten_sites.py --top 60 > $OUT/sites.txt 2>&1
rc=$?; echo "sites rc=$rc"; grep -v Warn $OUT/sites.txt | head -40 | cut -c1-220; [ $rc -ne 0 ] && exit $rc
bash tools/session_trainprof.sh ${T}_tp
