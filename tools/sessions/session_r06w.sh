#!/bin/bash
# round 6: fused MSDA training op (parity tests + A/B), then the training bench, aten sites and profile
set -u
T=${1:-r06w}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_train_ops.py -m gpu \
  -k "msda_bimodal_train" > $OUT/msda_tests.log 2>&1
rc=$?; tail -3 $OUT/msda_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $OUT/msda_tests.log | head -20; exit $rc; }
timeout -k 10 120 python -u tools/msda_train_ab.py 2>&1 | grep -v amdgpu.ids
rc=$?; [ $rc -ne 0 ] && exit $rc
bash tools/sessions/session_r06t.sh ${T}_s
