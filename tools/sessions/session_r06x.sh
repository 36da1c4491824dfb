#!/bin/bash
# round 6: fused encoder layers (query prep, [offsets | logits] GEMM, MSDA op, dropout-residuals, FFN): tests, then
# the training session (tests, bench --train, sites, profile)
set -u
T=${1:-r06x}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_gpu_train_ops.py -m gpu \
  -k "msda_bimodal_train or encoder" > $OUT/enc_tests.log 2>&1
rc=$?; tail -3 $OUT/enc_tests.log; grep worst $OUT/enc_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $OUT/enc_tests.log | head -20; exit $rc; }
bash tools/sessions/session_r06t.sh ${T}_s
