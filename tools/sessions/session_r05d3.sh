#!/bin/bash
# dW GEMMs of nearly a round of tiles unsplit: parity, interleaved training A/B, then the frame and training-step
# counter passes of this tree
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/r05d3; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_train_ops.py -m gpu -x -q --timeout 200 --timeout-method thread -k "mn_major or column_split or train or module or grad" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_lib_trainonly.sh r05d3 dwsplit 3 || exit 1
cd "$ROOT" && bash tools/pmc_session.sh r05pmc3 > $OUT/pmc.log 2>&1; rc=$?; tail -3 $OUT/pmc.log; [ $rc -ne 0 ] && exit $rc
cd "$ROOT" && bash tools/sessions/session_r05tpmc.sh
exit 0
