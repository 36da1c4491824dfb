#!/bin/bash
# round 6: MSDA value gathers with the stable bucket placement and the pipelined long-bucket sums -- their tests, and
# the spread / collapsed timing of the product library against the previous msda.hip (tools/build_file_variant.sh)
set -u
T=${1:-r06msda}; ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$T; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -s tests/test_gpu_backward_ops.py \
    "tests/test_gpu_train_ops.py::test_msda_bimodal_train_matches_generic" > "$OUT/pytest.txt" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "collapsed|passed|failed" "$OUT/pytest.txt" | tail -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/msda_sort_ab.py > "$OUT/ab_new.jsonl" 2>&1 || exit $?
MMT_HIP_LIB=multi-modal-tracking_amd/mmt_amd/_lib/msda_old/libmmt_hip.so timeout -k 10 300 python -u tools/msda_sort_ab.py > "$OUT/ab_old.jsonl" 2>&1
rc=$?; cat "$OUT/ab_new.jsonl" "$OUT/ab_old.jsonl"; exit $rc
