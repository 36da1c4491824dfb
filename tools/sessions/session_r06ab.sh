#!/bin/bash
# round 6: drop-in MSDA backward per-(n, m, level) value gather: tests, timing, rocprof of the timing run
set -u
OUT=gpurun_out/r06ab; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_backward_ops.py -m gpu > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 120 python -u tools/msda_bwd_value_ab.py 2>&1 | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o msda --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/msda_bwd_value_ab.py > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; grep -i "msda" $GRAFT_REPO_ROOT/$OUT/prof/msda_kernel_stats.csv | cut -c1-200
