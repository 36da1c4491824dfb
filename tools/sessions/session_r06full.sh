#!/bin/bash
# round 6: the full GPU test suite, smoke, and the default bench line (the driver's round-end tiers)
set -u
OUT=gpurun_out/${1:-r06full}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $OUT/pytest_gpu.txt; [ $rc -ne 0 ] && { grep -B5 -A40 "FAILED\|Error" $OUT/pytest_gpu.txt | head -80; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-400 $OUT/bench.json; exit $rc
