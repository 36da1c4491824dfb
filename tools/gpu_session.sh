#!/bin/bash
# One GPU session on the MI355X box: parity tests, smoke, bench, rocprofv3 kernel trace.
# Stops at the first crash / fault / timeout (any status other than 0 or pytest's 1 = "tests failed").
# Usage: tools/gpu_session.sh [tag] [bench args...]
set -u
TAG=${1:-r01}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"

timeout -k 10 900 python -m pytest tests -m gpu -q -rf --timeout 400 > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest rc=$rc" | tee -a "$OUT/pytest_gpu.log"
tail -3 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?
echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi

timeout -k 10 400 python bench.py "$@" > "$OUT/bench.log" 2>&1
rc=$?
echo "bench rc=$rc"; tail -c 3000 "$OUT/bench.log"
if [ $rc -ne 0 ]; then exit $rc; fi

export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o trace --output-format csv -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --no-kernel-profile --steps 100 --warmup 10 --dump-plan "$OUT/plan_names.json" "$@" \
    > "$OUT/bench_prof.log" 2>&1
rc=$?
echo "rocprof rc=$rc"
python3 "$ROOT/tools/trace_breakdown.py" "$OUT/prof/trace_kernel_trace.csv" "$OUT/plan_names.json" > "$OUT/breakdown.txt" 2>&1
head -40 "$OUT/breakdown.txt"
find "$OUT/prof" -name "*stats*" | head
exit $rc
