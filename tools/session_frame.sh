#!/bin/bash
# Frame-level check after a kernel change: the given pytest selection (-m gpu), then a rocprofv3
# kernel trace of the default bench mapped to plan entries.  Usage: tools/session_frame.sh TAG "pytest -k expression"
set -u
TAG=${1:-frame}; SEL=${2:-}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x ${SEL:+-k "$SEL"} --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o trace --output-format csv -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --no-kernel-profile --no-mam-batched --no-kv-cache --steps 100 --warmup 10 --dump-plan "$OUT/plan_names.json" > "$OUT/bench_prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; grep -o '"value": [0-9.]*' "$OUT/bench_prof.log" | head -1
python3 "$ROOT/tools/trace_breakdown.py" "$OUT/prof/trace_kernel_trace.csv" "$OUT/plan_names.json" > "$OUT/breakdown.txt" 2>&1
head -40 "$OUT/breakdown.txt"
exit $rc
