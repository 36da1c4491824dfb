#!/bin/bash
# Full GPU session: -m gpu suite, smoke, attention A/B, default bench (with the batched MAM lines),
# rocprof kernel trace of the bench.  Stops at the first crash / fault / timeout.
# Usage: [SKIP_TESTS=1] tools/session_full.sh TAG [bench args...]  (attention impls 24-28 are A/B-build only)
set -u
TAG=${1:-full}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$ROOT"
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" "$OUT/pytest_gpu.log" | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 "$OUT/smoke.log"; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python -u tools/attn_ab.py --impls 4,21,22,0 --batches 1,8,32 > "$OUT/attn_ab.jsonl" 2>&1
rc=$?; echo "attn_ab rc=$rc"; grep -v amdgpu "$OUT/attn_ab.jsonl" | cut -c1-400; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py "$@" > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; grep -o '"value": [0-9.]*\|"roofline_mam[_a-z0-9]*": {"kernel": "mam_attention", "bound": "mfma", "achieved": [0-9.]*, "peak": [0-9.]*, "unit": "TFLOP/s", "frac": [0-9.]*' "$OUT/bench.log"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o trace --output-format csv -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --no-kernel-profile --no-mam-batched --no-kv-cache --no-fp16-line --no-train-line --steps 100 --warmup 10 --dump-plan "$OUT/plan_names.json" "$@" > "$OUT/bench_prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
python3 "$ROOT/tools/trace_breakdown.py" "$OUT/prof/trace_kernel_trace.csv" "$OUT/plan_names.json" > "$OUT/breakdown.txt" 2>&1
head -8 "$OUT/breakdown.txt"
exit $rc
