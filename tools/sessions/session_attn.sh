#!/bin/bash
# attention parity tests, latency-kernel A/B and in-frame bench per attention impl
set -u
TAG=${1:-attn}; IMPLS=${2:-3,4}; FRAME=${3:-0 3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -k "mam_attention or token_pitch or query_parts" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" "$OUT/pytest.log" | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/attn_ab.py --impls "$IMPLS" --batches 1,2 > "$OUT/attn_ab.jsonl" 2>&1
rc=$?; echo "attn_ab rc=$rc"; grep -v amdgpu "$OUT/attn_ab.jsonl" | cut -c1-300; [ $rc -ne 0 ] && exit $rc
for impl in $FRAME; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-mam-batched --no-kv-cache --attn-impl $impl > "$OUT/bench_$impl.log" 2>&1
  rc=$?; echo "bench attn-impl $impl rc=$rc"; grep -o '"value": [0-9.]*\|"mam_attention": {"us": [0-9.]*' "$OUT/bench_$impl.log" | tr '\n' ' '; echo
  [ $rc -ne 0 ] && exit $rc
done
exit 0
