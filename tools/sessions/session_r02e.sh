#!/bin/bash
# r02e: registry / attention tests, B=1 attention XCD-map A/B in the frame, K/V cache at B=1/8, stage errors
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/r02e; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -k "registry or mam_attention" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for impl in 0 6; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-mam-batched --attn-impl $impl > "$OUT/bench_attn$impl.log" 2>&1
  rc=$?; echo "bench attn-impl $impl rc=$rc"; grep -o '"value": [0-9.]*\|"mam_attention": {"us": [0-9.]*\|"tracking_kv_cache": {"value": [0-9.]*' "$OUT/bench_attn$impl.log" | tr '\n' ' '; echo
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python -u bench.py --batch 8 --no-cpu-baseline --no-mam-batched --no-kernel-profile > "$OUT/bench_b8.log" 2>&1
rc=$?; echo "bench b8 rc=$rc"; grep -o '"value": [0-9.]*\|"tracking_kv_cache": {"value": [0-9.]*' "$OUT/bench_b8.log" | tr '\n' ' '; echo
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/stage_error.py > "$OUT/stage_error.jsonl" 2>&1
rc=$?; echo "stage_error rc=$rc"; grep -v amdgpu "$OUT/stage_error.jsonl"
exit $rc
