#!/bin/bash
# Round 5: compact template K/V cache passes -- cache / tracker / model / attention GPU tests, then bench lines
# with the kv-cache rate at B = 1 and B = 8.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/${1:-r05f}; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_model.py::test_rgb_only_module_api_and_template_cache tests/test_gpu_model.py tests/test_capi.py > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for B in 1 8; do
  timeout -k 10 300 python -u bench.py --batch $B --steps 200 --warmup 20 --no-cpu-baseline --no-mam-batched --no-fp16-line --no-train-line > "$OUT/bench_b$B.json" 2> "$OUT/bench_b$B.err"
  rc=$?; echo "bench B=$B rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/bench_b$B.err"; exit $rc; }
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_b$B.json')); print('B=$B full', d['value'], d['ms_per_step'], 'kv', d.get('tracking_kv_cache'))"
done
