#!/bin/bash
# Round 5 mid-tree check: the GPU test suite, then the default bench line (all fields)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/${1:-r05k}; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.load(open('$OUT/bench.json'))
print('value', d['value'], d['ms_per_step'], 'roof', d['roofline']['kernel'], d['roofline']['frac'])
print('mam_b32', d.get('roofline_mam_batched',{}).get('frac'), 'b8', d.get('roofline_mam_batched_b8',{}).get('frac'))
print('kv', d.get('tracking_kv_cache')); print('fp16', d.get('fp16_line')); print('tracker', d.get('tracker_step'))
print('train', (d.get('train_step') or {}).get('value')); print('cpu', (d.get('cpu_baseline') or {}).get('value'))"
exit $rc
