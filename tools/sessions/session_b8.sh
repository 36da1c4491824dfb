#!/bin/bash
# Batch-8 bench lines (one GPU) of the RGB-T variants, appended to gpurun_out/TAG/b8.jsonl.
set -u
TAG=${1:-b8}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$ROOT"
for v in rgbt shared asym asym_ce; do
  timeout -k 10 300 python -u bench.py --variant $v --batch 8 --no-cpu-baseline --no-kernel-profile --no-mam-batched \
      --no-fp16-line --no-train-line --steps 100 --warmup 10 > "$OUT/$v.log" 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -ne 0 ] && exit $rc
  grep -h '^{' "$OUT/$v.log" | tail -1 >> "$OUT/b8.jsonl"
done
python3 -c "
import json
for l in open('$OUT/b8.jsonl'):
    d = json.loads(l); print(d['config']['variant'], d['value'], (d.get('tracking_kv_cache') or {}).get('value'))
"
