#!/bin/bash
# A/B of whole-library builds with another AMDGPU scheduler strategy (-mllvm -amdgpu-sched-strategy=...):
# MAM attention at B = 1 / 8 / 32 and the default bench, per build (MMT_HIP_LIB).
set -u
TAG=${1:-sched}; VARIANTS=${2:-"default ss_max-ilp ss_max-memory-clause"}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$ROOT"
for v in $VARIANTS; do
  if [ $v = default ]; then export MMT_HIP_LIB=; else export MMT_HIP_LIB=$ROOT/multi-modal-tracking_amd/mmt_amd/_lib/$v/libmmt_hip.so; fi
  timeout -k 10 200 python -u tools/attn_ab.py --impls 4,22 --batches 1,8,32 > "$OUT/attn_$v.jsonl" 2>&1
  rc=$?; echo "== $v attn rc=$rc"; grep -v amdgpu "$OUT/attn_$v.jsonl" | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['B'],d['asym'],{k:v['us'] for k,v in d.items() if k.startswith('impl')})"
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-mam-batched --no-kv-cache > "$OUT/bench_$v.log" 2>&1
  rc=$?; echo "== $v bench rc=$rc"; grep -o '"value": [0-9.]*' "$OUT/bench_$v.log" | head -1; [ $rc -ne 0 ] && exit $rc
done
exit 0
