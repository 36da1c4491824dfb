#!/bin/bash
# round 6: gemm_glds.hip under other machine-scheduler strategies (build variants v_gmc = max-memory-clause,
# v_gmr = iterative-minreg; the product uses max-ilp): interleaved frame rates
set -u
T=${1:-r06sched}; ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$T; mkdir -p "$OUT"; cd "$ROOT"
for rep in 1 2; do
  for lib in product v_gmc v_gmr; do
    if [ $lib = product ]; then unset MMT_HIP_LIB; else export MMT_HIP_LIB=multi-modal-tracking_amd/mmt_amd/_lib/$lib/libmmt_hip.so; fi
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-train-line --no-mam-batched --no-kv-cache --no-fp16-line --no-tracker-line --steps 400 > "$OUT/bench_${lib}_$rep.json" 2>/dev/null || exit $?
    python3 -c "
import json; d=json.loads(open('$OUT/bench_${lib}_$rep.json').read().strip().splitlines()[-1]); k=d.get('kernels') or {}
print(json.dumps({'lib': '$lib', 'rep': $rep, 'frames_per_s': d['value'], 'fc2_us': d['roofline']['avg_launch_us'], 'kernels_us': {n: v['us'] for n, v in list(k.items())[:6]}}))"
  done
done
