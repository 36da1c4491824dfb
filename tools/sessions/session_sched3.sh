#!/bin/bash
# Interleaved bench runs of several library builds (MMT_HIP_LIB), two rounds.
set -u
TAG=${1:-sched3}; VARIANTS=${2:-"default ss_max-ilp ss_gemm ss_other"}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$ROOT"
for i in 1 2; do
  for v in $VARIANTS; do
    if [ $v = default ]; then lib=; else lib=$ROOT/multi-modal-tracking_amd/mmt_amd/_lib/$v/libmmt_hip.so; fi
    MMT_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-mam-batched --no-kv-cache --no-kernel-profile --steps 400 > "$OUT/b.log" 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "bench $v rc=$rc"; exit $rc; }
    echo "run $i $v $(grep -o '"value": [0-9.]*' "$OUT/b.log" | head -1)" | tee -a "$OUT/runs.txt"
  done
done
exit 0
