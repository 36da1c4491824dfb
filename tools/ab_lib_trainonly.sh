#!/bin/bash
# Interleaved A/B of two library builds on the config-4 training step alone (separate processes, alternating,
# one box): tools/ab_lib_trainonly.sh TAG VARIANT [REPS]; VARIANT as tools/ab_lib_train.sh
set -u
TAG=${1:-abto}; VAR=${2:-bwdold}; REPS=${3:-3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$ROOT"
for rep in $(seq 1 "$REPS"); do
for v in $VAR cur; do
  if [ $v = cur ]; then unset MMT_HIP_LIB; else export MMT_HIP_LIB=$ROOT/multi-modal-tracking_amd/mmt_amd/_lib/$v/libmmt_hip.so; fi
  timeout -k 10 200 python -u bench.py --train --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/train_$v$rep.log" 2>&1
  rc=$?; echo "train $v $rep rc=$rc $(grep -o '"value": [0-9.]*' "$OUT/train_$v$rep.log" | head -1)"; [ $rc -ne 0 ] && exit $rc
done; done
exit 0
