#!/bin/bash
# Interleaved A/B of two library builds on the config-4 training step and the config-3 batched forward
# (separate processes, alternating, one box): tools/ab_lib_train.sh TAG VARIANT [REPS]
# VARIANT = multi-modal-tracking_amd/mmt_amd/_lib/<VARIANT>/libmmt_hip.so; "cur" = the in-tree library.
set -u
TAG=${1:-abt}; VAR=${2:-noocc2}; REPS=${3:-2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$ROOT"
for rep in $(seq 1 "$REPS"); do
for v in $VAR cur; do
  if [ $v = cur ]; then unset MMT_HIP_LIB; else export MMT_HIP_LIB=$ROOT/multi-modal-tracking_amd/mmt_amd/_lib/$v/libmmt_hip.so; fi
  timeout -k 10 200 python -u bench.py --train --steps 8 --warmup 3 > "$OUT/train_$v$rep.log" 2>&1
  rc=$?; echo "train $v $rep rc=$rc $(grep -o '"value": [0-9.]*' "$OUT/train_$v$rep.log" | head -1)"; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 200 python -u bench.py --variant shared --total-seqs 64 --no-cpu-baseline --no-kernel-profile --no-mam-batched \
      --no-kv-cache --no-fp16-line --no-train-line --steps 50 --warmup 10 > "$OUT/cfg3_$v$rep.log" 2>&1
  rc=$?; echo "cfg3 $v $rep rc=$rc $(grep -o '"value": [0-9.]*' "$OUT/cfg3_$v$rep.log" | head -1)"; [ $rc -ne 0 ] && exit $rc
done; done
exit 0
