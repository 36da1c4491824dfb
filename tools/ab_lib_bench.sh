#!/bin/bash
# Interleaved headline bench of two library builds in one GPU session (methodology rule 24):
#   tools/ab_lib_bench.sh TAG VARIANT [REPS] [bench args...]
# VARIANT = multi-modal-tracking_amd/mmt_amd/_lib/<VARIANT>/libmmt_hip.so (the "base" arm); "cur" = the
# in-tree library.  Each arm runs bench.py without the side measurements; one line per run.
set -u
TAG=${1:-ab}; VAR=${2:-base}; REPS=${3:-3}; shift 3 || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$ROOT"
for rep in $(seq 1 "$REPS"); do
for v in $VAR cur; do
  if [ $v = cur ]; then unset MMT_HIP_LIB; else export MMT_HIP_LIB=$ROOT/multi-modal-tracking_amd/mmt_amd/_lib/$v/libmmt_hip.so; fi
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-kernel-profile --no-mam-batched --no-kv-cache \
      --no-fp16-line --no-train-line --steps 400 --warmup 50 "$@" > "$OUT/$v$rep.log" 2>&1
  rc=$?; echo "$v $rep rc=$rc $(grep -o '"value": [0-9.]*' "$OUT/$v$rep.log" | head -1)"
  [ $rc -ne 0 ] && exit $rc
done; done
exit 0
