#!/bin/bash
# MAM attention ablation timing (tools/build_ablate.sh aab1..3): which resource bounds the kernel.
set -u
TAG=${1:-aab}; IMPLS=${2:-16,19}; BATCHES=${3:-32}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"; cd "$ROOT"
for v in ${VARIANTS:-default aab1 aab2 aab3 aab4}; do
  if [ $v = default ]; then export MMT_HIP_LIB=; else export MMT_HIP_LIB=$ROOT/multi-modal-tracking_amd/mmt_amd/_lib/$v/libmmt_hip.so; fi
  timeout -k 10 200 python -u tools/attn_ab.py --impls "$IMPLS" --batches "$BATCHES" > "$OUT/ab_$v.jsonl" 2>&1
  rc=$?; echo "== $v rc=$rc"; grep -v amdgpu.ids "$OUT/ab_$v.jsonl"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
