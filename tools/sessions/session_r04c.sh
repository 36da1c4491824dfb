#!/bin/bash
# impl 24 diagnosis: ablation builds (1 no refills, 3 no exponentials, 5 free-running) and SQ counters.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r04c
mkdir -p "$OUT"; cd "$ROOT"
for v in product aab1 aab3 aab5; do
  if [ $v = product ]; then LIBV=""; else LIBV=$ROOT/multi-modal-tracking_amd/mmt_amd/_lib/$v/libmmt_hip.so; fi
  MMT_HIP_LIB=$LIBV timeout -k 10 200 python -u tools/attn_ab.py --impls 22,24 --batches 4,32 > "$OUT/ab_$v.jsonl" 2>&1
  rc=$?; echo "ab $v rc=$rc"; grep -v amdgpu.ids "$OUT/ab_$v.jsonl" | grep '"asym": 0' | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
done
for impl in 24 22; do
  bash tools/attn_pmc.sh r04c/pmc_i$impl --batch 32 --impl $impl > "$OUT/pmc_i$impl.log" 2>&1
  rc=$?; echo "pmc $impl rc=$rc"; tail -30 "$OUT/pmc_i$impl.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
