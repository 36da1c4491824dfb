#!/bin/bash
# SQ counter passes over the MAM attention kernel alone (tools/attn_pmc.py), one rocprofv3 run per set.
set -u
TAG=${1:-apmc}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS" \
            "SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $CTRS -d "$OUT/p$i" -o pmc --output-format csv -- \
      python3 "$ROOT/tools/attn_pmc.py" "$@" > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
