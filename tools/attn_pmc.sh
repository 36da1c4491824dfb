#!/bin/bash
# Counter passes over the MAM attention kernel alone (tools/attn_pmc.py), one rocprofv3 run per set,
# summarised by tools/kernel_pmc.py.  Usage: tools/attn_pmc.sh TAG [attn_pmc.py args]
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
            "SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU" \
            "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $CTRS -d "$OUT/p$i" -o pmc --output-format csv -- \
      python3 "$ROOT/tools/attn_pmc.py" "$@" > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
python3 "$ROOT/tools/kernel_pmc.py" mam_attention "$OUT"/p* > "$OUT/summary.json"
cat "$OUT/summary.json"
