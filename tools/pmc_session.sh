#!/bin/bash
# PMC passes (each counter set in its own rocprofv3 run, no tracing domains) over a short bench.
set -u
TAG=${1:-pmc}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for CTRS in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CTRS -d "$OUT/p$i" -o pmc --output-format csv -- \
      python3 "$ROOT/bench.py" --no-cpu-baseline --steps 10 --warmup 3 --no-kernel-profile --no-train-line --no-mam-batched --no-kv-cache --no-fp16-line ${PMC_BENCH_ARGS:-} --dump-plan "$OUT/plan_names.json" "$@" \
      > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($CTRS) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
python3 "$ROOT/tools/pmc_traffic.py" "$OUT" "$OUT/plan_names.json" "${PMC_KEY:-rgbt/B1/bf16}" "$OUT/pmc_traffic.json"
