#!/bin/bash
# whole training step under one FETCH_SIZE / WRITE_SIZE counter pass each (bench.py --train, 3 steps): per-step HBM bytes
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/r05tpmc; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for CTRS in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $CTRS -d "$OUT/p$i" -o pmc --output-format csv -- \
      python3 "$ROOT/bench.py" --train --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i ($CTRS) rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/p$i.log"; exit $rc; }
done
