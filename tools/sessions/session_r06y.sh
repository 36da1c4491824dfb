#!/bin/bash
# round 6, closing tree: the whole GPU suite, smoke, the training counter passes again (train.py changed: the DDP
# exchange; the frame's sources are unchanged since r06z, digest 3272c718), the default bench line
set -u
T=${1:-r06y}; ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$T; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest_gpu.txt"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 "$OUT/smoke.txt"; [ $rc -ne 0 ] && exit $rc
cp profiles/pmc_traffic.json "$OUT/pmc_traffic_in.json"
TO=$ROOT/gpurun_out/${T}tpmc; mkdir -p "$TO"
cd /tmp && export TMPDIR=/tmp
i=0
for CTRS in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $CTRS -d "$TO/p$i" -o pmc --output-format csv -- \
      python3 "$ROOT/bench.py" --train --steps 3 --warmup 2 --no-cpu-baseline > "$TO/p$i.log" 2>&1
  rc=$?; echo "train pass $i ($CTRS) rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$TO/p$i.log"; exit $rc; }
done
cd "$ROOT"
python3 tools/pmc_train_traffic.py "$TO" 16 profiles/pmc_traffic.json | cut -c1-300
rc=$?; cp profiles/pmc_traffic.json "$OUT/pmc_traffic.json"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cut -c1-300 "$OUT/bench.json"; exit $rc
