#!/bin/bash
# GPU session: the -m gpu suite (optionally filtered by -k EXPR), then one bench.py line per
# argument group.  Stops at the first crash / fault / timeout.
# Usage: tools/bench_session.sh TAG 'PYTEST_K_EXPR|all|none' 'bench args 1' ['bench args 2' ...]
set -u
TAG=$1; K=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"; cd "$ROOT"
if [ "$K" != "none" ]; then
  KARG=(); [ "$K" != "all" ] && KARG=(-k "$K")
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread "${KARG[@]}" > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" "$OUT/pytest_gpu.log" | tail -12
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
i=0
for args in "$@"; do
  i=$((i+1))
  timeout -k 10 400 python -u bench.py $args > "$OUT/bench$i.log" 2>&1
  rc=$?; echo "bench$i ($args) rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"dtype": "[a-z0-9]*"' "$OUT/bench$i.log" | head -3 | tr '\n' ' '; echo
  if [ $rc -ne 0 ]; then tail -5 "$OUT/bench$i.log"; exit $rc; fi
done
