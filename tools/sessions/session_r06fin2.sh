#!/bin/bash
# round 6 final, part 2: the default bench line (traffic from the committed counter passes), its rocprof kernel trace
# and frame breakdown, and the training step's one-step breakdown
set -u
T=${1:-r06fin}; ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$T; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cut -c1-300 "$OUT/bench.json"; [ $rc -ne 0 ] && { tail -5 "$OUT/bench.err"; exit $rc; }
SKIP_TESTS=1 bash tools/session_full.sh ${T}_frame --no-cpu-baseline
rc=$?; echo "frame session rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd "$ROOT"; bash tools/session_trainprof.sh ${T}_tp
