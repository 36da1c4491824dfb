#!/bin/bash
# rocprofv3 kernel trace + stats of the training step (bench.py --train), for the per-kernel breakdown.
set -u
TAG=${1:-trainprof}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o trace --output-format csv -- \
    python3 "$ROOT/bench.py" --train --steps 3 --warmup 2 > "$OUT/train_prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 "$OUT/train_prof.log" | cut -c1-400
python3 "$ROOT/tools/train_breakdown.py" "$OUT/prof/trace_kernel_trace.csv" > "$OUT/breakdown.txt" 2>&1
head -30 "$OUT/breakdown.txt" | cut -c1-160
exit $rc
