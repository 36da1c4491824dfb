#!/bin/bash
# rocprofv3 kernel trace of config 3 (shared backbone, 64 sequences on one GPU), per plan entry
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/r05b1; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o trace --output-format csv -- \
    python3 "$ROOT/bench.py" --variant shared --total-seqs 64 --no-cpu-baseline --no-kernel-profile --no-mam-batched --no-kv-cache \
    --no-fp16-line --no-train-line --steps 20 --warmup 5 --dump-plan "$OUT/plan_names.json" > "$OUT/bench_prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
python3 "$ROOT/tools/trace_breakdown.py" "$OUT/prof/trace_kernel_trace.csv" "$OUT/plan_names.json" > "$OUT/breakdown.txt" 2>&1
head -40 "$OUT/breakdown.txt"
exit $rc
