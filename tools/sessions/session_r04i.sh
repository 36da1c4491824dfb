#!/bin/bash
# Batch-1 frame after the compact GEMM epilogues: GEMM phase stamps (library's choice), MAM impl-4 stamps, and
# the rocprofv3 per-entry breakdown of the frame.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/r04i; mkdir -p "$OUT"; cd "$ROOT"
SL=$ROOT/multi-modal-tracking_amd/mmt_amd/_lib/stamp/libmmt_hip.so
[ -s "$OUT/gemm_stamps.jsonl" ] || GEMM_STAMP_IMPLS=0 MMT_HIP_LIB=$SL timeout -k 10 200 python -u tools/gemm_stamps.py > "$OUT/gemm_stamps.jsonl" 2>&1
rc=$?; echo "gemm stamps rc=$rc"; [ $rc -ne 0 ] && exit $rc
MMT_HIP_LIB=$SL timeout -k 10 200 python -u tools/attn_stamps.py --batch 1 > "$OUT/attn_stamps.jsonl" 2>&1
rc=$?; echo "attn stamps rc=$rc"; grep -v amdgpu "$OUT/attn_stamps.jsonl" | cut -c1-400; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o trace --output-format csv -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --no-kernel-profile --no-mam-batched --no-kv-cache --no-fp16-line --no-train-line --steps 100 --warmup 10 --dump-plan "$OUT/plan_names.json" > "$OUT/bench_prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
python3 "$ROOT/tools/trace_breakdown.py" "$OUT/prof/trace_kernel_trace.csv" "$OUT/plan_names.json" > "$OUT/breakdown.txt" 2>&1
head -30 "$OUT/breakdown.txt"
exit $rc
