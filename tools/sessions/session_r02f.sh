#!/bin/bash
# r02f: GEMM / model parity after the LayerNorm statistics hand-off, stamps, bench + rocprof
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/r02f; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -k "gemm or model or smoke or tracker or cache or vitl" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" "$OUT/pytest.log" | tail -12; [ $rc -ne 0 ] && exit $rc
[ "${NOSTAMP:-0}" = 1 ] || MMT_HIP_LIB=multi-modal-tracking_amd/mmt_amd/_lib/stamp/libmmt_hip.so timeout -k 10 300 python -u tools/gemm_stamps.py > "$OUT/gemm_stamps.jsonl" 2>&1
rc=$?; echo "stamps rc=$rc"; grep -E '"impl": 1,' "$OUT/gemm_stamps.jsonl" | cut -c1-260; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --no-mam-batched > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; grep -o '"value": [0-9.]*' "$OUT/bench.log" | head -2; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o trace --output-format csv -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --no-kernel-profile --no-mam-batched --no-kv-cache --steps 100 --warmup 10 --dump-plan "$OUT/plan_names.json" > "$OUT/bench_prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
python3 "$ROOT/tools/trace_breakdown.py" "$OUT/prof/trace_kernel_trace.csv" "$OUT/plan_names.json" > "$OUT/breakdown.txt" 2>&1
head -12 "$OUT/breakdown.txt"
exit $rc
