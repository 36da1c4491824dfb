#!/bin/bash
# Interleaved bench runs of the default build and a scheduler-strategy build, then a rocprof breakdown of each.
set -u
TAG=${1:-sched2}; V=${2:-ss_max-ilp}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$ROOT"
ALT=$ROOT/multi-modal-tracking_amd/mmt_amd/_lib/$V/libmmt_hip.so
for i in 1 2 3; do
  for lib in "" "$ALT"; do
    MMT_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-mam-batched --no-kv-cache --no-kernel-profile --steps 400 > "$OUT/b.log" 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "bench rc=$rc"; exit $rc; }
    echo "run $i ${lib:+$V}${lib:-default} $(grep -o '"value": [0-9.]*' "$OUT/b.log" | head -1)"
  done
done
cd /tmp && export TMPDIR=/tmp
for lib in "" "$ALT"; do
  n=${lib:+alt}; n=${n:-def}
  MMT_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$n" -o trace --output-format csv -- \
      python3 "$ROOT/bench.py" --no-cpu-baseline --no-kernel-profile --no-mam-batched --no-kv-cache --steps 100 --warmup 10 \
      --dump-plan "$OUT/plan_$n.json" > "$OUT/bench_prof_$n.log" 2>&1
  rc=$?; echo "rocprof $n rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 "$ROOT/tools/trace_breakdown.py" "$OUT/prof_$n/trace_kernel_trace.csv" "$OUT/plan_$n.json" > "$OUT/breakdown_$n.txt" 2>&1
  head -12 "$OUT/breakdown_$n.txt"
done
exit 0
