#!/bin/bash
# training-step kernels in isolation under counter collection: FETCH_SIZE and WRITE_SIZE in separate passes
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05q/pmc; mkdir -p $OUT
timeout -k 10 120 python3 -u $ROOT/tools/train_kernels_pmc.py --reps 3 > $OUT/plain.log 2>&1
rc=$?; echo "plain rc=$rc"; tail -2 $OUT/plain.log; [ $rc -ne 0 ] && exit $rc
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $C -d $OUT/$C -o pmc --output-format csv -- python3 $ROOT/tools/train_kernels_pmc.py --reps 3 > $OUT/$C.log 2>&1
  rc=$?; echo "$C rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/$C.log; exit $rc; }
done
python3 $ROOT/tools/train_kernels_pmc.py --reps 3 --summarize $OUT $OUT/train_kernels_traffic.json
