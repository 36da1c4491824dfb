#!/bin/bash
# RGB-only fp16 (config 1's model) and the two-stream headline: round-4 tree (_ab_r04, its own library) vs this tree,
# interleaved on one box
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/r05c1; mkdir -p "$OUT"
A="--no-cpu-baseline --no-mam-batched --no-kv-cache --no-train-line --no-fp16-line --no-kernel-profile --steps 200 --warmup 20"
for rep in 1 2; do
  for t in r04 cur; do
    if [ $t = r04 ]; then D=$ROOT/_ab_r04; else D=$ROOT; fi
    cd $D
    timeout -k 10 200 python -u bench.py --variant rgb --dtype fp16 $A > $OUT/rgb_${t}_$rep.log 2>&1
    rc=$?; echo "rgb $t $rep rc=$rc $(grep -o '"value": [0-9.]*' $OUT/rgb_${t}_$rep.log | head -1)"; [ $rc -ne 0 ] && { tail -3 $OUT/rgb_${t}_$rep.log; exit $rc; }
    timeout -k 10 200 python -u bench.py $A > $OUT/rgbt_${t}_$rep.log 2>&1
    rc=$?; echo "rgbt $t $rep rc=$rc $(grep -o '"value": [0-9.]*' $OUT/rgbt_${t}_$rep.log | head -1)"; [ $rc -ne 0 ] && { tail -3 $OUT/rgbt_${t}_$rep.log; exit $rc; }
  done
done
