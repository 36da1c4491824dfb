#!/bin/bash
# config 3 (shared, 64 sequences on one GPU): impl 8 for the LayerNorm-statistics residual producers (product)
# vs kept off (occ2nores), interleaved
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05a3; mkdir -p $OUT; cd $ROOT
ARGS="--variant shared --total-seqs 64 --no-cpu-baseline --no-kv-cache --no-train-line --no-mam-batched --no-fp16-line --no-kernel-profile --steps 30 --warmup 5"
for rep in 1 2; do
  for v in product occ2nores; do
    if [ $v = product ]; then L=""; else L=multi-modal-tracking_amd/mmt_amd/_lib/occ2nores/libmmt_hip.so; fi
    MMT_HIP_LIB=$L timeout -k 10 300 python -u bench.py $ARGS > $OUT/c3_${v}_$rep.log 2>&1
    rc=$?; echo "$v $rep rc=$rc $(grep -o '"value": [0-9.]*' $OUT/c3_${v}_$rep.log | head -1)"; [ $rc -ne 0 ] && { tail -3 $OUT/c3_${v}_$rep.log; exit $rc; }
  done
done
