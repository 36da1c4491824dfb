#!/bin/bash
# round 5 session: GEMM / training-op parity, training bench, config-3 interleaved A/B (impl 8 for the
# LayerNorm-statistics residual producers: product vs occ2nores)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05a4; mkdir -p $OUT; cd $ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_train_ops.py -m gpu -x -q --timeout 200 \
    --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --train --steps 20 --warmup 5 --no-cpu-baseline > $OUT/train_bench.log 2>&1
rc=$?; echo "train rc=$rc $(grep -o '"value": [0-9.]*' $OUT/train_bench.log | head -1)"; [ $rc -ne 0 ] && { tail -5 $OUT/train_bench.log; exit $rc; }
ARGS="--variant shared --total-seqs 64 --no-cpu-baseline --no-kv-cache --no-train-line --no-mam-batched --no-fp16-line --no-kernel-profile --steps 30 --warmup 5"
for rep in 1 2; do
  for v in product occ2nores; do
    if [ $v = product ]; then L=""; else L=multi-modal-tracking_amd/mmt_amd/_lib/occ2nores/libmmt_hip.so; fi
    MMT_HIP_LIB=$L timeout -k 10 300 python -u bench.py $ARGS > $OUT/c3_${v}_$rep.log 2>&1
    rc=$?; echo "$v $rep rc=$rc $(grep -o '"value": [0-9.]*' $OUT/c3_${v}_$rep.log | head -1)"; [ $rc -ne 0 ] && { tail -3 $OUT/c3_${v}_$rep.log; exit $rc; }
  done
done
timeout -k 10 300 python -u tools/train_ops_profile.py --top 30 > $OUT/train_ops.txt 2>&1
echo "ops rc=$?"
