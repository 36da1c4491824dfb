#!/bin/bash
# attention backward with the next tile's loads in flight: training-op parity, training bench, op table
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05a5; mkdir -p $OUT; cd $ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_ops.py tests/test_gpu_ops_registry.py -m gpu -x -q --timeout 200 \
    --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --train --steps 20 --warmup 5 --no-cpu-baseline > $OUT/train_bench.log 2>&1
rc=$?; echo "train rc=$rc $(grep -o '"value": [0-9.]*' $OUT/train_bench.log | head -1)"; [ $rc -ne 0 ] && { tail -5 $OUT/train_bench.log; exit $rc; }
timeout -k 10 300 python -u tools/train_ops_profile.py --top 12 > $OUT/train_ops.txt 2>&1
echo "ops rc=$?"; grep -E "mam_bwd|fa_kernel" $OUT/train_ops.txt
