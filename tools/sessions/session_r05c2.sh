#!/bin/bash
# split-K hand-off: store-first (product) vs ticket-first (skticket): split-K parity, head entries in place,
# interleaved headline bench
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/r05c2; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_cache.py -m gpu -x -q --timeout 200 --timeout-method thread -k "splitk or split or conv or model or cache" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for v in cur skticket; do
  if [ $v = cur ]; then unset MMT_HIP_LIB; else export MMT_HIP_LIB=$ROOT/multi-modal-tracking_amd/mmt_amd/_lib/$v/libmmt_hip.so; fi
  timeout -k 10 200 python -u tools/plan_entry_ab.py --names head_conv1_adj12,head_conv2,enc_linear2 --cfgs 0:0 > $OUT/entry_$v.jsonl 2>&1
  echo "$v entries rc=$?"; grep '^{' $OUT/entry_$v.jsonl | cut -c1-200
done
unset MMT_HIP_LIB
A="--no-cpu-baseline --no-mam-batched --no-kv-cache --no-train-line --no-fp16-line --no-kernel-profile --steps 300 --warmup 30"
for rep in 1 2 3; do
  for v in skticket cur; do
    if [ $v = cur ]; then unset MMT_HIP_LIB; else export MMT_HIP_LIB=$ROOT/multi-modal-tracking_amd/mmt_amd/_lib/$v/libmmt_hip.so; fi
    timeout -k 10 200 python -u bench.py $A > $OUT/b_${v}_$rep.log 2>&1
    rc=$?; echo "bench $v $rep rc=$rc $(grep -o '"value": [0-9.]*' $OUT/b_${v}_$rep.log | head -1)"; [ $rc -ne 0 ] && exit $rc
  done
done
