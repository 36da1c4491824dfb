#!/bin/bash
# round 6: impl 29 parity, A/B vs impl 22, stamps, free-running variant
set -u
OUT=gpurun_out/r06h; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -v -k "persistent or pipelined_is_default" --timeout 120 --timeout-method thread > $OUT/ps_test.log 2>&1
rc=$?; echo "ps test rc=$rc"; tail -3 $OUT/ps_test.log; [ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" $OUT/ps_test.log | head -60; exit $rc; }
timeout -k 10 300 python -u tools/attn_ab.py --batches 1,8,16,32 --impls 22,29 > $OUT/attn_ab.jsonl 2> $OUT/attn_ab.err
rc=$?; echo "ab rc=$rc"; cat $OUT/attn_ab.jsonl; [ $rc -ne 0 ] && exit $rc
MMT_HIP_LIB=multi-modal-tracking_amd/mmt_amd/_lib/stamp/libmmt_hip.so timeout -k 10 120 python -u tools/attn_ps_stamps.py --batches 1,32 > $OUT/stamps.jsonl 2> $OUT/stamps.err
rc=$?; echo "stamps rc=$rc"; cat $OUT/stamps.jsonl; [ $rc -ne 0 ] && { tail -5 $OUT/stamps.err; exit $rc; }
MMT_HIP_LIB=multi-modal-tracking_amd/mmt_amd/_lib/free/libmmt_hip.so timeout -k 10 120 python -u tools/attn_ab.py --batches 32 --impls 29 > $OUT/ab_free.jsonl 2> $OUT/ab_free.err
rc=$?; echo "free rc=$rc"; cat $OUT/ab_free.jsonl; exit $rc
