#!/bin/bash
# round 6: impl 29 (persistent MAM kernel) parity vs impl 22 and A/B timing
set -u
OUT=gpurun_out/r06b; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -v -k "persistent or pipelined_is_default" --timeout 120 --timeout-method thread > $OUT/ps_test.log 2>&1
rc=$?; echo "ps test rc=$rc"; tail -15 $OUT/ps_test.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/attn_ab.py --batches 1,8,16,32 --impls 22,29 > $OUT/attn_ab.jsonl 2> $OUT/attn_ab.err
rc=$?; echo "ab rc=$rc"; cat $OUT/attn_ab.jsonl; exit $rc
