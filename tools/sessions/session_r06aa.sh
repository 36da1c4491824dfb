#!/bin/bash
# round 6: dual-stream pair backward: graph-replay / gradient tests, then an interleaved A/B against one stream
set -u
OUT=gpurun_out/r06aa; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train_ops.py -m gpu \
  -k "graph_replay or train_step or module_forward or lockstep or fused_residual" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 800 python -u tools/train_ab.py --rounds 3 --steps 10 --warmup 3 --only hip,single_stream 2>&1 | grep -v amdgpu.ids | tee $OUT/ab.jsonl
