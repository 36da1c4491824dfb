#!/bin/bash
# round 6: the DDP step over a one-rank RCCL group (test + world-1 --force-ddp bench), training GPU tests
set -u
OUT=gpurun_out/r06a; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ddp.py -x -v -s --timeout 200 --timeout-method thread > $OUT/ddp_test.log 2>&1
rc=$?; echo "ddp test rc=$rc"; tail -5 $OUT/ddp_test.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --train --force-ddp > $OUT/train_ddp.json 2> $OUT/train_ddp.err
rc=$?; echo "train ddp rc=$rc"; cut -c1-600 $OUT/train_ddp.json; [ $rc -ne 0 ] && { tail -20 $OUT/train_ddp.err; exit $rc; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_train_ops.py -x -q --timeout 200 --timeout-method thread > $OUT/train_tests.log 2>&1
rc=$?; echo "train tests rc=$rc"; tail -3 $OUT/train_tests.log; exit $rc
