#!/bin/bash
# head chain error with conv5 in fp32; frame PMC traffic (FETCH_SIZE / WRITE_SIZE passes) after the ticket-first
# split-K hand-off
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05s; mkdir -p $OUT
timeout -k 10 200 python -u tools/head_stage_error.py > $OUT/head_stage.jsonl 2> $OUT/head_stage.err
rc=$?; echo "head rc=$rc"; grep chain $OUT/head_stage.jsonl; [ $rc -ne 0 ] && { tail -5 $OUT/head_stage.err; exit $rc; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_train_ops.py -k "head_forward" > $OUT/pytest_head.log 2>&1
rc=$?; echo "head tests rc=$rc"; tail -3 $OUT/pytest_head.log; [ $rc -ne 0 ] && exit $rc
bash $ROOT/tools/pmc_session.sh r05s_pmc
