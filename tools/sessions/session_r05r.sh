#!/bin/bash
# ticket-first split-K: GEMM split-K tests, model / cache parity, then the default bench line
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05r; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "splitk or ksplit or column_split or mn_major" > $OUT/pytest_splitk.log 2>&1
rc=$?; echo "splitk tests rc=$rc"; tail -3 $OUT/pytest_splitk.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_model.py tests/test_gpu_cache.py > $OUT/pytest_model.log 2>&1
rc=$?; echo "model tests rc=$rc"; tail -3 $OUT/pytest_model.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --no-train-line > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.load(open('$OUT/bench.json'))
print('value', d['value'], d['ms_per_step'], 'roof', d['roofline']['kernel'], d['roofline']['frac'])
k=d.get('kernels') or {}
print({n: k[n] for n in k if 'conv1' in n or 'linear2' in n})"
exit $rc
