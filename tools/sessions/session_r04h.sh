#!/bin/bash
# Training head on HIP: conv tests, the module-level training gradients, whole-step capture, step timing.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r04h
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_ops.py -m gpu -q -rf --timeout 300 --timeout-method thread \
    -k "not graph_replay" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|^E |FAILED" "$OUT/pytest.log" | tail -12
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_ops.py -m gpu -q -rf --timeout 240 --timeout-method thread \
    -k "graph_replay" > "$OUT/pytest_graph.log" 2>&1
rc=$?; echo "pytest graph rc=$rc"; grep -E "passed|failed|^E |FAILED" "$OUT/pytest_graph.log" | tail -8
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --train --steps 10 --warmup 3 > "$OUT/train.log" 2>&1
rc=$?; echo "train rc=$rc"; tail -c 1200 "$OUT/train.log"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --train --train-eager --steps 10 --warmup 3 > "$OUT/train_eager.log" 2>&1
rc=$?; echo "train eager rc=$rc"; tail -c 600 "$OUT/train_eager.log"
exit $rc
