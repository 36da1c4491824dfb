#!/bin/bash
# Development GPU session: the whole -m gpu suite, then MAM attention A/B timings.
# Usage: tools/dev_session.sh TAG [IMPLS] [BATCHES]
set -u
TAG=${1:-dev}; IMPLS=${2:-8,17}; BATCHES=${3:-1,8,32}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" "$OUT/pytest_gpu.log" | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/attn_ab.py --impls "$IMPLS" --batches "$BATCHES" > "$OUT/ab.jsonl" 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids "$OUT/ab.jsonl"
exit $rc
