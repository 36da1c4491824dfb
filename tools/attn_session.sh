#!/bin/bash
# GPU session for the MAM attention kernels: parity tests, then A/B timing.
# Usage: tools/attn_session.sh TAG IMPLS BATCHES
set -u
TAG=${1:-attn}; IMPLS=${2:-8,16,17}; BATCHES=${3:-1,8,32}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -x -k "mam_attention" --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/attn_ab.py --impls "$IMPLS" --batches "$BATCHES" > "$OUT/ab.jsonl" 2>&1
rc=$?; echo "ab rc=$rc"; cat "$OUT/ab.jsonl" | grep -v amdgpu.ids
exit $rc
