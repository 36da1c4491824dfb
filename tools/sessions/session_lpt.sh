#!/bin/bash
# MAM attention block-order A/B (impls 23 / 24, longest-first orders; measured in profiles/r02_attn_order_ab.jsonl and
# since removed from the library): parity of the given impls and their times vs impl 22
set -u
TAG=${1:-lpt}; IMPLS=${2:-22,23,24,0}; BATCHES=${3:-8,16,32}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -rf --timeout 120 --timeout-method thread -k "mam_attention and (23 or 24 or bitwise)" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" "$OUT/pytest.log" | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/attn_ab.py --impls "$IMPLS" --batches "$BATCHES" > "$OUT/attn_ab.jsonl" 2>&1
rc=$?; echo "attn_ab rc=$rc"; grep -v amdgpu "$OUT/attn_ab.jsonl" | cut -c1-400; exit $rc
