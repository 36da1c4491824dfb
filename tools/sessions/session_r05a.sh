#!/bin/bash
# Round 5: first GPU run of the ping-pong MAM kernel (impl 26): bitwise check vs impl 22 (small shapes
# first), the attention tests, then the A/B timing at B = 1 / 8 / 32.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/${1:-r05a}; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 120 python -u tools/pg_check.py --impl 28 --batches 1 > "$OUT/pg_check_small.jsonl" 2>&1
rc=$?; echo "pg_check small rc=$rc"; tail -3 "$OUT/pg_check_small.jsonl"; [ $rc -ge 124 ] && exit $rc
timeout -k 10 120 python -u tools/pg_check.py --impl 28 --batches 8,32 > "$OUT/pg_check.jsonl" 2>&1
rc2=$?; echo "pg_check rc=$rc2"; tail -2 "$OUT/pg_check.jsonl"; [ $rc2 -ge 124 ] && exit $rc2
timeout -k 10 300 python -u tools/attn_ab.py --impls 22,28 --batches 1,8,32 > "$OUT/attn_ab.jsonl" 2>&1
rc3=$?; echo "attn_ab rc=$rc3"; cat "$OUT/attn_ab.jsonl" | cut -c1-400; [ $rc3 -ge 124 ] && exit $rc3
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "mam_attention" tests/test_capi.py > "$OUT/pytest_attn.log" 2>&1
rc4=$?; echo "pytest rc=$rc4"; tail -5 "$OUT/pytest_attn.log"
exit $(( rc + rc2 + rc3 + rc4 ))
