#!/bin/bash
# round 6: the DDP step's bucket all-reduces asynchronous (joined in finish()): the one-rank RCCL test, then the
# world-1 --force-ddp step beside the plain step, twice each, interleaved
set -u
T=${1:-r06ddp2}; ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$T; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_ddp.py > "$OUT/test.txt" 2>&1
rc=$?; echo "test rc=$rc"; tail -3 "$OUT/test.txt"; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --train --force-ddp > "$OUT/ddp_$i.json" 2> "$OUT/ddp_$i.err" || exit $?
  timeout -k 10 300 python -u bench.py --train > "$OUT/plain_$i.json" 2> "$OUT/plain_$i.err" || exit $?
  for f in ddp_$i plain_$i; do python3 -c "import json,sys; d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d.get('config',{}).get('parallelism'))"; done
done
