#!/bin/bash
# round 6, last tree, part 1: the whole GPU suite, smoke, the frame and training counter passes (stamped, merged into
# profiles/pmc_traffic.json), then the backbone / head storage-type box-error probe (tools/box_err_mixed.py)
set -u
T=${1:-r06z}; ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$T; mkdir -p "$OUT"; cd "$ROOT"
bash tools/sessions/session_r06fin1.sh "$T"
rc=$?; echo "part 1 rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd "$ROOT"
timeout -k 10 300 python -u tools/box_err_mixed.py > "$OUT/box_err_mixed.jsonl" 2>&1
rc=$?; grep '^{' "$OUT/box_err_mixed.jsonl"; exit $rc
