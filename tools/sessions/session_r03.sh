#!/bin/bash
# Round-3 GPU session: the given pytest selection, then optional tools, then the bench with the in-frame
# profile.  Stops at the first crash / fault / timeout.  Usage: tools/sessions/session_r03.sh TAG "pytest args" [tool cmds...]
set -u
TAG=$1; shift
PT=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$ROOT"
if [ -n "$PT" ]; then
  timeout -k 10 700 python -u -m pytest $PT -x -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" "$OUT/pytest.log" | tail -12
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
i=0
for cmd in "$@"; do
  i=$((i+1))
  timeout -k 10 400 bash -c "$cmd" > "$OUT/tool$i.log" 2>&1
  rc=$?; echo "tool$i rc=$rc: $cmd"; grep -v amdgpu.ids "$OUT/tool$i.log" | tail -c 2500
  if [ $rc -ne 0 ]; then exit $rc; fi
done
