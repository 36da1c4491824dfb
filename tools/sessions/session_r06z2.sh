#!/bin/bash
# round 6, last tree, part 2: the default bench line, its frame rocprof trace / breakdown, the training step's one-step
# breakdown (session_r06fin2.sh), then the other BASELINE configurations (tools/session_configs.sh)
set -u
T=${1:-r06z}; ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
bash tools/sessions/session_r06fin2.sh "$T"
rc=$?; echo "part 2 rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd "$ROOT"; bash tools/session_configs.sh "${T}_configs"
