#!/bin/bash
# Counter passes: the frame (tools/pmc_session.sh) and the MAM kernel alone at batch 32 / 1 (tools/attn_pmc.sh)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
bash tools/pmc_session.sh r02pmc
rc=$?; echo "frame pmc rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd "$ROOT"; python3 tools/pmc_sq.py "$(find gpurun_out/r02pmc/p4 -name "*counter_collection.csv" | head -1)" gpurun_out/r02pmc/plan_names.json > gpurun_out/r02pmc/sq.txt 2>&1; head -14 gpurun_out/r02pmc/sq.txt
bash tools/attn_pmc.sh r02apmc32 --batch 32
rc=$?; echo "attn pmc b32 rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd "$ROOT"; bash tools/attn_pmc.sh r02apmc1 --batch 1 --launches 50
rc=$?; echo "attn pmc b1 rc=$rc"
exit $rc
