#!/bin/bash
# head per-stage error table; split-K vs unsplit tiles for the two split-K entries; training kernels under PMC
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05q; mkdir -p $OUT
timeout -k 10 200 python -u tools/head_stage_error.py > $OUT/head_stage.jsonl 2> $OUT/head_stage.err
rc=$?; echo "head rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/head_stage.err; exit $rc; }
timeout -k 10 200 python -u tools/plan_entry_ab.py --names head_conv1_adj12,enc_linear2 --cfgs 0:0,3:1,2:1,1:1,2:2,2:3,3:2 > $OUT/entry_ab.jsonl 2> $OUT/entry_ab.err
rc=$?; echo "entry rc=$rc"; cat $OUT/entry_ab.jsonl; [ $rc -ne 0 ] && { tail -5 $OUT/entry_ab.err; exit $rc; }
bash tools/sessions/session_r05p.sh
