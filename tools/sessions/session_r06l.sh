#!/bin/bash
# round 6: full GPU suite + smoke + default bench, then the training step's aten call sites and a
# one-step rocprof kernel breakdown
set -u
bash tools/sessions/session_r06full.sh r06full1 || exit $?
OUT=gpurun_out/r06full1
timeout -k 10 300 python -u tools/train_aten_sites.py > $OUT/train_aten_sites.txt 2>&1
rc=$?; echo "aten sites rc=$rc"; head -30 $OUT/train_aten_sites.txt | cut -c1-200; [ $rc -ne 0 ] && exit $rc
bash tools/session_trainprof.sh r06tp
