#!/bin/bash
# round 6: training step after the head changes: bench --train, aten call sites, one-step rocprof breakdown
set -u
OUT=gpurun_out/r06s; mkdir -p $OUT
timeout -k 10 300 python -u bench.py --train > $OUT/train.json 2> $OUT/train.err
rc=$?; echo "train rc=$rc"; cut -c1-300 $OUT/train.json; [ $rc -ne 0 ] && { tail -5 $OUT/train.err; exit $rc; }
timeout -k 10 300 python -u tools/train_aten_sites.py --top 30 > $OUT/sites.txt 2>&1
rc=$?; echo "sites rc=$rc"; grep -v Warn $OUT/sites.txt | head -34 | cut -c1-200; [ $rc -ne 0 ] && exit $rc
bash tools/session_trainprof.sh r06s_tp
