#!/bin/bash
set -u
OUT=gpurun_out/r06n; mkdir -p $OUT
timeout -k 10 300 python -u tools/train_aten_sites.py --top 60 > $OUT/train_aten_sites.txt 2>&1
rc=$?; echo "aten sites rc=$rc"; grep -v Warning $OUT/train_aten_sites.txt | head -64 | cut -c1-230; [ $rc -ne 0 ] && exit $rc
GAINS=30,6,2 timeout -k 10 600 python -u tools/grad_fixture_probe.py > $OUT/grad_probe.jsonl 2> $OUT/grad_probe.err
rc=$?; echo "probe rc=$rc"; cat $OUT/grad_probe.jsonl; tail -3 $OUT/grad_probe.err; exit $rc
