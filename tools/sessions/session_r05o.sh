#!/bin/bash
# training corner head: per-stage error table (HIP vs aten bf16 autocast vs aten fp32)
set -u
OUT=gpurun_out/r05o; mkdir -p $OUT
timeout -k 10 200 python -u tools/head_stage_error.py > $OUT/head_stage.jsonl 2> $OUT/head_stage.err
rc=$?; echo "rc=$rc"; cat $OUT/head_stage.jsonl; tail -3 $OUT/head_stage.err; exit $rc
