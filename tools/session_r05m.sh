#!/bin/bash
# prototype 256x256 four-wave GEMM tile: ablation builds (1 no DMA, 2 no MFMA, 3 no fragment reads)
set -u
OUT=gpurun_out/r05m2; mkdir -p $OUT
for a in 1 2 3; do
  timeout -k 10 200 python -u tools/proto_gemm256.py --no-mmt --no-check --only fc2_T16,fc1_T16 --tag abl$a --lib tools/proto/libproto_gemm256_abl$a.so >> $OUT/proto.jsonl 2>> $OUT/proto.err
  rc=$?; echo "abl$a rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
cat $OUT/proto.jsonl
