#!/bin/bash
# prototype 256x256 four-wave GEMM tile without s_nop pads: LDS-DMA ring, register-staged, ablations
set -u
OUT=gpurun_out/r05m3; mkdir -p $OUT
timeout -k 10 200 python -u tools/proto_gemm256.py --no-mmt --tag k32ring4_nonop >> $OUT/proto.jsonl 2>> $OUT/proto.err
rc=$?; echo "dma rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/proto_gemm256.py --no-mmt --tag regstaged_nonop --lib tools/proto/libproto_gemm256_rs.so >> $OUT/proto.jsonl 2>> $OUT/proto.err
rc=$?; echo "rs rc=$rc"; [ $rc -ne 0 ] && exit $rc
for a in 1 2 3; do
  timeout -k 10 200 python -u tools/proto_gemm256.py --no-mmt --no-check --only fc2_T16,fc1_T16 --tag abl${a}_nonop --lib tools/proto/libproto_gemm256_abl$a.so >> $OUT/proto.jsonl 2>> $OUT/proto.err
  rc=$?; echo "abl$a rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
cat $OUT/proto.jsonl
