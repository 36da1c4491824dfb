#!/bin/bash
set -u
OUT=gpurun_out/r06k; mkdir -p $OUT
for v in nostage nostore free; do
  MMT_HIP_LIB=multi-modal-tracking_amd/mmt_amd/_lib/$v/libmmt_hip.so timeout -k 10 120 python -u tools/attn_ab.py --batches 32 --impls 29 > $OUT/ab_$v.jsonl 2> $OUT/ab_$v.err
  rc=$?; echo "ab $v rc=$rc"; cat $OUT/ab_$v.jsonl; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 120 python -u tools/attn_ab.py --batches 32 --impls 22,29 > $OUT/ab.jsonl 2> $OUT/ab.err; cat $OUT/ab.jsonl
