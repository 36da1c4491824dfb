#!/bin/bash
# round 6: impl 29 stamps + ablation variants (free-running, no exponentials)
set -u
OUT=gpurun_out/r06c; mkdir -p $OUT
MMT_HIP_LIB=multi-modal-tracking_amd/mmt_amd/_lib/stamp/libmmt_hip.so timeout -k 10 120 python -u tools/attn_ps_stamps.py --batches 1,8,32 > $OUT/stamps.jsonl 2> $OUT/stamps.err
rc=$?; echo "stamps rc=$rc"; cat $OUT/stamps.jsonl; [ $rc -ne 0 ] && { tail -5 $OUT/stamps.err; exit $rc; }
for v in free noexp; do
  MMT_HIP_LIB=multi-modal-tracking_amd/mmt_amd/_lib/$v/libmmt_hip.so timeout -k 10 120 python -u tools/attn_ab.py --batches 1,32 --impls 22,29 > $OUT/ab_$v.jsonl 2> $OUT/ab_$v.err
  rc=$?; echo "ab $v rc=$rc"; cat $OUT/ab_$v.jsonl; [ $rc -ne 0 ] && exit $rc
done
exit 0
