#!/bin/bash
set -u
OUT=gpurun_out/r06d; mkdir -p $OUT
MMT_HIP_LIB=multi-modal-tracking_amd/mmt_amd/_lib/stamp/libmmt_hip.so timeout -k 10 120 python -u tools/attn_ps_stamps.py --batches 32 > $OUT/stamps.jsonl 2> $OUT/stamps.err
rc=$?; echo "stamps rc=$rc"; cat $OUT/stamps.jsonl; [ $rc -ne 0 ] && { tail -5 $OUT/stamps.err; exit $rc; }
exit 0
