#!/bin/bash
# impl 26 stamps: the stamp build and the ablation builds (no exp / no MFMA / no loop barrier / no fragment reads)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/${1:-r05c}; mkdir -p "$OUT"; cd "$ROOT"
for v in ${VARIANTS:-pgp0 pgp1 pgp2 pgp2nb}; do
  MMT_HIP_LIB=$ROOT/multi-modal-tracking_amd/mmt_amd/_lib/$v/libmmt_hip.so timeout -k 10 120 python -u tools/pg_stamps.py --batches 8,32 --label $v >> "$OUT/pg_stamps.jsonl" 2> "$OUT/pg_stamps_$v.err"
  rc=$?; echo "$v rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/pg_stamps_$v.err"; exit $rc; }
done
cat "$OUT/pg_stamps.jsonl"
