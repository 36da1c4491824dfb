#!/bin/bash
# row-group tile order for the two-per-CU tiles (impl 8): per-shape GEMM A/B, then interleaved training / config-3
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05t; mkdir -p $OUT
for v in base cur; do
  if [ $v = cur ]; then unset MMT_HIP_LIB; else export MMT_HIP_LIB=$ROOT/multi-modal-tracking_amd/mmt_amd/_lib/$v/libmmt_hip.so; fi
  timeout -k 10 300 python -u tools/gemm_ab.py --impls 0:0 --no-torch --only qkv_T16,fc1_T16,fc2_T16,proj_T16,dX_fc2_T16,dW_fc1_T16,dW_fc2_T16,fc1_B8,fc2_B8,g1_dX_fc1,g1_dW_fc1 > $OUT/gemm_$v.jsonl 2> $OUT/gemm_$v.err
  rc=$?; echo "gemm $v rc=$rc"; [ $rc -ne 0 ] && { tail -3 $OUT/gemm_$v.err; exit $rc; }
done
unset MMT_HIP_LIB
python3 - <<PY
import json
b=[json.loads(l) for l in open("$OUT/gemm_base.jsonl")]; c=[json.loads(l) for l in open("$OUT/gemm_cur.jsonl")]
for x,y in zip(b,c): print(x["gemm"], x["impl0:0"]["us"], "->", y["impl0:0"]["us"])
PY
bash tools/ab_lib_train.sh r05t_ab base 2
