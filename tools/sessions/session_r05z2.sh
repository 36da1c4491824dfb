#!/bin/bash
# impl 9 on the config-3 shapes (LayerNorm fold with handed-in statistics; residual producers)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05z; mkdir -p $OUT; cd $ROOT
timeout -k 10 300 python -u tools/gemm_ab.py --impls 0:0,9:1 --only c3_qkv_ln2,c3_fc1_ln2 > $OUT/gemm_ab_c3.jsonl 2> $OUT/gemm_ab_c3.err
rc=$?; echo "ab rc=$rc"; [ $rc -ne 0 ] && { tail -3 $OUT/gemm_ab_c3.err; exit $rc; }
timeout -k 10 300 python -u tools/gemm_ab.py --impls 0:0,8:1,9:1 --only c3_proj,c3_fc2 >> $OUT/gemm_ab_c3.jsonl 2>> $OUT/gemm_ab_c3.err
rc=$?; echo "ab rc=$rc"; cat $OUT/gemm_ab_c3.jsonl | cut -c1-600; tail -3 $OUT/gemm_ab_c3.err; exit $rc
