#!/bin/bash
# impl 9 (256x256 at one wave per SIMD): GEMM parity tests, then A/B against the library's choice / impl 7 / 8
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05z; mkdir -p $OUT; cd $ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "tile_paths or gelu_backward or column_split or row_scale or stats_handoff" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u tools/gemm_ab.py --impls 0:0,7:1,8:1,9:1 \
    --only qkv_T16,fc1_T16,fc2_T16,proj_T16,dX_fc2_T16,fc2_B8,fc1_B8,g1_qkv,g1_fc2,c3_qkv_ln2,c3_fc1_ln2,c3_proj,c3_fc2 \
    > $OUT/gemm_ab.jsonl 2> $OUT/gemm_ab.err
rc=$?; echo "ab rc=$rc"; cat $OUT/gemm_ab.jsonl | cut -c1-600; tail -3 $OUT/gemm_ab.err; exit $rc
