#!/bin/bash
# training gradient GEMMs: tile / split-K choices (dW and dX of the four ViT Linears, lockstep pair)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05v; mkdir -p $OUT
timeout -k 10 400 python -u tools/train_gemm_ab.py > $OUT/train_gemm_ab.jsonl 2> $OUT/train_gemm_ab.err
rc=$?; echo "rc=$rc"; cat $OUT/train_gemm_ab.jsonl; tail -3 $OUT/train_gemm_ab.err; exit $rc
