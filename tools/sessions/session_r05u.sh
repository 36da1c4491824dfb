#!/bin/bash
# row tiles per row group of the large-grid GEMM tile order: 4 / 16 vs the product's 8 (training + config 3)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
bash tools/ab_lib_train.sh r05u_gm4 gm4 1 && bash tools/ab_lib_train.sh r05u_gm16 gm16 1
