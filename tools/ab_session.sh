#!/bin/bash
# GEMM kernel A/B (+ ablation / stamp builds) and the GPU parity tests; outputs under gpurun_out/ab2.
set -o pipefail
mkdir -p gpurun_out/ab2
LIBDIR=$PWD/multi-modal-tracking_amd/mmt_amd/_lib
timeout -k 10 400 python -m pytest tests/test_gpu_ops.py -q -x > gpurun_out/ab2/pytest_ops.log 2>&1; rc=$?
tail -3 gpurun_out/ab2/pytest_ops.log
if [ $rc -gt 1 ]; then exit $rc; fi
MMT_HIP_LIB=$LIBDIR/stamp/libmmt_hip.so timeout -k 10 200 python tools/gemm_stamps.py > gpurun_out/ab2/stamps.log 2>&1 || exit $?
timeout -k 10 300 python tools/gemm_ab.py > gpurun_out/ab2/full.log 2>&1 || exit $?
timeout -k 10 400 python -m pytest tests/test_gpu_model.py -q -x > gpurun_out/ab2/pytest_model.log 2>&1; tail -3 gpurun_out/ab2/pytest_model.log
