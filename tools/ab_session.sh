#!/bin/bash
# GEMM kernel A/B (+ ablation builds) and the GPU op parity tests; outputs under gpurun_out/ab2.
set -o pipefail
mkdir -p gpurun_out/ab2
timeout -k 10 400 python -m pytest tests/test_gpu_ops.py -q -x > gpurun_out/ab2/pytest_ops.log 2>&1; rc=$?
tail -3 gpurun_out/ab2/pytest_ops.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/gemm_ab.py > gpurun_out/ab2/full.log 2>&1 || exit $?
MMT_HIP_LIB=$PWD/multi-modal-tracking_amd/mmt_amd/_lib/ablate1/libmmt_hip.so timeout -k 10 200 python tools/gemm_ab.py --impls 1,2,3 --no-torch > gpurun_out/ab2/ablate1.log 2>&1 || exit $?
MMT_HIP_LIB=$PWD/multi-modal-tracking_amd/mmt_amd/_lib/ablate2/libmmt_hip.so timeout -k 10 200 python tools/gemm_ab.py --impls 1,2,3 --no-torch > gpurun_out/ab2/ablate2.log 2>&1 || exit $?
timeout -k 10 400 python -m pytest tests/test_gpu_model.py -q -x > gpurun_out/ab2/pytest_model.log 2>&1; tail -3 gpurun_out/ab2/pytest_model.log
