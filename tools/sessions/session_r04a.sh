#!/bin/bash
# Round-4 first session: the new / changed GPU tests, the MAM and batch-1 GEMM baselines (hipBLASLt bar).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r04a
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_train_ops.py -m gpu -q -rf --timeout 300 \
    --timeout-method thread -k "reference_fixture or groupnorm or adamw or layernorm_backward" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest.log"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/attn_ab.py --impls 22 --batches 8,32 > "$OUT/attn_ab.jsonl" 2>&1
rc=$?; echo "attn rc=$rc"; grep -v amdgpu.ids "$OUT/attn_ab.jsonl" | tail -6
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/gemm_ab.py --only qkv,proj,fc1,fc2,qkv_ln,fc1_ln --impls 0:0 > "$OUT/gemm_b1.jsonl" 2>&1
rc=$?; echo "gemm rc=$rc"; grep -v amdgpu.ids "$OUT/gemm_b1.jsonl" | tail -8
exit $rc
