#!/bin/bash
# Round 4: the new / changed GPU tests (impl 24 MAM kernel, reference MAM fixture, GroupNorm / AdamW),
# MAM A/B (impl 22 vs 24), batch-1 GEMMs vs hipBLASLt.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r04b
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -rf --timeout 120 --timeout-method thread \
    -k "mam or attention" > "$OUT/pytest_attn.log" 2>&1
rc=$?; echo "pytest attn rc=$rc"; tail -5 "$OUT/pytest_attn.log"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/attn_ab.py --impls 4,22,24,25 --batches 1,2,4,8,32 > "$OUT/attn_ab.jsonl" 2>&1
rc=$?; echo "attn rc=$rc"; grep -v amdgpu.ids "$OUT/attn_ab.jsonl" | tail -8
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_ops.py tests/test_gpu_cache.py tests/test_gpu_ce.py -m gpu -q -rf --timeout 120 \
    --timeout-method thread -k "groupnorm or adamw or layernorm_backward or impl" > "$OUT/pytest_misc.log" 2>&1
rc=$?; echo "pytest misc rc=$rc"; tail -5 "$OUT/pytest_misc.log"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/gemm_ab.py --only qkv,proj,fc1,fc2,qkv_ln,fc1_ln --impls 0:0 > "$OUT/gemm_b1.jsonl" 2>&1
rc=$?; echo "gemm rc=$rc"; grep -v amdgpu.ids "$OUT/gemm_b1.jsonl" | tail -8
exit $rc
