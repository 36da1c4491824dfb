#!/bin/bash
# round 6: a 5-slot LDS-DMA ring for the one-per-CU 128x128 / 64x64 tiles (MMT_GEMM_ST_B1=5, build variant st5):
# the GEMM tests on the variant, per-entry times, then interleaved frame rates (product / st5)
set -u
T=${1:-r06st5}; ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$T; mkdir -p "$OUT"; cd "$ROOT"
V=multi-modal-tracking_amd/mmt_amd/_lib/st5/libmmt_hip.so
MMT_HIP_LIB=$V timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_model.py -k "gemm or conv or model or golden" > "$OUT/gemm_tests.txt" 2>&1
rc=$?; echo "gemm tests (st5) rc=$rc"; tail -2 "$OUT/gemm_tests.txt"; [ $rc -ne 0 ] && exit $rc
N=qkv,fc1,fc2,proj,patch_gemm,head_conv1_adj12,head_conv2,enc_linear2,fusion_adjust
for lib in product st5 product st5; do
  if [ $lib = st5 ]; then export MMT_HIP_LIB=$V; else unset MMT_HIP_LIB; fi
  timeout -k 10 200 python -u tools/plan_entry_ab.py --names $N --cfgs 0:0 > "$OUT/entries_$lib.jsonl" 2>/dev/null || exit $?
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-train-line --no-mam-batched --no-kv-cache --no-fp16-line --no-tracker-line --steps 400 > "$OUT/bench_$lib.json" 2>/dev/null || exit $?
  python3 -c "
import json; d=json.loads(open('$OUT/bench_$lib.json').read().strip().splitlines()[-1]); e=[json.loads(l) for l in open('$OUT/entries_$lib.jsonl')]
print('$lib', d['value'], {x['name']: x['0:0'] for x in e})"
done
