#!/bin/bash
# Round 5: deterministic MSDA backward + unique bimodal queries in training; compact cache passes (32-bit row map)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/${1:-r05i}; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_backward_ops.py tests/test_gpu_cache.py tests/test_capi.py "tests/test_gpu_train_ops.py::test_train_step_graph_replay_matches_eager" "tests/test_gpu_train_ops.py::test_hip_adamw_load_state_dict_with_missing_entries" "tests/test_gpu_train_ops.py::test_head_forward_nhwc_sync_and_frozen_bn" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 "$OUT/pytest.log"
timeout -k 10 300 python -u tools/kv_breakdown.py --batch 1 > "$OUT/kv_b1.txt" 2>&1; echo "kv rc=$?"; grep -E "^qkv|^fc|^proj|^mam" "$OUT/kv_b1.txt"; grep -o '"span_us": [0-9.]*' "$OUT/kv_b1.txt"
timeout -k 10 400 python -u bench.py --train --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/train.json" 2> "$OUT/train.err"; echo "train rc=$?"; python3 -c "import json; d=json.load(open('$OUT/train.json')); print(d['value'], d['ms_per_step'])"
exit $rc
