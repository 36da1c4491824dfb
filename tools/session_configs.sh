#!/bin/bash
# Bench lines of the other BASELINE configurations on one GPU (appended to gpurun_out/TAG/configs.jsonl):
# RGB-only MixViT-B fp16 (config 1's model), shared backbone with 64 sequences (config 3's per-node
# workload), ViT-L + score head fp16 (config 5), the training step (config 4, tools/train_bench.py).
set -u
TAG=${1:-configs}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$ROOT"
run() {  # name, command...
  local name=$1; shift
  timeout -k 10 400 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && return $rc
  grep -h '^{' "$OUT/$name.log" | tail -1 >> "$OUT/configs.jsonl"
}
run rgb_fp16 python -u bench.py --variant rgb --dtype fp16 --no-cpu-baseline --no-mam-batched --no-kv-cache &&
run shared64 python -u bench.py --variant shared --total-seqs 64 --no-cpu-baseline --no-kv-cache &&
run vitl_fp16 python -u bench.py --vitl --variant asym_online --dtype fp16 --no-cpu-baseline --no-mam-batched --no-kv-cache &&
run train python -u tools/train_bench.py
rc=$?
cut -c1-200 "$OUT/configs.jsonl"
exit $rc
