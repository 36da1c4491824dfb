#!/bin/bash
# Round 6: impl 8 split-K for the weight gradients -- GEMM tests, then the training step interleaved against the
# library built before the change (MMT_HIP_LIB=.../pre_sk2), one process per run.
# usage: bash tools/sessions/session_r06sk.sh TAG [ROUNDS]
set -o pipefail
TAG=${1:-r06sk}; ROUNDS=${2:-3}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -m gpu \
    -k "mn_major or splitk" > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in $(seq 1 $ROUNDS); do
    for v in product pre_sk2; do
        if [ $v = product ]; then unset MMT_HIP_LIB; else export MMT_HIP_LIB=multi-modal-tracking_amd/mmt_amd/_lib/$v/libmmt_hip.so; fi
        timeout -k 10 240 python -u bench.py --train --steps 20 --warmup 5 --no-cpu-baseline > $OUT/train_${v}_$i.log 2>&1 \
            || { tail -20 $OUT/train_${v}_$i.log; exit 1; }
        python - "$v" "$i" $OUT/train_${v}_$i.log <<'EOF' | tee -a $OUT/ab.jsonl
import json, sys
line = [l for l in open(sys.argv[3]) if l.startswith("{")][-1]
d = json.loads(line)
print(json.dumps({"variant": sys.argv[1], "round": int(sys.argv[2]), "samples_per_s": d["value"], "ms_per_step": d["ms_per_step"]}))
EOF
    done
done
unset MMT_HIP_LIB
