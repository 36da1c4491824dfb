#!/bin/bash
# round 6, timing only: the split-K partial tiles stored plain (kept in the XCD's L2) instead of sc1 (write-through,
# dropped from L2), build variant v_skplain -- NOT coherent across XCDs, so no results are checked or kept; it
# measures how much of the split penalty is the last arriver reading the partials at the cross-XCD rate
set -u
T=${1:-r06skplain}; ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/$T; mkdir -p "$OUT"; cd "$ROOT"
N=fc2,qkv,fc1,proj,head_conv1_adj12,head_conv2,enc_linear2
C=0:0,1:1,1:2,1:3,1:4,2:1,2:2,2:3,3:1,3:2,3:3
for lib in product v_skplain; do
  if [ $lib = product ]; then unset MMT_HIP_LIB; else export MMT_HIP_LIB=multi-modal-tracking_amd/mmt_amd/_lib/$lib/libmmt_hip.so; fi
  timeout -k 10 240 python -u tools/plan_entry_ab.py --names $N --cfgs $C > "$OUT/entries_$lib.jsonl" 2>/dev/null || exit $?
done
python3 - "$OUT" <<'PY'
import json, sys
out = sys.argv[1]
a = {json.loads(l)["name"]: json.loads(l) for l in open(out + "/entries_product.jsonl")}
b = {json.loads(l)["name"]: json.loads(l) for l in open(out + "/entries_v_skplain.jsonl")}
for n in a:
    print(n, " ".join("%s %.1f/%.1f" % (k, a[n][k], b[n][k]) for k in a[n] if ":" in k))
PY
