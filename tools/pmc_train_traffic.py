#!/usr/bin/env python3
"""HBM traffic of one whole training step from the FETCH_SIZE / WRITE_SIZE passes of tools/sessions/session_r05tpmc.sh
(rocprofv3 --pmc over `bench.py --train`, the step one hipGraph replay): the dispatches between consecutive AdamW
update kernels are one step; traffic = 2 x FETCH_SIZE + WRITE_SIZE (KiB, gfx950 correction, MI355X_MICROARCH.md),
the median over the recorded steps, merged into profiles/pmc_traffic.json under "train/B<batch>/bf16" with the
kernel-source stamp (bench.py reports it in train_step.roofline.traffic for the same digest).

usage: tools/pmc_train_traffic.py OUT_DIR [BATCH] [profiles/pmc_traffic.json]
"""
import csv
import glob
import json
import os
import statistics
import sys


def per_step(path, counter, family=None):
    """(launches, counter sum) of every step; family: only kernels whose name contains it (the dominant
    training family, "gemm")."""
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    ends = [i for i, r in enumerate(rows) if "adamw_step_kernel" in r["Kernel_Name"]]
    sel = (lambda r: True) if family is None else (lambda r: family in r["Kernel_Name"])
    steps = [(sum(1 for r in rows[a + 1:b + 1] if sel(r)), sum(float(r["Counter_Value"]) for r in rows[a + 1:b + 1] if sel(r)))
             for a, b in zip(ends, ends[1:])]
    return steps


def main():
    out = sys.argv[1]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    dst = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(__file__), "..", "profiles", "pmc_traffic.json")
    vals, gvals = {}, {}
    for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
        names = {r["Counter_Name"] for r in csv.DictReader(open(f))}
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            if c in names:
                vals[c] = per_step(f, c)
                gvals[c] = per_step(f, c, "gemm")
    if len(vals) != 2:
        sys.exit("FETCH_SIZE / WRITE_SIZE passes not found under %s" % out)
    fb = 2 * statistics.median(v for _, v in vals["FETCH_SIZE"]) * 1024
    wb = statistics.median(v for _, v in vals["WRITE_SIZE"]) * 1024
    launches = statistics.median(n for n, _ in vals["FETCH_SIZE"])
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multi-modal-tracking_amd"))
    from mmt_amd.stamp import source_digest
    gfb = 2 * statistics.median(v for _, v in gvals["FETCH_SIZE"]) * 1024
    gwb = statistics.median(v for _, v in gvals["WRITE_SIZE"]) * 1024
    res = {"step": {"fetch_bytes": round(fb), "write_bytes": round(wb), "traffic_bytes": round(fb + wb),
                    "launches": launches, "steps": len(vals["FETCH_SIZE"])},
           "gemm": {"fetch_bytes": round(gfb), "write_bytes": round(gwb), "traffic_bytes": round(gfb + gwb),
                    "launches": statistics.median(n for n, _ in gvals["FETCH_SIZE"])},
           "_stamp": {"source_digest": source_digest(train=True), "git_head": os.environ.get("MMT_GIT_HEAD", "")}}
    try:
        allres = json.load(open(dst))
    except (OSError, ValueError):
        allres = {}
    allres["train/B%d/bf16" % B] = res
    with open(dst, "w") as f:
        json.dump(allres, f, indent=1, sort_keys=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
