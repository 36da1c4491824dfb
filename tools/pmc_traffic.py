#!/usr/bin/env python3
"""HBM traffic per launch of each plan entry from the FETCH_SIZE / WRITE_SIZE passes of
tools/pmc_session.sh, merged into profiles/pmc_traffic.json under "<variant>/B<batch>/<dtype>".

gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE counts half the bytes of wide coalesced
reads (16 B/lane, global_load and LDS-DMA alike), so traffic = 2 x FETCH_SIZE + WRITE_SIZE (KiB).
Dispatches are mapped to plan entries by order: every step starts with the patch_im2col kernel
and dispatches len(plan) kernels (the plan names come from bench.py --dump-plan).

usage: tools/pmc_traffic.py OUT_DIR PLAN_NAMES.json KEY [profiles/pmc_traffic.json]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_name(csv_path, counter, names):
    rows = [r for r in csv.DictReader(open(csv_path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    starts = [i for i, r in enumerate(rows) if "patch_im2col" in r["Kernel_Name"]]
    acc = defaultdict(list)
    for st in starts:
        seq = rows[st:st + len(names)]
        if len(seq) < len(names):
            break
        for nm, r in zip(names, seq):
            acc[nm].append(float(r["Counter_Value"]))
    return {nm: sum(v) / len(v) for nm, v in acc.items()}


def main():
    out_dir, names_file, key = sys.argv[1], sys.argv[2], sys.argv[3]
    dst = sys.argv[4] if len(sys.argv) > 4 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                             "pmc_traffic.json")
    names = json.load(open(names_file))
    fetch = write = None
    for f in glob.glob(os.path.join(out_dir, "p*", "**", "*counter_collection.csv"), recursive=True):
        hdr = open(f).read(4096)
        if "FETCH_SIZE" in hdr or any("FETCH_SIZE" in r["Counter_Name"] for r in csv.DictReader(open(f))):
            fetch = per_name(f, "FETCH_SIZE", names) or fetch
        if any("WRITE_SIZE" == r["Counter_Name"] for r in csv.DictReader(open(f))):
            write = per_name(f, "WRITE_SIZE", names) or write
    if not fetch or not write:
        sys.exit("FETCH_SIZE / WRITE_SIZE passes not found under %s" % out_dir)
    res = {}
    for nm in names:
        if nm in fetch and nm in write:
            fb, wb = 2 * fetch[nm] * 1024, write[nm] * 1024
            res[nm] = {"fetch_bytes": round(fb), "write_bytes": round(wb), "traffic_bytes": round(fb + wb)}
    try:
        allres = json.load(open(dst))
    except (OSError, ValueError):
        allres = {}
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multi-modal-tracking_amd"))
    from mmt_amd.stamp import source_digest
    # the kernel sources these counts were taken on: bench.py reports them only for the same digest
    res["_stamp"] = {"source_digest": source_digest(), "git_head": os.environ.get("MMT_GIT_HEAD", "")}
    allres[key] = res
    with open(dst, "w") as f:
        json.dump(allres, f, indent=1, sort_keys=True)
    for nm in sorted((k for k in res if not k.startswith("_")), key=lambda k: -res[k]["traffic_bytes"])[:12]:
        print("%-22s fetch %8.2f MB  write %8.2f MB" % (nm, res[nm]["fetch_bytes"] / 1e6, res[nm]["write_bytes"] / 1e6))


if __name__ == "__main__":
    main()
