#!/usr/bin/env python3
"""Per-plan-entry device time from a rocprofv3 kernel trace of bench.py.

Each hipGraph replay dispatches the plan's kernels in plan order; this maps dispatches to plan
entry names (re-building the plan on CPU is not possible, so the names are read from a JSON list
written by `bench.py --dump-plan`, or by matching kernel-name prefixes) and prints the average
duration per entry and per step.

usage: tools/trace_breakdown.py TRACE.csv PLAN_NAMES.json
"""
import csv
import json
import sys
from collections import defaultdict


def main():
    trace, names_file = sys.argv[1], sys.argv[2]
    names = json.load(open(names_file))
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    first = names[0]
    # the plan's first kernel (patch im2col) starts every step
    starts = [i for i, r in enumerate(rows) if "patch_im2col" in r["Kernel_Name"]]
    per = defaultdict(list)
    step_spans = []
    for s in starts:
        seq = rows[s:s + len(names)]
        if len(seq) < len(names):
            break
        step_spans.append((int(seq[-1]["End_Timestamp"]) - int(seq[0]["Start_Timestamp"])) / 1e3)
        for nm, r in zip(names, seq):
            per[nm].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for nm, v in per.items():
        tot[nm] = sum(v)
        cnt[nm] = len(v)
    nsteps = len(step_spans)
    print("steps %d, span per step %.1f us (median), kernel sum per step %.1f us" % (
        nsteps, sorted(step_spans)[nsteps // 2], sum(tot.values()) / max(nsteps, 1)))
    for nm in sorted(tot, key=lambda k: -tot[k]):
        launches = cnt[nm] / nsteps
        print("%-22s %8.2f us avg  x%-3d  %6.1f us/step" % (nm, tot[nm] / cnt[nm], launches, tot[nm] / nsteps))
    _ = first


if __name__ == "__main__":
    main()
