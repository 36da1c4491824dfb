#!/usr/bin/env python3
"""Per-kernel device time of ONE steady-state training step from a rocprofv3 kernel trace of
`bench.py --train` (tools/session_trainprof.sh): the window after the last-but-one step's final
attention-backward dQ launch (24 per step for the two-stream ViT-B: 12 blocks x 2 backbones), i.e. the
last step, so MIOpen's first-call algorithm searches in the warm-up steps are excluded.

usage: tools/train_breakdown.py TRACE.csv [dq_per_step]"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    per_step = int(sys.argv[2]) if len(sys.argv) > 2 else 24
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dq = [i for i, r in enumerate(rows) if "mam_bwd_dq" in r["Kernel_Name"]]
    win = rows[dq[-per_step - 1] + 1:]
    t0, t1 = int(win[0]["Start_Timestamp"]), int(win[-1]["End_Timestamp"])
    agg = collections.defaultdict(lambda: [0, 0])
    for r in win:
        agg[r["Kernel_Name"][:100]][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg[r["Kernel_Name"][:100]][1] += 1
    tot = sum(v[0] for v in agg.values())
    print("last step: span %.2f ms, kernel sum %.2f ms, %d launches" % ((t1 - t0) / 1e6, tot / 1e6, len(win)))
    for n, (d, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:40]:
        print("%8.3f ms %5d  %s" % (d / 1e6, c, n))


if __name__ == "__main__":
    main()
