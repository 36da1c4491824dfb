#!/usr/bin/env python3
"""Per-kernel device time of ONE steady-state training step from a rocprofv3 kernel trace of
`bench.py --train` (tools/session_trainprof.sh).  The step is bracketed by the optimizer: every step ends
with exactly one `adamw_step_kernel` launch (mmt_amd.optim.HipAdamW, csrc/optim.hip), so the window is
the launches after one adamw_step up to and including the next -- the last complete step before the
final one, so that whatever the harness launches after its timed region is excluded.  (Round 5 took the
window from a count of attention-backward dQ launches, which the lockstep two-stream backbone halved:
that window spanned ~2.15 steps.)

usage: tools/train_breakdown.py TRACE.csv"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    opt = [i for i, r in enumerate(rows) if "adamw_step_kernel" in r["Kernel_Name"]]
    if len(opt) < 2:
        sys.exit("need at least two optimizer steps in the trace")
    a, b = (opt[-3], opt[-2]) if len(opt) >= 3 else (opt[-2], opt[-1])
    win = rows[a + 1:b + 1]
    t0, t1 = int(win[0]["Start_Timestamp"]), int(win[-1]["End_Timestamp"])
    agg = collections.defaultdict(lambda: [0, 0])
    for r in win:
        agg[r["Kernel_Name"][:100]][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg[r["Kernel_Name"][:100]][1] += 1
    tot = sum(v[0] for v in agg.values())
    ours = sum(v[0] for k, v in agg.items() if "anonymous namespace" in k)
    print("one step (between optimizer launches %d and %d of %d): span %.2f ms, kernel sum %.2f ms, %d launches, "
          "libmmt_hip kernels %.1f %% of the kernel sum" % (len(opt) - (3 if len(opt) >= 3 else 2) + 1,
                                                             len(opt) - (2 if len(opt) >= 3 else 1) + 1, len(opt),
                                                             (t1 - t0) / 1e6, tot / 1e6, len(win), 100.0 * ours / tot))
    for n, (d, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:40]:
        print("%8.3f ms %5d  %s" % (d / 1e6, c, n))


if __name__ == "__main__":
    main()
