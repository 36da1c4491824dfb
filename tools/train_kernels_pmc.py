#!/usr/bin/env python3
"""Training-step kernels in isolation, for counter collection: the config-4 shapes (16 pairs,
lockstep backbones: 2 x 8448 rows) of the backbone's Linear / MLP autograd Functions (forward, dX, dW) and the
fusion encoder's MSDA forward + backward, each case run `--reps` times between marker kernels
(torch.cuda._sleep), so that a rocprofv3 --pmc pass of this script (tools/sessions/session_r05p.sh) maps every dispatch to
its case without the bench's training line (the profiler crashed under the full bench with counters on).

  python tools/train_kernels_pmc.py --reps 3                 # run (under rocprofv3 --pmc ...)
  python tools/train_kernels_pmc.py --summarize DIR OUT.json  # FETCH_SIZE / WRITE_SIZE passes -> bytes per launch

Traffic per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB; gfx950 FETCH_SIZE counts half of wide coalesced reads,
MI355X_MICROARCH.md HBM section), per kernel name within each case, next to the algorithmic bytes of the GEMMs
(operands read once, outputs written once).
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))

CASES = ["qkv_linear2", "proj_linear_residual2", "mlp_residual2", "msda"]
M2, C, HID = 2 * 8448, 768, 3072
# algorithmic bytes per case and direction (bf16 operands, fp32 residual stream / dW): forward, dX, dW
ALGO = {
    "qkv_linear2": {"fwd": M2 * C * 2 + 2 * 3 * C * C * 2 + M2 * 3 * C * 2,
                    "dX": M2 * 3 * C * 2 + 2 * 3 * C * C * 2 + M2 * C * 2,
                    "dW": M2 * 3 * C * 2 + M2 * C * 2 + 2 * 3 * C * C * 4},
}


def run(reps):
    import torch
    from mmt_amd.train import HipOps
    torch.manual_seed(0)
    dev = "cuda"
    bf = torch.bfloat16
    mk = lambda *s, dt=torch.float32: (torch.randn(*s, device=dev) * 0.05).to(dt).requires_grad_(True)  # noqa: E731
    x32 = mk(M2, C)
    xb = mk(M2, C, dt=bf)
    wq = [mk(3 * C, C), mk(3 * C, C)]
    bq = [mk(3 * C), mk(3 * C)]
    wp = [mk(C, C), mk(C, C)]
    bp = [mk(C), mk(C)]
    p0 = (mk(HID, C), mk(HID), mk(C, HID), mk(C))
    p1 = (mk(HID, C), mk(HID), mk(C, HID), mk(C))
    keep = torch.ones(32, device=dev)
    value = mk(16, 800, 8, 64)
    loc = (torch.rand(16, 400, 8, 2, 4, 2, device=dev)).requires_grad_(True)
    aw = torch.softmax(torch.randn(16, 400, 8, 8, device=dev), -1).view(16, 400, 8, 2, 4).detach().requires_grad_(True)
    cases = {
        "qkv_linear2": lambda: HipOps.linear2(xb, wq[0], bq[0], wq[1], bq[1]).float().sum(),
        "proj_linear_residual2": lambda: HipOps.linear_residual2(x32, xb, wp[0], bp[0], wp[1], bp[1], keep).sum(),
        "mlp_residual2": lambda: HipOps.mlp_residual2(x32, xb, p0, p1, keep).sum(),
        "msda": lambda: HipOps.ms_deform_attn(value, 20, loc, aw).sum(),
    }
    for nm in CASES:  # warm-up (allocations, constants) outside the marked region
        cases[nm]().backward()
    torch.cuda.synchronize()
    for nm in CASES:
        torch.cuda._sleep(1000)  # marker
        for _ in range(reps):
            cases[nm]().backward()
        torch.cuda.synchronize()
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    print(json.dumps({"cases": CASES, "reps": reps}))


def read_pass(d, counter):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return rows


def summarize(d, out, reps):
    res = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        rows = read_pass(os.path.join(d, counter), counter)
        marks = [i for i, r in enumerate(rows) if "sleep" in r["Kernel_Name"].lower() or "spin" in r["Kernel_Name"].lower()]
        marks = marks[-(len(CASES) + 1):]  # the case markers (the last len(CASES) + 1 sleeps)
        for ci, nm in enumerate(CASES):
            seg = rows[marks[ci] + 1:marks[ci + 1]]
            by = defaultdict(list)
            for r in seg:
                by[r["Kernel_Name"][:90]].append(float(r["Counter_Value"]))
            for k, v in by.items():
                e = res.setdefault(nm, {}).setdefault(k, {"launches_per_rep": len(v) / reps})
                e[counter + "_KiB_per_launch"] = sum(v) / len(v)
    for nm, ks in res.items():
        for k, e in ks.items():
            f, w = e.get("FETCH_SIZE_KiB_per_launch"), e.get("WRITE_SIZE_KiB_per_launch")
            if f is not None and w is not None:
                e["traffic_MB_per_launch"] = round((2 * f + w) * 1024 / 1e6, 3)
    res["_note"] = "traffic = 2 x FETCH_SIZE + WRITE_SIZE per launch (gfx950 FETCH_SIZE halves wide reads)"
    res["_algorithmic_bytes"] = ALGO
    json.dump(res, open(out, "w"), indent=1)
    for nm in CASES:
        for k, e in res.get(nm, {}).items():
            print("%-22s %-70s %5.1f %10s" % (nm, k[:70], e["launches_per_rep"], e.get("traffic_MB_per_launch")))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--summarize", nargs=2, metavar=("DIR", "OUT"))
    args = ap.parse_args()
    if args.summarize:
        summarize(args.summarize[0], args.summarize[1], args.reps)
    else:
        run(args.reps)


if __name__ == "__main__":
    main()
