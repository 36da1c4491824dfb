#!/usr/bin/env python3
"""Container-side validation of bench.py's CPU baseline (BASELINE.md "CPU-baseline plan"): the
oracle's fp32 CPU forward (oracle/forward.py, the `port` bench.py times on the GPU box's host) must
run within +-15 % of the REFERENCE's own forward on the same threads and inputs, so that the GPU/CPU
ratio bench.py reports is not flattered by a slow restatement.

Runs here only (the reference does not travel): the reference is imported read-only with the stub
recipe of tests/golden/make_golden.py.  Interleaved timing (reference, oracle, ...),
median of N forwards each after warm-up, B = 1, torch.set_num_threads(THREADS); writes one JSON line
per variant (and profiles/cpu_baseline_check.json with --out).

usage: python tools/cpu_baseline_check.py [--threads 8] [--n 5] [--variants rgbt,shared,asym] [--out PATH]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import make_golden as mg  # noqa: E402  (stubs, reference builders; nothing is written under /root/reference)
import torch  # noqa: E402


def lscpu():
    info = {}
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for ln in out.splitlines():
            k, _, v = ln.partition(":")
            if k.strip() in ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core", "CPU(s)"):
                info[k.strip()] = v.strip()
    except Exception:
        pass
    return info


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--n", type=int, default=5)
    ap.add_argument("--variants", default="rgbt,shared,asym")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    mg.install_stubs()
    from mmt_amd import synthetic
    from oracle.forward import forward as oracle_forward
    rows = []
    for variant in a.variants.split(","):
        torch.manual_seed(0)
        model = mg.build(variant, mg.make_cfg()).eval()
        keys = [(k, list(v.shape)) for k, v in model.state_dict().items()]
        sd_np = synthetic.synth_state_dict(keys)
        sd = {k: torch.from_numpy(v) for k, v in sd_np.items()}
        model.load_state_dict(sd, strict=True)
        t, o, s = synthetic.synth_inputs(1)
        with torch.no_grad():
            ref_out, _ = model(t, o, s)
        mine, _ = oracle_forward(sd, variant, t, o, s)
        err = (mine["pred_boxes"] - ref_out["pred_boxes"]).abs().max().item()
        tr, to = [], []
        for i in range(a.n + 2):
            t0 = time.perf_counter()
            with torch.no_grad():
                model(t, o, s)
            t1 = time.perf_counter()
            oracle_forward(sd, variant, t, o, s)
            t2 = time.perf_counter()
            if i >= 2:
                tr.append(t1 - t0)
                to.append(t2 - t1)
        fr, fo = 1.0 / statistics.median(tr), 1.0 / statistics.median(to)
        row = {"variant": variant, "threads": a.threads, "reference_fps": round(fr, 3), "oracle_fps": round(fo, 3),
               "oracle_over_reference": round(fo / fr, 3), "within_15pct": abs(fo / fr - 1.0) <= 0.15,
               "box_err_vs_reference": err, "n": a.n}
        rows.append(row)
        print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"host": lscpu(), "rows": rows}, f, indent=1)
    if not all(r["within_15pct"] for r in rows):
        sys.exit(1)


if __name__ == "__main__":
    main()
