#!/usr/bin/env python3
"""In-frame device time per plan entry of the full forward and of the template-K/V-cache search pass
(the same profiler mapping as bench.inframe_profile), summed by entry name, side by side.

usage: python tools/kv_breakdown.py --batch 1
"""
import argparse
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--variant", default="rgbt")
    args = ap.parse_args()
    import bench
    from mmt_amd import synthetic
    from mmt_amd.runtime import MixFormerRGBTRuntime

    keys = bench.state_dict_keys(args.variant, **bench.GEO_B)
    sd = {k: torch.from_numpy(v) for k, v in synthetic.synth_state_dict(keys).items()}
    rt = MixFormerRGBTRuntime(sd, args.variant, dtype=torch.bfloat16)
    t, o, s = [[x.cuda() for x in z] for z in synthetic.synth_inputs(args.batch, 128, 320, seed=0)]
    out = {"B": args.batch}
    for part in (None, "s"):
        if part == "s":
            tg = rt.capture_plan(rt.plan_for_inputs(t, o, None, part="t"))
            tg.replay()
            plan = rt.plan_for_inputs(None, None, s, part="s")
        else:
            plan = rt.plan_for_inputs(t, o, s)
        g = rt.capture_plan(plan)
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        times, span = bench.inframe_profile([g], plan, frames=20)
        by = defaultdict(float)
        for e, ms in zip(plan, times or []):
            by[e[2]] += ms * 1e3
        out["full" if part is None else "search_pass"] = {"span_us": round(span * 1e3, 1) if span else None,
                                                           "launches": len(plan),
                                                           "us": {k: round(v, 1) for k, v in by.items()}}
    print(json.dumps(out), flush=True)
    f, sp = out["full"]["us"], out["search_pass"]["us"]
    for k in f:
        print("%-34s %8.1f %8.1f" % (k, f[k], sp.get(k, 0.0)), flush=True)


if __name__ == "__main__":
    main()
