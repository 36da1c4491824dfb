#!/usr/bin/env python3
"""A/B timing of single frame-plan GEMM entries under forced (impl, splitk) choices, in place in the
real launch plan (same pointers, strides, conv / LN-fold flags as the tracked frame): `per_graph`
back-to-back launches of the entry in one hipGraph, timed with HIP events (as bench.kernel_profile).

usage: python tools/plan_entry_ab.py --names head_conv1_adj12,head_conv2 --cfgs 0:0,1:4,2:3,3:1
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def time_entry(fn, args, per_graph=20, replays=5):
    s = torch.cuda.current_stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(per_graph):
            fn(*args, torch.cuda.current_stream().cuda_stream)
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(replays):
        g.replay()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (replays * per_graph)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--names", required=True)
    ap.add_argument("--cfgs", default="0:0,1:1,2:1,3:1")
    ap.add_argument("--variant", default="rgbt")
    ap.add_argument("--batch", type=int, default=1)
    args = ap.parse_args()
    import bench
    from mmt_amd import synthetic
    from mmt_amd.runtime import MixFormerRGBTRuntime

    keys = bench.state_dict_keys(args.variant, **bench.GEO_B)
    sd = {k: torch.from_numpy(v) for k, v in synthetic.synth_state_dict(keys).items()}
    rt = MixFormerRGBTRuntime(sd, args.variant, dtype=torch.bfloat16)
    t, o, s = synthetic.synth_inputs(args.batch, 128, 320, seed=0)
    plan = rt.plan_for_inputs([x.cuda() for x in t], [x.cuda() for x in o], [x.cuda() for x in s])
    rt.run_plan(plan)
    torch.cuda.synchronize()
    for nm in args.names.split(","):
        e = next(e for e in plan if e[2] == nm)
        fn, fargs, _, keep = e
        ps = list(keep) if isinstance(keep, ctypes.Array) else [keep]  # mmt_gemm_multi: every problem
        row = {"name": nm, "problems": [{"M": p.M, "N": p.N, "K": p.K, "groups": p.groups, "conv": int(p.conv_h > 0)}
                                        for p in ps]}
        saved = [(p.impl, p.splitk) for p in ps]
        for cfg in args.cfgs.split(","):
            impl, sk = (int(v) for v in cfg.split(":"))
            for p in ps:
                p.impl, p.splitk = impl, sk
            row[cfg] = round(time_entry(fn, fargs), 2)
        for p, (i0, s0) in zip(ps, saved):
            p.impl, p.splitk = i0, s0
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
