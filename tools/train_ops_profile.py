#!/usr/bin/env python3
"""Which aten ops the config-4 training step still launches: torch.profiler over one step (after warm-up)
of bench.train_bench's workload, aten ops grouped by name with call counts and device time, top N.

    python tools/train_ops_profile.py [--top 30]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--shapes", default="", help="comma-separated aten ops to list by input shapes + Python stack")
    args = ap.parse_args()
    from mmt_amd.model import build_mixformer_vit_rgbt, hot_path_cfg
    from mmt_amd.train import HipOps, TrainStep, synthetic_batch
    torch.manual_seed(0)
    net = build_mixformer_vit_rgbt(hot_path_cfg(), train=False).cuda().train()
    step = TrainStep(net, HipOps, ddp=False)
    g = torch.Generator().manual_seed(100)
    batch = synthetic_batch(args.batch, "cuda", g)
    for _ in range(3):
        step(*batch)
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, record_shapes=bool(args.shapes), with_stack=bool(args.shapes)) as prof:
        step(*batch)
        torch.cuda.synchronize()
    ka = prof.key_averages()
    dev = lambda e: getattr(e, "self_device_time_total", getattr(e, "self_cuda_time_total", 0.0))  # noqa: E731
    rows = [e for e in ka if e.key.startswith("aten::")]
    rows.sort(key=lambda e: -e.count)
    print("%-44s %7s %12s %12s" % ("aten op", "calls", "self cpu us", "device us"))
    for e in rows[:args.top]:
        print("%-44s %7d %12.0f %12.0f" % (e.key[:44], e.count, e.self_cpu_time_total, dev(e)))
    if args.shapes:
        want = set("aten::" + n for n in args.shapes.split(","))
        by = prof.key_averages(group_by_input_shape=True, group_by_stack_n=4)
        sel = [e for e in by if e.key in want]
        sel.sort(key=lambda e: -dev(e))
        print("\n%-16s %6s %10s  %s" % ("op", "calls", "device us", "input shapes / stack"))
        for e in sel[:60]:
            stack = " <- ".join(str(f).split("(")[0].split("/")[-1] + ":" + str(f).split("(")[-1].rstrip(")")
                                for f in (e.stack or [])[:4])
            print("%-16s %6d %10.0f  %s | %s" % (e.key[6:22], e.count, dev(e), str(e.input_shapes)[:90], stack[:200]))
    kern = [e for e in ka if not e.key.startswith("aten::") and dev(e) > 0 and e.self_cpu_time_total == 0]
    kern.sort(key=lambda e: -dev(e))
    print("\n%-90s %7s %12s" % ("device kernel", "calls", "device us"))
    for e in kern[:args.top]:
        print("%-90s %7d %12.0f" % (e.key[:90], e.count, dev(e)))


if __name__ == "__main__":
    main()
