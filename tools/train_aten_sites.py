#!/usr/bin/env python3
"""Where the training step's PyTorch (aten) device work comes from: one eager step of the config-4 training
step (bench.py train_bench's model, 16 pairs, HIP ops) under torch.profiler with Python stacks; prints the
aten ops with device time grouped by their innermost call site in mmt_amd/ (file:line), so that the glue
the verdict counts (casts, adds, cats, upsampling, the hipBLASLt 48 -> 1 conv) can be traced to its line.

usage: python tools/train_aten_sites.py [--batch 16] [--top 40]
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--top", type=int, default=40)
    args = ap.parse_args()
    from torch.profiler import ProfilerActivity, profile
    from mmt_amd.model import build_mixformer_vit_rgbt, hot_path_cfg
    from mmt_amd.train import HipOps, TrainStep, synthetic_batch
    torch.manual_seed(0)
    net = build_mixformer_vit_rgbt(hot_path_cfg(), train=False).cuda().train()
    step = TrainStep(net, HipOps)
    batch = synthetic_batch(args.batch, "cuda", torch.Generator().manual_seed(100))
    for _ in range(2):
        step(*batch)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        step(*batch)
        torch.cuda.synchronize()
    # aten ops with device time, grouped by their 6 innermost Python frames (forward ops; the backward's run on
    # autograd's thread without a Python stack and show as the op that created them is listed by name only)
    ka = prof.key_averages(group_by_stack_n=6)
    rows = []
    for e in ka:
        if not e.key.startswith("aten::"):
            continue
        sdev = getattr(e, "self_device_time_total", None)
        if sdev is None:
            sdev = getattr(e, "self_cuda_time_total", 0.0)
        if sdev <= 0:
            continue
        frames = [f.split("multi-modal-tracking_amd/")[-1] for f in (e.stack or []) if "mmt_amd" in f or "tools/" in f]
        rows.append((sdev, e.count, e.key, " <- ".join(frames[:3]) or "(no python stack: autograd backward)"))
    rows.sort(key=lambda r: -r[0])
    print("aten self device time, one step: %.1f us" % sum(r[0] for r in rows))
    for sdev, n, key, where in rows[:args.top]:
        print("%9.1f us %4d  %-32s %s" % (sdev, n, key, where[:160]))


if __name__ == "__main__":
    main()
