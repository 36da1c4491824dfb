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
    ap.add_argument("--top", type=int, default=60)
    args = ap.parse_args()
    from torch.profiler import ProfilerActivity, profile
    from mmt_amd.model import build_mixformer_vit_rgbt, hot_path_cfg
    from mmt_amd.train import HipOps, TrainStep, synthetic_batch
    # forward attribution: every function of mmt_amd.train (and HipOps' static methods) runs inside a
    # record_function range of its own name, so an aten op's innermost enclosing range names its call site
    import functools
    import inspect
    import mmt_amd.train as T
    from torch.profiler import record_function

    def wrap(name, fn):
        @functools.wraps(fn)
        def w(*a, **k):
            with record_function("site::" + name):
                return fn(*a, **k)
        return w
    for name, fn in list(vars(T).items()):
        if inspect.isfunction(fn) and fn.__module__ == T.__name__ and not name.startswith("__"):
            setattr(T, name, wrap(name, fn))
    for name, fn in list(vars(T.HipOps).items()):
        if isinstance(fn, staticmethod):
            setattr(T.HipOps, name, staticmethod(wrap("HipOps." + name, fn.__func__)))
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
    # every aten op with device time: attributed to its autograd backward node (the enclosing
    # "autograd::engine::evaluate_function: <Node>" event) or, in the forward, to its innermost mmt_amd frames
    def site_of(e):  # the innermost two site:: ranges enclosing a forward event
        par, names = e.cpu_parent, []
        while par is not None and len(names) < 2:
            if par.name.startswith("site::"):
                names.append(par.name[6:])
            par = par.cpu_parent
        return " <- ".join(names) if names else "?"
    # backward nodes carry the sequence number of the forward op that created them: name the node's forward site
    fwd_site = {}
    for e in prof.events():
        if e.name.startswith("aten::") and getattr(e, "sequence_nr", -1) >= 0 and e.sequence_nr not in fwd_site:
            fwd_site[e.sequence_nr] = "%s@%s" % (e.name[6:], site_of(e))
    agg = collections.defaultdict(lambda: [0.0, 0, set()])
    top_total = 0.0
    for e in prof.events():
        if not e.name.startswith("aten::"):
            continue
        sdev = getattr(e, "self_device_time_total", None)
        if sdev is None:
            sdev = getattr(e, "self_cuda_time_total", 0.0)
        if sdev <= 0:
            continue
        where, par = None, e.cpu_parent
        while par is not None:
            if par.name.startswith("autograd::engine::evaluate_function"):
                where = "bwd " + par.name.split(": ", 1)[-1]
                seq = getattr(par, "sequence_nr", -1)
                if seq in fwd_site:
                    where += " <- " + fwd_site[seq]
                break
            par = par.cpu_parent
        if where is None:
            where = "fwd " + site_of(e)
        a = agg[where]
        a[0] += sdev
        a[1] += 1
        a[2].add(e.name)
        top_total += sdev
    print("aten self device time, one step: %.1f us" % top_total)
    for where, (us, n, names) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:args.top]:
        print("%9.1f us %4d  %-110s %s" % (us, n, where[:110], ",".join(sorted(names))[:100]))


if __name__ == "__main__":
    main()
