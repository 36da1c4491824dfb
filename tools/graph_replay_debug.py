"""Debug: forward + backward of the training step captured once, replayed twice on the same weights
(gradients zeroed in between): do the replays agree, and which gradients differ / are non-finite?"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))
from mmt_amd.model import build_mixformer_vit_rgbt, hot_path_cfg  # noqa: E402
from mmt_amd.train import HipOps, TrainStep, synthetic_batch  # noqa: E402

torch.manual_seed(0)
if os.environ.get("NO_MIOPEN"):
    torch.backends.cudnn.enabled = False
net = build_mixformer_vit_rgbt(hot_path_cfg(), train=False).cuda().eval()
batch = synthetic_batch(2, "cuda", torch.Generator().manual_seed(5))
step = TrainStep(net, HipOps)
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    for _ in range(2):
        step(*batch)
torch.cuda.current_stream().wait_stream(side)
named = [(n, p) for n, p in net.named_parameters() if p.grad is not None]
eager_stats = None
with torch.cuda.stream(side):
    for _, p in named:
        p.grad.zero_()
    eager_stats = step.backward(*batch)
torch.cuda.synchronize()
eager = {n: p.grad.clone() for n, p in named}
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=side):
    stats = step.backward(*batch)
reps = []
for r in range(3):
    for _, p in named:
        p.grad.zero_()
    g.replay()
    torch.cuda.synchronize()
    reps.append({n: p.grad.clone() for n, p in named})
    print("replay %d loss %.5f (eager %.5f)" % (r, stats["loss"].item(), eager_stats["loss"].item()), flush=True)
for r in range(3):
    bad = []
    for n, _ in named:
        a, e = reps[r][n], eager[n]
        rel = ((a - e).norm() / (e.norm() + 1e-20)).item()
        if not torch.isfinite(a).all() or rel > 2e-2:
            bad.append((n, round(rel, 4), int((~torch.isfinite(a)).sum())))
    print("replay %d: %d params off" % (r, len(bad)), flush=True)
    for n, rel, nf in bad:
        if "backbone" not in n:
            print("   ", n, rel, nf, flush=True)
