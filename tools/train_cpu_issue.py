"""Is the training step launch-bound?  Times the host's issue of one step (no synchronisation
inside) against the step's wall time with a synchronisation, at the bench shapes (16 pairs)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))
from mmt_amd.model import build_mixformer_vit_rgbt, hot_path_cfg  # noqa: E402
from mmt_amd.train import HipOps, TrainStep, synthetic_batch  # noqa: E402

torch.manual_seed(0)
net = build_mixformer_vit_rgbt(hot_path_cfg(), train=False).cuda().train()
step = TrainStep(net, HipOps)
batch = synthetic_batch(16, "cuda", torch.Generator().manual_seed(1))
for _ in range(3):
    step(*batch)
torch.cuda.synchronize()
for rep in range(3):
    t0 = time.perf_counter()
    step(*batch)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("issue %.2f ms, wall %.2f ms" % ((t1 - t0) * 1e3, (t2 - t0) * 1e3), flush=True)
# issue of forward / backward / optimizer separately
for name, fn in (("backward(fwd+bwd)", lambda: step.backward(*batch)), ("apply", step.apply)):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("%s: issue %.2f ms, wall %.2f ms" % (name, (t1 - t0) * 1e3, (t2 - t0) * 1e3), flush=True)
