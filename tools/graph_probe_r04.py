#!/usr/bin/env python3
"""hipGraph capture / replay of the training step's pieces against eager on the same inputs (round 4: the HIP
head convs, HIP batch norm, the HIP norms / residual GEMMs, the whole head, the whole fusion, the loss).  Uses
tools/graph_capture_probe.check: three replays, each gradient's max error relative to the eager one."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))
sys.argv = sys.argv[:1]
import mmt_amd.model as M  # noqa: E402
import mmt_amd.train as T  # noqa: E402
from mmt_amd.train import HipOps  # noqa: E402

dev = "cuda"
torch.manual_seed(0)
exec(open(os.path.join(ROOT, "tools", "graph_capture_probe.py")).read().split("\nB = 16")[0].split("torch.manual_seed(0)\ndev = \"cuda\"\n")[1])

B = 4
x = torch.randn(B, 20, 20, 768, device=dev).bfloat16().requires_grad_(True)
w = torch.nn.Parameter(torch.randn(384, 768, 3, 3, device=dev) / 80)
b = torch.nn.Parameter(torch.randn(384, device=dev))
check("HipOps.conv3x3 768->384", [w, b, x], [x], lambda t: HipOps.conv3x3(t, w, b))
x1 = torch.randn(B, 40, 40, 48, device=dev).bfloat16().requires_grad_(True)
w1 = torch.nn.Parameter(torch.randn(1, 48, 3, 3, device=dev) / 20)
b1 = torch.nn.Parameter(torch.randn(1, device=dev))
check("HipOps.conv3x3 48->1", [w1, b1, x1], [x1], lambda t: HipOps.conv3x3(t, w1, b1))
bn = torch.nn.BatchNorm2d(96).to(dev)
xb = torch.randn(B, 40, 40, 96, device=dev).bfloat16().requires_grad_(True)
check("HipOps.bn_relu train", list(bn.parameters()) + [xb], [xb], lambda t: HipOps.bn_relu(t, bn))
bn1 = torch.nn.BatchNorm2d(1).to(dev)
xb1 = torch.randn(B, 40, 40, 1, device=dev).bfloat16().requires_grad_(True)
check("HipOps.bn_relu C=1 train", list(bn1.parameters()) + [xb1], [xb1], lambda t: HipOps.bn_relu(t, bn1))

net = M.build_mixformer_vit_rgbt(M.hot_path_cfg(), train=False).to(dev).train()
for m in net.modules():  # no dropout: replays must reproduce the eager step exactly
    if isinstance(m, torch.nn.Dropout):
        m.p = 0.0
hd = net.box_head
xf = torch.randn(B, 768, 20, 20, device=dev, requires_grad=True)


def head_fn(t):
    with torch.autocast("cuda", dtype=torch.bfloat16):
        return T.head_forward(hd, t, HipOps)


check("head_forward HIP (train BN)", [p for p in hd.parameters()] + [xf], [xf], head_fn)
sv = torch.randn(B, 768, 20, 20, device=dev, requires_grad=True)
si = torch.randn(B, 768, 20, 20, device=dev, requires_grad=True)


def fusion_fn(a, c):
    with torch.autocast("cuda", dtype=torch.bfloat16):
        return T.fusion_forward(net.fusion_vi, a, c, HipOps)


check("fusion_forward HIP", [p for p in net.fusion_vi.parameters()] + [sv, si], [sv, si], fusion_fn)
t, o, s, gt = T.synthetic_batch(B, dev, torch.Generator().manual_seed(1))


def bb_fn(a, c, d):
    return T.backbone_forward(net.backbone_v, a, c, d, HipOps, 0.0)


check("backbone_forward HIP", [p for p in net.backbone_v.blocks[3].parameters()], [t[0], o[0], s[0]], bb_fn)
pred = torch.rand(B, 1, 4, device=dev) * 0.3 + 0.3
pred.requires_grad_(True)
check("box_loss", [pred], [pred], lambda q: T.box_loss(q, gt)[0].view(1))


def fwd(a, c, d, e, f, g):
    with torch.autocast("cuda", dtype=torch.bfloat16):
        return T.forward_boxes(net, [a, b_], [c, d_], [e, f_], HipOps) if False else T.forward_boxes(net, [a, c], [d, e], [f, g], HipOps)


check("forward_boxes HIP", [p for p in net.parameters() if p.requires_grad][::7], [t[0], t[1], o[0], o[1], s[0], s[1]], fwd)
