"""Which op's backward goes wrong under hipGraph capture?  For each candidate (forward + backward of
one op at training shapes, bf16 autocast where the training step uses it), the gradients of a
captured-and-replayed graph against the eager ones on the same inputs."""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))
from mmt_amd.train import HipOps  # noqa: E402

torch.manual_seed(0)
dev = "cuda"


def check(name, params, inputs, fn):
    def run():
        for p in params:
            p.grad = None
        out = fn(*inputs)
        out.float().square().mean().backward()
        return out
    run()
    ref = [p.grad.clone() for p in params]
    refo = run().detach().clone()
    # capture (grads accumulate in place into existing .grad during capture)
    for p in params:
        p.grad = torch.zeros_like(p)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            for p in params:
                p.grad.zero_()
            out = fn(*inputs)
            out.float().square().mean().backward()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    for p in params:
        p.grad.zero_()
    with torch.cuda.graph(g):
        out = fn(*inputs)
        out.float().square().mean().backward()
    errs = []
    for rep in range(3):
        for p in params:
            p.grad.zero_()
        g.replay()
        torch.cuda.synchronize()
        e = max(((p.grad - r).abs().max() / (r.abs().max() + 1e-12)).item() for p, r in zip(params, ref))
        errs.append(e)
    eo = ((out.float() - refo.float()).abs().max() / (refo.float().abs().max() + 1e-12)).item()
    print("%-28s out %.2e  grads %s" % (name, eo, " ".join("%.2e" % x for x in errs)), flush=True)


B = 16
x = torch.randn(B, 768, 20, 20, device=dev, requires_grad=True)
conv = torch.nn.Conv2d(768, 384, 3, padding=1).to(dev)
bn = torch.nn.BatchNorm2d(384).to(dev).eval()


def conv_fn(x):
    with torch.autocast("cuda", dtype=torch.bfloat16):
        return F.relu(bn(conv(x)))


check("conv3x3 bf16 autocast", list(conv.parameters()) + [x], [x], conv_fn)
lin = torch.nn.Linear(1024, 512).to(dev)
xl = torch.randn(B, 800, 1024, device=dev, requires_grad=True)


def lin_fn(x):
    with torch.autocast("cuda", dtype=torch.bfloat16):
        return lin(x)


check("nn.Linear bf16 autocast", list(lin.parameters()) + [xl], [xl], lin_fn)
gn = torch.nn.GroupNorm(32, 512).to(dev)
xg = torch.randn(B, 512, 20, 20, device=dev, requires_grad=True)
check("GroupNorm", list(gn.parameters()) + [xg], [xg], lambda x: gn(x))
w = torch.nn.Parameter(torch.randn(3072, 768, device=dev) / 28)
b = torch.nn.Parameter(torch.randn(3072, device=dev))
xh = torch.randn(B * 528, 768, device=dev).bfloat16().requires_grad_(True)
check("HipLinear", [w, b, xh], [xh], lambda x: HipOps.linear(x, w, b))
xh2 = torch.randn(B * 528, 3072, device=dev).bfloat16().requires_grad_(True)
w2 = torch.nn.Parameter(torch.randn(768, 3072, device=dev) / 55)
b2 = torch.nn.Parameter(torch.randn(768, device=dev))
check("HipLinear out_f32", [w2, b2, xh2], [xh2], lambda x: HipOps.linear(x, w2, b2, out_f32=True))
qkv = (torch.randn(B, 528, 2304, device=dev) * 0.5).bfloat16().requires_grad_(True)
check("HipOps.mam_attention", [qkv], [qkv], lambda q: HipOps.mam_attention(q, 128, 12))
ln = torch.nn.LayerNorm(768, eps=1e-6).to(dev)
xn = torch.randn(B, 528, 768, device=dev, requires_grad=True)
check("LayerNorm fp32 -> bf16", list(ln.parameters()) + [xn], [xn], lambda x: ln(x).bfloat16())
val = torch.randn(B, 800, 8, 64, device=dev, requires_grad=True)
loc = torch.rand(B, 800, 8, 2, 4, 2, device=dev, requires_grad=True)
aw = torch.softmax(torch.randn(B, 800, 8, 8, device=dev), -1).view(B, 800, 8, 2, 4).requires_grad_(True)
check("HipOps.ms_deform_attn", [val, loc, aw], [val, loc, aw], lambda v, l, a: HipOps.ms_deform_attn(v, 20, l, a))
