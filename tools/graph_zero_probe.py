#!/usr/bin/env python3
"""Are zero-initialised tensors re-zeroed on hipGraph replay?  Each case allocates a zero-filled tensor inside
the captured region (torch.zeros, zeros_like, new_zeros, F.pad, fill_(0), the slicing backward), the tensor's
memory is overwritten with 7.0 after capture, and one replay must leave the zero part at 0 again."""
import torch
import torch.nn.functional as F

N = 1 << 16
dev = "cuda"


def case(name, fn):
    x = torch.randn(N, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn(x)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out, zero_part = fn(x)
    zero_part.fill_(7.0)  # eager write into the graph's tensor
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    ok = bool((zero_part == 0).all())
    print("%-22s re-zeroed on replay: %s" % (name, ok), flush=True)


def zeros(x):
    z = torch.zeros(N + 64, device=dev)
    z[:N] += x
    return z, z[N:]


def zeros_like(x):
    z = torch.zeros_like(torch.cat([x, x[:64]]))
    z[:N] += x
    return z, z[N:]


def new_zeros(x):
    z = x.new_zeros(N + 64)
    z[:N] += x
    return z, z[N:]


def pad(x):
    z = F.pad(x.view(1, N), (0, 64))
    return z, z[0, N:]


def fill0(x):
    z = torch.empty(N + 64, device=dev).fill_(0.0)
    z[:N] += x
    return z, z[N:]


def slice_backward(x):
    w = torch.randn(N + 64, device=dev, requires_grad=True)
    y = w[:N] * x
    gw, = torch.autograd.grad(y.sum(), w)
    return gw, gw[N:]


def bf16_zeros(x):
    z = torch.zeros(N + 64, device=dev, dtype=torch.bfloat16)
    z[:N] += x.bfloat16()
    zf = z.float()
    return z, z[N:]


for name, fn in (("torch.zeros", zeros), ("zeros_like", zeros_like), ("new_zeros", new_zeros), ("F.pad", pad),
                 ("fill_(0)", fill0), ("slice backward", slice_backward), ("torch.zeros bf16", bf16_zeros)):
    case(name, fn)
