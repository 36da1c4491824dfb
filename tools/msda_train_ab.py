#!/usr/bin/env python3
"""Device time of the training step's bimodal MSDA middle, forward + backward, at config 4 (16 pairs, 20 x 20
maps): the fused HIP op (HipOps.msda_bimodal) vs the previous composition (softmax / location glue + the fp32
drop-in MSDA kernels + casts).  HIP events around 20 iterations of each."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "multi-modal-tracking_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def main(B=16, hw=20):
    from mmt_amd.functional import MSDeformAttnFunction
    from mmt_amd.train import HipOps, _ref_points
    nq = hw * hw
    value = torch.randn(B, 2 * nq, 512, device="cuda").bfloat16().requires_grad_(True)
    off = (torch.randn(B, nq, 128, device="cuda") * 2).bfloat16().requires_grad_(True)
    awl = torch.randn(B, nq, 64, device="cuda").bfloat16().requires_grad_(True)
    gout = torch.randn(B, nq, 512, device="cuda").bfloat16()
    ref4 = _ref_points(hw, hw, B, 2, "cuda")
    ref_q = ref4[0, :nq, 0, :].contiguous()
    wh = torch.tensor([hw, hw], dtype=torch.float32, device="cuda")
    shapes = torch.tensor([[hw, hw]] * 2, dtype=torch.long, device="cuda")
    starts = torch.arange(2, dtype=torch.long, device="cuda") * nq

    def old():
        a = F.softmax(awl.view(B, nq, 8, 8).float(), -1).view(B, nq, 8, 2, 4)
        loc = ref4[:, :nq, None, :, None, :] + off.view(B, nq, 8, 2, 4, 2).float() / wh
        y = MSDeformAttnFunction.apply(value.view(B, 2 * nq, 8, 64).float().contiguous(), shapes, starts,
                                       loc.contiguous(), a.contiguous(), 64).to(torch.bfloat16)
        y.backward(gout)

    def new():
        HipOps.msda_bimodal(value, off, awl, ref_q, hw).backward(gout)

    for name, fn in (("previous composition", old), ("fused HIP op", new)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print("%-22s fwd+bwd %.1f us (including autograd's grad accumulation into .grad)" % (name, e0.elapsed_time(e1) * 1e3 / 20))
        value.grad = off.grad = awl.grad = None


if __name__ == "__main__":
    main()
