#!/usr/bin/env python3
"""Stage-by-stage comparison of the training corner head on the HIP ops (head_forward_nhwc) against the same
head with every conv() block run as nn.Conv2d + module BN + ReLU on the same NHWC bf16 inputs: prints the
relative error of each block's output (the inputs of each stage are the HIP path's)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import mmt_amd.model as M  # noqa: E402
from mmt_amd.train import HipOps  # noqa: E402


def main():
    torch.manual_seed(3)
    net = M.build_mixformer_vit_rgbt(M.hot_path_cfg(), train=False)
    hd = net.box_head.cuda().eval()
    x = torch.randn(2, hd.conv1_tl[0].weight.shape[1], 20, 20, device="cuda")
    xh = x.permute(0, 2, 3, 1).bfloat16().contiguous()

    def ref_block(seq, t):
        y = F.conv2d(t.float().permute(0, 3, 1, 2), seq[0].weight, seq[0].bias, padding=1)
        return torch.relu(seq[1](y)).permute(0, 2, 3, 1)

    def hip_block(seq, t):
        y = HipOps.conv3x3(t.contiguous(), seq[0].weight, seq[0].bias)
        yc = F.conv2d(t.float().permute(0, 3, 1, 2), seq[0].weight, seq[0].bias, padding=1).permute(0, 2, 3, 1)
        e = ((y.float() - yc).norm() / yc.norm()).item()
        if y.shape[-1] % 8 == 0:
            out = HipOps.bn_relu(y, seq[1])
        else:
            out = torch.relu(seq[1](y.permute(0, 3, 1, 2).contiguous())).permute(0, 2, 3, 1)
        r = ref_block(seq, t)
        e2 = ((out.float() - r).norm() / r.norm().clamp_min(1e-12)).item()
        print("  conv %s -> %s on %s: conv err %.3e, block err %.3e" % (tuple(seq[0].weight.shape[:2]), tuple(y.shape),
                                                                      tuple(t.shape), e, e2), flush=True)
        return out.contiguous()

    with torch.no_grad():
        for br in ("tl",):
            g = lambda n: getattr(hd, n + "_" + br)  # noqa: E731
            up = lambda t, f: F.interpolate(t.permute(0, 3, 1, 2), scale_factor=f).permute(0, 2, 3, 1)  # noqa: E731
            x1 = hip_block(g("conv1"), xh)
            x2 = hip_block(g("conv2"), x1)
            a1 = hip_block(g("adjust1"), xh)
            x3 = hip_block(g("conv3"), (up(a1, 2) + up(x2, 2)).contiguous())
            a2 = hip_block(g("adjust2"), xh)
            x4 = hip_block(g("conv4"), (up(a2, 4) + up(x3, 2)).contiguous())
            a3 = g("adjust3")
            hip_block(a3[2], hip_block(a3[1], hip_block(a3[0], x2)))
            a4 = g("adjust4")
            hip_block(a4[1], hip_block(a4[0], x3))
            print("x4", tuple(x4.shape))


if __name__ == "__main__" and not os.environ.get("HEAD_DIAG_WHOLE") and not os.environ.get("HEAD_DIAG_TRACE"):
    main()


def whole():
    """The whole head: HIP ops under autocast, a GPU stand-in (F.conv2d convs, module BN) under autocast, aten fp32."""
    import mmt_amd.train as T
    torch.manual_seed(3)
    net = M.build_mixformer_vit_rgbt(M.hot_path_cfg(), train=False)
    hd = net.box_head.cuda().eval()
    with torch.no_grad():
        for br in ("tl", "br"):
            getattr(hd, "conv5_" + br).weight.mul_(30.0)
    x = torch.randn(2, hd.conv1_tl[0].weight.shape[1], 20, 20, device="cuda").bfloat16().float()

    class StandIn:
        @staticmethod
        def conv3x3(t, w, b):
            return F.conv2d(t.float().permute(0, 3, 1, 2), w, b, padding=1).permute(0, 2, 3, 1).to(t.dtype)

    maps = []
    orig = T._soft_argmax

    def rec(sm, stride):
        maps.append(sm.float())
        return orig(sm, stride)

    T._soft_argmax = rec
    with torch.no_grad():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            a = T.head_forward(hd, x, HipOps)
            b = T.head_forward(hd, x, StandIn)
        c = T.head_forward(hd, x, None)
    T._soft_argmax = orig
    print("hip", a.float().tolist())
    print("standin", b.float().tolist())
    print("aten fp32", c.float().tolist())
    for i, m in enumerate(maps):
        print("map", i, tuple(m.shape), "mean %.4f std %.4f max %.4f" % (m.mean().item(), m.std().item(), m.max().item()))


if __name__ == "__main__" and os.environ.get("HEAD_DIAG_WHOLE"):
    whole()


def trace():
    """Op-by-op outputs of head_forward_nhwc under autocast: HIP convs / bn_relu against the stand-in."""
    import mmt_amd.train as T
    torch.manual_seed(3)
    net = M.build_mixformer_vit_rgbt(M.hot_path_cfg(), train=False)
    hd = net.box_head.cuda().eval()
    x = torch.randn(2, hd.conv1_tl[0].weight.shape[1], 20, 20, device="cuda").bfloat16().float()
    rec = {"hip": [], "std": []}

    class Hip:
        @staticmethod
        def conv3x3(t, w, b):
            y = HipOps.conv3x3(t, w, b)
            rec["hip"].append(("conv", y.float().clone()))
            return y

        @staticmethod
        def bn_relu(t, bn):
            y = HipOps.bn_relu(t, bn)
            rec["hip"].append(("bn", y.float().clone()))
            return y

    class Std:
        @staticmethod
        def conv3x3(t, w, b):
            y = F.conv2d(t.float().permute(0, 3, 1, 2), w, b, padding=1).permute(0, 2, 3, 1).to(t.dtype)
            rec["std"].append(("conv", y.float().clone()))
            return y

        @staticmethod
        def bn_relu(t, bn):
            y = torch.relu(bn(t.permute(0, 3, 1, 2).contiguous())).permute(0, 2, 3, 1).contiguous()
            rec["std"].append(("bn", y.float().clone()))
            return y

    with torch.no_grad():
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=os.environ.get("HEAD_DIAG_AUTOCAST", "1") == "1"):
            T.head_forward(hd, x, Hip)
            T.head_forward(hd, x, Std)
    for i, ((k, a), (_, b)) in enumerate(zip(rec["hip"], rec["std"])):
        e = ((a - b).norm() / b.norm().clamp_min(1e-12)).item()
        print(i, k, tuple(a.shape), "err %.3e finite %s" % (e, bool(torch.isfinite(a).all())), flush=True)


if __name__ == "__main__" and os.environ.get("HEAD_DIAG_TRACE"):
    trace()
