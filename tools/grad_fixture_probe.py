#!/usr/bin/env python3
"""Conditioning of the config-4 module-gradient fixture (tests/test_gpu_train_ops.py::
test_module_forward_training_gpu_grads, B = 16, train-mode BatchNorm): for several corner-head output gains,
the relative-L2 distance of each parameter group's gradient from the fp32 CPU stand-in, for the PyTorch-bf16
ops (the bar's reference) and for the HIP ops (the product), plus the HIP path with one backward perturbed
(dW of every plain HIP Linear x 0.9: a negative control the check must flag)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402


def main():
    import mmt_amd.model as M
    import mmt_amd.train as T
    from mmt_amd.train import box_loss, synthetic_batch
    from test_train import TorchOps
    from test_gpu_train_ops import _TorchBf16Ops
    B = int(os.environ.get("B", "16"))
    for gain in [float(x) for x in os.environ.get("GAINS", "30,10,3,1").split(",")]:
        torch.manual_seed(0)
        net = M.build_mixformer_vit_rgbt(M.hot_path_cfg(), train=False)
        with torch.no_grad():
            for br in ("tl", "br"):
                getattr(net.box_head, "conv5_" + br).weight.mul_(gain)
            for m in net.modules():
                if hasattr(m, "sampling_offsets"):
                    m.sampling_offsets.bias.add_(1.0 / 3.0)
        net.train()
        net.drop_path_rate = 0.0
        for m in net.modules():
            if isinstance(m, torch.nn.Dropout):
                m.p = 0.0
        t, o, s, gt = synthetic_batch(B, "cpu", torch.Generator().manual_seed(7))

        def run(ops, dev):
            net.zero_grad(set_to_none=True)
            net.train_ops = ops
            args = [[x.to(dev) for x in z] for z in (t, o, s)]
            _, coord = net(*args, gt_bboxes=None)
            loss, _ = box_loss(coord, gt.to(dev))
            loss.backward()
            return loss.item(), {n: p.grad.float().cpu().clone() for n, p in net.named_parameters() if p.grad is not None}

        net.cpu()
        ref_loss, ref = run(TorchOps, "cpu")
        net.cuda()
        tb_loss, tb = run(_TorchBf16Ops, "cuda")
        hip_loss, hip = run(None, "cuda")
        orig = T._weight_grads2

        def bad_wg2(*a, **k):
            return [(dw * 0.9, db * 0.9) for dw, db in orig(*a, **k)]
        T._weight_grads2 = bad_wg2
        try:
            _, neg = run(None, "cuda")
        finally:
            T._weight_grads2 = orig
        row = {"gain": gain, "B": B, "loss": [ref_loss, tb_loss, hip_loss]}
        for grp in ("backbone_v", "backbone_i", "fusion_vi", "box_head"):
            names = [n for n in ref if n.startswith(grp + ".")]
            r = torch.cat([ref[n].flatten() for n in names])
            rel = lambda d: round((torch.cat([d[n].flatten() for n in names]) - r).norm().item() / r.norm().item(), 4)  # noqa: E731
            row[grp] = {"torch_bf16": rel(tb), "hip": rel(hip), "hip_dW_x0.9": rel(neg)}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
