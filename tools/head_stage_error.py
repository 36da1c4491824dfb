#!/usr/bin/env python3
"""Per-stage error table of the training corner head: the HIP path (head_forward_nhwc:
HIP 3x3 convs + HIP BatchNorm+ReLU on NHWC bf16 maps, under autocast) and aten's bf16 autocast path, each
against aten fp32, stage by stage (head.py:147-212: conv1, conv2, adjust1, conv3, adjust2, conv4, conv5,
adjust3, adjust4, the score map and the normalised corners), for both branches, BatchNorm in train and eval
mode, on the fixture of tests/test_gpu_train_ops.py::test_head_forward_nhwc_matches_aten (B = 2, conv5 x30).
Each stage is fed the SAME fp32 input in all three paths (the fp32 path's previous stage), so a row is that
stage's own error, not the accumulated one; the `chain` columns run each path end to end.

usage: python tools/head_stage_error.py [--variant pyramid_fp32]
"""
import argparse
import copy
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.parse_args()
    import mmt_amd.model as M
    from mmt_amd.train import HipOps, _hip_bn_ok, _soft_argmax, head_forward
    nchw = lambda t: t.permute(0, 3, 1, 2)  # noqa: E731
    nhwc = lambda t: t.permute(0, 2, 3, 1)  # noqa: E731

    for bn_train in (False, True):
        torch.manual_seed(3)
        net = M.build_mixformer_vit_rgbt(M.hot_path_cfg(), train=False)
        hd = net.box_head.cuda()
        with torch.no_grad():
            for br in ("tl", "br"):
                getattr(hd, "conv5_" + br).weight.mul_(30.0)
        hd.train(bn_train)
        x = torch.randn(2, hd.conv1_tl[0].weight.shape[1], 20, 20, device="cuda").bfloat16().float()
        heads = {"hip": hd, "aten_bf16": copy.deepcopy(hd), "fp32": copy.deepcopy(hd)}

        def stage_hip(h, name, seq, t):  # one conv() block of head_forward_nhwc on an NCHW fp32 input
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = HipOps.conv3x3(nhwc(t).to(torch.bfloat16).contiguous(), seq[0].weight, seq[0].bias)
                bn = seq[1]
                assert _hip_bn_ok(bn)
                return nchw(HipOps.bn_relu(y, bn)).float()

        def stage_aten(h, name, seq, t, bf16):
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
                return seq(t).float()

        rows = []
        for br in ("tl", "br"):
            g = {k: (lambda n, h=h: getattr(h, n + "_" + br)) for k, h in heads.items()}
            ref = {}

            def run(name, mod_name, t, idx=None):
                outs = {}
                for k in heads:
                    seq = g[k](mod_name) if idx is None else g[k](mod_name)[idx]
                    if k == "hip":
                        outs[k] = stage_hip(heads[k], name, seq, t)
                    else:
                        outs[k] = stage_aten(heads[k], name, seq, t, k == "aten_bf16")
                r = outs["fp32"]
                sc = r.abs().max().item() + 1e-12
                rows.append({"bn_train": bn_train, "branch": br, "stage": name,
                             "hip_rel": float("%.3g" % ((outs["hip"] - r).abs().max().item() / sc)),
                             "aten_bf16_rel": float("%.3g" % ((outs["aten_bf16"] - r).abs().max().item() / sc))})
                return r

            up = lambda t, f: F.interpolate(t, scale_factor=f)  # noqa: E731
            x1 = run("conv1", "conv1", x)
            x2 = run("conv2", "conv2", x1)
            a1 = run("adjust1", "adjust1", x)
            x3 = run("conv3", "conv3", up(a1, 2) + up(x2, 2))
            a2 = run("adjust2", "adjust2", x)
            x4 = run("conv4", "conv4", up(a2, 4) + up(x3, 2))
            a30 = run("adjust3[0]", "adjust3", x2, 0)
            a31 = run("adjust3[1]", "adjust3", a30, 1)
            a40 = run("adjust4[0]", "adjust4", x3, 0)
            # the 1-channel stages (conv5 48 -> 1 as F.linear in the HIP path, adjust3[2] / adjust4[1] convs)
            # and the score-map sum, each from the fp32 inputs
            outs = {}
            for k, h in heads.items():
                gg = g[k]
                with torch.autocast("cuda", dtype=torch.bfloat16, enabled=k != "fp32"):
                    if k == "hip":
                        c5 = nchw(F.linear(nhwc(x4).to(torch.bfloat16), gg("conv5").weight.view(1, -1), gg("conv5").bias))
                        s3 = stage_hip(h, "adjust3[2]", gg("adjust3")[2], a31)
                        s4 = stage_hip(h, "adjust4[1]", gg("adjust4")[1], a40)
                    else:
                        c5 = gg("conv5")(x4)
                        s3 = gg("adjust3")[2](a31)
                        s4 = gg("adjust4")[1](a40)
                    sm = c5.float() + up(s3.float(), 4) + up(s4.float(), 2)
                outs[k] = {"conv5": c5.float(), "adjust3[2]": s3.float(), "adjust4[1]": s4.float(), "score_map": sm,
                           "corner": torch.stack(_soft_argmax(sm, hd.stride), 1) / hd.img_sz}
            for name in ("conv5", "adjust3[2]", "adjust4[1]", "score_map", "corner"):
                r = outs["fp32"][name]
                sc = 1.0 if name == "corner" else r.abs().max().item() + 1e-12  # corners: absolute (image units)
                rows.append({"bn_train": bn_train, "branch": br, "stage": name + (" (abs)" if name == "corner" else ""),
                             "hip_rel": float("%.3g" % ((outs["hip"][name] - r).abs().max().item() / sc)),
                             "aten_bf16_rel": float("%.3g" % ((outs["aten_bf16"][name] - r).abs().max().item() / sc))})
        # whole chains (as the test): HIP head_forward_nhwc (conv5 in fp32, and in bf16 as before round 5),
        # aten autocast, aten fp32
        import mmt_amd.train as T
        chain = {}
        for k, h in list(heads.items()) + [("hip_c5bf16", hd)]:
            h2 = copy.deepcopy(h)
            T.HEAD_SCORE_FP32 = k != "hip_c5bf16"
            with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16, enabled=k != "fp32"):
                chain[k] = head_forward(h2, x, HipOps if k.startswith("hip") else None).float()
        T.HEAD_SCORE_FP32 = True
        rows.append({"bn_train": bn_train, "branch": "both", "stage": "chain corners (abs)",
                     "hip_rel": float("%.3g" % (chain["hip"] - chain["fp32"]).abs().max().item()),
                     "hip_c5bf16_rel": float("%.3g" % (chain["hip_c5bf16"] - chain["fp32"]).abs().max().item()),
                     "aten_bf16_rel": float("%.3g" % (chain["aten_bf16"] - chain["fp32"]).abs().max().item())})
        for r in rows:
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
