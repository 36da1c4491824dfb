#!/usr/bin/env python3
"""Interleaved A/B of training-step variants in one process (methodology rule 24): the config-4 step
(bench.train_bench, two-stream MixViT-B RGB-T, --batch pairs) with the product HipOps against
variants that swap one op back to aten.  One JSON line per (round, variant).

    python tools/train_ab.py --rounds 3 --steps 8 --warmup 3
"""
import argparse
import contextlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))

import bench  # noqa: E402
import torch  # noqa: E402
from mmt_amd.train import HipOps  # noqa: E402


class AtenLayerNormOps(HipOps):
    """HipOps with the backbone LayerNorms on aten (F.layer_norm + bf16 cast, autograd backward)."""
    layer_norm = None


class AtenGroupNormOps(HipOps):
    """HipOps with the fusion's adjust_* as NCHW Conv2d (MIOpen) + nn.GroupNorm (aten), as before."""
    group_norm = None


class UnfusedResidualOps(HipOps):
    """HipOps with the blocks' residual branches as GEMM + addcmul (DropPath) + autograd's adds."""
    linear_residual = None
    mlp_residual = None
    linear2 = None  # (the lockstep pair needs the fused residual Functions)


class ComposedEncoderOps(HipOps):
    """HipOps with the deformable encoder layers as before round 6's fusion: HIP Linears / LayerNorms, aten glue
    (adds, cats, casts, softmax, dropout) and the drop-in fp32 MSDA kernels."""
    encoder_layer = None


class SplitMlpOps(HipOps):
    """HipOps with each MLP as fc1 / aten GELU / fc2 (three autograd nodes) instead of _HipMlp."""
    mlp = None


@contextlib.contextmanager
def accumulated_grads():
    """The previous gradient handling: persistent .grad buffers zeroed by the AdamW update, autograd
    adding each step's (strided [N][K+8] view) dW into them."""
    from mmt_amd import optim, train
    saved = train._weight_grads, optim.HipAdamW.__init__, optim.HipAdamW.zero_grad

    def weight_grads(dy, x, M, N, K):
        Mp = (M + 7) // 8 * 8
        dwb = train._gemm(train._transpose(dy, M, N, Mp), train._transpose(x, M, K, Mp, ones_row=True), N, K + 8,
                          Mp, out_f32=True)
        return dwb[:, :K], dwb[:, K]

    def init(self, *a, **kw):
        kw["set_to_none"] = False
        saved[1](self, *a, **kw)

    train._weight_grads = weight_grads
    optim.HipAdamW.__init__ = init
    optim.HipAdamW.zero_grad = lambda self, set_to_none=False: saved[2](self, False)
    try:
        yield
    finally:
        train._weight_grads, optim.HipAdamW.__init__, optim.HipAdamW.zero_grad = saved


@contextlib.contextmanager
def transposed_copies():
    """The Linear backward through transposed operand copies (mmt_transpose_bf16) instead of MN-major reads."""
    from mmt_amd import train
    train.MN_MAJOR = False
    try:
        yield
    finally:
        train.MN_MAJOR = True


@contextlib.contextmanager
def aten_scale_cast():
    """The residual branches' DropPath-scaled gradient cast as aten's broadcasting torch.mul into bf16 instead of
    mmt_scale_rows_cast."""
    from mmt_amd import train
    saved = train._scaled_bf16

    def scaled(dy, keep, rows_per):
        if keep is None:
            return dy.to(torch.bfloat16).contiguous()
        out = torch.empty(dy.shape, device=dy.device, dtype=torch.bfloat16)
        torch.mul(dy.view(keep.shape[0], rows_per, -1), keep.view(-1, 1, 1), out=out.view(keep.shape[0], rows_per, -1))
        return out

    train._scaled_bf16 = scaled
    try:
        yield
    finally:
        train._scaled_bf16 = saved


@contextlib.contextmanager
def dual_stream():
    """The pair backward's weight-gradient GEMMs on a side stream beside the input-gradient GEMMs."""
    from mmt_amd import train
    train.DUAL_STREAM = True
    try:
        yield
    finally:
        train.DUAL_STREAM = False


@contextlib.contextmanager
def sequential_backbones():
    """The two-stream backbones one after the other (one-group GEMMs) instead of backbone_forward_pair."""
    from mmt_amd import train
    train.PAIR = False
    try:
        yield
    finally:
        train.PAIR = True


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--only", default="", help="comma-separated variant names")
    args = ap.parse_args()
    variants = {"hip": HipOps, "aten_groupnorm": AtenGroupNormOps, "aten_layernorm": AtenLayerNormOps,
                "split_mlp": SplitMlpOps, "unfused_residual": UnfusedResidualOps, "accum_grads": (HipOps, accumulated_grads),
                "transposed": (HipOps, transposed_copies), "aten_scale_cast": (HipOps, aten_scale_cast),
                "sequential": (HipOps, sequential_backbones), "composed_encoder": ComposedEncoderOps,
                "dual_stream": (HipOps, dual_stream)}
    if args.only:
        variants = {k: v for k, v in variants.items() if k in args.only.split(",")}
    for r in range(args.rounds):
        for name, ops in variants.items():
            ops, ctx = ops if isinstance(ops, tuple) else (ops, contextlib.nullcontext)
            with ctx():
                o = bench.train_bench(1, 0, args.batch, args.steps, args.warmup, ops=ops)
            print(json.dumps({"round": r, "variant": name, "samples_per_s": o["value"], "ms_per_step": o["ms_per_step"],
                              "frac": o["roofline"]["frac"], "loss": o["last_loss"], "table_writes": o.get("opt_table_writes")}), flush=True)


if __name__ == "__main__":
    main()
