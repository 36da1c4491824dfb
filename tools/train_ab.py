#!/usr/bin/env python3
"""Interleaved A/B of training-step variants in one process (methodology rule 24): the config-4 step
(bench.train_bench, two-stream MixViT-B RGB-T, --batch pairs) with the product HipOps against
variants that swap one op back to aten.  One JSON line per (round, variant).

    python tools/train_ab.py --rounds 3 --steps 8 --warmup 3
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))

import bench  # noqa: E402
from mmt_amd.train import HipOps  # noqa: E402


class AtenLayerNormOps(HipOps):
    """HipOps with the backbone LayerNorms on aten (F.layer_norm + bf16 cast, autograd backward)."""
    layer_norm = None


class AtenGroupNormOps(HipOps):
    """HipOps with the fusion's adjust_* as NCHW Conv2d (MIOpen) + nn.GroupNorm (aten), as before."""
    group_norm = None


class SplitMlpOps(HipOps):
    """HipOps with each MLP as fc1 / aten GELU / fc2 (three autograd nodes) instead of _HipMlp."""
    mlp = None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--only", default="", help="comma-separated variant names")
    args = ap.parse_args()
    variants = {"hip": HipOps, "aten_groupnorm": AtenGroupNormOps, "aten_layernorm": AtenLayerNormOps,
                "split_mlp": SplitMlpOps}
    if args.only:
        variants = {k: v for k, v in variants.items() if k in args.only.split(",")}
    for r in range(args.rounds):
        for name, ops in variants.items():
            o = bench.train_bench(1, 0, args.batch, args.steps, args.warmup, ops=ops)
            print(json.dumps({"round": r, "variant": name, "samples_per_s": o["value"], "ms_per_step": o["ms_per_step"],
                              "frac": o["roofline"]["frac"], "loss": o["last_loss"]}), flush=True)


if __name__ == "__main__":
    main()
