#!/usr/bin/env python3
"""The two-stream backbones in lockstep (train.PAIR, grouped GEMMs) against one after the other:
  1. the same function: eager TrainStep losses over a few steps from one init and batch without stochastic
     depth (drop_path_rate 0: no random draws, so the two forms see identical inputs);
  2. speed: the default bench's config-4 step (whole step one hipGraph replay), interleaved rounds."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))

import bench  # noqa: E402
import torch  # noqa: E402
from mmt_amd import train  # noqa: E402


def losses(pair, steps=6, B=16):
    from mmt_amd.model import build_mixformer_vit_rgbt, hot_path_cfg
    train.PAIR = pair
    torch.manual_seed(0)
    net = build_mixformer_vit_rgbt(hot_path_cfg(), train=False).cuda().train()
    net.drop_path_rate = 0.0
    step = train.TrainStep(net, train.HipOps)
    batch = train.synthetic_batch(B, "cuda", torch.Generator().manual_seed(5))
    out = [float(step(*batch)["loss"]) for _ in range(steps)]
    train.PAIR = True
    return out


def main():
    a, b = losses(False), losses(True)
    print(json.dumps({"check": "losses_dp0", "sequential": a, "pair": b,
                      "max_rel": max(abs(u - v) / abs(u) for u, v in zip(a, b))}), flush=True)
    for r in range(int(os.environ.get("ROUNDS", "3"))):
        for name, pair in (("pair", True), ("sequential", False)):
            train.PAIR = pair
            o = bench.train_bench(1, 0, 16, 10, 3)
            train.PAIR = True
            print(json.dumps({"round": r, "variant": name, "samples_per_s": o["value"], "ms_per_step": o["ms_per_step"],
                              "step_issue": o["step_issue"][:40], "loss": o.get("last_loss")}), flush=True)


if __name__ == "__main__":
    main()
