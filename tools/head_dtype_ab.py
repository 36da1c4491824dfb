#!/usr/bin/env python3
"""Box error vs the reference goldens of the 16-bit plans with the corner head stored in bf16, fp16 or
fp32 (MixFormerRGBTRuntime head_dtype), per variant, plus each plan's frame time (hipGraph replay).
usage: python tools/head_dtype_ab.py [rgb,rgbt,...]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multi-modal-tracking_amd")]
GOLDEN = os.path.join(ROOT, "tests", "golden")


def main():
    from mmt_amd import synthetic
    from mmt_amd.runtime import MixFormerRGBTRuntime
    only = sys.argv[1].split(",") if len(sys.argv) > 1 else None
    for variant, B in (("rgb", 1), ("rgb", 2), ("rgbt", 1), ("shared", 1), ("asym", 1), ("shared", 2)):
        if only and variant not in only:
            continue
        search = 288 if variant == "rgb" else 320
        keys = json.load(open(os.path.join(GOLDEN, "state_dict_%s.json" % variant)))
        sd = {k: torch.from_numpy(v) for k, v in synthetic.synth_state_dict(keys).items()}
        gold = np.load(os.path.join(GOLDEN, "model_%s_b%d.npz" % (variant, B)))["pred_boxes"].reshape(B, 4)
        t, o, s = synthetic.synth_inputs(B, 128, search)
        n = 1 if variant == "rgb" else 2
        t, o, s = [[x.cuda() for x in g[:n]] for g in (t, o, s)]
        for dt, hd in ((torch.bfloat16, None), (torch.bfloat16, torch.float16), (torch.bfloat16, torch.float32),
                       (torch.float16, None)):
            rt = MixFormerRGBTRuntime(sd, variant, dtype=dt, head_dtype=hd)
            box, _ = rt.forward(t, o, s)
            torch.cuda.synchronize()
            err = float(np.abs(box.cpu().numpy() - gold).max())
            g = rt.capture(B)
            g.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            print(json.dumps({"variant": variant, "B": B, "dtype": str(dt)[6:], "head": str(hd or dt)[6:],
                              "box_err": err, "ms": round(e0.elapsed_time(e1) / 50, 4)}), flush=True)
            del rt, g
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
