#!/usr/bin/env python3
"""Box error against the reference-made B = 1 golden (tests/golden/model_rgbt_b1.npz) and frame rate of the batch-1
two-stream forward for backbone / head storage-type pairs: is the bf16 headline's 1.8e-3 box error the backbone's or
the corner head's?  One JSON line per pair (graph replays timed like bench.py's value)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main(steps=300, warmup=30):
    from mmt_amd import synthetic
    from mmt_amd.runtime import MixFormerRGBTRuntime
    gdir = os.path.join(ROOT, "tests", "golden")
    keys = json.load(open(os.path.join(gdir, "state_dict_rgbt.json")))
    sd = {k: torch.from_numpy(v) for k, v in synthetic.synth_state_dict(keys).items()}
    gold = np.load(os.path.join(gdir, "model_rgbt_b1.npz"))["pred_boxes"].reshape(1, 4)
    t, o, s = [[x.cuda() for x in z] for z in synthetic.synth_inputs(1)]
    bf, fp, f32 = torch.bfloat16, torch.float16, torch.float32
    for dt, hdt in ((bf, bf), (bf, fp), (bf, f32), (fp, fp), (bf, bf), (bf, fp)):
        rt = MixFormerRGBTRuntime(sd, "rgbt", dtype=dt, head_dtype=hdt)
        box, _ = rt.forward(t, o, s)
        torch.cuda.synchronize()
        err = float(np.abs(box.cpu().numpy() - gold).max())
        g = rt.capture_plan(rt.plan_for_inputs(t, o, s))
        for _ in range(warmup):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            g.replay()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(json.dumps({"dtype": str(dt).split(".")[-1], "head_dtype": str(hdt).split(".")[-1],
                          "box_err_vs_reference": err, "frames_per_s": round(steps / el, 1)}), flush=True)
        del rt, g


if __name__ == "__main__":
    main()
