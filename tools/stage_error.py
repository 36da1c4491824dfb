#!/usr/bin/env python3
"""Per-stage error of the 16-bit forward against the reference golden vectors (tests/golden/, made by
the reference itself): backbone search tokens of both modalities (the fusion's inputs), the fused map
(the fusion's output), both score maps and the boxes, for each variant and plan (LayerNorm folded /
explicit) and dtype (bf16 / fp16).  Errors are max |got - golden| / max |golden| on the golden's
deterministic subsample (make_golden.sub), boxes absolute.  Diagnostic only (what to keep in fp32 to
give the 16-bit path headroom under the north star's 1e-2 box bound).

usage: python tools/stage_error.py [--variants rgbt,shared,asym,asym_online] [--dtypes bf16,fp16]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multi-modal-tracking_amd")]
GOLDEN = os.path.join(ROOT, "tests", "golden")


def sub(x, n=4096):  # tests/golden/make_golden.py:163-167
    f = x.detach().reshape(-1).double()
    step = max(1, f.numel() // n)
    return f[::step][:n].float().cpu().numpy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="rgbt,shared,asym,asym_online")
    ap.add_argument("--dtypes", default="bf16,fp16")
    a = ap.parse_args()
    from mmt_amd import synthetic
    from mmt_amd.runtime import MixFormerRGBTRuntime
    t, o, s = synthetic.synth_inputs(1)
    t, o, s = [[x.cuda() for x in g] for g in (t, o, s)]
    for variant in a.variants.split(","):
        gold = np.load(os.path.join(GOLDEN, "model_%s_b1.npz" % variant))
        keys = json.load(open(os.path.join(GOLDEN, "state_dict_%s.json" % variant)))
        sd = {k: torch.from_numpy(v) for k, v in synthetic.synth_state_dict(keys).items()}
        for dname in a.dtypes.split(","):
            dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "f32": torch.float32}[dname]
            for fold in ((True, False) if dt != torch.float32 else (False,)):
                rt = MixFormerRGBTRuntime(sd, variant, dtype=dt, fold_ln=fold)
                score = variant == "asym_online"
                box, sc = rt.forward(t, o, s, run_score_head=score)
                torch.cuda.synchronize()
                ws = rt.workspace(1)
                d = rt.d
                X = ws["XN"] if rt.fold_ln else ws["XT"]  # the fusion's input (the backbone output, dtype)
                X = X.float().reshape(2, d.ntok, d.C)[:, d.n_t:]  # [m][400][C]
                row = {"variant": variant, "dtype": dname, "fold_ln": fold}
                for m, nm in ((0, "search_v"), (1, "search_i")):
                    nchw = X[m].reshape(d.gs, d.gs, d.C).permute(2, 0, 1)[None]
                    g = gold[nm + "_sub"]
                    row[nm] = float(np.abs(sub(nchw) - g).max() / np.abs(g).max())
                fus = ws["FUS"].float().reshape(d.gs, d.gs, d.C).permute(2, 0, 1)[None]
                g = gold["fused_sub"]
                row["fused"] = float(np.abs(sub(fus) - g).max() / np.abs(g).max())
                maps = ws["MAPS"].float().reshape(2, d.fh, d.fh).cpu().numpy()
                for i, nm in enumerate(("score_map_tl", "score_map_br")):
                    g = gold[nm].reshape(d.fh, d.fh)
                    row[nm] = float(np.abs(maps[i] - g).max() / np.abs(g).max())
                row["box"] = float(np.abs(box.cpu().numpy().reshape(4) - gold["pred_boxes"].reshape(4)).max())
                if score:
                    row["score"] = float(abs(sc.cpu().reshape(-1)[0].item() - gold["pred_scores"].reshape(-1)[0]))
                print(json.dumps(row), flush=True)
                del rt
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
