"""Golden vectors of the RGB-only MixFormer (BASELINE config 1: lib/models/mixformer_vit, MixViT-B,
128 px templates / 288 px search, CORNER_UP head) from the REFERENCE's own Python (CPU), with the stub
recipe of make_golden.py.  Run here only:
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_rgb.py
Writes model_rgb_b{1,2}.npz (inputs are the RGB halves of mmt_amd.synthetic.synth_inputs) and
state_dict_rgb.json; adds the reference's CPU rate to meta.json ("cpu_fps_ref"."rgb")."""
import json
import os
import sys
import time

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (stubs; nothing is written under /root/reference)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mmt_amd import synthetic  # noqa: E402

SEARCH, TEMPLATE = 288, 128


def cfg_rgb():
    cfg = mg.make_cfg(search=SEARCH, template=TEMPLATE)
    cfg.MODEL.RGB_PRETRAINED_PATH = ""
    return cfg


def run(B, timing):
    mg.install_stubs()
    from lib.models.mixformer_vit.mixformer import build_mixformer_vit
    torch.manual_seed(0)
    model = build_mixformer_vit(cfg_rgb(), train=False).eval()
    keys = [(k, list(v.shape)) for k, v in model.state_dict().items()]
    sd = synthetic.synth_state_dict(keys)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    t, o, s = synthetic.synth_inputs(B, TEMPLATE, SEARCH)
    t, o, s = t[0], o[0], s[0]
    rec = {}
    head = model.box_head
    orig = head.get_score_map

    def gsm(x):
        a, b = orig(x)
        rec["tl"], rec["br"] = a, b
        return a, b

    head.get_score_map = gsm
    hk = model.box_head.register_forward_hook(lambda m, i, out: rec.__setitem__("head_in", i[0]))
    with torch.no_grad():
        out, coord = model(t, o, s)
    hk.remove()
    res = {"pred_boxes": out["pred_boxes"].numpy(), "coord": coord.numpy(), "score_map_tl": rec["tl"].numpy(),
           "score_map_br": rec["br"].numpy()}
    res["search_sub"], res["search_sum"] = mg.sub(rec["head_in"])
    fps = None
    if timing:
        with torch.no_grad():
            model(t, o, s)
            t0 = time.perf_counter()
            for _ in range(3):
                model(t, o, s)
            fps = 3 * B / (time.perf_counter() - t0)
    return res, keys, fps


def main():
    torch.set_num_threads(8)
    meta_p = os.path.join(HERE, "meta.json")
    meta = json.load(open(meta_p))
    for B in (1, 2):
        res, keys, fps = run(B, B == 1)
        np.savez_compressed(os.path.join(HERE, "model_rgb_b%d.npz" % B), **res)
        if B == 1:
            json.dump(keys, open(os.path.join(HERE, "state_dict_rgb.json"), "w"))
            meta.setdefault("cpu_fps_ref", {})["rgb"] = fps
        print("rgb", B, res["pred_boxes"].reshape(-1, 4).tolist(), "fps", fps)
    json.dump(meta, open(meta_p, "w"), indent=1)


if __name__ == "__main__":
    main()
