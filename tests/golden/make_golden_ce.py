"""Golden vectors of the candidate-elimination model (asymmetric_shared_ce) from
the REFERENCE's own Python (CPU), with the same stubs, weights and inputs as make_golden.py.

Run here only (the reference tree does not exist on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_ce.py

Model: build_asymmetric_shared_ce (asymmetric_shared_ce.py:611-675) with the reference config's
CE_LOC [3, 6, 9] and CE_KEEP_RATIO [0.7, 0.7, 0.7] (lib/config/asymmetric_shared_ce/config.py:23-24),
forward as the tracker calls it (ce_template_mask=None, ce_keep_rate=None; lib/test/tracker/
asymmetric_shared_ce.py:90-98); with --mask, as the training actor calls it (ce_template_mask =
generate_mask_cond's CTR_POINT mask, actors/mixformer_rgbt.py:67-90).  Besides the outputs it records, per elimination stage, the kept
search-token indices of each modality in the reference's order (candidate_elimination,
asymmetric_shared_ce.py:52-102, wrapped), so the selection itself is pinned."""
import json
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import make_golden as mg  # noqa: E402  (stubs, cfg, subsample helper)
from mmt_amd import synthetic  # noqa: E402

CE_LOC, CE_KEEP = [3, 6, 9], [0.7, 0.7, 0.7]


def ctr_point_mask(B):
    """The reference actor's template mask (actors/mixformer_rgbt.py:67-73): lib/utils/ce_utils.py
    generate_mask_cond with CE_TEMPLATE_RANGE = CTR_POINT, template 128 px / stride 16."""
    from lib.utils.ce_utils import generate_mask_cond
    cfg = mg.make_cfg()
    cfg.MODEL.BACKBONE.CE_TEMPLATE_RANGE = "CTR_POINT"
    cfg.MODEL.BACKBONE.STRIDE = 16
    return generate_mask_cond(cfg, B, torch.device("cpu"), None)


def run(B, masked=False):
    import lib.models.mixformer_vit_rgbt.asymmetric_shared_ce as ce
    torch.manual_seed(0)
    cfg = mg.make_cfg()
    cfg.MODEL.BACKBONE.CE_LOC = CE_LOC
    cfg.MODEL.BACKBONE.CE_KEEP_RATIO = CE_KEEP
    model = ce.build_asymmetric_shared_ce(cfg, train=False).eval()
    keys_shapes = [(k, list(v.shape)) for k, v in model.state_dict().items()]
    sd = synthetic.synth_state_dict(keys_shapes)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    t, o, s = synthetic.synth_inputs(B)
    stages = []
    orig_ce = ce.candidate_elimination

    def rec_ce(attn, *a):
        outs = orig_ce(attn, *a)
        am, box_mask_z = attn, a[-1]
        if box_mask_z is not None:  # the masked rows, as candidate_elimination :81-86 averages them
            bs, hn, _, L = attn.shape
            am = attn[box_mask_z.unsqueeze(1).unsqueeze(-1).expand(-1, hn, -1, L)].view(bs, hn, -1, L)
        stages.append((am.mean(dim=2).mean(dim=1).numpy(), outs[2].numpy(), outs[3].numpy()))
        return outs

    ce.candidate_elimination = rec_ce
    rec = {}
    head = model.box_head
    orig = head.get_score_map

    def gsm(x):
        a, b = orig(x)
        rec["score_map_tl"], rec["score_map_br"] = a, b
        return a, b

    head.get_score_map = gsm
    fz = model.fusion_vi.register_forward_hook(lambda m, i, out: rec.__setitem__("fusion", (i, out)))
    mask = ctr_point_mask(B) if masked else None
    try:
        with torch.no_grad():
            out, coord = model(t, o, s, ce_template_mask=mask)
    finally:
        ce.candidate_elimination = orig_ce
        fz.remove()
    (sv, si), fused = rec["fusion"]
    res = {"pred_boxes": out["pred_boxes"].numpy(), "coord": coord.numpy(),
           "score_map_tl": rec["score_map_tl"].numpy(), "score_map_br": rec["score_map_br"].numpy()}
    for nm, x in (("search_v", sv), ("search_i", si), ("fused", fused)):
        res[nm + "_sub"], res[nm + "_sum"] = mg.sub(x)
    for k, (attn_mean, kv, ki) in enumerate(stages):
        res["ce%d_attn_mean" % k] = attn_mean.astype(np.float32)  # (B, 2 * lens_s): [RGB | TIR] search tokens
        res["ce%d_keep_v" % k] = kv.astype(np.int32)  # global search-token index, reference order
        res["ce%d_keep_i" % k] = ki.astype(np.int32)
    if mask is not None:
        res["ce_template_mask"] = mask.numpy()
    return res, keys_shapes


def main():
    mg.install_stubs()
    if "--mask" in sys.argv:  # ce_template_mask = the actor's CTR_POINT mask (model_asym_ce_mask_b*.npz)
        for B in (1, 2):
            res, _ = run(B, masked=True)
            np.savez_compressed(os.path.join(HERE, "model_asym_ce_mask_b%d.npz" % B), **res)
            print("asym_ce mask", B, "boxes", res["pred_boxes"].reshape(-1, 4).tolist(),
                  "mask", int(res["ce_template_mask"].sum()), flush=True)
        return
    for B in (1, 2):
        res, keys = run(B)
        np.savez_compressed(os.path.join(HERE, "model_asym_ce_b%d.npz" % B), **res)
        if B == 1:
            with open(os.path.join(HERE, "state_dict_asym_ce.json"), "w") as f:
                json.dump(keys, f)
        print("asym_ce", B, "boxes", res["pred_boxes"].reshape(-1, 4).tolist(),
              "kept", [res["ce%d_keep_v" % k].shape for k in range(3)], flush=True)


if __name__ == "__main__":
    main()
