"""Generate the golden vectors in tests/golden/ from the REFERENCE's own Python (CPU).

Run here only (the reference tree does not exist on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Recipe: install stub modules for the absent third-party packages (timm, mmcv,
easydict, torchvision) and for the two native ops (MultiScaleDeformableAttention -> the
reference's own `ms_deform_attn_core_pytorch`; PrRoIPool -> oracle/prroi.py, because the
reference has no CPU path and its JIT build must never run: it would write into the read-only
tree), then import /root/reference/lib read-only, build each hot-path model with the
seed-derived weights of mmt_amd.synthetic, and record outputs and intermediates.
Nothing is written under /root/reference (sys.dont_write_bytecode, no JIT, no env_settings()).
"""
import json
import os
import sys
import time
import types

sys.dont_write_bytecode = True
REF = "/root/reference"
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.dirname(os.path.abspath(__file__))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

sys.path.insert(0, REF)
sys.path.append(REPO)
sys.path.append(os.path.join(REPO, "multi-modal-tracking_amd"))

from mmt_amd import synthetic  # noqa: E402
from oracle.prroi import prroi_pool2d as prroi_np  # noqa: E402


# ----------------------------------------------------------------------------- stubs
def _mod(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


class EasyDict(dict):
    def __init__(self, d=None, **kw):
        super().__init__()
        for k, v in dict(d or {}, **kw).items():
            self[k] = v

    def __setitem__(self, k, v):
        if isinstance(v, dict) and not isinstance(v, EasyDict):
            v = EasyDict(v)
        super().__setitem__(k, v)

    __setattr__ = __setitem__

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k)


class _TimmViT(nn.Module):
    def __init__(self, drop_rate=0.0, **kw):
        super().__init__()
        self.pos_drop = nn.Dropout(drop_rate)

    def init_weights(self, *a, **k):
        pass


class _Mlp(nn.Module):
    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU, drop=0.0):
        super().__init__()
        hidden_features = hidden_features or in_features
        out_features = out_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.act = act_layer()
        self.drop1 = nn.Dropout(drop)
        self.fc2 = nn.Linear(hidden_features, out_features)
        self.drop2 = nn.Dropout(drop)

    def forward(self, x):
        return self.drop2(self.fc2(self.drop1(self.act(self.fc1(x)))))


class _DropPath(nn.Module):
    def __init__(self, p=0.0):
        super().__init__()

    def forward(self, x):
        return x


class _PrRoIPool2D(nn.Module):
    def __init__(self, ph, pw, spatial_scale):
        super().__init__()
        self.ph, self.pw, self.scale = int(ph), int(pw), float(spatial_scale)

    def forward(self, features, rois):
        return torch.from_numpy(prroi_np(features.detach().numpy(), rois.detach().numpy(), self.ph, self.pw, self.scale))


def _box_area(b):
    return (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])


def _msda_forward(value, shapes, level_start, loc, w, step):
    from lib.models.mixformer_vit_rgbt.deformable_attention.ops.functions.ms_deform_attn_func import (
        ms_deform_attn_core_pytorch,
    )
    return ms_deform_attn_core_pytorch(value, shapes, loc, w)


def install_stubs():
    _mod("timm")
    _mod("timm.models")
    _mod("timm.models.vision_transformer", VisionTransformer=_TimmViT)
    _mod("timm.models.layers", DropPath=_DropPath, Mlp=_Mlp, trunc_normal_=nn.init.trunc_normal_)
    sys.modules["timm"].models = sys.modules["timm.models"]
    sys.modules["timm.models"].vision_transformer = sys.modules["timm.models.vision_transformer"]
    sys.modules["timm.models"].layers = sys.modules["timm.models.layers"]
    _mod("mmcv")
    _mod("mmcv.ops", ModulatedDeformConv2d=None, ModulatedDeformConv2dPack=None)
    _mod("easydict", EasyDict=EasyDict)
    tv = _mod("torchvision", _is_tracing=lambda: False, __version__="0.0-stub")
    tv.ops = _mod("torchvision.ops")
    tv.ops.boxes = _mod("torchvision.ops.boxes", box_area=_box_area)
    tv.ops.misc = _mod("torchvision.ops.misc")
    _mod("MultiScaleDeformableAttention", ms_deform_attn_forward=_msda_forward)
    for n in ("external", "external.PreciseRoIPooling", "external.PreciseRoIPooling.pytorch"):
        _mod(n)
    _mod("external.PreciseRoIPooling.pytorch.prroi_pool", PrRoIPool2D=_PrRoIPool2D)
    torch.Tensor.cuda = lambda self, *a, **k: self  # head.py:143-145 call .cuda() at init


# ----------------------------------------------------------------------------- config
def make_cfg(search=320, template=128, fusion_layers=2, vit="base_patch16", hidden=768):
    cfg = EasyDict()
    cfg.MODEL = EasyDict(
        VIT_TYPE=vit, HIDDEN_DIM=hidden, HEAD_TYPE="CORNER_UP", FUSION_CLASS="Attention_Fusion_Bimodal_LNSpecific",
        FUSION_LAYERS=fusion_layers, RGBT_PRETRAINED_PATH="", TRACKER_PRETRAINED_PATH="", SCORE_PRETRAINED_PATH="",
        BACKBONE=EasyDict(PRETRAINED=False, PRETRAINED_PATH=""),
    )
    cfg.DATA = EasyDict(SEARCH=EasyDict(SIZE=search), TEMPLATE=EasyDict(SIZE=template))
    return cfg


def build(variant, cfg):
    if variant == "rgbt":
        from lib.models.mixformer_vit_rgbt import build_mixformer_vit_rgbt as b
    elif variant == "shared":
        from lib.models.mixformer_vit_rgbt import build_mixformer_vit_rgbt_shared as b
    elif variant == "asym":
        from lib.models.mixformer_vit_rgbt.asymmetric_shared import build_asymmetric_shared as b
    else:
        from lib.models.mixformer_vit_rgbt.asymmetric_shared_online import build_asymmetric_shared_online_score as b
    return b(cfg, train=False)


def sub(x, n=4096):
    """Deterministic subsample + checksums of a tensor."""
    f = x.detach().reshape(-1).double()
    step = max(1, f.numel() // n)
    return f[::step][:n].float().numpy(), np.array([f.sum().item(), f.abs().sum().item(), f.numel()], dtype=np.float64)


def run_model(variant, B, timing=True):
    torch.manual_seed(0)
    cfg = make_cfg()
    model = build(variant, cfg).eval()
    keys_shapes = [(k, list(v.shape)) for k, v in model.state_dict().items()]
    sd = synthetic.synth_state_dict(keys_shapes)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    t, o, s = synthetic.synth_inputs(B)

    rec = {}
    head = model.box_head
    orig = head.get_score_map

    def gsm(x):
        a, b = orig(x)
        rec["score_map_tl"], rec["score_map_br"] = a, b
        return a, b

    head.get_score_map = gsm
    fz = model.fusion_vi.register_forward_hook(lambda m, i, out: rec.__setitem__("fusion", (i, out)))
    with torch.no_grad():
        kw = {"run_score_head": True} if variant == "asym_online" else {}
        out, coord = model(t, o, s, **kw)
    fz.remove()
    (sv, si), fused = rec["fusion"]
    res = {"pred_boxes": out["pred_boxes"].numpy(), "coord": coord.numpy(),
           "score_map_tl": rec["score_map_tl"].numpy(), "score_map_br": rec["score_map_br"].numpy()}
    if "pred_scores" in out:
        res["pred_scores"] = out["pred_scores"].numpy()
    for nm, x in (("search_v", sv), ("search_i", si), ("fused", fused)):
        res[nm + "_sub"], res[nm + "_sum"] = sub(x)
    for nm, x in (("t_v", t[0]), ("t_i", t[1]), ("o_v", o[0]), ("o_i", o[1]), ("s_v", s[0]), ("s_i", s[1])):
        res["in_" + nm + "_sum"] = np.array([x.double().sum().item(), x.double().abs().sum().item()])
    res["weights_abs_sum"] = np.array([sum(float(np.abs(v).astype(np.float64).sum()) for v in sd.values())])
    fps = None
    if timing:
        torch.set_num_threads(8)
        with torch.no_grad():
            model(t, o, s)
            n = 3
            t0 = time.perf_counter()
            for _ in range(n):
                model(t, o, s)
            fps = n * B / (time.perf_counter() - t0)
    return res, keys_shapes, fps


def attention_fixture():
    """One MAM attention module of each kind on N(0,1) tokens (B=1, 528 tokens, C=768)."""
    from lib.models.mixformer_vit_rgbt.mixformer import Attention as A
    from lib.models.mixformer_vit_rgbt.asymmetric_shared import Attention as AA

    res = {}
    g = torch.Generator().manual_seed(5)
    x = torch.randn(1, 528, 768, generator=g)
    xi = torch.randn(1, 528, 768, generator=g)
    for nm, cls in (("mam", A), ("mam_asym", AA)):
        m = cls(768, num_heads=12, qkv_bias=True).eval()
        sd = synthetic.synth_state_dict([("attn." + k, list(v.shape)) for k, v in m.state_dict().items()])
        m.load_state_dict({k[5:]: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
        with torch.no_grad():
            if nm == "mam":
                y = m(x, 8, 8, 20, 20)
                res[nm + "_sub"], res[nm + "_sum"] = sub(y)
            else:
                yv, yi = m(x, xi, 8, 8, 20, 20)
                res[nm + "_v_sub"], res[nm + "_v_sum"] = sub(yv)
                res[nm + "_i_sub"], res[nm + "_i_sum"] = sub(yi)
    return res


def msda_fixture():
    from lib.models.mixformer_vit_rgbt.deformable_attention.ops.functions.ms_deform_attn_func import (
        ms_deform_attn_core_pytorch,
    )

    res = {}
    # ops/test.py:20-59 shapes and seed, in the test's draw order (double check, then float check)
    N, M, D, Lq, L, P = 1, 2, 2, 2, 2, 2
    shapes = torch.as_tensor([(6, 4), (3, 2)], dtype=torch.long)
    S = int(sum(h * w for h, w in shapes.tolist()))
    torch.manual_seed(3)
    for tag in ("double", "float"):
        value = torch.rand(N, S, M, D) * 0.01
        loc = torch.rand(N, Lq, M, L, P, 2)
        w = torch.rand(N, Lq, M, L, P) + 1e-5
        w /= w.sum(-1, keepdim=True).sum(-2, keepdim=True)
        if tag == "double":
            out = ms_deform_attn_core_pytorch(value.double(), shapes, loc.double(), w.double())
        else:
            out = ms_deform_attn_core_pytorch(value, shapes, loc, w)
        res["test_%s_value" % tag], res["test_%s_loc" % tag], res["test_%s_w" % tag] = value.numpy(), loc.numpy(), w.numpy()
        res["test_%s_out" % tag] = out.numpy()
    # the hot-path bimodal shape: value (1,800,8,64), 2 levels of 20x20, 4 points; seeded inputs
    g = torch.Generator().manual_seed(7)
    value = torch.randn(1, 800, 8, 64, generator=g)
    loc = torch.rand(1, 800, 8, 2, 4, 2, generator=g) * 1.2 - 0.1
    w = torch.rand(1, 800, 8, 2, 4, generator=g)
    w = w / w.sum((-1, -2), keepdim=True)
    shapes = torch.as_tensor([(20, 20), (20, 20)], dtype=torch.long)
    out = ms_deform_attn_core_pytorch(value, shapes, loc, w)
    res["bimodal_out_sub"], res["bimodal_out_sum"] = sub(out)
    return res


def main():
    install_stubs()
    if len(sys.argv) > 2 and sys.argv[1] == "--cases":
        # extra (variant, batch) fixtures only, e.g. --cases shared:8,asym:8 (BASELINE config 3's
        # per-rank batch; the default run below leaves them untouched)
        for case in sys.argv[2].split(","):
            variant, B = case.split(":")
            t0 = time.time()
            res, _, _ = run_model(variant, int(B), timing=False)
            np.savez_compressed(os.path.join(OUT, "model_%s_b%d.npz" % (variant, int(B))), **res)
            print(variant, B, "boxes", res["pred_boxes"].reshape(-1, 4).tolist(), "%.1fs" % (time.time() - t0), flush=True)
        return
    meta = {"reference": "LZ-QWQ/Multi-modal-Tracking @ /root/reference (read-only)", "torch": torch.__version__,
            "weights": "mmt-synth-v1 (mmt_amd/synthetic.py), HEAD_GAIN=%g" % synthetic.HEAD_GAIN,
            "inputs": "synth_inputs(B, 128, 320, seed=1)", "cpu_fps_ref": {}}
    for variant, B in (("rgbt", 1), ("shared", 1), ("asym", 1), ("asym_online", 1), ("shared", 2)):
        t0 = time.time()
        res, keys, fps = run_model(variant, B, timing=(B == 1))
        np.savez_compressed(os.path.join(OUT, "model_%s_b%d.npz" % (variant, B)), **res)
        if B == 1:
            with open(os.path.join(OUT, "state_dict_%s.json" % variant), "w") as f:
                json.dump(keys, f)
            meta["cpu_fps_ref"][variant] = fps
        print(variant, B, "boxes", res["pred_boxes"].reshape(-1, 4).tolist(),
              "scores", res.get("pred_scores"), "fps", fps, "%.1fs" % (time.time() - t0), flush=True)
    np.savez_compressed(os.path.join(OUT, "op_attention.npz"), **attention_fixture())
    np.savez_compressed(os.path.join(OUT, "op_msda.npz"), **msda_fixture())
    meta["torch_threads"] = torch.get_num_threads()
    with open(os.path.join(OUT, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
