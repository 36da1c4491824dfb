"""Pin the oracle (CPU restatement) to the reference's own outputs (tests/golden, made by
tests/golden/make_golden.py from /root/reference under import stubs) and to the reference's
known-answer tests.  CPU only."""
import json

import numpy as np
import pytest
import torch

from conftest import GOLDEN

# B = 8: BASELINE config 3's per-rank batch (64 sequences over 8 GPUs)
CASES = [("rgbt", 1), ("shared", 1), ("asym", 1), ("asym_online", 1), ("shared", 2), ("shared", 8), ("asym", 8)]


def _sub(x, n=4096):
    f = x.detach().reshape(-1).double()
    step = max(1, f.numel() // n)
    return f[::step][:n].float().numpy(), np.array([f.sum().item(), f.abs().sum().item(), f.numel()])


@pytest.fixture(scope="module")
def weights():
    from mmt_amd import synthetic
    from oracle.forward import state_dict_to_torch
    out = {}
    for v in ("rgbt", "shared", "asym", "asym_online"):
        keys = json.load(open(GOLDEN + "/state_dict_%s.json" % v))
        out[v] = state_dict_to_torch(synthetic.synth_state_dict(keys))
    return out


@pytest.mark.parametrize("variant,B", CASES)
def test_oracle_forward_matches_reference(weights, variant, B):
    from mmt_amd import synthetic
    from oracle import forward as of
    torch.set_num_threads(8)
    g = np.load(GOLDEN + "/model_%s_b%d.npz" % (variant, B))
    t, o, s = synthetic.synth_inputs(B)
    for nm, x in (("t_v", t[0]), ("t_i", t[1]), ("o_v", o[0]), ("o_i", o[1]), ("s_v", s[0]), ("s_i", s[1])):
        np.testing.assert_allclose([x.double().sum().item(), x.double().abs().sum().item()], g["in_" + nm + "_sum"], rtol=1e-12)
    sd = weights[variant]
    wsum = sum(float(v.double().abs().sum()) for v in sd.values())
    assert abs(wsum - float(g["weights_abs_sum"][0])) <= 1e-9 * wsum
    out, coord, aux = of.forward(sd, variant, t, o, s, run_score_head=(variant == "asym_online"), return_aux=True)
    assert np.abs(out["pred_boxes"].numpy() - g["pred_boxes"]).max() < 1e-5
    assert np.abs(coord.numpy() - g["coord"]).max() < 1e-5
    for nm in ("score_map_tl", "score_map_br"):
        assert np.abs(aux[nm].numpy() - g[nm]).max() < 1e-4 * max(1.0, np.abs(g[nm]).max())
    for nm in ("search_v", "search_i", "fused"):
        sub, sums = _sub(aux[nm])
        assert np.abs(sub - g[nm + "_sub"]).max() < 1e-4 * max(1.0, np.abs(g[nm + "_sub"]).max())
        assert abs(sums[0] - g[nm + "_sum"][0]) <= 1e-5 * g[nm + "_sum"][1]
        assert abs(sums[1] - g[nm + "_sum"][1]) <= 1e-5 * g[nm + "_sum"][1]
    if variant == "asym_online":
        assert np.abs(out["pred_scores"].numpy() - g["pred_scores"]).max() < 1e-5


@pytest.mark.parametrize("B", [1, 2])
def test_oracle_rgb_only_matches_reference(B):
    """BASELINE config 1: the RGB-only MixFormer (lib/models/mixformer_vit, 128/288) through the
    oracle vs the reference's own outputs (tests/golden/make_golden_rgb.py)."""
    from mmt_amd import synthetic
    from oracle import forward as of
    keys = json.load(open(GOLDEN + "/state_dict_rgb.json"))
    sd = of.state_dict_to_torch(synthetic.synth_state_dict(keys))
    g = np.load(GOLDEN + "/model_rgb_b%d.npz" % B)
    t, o, s = synthetic.synth_inputs(B, 128, 288)
    out, coord, aux = of.forward(sd, "rgb", t[0], o[0], s[0], return_aux=True)
    assert np.abs(out["pred_boxes"].numpy() - g["pred_boxes"]).max() < 1e-5
    assert np.abs(coord.numpy() - g["coord"]).max() < 1e-5
    for nm in ("score_map_tl", "score_map_br"):
        assert np.abs(aux[nm].numpy() - g[nm]).max() < 1e-4 * max(1.0, np.abs(g[nm]).max())
    sub, sums = _sub(aux["search"])
    assert np.abs(sub - g["search_sub"]).max() < 1e-4 * max(1.0, np.abs(g["search_sub"]).max())


def test_oracle_boxes_depend_on_input(weights):
    """Guard against vacuous box parity (SURVEY defect D8): different frames -> different boxes."""
    from mmt_amd import synthetic
    from oracle import forward as of
    sd = weights["asym"]
    boxes = []
    for seed in (1, 2, 3):
        t, o, s = synthetic.synth_inputs(1, seed=seed)
        boxes.append(of.forward(sd, "asym", t, o, s)[0]["pred_boxes"].reshape(4))
    spread = torch.stack(boxes).std(0).max().item()
    assert spread > 0.01, spread


def test_oracle_mam_attention_matches_reference_module():
    from mmt_amd import synthetic
    from oracle.forward import mam_attention, mam_attention_asym
    z = np.load(GOLDEN + "/op_attention.npz")
    g = torch.Generator().manual_seed(5)
    x = torch.randn(1, 528, 768, generator=g)
    xi = torch.randn(1, 528, 768, generator=g)
    shapes = [("attn.qkv.weight", [2304, 768]), ("attn.qkv.bias", [2304]), ("attn.proj.weight", [768, 768]),
              ("attn.proj.bias", [768])]
    sd = {k: torch.from_numpy(v) for k, v in synthetic.synth_state_dict(shapes).items()}
    args = (sd["attn.qkv.weight"], sd["attn.qkv.bias"], sd["attn.proj.weight"], sd["attn.proj.bias"])
    y = mam_attention(*args, x, 128, 12)
    sub, sums = _sub(y)
    assert np.abs(sub - z["mam_sub"]).max() < 1e-5
    yv, yi = mam_attention_asym(*args, x, xi, 128, 12)
    assert np.abs(_sub(yv)[0] - z["mam_asym_v_sub"]).max() < 1e-5
    assert np.abs(_sub(yi)[0] - z["mam_asym_i_sub"]).max() < 1e-5


@pytest.mark.parametrize("tag", ["double", "float"])
def test_oracle_msda_reference_test_vectors(tag):
    from oracle.msda import ms_deform_attn
    z = np.load(GOLDEN + "/op_msda.npz")
    dt = torch.float64 if tag == "double" else torch.float32
    v = torch.from_numpy(z["test_%s_value" % tag]).to(dt)
    loc = torch.from_numpy(z["test_%s_loc" % tag]).to(dt)
    w = torch.from_numpy(z["test_%s_w" % tag]).to(dt)
    out = ms_deform_attn(v, [(6, 4), (3, 2)], [0, 24], loc, w)
    ref = torch.from_numpy(z["test_%s_out" % tag])
    assert torch.allclose(out, ref.to(dt), rtol=1e-6 if tag == "float" else 1e-12, atol=1e-9 if tag == "float" else 1e-15)


def test_oracle_msda_bimodal_shape():
    from oracle.msda import ms_deform_attn
    z = np.load(GOLDEN + "/op_msda.npz")
    g = torch.Generator().manual_seed(7)
    value = torch.randn(1, 800, 8, 64, generator=g)
    loc = torch.rand(1, 800, 8, 2, 4, 2, generator=g) * 1.2 - 0.1
    w = torch.rand(1, 800, 8, 2, 4, generator=g)
    w = w / w.sum((-1, -2), keepdim=True)
    out = ms_deform_attn(value, [(20, 20), (20, 20)], [0, 400], loc, w)
    sub, sums = _sub(out)
    assert np.abs(sub - z["bimodal_out_sub"]).max() < 1e-5
    np.testing.assert_allclose(sums[:2], z["bimodal_out_sum"][:2], rtol=1e-6)


def test_oracle_prroi_known_answer():
    """external/PreciseRoIPooling/pytorch/tests/test_prroi_pooling2d.py:21-35."""
    import torch.nn.functional as F
    from oracle.prroi import prroi_pool2d
    g = torch.Generator().manual_seed(0)
    feat = torch.rand(4, 16, 24, 32, generator=g)
    rois = np.array([[0, 0, 0, 14, 14], [1, 14, 14, 28, 28]], dtype=np.float32)
    out = torch.from_numpy(prroi_pool2d(feat.numpy(), rois, 7, 7, 0.5))
    gold = F.avg_pool2d(feat, kernel_size=2, stride=1)
    assert torch.allclose(out, torch.stack((gold[0, :, :7, :7], gold[1, :, 7:14, 7:14])), atol=1e-6)


def test_oracle_prroi_empty_and_outside():
    from oracle.prroi import prroi_pool2d
    feat = np.ones((1, 2, 5, 5), dtype=np.float32)
    rois = np.array([[0, 2, 2, 2, 4], [0, 10, 10, 12, 12], [0, -1, -1, 1, 1]], dtype=np.float32)
    out = prroi_pool2d(feat, rois, 2, 2, 1.0)
    assert np.all(out[0] == 0)          # zero-width RoI -> empty bins
    assert np.all(out[1] == 0)          # fully outside -> zero-padded integral
    assert 0 < out[2, 0, 1, 1] <= 1.0   # partially outside -> partial mass


@pytest.mark.parametrize("masked", [False, True])
@pytest.mark.parametrize("B", [1, 2])
def test_oracle_candidate_elimination_matches_reference(B, masked):
    """asymmetric_shared_ce: boxes, maps and features, plus every elimination
    stage's mean template->search attention and kept token indices (reference order), vs the
    reference's own forward (tests/golden/make_golden_ce.py); masked: with the training actor's
    CTR_POINT ce_template_mask (lib/utils/ce_utils.py:14-38, the reference's own mask in the fixture)."""
    from mmt_amd import synthetic
    from oracle import forward as of
    torch.set_num_threads(8)
    g = np.load(GOLDEN + "/model_asym_ce_%sb%d.npz" % ("mask_" if masked else "", B))
    sd = of.state_dict_to_torch(synthetic.synth_state_dict(json.load(open(GOLDEN + "/state_dict_asym_ce.json"))))
    t, o, s = synthetic.synth_inputs(B)
    mask = torch.from_numpy(g["ce_template_mask"]) if masked else None
    if masked:  # CTR_POINT: the centre token (3, 3) of each of the four 8x8 templates
        assert mask.shape == (B, 256) and mask.sum().item() == 4 * B
        assert all(bool(mask[:, 64 * j + 27].all()) for j in range(4))
    out, coord, aux = of.forward(sd, "asym_ce", t, o, s, return_aux=True, ce_template_mask=mask)
    assert np.abs(out["pred_boxes"].numpy() - g["pred_boxes"]).max() < 1e-5
    for nm in ("score_map_tl", "score_map_br"):
        assert np.abs(aux[nm].numpy() - g[nm]).max() < 1e-4 * max(1.0, np.abs(g[nm]).max())
    for nm in ("search_v", "search_i", "fused"):
        sub, sums = _sub(aux[nm])
        assert np.abs(sub - g[nm + "_sub"]).max() < 1e-4 * max(1.0, np.abs(g[nm + "_sub"]).max())
    assert len(aux["ce_stages"]) == 3
    for k, (am, kv, ki) in enumerate(aux["ce_stages"]):
        assert np.abs(am.numpy() - g["ce%d_attn_mean" % k]).max() <= 1e-6 * np.abs(g["ce%d_attn_mean" % k]).max()
        assert np.array_equal(kv.numpy(), g["ce%d_keep_v" % k]) and np.array_equal(ki.numpy(), g["ce%d_keep_i" % k])
    assert [g["ce%d_keep_v" % k].shape[1] for k in range(3)] == [280, 196, 138]
