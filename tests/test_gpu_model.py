"""End-to-end parity of the HIP forward (mmt_amd.runtime) with the reference golden vectors.

Boxes (cxcywh in [0,1] of the search crop) must match within 1e-3 (fp32 path) / 1e-2 (bf16 path),
the tolerances BASELINE.json's north_star states; the score logit within the same bounds."""
import json

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

# B = 8: BASELINE config 3's per-rank batch (64 sequences over 8 GPUs): the batched MAM kernel
# (impl 22) and the large-M GEMM tile / split choices inside the model
CASES = [("rgbt", 1), ("shared", 1), ("asym", 1), ("asym_online", 1), ("shared", 2), ("shared", 8), ("asym", 8)]
_RT = {}


def _runtime(variant, dtype, fold_ln=None):
    key = (variant, dtype, fold_ln)
    if key not in _RT:
        from mmt_amd import synthetic
        from mmt_amd.runtime import MixFormerRGBTRuntime
        keys = json.load(open(GOLDEN + "/state_dict_%s.json" % variant))
        sd = {k: torch.from_numpy(v) for k, v in synthetic.synth_state_dict(keys).items()}
        _RT[key] = MixFormerRGBTRuntime(sd, variant, dtype=dtype, fold_ln=fold_ln)
    return _RT[key]


def _inputs(B):
    from mmt_amd import synthetic
    t, o, s = synthetic.synth_inputs(B)
    return [x.cuda() for x in t], [x.cuda() for x in o], [x.cuda() for x in s]


@pytest.mark.parametrize("dname,tol", [("f32", 1e-3), ("bf16", 1e-2)])
@pytest.mark.parametrize("variant,B", CASES)
def test_model_matches_reference(variant, B, dname, tol):
    dtype = torch.float32 if dname == "f32" else torch.bfloat16
    rt = _runtime(variant, dtype)
    t, o, s = _inputs(B)
    score = variant == "asym_online"
    box, sc = rt.forward(t, o, s, run_score_head=score)
    torch.cuda.synchronize()
    gold = np.load(GOLDEN + "/model_%s_b%d.npz" % (variant, B))
    err = np.abs(box.cpu().numpy() - gold["pred_boxes"].reshape(B, 4)).max()
    print("%s B=%d %s box err %.3g" % (variant, B, dname, err))
    assert err <= tol, err
    maps = rt.workspace(B)["MAPS"].cpu().numpy()  # [2][B][80*80] corner score maps
    for g, nm in enumerate(("score_map_tl", "score_map_br")):
        ref = gold[nm].reshape(B, -1)
        merr = np.abs(maps[g] - ref).max() / max(1.0, np.abs(ref).max())
        print("%s rel map err %.3g" % (nm, merr))
        assert merr <= (1e-4 if dname == "f32" else 5e-2), merr
    if score:
        serr = np.abs(sc.cpu().numpy() - gold["pred_scores"].reshape(-1)).max()
        print("score err %.3g" % serr)
        assert serr <= tol * max(1.0, float(np.abs(gold["pred_scores"]).max())), serr


@pytest.mark.parametrize("variant", ["rgbt", "asym_online"])
def test_graph_replay_is_bitwise_eager(variant):
    rt = _runtime(variant, torch.bfloat16)
    t, o, s = _inputs(1)
    score = variant == "asym_online"
    b0, s0 = rt.forward(t, o, s, run_score_head=score)
    b0, s0 = b0.clone(), (s0.clone() if s0 is not None else None)
    b1, s1 = rt.forward(t, o, s, run_score_head=score, use_graph=True)
    torch.cuda.synchronize()
    assert torch.equal(b0, b1)
    if score:
        assert torch.equal(s0, s1)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-5), (torch.bfloat16, 5e-3)])
def test_batch_rows_independent(dtype, tol):
    """Frame b of a batch equals the same frame run alone (no cross-batch leakage).  Not bitwise:
    the GEMM tile shape (hence the fp32 summation order) is chosen per M, i.e. per batch size."""
    rt = _runtime("asym", dtype)
    t, o, s = _inputs(2)
    b2, _ = rt.forward(t, o, s)
    b2 = b2.clone()
    b1, _ = rt.forward([x[1:2] for x in t], [x[1:2] for x in o], [x[1:2] for x in s])
    torch.cuda.synchronize()
    assert (b2[1] - b1[0]).abs().max().item() < tol


@pytest.mark.parametrize("variant", ["shared", "asym"])
def test_batch64_rows_match_single_frames(variant):
    """BASELINE config 3 on one GPU (64 sequences, mixformer_vit_rgbt_shared; the asymmetric model too):
    rows of the B = 64 forward equal the same frames run alone at B = 1 within the bf16 row bound of
    test_batch_rows_independent (different GEMM tiles / attention kernels per batch size, so not
    bitwise), and every row is finite."""
    rt = _runtime(variant, torch.bfloat16)
    t, o, s = _inputs(64)
    b64, _ = rt.forward(t, o, s)
    b64 = b64.clone()
    torch.cuda.synchronize()
    assert torch.isfinite(b64).all()
    for r in (0, 1, 31, 47, 63):
        b1, _ = rt.forward([x[r:r + 1] for x in t], [x[r:r + 1] for x in o], [x[r:r + 1] for x in s])
        torch.cuda.synchronize()
        err = (b64[r] - b1[0]).abs().max().item()
        assert err < 5e-3, (r, err)


def test_zero_copy_plan_matches_copy_path():
    """Graph of a plan whose patch staging reads resident frames in place == the copying forward."""
    rt = _runtime("rgbt", torch.bfloat16)
    t, o, s = _inputs(1)
    b0, _ = rt.forward(t, o, s)
    b0 = b0.clone()
    g = rt.capture_plan(rt.plan_for_inputs(t, o, s))
    rt.workspace(1)["BOX"].zero_()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(b0, rt.workspace(1)["BOX"])


@pytest.mark.parametrize("variant", ["rgbt", "asym"])
def test_bf16_layernorm_fold_vs_explicit(variant):
    """bf16 plan with the ViT LayerNorms folded into qkv / fc1 (default) against the plan with the
    explicit LayerNorm kernels: both within the bf16 bound of the golden boxes, and of each other."""
    t, o, s = _inputs(1)
    gold = np.load(GOLDEN + "/model_%s_b1.npz" % variant)["pred_boxes"].reshape(1, 4)
    boxes = []
    for fold in (True, False):
        rt = _runtime(variant, torch.bfloat16, fold_ln=fold)
        assert any(e[2] == "ln1" for e in rt.workspace(1)["plan"]) != fold
        box, _ = rt.forward(t, o, s)
        torch.cuda.synchronize()
        boxes.append(box.cpu().numpy().copy())
        assert np.abs(boxes[-1] - gold).max() <= 1e-2
    assert np.abs(boxes[0] - boxes[1]).max() <= 1e-2


@pytest.mark.parametrize("variant", ["rgbt", "asym_online"])
def test_module_api_after_cuda(variant):
    """The drop-in path a tracker takes (mixformer_vit_rgbt.py:16-24): build -> load_state_dict ->
    .cuda() -> .eval() -> forward([rgb, tir] lists) under no_grad, with the weights already on the
    device when the HIP runtime prepares them."""
    from mmt_amd import model as M
    from mmt_amd import synthetic
    builder = {"rgbt": M.build_mixformer_vit_rgbt, "asym_online": M.build_asymmetric_shared_online_score}[variant]
    net = builder(M.hot_path_cfg(), train=False)
    keys = json.load(open(GOLDEN + "/state_dict_%s.json" % variant))
    net.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.synth_state_dict(keys).items()}, strict=True)
    net = net.cuda().eval()
    t, o, s = _inputs(1)
    score = variant == "asym_online"
    with torch.no_grad():
        out, coord = net(t, o, s, run_score_head=score)
    torch.cuda.synchronize()
    gold = np.load(GOLDEN + "/model_%s_b1.npz" % variant)
    err = np.abs(out["pred_boxes"].cpu().numpy().reshape(1, 4) - gold["pred_boxes"].reshape(1, 4)).max()
    assert err <= 1e-2, err
    assert coord.shape == (1, 1, 4)
    if score:
        assert out["pred_scores"].shape == (1,)


def test_forward_ignores_gt_bboxes_like_reference():
    """asymmetric_shared_online.py:374: forward(..., run_score_head=True, gt_bboxes=...) drops gt_bboxes
    (forward_head is called without it), so the score pools the predicted box whatever boxes the actor
    passes (actors/mixformer_rgbt.py:92-98).  The module's score equals the one without gt_bboxes and
    the oracle's (fp32)."""
    from mmt_amd import model as M
    from mmt_amd import synthetic
    from oracle.forward import forward as oracle_forward
    net = M.build_asymmetric_shared_online_score(M.hot_path_cfg(), train=False)
    keys = json.load(open(GOLDEN + "/state_dict_asym_online.json"))
    sd = {k: torch.from_numpy(v) for k, v in synthetic.synth_state_dict(keys).items()}
    net.load_state_dict(sd, strict=True)
    net = net.cuda().eval().set_compute_dtype(torch.float32)
    B = 2
    t, o, s = synthetic.synth_inputs(B, seed=11)
    gt = torch.tensor([[0.30, 0.35, 0.62, 0.70], [0.12, 0.20, 0.48, 0.41]])
    args = ([x.cuda() for x in t], [x.cuda() for x in o], [x.cuda() for x in s])
    with torch.no_grad():
        a, _ = net(*args, run_score_head=True, gt_bboxes=gt.cuda())
        a = a["pred_scores"].cpu()
        b, _ = net(*args, run_score_head=True)
        b = b["pred_scores"].cpu()
    assert torch.equal(a, b)
    ref, _ = oracle_forward(sd, "asym_online", t, o, s, run_score_head=True)
    err = (a - ref["pred_scores"]).abs().max().item()
    assert err <= 1e-3 * max(1.0, ref["pred_scores"].abs().max().item()), err


def test_score_on_boxes_api_matches_oracle_decoder():
    """The runtime's explicit score_on_boxes (not a reference entry point: the score decoder on caller
    boxes, score_decoder.py:32-66) vs the oracle's score decoder on the same boxes (fp32)."""
    from mmt_amd import synthetic
    from oracle.forward import forward as oracle_forward
    from oracle.forward import score_decoder
    rt = _runtime("asym_online", torch.float32)
    keys = json.load(open(GOLDEN + "/state_dict_asym_online.json"))
    sd = {k: torch.from_numpy(v) for k, v in synthetic.synth_state_dict(keys).items()}
    B = 2
    t, o, s = synthetic.synth_inputs(B, seed=11)
    gt = torch.tensor([[0.30, 0.35, 0.62, 0.70], [0.12, 0.20, 0.48, 0.41]])
    rt.forward([x.cuda() for x in t], [x.cuda() for x in o], [x.cuda() for x in s], run_score_head=False)
    sc = rt.score_on_boxes(B, gt.cuda()).cpu()
    _, _, aux = oracle_forward(sd, "asym_online", t, o, s, run_score_head=True, return_aux=True)
    ref = score_decoder(sd, "score_branch.", aux["fused"], aux["score_template"], gt,
                        num_heads=aux["fused"].shape[1] // 64).view(-1)
    err = (sc - ref).abs().max().item()
    assert err <= 1e-3 * max(1.0, ref.abs().max().item()), err


def test_ce_keep_rate_argument():
    """asymmetric_shared_ce.py:557-567 signature: ce_keep_rate >= 1 disables the elimination (the
    result is the asymmetric model's), the configured rate gives the default forward; a template
    mask over every token is accepted."""
    from mmt_amd import model as M
    from mmt_amd import synthetic
    net = M.build_asymmetric_shared_ce(M.hot_path_cfg(), train=False)
    keys = [(k, list(v.shape)) for k, v in net.state_dict().items()]
    sd = {k: torch.from_numpy(v) for k, v in synthetic.synth_state_dict(keys).items()}
    net.load_state_dict(sd, strict=True)
    net = net.cuda().eval().set_compute_dtype(torch.float32)
    asym = M.build_asymmetric_shared(M.hot_path_cfg(), train=False)
    asym.load_state_dict(sd, strict=True)
    asym = asym.cuda().eval().set_compute_dtype(torch.float32)
    t, o, s = _inputs(1)
    with torch.no_grad():
        full, _ = net(t, o, s, False, None, torch.ones(1, 256, dtype=torch.bool), 1.0)
        ref, _ = asym(t, o, s)
        b_def, _ = net(t, o, s)
        b_07, _ = net(t, o, s, ce_keep_rate=0.7)
    assert (full["pred_boxes"] - ref["pred_boxes"]).abs().max().item() <= 1e-5
    assert torch.equal(b_def["pred_boxes"], b_07["pred_boxes"])


@pytest.mark.parametrize("dname,bound", [("bf16", 5e-3), ("fp16", 1e-3)])
@pytest.mark.parametrize("variant", ["rgbt", "shared", "asym", "asym_online"])
def test_16bit_headroom(variant, dname, bound):
    """Headroom under the north star's 1e-2 bound: the default (LayerNorm-folded) 16-bit plans keep the
    boxes within 5e-3 (bf16) / 1e-3 (fp16) of the reference's golden boxes (per-stage errors:
    tools/stage_error.py, profiles/r02_stage_error.jsonl)."""
    rt = _runtime(variant, {"bf16": torch.bfloat16, "fp16": torch.float16}[dname])
    t, o, s = _inputs(1)
    box, _ = rt.forward(t, o, s, run_score_head=variant == "asym_online")
    torch.cuda.synchronize()
    gold = np.load(GOLDEN + "/model_%s_b1.npz" % variant)["pred_boxes"].reshape(1, 4)
    err = np.abs(box.cpu().numpy() - gold).max()
    assert err <= bound, err


@pytest.mark.parametrize("dname,tol", [("f32", 1e-3), ("fp16", 1e-2)])
@pytest.mark.parametrize("B", [1, 2])
def test_rgb_only_model_matches_reference(B, dname, tol):
    """BASELINE config 1 on the GPU: the RGB-only MixFormer (lib/models/mixformer_vit, 128/288: one
    modality, corner head on the backbone's search tokens through the conv's image pitch) vs the
    reference's goldens (tests/golden/make_golden_rgb.py).  The reference runs this config in fp32;
    its 16-bit type here is fp16 (1e-2); bf16 is refused (test_rgb_only_refuses_bf16)."""
    from mmt_amd import synthetic
    from mmt_amd.runtime import MixFormerRGBTRuntime
    keys = json.load(open(GOLDEN + "/state_dict_rgb.json"))
    sd = {k: torch.from_numpy(v) for k, v in synthetic.synth_state_dict(keys).items()}
    rt = MixFormerRGBTRuntime(sd, "rgb", dtype={"f32": torch.float32, "fp16": torch.float16}[dname])
    t, o, s = synthetic.synth_inputs(B, 128, 288)
    box, _ = rt.forward([t[0].cuda()], [o[0].cuda()], [s[0].cuda()])
    torch.cuda.synchronize()
    g = np.load(GOLDEN + "/model_rgb_b%d.npz" % B)
    err = np.abs(box.cpu().numpy() - g["pred_boxes"].reshape(B, 4)).max()
    assert err <= tol, err
    maps = rt.workspace(B)["MAPS"].float().cpu().numpy().reshape(2, B, -1)
    for i, nm in enumerate(("score_map_tl", "score_map_br")):
        ref = g[nm].reshape(B, -1)
        assert np.abs(maps[i] - ref).max() <= (2e-3 if dname == "f32" else 1e-1) * np.abs(ref).max()


def test_rgb_only_module_api_and_template_cache():
    """build_mixformer_vit -> load_state_dict -> .cuda() -> forward(t, o, s) with single tensors, and
    set_online / forward_test (mixformer_vit/mixformer.py:308-321) equal to the full forward."""
    from mmt_amd import model as M
    from mmt_amd import synthetic
    net = M.build_mixformer_vit(M.hot_path_cfg(search=288), train=False)
    keys = json.load(open(GOLDEN + "/state_dict_rgb.json"))
    net.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.synth_state_dict(keys).items()}, strict=True)
    net = net.cuda().eval()
    t, o, s = synthetic.synth_inputs(1, 128, 288)
    t, o, s = t[0].cuda(), o[0].cuda(), s[0].cuda()
    with torch.no_grad():
        out, coord = net(t, o, s)
        net.set_online(t, o)
        out2, _ = net.forward_test(s)
    torch.cuda.synchronize()
    g = np.load(GOLDEN + "/model_rgb_b1.npz")["pred_boxes"].reshape(1, 1, 4)
    assert np.abs(out["pred_boxes"].cpu().numpy() - g).max() <= 1e-2
    assert coord.shape == (1, 1, 4)
    # the cached passes run compact activations (other GEMM tile / split-K choices for 128 / 324 rows than for
    # 452: another fp32 summation order), and this model's peaked maps amplify fp16 rounding (DESIGN.md §4:
    # 1.8e-3 from the golden at B = 1): both paths within the golden bar, and within 5e-3 of each other
    assert np.abs(out2["pred_boxes"].cpu().numpy() - g).max() <= 1e-2
    assert torch.allclose(out2["pred_boxes"], out["pred_boxes"], atol=5e-3)
