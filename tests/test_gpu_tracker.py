"""GPU parity of the tracker pre/post-processing (csrc/preprocess.hip through the C ABI) with the
oracle restatement (oracle/preprocess.py, itself pinned to the reference's sample_target geometry and
map_box_back / clip_box by tests/golden/tracker_geometry.npz), and of the device-resident tracking
loop (lib/test/tracker/*, mmt_amd.tracking) with the oracle's host tracking loop
(lib/test/tracker/mixformer_vit_rgbt.py:45-121 restated: crop, preprocess, fp32 CPU forward,
map back, clip, template update).

Bars: the uint8 crops, the crop geometry and the box update are bit-exact; the normalised fp32
crops are bit-exact (the kernel keeps torch's operation order, no FMA contraction); the tracked
boxes of the fp32 HIP forward are within 1e-3 of the search-crop size (the north_star tolerance on
normalised boxes, scaled to pixels by search_size / resize_factor)."""
import numpy as np
import pytest
import torch

from oracle import preprocess as pp

pytestmark = pytest.mark.gpu


def _frame(H, W, seed):
    """A smooth-ish random uint8 frame (HWC), so resize interpolation is exercised."""
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, (H // 8 + 2, W // 8 + 2, 3)).astype(np.float64)
    t = torch.from_numpy(base).permute(2, 0, 1)[None]
    sm = torch.nn.functional.interpolate(t, size=(H, W), mode="bilinear", align_corners=False)[0].permute(1, 2, 0).numpy()
    noise = rng.integers(-20, 21, (H, W, 3))
    return np.clip(sm + noise, 0, 255).astype(np.uint8)


# (box x, y, w, h), factor, out_sz: interior, every edge / corner, crop larger than the frame,
# non-integer boxes on .5 rounding ties, exact 2x downscale (INTER_AREA path), upscale
CROPS = [
    ((200.0, 150.0, 60.0, 40.0), 5.0, 320),
    ((2.0, 3.0, 30.0, 50.0), 5.0, 320),
    ((440.0, 330.0, 35.0, 25.0), 5.0, 320),
    ((-10.0, 300.0, 40.0, 40.0), 2.0, 128),
    ((100.25, 80.5, 33.3, 21.7), 2.0, 128),
    ((10.0, 10.0, 400.0, 300.0), 5.0, 320),
    ((150.0, 100.0, 64.0, 64.0), 4.0, 128),   # crop 256 -> 128: exact 2x
    ((150.0, 100.0, 80.0, 80.0), 4.0, 160),   # crop 320 -> 160: exact 2x
    ((300.5, 200.5, 7.0, 9.0), 2.0, 128),     # upscale
    ((0.0, 0.0, 480.0, 360.0), 1.0, 320),
]


def _run_crops(im_dev, specs, lut_dev):
    from mmt_amd import tracking
    outs = []
    params = []
    for box, factor, osz in specs:
        b = torch.tensor(box, dtype=torch.float64, device="cuda")
        out = torch.empty(3 * osz * osz, device="cuda")
        patch = torch.empty(osz * osz * 3, dtype=torch.uint8, device="cuda")
        crop = torch.empty(4, dtype=torch.float64, device="cuda")
        params.append(tracking.crop_params(im_dev, b, factor, osz, out=out, patch=patch, crop=crop, lut=lut_dev))
        outs.append((b, out, patch, crop))
    tracking.sample_target(params)
    torch.cuda.synchronize()
    return outs


@pytest.mark.parametrize("colormap", [False, True])
@pytest.mark.parametrize("ci", range(len(CROPS)))
def test_sample_target_bit_exact(ci, colormap):
    from mmt_amd import tracking
    im = _frame(360, 480, 7)
    im_dev = torch.from_numpy(im).cuda()
    lut = pp.jet_lut()
    np.testing.assert_array_equal(tracking.jet_lut(), lut)
    lut_dev = torch.from_numpy(lut.reshape(-1)).cuda() if colormap else None
    box, factor, osz = CROPS[ci]
    (_, out, patch, crop), = _run_crops(im_dev, [(box, factor, osz)], lut_dev)
    ref_norm, ref_patch, rf = pp.preprocess(im, box, factor, osz, lut=lut if colormap else None)
    x1, y1, csz = pp.crop_geometry(box, factor)
    assert crop.cpu().tolist() == [float(x1), float(y1), float(csz), rf]
    np.testing.assert_array_equal(patch.cpu().numpy().reshape(osz, osz, 3), ref_patch)
    got = out.cpu().numpy().reshape(3, osz, osz)
    assert np.array_equal(got.view(np.uint32), ref_norm.view(np.uint32)), np.abs(got - ref_norm).max()


def test_sample_target_batched_crops_independent():
    """Four crops in one launch (both modalities' search + template crops) equal four single launches."""
    im = _frame(360, 480, 8)
    im_dev = torch.from_numpy(im).cuda()
    specs = [CROPS[0], CROPS[1], CROPS[2], CROPS[5]]
    many = _run_crops(im_dev, specs, None)
    for s, (_, out, patch, crop) in zip(specs, many):
        (_, out1, patch1, crop1), = _run_crops(im_dev, [s], None)
        assert torch.equal(out, out1) and torch.equal(patch, patch1) and torch.equal(crop, crop1)


def test_sample_target_rejects_bad_args():
    from mmt_amd import tracking
    from mmt_amd._lib import LIB, CropParams
    im_dev = torch.zeros(16, 16, 3, dtype=torch.uint8, device="cuda")
    b = torch.tensor([1.0, 1.0, 4.0, 4.0], dtype=torch.float64, device="cuda")
    out = torch.empty(3 * 32 * 32, device="cuda")
    out2 = torch.empty(3 * 16 * 16, device="cuda")
    p1 = tracking.crop_params(im_dev, b, 2.0, 32, out=out)
    p2 = tracking.crop_params(im_dev, b, 2.0, 16, out=out2)
    s = torch.cuda.current_stream().cuda_stream
    assert LIB.mmt_sample_target((CropParams * 2)(p1, p2), 2, s) != 0  # mixed out_sz
    assert LIB.mmt_sample_target((CropParams * 5)(*([p1] * 5)), 5, s) != 0  # > MMT_MAX_CROPS
    with pytest.raises(ValueError):
        tracking.crop_params(im_dev.float(), b, 2.0, 32, out=out)


def test_track_update_bit_exact():
    from mmt_amd._lib import LIB, check
    rng = np.random.default_rng(3)
    n, H, W, ss = 257, 360, 480, 320
    pred = rng.uniform(-0.2, 1.2, (n, 4)).astype(np.float32)
    pred[:, 2:] = np.abs(pred[:, 2:])
    state = np.stack([rng.uniform(-50, W, n), rng.uniform(-50, H, n), rng.uniform(1, 300, n),
                      rng.uniform(1, 300, n)], 1)
    rf = rng.uniform(0.2, 6.0, n)
    crop = np.zeros((n, 4))
    crop[:, 3] = rf
    st_dev = torch.from_numpy(state.copy()).cuda()
    pred_dev, crop_dev = torch.from_numpy(pred).cuda(), torch.from_numpy(crop).cuda()  # alive across the launch
    check(LIB.mmt_track_update(pred_dev.data_ptr(), crop_dev.data_ptr(), st_dev.data_ptr(), n, H, W, ss, 10.0, torch.cuda.current_stream().cuda_stream),
          "mmt_track_update")
    got = st_dev.cpu().numpy()
    for i in range(n):
        ref = pp.track_update(pred[i], list(state[i]), float(rf[i]), H, W, ss)
        assert got[i].tolist() == ref, (i, got[i].tolist(), ref)


# ------------------------------------------------------------------ tracking loop
def _params(variant):
    from types import SimpleNamespace

    from mmt_amd.model import hot_path_cfg
    cfg = hot_path_cfg()
    return SimpleNamespace(cfg=cfg, template_factor=2.0, template_size=128, search_factor=5.0, search_size=320,
                           checkpoint=None, save_all_boxes=False)


def _tracker(variant, module):
    import importlib
    import json

    from conftest import GOLDEN
    from mmt_amd import synthetic
    mod = importlib.import_module("lib.test.tracker.%s" % module)
    params = _params(variant)
    params.cfg.TEST.UPDATE_INTERVALS = {"SYNTH": [3]}
    keys = json.load(open(GOLDEN + "/state_dict_%s.json" % variant))
    sd = {k: torch.from_numpy(v) for k, v in synthetic.synth_state_dict(keys).items()}
    trk = mod.get_tracker_class()(params, "synth")
    trk.network.load_state_dict({k: v for k, v in sd.items()}, strict=True)
    trk.network.set_compute_dtype(torch.float32)  # the fp32 HIP path: the 1e-3 bar of north_star
    trk.core._plan = trk.core._graph = None
    return trk, sd


def _seq(n, H=360, W=480):
    """n RGB / TIR frame pairs of a textured square drifting over a textured background."""
    rng = np.random.default_rng(11)
    bg_v, bg_i = _frame(H, W, 21), _frame(H, W, 22)
    obj = rng.integers(0, 256, (48, 48, 3), dtype=np.uint8)
    frames = []
    for f in range(n):
        x, y = 200 + 4 * f, 150 + 3 * f
        fv, fi = bg_v.copy(), bg_i.copy()
        fv[y:y + 48, x:x + 48] = obj
        fi[y:y + 48, x:x + 48] = 255 - obj
        frames.append([fv, fi])
    return frames, [200.0, 150.0, 48.0, 48.0]


@pytest.mark.parametrize("variant,module,multimodal,kv_cache", [
    ("rgbt", "mixformer_vit_rgbt", False, True), ("rgbt", "mixformer_vit_rgbt", False, False),
    ("asym", "asymmetric_shared", True, True), ("asym", "asymmetric_shared", True, False),
    ("asym_ce", "asymmetric_shared_ce", True, False)])
def test_tracking_loop_matches_oracle(variant, module, multimodal, kv_cache):
    """Each frame: the HIP tracker's new box vs the oracle's tracking step started from the HIP
    tracker's previous box (teacher forcing, so bf16/fp32 rounding cannot compound).  kv_cache:
    template pass on template updates + search-only frames (the default) or the full forward."""
    from oracle.forward import forward as oracle_forward
    trk, sd = _tracker(variant, module)
    trk.core.kv_cache = kv_cache
    frames, init = _seq(5)
    lut = pp.jet_lut() if multimodal else None
    trk.initialize(frames[0], {"init_bbox": [init, init]})
    H, W = frames[0][0].shape[:2]

    def prep(im_pair, box, factor, sz):
        t = [pp.preprocess(im_pair[m], box, factor, sz, lut=lut if m == 1 else None) for m in range(2)]
        return [torch.from_numpy(x[0])[None] for x in t], t[0][2]

    tmpl, _ = prep(frames[0], init, 2.0, 128)
    online = list(tmpl)
    # templates on the device are bit-exact with the oracle's
    for m in range(2):
        assert torch.equal(trk.core.template[m].cpu(), tmpl[m])
    state = list(init)
    for f in range(1, len(frames)):
        srch, rf = prep(frames[f], state, 5.0, 320)
        out, _ = oracle_forward(sd, variant, tmpl, online, srch)
        ref = pp.track_update(out["pred_boxes"].view(4).numpy(), state, rf, H, W, 320)
        got = trk.track(frames[f], {})["target_bbox"]
        tol = 1e-3 * 320 / rf
        err = max(abs(a - b) for a, b in zip(got, ref))
        print("frame %d err %.3g px (tol %.3g)" % (f, err, tol))
        assert err <= tol, (f, got, ref)
        state = got
        if f % 3 == 0:  # update interval 3: the online template is re-cropped at the new box
            online, _ = prep(frames[f], state, 2.0, 128)
            for m in range(2):
                assert torch.equal(trk.core.online_template[m].cpu(), online[m])


@pytest.mark.parametrize("kv_cache", [True, False])
def test_online_score_tracking_loop_matches_oracle(kv_cache):
    """asymmetric_shared_online tracker (lib/test/tracker/asymmetric_shared_online.py:73-130): each frame
    the score head runs; a crop at the new box becomes the best online candidate when sigmoid(score) >
    0.5 and beats the best so far; every update interval the candidate becomes the online template and
    the candidate resets to the template (the reference's D6 read-before-assignment is started from the
    template).  Teacher-forced like the loop above: boxes within 1e-3 of the crop, scores within 1e-3,
    and the online template bit-exact with the oracle's choice after every update."""
    from oracle.forward import forward as oracle_forward
    trk, sd = _tracker("asym_online", "asymmetric_shared_online")
    # the synthetic weights score every frame sigmoid(-0.22) = 0.445; lift the last score bias so the
    # gate (> 0.5) opens and the candidate / update logic is exercised (same weights for the oracle)
    key = "score_branch.score_head.layers.2.bias"
    sd[key] = sd[key] + 0.25
    trk.network.load_state_dict(sd, strict=True)
    trk.core._plan = trk.core._graph = None
    trk.core.kv_cache = kv_cache
    frames, init = _seq(7)
    lut = pp.jet_lut()
    trk.initialize(frames[0], {"init_bbox": [init, init]})
    H, W = frames[0][0].shape[:2]

    def prep(im_pair, box, factor, sz):
        t = [pp.preprocess(im_pair[m], box, factor, sz, lut=lut if m == 1 else None) for m in range(2)]
        return [torch.from_numpy(x[0])[None] for x in t], t[0][2]

    tmpl, _ = prep(frames[0], init, 2.0, 128)
    online, cand, best = list(tmpl), list(tmpl), -1.0
    state = list(init)
    took = 0
    for f in range(1, len(frames)):
        srch, rf = prep(frames[f], state, 5.0, 320)
        out, _ = oracle_forward(sd, "asym_online", tmpl, online, srch, run_score_head=True)
        ref = pp.track_update(out["pred_boxes"].view(4).numpy(), state, rf, H, W, 320)
        ref_score = torch.sigmoid(out["pred_scores"].view(1)).item()
        got = trk.track(frames[f], {})["target_bbox"]
        score = torch.sigmoid(trk.core._ws["SC"].view(1)).item()
        err = max(abs(a - b) for a, b in zip(got, ref))
        print("frame %d err %.3g px, score %.4f (oracle %.4f)" % (f, err, score, ref_score))
        assert err <= 1e-3 * 320 / rf, (f, got, ref)
        assert abs(score - ref_score) <= 1e-3
        state = got
        if ref_score > 0.5 and ref_score > best:
            cand, _ = prep(frames[f], state, 2.0, 128)
            best = ref_score
            took += 1
        if f % 3 == 0:
            online, cand, best = cand, list(tmpl), -1.0
            for m in range(2):
                assert torch.equal(trk.core.online_template[m].cpu(), online[m])
    print("candidate crops taken:", took)


def test_weights_reloaded_mid_sequence():
    """The tracker's captured graphs point into the network's runtime: after load_state_dict mid
    sequence the next frame must re-plan on the new weights (not replay against freed memory).
    A tracker reloaded with weights W2 tracks exactly like a fresh tracker built on W2."""
    from mmt_amd import synthetic
    trk, sd = _tracker("rgbt", "mixformer_vit_rgbt")
    frames, init = _seq(4)
    keys = [(k, list(v.shape)) for k, v in sd.items()]
    sd2 = {k: torch.from_numpy(v) for k, v in synthetic.synth_state_dict(keys, seed=5).items()}
    trk.initialize(frames[0], {"init_bbox": [init, init]})
    trk.track(frames[1], {})
    state = list(trk.core.state.cpu().tolist())
    trk.network.load_state_dict(sd2, strict=True)
    trk.network.set_compute_dtype(torch.float32)
    got = [trk.track(frames[f], {})["target_bbox"] for f in (2, 3)]
    fresh, _ = _tracker("rgbt", "mixformer_vit_rgbt")
    fresh.network.load_state_dict(sd2, strict=True)
    fresh.network.set_compute_dtype(torch.float32)
    fresh.initialize(frames[0], {"init_bbox": [init, init]})
    fresh.core.state.copy_(torch.tensor(state, dtype=torch.float64))
    ref = [fresh.track(frames[f], {})["target_bbox"] for f in (2, 3)]
    for a, b in zip(got, ref):
        assert max(abs(x - y) for x, y in zip(a, b)) <= 1e-6, (got, ref)
