"""Tracker pre/post-processing oracle (oracle/preprocess.py) against the reference's own outputs
(tests/golden/tracker_geometry.npz, made by tests/golden/make_golden_tracker.py), plus
size-independent properties of the restated cv2 arithmetic (which cv2's absence leaves unpinned)."""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import preprocess as pp

G = np.load(os.path.join(GOLDEN, "tracker_geometry.npz"))


@pytest.mark.parametrize("bi", range(len(G["boxes"])))
@pytest.mark.parametrize("fi", range(2))
def test_padded_crop_matches_reference(bi, fi):
    crop = pp.padded_crop(G["im"], list(G["boxes"][bi]), float(G["factors"][fi]))
    assert list(crop.shape) == list(G["crop_shape_%d_%d" % (bi, fi)])
    if ("crop_%d_%d" % (bi, fi)) in G:
        np.testing.assert_array_equal(crop, G["crop_%d_%d" % (bi, fi)])
    assert hashlib.sha256(np.ascontiguousarray(crop).tobytes()).digest() == G["crop_sha256_%d_%d" % (bi, fi)].tobytes()


def test_track_update_matches_reference():
    H, W, ss = int(G["H"]), int(G["W"]), int(G["search_size"])
    for i in range(len(G["pred"])):
        st, rf = [float(v) for v in G["state"][i]], float(G["rf"][i])
        assert pp.scale_pred(G["pred"][i], rf, ss) == [float(v) for v in G["pred_box"][i]], i
        assert pp.map_back_clip([float(v) for v in G["pred_box"][i]], st, rf, H, W, ss) == \
            [float(v) for v in G["new_state"][i]], i


def test_resize_identity_and_constant():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (37, 37, 3), dtype=np.uint8)
    np.testing.assert_array_equal(pp.resize_linear_u8(img, 37), img)  # scale 1: exact copy
    for n, o in ((50, 128), (300, 128), (640, 320), (100, 37)):
        c = np.full((n, n, 3), 173, dtype=np.uint8)
        np.testing.assert_array_equal(pp.resize_linear_u8(c, o), np.full((o, o, 3), 173, dtype=np.uint8))


def test_resize_area_2x():
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (64, 64, 3), dtype=np.uint8)
    out = pp.resize_linear_u8(img, 32)
    ref = (img.astype(np.int64).reshape(32, 2, 32, 2, 3).sum((1, 3)) + 2) >> 2
    np.testing.assert_array_equal(out, ref.astype(np.uint8))


def test_resize_close_to_float_bilinear():
    """The fixed-point result is within 1 of the float bilinear (align_corners=False, edge clamp)."""
    import torch
    import torch.nn.functional as F
    rng = np.random.default_rng(2)
    for n, o in ((90, 128), (500, 320)):
        img = rng.integers(0, 256, (n, n, 3), dtype=np.uint8)
        out = pp.resize_linear_u8(img, o).astype(np.int64)
        t = torch.from_numpy(img).permute(2, 0, 1)[None].double()
        ref = F.interpolate(t, size=(o, o), mode="bilinear", align_corners=False)[0].permute(1, 2, 0).numpy()
        assert np.abs(out - ref).max() <= 1.0


def test_jet_lut_shape():
    lut = pp.jet_lut()
    assert lut.shape == (256, 3) and lut.dtype == np.uint8
    assert tuple(lut[0]) == (128, 0, 0) and tuple(lut[255]) == (0, 0, 128)  # dark blue -> dark red (BGR)
