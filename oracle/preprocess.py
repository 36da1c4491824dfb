"""Tracker pre/post-processing, CPU restatement (oracle; test infrastructure only).

Follows, per tracking step of the RGB-T trackers (lib/test/tracker/mixformer_vit_rgbt.py:75-106,
asymmetric_shared_online.py:76-101):
  sample_target            lib/train/data/processing_utils.py:15-77  crop box, zero padding
                           (cv2.copyMakeBorder BORDER_CONSTANT), cv2.resize(INTER_LINEAR)
  Preprocessor_wo_mask /   lib/test/tracker/tracker_utils.py:24-48   (cv2.applyColorMap JET on the
  Preprocessor_Multimodal  TIR crop), HWC uint8 -> CHW fp32, /255, -mean, /std (torch on the GPU)
  map_box_back + clip_box  mixformer_vit_rgbt.py:92-95, :124-131; lib/utils/box_ops.py:155-164

Pinning.  The crop geometry and padding (`padded_crop`) and the box post-processing
(`track_update`) are pinned by golden vectors produced by the reference's own sample_target (with
output_sz=None, cv2.copyMakeBorder stubbed by an exact numpy constant pad) and its own
map_box_back / clip_box (tests/golden/make_golden_tracker.py).  cv2 is absent from this image,
so the resize and the colour map are restated from OpenCV's published 8-bit arithmetic and are
PARITY UNPINNED against cv2 itself:
  - INTER_LINEAR (imgproc/src/resize.cpp): source coordinate (float)((d+0.5)*scale-0.5), floor,
    columns clamped with weight 2048 at the edges, rows clamped; 11-bit weights
    saturate_cast<short>(w*2048) (round half to even); horizontal pass in int; vertical pass as
    VResizeLinearVec_32s8u: ((h0>>4)*b0>>16) + ((h1>>4)*b1>>16), then (t+2)>>2, saturate.
  - exact 2x downscale: INTER_AREA fast path, (a+b+c+d+2)>>2.
  - applyColorMap on CV_8UC3: cvtColor BGR2GRAY (fixed point 1868/9617/4899, >>14), then the
    per-channel LUT; the JET table is built from the piecewise-linear jet formula (below).
The GPU kernels (csrc/preprocess.hip) must match this restatement bit for bit.
"""
import math

import numpy as np

MEAN = np.array([0.485, 0.456, 0.406], dtype=np.float32)
STD = np.array([0.229, 0.224, 0.225], dtype=np.float32)


def crop_geometry(box, factor):
    """processing_utils.py:28-48 (Python floats; round() is half-to-even)."""
    x, y, w, h = [float(v) for v in box]
    crop_sz = math.ceil(math.sqrt(w * h) * factor)
    if crop_sz < 1:
        raise Exception("Too small bounding box.")
    x1 = int(round(x + 0.5 * w - crop_sz * 0.5))
    y1 = int(round(y + 0.5 * h - crop_sz * 0.5))
    return x1, y1, crop_sz


def padded_crop(im, box, factor):
    """sample_target(..., output_sz=None)'s image: the crop with constant-0 padding, including the
    reference's x2_pad = max(x2 - W + 1, 0) (the last column / row is dropped when padding)."""
    H, W = im.shape[:2]
    x1, y1, crop = crop_geometry(box, factor)
    x2, y2 = x1 + crop, y1 + crop
    xlim = W - 1 if x2 >= W else W
    ylim = H - 1 if y2 >= H else H
    out = np.zeros((crop, crop, 3), dtype=np.uint8)
    ys = np.arange(y1, y2)
    xs = np.arange(x1, x2)
    vy = (ys >= 0) & (ys < ylim)
    vx = (xs >= 0) & (xs < xlim)
    if vy.any() and vx.any():
        out[np.ix_(vy, vx)] = im[ys[vy]][:, xs[vx]]
    return out


def _coef(v):
    return np.clip(np.rint(np.float32(v) * np.float32(2048.0)), -32768, 32767).astype(np.int64)


def resize_linear_u8(img, out_sz):
    """cv2.resize(img, (out_sz, out_sz)) for a square uint8 HxWx3 image (see module docstring)."""
    n = img.shape[0]
    assert img.shape[1] == n
    inv = float(out_sz) / n
    scale = 1.0 / inv
    iscale = int(round(scale))
    src = img.astype(np.int64)
    if iscale == 2 and abs(scale - iscale) < 2.220446049250313e-16:
        d = np.arange(out_sz)
        a = src[2 * d][:, 2 * d] + src[2 * d][:, 2 * d + 1] + src[2 * d + 1][:, 2 * d] + src[2 * d + 1][:, 2 * d + 1]
        return ((a + 2) >> 2).astype(np.uint8)
    d = np.arange(out_sz)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    fx = (f - s.astype(np.float32)).astype(np.float32)
    sx = s.copy()
    fx = np.where(sx < 0, np.float32(0), fx)
    sx = np.where(sx < 0, 0, sx)
    edge = sx >= n - 1
    fx = np.where(edge, np.float32(0), fx).astype(np.float32)
    sx = np.where(edge, n - 1, sx)
    sx1 = np.minimum(sx + 1, n - 1)
    a0, a1 = _coef(np.float32(1) - fx), _coef(fx)
    fy = (f - s.astype(np.float32)).astype(np.float32)
    b0, b1 = _coef(np.float32(1) - fy), _coef(fy)
    r0 = np.clip(s, 0, n - 1)
    r1 = np.clip(s + 1, 0, n - 1)
    hrow = src[:, sx, :] * a0[None, :, None] + src[:, sx1, :] * a1[None, :, None]  # [rows][out][3]
    h0 = hrow[r0]
    h1 = hrow[r1]
    t = (((h0 >> 4) * b0[:, None, None]) >> 16) + (((h1 >> 4) * b1[:, None, None]) >> 16)
    return np.clip((t + 2) >> 2, 0, 255).astype(np.uint8)


def sample_target(im, box, factor, out_sz):
    """(resized crop uint8, resize_factor) of processing_utils.sample_target."""
    x1, y1, crop = crop_geometry(box, factor)
    return resize_linear_u8(padded_crop(im, box, factor), out_sz), out_sz / crop


def jet_lut():
    """256 x 3 (B, G, R) uint8 JET table: r = clip(min(4x - 1.5, -4x + 4.5)), g = clip(min(4x - 0.5,
    -4x + 3.5)), b = clip(min(4x + 0.5, -4x + 2.5)), x = i / 255, scaled by 255 and rounded
    (the shape of OpenCV's COLORMAP_JET; its exact table is unpinned here, cv2 being absent)."""
    x = np.arange(256, dtype=np.float64) / 255.0
    r = np.clip(np.minimum(4 * x - 1.5, -4 * x + 4.5), 0, 1)
    g = np.clip(np.minimum(4 * x - 0.5, -4 * x + 3.5), 0, 1)
    b = np.clip(np.minimum(4 * x + 0.5, -4 * x + 2.5), 0, 1)
    lut = np.stack([b, g, r], 1).astype(np.float32) * np.float32(255.0)
    return np.clip(np.rint(lut), 0, 255).astype(np.uint8)


def apply_colormap(img, lut):
    """cv2.applyColorMap(img (H,W,3) uint8, lut): BGR2GRAY fixed point, then lut[gray][c]."""
    v = img.astype(np.int64)
    gray = (v[..., 0] * 1868 + v[..., 1] * 9617 + v[..., 2] * 4899 + (1 << 13)) >> 14
    return lut[gray]


def normalise(img):
    """Preprocessor.process: torch CUDA fp32, x / 255.0 (CPU scalar: x * (1/255)), - mean, / std."""
    inv = np.float32(1.0) / np.float32(255.0)
    t = img.astype(np.float32).transpose(2, 0, 1) * inv
    return ((t - MEAN[:, None, None]) / STD[:, None, None]).astype(np.float32)


def preprocess(im, box, factor, out_sz, lut=None):
    patch, rf = sample_target(im, box, factor, out_sz)
    if lut is not None:
        patch_c = apply_colormap(patch, lut)
    else:
        patch_c = patch
    return normalise(patch_c), patch, rf


def scale_pred(pred_cxcywh, resize_factor, search_size):
    """(pred_boxes.mean(0) * search_size / resize_factor).tolist() as torch computes it on the GPU:
    fp32, and an fp32 tensor divided by a Python float is x * (1 / float32(rf))
    (aten/src/ATen/native/cuda/BinaryDivTrueKernel.cu, CPU-scalar divisor)."""
    p = np.asarray(pred_cxcywh, dtype=np.float32).reshape(4)
    inv = np.float32(1.0) / np.float32(resize_factor)
    return [float(v) for v in (p * np.float32(search_size)) * inv]


def map_back_clip(pred_box, state, resize_factor, H, W, search_size, margin=10):
    """map_box_back (mixformer_vit_rgbt.py:124-131) then clip_box (box_ops.py:155-164), Python floats."""
    cx_prev, cy_prev = state[0] + 0.5 * state[2], state[1] + 0.5 * state[3]
    cx, cy, w, h = pred_box
    half_side = 0.5 * search_size / resize_factor
    cx_real = cx + (cx_prev - half_side)
    cy_real = cy + (cy_prev - half_side)
    x1, y1 = cx_real - 0.5 * w, cy_real - 0.5 * h
    x2, y2 = x1 + w, y1 + h
    x1 = min(max(0, x1), W - margin)
    x2 = min(max(margin, x2), W)
    y1 = min(max(0, y1), H - margin)
    y2 = min(max(margin, y2), H)
    return [float(x1), float(y1), float(max(margin, x2 - x1)), float(max(margin, y2 - y1))]


def track_update(pred_cxcywh, state, resize_factor, H, W, search_size, margin=10):
    return map_back_clip(scale_pred(pred_cxcywh, resize_factor, search_size), state, resize_factor, H, W,
                         search_size, margin)
