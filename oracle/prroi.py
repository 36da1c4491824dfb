"""PrRoIPool2D forward, CPU restatement (oracle; test infrastructure only).

Follows external/PreciseRoIPooling/pytorch/prroi_pool/src/prroi_pooling_gpu_impl.cu:
  PrRoIPoolingGetData              :37-42   (zero outside the map)
  PrRoIPoolingMatCalculation       :71-106  (closed-form integral of the bilinear surface over
                                             one cell, four corner terms, fp32)
  PrRoIPoolingForward              :149-212 (bin windows, floor/ceil cell range, w-outer /
                                             h-inner accumulation, divide by bin area, 0 for an
                                             empty bin)
All arithmetic is float32, in the kernel's order, vectorised over channels only.
"""
import math

import numpy as np

f32 = np.float32


def _get(data, h, w, height, width):
    if h < 0 or w < 0 or h >= height or w >= width:
        return np.zeros(data.shape[0], dtype=np.float32)
    return data[:, h, w]


def _term(alpha, beta, lim_alpha, lim_beta):
    half = f32(0.5)
    return (lim_alpha - half * lim_alpha * lim_alpha - alpha + half * alpha * alpha) * (
        lim_beta - half * lim_beta * lim_beta - beta + half * beta * beta
    )


def _mat(data, s_h, s_w, e_h, e_w, y0, x0, y1, x1, h0, w0):
    s = np.zeros(data.shape[0], dtype=np.float32)
    alpha = x0 - f32(s_w)
    beta = y0 - f32(s_h)
    lim_alpha = x1 - f32(s_w)
    lim_beta = y1 - f32(s_h)
    s = s + _get(data, s_h, s_w, h0, w0) * _term(alpha, beta, lim_alpha, lim_beta)
    alpha = f32(e_w) - x1
    lim_alpha = f32(e_w) - x0
    s = s + _get(data, s_h, e_w, h0, w0) * _term(alpha, beta, lim_alpha, lim_beta)
    alpha = x0 - f32(s_w)
    beta = f32(e_h) - y1
    lim_alpha = x1 - f32(s_w)
    lim_beta = f32(e_h) - y0
    s = s + _get(data, e_h, s_w, h0, w0) * _term(alpha, beta, lim_alpha, lim_beta)
    alpha = f32(e_w) - x1
    lim_alpha = f32(e_w) - x0
    s = s + _get(data, e_h, e_w, h0, w0) * _term(alpha, beta, lim_alpha, lim_beta)
    return s


def prroi_pool2d(features, rois, pooled_height, pooled_width, spatial_scale):
    """features (N,C,H,W) float32, rois (R,5) [batch_idx, x0, y0, x1, y1] -> (R,C,PH,PW)."""
    feats = np.ascontiguousarray(np.asarray(features, dtype=np.float32))
    rois = np.asarray(rois, dtype=np.float32)
    N, C, H, W = feats.shape
    R = rois.shape[0]
    PH, PW = int(pooled_height), int(pooled_width)
    scale = f32(spatial_scale)
    out = np.zeros((R, C, PH, PW), dtype=np.float32)
    for r in range(R):
        n = int(rois[r, 0])
        data = feats[n]
        x0s = rois[r, 1] * scale
        y0s = rois[r, 2] * scale
        x1s = rois[r, 3] * scale
        y1s = rois[r, 4] * scale
        roi_w = max(x1s - x0s, f32(0.0))
        roi_h = max(y1s - y0s, f32(0.0))
        bin_h = roi_h / f32(PH)
        bin_w = roi_w / f32(PW)
        for ph in range(PH):
            for pw in range(PW):
                ws = x0s + bin_w * f32(pw)
                hs = y0s + bin_h * f32(ph)
                we = ws + bin_w
                he = hs + bin_h
                win = max(f32(0.0), bin_w * bin_h)
                if win == 0:
                    continue
                s_w, e_w = math.floor(ws), math.ceil(we)
                s_h, e_h = math.floor(hs), math.ceil(he)
                acc = np.zeros(C, dtype=np.float32)
                for wi in range(s_w, e_w):
                    for hi in range(s_h, e_h):
                        acc = acc + _mat(
                            data, hi, wi, hi + 1, wi + 1,
                            max(hs, f32(hi)), max(ws, f32(wi)),
                            min(he, f32(hi + 1)), min(we, f32(wi + 1)),
                            H, W,
                        )
                out[r, :, ph, pw] = acc / win
    return out
