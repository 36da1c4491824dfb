"""PrRoIPool2D forward, CPU restatement (oracle; test infrastructure only).

Follows external/PreciseRoIPooling/pytorch/prroi_pool/src/prroi_pooling_gpu_impl.cu:
  PrRoIPoolingGetData              :37-42   (zero outside the map)
  PrRoIPoolingMatCalculation       :71-106  (closed-form integral of the bilinear surface over
                                             one cell, four corner terms, fp32)
  PrRoIPoolingForward              :149-212 (bin windows, floor/ceil cell range, w-outer /
                                             h-inner accumulation, divide by bin area, 0 for an
                                             empty bin)
  PrRoIPoolingBackward             :214-270 (MatDistributeDiff :108-147: the same four corner
                                             terms, scattered with top_diff / bin area)
  PrRoIPoolingCoorBackward         :272-378 (SingleCoorIntegral / Interpolation :44-69, early
                                             return on a zero top_diff)
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


def _bins(roi, scale, PH, PW):
    x0s, y0s, x1s, y1s = (roi[1] * scale, roi[2] * scale, roi[3] * scale, roi[4] * scale)
    bin_h = max(y1s - y0s, f32(0.0)) / f32(PH)
    bin_w = max(x1s - x0s, f32(0.0)) / f32(PW)
    for ph in range(PH):
        for pw in range(PW):
            ws = x0s + bin_w * f32(pw)
            hs = y0s + bin_h * f32(ph)
            yield ph, pw, ws, hs, ws + bin_w, hs + bin_h, max(f32(0.0), bin_w * bin_h)


def prroi_pool2d_backward(features_shape, rois, grad_out, pooled_height, pooled_width, spatial_scale):
    """d loss / d features (N,C,H,W) for grad_out (R,C,PH,PW) (PrRoIPoolingBackward)."""
    N, C, H, W = features_shape
    rois = np.asarray(rois, dtype=np.float32)
    g = np.asarray(grad_out, dtype=np.float32)
    PH, PW = int(pooled_height), int(pooled_width)
    scale = f32(spatial_scale)
    gf = np.zeros((N, C, H, W), dtype=np.float32)

    def dist(n, top, h, w, coeff):
        if 0 <= h < H and 0 <= w < W:
            gf[n, :, h, w] += top * coeff

    for r in range(rois.shape[0]):
        n = int(rois[r, 0])
        for ph, pw, ws, hs, we, he, win in _bins(rois[r], scale, PH, PW):
            top = np.zeros(C, np.float32) if win == 0 else g[r, :, ph, pw] / win
            for wi in range(math.floor(ws), math.ceil(we)):
                for hi in range(math.floor(hs), math.ceil(he)):
                    y0, x0 = max(hs, f32(hi)), max(ws, f32(wi))
                    y1, x1 = min(he, f32(hi + 1)), min(we, f32(wi + 1))
                    dist(n, top, hi, wi, _term(x0 - f32(wi), y0 - f32(hi), x1 - f32(wi), y1 - f32(hi)))
                    dist(n, top, hi, wi + 1, _term(f32(wi + 1) - x1, y0 - f32(hi), f32(wi + 1) - x0, y1 - f32(hi)))
                    dist(n, top, hi + 1, wi, _term(x0 - f32(wi), f32(hi + 1) - y1, x1 - f32(wi), f32(hi + 1) - y0))
                    dist(n, top, hi + 1, wi + 1,
                         _term(f32(wi + 1) - x1, f32(hi + 1) - y1, f32(wi + 1) - x0, f32(hi + 1) - y0))
    return gf


def _interp(data, h, w, H, W):
    h1, w1 = math.floor(h), math.floor(w)
    r = np.zeros(data.shape[0], np.float32)
    for hh, ww in ((h1, w1), (h1 + 1, w1), (h1, w1 + 1), (h1 + 1, w1 + 1)):
        r = r + _get(data, hh, ww, H, W) * ((f32(1) - abs(f32(h) - f32(hh))) * (f32(1) - abs(f32(w) - f32(ww))))
    return r


def _coor_int(s, t, c1, c2):
    return f32(0.5) * (t * t - s * s) * c2 + (t - f32(0.5) * t * t - s + f32(0.5) * s * s) * c1


def prroi_pool2d_coor_backward(features, rois, out, grad_out, pooled_height, pooled_width, spatial_scale):
    """d loss / d rois (R,5) (PrRoIPoolingCoorBackward); column 0 (batch index) is 0."""
    feats = np.asarray(features, dtype=np.float32)
    rois = np.asarray(rois, dtype=np.float32)
    out = np.asarray(out, dtype=np.float32)
    g = np.asarray(grad_out, dtype=np.float32)
    N, C, H, W = feats.shape
    PH, PW = int(pooled_height), int(pooled_width)
    scale = f32(spatial_scale)
    gr = np.zeros((rois.shape[0], 5), dtype=np.float64)
    for r in range(rois.shape[0]):
        data = feats[int(rois[r, 0])]
        for ph, pw, ws, hs, we, he, win in _bins(rois[r], scale, PH, PW):
            if win == 0:
                continue
            go = g[r, :, ph, pw]
            live = (go / win) != 0
            gx1 = gx2 = gy1 = gy2 = np.zeros(C, np.float32)
            for hi in range(math.floor(hs), math.ceil(he)):
                a, b = max(hs, f32(hi)) - f32(hi), min(he, f32(hi + 1)) - f32(hi)
                gx1 = gx1 + _coor_int(a, b, _interp(data, hi, ws, H, W), _interp(data, hi + 1, ws, H, W))
                gx2 = gx2 + _coor_int(a, b, _interp(data, hi, we, H, W), _interp(data, hi + 1, we, H, W))
            for wi in range(math.floor(ws), math.ceil(we)):
                a, b = max(ws, f32(wi)) - f32(wi), min(we, f32(wi + 1)) - f32(wi)
                gy1 = gy1 + _coor_int(a, b, _interp(data, hs, wi, H, W), _interp(data, hs, wi + 1, H, W))
                gy2 = gy2 + _coor_int(a, b, _interp(data, he, wi, H, W), _interp(data, he, wi + 1, H, W))
            top = out[r, :, ph, pw]
            px1 = (-gx1 + (he - hs) * top) / win * scale
            py1 = (-gy1 + (we - ws) * top) / win * scale
            px2 = (gx2 - (he - hs) * top) / win * scale
            py2 = (gy2 - (we - ws) * top) / win * scale
            fw0, fw1 = f32(pw) / f32(PW), f32(pw + 1) / f32(PW)
            fh0, fh1 = f32(ph) / f32(PH), f32(ph + 1) / f32(PH)
            gr[r, 1] += np.sum(((px1 * (1 - fw0) + px2 * (1 - fw1)) * go)[live])
            gr[r, 2] += np.sum(((py1 * (1 - fh0) + py2 * (1 - fh1)) * go)[live])
            gr[r, 3] += np.sum(((px2 * fw1 + px1 * fw0) * go)[live])
            gr[r, 4] += np.sum(((py2 * fh1 + py1 * fh0) * go)[live])
    return gr.astype(np.float32)
