"""Multi-scale deformable attention forward, CPU restatement (oracle; test infrastructure only).

Restates the reference CUDA op, not its grid_sample debug path:
  ms_deformable_im2col_gpu_kernel  ops/src/cuda/ms_deform_im2col_cuda.cuh:237-299
      per (n, q, m, c): col = sum_l sum_p w * bilinear(V_l, h_im, w_im), accumulated l-outer,
      p-inner; h_im = loc_y * H - 0.5, w_im = loc_x * W - 0.5; a sample contributes only if
      -1 < h_im < H and -1 < w_im < W (:285-291)
  ms_deform_attn_im2col_bilinear   :33-84   four taps, each zero when outside the map
The reference's own pure-PyTorch core (ops/functions/ms_deform_attn_func.py:41-61) is the
same function via grid_sample(align_corners=False, padding zeros); the golden vectors are made
with that core and pin this restatement.

Backward (ms_deform_attn_backward, ms_deform_attn_cuda.cu:83-153; per-tap arithmetic
ms_deform_im2col_cuda.cuh:86-150 ms_deform_attn_col2im_bilinear): autograd of the restatement
above.  floor() has zero derivative, so d/dloc flows only through lh / lw, exactly the
reference's grad_h_weight / grad_w_weight sums scaled by H / W; taps outside the map and skipped
samples contribute zero, as the reference's zero-initialised gradients.  Pinned by a numerical
gradient check in float64 (the reference's ops/test.py check_gradient_numerical).
"""
import torch


def ms_deform_attn(value, spatial_shapes, level_start_index, sampling_locations, attention_weights):
    """value (N,S,M,D); spatial_shapes [(H,W)]*L; level_start_index [L];
    sampling_locations (N,Lq,M,L,P,2) as (x, y) in [0,1]; attention_weights (N,Lq,M,L,P)
    -> (N, Lq, M*D), same dtype as value."""
    N, S, M, D = value.shape
    _, Lq, _, L, P, _ = sampling_locations.shape
    dt = value.dtype
    out = torch.zeros(N, Lq, M, D, dtype=dt)
    n_idx = torch.arange(N).view(N, 1, 1).expand(N, Lq, M)
    m_idx = torch.arange(M).view(1, 1, M).expand(N, Lq, M)
    for l in range(L):
        H, W = int(spatial_shapes[l][0]), int(spatial_shapes[l][1])
        start = int(level_start_index[l])
        V = value[:, start:start + H * W].reshape(N, H, W, M, D)
        for p in range(P):
            lx = sampling_locations[:, :, :, l, p, 0]
            ly = sampling_locations[:, :, :, l, p, 1]
            w = attention_weights[:, :, :, l, p]
            h_im = ly * H - 0.5
            w_im = lx * W - 0.5
            inside = (h_im > -1) & (w_im > -1) & (h_im < H) & (w_im < W)
            h_low = torch.floor(h_im)
            w_low = torch.floor(w_im)
            lh = h_im - h_low
            lw = w_im - w_low
            hh = 1 - lh
            hw = 1 - lw
            h_low = h_low.long()
            w_low = w_low.long()
            h_high = h_low + 1
            w_high = w_low + 1

            def tap(hi, wi):
                ok = (hi >= 0) & (wi >= 0) & (hi <= H - 1) & (wi <= W - 1) & inside
                v = V[n_idx, hi.clamp(0, H - 1), wi.clamp(0, W - 1), m_idx]
                return v * ok.unsqueeze(-1).to(dt)

            v1 = tap(h_low, w_low)
            v2 = tap(h_low, w_high)
            v3 = tap(h_high, w_low)
            v4 = tap(h_high, w_high)
            w1 = (hh * hw).unsqueeze(-1)
            w2 = (hh * lw).unsqueeze(-1)
            w3 = (lh * hw).unsqueeze(-1)
            w4 = (lh * lw).unsqueeze(-1)
            val = w1 * v1 + w2 * v2 + w3 * v3 + w4 * v4
            out = out + torch.where(inside.unsqueeze(-1), val * w.unsqueeze(-1), torch.zeros((), dtype=dt))
    return out.reshape(N, Lq, M * D)


def ms_deform_attn_backward(value, spatial_shapes, level_start_index, sampling_locations, attention_weights,
                            grad_output):
    """-> (grad_value, grad_sampling_loc, grad_attn_weight), same shapes/dtypes as the inputs."""
    v = value.detach().clone().requires_grad_(True)
    loc = sampling_locations.detach().clone().requires_grad_(True)
    aw = attention_weights.detach().clone().requires_grad_(True)
    with torch.enable_grad():
        out = ms_deform_attn(v, spatial_shapes, level_start_index, loc, aw)
        gv, gl, ga = torch.autograd.grad(out, (v, loc, aw), grad_output)
    return gv, gl, ga
