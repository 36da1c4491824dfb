"""Pins of the oracle's backward restatements (CPU, test infrastructure): SURVEY §8(f) row 4.

* MSDA: a float64 numerical gradient check of the restated forward, as the reference's own
  ops/test.py (check_gradient_numerical, gradcheck over value / loc / attn) does for its CUDA op.
* PrRoIPool features: the forward is linear in the features, so the backward is its exact adjoint:
  <g, pool(f)> == <pool^T(g), f> for any g, f.
* PrRoIPool coordinates: central finite differences of the restated forward (the reference's
  test_prroi_pooling2d.py only checks shapes for this gradient).
Shapes follow the reference's op tests (two levels (6,4), (3,2); 7x7 / 2x2 pooling)."""
import numpy as np
import torch

SHAPES = [(6, 4), (3, 2)]
STARTS = [0, 24]


def _msda_inputs(N=1, Lq=2, M=2, D=3, P=2, seed=0):
    g = torch.Generator().manual_seed(seed)
    S = sum(h * w for h, w in SHAPES)
    L = len(SHAPES)
    v = torch.rand(N, S, M, D, generator=g, dtype=torch.float64) * 0.01
    loc = torch.rand(N, Lq, M, L, P, 2, generator=g, dtype=torch.float64) * 1.2 - 0.1  # some samples outside
    w = torch.rand(N, Lq, M, L, P, generator=g, dtype=torch.float64) + 1e-5
    w = w / w.sum(-1, keepdim=True).sum(-2, keepdim=True)
    return v, loc, w


def test_msda_oracle_gradcheck():
    from oracle.msda import ms_deform_attn
    v, loc, w = _msda_inputs()
    v.requires_grad_(True)
    loc.requires_grad_(True)
    w.requires_grad_(True)
    assert torch.autograd.gradcheck(lambda a, b, c: ms_deform_attn(a, SHAPES, STARTS, b, c), (v, loc, w),
                                    eps=1e-6, atol=1e-7, rtol=1e-4)


def test_msda_oracle_backward_zero_outside():
    """Samples the forward skips (outside (-1,H) x (-1,W)) get zero loc / attn gradients."""
    from oracle.msda import ms_deform_attn_backward
    v, loc, w = _msda_inputs(seed=3)
    loc[0, 0, 0, 0, 0] = torch.tensor([1.5, 0.5], dtype=torch.float64)  # w_im = 1.5*4 - .5 > W
    g = torch.ones(1, loc.shape[1], v.shape[2] * v.shape[3], dtype=torch.float64)
    _, gl, ga = ms_deform_attn_backward(v, SHAPES, STARTS, loc, w, g)
    assert float(gl[0, 0, 0, 0, 0].abs().sum()) == 0.0 and float(ga[0, 0, 0, 0, 0]) == 0.0


def _prroi_case(seed=0):
    rng = np.random.default_rng(seed)
    feats = rng.standard_normal((2, 3, 8, 9)).astype(np.float32)
    rois = np.array([[0, 1.3, 0.7, 6.2, 5.9], [1, 0.0, 0.0, 8.0, 7.5], [0, 2.5, 3.5, 2.5, 6.0],
                     [1, -1.2, 2.1, 4.4, 9.6]], dtype=np.float32)
    return feats, rois


def test_prroi_oracle_backward_is_adjoint():
    from oracle.prroi import prroi_pool2d, prroi_pool2d_backward
    feats, rois = _prroi_case()
    rng = np.random.default_rng(1)
    for ph, scale in ((2, 1.0), (7, 0.5)):
        g = rng.standard_normal((rois.shape[0], 3, ph, ph)).astype(np.float32)
        lhs = float(np.sum(g.astype(np.float64) * prroi_pool2d(feats, rois, ph, ph, scale)))
        gf = prroi_pool2d_backward(feats.shape, rois, g, ph, ph, scale)
        rhs = float(np.sum(gf.astype(np.float64) * feats))
        assert abs(lhs - rhs) <= 1e-4 * max(1.0, abs(lhs)), (lhs, rhs)


def test_prroi_oracle_coor_backward_finite_differences():
    from oracle.prroi import prroi_pool2d, prroi_pool2d_coor_backward
    feats, rois = _prroi_case(2)
    rois = rois[[0, 1, 3]]  # the zero-width ROI sits on a kink
    ph, scale = 3, 1.0
    g = np.random.default_rng(4).standard_normal((rois.shape[0], 3, ph, ph)).astype(np.float32)
    out = prroi_pool2d(feats, rois, ph, ph, scale)
    gr = prroi_pool2d_coor_backward(feats, rois, out, g, ph, ph, scale)
    assert np.all(gr[:, 0] == 0)
    eps = 1e-2
    for r in range(rois.shape[0]):
        for k in range(1, 5):
            rp, rm = rois.copy(), rois.copy()
            rp[r, k] += eps
            rm[r, k] -= eps
            fd = (np.sum(g[r] * prroi_pool2d(feats, rp, ph, ph, scale)[r], dtype=np.float64)
                  - np.sum(g[r] * prroi_pool2d(feats, rm, ph, ph, scale)[r], dtype=np.float64)) / (2 * eps)
            assert abs(fd - gr[r, k]) <= 2e-2 * max(1.0, abs(fd)), (r, k, fd, gr[r, k])
