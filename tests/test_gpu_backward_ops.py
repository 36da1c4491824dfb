"""HIP backward kernels of the reference's native ops vs the oracle.

* mmt_ms_deform_attn_backward (through mmt_amd.functional.MSDeformAttnFunction) vs autograd of the
  oracle restatement (tests/test_oracle_backward.py pins it by a float64 numerical gradient check):
  float64 within 1e-10 of the largest gradient; float32 within 1e-4 (another summation order);
  at the reference's op-test shapes and at the bimodal encoder's training shape
  (N 2, 800 keys / queries, 8 heads x 64, 2 levels of 20x20, 4 points).  Heads of up to 64 channels
  take the deterministic grad_value gather (bitwise equal on repeat), wider ones the float atomics.
* mmt_prroi_pool_backward / _coor_backward (PrRoIPool2DFunction) vs the oracle's numpy
  restatement of prroi_pooling_gpu_impl.cu:214-378, fp32, within 1e-4 relative, including the
  score head's shape (768 channels, 20x20 map, 4x4 bins, scale 1)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _msda_case(N, Lq, M, D, shapes, P, dtype, seed=0):
    g = torch.Generator().manual_seed(seed)
    S = sum(h * w for h, w in shapes)
    L = len(shapes)
    starts = np.cumsum([0] + [h * w for h, w in shapes])[:-1].tolist()
    v = torch.rand(N, S, M, D, generator=g, dtype=torch.float64)
    loc = torch.rand(N, Lq, M, L, P, 2, generator=g, dtype=torch.float64) * 1.3 - 0.15  # some samples outside
    # grad_loc is discontinuous where h_im / w_im crosses an integer (the tap cell and the inside test
    # change): keep samples 1e-3 away from those points, so fp32 and fp64 take the same branches
    for lv, (h, wd) in enumerate(shapes):
        for k, ext in ((0, wd), (1, h)):
            im = loc[:, :, :, lv, :, k] * ext - 0.5
            fr = im - im.floor()
            loc[:, :, :, lv, :, k] += torch.where((fr < 1e-3) | (fr > 1 - 1e-3), 2e-3 / ext, 0.0)
    w = torch.rand(N, Lq, M, L, P, generator=g, dtype=torch.float64) + 1e-5
    w = w / w.sum((-1, -2), keepdim=True)
    go = torch.randn(N, Lq, M * D, generator=g, dtype=torch.float64)
    return [x.to(dtype) for x in (v, loc, w, go)], shapes, starts


@pytest.mark.parametrize("dtype,tol", [(torch.float64, 1e-10), (torch.float32, 1e-4)])
@pytest.mark.parametrize("N,Lq,M,D,shapes,P", [(1, 2, 2, 2, [(6, 4), (3, 2)], 2), (2, 7, 2, 71, [(6, 4), (3, 2)], 3),
                                               (1, 5, 3, 130, [(5, 5)], 4), (2, 800, 8, 64, [(20, 20), (20, 20)], 4)])
def test_msda_backward_matches_oracle(N, Lq, M, D, shapes, P, dtype, tol):
    from mmt_amd.functional import MSDeformAttnFunction
    from oracle.msda import ms_deform_attn_backward
    (v, loc, w, go), shapes, starts = _msda_case(N, Lq, M, D, shapes, P, dtype)
    ref = ms_deform_attn_backward(v.double(), shapes, starts, loc.double(), w.double(), go.double())
    vc, lc, wc = (x.cuda().requires_grad_(True) for x in (v, loc, w))
    sh = torch.tensor(shapes, dtype=torch.long, device="cuda")
    st = torch.tensor(starts, dtype=torch.long, device="cuda")
    out = MSDeformAttnFunction.apply(vc, sh, st, lc, wc, 64)
    out.backward(go.cuda())
    for got, want, nm in zip((vc.grad, lc.grad, wc.grad), ref, ("value", "loc", "attn")):
        scale = max(1.0, float(want.abs().max()))
        err = float((got.double().cpu() - want).abs().max()) / scale
        print("%s grad_%s err %.3g" % (dtype, nm, err))
        assert err <= tol, (nm, err)


@pytest.mark.parametrize("N,Lq,M,D,shapes,P", [(2, 400, 8, 64, [(20, 20), (20, 20)], 4), (1, 7, 2, 33, [(6, 4), (3, 2)], 3)])
def test_msda_backward_deterministic(N, Lq, M, D, shapes, P):
    """grad_value, grad_loc and grad_attn bitwise equal across repeats (no atomics for heads <= 64 channels);
    the training shape (400 unique bimodal queries, 1600 samples per head and level: two sample batches)."""
    from mmt_amd.functional import MSDeformAttnFunction
    (v, loc, w, go), shapes, starts = _msda_case(N, Lq, M, D, shapes, P, torch.float32, seed=3)
    sh = torch.tensor(shapes, dtype=torch.long, device="cuda")
    st = torch.tensor(starts, dtype=torch.long, device="cuda")
    grads = []
    for _ in range(3):
        vc, lc, wc = (x.cuda().requires_grad_(True) for x in (v, loc, w))
        MSDeformAttnFunction.apply(vc, sh, st, lc, wc, 64).backward(go.cuda())
        torch.cuda.synchronize()
        grads.append((vc.grad.clone(), lc.grad.clone(), wc.grad.clone()))
    for g in grads[1:]:
        assert all(torch.equal(a, b) for a, b in zip(grads[0], g))


@pytest.mark.parametrize("N,Lq,M,D,shapes,P", [(16, 400, 8, 64, [(20, 20), (20, 20)], 4),
                                              (2, 37, 3, 32, [(6, 5), (3, 7), (1, 1)], 3),
                                              (1, 512, 2, 64, [(32, 32)], 4)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_msda_backward_value_gathers_equal(N, Lq, M, D, shapes, P, dtype):
    """grad_value from the per-(n, m, level) gather (value_impl 2) equals the 64-pixel-chunk
    gather's (value_impl 1) bit for bit -- both sum each pixel's taps in (sample, tap) order -- and so do grad_loc /
    grad_attn; the auto choice (the plain entry) equals them too."""
    from mmt_amd import _lib as L_
    (v, loc, w, go), shp, starts = _msda_case(N, Lq, M, D, shapes, P, dtype, seed=5)
    v, loc, w, go = (x.cuda().contiguous() for x in (v, loc, w, go))
    sh = torch.tensor(shp, dtype=torch.long, device="cuda")
    st = torch.tensor(starts, dtype=torch.long, device="cuda")
    S = v.shape[1]
    dt = L_.MMT_F32 if dtype == torch.float32 else L_.MMT_F64
    outs = []
    for impl in (1, 2, None):
        gv, gl, ga = torch.empty_like(v), torch.empty_like(loc), torch.empty_like(w)
        args = (v.data_ptr(), sh.data_ptr(), st.data_ptr(), loc.data_ptr(), w.data_ptr(), go.data_ptr(), gv.data_ptr(),
                gl.data_ptr(), ga.data_ptr(), N, S, M, D, Lq, len(shapes), P)
        stream = torch.cuda.current_stream().cuda_stream
        if impl is None:
            L_.check(L_.LIB.mmt_ms_deform_attn_backward(*args, dt, stream), "auto")
        else:
            L_.check(L_.LIB.mmt_ms_deform_attn_backward_impl(*args, max(h * w_ for h, w_ in shp), impl, dt, stream),
                     "impl %d" % impl)
        torch.cuda.synchronize()
        outs.append((gv, gl, ga))
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)


def _msda_bwd_raw(v, sh, st, loc, w, go, shp, impl, dt):
    from mmt_amd import _lib as L_
    N, S, M, D = v.shape
    Lq, L, P = loc.shape[1], loc.shape[3], loc.shape[4]
    gv, gl, ga = torch.empty_like(v), torch.empty_like(loc), torch.empty_like(w)
    args = (v.data_ptr(), sh.data_ptr(), st.data_ptr(), loc.data_ptr(), w.data_ptr(), go.data_ptr(), gv.data_ptr(),
            gl.data_ptr(), ga.data_ptr(), N, S, M, D, Lq, L, P)
    L_.check(L_.LIB.mmt_ms_deform_attn_backward_impl(*args, max(h * w_ for h, w_ in shp), impl, dt,
                                                     torch.cuda.current_stream().cuda_stream), "impl %d" % impl)
    return gv, gl, ga


def test_msda_backward_collapsed_locations():
    """Every sample of a level on (almost) one point, so four pixels each receive all Lq x P = 1600 taps of a
    (batch, head, level): the gathers' stable bucket placement (the former one-thread insertion sort of
    each bucket was quadratic in its length here) keeps grad_value within 1e-4 of the oracle, both gathers bitwise
    equal, and the backward within 4x (+ 0.5 ms) of the same op on spread-out locations."""
    from mmt_amd import _lib as L_
    from oracle.msda import ms_deform_attn_backward
    N, Lq, M, D, shapes, P = 2, 400, 8, 64, [(20, 20), (20, 20)], 4
    (v, loc, w, go), shp, starts = _msda_case(N, Lq, M, D, shapes, P, torch.float32, seed=7)
    g = torch.Generator().manual_seed(11)
    spread = loc.clone()
    loc = 0.4737 + (torch.rand(loc.shape, generator=g) - 0.5) * 2e-3  # h_im, w_im in 8.95 .. 8.99: taps 8 / 9
    ref = ms_deform_attn_backward(v.double(), shp, starts, loc.double(), w.double(), go.double())
    v, loc, spread, w, go = (x.cuda().contiguous() for x in (v, loc, spread, w, go))
    sh = torch.tensor(shp, dtype=torch.long, device="cuda")
    st = torch.tensor(starts, dtype=torch.long, device="cuda")
    outs = [_msda_bwd_raw(v, sh, st, loc, w, go, shp, impl, L_.MMT_F32) for impl in (1, 2)]
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    for got, want, nm in zip(outs[1], ref, ("value", "loc", "attn")):
        err = float((got.double().cpu() - want).abs().max()) / max(1.0, float(want.abs().max()))
        assert err <= 1e-4, (nm, err)

    def timed(lc, impl):
        for _ in range(2):
            _msda_bwd_raw(v, sh, st, lc, w, go, shp, impl, L_.MMT_F32)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            _msda_bwd_raw(v, sh, st, lc, w, go, shp, impl, L_.MMT_F32)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / 5

    for impl in (1, 2):
        t_c, t_s = timed(loc, impl), timed(spread, impl)
        print("impl %d: collapsed %.3f ms, spread %.3f ms" % (impl, t_c, t_s))
        assert t_c <= 4 * t_s + 0.5, (impl, t_c, t_s)  # the sorted buckets took 14-42 ms here


def test_msda_backward_zero_for_skipped_samples():
    from mmt_amd.functional import MSDeformAttnFunction
    (v, loc, w, go), shapes, starts = _msda_case(1, 3, 2, 8, [(6, 4), (3, 2)], 2, torch.float32)
    loc[0, 1] = 1.6  # every sample of query 1 lies outside its map -> skipped by the forward
    vc, lc, wc = (x.cuda().requires_grad_(True) for x in (v, loc, w))
    out = MSDeformAttnFunction.apply(vc, torch.tensor(shapes, device="cuda"), torch.tensor(starts, device="cuda"),
                                     lc, wc, 64)
    assert float(out[0, 1].abs().max()) == 0.0
    out.backward(go.cuda())
    assert float(lc.grad[0, 1].abs().max()) == 0.0 and float(wc.grad[0, 1].abs().max()) == 0.0


def test_msda_rejects_non_contiguous():
    from mmt_amd.functional import MSDeformAttnFunction
    (v, loc, w, _), shapes, starts = _msda_case(1, 2, 2, 4, [(6, 4), (3, 2)], 2, torch.float32)
    vt = v.cuda().transpose(2, 3)
    with pytest.raises(RuntimeError):
        MSDeformAttnFunction.apply(vt, torch.tensor(shapes, device="cuda"), torch.tensor(starts, device="cuda"),
                                   loc.cuda(), w.cuda(), 64)


def _prroi_case(B, C, H, W, seed=0):
    rng = np.random.default_rng(seed)
    feats = rng.standard_normal((B, C, H, W)).astype(np.float32)
    rois = []
    for r in range(2 * B + 1):
        x0, y0 = rng.uniform(-1.5, W * 0.6), rng.uniform(-1.5, H * 0.6)
        rois.append([r % B, x0, y0, x0 + rng.uniform(0.0, W * 0.7), y0 + rng.uniform(0.0, H * 0.7)])
    rois.append([0, 2.0, 3.0, 2.0, 7.0])  # zero-width ROI: empty bins, zero gradients
    return feats, np.array(rois, dtype=np.float32)


@pytest.mark.parametrize("B,C,H,W,ph,scale", [(2, 5, 9, 8, 7, 0.5), (2, 16, 20, 20, 4, 1.0), (1, 768, 20, 20, 4, 1.0)])
def test_prroi_backward_matches_oracle(B, C, H, W, ph, scale):
    from mmt_amd.functional import prroi_pool2d
    from oracle.prroi import prroi_pool2d as ref_fwd, prroi_pool2d_backward, prroi_pool2d_coor_backward
    feats, rois = _prroi_case(B, C, H, W)
    g = np.random.default_rng(7).standard_normal((rois.shape[0], C, ph, ph)).astype(np.float32)
    fc = torch.from_numpy(feats).cuda().requires_grad_(True)
    rc = torch.from_numpy(rois).cuda().requires_grad_(True)
    out = prroi_pool2d(fc, rc, ph, ph, scale)
    ref_out = ref_fwd(feats, rois, ph, ph, scale)
    assert np.abs(out.detach().cpu().numpy() - ref_out).max() <= 1e-4 * max(1.0, np.abs(ref_out).max())
    out.backward(torch.from_numpy(g).cuda())
    gf_ref = prroi_pool2d_backward(feats.shape, rois, g, ph, ph, scale)
    gr_ref = prroi_pool2d_coor_backward(feats, rois, ref_out, g, ph, ph, scale)
    ef = np.abs(fc.grad.cpu().numpy() - gf_ref).max() / max(1.0, np.abs(gf_ref).max())
    er = np.abs(rc.grad.cpu().numpy() - gr_ref).max() / max(1.0, np.abs(gr_ref).max())
    print("prroi grad feat err %.3g roi err %.3g" % (ef, er))
    assert ef <= 1e-4 and er <= 1e-4, (ef, er)
    assert float(rc.grad[-1].abs().max()) == 0.0  # the zero-width ROI


def test_prroi_backward_non_fp32_and_strided_inputs():
    """Gradients reach leaves that are not fp32 / not contiguous (forward works on fp32 copies):
    returned in the inputs' dtypes and equal to the fp32 path's."""
    from mmt_amd.functional import prroi_pool2d
    feats, rois = _prroi_case(2, 8, 12, 12)
    g = torch.from_numpy(np.random.default_rng(3).standard_normal((rois.shape[0], 8, 4, 4)).astype(np.float32)).cuda()
    f32 = torch.from_numpy(feats).cuda().requires_grad_(True)
    r32 = torch.from_numpy(rois).cuda().requires_grad_(True)
    prroi_pool2d(f32, r32, 4, 4, 1.0).backward(g)
    f64 = torch.from_numpy(feats).double().cuda().requires_grad_(True)
    base = torch.from_numpy(np.ascontiguousarray(feats.transpose(0, 1, 3, 2))).cuda()
    ft = base.transpose(2, 3).requires_grad_(True)  # non-contiguous view
    r64 = torch.from_numpy(rois).double().cuda().requires_grad_(True)
    prroi_pool2d(f64, r64, 4, 4, 1.0).backward(g)
    prroi_pool2d(ft, r32.detach(), 4, 4, 1.0).backward(g)
    assert f64.grad is not None and f64.grad.dtype == torch.float64 and r64.grad.dtype == torch.float64
    assert torch.allclose(f64.grad.float(), f32.grad, atol=1e-6) and torch.allclose(r64.grad.float(), r32.grad, atol=1e-5)
    assert ft.grad is not None and torch.allclose(ft.grad, f32.grad, atol=1e-6)
