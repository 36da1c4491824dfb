"""Template K/V cache: the template pass once + search passes per frame must
reproduce the full forward (reference semantics: the RGB MixFormer's set_online / forward_test,
lib/models/mixformer_vit/mixformer.py:308-323, exact because template queries never attend search
keys, mixformer.py:61-76).

Bars: boxes vs the reference golden vectors within the north_star tolerances (1e-3 fp32, 1e-2
bf16), and the cached path vs the full path on the same inputs within the same tolerance (the
kernels are the same; only GEMM tile / split choices for the smaller row counts can change the fp32
summation order).  The kernel-level pieces are checked bit for bit: the attention's query parts
write exactly the full launch's rows of that part and nothing else, and the GEMM output row map
stores exactly the unmapped GEMM's rows."""
import ctypes
import json

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _runtime(variant, dtype):
    from mmt_amd import synthetic
    from mmt_amd.runtime import MixFormerRGBTRuntime
    keys = json.load(open(GOLDEN + "/state_dict_%s.json" % variant))
    sd = {k: torch.from_numpy(v) for k, v in synthetic.synth_state_dict(keys).items()}
    return MixFormerRGBTRuntime(sd, variant, dtype=dtype)


def _inputs(B, seed=None):
    from mmt_amd import synthetic
    t, o, s = synthetic.synth_inputs(B) if seed is None else synthetic.synth_inputs(B, seed=seed)
    return [x.cuda() for x in t], [x.cuda() for x in o], [x.cuda() for x in s]


@pytest.mark.parametrize("dname,tol", [("f32", 1e-3), ("bf16", 1e-2)])
@pytest.mark.parametrize("variant,B", [("rgbt", 1), ("shared", 2), ("asym", 1), ("asym_online", 1)])
def test_cached_forward_matches_full_and_golden(variant, B, dname, tol):
    dtype = torch.float32 if dname == "f32" else torch.bfloat16
    rt = _runtime(variant, dtype)
    t, o, s = _inputs(B)
    score = variant == "asym_online"
    box_full, sc_full = rt.forward(t, o, s, run_score_head=score)
    box_full, sc_full = box_full.clone(), (sc_full.clone() if score else None)
    rt.set_template(t, o)
    box, sc = rt.forward_search(s, run_score_head=score)
    torch.cuda.synchronize()
    gold = np.load(GOLDEN + "/model_%s_b%d.npz" % (variant, B))
    err_g = np.abs(box.cpu().numpy() - gold["pred_boxes"].reshape(B, 4)).max()
    err_f = (box - box_full).abs().max().item()
    print("%s B=%d %s: cached vs golden %.3g, vs full %.3g" % (variant, B, dname, err_g, err_f))
    assert err_g <= tol and err_f <= tol
    if score:
        assert np.abs(sc.cpu().numpy() - gold["pred_scores"].reshape(B)).max() <= tol * max(
            1.0, np.abs(gold["pred_scores"]).max())
        assert (sc - sc_full).abs().max().item() <= tol


@pytest.mark.parametrize("variant", ["rgbt", "asym"])
def test_cache_reused_across_frames(variant):
    """One template pass, several search frames: each equals the full forward of that frame."""
    rt = _runtime(variant, torch.bfloat16)
    t, o, _ = _inputs(1)
    rt.set_template(t, o)
    for seed in (11, 12, 13):
        _, _, s = _inputs(1, seed=seed)
        box, _ = rt.forward_search(s)
        box = box.clone()
        ref, _ = rt.forward(t, o, s)  # full forward overwrites the cache's template rows identically
        torch.cuda.synchronize()
        assert (box - ref).abs().max().item() <= 1e-2
        rt.set_template(t, o)


def test_model_set_online_forward_test():
    from mmt_amd import synthetic
    from mmt_amd.model import build_mixformer_vit_rgbt, hot_path_cfg
    keys = json.load(open(GOLDEN + "/state_dict_rgbt.json"))
    model = build_mixformer_vit_rgbt(hot_path_cfg(), train=False)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.synth_state_dict(keys).items()})
    model = model.cuda().eval()
    t, o, s = _inputs(1)
    with torch.no_grad():
        full, _ = model(t, o, s)
        model.set_online(t, o)
        out, coord = model.forward_test(s)
    assert (out["pred_boxes"] - full["pred_boxes"]).abs().max().item() <= 1e-2
    with pytest.raises(RuntimeError):
        model.forward_test([x.repeat(2, 1, 1, 1) for x in s])  # batch differs from set_online's


@pytest.mark.parametrize("impl", [0, 4, 8, 17, 21, 22])
@pytest.mark.parametrize("asym", [0, 1])
def test_attention_query_parts_bit_exact(impl, asym):
    from mmt_amd._lib import LIB, AttnParams, MMT_BF16, check
    S, ntok, n_t, H = 2, 528, 128, 12
    C = 64 * H
    qkv = (torch.randn(S, ntok, 3 * C, generator=torch.Generator().manual_seed(5)) * 0.5).bfloat16().cuda()

    def run(part):
        out = torch.full((S, ntok, C), 7.0, device="cuda", dtype=torch.bfloat16)
        p = AttnParams()
        p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym = qkv.data_ptr(), out.data_ptr(), S, 1, ntok, n_t, C, H, asym
        p.scale, p.impl, p.q_part = 0.125, impl, part
        check(LIB.mmt_mam_attention(ctypes.byref(p), MMT_BF16, torch.cuda.current_stream().cuda_stream), "attn")
        torch.cuda.synchronize()
        return out
    full, tp, sp = run(0), run(1), run(2)
    assert torch.equal(tp[:, :n_t], full[:, :n_t]) and bool((tp[:, n_t:] == 7.0).all())
    assert torch.equal(sp[:, n_t:], full[:, n_t:]) and bool((sp[:, :n_t] == 7.0).all())
    # compact outputs of the cache passes (out_pitch / out_q0): the part's rows back to back per sequence
    for part, rows, q0 in ((1, n_t, 0), (2, ntok - n_t, n_t)):
        out = torch.full((S, rows + 3, C), 7.0, device="cuda", dtype=torch.bfloat16)  # 3 guard rows per sequence
        p = AttnParams()
        p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym = qkv.data_ptr(), out.data_ptr(), S, 1, ntok, n_t, C, H, asym
        p.scale, p.impl, p.q_part, p.out_pitch, p.out_q0 = 0.125, impl, part, rows + 3, q0
        check(LIB.mmt_mam_attention(ctypes.byref(p), MMT_BF16, torch.cuda.current_stream().cuda_stream), "attn")
        torch.cuda.synchronize()
        assert torch.equal(out[:, :rows], full[:, q0:q0 + rows]), part
        assert bool((out[:, rows:] == 7.0).all()), part


@pytest.mark.parametrize("ln_fold", [0, 1])
def test_gemm_output_row_map(ln_fold):
    """c_seg_rows / c_seg_pitch: GEMM over the search rows of a [S][ntok] stream == the same rows of
    the GEMM over all rows (residual read through the map too); other rows untouched."""
    from mmt_amd._lib import LIB, GemmParams, MMT_BF16, check
    S, ntok, n_t, K, N = 2, 528, 128, 768, 768
    ns = ntok - n_t
    g = torch.Generator().manual_seed(9)
    a = torch.randn(S * ntok, K, generator=g).bfloat16().cuda()
    w = (torch.randn(N, K, generator=g) * K ** -0.5).bfloat16().cuda()
    bias = torch.randn(N, generator=g).cuda()
    res = torch.randn(S * ntok, N, generator=g).cuda()
    colsum = w.float().sum(1).contiguous()

    def run(rows, off, pitch):
        c = torch.full((S * ntok, N), 3.0, device="cuda")
        p = GemmParams()
        p.a[0], p.w[0], p.c[0] = a.data_ptr() + off * K * 2, w.data_ptr(), c.data_ptr() + off * N * 4
        p.bias[0], p.r[0] = bias.data_ptr(), res.data_ptr() + off * N * 4
        p.lda, p.ldc, p.ldr = K, N, N
        p.a_seg_rows, p.a_segs_a, p.a_stride_a = rows, 1 << 30, ntok * K
        p.M, p.N, p.K, p.groups, p.c_f32 = S * rows, N, K, 1, 1
        if pitch:
            p.c_seg_rows, p.c_seg_pitch = rows, pitch
        if ln_fold:
            p.ln_fold, p.ln_eps, p.ln_colsum[0] = 1, 1e-6, colsum.data_ptr()
        p.splitk = 1
        check(LIB.mmt_gemm(ctypes.byref(p), MMT_BF16, torch.cuda.current_stream().cuda_stream), "gemm")
        torch.cuda.synchronize()
        return c.view(S, ntok, N)
    full = run(ntok, 0, 0)
    part = run(ns, n_t, ntok)
    assert bool((part[:, :n_t] == 3.0).all())
    err = (part[:, n_t:] - full[:, n_t:]).abs().max().item()
    assert err <= 1e-4 * full.abs().max().item(), err
