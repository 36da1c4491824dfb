"""Candidate elimination (asymmetric_shared_ce) on the GPU.

* The selection kernels against the reference's own choices: for every elimination stage of the
  golden forward (tests/golden/make_golden_ce.py), the fp32 path's mean template->search attention
  (within 1e-5 relative) and its kept token indices, in the reference's sorted order (exact).
* End to end, fp32: boxes within 1e-3 of the golden vectors and every stage's selection identical.
* End to end, bf16: the selection is a discrete function of attention means whose cut gaps in the
  golden forward are 1e-4 .. 1e-3 relative, below bf16's resolution, so bf16 keeps a slightly different
  token set (overlap printed, >= 90 % required).  The bf16 arithmetic is checked on the bf16 path's
  own choices: the oracle replays them (ce_forced) and the boxes must agree within 1e-2.
* mmt_ce_select alone on fixed scores: the kept set and order equal torch.sort's (distinct values),
  and the identity start (gidx_in NULL).
* Attention with tok_pitch (the compacted rows of a stage) equals attention on the same rows packed."""
import ctypes
import json

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
_RT = {}


def _runtime(dtype, mask_count=None):
    key = (dtype, mask_count)
    if key not in _RT:
        from mmt_amd import synthetic
        from mmt_amd.runtime import MixFormerRGBTRuntime
        keys = json.load(open(GOLDEN + "/state_dict_asym_ce.json"))
        sd = {k: torch.from_numpy(v) for k, v in synthetic.synth_state_dict(keys).items()}
        _RT[key] = MixFormerRGBTRuntime(sd, "asym_ce", dtype=dtype, ce_mask_count=mask_count)
    return _RT[key]


def _inputs(B):
    from mmt_amd import synthetic
    t, o, s = synthetic.synth_inputs(B)
    return [x.cuda() for x in t], [x.cuda() for x in o], [x.cuda() for x in s]


@pytest.mark.parametrize("masked", [False, True])
@pytest.mark.parametrize("dname,tol", [("f32", 1e-3), ("bf16", 1e-2)])
@pytest.mark.parametrize("B", [1, 2])
def test_ce_model_matches_reference(B, dname, tol, masked):
    """masked: ce_template_mask = the training actor's CTR_POINT mask (generate_mask_cond,
    lib/utils/ce_utils.py:14-38, taken from the reference-made fixture): the elimination averages
    the attention of the 4 masked template queries per frame only."""
    gold = np.load(GOLDEN + "/model_asym_ce_%sb%d.npz" % ("mask_" if masked else "", B))
    mask = torch.from_numpy(gold["ce_template_mask"]) if masked else None
    rt = _runtime(torch.float32 if dname == "f32" else torch.bfloat16, 4 if masked else None)
    inputs = _inputs(B)
    box, _ = rt.forward(*inputs, ce_template_mask=None if mask is None else mask.cuda())
    torch.cuda.synchronize()
    err = np.abs(box.cpu().numpy() - gold["pred_boxes"].reshape(B, 4)).max()
    ws = rt.workspace(B)
    same, overlap, forced = [], [], []
    for k in range(3):
        pair = []
        for m, nm in enumerate(("v", "i")):
            ref = gold["ce%d_keep_%s" % (k, nm)]
            got = ws["CEG"][k].view(2, B, -1)[m, :, :ref.shape[1]].cpu().numpy()
            same.append(bool(np.array_equal(got, ref)))
            overlap.append(min(len(set(got[b]) & set(ref[b])) / ref.shape[1] for b in range(B)))
            pair.append(got)
        forced.append(tuple(pair))
    print("asym_ce B=%d %s box err vs reference %.3g, stages identical: %s, kept-set overlap %s"
          % (B, dname, err, same, ["%.3f" % x for x in overlap]))
    if dname == "bf16":
        from mmt_amd import synthetic
        from oracle.forward import forward as oracle_forward, state_dict_to_torch
        sd = state_dict_to_torch(synthetic.synth_state_dict(json.load(open(GOLDEN + "/state_dict_asym_ce.json"))))
        out, _ = oracle_forward(sd, "asym_ce", *[[x.cpu() for x in grp] for grp in inputs], ce_forced=forced,
                                ce_template_mask=mask)
        rerr = np.abs(box.cpu().numpy() - out["pred_boxes"].reshape(B, 4).numpy()).max()
        print("bf16 box err vs the oracle replaying the bf16 selections %.3g" % rerr)
        assert rerr <= tol, rerr
        assert min(overlap) >= 0.9, overlap
        return
    assert err <= tol, err
    maps = ws["MAPS"].cpu().numpy()
    for g, nm in enumerate(("score_map_tl", "score_map_br")):
        ref = gold[nm].reshape(B, -1)
        merr = np.abs(maps[g] - ref).max() / max(1.0, np.abs(ref).max())
        assert merr <= (1e-4 if dname == "f32" else 5e-2), merr
    if dname == "f32":
        assert all(same), same
        for k in range(3):
            ref = gold["ce%d_attn_mean" % k]
            n = ref.shape[1]  # 2 * the stage's search tokens; mmt_ce_select writes [Bm][2 * n_s] packed
            am = ws["CEM"][k].view(-1)[:B * n].view(B, n).cpu().numpy()
            aerr = np.abs(am - ref).max() / np.abs(ref).max()
            assert aerr <= 1e-5, (k, aerr)


def test_ce_module_accepts_actor_mask():
    """The module API as the actor calls it (actors/mixformer_rgbt.py:82-90): net(t, o, s,
    ce_template_mask=CTR_POINT mask, ce_keep_rate=...) in eval / no_grad equals the runtime's masked
    forward, an all-True mask equals no mask, and a mask with unequal per-frame counts is refused."""
    from mmt_amd import model as M
    from mmt_amd import synthetic
    net = M.build_asymmetric_shared_ce(M.hot_path_cfg(), train=False)
    keys = [(k, list(v.shape)) for k, v in net.state_dict().items()]
    net.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.synth_state_dict(keys).items()}, strict=True)
    net = net.cuda().eval().set_compute_dtype(torch.float32)
    gold = np.load(GOLDEN + "/model_asym_ce_mask_b2.npz")
    mask = torch.from_numpy(gold["ce_template_mask"]).cuda()
    t, o, s = _inputs(2)
    with torch.no_grad():
        out, _ = net(t, o, s, ce_template_mask=mask, ce_keep_rate=0.7)
        assert np.abs(out["pred_boxes"].cpu().numpy() - gold["pred_boxes"]).max() <= 1e-3
        full, _ = net(t, o, s, ce_template_mask=torch.ones(2, 256, dtype=torch.bool, device="cuda"))
        plain, _ = net(t, o, s)
        assert torch.equal(full["pred_boxes"], plain["pred_boxes"])
        bad = mask.clone()
        bad[0, 0] = True
        with pytest.raises(ValueError):
            net(t, o, s, ce_template_mask=bad)


def test_ce_select_matches_torch_sort():
    from mmt_amd._lib import LIB, check
    g = torch.Generator().manual_seed(3)
    Bm, k, ns, nparts, keep = 2, 300, 400, 5, 210
    part = torch.rand(Bm, nparts, 2 * k, generator=g).cuda()
    gin = torch.stack([torch.randperm(ns, generator=g).int() for _ in range(2 * Bm)]).cuda()
    gout = torch.full((2 * Bm, ns), -7, dtype=torch.int32, device="cuda")
    order = torch.full_like(gout, -7)
    mean = torch.empty(Bm, 2 * k, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    tot = part.cpu().double().sum(1)  # (mmt_ce_select overwrites each frame's first partial row with the sum)
    check(LIB.mmt_ce_select(part.data_ptr(), nparts, Bm, k, keep, ns, gin.data_ptr(), gout.data_ptr(), order.data_ptr(),
                            mean.data_ptr(), 0.5, st), "ce_select")
    torch.cuda.synchronize()
    for s in range(2 * Bm):
        m, b = s // Bm, s % Bm
        a = tot[b, m * k:(m + 1) * k]
        ref = torch.sort(a, descending=True)[1][:keep]
        assert torch.equal(order[s, :keep].cpu().long(), ref)
        assert torch.equal(gout[s, :keep].cpu(), gin[s].cpu()[ref])
    assert torch.allclose(mean.cpu().double(), 0.5 * tot, rtol=1e-6)
    check(LIB.mmt_ce_select(part.data_ptr(), nparts, Bm, k, keep, ns, None, gout.data_ptr(), order.data_ptr(),
                            None, 1.0, st), "ce_select")
    torch.cuda.synchronize()
    for s in range(2 * Bm):
        assert torch.equal(gout[s, :keep].cpu(), order[s, :keep].cpu())  # identity start


@pytest.mark.parametrize("impl", [0, 4, 8, 17, 21, 22])
def test_attention_token_pitch(impl):
    from mmt_amd._lib import LIB, AttnParams, MMT_BF16, check
    S, pitch, n_t, H = 2, 528, 128, 12
    ntok = n_t + 280
    C = 64 * H
    qkv = (torch.randn(S, pitch, 3 * C, generator=torch.Generator().manual_seed(2)) * 0.5).bfloat16().cuda()
    packed = qkv[:, :ntok].contiguous()

    def run(src, p_rows, pitch_arg):
        out = torch.full((S, p_rows, C), 3.0, device="cuda", dtype=torch.bfloat16)
        p = AttnParams()
        p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym = src.data_ptr(), out.data_ptr(), S, 1, ntok, n_t, C, H, 1
        p.scale, p.impl, p.tok_pitch = 0.125, impl, pitch_arg
        check(LIB.mmt_mam_attention(ctypes.byref(p), MMT_BF16, torch.cuda.current_stream().cuda_stream), "attn")
        torch.cuda.synchronize()
        return out
    a = run(qkv, pitch, pitch)
    b = run(packed, ntok, 0)
    assert torch.equal(a[:, :ntok], b) and bool((a[:, ntok:] == 3.0).all())
