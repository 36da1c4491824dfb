"""GPU parity of the training-step kernels with torch fp32 autograd on the same
bf16-rounded inputs: the MAM attention forward's log-sum-exp output and its backward
(mmt_mam_attention_bwd), the bf16 transpose, and the HIP Linear autograd Function.

Bars (bf16 operands, fp32 accumulation): attention dQ/dK/dV within 2e-2 of the largest gradient
magnitude; the backward is deterministic (bitwise equal on repeat)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

LOG2E = 1.4426950408889634


def _lib():
    from mmt_amd import _lib
    return _lib


def _attn_ref(q, k, v, n_t):
    """MAM (mixformer.py:52-78): template queries -> template keys, search queries -> all keys."""
    d = q.shape[-1]
    sc = d ** -0.5
    ot = torch.softmax(q[:, :, :n_t] @ k[:, :, :n_t].transpose(-1, -2) * sc, -1) @ v[:, :, :n_t]
    os_ = torch.softmax(q[:, :, n_t:] @ k.transpose(-1, -2) * sc, -1) @ v
    return torch.cat([ot, os_], 2)


def _run_fwd_bwd(qkv, dout, S, ntok, n_t, H, impl=0):
    L = _lib()
    C = 64 * H
    out = torch.empty(S, ntok, C, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(S, H, ntok, device="cuda")
    p = L.AttnParams()
    p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym = qkv.data_ptr(), out.data_ptr(), S, S // 2, ntok, n_t, C, H, 0
    p.scale, p.impl, p.lse = 0.125, impl, lse.data_ptr()
    L.check(L.LIB.mmt_mam_attention(p, L.MMT_BF16, torch.cuda.current_stream().cuda_stream), "attn fwd")
    delta = torch.empty(S, H, ntok, device="cuda")
    dqkv = torch.empty(S, ntok, 3 * C, device="cuda", dtype=torch.bfloat16)
    b = L.AttnBwdParams()
    b.qkv, b.out, b.dout, b.lse, b.delta, b.dqkv = qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(), \
        delta.data_ptr(), dqkv.data_ptr()
    b.S, b.Bm, b.ntok, b.n_t, b.C, b.H, b.asym, b.scale = S, S // 2, ntok, n_t, C, H, 0, 0.125
    L.check(L.LIB.mmt_mam_attention_bwd(b, L.MMT_BF16, torch.cuda.current_stream().cuda_stream), "attn bwd")
    torch.cuda.synchronize()
    return out, lse, dqkv


@pytest.mark.parametrize("impl", [0, 8, 21])
@pytest.mark.parametrize("S,ntok,n_t,H", [(2, 528, 128, 12), (4, 100, 36, 2), (2, 70, 8, 1), (2, 864, 288, 2)])
def test_attention_backward(S, ntok, n_t, H, impl):
    """The training forward with log-sum-exp (impl 8: running maximum; 21: range-checked exponent, lse = log2 of
    its row sums, the auto choice on training-size grids) and the deterministic backward against fp32 autograd."""
    C = 64 * H
    g = torch.Generator().manual_seed(ntok + H)
    qkv = torch.randn(S, ntok, 3 * C, generator=g).bfloat16()
    dout = torch.randn(S, ntok, C, generator=g).bfloat16()
    out, lse, dqkv = _run_fwd_bwd(qkv.cuda(), dout.cuda(), S, ntok, n_t, H, impl)
    # reference: fp32 autograd on the same bf16 inputs (q rounded as the kernels see it)
    x = qkv.float().view(S, ntok, 3, H, 64).permute(2, 0, 3, 1, 4)
    q = x[0].clone().requires_grad_(True)
    k = x[1].clone().requires_grad_(True)
    v = x[2].clone().requires_grad_(True)
    o = _attn_ref(q, k, v, n_t)
    o.backward(dout.float().view(S, ntok, H, 64).permute(0, 2, 1, 3))
    o_ref = o.detach().permute(0, 2, 1, 3).reshape(S, ntok, C)
    assert (out.float().cpu() - o_ref).abs().max().item() <= 2e-2
    # lse: log2-sum-exp2 of q' k, q' = bf16(q * scale * log2 e)
    qs = (x[0] * 0.125 * LOG2E).bfloat16().float()
    s2 = qs @ x[1].transpose(-1, -2)
    mask = torch.zeros(ntok, ntok, dtype=torch.bool)
    mask[:n_t, n_t:] = True
    lse_ref = torch.logsumexp(s2.masked_fill(mask, float("-inf")) / LOG2E, -1) * LOG2E
    assert (lse.cpu() - lse_ref).abs().max().item() <= 2e-2
    grads = torch.stack([q.grad, k.grad, v.grad]).permute(1, 3, 0, 2, 4).reshape(S, ntok, 3 * C)
    got = dqkv.float().cpu()
    for i, nm in enumerate("qkv"):
        gr, gg = grads[..., i * C:(i + 1) * C], got[..., i * C:(i + 1) * C]
        err = (gg - gr).abs().max().item() / gr.abs().max().item()
        print("d%s rel err %.3g" % (nm, err))
        assert err <= 2e-2, (nm, err)


def test_attention_backward_deterministic():
    S, ntok, n_t, H = 4, 528, 128, 4
    g = torch.Generator().manual_seed(3)
    qkv = torch.randn(S, ntok, 3 * 64 * H, generator=g).bfloat16().cuda()
    dout = torch.randn(S, ntok, 64 * H, generator=g).bfloat16().cuda()
    a = _run_fwd_bwd(qkv, dout, S, ntok, n_t, H)
    b = _run_fwd_bwd(qkv, dout, S, ntok, n_t, H)
    assert all(torch.equal(x, y) for x, y in zip(a, b))


@pytest.mark.parametrize("rows,cols", [(64, 64), (528, 768), (1056, 2304), (37, 200), (300, 13)])
def test_transpose_bf16_bit_exact(rows, cols):
    from mmt_amd.train import _transpose
    x = torch.randn(rows, cols, generator=torch.Generator().manual_seed(rows * cols)).bfloat16().cuda()
    y = _transpose(x, rows, cols)
    torch.cuda.synchronize()
    assert torch.equal(y.cpu(), x.cpu().t().contiguous())
    # the dW GEMM's padded operand in one launch: zero padding columns up to ld_out (fill 1) and the
    # appended ones row block (fill 2), written into poisoned memory
    ld = (rows + 7) // 8 * 8 + 8
    for ones in (False, True):
        poison = torch.full(((cols + 8) * ld,), float("nan"), device="cuda").bfloat16()
        del poison  # the allocator hands these NaN bytes to the output below: every element must be written
        yp = _transpose(x, rows, cols, ld, ones_row=ones)
        torch.cuda.synchronize()
        ref = torch.zeros(cols + (8 if ones else 0), ld, dtype=torch.bfloat16)
        ref[:cols, :rows] = x.cpu().t()
        if ones:
            ref[cols, :rows] = 1.0
        assert torch.equal(yp.cpu(), ref), ones


@pytest.mark.parametrize("M,N,K", [(1056, 2304, 768), (1056, 768, 3072), (130, 96, 768)])
def test_hip_linear_autograd(M, N, K):
    """_HipLinear (bf16 operands, fp32 accumulation) against fp32 autograd on the same bf16 values."""
    from mmt_amd.train import HipOps
    g = torch.Generator().manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g).bfloat16()
    w = (torch.randn(N, K, generator=g) * K ** -0.5)
    b = torch.randn(N, generator=g)
    dy = torch.randn(M, N, generator=g).bfloat16()
    xg = x.cuda().requires_grad_(True)
    wg, bg = w.cuda().requires_grad_(True), b.cuda().requires_grad_(True)
    y = HipOps.linear(xg, wg, bg)
    y.backward(dy.cuda())
    xr = x.float().requires_grad_(True)
    wr, br = w.bfloat16().float().requires_grad_(True), b.clone().requires_grad_(True)
    yr = torch.nn.functional.linear(xr, wr, br)
    yr.backward(dy.float())
    for got, ref, nm in ((y, yr, "y"), (xg.grad, xr.grad, "dx"), (wg.grad, wr.grad, "dw"), (bg.grad, br.grad, "db")):
        err = (got.float().cpu() - ref.detach()).abs().max().item() / ref.detach().abs().max().item()
        print("%s rel err %.3g" % (nm, err))
        assert err <= 1e-2, (nm, err)


class _TorchBf16Ops:
    """Same bf16 roundings as HipOps, PyTorch-ROCm ops (hipBLASLt GEMMs, fp32 softmax): measures
    how far bf16 alone moves the gradients from fp32, so the HIP path is held to that bar."""

    dtype = torch.bfloat16

    @staticmethod
    def linear(x, weight, bias, out_f32=False):
        y = torch.nn.functional.linear(x.bfloat16(), weight.bfloat16(), bias.bfloat16())
        return y.float() if out_f32 else y

    @staticmethod
    def mam_attention(qkv, n_t, heads):
        import sys
        import os
        sys.path.insert(0, os.path.dirname(__file__))
        from test_train import TorchOps
        return TorchOps.mam_attention(qkv.float(), n_t, heads).bfloat16()

    @staticmethod
    def mam_attention_asym(qkv, Bh, n_t, heads):
        from mmt_amd.train import asym_attention_from_mam
        return asym_attention_from_mam(_TorchBf16Ops.mam_attention, qkv, Bh, n_t, heads)

    @staticmethod
    def ms_deform_attn(value, hw, loc, aw):
        import sys
        import os
        sys.path.insert(0, os.path.dirname(__file__))
        from test_train import TorchOps
        return TorchOps.ms_deform_attn(value, hw, loc, aw)


def test_train_step_gpu_matches_fp32_grads():
    """One two-stream training step at the bench shapes (128/320, B=2): HIP backbone ops in bf16 vs
    the fp32 stand-in on the CPU.  Loss within 2e-2; each parameter group's gradient within
    max(5e-2, 1.5 x the PyTorch-bf16 path's own distance from fp32) (relative L2); then a few steps
    on the fixed batch lower the loss."""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(__file__))
    from test_train import TorchOps
    from mmt_amd.model import build_mixformer_vit_rgbt, hot_path_cfg
    from mmt_amd.train import HipOps, TrainStep, synthetic_batch
    torch.manual_seed(0)
    net = build_mixformer_vit_rgbt(hot_path_cfg(), train=False)
    with torch.no_grad():
        for br in ("tl", "br"):
            getattr(net.box_head, "conv5_" + br).weight.mul_(30.0)
    net.eval()
    batch = synthetic_batch(2, "cpu", torch.Generator().manual_seed(7))
    ref_step = TrainStep(net, TorchOps)
    ref_stats = ref_step.backward(*batch)
    ref_grads = {n: p.grad.clone() for n, p in net.named_parameters() if p.grad is not None}
    net.cuda()
    gb = [[x.cuda() for x in batch[i]] for i in range(3)] + [batch[3].cuda()]
    tb_stats = TrainStep(net, _TorchBf16Ops).backward(*gb)
    tb_grads = {n: p.grad.float().cpu() for n, p in net.named_parameters() if p.grad is not None}
    step = TrainStep(net, HipOps)
    stats = step.backward(*gb)
    torch.cuda.synchronize()
    print("loss hip %.5f torch-bf16 %.5f fp32 %.5f" % (stats["loss"].item(), tb_stats["loss"].item(),
                                                      ref_stats["loss"].item()))
    assert abs(stats["loss"].item() - ref_stats["loss"].item()) <= 2e-2
    params = dict(net.named_parameters())
    bad = []
    for grp in ("backbone_v", "backbone_i", "fusion_vi", "box_head"):
        names = [n for n in ref_grads if n.startswith(grp)]
        ref = torch.cat([ref_grads[n].flatten() for n in names])
        got = torch.cat([params[n].grad.float().cpu().flatten() for n in names])
        tb = torch.cat([tb_grads[n].flatten() for n in names])
        rel, rel_tb = ((got - ref).norm() / ref.norm()).item(), ((tb - ref).norm() / ref.norm()).item()
        print("%s grad rel L2: hip %.3g, torch-bf16 %.3g" % (grp, rel, rel_tb))
        if rel > max(5e-2, 1.5 * rel_tb):
            bad.append((grp, rel, rel_tb))
    assert not bad, bad
    step.apply()
    losses = [step(*gb)["loss"].item() for _ in range(4)]
    print("losses", losses)
    assert losses[-1] < stats["loss"].item(), losses


def test_score_train_step_matches_oracle_grads():
    """TRAIN_SCORE stage on the online-score model: the frozen trunk on the HIP runtime (fp32), the
    score decoder with autograd over the HIP PrRoIPool.  Logits and every score-branch gradient
    vs autograd through the oracle's ScoreDecoder restatement on the CPU (same trunk outputs):
    within 1e-3 (relative L2); only "score" parameters receive gradients; AdamW steps lower the loss."""
    import json
    from conftest import GOLDEN
    from mmt_amd import synthetic
    from mmt_amd.model import build_asymmetric_shared_online_score, hot_path_cfg
    from mmt_amd.runtime import MixFormerRGBTRuntime
    from mmt_amd.train import ScoreTrainStep
    from oracle.forward import score_decoder
    keys = json.load(open(GOLDEN + "/state_dict_asym_online.json"))
    sd = {k: torch.from_numpy(v) for k, v in synthetic.synth_state_dict(keys).items()}
    net = build_asymmetric_shared_online_score(hot_path_cfg(), train=False)
    net.load_state_dict(sd, strict=True)
    net = net.cuda().eval()
    rt = MixFormerRGBTRuntime(sd, "asym_online", dtype=torch.float32)
    step = ScoreTrainStep(net, rt)
    B = 3
    t, o, s = synthetic.synth_inputs(B)
    t, o, s = [x.cuda() for x in t], [x.cuda() for x in o], [x.cuda() for x in s]
    labels = torch.tensor([1.0, 0.0, 1.0], device="cuda")
    stats = step.backward(t, o, s, labels)
    fused, templ, xyxy = step.trunk(t, o, s)
    leaf = {k: v.detach().cpu().float().requires_grad_(k.startswith("score_branch.")) for k, v in
            net.state_dict().items() if k.startswith("score_branch.")}
    ref = score_decoder(leaf, "score_branch.", fused.cpu(), templ.cpu(), xyxy.cpu(), num_heads=fused.shape[1] // 64)
    loss = torch.nn.functional.binary_cross_entropy_with_logits(ref.view(-1), labels.cpu())
    loss.backward()
    serr = (stats["scores"].cpu() - ref.view(-1).detach()).abs().max().item()
    print("score logits err %.3g, loss hip %.6f oracle %.6f" % (serr, stats["loss"].item(), loss.item()))
    assert serr <= 1e-3 and abs(stats["loss"].item() - loss.item()) <= 1e-4
    named = dict(net.named_parameters())
    for n, p in named.items():
        if "score" not in n:
            assert p.grad is None, n
    # proj_k biases get mathematically zero gradients (softmax is shift-invariant): measure each
    # gradient against max(its own norm, 1e-4 x the largest one) so rounding noise there is not a ratio
    gmax = max(v.grad.norm().item() for v in leaf.values() if v.grad is not None)
    for k, v in leaf.items():
        if v.grad is None:
            continue
        got = named[k].grad.float().cpu()
        rel = ((got - v.grad).norm() / max(v.grad.norm().item(), 1e-4 * gmax)).item()
        assert rel <= 1e-3, (k, rel)
    step.apply()
    losses = [step(t, o, s, labels)["loss"].item() for _ in range(5)]
    print("score losses", stats["loss"].item(), losses)
    assert losses[-1] < stats["loss"].item()


@pytest.mark.gpu
@pytest.mark.parametrize("variant,B", [("rgbt", 2), ("shared", 2), ("asym", 2), ("rgbt", 16)])
def test_module_forward_training_gpu_grads(variant, B):
    """The drop-in module itself in train() mode (boundary b2: what the reference actor and DDP call,
    actors/mixformer_rgbt.py:82-98): net(t, o, s, gt_bboxes=...) on the HIP ops (bf16) at the bench
    shapes, B = 2 (head BatchNorms in eval mode) and B = 16 (the config-4 batch, BatchNorms in train mode:
    batch statistics on the HIP batch norm).  Box loss within 2e-2 of the fp32 stand-in on the CPU, each
    parameter group's gradient within max(3e-2, 1.2 x the PyTorch-bf16 path's distance from fp32) (relative
    L2).  Round 6: the corner head's output convs x6 (the golden fixtures' gain) instead of x30, whose peaked
    score maps put torch-bf16 itself 22 % from fp32 (tools/grad_fixture_probe.py, profiles/r06_grad_fixture_probe.jsonl:
    x6 -> 8-9 %, x2 -> 6-8 %; the floor is the train-mode BatchNorm's batch statistics at B = 16), and a
    negative control at B = 16: every two-stream Linear weight gradient scaled by 0.9 (mmt_amd.train._weight_grads2)
    must fail the same check."""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(__file__))
    from test_train import TorchOps
    import mmt_amd.model as M
    import mmt_amd.train as T
    from mmt_amd.train import box_loss, synthetic_batch
    builders = {"rgbt": M.build_mixformer_vit_rgbt, "shared": M.build_mixformer_vit_rgbt_shared,
                "asym": M.build_asymmetric_shared}
    torch.manual_seed(0)
    net = builders[variant](M.hot_path_cfg(), train=False)
    with torch.no_grad():
        for br in ("tl", "br"):
            getattr(net.box_head, "conv5_" + br).weight.mul_(6.0)
        # The deformable encoder's default init (zero offset weights, integer grid bias) samples exactly on pixel
        # centres, where the bilinear location gradient is discontinuous: an ulp of difference anywhere upstream
        # then flips the branch and moves the gradients ~0.65 (relative L2) in either direction (DESIGN.md §7,
        # round 5).  A third of a pixel off the centres keeps the comparison well-conditioned.
        for m in net.modules():
            if hasattr(m, "sampling_offsets"):
                m.sampling_offsets.bias.add_(1.0 / 3.0)
    net.train()
    net.drop_path_rate = 0.0
    for m in net.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
        if isinstance(m, torch.nn.BatchNorm2d) and B == 2:
            m.eval()
    t, o, s, gt = synthetic_batch(B, "cpu", torch.Generator().manual_seed(7))

    def run(ops, dev):
        net.zero_grad(set_to_none=True)
        net.train_ops = ops
        args = [[x.to(dev) for x in z] for z in (t, o, s)]
        _, coord = net(*args, gt_bboxes=None)
        loss, _ = box_loss(coord, gt.to(dev))
        loss.backward()
        return loss.item(), {n: p.grad.float().cpu().clone() for n, p in net.named_parameters() if p.grad is not None}

    ref_loss, ref = run(TorchOps, "cpu")
    net.cuda()
    tb_loss, tb = run(_TorchBf16Ops, "cuda")
    hip_loss, hip = run(None, "cuda")  # None = HipOps, the product path
    print("%s loss hip %.5f torch-bf16 %.5f fp32 %.5f" % (variant, hip_loss, tb_loss, ref_loss))
    assert abs(hip_loss - ref_loss) <= 2e-2
    groups = ("backbone_v", "backbone_i", "fusion_vi", "box_head") if variant == "rgbt" else ("backbone", "fusion_vi", "box_head")

    def check(grads, tag):
        bad = []
        for grp in groups:
            names = [n for n in ref if n.startswith(grp + ".")]
            r = torch.cat([ref[n].flatten() for n in names])
            g = torch.cat([grads[n].flatten() for n in names])
            b = torch.cat([tb[n].flatten() for n in names])
            rel, rel_tb = ((g - r).norm() / r.norm()).item(), ((b - r).norm() / r.norm()).item()
            print("%s %s %s grad rel L2: %.3g, torch-bf16 %.3g" % (variant, tag, grp, rel, rel_tb))
            if rel > max(3e-2, 1.2 * rel_tb):
                bad.append((grp, rel, rel_tb))
        return bad

    bad = check(hip, "hip")
    assert not bad, bad
    if variant == "rgbt" and B == 16:  # negative control: a 10 % weight-gradient error is flagged
        orig = T._weight_grads2
        T._weight_grads2 = lambda *a, **k: [(dw * 0.9, db * 0.9) for dw, db in orig(*a, **k)]
        try:
            _, neg = run(None, "cuda")
        finally:
            T._weight_grads2 = orig
        assert check(neg, "dW x0.9"), "the perturbed weight gradients passed the check"


@pytest.mark.parametrize("max_norm", [0.0, 0.1, 1e6])
@pytest.mark.parametrize("set_to_none", [False, True])
def test_hip_adamw_matches_torch(max_norm, set_to_none):
    """mmt_adamw_grad_norm / mmt_adamw_step (mmt_amd.optim.HipAdamW) against
    torch.nn.utils.clip_grad_norm_ + torch.optim.AdamW(fused=True) over three parameter groups with their own
    lr / weight decay, tensor sizes below / across the 65536-element chunk and not multiples of 4,
    five steps: parameters and moments within 1e-6 relative per step, the norm within 1e-5, the
    gradients zeroed by the update, and the bf16 shadow equal to the bf16 cast of the new weights.
    set_to_none (the training step's mode): fresh gradient tensors every step (new addresses: the
    pointer table is refreshed), left untouched by the update."""
    from mmt_amd.optim import HipAdamW
    g = torch.Generator().manual_seed(3)
    shapes = [(7,), (768, 768), (3, 65537), (130001,), (12, 64)]
    init = [torch.randn(s, generator=g) for s in shapes]
    ref = [torch.nn.Parameter(t.clone().cuda()) for t in init]
    hip = [torch.nn.Parameter(t.clone().cuda()) for t in init]
    groups = lambda ps: [{"params": ps[:2], "lr": 1e-3}, {"params": ps[2:4], "lr": 2e-4, "weight_decay": 0.05},  # noqa: E731
                         {"params": ps[4:]}]
    opt_ref = torch.optim.AdamW(groups(ref), lr=5e-4, weight_decay=1e-4, fused=True)  # the form it replaces
    opt = HipAdamW(groups(hip), lr=5e-4, weight_decay=1e-4, shadow=[hip[1]], set_to_none=set_to_none)
    for step in range(5):
        grads = [torch.randn(s, generator=g).cuda() * (10.0 if step == 2 else 1.0) for s in shapes]
        opt_ref.zero_grad(set_to_none=True)
        opt.zero_grad(set_to_none=set_to_none)
        keep = [torch.empty(1 << 16, device="cuda") for _ in range(step)]  # moves the next allocations
        for p, q, gr in zip(ref, hip, grads):
            p.grad = gr.clone()
            if q.grad is None:
                q.grad = gr.clone()
            else:
                q.grad.add_(gr)  # accumulates into the zeroed gradient, as autograd does
        if max_norm > 0:
            n_ref = torch.nn.utils.clip_grad_norm_(ref, max_norm)
        opt_ref.step()
        opt.step(max_norm)
        torch.cuda.synchronize()
        if max_norm > 0:
            assert abs(opt.last_norm.item() - n_ref.item()) <= 1e-5 * n_ref.item()
        else:
            assert opt.last_norm is None
        del keep
        for k, (p, q) in enumerate(zip(ref, hip)):
            assert torch.allclose(q, p, rtol=1e-6, atol=1e-7), (step, (q - p).abs().max().item())
            m_r, v_r = opt_ref.state[p]["exp_avg"], opt_ref.state[p]["exp_avg_sq"]
            m_h, v_h = opt.state[q]["exp_avg"], opt.state[q]["exp_avg_sq"]
            assert torch.allclose(m_h, m_r, rtol=1e-5, atol=1e-7) and torch.allclose(v_h, v_r, rtol=1e-5, atol=1e-9)
            if set_to_none:
                assert torch.equal(q.grad, grads[k])
            else:
                assert int((q.grad != 0).sum()) == 0
        sh, ver = hip[1]._mmt_bf16
        assert ver == hip[1]._version and torch.equal(sh, hip[1].detach().to(torch.bfloat16))


def test_hip_adamw_state_dict_resume_and_scheduler():
    """HipAdamW is a torch.optim.Optimizer: a state_dict written by torch.optim.AdamW after
    three steps loads into it (moments + the shared step, so the bias corrections continue from t = 4, not
    t = 1), its own state_dict round-trips into torch.optim.AdamW, and an LR scheduler attached to it
    changes the lr the next update uses; two steps after the resume both optimizers agree within 1e-6."""
    from mmt_amd.optim import HipAdamW
    g = torch.Generator().manual_seed(5)
    shapes = [(300,), (64, 65)]
    init = [torch.randn(s, generator=g) for s in shapes]
    ref = [torch.nn.Parameter(t.clone().cuda()) for t in init]
    opt_ref = torch.optim.AdamW([{"params": ref, "lr": 1e-3}], weight_decay=0.01)
    sched_ref = torch.optim.lr_scheduler.StepLR(opt_ref, step_size=1, gamma=0.5)
    grads = [[torch.randn(s, generator=g).cuda() for s in shapes] for _ in range(5)]
    for k in range(3):
        for p, gr in zip(ref, grads[k]):
            p.grad = gr.clone()
        opt_ref.step()
        sched_ref.step()
    hip = [torch.nn.Parameter(p.detach().clone()) for p in ref]
    opt = HipAdamW([{"params": hip, "lr": 1e-3}], weight_decay=0.01, set_to_none=True)
    opt.load_state_dict(opt_ref.state_dict())
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=1, gamma=0.5)
    sched.load_state_dict(sched_ref.state_dict())
    assert opt.param_groups[0]["lr"] == opt_ref.param_groups[0]["lr"]
    for k in range(3, 5):
        for p, q, gr in zip(ref, hip, grads[k]):
            p.grad, q.grad = gr.clone(), gr.clone()
        opt_ref.step()
        sched_ref.step()
        opt.step()
        sched.step()
        torch.cuda.synchronize()
        for p, q in zip(ref, hip):
            assert torch.allclose(q, p, rtol=1e-6, atol=1e-7), (k, (q - p).abs().max().item())
    sd = opt.state_dict()
    assert all(float(st["step"]) == 5.0 for st in sd["state"].values())
    back = torch.optim.AdamW([{"params": [torch.nn.Parameter(p.detach().clone()) for p in hip], "lr": 1e-3}],
                             weight_decay=0.01)
    back.load_state_dict(sd)
    for a, b in zip(back.state.values(), opt_ref.state.values()):
        assert torch.allclose(a["exp_avg"], b["exp_avg"], rtol=1e-5, atol=1e-6)  # fma vs torch's lerp


def test_hip_adamw_load_state_dict_with_missing_entries():
    """a torch.optim.AdamW state_dict saved before its first step (no per-parameter state)
    and one where a parameter never had a gradient both load into HipAdamW; the next steps run (zero
    moments for the missing entries) and match torch.optim.AdamW resumed from the same state_dict."""
    from mmt_amd.optim import HipAdamW
    g = torch.Generator().manual_seed(11)
    shapes = [(40,), (8, 9)]
    init = [torch.randn(s, generator=g) for s in shapes]
    grads = [[torch.randn(s, generator=g).cuda() for s in shapes] for _ in range(2)]
    # (a) empty state: both continue from t = 1
    ref = [torch.nn.Parameter(t.clone().cuda()) for t in init]
    opt_ref = torch.optim.AdamW(ref, lr=1e-3, weight_decay=0.01)
    hip = [torch.nn.Parameter(t.clone().cuda()) for t in init]
    opt = HipAdamW([{"params": hip, "lr": 1e-3}], weight_decay=0.01)
    opt.load_state_dict(opt_ref.state_dict())
    for k in range(2):
        for p, q, gr in zip(ref, hip, grads[k]):
            p.grad, q.grad = gr.clone(), gr.clone()
        opt_ref.step()
        opt.step()
    torch.cuda.synchronize()
    for p, q in zip(ref, hip):
        assert torch.allclose(q, p, rtol=1e-6, atol=1e-7)
    # (b) the second parameter never had a gradient: its moments start at zero, the step continues
    ref = [torch.nn.Parameter(t.clone().cuda()) for t in init]
    opt_ref = torch.optim.AdamW(ref, lr=1e-3, weight_decay=0.01)
    ref[0].grad = grads[0][0].clone()
    opt_ref.step()
    sd = opt_ref.state_dict()
    assert len(sd["state"]) == 1
    hip = [torch.nn.Parameter(p.detach().clone()) for p in ref]
    opt = HipAdamW([{"params": hip, "lr": 1e-3}], weight_decay=0.01)
    opt.load_state_dict(sd)
    assert all(torch.equal(opt.state[p]["exp_avg"], torch.zeros_like(p)) for p in hip[1:])
    for q, gr in zip(hip, grads[1]):
        q.grad = gr.clone()
    opt.step()
    torch.cuda.synchronize()
    assert all(torch.isfinite(q).all() for q in hip)
    for p, gr in zip(ref, grads[1]):
        p.grad = gr.clone()
    opt_ref.step()
    assert torch.allclose(hip[0], ref[0], rtol=1e-6, atol=1e-7)  # the parameter with state: same as torch



@pytest.mark.parametrize("C,rows,two,dyt", [(768, 1056, False, "bf16"), (768, 1000, True, "bf16"), (512, 77, True, "f32"),
                                            (1024, 300, False, "f32"), (256, 33, True, "bf16")])
def test_layernorm_backward_matches_autograd(C, rows, two, dyt):
    """mmt_layernorm_bwd (the training step's backbone LayerNorms) against torch fp32 autograd of
    F.layer_norm on the same input and output gradient: dx, and dgamma / dbeta of each row group
    (rows [0, rows0) -> norm 0, the rest -> norm 1), including a ragged last workgroup; bitwise
    repeatable (fixed-order partial sums) and accumulating into dgb on request."""
    L = _lib()
    g = torch.Generator().manual_seed(C + rows)
    x = torch.randn(rows, C, generator=g) * 3 + 0.5
    gam = torch.randn(2, C, generator=g)
    dt = {"bf16": torch.bfloat16, "f32": torch.float32}[dyt]
    dy = torch.randn(rows, C, generator=g).to(dt)
    rows0 = rows // 2 if two else rows
    xd, gd, dyd = x.cuda(), gam.cuda(), dy.cuda()
    outs = []
    for rep in range(2):
        dx = torch.empty(rows, C, device="cuda")
        dgb = torch.full((4 if two else 2, C), 1.0 if rep else 0.0, device="cuda")
        ws = torch.empty((rows + 31) // 32 * 4 * C, device="cuda")
        L.check(L.LIB.mmt_layernorm_bwd(xd.data_ptr(), dyd.data_ptr(), {"bf16": L.MMT_BF16, "f32": L.MMT_F32}[dyt],
                                        gd[0].data_ptr(), gd[1].data_ptr() if two else None, dx.data_ptr(),
                                        dgb.data_ptr(), rep, ws.data_ptr(), ws.numel(), rows, rows0, C, 1e-6,
                                        torch.cuda.current_stream().cuda_stream), "ln bwd")
        torch.cuda.synchronize()
        outs.append((dx.cpu(), dgb.cpu() - (1.0 if rep else 0.0)))
    assert torch.equal(outs[0][0], outs[1][0])
    assert (outs[0][1] - outs[1][1]).abs().max().item() <= 1e-6 * max(1.0, outs[0][1].abs().max().item())
    dx, dgb = outs[0]
    xr = x.clone().requires_grad_(True)
    # row groups alternate every rows0 rows (an odd row count puts the last row back in group 0)
    grp = (torch.arange(rows) // rows0) % 2 if two else torch.zeros(rows, dtype=torch.long)
    ws_ = [gam[h].clone().requires_grad_(True) for h in range(2)]
    bs_ = [torch.zeros(C, requires_grad=True) for _ in range(2)]
    ys = [torch.nn.functional.layer_norm(xr[grp == h], (C,), ws_[h], bs_[h], 1e-6) for h in range(2)]
    y = torch.zeros(rows, C).index_put((torch.nonzero(grp == 0).view(-1),), ys[0]) \
        .index_put((torch.nonzero(grp == 1).view(-1),), ys[1])
    y.backward(dy.float())
    assert (dx - xr.grad).abs().max().item() <= 2e-4 * max(1.0, xr.grad.abs().max().item())
    for i in range(2 if two else 1):
        w, bb = ws_[i], bs_[i]
        assert (dgb[2 * i] - w.grad).abs().max().item() <= 2e-4 * max(1.0, w.grad.abs().max().item())
        assert (dgb[2 * i + 1] - bb.grad).abs().max().item() <= 2e-4 * max(1.0, bb.grad.abs().max().item())


@pytest.mark.parametrize("two", [False, True])
def test_hip_layernorm_autograd(two):
    """HipOps.layer_norm (mmt_layernorm -> bf16, mmt_layernorm_bwd) as the training forward calls it
    (fp32 residual stream in, the next Linear's bf16 operand out) against aten's layer_norm + cast."""
    from mmt_amd.train import HipOps
    g = torch.Generator().manual_seed(3 + two)
    B, ntok, C = 4, 100, 768
    x = (torch.randn(B, ntok, C, generator=g) * 2).cuda()
    n = [torch.nn.LayerNorm(C, eps=1e-6).cuda() for _ in range(2)]
    for m in n:
        with torch.no_grad():
            m.weight.copy_(torch.randn(C, generator=g).cuda())
            m.bias.copy_(torch.randn(C, generator=g).cuda())
    dy = torch.randn(B, ntok, C, generator=g).cuda().bfloat16()
    xa = x.clone().requires_grad_(True)
    ya = HipOps.layer_norm(xa, n[0].weight, n[0].bias, 1e-6, n[1].weight if two else None, n[1].bias if two else None)
    assert ya.dtype == torch.bfloat16 and ya.shape == x.shape
    ya.backward(dy)
    ga = [xa.grad] + [p.grad.clone() for m in (n if two else n[:1]) for p in (m.weight, m.bias)]
    for m in n:
        m.weight.grad = m.bias.grad = None
    xb = x.clone().requires_grad_(True)
    if two:
        yb = torch.cat([n[0](xb[:B // 2]), n[1](xb[B // 2:])]).bfloat16()
    else:
        yb = n[0](xb).bfloat16()
    assert (ya.float() - yb.float()).abs().max().item() <= 3e-2
    yb.backward(dy)
    gb = [xb.grad] + [p.grad for m in (n if two else n[:1]) for p in (m.weight, m.bias)]
    for a, b in zip(ga, gb):
        assert (a - b).abs().max().item() <= 1e-3 * max(1.0, b.abs().max().item())


@pytest.mark.parametrize("two", [False, True])
def test_hip_layernorm_pass_through_gradient(two):
    """HipOps.layer_norm_pass (_HipLayerNormPass): the LayerNorm output and x handed through for the residual
    op, as a pre-LN block uses them (y = x + f(LN(x))); the two gradients of x are summed inside the LayerNorm
    backward kernel (mmt_layernorm_bwd_add).  Equal to HipOps.layer_norm with autograd's separate add up to
    one rounding (the kernel may contract the last multiply into the add), the parameters' gradients identical."""
    from mmt_amd.train import HipOps
    g = torch.Generator().manual_seed(5 + two)
    B, ntok, C = 4, 100, 768
    x = (torch.randn(B, ntok, C, generator=g) * 2).cuda()
    n = [torch.nn.LayerNorm(C, eps=1e-6).cuda() for _ in range(2)]
    for m in n:
        with torch.no_grad():
            m.weight.copy_(torch.randn(C, generator=g).cuda())
            m.bias.copy_(torch.randn(C, generator=g).cuda())
    wq = torch.randn(C, C, generator=g).cuda() / C ** 0.5
    dy = torch.randn(B, ntok, C, generator=g).cuda()
    args = (n[0].weight, n[0].bias, 1e-6, n[1].weight if two else None, n[1].bias if two else None)
    grads = []
    for fused in (True, False):
        for m in n:
            m.weight.grad = m.bias.grad = None
        xa = x.clone().requires_grad_(True)
        if fused:
            xn, xr = HipOps.layer_norm_pass(xa, *args)
        else:
            xn, xr = HipOps.layer_norm(xa, *args), xa
        y = xr * 0.5 + (xn.float() @ wq)  # a residual consumer of the pass-through and a LayerNorm consumer
        y.backward(dy)
        grads.append([xa.grad] + [p.grad.clone() for m in (n if two else n[:1]) for p in (m.weight, m.bias)])
    dxa, dxb = grads[0][0], grads[1][0]
    assert (dxa - dxb).abs().max().item() <= 1e-6 * dxb.abs().max().item()
    for a, b in zip(grads[0][1:], grads[1][1:]):
        assert torch.equal(a, b)


def test_hip_mlp_autograd():
    """HipOps.mlp (_HipMlp: fc1 with the GELU epilogue storing its pre-activation, fc2, and a backward
    whose fc2 dX GEMM applies GELU' in its epilogue) against the same MLP as torch fp32 autograd on the
    bf16-rounded operands (timm Mlp, mixformer.py:136-139): output and every gradient."""
    from mmt_amd.train import HipOps
    g = torch.Generator().manual_seed(17)
    M, C, F4 = 1056, 768, 3072
    x = torch.randn(M, C, generator=g).bfloat16()
    w1 = torch.randn(F4, C, generator=g) / math.sqrt(C)
    b1 = torch.randn(F4, generator=g) * 0.1
    w2 = torch.randn(C, F4, generator=g) / math.sqrt(F4)
    b2 = torch.randn(C, generator=g) * 0.1
    dy = torch.randn(M, C, generator=g)
    ps = [t.cuda().requires_grad_(True) for t in (w1, b1, w2, b2)]
    xa = x.cuda().requires_grad_(True)
    y = HipOps.mlp(xa, *ps)
    assert y.dtype == torch.float32
    y.backward(dy.cuda())
    got = [y.detach().cpu(), xa.grad.float().cpu()] + [p.grad.cpu() for p in ps]
    # reference: fp32 math on the bf16 operands the kernels read (x, bf16 weights, bf16 h / pre-activation)
    xr = x.float().requires_grad_(True)
    rs = [w1.bfloat16().float().requires_grad_(True), b1.clone().requires_grad_(True),
          w2.bfloat16().float().requires_grad_(True), b2.clone().requires_grad_(True)]
    yr = torch.nn.functional.linear(torch.nn.functional.gelu(torch.nn.functional.linear(xr, rs[0], rs[1])), rs[2], rs[3])
    yr.backward(dy)
    ref = [yr.detach(), xr.grad] + [r.grad for r in rs]
    for name, a, b in zip(("y", "dx", "dw1", "db1", "dw2", "db2"), got, ref):
        err = (a - b).abs().max().item() / max(1.0, b.abs().max().item())
        assert err <= 2e-2, (name, err)


@pytest.mark.parametrize("drop", [False, True])
def test_hip_fused_residual_branches(drop):
    """HipOps.linear_residual / mlp_residual (_HipLinearResidual / _HipMlpResidual: the block's proj and
    MLP with DropPath and the residual add in the GEMM epilogue, row_scale = keep[m // ntok]) against
    x + keep * branch(a) in torch fp32 autograd on the bf16 operands: outputs and every gradient, with
    keep = (1 / (1 - p), 0, 1 / (1 - p), 1 / (1 - p)) (a dropped sample) or None."""
    from mmt_amd.train import HipOps
    g = torch.Generator().manual_seed(23)
    B, ntok, C, F4 = 4, 264, 768, 3072
    M = B * ntok
    x = torch.randn(B, ntok, C, generator=g)
    a = torch.randn(M, C, generator=g).bfloat16()
    w = torch.randn(C, C, generator=g) / math.sqrt(C)
    b = torch.randn(C, generator=g) * 0.1
    w1 = torch.randn(F4, C, generator=g) / math.sqrt(C)
    b1 = torch.randn(F4, generator=g) * 0.1
    w2 = torch.randn(C, F4, generator=g) / math.sqrt(F4)
    b2 = torch.randn(C, generator=g) * 0.1
    dy = torch.randn(B, ntok, C, generator=g)
    keep = torch.tensor([1 / 0.9, 0.0, 1 / 0.9, 1 / 0.9]) if drop else None
    F = torch.nn.functional
    cases = (("linear", HipOps.linear_residual, [w, b], lambda t, ps: F.linear(t, ps[0], ps[1])),
             ("mlp", HipOps.mlp_residual, [w1, b1, w2, b2],
              lambda t, ps: F.linear(F.gelu(F.linear(t, ps[0], ps[1])), ps[2], ps[3])))
    for name, fn, params, branch in cases:
        xd = x.cuda().requires_grad_(True)
        ad = a.cuda().requires_grad_(True)
        ps = [t.cuda().requires_grad_(True) for t in params]
        y = fn(xd, ad, *ps, keep.cuda() if drop else None)
        y.backward(dy.cuda())
        got = [y.detach().cpu(), xd.grad.cpu(), ad.grad.float().cpu()] + [p.grad.cpu() for p in ps]
        xr = x.clone().requires_grad_(True)
        ar = a.float().requires_grad_(True)
        rs = [(t.bfloat16().float() if t.dim() == 2 else t.clone()).requires_grad_(True) for t in params]
        br = branch(ar, rs).view(B, ntok, C)
        yr = xr + (br * keep.view(B, 1, 1) if drop else br)
        yr.backward(dy)
        ref = [yr.detach(), xr.grad, ar.grad] + [r.grad for r in rs]
        for what, u, v in zip(("y", "dx", "da") + tuple("d%d" % i for i in range(len(ps))), got, ref):
            err = (u - v).abs().max().item() / max(1.0, v.abs().max().item())
            assert err <= 2e-2, (name, what, err)


def test_hip_layernorm_alternating_groups_fp32():
    """The fusion encoder's LN-specific norms in training (deformable_encoder_lnspecific.py:94-148):
    norm_v on the first half of every sequence's 2hw tokens and norm_i on the second, fp32 in / out
    (HipOps.layer_norm with rows0 = hw alternating groups) against chunk + two nn.LayerNorm + cat."""
    from mmt_amd.train import HipOps
    g = torch.Generator().manual_seed(5)
    b, hw, d = 3, 400, 512
    x = (torch.randn(b, 2 * hw, d, generator=g) * 2).cuda()
    nv, ni = torch.nn.LayerNorm(d).cuda(), torch.nn.LayerNorm(d).cuda()
    with torch.no_grad():
        for m in (nv, ni):
            m.weight.copy_(torch.randn(d, generator=g).cuda())
            m.bias.copy_(torch.randn(d, generator=g).cuda())
    dy = torch.randn(b, 2 * hw, d, generator=g).cuda()
    xa = x.clone().requires_grad_(True)
    ya = HipOps.layer_norm(xa, nv.weight, nv.bias, 1e-5, ni.weight, ni.bias, rows0=hw, out_f32=True)
    assert ya.dtype == torch.float32
    ya.backward(dy)
    ga = [xa.grad] + [p.grad.clone() for m in (nv, ni) for p in (m.weight, m.bias)]
    for m in (nv, ni):
        m.weight.grad = m.bias.grad = None
    xb = x.clone().requires_grad_(True)
    s1, s2 = torch.chunk(xb, 2, 1)
    yb = torch.cat([nv(s1), ni(s2)], 1)
    assert (ya - yb).abs().max().item() <= 1e-4 * max(1.0, yb.abs().max().item())
    yb.backward(dy)
    gb = [xb.grad] + [p.grad for m in (nv, ni) for p in (m.weight, m.bias)]
    for a, r in zip(ga, gb):
        assert (a - r).abs().max().item() <= 2e-4 * max(1.0, r.abs().max().item())


@pytest.mark.parametrize("B,P,C,groups", [(4, 400, 512, 32), (2, 400, 768, 32), (3, 64, 256, 8),
                                          (2, 576, 1024, 32), (2, 400, 1024, 32), (1, 1000, 768, 32)])
def test_hip_groupnorm_autograd(B, P, C, groups):
    """HipOps.group_norm (mmt_groupnorm / mmt_groupnorm_bwd on channels-last token rows) against
    nn.GroupNorm on the NCHW map the reference applies it to (fusion_utils.py:252-279): output, dx,
    dgamma, dbeta; the backward is bitwise repeatable."""
    from mmt_amd.train import HipOps
    g = torch.Generator().manual_seed(B * P + C)
    x = (torch.randn(B, P, C, generator=g) * 3 + 1).cuda()
    gn = torch.nn.GroupNorm(groups, C).cuda()
    with torch.no_grad():
        gn.weight.copy_(torch.randn(C, generator=g).cuda())
        gn.bias.copy_(torch.randn(C, generator=g).cuda())
    dy = torch.randn(B, P, C, generator=g).cuda()
    grads = []
    for rep in range(2):
        xa = x.clone().requires_grad_(True)
        ya = HipOps.group_norm(xa, gn.weight, gn.bias, groups, 1e-5)
        ya.backward(dy)
        grads.append([ya.detach(), xa.grad] + [p.grad.clone() for p in (gn.weight, gn.bias)])
        gn.weight.grad = gn.bias.grad = None
    assert all(torch.equal(a, b) for a, b in zip(grads[0], grads[1]))
    xb = x.clone().requires_grad_(True)
    yb = gn(xb.transpose(1, 2).reshape(B, C, P, 1)).reshape(B, C, P).transpose(1, 2)
    yb.backward(dy)
    ref = [yb.detach(), xb.grad, gn.weight.grad, gn.bias.grad]
    for name, a, r in zip(("y", "dx", "dgamma", "dbeta"), grads[0], ref):
        err = (a - r).abs().max().item() / max(1.0, r.abs().max().item())
        assert err <= 2e-4, (name, err)


@pytest.mark.parametrize("B,H,Cin,Cout", [(2, 20, 768, 384), (2, 40, 192, 96), (1, 80, 96, 48), (2, 40, 48, 1),
                                          (3, 20, 48, 1), (2, 20, 384, 192), (2, 20, 768, 192), (2, 20, 768, 96),
                                          (2, 20, 192, 96), (2, 20, 96, 48), (2, 40, 96, 48), (2, 80, 96, 48),
                                          (2, 20, 48, 1), (16, 20, 768, 384), (16, 80, 96, 48)])
def test_hip_conv3x3_autograd(B, H, Cin, Cout):
    """HipOps.conv3x3 (_HipConv3x3: implicit-GEMM conv forward and dX, im2col + GEMM dW / db) against
    F.conv2d autograd in fp32 on the same bf16-rounded input and weights (NHWC in, NHWC out), including
    the corner head's 48 -> 1 convs (output channels padded to 8 inside).  Relative errors: output 1e-2,
    dX / dW / db 2e-2 (bf16 operands, bf16 dY)."""
    import torch.nn.functional as F
    from mmt_amd.train import HipOps
    g = torch.Generator().manual_seed(B * H + Cin + Cout)
    x = torch.randn(B, H, H, Cin, generator=g).bfloat16().float()
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) / (3 * Cin ** 0.5)).bfloat16().float()
    b = torch.randn(Cout, generator=g)
    dy = torch.randn(B, H, H, Cout, generator=g).bfloat16().float()
    xr, wr, br = x.clone().requires_grad_(True), w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = F.conv2d(xr.permute(0, 3, 1, 2), wr, br, padding=1).permute(0, 2, 3, 1)
    yr.backward(dy)
    xd = x.bfloat16().cuda().requires_grad_(True)
    wd, bd = w.cuda().requires_grad_(True), b.cuda().requires_grad_(True)
    yd = HipOps.conv3x3(xd, wd, bd)
    yd.backward(dy.bfloat16().cuda())
    torch.cuda.synchronize()
    for name, a, r, tol in (("y", yd, yr, 1e-2), ("dx", xd.grad, xr.grad, 2e-2), ("dw", wd.grad, wr.grad, 2e-2),
                            ("db", bd.grad, br.grad, 2e-2)):
        a = a.detach().float().cpu()
        assert a.shape == r.shape, (name, a.shape, r.shape)
        err = ((a - r).norm() / r.norm()).item()
        assert err <= tol, (name, err)


@pytest.mark.parametrize("padded", [False, True])
@pytest.mark.parametrize("B,fh,c4", [(16, 80, 48), (3, 80, 48), (2, 96, 48), (1, 16, 8)])
def test_hip_corner_score_autograd(B, fh, c4, padded):
    """HipOps.corner_score (_HipCornerScore: one corner branch's conv5 in fp32 + up4(adjust3) + up2(adjust4),
    head.py:191-192) against the aten path it replaces (F.linear in fp32 + F.interpolate + adds) under fp32
    autograd, on the same bf16 inputs; the adjust maps as the HIP BatchNorm leaves them (1-channel views of
    8-channel rows, as (B, h, w, 1) views or -- padded, the fused head's form -- the 8-channel rows themselves,
    whose padding channels' gradient is 0).  Score map within 1e-5 (relative L2; fp32 sums in another order);
    dX4 / dA3 / dA4 within 1e-2 (bf16 results); dW5 / db5 within 1e-5; the backward bitwise repeatable."""
    import torch.nn.functional as F
    from mmt_amd.train import HipOps
    g = torch.Generator().manual_seed(B + fh + c4)
    x4 = torch.randn(B, fh, fh, c4, generator=g).bfloat16()
    pad3 = torch.randn(B, fh // 4, fh // 4, 8, generator=g).bfloat16()
    pad4 = torch.randn(B, fh // 2, fh // 2, 8, generator=g).bfloat16()
    conv5 = torch.nn.Conv2d(c4, 1, 1)
    with torch.no_grad():
        conv5.weight.mul_(30.0)
    dsm = torch.randn(B, fh * fh, generator=g)

    def aten(x, a3, a4, w, b):
        sm = F.linear(x.float().reshape(-1, c4), w.view(1, -1), b).view(B, fh, fh, 1)
        up = lambda t, f: F.interpolate(t.float().permute(0, 3, 1, 2), scale_factor=f).permute(0, 2, 3, 1)  # noqa: E731
        return (sm + up(a3, 4) + up(a4, 2)).reshape(B, fh * fh)

    xr = x4.float().requires_grad_(True)
    a3r = pad3[..., :1].float().requires_grad_(True)
    a4r = pad4[..., :1].float().requires_grad_(True)
    wr = conv5.weight.detach().clone().requires_grad_(True)
    br = conv5.bias.detach().clone().requires_grad_(True)
    ref = aten(xr, a3r, a4r, wr, br)
    ref.backward(dsm)

    conv = conv5.cuda()
    xd = x4.cuda().requires_grad_(True)
    p3, p4 = pad3.cuda().requires_grad_(True), pad4.cuda().requires_grad_(True)

    def run():
        for t in (xd, p3, p4, conv.weight, conv.bias):
            t.grad = None
        out = HipOps.corner_score(xd, conv, p3 if padded else p3[..., :1], p4 if padded else p4[..., :1])
        out.backward(dsm.cuda())
        torch.cuda.synchronize()
        return [t.detach().float().cpu().clone() for t in (out, xd.grad, p3.grad[..., :1], p4.grad[..., :1],
                                                            conv.weight.grad, conv.bias.grad)]

    got = run()
    again = run()
    for a, b in zip(got, again):
        assert torch.equal(a, b)
    assert p3.grad[..., 1:].abs().max().item() == 0.0 and p4.grad[..., 1:].abs().max().item() == 0.0
    for name, a, r, tol in (("sm", got[0], ref.detach(), 1e-5), ("dx4", got[1], xr.grad, 1e-2), ("da3", got[2], a3r.grad, 1e-2),
                            ("da4", got[3], a4r.grad, 1e-2), ("dw5", got[4], wr.grad, 1e-5), ("db5", got[5], br.grad, 1e-5)):
        assert a.shape == r.shape, (name, a.shape, r.shape)
        err = ((a - r).norm() / r.norm()).item()
        assert err <= tol, (name, err)


@pytest.mark.parametrize("B,H,Cin,Cout,up", [(2, 20, 192, 96, 2), (16, 40, 96, 48, 2), (2, 20, 48, 8, 4), (3, 10, 96, 1, 2)])
def test_hip_conv3x3_upsampled_input(B, H, Cin, Cout, up):
    """HipOps.conv3x3(x, w, b, up): the 3x3 conv of the nearest upsampling (x up) of x, the map never materialised
    (the GEMM's conv_up addressing; dX = the flipped conv at the upsampled size + the up x up block sums, dW over
    mmt_im2col3x3_up_bf16), against F.conv2d(F.interpolate(x)) autograd in fp32 on the same bf16 inputs: output
    1e-2, dX / dW / db 2e-2 (relative L2); keep_pad leaves a 1-channel output in its 8-channel rows (padding 0)."""
    import torch.nn.functional as F
    from mmt_amd.train import HipOps
    g = torch.Generator().manual_seed(B * H + Cin + Cout + up)
    x = torch.randn(B, H, H, Cin, generator=g).bfloat16().float()
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) / (3 * Cin ** 0.5)).bfloat16().float()
    b = torch.randn(Cout, generator=g)
    dy = torch.randn(B, H * up, H * up, Cout, generator=g).bfloat16().float()
    xr, wr, br = x.clone().requires_grad_(True), w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = F.conv2d(F.interpolate(xr.permute(0, 3, 1, 2), scale_factor=up), wr, br, padding=1).permute(0, 2, 3, 1)
    yr.backward(dy)
    xd = x.bfloat16().cuda().requires_grad_(True)
    wd, bd = w.cuda().requires_grad_(True), b.cuda().requires_grad_(True)
    keep = Cout % 8 != 0
    yd = HipOps.conv3x3(xd, wd, bd, up, keep)
    if keep:
        assert yd.shape[-1] == 8 and yd[..., Cout:].abs().max().item() == 0.0
        dyd = torch.zeros(B, H * up, H * up, 8, device="cuda", dtype=torch.bfloat16)
        dyd[..., :Cout] = dy.bfloat16().cuda()
        yd.backward(dyd)
        yd = yd[..., :Cout]
    else:
        yd.backward(dy.bfloat16().cuda())
    torch.cuda.synchronize()
    for name, a, r, tol in (("y", yd, yr, 1e-2), ("dx", xd.grad, xr.grad, 2e-2), ("dw", wd.grad, wr.grad, 2e-2),
                            ("db", bd.grad, br.grad, 2e-2)):
        a = a.detach().float().cpu()
        assert a.shape == r.shape, (name, a.shape, r.shape)
        err = ((a - r).norm() / r.norm()).item()
        assert err <= tol, (name, err)


@pytest.mark.parametrize("B,hw,grid", [(2, 20, False), (16, 20, True), (3, 7, False), (1, 22, True), (2, 20, "collapse")])
def test_msda_bimodal_train_matches_generic(B, hw, grid):
    """HipOps.msda_bimodal (mmt_msda_bimodal_train_fwd / _bwd: softmax, locations, sampling and the backward fused,
    bf16 in / out) against the step's previous composition -- F.softmax(aw.float()), ref + off.float() / wh and
    MSDeformAttnFunction (the drop-in mmt_ms_deform_attn_forward / _backward, fp32) on value.float(), with the
    casts -- on the same bf16 inputs.  grid: integer offsets (Deformable DETR's initial pattern), so that samples
    sit on pixel edges where the location gradient is discontinuous; "collapse": every sample of a level near one
    point, so that four pixels take all 1600 taps of a (batch, head, level) (the value gather's stable bucket
    placement).  Forward and grad_value within one bf16
    rounding (relative L2 1e-2; the fp32 sums are the same, only torch's softmax may differ in the last ulp),
    grad_off / grad_awl 1e-2; two runs bitwise equal (deterministic value gather)."""
    import torch.nn.functional as F
    from mmt_amd.functional import MSDeformAttnFunction
    from mmt_amd.train import HipOps, _ref_points
    g = torch.Generator().manual_seed(B * 100 + hw)
    nq = hw * hw
    value = torch.randn(B, 2 * nq, 512, generator=g).bfloat16().cuda()
    ref4 = _ref_points(hw, hw, B, 2, "cuda")
    ref_q = ref4[0, :nq, 0, :].contiguous()
    if grid == "collapse":  # loc = ref + off / hw near (0.4737, 0.4737) for every query: off = (0.4737 - ref) * hw
        tgt = 0.4737 + (torch.rand(B, nq, 8, 2, 4, 2, generator=g) - 0.5) * 2e-3
        off = ((tgt - ref_q.cpu().view(1, nq, 1, 1, 1, 2)) * hw).reshape(B, nq, 128)
    elif grid:
        base = torch.tensor([[1., 0.], [0., 1.], [-1., 0.], [0., -1.], [1., 1.], [-1., 1.], [-1., -1.], [1., -1.]])
        pts = torch.arange(1, 5).float().view(1, 1, 4, 1)
        off = (base.view(8, 1, 1, 2) * pts).expand(8, 2, 4, 2).reshape(1, 1, 128).repeat(B, nq, 1)
        off = off + torch.randint(-1, 2, off.shape, generator=g).float() * (torch.rand(off.shape, generator=g) < 0.3)
    else:
        off = torch.randn(B, nq, 128, generator=g) * 2.0
    off = off.bfloat16().cuda()
    awl = torch.randn(B, nq, 64, generator=g).bfloat16().cuda()
    gout = torch.randn(B, nq, 512, generator=g).bfloat16().cuda()

    # the previous composition (fp32 MSDA through autograd)
    vr, orr, ar = value.clone().requires_grad_(True), off.clone().requires_grad_(True), awl.clone().requires_grad_(True)
    a = F.softmax(ar.view(B, nq, 8, 8).float(), -1).view(B, nq, 8, 2, 4)
    wh = torch.tensor([hw, hw], dtype=torch.float32, device="cuda")
    loc = ref4[:, :nq, None, :, None, :] + orr.view(B, nq, 8, 2, 4, 2).float() / wh
    shapes = torch.tensor([[hw, hw]] * 2, dtype=torch.long, device="cuda")
    starts = torch.arange(2, dtype=torch.long, device="cuda") * nq
    yr = MSDeformAttnFunction.apply(vr.view(B, 2 * nq, 8, 64).float(), shapes, starts, loc.contiguous(), a.contiguous(),
                                    64).to(torch.bfloat16)
    yr.backward(gout)

    def run():  # the offsets | logits as one (B, nq, 192) tensor, as the fused Linear writes them
        v, ow = value.clone().requires_grad_(True), torch.cat([off, awl], -1).requires_grad_(True)
        y = HipOps.msda_bimodal(v, ow, ref_q, hw)
        y.backward(gout)
        return y.detach(), v.grad, ow.grad[..., :128], ow.grad[..., 128:]

    y1, gv1, go1, ga1 = run()
    y2, gv2, go2, ga2 = run()
    torch.cuda.synchronize()
    for p1, p2 in ((y1, y2), (gv1, gv2), (go1, go2), (ga1, ga2)):
        assert torch.equal(p1.view(torch.int16), p2.view(torch.int16))
    for name, a_, r_ in (("out", y1, yr), ("grad_value", gv1, vr.grad), ("grad_off", go1, orr.grad),
                         ("grad_awl", ga1, ar.grad)):
        assert a_.dtype == torch.bfloat16 and a_.shape == r_.shape, name
        a_, r_ = a_.float(), r_.float()
        err = ((a_ - r_).norm() / r_.norm().clamp_min(1e-30)).item()
        assert err <= 1e-2, (name, err)


@pytest.mark.parametrize("B,fh,stride", [(16, 80, 4), (3, 20, 16), (1, 7, 2)])
def test_hip_corner_boxes_autograd(B, fh, stride):
    """HipOps.corner_boxes (mmt_corner_boxes / _bwd) against the composition it replaces -- _soft_argmax of both
    maps (head.py:200-212), torch.stack / img_sz -- with autograd in fp32: xyxy within 1e-5 relative, the score
    maps' gradients within 1e-4 (relative L2)."""
    from mmt_amd.train import HipOps, _soft_argmax
    g = torch.Generator().manual_seed(B * fh)
    maps = [(torch.randn(B, fh * fh, generator=g) * 3).cuda() for _ in range(2)]
    dxy = torch.randn(B, 4, generator=g).cuda()
    img = fh * stride
    ref = [m.clone().requires_grad_(True) for m in maps]
    coords = []
    for m in ref:
        coords += list(_soft_argmax(m.view(B, 1, fh, fh), stride))
    yr = torch.stack(coords, 1) / img
    yr.backward(dxy)
    hip = [m.clone().requires_grad_(True) for m in maps]
    y = HipOps.corner_boxes(hip[0], hip[1], fh, stride, img)
    y.backward(dxy)
    torch.cuda.synchronize()
    assert ((y - yr).abs().max() / yr.abs().max()).item() < 1e-5
    for a, r in zip(hip, ref):
        err = ((a.grad - r.grad).norm() / r.grad.norm()).item()
        assert err < 1e-4, err


def test_hip_box_loss_matches_autograd():
    """HipOps.box_loss (mmt_box_loss / _bwd: CIoU + L1 of MixFormerRGBTActor.compute_losses with the hand-derived
    backward) against train.box_loss under autograd in fp32, on random boxes and the edge cases the chain rule
    has to get right: pred equal to gt (min / max ties split the gradient), disjoint boxes (intersection clamped to
    0), IoU > 0.5 (alpha active), boxes reaching outside [0, 1] (gt clamped), equal widths (atan term 0):
    loss and statistics within 1e-5 relative, d pred within 1e-4 of the gradient's scale (max abs)."""
    from mmt_amd.train import HipOps, box_loss
    g = torch.Generator().manual_seed(7)
    B = 64
    gt = torch.cat([torch.rand(B, 2, generator=g) * 0.6, 0.1 + torch.rand(B, 2, generator=g) * 0.4], 1)
    pred = torch.cat([gt[:, :2] + gt[:, 2:] / 2 + torch.randn(B, 2, generator=g) * 0.05,
                      gt[:, 2:] * (1 + torch.randn(B, 2, generator=g) * 0.2)], 1)
    gt[0] = torch.tensor([0.25, 0.25, 0.5, 0.5])
    pred[0] = torch.tensor([0.5, 0.5, 0.5, 0.52])                # shared x edges (ties); identical boxes would give
    # the reference's NaN (alpha = 0 / 0), which the HIP loss propagates as well (checked below)
    pred[1] = torch.tensor([0.9, 0.9, 0.05, 0.05])               # disjoint
    gt[1] = torch.tensor([0.05, 0.05, 0.1, 0.1])
    gt[2] = torch.tensor([0.8, 0.8, 0.5, 0.5])                   # reaches past 1: clamped
    pred[2] = torch.tensor([0.95, 0.95, 0.3, 0.3])
    pred[3] = torch.tensor([gt[3, 0] + gt[3, 2] / 2 + 0.01, gt[3, 1] + gt[3, 3] / 2, gt[3, 2], gt[3, 3]])  # same size
    gt[4] = torch.tensor([0.3, 0.3, 0.2, 0.2])
    pred[4] = torch.tensor([0.4, 0.45, 0.2, 0.3])                # shared left / right edges (ties)
    pred, gt = pred.cuda().view(B, 1, 4), gt.cuda()
    pr = pred.clone().requires_grad_(True)
    loss_r, st_r = box_loss(pr, gt, 2.0, 5.0)
    (3.0 * loss_r).backward()
    ph = pred.clone().requires_grad_(True)
    loss_h, st_h = HipOps.box_loss(ph, gt, 2.0, 5.0)
    (3.0 * loss_h).backward()
    torch.cuda.synchronize()
    for a, r in ((loss_h, loss_r), (st_h["ciou"], st_r["ciou"]), (st_h["l1"], st_r["l1"]), (st_h["iou"], st_r["iou"])):
        assert abs(a.item() - r.item()) <= 1e-5 * abs(r.item()) + 1e-7, (a.item(), r.item())
    err = (ph.grad - pr.grad).abs().max().item() / pr.grad.abs().max().item()
    assert err < 1e-4, (err, (ph.grad - pr.grad).abs().view(B, 4).max(1).values[:8])
    same = gt[:1].clone()
    same_pred = torch.cat([same[:, :2] + same[:, 2:] / 2, same[:, 2:]], 1).view(1, 1, 4)
    assert math.isnan(box_loss(same_pred, same)[0].item()) and math.isnan(HipOps.box_loss(same_pred, same)[0].item())


def test_token_rows_match_maps():
    """The backbones handing the fusion bf16 token rows (_HipSearchTokens, the adjust_v / adjust_i Linears as one
    grouped launch and _HipGroupNorm2; round 6) against the NCHW search maps and per-modality adjusts
    (TOKEN_ROWS False): pred boxes and every gradient of the rgbt module at B = 2 equal within 1e-6 relative L2
    (the same values through the same kernels; only the dispatch differs)."""
    import mmt_amd.model as M
    import mmt_amd.train as T
    from mmt_amd.train import HipOps, module_forward, synthetic_batch
    torch.manual_seed(0)
    net = M.build_mixformer_vit_rgbt(M.hot_path_cfg(), train=False).cuda().train()
    net.drop_path_rate = 0.0
    for m in net.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
        if isinstance(m, torch.nn.BatchNorm2d):
            m.eval()
    t, o, s, gt = synthetic_batch(2, "cuda", torch.Generator().manual_seed(7))
    res = []
    for rows in (True, False):
        T.TOKEN_ROWS = rows
        try:
            net.zero_grad(set_to_none=True)
            _, coord = module_forward(net, t, o, s, HipOps)
            (coord.float() * torch.arange(1, 5, device="cuda").view(1, 1, 4)).sum().backward()
        finally:
            T.TOKEN_ROWS = True
        res.append((coord.detach().float(), {n: p.grad.detach().clone() for n, p in net.named_parameters()
                                             if p.grad is not None}))
    (c1, g1), (c0, g0) = res
    assert set(g1) == set(g0)
    assert ((c1 - c0).norm() / c0.norm()).item() <= 1e-6
    for n in g0:
        err = ((g1[n].float() - g0[n].float()).norm() / g0[n].float().norm().clamp_min(1e-30)).item()
        assert err <= 1e-6, (n, err)


def _fusion_module(seed=3):
    from mmt_amd.model import Attention_Fusion_Bimodal_LNSpecific
    torch.manual_seed(seed)
    fu = Attention_Fusion_Bimodal_LNSpecific(768).cuda().train()
    with torch.no_grad():  # non-trivial offsets (Deformable DETR's zero init would sample the reference points only)
        for layer in fu.fusion_attention.encoder.layers:
            layer.self_attn.sampling_offsets.weight.normal_(0, 0.02)
            layer.self_attn.sampling_offsets.bias.uniform_(-2, 2)
            layer.self_attn.attention_weights.weight.normal_(0, 0.02)
        fu.fusion_attention.level_embed.normal_()
    return fu


def test_hip_encoder_layers_match_composition():
    """fusion_forward with every deformable encoder layer on the fused HIP ops (_encoder_layer_hip: query prep,
    [offsets | logits] GEMM, MSDA op, dropout-residuals, FFN) against the step's previous composition of HIP
    Linears / LayerNorms and aten glue (HipOps without encoder_layer), dropout off, 16 pairs at 20 x 20: output
    and every gradient (inputs, encoder weights, level embedding) within 2e-2 relative L2."""
    from mmt_amd.train import HipOps, fusion_forward

    class Composed(HipOps):
        encoder_layer = None

    fu = _fusion_module()
    for m in fu.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    g = torch.Generator().manual_seed(11)
    sv, si = (torch.randn(16, 768, 20, 20, generator=g).cuda() for _ in range(2))
    dout = torch.randn(16, 768, 20, 20, generator=g).cuda()
    res = []
    for ops in (HipOps, Composed):
        fu.zero_grad(set_to_none=True)
        a, b = sv.clone().requires_grad_(True), si.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = fusion_forward(fu, a, b, ops)
        y.float().backward(dout)
        grads = {n: p.grad.detach().clone() for n, p in fu.named_parameters() if p.grad is not None}
        res.append((y.detach().float(), a.grad, b.grad, grads))
    (y1, a1, b1, g1), (y0, a0, b0, g0) = res
    assert set(g1) == set(g0)
    checks = [("out", y1, y0), ("d s_v", a1, a0), ("d s_i", b1, b0)] + [(n, g1[n], g0[n]) for n in sorted(g0)]
    worst = []
    for name, x, r in checks:
        err = ((x.float() - r.float()).norm() / r.float().norm().clamp_min(1e-30)).item()
        worst.append((err, name))
        assert err <= 2e-2, (name, err)
    print("worst:", sorted(worst)[-3:])


def test_hip_encoder_dropout_masks():
    """The encoder's dropout kernels (csrc/fusion_train.hip): keep rate 1 - p (10^6 draws, p = 0.1: within 0.002),
    survivors scaled by bf16(1 / (1 - p)) in the forward; the backward regenerates the same mask (the dropped
    elements of the forward are exactly the zero gradients); the duplicated-halves form draws independently on the
    two halves; the step counter changes the draws; equal keys reproduce them bitwise."""
    from mmt_amd._lib import LIB, check
    from mmt_amd.train import _drop_rng
    st = torch.cuda.current_stream().cuda_stream
    rng = _drop_rng("cuda")
    B, rows, d, p = 4, 500, 512, 0.1
    x = torch.zeros(B, rows, d, device="cuda")
    y = torch.ones(B, rows // 2, d, device="cuda", dtype=torch.bfloat16)
    out, out2 = torch.empty_like(x), torch.empty_like(x)
    check(LIB.mmt_ft_drop_residual(x.data_ptr(), y.data_ptr(), out.data_ptr(), rng.data_ptr(), 5, p, B, rows, d, 1, st), "fwd")
    check(LIB.mmt_ft_drop_residual(x.data_ptr(), y.data_ptr(), out2.data_ptr(), rng.data_ptr(), 5, p, B, rows, d, 1, st), "fwd")
    dy = torch.empty(B, rows // 2, d, device="cuda", dtype=torch.bfloat16)
    dout = torch.zeros(B, rows, d, device="cuda")
    dout[:, :rows // 2] = 1.0  # the first half's gradient only: dy = its mask
    check(LIB.mmt_ft_drop_residual_bwd(dout.data_ptr(), dy.data_ptr(), rng.data_ptr(), 5, p, B, rows, d, 1, st), "bwd")
    torch.cuda.synchronize()
    assert torch.equal(out, out2)
    sc = torch.tensor(1 / (1 - p)).bfloat16().float().item()
    vals = set(out.unique().tolist())
    assert vals <= {0.0, sc}, vals
    rate = (out != 0).float().mean().item()
    assert abs(rate - (1 - p)) < 0.002, rate
    assert torch.equal(dy.float() != 0, out[:, :rows // 2] != 0)
    assert not torch.equal(out[:, :rows // 2] != 0, out[:, rows // 2:] != 0)  # the halves draw independently
    rng[1:].add_(1)
    check(LIB.mmt_ft_drop_residual(x.data_ptr(), y.data_ptr(), out2.data_ptr(), rng.data_ptr(), 5, p, B, rows, d, 1, st), "fwd")
    h = torch.rand(1000, 2048, device="cuda").sub_(0.3).clamp_min_(0).bfloat16()
    hd, dh = torch.empty_like(h), torch.empty_like(h)
    check(LIB.mmt_ft_relu_drop(h.data_ptr(), hd.data_ptr(), rng.data_ptr(), 9, p, h.numel(), st), "relu_drop")
    ones = torch.ones_like(h)
    check(LIB.mmt_ft_relu_drop_bwd(ones.data_ptr(), h.data_ptr(), dh.data_ptr(), rng.data_ptr(), 9, p, h.numel(), st),
          "relu_drop_bwd")
    torch.cuda.synchronize()
    assert not torch.equal(out, out2)
    kept = hd != 0
    assert torch.equal(hd.float()[kept], (h.float() * (1 / (1 - p))).bfloat16().float()[kept])
    assert torch.equal(dh != 0, kept)  # h > 0 and kept
    r2 = kept.float().sum().item() / (h > 0).float().sum().item()
    assert abs(r2 - (1 - p)) < 0.002, r2


@pytest.mark.parametrize("B,H,C,up", [(16, 20, 768, 1), (2, 40, 96, 2), (3, 16, 48, 4), (1, 5, 8, 1)])
def test_im2col3x3_channel_major_bitwise(B, H, C, up):
    """mmt_im2col3x3_cm_bf16 (channel-major columns c * 9 + tap, LDS-staged) is the tap-major
    mmt_im2col3x3_up_bf16 with its columns permuted: bitwise, on the upsampled (H = the output size) map."""
    L = _lib()
    g = torch.Generator().manual_seed(B + H + C + up)
    x = torch.randn(B, H // up, H // up, C, generator=g).bfloat16().cuda()
    M = B * H * H
    tm = torch.empty(M, 9 * C, device="cuda", dtype=torch.bfloat16)
    cm = torch.full((M, 9 * C), float("nan"), device="cuda", dtype=torch.bfloat16)
    st = torch.cuda.current_stream().cuda_stream
    L.check(L.LIB.mmt_im2col3x3_up_bf16(x.data_ptr(), tm.data_ptr(), B, H, H, C, up, st), "tap-major")
    L.check(L.LIB.mmt_im2col3x3_cm_bf16(x.data_ptr(), cm.data_ptr(), B, H, H, C, up, st), "channel-major")
    torch.cuda.synchronize()
    want = tm.view(M, 9, C).transpose(1, 2).reshape(M, 9 * C)
    assert torch.equal(cm.view(torch.int16), want.view(torch.int16))


def test_conv_wprep_layouts_bitwise():
    """mmt_conv3x3_wprep: several convs' weights in one launch -> wf [Cp][ky][kx][Cin] and wb [Cin][ky][kx][Cp]
    (bf16, RNE as .to(bfloat16)), rows / columns past Cout zero, bp = the bias zero-padded (no bias: zeros)."""
    from mmt_amd.train import _conv_wprep
    g = torch.Generator().manual_seed(5)
    shapes = [(384, 768), (1, 48), (96, 192), (8, 8), (3, 16)]
    convs = [(torch.randn(co, ci, 3, 3, generator=g).cuda(), torch.randn(co, generator=g).cuda() if k != 4 else None)
             for k, (co, ci) in enumerate(shapes)]
    out = _conv_wprep(convs)
    torch.cuda.synchronize()
    for (w, b), (wf, wb, bp) in zip(convs, out):
        co, ci = w.shape[:2]
        cp = (co + 7) // 8 * 8
        wpad = torch.zeros(cp, ci, 3, 3, device="cuda")
        wpad[:co] = w
        assert torch.equal(wf.view(torch.int16), wpad.permute(0, 2, 3, 1).reshape(cp, 9 * ci).bfloat16().view(torch.int16))
        assert torch.equal(wb.view(torch.int16), wpad.permute(1, 2, 3, 0).reshape(ci, 9 * cp).bfloat16().view(torch.int16))
        want = torch.zeros(cp, device="cuda")
        if b is not None:
            want[:co] = b
        assert torch.equal(bp, want)


@pytest.mark.parametrize("B,H,C,up", [(16, 40, 96, 2), (2, 20, 192, 1), (3, 80, 48, 4)])
def test_hip_add_up(B, H, C, up):
    """HipOps.add_up(a, b, up) = bf16(up(a) + b) and its backward (db = dout, da = the up x up block sums of dout,
    fp32 sums) against the fp32 aten composition on the same bf16 inputs: the forward bit-identical to rounding
    the fp32 sum, the gradients within 1e-2 (bf16)."""
    import torch.nn.functional as F
    from mmt_amd.train import HipOps
    g = torch.Generator().manual_seed(B + H + C + up)
    a = torch.randn(B, H // up, H // up, C, generator=g).bfloat16()
    b = torch.randn(B, H, H, C, generator=g).bfloat16()
    dout = torch.randn(B, H, H, C, generator=g).bfloat16()
    ar, br = a.float().requires_grad_(True), b.float().requires_grad_(True)
    ref = F.interpolate(ar.permute(0, 3, 1, 2), scale_factor=up).permute(0, 2, 3, 1) + br
    ref.backward(dout.float())
    ad, bd = a.cuda().requires_grad_(True), b.cuda().requires_grad_(True)
    out = HipOps.add_up(ad, bd, up)
    out.backward(dout.cuda())
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), ref.detach().bfloat16())
    for name, got, r in (("da", ad.grad, ar.grad), ("db", bd.grad, br.grad)):
        err = ((got.float().cpu() - r).norm() / r.norm()).item()
        assert err <= 1e-2, (name, err)


@pytest.mark.parametrize("B,H,C,train", [(2, 20, 384, True), (16, 80, 48, True), (3, 40, 96, True), (2, 20, 192, False),
                                         (1, 7, 8, True), (2, 20, 1, True), (16, 40, 1, True), (2, 40, 1, False)])
def test_hip_batchnorm_relu(B, H, C, train):
    """HipOps.bn_relu (mmt_batchnorm_relu / _bwd on NHWC bf16) against nn.BatchNorm2d -> ReLU in fp32 on the same
    bf16-rounded map: output (1e-2 relative, bf16 storage), the running mean / variance after the update
    (1e-5 / 1e-4), num_batches_tracked, dX (2e-2) and dgamma / dbeta (1e-3 relative L2; bf16 dY); eval mode
    normalises with the running statistics.  Bitwise repeatable."""
    from mmt_amd.train import HipOps
    g = torch.Generator().manual_seed(B * H + C)
    x = (torch.randn(B, H, H, C, generator=g) * 2.0 + 0.7).bfloat16().float()
    dy = torch.randn(B, H, H, C, generator=g).bfloat16().float()
    ref = torch.nn.BatchNorm2d(C)
    with torch.no_grad():
        ref.weight.copy_(torch.rand(C, generator=g) + 0.5)
        ref.bias.copy_(torch.randn(C, generator=g) * 0.3)
        ref.running_mean.copy_(torch.randn(C, generator=g) * 0.1)
        ref.running_var.copy_(torch.rand(C, generator=g) + 0.5)
    import copy
    hip = copy.deepcopy(ref).cuda()
    ref.train(train)
    hip.train(train)
    xr = x.clone().requires_grad_(True)
    yr = torch.relu(ref(xr.permute(0, 3, 1, 2))).permute(0, 2, 3, 1)
    yr.backward(dy)
    xd = x.bfloat16().cuda().requires_grad_(True)
    yd = HipOps.bn_relu(xd, hip)
    yd.backward(dy.bfloat16().cuda())
    torch.cuda.synchronize()
    rel = lambda a, r: ((a.detach().float().cpu() - r).norm() / r.norm().clamp_min(1e-12)).item()  # noqa: E731
    assert rel(yd, yr.detach()) <= 1e-2
    assert rel(xd.grad, xr.grad) <= 2e-2
    assert rel(hip.weight.grad, ref.weight.grad) <= 1e-3 and rel(hip.bias.grad, ref.bias.grad) <= 1e-3
    assert torch.allclose(hip.running_mean.cpu(), ref.running_mean, rtol=1e-5, atol=1e-6)
    assert torch.allclose(hip.running_var.cpu(), ref.running_var, rtol=1e-4, atol=1e-6)
    assert int(hip.num_batches_tracked) == int(ref.num_batches_tracked)
    y2 = HipOps.bn_relu(xd.detach(), hip.eval())
    y3 = HipOps.bn_relu(xd.detach(), hip)
    assert torch.equal(y2, y3)


@pytest.mark.parametrize("bn_train", [False, True])
def test_head_forward_nhwc_matches_aten(bn_train):
    """The corner head on the HIP convs and batch norm (head_forward_nhwc, bf16 maps under autocast, as
    module_forward runs it) against head_forward on aten's fp32 convs (head.py:147-212) for the same module and
    fused map, B = 2, output convs x30 (peaked maps): the normalised corners within max(2e-2 (eval BN) / 3e-2
    (train BN), 1.5 x), the
    gradients of the map and of every head parameter within max(0.1, 4 x) (a gross-error check: single bias /
    BN vectors of the 1-channel maps carry few, cancelling terms) and all head parameter gradients
    together within max(5e-2, 1.5 x) the distance of aten's own bf16 autocast path from fp32 --
    corners absolute, gradients relative L2 (BatchNorm in eval mode, or in train mode with its batch
    statistics)."""
    import copy
    import mmt_amd.model as M
    from mmt_amd.train import HipOps, head_forward
    torch.manual_seed(3)
    net = M.build_mixformer_vit_rgbt(M.hot_path_cfg(), train=False)
    hd = net.box_head.cuda()
    with torch.no_grad():
        for br in ("tl", "br"):
            getattr(hd, "conv5_" + br).weight.mul_(30.0)
    hd.train(bn_train)
    heads = [hd, copy.deepcopy(hd), copy.deepcopy(hd)]  # HIP, aten bf16 (autocast), aten fp32
    x = torch.randn(2, hd.conv1_tl[0].weight.shape[1], 20, 20, device="cuda").bfloat16().float()
    xs = [x.clone().requires_grad_(True) for _ in heads]
    wgt = torch.linspace(0.5, 1.5, 8, device="cuda").view(2, 4)
    outs = []
    for h, xi, ops in zip(heads, xs, (HipOps, None, None)):
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=h is not heads[2]):
            out = head_forward(h, xi, ops).float()
        (out * wgt).sum().backward()
        outs.append(out.detach())
    torch.cuda.synchronize()
    err = lambda a, r: (a - r).abs().max().item()  # noqa: E731
    # bf16 maps into x30 peaked soft-argmaxes.  Eval-mode BN: the HIP corners sit 1.0e-3 from fp32 (aten's
    # autocast path 7.3e-3): floor 2e-2.  Train-mode BN: the batch statistics amplify every stage's bf16 rounding
    # along the chain in BOTH paths (aten's own autocast path 1.2e-2-1.9e-2 from fp32 depending on its MIOpen
    # algorithm choice, the HIP path 2.05e-2) although each stage of the HIP head is closer to fp32 than aten's
    # (profiles/r05_head_stage_error.jsonl; test_head_stages_match_aten_per_stage below), so that chain keeps 3e-2
    floor = 3e-2 if bn_train else 2e-2
    assert err(outs[0], outs[2]) <= max(floor, 1.5 * err(outs[1], outs[2])), outs
    grads = [[xi.grad] + [p.grad for _, p in h.named_parameters()] for h, xi in zip(heads, xs)]
    names = ["x"] + [n for n, _ in hd.named_parameters()]
    # gradients that vanish mathematically (biases ahead of a train-mode BatchNorm or of the soft-argmax's
    # softmax) are rounding noise in every path: measured against the median gradient norm instead of their own
    floor = torch.tensor([r.norm().item() for r in grads[2] if r is not None]).median().item() * 5e-2
    rel = lambda a, r: ((a.float() - r).norm() / max(r.norm().item(), floor)).item()  # noqa: E731
    for name, a, b, r in zip(names, *grads):
        if r is None:
            continue
        assert a is not None, name
        assert rel(a, r) <= max(1e-1, 4.0 * rel(b, r)), (name, rel(a, r), rel(b, r))
    # all head parameters as one vector (as test_module_forward_training_gpu_grads' groups)
    cat = [torch.cat([g.flatten().float() for g, r in zip(gs[1:], grads[2][1:]) if r is not None]) for gs in grads]
    assert rel(cat[0], cat[2]) <= max(5e-2, 1.5 * rel(cat[1], cat[2])), (rel(cat[0], cat[2]), rel(cat[1], cat[2]))


@pytest.mark.parametrize("bn_train", [False, True])
def test_head_stages_match_aten_per_stage(bn_train):
    """VERDICT r4 #6, per stage: every conv() block of the HIP training head (HIP 3x3 conv + HIP BatchNorm+ReLU,
    bf16 operands) and aten's bf16 autocast block, each fed the SAME fp32 input, against the aten fp32 block --
    the HIP block within max(1e-2, 1.5 x aten's) relative (measured: HIP 0.3-0.7 %, aten 0.5-1.6 %), so the
    head's own arithmetic is not noisier than aten's; tools/head_stage_error.py prints the full table."""
    import copy
    import torch.nn.functional as F
    import mmt_amd.model as M
    from mmt_amd.train import HipOps
    torch.manual_seed(3)
    net = M.build_mixformer_vit_rgbt(M.hot_path_cfg(), train=False)
    hd = net.box_head.cuda()
    hd.train(bn_train)
    heads = [hd, copy.deepcopy(hd), copy.deepcopy(hd)]  # HIP, aten bf16, aten fp32
    x = torch.randn(2, hd.conv1_tl[0].weight.shape[1], 20, 20, device="cuda").bfloat16().float()
    nchw, nhwc = (lambda t: t.permute(0, 3, 1, 2)), (lambda t: t.permute(0, 2, 3, 1))
    up = lambda t, f: F.interpolate(t, scale_factor=f)  # noqa: E731
    bad = []

    def stage(name, inp, idx=None):
        outs = []
        for i, h in enumerate(heads):
            seq = getattr(h, name)
            seq = seq if idx is None else seq[idx]
            with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16, enabled=i < 2):
                if i == 0:
                    y = HipOps.conv3x3(nhwc(inp).to(torch.bfloat16).contiguous(), seq[0].weight, seq[0].bias)
                    outs.append(nchw(HipOps.bn_relu(y, seq[1])).float())
                else:
                    outs.append(seq(inp).float())
        sc = outs[2].abs().max().item() + 1e-12
        e_hip, e_aten = [(o - outs[2]).abs().max().item() / sc for o in outs[:2]]
        if e_hip > max(1e-2, 1.5 * e_aten):
            bad.append((name, idx, e_hip, e_aten))
        return outs[2]

    for br in ("tl", "br"):
        x1 = stage("conv1_" + br, x)
        x2 = stage("conv2_" + br, x1)
        a1 = stage("adjust1_" + br, x)
        x3 = stage("conv3_" + br, up(a1, 2) + up(x2, 2))
        stage("conv4_" + br, up(stage("adjust2_" + br, x), 4) + up(x3, 2))
        stage("adjust3_" + br, stage("adjust3_" + br, stage("adjust3_" + br, x2, 0), 1), 2)
        stage("adjust4_" + br, stage("adjust4_" + br, x3, 0), 1)
    assert not bad, bad


@pytest.mark.parametrize("norm", ["sync", "frozen"])
def test_head_forward_nhwc_sync_and_frozen_bn(norm):
    """the norms of the reference trainer's head -- SyncBatchNorm (train_script_mixformer.py:105
    converts every head BatchNorm, even on one GPU) and FrozenBatchNorm2d (head.py:7-20 freeze_bn) -- take the
    HIP batch norm (world size 1 / fixed statistics), run in train mode without error, and match the aten fp32
    head on the same module within the bf16 bar of test_head_forward_nhwc_matches_aten; SyncBatchNorm updates
    its running statistics like BatchNorm2d."""
    import copy
    import mmt_amd.model as M
    import mmt_amd.train as T
    from mmt_amd.train import HipOps, head_forward
    torch.manual_seed(4)
    hd = M.Pyramid_Corner_Predictor(inplanes=64, channel=64, feat_sz=20, stride=16, freeze_bn=norm == "frozen")
    if norm == "sync":
        hd = torch.nn.SyncBatchNorm.convert_sync_batchnorm(hd)
        assert any(type(m) is torch.nn.SyncBatchNorm for m in hd.modules())
    else:  # non-trivial fixed statistics
        with torch.no_grad():
            for m in hd.modules():
                if isinstance(m, M.FrozenBatchNorm2d):
                    m.weight.uniform_(0.5, 1.5)
                    m.bias.uniform_(-0.2, 0.2)
                    m.running_mean.uniform_(-0.2, 0.2)
                    m.running_var.uniform_(0.5, 2.0)
    hd = hd.cuda().train()
    assert all(T._hip_bn_ok(m) for m in hd.modules() if isinstance(m, (torch.nn.SyncBatchNorm, M.FrozenBatchNorm2d)))
    heads = [hd, copy.deepcopy(hd)]
    x = torch.randn(2, 64, 20, 20, device="cuda").bfloat16().float()
    xs = [x.clone().requires_grad_(True) for _ in heads]
    outs = []
    for h, xi, ops in zip(heads, xs, (HipOps, None)):
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=ops is not None):
            out = head_forward(h, xi, ops).float()
        out.sum().backward()
        outs.append(out.detach())
    torch.cuda.synchronize()
    assert torch.isfinite(outs[0]).all() and torch.isfinite(xs[0].grad).all()
    assert (outs[0] - outs[1]).abs().max().item() <= 3e-2, outs
    rel = ((xs[0].grad - xs[1].grad).norm() / xs[1].grad.norm()).item()
    assert rel <= 1e-1, rel
    if norm == "sync":
        for (n, a), b in zip(heads[0].named_buffers(), heads[1].buffers()):
            if "running" in n:
                assert torch.allclose(a, b, rtol=2e-2, atol=2e-3), n


def test_train_step_graph_replay_matches_eager():
    """TrainStep.capture / replay (the whole step -- forward on the HIP ops incl. the HIP head convs, box
    loss, backward, clip + HipAdamW -- as one hipGraph) against the same steps run eagerly from identical
    weights on the same batches (drop-path and dropout off, BatchNorm in train mode): two eager runs are bitwise
    equal (a deterministic step), the replayed losses and parameters within 1e-6 of the eager ones, and every
    parameter's update direction over the four steps at cosine >= 0.99 to the eager one (two eager warm-up steps,
    then two replays with new batches copied into the static inputs); a third replay changes the weights again
    (it is not a no-op)."""
    import copy
    import mmt_amd.model as M
    from mmt_amd.train import HipOps, TrainStep, synthetic_batch
    torch.manual_seed(0)
    net = M.build_mixformer_vit_rgbt(M.hot_path_cfg(), train=False)
    net.drop_path_rate = 0.0
    for m in net.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    net_b = copy.deepcopy(net)
    net, net_b = net.cuda().train(), net_b.cuda().train()
    g = torch.Generator().manual_seed(11)
    batches = [synthetic_batch(2, "cuda", g) for _ in range(4)]
    net_c = copy.deepcopy(net)
    p0 = [p.detach().clone() for p in net.parameters()]
    eager, graphed, eager2 = TrainStep(net, HipOps), TrainStep(net_b, HipOps), TrainStep(net_c, HipOps)
    le = [float(eager(*b)["loss"]) for b in batches]
    le2 = [float(eager2(*b)["loss"]) for b in batches]  # the eager step's own run-to-run spread (atomics)
    static = [[x.clone() for x in z] if isinstance(z, list) else z.clone() for z in batches[0]]
    graphed.capture(*static, warmup=1)  # one eager warm-up step: batch 0 (its static copy)
    lg = [None]
    graphed.replay(*batches[1])  # the captured step on batch 1
    torch.cuda.synchronize()
    for b in batches[2:]:
        lg.append(float(graphed.replay(*b)["loss"]))
        torch.cuda.synchronize()
    spread = max(abs(a - a2) for a, a2 in zip(le, le2))  # over the four steps
    # the step is deterministic (round 5: the MSDA backward gathers grad_value in a fixed order instead of float
    # atomics): two eager runs agree bit for bit, and the replayed step matches the eager one to 1e-6
    assert spread == 0.0, (le, le2)
    assert all(torch.equal(pa, pc) for pa, pc in zip(net.parameters(), net_c.parameters()))
    for a, b in zip(le[2:], lg[1:]):
        assert abs(a - b) <= 1e-6 * max(1.0, abs(a)), (le, le2, lg)
    for (n, pa), pb in zip(net.named_parameters(), net_b.parameters()):
        if pa.requires_grad:
            err = (pa - pb).abs().max().item()
            assert err <= 1e-6 * max(1.0, pa.abs().max().item()), (n, err)
    # compare the update DIRECTIONS (p_after - p_before), which a replay with stale or
    # mis-addressed gradients would turn, not only their size (AdamW moves every element by ~lr whatever
    # its gradient).  Parameters whose two eager runs already disagree in direction (noise-level gradients,
    # e.g. the BatchNorm bias of a 1-channel map) are exempt; they must be a small share of the elements.
    bad, checked, total = [], 0, 0
    cos = torch.nn.functional.cosine_similarity
    for (n, pa), pb, pc, pi in zip(net.named_parameters(), net_b.parameters(), net_c.parameters(), p0):
        if not pa.requires_grad:
            continue
        de, dg, de2 = (pa - pi).flatten(), (pb - pi).flatten(), (pc - pi).flatten()
        total += pa.numel()
        if de.norm() == 0 or cos(de, de2, dim=0).item() < 0.999:
            continue
        checked += pa.numel()
        c = cos(de, dg, dim=0).item()
        if c < 0.99:
            bad.append((n, c))
    assert not bad, bad[:5]
    assert checked >= 0.95 * total, (checked, total)
    before = [p.detach().clone() for p in net_b.parameters() if p.requires_grad][:4]
    graphed.replay(*batches[0])
    torch.cuda.synchronize()
    after = [p.detach() for p in net_b.parameters() if p.requires_grad][:4]
    assert any(not torch.equal(a, b) for a, b in zip(before, after))
    # the captured AdamW launches hold capture-time learning rates: a scheduler step must not replay silently
    graphed.opt.param_groups[0]["lr"] *= 0.5
    with pytest.raises(RuntimeError, match="hyper-parameters changed"):
        graphed.replay(*batches[0])


@pytest.mark.parametrize("drop", [False, True])
def test_hip_lockstep_pair_functions(drop):
    """HipOps.linear2 / linear_residual2 / mlp_residual2 (the two-stream backbones in lockstep: rows [0, M)
    with the RGB weights, [M, 2M) with the TIR weights, grouped GEMMs forward and backward, per-modality
    launches for the DropPath row scale) against torch fp32 autograd on the bf16 operands, per half:
    outputs and every gradient within 2e-2 of the largest magnitude, as the one-modality Functions."""
    from mmt_amd.train import HipOps
    g = torch.Generator().manual_seed(31)
    B, ntok, C, F4 = 4, 264, 768, 3072
    M = B * ntok
    F = torch.nn.functional
    x = torch.randn(2 * B, ntok, C, generator=g)
    a = torch.randn(2 * M, C, generator=g).bfloat16()
    lin = [[torch.randn(C, C, generator=g) / math.sqrt(C), torch.randn(C, generator=g) * 0.1] for _ in range(2)]
    mlp = [[torch.randn(F4, C, generator=g) / math.sqrt(C), torch.randn(F4, generator=g) * 0.1,
            torch.randn(C, F4, generator=g) / math.sqrt(F4), torch.randn(C, generator=g) * 0.1] for _ in range(2)]
    dy = torch.randn(2 * B, ntok, C, generator=g)
    keep = torch.tensor([1 / 0.9, 0.0, 1 / 0.9, 1 / 0.9, 0.0, 1 / 0.9, 1 / 0.9, 1 / 0.9]) if drop else None

    def run(kind, xd, ad, ps):
        if kind == "linear2":
            return HipOps.linear2(ad, *ps[0], *ps[1], out_f32=True)
        if kind == "linear_residual2":
            return HipOps.linear_residual2(xd, ad, *ps[0], *ps[1], keep.cuda() if drop else None)
        return HipOps.mlp_residual2(xd, ad, ps[0], ps[1], keep.cuda() if drop else None)

    def ref_branch(kind, u, ps):
        return F.linear(u, ps[0], ps[1]) if kind != "mlp_residual2" else \
            F.linear(F.gelu(F.linear(u, ps[0], ps[1])), ps[2], ps[3])

    for kind, params in (("linear2", lin), ("linear_residual2", lin), ("mlp_residual2", mlp)):
        xd = x.cuda().requires_grad_(True)
        ad = a.cuda().requires_grad_(True)
        ps = [[t.cuda().requires_grad_(True) for t in pm] for pm in params]
        y = run(kind, xd, ad, ps)
        y.backward(dy.cuda().view(y.shape))
        got = [y.detach().cpu().view(2 * B, ntok, C), ad.grad.float().cpu()] + [t.grad.cpu() for pm in ps for t in pm]
        if kind != "linear2":
            got.append(xd.grad.cpu())
        xr = x.clone().requires_grad_(True)
        ar = a.float().requires_grad_(True)
        rs = [[(t.bfloat16().float() if t.dim() == 2 else t.clone()).requires_grad_(True) for t in pm] for pm in params]
        br = torch.cat([ref_branch(kind, ar[:M], rs[0]), ref_branch(kind, ar[M:], rs[1])], 0).view(2 * B, ntok, C)
        yr = br if kind == "linear2" else xr + (br * keep.view(-1, 1, 1) if drop else br)
        yr.backward(dy)
        ref = [yr.detach(), ar.grad] + [t.grad for pm in rs for t in pm]
        if kind != "linear2":
            ref.append(xr.grad)
        for i, (u, v) in enumerate(zip(got, ref)):
            err = (u - v).abs().max().item() / max(1.0, v.abs().max().item())
            assert err <= 2e-2, (kind, i, err)
