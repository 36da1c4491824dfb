"""Training step on CPU: the step's autograd graph against the oracle's, and the
data-parallel gradient exchange over a world_size-2 gloo group.

The backbone's matrix work is injected (`ops`); here it is a plain fp32 PyTorch stand-in (test
infrastructure, like the oracle), so these tests check the step's structure — forward, box loss
(actors/mixformer_rgbt.py:127-168), parameter groups (base_functions.py:362-400), DDP averaging,
clip + AdamW — while tests/test_gpu_train.py checks the HIP ops themselves on the MI355X.
Small images (64 px search, 32 px template) keep the full-width ViT-B step within seconds."""
import os

import pytest
import torch
import torch.nn.functional as F

from conftest import ROOT

SEARCH, TEMPLATE = 64, 32


class TorchOps:
    """fp32 stand-in for HipOps: nn.Linear and the MAM softmax attention (mixformer.py:52-78)."""

    dtype = torch.float32

    @staticmethod
    def linear(x, weight, bias, out_f32=False):
        y = F.linear(x, weight, bias)
        return y.float() if out_f32 else y

    @staticmethod
    def mam_attention(qkv, n_t, heads):
        S, ntok, C3 = qkv.shape
        C = C3 // 3
        q, k, v = qkv.view(S, ntok, 3, heads, C // heads).permute(2, 0, 3, 1, 4)
        sc = (C // heads) ** -0.5
        ot = torch.softmax(q[:, :, :n_t] @ k[:, :, :n_t].transpose(-1, -2) * sc, -1) @ v[:, :, :n_t]
        os_ = torch.softmax(q[:, :, n_t:] @ k.transpose(-1, -2) * sc, -1) @ v
        return torch.cat([ot, os_], 2).transpose(1, 2).reshape(S, ntok, C)

    @staticmethod
    def mam_attention_asym(qkv, Bh, n_t, heads):
        from mmt_amd.train import asym_attention_from_mam
        return asym_attention_from_mam(TorchOps.mam_attention, qkv, Bh, n_t, heads)

    @staticmethod
    def ms_deform_attn(value, hw, loc, aw):
        return _msda_core(value, hw, loc, aw)


def _msda_core(value, hw, loc, aw):
    """ms_deform_attn_core_pytorch (ms_deform_attn_func.py:41-61): bilinear, zero padding,
    align_corners=False; value (N, L*hw*hw, M, D), loc (N, Lq, M, L, P, 2), aw (N, Lq, M, L, P)."""
    N, _, M, D = value.shape
    _, Lq, _, L, P, _ = loc.shape
    vl = value.split([hw * hw] * L, dim=1)
    grids = 2 * loc - 1
    outs = []
    for lid in range(L):
        v = vl[lid].flatten(2).transpose(1, 2).reshape(N * M, D, hw, hw)
        g = grids[:, :, :, lid].transpose(1, 2).flatten(0, 1)
        outs.append(F.grid_sample(v, g, mode="bilinear", padding_mode="zeros", align_corners=False))
    aw = aw.transpose(1, 2).reshape(N * M, 1, Lq, L * P)
    out = (torch.stack(outs, dim=-2).flatten(-2) * aw).sum(-1).view(N, M * D, Lq)
    return out.transpose(1, 2)


def _net(seed=0):
    from mmt_amd.model import build_mixformer_vit_rgbt, hot_path_cfg
    torch.manual_seed(seed)
    net = build_mixformer_vit_rgbt(hot_path_cfg(search=SEARCH, template=TEMPLATE), train=False)
    with torch.no_grad():  # non-trivial corner heatmaps (default init is near-flat)
        for br in ("tl", "br"):
            getattr(net.box_head, "conv5_" + br).weight.mul_(30.0)
    return net.eval()  # BatchNorm on running statistics (SyncBN needs a GPU)


def _batch(B, seed):
    from mmt_amd.train import synthetic_batch
    return synthetic_batch(B, "cpu", torch.Generator().manual_seed(seed), TEMPLATE, SEARCH)


def test_forward_and_grads_match_oracle():
    from mmt_amd.train import box_loss, forward_boxes
    from oracle.forward import forward as oracle_forward
    torch.set_num_threads(8)
    net = _net()
    t, o, s, gt = _batch(2, 1)
    pred = forward_boxes(net, t, o, s, TorchOps)
    loss, _ = box_loss(pred, gt)
    loss.backward()

    sd = {k: v.detach().clone() for k, v in net.state_dict().items()}
    leaves = {k: sd[k].requires_grad_() for k, p in net.named_parameters() if p.requires_grad}
    ref, _ = oracle_forward.__wrapped__(sd, "rgbt", t, o, s)  # undecorated: autograd on
    ref_loss, _ = box_loss(ref["pred_boxes"], gt)
    ref_loss.backward()
    assert (pred - ref["pred_boxes"]).abs().max().item() < 1e-5
    assert abs(loss.item() - ref_loss.item()) < 1e-5
    for k, p in net.named_parameters():
        if not p.requires_grad:
            continue
        g, rg = p.grad, leaves[k].grad
        assert g is not None and rg is not None, k
        # 1e-3 of the tensor's largest gradient; the 1e-6 floor covers the corner-map biases, whose
        # exact gradient is 0 (softmax is shift-invariant) and whose computed one is rounding noise.
        assert (g - rg).abs().max().item() <= 1e-3 * rg.abs().max().item() + 1e-6, k


class TorchPairOps(TorchOps):
    """TorchOps with the grouped two-modality Linears of HipOps (linear2 / linear_residual2 / mlp_residual2):
    rows [0, M) take the first weights, rows [M, 2M) the second; keep [2B] scales the branch per sequence."""

    @staticmethod
    def linear2(x, w0, b0, w1, b1, out_f32=False):
        h = x.shape[0] // 2
        return torch.cat([F.linear(x[:h], w0, b0), F.linear(x[h:], w1, b1)], 0)

    @staticmethod
    def linear_residual2(x, a, w0, b0, w1, b1, keep):
        y = TorchPairOps.linear2(a, w0, b0, w1, b1).view(x.shape)
        return x + (y if keep is None else y * keep.view(-1, 1, 1))

    @staticmethod
    def mlp_residual2(x, xn, p0, p1, keep):
        h = xn.shape[0] // 2
        y = torch.cat([F.linear(F.gelu(F.linear(u, p[0], p[1])), p[2], p[3]) for u, p in ((xn[:h], p0), (xn[h:], p1))],
                      0).view(x.shape)
        return x + (y if keep is None else y * keep.view(-1, 1, 1))


def test_lockstep_backbone_pair_matches_sequential():
    """backbone_forward_pair (both backbones in lockstep on the stacked batch, HipOps' grouped-GEMM form)
    against backbone_forward run once per modality: boxes, loss and every parameter gradient (eval-mode
    module: no stochastic depth draws, so both forms compute the same function)."""
    from mmt_amd import train
    torch.set_num_threads(8)
    t, o, s, gt = _batch(2, 3)
    out = []
    for ops in (TorchOps, TorchPairOps):
        net = _net(seed=1)
        pred = train.forward_boxes(net, t, o, s, ops)
        loss, _ = train.box_loss(pred, gt)
        loss.backward()
        out.append((pred.detach(), {k: p.grad for k, p in net.named_parameters() if p.requires_grad}))
    (p0, g0), (p1, g1) = out
    assert (p0 - p1).abs().max().item() < 1e-5
    for k, g in g0.items():
        assert g1[k] is not None, k
        assert (g - g1[k]).abs().max().item() <= 1e-4 * g.abs().max().item() + 1e-7, k


def test_param_groups_follow_reference():
    from mmt_amd.train import param_groups
    net = _net()
    groups = param_groups(net, 1e-4)
    lrs = [g.get("lr", 1e-4) for g in groups]
    assert lrs == pytest.approx([1e-5, 2e-6, 2e-6, 1e-4, 1e-5])
    grouped = {id(p) for g in groups for p in g["params"]}
    for n, p in net.named_parameters():
        assert (id(p) in grouped) == ("pos_embed" not in n), n
        assert p.requires_grad == ("pos_embed" not in n), n


def test_train_step_reduces_loss_on_fixed_batch():
    from mmt_amd.train import TrainStep
    torch.set_num_threads(8)
    net = _net()
    step = TrainStep(net, TorchOps, lr=1e-4)
    batch = _batch(2, 3)
    losses = [step(*batch)["loss"].item() for _ in range(4)]
    assert losses[-1] < losses[0], losses


def _ddp_worker(rank, world, port, out_dir):
    import torch.distributed as dist
    from mmt_amd.train import TrainStep
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(4)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # the step's own bucketed all-reduce (fp32, the default, and bf16-compressed buckets) and the torch
        # DistributedDataParallel wrapper (ddp="torch", fp32)
        for mode, comp in ((True, "none"), (True, "bf16"), ("torch", "none")):
            net = _net()
            step = TrainStep(net, TorchOps, lr=1e-4, ddp=mode, grad_compress=comp)
            t, o, s, gt = _batch(2, 5)
            sl = slice(rank, rank + 1)  # each rank its own sequence of the global batch of 2
            step.backward([x[sl] for x in t], [x[sl] for x in o], [x[sl] for x in s], gt[sl])
            grads = {n: p.grad.clone() for n, p in net.named_parameters() if p.grad is not None}
            step.apply()
            params = {n: p.detach().clone() for n, p in net.named_parameters()}
            tag = comp if mode is True else "torch_" + comp
            torch.save({"grads": grads, "params": params}, os.path.join(out_dir, "rank%d_%s.pt" % (rank, tag)))
    finally:
        dist.destroy_process_group()


def test_ddp_gloo_two_ranks_matches_full_batch(tmp_path):
    import socket
    import torch.multiprocessing as mp
    from mmt_amd.train import TrainStep
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    mp.spawn(_ddp_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)

    torch.set_num_threads(8)
    net = _net()
    step = TrainStep(net, TorchOps, lr=1e-4)
    step.backward(*_batch(2, 5))
    full = {n: p.grad for n, p in net.named_parameters() if p.grad is not None}
    # fp32 all-reduce: the batch mean within fp32 summation noise; bf16-compressed buckets: the
    # mean rounded to bf16 (8 significant bits) once, within 2^-7 of each tensor's largest gradient
    for comp, tol in (("none", 1e-4), ("bf16", 2 ** -7), ("torch_none", 1e-4)):
        r0 = torch.load(tmp_path / ("rank0_%s.pt" % comp), weights_only=True)
        r1 = torch.load(tmp_path / ("rank1_%s.pt" % comp), weights_only=True)
        assert set(full) == set(r0["grads"]) == set(r1["grads"])
        for n, g in full.items():
            assert torch.equal(r0["grads"][n], r1["grads"][n]), (comp, n)  # all-reduced: identical on both ranks
            scale = g.abs().max().item() + 1e-12
            assert (r0["grads"][n] - g).abs().max().item() <= tol * scale + 1e-6, (comp, n)  # mean == batch mean
        for n in r0["params"]:
            assert torch.equal(r0["params"][n], r1["params"][n]), (comp, n)  # replicas stay in lockstep


# ----------------------------------------------------------------------------- module-level autograd
BUILDERS = {"rgbt": "build_mixformer_vit_rgbt", "shared": "build_mixformer_vit_rgbt_shared", "asym": "build_asymmetric_shared"}


def _train_net(variant, seed=0):
    """The drop-in module in train() mode with the test's fp32 op stand-in; stochastic depth and
    dropout off and BatchNorm on running statistics, so that the forward is deterministic."""
    import mmt_amd.model as M
    torch.manual_seed(seed)
    net = getattr(M, BUILDERS[variant])(M.hot_path_cfg(search=SEARCH, template=TEMPLATE), train=False)
    with torch.no_grad():
        for br in ("tl", "br"):
            getattr(net.box_head, "conv5_" + br).weight.mul_(30.0)
    net.train()
    net.train_ops = TorchOps
    net.drop_path_rate = 0.0
    for m in net.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
        if isinstance(m, torch.nn.BatchNorm2d):
            m.eval()
    return net


@pytest.mark.parametrize("variant", ["rgbt", "shared", "asym"])
def test_module_forward_autograd_matches_oracle(variant):
    """net.train(); out, coord = net(t, o, s, gt_bboxes=...) builds the autograd graph (the reference
    actor's call, actors/mixformer_rgbt.py:82-98): boxes and every parameter gradient of the box loss
    equal autograd through the oracle's restatement of the same variant.  For the cross-modal variant
    this also pins the training path's asymmetric attention (two standard attentions composed) against
    the oracle's direct formula (asymmetric_shared.py:55-104)."""
    from mmt_amd.train import box_loss
    from oracle.forward import forward as oracle_forward
    torch.set_num_threads(8)
    net = _train_net(variant)
    t, o, s, gt = _batch(2, 3)
    gt_xyxy = torch.cat([gt[:, :2], gt[:, :2] + gt[:, 2:]], 1)
    out, coord = net(t, o, s, run_score_head=False, gt_bboxes=gt_xyxy)
    assert out["pred_boxes"] is coord and coord.requires_grad
    loss, _ = box_loss(coord, gt)
    loss.backward()
    sd = {k: v.detach().clone() for k, v in net.state_dict().items()}
    leaves = {k: sd[k].requires_grad_() for k, p in net.named_parameters() if p.requires_grad}
    ref, _ = oracle_forward.__wrapped__(sd, variant, t, o, s)
    ref_loss, _ = box_loss(ref["pred_boxes"], gt)
    ref_loss.backward()
    assert (coord - ref["pred_boxes"]).abs().max().item() < 1e-5
    n = 0
    for k, p in net.named_parameters():
        if not p.requires_grad or leaves[k].grad is None:
            continue
        g, rg = p.grad, leaves[k].grad
        assert g is not None, k
        assert (g - rg).abs().max().item() <= 1e-3 * rg.abs().max().item() + 1e-6, k
        n += 1
    assert n > 100


def test_module_forward_eval_still_refuses_cpu():
    """Outside training (or with the product ops) the module has no CPU path."""
    net = _train_net("rgbt").eval()
    t, o, s, _ = _batch(1, 4)
    with pytest.raises(RuntimeError):
        net(t, o, s)
    net.train()
    net.train_ops = None
    with pytest.raises(RuntimeError):
        net(t, o, s)


def _ddp_module_worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from mmt_amd.train import box_loss
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(2)
        net = _train_net("rgbt")
        ddp = torch.nn.parallel.DistributedDataParallel(net)  # the reference's wrap, unchanged
        t, o, s, gt = _batch(2, 5)
        sl = slice(rank, rank + 1)
        out, coord = ddp([x[sl] for x in t], [x[sl] for x in o], [x[sl] for x in s], gt_bboxes=None)
        loss, _ = box_loss(coord, gt[sl])
        loss.backward()
        grads = {n: p.grad.clone() for n, p in net.named_parameters() if p.grad is not None}
        torch.save({"grads": grads}, os.path.join(out_dir, "mrank%d.pt" % rank))
    finally:
        dist.destroy_process_group()


def test_ddp_gloo_two_ranks_through_module_forward(tmp_path):
    """DistributedDataParallel wraps the drop-in module itself (not a training wrapper): two gloo
    ranks with one sample each all-reduce to the full-batch gradient of the module's own forward."""
    import socket
    import torch.multiprocessing as mp
    from mmt_amd.train import box_loss
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    mp.spawn(_ddp_module_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "mrank0.pt", weights_only=True)["grads"]
    r1 = torch.load(tmp_path / "mrank1.pt", weights_only=True)["grads"]
    torch.set_num_threads(8)
    net = _train_net("rgbt")
    t, o, s, gt = _batch(2, 5)
    _, coord = net(t, o, s)
    loss, _ = box_loss(coord, gt)
    loss.backward()
    full = {n: p.grad for n, p in net.named_parameters() if p.grad is not None}
    assert set(full) == set(r0) == set(r1)
    for n, g in full.items():
        assert torch.equal(r0[n], r1[n]), n
        assert (r0[n] - g).abs().max().item() <= 1e-4 * (g.abs().max().item() + 1e-12) + 1e-6, n


def _ciou_loss_columns(b1, b2):
    """The scalar-column form of lib/utils/box_ops.py:100-152 (mmt_amd.train.ciou_loss before round 5's (N, 2)
    pairing), kept as the test's restatement."""
    import math
    w1, h1 = b1[:, 2] - b1[:, 0], b1[:, 3] - b1[:, 1]
    w2, h2 = b2[:, 2] - b2[:, 0], b2[:, 3] - b2[:, 1]
    cx1, cy1 = (b1[:, 0] + b1[:, 2]) / 2.0, (b1[:, 1] + b1[:, 3]) / 2.0
    cx2, cy2 = (b2[:, 0] + b2[:, 2]) / 2.0, (b2[:, 1] + b2[:, 3]) / 2.0
    il, ir = torch.max(cx1 - w1 / 2, cx2 - w2 / 2), torch.min(cx1 + w1 / 2, cx2 + w2 / 2)
    it, ib = torch.max(cy1 - h1 / 2, cy2 - h2 / 2), torch.min(cy1 + h1 / 2, cy2 + h2 / 2)
    inter = torch.clamp(ir - il, min=0) * torch.clamp(ib - it, min=0)
    cl, cr = torch.min(cx1 - w1 / 2, cx2 - w2 / 2), torch.max(cx1 + w1 / 2, cx2 + w2 / 2)
    ct, cb = torch.min(cy1 - h1 / 2, cy2 - h2 / 2), torch.max(cy1 + h1 / 2, cy2 + h2 / 2)
    inter_diag = (cx2 - cx1) ** 2 + (cy2 - cy1) ** 2
    c_diag = torch.clamp(cr - cl, min=0) ** 2 + torch.clamp(cb - ct, min=0) ** 2
    union = w1 * h1 + w2 * h2 - inter
    u = inter_diag / c_diag
    iou = inter / union
    v = (4 / (math.pi ** 2)) * torch.pow(torch.atan(w2 / h2) - torch.atan(w1 / h1), 2)
    with torch.no_grad():
        alpha = (iou > 0.5).float() * v / (1 - iou + v)
    cious = torch.clamp(iou - u - alpha * v, min=-1.0, max=1.0)
    return torch.mean(1 - cious), iou


def test_ciou_loss_matches_column_form():
    """mmt_amd.train.ciou_loss (x / y as (N, 2) pairs) against the scalar-column restatement of box_ops.py:100-152:
    the same loss values bitwise, gradients within rounding, both iou > 0.5 (alpha active) and disjoint boxes."""
    from mmt_amd.train import ciou_loss
    g = torch.Generator().manual_seed(0)
    for trial in range(12):
        c = torch.rand(16, 2, generator=g) * 0.8 + 0.1
        wh = torch.rand(16, 2, generator=g) * 0.3 + 0.05
        b1 = torch.cat([c - wh / 2, c + wh / 2], 1).requires_grad_(True)
        if trial % 2:
            b2 = torch.cat([c - wh / 2 + 0.01, c + wh / 2 * 0.9], 1)  # overlapping: the alpha branch
        else:
            c2 = torch.rand(16, 2, generator=g)
            b2 = torch.cat([c2 - wh / 3, c2 + wh / 3], 1)
        la, ia = ciou_loss(b1, b2)
        lb, ib = _ciou_loss_columns(b1, b2)
        assert torch.equal(la, lb) and torch.equal(ia, ib)
        ga, = torch.autograd.grad(la, b1)
        gb, = torch.autograd.grad(lb, b1)
        assert (ga - gb).abs().max().item() <= 1e-6 * gb.abs().max().item()
