"""torch.library.opcheck of the registered native ops on the GPU (schema, fake kernel vs the real
output's metadata, autograd registration, AOT dispatch), plus gradients through the registered
autograd formulas equal the autograd.Function drop-ins (mmt_amd.functional), which the reference
API exposes (ms_deform_attn_func.py:22-38, prroi_pool/functional.py:38-76)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _msda_inputs(dtype=torch.float32, seed=0):
    g = torch.Generator().manual_seed(seed)
    N, M, D, Lq, L, P = 2, 2, 8, 5, 2, 2
    shapes = torch.tensor([[6, 4], [3, 2]], dtype=torch.long)
    starts = torch.tensor([0, 24], dtype=torch.long)
    S = 30
    value = torch.rand(N, S, M, D, generator=g, dtype=torch.float64).to(dtype)
    loc = torch.rand(N, Lq, M, L, P, 2, generator=g, dtype=torch.float64).to(dtype)
    aw = torch.rand(N, Lq, M, L, P, generator=g, dtype=torch.float64).to(dtype) + 1e-5
    aw = aw / aw.sum(-1, keepdim=True).sum(-2, keepdim=True)
    return [x.cuda() for x in (value, shapes, starts, loc, aw)]


def test_opcheck_ms_deform_attn():
    import mmt_amd.ops  # noqa: F401
    value, shapes, starts, loc, aw = _msda_inputs()
    value.requires_grad_(True)
    loc.requires_grad_(True)
    aw.requires_grad_(True)
    torch.library.opcheck(torch.ops.mmt.ms_deform_attn_forward.default, (value, shapes, starts, loc, aw))


def test_opcheck_prroi_pool():
    import mmt_amd.ops  # noqa: F401
    g = torch.Generator().manual_seed(1)
    f = torch.randn(2, 4, 10, 12, generator=g).cuda().requires_grad_(True)
    rois = torch.tensor([[0, 1.2, 0.5, 7.3, 6.1], [1, 0.0, 2.0, 9.5, 8.0]]).cuda().requires_grad_(True)
    torch.library.opcheck(torch.ops.mmt.prroi_pool_forward.default, (f, rois, 4, 4, 1.0))


def test_opcheck_mam_attention():
    import mmt_amd.ops  # noqa: F401
    g = torch.Generator().manual_seed(2)
    qkv = torch.randn(2, 100, 3 * 128, generator=g).bfloat16().cuda().requires_grad_(True)
    torch.library.opcheck(torch.ops.mmt.mam_attention_forward.default, (qkv, 36, 2))


def test_registered_autograd_equals_function():
    """Gradients through the ops' registered autograd == through the autograd.Function drop-ins."""
    from mmt_amd import ops
    from mmt_amd.functional import MSDeformAttnFunction, prroi_pool2d
    value, shapes, starts, loc, aw = _msda_inputs(torch.float64, seed=3)
    go = torch.randn(2, 5, 16, dtype=torch.float64, device="cuda")
    grads = []
    for fn in (lambda *a: ops.ms_deform_attn(*a), lambda *a: MSDeformAttnFunction.apply(*a, 64)):
        v, lo, a_ = [x.detach().clone().requires_grad_(True) for x in (value, loc, aw)]
        (fn(v, shapes, starts, lo, a_) * go).sum().backward()
        grads.append([v.grad, lo.grad, a_.grad])
    for x, y in zip(*grads):
        assert torch.allclose(x, y, rtol=0, atol=1e-14)
    f = torch.randn(1, 3, 8, 8, device="cuda")
    rois = torch.tensor([[0, 0.5, 1.0, 6.5, 7.0]], device="cuda")
    gr = []
    for fn in (ops.prroi_pool2d, prroi_pool2d):
        ff, rr = f.clone().requires_grad_(True), rois.clone().requires_grad_(True)
        fn(ff, rr, 2, 2, 1.0).square().sum().backward()
        gr.append((ff.grad, rr.grad))
    assert torch.equal(gr[0][0], gr[1][0]) and torch.equal(gr[0][1], gr[1][1])
