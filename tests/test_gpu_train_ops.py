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


def _run_fwd_bwd(qkv, dout, S, ntok, n_t, H):
    L = _lib()
    C = 64 * H
    out = torch.empty(S, ntok, C, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(S, H, ntok, device="cuda")
    p = L.AttnParams()
    p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym = qkv.data_ptr(), out.data_ptr(), S, S // 2, ntok, n_t, C, H, 0
    p.scale, p.impl, p.lse = 0.125, 0, lse.data_ptr()
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


@pytest.mark.parametrize("S,ntok,n_t,H", [(2, 528, 128, 12), (4, 100, 36, 2), (2, 70, 8, 1), (2, 864, 288, 2)])
def test_attention_backward(S, ntok, n_t, H):
    C = 64 * H
    g = torch.Generator().manual_seed(ntok + H)
    qkv = torch.randn(S, ntok, 3 * C, generator=g).bfloat16()
    dout = torch.randn(S, ntok, C, generator=g).bfloat16()
    out, lse, dqkv = _run_fwd_bwd(qkv.cuda(), dout.cuda(), S, ntok, n_t, H)
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
