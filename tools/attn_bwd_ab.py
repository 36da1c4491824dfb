#!/usr/bin/env python3
"""Device time of the MAM attention backward (mmt_mam_attention_bwd: dq + dkv kernels) at the training step's shape
(32 sequences = 16 pairs x 2 modalities, 528 tokens, 128 template, 12 heads), HIP events around 20 calls; run once
per library (MMT_HIP_LIB) to compare builds.  Prints a checksum of dQKV so that builds can be checked for equality."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "multi-modal-tracking_amd"))
import torch  # noqa: E402


def main(S=32, ntok=528, n_t=128, H=12):
    from mmt_amd import _lib as L
    C = 64 * H
    g = torch.Generator().manual_seed(0)
    qkv = (torch.randn(S, ntok, 3 * C, generator=g) * 0.5).bfloat16().cuda()
    dout = torch.randn(S, ntok, C, generator=g).bfloat16().cuda()
    out = torch.empty(S, ntok, C, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(S, H, ntok, device="cuda", dtype=torch.float32)
    p = L.AttnParams()
    p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym = qkv.data_ptr(), out.data_ptr(), S, S, ntok, n_t, C, H, 0
    p.scale, p.impl, p.lse = 0.125, 0, lse.data_ptr()
    st = torch.cuda.current_stream().cuda_stream
    L.check(L.LIB.mmt_mam_attention(p, L.MMT_BF16, st), "fwd")
    delta = torch.empty(S, H, ntok, device="cuda", dtype=torch.float32)
    dqkv = torch.empty_like(qkv)
    b = L.AttnBwdParams()
    b.qkv, b.out, b.dout, b.lse, b.delta, b.dqkv = (qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(),
                                                    delta.data_ptr(), dqkv.data_ptr())
    b.S, b.Bm, b.ntok, b.n_t, b.C, b.H, b.asym, b.scale = S, S, ntok, n_t, C, H, 0, 0.125
    for _ in range(3):
        L.check(L.LIB.mmt_mam_attention_bwd(b, L.MMT_BF16, st), "bwd")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        L.check(L.LIB.mmt_mam_attention_bwd(b, L.MMT_BF16, st), "bwd")
    e1.record()
    torch.cuda.synchronize()
    print("%s: backward %.1f us per call, dqkv checksum %.6f" % (os.environ.get("MMT_HIP_LIB", "product"),
                                                              e0.elapsed_time(e1) * 1e3 / 20, dqkv.float().abs().sum().item()))


if __name__ == "__main__":
    main()
