#!/usr/bin/env python3
"""Device time of the training forward's MAM attention (with the log-sum-exp the backward reads) at the training
shape (32 sequences, 528 tokens, 128 template, 12 heads) per forced kernel impl: 8 (the running-maximum throughput
kernel, the auto choice before round 6), 17 / 21 (the range-checked exponent kernels, 21 software-pipelined).
HIP events around 20 launches; the output / lse checksums are printed so the impls can be compared."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "multi-modal-tracking_amd"))
import torch  # noqa: E402


def main(S=32, ntok=528, n_t=128, H=12):
    from mmt_amd import _lib as L
    C = 64 * H
    g = torch.Generator().manual_seed(0)
    qkv = (torch.randn(S, ntok, 3 * C, generator=g) * 0.5).bfloat16().cuda()
    st = torch.cuda.current_stream().cuda_stream
    for impl in (8, 17, 21, 8, 17, 21):
        out = torch.empty(S, ntok, C, device="cuda", dtype=torch.bfloat16)
        lse = torch.empty(S, H, ntok, device="cuda", dtype=torch.float32)
        p = L.AttnParams()
        p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym = qkv.data_ptr(), out.data_ptr(), S, S, ntok, n_t, C, H, 0
        p.scale, p.impl, p.lse = 0.125, impl, lse.data_ptr()
        for _ in range(3):
            L.check(L.LIB.mmt_mam_attention(p, L.MMT_BF16, st), "fwd")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            L.check(L.LIB.mmt_mam_attention(p, L.MMT_BF16, st), "fwd")
        e1.record()
        torch.cuda.synchronize()
        print("impl %d: %.1f us, out checksum %.4f, lse checksum %.4f" % (impl, e0.elapsed_time(e1) * 1e3 / 20,
                                                                      out.float().abs().sum().item(), lse.sum().item()))


if __name__ == "__main__":
    main()
