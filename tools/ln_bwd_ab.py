#!/usr/bin/env python3
"""Device time of the pair LayerNorm backward with the residual gradient (mmt_layernorm_bwd_add) at the training
step's shape (16896 rows = 2 x 16 x 528, C 768, bf16 dy, two affine sets alternating every 8448 rows), HIP events
around 50 calls; run once per library (MMT_HIP_LIB) to compare builds (dx checksum printed)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "multi-modal-tracking_amd"))
import torch  # noqa: E402


def main(rows=16896, C=768):
    from mmt_amd import _lib as L
    g = torch.Generator().manual_seed(0)
    x = torch.randn(rows, C, generator=g).cuda()
    dy = torch.randn(rows, C, generator=g).bfloat16().cuda()
    dres = torch.randn(rows, C, generator=g).cuda()
    g0, g1 = torch.rand(C, generator=g).cuda(), torch.rand(C, generator=g).cuda()
    nws = (rows + 31) // 32 * 4 * C
    dx = torch.empty(rows, C, device="cuda")
    ws = torch.empty(nws, device="cuda")
    dgb = torch.empty(4, C, device="cuda")
    st = torch.cuda.current_stream().cuda_stream

    def run():
        L.check(L.LIB.mmt_layernorm_bwd_add(x.data_ptr(), dy.data_ptr(), L.MMT_BF16, g0.data_ptr(), g1.data_ptr(),
                                            dres.data_ptr(), dx.data_ptr(), dgb.data_ptr(), 0, ws.data_ptr(), nws, rows,
                                            rows // 2, C, 1e-6, st), "ln bwd")
    for _ in range(3):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 50
    print("%s: LN backward %.1f us per call (%.2f TB/s on x, dy, dres, dx), checksum %.4f" % (
        os.environ.get("MMT_HIP_LIB", "product"), us, rows * C * (4 + 2 + 4 + 4) / us / 1e6, dx.abs().sum().item()))


if __name__ == "__main__":
    main()
