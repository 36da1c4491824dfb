#!/usr/bin/env python3
"""Device time of the training head's batch norm (mmt_batchnorm_relu + _bwd, training statistics) at the head's map
shapes (16 pairs: 20 / 40 / 80-pixel maps), HIP events around 20 forward + backward pairs per shape; run once per
library (MMT_HIP_LIB) to compare builds (output checksums printed)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "multi-modal-tracking_amd"))
import torch  # noqa: E402

SHAPES = [(16 * 400, 384, 384), (16 * 1600, 192, 192), (16 * 6400, 96, 96), (16 * 6400, 48, 48), (16 * 1600, 1, 8)]


def main():
    from mmt_amd import _lib as L
    st = torch.cuda.current_stream().cuda_stream
    tot, cs = 0.0, 0.0
    for M, C, pitch in SHAPES:
        g = torch.Generator().manual_seed(M + C)
        x = torch.randn(M, pitch, generator=g).bfloat16().cuda()
        dy = torch.randn(M, pitch, generator=g).bfloat16().cuda()
        y, dx = torch.empty_like(x), torch.empty_like(x)
        w, b = torch.rand(C, generator=g).cuda(), torch.rand(C, generator=g).cuda()
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        save = torch.empty(4, C, device="cuda")
        nws = int(L.LIB.mmt_batchnorm_ws_floats(M, C))
        ws, ws2 = torch.empty(nws, device="cuda"), torch.empty(nws, device="cuda")
        dgb = torch.empty(2, C, device="cuda")

        def run():
            L.check(L.LIB.mmt_batchnorm_relu(x.data_ptr(), y.data_ptr(), M, C, pitch, w.data_ptr(), b.data_ptr(),
                                             rm.data_ptr(), rv.data_ptr(), 0.1, 1e-5, 1, 1, save.data_ptr(), ws.data_ptr(),
                                             nws, st), "bn")
            L.check(L.LIB.mmt_batchnorm_relu_bwd(x.data_ptr(), dy.data_ptr(), dx.data_ptr(), M, C, pitch, w.data_ptr(),
                                                 save.data_ptr(), 1, 1, dgb.data_ptr(), ws2.data_ptr(), nws, st), "bn bwd")
        for _ in range(3):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 20
        tot += us
        cs += y.float().abs().sum().item() + dx.float().abs().sum().item() + dgb.abs().sum().item()
        print("M %d C %d: fwd + bwd %.1f us" % (M, C, us))
    print("%s: total %.1f us, checksum %.6f" % (os.environ.get("MMT_HIP_LIB", "product"), tot, cs))


if __name__ == "__main__":
    main()
