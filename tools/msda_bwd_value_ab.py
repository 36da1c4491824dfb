#!/usr/bin/env python3
"""Device time of the drop-in MSDA backward (mmt_ms_deform_attn_backward_impl, fp32) at the training shape of 16 pairs
(N 16, 400 queries, 8 heads x 64, two 20 x 20 levels, 4 points): the 64-pixel-chunk value gather (value_impl 1)
vs one workgroup per (n, m, level) (value_impl 2).  HIP events around 20 launches of the whole backward (the
sample kernel included) and rocprof-style per-kernel times are left to rocprofv3."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "multi-modal-tracking_amd"))
import torch  # noqa: E402
from mmt_amd import _lib as L  # noqa: E402


def main(N=16, Lq=400, M=8, D=64, hw=20, P=4):
    shapes = [(hw, hw), (hw, hw)]
    S = 2 * hw * hw
    v = torch.rand(N, S, M, D, device="cuda")
    loc = torch.rand(N, Lq, M, 2, P, 2, device="cuda") * 1.2 - 0.1
    w = torch.rand(N, Lq, M, 2, P, device="cuda")
    go = torch.randn(N, Lq, M * D, device="cuda")
    sh = torch.tensor(shapes, dtype=torch.long, device="cuda")
    st = torch.tensor([0, hw * hw], dtype=torch.long, device="cuda")
    gv, gl, ga = torch.empty_like(v), torch.empty_like(loc), torch.empty_like(w)
    stream = torch.cuda.current_stream().cuda_stream
    for impl in (1, 2, 1, 2):
        def run():
            L.check(L.LIB.mmt_ms_deform_attn_backward_impl(v.data_ptr(), sh.data_ptr(), st.data_ptr(), loc.data_ptr(),
                                                           w.data_ptr(), go.data_ptr(), gv.data_ptr(), gl.data_ptr(),
                                                           ga.data_ptr(), N, S, M, D, Lq, 2, P, hw * hw, impl, L.MMT_F32,
                                                           stream), "bwd")
        for _ in range(3):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            run()
        e1.record()
        torch.cuda.synchronize()
        print("value_impl %d: whole backward %.1f us per call" % (impl, e0.elapsed_time(e1) * 1e3 / 20))


if __name__ == "__main__":
    main()
