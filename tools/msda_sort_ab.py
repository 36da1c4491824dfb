#!/usr/bin/env python3
"""Device time of the MSDA value gathers on spread-out and on collapsed sampling locations (every sample of a level
near one point: four pixels take all 1600 taps of a (batch, head, level)), at the training shape of 16 pairs
(N 16, 400 queries, 8 heads x 64, two 20 x 20 levels, 4 points):
* the drop-in backward (mmt_ms_deform_attn_backward_impl, fp32), value_impl 1 (64-pixel chunks) and 2 (per level);
* the training op's backward (mmt_msda_bimodal_train_bwd, bf16).
HIP events around 20 calls each.  Run once per library (MMT_HIP_LIB) to A/B the bucket placement."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "multi-modal-tracking_amd"))
import torch  # noqa: E402
from mmt_amd import _lib as L  # noqa: E402


def timed(fn, n=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def main(N=16, Lq=400, M=8, D=64, hw=20, P=4):
    from mmt_amd.train import _ref_points
    g = torch.Generator(device="cuda").manual_seed(0)
    S, nq = 2 * hw * hw, hw * hw
    v = torch.rand(N, S, M, D, device="cuda", generator=g)
    locs = {"spread": torch.rand(N, Lq, M, 2, P, 2, device="cuda", generator=g) * 1.2 - 0.1,
            "collapsed": 0.4737 + (torch.rand(N, Lq, M, 2, P, 2, device="cuda", generator=g) - 0.5) * 2e-3}
    w = torch.rand(N, Lq, M, 2, P, device="cuda", generator=g)
    go = torch.randn(N, Lq, M * D, device="cuda", generator=g)
    sh = torch.tensor([(hw, hw)] * 2, dtype=torch.long, device="cuda")
    st = torch.tensor([0, hw * hw], dtype=torch.long, device="cuda")
    gv, gl, ga = torch.empty_like(v), torch.empty_like(locs["spread"]), torch.empty_like(w)
    stream = torch.cuda.current_stream().cuda_stream
    rows = []
    for kind, loc in locs.items():
        for impl in (1, 2):
            def run():
                L.check(L.LIB.mmt_ms_deform_attn_backward_impl(v.data_ptr(), sh.data_ptr(), st.data_ptr(), loc.data_ptr(),
                                                               w.data_ptr(), go.data_ptr(), gv.data_ptr(), gl.data_ptr(),
                                                               ga.data_ptr(), N, S, M, D, Lq, 2, P, nq, impl, L.MMT_F32,
                                                               stream), "bwd")
            rows.append({"op": "drop-in backward", "value_impl": impl, "locations": kind, "us": round(timed(run), 1)})
    # the training op: offsets such that loc = ref + off / hw is spread (randn * 2) or near (0.4737, 0.4737)
    ref_q = _ref_points(hw, hw, 1, 2, "cuda")[0, :nq, 0, :].contiguous()
    value = torch.randn(N, 2 * nq, 512, device="cuda", generator=g).bfloat16()
    awl = torch.randn(N, nq, 64, device="cuda", generator=g).bfloat16()
    gout = torch.randn(N, nq, 512, device="cuda", generator=g).bfloat16()
    offs = {"spread": (torch.randn(N, nq, 128, device="cuda", generator=g) * 2).bfloat16(),
            "collapsed": ((0.4737 - ref_q.view(1, nq, 1, 1, 1, 2)) * hw
                          + torch.zeros(N, nq, 8, 2, 4, 2, device="cuda")).reshape(N, nq, 128).bfloat16()}
    gvalue, goff, gawl = torch.empty_like(value), torch.empty(N, nq, 128, device="cuda").bfloat16(), torch.empty_like(awl)
    for kind, off in offs.items():
        def run_t():
            L.check(L.LIB.mmt_msda_bimodal_train_bwd(value.data_ptr(), off.data_ptr(), 128, awl.data_ptr(), 64,
                                                     ref_q.data_ptr(), gout.data_ptr(), gvalue.data_ptr(),
                                                     goff.data_ptr(), gawl.data_ptr(), N, hw, stream), "train bwd")
        rows.append({"op": "training op backward", "locations": kind, "us": round(timed(run_t), 1)})
    lib = os.environ.get("MMT_HIP_LIB", "product")
    for r in rows:
        r["lib"] = lib
        print(json.dumps(r))


if __name__ == "__main__":
    main()
