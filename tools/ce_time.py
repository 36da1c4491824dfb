#!/usr/bin/env python3
"""Device time of the candidate-elimination kernels at the B=1 / B=8 stage-0 shapes (ViT-B, 400 search
tokens per modality, keep 280): each entry point launched back to back in one hipGraph, HIP events."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from gemm_ab import graph_time  # noqa: E402
from mmt_amd._lib import LIB, MMT_BF16, check  # noqa: E402

for B in (1, 8):
    S, ntok, n_t, k, keep, H, C = 2 * B, 528, 128, 400, 280, 12, 768
    nparts = H * (2 * n_t // 16)
    qkv = (torch.randn(S, ntok, 3 * C, device="cuda") * 0.5).bfloat16()
    part = torch.empty(B * nparts * 2 * k, device="cuda")
    g0 = torch.empty(S, k, dtype=torch.int32, device="cuda")
    order = torch.empty_like(g0)
    X, XC = torch.randn(S * ntok, C, device="cuda"), torch.empty(S * ntok, C, device="cuda")
    XN = torch.empty(S * ntok, C, device="cuda", dtype=torch.bfloat16)
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    fns = {
        "t2s": lambda: check(LIB.mmt_ce_t2s_attention(qkv.data_ptr(), part.data_ptr(), B, ntok, n_t, k, C, H, 0.125,
                                                      MMT_BF16, st()), "t2s"),
        "select": lambda: check(LIB.mmt_ce_select(part.data_ptr(), nparts, B, k, keep, k, None, g0.data_ptr(),
                                                  order.data_ptr(), None, 1.0, st()), "select"),
        "gather": lambda: check(LIB.mmt_ce_gather(X.data_ptr(), XC.data_ptr(), XN.data_ptr(), order.data_ptr(), S, ntok,
                                                  n_t, keep, k, C, MMT_BF16, st()), "gather"),
    }
    fns["t2s"]()
    fns["select"]()
    for nm, fn in fns.items():
        print("B=%d %s %.2f us" % (B, nm, graph_time(fn, 200)), flush=True)
