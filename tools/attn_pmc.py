#!/usr/bin/env python3
"""Drive only the bf16 MAM attention kernel (direct launches, no graph) for rocprofv3 --pmc passes:
python tools/attn_pmc.py [--batch 32] [--impl 0] [--launches 20] [--asym 0]"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))
import torch  # noqa: E402

from mmt_amd import _lib as L  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--impl", type=int, default=0)
ap.add_argument("--launches", type=int, default=20)
ap.add_argument("--asym", type=int, default=0)
a = ap.parse_args()
ntok, n_t, H = 528, 128, 12
C, S = 64 * H, 2 * a.batch
qkv = (torch.randn(S, ntok, 3 * C, device="cuda") * 0.7).bfloat16()
out = torch.empty(S, ntok, C, device="cuda", dtype=torch.bfloat16)
p = L.AttnParams()
p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym = qkv.data_ptr(), out.data_ptr(), S, a.batch, ntok, n_t, C, H, a.asym
p.scale, p.impl = 1.0 / 1.4426950408889634, a.impl
for _ in range(a.launches):
    L.check(L.LIB.mmt_mam_attention(ctypes.byref(p), L.MMT_BF16, torch.cuda.current_stream().cuda_stream), "attn")
torch.cuda.synchronize()
print("ok")
