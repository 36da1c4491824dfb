#!/usr/bin/env python3
"""A/B timing of the bf16 MAM attention kernels (mmt_attn_params.impl 2 / 4 = latency kernel with
2 / 4 key groups, 8 = throughput kernel, 0 = library's choice) at the hot path's shapes and several
batch sizes: back-to-back launches in one hipGraph, timed with HIP events (device time).
FLOPs per launch = 4 * d * H * S * (n_t^2 + n_s * Lk_search).

usage: python tools/attn_ab.py [--batches 1,4,8,32] [--impls 4,8,0]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))
import torch  # noqa: E402

from mmt_amd import _lib as L  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tools"))
from gemm_ab import graph_time  # noqa: E402


def flops(S, H, ntok, n_t, asym, d=64):
    ns = ntok - n_t
    lk = ntok + n_t if asym else ntok
    return 4.0 * d * H * S * (n_t * n_t + ns * lk)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,2,4,8,16,32")
    ap.add_argument("--impls", default="4,8,0")
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--vitl", action="store_true", help="ViT-L 192/384 shape (ntok 864, n_t 288, H 16)")
    args = ap.parse_args()
    ntok, n_t, H = (864, 288, 16) if args.vitl else (528, 128, 12)
    C = 64 * H
    for asym in (0, 1):
        for B in [int(x) for x in args.batches.split(",")]:
            S = 2 * B
            qkv = (torch.randn(S, ntok, 3 * C, device="cuda") * 0.7).bfloat16()
            out = torch.empty(S, ntok, C, device="cuda", dtype=torch.bfloat16)
            fl = flops(S, H, ntok, n_t, asym)
            row = {"B": B, "asym": asym, "gflop": round(fl / 1e9, 3)}
            ref = None
            for impl in [int(x) for x in args.impls.split(",")]:
                p = L.AttnParams()
                p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym = (qkv.data_ptr(), out.data_ptr(), S, B, ntok,
                                                                         n_t, C, H, asym)
                p.scale, p.impl = 1.0 / 1.4426950408889634, impl
                fn = lambda: L.check(L.LIB.mmt_mam_attention(L.ctypes.byref(p), L.MMT_BF16,  # noqa: E731
                                                             torch.cuda.current_stream().cuda_stream), "attn")
                us = graph_time(fn, args.reps)
                o = out.float()
                diff = 0.0 if ref is None else (o - ref).abs().max().item()
                ref = o if ref is None else ref
                row["impl%d" % impl] = {"us": round(us, 2), "tflops": round(fl / us / 1e6, 1),
                                        "frac": round(fl / us / 1e6 / 2500.0, 4), "maxdiff": float("%.2e" % diff)}
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
