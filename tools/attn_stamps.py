#!/usr/bin/env python3
"""Per-phase timing of the bf16 MAM attention kernel from in-kernel timestamps (stamp build of
tools/build_ablate.sh), plus its graph-replayed launch time.  Phases per workgroup (leader thread):
prologue = start -> first K/V tile landed, loop = the key tiles, epilogue = normalise + stores.

usage: MMT_HIP_LIB=.../_lib/stamp/libmmt_hip.so python tools/attn_stamps.py [--batch 1]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mmt_amd import _lib as L  # noqa: E402
from gemm_ab import graph_time  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    args = ap.parse_args()
    has_stamps = hasattr(L.LIB, "mmt_attn_stamps")
    if has_stamps:
        L.LIB.mmt_attn_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    B, ntok, n_t, C, H = args.batch, 528, 128, 768, 12
    S = 2 * B
    qkv = torch.randn(S * ntok, 3 * C, device="cuda").bfloat16()
    out = torch.empty(S * ntok, C, device="cuda", dtype=torch.bfloat16)
    for asym, impl in ((0, 4), (1, 4)):
        p = L.AttnParams()
        p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym, p.scale = (
            qkv.data_ptr(), out.data_ptr(), S, B, ntok, n_t, C, H, asym, 0.125)
        p.impl = impl
        fn = lambda: L.check(L.LIB.mmt_mam_attention(ctypes.byref(p), L.MMT_BF16,  # noqa: E731
                                                      torch.cuda.current_stream().cuda_stream), "attn")
        us = graph_time(fn, 200)
        lk_s = ntok + (n_t if asym else 0)
        flops = 4.0 * 64 * H * S * (n_t * n_t + (ntok - n_t) * lk_s)
        row = {"asym": asym, "impl": impl, "B": B, "graph_us": round(us, 2), "tflops": round(flops / us / 1e6, 1)}
        if has_stamps:
            fn()
            torch.cuda.synchronize()
            nqb = (n_t + 63) // 64 + (ntok - n_t + 63) // 64
            nwg = nqb * H * S
            buf = (ctypes.c_ulonglong * (nwg * 8))()
            L.check(L.LIB.mmt_attn_stamps(buf, nwg * 8), "stamps")
            st = np.frombuffer(buf, dtype=np.uint64).reshape(S, H, nqb, 8).astype(np.int64)
            freq = float(np.median((st[..., 4] - st[..., 1]) / np.maximum(st[..., 5] - st[..., 0], 1))) * 100.0
            for kind, sl in (("tmpl", slice(0, (n_t + 63) // 64)), ("search", slice((n_t + 63) // 64, nqb))):
                x = st[:, :, sl].reshape(-1, 8)
                row[kind] = {"prologue_us": round(float(np.median(x[:, 2] - x[:, 1])) / freq, 2),
                             "loop_us": round(float(np.median(x[:, 3] - x[:, 2])) / freq, 2),
                             "epilogue_us": round(float(np.median(x[:, 4] - x[:, 3])) / freq, 2),
                             "total_max_us": round(float(np.max(x[:, 4] - x[:, 1])) / freq, 2)}
            rt = st[..., 0].reshape(-1)
            row["start_spread_us"] = round(float(rt.max() - rt.min()) / 100.0, 2)
            row["span_us"] = round(float(st[..., 5].max() - rt.min()) / 100.0, 2)
            row["clock_mhz"] = round(freq)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
