#!/usr/bin/env python3
"""Per-phase timing of the ping-pong MAM kernel (impl 28) from in-kernel timestamps (stamp build of
tools/build_ablate.sh): per workgroup (wave 0) prologue, block loop (cycles per 32-key block, i.e. per two
segment intervals), epilogue, split by search / template workgroups, plus the launch span.
usage: MMT_HIP_LIB=.../_lib/stamp/libmmt_hip.so python tools/pg_stamps.py --batches 8,32"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mmt_amd import _lib as L  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batches", default="8,32")
ap.add_argument("--label", default="")
args = ap.parse_args()
L.LIB.mmt_attn_pg_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
HAS_SEG = hasattr(L.LIB, "mmt_attn_pg_seg")
if HAS_SEG:
    L.LIB.mmt_attn_pg_seg.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
ntok, n_t, C, H = 528, 128, 768, 12
for B in [int(b) for b in args.batches.split(",")]:
    S = 2 * B
    qkv = (torch.randn(S * ntok, 3 * C, device="cuda") * 0.5).bfloat16()
    out = torch.empty(S * ntok, C, device="cuda", dtype=torch.bfloat16)
    for asym in (0, 1):
        p = L.AttnParams()
        p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym, p.scale = (
            qkv.data_ptr(), out.data_ptr(), S, B, ntok, n_t, C, H, asym, 1.0 / 1.4426950408889634)
        p.impl = 28
        for _ in range(20):
            L.check(L.LIB.mmt_mam_attention(ctypes.byref(p), L.MMT_BF16, torch.cuda.current_stream().cuda_stream), "attn")
        torch.cuda.synchronize()
        nwg = S * H + (S * H + 3) // 4
        buf = (ctypes.c_ulonglong * (nwg * 8))()
        L.check(L.LIB.mmt_attn_pg_stamps(buf, nwg * 8), "stamps")
        st = np.frombuffer(buf, dtype=np.uint64).reshape(nwg, 8).astype(np.int64)
        freq = float(np.median((st[:, 4] - st[:, 1]) / np.maximum(st[:, 5] - st[:, 0], 1))) * 100.0  # MHz
        row = {"label": args.label, "B": B, "asym": asym, "clock_mhz": round(freq),
               "span_us": round(float(st[:, 5].max() - st[:, 0].min()) / 100.0, 2)}
        for kind, sel in (("search", st[:, 6] < 1000), ("tmpl", st[:, 6] >= 1000)):
            x = st[sel]
            nb = int(np.median(x[:, 6] % 1000))
            row[kind] = {"n": int(len(x)), "blocks": nb,
                         "prologue_cyc": int(np.median(x[:, 2] - x[:, 1])),
                         "loop_cyc_per_block": int(np.median(x[:, 3] - x[:, 2]) / nb),
                         "w4_loop_cyc_per_block": int(np.median(x[:, 7] - x[:, 2]) / nb),
                         "epilogue_cyc": int(np.median(x[:, 4] - x[:, 3])),
                         "total_us": round(float(np.median(x[:, 4] - x[:, 1])) / freq, 2),
                         "start_spread_us": round(float(np.percentile(x[:, 0], 90) - np.percentile(x[:, 0], 10)) / 100, 2)}
        if HAS_SEG:
            sb = (ctypes.c_ulonglong * (nwg * 16))()
            L.check(L.LIB.mmt_attn_pg_seg(sb, nwg * 16), "seg")
            sg = np.frombuffer(sb, dtype=np.uint64).reshape(nwg, 16).astype(np.int64)[st[:, 6] < 1000]
            base = sg[:, 0:1]
            rel = np.median(sg - base, axis=0).astype(int).tolist()
            # per wave: [X6 start, X6 end, Y6 start, Y6 end, X7 start, X7 end, Y7 start, Y7 end] rel. to w0's X6 start
            row["seg_w0"] = rel[:8]
            row["seg_w4"] = rel[8:]
        print(json.dumps(row), flush=True)
