#!/usr/bin/env python3
"""Per-phase timing of the MAM impl 24 / 25 kernels from in-kernel timestamps (stamp build of
tools/build_ablate.sh): per workgroup (wave 0) prologue, main loop (cycles per 32-key block), last block
+ epilogue.  usage: MMT_HIP_LIB=.../_lib/stamp/libmmt_hip.so python tools/attn_pp_stamps.py --batch 4"""
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
ap.add_argument("--batch", type=int, default=4)
ap.add_argument("--impls", default="24,25")
args = ap.parse_args()
L.LIB.mmt_attn_pp_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
B, ntok, n_t, C, H = args.batch, 528, 128, 768, 12
S = 2 * B
qkv = (torch.randn(S * ntok, 3 * C, device="cuda") * 0.7).bfloat16()
out = torch.empty(S * ntok, C, device="cuda", dtype=torch.bfloat16)
for asym in (0, 1):
    for impl in [int(x) for x in args.impls.split(",")]:
        p = L.AttnParams()
        p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym, p.scale = (
            qkv.data_ptr(), out.data_ptr(), S, B, ntok, n_t, C, H, asym, 1.0 / 1.4426950408889634)
        p.impl = impl
        for _ in range(3):
            L.check(L.LIB.mmt_mam_attention(ctypes.byref(p), L.MMT_BF16, torch.cuda.current_stream().cuda_stream), "attn")
        torch.cuda.synchronize()
        nwg = (1 + 4) * H * S
        buf = (ctypes.c_ulonglong * (nwg * 8))()
        L.check(L.LIB.mmt_attn_pp_stamps(buf, nwg * 8), "stamps")
        st = np.frombuffer(buf, dtype=np.uint64).reshape(nwg, 8).astype(np.int64)
        freq = float(np.median((st[:, 4] - st[:, 1]) / np.maximum(st[:, 5] - st[:, 0], 1))) * 100.0  # MHz
        row = {"asym": asym, "impl": impl, "B": B, "clock_mhz": round(freq)}
        for kind, sel in (("search2", (st[:, 6] >= 10) & (st[:, 7] == 2)), ("tmpl", st[:, 6] <= 4)):
            x = st[sel]
            if not len(x):
                continue
            nb = np.median(x[:, 6])
            loop_blocks = max(nb - 2, 1)  # the loop covers blocks 1 .. nb - 2 (block 0 before it, the last after)
            row[kind] = {"n": int(len(x)), "blocks": int(nb),
                         "prologue_cyc": int(np.median(x[:, 2] - x[:, 1])),
                         "loop_cyc_per_block": int(np.median(x[:, 3] - x[:, 2]) / (loop_blocks + 1)),
                         "tail_cyc": int(np.median(x[:, 4] - x[:, 3])),
                         "total_us": round(float(np.median(x[:, 4] - x[:, 1])) / freq, 2)}
        rt = st[:, 0]
        row["span_us"] = round(float(st[:, 5].max() - rt.min()) / 100.0, 2)
        print(json.dumps(row), flush=True)
