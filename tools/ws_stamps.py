#!/usr/bin/env python3
"""Per-phase cycles of the whole-sequence MAM attention kernel (impl 20-23) from in-kernel stamps
(stamp build of tools/build_ablate.sh): per workgroup, waves 0 and 4 record s_memtime at the start,
after the first barrier (prologue: Q + first tiles landed), after each key tile, and at the end.
usage: MMT_HIP_LIB=.../_lib/stamp/libmmt_hip.so python tools/ws_stamps.py [--batch 32] [--impl 22]"""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--impls", default="22,23")
    ap.add_argument("--asym", type=int, default=0)
    a = ap.parse_args()
    L.LIB.mmt_ws_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    B, ntok, n_t, C, H = a.batch, 528, 128, 768, 12
    S = 2 * B
    qkv = (torch.randn(S * ntok, 3 * C, device="cuda") * 0.7).bfloat16()
    out = torch.empty(S * ntok, C, device="cuda", dtype=torch.bfloat16)
    for impl in [int(x) for x in a.impls.split(",")]:
        p = L.AttnParams()
        p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym = qkv.data_ptr(), out.data_ptr(), S, B, ntok, n_t, C, H, a.asym
        p.scale, p.impl = 1.0 / 1.4426950408889634, impl
        for _ in range(30):  # warm clocks
            L.check(L.LIB.mmt_mam_attention(ctypes.byref(p), L.MMT_BF16, torch.cuda.current_stream().cuda_stream), "attn")
        torch.cuda.synchronize()
        nwg = H * S
        buf = (ctypes.c_ulonglong * (nwg * 2 * 16))()
        L.check(L.LIB.mmt_ws_stamps(buf, nwg * 32), "stamps")
        st = np.frombuffer(buf, dtype=np.uint64).reshape(nwg, 2, 16).astype(np.int64)
        clk = float(np.median((st[:, 0, 14] - st[:, 0, 1]) / np.maximum(st[:, 0, 15] - st[:, 0, 0], 1))) * 100.0  # MHz
        row = {"impl": impl, "B": B, "asym": a.asym, "clock_mhz": round(clk)}
        for wv in (0, 1):
            x = st[:, wv]
            row["wave%d" % (4 * wv)] = {
                "prologue_cyc": int(np.median(x[:, 2] - x[:, 1])),
                "tile_cyc": [int(np.median(x[:, 3 + t] - x[:, 2 + t])) for t in range(8)],
                "total_cyc": int(np.median(x[:, 14] - x[:, 1])),
            }
        t0 = st[:, 0, 0]
        row["wg_start_spread_us"] = round(float(t0.max() - t0.min()) / 100.0, 2)
        row["kernel_span_us"] = round(float(st[:, 0, 15].max() - t0.min()) / 100.0, 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
