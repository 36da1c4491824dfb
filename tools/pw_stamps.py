#!/usr/bin/env python3
"""Per-pair timing of the persistent whole-pair MAM kernel (impl 20) from in-kernel timestamps
(stamp build of tools/build_ablate.sh, shader cycles: prologue, the first step, the
steady steps, the partial last step and the output stores of each workgroup's first pair), plus the graph-replayed launch time of the library the run loads (MMT_HIP_LIB: the
ablation builds aab1/2/3 time the kernel without DMA refills / compute / exponentials).

usage: MMT_HIP_LIB=.../_lib/stamp/libmmt_hip.so python tools/pw_stamps.py [--batches 1,8,32]
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
    ap.add_argument("--batches", default="1,8,32")
    ap.add_argument("--impl", type=int, default=20)
    args = ap.parse_args()
    has_stamps = hasattr(L.LIB, "mmt_attn_stamps")
    if has_stamps:
        L.LIB.mmt_attn_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    ntok, n_t, C, H = 528, 128, 768, 12
    for B in [int(x) for x in args.batches.split(",")]:
        S = 2 * B
        qkv = (torch.randn(S * ntok, 3 * C, device="cuda") * 0.5).bfloat16()
        out = torch.empty(S * ntok, C, device="cuda", dtype=torch.bfloat16)
        for asym in (0, 1):
            p = L.AttnParams()
            p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym, p.scale = (
                qkv.data_ptr(), out.data_ptr(), S, B, ntok, n_t, C, H, asym, 0.125)
            p.impl = args.impl
            fn = lambda: L.check(L.LIB.mmt_mam_attention(ctypes.byref(p), L.MMT_BF16,  # noqa: E731
                                                          torch.cuda.current_stream().cuda_stream), "attn")
            us = graph_time(fn, 200)
            lk_s = ntok + (n_t if asym else 0)
            flops = 4.0 * 64 * H * S * (n_t * n_t + (ntok - n_t) * lk_s)
            row = {"B": B, "asym": asym, "impl": args.impl, "graph_us": round(us, 2), "tflops": round(flops / us / 1e6, 1)}
            if has_stamps and args.impl == 20:
                fn()
                torch.cuda.synchronize()
                npairs = S * H
                G = min(npairs, ncu)
                buf = (ctypes.c_ulonglong * (G * 8))()
                L.check(L.LIB.mmt_attn_stamps(buf, G * 8), "stamps")
                st = np.frombuffer(buf, dtype=np.uint64).reshape(G, 8).astype(np.int64)
                npk = (npairs - np.arange(G) + G - 1) // G
                row["pairs_per_wg"] = sorted(set(npk.tolist()))
                d = np.median(st[:, 1:7] - st[:, 0:6], axis=0)
                row["pair0_cycles"] = {"prologue": int(d[0]), "step0": int(d[1]), "steps1_3_each": int(d[2] / 3),
                                       "steps4_7_each": int(d[3] / 4), "tail_step": int(d[4]), "finish": int(d[5])}
                row["wg_total_cycles_max"] = int((st[:, 7] - st[:, 0]).max())
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
