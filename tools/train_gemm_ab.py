#!/usr/bin/env python3
"""A/B of tile config / K-split choices for the training step's gradient GEMMs as the lockstep backbones issue
them (mmt_amd.train._gemm: 16 pairs, two groups of 8448 rows): dW = dY^T [X | 1] (A and W MN-major, fp32 out
with the bias column block, split-K workspace) and dX = dY W (W MN-major, bf16 out; fc2's with the GELU
backward), per ViT Linear.  Each (impl, nsk) is timed as back-to-back launches in one hipGraph.

usage: python tools/train_gemm_ab.py [--cfgs 0:0,8:1,1:1,1:2,1:3,1:4]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

import gemm_ab  # noqa: E402

M = 8448
LIN = {"qkv": (768, 2304), "proj": (768, 768), "fc1": (768, 3072), "fc2": (3072, 768)}  # (in K, out N)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default="0:0,8:0,1:1,1:2,1:3,1:4")
    ap.add_argument("--kinds", default="dW,dX")
    args = ap.parse_args()
    from mmt_amd import train as T
    torch.manual_seed(0)
    dev = "cuda"
    for kind in args.kinds.split(","):
        for name, (K, N) in LIN.items():
            dy = (torch.randn(2 * M, N, device=dev) * 0.1).bfloat16()
            x = (torch.randn(2 * M, K, device=dev) * 0.1).bfloat16()
            w = [(torch.randn(N, K, device=dev) / K ** 0.5).bfloat16() for _ in range(2)]
            hp = (torch.randn(2 * M, K, device=dev)).bfloat16()  # fc1's pre-activation, for fc2's dX
            row = {"kind": kind, "linear": name, "M": M, "N": N, "K": K}
            if kind == "dW":
                bufs = [torch.empty(N * (K + 8), device=dev) for _ in range(2)]
                dws = tuple(b[:N * K].view(N, K) for b in bufs)
                dbs = tuple(b[N * K:].view(N, 8) for b in bufs)
                fl = 2.0 * 2 * N * (K + 8) * M
            else:
                fl = 2.0 * 2 * M * K * N
            ref = None
            for cfg in args.cfgs.split(","):
                impl, nsk = (int(v) for v in cfg.split(":"))
                if kind == "dW":
                    fn = lambda: T._gemm(T._halves(dy, M), T._halves(x, M), N, K + 8, M, out_f32=True, c=dws,  # noqa
                                         ldc=K, c2=dbs, c2_copy=3, a_t=1, w_t=2, ldw=K, lda=N, splitk=True,
                                         impl=impl, nsk=nsk)
                else:
                    act, r = (5, T._halves(hp, M)) if name == "fc2" else (0, None)  # fc2's dX: times GELU'(hp)
                    fn = lambda: T._gemm(T._halves(dy, M), tuple(w), M, K, N, act=act, r=r, w_t=1, ldw=K,  # noqa
                                         impl=impl, splitk=nsk > 0, nsk=nsk)
                try:
                    out = fn()
                    torch.cuda.synchronize()
                except RuntimeError as e:
                    row[cfg] = "rejected: %s" % str(e)[:60]
                    continue
                val = torch.cat([b.clone() for b in bufs]) if kind == "dW" else out.clone()
                if ref is None:
                    ref = val
                err = ((val - ref).abs().max() / ref.abs().max()).item()
                us = gemm_ab.graph_time(fn, 100)
                row[cfg] = {"us": round(us, 2), "tflops": round(fl / us / 1e6, 1), "relerr_vs_first": float("%.1e" % err)}
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
