#!/usr/bin/env python3
"""Which kernel hipBLASLt (torch.bmm / torch.matmul, tools only: the product never calls it) picks for the
large-M GEMM shapes of the training step and config 3, and its device time per launch from the profiler's
kernel records, beside this repo's `mmt_gemm` (auto pick) on the same shape. The kernel name carries the
vendor's tile choice (MT = macro tile MxNxDepthU, MI = matrix instruction, MIWT = wave tile in MI blocks,
WG = workgroup shape, PGR / PLR = global / local prefetch depth, 1LDSB / DTL = LDS buffering / direct-to-LDS).

usage: python tools/hipblaslt_kernels.py [--only fc2_T16,proj_T16]

Round 5: the NT-layout torch.bmm of fc1_B8 (G 2, M 4224, N 3072, K 768) faulted the GPU (illegal address at the
synchronize after hipBLASLt's warm-up calls, with this repo's previous GEMM already synchronized and checked), so
the default list holds only the shapes that ran (profiles/r05_hipblaslt_kernels.jsonl).
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

SHAPES = {n: s for n, *s in gemm_ab.SHAPES}


def profile_kernels(fn, reps=20):
    from torch.profiler import ProfilerActivity, profile
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
    by = {}
    for e in prof.events():
        if str(getattr(e, "device_type", "")).endswith("CUDA") and e.time_range.end > e.time_range.start:
            by.setdefault(e.name, []).append((e.time_range.end - e.time_range.start))
    return {k: (len(v), sorted(v)[len(v) // 2]) for k, v in by.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="fc2_T16,proj_T16,fc1_T16,qkv_T16,dW_fc1_T16")
    args = ap.parse_args()
    for name in args.only.split(","):
        G, M, N, K, act, res = SHAPES[name]
        fl = 2.0 * G * M * N * K
        A = torch.randn(G, M, K, device="cuda").bfloat16()
        W = (torch.randn(G, N, K, device="cuda") / K ** 0.5).bfloat16()
        Wt = W.transpose(1, 2).contiguous()
        out = torch.empty(G, M, N, device="cuda", dtype=torch.bfloat16)
        row = {"gemm": name, "G": G, "M": M, "N": N, "K": K}
        for lay, fn in (("NT", lambda: torch.bmm(A, W.transpose(1, 2), out=out)),
                        ("NN", lambda: torch.bmm(A, Wt, out=out))):
            ks = profile_kernels(fn)
            main_k = max(ks.items(), key=lambda kv: kv[1][0] * kv[1][1])
            us = main_k[1][1]  # profiler time ranges are in us
            row["hipblaslt_" + lay] = {"kernel": main_k[0], "us": round(us, 2), "tflops": round(fl / us / 1e6, 1)}
        us, err = gemm_ab.run(name, G, M, N, K, act, res, 0, 200, 0)
        row["mmt_auto"] = {"us": round(us, 2), "tflops": round(fl / us / 1e6, 1), "relerr": float("%.2e" % err)}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
