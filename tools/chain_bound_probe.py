#!/usr/bin/env python3
"""Upper bound of what a persistent batch-1 GEMM chain can save at a stage seam.

Times the batch-1 MLP pair (fc1: 2 x 528 rows, N 3072, K 768, GELU, bf16 out; fc2: K 3072, N 768, fp32 out
+ residual) three ways, each as back-to-back launches captured in one hipGraph (tools/gemm_ab.graph_time):
  seq    fc1 launch, then fc2 launch (what the frame runs, one forced tile config for both);
  fused  ONE mmt_gemm_multi launch holding both problems with NO dependency between them: fc2's workgroups
         start as soon as CUs free up, without waiting for fc1's rows (results wrong for a real chain).
         This is the most a persistent kernel could save at the seam -- boundary, launch ramp, prologue and
         tail overlap -- before paying for any hand-off (release / poll / acquire: MI355X_MICROARCH.md price
         list rows handoff-flag, fanin, fence table);
  alone  each launch by itself (sum = seq without the seam's interaction); the bound is taken inside the multi
         kernel (general epilogue): multi(fc1) + multi(fc2) - multi(fc1, fc2).

usage: python tools/chain_bound_probe.py [--impls 1,3]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

import gemm_ab  # noqa: E402
from mmt_amd import _lib as L  # noqa: E402


def params(G, M, N, K, act, res, impl, keep):
    A = torch.randn(G, M, K, device="cuda").bfloat16()
    W = (torch.randn(G, N, K, device="cuda") / K ** 0.5).bfloat16()
    b = torch.randn(G, N, device="cuda")
    R = torch.randn(G, M, N, device="cuda")
    C = torch.empty(G, M, N, device="cuda", dtype=torch.float32 if res else torch.bfloat16)
    keep += [A, W, b, R, C]
    p = L.GemmParams()
    for g in range(G):
        p.a[g], p.w[g], p.c[g], p.bias[g] = A[g].data_ptr(), W[g].data_ptr(), C[g].data_ptr(), b[g].data_ptr()
        p.r[g] = R[g].data_ptr() if res else None
    p.lda, p.ldc, p.ldr = K, N, N
    p.a_seg_rows, p.a_segs_a = M, 1
    p.M, p.N, p.K, p.act, p.c_f32, p.groups, p.impl, p.splitk = M, N, K, act, 1 if res else 0, G, impl, 1
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--impls", default="1,3")
    ap.add_argument("--reps", type=int, default=400)
    args = ap.parse_args()
    torch.manual_seed(0)
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    for impl in (int(x) for x in args.impls.split(",")):
        keep = []
        p1 = params(2, 528, 3072, 768, 1, 0, impl, keep)
        p2 = params(2, 528, 768, 3072, 0, 1, impl, keep)
        arr = (L.GemmParams * 2)(p1, p2)

        def one(p, nm):
            return lambda: L.check(L.LIB.mmt_gemm(ctypes.byref(p), L.MMT_BF16, st()), nm)

        def seq():
            one(p1, "fc1")()
            one(p2, "fc2")()

        def fused():
            L.check(L.LIB.mmt_gemm_multi(arr, 2, L.MMT_BF16, st()), "multi")

        row = {"impl": impl, "fc1_alone_us": round(gemm_ab.graph_time(one(p1, "fc1"), args.reps), 2),
               "fc2_alone_us": round(gemm_ab.graph_time(one(p2, "fc2"), args.reps), 2),
               "seq_us": round(gemm_ab.graph_time(seq, args.reps), 2),
               "fused_no_dependency_us": round(gemm_ab.graph_time(fused, args.reps), 2)}
        a1, a2 = (L.GemmParams * 1)(p1), (L.GemmParams * 1)(p2)
        row["multi_fc1_us"] = round(gemm_ab.graph_time(lambda: L.check(L.LIB.mmt_gemm_multi(a1, 1, L.MMT_BF16, st()), "m1"), args.reps), 2)
        row["multi_fc2_us"] = round(gemm_ab.graph_time(lambda: L.check(L.LIB.mmt_gemm_multi(a2, 1, L.MMT_BF16, st()), "m2"), args.reps), 2)
        # the multi kernel runs the general epilogue (the frame's launches the compact ones), so the bound is
        # taken within the multi kernel: its two problems one launch each vs both in one launch
        row["seam_bound_us"] = round(row["multi_fc1_us"] + row["multi_fc2_us"] - row["fused_no_dependency_us"], 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
