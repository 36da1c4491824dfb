#!/usr/bin/env python3
"""Prototype check and timing of tools/proto/gemm256.hip (256x256 four-wave bf16 tile, tools only) on the
training step's large-M GEMM shapes, beside the product library's auto pick (tools/gemm_ab.py) and the
hipBLASLt times recorded in profiles/r05_hipblaslt_kernels.jsonl.

usage: python tools/proto_gemm256.py [--lib tools/proto/libproto_gemm256.so]
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

SHAPES = [("fc2_T16", 2, 8448, 768, 3072), ("proj_T16", 2, 8448, 768, 768), ("fc1_T16", 2, 8448, 3072, 768),
          ("qkv_T16", 2, 8448, 2304, 768), ("dXlike_fc2_T16", 2, 8448, 3072, 768), ("fc2_B8", 2, 4096, 768, 3072)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "tools", "proto", "libproto_gemm256.so"))
    ap.add_argument("--no-mmt", action="store_true")
    ap.add_argument("--tag", default="")
    ap.add_argument("--only", default="")
    ap.add_argument("--no-check", action="store_true", help="ablation builds: results are not a GEMM")
    args = ap.parse_args()
    lib = ctypes.CDLL(args.lib)
    lib.proto_gemm256.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 4 + [ctypes.c_void_p]
    torch.manual_seed(0)
    for name, G, M, N, K in SHAPES:
        if args.only and name not in args.only.split(","):
            continue
        A = torch.randn(G, M, K, device="cuda").bfloat16()
        W = (torch.randn(G, N, K, device="cuda") / K ** 0.5).bfloat16()
        C = torch.zeros(G, M, N, device="cuda")
        fn = lambda: lib.proto_gemm256(A.data_ptr(), W.data_ptr(), C.data_ptr(), G, M, N, K,  # noqa: E731
                                       ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        rc = fn()
        assert rc == 0, rc
        torch.cuda.synchronize()
        ref = torch.bmm(A.float(), W.float().transpose(1, 2).contiguous())  # NN layout (the NT bf16 bmm faulted once)
        err = ((C - ref).abs().max() / ref.abs().max()).item()
        us = gemm_ab.graph_time(fn, 200)
        fl = 2.0 * G * M * N * K
        row = {"gemm": name, "G": G, "M": M, "N": N, "K": K, "tag": args.tag,
               "proto256": {"us": round(us, 2), "tflops": round(fl / us / 1e6, 1), "relerr": float("%.2e" % err)}}
        if not args.no_mmt:
            u2, e2 = gemm_ab.run(name, G, M, N, K, 0, 0, 0, 200, 0)
            row["mmt_auto_plain"] = {"us": round(u2, 2), "tflops": round(fl / u2 / 1e6, 1)}
        print(json.dumps(row), flush=True)
        assert args.no_check or err < 1e-2, (name, err)


if __name__ == "__main__":
    main()
