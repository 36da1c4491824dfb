#!/usr/bin/env python3
"""The training step's weight-gradient GEMMs (dW [N][K+8] = dY^T [X | 1], both operands MN-major, fp32 out with the
bias-gradient column block) at one backbone's 8448 tokens: the library's choice against forced tile / split-K
choices (impl 1 with 1-6 K slices, impl 8).  Device time of back-to-back calls (HIP events)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))
import torch  # noqa: E402

from mmt_amd import train  # noqa: E402
from mmt_amd._lib import LIB, GemmParams, MMT_BF16, check  # noqa: E402

SHAPES = [("qkv", 8448, 2304, 768), ("proj", 8448, 768, 768), ("fc1", 8448, 3072, 768), ("fc2", 8448, 768, 3072)]


def dw_call(dy, x, M, N, K, impl, splitk, G=1):
    buf = torch.empty(G, N * (K + 8), device="cuda", dtype=torch.float32)
    dw, db8 = buf[:, :N * K].view(G, N, K), buf[:, N * K:].view(G, N, 8)
    ws, cnt = train._splitk_ws(dy.device)

    def fn():
        p = GemmParams()
        for g in range(G):
            p.a[g], p.w[g], p.c[g], p.c2[g] = dy[g].data_ptr(), x[g].data_ptr(), dw[g].data_ptr(), db8[g].data_ptr()
        p.lda, p.ldc, p.a_t, p.w_t, p.ldw, p.impl, p.splitk = N, K, 1, 2, K, impl, splitk
        p.sk_ws, p.sk_ws_floats, p.sk_cnt, p.sk_cnt_n = ws.data_ptr(), ws.numel(), cnt.data_ptr(), cnt.numel()
        p.a_seg_rows, p.a_segs_a = N, 1
        p.M, p.N, p.K, p.groups, p.c_f32, p.c2_copy = N, K + 8, M, G, 1, 3
        check(LIB.mmt_gemm(p, MMT_BF16, torch.cuda.current_stream().cuda_stream), "dW")
    return fn, dw


def timed(fn, reps=30):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    G = int(os.environ.get("DW_GROUPS", "1"))  # 2: the lockstep pair's grouped dW (one launch for both modalities)
    for name, M, N, K in SHAPES:
        x = torch.randn(G, M, K, device="cuda", generator=g).bfloat16()
        dy = torch.randn(G, M, N, device="cuda", generator=g).bfloat16()
        row = {"gemm": "dW_" + name, "groups": G, "M": M, "N": N, "K": K}
        ref = None
        for impl, sk in [(0, 0), (1, 1), (1, 2), (1, 3), (1, 4), (1, 6), (1, 8), (8, 1)]:
            fn, dw = dw_call(dy, x, M, N, K, impl, sk, G)
            us = timed(fn)
            d = 0.0 if ref is None else float((dw - ref).abs().max() / ref.abs().max())
            ref = dw.clone() if ref is None else ref
            row["%d:%d" % (impl, sk)] = {"us": round(us, 2), "tflops": round(2.0 * G * M * N * K / us / 1e6, 1), "rel": d}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
