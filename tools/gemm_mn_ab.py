#!/usr/bin/env python3
"""The Linear backward's GEMMs with MN-major operands (mmt_gemm_params.a_t / w_t: dY, X and W read as
they are, ds_read_b64_tr_b16 fragments) against the transposing form (mmt_transpose_bf16 copies, then
the plain GEMM), interleaved, at the training step's shapes (16 pairs: 8448 tokens per backbone GEMM).
One JSON line per shape: microseconds per dX and per dW (+ db) call, both forms, and their agreement.

    python tools/gemm_mn_ab.py [--reps 50] [--rounds 3]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))

import torch  # noqa: E402

from mmt_amd import train  # noqa: E402

SHAPES = [("qkv", 8448, 2304, 768), ("proj", 8448, 768, 768), ("fc1", 8448, 3072, 768), ("fc2", 8448, 768, 3072)]


def timed(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, M, N, K in SHAPES:  # y [M][N] = x [M][K] W^T
        x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
        dy = torch.randn(M, N, device="cuda", generator=g).bfloat16()
        w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
        res = {"gemm": name, "M": M, "N": N, "K": K}
        outs = {}
        for r in range(args.rounds):
            for mode in (True, False):
                train.MN_MAJOR = mode
                tag = "mn_major" if mode else "transposed"
                res.setdefault(tag + "_dx_us", []).append(round(timed(lambda: train._dx(dy, w, M, N, K), args.reps), 2))
                res.setdefault(tag + "_dw_us", []).append(
                    round(timed(lambda: train._weight_grads(dy, x, M, N, K), args.reps), 2))
                outs[mode] = (train._dx(dy, w, M, N, K).float(), *train._weight_grads(dy, x, M, N, K))
        train.MN_MAJOR = True
        for impl in (1, 8):  # the MN-major dX GEMM on each of its two tile configurations
            res["mn_major_dx_impl%d_us" % impl] = round(
                timed(lambda: train._gemm(dy, w, M, K, N, w_t=1, ldw=K, impl=impl), args.reps), 2)
        for i, part in enumerate(("dx", "dw", "db")):
            a, b = outs[True][i], outs[False][i]
            res["rel_diff_" + part] = float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
