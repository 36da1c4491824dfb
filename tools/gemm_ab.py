#!/usr/bin/env python3
"""A/B timing of the bf16 GEMM kernels (mmt_gemm impl -1 / 1 / 2 / 3 / auto) against torch.bmm
(hipBLASLt) on the hot path's GEMM shapes: back-to-back launches captured in a hipGraph and timed
with HIP events (device time, no host launch cost).

usage: python tools/gemm_ab.py [--reps 200]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))
import torch  # noqa: E402

from mmt_amd import _lib as L  # noqa: E402

# (name, groups, M per group, N, K, act, residual) at B = 1: rgbt two-stream (groups = modalities)
SHAPES = [("qkv_ln", 2, 528, 2304, 768, 0, 0), ("fc1_ln", 2, 528, 3072, 768, 1, 0), ("qkv", 2, 528, 2304, 768, 0, 0), ("proj", 2, 528, 768, 768, 0, 1), ("fc1", 2, 528, 3072, 768, 1, 0),
          ("fc2", 2, 528, 768, 3072, 0, 1), ("qkv_B4", 2, 2112, 2304, 768, 0, 0), ("fc2_B4", 2, 2112, 768, 3072, 0, 1),
          ("head1_like", 1, 400, 1344, 6912, 2, 0), ("enc_lin2_like", 1, 800, 512, 2048, 0, 1),
          ("conv2_like", 2, 400, 192, 3456, 2, 0),
          # large M: config-4 training step (16 pairs, two-stream: 8448 rows per backbone) and its
          # backward dX / dW shapes (dW: K = rows), config-3 batched inference (B = 8: 4224 rows)
          ("qkv_T16", 2, 8448, 2304, 768, 0, 0), ("fc1_T16", 2, 8448, 3072, 768, 1, 0),
          ("fc2_T16", 2, 8448, 768, 3072, 0, 1), ("proj_T16", 2, 8448, 768, 768, 0, 1),
          ("dW_fc1_T16", 2, 3072, 768, 8448, 0, 0), ("dW_fc2_T16", 2, 768, 3072, 8448, 0, 0),
          ("dX_fc2_T16", 2, 8448, 3072, 768, 0, 0), ("fc1_B8", 2, 4224, 3072, 768, 1, 0),
          ("fc2_B8", 2, 4224, 768, 3072, 0, 1),
          # the training step's GEMMs as it issues them (one backbone per call, 16 pairs: 8448 rows;
          # dW with the bias column block: N = K_fwd + 8, contraction over the 8448 rows)
          ("g1_qkv", 1, 8448, 2304, 768, 0, 0), ("g1_fc1", 1, 8448, 3072, 768, 1, 0),
          ("g1_fc2", 1, 8448, 768, 3072, 0, 1), ("g1_proj", 1, 8448, 768, 768, 0, 1),
          ("g1_dX_qkv", 1, 8448, 768, 2304, 0, 0), ("g1_dX_fc1", 1, 8448, 768, 3072, 0, 0),
          ("g1_dX_fc2", 1, 8448, 3072, 768, 0, 0), ("g1_dX_proj", 1, 8448, 768, 768, 0, 0),
          ("g1_dW_qkv", 1, 2304, 776, 8448, 0, 0), ("g1_dW_fc1", 1, 3072, 776, 8448, 0, 0),
          ("g1_dW_fc2", 1, 768, 3080, 8448, 0, 0), ("g1_dW_proj", 1, 768, 776, 8448, 0, 0),
          # config 3 on one GPU (shared backbone, 64 sequences: 2 modality groups of 33792 rows; qkv / fc1 with
          # the LayerNorm fold on handed-in statistics, "_ln2")
          ("c3_qkv_ln2", 2, 33792, 2304, 768, 0, 0), ("c3_fc1_ln2", 2, 33792, 3072, 768, 1, 0),
          ("c3_proj", 2, 33792, 768, 768, 0, 1), ("c3_fc2", 2, 33792, 768, 3072, 0, 1)]


SK_WS = None


def run(name, G, M, N, K, act, res, impl, reps, splitk=1):
    global SK_WS
    if SK_WS is None:
        SK_WS = (torch.empty(8 << 20, device="cuda"), torch.zeros(1 << 16, device="cuda", dtype=torch.int32))
    A = torch.randn(G, M, K, device="cuda").bfloat16()
    W = (torch.randn(G, N, K, device="cuda") / K ** 0.5).bfloat16()
    b = torch.randn(G, N, device="cuda")
    R = torch.randn(G, M, N, device="cuda")
    C = torch.empty(G, M, N, device="cuda", dtype=torch.float32 if res else torch.bfloat16)
    p = L.GemmParams()
    for g in range(G):
        p.a[g], p.w[g], p.c[g], p.bias[g] = A[g].data_ptr(), W[g].data_ptr(), C[g].data_ptr(), b[g].data_ptr()
        p.r[g] = R[g].data_ptr() if res else None
    p.lda, p.ldc, p.ldr = K, N, N
    p.a_seg_rows, p.a_segs_a = M, 1
    p.M, p.N, p.K, p.act, p.c_f32, p.groups, p.impl = M, N, K, act, 1 if res else 0, G, impl
    p.splitk, p.sk_ws, p.sk_ws_floats = splitk, SK_WS[0].data_ptr(), SK_WS[0].numel()
    p.sk_cnt, p.sk_cnt_n = SK_WS[1].data_ptr(), SK_WS[1].numel()
    if name.endswith("_ln") or name.endswith("_ln2"):  # LayerNorm folded (timing only: colsum = bias, no check)
        p.ln_fold, p.ln_eps = (2 if name.endswith("_ln2") else 1), 1e-6
        st = torch.zeros(G, M, K // 64, 2, device="cuda")
        st[..., 1] = 64.0  # (sum, sum of squares) per 64 columns: mean 0, variance 1
        run.keep = st
        for g in range(G):
            p.ln_colsum[g] = b[g].data_ptr()
            if p.ln_fold == 2:
                p.ln_stats_in[g] = st[g].data_ptr()
    fn = lambda: L.check(L.LIB.mmt_gemm(L.ctypes.byref(p), L.MMT_BF16,  # noqa: E731
                                        torch.cuda.current_stream().cuda_stream), name)
    fn()
    torch.cuda.synchronize()
    first = C.clone()
    us = graph_time(fn, reps)
    assert torch.equal(first, C), "%s impl %d splitk %d: repeated calls differ" % (name, impl, splitk)
    ref = torch.baddbmm(b[:, None, :], A.float(), W.float().transpose(1, 2))
    if act == 1:
        ref = torch.nn.functional.gelu(ref)
    elif act == 2:
        ref = torch.relu(ref)
    if res:
        ref = ref + R
    err = ((C.float() - ref).abs().max() / ref.abs().max()).item() if "_ln" not in name else float("nan")
    return us, err


def torch_ref(G, M, N, K, reps):
    A = torch.randn(G, M, K, device="cuda").bfloat16()
    Wt = (torch.randn(G, K, N, device="cuda") / K ** 0.5).bfloat16()
    out = torch.empty(G, M, N, device="cuda", dtype=torch.bfloat16)
    return graph_time(lambda: torch.bmm(A, Wt, out=out), reps)


def graph_time(fn, reps, per_graph=20):
    """Device time per call: `per_graph` back-to-back calls captured in one hipGraph, replayed."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(per_graph):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = max(1, reps // per_graph)
    e0.record(s)
    for _ in range(n):
        g.replay()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (n * per_graph)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--impls", default="-1,1,2,3,4,0", help="impl[:splitk] list, e.g. 1:1,1:4,0:0")
    ap.add_argument("--only", default="", help="comma list of shape names")
    ap.add_argument("--no-torch", action="store_true")
    args = ap.parse_args()
    impls = [tuple(int(v) for v in (x.split(":") + ["1"])[:2]) for x in args.impls.split(",")]
    rows = []
    for name, G, M, N, K, act, res in SHAPES:
        if args.only and name not in args.only.split(","):
            continue
        fl = 2.0 * G * M * N * K
        row = {"gemm": name, "G": G, "M": M, "N": N, "K": K}
        for impl, sk in impls:
            us, err = run(name, G, M, N, K, act, res, impl, args.reps, sk)
            row["impl%d:%d" % (impl, sk)] = {"us": round(us, 2), "tflops": round(fl / us / 1e6, 1), "relerr": float("%.2e" % err)}
        if not args.no_torch:
            tu = torch_ref(G, M, N, K, args.reps)
            row["torch_bmm"] = {"us": round(tu, 2), "tflops": round(fl / tu / 1e6, 1)}
        rows.append(row)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
