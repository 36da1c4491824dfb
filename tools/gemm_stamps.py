#!/usr/bin/env python3
"""Per-phase timing of the LDS-DMA GEMM from in-kernel timestamps (stamp build of tools/build_ablate.sh).

Phases per workgroup (leader thread): prologue = start -> first K-step landed (DMA latency + address
setup); loop = the K loop; epilogue = loop end -> stores retired, split into the accumulator tile's LDS
assembly (+ barriers), the strip passes (loads, epilogue math, stores issued) and the store drain.  Cycle counts come from s_memtime;
start / end skew across workgroups from s_memrealtime (100 MHz).

usage: MMT_HIP_LIB=.../_lib/stamp/libmmt_hip.so python tools/gemm_stamps.py
"""
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

SHAPES = [("qkv", 2, 528, 2304, 768, 0, 0), ("proj", 2, 528, 768, 768, 0, 1), ("fc1", 2, 528, 3072, 768, 1, 0),
          ("fc2", 2, 528, 768, 3072, 0, 1), ("qkv_ln", 2, 528, 2304, 768, 0, 0), ("fc1_ln", 2, 528, 3072, 768, 1, 0),
          ("qkv_ln2", 2, 528, 2304, 768, 0, 0), ("fc1_ln2", 2, 528, 3072, 768, 1, 0)]
if os.environ.get("GEMM_STAMP_SHAPES") == "train":  # the training step's forward GEMMs (16 pairs: 8448 rows per backbone)
    SHAPES = [("t_qkv", 1, 8448, 2304, 768, 0, 0), ("t_fc1", 1, 8448, 3072, 768, 1, 0), ("t_proj", 1, 8448, 768, 768, 0, 1),
              ("t_fc2", 1, 8448, 768, 3072, 0, 1)]
TILES = {1: (128, 128), 2: (128, 64), 3: (64, 64), 4: (128, 128), 8: (128, 128)}
IMPLS = [int(x) for x in os.environ.get("GEMM_STAMP_IMPLS", "1,2,3,4").split(",")]
SK_WS = None


def main():
    global SK_WS
    L.LIB.mmt_gemm_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    SK_WS = (torch.empty(8 << 20, device="cuda"), torch.zeros(1 << 16, device="cuda", dtype=torch.int32))
    for name, G, M, N, K, act, res in SHAPES:
        A = torch.randn(G, M, K, device="cuda").bfloat16()
        W = (torch.randn(G, N, K, device="cuda") / K ** 0.5).bfloat16()
        b = torch.randn(G, N, device="cuda")
        R = torch.randn(G, M, N, device="cuda")
        C = torch.empty(G, M, N, device="cuda", dtype=torch.float32 if res else torch.bfloat16)
        for impl in IMPLS:
            p = L.GemmParams()
            for g in range(G):
                p.a[g], p.w[g], p.c[g], p.bias[g] = A[g].data_ptr(), W[g].data_ptr(), C[g].data_ptr(), b[g].data_ptr()
                p.r[g] = R[g].data_ptr() if res else None
            p.lda, p.ldc, p.ldr = K, N, N
            p.a_seg_rows, p.a_segs_a = M, 1
            p.M, p.N, p.K, p.act, p.c_f32, p.groups, p.impl = M, N, K, act, 1 if res else 0, G, impl
            if "_ln" in name:  # _ln: statistics in the K loop; _ln2: handed in (ln_stats_in)
                p.ln_fold, p.ln_eps = (2 if name.endswith("_ln2") else 1), 1e-6
                stats = torch.ones(G, M, 2 * (K // 64), device="cuda")
                for g in range(G):
                    p.ln_colsum[g] = b[g].data_ptr()
                    p.ln_stats_in[g] = stats[g].data_ptr()
            if impl == 0:  # the library's choice, split-K allowed (as the frame's plan entries)
                p.splitk, p.sk_ws, p.sk_ws_floats = 0, SK_WS[0].data_ptr(), SK_WS[0].numel()
                p.sk_cnt, p.sk_cnt_n = SK_WS[1].data_ptr(), SK_WS[1].numel()
            s = torch.cuda.current_stream().cuda_stream
            for _ in range(10):
                L.check(L.LIB.mmt_gemm(ctypes.byref(p), L.MMT_BF16, s), name)
            torch.cuda.synchronize()
            if impl == 0:  # grid unknown here: the rows the last launch wrote (ended within 30 us of the last end)
                buf = (ctypes.c_ulonglong * (4096 * 8))()
                L.check(L.LIB.mmt_gemm_stamps(buf, 4096 * 8), "stamps")
                st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 8).astype(np.int64)
                st = st[st[:, 7] >= st[:, 7].max() - 3000]
                nwg = st.shape[0]
            else:
                bm, bn = TILES[impl]
                nwg = ((M + bm - 1) // bm) * ((N + bn - 1) // bn) * G
                buf = (ctypes.c_ulonglong * (nwg * 8))()
                L.check(L.LIB.mmt_gemm_stamps(buf, nwg * 8), "stamps")
                st = np.frombuffer(buf, dtype=np.uint64).reshape(nwg, 8).astype(np.int64)
            rt0, c0, c1, c2, e1, e2, c3, rt1 = st.T
            freq = np.median((c3 - c0) / np.maximum(rt1 - rt0, 1)) * 100.0  # MHz (realtime = 100 MHz)
            row = {"gemm": name, "impl": impl, "nwg": nwg, "clock_mhz": round(float(freq), 0),
                   "prologue_us": round(float(np.median(c1 - c0)) / freq, 2),
                   "loop_us": round(float(np.median(c2 - c1)) / freq, 2),
                   "epilogue_us": round(float(np.median(c3 - c2)) / freq, 2),
                   "epi_lds_tile_us": round(float(np.median(e1 - c2)) / freq, 2),
                   "epi_passes_us": round(float(np.median(e2 - e1)) / freq, 2),
                   "epi_store_drain_us": round(float(np.median(c3 - e2)) / freq, 2),
                   "wg_total_us_med": round(float(np.median(c3 - c0)) / freq, 2),
                   "wg_total_us_max": round(float(np.max(c3 - c0)) / freq, 2),
                   "start_spread_us": round(float(rt0.max() - rt0.min()) / 100.0, 2),
                   "span_us": round(float(rt1.max() - rt0.min()) / 100.0, 2)}
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
