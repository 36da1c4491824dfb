#!/usr/bin/env python3
"""Quick check of a forced MAM attention kernel against impl 22 (bitwise) on the hot-path shapes and
the small test shapes, one launch each, printing one JSON line per case.  Used before a timing run of
a new kernel (a mismatch or a fault stops the session before the long steps).

usage: python tools/pg_check.py [--impl 26] [--batches 1,8,32]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))
import torch  # noqa: E402

from mmt_amd import _lib as L  # noqa: E402


def run(qkv, S, Bm, ntok, n_t, C, H, asym, impl, scale, q_part=0):
    out = torch.full((S, ntok, C), 3.0, device="cuda", dtype=torch.bfloat16)
    p = L.AttnParams()
    p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym = qkv.data_ptr(), out.data_ptr(), S, Bm, ntok, n_t, C, H, asym
    p.scale, p.impl, p.q_part = scale, impl, q_part
    L.check(L.LIB.mmt_mam_attention(ctypes.byref(p), L.MMT_BF16, torch.cuda.current_stream().cuda_stream), "attn")
    torch.cuda.synchronize()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--impl", type=int, default=28)
    ap.add_argument("--batches", default="1,8,32")
    args = ap.parse_args()
    cases = [(Bm, 528, 128, 12) for Bm in [int(b) for b in args.batches.split(",")]]
    cases += [(2, 100, 36, 2), (1, 70, 8, 1), (1, 864, 288, 2)]
    bad = 0
    for Bm, ntok, n_t, H in cases:
        for asym in (0, 1):
            S, C = 2 * Bm, 64 * H
            g = torch.Generator().manual_seed(ntok + asym + Bm)
            qkv = (torch.randn(S, ntok, 3 * C, generator=g) * 0.5).bfloat16().cuda()
            for scale in (0.125, 1.0 / 1.4426950408889634):
                ref = run(qkv, S, Bm, ntok, n_t, C, H, asym, 22, scale)
                out = run(qkv, S, Bm, ntok, n_t, C, H, asym, args.impl, scale)
                eq = bool(torch.equal(ref, out))
                diff = (ref.float() - out.float()).abs().max().item()
                bad += 0 if eq else 1
                print(json.dumps({"Bm": Bm, "ntok": ntok, "n_t": n_t, "H": H, "asym": asym, "scale": round(scale, 4),
                                  "impl": args.impl, "bitwise_vs_22": eq, "maxdiff": diff}), flush=True)
    print(json.dumps({"mismatches": bad}))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
