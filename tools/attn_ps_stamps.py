#!/usr/bin/env python3
"""Event log of impl 29 (the persistent MAM kernel) under the stamp build (tools/build_ps_variant.sh stamp;
MMT_HIP_LIB=.../_lib/stamp/libmmt_hip.so): wave 0 and wave 3 of every workgroup record s_memtime at each
sync point (before its wait, after the wait, after the barrier), at each task start, at the end of a task's
block loop and after its output stores.  Printed per batch size: median cycles of each phase, split by item
kind (A = four search waves, M = three search waves + the template wave) and, for the sync points, by the
tile's position in the item.

usage: MMT_HIP_LIB=... python tools/attn_ps_stamps.py [--batches 1,32] [--asym 0]
"""
import argparse
import collections
import ctypes
import json
import os
import statistics as stt
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))
import torch  # noqa: E402

from mmt_amd import _lib as L  # noqa: E402

NEV = 512
SYNC, WAITED, BARRIER, TSTART, LOOPEND, STORED, END, STAGED, READ = 1, 2, 3, 4, 5, 6, 7, 8, 9


def med(v):
    return round(stt.median(v)) if v else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,32")
    ap.add_argument("--asym", type=int, default=0)
    args = ap.parse_args()
    ntok, n_t, H = 528, 128, 12
    C = 64 * H
    Lk = ntok + n_t if args.asym else ntok
    nkt = (Lk + 63) // 64
    fn = L.LIB.mmt_attn_ps_stamps
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    for B in [int(x) for x in args.batches.split(",")]:
        S = 2 * B
        qkv = (torch.randn(S, ntok, 3 * C, device="cuda") * 0.5).bfloat16()
        out = torch.empty(S, ntok, C, device="cuda", dtype=torch.bfloat16)
        p = L.AttnParams()
        p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym = (qkv.data_ptr(), out.data_ptr(), S, B, ntok, n_t,
                                                                 C, H, args.asym)
        p.scale, p.impl = 1.0 / 1.4426950408889634, 29
        for _ in range(20):  # warm (clocks); the log of the last launch is read
            L.check(L.LIB.mmt_mam_attention(ctypes.byref(p), L.MMT_BF16, torch.cuda.current_stream().cuda_stream), "attn")
        torch.cuda.synchronize()
        n = 1024 * 2 * NEV
        buf = (ctypes.c_ulonglong * n)()
        L.check(fn(buf, n), "stamps")
        NI = S * H * 2
        G = (min(NI, 256) + 7) // 8 * 8
        gper, q8, r8 = G // 8, NI // 8, NI % 8
        ph = collections.defaultdict(list)
        kernel = []
        for g in range(G):
            xcd, gi = g & 7, g >> 3
            ibase = xcd * q8 + min(xcd, r8)
            for wv, wname in ((0, "w0"), (1, "w3")):
                base = (g * 2 + wv) * NEV
                cnt = buf[base]
                ev = [(buf[base + 1 + i] & 0xffffffffffff, (buf[base + 1 + i] >> 48) & 255, buf[base + 1 + i] >> 56)
                      for i in range(cnt)]
                if not ev:
                    continue
                if wv == 0:
                    kernel.append(ev[-1][0] - ev[0][0])
                for (t0, a0, c0), (t1, a1, c1) in zip(ev, ev[1:]):
                    d = t1 - t0
                    T = a0 if c0 in (SYNC, WAITED, BARRIER) else None
                    kind = pos = None
                    if T is not None:
                        it = ibase + gi + (T // nkt) * gper
                        kind, pos = ("A" if it % 2 == 0 else "M"), T % nkt
                    if c0 == SYNC and c1 == WAITED:
                        ph["%s %s wait@%d" % (wname, kind, pos)].append(d)
                    elif c0 == WAITED and c1 == BARRIER:
                        ph["%s %s barrier@%d" % (wname, kind, pos)].append(d)
                    elif c0 == BARRIER and c1 == SYNC:
                        ph["%s %s compute_after@%d" % (wname, kind, pos)].append(d)
                    elif c0 == BARRIER and c1 == TSTART:
                        ph["%s %s sync@%d_to_task_start" % (wname, kind, pos)].append(d)
                    elif c0 == BARRIER and c1 == LOOPEND:
                        ph["%s %s sync@%d_to_loop_end" % (wname, kind, pos)].append(d)
                    elif c0 == TSTART and c1 == SYNC:
                        ph["%s task_start_to_first_sync" % wname].append(d)
                    elif c0 == LOOPEND and c1 == STAGED:
                        ph["%s epilogue: loop end -> staged (range check, normalise, LDS writes)" % wname].append(d)
                    elif c0 == BARRIER and c1 == STAGED:
                        ph["%s %s epilogue: sync@%d -> staged" % (wname, kind, pos)].append(d)
                    elif c0 == STAGED and c1 == READ:
                        ph["%s epilogue: staged -> rows read" % wname].append(d)
                    elif c0 == READ and c1 == STORED:
                        ph["%s epilogue: rows read -> stores issued" % wname].append(d)
                    elif c0 == STORED and c1 == SYNC:
                        ph["%s stored_to_next_sync" % wname].append(d)
                    elif c0 == STORED and c1 == TSTART:
                        ph["%s stored_to_task_start" % wname].append(d)
        print(json.dumps({"B": B, "asym": args.asym, "workgroups": G, "kernel_cycles_med": med(kernel),
                          "phases_med": {k: [med(v), len(v)] for k, v in sorted(ph.items())}}), flush=True)


if __name__ == "__main__":
    main()
