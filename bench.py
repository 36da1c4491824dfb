#!/usr/bin/env python3
"""Tracker FPS benchmark of the MI355X MixFormer RGB-T forward path (BASELINE.json `metric`).

A step = one template+search forward (both modalities, boxes out) of B frames per GPU on synthetic
inputs resident in HBM.  Four distinct input sets are rotated; each has its own captured hipGraph
whose patch-staging kernel reads that set in place, so a step is one graph replay.

Multi-GPU (one process per GPU, no data-path collective):
  default          single-stream tracking (config 2): every rank is an independent replica tracking
                   its own sequences at B frames per step ("replicas only": each frame depends on the
                   previous box, nothing to exchange); scaling "weak", value = frames of all ranks /
                   max-over-ranks time.
  --total-seqs T   batched multi-sequence inference (config 3, e.g. `--variant shared --total-seqs 64`):
                   the T sequences are sharded over the ranks, T/N per rank (rank r owns sequences
                   [r*T/N, (r+1)*T/N), each sequence's frames seeded by its global index, so the union
                   of the shards is exactly the single-process batch); scaling "strong".
  `python bench.py --gpus N` with no WORLD_SIZE in the environment starts N worker processes itself
  (before any GPU call), each with RANK / LOCAL_RANK / WORLD_SIZE set; under torchrun, WORLD_SIZE must
  equal --gpus.

Extra fields:
  kernels        device time per launch of every plan entry inside the frame (inframe_profile: the
                 profiler's dispatch timestamps of graph-replayed frames, after the timed region)
  roofline       the kernel with the largest share of device time: algorithmic FLOPs per launch /
                 that average in-frame launch time (the warm back-to-back figure of kernel_profile
                 beside it as warm_avg_launch_us); `traffic` = HBM bytes per launch from the PMC pass in
                 profiles/pmc_traffic.json (2 x FETCH_SIZE + WRITE_SIZE, gfx950 correction) when it
                 was measured for this workload, else null
  roofline_mam   the same for the MAM attention kernel
  roofline_mam_batched  the MAM attention kernel alone at the batched-inference size (SURVEY §8(e)
                 C3: 32 frames per GPU, the grid where the throughput kernel runs), same definition
  cpu_baseline   the oracle's fp32 CPU forward (oracle/forward.py, a restatement of the reference)
                 on a bounded sample, rank 0 at N=1 only, on every physical core available to the
                 process (lscpu sockets x cores, capped by the affinity mask and cgroup quota);
                 cpu_baseline_b8 the same at B = 8
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "tracker FPS (template+search fwd) MixViT-B RGB-T @320px, 1/2/4/8 MI355X"
PEAK = {"bf16": 2500.0, "fp16": 2500.0, "f32": 157.3}  # dense MFMA TFLOP/s, MI355X_MICROARCH.md
HBM_PEAK = 8.0  # TB/s, MI355X_MICROARCH.md (6.29 measured for a float4 copy)


def mam_memory_roofline(obj, S, ntok, C, elem_bytes):
    """Adds the MAM kernel's memory side to a roofline object: its algorithmic HBM bytes per launch
    (Q, K, V read once, O written once: S * ntok * 4C elements), their rate against the
    8 TB/s peak, and `attainable_frac` = max(FLOP / MFMA peak, bytes / HBM peak) / launch time -- at
    d = 64 the kernel's arithmetic intensity (~215 FLOP/B at the ViT-B shapes) is below the chip's
    ridge (2.5 PF / 8 TB/s = 312 FLOP/B), so the bytes, not the MFMAs, set its floor."""
    if obj is None:  # (no per-kernel profile in this run)
        return None
    by = float(S) * ntok * 4 * C * elem_bytes
    us = obj["avg_launch_us"]
    t_min = max(obj["flops_per_launch"] / (obj["peak"] * 1e12), by / (HBM_PEAK * 1e12)) * 1e6
    obj.update({"hbm_bytes_per_launch": by, "hbm_tbps": round(by / (us * 1e-6) / 1e12, 3),
                "hbm_frac": round(by / (us * 1e-6) / 1e12 / HBM_PEAK, 4),
                "arith_intensity": round(obj["flops_per_launch"] / by, 1),
                "attainable_frac": round(t_min / us, 4)})
    return obj
# model geometry: ViT-B 128/320 (configs 2-4) and ViT-L 192/384 (config 5; fusion width = HIDDEN_DIM, defect D1)
GEO_B = {"hidden": 768, "depth": 12, "search": 320, "template": 128}
GEO_L = {"hidden": 1024, "depth": 24, "search": 384, "template": 192}
VARIANT_NAMES = {"rgbt": "mixformer_vit_rgbt (two-stream)", "shared": "mixformer_vit_rgbt_shared",
                 "asym": "asymmetric_shared", "asym_online": "asymmetric_shared_online_score",
                 "asym_ce": "asymmetric_shared_ce (candidate elimination 3/6/9 x0.7)",
                 "rgb": "mixformer_vit (RGB-only, BASELINE config 1)"}
GEO_RGB = {"hidden": 768, "depth": 12, "search": 288, "template": 128}  # config 1: MixViT-B 128/288


def state_dict_keys(variant, hidden=768, depth=12, search=320, template=128, fusion_layers=2):
    """(name, shape) list of the reference model's state_dict (drop-in key names)."""
    from mmt_amd.model import reference_state_dict_shapes
    return reference_state_dict_shapes(variant, hidden=hidden, depth=depth, search=search, template=template,
                                       fusion_layers=fusion_layers)


def plan_flops(rt, entry):
    """Algorithmic FLOPs of one plan entry (GEMM: 2MNK per group; MAM: 4*d*H*sum(Lq*Lk))."""
    fn, args, name, keep = entry
    if keep is None:
        return 0.0
    if hasattr(keep, "K"):
        return 2.0 * keep.M * keep.N * keep.K * keep.groups
    if isinstance(keep, ctypes.Array):  # mmt_gemm_multi: independent problems in one launch
        return sum(2.0 * q.M * q.N * q.K * q.groups for q in keep)
    d = rt.d
    ntok = keep.ntok  # < d.ntok after a candidate-elimination stage
    lk_s = ntok + (d.n_t if keep.asym else 0)
    qpart = getattr(keep, "q_part", 0)
    return 4.0 * 64 * keep.H * keep.S * ((d.n_t * d.n_t if qpart != 2 else 0) + ((ntok - d.n_t) * lk_s if qpart != 1 else 0))


def kernel_profile(rt, plan, per_graph=20, replays=5):
    """Average device time per launch of each plan entry name: `per_graph` back-to-back launches of
    the name's first entry captured in one hipGraph on the launch stream and replayed, timed with
    HIP events on that stream (launch gaps excluded, as in a rocprofv3 kernel trace).  Run after
    the timed region: repeated in-place launches leave the workspace scrambled."""
    s = torch.cuda.current_stream()
    first = {}
    for e in plan:
        first.setdefault(e[2], e)
    per_name = {}
    for nm, (fn, args, _, _) in first.items():
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(per_graph):
                fn(*args, torch.cuda.current_stream().cuda_stream)
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(replays):
            g.replay()
        e1.record(s)
        torch.cuda.synchronize()
        per_name[nm] = e0.elapsed_time(e1) / (replays * per_graph)
        del g
    return [per_name[e[2]] for e in plan]  # ms per launch


def inframe_profile(graphs, plan, frames=20):
    """Device time of every launch of the frame as it runs inside the frame (the cache state the
    previous launch leaves, no repeated copies, no host gaps): `frames` replays of the captured frame
    graphs under torch.profiler (ROCm: the kernel-dispatch activity records of the profiler SDK, the
    same device timestamps a rocprofv3 kernel trace reports), each frame's dispatches mapped onto the
    plan entries in order (one kernel per entry; a frame starts at the plan's first kernel).
    Returns ms per launch (median over the frames) in plan order and the median frame span, or
    None when the profiler saw no complete frame."""
    from torch.profiler import ProfilerActivity, profile
    first = plan[0][2]
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        for i in range(frames):
            graphs[i % len(graphs)].replay()
        torch.cuda.synchronize()
    ev = []
    for e in prof.events():
        if str(getattr(e, "device_type", "")).endswith("CUDA") and e.time_range.end > e.time_range.start:
            ev.append((e.time_range.start, e.time_range.end, e.name))
    ev.sort()
    key = {"patch_im2col": "patch_im2col"}.get(first, first)
    starts = [i for i, (_, _, nm) in enumerate(ev) if key in nm]
    n = len(plan)
    per = [[] for _ in range(n)]
    spans = []
    for st in starts:
        seq = ev[st:st + n]
        if len(seq) < n:
            break
        spans.append((seq[-1][1] - seq[0][0]) / 1e3)
        for k, (a, b, _) in enumerate(seq):
            per[k].append((b - a) / 1e3)  # us -> ms
    if not spans:
        return None, None
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    return [med(v) for v in per], med(spans)


def load_traffic(variant, B, dtype):
    """HBM bytes per launch by plan-entry name, from the committed PMC pass (tools/pmc_traffic.py),
    and the stamp check: the counts are used only if they were taken on kernel sources with this
    tree's digest (mmt_amd.stamp); otherwise `traffic` is null and the reason is reported."""
    from mmt_amd.stamp import source_digest
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            res = json.load(f).get("%s/B%d/%s" % (variant, B, dtype), {})
    except (OSError, ValueError):
        return {}, "no PMC traffic file"
    if not res:
        return {}, "no PMC pass for this workload"
    stamp = res.get("_stamp", {}).get("source_digest")
    here = source_digest(train=variant == "train")
    if stamp != here:
        return {}, "PMC pass taken on sources %s, this tree is %s: not reported" % (stamp, here)
    return res, "PMC pass on this tree's sources (%s)" % here


def roofline(rt, plan, times, dtype, traffic=None, warm_times=None):
    """times: in-frame ms per launch (inframe_profile); warm_times: the warm back-to-back copies of
    kernel_profile, reported beside it as `warm_avg_launch_us` / `warm_frac`."""
    traffic = traffic or {}
    by = {}
    for i, (e, t) in enumerate(zip(plan, times)):
        nm = e[2]
        a = by.setdefault(nm, {"t": 0.0, "n": 0, "flops": 0.0, "tw": 0.0})
        a["t"] += t
        a["n"] += 1
        a["flops"] += plan_flops(rt, e)
        a["tw"] += warm_times[i] if warm_times else 0.0
    total = sum(a["t"] for a in by.values())
    dom = max(by, key=lambda k: by[k]["t"])

    def obj(nm):
        a = by[nm]
        avg_ms = a["t"] / a["n"]
        ach = (a["flops"] / a["n"]) / (avg_ms * 1e-3) / 1e12
        tb = traffic.get(nm, {}).get("traffic_bytes")
        o = {"kernel": nm, "bound": "mfma", "achieved": round(ach, 2), "peak": PEAK[dtype], "unit": "TFLOP/s",
             "frac": round(ach / PEAK[dtype], 4), "traffic": tb, "traffic_unit": "bytes/launch (HBM, PMC)",
             "flops_per_launch": a["flops"] / a["n"], "avg_launch_us": round(avg_ms * 1e3, 2),
             "launches_per_step": a["n"], "share_of_device_time": round(a["t"] / total, 4)}
        if warm_times:
            w_ms = a["tw"] / a["n"]
            o["warm_avg_launch_us"] = round(w_ms * 1e3, 2)
            o["warm_frac"] = round((a["flops"] / a["n"]) / (w_ms * 1e-3) / 1e12 / PEAK[dtype], 4)
        return o

    return obj(dom), obj("mam_attention"), total, by


def mam_batched(rt, B=32, per_graph=20, replays=10):
    """Roofline of the MAM attention launch at B frames (2B sequences) on random bf16 q/k/v in the
    runtime's convention (q pre-scaled), timed like kernel_profile (median of 5 timed segments)."""
    import ctypes
    from mmt_amd._lib import LIB, AttnParams, MMT_BF16, check
    d = rt.d
    S = 2 * B
    qkv = (torch.randn(S, d.ntok, 3 * d.C, device="cuda") * 0.5).bfloat16()
    out = torch.empty(S, d.ntok, d.C, device="cuda", dtype=torch.bfloat16)
    p = AttnParams()
    p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H = qkv.data_ptr(), out.data_ptr(), S, B, d.ntok, d.n_t, d.C, d.H
    p.asym = 1 if rt.variant in ("asym", "asym_online") else 0
    p.scale, p.impl = 1.0 / 1.4426950408889634, 0
    st = torch.cuda.current_stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(per_graph):
            check(LIB.mmt_mam_attention(ctypes.byref(p), MMT_BF16, torch.cuda.current_stream().cuda_stream), "attn")
    for _ in range(3):  # warm-up replays (clocks, caches)
        g.replay()
    segs = []  # median of 5 timed segments: the box's clock state moves single segments by several %
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(replays):
            g.replay()
        e1.record(st)
        torch.cuda.synchronize()
        segs.append(e0.elapsed_time(e1) * 1e3 / (replays * per_graph))
    us = sorted(segs)[len(segs) // 2]
    lk_s = d.ntok + (d.n_t if p.asym else 0)
    fl = 4.0 * 64 * d.H * S * (d.n_t * d.n_t + d.ns * lk_s)
    ach = fl / (us * 1e-6) / 1e12
    return mam_memory_roofline({"kernel": "mam_attention", "bound": "mfma", "achieved": round(ach, 2),
                                "peak": PEAK["bf16"], "unit": "TFLOP/s", "frac": round(ach / PEAK["bf16"], 4),
                                "traffic": None, "frames": B, "flops_per_launch": fl, "avg_launch_us": round(us, 2)},
                               S, d.ntok, d.C, 2)


def golden_box_err(variant, dtype):
    """Box error of the forward in `dtype` against the reference-made golden of `variant` at B = 1
    (tests/golden/model_<variant>_b1.npz: the reference's outputs for its own synthetic weights and inputs,
    tests/golden/make_golden.py), measured in this run (None when the variant has no golden)."""
    import json as _json
    import numpy as np
    from mmt_amd import synthetic
    from mmt_amd.runtime import MixFormerRGBTRuntime
    gdir = os.path.join(ROOT, "tests", "golden")
    gpath, kpath = os.path.join(gdir, "model_%s_b1.npz" % variant), os.path.join(gdir, "state_dict_%s.json" % variant)
    if not (os.path.exists(gpath) and os.path.exists(kpath)):
        return None
    keys = _json.load(open(kpath))
    sd = {k: torch.from_numpy(v) for k, v in synthetic.synth_state_dict(keys).items()}
    rt = MixFormerRGBTRuntime(sd, variant, dtype=dtype)
    t, o, s = [[x.cuda() for x in z] for z in synthetic.synth_inputs(1)]
    box, _ = rt.forward(t, o, s)
    torch.cuda.synchronize()
    gold = np.load(gpath)["pred_boxes"].reshape(1, 4)
    return float(np.abs(box.cpu().numpy() - gold).max())


def tracker_step(sd, variant, steps, warmup, H=480, W=640):
    """The tracking loop's per-frame rate (the reference's per-frame time covers crop, H2D and the
    D2H sync, tracker_rgbt.py:172-179): RGBTTrackerCore.track on a pair of uint8 (H, W, 3) frames already resident
    in HBM -- the frame copy into the tracker's buffers, ONE hipGraph replay (both search crops with the resize /
    normalise, the full template + search forward, map-back and clip on the device) and the `.tolist()` of the new
    state, the step's one host round trip.  Synthetic frames and random-init weights: the predicted box wanders, so
    the state is put back to the initial box before every frame (a 32-byte device copy) to keep the crops
    stationary.  Beside the model-only `value`, not instead."""
    if variant != "rgbt":
        return None
    from mmt_amd import model as M
    from mmt_amd.tracking import RGBTTrackerCore
    net = M.build_mixformer_vit_rgbt(M.hot_path_cfg(), train=False)
    net.load_state_dict(sd, strict=True)
    net = net.cuda().eval()
    g = torch.Generator().manual_seed(5)
    frames = [[torch.randint(0, 256, (H, W, 3), generator=g, dtype=torch.uint8).cuda() for _ in range(2)]
              for _ in range(4)]
    core = RGBTTrackerCore(net, 2.0, 128, 5.0, 320, [200], multimodal=False)
    init = [W * 0.4, H * 0.4, 64.0, 48.0]
    core.initialize(frames[0], init)
    init_state = core.state.clone()
    for i in range(warmup):
        core.state.copy_(init_state)
        core.track(frames[i % len(frames)])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        core.state.copy_(init_state)
        core.track(frames[i % len(frames)])
    el = time.perf_counter() - t0  # track() ends in a host sync (.tolist())
    return {"value": round(steps / el, 2), "unit": "frames/s", "ms_per_frame": round(el / steps * 1e3, 4),
            "frame": [H, W], "hip_graph": core._graph is not None,
            "note": "RGBTTrackerCore.track per frame: uint8 frames resident, crop + resize + normalise + forward + "
                    "map-back + clip as one hipGraph replay, plus the host round trip of the new box"}


def fp16_line(sd, variant, pool, score, steps, warmup):
    """The headline workload with the fp16 compute type (same kernels, fp16 operands): its boxes meet
    the north star's 1e-3 on the reference goldens (<= 5.4e-4, tests/test_gpu_model.py) where bf16's
    sit at 1.3-3.5e-3 (within the 1e-2 bf16 bound).  Reported beside the bf16 `value`, not instead."""
    from mmt_amd.runtime import MixFormerRGBTRuntime
    rt = MixFormerRGBTRuntime(sd, variant, dtype=torch.float16)
    graphs = [rt.capture_plan(rt.plan_for_inputs(t, o, s, run_score_head=score)) for t, o, s in pool]
    for i in range(warmup):
        graphs[i % len(graphs)].replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        graphs[i % len(graphs)].replay()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    B = pool[0][0][0].shape[0]
    return {"value": round(B * steps / el, 2), "unit": "frames/s", "ms_per_step": round(el / steps * 1e3, 4),
            "dtype": "fp16", "box_err_vs_reference": golden_box_err(variant, torch.float16),
            "box_err_vs_reference_bf16": golden_box_err(variant, torch.bfloat16),
            "box_err_note": "max |box - reference golden| at B = 1, measured in this run (tests/golden)"}


def kv_cache_tracking(rt, pool, score, steps, warmup):
    """Tracking-loop rate with the template K/V cache: per frame only the search
    pass (one graph replay per resident input set, zero-copy); the template pass runs once per
    template update (every 200 frames in the reference's TEST.UPDATE_INTERVALS) and is timed
    separately.  Returns frames/s of the search pass, its ms, and the template pass's ms."""
    t0_, o0_, _ = pool[0]
    tplan = rt.plan_for_inputs(t0_, o0_, None, part="t")
    tg = rt.capture_plan(tplan)
    sg = [rt.capture_plan(rt.plan_for_inputs(None, None, s, run_score_head=score, part="s")) for _, _, s in pool]
    tg.replay()
    for i in range(warmup):
        sg[i % len(sg)].replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        sg[i % len(sg)].replay()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    n_t = 20
    t1 = time.perf_counter()
    for _ in range(n_t):
        tg.replay()
    torch.cuda.synchronize()
    tel = time.perf_counter() - t1
    B = t0_[0].shape[0]
    return {"value": round(B * steps / el, 2), "unit": "frames/s", "ms_per_step": round(el / steps * 1e3, 4),
            "template_pass_ms": round(tel / n_t * 1e3, 4),
            "note": "search-only pass per frame against the cached template K/V (template pass once per "
                    "template update); not the headline `value`, which runs the full template+search forward"}


def host_cpu():
    """lscpu model / sockets / cores / SMT of the host the CPU baseline ran on."""
    info = {}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        keys = {"Model name": "model", "Socket(s)": "sockets", "Core(s) per socket": "cores_per_socket",
                "Thread(s) per core": "threads_per_core", "CPU(s)": "logical_cpus"}
        for ln in out.splitlines():
            k, _, v = ln.partition(":")
            if k.strip() in keys:
                info[keys[k.strip()]] = v.strip()
    except Exception:  # lscpu absent: report what the OS says
        info["logical_cpus"] = str(os.cpu_count())
    return info


def cgroup_cpus():
    """CPUs the process's cgroup may use (cpu.max quota / period; None = no quota)."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                return max(1, int(int(q) / int(per)))
        except (OSError, ValueError):
            pass
    try:  # cgroup v1
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return max(1, q // per)
    except (OSError, ValueError):
        pass
    return None


def baseline_threads(info):
    """All physical cores available to this process (BASELINE.md:53): lscpu sockets x cores per
    socket, capped by the CPUs of the process's affinity mask and by its cgroup CPU quota (the
    OMP_NUM_THREADS default of the job environment is deliberately not used)."""
    try:
        phys = int(info["sockets"]) * int(info["cores_per_socket"])
    except (KeyError, ValueError):
        phys = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = cgroup_cpus()
    n = min(phys, aff, quota or aff)
    return n, {"physical_cores": phys, "affinity_cpus": aff, "cgroup_cpus": quota}


def cpu_baseline(variant, B, budget_s=12.0, geo=None):
    """Oracle (fp32 CPU restatement of the reference forward; within +-15 % of the reference's own
    CPU time on the same threads, tools/cpu_baseline_check.py -> profiles/cpu_baseline_check.json):
    3 warm-up forwards, then the median of >= 10 timed forwards or as many as fit the budget, on
    every physical core available to the process (baseline_threads)."""
    geo = geo or GEO_B
    from mmt_amd import synthetic
    from oracle.forward import forward as oracle_forward, state_dict_to_torch
    info = host_cpu()
    threads, avail = baseline_threads(info)
    info.update(avail)
    torch.set_num_threads(threads)
    sd = state_dict_to_torch(synthetic.synth_state_dict(state_dict_keys(variant, **geo)))
    t, o, s = synthetic.synth_inputs(B, geo["template"], geo["search"])
    for _ in range(3):
        oracle_forward(sd, variant, t, o, s)
    times, t0 = [], time.perf_counter()
    while len(times) < 10 or time.perf_counter() - t0 < budget_s:
        t1 = time.perf_counter()
        oracle_forward(sd, variant, t, o, s)
        times.append(time.perf_counter() - t1)
        if len(times) >= 200 or (len(times) >= 3 and time.perf_counter() - t0 > 4 * budget_s):
            break
    med = sorted(times)[len(times) // 2]
    return {"value": round(B / med, 3), "unit": "frames/s", "cores": threads, "kind": "port",
            "host": info,
            "sample": "median of %d fp32 CPU forwards of B=%d after 3 warm-up (%s, %d/%d), %.1f s, oracle/forward.py"
                      % (len(times), B, variant, geo["template"], geo["search"], sum(times))}


TRAIN_FLOP_PER_SAMPLE = 3 * 218.59e9  # forward + backward ~ 3 x the 218.59 GFLOP forward


def train_bench(world, rank, B, steps, warmup, device="cuda", ops=None, search=320, template=128, graph=True,
                force_ddp=False):
    """BASELINE config 4: DDP training step of the two-stream MixViT-B RGB-T,
    B LaSOT-shaped synthetic pairs per GPU: forward with autograd on the HIP ops, CIoU + L1 box
    loss, backward with the RCCL gradient all-reduce (DistributedDataParallel, bucketed, overlapped
    with the backward; SyncBatchNorm in the head when world > 1), clip, AdamW
    (mmt_amd.train.TrainStep; reference train_script_mixformer.py:105-140,
    actors/mixformer_rgbt.py:33-168).  Returns the result object (samples/s over all ranks by the
    max-over-ranks time, ms per step, an MFMA roofline of the whole step).  device / ops / image sizes:
    the CPU harness test runs it over gloo with stand-in ops at small images (the product: HipOps).
    force_ddp: the data-parallel step (bucketed all-reduce over the process group) even at world 1."""
    from mmt_amd.model import build_mixformer_vit_rgbt, hot_path_cfg
    from mmt_amd.train import HipOps, TrainStep, synthetic_batch
    torch.manual_seed(0)  # identical initial replicas (DDP also broadcasts rank 0's weights)
    net = build_mixformer_vit_rgbt(hot_path_cfg(search=search, template=template), train=False).to(device).train()
    ddp = world > 1 or force_ddp
    step_fn = TrainStep(net, ops or HipOps, ddp=ddp)
    g = torch.Generator().manual_seed(100 + rank)  # each rank its own shard of the clip batch
    batches = [synthetic_batch(B, device, g, template, search) for _ in range(2)]
    sync = torch.cuda.synchronize if device != "cpu" else (lambda: None)
    last = {}
    # on the device: the whole step captured as one hipGraph (TrainStep.capture; its eager warm-up steps
    # count as this harness's warm-up), each timed step = the copy of that step's batch into the static
    # inputs + one replay.  Under DDP the bucketed RCCL all-reduces are captured with it.
    graphed = graph and device != "cpu" and ops is None
    if graphed:
        static = [[x.clone() for x in z] if isinstance(z, (list, tuple)) else z.clone() for z in batches[0]]
        import mmt_amd.train as _T
        _T.GEMM_ACCOUNT = {}  # every GEMM launch of the capture's steps (warm-up + the captured one), per step below
        try:
            step_fn.capture(*static, warmup=max(1, warmup))
        except RuntimeError as e:
            # no eager fallback in this process: the warm-up steps have already moved the weights and a failed
            # capture can leave the optimizer's pointer table half written and the stream invalidated
            # (ADVICE r4); the caller reports the error (default line) or the run exits non-zero (--train)
            raise RuntimeError("train step capture failed: %s" % str(e)[:300]) from e
    gemm_acc = None
    if graphed:
        gemm_acc = {k: v / (max(1, warmup) + 1) for k, v in _T.GEMM_ACCOUNT.items()}
        _T.GEMM_ACCOUNT = None

        def step(i):
            last["stats"] = step_fn.replay(*batches[i % 2])

        step(0)
    else:
        def step(i):
            last["stats"] = step_fn(*batches[i % 2])

        for i in range(warmup):
            step(i)
    elapsed = timed_steps(step, steps, world, sync, device)
    sps = world * B * steps / elapsed
    ach = sps / world * TRAIN_FLOP_PER_SAMPLE / 1e12  # per GPU
    # HBM bytes of one whole step from the committed counter pass (tools/pmc_train_traffic.py; one GPU, graphed
    # step, this batch), reported only on the kernel sources it was taken on
    tr, tr_note = load_traffic("train", B, "bf16")
    step_bytes = tr.get("step", {}).get("traffic_bytes") if (world == 1 and graphed) else None
    dominant = None
    if graphed and rank == 0 and gemm_acc:
        dominant = train_gemm_roofline(step, gemm_acc, tr if world == 1 else {}, tr_note)
    return {"value": round(sps, 2), "unit": "samples/s", "ms_per_step": round(elapsed / steps * 1e3, 3),
            "batch_per_gpu": B, "steps": steps, "warmup": warmup,
            "parallelism": ("ddp%d (bucketed RCCL gradient all-reduce, fp32)" % world if ddp else "single"),
            "step_issue": "one hipGraph replay per step (whole step captured)" if graphed else "eager",
            "roofline": {"kernel": "train_step (whole step)", "bound": "mfma", "achieved": round(ach, 2),
                         "peak": PEAK["bf16"], "unit": "TFLOP/s", "frac": float("%.4g" % (ach / PEAK["bf16"])),
                         "flops_per_sample": TRAIN_FLOP_PER_SAMPLE, "traffic": step_bytes,
                         "traffic_unit": "bytes/step (HBM, PMC)",
                         "traffic_source": tr_note if (world == 1 and graphed) else "not measured for this setup",
                         "hbm_TBps": round(step_bytes / (elapsed / steps) / 1e12, 3) if step_bytes else None,
                         "dominant": dominant},
            "last_loss": round(float(last["stats"]["loss"]), 5),
            "opt_table_writes": getattr(step_fn.opt, "table_writes", None)}


def train_gemm_roofline(step, acc, tr, tr_note, steps=6):
    """The training step's dominant kernel family, the GEMMs (every mmt_gemm launch: Linear forward / dX / dW,
    the head's implicit-GEMM convolutions): per step the FLOPs and algorithmic bytes counted by the step's own
    GEMM calls (mmt_amd.train.GEMM_ACCOUNT over the capture), the device time of the gemm kernels from
    `steps` graph replays under torch.profiler (the dispatch timestamps a rocprofv3 kernel trace reports), and
    the family's HBM bytes per step from the committed counter pass when it was taken on these sources
    (tools/pmc_train_traffic.py)."""
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        for i in range(steps):
            step(i)
        torch.cuda.synchronize()
    tot = gem = 0.0
    n_gem = n_all = 0
    for e in prof.events():
        if str(getattr(e, "device_type", "")).endswith("CUDA") and e.time_range.end > e.time_range.start:
            d = (e.time_range.end - e.time_range.start) * 1e-6  # us -> s
            tot += d
            n_all += 1
            if "gemm" in e.name:
                gem += d
                n_gem += 1
    if gem <= 0:
        return None
    gem_s, tot_s = gem / steps, tot / steps
    ach = acc["flops"] / gem_s / 1e12
    fam = tr.get("gemm", {}) if tr else {}
    traffic = fam.get("traffic_bytes")
    return {"kernel": "gemm (every mmt_gemm launch of the step)", "bound": "mfma", "achieved": round(ach, 2),
            "peak": PEAK["bf16"], "unit": "TFLOP/s", "frac": float("%.4g" % (ach / PEAK["bf16"])),
            "flops_per_step": acc["flops"], "launches_per_step": round(acc.get("launches", 0)),
            "device_ms_per_step": round(gem_s * 1e3, 3), "share_of_step_device_time": round(gem_s / tot_s, 4),
            "kernel_launches_per_step": round(n_all / steps), "algorithmic_bytes_per_step": round(acc["bytes"]),
            "traffic": traffic, "traffic_unit": "bytes/step (HBM, PMC, gemm kernels)",
            "traffic_over_algorithmic": round(traffic / acc["bytes"], 3) if traffic else None,
            "traffic_source": tr_note if traffic else "no gemm-family counter pass on these sources"}


def timed_steps(step, steps, world, sync, device):
    """The contract's timed region: barrier + sync, exactly `steps` steps, barrier + sync, and the MAX of
    the ranks' elapsed times (the slowest replica sets the job's rate)."""
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    sync()
    if world > 1:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = tt.item()
    return elapsed


def frame_seeds(rank, n=4):
    """Seeds of the resident input sets of one rank: disjoint across ranks (each replica tracks its own
    frames, SURVEY §8(e): single-stream tracking shards by sequence, no data-path collective)."""
    return [1 + n * rank + i for i in range(n)]


def shard_range(total, world, rank):
    """Sequences [lo, hi) of rank `rank` when `total` sequences are sharded over `world` ranks
    (the reference's running.py:134-141 deals whole sequences to workers)."""
    if total % world:
        raise SystemExit("bench.py: --total-seqs %d is not divisible by %d ranks" % (total, world))
    per = total // world
    return rank * per, (rank + 1) * per


def sequence_inputs(seqs, set_idx, template=128, search=320):
    """Synthetic frames of the global sequences `seqs` for input set `set_idx`: each sequence's frame is
    drawn from its own seed (1 + 1000 * set_idx + global index), so a rank's shard is the same data the
    single-process run holds for those sequences."""
    from mmt_amd import synthetic
    parts = [synthetic.synth_inputs(1, template, search, seed=1 + 1000 * set_idx + q) for q in seqs]
    cat = lambda i, m: torch.cat([p[i][m] for p in parts], 0)  # noqa: E731
    return tuple([cat(i, 0), cat(i, 1)] for i in range(3))


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_workers(nprocs, argv, script=None):
    """Start `nprocs` copies of this script, one per GPU (RANK = LOCAL_RANK = i, WORLD_SIZE = nprocs,
    rendezvous on 127.0.0.1), wait for all of them and return the worst exit status.  Runs before
    anything touches the GPU; the workers are children, never an exec of this process."""
    script = script or os.path.abspath(__file__)
    port = str(free_port())
    procs = []
    for r in range(nprocs):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs), LOCAL_WORLD_SIZE=str(nprocs),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def resolve_world(gpus):
    """(world, rank, local_rank) from the launcher's environment; refuses a world size that disagrees
    with --gpus (the line's n_gpus must be what ran)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != gpus:
        raise SystemExit("bench.py: WORLD_SIZE=%d but --gpus %d" % (world, gpus))
    return world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=1, help="frames (sequences) per GPU per step")
    ap.add_argument("--variant", default="rgbt", choices=list(VARIANT_NAMES))
    ap.add_argument("--dtype", default=None, choices=["bf16", "fp16", "f32"],
                    help="default bf16; fp16 for --variant rgb (the RGB-only model refuses bf16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--gemm-impl", type=int, default=0, help="mmt_gemm_params.impl for every GEMM (A/B)")
    ap.add_argument("--attn-impl", type=int, default=0, help="mmt_attn_params.impl for every MAM attention (A/B)")
    ap.add_argument("--no-kernel-profile", action="store_true",
                    help="skip the per-kernel timing (profiler runs that map dispatches to plan entries)")
    ap.add_argument("--dump-plan", default=None, help="write the plan's launch names (JSON) to this path")
    ap.add_argument("--no-mam-batched", action="store_true", help="skip the batched MAM attention roofline")
    ap.add_argument("--no-kv-cache", action="store_true", help="skip the template K/V cache tracking-rate line")
    ap.add_argument("--no-fp16-line", action="store_true", help="skip the fp16 rate of the same workload")
    ap.add_argument("--no-tracker-line", action="store_true", help="skip the tracking-loop (crop + forward + map-back) rate")
    ap.add_argument("--vitl", action="store_true",
                    help="BASELINE config 5 geometry: ViT-L (1024 wide, 24 blocks), 192px templates / 384px search")
    ap.add_argument("--total-seqs", type=int, default=0,
                    help="batched multi-sequence inference (config 3): shard this many sequences over the ranks")
    ap.add_argument("--dry-run", action="store_true",
                    help="harness check without a GPU: resolve ranks and shards over gloo, print them, exit")
    ap.add_argument("--train", action="store_true",
                    help="BASELINE config 4: DDP training step (RCCL gradient all-reduce), --batch pairs per GPU "
                         "(default 16), --steps / --warmup default 20 / 5")
    ap.add_argument("--train-eager", action="store_true",
                    help="training step without the whole-step hipGraph (Python-issued kernels; A/B)")
    ap.add_argument("--force-ddp", action="store_true",
                    help="with --train at one GPU: the data-parallel step over a one-rank RCCL group (bucketed "
                         "all-reduce captured into the step's hipGraph), timed beside the plain step")
    ap.add_argument("--no-train-line", action="store_true",
                    help="skip the short DDP training measurement (train_step) appended to the inference line")
    args = ap.parse_args()
    if args.dtype is None:
        args.dtype = "fp16" if args.variant == "rgb" else "bf16"
    if args.train:
        if args.batch == 1:
            args.batch = 16  # yaml TRAIN.BATCH_SIZE
        if args.steps == 200:
            args.steps = 20
        if args.warmup == 20:
            args.warmup = 5

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:  # self-launch: one worker process per GPU
        sys.exit(launch_workers(args.gpus, sys.argv[1:]))
    world, rank, local = resolve_world(args.gpus)
    sharded = args.total_seqs > 0
    if sharded:
        lo, hi = shard_range(args.total_seqs, world, rank)
        args.batch = hi - lo
    if args.dry_run:
        if world > 1:
            dist.init_process_group("gloo")
        shard = [lo, hi] if sharded else None
        shards = [None] * world
        if world > 1:
            dist.all_gather_object(shards, shard)
        else:
            shards = [shard]
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "batch_per_gpu": args.batch, "shards": shards,
                              "scaling": "strong" if sharded else "weak"}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from mmt_amd import synthetic
    from mmt_amd.runtime import MixFormerRGBTRuntime

    if args.train:
        if args.force_ddp and world == 1:  # a one-rank RCCL group for the DDP step
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(free_port()))
            dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", local))
            plain = train_bench(1, 0, args.batch, args.steps, args.warmup, graph=not args.train_eager)
            torch.cuda.empty_cache()
        res = train_bench(world, rank, args.batch, args.steps, args.warmup, graph=not args.train_eager,
                          force_ddp=args.force_ddp)
        if rank == 0:
            out = {"metric": "train samples/s (two-stream MixViT-B RGB-T DDP step, BASELINE config 4)",
                   "value": res["value"], "unit": "samples/s", "n_gpus": world, "steps": args.steps,
                   "warmup": args.warmup, "ms_per_step": res["ms_per_step"], "higher_is_better": True,
                   "scaling": "weak", "vs_baseline": None,
                   "dtype": "bf16 (backbone GEMM / attention operands), fp32 master weights and accumulation",
                   "data": "synthetic LaSOT-shaped pairs (N(0,1) images, random boxes), random-init weights",
                   "config": {"workload": "mixformer_vit_rgbt ViT-B 128/320 DDP train step, %d pairs/GPU" % args.batch,
                              "batch_per_gpu": args.batch, "parallelism": res["parallelism"]},
                   "roofline": res["roofline"], "cpu_baseline": None, "last_loss": res["last_loss"],
                   "step_issue": res["step_issue"]}
            if args.force_ddp and world == 1:
                out["plain_step"] = {k: plain[k] for k in ("value", "ms_per_step", "parallelism", "step_issue")}
                out["ddp_vs_plain"] = round(res["value"] / plain["value"], 4)
            print(json.dumps(out), flush=True)
        if world > 1 or args.force_ddp:
            dist.barrier()
            dist.destroy_process_group()
        return

    dtype = {"bf16": torch.bfloat16, "fp16": torch.float16}.get(args.dtype, torch.float32)
    geo = GEO_L if args.vitl else (GEO_RGB if args.variant == "rgb" else GEO_B)
    nmod = 1 if args.variant == "rgb" else 2  # modalities per frame
    keys = state_dict_keys(args.variant, **geo)
    sd = {k: torch.from_numpy(v) for k, v in synthetic.synth_state_dict(keys).items()}
    rt = MixFormerRGBTRuntime(sd, args.variant, dtype=dtype)
    rt.gemm_impl = args.gemm_impl
    rt.attn_impl = args.attn_impl
    B = args.batch
    score = args.variant == "asym_online"
    pool = []
    for i, seed in enumerate(frame_seeds(rank)):  # distinct frames per rank, resident in HBM before timing
        if sharded:  # this rank's slice of the global batch
            t, o, s = sequence_inputs(range(lo, hi), i, geo["template"], geo["search"])
        else:
            t, o, s = synthetic.synth_inputs(B, geo["template"], geo["search"], seed=seed)
        t, o, s = t[:nmod], o[:nmod], s[:nmod]
        pool.append(([x.cuda() for x in t], [x.cuda() for x in o], [x.cuda() for x in s]))
    use_graph = not args.no_graph
    # one hipGraph per resident input set: the patch staging reads that set in place (zero-copy)
    plans = [rt.plan_for_inputs(t, o, s, run_score_head=score) for t, o, s in pool]
    graphs = [rt.capture_plan(p) for p in plans] if use_graph else None

    def step(i):
        if use_graph:
            graphs[i % len(pool)].replay()
        else:
            rt.run_plan(plans[i % len(pool)])

    for i in range(args.warmup):
        step(i)
    elapsed = timed_steps(step, args.steps, world, torch.cuda.synchronize, "cuda")

    ws = rt.workspace(B)
    plan = ws["plan_score"] if score else ws["plan"]
    if args.dump_plan and rank == 0:
        with open(args.dump_plan, "w") as f:
            json.dump([e[2] for e in plan], f)
    if args.no_kernel_profile:
        dom = mam = by = None
        dev_ms = span_ms = None
    else:
        times, span_ms = inframe_profile(graphs, plan) if use_graph else (None, None)
        warm = kernel_profile(rt, plan)
        timing = "in-frame (profiler dispatch timestamps of graph-replayed frames, median of 20)"
        if times is None:  # no profiler records: the warm back-to-back figure, labelled as such
            times, timing = warm, "warm back-to-back launches (no in-frame records)"
        traffic, traffic_note = load_traffic(args.variant, B, args.dtype)
        dom, mam, dev_ms, by = roofline(rt, plan, times, args.dtype, traffic, warm)
        for o in (dom, mam):
            o["traffic_source"] = traffic_note
        for o in (dom, mam):
            o["timing"] = timing

    if rank == 0:
        frames = world * B * args.steps
        if sharded:
            load = "%d sequences sharded over %d GPU(s) (%d per GPU), one frame each per step" % (
                args.total_seqs, world, B)
        else:
            load = "%d frame(s)/GPU/step" % B
        out = {
            "metric": METRIC, "value": round(frames / elapsed, 2), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "strong" if sharded else "weak", "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic N(0,1) frames (seeded), seed-hash random-init weights (mmt-synth-v1)",
            "config": {"workload": "%s %s %dpx template x2 + %dpx search, %s, %s%s"
                                   % (VARIANT_NAMES[args.variant], "ViT-L" if args.vitl else "ViT-B", geo["template"],
                                      geo["search"], "RGB" if args.variant == "rgb" else "RGB+TIR", load,
                                      ", score head on" if score else ""),
                       "variant": args.variant, "batch_per_gpu": B, "total_sequences": args.total_seqs or None,
                       "template": geo["template"], "search": geo["search"], "hidden": geo["hidden"],
                       "depth": geo["depth"],
                       "parallelism": ("dp%d sharded sequences" % world if sharded else
                                       "replicas x%d" % world if world > 1 else "single"),
                       "hip_graph": use_graph},
            "roofline": dom,
            "roofline_mam": mam_memory_roofline(mam, nmod * B, rt.d.ntok, rt.d.C, 4 if args.dtype == "f32" else 2),
            "device_ms_per_step_sum": round(dev_ms, 4) if dev_ms else None,
            "inframe_span_ms": round(span_ms, 4) if span_ms else None, "launches_per_step": len(plan),
            "kernels": {k: {"us": round(a["t"] * 1e3 / a["n"], 2), "n": a["n"],
                            "tflops": round(a["flops"] / a["n"] / (a["t"] / a["n"] * 1e-3) / 1e12, 1) if a["flops"] else None}
                        for k, a in sorted(by.items(), key=lambda kv: -kv[1]["t"])} if by else None,
        }
        if args.dtype == "bf16" and not args.no_kernel_profile and not args.no_mam_batched:
            out["roofline_mam_batched"] = mam_batched(rt)
            out["roofline_mam_batched_b8"] = mam_batched(rt, B=8)
        if use_graph and not args.no_kv_cache and args.variant != "asym_ce":  # no template cache with CE
            out["tracking_kv_cache"] = kv_cache_tracking(rt, pool, score, args.steps, args.warmup)
        if use_graph and args.dtype == "bf16" and not args.no_fp16_line and args.variant != "asym_ce":
            out["fp16_line"] = fp16_line(sd, args.variant, pool, score, args.steps, args.warmup)
        if use_graph and args.dtype == "bf16" and B == 1 and not args.no_tracker_line and not args.vitl:
            try:
                out["tracker_step"] = tracker_step(sd, args.variant, args.steps, args.warmup)
            except Exception as e:  # noqa: BLE001  (reported, not raised: the headline line must still print)
                out["tracker_step"] = {"error": "%s: %s" % (type(e).__name__, e)}
    if not args.no_train_line and args.variant == "rgbt" and not args.vitl and not sharded:
        # config 4's DDP step beside the replicas: the one data-path collective (RCCL gradient
        # all-reduce) is timed at every N of a scaling run; a failure is reported, not raised
        del graphs, plans, pool
        torch.cuda.empty_cache()
        try:
            train_res = train_bench(world, rank, 16, 10, 3, graph=not args.train_eager)  # 10 timed steps: 5 read one-off stalls
        except Exception as e:  # noqa: BLE001
            train_res = {"error": "%s: %s" % (type(e).__name__, e)}
    else:
        train_res = None
    if rank == 0:
        out["train_step"] = train_res
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.variant, B, budget_s=20.0 if args.vitl else 12.0, geo=geo)
            if B == 1 and not args.vitl:  # BASELINE.md:58: B = 1 and B = 8
                out["cpu_baseline_b8"] = cpu_baseline(args.variant, 8, budget_s=12.0, geo=geo)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
