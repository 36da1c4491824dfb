#!/usr/bin/env python3
"""Training-step throughput of the two-stream MixFormer RGB-T (BASELINE.json config 4, SURVEY
§8(e) C4): forward with autograd, CIoU + L1 box loss, backward, RCCL gradient all-reduce
(DistributedDataParallel, SyncBatchNorm in the head), clip and AdamW, on LaSOT-shaped synthetic
pairs (mmt_amd.train.synthetic_batch), `--batch` sequences per GPU.

    python tools/train_bench.py --steps 10 --warmup 3
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/train_bench.py ...

One JSON line from rank 0: samples/s over all ranks (max-over-ranks time), ms per step."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=16, help="sequences per GPU (yaml TRAIN.BATCH_SIZE)")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from mmt_amd.model import build_mixformer_vit_rgbt, hot_path_cfg
    from mmt_amd.train import HipOps, TrainStep, synthetic_batch

    torch.manual_seed(0)  # identical initial replicas (DDP also broadcasts rank 0's weights)
    net = build_mixformer_vit_rgbt(hot_path_cfg(), train=False).cuda().train()
    step = TrainStep(net, HipOps, ddp=world > 1)
    g = torch.Generator().manual_seed(100 + rank)
    batches = [synthetic_batch(args.batch, "cuda", g) for _ in range(2)]
    for i in range(args.warmup):
        step(*batches[i % 2])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        stats = step(*batches[i % 2])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    if rank == 0:
        print(json.dumps({
            "metric": "train samples/s (two-stream MixViT-B RGB-T DDP step)", "value": round(world * args.batch * args.steps / el, 2),
            "unit": "samples/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 2), "higher_is_better": True, "scaling": "weak",
            "dtype": "bf16 backbone GEMM/attention, fp32 master weights",
            "data": "synthetic LaSOT-shaped pairs (N(0,1) images, random boxes), random-init weights",
            "config": {"workload": "mixformer_vit_rgbt ViT-B 128/320 train step", "batch_per_gpu": args.batch,
                       "parallelism": "ddp%d" % world},
            "last_loss": round(stats["loss"].item(), 5)}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
