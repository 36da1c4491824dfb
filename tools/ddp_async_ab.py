#!/usr/bin/env python3
"""World-1 DDP training step (bench.train_bench with force_ddp, one-rank RCCL group, the step captured as one
hipGraph) with the bucket all-reduces asynchronous (joined after the backward) vs joined at their launch
(mmt_amd.train.ALLREDUCE_ASYNC), interleaved, beside the plain single-process step."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main(steps=10, warmup=3):
    import bench
    import mmt_amd.train as T
    dist.init_process_group("nccl", rank=0, world_size=1)
    torch.cuda.set_device(0)
    for rep in range(2):
        for mode in ("async", "joined", "plain"):
            T.ALLREDUCE_ASYNC = mode == "async"
            r = bench.train_bench(1, 0, 16, steps, warmup, force_ddp=mode != "plain")
            print(json.dumps({"mode": mode, "rep": rep, "samples_per_s": r["value"], "ms_per_step": r["ms_per_step"],
                              "parallelism": r["parallelism"]}), flush=True)
            torch.cuda.empty_cache()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
