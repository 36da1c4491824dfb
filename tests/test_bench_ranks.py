"""bench.py's multi-GPU contract on CPU (gloo, world size 2): each replica runs its own frames (disjoint
input seeds, no data-path collective) and the job time is the MAX over ranks of the barrier-bracketed
timed region, so value = frames of all ranks / the slowest rank's time (SURVEY §8(e) replicas)."""
import os

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    """A port the OS reports free on 127.0.0.1 (fixed ports collided under parallel test runs)."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _worker(rank, world, port, out):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import time

    import bench
    calls = []

    def step(i):
        calls.append(i)
        time.sleep(0.02 * (rank + 1) / 5)  # rank 1 is the slower replica

    elapsed = bench.timed_steps(step, 5, world, lambda: None, "cpu")
    out[rank] = (elapsed, calls, bench.frame_seeds(rank))
    dist.destroy_process_group()


def test_timed_region_is_max_over_ranks_and_seeds_disjoint():
    world, port = 2, _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    (e0, c0, s0), (e1, c1, s1) = res[0], res[1]
    assert c0 == c1 == list(range(5))  # exactly `steps` steps on every rank
    assert e0 == e1  # every rank reports the same (max) time
    assert e0 >= 5 * 0.02 * 2 / 5 * 0.95  # >= the slower rank's own time
    assert not set(s0) & set(s1)
