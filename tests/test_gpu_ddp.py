"""The data-parallel training step over a real RCCL process group on the GPU (reference
train_script_mixformer.py:104-110, run_training_ddp.py:94): a fresh child process with a one-rank "nccl" group
runs TrainStep(ddp=True) (the step's own bucketed all-reduce, SyncBatchNorm in the head) eagerly and captured
as one hipGraph, against the single-process step (tests/ddp_nccl_child.py holds the checks)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


def test_ddp_step_over_rccl_matches_single_process(tmp_path):
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    out = tmp_path / "ddp.json"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    child = os.path.join(os.path.dirname(__file__), "ddp_nccl_child.py")
    r = subprocess.run([sys.executable, "-u", child, str(out)], env=env, capture_output=True, text=True, timeout=100)
    print(r.stdout[-4000:], r.stderr[-4000:])
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads(out.read_text())
    print(json.dumps(rec))
    assert rec["ok"] and rec["backend"] == "nccl" and rec["sync_bn_modules"] > 0
