"""Source stamp of the measured code: a digest of everything that decides which kernels a frame
launches and what they do (the HIP sources and build file, the C ABI header, the launch-plan
runtime).  Measurements committed under profiles/ that depend on the kernels (the PMC traffic
per launch, tools/pmc_traffic.py) carry it, and bench.py only reports them for a tree with the
same digest.  Sources, not the built .so: hipcc stamps each object with a random CUID, so the
library's bytes change on every rebuild of identical sources."""
import glob
import hashlib
import os

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # multi-modal-tracking_amd/
ROOT = os.path.dirname(PKG)


def source_files():
    files = sorted(glob.glob(os.path.join(PKG, "csrc", "*.hip")) + glob.glob(os.path.join(PKG, "csrc", "*.hpp")))
    files += [os.path.join(PKG, "csrc", "Makefile"), os.path.join(ROOT, "include", "mmt_hip.h"),
              os.path.join(PKG, "mmt_amd", "runtime.py"), os.path.join(PKG, "mmt_amd", "_lib.py")]
    return files


def train_source_files():
    """The training step's launch mix also lives in the autograd Functions and the optimizer."""
    return source_files() + [os.path.join(PKG, "mmt_amd", n) for n in ("train.py", "optim.py", "functional.py")]


def source_digest(train=False):
    h = hashlib.sha256()
    for f in (train_source_files() if train else source_files()):
        h.update(os.path.relpath(f, ROOT).encode())
        with open(f, "rb") as fh:
            h.update(hashlib.sha256(fh.read()).digest())
    return h.hexdigest()[:16]
