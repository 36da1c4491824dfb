"""Golden vectors for the tracker pre/post-processing, from the REFERENCE's own Python (CPU).

Run here only (the reference tree does not exist on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_tracker.py

What is recorded (tests/golden/tracker_geometry.npz):
  - sample_target(im, box, factor, output_sz=None) of lib/train/data/processing_utils.py:15-77 for
    boxes inside, across each edge and corner of a random frame: the padded crop's shape and
    SHA-256 digest (the crop itself when it is small).
    cv2 is absent from this image; the only cv2 call on that path is copyMakeBorder(...,
    BORDER_CONSTANT), stubbed here by the exact numpy constant pad.  The resize (cv2.resize) is not
    on that path and stays unpinned (oracle/preprocess.py says so).
  - MixFormer.map_box_back (lib/test/tracker/mixformer_vit_rgbt.py:124-131) + clip_box
    (lib/utils/box_ops.py:155-164) of the reference on random predictions; the tracker's
    (pred * search_size / resize_factor).tolist() step is computed as torch does it on the GPU.
Nothing is written under /root/reference (sys.dont_write_bytecode).
"""
import hashlib
import os
import sys
import types

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import make_golden  # noqa: E402  (stub recipe of SURVEY §8c; inserts /root/reference into sys.path)


def _copy_make_border(img, top, bottom, left, right, border_type, value=None):
    assert border_type == 0  # cv.BORDER_CONSTANT
    return np.pad(img, ((top, bottom), (left, right)) + ((0, 0),) * (img.ndim - 2), mode="constant")


def _no_resize(*a, **k):
    raise RuntimeError("cv2.resize is not part of the pinned geometry path")


def install():
    make_golden.install_stubs()
    cv = types.ModuleType("cv2")
    cv.BORDER_CONSTANT = 0
    cv.copyMakeBorder = _copy_make_border
    cv.resize = _no_resize
    sys.modules["cv2"] = cv
    mpl = types.ModuleType("matplotlib")
    mpl.pyplot = types.ModuleType("matplotlib.pyplot")
    sys.modules["matplotlib"] = mpl
    sys.modules["matplotlib.pyplot"] = mpl.pyplot
    # lib/train/__init__.py pulls in the training admin (tensorboardX, ...): load processing_utils.py
    # by path under its package name instead, with empty parent packages.
    import importlib.util
    for pkg in ("lib.train", "lib.train.data"):
        m = types.ModuleType(pkg)
        m.__path__ = []
        sys.modules[pkg] = m
    path = os.path.join(make_golden.REF, "lib", "train", "data", "processing_utils.py")
    spec = importlib.util.spec_from_file_location("lib.train.data.processing_utils", path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[spec.name] = mod
    spec.loader.exec_module(mod)


def main():
    install()
    from lib.train.data.processing_utils import sample_target
    from lib.test.tracker.mixformer_vit_rgbt import MixFormer
    from lib.utils.box_ops import clip_box

    rng = np.random.default_rng(7)
    H, W = 240, 320
    im = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    boxes = [[100.3, 80.7, 40.2, 30.9], [2.0, 3.0, 50.0, 40.0], [290.5, 200.25, 25.0, 35.5], [-10.0, -5.0, 30.0, 20.0],
             [300.0, 100.0, 60.0, 60.0], [150.0, 220.0, 20.0, 30.0], [0.0, 0.0, 320.0, 240.0], [159.5, 119.5, 1.0, 1.0],
             [10.25, 200.75, 12.5, 33.0], [200.0, 10.0, 64.0, 64.0]]
    rec = {"im": im, "boxes": np.array(boxes, dtype=np.float64), "factors": np.array([2.0, 4.5], dtype=np.float64)}
    for bi, b in enumerate(boxes):
        for fi, f in enumerate(rec["factors"]):
            crop, att, one = sample_target(im, b, float(f), output_sz=None)
            # large random crops do not compress: keep the full array for small ones, a digest for all
            rec["crop_shape_%d_%d" % (bi, fi)] = np.array(crop.shape, dtype=np.int64)
            rec["crop_sha256_%d_%d" % (bi, fi)] = np.frombuffer(hashlib.sha256(np.ascontiguousarray(crop).tobytes()).digest(), np.uint8)
            if crop.size <= 64 * 64 * 3:
                rec["crop_%d_%d" % (bi, fi)] = crop
    # box post-processing: the tracker's own arithmetic on random predictions
    n = 64
    preds = rng.uniform(0.0, 1.0, (n, 4)).astype(np.float32)
    preds[:, 2:] *= 0.6
    states = np.stack([rng.uniform(-20, W, n), rng.uniform(-20, H, n), rng.uniform(5, 120, n), rng.uniform(5, 120, n)], 1)
    rfs = rng.uniform(0.5, 4.0, n)
    out, pred_list = [], []
    search_size = 320
    for i in range(n):
        tr = types.SimpleNamespace(state=[float(v) for v in states[i]], params=types.SimpleNamespace(search_size=search_size))
        pred_boxes = torch.from_numpy(preds[i:i + 1]).view(-1, 4)
        # the tracker's `(pred_boxes.mean(dim=0) * search_size / resize_factor).tolist()` runs on the
        # GPU, where torch divides an fp32 tensor by a Python float as x * (1 / float32(rf))
        # (BinaryDivTrueKernel.cu's CPU-scalar path); the CPU build here would divide exactly, so that
        # step is written out in the GPU's form and the reference code pins what follows it
        inv = torch.tensor(1.0, dtype=torch.float32) / torch.tensor(float(rfs[i]), dtype=torch.float32)
        pred_box = ((pred_boxes.mean(dim=0) * search_size) * inv).tolist()
        pred_list.append(pred_box)
        out.append(clip_box(MixFormer.map_box_back(tr, pred_box, float(rfs[i])), H, W, margin=10))
    rec.update({"pred": preds, "state": states, "rf": rfs, "new_state": np.array(out, dtype=np.float64),
                "pred_box": np.array(pred_list, dtype=np.float64),
                "H": np.int64(H), "W": np.int64(W), "search_size": np.int64(search_size)})
    np.savez_compressed(os.path.join(HERE, "tracker_geometry.npz"), **rec)
    print("wrote tracker_geometry.npz (%d crops, %d box updates)" % (len(boxes) * 2, n))


if __name__ == "__main__":
    main()
