"""Device-resident RGB-T tracking loop: the host side of the reference trackers
(lib/test/tracker/mixformer_vit_rgbt.py, mixformer_vit_rgbt_shared.py, asymmetric_shared.py,
asymmetric_shared_online.py) with their per-frame work moved onto the MI355X.

Per frame the reference does, on the host: two cv2 crops (sample_target), the preprocessor
(H2D copy, /255, normalise; cv2.applyColorMap JET on the TIR crop for the multimodal
preprocessor), the network forward, `.tolist()` of the box (a device sync), map_box_back and
clip_box in Python (tracker.py:75-106).  Here one tracking step is ONE hipGraph replay of
  mmt_sample_target (both search crops, computed from the device-resident state)
  -> the model's launch plan (zero-copy: its patch staging reads the crop buffers in place)
  -> mmt_track_update (box scaling, map_box_back, clip_box; the state is updated on the device)
and the only host round trip is the one the API needs: returning `target_bbox` as a list (and,
for the online-score tracker, its `pred_score.item()` decision, as in the reference).

The arithmetic of both kernels follows the reference bit for bit where it is pinned (crop
geometry and padding, map-back, clip) and OpenCV's fixed-point resize / colour map where cv2
would run (see csrc/preprocess.hip; oracle/preprocess.py restates both).
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import LIB, CropParams, check

MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)


def jet_lut():
    """[256][3] (B, G, R) uint8 JET colour map: the piecewise-linear jet of OpenCV's COLORMAP_JET,
    x = i / 255 (r = clip(min(4x - 1.5, 4.5 - 4x)), g = .. 0.5 / 3.5, b = .. -0.5 / 2.5), x255, rounded."""
    x = np.arange(256, dtype=np.float64) / 255.0
    r = np.clip(np.minimum(4 * x - 1.5, -4 * x + 4.5), 0, 1)
    g = np.clip(np.minimum(4 * x - 0.5, -4 * x + 3.5), 0, 1)
    b = np.clip(np.minimum(4 * x + 0.5, -4 * x + 2.5), 0, 1)
    lut = np.stack([b, g, r], 1).astype(np.float32) * np.float32(255.0)
    return np.clip(np.rint(lut), 0, 255).astype(np.uint8)


def _ptr(t):
    return t.data_ptr() if t is not None else None


def crop_params(image, box, factor, out_sz, out=None, patch=None, crop=None, lut=None):
    """mmt_crop_params for one crop.  image (H,W,3) uint8, box (4,) fp64, out (1,3,s,s) fp32,
    patch (s,s,3) uint8, crop (4,) fp64, lut (256,3) uint8 -- all device tensors."""
    if image.dtype != torch.uint8 or image.dim() != 3 or image.shape[2] != 3 or not image.is_contiguous():
        raise ValueError("image must be a contiguous (H, W, 3) uint8 device tensor")
    if box.dtype != torch.float64 or box.numel() != 4:
        raise ValueError("box must be 4 float64 values (x, y, w, h)")
    for t, shape, dt in ((out, (3 * out_sz * out_sz,), torch.float32), (patch, (out_sz * out_sz * 3,), torch.uint8),
                         (crop, (4,), torch.float64), (lut, (768,), torch.uint8)):
        if t is not None and (t.dtype != dt or t.numel() != shape[0] or not t.is_contiguous() or t.device != image.device):
            raise ValueError("crop buffer of shape %s / %s on %s expected" % (shape, dt, image.device))
    p = CropParams()
    p.image, p.H, p.W = image.data_ptr(), image.shape[0], image.shape[1]
    p.box, p.factor, p.out_sz = box.data_ptr(), float(factor), int(out_sz)
    p.lut = _ptr(lut)
    for c in range(3):
        p.mean[c], p.std[c] = MEAN[c], STD[c]
    p.out, p.patch, p.crop = _ptr(out), _ptr(patch), _ptr(crop)
    return p


def sample_target(params_list, stream=None):
    """Launch mmt_sample_target for up to 4 crops of equal out_sz."""
    n = len(params_list)
    arr = (CropParams * n)(*params_list)
    s = torch.cuda.current_stream().cuda_stream if stream is None else stream
    check(LIB.mmt_sample_target(arr, n, s), "mmt_sample_target")
    return arr


class RGBTTrackerCore:
    """Tracking state and per-frame step of one sequence on the current device.

    network: a built HIP model (mmt_amd.model); multimodal: apply the JET colour map to the TIR
    crops (Preprocessor_Multimodal) or not (Preprocessor_wo_mask); online_score: the
    asymmetric_shared_online tracker's score-gated online-template update."""

    def __init__(self, network, template_factor, template_size, search_factor, search_size, update_intervals,
                 multimodal, online_score=False, use_graph=True, kv_cache=False):
        self.net = network
        # kv_cache: the template tokens' per-layer qkv are computed once per template update (a
        # separate template pass) and each frame runs only the search tokens (runtime.cache_workspace);
        # off by default: no faster at batch 1 (lib/test/tracker/_rgbt.py KV_CACHE_DEFAULT)
        self.kv_cache = bool(kv_cache)
        self._tmpl_dirty = True
        self._tmpl_graph = self._tmpl_plan = None
        self.tf, self.ts, self.sf, self.ss = float(template_factor), int(template_size), float(search_factor), int(search_size)
        self.update_intervals = list(update_intervals)
        self.online_score = bool(online_score)
        self.use_graph = bool(use_graph)
        self.dev = torch.device("cuda", torch.cuda.current_device())
        dev = self.dev
        self.lut = torch.from_numpy(jet_lut().reshape(-1)).to(dev) if multimodal else None
        e = lambda *s, dt=torch.float32: torch.empty(*s, device=dev, dtype=dt)  # noqa: E731
        self.state = e(4, dt=torch.float64)
        self.template = [e(1, 3, self.ts, self.ts) for _ in range(2)]
        self.online_template = [e(1, 3, self.ts, self.ts) for _ in range(2)]
        self.online_max_template = [e(1, 3, self.ts, self.ts) for _ in range(2)]
        self.search = [e(1, 3, self.ss, self.ss) for _ in range(2)]
        self.search_crop = e(2, 4, dt=torch.float64)
        self.tmpl_crop = e(2, 4, dt=torch.float64)
        self.frames = None
        self._graph = None
        self._plan = None
        self._rt = None
        self._tmpl_graph = None
        self.frame_id = 0
        self.max_pred_score = -1.0

    # ------------------------------------------------------------------ frames
    def _load_frames(self, image):
        """Copy the two (H, W, 3) uint8 frames (numpy or torch) into fixed device buffers."""
        if not isinstance(image, (list, tuple)) or len(image) != 2:
            raise ValueError("image must be [image_v, image_i]")
        ims = [torch.as_tensor(np.ascontiguousarray(x)) if isinstance(x, np.ndarray) else x for x in image]
        H, W = ims[0].shape[:2]
        if any(tuple(x.shape) != (H, W, 3) or x.dtype != torch.uint8 for x in ims):
            raise ValueError("frames must be two (H, W, 3) uint8 images of the same size")
        if self.frames is None or tuple(self.frames[0].shape) != (H, W, 3):
            self.frames = [torch.empty(H, W, 3, device=self.dev, dtype=torch.uint8) for _ in range(2)]
            self._graph = self._plan = None
        for dst, src in zip(self.frames, ims):
            dst.copy_(src, non_blocking=src.device.type == "cuda")
        return H, W

    def _crop_templates(self, dst, box):
        """Both modalities' template crops at `box` (device fp64) into dst[0] / dst[1]."""
        ps = [crop_params(self.frames[m], box, self.tf, self.ts, out=dst[m].view(-1), crop=self.tmpl_crop[m],
                          lut=self.lut if m == 1 else None) for m in range(2)]
        sample_target(ps)

    # ------------------------------------------------------------------ per-frame plan
    def _build_step(self):
        rt = self.net._runtime(self.dev)
        # the captured graphs hold raw pointers into this runtime's weights and workspace: keep it
        # alive, and rebuild when the network swaps it (load_state_dict / .to() / refresh_kernels)
        self._rt = rt
        score = self.online_score
        H, W = self.frames[0].shape[:2]
        self._keep = [crop_params(self.frames[m], self.state, self.sf, self.ss, out=self.search[m].view(-1),
                                  crop=self.search_crop[m], lut=self.lut if m == 1 else None) for m in range(2)]
        arr = (CropParams * 2)(*self._keep)
        part = "s" if self.kv_cache else None
        model_plan = rt.plan_for_inputs(self.template, self.online_template, self.search, run_score_head=score,
                                        part=part)
        ws = rt.workspace(1)
        if self.kv_cache:
            self._tmpl_plan = rt.plan_for_inputs(self.template, self.online_template, None, part="t")
            self._tmpl_graph = rt.capture_plan(self._tmpl_plan) if self.use_graph else None
            self._tmpl_dirty = True
        self._ws = ws
        plan = [(LIB.mmt_sample_target, (arr, 2), "track_sample_target", arr)]
        plan += model_plan
        plan.append((LIB.mmt_track_update, (ws["BOX"].data_ptr(), self.search_crop.data_ptr(), self.state.data_ptr(), 1,
                                            H, W, self.ss, 10.0), "track_update", None))
        self._plan = plan
        if self.use_graph:
            # capture_plan runs the plan once before recording it, and mmt_track_update moves the
            # state: keep the state of this frame across the capture
            saved = self.state.clone()
            self._graph = rt.capture_plan(plan)
            self.state.copy_(saved)
        else:
            self._graph = None

    def _step(self):
        if self._plan is not None and self.net._runtime(self.dev) is not self._rt:
            self._graph = self._plan = self._tmpl_graph = None  # weights reloaded: re-plan, re-capture
            self._tmpl_dirty = True
        if self._plan is None or (self.use_graph and self._graph is None):
            self._build_step()
        if self.kv_cache and self._tmpl_dirty:  # template pass after a template / online-template change
            if self._tmpl_graph is not None:
                self._tmpl_graph.replay()
            else:
                self._rt.run_plan(self._tmpl_plan)
            self._tmpl_dirty = False
        if self._graph is not None:
            self._graph.replay()
        else:
            self._rt.run_plan(self._plan)

    # ------------------------------------------------------------------ tracker API
    def initialize(self, image, init_bbox):
        self._load_frames(image)
        self.state.copy_(torch.tensor([float(v) for v in init_bbox], dtype=torch.float64))
        self._crop_templates(self.template, self.state)
        for m in range(2):
            self.online_template[m].copy_(self.template[m])
            # reference defect D6 (asymmetric_shared_online.py:115): online_max_template is read
            # before it is ever assigned if no frame scores > 0.5 before the first update frame;
            # here it starts as the template instead of raising AttributeError
            self.online_max_template[m].copy_(self.template[m])
        self.frame_id = 0
        self.max_pred_score = -1.0
        self._tmpl_dirty = True
        self._check_crop(self.tmpl_crop)

    def track(self, image):
        """One frame: returns the new state [x, y, w, h] (Python floats)."""
        self._load_frames(image)
        self.frame_id += 1
        self._step()
        if self.online_score:
            pred_score = torch.sigmoid(self._ws["SC"].view(1)).item()
            if pred_score > 0.5 and pred_score > self.max_pred_score:
                self._crop_templates(self.online_max_template, self.state)
                self.max_pred_score = pred_score
            for update_i in self.update_intervals:
                if self.frame_id % update_i == 0:
                    for m in range(2):
                        self.online_template[m].copy_(self.online_max_template[m])
                        self.online_max_template[m].copy_(self.template[m])
                    self.max_pred_score = -1
                    self._tmpl_dirty = True
        else:
            for update_i in self.update_intervals:
                if self.frame_id % update_i == 0:
                    self._crop_templates(self.online_template, self.state)
                    self._tmpl_dirty = True
        vals = torch.cat([self.state, self.search_crop[:, 2]]).tolist()  # the step's one host round trip
        if min(vals[4:]) < 1:
            raise Exception("Too small bounding box.")  # processing_utils.py:36-37
        self.last_crop_sz = vals[4]  # this frame's RGB search crop side (resize factor = search_size / it)
        return vals[:4]

    def last_pred_box(self):
        """This frame's network box (cx, cy, w, h), normalised to the search crop (one extra host copy)."""
        return self._ws["BOX"].view(-1, 4)[0].tolist()

    def _check_crop(self, crop):
        if float(crop[:, 2].min()) < 1:
            raise Exception("Too small bounding box.")  # processing_utils.py:36-37
