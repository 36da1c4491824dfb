"""Shared body of the four RGB-T tracker entry points (drop-in for lib/test/tracker/
mixformer_vit_rgbt.py, mixformer_vit_rgbt_shared.py, asymmetric_shared.py,
asymmetric_shared_online.py, asymmetric_shared_ce.py; each defines `MixFormer` and `get_tracker_class()`).

Same constructor, `initialize(image, info)` and `track(image, info)` contract as the reference
(mixformer_vit_rgbt.py:13-121): `params` carries cfg, template_factor, template_size,
search_factor, search_size, checkpoint, save_all_boxes; `image` is [image_v, image_i] (H, W, 3)
uint8 frames (numpy, or torch uint8 tensors already on the device); `track` returns
{"target_bbox": [x, y, w, h]}.  The per-frame crop, preprocessing, forward and box
post-processing run on the MI355X as one hipGraph (mmt_amd.tracking.RGBTTrackerCore).
"""
import torch

from mmt_amd.tracking import RGBTTrackerCore

try:  # the reference's BaseTracker (with its visdom helpers) when its lib/ is overlaid
    from lib.test.tracker.basetracker import BaseTracker
except ModuleNotFoundError:  # standalone: the same interface, lib/test/tracker/basetracker.py:4-22
    from ._basetracker import BaseTracker


def _update_intervals(cfg, dataset_name):
    """mixformer_vit_rgbt.py:39-44: per-dataset template update intervals."""
    name = dataset_name.upper()
    ui = cfg.TEST.UPDATE_INTERVALS
    if hasattr(ui, name) or (isinstance(ui, dict) and name in ui):
        return ui[name]
    return cfg.DATA.MAX_SAMPLE_INTERVAL


# Template K/V cache default, from measurement (profiles/r02_kv_cache.json): a single-sequence tracker
# runs batch 1, where the search-only pass is no faster than the full forward (906 vs 912 frames/s:
# the batch-1 GEMMs are one wave of tiles with or without the 128 template rows); at batch 8 it
# gains 12 % (1981 vs 1764).  params.kv_cache overrides it.
KV_CACHE_DEFAULT = False


def make_tracker_class(builder, multimodal, online_score=False, kv_cache=KV_CACHE_DEFAULT):
    class MixFormer(BaseTracker):
        def __init__(self, params, dataset_name):
            super().__init__(params)
            network = builder(params.cfg, train=False)
            if getattr(params, "checkpoint", None):
                ck = torch.load(params.checkpoint, map_location="cpu", weights_only=True)
                network.load_state_dict(ck["net"], strict=True)
            self.cfg = params.cfg
            self.network = network.cuda()
            self.network.eval()
            self.save_all_boxes = getattr(params, "save_all_boxes", False)
            self.update_intervals = _update_intervals(self.cfg, dataset_name)
            self.core = RGBTTrackerCore(self.network, params.template_factor, params.template_size,
                                        params.search_factor, params.search_size, self.update_intervals,
                                        multimodal=multimodal, online_score=online_score,
                                        kv_cache=getattr(params, "kv_cache", kv_cache))
            self.state = None
            self.frame_id = 0

        def initialize(self, image, info: dict):
            """image: [image_v, image_i]; info["init_bbox"]: (bbox_v, bbox_i), the RGB box is used."""
            self.core.initialize(image, info["init_bbox"][0])
            self.state = [float(v) for v in info["init_bbox"][0]]
            self.frame_id = 0
            if self.save_all_boxes:
                return {"all_boxes": info["init_bbox"] * self.cfg.MODEL.NUM_OBJECT_QUERIES}

        def track(self, image, info: dict = None):
            self.frame_id += 1
            self.state = self.core.track(image)
            if self.save_all_boxes:  # mixformer_vit_rgbt.py:131-134: the unclipped box mapped back
                rf = self.params.search_size / self.core.last_crop_sz
                box = [v * self.params.search_size / rf for v in self.core.last_pred_box()]
                return {"target_bbox": self.state, "all_boxes": self.map_box_back(box, rf)}
            return {"target_bbox": self.state}

        def map_box_back(self, pred_box: list, resize_factor: float):
            """mixformer_vit_rgbt.py:124-131 (host form; the tracking step runs it on the device).  Like
            the reference's map_box_back_batch for all_boxes (:133-139), it reads the current state,
            which at that point is already this frame's (clipped) result."""
            cx_prev, cy_prev = self.state[0] + 0.5 * self.state[2], self.state[1] + 0.5 * self.state[3]
            cx, cy, w, h = pred_box
            half_side = 0.5 * self.params.search_size / resize_factor
            cx_real, cy_real = cx + (cx_prev - half_side), cy + (cy_prev - half_side)
            return [cx_real - 0.5 * w, cy_real - 0.5 * h, w, h]

    return MixFormer
