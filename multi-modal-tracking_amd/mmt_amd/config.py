"""EasyDict-style config tree + yaml overlay, the subset of the reference's config system the hot
path reads (lib/config/mixformer_vit_rgbt/config.py:7-96, update_config_from_file :134-138).
`easydict` is not installed here, so a minimal compatible EasyDict is provided."""
import copy

import yaml


class EasyDict(dict):
    """dict with recursive attribute access (drop-in for easydict.EasyDict)."""

    def __init__(self, d=None, **kw):
        super().__init__()
        for k, v in dict(d or {}, **kw).items():
            self[k] = v

    def __setitem__(self, k, v):
        if isinstance(v, dict) and not isinstance(v, EasyDict):
            v = EasyDict(v)
        elif isinstance(v, list):
            v = [EasyDict(x) if isinstance(x, dict) and not isinstance(x, EasyDict) else x for x in v]
        super().__setitem__(k, v)

    __setattr__ = __setitem__

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k)

    def __deepcopy__(self, memo):
        return EasyDict(copy.deepcopy(dict(self), memo))


def default_cfg(model="mixformer_vit_rgbt"):
    """Defaults of lib/config/<model>/config.py (hot-path relevant keys and the TEST block)."""
    cfg = EasyDict()
    cfg.MODEL = EasyDict(
        VIT_TYPE="base_patch16", HEAD_TYPE="CORNER", HIDDEN_DIM=768, NUM_OBJECT_QUERIES=1, POSITION_EMBEDDING="sine",
        PREDICT_MASK=False, BACKBONE=EasyDict(PRETRAINED=True, PRETRAINED_PATH=""), FUSION_LAYERS=6,
        FUSION_CLASS="Attention_Fusion_Bimodal",
    )
    if model == "asymmetric_shared_online":
        cfg.MODEL.TRACKER_PRETRAINED_PATH = ""
        cfg.MODEL.SCORE_PRETRAINED_PATH = ""
    else:
        cfg.MODEL.RGBT_PRETRAINED_PATH = ""
    cfg.TRAIN = EasyDict(RGBT_TRACK=True, AMP=False, BATCH_SIZE=16, LR=0.0001, WEIGHT_DECAY=0.0001, EPOCH=300,
                         IOU_WEIGHT=2.0, L1_WEIGHT=5.0, GRAD_CLIP_NORM=0.1, BACKBONE_MULTIPLIER=0.1)
    cfg.DATA = EasyDict(MEAN=[0.485, 0.456, 0.406], STD=[0.229, 0.224, 0.225], MAX_SAMPLE_INTERVAL=[200],
                        SEARCH=EasyDict(SIZE=288, FACTOR=5.0, CENTER_JITTER=4.5, SCALE_JITTER=0.5),
                        TEMPLATE=EasyDict(SIZE=128, FACTOR=2.0, NUMBER=1, CENTER_JITTER=0, SCALE_JITTER=0))
    cfg.TEST = EasyDict(LOAD_FROME_TRAIN_RESULT=False, TEMPLATE_FACTOR=2.0, TEMPLATE_SIZE=128, SEARCH_FACTOR=5.0,
                        SEARCH_SIZE=288, EPOCH=500,
                        UPDATE_INTERVALS=EasyDict(LASOT=[200], GOT10K_TEST=[200], TRACKINGNET=[200], VOT20=[200],
                                                  VOT20LT=[200]))
    return cfg


def _update(base, exp):
    for k, v in exp.items():
        if k in base and isinstance(v, dict) and isinstance(base[k], dict):
            _update(base[k], v)
        else:
            base[k] = v


def update_config_from_file(cfg, filename):
    """Overlay a yaml file onto cfg (reference: update_config_from_file, config.py:134-138)."""
    with open(filename) as f:
        exp = EasyDict(yaml.safe_load(f))
    _update(cfg, exp)
    return cfg
