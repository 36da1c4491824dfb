"""Drop-in for lib/test/tracker/mixformer_vit_rgbt.py: MixFormer RGB-T tracker (build_mixformer_vit_rgbt, Preprocessor_wo_mask) on the MI355X."""
from lib.models.mixformer_vit_rgbt import build_mixformer_vit_rgbt

from ._rgbt import make_tracker_class

MixFormer = make_tracker_class(build_mixformer_vit_rgbt, multimodal=False, online_score=False)


def get_tracker_class():
    return MixFormer
