"""Drop-in for lib/test/tracker/mixformer_vit_rgbt_shared.py: MixFormer RGB-T tracker (build_mixformer_vit_rgbt_shared, Preprocessor_Multimodal) on the MI355X."""
from lib.models.mixformer_vit_rgbt import build_mixformer_vit_rgbt_shared

from ._rgbt import make_tracker_class

MixFormer = make_tracker_class(build_mixformer_vit_rgbt_shared, multimodal=True, online_score=False)


def get_tracker_class():
    return MixFormer
