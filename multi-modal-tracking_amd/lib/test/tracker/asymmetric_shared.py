"""Drop-in for lib/test/tracker/asymmetric_shared.py: MixFormer RGB-T tracker (build_asymmetric_shared, Preprocessor_Multimodal) on the MI355X."""
from lib.models.mixformer_vit_rgbt.asymmetric_shared import build_asymmetric_shared

from ._rgbt import make_tracker_class

MixFormer = make_tracker_class(build_asymmetric_shared, multimodal=True, online_score=False)


def get_tracker_class():
    return MixFormer
