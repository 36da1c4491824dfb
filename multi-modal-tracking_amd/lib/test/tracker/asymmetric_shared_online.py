"""Drop-in for lib/test/tracker/asymmetric_shared_online.py: MixFormer RGB-T tracker (build_asymmetric_shared_online_score, Preprocessor_Multimodal, score-gated online template) on the MI355X."""
from lib.models.mixformer_vit_rgbt.asymmetric_shared_online import build_asymmetric_shared_online_score

from ._rgbt import make_tracker_class

MixFormer = make_tracker_class(build_asymmetric_shared_online_score, multimodal=True, online_score=True)


def get_tracker_class():
    return MixFormer
