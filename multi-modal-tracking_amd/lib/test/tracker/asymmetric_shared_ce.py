"""Drop-in for lib/test/tracker/asymmetric_shared_ce.py: MixFormer RGB-T tracker with candidate elimination
(build_asymmetric_shared_ce, Preprocessor_Multimodal) on the MI355X.  Every frame runs the full forward
(the elimination depends on the search tokens, so there is no template-only pass)."""
from lib.models.mixformer_vit_rgbt.asymmetric_shared_ce import build_asymmetric_shared_ce

from ._rgbt import make_tracker_class

MixFormer = make_tracker_class(build_asymmetric_shared_ce, multimodal=True, online_score=False, kv_cache=False)


def get_tracker_class():
    return MixFormer
