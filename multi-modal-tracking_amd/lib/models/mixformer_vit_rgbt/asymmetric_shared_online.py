"""Drop-in for lib/models/mixformer_vit_rgbt/asymmetric_shared_online.py (+ score prediction module)."""
from mmt_amd.model import MixFormer_RGBT_OnlineScore, build_asymmetric_shared_online_score  # noqa: F401
