"""Drop-in for lib/models/mixformer_vit_rgbt/asymmetric_shared.py (cross-modal asymmetric MAM)."""
from mmt_amd.model import MixFormer_RGBT_Asymmetric as MixFormer_RGBT, build_asymmetric_shared  # noqa: F401
