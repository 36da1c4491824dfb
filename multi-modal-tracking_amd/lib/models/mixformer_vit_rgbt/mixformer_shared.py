"""Drop-in for lib/models/mixformer_vit_rgbt/mixformer_shared.py (shared backbone)."""
from mmt_amd.model import MixFormer_RGBT_Shared as MixFormer_RGBT, build_mixformer_vit_rgbt_shared  # noqa: F401
