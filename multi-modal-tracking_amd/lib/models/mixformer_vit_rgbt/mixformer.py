"""Drop-in for lib/models/mixformer_vit_rgbt/mixformer.py (two-stream model)."""
from mmt_amd.model import MixFormer_RGBT, build_mixformer_vit_rgbt  # noqa: F401
