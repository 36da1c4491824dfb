"""Drop-in for lib/models/mixformer_vit/__init__.py (RGB-only MixFormer-ViT, BASELINE config 1)."""
from mmt_amd.model import build_mixformer_vit  # noqa: F401
