"""Drop-in for lib/models/mixformer_vit/mixformer.py (RGB-only MixFormer, BASELINE config 1)."""
from mmt_amd.model import MixFormer, build_mixformer_vit  # noqa: F401
