"""Drop-in for lib/models/mixformer_vit_rgbt/__init__.py:1-2 (HIP-backed builders)."""
from mmt_amd.model import build_mixformer_vit_rgbt, build_mixformer_vit_rgbt_shared  # noqa: F401
