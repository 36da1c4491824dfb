"""Drop-in for lib/models/mixformer_vit_rgbt/asymmetric_shared_ce.py (asymmetric MAM with candidate
elimination)."""
from mmt_amd.model import MixFormer_RGBT_CE as MixFormer_RGBT, build_asymmetric_shared_ce  # noqa: F401
