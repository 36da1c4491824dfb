"""Drop-in for lib/models/mixformer_vit_rgbt/__init__.py:1-2 (HIP-backed builders); the reference's
other modules of this package (fusion_utils, deformable_attention, ...) stay importable through the overlay."""
from pkgutil import extend_path

# Overlay, not replacement: the same package directories found later on sys.path (the reference
# checkout's lib/, e.g. appended by tracking/test.py:10-12) join this package's search path, so the
# modules this tree does not provide (lib.config, lib.train, lib.test.evaluation, lib.utils, ...)
# still import from there, while the ones it does provide come from here.
__path__ = extend_path(__path__, __name__)

from mmt_amd.model import build_mixformer_vit_rgbt, build_mixformer_vit_rgbt_shared  # noqa: E402,F401
