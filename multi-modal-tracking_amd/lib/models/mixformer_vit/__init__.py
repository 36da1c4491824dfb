"""Drop-in for lib/models/mixformer_vit/__init__.py (RGB-only MixFormer-ViT, BASELINE config 1)."""
from pkgutil import extend_path

# Overlay, not replacement: the same package directories found later on sys.path (the reference
# checkout's lib/, e.g. appended by tracking/test.py:10-12) join this package's search path, so the
# modules this tree does not provide (lib.config, lib.train, lib.test.evaluation, lib.utils, ...)
# still import from there, while the ones it does provide come from here.
__path__ = extend_path(__path__, __name__)

from mmt_amd.model import build_mixformer_vit  # noqa: E402,F401
