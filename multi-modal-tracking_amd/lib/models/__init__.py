"""lib.models: the RGB-T hot-path family (mixformer_vit_rgbt) and the RGB-only MixViT (mixformer_vit, config 1)."""
