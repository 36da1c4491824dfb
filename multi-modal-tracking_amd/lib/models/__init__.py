"""lib.models: only the RGB-T hot-path family (mixformer_vit_rgbt) is provided."""
