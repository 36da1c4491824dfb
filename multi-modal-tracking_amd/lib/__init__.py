"""Drop-in mirror of the reference package paths for the MixFormer RGB-T hot path (MI355X build)."""
