"""Drop-in mirror of the reference's lib/test (tracker entry points of the RGB-T models)."""
