"""MI355X-native MixFormer RGB-T tracking path (host side)."""
