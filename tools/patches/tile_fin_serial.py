"""The tile kernel as committed before the finaliser's norm-copy reads were issued back to back (one round trip per
copy)."""
SOURCE_OVERRIDE = {"tv_tile.hip": "/tmp/tv_tile_head.hip"}
