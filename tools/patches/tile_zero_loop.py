"""The tile kernel's finaliser reading the norm copies with fetch_add(0) and zeroing them in a separate store pass
(before round 4's read-and-reset exchanges)."""
SOURCE_OVERRIDE = {"tv_tile.hip": "/tmp/tv_tile_zeroloop.hip"}
