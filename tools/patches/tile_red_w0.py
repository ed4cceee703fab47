"""The tile kernel with the rel-err sums of all iterations on wave 0's lanes (before round 4's spread over waves)."""
SOURCE_OVERRIDE = {"tv_tile.hip": "/tmp/tv_tile_redw0.hip"}
