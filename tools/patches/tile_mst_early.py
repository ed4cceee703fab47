"""The tile kernel as committed before the deferred mean / sq DMA (issued with the other loads at the start)."""
SOURCE_OVERRIDE = {"tv_tile.hip": "/tmp/tv_tile_head.hip"}
