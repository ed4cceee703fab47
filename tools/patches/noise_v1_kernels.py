"""The row-stream and tile kernels as of round 4 before psgla noise v2 (flat quad numbering: W % 4 != 0 rows
straddle two quads, two Philox per lane), for an interleaved A/B against the product.  Requires
/tmp/tv_stream_main.hip and /tmp/tv_tile_main.hip (git show main:psgla_for_posterior_sampling_amd/csrc/...)."""
SOURCE_OVERRIDE = {"tv_stream.hip": "/tmp/tv_stream_main.hip", "tv_tile.hip": "/tmp/tv_tile_main.hip"}
