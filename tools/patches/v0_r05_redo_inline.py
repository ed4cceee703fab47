"""Diagnostic variant: the parallel early-stop redo inlined ahead of the step kernel's main pass (next launch, grid
barrier) instead of its own kernel -- sources saved from the working tree of round 5 in /tmp/v0_src."""
SOURCE_OVERRIDE = {f: "/tmp/v0_src/" + f for f in ("api.hip", "tv_stream.hip", "tv_tile.hip", "psgla_common.hpp")}
PATCHES = []
