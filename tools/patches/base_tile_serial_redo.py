"""Diagnostic baseline: the library before the tile kernel's parallel early-stop redo (round 5: the tile kernel's
finalising workgroup recomputes stopped chains serially), from a commit's sources against the current ABI header --
for interleaved A/Bs of the step itself (tools/ab_bench.sh).  Needs /tmp/base_head/*.hip|hpp exported from git first:
    for f in api.hip tv_stream.hip tv_tile.hip psgla_common.hpp; do git show 8fd98e3:psgla_for_posterior_sampling_amd/csrc/$f > /tmp/base_head/$f; done"""
SOURCE_OVERRIDE = {f: "/tmp/base_head/" + f for f in ("api.hip", "tv_stream.hip", "tv_tile.hip", "psgla_common.hpp")}
PATCHES = []
