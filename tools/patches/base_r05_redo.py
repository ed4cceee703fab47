"""Diagnostic baseline: the library as before the parallel early-stop redo (commit 8e78aeb: serial recompute by the
finalising workgroup, no redo buffer), built from that commit's sources against the current ABI header -- for
interleaved A/Bs of the step itself (tools/ab_bench.sh).  Needs /tmp/base_src/*.hip|hpp exported from git first:
    for f in api.hip tv_stream.hip tv_tile.hip psgla_common.hpp; do git show 8e78aeb:psgla_for_posterior_sampling_amd/csrc/$f > /tmp/base_src/$f; done"""
SOURCE_OVERRIDE = {f: "/tmp/base_src/" + f for f in ("api.hip", "tv_stream.hip", "tv_tile.hip", "psgla_common.hpp")}
PATCHES = []
