# The row-stream kernel as committed at the start of round 4 (510e06e), linked against the current library:
# A/B baseline for the stream-kernel changes of round 4.  Run it with --stream-windows whole (it has no
# half-wave windows).  git show 510e06e:psgla_for_posterior_sampling_amd/csrc/tv_stream.hip > /tmp/tv_stream_r04base.hip
SOURCE_OVERRIDE = {"tv_stream.hip": "/tmp/tv_stream_r04base.hip"}
PATCHES = [
    ("void launch_stream(const TvArgs& s, dim3 grid, hipStream_t st, bool exact, bool alpha1, bool gen) {",
     "void launch_stream(const TvArgs& s, dim3 grid, hipStream_t st, bool exact, bool alpha1, bool gen, bool) {", 1),
]
