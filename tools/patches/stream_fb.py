# The phase-unrolled front / back with cached segment geometry, before ring 0 was removed (round 4, exp_libs/src/fb).
SOURCE_OVERRIDE = {"tv_stream.hip": "/tmp/tv_stream_fb.hip"}
PATCHES = [
    ("void launch_stream(const TvArgs& s, dim3 grid, hipStream_t st, bool exact, bool alpha1, bool gen) {",
     "void launch_stream(const TvArgs& s, dim3 grid, hipStream_t st, bool exact, bool alpha1, bool gen, bool) {", 1),
]
