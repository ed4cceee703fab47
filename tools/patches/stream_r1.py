# The row-stream kernel at d74b03e (round 4: unrolled front / back, no ring 0, half-wave windows) -- A/B baseline
# for the front's noise spread.  git show d74b03e:psgla_for_posterior_sampling_amd/csrc/tv_stream.hip > /tmp/tv_stream_r1.hip
SOURCE_OVERRIDE = {"tv_stream.hip": "/tmp/tv_stream_r1.hip"}
PATCHES = []
