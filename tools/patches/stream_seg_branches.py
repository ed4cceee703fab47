"""The row-stream kernel as committed before round 4's segment-edge selects (two inlined copies of the dual and the
primal per stage step, chosen by scalar branches)."""
SOURCE_OVERRIDE = {"tv_stream.hip": "/tmp/tv_stream_head.hip"}
