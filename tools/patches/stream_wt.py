PATCHES = []
FORCE = ["tv_stream.hip"]   # the working tree stream kernel (phase-unrolled front / back, cached segment geometry)
