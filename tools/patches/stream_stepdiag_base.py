# The step diagnostic of stream_stepdiag.py applied to the stream kernel as committed at the start of round 4
# (git show 510e06e:psgla_for_posterior_sampling_amd/csrc/tv_stream.hip > /tmp/tv_stream_r04base.hip).
import os as _os
import runpy as _runpy
_d = _runpy.run_path(_os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "stream_stepdiag.py"))
SOURCE_OVERRIDE = {"tv_stream.hip": "/tmp/tv_stream_r04base.hip"}
_N = open(SOURCE_OVERRIDE["tv_stream.hip"]).read().count("step_barrier();")
PATCHES = [
    ("struct StreamShared {\n", _d["DIAG"] + "struct StreamShared {\n", 1),
    ("    float red[SP_MAXSEG][SP_MAXST][2];\n};\n", "    float red[SP_MAXSEG][SP_MAXST][2];\n    StepDiag sd;\n};\n" + _d["FN"], 1),
    ("step_barrier();", "diag_barrier(sh);", _N),
    _d["PATCHES"][-1],
]
