# Diagnostic (never in the product): tools/patches/tile_phasediag.py plus stamp 7 in the finalising workgroup right
# after the norms' exchange loop (its __syncthreads), splitting the finalisation into the norms round trip and the rest.
import os
import runpy

_base = runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "tile_phasediag.py"))
PATCHES = list(_base["PATCHES"]) + [
    ("            if (rel < a.tol) atomicOr(&sh.s_stop[g], 1 << t);\n        }\n    }\n    __syncthreads();\n",
     "            if (rel < a.tol) atomicOr(&sh.s_stop[g], 1 << t);\n        }\n    }\n    __syncthreads();\n    tdiag(step, 7);\n", 1),
]
