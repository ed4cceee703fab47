"""Timing variant: the row stream's front waves at issue priority 2 during phase 0 (the Philox of the row), 0 otherwise."""
PATCHES = [("            // ---- phase 0: Philox of row q; DMA part 0 of row q + 4\n",
            "            // ---- phase 0: Philox of row q; DMA part 0 of row q + 4\n            __builtin_amdgcn_s_setprio(2);\n", 1),
           ("            // ---- phase 1: Box-Muller pair 1; DMA part 1\n",
            "            // ---- phase 1: Box-Muller pair 1; DMA part 1\n            __builtin_amdgcn_s_setprio(0);\n", 1)]
