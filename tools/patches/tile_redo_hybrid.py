"""Diagnostic: the pending bit from the flag word (bit 1 only), the redone step's restart flag from redo[0]."""
PATCHES = [
    ("""                    if (nstop < a.n_tv)
                        sb_tile<EXACT, ALPHA1, R, GEN, NW>(a, sh, plane, seg, band, nstop, false, step - 1,
                                                           lf.pfresh, [] {});""",
     """                    if (nstop < a.n_tv) {
                        const int pend0 = __builtin_amdgcn_readfirstlane(a.redo[0]);
                        sb_tile<EXACT, ALPHA1, R, GEN, NW>(a, sh, plane, seg, band, nstop, false, step - 1,
                                                           (pend0 & 2) != 0, [] {});
                    }""", 1),
    ("""        for (int g = threadIdx.x; g < G; g += blockDim.x) a.redo[4 + g] = sh.s_stop[g];
        if (threadIdx.x == 0) a.redo[1] = 0;
    } else if (sh.s_item) {""", """        for (int g = threadIdx.x; g < G; g += blockDim.x) a.redo[4 + g] = sh.s_stop[g];
        if (threadIdx.x == 0) {
            a.redo[1] = 0;
            a.redo[0] = sh.s_item ? (1 | (fresh ? 2 : 0)) : 0;
        }
    } else if (sh.s_item) {""", 1),
]
