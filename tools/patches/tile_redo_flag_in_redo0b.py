"""Diagnostic (redo0b: as redo0, but the flag word still carries the pending bits): the tile kernel's pending early-stop redo flag in redo[0] (as first built in round 5) instead of the
step's flag word -- isolates the flag's location in the 72-row tile's exact-mode parity."""
PATCHES = [
    ("""        if (a.par_redo && (a.fin_inline || a.redo_only)) {
            if (lf.pend) {""", """        if (a.par_redo && (a.fin_inline || a.redo_only)) {
            const int pend0 = __builtin_amdgcn_readfirstlane(a.redo[0]);
            if (pend0 & 1) {""", 1),
    ("""                        sb_tile<EXACT, ALPHA1, R, GEN, NW>(a, sh, plane, seg, band, nstop, false, step - 1,
                                                           lf.pfresh, [] {});""",
     """                        sb_tile<EXACT, ALPHA1, R, GEN, NW>(a, sh, plane, seg, band, nstop, false, step - 1,
                                                           (pend0 & 2) != 0, [] {});""", 1),
    ("""        for (int g = threadIdx.x; g < G; g += blockDim.x) a.redo[4 + g] = sh.s_stop[g];
        if (threadIdx.x == 0) a.redo[1] = 0;
    } else if (sh.s_item) {""", """        for (int g = threadIdx.x; g < G; g += blockDim.x) a.redo[4 + g] = sh.s_stop[g];
        if (threadIdx.x == 0) {
            a.redo[1] = 0;
            a.redo[0] = sh.s_item ? (1 | (fresh ? 2 : 0)) : 0;
        }
    } else if (sh.s_item) {""", 1),
]
