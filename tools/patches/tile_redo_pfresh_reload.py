"""Diagnostic: the pending bit from the flag word, but the redone step's restart flag re-read inside the redo branch
(an agent-scope atomic load of the word, not the value loaded at kernel entry)."""
PATCHES = [
    ("""                    if (nstop < a.n_tv)
                        sb_tile<EXACT, ALPHA1, R, GEN, NW>(a, sh, plane, seg, band, nstop, false, step - 1,
                                                           lf.pfresh, [] {});""",
     """                    if (nstop < a.n_tv) {
                        const int fw = __builtin_amdgcn_readfirstlane(
                            __hip_atomic_load(a.fresh_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                        sb_tile<EXACT, ALPHA1, R, GEN, NW>(a, sh, plane, seg, band, nstop, false, step - 1,
                                                           (fw & 4) != 0, [] {});
                    }""", 1),
]
