"""Variant: the tile kernel's pending-redo word redo[0] loaded at kernel entry, beside the step counter and the
restart flag (its latency overlaps theirs), instead of inside the redo branch."""
PATCHES = [
    ("""    const long long step = launch_step(a);
    const bool fresh = launch_fresh(a);
    const int P = a.B * a.C;""", """    const long long step = launch_step(a);
    const bool fresh = launch_fresh(a);
    const int pend_w = __builtin_amdgcn_readfirstlane(a.par_redo ? a.redo[0] : 0);
    const int P = a.B * a.C;""", 1),
    ("""            const int pend = __builtin_amdgcn_readfirstlane(a.redo[0]);
            if (pend & 1) {""", """            const int pend = pend_w;
            if (pend & 1) {""", 1),
]
