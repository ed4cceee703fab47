# Tile kernel: the primal of each wave's first row (the only one that needs the LDS hand-off from the
# wave above) last, so the LDS read's latency overlaps the other rows' primal.  Bit-identical TV
# arithmetic; the rel-err partial sums add the rows in the order 1, 2, 0.
PATCHES = [("""        for (int r = 0; r < R; ++r) {
            if (!act_p) break;
            const float u1l = __int_as_float(""", """        for (int rr = 0; rr < R; ++rr) {
            const int r = (rr + 1) % R;
            if (!act_p) break;
            const float u1l = __int_as_float(""", 1)]
