"""The row stream's fast primal with the TV anchor Y (rounds 1-5) instead of tau_opt Y (A/B of the round-6 change)."""
PATCHES = [
    ("""                    sh.y[q & (SP_YRING - 1)][lane] = EXACT ? Y4 : make_float4(a.tau_opt * Y4.x, a.tau_opt * Y4.y,
                                                                              a.tau_opt * Y4.z, a.tau_opt * Y4.w);""",
     """                    sh.y[q & (SP_YRING - 1)][lane] = Y4;""", 1),
    ("""        } else if (A1) {
            // (x2 - tau tt + tau Y) / (1 + tau) with the anchor held as tau_opt Y (round 6: one VALU fewer)""",
     """        } else if (false) {
            // (x2 - tau tt + tau Y) / (1 + tau) with the anchor held as tau_opt Y (round 6: one VALU fewer)""", 1),
]
