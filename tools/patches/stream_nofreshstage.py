"""The row stream's stage 1 selecting the TV restart itself (rounds 4-5) instead of the front overwriting the staging
(A/B of the round-6 change)."""
PATCHES = [
    ("""            X2 = sh.stX(j & 3, j)[lane];
            A = sh.stUa(j & 3, j)[lane];
            B = sh.stUb(j & 3, j)[lane];""",
     """            const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
            X2 = sel4(fresh, YY, sh.stX(j & 3, j)[lane]);
            A = sel4(fresh, zero4, sh.stUa(j & 3, j)[lane]);
            B = sel4(fresh, zero4, sh.stUb(j & 3, j)[lane]);""", 1),
    ("""                    if (fresh) {
                        sh.stX(fw, q)[lane] = Y4;
                        sh.stUa(fw, q)[lane] = zero4;
                        sh.stUb(fw, q)[lane] = zero4;
                    }""", "", 1),
]
