"""Timing-only ablation (wrong data): the classic row stream's stage waves 2..n neither read nor write their LDS rings
(stage 1 still reads the front's staging; the back still reads ring n, never written)."""
PATCHES = [
    ("""            const int sl = j & 1;
            X2 = sh.x2[rin][sl][lane];
            A = sh.ua[rin][sl][lane];
            B = sh.ub[rin][sl][lane];
        }
        U0 = make_float4(A.x, A.z, B.x, B.z);
        U1 = make_float4(A.y, A.w, B.y, B.w);
    };
    auto store_row = [&](int i, const StageRow& r, const float (&un0)[CPL], const float (&un1)[CPL]) {
        const int so = i & 1;
        sh.x2[rout][so][lane] = make_float4(r.x2n[0], r.x2n[1], r.x2n[2], r.x2n[3]);
        sh.ua[rout][so][lane] = make_float4(un0[0], un1[0], un0[1], un1[1]);
        sh.ub[rout][so][lane] = make_float4(un0[2], un1[2], un0[3], un1[3]);
    };
    // rows 0 and 1: primal update only (segments hold >= 2 rows: row 1 never starts one)""", """            X2 = YY; A = YY; B = make_float4(YY.y, YY.x, YY.w, YY.z);
        }
        U0 = make_float4(A.x, A.z, B.x, B.z);
        U1 = make_float4(A.y, A.w, B.y, B.w);
    };
    auto store_row = [&](int i, const StageRow& r, const float (&un0)[CPL], const float (&un1)[CPL]) {
        asm volatile("" :: "v"(r.x2n[0]), "v"(r.x2n[1]), "v"(r.x2n[2]), "v"(r.x2n[3]), "v"(un0[0]), "v"(un0[1]), "v"(un0[2]),
                     "v"(un0[3]), "v"(un1[0]), "v"(un1[1]), "v"(un1[2]), "v"(un1[3]));
    };
    // rows 0 and 1: primal update only (segments hold >= 2 rows: row 1 never starts one)""", 1),
]
