"""Timing-only ablation (wrong samples): the tile kernel's noise replaced by a cheap hash of its quad (no Philox, no
Box-Muller); run with --tv-tol 0.  Measures whether the tile's head (loads + noise) waits on the noise's VALU."""
PATCHES = [
    ("""        normal_quad(a.seed, (uint32_t)(a.chain0 + b), (uint32_t)step, TAG_LANGEVIN,
                    noise_quad((size_t)c * H + (rv[r] ? gi[r] : 0), gj0, W), Zn[r]);""",
     """        {
            const uint32_t hq = noise_quad((size_t)c * H + (rv[r] ? gi[r] : 0), gj0, W) * 2654435761u + (uint32_t)step;
            Zn[r][0] = (float)(int)hq * 4.6566e-10f; Zn[r][1] = (float)(int)(hq ^ 0x5bd1e995u) * 4.6566e-10f;
            Zn[r][2] = (float)(int)(hq * 3u) * 4.6566e-10f; Zn[r][3] = (float)(int)(hq * 7u) * 4.6566e-10f;
        }""", 1),
]
