"""Timing-only ablation (wrong samples): the fast dual's projection without the transcendental (ths * s2 instead
of ths * rsq(s2)) -- what v_rsq_f32 costs (run with --tv-tol 0)."""
PATCHES = [
    ("a.ths * __builtin_amdgcn_rsqf(s2)", "a.ths * s2", 3),
]
