"""Timing-only ablation: no rel-err tracking in the inner iterations (stream stage waves; tile kernel's tracked loop
runs untracked) -- what the early-stop sums cost (run with --tv-tol 0: the stop never fires in any leg)."""
PATCHES = [
    ("const bool trk = track && role == 1 &&", "const bool trk = false && track && role == 1 &&", 1),
    ("for (int it = t0; it < t1; ++it) iteration(it, std::false_type{}, TM1{});",
     "for (int it = t0; it < t1; ++it) iteration(it, std::false_type{}, TM0{});", 1),
]
