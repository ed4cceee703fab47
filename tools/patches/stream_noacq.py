# Variant: with the parallel redo the stream's finaliser reads the rel-err sums by agent-scope atomic loads (they were
# written by agent atomics) and skips the L2-invalidating agent acquire, which only the serial recompute's re-stream
# of other workgroups' outputs needs.
PATCHES = [
    ("""        if (s_flag) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");""",
     """        if (s_flag && !a.par_redo) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");""", 1),
    ("""            const double nd = a.norms[((size_t)g * a.n_tv + t) * 2];
            const double nn = a.norms[((size_t)g * a.n_tv + t) * 2 + 1];""",
     """            const double nd = __hip_atomic_load(&a.norms[((size_t)g * a.n_tv + t) * 2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const double nn = __hip_atomic_load(&a.norms[((size_t)g * a.n_tv + t) * 2 + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);""", 1),
]
