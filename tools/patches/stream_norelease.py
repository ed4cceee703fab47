# Variant: the row stream's per-workgroup agent release before the arrival count only when the finaliser may
# re-stream chains in this launch (serial early-stop recompute, par_redo = 0): with the parallel redo nothing in this
# launch reads another workgroup's plain stores (the rel-err sums are agent atomics; the kernel boundary releases).
PATCHES = [("""        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const int old = __hip_atomic_fetch_add(a.arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);""",
            """        if (!a.par_redo) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const int old = __hip_atomic_fetch_add(a.arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);""", 1)]
