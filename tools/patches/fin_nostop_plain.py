# Variant: the no-stop finaliser path zeroes the sums with plain stores instead of agent-scope atomic stores.
PATCHES = [("""                __hip_atomic_store(n0, 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(n0 + 1, 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (a.par_redo && threadIdx.x == 0) {""", """                n0[0] = 0.0;
                n0[1] = 0.0;
            }
        }
        if (a.par_redo && threadIdx.x == 0) {""", 1)]
