# Tile kernel: the mean / sq LDS-DMA of the core rows issued after the data term (so the data term's
# vector-memory wait does not include them) and LDS-only barriers in the iteration loop (the DMA stays in
# flight through the iterations; the wave waits vmcnt(0) before reading the staged rows at the end).
MST = """    if (need_prev && n_it >= 0) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (rv[r] && core[r]) {
                const size_t base = poff + (size_t)gi[r] * L + gjc;
                glds16(a.mean[par_in] + base, &sh.mst[w * R + r][0][0]);
                glds16(a.sq[par_in] + base, &sh.mst[w * R + r][1][0]);
            }
        }
    }
"""
PATCHES = [
    (MST, "", 1),
    ("""    sh.urow[w][lane] = make_float4(u0[R - 1][0], u0[R - 1][1], u0[R - 1][2], u0[R - 1][3]);
    __syncthreads();
""", """    sh.urow[w][lane] = make_float4(u0[R - 1][0], u0[R - 1][1], u0[R - 1][2], u0[R - 1][3]);
""" + MST + """    lds_barrier();
""", 1),
    ("""            if ((lane & 15) == 0) sh.red[it][w][lane >> 4] = rs;
        }
        __syncthreads();""", """            if ((lane & 15) == 0) sh.red[it][w][lane >> 4] = rs;
        }
        lds_barrier();""", 1),
    ("""        if (act_d) sh.urow[w][lane] = make_float4(u0[R - 1][0], u0[R - 1][1], u0[R - 1][2], u0[R - 1][3]);
        __syncthreads();""", """        if (act_d) sh.urow[w][lane] = make_float4(u0[R - 1][0], u0[R - 1][1], u0[R - 1][2], u0[R - 1][3]);
        lds_barrier();""", 1),
]
