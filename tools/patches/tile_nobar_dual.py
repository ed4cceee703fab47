# timing-only (wrong results): the tile kernel without the barrier after the dual
PATCHES = [("""        if (act_d) sh.urow[w][lane] = make_float4(u0[R - 1][0], u0[R - 1][1], u0[R - 1][2], u0[R - 1][3]);
        __syncthreads();""", """        if (act_d) sh.urow[w][lane] = make_float4(u0[R - 1][0], u0[R - 1][1], u0[R - 1][2], u0[R - 1][3]);""", 1)]
