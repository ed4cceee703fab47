# timing-only (wrong results): the tile kernel without the barrier between primal and dual
PATCHES = [("""            if ((lane & 15) == 0) sh.red[it][w][lane >> 4] = rs;
        }
        __syncthreads();""", """            if ((lane & 15) == 0) sh.red[it][w][lane >> 4] = rs;
        }""", 1)]
