# Variant: the no-stop finaliser path waits for its zeroing stores (vmcnt 0) before the resets.
PATCHES = [("""        if (a.par_redo && threadIdx.x == 0) {
            a.redo[1] = 0;
            a.redo[0] = 0;
        }
    } else {""", """        if (a.par_redo && threadIdx.x == 0) {
            a.redo[1] = 0;
            a.redo[0] = 0;
        }
        wait_vm0();
    } else {""", 1)]
