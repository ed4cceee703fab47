# Variant: the tile (and band) kernels' fast iteration constants as VGPR operands.  tools/valu_probe2 measured
# any SGPR source at 4.24-4.30 SIMD cycles per wave-instruction at 4 waves per SIMD against 2.17 (VOP2) / 2.57
# (VOP3) with VGPR sources; vconst() copies a kernel constant into a VGPR once (non-volatile asm: CSE'd and hoisted).
PATCHES = [
    ("__device__ __forceinline__ float2 row_sum2(float a, float b) {",
     "__device__ __forceinline__ float vconst(float s) {\n    float v;\n    asm(\"v_mov_b32 %0, %1\" : \"=v\"(v) : \"s\"(s));\n    return v;\n}\n"
     "__device__ __forceinline__ float2 row_sum2(float a, float b) {", 1),
    ("xv = __builtin_fmaf(a.tau, yv[r][k] - tt, xo) * a.inv_opt;",
     "xv = __builtin_fmaf(vconst(a.tau), yv[r][k] - tt, xo) * vconst(a.inv_opt);", 1),
    ("                    xn = __builtin_fmaf(a.rho, xv - xo, xo);",
     "                    xn = __builtin_fmaf(vconst(a.rho), xv - xo, xo);", 2),
    ("const float sg0 = down ? a.sig_tv : 0.f;", "const float sg0 = down ? vconst(a.sig_tv) : 0.f;", 1),
    ("                    const float f = fminf(1.0f, a.ths * __builtin_amdgcn_rsqf(s2));",
     "                    const float f = fminf(1.0f, vconst(a.ths) * __builtin_amdgcn_rsqf(s2));", 2),
    ("                    u0[r][k] = __builtin_fmaf(a.rho, __builtin_fmaf(v0, f, -uo0), uo0);",
     "                    u0[r][k] = __builtin_fmaf(vconst(a.rho), __builtin_fmaf(v0, f, -uo0), uo0);", 2),
    ("                    u1[r][k] = __builtin_fmaf(a.rho, __builtin_fmaf(v1, f, -uo1), uo1);",
     "                    u1[r][k] = __builtin_fmaf(vconst(a.rho), __builtin_fmaf(v1, f, -uo1), uo1);", 2),
]
