#!/usr/bin/env python3
"""Generate tools/valu_probe2.hip: VALU issue cost by operand form on gfx950 (diagnostic, never in the product).

tools/valu_probe.hip measured the tile iteration's instruction mix at ~4.1 SIMD cycles per wave-instruction with 4
waves per SIMD, against ~2.1 for plain VOP2 adds: this probe splits that by operand form (VOP2 / VOP3, VGPR / SGPR /
inline-constant sources, VGPR bank of each source, operand reuse, dependence distance, DPP, transcendentals).

Every form is a straight-line block of 128 instructions (no branch inside), repeated ITERS times, run at 1 and 4
waves per SIMD (grid 256, one workgroup per CU); reported: the slowest wave's shader cycles per instruction (1 wave)
and per wave-instruction of the SIMD (4 waves: slowest wave's cycles / (instructions x 4)).

    python3 tools/valu_probe_gen.py && hipcc --offload-arch=gfx950 -O3 -o tools/valu_probe2 tools/valu_probe2.hip
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# 16 accumulators alternating banks 0 and 3 (bank = VGPR index mod 4)
ACC = [32, 35, 36, 39, 40, 43, 44, 47, 48, 51, 52, 55, 56, 59, 60, 63]
ACC0 = [32, 36, 40, 44, 48, 52, 56, 60]          # bank 0 only
# source registers: bank 1: v1 v5 v9 v13 v17 v21 v25 v29; bank 2: v2 v6 ... v30; bank 0: v4 v8 ...; bank 3: v3 v7 ...
B1 = [1, 5, 9, 13, 17, 21, 25, 29]
B2 = [2, 6, 10, 14, 18, 22, 26, 30]
B0 = [4, 8, 12, 16, 20, 24, 28]
B3 = [3, 7, 11, 15, 19, 23, 27, 31]


def blk(f):
    return [f(i) for i in range(16)]


FORMS = {
    # VOP2
    "add_vv":        blk(lambda i: f"v_add_f32 v{ACC[i]}, v1, v{ACC[i]}"),
    "add_sv":        blk(lambda i: f"v_add_f32 v{ACC[i]}, %1, v{ACC[i]}"),
    "add_cv":        blk(lambda i: f"v_add_f32 v{ACC[i]}, 1.0, v{ACC[i]}"),
    "add_vv_fresh":  blk(lambda i: f"v_add_f32 v{ACC[i]}, v{B1[i % 8]}, v{B2[i % 8]}"),
    "mul_sv":        blk(lambda i: f"v_mul_f32 v{ACC[i]}, %1, v{ACC[i]}"),
    "fmac_vv":       blk(lambda i: f"v_fmac_f32 v{ACC[i]}, v1, v2"),
    "fmac_vv_fresh": blk(lambda i: f"v_fmac_f32 v{ACC[i]}, v{B1[i % 8]}, v{B2[i % 8]}"),
    "fmac_sv":       blk(lambda i: f"v_fmac_f32 v{ACC[i]}, %1, v2"),
    "fmac_conf":     blk(lambda i: f"v_fmac_f32 v{ACC0[i % 8]}, v4, v2"),     # src0 and acc in bank 0
    "min_cv":        blk(lambda i: f"v_min_f32 v{ACC[i]}, 1.0, v{ACC[i]}"),
    "sub_vv_conf":   blk(lambda i: f"v_sub_f32 v{ACC[i]}, v1, v5"),           # both sources bank 1
    # VOP3
    "fma_vvv":       blk(lambda i: f"v_fma_f32 v{ACC[i]}, v1, v2, v{ACC[i]}"),
    "fma_vvv_fresh": blk(lambda i: f"v_fma_f32 v{ACC[i]}, v{B1[i % 8]}, v{B2[i % 8]}, v{ACC[i]}"),
    "fma_vvv_conf2": blk(lambda i: f"v_fma_f32 v{ACC[i]}, v1, v5, v{ACC[i]}"),   # src0, src1 bank 1
    "fma_vvv_confa": blk(lambda i: f"v_fma_f32 v{ACC0[i % 8]}, v4, v2, v{ACC0[i % 8]}"),  # src0, src2 bank 0
    "fma_vvv_conf3": blk(lambda i: f"v_fma_f32 v{ACC0[i % 8]}, v4, v8, v{ACC0[i % 8]}"),  # all bank 0
    "fma_svv":       blk(lambda i: f"v_fma_f32 v{ACC[i]}, %1, v2, v{ACC[i]}"),
    "fma_vsv":       blk(lambda i: f"v_fma_f32 v{ACC[i]}, v2, %1, v{ACC[i]}"),
    "fma_vvs":       blk(lambda i: f"v_fma_f32 v{ACC[i]}, v1, v2, %1"),
    "fma_cvv":       blk(lambda i: f"v_fma_f32 v{ACC[i]}, 2.0, v2, v{ACC[i]}"),
    "fma_svv_neg":   blk(lambda i: f"v_fma_f32 v{ACC[i]}, %1, v2, -v{ACC[i]}"),
    "add_vv_e64":    blk(lambda i: f"v_add_f32_e64 v{ACC[i]}, v1, v{ACC[i]}"),
    "add_vv_neg":    blk(lambda i: f"v_add_f32_e64 v{ACC[i]}, -v1, v{ACC[i]}"),
    "mul_sv_e64":    blk(lambda i: f"v_mul_f32_e64 v{ACC[i]}, %1, v{ACC[i]}"),
    # round 6, second pass: the forms a rewrite of the iteration loop would use
    "min_vv":        blk(lambda i: f"v_min_f32 v{ACC[i]}, v1, v{ACC[i]}"),
    "max_vv":        blk(lambda i: f"v_max_f32 v{ACC[i]}, v1, v{ACC[i]}"),
    "med3_vvv":      blk(lambda i: f"v_med3_f32 v{ACC[i]}, v1, v2, v{ACC[i]}"),
    "min3_vcv":      blk(lambda i: f"v_min3_f32 v{ACC[i]}, v1, 1.0, v{ACC[i]}"),
    "mul_vv":        blk(lambda i: f"v_mul_f32 v{ACC[i]}, v1, v{ACC[i]}"),
    "mul_cv":        blk(lambda i: f"v_mul_f32 v{ACC[i]}, 2.0, v{ACC[i]}"),
    "pk_fma_vvv":    blk(lambda i: f"v_pk_fma_f32 v[{ACC0[i % 8]}:{ACC0[i % 8] + 1}], v[2:3], v[6:7], v[{ACC0[i % 8]}:{ACC0[i % 8] + 1}]"),
    "pk_mul_vv":     blk(lambda i: f"v_pk_mul_f32 v[{ACC0[i % 8]}:{ACC0[i % 8] + 1}], v[2:3], v[{ACC0[i % 8]}:{ACC0[i % 8] + 1}]"),
    "pk_add_vv":     blk(lambda i: f"v_pk_add_f32 v[{ACC0[i % 8]}:{ACC0[i % 8] + 1}], v[2:3], v[{ACC0[i % 8]}:{ACC0[i % 8] + 1}]"),
    "cndmask_vv":    blk(lambda i: f"v_cndmask_b32 v{ACC[i]}, v1, v{ACC[i]}, vcc"),
    "add_dpp":       blk(lambda i: f"v_add_f32_dpp v{ACC[i]}, v1, v{ACC[i]} row_shr:1 row_mask:0xf bank_mask:0xf"),
    "fmac_kv":       blk(lambda i: f"v_fmac_f32 v{ACC[i]}, v{B1[i % 8]}, v{B2[i % 8]}"),
    "mix_vgpr":      [f"v_sub_f32 v{ACC[i]}, v{B1[i % 8]}, v{B2[i % 8]}" for i in range(6)] +
                     [f"v_fma_f32 v{ACC[6 + i]}, v{B1[i]}, v{B2[i]}, v{ACC[6 + i]}" for i in range(6)] +
                     [f"v_mul_f32 v{ACC[12 + i]}, v{B1[i]}, v{ACC[12 + i]}" for i in range(4)],
    # literal constants (VOP2 src0 literal, fmamk / fmaak) and selects
    "mul_lit":       blk(lambda i: f"v_mul_f32 v{ACC[i]}, 0x3e000000, v{ACC[i]}"),
    "fmac_lit":      blk(lambda i: f"v_fmac_f32 v{ACC[i]}, 0x3e000000, v2"),
    "fmamk":         blk(lambda i: f"v_fmamk_f32 v{ACC[i]}, v1, 0x3e000000, v{ACC[i]}"),
    "fmaak":         blk(lambda i: f"v_fmaak_f32 v{ACC[i]}, v1, v{ACC[i]}, 0x3e000000"),
    "fmamk_conf":    blk(lambda i: f"v_fmamk_f32 v{ACC0[i % 8]}, v4, 0x3e000000, v{ACC0[i % 8]}"),
    "cndmask_s":     ["s_mov_b64 s[40:41], exec"] + blk(lambda i: f"v_cndmask_b32_e64 v{ACC[i]}, v1, v{ACC[i]}, s[40:41]")[:15],
    "cndmask_vcc":   ["s_mov_b64 vcc, exec"] + blk(lambda i: f"v_cndmask_b32 v{ACC[i]}, v1, v{ACC[i]}, vcc")[:15],
    "cmp_cnd_vcc":   [x for j in range(4) for x in (f"v_cmp_gt_f32 vcc, v{ACC[4 * j]}, v1",
                                                    f"v_cndmask_b32 v{ACC[4 * j + 1]}, v1, v2, vcc",
                                                    f"v_cndmask_b32 v{ACC[4 * j + 2]}, v2, v1, vcc",
                                                    f"v_cndmask_b32 v{ACC[4 * j + 3]}, v1, v{ACC[4 * j + 3]}, vcc")],
    "cmp_cnd_s":     [x for j in range(4) for x in (f"v_cmp_gt_f32_e64 s[40:41], v{ACC[4 * j]}, v1",
                                                    f"v_cndmask_b32_e64 v{ACC[4 * j + 1]}, v1, v2, s[40:41]",
                                                    f"v_cndmask_b32_e64 v{ACC[4 * j + 2]}, v2, v1, s[40:41]",
                                                    f"v_cndmask_b32_e64 v{ACC[4 * j + 3]}, v1, v{ACC[4 * j + 3]}, s[40:41]")],
    "cnd_vcc_after_cmp": ["v_cmp_gt_f32 vcc, v1, v2"] + blk(lambda i: f"v_cndmask_b32 v{ACC[i]}, v1, v{ACC[i]}, vcc")[:15],
    # one compare + one select among 14 independent adds: the marginal price of a select reading VCC (e32) or an
    # SGPR pair (e64), against the same block with an add in the select's place
    "mix_cnd_vcc":   ["v_cmp_gt_f32 vcc, v1, v2"] + [f"v_add_f32 v{ACC[i]}, v1, v{ACC[i]}" for i in range(7)] +
                     ["v_cndmask_b32 v5, v1, v2, vcc"] + [f"v_add_f32 v{ACC[i]}, v1, v{ACC[i]}" for i in range(7, 14)],
    "mix_cnd_s":     ["v_cmp_gt_f32_e64 s[40:41], v1, v2"] + [f"v_add_f32 v{ACC[i]}, v1, v{ACC[i]}" for i in range(7)] +
                     ["v_cndmask_b32_e64 v5, v1, v2, s[40:41]"] + [f"v_add_f32 v{ACC[i]}, v1, v{ACC[i]}" for i in range(7, 14)],
    "mix_add":       ["v_cmp_gt_f32 vcc, v1, v2"] + [f"v_add_f32 v{ACC[i]}, v1, v{ACC[i]}" for i in range(7)] +
                     ["v_add_f32 v5, v1, v2"] + [f"v_add_f32 v{ACC[i]}, v1, v{ACC[i]}" for i in range(7, 14)],
    "mix_nocmp":     [f"v_add_f32 v{ACC[i]}, v1, v{ACC[i]}" for i in range(16)],
    # integer forms of the Philox rounds (round 6): 32x32 -> 64 multiply-add, high half, xors with an SGPR key
    "mad_u64_vv":    [f"v_mad_u64_u32 v[{ACC0[i % 8]}:{ACC0[i % 8] + 1}], s[42:43], v{B1[i % 8]}, v2, 0" for i in range(16)],
    "mad_u64_sv":    [f"v_mad_u64_u32 v[{ACC0[i % 8]}:{ACC0[i % 8] + 1}], s[42:43], %1, v{B1[i % 8]}, 0" for i in range(16)],
    "mul_hi_vv":     blk(lambda i: f"v_mul_hi_u32 v{ACC[i]}, v{B1[i % 8]}, v2"),
    "mul_hi_sv":     blk(lambda i: f"v_mul_hi_u32 v{ACC[i]}, %1, v{B1[i % 8]}"),
    "mul_lo_vv":     blk(lambda i: f"v_mul_lo_u32 v{ACC[i]}, v{B1[i % 8]}, v2"),
    "xor_vv":        blk(lambda i: f"v_xor_b32 v{ACC[i]}, v1, v{ACC[i]}"),
    "xor_sv":        blk(lambda i: f"v_xor_b32 v{ACC[i]}, %1, v{ACC[i]}"),
    "sqrt":          blk(lambda i: f"v_sqrt_f32 v{ACC[i]}, v1"),
    "cvt_f32_u32":   blk(lambda i: f"v_cvt_f32_u32 v{ACC[i]}, v{B1[i % 8]}"),
    # transcendental and data movement
    "rsq":           blk(lambda i: f"v_rsq_f32 v{ACC[i]}, v1"),
    "mov_dpp":       blk(lambda i: f"v_mov_b32_dpp v{ACC[i]}, v1 row_shr:1 row_mask:0xf bank_mask:0xf"),
    "mov_wshr":      blk(lambda i: f"v_mov_b32_dpp v{ACC[i]}, v1 wave_shr:1 row_mask:0xf bank_mask:0xf"),
    # dependence: chains of 4 / 2 / 1 accumulators
    "add_dep4":      blk(lambda i: f"v_add_f32 v{ACC[i % 4]}, v1, v{ACC[i % 4]}"),
    "add_dep2":      blk(lambda i: f"v_add_f32 v{ACC[i % 2]}, v1, v{ACC[i % 2]}"),
    "add_dep1":      blk(lambda i: f"v_add_f32 v32, v1, v32"),
    "fma_dep4":      blk(lambda i: f"v_fma_f32 v{ACC[i % 4]}, v1, v2, v{ACC[i % 4]}"),
    "rsq_use4":      [x for j in range(8) for x in (f"v_rsq_f32 v{ACC[2 * j]}, v1",
                                                    f"v_add_f32 v{ACC[(2 * j + 7) % 16]}, v{ACC[(2 * j - 6) % 16]}, v2")],
}


def hip_src():
    clob = ", ".join(f'"v{r}"' for r in range(1, 64)) + ', "s40", "s41", "s42", "s43", "vcc"' 
    init = " ".join(f"v_mov_b32 v{r}, 0.5\\n" for r in range(1, 64))
    out = ['// generated by tools/valu_probe_gen.py -- VALU issue cost by operand form (diagnostic)',
           '#include <hip/hip_runtime.h>', '#include <cstdio>', '#include <cstdlib>', '#include <vector>', '']
    for name, body in FORMS.items():
        asm = "\\n".join(body * 8) + "\\n"
        out.append(f'__global__ __launch_bounds__(1024) void probe_{name}(unsigned long long* out, int iters, float s) {{')
        out.append(f'    asm volatile("{init}" ::: {clob});')
        out.append('    const unsigned long long t0 = __builtin_amdgcn_s_memtime();')
        out.append('    for (int i = 0; i < iters; ++i) {')
        out.append(f'        asm volatile("{asm}" : "+s"(i) : "s"(s) : {clob});')
        out.append('    }')
        out.append('    const unsigned long long t1 = __builtin_amdgcn_s_memtime();')
        out.append('    if ((threadIdx.x & 63) == 0) out[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0;')
        out.append('}')
    out.append(r'''
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)
template <typename K>
static void run(const char* name, K kern, unsigned long long* d_out) {
    const int grid = 256, iters = 400, ninst = 128;
    double r[2];
    int k = 0;
    for (int wps : {1, 4}) {
        const int threads = 256 * wps, waves = grid * threads / 64;
        hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), 0, 0, d_out, iters, 0.5f);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), 0, 0, d_out, iters, 0.5f);
        CHECK(hipDeviceSynchronize());
        std::vector<unsigned long long> h(waves);
        CHECK(hipMemcpy(h.data(), d_out, h.size() * 8, hipMemcpyDeviceToHost));
        double mx = 0;
        for (int w = 0; w < waves; ++w) mx = h[w] > mx ? (double)h[w] : mx;
        r[k++] = mx / ((double)ninst * iters * wps);
    }
    printf("%-14s 1 wave: %5.2f cyc/inst | 4 waves/SIMD: %5.2f SIMD cyc per wave-inst\n", name, r[0], r[1]);
}
int main() {
    unsigned long long* d_out;
    CHECK(hipMalloc(&d_out, 256 * 16 * 8));''')
    for name in FORMS:
        out.append(f'    run("{name}", probe_{name}, d_out);')
    out.append('    CHECK(hipFree(d_out));\n    return 0;\n}')
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    open(os.path.join(HERE, "valu_probe2.hip"), "w").write(hip_src())
