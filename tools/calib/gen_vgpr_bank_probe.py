#!/usr/bin/env python3
"""Generate vgpr_bank_probe.hip: does the VGPR bank of a VALU instruction's sources set its
issue rate on gfx950?

The tile stencil's v_bitop3 stream issues at 2.5-2.7 SIMD cycles per instruction at 4-8 waves
per SIMD (stencil_issue.hip) against the 2-cycle wave64 floor.  A candidate cause is operand
reads: three source VGPRs in one bank.  Each kernel here runs a loop of 128 independent VALU
instructions (destinations v48..v63, never read; sources v0..v47, never written in the loop)
on hand-numbered registers -- one kernel per source-bank pattern -- with W waves per SIMD
resident (LDS per workgroup forces the occupancy, as in stencil_issue.hip).  Each wave's
s_memtime span over its loop gives
    SIMD cycles per instruction = median wave cycles / (W x instructions per wave).
Usage: python3 gen_vgpr_bank_probe.py > vgpr_bank_probe.hip
       hipcc --offload-arch=gfx950 -O3 -o vgpr_bank_probe vgpr_bank_probe.hip
"""
import os


def pattern(v, i):
    d = 48 + i % 16
    k = (i % 10) * 4                     # base register: bank 0 if banks are (index mod 4)
    A, B = 48 + (2 * i) % 16, 49 + (2 * i) % 16          # rotating DPP destinations
    b3 = "v_bitop3_b32 v%d, v%d, v%d, v%d bitop3:0x96"
    return {
        0: b3 % (d, k, k + 1, k + 2),
        1: b3 % (d, k, k + 4, k + 8),
        2: b3 % (d, k, k + 4, k + 1),
        3: b3 % (d, k, k + 2, k + 6),
        4: b3 % (d, k, k, k),
        5: "v_xor_b32 v%d, v%d, v%d" % (d, k, k + 1),
        6: "v_xor_b32 v%d, v%d, v%d" % (d, k, k + 4),
        7: "v_mov_b32 v%d, v%d" % (d, k),
        8: "v_alignbit_b32 v%d, v%d, v%d, 31" % (d, k, k + 1),
        9: "v_mov_b32_dpp v%d, v%d row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0" % (d, k),
        10: b3 % (48 + (i % 4) * 4, k, k + 1, k + 2),
        11: b3 % (d, k + 1, k + 2, k + 3),
        12: "v_add3_u32 v%d, v%d, v%d, v%d" % (d, k, k + 1, k + 2),
        13: "v_add3_u32 v%d, v%d, v%d, v%d" % (d, k, k + 4, k + 8),
        14: b3 % (d, k, k + 1, k + 5),
        15: b3 % (d, k, k + 3, k + 2),
        16: "v_or_b32_dpp v%d, v%d, v%d wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" % (d, k, k + 1),
        17: "v_add_u32_dpp v%d, v%d, v%d row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" % (d, k, k + 1),
        18: "v_addc_co_u32_e32 v%d, vcc, v%d, v%d, vcc" % (d, k, k + 1),
        19: "v_addc_co_u32_e64 v%d, s[42:43], v%d, v%d, s[44:45]" % (d, k, k + 1),
        20: "v_cmp_gt_i32_e32 vcc, 0, v%d" % (k,),
        21: "v_lshl_or_b32 v%d, v%d, 1, v%d" % (d, k, k + 1),
        22: "v_lshrrev_b32 v%d, 31, v%d" % (d, k),
        23: "v_cndmask_b32_e32 v%d, v%d, v%d, vcc" % (d, k, k + 1),
        24: "v_bfi_b32 v%d, v%d, v%d, v%d" % (d, k, k + 1, k + 2),
        25: "v_bitop3_b32 v%d, v%d, v%d, s44 bitop3:0x96" % (d, k, k + 1),
        26: "v_bitop3_b32 v%d, v%d, v%d, s44 bitop3:0x96" % (d, k, k + 2),
        27: "v_alignbit_b32 v%d, v%d, v%d, 1" % (d, k, k),
        28: "v_alignbyte_b32 v%d, v%d, v%d, 1" % (d, k, k + 1),
        29: "v_cmp_ne_u32_e64 s[42:43], 0, v%d" % (k,),
        30: ("v_cmp_gt_i32_e32 vcc, 0, v%d|s_lshl_b64 vcc, vcc, 1|v_addc_co_u32_e32 v%d, vcc, v%d, v%d, vcc" % (k, d, k, k)) if i % 2 == 0 else b3 % (d, k, k + 1, k + 2),
        31: ("v_mov_b32_dpp v%d, v%d wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" % (d, k)) if i % 4 == 0 else b3 % (d, k, k + 1, k + 2),
        32: "v_mov_b32_dpp v%d, v%d wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" % (d, k),
        33: "v_xor_b32_sdwa v%d, v%d, v%d dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD" % (d, k, k + 1),
        # the stencil's lane-shift pairs (4 instructions per slot): DPP A, DPP B, then each
        # v_alignbit reading its DPP result -- 2 instructions later (the generated ORD 8 turn),
        # right after (the compiler's ORD 5), or 4 later with two bitop3 between
        34: "|".join(["v_mov_b32_dpp v%d, v%d wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" % (A, k + 1),
                      "v_mov_b32_dpp v%d, v%d wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" % (B, k),
                      "v_alignbit_b32 v%d, v%d, v%d, 31" % (A, k + 1, A),
                      "v_alignbit_b32 v%d, v%d, v%d, 1" % (B, B, k)]),
        35: "|".join(["v_mov_b32_dpp v%d, v%d wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" % (A, k + 1),
                      "v_alignbit_b32 v%d, v%d, v%d, 31" % (A, k + 1, A),
                      "v_mov_b32_dpp v%d, v%d wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" % (B, k),
                      "v_alignbit_b32 v%d, v%d, v%d, 1" % (B, B, k)]),
        36: "|".join(["v_mov_b32_dpp v%d, v%d wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" % (A, k + 1),
                      "v_mov_b32_dpp v%d, v%d wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" % (B, k),
                      b3 % (d, k, k + 1, k + 2), b3 % (d + 1 if d < 63 else 48, k + 1, k + 2, k + 3),
                      "v_alignbit_b32 v%d, v%d, v%d, 31" % (A, k + 1, A),
                      "v_alignbit_b32 v%d, v%d, v%d, 1" % (B, B, k)]),
        # the same DPP pairs with fixed destinations (ORD 8 uses one register pair for every row)
        # 6 half-rate (3 DPP, 3 v_alignbit) and 18 full-rate v_bitop3 per 24 slots: grouped
        # (the half-rate ones first) or spread (one every 4 slots)
        38: (["v_mov_b32_dpp v%d, v%d wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" % (A, k + 1),
              "v_alignbit_b32 v%d, v%d, v%d, 31" % (B, k + 1, k)][i % 2] if i % 24 < 6
             else b3 % (d, k, k + 1, k + 2)),
        39: (["v_mov_b32_dpp v%d, v%d wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" % (A, k + 1),
              "v_alignbit_b32 v%d, v%d, v%d, 31" % (B, k + 1, k)][(i // 4) % 2] if i % 4 == 0
             else b3 % (d, k, k + 1, k + 2)),
        # 2 half-rate per 24 (one DPP, one v_alignbit), grouped or spread
        40: (["v_mov_b32_dpp v%d, v%d wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" % (A, k + 1),
              "v_alignbit_b32 v%d, v%d, v%d, 31" % (B, k + 1, k)][i % 2] if i % 24 < 2
             else b3 % (d, k, k + 1, k + 2)),
        41: (["v_mov_b32_dpp v%d, v%d wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" % (A, k + 1),
              "v_alignbit_b32 v%d, v%d, v%d, 31" % (B, k + 1, k)][(i // 12) % 2] if i % 12 == 0
             else b3 % (d, k, k + 1, k + 2)),
        37: "|".join(["v_mov_b32_dpp v56, v%d wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" % (k + 1),
                      "v_mov_b32_dpp v61, v%d wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" % k,
                      "v_alignbit_b32 v56, v%d, v56, 31" % (k + 1),
                      "v_alignbit_b32 v61, v61, v%d, 1" % k]),
    }[v]


NAMES = [
    "bitop3 banks 0,1,2", "bitop3 banks 0,0,0", "bitop3 banks 0,0,1", "bitop3 banks 0,2,2",
    "bitop3 one register x3", "xor (VOP2) banks 0,1", "xor (VOP2) banks 0,0", "v_mov",
    "alignbit banks 0,1", "DPP mov", "bitop3 banks 0,1,2 dst bank 0", "bitop3 banks 1,2,3",
    "add3 banks 0,1,2", "add3 banks 0,0,0", "bitop3 banks 0,1,1", "bitop3 banks 0,3,2",
    "v_or_b32_dpp wave_shr", "v_add_u32_dpp row_shr", "v_addc_co_u32_e32 (vcc)", "v_addc_co_u32_e64 (sgpr pair)",
    "v_cmp_gt_i32_e32 vcc", "v_lshl_or_b32", "v_lshrrev_b32", "v_cndmask_b32_e32", "v_bfi_b32",
    "bitop3 2 vgpr (banks 0,1) + sgpr", "bitop3 2 vgpr (banks 0,0) + sgpr", "alignbit same reg",
    "v_alignbyte_b32", "v_cmp_ne_u32_e64 sgpr pair", "carry west shift (cmp, s_lshl, addc) / bitop3 alt",
    "1 DPP mov per 4 (3 bitop3)", "v_mov_b32_dpp wave_shr", "v_xor_b32_sdwa",
    "DPP,DPP,align(2 later),align (ORD 8 order)", "DPP,align,DPP,align (compiler order)",
    "DPP,DPP,2 bitop3,align,align", "DPP pairs, fixed dst v56/v61 (ORD 8 registers)",
    "6 half-rate grouped + 18 bitop3 (per 24)", "6 half-rate spread 1-in-4 + 18 bitop3",
    "2 half-rate grouped + 22 bitop3 (per 24)", "2 half-rate spread 1-in-12 + 22 bitop3",
]
ONLY = [int(x) for x in os.environ.get("PROBE_ONLY", "").split(",") if x]
NV = len(NAMES)
NI = 128

out = []
out.append("// GENERATED by gen_vgpr_bank_probe.py -- do not edit\n")
out.append("#include <hip/hip_runtime.h>\n#include <algorithm>\n#include <cstdio>\n#include <vector>\n#include <map>\n#include <array>\n")
clob = ", ".join('"v%d"' % r for r in range(64)) + ', "s40", "s42", "s43", "s44", "s45", "vcc", "scc"'
for v in range(NV):
    body = "".join('        "%s\\n"\n' % ins for i in range(NI) for ins in pattern(v, i).split("|"))
    init = "".join('        "v_add_u32 v%d, %d, %%[seed]\\n"\n' % (r, r * 7 + 1) for r in range(48))
    init += "".join('        "v_mov_b32 v%d, 0\\n"\n' % r for r in range(48, 64))
    out.append("""
__global__ __launch_bounds__(1024) void k_probe%d(unsigned *out, unsigned long long *clk, int iters)
{
    extern __shared__ unsigned pad[];
    const unsigned seed = blockIdx.x * 0x9e3779b9u + threadIdx.x;
    unsigned res;
    unsigned long long t0, t1;
    unsigned hw, xcc;
    if (threadIdx.x == 0) pad[0] = seed;
    asm volatile("s_getreg_b32 %%0, hwreg(HW_REG_HW_ID)\\n s_getreg_b32 %%1, hwreg(HW_REG_XCC_ID)" : "=s"(hw), "=s"(xcc));
    asm volatile(
%s        "s_mov_b32 s40, %%[n]\\n"
        "s_mov_b64 s[42:43], 0\\n"
        "s_mov_b64 s[44:45], 0\\n"
        "s_mov_b64 vcc, 0\\n"
        "s_memtime %%[t0]\\n"
        "s_waitcnt lgkmcnt(0)\\n"
        "1:\\n"
%s        "s_sub_u32 s40, s40, 1\\n"
        "s_cmp_lg_u32 s40, 0\\n"
        "s_cbranch_scc1 1b\\n"
        "s_memtime %%[t1]\\n"
        "s_waitcnt lgkmcnt(0)\\n"
        "v_bitop3_b32 %%[res], v48, v55, v63 bitop3:0x96\\n"
        : [res] "=v"(res), [t0] "=&s"(t0), [t1] "=&s"(t1)
        : [seed] "v"(seed), [n] "s"(iters)
        : %s);
    out[blockIdx.x * blockDim.x + threadIdx.x] = res ^ (pad[0] & 0u);
    if ((threadIdx.x & 63) == 0) {
        const int w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        clk[3 * w] = t0;
        clk[3 * w + 1] = t1;
        clk[3 * w + 2] = ((unsigned long long)xcc << 32) | hw;
    }
}
""" % (v, init, body, clob))

out.append("static void *kFn[] = {%s};\n" % ", ".join("(void *)&k_probe%d" % v for v in range(NV)))
out.append("static const char *kName[] = {%s};\n" % ", ".join('"%s"' % n for n in NAMES))
RUN = ONLY or list(range(NV))
out.append("static const int kRun[] = {%s};\n" % ", ".join(str(v) for v in RUN))
out.append("""
int main(int argc, char **argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    for (int v : kRun) {
        for (int W : {1, 2, 3, 4, 6, 8}) {
            // W waves per SIMD: workgroups of 4 x min(W, 4) waves, LDS so that W / 4 of them
            // (or one) fit a CU; the per-SIMD spans below show what was co-resident
            const int wg_waves = 4 * (W < 4 ? W : 4), per_cu = W <= 4 ? 1 : W / 4;
            const int threads = 64 * wg_waves, blocks = ncu * per_cu;
            const size_t lds = (size_t)160 * 1024 / per_cu - 1024;
            unsigned *d_out;
            unsigned long long *d_clk;
            (void)hipMalloc(&d_out, (size_t)blocks * threads * 4);
            (void)hipMalloc(&d_clk, (size_t)blocks * wg_waves * 3 * 8);
            void *args[3];
            int it = iters;
            args[0] = &d_out;
            args[1] = &d_clk;
            args[2] = &it;
            for (int rep = 0; rep < 2; ++rep)
                if (hipLaunchKernel(kFn[v], dim3(blocks), dim3(threads), args, lds, 0) != hipSuccess) { printf("launch error\\n"); return 1; }
            if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\\n"); return 1; }
            const int nw = blocks * wg_waves;
            std::vector<unsigned long long> h((size_t)nw * 3);
            (void)hipMemcpy(h.data(), d_clk, h.size() * 8, hipMemcpyDeviceToHost);
            // per SIMD (xcc, se, cu, simd from HW_ID): waves, first start, last end
            std::map<unsigned long long, std::array<unsigned long long, 3>> simd;
            std::vector<double> span;
            for (int w = 0; w < nw; ++w) {
                const unsigned long long id = h[3 * w + 2];
                const unsigned hwid = (unsigned)id;
                // (HW_ID: SIMD_ID [5:4], CU_ID [11:8], SH_ID [12], SE_ID [15:13]; plus the XCC)
                const unsigned long long key = ((id >> 32) << 32) | (hwid & 0xff30u);
                auto it = simd.find(key);
                if (it == simd.end()) simd[key] = {1, h[3 * w], h[3 * w + 1]};
                else {
                    it->second[0] += 1;
                    it->second[1] = std::min(it->second[1], h[3 * w]);
                    it->second[2] = std::max(it->second[2], h[3 * w + 1]);
                }
                span.push_back((double)(h[3 * w + 1] - h[3 * w]));
            }
            std::vector<double> cyc, nws;
            for (auto &kv : simd) {
                cyc.push_back((double)(kv.second[2] - kv.second[1]) / ((double)kv.second[0] * iters * %d));
                nws.push_back((double)kv.second[0]);
            }
            std::sort(cyc.begin(), cyc.end());
            std::sort(nws.begin(), nws.end());
            std::sort(span.begin(), span.end());
            printf("{\\"variant\\": \\"%%s\\", \\"waves_per_simd\\": %%d, \\"simds\\": %%zu, \\"waves_on_simd_min_max\\": [%%g, %%g], "
                   "\\"wave_cycles_per_inst\\": %%.3f, \\"simd_cycles_per_inst\\": %%.3f}\\n", kName[v], W, simd.size(), nws.front(), nws.back(),
                   span[span.size() / 2] / ((double)iters * %d), cyc[cyc.size() / 2]);
            (void)hipFree(d_out);
            (void)hipFree(d_clk);
        }
    }
    return 0;
}
""" % (NI, NI))
print("".join(out))
