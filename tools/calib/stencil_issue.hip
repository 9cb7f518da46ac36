// stencil_issue.hip -- the VALU issue roof of the tile stencil (K1t), measured with the
// stencil's own instruction stream at 4, 6 and 8 resident waves per SIMD.
//
// Each wave keeps SEG rows x 2 dwords (interleaved layout, 64 cells per lane) in registers and
// runs `turns` turns of K1t's turn body -- per row the 3-cell row sums (2 DPP moves, 2
// v_alignbit, 4 v_bitop3) and the 7-op rule (14 v_bitop3), built from the same device
// functions as the product kernel (gol_device.h) -- with the segment's rows wrapped onto
// themselves (no LDS exchange, no barrier, no memory inside the loop).  So the loop is exactly
// the stencil's 22 VALU per row with its real dependency chains.
//
// Occupancy is forced, not hoped for: every workgroup is 4 waves (one per SIMD) and takes
// 160 KiB / W of LDS, so exactly W workgroups fit a CU; the grid is CUs x W workgroups, so all
// waves are resident at once for the whole kernel.  The kernel's duration (HIP events; the
// same launches under rocprofv3 --kernel-trace give the trace durations) and the shader clock
// (each wave's s_memtime / s_memrealtime over its loop) give
//   SIMD cycles per VALU instruction = duration x clock / (W x VALU per wave),
// with VALU per wave = turns x SEG x 22 (checked against SQ_INSTS_VALU in a --pmc pass).
// Variants: MIX 0 = the stencil's stream; 1 = the same with the DPP moves and v_alignbit
// replaced by full-rate v_xor / v_lshlrev (what the half-rate instructions cost); 2 = v_bitop3
// only (the floor of the mix's dominant instruction).
// Build: hipcc --offload-arch=gfx950 -O3 -I../../conway-s-gol-distributed_amd/csrc \
//        -I../../include -o stencil_issue stencil_issue.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "gol_device.h"

using namespace golk;

template <int MIX>
__device__ __forceinline__ void rsum(const uint32_t (&x)[2], uint32_t (&s)[4])
{
    const uint32_t e = x[0], o = x[1];
    uint32_t wl, er;
    if constexpr (MIX == 0) {
        const uint32_t L = dpp_from_lower_z(o);          // west lane's odd cells
        const uint32_t R = dpp_from_upper_z(e);          // east lane's even cells
        wl = __builtin_amdgcn_alignbit(o, L, 31);
        er = __builtin_amdgcn_alignbit(R, e, 1);
    } else if constexpr (MIX == 1) {
        // full-rate VOP2 stand-ins, one for each DPP move and v_alignbit (asm: the compiler
        // must neither fold them into the row sums nor fuse them into 3-input ops)
        uint32_t L, R;
        asm("v_lshlrev_b32 %0, 1, %1" : "=v"(L) : "v"(o));
        asm("v_lshrrev_b32 %0, 1, %1" : "=v"(R) : "v"(e));
        asm("v_xor_b32 %0, %1, %2" : "=v"(wl) : "v"(L), "v"(o));
        asm("v_xor_b32 %0, %1, %2" : "=v"(er) : "v"(R), "v"(e));
    } else if constexpr (MIX == 3) {
        // the west funnel shift without DPP / v_alignbit: the sign bits of the odd dwords as
        // a lane mask (one VOPC compare), shifted up one lane on the scalar unit, and added
        // in as the carry of o + o (v_addc_co_u32, VOP3 form with the mask as carry-in):
        // wl = (o << 1) | (west lane's o >> 31); the east shift stays DPP + v_alignbit
        const uint64_t m = __builtin_amdgcn_ballot_w64((int)o < 0) << 1;
        uint64_t co;
        asm("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(wl), "=&s"(co) : "v"(o), "s"(m));
        const uint32_t R = dpp_from_upper_z(e);
        er = __builtin_amdgcn_alignbit(R, e, 1);
    } else {                                             // v_bitop3 stand-ins
        uint32_t L, R;
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x6a" : "=v"(L) : "v"(o), "v"(e), "v"(o));
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x6a" : "=v"(R) : "v"(e), "v"(o), "v"(e));
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x1e" : "=v"(wl) : "v"(L), "v"(o), "v"(e));
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x1e" : "=v"(er) : "v"(R), "v"(e), "v"(o));
    }
    s[0] = xor3(wl, e, o);
    s[1] = maj(wl, e, o);
    s[2] = xor3(e, o, er);
    s[3] = maj(e, o, er);
}

__device__ __forceinline__ void rule(const uint32_t (&A)[4], const uint32_t (&B)[4],
                                     const uint32_t (&C)[4], uint32_t (&x)[2])
{
    const uint32_t n0 = life_rule7(A[0], B[0], C[0], A[1], B[1], C[1], x[0]);
    const uint32_t n1 = life_rule7(A[2], B[2], C[2], A[3], B[3], C[3], x[1]);
    x[0] = n0;
    x[1] = n1;
}

template <int SEG, int MIX>
__global__ __launch_bounds__(256, (SEG <= 16 ? 8 : 6)) void k_mix(uint32_t *out, unsigned long long *clk, int turns)
{
    extern __shared__ uint32_t pad[];                    // (occupancy: LDS per workgroup)
    uint32_t v[SEG][2];
    const uint32_t seed = blockIdx.x * 0x9e3779b9u + threadIdx.x * 0x85ebca6bu;
#pragma unroll
    for (int i = 0; i < SEG; ++i) {
        v[i][0] = seed * (2u * i + 1u) ^ 0x5bd1e995u;
        v[i][1] = (seed + 0x27d4eb2fu * i) * 0x165667b1u;
    }
    if (threadIdx.x == 0) pad[0] = seed;                 // (keep the allocation)
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int t = 0; t < turns; ++t) {
        // exactly SEG row sums and SEG rules per turn: rows 0 and SEG-1's sums are taken
        // before any row changes and reused at the wrap
        uint32_t first[4], last[4], P[4], Q[4];
        rsum<MIX>(v[SEG - 1], last);
        rsum<MIX>(v[0], first);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            P[k] = last[k];
            Q[k] = first[k];
        }
#pragma unroll
        for (int i = 0; i < SEG; ++i) {
            uint32_t R[4];
            if (i + 2 < SEG) rsum<MIX>(v[i + 1], R);
            else if (i + 2 == SEG)
#pragma unroll
                for (int k = 0; k < 4; ++k) R[k] = last[k];
            else
#pragma unroll
                for (int k = 0; k < 4; ++k) R[k] = first[k];
            rule(P, Q, R, v[i]);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                P[k] = Q[k];
                Q[k] = R[k];
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = pad[0] & 0u;
#pragma unroll
    for (int i = 0; i < SEG; ++i) acc ^= v[i][0] ^ v[i][1];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) {
        const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
        clk[2 * w] = t1 - t0;
        clk[2 * w + 1] = r1 - r0;
    }
}

static const char *kMix[] = {"stencil (22 VALU per row: 18 v_bitop3, 2 DPP, 2 v_alignbit)",
                             "DPP / v_alignbit -> v_xor / v_lshlrev (full-rate stand-ins)",
                             "v_bitop3 only",
                             "west shift by lane-mask carry (v_cmp + s_lshl + v_addc)"};

template <int SEG, int MIX>
static void run(int W, int turns, int ncu, int reps)
{
    auto fn = k_mix<SEG, MIX>;
    const int blocks = ncu * W;
    const size_t lds = (size_t)160 * 1024 / W - 1024;    // exactly W workgroups per CU
    int per_cu = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, lds);
    hipFuncAttributes attr;
    (void)hipFuncGetAttributes(&attr, reinterpret_cast<const void *>(fn));
    uint32_t *d_out;
    unsigned long long *d_clk;
    (void)hipMalloc(&d_out, (size_t)blocks * 256 * 4);
    (void)hipMalloc(&d_clk, (size_t)blocks * 4 * 2 * 8);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), lds, 0, d_out, d_clk, turns);   // warm
    float best = 0.f;
    for (int r = 0; r < reps; ++r) {
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), lds, 0, d_out, d_clk, turns);
        (void)hipEventRecord(e1, 0);
        if (hipEventSynchronize(e1) != hipSuccess) { std::printf("launch failed\n"); std::exit(1); }
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (best == 0.f || ms < best) best = ms;
    }
    std::vector<unsigned long long> h((size_t)blocks * 8);
    (void)hipMemcpy(h.data(), d_clk, h.size() * 8, hipMemcpyDeviceToHost);
    std::vector<double> ghz;
    for (int w = 0; w < blocks * 4; ++w) ghz.push_back((double)h[2 * w] / (double)h[2 * w + 1] * 0.1);
    std::sort(ghz.begin(), ghz.end());
    const double clock = ghz[ghz.size() / 2];
    const double valu_per_wave = (double)turns * SEG * 22.0;
    const double cyc = best * 1e-3 * clock * 1e9 / ((double)W * valu_per_wave);
    // the GCUPS this issue rate gives a stencil with no halo / sync overhead at this clock and
    // at 2.4 GHz: 4096 cell-updates per 22 VALU per SIMD
    const double simds = ncu * 4.0;
    const double gcups = simds * clock * 1e9 / (cyc * 22.0) * 4096.0 / 1e9;
    std::printf("{\"mix\": \"%s\", \"seg\": %d, \"waves_per_simd\": %d, \"occupancy_api_wg_per_cu\": "
                "%d, \"vgprs\": %d, \"turns\": %d, \"kernel_ms\": %.4f, \"clock_ghz\": %.3f, "
                "\"simd_cycles_per_valu\": %.4f, \"cycles_per_4096_cell_updates\": %.2f, "
                "\"gcups_no_overhead\": %.0f, \"gcups_no_overhead_at_2p4\": %.0f}\n",
                kMix[MIX], SEG, W, per_cu, attr.numRegs, turns, best, clock, cyc, cyc * 22.0, gcups,
                gcups * 2.4 / clock);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(d_out);
    (void)hipFree(d_clk);
}

int main(int argc, char **argv)
{
    const int turns = argc > 1 ? std::atoi(argv[1]) : 4000;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    for (int W : {4, 6, 8}) run<16, 0>(W, turns, ncu, reps);
    for (int W : {4, 6, 8}) run<16, 1>(W, turns, ncu, reps);
    for (int W : {4, 6, 8}) run<16, 2>(W, turns, ncu, reps);
    for (int W : {4, 6, 8}) run<16, 3>(W, turns, ncu, reps);
    for (int W : {4, 6}) run<24, 0>(W, turns, ncu, reps);
    return 0;
}
