// turn_issue.hip -- the issue rate of K1t's turn body: the compiler's schedule and register
// assignment (ORD 5's stream, as stencil_issue.hip MIX 0) against the hand-assigned inline-asm
// turn of gen_tile_turn.py (ORD 8, every v_bitop3 with mixed-parity sources), both without
// the LDS exchange and barrier, at forced occupancy (4-wave workgroups, LDS per workgroup so
// exactly W fit a CU).  SIMD cycles per VALU = kernel time x clock / (W x VALU per wave), the
// clock from each wave's s_memtime / s_memrealtime; VALU per wave = turns x SEG x 22.
// Build: hipcc --offload-arch=gfx950 -O3 -DGOL_TURN_ISO -I../../conway-s-gol-distributed_amd/csrc \
//        -o turn_issue turn_issue.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gol_device.h"
#include "gol_tile_turn.h"

using namespace golk;

__device__ __forceinline__ void rsum(const uint32_t (&x)[2], uint32_t (&s)[4])
{
    const uint32_t e = x[0], o = x[1];
    const uint32_t L = dpp_from_lower_z(o), R = dpp_from_upper_z(e);
    const uint32_t wl = __builtin_amdgcn_alignbit(o, L, 31), er = __builtin_amdgcn_alignbit(R, e, 1);
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

template <int SEG, int HAND>
__global__ __launch_bounds__(256, 6) void k_turn(uint32_t *out, unsigned long long *clk, int turns)
{
    extern __shared__ uint32_t pad[];
    uint32_t v[SEG][2];
    const uint32_t seed = blockIdx.x * 0x9e3779b9u + threadIdx.x * 0x85ebca6bu;
#pragma unroll
    for (int i = 0; i < SEG; ++i) {
        v[i][0] = seed * (2u * i + 1u) ^ 0x5bd1e995u;
        v[i][1] = (seed + 0x27d4eb2fu * i) * 0x165667b1u;
    }
    if (threadIdx.x == 0) pad[0] = seed;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int t = 0; t < turns; ++t) {
        if constexpr (HAND >= 0) {
            tile_turn_iso<SEG, HAND>(v);
        } else {
            uint32_t first[4], last[4], P[4], Q[4];
            rsum(v[SEG - 1], last);
            rsum(v[0], first);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                P[k] = last[k];
                Q[k] = first[k];
            }
#pragma unroll
            for (int i = 0; i < SEG; ++i) {
                uint32_t R[4];
                if (i + 2 < SEG) rsum(v[i + 1], R);
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

template <int SEG, int HAND>
static void run(int W, int turns, int ncu, int reps)
{
    auto fn = k_turn<SEG, HAND>;
    const int blocks = ncu * W;
    const size_t lds = (size_t)160 * 1024 / W - 1024;
    hipFuncAttributes attr;
    (void)hipFuncGetAttributes(&attr, reinterpret_cast<const void *>(fn));
    uint32_t *d_out;
    unsigned long long *d_clk;
    (void)hipMalloc(&d_out, (size_t)blocks * 256 * 4);
    (void)hipMalloc(&d_clk, (size_t)blocks * 4 * 2 * 8);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), lds, 0, d_out, d_clk, turns);
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
    std::printf("{\"body\": \"%s\", \"seg\": %d, \"waves_per_simd\": %d, \"vgprs\": %d, \"kernel_ms\": %.4f, "
                "\"clock_ghz\": %.3f, \"simd_cycles_per_valu\": %.4f, \"cycles_per_row\": %.2f}\n",
                HAND < 0 ? "compiler (ORD 5 stream)" : HAND ? "hand-assigned asm, DPP two rows ahead" : "hand-assigned asm (ORD 8)", SEG, W, attr.numRegs,
                best, clock, cyc, cyc * 22.0);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(d_out);
    (void)hipFree(d_clk);
}

int main(int argc, char **argv)
{
    const int turns = argc > 1 ? std::atoi(argv[1]) : 4000;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 3;
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    for (int W : {4, 6}) {
        run<24, -1>(W, turns, ncu, reps);
        run<24, 0>(W, turns, ncu, reps);
        run<24, 8>(W, turns, ncu, reps);
    }
    for (int W : {4, 8}) {
        run<12, -1>(W, turns, ncu, reps);
        run<12, 0>(W, turns, ncu, reps);
        run<12, 8>(W, turns, ncu, reps);
        run<6, -1>(W, turns, ncu, reps);
        run<6, 0>(W, turns, ncu, reps);
        run<6, 8>(W, turns, ncu, reps);
    }
    return 0;
}
