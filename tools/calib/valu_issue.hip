// valu_issue.hip -- issue cost of the stencil's VALU instructions on one gfx950 SIMD.
//
// Every wave runs `iters` x 32 instructions of one kind over 8 independent accumulators
// (no dependency stalls from a single chain), timed with s_memtime (shader clock) and
// s_memrealtime (100 MHz).  W waves share each SIMD (grid = 256 CUs x 4 SIMDs x W waves,
// one wave per SIMD per workgroup), so cycles per instruction per SIMD = dt / (W x n).
// Build: hipcc --offload-arch=gfx950 -O3 -o valu_issue valu_issue.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define OP8(INS)                                                                             \
    asm volatile(INS : "+v"(a0) : "v"(b), "v"(c));                                           \
    asm volatile(INS : "+v"(a1) : "v"(b), "v"(c));                                           \
    asm volatile(INS : "+v"(a2) : "v"(b), "v"(c));                                           \
    asm volatile(INS : "+v"(a3) : "v"(b), "v"(c));                                           \
    asm volatile(INS : "+v"(a4) : "v"(b), "v"(c));                                           \
    asm volatile(INS : "+v"(a5) : "v"(b), "v"(c));                                           \
    asm volatile(INS : "+v"(a6) : "v"(b), "v"(c));                                           \
    asm volatile(INS : "+v"(a7) : "v"(b), "v"(c));

template <int OP>
__global__ __launch_bounds__(256) void k_issue(unsigned long long *cyc, unsigned *sink, int iters)
{
    uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 ^ 9, a5 = a0 + 11,
             a6 = a0 * 13, a7 = a0 ^ 0x55;
    const uint32_t b = blockIdx.x * 0x9e37u + threadIdx.x, c = b * 0x85ebu;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if constexpr (OP == 0) { OP8("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96") }
            if constexpr (OP == 1) { OP8("v_alignbit_b32 %0, %0, %1, 31") }
            if constexpr (OP == 2) { OP8("v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0") }
            if constexpr (OP == 3) { OP8("v_xor_b32 %0, %0, %1") }
            if constexpr (OP == 4) { OP8("v_or3_b32 %0, %0, %1, %2") }
            if constexpr (OP == 5) { OP8("v_lshl_or_b32 %0, %0, 1, %1") }
            if constexpr (OP == 6) { OP8("v_add_u32 %0, %0, %1") }
            if constexpr (OP == 7) { OP8("v_and_or_b32 %0, %0, %1, %2") }
            if constexpr (OP == 8) { OP8("v_xor_b32_dpp %0, %1, %0 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0") }
            if constexpr (OP == 9) { OP8("v_fma_f32 %0, %0, %1, %2") }
            if constexpr (OP == 10) {   // one dependent chain (8 deep per OP8 group)
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a0) : "v"(b), "v"(c));
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a0) : "v"(b), "v"(c));
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a0) : "v"(b), "v"(c));
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a0) : "v"(b), "v"(c));
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a0) : "v"(b), "v"(c));
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a0) : "v"(b), "v"(c));
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a0) : "v"(b), "v"(c));
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a0) : "v"(b), "v"(c));
            }
            if constexpr (OP == 11) {   // two interleaved dependent chains
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a0) : "v"(b), "v"(c));
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a1) : "v"(b), "v"(c));
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a0) : "v"(b), "v"(c));
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a1) : "v"(b), "v"(c));
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a0) : "v"(b), "v"(c));
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a1) : "v"(b), "v"(c));
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a0) : "v"(b), "v"(c));
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a1) : "v"(b), "v"(c));
            }
            if constexpr (OP == 12) {   // the stencil's mix: 9 bitop3 : 1 alignbit : 1 DPP
                OP8("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")
                asm volatile("v_alignbit_b32 %0, %0, %1, 31" : "+v"(a0) : "v"(b));
                asm volatile("v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0" : "+v"(a1) : "v"(c));
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    const uint32_t s = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (s == 0x12345678u) sink[0] = s;                  // keep the work alive
    if ((threadIdx.x & 63) == 0) {
        const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
        cyc[2 * w] = t1 - t0;
        cyc[2 * w + 1] = r1 - r0;
    }
}

static const char *kNames[] = {"v_bitop3_b32", "v_alignbit_b32", "v_mov_b32_dpp", "v_xor_b32",
                               "v_or3_b32", "v_lshl_or_b32", "v_add_u32", "v_and_or_b32",
                               "v_xor_b32_dpp", "v_fma_f32", "bitop3 chain x1", "bitop3 chains x2",
                               "mix 8 bitop3+1 align+1 dpp"};

template <int OP>
static void run(int W, int iters, int ncu)
{
    const int blocks = ncu * W;
    unsigned long long *d_cyc;
    unsigned *d_sink;
    (void)hipMalloc(&d_cyc, (size_t)blocks * 4 * 2 * 8);
    (void)hipMalloc(&d_sink, 4);
    hipLaunchKernelGGL(k_issue<OP>, dim3(blocks), dim3(256), 0, 0, d_cyc, d_sink, iters / 10);
    hipLaunchKernelGGL(k_issue<OP>, dim3(blocks), dim3(256), 0, 0, d_cyc, d_sink, iters);
    if (hipDeviceSynchronize() != hipSuccess) { std::printf("launch failed\n"); std::exit(1); }
    std::vector<unsigned long long> h((size_t)blocks * 8);
    (void)hipMemcpy(h.data(), d_cyc, h.size() * 8, hipMemcpyDeviceToHost);
    std::vector<double> cpi, ghz;
    for (int w = 0; w < blocks * 4; ++w) {
        const double per_iter = OP == 12 ? 40.0 : 32.0;
        cpi.push_back((double)h[2 * w] / ((double)W * iters * per_iter));
        ghz.push_back((double)h[2 * w] / (double)h[2 * w + 1] * 0.1);
    }
    std::sort(cpi.begin(), cpi.end());
    std::sort(ghz.begin(), ghz.end());
    std::printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"cyc_per_instr_per_simd\": %.3f, "
                "\"p10\": %.3f, \"p90\": %.3f, \"clock_ghz\": %.3f}\n",
                kNames[OP], W, cpi[cpi.size() / 2], cpi[cpi.size() / 10], cpi[cpi.size() * 9 / 10],
                ghz[ghz.size() / 2]);
    (void)hipFree(d_cyc);
    (void)hipFree(d_sink);
}

template <int OP>
static void sweep(int iters, int ncu)
{
    for (int W : {1, 2, 3, 4, 8}) run<OP>(W, iters, ncu);
}

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? std::atoi(argv[1]) : 20000;
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    if (argc > 2 && std::string(argv[2]) == "occupancy") {
        // the stencil's mix and the lone bitop3 at every resident-wave count 1..8 per SIMD
        for (int W = 1; W <= 8; ++W) run<12>(W, iters, ncu);
        for (int W = 1; W <= 8; ++W) run<0>(W, iters, ncu);
        for (int W = 1; W <= 8; ++W) run<10>(W, iters, ncu);
        return 0;
    }
    sweep<0>(iters, ncu);
    sweep<1>(iters, ncu);
    sweep<2>(iters, ncu);
    sweep<3>(iters, ncu);
    sweep<4>(iters, ncu);
    sweep<5>(iters, ncu);
    sweep<6>(iters, ncu);
    sweep<7>(iters, ncu);
    sweep<8>(iters, ncu);
    sweep<9>(iters, ncu);
    sweep<10>(iters, ncu);
    sweep<11>(iters, ncu);
    sweep<12>(iters, ncu);
    return 0;
}
