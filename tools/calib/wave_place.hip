// wave_place.hip -- where the dispatcher puts the 4 wavefronts of a 256-thread workgroup.
// Every wave records its hardware id (HW_ID: SIMD, CU, SE) and XCC id; the host prints,
// per wave index w, how often wave w lands on SIMD (w + r) mod 4 for r = 0..3, and how many
// workgroups keep all 4 waves on distinct SIMDs.  k_step_wg's roles (wave 0 streams, the
// last stores) are per wave index, so this says whether a SIMD ends up holding one role.
// Build: hipcc --offload-arch=gfx950 -O3 -o wave_place wave_place.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <map>
#include <vector>

__global__ __launch_bounds__(256) void k_place(unsigned *rec, int spin)
{
    __shared__ unsigned pad[4096];                      // 16 KB: at most 10 workgroups per CU
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    pad[threadIdx.x] = hw;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - t0 < (unsigned long long)spin) __builtin_amdgcn_s_sleep(2);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        const int w = threadIdx.x >> 6;
        rec[(blockIdx.x * 4 + w) * 2] = hw + pad[(threadIdx.x + 64) & 255] * 0;
        rec[(blockIdx.x * 4 + w) * 2 + 1] = xcc;
    }
}

int main()
{
    const int blocks = 256 * 8;
    unsigned *d;
    (void)hipMalloc(&d, blocks * 8 * sizeof(unsigned));
    hipLaunchKernelGGL(k_place, dim3(blocks), dim3(256), 0, 0, d, 200000);
    std::vector<unsigned> h(blocks * 8);
    (void)hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    int rot[4][4] = {}, distinct = 0;
    std::map<unsigned, int> per_cu;                     // workgroups per (xcc, se, cu)
    std::map<unsigned, std::vector<int>> first_simd;     // wave 0's SIMD per CU
    for (int b = 0; b < blocks; ++b) {
        int mask = 0;
        unsigned key = 0;
        for (int w = 0; w < 4; ++w) {
            const unsigned hw = h[(b * 4 + w) * 2], xcc = h[(b * 4 + w) * 2 + 1] & 0xf;
            const int simd = (hw >> 4) & 3;
            rot[w][(simd - w + 4) & 3]++;
            mask |= 1 << simd;
            if (w == 0) {
                key = (xcc << 16) | (((hw >> 13) & 7) << 8) | ((hw >> 8) & 15);
                first_simd[key].push_back(simd);
            }
        }
        distinct += mask == 15;
        per_cu[key]++;
    }
    printf("workgroups %d, all 4 waves on distinct SIMDs: %d\n", blocks, distinct);
    for (int w = 0; w < 4; ++w)
        printf("wave %d on SIMD (w + r) %% 4: r=0 %d  r=1 %d  r=2 %d  r=3 %d\n", w, rot[w][0],
               rot[w][1], rot[w][2], rot[w][3]);
    printf("CUs seen %zu; first CU's workgroups' wave-0 SIMDs:", per_cu.size());
    int shown = 0;
    for (auto &kv : first_simd) {
        if (shown++ >= 4) break;
        printf("\n  cu %06x:", kv.first);
        for (int s : kv.second) printf(" %d", s);
    }
    printf("\n");
    // the same for the k_step_wg shape: 1 wave per SIMD per WG assumed above
    return 0;
}
