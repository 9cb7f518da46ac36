// FETCH_SIZE / WRITE_SIZE calibration on gfx950 for the access widths the stencils use:
// stream-copy BYTES (1 GiB, beyond the 256 MiB MALL) with 8-B/lane (dwordx2) and
// 16-B/lane (dwordx4) coalesced loads and stores.  Run under
//   rocprofv3 --pmc FETCH_SIZE  -- ./calib_fetch     (and again with WRITE_SIZE)
// and compare the per-dispatch counters (KiB) with BYTES / 1024.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <typename T>
__global__ __launch_bounds__(256) void k_copy(const T *__restrict__ in, T *__restrict__ out,
                                              size_t n)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}

int main()
{
    const size_t bytes = 1ull << 30;
    void *a = nullptr, *b = nullptr;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
    hipMemset(a, 1, bytes);
    hipMemset(b, 0, bytes);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_copy<uint2>, dim3(8192), dim3(256), 0, 0, (const uint2 *)a, (uint2 *)b,
                           bytes / 8);
        hipLaunchKernelGGL(k_copy<uint4>, dim3(8192), dim3(256), 0, 0, (const uint4 *)a, (uint4 *)b,
                           bytes / 16);
    }
    hipDeviceSynchronize();
    printf("calib_fetch: %zu bytes per copy (%zu KiB)\n", bytes, bytes / 1024);
    hipFree(a);
    hipFree(b);
    return 0;
}
