// FETCH_SIZE / WRITE_SIZE calibration on gfx950 for the access widths the stencils use:
// stream-copy BYTES (1 GiB, beyond the 256 MiB MALL) with 8-B/lane (dwordx2) and
// 16-B/lane (dwordx4) coalesced loads and stores, and stream-read BYTES with
// 4-B/lane LDS-DMA (buffer_load_dword ... lds: the temporal-blocking kernel's row loads,
// two dwords per lane of an 8-B word).  Run under
//   rocprofv3 --pmc FETCH_SIZE  -- ./calib_fetch     (and again with WRITE_SIZE)
// and compare the per-dispatch counters (KiB) with BYTES / 1024.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef __attribute__((address_space(3))) void lds_void;

// each wavefront streams 512-B rows (64 lanes x 8 B) as two 4-B LDS-DMA loads per lane
__global__ __launch_bounds__(256) void k_dma_read(const uint32_t *__restrict__ in, size_t rows,
                                                  unsigned *sink)
{
    __shared__ uint32_t slot[4][2][64];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc((void *)in, (short)0, 0x7fffffff, 0x00020000);
    for (size_t row = (size_t)blockIdx.x * 4 + w; row < rows; row += (size_t)gridDim.x * 4) {
        const uint32_t off = (uint32_t)(row * 512);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void *)&slot[w][0][0], 4, lane * 8u, off,
                                                 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void *)&slot[w][1][0], 4, lane * 8u,
                                                 off + 4, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0);
    if (slot[w][0][lane] == 0x12345678u && slot[w][1][lane] == 0x9abcdef0u) sink[0] = 1;
}

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
    unsigned *sink = nullptr;
    if (hipMalloc(&sink, 4) != hipSuccess) return 1;
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_dma_read, dim3(8192), dim3(256), 0, 0, (const uint32_t *)a,
                           (bytes - 4096) / 512, sink);   // < 2 GiB buffer range
        hipLaunchKernelGGL(k_copy<uint2>, dim3(8192), dim3(256), 0, 0, (const uint2 *)a, (uint2 *)b,
                           bytes / 8);
        hipLaunchKernelGGL(k_copy<uint4>, dim3(8192), dim3(256), 0, 0, (const uint4 *)a, (uint4 *)b,
                           bytes / 16);
    }
    hipDeviceSynchronize();
    printf("calib_fetch: %zu bytes per copy (%zu KiB)\n", bytes, bytes / 1024);
    hipFree(a);
    hipFree(b);
    hipFree(sink);
    return 0;
}
