// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths the
// relaxation kernels use (1, 2, 4, 8, 16 B per lane).  Every kernel streams a 1 GiB
// buffer (4x the 256 MiB Infinity Cache) exactly once, fully coalesced, so the true HBM
// bytes per launch are known: 1 GiB read (rd_*) or written (wr_*).  Run under
//   rocprofv3 --pmc FETCH_SIZE ... -- ./calib_fetch   (and a second pass with WRITE_SIZE)
// and divide the counter (KB) by the known bytes: tools/calib/calib_table.py.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

constexpr size_t kBytes = size_t(1) << 30;

template <typename T>
__device__ __forceinline__ uint32_t fold(T v) {
    if constexpr (sizeof(T) <= 4) return (uint32_t)v;
    else if constexpr (sizeof(T) == 8) return (uint32_t)v ^ (uint32_t)(v >> 32);
    else return v.x ^ v.y ^ v.z ^ v.w;
}

// grid-stride coalesced read of n elements of T; one store per thread keeps the loads live
template <typename T>
__global__ void __launch_bounds__(256) rd(const T *__restrict__ p, size_t n, uint32_t *sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc = acc * 31u + fold(p[i]);         // every loaded byte reaches the result
    if (acc == 0x9E3779B9u) sink[0] = acc;   // practically never: no write traffic
}

template <typename T>
__global__ void __launch_bounds__(256) wr(T *__restrict__ p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        T v{};
        if constexpr (sizeof(T) == 16) v = T{(uint32_t)i, 1u, 2u, 3u};
        else v = (T)i;
        p[i] = v;
    }
}

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                 \
            return 1;                                                              \
        }                                                                          \
    } while (0)

int main() {
    uint8_t *buf = nullptr;
    uint32_t *sink = nullptr;
    CHECK(hipMalloc(&buf, kBytes));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(buf, 1, kBytes));
    const dim3 grid(256 * 8 * 4), block(256);
    // read widths (kernel names carry the width: rd<unsigned char> ... rd<uint4>)
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(rd<uint8_t>, grid, block, 0, 0, buf, kBytes, sink);
        hipLaunchKernelGGL(rd<uint16_t>, grid, block, 0, 0, (const uint16_t *)buf, kBytes / 2, sink);
        hipLaunchKernelGGL(rd<uint32_t>, grid, block, 0, 0, (const uint32_t *)buf, kBytes / 4, sink);
        hipLaunchKernelGGL(rd<uint64_t>, grid, block, 0, 0, (const uint64_t *)buf, kBytes / 8, sink);
        hipLaunchKernelGGL(rd<uint4>, grid, block, 0, 0, (const uint4 *)buf, kBytes / 16, sink);
        hipLaunchKernelGGL(wr<uint8_t>, grid, block, 0, 0, buf, kBytes);
        hipLaunchKernelGGL(wr<uint16_t>, grid, block, 0, 0, (uint16_t *)buf, kBytes / 2);
        hipLaunchKernelGGL(wr<uint32_t>, grid, block, 0, 0, (uint32_t *)buf, kBytes / 4);
        hipLaunchKernelGGL(wr<uint64_t>, grid, block, 0, 0, (uint64_t *)buf, kBytes / 8);
        hipLaunchKernelGGL(wr<uint4>, grid, block, 0, 0, (uint4 *)buf, kBytes / 16);
        CHECK(hipDeviceSynchronize());
    }
    CHECK(hipGetLastError());
    printf("calib_fetch: 10 kernels x 2 reps, %zu bytes each\n", kBytes);
    CHECK(hipFree(buf));
    CHECK(hipFree(sink));
    return 0;
}
