// Single-wave building blocks shared by the relaxation and subproblem kernels (gfx950,
// wave64, one wave per workgroup).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "dd_device.hpp"

namespace sgufp {

#define LDS __attribute__((address_space(3)))
#define GBL SGUFP_GBL

// lane within the wave; translation units with multi-wave workgroups (SGUFP_MULTI_WAVE_TU)
// mask the thread id, the single-wave ones use it as is
#ifdef SGUFP_MULTI_WAVE_TU
__device__ __forceinline__ int lane() { return (int)(threadIdx.x & (kWave - 1)); }
#else
__device__ __forceinline__ int lane() { return (int)threadIdx.x; }
#endif
// a wave-uniform value read from LDS / memory, moved to an SGPR (scalar branches and
// address arithmetic instead of per-lane ones)
__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint32_t uni(uint8_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ double smax(double a, double b) { return (a < b) ? b : a; }  // std::max
__device__ __forceinline__ double smin(double a, double b) { return (b < a) ? b : a; }  // std::min
__device__ __forceinline__ uint32_t gsub(GBL uint32_t *p, uint32_t v) {
    return __hip_atomic_fetch_sub(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// LDS is in order within a wavefront; this only stops the compiler from moving
// LDS accesses across the point (the workgroup is a single wave).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// Scheduling fence: the compiler moves no instruction across it.  At 256 VGPRs the
// machine scheduler otherwise interleaves each LDS load with its first use (one
// s_waitcnt lgkmcnt(0) per load); a fence after a block of independent loads keeps them
// issued back to back, so the block costs one LDS latency instead of one per load.
__device__ __forceinline__ void sched_fence() { __builtin_amdgcn_sched_barrier(0); }

// Global-memory hand-off between lanes of the wave (stores complete, then loads).
__device__ __forceinline__ void wave_mem_sync() { __syncthreads(); }

// Inclusive prefix sum over the wave with DPP (no LDS crossbar round trips): row_shr 1, 2,
// 4, 8 scan each 16-lane row, then row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3)
// carry the row totals.  Lanes whose DPP source is outside the row read old = 0.
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);   // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);   // row_bcast:31
    return x;
}
// Butterfly partner exchange without the LDS path: DPP row rotations inside 16-lane
// rows (a rotation by S pairs the same orbits as xor S for an all-reduce), and the
// gfx950 permlane swaps across rows (16) and half-waves (32).  Every lane of the wave
// must be active.
template <int S>
__device__ __forceinline__ uint32_t lane_x(uint32_t x) {
    if constexpr (S == 32) {
        auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return lane() < 32 ? r[1] : r[0];
    } else if constexpr (S == 16) {
        auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        return (lane() & 16) ? r[0] : r[1];
    } else {
        static_assert(S == 1 || S == 2 || S == 4 || S == 8, "row rotation");
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x120 + S, 0xF, 0xF, false);
    }
}
template <int S>
__device__ __forceinline__ int lane_x(int x) { return (int)lane_x<S>((uint32_t)x); }
template <int S>
__device__ __forceinline__ int64_t lane_x(int64_t x) {
    const uint64_t b = (uint64_t)x;
    const uint32_t lo = lane_x<S>((uint32_t)b), hi = lane_x<S>((uint32_t)(b >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
template <int S>
__device__ __forceinline__ double lane_x(double x) {
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    const uint32_t lo = lane_x<S>((uint32_t)b), hi = lane_x<S>((uint32_t)(b >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
// all-reduce over the lanes that differ in bits log2(S0) .. 5 of the lane id
template <int S0, typename T, typename Op>
__device__ __forceinline__ T lane_reduce(T x, Op op) {
    if constexpr (S0 < kWave) {
        x = op(x, lane_x<S0>(x));
        return lane_reduce<S0 * 2>(x, op);
    } else {
        return x;
    }
}
// value of lane l (wave-uniform l) in every lane
__device__ __forceinline__ double lane_get(double x, int l) {
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
    return lane_reduce<1>(x, [](uint32_t a, uint32_t b) { return a + b; });
}
__device__ __forceinline__ uint32_t wave_or(uint32_t x) {
    return lane_reduce<1>(x, [](uint32_t a, uint32_t b) { return a | b; });
}

}  // namespace sgufp
