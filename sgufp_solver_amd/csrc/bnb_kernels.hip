// Device frontier kernels of the batched B&B (the GPU-resident replacement of the
// reference's lock_free_queue / lf_node lists, lock_free_queue.h:24-165, DDSolver.h:264-291).
//
//   k_gather_paths    argmax paths of the exact DDs still in their refinement loop, packed
//                     for the host's seen-path check (NodeExplorer.cpp:948-956)
//   k_push_children   cutset children of the kept parents, compacted from the emit buffers
//                     onto the frontier stack (Worker::startWorker pushes result.nodes when
//                     result.ub > zOpt, DDSolver.cpp:744-748)
//
// Both are copy kernels: one wave per parent / path, lanes stride over the records and the
// int16 solution spans, so the HBM traffic is the bytes moved.
#include <hip/hip_runtime.h>

#include "dd_device.hpp"
#include "wave.hpp"

namespace sgufp {

__global__ void __launch_bounds__(kWave) k_gather_paths(BatchOut out, int Lcap, const int32_t *idx,
                                                        const int64_t *off, int n, int16_t *dst) {
    const int w = blockIdx.x;
    if (w >= n) return;
    const int slot = idx[w];
    const int64_t o = off[w];
    const int len = (int)(off[w + 1] - o);
    const GBL int16_t *src = out.path + (size_t)slot * Lcap;
    for (int t = lane(); t < len; t += kWave) dst[o + t] = src[t];
}

// parents[w]: batch index of kept parent w; dst_child[w] / dst_sol[w]: first frontier entry /
// first arena entry of its children.  The emit kernel laid a parent's children solutions out
// in one span [sol_base[p], sol_base[p] + sol_need[p]) (stride = len + cut layer, each child
// possibly shorter, DD.cpp:3803-3818); the span moves as a whole, offsets are rebased.
__global__ void __launch_bounds__(kWave) k_push_children(ChildOut co, BatchOut out, const int32_t *parents,
                                                         const int64_t *dst_child, const int64_t *dst_sol, int n,
                                                         FrontierDev fr) {
    const int w = blockIdx.x;
    if (w >= n) return;
    const int p = parents[w];
    const uint64_t c0 = co.child_off[p], c1 = co.child_off[p + 1];
    const uint64_t s0 = co.sol_base[p];
    const uint32_t span = out.sol_need[p];
    const int64_t dc = dst_child[w];
    const int64_t ds = dst_sol[w];
    for (uint64_t c = c0 + lane(); c < c1; c += kWave) {
        const int64_t e = dc + (int64_t)(c - c0);
        fr.gl[e] = co.gl[c];
        fr.lb[e] = co.lb[c];
        fr.ub[e] = co.ub[c];
        fr.mask[e] = co.mask[c];
        fr.valid[e] = 1;
        fr.sol_off[e] = ds + (co.sol_off[c] - (int64_t)s0);
        fr.sol_len[e] = co.sol_len[c];
    }
    for (uint32_t t = lane(); t < span; t += kWave) fr.sol[ds + t] = co.sol[s0 + t];
}

hipError_t launch_gather_paths(const BatchOut &out, int Lcap, const int32_t *idx, const int64_t *off, int n,
                               int16_t *dst, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_gather_paths, dim3(n), dim3(kWave), 0, st, out, Lcap, idx, off, n, dst);
    return hipGetLastError();
}

hipError_t launch_push_children(const ChildOut &co, const BatchOut &out, const int32_t *parents,
                                const int64_t *dst_child, const int64_t *dst_sol, int n, const FrontierDev &fr,
                                hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_push_children, dim3(n), dim3(kWave), 0, st, co, out, parents, dst_child, dst_sol, n, fr);
    return hipGetLastError();
}

}  // namespace sgufp
