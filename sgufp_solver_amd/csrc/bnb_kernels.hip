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

namespace sgufp {

// ---- cut-pool rows and frontier records between frontier shards (shard.cpp) ----------

// pool rows ids[k] -> out[k] = {rhs, row[0 .. stride)}: one send block for the RCCL all-gather
__global__ void __launch_bounds__(256) k_gather_rows(const double *rows, const double *rhs, const int32_t *ids, int k,
                                                     int stride, double *out) {
    const int c = blockIdx.x;
    if (c >= k) return;
    const size_t r = (size_t)ids[c];
    double *o = out + (size_t)c * (stride + 1);
    if (threadIdx.x == 0) o[0] = rhs[r];
    for (int v = threadIdx.x; v < stride; v += blockDim.x) o[1 + v] = rows[r * stride + v];
}

// n rows {rhs, row} appended at pool rows first ..: the dense row (its last, absent-key slot
// zeroed), the RHS, the per-(layer, state rank) table of the batched sweeps and the
// node-independent bound of the screening order -- what sgufp_ctx::append_rows builds on
// the host, in the same order of operations (the bound: RHS + sum over layers, in layer
// order, of max(0, max over ranks)).
__global__ void __launch_bounds__(256) k_append_rows(const double *src, int n, int stride, int first, double *rows,
                                                     double *rhs, double *coefT, const int32_t *slot_tab, int L,
                                                     int us, double *row_ub) {
    const int c = blockIdx.x;
    if (c >= n) return;
    const double *s = src + (size_t)c * (stride + 1);
    const size_t r = (size_t)(first + c);
    for (int v = threadIdx.x; v < stride; v += blockDim.x) rows[r * stride + v] = (v == stride - 1) ? 0.0 : s[1 + v];
    const size_t tstride = (size_t)(L > 0 ? L : 1) * us;
    for (int e = threadIdx.x; e < L * us; e += blockDim.x) {
        const int l = e / us, k = e - l * us;
        const int sl = slot_tab[(size_t)l * kMaxU + k];
        coefT[r * tstride + e] = (sl >= 0 && sl < stride - 1) ? s[1 + sl] : 0.0;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        rhs[r] = s[0];
        double b = s[0];
        for (int l = 0; l < L; l++) {
            double m = 0.0;
            for (int k = 0; k < us; k++) {
                const int sl = slot_tab[(size_t)l * kMaxU + k];
                const double x = (sl >= 0 && sl < stride - 1) ? s[1 + sl] : 0.0;
                m = (m < x) ? x : m;   // std::max(m, x)
            }
            b += m;
        }
        row_ub[c] = b;
    }
}

__global__ void __launch_bounds__(256) k_rebase(int64_t *off, int n, int64_t delta) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) off[i] += delta;
}

hipError_t launch_gather_rows(const double *rows, const double *rhs, const int32_t *ids, int k, int stride, double *out,
                              hipStream_t st) {
    if (k <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_gather_rows, dim3(k), dim3(256), 0, st, rows, rhs, ids, k, stride, out);
    return hipGetLastError();
}

hipError_t launch_append_rows(const double *src, int n, int stride, int first, double *rows, double *rhs,
                              double *coefT, const int32_t *slot_tab, int L, int us, double *row_ub, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_append_rows, dim3(n), dim3(256), 0, st, src, n, stride, first, rows, rhs, coefT, slot_tab, L,
                       us, row_ub);
    return hipGetLastError();
}

hipError_t launch_rebase(int64_t *off, int n, int64_t delta, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_rebase, dim3((n + 255) / 256), dim3(256), 0, st, off, n, delta);
    return hipGetLastError();
}

}  // namespace sgufp

namespace sgufp {

// ---- device-resident refinement loop of the exact DDs (NodeExplorer.cpp:946-969) --------
// The loop's seen-path lists live in HBM (one list per batch slot, `cap` paths of Lcap
// int16 each, with their lengths and a 64-bit order-free hash), so one iteration -- check
// the argmax paths, solve the fresh ones' scenario subproblems, append the cuts to the pool,
// apply them -- is one stream sequence with a single host synchronisation (bnb.cpp).

__device__ __forceinline__ uint64_t mix64(uint64_t z) {   // splitmix64 finaliser
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// hash of a path (sum over positions, so the lanes add their parts in any order) and the
// number of decided arcs (the scenario subproblem's chain count is m minus that)
__device__ inline void path_hash(const GBL int16_t *path, int len, int m, uint64_t &h, uint32_t &decided) {
    uint64_t x = 0;
    uint32_t d = 0;
    for (int t = lane(); t < len; t += kWave) {
        const int v = path[t];
        x += mix64(((uint64_t)(uint32_t)t << 16) ^ (uint64_t)(uint16_t)v ^ 0x9E3779B97F4A7C15ull);
        d += (v >= 0 && v < m) ? 1u : 0u;
    }
    for (int o = 32; o > 0; o >>= 1) {
        x += (uint64_t)__shfl_xor((long long)x, o, kWave);
        d += (uint32_t)__shfl_xor((int)d, o, kWave);
    }
    h = x + mix64((uint64_t)len + 1);
    decided = d;
}

// One wave per record still in the loop: flag[a] = 1 its argmax path was seen ({ub, ub}),
// 2 fresh (the subproblem is next), 3 + status when the last cut pruned it (status 1 / 2);
// chains[a] = m - decided arcs of a fresh path.
__global__ void __launch_bounds__(kWave) k_loop_check(BatchOut out, SeenLists S, const int32_t *act, int na, int m,
                                                      int32_t *flag, int32_t *chains) {
    const int a = blockIdx.x;
    if (a >= na) return;
    const int slot = act[a];
    const int st = out.status[slot];
    if (st != kNeedsSubproblem) {
        if (lane() == 0) { flag[a] = 3 + st; chains[a] = 0; }
        return;
    }
    const int len = out.path_len[slot];
    const GBL int16_t *path = out.path + (size_t)slot * S.Lcap;
    uint64_t h;
    uint32_t decided;
    path_hash(path, len, m, h, decided);
    const int ns = S.n[slot];
    bool found = false;
    for (int i = 0; i < ns && !found; i++) {
        const size_t e = (size_t)slot * S.cap + i;
        if (S.hash[e] != h || S.len[e] != (uint16_t)len) continue;
        const GBL int16_t *sp = S.paths + e * S.Lcap;
        uint32_t diff = 0;
        for (int t = lane(); t < len; t += kWave) diff |= (sp[t] != path[t]) ? 1u : 0u;
        found = !wave_or(diff);
    }
    if (lane() == 0) {
        flag[a] = found ? 1 : 2;
        chains[a] = m - (int)decided;
    }
}

// the fresh records' paths join their seen lists
__global__ void __launch_bounds__(kWave) k_seen_append(BatchOut out, SeenLists S, const int32_t *fresh, int nf, int m) {
    const int f = blockIdx.x;
    if (f >= nf) return;
    const int slot = fresh[f];
    const int len = out.path_len[slot];
    const GBL int16_t *path = out.path + (size_t)slot * S.Lcap;
    uint64_t h;
    uint32_t decided;
    path_hash(path, len, m, h, decided);
    const int i = S.n[slot];
    const size_t e = (size_t)slot * S.cap + i;
    for (int t = lane(); t < len; t += kWave) S.paths[e * S.Lcap + t] = path[t];
    if (lane() == 0) {
        S.len[e] = (uint16_t)len;
        S.hash[e] = h;
        S.n[slot] = i + 1;
    }
}

// The subproblem's cuts (k_sub_reduce: cut_type / cut_rhs / cut_row per fresh record) join the
// pool at rows first + f (Container::add; the host files each row under the feasibility or the
// optimality list from cut_type at its next synchronisation): dense row, RHS, the batched
// sweeps' (layer, rank) table and the screening bound as sgufp_ctx::append_rows builds them;
// row_id / is_feas feed k_refine.
__global__ void __launch_bounds__(256) k_append_cuts(const int32_t *cut_type, const double *cut_rhs,
                                                     const double *cut_row, int nf, int stride, int first,
                                                     double *rows, double *rhs, double *coefT,
                                                     const int32_t *slot_tab, int L, int us, double *row_ub,
                                                     int32_t *row_id, uint8_t *is_feas) {
    const int f = blockIdx.x;
    if (f >= nf) return;
    const double *s = cut_row + (size_t)f * stride;
    const size_t r = (size_t)(first + f);
    for (int v = threadIdx.x; v < stride; v += blockDim.x) rows[r * stride + v] = (v == stride - 1) ? 0.0 : s[v];
    const size_t tstride = (size_t)(L > 0 ? L : 1) * us;
    for (int e = threadIdx.x; e < L * us; e += blockDim.x) {
        const int l = e / us, k = e - l * us;
        const int sl = slot_tab[(size_t)l * kMaxU + k];
        coefT[r * tstride + e] = (sl >= 0 && sl < stride - 1) ? s[sl] : 0.0;
    }
    if (threadIdx.x == 0) {
        const double h = cut_rhs[f];
        rhs[r] = h;
        double b = h;
        for (int l = 0; l < L; l++) {
            double mx = 0.0;
            for (int k = 0; k < us; k++) {
                const int sl = slot_tab[(size_t)l * kMaxU + k];
                const double x = (sl >= 0 && sl < stride - 1) ? s[sl] : 0.0;
                mx = (mx < x) ? x : mx;
            }
            b += mx;
        }
        row_ub[f] = b;
        row_id[f] = (int32_t)r;
        is_feas[f] = cut_type[f] == 1 ? 1 : 0;
    }
}

hipError_t launch_loop_check(const BatchOut &out, const SeenLists &S, const int32_t *act, int na, int m, int32_t *flag,
                             int32_t *chains, hipStream_t st) {
    if (na <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_loop_check, dim3(na), dim3(kWave), 0, st, out, S, act, na, m, flag, chains);
    return hipGetLastError();
}

hipError_t launch_seen_append(const BatchOut &out, const SeenLists &S, const int32_t *fresh, int nf, int m,
                              hipStream_t st) {
    if (nf <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_seen_append, dim3(nf), dim3(kWave), 0, st, out, S, fresh, nf, m);
    return hipGetLastError();
}

hipError_t launch_append_cuts(const int32_t *cut_type, const double *cut_rhs, const double *cut_row, int nf, int stride,
                              int first, double *rows, double *rhs, double *coefT, const int32_t *slot_tab, int L,
                              int us, double *row_ub, int32_t *row_id, uint8_t *is_feas, hipStream_t st) {
    if (nf <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_append_cuts, dim3(nf), dim3(256), 0, st, cut_type, cut_rhs, cut_row, nf, stride, first, rows,
                       rhs, coefT, slot_tab, L, us, row_ub, row_id, is_feas);
    return hipGetLastError();
}

}  // namespace sgufp
