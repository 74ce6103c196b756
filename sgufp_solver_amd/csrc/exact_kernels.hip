// Optimality phase of exact DDs, cut-parallel (see ExactIO in dd_device.hpp).
//
// An exact DD below a deep B&B record is a small tree (at 1k arcs: ~7 layers, ~6.8k nodes,
// ~5k leaves) swept by every optimality cut of a pool that grows to tens of thousands of
// rows.  k_relax sweeps one cut (or a batch of four) at a time with the lanes over the
// nodes of a layer; for these records that costs ~20 us per cut and a 1 024-record B&B
// launch lasts as long as its slowest record.  Here the lanes are the
// cuts instead: every lane walks the same tree with its own cut's values, so there is no
// cross-lane traffic until the very end, the coefficient of a node is one conflict-free
// LDS read, and the records split into independent (record, leaf pass) work items that
// persistent workgroups pull from a counter -- no record can hold a launch up.
//
//   k_exact_cols  new optimality rows -> the cut-minor copy coefO (row n_slots + 1 = RHS)
//   k_exact_root  the root prefix (DD.cpp:3938-3949: RHS, then + coef per decision of the
//                 record's solution, in order) of every (pending record, cut): lanes = cuts
//   k_exact_leaf  per (record, pass of kLeafPass leaves): 8 waves x 16 leaves, lanes = cuts
//                 of a 64-cut block staged in LDS; per leaf the lane keeps the running
//                 std::min of its cuts' path values (DD.cpp:3975-3984) in a register; a
//                 pass stops early once every leaf is <= optimalLB (the outcome no longer
//                 changes); at the end a wave-min per leaf is the terminal weight
//
// Bit-exactness: every path value is the reference's fold, in its order -- the root
// prefix left to right, then parent + coefficient layer by layer (no add for a -1
// decision, DMIN below a dead in-arc) -- and each lane meets its cuts in pool order, so
// its running min keeps the first of equal values like std::min.  Across lanes equal
// minima can differ only in the sign of zero; a leaf whose minimum is zero and above
// optimalLB (so that the value can still be the DD's maximum) is re-scanned in pool order
// for the first cut that reaches it (first_zero).  The file is compiled with
// -ffp-contract=off like the rest.
#define SGUFP_MULTI_WAVE_TU 1
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dd_device.hpp"
#include "wave.hpp"

namespace sgufp {

#define EDMIN (-__DBL_MAX__)
#define EDMAX (__DBL_MAX__)

__device__ __forceinline__ int wid() { return (int)(threadIdx.x >> 6); }

// Coefficient slot of state rank r at DD layer k of a record (rank_slot in dd_kernels.hip):
// structural layer g + k - 1, coefficient layer len + k - 1 (they differ only for records
// whose solution vector is shorter than their global layer).  -1: no slot (coefficient 0).
__device__ __forceinline__ int slot_of(const NetDev &net, int g, int len, int aligned, int k, int r) {
    const int ls = g + k - 1;
    if (aligned) return net.slot_tab[ls * kMaxU + r];
    const int u = net.layer_universe[ls];
    if (u < 0 || r >= net.set_len[u]) return -1;
    const int dec = net.set_val[net.set_off[u] + r];
    if (dec < 0) return -1;
    const int lc = len + k - 1;
    const int j = net.arc_head[dec];
    for (int s = net.slot_off[lc]; s < net.slot_off[lc + 1]; s++)
        if (net.slot_head[s] == j) return s;
    return net.n_slots;
}

// ---- k_exact_cols: columns [first, no) of coefO from the pool rows ------------------------
// (reverse = 1: column j = o_order[no - 1 - j], o_order newest first; 0: column j = o_order[j])
__global__ void __launch_bounds__(256) k_exact_cols(const double *rows, const double *rhs, const int32_t *o_order,
                                                    int no, int first, int stride, int n_slots, int ostride,
                                                    double *coefO, int reverse) {
    const int j = first + (int)blockIdx.x;
    if (j >= no) return;
    const int row = reverse ? o_order[no - 1 - j] : o_order[j];
    const double *src = rows + (size_t)row * stride;
    for (int s = threadIdx.x; s < n_slots; s += blockDim.x) coefO[(size_t)s * ostride + j] = src[s];
    if (threadIdx.x == 0) {
        coefO[(size_t)n_slots * ostride + j] = 0.0;
        coefO[(size_t)(n_slots + 1) * ostride + j] = rhs[row];
    }
}

// ---- k_exact_root: R[i][s] = root prefix of pending record i under O cut s (newest first) --
// The records of a batch are mostly siblings of a few cutsets: neighbouring batch slots share
// long solution prefixes.  A work item is (a chunk of kRootChunk batch slots, a 64-cut block);
// its wave folds the chunk's pending records in slot order and keeps the partial sums at every
// st-th solution position (checkpoints in LDS): a record restarts from the last checkpoint inside
// its common prefix with the previous record.  The partial sums are the same additions in the same
// order, so the values are bit-identical to a fold from the RHS (DD.cpp:3938-3949).
constexpr int kFold = 16;
constexpr int kRootChunk = 64;        // batch slots per work item
constexpr int kRootCk = 24;           // checkpoints per wave
constexpr int kRootWaves = 4;
__global__ void __launch_bounds__(kRootWaves * kWave) k_exact_root(NetDev net, Scratch sc, ExactIO ex) {
    __shared__ int32_t item_s[kRootWaves];
    __shared__ double ck_s[kRootWaves][kRootCk][kWave];
    const int w = wid();
    const unsigned long long packed = ex.ctr[0];
    const int npend = (int)(packed >> 32);
    if (npend == 0) return;   // no exact record in the batch (a DD-only batch): no counter traffic
    const int nbs = (ex.nsc + kWave - 1) / kWave;              // screening blocks
    const int nblk = nbs + (ex.no + kWave - 1) / kWave;        // + pool blocks
    const int nchunk = (ex.nslots + kRootChunk - 1) / kRootChunk;
    const long long total = (long long)nchunk * nblk;
    const int ns = net.n_slots;
    // checkpoint stride: positions 0, st, 2 st, ... (ck[q] = the sum after q * st entries)
    const int st = max(kFold, ((sc.Lcap + kRootCk - 1) / kRootCk + kFold - 1) / kFold * kFold);
    double(&ck)[kRootCk][kWave] = ck_s[w];
    for (;;) {
        if (lane() == 0) item_s[w] = (int32_t)atomicAdd(&ex.ctr[1], 1ull);
        __builtin_amdgcn_wave_barrier();
        const long long item = (long long)uni(item_s[w]);
        __builtin_amdgcn_wave_barrier();
        if (item >= total) break;
        const int c = (int)(item / nblk), bb = (int)(item % nblk);
        const bool scr = bb < nbs;
        const int b = scr ? bb : bb - nbs;
        const int s = b * kWave + lane();
        const bool vc = s < (scr ? ex.nsc : ex.no);
        const int col = vc ? (scr ? s : ex.no - 1 - s) : 0;
        const GBL double *cm = scr ? ex.coefS : ex.coefO;
        const size_t cs = scr ? (size_t)kExactScreen : (size_t)ex.ostride;
        const double rhs = cm[(size_t)(ns + 1) * cs + col];
        const GBL int32_t *prs = nullptr;   // previous record's slots and length, valid checkpoints
        int plen = 0, qvalid = 0;
        const int s0 = c * kRootChunk, s1 = min(ex.nslots, s0 + kRootChunk);
        for (int slot = s0; slot < s1; slot++) {
            const int i = uni(ex.pidx[slot]);
            if (i < 0) continue;
            const int len = uni(sc.meta[(size_t)slot * 8 + 1]);
            const GBL int32_t *rs = sc.rslot + (size_t)slot * sc.Lcap;
            // common prefix with the previous record (64 positions per step)
            int lcp = 0;
            if (prs) {
                const int m = min(len, plen);
                lcp = m;
                for (int t0 = 0; t0 < m; t0 += kWave) {
                    const int t = t0 + lane();
                    const uint64_t diff = __ballot(t < m && rs[t] != prs[t]);
                    if (diff) {
                        lcp = t0 + (int)(__ffsll((unsigned long long)diff) - 1);
                        break;
                    }
                }
            }
            const int q0 = min(lcp / st, qvalid);
            double v = q0 > 0 ? ck[q0][lane()] : rhs;
            for (int t0 = q0 * st; t0 < len; t0 += kFold) {
                if (t0 % st == 0 && t0 / st < kRootCk) ck[t0 / st][lane()] = v;
                double x[kFold];
                bool ok[kFold];
#pragma unroll
                for (int j = 0; j < kFold; j++) {
                    const int t = t0 + j;
                    const int sl = t < len ? uni(rs[t]) : -1;
                    ok[j] = sl >= 0;
                    x[j] = cm[(size_t)(ok[j] ? sl : ns) * cs + col];
                }
                sched_fence();
#pragma unroll
                for (int j = 0; j < kFold; j++)
                    if (ok[j]) v = v + x[j];
            }
            // checkpoints 0 .. floor(len / st) hold this record's prefix (the one at len itself
            // only when len is a multiple of st: written here)
            if (len % st == 0 && len / st < kRootCk) ck[len / st][lane()] = v;
            qvalid = min(len / st, kRootCk - 1);
            prs = rs;
            plen = len;
            if (vc) {
                if (scr) ex.RS[(size_t)i * kExactScreen + s] = v;
                else ex.R[(size_t)i * ex.ostride + s] = v;
            }
        }
    }
}

// ---- k_exact_leaf ------------------------------------------------------------------------
// Per-wave tables of one pass: for leaf j of the wave and DD layer k (1 .. T-1) the rank of
// the decision into its ancestor at layer k (bits 0-5) and that node's in-arc alive flag
// (bit 7); dv[j] = the first layer where leaf j's ancestors differ from leaf j-1's.
struct LeafWave {
    uint8_t info[kLeavesPerWave][kExactMaxT];
    uint8_t dv[kLeavesPerWave];
};

struct LeafShared {
    double C[kExactMaxEntries][kWave];   // staged coefficients of a 64-cut block, row = (k-1)*us + r
    int32_t stab[kExactMaxEntries];      // their slots (-1: no coefficient)
    LeafWave lw[kLeafWaves];
    double vb[kLeafWaves][kExactMaxT - 1][kWave];   // ancestor values of the current leaf (layers 0 .. T - 2), per wave
    int32_t item, flags[kLeafWaves];
};

// running min of a lane's cuts meeting a path value (std::min(w, v): keeps w on ties)
__device__ __forceinline__ double rmin(double w, double v) { return (v < w) ? v : w; }

// ancestors of leaf j (wave-local) from layer dj down to the leaf's parent, values in vb;
// returns the parent value
__device__ __forceinline__ double walk_down(LeafShared &S, int w, int j, int dj, int T, int us, double root) {
    double prev = (dj <= 1) ? root : S.vb[w][dj - 1][lane()];
    for (int k = dj; k < T - 1; k++) {
        const uint32_t b = uni((uint32_t)S.lw[w].info[j][k]);
        const uint32_t r = b & 63u;
        const double x = !(b & 128u) ? EDMIN : (r ? prev + S.C[(k - 1) * us + r][lane()] : prev);
        S.vb[w][k][lane()] = x;
        prev = x;
    }
    return prev;
}

// the first cut in pool order whose value at the leaf equals the leaf's minimum zero: its
// bits (the sign std::min's sequential fold keeps; the screening columns repeat pool cuts,
// so they add no value of their own).  Coefficients straight from coefO.
__device__ double first_zero(const NetDev &net, const ExactIO &ex, LeafShared &S, int w, int j, int T, int us, int i) {
    const int nblk = (ex.no + kWave - 1) / kWave;
    for (int b = 0; b < nblk; b++) {
        const int s = b * kWave + lane();
        const bool vc = s < ex.no;
        const int oidx = vc ? ex.no - 1 - s : 0;
        double v = vc ? ex.R[(size_t)i * ex.ostride + s] : 1.0;
        for (int k = 1; k < T; k++) {
            const uint32_t bb = uni((uint32_t)S.lw[w].info[j][k]);
            const uint32_t r = bb & 63u;
            const int sl = S.stab[(k - 1) * us + (int)r];
            const double c = (sl >= 0 && vc) ? ex.coefO[(size_t)sl * ex.ostride + oidx] : 0.0;
            v = !(bb & 128u) ? EDMIN : (r ? v + c : v);
        }
        const uint64_t hit = __ballot(vc && v == 0.0);
        if (hit) return lane_get(v, (int)(__ffsll((unsigned long long)hit) - 1));
    }
    return 0.0;
}

#ifndef SGUFP_LEAF_MIN_WAVES
#define SGUFP_LEAF_MIN_WAVES 6   // three 8-wave workgroups per CU (VGPRs <= 85)
#endif
__global__ void __launch_bounds__(kLeafWaves * kWave, SGUFP_LEAF_MIN_WAVES) k_exact_leaf(NetDev net, Scratch sc, ExactIO ex, double incumbent) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    LeafShared &S = *(LeafShared *)smem_raw;
    const int w = wid();
    const int tid = (int)threadIdx.x;
    const unsigned long long packed = ex.ctr[0];
    const int npend = (int)(packed >> 32);
    const uint32_t total = (uint32_t)(packed & 0xFFFFFFFFull);
    const int nbs = (ex.nsc + kWave - 1) / kWave;              // screening blocks first
    const int nblk = nbs + (ex.no + kWave - 1) / kWave;
    const int us = sc.us;
    for (;;) {
        if (tid == 0) S.item = (int32_t)atomicAdd(&ex.ctr[2], 1ull);
        __syncthreads();
        const uint32_t item = (uint32_t)uni(S.item);
        __syncthreads();
        if (item >= total) break;
        // record of the item: the last pending record whose first pass is <= item
        int lo = 0, hi = npend - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (ex.pend_base[mid] <= item) lo = mid;
            else hi = mid - 1;
        }
        const int i = lo;
        const int slot = ex.pend_slot[i];
        const int pass = (int)(item - ex.pend_base[i]);
        const GBL int32_t *meta = sc.meta + (size_t)slot * 8;
        const int g = uni(meta[0]), len = uni(meta[1]), T = uni(meta[2]), aligned = uni(meta[4]);
        const GBL uint32_t *lay = sc.lay + (size_t)slot * sc.Tcap * 5;
        const uint32_t lnoff = uni(lay[T - 1]), lnn = uni(lay[sc.Tcap + T - 1]);
        const size_t N = (size_t)slot * sc.Ncap;
        const int E = (T - 1) * us;
        for (int e = tid; e < E; e += kLeafWaves * kWave) {
            const int k = e / us + 1, r = e % us;
            S.stab[e] = r == 0 ? -1 : slot_of(net, g, len, aligned, k, r);
        }
        // this wave's leaves: ancestry tables and alive mask
        const int j0 = pass * kLeafPass + w * kLeavesPerWave;
        const int cnt = max(0, min(kLeavesPerWave, (int)lnn - j0));
        uint32_t alive = 0;
        {
            const int j = lane();
            bool al = false;
            uint32_t anc[kExactMaxT];
            if (j < cnt) {
                uint32_t node = lnoff + (uint32_t)(j0 + j);
                al = (sc.nflag[N + node] & kAlive) != 0;
#pragma unroll
                for (int k = kExactMaxT - 1; k >= 1; k--) {
                    if (k < T) {
                        const uint32_t t = sc.ntopo[N + node];
                        const uint8_t f = sc.nflag[N + node];
                        S.lw[w].info[j][k] = (uint8_t)(((t >> kRankShift) & 63u) | ((f & kInAlive) ? 128u : 0u));
                        anc[k] = node;
                        node = lay[k - 1] + (t & kParentMask);
                    }
                }
            }
            // first layer where this leaf's ancestors leave the previous leaf's
            int dv = 1;
#pragma unroll
            for (int k = 1; k < kExactMaxT; k++) {
                if (k < T - 1) {
                    const uint32_t prev = (uint32_t)__shfl_up((int)anc[k], 1, kWave);
                    if (j > 0 && j < cnt && prev == anc[k] && dv == k) dv = k + 1;
                }
            }
            if (j < cnt) S.lw[w].dv[j] = (uint8_t)((j == 0) ? 1 : dv);
            alive = (uint32_t)__ballot(j < cnt && al);
        }
        __syncthreads();
        // per leaf, in scalar registers for the whole pass: 16 bits = the LDS row of its
        // last-layer coefficient (bits 0-6; kRowNoAdd: a -1 decision, kRowDead: in-arc dead) |
        // dv << 8 (the first layer to recompute for it)
        // (lane j holds leaf j's word; the leaf loop reads it with v_readlane)
        constexpr uint32_t kRowNoAdd = 127u, kRowDead = 126u;
        uint32_t lp = 0;
        if (lane() < kLeavesPerWave) {
            const uint32_t b = S.lw[w].info[lane()][T - 1];
            const uint32_t r = b & 63u;
            const uint32_t row = !(b & 128u) ? kRowDead : (r ? (uint32_t)((T - 2) * us) + r : kRowNoAdd);
            lp = row | (uint32_t)S.lw[w].dv[lane()] << 8;
        }
        double m[kLeavesPerWave];
#pragma unroll
        for (int j = 0; j < kLeavesPerWave; j++) m[j] = EDMAX;
        uint32_t done = 0;
        int nb_done = 0;
        bool finished = false;   // every leaf of the pass <= optimalLB
        // lazy passes stop after ex.lazy blocks (the newest cuts); see ExactIO::lazy
        const int nlim = (ex.lazy > 0 && nbs == 0) ? min(nblk, ex.lazy) : nblk;
        for (int bb = 0; bb < nlim; bb++) {
            nb_done = bb + 1;
            const bool scr = bb < nbs;
            const int b = scr ? bb : bb - nbs;
            const int ncut = scr ? ex.nsc : ex.no;
            const GBL double *cm = scr ? ex.coefS : ex.coefO;
            const size_t cs = scr ? (size_t)kExactScreen : (size_t)ex.ostride;
            // stage the block's coefficients: row e = (layer, rank), lane = cut
            for (int x = tid; x < E * kWave; x += kLeafWaves * kWave) {
                const int e = x >> 6, l = x & (kWave - 1);
                const int s = b * kWave + l;
                const int sl = S.stab[e];
                S.C[e][l] = (sl >= 0 && s < ncut) ? cm[(size_t)sl * cs + (scr ? s : ncut - 1 - s)] : 0.0;
            }
            __syncthreads();
            const int s = b * kWave + lane();
            const bool vc = s < ncut;
            if (cnt > 0 && (done & alive) != alive) {
                const double root = vc ? (scr ? ex.RS[(size_t)i * kExactScreen + s] : ex.R[(size_t)i * ex.ostride + s]) : 0.0;
                const uint32_t open = alive & ~done;
                double par = root;
#pragma unroll
                for (int j = 0; j < kLeavesPerWave; j++) {
                    if (j < cnt) {
                        const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)lp, j);
                        const int dj = (int)(x >> 8);
                        if (dj < T - 1 || j == 0) par = walk_down(S, w, j, dj, T, us, root);
                        if ((open >> j) & 1u) {
                            const uint32_t row = x & 0x7Fu;
                            double v;
                            if (row == kRowDead) v = EDMIN;
                            else if (row == kRowNoAdd) v = par;
                            else v = par + S.C[row][lane()];
                            if (vc) m[j] = rmin(m[j], v);
                        }
                    }
                }
                // every fourth block (and the last): leaves some lane already took to <= optimalLB
                if ((bb & 3) == 3 || bb == nlim - 1) {
#pragma unroll
                    for (int j = 0; j < kLeavesPerWave; j++)
                        if ((open >> j) & 1u)
                            if (__ballot(vc && m[j] <= incumbent)) done |= 1u << j;
                }
            }
            if (lane() == 0) S.flags[w] = ((done & alive) == alive) ? 1 : 0;
            __syncthreads();
            int all = 1;
#pragma unroll
            for (int q = 0; q < kLeafWaves; q++) all &= S.flags[q];
            __syncthreads();
            if (all) {
                finished = true;
                break;
            }
        }
        const bool lazy = !finished && nlim < nblk;
        if (tid == 0) atomicAdd(&ex.ctr[3], (unsigned long long)nb_done);   // diagnostics: cut blocks swept
        // terminal weights: min over the lanes
#pragma unroll
        for (int j = 0; j < kLeavesPerWave; j++) {
            if ((alive >> j) & 1u) {
                double v = lane_reduce<1>(m[j], [](double a, double b) { return rmin(a, b); });
                if (!lazy && v == 0.0 && v > incumbent && !((done >> j) & 1u)) v = first_zero(net, ex, S, w, j, T, us, i);
                if (lane() == 0) {
                    sc.tw[N + lnoff + (uint32_t)(j0 + j)] = v;
                    if (lazy) sc.nflag[N + lnoff + (uint32_t)(j0 + j)] |= kLazy;
                }
            }
        }
        __syncthreads();
    }
}

size_t exact_leaf_lds_bytes() { return sizeof(LeafShared); }

hipError_t launch_exact_cols(const double *rows, const double *rhs, const int32_t *o_order, int no, int first,
                             int stride, int n_slots, int ostride, double *coefO, int reverse, hipStream_t st) {
    if (no <= first) return hipSuccess;
    hipLaunchKernelGGL(k_exact_cols, dim3(no - first), dim3(256), 0, st, rows, rhs, o_order, no, first, stride, n_slots,
                       ostride, coefO, reverse);
    return hipGetLastError();
}

// the pending records' root folds and terminal weights; k_exact_fin (dd_kernels.hip) ends them
hipError_t launch_exact(const NetDev &net, const Scratch &sc, const ExactIO &ex, double incumbent, int cus,
                        hipStream_t st) {
    hipLaunchKernelGGL(k_exact_root, dim3(4 * cus), dim3(kRootWaves * kWave), 0, st, net, sc, ex);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_exact_leaf, dim3(4 * cus), dim3(kLeafWaves * kWave), sizeof(LeafShared), st, net, sc, ex,
                       incumbent);
    return hipGetLastError();
}

}  // namespace sgufp
