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

#include <climits>
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
    int32_t fle[kLeavesPerWave];   // non-exact entries: first cut <= optimalLB per leaf
};

template <int ROWS>
struct LeafSharedT {
    double C[ROWS][kWave];               // staged coefficients of a 64-cut block, row = (k-1)*us + r
    int32_t stab[ROWS];                  // their slots (-1: no coefficient)
    LeafWave lw[kLeafWaves];
    double vb[kLeafWaves][kExactMaxT - 1][kWave];   // ancestor values of the current leaf (layers 0 .. T - 2), per wave
    int32_t item, flags[2][kLeafWaves];   // per block, double-buffered (exact entries: one barrier fewer)
    uint32_t rmask[2];                   // rows (layer, rank) some leaf of the pass adds a coefficient of
};

// order-preserving key of a double (unsigned compare = numeric order, -0 below +0): the
// per-cut maxState of a non-exact record is an atomic max over its leaf passes
__device__ __forceinline__ unsigned long long nx_key(double x) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(x);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

// running min of a lane's cuts meeting a path value (std::min(w, v): keeps w on ties)
__device__ __forceinline__ double rmin(double w, double v) { return (v < w) ? v : w; }
// the same as one v_min_f64 (no NaN operands here; it may keep either of +0 / -0 on a tie, the
// callers re-scan zero minima in pool order): fmin would add two canonicalizing v_max_f64
__device__ __forceinline__ double vmin64(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// ancestors of leaf j (wave-local) from layer dj down to the leaf's parent, values in vb;
// returns the parent value
#ifndef SGUFP_LEAF_INFOREG
#define SGUFP_LEAF_INFOREG 1   // the walk's per-layer info bytes from registers (v_readlane), not LDS
#endif
template <class LeafShared>
__device__ __forceinline__ double walk_down(LeafShared &S, int w, int j, int dj, int T, int us, double root, uint32_t ilo,
                                            uint32_t ihi) {
    double prev = (dj <= 1) ? root : S.vb[w][dj - 1][lane()];
    for (int k = dj; k < T - 1; k++) {
#if SGUFP_LEAF_INFOREG
        static_assert(kExactMaxT <= 9, "layers 1-8 in two packed words");
        // lane j packs leaf j's info bytes of layers 1-4 (ilo) and 5-7 (ihi): a scalar read with
        // no LDS round trip before the coefficient's
        const uint32_t src = k <= 4 ? ilo : ihi;
        const uint32_t b = ((uint32_t)__builtin_amdgcn_readlane((int)src, j) >> (8 * ((k - 1) & 3))) & 0xFFu;
#else
        const uint32_t b = uni((uint32_t)S.lw[w].info[j][k]);
#endif
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
template <class LeafShared>
__device__ double first_zero(const NetDev &net, const ExactIO &ex, LeafShared &S, int w, int j, int T, int us, int i,
                             int s0 = 0) {
    const int nblk = (ex.no + kWave - 1) / kWave;
    for (int b = s0 / kWave; b < nblk; b++) {
        const int s = b * kWave + lane();
        const bool vc = s < ex.no && s >= s0;
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

#ifndef SGUFP_LEAF_REGS
#define SGUFP_LEAF_REGS 0   // 1: ancestor values in registers (spills at the 6-wave bound; measured slower)
#endif
#ifndef SGUFP_LEAF_PIPE
#define SGUFP_LEAF_PIPE 1   // the next cut block's coefficients load while this one is swept
#endif
#ifndef SGUFP_LEAF_ROWMASK
#define SGUFP_LEAF_ROWMASK 1   // stage only the rows the pass's leaves add (0: all rows, A/B)
#endif
#ifndef SGUFP_LEAF_BALANCE
#define SGUFP_LEAF_BALANCE 1   // a pass's leaves split evenly over its eight waves
#endif
#ifndef SGUFP_LEAF_FAST
#define SGUFP_LEAF_FAST 0   // 1: exact entries with lazy walks, mask tests, row offsets (measured: no gain)
#endif
#ifndef SGUFP_LEAF_LASTREG
#define SGUFP_LEAF_LASTREG 0   // 1: the last layer's rows of a block in registers (measured slower)
#endif
constexpr int kLastRegs = 4;   // ranks 1 .. 4 (C3 / C4 trees: 3; higher ranks read LDS)
#ifndef SGUFP_LEAF_MIN_WAVES
#define SGUFP_LEAF_MIN_WAVES 6   // three 8-wave workgroups per CU (VGPRs <= 85)
#endif
// Instantiations: NX = the non-exact entries (k_nx_dag's roots); ROWS = the staged rows, the
// narrow one (kExactMaxEntries, three workgroups per CU) for tails of (T - 1) x ustride <= 40
// rows, the wide one (kExactMaxEntriesWide, two per CU) for deeper or wider exact trees (C5's
// 6-rank universes: 7 x 6 = 42 rows).  Each pulls its items from its own counter and skips the
// entries of the others.
template <bool NX, int ROWS>
__global__ void __launch_bounds__(kLeafWaves * kWave, SGUFP_LEAF_MIN_WAVES) k_exact_leaf(NetDev net, Scratch sc, ExactIO ex, double incumbent) {
    using LeafShared = LeafSharedT<ROWS>;
    constexpr bool kWide = ROWS > kExactMaxEntries;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    LeafShared &S = *(LeafShared *)smem_raw;
    if (NX && ex.ctr[12] == 0) return;   // no non-exact entry in this batch
    const int w = uni(wid());   // (wave-uniform: the per-leaf tests below stay scalar branches)
    const int tid = (int)threadIdx.x;
    const unsigned long long packed = ex.ctr[0];
    const int npend = (int)(packed >> 32);
    const uint32_t total = (uint32_t)(packed & 0xFFFFFFFFull);
    const int nbs = (ex.nsc + kWave - 1) / kWave;              // screening blocks first
    const int nblk = nbs + (ex.no + kWave - 1) / kWave;
    const int us = sc.us;
    // open-leaf compaction (ExactIO::leaf_split): phase A sweeps blocks [0, split) of every pass,
    // phase B (pb) the rest over passes of open leaves
    const bool split = !NX && ex.leaf_split > 0 && ex.lazy == 0;
    const bool pb = split && ex.leaf_phase == 1;
    for (;;) {
        if (tid == 0) {
            S.item = (int32_t)atomicAdd(&ex.ctr[NX ? (ex.nx_ms ? 11 : 8) : (pb ? (kWide ? 17 : 16) : (kWide ? 10 : 2))], 1ull);
            S.rmask[0] = S.rmask[1] = 0u;
        }
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
        const int g = uni(meta[0]), len = uni(meta[1]), Tdd = uni(meta[2]), aligned = uni(meta[4]);
        // a non-exact record (k_nx_dag): the tree below its last width-1 layer k0, rooted at
        // the value k_nx_dag left in R; layers are counted from k0 (local layer k = DD layer
        // k0 + k), and the pass also reports per cut maxState and per leaf the first cut <=
        // optimalLB (nx_kernels.hip)
        const int k0 = ex.pkind ? uni(ex.pkind[i]) : -1;
        if ((k0 >= 0) != NX) continue;   // the other instantiation's entry
        constexpr bool nx = NX;
        // non-exact: k_relax applied pool positions [0, first) in order (tw holds their minima)
        const int first = nx ? uni(ex.nxh[(size_t)slot * 4 + 3]) : 0;
        // second non-exact launch (ex.nx_ms): only the maxState of the blocks after this pass
        // stopped (all its leaves <= optimalLB) up to the record's pruning position
        const bool ph2 = nx && ex.nx_ms;
        int bfrom = nx ? first / kWave : 0, bto = -1;
        if (ph2) {
            const int p = uni(ex.P[i]);
            const int lastpos = (p < ex.no ? p : ex.no) - 1;
            bfrom = uni(ex.pstop[item]) + 1;
            bto = lastpos / kWave;
            if (lastpos < first || bfrom > bto) continue;
        }
        const int kb = nx ? k0 : 0;
        const int T = Tdd - kb;
        const int E = (T - 1) * us;
        if (!NX && (E > kExactMaxEntries) != kWide) continue;   // the other row count's entry
        // phase B: this item is chunk `pass` of the record's open list
        const int nopen = pb ? uni(ex.open_cnt[i]) : 0;
        if (pb && pass * kLeafPass >= nopen) continue;
        const GBL int32_t *olist = pb ? ex.open_list + (size_t)ex.pend_base[i] * kLeafPass : nullptr;
        const GBL uint32_t *lay = sc.lay + (size_t)slot * sc.Tcap * 5;
        const uint32_t lnoff = uni(lay[Tdd - 1]), lnn = uni(lay[sc.Tcap + Tdd - 1]);
        const size_t N = (size_t)slot * sc.Ncap;
        for (int e = tid; e < E; e += kLeafWaves * kWave) {
            const int k = e / us + 1, r = e % us;
            S.stab[e] = r == 0 ? -1 : slot_of(net, g, len, aligned, kb + k, r);
        }
        // this wave's leaves: ancestry tables and alive mask.  A pass's n leaves are split into
        // eight runs of ceil(n / 8) consecutive leaves (not 16 for the first waves and none for the
        // rest): a partial pass -- every record's last one, and phase B's open lists are mostly
        // short -- keeps all waves busy, and each barrier waits for ceil(n / 8) leaves, not 16
#if SGUFP_LEAF_BALANCE
        const int npass = min(kLeafPass, (pb ? nopen : (int)lnn) - pass * kLeafPass);
        const int per = (npass + kLeafWaves - 1) / kLeafWaves;
        const int j0 = pass * kLeafPass + w * per;
        const int cnt = uni(max(0, min(per, npass - w * per)));
#else
        const int j0 = pass * kLeafPass + w * kLeavesPerWave;
        const int cnt = uni(max(0, min(kLeavesPerWave, (pb ? nopen : (int)lnn) - j0)));
#endif
        // lane j's leaf (index among the record's leaves): consecutive in phase A, from the open
        // list in phase B (in the order phase A's passes appended them)
        const int lid = lane() < cnt ? (pb ? olist[j0 + lane()] : j0 + lane()) : 0;
        uint32_t alive = 0;
        {
            const int j = lane();
            bool al = false;
            uint32_t anc[kExactMaxT];
            uint64_t used = 0;   // rows this leaf's path adds: (layer, rank) with an alive in-arc, rank > 0
            if (j < cnt) {
                uint32_t node = lnoff + (uint32_t)lid;
                al = (sc.nflag[N + node] & kAlive) != 0;
#pragma unroll
                for (int k = kExactMaxT - 1; k >= 1; k--) {
                    if (k < T) {
                        const uint32_t t = sc.ntopo[N + node];
                        const uint8_t f = sc.nflag[N + node];
                        const uint32_t r = (t >> kRankShift) & 63u;
                        S.lw[w].info[j][k] = (uint8_t)(r | ((f & kInAlive) ? 128u : 0u));
                        if ((f & kInAlive) && r) used |= 1ull << ((k - 1) * us + (int)r);
                        anc[k] = node;
                        node = lay[kb + k - 1] + (t & kParentMask);
                    }
                }
            }
            used = (uint64_t)lane_reduce<1>((int64_t)used, [](int64_t a, int64_t b) { return a | b; });
            if (lane() == 0) {
                if ((uint32_t)used) atomicOr(&S.rmask[0], (uint32_t)used);
                if ((uint32_t)(used >> 32)) atomicOr(&S.rmask[1], (uint32_t)(used >> 32));
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
        // leaf j's info bytes in lane j's registers (walk_down reads them with v_readlane)
        uint32_t ilo = 0, ihi = 0;
#if SGUFP_LEAF_INFOREG
        if (lane() < kLeavesPerWave) {
#pragma unroll
            for (int k = 1; k < kExactMaxT; k++) {
                if (k < T) {
                    const uint32_t b = (uint32_t)S.lw[w].info[lane()][k];
                    if (k <= 4) ilo |= b << (8 * (k - 1));
                    else ihi |= b << (8 * (k - 5));
                }
            }
        }
#endif
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
#if SGUFP_LEAF_FAST
        // exact entries' leaf loop (below): per pass, wave-uniform masks of the leaves that start a
        // walk (a new parent) and of the leaves whose last arc adds nothing (dead in-arc, -1
        // decision), and per leaf the byte offset of its coefficient row in S.C
        const uint32_t walkm = uni((uint32_t)__ballot(lane() < cnt && (lane() == 0 || (int)(lp >> 8) < T - 1)));
        const uint32_t specm = uni((uint32_t)__ballot(lane() < cnt && (lp & 0x7Fu) >= kRowDead));
        const uint32_t lpo = (lp & 0x7Fu) < kRowDead ? (lp & 0x7Fu) * (uint32_t)(kWave * sizeof(double)) : 0u;
#endif
        double m[kLeavesPerWave];
#pragma unroll
        for (int j = 0; j < kLeavesPerWave; j++) m[j] = EDMAX;
        uint32_t done = 0;
        int nb_done = 0;
        bool finished = false;   // every leaf of the pass <= optimalLB
        // non-exact: pool order only (no screening columns, no lazy passes); a pass stops once
        // its leaves are <= optimalLB, and the second launch completes the maxState of the later
        // blocks before the record's pruning position (every leaf's value at every such cut)
        const int nbs_r = nx ? 0 : nbs;
        const int nblk_r = nx ? (ex.no + kWave - 1) / kWave : nblk;
        // lazy passes stop after ex.lazy blocks (the newest cuts); see ExactIO::lazy
        const int nlim = (!nx && ex.lazy > 0 && nbs == 0) ? min(nblk, ex.lazy) : nblk_r;
        // non-exact: per leaf the first cut (pool position) with value <= optimalLB; a leaf whose
        // in-order minimum already is counts as done before the phase
        double twold = EDMAX;
        if (!nx && !pb && lane() == 0) atomicAdd(&ex.ctr[15], (unsigned long long)__popc(alive));
        if (pb && lane() < cnt) twold = sc.tw[N + lnoff + (uint32_t)lid];   // phase A's partial minimum
        if (nx) {
            const bool al = lane() < cnt && ((alive >> lane()) & 1u);
            if (al) twold = sc.tw[N + lnoff + (uint32_t)(j0 + lane())];
            const bool pre = al && twold <= incumbent;
            done = (uint32_t)__ballot(pre);
            if (lane() < kLeavesPerWave) S.lw[w].fle[lane()] = pre ? 0 : INT_MAX;
        }
        int bb_last = -1;
        // phase A stops after the split blocks, phase B starts there
        const int bsplit = split ? min(nlim, ex.leaf_split) : nlim;
        if (pb) bfrom = bsplit;
        const int bend = ph2 ? bto + 1 : (split && !pb ? bsplit : nlim);
#if SGUFP_LEAF_PIPE
        // a block's coefficients are loaded into registers while the previous block is swept
        // (every load of a block issued at once), stored to LDS at the top of its iteration --
        // the end of the previous iteration's barriers found every wave done with the old ones.
        // Only the rows some leaf of the pass adds are staged (S.rmask: the pass's 128 leaves
        // share their upper ancestors, so about 14 of the C4 trees' 24 coefficient rows): the
        // others are never read.  Wave w stages the pass's used rows w, w + 8, ... (in row
        // order), one row per 64 lanes, the same in every block.
        constexpr int kSU = (ROWS * kWave + kLeafWaves * kWave - 1) / (kLeafWaves * kWave);
        double stg[kSU];
        int srow[kSU], sslot[kSU];
        {
            // (a used row with no coefficient slot is staged as zeros, as before)
#if SGUFP_LEAF_ROWMASK
            uint64_t mm = (uint64_t)S.rmask[0] | (uint64_t)S.rmask[1] << 32;
#else
            uint64_t mm = E >= 64 ? ~0ull : (1ull << E) - 1ull;   // A/B: every row of the tree
#endif
            // the (w + 8 u)-th set bit of mm for u = 0 .. kSU - 1 (uniform scalar walk, once a pass)
            for (int c = 0; c < w && mm; c++) mm &= mm - 1;
#pragma unroll
            for (int u = 0; u < kSU; u++) {
                srow[u] = mm ? (int)__builtin_ctzll(mm) : -1;
                sslot[u] = srow[u] >= 0 ? uni(S.stab[srow[u]]) : -1;
#pragma unroll
                for (int c = 0; c < kLeafWaves; c++) mm &= mm - 1;
            }
        }
        auto stage_load = [&](int bbx) {
            const bool scrx = bbx < nbs_r;
            const int bx = scrx ? bbx : bbx - nbs_r;
            const int ncx = scrx ? ex.nsc : ex.no;
            const GBL double *cmx = scrx ? ex.coefS : ex.coefO;
            const size_t csx = scrx ? (size_t)kExactScreen : (size_t)ex.ostride;
            const int sx = bx * kWave + lane();
#pragma unroll
            for (int u = 0; u < kSU; u++)
                stg[u] = (sslot[u] >= 0 && sx < ncx) ? cmx[(size_t)sslot[u] * csx + (scrx ? sx : ncx - 1 - sx)] : 0.0;
        };
        if (bfrom < bend) stage_load(bfrom);
#endif
#ifdef SGUFP_LEAF_CLOCKS
        // diagnostics build: per wave the cycles of (staging + first barrier, leaf loop, the rest)
        uint64_t ck[3] = {0, 0, 0}, ct = clock64();
#define LEAF_CK(x) { const uint64_t c2 = clock64(); ck[x] += c2 - ct; ct = c2; }
#else
#define LEAF_CK(x)
#endif
        for (int bb = bfrom; bb < bend; bb++) {
            bb_last = bb;
            nb_done = bb + 1;
            const bool scr = bb < nbs_r;
            const int b = scr ? bb : bb - nbs_r;
            const int ncut = scr ? ex.nsc : ex.no;
#if SGUFP_LEAF_PIPE
#pragma unroll
            for (int u = 0; u < kSU; u++)
                if (srow[u] >= 0) S.C[srow[u]][lane()] = stg[u];
            __syncthreads();
            LEAF_CK(0);
            if (bb + 1 < bend) stage_load(bb + 1);
#else
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
#endif
            const int s = b * kWave + lane();
            const bool vc = s < ncut && s >= first;
            double ms = -INFINITY;   // non-exact: max over this wave's alive leaves, this lane's cut
            if (cnt > 0 && (nx || (done & alive) != alive)) {
#if SGUFP_LEAF_LASTREG
                // the last layer's rows (ranks 1 .. kLastRegs) of this block in registers, read once:
                // a leaf's own coefficient is then a select, not an LDS round trip per leaf
                const int lrow1 = (T - 2) * us + 1;
                double cl[kLastRegs];
#pragma unroll
                for (int q = 0; q < kLastRegs; q++) cl[q] = (q + 1 < us) ? S.C[lrow1 + q][lane()] : 0.0;
#endif
                // exact entries: a lane past the pool's end starts at +inf, so its values leave every
                // running minimum alone (a dead path gives DOUBLE_MIN on every lane, valid or not)
                // and the leaf loop below needs no per-lane condition -- no exec-mask switching
                const double root = vc ? (scr ? ex.RS[(size_t)i * kExactScreen + s] : ex.R[(size_t)i * ex.ostride + s])
                                       : (nx ? 0.0 : INFINITY);
                // (wave-uniform: in scalar registers, so the leaf tests below are scalar branches)
                const uint32_t open = uni(alive & ~done);
                const uint32_t need = uni(nx ? alive : open);
                double par = root;
#if SGUFP_LEAF_FAST
                if constexpr (!NX) {
                    // exact entries: walks only for open leaves (a skipped leaf's walk is owed to the
                    // next open one: it starts at the shallowest first-differing layer since the last
                    // walk, `pend`), scalar-branch tests on the masks, the row read at a precomputed
                    // offset.  The same adds in the same order as the general loop below.
                    const LDS char *cbase = (const LDS char *)&S.C[0][lane()];
                    int pend = T - 1;
#if SGUFP_LEAF_FAST == 2
                    // pairs of leaves: both coefficient reads are issued before either leaf's walk or
                    // add (they do not depend on the parent's value), one LDS round trip per pair
                    static_assert(kLeavesPerWave % 2 == 0, "leaf pairs");
#pragma unroll
                    for (int jp = 0; jp < kLeavesPerWave; jp += 2) {
                        const uint32_t o2 = (open >> jp) & 3u;
                        if (!o2 && !((walkm >> jp) & 3u)) continue;
                        double c2[2] = {0.0, 0.0};
#pragma unroll
                        for (int q = 0; q < 2; q++)
                            if (((o2 >> q) & 1u) && !((specm >> (jp + q)) & 1u))
                                c2[q] = *(const LDS double *)(cbase + (uint32_t)__builtin_amdgcn_readlane((int)lpo, jp + q));
#pragma unroll
                        for (int q = 0; q < 2; q++) {
                            const int j = jp + q;
                            if ((o2 >> q) & 1u) {
                                if (((walkm >> j) & 1u) || pend < T - 1) {
                                    const int dj = j == 0 ? 1 : (int)((uint32_t)__builtin_amdgcn_readlane((int)lp, j) >> 8);
                                    par = walk_down(S, w, j, min(pend, dj), T, us, root, ilo, ihi);
                                    pend = T - 1;
                                }
                                double v;
                                if ((specm >> j) & 1u)
                                    v = ((uint32_t)__builtin_amdgcn_readlane((int)lp, j) & 0x7Fu) == kRowDead ? EDMIN : par;
                                else
                                    v = par + c2[q];
                                m[j] = vmin64(m[j], v);
                            } else if ((walkm >> j) & 1u) {
                                const int dj = j == 0 ? 1 : (int)((uint32_t)__builtin_amdgcn_readlane((int)lp, j) >> 8);
                                pend = min(pend, dj);
                            }
                        }
                    }
                    if (false)
#endif
#pragma unroll
                    for (int j = 0; j < kLeavesPerWave; j++) {
                        if ((open >> j) & 1u) {
                            if (((walkm >> j) & 1u) || pend < T - 1) {
                                const int dj = j == 0 ? 1 : (int)((uint32_t)__builtin_amdgcn_readlane((int)lp, j) >> 8);
                                par = walk_down(S, w, j, min(pend, dj), T, us, root, ilo, ihi);
                                pend = T - 1;
                            }
                            double v;
                            if ((specm >> j) & 1u) {
                                v = ((uint32_t)__builtin_amdgcn_readlane((int)lp, j) & 0x7Fu) == kRowDead ? EDMIN : par;
                            } else {
                                const uint32_t off = (uint32_t)__builtin_amdgcn_readlane((int)lpo, j);
                                v = par + *(const LDS double *)(cbase + off);
                            }
                            m[j] = vmin64(m[j], v);
                        } else if ((walkm >> j) & 1u) {
                            const int dj = j == 0 ? 1 : (int)((uint32_t)__builtin_amdgcn_readlane((int)lp, j) >> 8);
                            pend = min(pend, dj);
                        }
                    }
                } else
#endif
                {
#if SGUFP_LEAF_REGS
                // ancestor values in registers (anc[k] = local layer k): a leaf recomputes the
                // levels from its first ancestor that differs from the previous leaf's (dv), the
                // same adds in the same order as walk_down, without its LDS round trip per level
                double anc[kExactMaxT - 1];
                anc[0] = root;
#pragma unroll
                for (int k = 1; k < kExactMaxT - 1; k++) anc[k] = root;
#endif
#pragma unroll
                for (int j = 0; j < kLeavesPerWave; j++) {
                    if (j < cnt) {
                        const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)lp, j);
                        const int dj = (int)(x >> 8);
#if SGUFP_LEAF_REGS
                        if (dj < T - 1 || j == 0) {
#pragma unroll
                            for (int k = 1; k < kExactMaxT - 1; k++) {
                                if (k < T - 1 && k >= dj) {
                                    const uint32_t bq = uni((uint32_t)S.lw[w].info[j][k]);
                                    const uint32_t r = bq & 63u;
                                    anc[k] = !(bq & 128u) ? EDMIN : (r ? anc[k - 1] + S.C[(k - 1) * us + r][lane()] : anc[k - 1]);
                                }
                            }
                            par = anc[0];
#pragma unroll
                            for (int k = 1; k < kExactMaxT - 1; k++) par = (k == T - 2) ? anc[k] : par;
                        }
#else
                        if (dj < T - 1 || j == 0) par = walk_down(S, w, j, dj, T, us, root, ilo, ihi);
#endif
                        if ((need >> j) & 1u) {
                            const uint32_t row = x & 0x7Fu;
                            double v;
                            if (row == kRowDead) v = EDMIN;
                            else if (row == kRowNoAdd) v = par;
                            else {
#if SGUFP_LEAF_LASTREG
                                const uint32_t q = row - (uint32_t)lrow1;   // rank - 1 (wave-uniform)
                                double c;
                                if (q < (uint32_t)kLastRegs) {
                                    c = cl[0];
#pragma unroll
                                    for (int qq = 1; qq < kLastRegs; qq++) c = (q == (uint32_t)qq) ? cl[qq] : c;
                                } else {
                                    c = S.C[row][lane()];
                                }
                                v = par + c;
#else
                                v = par + S.C[row][lane()];
#endif
                            }
                            if (nx) {
                                if (!ph2 && vc && ((open >> j) & 1u)) m[j] = rmin(m[j], v);
                            } else if ((open >> j) & 1u) {
                                // v_min_f64: it may keep either of +0 / -0 where std::min keeps the
                                // first; a zero minimum above optimalLB is re-scanned in pool order
                                // (first_zero) as it is across lanes, so the result is the same
                                m[j] = vmin64(m[j], v);
                            }
                            if (nx) {
                                ms = (vc && v > ms) ? v : ms;
                                if (!ph2 && ((open >> j) & 1u)) {
                                    const uint64_t hit = __ballot(vc && v <= incumbent);
                                    if (hit) {
                                        if (lane() == 0) S.lw[w].fle[j] = b * kWave + (int)(__ffsll((unsigned long long)hit) - 1);
                                        done |= 1u << j;
                                    }
                                }
                            }
                        }
                    }
                }
                }
                // every fourth block (and the last): leaves some lane already took to <= optimalLB
                if (!nx && ((bb & 3) == 3 || bb == nlim - 1)) {
#pragma unroll
                    for (int j = 0; j < kLeavesPerWave; j++)
                        if ((open >> j) & 1u)
                            if (__ballot(m[j] <= incumbent)) done |= 1u << j;   // (+inf on lanes past the pool)
                    // diagnostics: leaves still open after 16 / 64 blocks
                    if (lane() == 0 && (bb == 15 || bb == 63))
                        atomicAdd(&ex.ctr[bb == 15 ? 14 : 13], (unsigned long long)__popc(alive & ~done));
                }
            }
            LEAF_CK(1);
            if (nx) S.vb[w][0][lane()] = ms;   // free until the next block's walks
            if (lane() == 0) S.flags[bb & 1][w] = ((done & alive) == alive) ? 1 : 0;
            __syncthreads();
            int all = 1;
#pragma unroll
            for (int q = 0; q < kLeafWaves; q++) all &= S.flags[bb & 1][q];
            if (nx && w == 0 && vc) {
                double mx = -INFINITY;
#pragma unroll
                for (int q = 0; q < kLeafWaves; q++) mx = S.vb[q][0][lane()] > mx ? S.vb[q][0][lane()] : mx;
                if (mx != -INFINITY) atomicMax(&ex.MS[(size_t)i * ex.ostride + s], nx_key(mx));
            }
            // exact entries: the barrier above already found every wave done with this block's
            // coefficients (the next block's are stored after it) and the flags alternate
            // buffers, so only the non-exact maxState (vb, rewritten by the next walks) waits here
            if (nx) __syncthreads();
            LEAF_CK(2);
            if (all && !ph2) {
                finished = true;
                break;
            }
        }
        if (ph2) {
            __syncthreads();
            continue;
        }
        if (nx && tid == 0) ex.pstop[item] = bb_last;   // k_nx leaf phase 2 resumes after it
        if (nx) {
            // the pass's pruning position: max over its alive leaves of their first cut <= optimalLB
            const int fl = (lane() < kLeavesPerWave && ((alive >> lane()) & 1u)) ? S.lw[w].fle[lane()] : 0;
            const int pm = lane_reduce<1>(fl, [](int a, int b) { return a > b ? a : b; });
            if (lane() == 0 && cnt > 0) atomicMax(&ex.P[i], pm);
        }
        const bool lazy = !nx && !finished && nlim < nblk;
        // phase A with blocks left: the open leaves' partial minima go to tw and the leaves to
        // the record's open list (no zero re-scan yet: phase B decides the final value)
        const bool to_b = split && !pb && !finished && bsplit < nlim;
        if (tid == 0) {   // diagnostics: cut blocks swept; staged row-blocks (the byte model)
            const int nbs_item = max(0, nb_done - bfrom);   // (phase B: bfrom = bsplit)
            atomicAdd(&ex.ctr[pb ? 19 : 3], (unsigned long long)max(0, nb_done - (pb ? bsplit : 0)));
            const uint64_t rm = (uint64_t)S.rmask[0] | (uint64_t)S.rmask[1] << 32;
            atomicAdd(&ex.ctr[20], (unsigned long long)(SGUFP_LEAF_ROWMASK ? __popcll(rm) : E) * (unsigned long long)nbs_item);
            atomicAdd(&ex.ctr[21], (unsigned long long)nbs_item);
        }
#ifdef SGUFP_LEAF_CLOCKS
        if (lane() == 0)
            for (int x = 0; x < 3; x++) atomicAdd(&ex.ctr[22 + x], (unsigned long long)ck[x]);
#endif
#undef LEAF_CK
        // terminal weights: min over the lanes
        uint32_t openb = 0;
#pragma unroll
        for (int j = 0; j < kLeavesPerWave; j++) {
            if ((alive >> j) & 1u) {
                double v = lane_reduce<1>(m[j], [](double a, double b) { return rmin(a, b); });
                if (nx) {
                    // std::min(w, v) over the phase's cuts after the in-order ones: the old weight
                    // stays on ties; a new zero minimum takes the first zero's sign
                    const double old = lane_get(twold, j);
                    if (!(v < old)) v = old;
                    else if (v == 0.0 && v > incumbent && !((done >> j) & 1u)) v = first_zero(net, ex, S, w, j, T, us, i, first);
                } else if (pb) {
                    // phase A's minimum covers the earlier blocks (pool order: it stays on ties); a
                    // zero from either phase (lane minima of equal values differ only in the sign of
                    // zero) is re-scanned in pool order from the first cut
                    const double old = lane_get(twold, j);
                    if (!(v < old)) v = old;
                    if (v == 0.0 && v > incumbent) v = first_zero(net, ex, S, w, j, T, us, i);
                } else if (to_b && v > incumbent) {
                    openb |= 1u << j;
                } else if (!lazy && v == 0.0 && v > incumbent && !((done >> j) & 1u))
                    v = first_zero(net, ex, S, w, j, T, us, i);
                const int lj = __builtin_amdgcn_readlane(lid, j);
                if (lane() == 0) {
                    sc.tw[N + lnoff + (uint32_t)lj] = v;
                    if (lazy) sc.nflag[N + lnoff + (uint32_t)lj] |= kLazy;
                }
            }
        }
        if (to_b && openb) {
            int base = 0;
            if (lane() == 0) {
                base = atomicAdd(&ex.open_cnt[i], __popc(openb));
                atomicAdd(&ex.ctr[18], (unsigned long long)__popc(openb));
            }
            base = __builtin_amdgcn_readfirstlane(base);
            const int j = lane();
            if (j < kLeavesPerWave && ((openb >> j) & 1u))
                ex.open_list[(size_t)ex.pend_base[i] * kLeafPass + base + __popc(openb & ((1u << j) - 1u))] = lid;
        }
        __syncthreads();
    }
}

size_t exact_leaf_lds_bytes() { return sizeof(LeafSharedT<kExactMaxEntries>); }

// ---- k_nx_dag: the DAG part of non-exact records (kNxPending) ------------------------------
// One wave per work item (pending record, block of kNxCuts cuts), blocks outermost so that the
// waves in flight read the same coefO columns.  Lanes = 4 node groups x 16 cuts: the wave
// sweeps layers 1 .. k0 like dd_sweep, four nodes (or merged arcs) of a layer per step, from
// the packed topology words of the slot (tmir, build_stream: parent:7 | rank:5 | alive |
// in-arc alive; every layer below kg has <= 127 nodes), the previous and the current layer's
// values in this wave's LDS ([2][128][16] doubles), the layer's per-rank coefficients in
// registers (the next layer's load meanwhile).  A merged node folds its arcs per group, then
// the four partial (value, priority) maxima combine -- the fold is order-free given the
// priorities (DD.cpp:3952-3973).  Out: R = the value at k0 (the leaf passes' root), G = min
// over the width-1 pruning layers (3 <= k < T - 2) of fl(xmin - state2) lowered by 1e-12
// (|xmin| + |state2| + 1) (the reference tests fl(xmin + fl(maxState - state2)) <= thresh;
// the two differ by a few ulp of those magnitudes), -inf when such a layer holds a non-finite
// or DOUBLE_MIN/MAX value; MS cleared for the leaf passes' atomic max.
constexpr int kNxGroups = kWave / kNxCuts;
struct NxShared {
    double V[2][128][kNxCuts];
    int32_t item;
};

__device__ __forceinline__ double nx_pick(uint32_t r, const double (&cf)[kNxRanks]) {
    return r == 1u ? cf[0] : (r == 2u ? cf[1] : (r == 3u ? cf[2] : cf[3]));
}

__device__ void nx_dag_item(const NetDev &net, const Scratch &sc, const ExactIO &ex, NxShared &X, int i, int b) {
    const int slot = uni(ex.pend_slot[i]);
    const GBL int32_t *meta = sc.meta + (size_t)slot * 8;
    const int g = uni(meta[0]), len = uni(meta[1]), T = uni(meta[2]), aligned = uni(meta[4]);
    const GBL int32_t *h = ex.nxh + (size_t)slot * 4;
    const int k0 = uni(h[0]);
    const uint32_t Nn = (uint32_t)uni(h[1]), q0 = (uint32_t)uni(h[2]);
    const GBL uint32_t *lay = sc.lay + (size_t)slot * sc.Tcap * 5;
    const GBL uint16_t *tm = sc.tmir + (size_t)slot * sc.tmir_cap;
    const int q = lane() / kNxCuts, c = lane() % kNxCuts;
    const int s = b * kNxCuts + c;
    const bool vc = s < ex.no;
    const int col = vc ? ex.no - 1 - s : 0;
    const size_t os = (size_t)ex.ostride;
    auto load_coef = [&](int k, double (&dst)[kNxRanks]) {
#pragma unroll
        for (int r = 0; r < kNxRanks; r++) {
            const int sl = slot_of(net, g, len, aligned, k, r + 1);
            dst[r] = (sl >= 0 && vc) ? ex.coefO[(size_t)sl * os + col] : 0.0;
        }
    };
    double cf[kNxRanks], nf[kNxRanks];
    load_coef(1, cf);
    const double root = vc ? ex.R[(size_t)i * os + s] : 0.0;
    if (q == 0) X.V[0][0][c] = root;
    wave_lds_sync();
    int cur = 0;
    double gap = INFINITY, mag = 0.0;
    bool unc = false;
    auto summary = [&](double val, double xm) {
        if (!(fabs(val) < 1e300) || !(fabs(xm) < 1e300)) unc = true;
        else {
            gap = fmin(gap, xm - val);
            mag = fmax(mag, fabs(xm) + fabs(val));
        }
    };
    for (int k = 1; k <= k0; k++) {
        if (k < k0) load_coef(k + 1, nf);
        const uint32_t noff = uni(lay[k]), n = uni(lay[sc.Tcap + k]), nal = uni(lay[2 * sc.Tcap + k]);
        const uint32_t aoff = uni(lay[3 * sc.Tcap + k]), acnt = uni(lay[4 * sc.Tcap + k]);
        const bool summ = nal == 1u && k >= 3 && k <= T - 3;
        if (acnt == 0) {
            // exact layer: words of nodes lane and lane + 64 (n <= 127), node base + q per step
            const uint32_t w0 = lane() < (int)n ? (uint32_t)tm[noff + lane()] : 0u;
            const uint32_t w1 = lane() + kWave < (int)n ? (uint32_t)tm[noff + kWave + lane()] : 0u;
            for (uint32_t base = 0; base < n; base += kNxGroups) {
                const uint32_t idx = base + (uint32_t)q;
                const int src = (int)(idx & (kWave - 1));
                const uint32_t wa = (uint32_t)__shfl((int)w0, src, kWave), wb = (uint32_t)__shfl((int)w1, src, kWave);
                const uint32_t w = idx < (uint32_t)kWave ? wa : wb;
                const bool ok = idx < n && (w & kMirAlive);
                const uint32_t p = w & 127u, r = (w >> 7) & 31u;
                const double px = X.V[cur][p][c];
                const bool inal = (w & kMirIn) != 0;
                const double x = !inal ? EDMIN : (r ? px + nx_pick(r, cf) : px);
                if (ok) {
                    X.V[cur ^ 1][idx][c] = x;
                    if (summ) summary(x, !inal ? EDMAX : (r ? x : px + 0.0));
                }
            }
        } else {
            // merged node: its alive in-arcs, four per step, per-group (value, priority) fold
            double bv = 0.0, xmin = EDMAX;
            int bp = INT_MIN;
            for (uint32_t a0 = 0; a0 < acnt; a0 += kWave) {
                const uint32_t wl = a0 + lane() < acnt ? (uint32_t)tm[Nn + aoff + a0 + lane()] : 0u;
                const uint32_t m = min((uint32_t)kWave, acnt - a0);
                for (uint32_t base = 0; base < m; base += kNxGroups) {
                    const uint32_t j = base + (uint32_t)q;
                    const uint32_t w = (uint32_t)__shfl((int)wl, (int)(j & (kWave - 1)), kWave);
                    if (j < m && (w & kMirAlive)) {
                        const uint32_t p = w & 127u, r = (w >> 7) & 31u;
                        const double px = X.V[cur][p][c];
                        const double cand = r ? px + nx_pick(r, cf) : px;
                        const int a = (int)(a0 + j);
                        const int pr = r ? a : -a - 2;
                        const bool take = (bp == INT_MIN) | ((cand > bv) | (!(bv > cand) & (pr > bp)));
                        bv = take ? cand : bv;
                        bp = take ? pr : bp;
                        xmin = fmin(xmin, r ? cand : px + 0.0);
                    }
                }
            }
#pragma unroll
            for (int sh = kNxCuts; sh < kWave; sh <<= 1) {
                const double ov = __shfl_xor(bv, sh, kWave);
                const int op = __shfl_xor(bp, sh, kWave);
                const bool take = (bp == INT_MIN) | ((op != INT_MIN) & ((ov > bv) | (!(bv > ov) & (op > bp))));
                bv = take ? ov : bv;
                bp = take ? op : bp;
                xmin = fmin(xmin, __shfl_xor(xmin, sh, kWave));
            }
            const double val = (bp == INT_MIN) ? EDMIN : smax(bv, EDMIN);
            if (q == 0) X.V[cur ^ 1][0][c] = val;
            if (summ && q == 0) summary(val, xmin);
        }
        wave_lds_sync();
        cur ^= 1;
        if (k < k0) {
#pragma unroll
            for (int r = 0; r < kNxRanks; r++) cf[r] = nf[r];
        }
    }
    const double v0 = X.V[cur][q0][c];
#pragma unroll
    for (int sh = kNxCuts; sh < kWave; sh <<= 1) {
        gap = fmin(gap, __shfl_xor(gap, sh, kWave));
        mag = fmax(mag, __shfl_xor(mag, sh, kWave));
        unc = unc | (__shfl_xor((int)unc, sh, kWave) != 0);
    }
    wave_lds_sync();   // every lane read the last layer before the next item overwrites it
    if (q == 0 && vc) {
        ex.R[(size_t)i * os + s] = v0;
        ex.G[(size_t)i * os + s] = unc ? -INFINITY : gap - 1e-12 * (mag + 1.0);
        ex.MS[(size_t)i * os + s] = 0ull;
    }
}

__global__ void __launch_bounds__(kWave) k_nx_dag(NetDev net, Scratch sc, ExactIO ex) {
    __shared__ NxShared S;
    const int nnx = (int)ex.ctr[12];   // non-exact entries (ExactIO::nxlist)
    if (nnx == 0) return;
    const long long nblk = (ex.no + kNxCuts - 1) / kNxCuts;
    const long long total = nblk * nnx;
    for (;;) {
        if (lane() == 0) S.item = (int32_t)atomicAdd(&ex.ctr[6], 1ull);
        __builtin_amdgcn_wave_barrier();
        const long long item = (long long)uni(S.item);
        __builtin_amdgcn_wave_barrier();
        if (item >= total) break;
        const int b = (int)(item / nnx);
        const int i = uni(ex.nxlist[item % nnx]);
        // blocks k_relax already applied in order
        if ((b + 1) * kNxCuts <= uni(ex.nxh[(size_t)uni(ex.pend_slot[i]) * 4 + 3])) continue;
        nx_dag_item(net, sc, ex, S, i, b);
    }
}

hipError_t launch_exact_cols(const double *rows, const double *rhs, const int32_t *o_order, int no, int first,
                             int stride, int n_slots, int ostride, double *coefO, int reverse, hipStream_t st) {
    if (no <= first) return hipSuccess;
    hipLaunchKernelGGL(k_exact_cols, dim3(no - first), dim3(256), 0, st, rows, rhs, o_order, no, first, stride, n_slots,
                       ostride, coefO, reverse);
    return hipGetLastError();
}

// the pending records' root folds and terminal weights; k_exact_fin (dd_kernels.hip) ends them
// (with non-exact records: k_nx_dag between the root folds and the leaf passes, k_nx_fin after)
hipError_t launch_exact(const NetDev &net, const Scratch &sc, const ExactIO &ex, double incumbent, int cus,
                        hipStream_t st) {
    hipLaunchKernelGGL(k_exact_root, dim3(4 * cus), dim3(kRootWaves * kWave), 0, st, net, sc, ex);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (ex.nx && ex.pkind) {
        hipLaunchKernelGGL(k_nx_dag, dim3(5 * cus), dim3(kWave), 0, st, net, sc, ex);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    using Narrow = LeafSharedT<kExactMaxEntries>;
    using Wide = LeafSharedT<kExactMaxEntriesWide>;
    // exact DDs: phase A (or the single phase), then phase B over the open leaves
    ExactIO pb = ex;
    pb.leaf_phase = 1;
    const bool two = ex.leaf_split > 0 && ex.lazy == 0;
    hipLaunchKernelGGL((k_exact_leaf<false, kExactMaxEntries>), dim3(4 * cus), dim3(kLeafWaves * kWave), sizeof(Narrow), st,
                       net, sc, ex, incumbent);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (two) {
        hipLaunchKernelGGL((k_exact_leaf<false, kExactMaxEntries>), dim3(4 * cus), dim3(kLeafWaves * kWave), sizeof(Narrow),
                           st, net, sc, pb, incumbent);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if ((kExactMaxT - 1) * sc.us > kExactMaxEntries) {   // deeper / wider exact trees are possible
        hipLaunchKernelGGL((k_exact_leaf<false, kExactMaxEntriesWide>), dim3(4 * cus), dim3(kLeafWaves * kWave), sizeof(Wide),
                           st, net, sc, ex, incumbent);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if (two) {
            hipLaunchKernelGGL((k_exact_leaf<false, kExactMaxEntriesWide>), dim3(4 * cus), dim3(kLeafWaves * kWave),
                               sizeof(Wide), st, net, sc, pb, incumbent);
            if ((e = hipGetLastError()) != hipSuccess) return e;
        }
    }
    if (!ex.nx || !ex.pkind) return hipSuccess;
    hipLaunchKernelGGL((k_exact_leaf<true, kExactMaxEntries>), dim3(4 * cus), dim3(kLeafWaves * kWave), sizeof(Narrow), st,
                       net, sc, ex, incumbent);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    ExactIO ms = ex;
    ms.nx_ms = 1;
    hipLaunchKernelGGL((k_exact_leaf<true, kExactMaxEntries>), dim3(4 * cus), dim3(kLeafWaves * kWave), sizeof(Narrow), st,
                       net, sc, ms, incumbent);
    return hipGetLastError();
}

}  // namespace sgufp
