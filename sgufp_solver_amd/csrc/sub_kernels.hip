// MI355X (gfx950) kernels for the scenario subproblem of SGUFP_Solver's exact leaves:
// GuroSolver::solveSubProblem(path) (/root/reference/grb.cpp:139-360), which the reference
// solves as one Gurobi LP per scenario (the dual of a flow problem, grb.cpp:42-136).
//
// One workgroup per (path, scenario): a single 64-lane wave on the 1k-arc networks, eight
// waves on the large ones whose LDS holds one scenario per CU (Blk<NW> below):
//   1. y-bar from the path (grb.cpp:139-150): at every V-bar node q each incoming arc is
//      matched to the out-arc its DD layer decided, or to nothing (-1).
//   2. Contraction.  The primal of the reference's dual is max sum r x over the network
//      with conservation at nodes that have in- and out-arcs, l <= x <= u, and at a
//      V-bar node: matched pairs carry equal flow (lambda / mu rows), unmatched arcs carry
//      none (sigma / phi rows).  Following the matching turns every arc into one "chain"
//      through V-bar nodes; a chain from a non-V-bar tail to a non-V-bar head is one
//      arc with bounds [max l, min u] and reward sum r, any other chain is fixed at 0.
//   3. Max-reward flow on the contracted DAG (free supply at sources, free demand at
//      sinks): successive shortest paths (Bellman-Ford in LDS over the residual graph,
//      Gauss-Seidel sweeps in topological chain order, 64-bit (cost, hops) keys so the
//      predecessor graph of equal-cost paths has no cycles, resumed after each
//      augmentation from the labels it left intact).  Lower bounds ride on a big-M reward; a lower
//      bound left unmet at the end is primal infeasibility.
//   4. An optimal dual of the reference formulation (alpha from shortest-path potentials
//      of the final residual, beta / gamma from reduced costs, lambda / mu as the free
//      transfers along matched pairs, sigma / phi on unmatched arcs), or, for an
//      infeasible scenario, an unbounded dual ray (Farkas certificate).  From it the
//      scenario's contribution to the cut, exactly as grb.cpp:236-281 / 288-350 assemble
//      it.  All of it is integer arithmetic (integral data), written out as f64.
// A second kernel reduces over scenarios per path in scenario order: the first infeasible
// scenario's ray (feasibility cut), else the 1/S-weighted sum (optimality cut).
//
// Duals are not unique, so the cut coefficients differ from Gurobi's; what is pinned is
// the scenario objective (== HiGHS on the reference formulation, tests/), that the cut is
// tight at y-bar (RHS + coef.y-bar == mean objective) and valid for other y.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>
#include <type_traits>

#include "sub_device.hpp"
#define SGUFP_MULTI_WAVE_TU   // k_sub_scenario runs 1 or kLargeWaves (8) waves per workgroup
#include "wave.hpp"

namespace sgufp {

namespace {

// Bellman-Ford keys: (cost << hop bits) | hops.  64-bit keys in general (big-M costs of the
// lower bounds); 32-bit keys when the launch has no lower bound and the rewards are small
// (host check, launch_subproblem): half the LDS bytes and atomics, single-register adds.
template <typename KT> struct KeyT;
template <> struct KeyT<int64_t> {
    static constexpr int hop_bits = 16;
    static constexpr int64_t inf = INT64_MAX / 4;
};
template <> struct KeyT<int32_t> {
    // |path cost| <= sum_a |r_a| < 2^18 (host), hops < 2^11: keys below 2^29 in magnitude
    static constexpr int hop_bits = 11;
    static constexpr int32_t inf = 1 << 30;
};
constexpr int64_t kInf = INT64_MAX / 4;   // 64-bit sentinel for capacities (delta)
constexpr int kMaxChain = 64;      // arcs per chain (V-bar nodes in a row + 1)
constexpr int32_t kNoPred = INT32_MAX;

// Chain k of the contracted network lives in two 64-bit LDS words, so a Bellman-Ford pass
// reads one arc with two ds_read_b64:
//   cta: tail:16 | head:16 | reward sum:32          (-1 ends as 0xFFFF)
//   ctb: max l:16 | min u:16 | flow x:16 | first arc:16
// Node / arc ids fit 16 bits (Cut.h:342-344 packs them so); the host checks the bounds.
// ALLREG: every chain group of the launch sits in registers (single wave: nct_cap <= 16 x 64;
// eight waves: <= 10 x 8 x 64): no sweep reads chain records from LDS, predecessors come from
// the registers too
__device__ __forceinline__ int ch_t(uint64_t a);
__device__ __forceinline__ int ch_h(uint64_t a);
__device__ __forceinline__ int ch_R(uint64_t a);
__device__ __forceinline__ uint64_t pack_a(int t, int h, int R);

template <typename KT, bool ALLREG = false, bool PACK = false>
struct SubLds {
    using Key = KT;
    static constexpr bool kAllReg = ALLREG;
    // work-list Bellman-Ford (bf_converge_wl): single wave (PACK is "one wave per scenario"),
    // every chain group in registers (<= 16 groups)
#ifdef SGUFP_SUB_WL
    static constexpr bool kWL = ALLREG && PACK;
    // 2: a group with a lowered key marks its precomputed successor groups (all the groups of
    // the arcs out of the group's heads / tails: a superset, no per-lane mask or wave OR);
    // 1: the exact groups of the lowered keys (an LDS table read per arc, a wave OR per group)
    static constexpr bool kCoarse = SGUFP_SUB_WL == 2;
#else
    static constexpr bool kWL = false;   // full sweeps (the work list measured slower)
    static constexpr bool kCoarse = false;
#endif
    LDS uint32_t *inc;      // [n+2] kWL: groups with a chain out of v (bits 0-15) / into v (16-31)
    static constexpr int kHop = KeyT<KT>::hop_bits;
    static constexpr KT kKInf = KeyT<KT>::inf;
    LDS int32_t *imb;       // [n+2] warm starts: node imbalances of the initial flow
    LDS uint64_t *cta;      // [nct_cap] chains, in the topological order of their tails
    // 16-byte records: cta (above) and ctb = L:16 | U:16 | x:16 | first arc:16.  With 32-bit
    // keys (no lower bound anywhere, u < 2^11, n + 2 < 2^11, sum |r| < 2^18: host) the first
    // arc is not stored (re-derived from the path where it is needed) and L = 0: 12-byte
    // records, ctb = U:16 | x:16, in the eight-wave kernel; one 8-byte word per chain in the
    // single-wave one (PACK), tail:11 | head:11 | R:19 | U:11 | x:11 -- 16 instead of 12
    // scenarios of a 1k-arc network fit the LDS of a CU (C4 32 x 256: 23.4 -> 21.7 ms); the
    // eight-wave kernel, two scenarios per CU either way, keeps the 12-byte records.
    // ra / rb / wa / wb / add_x read and write the fields in the 16-byte layout's encoding
    // whatever the storage.
    static constexpr bool kCompact = sizeof(KT) == 4;
    static constexpr bool kPack = kCompact && PACK;
    using CBT = std::conditional_t<kCompact, uint32_t, uint64_t>;
    LDS CBT *ctb;           // [nct_cap], none with kPack
    // 11-bit node id, 0x7FF = -1 (no node; ids < 2^11 - 2 by the host check)
    static __device__ __forceinline__ int id11(uint64_t v) {
        const int x = (int)(v & 0x7FFull);
        return x == 0x7FF ? -1 : x;
    }
    __device__ __forceinline__ uint64_t ra(int k) const {
        if constexpr (kPack) {
            const uint64_t w = cta[k];
            return pack_a(id11(w), id11(w >> 11), (int)((int64_t)(w << 23) >> 45));   // R: bits 22..40, signed
        } else {
            return cta[k];
        }
    }
    __device__ __forceinline__ uint64_t rb(int k) const {
        if constexpr (kPack) {
            const uint64_t w = cta[k];
            return ((w >> 41) & 0x7FFull) << 16 | ((w >> 52) & 0x7FFull) << 32;
        } else if constexpr (kCompact) {
            const uint32_t v = ctb[k];
            return (uint64_t)(v & 0xFFFFu) << 16 | (uint64_t)(v >> 16) << 32;
        } else {
            return ctb[k];
        }
    }
    __device__ __forceinline__ void wa(int k, uint64_t a) const {
        if constexpr (kPack) {
            const uint64_t f = ((uint64_t)(uint32_t)ch_t(a) & 0x7FFull) | ((uint64_t)(uint32_t)ch_h(a) & 0x7FFull) << 11 |
                               ((uint64_t)(uint32_t)ch_R(a) & 0x7FFFFull) << 22;
            cta[k] = (cta[k] & ~((1ull << 41) - 1ull)) | f;
        } else {
            cta[k] = a;
        }
    }
    __device__ __forceinline__ void wb(int k, uint64_t b) const {
        if constexpr (kPack) {
            const uint64_t f = ((b >> 16) & 0x7FFull) << 41 | ((b >> 32) & 0x7FFull) << 52;
            cta[k] = (cta[k] & ((1ull << 41) - 1ull)) | f;
        } else if constexpr (kCompact) {
            ctb[k] = (uint32_t)((b >> 16) & 0xFFFFu) | (uint32_t)((b >> 32) & 0xFFFFu) << 16;
        } else {
            ctb[k] = b;
        }
    }
    // flow of chain k += d (0 <= x + d <= U)
    __device__ __forceinline__ void add_x(int k, int d) const {
        if constexpr (kPack) cta[k] += (uint64_t)(int64_t)d << 52;
        else *((LDS int16_t *)&ctb[k] + (kCompact ? 1 : 2)) += (int16_t)d;
    }
    LDS KT *key;            // [n+2] Bellman-Ford keys (cost << hop bits | hops); then alpha in place
    LDS KT *alpha;          // == key: dual node potentials after the last Bellman-Ford
    LDS int32_t *pred;      // [n+2] code of the tight in-arc << 15 | its tail (kNoPred: none)
    LDS uint16_t *plist;    // [n+2] arc codes of the augmenting path (sink to source)
    double GBL *coef;       // [n_slots] this (path, scenario)'s row of SubIO::coef (phase 5)
    LDS int64_t *acc;       // [n_slots] phase 5's row in LDS (over the chain records) when
    bool use_acc;           //     use_acc, else atomic adds straight into coef (a flag: LDS
                            //     address 0 is the null pointer of that address space)
    LDS int32_t *zlist;     // [nz] free-supply / free-demand nodes: v | src << 30 | snk << 29
    LDS int32_t *misc;      // [8] flags
    LDS int64_t *red;       // [8] cross-wave reduction slots (multi-wave workgroups)
#ifdef SGUFP_SUB_VERIFY
    LDS KT *vkey;           // [n+2] warm Bellman-Ford keys, compared with a cold run
#endif
};

__host__ __device__ inline size_t a16(size_t x) { return (x + 15) & ~(size_t)15; }

// One scenario per workgroup of NW waves.  NW = 1 on the 1k-arc networks (a single wave;
// nine of them share a CU's LDS); NW = 8 on the large ones, whose LDS holds one scenario per
// CU: the waves then share every per-chain / per-node loop, and a Bellman-Ford step relaxes
// NW chain groups at once (see bf_sweep).
template <int NW>
struct Blk {
    static constexpr int T = NW * kWave;
    __device__ static __forceinline__ int tid() { return (int)threadIdx.x; }
    __device__ static __forceinline__ int wid() { return NW == 1 ? 0 : (int)threadIdx.x / kWave; }
    __device__ static __forceinline__ void sync() {
        if constexpr (NW == 1) wave_lds_sync();
        else __syncthreads();
    }
    // all-reduce over the workgroup (associative, commutative op)
    template <typename V, typename Op>
    __device__ static __forceinline__ V all(V x, Op op, LDS int64_t *red) {
        x = lane_reduce<1>(x, op);
        if constexpr (NW == 1) {
            return x;
        } else {
            if (lane() == 0) red[wid()] = (int64_t)x;
            __syncthreads();
            V r = (V)red[0];
            for (int w = 1; w < NW; w++) r = op(r, (V)red[w]);
            __syncthreads();
            return r;
        }
    }
    __device__ static __forceinline__ uint32_t any(uint32_t x, LDS int64_t *red) {
        return all(x, [](uint32_t a, uint32_t b) { return a | b; }, red);
    }
};

// LDS: chains, key (alpha), pred, plist, the warm start's imbalances, the free-node list and
// flags.  (The chains' arcs come from k_sub_paths' lists in HBM.)
constexpr int kSubLdsParts = 12;
__host__ __device__ inline size_t sub_lds_layout(int n, int m, int nct_cap, int nz, int nw, size_t *off, int kbytes = 8,
                                                 bool warm = false, bool wl = false) {
    size_t o = 0;
    off[1] = o; o = a16(o + (size_t)nct_cap * 8);
    // b words: 8 bytes, 4 with 32-bit keys, none in the single-wave kernel's 8-byte records
    off[2] = o; o = a16(o + (size_t)nct_cap * (kbytes == 4 ? (nw == 1 ? 0 : 4) : 8));
    off[3] = o; o = a16(o + (size_t)(n + 2) * kbytes);   // key
    off[4] = o; o = a16(o + (size_t)(n + 2) * 4);   // pred
    off[8] = o; o = a16(o + (size_t)(n + 2) * 2);   // plist
    off[0] = o; o = a16(o + (warm ? (size_t)(n + 2) * 4 : 0));   // imbalances
    off[5] = o;
    off[6] = o; o = a16(o + (size_t)nz * 4);
    off[7] = o; o = a16(o + 8 * 4);
    off[10] = o; o = a16(o + (nw > 1 ? 8 * 8 : 0));   // red
    off[11] = o; o = a16(o + (wl ? (size_t)(n + 2 + 32) * 4 : 0));   // inc + group successors (work list)
#ifdef SGUFP_SUB_VERIFY
    off[9] = o; o = a16(o + (size_t)(n + 2) * kbytes);
#endif
    return o;
}

__device__ __forceinline__ int ch_t(uint64_t a) { return (int)(int16_t)(uint16_t)a; }
__device__ __forceinline__ int ch_h(uint64_t a) { return (int)(int16_t)(uint16_t)(a >> 16); }
__device__ __forceinline__ int ch_R(uint64_t a) { return (int)(int32_t)(uint32_t)(a >> 32); }
__device__ __forceinline__ int ch_L(uint64_t b) { return (int)(int16_t)(uint16_t)b; }
__device__ __forceinline__ int ch_U(uint64_t b) { return (int)(int16_t)(uint16_t)(b >> 16); }
__device__ __forceinline__ int ch_x(uint64_t b) { return (int)(int16_t)(uint16_t)(b >> 32); }
__device__ __forceinline__ int ch_first(uint64_t b) { return (int)(int16_t)(uint16_t)(b >> 48); }
__device__ __forceinline__ uint64_t pack_a(int t, int h, int R) {
    return (uint64_t)(uint16_t)t | (uint64_t)(uint16_t)h << 16 | (uint64_t)(uint32_t)R << 32;
}
__device__ __forceinline__ uint64_t pack_b(int L, int U, int x, int first) {
    return (uint64_t)(uint16_t)L | (uint64_t)(uint16_t)U << 16 | (uint64_t)(uint16_t)x << 32 |
           (uint64_t)(uint16_t)first << 48;
}
// the flow field of chain k (lane 0 augments)

__device__ __forceinline__ bool is_src(const SubNet &N, int v) { return N.in_off[v + 1] == N.in_off[v]; }
__device__ __forceinline__ bool is_snk(const SubNet &N, int v) { return N.out_off[v + 1] == N.out_off[v]; }

// ---------------------------------------------------------------------------------------
// Bellman-Ford over the residual graph of the contracted network.
//   SSP mode: shortest paths from Z_out (node n) to Z_in (node n+1) under the big-M costs;
//             arcs Z_out -> source and sink -> Z_in are free and uncapacitated.
//   POT mode: potentials; every node starts at 0 (virtual root), Z (node n) is tied to
//             every source and sink by free arcs in both directions (alpha = 0 there);
//             BIGM selects the big-M costs (dual ray) or the plain ones (optimal duals).
enum BfMode { kSsp = 0, kPotPlain = 1, kPotBigM = 2 };

template <int NW, typename F, class WS>
__device__ __forceinline__ void for_residual(const SubNet &N, const WS &W, int nct, int nz, int mode, int64_t M, F visit) {
    using B = Blk<NW>;
    // contracted arcs: code 2k (forward), 2k+1 (backward)
    for (int k = B::tid(); k < nct; k += B::T) {
        const uint64_t ca = W.ra(k), cb = W.rb(k);
        const int t = ch_t(ca), h = ch_h(ca);
        if (t < 0 || h < 0) continue;
        const int64_t x = ch_x(cb), L = ch_L(cb), U = ch_U(cb), R = ch_R(ca);
        if (mode == kPotPlain) {
            if (x < U) visit(t, h, -R, 2 * k);
            if (x > L) visit(h, t, R, 2 * k + 1);
        } else {
            if (x < U) visit(t, h, -(R + (x < L ? M : 0)), 2 * k);
            if (x > 0) visit(h, t, R + (x <= L ? M : 0), 2 * k + 1);
        }
    }
    // Z arcs: code 2m + 2v (+1), from the LDS list of non-inner nodes
    for (int i = B::tid(); i < nz; i += B::T) {
        const uint32_t e = (uint32_t)W.zlist[i];
        const int v = (int)(e & 0x1FFFFFFFu);
        const bool src = (e >> 30) & 1u, snk = (e >> 29) & 1u;
        if (mode == kSsp) {
            if (src) visit(N.n, v, 0, 2 * N.m + 2 * v);
            if (snk) visit(v, N.n + 1, 0, 2 * N.m + 2 * v + 1);
        } else {
            visit(N.n, v, 0, 2 * N.m + 2 * v);
            visit(v, N.n, 0, 2 * N.m + 2 * v + 1);
        }
    }
}

// The residual arcs of chain group g (chains g*64 .. g*64+63, one per lane) for one
// Bellman-Ford: ends packed tail | head << 16, forward / backward key increments
// ((cost << 16) + 1) and which of the two arcs exist.  Flows only change between
// Bellman-Fords, so the first RG groups of each wave live in registers for all its passes:
// 16 groups (80 VGPRs) on the 1k-arc networks, whose small LDS footprint runs 9 waves per CU;
// on the large ones (one scenario per CU, NW = 8 waves; C5, 4 paths x 512 scenarios: 1 / 2 /
// 4 / 8 waves 2408 / 1549 / 918 / 732 ms) 80 / NW groups per wave with 32-bit costs.  Groups
// beyond them are read from LDS (one group ahead of their use with one wave).
#ifndef SGUFP_LARGE_WAVES
#define SGUFP_LARGE_WAVES 8
#endif
constexpr int kLargeWaves = SGUFP_LARGE_WAVES;
// Blk<NW>::all and the chain-numbering scan write one `red` slot per wave (8 in the layout)
static_assert(kLargeWaves >= 1 && kLargeWaves <= 8, "the cross-wave reduction array holds 8 waves");
constexpr int kRegGroupsSmall = 16, kRegGroupsLarge = (80 + kLargeWaves - 1) / kLargeWaves;
#ifndef SGUFP_REG_GROUPS_WARM
#define SGUFP_REG_GROUPS_WARM 13
#endif
constexpr int kRegGroupsWarm = SGUFP_REG_GROUPS_WARM;

template <typename KT>
struct ChainArcs {
    uint32_t th;
    KT wf, wb;          // key increments (cost << hop bits) + 1
    int64_t cf, cbk;    // the costs
    bool fwd, bwd;
};

template <typename KT>
__device__ __forceinline__ ChainArcs<KT> chain_arcs(uint64_t ca, uint64_t cb, bool in_range, int n, int mode, int64_t M) {
    ChainArcs<KT> c;
    const int t = ch_t(ca), h = ch_h(ca);
    const bool ok = in_range && t >= 0 && h >= 0;
    c.th = ok ? ((uint32_t)t | (uint32_t)h << 16) : ((uint32_t)n | (uint32_t)n << 16);
    const int x = ch_x(cb), L = ch_L(cb), U = ch_U(cb);
    const int64_t R = ch_R(ca);
    const int64_t w_f = (mode == kPotPlain) ? -R : -(R + (x < L ? M : 0));
    const int64_t w_b = (mode == kPotPlain) ? R : R + (x <= L ? M : 0);
    c.cf = w_f;
    c.cbk = w_b;
    c.wf = (KT)((w_f << KeyT<KT>::hop_bits) + 1);
    c.wb = (KT)((w_b << KeyT<KT>::hop_bits) + 1);
    c.fwd = ok && x < U;
    c.bwd = ok && (mode == kPotPlain ? x > L : x > 0);
    return c;
}

// WT: the type the costs are kept in: key increments (cost << hop bits) + 1, formed once, when
// WT is the key type; costs, the increment formed at use, for the large variant with 64-bit keys
// (int32_t, whose host check bounds the big-M costs below 2^30)
template <int RG, typename WT>
struct ChainRegs {
    uint32_t th[RG];
    WT wf[RG], wb[RG];
    uint64_t fmask, bmask;
};

// register slot j of wave w holds chain group j * NW + w
template <int RG, typename WT, int NW, class WS>
__device__ __forceinline__ void load_chain_regs(const WS &W, int n, int nct, int mode, int64_t M, ChainRegs<RG, WT> &C) {
    using KT = typename WS::Key;
    C.fmask = 0;
    C.bmask = 0;
#pragma unroll
    for (int g = 0; g < RG; g++) {
        const int k = (g * NW + Blk<NW>::wid()) * kWave + lane();
        uint64_t ca = 0, cb = 0;
        if (k < nct) { ca = W.ra(k); cb = W.rb(k); }
        const ChainArcs<KT> c = chain_arcs<KT>(ca, cb, k < nct, n, mode, M);
        C.th[g] = c.th;
        if constexpr (sizeof(WT) == sizeof(KT)) {   // key increments, formed once
            C.wf[g] = c.wf;
            C.wb[g] = c.wb;
        } else {                           // costs, the increment formed at use
            C.wf[g] = (WT)c.cf;
            C.wb[g] = (WT)c.cbk;
        }
        C.fmask |= (c.fwd ? 1ull : 0ull) << g;
        C.bmask |= (c.bwd ? 1ull : 0ull) << g;
    }
}

// One Bellman-Ford pass over the residual arcs of for_residual (same arcs, same costs):
// a forward sweep over the chains in order (tails in topological order) relaxes the
// forward residual arcs, a backward sweep in reverse order the backward ones, 64 chains
// at a time, so a label travels down a run of forward arcs (or up a run of backward ones)
// within one sweep.  LDS is in order within the wave, so a group's key loads see the
// previous group's atomic minima (a pass that changes nothing read only settled keys, so
// convergence never depends on that ordering).  The fixed point -- the shortest (cost,
// hops) keys -- is unique, so the order changes only how many passes it takes; the caller
// iterates until a forward and a backward sweep in a row (either order) change nothing:
// then every residual arc is settled on the same keys.  `forward` picks the half: the Z
// arcs out of Z_out / Z and the forward residual arcs, then the arcs into Z_in / Z; or the
// backward residual arcs.
// With NW waves, step j of a sweep relaxes groups j * NW .. j * NW + NW - 1 at once (one per
// wave) and a barrier closes the step: the groups of one step are consecutive chains, almost
// always tails of one layer of the network, so the in-order propagation along runs of arcs
// is kept.
template <int RG, typename WT, int NW, class WS>
__device__ __forceinline__ uint32_t bf_sweep(const SubNet &N, const WS &W, int nct, int nz, int mode, int64_t M,
                                    const ChainRegs<RG, WT> &C, bool forward) {
    using KT = typename WS::Key;
    constexpr KT kKInf = WS::kKInf;
    uint32_t changed = 0;
    auto relax = [&](int v, KT nk) {
        if (nk < W.key[v]) {
            __hip_atomic_fetch_min(&W.key[v], nk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            changed = 1;
        }
    };
    // one arc of a group: both end keys in one LDS round trip, then the atomic minimum
    auto arc = [&](uint32_t th, KT w, bool exists, bool forward) {
        const int t = (int)(th & 0xFFFFu), h = (int)(th >> 16);
        const int u = forward ? t : h, v = forward ? h : t;
        // both end keys in one LDS round trip (fenced: the compiler would otherwise sink the
        // second load under the first comparison and pay two)
        const KT ku = W.key[u], kv = W.key[v];
        sched_fence();
        const KT nk = ku + w;
        if (exists & (ku < kKInf) & (nk < kv)) {
            __hip_atomic_fetch_min(&W.key[v], nk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            changed = 1;
        }
    };
    auto reg_w = [&](WT w) -> KT { return sizeof(WT) == sizeof(KT) ? (KT)w : (KT)(((int64_t)w << WS::kHop) + 1); };
    const int n = N.n;
    const int G = (nct + kWave - 1) / kWave;
    // chains of group g from LDS (groups past the register-resident ones)
    auto fetch = [&](int g, uint64_t &ca, uint64_t &cb) {
        const int k = g * kWave + lane();
        ca = 0;
        cb = 0;
        if (k < nct) { ca = W.ra(k); cb = W.rb(k); }
    };
    if constexpr (NW > 1) {
        using B = Blk<NW>;
        const int S = (G + NW - 1) / NW, wv = B::wid();
        if (!forward) {
            for (int j = S - 1; j >= RG && !WS::kAllReg; j--) {
                const int g = j * NW + wv;
                if (g < G) {
                    uint64_t ca, cb;
                    fetch(g, ca, cb);
                    const ChainArcs<KT> c = chain_arcs<KT>(ca, cb, g * kWave + lane() < nct, n, mode, M);
                    arc(c.th, c.wb, c.bwd, false);
                }
                __syncthreads();
            }
            // fixed trip count with uniform guards: a data-dependent exit would keep the
            // loop rolled (it holds a barrier) and index the register arrays dynamically,
            // i.e. from scratch memory
#pragma unroll
            for (int j = RG - 1; j >= 0; j--) {
                if (j < S) {
                    if (j * NW + wv < G) arc(C.th[j], reg_w(C.wb[j]), (C.bmask >> j) & 1ull, false);
                    __syncthreads();
                }
            }
            return changed;
        }
        {
            const KT kz = W.key[n];
            if (kz < kKInf)
                for (int i = B::tid(); i < nz; i += B::T) {
                    const uint32_t e = (uint32_t)W.zlist[i];
                    if (mode != kSsp || ((e >> 30) & 1u)) relax((int)(e & 0x1FFFFFFFu), kz + 1);
                }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < RG; j++) {
            if (j < S) {
                if (j * NW + wv < G) arc(C.th[j], reg_w(C.wf[j]), (C.fmask >> j) & 1ull, true);
                __syncthreads();
            }
        }
        for (int j = RG; j < S && !WS::kAllReg; j++) {
            const int g = j * NW + wv;
            if (g < G) {
                uint64_t ca, cb;
                fetch(g, ca, cb);
                const ChainArcs<KT> c = chain_arcs<KT>(ca, cb, g * kWave + lane() < nct, n, mode, M);
                arc(c.th, c.wf, c.fwd, true);
            }
            __syncthreads();
        }
        for (int i = B::tid(); i < nz; i += B::T) {
            const uint32_t e = (uint32_t)W.zlist[i];
            const int v = (int)(e & 0x1FFFFFFFu);
            const KT kv = W.key[v];
            if (kv >= kKInf) continue;
            if (mode == kSsp) { if ((e >> 29) & 1u) relax(n + 1, kv + 1); }
            else relax(n, kv + 1);
        }
        return changed;
    }
    constexpr bool kPrefetch = RG >= 32;
    if (!forward) {
        if constexpr (WS::kAllReg) {
        } else if (!kPrefetch) {
            for (int g = G - 1; g >= RG; g--) {
                uint64_t ca, cb;
                fetch(g, ca, cb);
                const ChainArcs<KT> c = chain_arcs<KT>(ca, cb, g * kWave + lane() < nct, n, mode, M);
                arc(c.th, c.wb, c.bwd, false);
            }
        } else if (G > RG) {
            uint64_t na, nb;
            fetch(G - 1, na, nb);
            for (int g = G - 1; g >= RG; g--) {
                const uint64_t ca = na, cb = nb;
                if (g > RG) fetch(g - 1, na, nb);   // next group's chains load under this group's keys
                const ChainArcs<KT> c = chain_arcs<KT>(ca, cb, g * kWave + lane() < nct, n, mode, M);
                arc(c.th, c.wb, c.bwd, false);
            }
        }
#pragma unroll
        for (int g = RG - 1; g >= 0; g--) {
            if (g < G) arc(C.th[g], reg_w(C.wb[g]), (C.bmask >> g) & 1ull, false);
        }
        return changed;
    }
    // Z_out -> sources (SSP) / Z -> every free node (potentials), cost 0
    {
        const KT kz = W.key[n];
        if (kz < kKInf)
            for (int i = lane(); i < nz; i += kWave) {
                const uint32_t e = (uint32_t)W.zlist[i];
                if (mode != kSsp || ((e >> 30) & 1u)) relax((int)(e & 0x1FFFFFFFu), kz + 1);
            }
    }
    wave_lds_sync();
#pragma unroll
    for (int g = 0; g < RG; g++) {
        if (g < G) arc(C.th[g], reg_w(C.wf[g]), (C.fmask >> g) & 1ull, true);
    }
    if constexpr (WS::kAllReg) {
    } else if (!kPrefetch) {
        for (int g = RG; g < G; g++) {
            uint64_t ca, cb;
            fetch(g, ca, cb);
            const ChainArcs<KT> c = chain_arcs<KT>(ca, cb, g * kWave + lane() < nct, n, mode, M);
            arc(c.th, c.wf, c.fwd, true);
        }
    } else if (G > RG) {
        uint64_t na, nb;
        fetch(RG, na, nb);
        for (int g = RG; g < G; g++) {
            const uint64_t ca = na, cb = nb;
            if (g + 1 < G) fetch(g + 1, na, nb);
            const ChainArcs<KT> c = chain_arcs<KT>(ca, cb, g * kWave + lane() < nct, n, mode, M);
            arc(c.th, c.wf, c.fwd, true);
        }
    }
    // sinks -> Z_in (SSP) / free nodes -> Z (potentials), cost 0
    for (int i = lane(); i < nz; i += kWave) {
        const uint32_t e = (uint32_t)W.zlist[i];
        const int v = (int)(e & 0x1FFFFFFFu);
        const KT kv = W.key[v];
        if (kv >= kKInf) continue;
        if (mode == kSsp) { if ((e >> 29) & 1u) relax(n + 1, kv + 1); }
        else relax(n, kv + 1);
    }
    return changed;
}

// Iterate sweeps, forward and backward alternating, to the fixed point (false: not within
// the pass bound).
template <int RG, typename WT, int NW, class WS>
__device__ __forceinline__ bool bf_converge(const SubNet &N, const WS &W, int nct, int nz, int mode, int64_t M,
                                   const ChainRegs<RG, WT> &C) {
    using B = Blk<NW>;
    bool prev_quiet = false;   // the sweep before the current one changed nothing
    for (int it = 0; it < 2 * (N.n + 4); it++) {
        if (B::tid() == 0 && !(it & 1)) W.misc[5]++;   // passes (io.wstat)
        const uint32_t changed = bf_sweep<RG, WT, NW>(N, W, nct, nz, mode, M, C, !(it & 1));
        B::sync();
        const bool quiet = !B::any(changed, W.red);
        if (quiet && prev_quiet) return true;
        prev_quiet = quiet;
    }
    return false;
}

// Work-list Bellman-Ford (one wave, every chain group in registers: WS::kWL).  The full sweeps
// above relax every group of 64 chains per sweep -- one dependent LDS round trip each -- and
// need two quiet sweeps to stop; after an augmentation most groups hold no arc whose end keys
// moved.  Here a group is relaxed only while its bit is set in df (forward residual arcs) / db
// (backward ones).  An arc u -> v can be unsettled only if key[u] fell or key[v] rose since it
// was last relaxed, or it changed itself, so:
//   * a lowered key[v] sets the groups of the arcs out of v: chains with tail v in df (W.inc
//     bits 0-15), chains with head v in db (bits 16-31) -- read with the arc's end keys, one
//     round trip, and OR-ed over the wave right away, so a group later in the sweep's order
//     sees it in the same sweep (the Gauss-Seidel propagation of the full sweeps);
//   * keys raised to infinity (invalidate_subtrees) set the groups of the arcs into them, and
//     the chains whose flow an augmentation changed set their own group in both: those callers
//     OR their bits into W.misc[1] / misc[2], which the next warm Bellman-Ford starts from
//     (wl_mark); a cold one starts with every group set.
// The Z arcs (a list of at most a few groups) are relaxed every forward sweep.  A forward +
// backward iteration that lowers no key ends it: every group is then clean, so every arc is
// settled -- the same fixed point (the unique shortest (cost, hops) keys) as the full sweeps.
template <class WS>
__device__ __forceinline__ void wl_mark(const WS &W, uint32_t mf, uint32_t mb) {
    // uniform control flow (wave_or); single wave: lane 0's read-modify-write is not raced
    mf = uni(wave_or(mf));
    mb = uni(wave_or(mb));
    if ((mf | mb) && lane() == 0) {
        W.misc[1] |= (int32_t)mf;
        W.misc[2] |= (int32_t)mb;
    }
}

template <int RG, typename WT, class WS>
__device__ __forceinline__ bool bf_converge_wl(const SubNet &N, const WS &W, int nct, int nz, int mode,
                                               const ChainRegs<RG, WT> &C, uint32_t df, uint32_t db) {
    static_assert(RG <= 16, "group masks are 16 bits");
    using KT = typename WS::Key;
    constexpr KT kKInf = WS::kKInf;
    const int n = N.n;
    const int G = (nct + kWave - 1) / kWave;
    const uint32_t all = G >= 16 ? 0xFFFFu : ((1u << G) - 1u);
    df &= all;
    db &= all;
    auto reg_w = [&](WT w) -> KT { return sizeof(WT) == sizeof(KT) ? (KT)w : (KT)(((int64_t)w << WS::kHop) + 1); };
    // coarse marks: lane g holds group g's successor masks (forward arcs: the groups of the arcs
    // out of its heads; backward arcs: out of its tails), wave-uniform through readlane
    uint32_t sucF = 0, sucB = 0;
    if constexpr (WS::kCoarse) {
        sucF = lane() < 16 ? W.inc[n + 2 + lane()] : 0u;
        sucB = lane() < 16 ? W.inc[n + 2 + 16 + lane()] : 0u;
    }
    for (int it = 0; it < 2 * (n + 4); it++) {
        if (lane() == 0) W.misc[5]++;   // passes (io.wstat)
        bool lowered = false;            // uniform: some key fell in this iteration
        // the wave's lowered keys -> groups to (re)relax
        auto note = [&](bool c, uint32_t iv) {
            if (__ballot(c)) {
                const uint32_t mo = uni(wave_or(c ? iv : 0u));
                df |= mo & 0xFFFFu;
                db |= mo >> 16;
                lowered = true;
            }
        };
        auto arc = [&](uint32_t th, KT w, bool exists, bool forward, int g) {
            const int t = (int)(th & 0xFFFFu), h = (int)(th >> 16);
            const int u = forward ? t : h, v = forward ? h : t;
            const KT ku = W.key[u], kv = W.key[v];
            uint32_t iv = 0;
            if constexpr (!WS::kCoarse) iv = W.inc[v];
            sched_fence();
            const KT nk = ku + w;
            const bool c = exists & (ku < kKInf) & (nk < kv);
            if (c) __hip_atomic_fetch_min(&W.key[v], nk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if constexpr (WS::kCoarse) {
                // (readfirstlane keeps df / db in scalar registers: the group tests stay scalar
                // branches, not exec-mask regions)
                const uint32_t any = uni((uint32_t)(__ballot(c) != 0));
                const uint32_t mo = any ? (uint32_t)__builtin_amdgcn_readlane((int)(forward ? sucF : sucB), g) : 0u;
                df = uni(df | (mo & 0xFFFFu));
                db = uni(db | (mo >> 16));
                lowered = lowered || any;
            } else {
                note(c, iv);
            }
        };
        // Z_out -> sources (SSP) / Z -> every free node (potentials), cost 0
        {
            const KT kz = W.key[n];
            bool c = false;
            uint32_t iv = 0;
            if (kz < kKInf)
                for (int i = lane(); i < nz; i += kWave) {
                    const uint32_t e = (uint32_t)W.zlist[i];
                    const int v = (int)(e & 0x1FFFFFFFu);
                    if (mode != kSsp || ((e >> 30) & 1u)) {
                        const KT kv = W.key[v];
                        const uint32_t i2 = W.inc[v];
                        sched_fence();
                        if (kz + 1 < kv) {
                            __hip_atomic_fetch_min(&W.key[v], (KT)(kz + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            c = true;
                            iv |= i2;
                        }
                    }
                }
            note(c, iv);
        }
        wave_lds_sync();
#pragma unroll
        for (int g = 0; g < RG; g++) {
            if (g < G && ((uni(df) >> g) & 1u)) {
                df = uni(df & ~(1u << g));
#ifdef SGUFP_SUB_TRACE
                if (lane() == 0) W.misc[7]++;   // groups relaxed
#endif
                arc(C.th[g], reg_w(C.wf[g]), (C.fmask >> g) & 1ull, true, g);
            }
        }
        // sinks -> Z_in (SSP) / free nodes -> Z (potentials), cost 0 (Z_in has no out-arc; Z's
        // arcs out are the list above)
        {
            bool c = false;
            for (int i = lane(); i < nz; i += kWave) {
                const uint32_t e = (uint32_t)W.zlist[i];
                const int v = (int)(e & 0x1FFFFFFFu);
                const KT kv = W.key[v];
                if (kv >= kKInf) continue;
                const int z = mode == kSsp ? n + 1 : n;
                if (mode == kSsp && !((e >> 29) & 1u)) continue;
                if (kv + 1 < W.key[z]) {
                    __hip_atomic_fetch_min(&W.key[z], (KT)(kv + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    c = true;
                }
            }
            if (__ballot(c)) lowered = true;
        }
        wave_lds_sync();
#pragma unroll
        for (int g = RG - 1; g >= 0; g--) {
            if (g < G && ((uni(db) >> g) & 1u)) {
                db = uni(db & ~(1u << g));
#ifdef SGUFP_SUB_TRACE
                if (lane() == 0) W.misc[7]++;
#endif
                arc(C.th[g], reg_w(C.wb[g]), (C.bmask >> g) & 1ull, false, g);
            }
        }
        if (!lowered) return true;
        wave_lds_sync();
    }
    return false;
}

// Predecessors of the SSP labels: the smallest arc code among the residual arcs into each
// node that are tight in (cost, hops).  Hops grow by one along such arcs, so the
// predecessor graph has no cycle and the walk from Z_in ends at Z_out.
template <int NW, class WS>
__device__ __forceinline__ void ssp_preds(const SubNet &N, const WS &W, int nct, int nz, int64_t M, int mode = kSsp) {
    using KT = typename WS::Key;
    for_residual<NW>(N, W, nct, nz, mode, M, [&](int u, int v, int64_t w, int code) {
        const KT ku = W.key[u];
        if (ku >= WS::kKInf) return;
        if ((KT)(ku + (KT)((w << WS::kHop) + 1)) == W.key[v])
            __hip_atomic_fetch_min(&W.pred[v], code << 15 | u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    });
    Blk<NW>::sync();
}

// Predecessors (as ssp_preds) from the register groups (every chain group of the launch in
// registers; slot j of wave w holds group j * NW + w): the costs are the ones the Bellman-Ford
// used, no chain record is re-read.
template <int RG, typename WT, int NW, class WS>
__device__ __forceinline__ void ssp_preds_regs(const SubNet &N, const WS &W, int nct, int nz, const ChainRegs<RG, WT> &C,
                                               int mode = kSsp) {
    using KT = typename WS::Key;
    using B = Blk<NW>;
    const int n = N.n, m = N.m;
    const int G = (nct + kWave - 1) / kWave;
    auto reg_w = [&](WT w) -> KT { return sizeof(WT) == sizeof(KT) ? (KT)w : (KT)(((int64_t)w << WS::kHop) + 1); };
    auto tight = [&](int u, int v, KT w, int code, bool exists) {
        const KT ku = W.key[u], kv = W.key[v];
        sched_fence();
        if (exists & (ku < WS::kKInf) & ((KT)(ku + w) == kv))
            __hip_atomic_fetch_min(&W.pred[v], code << 15 | u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
#pragma unroll
    for (int j = 0; j < RG; j++) {
        const int g = j * NW + B::wid();
        if (g < G) {
            const uint32_t th = C.th[j];
            tight((int)(th & 0xFFFFu), (int)(th >> 16), reg_w(C.wf[j]), 2 * (g * kWave + lane()), (C.fmask >> j) & 1ull);
        }
    }
#pragma unroll
    for (int j = 0; j < RG; j++) {
        const int g = j * NW + B::wid();
        if (g < G) {
            const uint32_t th = C.th[j];
            tight((int)(th >> 16), (int)(th & 0xFFFFu), reg_w(C.wb[j]), 2 * (g * kWave + lane()) + 1, (C.bmask >> j) & 1ull);
        }
    }
    for (int i = B::tid(); i < nz; i += B::T) {
        const uint32_t e = (uint32_t)W.zlist[i];
        const int v = (int)(e & 0x1FFFFFFFu);
        if (mode == kSsp) {
            if ((e >> 30) & 1u) tight(n, v, (KT)1, 2 * m + 2 * v, true);
            if ((e >> 29) & 1u) tight(v, n + 1, (KT)1, 2 * m + 2 * v + 1, true);
        } else {   // Z tied to every free node both ways (for_residual's potential mode)
            tight(n, v, (KT)1, 2 * m + 2 * v, true);
            tight(v, n, (KT)1, 2 * m + 2 * v + 1, true);
        }
    }
    B::sync();
}

// warm: keep the keys (exact or infinite, see invalidate_subtrees) instead of starting from
// Z_out alone -- Bellman-Ford from any upper bounds of the shortest keys reaches them.
template <int RG, typename WT, int NW, class WS>
__device__ __forceinline__ bool bellman_ford(const SubNet &N, const WS &W, int nct, int nz, int mode, int64_t M,
                                    bool warm = false, bool preds = false) {
    using B = Blk<NW>;
    const int nn = N.n + 2;
    for (int v = B::tid(); v < nn; v += B::T) {
        if (!warm) W.key[v] = (mode == kSsp) ? (v == N.n ? 0 : WS::kKInf) : 0;
        W.pred[v] = kNoPred;
    }
    ChainRegs<RG, WT> C;
    load_chain_regs<RG, WT, NW>(W, N.n, nct, mode, M, C);
    B::sync();
    bool converged;
    if constexpr (NW == 1 && WS::kWL) {
        // a warm start resumes from the groups its callers marked (wl_mark), a cold one
        // relaxes every group; the marks restart for the next call
        uint32_t df = 0xFFFFu, db = 0xFFFFu;
        if (warm) {
            df = uni((uint32_t)W.misc[1]);
            db = uni((uint32_t)W.misc[2]);
        }
        wave_lds_sync();
        if (lane() == 0) { W.misc[1] = 0; W.misc[2] = 0; }
        wave_lds_sync();
        converged = bf_converge_wl<RG, WT>(N, W, nct, nz, mode, C, df, db);
    } else {
        converged = bf_converge<RG, WT, NW>(N, W, nct, nz, mode, M, C);
    }
    if (!converged) return false;
    if (mode != kSsp) {
        // potentials; with preds (the warm start's repair): the tight in-arcs under the
        // potential mode's Z arcs
        if (preds) {
            if constexpr (WS::kAllReg) ssp_preds_regs<RG, WT, NW>(N, W, nct, nz, C, mode);
            else ssp_preds<NW>(N, W, nct, nz, M, mode);
        }
        return true;
    }
#ifdef SGUFP_SUB_VERIFY
    // Debug build: the labels a warm start converged to must equal those of a cold
    // Bellman-Ford from Z_out alone (invalidate_subtrees' exactness argument, checked).
    if (warm) {
        for (int v = B::tid(); v < nn; v += B::T) {
            W.vkey[v] = W.key[v];
            W.key[v] = (v == N.n) ? 0 : WS::kKInf;
        }
        B::sync();
        const bool cold_ok = bf_converge<RG, WT, NW>(N, W, nct, nz, mode, M, C);
        uint32_t diff = cold_ok ? 0u : 1u;
        for (int v = B::tid(); v < nn; v += B::T) diff |= (W.vkey[v] != W.key[v]) ? 1u : 0u;
        if (B::any(diff, W.red) && B::tid() == 0) W.misc[6] = 1;
        B::sync();
    }
#endif
    // one wave with every chain group in registers: predecessors from the registers
    if constexpr (WS::kAllReg) ssp_preds_regs<RG, WT, NW>(N, W, nct, nz, C);
    else ssp_preds<NW>(N, W, nct, nz, M);
    return true;
}

template <class WS>
__device__ __forceinline__ int64_t key_cost(typename WS::Key k) { return (int64_t)(k >> WS::kHop); }

// After an augmentation along the predecessor path of Z_in, whose used-up arcs (those whose
// residual segment the bottleneck exhausted: the arc vanishes or its big-M cost changes)
// already had their heads' keys set to infinity by the caller: every node whose predecessor-
// tree path crosses one of them restarts at infinity, the others keep their keys.  Those are
// still the shortest: the tree path survives, and SSP keys never decrease -- also in (cost,
// hops) order, since a new path uses reverse arcs of the augmenting path, which come back
// at equal cost with more hops.  Pointer jumping over the tree: each 16-bit word holds an
// ancestor anc(v) (15 bits) and a flag D(v) = "some node on the tree path v..anc(v), both
// ends included, is dead (infinite key)".  A jump combines two words, (anc(a), D(v)|D(a))
// with a = anc(v), which is again such a pair, so a lane may read any mix of this and the
// previous round's words (other lanes and waves write concurrently; a 16-bit LDS word is read
// and written whole): no double buffering, and each lane jumps kInvU nodes at once to overlap
// their LDS round trips.  Once no pointer moves, every anc(v) is a root and D(v) covers the
// whole path.
#ifndef SGUFP_INV_U
#define SGUFP_INV_U 4
#endif
constexpr int kInvU = SGUFP_INV_U;
template <int NW, class WS>
__device__ __forceinline__ void invalidate_subtrees(const SubNet &N, const WS &W) {
    using B = Blk<NW>;
    constexpr auto kKInf = WS::kKInf;
    const int nn = N.n + 2;
    LDS uint16_t *anc = W.plist;
    for (int v = B::tid(); v < nn; v += B::T) {
        const int32_t pr = W.pred[v];
        const int a = pr == kNoPred ? v : (pr & 0x7FFF);
        const bool dead = W.key[v] >= kKInf || W.key[a] >= kKInf;
        anc[v] = (uint16_t)(a | (dead ? 0x8000 : 0));
    }
    B::sync();
    for (int r = 0; r < 32; r++) {
        uint32_t moved = 0;
        for (int base = B::tid(); base < nn; base += kInvU * B::T) {
            uint32_t w[kInvU], wa[kInvU];
#pragma unroll
            for (int k = 0; k < kInvU; k++) {
                const int v = base + k * B::T;
                w[k] = v < nn ? (uint32_t)anc[v] : 0u;
            }
#pragma unroll
            for (int k = 0; k < kInvU; k++) wa[k] = anc[w[k] & 0x7FFFu];
#pragma unroll
            for (int k = 0; k < kInvU; k++) {
                const int v = base + k * B::T;
                if (v < nn && (wa[k] & 0x7FFFu) != (w[k] & 0x7FFFu)) {
                    anc[v] = (uint16_t)((wa[k] & 0x7FFFu) | ((w[k] | wa[k]) & 0x8000u));
                    moved = 1;
                }
            }
        }
        B::sync();
        if (!B::any(moved, W.red)) break;
    }
    uint32_t mf = 0, mb = 0;   // work list: the arcs into a restarted node (forward: chains with
                               // head v, backward: chains with tail v)
    for (int v = B::tid(); v < nn; v += B::T)
        if (anc[v] & 0x8000u) {
            W.key[v] = kKInf;
            if constexpr (WS::kWL) {
                const uint32_t iv = W.inc[v];
                mf |= iv >> 16;
                mb |= iv & 0xFFFFu;
            }
        }
    if constexpr (WS::kWL) wl_mark(W, mf, mb);
    B::sync();
}

// ---------------------------------------------------------------------------------------
__device__ __forceinline__ bool is_cons(const SubNet &N, int v) { return N.inner[v] && !N.vbar[v]; }
#ifndef SGUFP_REPAIR_MULTI
#define SGUFP_REPAIR_MULTI 16   // augmentations along one predecessor tree (1: one per Bellman-Ford)
#endif
constexpr int kRepairMulti = SGUFP_REPAIR_MULTI;

// Warm start.  The chains of a new path start from an earlier optimal state of the same
// scenario (flow per arc, potentials alpha): a chain keeps the smallest earlier flow of its
// arcs, then its reduced reward E = R - alpha(h) + alpha(t) under the old potentials fixes it
// -- E > 0: x = U, E < 0: x = 0, E = 0: kept within [0, U] -- so every residual arc has a
// non-negative reduced cost (no negative cycle: the pseudoflow is optimal for its imbalances).
// Chains that did not change keep their flow, so only the nodes around the changed V-bar
// matchings are out of balance.  The repair is successive shortest paths from the excess to
// the deficit nodes (potential mode: every free node is tied to Z both ways at cost 0, so
// free supply / demand absorbs anything):
//   stage 0: multi-source Bellman-Ford from every excess node (key 0), augment towards the
//            closest deficit node or Z (absorbed by a free node);
//   stage 1: from Z (free supply) to the remaining deficit nodes.
// Each augmentation is a shortest path of the extended network (super source -> sources at
// cost 0, targets -> super sink at cost 0), so the residual stays free of negative cycles and
// the repaired flow is optimal.  Between augmentations the Bellman-Ford resumes from its
// labels as the cold SSP does: the heads of used-up arcs and a source whose excess is gone
// restart at infinity with their predecessor subtrees (invalidate_subtrees).  Returns false
// (the caller falls back to the cold SSP) if a target is unreachable or the augmentation
// bound is hit (why: 1 Bellman-Ford, 2 unreachable, 3 path, 4 bound); neither happens with
// lower bounds 0.  With lower bounds the flows stay within [max l, min u] throughout (the
// potential mode's residual arcs), so a repaired flow meets every bound; a deficit no excess
// can reach within the bounds (the scenario may be infeasible for the new path) falls back to
// the cold SSP, whose big-M costs find the ray.  Only the WARM instantiations of
// k_sub_scenario carry it (launches with warm starts); the cold ones are unchanged.
template <int RG, typename WT, int NW, class WS>
__device__ __forceinline__ bool warm_repair(const SubNet &N, const WS &W, int nct, int nz, int64_t M,
                                                      LDS int32_t *imb, int64_t max_aug, int &augs, int &why,
                                                      uint64_t *tw) {
    using B = Blk<NW>;
#ifdef SGUFP_SUB_PHASES
    uint64_t t0 = wall_clock64();
#define WR_T(k) { const uint64_t t1 = wall_clock64(); tw[k] += t1 - t0; t0 = t1; }
#else
#define WR_T(k)
#endif
    using KT = typename WS::Key;
    constexpr KT kKInf = WS::kKInf;
    const int n = N.n, m = N.m;
    const int tid = B::tid();
    constexpr int T = B::T;
    // conservation nodes among this thread's nodes tid + j T (n + 2 <= 32 T: host), so the
    // loops below test a register bit instead of loading inner / vbar
    uint32_t cm = 0;
    for (int v = tid, j = 0; v < n; v += T, j++) cm |= (is_cons(N, v) ? 1u : 0u) << j;
    auto cons = [&](int j) -> bool { return (cm >> j) & 1u; };
    for (int stage = 0; stage < 2; stage++) {
        bool fresh = true;
        for (;;) {
            uint32_t left = 0;
            for (int v = tid, j = 0; v < n; v += T, j++)
                if (cons(j) && (stage == 0 ? imb[v] > 0 : imb[v] < 0)) left = 1;
            if (!B::any(left, W.red)) break;
            if (fresh) {
                for (int v = tid, j = 0; v < n + 2; v += T, j++) {
                    KT k = kKInf;
                    if (stage == 0 ? (v < n && cons(j) && imb[v] > 0) : v == n) k = 0;
                    W.key[v] = k;
                }
                if constexpr (WS::kWL)   // new keys everywhere: every group
                    if (tid == 0) { W.misc[1] = 0xFFFF; W.misc[2] = 0xFFFF; }
                B::sync();
                fresh = false;
            }
            WR_T(3);
            if (!bellman_ford<RG, WT, NW>(N, W, nct, nz, kPotPlain, M, true, true)) { why = 1; return false; }
            WR_T(0);
            // every target the predecessor tree reaches, closest first (key, then node id):
            // deficit nodes, and Z in stage 0.  The first one's tree path is a shortest path of
            // the extended network; the labels stay feasible potentials after it (its reverse
            // arcs come back tight), so the tree paths of the further targets -- tight arcs --
            // are shortest paths as well as long as every arc on them still has residual
            // capacity and their source still has excess (the primal-dual step of several
            // augmentations per Bellman-Ford); one whose path ran dry waits for the next one.
            int64_t last = INT64_MIN;
            for (int rep = 0; rep < kRepairMulti; rep++) {
                int64_t best = INT64_MAX;
                for (int v = tid, j = 0; v <= n; v += T, j++) {
                    const bool tgt = v < n ? (cons(j) && imb[v] < 0) : stage == 0;
                    const KT k = W.key[v];
                    if (tgt && k < kKInf) {
                        // (key, node) in one int64: potential-mode keys carry no big-M (|cost| <=
                        // sum |r|, so |key| < 2^35 with 64-bit keys, < 2^30 with 32-bit ones), ids
                        // < 2^15
                        const int64_t c = (int64_t)k * 32768 + v;
                        if (c > last) best = c < best ? c : best;
                    }
                }
                best = B::all(best, [](int64_t x, int64_t y) { return x < y ? x : y; }, W.red);
                if (best == INT64_MAX) {
                    if (rep == 0) { why = 2; return false; }
                    break;
                }
                last = best;
                const int tgt = (int)(best & 32767);
                if (tid == 0) {
                    int v = tgt, len = 0;
                    while (len < n + 2) {
                        const int32_t pr = W.pred[v];
                        if (pr == kNoPred) break;
                        W.plist[len++] = (uint16_t)(pr >> 15);
                        v = (int)(pr & 0x7FFF);
                    }
                    W.misc[3] = len;
                    W.misc[4] = v;
                }
                B::sync();
                const int plen = W.misc[3], src = W.misc[4];
                const bool src_ok = stage == 0 ? (src < n && is_cons(N, src) && imb[src] > 0) : src == n;
                int64_t delta = kInf;
                for (int i = tid; i < plen; i += T) {
                    const int code = W.plist[i];
                    if (code >= 2 * m) continue;   // Z arcs: uncapacitated
                    const uint64_t cb = W.rb(code >> 1);
                    const int64_t x = ch_x(cb), L = ch_L(cb), U = ch_U(cb);   // (compact: L = 0)
                    const int64_t cap = (code & 1) ? x - L : U - x;           // potential mode: [L, U]
                    delta = cap < delta ? cap : delta;
                }
                delta = B::all(delta, [](int64_t p, int64_t q) { return p < q ? p : q; }, W.red);
                if (stage == 0 && src_ok) delta = (int64_t)imb[src] < delta ? (int64_t)imb[src] : delta;
                if (tgt < n) delta = (int64_t)(-imb[tgt]) < delta ? (int64_t)(-imb[tgt]) : delta;
                if (!src_ok || plen >= n + 2 || delta <= 0 || delta >= kInf) {
                    if (rep == 0) { why = 3; return false; }
                    B::sync();
                    continue;
                }
                B::sync();   // every lane read the imbalances before they change
                uint32_t pm = 0;   // work list: the path's chains changed their residual arcs
                for (int i = tid; i < plen; i += T) {
                    const int code = W.plist[i];
                    if (code >= 2 * m) continue;
                    const int k = code >> 1;
                    const uint64_t ca = W.ra(k), cb = W.rb(k);
                    const int64_t x = ch_x(cb), L = ch_L(cb), U = ch_U(cb);
                    const int64_t cap = (code & 1) ? x - L : U - x;
                    W.add_x(k, (int)((code & 1) ? -delta : delta));
                    if (cap == delta) W.key[(code & 1) ? ch_t(ca) : ch_h(ca)] = kKInf;   // segment used up
                    pm |= 1u << ((k >> 6) & 31);
                }
                if constexpr (WS::kWL) wl_mark(W, pm, pm);
                if (tid == 0) {
                    if (stage == 0) {
                        imb[src] -= (int32_t)delta;
                        if (imb[src] == 0) W.key[src] = kKInf;   // no longer a source
                    }
                    if (tgt < n) imb[tgt] += (int32_t)delta;
                }
                B::sync();
                if (++augs > max_aug) { why = 4; return false; }
            }
            WR_T(1);
            invalidate_subtrees<NW>(N, W);
            // a source reached from another source (cheaper than its own key 0) hangs in that
            // one's predecessor tree: when that source runs dry the invalidation drops it too,
            // so every remaining source (and Z) restarts from 0 at most
            uint32_t mf = 0, mb = 0;   // work list: the arcs out of a re-seeded source
            for (int v = tid, j = 0; v <= n; v += T, j++) {
                const bool src = stage == 0 ? (v < n && cons(j) && imb[v] > 0) : v == n;
                if (src && W.key[v] > (KT)0) {
                    W.key[v] = (KT)0;
                    if constexpr (WS::kWL) {
                        const uint32_t iv = W.inc[v];
                        mf |= iv & 0xFFFFu;
                        mb |= iv >> 16;
                    }
                }
            }
            if constexpr (WS::kWL) wl_mark(W, mf, mb);
            B::sync();
            WR_T(2);
        }
    }
#undef WR_T
    return true;
}

// ---------------------------------------------------------------------------------------
// Dual assembly for one chain a_1..a_k.  e_a = r_a - P_a - V_a is the arc's reduced reward
// (gamma - beta); P_a = alpha(head) - alpha(tail) with alpha = 0 at free and V-bar nodes;
// V_a collects lambda - mu (matched pairs, transfer t), sigma (unmatched in-arc of a V-bar
// head), phi (unchosen out-arc of a V-bar tail).  Targets: a complete chain puts all of
// E = sum r - alpha(h) + alpha(t) on its binding arc (min u if E > 0, max l if E < 0); a
// chain fixed at 0 keeps e = 0 and lets sigma (broken end) or phi (broken start) absorb
// the rest (e <= 0 there).  Ray mode uses r = 0 and the given targets.
struct ChainOut {
    int64_t rhs;     // sum (u gamma - l beta) + sum (u_iq lambda + u_qj mu)
    int64_t obj;     // sum (u gamma - l beta): the dual objective at y-bar
};

template <class WS>
__device__ __forceinline__ void add_coef(const WS &W, int s, int64_t v) {
    // integers (the row's doubles: values far below 2^53, so any summation order is exact)
    if (v == 0 || s < 0) return;
    if (W.use_acc) __hip_atomic_fetch_add(&W.acc[s], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else __hip_atomic_fetch_add(&W.coef[s], (double)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// slot of the root variable (layer, head(b)) for an out-arc b of the layer's V-bar node
__device__ __forceinline__ int slot_at(const SubNet &N, int layer, int b) {
    return layer >= 0 ? N.slot_off[layer] + N.orank[b] : -1;
}

// sigma on in-arc a of V-bar node q: every (i, q, j) of q gets u_iq * sigma (grb.cpp:257-266)
template <class WS>
__device__ __forceinline__ void add_sigma(const SubNet &N, const WS &W, int a, int64_t sig, int s) {
    if (sig == 0) return;
    const int q = N.head[a], layer = N.arc_layer[a];
    const int64_t u = N.ub[(size_t)s * N.m + a];
    for (int k = N.out_off[q]; k < N.out_off[q + 1]; k++) add_coef(W, slot_at(N, layer, N.out_list[k]), u * sig);
}
// phi on out-arc b of V-bar node q: every (i, q, j) of q gets u_qj * phi (grb.cpp:268-277)
template <class WS>
__device__ __forceinline__ void add_phi(const SubNet &N, const WS &W, int b, int64_t ph, int s) {
    if (ph == 0) return;
    const int q = N.tail[b];
    const int64_t u = N.ub[(size_t)s * N.m + b];
    for (int k = N.in_off[q]; k < N.in_off[q + 1]; k++) add_coef(W, slot_at(N, N.arc_layer[N.in_list[k]], b), u * ph);
}

// alpha of node v (-1: none); k_sub_scenario leaves 0 at free and V-bar nodes
template <class WS>
__device__ __forceinline__ int64_t alpha_of(const SubNet &N, const WS &W, int v) {
    return v >= 0 ? (int64_t)W.alpha[v] : 0;
}

// Decision at the head of arc a from the path in HBM (phase 1 keeps it in LDS as dec; the
// dual assembly re-reads it, the LDS space being reused)
__device__ __forceinline__ int dec_of(const SubNet &N, const SubIO &io, int64_t poff, int64_t plen, int a) {
    const int q = N.head[a];
    if (!N.vbar[q]) return -2;
    const int l = N.arc_layer[a];
    int d = (l >= 0 && l < plen) ? (int)io.paths[poff + l] : -1;
    if (d < -1 || d >= N.m || (d >= 0 && N.tail[d] != q)) d = -3;   // not an out-arc of q
    return d;
}

// ray_mode: r = 0; prescribed targets (ray_p / ray_q) for the chain that certifies an
// infeasibility up front.  The chain's arcs come from its path's list (k_sub_paths); they are
// walked twice without per-arc arrays (a lane's chain of up to 63 arcs would otherwise live in
// scratch memory): the first walk gets its length, reward sum, binding arcs and the transfer
// total of a broken start; the second emits e, the transfers of the matched pairs and sigma /
// phi, in the order of the closed forms below (all integers: any summation order is exact).
template <class WS>
__device__ __forceinline__ ChainOut assemble_chain(const SubNet &N, const WS &W, const GBL uint32_t *arcs,
                                                   const GBL int32_t *rws, int nl, int t, int h, int s, bool ray_mode,
                                                   int ray_p, int ray_q, bool &ok) {
    ChainOut o{0, 0};
    const size_t so = (size_t)s * N.m;
    // the chain's arcs in order, arcs[0 .. nl) with their rewards rws (k_sub_paths): arc id,
    // coefficient slot of the pair with the next arc, u, l (0 in the compact kernels: no lower
    // bounds, host) and r; walk 1 keeps the first two in registers for walk 2 (most chains
    // have one or two arcs)
    struct Arc {
        int a, slot;
        int64_t u, l, r;
    };
    auto load = [&](int i) -> Arc {
        const uint32_t w = arcs[i];
        Arc x;
        x.a = (int)(w & 0xffffu);
        x.slot = (int16_t)(w >> 16);
        x.u = N.ub[so + x.a];
        x.l = WS::kCompact ? 0 : N.lb[so + x.a];
        x.r = ray_mode ? 0 : rws[i];
        return x;
    };
    Arc c0{}, c1{};
    auto get = [&](int i) -> Arc { return i == 0 ? c0 : (i == 1 ? c1 : load(i)); };
    auto cost = [&](const Arc &x, int64_t e) -> int64_t { return e >= 0 ? x.u * e : x.l * e; };
    // prescribed targets: beta = 1 on the max-l arc (e - 1), gamma = 1 on the min-u arc (e + 1)
    const bool prescribed = ray_mode && ray_p >= 0;
    auto pres = [&](int a) -> int64_t { return prescribed ? (int64_t)(a == ray_q) - (int64_t)(a == ray_p) : 0; };
    // matched pair (x, y) at q = head(x) with transfer tt: lambda = max(tt, 0), mu = max(-tt, 0),
    // coefficient slot (layer(x), head(y)) from the list
    auto pair = [&](const Arc &x, const Arc &y, int64_t tt) {
        const int64_t lam = tt > 0 ? tt : 0, mu = tt < 0 ? -tt : 0;
        const int64_t v = x.u * lam + y.u * mu;
        o.rhs += v;
        add_coef(W, x.slot, -v);
    };
    // walk 1: length, sum r, first min-u / first max-l arc, sum_{i >= 1} (e_i - r_i)
    int len = 0, bmin = 0, bmax = 0;
    int64_t sumr = 0, dsum = 0, umin = 0, lmax = 0;
    for (int i = 0; i < nl; i++) {
        const Arc x = load(i);
        if (i == 0) c0 = x;
        else if (i == 1) c1 = x;
        if (len == 0 || x.u < umin) { umin = x.u; bmin = len; }
        if (len == 0 || x.l > lmax) { lmax = x.l; bmax = len; }
        sumr += x.r;
        if (len > 0) dsum += pres(x.a) - x.r;
        if (++len >= kMaxChain) { ok = false; return o; }
    }
    const bool complete = t >= 0 && h >= 0;
    Arc x = c0, y{};
    if (complete) {
        // all of E = sum r - alpha(h) + alpha(t) on the binding arc (min u if E > 0, max l if
        // E < 0); transfers t_i = r_i - e_i + t_{i-1} from t_0 = r_0 + alpha(t) - e_0
        const int64_t E = sumr - alpha_of(N, W, h) + alpha_of(N, W, t);
        const int bind = E > 0 ? bmin : bmax;
        int64_t tp = 0;
        for (int i = 0; i < nl; i++) {
            const bool more = i + 1 < nl;
            if (more) y = get(i + 1);
            int64_t e = pres(x.a);
            if (!prescribed && i == bind && E != 0) e = E;
            o.obj += cost(x, e);
            if (more) {
                tp = (i == 0) ? x.r + alpha_of(N, W, t) - e : x.r - e + tp;
                pair(x, y, tp);
            }
            x = y;
        }
    } else if (h < 0) {
        // broken end: forward transfers, sigma at the unmatched last in-arc absorbs (e <= 0)
        int64_t tp = 0;
        for (int i = 0; i < nl; i++) {
            const bool more = i + 1 < nl;
            if (more) y = get(i + 1);
            const int64_t P = (i == 0) ? -alpha_of(N, W, t) : 0;
            int64_t e = pres(x.a);
            if (more) {
                tp = x.r - P - e + tp;
                pair(x, y, tp);
            } else {
                const int64_t free_e = x.r - P + tp;     // e with sigma = 0
                int64_t sig;
                if (prescribed) sig = free_e - e;
                else { sig = free_e > 0 ? free_e : 0; e = free_e - sig; }
                if (sig < 0) ok = false;
                add_sigma(N, W, x.a, sig, s);
            }
            o.obj += cost(x, e);
            x = y;
        }
    } else {
        // broken start only: backward transfers t_{j} = sum_{i > j} (e_i - r_i) + alpha(h),
        // i.e. T - sum_{1 <= i <= j} (e_i - r_i); phi at the unchosen first out-arc absorbs
        const int64_t T = len >= 2 ? dsum + alpha_of(N, W, h) : 0;
        int64_t pre = 0;
        for (int i = 0; i < nl; i++) {
            const bool more = i + 1 < nl;
            if (more) y = get(i + 1);
            int64_t e = pres(x.a);
            if (i == 0) {
                const int64_t P0 = (len == 1) ? alpha_of(N, W, h) : 0;
                const int64_t free_e = x.r - P0 - T;       // e with phi = 0
                int64_t ph;
                if (prescribed) ph = free_e - e;
                else { ph = free_e > 0 ? free_e : 0; e = free_e - ph; }
                if (ph < 0) ok = false;
                add_phi(N, W, x.a, ph, s);
            } else {
                pre += e - x.r;
            }
            o.obj += cost(x, e);
            if (more) pair(x, y, T - pre);
            x = y;
        }
    }
    o.rhs += o.obj;
    return o;
}

// A path's slice of the decisions (io.paths)
__device__ __forceinline__ void path_span(const SubIO &io, int p, int64_t &poff, int64_t &plen) {
    if (io.path_slot) {
        const int sl = io.path_slot[p];
        poff = (int64_t)sl * io.path_stride;
        plen = io.path_len[sl];
    } else {
        poff = io.path_off[p];
        plen = io.path_off[p + 1] - poff;
    }
}

}  // namespace

// ---------------------------------------------------------------------------------------
template <int RG, typename WT, int NW, typename KT, bool ALLREG, bool WARM = false>
__global__ void __launch_bounds__(kWave * NW, NW == 1 ? (sizeof(KT) == 4 ? 4 : 3) : (sizeof(KT) == 4 ? 4 : 1)) k_sub_scenario(SubNet N, SubIO io) {
    using WS = SubLds<KT, ALLREG, NW == 1>;
    using B = Blk<NW>;
    const int tid = B::tid();
    constexpr int T = B::T;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    LDS uint8_t *smem = (LDS uint8_t *)smem_raw;
    const int S = N.S;
    const int p = blockIdx.x / S, s = blockIdx.x - p * S;
    if (p >= io.n_paths) return;
    size_t off[kSubLdsParts];
    sub_lds_layout(N.n, N.m, io.nct_cap, N.nz, NW, off, (int)sizeof(KT), WARM, WS::kWL);
    WS W;
    W.inc = (LDS uint32_t *)(smem + off[11]);
    W.imb = (LDS int32_t *)(smem + off[0]);
    W.cta = (LDS uint64_t *)(smem + off[1]);
    W.ctb = (LDS typename WS::CBT *)(smem + off[2]);
    W.key = (LDS KT *)(smem + off[3]);
    W.alpha = W.key;
    W.pred = (LDS int32_t *)(smem + off[4]);
    W.plist = (LDS uint16_t *)(smem + off[8]);
    W.coef = io.coef + ((size_t)p * S + s) * N.n_slots;
    W.acc = nullptr;
    W.use_acc = false;
    W.zlist = (LDS int32_t *)(smem + off[6]);
    W.misc = (LDS int32_t *)(smem + off[7]);
    W.red = (LDS int64_t *)(smem + off[10]);
#ifdef SGUFP_SUB_VERIFY
    W.vkey = (LDS KT *)(smem + off[9]);
#endif
    const int n = N.n, m = N.m;
    const size_t so = (size_t)s * m;
    const size_t b = (size_t)p * S + s;
    // warm start: the source slot's state of this scenario, if its solve stored one
    const int wsrc = (WARM && io.warm_src) ? io.warm_src[p] : -1;
    const int wdst = (WARM && io.warm_dst) ? io.warm_dst[p] : -1;
    const bool wok = wsrc >= 0 && io.wst_ok[(size_t)wsrc * S + s];
    const GBL int16_t *xprev = wok ? io.wst_x + ((size_t)wsrc * S + s) * m : nullptr;
    const GBL int32_t *aprev = wok ? io.wst_a + ((size_t)wsrc * S + s) * n : nullptr;

#ifdef SGUFP_SUB_PHASES
    uint64_t tph[6];
    uint64_t twr[4] = {0, 0, 0, 0};   // warm repair: Bellman-Fords, augmentations, invalidation, checks
    tph[0] = wall_clock64();
#define SUB_PH(k) tph[k] = wall_clock64()
#else
#define SUB_PH(k)
    uint64_t *twr = nullptr;
#endif
    // 1-2. the path's chains (k_sub_paths: numbered in the topological order of their first
    //      arc's tail, with ends, reward sums and arc lists) and the free-supply / free-demand
    //      nodes (structural, from the host; read by every pass)
    const size_t pcb = (size_t)p * m;
    const int perr = io.pc_info[2 * p + 1];
    const int nct = perr ? 0 : io.pc_info[2 * p];
    if (tid < 8) W.misc[tid] = (tid == 0 && perr) ? 1 : 0;
    const int nz = N.nz;
    for (int i = tid; i < nz; i += T) W.zlist[i] = N.zlist[i];
    int first_bad = INT_MAX;   // first chain (rank) that makes the scenario infeasible up front
    for (int k = tid; k < nct; k += T) {
        const uint32_t th = io.pc_th[pcb + k], ol = io.pc_ol[pcb + k];
        const int t = (int16_t)(th & 0xffffu), h = (int16_t)(th >> 16), len = (int)(ol >> 16);
        const GBL uint32_t *arcs = io.pc_arcs + pcb + (ol & 0xffffu);
        const int R = io.pc_R[pcb + k];
        const int first = (int)(arcs[0] & 0xffffu);
        int L = WS::kCompact ? 0 : N.lb[so + first], U = N.ub[so + first];   // (compact: no lower bounds)
        int xw = xprev ? (int)xprev[first] : 0;   // warm start: the smallest earlier flow of the chain's arcs
        for (int i = 1; i < len; i++) {
            const int a = (int)(arcs[i] & 0xffffu);
            if (!WS::kCompact) L = max(L, (int)N.lb[so + a]);
            U = min(U, (int)N.ub[so + a]);
            if (xprev) xw = min(xw, (int)xprev[a]);
        }
        const bool complete = t >= 0 && h >= 0;
        int x0 = 0;
        if (xprev && complete) {
            // reduced reward under the earlier potentials (alpha 0 at free / V-bar nodes); the
            // flow goes to the bound it favours within [max l, min u] (a chain with max l >
            // min u is infeasible up front, first_bad below, and never solved)
            const int64_t E = (int64_t)R - (int64_t)aprev[h] + (int64_t)aprev[t];
            x0 = E > 0 ? U : (E < 0 ? L : max(L, min(xw, U)));
        }
        W.wa(k, pack_a(t, h, R));
        W.wb(k, pack_b(L, U, x0, first));   // compact: L = 0 (host), no first arc
        if ((complete && L > U) || (!complete && L > 0)) first_bad = min(first_bad, k);
    }
    first_bad = B::all(first_bad, [](int x, int y) { return x < y ? x : y; }, W.red);
    B::sync();
    if constexpr (WS::kWL) {
        // work list: per node the groups of the complete chains out of it / into it
        for (int v = tid; v < n + 2; v += T) W.inc[v] = 0;
        B::sync();
        for (int k = tid; k < nct; k += T) {
            const uint64_t ca = W.ra(k);
            const int t = ch_t(ca), h = ch_h(ca);
            if (t >= 0 && h >= 0) {
                __hip_atomic_fetch_or(&W.inc[t], 1u << (k >> 6), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_or(&W.inc[h], 1u << (16 + (k >> 6)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        B::sync();
        if constexpr (WS::kCoarse) {
            // per group: the groups of the arcs out of its chains' heads (a forward relaxation
            // lowers a head) and out of their tails (a backward one lowers a tail)
            for (int g = 0; g * kWave < nct; g++) {
                const int k = g * kWave + lane();
                uint32_t mh = 0, mt = 0;
                if (k < nct) {
                    const uint64_t ca = W.ra(k);
                    const int t = ch_t(ca), h = ch_h(ca);
                    if (t >= 0 && h >= 0) { mh = W.inc[h]; mt = W.inc[t]; }
                }
                mh = uni(wave_or(mh));
                mt = uni(wave_or(mt));
                if (lane() == 0) { W.inc[n + 2 + g] = mh; W.inc[n + 2 + 16 + g] = mt; }
            }
            B::sync();
        }
    }
    // The reference returns at the first infeasible scenario (grb.cpp:284-351): only its ray
    // reaches the cut.  A scenario infeasible up front records itself in first_inf[p]; one that
    // finds an earlier infeasible scenario of its path recorded stops (kSubSkipped), here or
    // between its augmentations below.  (The cut is the same whichever later scenarios stop.)
    auto skip_now = [&]() -> bool {
        if (!io.first_inf) return false;
        int fi = __hip_atomic_load(&io.first_inf[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        fi = B::all(fi, [](int x, int y) { return x < y ? x : y; }, W.red);
        return fi < s;
    };
    auto skip_out = [&]() {
        if (tid == 0) {
            io.status[b] = kSubSkipped;
            io.obj[b] = 0;
            io.dual[b] = 0;
            io.rhs[b] = 0;
            if (io.wstat) { io.wstat[2 * b] = 0; io.wstat[2 * b + 1] = 0; }
            if (wdst >= 0) io.wst_ok[(size_t)wdst * S + s] = 0;
        }
    };
    if (io.first_inf && first_bad != INT_MAX && tid == 0) atomicMin(&io.first_inf[p], s);
    if (skip_now()) {
        skip_out();
        return;
    }
    // phase 5 sums the cut row in LDS when it fits over the chain records (int64 per slot) and
    // the chains' flows fit the predecessor / path / imbalance space (int16 per chain)
#ifdef SGUFP_SUB_NO_LACC
    const bool lacc = false;   // A/B: atomic adds into the HBM row
#else
    const bool lacc = (size_t)N.n_slots * 8 <= off[3] - off[1] && (size_t)nct * 2 <= off[5] - off[4];
#endif
    if (!lacc) {
        for (int v = tid; v < N.n_slots; v += T) W.coef[v] = 0.0;
        __threadfence();   // zeros stored before any lane's atomic adds of phase 5
    }
    B::sync();
    if (W.misc[0]) {
        if (tid == 0) { io.status[b] = kSubError; io.obj[b] = 0; io.dual[b] = 0; io.rhs[b] = 0; }
        for (int v = tid; v < N.n_slots; v += T) io.coef[b * N.n_slots + v] = 0.0;
        return;
    }

    // warm start: node imbalances of the initial flow (conservation rows only)
    LDS int32_t *imb = W.imb;
    if (xprev) {
        for (int v = tid; v < n + 2; v += T) imb[v] = 0;
        B::sync();
        for (int k = tid; k < nct; k += T) {
            const uint64_t ca = W.ra(k);
            const int t = ch_t(ca), h = ch_h(ca), x = ch_x(W.rb(k));
            if (t >= 0 && h >= 0 && x) {
                __hip_atomic_fetch_add(&imb[h], x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_add(&imb[t], -x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        B::sync();
    }

    int status = kSubOptimal;
    int64_t M = 0, max_aug = 0;
    for (int k = tid; k < nct; k += T) {
        const uint64_t ca = W.ra(k);
        if (ch_t(ca) >= 0 && ch_h(ca) >= 0) {
            const int64_t R = ch_R(ca), U = ch_U(W.rb(k));
            M += 2 * (R < 0 ? -R : R) * (U + 1);
            max_aug += U > 0 ? U : 0;
        }
    }
    M = 1 + B::all(M, [](int64_t x, int64_t y) { return x + y; }, W.red);
    // Every augmentation moves delta >= 1 more units from Z_out to Z_in, and that flow
    // crosses at least one complete chain, so the number of augmentations is at most the
    // sum of the chains' capacities (min u): the loop below stops after that many.
    max_aug = B::all(max_aug, [](int64_t x, int64_t y) { return x + y; }, W.red);
    int ray_chain = -1, ray_p = -1, ray_q = -1;
    int err_site = 0;   // which check failed (an error scenario reports it as its dual: diagnostics)
    int64_t primal = 0;

    if (WS::kCompact && first_bad != INT_MAX) {
        // compact records come with no lower bound and ub >= 0 (host): cannot happen
        status = kSubError;
        err_site = 8;
    } else if (first_bad != INT_MAX) {
        // (i) a chain fixed at 0 with a positive lower bound, or (ii) a chain with max l > min u
        status = kSubInfeasible;
        ray_chain = first_bad;
        const int k = first_bad;
        const uint32_t ol = io.pc_ol[pcb + k];
        const GBL uint32_t *arcs = io.pc_arcs + pcb + (ol & 0xffffu);
        const bool complete = ch_t(W.ra(k)) >= 0 && ch_h(W.ra(k)) >= 0;
        int bp = (int)(arcs[0] & 0xffffu), bq = bp;
        int64_t bl = N.lb[so + bp], bu = N.ub[so + bp];
        for (int i = 1; i < (int)(ol >> 16); i++) {
            const int a = (int)(arcs[i] & 0xffffu);
            const int64_t l = N.lb[so + a], u = N.ub[so + a];
            if (l > bl) { bl = l; bp = a; }
            if (u < bu) { bu = u; bq = a; }
        }
        if (complete) { ray_p = bp; ray_q = bq; }
        else { ray_p = bp; ray_q = -1; }
        B::sync();
        for (int v = tid; v <= n; v += T) W.alpha[v] = 0;
        B::sync();
    } else {
        SUB_PH(1);
        // 3. successive shortest paths (max reward) from the sources to the sinks
#ifdef SGUFP_SUB_TRACE
        const uint64_t tr0 = wall_clock64();
        uint64_t t_bf = 0, t_pred = 0, t_walk = 0, tq;
        int nbf = 0;
#define SUB_T0() tq = wall_clock64()
#define SUB_T1(acc) acc += wall_clock64() - tq
#else
#define SUB_T0()
#define SUB_T1(acc)
#endif
        int iters = 0;
        int warm_augs = 0, why = 0;
        bool repaired = false, fell_back = false;
#ifdef SGUFP_SUB_VERIFY
        int64_t verify_primal = INT64_MIN;
#endif
        if (xprev) {
            int64_t imb_tot = 0;
            for (int v = tid; v < n; v += T)
                if (is_cons(N, v)) imb_tot += imb[v] > 0 ? imb[v] : -imb[v];
            imb_tot = B::all(imb_tot, [](int64_t x, int64_t y) { return x + y; }, W.red);
            repaired = warm_repair<RG, WT, NW>(N, W, nct, nz, M, imb, imb_tot + 2 * (int64_t)nct + 8, warm_augs, why, twr);
#ifdef SGUFP_SUB_VERIFY
            if (repaired) {   // debug build: the cold SSP below must reach the same objective
                int64_t pw = 0;
                for (int k = tid; k < nct; k += T) {
                    const uint64_t ca = W.ra(k);
                    if (ch_t(ca) >= 0 && ch_h(ca) >= 0) pw += (int64_t)ch_R(ca) * ch_x(W.rb(k));
                }
                verify_primal = B::all(pw, [](int64_t x, int64_t y) { return x + y; }, W.red);
                repaired = false;
            }
#endif
            if (!repaired) {   // cold from zero flow
                fell_back = true;
                B::sync();
                for (int k = tid; k < nct; k += T) {
                    const int x = ch_x(W.rb(k));
                    if (x) W.add_x(k, -x);
                }
                B::sync();
            }
        }
        // Each round: Bellman-Ford labels and predecessors, stop when the shortest Z_out ->
        // Z_in path no longer gains, else augment along it.  After the first round the
        // Bellman-Ford resumes from the previous labels, with only the subtrees under the
        // used-up arcs restarted (invalidate_subtrees).  (Reusing the labels without any
        // Bellman-Ford while a tight residual path survives never found one on C3 / C4.)
        bool warm = false;
        bool skipped = false;
        for (; status == kSubOptimal && !repaired; iters++) {
            if ((iters & 7) == 7 && skip_now()) {
                skipped = true;
                break;
            }
            SUB_T0();
            if (!bellman_ford<RG, WT, NW>(N, W, nct, nz, kSsp, M, warm)) { status = kSubError; err_site = 1; break; }
            SUB_T1(t_bf);
#ifdef SGUFP_SUB_VERIFY
            if (W.misc[6]) { status = kSubError; break; }
#endif
            const KT kz = W.key[n + 1];
            if (kz >= WS::kKInf || key_cost<WS>(kz) >= 0) break;
            if (iters >= max_aug) { status = kSubError; err_site = 2; break; }   // cannot happen (bound above)
            // lane 0 chases the predecessors from Z_in back to Z_out into a list (one LDS
            // round trip per arc: the entry holds the tail), then the wave takes the
            // bottleneck and augments (a simple path uses each chain once)
            SUB_T0();
            if (tid == 0) {
                int v = n + 1, len = 0;
                while (v != n && len < n + 2) {
                    const int32_t pr = W.pred[v];
                    if (pr == kNoPred) break;
                    W.plist[len++] = (uint16_t)(pr >> 15);
                    v = (int)(pr & 0x7FFF);
                }
                W.misc[3] = (v == n) ? len : -1;
            }
            B::sync();
            const int plen = W.misc[3];
            int64_t delta = kInf;
            for (int i = tid; i < plen; i += T) {
                const int code = W.plist[i];
                if (code >= 2 * m) continue;   // Z arcs: uncapacitated
                const uint64_t cb = W.rb(code >> 1);
                const int64_t x = ch_x(cb), L = ch_L(cb), U = ch_U(cb);
                const int64_t cap = (code & 1) ? (x > L ? x - L : x) : (x < L ? L - x : U - x);
                delta = cap < delta ? cap : delta;
            }
            delta = B::all(delta, [](int64_t p, int64_t q) { return p < q ? p : q; }, W.red);
            if (plen < 0 || delta <= 0 || delta >= kInf) { status = kSubError; err_site = plen < 0 ? 3 : 4; break; }
            uint32_t pm = 0;   // work list: the path's chains changed their residual arcs
            for (int i = tid; i < plen; i += T) {
                const int code = W.plist[i];
                if (code >= 2 * m) continue;
                const int k = code >> 1;
                const uint64_t ca = W.ra(k), cb = W.rb(k);
                const int64_t x = ch_x(cb), L = ch_L(cb), U = ch_U(cb);
                const int64_t cap = (code & 1) ? (x > L ? x - L : x) : (x < L ? L - x : U - x);
                W.add_x(k, (int)((code & 1) ? -delta : delta));
                if (cap == delta) W.key[(code & 1) ? ch_t(ca) : ch_h(ca)] = WS::kKInf;   // segment used up
                pm |= 1u << ((k >> 6) & 31);
            }
            if constexpr (WS::kWL) wl_mark(W, pm, pm);
            B::sync();
            SUB_T1(t_walk);
            SUB_T0();
            invalidate_subtrees<NW>(N, W);
            warm = true;
            SUB_T1(t_pred);
#ifdef SGUFP_SUB_TRACE
            nbf++;
#endif
        }
#ifdef SGUFP_SUB_TRACE
        if (blockIdx.x % 997 == 0 && tid == 0)
            printf("SUB blk=%d nct=%d nz=%d aug=%d bf=%d passes=%d groups=%d ticks=%llu t_bf=%llu t_pred=%llu t_walk=%llu\n",
                   (int)blockIdx.x, nct, nz, iters, nbf, W.misc[5], W.misc[7], (unsigned long long)(wall_clock64() - tr0),
                   (unsigned long long)t_bf, (unsigned long long)t_pred, (unsigned long long)t_walk);
#endif
        if (skipped) {
            skip_out();
            return;
        }
        // lower bounds met?
        int unmet = 0;
        for (int k = tid; k < nct; k += T) {
            const uint64_t ca = W.ra(k), cb = W.rb(k);
            if (ch_t(ca) >= 0 && ch_h(ca) >= 0) {
                if (ch_x(cb) < ch_L(cb)) unmet = 1;
                primal += (int64_t)ch_R(ca) * ch_x(cb);
            }
        }
        primal = B::all(primal, [](int64_t x, int64_t y) { return x + y; }, W.red);
        unmet = (int)B::any((uint32_t)unmet, W.red);
#ifdef SGUFP_SUB_VERIFY
        if (verify_primal != INT64_MIN && verify_primal != primal && status == kSubOptimal) {
            status = kSubError;
            err_site = 9;
        }
#endif
        const int passes_flow = W.misc[5];
        if (io.wstat && tid == 0) {
            // fell back: -(why * 100000 + cold augmentations) - 1
            io.wstat[2 * b] = repaired ? warm_augs : (fell_back ? -(why * 100000 + iters) - 1 : iters);
            io.wstat[2 * b + 1] = passes_flow;
        }
        SUB_PH(2);
        if (status == kSubOptimal) {
            // 4. potentials of the final residual: plain costs (optimal duals) or big-M
            //    costs (their M-multiple is a dual ray, case (iii))
            const int mode = unmet ? kPotBigM : kPotPlain;
            if (unmet) {
                status = kSubInfeasible;
                if (io.first_inf && tid == 0) atomicMin(&io.first_inf[p], s);
            }
            if (!bellman_ford<RG, WT, NW>(N, W, nct, nz, mode, M)) { status = kSubError; err_site = 5; }
            const int64_t dz = key_cost<WS>(W.key[n]);
            B::sync();   // every thread read Z's key before the alphas overwrite it in place
            for (int v = tid; v < n; v += T) {
                int64_t d = key_cost<WS>(W.key[v]) - dz;
                int64_t al;
                if (mode == kPotPlain) al = -d;
                else {
                    const int64_t r = (d >= 0 ? d + M / 2 : d - M / 2) / M;   // round(d / M)
                    al = -r;
                }
                W.alpha[v] = (KT)((N.inner[v] && !N.vbar[v]) ? al : 0);
            }
            B::sync();
            // passes: the flow's (bits 0-19) and the potentials' (bits 20-30)
            if (io.wstat && tid == 0) io.wstat[2 * b + 1] = passes_flow | (min(W.misc[5] - passes_flow, 2047) << 20);
        }
    }

    // the final state for later warm starts: potentials now, flows per arc with the chain walk
    // below (zeros first: arcs outside complete chains carry none)
    const bool save = wdst >= 0 && status == kSubOptimal;
    GBL int16_t *xs = save ? io.wst_x + ((size_t)wdst * S + s) * m : nullptr;
    if (save) {
        GBL int32_t *as = io.wst_a + ((size_t)wdst * S + s) * n;
        for (int a = tid; a < m; a += T) xs[a] = 0;
        for (int v = tid; v < n; v += T) as[v] = (int32_t)W.alpha[v];
        __threadfence();
        B::sync();
    }

    SUB_PH(3);
    // 5. dual solution / ray and the scenario's cut contribution
    int64_t rhs = 0, dual = 0;
    bool ok = true;
    const bool run5 = status != kSubError;
    if (run5) {
        const bool ray = status == kSubInfeasible;
        // the flows of the complete chains (the warm save) move out of the chain records, whose
        // space then holds the LDS row; ends and arcs come from the path's lists
        LDS int16_t *xk = (LDS int16_t *)(smem + off[4]);
        if (lacc) {
            if (save)
                for (int k = tid; k < nct; k += T) {
                    const uint64_t ca = W.ra(k);
                    xk[k] = (ch_t(ca) >= 0 && ch_h(ca) >= 0) ? (int16_t)ch_x(W.rb(k)) : (int16_t)0;
                }
            B::sync();
            W.acc = (LDS int64_t *)(smem + off[1]);
            W.use_acc = true;
            for (int v = tid; v < N.n_slots; v += T) W.acc[v] = 0;
            B::sync();
        }
        for (int k = tid; k < nct; k += T) {
            if (ray && ray_chain >= 0 && k != ray_chain) continue;   // (i)/(ii): only the bad chain
            const uint32_t ol = io.pc_ol[pcb + k], th = io.pc_th[pcb + k];
            const GBL uint32_t *arcs = io.pc_arcs + pcb + (ol & 0xffffu);
            const int nl = (int)(ol >> 16);
            const int t = (int16_t)(th & 0xffffu), h = (int16_t)(th >> 16);
            ChainOut c = assemble_chain(N, W, arcs, io.pc_rw + pcb + (ol & 0xffffu), nl, t, h, s, ray,
                                        (k == ray_chain) ? ray_p : -1, (k == ray_chain) ? ray_q : -1, ok);
            rhs += c.rhs;
            dual += c.obj;
            if (save) {
                const int x = lacc ? (int)xk[k] : ((t >= 0 && h >= 0) ? ch_x(W.rb(k)) : 0);
                if (x)
                    for (int i = 0; i < nl; i++) xs[arcs[i] & 0xffffu] = (int16_t)x;
            }
        }
        rhs = B::all(rhs, [](int64_t x, int64_t y) { return x + y; }, W.red);
        dual = B::all(dual, [](int64_t x, int64_t y) { return x + y; }, W.red);
        ok = B::any(ok ? 0u : 1u, W.red) == 0;
        if (ray && ray_chain >= 0 && ray_p >= 0 && ray_p == ray_q) {
            // single arc with l > u: beta = gamma = 1 on it
            const int64_t d0 = (int64_t)N.ub[so + ray_p] - N.lb[so + ray_p];
            rhs += d0;
            dual += d0;
        }
        if (!ok || (ray ? dual >= 0 : dual != primal)) { status = kSubError; err_site = ok ? 6 : 7; }
    }
    B::sync();
    if (lacc)   // the row (zeros where phase 5 did not run)
        for (int v = tid; v < N.n_slots; v += T) W.coef[v] = run5 ? (double)W.acc[v] : 0.0;
    if (tid == 0) {
        io.status[b] = status;
        io.obj[b] = (double)primal;
        io.dual[b] = status == kSubError ? -(double)err_site : (double)dual;
        io.rhs[b] = (double)rhs;
        // the destination's state of this scenario is usable only if this solve stored it
        if (wdst >= 0) io.wst_ok[(size_t)wdst * S + s] = (save && status == kSubOptimal) ? 1 : 0;
    }
#ifdef SGUFP_SUB_PHASES
    SUB_PH(4);
    if (tid == 0 && blockIdx.x % 2047 == 0)
        printf("SUBPH warm=%d chains %llu flow %llu potentials %llu dual %llu (ticks) repair bf %llu aug %llu inv %llu chk %llu\n",
               xprev != nullptr, (unsigned long long)(tph[1] - tph[0]), (unsigned long long)(tph[2] - tph[1]),
               (unsigned long long)(tph[3] - tph[2]), (unsigned long long)(tph[4] - tph[3]),
               (unsigned long long)twr[0], (unsigned long long)twr[1], (unsigned long long)twr[2], (unsigned long long)twr[3]);
#endif
}

// Per path, once for all its scenarios: the chains (maximal runs of arcs joined by the path's
// decisions at V-bar nodes, grb.cpp's constraint (1) pairs), numbered in the topological order
// of their first arc's tail, each with its ends (t: -1 at a V-bar tail, h: -1 at an open end),
// reward sum and arcs in order (with the coefficient slot of each matched pair).  k_sub_scenario's phases 2 and 5 read these lists instead of
// walking the decisions per scenario (a dependent load per arc).  pc_info[2p + 1] flags a
// path that no exact DD could have produced: a decision that is not an out-arc of its node,
// two in-arcs choosing one out-arc, more chains than nct_cap or a chain over kMaxChain arcs.
// One wave per path; LDS: decisions, their inverse, the chains' first arcs (int16 each).
__global__ void __launch_bounds__(kWave) k_sub_paths(SubNet N, SubIO io) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    const int p = blockIdx.x;
    if (p >= io.n_paths) return;
    const int m = N.m, ln = lane();
    LDS int16_t *dec = (LDS int16_t *)smem_raw;
    LDS int16_t *chosen = dec + m, *first = chosen + m;
    int64_t poff, plen;
    path_span(io, p, poff, plen);
    bool err = false;
    for (int a = ln; a < m; a += kWave) {
        const int d = dec_of(N, io, poff, plen, a);
        chosen[a] = -1;
        dec[a] = (int16_t)d;
        err |= d == -3;
    }
    __syncthreads();
    for (int a = ln; a < m; a += kWave) {
        const int d = dec[a];
        if (d >= 0) chosen[d] = (int16_t)a;   // one of several writers wins ...
    }
    __syncthreads();
    for (int a = ln; a < m; a += kWave) {
        const int d = dec[a];
        err |= d >= 0 && chosen[d] != a;       // ... the others: two in-arcs chose one out-arc
    }
    int nct = 0;
    for (int base = 0; base < m; base += kWave) {
        const int a = base + ln < m ? N.arc_topo[base + ln] : -1;
        const bool st = a >= 0 && (!N.vbar[N.tail[a]] || chosen[a] < 0);
        const uint32_t incl = wave_scan_incl(st ? 1u : 0u);
        if (st) first[nct + (int)incl - 1] = (int16_t)a;
        nct += __builtin_amdgcn_readlane((int)incl, kWave - 1);
    }
    if (nct > io.nct_cap) { err = true; nct = io.nct_cap; }
    __syncthreads();
    const size_t pcb = (size_t)p * m;
    int run = 0;
    for (int base = 0; base < nct; base += kWave) {
        const int k = base + ln;
        int len = 0, t = -1, h = -1, R = 0, a = -1;
        if (k < nct) {
            a = first[k];
            const int t0 = N.tail[a];
            t = N.vbar[t0] ? -1 : t0;
            len = 1;
            R = N.reward[a];
            for (int e = a;;) {
                const int q = N.head[e];
                if (!N.vbar[q]) { h = q; break; }
                const int d = dec[e];
                if (d < 0) break;
                if (++len > kMaxChain) { err = true; break; }
                e = d;
                R += N.reward[e];
            }
        }
        const uint32_t incl = wave_scan_incl((uint32_t)len);
        const int o = run + (int)incl - len;
        if (k < nct && o + len <= m) {
            io.pc_th[pcb + k] = (uint32_t)(uint16_t)t | (uint32_t)(uint16_t)h << 16;
            io.pc_ol[pcb + k] = (uint32_t)o | (uint32_t)len << 16;
            io.pc_R[pcb + k] = R;
            for (int i = 0; i < len; i++) {
                const int b = i + 1 < len ? dec[a] : -1;
                const int slot = b >= 0 ? slot_at(N, N.arc_layer[a], b) : -1;
                io.pc_arcs[pcb + o + i] = (uint32_t)a | (uint32_t)(uint16_t)slot << 16;
                io.pc_rw[pcb + o + i] = N.reward[a];
                a = b;
            }
        }
        run += __builtin_amdgcn_readlane((int)incl, kWave - 1);
    }
    err = __builtin_amdgcn_ballot_w64(err) != 0;   // (a chain over kMaxChain arcs: its lane wrote
    if (ln == 0) {                                  //  no further than the first kMaxChain + 1)
        io.pc_info[2 * p] = nct;
        io.pc_info[2 * p + 1] = err ? 1 : 0;
    }
}

// Per path, in scenario order: the first infeasible scenario's ray (grb.cpp:288-350,
// rhs and coefficients reset, no 1/S), else sum_s contribution / S (grb.cpp:236-281).
__global__ void __launch_bounds__(256) k_sub_reduce(SubNet N, SubIO io) {
    const int p = blockIdx.x;
    if (p >= io.n_paths) return;
    const int S = N.S;
    __shared__ int first_inf, any_err;
    if (threadIdx.x == 0) { first_inf = INT_MAX; any_err = 0; }
    __syncthreads();
    for (int s = threadIdx.x; s < S; s += blockDim.x) {
        const int st = io.status[(size_t)p * S + s];
        if (st == kSubInfeasible) atomicMin(&first_inf, s);
        if (st == kSubError) atomicOr(&any_err, 1);
    }
    __syncthreads();
    const int stride = N.n_slots + 1;
    // a scenario before the first infeasible one that failed poisons the path
    bool err = false;
    if (any_err) {
        for (int s = 0; s < S && s <= first_inf && s < S; s++)
            if (io.status[(size_t)p * S + s] == kSubError) { err = true; break; }
    }
    if (err) {
        if (threadIdx.x == 0) { io.cut_type[p] = -1; io.cut_rhs[p] = 0; io.obj_mean[p] = 0; }
        for (int v = threadIdx.x; v < stride; v += blockDim.x) io.cut_row[(size_t)p * stride + v] = 0.0;
        return;
    }
    if (first_inf != INT_MAX) {
        const size_t b = (size_t)p * S + first_inf;
        if (threadIdx.x == 0) { io.cut_type[p] = 1; io.cut_rhs[p] = io.rhs[b]; io.obj_mean[p] = 0; }
        for (int v = threadIdx.x; v < stride; v += blockDim.x)
            io.cut_row[(size_t)p * stride + v] = v < N.n_slots ? io.coef[b * N.n_slots + v] : 0.0;
        return;
    }
    const double inv = (double)S;
    for (int v = threadIdx.x; v < stride; v += blockDim.x) {
        double acc = 0.0;
        if (v < N.n_slots)
            for (int s = 0; s < S; s++) acc += io.coef[((size_t)p * S + s) * N.n_slots + v] / inv;
        io.cut_row[(size_t)p * stride + v] = acc;
    }
    if (threadIdx.x == 0) {
        double r = 0.0, o = 0.0;
        for (int s = 0; s < S; s++) {
            r += io.rhs[(size_t)p * S + s] / inv;
            o += io.obj[(size_t)p * S + s] / inv;
        }
        io.cut_type[p] = 0;
        io.cut_rhs[p] = r;
        io.obj_mean[p] = o;
    }
}

// ---------------------------------------------------------------------------------------
// Warm-start donors (WarmRing): one workgroup per path of the launch.  Every valid ring slot
// outside this launch's destinations [ptr, ptr + n) is a candidate; the distance is the
// number of DD layers whose decisions differ (a missing entry counts as -1); ties go to the
// lowest slot.  Then the path is recorded in its destination slot (ptr + p) mod R.
__global__ void __launch_bounds__(256) k_warm_pick(SubIO io, WarmRing wr, int ptr) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    LDS int16_t *sp = (LDS int16_t *)smem_raw;                       // [Lcap]
    LDS unsigned long long *red = (LDS unsigned long long *)(smem_raw + (((size_t)wr.Lcap * 2 + 15) & ~(size_t)15));
    const int p = blockIdx.x;
    const int n = io.n_paths;
    if (p >= n) return;
    int64_t poff, plen;
    path_span(io, p, poff, plen);
    if (plen > wr.Lcap) plen = wr.Lcap;
    for (int l = threadIdx.x; l < wr.Lcap; l += blockDim.x) sp[l] = l < plen ? io.paths[poff + l] : (int16_t)-1;
    __syncthreads();
    unsigned long long best = ~0ull;
    for (int c = threadIdx.x; c < wr.R; c += blockDim.x) {
        const int rel = (c - ptr % wr.R + wr.R) % wr.R;
        if (rel < n || !wr.valid[c]) continue;
        const GBL int16_t *q = wr.path + (size_t)c * wr.Lcap;
        const int ql = wr.plen[c];
        const int L = ql > (int)plen ? ql : (int)plen;
        int d = 0;
        for (int l = 0; l < L; l++) d += (l < ql ? (int)q[l] : -1) != (int)sp[l];
        const unsigned long long key = (unsigned long long)d << 32 | (unsigned)c;
        best = key < best ? key : best;
    }
    red[threadIdx.x] = best;
    __syncthreads();
    for (int h = blockDim.x / 2; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) red[threadIdx.x] = red[threadIdx.x + h] < red[threadIdx.x] ? red[threadIdx.x + h] : red[threadIdx.x];
        __syncthreads();
    }
    const int dst = (ptr + p) % wr.R;
    if (threadIdx.x == 0) {
        const unsigned long long b = red[0];
        const int d = b == ~0ull ? -1 : (int)(b >> 32);
        wr.src[p] = (d >= 0 && d <= wr.max_dist) ? (int)(b & 0xFFFFFFFFull) : -1;
        wr.dst[p] = dst;
        wr.dist[p] = d;
        wr.plen[dst] = (uint16_t)plen;
        wr.valid[dst] = 1;
    }
    for (int l = threadIdx.x; l < wr.Lcap; l += blockDim.x) wr.path[(size_t)dst * wr.Lcap + l] = sp[l];
}

hipError_t launch_warm_pick(const SubIO &io, const WarmRing &wr, int ptr, hipStream_t st) {
    if (io.n_paths <= 0) return hipSuccess;
    const size_t lds = (((size_t)wr.Lcap * 2 + 15) & ~(size_t)15) + 256 * 8;
    hipLaunchKernelGGL(k_warm_pick, dim3((unsigned)io.n_paths), dim3(256), lds, st, io, wr, ptr);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
size_t sub_lds_bytes(int n, int m, int nct_cap, int nz, int nw, int kbytes, bool warm, bool wl) {
    size_t off[kSubLdsParts];
    return sub_lds_layout(n, m, nct_cap, nz, nw, off, kbytes, warm, wl);
}

namespace {
template <typename KT, bool WARM>
hipError_t launch_scenarios(const SubNet &N, const SubIO &io, hipStream_t st) {
    constexpr int kb = (int)sizeof(KT);
    constexpr bool kw = WARM;   // the warm layout (k_sub_scenario's)
    size_t lds = sub_lds_bytes(N.n, N.m, io.nct_cap, N.nz, 1, kb, kw, false);
    // the single-wave kernels with every chain group in registers carry the work-list table
#ifdef SGUFP_SUB_WL
    const size_t lds_wl = sub_lds_bytes(N.n, N.m, io.nct_cap, N.nz, 1, kb, kw, true);
#else
    const size_t lds_wl = lds;
#endif
#ifdef SGUFP_SUB_LDS_MIN
    if (lds < SGUFP_SUB_LDS_MIN) lds = SGUFP_SUB_LDS_MIN;   // occupancy experiments
#endif
    // the large variant (kLargeWaves waves per scenario, 32-bit costs in registers) once the
    // LDS allows at most two scenarios per CU (in its own layout: the single-wave 8-byte
    // records would bring C5 under the bar and back to one wave per scenario, 4x slower) and
    // the big-M costs fit 32 bits (host bound)
    const bool large = sub_lds_bytes(N.n, N.m, io.nct_cap, N.nz, kLargeWaves, kb, false, false) > 64 * 1024 &&
                       io.nct_cap > kRegGroupsSmall * kWave && N.cost_bound < ((int64_t)1 << 30);
    const char *ev = getenv("SGUFP_SUB_WAVES");
    if (large && !(ev && atoi(ev) == 1)) {
        lds = sub_lds_bytes(N.n, N.m, io.nct_cap, N.nz, kLargeWaves, kb, kw, false);
        if (io.nct_cap <= kRegGroupsLarge * kLargeWaves * kWave && !N.preds_lds)
            hipLaunchKernelGGL((k_sub_scenario<kRegGroupsLarge, int32_t, kLargeWaves, KT, true, WARM>),
                               dim3((unsigned)io.n_paths * N.S), dim3(kWave * kLargeWaves), lds, st, N, io);
        else
            hipLaunchKernelGGL((k_sub_scenario<kRegGroupsLarge, int32_t, kLargeWaves, KT, false, WARM>),
                               dim3((unsigned)io.n_paths * N.S), dim3(kWave * kLargeWaves), lds, st, N, io);
    } else if (WARM && io.nct_cap <= kRegGroupsWarm * kWave && !N.preds_lds) {
        // warm starts: the repair's code needs registers too; 13 groups (the 1k-arc networks'
        // ~800 chains) keep the all-in-registers kernel without the 16-group one's spills
        hipLaunchKernelGGL((k_sub_scenario<kRegGroupsWarm, KT, 1, KT, true, WARM>), dim3((unsigned)io.n_paths * N.S),
                           dim3(kWave), lds_wl, st, N, io);
    } else if (io.nct_cap <= kRegGroupsSmall * kWave && !N.preds_lds) {
        // register groups hold key increments: 64-bit with 64-bit keys, 32-bit with 32-bit keys
        hipLaunchKernelGGL((k_sub_scenario<kRegGroupsSmall, KT, 1, KT, true, WARM>), dim3((unsigned)io.n_paths * N.S),
                           dim3(kWave), lds_wl, st, N, io);
    } else {
        hipLaunchKernelGGL((k_sub_scenario<kRegGroupsSmall, KT, 1, KT, false, WARM>), dim3((unsigned)io.n_paths * N.S),
                           dim3(kWave), lds, st, N, io);
    }
    return hipGetLastError();
}
}  // namespace

hipError_t launch_subproblem(const SubNet &N, const SubIO &io_in, hipStream_t st) {
    if (io_in.n_paths <= 0) return hipSuccess;
    // SGUFP_SUB_SKIP=0: every scenario solved to the end (A/B of the first-infeasible stop)
    static const bool no_skip = [] {
        const char *e = getenv("SGUFP_SUB_SKIP");
        return e && atoi(e) == 0;
    }();
    SubIO io = io_in;
    if (no_skip) io.first_inf = nullptr;
    // 32-bit keys (N.key32, host: no lower bound in any scenario, sum_a |r_a| < 2^18, n + 2 <
    // 2^11); SGUFP_SUB_KEY64=1 forces the 64-bit keys (A/B)
    const char *ek = getenv("SGUFP_SUB_KEY64");
    // warm starts (io.warm_src / warm_dst) in both key widths: with lower bounds the repair keeps
    // every flow within [max l, min u]
    const bool k32 = N.key32 && !(ek && atoi(ek) == 1);
    const bool warm = io.warm_src || io.warm_dst;
    if (io.first_inf && hipMemsetAsync(io.first_inf, 0x7F, (size_t)io.n_paths * sizeof(int32_t), st) != hipSuccess)
        return hipGetLastError();
    hipLaunchKernelGGL(k_sub_paths, dim3((unsigned)io.n_paths), dim3(kWave), (size_t)N.m * 3 * sizeof(int16_t), st, N, io);
    const hipError_t e = !k32 ? (warm ? launch_scenarios<int64_t, true>(N, io, st) : launch_scenarios<int64_t, false>(N, io, st))
                              : (warm ? launch_scenarios<int32_t, true>(N, io, st) : launch_scenarios<int32_t, false>(N, io, st));
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_sub_reduce, dim3((unsigned)io.n_paths), dim3(256), 0, st, N, io);
    return hipGetLastError();
}

}  // namespace sgufp
