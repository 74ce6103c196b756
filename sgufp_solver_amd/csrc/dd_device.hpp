// Device-side data layout shared by the relaxation kernels (dd_kernels.hip) and the
// host context (capi.cpp).  See DESIGN.md "Data layout in HBM".
#pragma once

#include <cstdint>

// Device code sees every HBM pointer of the structs below in the global address space, so
// the compiler emits global_load/global_store (vmcnt only) instead of flat_* accesses, which
// would make every LDS access wait for all outstanding HBM loads.  The host sees plain
// pointers; both are 64-bit with the same value, so the kernel-argument layout is identical.
// Host-only translation units (capi.cpp) define SGUFP_HOST_ONLY for their device pass.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(SGUFP_HOST_ONLY)
#define SGUFP_GBL __attribute__((address_space(1)))
#else
#define SGUFP_GBL
#endif

namespace sgufp {

constexpr int kWave = 64;          // one DD per 64-lane wavefront (one single-wave workgroup)
constexpr int kMaxU = 32;          // state universe <= 32 -> u32 masks
constexpr int kLdsWidth = 512;     // layers up to this width keep their state2 in LDS during a sweep

// per-node result status (Inavap::OutObject::STATUS_OP, NodeExplorer.h:81-85, plus extensions)
enum NodeStatus : int32_t {
    kSuccess = 0,
    kPrunedFeasibility = 1,
    kPrunedOptimality = 2,
    kNeedsSubproblem = 3,      // exact DD: the argmax path waits for the scenario subproblem
    kPrunedBound = 4,          // ub <= incumbent before processing (DDSolver.cpp:707-711), B&B rounds only
    kErrRecord = 16,           // record not representable (states not a sorted subset, bad decision id)
    kErrCapacity = 17,         // DD larger than the per-slot capacity
    kErrCutset = 18,           // getCutset would run into the terminal layer (reference UB)
};

// node flags
constexpr uint8_t kAlive = 1;      // node is in tree[layer] (not deleted)
constexpr uint8_t kInAlive = 2;    // its (single, exact-layer) incoming arc is alive
constexpr uint8_t kKill = 4;       // scheduled for deletion in the current cascade
constexpr uint8_t kLazy = 8;       // exact DD leaf: tw is an upper bound (ExactIO::lazy), see exact_resolve

// packed topology word of a narrow layer (Scratch::tmir, build_stream in dd_kernels.hip):
// parent:7 | rank:5 | alive | in-arc alive
constexpr uint16_t kMirParent = 127, kMirRankShift = 7, kMirAlive = 1u << 12, kMirIn = 1u << 13;

// topology word: parent index inside the previous layer (22 bits) | decision rank (6 bits)
constexpr uint32_t kParentMask = (1u << 22) - 1;
constexpr uint32_t kRankShift = 22;
constexpr uint32_t kNoRank = 63;

struct NetDev {
    int L;                 // totalLayers
    unsigned L5;           // (unsigned)(totalLayers - 5), the reference's unsigned arithmetic
    int m;
    int n_slots;           // cut row = n_slots coefficients + 1 zero slot
    const int32_t SGUFP_GBL *layer_update;    // [L+1]
    const int32_t SGUFP_GBL *layer_universe;  // [L+1]
    const uint8_t SGUFP_GBL *changed;         // [L+1]
    const int32_t SGUFP_GBL *set_off;         // [n_sets]
    const int32_t SGUFP_GBL *set_len;         // [n_sets]
    const int16_t SGUFP_GBL *set_val;         // concatenated sorted sets
    const int32_t SGUFP_GBL *slot_tab;        // [L * kMaxU]
    const int32_t SGUFP_GBL *slot_off;        // [L+1]
    const int32_t SGUFP_GBL *slot_head;       // [n_slots]
    const int32_t SGUFP_GBL *arc_head;        // [m]
};

// Per-slot DD scratch.  Every array is [max_batch * cap], slot-major.
struct Scratch {
    int Ncap, Acap, Tcap, Lcap;
    uint32_t SGUFP_GBL *ntopo;   // [Ncap]
    uint8_t SGUFP_GBL *nflag;    // [Ncap]
    uint32_t SGUFP_GBL *nmask;   // [Ncap]
    uint32_t SGUFP_GBL *outcnt;  // [Ncap]
    double SGUFP_GBL *s2;        // [Ncap]  state2 of the last sweep
    double SGUFP_GBL *tw;        // [Ncap]  terminal-arc weight (running min over optimality cuts), last layer only
    uint32_t SGUFP_GBL *atopo;   // [Acap]  merged-layer incoming arcs
    uint8_t SGUFP_GBL *aflag;    // [Acap]
    uint32_t SGUFP_GBL *lay;     // [Tcap * 5] noff, n, alive, aoff, acnt
    int32_t SGUFP_GBL *rslot;    // [Lcap] coefficient slot of each root-solution decision (-1: decision -1)
    int32_t SGUFP_GBL *meta;     // [8] g, sol_len, T, exact, aligned, last_cut, status, cut_layer
    double SGUFP_GBL *ubv;       // [1] running upper bound
    // single-cut sweep summaries (dd_sweep / dd_prune), [Tcap] per slot: HBM, so that the
    // batched kernels' LDS fits eight waves per CU
    double SGUFP_GBL *sm1;
    double SGUFP_GBL *xm1;
    uint8_t SGUFP_GBL *v1;
    int us;                      // coefficient table entries per layer (the network's max state count)
    // multi-cut sweeps (k_relax with CB > 1)
    int tail_cap;      // nodes of the HBM-resident tail layers (wide layers + last layer)
    int cb_max;        // cuts per batched sweep the buffers are sized for
    double SGUFP_GBL *s2b;       // [tail_cap * cb_max]
    double SGUFP_GBL *sm;        // [Tcap * cb_max]
    double SGUFP_GBL *xm;        // [Tcap * cb_max]
    int tmir_cap;                // packed narrow-layer topology words per slot (Ncap + Acap)
    uint16_t SGUFP_GBL *tmir;    // [tmir_cap]
};

// Staged batch of open nodes (Inavap::Node records, DD.h:456-478), SoA.
struct BatchIn {
    int n;
    const uint16_t SGUFP_GBL *gl;
    const double SGUFP_GBL *lb;
    const double SGUFP_GBL *ub;
    const uint32_t SGUFP_GBL *mask;      // states as a mask over the universe in force at gl
    const uint8_t SGUFP_GBL *valid;      // host-side record validation
    const int64_t SGUFP_GBL *sol_off;
    const uint16_t SGUFP_GBL *sol_len;
    const int16_t SGUFP_GBL *sol;
    int bound_prune;                     // 1: records with ub <= incumbent are pruned unprocessed
    const int32_t SGUFP_GBL *perm;       // k_relax dispatch order: workgroup b relaxes record
                                         // perm[b] (null: b), see sgufp_ctx::relax_current
};

// Device frontier (B&B open nodes), SoA stack; sol_off are absolute offsets into sol.
struct FrontierDev {
    uint16_t SGUFP_GBL *gl;
    double SGUFP_GBL *lb;
    double SGUFP_GBL *ub;
    uint32_t SGUFP_GBL *mask;
    uint8_t SGUFP_GBL *valid;
    int64_t SGUFP_GBL *sol_off;
    uint16_t SGUFP_GBL *sol_len;
    int16_t SGUFP_GBL *sol;
};

struct Pool {
    const double SGUFP_GBL *rows;        // [cap][n_slots + 1]
    const double SGUFP_GBL *rhs;         // [cap]
    int stride;                // n_slots + 1
    const int32_t SGUFP_GBL *f_order;    // feasibility cuts, newest first
    int nf;
    const int32_t SGUFP_GBL *o_order;    // optimality cuts, newest first
    int no;
    const double SGUFP_GBL *coefT;       // [cap][L][ustride]: coefficient of state rank r at layer l
    int ustride;               // max state-set size of the network
    // optimality-cut screening (see screen_opt in dd_kernels.hip): the first nscreen rows
    // of o_rank (strongest first by a node-independent bound) are tried before the exact
    // optimality phase; 0 disables it
    const int32_t SGUFP_GBL *o_rank;
    int nscreen;
};

struct BatchOut {
    int32_t SGUFP_GBL *status;
    uint8_t SGUFP_GBL *exact;
    double SGUFP_GBL *lb;
    double SGUFP_GBL *ub;
    uint32_t SGUFP_GBL *nchild;
    uint32_t SGUFP_GBL *sol_need;        // solution entries the children need (upper bound)
    uint32_t SGUFP_GBL *dd_nodes;
    uint32_t SGUFP_GBL *dd_arcs;
    uint32_t SGUFP_GBL *dd_layers;
    uint32_t SGUFP_GBL *sweeps;          // cuts swept over this node's DD
    int16_t SGUFP_GBL *path;             // [max_batch * Lcap] argmax path of exact DDs
    uint16_t SGUFP_GBL *path_len;
    uint64_t SGUFP_GBL *ticks;           // wall_clock64 ticks (100 MHz) spent by each node's wave
    uint64_t SGUFP_GBL *phase;           // [max_batch * 8] ticks per phase: build, narrow, tail, last, post, redo, finish
    uint32_t SGUFP_GBL *redo;            // batched sweeps restarted after an exact single-cut redo
};

// Children written by the emit kernel (device-resident frontier format).
struct ChildOut {
    const uint64_t SGUFP_GBL *child_off;  // [n+1] exclusive scan of nchild
    const uint64_t SGUFP_GBL *sol_base;   // [n+1] exclusive scan of sol_need
    uint16_t SGUFP_GBL *gl;
    double SGUFP_GBL *lb;
    double SGUFP_GBL *ub;
    uint32_t SGUFP_GBL *mask;
    int64_t SGUFP_GBL *sol_off;
    uint16_t SGUFP_GBL *sol_len;
    int16_t SGUFP_GBL *sol;
};

// Optimality phase of exact DDs (exact_kernels.hip).  An exact DD is a tree: every leaf is
// one path, applyOptimalityCut makes no edit on it (DD.cpp:3986-4022 run only for non-exact
// DDs), and its terminal weight ends as min over the O cuts of the path's value (a running
// std::min, DD.cpp:3975-3984).  The outcome is therefore the same for any processing order
// of the cuts: PRUNED_BY_OPTIMALITY_CUT iff max over leaves of that minimum <= optimalLB (the
// running maximum only decreases), else ub = that maximum and the argmax path.  k_relax
// hands such records over after the feasibility phase and screening (status
// kExactPending); the leaf kernel computes the minima with lanes = cuts (all lanes walk the
// same tree), a workgroup per pass of kLeafPass leaves of one record, every cut column read
// once per pass from a cut-minor copy of the O rows.
constexpr int32_t kExactPending = 5;
#ifndef SGUFP_EXACT_MAXT
#define SGUFP_EXACT_MAXT 8
#endif
#ifndef SGUFP_EXACT_ENTRIES
#define SGUFP_EXACT_ENTRIES 40
#endif
#ifndef SGUFP_LEAVES_PER_WAVE
#define SGUFP_LEAVES_PER_WAVE 16
#endif
// Leaf-kernel sizing (seeded C3 B&B, tools/gpu_r04o.sh, gpu_r04r.sh): 16 layers / 64 staged rows /
// 32 leaves per wave at 2 waves per SIMD (101 KB of LDS per workgroup) 1 915 relaxations/s; 8 / 64 /
// 16, two workgroups per CU at 4 waves per SIMD (105 VGPRs) 2 232; 8 / 40 / 16, three workgroups
// per CU at 6 waves per SIMD (80 VGPRs, 50 KB): k_relax 4.08 -> 3.30 s over the same 88 rounds.
// The exact DDs of the C3 / C4 searches all have 7 layers and 5 state ranks (30 rows); deeper or
// wider ones take k_relax's own path.
constexpr int kExactMaxT = SGUFP_EXACT_MAXT;           // DD layers (root included) the hand-off takes
constexpr int kExactMaxEntries = SGUFP_EXACT_ENTRIES;  // (T - 1) * ustride coefficient rows staged per cut block
constexpr int kExactMaxEntriesWide = 64;               // ... by the wide leaf-kernel instantiation
constexpr int kLeafWaves = 8;                          // waves per leaf-kernel workgroup
constexpr int kLeavesPerWave = SGUFP_LEAVES_PER_WAVE;
constexpr int kLeafPass = kLeafWaves * kLeavesPerWave;

struct ExactIO {
    int enabled;
    int no;                               // optimality cuts in the pool at launch
    int ostride;                          // column capacity of coefO / R
    const double SGUFP_GBL *coefO;        // [n_slots + 2][ostride]: column j = O cut o_rows[j] (oldest
                                          // first); row n_slots = 0 (absent key), row n_slots + 1 = RHS
    double SGUFP_GBL *R;                  // [max_batch][ostride]: root folds, pending index x newest-first position
    int32_t SGUFP_GBL *pend_slot;         // [max_batch] batch slot of pending record i
    uint32_t SGUFP_GBL *pend_base;        // [max_batch] first leaf pass of pending record i
    unsigned long long SGUFP_GBL *ctr;    // [32]: (pending << 32 | leaf passes), root work, leaf work,
                                          // blocks swept, lazy resolves, blocks they swept, non-exact:
                                          // DAG work, fallbacks, leaf work, kept back; wide leaf work,
                                          // maxState completion work, non-exact entries;
                                          // diagnostics: exact leaves open after 64 / 16 blocks, alive;
                                          // 16 / 17: phase-B leaf work (narrow / wide), 18: leaves
                                          // open after phase A, 19: phase-B blocks swept
    // Lazy terminal weights: a leaf pass sweeps at most `lazy` cut blocks (the newest 64 x lazy
    // O cuts); when that leaves some leaf above optimalLB the pass's leaves keep the partial
    // minimum (an upper bound of the terminal weight) flagged kLazy, and the argmax scans
    // (k_exact_fin, k_refine) complete a flagged leaf over the remaining blocks only when it
    // is the maximum (exact_resolve).  0: every pass sweeps the whole pool.
    int lazy;
    int32_t SGUFP_GBL *pidx;              // [nslots] batch slot -> pending index (-1: none)
    int nslots;                           // batch slots (max_batch)
    // screening columns swept first (any order gives the same terminal minima; these -- the
    // strongest O cuts by their node-independent bound, Pool::o_rank -- end pruned records
    // early): nsc of them, kExactScreen columns allocated
    int nsc;
    const double SGUFP_GBL *coefS;        // [n_slots + 2][kExactScreen]
    double SGUFP_GBL *RS;                 // [max_batch][kExactScreen]
    // Cut-parallel optimality phase of NON-exact DDs (nx_kernels.hip, see kNxPending): pending
    // entries of both kinds share the index space, root folds and leaf passes above.
    int nx;                               // 1: k_relax hands such records off
    int nx_min;                           // ... when the pool holds at least this many O cuts,
    int nx_skip;                          // ... after this many of them in order

    int redo;                             // k_relax re-run: only the kNxFallback slots, no hand-off
    int nx_ms;                            // the leaf kernel's second non-exact launch (maxState completion)
    int32_t SGUFP_GBL *pstop;             // [leaf passes] the last cut block a non-exact pass swept
    int32_t SGUFP_GBL *nxlist;            // [max_batch] pending indices of the non-exact entries (ctr[12] of them)
    int32_t SGUFP_GBL *pkind;             // [max_batch] per pending entry: -1 exact, else the DAG's last width-1 layer k0
    int32_t SGUFP_GBL *P;                 // [max_batch] first pruning position (max over leaves of the first cut <= optimalLB)
    double SGUFP_GBL *G;                  // [max_batch][ostride] width-1 pruning gap per cut (k_nx_dag), lowered by its error bound
    unsigned long long SGUFP_GBL *MS;     // [max_batch][ostride] maxState per cut (order-preserving key, atomic max)
    int32_t SGUFP_GBL *nxh;               // [nslots][4] per handed-off slot: k0, packed node words, k0's node,
                                          // first pool position of the phase
    // Open-leaf compaction of the exact DDs' leaf passes (k_exact_leaf, phase A / B): phase A
    // sweeps the first leaf_split cut blocks of every pass; a leaf still above optimalLB after
    // them joins its record's open list (leaf indices from pend_base[i] x kLeafPass) with its
    // partial minimum in tw, and phase B sweeps the remaining blocks over passes of kLeafPass OPEN
    // leaves, so a pass whose leaves are all settled stops holding the other leaves' sweep.
    // leaf_split 0: one phase (every pass sweeps until its leaves are settled).
    int leaf_split;
    int leaf_phase;                       // 0: single phase / phase A, 1: phase B
    int32_t SGUFP_GBL *open_cnt;          // [nslots] open leaves per pending record after phase A
    int32_t SGUFP_GBL *open_list;         // [leaf passes x kLeafPass] their leaf indices
};
constexpr int kExactScreen = 256;

// Non-exact DDs (nx_kernels.hip).  Past the feasibility phase an optimality cut edits a
// non-exact DD only when a width-1 layer's arc pruning fires (DD.cpp:3986-4022); a pool that
// fires nowhere leaves the optimality phase order-free like an exact DD's: per-leaf running
// minima, the terminal state non-increasing, so the record is pruned at the first cut where
// every leaf's minimum is <= optimalLB, else ub = the last terminal state.  Below the last
// width-1 layer k0 the DD is a tree (merged layers have one node), so the leaf passes of
// k_exact_leaf apply with the value at k0 as their root; above it k_nx_dag sweeps each cut's
// values through the DAG (lanes = node groups x cuts) into that root value and a conservative
// per-cut gap of the width-1 pruning test.  k_nx_fin checks that no cut before the pruning position can
// fire; a record where one might (status kNxFallback) is re-run by k_relax in order.
constexpr int32_t kNxPending = 6;
constexpr int32_t kNxFallback = 7;
// ExactIO::pkind of a non-exact entry k_nx_fin sent back to k_relax (read by sgufp_batch_routes)
constexpr int32_t kNxRouteFallback = INT32_MIN;
constexpr int kNxRanks = 4;     // nonzero state ranks (ustride <= 5)
constexpr int kNxCuts = 16;     // cuts per k_nx_dag work item (lanes = 4 node groups x 16 cuts)

// Seen-path lists of the exact DDs' refinement loops (bnb_kernels.hip), per batch slot.
struct SeenLists {
    int16_t SGUFP_GBL *paths;   // [slots][cap][Lcap]
    uint16_t SGUFP_GBL *len;    // [slots][cap]
    uint64_t SGUFP_GBL *hash;   // [slots][cap]
    int32_t SGUFP_GBL *n;       // [slots]
    int cap;
    int Lcap;
};

}  // namespace sgufp
