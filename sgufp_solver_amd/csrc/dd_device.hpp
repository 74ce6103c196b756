// Device-side data layout shared by the relaxation kernels (dd_kernels.hip) and the
// host context (capi.cpp).  See DESIGN.md "Data layout in HBM".
#pragma once

#include <cstdint>

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
    kErrRecord = 16,           // record not representable (states not a sorted subset, bad decision id)
    kErrCapacity = 17,         // DD larger than the per-slot capacity
    kErrCutset = 18,           // getCutset would run into the terminal layer (reference UB)
};

// node flags
constexpr uint8_t kAlive = 1;      // node is in tree[layer] (not deleted)
constexpr uint8_t kInAlive = 2;    // its (single, exact-layer) incoming arc is alive
constexpr uint8_t kKill = 4;       // scheduled for deletion in the current cascade

// topology word: parent index inside the previous layer (22 bits) | decision rank (6 bits)
constexpr uint32_t kParentMask = (1u << 22) - 1;
constexpr uint32_t kRankShift = 22;
constexpr uint32_t kNoRank = 63;

struct NetDev {
    int L;                 // totalLayers
    unsigned L5;           // (unsigned)(totalLayers - 5), the reference's unsigned arithmetic
    int m;
    int n_slots;           // cut row = n_slots coefficients + 1 zero slot
    const int32_t *layer_update;    // [L+1]
    const int32_t *layer_universe;  // [L+1]
    const uint8_t *changed;         // [L+1]
    const int32_t *set_off;         // [n_sets]
    const int32_t *set_len;         // [n_sets]
    const int16_t *set_val;         // concatenated sorted sets
    const int32_t *slot_tab;        // [L * kMaxU]
    const int32_t *slot_off;        // [L+1]
    const int32_t *slot_head;       // [n_slots]
    const int32_t *arc_head;        // [m]
};

// Per-slot DD scratch.  Every array is [max_batch * cap], slot-major.
struct Scratch {
    int Ncap, Acap, Tcap, Lcap;
    uint32_t *ntopo;   // [Ncap]
    uint8_t *nflag;    // [Ncap]
    uint32_t *nmask;   // [Ncap]
    uint32_t *outcnt;  // [Ncap]
    double *s2;        // [Ncap]  state2 of the last sweep
    double *tw;        // [Ncap]  terminal-arc weight (running min over optimality cuts), last layer only
    uint32_t *atopo;   // [Acap]  merged-layer incoming arcs
    uint8_t *aflag;    // [Acap]
    uint32_t *lay;     // [Tcap * 5] noff, n, alive, aoff, acnt
    int32_t *rslot;    // [Lcap] coefficient slot of each root-solution decision (-1: decision -1)
    int32_t *meta;     // [8] g, sol_len, T, exact, aligned, last_cut, status, cut_layer
    double *ubv;       // [1] running upper bound
    // multi-cut sweeps (k_relax with CB > 1)
    int tail_cap;      // nodes of the HBM-resident tail layers (wide layers + last layer)
    int cb_max;        // cuts per batched sweep the buffers are sized for
    int mir_cap;       // LDS mirror entries (16-bit) of the narrow-layer topology
    double *s2b;       // [tail_cap * cb_max]
    double *sm;        // [Tcap * cb_max]
    double *xm;        // [Tcap * cb_max]
};

// Staged batch of open nodes (Inavap::Node records, DD.h:456-478), SoA.
struct BatchIn {
    int n;
    const uint16_t *gl;
    const double *lb;
    const double *ub;
    const uint32_t *mask;      // states as a mask over the universe in force at gl
    const uint8_t *valid;      // host-side record validation
    const int64_t *sol_off;
    const uint16_t *sol_len;
    const int16_t *sol;
};

struct Pool {
    const double *rows;        // [cap][n_slots + 1]
    const double *rhs;         // [cap]
    int stride;                // n_slots + 1
    const int32_t *f_order;    // feasibility cuts, newest first
    int nf;
    const int32_t *o_order;    // optimality cuts, newest first
    int no;
    const double *coefT;       // [cap][L][ustride]: coefficient of state rank r at layer l
    int ustride;               // max state-set size of the network
};

struct BatchOut {
    int32_t *status;
    uint8_t *exact;
    double *lb;
    double *ub;
    uint32_t *nchild;
    uint32_t *sol_need;        // solution entries the children need (upper bound)
    uint32_t *dd_nodes;
    uint32_t *dd_arcs;
    uint32_t *dd_layers;
    uint32_t *sweeps;          // cuts swept over this node's DD
    int16_t *path;             // [max_batch * Lcap] argmax path of exact DDs
    uint16_t *path_len;
    uint64_t *ticks;           // wall_clock64 ticks (100 MHz) spent by each node's wave
    uint32_t *redo;            // batched sweeps restarted after an exact single-cut redo
};

// Children written by the emit kernel (device-resident frontier format).
struct ChildOut {
    const uint64_t *child_off;  // [n+1] exclusive scan of nchild
    const uint64_t *sol_base;   // [n+1] exclusive scan of sol_need
    uint16_t *gl;
    double *lb;
    double *ub;
    uint32_t *mask;
    int64_t *sol_off;
    uint16_t *sol_len;
    int16_t *sol;
};

}  // namespace sgufp
