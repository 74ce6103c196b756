// Device-side data of the scenario subproblem (GuroSolver::solveSubProblem,
// /root/reference/grb.cpp:139-360), shared by sub_kernels.hip and capi.cpp.
#pragma once

#include <cstdint>

#include "dd_device.hpp"

namespace sgufp {

// per (path, scenario) outcome
enum SubStatus : int32_t {
    kSubOptimal = 0,      // optimality-cut contribution written
    kSubInfeasible = 1,   // feasibility ray written (grb.cpp:288-350)
    kSubError = 2,        // invalid path (two in-arcs choosing one out-arc) or certificate failure
    kSubSkipped = 3,      // not solved: an earlier scenario of the path is infeasible, and the
                          // reference stops at the first infeasible one (grb.cpp:284-351)
};

struct SubNet {
    int n, m, S, L, n_slots, nz;
    int64_t cost_bound;                  // bound on |residual costs| incl. big-M: 2 M with
                                         // M <= 1 + 2 sum_a |r_a| (max u + 1) (host)
    int key32;                           // 32-bit Bellman-Ford keys and 12-byte chain records (host):
                                         // no lower bound and no negative upper bound in any
                                         // scenario, sum_a |r_a| < 2^18, n + 2 < 2^11
    int preds_lds;                       // SGUFP_SUB_PREDS_LDS=1: predecessors from the LDS chain
                                         // records, not the register groups (A/B)
    const int32_t SGUFP_GBL *tail;       // [m]
    const int32_t SGUFP_GBL *head;       // [m]
    const uint8_t SGUFP_GBL *vbar;       // [n]
    const uint8_t SGUFP_GBL *inner;      // [n] node has in- and out-arcs (conservation row, alpha)
    const int32_t SGUFP_GBL *arc_layer;  // [m] DD layer of an arc into a V-bar node, else -1
    const int32_t SGUFP_GBL *lb;         // [S][m]
    const int32_t SGUFP_GBL *ub;         // [S][m]
    const int32_t SGUFP_GBL *reward;     // [m] scenario-0 rewards (grb.cpp:53,71,89)
    const int32_t SGUFP_GBL *in_off;     // [n+1]
    const int32_t SGUFP_GBL *in_list;    // [m]
    const int32_t SGUFP_GBL *out_off;    // [n+1]
    const int32_t SGUFP_GBL *out_list;   // [m]
    const int32_t SGUFP_GBL *slot_off;   // [L+1]
    const int32_t SGUFP_GBL *slot_head;  // [n_slots]
    const int32_t SGUFP_GBL *zlist;      // [nz] free-supply / free-demand nodes: v | src << 30 | snk << 29
    const int32_t SGUFP_GBL *arc_topo;   // [m] arcs by topological rank of their tail (chain order)
    const int16_t SGUFP_GBL *orank;      // [m] rank of head(b) among the distinct heads of tail(b)'s
                                         // out-arcs: b's coefficient slot in a layer (i, tail(b))
                                         // is slot_off[layer] + orank[b] (network.cpp slots)
};

struct SubIO {
    int n_paths;
    int nct_cap;                         // chains per (path, scenario) the LDS holds: m minus the
                                         // fewest decided arcs over the batch (host, per call)
    const int64_t SGUFP_GBL *path_off;   // [n_paths+1]
    const int16_t SGUFP_GBL *paths;
    // paths read in place from the relaxation outputs (B&B refinement loop): path p is
    // paths[path_slot[p] * path_stride ...] of length path_len[path_slot[p]]; path_off unused
    const int32_t SGUFP_GBL *path_slot;  // null: path_off / paths as above
    const uint16_t SGUFP_GBL *path_len;
    int64_t path_stride;
    // per (path, scenario)
    int32_t SGUFP_GBL *status;           // [P*S]
    double SGUFP_GBL *obj;               // [P*S] scenario objective (optimal scenarios)
    double SGUFP_GBL *dual;              // [P*S] objective of the dual solution built (check)
    double SGUFP_GBL *rhs;               // [P*S] RHS contribution (before the 1/S of the reference)
    double SGUFP_GBL *coef;              // [P*S][n_slots] coefficient contributions
    // per path
    int32_t SGUFP_GBL *cut_type;         // [P] 0 optimality, 1 feasibility, -1 error
    double SGUFP_GBL *cut_rhs;           // [P]
    double SGUFP_GBL *cut_row;           // [P][n_slots+1] dense cut row (last slot 0)
    double SGUFP_GBL *obj_mean;          // [P] sum_s obj_s / S (optimality)
    // Warm starts (32- and 64-bit-key launches).  The state of (slot, scenario) is an optimal
    // flow per network arc and the optimal node potentials (alpha of grb.cpp's dual, 0 at free
    // and V-bar nodes) of an earlier solve of a feasible scenario; wst_ok marks the (slot,
    // scenario) pairs whose last solve stored one (an infeasible or failed scenario stores none,
    // and that scenario of a later path starts cold).  Path p starts scenario s from slot
    // warm_src[p]'s state (-1: cold) and writes its own final state to slot warm_dst[p] (-1:
    // none).  A solve reads only its source slot and writes only its destination: two paths of
    // one launch may share neither a destination nor a destination with another path's source
    // (the host guarantees it).
    const int32_t SGUFP_GBL *warm_src;   // [P] or null
    const int32_t SGUFP_GBL *warm_dst;   // [P] or null
    int16_t SGUFP_GBL *wst_x;            // [slots][S][m]
    int32_t SGUFP_GBL *wst_a;            // [slots][S][n]
    uint8_t SGUFP_GBL *wst_ok;           // [slots][S]
    int32_t SGUFP_GBL *first_inf;        // [P] or null: smallest scenario of the path found infeasible so
                                         // far (launch_subproblem sets INT_MAX-like); later scenarios stop
    int32_t SGUFP_GBL *wstat;            // [P*S][2] or null: augmentations (negative: a warm start fell
                                         // back to the cold SSP), Bellman-Ford passes
    // The chains of each path (k_sub_paths, once per path for all its scenarios: the chains
    // depend on the decisions only).  Stride m per path; chains in phase 2's numbering (the
    // topological order of their first arc's tail).
    int32_t SGUFP_GBL *pc_info;          // [P][2] chains, error (invalid path / more chains than nct_cap)
    uint32_t SGUFP_GBL *pc_th;           // [P][m] tail (-1: V-bar or none) | head << 16 (-1: open end), int16 each
    uint32_t SGUFP_GBL *pc_ol;           // [P][m] offset of the chain's arcs in pc_arcs | length << 16
    int32_t SGUFP_GBL *pc_R;             // [P][m] reward sum
    uint32_t SGUFP_GBL *pc_arcs;         // [P][m] the chains' arcs, chain after chain: arc | slot << 16
                                         // (int16; slot of the pair with the next arc, -1 at the end)
    int32_t SGUFP_GBL *pc_rw;            // [P][m] their rewards, in the same order
};

// Ring of warm-start states (the B&B's refinement loops, bnb.cpp): R slots, each holding the
// path it was solved for here and its flows / potentials for every scenario in SubIO::wst_x /
// wst_a.  k_warm_pick gives each path of a launch the slot whose path differs in the fewest
// decisions (slots written by the same launch excluded) and the slot its own state goes to.
struct WarmRing {
    int R;                                // slots
    int Lcap;                             // decisions per stored path
    int max_dist;                         // farther than this: cold start
    int16_t SGUFP_GBL *path;              // [R][Lcap]
    uint16_t SGUFP_GBL *plen;             // [R]
    uint8_t SGUFP_GBL *valid;             // [R]
    int32_t SGUFP_GBL *src;               // [paths per launch] chosen source slot (-1: cold)
    int32_t SGUFP_GBL *dst;               // [paths per launch] destination slot
    int32_t SGUFP_GBL *dist;              // [paths per launch] decisions that differ (-1: none)
};

}  // namespace sgufp
