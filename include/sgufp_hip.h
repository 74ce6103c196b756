/*
 * sgufp_hip.h -- C ABI of the MI355X relaxation engine (libsgufp_hip.so).
 *
 * Plain pointers and sizes only.  Every entry point replaces one piece of the
 * reference's per-B&B-node relaxation path (var-nan/SGUFP_Solver @ 2025-07-18):
 *
 *   sgufp_create_from_file / sgufp_create
 *       Network::Network(const std::string&)           Network.cpp:10-129, Network.h:113
 *       (+ shuffleVBarNodes, Network.cpp:132-186)
 *   sgufp_cuts_append
 *       Inavap::Container::add(cut_node_t*)              Cut.h:461-465
 *       (cut = Inavap::Cut{RHS, (key, coef)}            Cut.h:201-337; key = getKey(q,i,j) Cut.h:342-344)
 *   sgufp_batch_upload + sgufp_batch_relax + sgufp_batch_results/_children/_paths
 *       Inavap::NodeExplorer::process(Node, double optimalLB, Container&, Container&)
 *                                                        NodeExplorer.cpp:915-986, NodeExplorer.h:130
 *       i.e. RelaxedDDNew::buildTree / applyFeasibilityCut / applyOptimalityCut /
 *       getCutset / getSolution                          DD.cpp:3528-4218, DD.h:797-808
 *       for a whole batch of open nodes, up to the first scenario-subproblem call.
 *   sgufp_batch_refine
 *       the exact-DD refinement step of process: apply the cut the subproblem just
 *       produced and return the next argmax path        NodeExplorer.cpp:946-969
 *   sgufp_subproblem
 *       GuroSolver::solveSubProblem(const vector<int16_t>&) grb.h:75, grb.cpp:139-360
 *   sgufp_frontier_* + sgufp_bnb_step
 *       the open-node queues and the worker loop of Inavap::DDSolver
 *       (lf_queue lock_free_queue.h:24-165, Worker::startWorker DDSolver.cpp:658-776,
 *       Master::processNodes :556-579), as a device-resident stack and batched rounds
 *
 * Conventions: functions return SGUFP_OK (0) or a negative SGUFP_ERR_* code; the
 * caller owns every host buffer; a context is driven by one host thread at a time and
 * owns one HIP stream.  Per-node outcomes use the reference's STATUS_OP values
 * (NodeExplorer.h:81-85) plus SGUFP_NEEDS_SUBPROBLEM and error codes >= 16.
 * Doubles are IEEE binary64 and bit-identical to the reference's results.
 */
#ifndef SGUFP_HIP_H
#define SGUFP_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct sgufp_ctx sgufp_ctx;

/* return codes */
#define SGUFP_OK 0
#define SGUFP_ERR_ARG (-1)
#define SGUFP_ERR_NETWORK (-2)
#define SGUFP_ERR_HIP (-3)
#define SGUFP_ERR_CAPACITY (-4)
#define SGUFP_ERR_STATE (-5)
#define SGUFP_ERR_KEY (-6)

/* per-node status (OutObject::STATUS_OP, NodeExplorer.h:81-85, + extensions) */
#define SGUFP_SUCCESS 0
#define SGUFP_PRUNED_BY_FEASIBILITY_CUT 1
#define SGUFP_PRUNED_BY_OPTIMALITY_CUT 2
#define SGUFP_NEEDS_SUBPROBLEM 3
#define SGUFP_PRUNED_BY_BOUND 4   /* B&B rounds only: ub <= zOpt before processing (DDSolver.cpp:707-711) */
#define SGUFP_NODE_ERR_RECORD 16
#define SGUFP_NODE_ERR_CAPACITY 17
#define SGUFP_NODE_ERR_CUTSET 18

typedef struct {
    int32_t n, m, scenarios;     /* nodes, arcs, scenarios */
    int32_t total_layers;        /* Network::totalLayers */
    int32_t n_vbar;
    int32_t max_states;          /* largest |out-arcs(q)| + 1 over V-bar nodes */
    int32_t n_slots;             /* dense coefficients per cut row */
    int32_t max_batch;
    int64_t node_capacity;       /* DD nodes per slot */
    int64_t arc_capacity;        /* merged-layer arcs per slot */
    int64_t scratch_bytes;       /* device bytes held by the context */
} sgufp_network_info;

/* -- context ---------------------------------------------------------------- */
sgufp_ctx *sgufp_create_from_file(const char *path, int device, int max_batch, int *err);
sgufp_ctx *sgufp_create(int n, int m, int scenarios, const int32_t *tails, const int32_t *heads,
                        const int32_t *lb, const int32_t *ub, const int32_t *reward, /* [m*scenarios] */
                        int n_vbar, const int32_t *vbar, int device, int max_batch, int *err);
void sgufp_destroy(sgufp_ctx *ctx);
int sgufp_get_network_info(const sgufp_ctx *ctx, sgufp_network_info *out);
/* processingOrder arc ids [total_layers] and V-bar order [n_vbar] */
int sgufp_processing_order(const sgufp_ctx *ctx, int32_t *layer_arcs, int32_t *vbar_order);
const char *sgufp_last_error(const sgufp_ctx *ctx);
void *sgufp_stream(const sgufp_ctx *ctx); /* hipStream_t the kernels run on */

/* Host-only parse of an instance file (no device is touched): totalLayers, then up to
 * cap processingOrder arc ids and V-bar ids.  Returns SGUFP_OK or SGUFP_ERR_NETWORK. */
int sgufp_probe_network(const char *path, int32_t *total_layers, int32_t *n_vbar, int32_t cap, int32_t *layer_arcs,
                        int32_t *vbar_order);

/* -- cut pool (global F and O Containers) ---------------------------------- */
/* n_cuts cuts in insertion order; cut c has keys/vals [nnz_off[c], nnz_off[c+1]).
 * keys are Inavap::getKey(q,i,j); lookup is first-match on the low 48 bits, zero
 * coefficients may be present.  Keys that are not (i,q,j) of a V-bar arc pair are
 * rejected with SGUFP_ERR_KEY.  Application order is newest first (LIFO list). */
int sgufp_cuts_append(sgufp_ctx *ctx, int is_feasibility, int n_cuts, const double *rhs, const int64_t *nnz_off,
                      const uint64_t *keys, const double *vals);
int sgufp_cuts_clear(sgufp_ctx *ctx);
int sgufp_cuts_count(const sgufp_ctx *ctx, int is_feasibility);

/* -- batched relaxation ----------------------------------------------------- */
/* Stage n open nodes (Inavap::Node, DD.h:456-478).  states of node k are
 * states[states_off[k] .. states_off[k+1]), solution likewise. */
int sgufp_batch_upload(sgufp_ctx *ctx, int n, const uint16_t *global_layer, const double *lb, const double *ub,
                       const int64_t *states_off, const int16_t *states, const int64_t *sol_off,
                       const int16_t *sol);
/* Relax the staged batch against the current pools (asynchronous on the ctx stream). */
int sgufp_batch_relax(sgufp_ctx *ctx, double optimal_lb);
int sgufp_batch_sync(sgufp_ctx *ctx);
/* Per node: status, exact flag, lb, ub, number of cutset children (any pointer may be NULL). */
int sgufp_batch_results(sgufp_ctx *ctx, int32_t *status, uint8_t *exact, double *lb, double *ub,
                        int32_t *n_children);
/* Totals needed to size the children buffers. */
int sgufp_batch_children_size(sgufp_ctx *ctx, int64_t *n_children, int64_t *n_states, int64_t *n_sol);
/* Children of every node, concatenated in node order (child_off has n+1 entries). */
int sgufp_batch_children(sgufp_ctx *ctx, int64_t *child_off, uint16_t *global_layer, double *lb, double *ub,
                         int64_t *states_off, int16_t *states, int64_t *sol_off, int16_t *sol);
/* Argmax paths of nodes with SGUFP_NEEDS_SUBPROBLEM (path_off has n+1 entries; others empty). */
int sgufp_batch_paths(sgufp_ctx *ctx, int64_t *path_off, int16_t *paths);
/* DD statistics: nodes / arcs right after the build, layers, cuts swept. */
int sgufp_batch_stats(sgufp_ctx *ctx, int64_t *dd_nodes, int64_t *dd_arcs, int32_t *dd_layers, int32_t *sweeps);
/* Apply, for each listed staged node (still SGUFP_NEEDS_SUBPROBLEM), the pool cut
 * (is_feasibility[k], index in that pool) -- appended beforehand with
 * sgufp_cuts_append -- and recompute status / ub / path.  optimal_lb must not be below the
 * optimalLB the batch was relaxed with (NodeExplorer::process keeps it fixed within a call,
 * NodeExplorer.cpp:946-969): the cut-parallel phase of exact DDs stops a leaf's minimum once it
 * is <= that optimalLB, so a lower value returns SGUFP_ERR_ARG. */
int sgufp_batch_refine(sgufp_ctx *ctx, int n, const int32_t *node_idx, const uint8_t *is_feasibility,
                       const int32_t *cut_index, double optimal_lb);

/* -- one DD at a time: Inavap::RelaxedDDNew (DD.h:797-808) ------------------------------
 * The C++ API's Inavap::RelaxedDDNew is a batch of one through these calls; any staged node
 * can be driven this way.  The DD stays resident in the node's slot between calls.
 *   sgufp_dd_build     buildTree(Node) for every staged node, no cut applied (DD.cpp:3528-3600);
 *                      sgufp_batch_results then gives the exact flag (isTreeExact) and status
 *                      SUCCESS (non-exact) / NEEDS_SUBPROBLEM (exact)
 *   sgufp_dd_apply     applyFeasibilityCut(cut) -> *value 1 / 0 (DD.cpp:3842-3930), or
 *                      applyOptimalityCut(cut, optimal, ub) -> *value (DD.cpp:3932-4023; the
 *                      reference ignores ub); the cut as sgufp_cuts_append takes it (keys
 *                      getKey(q,i,j), first match).  After a call that prunes the node (0, or a
 *                      value <= optimal) the DD is only good for a new sgufp_dd_build.
 *   sgufp_dd_solution  getSolution() (DD.cpp:3825-3840): the argmax path under the last cut
 *                      applied; path holds total_layers entries, *len gets its length
 *   sgufp_dd_cutset    getCutset(ub) (DD.cpp:4179-4218) of a non-exact DD; the children are
 *                      then read with sgufp_batch_children_size / sgufp_batch_children (other
 *                      staged nodes contribute none).  SGUFP_ERR_STATE for an exact tree. */
int sgufp_dd_build(sgufp_ctx *ctx);
int sgufp_dd_apply(sgufp_ctx *ctx, int node, int is_feasibility, double rhs, int64_t nnz, const uint64_t *keys,
                   const double *vals, double optimal, double *value);
int sgufp_dd_solution(sgufp_ctx *ctx, int node, int16_t *path, int32_t *len);
int sgufp_dd_cutset(sgufp_ctx *ctx, int node, double ub, int64_t *n_children);

/* Diagnostics of the last relax: wall_clock64 ticks (100 MHz) of each node's wave and
 * the number of batched-sweep restarts (exact single-cut redo after pruning).  Ticks and
 * phases are stamped only by the profiling build (sgufp_solver_amd/lib_prof, -DSGUFP_PHASES);
 * the production library returns zeros for them. */
int sgufp_batch_debug(sgufp_ctx *ctx, int64_t *ticks, int32_t *redo);
/* ticks per phase [n * 8]: build, narrow sweep, tail layers, last layer, replay/post, redo, finish, tail */
int sgufp_batch_phases(sgufp_ctx *ctx, int64_t *phase);

/* Which kernels took each node's optimality phase in the last sgufp_batch_relax (parity
 * tests of the cut-parallel phases at the pool sizes the B&B reaches; any staged node):
 *   SGUFP_ROUTE_IN_ORDER     k_relax's in-order sweeps only (DD.cpp:3932-4023 cut by cut)
 *   SGUFP_ROUTE_EXACT_PHASE  exact DD handed to k_exact_root / k_exact_leaf / k_exact_fin
 *   SGUFP_ROUTE_NX_PHASE     non-exact DD settled by k_nx_dag / k_exact_leaf<nx> / k_nx_fin
 *   SGUFP_ROUTE_NX_FALLBACK  non-exact DD handed off, then re-run in order by k_relax because a
 *                            width-1 pruning might have fired (DD.cpp:3986-4022)
 * All SGUFP_ROUTE_IN_ORDER after sgufp_dd_build.  SGUFP_ERR_STATE before any relaxation. */
#define SGUFP_ROUTE_IN_ORDER 0
#define SGUFP_ROUTE_EXACT_PHASE 1
#define SGUFP_ROUTE_NX_PHASE 2
#define SGUFP_ROUTE_NX_FALLBACK 3
int sgufp_batch_routes(sgufp_ctx *ctx, int32_t *route);

/* -- scenario subproblem (replaces GuroSolver::solveSubProblem, grb.h:75 / grb.cpp:139-360) --
 * For n paths (concatenated int16 decisions, one per DD layer, path_off has n+1 entries)
 * solve every scenario's flow LP on the device and build the cut the reference would add:
 * type[k] = 0 optimality cut (sum over scenarios / S, grb.cpp:236-281), 1 feasibility cut
 * (ray of the first infeasible scenario, grb.cpp:288-350), -1 invalid path / numerical
 * failure.  rhs[k], rows[k * (n_slots + 1) ...] (dense coefficient row, slot keys from
 * sgufp_slot_keys, last entry 0) and obj_mean[k] = sum_s objective_s / S; any output
 * pointer may be NULL.  Paths longer than totalLayers are an argument error. */
int sgufp_subproblem(sgufp_ctx *ctx, int n, const int64_t *path_off, const int16_t *paths, int32_t *type,
                     double *rhs, double *rows, double *obj_mean);
/* Per (path, scenario) detail of the last sgufp_subproblem call, [n * S] each: status (0
 * optimal, 1 infeasible, 2 error, 3 not solved: an earlier scenario of the path is infeasible
 * -- the reference stops at the first infeasible one, grb.cpp:284-351 -- which later scenarios
 * stop depends on timing, the cut does not), primal objective, objective of the dual built. */
int sgufp_subproblem_detail(sgufp_ctx *ctx, int32_t *status, double *objective, double *dual_objective);
/* Warm-started subproblems (networks of up to 2046 nodes, with or without lower bounds): path k
 * starts every scenario from the optimal flow and potentials stored in ring slot warm_src[k]
 * (-1: cold) and stores its own in slot warm_dst[k] (-1: none).  The ring has
 * 2 x max(max_batch, 32) slots, allocated zeroed on first use and never resized; a scenario
 * whose source slot holds no stored state (never written, or that scenario was infeasible or
 * failed there) starts cold.  n <= max_batch; no slot may be both written and read, or written
 * twice, by one call (SGUFP_ERR_ARG).  Results are those of sgufp_subproblem (the same statuses
 * and optimal objectives, the same feasibility rays -- an infeasible scenario is solved by the
 * cold big-M path; the duals of an optimality cut may be another optimal one).  The B&B's
 * refinement loops (sgufp_bnb_step) pick the closest earlier path themselves. */
int sgufp_subproblem_warm(sgufp_ctx *ctx, int n, const int64_t *path_off, const int16_t *paths, const int32_t *warm_src,
                          const int32_t *warm_dst, int32_t *type, double *rhs, double *rows, double *obj_mean);
/* Per (path, scenario) of the last subproblem call: augmenting paths of the successive-
 * shortest-path solve (warm: of the repair; a warm start that fell back to a cold solve
 * reports -1 - cold augmentations) and Bellman-Ford passes. */
int sgufp_subproblem_stats(sgufp_ctx *ctx, int32_t *augmentations, int32_t *passes);
/* Inavap::getKey(q, i, j) (Cut.h:342-344) of every coefficient slot (n_slots entries). */
int sgufp_slot_keys(const sgufp_ctx *ctx, uint64_t *keys);
/* Append cuts given as dense rows (n_slots + 1 doubles each, as sgufp_subproblem returns
 * them) -- the device-side counterpart of Container::add (Cut.h:461-465). */
int sgufp_cuts_append_rows(sgufp_ctx *ctx, int is_feasibility, int n_cuts, const double *rhs, const double *rows);

/* -- batched branch-and-bound (Inavap::DDSolver, DDSolver.cpp:556-846) ------------------
 * The frontier is a LIFO stack of open-node records in HBM.  sgufp_bnb_step pops up to
 * max_nodes (<= max_batch; <= 0: max_batch) records from the top and does for all of them
 * what a worker does for one popped node: skip it if ub <= *incumbent (DDSolver.cpp:707),
 * NodeExplorer::process it against the current pools (exact DDs run their refinement loop
 * with the device subproblem, new cuts are appended to the pools: Container::add), raise
 * *incumbent to the best closed exact bound (CAS-max, :723-731), and push the cutset
 * children of parents with ub > *incumbent (:744-748).  Returns SGUFP_ERR_STATE if any
 * record fails (node status >= 16) or a subproblem fails; sgufp_last_error says which. */
typedef struct {
    int64_t popped;              /* records taken from the frontier */
    int64_t relaxed;             /* NodeExplorer::process calls (popped - pruned_bound) */
    int64_t pruned_bound;
    int64_t pruned_feasibility;
    int64_t pruned_optimality;
    int64_t exact;               /* exact DDs (refinement loop entered) */
    int64_t exact_closed;        /* exact DDs that returned {ub, ub} (incumbent candidates) */
    int64_t subproblems;         /* paths sent to the scenario subproblem */
    int64_t new_feasibility_cuts;
    int64_t new_optimality_cuts;
    int64_t children;            /* cutset children produced */
    int64_t pushed;              /* children pushed (parent ub > incumbent) */
    int64_t frontier;            /* frontier size after the round */
    int64_t dd_nodes, dd_arcs, sweeps;   /* sums over the relaxed records */
    int32_t refine_iters;
    int32_t improved;            /* 1 if *incumbent rose */
    double ms_relax;             /* k_relax time of the round (sgufp_set_timing) */
    int64_t deferred;            /* records whose refinement loop hit the round's limit and
                                    went back on top of the frontier (sgufp_bnb_set_limits) */
    int64_t resumed;             /* deferred records whose loop this round resumed */
} sgufp_bnb_stats;

int sgufp_frontier_clear(sgufp_ctx *ctx);
int sgufp_frontier_size(const sgufp_ctx *ctx, int64_t *n, int64_t *sol_entries);
/* Push n host records on top of the stack (the last record ends on top). */
int sgufp_frontier_push(sgufp_ctx *ctx, int n, const uint16_t *gl, const double *lb, const double *ub,
                        const int64_t *states_off, const int16_t *states, const int64_t *sol_off, const int16_t *sol);
/* Remove n records from the top (from_bottom = 0) or the bottom (oldest, from_bottom = 1:
 * work stealing, cf. lf_queue::m_pop) and return them as host records, in stack order.
 * sgufp_frontier_take_size gives the states / solution entries they need. */
int sgufp_frontier_take_size(sgufp_ctx *ctx, int n, int from_bottom, int64_t *n_states, int64_t *n_sol);
int sgufp_frontier_take(sgufp_ctx *ctx, int n, int from_bottom, uint16_t *gl, double *lb, double *ub,
                        int64_t *states_off, int16_t *states, int64_t *sol_off, int16_t *sol);
/* Copy the n records at stack positions [first, first + n) (0 = bottom) without removing them. */
int sgufp_frontier_peek_size(sgufp_ctx *ctx, int64_t first, int n, int64_t *n_states, int64_t *n_sol);
int sgufp_frontier_peek(sgufp_ctx *ctx, int64_t first, int n, uint16_t *gl, double *lb, double *ub,
                        int64_t *states_off, int16_t *states, int64_t *sol_off, int16_t *sol);
int sgufp_bnb_step(sgufp_ctx *ctx, int max_nodes, double *incumbent, sgufp_bnb_stats *stats);
/* Bound the exact-leaf refinement loops of one sgufp_bnb_step: at most max_refine_iters
 * iterations (subproblem batches) and round_seconds of wall time (0: no limit).  Records
 * still in their loop are pushed back on top of the frontier with the bound reached; popped
 * again they rebuild, apply the pool (their own new cuts included) and resume the loop with
 * the paths it had seen (kept by the context until then; sgufp_frontier_clear drops them). */
int sgufp_bnb_set_limits(sgufp_ctx *ctx, int max_refine_iters, double round_seconds);
/* Round trace for tests and diagnostics (off by default).  With it on, every sgufp_bnb_step
 * keeps what its round did, readable until the next step:
 *   kind 0  popped records: record = index in the popped batch (0 = the deepest of the top b
 *           stack entries), code = node status after the relaxation (SGUFP_PRUNED_BY_BOUND for
 *           ub <= zOpt, DDSolver.cpp:707-711), value = the record's ub as popped, no path;
 *   kind 1  scenario subproblems of the refinement loops, in the order they were solved
 *           (NodeExplorer.cpp:957-969): record, code = cut type (0 optimality, 1 feasibility),
 *           row = index of the appended cut in that list (sgufp_cuts_rows), value = sum_s obj_s / S,
 *           path = the argmax path sent to the subproblem;
 *   kind 2  closed loops (the argmax path repeated, {ub, ub}, NodeExplorer.cpp:948-956): record,
 *           value = ub (the incumbent candidate), path = the repeated path;
 *   kind 3  the popped records' k_relax waves: record, code = exact single-cut redos, row = cuts
 *           swept, value = the wave's wall_clock64 ticks (100 MHz; 0 unless the profiling
 *           build lib_prof/ stamps them).
 * Any output pointer may be NULL; path_off has count + 1 entries. */
int sgufp_bnb_set_trace(sgufp_ctx *ctx, int enabled);
int sgufp_bnb_trace(sgufp_ctx *ctx, int kind, int64_t *count, int64_t *path_entries, int32_t *record, int32_t *code,
                    int32_t *row, double *value, int64_t *path_off, int16_t *paths);
/* Read back pool cuts [first, first + count) of one list (insertion order) as dense rows,
 * e.g. to all-gather the cuts a round produced to the other frontier shards. */
int sgufp_cuts_rows(sgufp_ctx *ctx, int is_feasibility, int first, int count, double *rhs, double *rows);

/* -- frontier shards over RCCL (one context per GPU / process; shard.cpp) -------------
 * The reference's threads share the incumbent (std::atomic<double> CAS, DDSolver.cpp:723-731),
 * the global cut Containers (DDSolver.h:415-416) and the work queues (master half-split and
 * 40 % steal, DDSolver.cpp:603-652).  A sharded DDSolver runs one context per GPU and, after
 * every sgufp_bnb_step, makes those exchanges between the contexts of one RCCL communicator,
 * device buffer to device buffer on the context stream.  Without sgufp_comm_init (one shard)
 * every call below is a no-op that leaves its outputs as for a single shard. */
#define SGUFP_COMM_ID_BYTES 128
/* On one rank; the bytes reach the other ranks by any side channel (MPI, a file, a store). */
int sgufp_comm_unique_id(uint8_t *id, int bytes);
int sgufp_comm_init(sgufp_ctx *ctx, int world, int rank, const uint8_t *id);
int sgufp_comm_info(const sgufp_ctx *ctx, int *world, int *rank);
/* The same exchanges between `world` contexts of ONE process, each driven by its own host
 * thread (several shards on one GPU; tests of the multi-shard protocol on one card): a group
 * handle, then sgufp_comm_init_loopback on every context with its rank.  Collectives become
 * device-to-device copies between two barriers; every rank must make the same calls in the
 * same order (a rank that stops makes the others fail after 300 s instead of hanging). */
typedef struct sgufp_loopback sgufp_loopback;
sgufp_loopback *sgufp_loopback_create(int world);
void sgufp_loopback_destroy(sgufp_loopback *group);   /* after sgufp_comm_destroy / sgufp_destroy of its contexts */
int sgufp_comm_init_loopback(sgufp_ctx *ctx, sgufp_loopback *group, int rank);
void sgufp_comm_destroy(sgufp_ctx *ctx);
/* *inout := max over the shards (replaces the CAS-max, DDSolver.cpp:723-731). */
int sgufp_incumbent_allreduce(sgufp_ctx *ctx, double *inout);
/* Every shard's pool rows appended since the last exchange are appended on every other
 * shard, in rank order, feasibility list then optimality list (Container::add of another
 * worker's cut).  *received = rows this shard appended. */
int sgufp_cuts_exchange(sgufp_ctx *ctx, int64_t *received);
/* sizes[world] := every shard's frontier size (termination: all zero). */
int sgufp_frontier_sizes(sgufp_ctx *ctx, int64_t *sizes);
/* While a shard is idle, every busy shard gives records from the bottom of its stack (40 %
 * of >= 32, lf_queue::m_pop; half of fewer, the master's hand-out) and the idle shards
 * split each donor's records in contiguous chunks.  *received = records this shard got. */
int sgufp_frontier_balance(sgufp_ctx *ctx, int64_t *received);
/* The plan sgufp_frontier_balance follows, host only (no device is touched): from every
 * shard's stack size, give[r] = records shard r gives (0 when no shard is idle), idle[0..ni)
 * = the idle shards in rank order, and idle shard j gets records [chunk_lo[r * world + j],
 * chunk_hi[r * world + j]) of donor r's bottom records (chunk arrays [world * world], may be
 * NULL).  Returns ni (< 0: bad arguments). */
int sgufp_balance_plan(int world, const int64_t *sizes, int64_t *give, int32_t *idle, int64_t *chunk_lo,
                       int64_t *chunk_hi);
/* all[world * k] := every shard's k (<= 4) int64 values (e.g. the per-shard counters that a
 * sharded DDSolver prints on rank 0). */
int sgufp_comm_allgather_i64(sgufp_ctx *ctx, const int64_t *mine, int k, int64_t *all);

/* -- restricted decision diagram (replaces Inavap::RestrictedDDNew, DD.h:653-730 /
 *    DD.cpp:3090-3505, driven as in NodeExplorer::processX3, NodeExplorer.cpp:605-656) --
 * For every staged node (sgufp_batch_upload): RestrictedDDNew{net, width}.compile(node)
 * (width <= 128), then the pool's feasibility cuts and then its optimality cuts, each list
 * newest first (applyFeasibilityCut / applyOptimalityCut); the first false ends the node
 * with status 1, the first bound <= optimal_lb with status 2. */
int sgufp_restricted_relax(sgufp_ctx *ctx, int width, double optimal_lb);
/* Per staged node: status (0, 1, 2; 16 = record not representable), isTreeExact(), the
 * bound of the last optimality cut applied (node.lb when none), the length of the max path
 * (getSolution, status 0 only, else 0) and the number of exact-cutset records compile()
 * returned (0 for an exact tree).  Any pointer may be NULL. */
int sgufp_restricted_results(sgufp_ctx *ctx, int32_t *status, uint8_t *exact, double *lb, int32_t *path_len,
                             int32_t *cutset_n);
/* Max paths (path_off has n+1 entries). */
int sgufp_restricted_paths(sgufp_ctx *ctx, int64_t *path_off, int16_t *paths);
/* The exact cutsets as Inavap::Node records (getExactCutSet, DD.cpp:3279-3288: states,
 * solution, lb = ub = DOUBLE_MIN, globalLayer); node k's are [rec_off[k], rec_off[k+1]). */
int sgufp_restricted_cutset_size(sgufp_ctx *ctx, int64_t *n_records, int64_t *n_states, int64_t *n_sol);
int sgufp_restricted_cutset(sgufp_ctx *ctx, int64_t *rec_off, uint16_t *gl, double *lb, double *ub,
                            int64_t *states_off, int16_t *states, int64_t *sol_off, int16_t *sol);

/* -- timing (hipEvents on the ctx stream around each kernel of the last relax) -- */
int sgufp_set_timing(sgufp_ctx *ctx, int enabled);
int sgufp_last_timing(const sgufp_ctx *ctx, float *ms_relax, float *ms_emit);

#ifdef __cplusplus
}
#endif

#endif /* SGUFP_HIP_H */
