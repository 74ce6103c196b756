// Context of libsgufp_hip.so shared by capi.cpp (C ABI) and bnb.cpp (B&B rounds):
// device tables, scratch, cut pool, staged batch / device frontier and outputs.
#pragma once

#include "sgufp_hip.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#define SGUFP_HOST_ONLY 1  // no device code here: plain pointers in the device pass too
#include "dd_device.hpp"
#include "network.hpp"
#include "sub_device.hpp"
#include "rdd_device.hpp"

namespace sgufp {
struct Transport;   // shard.cpp
// dd_kernels.hip
size_t relax_lds_bytes(int Tcap, int Lcap, int cb, int us);
size_t sub_lds_bytes(int n, int m, int nct_cap, int nz, int nw, int kbytes = 8, bool warm = false, bool wl = false);
hipError_t launch_subproblem(const SubNet &N, const SubIO &io, hipStream_t st);
hipError_t launch_warm_pick(const SubIO &io, const WarmRing &wr, int ptr, hipStream_t st);
hipError_t launch_relax(const NetDev &, const Scratch &, const BatchIn &, const Pool &, const BatchOut &, double, int,
                        const ExactIO &, int, hipStream_t);
// exact_kernels.hip
hipError_t launch_exact_cols(const double *rows, const double *rhs, const int32_t *o_order, int no, int first,
                             int stride, int n_slots, int ostride, double *coefO, int reverse, hipStream_t st);
hipError_t launch_scan(const uint32_t *, const uint32_t *, int, uint64_t *, uint64_t *, hipStream_t);
hipError_t launch_emit(const NetDev &, const Scratch &, const BatchIn &, const Pool &, const BatchOut &,
                       const ChildOut &, hipStream_t);
hipError_t launch_refine(const NetDev &, const Scratch &, const BatchIn &, const Pool &, const BatchOut &,
                         const int32_t *, const int32_t *, const uint8_t *, int, double, const ExactIO &, hipStream_t);
hipError_t launch_gather_paths(const BatchOut &, int Lcap, const int32_t *idx, const int64_t *off, int n,
                               int16_t *dst, hipStream_t);
hipError_t launch_push_children(const ChildOut &, const BatchOut &, const int32_t *parents, const int64_t *dst_child,
                                const int64_t *dst_sol, int n, const FrontierDev &, hipStream_t);
// one DD at a time (RelaxedDDNew surface): build without cuts, one cut, argmax path, cutset
hipError_t launch_dd_build(const NetDev &, const Scratch &, const BatchIn &, const BatchOut &, int stride, hipStream_t);
hipError_t launch_dd_apply(const NetDev &, const Scratch &, const BatchIn &, const BatchOut &, int slot, const double *rows,
                           int stride, double rhs, int is_feas, double optimal, double *value, hipStream_t);
hipError_t launch_dd_solution(const NetDev &, const Scratch &, const BatchIn &, const BatchOut &, int slot,
                              const double *rows, int stride, hipStream_t);
hipError_t launch_dd_cutset(const NetDev &, const Scratch &, const BatchOut &, int slot, double ub, hipStream_t);
// 1 when k_relax was built with its per-wave clock stamps (SGUFP_PHASES, lib_prof/)
bool relax_has_phases();
// rdd_kernels.hip
size_t rdd_lds_bytes(int Tcap, int Lcap, int us);
hipError_t launch_restrict(const NetDev &, const BatchIn &, const Pool &, const RddIO &, double, hipStream_t);
}  // namespace sgufp

using namespace sgufp;

namespace {

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
};

}  // namespace

struct EncodedRecords {
    std::vector<uint32_t> mask;
    std::vector<uint8_t> valid;
    std::vector<int64_t> soff;
    std::vector<uint16_t> slen;
    std::vector<int16_t> sols;
};

struct sgufp_ctx {
    Network net;
    int device = 0;
    int max_batch = 0;
    hipStream_t stream = nullptr;
    std::string err;
    std::vector<DevBuf> allocs;
    size_t held = 0;

    NetDev nd{};
    Scratch sc{};
    BatchOut out{};

    // key (low 48 bits) -> slots carrying it
    std::unordered_map<uint64_t, std::vector<int>> key_slots;

    // cut pool
    int row_cap = 0, n_rows = 0;
    double *d_rows = nullptr, *d_rhs = nullptr, *d_coefT = nullptr;
    int ustride = 1;
    int cb = 4;                               // cuts per batched sweep
    std::vector<int32_t> f_rows, o_rows;      // insertion order, row ids
    int32_t *d_forder = nullptr, *d_oorder = nullptr;
    int32_t *d_orank = nullptr;               // optimality rows by ascending row_ub (screening order)
    std::vector<double> row_ub;               // per row: RHS + sum_l max_r coef (node-independent bound)
    int nscreen = 4;                          // optimality cuts screened before the exact phase
    int order_cap = 0;
    bool order_dirty = true;

    // current batch: the staged arrays below (sgufp_batch_upload) or a slice of the
    // device frontier (sgufp_bnb_step)
    BatchIn cur{};
    // device frontier: the open-node work list of the B&B (lock_free_queue / lf_node lists,
    // lock_free_queue.h:24-165, DDSolver.h:264-291), a LIFO stack in HBM
    FrontierDev fr{};
    int64_t fr_n = 0, fr_cap = 0;
    size_t fr_sol_cap = 0;
    int64_t fr_sol_top = 0;                   // arena entries in use (host mirror)
    bool frontier_reserve(int64_t entries, size_t sol_entries);
    // B&B step staging (host mirrors + small device index arrays)
    int32_t *d_bidx = nullptr;                // [max_batch] node indices (paths / parents)
    int32_t *d_perm = nullptr;                // [max_batch] k_relax dispatch order (relax_current)
    int perm_n = -1;                          // batch size d_perm was drawn for
    int64_t *d_boff = nullptr, *d_bsol = nullptr;  // [max_batch + 1]
    int16_t *d_bpaths = nullptr;              // [max_batch * Lcap] gathered paths
    // seen-path lists of records whose refinement loop a round deferred, keyed by the
    // record (gl, state mask, solution): restored when the record is popped again
    std::unordered_map<std::string, std::vector<std::vector<int16_t>>> deferred_seen;
    static void make_record_key(uint16_t gl, uint32_t mask, const int16_t *sol, size_t len, std::string &key);
    // keys of the frontier entries [lo, lo + count) (bulk downloads, one synchronisation)
    bool slice_keys(int64_t lo, int count, std::vector<std::string> &keys);
    // round trace (sgufp_bnb_set_trace): what the last sgufp_bnb_step did, for tests
    bool trace = false;
    struct TraceItem {
        int32_t record = -1, code = 0, row = -1;
        double value = 0.0;
        std::vector<int16_t> path;
    };
    std::vector<TraceItem> trace_items[4];    // 0 popped, 1 subproblems, 2 closed loops, 3 k_relax waves
    // device-resident refinement loop (bnb.cpp, bnb_kernels.hip): seen-path lists per batch
    // slot and the per-iteration index / flag arrays
    SeenLists seen{};
    int seen_slots = 0;
    int32_t *d_lact = nullptr, *d_lflag = nullptr, *d_lchain = nullptr;
    double *d_lrowub = nullptr;
    bool loop_reserve(int slots, int cap);
    bool seen_upload(int slot, const std::vector<std::vector<int16_t>> &paths);
    bool seen_download(int slot, int count, std::vector<std::vector<int16_t>> &paths);
    int bnb_max_iters = 0;                    // refinement iterations per round (0: no limit)
    int64_t chunk_lps = 32768;                // scenario LPs per refinement iteration under a round
                                              // deadline (SGUFP_CHUNK_LPS)
    double bnb_seconds = 0.0;                 // refinement-loop seconds per round (0: no limit)
    bool relax_current(double optimal_lb);
    bool relax_order(BatchIn &in);
    void encode_records(int n, const uint16_t *gl, const int64_t *states_off, const int16_t *states,
                        const int64_t *sol_off, const int16_t *sol, EncodedRecords &e) const;
    // device records [count] (mask over the layer's universe) -> host states, as sgufp_batch_children
    void decode_states(const uint16_t *gl, const uint32_t *mask, size_t count, int64_t *states_off,
                       int16_t *states) const;

    // staged batch
    int n = 0;
    uint16_t *d_gl = nullptr, *d_sollen = nullptr;
    double *d_lb = nullptr, *d_ub = nullptr;
    uint32_t *d_mask = nullptr;
    uint8_t *d_valid = nullptr;
    int64_t *d_soloff = nullptr;
    int16_t *d_sol = nullptr;
    size_t sol_cap = 0;

    // outputs / children
    uint64_t *d_coff = nullptr, *d_soff = nullptr;
    size_t child_cap = 0, csol_cap = 0;
    uint16_t *d_cgl = nullptr, *d_csollen = nullptr;
    double *d_clb = nullptr, *d_cub = nullptr;
    uint32_t *d_cmask = nullptr;
    int64_t *d_csoloff = nullptr;
    int16_t *d_csol = nullptr;
    int64_t total_children = 0, total_csol = 0;
    bool relaxed = false;
    double relax_lb = 0.0;       // optimalLB of the last relaxation (sgufp_batch_refine may not go lower)
    bool exact_capped = false;   // the exact phase's column store outgrew device memory: k_relax sweeps

    // one DD at a time (sgufp_dd_*): per staged slot, the dense row of the last cut applied
    bool dd_built = false;
    double *d_ddrow = nullptr, *d_ddval = nullptr;
    bool emit_current(const BatchIn &in, const Pool &p);   // scan + k_emit_children of the batch
    int densify(int64_t nnz, const uint64_t *keys, const double *vals, double *row);   // cutToCut + Cut::get

    // refine staging
    int32_t *d_rslots = nullptr, *d_rcuts = nullptr;
    uint8_t *d_rfeas = nullptr;

    // scenario subproblem (built on first use)
    bool sub_ready = false;
    SubNet sn{};
    SubIO sio{};
    int sub_cap = 0;                          // paths the per-path buffers hold
    size_t sub_path_cap = 0;                  // int16 decisions
    int64_t *d_spoff = nullptr;
    int16_t *d_spaths = nullptr;
    int sub_last_n = 0;
    int32_t *d_wstat = nullptr;               // [sub_cap * S * 2] per (path, scenario): augmentations, passes
    // warm-start ring of the scenario subproblem (SGUFP_SUB_WARM=0: off): flows + potentials of
    // earlier solves, for the refinement loops' next paths (bnb.cpp)
    bool warm_on = true;
    WarmRing wring{};
    int warm_ptr = 0;
    int16_t *d_wx = nullptr;
    int32_t *d_wa = nullptr;
    uint8_t *d_wok = nullptr;                 // [R][S] the (slot, scenario) holds a stored state
    bool warm_reserve();                      // ring of 2 x max(max_batch, 32) slots, sized once
                                              // (false: no ring, cold subproblems)
    // SGUFP_SUB_STATS=1: the B&B's subproblem launches' augmentations and Bellman-Ford passes
    // (io.wstat), summed and printed to stderr every 200 launches (diagnostics; syncs per launch)
    bool sub_stats = false;
    double ss[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // launches, scenarios, warm, augs, flow passes, potential passes, fallbacks, cold augs
    void sub_stats_add(int n_paths);
    bool sub_init();
    bool sub_grow(int n, size_t total);
    bool append_rows(int is_feasibility, int n_cuts, const double *rhs, const std::vector<double> &rows);

    // restricted DD (built on first use)
    bool rdd_ready = false;
    bool restricted_done = false;
    RddIO rio{};
    bool rdd_init();

    // frontier shards (shard.cpp): the exchanges go through a transport -- RCCL between
    // processes / GPUs, or an in-process loopback between contexts driven by threads of one
    // process (tests, several shards on one GPU); nullptr for one shard
    sgufp::Transport *comm = nullptr;
    int world = 1, rank = 0;
    int shared[2] = {0, 0};                   // rows of the optimality [0] / feasibility [1] list
                                              // already exchanged (own rows after that are new)
    int64_t *d_comm_i64 = nullptr;            // [4 * world + 4] small all-gathers
    double *d_comm_f64 = nullptr;             // [1] incumbent all-reduce
    double *d_xsend = nullptr, *d_xrecv = nullptr, *d_xub = nullptr;
    int32_t *d_xids = nullptr;
    int64_t *d_xspan = nullptr;
    size_t xsend_cap = 0, xrecv_cap = 0, xub_cap = 0, xids_cap = 0, xspan_cap = 0;
    uint8_t *bounce = nullptr;                // overlapping frontier moves (frontier_drop_bottom)
    size_t bounce_cap = 0;
    bool frontier_drop_bottom(int64_t count);
    double *d_rowbuf = nullptr;               // sgufp_cuts_rows gather buffer
    int32_t *d_rowids = nullptr;
    size_t rowbuf_cap = 0, rowids_cap = 0;

    // cut-parallel optimality phase of exact DDs (exact_kernels.hip; SGUFP_EXACT_FAST=0: off)
    bool exact_fast = true;
    int cus = 256;                            // compute units (persistent grids)
    ExactIO ex{};
    double *d_coefO = nullptr, *d_R = nullptr, *d_coefS = nullptr, *d_RS = nullptr;
    int exact_screen = 0;                     // screening columns (SGUFP_EXACT_SCREEN; measured no gain)
    int ocap = 0, o_built = 0;                // columns of coefO allocated / filled
    int32_t *d_pslot = nullptr;
    uint32_t *d_pbase = nullptr;
    unsigned long long *d_ectr = nullptr;
    int32_t *d_pidx = nullptr;
    int exact_lazy = 0;                       // ExactIO::lazy (SGUFP_EXACT_LAZY)
    // the same for non-exact DDs under large pools (nx_kernels: SGUFP_NX=0 off, SGUFP_NX_MIN)
    bool nx_on = true;
    int nx_min = 2048;
    int nx_skip = 256;
    int32_t *d_pkind = nullptr, *d_P = nullptr, *d_nxh = nullptr, *d_pstop = nullptr, *d_nxlist = nullptr;
    // open-leaf compaction of the exact leaf passes (SGUFP_LEAF_SPLIT cut blocks in phase A; 0: off)
    int leaf_split = 16;
    unsigned long long leaf_cum[5] = {0, 0, 0, 0, 0};   // SGUFP_EXACT_STATS: leaf pass-blocks, staged row-blocks (summed)
    int32_t *d_open_cnt = nullptr, *d_open_list = nullptr;
    double *d_G = nullptr;
    unsigned long long *d_MS = nullptr;
    int nx_cap = 0;                           // columns of G / MS allocated
    bool nx_prepare(int no);
    bool exact_prepare();

    bool timing = false;
    hipEvent_t ev[4] = {};
    float ms_relax = 0, ms_emit = 0;

    ~sgufp_ctx();
    void destroy_all() {
        if (device >= 0) (void)hipSetDevice(device);
        for (auto &b : allocs) (void)hipFree(b.p);
        for (auto &e : ev)
            if (e) (void)hipEventDestroy(e);
        if (stream) (void)hipStreamDestroy(stream);
    }

    bool hip_ok(hipError_t e, const char *what) {
        if (e == hipSuccess) return true;
        err = std::string(what) + ": " + hipGetErrorString(e);
        return false;
    }

    template <typename T>
    bool alloc(T *&ptr, size_t count, const char *what) {
        void *p = nullptr;
        size_t bytes = std::max<size_t>(count, 1) * sizeof(T);
        if (!hip_ok(hipMalloc(&p, bytes), what)) return false;
        allocs.push_back({p, bytes});
        held += bytes;
        ptr = (T *)p;
        return true;
    }
    template <typename T>
    void release(T *&ptr) {
        for (size_t k = 0; k < allocs.size(); k++)
            if (allocs[k].p == (void *)ptr) {
                (void)hipFree(ptr);
                held -= allocs[k].bytes;
                allocs.erase(allocs.begin() + (long)k);
                break;
            }
        ptr = nullptr;
    }
    template <typename T>
    bool upload(T *dst, const T *src, size_t count) {
        if (!count) return true;
        return hip_ok(hipMemcpyAsync(dst, src, count * sizeof(T), hipMemcpyHostToDevice, stream), "H2D");
    }
    template <typename T>
    bool download(T *dst, const T *src, size_t count) {
        if (!count) return true;
        return hip_ok(hipMemcpyAsync(dst, src, count * sizeof(T), hipMemcpyDeviceToHost, stream), "D2H");
    }
    bool sync() { return hip_ok(hipStreamSynchronize(stream), "stream sync"); }

    bool init();
    bool grow_rows(int need);
    bool push_orders();
    bool grow_children(size_t nchild, size_t nsol);
    Pool pool() const {
        Pool p;
        p.rows = d_rows; p.rhs = d_rhs; p.stride = net.n_slots + 1;
        p.f_order = d_forder; p.nf = (int)f_rows.size();
        p.o_order = d_oorder; p.no = (int)o_rows.size();
        p.coefT = d_coefT; p.ustride = ustride;
        p.o_rank = d_orank; p.nscreen = d_orank ? nscreen : 0;
        return p;
    }
    BatchIn staged() const {
        BatchIn b;
        b.n = n; b.gl = d_gl; b.lb = d_lb; b.ub = d_ub; b.mask = d_mask; b.valid = d_valid;
        b.sol_off = d_soloff; b.sol_len = d_sollen; b.sol = d_sol;
        b.bound_prune = 0;
        b.perm = nullptr;
        return b;
    }
    BatchIn frontier_slice(int64_t base, int count) const {
        BatchIn b;
        b.n = count; b.gl = fr.gl + base; b.lb = fr.lb + base; b.ub = fr.ub + base; b.mask = fr.mask + base;
        b.valid = fr.valid + base; b.sol_off = fr.sol_off + base; b.sol_len = fr.sol_len + base; b.sol = fr.sol;
        b.bound_prune = 1;   // Worker::startWorker skips nodes with ub <= zOpt (DDSolver.cpp:707-711)
        b.perm = nullptr;
        return b;
    }
    const BatchIn &batch() const { return cur; }
    ChildOut children_view() const {
        ChildOut co;
        co.child_off = d_coff; co.sol_base = d_soff;
        co.gl = d_cgl; co.lb = d_clb; co.ub = d_cub; co.mask = d_cmask;
        co.sol_off = d_csoloff; co.sol_len = d_csollen; co.sol = d_csol;
        return co;
    }
};
