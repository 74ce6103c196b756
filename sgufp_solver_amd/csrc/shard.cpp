// Frontier shards over RCCL: the exchanges the reference's threads make through shared
// memory, between the contexts of one communicator (one context per GPU / process):
//
//   sgufp_incumbent_allreduce   the CAS-max on the std::atomic<double> incumbent
//                               (DDSolver.cpp:723-731): ncclAllReduce(MAX) of one f64;
//   sgufp_cuts_exchange         the global feasCutsGlobal / optCutsGlobal Containers every
//                               worker reads (DDSolver.h:415-416, Container::add Cut.h:461-465):
//                               the rows each shard appended since the last exchange are
//                               gathered on the device (k_gather_rows), all-gathered as one
//                               padded block per shard, and appended on every other shard in
//                               rank order without leaving HBM (k_append_rows);
//   sgufp_frontier_sizes        termination (DDSolver.cpp:630-640): all-gather of the stack
//                               sizes;
//   sgufp_frontier_balance      work sharing while a shard is idle: every busy shard gives
//                               records from the bottom of its stack -- 40 % of a stack of at
//                               least 32 (lf_queue::m_pop(0.4), lock_free_queue.h:14,125-164,
//                               the master's steal from every busy worker, DDSolver.cpp:642-652),
//                               half of a smaller one (the master's ceil(q/2) hand-out,
//                               DDSolver.cpp:603-621) -- and the idle shards split every donor's
//                               records in contiguous chunks, sent field by field straight
//                               from / into the SoA frontier arrays (ncclSend / ncclRecv).
// The same plan is computed by sgufp_solver_amd/shards.py (the torch.distributed driver).
//
// The collectives go through a Transport: RCCL (one context per GPU / process, the production
// path) or an in-process loopback between contexts of one process driven by one host thread
// each (sgufp_comm_init_loopback: device-to-device copies on the contexts' streams between two
// barriers), which runs this very code -- plan, packing, rebase, drop-bottom, row append -- with
// W > 1 shards on a single GPU.
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <vector>

#include "ctx.hpp"

namespace sgufp {
hipError_t launch_gather_rows(const double *rows, const double *rhs, const int32_t *ids, int k, int stride, double *out,
                              hipStream_t st);
hipError_t launch_append_rows(const double *src, int n, int stride, int first, double *rows, double *rhs,
                              double *coefT, const int32_t *slot_tab, int L, int us, double *row_ub, hipStream_t st);
hipError_t launch_rebase(int64_t *off, int n, int64_t delta, hipStream_t st);
}  // namespace sgufp

namespace {

constexpr int kQueueLimit = 32;        // _queue_limit_ (lock_free_queue.h:14)
constexpr double kStealShare = 0.4;    // PROPORTION_OF_SHARE (DDSolver.h:22-38)

int64_t give_count(int64_t size) {
    if (size >= kQueueLimit) return size - (int64_t)((double)size * (1.0 - kStealShare));
    if (size >= 2) return size / 2;
    return 0;
}

// The work-sharing plan every shard computes from the all-gathered stack sizes (identical on
// every rank): give[r] records from the bottom of shard r, the idle shards in rank order, and
// idle shard j receiving records [give[r] * j / ni, give[r] * (j + 1) / ni) of every donor r.
// Returns the number of idle shards (0: nothing moves).
int balance_plan(int world, const int64_t *sizes, int64_t *give, int32_t *idle) {
    int ni = 0;
    bool any = false;
    for (int r = 0; r < world; r++) {
        if (sizes[r] == 0) idle[ni++] = r;
        give[r] = sizes[r] > 0 ? give_count(sizes[r]) : 0;
        any = any || give[r] > 0;
    }
    if (ni == 0 || !any) {
        std::fill(give, give + world, 0);
        return 0;
    }
    return ni;
}

void chunk_of(int64_t give, int j, int ni, int64_t &lo, int64_t &hi) {
    lo = give * j / ni;
    hi = give * (j + 1) / ni;
}

bool nccl_ok(sgufp_ctx *ctx, ncclResult_t r, const char *what) {
    if (r == ncclSuccess) return true;
    ctx->err = std::string(what) + ": " + ncclGetErrorString(r);
    return false;
}

template <typename T>
bool grow(sgufp_ctx *ctx, T *&p, size_t &cap, size_t need, const char *what) {
    if (need <= cap && p) return true;
    if (p) ctx->release(p);
    cap = std::max(need, 2 * cap);
    return ctx->alloc(p, cap, what);
}

}  // namespace

namespace sgufp {

// The four collectives of the shard protocol, on device buffers of the calling context's
// stream.  Every rank calls them in the same order.
struct Transport {
    virtual ~Transport() = default;
    virtual bool allreduce_max_f64(sgufp_ctx *ctx, double *d) = 0;                      // one f64, in place
    virtual bool allgather(sgufp_ctx *ctx, const void *send, void *recv, size_t bytes) = 0;   // recv [world][bytes]
    virtual bool group_start(sgufp_ctx *ctx) = 0;                                        // point-to-point group
    virtual bool send(sgufp_ctx *ctx, const void *p, size_t bytes, int peer) = 0;
    virtual bool recv(sgufp_ctx *ctx, void *p, size_t bytes, int peer) = 0;
    virtual bool group_end(sgufp_ctx *ctx) = 0;
};

struct RcclTransport : Transport {
    ncclComm_t c;
    ncclResult_t pending = ncclSuccess;
    explicit RcclTransport(ncclComm_t c_) : c{c_} {}
    ~RcclTransport() override { (void)ncclCommDestroy(c); }
    bool allreduce_max_f64(sgufp_ctx *ctx, double *d) override {
        return nccl_ok(ctx, ncclAllReduce(d, d, 1, ncclFloat64, ncclMax, c, ctx->stream), "ncclAllReduce");
    }
    bool allgather(sgufp_ctx *ctx, const void *send, void *recv, size_t bytes) override {
        return nccl_ok(ctx, ncclAllGather(send, recv, bytes, ncclUint8, c, ctx->stream), "ncclAllGather");
    }
    bool group_start(sgufp_ctx *ctx) override {
        pending = ncclSuccess;
        return nccl_ok(ctx, ncclGroupStart(), "ncclGroupStart");
    }
    bool send(sgufp_ctx *ctx, const void *p, size_t bytes, int peer) override {
        if (bytes && pending == ncclSuccess) pending = ncclSend(p, bytes, ncclUint8, peer, c, ctx->stream);
        return true;
    }
    bool recv(sgufp_ctx *ctx, void *p, size_t bytes, int peer) override {
        if (bytes && pending == ncclSuccess) pending = ncclRecv(p, bytes, ncclUint8, peer, c, ctx->stream);
        return true;
    }
    bool group_end(sgufp_ctx *ctx) override {
        const ncclResult_t re = ncclGroupEnd();
        return nccl_ok(ctx, pending, "ncclSend/ncclRecv") && nccl_ok(ctx, re, "ncclGroupEnd");
    }
};

// Shared state of the loopback shards: a generation barrier (with a time limit, so that a
// rank that stops calling fails the others instead of hanging them), published pointers /
// values, and per (from, to) queues of posted sends.
struct LoopGroup {
    int world;
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    bool broken = false;
    std::vector<const void *> ptr;
    std::vector<double> val;
    std::vector<std::deque<std::pair<const void *, size_t>>> q;   // [from * world + to]
    explicit LoopGroup(int w) : world{w}, ptr(w, nullptr), val(w, 0.0), q((size_t)w * w) {}
    bool barrier() {
        std::unique_lock<std::mutex> lk(m);
        if (broken) return false;
        const uint64_t g = gen;
        if (++arrived == world) {
            arrived = 0;
            gen++;
            cv.notify_all();
            return true;
        }
        static const int secs = [] {
            const char *e = std::getenv("SGUFP_LOOPBACK_TIMEOUT");   // seconds a rank waits for the others
            return e && std::atoi(e) > 0 ? std::atoi(e) : 300;
        }();
        if (!cv.wait_for(lk, std::chrono::seconds(secs), [&] { return gen != g || broken; }) || broken) {
            broken = true;
            cv.notify_all();
            return false;
        }
        return true;
    }
};

struct LoopbackTransport : Transport {
    std::shared_ptr<LoopGroup> g;
    int rank;
    std::vector<std::pair<void *, std::pair<size_t, int>>> recvs;
    std::vector<std::pair<const void *, std::pair<size_t, int>>> sends;
    LoopbackTransport(std::shared_ptr<LoopGroup> g_, int r) : g{std::move(g_)}, rank{r} {}
    bool fail(sgufp_ctx *ctx, const char *what) {
        ctx->err = std::string("loopback transport: ") + what;
        std::lock_guard<std::mutex> lk(g->m);
        g->broken = true;
        g->cv.notify_all();
        return false;
    }
    bool allreduce_max_f64(sgufp_ctx *ctx, double *d) override {
        double v = 0.0;
        if (!ctx->download(&v, d, 1) || !ctx->sync()) return false;
        g->val[rank] = v;
        if (!g->barrier()) return fail(ctx, "barrier");
        double mx = g->val[0];
        for (int r = 1; r < g->world; r++) mx = std::max(mx, g->val[r]);
        if (!g->barrier()) return fail(ctx, "barrier");
        return ctx->upload(d, &mx, 1) && ctx->sync();
    }
    bool allgather(sgufp_ctx *ctx, const void *send, void *recv, size_t bytes) override {
        if (!ctx->sync()) return false;   // the send block is complete on this stream
        g->ptr[rank] = send;
        if (!g->barrier()) return fail(ctx, "barrier");
        for (int r = 0; r < g->world && bytes; r++)
            if (!ctx->hip_ok(hipMemcpyAsync((uint8_t *)recv + (size_t)r * bytes, g->ptr[r], bytes,
                                            hipMemcpyDeviceToDevice, ctx->stream), "loopback D2D"))
                return fail(ctx, "copy");
        if (!ctx->sync()) return fail(ctx, "sync");
        return g->barrier() || fail(ctx, "barrier");   // every rank copied: send blocks reusable
    }
    bool group_start(sgufp_ctx *) override {
        sends.clear();
        recvs.clear();
        return true;
    }
    bool send(sgufp_ctx *, const void *p, size_t bytes, int peer) override {
        if (bytes) sends.push_back({p, {bytes, peer}});
        return true;
    }
    bool recv(sgufp_ctx *, void *p, size_t bytes, int peer) override {
        if (bytes) recvs.push_back({p, {bytes, peer}});
        return true;
    }
    bool group_end(sgufp_ctx *ctx) override {
        if (!ctx->sync()) return false;
        {
            std::lock_guard<std::mutex> lk(g->m);
            for (auto &x : sends) g->q[(size_t)rank * g->world + x.second.second].push_back({x.first, x.second.first});
        }
        if (!g->barrier()) return fail(ctx, "barrier");
        for (auto &x : recvs) {
            std::pair<const void *, size_t> src;
            {
                std::lock_guard<std::mutex> lk(g->m);
                auto &dq = g->q[(size_t)x.second.second * g->world + rank];
                if (dq.empty()) return fail(ctx, "receive without a matching send");
                src = dq.front();
                dq.pop_front();
            }
            if (src.second != x.second.first) return fail(ctx, "send / receive sizes differ");
            if (!ctx->hip_ok(hipMemcpyAsync(x.first, src.first, src.second, hipMemcpyDeviceToDevice, ctx->stream),
                             "loopback D2D"))
                return fail(ctx, "copy");
        }
        if (!ctx->sync()) return fail(ctx, "sync");
        return g->barrier() || fail(ctx, "barrier");
    }
};

}  // namespace sgufp

struct sgufp_loopback {
    std::shared_ptr<sgufp::LoopGroup> g;
};

sgufp_ctx::~sgufp_ctx() {
    if (comm) {
        if (device >= 0) (void)hipSetDevice(device);
        delete comm;
        comm = nullptr;
    }
    destroy_all();
}

bool sgufp_ctx::frontier_drop_bottom(int64_t g) {
    // remove records [0, g) of the stack: the rest moves down through a persistent bounce
    // buffer (source and destination overlap), solution offsets rebased on the device
    if (g <= 0) return true;
    if (g >= fr_n) {
        fr_n = 0;
        fr_sol_top = 0;
        return true;
    }
    const size_t rest = (size_t)(fr_n - g);
    int64_t s_hi = 0;
    if (!download(&s_hi, fr.sol_off + g, 1) || !sync()) return false;
    const size_t srest = (size_t)(fr_sol_top - s_hi);
    const size_t need = std::max(rest * 8, srest * 2);
    if (!grow(this, bounce, bounce_cap, std::max<size_t>(need, 8), "bounce")) return false;
    auto move = [&](void *dst, const void *src, size_t bytes) {
        return bytes == 0 || (hip_ok(hipMemcpyAsync(bounce, src, bytes, hipMemcpyDeviceToDevice, stream), "D2D") &&
                              hip_ok(hipMemcpyAsync(dst, bounce, bytes, hipMemcpyDeviceToDevice, stream), "D2D"));
    };
    const bool ok = move(fr.gl, fr.gl + g, rest * 2) && move(fr.lb, fr.lb + g, rest * 8) &&
                    move(fr.ub, fr.ub + g, rest * 8) && move(fr.mask, fr.mask + g, rest * 4) &&
                    move(fr.valid, fr.valid + g, rest) && move(fr.sol_len, fr.sol_len + g, rest * 2) &&
                    move(fr.sol_off, fr.sol_off + g, rest * 8) && move(fr.sol, fr.sol + s_hi, srest * 2) &&
                    hip_ok(launch_rebase(fr.sol_off, (int)rest, -s_hi, stream), "k_rebase") && sync();
    if (!ok) return false;
    fr_n = (int64_t)rest;
    fr_sol_top = (int64_t)srest;
    return true;
}

extern "C" {

int sgufp_comm_unique_id(uint8_t *id, int bytes) {
    if (!id || bytes < (int)sizeof(ncclUniqueId)) return SGUFP_ERR_ARG;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return SGUFP_ERR_HIP;
    std::memcpy(id, &u, sizeof u);
    return SGUFP_OK;
}

int sgufp_comm_init(sgufp_ctx *ctx, int world, int rank, const uint8_t *id) {
    if (!ctx || !id || world < 1 || rank < 0 || rank >= world || ctx->comm) return SGUFP_ERR_ARG;
    if (!ctx->hip_ok(hipSetDevice(ctx->device), "hipSetDevice")) return SGUFP_ERR_HIP;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    ncclComm_t c = nullptr;
    if (!nccl_ok(ctx, ncclCommInitRank(&c, world, u, rank), "ncclCommInitRank")) return SGUFP_ERR_HIP;
    ctx->comm = new RcclTransport(c);
    ctx->world = world;
    ctx->rank = rank;
    ctx->shared[0] = (int)ctx->o_rows.size();
    ctx->shared[1] = (int)ctx->f_rows.size();
    if (!ctx->alloc(ctx->d_comm_i64, (size_t)4 * world + 4, "comm") || !ctx->alloc(ctx->d_comm_f64, 1, "comm"))
        return SGUFP_ERR_HIP;
    return SGUFP_OK;
}

sgufp_loopback *sgufp_loopback_create(int world) {
    if (world < 1) return nullptr;
    auto *h = new sgufp_loopback;
    h->g = std::make_shared<LoopGroup>(world);
    return h;
}

void sgufp_loopback_destroy(sgufp_loopback *group) { delete group; }

int sgufp_comm_init_loopback(sgufp_ctx *ctx, sgufp_loopback *group, int rank) {
    if (!ctx || !group || rank < 0 || rank >= group->g->world || ctx->comm) return SGUFP_ERR_ARG;
    const int world = group->g->world;
    ctx->comm = new LoopbackTransport(group->g, rank);
    ctx->world = world;
    ctx->rank = rank;
    ctx->shared[0] = (int)ctx->o_rows.size();
    ctx->shared[1] = (int)ctx->f_rows.size();
    if (!ctx->alloc(ctx->d_comm_i64, (size_t)4 * world + 4, "comm") || !ctx->alloc(ctx->d_comm_f64, 1, "comm"))
        return SGUFP_ERR_HIP;
    return SGUFP_OK;
}

int sgufp_comm_info(const sgufp_ctx *ctx, int *world, int *rank) {
    if (!ctx) return SGUFP_ERR_ARG;
    if (world) *world = ctx->world;
    if (rank) *rank = ctx->rank;
    return SGUFP_OK;
}

int sgufp_incumbent_allreduce(sgufp_ctx *ctx, double *inout) {
    if (!ctx || !inout) return SGUFP_ERR_ARG;
    if (!ctx->comm) return SGUFP_OK;   // one shard
    double *d = ctx->d_comm_f64;
    if (!ctx->upload(d, inout, 1) || !ctx->comm->allreduce_max_f64(ctx, d) || !ctx->download(inout, d, 1) || !ctx->sync())
        return SGUFP_ERR_HIP;
    return SGUFP_OK;
}

// [world][k] int64 all-gather of k values per shard (k <= 4)
static bool allgather_i64(sgufp_ctx *ctx, const int64_t *mine, int k, std::vector<int64_t> &all) {
    const int W = ctx->world;
    int64_t *d = ctx->d_comm_i64;   // [4 * W + 4]: send slot at the end
    int64_t *send = d + (size_t)4 * W;
    all.assign((size_t)W * k, 0);
    return ctx->upload(send, mine, (size_t)k) && ctx->comm->allgather(ctx, send, d, (size_t)k * sizeof(int64_t)) &&
           ctx->download(all.data(), d, all.size()) && ctx->sync();
}

int sgufp_frontier_sizes(sgufp_ctx *ctx, int64_t *sizes) {
    if (!ctx || !sizes) return SGUFP_ERR_ARG;
    if (!ctx->comm) {
        sizes[0] = ctx->fr_n;
        return SGUFP_OK;
    }
    std::vector<int64_t> all;
    const int64_t mine = ctx->fr_n;
    if (!allgather_i64(ctx, &mine, 1, all)) return SGUFP_ERR_HIP;
    std::copy(all.begin(), all.end(), sizes);
    return SGUFP_OK;
}

int sgufp_cuts_exchange(sgufp_ctx *ctx, int64_t *received) {
    if (!ctx) return SGUFP_ERR_ARG;
    if (received) *received = 0;
    if (!ctx->comm) return SGUFP_OK;
    const int W = ctx->world, me = ctx->rank;
    const int stride = ctx->net.n_slots + 1, blk = stride + 1;
    const int L = ctx->net.L, us = ctx->ustride;
    int64_t got = 0;
    for (int want = 1; want >= 0; want--) {   // feasibility list, then optimality list
        auto &v = want ? ctx->f_rows : ctx->o_rows;
        const int mark = ctx->shared[want];
        const int64_t k = (int64_t)v.size() - mark;
        std::vector<int64_t> ks;
        if (!allgather_i64(ctx, &k, 1, ks)) return SGUFP_ERR_HIP;
        const int64_t kmax = *std::max_element(ks.begin(), ks.end());
        if (kmax == 0) continue;
        const size_t block = (size_t)kmax * blk;
        if (!grow(ctx, ctx->d_xsend, ctx->xsend_cap, block, "cut exchange") ||
            !grow(ctx, ctx->d_xrecv, ctx->xrecv_cap, block * W, "cut exchange") ||
            !grow(ctx, ctx->d_xids, ctx->xids_cap, (size_t)std::max<int64_t>(k, 1), "cut exchange") ||
            !grow(ctx, ctx->d_xub, ctx->xub_cap, (size_t)kmax, "cut exchange"))
            return SGUFP_ERR_HIP;
        if (k > 0 && (!ctx->upload(ctx->d_xids, v.data() + mark, (size_t)k) ||
                      !ctx->hip_ok(launch_gather_rows(ctx->d_rows, ctx->d_rhs, ctx->d_xids, (int)k, stride, ctx->d_xsend,
                                                      ctx->stream), "k_gather_rows")))
            return SGUFP_ERR_HIP;
        if (!ctx->comm->allgather(ctx, ctx->d_xsend, ctx->d_xrecv, block * sizeof(double))) return SGUFP_ERR_HIP;
        for (int r = 0; r < W; r++) {
            const int n = (int)ks[r];
            if (r == me || n == 0) continue;
            const int first = ctx->n_rows;
            if (!ctx->grow_rows(first + n)) return SGUFP_ERR_HIP;
            if (!ctx->hip_ok(launch_append_rows(ctx->d_xrecv + (size_t)r * block, n, stride, first, ctx->d_rows, ctx->d_rhs,
                                                ctx->d_coefT, ctx->nd.slot_tab, L, us, ctx->d_xub, ctx->stream),
                             "k_append_rows"))
                return SGUFP_ERR_HIP;
            ctx->row_ub.resize((size_t)first + n);
            if (!ctx->download(ctx->row_ub.data() + first, ctx->d_xub, (size_t)n) || !ctx->sync()) return SGUFP_ERR_HIP;
            for (int c = 0; c < n; c++) v.push_back(first + c);
            ctx->n_rows += n;
            ctx->order_dirty = true;
            got += n;
        }
        ctx->shared[want] = (int)v.size();
    }
    if (!ctx->sync()) return SGUFP_ERR_HIP;
    if (received) *received = got;
    return SGUFP_OK;
}

int sgufp_frontier_balance(sgufp_ctx *ctx, int64_t *received) {
    if (!ctx) return SGUFP_ERR_ARG;
    if (received) *received = 0;
    if (!ctx->comm) return SGUFP_OK;
    const int W = ctx->world, me = ctx->rank;
    std::vector<int64_t> sizes;
    const int64_t mine = ctx->fr_n;
    if (!allgather_i64(ctx, &mine, 1, sizes)) return SGUFP_ERR_HIP;
    std::vector<int64_t> give(W, 0);
    std::vector<int32_t> idle(W, -1);
    const int ni = balance_plan(W, sizes.data(), give.data(), idle.data());
    if (ni == 0) return SGUFP_OK;
    idle.resize(ni);
    auto chunk = [&](int r, int j, int64_t &lo, int64_t &hi) { chunk_of(give[r], j, ni, lo, hi); };
    // the given records leave this context: their deferred loops' seen lists go no further
    if (give[me] > 0 && !ctx->deferred_seen.empty()) {
        std::vector<std::string> keys;
        if (!ctx->slice_keys(0, (int)give[me], keys)) return SGUFP_ERR_HIP;
        for (auto &k : keys) ctx->deferred_seen.erase(k);
    }
    // solution spans of this shard's chunks: [sol_lo, sol_hi) per idle shard
    std::vector<int64_t> span((size_t)2 * ni, 0);
    if (give[me] > 0) {
        std::vector<int64_t> off((size_t)give[me] + 1);
        if (!ctx->download(off.data(), ctx->fr.sol_off, (size_t)give[me]) || !ctx->sync()) return SGUFP_ERR_HIP;
        off[give[me]] = give[me] < ctx->fr_n ? 0 : ctx->fr_sol_top;
        if (give[me] < ctx->fr_n && (!ctx->download(&off[give[me]], ctx->fr.sol_off + give[me], 1) || !ctx->sync()))
            return SGUFP_ERR_HIP;
        for (int j = 0; j < ni; j++) {
            int64_t lo, hi;
            chunk(me, j, lo, hi);
            span[2 * j] = off[lo];
            span[2 * j + 1] = off[hi];
        }
    }
    // every shard's spans (ni <= W - 1 pairs each, padded to W)
    std::vector<int64_t> all_span;
    {
        const int per = 2 * W;
        std::vector<int64_t> mine_sp((size_t)per, 0);
        std::copy(span.begin(), span.end(), mine_sp.begin());
        if (!grow(ctx, ctx->d_xspan, ctx->xspan_cap, (size_t)per * (W + 1), "balance")) return SGUFP_ERR_HIP;
        int64_t *send = ctx->d_xspan + (size_t)per * W;
        all_span.assign((size_t)per * W, 0);
        if (!ctx->upload(send, mine_sp.data(), (size_t)per) ||
            !ctx->comm->allgather(ctx, send, ctx->d_xspan, (size_t)per * sizeof(int64_t)) ||
            !ctx->download(all_span.data(), ctx->d_xspan, all_span.size()) || !ctx->sync())
            return SGUFP_ERR_HIP;
    }
    const int myj = (int)(std::find(idle.begin(), idle.end(), me) - idle.begin());
    const bool am_idle = myj < ni;
    // receiver: destinations on top of its (empty) stack, donors in rank order
    struct In { int r; int64_t n, e0, s0, slo, slen; };
    std::vector<In> ins;
    if (am_idle) {
        int64_t e = ctx->fr_n, s = ctx->fr_sol_top;
        for (int r = 0; r < W; r++) {
            if (give[r] == 0) continue;
            int64_t lo, hi;
            chunk(r, myj, lo, hi);
            const int64_t slo = all_span[(size_t)2 * W * r + 2 * myj], shi = all_span[(size_t)2 * W * r + 2 * myj + 1];
            if (hi > lo) ins.push_back({r, hi - lo, e, s, slo, shi - slo});
            e += hi - lo;
            s += shi - slo;
        }
        if (!ctx->frontier_reserve(e, (size_t)s)) return SGUFP_ERR_HIP;
    }
    FrontierDev &f = ctx->fr;
    Transport *X = ctx->comm;
    hipStream_t st = ctx->stream;
    auto xfer = [&](bool send, void *p, size_t bytes, int peer) {
        return send ? X->send(ctx, p, bytes, peer) : X->recv(ctx, p, bytes, peer);
    };
    auto fields = [&](bool send, int64_t e, int64_t n, int64_t s, int64_t slen, int peer) {
        const size_t k = (size_t)n;
        return xfer(send, f.gl + e, k * 2, peer) && xfer(send, f.lb + e, k * 8, peer) && xfer(send, f.ub + e, k * 8, peer) &&
               xfer(send, f.mask + e, k * 4, peer) && xfer(send, f.valid + e, k, peer) &&
               xfer(send, f.sol_len + e, k * 2, peer) && xfer(send, f.sol_off + e, k * 8, peer) &&
               xfer(send, f.sol + s, (size_t)slen * 2, peer);
    };
    if (!X->group_start(ctx)) return SGUFP_ERR_HIP;
    bool ok = true;
    if (give[me] > 0) {
        for (int j = 0; j < ni && ok; j++) {
            int64_t lo, hi;
            chunk(me, j, lo, hi);
            if (hi > lo) ok = fields(true, lo, hi - lo, span[2 * j], span[2 * j + 1] - span[2 * j], idle[j]);
        }
    }
    for (const In &x : ins)
        if (ok) ok = fields(false, x.e0, x.n, x.s0, x.slen, x.r);
    if (!X->group_end(ctx) || !ok) return SGUFP_ERR_HIP;
    int64_t got = 0;
    for (const In &x : ins) {
        if (!ctx->hip_ok(launch_rebase(f.sol_off + x.e0, (int)x.n, x.s0 - x.slo, st), "k_rebase")) return SGUFP_ERR_HIP;
        got += x.n;
    }
    if (!ctx->sync()) return SGUFP_ERR_HIP;
    if (!ins.empty()) {
        const In &last = ins.back();
        ctx->fr_n = last.e0 + last.n;
        ctx->fr_sol_top = last.s0 + last.slen;
    }
    if (give[me] > 0 && !ctx->frontier_drop_bottom(give[me])) return SGUFP_ERR_HIP;
    if (received) *received = got;
    return SGUFP_OK;
}

int sgufp_balance_plan(int world, const int64_t *sizes, int64_t *give, int32_t *idle, int64_t *chunk_lo,
                       int64_t *chunk_hi) {
    if (world < 1 || !sizes || !give || !idle) return -1;
    for (int r = 0; r < world; r++)
        if (sizes[r] < 0) return -1;
    const int ni = balance_plan(world, sizes, give, idle);
    for (int r = 0; r < world; r++)
        for (int j = 0; j < ni; j++) {
            int64_t lo, hi;
            chunk_of(give[r], j, ni, lo, hi);
            if (chunk_lo) chunk_lo[(size_t)r * world + j] = lo;
            if (chunk_hi) chunk_hi[(size_t)r * world + j] = hi;
        }
    return ni;
}

int sgufp_comm_allgather_i64(sgufp_ctx *ctx, const int64_t *mine, int k, int64_t *all) {
    if (!ctx || k < 0 || k > 4 || (k && (!mine || !all))) return SGUFP_ERR_ARG;
    if (!ctx->comm) {
        std::copy(mine, mine + k, all);
        return SGUFP_OK;
    }
    std::vector<int64_t> v;
    if (!allgather_i64(ctx, mine, k, v)) return SGUFP_ERR_HIP;
    std::copy(v.begin(), v.end(), all);
    return SGUFP_OK;
}

void sgufp_comm_destroy(sgufp_ctx *ctx) {
    if (!ctx || !ctx->comm) return;
    delete ctx->comm;
    ctx->comm = nullptr;
    ctx->world = 1;
    ctx->rank = 0;
}

}  // extern "C"
