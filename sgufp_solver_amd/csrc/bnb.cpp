// Batched branch-and-bound rounds on the device: the replacement of the reference's
// DDSolver master/worker loop (DDSolver.cpp:556-846) around NodeExplorer::process
// (NodeExplorer.cpp:915-986), with the open-node frontier resident in HBM.
//
// One round (sgufp_bnb_step) = what the reference's workers do for a batch of popped nodes:
//   1. pop the top `b` records of the frontier stack (LIFO like lf_queue::pop);
//   2. prune records with ub <= zOpt unprocessed (DDSolver.cpp:707-711) -- inside k_relax;
//   3. process every other record against the current pools and zOpt (k_relax + k_emit);
//   4. exact DDs run the refinement loop of NodeExplorer.cpp:946-969: argmax path, stop when
//      the path was seen ({ub, ub}), else the device scenario subproblem, the new cut is
//      appended to the global pool (Container::add) and applied to that DD (k_refine);
//   5. incumbent = max(zOpt, lb of closed exact DDs)  (the CAS at DDSolver.cpp:723-731);
//   6. cutset children of parents with ub > zOpt are pushed (DDSolver.cpp:744-748),
//      compacted from the emit buffers onto the stack where the popped batch was.
// Records processed in one round all see the same zOpt and pools, as concurrent workers
// of the reference may.  Children of a parent keep the reference's cutset order; parents
// keep their frontier order, so the top of the stack is the last parent's first child.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "ctx.hpp"

namespace sgufp {
hipError_t launch_loop_check(const BatchOut &out, const SeenLists &S, const int32_t *act, int na, int m, int32_t *flag,
                             int32_t *chains, hipStream_t st);
hipError_t launch_seen_append(const BatchOut &out, const SeenLists &S, const int32_t *fresh, int nf, int m,
                              hipStream_t st);
hipError_t launch_append_cuts(const int32_t *cut_type, const double *cut_rhs, const double *cut_row, int nf, int stride,
                              int first, double *rows, double *rhs, double *coefT, const int32_t *slot_tab, int L,
                              int us, double *row_ub, int32_t *row_id, uint8_t *is_feas, hipStream_t st);
hipError_t launch_gather_rows(const double *rows, const double *rhs, const int32_t *ids, int k, int stride, double *out,
                              hipStream_t st);
}  // namespace sgufp

void sgufp_ctx::decode_states(const uint16_t *gl, const uint32_t *mask, size_t count, int64_t *states_off,
                              int16_t *states) const {
    int64_t ss = 0;
    for (size_t c = 0; c < count; c++) {
        if (states_off) states_off[c] = ss;
        const int u = net.layer_universe[gl[c]];
        for (uint32_t m = mask[c]; m; m &= m - 1) {
            if (states) states[ss] = net.sets[u][__builtin_ctz(m)];
            ss++;
        }
    }
    if (states_off) states_off[count] = ss;
}

bool sgufp_ctx::frontier_reserve(int64_t entries, size_t sol_entries) {
    if (entries > fr_cap) {
        const int64_t cap = std::max<int64_t>(entries, std::max<int64_t>(2 * fr_cap, 4096));
        FrontierDev f{};
        if (!alloc(f.gl, cap, "frontier") || !alloc(f.lb, cap, "frontier") || !alloc(f.ub, cap, "frontier") ||
            !alloc(f.mask, cap, "frontier") || !alloc(f.valid, cap, "frontier") ||
            !alloc(f.sol_off, cap, "frontier") || !alloc(f.sol_len, cap, "frontier"))
            return false;
        const size_t k = (size_t)fr_n;
        if (k && (!hip_ok(hipMemcpyAsync(f.gl, fr.gl, k * 2, hipMemcpyDeviceToDevice, stream), "D2D") ||
                  !hip_ok(hipMemcpyAsync(f.lb, fr.lb, k * 8, hipMemcpyDeviceToDevice, stream), "D2D") ||
                  !hip_ok(hipMemcpyAsync(f.ub, fr.ub, k * 8, hipMemcpyDeviceToDevice, stream), "D2D") ||
                  !hip_ok(hipMemcpyAsync(f.mask, fr.mask, k * 4, hipMemcpyDeviceToDevice, stream), "D2D") ||
                  !hip_ok(hipMemcpyAsync(f.valid, fr.valid, k, hipMemcpyDeviceToDevice, stream), "D2D") ||
                  !hip_ok(hipMemcpyAsync(f.sol_off, fr.sol_off, k * 8, hipMemcpyDeviceToDevice, stream), "D2D") ||
                  !hip_ok(hipMemcpyAsync(f.sol_len, fr.sol_len, k * 2, hipMemcpyDeviceToDevice, stream), "D2D")))
            return false;
        if (!sync()) return false;
        release(fr.gl); release(fr.lb); release(fr.ub); release(fr.mask); release(fr.valid);
        release(fr.sol_off); release(fr.sol_len);
        f.sol = fr.sol;
        fr = f;
        fr_cap = cap;
    }
    if (sol_entries > fr_sol_cap) {
        const size_t cap = std::max(sol_entries, std::max<size_t>(2 * fr_sol_cap, 1 << 20));
        int16_t *s = nullptr;
        if (!alloc(s, cap, "frontier sol")) return false;
        if (fr_sol_top && !hip_ok(hipMemcpyAsync(s, fr.sol, (size_t)fr_sol_top * 2, hipMemcpyDeviceToDevice, stream), "D2D"))
            return false;
        if (!sync()) return false;
        release(fr.sol);
        fr.sol = s;
        fr_sol_cap = cap;
    }
    return true;
}

// Seen-path lists of the refinement loops: slots x cap entries of Lcap int16 + len + hash, i.e.
// slots x cap x (2 Lcap + 10) bytes (1 024 slots x 64 x 572 B = 37 MB at 1k arcs).  cap doubles
// when one loop outgrows it and is kept for the search (the longest loop sets it); the lists go
// with sgufp_frontier_clear.
bool sgufp_ctx::loop_reserve(int slots, int cap) {
    const int Lc = std::max(sc.Lcap, 1);
    if (!d_lact) {
        const size_t B = (size_t)std::max(max_batch, 1);
        if (!alloc(d_lact, B, "loop") || !alloc(d_lflag, B, "loop") || !alloc(d_lchain, B, "loop") ||
            !alloc(d_lrowub, B, "loop"))
            return false;
    }
    if (seen.paths && slots <= seen_slots && cap <= seen.cap) return true;
    // grow (keeping the lists: a loop can outgrow the capacity mid-round)
    const int ns = std::max(slots, seen_slots);
    const int nc = std::max(cap, std::max(64, seen.cap ? 2 * seen.cap : 0));
    SeenLists t{};
    t.cap = nc;
    t.Lcap = Lc;
    if (!alloc(t.paths, (size_t)ns * nc * Lc, "seen paths") || !alloc(t.len, (size_t)ns * nc, "seen paths") ||
        !alloc(t.hash, (size_t)ns * nc, "seen paths") || !alloc(t.n, (size_t)ns, "seen paths"))
        return false;
    if (seen.paths) {
        const int oc = seen.cap;
        for (int sl = 0; sl < seen_slots; sl++) {
            if (!hip_ok(hipMemcpyAsync(t.paths + (size_t)sl * nc * Lc, seen.paths + (size_t)sl * oc * Lc,
                                       (size_t)oc * Lc * 2, hipMemcpyDeviceToDevice, stream), "D2D") ||
                !hip_ok(hipMemcpyAsync(t.len + (size_t)sl * nc, seen.len + (size_t)sl * oc, (size_t)oc * 2,
                                       hipMemcpyDeviceToDevice, stream), "D2D") ||
                !hip_ok(hipMemcpyAsync(t.hash + (size_t)sl * nc, seen.hash + (size_t)sl * oc, (size_t)oc * 8,
                                       hipMemcpyDeviceToDevice, stream), "D2D"))
                return false;
        }
        if (!hip_ok(hipMemcpyAsync(t.n, seen.n, (size_t)seen_slots * 4, hipMemcpyDeviceToDevice, stream), "D2D") ||
            !sync())
            return false;
        release(seen.paths); release(seen.len); release(seen.hash); release(seen.n);
    } else if (!hip_ok(hipMemsetAsync(t.n, 0, (size_t)ns * 4, stream), "memset")) {
        return false;
    }
    seen = t;
    seen_slots = ns;
    return true;
}

// the same 64-bit order-free hash as path_hash (bnb_kernels.hip)
static uint64_t mix64h(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

bool sgufp_ctx::seen_upload(int slot, const std::vector<std::vector<int16_t>> &paths) {
    const int cnt = (int)paths.size();
    if (cnt > seen.cap) return false;
    std::vector<int16_t> flat((size_t)cnt * seen.Lcap, 0);
    std::vector<uint16_t> len(cnt);
    std::vector<uint64_t> h(cnt);
    for (int i = 0; i < cnt; i++) {
        const auto &p = paths[i];
        len[i] = (uint16_t)p.size();
        uint64_t x = 0;
        for (size_t t = 0; t < p.size(); t++) {
            flat[(size_t)i * seen.Lcap + t] = p[t];
            x += mix64h(((uint64_t)(uint32_t)t << 16) ^ (uint64_t)(uint16_t)p[t] ^ 0x9E3779B97F4A7C15ull);
        }
        h[i] = x + mix64h((uint64_t)p.size() + 1);
    }
    const size_t e = (size_t)slot * seen.cap;
    const int32_t n32 = cnt;
    return upload(seen.paths + e * seen.Lcap, flat.data(), flat.size()) && upload(seen.len + e, len.data(), len.size()) &&
           upload(seen.hash + e, h.data(), h.size()) && upload(seen.n + slot, &n32, 1) && sync();
}

bool sgufp_ctx::seen_download(int slot, int count, std::vector<std::vector<int16_t>> &paths) {
    const size_t e = (size_t)slot * seen.cap;
    std::vector<int16_t> flat((size_t)count * seen.Lcap);
    std::vector<uint16_t> len(count);
    if (!download(flat.data(), seen.paths + e * seen.Lcap, flat.size()) || !download(len.data(), seen.len + e, len.size()) ||
        !sync())
        return false;
    paths.resize(count);
    for (int i = 0; i < count; i++)
        paths[i].assign(flat.begin() + (size_t)i * seen.Lcap, flat.begin() + (size_t)i * seen.Lcap + len[i]);
    return true;
}

static double seconds_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

extern "C" {

int sgufp_bnb_set_trace(sgufp_ctx *ctx, int enabled) {
    if (!ctx) return SGUFP_ERR_ARG;
    ctx->trace = enabled != 0;
    for (auto &t : ctx->trace_items) t.clear();
    return SGUFP_OK;
}

int sgufp_bnb_trace(sgufp_ctx *ctx, int kind, int64_t *count, int64_t *path_entries, int32_t *record, int32_t *code,
                    int32_t *row, double *value, int64_t *path_off, int16_t *paths) {
    if (!ctx || kind < 0 || kind > 3) return SGUFP_ERR_ARG;
    const auto &items = ctx->trace_items[kind];
    int64_t pe = 0;
    for (size_t i = 0; i < items.size(); i++) {
        if (record) record[i] = items[i].record;
        if (code) code[i] = items[i].code;
        if (row) row[i] = items[i].row;
        if (value) value[i] = items[i].value;
        if (path_off) path_off[i] = pe;
        if (paths && !items[i].path.empty())
            std::memcpy(paths + pe, items[i].path.data(), items[i].path.size() * sizeof(int16_t));
        pe += (int64_t)items[i].path.size();
    }
    if (path_off) path_off[items.size()] = pe;
    if (count) *count = (int64_t)items.size();
    if (path_entries) *path_entries = pe;
    return SGUFP_OK;
}

int sgufp_bnb_set_limits(sgufp_ctx *ctx, int max_refine_iters, double round_seconds) {
    if (!ctx || max_refine_iters < 0 || !(round_seconds >= 0.0)) return SGUFP_ERR_ARG;
    ctx->bnb_max_iters = max_refine_iters;
    ctx->bnb_seconds = round_seconds;
    return SGUFP_OK;
}

void sgufp_ctx::make_record_key(uint16_t gl, uint32_t mask, const int16_t *sol, size_t len, std::string &key) {
    key.resize(6 + 2 * len);
    std::memcpy(&key[0], &gl, 2);
    std::memcpy(&key[2], &mask, 4);
    if (len) std::memcpy(&key[6], sol, 2 * len);
}

bool sgufp_ctx::slice_keys(int64_t lo, int count, std::vector<std::string> &keys) {
    keys.assign((size_t)count, std::string());
    if (count <= 0) return true;
    std::vector<uint16_t> gl(count), len(count);
    std::vector<uint32_t> mask(count);
    std::vector<int64_t> so(count);
    if (!download(gl.data(), fr.gl + lo, count) || !download(mask.data(), fr.mask + lo, count) ||
        !download(len.data(), fr.sol_len + lo, count) || !download(so.data(), fr.sol_off + lo, count) || !sync())
        return false;
    // solution offsets grow with the entry index: one span covers the slice
    int64_t s_lo = so[0], s_hi = so[0];
    for (int k = 0; k < count; k++) {
        s_lo = std::min(s_lo, so[k]);
        s_hi = std::max(s_hi, so[k] + (int64_t)len[k]);
    }
    std::vector<int16_t> arena((size_t)(s_hi - s_lo));
    if (!arena.empty() && (!download(arena.data(), fr.sol + s_lo, arena.size()) || !sync())) return false;
    for (int k = 0; k < count; k++)
        make_record_key(gl[k], mask[k], arena.data() + (so[k] - s_lo), len[k], keys[k]);
    return true;
}

int sgufp_frontier_clear(sgufp_ctx *ctx) {
    if (!ctx) return SGUFP_ERR_ARG;
    ctx->fr_n = 0;
    ctx->fr_sol_top = 0;
    ctx->deferred_seen.clear();
    if (ctx->seen.paths) {   // a new search starts with small seen-path lists again
        if (!ctx->sync()) return SGUFP_ERR_HIP;
        ctx->release(ctx->seen.paths);
        ctx->release(ctx->seen.len);
        ctx->release(ctx->seen.hash);
        ctx->release(ctx->seen.n);
        ctx->seen = SeenLists{};
        ctx->seen_slots = 0;
    }
    return SGUFP_OK;
}

int sgufp_frontier_size(const sgufp_ctx *ctx, int64_t *n, int64_t *sol_entries) {
    if (!ctx) return SGUFP_ERR_ARG;
    if (n) *n = ctx->fr_n;
    if (sol_entries) *sol_entries = ctx->fr_sol_top;
    return SGUFP_OK;
}

int sgufp_frontier_push(sgufp_ctx *ctx, int n, const uint16_t *gl, const double *lb, const double *ub,
                        const int64_t *states_off, const int16_t *states, const int64_t *sol_off, const int16_t *sol) {
    if (!ctx || n < 0 || (n && (!gl || !lb || !ub || !states_off || !sol_off))) return SGUFP_ERR_ARG;
    if (n == 0) return SGUFP_OK;
    EncodedRecords e;
    ctx->encode_records(n, gl, states_off, states, sol_off, sol, e);
    const int64_t base = ctx->fr_n;
    const int64_t sbase = ctx->fr_sol_top;
    if (!ctx->frontier_reserve(base + n, (size_t)sbase + e.sols.size())) return SGUFP_ERR_HIP;
    for (auto &o : e.soff) o += sbase;
    FrontierDev &f = ctx->fr;
    if (!ctx->upload(f.gl + base, gl, n) || !ctx->upload(f.lb + base, lb, n) || !ctx->upload(f.ub + base, ub, n) ||
        !ctx->upload(f.mask + base, e.mask.data(), n) || !ctx->upload(f.valid + base, e.valid.data(), n) ||
        !ctx->upload(f.sol_off + base, e.soff.data(), n) || !ctx->upload(f.sol_len + base, e.slen.data(), n) ||
        !ctx->upload(f.sol + sbase, e.sols.data(), e.sols.size()) || !ctx->sync())
        return SGUFP_ERR_HIP;
    ctx->fr_n += n;
    ctx->fr_sol_top += (int64_t)e.sols.size();
    return SGUFP_OK;
}

// host copies of the frontier entries [lo, lo + n): records (states decoded, solutions
// re-based to 0) and, when keys is given, their deferred-loop keys
static int read_records(sgufp_ctx *ctx, int64_t lo, int n, uint16_t *gl, double *lb, double *ub, int64_t *states_off,
                        int16_t *states, int64_t *sol_off, int16_t *sol, std::vector<std::string> *keys) {
    FrontierDev &f = ctx->fr;
    std::vector<uint16_t> g(n), len(n);
    std::vector<double> l(n), u(n);
    std::vector<uint32_t> mask(n);
    std::vector<int64_t> so(n + 1);
    if (!ctx->download(g.data(), f.gl + lo, n) || !ctx->download(l.data(), f.lb + lo, n) ||
        !ctx->download(u.data(), f.ub + lo, n) || !ctx->download(mask.data(), f.mask + lo, n) ||
        !ctx->download(len.data(), f.sol_len + lo, n) || !ctx->download(so.data(), f.sol_off + lo, n) || !ctx->sync())
        return SGUFP_ERR_HIP;
    // arena span of the records (offsets increase with the entry index)
    int64_t s_hi = ctx->fr_sol_top;
    if (lo + n < ctx->fr_n && (!ctx->download(&s_hi, f.sol_off + lo + n, 1) || !ctx->sync())) return SGUFP_ERR_HIP;
    const int64_t s_lo = so[0];
    std::vector<int16_t> arena((size_t)(s_hi - s_lo));
    if (!ctx->download(arena.data(), f.sol + s_lo, arena.size()) || !ctx->sync()) return SGUFP_ERR_HIP;
    if (gl) std::copy(g.begin(), g.end(), gl);
    if (lb) std::copy(l.begin(), l.end(), lb);
    if (ub) std::copy(u.begin(), u.end(), ub);
    ctx->decode_states(g.data(), mask.data(), (size_t)n, states_off, states);
    int64_t o = 0;
    for (int k = 0; k < n; k++) {
        if (sol_off) sol_off[k] = o;
        if (sol) std::memcpy(sol + o, arena.data() + (so[k] - s_lo), len[k] * sizeof(int16_t));
        o += len[k];
    }
    if (sol_off) sol_off[n] = o;
    if (keys) {
        keys->assign((size_t)n, std::string());
        for (int k = 0; k < n; k++)
            sgufp_ctx::make_record_key(g[k], mask[k], arena.data() + (so[k] - s_lo), len[k], (*keys)[k]);
    }
    return SGUFP_OK;
}

static int records_size(sgufp_ctx *ctx, int64_t lo, int n, int64_t *n_states, int64_t *n_sol) {
    std::vector<uint32_t> mask(n);
    std::vector<uint16_t> len(n);
    if (!ctx->download(mask.data(), ctx->fr.mask + lo, n) || !ctx->download(len.data(), ctx->fr.sol_len + lo, n) ||
        !ctx->sync())
        return SGUFP_ERR_HIP;
    int64_t ns = 0, nl = 0;
    for (int k = 0; k < n; k++) {
        ns += __builtin_popcount(mask[k]);
        nl += len[k];
    }
    if (n_states) *n_states = ns;
    if (n_sol) *n_sol = nl;
    return SGUFP_OK;
}

int sgufp_frontier_take_size(sgufp_ctx *ctx, int n, int from_bottom, int64_t *n_states, int64_t *n_sol) {
    if (!ctx || n < 0 || n > ctx->fr_n) return SGUFP_ERR_ARG;
    return records_size(ctx, from_bottom ? 0 : ctx->fr_n - n, n, n_states, n_sol);
}

int sgufp_frontier_peek_size(sgufp_ctx *ctx, int64_t first, int n, int64_t *n_states, int64_t *n_sol) {
    if (!ctx || n < 0 || first < 0 || first + n > ctx->fr_n) return SGUFP_ERR_ARG;
    return records_size(ctx, first, n, n_states, n_sol);
}

int sgufp_frontier_peek(sgufp_ctx *ctx, int64_t first, int n, uint16_t *gl, double *lb, double *ub,
                        int64_t *states_off, int16_t *states, int64_t *sol_off, int16_t *sol) {
    if (!ctx || n < 0 || first < 0 || first + n > ctx->fr_n) return SGUFP_ERR_ARG;
    if (n == 0) {
        if (states_off) states_off[0] = 0;
        if (sol_off) sol_off[0] = 0;
        return SGUFP_OK;
    }
    return read_records(ctx, first, n, gl, lb, ub, states_off, states, sol_off, sol, nullptr);
}

int sgufp_frontier_take(sgufp_ctx *ctx, int n, int from_bottom, uint16_t *gl, double *lb, double *ub,
                        int64_t *states_off, int16_t *states, int64_t *sol_off, int16_t *sol) {
    if (!ctx || n < 0 || n > ctx->fr_n) return SGUFP_ERR_ARG;
    if (n == 0) {
        if (states_off) states_off[0] = 0;
        if (sol_off) sol_off[0] = 0;
        return SGUFP_OK;
    }
    const int64_t total = ctx->fr_n;
    const int64_t lo = from_bottom ? 0 : total - n;
    std::vector<std::string> keys;
    const int rc = read_records(ctx, lo, n, gl, lb, ub, states_off, states, sol_off, sol,
                                ctx->deferred_seen.empty() ? nullptr : &keys);
    if (rc != SGUFP_OK) return rc;
    // a taken record leaves this context (another shard, or the caller): its deferred loop's
    // seen list goes no further (the receiver restarts the loop; re-solving a path only
    // re-adds a valid cut)
    for (auto &k : keys) ctx->deferred_seen.erase(k);
    if (!from_bottom || n == total) {
        int64_t s_lo = 0;
        if (!ctx->download(&s_lo, ctx->fr.sol_off + lo, 1) || !ctx->sync()) return SGUFP_ERR_HIP;
        ctx->fr_n -= n;
        ctx->fr_sol_top = ctx->fr_n ? s_lo : 0;
        return SGUFP_OK;
    }
    // from the bottom: the remaining entries move down (frontier_drop_bottom, shard.cpp)
    return ctx->frontier_drop_bottom(n) ? SGUFP_OK : SGUFP_ERR_HIP;
}

int sgufp_cuts_rows(sgufp_ctx *ctx, int is_feasibility, int first, int count, double *rhs, double *rows) {
    if (!ctx || first < 0 || count < 0) return SGUFP_ERR_ARG;
    const auto &v = is_feasibility ? ctx->f_rows : ctx->o_rows;
    if (first + count > (int)v.size()) return SGUFP_ERR_ARG;
    if (count == 0) return SGUFP_OK;
    // one gather kernel ({rhs, row} blocks) and one download instead of a copy per row
    const size_t stride = (size_t)ctx->net.n_slots + 1, blk = stride + 1;
    if ((size_t)count * blk > ctx->rowbuf_cap) {
        if (ctx->d_rowbuf) ctx->release(ctx->d_rowbuf);
        ctx->rowbuf_cap = std::max((size_t)count * blk, 2 * ctx->rowbuf_cap);
        if (!ctx->alloc(ctx->d_rowbuf, ctx->rowbuf_cap, "cut rows")) return SGUFP_ERR_HIP;
    }
    if ((size_t)count > ctx->rowids_cap) {
        if (ctx->d_rowids) ctx->release(ctx->d_rowids);
        ctx->rowids_cap = std::max((size_t)count, 2 * ctx->rowids_cap);
        if (!ctx->alloc(ctx->d_rowids, ctx->rowids_cap, "cut rows")) return SGUFP_ERR_HIP;
    }
    std::vector<double> buf((size_t)count * blk);
    if (!ctx->upload(ctx->d_rowids, v.data() + first, (size_t)count) ||
        !ctx->hip_ok(launch_gather_rows(ctx->d_rows, ctx->d_rhs, ctx->d_rowids, count, (int)stride, ctx->d_rowbuf,
                                        ctx->stream), "k_gather_rows") ||
        !ctx->download(buf.data(), ctx->d_rowbuf, buf.size()) || !ctx->sync())
        return SGUFP_ERR_HIP;
    for (int c = 0; c < count; c++) {
        if (rhs) rhs[c] = buf[(size_t)c * blk];
        if (rows) std::memcpy(rows + (size_t)c * stride, &buf[(size_t)c * blk + 1], stride * sizeof(double));
    }
    return SGUFP_OK;
}

int sgufp_bnb_step(sgufp_ctx *ctx, int max_nodes, double *incumbent, sgufp_bnb_stats *stats) {
    if (!ctx || !incumbent) return SGUFP_ERR_ARG;
    sgufp_bnb_stats S{};
    const auto t_round = std::chrono::steady_clock::now();
    const double z = *incumbent;
    const int64_t T = ctx->fr_n;
    if (T == 0) {
        if (stats) *stats = S;
        return SGUFP_OK;
    }
    int b = ctx->max_batch;
    if (max_nodes > 0) b = std::min(b, max_nodes);
    b = (int)std::min<int64_t>(b, T);
    const int64_t base = T - b;
    S.popped = b;

    for (auto &t : ctx->trace_items) t.clear();
    // deferred loops: keys of the popped records (resumed below, or dropped when pruned)
    std::vector<std::string> keys;
    if (!ctx->deferred_seen.empty() && !ctx->slice_keys(base, b, keys)) return SGUFP_ERR_HIP;
    std::vector<double> ub_in;
    if (ctx->trace) {
        ub_in.resize(b);
        if (!ctx->download(ub_in.data(), ctx->fr.ub + base, b) || !ctx->sync()) return SGUFP_ERR_HIP;
    }

    // 1-3: relax the top of the stack in place
    ctx->n = b;
    ctx->cur = ctx->frontier_slice(base, b);
    ctx->restricted_done = false;
    if (!ctx->relax_current(z)) return SGUFP_ERR_HIP;
    std::vector<int32_t> st(b);
    std::vector<double> ub(b), lbv(b, -__DBL_MAX__);
    std::vector<uint32_t> nch(b), need(b), dn(b), da(b), sw(b);
    std::vector<uint64_t> coff(b + 1), soff(b + 1);
    int64_t sol_start = 0;
    BatchOut &o = ctx->out;
    if (!ctx->download(st.data(), o.status, b) || !ctx->download(ub.data(), o.ub, b) ||
        !ctx->download(nch.data(), o.nchild, b) || !ctx->download(need.data(), o.sol_need, b) ||
        !ctx->download(coff.data(), ctx->d_coff, b + 1) || !ctx->download(soff.data(), ctx->d_soff, b + 1) ||
        !ctx->download(dn.data(), o.dd_nodes, b) || !ctx->download(da.data(), o.dd_arcs, b) ||
        !ctx->download(sw.data(), o.sweeps, b) || !ctx->download(&sol_start, ctx->fr.sol_off + base, 1) ||
        !ctx->sync())
        return SGUFP_ERR_HIP;
    if (ctx->timing) hipEventElapsedTime(&ctx->ms_relax, ctx->ev[0], ctx->ev[1]);
    S.ms_relax = ctx->timing ? ctx->ms_relax : 0.0;
    std::vector<int> act, closed;
    for (int k = 0; k < b; k++) {
        switch (st[k]) {
            case SGUFP_PRUNED_BY_BOUND: S.pruned_bound++; continue;
            case SGUFP_PRUNED_BY_FEASIBILITY_CUT: S.pruned_feasibility++; break;
            case SGUFP_PRUNED_BY_OPTIMALITY_CUT: S.pruned_optimality++; break;
            case SGUFP_NEEDS_SUBPROBLEM: act.push_back(k); break;
            case SGUFP_SUCCESS: break;
            default: {
                char msg[128];
                std::snprintf(msg, sizeof msg, "B&B round: frontier record %lld failed with node status %d",
                              (long long)(base + k), st[k]);
                ctx->err = msg;
                return SGUFP_ERR_STATE;
            }
        }
        S.relaxed++;
        S.children += nch[k];
        S.dd_nodes += dn[k];
        S.dd_arcs += da[k];
        S.sweeps += sw[k];
    }
    S.exact = (int64_t)act.size();
    if (ctx->trace) {
        std::vector<uint64_t> ticks(b);
        std::vector<uint32_t> redo(b);
        if (!ctx->download(ticks.data(), o.ticks, b) || !ctx->download(redo.data(), o.redo, b) || !ctx->sync())
            return SGUFP_ERR_HIP;
        const bool stamped = relax_has_phases();
        for (int k = 0; k < b; k++) {
            ctx->trace_items[0].emplace_back();
            auto &t = ctx->trace_items[0].back();
            t.record = k;
            t.code = st[k];
            t.value = ub_in[k];
            ctx->trace_items[3].emplace_back();
            auto &u = ctx->trace_items[3].back();
            u.record = k;
            u.code = (int32_t)(redo[k] & 0xFF);
            u.row = (int32_t)sw[k];
            u.value = stamped ? (double)ticks[k] : 0.0;
        }
    }
    // a popped record that left its deferred loop without re-entering it (pruned by bound
    // or by a cut of the grown pool) drops its seen list
    if (!keys.empty())
        for (int k = 0; k < b; k++)
            if (st[k] != SGUFP_NEEDS_SUBPROBLEM) ctx->deferred_seen.erase(keys[k]);

    // 4: refinement loop of the exact DDs (NodeExplorer.cpp:946-969), device-resident: per
    // iteration k_loop_check (argmax path seen? -> {ub, ub}; else fresh), one synchronisation,
    // then k_seen_append, the scenario subproblem on the fresh paths read in place,
    // k_append_cuts (Container::add on the device) and k_refine, back to back on the stream.
    // The host files the appended rows under the F / O lists at the next synchronisation.
    // The loop of one record is a chain of dependent subproblems (one new cut per iteration);
    // a round stops it after ctx->bnb_max_iters iterations or ctx->bnb_seconds, and the
    // records still in their loop go back on top of the frontier (deferred) with the paths
    // they have seen.  Popped again, such a record rebuilds its DD, applies the pool (its own
    // new cuts included, so its bound is where the loop left it) and resumes the loop with
    // that seen list: it ends exactly where the uninterrupted loop would (a path repeats).
    std::vector<int> deferred;
    std::vector<std::vector<std::vector<int16_t>>> seen_host;   // deferred records' lists
    const int stride = ctx->net.n_slots + 1;
    if (!act.empty()) {
        if (!ctx->loop_reserve(b, 64)) return SGUFP_ERR_HIP;
        std::vector<int32_t> nseen(b, 0);
        if (!ctx->hip_ok(hipMemsetAsync(ctx->seen.n, 0, (size_t)b * 4, ctx->stream), "memset")) return SGUFP_ERR_HIP;
        if (!keys.empty()) {
            for (int k : act) {
                auto it = ctx->deferred_seen.find(keys[k]);
                if (it == ctx->deferred_seen.end()) continue;
                const int cnt = (int)it->second.size();
                if (!ctx->loop_reserve(b, cnt + 1)) return SGUFP_ERR_HIP;
                if (!ctx->seen_upload(k, it->second)) return SGUFP_ERR_HIP;
                nseen[k] = cnt;
                ctx->deferred_seen.erase(it);
                S.resumed++;
            }
        }
        int na = (int)act.size();
        if (!ctx->upload(ctx->d_lact, act.data(), (size_t)na)) return SGUFP_ERR_HIP;
        std::vector<int32_t> flag, chains, ptype;
        std::vector<double> pub;
        std::vector<int> prev;            // fresh records of the previous iteration (rows filed below)
        int prev_first = 0;
        std::vector<double> pobj;         // trace: the previous iteration's sum_s obj_s / S
        std::vector<size_t> prev_trace;   // trace: items of the previous iteration's subproblems
        auto file_rows = [&]() -> bool {  // Container::add: feasibility list, optimality list
            for (size_t i = 0; i < prev.size(); i++) {
                if (ptype[i] < 0) {
                    // the rows of that launch leave the pool again (they were appended and
                    // applied on the device before the host saw the type); the batch's results
                    // are not used past the error
                    ctx->n_rows = prev_first;
                    ctx->err = "scenario subproblem failed (invalid path or numerical failure)";
                    return false;
                }
            }
            ctx->row_ub.resize((size_t)ctx->n_rows);
            for (int want = 1; want >= 0; want--)
                for (size_t i = 0; i < prev.size(); i++) {
                    if (ptype[i] != want) continue;
                    auto &list = want ? ctx->f_rows : ctx->o_rows;
                    if (ctx->trace) {
                        auto &t = ctx->trace_items[1][prev_trace[i]];
                        t.code = want;
                        t.row = (int32_t)list.size();
                        t.value = pobj[i];
                    }
                    list.push_back(prev_first + (int)i);
                    ctx->row_ub[(size_t)prev_first + i] = pub[i];
                    (want ? S.new_feasibility_cuts : S.new_optimality_cuts)++;
                }
            ctx->order_dirty = true;
            prev.clear();
            return true;
        };
        // trace: the argmax path of batch slot k as the loop check saw it
        std::vector<uint16_t> tlen;
        std::vector<int16_t> tpath;
        const size_t Lc = (size_t)ctx->sc.Lcap;
        auto slot_path = [&](int k) {
            return std::vector<int16_t>(tpath.begin() + (long)(k * Lc), tpath.begin() + (long)(k * Lc + tlen[k]));
        };
        while (na > 0) {
            if (!ctx->hip_ok(launch_loop_check(o, ctx->seen, ctx->d_lact, na, ctx->net.m, ctx->d_lflag, ctx->d_lchain,
                                               ctx->stream), "k_loop_check"))
                return SGUFP_ERR_HIP;
            flag.resize(na);
            chains.resize(na);
            ptype.resize(prev.size());
            pub.resize(prev.size());
            pobj.resize(prev.size());
            if (!ctx->download(flag.data(), ctx->d_lflag, (size_t)na) ||
                !ctx->download(chains.data(), ctx->d_lchain, (size_t)na) ||
                !ctx->download(ptype.data(), ctx->sio.cut_type, prev.size()) ||
                !ctx->download(pub.data(), ctx->d_lrowub, prev.size()) ||
                (ctx->trace && !ctx->download(pobj.data(), ctx->sio.obj_mean, prev.size())) || !ctx->sync())   // the one sync
                return SGUFP_ERR_HIP;
            if (!file_rows()) return SGUFP_ERR_STATE;
            if (ctx->trace) {
                tlen.resize((size_t)b);
                tpath.resize((size_t)b * Lc);
                if (!ctx->download(tlen.data(), o.path_len, (size_t)b) || !ctx->download(tpath.data(), o.path, tpath.size()) ||
                    !ctx->sync())
                    return SGUFP_ERR_HIP;
            }
            std::vector<int> fresh;
            int nct = 1;
            for (int a = 0; a < na; a++) {
                const int k = act[a];
                if (flag[a] == 1) {                 // {ub, ub, {}, SUCCESS}
                    closed.push_back(k);
                    S.exact_closed++;
                    if (ctx->trace) {
                        ctx->trace_items[2].emplace_back();
                        ctx->trace_items[2].back().record = k;
                        ctx->trace_items[2].back().path = slot_path(k);
                    }
                } else if (flag[a] == 2) {
                    fresh.push_back(k);
                    nct = std::max(nct, chains[a]);
                } else {
                    st[k] = flag[a] - 3;
                    if (st[k] == SGUFP_PRUNED_BY_FEASIBILITY_CUT) S.pruned_feasibility++;
                    else if (st[k] == SGUFP_PRUNED_BY_OPTIMALITY_CUT) S.pruned_optimality++;
                }
            }
            if (fresh.empty()) break;
            if ((ctx->bnb_max_iters > 0 && S.refine_iters >= ctx->bnb_max_iters) ||
                (ctx->bnb_seconds > 0 && S.refine_iters > 0 && seconds_since(t_round) >= ctx->bnb_seconds)) {
                // (every round runs at least one iteration: a batch whose relaxation alone
                // outlasts round_seconds still makes progress)
                deferred.swap(fresh);    // their current path is unseen: solved when resumed
                break;
            }
            // With a round deadline, one iteration solves at most chunk_lps scenario LPs
            // (a 1024-leaf iteration of the 512-scenario C5 network would take minutes); the
            // other fresh records stay in the loop unchanged (path not yet seen) for the next
            // iteration, or are deferred at the deadline.
            std::vector<int> rest;
            if (ctx->bnb_seconds > 0) {
                const size_t chunk = (size_t)std::max<int64_t>(1, ctx->chunk_lps / std::max(1, ctx->net.S));
                if (fresh.size() > chunk) {
                    rest.assign(fresh.begin() + (long)chunk, fresh.end());
                    fresh.resize(chunk);
                    nct = 1;
                    for (int a = 0; a < na; a++)
                        if (flag[a] == 2 && std::find(fresh.begin(), fresh.end(), act[a]) != fresh.end())
                            nct = std::max(nct, chains[a]);
                }
            }
            S.refine_iters++;
            const int nf = (int)fresh.size();
            int most = 0;
            for (int k : fresh) most = std::max(most, ++nseen[k]);
            if (!ctx->loop_reserve(b, most) || !ctx->upload(ctx->d_lact, fresh.data(), (size_t)nf) ||
                !ctx->hip_ok(launch_seen_append(o, ctx->seen, ctx->d_lact, nf, ctx->net.m, ctx->stream), "k_seen_append") ||
                !ctx->sub_init() || !ctx->sub_grow(nf, 1) || !ctx->grow_rows(ctx->n_rows + nf))
                return SGUFP_ERR_HIP;
            SubIO io = ctx->sio;
            io.n_paths = nf;
            io.nct_cap = nct;
            io.path_slot = ctx->d_lact;
            io.path_len = o.path_len;
            io.path_stride = ctx->sc.Lcap;
            io.paths = o.path;
            io.path_off = nullptr;
            // warm starts: every path starts from the stored state of the closest path solved
            // before (the record's own previous path, a sibling's, ...) and leaves its own state
            // in the ring for the next ones (k_warm_pick, k_sub_scenario<..., WARM>)
            if (ctx->warm_reserve()) {
                if (!ctx->hip_ok(launch_warm_pick(io, ctx->wring, ctx->warm_ptr, ctx->stream), "k_warm_pick"))
                    return SGUFP_ERR_HIP;
                io.warm_src = ctx->wring.src;
                io.warm_dst = ctx->wring.dst;
                io.wst_x = ctx->d_wx;
                io.wst_a = ctx->d_wa;
                io.wst_ok = ctx->d_wok;
                ctx->warm_ptr = (ctx->warm_ptr + nf) % ctx->wring.R;
            }
            if (!ctx->hip_ok(launch_subproblem(ctx->sn, io, ctx->stream), "subproblem launch")) return SGUFP_ERR_HIP;
            ctx->sub_last_n = nf;
            if (ctx->sub_stats) ctx->sub_stats_add(nf);
            const int first = ctx->n_rows;
            if (!ctx->hip_ok(launch_append_cuts(io.cut_type, io.cut_rhs, io.cut_row, nf, stride, first, ctx->d_rows,
                                                ctx->d_rhs, ctx->d_coefT, ctx->nd.slot_tab, ctx->net.L, ctx->ustride,
                                                ctx->d_lrowub, ctx->d_rcuts, ctx->d_rfeas, ctx->stream),
                             "k_append_cuts") ||
                !ctx->hip_ok(launch_refine(ctx->nd, ctx->sc, ctx->batch(), ctx->pool(), o, ctx->d_lact, ctx->d_rcuts,
                                           ctx->d_rfeas, nf, z, ctx->ex, ctx->stream), "k_refine"))
                return SGUFP_ERR_HIP;
            ctx->n_rows += nf;
            S.subproblems += nf;
            prev = fresh;
            prev_first = first;
            if (ctx->trace) {
                prev_trace.clear();
                for (int i = 0; i < nf; i++) {
                    prev_trace.push_back(ctx->trace_items[1].size());
                    ctx->trace_items[1].emplace_back();
                    auto &t = ctx->trace_items[1].back();
                    t.record = fresh[i];
                    t.code = -1;
                    t.path = slot_path(fresh[i]);
                }
            }
            act = fresh;
            act.insert(act.end(), rest.begin(), rest.end());
            na = (int)act.size();
            if (!rest.empty() && !ctx->upload(ctx->d_lact + nf, rest.data(), rest.size())) return SGUFP_ERR_HIP;
        }
        if (!prev.empty()) {
            ptype.resize(prev.size());
            pub.resize(prev.size());
            pobj.resize(prev.size());
            if (!ctx->download(ptype.data(), ctx->sio.cut_type, prev.size()) ||
                !ctx->download(pub.data(), ctx->d_lrowub, prev.size()) ||
                (ctx->trace && !ctx->download(pobj.data(), ctx->sio.obj_mean, prev.size())) || !ctx->sync())
                return SGUFP_ERR_HIP;
            if (!file_rows()) return SGUFP_ERR_STATE;
        }
        // bounds after the loop: closed records' lb (the incumbent candidates) and the
        // deferred records' bound
        if (!ctx->download(ub.data(), o.ub, b) || !ctx->sync()) return SGUFP_ERR_HIP;
        for (int k : closed) lbv[k] = ub[k];
        for (auto &t : ctx->trace_items[2]) t.value = ub[t.record];
        for (int k : deferred) {
            seen_host.emplace_back();
            if (!ctx->seen_download(k, nseen[k], seen_host.back())) return SGUFP_ERR_HIP;
        }
    }

    // deferred records: saved before the children overwrite the popped slice
    const int nd = (int)deferred.size();
    std::vector<uint16_t> d_gl(nd), d_len(nd);
    std::vector<double> d_lb(nd), d_ub(nd);
    std::vector<uint32_t> d_mask(nd);
    std::vector<uint8_t> d_valid(nd);
    std::vector<int64_t> d_soff(nd);
    std::vector<std::vector<int16_t>> d_sol(nd);
    {
        FrontierDev &f = ctx->fr;
        for (int i = 0; i < nd; i++) {
            const int64_t e = base + deferred[i];
            if (!ctx->download(&d_gl[i], f.gl + e, 1) || !ctx->download(&d_lb[i], f.lb + e, 1) ||
                !ctx->download(&d_mask[i], f.mask + e, 1) || !ctx->download(&d_valid[i], f.valid + e, 1) ||
                !ctx->download(&d_len[i], f.sol_len + e, 1) || !ctx->download(&d_soff[i], f.sol_off + e, 1))
                return SGUFP_ERR_HIP;
            d_ub[i] = ub[deferred[i]];   // the bound the loop reached (every pool cut is valid)
        }
        if (nd && !ctx->sync()) return SGUFP_ERR_HIP;
        for (int i = 0; i < nd; i++) {
            d_sol[i].resize(d_len[i]);
            if (!ctx->download(d_sol[i].data(), f.sol + d_soff[i], d_len[i])) return SGUFP_ERR_HIP;
        }
        if (nd && !ctx->sync()) return SGUFP_ERR_HIP;
        for (int i = 0; i < nd; i++) {
            std::string key;
            sgufp_ctx::make_record_key(d_gl[i], d_mask[i], d_sol[i].data(), d_len[i], key);
            ctx->deferred_seen[key] = std::move(seen_host[i]);
        }
    }
    S.deferred = nd;

    // 5: incumbent (DDSolver.cpp:723-731)
    double znew = z;
    for (int k = 0; k < b; k++)
        if (lbv[k] > znew) znew = lbv[k];
    S.improved = znew > z ? 1 : 0;
    *incumbent = znew;

    // 6: push the children of parents with ub > zOpt (DDSolver.cpp:744-748)
    std::vector<int32_t> par;
    std::vector<int64_t> dchild, dsol;
    int64_t nc = 0, ns = 0;
    for (int k = 0; k < b; k++) {
        if (st[k] != SGUFP_SUCCESS || nch[k] == 0 || !(ub[k] > znew)) continue;
        par.push_back(k);
        dchild.push_back(base + nc);
        dsol.push_back(sol_start + ns);
        nc += nch[k];
        ns += need[k];
    }
    ctx->relaxed = false;   // the popped slice is overwritten below
    ctx->dd_built = false;
    if (!ctx->frontier_reserve(base + nc, (size_t)(sol_start + ns))) return SGUFP_ERR_HIP;
    const int np = (int)par.size();
    if (np) {
        int32_t *d_par = nullptr;
        int64_t *d_dc = nullptr, *d_ds = nullptr;
        if (np > ctx->max_batch) return SGUFP_ERR_STATE;
        d_par = ctx->d_bidx;
        d_dc = ctx->d_boff;
        d_ds = ctx->d_bsol;
        if (!ctx->upload(d_par, par.data(), np) || !ctx->upload(d_dc, dchild.data(), np) ||
            !ctx->upload(d_ds, dsol.data(), np) ||
            !ctx->hip_ok(launch_push_children(ctx->children_view(), o, d_par, d_dc, d_ds, np, ctx->fr, ctx->stream),
                         "k_push_children") ||
            !ctx->sync())
            return SGUFP_ERR_HIP;
    }
    ctx->fr_n = base + nc;
    ctx->fr_sol_top = ctx->fr_n ? sol_start + ns : 0;
    if (nd) {
        // the deferred records on top, in their frontier order: popped first next round
        int64_t stot = 0;
        for (int i = 0; i < nd; i++) stot += d_len[i];
        const int64_t e0 = ctx->fr_n, s0 = ctx->fr_sol_top;
        if (!ctx->frontier_reserve(e0 + nd, (size_t)(s0 + stot))) return SGUFP_ERR_HIP;
        std::vector<int64_t> so(nd);
        std::vector<int16_t> flat;
        flat.reserve((size_t)stot);
        for (int i = 0; i < nd; i++) {
            so[i] = s0 + (int64_t)flat.size();
            flat.insert(flat.end(), d_sol[i].begin(), d_sol[i].end());
        }
        FrontierDev &f = ctx->fr;
        if (!ctx->upload(f.gl + e0, d_gl.data(), nd) || !ctx->upload(f.lb + e0, d_lb.data(), nd) ||
            !ctx->upload(f.ub + e0, d_ub.data(), nd) || !ctx->upload(f.mask + e0, d_mask.data(), nd) ||
            !ctx->upload(f.valid + e0, d_valid.data(), nd) || !ctx->upload(f.sol_len + e0, d_len.data(), nd) ||
            !ctx->upload(f.sol_off + e0, so.data(), nd) || !ctx->upload(f.sol + s0, flat.data(), flat.size()) ||
            !ctx->sync())
            return SGUFP_ERR_HIP;
        ctx->fr_n = e0 + nd;
        ctx->fr_sol_top = s0 + stot;
    }
    S.pushed = nc;
    S.frontier = ctx->fr_n;
    if (stats) *stats = S;
    return SGUFP_OK;
}

}  // extern "C"
