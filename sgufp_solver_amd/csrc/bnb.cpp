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

static double seconds_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

extern "C" {

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

bool sgufp_ctx::record_key(int64_t e, std::string &key) {
    uint16_t gl = 0, len = 0;
    uint32_t mask = 0;
    int64_t so = 0;
    if (!download(&gl, fr.gl + e, 1) || !download(&mask, fr.mask + e, 1) || !download(&len, fr.sol_len + e, 1) ||
        !download(&so, fr.sol_off + e, 1) || !sync())
        return false;
    std::vector<int16_t> sol(len);
    if (len && (!download(sol.data(), fr.sol + so, len) || !sync())) return false;
    make_record_key(gl, mask, sol.data(), len, key);
    return true;
}

int sgufp_frontier_clear(sgufp_ctx *ctx) {
    if (!ctx) return SGUFP_ERR_ARG;
    ctx->fr_n = 0;
    ctx->fr_sol_top = 0;
    ctx->deferred_seen.clear();
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

int sgufp_frontier_take_size(sgufp_ctx *ctx, int n, int from_bottom, int64_t *n_states, int64_t *n_sol) {
    if (!ctx || n < 0 || n > ctx->fr_n) return SGUFP_ERR_ARG;
    const int64_t lo = from_bottom ? 0 : ctx->fr_n - n;
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

int sgufp_frontier_take(sgufp_ctx *ctx, int n, int from_bottom, uint16_t *gl, double *lb, double *ub,
                        int64_t *states_off, int16_t *states, int64_t *sol_off, int16_t *sol) {
    if (!ctx || n < 0 || n > ctx->fr_n) return SGUFP_ERR_ARG;
    if (n == 0) {
        if (states_off) states_off[0] = 0;
        if (sol_off) sol_off[0] = 0;
        return SGUFP_OK;
    }
    FrontierDev &f = ctx->fr;
    const int64_t total = ctx->fr_n;
    const int64_t lo = from_bottom ? 0 : total - n;
    std::vector<uint16_t> g(n), len(n);
    std::vector<double> l(n), u(n);
    std::vector<uint32_t> mask(n);
    std::vector<int64_t> so(n + 1);
    if (!ctx->download(g.data(), f.gl + lo, n) || !ctx->download(l.data(), f.lb + lo, n) ||
        !ctx->download(u.data(), f.ub + lo, n) || !ctx->download(mask.data(), f.mask + lo, n) ||
        !ctx->download(len.data(), f.sol_len + lo, n) || !ctx->download(so.data(), f.sol_off + lo, n) || !ctx->sync())
        return SGUFP_ERR_HIP;
    // arena span of the taken records (offsets increase with the entry index)
    int64_t s_hi = ctx->fr_sol_top;
    if (from_bottom && n < total) {
        if (!ctx->download(&s_hi, f.sol_off + n, 1) || !ctx->sync()) return SGUFP_ERR_HIP;
    }
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
    if (!from_bottom || n == total) {
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
    std::vector<int> act;
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

    // 4: refinement loop of the exact DDs (NodeExplorer.cpp:946-969).  The loop of one record
    // is a chain of dependent subproblems (one new cut per iteration); a round stops it after
    // ctx->bnb_max_iters iterations or ctx->bnb_seconds, and the records still in their loop
    // go back on top of the frontier (deferred) with the paths they have seen.  Popped again,
    // such a record rebuilds its DD, applies the pool (its own new cuts included, so its bound
    // is where the loop left it) and resumes the loop with that seen list: the loop ends
    // exactly where the uninterrupted one would (a path repeats), whatever happened between.
    std::vector<std::vector<std::vector<int16_t>>> seen(b);
    std::vector<uint16_t> plen(b);
    const size_t stride = (size_t)ctx->net.n_slots + 1;
    std::vector<int> deferred;
    if (!act.empty() && !ctx->deferred_seen.empty()) {
        for (int k : act) {
            std::string key;
            if (!ctx->record_key(base + k, key)) return SGUFP_ERR_HIP;
            auto it = ctx->deferred_seen.find(key);
            if (it != ctx->deferred_seen.end()) {
                seen[k] = std::move(it->second);
                ctx->deferred_seen.erase(it);
                S.resumed++;
            }
        }
    }
    while (!act.empty()) {
        if (!ctx->download(plen.data(), o.path_len, b) || !ctx->sync()) return SGUFP_ERR_HIP;
        const int na = (int)act.size();
        std::vector<int64_t> off(na + 1, 0);
        for (int a = 0; a < na; a++) off[a + 1] = off[a] + plen[act[a]];
        std::vector<int16_t> packed((size_t)off[na]);
        if (!ctx->upload(ctx->d_bidx, act.data(), na) || !ctx->upload(ctx->d_boff, off.data(), na + 1) ||
            !ctx->hip_ok(launch_gather_paths(o, ctx->sc.Lcap, ctx->d_bidx, ctx->d_boff, na, ctx->d_bpaths, ctx->stream),
                         "k_gather_paths") ||
            !ctx->download(packed.data(), ctx->d_bpaths, packed.size()) || !ctx->sync())
            return SGUFP_ERR_HIP;
        std::vector<int> fresh;
        std::vector<int64_t> poff{0};
        std::vector<int16_t> paths;
        for (int a = 0; a < na; a++) {
            const int k = act[a];
            std::vector<int16_t> p(packed.begin() + off[a], packed.begin() + off[a + 1]);
            auto &sv = seen[k];
            if (std::find(sv.begin(), sv.end(), p) != sv.end()) {   // {ub, ub, {}, SUCCESS}
                lbv[k] = ub[k];
                S.exact_closed++;
                continue;
            }
            paths.insert(paths.end(), p.begin(), p.end());
            poff.push_back((int64_t)paths.size());
            fresh.push_back(k);
        }
        act.clear();
        if (fresh.empty()) break;
        if ((ctx->bnb_max_iters > 0 && S.refine_iters >= ctx->bnb_max_iters) ||
            (ctx->bnb_seconds > 0 && seconds_since(t_round) >= ctx->bnb_seconds)) {
            deferred.swap(fresh);    // their current path is unseen: solved when resumed
            break;
        }
        S.refine_iters++;
        for (size_t i = 0; i < fresh.size(); i++)
            seen[fresh[i]].emplace_back(paths.begin() + poff[i], paths.begin() + poff[i + 1]);
        const int nf = (int)fresh.size();
        std::vector<int32_t> type(nf);
        std::vector<double> rhs(nf), rows((size_t)nf * stride);
        int rc = sgufp_subproblem(ctx, nf, poff.data(), paths.data(), type.data(), rhs.data(), rows.data(), nullptr);
        if (rc != SGUFP_OK) return rc;
        S.subproblems += nf;
        // Container::add in node order, feasibility list then optimality list
        std::vector<int32_t> idx(nf), cut(nf);
        std::vector<uint8_t> isf(nf);
        for (int want = 1; want >= 0; want--) {
            std::vector<double> r, h;
            int cnt = 0, first = sgufp_cuts_count(ctx, want);
            for (int i = 0; i < nf; i++) {
                if (type[i] < 0) {
                    ctx->err = "scenario subproblem failed (invalid path or numerical failure)";
                    return SGUFP_ERR_STATE;
                }
                if (type[i] != want) continue;
                r.insert(r.end(), rows.begin() + (size_t)i * stride, rows.begin() + (size_t)(i + 1) * stride);
                h.push_back(rhs[i]);
                idx[i] = fresh[i];
                isf[i] = (uint8_t)want;
                cut[i] = first + cnt++;
            }
            if (cnt && (rc = sgufp_cuts_append_rows(ctx, want, cnt, h.data(), r.data())) != SGUFP_OK) return rc;
            (want ? S.new_feasibility_cuts : S.new_optimality_cuts) += cnt;
        }
        if ((rc = sgufp_batch_refine(ctx, nf, idx.data(), isf.data(), cut.data(), z)) != SGUFP_OK) return rc;
        std::vector<int32_t> st2(b);
        if (!ctx->download(st2.data(), o.status, b) || !ctx->download(ub.data(), o.ub, b) || !ctx->sync())
            return SGUFP_ERR_HIP;
        for (int k : fresh) {
            if (st2[k] == SGUFP_NEEDS_SUBPROBLEM) act.push_back(k);
            else if (st2[k] == SGUFP_PRUNED_BY_FEASIBILITY_CUT) S.pruned_feasibility++;
            else if (st2[k] == SGUFP_PRUNED_BY_OPTIMALITY_CUT) S.pruned_optimality++;
            st[k] = st2[k];
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
            ctx->deferred_seen[key] = std::move(seen[deferred[i]]);
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
