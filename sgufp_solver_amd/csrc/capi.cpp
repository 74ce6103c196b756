// C ABI of libsgufp_hip.so (declared in include/sgufp_hip.h): context, device
// memory, cut-pool densification, batch staging and result retrieval.
#include <cstdio>

#include "ctx.hpp"
#include <algorithm>
#include <cstdlib>


namespace {

// Upper bound on DD nodes: every layer outside the last five has < 120 nodes or is a
// single merged node (collapse rule, DD.cpp:3614); the last five expand exactly, and a
// node with c states (-1 included) has one child with c states and c-1 with c-1.
int64_t node_bound(const Network &net, int64_t *tail = nullptr) {
    const int L = net.L;
    auto set_size = [&](int sid) { return sid >= 0 ? (int)net.sets[sid].size() : 1; };
    int start = std::max(0, L - 5);
    std::vector<int64_t> h(kMaxStates + 2, 0);
    int c0 = set_size(net.layer_universe[start]);
    h[c0] = (L > 5) ? kRelaxedMaxWidth - 1 : 1;
    int64_t total = (int64_t)(kRelaxedMaxWidth - 1) * (start + 1);
    int64_t tail_nodes = 0;
    for (int l = start; l < L; l++) {
        if (net.layer_update[l] >= 0) {
            int64_t w = 0;
            for (auto x : h) w += x;
            std::fill(h.begin(), h.end(), 0);
            h[set_size(net.layer_update[l])] = w;
        }
        std::vector<int64_t> nh(h.size(), 0);
        for (int c = 1; c < (int)h.size(); c++) {
            if (!h[c]) continue;
            nh[c] += h[c];
            if (c > 1) nh[c - 1] += h[c] * (c - 1);
        }
        h.swap(nh);
        int64_t w = 0;
        for (auto x : h) w += x;
        total += w;
        tail_nodes += w;
    }
    if (tail) *tail = std::max<int64_t>(tail_nodes, 128) + 8;
    return total + 8;
}

}  // namespace

bool sgufp_ctx::init() {
    if (!hip_ok(hipSetDevice(device), "hipSetDevice")) return false;
    if (!hip_ok(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "hipStreamCreate")) return false;
    for (auto &e : ev)
        if (!hip_ok(hipEventCreate(&e), "hipEventCreate")) return false;
    const int L = net.L;

    // network tables
    std::vector<int32_t> set_off, set_len;
    std::vector<int16_t> set_val;
    for (auto &s : net.sets) {
        set_off.push_back((int32_t)set_val.size());
        set_len.push_back((int32_t)s.size());
        set_val.insert(set_val.end(), s.begin(), s.end());
    }
    int32_t *p_upd, *p_univ, *p_soff, *p_slen, *p_tab, *p_slotoff, *p_slothead, *p_head;
    int16_t *p_sval;
    uint8_t *p_changed;
    if (!alloc(p_upd, L + 1, "net") || !alloc(p_univ, L + 1, "net") || !alloc(p_changed, L + 1, "net") ||
        !alloc(p_soff, set_off.size(), "net") || !alloc(p_slen, set_len.size(), "net") ||
        !alloc(p_sval, set_val.size(), "net") || !alloc(p_tab, net.slot_tab.size(), "net") ||
        !alloc(p_slotoff, net.slot_off.size(), "net") || !alloc(p_slothead, net.slot_head.size(), "net") ||
        !alloc(p_head, net.head.size(), "net"))
        return false;
    std::vector<uint8_t> changed(net.state_changed.begin(), net.state_changed.end());
    changed.resize(L + 1, 0);
    upload(p_upd, net.layer_update.data(), L + 1);
    upload(p_univ, net.layer_universe.data(), L + 1);
    upload(p_changed, changed.data(), L + 1);
    upload(p_soff, set_off.data(), set_off.size());
    upload(p_slen, set_len.data(), set_len.size());
    upload(p_sval, set_val.data(), set_val.size());
    upload(p_tab, net.slot_tab.data(), net.slot_tab.size());
    upload(p_slotoff, net.slot_off.data(), net.slot_off.size());
    upload(p_slothead, net.slot_head.data(), net.slot_head.size());
    upload(p_head, net.head.data(), net.head.size());
    nd.L = L;
    nd.L5 = (unsigned)(L - 5);
    nd.m = net.m;
    nd.n_slots = net.n_slots;
    nd.layer_update = p_upd; nd.layer_universe = p_univ; nd.changed = p_changed;
    nd.set_off = p_soff; nd.set_len = p_slen; nd.set_val = p_sval;
    nd.slot_tab = p_tab; nd.slot_off = p_slotoff; nd.slot_head = p_slothead; nd.arc_head = p_head;

    for (int s = 0; s < net.n_slots; s++) key_slots[net.slot_key(s) & 0xFFFFFFFFFFFFull].push_back(s);

    // per-slot scratch
    const int maxU = std::max(1, net.max_states);
    sc.Tcap = L + 2;
    sc.Lcap = L + 1;
    int64_t tail = 0;
    int64_t ncap = node_bound(net, &tail);
    ustride = std::max(1, net.max_states);
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
            cus = prop.multiProcessorCount;
    }
    // Cuts per batched sweep: 4 (k_relax runs 2 waves per SIMD, 20 KB of LDS each).  A context
    // whose batches fill at most half of those wave slots (the B&B rounds: 1 024 records on 2 048
    // slots) sweeps 8 cuts at a time (28 KB, 5 waves per CU, still one wave per record): the
    // non-exact survivors of a seeded C3 search that sweep a pool of 39k / 75k cuts take 791 ->
    // 545 / 2 462 -> 2 081 ms per round (tools/gpu_r04v.sh).  SGUFP_CUT_BATCH forces a size.
    const char *ecb = getenv("SGUFP_CUT_BATCH");
    if (ecb) cb = atoi(ecb);
    else if (2 * (int64_t)max_batch <= 8 * (int64_t)cus) cb = 8;
    if (cb != 1 && cb != 4 && cb != 8 && cb != 16) cb = 4;
    nscreen = cb;
    if (const char *e = getenv("SGUFP_SCREEN")) nscreen = std::max(0, atoi(e));
    if (const char *e = getenv("SGUFP_EXACT_FAST")) exact_fast = atoi(e) != 0;
    if (const char *e = getenv("SGUFP_SUB_WARM")) warm_on = atoi(e) != 0;   // warm-started subproblems (A/B)
    if (const char *e = getenv("SGUFP_EXACT_SCREEN")) exact_screen = std::max(0, std::min(kExactScreen, atoi(e)));
    if (const char *e = getenv("SGUFP_EXACT_LAZY")) exact_lazy = std::max(0, atoi(e));
    if (const char *e = getenv("SGUFP_CHUNK_LPS")) chunk_lps = std::max(1, atoi(e));
    if (const char *e = getenv("SGUFP_NX")) nx_on = atoi(e) != 0;
    if (const char *e = getenv("SGUFP_SUB_STATS")) sub_stats = atoi(e) != 0;
    if (const char *e = getenv("SGUFP_LEAF_SPLIT")) leaf_split = std::max(0, atoi(e));
    if (const char *e = getenv("SGUFP_NX_MIN")) nx_min = std::max(1, atoi(e));
    if (const char *e = getenv("SGUFP_NX_SKIP")) nx_skip = std::max(0, atoi(e));
    int64_t acap = std::max<int64_t>(1, (int64_t)std::max(0, L - 4) * (kRelaxedMaxWidth - 1) * maxU);
    if (ncap > (int64_t)kParentMask || acap > (int64_t)0x7FFFFFFF) { err = "DD capacity beyond 22-bit indices"; return false; }
    sc.Ncap = (int)ncap;
    sc.Acap = (int)acap;
    // LDS per relax workgroup (one wave): layer table, value buffers and staging rings
    sc.us = ustride;
    if (net.n_slots >= 32767) { err = "more than 32766 coefficient slots (int16 root-solution slots)"; return false; }
    if (relax_lds_bytes(sc.Tcap, sc.Lcap, cb, sc.us) > 160 * 1024) { err = "too many layers for the LDS layer table"; return false; }
    sc.tmir_cap = cb > 1 ? (int)(sc.Ncap + sc.Acap) : 0;
    sc.tail_cap = (int)tail;
    sc.cb_max = cb;
    const size_t B = (size_t)max_batch;
    if (!alloc(sc.ntopo, B * sc.Ncap, "scratch") || !alloc(sc.nflag, B * sc.Ncap, "scratch") ||
        !alloc(sc.nmask, B * sc.Ncap, "scratch") || !alloc(sc.outcnt, B * sc.Ncap, "scratch") ||
        !alloc(sc.s2, B * sc.Ncap, "scratch") || !alloc(sc.tw, B * sc.Ncap, "scratch") ||
        !alloc(sc.atopo, B * sc.Acap, "scratch") || !alloc(sc.aflag, B * sc.Acap, "scratch") ||
        !alloc(sc.lay, B * sc.Tcap * 5, "scratch") || !alloc(sc.rslot, B * sc.Lcap, "scratch") ||
        !alloc(sc.meta, B * 8, "scratch") || !alloc(sc.ubv, B, "scratch") ||
        !alloc(sc.sm1, B * sc.Tcap, "scratch") || !alloc(sc.xm1, B * sc.Tcap, "scratch") ||
        !alloc(sc.v1, B * sc.Tcap, "scratch"))
        return false;
    if (cb > 1 && (!alloc(sc.s2b, B * sc.tail_cap * cb, "scratch") || !alloc(sc.sm, B * sc.Tcap * cb, "scratch") ||
                   !alloc(sc.xm, B * sc.Tcap * cb, "scratch") || !alloc(sc.tmir, B * (size_t)sc.tmir_cap, "scratch")))
        return false;
    // outputs
    if (!alloc(out.status, B, "out") || !alloc(out.exact, B, "out") || !alloc(out.lb, B, "out") ||
        !alloc(out.ub, B, "out") || !alloc(out.nchild, B, "out") || !alloc(out.sol_need, B, "out") ||
        !alloc(out.dd_nodes, B, "out") || !alloc(out.dd_arcs, B, "out") || !alloc(out.dd_layers, B, "out") ||
        !alloc(out.sweeps, B, "out") || !alloc(out.path, B * sc.Lcap, "out") || !alloc(out.path_len, B, "out") ||
        !alloc(out.ticks, B, "out") || !alloc(out.redo, B, "out") || !alloc(out.phase, B * 8, "out"))
        return false;
    // batch input
    if (!alloc(d_gl, B, "batch") || !alloc(d_sollen, B, "batch") || !alloc(d_lb, B, "batch") ||
        !alloc(d_ub, B, "batch") || !alloc(d_mask, B, "batch") || !alloc(d_valid, B, "batch") ||
        !alloc(d_soloff, B, "batch") || !alloc(d_coff, B + 1, "batch") || !alloc(d_soff, B + 1, "batch") ||
        !alloc(d_rslots, B, "batch") || !alloc(d_rcuts, B, "batch") || !alloc(d_rfeas, B, "batch"))
        return false;
    sol_cap = B * (size_t)std::max(1, L);
    if (!alloc(d_sol, sol_cap, "batch")) return false;
    if (!alloc(d_bidx, B, "bnb") || !alloc(d_boff, B + 1, "bnb") || !alloc(d_bsol, B + 1, "bnb") ||
        !alloc(d_bpaths, B * (size_t)sc.Lcap, "bnb"))
        return false;
    if (!grow_rows(64)) return false;
    cur = staged();
    return sync();
}

bool sgufp_ctx::grow_rows(int need) {
    if (need <= row_cap) return true;
    int cap = std::max(need, row_cap * 2);
    const size_t stride = (size_t)net.n_slots + 1;
    const size_t tstride = (size_t)std::max(net.L, 1) * ustride;
    double *rows = nullptr, *rhs = nullptr, *coefT = nullptr;
    if (!alloc(rows, (size_t)cap * stride, "cut rows") || !alloc(rhs, (size_t)cap, "cut rhs") ||
        !alloc(coefT, (size_t)cap * tstride, "cut coefT"))
        return false;
    if (n_rows) {
        if (!hip_ok(hipMemcpyAsync(rows, d_rows, (size_t)n_rows * stride * 8, hipMemcpyDeviceToDevice, stream), "D2D") ||
            !hip_ok(hipMemcpyAsync(rhs, d_rhs, (size_t)n_rows * 8, hipMemcpyDeviceToDevice, stream), "D2D") ||
            !hip_ok(hipMemcpyAsync(coefT, d_coefT, (size_t)n_rows * tstride * 8, hipMemcpyDeviceToDevice, stream), "D2D"))
            return false;
        if (!sync()) return false;
    }
    release(d_rows);
    release(d_rhs);
    release(d_coefT);
    d_rows = rows;
    d_rhs = rhs;
    d_coefT = coefT;
    row_cap = cap;
    return true;
}

bool sgufp_ctx::push_orders() {
    if (!order_dirty) return true;
    int need = (int)std::max(f_rows.size(), o_rows.size());
    if (need > order_cap) {
        release(d_forder);
        release(d_oorder);
        release(d_orank);
        order_cap = std::max(need, 2 * order_cap);
        if (!alloc(d_forder, order_cap, "orders") || !alloc(d_oorder, order_cap, "orders") ||
            !alloc(d_orank, order_cap, "orders"))
            return false;
    }
    // newest first: the Container is a LIFO list read from its head (Cut.h:456-465)
    std::vector<int32_t> f(f_rows.rbegin(), f_rows.rend()), o(o_rows.rbegin(), o_rows.rend());
    // screening order: strongest node-independent bound first, newest first among equals
    std::vector<int32_t> rank(o);
    std::stable_sort(rank.begin(), rank.end(), [&](int32_t a, int32_t b) { return row_ub[a] < row_ub[b]; });
    if (!upload(d_forder, f.data(), f.size()) || !upload(d_oorder, o.data(), o.size()) ||
        !upload(d_orank, rank.data(), rank.size()))
        return false;
    if (!sync()) return false;
    order_dirty = false;
    return true;
}

bool sgufp_ctx::grow_children(size_t nchild, size_t nsol) {
    if (nchild > child_cap) {
        release(d_cgl); release(d_csollen); release(d_clb); release(d_cub); release(d_cmask); release(d_csoloff);
        child_cap = std::max(nchild, child_cap * 2);
        if (!alloc(d_cgl, child_cap, "children") || !alloc(d_csollen, child_cap, "children") ||
            !alloc(d_clb, child_cap, "children") || !alloc(d_cub, child_cap, "children") ||
            !alloc(d_cmask, child_cap, "children") || !alloc(d_csoloff, child_cap, "children"))
            return false;
    }
    if (nsol > csol_cap) {
        release(d_csol);
        csol_cap = std::max(nsol, csol_cap * 2);
        if (!alloc(d_csol, csol_cap, "children")) return false;
    }
    return true;
}

static sgufp_ctx *finish_create(sgufp_ctx *ctx, int *err) {
    if (!ctx->init()) {
        if (err) *err = SGUFP_ERR_HIP;
        delete ctx;
        return nullptr;
    }
    if (err) *err = SGUFP_OK;
    return ctx;
}

// Dispatch order of k_relax.  Neighbouring records of a batch are often siblings (one
// parent's cutset) of similar cost, so in batch order heavy records start together, share
// CUs, and a run of them can start last.  Workgroup b relaxes record perm[b], a fixed
// pseudo-random permutation per batch size (results stay indexed by record).  Bench batch
// (8192 C4 records): 59.7 ms in batch order, 53.8 ms permuted.  SGUFP_RELAX_ORDER=0 keeps
// batch order.
bool sgufp_ctx::relax_order(BatchIn &in) {
    static const bool enabled = [] {
        const char *e = std::getenv("SGUFP_RELAX_ORDER");
        return !(e && e[0] == '0');
    }();
    in.perm = nullptr;
    if (!enabled || in.n < 3) return true;
    if (!d_perm && !alloc(d_perm, (size_t)max_batch, "dispatch order")) return false;
    if (perm_n != in.n) {
        std::vector<int32_t> p(in.n);
        for (int i = 0; i < in.n; i++) p[i] = i;
        uint64_t x = 0x9E3779B97F4A7C15ull ^ (uint64_t)in.n;
        for (int i = in.n - 1; i > 0; i--) {   // Fisher-Yates, splitmix64
            x += 0x9E3779B97F4A7C15ull;
            uint64_t z = x;
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            z ^= z >> 31;
            std::swap(p[i], p[(int)(z % (uint64_t)(i + 1))]);
        }
        if (!upload(d_perm, p.data(), (size_t)in.n) || !sync()) return false;
        perm_n = in.n;
    }
    in.perm = d_perm;
    return true;
}

// The cut-minor copy of the optimality rows (coefO, column j = o_rows[j]) grows with the
// pool: new columns are transposed on the device before a relaxation; the root-fold buffer
// holds one column per O cut for every batch slot.  The pending counters start at zero.
bool sgufp_ctx::exact_prepare() {
    const int no = (int)o_rows.size();
    ex.enabled = (exact_fast && no > 0) ? 1 : 0;
    ex.no = no;
    if (!ex.enabled) return true;
    const size_t rows_c = (size_t)net.n_slots + 2;
    if (no > ocap) {
        int cap = std::max(no, std::max(2 * ocap, 256));
        // footprint (n_slots + 2 + max_batch) x cap doubles: the doubling stops at what fits in
        // half of the free device memory; a pool past that leaves the exact DDs to k_relax's own
        // in-order sweeps (same results) instead of failing the search
        size_t fr = 0, tot = 0;
        const size_t per_col = (rows_c + (size_t)max_batch) * sizeof(double);
        if (hipMemGetInfo(&fr, &tot) == hipSuccess) {
            const size_t have = (size_t)ocap * per_col;   // released when the copy is done
            const size_t fit = (fr + have) / 2 / per_col;
            if ((size_t)cap > fit) cap = (int)std::max<size_t>((size_t)no, fit);
            if ((size_t)no > fit) {
                ex.enabled = 0;
                exact_capped = true;
                return true;
            }
        }
        double *c = nullptr, *r = nullptr;
        if (hipMalloc((void **)&c, rows_c * cap * sizeof(double)) != hipSuccess) {
            (void)hipGetLastError();
            ex.enabled = 0;
            exact_capped = true;
            return true;
        }
        (void)hipFree(c);
        c = nullptr;
        if (!alloc(c, rows_c * cap, "exact coefO")) return false;
        if (o_built && !hip_ok(hipMemcpy2DAsync(c, (size_t)cap * 8, d_coefO, (size_t)ocap * 8, (size_t)o_built * 8, rows_c,
                                                hipMemcpyDeviceToDevice, stream), "D2D 2D"))
            return false;
        if (d_R) release(d_R);
        if (!alloc(r, (size_t)max_batch * cap, "exact root folds")) return false;
        if (!sync()) return false;
        if (d_coefO) release(d_coefO);
        d_coefO = c;
        d_R = r;
        ocap = cap;
    }
    if (!d_pslot && (!alloc(d_pslot, (size_t)max_batch, "exact pending") || !alloc(d_pbase, (size_t)max_batch, "exact pending") ||
                     !alloc(d_ectr, 32, "exact pending") || !alloc(d_pidx, (size_t)max_batch, "exact pending")))
        return false;
    // open-leaf compaction of the leaf passes: per pending record its open leaves after phase A
    // (at most all its leaves: the leaf-pass space x kLeafPass entries)
    if (leaf_split > 0 && !d_open_cnt) {
        const size_t npass = (size_t)max_batch * ((size_t)sc.Ncap / kLeafPass + 1);
        if (!alloc(d_open_cnt, (size_t)max_batch, "exact open leaves") ||
            !alloc(d_open_list, npass * kLeafPass, "exact open leaves"))
            return false;
    }
    if (!nx_prepare(no)) return false;
    if (o_built < no) {
        if (!hip_ok(launch_exact_cols(d_rows, d_rhs, d_oorder, no, o_built, net.n_slots + 1, net.n_slots, ocap, d_coefO,
                                      1, stream), "k_exact_cols"))
            return false;
        o_built = no;
    }
    // screening columns: the strongest optimality cuts (push_orders' o_rank), rebuilt per launch
    ex.nsc = std::min(no, exact_screen);
    if (ex.nsc > 0) {
        if (!d_coefS && (!alloc(d_coefS, rows_c * kExactScreen, "exact screen") ||
                         !alloc(d_RS, (size_t)max_batch * kExactScreen, "exact screen")))
            return false;
        if (!hip_ok(launch_exact_cols(d_rows, d_rhs, d_orank, ex.nsc, 0, net.n_slots + 1, net.n_slots, kExactScreen,
                                      d_coefS, 0, stream), "k_exact_cols"))
            return false;
    }
    ex.coefS = d_coefS;
    ex.RS = d_RS;
    if (!hip_ok(hipMemsetAsync(d_ectr, 0, 32 * sizeof(unsigned long long), stream), "memset") ||
        !hip_ok(hipMemsetAsync(d_pidx, 0xFF, (size_t)max_batch * sizeof(int32_t), stream), "memset") ||
        (d_open_cnt && !hip_ok(hipMemsetAsync(d_open_cnt, 0, (size_t)max_batch * sizeof(int32_t), stream), "memset")))
        return false;
    ex.leaf_split = d_open_cnt ? leaf_split : 0;
    ex.leaf_phase = 0;
    ex.open_cnt = d_open_cnt;
    ex.open_list = d_open_list;
    ex.lazy = ex.nsc == 0 ? exact_lazy : 0;
    ex.pidx = d_pidx;
    ex.nslots = max_batch;
    ex.ostride = ocap;
    ex.coefO = d_coefO;
    ex.R = d_R;
    ex.pend_slot = d_pslot;
    ex.pend_base = d_pbase;
    ex.ctr = d_ectr;
    return true;
}

void sgufp_ctx::sub_stats_add(int n_paths) {
    const size_t n = (size_t)n_paths * (size_t)sn.S;
    std::vector<int32_t> w(2 * n);
    if (!sio.wstat || !download(w.data(), sio.wstat, 2 * n) || !sync()) return;
    ss[0] += 1;
    ss[1] += (double)n;
    for (size_t k = 0; k < n; k++) {
        const int a = w[2 * k], p = w[2 * k + 1];
        if (a < 0) ss[6] += 1;
        else ss[3] += a;
        ss[4] += p & 0xFFFFF;
        ss[5] += (p >> 20) & 2047;
    }
    if ((int)ss[0] % 200 == 0)
        std::fprintf(stderr, "[sub] launches %.0f scenarios %.0f: augmentations %.2f, flow passes %.2f, potential passes "
                             "%.2f per scenario, fallbacks %.0f\n",
                     ss[0], ss[1], ss[3] / ss[1], ss[4] / ss[1], ss[5] / ss[1], ss[6]);
}

// Buffers of the non-exact hand-off (ExactIO::nx): per pending entry its kind and pruning
// position, per (entry, O cut) the pruning gap and maxState (as wide as the root folds), a
// small header per slot.  Only under pools of nx_min O cuts or more, with the batched sweeps
// (aligned records, packed topology); a device without the memory runs every record in
// k_relax (same results).
bool sgufp_ctx::nx_prepare(int no) {
    ex.nx = 0;
    ex.redo = 0;
    ex.nx_min = nx_min;
    ex.nx_skip = nx_skip;
    ex.pkind = nullptr;
    if (!nx_on || no < nx_min || cb <= 1) return true;
    const size_t B = (size_t)max_batch;
    // leaf passes: at most ceil(leaves / kLeafPass) per record
    const size_t npass = B * ((size_t)sc.Ncap / kLeafPass + 1);
    if (!d_nxh && (!alloc(d_nxh, B * 4, "nx header") || !alloc(d_pkind, B, "nx pending") || !alloc(d_P, B, "nx pending") ||
                   !alloc(d_pstop, npass, "nx pending") || !alloc(d_nxlist, B, "nx pending")))
        return false;
    if (nx_cap < ocap) {
        size_t fr = 0, tot = 0;
        const size_t have = (size_t)nx_cap * B * 16;
        if (hipMemGetInfo(&fr, &tot) == hipSuccess && (size_t)ocap * B * 16 > (fr + have) / 2) return true;
        if (d_G) release(d_G);
        if (d_MS) release(d_MS);
        nx_cap = 0;
        if (!alloc(d_G, B * (size_t)ocap, "nx gaps") || !alloc(d_MS, B * (size_t)ocap, "nx maxState")) return false;
        nx_cap = ocap;
    }
    ex.nx = 1;
    ex.pkind = d_pkind;
    ex.P = d_P;
    ex.G = d_G;
    ex.MS = d_MS;
    ex.nxh = d_nxh;
    ex.pstop = d_pstop;
    ex.nxlist = d_nxlist;
    ex.nx_ms = 0;
    return true;
}

bool sgufp_ctx::relax_current(double optimal_lb) {
    // the slots' meta[5] become pool cut indices: the sgufp_dd_* view of the batch ends here
    dd_built = false;
    if (!push_orders() || !exact_prepare()) return false;
    relax_lb = optimal_lb;
    BatchIn in = cur;
    if (!relax_order(in)) return false;
    const Pool p = pool();
    hipStream_t st = stream;
    if (timing) hipEventRecord(ev[0], st);
    if (!hip_ok(launch_relax(nd, sc, in, p, out, optimal_lb, cb, ex, cus, st), "k_relax")) return false;
    if (timing) hipEventRecord(ev[1], st);
    return emit_current(in, p);
}

bool sgufp_ctx::emit_current(const BatchIn &in, const Pool &p) {
    hipStream_t st = stream;
    if (in.n > 0 && !hip_ok(launch_scan(out.nchild, out.sol_need, in.n, d_coff, d_soff, st), "k_scan2")) return false;
    uint64_t tot[2] = {0, 0};
    if (in.n > 0) {
        if (!download(&tot[0], d_coff + in.n, 1) || !download(&tot[1], d_soff + in.n, 1)) return false;
    }
    if (!sync()) return false;
    const char *es = std::getenv("SGUFP_EXACT_STATS");   // diagnostics (tests read them from stderr)
    const bool estats = es && es[0] == '1';
    if (estats && ex.enabled) {
        unsigned long long c[32];
        if (download(c, d_ectr, 32) && sync())
            std::fprintf(stderr,
                         "[exact] pending %llu passes %llu blocks swept %llu of %llu (no %d, screen %d, lazy %d: "
                         "%llu resolves, %llu blocks); non-exact: dag items %llu, fallbacks %llu, kept back "
                         "(ranks %llu, tail %llu, segment %llu, program %llu, other %llu), handed off %llu; exact "
                         "leaves %llu, open after 16 blocks %llu, after 64 %llu; split %d: open after it %llu, "
                         "phase-B blocks %llu\n",
                         c[0] >> 32, c[0] & 0xFFFFFFFFull, c[3],
                         (c[0] & 0xFFFFFFFFull) * (unsigned long long)((ex.no + 63) / 64 + (ex.nsc + 63) / 64), ex.no,
                         ex.nsc, ex.lazy, c[4], c[5], c[6], c[7], c[9] & 1023, (c[9] >> 10) & 1023, (c[9] >> 20) & 1023,
                         (c[9] >> 30) & 1023, (c[9] >> 40) & 1023, c[12], c[15], c[14], c[13], ex.leaf_split, c[18],
                         c[19]);
        if (estats && ex.enabled && download(c, d_ectr, 32) && sync()) {
            // the leaf passes' algorithmic bytes, summed over the context's launches: per swept cut
            // block of a pass, its staged coefficient rows and the root-fold column (64 cuts x 8 B each)
            leaf_cum[0] += c[21];
            leaf_cum[1] += c[20];
            for (int x = 0; x < 3; x++) leaf_cum[2 + x] += c[22 + x];   // SGUFP_LEAF_CLOCKS builds
            std::fprintf(stderr, "[exact-cum] leaf pass-blocks %llu row-blocks %llu bytes %.6e wave-cycles stage %llu "
                                 "leaves %llu sync %llu\n",
                         (unsigned long long)leaf_cum[0], (unsigned long long)leaf_cum[1],
                         (double)(leaf_cum[0] + leaf_cum[1]) * 64.0 * 8.0, leaf_cum[2], leaf_cum[3], leaf_cum[4]);
        }
    }
    total_children = (int64_t)tot[0];
    total_csol = (int64_t)tot[1];
    if (!grow_children((size_t)tot[0], (size_t)tot[1])) return false;
    ChildOut co = children_view();
    if (timing) hipEventRecord(ev[2], st);
    if (tot[0] > 0 && !hip_ok(launch_emit(nd, sc, in, p, out, co, st), "k_emit_children")) return false;
    if (timing) hipEventRecord(ev[3], st);
    relaxed = true;
    return true;
}

// Host records (Inavap::Node, DD.h:456-478) -> device encoding: states as a mask over the
// universe in force at the record's layer, solutions packed; invalid records are flagged
// (the kernels answer them with SGUFP_NODE_ERR_RECORD) rather than rejected.
void sgufp_ctx::encode_records(int n, const uint16_t *gl, const int64_t *states_off, const int16_t *states,
                               const int64_t *sol_off, const int16_t *sol, EncodedRecords &e) const {
    e.mask.assign(n, 0);
    e.valid.assign(n, 1);
    e.soff.resize(n);
    e.slen.resize(n);
    size_t total = 0;
    for (int k = 0; k < n; k++) {
        int64_t l = sol_off[k + 1] - sol_off[k];
        if (l < 0 || l > net.L) { e.valid[k] = 0; l = 0; }
        e.soff[k] = (int64_t)total;
        e.slen[k] = (uint16_t)l;
        total += (size_t)l;
    }
    e.sols.resize(total);
    for (int k = 0; k < n; k++) {
        if (e.slen[k]) std::memcpy(e.sols.data() + e.soff[k], sol + sol_off[k], e.slen[k] * sizeof(int16_t));
        for (int t = 0; t < e.slen[k]; t++) {
            int d = e.sols[e.soff[k] + t];
            if (d != -1 && (d < 0 || d >= net.m)) e.valid[k] = 0;
        }
        int g = gl[k];
        if (g > net.L) { e.valid[k] = 0; continue; }
        // at a layer with a state update the build replaces the states (DD.cpp:3557-3571): they
        // are kept when they fit the layer's universe (frontier round trips) and never invalid
        const bool replaced = g < net.L && net.layer_update[g] >= 0;
        int u = net.layer_universe[g];
        int prev = -1;
        for (int64_t t = states_off[k]; t < states_off[k + 1]; t++) {
            int r = -1;
            if (u >= 0) {
                const auto &U = net.sets[u];
                auto it = std::lower_bound(U.begin(), U.end(), states[t]);
                if (it != U.end() && *it == states[t]) r = (int)(it - U.begin());
            }
            if (r < 0 || r <= prev) {   // not a sorted subset of the universe
                if (replaced) e.mask[k] = 0;
                else e.valid[k] = 0;
                break;
            }
            e.mask[k] |= 1u << r;
            prev = r;
        }
    }
}

bool sgufp_ctx::rdd_init() {
    if (rdd_ready) return true;
    const size_t B = (size_t)max_batch;
    rio.Tcap = sc.Tcap;
    rio.Lcap = sc.Lcap;
    if (rdd_lds_bytes(rio.Tcap, rio.Lcap, ustride) > 64 * 1024) { err = "too many layers for the restricted DD"; return false; }
    if (!alloc(rio.topo, B * rio.Tcap * kRddMax, "restricted") || !alloc(rio.cmask, B * kRddMax, "restricted") ||
        !alloc(rio.csm, B * kRddMax, "restricted") || !alloc(rio.csdec, B * kRddMax * rio.Tcap, "restricted") ||
        !alloc(rio.status, B, "restricted") || !alloc(rio.exact, B, "restricted") || !alloc(rio.lb, B, "restricted") ||
        !alloc(rio.path, B * rio.Lcap, "restricted") || !alloc(rio.path_len, B, "restricted") ||
        !alloc(rio.cs_n, B, "restricted") || !alloc(rio.cs_gl, B, "restricted"))
        return false;
    rdd_ready = true;
    return true;
}

extern "C" {


sgufp_ctx *sgufp_create_from_file(const char *path, int device, int max_batch, int *err) {
    if (!path || max_batch <= 0) { if (err) *err = SGUFP_ERR_ARG; return nullptr; }
    auto *ctx = new sgufp_ctx();
    ctx->device = device;
    ctx->max_batch = max_batch;
    if (!ctx->net.load_file(path)) {
        if (err) *err = SGUFP_ERR_NETWORK;
        delete ctx;
        return nullptr;
    }
    return finish_create(ctx, err);
}

sgufp_ctx *sgufp_create(int n, int m, int scenarios, const int32_t *tails, const int32_t *heads, const int32_t *lb,
                        const int32_t *ub, const int32_t *reward, int n_vbar, const int32_t *vbar, int device,
                        int max_batch, int *err) {
    if (n <= 0 || m < 0 || scenarios <= 0 || max_batch <= 0 || (m && (!tails || !heads || !lb || !ub || !reward)) ||
        (n_vbar && !vbar)) {
        if (err) *err = SGUFP_ERR_ARG;
        return nullptr;
    }
    auto *ctx = new sgufp_ctx();
    ctx->device = device;
    ctx->max_batch = max_batch;
    if (!ctx->net.load_arrays(n, m, scenarios, tails, heads, lb, ub, reward, n_vbar, vbar)) {
        if (err) *err = SGUFP_ERR_NETWORK;
        delete ctx;
        return nullptr;
    }
    return finish_create(ctx, err);
}

void sgufp_destroy(sgufp_ctx *ctx) { delete ctx; }

const char *sgufp_last_error(const sgufp_ctx *ctx) {
    if (!ctx) return "null context";
    return ctx->err.empty() ? ctx->net.error.c_str() : ctx->err.c_str();
}

void *sgufp_stream(const sgufp_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

int sgufp_get_network_info(const sgufp_ctx *ctx, sgufp_network_info *o) {
    if (!ctx || !o) return SGUFP_ERR_ARG;
    o->n = ctx->net.n; o->m = ctx->net.m; o->scenarios = ctx->net.S;
    o->total_layers = ctx->net.L;
    o->n_vbar = (int32_t)ctx->net.vbar.size();
    o->max_states = ctx->net.max_states;
    o->n_slots = ctx->net.n_slots;
    o->max_batch = ctx->max_batch;
    o->node_capacity = ctx->sc.Ncap;
    o->arc_capacity = ctx->sc.Acap;
    o->scratch_bytes = (int64_t)ctx->held;
    return SGUFP_OK;
}

int sgufp_processing_order(const sgufp_ctx *ctx, int32_t *layer_arcs, int32_t *vbar_order) {
    if (!ctx) return SGUFP_ERR_ARG;
    if (layer_arcs) std::copy(ctx->net.layer_arc.begin(), ctx->net.layer_arc.end(), layer_arcs);
    if (vbar_order) std::copy(ctx->net.vbar.begin(), ctx->net.vbar.end(), vbar_order);
    return SGUFP_OK;
}

int sgufp_probe_network(const char *path, int32_t *total_layers, int32_t *n_vbar, int32_t cap, int32_t *layer_arcs,
                        int32_t *vbar_order) {
    if (!path) return SGUFP_ERR_ARG;
    Network net;
    if (!net.load_file(path)) return SGUFP_ERR_NETWORK;
    if (total_layers) *total_layers = net.L;
    if (n_vbar) *n_vbar = (int32_t)net.vbar.size();
    for (int k = 0; layer_arcs && k < std::min<int>(cap, net.L); k++) layer_arcs[k] = net.layer_arc[k];
    for (int k = 0; vbar_order && k < std::min<int>(cap, (int)net.vbar.size()); k++) vbar_order[k] = net.vbar[k];
    return SGUFP_OK;
}

// One cut's (key, value) list -> dense row of n_slots + 1 doubles (the last slot 0: absent key)
int sgufp_ctx::densify(int64_t nnz, const uint64_t *keys, const double *vals, double *row) {
    const size_t stride = (size_t)net.n_slots + 1;
    std::fill(row, row + stride, 0.0);
    std::vector<uint8_t> seen(stride, 0);
    for (int64_t k = 0; k < nnz; k++) {
        uint64_t key = keys[k] & 0xFFFFFFFFFFFFull;
        auto it = key_slots.find(key);
        if (it == key_slots.end()) {
            err = "cut key is not an (i,q,j) triple of a DD layer";
            return SGUFP_ERR_KEY;
        }
        for (int s : it->second) {
            if (seen[s]) continue;  // Cut::get returns the first match (Cut.h:278-281)
            seen[s] = 1;
            row[s] = vals[k];
        }
    }
    return SGUFP_OK;
}

int sgufp_cuts_append(sgufp_ctx *ctx, int is_feasibility, int n_cuts, const double *rhs, const int64_t *nnz_off,
                      const uint64_t *keys, const double *vals) {
    if (!ctx || n_cuts < 0 || (n_cuts && (!rhs || !nnz_off))) return SGUFP_ERR_ARG;
    if (n_cuts == 0) return SGUFP_OK;
    const size_t stride = (size_t)ctx->net.n_slots + 1;
    std::vector<double> rows((size_t)n_cuts * stride, 0.0);
    for (int c = 0; c < n_cuts; c++) {
        const int rc = ctx->densify(nnz_off[c + 1] - nnz_off[c], keys + nnz_off[c], vals + nnz_off[c],
                                    rows.data() + (size_t)c * stride);
        if (rc != SGUFP_OK) return rc;
    }
    return ctx->append_rows(is_feasibility, n_cuts, rhs, rows) ? SGUFP_OK : SGUFP_ERR_HIP;
}

bool sgufp_ctx::append_rows(int is_feasibility, int n_cuts, const double *rhs_in, const std::vector<double> &rows) {
    // per (layer, state rank) coefficients for the batched sweeps: coefT[l][r] = row[slot_tab[l][r]]
    const size_t stride = (size_t)net.n_slots + 1;
    const int us = ustride;
    const size_t tstride = (size_t)std::max(net.L, 1) * us;
    std::vector<double> coefT((size_t)n_cuts * tstride, 0.0);
    for (int c = 0; c < n_cuts; c++)
        for (int l = 0; l < net.L; l++)
            for (int r = 0; r < us; r++) {
                int sl = net.slot_tab[(size_t)l * kMaxStates + r];
                if (sl >= 0) coefT[(size_t)c * tstride + (size_t)l * us + r] = rows[(size_t)c * stride + sl];
            }
    int first = n_rows;
    if (!grow_rows(first + n_cuts)) return false;
    row_ub.resize((size_t)first + n_cuts);
    for (int c = 0; c < n_cuts; c++) {
        double b = rhs_in[c];
        for (int l = 0; l < net.L; l++) {
            double m = 0.0;
            for (int r = 0; r < us; r++) m = std::max(m, coefT[(size_t)c * tstride + (size_t)l * us + r]);
            b += m;
        }
        row_ub[(size_t)first + c] = b;
    }
    if (!upload(d_coefT + (size_t)first * tstride, coefT.data(), coefT.size()) ||
        !upload(d_rows + (size_t)first * stride, rows.data(), rows.size()) ||
        !upload(d_rhs + first, rhs_in, (size_t)n_cuts) || !sync())
        return false;
    for (int c = 0; c < n_cuts; c++) (is_feasibility ? f_rows : o_rows).push_back(first + c);
    n_rows += n_cuts;
    order_dirty = true;
    return true;
}

int sgufp_cuts_append_rows(sgufp_ctx *ctx, int is_feasibility, int n_cuts, const double *rhs, const double *rows) {
    if (!ctx || n_cuts < 0 || (n_cuts && (!rhs || !rows))) return SGUFP_ERR_ARG;
    if (n_cuts == 0) return SGUFP_OK;
    const size_t stride = (size_t)ctx->net.n_slots + 1;
    std::vector<double> r(rows, rows + (size_t)n_cuts * stride);
    for (int c = 0; c < n_cuts; c++) r[(size_t)c * stride + stride - 1] = 0.0;   // the absent-key slot
    return ctx->append_rows(is_feasibility, n_cuts, rhs, r) ? SGUFP_OK : SGUFP_ERR_HIP;
}

int sgufp_slot_keys(const sgufp_ctx *ctx, uint64_t *keys) {
    if (!ctx || !keys) return SGUFP_ERR_ARG;
    for (int s = 0; s < ctx->net.n_slots; s++) keys[s] = ctx->net.slot_key(s);
    return SGUFP_OK;
}

// ---- scenario subproblem ------------------------------------------------------------
bool sgufp_ctx::sub_init() {
    if (sub_ready) return true;
    const Network &N = net;
    const int n = N.n, m = N.m, S = N.S;
    // chain records keep node / arc ids and bounds in 16 bits (ids already are: Cut.h:342-344)
    // (predecessor words pack arc code << 15 | node: 2 (m + n + 1) codes must fit 16 bits)
    if (n > 32767 || m > 32767 || 2 * (m + n + 1) > 65535) { err = "subproblem: more than 32766 nodes + arcs"; return false; }
    for (size_t i = 0; i < N.lb.size(); i++)
        if (N.lb[i] < -32768 || N.lb[i] > 32767 || N.ub[i] < -32768 || N.ub[i] > 32767) {
            err = "subproblem: arc bounds outside 16 bits";
            return false;
        }
    std::vector<int32_t> zlist;   // free-supply / free-demand nodes (no conservation row)
    for (int v = 0; v < n; v++) {
        const bool src = N.in_arcs[v].empty(), snk = N.out_arcs[v].empty();
        if ((src || snk) && !(src && snk))
            zlist.push_back((int32_t)((uint32_t)v | (src ? 1u << 30 : 0u) | (snk ? 1u << 29 : 0u)));
    }
    const int nz = (int)zlist.size();
    // chains are numbered in the topological order of their tails, so that one sweep in
    // chain order carries a label down a whole run of forward arcs (Kahn's order; on a
    // cycle the remaining nodes follow in id order -- only the speed depends on it)
    std::vector<int32_t> rank(n, -1), indeg(n, 0), arc_topo(m);
    {
        std::vector<int32_t> q;
        for (int v = 0; v < n; v++) indeg[v] = (int32_t)N.in_arcs[v].size();
        for (int v = 0; v < n; v++) if (indeg[v] == 0) q.push_back(v);
        int r = 0;
        for (size_t i = 0; i < q.size(); i++) {
            const int v = q[i];
            rank[v] = r++;
            for (int a : N.out_arcs[v]) if (--indeg[N.head[a]] == 0) q.push_back(N.head[a]);
        }
        for (int v = 0; v < n; v++) if (rank[v] < 0) rank[v] = r++;
        for (int a = 0; a < m; a++) arc_topo[a] = a;
        std::stable_sort(arc_topo.begin(), arc_topo.end(), [&](int a, int b) { return rank[N.tail[a]] < rank[N.tail[b]]; });
    }
    if (sub_lds_bytes(n, m, m, nz, 4) > 160 * 1024) { err = "network too large for the LDS subproblem"; return false; }
    std::vector<int32_t> inner(n), arc_layer(m, -1), lb((size_t)S * m), ub((size_t)S * m), rew(m);
    std::vector<uint8_t> vb(n), in8(n);
    std::vector<int32_t> in_off(n + 1, 0), out_off(n + 1, 0), in_list, out_list;
    for (int v = 0; v < n; v++) {
        vb[v] = N.is_vbar[v];
        in8[v] = (!N.in_arcs[v].empty() && !N.out_arcs[v].empty()) ? 1 : 0;
        in_off[v] = (int32_t)in_list.size();
        for (int a : N.in_arcs[v]) in_list.push_back(a);
        out_off[v] = (int32_t)out_list.size();
        for (int a : N.out_arcs[v]) out_list.push_back(a);
    }
    in_off[n] = (int32_t)in_list.size();
    out_off[n] = (int32_t)out_list.size();
    for (int l = 0; l < N.L; l++) arc_layer[N.layer_arc[l]] = l;
    for (int a = 0; a < m; a++) {
        rew[a] = N.reward[(size_t)a * S];
        for (int s = 0; s < S; s++) {
            lb[(size_t)s * m + a] = N.lb[(size_t)a * S + s];
            ub[(size_t)s * m + a] = N.ub[(size_t)a * S + s];
        }
    }
    // rank of head(b) among the distinct heads of tail(b)'s out-arcs (network.cpp's slot order)
    std::vector<int16_t> orank(m, 0);
    for (int v = 0; v < n; v++) {
        std::vector<int32_t> hs;
        for (int a : N.out_arcs[v]) {
            const auto it = std::find(hs.begin(), hs.end(), N.head[a]);
            orank[a] = (int16_t)(it - hs.begin());
            if (it == hs.end()) hs.push_back(N.head[a]);
        }
    }
    int32_t *d_tail, *d_head, *d_layer, *d_lb, *d_ub, *d_rew, *d_ioff, *d_il, *d_ooff, *d_ol, *d_soff, *d_shead, *d_z, *d_topo;
    uint8_t *d_vb, *d_inner;
    int16_t *d_orank;
    if (!alloc(d_tail, m, "sub") || !alloc(d_head, m, "sub") || !alloc(d_layer, m, "sub") ||
        !alloc(d_lb, (size_t)S * m, "sub") || !alloc(d_ub, (size_t)S * m, "sub") || !alloc(d_rew, m, "sub") ||
        !alloc(d_ioff, n + 1, "sub") || !alloc(d_il, m, "sub") || !alloc(d_ooff, n + 1, "sub") ||
        !alloc(d_ol, m, "sub") || !alloc(d_soff, N.L + 1, "sub") || !alloc(d_shead, N.n_slots, "sub") ||
        !alloc(d_vb, n, "sub") || !alloc(d_inner, n, "sub") || !alloc(d_z, std::max(nz, 1), "sub") ||
        !alloc(d_topo, m, "sub") || !alloc(d_orank, m, "sub"))
        return false;
    if (!upload(d_tail, N.tail.data(), m) || !upload(d_head, N.head.data(), m) || !upload(d_layer, arc_layer.data(), m) ||
        !upload(d_lb, lb.data(), lb.size()) || !upload(d_ub, ub.data(), ub.size()) || !upload(d_rew, rew.data(), m) ||
        !upload(d_ioff, in_off.data(), in_off.size()) || !upload(d_il, in_list.data(), in_list.size()) ||
        !upload(d_ooff, out_off.data(), out_off.size()) || !upload(d_ol, out_list.data(), out_list.size()) ||
        !upload(d_soff, N.slot_off.data(), N.slot_off.size()) || !upload(d_shead, N.slot_head.data(), N.slot_head.size()) ||
        !upload(d_vb, vb.data(), n) || !upload(d_inner, in8.data(), n) || (nz && !upload(d_z, zlist.data(), nz)) || !upload(d_topo, arc_topo.data(), m) ||
        !upload(d_orank, orank.data(), m) || !sync())
        return false;
    sn.n = n; sn.m = m; sn.S = S; sn.L = N.L; sn.n_slots = N.n_slots; sn.nz = nz; sn.zlist = d_z; sn.arc_topo = d_topo; sn.orank = d_orank;
    {
        // every arc sits in one chain, so M = 1 + sum_chains 2 |R| (U + 1) (k_sub_scenario)
        // is at most 1 + 2 sum_a |r_a| (max u + 1); residual costs are below R + M <= 2 M
        int64_t sr = 0, umax = 0;
        for (int a = 0; a < m; a++) sr += std::abs((int64_t)rew[a]);
        for (size_t i = 0; i < ub.size(); i++) umax = std::max<int64_t>(umax, ub[i]);
        sn.cost_bound = 2 * (1 + 2 * sr * (umax + 1));
        // 32-bit keys and 8-byte chain records (k_sub_scenario): no lower bound, no negative
        // upper bound (a chain is then never infeasible up front), small rewards, ids and
        // upper bounds (11-bit fields)
        bool any_lb = false, neg_ub = false;
        for (size_t i = 0; i < lb.size(); i++) any_lb |= lb[i] != 0;
        for (size_t i = 0; i < ub.size(); i++) neg_ub |= ub[i] < 0;
        sn.key32 = (!any_lb && !neg_ub && sr < ((int64_t)1 << 18) && n + 2 < (1 << 11) && umax < (1 << 11)) ? 1 : 0;
        const char *ep = getenv("SGUFP_SUB_PREDS_LDS");
        sn.preds_lds = (ep && atoi(ep) == 1) ? 1 : 0;
    }
    sn.tail = d_tail; sn.head = d_head; sn.vbar = d_vb; sn.inner = d_inner; sn.arc_layer = d_layer;
    sn.lb = d_lb; sn.ub = d_ub; sn.reward = d_rew;
    sn.in_off = d_ioff; sn.in_list = d_il; sn.out_off = d_ooff; sn.out_list = d_ol;
    sn.slot_off = d_soff; sn.slot_head = d_shead;
    sub_ready = true;
    return true;
}

bool sgufp_ctx::sub_grow(int n, size_t total) {
    const int S = net.S, ns = net.n_slots;
    if (n > sub_cap) {
        int cap = std::max(n, 2 * sub_cap);
        int32_t *st, *ct;
        double *ob, *du, *rh, *cf, *crh, *crow, *om;
        if (!alloc(st, (size_t)cap * S, "sub io") || !alloc(ob, (size_t)cap * S, "sub io") ||
            !alloc(du, (size_t)cap * S, "sub io") || !alloc(rh, (size_t)cap * S, "sub io") ||
            !alloc(cf, (size_t)cap * S * std::max(ns, 1), "sub io") || !alloc(ct, cap, "sub io") ||
            !alloc(crh, cap, "sub io") || !alloc(crow, (size_t)cap * (ns + 1), "sub io") || !alloc(om, cap, "sub io"))
            return false;
        if (sub_cap) {
            int32_t *ost = sio.status, *oct = sio.cut_type;
            double *oob = sio.obj, *odu = sio.dual, *orh = sio.rhs, *ocf = sio.coef, *ocrh = sio.cut_rhs,
                   *ocrow = sio.cut_row, *oom = sio.obj_mean;
            release(ost); release(oct); release(oob); release(odu); release(orh); release(ocf);
            release(ocrh); release(ocrow); release(oom);
        }
        sio.status = st; sio.obj = ob; sio.dual = du; sio.rhs = rh; sio.coef = cf;
        sio.cut_type = ct; sio.cut_rhs = crh; sio.cut_row = crow; sio.obj_mean = om;
        if (d_wstat) release(d_wstat);
        if (!alloc(d_wstat, (size_t)cap * S * 2, "sub io")) return false;
        sio.wstat = d_wstat;
        if (sio.first_inf) release(sio.first_inf);
        if (!alloc(sio.first_inf, (size_t)cap, "sub io")) return false;
        // per path: its chains (k_sub_paths), m entries each at most
        const size_t pm = (size_t)cap * std::max(net.m, 1);
        if (sio.pc_info) { release(sio.pc_info); release(sio.pc_th); release(sio.pc_ol); release(sio.pc_R); release(sio.pc_arcs); release(sio.pc_rw); }
        if (!alloc(sio.pc_info, (size_t)cap * 2, "sub paths") || !alloc(sio.pc_th, pm, "sub paths") ||
            !alloc(sio.pc_ol, pm, "sub paths") || !alloc(sio.pc_R, pm, "sub paths") || !alloc(sio.pc_arcs, pm, "sub paths") ||
            !alloc(sio.pc_rw, pm, "sub paths"))
            return false;
        int64_t *po;
        if (!alloc(po, (size_t)cap + 1, "sub io")) return false;
        if (d_spoff) release(d_spoff);
        d_spoff = po;
        sub_cap = cap;
    }
    if (total > sub_path_cap) {
        size_t cap = std::max(total, 2 * sub_path_cap);
        int16_t *pp;
        if (!alloc(pp, cap, "sub paths")) return false;
        if (d_spaths) release(d_spaths);
        d_spaths = pp;
        sub_path_cap = cap;
    }
    return true;
}

// The warm-start ring: R = 2 x max(max_batch, 32) slots (a launch solves at most max_batch
// paths, so every launch has candidates outside its own destinations), states of every
// scenario per slot.  Allocated once, on first use, and zeroed (no slot holds a state until a
// solve stores one: SubIO::wst_ok); its size never changes, so slot numbers a caller holds stay
// valid.  The repair's per-thread node masks need n + 2 <= 32 x 64; a larger network or a failed
// allocation leaves the subproblems cold.
bool sgufp_ctx::warm_reserve() {
    if (!warm_on) return false;
    if (wring.R) return true;
    if (net.n + 2 > 32 * 64) { warm_on = false; return false; }
    const int R = 2 * std::max(max_batch, 32);
    const size_t S = (size_t)net.S, m = (size_t)net.m, n_ = (size_t)net.n;
    const size_t bytes = (size_t)R * S * (m * 2 + n_ * 4 + 1);
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess && bytes > fr / 2) {
        warm_on = false;
        return false;
    }
    WarmRing w{};
    int16_t *wx = nullptr;
    int32_t *wa = nullptr;
    uint8_t *wok = nullptr;
    if (!alloc(wx, (size_t)R * S * m, "warm ring") || !alloc(wa, (size_t)R * S * n_, "warm ring") ||
        !alloc(wok, (size_t)R * S, "warm ring") ||
        !alloc(w.path, (size_t)R * std::max(sc.Lcap, 1), "warm ring") || !alloc(w.plen, (size_t)R, "warm ring") ||
        !alloc(w.valid, (size_t)R, "warm ring") || !alloc(w.src, (size_t)R, "warm ring") ||
        !alloc(w.dst, (size_t)R, "warm ring") || !alloc(w.dist, (size_t)R, "warm ring") ||
        !hip_ok(hipMemsetAsync(w.valid, 0, (size_t)R, stream), "memset") ||
        !hip_ok(hipMemsetAsync(wok, 0, (size_t)R * S, stream), "memset") ||
        !hip_ok(hipMemsetAsync(wx, 0, (size_t)R * S * m * sizeof(int16_t), stream), "memset") ||
        !hip_ok(hipMemsetAsync(wa, 0, (size_t)R * S * n_ * sizeof(int32_t), stream), "memset") || !sync())
        return false;
    static const int maxd = [] {
        const char *e = std::getenv("SGUFP_SUB_WARM_DIST");   // farther donors: cold start
        return e ? std::atoi(e) : 48;
    }();
    w.R = R;
    w.Lcap = std::max(sc.Lcap, 1);
    w.max_dist = maxd;
    wring = w;
    d_wx = wx;
    d_wa = wa;
    d_wok = wok;
    warm_ptr = 0;
    return true;
}

// shared body of sgufp_subproblem / sgufp_subproblem_warm: explicit warm slots (src / dst,
// host arrays of n entries) or none
static int subproblem_run(sgufp_ctx *ctx, int n, const int64_t *path_off, const int16_t *paths, const int32_t *src,
                          const int32_t *dst, int32_t *type, double *rhs, double *rows, double *obj_mean);

int sgufp_subproblem(sgufp_ctx *ctx, int n, const int64_t *path_off, const int16_t *paths, int32_t *type,
                     double *rhs, double *rows, double *obj_mean) {
    return subproblem_run(ctx, n, path_off, paths, nullptr, nullptr, type, rhs, rows, obj_mean);
}

int sgufp_subproblem_warm(sgufp_ctx *ctx, int n, const int64_t *path_off, const int16_t *paths, const int32_t *warm_src,
                          const int32_t *warm_dst, int32_t *type, double *rhs, double *rows, double *obj_mean) {
    if (!ctx || n < 0 || (n && (!warm_src || !warm_dst))) return SGUFP_ERR_ARG;
    if (!ctx->sub_init()) return SGUFP_ERR_HIP;
    if (n > ctx->max_batch) return SGUFP_ERR_ARG;
    if (!ctx->warm_reserve()) {
        ctx->err = "warm starts need n + 2 <= 2048 network nodes and device memory for the ring";
        return SGUFP_ERR_STATE;
    }
    // a slot is read or written by at most one path of the call, and never both
    std::vector<uint8_t> use((size_t)ctx->wring.R, 0);
    for (int k = 0; k < n; k++) {
        if (warm_src[k] < -1 || warm_src[k] >= ctx->wring.R || warm_dst[k] < -1 || warm_dst[k] >= ctx->wring.R)
            return SGUFP_ERR_ARG;
        if (warm_dst[k] >= 0) {
            if (use[warm_dst[k]] & 2) { ctx->err = "warm_dst: a slot written twice"; return SGUFP_ERR_ARG; }
            use[warm_dst[k]] |= 2;
        }
    }
    for (int k = 0; k < n; k++)
        if (warm_src[k] >= 0 && (use[warm_src[k]] & 2)) {
            ctx->err = "warm_src: a slot this call also writes";
            return SGUFP_ERR_ARG;
        }
    return subproblem_run(ctx, n, path_off, paths, warm_src, warm_dst, type, rhs, rows, obj_mean);
}

int sgufp_subproblem_stats(sgufp_ctx *ctx, int32_t *augmentations, int32_t *passes) {
    if (!ctx) return SGUFP_ERR_ARG;
    const size_t cnt = (size_t)ctx->sub_last_n * ctx->net.S;
    std::vector<int32_t> w(cnt * 2);
    if (cnt && (!ctx->download(w.data(), ctx->d_wstat, w.size()) || !ctx->sync())) return SGUFP_ERR_HIP;
    for (size_t i = 0; i < cnt; i++) {
        if (augmentations) augmentations[i] = w[2 * i];
        if (passes) passes[i] = w[2 * i + 1];
    }
    return SGUFP_OK;
}

static int subproblem_run(sgufp_ctx *ctx, int n, const int64_t *path_off, const int16_t *paths, const int32_t *src,
                          const int32_t *dst, int32_t *type, double *rhs, double *rows, double *obj_mean) {
    if (!ctx || n < 0 || (n && (!path_off || !paths))) return SGUFP_ERR_ARG;
    if (n == 0) return SGUFP_OK;
    for (int k = 0; k < n; k++)
        if (path_off[k + 1] < path_off[k] || path_off[k + 1] - path_off[k] > ctx->net.L) {
            ctx->err = "path longer than totalLayers";
            return SGUFP_ERR_ARG;
        }
    const size_t total = (size_t)(path_off[n] - path_off[0]);
    if (!ctx->sub_init() || !ctx->sub_grow(n, std::max<size_t>(total, 1))) return SGUFP_ERR_HIP;
    std::vector<int64_t> off(path_off, path_off + n + 1);
    for (auto &o : off) o -= path_off[0];
    if (!ctx->upload(ctx->d_spoff, off.data(), off.size()) || !ctx->upload(ctx->d_spaths, paths + path_off[0], total))
        return SGUFP_ERR_HIP;
    SubIO io = ctx->sio;
    io.n_paths = n;
    // chains of a path = m minus its matched out-arcs (distinct valid decisions); the LDS
    // holds the most any path of the batch needs (a wave that finds more flags an error)
    {
        const int m = ctx->net.m;
        std::vector<uint8_t> used((size_t)m, 0);
        int cap = 0;
        for (int k = 0; k < n; k++) {
            int matched = 0;
            for (int64_t i = path_off[k]; i < path_off[k + 1]; i++) {
                const int d = paths[i];
                if (d >= 0 && d < m && !used[d]) { used[d] = 1; matched++; }
            }
            for (int64_t i = path_off[k]; i < path_off[k + 1]; i++) {
                const int d = paths[i];
                if (d >= 0 && d < m) used[d] = 0;
            }
            cap = std::max(cap, m - matched);
        }
        io.nct_cap = std::max(cap, 1);
    }
    io.path_off = ctx->d_spoff;
    io.paths = ctx->d_spaths;
    io.path_slot = nullptr;
    io.path_len = nullptr;
    io.path_stride = 0;
    if (src) {   // explicit warm slots (sgufp_subproblem_warm)
        if (!ctx->upload(ctx->wring.src, src, (size_t)n) || !ctx->upload(ctx->wring.dst, dst, (size_t)n))
            return SGUFP_ERR_HIP;
        io.warm_src = ctx->wring.src;
        io.warm_dst = ctx->wring.dst;
        io.wst_x = ctx->d_wx;
        io.wst_a = ctx->d_wa;
        io.wst_ok = ctx->d_wok;
    }
    if (!ctx->hip_ok(launch_subproblem(ctx->sn, io, ctx->stream), "subproblem launch")) return SGUFP_ERR_HIP;
    ctx->sub_last_n = n;
    const size_t stride = (size_t)ctx->net.n_slots + 1;
    if ((type && !ctx->download(type, io.cut_type, n)) || (rhs && !ctx->download(rhs, io.cut_rhs, n)) ||
        (rows && !ctx->download(rows, io.cut_row, (size_t)n * stride)) ||
        (obj_mean && !ctx->download(obj_mean, io.obj_mean, n)) || !ctx->sync())
        return SGUFP_ERR_HIP;
    return SGUFP_OK;
}

int sgufp_subproblem_detail(sgufp_ctx *ctx, int32_t *status, double *objective, double *dual_objective) {
    if (!ctx) return SGUFP_ERR_ARG;
    const size_t cnt = (size_t)ctx->sub_last_n * ctx->net.S;
    if ((status && !ctx->download(status, ctx->sio.status, cnt)) || (objective && !ctx->download(objective, ctx->sio.obj, cnt)) ||
        (dual_objective && !ctx->download(dual_objective, ctx->sio.dual, cnt)) || !ctx->sync())
        return SGUFP_ERR_HIP;
    return SGUFP_OK;
}

int sgufp_cuts_clear(sgufp_ctx *ctx) {
    if (!ctx) return SGUFP_ERR_ARG;
    ctx->f_rows.clear();
    ctx->o_rows.clear();
    ctx->n_rows = 0;
    ctx->order_dirty = true;
    ctx->o_built = 0;
    ctx->shared[0] = ctx->shared[1] = 0;   // frontier shards: nothing of the new pool exchanged yet
    return SGUFP_OK;
}

int sgufp_cuts_count(const sgufp_ctx *ctx, int is_feasibility) {
    if (!ctx) return SGUFP_ERR_ARG;
    return (int)(is_feasibility ? ctx->f_rows.size() : ctx->o_rows.size());
}

int sgufp_batch_upload(sgufp_ctx *ctx, int n, const uint16_t *gl, const double *lb, const double *ub,
                       const int64_t *states_off, const int16_t *states, const int64_t *sol_off, const int16_t *sol) {
    if (!ctx || n < 0 || n > ctx->max_batch || (n && (!gl || !lb || !ub || !states_off || !sol_off)))
        return SGUFP_ERR_ARG;
    EncodedRecords e;
    ctx->encode_records(n, gl, states_off, states, sol_off, sol, e);
    const size_t total = e.sols.size();
    if (total > ctx->sol_cap) {
        ctx->release(ctx->d_sol);
        ctx->sol_cap = std::max(total, 2 * ctx->sol_cap);
        if (!ctx->alloc(ctx->d_sol, ctx->sol_cap, "batch")) return SGUFP_ERR_HIP;
    }
    ctx->n = n;
    if (!ctx->upload(ctx->d_gl, gl, n) || !ctx->upload(ctx->d_lb, lb, n) || !ctx->upload(ctx->d_ub, ub, n) ||
        !ctx->upload(ctx->d_mask, e.mask.data(), n) || !ctx->upload(ctx->d_valid, e.valid.data(), n) ||
        !ctx->upload(ctx->d_soloff, e.soff.data(), n) || !ctx->upload(ctx->d_sollen, e.slen.data(), n) ||
        !ctx->upload(ctx->d_sol, e.sols.data(), total) || !ctx->sync())
        return SGUFP_ERR_HIP;
    ctx->cur = ctx->staged();
    ctx->relaxed = false;
    ctx->dd_built = false;
    ctx->restricted_done = false;   // sgufp_restricted_* results belong to the previous batch
    return SGUFP_OK;
}

// ---- one DD at a time: Inavap::RelaxedDDNew (DD.h:797-808) -------------------------------
int sgufp_dd_build(sgufp_ctx *ctx) {
    if (!ctx) return SGUFP_ERR_ARG;
    const size_t stride = (size_t)ctx->net.n_slots + 1;
    if (!ctx->d_ddrow && (!ctx->alloc(ctx->d_ddrow, (size_t)ctx->max_batch * stride, "dd rows") ||
                          !ctx->alloc(ctx->d_ddval, 1, "dd value")))
        return SGUFP_ERR_HIP;
    BatchIn in = ctx->cur;
    in.bound_prune = 0;
    in.perm = nullptr;
    if (!ctx->hip_ok(launch_dd_build(ctx->nd, ctx->sc, in, ctx->out, (int)stride, ctx->stream), "k_relax (build)") ||
        !ctx->sync())
        return SGUFP_ERR_HIP;
    ctx->total_children = 0;
    ctx->total_csol = 0;
    ctx->relaxed = true;   // sgufp_batch_results: SUCCESS (non-exact) / NEEDS_SUBPROBLEM (exact), exact flag
    ctx->dd_built = true;
    // the build ran k_relax with no cut-parallel hand-off: sgufp_batch_refine must not read the
    // previous relaxation's pending entries or optimalLB
    ctx->relax_lb = -__DBL_MAX__;
    ctx->ex.enabled = 0;
    ctx->ex.lazy = 0;
    return SGUFP_OK;
}

int sgufp_dd_apply(sgufp_ctx *ctx, int node, int is_feasibility, double rhs, int64_t nnz, const uint64_t *keys,
                   const double *vals, double optimal, double *value) {
    if (!ctx || !ctx->dd_built || node < 0 || node >= ctx->n || nnz < 0 || (nnz && (!keys || !vals)) || !value)
        return ctx && !ctx->dd_built ? SGUFP_ERR_STATE : SGUFP_ERR_ARG;
    const size_t stride = (size_t)ctx->net.n_slots + 1;
    std::vector<double> row(stride);
    const int rc = ctx->densify(nnz, keys, vals, row.data());
    if (rc != SGUFP_OK) return rc;
    if (!ctx->upload(ctx->d_ddrow + (size_t)node * stride, row.data(), stride) ||
        !ctx->hip_ok(launch_dd_apply(ctx->nd, ctx->sc, ctx->cur, ctx->out, node, ctx->d_ddrow, (int)stride, rhs,
                                     is_feasibility ? 1 : 0, optimal, ctx->d_ddval, ctx->stream),
                     "k_dd_apply") ||
        !ctx->download(value, ctx->d_ddval, 1) || !ctx->sync())
        return SGUFP_ERR_HIP;
    return SGUFP_OK;
}

int sgufp_dd_solution(sgufp_ctx *ctx, int node, int16_t *path, int32_t *len) {
    if (!ctx || !ctx->dd_built || node < 0 || node >= ctx->n || !len)
        return ctx && !ctx->dd_built ? SGUFP_ERR_STATE : SGUFP_ERR_ARG;
    const int stride = ctx->net.n_slots + 1;
    uint16_t pl = 0;
    if (!ctx->hip_ok(launch_dd_solution(ctx->nd, ctx->sc, ctx->cur, ctx->out, node, ctx->d_ddrow, stride, ctx->stream),
                     "k_dd_solution") ||
        !ctx->download(&pl, ctx->out.path_len + node, 1) || !ctx->sync())
        return SGUFP_ERR_HIP;
    *len = pl;
    if (path && (!ctx->download(path, ctx->out.path + (size_t)node * ctx->sc.Lcap, pl) || !ctx->sync()))
        return SGUFP_ERR_HIP;
    return SGUFP_OK;
}

int sgufp_dd_cutset(sgufp_ctx *ctx, int node, double ub, int64_t *n_children) {
    if (!ctx || !ctx->dd_built || node < 0 || node >= ctx->n)
        return ctx && !ctx->dd_built ? SGUFP_ERR_STATE : SGUFP_ERR_ARG;
    int32_t st = 0;
    Pool p = ctx->pool();
    p.rows = ctx->d_ddrow;   // the slot's own row (k_dd_apply keeps meta last_cut = slot)
    if (!ctx->hip_ok(hipMemsetAsync(ctx->out.nchild, 0, (size_t)ctx->n * sizeof(uint32_t), ctx->stream), "memset") ||
        !ctx->hip_ok(hipMemsetAsync(ctx->out.sol_need, 0, (size_t)ctx->n * sizeof(uint32_t), ctx->stream), "memset") ||
        !ctx->hip_ok(launch_dd_cutset(ctx->nd, ctx->sc, ctx->out, node, ub, ctx->stream), "k_dd_cutset") ||
        !ctx->emit_current(ctx->cur, p) || !ctx->download(&st, ctx->out.status + node, 1) || !ctx->sync())
        return SGUFP_ERR_HIP;
    if (st != SGUFP_SUCCESS) {
        ctx->err = "getCutset: the DD has no width-1 layer at index >= 3 (an exact tree)";
        return SGUFP_ERR_STATE;
    }
    if (n_children) *n_children = ctx->total_children;
    return SGUFP_OK;
}

int sgufp_batch_relax(sgufp_ctx *ctx, double optimal_lb) {
    if (!ctx) return SGUFP_ERR_ARG;
    return ctx->relax_current(optimal_lb) ? SGUFP_OK : SGUFP_ERR_HIP;
}

int sgufp_batch_sync(sgufp_ctx *ctx) {
    if (!ctx) return SGUFP_ERR_ARG;
    if (!ctx->sync()) return SGUFP_ERR_HIP;
    if (ctx->timing && ctx->relaxed) {
        hipEventElapsedTime(&ctx->ms_relax, ctx->ev[0], ctx->ev[1]);
        hipEventElapsedTime(&ctx->ms_emit, ctx->ev[2], ctx->ev[3]);
    }
    return SGUFP_OK;
}

int sgufp_batch_results(sgufp_ctx *ctx, int32_t *status, uint8_t *exact, double *lb, double *ub, int32_t *n_children) {
    if (!ctx || !ctx->relaxed) return ctx ? SGUFP_ERR_STATE : SGUFP_ERR_ARG;
    const int n = ctx->n;
    std::vector<uint32_t> nc(n);
    if ((status && !ctx->download(status, ctx->out.status, n)) || (exact && !ctx->download(exact, ctx->out.exact, n)) ||
        (lb && !ctx->download(lb, ctx->out.lb, n)) || (ub && !ctx->download(ub, ctx->out.ub, n)) ||
        (n_children && !ctx->download(nc.data(), ctx->out.nchild, n)) || !ctx->sync())
        return SGUFP_ERR_HIP;
    if (n_children)
        for (int k = 0; k < n; k++) n_children[k] = (int32_t)nc[k];
    return SGUFP_OK;
}

int sgufp_batch_children_size(sgufp_ctx *ctx, int64_t *n_children, int64_t *n_states, int64_t *n_sol) {
    if (!ctx || !ctx->relaxed) return ctx ? SGUFP_ERR_STATE : SGUFP_ERR_ARG;
    const size_t nc = (size_t)ctx->total_children;
    std::vector<uint16_t> gl(nc), sl(nc);
    std::vector<uint32_t> mask(nc);
    if (!ctx->download(gl.data(), ctx->d_cgl, nc) || !ctx->download(sl.data(), ctx->d_csollen, nc) ||
        !ctx->download(mask.data(), ctx->d_cmask, nc) || !ctx->sync())
        return SGUFP_ERR_HIP;
    int64_t ns = 0, nsol = 0;
    for (size_t c = 0; c < nc; c++) {
        ns += __builtin_popcount(mask[c]);
        nsol += sl[c];
    }
    if (n_children) *n_children = (int64_t)nc;
    if (n_states) *n_states = ns;
    if (n_sol) *n_sol = nsol;
    return SGUFP_OK;
}

int sgufp_batch_children(sgufp_ctx *ctx, int64_t *child_off, uint16_t *gl, double *lb, double *ub,
                         int64_t *states_off, int16_t *states, int64_t *sol_off, int16_t *sol) {
    if (!ctx || !ctx->relaxed) return ctx ? SGUFP_ERR_STATE : SGUFP_ERR_ARG;
    const int n = ctx->n;
    const size_t nc = (size_t)ctx->total_children;
    std::vector<uint64_t> coff(n + 1);
    std::vector<uint16_t> cgl(nc), csl(nc);
    std::vector<double> clb(nc), cub(nc);
    std::vector<uint32_t> cmask(nc);
    std::vector<int64_t> csoff(nc);
    std::vector<int16_t> csol((size_t)ctx->total_csol);
    if (!ctx->download(coff.data(), ctx->d_coff, n + 1) || !ctx->download(cgl.data(), ctx->d_cgl, nc) ||
        !ctx->download(csl.data(), ctx->d_csollen, nc) || !ctx->download(clb.data(), ctx->d_clb, nc) ||
        !ctx->download(cub.data(), ctx->d_cub, nc) || !ctx->download(cmask.data(), ctx->d_cmask, nc) ||
        !ctx->download(csoff.data(), ctx->d_csoloff, nc) || !ctx->download(csol.data(), ctx->d_csol, csol.size()) ||
        !ctx->sync())
        return SGUFP_ERR_HIP;
    const Network &net = ctx->net;
    if (child_off)
        for (int k = 0; k <= n; k++) child_off[k] = (int64_t)coff[k];
    int64_t so = 0, ss = 0;
    for (size_t c = 0; c < nc; c++) {
        if (gl) gl[c] = cgl[c];
        if (lb) lb[c] = clb[c];
        if (ub) ub[c] = cub[c];
        if (states_off) states_off[c] = ss;
        int u = net.layer_universe[cgl[c]];
        for (uint32_t m = cmask[c]; m; m &= m - 1) {
            int r = __builtin_ctz(m);
            if (states) states[ss] = net.sets[u][r];
            ss++;
        }
        if (sol_off) sol_off[c] = so;
        if (sol) std::memcpy(sol + so, csol.data() + csoff[c], csl[c] * sizeof(int16_t));
        so += csl[c];
    }
    if (states_off) states_off[nc] = ss;
    if (sol_off) sol_off[nc] = so;
    return SGUFP_OK;
}

int sgufp_batch_paths(sgufp_ctx *ctx, int64_t *path_off, int16_t *paths) {
    if (!ctx || !ctx->relaxed || !path_off) return ctx ? SGUFP_ERR_STATE : SGUFP_ERR_ARG;
    const int n = ctx->n;
    std::vector<int32_t> st(n);
    std::vector<uint16_t> pl(n);
    if (!ctx->download(st.data(), ctx->out.status, n) || !ctx->download(pl.data(), ctx->out.path_len, n) || !ctx->sync())
        return SGUFP_ERR_HIP;
    int64_t off = 0;
    for (int k = 0; k < n; k++) {
        path_off[k] = off;
        if (st[k] == SGUFP_NEEDS_SUBPROBLEM) {
            if (paths && !ctx->download(paths + off, ctx->out.path + (size_t)k * ctx->sc.Lcap, pl[k])) return SGUFP_ERR_HIP;
            off += pl[k];
        }
    }
    path_off[n] = off;
    return ctx->sync() ? SGUFP_OK : SGUFP_ERR_HIP;
}

int sgufp_batch_stats(sgufp_ctx *ctx, int64_t *dd_nodes, int64_t *dd_arcs, int32_t *dd_layers, int32_t *sweeps) {
    if (!ctx || !ctx->relaxed) return ctx ? SGUFP_ERR_STATE : SGUFP_ERR_ARG;
    const int n = ctx->n;
    std::vector<uint32_t> a(n), b(n), c(n), d(n);
    if (!ctx->download(a.data(), ctx->out.dd_nodes, n) || !ctx->download(b.data(), ctx->out.dd_arcs, n) ||
        !ctx->download(c.data(), ctx->out.dd_layers, n) || !ctx->download(d.data(), ctx->out.sweeps, n) ||
        !ctx->sync())
        return SGUFP_ERR_HIP;
    for (int k = 0; k < n; k++) {
        if (dd_nodes) dd_nodes[k] = a[k];
        if (dd_arcs) dd_arcs[k] = b[k];
        if (dd_layers) dd_layers[k] = (int32_t)c[k];
        if (sweeps) sweeps[k] = (int32_t)d[k];
    }
    return SGUFP_OK;
}

int sgufp_batch_refine(sgufp_ctx *ctx, int n, const int32_t *node_idx, const uint8_t *is_feasibility,
                       const int32_t *cut_index, double optimal_lb) {
    if (!ctx || !ctx->relaxed || n < 0 || n > ctx->max_batch || (n && (!node_idx || !is_feasibility || !cut_index)))
        return SGUFP_ERR_ARG;
    if (n == 0) return SGUFP_OK;
    ctx->dd_built = false;   // k_refine rewrites the listed slots' meta[5] with pool cut indices
    if (ctx->ex.enabled && optimal_lb < ctx->relax_lb) {
        // the cut-parallel phase left partial leaf minima (upper bounds, all <= the relax-time
        // optimalLB) as terminal weights; a lower optimalLB could make one of them the argmax
        ctx->err = "sgufp_batch_refine: optimal_lb below the batch's relaxation incumbent";
        return SGUFP_ERR_ARG;
    }
    std::vector<int32_t> rows(n);
    for (int k = 0; k < n; k++) {
        const auto &v = is_feasibility[k] ? ctx->f_rows : ctx->o_rows;
        if (node_idx[k] < 0 || node_idx[k] >= ctx->n || cut_index[k] < 0 || cut_index[k] >= (int)v.size())
            return SGUFP_ERR_ARG;
        rows[k] = v[cut_index[k]];
    }
    if (!ctx->upload(ctx->d_rslots, node_idx, n) || !ctx->upload(ctx->d_rcuts, rows.data(), n) ||
        !ctx->upload(ctx->d_rfeas, is_feasibility, n))
        return SGUFP_ERR_HIP;
    if (!ctx->hip_ok(launch_refine(ctx->nd, ctx->sc, ctx->batch(), ctx->pool(), ctx->out, ctx->d_rslots, ctx->d_rcuts,
                                   ctx->d_rfeas, n, optimal_lb, ctx->ex, ctx->stream),
                     "k_refine"))
        return SGUFP_ERR_HIP;
    return ctx->sync() ? SGUFP_OK : SGUFP_ERR_HIP;
}

int sgufp_batch_phases(sgufp_ctx *ctx, int64_t *phase) {
    if (!ctx || !ctx->relaxed || !phase) return ctx ? SGUFP_ERR_STATE : SGUFP_ERR_ARG;
    if (!relax_has_phases()) {   // production build: no clock stamps in k_relax
        std::fill(phase, phase + (size_t)ctx->n * 8, (int64_t)0);
        return SGUFP_OK;
    }
    std::vector<uint64_t> t((size_t)ctx->n * 8);
    if (!ctx->download(t.data(), ctx->out.phase, t.size()) || !ctx->sync()) return SGUFP_ERR_HIP;
    for (size_t k = 0; k < t.size(); k++) phase[k] = (int64_t)t[k];
    return SGUFP_OK;
}

int sgufp_batch_debug(sgufp_ctx *ctx, int64_t *ticks, int32_t *redo) {
    if (!ctx || !ctx->relaxed) return ctx ? SGUFP_ERR_STATE : SGUFP_ERR_ARG;
    const int n = ctx->n;
    std::vector<uint64_t> t(n);
    std::vector<uint32_t> r(n);
    if (!ctx->download(t.data(), ctx->out.ticks, n) || !ctx->download(r.data(), ctx->out.redo, n) || !ctx->sync())
        return SGUFP_ERR_HIP;
    const bool stamped = relax_has_phases();
    for (int k = 0; k < n; k++) {
        if (ticks) ticks[k] = stamped ? (int64_t)t[k] : 0;
        if (redo) redo[k] = (int32_t)r[k];
    }
    return SGUFP_OK;
}

int sgufp_batch_routes(sgufp_ctx *ctx, int32_t *route) {
    if (!ctx || !route) return SGUFP_ERR_ARG;
    if (!ctx->relaxed) return SGUFP_ERR_STATE;
    const int n = ctx->n;
    std::fill(route, route + n, SGUFP_ROUTE_IN_ORDER);
    if (!ctx->ex.enabled || n == 0) return SGUFP_OK;   // no hand-off in the last relaxation
    unsigned long long c0 = 0;
    std::vector<int32_t> pidx((size_t)n);
    if (!ctx->download(&c0, ctx->d_ectr, 1) || !ctx->download(pidx.data(), ctx->d_pidx, (size_t)n) || !ctx->sync())
        return SGUFP_ERR_HIP;
    const int pending = (int)(c0 >> 32);
    std::vector<int32_t> kind((size_t)std::max(pending, 1), -1);
    if (pending > 0 && ctx->ex.nx && ctx->ex.pkind &&
        (!ctx->download(kind.data(), ctx->ex.pkind, (size_t)pending) || !ctx->sync()))
        return SGUFP_ERR_HIP;
    for (int k = 0; k < n; k++) {
        const int i = pidx[k];
        if (i < 0 || i >= pending) continue;
        route[k] = kind[i] == -1 ? SGUFP_ROUTE_EXACT_PHASE
                                 : (kind[i] == kNxRouteFallback ? SGUFP_ROUTE_NX_FALLBACK : SGUFP_ROUTE_NX_PHASE);
    }
    return SGUFP_OK;
}

int sgufp_restricted_relax(sgufp_ctx *ctx, int width, double optimal_lb) {
    if (!ctx || width < 1 || width > kRddMax) return SGUFP_ERR_ARG;
    if (!ctx->push_orders() || !ctx->rdd_init()) return SGUFP_ERR_HIP;
    ctx->rio.width = width;
    ctx->restricted_done = false;
    const BatchIn in = ctx->staged();
    if (!ctx->hip_ok(launch_restrict(ctx->nd, in, ctx->pool(), ctx->rio, optimal_lb, ctx->stream), "k_restrict") ||
        !ctx->sync())
        return SGUFP_ERR_HIP;
    ctx->restricted_done = true;
    return SGUFP_OK;
}

int sgufp_restricted_results(sgufp_ctx *ctx, int32_t *status, uint8_t *exact, double *lb, int32_t *path_len,
                             int32_t *cutset_n) {
    if (!ctx || !ctx->restricted_done) return ctx ? SGUFP_ERR_STATE : SGUFP_ERR_ARG;
    const int n = ctx->n;
    std::vector<uint16_t> pl(n);
    std::vector<uint32_t> cn(n);
    if ((status && !ctx->download(status, ctx->rio.status, n)) || (exact && !ctx->download(exact, ctx->rio.exact, n)) ||
        (lb && !ctx->download(lb, ctx->rio.lb, n)) || !ctx->download(pl.data(), ctx->rio.path_len, n) ||
        !ctx->download(cn.data(), ctx->rio.cs_n, n) || !ctx->sync())
        return SGUFP_ERR_HIP;
    for (int k = 0; k < n; k++) {
        if (path_len) path_len[k] = pl[k];
        if (cutset_n) cutset_n[k] = (int32_t)cn[k];
    }
    return SGUFP_OK;
}

int sgufp_restricted_paths(sgufp_ctx *ctx, int64_t *path_off, int16_t *paths) {
    if (!ctx || !ctx->restricted_done || !path_off) return ctx ? SGUFP_ERR_STATE : SGUFP_ERR_ARG;
    const int n = ctx->n;
    const int Lcap = ctx->sc.Lcap;
    std::vector<uint16_t> pl(n);
    std::vector<int16_t> all((size_t)n * Lcap);
    if (!ctx->download(pl.data(), ctx->rio.path_len, n) || !ctx->download(all.data(), ctx->rio.path, all.size()) ||
        !ctx->sync())
        return SGUFP_ERR_HIP;
    int64_t o = 0;
    for (int k = 0; k < n; k++) {
        path_off[k] = o;
        if (paths) std::memcpy(paths + o, all.data() + (size_t)k * Lcap, pl[k] * sizeof(int16_t));
        o += pl[k];
    }
    path_off[n] = o;
    return SGUFP_OK;
}

// host copies of what the cutset records need: counts, layers, masks, decisions, root solutions
struct RddCutset {
    std::vector<uint32_t> n, mask;
    std::vector<uint16_t> gl, sl, rg;   // cutset layer, root solution length, record layer
    std::vector<int64_t> so;
    std::vector<int16_t> dec, sol;
};

static bool rdd_cutset_download(sgufp_ctx *ctx, RddCutset &c) {
    const int n = ctx->n, T = ctx->rio.Tcap;
    c.n.resize(n); c.gl.resize(n); c.sl.resize(n); c.so.resize(n); c.rg.resize(n);
    c.mask.resize((size_t)n * kRddMax);
    c.dec.resize((size_t)n * kRddMax * T);
    if (!ctx->download(c.n.data(), ctx->rio.cs_n, n) || !ctx->download(c.gl.data(), ctx->rio.cs_gl, n) ||
        !ctx->download(c.sl.data(), ctx->d_sollen, n) || !ctx->download(c.so.data(), ctx->d_soloff, n) ||
        !ctx->download(c.rg.data(), ctx->d_gl, n) ||
        !ctx->download(c.mask.data(), ctx->rio.csm, c.mask.size()) ||
        !ctx->download(c.dec.data(), ctx->rio.csdec, c.dec.size()) || !ctx->sync())
        return false;
    size_t tot = 0;
    for (int k = 0; k < n; k++) tot = std::max(tot, (size_t)(c.so[k] + c.sl[k]));
    c.sol.resize(tot);
    return ctx->download(c.sol.data(), ctx->d_sol, tot) && ctx->sync();
}

int sgufp_restricted_cutset_size(sgufp_ctx *ctx, int64_t *n_records, int64_t *n_states, int64_t *n_sol) {
    if (!ctx || !ctx->restricted_done) return ctx ? SGUFP_ERR_STATE : SGUFP_ERR_ARG;
    RddCutset c;
    if (!rdd_cutset_download(ctx, c)) return SGUFP_ERR_HIP;
    int64_t nr = 0, ns = 0, nsol = 0;
    for (int k = 0; k < ctx->n; k++) {
        nr += c.n[k];
        const int E = (int)c.gl[k] - (int)c.rg[k];
        for (uint32_t j = 0; j < c.n[k]; j++) {
            ns += __builtin_popcount(c.mask[(size_t)k * kRddMax + j]);
            nsol += c.sl[k] + E;
        }
    }
    if (n_records) *n_records = nr;
    if (n_states) *n_states = ns;
    if (n_sol) *n_sol = nsol;
    return SGUFP_OK;
}

int sgufp_restricted_cutset(sgufp_ctx *ctx, int64_t *rec_off, uint16_t *gl, double *lb, double *ub,
                            int64_t *states_off, int16_t *states, int64_t *sol_off, int16_t *sol) {
    if (!ctx || !ctx->restricted_done) return ctx ? SGUFP_ERR_STATE : SGUFP_ERR_ARG;
    RddCutset c;
    if (!rdd_cutset_download(ctx, c)) return SGUFP_ERR_HIP;
    const Network &net = ctx->net;
    const int T = ctx->rio.Tcap;
    int64_t r = 0, ss = 0, so = 0;
    for (int k = 0; k < ctx->n; k++) {
        if (rec_off) rec_off[k] = r;
        const int E = (int)c.gl[k] - (int)c.rg[k];
        const int u = net.layer_universe[c.gl[k]];
        for (uint32_t j = 0; j < c.n[k]; j++, r++) {
            if (gl) gl[r] = c.gl[k];
            if (lb) lb[r] = -__DBL_MAX__;
            if (ub) ub[r] = -__DBL_MAX__;
            if (states_off) states_off[r] = ss;
            for (uint32_t m = c.mask[(size_t)k * kRddMax + j]; m; m &= m - 1) {
                if (states) states[ss] = net.sets[u][__builtin_ctz(m)];
                ss++;
            }
            if (sol_off) sol_off[r] = so;
            if (sol) {
                std::memcpy(sol + so, c.sol.data() + c.so[k], c.sl[k] * sizeof(int16_t));
                std::memcpy(sol + so + c.sl[k], c.dec.data() + ((size_t)k * kRddMax + j) * T, (size_t)E * sizeof(int16_t));
            }
            so += c.sl[k] + E;
        }
    }
    if (rec_off) rec_off[ctx->n] = r;
    if (states_off) states_off[r] = ss;
    if (sol_off) sol_off[r] = so;
    return SGUFP_OK;
}

int sgufp_set_timing(sgufp_ctx *ctx, int enabled) {
    if (!ctx) return SGUFP_ERR_ARG;
    ctx->timing = enabled != 0;
    return SGUFP_OK;
}

int sgufp_last_timing(const sgufp_ctx *ctx, float *ms_relax, float *ms_emit) {
    if (!ctx) return SGUFP_ERR_ARG;
    if (ms_relax) *ms_relax = ctx->ms_relax;
    if (ms_emit) *ms_emit = ctx->ms_emit;
    return SGUFP_OK;
}

}  // extern "C"
