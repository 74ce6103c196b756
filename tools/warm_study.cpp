// Study tool (not product, not test): how much of the scenario subproblem's max-reward flow
// (sub_kernels.hip, GuroSolver::solveSubProblem /root/reference/grb.cpp:139-360) a warm start
// from an earlier path's optimal flow + potentials saves, on the paths the device B&B actually
// solved (tools/sub_paths_dump.py -> tools/warm_study.py writes the input).
//
//   g++ -O2 -std=c++17 tools/warm_study.cpp -o /tmp/warm_study && /tmp/warm_study in.txt S0 NS
//
// Per (path, scenario): the cold successive-shortest-path count (what k_sub_scenario runs)
// and, warm-started from the previous path's state of the same scenario, the shortest-path
// computations and augmentations of the repair (excess -> deficit SSP under reduced costs).
#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <queue>
#include <vector>

using namespace std;
typedef long long ll;
const ll INF = (ll)1 << 60;

struct Inst {
    int n, m, S;
    vector<int> tl, hd;
    vector<vector<int>> ub, rw;   // [s][a]
    vector<char> vb;
    vector<int> arc_layer;
    vector<int> indeg, outdeg;
};

struct Chain { int t, h, U, R; vector<int> arcs; };

// chains of a path (sub_kernels.hip phase 2): only complete ones carry flow
static vector<Chain> chains_of(const Inst &I, const vector<int> &path, int s) {
    vector<int> dec(I.m, -2), chosen(I.m, -1);
    for (int a = 0; a < I.m; a++) {
        if (!I.vb[I.hd[a]]) continue;
        const int l = I.arc_layer[a];
        int d = (l >= 0 && l < (int)path.size()) ? path[l] : -1;
        if (d >= 0 && I.tl[d] != I.hd[a]) d = -1;
        dec[a] = d;
        if (d >= 0) chosen[d] = a;
    }
    vector<Chain> out;
    for (int a0 = 0; a0 < I.m; a0++) {
        if (I.vb[I.tl[a0]] && chosen[a0] >= 0) continue;
        Chain c;
        c.t = I.vb[I.tl[a0]] ? -1 : I.tl[a0];
        c.h = -1;
        c.U = INT_MAX;
        c.R = 0;
        int a = a0;
        for (;;) {
            c.arcs.push_back(a);
            c.U = min(c.U, I.ub[s][a]);
            c.R += I.rw[s][a];
            if (!I.vb[I.hd[a]]) { c.h = I.hd[a]; break; }
            if (dec[a] < 0) break;
            a = dec[a];
        }
        if (c.t >= 0 && c.h >= 0) out.push_back(c);
    }
    return out;
}

// circulation: nodes 0..n-1, Z = n; arcs: chains, Z -> source, sink -> Z (uncapacitated)
struct Flow {
    int N;
    vector<int> u, v;
    vector<ll> cap, cost, x;
    vector<vector<int>> adj;   // residual arc ids: 2e (forward), 2e+1 (backward)
    void init(int n) { N = n; adj.assign(n, {}); u.clear(); v.clear(); cap.clear(); cost.clear(); x.clear(); }
    int add(int a, int b, ll c, ll w) {
        const int e = (int)u.size();
        u.push_back(a); v.push_back(b); cap.push_back(c); cost.push_back(w); x.push_back(0);
        adj[a].push_back(2 * e);
        adj[b].push_back(2 * e + 1);
        return e;
    }
    int from(int r) const { return r & 1 ? v[r >> 1] : u[r >> 1]; }
    int to(int r) const { return r & 1 ? u[r >> 1] : v[r >> 1]; }
    ll rcap(int r) const { return r & 1 ? x[r >> 1] : cap[r >> 1] - x[r >> 1]; }
    ll rcost(int r) const { return r & 1 ? -cost[r >> 1] : cost[r >> 1]; }
};

struct Counts { ll sp = 0, aug = 0, phases = 0; };

// Bellman-Ford (SPFA) from a set of sources with initial labels; returns labels and preds
static void spfa(const Flow &F, const vector<ll> &d0, vector<ll> &d, vector<int> &pred, const vector<ll> *pi) {
    d = d0;
    pred.assign(F.N, -1);
    deque<int> q;
    vector<char> inq(F.N, 0);
    for (int i = 0; i < F.N; i++)
        if (d[i] < INF) { q.push_back(i); inq[i] = 1; }
    while (!q.empty()) {
        const int a = q.front();
        q.pop_front();
        inq[a] = 0;
        for (int r : F.adj[a]) {
            if (F.rcap(r) <= 0) continue;
            const int b = F.to(r);
            const ll w = F.rcost(r) + (pi ? (*pi)[a] - (*pi)[b] : 0);
            if (d[a] + w < d[b]) {
                d[b] = d[a] + w;
                pred[b] = r;
                if (!inq[b]) { q.push_back(b); inq[b] = 1; }
            }
        }
    }
}

// cold: SSP from Z (as Z_out) to Z (as Z_in), i.e. on the split network; augment while the
// shortest source -> sink path has negative cost
static ll solve_cold(const Inst &I, const vector<Chain> &ch, Flow &F, vector<int> &chain_arc, Counts &C) {
    const int n = I.n;
    F.init(n + 2);   // Z_out = n, Z_in = n + 1
    chain_arc.clear();
    for (auto &c : ch) chain_arc.push_back(F.add(c.t, c.h, c.U, -c.R));
    for (int v = 0; v < n; v++) {
        if (I.vb[v]) continue;
        if (I.indeg[v] == 0) F.add(n, v, INF / 4, 0);
        if (I.outdeg[v] == 0) F.add(v, n + 1, INF / 4, 0);
    }
    ll last = 1;
    for (;;) {
        vector<ll> d0(F.N, INF), d;
        vector<int> pred;
        d0[n] = 0;
        spfa(F, d0, d, pred, nullptr);
        C.sp++;
        if (d[n + 1] >= 0) break;
        if (d[n + 1] != last) { C.phases++; last = d[n + 1]; }
        ll delta = INF;
        for (int b = n + 1; b != n; b = F.from(pred[b])) delta = min(delta, F.rcap(pred[b]));
        for (int b = n + 1; b != n; b = F.from(pred[b])) {
            const int r = pred[b];
            F.x[r >> 1] += (r & 1) ? -delta : delta;
        }
        C.aug++;
    }
    ll obj = 0;
    for (size_t k = 0; k < ch.size(); k++) obj += (ll)ch[k].R * F.x[chain_arc[k]];
    return obj;
}

// state carried to the next path: flow per original arc, flow per Z arc (per free node, both
// directions), potentials of the merged circulation
struct State {
    bool valid = false;
    vector<ll> xarc;          // [m]
    vector<ll> zsrc, zsnk;    // [n]
    vector<ll> pi;            // [n + 1]
};

// potentials of an optimal circulation (merged Z): shortest distances from a virtual root
static vector<ll> potentials(const Flow &F) {
    vector<ll> d0(F.N, 0), d;
    vector<int> pred;
    spfa(F, d0, d, pred, nullptr);
    return d;
}

static void build_merged(const Inst &I, const vector<Chain> &ch, Flow &F, vector<int> &chain_arc, vector<int> &zs,
                         vector<int> &zt) {
    const int n = I.n;
    F.init(n + 1);
    chain_arc.clear();
    for (auto &c : ch) chain_arc.push_back(F.add(c.t, c.h, c.U, -c.R));
    zs.assign(n, -1);
    zt.assign(n, -1);
    for (int v = 0; v < n; v++) {
        if (I.vb[v]) continue;
        if (I.indeg[v] == 0) zs[v] = F.add(n, v, INF / 4, 0);
        if (I.outdeg[v] == 0) zt[v] = F.add(v, n, INF / 4, 0);
    }
}

static void save_state(const Inst &I, const vector<Chain> &ch, const Flow &F, const vector<int> &chain_arc,
                       const vector<int> &zs, const vector<int> &zt, State &st) {
    st.valid = true;
    st.xarc.assign(I.m, 0);
    for (size_t k = 0; k < ch.size(); k++)
        for (int a : ch[k].arcs) st.xarc[a] = F.x[chain_arc[k]];
    st.zsrc.assign(I.n, 0);
    st.zsnk.assign(I.n, 0);
    for (int v = 0; v < I.n; v++) {
        if (zs[v] >= 0) st.zsrc[v] = F.x[zs[v]];
        if (zt[v] >= 0) st.zsnk[v] = F.x[zt[v]];
    }
    st.pi = potentials(F);
}

// cold solution in the merged form (for the state): the split solution's flows, Z arcs by
// the sources' / sinks' net flows
static void cold_to_merged(const Inst &I, const vector<Chain> &ch, const Flow &Fs, const vector<int> &ca_s, Flow &F,
                           vector<int> &ca, vector<int> &zs, vector<int> &zt) {
    build_merged(I, ch, F, ca, zs, zt);
    vector<ll> net(I.n, 0);
    for (size_t k = 0; k < ch.size(); k++) {
        F.x[ca[k]] = Fs.x[ca_s[k]];
        net[ch[k].t] -= F.x[ca[k]];
        net[ch[k].h] += F.x[ca[k]];
    }
    for (int v = 0; v < I.n; v++) {
        if (zs[v] >= 0 && net[v] < 0) F.x[zs[v]] = -net[v];
        if (zt[v] >= 0 && net[v] > 0) F.x[zt[v]] = net[v];
    }
}

// warm: previous state's flows (a chain keeps the common flow of its arcs, if they agree),
// reduced-cost rule with the previous potentials, then excess -> deficit SSP
static ll solve_warm(const Inst &I, const vector<Chain> &ch, const State &prev, Flow &F, vector<int> &ca,
                     vector<int> &zs, vector<int> &zt, Counts &C, ll *imb_total) {
    build_merged(I, ch, F, ca, zs, zt);
    const int N = I.n + 1;
    vector<ll> pi = prev.pi;
    for (size_t k = 0; k < ch.size(); k++) {
        ll f = prev.xarc[ch[k].arcs[0]];
        for (int a : ch[k].arcs) f = min(f, prev.xarc[a]);
        const int e = ca[k];
        const ll rc = F.cost[e] + pi[F.u[e]] - pi[F.v[e]];
        if (rc < 0) f = F.cap[e];
        else if (rc > 0) f = 0;
        else f = max(0ll, min(f, F.cap[e]));
        F.x[e] = f;
    }
    for (int v = 0; v < I.n; v++) {
        if (zs[v] >= 0) F.x[zs[v]] = prev.zsrc[v];
        if (zt[v] >= 0) F.x[zt[v]] = prev.zsnk[v];
    }
    vector<ll> e(N, 0);
    for (size_t a = 0; a < F.u.size(); a++) {
        e[F.u[a]] -= F.x[a];
        e[F.v[a]] += F.x[a];
    }
    ll tot = 0;
    for (int v = 0; v < N; v++) tot += e[v] > 0 ? e[v] : 0;
    *imb_total = tot;
    for (;;) {
        vector<ll> d0(N, INF), d;
        vector<int> pred;
        bool any = false;
        for (int v = 0; v < N; v++)
            if (e[v] > 0) { d0[v] = 0; any = true; }
        if (!any) break;
        spfa(F, d0, d, pred, &pi);
        C.sp++;
        int t = -1;
        for (int v = 0; v < N; v++)
            if (e[v] < 0 && d[v] < INF && (t < 0 || d[v] < d[t])) t = v;
        if (t < 0) { fprintf(stderr, "warm: excess cannot reach a deficit\n"); exit(1); }
        for (int v = 0; v < N; v++) pi[v] += min(d[v], d[t]);
        C.phases++;
        // primal-dual phase: augment along admissible (reduced cost 0) paths while one exists
        for (;;) {
            vector<ll> d1(N, INF), dd;
            vector<int> pr;
            for (int v = 0; v < N; v++)
                if (e[v] > 0) d1[v] = 0;
            spfa(F, d1, dd, pr, &pi);
            int tt = -1;
            for (int v = 0; v < N; v++)
                if (e[v] < 0 && dd[v] == 0) { tt = v; break; }
            if (tt < 0) break;
            int s = tt;
            ll delta = -e[tt];
            for (int b = tt; pr[b] >= 0; b = F.from(pr[b])) { delta = min(delta, F.rcap(pr[b])); s = F.from(pr[b]); }
            delta = min(delta, e[s]);
            for (int b = tt; pr[b] >= 0; b = F.from(pr[b])) {
                const int r = pr[b];
                F.x[r >> 1] += (r & 1) ? -delta : delta;
            }
            e[s] -= delta;
            e[tt] += delta;
            C.aug++;
        }
    }
    ll obj = 0;
    for (size_t k = 0; k < ch.size(); k++) obj += (ll)ch[k].R * F.x[ca[k]];
    return obj;
}

int main(int argc, char **argv) {
    if (argc < 4) { fprintf(stderr, "usage: warm_study in.txt s0 ns [max_paths]\n"); return 2; }
    FILE *f = fopen(argv[1], "r");
    const int s0 = atoi(argv[2]), ns = atoi(argv[3]);
    const int maxp = argc > 4 ? atoi(argv[4]) : INT_MAX;
    Inst I;
    if (fscanf(f, "%d %d %d", &I.n, &I.m, &I.S) != 3) return 1;
    I.tl.resize(I.m); I.hd.resize(I.m);
    I.ub.assign(I.S, vector<int>(I.m)); I.rw.assign(I.S, vector<int>(I.m));
    for (int a = 0; a < I.m; a++) {
        if (fscanf(f, "%d %d", &I.tl[a], &I.hd[a]) != 2) return 1;
        for (int s = 0; s < I.S; s++) {
            int l;
            if (fscanf(f, "%d %d %d", &l, &I.ub[s][a], &I.rw[s][a]) != 3) return 1;
        }
    }
    int nv;
    if (fscanf(f, "%d", &nv) != 1) return 1;
    I.vb.assign(I.n, 0);
    for (int i = 0; i < nv; i++) { int v; if (fscanf(f, "%d", &v) != 1) return 1; I.vb[v] = 1; }
    int L;
    if (fscanf(f, "%d", &L) != 1) return 1;
    I.arc_layer.assign(I.m, -1);
    for (int l = 0; l < L; l++) { int a; if (fscanf(f, "%d", &a) != 1) return 1; I.arc_layer[a] = l; }
    I.indeg.assign(I.n, 0); I.outdeg.assign(I.n, 0);
    for (int a = 0; a < I.m; a++) { I.outdeg[I.tl[a]]++; I.indeg[I.hd[a]]++; }
    int np;
    if (fscanf(f, "%d", &np) != 1) return 1;
    vector<vector<int>> paths(np);
    vector<int> rec(np);
    for (int p = 0; p < np; p++) {
        int len;
        if (fscanf(f, "%d %d", &rec[p], &len) != 2) return 1;
        paths[p].resize(len);
        for (int i = 0; i < len; i++) if (fscanf(f, "%d", &paths[p][i]) != 1) return 1;
    }
    np = min(np, maxp);
    const bool scen = argc > 5 && argv[5][0] == 's';   // warm from the previous scenario of the same path
    const bool nearest = argc > 5 && argv[5][0] == 'n';   // warm from the nearest of the last 256 paths
    if (nearest) {
        Counts warm2;
        ll nsolve2 = 0, ndist = 0;
        for (int s = s0; s < s0 + ns && s < I.S; s++) {
            std::vector<State> ring(256);
            std::vector<int> ring_p(256, -1);
            for (int p = 0; p < np; p++) {
                const auto ch = chains_of(I, paths[p], s);
                int best = -1, bd = INT_MAX;
                for (int r = 0; r < 256; r++) {
                    if (ring_p[r] < 0) continue;
                    const auto &a = paths[ring_p[r]], &b = paths[p];
                    int d = 0;
                    for (size_t i = 0; i < max(a.size(), b.size()); i++)
                        d += (i < a.size() ? a[i] : -1) != (i < b.size() ? b[i] : -1);
                    if (d < bd) { bd = d; best = r; }
                }
                Flow F;
                vector<int> ca, zs, zt;
                if (best >= 0) {
                    ll it = 0;
                    solve_warm(I, ch, ring[best], F, ca, zs, zt, warm2, &it);
                    nsolve2++;
                    ndist += bd;
                } else {
                    Flow Fs;
                    vector<int> ca_s;
                    Counts tmp;
                    solve_cold(I, ch, Fs, ca_s, tmp);
                    cold_to_merged(I, ch, Fs, ca_s, F, ca, zs, zt);
                }
                const int slot = p % 256;
                save_state(I, ch, F, ca, zs, zt, ring[slot]);
                ring_p[slot] = p;
            }
        }
        const double k = nsolve2 ? (double)nsolve2 : 1.0;
        printf("{\"mode\": \"nearest\", \"solves\": %lld, \"warm_sp\": %.2f, \"warm_aug\": %.2f, \"dist\": %.2f}\n",
               nsolve2, warm2.sp / k, warm2.aug / k, ndist / k);
        return 0;
    }
    Counts cold, warm;
    if (scen) {
        ll imb = 0, nsolve = 0;
        for (int p = 0; p < np; p++) {
            State st;
            for (int s = s0; s < s0 + ns && s < I.S; s++) {
                const auto ch = chains_of(I, paths[p], s);
                Flow Fs, F;
                vector<int> ca_s, ca, zs, zt;
                const ll oc = solve_cold(I, ch, Fs, ca_s, cold);
                if (st.valid) {
                    ll it = 0;
                    const ll ow = solve_warm(I, ch, st, F, ca, zs, zt, warm, &it);
                    if (ow != oc) { fprintf(stderr, "objective mismatch p=%d s=%d\n", p, s); return 1; }
                    imb += it;
                    nsolve++;
                } else {
                    cold_to_merged(I, ch, Fs, ca_s, F, ca, zs, zt);
                }
                save_state(I, ch, F, ca, zs, zt, st);
            }
        }
        const double k = nsolve ? (double)nsolve : 1.0, kc = (double)np * ns;
        printf("{\"mode\": \"scenario\", \"solves\": %lld, \"cold_sp\": %.2f, \"cold_aug\": %.2f, \"cold_phases\": %.2f, "
               "\"warm_sp\": %.2f, \"warm_aug\": %.2f, \"warm_imbalance\": %.2f}\n",
               nsolve, cold.sp / kc, cold.aug / kc, cold.phases / kc, warm.sp / k, warm.aug / k, imb / k);
        return 0;
    }
    ll imb = 0, nsolve = 0, ndiff = 0;
    for (int s = s0; s < s0 + ns && s < I.S; s++) {
        State st;
        for (int p = 0; p < np; p++) {
            const auto ch = chains_of(I, paths[p], s);
            Flow Fs, F;
            vector<int> ca_s, ca, zs, zt;
            const ll oc = solve_cold(I, ch, Fs, ca_s, cold);
            if (st.valid) {
                ll it = 0;
                const ll ow = solve_warm(I, ch, st, F, ca, zs, zt, warm, &it);
                if (ow != oc) { fprintf(stderr, "objective mismatch p=%d s=%d cold %lld warm %lld\n", p, s, oc, ow); return 1; }
                imb += it;
                if (p > 0) {
                    int dif = 0;
                    for (size_t i = 0; i < max(paths[p].size(), paths[p - 1].size()); i++) {
                        const int x = i < paths[p].size() ? paths[p][i] : -1, y = i < paths[p - 1].size() ? paths[p - 1][i] : -1;
                        dif += x != y;
                    }
                    ndiff += dif;
                }
                nsolve++;
            } else {
                cold_to_merged(I, ch, Fs, ca_s, F, ca, zs, zt);
            }
            save_state(I, ch, F, ca, zs, zt, st);
        }
    }
    const double k = nsolve ? (double)nsolve : 1.0;
    printf("{\"solves\": %lld, \"cold_sp_per_solve\": %.2f, \"cold_aug\": %.2f, \"cold_phases\": %.2f, "
           "\"warm_sp_per_solve\": %.2f, \"warm_aug\": %.2f, \"warm_imbalance\": %.2f, \"decisions_changed\": %.2f}\n",
           nsolve, cold.sp / (k + ns), cold.aug / (k + ns), cold.phases / (k + ns), warm.sp / k, warm.aug / k, imb / k,
           ndiff / k);
    return 0;
}
