// ORACLE / TEST INFRASTRUCTURE ONLY -- never linked into, loaded by or called from
// the product.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
// run it, and only as the checker or as the timed CPU baseline ("port").
//
// Clean-room CPU restatement of the reference's per-B&B-node relaxation:
//   * Network loader and DD layer order .......... /root/reference/Network.cpp:10-186
//   * Inavap::Cut key packing / lookup ............ /root/reference/Cut.h:275-282, 342-344
//   * cutToCut (zero coefficients dropped) ......... /root/reference/Cut.h:406-421
//   * RelaxedDDNew::buildTree / buildNextLayer .... /root/reference/DD.cpp:3528-3694
//   * getPathForNode / getSolution ................ /root/reference/DD.cpp:3796-3840
//   * applyFeasibilityCut ......................... /root/reference/DD.cpp:3842-3930
//   * applyOptimalityCut .......................... /root/reference/DD.cpp:3932-4023
//   * node / arc deletion and updateTree .......... /root/reference/DD.cpp:4025-4177
//   * getCutset ................................... /root/reference/DD.cpp:4179-4218
//   * NodeExplorer::process (up to the first LP) .. /root/reference/NodeExplorer.cpp:915-986
//   * RestrictedDDNew (compile, cut sweeps,
//     getMaxPath, exact cutset) ................... /root/reference/DD.cpp:3090-3505
//   * the restricted cut phases of processX3 ....... /root/reference/NodeExplorer.cpp:605-656
// Data structures are plain index arrays (no hash maps).  Pinned against the
// reference compiled from its own sources (oracle/_ref/ref_dd, see oracle/Makefile)
// and the fixtures under tests/golden/.
//
// Same CLI and text formats as oracle/ref_driver.cpp:
//   dd_oracle relax <network> <cuts> <nodes> <incumbent> <out>
//   dd_oracle time  <network> <cuts> <nodes> <incumbent> <threads> <seconds>
//   dd_oracle restricted <network> <cuts> <nodes> <incumbent> <width> <out>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <limits>
#include <map>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

namespace oracle {

static constexpr double DMIN = std::numeric_limits<double>::lowest();
static constexpr double DMAX = std::numeric_limits<double>::max();

// std::max / std::min exactly as the reference calls them (tie -> first argument).
static inline double smax(double a, double b) { return (a < b) ? b : a; }
static inline double smin(double a, double b) { return (b < a) ? b : a; }

struct Net {
    int n = 0, m = 0, S = 0;
    std::vector<int> tail, head;
    std::vector<std::vector<int>> out_arcs, in_arcs;
    std::vector<int> vbar;
    std::vector<int> order_arc;             // layer -> network arc (processingOrder[l].second)
    std::map<int, std::vector<int>> update; // stateUpdateMap (sorted sets incl. -1)
    std::vector<uint8_t> changed;           // hasStateChanged (size L+1)
    int L = 0;                              // totalLayers
};

// Network::Network + shuffleVBarNodes (Network.cpp:10-186), with the parent list
// de-duplicated (first occurrence kept), which yields the identical V-bar order.
static bool load_network(const char *path, Net &net) {
    std::ifstream in(path);
    if (!in) return false;
    int n, m, S;
    in >> n >> m >> S;
    net.n = n; net.m = m; net.S = S;
    net.tail.resize(m); net.head.resize(m);
    net.out_arcs.assign(n, {}); net.in_arcs.assign(n, {});
    for (int a = 0; a < m; a++) {
        in >> net.tail[a] >> net.head[a];
        for (int s = 0; s < S; s++) { int x; in >> x >> x >> x; }
        net.out_arcs[net.tail[a]].push_back(a);
        net.in_arcs[net.head[a]].push_back(a);
    }
    std::string tok; in >> tok;
    std::vector<int> vb; int id;
    while (in >> id) vb.push_back(id);

    // shuffleVBarNodes (Network.cpp:132-186)
    std::vector<int> rest = vb, neworder, demand;
    for (int v = 0; v < n; v++)
        if (net.out_arcs[v].size() == 1 && net.head[net.out_arcs[v][0]] == n - 1) demand.push_back(v);
    auto contains = [](const std::vector<int> &xs, int x) { return std::find(xs.begin(), xs.end(), x) != xs.end(); };
    for (int v : demand) if (contains(rest, v) && !contains(neworder, v)) neworder.push_back(v);
    for (int v : neworder) { auto it = std::find(rest.begin(), rest.end(), v); if (it != rest.end()) rest.erase(it); }
    std::vector<int> child = demand;
    int guard = 0;
    while (!rest.empty()) {
        if (++guard > n + 5) return false;  // reference would loop forever here
        std::vector<int> parents, seen(n, 0);
        for (int c : child)
            for (int a : net.in_arcs[c]) {
                int t = net.tail[a];
                if (!seen[t]) { seen[t] = 1; parents.push_back(t); }
            }
        for (int p : parents)
            if (contains(rest, p) && !contains(neworder, p)) neworder.push_back(p);
        for (int v : neworder) { auto it = std::find(rest.begin(), rest.end(), v); if (it != rest.end()) rest.erase(it); }
        child = parents;
    }
    net.vbar = neworder;

    // processingOrder / stateUpdateMap / hasStateChanged (Network.cpp:100-121)
    int i = 0;
    for (int q : net.vbar) {
        std::vector<int> st(net.out_arcs[q].begin(), net.out_arcs[q].end());
        st.push_back(-1);
        std::sort(st.begin(), st.end());
        st.erase(std::unique(st.begin(), st.end()), st.end());
        net.update.insert({i, st});  // insert: an existing key is kept
        bool first = true;
        for (int a : net.in_arcs[q]) {
            net.changed.push_back(first ? 1 : 0);
            first = false;
            net.order_arc.push_back(a);
            i++;
        }
    }
    net.changed.push_back(0);
    net.L = (int)net.order_arc.size();
    return true;
}

// Sparse cut exactly as Inavap::Cut: (key, value) list, linear first-match lookup.
struct Cut {
    int type = 0;  // 0 optimality, 1 feasibility
    double rhs = 0;
    std::vector<std::pair<uint64_t, double>> coeff;
    double get(uint64_t key) const {
        const uint64_t mask = 0xFFFFFFFFFFFFull;
        for (auto &kv : coeff)
            if ((kv.first & mask) == (key & mask)) return kv.second;
        return 0.0;
    }
};
static inline uint64_t key_of(uint64_t q, uint64_t i, uint64_t j) { return q | (i << 16) | (j << 32); }

static std::vector<Cut> read_cuts(const char *path) {
    std::ifstream in(path);
    size_t nc; in >> nc;
    std::vector<Cut> cuts(nc);
    for (auto &c : cuts) {
        std::string rhs; size_t nnz;
        in >> c.type >> rhs >> nnz;
        c.rhs = std::strtod(rhs.c_str(), nullptr);
        std::map<std::tuple<int, int, int>, double> mp;  // cutToCut walks the map in (i,q,j) order
        for (size_t k = 0; k < nnz; k++) {
            int i, q, j; std::string v;
            in >> i >> q >> j >> v;
            mp[std::make_tuple(i, q, j)] = std::strtod(v.c_str(), nullptr);
        }
        for (auto &kv : mp) {
            if (kv.second == 0) continue;
            auto [i, q, j] = kv.first;
            c.coeff.push_back({key_of((uint64_t)q, (uint64_t)i, (uint64_t)j), kv.second});
        }
    }
    return cuts;
}

struct NodeRec {
    int gl = 0;
    double lb = DMIN, ub = DMIN;
    std::vector<int16_t> states, sol;
};

static std::vector<NodeRec> read_nodes(const char *path) {
    std::ifstream in(path);
    size_t n; in >> n;
    std::vector<NodeRec> out(n);
    for (auto &r : out) {
        std::string lb, ub; size_t ns, nsol;
        in >> r.gl >> lb >> ub >> ns;
        r.lb = std::strtod(lb.c_str(), nullptr); r.ub = std::strtod(ub.c_str(), nullptr);
        r.states.resize(ns);
        for (auto &s : r.states) { int v; in >> v; s = (int16_t)v; }
        in >> nsol;
        r.sol.resize(nsol);
        for (auto &s : r.sol) { int v; in >> v; s = (int16_t)v; }
    }
    return out;
}

// ------------------------------------------------------------------ DD
struct DDNode {
    int layer = 0;                 // tree layer (nodeLayer); terminal uses 0
    int gl = 0;                    // globalLayer
    std::vector<int16_t> states;
    std::vector<int> in, out;      // arc ids, order preserved under erase
    double s2 = DMIN;              // state2
};
struct DDArc {
    int tail = 0, head = 0;
    int16_t dec = 0;
    double w = 0;
};

struct DD {
    const Net *net = nullptr;
    std::vector<DDNode> nodes;
    std::vector<DDArc> arcs;
    std::vector<std::vector<int>> tree;   // alive node ids per layer, terminal layer last
    std::vector<int16_t> root_sol;
    int start = 0;
    int terminal = 0;
    bool exact = true;
    std::vector<int> deleted;

    int new_node() { nodes.emplace_back(); return (int)nodes.size() - 1; }
    int new_arc(int t, int h, int16_t d) {
        arcs.push_back(DDArc{t, h, d, 0.0});
        int a = (int)arcs.size() - 1;
        nodes[t].out.push_back(a);
        nodes[h].in.push_back(a);
        return a;
    }

    // buildTree + buildNextLayer (DD.cpp:3528-3694)
    void build(const NodeRec &rec) {
        nodes.clear(); arcs.clear(); tree.clear(); deleted.clear();
        exact = true;
        start = rec.gl;
        root_sol = rec.sol;
        int r = new_node();
        nodes[r].states = rec.states;
        nodes[r].gl = rec.gl;
        tree.push_back({r});
        unsigned next_size = 0;
        int idx = 0;
        for (int a = start; a < net->L; a++, idx++) {
            auto it = net->update.find(a);
            if (it != net->update.end()) {
                std::vector<int16_t> st(it->second.begin(), it->second.end());
                for (int id : tree[idx]) nodes[id].states = st;
                next_size = (unsigned)(tree[idx].size() * st.size());
            }
            const std::vector<int> cur = tree[idx];
            unsigned gfront = (unsigned)nodes[cur.front()].gl;
            if (next_size >= 120u && gfront < (unsigned)(net->L - 5)) {
                exact = false;
                int mnode = new_node();
                std::vector<int16_t> uni;
                for (int p : cur)
                    for (int16_t s : nodes[p].states) {
                        new_arc(p, mnode, s);
                        uni.push_back(s);
                    }
                std::sort(uni.begin(), uni.end());
                uni.erase(std::unique(uni.begin(), uni.end()), uni.end());
                next_size = (unsigned)uni.size();
                nodes[mnode].layer = nodes[cur[0]].layer + 1;
                nodes[mnode].gl = nodes[cur[0]].gl + 1;
                nodes[mnode].states = uni;
                tree.push_back({mnode});
            } else {
                std::vector<int> nxt;
                next_size = 0;
                for (int p : cur) {
                    const std::vector<int16_t> pst = nodes[p].states;
                    for (int16_t s : pst) {
                        std::vector<int16_t> cst;
                        for (int16_t x : pst) if (s == -1 || x != s) cst.push_back(x);
                        next_size += (unsigned)cst.size();
                        int c = new_node();
                        nodes[c].layer = nodes[p].layer + 1;
                        nodes[c].gl = nodes[p].gl + 1;
                        nodes[c].states = std::move(cst);
                        new_arc(p, c, s);
                        nxt.push_back(c);
                    }
                }
                tree.push_back(std::move(nxt));
            }
        }
        terminal = new_node();
        for (int p : tree[idx]) {
            int a = new_arc(p, terminal, 1);
            arcs[a].w = DMAX;
        }
        tree.push_back({terminal});
    }

    double coef_for(const Cut &cut, size_t layer_idx, int16_t dec) const {
        int na = net->order_arc[layer_idx];
        uint64_t i = (uint64_t)net->tail[na], q = (uint64_t)net->head[na];
        uint64_t j = (uint64_t)net->head[dec];
        return cut.get(key_of(q, i, j));
    }

    // the shared sweep of applyFeasibilityCut / applyOptimalityCut (DD.cpp:3846-3878, 3936-3973)
    void sweep(const Cut &cut) {
        size_t i = 0;
        double v = cut.rhs;
        for (int16_t d : root_sol) {
            if (d == -1) { i++; continue; }
            v = v + coef_for(cut, i, d);
            i++;
        }
        nodes[tree[0][0]].s2 = v;
        for (size_t layer = 1; layer + 1 < tree.size(); layer++) {
            size_t li = i++;
            for (int id : tree[layer]) {
                double ns = DMIN;
                for (int a : nodes[id].in) {
                    DDArc &arc = arcs[a];
                    const DDNode &par = nodes[arc.tail];
                    if (arc.dec != -1) {
                        arc.w = coef_for(cut, li, arc.dec);
                        ns = smax(par.s2 + arc.w, ns);
                    } else {
                        ns = smax(ns, par.s2);
                    }
                }
                nodes[id].s2 = ns;
            }
        }
    }

    void erase_arc(int a) {
        auto &o = nodes[arcs[a].tail].out;
        o.erase(std::remove(o.begin(), o.end(), a), o.end());
        auto &in = nodes[arcs[a].head].in;
        in.erase(std::remove(in.begin(), in.end(), a), in.end());
    }

    void bottom_up(int id) {  // DD.cpp:4081-4099
        std::vector<int> ins = nodes[id].in;
        for (int a : ins) {
            int p = arcs[a].tail;
            erase_arc(a);
            if (nodes[p].out.empty()) bottom_up(p);
        }
        deleted.push_back(id);
    }

    void remove_last_layer_node(int id) {  // removeNode (DD.cpp:4040-4059)
        erase_arc(nodes[id].out.back());
        std::vector<int> ins = nodes[id].in;
        for (int a : ins) {
            int p = arcs[a].tail;
            erase_arc(a);
            if (nodes[p].out.empty()) bottom_up(p);
        }
        deleted.push_back(id);
    }

    void update_tree() {  // DD.cpp:4121-4153 (ids grow with layer; drop deleted ids)
        std::vector<char> dead(nodes.size(), 0);
        for (int id : deleted) dead[id] = 1;
        for (auto &layer : tree) {
            std::vector<int> keep;
            for (int id : layer) if (!dead[id]) keep.push_back(id);
            layer.swap(keep);
        }
        deleted.clear();
    }

    // width-1 arc pruning shared by both cut types (DD.cpp:3895-3928, 3987-4021).
    // Returns false when some width-1 layer loses every incoming arc.
    bool prune(size_t first, size_t end, double thresh) {
        size_t llayer = tree.size() - 2;
        double maxState = DMIN;
        for (int id : tree[llayer]) maxState = smax(maxState, nodes[id].s2);
        std::vector<int> rm;
        for (size_t layer = first; layer < end; layer++) {
            if (tree[layer].size() != 1) continue;
            size_t total = 0, pruned = 0;
            double gain = maxState - nodes[tree[layer][0]].s2;
            for (int id : tree[layer - 1])
                for (int a : nodes[id].out) {
                    const DDArc &arc = arcs[a];
                    if ((nodes[arc.tail].s2 + arc.w + gain) <= thresh) { rm.push_back(a); pruned++; }
                    total++;
                }
            if (total == pruned) return false;
        }
        for (int a : rm) erase_arc(a);
        return true;
    }

    bool apply_feasibility(const Cut &cut) {  // DD.cpp:3842-3930
        sweep(cut);
        size_t llayer = tree.size() - 2;
        std::vector<int> rm;
        for (int id : tree[llayer]) if (nodes[id].s2 < -0.01) rm.push_back(id);
        if (rm.size() == tree[llayer].size()) return false;
        if (!rm.empty()) {
            for (int id : rm) remove_last_layer_node(id);
            update_tree();
        }
        if (!exact) return prune(1, llayer, -0.01);
        return true;
    }

    double apply_optimality(const Cut &cut, double optimal) {  // DD.cpp:3932-4023
        sweep(cut);
        double term = DMIN;
        for (int a : nodes[terminal].in) {
            DDArc &arc = arcs[a];
            arc.w = smin(arc.w, nodes[arc.tail].s2);
            term = smax(term, arc.w);
        }
        nodes[terminal].s2 = term;
        if (term <= optimal) return term;
        if (!exact) {
            size_t llayer = tree.size() - 2;
            if (!prune(3, llayer - 1, optimal - 0.01)) return DMIN;
        }
        return term;
    }

    std::vector<int16_t> path_for(int id) const {  // DD.cpp:3796-3820
        const DDNode *cur = &nodes[id];
        std::vector<int16_t> path;
        while (cur->layer) {
            const DDNode *pp = &nodes[arcs[cur->in[0]].tail];
            for (int a : cur->in) {
                const DDArc &arc = arcs[a];
                const DDNode *par = &nodes[arc.tail];
                if ((par->s2 + arc.w) == cur->s2) { path.push_back(arc.dec); pp = par; break; }
            }
            cur = pp;
        }
        std::vector<int16_t> sol(root_sol.begin(), root_sol.end());
        sol.insert(sol.end(), path.rbegin(), path.rend());
        return sol;
    }

    std::vector<int16_t> solution() const {  // DD.cpp:3825-3840
        int best = 0;
        double bw = DMIN;
        for (int a : nodes[terminal].in)
            if (arcs[a].w > bw) { bw = arcs[a].w; best = arcs[a].tail; }
        return path_for(best);
    }

    std::vector<NodeRec> cutset(double ub) const {  // DD.cpp:4179-4218
        size_t layer = 3;
        while (tree[layer].size() != 1) layer++;
        int gl = nodes[tree[layer][0]].gl;
        std::vector<NodeRec> out;
        bool changed = net->changed[gl] != 0;
        std::vector<int16_t> upd;
        if (changed) {
            auto &st = net->update.at(gl);
            upd.assign(st.begin(), st.end());
        }
        for (int id : tree[layer - 1]) {
            std::vector<int16_t> part = path_for(id);
            for (int a : nodes[id].out) {
                int16_t d = arcs[a].dec;
                NodeRec c;
                c.sol = part;
                c.sol.push_back(d);
                if (changed) c.states = upd;
                else {
                    c.states = nodes[id].states;
                    if (d != -1) c.states.erase(std::remove(c.states.begin(), c.states.end(), d), c.states.end());
                }
                c.lb = DMIN; c.ub = ub; c.gl = gl;
                out.push_back(std::move(c));
            }
        }
        return out;
    }
};

struct Result {
    int status = 0, exact = 0;
    double lb = DMIN, ub = DMIN;
    std::vector<NodeRec> children;
    std::vector<int16_t> path;
    size_t dd_nodes = 0, dd_arcs = 0, dd_layers = 0;
};

// NodeExplorer::process (NodeExplorer.cpp:915-986) up to the first subproblem.
static Result process(DD &dd, const NodeRec &nd, double inc, const std::vector<Cut> &cuts) {
    Result r;
    double ub = nd.ub;
    dd.build(nd);
    r.dd_layers = dd.tree.size();
    for (auto &layer : dd.tree) {
        r.dd_nodes += layer.size();
        for (int id : layer) r.dd_arcs += dd.nodes[id].in.size();
    }
    r.exact = dd.exact ? 1 : 0;
    for (size_t k = cuts.size(); k-- > 0;) {
        if (cuts[k].type != 1) continue;
        if (!dd.apply_feasibility(cuts[k])) { r.status = 1; return r; }
    }
    for (size_t k = cuts.size(); k-- > 0;) {
        if (cuts[k].type != 0) continue;
        double v = dd.apply_optimality(cuts[k], inc);
        ub = r.exact ? v : smin(v, ub);
        if (ub <= inc) { r.status = 2; return r; }
    }
    if (r.exact) { r.status = 3; r.ub = ub; r.path = dd.solution(); return r; }
    r.status = 0; r.lb = DMIN; r.ub = ub;
    r.children = dd.cutset(ub);
    return r;
}

static void write_node(FILE *f, const NodeRec &nd) {
    std::fprintf(f, "%u %a %a %zu", (unsigned)nd.gl, nd.lb, nd.ub, nd.states.size());
    for (auto s : nd.states) std::fprintf(f, " %d", (int)s);
    std::fprintf(f, " %zu", nd.sol.size());
    for (auto s : nd.sol) std::fprintf(f, " %d", (int)s);
    std::fprintf(f, "\n");
}

static void write_result(FILE *f, const Result &r) {
    std::fprintf(f, "R %d %d %a %a %zu %zu %zu %zu %zu\n", r.status, r.exact, r.lb, r.ub, r.children.size(),
                 r.path.size(), r.dd_nodes, r.dd_arcs, r.dd_layers);
    if (!r.path.empty()) {
        for (size_t k = 0; k < r.path.size(); k++) std::fprintf(f, "%s%d", k ? " " : "", (int)r.path[k]);
        std::fprintf(f, "\n");
    }
    for (auto &c : r.children) write_node(f, c);
}

// ------------------------------------------------------------------ restricted DD
// RestrictedDDNew (DD.cpp:3090-3505): a tree.  Layers expand exactly -- each node's states
// in reverse stored order, child states = parent minus the decision (-1 keeps all) --
// until a layer would exceed `width` nodes: that layer keeps its first `width` children
// and from then on every node gets one child, the decision its largest state
// (buildRestrictedLayer, DD.cpp:3161-3220).  Only last-layer nodes are ever removed.
struct RDD {
    const Net *net = nullptr;
    unsigned width = 128;
    struct RNode { int parent = -1; int16_t dec = 0; int gl = 0; int layer = 0; std::vector<int16_t> states; double s2 = 0; };
    std::vector<RNode> nodes;
    std::vector<std::vector<int>> tree;      // node ids per layer (no terminal layer)
    std::vector<int> term;                   // last-layer nodes with a terminal arc, in order
    std::vector<double> tw;                  // terminal arc weight per node id (only leaves)
    std::vector<int16_t> root_sol;
    bool exact = true;
    size_t exact_layer = 0;

    void compile(const NodeRec &rec) {      // DD.cpp:3090-3159
        nodes.clear(); tree.clear(); term.clear();
        root_sol = rec.sol;
        RNode root; root.gl = rec.gl; root.states = rec.states; root.layer = 0;
        nodes.push_back(root);
        tree.push_back({0});
        exact = true;
        exact_layer = 0;
        for (int a = rec.gl; a < net->L; a++) {
            std::vector<int> &cur = tree.back();
            auto it = net->update.find(a);
            if (it != net->update.end()) {
                std::vector<int16_t> st(it->second.begin(), it->second.end());
                for (int id : cur) nodes[id].states = st;
            }
            std::vector<int> nxt;
            const std::vector<int> curc = cur;
            if (exact) {
                size_t count = 0;
                bool stop = false;
                for (int id : curc) {
                    const std::vector<int16_t> st = nodes[id].states;
                    for (size_t r = st.size(); r-- > 0;) {
                        if (count >= width) { exact = false; stop = true; break; }
                        RNode ch;
                        ch.parent = id; ch.dec = st[r];
                        ch.states = st;
                        if (ch.dec != -1) ch.states.erase(std::find(ch.states.begin(), ch.states.end(), ch.dec));
                        ch.gl = nodes[id].gl + 1; ch.layer = nodes[id].layer + 1;
                        nodes.push_back(ch);
                        nxt.push_back((int)nodes.size() - 1);
                        count++;
                    }
                    if (stop) break;
                }
            } else {
                for (int id : curc) {
                    const std::vector<int16_t> &st = nodes[id].states;
                    RNode ch;
                    ch.parent = id;
                    ch.dec = *std::max_element(st.begin(), st.end());
                    ch.states = st;
                    if (ch.dec != -1) ch.states.erase(std::find(ch.states.begin(), ch.states.end(), ch.dec));
                    ch.gl = nodes[id].gl + 1; ch.layer = nodes[id].layer + 1;
                    nodes.push_back(ch);
                    nxt.push_back((int)nodes.size() - 1);
                }
            }
            if (exact) exact_layer++;
            tree.push_back(nxt);
        }
        term = tree.back();
        tw.assign(nodes.size(), DMAX);
    }

    std::vector<int16_t> path_of(int id) const {   // getPathForNode (DD.cpp:3262-3277)
        std::vector<int16_t> rev;
        while (nodes[id].layer) { rev.push_back(nodes[id].dec); id = nodes[id].parent; }
        std::vector<int16_t> sol(root_sol.begin(), root_sol.end());
        sol.insert(sol.end(), rev.rbegin(), rev.rend());
        return sol;
    }

    std::vector<NodeRec> cutset() const {          // getExactCutSet (DD.cpp:3279-3288)
        std::vector<NodeRec> out;
        for (int id : tree[exact_layer]) {
            NodeRec r;
            r.gl = nodes[id].gl; r.lb = DMIN; r.ub = DMIN;
            r.states = nodes[id].states;
            r.sol = path_of(id);
            out.push_back(r);
        }
        return out;
    }

    double coef_for(const Cut &cut, size_t layer_idx, int16_t dec) const {
        int na = net->order_arc[layer_idx];
        uint64_t i = (uint64_t)net->tail[na], q = (uint64_t)net->head[na];
        return cut.get(key_of(q, i, (uint64_t)net->head[dec]));
    }

    void sweep(const Cut &cut) {                   // DD.cpp:3346-3374 / 3431-3461
        size_t i = 0;
        double v = cut.rhs;
        for (int16_t d : root_sol) {
            if (d == -1) { i++; continue; }
            v = v + coef_for(cut, i, d);
            i++;
        }
        nodes[0].s2 = v;
        for (size_t layer = 1; layer < tree.size(); layer++) {
            size_t li = i++;
            const std::vector<int> &ids = (layer + 1 == tree.size()) ? term : tree[layer];
            for (int id : ids) {
                RNode &nd = nodes[id];
                const double ps = nodes[nd.parent].s2;
                nd.s2 = nd.dec != -1 ? coef_for(cut, li, nd.dec) + ps : ps;
            }
        }
    }

    bool apply_feasibility(const Cut &cut) {      // DD.cpp:3340-3423
        sweep(cut);
        if (term.empty()) return false;
        std::vector<int> keep;
        for (int id : term)
            if (!(nodes[id].s2 < -0.5)) keep.push_back(id);
        term = keep;
        return !term.empty();
    }

    double apply_optimality(const Cut &cut) {     // DD.cpp:3425-3505
        sweep(cut);
        double t = DMIN;
        for (int id : term) {
            tw[id] = smin(tw[id], nodes[id].s2);
            t = smax(t, tw[id]);
        }
        return t;
    }

    std::vector<int16_t> max_path() const {        // getMaxPath (DD.cpp:3290-3305)
        int best = 0;
        double bw = DMIN;
        for (int id : term)
            if (tw[id] > bw) { bw = tw[id]; best = id; }
        return path_of(best);
    }
};

static void restricted(FILE *f, const Net &net, const NodeRec &nd, double optimalLB, const std::vector<Cut> &cuts,
                       unsigned width) {
    RDD dd; dd.net = &net; dd.width = width;
    dd.compile(nd);
    double lowerBound = nd.lb;
    int status = 0;
    for (size_t k = cuts.size(); k-- > 0 && status == 0;)
        if (cuts[k].type == 1 && !dd.apply_feasibility(cuts[k])) status = 1;
    for (size_t k = cuts.size(); k-- > 0 && status == 0;) {
        if (cuts[k].type != 0) continue;
        lowerBound = dd.apply_optimality(cuts[k]);
        if (lowerBound <= optimalLB) status = 2;
    }
    std::vector<int16_t> path;
    if (status == 0) path = dd.max_path();
    std::vector<NodeRec> cs;
    if (!dd.exact) cs = dd.cutset();
    std::fprintf(f, "Q %d %d %a %zu %zu\n", status, dd.exact ? 1 : 0, lowerBound, cs.size(), path.size());
    if (!path.empty()) {
        for (size_t k = 0; k < path.size(); k++) std::fprintf(f, "%s%d", k ? " " : "", (int)path[k]);
        std::fprintf(f, "\n");
    }
    for (auto &c : cs) write_node(f, c);
}

}  // namespace oracle

int main(int argc, char **argv) {
    using namespace oracle;
    if (argc < 2) return 2;
    std::string mode = argv[1];
    if (mode == "widths" && argc == 4) {
        // diagnostic: tree layer widths (and merged in-arc counts) of each node's DD
        Net net;
        if (!load_network(argv[2], net)) return 2;
        auto nodes = read_nodes(argv[3]);
        DD dd; dd.net = &net;
        for (auto &nd : nodes) {
            dd.build(nd);
            for (size_t k = 0; k + 1 < dd.tree.size(); k++) {
                int id = dd.tree[k][0];
                std::printf("%zu%s ", dd.tree[k].size(), (dd.tree[k].size() == 1 && dd.nodes[id].in.size() > 1) ? "m" : "");
            }
            std::printf("\n");
        }
        return 0;
    }
    if (mode == "restricted" && argc == 8) {
        Net net;
        if (!load_network(argv[2], net)) return 2;
        auto cuts = read_cuts(argv[3]);
        auto nodes = read_nodes(argv[4]);
        double inc = std::strtod(argv[5], nullptr);
        unsigned width = (unsigned)std::strtoul(argv[6], nullptr, 10);
        FILE *f = std::fopen(argv[7], "w");
        std::fprintf(f, "%zu\n", nodes.size());
        for (auto &nd : nodes) restricted(f, net, nd, inc, cuts, width);
        std::fclose(f);
        return 0;
    }
    if (mode == "refine" && argc == 8) {
        // process() then the refinement loop (NodeExplorer.cpp:957-969) fed with <extra>
        Net net;
        if (!load_network(argv[2], net)) return 2;
        auto cuts = read_cuts(argv[3]);
        auto nodes = read_nodes(argv[4]);
        double inc = std::strtod(argv[5], nullptr);
        auto extra = read_cuts(argv[6]);
        DD dd; dd.net = &net;
        FILE *f = std::fopen(argv[7], "w");
        std::fprintf(f, "%zu\n", nodes.size());
        for (auto &nd : nodes) {
            Result r = process(dd, nd, inc, cuts);
            if (r.status == 3) {
                double ub = r.ub;
                for (auto &c : extra) {
                    if (c.type == 1) {
                        if (!dd.apply_feasibility(c)) { r.status = 1; break; }
                    } else {
                        ub = dd.apply_optimality(c, inc);
                        if (ub <= inc) { r.status = 2; break; }
                    }
                }
                r.path.clear();
                if (r.status == 3) { r.ub = ub; r.path = dd.solution(); }
                else { r.ub = DMIN; r.lb = DMIN; }
            }
            write_result(f, r);
        }
        std::fclose(f);
        return 0;
    }
    if ((mode == "relax" && argc == 7) || (mode == "time" && argc == 8)) {
        Net net;
        if (!load_network(argv[2], net)) { std::fprintf(stderr, "bad network\n"); return 2; }
        auto cuts = read_cuts(argv[3]);
        auto nodes = read_nodes(argv[4]);
        double inc = std::strtod(argv[5], nullptr);
        if (mode == "relax") {
            DD dd; dd.net = &net;
            FILE *f = std::fopen(argv[6], "w");
            std::fprintf(f, "%zu\n", nodes.size());
            for (auto &nd : nodes) write_result(f, process(dd, nd, inc, cuts));
            std::fclose(f);
            return 0;
        }
        int threads = std::atoi(argv[6]);
        double budget = std::atof(argv[7]);
        std::atomic<size_t> next{0}, done{0};
        std::atomic<bool> stop{false};
        auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> pool;
        for (int t = 0; t < threads; t++)
            pool.emplace_back([&]() {
                DD dd; dd.net = &net;
                for (;;) {
                    if (stop.load(std::memory_order_relaxed)) break;
                    size_t k = next.fetch_add(1);
                    if (k >= nodes.size()) break;
                    Result r = process(dd, nodes[k], inc, cuts);
                    (void)r;
                    done.fetch_add(1);
                    double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                    if (el > budget) stop.store(true);
                }
            });
        for (auto &th : pool) th.join();
        double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::printf("{\"relaxations\": %zu, \"seconds\": %.6f, \"threads\": %d}\n", done.load(), el, threads);
        return 0;
    }
    return 2;
}
