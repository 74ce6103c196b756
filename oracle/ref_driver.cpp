// ORACLE / TEST INFRASTRUCTURE ONLY -- never linked into the product.
//
// Driver around the reference's own RelaxedDDNew (/root/reference/DD.cpp:3507-4230),
// Network (/root/reference/Network.cpp:10-186) and Inavap::Cut / cutToCut
// (/root/reference/Cut.h:185-446), compiled from the sources where they lie by
// oracle/Makefile into oracle/_ref/ref_dd.  Nothing of the reference is copied here:
// this file only includes the reference headers and drives them.
//
// The per-node control flow restates Inavap::NodeExplorer::process
// (/root/reference/NodeExplorer.cpp:915-986) up to the first subproblem call
// (NodeExplorer.cpp:957), because grb.cpp needs Gurobi, which is absent.  For an
// exact tree the driver reports the argmax path the reference would hand to
// GuroSolver::solveSubProblem (status 3 = "needs LP").
//
// Usage:
//   ref_dd relax  <network> <cuts> <nodes> <incumbent-hex> <out>
//   ref_dd bfs    <network> <cuts> <incumbent-hex> <max-nodes> <out-nodes>
//   ref_dd time   <network> <cuts> <nodes> <incumbent-hex> <threads> <seconds>
//   ref_dd relaxp <network> <cuts> <nodes> <incumbent-hex> <threads> <out>
//                  (every node, static work queue over threads; timing JSON on stdout,
//                   results in node order as "relax" writes them: CPU baseline + parity)
//   ref_dd apply  <network> <cuts> <nodes> <out>     (per-cut trace, exact/non-exact alike)
//   ref_dd api    <network> <cuts> <nodes> <incumbent-hex> <out>
//                  (RelaxedDDNew call by call: values, getSolution, getCutset)
//   ref_dd restricted <network> <cuts> <nodes> <incumbent-hex> <width> <out>
//                  (Inavap::RestrictedDDNew, DD.cpp:3090-3505, under the cut phases of
//                   NodeExplorer::processX3, NodeExplorer.cpp:605-656)
//
// File formats (text; doubles as C99 hex floats, "%a"):
//   cuts : <ncuts>\n then per cut "<type 0=opt 1=feas> <rhs> <nnz>\n" and nnz lines "<i> <q> <j> <val>"
//          (or a binary dense-row pool, file name *.bin: read_cuts_bin)
//          (insertion order; the Container is a LIFO list, Cut.h:456-485, so application is newest first)
//   nodes: <n>\n then per node "<gl> <lb> <ub> <ns> s... <nsol> d..."
#include "DD.h"
#include "Network.h"
#include "Cut.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fstream>
#include <iostream>
#include <memory>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

using Inavap::DOUBLE_MAX;
using Inavap::DOUBLE_MIN;

struct PoolCut {
    int type;  // 0 = optimality, 1 = feasibility
    Inavap::Cut cut;
};

static double parse_double(const std::string &s) { return std::strtod(s.c_str(), nullptr); }

// Binary pool (large pools read back from a running device search, oracle/bnb_parity.py):
// int64 n_cuts, int64 n_slots, uint64 slot keys [n_slots] (getKey(q,i,j)), int32 types [n_cuts],
// f64 rhs [n_cuts], f64 dense rows [n_cuts][n_slots]; non-zero slots become (i,q,j) entries.
static std::vector<PoolCut> read_cuts_bin(const std::string &path) {
    FILE *f = std::fopen(path.c_str(), "rb");
    if (!f) { std::cerr << "cannot open " << path << "\n"; std::exit(2); }
    int64_t nc = 0, ns = 0;
    if (std::fread(&nc, 8, 1, f) != 1 || std::fread(&ns, 8, 1, f) != 1) std::exit(2);
    std::vector<uint64_t> keys((size_t)ns);
    std::vector<int32_t> types((size_t)nc);
    std::vector<double> rhs((size_t)nc), row((size_t)ns);
    if (std::fread(keys.data(), 8, (size_t)ns, f) != (size_t)ns || std::fread(types.data(), 4, (size_t)nc, f) != (size_t)nc ||
        std::fread(rhs.data(), 8, (size_t)nc, f) != (size_t)nc)
        std::exit(2);
    std::vector<PoolCut> cuts;
    cuts.reserve((size_t)nc);
    for (int64_t c = 0; c < nc; c++) {
        if (std::fread(row.data(), 8, (size_t)ns, f) != (size_t)ns) std::exit(2);
        CutCoefficients coeff;
        for (int64_t s = 0; s < ns; s++) {
            if (row[(size_t)s] == 0.0) continue;
            const uint64_t k = keys[(size_t)s];
            coeff[std::make_tuple((int)((k >> 16) & 0xFFFF), (int)(k & 0xFFFF), (int)((k >> 32) & 0xFFFF))] = row[(size_t)s];
        }
        ::Cut legacy{types[(size_t)c] ? FEASIBILITY : OPTIMALITY, rhs[(size_t)c], coeff};
        cuts.push_back(PoolCut{types[(size_t)c], Inavap::cutToCut(legacy, nullptr)});
    }
    std::fclose(f);
    return cuts;
}

static std::vector<PoolCut> read_cuts(const std::string &path) {
    if (path.size() > 4 && path.compare(path.size() - 4, 4, ".bin") == 0) return read_cuts_bin(path);
    std::ifstream in(path);
    if (!in) { std::cerr << "cannot open " << path << "\n"; std::exit(2); }
    size_t n;
    in >> n;
    std::vector<PoolCut> cuts;
    cuts.reserve(n);
    for (size_t c = 0; c < n; c++) {
        int type; std::string rhs_s; size_t nnz;
        in >> type >> rhs_s >> nnz;
        CutCoefficients coeff;
        for (size_t k = 0; k < nnz; k++) {
            int i, q, j; std::string v;
            in >> i >> q >> j >> v;
            coeff[std::make_tuple(i, q, j)] = parse_double(v);
        }
        ::Cut legacy{type ? FEASIBILITY : OPTIMALITY, parse_double(rhs_s), coeff};
        cuts.push_back(PoolCut{type, Inavap::cutToCut(legacy, nullptr)});
    }
    return cuts;
}

static std::vector<Inavap::Node> read_nodes(const std::string &path) {
    std::ifstream in(path);
    if (!in) { std::cerr << "cannot open " << path << "\n"; std::exit(2); }
    size_t n;
    in >> n;
    std::vector<Inavap::Node> nodes;
    for (size_t k = 0; k < n; k++) {
        int gl; std::string lb, ub; size_t ns, nsol;
        in >> gl >> lb >> ub >> ns;
        std::vector<int16_t> st(ns);
        for (auto &s : st) { int v; in >> v; s = (int16_t)v; }
        in >> nsol;
        std::vector<int16_t> sol(nsol);
        for (auto &s : sol) { int v; in >> v; s = (int16_t)v; }
        nodes.emplace_back(std::move(st), std::move(sol), parse_double(lb), parse_double(ub), (uint16_t)gl);
    }
    return nodes;
}

static void write_node(FILE *f, const Inavap::Node &nd) {
    std::fprintf(f, "%u %a %a %zu", (unsigned)nd.globalLayer, nd.lb, nd.ub, nd.states.size());
    for (auto s : nd.states) std::fprintf(f, " %d", (int)s);
    std::fprintf(f, " %zu", nd.solutionVector.size());
    for (auto s : nd.solutionVector) std::fprintf(f, " %d", (int)s);
    std::fprintf(f, "\n");
}

struct Result {
    int status = 0;        // 0 SUCCESS, 1 PRUNED_BY_FEASIBILITY_CUT, 2 PRUNED_BY_OPTIMALITY_CUT, 3 NEEDS_LP (exact)
    int exact = 0;
    double lb = DOUBLE_MIN, ub = DOUBLE_MIN;
    std::vector<Inavap::Node> children;
    std::vector<int16_t> path;   // exact trees: getSolution() after the pool sweeps
    size_t dd_nodes = 0, dd_arcs = 0, dd_layers = 0;
    size_t cuts_applied = 0;
};

// Restatement of NodeExplorer::process (NodeExplorer.cpp:915-986) over the
// reference DD, stopping at the first subproblem solve.
static Result process(Inavap::RelaxedDDNew &dd, const Inavap::Node &node, double optimalLB,
                      const std::vector<PoolCut> &cuts) {
    Result r;
    double upperBound = node.ub;
    dd.buildTree(node);
    r.dd_layers = dd.tree.size();
    for (auto &layer : dd.tree) {
        r.dd_nodes += layer.size();
        for (auto id : layer) r.dd_arcs += dd.nodes.at(id).incomingArcs.size();
    }
    r.exact = dd.isTreeExact() ? 1 : 0;

    // Feasibility list then optimality list, each newest -> oldest (Container LIFO).
    for (size_t k = cuts.size(); k-- > 0;) {
        if (cuts[k].type != 1) continue;
        r.cuts_applied++;
        if (!dd.applyFeasibilityCut(cuts[k].cut)) { r.status = 1; return r; }
    }
    for (size_t k = cuts.size(); k-- > 0;) {
        if (cuts[k].type != 0) continue;
        r.cuts_applied++;
        double v = dd.applyOptimalityCut(cuts[k].cut, optimalLB, upperBound);
        if (r.exact) upperBound = v;
        else upperBound = std::min(v, upperBound);
        if (upperBound <= optimalLB) { r.status = 2; return r; }
    }
    if (r.exact) {
        r.status = 3;
        r.ub = upperBound;
        r.path = dd.getSolution();
        return r;
    }
    r.status = 0;
    r.lb = DOUBLE_MIN;
    r.ub = upperBound;
    r.children = dd.getCutset(upperBound);
    return r;
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

// The restricted-DD half of NodeExplorer::processX3 (NodeExplorer.cpp:605-656): compile a
// width-limited restricted DD (RestrictedDDNew::compile, DD.cpp:3090-3159), apply the pool's
// feasibility cuts then its optimality cuts (each list newest first; the first false /
// the first bound <= optimalLB ends the node), then the max path (getSolution ->
// getMaxPath, DD.cpp:3290-3305).  status 0 = ok, 1 = infeasible, 2 = bound <= optimalLB.
static void restricted(FILE *f, const std::shared_ptr<Network> &np, const Inavap::Node &nd, double optimalLB,
                       const std::vector<PoolCut> &cuts, unsigned width) {
    Inavap::RestrictedDDNew dd{np, width};
    auto cs = dd.compile(nd);
    int exact = dd.isTreeExact() ? 1 : 0;
    double lowerBound = nd.lb;
    int status = 0;
    for (size_t k = cuts.size(); k-- > 0 && status == 0;) {
        if (cuts[k].type != 1) continue;
        if (!dd.applyFeasibilityCut(cuts[k].cut)) status = 1;
    }
    for (size_t k = cuts.size(); k-- > 0 && status == 0;) {
        if (cuts[k].type != 0) continue;
        lowerBound = dd.applyOptimalityCut(cuts[k].cut);
        if (lowerBound <= optimalLB) status = 2;
    }
    std::vector<int16_t> path;
    if (status == 0) path = dd.getSolution();
    size_t nc = cs ? cs->size() : 0;
    std::fprintf(f, "Q %d %d %a %zu %zu\n", status, exact, lowerBound, nc, path.size());
    if (!path.empty()) {
        for (size_t k = 0; k < path.size(); k++) std::fprintf(f, "%s%d", k ? " " : "", (int)path[k]);
        std::fprintf(f, "\n");
    }
    if (cs)
        for (auto &c : *cs) write_node(f, c);
}

int main(int argc, char **argv) {
    if (argc < 2) { std::cerr << "usage: see header\n"; return 2; }
    std::string mode = argv[1];
    if (mode == "relax" && argc == 7) {
        Network net{argv[2]};
        auto cuts = read_cuts(argv[3]);
        auto nodes = read_nodes(argv[4]);
        double inc = parse_double(argv[5]);
        Inavap::RelaxedDDNew dd{&net};
        FILE *f = std::fopen(argv[6], "w");
        std::fprintf(f, "%zu\n", nodes.size());
        for (auto &nd : nodes) write_result(f, process(dd, nd, inc, cuts));
        std::fclose(f);
        return 0;
    }
    if (mode == "bfs" && argc == 7) {
        // Frontier generation: BFS over cutset children from the root node
        // (DDSolver::startSolver builds the root with Node{} and getCutset(DOUBLE_MAX),
        // DDSolver.cpp:788-791), relaxing every popped node under the pool.
        Network net{argv[2]};
        auto cuts = read_cuts(argv[3]);
        double inc = parse_double(argv[4]);
        size_t maxn = std::strtoul(argv[5], nullptr, 10);
        Inavap::RelaxedDDNew dd{&net};
        dd.buildTree(Inavap::Node{});
        std::deque<Inavap::Node> q;
        for (auto &c : dd.getCutset(DOUBLE_MAX)) q.push_back(c);
        std::vector<Inavap::Node> out;
        while (!q.empty() && out.size() < maxn) {
            Inavap::Node nd = q.front();
            q.pop_front();
            out.push_back(nd);
            if (q.size() + out.size() >= maxn) continue;
            Result r = process(dd, nd, inc, cuts);
            if (r.status == 0)
                for (auto &c : r.children) q.push_back(c);
        }
        while (!q.empty() && out.size() < maxn) { out.push_back(q.front()); q.pop_front(); }
        FILE *f = std::fopen(argv[6], "w");
        std::fprintf(f, "%zu\n", out.size());
        for (auto &nd : out) write_node(f, nd);
        std::fclose(f);
        return 0;
    }
    if (mode == "dfs" && argc == 7) {
        // Frontier generation in the solver's own order: LIFO over cutset children
        // (workers pop their private queue LIFO, DDSolver.cpp:703; children are pushed
        // in cutset order), so the walk dives to exact leaves quickly.
        Network net{argv[2]};
        auto cuts = read_cuts(argv[3]);
        double inc = parse_double(argv[4]);
        size_t maxn = std::strtoul(argv[5], nullptr, 10);
        Inavap::RelaxedDDNew dd{&net};
        dd.buildTree(Inavap::Node{});
        std::vector<Inavap::Node> st;
        auto root = dd.getCutset(DOUBLE_MAX);
        for (size_t k = root.size(); k-- > 0;) st.push_back(root[k]);
        std::vector<Inavap::Node> out;
        while (!st.empty() && out.size() < maxn) {
            Inavap::Node nd = st.back();
            st.pop_back();
            out.push_back(nd);
            Result r = process(dd, nd, inc, cuts);
            if (r.status == 0)
                for (auto &c : r.children) st.push_back(c);
        }
        FILE *f = std::fopen(argv[6], "w");
        std::fprintf(f, "%zu\n", out.size());
        for (auto &nd : out) write_node(f, nd);
        std::fclose(f);
        return 0;
    }
    if (mode == "refine" && argc == 8) {
        // process() up to the first subproblem, then the refinement loop of
        // NodeExplorer.cpp:957-969 fed with the cuts of <extra> in order (instead of
        // Gurobi's): each is applied to the exact DD, status/ub updated, path recomputed.
        Network net{argv[2]};
        auto cuts = read_cuts(argv[3]);
        auto nodes = read_nodes(argv[4]);
        double inc = parse_double(argv[5]);
        auto extra = read_cuts(argv[6]);
        Inavap::RelaxedDDNew dd{&net};
        FILE *f = std::fopen(argv[7], "w");
        std::fprintf(f, "%zu\n", nodes.size());
        for (auto &nd : nodes) {
            Result r = process(dd, nd, inc, cuts);
            if (r.status == 3) {
                double ub = r.ub;
                for (auto &c : extra) {
                    if (c.type == 1) {
                        if (!dd.applyFeasibilityCut(c.cut)) { r.status = 1; break; }
                    } else {
                        ub = dd.applyOptimalityCut(c.cut, inc, ub);
                        if (ub <= inc) { r.status = 2; break; }
                    }
                }
                r.path.clear();
                if (r.status == 3) { r.ub = ub; r.path = dd.getSolution(); }
                else { r.ub = DOUBLE_MIN; r.lb = DOUBLE_MIN; }
            }
            write_result(f, r);
        }
        std::fclose(f);
        return 0;
    }
    if (mode == "restricted" && argc == 8) {
        auto np = std::make_shared<Network>(argv[2]);
        auto cuts = read_cuts(argv[3]);
        auto nodes = read_nodes(argv[4]);
        double inc = parse_double(argv[5]);
        unsigned width = (unsigned)std::strtoul(argv[6], nullptr, 10);
        FILE *f = std::fopen(argv[7], "w");
        std::fprintf(f, "%zu\n", nodes.size());
        for (auto &nd : nodes) restricted(f, np, nd, inc, cuts, width);
        std::fclose(f);
        return 0;
    }
    if (mode == "order" && argc == 4) {
        // processingOrder / Vbar order / totalLayers of the reference loader
        Network net{argv[2]};
        FILE *f = std::fopen(argv[3], "w");
        std::fprintf(f, "%u %zu %zu\n", net.totalLayers, net.processingOrder.size(), net.Vbar.size());
        for (auto &p : net.processingOrder) std::fprintf(f, "%d ", p.second);
        std::fprintf(f, "\n");
        for (auto v : net.Vbar) std::fprintf(f, "%u ", v);
        std::fprintf(f, "\n");
        std::fclose(f);
        return 0;
    }
    if (mode == "time" && argc == 8) {
        // CPU baseline: static partition of the frontier over std::threads, each with
        // its own RelaxedDDNew (one NodeExplorer per thread, NodeExplorer.h:113-116).
        Network net{argv[2]};
        auto cuts = read_cuts(argv[3]);
        auto nodes = read_nodes(argv[4]);
        double inc = parse_double(argv[5]);
        int threads = std::atoi(argv[6]);
        double budget = std::atof(argv[7]);
        std::atomic<size_t> next{0}, done{0};
        std::atomic<bool> stop{false};
        auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> pool;
        for (int t = 0; t < threads; t++) {
            pool.emplace_back([&]() {
                Inavap::RelaxedDDNew dd{&net};
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
        }
        for (auto &th : pool) th.join();
        double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::printf("{\"relaxations\": %zu, \"seconds\": %.6f, \"threads\": %d}\n", done.load(), el, threads);
        return 0;
    }
    if (mode == "relaxp" && argc == 8) {
        Network net{argv[2]};
        auto cuts = read_cuts(argv[3]);
        auto nodes = read_nodes(argv[4]);
        double inc = parse_double(argv[5]);
        int threads = std::max(1, std::atoi(argv[6]));
        std::vector<Result> res(nodes.size());
        std::atomic<size_t> next{0};
        auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> pool;
        for (int t = 0; t < threads; t++) {
            pool.emplace_back([&]() {
                Inavap::RelaxedDDNew dd{&net};
                for (;;) {
                    size_t k = next.fetch_add(1);
                    if (k >= nodes.size()) break;
                    res[k] = process(dd, nodes[k], inc, cuts);
                }
            });
        }
        for (auto &th : pool) th.join();
        double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        FILE *f = std::fopen(argv[7], "w");
        std::fprintf(f, "%zu\n", nodes.size());
        for (auto &r : res) write_result(f, r);
        std::fclose(f);
        std::printf("{\"relaxations\": %zu, \"seconds\": %.6f, \"threads\": %d}\n", nodes.size(), el, threads);
        return 0;
    }
    if (mode == "api" && argc == 7) {
        // The RelaxedDDNew surface one call at a time (DD.h:797-808), as the C++ API's
        // Inavap::RelaxedDDNew drives the device: buildTree, then every pool cut newest first
        // in pool order (types interleaved as inserted) with optimalLB = the incumbent, the
        // value each call returns, getSolution() after every 4th cut and at the end, and for
        // a non-exact tree getCutset(min(node.ub, returned bounds)) (NodeExplorer.cpp:975-985).
        // A call that prunes (F 0, or O <= optimalLB) ends the node: NodeExplorer::process
        // never touches the DD after that.
        Network net{argv[2]};
        auto cuts = read_cuts(argv[3]);
        auto nodes = read_nodes(argv[4]);
        const double inc = parse_double(argv[5]);
        Inavap::RelaxedDDNew dd{&net};
        FILE *f = std::fopen(argv[6], "w");
        std::fprintf(f, "%zu %zu\n", nodes.size(), cuts.size());
        auto put_path = [&](const std::vector<int16_t> &p) {
            std::fprintf(f, "P %zu", p.size());
            for (auto d : p) std::fprintf(f, " %d", (int)d);
            std::fprintf(f, "\n");
        };
        for (auto &nd : nodes) {
            dd.buildTree(nd);
            const int exact = dd.isTreeExact() ? 1 : 0;
            double ub = nd.ub;
            bool pruned = false;
            std::vector<std::string> vals;
            std::vector<std::vector<int16_t>> sols;
            size_t applied = 0;
            for (size_t k = cuts.size(); k-- > 0 && !pruned;) {
                char buf[64];
                if (cuts[k].type == 1) {
                    const int ok = dd.applyFeasibilityCut(cuts[k].cut);
                    std::snprintf(buf, sizeof buf, "F%d", ok);
                    pruned = !ok;
                } else {
                    const double v = dd.applyOptimalityCut(cuts[k].cut, inc, ub);
                    std::snprintf(buf, sizeof buf, "O%a", v);
                    ub = exact ? v : std::min(v, ub);
                    pruned = v <= inc;
                }
                vals.emplace_back(buf);
                applied++;
                if (!pruned && applied % 4 == 0) sols.push_back(dd.getSolution());
            }
            std::fprintf(f, "N %d %zu %zu\n", exact, applied, sols.size());
            std::fprintf(f, "V");
            for (auto &v : vals) std::fprintf(f, " %s", v.c_str());
            std::fprintf(f, "\n");
            for (auto &p : sols) put_path(p);
            if (pruned) { std::fprintf(f, "E 0\n"); continue; }
            put_path(dd.getSolution());
            if (exact) { std::fprintf(f, "E 1\n"); continue; }
            auto ch = dd.getCutset(ub);
            std::fprintf(f, "C %a %zu\n", ub, ch.size());
            for (auto &c : ch) write_node(f, c);
        }
        std::fclose(f);
        return 0;
    }
    if (mode == "apply" && argc == 6) {
        // Per-cut trace on every node: the bound / feasibility flag each cut returns,
        // applying all cuts in pool order (newest first) with incumbent DOUBLE_MIN and
        // no early exit.  Used to pin the sweep kernel cut by cut.
        Network net{argv[2]};
        auto cuts = read_cuts(argv[3]);
        auto nodes = read_nodes(argv[4]);
        Inavap::RelaxedDDNew dd{&net};
        FILE *f = std::fopen(argv[5], "w");
        std::fprintf(f, "%zu %zu\n", nodes.size(), cuts.size());
        for (auto &nd : nodes) {
            dd.buildTree(nd);
            std::fprintf(f, "N %d", dd.isTreeExact() ? 1 : 0);
            for (size_t k = cuts.size(); k-- > 0;) {
                if (cuts[k].type == 1) {
                    int ok = dd.applyFeasibilityCut(cuts[k].cut);
                    std::fprintf(f, " F%d", ok);
                    if (!ok) break;
                } else {
                    double v = dd.applyOptimalityCut(cuts[k].cut, DOUBLE_MIN, DOUBLE_MAX);
                    std::fprintf(f, " O%a", v);
                }
            }
            std::fprintf(f, "\n");
        }
        std::fclose(f);
        return 0;
    }
    std::cerr << "bad arguments\n";
    return 2;
}
