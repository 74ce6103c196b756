// Drives the C++ host mirror (include/sgufp/inavap.hpp) the way the reference's main /
// workers do (main.cpp:56-81, DDSolver.cpp:658-776), for tests/test_host_api.py:
//
//   host_api_test <network file> <known optimum as hex float | none>
//
// prints "ddsolver <optimum %a>" (Inavap::DDSolver::start, batched device rounds) and
// "explorer <optimum %a> <processed>" (a single-worker LIFO loop over
// Inavap::NodeExplorer::process with two global Containers, as Worker::startWorker).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <map>
#include <string>
#include <tuple>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <vector>

#include "sgufp/inavap.hpp"

// "dd" mode: Inavap::RelaxedDDNew call by call, printed as `ref_dd api` prints the
// reference's (oracle/ref_driver.cpp; tests/test_dd_api.py reads both):
//   host_api_test dd <network> <cuts> <nodes> <incumbent hex>
static std::vector<std::pair<int, Inavap::Cut>> read_cuts(const char *path) {
    FILE *f = std::fopen(path, "r");
    if (!f) throw std::runtime_error("cannot open cuts");
    size_t n = 0;
    if (std::fscanf(f, "%zu", &n) != 1) throw std::runtime_error("bad cuts");
    std::vector<std::pair<int, Inavap::Cut>> cuts;
    for (size_t c = 0; c < n; c++) {
        int type;
        char rhs[64];
        size_t nnz;
        if (std::fscanf(f, "%d %63s %zu", &type, rhs, &nnz) != 3) throw std::runtime_error("bad cut");
        std::map<std::tuple<int, int, int>, double> m;   // the reference's CutCoefficients map
        for (size_t k = 0; k < nnz; k++) {
            int i, q, j;
            char v[64];
            if (std::fscanf(f, "%d %d %d %63s", &i, &q, &j, v) != 4) throw std::runtime_error("bad coefficient");
            m[std::make_tuple(i, q, j)] = std::strtod(v, nullptr);
        }
        std::vector<std::pair<uint64_t, double>> coeff;   // cutToCut (Cut.h:406-421): map order, no zeros
        for (auto &[k, v] : m)
            if (v != 0.0) coeff.emplace_back(Inavap::getKey(std::get<1>(k), std::get<0>(k), std::get<2>(k)), v);
        cuts.emplace_back(type, Inavap::Cut{std::strtod(rhs, nullptr), std::move(coeff)});
    }
    std::fclose(f);
    return cuts;
}

static std::vector<Inavap::Node> read_nodes(const char *path) {
    FILE *f = std::fopen(path, "r");
    if (!f) throw std::runtime_error("cannot open nodes");
    size_t n = 0;
    if (std::fscanf(f, "%zu", &n) != 1) throw std::runtime_error("bad nodes");
    std::vector<Inavap::Node> out;
    for (size_t k = 0; k < n; k++) {
        int gl;
        char lb[64], ub[64];
        size_t ns, nsol;
        if (std::fscanf(f, "%d %63s %63s %zu", &gl, lb, ub, &ns) != 4) throw std::runtime_error("bad node");
        std::vector<int16_t> st(ns), sol;
        for (auto &x : st) { int v; if (std::fscanf(f, "%d", &v) != 1) throw std::runtime_error("bad node"); x = (int16_t)v; }
        if (std::fscanf(f, "%zu", &nsol) != 1) throw std::runtime_error("bad node");
        sol.resize(nsol);
        for (auto &x : sol) { int v; if (std::fscanf(f, "%d", &v) != 1) throw std::runtime_error("bad node"); x = (int16_t)v; }
        out.emplace_back(std::move(st), std::move(sol), std::strtod(lb, nullptr), std::strtod(ub, nullptr), (uint16_t)gl);
    }
    std::fclose(f);
    return out;
}

static int dd_mode(char **argv) {
    Network net(argv[2]);
    auto cuts = read_cuts(argv[3]);
    auto nodes = read_nodes(argv[4]);
    const double inc = std::strtod(argv[5], nullptr);
    Inavap::RelaxedDDNew dd{&net};
    std::printf("%zu %zu\n", nodes.size(), cuts.size());
    auto put_path = [](const Inavap::Path &p) {
        std::printf("P %zu", p.size());
        for (auto d : p) std::printf(" %d", (int)d);
        std::printf("\n");
    };
    for (auto &nd : nodes) {
        dd.buildTree(nd);
        const int exact = dd.isTreeExact() ? 1 : 0;
        double ub = nd.ub;
        bool pruned = false;
        std::vector<std::string> vals;
        std::vector<Inavap::Path> sols;
        for (size_t k = cuts.size(); k-- > 0 && !pruned;) {
            char buf[64];
            if (cuts[k].first == 1) {
                const int ok = dd.applyFeasibilityCut(cuts[k].second);
                std::snprintf(buf, sizeof buf, "F%d", ok);
                pruned = !ok;
            } else {
                const double v = dd.applyOptimalityCut(cuts[k].second, inc, ub);
                std::snprintf(buf, sizeof buf, "O%a", v);
                ub = exact ? v : std::min(v, ub);
                pruned = v <= inc;
            }
            vals.emplace_back(buf);
            if (!pruned && vals.size() % 4 == 0) sols.push_back(dd.getSolution());
        }
        std::printf("N %d %zu %zu\nV", exact, vals.size(), sols.size());
        for (auto &v : vals) std::printf(" %s", v.c_str());
        std::printf("\n");
        for (auto &p : sols) put_path(p);
        if (pruned) { std::printf("E 0\n"); continue; }
        put_path(dd.getSolution());
        if (exact) { std::printf("E 1\n"); continue; }
        auto ch = dd.getCutset(ub);
        std::printf("C %a %zu\n", ub, ch.size());
        for (auto &c : ch) {
            std::printf("%u %a %a %zu", (unsigned)c.globalLayer, c.lb, c.ub, c.states.size());
            for (auto x : c.states) std::printf(" %d", (int)x);
            std::printf(" %zu", c.solutionVector.size());
            for (auto x : c.solutionVector) std::printf(" %d", (int)x);
            std::printf("\n");
        }
    }
    return 0;
}

// "search" mode: Inavap::DDSolver at scale, as the bench's B&B legs drive the Python solver
// (bench.py bnb_run): a warm-up search of 2 s whose pool is dropped, then the timed search
// (no warm-up with a round cap: the search is then reproducible round for round)
//   host_api_test search <network> <restricted width> <seconds> <batch> <round seconds>
//                        <round iters> <max rounds (0: none)>
// prints "search <incumbent %a> <heuristic %a> <seconds> <rounds> <complete>" and one
// "counter <name> <value>" line per sgufp_bnb_stats total.
static int search_mode(char **argv) {
    auto net = std::make_shared<Network>(argv[2]);
    const int width = std::atoi(argv[3]);
    const double seconds = std::strtod(argv[4], nullptr);
    const int batch = std::atoi(argv[5]);
    const double round_seconds = std::strtod(argv[6], nullptr);
    const int round_iters = std::atoi(argv[7]);
    const long max_rounds = std::atol(argv[8]);
    Inavap::DDSolver solver{net, 1, batch};
    if (max_rounds == 0) {   // a timed run: warm-up first (a round cap asks for a reproducible search)
        solver.roundLimits(round_iters, std::min(round_seconds, 2.0));
        solver.timeBudget(2.0);
        solver.startSolver(Inavap::DOUBLE_MIN);                 // kernels, allocations
        if (sgufp_cuts_clear(solver.context()) != SGUFP_OK) throw std::runtime_error("cuts clear");
    }
    solver.roundLimits(round_iters, round_seconds);
    solver.timeBudget(seconds);
    solver.restrictedSeed(width);
    solver.maxRounds = max_rounds;
    const auto t0 = std::chrono::steady_clock::now();
    const double z = solver.startSolver(Inavap::DOUBLE_MIN);
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("search %a %a %.6f %lld %d\n", z, solver.heuristicIncumbent, secs, (long long)solver.rounds,
                solver.complete ? 1 : 0);
    const sgufp_bnb_stats &t = solver.totals;
    const std::pair<const char *, int64_t> cs[] = {
        {"popped", t.popped}, {"relaxed", t.relaxed}, {"pruned_bound", t.pruned_bound},
        {"pruned_feasibility", t.pruned_feasibility}, {"pruned_optimality", t.pruned_optimality}, {"exact", t.exact},
        {"exact_closed", t.exact_closed}, {"subproblems", t.subproblems},
        {"new_feasibility_cuts", t.new_feasibility_cuts}, {"new_optimality_cuts", t.new_optimality_cuts},
        {"children", t.children}, {"pushed", t.pushed}, {"deferred", t.deferred}, {"resumed", t.resumed}};
    for (auto &[k, v] : cs) std::printf("counter %s %lld\n", k, (long long)v);
    std::printf("pool %d %d\n", sgufp_cuts_count(solver.context(), 1), sgufp_cuts_count(solver.context(), 0));
    return 0;
}

int main(int argc, char **argv) {
    if (argc == 9 && std::strcmp(argv[1], "search") == 0) {
        try {
            return search_mode(argv);
        } catch (const std::exception &e) {
            std::fprintf(stderr, "error: %s\n", e.what());
            return 1;
        }
    }
    if (argc == 6 && std::strcmp(argv[1], "dd") == 0) {
        try {
            return dd_mode(argv);
        } catch (const std::exception &e) {
            std::fprintf(stderr, "error: %s\n", e.what());
            return 1;
        }
    }
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s <network> <known optimum hex|none>\n", argv[0]);
        return 2;
    }
    const double known = std::strcmp(argv[2], "none") == 0 ? Inavap::DOUBLE_MIN : std::strtod(argv[2], nullptr);
    try {
        auto net = std::make_shared<Network>(argv[1]);
        {
            Inavap::DDSolver solver{net, 4};
            auto [sol, secs] = solver.start(known);
            std::printf("ddsolver %a %.3f\n", sol, secs);
        }
        {
            // the same search as a one-shard communicator: every round runs the RCCL
            // exchanges of a multi-GPU search (shard.cpp) with a bounded refinement loop
            uint8_t id[SGUFP_COMM_ID_BYTES];
            if (sgufp_comm_unique_id(id, SGUFP_COMM_ID_BYTES) != SGUFP_OK) throw std::runtime_error("unique id");
            Inavap::DDSolver solver{net, 4, 64};
            solver.shard(1, 0, id);
            solver.roundLimits(2, 0.0);
            auto [sol, secs] = solver.start(known);
            std::printf("sharded %a %.3f %lld\n", sol, secs, (long long)solver.totals.deferred);
        }
        Inavap::NodeExplorer explorer{net};
        Inavap::Container feas, opt;
        std::vector<Inavap::Node> stack;
        stack.emplace_back(std::vector<int16_t>{}, std::vector<int16_t>{}, Inavap::DOUBLE_MIN, Inavap::DOUBLE_MAX, 0);
        double zOpt = known;
        long processed = 0;
        while (!stack.empty()) {
            Inavap::Node node = std::move(stack.back());
            stack.pop_back();
            if (node.ub <= zOpt) continue;                     // DDSolver.cpp:707-711
            auto result = explorer.process(node, zOpt, feas, opt);
            processed++;
            if (result.status != Inavap::OutObj::SUCCESS) continue;
            if (result.lb > zOpt) zOpt = result.lb;            // DDSolver.cpp:723-731
            if (result.ub > zOpt && !result.nodes.empty())     // DDSolver.cpp:744-748
                for (auto it = result.nodes.rbegin(); it != result.nodes.rend(); ++it) stack.push_back(*it);
        }
        std::printf("explorer %a %ld\n", zOpt, processed);
    } catch (const std::exception &e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}
