// Host C++ mirror of the reference's solver API over the C ABI (include/sgufp/inavap.hpp).
// Built into libsgufp_host.so (g++, links libsgufp_hip.so); no device code here.
#include "sgufp/inavap.hpp"

#include <algorithm>
#include <chrono>
#include <ctime>
#include <sstream>
#include <vector>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <tuple>

// ---- Network -------------------------------------------------------------------------
Network::Network(const std::string &path_, int device_) : path{path_}, device{device_} {
    std::ifstream in(path);
    if (!in || !(in >> n >> edges >> nScenarios)) throw sgufp_error("cannot read network file " + path);
    int32_t L = 0, nv = 0;
    if (sgufp_probe_network(path.c_str(), &L, &nv, 0, nullptr, nullptr) != SGUFP_OK)
        throw sgufp_error("cannot parse network file " + path);
    std::vector<int32_t> la(std::max(L, 1)), vb(std::max(nv, 1));
    sgufp_probe_network(path.c_str(), &L, &nv, std::max(L, nv), la.data(), vb.data());
    totalLayers = L;
    Vbar.assign(vb.begin(), vb.begin() + nv);
    for (int l = 0; l < L; l++) processingOrder.emplace_back((uint32_t)l, (uint32_t)la[l]);
}

namespace Inavap {

double Cut::get(uint64_t key) const {
    for (const auto &[k, v] : coeff)
        if ((k & 0xFFFFFFFFFFFFull) == (key & 0xFFFFFFFFFFFFull)) return v;
    return 0.0;
}


// ---- device handle -----------------------------------------------------------------------
Device::Device(const Network &net, int max_batch) {
    int err = 0;
    ctx_ = sgufp_create_from_file(net.path.c_str(), net.device, max_batch, &err);
    if (!ctx_) throw sgufp_error("sgufp_create_from_file failed (" + std::to_string(err) + ") for " + net.path);
}

Device::~Device() { sgufp_destroy(ctx_); }

void Device::check(int rc, const char *what) const {
    if (rc != SGUFP_OK) throw sgufp_error(std::string(what) + ": " + sgufp_last_error(ctx_));
}

// ---- RelaxedDDNew: one device slot ---------------------------------------------------------
RelaxedDDNew::RelaxedDDNew(const Network *pointer) : networkPtr{pointer}, dev{new Device(*pointer, 1)} {}

void RelaxedDDNew::buildTree(Node root) {
    sgufp_ctx *g = dev->get();
    uint16_t gl = root.globalLayer;
    int64_t so[2] = {0, (int64_t)root.states.size()}, po[2] = {0, (int64_t)root.solutionVector.size()};
    static const int16_t empty = 0;
    dev->check(sgufp_batch_upload(g, 1, &gl, &root.lb, &root.ub, so, root.states.empty() ? &empty : root.states.data(),
                                  po, root.solutionVector.empty() ? &empty : root.solutionVector.data()),
               "buildTree upload");
    dev->check(sgufp_dd_build(g), "buildTree");
    int32_t st = 0;
    uint8_t ex = 0;
    dev->check(sgufp_batch_results(g, &st, &ex, nullptr, nullptr, nullptr), "buildTree results");
    if (st != SGUFP_SUCCESS && st != SGUFP_NEEDS_SUBPROBLEM)
        throw sgufp_error("buildTree: record rejected by the device (status " + std::to_string(st) + ")");
    exact = ex != 0;
    built = true;
}

void RelaxedDDNew::upload_cut(const Cut &cut, std::vector<uint64_t> &keys, std::vector<double> &vals) const {
    if (!built) throw sgufp_error("RelaxedDDNew: buildTree first");
    keys.clear();
    vals.clear();
    for (auto &[k, v] : cut.coeff) {
        keys.push_back(k);
        vals.push_back(v);
    }
}

uint8_t RelaxedDDNew::applyFeasibilityCut(const Cut &cut) {
    std::vector<uint64_t> keys;
    std::vector<double> vals;
    upload_cut(cut, keys, vals);
    double v = 0.0;
    dev->check(sgufp_dd_apply(dev->get(), 0, 1, cut.RHS, (int64_t)keys.size(), keys.data(), vals.data(), DOUBLE_MIN, &v),
               "applyFeasibilityCut");
    return v != 0.0 ? 1 : 0;
}

double RelaxedDDNew::applyOptimalityCut(const Cut &cut, double optimal, double /*upperbound: unused, DD.cpp:3932*/) {
    std::vector<uint64_t> keys;
    std::vector<double> vals;
    upload_cut(cut, keys, vals);
    double v = 0.0;
    dev->check(sgufp_dd_apply(dev->get(), 0, 0, cut.RHS, (int64_t)keys.size(), keys.data(), vals.data(), optimal, &v),
               "applyOptimalityCut");
    return v;
}

Path RelaxedDDNew::getSolution() const {
    if (!built) throw sgufp_error("RelaxedDDNew: buildTree first");
    Path p((size_t)std::max(networkPtr->totalLayers, 1));
    int32_t len = 0;
    dev->check(sgufp_dd_solution(dev->get(), 0, p.data(), &len), "getSolution");
    p.resize((size_t)len);
    return p;
}

std::vector<Node> RelaxedDDNew::getCutset(double ub) {
    if (!built) throw sgufp_error("RelaxedDDNew: buildTree first");
    sgufp_ctx *g = dev->get();
    int64_t n = 0, ns = 0, nsol = 0;
    dev->check(sgufp_dd_cutset(g, 0, ub, &n), "getCutset");
    dev->check(sgufp_batch_children_size(g, &n, &ns, &nsol), "getCutset size");
    std::vector<int64_t> coff(2), soff(n + 1), poff(n + 1);
    std::vector<uint16_t> cg(n + 1);
    std::vector<double> cl(n + 1), cu(n + 1);
    std::vector<int16_t> st(ns + 1), sol(nsol + 1);
    dev->check(sgufp_batch_children(g, coff.data(), cg.data(), cl.data(), cu.data(), soff.data(), st.data(), poff.data(),
                                    sol.data()),
               "getCutset children");
    std::vector<Node> out;
    out.reserve((size_t)n);
    for (int64_t c = 0; c < n; c++)
        out.emplace_back(std::vector<int16_t>(st.begin() + soff[c], st.begin() + soff[c + 1]),
                         std::vector<int16_t>(sol.begin() + poff[c], sol.begin() + poff[c + 1]), cl[c], cu[c], cg[c]);
    return out;
}

// ---- scenario subproblem -------------------------------------------------------------------
GuroSolver::GuroSolver(const std::shared_ptr<Network> &networkPtr) : net{networkPtr}, dev{*networkPtr, 1} {
    sgufp_network_info info{};
    dev.check(sgufp_get_network_info(dev.get(), &info), "network info");
    slot_keys.resize(info.n_slots);
    if (info.n_slots) dev.check(sgufp_slot_keys(dev.get(), slot_keys.data()), "slot keys");
}

std::pair<CutType, Cut> GuroSolver::solveSubProblem(const std::vector<int16_t> &path) {
    const size_t ns = slot_keys.size();
    int64_t off[2] = {0, (int64_t)path.size()};
    int32_t type = -1;
    double rhs = 0.0;
    std::vector<double> row(ns + 1);
    static const int16_t empty = 0;
    dev.check(sgufp_subproblem(dev.get(), 1, off, path.empty() ? &empty : path.data(), &type, &rhs, row.data(),
                               nullptr),
              "subproblem");
    if (type < 0) throw sgufp_error("scenario subproblem failed for the given path");
    // cutToCut (Cut.h:406-421): walk (i,q,j) in map order, drop exact zeros
    std::vector<std::tuple<uint64_t, uint64_t, uint64_t, double>> e;
    for (size_t s = 0; s < ns; s++) {
        if (row[s] == 0) continue;
        const uint64_t k = slot_keys[s];
        e.emplace_back(k >> 16 & 0xFFFF, k & 0xFFFF, k >> 32 & 0xFFFF, row[s]);
    }
    std::sort(e.begin(), e.end(), [](const auto &a, const auto &b) {
        return std::tie(std::get<0>(a), std::get<1>(a), std::get<2>(a)) <
               std::tie(std::get<0>(b), std::get<1>(b), std::get<2>(b));
    });
    std::vector<std::pair<uint64_t, double>> coeff;
    for (auto &[i, q, j, v] : e) coeff.emplace_back(getKey(q, i, j), v);
    return {type == 1 ? FEASIBILITY : OPTIMALITY, Cut{rhs, std::move(coeff)}};
}

// ---- NodeExplorer --------------------------------------------------------------------------
NodeExplorer::NodeExplorer(const std::shared_ptr<Network> &networkPtr_)
    : networkPtr{networkPtr_}, dev{*networkPtr_, 1}, solver{networkPtr_} {}

// Upload the cuts added to a Container since the last call, oldest first (the list is LIFO).
void NodeExplorer::sync_pool(int is_feas, const cut_node_t *head, const cut_node_t *&seen) {
    std::vector<const Cut *> fresh;
    for (auto *c = head; c && c != seen; c = c->next) fresh.push_back(&c->cut);
    seen = head;
    if (fresh.empty()) return;
    std::reverse(fresh.begin(), fresh.end());
    std::vector<double> rhs;
    std::vector<int64_t> off{0};
    std::vector<uint64_t> keys;
    std::vector<double> vals;
    for (auto *c : fresh) {
        rhs.push_back(c->RHS);
        for (auto &[k, v] : c->coeff) {
            keys.push_back(k);
            vals.push_back(v);
        }
        off.push_back((int64_t)keys.size());
    }
    dev.check(sgufp_cuts_append(dev.get(), is_feas, (int)fresh.size(), rhs.data(), off.data(), keys.data(), vals.data()),
              "cuts append");
}

OutObject NodeExplorer::process(Node node, double optimalLB, Container &globalFeasCuts, Container &globalOptCuts) {
    sgufp_ctx *g = dev.get();
    // the snapshot of NodeExplorer.cpp:930-931
    sync_pool(1, globalFeasCuts.get(), f_seen);
    sync_pool(0, globalOptCuts.get(), o_seen);
    uint16_t gl = node.globalLayer;
    int64_t so[2] = {0, (int64_t)node.states.size()}, po[2] = {0, (int64_t)node.solutionVector.size()};
    static const int16_t empty = 0;
    dev.check(sgufp_batch_upload(g, 1, &gl, &node.lb, &node.ub, so, node.states.empty() ? &empty : node.states.data(),
                                 po, node.solutionVector.empty() ? &empty : node.solutionVector.data()),
              "upload");
    dev.check(sgufp_batch_relax(g, optimalLB), "relax");
    dev.check(sgufp_batch_sync(g), "sync");
    int32_t st = 0, nch = 0;
    uint8_t ex = 0;
    double lb = 0, ub = 0;
    dev.check(sgufp_batch_results(g, &st, &ex, &lb, &ub, &nch), "results");
    auto pruned = [](int32_t s) {
        return OutObject{DOUBLE_MIN, DOUBLE_MIN, {},
                         (uint16_t)(s == SGUFP_PRUNED_BY_FEASIBILITY_CUT ? OutObj::PRUNED_BY_FEASIBILITY_CUT
                                                                         : OutObj::PRUNED_BY_OPTIMALITY_CUT)};
    };
    if (st == SGUFP_PRUNED_BY_FEASIBILITY_CUT || st == SGUFP_PRUNED_BY_OPTIMALITY_CUT) return pruned(st);
    if (st == SGUFP_SUCCESS) {   // non-exact: {DOUBLE_MIN, ub, getCutset(ub)}
        int64_t n = 0, ns = 0, nsol = 0;
        dev.check(sgufp_batch_children_size(g, &n, &ns, &nsol), "children size");
        std::vector<uint16_t> cg(n + 1);
        std::vector<double> cl(n + 1), cu(n + 1);
        std::vector<int64_t> coff(2), sof(n + 1), pof(n + 1);
        std::vector<int16_t> s(ns + 1), p(nsol + 1);
        dev.check(sgufp_batch_children(g, coff.data(), cg.data(), cl.data(), cu.data(), sof.data(), s.data(), pof.data(),
                                       p.data()),
                  "children");
        std::vector<Node> kids;
        kids.reserve(n);
        for (int64_t c = 0; c < n; c++)
            kids.emplace_back(std::vector<int16_t>(s.begin() + sof[c], s.begin() + sof[c + 1]),
                              std::vector<int16_t>(p.begin() + pof[c], p.begin() + pof[c + 1]), cl[c], cu[c], cg[c]);
        return OutObject{lb, ub, std::move(kids), OutObj::SUCCESS};
    }
    if (st != SGUFP_NEEDS_SUBPROBLEM) throw sgufp_error("process: node failed with status " + std::to_string(st));
    // exact DD: refinement loop (NodeExplorer.cpp:946-969); the DD stays resident in slot 0
    std::vector<Path> allSolutions;
    for (;;) {
        int64_t poff[2] = {0, 0};
        dev.check(sgufp_batch_paths(g, poff, nullptr), "paths");
        Path path(poff[1]);
        dev.check(sgufp_batch_paths(g, poff, path.data()), "paths");
        if (std::find(allSolutions.begin(), allSolutions.end(), path) != allSolutions.end())
            return OutObject{ub, ub, {}, OutObj::SUCCESS};
        allSolutions.push_back(path);
        auto [cutType, cut] = solver.solveSubProblem(path);
        auto *new_cut = new cut_node_t{cut};
        const int is_feas = cutType == FEASIBILITY ? 1 : 0;
        Container &pool = is_feas ? globalFeasCuts : globalOptCuts;
        pool.add(new_cut);
        // upload everything newer than the last sync (other threads' cuts included, oldest
        // first); the new cut's device index follows from its depth in that snapshot
        const cut_node_t *head = pool.get();
        int above = 0;
        for (auto *c = head; c && c != new_cut; c = c->next) above++;
        sync_pool(is_feas, head, is_feas ? f_seen : o_seen);
        int32_t idx = 0, cut_index = sgufp_cuts_count(g, is_feas) - 1 - above;
        uint8_t f8 = (uint8_t)is_feas;
        dev.check(sgufp_batch_refine(g, 1, &idx, &f8, &cut_index, optimalLB), "refine");
        dev.check(sgufp_batch_results(g, &st, &ex, &lb, &ub, &nch), "results");
        if (st == SGUFP_PRUNED_BY_FEASIBILITY_CUT || st == SGUFP_PRUNED_BY_OPTIMALITY_CUT) return pruned(st);
    }
}

// ---- DDSolver ------------------------------------------------------------------------------
DDSolver::DDSolver(const std::shared_ptr<Network> &networkPtr_, uint16_t nWorkers, int batch_)
    : networkPtr{networkPtr_}, N_WORKERS{nWorkers}, dev{*networkPtr_, std::max(1, batch_)}, batch{std::max(1, batch_)} {}

void DDSolver::shard(int world, int rank, const uint8_t *id) {
    dev.check(sgufp_comm_init(dev.get(), world, rank, id), "comm init");
}

void DDSolver::roundLimits(int maxRefineIters, double roundSeconds) {
    maxIters = maxRefineIters;
    roundSecs = roundSeconds;
    dev.check(sgufp_bnb_set_limits(dev.get(), maxRefineIters, roundSeconds), "round limits");
}

// The restricted-DD seed on the root record (NodeExplorer.cpp:605-664, the exact-tree loop of
// processX3; sgufp_solver_amd/restricted.py is the same loop): relax, then until the max path
// repeats with an unchanged bound, solve its subproblem and add the cut to the pool.  Returns
// the converged bound, or z when the record is pruned or does not converge within 500 cuts.
double DDSolver::restricted_incumbent(double z) {
    sgufp_ctx *g = dev.get();
    sgufp_network_info info{};
    dev.check(sgufp_get_network_info(g, &info), "network info");
    const size_t stride = (size_t)info.n_slots + 1;
    uint16_t gl = 0;
    double lb = DOUBLE_MIN, ub = DOUBLE_MAX;
    int64_t z2[2] = {0, 0};
    static const int16_t empty = 0;
    Path prev;
    double prev_lb = 0.0;
    bool have = false;
    for (int it = 0; it <= 500; it++) {
        dev.check(sgufp_batch_upload(g, 1, &gl, &lb, &ub, z2, &empty, z2, &empty), "restricted upload");
        dev.check(sgufp_restricted_relax(g, seedWidth, z), "restricted relax");
        int32_t st = 0, plen = 0, cn = 0;
        uint8_t ex = 0;
        double rlb = 0.0;
        dev.check(sgufp_restricted_results(g, &st, &ex, &rlb, &plen, &cn), "restricted results");
        if (st >= 16) throw sgufp_error("restricted heuristic: root record failed on the device");
        if (st != 0) return z;                                       // INVALID_OBJECT
        int64_t poff[2] = {0, 0};
        dev.check(sgufp_restricted_paths(g, poff, nullptr), "restricted paths");
        Path path((size_t)poff[1]);
        dev.check(sgufp_restricted_paths(g, poff, path.empty() ? nullptr : path.data()), "restricted paths");
        if (have && path == prev) {
            if (rlb == prev_lb) return std::max(z, rlb);             // {lowerBound, ...}
        }
        prev = path;
        prev_lb = rlb;
        have = true;
        if (it == 500) break;
        int64_t off[2] = {0, (int64_t)path.size()};
        int32_t type = -1;
        double rhs = 0.0;
        std::vector<double> row(stride);
        dev.check(sgufp_subproblem(g, 1, off, path.empty() ? &empty : path.data(), &type, &rhs, row.data(), nullptr),
                  "restricted subproblem");
        if (type < 0) throw sgufp_error("restricted heuristic: subproblem failed");
        dev.check(sgufp_cuts_append_rows(g, type, 1, &rhs, row.data()), "restricted cut");
    }
    return z;
}

double DDSolver::startSolver(double known_optimal) {
    sgufp_ctx *g = dev.get();
    dev.check(sgufp_frontier_clear(g), "frontier clear");
    int world = 1, rank = 0;
    dev.check(sgufp_comm_info(g, &world, &rank), "comm info");
    // root record Node{} (DDSolver.cpp:788-791) on the first shard; its cutset is taken with
    // ub = DOUBLE_MAX
    uint16_t gl = 0;
    double lb = DOUBLE_MIN, ub = DOUBLE_MAX;
    int64_t z2[2] = {0, 0};
    static const int16_t empty = 0;
    received = 0;
    std::vector<int64_t> sizes((size_t)world);
    double z = known_optimal;
    const auto t_start = std::chrono::steady_clock::now();
    auto elapsed = [&] { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count(); };
    heuristicIncumbent = DOUBLE_MIN;
    if (seedWidth > 0 && rank == 0) {
        heuristicIncumbent = restricted_incumbent(z);
        z = std::max(z, heuristicIncumbent);
    }
    if (rank == 0) dev.check(sgufp_frontier_push(g, 1, &gl, &lb, &ub, z2, &empty, z2, &empty), "frontier push");
    complete = false;
    totals = sgufp_bnb_stats{};
    rounds = 0;
    // dive depth-first with small rounds until the first exact leaves are reached (no cut
    // can prune before that), then full batches
    bool diving = true;
    for (;;) {
        if (budget > 0) {
            // the round's refinement loops stop at the budget (or the round limit): the
            // unfinished exact records go back on top of the frontier
            const double left = budget - elapsed();
            const double secs = std::max(1e-3, roundSecs > 0 ? std::min(left, roundSecs) : left);
            dev.check(sgufp_bnb_set_limits(g, maxIters, secs), "round limits");
        }
        sgufp_bnb_stats st{};
        dev.check(sgufp_bnb_step(g, diving ? std::min(batch, kDiveBatch) : batch, &z, &st), "B&B round");
        if (st.exact > 0) diving = false;
#ifdef SOLVER_COUNTERS
        if (st.improved) {   // DDSolver.cpp:732-738 (the device is worker 0)
            const auto t_c = std::chrono::system_clock::to_time_t(std::chrono::system_clock::now());
            std::cout << "Thread: " << 0 << " , optimal lb: " << z << " set at, " << std::ctime(&t_c) << std::endl;
        }
#endif
        rounds++;
        totals.popped += st.popped;
        totals.relaxed += st.relaxed;
        totals.pruned_bound += st.pruned_bound;
        totals.pruned_feasibility += st.pruned_feasibility;
        totals.pruned_optimality += st.pruned_optimality;
        totals.exact += st.exact;
        totals.exact_closed += st.exact_closed;
        totals.subproblems += st.subproblems;
        totals.new_feasibility_cuts += st.new_feasibility_cuts;
        totals.new_optimality_cuts += st.new_optimality_cuts;
        totals.children += st.children;
        totals.pushed += st.pushed;
        totals.dd_nodes += st.dd_nodes;
        totals.dd_arcs += st.dd_arcs;
        totals.sweeps += st.sweeps;
        totals.frontier = st.frontier;
        totals.deferred += st.deferred;
        totals.resumed += st.resumed;
        const bool over = (budget > 0 && elapsed() > budget) || (maxRounds > 0 && rounds >= maxRounds);
        if (world == 1) {
            if (st.frontier == 0) {
                complete = true;
                break;
            }
            if (over) break;
            continue;
        }
        // the round's exchanges between the shards (shard.cpp)
        int64_t got = 0;
        dev.check(sgufp_incumbent_allreduce(g, &z), "incumbent all-reduce");
        dev.check(sgufp_cuts_exchange(g, &got), "cut exchange");
        dev.check(sgufp_frontier_sizes(g, sizes.data()), "frontier sizes");
        int64_t left = 0;
        for (int64_t s : sizes) left += s;
        if (left == 0) {
            complete = true;
            break;
        }
        // every shard stops in the same round once one of them is over the budget
        double stop = over ? 1.0 : 0.0;
        dev.check(sgufp_incumbent_allreduce(g, &stop), "budget all-reduce");
        if (stop > 0.0) break;
        dev.check(sgufp_frontier_balance(g, &got), "work sharing");
        received += got;
        if (st.exact > 0 || got > 0) diving = false;
    }
    return z;
}

std::string DDSolver::workerStats() const {
    // DDSolver.h:441-501: the dash line is 72 wide (its size is taken before the list fills)
    const std::string dash(72, '-');
    const double processed = (double)totals.relaxed;   // nProcessed of the single device worker
    std::ostringstream o;
    o << dash << "\n";
    o << "Processed: " << totals.relaxed << "  " << "\n";
    o << "Total: " << processed << "\t Mean: " << processed << "\t Deviation: " << 0.0 << "\t Min: " << processed
      << "\t Max: " << processed << "\n";
    o << dash << "\n\n";
    o << "Cuts (feasibility, optimality): " << sgufp_cuts_count(dev.get(), 1) << " , " << sgufp_cuts_count(dev.get(), 0)
      << "\n";
    o << dash << "\n";
    o << "Nodes pruned (feasibility, optimality, bound): " << "\n";
    o << "(" << totals.pruned_feasibility << ", " << totals.pruned_optimality << ", " << totals.pruned_bound << ")"
      << "  " << "\n";
    o << dash << "\n";
    o << "Waiting Time (seconds): " << 0 << "   " << "\n";
    o << dash << "\n\n";
    return o.str();
}

std::pair<double, double> DDSolver::start(double known_opt) {
    const auto t0 = std::chrono::high_resolution_clock::now();
    const double solution = startSolver(known_opt);
    const auto t1 = std::chrono::high_resolution_clock::now();
    const double secs = std::chrono::duration<double>(t1 - t0).count();
#ifdef SOLVER_COUNTERS
    std::cout << workerStats();
#endif
    // DDSolver.cpp:863-865 ("Explored" = children enqueued, sum of nQueue)
    std::cout << "Optimal solution: " << solution << ". Explored " << totals.children
              << " nodes (entire search space) in " << secs << " seconds." << std::endl;
    std::cout << "Device rounds : " << rounds << " (batch " << batch << ", " << N_WORKERS << " workers requested)."
              << std::endl;
    return {solution, secs};
}

}  // namespace Inavap
