// inavap.hpp -- C++ host API of the MI355X build, mirroring the reference's names and
// signatures (var-nan/SGUFP_Solver @ 2025-07-18) on top of the C ABI (sgufp_hip.h):
//
//   Network(const std::string&)                         Network.h:65-113, Network.cpp:10-186
//   Inavap::Node                                        DD.h:456-478
//   Inavap::Cut / cut_node_t / Container / getKey        Cut.h:201-337, 342-344, 448-485
//   CutType                                             Cut.h:22-25
//   Inavap::OutObject (STATUS_OP)                        NodeExplorer.h:78-110
//   Inavap::RelaxedDDNew (buildTree / isTreeExact /     DD.h:797-808, DD.cpp:3528-4218
//     applyFeasibilityCut / applyOptimalityCut / getSolution / getCutset)
//   Inavap::GuroSolver::solveSubProblem(path)            grb.h:75, grb.cpp:139-360 (device LP)
//   Inavap::NodeExplorer::process(node, lb, F, O)        NodeExplorer.h:124-130, NodeExplorer.cpp:915-986
//   Inavap::DDSolver(net, nWorkers) / start / startSolver DDSolver.h:431-439, DDSolver.cpp:782-867
//
// Differences a maintainer should know: a Network owns only host metadata -- every
// NodeExplorer / GuroSolver / DDSolver opens its own device context on it (one HIP
// stream each, used by one thread at a time, like the reference's per-thread explorers).
// Failures of the device path throw sgufp_error (the reference builds with
// -fno-exceptions and terminates inside Gurobi instead).
#pragma once

#include <atomic>
#include <cstdint>
#include <limits>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "sgufp_hip.h"

enum CutType { OPTIMALITY, FEASIBILITY };

struct sgufp_error : std::runtime_error {
    using std::runtime_error::runtime_error;
};

class Network {
  public:
    explicit Network(const std::string &path, int device = 0);
    std::string path;
    int device = 0;
    uint32_t n = 0, edges = 0, nScenarios = 0;
    int totalLayers = 0;
    std::vector<uint32_t> Vbar;                                 // shuffled V-bar order (Network.cpp:132-186)
    std::vector<std::pair<uint32_t, uint32_t>> processingOrder; // (layer, arc id) (Network.cpp:111-116)
};

namespace Inavap {

static constexpr double DOUBLE_MIN = std::numeric_limits<double>::lowest();
static constexpr double DOUBLE_MAX = std::numeric_limits<double>::max();

using Path = std::vector<int16_t>;

class Node {
  public:
    std::vector<int16_t> states{};
    std::vector<int16_t> solutionVector{};
    double lb;
    double ub;
    uint16_t globalLayer;
    Node *next = nullptr;

    Node() : lb{DOUBLE_MIN}, ub{DOUBLE_MIN}, globalLayer{0} {}
    Node(std::vector<int16_t> states_, std::vector<int16_t> solutionVector_, double lb_, double ub_, uint16_t gl_)
        : states{std::move(states_)}, solutionVector{std::move(solutionVector_)}, lb{lb_}, ub{ub_}, globalLayer{gl_} {}
};

inline uint64_t getKey(uint64_t q, uint64_t i, uint64_t j) { return q | (i << 16) | (j << 32); }

class Cut {
  public:
    size_t hash_val = 0;
    double RHS = 0.0;
    std::vector<std::pair<uint64_t, double>> coeff;   // (getKey(q,i,j), value), (i,q,j) order
    Cut() = default;
    Cut(double rhs, std::vector<std::pair<uint64_t, double>> c) : RHS{rhs}, coeff{std::move(c)} {}
    // Cut::get (Cut.h:275-282): first entry whose low 48 bits match, else 0
    double get(uint64_t key) const;
};

class cut_node_t {
  public:
    Cut cut;
    cut_node_t *next = nullptr;
    explicit cut_node_t(const Cut &cut_) : cut{cut_.RHS, cut_.coeff} {}
};

// Global cut pool: lock-free LIFO list, readers see newest first (Cut.h:448-485).
class Container {
    std::atomic<cut_node_t *> head{nullptr};

  public:
    const cut_node_t *get() const { return head.load(std::memory_order_acquire); }
    // Container::add (Cut.h:461-465): push onto the list head with a release CAS; a reader that
    // acquires the head sees every cut pushed before it, newest first
    void add(cut_node_t *node) {
        node->next = head.load(std::memory_order_relaxed);
        while (!head.compare_exchange_weak(node->next, node, std::memory_order_release, std::memory_order_relaxed)) {
        }
    }
    ~Container() {
        cut_node_t *cur = head.load(std::memory_order_acquire);
        while (cur) {
            cut_node_t *nx = cur->next;
            delete cur;
            cur = nx;
        }
    }
};

struct OutObj {
    enum STATUS_OP { SUCCESS = 0x0, PRUNED_BY_FEASIBILITY_CUT = 0x1, PRUNED_BY_OPTIMALITY_CUT = 0x2 };
    double lb = DOUBLE_MIN;
    double ub = DOUBLE_MIN;
    std::vector<Node> nodes;
    uint16_t status = SUCCESS;
    OutObj(double lb_, double ub_, std::vector<Node> nodes_, uint16_t status_)
        : lb{lb_}, ub{ub_}, nodes{std::move(nodes_)}, status{status_} {}
};
using OutObject = OutObj;

// Owning handle of one device context.
class Device {
    sgufp_ctx *ctx_ = nullptr;

  public:
    Device(const Network &net, int max_batch);
    ~Device();
    Device(const Device &) = delete;
    Device &operator=(const Device &) = delete;
    sgufp_ctx *get() const { return ctx_; }
    void check(int rc, const char *what) const;
};

// RelaxedDDNew (DD.h:797-808) on the device, one DD at a time: the DD is built and kept in
// a device slot (sgufp_dd_* of the C ABI); every call is one kernel launch and returns what
// the reference returns, bit for bit.  DDSolver::startSolver's root DD (DDSolver.cpp:788-791)
// and a NodeExplorer written against the reference's DD class use it unchanged.  For
// throughput use NodeExplorer::process / DDSolver, which batch the same work.
class RelaxedDDNew {
    const Network *networkPtr;
    std::unique_ptr<Device> dev;
    bool built = false, exact = false;
    void upload_cut(const Cut &cut, std::vector<uint64_t> &keys, std::vector<double> &vals) const;

  public:
    explicit RelaxedDDNew(const Network *pointer);
    void buildTree(Node root);
    Path getSolution() const;
    bool isTreeExact() const noexcept { return exact; }
    uint8_t applyFeasibilityCut(const Cut &cut);
    double applyOptimalityCut(const Cut &cut, double optimal, double upperbound);
    std::vector<Node> getCutset(double ub);
};

// The scenario subproblem on the device; returns the cut the reference builds (cutToCut
// order: (i,q,j) ascending, exact zeros dropped, Cut.h:406-421).
class GuroSolver {
    std::shared_ptr<Network> net;
    Device dev;
    std::vector<uint64_t> slot_keys;

  public:
    explicit GuroSolver(const std::shared_ptr<Network> &networkPtr);
    std::pair<CutType, Inavap::Cut> solveSubProblem(const std::vector<int16_t> &path);
};

class NodeExplorer {
    std::shared_ptr<Network> networkPtr;
    Device dev;
    GuroSolver solver;
    const cut_node_t *f_seen = nullptr, *o_seen = nullptr;   // Container heads already on the device
    void sync_pool(int is_feas, const cut_node_t *head, const cut_node_t *&seen);

  public:
    explicit NodeExplorer(const std::shared_ptr<Network> &networkPtr_);
    OutObject process(Node node, double optimalLB, Container &feasCuts, Container &optCuts);
};

// Batched B&B over the device frontier.  nWorkers is kept for the reference's signature;
// the device runs rounds of up to `batch` open nodes (sgufp_bnb_step).
class DDSolver {
    std::shared_ptr<Network> networkPtr;
    const uint16_t N_WORKERS;
    Device dev;
    int batch;
    static constexpr int kDiveBatch = 64;
    double budget = 0.0;
    int seedWidth = 0;
    int maxIters = 0;
    double roundSecs = 0.0;
    double restricted_incumbent(double z);

  public:
    explicit DDSolver(const std::shared_ptr<Network> &networkPtr_, uint16_t nWorkers, int batch = 4096);
    std::pair<double, double> start(double opt);
    double startSolver(double optimal);
    // One shard of a multi-GPU search (one process and one DDSolver per GPU): after every
    // round the shards exchange the incumbent (CAS-max, DDSolver.cpp:723-731), the new cut
    // rows (the global Containers, DDSolver.h:415-416) and work (half-split / 40 % steal,
    // DDSolver.cpp:603-652) over RCCL; the root record starts on rank 0.  id comes from
    // sgufp_comm_unique_id on one rank (SGUFP_COMM_ID_BYTES bytes).
    void shard(int world, int rank, const uint8_t *id);
    // bound a round's exact-leaf refinement loops (sgufp_bnb_set_limits)
    void roundLimits(int maxRefineIters, double roundSeconds);
    // throughput runs of searches that would take hours: stop after `seconds` of search (0:
    // none); the last round's loops are cut at the budget and `complete` stays false
    void timeBudget(double seconds) { budget = seconds; }
    // primal heuristic (0: off): before the search, the restricted half of
    // NodeExplorer::processX3 (NodeExplorer.cpp:605-796) on the root record -- a restricted DD
    // of `width` nodes per layer swept with the pool, its max path sent to the subproblem and
    // the cut added until the path repeats with an unchanged bound -- raises the incumbent to
    // the routing's value, as the reference is seeded with a known value (main.cpp:75)
    void restrictedSeed(int width) { seedWidth = width; }
    bool complete = false;                           // the last search emptied every frontier
    int64_t maxRounds = 0;                           // stop after this many rounds (0: none)
    double heuristicIncumbent = DOUBLE_MIN;          // the seed's value (DOUBLE_MIN: none)
    int64_t received = 0;   // records this shard got through work sharing
    // counters of the last solve (SOLVER_COUNTERS, DDSolver.h:380-392)
    sgufp_bnb_stats totals{};
    // the reference's printWorkerStats report (DDSolver.h:441-501) for the last solve: one
    // "worker" (the device); start() prints it when built with -DSOLVER_COUNTERS
    std::string workerStats() const;
    int64_t rounds = 0;
    sgufp_ctx *context() const { return dev.get(); }
};

}  // namespace Inavap
