// Drives the C++ host mirror (include/sgufp/inavap.hpp) the way the reference's main /
// workers do (main.cpp:56-81, DDSolver.cpp:658-776), for tests/test_host_api.py:
//
//   host_api_test <network file> <known optimum as hex float | none>
//
// prints "ddsolver <optimum %a>" (Inavap::DDSolver::start, batched device rounds) and
// "explorer <optimum %a> <processed>" (a single-worker LIFO loop over
// Inavap::NodeExplorer::process with two global Containers, as Worker::startWorker).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <vector>

#include "sgufp/inavap.hpp"

int main(int argc, char **argv) {
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
