// ThreadSanitizer check of Inavap::Container (include/sgufp/inavap.hpp), the lock-free cut pool
// every worker of the reference's DDSolver adds to and reads from (Cut.h:448-485,
// DDSolver.h:415-416): writer threads add cuts while reader threads walk the list from an
// acquired head (NodeExplorer::process snapshots the heads, NodeExplorer.cpp:930-931).  Built
// with -fsanitize=thread by tests/test_host_api.py; a race report fails the run.
#include <sgufp/inavap.hpp>

#include <atomic>
#include <cstdio>
#include <thread>
#include <vector>

int main() {
    constexpr int kWriters = 4, kReaders = 4, kPerWriter = 2000;
    Inavap::Container pool;
    std::atomic<int> done{0};
    std::vector<std::thread> th;
    for (int w = 0; w < kWriters; w++)
        th.emplace_back([&, w]() {
            for (int i = 0; i < kPerWriter; i++) {
                std::vector<std::pair<uint64_t, double>> c{{Inavap::getKey(1, 2, 3), (double)(w * kPerWriter + i)}};
                pool.add(new Inavap::cut_node_t(Inavap::Cut((double)i, c)));
            }
            done.fetch_add(1);
        });
    std::atomic<long> seen{0};
    for (int r = 0; r < kReaders; r++)
        th.emplace_back([&]() {
            while (done.load() < kWriters) {
                long n = 0;
                double acc = 0.0;
                for (const Inavap::cut_node_t *p = pool.get(); p; p = p->next) {
                    acc += p->cut.RHS + p->cut.coeff[0].second;   // read every published cut
                    n++;
                }
                seen.fetch_add(n > 0 && acc >= 0.0 ? 1 : 0);
            }
        });
    for (auto &t : th) t.join();
    long total = 0;
    for (const Inavap::cut_node_t *p = pool.get(); p; p = p->next) total++;
    std::printf("cuts %ld (expected %d), reader passes %ld\n", total, kWriters * kPerWriter, seen.load());
    return total == kWriters * kPerWriter ? 0 : 1;
}
