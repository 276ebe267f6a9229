// ThreadSanitizer driver for csrc/host_pool.h (tests/test_host_sanitizers.py):
// several caller threads submit jobs to the shared pool at once, as the bench's
// enqueue threads do (one msg_render_batch per context); every index of every
// job must run exactly once and each run() must return only after its own
// job finished.  Exit code 0 = pass; TSan reports fail the test.
#include <atomic>
#include <cstdio>
#include <thread>
#include <vector>

#include "host_pool.h"

int main() {
    constexpr int CALLERS = 4, JOBS = 150;
    std::atomic<int> bad{0};
    std::vector<std::thread> callers;
    for (int c = 0; c < CALLERS; ++c) {
        callers.emplace_back([c, &bad] {
            for (int j = 0; j < JOBS; ++j) {
                const int n = 1 + (j * 37 + c * 11) % 97;
                std::vector<int> hits(n, 0);          // plain ints: written by whichever thread ran the index
                long sum = 0;
                std::atomic<long> asum{0};
                HostPool::get().run(n, [&](int i) {
                    hits[i] += 1;
                    asum.fetch_add(i);
                });
                for (int i = 0; i < n; ++i) {
                    if (hits[i] != 1) bad.fetch_add(1);
                    sum += i;
                }
                if (asum.load() != sum) bad.fetch_add(1);
            }
        });
    }
    for (auto& t : callers) t.join();
    std::printf("pool threads %d, bad %d\n", HostPool::get().threads(), bad.load());
    return bad.load() == 0 ? 0 : 1;
}
