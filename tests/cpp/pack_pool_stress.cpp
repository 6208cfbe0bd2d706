// Stress test of the staging thread pool (noetic-slam_amd/csrc/pack_pool.h) on the CPU: run() over
// all parts, start()/wait() of several pools side by side with part offsets (tsdf_integrate_sectors'
// pattern), back to back and with pauses long enough for the workers to fall asleep.  Every part
// must run exactly once per job; exits non-zero on the first miss.
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "../../noetic-slam_amd/csrc/pack_pool.h"

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 2000;
    tsdf::PackPool a(3), b(2), c(4);
    const int total = a.parts() + (b.parts() - 1) + (c.parts() - 1);
    std::vector<std::atomic<int>> hits(total);
    for (int r = 0; r < rounds; r++) {
        for (auto& h : hits) h.store(0);
        auto f = [&](int part) { hits[part].fetch_add(1); };
        if (r % 3 == 0) {  // one pool
            a.run(f);
            for (int p = 0; p < a.parts(); p++)
                if (hits[p].load() != 1) { std::printf("run: part %d ran %d times (round %d)\n", p, hits[p].load(), r); return 1; }
            continue;
        }
        // three pools, the second and third through start(base) / wait()
        b.start(f, a.parts() - 1);
        c.start(f, a.parts() + b.parts() - 2);
        a.run(f);
        b.wait();
        c.wait();
        for (int p = 0; p < total; p++)
            if (hits[p].load() != 1) { std::printf("multi: part %d ran %d times (round %d)\n", p, hits[p].load(), r); return 1; }
        if (r % 97 == 0) std::this_thread::sleep_for(std::chrono::microseconds(400));  // let them sleep
    }
    std::printf("ok %d rounds, %d parts\n", rounds, total);
    return 0;
}
