// CPU check of csrc/skm_pool.h (the host pool that packs skm_build_add_batch's residues): every
// part of every run executes exactly once, runs of 0 / 1 / many parts, back-to-back runs with no
// lost wake-ups, and a byte-balanced packing of random sequences equals the serial packing.
#include <atomic>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "skm_pool.h"

int main() {
    int bad = 0;
    for (int threads : {1, 2, 7, 16}) {
        skm::HostPool pool(threads);
        std::vector<std::atomic<int>> hits(4096);
        for (int it = 0; it < 2000; ++it) {
            const int n = (it * 37) % 300;
            for (int p = 0; p < n; ++p) hits[p].store(0);
            pool.run(n, [&](int p) { hits[p].fetch_add(1); });
            for (int p = 0; p < n; ++p) bad += hits[p].load() != 1;
        }
        // packing: sequences of random lengths into one buffer with a 0 separator each
        std::mt19937_64 rng(threads);
        const size_t ns = 20000;
        std::vector<uint32_t> len(ns);
        std::vector<uint64_t> cum(ns + 1, 0);
        for (size_t s = 0; s < ns; ++s) {
            len[s] = (uint32_t)(rng() % 700);
            cum[s + 1] = cum[s] + len[s] + 1;
        }
        std::vector<uint8_t> src(cum[ns]), a(cum[ns], 0xAA), b(cum[ns], 0x55);
        for (auto& c : src) c = (uint8_t)('A' + rng() % 20);
        for (size_t s = 0; s < ns; ++s) {
            std::memcpy(&a[cum[s]], &src[cum[s]], len[s]);
            a[cum[s] + len[s]] = 0;
        }
        const uint64_t bytes = cum[ns];
        const int parts = 4 * pool.threads();
        pool.run(parts, [&](int p) {
            const uint64_t lo = bytes * p / parts, hi = bytes * (p + 1) / parts;
            const size_t x = std::lower_bound(cum.begin(), cum.begin() + ns, lo) - cum.begin();
            const size_t e = std::lower_bound(cum.begin(), cum.begin() + ns, hi) - cum.begin();
            for (size_t s = x; s < e; ++s) {
                std::memcpy(&b[cum[s]], &src[cum[s]], len[s]);
                b[cum[s] + len[s]] = 0;
            }
        });
        bad += a != b;
    }
    std::printf("pool bad %d\n", bad);
    return bad != 0;
}
