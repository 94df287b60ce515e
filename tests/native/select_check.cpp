// CPU check of signature_kmers_amd/csrc/skm_select.h (the device's restatement of libstdc++
// std::nth_element and the older Boost.Math median / MAD) against std::nth_element itself, on
// tie-heavy random arrays: identical permutations, identical (median, mad) bits.
// Build: g++ -O2 -std=c++17 -I signature_kmers_amd/csrc tests/native/select_check.cpp
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "skm_select.h"

static float ref_median(std::vector<float>& v) {  // boost::math::statistics::median
    size_t n = v.size();
    if (n & 1) {
        auto m = v.begin() + (n - 1) / 2;
        std::nth_element(v.begin(), m, v.end());
        return *m;
    }
    auto m = v.begin() + n / 2 - 1;
    std::nth_element(v.begin(), m, v.end());
    std::nth_element(m, m + 1, v.end());
    return (*m + *(m + 1)) / 2;
}

static float ref_mad_legacy(std::vector<float>& v) {  // median_absolute_deviation returning |x(mid)|
    float c = ref_median(v);
    size_t n = v.size();
    auto cmp = [&c](float a, float b) { return std::abs(a - c) < std::abs(b - c); };
    if (n & 1) {
        auto m = v.begin() + (n - 1) / 2;
        std::nth_element(v.begin(), m, v.end(), cmp);
        return std::abs(*m);
    }
    auto m = v.begin() + n / 2 - 1;
    std::nth_element(v.begin(), m, v.end(), cmp);
    std::nth_element(m, m + 1, v.end(), cmp);
    return (std::abs(*m) + std::abs(*(m + 1))) / std::abs(2.0f);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 20000;
    std::mt19937_64 rng(12345);
    long bad_perm = 0, bad_stat = 0, checked = 0;
    for (int it = 0; it < iters; ++it) {
        const uint32_t n = 1 + (uint32_t)(rng() % (it % 10 == 0 ? 20000 : 300));
        const uint32_t span = 1 + (uint32_t)(rng() % (it % 3 == 0 ? 4 : 200));
        const uint32_t base = (uint32_t)(rng() % 3000);
        std::vector<uint32_t> x(n);
        for (auto& e : x) e = base + (uint32_t)(rng() % span);
        if (it % 7 == 0) std::sort(x.begin(), x.end());                         // presorted
        if (it % 11 == 0) std::sort(x.begin(), x.end(), std::greater<uint32_t>());  // reversed
        // 1. one nth_element, plain order
        {
            const uint32_t nth = (uint32_t)(rng() % n);
            std::vector<float> a(x.begin(), x.end());
            std::vector<uint32_t> b = x;
            std::nth_element(a.begin(), a.begin() + nth, a.end());
            stl_nth_element(b.data(), 0, nth, n, [](uint32_t p, uint32_t q) { return p < q; });
            for (uint32_t i = 0; i < n; ++i)
                if ((uint32_t)a[i] != b[i]) {
                    ++bad_perm;
                    break;
                }
        }
        // 2. the legacy median + MAD sequence
        {
            std::vector<float> a(x.begin(), x.end());
            std::vector<uint32_t> b = x;
            const float med_ref = ref_median(a);       // HitSet::process: median(v) ...
            const float mad_ref = ref_mad_legacy(a);   // ... then MAD(v), which recomputes the median
            float med = 0, mad = 0;
            legacy_median_mad(b.data(), n, med, mad);
            if (std::memcmp(&med, &med_ref, 4) || std::memcmp(&mad, &mad_ref, 4)) ++bad_stat;
            for (uint32_t i = 0; i < n; ++i)
                if ((uint32_t)a[i] != b[i]) {
                    ++bad_perm;
                    break;
                }
        }
        ++checked;
    }
    std::printf("checked %ld bad_perm %ld bad_stat %ld\n", checked, bad_perm, bad_stat);
    return (bad_perm || bad_stat) ? 1 : 0;
}
