// skm_select.h -- GNU libstdc++ std::nth_element restated (host and device), and the older
// Boost.Math median / median_absolute_deviation built on it (mad_mode 1).  Header-only so the CPU
// tests compile the same code against std::nth_element itself (tests/test_select_cpu.py).
#pragma once
#include <cstdint>

#ifndef SKM_HD
#if defined(__HIPCC__)
#define SKM_HD __host__ __device__
#else
#define SKM_HD
#endif
#endif

// ---- Boost.Math <= 1.75 median_absolute_deviation (mad_mode 1, call_functions.tcc:51-53) ----
// That version returns |x| of the element(s) std::nth_element places at the middle under the
// |x - median| order, not |x - median|: with ties in distance (x = median - d and median + d) the
// value depends on the permutation GNU libstdc++'s introselect produces, after the two
// nth_element calls of boost::math::statistics::median have already reordered the hit-order
// array.  Restated here from the published libstdc++ algorithm (bits/stl_algo.h __introselect,
// __unguarded_partition_pivot, __move_median_to_first, __insertion_sort, __heap_select and
// bits/stl_heap.h __adjust_heap / __push_heap), one lane, in place.  Values are integer-valued
// floats, so `less` is integer order and the distance order is |2x - C2| with C2 = 2 * median.
template <class T, class Less>
SKM_HD void stl_push_heap(T* f, int64_t hole, int64_t top, T val, Less lt) {
    int64_t parent = (hole - 1) / 2;
    while (hole > top && lt(f[parent], val)) {
        f[hole] = f[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    f[hole] = val;
}
template <class T, class Less>
SKM_HD void stl_adjust_heap(T* f, int64_t hole, int64_t len, T val, Less lt) {
    const int64_t top = hole;
    int64_t child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (lt(f[child], f[child - 1])) --child;
        f[hole] = f[child];
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        f[hole] = f[child - 1];
        hole = child - 1;
    }
    stl_push_heap(f, hole, top, val, lt);
}
template <class T, class Less>
SKM_HD void stl_heap_select(T* f, int64_t mid, int64_t last, Less lt) {
    if (mid >= 2)  // make_heap over [0, mid)
        for (int64_t parent = (mid - 2) / 2;; --parent) {
            stl_adjust_heap(f, parent, mid, f[parent], lt);
            if (parent == 0) break;
        }
    for (int64_t i = mid; i < last; ++i)
        if (lt(f[i], f[0])) {  // pop_heap(first, middle, i)
            const T v = f[i];
            f[i] = f[0];
            stl_adjust_heap(f, 0, mid, v, lt);
        }
}
template <class T, class Less>
SKM_HD void stl_nth_element(T* v, int64_t first, int64_t nth, int64_t last, Less lt) {
    if (first == last || nth == last) return;
    int depth = 0;
    for (uint64_t m = (uint64_t)(last - first); m > 1; m >>= 1) ++depth;  // std::__lg
    depth *= 2;
    auto swp = [&](int64_t a, int64_t b) {
        const T t = v[a];
        v[a] = v[b];
        v[b] = t;
    };
    while (last - first > 3) {
        if (depth == 0) {
            stl_heap_select(v + first, nth + 1 - first, last - first, lt);
            swp(first, nth);
            return;
        }
        --depth;
        // __unguarded_partition_pivot: median of (first+1, mid, last-1) moved to first
        const int64_t mid = first + (last - first) / 2, a = first + 1, b = mid, c = last - 1;
        if (lt(v[a], v[b])) {
            if (lt(v[b], v[c])) swp(first, b);
            else if (lt(v[a], v[c])) swp(first, c);
            else swp(first, a);
        } else if (lt(v[a], v[c])) {
            swp(first, a);
        } else if (lt(v[b], v[c])) {
            swp(first, c);
        } else {
            swp(first, b);
        }
        int64_t lo = first + 1, hi = last;  // __unguarded_partition(first + 1, last, first)
        for (;;) {
            while (lt(v[lo], v[first])) ++lo;
            --hi;
            while (lt(v[first], v[hi])) --hi;
            if (!(lo < hi)) break;
            swp(lo, hi);
            ++lo;
        }
        if (lo <= nth)
            first = lo;
        else
            last = lo;
    }
    for (int64_t i = first + 1; i < last; ++i) {  // __insertion_sort(first, last)
        const T val = v[i];
        if (lt(val, v[first])) {
            for (int64_t k = i; k > first; --k) v[k] = v[k - 1];
            v[first] = val;
        } else {
            int64_t k = i;
            while (lt(val, v[k - 1])) {
                v[k] = v[k - 1];
                --k;
            }
            v[k] = val;
        }
    }
}

// boost::math::statistics::median (nth_element, and for even n a second one on the upper part)
// followed by the older median_absolute_deviation, over v[0..n) in hit order, permuting v exactly
// as the reference does: median() in HitSet::process, then median_absolute_deviation(v) (default
// center = NaN) recomputes the median on the permuted array before its own selections.
template <class T>
SKM_HD void legacy_median_mad(T* v, uint32_t n, float& median, float& mad) {
    auto lt = [](T x, T y) { return (uint32_t)x < (uint32_t)y; };
    uint32_t C2 = 0;
    for (int rep = 0; rep < 2; ++rep) {
        if (n & 1) {
            const int64_t mid = (n - 1) / 2;
            stl_nth_element(v, 0, mid, n, lt);
            median = (float)(uint32_t)v[mid];
            C2 = 2u * (uint32_t)v[mid];
        } else {
            const int64_t mid = n / 2 - 1;
            stl_nth_element(v, 0, mid, n, lt);
            stl_nth_element(v, mid, mid + 1, n, lt);
            const uint32_t a = v[mid], b = v[mid + 1];
            median = ((float)a + (float)b) / 2;
            C2 = a + b;
        }
    }
    auto dist = [C2](T x) {
        const int32_t d = 2 * (int32_t)(uint32_t)x - (int32_t)C2;
        return (uint32_t)(d < 0 ? -d : d);
    };
    auto dl = [&](T x, T y) { return dist(x) < dist(y); };
    if (n & 1) {
        const int64_t mid = (n - 1) / 2;
        stl_nth_element(v, 0, mid, n, dl);
        mad = (float)(uint32_t)v[mid];  // |x|, not |x - median|
    } else {
        const int64_t mid = n / 2 - 1;
        stl_nth_element(v, 0, mid, n, dl);
        stl_nth_element(v, mid, mid + 1, n, dl);
        mad = ((float)(uint32_t)v[mid] + (float)(uint32_t)v[mid + 1]) / 2.0f;
    }
}

