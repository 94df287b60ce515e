// gather_probe -- the random-access ceiling of the annotate lookup: the same
// number of independent random 4-byte gathers k_lookup<0> makes (3 into the interleaved g/rank
// lines, 1 dependent into the 4-byte records), over tables of the C2 DB's sizes, with no hashing
// or window logic.  Build: hipcc --offload-arch=gfx950 -O3 -x hip tools/gather_probe.cpp -o bin/gather_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

// mode 0: 3 line gathers + 1 dependent record gather per window (the lookup's pattern)
// mode 1: 1 record gather per window     mode 2: 3 line gathers per window
// mode 3: streaming read of n windows' worth of 1 byte (the residue stream), for scale
__global__ void k_probe(const uint32_t* __restrict__ lines, uint64_t nlines_words, const uint32_t* __restrict__ recs,
                        uint64_t nrecs, uint64_t n, int mode, uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t h = mix(i + 0x9e3779b97f4a7c15ull);
        if (mode == 3) {
            acc += reinterpret_cast<const uint8_t*>(lines)[i % (nlines_words * 4)];
            continue;
        }
        uint32_t r = (uint32_t)h;
        if (mode != 1) {
            const uint32_t a = lines[(h % nlines_words)];
            const uint32_t b = lines[((h >> 21) * 0x9e3779b1ull) % nlines_words];
            const uint32_t c = lines[((h >> 42) * 0x85ebca6bull) % nlines_words];
            r = a + b + c + (uint32_t)h;
            acc ^= r;
        }
        if (mode != 2) acc += recs[mix(r) % nrecs];
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 606345516ull;      // windows
    const uint64_t line_bytes = argc > 2 ? strtoull(argv[2], nullptr, 10) : 103ull << 20;  // g/rank lines
    const uint64_t rec_bytes = argc > 3 ? strtoull(argv[3], nullptr, 10) : 675ull << 20;   // records
    uint32_t *lines, *recs, *out;
    CK(hipMalloc(&lines, line_bytes));
    CK(hipMalloc(&recs, rec_bytes));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(lines, 1, line_bytes));
    CK(hipMemset(recs, 2, rec_bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* names[4] = {"lookup pattern (3 line + 1 record gathers)", "record gathers only",
                            "line gathers only (3)", "streaming 1 B/window"};
    const int gathers[4] = {4, 1, 3, 0};
    for (int mode = 0; mode < 4; ++mode) {
        float best = 1e30f;
        for (int rep = 0; rep < 4; ++rep) {
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(k_probe, dim3(256 * 64), dim3(256), 0, 0, lines, line_bytes / 4, recs, rec_bytes / 4, n,
                               mode, out);
            CK(hipGetLastError());
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep && ms < best) best = ms;
        }
        printf("{\"mode\": %d, \"what\": \"%s\", \"windows\": %llu, \"ms\": %.3f, \"gathers_per_s\": %.4g}\n", mode,
               names[mode], (unsigned long long)n, best, gathers[mode] * (double)n / (best * 1e-3));
    }
    CK(hipFree(lines));
    CK(hipFree(recs));
    CK(hipFree(out));
    return 0;
}
