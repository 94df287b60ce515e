// fetch_calib -- calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE against known byte counts for the
// access shapes of this repo's kernels (roofline.traffic in bench.py): coalesced 16-byte and
// 8-byte per-lane streaming reads, a coalesced 8-byte streaming write, and independent random
// 8-byte / 4-byte gathers over a table far beyond the Infinity Cache.  Each kernel runs once;
// the byte count each one moves is printed, to be divided into the counter of its dispatch.
// Build: hipcc --offload-arch=gfx950 -O3 -x hip tools/probes/fetch_calib.hip -o bin/fetch_calib
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

__global__ void k_read16(const uint4* __restrict__ a, uint64_t n, unsigned long long* out) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) atomicAdd(out, 1ull);
}

__global__ void k_read8(const uint64_t* __restrict__ a, uint64_t n, unsigned long long* out) {
    uint64_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        acc ^= a[i];
    if (acc == 0x1234567812345678ull) atomicAdd(out, 1ull);
}

__global__ void k_write8(uint64_t* __restrict__ a, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        a[i] = i * 0x9E3779B97F4A7C15ull;
}

__device__ __forceinline__ uint64_t mix(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

template <class T>
__global__ void k_gather(const T* __restrict__ a, uint64_t nt, uint64_t ng, unsigned long long* out) {
    uint64_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ng; i += (uint64_t)gridDim.x * blockDim.x)
        acc = acc * 0x9E3779B97F4A7C15ull + (uint64_t)a[mix(i) % nt];  // every bit live: no load elided
    if (acc == 0x1234567812345678ull) atomicAdd(out, 1ull);
}

int main() {
    const uint64_t bytes = 4ull << 30;  // 4 GiB: beyond the 256 MB Infinity Cache
    uint8_t* a = nullptr;
    unsigned long long* out = nullptr;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&out, 8));
    CK(hipMemset(a, 1, bytes));
    CK(hipDeviceSynchronize());
    const dim3 g(4096), b(256);
    const uint64_t ng = 1ull << 26;
    hipLaunchKernelGGL(k_read16, g, b, 0, 0, reinterpret_cast<const uint4*>(a), bytes / 16, out);
    hipLaunchKernelGGL(k_read8, g, b, 0, 0, reinterpret_cast<const uint64_t*>(a), bytes / 8, out);
    hipLaunchKernelGGL(k_write8, g, b, 0, 0, reinterpret_cast<uint64_t*>(a), bytes / 8);
    hipLaunchKernelGGL(k_gather<uint64_t>, g, b, 0, 0, reinterpret_cast<const uint64_t*>(a), bytes / 8, ng, out);
    hipLaunchKernelGGL(k_gather<uint32_t>, g, b, 0, 0, reinterpret_cast<const uint32_t*>(a), bytes / 4, ng, out);
    CK(hipDeviceSynchronize());
    printf("{\"k_read16\": %llu, \"k_read8\": %llu, \"k_write8\": %llu, \"k_gather<unsigned long>\": %llu, "
           "\"k_gather<unsigned int>\": %llu}\n",
           (unsigned long long)bytes, (unsigned long long)bytes, (unsigned long long)bytes,
           (unsigned long long)(ng * 8), (unsigned long long)(ng * 4));
    CK(hipFree(a));
    CK(hipFree(out));
    return 0;
}
