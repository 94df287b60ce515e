// Probe: does v_rcp_f64 + ONE Newton step give RN(1/m) for every integer m in [1, N)?
// (Markstein's corrected quotient needs y = RN(1/m).)  Standalone diagnostic, not product code.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned long long n, unsigned long long* bad1, unsigned long long* bad0) {
    unsigned long long m = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x + 1;
    if (m >= n) return;
    const double md = (double)m;
    const double ex = 1.0 / md;
    double y = __builtin_amdgcn_rcp(md);
    if (y != ex) atomicAdd(bad0, 1ull);
    y = __builtin_fma(__builtin_fma(-md, y, 1.0), y, y);
    if (y != ex) atomicAdd(bad1, 1ull);
}
int main() {
    const unsigned long long n = 1ull << 26;
    unsigned long long *d, h[2];
    hipMalloc(&d, 16);
    hipMemset(d, 0, 16);
    hipLaunchKernelGGL(k, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, n, d, d + 1);
    hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    printf("m in [1, 2^26): rcp+1NR mismatches %llu, bare v_rcp_f64 mismatches %llu\n", h[0], h[1]);
    return 0;
}
