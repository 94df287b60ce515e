// skm_build.hip -- signature build on MI355X (gfx950).
//
// Replaces the reference's SignatureBuilder<8>::extract_kmers + process_kmers
// (signature_build.tcc:48-293): sliding 8-mer extraction, grouping of equal k-mers, the 80 %
// best-function cut and the per-k-mer statistics, with `--n-threads 1` semantics.
//
// Device pipeline (one GPU; the multi-GPU form inserts an RCCL all-to-all between 3 and 4):
//   1. k_extract<count>   residues -> per-workgroup histogram of level-1 buckets (LDS atomics)
//   2. k_colsum/k_bstart/k_coloffs   exclusive scan of the [workgroup][bucket] matrix
//   3. k_extract<scatter> residues -> 16-byte occurrence elements (SoA hi/lo, see make_elem),
//                         partitioned by level-1 bucket (owner-major)
//   4. k_bucket_process   one workgroup per level-1 bucket: level-2 partition in HBM, then per
//                         sub-bucket LDS hash grouping, cut, statistics (short P^2/variance
//                         chains inline, long ones deferred as jobs), compaction of kept k-mers
//   5. k_overflow         sub-buckets larger than LDS: global-memory bitonic sort + the same
//                         group processing
//   6. k_job_* / k_chains deferred P^2 median / variance recurrences, longest first
//   7. k_func_hist_* / k_count_flags   distinct_functions, seqs_with_func, signature flags
//
// Exactness notes: group members are visited in reverse ordinal order
// (TBB 2020 multimap LIFO), the cut is fp32 `(float)best < (float)count*0.8f`, statistics are
// the Boost.Accumulators recurrences in fp64 with contraction disabled (-ffp-contract=off).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "skm_common.h"
#include "skm_pool.h"
#include "skm_output.h"
#include "skm_util.h"

#if defined(SKM_WITH_RCCL)
#include <rccl/rccl.h>
#endif

namespace skm {

// ------------------------------------------------------------------------------------------
// Tunables
// ------------------------------------------------------------------------------------------
constexpr int EX_THREADS = 512;        // extract workgroup
constexpr int EX_POS_PER_THREAD = 16;  // windows per thread per step (one 16-byte load + halo)
constexpr int EX_MAX_WG = 512;         // rows of the histogram matrix
constexpr int SCAN_ROWS = 32;          // rows per column-scan block
constexpr int BP_THREADS = 512;        // bucket-process workgroup: two per CU (LDS ~72 KB each)
constexpr int CAP = 2048;              // LDS sub-bucket capacity (records)
#ifndef SKM_BPK_THREADS                // k_bucket_process workgroup (A/B builds: -DSKM_BPK_THREADS=256)
#define SKM_BPK_THREADS 512
#endif
constexpr int BPK_THREADS = SKM_BPK_THREADS;
constexpr int BPK_WAVES_EU = BPK_THREADS == 512 ? 4 : 2;  // two workgroups per CU (LDS ~78 KB each)
constexpr int TAB_BITS = 12;
constexpr int TAB = 1 << TAB_BITS;     // LDS hash slots per sub-bucket (load <= 0.5)
// target records per level-2 sub-bucket.  768 (round 6, C3 A/B on one box, three alternations each):
// k_bucket_process 642 -> 617, overflow path 500 -> 450 ms of GPU time per step; the step itself
// 1357 -> 1349 ms (within noise: the partition's 200 / 245 ms spread between runs dominates);
// 512 takes the group-by to 600 ms but slows the partition as much
constexpr int SUB_TARGET = 768;
constexpr int MAX_B2 = 11;             // <= 2048 sub-buckets per level-1 bucket
constexpr int SUB_TAB = (1 << MAX_B2) + 2;  // per-bucket sub-bucket table: count + offsets

struct SeqMeta {        // 16 bytes, one dwordx4 load
    uint64_t pstart;    // first residue in the packed buffer
    uint32_t len;       // protein length
    uint16_t func;      // FunctionIndex
    uint16_t pad;
};

struct OvfEntry {
    uint64_t off;       // first record (in the records buffer given to the overflow kernel)
    uint32_t n;         // records
    uint32_t bucket;    // level-1 bucket (hash prefix)
    uint64_t scratch;   // element offset in scratch (host fills)
    uint32_t npad;      // pow2 >= n (host fills)
    uint32_t src;       // 0 = recs, 1 = tmp
};

// ------------------------------------------------------------------------------------------
// Device helpers
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint16_t d2u16(double d) {
    // gcc/x86-64: cvttsd2si to int32 then keep 16 bits; out of range -> 0x80000000 -> 0
    if (!(d > -2147483649.0 && d < 2147483648.0)) return 0;
    return (uint16_t)(int32_t)d;
}

// ------------------------------------------------------------------------------------------
// Exact fp64 division without the division on the dependent chain.  Every divisor in the
// statistics recurrences is an integer m (marker position differences, sample counts), so
//   y = RN(1/m): v_rcp_f64 + two Newton steps (error ~2^-92 relative; 1/m of an integer below
//                2^45 is never within 2^-75 of a rounding midpoint, so the last FMA rounds to
//                RN(1/m) exactly), computed as soon as m is known, off the height chain;
//   RN(a/m) = fma(fma(-q, m, a), y, q) with q = RN(a*y)  (Markstein's correction theorem:
//                y within 1/2 ulp of 1/m and q within 1 ulp of a/m give the correctly
//                rounded quotient).
// Bit-identical to IEEE division (checked against the CPU oracle by the parity tests and by
// skm_debug_div_check on the device).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ double rcp_int(double m) {
    double y = __builtin_amdgcn_rcp(m);
    y = __builtin_fma(__builtin_fma(-m, y, 1.0), y, y);
    y = __builtin_fma(__builtin_fma(-m, y, 1.0), y, y);
    return y;
}
__device__ __forceinline__ double div_by(double a, double m, double y) {
    const double q = a * y;
    return __builtin_fma(__builtin_fma(-q, m, a), y, q);
}

// Boost.Accumulators p_square_quantile(p=0.5) + lazy mean over a u16 sum + immediate variance.
// P^2 parabolic height update of one marker (Boost p_square_quantile): neighbours
// hm_ / hp_, actual-position gaps dp = n[i+1]-n[i] > 1 or dm = n[i-1]-n[i] < -1, direction
// sg = +-1.  Quotients by integers take the reciprocal + corrected-quotient route; sg / (dp - dm)
// is exactly +-RN(1/(dp - dm)), so the product by it is +-RN(ym * S) (same rounding).
__device__ __forceinline__ double p2_height_y(double hm_, double H, double hp_, int32_t dpi, int32_t dmi, int32_t sgi,
                                              double ydp, double ydm, double ym) {
    const double dp = (double)dpi, dm = (double)dmi;
    const double hp = div_by(hp_ - H, dp, ydp);
    const double hm = div_by(hm_ - H, dm, ydm);
    const double t = ym * ((double)(sgi - dmi) * hp + (double)(dpi - sgi) * hm);
    const double hh = sgi > 0 ? H + t : H - t;
    const double lin = sgi > 0 ? H + hp : H - hm;
    return (hm_ < hh && hh < hp_) ? hh : lin;
}
__device__ __forceinline__ double p2_height(double hm_, double H, double hp_, int32_t dpi, int32_t dmi, int32_t sgi) {
    return p2_height_y(hm_, H, hp_, dpi, dmi, sgi, rcp_int((double)dpi), rcp_int((double)dmi),
                       rcp_int((double)(dpi - dmi)));
}

struct SigStats {
    double h[5];
    int32_t act[5];
    uint32_t cnt;
    uint16_t sum;
    double var;

    __device__ void init() {
        for (int i = 0; i < 5; ++i) {
            h[i] = 0.0;
            act[i] = i + 1;
        }
        cnt = 0;
        sum = 0;
        var = 0.0;
    }

    __device__ void add_p2(uint32_t sample) {
        ++cnt;
        const double x = (double)sample;
        // ---- p_square_quantile ----
        if (cnt <= 5) {
#pragma unroll
            for (int i = 0; i < 5; ++i)
                if ((uint32_t)i == cnt - 1) h[i] = x;
            if (cnt == 5) {  // std::sort of 5 values (result is the unique sorted order)
#pragma unroll
                for (int i = 0; i < 5; ++i)
#pragma unroll
                    for (int j = 0; j < 4 - i; ++j) {  // bubble network: same sorted values as std::sort
                        const double a = h[j], b = h[j + 1];
                        h[j] = a > b ? b : a;
                        h[j + 1] = a > b ? a : b;
                    }
            }
        } else {
            // cell k with heights[k-1] <= x < heights[k] (std::upper_bound), extremes adjusted.
            // Branch-free: with sorted heights the cell is 1 + #{k in 1..3 : heights[k] <= x} in
            // all three cases (x < h0 -> 1, h4 <= x -> 4).
            const int cell = 1 + (h[1] <= x ? 1 : 0) + (h[2] <= x ? 1 : 0) + (h[3] <= x ? 1 : 0);
            h[0] = x < h[0] ? x : h[0];
            h[4] = h[4] <= x ? x : h[4];
#pragma unroll
            for (int i = 1; i < 5; ++i)
                if (i >= cell) act[i] += 1;
            // Desired positions accumulate exact multiples of 1/4 (desired_i = i+1 + (cnt-5)*i/4),
            // actual positions are integers: d, dp, dm and the adjust decision are exact in
            // quarter units, so only the height update itself needs fp64 (bit-identical).  Its
            // three divisions by integers take the reciprocal + corrected-quotient route.
            const int32_t k4 = (int32_t)(cnt - 5);
#pragma unroll
            for (int i = 1; i <= 3; ++i) {
                const int32_t d4 = 4 * (i + 1) + k4 * i - 4 * act[i];  // 4*d
                const int32_t dpi = act[i + 1] - act[i];
                const int32_t dmi = act[i - 1] - act[i];
                // (a branch-free form -- the height computed for every lane and selected -- measured
                // slower: 744 vs 514 ns/sample with 16 chains per wave, markers often adjust in no lane)
                if ((d4 >= 4 && dpi > 1) || (d4 <= -4 && dmi < -1)) {
                    const int32_t sgi = d4 > 0 ? 1 : -1;  // d / |d|, exactly +-1
                    h[i] = p2_height(h[i - 1], h[i], h[i + 1], dpi, dmi, sgi);
                    act[i] += sgi;
                }
            }
        }
    }
    // variance (immediate); its mean is the lazy sum/count over the u16 sum
    __device__ void add_var(uint32_t sample) {
        ++cnt;
        sum = (uint16_t)(sum + sample);
        const double x = (double)sample;
        if (cnt > 1) {
            const double c = (double)cnt, c1 = (double)(cnt - 1);
            const double yc = rcp_int(c), yc1 = rcp_int(c1);
            const double mean = div_by((double)sum, c, yc);
            const double tmp = x - mean;
            const double t2 = div_by(tmp * tmp, c1, yc1);
            var = div_by(var * c1, c, yc) + t2;
        }
    }
};

constexpr uint32_t REM_MASK = 0x7FFFFFFFu;   // rem <= 31 bits; bit 47 of hi is the big-length flag

// The 43-bit hashed key of an element from its level-1 bucket prefix and its 31-bit rem field.
// With key-range passes, a heavy k-mer may be grouped in an earlier pass than its hash names
// (k_pass_ids routes it; pass = top pass_bits of the hash): its rem field then carries (natural
// pass ^ this pass) above the rem bits, which restores the natural pass bits (pshift = 43 - pass
// bits); the bits are 0 for every other element.  Grouping compares the whole rem field, so keys
// routed in from different passes never merge.
__device__ __forceinline__ uint64_t key_h43(uint64_t hprefix, uint64_t remf, int rem_bits, int pshift) {
    return (hprefix ^ ((remf >> rem_bits) << pshift)) | (remf & ((1ull << rem_bits) - 1ull));
}

// protein length of an element: carried mod 2^16 unless the big-length flag is set
__device__ __forceinline__ uint32_t elem_len(uint64_t hi, uint64_t lo, const uint32_t* __restrict__ glen) {
    return ((hi >> 47) & 1u) ? glen[lo >> 36] : (uint32_t)(hi >> 48);
}

// 16-byte occurrence element (written by the extract-scatter kernel, read by the bucket kernel):
//   hi = len mod 2^16 << 48 | (len > 65535) << 47 | rem << 16 | func     (rem <= 31 bits)
//   lo = s << 36 | i << 16 | (len - i) mod 2^16                           (s = global sequence index)
// Everything the group-by needs rides in the element, so the bucket kernel never gathers
// per-sequence metadata (lo order = insertion order: sequence, then window).
__device__ __forceinline__ void make_elem(uint64_t rem, uint32_t s, uint32_t i, const SeqMeta& m, uint64_t& ohi,
                                          uint64_t& olo) {
    const uint32_t off16 = (m.len - i) & 0xFFFFu;
    ohi = ((uint64_t)(m.len & 0xFFFFu) << 48) | ((uint64_t)(m.len > 0xFFFFu) << 47) | (rem << 16) | m.func;
    olo = ((uint64_t)s << 36) | ((uint64_t)i << 16) | off16;
}

__device__ __forceinline__ bool elem_less(uint64_t ah, uint64_t al, uint64_t bh, uint64_t bl) {
    return ah < bh || (ah == bh && al < bl);
}

// Bitonic network over hi/lo[0..N) restricted to stages k in [kmin..kmax] (pow2), strides j of
// those stages up to jtop.  Ascending-only network: the first step of stage k pairs i with its mirror i ^ (k - 1) in the
// k-block, the later steps are half-cleaners; every block ends ascending, so maximum-key padding
// at the top never moves and work on it can be skipped.
__device__ void bitonic_lds(uint64_t* hi, uint64_t* lo, uint32_t N, uint32_t kmin, uint32_t kmax, uint32_t jtop) {
    for (uint32_t k = kmin; k <= kmax; k <<= 1) {
        for (uint32_t j = min(k >> 1, jtop); j > 0; j >>= 1) {
            for (uint32_t t = threadIdx.x; t < N / 2; t += blockDim.x) {
                uint32_t i = 2 * t - (t & (j - 1));
                uint32_t l = j == (k >> 1) ? (i ^ (k - 1)) : i + j;
                uint64_t ah = hi[i], al = lo[i], bh = hi[l], bl = lo[l];
                if (elem_less(bh, bl, ah, al)) {
                    hi[i] = bh;
                    lo[i] = bl;
                    hi[l] = ah;
                    lo[l] = al;
                }
            }
            __syncthreads();
        }
    }
}

// Exchange with lane ^ D without LDS addressing: DPP quad_perm (1, 2) and row_ror:8 (8) on the
// VALU, ds_swizzle bitmask mode (4, 16), v_permlane32_swap (32, CDNA4).
template <int D>
__device__ __forceinline__ uint32_t xshfl(uint32_t x) {
    static_assert(D == 1 || D == 2 || D == 4 || D == 8 || D == 16 || D == 32, "xor distance");
    if constexpr (D == 1) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);  // [1,0,3,2]
    } else if constexpr (D == 2) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);  // [2,3,0,1]
    } else if constexpr (D == 8) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x128, 0xF, 0xF, false);  // row_ror:8
    } else if constexpr (D == 4 || D == 16) {
        return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x1F | (D << 10));
    } else {
        const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return (threadIdx.x & 32u) ? (uint32_t)r[0] : (uint32_t)r[1];
    }
}
template <int D>
__device__ __forceinline__ uint64_t xshfl64(uint64_t v) {
    return ((uint64_t)xshfl<D>((uint32_t)(v >> 32)) << 32) | xshfl<D>((uint32_t)v);
}
// run-time (wave-uniform) distance
__device__ __forceinline__ uint64_t xshfl64_rt(uint64_t v, uint32_t d) {
    switch (d) {
        case 1: return xshfl64<1>(v);
        case 2: return xshfl64<2>(v);
        case 4: return xshfl64<4>(v);
        case 8: return xshfl64<8>(v);
        case 16: return xshfl64<16>(v);
        default: return xshfl64<32>(v);
    }
}

// distance known after unrolling (the switch folds away)
__device__ __forceinline__ uint32_t xs(uint32_t x, int d) {
    switch (d) {
        case 1: return xshfl<1>(x);
        case 2: return xshfl<2>(x);
        case 4: return xshfl<4>(x);
        case 8: return xshfl<8>(x);
        case 16: return xshfl<16>(x);
        default: return xshfl<32>(x);
    }
}
__device__ __forceinline__ uint64_t xs64(uint64_t v, int d) {
    return ((uint64_t)xs((uint32_t)(v >> 32), d) << 32) | xs((uint32_t)v, d);
}

// Inclusive wave scan on DPP: row_shr 1/2/4/8 within rows of 16, then row_bcast 15 / 31.
// LDS written by some lanes of a wave, read by others: a wave-scope fence pair around the barrier
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
    return x;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
    x += xshfl<1>(x);
    x += xshfl<2>(x);
    x += xshfl<4>(x);
    x += xshfl<8>(x);
    x += xshfl<16>(x);
    x += xshfl<32>(x);
    return x;
}
__device__ __forceinline__ uint32_t wave_min(uint32_t x) {
    x = min(x, xshfl<1>(x));
    x = min(x, xshfl<2>(x));
    x = min(x, xshfl<4>(x));
    x = min(x, xshfl<8>(x));
    x = min(x, xshfl<16>(x));
    x = min(x, xshfl<32>(x));
    return x;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
    x = max(x, xshfl<1>(x));
    x = max(x, xshfl<2>(x));
    x = max(x, xshfl<4>(x));
    x = max(x, xshfl<8>(x));
    x = max(x, xshfl<16>(x));
    x = max(x, xshfl<32>(x));
    return x;
}

// Workgroup exclusive scan of one u32 per thread (blockDim multiple of 64, <= 1024).
__device__ uint32_t wg_exclusive_scan(uint32_t v, uint32_t* s_wave, uint32_t& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const uint32_t x = wave_incl_scan(v);
    if (lane == 63) s_wave[wave] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int w = 0; w < nw; ++w) {
            uint32_t t = s_wave[w];
            s_wave[w] = acc;
            acc += t;
        }
        s_wave[nw] = acc;
    }
    __syncthreads();
    uint32_t r = s_wave[wave] + x - v;
    total = s_wave[nw];
    __syncthreads();
    return r;
}

// The same scan with one barrier: every thread sums the wave totals itself.  The caller must
// pass a barrier before s_wave is written again (the next scan on it).
__device__ __forceinline__ uint32_t wg_exclusive_scan1(uint32_t v, uint32_t* s_wave, uint32_t& total) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const uint32_t x = wave_incl_scan(v);
    if (lane == 63) s_wave[wave] = x;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
    for (uint32_t w = 0; w < nw; ++w) {
        const uint32_t t = s_wave[w];
        pre += w < wave ? t : 0u;
        tot += t;
    }
    total = tot;
    return pre + x - v;
}

// ------------------------------------------------------------------------------------------
// Group processing (process_kmer_set, signature_build.tcc:219-293).
//
// A group is the set of occurrences of one k-mer.  Groups arrive sorted by (func, ordinal), so
// function runs are contiguous in ascending FunctionIndex (the std::map order of func_count)
// and the best-function run is in ascending ordinal order.  Order-dependent statistics (P^2
// median, running variance) need the run in REVERSE ordinal order; when the run has >= 3
// members they are deferred to k_chains (one thread per chain), everything else is done here.
// ------------------------------------------------------------------------------------------
// Job.lens_off selector (top 2 bits): protein lengths live in the chain-lengths buffer, or in the
// (already consumed) record slots of the sub-bucket that produced the job, viewed as u32.
constexpr uint64_t LENS_SEL_SHIFT = 62;
constexpr uint64_t LENS_IN_RECS = 1, LENS_IN_TMP = 2, LENS_IN_BIG = 3;  // 0: chain-lengths buffer (overflow)
constexpr uint64_t LENS_OFF_MASK = (1ull << LENS_SEL_SHIFT) - 1;
constexpr int SMALLC = 8;    // thread-level groups up to this size, wave-level above

struct Job {                 // one deferred P^2 / variance chain
    uint64_t lens_off;       // protein lengths in visit order (reverse ordinal) at lens[lens_off..]
    uint32_t n;
    uint32_t out_idx;        // kept-k-mer output slot receiving median / var
};

struct GRes {
    uint32_t best_f, avg, cbest, rb;   // rb: first element of the best run (group-relative)
    uint16_t mean, median, var;
    bool kept;
};


// Sorted 16-byte elements in global memory (overflow path): hi = rem<<16|func
struct GlbView {
    const uint64_t* hi;
    const uint64_t* lo;
    __device__ __forceinline__ uint32_t func(uint64_t j) const { return (uint32_t)(hi[j] & 0xFFFFu); }
    __device__ __forceinline__ uint64_t lov(uint64_t j) const { return lo[j]; }
};

template <int N>
__device__ __forceinline__ void reg_sort(uint32_t* v) {
#pragma unroll
    for (int k = 2; k <= N; k <<= 1)
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1)
#pragma unroll
            for (int i = 0; i < N; ++i) {
                const int l = i ^ j;
                if (l > i) {
                    const bool asc = (i & k) == 0;
                    const uint32_t a = v[i], b = v[l];
                    v[i] = asc ? min(a, b) : max(a, b);
                    v[l] = asc ? max(a, b) : min(a, b);
                }
            }
}

__device__ __forceinline__ void stats_small(GRes& r, uint32_t x0, uint32_t x1, uint32_t n) {
    // n <= 2 samples in visit order: P^2 heights[2] is still 0; the variance recurrence of SigStats
    // after two samples is 0*(1)/2 + (x2 - mean2)^2 / 1 with mean2 over the u16 sum.
    r.median = 0;
    r.var = 0;
    if (n == 2) {
        const uint16_t sum = (uint16_t)(x0 + x1);
        const double mean = (double)sum / 2.0;
        const double tmp = (double)x1 - mean;
        const double v = 0.0 * 1.0 / 2.0 + tmp * tmp / 1.0;
        r.var = d2u16(v);
    }
}

// Thread-level group of c <= N members starting at a.
// A sequence's signature flag (process_kmer_set's seqs_with_a_signature.insert,
// signature_build.tcc:269).  Bit 0 of the pointer selects the form (option flag_bits): a byte per
// sequence, stored; or a bit per sequence, read first and set by a device-scope atomicOr only while
// it reads clear (most sequences are flagged by their first kept k-mer, later marks only read; a
// stale read costs one redundant atomic, never a lost flag).  k_flags_from_bits expands the bits.
__device__ __forceinline__ void mark_seq(uint8_t* f, uint32_t s) {
    const uintptr_t p = reinterpret_cast<uintptr_t>(f);
    if (p & 1u) {
        uint32_t* w = reinterpret_cast<uint32_t*>(p & ~(uintptr_t)1) + (s >> 5);
        const uint32_t m = 1u << (s & 31u);
        if (!(*w & m)) atomicOr(w, m);
    } else {
        f[s] = 1;
    }
}

// mark_seq for up to N sequences of one thread (0xFFFFFFFF: none): every flag read issued before
// the first atomic, so the reads overlap instead of waiting one after another behind the
// previous mark's atomic (a stale read costs one redundant atomic, never a lost flag)
template <int N>
__device__ __forceinline__ void mark_seqs(uint8_t* f, int flag_check, const uint32_t (&s)[N]) {
    const uintptr_t p = reinterpret_cast<uintptr_t>(f);
    if (p & 1u) {
        uint32_t* w = reinterpret_cast<uint32_t*>(p & ~(uintptr_t)1);
        uint32_t cur[N];
#pragma unroll
        for (int u = 0; u < N; ++u) cur[u] = s[u] != 0xFFFFFFFFu ? w[s[u] >> 5] : 0xFFFFFFFFu;
#pragma unroll
        for (int u = 0; u < N; ++u) {
            const uint32_t m = 1u << (s[u] & 31u);
            if (!(cur[u] & m)) atomicOr(w + (s[u] >> 5), m);
        }
    } else {
        uint8_t cur[N];
#pragma unroll
        for (int u = 0; u < N; ++u) cur[u] = s[u] != 0xFFFFFFFFu && flag_check ? f[s[u]] : (uint8_t)(s[u] == 0xFFFFFFFFu);
#pragma unroll
        for (int u = 0; u < N; ++u)
            if (cur[u] == 0) f[s[u]] = 1;
    }
}

template <int N, class V>
__device__ GRes group_thread(const V& v, uint64_t a, uint32_t c, const uint32_t* __restrict__ glen,
                             uint8_t* __restrict__ flags) {
    GRes r;
    r.kept = false;
    uint32_t fn[N], of[N];
#pragma unroll
    for (int t = 0; t < N; ++t) {
        if ((uint32_t)t < c) {
            fn[t] = v.func(a + t);
            of[t] = (uint32_t)(v.lov(a + t) & 0xFFFFu);
        } else {
            fn[t] = 0x10000u;
            of[t] = 0x10000u;  // sorts after every real offset
        }
    }
    uint32_t best_f = fn[0], best_c = 0, rb = 0, run_s = 0;
#pragma unroll
    for (int t = 1; t <= N; ++t) {
        if ((uint32_t)t <= c) {
            const bool end = ((uint32_t)t == c) || fn[t < N ? t : N - 1] != fn[t - 1];
            if (end) {
                const uint32_t len = t - run_s;
                if (len > best_c) {
                    best_c = len;
                    best_f = fn[t - 1];
                    rb = run_s;
                }
                run_s = t;
            }
        }
    }
    if ((float)best_c < float(c) * 0.8f) return r;
    r.kept = true;
    r.best_f = best_f;
    r.cbest = best_c;
    r.rb = rb;
    reg_sort<N>(of);
    const uint32_t k = c / 2;
    uint32_t avg = 0;
#pragma unroll
    for (int t = 0; t < N; ++t)
        if ((uint32_t)t == k) avg = of[t];
    r.avg = avg;
    uint32_t sum = 0;
    uint32_t lr0 = 0, lr1 = 0;
    for (uint32_t t = 0; t < c; ++t) {
        const uint64_t lo = v.lov(a + t);
        const uint32_t s = (uint32_t)(lo >> 36);
        if (flags) mark_seq(flags, s);
        if (t >= rb && t < rb + best_c) {
            const uint32_t len = glen[s];
            sum += len;
            const uint32_t q = rb + best_c - 1 - t;  // visit position (reverse ordinal)
            if (q == 0) lr0 = len;
            if (q == 1) lr1 = len;
        }
    }
    r.mean = d2u16((double)(uint16_t)sum / (double)best_c);
    r.median = 0;
    r.var = 0;
    if (best_c <= 2) stats_small(r, lr0, lr1, best_c);
    return r;
}

// Wave-level group (all 64 lanes, same a/c).  Only used for c > SMALLC, so the best run always
// has >= 3 members and its median/var are deferred.
template <class V>
__device__ GRes group_wave(const V& v, uint64_t a, uint32_t c, const uint32_t* __restrict__ glen,
                           uint8_t* __restrict__ flags) {
    const uint32_t lane = threadIdx.x & 63u;
    GRes r;
    r.kept = false;
    uint32_t best_f = 0, best_c = 0, rb = 0, run_s = 0;
    uint32_t run_f = v.func(a);
    for (uint32_t base = 0; base < c; base += 64) {
        const uint32_t t = base + lane;
        const bool valid = t < c;
        const uint32_t f = valid ? v.func(a + t) : 0xFFFFFFFFu;
        const uint32_t fp = (valid && t > 0) ? v.func(a + t - 1) : 0xFFFFFFFFu;
        uint64_t m = __ballot(valid && t > 0 && f != fp);
        while (m) {
            const int q = __ffsll((long long)m) - 1;
            m &= m - 1;
            const uint32_t pos = base + (uint32_t)q;
            const uint32_t len = pos - run_s;
            if (len > best_c) {
                best_c = len;
                best_f = run_f;
                rb = run_s;
            }
            run_s = pos;
            run_f = (uint32_t)__shfl((int)f, q, 64);
        }
    }
    {
        const uint32_t len = c - run_s;
        if (len > best_c) {
            best_c = len;
            best_f = run_f;
            rb = run_s;
        }
    }
    if ((float)best_c < float(c) * 0.8f) return r;
    r.kept = true;
    r.best_f = best_f;
    r.cbest = best_c;
    r.rb = rb;
    // avg_from_end: k-th smallest offset by binary search over the value range
    uint32_t vmin = 0xFFFFu, vmax = 0;
    for (uint32_t t = lane; t < c; t += 64) {
        const uint32_t o = (uint32_t)(v.lov(a + t) & 0xFFFFu);
        vmin = min(vmin, o);
        vmax = max(vmax, o);
    }
    vmin = wave_min(vmin);
    vmax = wave_max(vmax);
    const uint32_t k = c / 2;
    while (vmin < vmax) {
        const uint32_t mid = (vmin + vmax) >> 1;
        uint32_t cnt = 0;
        for (uint32_t t = lane; t < c; t += 64) cnt += (uint32_t)(v.lov(a + t) & 0xFFFFu) <= mid;
        cnt = wave_sum(cnt);
        if (cnt >= k + 1)
            vmax = mid;
        else
            vmin = mid + 1;
    }
    r.avg = vmin;
    uint32_t sum = 0;
    for (uint32_t t = lane; t < c; t += 64) {
        const uint32_t s = (uint32_t)(v.lov(a + t) >> 36);
        if (flags) mark_seq(flags, s);
        if (t >= rb && t < rb + best_c) sum += glen[s];
    }
    sum = wave_sum(sum);
    r.mean = d2u16((double)(uint16_t)sum / (double)best_c);
    r.median = 0;
    r.var = 0;
    return r;
}

__device__ __forceinline__ uint32_t wg_sum(uint32_t x, uint32_t* s_wave) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    x = wave_sum(x);
    if (lane == 0) s_wave[wave] = x;
    __syncthreads();
    uint32_t t = 0;
    for (uint32_t w = 0; w < nw; ++w) t += s_wave[w];
    __syncthreads();
    return t;
}

__device__ __forceinline__ uint32_t wg_max(uint32_t x, uint32_t* s_wave) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    x = wave_max(x);
    if (lane == 0) s_wave[wave] = x;
    __syncthreads();
    uint32_t t = 0;
    for (uint32_t w = 0; w < nw; ++w) t = max(t, s_wave[w]);
    __syncthreads();
    return t;
}

__device__ __forceinline__ uint32_t wg_min(uint32_t x, uint32_t* s_wave) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    x = wave_min(x);
    if (lane == 0) s_wave[wave] = x;
    __syncthreads();
    uint32_t t = 0xFFFFFFFFu;
    for (uint32_t w = 0; w < nw; ++w) t = min(t, s_wave[w]);
    __syncthreads();
    return t;
}

// group_wave's result for a large group computed by the whole workgroup (every thread calls it
// with the same a, c; the result is uniform).  Function runs from the run heads (compacted in
// order into heads[0..hcap)), the longest run with ties to the lowest FunctionIndex, the fp32
// cut, the upper-median offset by a 16-round radix select, flags, the u16 length sum.  Returns
// false (nothing written) when the group has more than hcap function runs.
template <class V>
__device__ bool group_block(const V& v, uint64_t a, uint32_t c, const uint32_t* __restrict__ glen,
                            uint8_t* __restrict__ flags, uint32_t* heads, uint32_t hcap, uint32_t* s_wave, GRes& r) {
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    r.kept = false;
    uint32_t H = 0;
    for (uint32_t t0 = 0; t0 < c; t0 += nt) {
        const uint32_t t = t0 + tid;
        const bool head = t < c && (t == 0 || v.func(a + t) != v.func(a + t - 1));
        uint32_t tot;
        const uint32_t pos = wg_exclusive_scan(head ? 1u : 0u, s_wave, tot);
        if (head && H + pos < hcap) heads[H + pos] = t;
        H += tot;
    }
    if (H > hcap) return false;
    __syncthreads();
    uint32_t lmax = 0;
    for (uint32_t j = tid; j < H; j += nt) lmax = max(lmax, (j + 1 < H ? heads[j + 1] : c) - heads[j]);
    const uint32_t best_c = wg_max(lmax, s_wave);
    uint32_t fmin = 0xFFFFFFFFu;  // (function << 16 | run index) of the best runs: lowest function wins
    for (uint32_t j = tid; j < H; j += nt)
        if ((j + 1 < H ? heads[j + 1] : c) - heads[j] == best_c) fmin = min(fmin, (v.func(a + heads[j]) << 16) | j);
    const uint32_t fj = wg_min(fmin, s_wave);
    if ((float)best_c < float(c) * 0.8f) return true;
    const uint32_t rb = heads[fj & 0xFFFFu];
    r.kept = true;
    r.best_f = fj >> 16;
    r.cbest = best_c;
    r.rb = rb;
    // upper median offset: the (c/2)-th smallest (0-based), radix select bit 15 down to 0
    uint32_t k = c / 2, pre = 0;
    for (int b = 15; b >= 0; --b) {
        uint32_t n0 = 0;
        for (uint32_t t = tid; t < c; t += nt) {
            const uint32_t o = (uint32_t)(v.lov(a + t) & 0xFFFFu);
            n0 += (o >> b) == (pre >> b);  // bits above b match the prefix and bit b is clear
        }
        n0 = wg_sum(n0, s_wave);
        if (k >= n0) {
            k -= n0;
            pre |= 1u << b;
        }
    }
    r.avg = pre;
    uint32_t sum = 0;
    for (uint32_t t = tid; t < c; t += nt) {
        const uint32_t s = (uint32_t)(v.lov(a + t) >> 36);
        if (flags) mark_seq(flags, s);
        if (t >= rb && t < rb + best_c) sum += glen[s];
    }
    sum = wg_sum(sum, s_wave);
    r.mean = d2u16((double)(uint16_t)sum / (double)best_c);
    r.median = 0;
    r.var = 0;
    return true;
}

// Chains run longest-first: jobs are counting-sorted by length class (floor(log2 n), descending)
// so a wave's 64 jobs have similar lengths.  Waves 2w and 2w+1 run the P^2 median and the
// variance recurrence of the same 64 jobs (wave-uniform branch).
// Run-level device slots (skm_build::d_run, cleared by begin_run): what the passes need to know
// about each other, kept on the device so a step issues every launch without a host round trip
enum : uint32_t {
    RUN_FLAGS = 0,          // RUN_F_* bits
    RUN_LONG_CUR = 1,       // stashed long-chain samples (run arena cursor)
    RUN_LONG_N = 2,         // stashed long jobs
    RUN_LONG_FLUSHED = 3,   // long jobs already handed to k_chain_long
    RUN_SNAP = 28,          // [28..61] k_long_snap ranges, one per stashed-chain batch (<= 17)
    RUN_DEM_TOT = 8,        // demands (max over passes): overflow scratch elements,
    RUN_DEM_SPLIT = 9,      //   split-path elements,
    RUN_DEM_LONG = 10,      //   stashed samples,
    RUN_DEM_LJOBS = 11,     //   stashed jobs
    RUN_LONG_WANT = 12,     // stashed samples / jobs asked for by every pass (the fitted ones and
    RUN_LONG_WANTJ = 13,    //   the ones that did not fit: the demand of a redo)
    RUN_ACC_NOVF = 16,      // run totals
    RUN_ACC_JOBS = 17,
    RUN_ACC_LENS = 18,
    RUN_ACC_OVF_ELEMS = 19,
    RUN_ACC_OVF_KEPT = 20,
    RUN_ACC_BIG = 21,
    RUN_ACC_BIG_KEPT = 22,
    RUN_ACC_GROUPED = 23,
    RUN_LAST_NOVF = 24,     // the last pass's overflow entries and chain jobs (diagnostics)
    RUN_LAST_JOBS = 25,
    RUN_NLOC = 26,          // world > 1: the pass's received element count (host-written)
    RUN_SLOTS = 64
};
constexpr unsigned long long RUN_F_ARENA = 1;  // the kept arena cannot take a pass: SKM_E_OOM
constexpr unsigned long long RUN_F_RERUN = 2;  // a work buffer was too small: grown to the demand, step redone
constexpr unsigned long long RUN_F_CAP = 4;    // a proven bound was exceeded: SKM_E_STATE
// k_ovf_plan's per-pass plan (skm_build::d_plan): list sizes and the work-queue counters of the
// persistent overflow kernels
enum : uint32_t {
    PLAN_NOVF = 0,      // overflow entries (0 when the pass is skipped)
    PLAN_NSPLIT = 1,    // the first NSPLIT entries (>= split_min elements) go through k_ovf_split
    PLAN_NHEAVY = 2,    // the first NHEAVY (>= ovf_heavy elements) run on stream 2, the rest on stream 3
    PLAN_SKIP = 3,      // nonzero: the run is abandoned (error or redo), the pass's group-by is skipped
    PLAN_Q_SPLIT = 4,   // queue counters
    PLAN_Q_HEAVY = 5,
    PLAN_Q_REST = 6,
    PLAN_SLOTS = 8
};

constexpr int JOB_CLASSES = 32;
constexpr int JOB_WG = 256;

__device__ __forceinline__ uint32_t job_class(uint32_t n) { return 31u - (uint32_t)__clz(n | 1u); }

// The job count is read on the device (capped at the list's capacity); each of the fixed
// gridDim.x workgroups takes one contiguous chunk of it.
__device__ __forceinline__ void job_chunk(const unsigned long long* nj_p, uint64_t cap, uint64_t& a, uint64_t& e) {
    const uint64_t nj = min((uint64_t)*nj_p, cap);
    const uint64_t chunk = (nj + gridDim.x - 1) / gridDim.x;
    a = min(nj, (uint64_t)blockIdx.x * chunk);
    e = min(nj, a + chunk);
}

__global__ __launch_bounds__(JOB_WG) void k_job_count(const Job* __restrict__ jobs, const unsigned long long* nj_p,
                                                      uint64_t cap, uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[JOB_CLASSES];
    if (threadIdx.x < JOB_CLASSES) h[threadIdx.x] = 0;
    __syncthreads();
    uint64_t a, e;
    job_chunk(nj_p, cap, a, e);
    for (uint64_t j = a + threadIdx.x; j < e; j += blockDim.x) atomicAdd(&h[job_class(jobs[j].n)], 1u);
    __syncthreads();
    if (threadIdx.x < JOB_CLASSES) hist[blockIdx.x * JOB_CLASSES + threadIdx.x] = h[threadIdx.x];
}

// one workgroup: offs[w][c] = start of (class c, workgroup w), classes in descending order
constexpr uint32_t LONG_CLASS = 14;  // chains of >= 16384 samples get a wave pair each (k_chain_long)

__global__ void k_job_scan(const uint32_t* __restrict__ hist, uint32_t nwg, uint64_t* __restrict__ offs,
                           uint32_t long_class) {
    __shared__ uint64_t tot[JOB_CLASSES];
    const uint32_t c = threadIdx.x;
    if (c < JOB_CLASSES) {
        uint64_t t = 0;
        for (uint32_t w = 0; w < nwg; ++w) t += hist[w * JOB_CLASSES + c];
        tot[c] = t;
    }
    __syncthreads();
    if (c == 0) {  // jobs of the long classes lead the sorted order
        uint64_t nl = 0;
        for (uint32_t cc = long_class; cc < JOB_CLASSES; ++cc) nl += tot[cc];
        offs[(uint64_t)nwg * JOB_CLASSES] = nl;
    }
    if (c < JOB_CLASSES) {
        uint64_t base = 0;
        for (uint32_t cc = JOB_CLASSES - 1; cc > c; --cc) base += tot[cc];
        for (uint32_t w = 0; w < nwg; ++w) {
            offs[w * JOB_CLASSES + c] = base;
            base += hist[w * JOB_CLASSES + c];
        }
    }
}

__global__ __launch_bounds__(JOB_WG) void k_job_scatter(const Job* __restrict__ jobs, const unsigned long long* nj_p,
                                                        uint64_t cap, const uint64_t* __restrict__ offs,
                                                        Job* __restrict__ sorted) {
    __shared__ unsigned long long cur[JOB_CLASSES];
    if (threadIdx.x < JOB_CLASSES) cur[threadIdx.x] = offs[blockIdx.x * JOB_CLASSES + threadIdx.x];
    __syncthreads();
    uint64_t a, e;
    job_chunk(nj_p, cap, a, e);
    for (uint64_t j = a + threadIdx.x; j < e; j += blockDim.x) {
        const Job jb = jobs[j];
        sorted[atomicAdd(&cur[job_class(jb.n)], 1ull)] = jb;
    }
}

// Long chains leave the pass: their samples (wherever the group-by left them: consumed element
// slots, the overflow's lengths buffer) are stashed into a run-persistent arena so the chains can
// run on their own streams while the next passes reuse every work buffer.  k_long_plan: one
// workgroup, exclusive offsets of the first nlong (class-sorted) jobs' sample counts; with `run`
// (key-range passes) it also reserves the samples' range of the run's arena and the jobs' slots of
// the run's long-job list:  off[nlong] = samples, [nlong+1] = nlong, [nlong+2] = arena base,
// [nlong+3] = job base, [nlong+4] = 1 if both fit (else the demand is recorded and the run redone).
__global__ __launch_bounds__(1024) void k_long_plan(const Job* __restrict__ jobs, const uint64_t* __restrict__ nlong_p,
                                                    uint64_t* __restrict__ off, unsigned long long* __restrict__ run,
                                                    uint64_t arena_cap, uint64_t jobs_cap) {
    __shared__ uint32_t s_wave[17];
    __shared__ unsigned long long s_run;
    const uint64_t nlong = *nlong_p;
    if (threadIdx.x == 0) s_run = 0;
    __syncthreads();
    for (uint64_t b = 0; b < nlong; b += blockDim.x) {
        const uint64_t j = b + threadIdx.x;
        const uint32_t n = j < nlong ? jobs[j].n : 0u;
        uint32_t tot;
        const uint32_t ex = wg_exclusive_scan(n, s_wave, tot);
        const unsigned long long run_ = s_run;
        if (j < nlong) off[j] = run_ + ex;
        __syncthreads();
        if (threadIdx.x == 0) s_run = run_ + tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const uint64_t total = s_run;
        off[nlong] = total;
        off[nlong + 1] = nlong;
        if (run) {
            uint64_t base = 0, jbase = 0;
            bool ok = true;
            if (nlong) {
                // the run's cursors advance only by reservations that fit (compare-and-swap), so
                // the long-job list [flushed, RUN_LONG_N) never names a slot k_long_stash skipped;
                // what every pass asked for accumulates separately as the redo's demand
                const unsigned long long want = atomicAdd(&run[RUN_LONG_WANT], (unsigned long long)total) + total;
                const unsigned long long wantj = atomicAdd(&run[RUN_LONG_WANTJ], (unsigned long long)nlong) + nlong;
                auto reserve = [&](unsigned long long* c, uint64_t n, uint64_t cap, uint64_t& at) {
                    unsigned long long cur = *(volatile unsigned long long*)c;
                    while (true) {
                        if (cur + n > cap) return false;
                        const unsigned long long seen = atomicCAS(c, cur, cur + n);
                        if (seen == cur) {
                            at = cur;
                            return true;
                        }
                        cur = seen;
                    }
                };
                ok = reserve(&run[RUN_LONG_CUR], total, arena_cap, base);
                // a job-slot failure after the samples fit leaves those samples unused (the run is redone)
                ok = ok && reserve(&run[RUN_LONG_N], nlong, jobs_cap, jbase);
                if (!ok) {
                    atomicMax(&run[RUN_DEM_LONG], want);
                    atomicMax(&run[RUN_DEM_LJOBS], wantj);
                    atomicOr(&run[RUN_FLAGS], (unsigned long long)RUN_F_RERUN);
                }
            }
            off[nlong + 2] = base;
            off[nlong + 3] = jbase;
            off[nlong + 4] = ok ? 1u : 0u;
        }
    }
}

// persistent grid over the long jobs (count on the device): copy each one's samples into the
// run's arena, append the rewritten job to the run's long-job list
__global__ __launch_bounds__(256) void k_long_stash(const Job* __restrict__ jobs, const uint64_t* __restrict__ nlong_p,
                                                    const uint64_t* __restrict__ off,
                                                    const uint32_t* __restrict__ lens, const uint32_t* __restrict__ recs32,
                                                    const uint32_t* __restrict__ tmp32, const uint32_t* __restrict__ big32,
                                                    uint32_t* __restrict__ arena, Job* __restrict__ out_jobs) {
    const uint64_t nlong = *nlong_p;
    if (nlong == 0 || off[nlong + 4] == 0) return;
    const uint64_t base = off[nlong + 2], jbase = off[nlong + 3];
    for (uint64_t q = blockIdx.x; q < nlong; q += gridDim.x) {
        const Job jb = jobs[q];
        const uint64_t sel = jb.lens_off >> LENS_SEL_SHIFT;
        const uint32_t* x = (sel == LENS_IN_RECS ? recs32 : sel == LENS_IN_TMP ? tmp32 : sel == LENS_IN_BIG ? big32 : lens) +
                            (jb.lens_off & LENS_OFF_MASK);
        const uint64_t o = base + off[q];
        for (uint32_t i = threadIdx.x; i < jb.n; i += blockDim.x) arena[o + i] = x[i];
        if (threadIdx.x == 0) out_jobs[jbase + q] = Job{reinterpret_cast<uint64_t>(arena + o), jb.n, jb.out_idx};
    }
}

// k_chain_long's job range of a stashed batch: [run's flushed mark, run's job count), then the mark
// moves (one thread, on the group-by stream after the passes' stashes)
__global__ void k_long_snap(unsigned long long* __restrict__ run, unsigned long long* __restrict__ range,
                            uint64_t jobs_cap) {
    // RUN_LONG_N only counts stashed jobs (k_long_plan reserves by compare-and-swap); the clamp to
    // the list's capacity is a second line of defence for k_chain_long, which has no bound check
    const unsigned long long hi = min(run[RUN_LONG_N], (unsigned long long)jobs_cap);
    range[0] = min(run[RUN_LONG_FLUSHED], hi);
    range[1] = hi;
    run[RUN_LONG_FLUSHED] = hi;
}

// One chain over x[0..n): blocks of 16 samples; the next block's loads (index clamped, so no
// per-element branch) are in flight while the current block is consumed.
template <bool VAR>
__device__ __forceinline__ void chain_run(SigStats& st, const uint32_t* __restrict__ x, uint32_t n) {
    constexpr uint32_t B = 16;
    const uint32_t last = n - 1;
    uint32_t cur[B], nxt[B];
#pragma unroll
    for (uint32_t i = 0; i < B; ++i) cur[i] = x[min(i, last)];
    for (uint32_t base = 0; base < n; base += B) {
#pragma unroll
        for (uint32_t i = 0; i < B; ++i) nxt[i] = x[min(base + B + i, last)];
        const uint32_t m = min(B, n - base);
        for (uint32_t i = 0; i < m; ++i) {
            // rotate the block through cur[0] without dynamic register indexing
            const uint32_t v = cur[0];
#pragma unroll
            for (uint32_t q = 0; q + 1 < B; ++q) cur[q] = cur[q + 1];
            if (VAR)
                st.add_var(v);
            else
                st.add_p2(v);
        }
#pragma unroll
        for (uint32_t i = 0; i < B; ++i) cur[i] = nxt[i];
    }
}

// ------------------------------------------------------------------------------------------
// Long chains: one wave pair per job (wave 0: P^2 median, wave 1: variance), 64 samples per
// round held one per lane.
//   P^2: the cells of all 64 samples come from three ballots of (height <= x) against the
//   current heights; the extremes h0/h4 are lane prefix min/max (they never feed the cell).
//   The walk over the round is scalar integer work (positions, quarter-unit decisions); only a
//   marker adjustment runs fp64, after which the three ballots are re-taken.
//   Variance: the sample-independent terms (u16 prefix sum, mean, (x-mean)^2/(n-1), 1/n) are
//   computed per lane; the walk is the 5-op recurrence var = var*(n-1)/n + t.
// Both give the bit-identical result of the one-lane recurrences in SigStats.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t incl_scan_min(uint32_t v) {
    const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = (uint32_t)__shfl_up((int)v, d, 64);
        if (lane >= (uint32_t)d) v = min(v, o);
    }
    return v;
}
__device__ __forceinline__ uint32_t incl_scan_max(uint32_t v) {
    const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = (uint32_t)__shfl_up((int)v, d, 64);
        if (lane >= (uint32_t)d) v = max(v, o);
    }
    return v;
}
__device__ __forceinline__ uint32_t incl_scan_add(uint32_t v) {
    const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = (uint32_t)__shfl_up((int)v, d, 64);
        if (lane >= (uint32_t)d) v += o;
    }
    return v;
}
__device__ __forceinline__ double readlane_f64(double v, uint32_t l) {
    const uint64_t b = __double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, (int)l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), (int)l);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// The adjusting markers of one step (mask M, bit i-1 = marker i): their nine reciprocals first
// (independent of the heights), then the dependent height chain marker 1 -> 2 -> 3, all in one
// basic block so the in-order issue overlaps the reciprocal latencies.
template <int M>
__device__ __forceinline__ void p2_adjust(double& h1, double& h2, double& h3, double h0, double h4,
                                          const int32_t (&dp)[3], const int32_t (&dm)[3], const int32_t (&sg)[3]) {
    double yp[3], ym[3], yd[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if ((M >> i) & 1) {
            yp[i] = rcp_int((double)dp[i]);
            ym[i] = rcp_int((double)dm[i]);
            yd[i] = rcp_int((double)(dp[i] - dm[i]));
        }
    }
    if constexpr ((M & 1) != 0) h1 = p2_height_y(h0, h1, h2, dp[0], dm[0], sg[0], yp[0], ym[0], yd[0]);
    if constexpr ((M & 2) != 0) h2 = p2_height_y(h1, h2, h3, dp[1], dm[1], sg[1], yp[1], ym[1], yd[1]);
    if constexpr ((M & 4) != 0) h3 = p2_height_y(h2, h3, h4, dp[2], dm[2], sg[2], yp[2], ym[2], yd[2]);
}

__device__ __forceinline__ double chain_long_p2(const uint32_t* __restrict__ x, uint32_t n_) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t n = (uint32_t)__builtin_amdgcn_readfirstlane((int)n_);  // wave-uniform: scalar walk
    SigStats st;
    st.init();
    const uint32_t n0 = min(n, 5u);
    for (uint32_t i = 0; i < n0; ++i) st.add_p2(x[i]);  // uniform: every lane runs the same start
    if (n <= 5) return st.h[2];
    double h1 = st.h[1], h2 = st.h[2], h3 = st.h[3];
    uint32_t h0i = (uint32_t)st.h[0], h4i = (uint32_t)st.h[4];  // extremes are always samples
    int32_t a1 = st.act[1], a2 = st.act[2], a3 = st.act[3], a4 = st.act[4];
    int32_t k4 = 0;  // cnt - 5 after the increment below
    uint32_t xn = 5 + lane < n ? x[5 + lane] : 0u;
    for (uint32_t base = 5; base < n; base += 64) {
        const uint32_t m = min(64u, n - base);
        const uint32_t xl = xn;
        const bool live = lane < m;
        xn = base + 64 + lane < n ? x[base + 64 + lane] : 0u;  // next round in flight
        const uint32_t imin = min(h0i, incl_scan_min(live ? xl : 0xFFFFFFFFu));
        const uint32_t imax = max(h4i, incl_scan_max(live ? xl : 0u));
        const double xd = (double)xl;
        uint64_t B1 = __ballot(live && h1 <= xd), B2 = __ballot(live && h2 <= xd), B3 = __ballot(live && h3 <= xd);
        for (uint32_t l = 0; l < m; ++l) {
            // integer walk (scalar): cell, positions, the three adjust decisions in marker order
            a1 += ((B1 >> l) & 1u) ? 0 : 1;
            a2 += ((B2 >> l) & 1u) ? 0 : 1;
            a3 += ((B3 >> l) & 1u) ? 0 : 1;
            a4 += 1;
            ++k4;
            int32_t dp[3], dm[3], sg[3];
            uint32_t mask = 0;
            {
                const int32_t d4 = 8 + k4 - 4 * a1;
                dp[0] = a2 - a1;
                dm[0] = 1 - a1;
                sg[0] = d4 > 0 ? 1 : -1;
                if ((d4 >= 4 && dp[0] > 1) || (d4 <= -4 && dm[0] < -1)) {
                    mask |= 1u;
                    a1 += sg[0];
                }
            }
            {
                const int32_t d4 = 12 + 2 * k4 - 4 * a2;
                dp[1] = a3 - a2;
                dm[1] = a1 - a2;
                sg[1] = d4 > 0 ? 1 : -1;
                if ((d4 >= 4 && dp[1] > 1) || (d4 <= -4 && dm[1] < -1)) {
                    mask |= 2u;
                    a2 += sg[1];
                }
            }
            {
                const int32_t d4 = 16 + 3 * k4 - 4 * a3;
                dp[2] = a4 - a3;
                dm[2] = a2 - a3;
                sg[2] = d4 > 0 ? 1 : -1;
                if ((d4 >= 4 && dp[2] > 1) || (d4 <= -4 && dm[2] < -1)) {
                    mask |= 4u;
                    a3 += sg[2];
                }
            }
            if (mask) {
                const double h0 = (double)(uint32_t)__builtin_amdgcn_readlane((int)imin, (int)l);
                const double h4 = (double)(uint32_t)__builtin_amdgcn_readlane((int)imax, (int)l);
                switch (mask) {
                    case 1: p2_adjust<1>(h1, h2, h3, h0, h4, dp, dm, sg); break;
                    case 2: p2_adjust<2>(h1, h2, h3, h0, h4, dp, dm, sg); break;
                    case 3: p2_adjust<3>(h1, h2, h3, h0, h4, dp, dm, sg); break;
                    case 4: p2_adjust<4>(h1, h2, h3, h0, h4, dp, dm, sg); break;
                    case 5: p2_adjust<5>(h1, h2, h3, h0, h4, dp, dm, sg); break;
                    case 6: p2_adjust<6>(h1, h2, h3, h0, h4, dp, dm, sg); break;
                    default: p2_adjust<7>(h1, h2, h3, h0, h4, dp, dm, sg); break;
                }
                B1 = __ballot(live && h1 <= xd);
                B2 = __ballot(live && h2 <= xd);
                B3 = __ballot(live && h3 <= xd);
            }
        }
        h0i = (uint32_t)__builtin_amdgcn_readlane((int)imin, (int)(m - 1));
        h4i = (uint32_t)__builtin_amdgcn_readlane((int)imax, (int)(m - 1));
    }
    return h2;
}

// The same walk with the adjust decisions branch-free (s_cselect instead of short-circuit
// branches) and the reciprocals of one step computed lane-parallel: lane 3(i-1) + {0, 1, 2} holds
// marker i's divisors dp, dm, dp - dm, one vector rcp + Newton sequence gives all nine RN(1/m),
// and each adjusting marker reads its three back with v_readlane (the same values as rcp_int).
// v_writelane_b32 (no clang builtin for it): lane L of v takes the wave-uniform x
template <int L>
__device__ __forceinline__ int32_t writelane_i32_(int32_t v, int32_t x) {
    asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(x), "i"(L));
    return v;
}
#define writelane_i32(v, x, L) writelane_i32_<L>((v), (x))

// p2_height_y split at the dependence on the lower neighbour: the upper quotient (hp_ - H) / dp
// uses only heights no earlier marker of this step changes, so every adjusting marker's upper
// half is issued first and only the lower half stays on the marker 1 -> 2 -> 3 chain.
struct P2Up {
    double hp, a, ym;
};
template <int L>
__device__ __forceinline__ P2Up p2_upper(double H, double hp_, int32_t dpi, int32_t dmi, int32_t sgi, double y) {
    P2Up u;
    u.hp = div_by(hp_ - H, (double)dpi, readlane_f64(y, L));
    u.a = (double)(sgi - dmi) * u.hp;
    u.ym = readlane_f64(y, L + 2);
    return u;
}
template <int L>
__device__ __forceinline__ double p2_lower(double hm_, double H, double hp_, int32_t dpi, int32_t dmi, int32_t sgi,
                                           const P2Up& u, double y) {
    const double hm = div_by(hm_ - H, (double)dmi, readlane_f64(y, L + 1));
    // H -+ RN(ym * S) == H + RN(+-ym * S): RN is odd, and x - y is x + (-y)
    const double ysg = sgi > 0 ? u.ym : -u.ym;
    const double hh = H + ysg * (u.a + (double)(dpi - sgi) * hm);
    const double lin = sgi > 0 ? H + u.hp : H - hm;
    return (hm_ < hh && hh < hp_) ? hh : lin;
}
template <int M>
__device__ __forceinline__ void p2_adjust_lanes(double& h1, double& h2, double& h3, uint32_t imin, uint32_t imax,
                                                uint32_t l, const int32_t (&dp)[3], const int32_t (&dm)[3],
                                                const int32_t (&sg)[3], double y) {
    // the extremes after sample l (lane-prefix min / max), read only by the markers next to them
    double h0 = 0.0, h4 = 0.0;
    if constexpr ((M & 1) != 0) h0 = (double)(uint32_t)__builtin_amdgcn_readlane((int)imin, (int)l);
    if constexpr ((M & 4) != 0) h4 = (double)(uint32_t)__builtin_amdgcn_readlane((int)imax, (int)l);
    const double o2 = h2, o3 = h3;  // upper neighbours as the step found them
    P2Up u1, u2, u3;
    if constexpr ((M & 1) != 0) u1 = p2_upper<0>(h1, o2, dp[0], dm[0], sg[0], y);
    if constexpr ((M & 2) != 0) u2 = p2_upper<3>(o2, o3, dp[1], dm[1], sg[1], y);
    if constexpr ((M & 4) != 0) u3 = p2_upper<6>(o3, h4, dp[2], dm[2], sg[2], y);
    if constexpr ((M & 1) != 0) h1 = p2_lower<0>(h0, h1, o2, dp[0], dm[0], sg[0], u1, y);
    if constexpr ((M & 2) != 0) h2 = p2_lower<3>(h1, o2, o3, dp[1], dm[1], sg[1], u2, y);
    if constexpr ((M & 4) != 0) h3 = p2_lower<6>(h2, o3, h4, dp[2], dm[2], sg[2], u3, y);
}

__device__ __forceinline__ double chain_long_p2v(const uint32_t* __restrict__ x, uint32_t n_) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t n = (uint32_t)__builtin_amdgcn_readfirstlane((int)n_);
    SigStats st;
    st.init();
    const uint32_t n0 = min(n, 5u);
    for (uint32_t i = 0; i < n0; ++i) st.add_p2(x[i]);
    if (n <= 5) return st.h[2];
    double h1 = st.h[1], h2 = st.h[2], h3 = st.h[3];
    uint32_t h0i = (uint32_t)st.h[0], h4i = (uint32_t)st.h[4];
    int32_t a1 = st.act[1], a2 = st.act[2], a3 = st.act[3], a4 = st.act[4];
    int32_t K1 = 8, K2 = 12, K3 = 16;  // 4 * desired positions: 4(i+1) + i*(cnt-5)
    uint32_t xn = 5 + lane < n ? x[5 + lane] : 0u;
    for (uint32_t base = 5; base < n; base += 64) {
        const uint32_t m = min(64u, n - base);
        const uint32_t xl = xn;
        const bool live = lane < m;
        xn = base + 64 + lane < n ? x[base + 64 + lane] : 0u;
        const uint32_t imin = min(h0i, incl_scan_min(live ? xl : 0xFFFFFFFFu));
        const uint32_t imax = max(h4i, incl_scan_max(live ? xl : 0u));
        const double xd = (double)xl;
        // bits of lanes >= m are never read: no live mask on the ballots
        uint64_t B1 = __ballot(h1 <= xd), B2 = __ballot(h2 <= xd), B3 = __ballot(h3 <= xd);
        for (uint32_t l = 0; l < m; ++l) {
            // positions: +1 below the sample's cell (B bit clear), a4 always
            a1 += 1 - (int32_t)((B1 >> l) & 1u);
            a2 += 1 - (int32_t)((B2 >> l) & 1u);
            a3 += 1 - (int32_t)((B3 >> l) & 1u);
            a4 += 1;
            K1 += 1;  // 4 * desired position of marker i = K_i
            K2 += 2;
            K3 += 3;
            // adjust decisions as sign bits, no compares: up = (d4 >= 4 && dp > 1) is the sign of
            // (3 - d4) & (1 - dp); down = (d4 <= -4 && dm < -1) the sign of (d4 + 3) & (dm + 1);
            // the two exclude each other and the step is up - down (sg = +1 up, -1 down)
            int32_t dp[3], dm[3], sg[3];
            uint32_t mask;
            {
                const int32_t d4 = K1 - 4 * a1;
                dp[0] = a2 - a1;
                dm[0] = 1 - a1;
                const uint32_t up = ((uint32_t)(3 - d4) & (uint32_t)(1 - dp[0])) >> 31;
                const uint32_t dn = ((uint32_t)(d4 + 3) & (uint32_t)(dm[0] + 1)) >> 31;
                a1 += (int32_t)up - (int32_t)dn;
                sg[0] = 1 - 2 * (int32_t)dn;
                mask = up | dn;
            }
            {
                const int32_t d4 = K2 - 4 * a2;
                dp[1] = a3 - a2;
                dm[1] = a1 - a2;
                const uint32_t up = ((uint32_t)(3 - d4) & (uint32_t)(1 - dp[1])) >> 31;
                const uint32_t dn = ((uint32_t)(d4 + 3) & (uint32_t)(dm[1] + 1)) >> 31;
                a2 += (int32_t)up - (int32_t)dn;
                sg[1] = 1 - 2 * (int32_t)dn;
                mask |= (up | dn) << 1;
            }
            {
                const int32_t d4 = K3 - 4 * a3;
                dp[2] = a4 - a3;
                dm[2] = a2 - a3;
                const uint32_t up = ((uint32_t)(3 - d4) & (uint32_t)(1 - dp[2])) >> 31;
                const uint32_t dn = ((uint32_t)(d4 + 3) & (uint32_t)(dm[2] + 1)) >> 31;
                a3 += (int32_t)up - (int32_t)dn;
                sg[2] = 1 - 2 * (int32_t)dn;
                mask |= (up | dn) << 2;
            }
            if (mask) {
                // lanes 0..8: marker i's dp, dm, dp - dm (the other lanes hold dm[0] = 1 - a1 < 0)
                int32_t dv = dm[0];
                dv = writelane_i32(dv, dp[0], 0);
                dv = writelane_i32(dv, dp[0] - dm[0], 2);
                dv = writelane_i32(dv, dp[1], 3);
                dv = writelane_i32(dv, dm[1], 4);
                dv = writelane_i32(dv, dp[1] - dm[1], 5);
                dv = writelane_i32(dv, dp[2], 6);
                dv = writelane_i32(dv, dm[2], 7);
                dv = writelane_i32(dv, dp[2] - dm[2], 8);
                const double y = rcp_int((double)dv);
                switch (mask) {
                    case 1: p2_adjust_lanes<1>(h1, h2, h3, imin, imax, l, dp, dm, sg, y); break;
                    case 2: p2_adjust_lanes<2>(h1, h2, h3, imin, imax, l, dp, dm, sg, y); break;
                    case 3: p2_adjust_lanes<3>(h1, h2, h3, imin, imax, l, dp, dm, sg, y); break;
                    case 4: p2_adjust_lanes<4>(h1, h2, h3, imin, imax, l, dp, dm, sg, y); break;
                    case 5: p2_adjust_lanes<5>(h1, h2, h3, imin, imax, l, dp, dm, sg, y); break;
                    case 6: p2_adjust_lanes<6>(h1, h2, h3, imin, imax, l, dp, dm, sg, y); break;
                    default: p2_adjust_lanes<7>(h1, h2, h3, imin, imax, l, dp, dm, sg, y); break;
                }
                B1 = __ballot(h1 <= xd);
                B2 = __ballot(h2 <= xd);
                B3 = __ballot(h3 <= xd);
            }
        }
        h0i = (uint32_t)__builtin_amdgcn_readlane((int)imin, (int)(m - 1));
        h4i = (uint32_t)__builtin_amdgcn_readlane((int)imax, (int)(m - 1));
    }
    return h2;
}

__device__ __forceinline__ double chain_long_var(const uint32_t* __restrict__ x, uint32_t n_) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t n = (uint32_t)__builtin_amdgcn_readfirstlane((int)n_);
    double var = 0.0;
    uint32_t sum = 0;  // running u32 sum; only its low 16 bits are the accumulator's sum
    uint32_t xn = lane < n ? x[lane] : 0u;
    for (uint32_t base = 0; base < n; base += 64) {
        const uint32_t m = min(64u, n - base);
        const uint32_t xl = xn;
        const bool live = lane < m;
        xn = base + 64 + lane < n ? x[base + 64 + lane] : 0u;
        const uint32_t ps = sum + incl_scan_add(live ? xl : 0u);
        const uint32_t c = base + lane + 1;  // count after this sample
        double cd = (double)c, c1d = (double)(c - 1), yc = 0.0, t2 = 0.0;
        if (live && c > 1) {
            yc = rcp_int(cd);
            const double mean = div_by((double)(ps & 0xFFFFu), cd, yc);
            const double tmp = (double)xl - mean;
            t2 = div_by(tmp * tmp, c1d, rcp_int(c1d));
        }
        for (uint32_t l = (base == 0 ? 1u : 0u); l < m; ++l)
            var = div_by(var * readlane_f64(c1d, l), readlane_f64(cd, l), readlane_f64(yc, l)) + readlane_f64(t2, l);
        sum = (uint32_t)__builtin_amdgcn_readlane((int)ps, (int)(m - 1));
    }
    return var;
}

// jobs [*lo_p (0 when null), *hi_p): a wave pair each, persistent grid
__global__ __launch_bounds__(128) void k_chain_long(const Job* __restrict__ jobs, const unsigned long long* lo_p,
                                                    const unsigned long long* hi_p,
                                                    const uint32_t* __restrict__ lens,
                                                    const uint32_t* __restrict__ recs32,
                                                    const uint32_t* __restrict__ tmp32,
                                                    const uint32_t* __restrict__ big32,
                                                    skm_stored_kmer_data* __restrict__ out, int prio,
                                                    uint32_t min_n = 0) {
    const uint64_t lo = lo_p ? (uint64_t)*lo_p : 0ull, hi = *hi_p;
    if (lo + blockIdx.x >= hi) return;
    if (prio == 1) __builtin_amdgcn_s_setprio(1);
    if (prio == 2) __builtin_amdgcn_s_setprio(2);
    if (prio >= 3) __builtin_amdgcn_s_setprio(3);
    for (uint64_t q = lo + blockIdx.x; q < hi; q += gridDim.x) {
        const Job jb = jobs[q];
        if (jb.n < min_n) continue;  // k_chains' (one lane each)
        const uint64_t sel = jb.lens_off >> LENS_SEL_SHIFT;
        // lens == nullptr: stashed jobs, lens_off is the samples' device address
        const uint32_t* x =
            !lens && sel == 0 ? reinterpret_cast<const uint32_t*>(jb.lens_off)
                              : (sel == LENS_IN_RECS ? recs32 : sel == LENS_IN_TMP ? tmp32 : sel == LENS_IN_BIG ? big32 : lens) +
                                    (jb.lens_off & LENS_OFF_MASK);
        if (threadIdx.x < 64) {
            const double med = chain_long_p2v(x, jb.n);
            if (threadIdx.x == 0) out[jb.out_idx].median = d2u16(med);
        } else {
            const double v = chain_long_var(x, jb.n);
            if (threadIdx.x == 64) out[jb.out_idx].var = d2u16(v);
        }
    }
}

// Giant chains of one pass, longest first: k_heavy appends a key's job when the key is done, so the
// heaviest keys (the longest reads) come late in the list, and k_chain_dyn's workgroups would
// start them after a first round of shorter chains.  One workgroup sorts the first GORD_MAX jobs
// in place by samples, descending (ties by list order): a bitonic network over (~n, index) keys
// in LDS, then every job moves to its rank.  The order of the chains does not change any result.
constexpr uint32_t GORD_MAX = 4096;
__global__ __launch_bounds__(1024) void k_giant_order(Job* __restrict__ jobs, const unsigned long long* __restrict__ njobs) {
    __shared__ uint64_t s_key[GORD_MAX];
    __shared__ uint32_t s_pos[GORD_MAX];
    constexpr uint32_t PER = GORD_MAX / 1024;
    const uint32_t tid = threadIdx.x;
    const uint32_t nj = (uint32_t)min((unsigned long long)GORD_MAX, *njobs);
    if (nj < 2) return;  // uniform
    Job mine[PER];
#pragma unroll
    for (uint32_t r = 0; r < PER; ++r) {
        const uint32_t i = tid + r * 1024u;
        if (i < nj) mine[r] = jobs[i];
        s_key[i] = i < nj ? ((uint64_t)(0xFFFFFFFFu - mine[r].n) << 32) | i : ~0ull;
    }
    __syncthreads();
    for (uint32_t k = 2; k <= GORD_MAX; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
            for (uint32_t r = 0; r < PER; ++r) {
                const uint32_t i = tid + r * 1024u, l = i ^ j;
                if (l > i) {
                    const uint64_t a = s_key[i], c = s_key[l];
                    if (((i & k) == 0) == (a > c)) {
                        s_key[i] = c;
                        s_key[l] = a;
                    }
                }
            }
            __syncthreads();
        }
#pragma unroll
    for (uint32_t r = 0; r < PER; ++r) {
        const uint32_t p = tid + r * 1024u;
        if (p < nj) s_pos[(uint32_t)s_key[p]] = p;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t r = 0; r < PER; ++r) {
        const uint32_t i = tid + r * 1024u;
        if (i < nj) jobs[s_pos[i]] = mine[r];
    }
}

// Giant chains of one pass (k_heavy's slot list): the job count is read on the device, so the
// launch needs no host round trip; one wave pair per job, idle workgroups exit at once.
__global__ __launch_bounds__(128) void k_chain_dyn(const Job* __restrict__ jobs, const unsigned long long* __restrict__ njobs,
                                                   skm_stored_kmer_data* __restrict__ out, int prio) {
    const uint64_t nj = *njobs;
    if (prio == 1) __builtin_amdgcn_s_setprio(1);
    if (prio == 2) __builtin_amdgcn_s_setprio(2);
    if (prio >= 3) __builtin_amdgcn_s_setprio(3);
    for (uint64_t q = blockIdx.x; q < nj; q += gridDim.x) {
        const Job jb = jobs[q];
        const uint32_t* x = reinterpret_cast<const uint32_t*>(jb.lens_off);
        if (threadIdx.x < 64) {
            const double med = chain_long_p2v(x, jb.n);
            if (threadIdx.x == 0) out[jb.out_idx].median = d2u16(med);
        } else {
            const double v = chain_long_var(x, jb.n);
            if (threadIdx.x == 64) out[jb.out_idx].var = d2u16(v);
        }
    }
}

// jobs [*lo_p, min(*hi_p, cap)) (the per-lane chains after the long ones of the class-sorted list)
__device__ __forceinline__ void chains_body(const Job* __restrict__ jobs, const unsigned long long* lo_p,
                                            const unsigned long long* hi_p, uint64_t cap,
                                            const uint32_t* __restrict__ lens, const uint32_t* __restrict__ recs32,
                                            const uint32_t* __restrict__ tmp32, const uint32_t* __restrict__ big32,
                                            skm_stored_kmer_data* __restrict__ out, uint32_t max_n,
                                            unsigned long long* queue) {
    // blocks of 64 jobs, one job per lane: the P^2 of a block on an even wave, its variance on an odd
    // one (grid may be smaller than the job count: a capped grid keeps few waves resident beside a
    // concurrent kernel, longest jobs first).  With `queue` (two zeroed counters) every wave takes
    // its next block from its half's counter, so a wave held by a block of long chains does not
    // also own a fixed share of the later blocks; without it, wave pairs stride over the blocks.
    const uint64_t lo = lo_p ? (uint64_t)*lo_p : 0ull;
    const uint64_t hi = min((uint64_t)*hi_p, cap);
    if (hi <= lo) return;
    jobs += lo;
    const uint64_t njobs = hi - lo;
    const bool var_wave = ((threadIdx.x >> 6) & 1u) != 0;
    const uint64_t pairs = (uint64_t)gridDim.x * (blockDim.x >> 7);
    auto take = [&]() -> uint64_t {
        uint32_t v = 0;
        if ((threadIdx.x & 63u) == 0) v = (uint32_t)atomicAdd(queue + (var_wave ? 1 : 0), 1ull);
        return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)v);
    };
    for (uint64_t pr = queue ? take() : (uint64_t)blockIdx.x * (blockDim.x >> 7) + (threadIdx.x >> 7); pr * 64 < njobs;
         pr = queue ? take() : pr + pairs) {
        const uint64_t j = pr * 64 + (threadIdx.x & 63u);
        if (j >= njobs) break;
        const Job jb = jobs[j];
        const uint64_t sel = jb.lens_off >> LENS_SEL_SHIFT;
        // lens == nullptr: stashed long jobs, lens_off is the samples' device address
        const uint32_t* x =
            !lens && sel == 0 ? reinterpret_cast<const uint32_t*>(jb.lens_off)
                              : (sel == LENS_IN_RECS ? recs32 : sel == LENS_IN_TMP ? tmp32 : sel == LENS_IN_BIG ? big32 : lens) +
                                    (jb.lens_off & LENS_OFF_MASK);
        const uint32_t n = jb.n;
        if (max_n && n >= max_n) continue;  // k_chain_long's (a wave pair each)
        SigStats st;
        st.init();
        if (var_wave)
            chain_run<true>(st, x, n);
        else
            chain_run<false>(st, x, n);
        if (var_wave)
            out[jb.out_idx].var = d2u16(st.var);
        else
            out[jb.out_idx].median = d2u16(st.h[2]);
    }
}

// the per-pass chains, and the stashed long chains of key-range passes (the same recurrences; a
// kernel symbol of their own so that profiles and counter passes tell the background batches apart)
__global__ __launch_bounds__(256) void k_chains(const Job* __restrict__ jobs, const unsigned long long* lo_p,
                                                const unsigned long long* hi_p, uint64_t cap,
                                                const uint32_t* __restrict__ lens, const uint32_t* __restrict__ recs32,
                                                const uint32_t* __restrict__ tmp32, const uint32_t* __restrict__ big32,
                                                skm_stored_kmer_data* __restrict__ out, uint32_t max_n = 0,
                                                unsigned long long* queue = nullptr) {
    chains_body(jobs, lo_p, hi_p, cap, lens, recs32, tmp32, big32, out, max_n, queue);
}
__global__ __launch_bounds__(256) void k_chains_stash(const Job* __restrict__ jobs, const unsigned long long* lo_p,
                                                      const unsigned long long* hi_p, uint64_t cap,
                                                      skm_stored_kmer_data* __restrict__ out, uint32_t max_n,
                                                      unsigned long long* queue) {
    chains_body(jobs, lo_p, hi_p, cap, nullptr, nullptr, nullptr, nullptr, out, max_n, queue);
}

// Diagnostics: one half of the wave-pair chain code alone (which 0: P^2, 1: variance).
__global__ __launch_bounds__(64) void k_chain_long_half(const Job* __restrict__ jobs, const uint32_t* __restrict__ lens,
                                                        int which, double* __restrict__ out) {
    const Job jb = jobs[blockIdx.x];
    const uint32_t* x = lens + (jb.lens_off & LENS_OFF_MASK);
    const double r = which == 0 ? chain_long_p2(x, jb.n) : which == 2 ? chain_long_p2v(x, jb.n) : chain_long_var(x, jb.n);
    if (threadIdx.x == 0) out[blockIdx.x] = r;
}

// Diagnostics: one chain, raw P^2 median and variance (mode 1: one lane; 2: wave pair).
__global__ __launch_bounds__(128) void k_chain_eval(const uint32_t* __restrict__ x, uint32_t n, int mode,
                                                    double* __restrict__ out) {
    if (mode == 2) {
        if (threadIdx.x < 64) {
            const double m = chain_long_p2v(x, n);
            if (threadIdx.x == 0) out[0] = m;
        } else {
            const double v = chain_long_var(x, n);
            if (threadIdx.x == 64) out[1] = v;
        }
    } else if ((threadIdx.x & 63u) == 0) {
        SigStats st;
        st.init();
        if (threadIdx.x == 0) {
            chain_run<false>(st, x, n);
            out[0] = st.h[2];
        } else {
            chain_run<true>(st, x, n);
            out[1] = st.var;
        }
    }
}

// Diagnostics: rcp_int / div_by against IEEE division.  Thread t checks m = t + 1 (and -m), then
// `per` pseudo-random (a, m) pairs with m up to 2^22 and a spanning heights and differences.
__global__ void k_div_check(uint64_t nm, uint32_t per, unsigned long long* __restrict__ bad) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nm) return;
    uint32_t nb = 0;
    const double m = (double)(t + 1);
    nb += rcp_int(m) != 1.0 / m;
    nb += rcp_int(-m) != 1.0 / -m;
    uint64_t x = t * 0x9E3779B97F4A7C15ull + 12345;
    for (uint32_t k = 0; k < per; ++k) {
        x ^= x >> 12;
        x ^= x << 25;
        x ^= x >> 27;
        const uint64_t r = x * 0x2545F4914F6CDD1Dull;
        const double b = (double)(1 + (r & 0x3FFFFFu)) * ((r >> 22) & 1 ? -1.0 : 1.0);
        const double a = ((double)(r >> 11) * (1.0 / 9007199254740992.0) - 0.5) *
                         (double)(1ull << ((r >> 23) & 31)) + (double)((r >> 40) & 0xFFFF);
        nb += div_by(a, b, rcp_int(b)) != a / b;
    }
    if (nb) atomicAdd(bad, (unsigned long long)nb);
}

// ------------------------------------------------------------------------------------------
// Kernels
// ------------------------------------------------------------------------------------------

// blk2seq[b] = sequence containing packed position 64*b
__global__ void k_blk2seq(const SeqMeta* __restrict__ meta, uint32_t nseq, uint32_t* __restrict__ blk2seq,
                          uint64_t nblk) {
    uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nseq) return;
    uint64_t a = meta[s].pstart, e = a + meta[s].len + 1;
    for (uint64_t b = (a + 63) >> 6; b < ((e + 63) >> 6) && b < nblk; ++b) blk2seq[b] = s;
}

struct ExtractArgs {
    const uint8_t* res;
    uint64_t rp, span;
    int owner_bits, b1_bits;
    int pass_bits;                  // key-range passes: windows whose mix43 top pass_bits == pass_id
    uint32_t pass_id;
    const uint8_t* ids;             // pass_bits > 0: per-window pass id (0xFF: no valid window)
    uint32_t* hist;                 // count pass: [wg][bucket]
    const uint32_t* offs;           // scatter pass: [wg][bucket] element offsets within the owner
    const uint64_t* owner_start;    // [owners+1]
    const uint32_t* blk2seq;        // sequence containing packed position 64*b
    const SeqMeta* meta;
    uint32_t s_base;                // global index of this shard's first sequence
    uint64_t pos_cap;               // key-range passes: capacity of the position list (pass_max)
    uint64_t* out_hi;
    uint64_t* out_lo;
};

// bit t set iff byte t of the 16 bytes equals v
__device__ __forceinline__ uint32_t match16(const uint4 w, uint32_t v) {
    const uint32_t x[4] = {w.x, w.y, w.z, w.w};
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) m |= (((x[j >> 2] >> (8 * (j & 3))) & 0xFFu) == v ? 1u : 0u) << j;
    return m;
}

// ------------------------------------------------------------------------------------------
// Key-range passes (out-of-core build).  A shard whose occurrence elements do not fit the work
// buffers is grouped in P = 2^pass_bits passes over disjoint k-mer ranges (the top pass_bits of
// mix43(key)); every k-mer lives in exactly one pass, so the passes' kept sets are disjoint and
// their union is the single-pass result.  k_pass_ids computes each window's pass id once per
// run (one scan of the resident residues); each pass's extract kernels then read the id bytes
// and hash only their own windows.  With counts != nullptr (prepare), it histograms the valid
// windows by pass id -- or, with pass_bits == 0, by the top 6 hash bits, which sizes the passes.
//
// Heavy-key routing.  The longest serial work of the build is the P^2 / variance chain of the
// heaviest k-mers (~10^6 samples at C3: ~0.3 s each); a pass that ends the run with such a chain
// leaves it as a tail after the last pass.  A Bloom filter of the keys with >= route_heavy_min
// occurrences (from a sampled count-min sketch at prepare) routes those keys of the second half of
// the passes into the first half (pass id - P/2), so their chains are stashed early and run beside
// the remaining passes.  Routing is a function of the key alone, so every occurrence of a k-mer is
// still in exactly one pass; the element keeps (natural ^ routed pass) above its rem bits
// (key_h43).  False positives of the filter only move a few light keys too.
// ------------------------------------------------------------------------------------------
constexpr int CMS_BITS = 22;        // count-min sketch of sampled windows: 2 rows of 2^22 u32 (32 MB)
constexpr int BLOOM_BITS = 18;      // Bloom filter of the heavy keys: 2^18 bits (32 KB of LDS), two probes
                                    // (C3: ~2*10^4 routed keys -> ~2 % false positives, harmless light
                                    // keys routed too)
constexpr int ROUTE_SAMPLE = 6;     // 1 in 2^6 window positions are sampled
constexpr uint32_t ROUTE_FIRST = 0x80000000u;  // k_pass_ids' vac flag: a heavy-only first pass

__device__ __forceinline__ uint32_t cms_slot(uint64_t h, int row) {
    return row == 0 ? (uint32_t)(h & ((1u << CMS_BITS) - 1u)) : (uint32_t)((h >> 21) & ((1u << CMS_BITS) - 1u));
}
__device__ __forceinline__ bool bloom_has(const uint32_t* bloom, uint64_t h) {
    const uint32_t b1 = (uint32_t)(h & ((1u << BLOOM_BITS) - 1u));
    const uint32_t b2 = (uint32_t)((h >> 24) & ((1u << BLOOM_BITS) - 1u));
    return ((bloom[b1 >> 5] >> (b1 & 31u)) & (bloom[b2 >> 5] >> (b2 & 31u)) & 1u) != 0;
}

// residue_code of every byte value in LDS (0xFF: not an ok_prot_ residue): the VALU-bound scans
// look a residue's code up instead of computing it (~10 VALU operations per byte)
__device__ __forceinline__ void fill_code_lut(uint8_t* lut) {
    for (uint32_t c = threadIdx.x; c < 256; c += blockDim.x) lut[c] = (uint8_t)residue_code(c);
}
// the 24 codes of a lane's 32 residue bytes (w[0..5] hold the first 24) and their validity bits
__device__ __forceinline__ uint32_t lut_codes24(const uint8_t* lut, const uint32_t (&w)[8], uint32_t (&code)[24]) {
    uint32_t valid = 0;
#pragma unroll
    for (int j = 0; j < 24; ++j) {
        const uint32_t cd = lut[(w[j >> 2] >> (8 * (j & 3))) & 0xFFu];
        valid |= (cd < 40u ? 1u : 0u) << j;
        code[j] = cd < 40u ? cd : 0u;
    }
    return valid;
}

// The base-40 keys of the 16 windows starting at codes[0..15] (24 codes): k = H * 40^4 + L with
// H, L the base-40 numbers of the window's first and last four codes, each rolled in 32-bit
// integer arithmetic (< 40^4 < 2^22: 24-bit multiply-adds), one 32 x 32 -> 64 multiply-add per
// key instead of a rolled 64-bit key (the emission and pass-id kernels are VALU-bound)
__device__ __forceinline__ void roll_keys16(const uint32_t (&code)[24], uint64_t (&k)[16]) {
    constexpr uint32_t P3 = 64000u, P4 = 2560000u;  // 40^3, 40^4
    uint32_t H = ((code[0] * 40u + code[1]) * 40u + code[2]) * 40u + code[3];
    uint32_t L = ((code[4] * 40u + code[5]) * 40u + code[6]) * 40u + code[7];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
        if (t > 0) {
            H = (H - code[t - 1] * P3) * 40u + code[t + 3];
            L = (L - code[t + 3] * P3) * 40u + code[t + 7];
        }
        k[t] = (uint64_t)H * P4 + L;
    }
}

// mix43 of the (valid) window at packed position p, or ~0 when the window is not valid
__device__ __forceinline__ uint64_t sampled_hash(const uint8_t* __restrict__ res, uint64_t p, uint64_t rp) {
    if (p >= rp) return ~0ull;
    const uint64_t a = p & ~7ull;  // the buffer is padded past rp
    const uint32_t sh = (uint32_t)(p & 7u) * 8u;
    const uint64_t w0 = *reinterpret_cast<const uint64_t*>(res + a);
    const uint64_t w1 = *reinterpret_cast<const uint64_t*>(res + a + 8);
    const uint64_t raw = sh ? (w0 >> sh) | (w1 << (64u - sh)) : w0;
    uint64_t k = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t cd = residue_code((uint32_t)((raw >> (8 * j)) & 0xFFu));
        if (cd >= 40u) return ~0ull;
        k = k * 40u + cd;
    }
    return mix43(k);
}

// the 8 residue bytes at packed position p (the buffer is padded past its end)
__device__ __forceinline__ uint64_t load_window(const uint8_t* __restrict__ res, uint64_t p) {
    const uint64_t a = p & ~7ull;
    const uint32_t sh = (uint32_t)(p & 7u) * 8u;
    const uint64_t w0 = *reinterpret_cast<const uint64_t*>(res + a);
    const uint64_t w1 = *reinterpret_cast<const uint64_t*>(res + a + 8);
    return sh ? (w0 >> sh) | (w1 << (64u - sh)) : w0;
}

// mix43 of the base-40 key of a (valid) window
__device__ __forceinline__ uint64_t window_hash(uint64_t raw) {
    uint64_t k = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) k = k * 40u + residue_code((uint32_t)((raw >> (8 * j)) & 0xFFu));
    return mix43(k);
}

// sketch (bloom == nullptr): count the sampled windows of every key into both rows;
// bloom pass: keys whose estimate (the smaller row) reaches `thresh` set their two filter bits,
// one byte per bit (bloom8[2^BLOOM_BITS]): at world > 1 the ranks' byte filters are combined by
// an element-wise max (= OR) over the ranks before k_bloom_pack, so every rank routes the same keys
__global__ __launch_bounds__(256) void k_route_sketch(const uint8_t* __restrict__ res, uint64_t rp,
                                                      uint32_t* __restrict__ cms, uint32_t thresh,
                                                      uint8_t* __restrict__ bloom) {
    const uint64_t ns = (rp + (1u << ROUTE_SAMPLE) - 1) >> ROUTE_SAMPLE;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ns; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t h = sampled_hash(res, i << ROUTE_SAMPLE, rp);
        if (h == ~0ull) continue;
        uint32_t* r0 = cms + cms_slot(h, 0);
        uint32_t* r1 = cms + (1u << CMS_BITS) + cms_slot(h, 1);
        if (!bloom) {
            atomicAdd(r0, 1u);
            atomicAdd(r1, 1u);
        } else if (min(*r0, *r1) >= thresh) {
            bloom[h & ((1u << BLOOM_BITS) - 1u)] = 1u;
            bloom[(h >> 24) & ((1u << BLOOM_BITS) - 1u)] = 1u;
        }
    }
}

// the byte filter -> the bit filter k_pass_ids keeps in LDS (one word per thread)
__global__ void k_bloom_pack(const uint8_t* __restrict__ bloom8, uint32_t* __restrict__ bloom) {
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= (1u << BLOOM_BITS) / 32u) return;
    const uint4* src = reinterpret_cast<const uint4*>(bloom8 + 32ull * w);
    const uint4 a = src[0], c = src[1];
    const uint32_t x[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
    uint32_t v = 0;
#pragma unroll
    for (int j = 0; j < 32; ++j) v |= (((x[j >> 2] >> (8 * (j & 3))) & 0xFFu) != 0u ? 1u : 0u) << j;
    bloom[w] = v;
}

// counts mode: pass_bits == owner_bits == 0 -> by the top 6 hash bits; else by (pass id <<
// owner_bits | owner),
// ncnt = 2^(pass_bits + owner_bits) counters (<= 4096).  Dynamic LDS: ncnt counters, then the Bloom
// filter when routing.
// rows != nullptr (the run's ids, with pass_bits > 0): workgroup w takes the contiguous windows
// [w * span, (w + 1) * span) (span a multiple of 16) and writes its windows per pass to
// rows[w * ncnt + pass] -- k_sel_scan turns them into each workgroup's output offsets in every
// pass's position list, so k_pass_emit writes the positions in order without atomics.
__global__ __launch_bounds__(256) void k_pass_ids(const uint8_t* __restrict__ res, uint64_t rp, int pass_bits,
                                                  int owner_bits, uint8_t* __restrict__ ids,
                                                  unsigned long long* __restrict__ counts,
                                                  const uint32_t* __restrict__ bloom, uint32_t ncnt,
                                                  uint32_t* __restrict__ rows = nullptr, uint64_t span = 0,
                                                  uint32_t vac = 0) {
    extern __shared__ uint32_t s_dyn[];
    __shared__ uint8_t s_code[256];
    uint32_t* s_cnt = s_dyn;
    uint32_t* s_bloom = s_dyn + ncnt;  // (1 << BLOOM_BITS) / 32 words when routing
    fill_code_lut(s_code);
    const bool tally = counts != nullptr || rows != nullptr;
    if (tally)
        for (uint32_t c = threadIdx.x; c < ncnt; c += blockDim.x) s_cnt[c] = 0;
    const bool route = bloom != nullptr && pass_bits >= 1;
    if (route)
        for (uint32_t w = threadIdx.x; w < (1u << BLOOM_BITS) / 32u; w += blockDim.x) s_bloom[w] = bloom[w];
    __syncthreads();
    const uint32_t half = pass_bits >= 1 ? 1u << (pass_bits - 1) : 0u;
    // routing vacates the last R passes: R = half (vac 0) maps pass p to p - P/2; any other R
    // spreads the heavy keys of the last R passes over the first P - R by 16 hash bits.
    // vac & ROUTE_FIRST: pass 0 holds the heavy keys only -- every heavy key goes to pass 0 and
    // the light keys of pass 0 spread over passes 1 .. P-1 by 16 hash bits
    const bool first = (vac & ROUTE_FIRST) != 0;
    vac &= ~ROUTE_FIRST;
    const uint32_t R = vac ? min(vac, (1u << pass_bits) - 1u) : half, keep = (1u << pass_bits) - R;
    const uint64_t nchunk = (rp + 15) >> 4;
    const uint64_t c0 = rows ? ((uint64_t)blockIdx.x * span >> 4) + threadIdx.x : (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t cend = rows ? min(nchunk, ((uint64_t)blockIdx.x + 1) * span >> 4) : nchunk;
    const uint64_t cstep = rows ? (uint64_t)blockDim.x : (uint64_t)gridDim.x * blockDim.x;
    // the next chunk's residues are loaded before this chunk is hashed
    uint4 n0 = make_uint4(0u, 0u, 0u, 0u), n1 = n0;
    if (c0 < cend) {
        n0 = *reinterpret_cast<const uint4*>(res + (c0 << 4));
        n1 = *reinterpret_cast<const uint4*>(res + (c0 << 4) + 16);
    }
    for (uint64_t c = c0; c < cend; c += cstep) {
        const uint64_t base = c << 4;
        const uint4 v0 = n0, v1 = n1;
        if (c + cstep < cend) {
            n0 = *reinterpret_cast<const uint4*>(res + ((c + cstep) << 4));
            n1 = *reinterpret_cast<const uint4*>(res + ((c + cstep) << 4) + 16);
        }
        const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        uint32_t code[24];
        const uint32_t valid = lut_codes24(s_code, w, code);
        uint64_t kk[16];
        roll_keys16(code, kk);
        uint32_t out[4] = {0u, 0u, 0u, 0u};
        // every lane computes every window's id with selects, one loop per (uniform) mode: the kernel
        // is VALU-bound, and per-window exec-mask branches cost more than the work they skip
        auto windows = [&](auto mode) {
            constexpr int M = decltype(mode)::value;  // 0: prepare counts, 1: no routing, 2: routing, 3: route_first
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const bool v = ((valid >> t) & 0xFFu) == 0xFFu && base + t < rp;
                const uint64_t h = mix43(kk[t]);
                uint32_t id = 0xFFu;
                if constexpr (M == 0) {
                    if (counts && v) atomicAdd(&s_cnt[(uint32_t)(h >> (KEY_BITS - 6))], 1u);
                } else {
                    id = pass_bits ? (uint32_t)(h >> (KEY_BITS - pass_bits)) : 0u;
                    if constexpr (M >= 2) {
                        const bool hb = bloom_has(s_bloom, h);
                        const uint32_t h16 = (uint32_t)(h & 0xFFFFu);
                        if constexpr (M == 3)
                            id = hb ? 0u : (id == 0 ? 1u + ((h16 * ((1u << pass_bits) - 1u)) >> 16) : id);
                        else
                            id = (id >= keep && hb) ? (R == half ? id - half : (h16 * keep) >> 16) : id;
                    }
                    if (tally && v) {
                        const uint32_t own = (uint32_t)(h >> (KEY_BITS - pass_bits - owner_bits)) & ((1u << owner_bits) - 1u);
                        atomicAdd(&s_cnt[(id << owner_bits) | own], 1u);
                    }
                    id = v ? id : 0xFFu;
                }
                out[t >> 2] |= id << (8 * (t & 3));
            }
        };
        if (pass_bits == 0 && owner_bits == 0)
            windows(std::integral_constant<int, 0>{});
        else if (!route)
            windows(std::integral_constant<int, 1>{});
        else if (first)
            windows(std::integral_constant<int, 3>{});
        else
            windows(std::integral_constant<int, 2>{});
        if (!counts && ids) *reinterpret_cast<uint4*>(ids + base) = make_uint4(out[0], out[1], out[2], out[3]);
    }
    if (counts) {
        __syncthreads();
        for (uint32_t c = threadIdx.x; c < ncnt; c += blockDim.x)
            if (s_cnt[c]) atomicAdd(&counts[c], (unsigned long long)s_cnt[c]);
    }
    if (rows) {
        __syncthreads();
        for (uint32_t c = threadIdx.x; c < ncnt; c += blockDim.x) rows[(uint64_t)blockIdx.x * ncnt + c] = s_cnt[c];
    }
}

// Every pass's position list: workgroup w of k_pass_ids / k_pass_emit writes its windows of
// pass p at off[p * (nwg + 1) + w] (exclusive scan over w), npos[p] = the pass's window count
// (checked against the list's capacity: a larger pass fails the run, SKM_E_STATE).  One workgroup
// per pass.
constexpr uint32_t SEL_WG = 8192;   // tally rows: k_pass_ids workgroups = k_pass_emit waves (at least;
                                    //   more when a row's span would pass 2^REL_BITS residues)
__global__ __launch_bounds__(1024) void k_sel_scan(const uint32_t* __restrict__ rows, uint32_t nwg, uint32_t P,
                                                   uint64_t* __restrict__ off, unsigned long long* __restrict__ npos,
                                                   uint64_t cap, unsigned long long* __restrict__ run) {
    __shared__ uint32_t s_wave[17];
    const uint32_t p = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
    const uint32_t per = (nwg + nt - 1) / nt, a = min(nwg, tid * per), e = min(nwg, a + per);
    uint64_t loc = 0;
    for (uint32_t w = a; w < e; ++w) loc += rows[(uint64_t)w * P + p];
    uint32_t tot32;
    // windows per pass fit 32 bits (prepare checks the largest pass against 2^32)
    uint64_t r = wg_exclusive_scan((uint32_t)loc, s_wave, tot32);
    for (uint32_t w = a; w < e; ++w) {
        off[(uint64_t)p * (nwg + 1) + w] = r;
        r += rows[(uint64_t)w * P + p];
    }
    if (tid == 0) {
        off[(uint64_t)p * (nwg + 1) + nwg] = tot32;
        npos[p] = tot32;
        if (tot32 > cap) atomicOr(&run[RUN_FLAGS], (unsigned long long)RUN_F_CAP);
    }
}

// The window positions of a GROUP of G consecutive key-range passes, each pass's list in position
// order (replaces round 3's per-pass k_pass_select, which re-read every pass-id byte and every
// matched window's residues on each of the P passes: 33 GB per pass at C3).  One wave per tally
// row (k_pass_ids' workgroup span, SEL_WG of them): per tile of 64 x 16 windows each lane loads its
// 16 pass ids and its 32 residue bytes (both coalesced), rolls the 16 keys in registers and mixes
// only the group's windows for their level-1 bucket; the wave ranks them pass-major with DPP
// scans, stages the tile's entries in its own 4 KB of LDS and writes one contiguous run per pass
// at its k_sel_scan offset -- no workgroup barrier anywhere (round-4 first form: 1024-thread
// workgroups hashing every window of every group, ~50 ms per group at C3).  An entry is the
// window's 43-bit key hash with the window's offset in its row's span above it (REL_BITS):
// the pass's histogram (k_pass_hist) and the staged scatter (k_extract_stage_pos) take the bucket
// and the rem bits from the hash, so neither looks at the residues again (round 6: the staging
// re-read every residue line and re-hashed every window once per pass -- 16.5 GB per pass at C3);
// the staging finds the window's position as row * span + offset, the row from k_sel_scan's
// offsets.  Reads 1 B of id + 1 B of residue per window per group, writes 8 B per window of the group.
constexpr uint32_t EMIT_THREADS = 64;
constexpr int REL_BITS = 21;                      // pass entry: offset in the row's span << 43 | mix43(key)
constexpr uint64_t H43_MASK = (1ull << KEY_BITS) - 1ull;
static_assert(KEY_BITS + REL_BITS == 64, "the pass entry is one u64");
template <uint32_t G>
__global__ __launch_bounds__(EMIT_THREADS) void k_pass_emit(const uint8_t* __restrict__ res, const uint8_t* __restrict__ ids,
                                                           uint64_t rp, uint32_t pass0, uint64_t span,
                                                           const uint64_t* __restrict__ seloff, uint32_t nrows,
                                                           uint64_t* __restrict__ pos, uint64_t cap) {
    __shared__ uint64_t s_out[16 * 64];  // the tile's entries, pass-major: window in the tile << 43 | hash
    __shared__ uint8_t s_code[256];
    const uint32_t lane = threadIdx.x;
    fill_code_lut(s_code);
    wave_sync();
    uint64_t run[G];
#pragma unroll
    for (uint32_t q = 0; q < G; ++q) run[q] = seloff[(uint64_t)(pass0 + q) * (nrows + 1) + blockIdx.x];
    const uint64_t a = (uint64_t)blockIdx.x * span, e = min(rp, a + span);
    // the next tile's ids and residues are loaded before this tile is processed (round 5 loaded
    // the residues only after the ids showed a window of the group: two serial latencies a tile)
    uint4 nid = make_uint4(~0u, ~0u, ~0u, ~0u), nr0 = make_uint4(0u, 0u, 0u, 0u), nr1 = nr0;
    if (a + 16ull * lane < e) {
        nid = *reinterpret_cast<const uint4*>(ids + a + 16ull * lane);
        nr0 = *reinterpret_cast<const uint4*>(res + a + 16ull * lane);
        nr1 = *reinterpret_cast<const uint4*>(res + a + 16ull * lane + 16);
    }
    for (uint64_t t0 = a; t0 < e; t0 += 16ull * 64) {
        const uint64_t base = t0 + 16ull * lane;
        const uint4 id4 = nid, v0 = nr0, v1 = nr1;
        {
            const uint64_t nb = base + 16ull * 64;
            if (nb < e) {  // the residue buffer is padded past rp, the id buffer to a multiple of 16
                nid = *reinterpret_cast<const uint4*>(ids + nb);
                nr0 = *reinterpret_cast<const uint4*>(res + nb);
                nr1 = *reinterpret_cast<const uint4*>(res + nb + 16);
            }
        }
        uint32_t qs[4] = {~0u, ~0u, ~0u, ~0u};  // byte t: the window's pass within the group (0xFF: none)
        uint64_t hs[16];                        // the window's key hash
        uint32_t cnt[G];
#pragma unroll
        for (uint32_t q = 0; q < G; ++q) cnt[q] = 0;
        constexpr bool PACK = G <= 4;  // the lane's counts as 8-bit fields of one word
        uint32_t pc = 0;
        if (base < e) {
            const uint32_t idw[4] = {id4.x, id4.y, id4.z, id4.w};
            uint32_t any = 0;
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const uint32_t q = ((idw[t >> 2] >> (8 * (t & 3))) & 0xFFu) - pass0;  // 0xFF (no window): >= G
                if (q < G && base + t < e) {
                    any |= 1u << t;
                    qs[t >> 2] &= ~(0xFFu << (8 * (t & 3)));
                    qs[t >> 2] |= q << (8 * (t & 3));
                    if constexpr (PACK) {
                        pc += 1u << (8u * q);
                    } else {
#pragma unroll
                        for (uint32_t j = 0; j < G; ++j) cnt[j] += q == j ? 1u : 0u;
                    }
                }
            }
            if (any) {  // the 16 keys rolled from the lane's 24 residues, mixed for the group's windows
                const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
                uint32_t code[24];
                (void)lut_codes24(s_code, w, code);
                uint64_t k[16];
                roll_keys16(code, k);
#pragma unroll
                for (int t = 0; t < 16; ++t) hs[t] = ((any >> t) & 1u) ? mix43(k[t]) : 0ull;
            }
        }
        if constexpr (PACK) {
#pragma unroll
            for (uint32_t q = 0; q < G; ++q) cnt[q] = (pc >> (8u * q)) & 0xFFu;
        }
        // pass-major ranks of the wave's tile: one DPP scan per pass of the group
        uint32_t off[G], qa[G + 1];
        qa[0] = 0;
#pragma unroll
        for (uint32_t q = 0; q < G; ++q) {
            const uint32_t inc = wave_incl_scan(cnt[q]);
            const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
            off[q] = qa[q] + inc - cnt[q];
            qa[q + 1] = qa[q] + tot;
        }
        if constexpr (PACK) {  // the lane's running offsets as 16-bit fields of one u64 (< 1024 each)
            uint64_t op = 0;
#pragma unroll
            for (uint32_t q = 0; q < G; ++q) op |= (uint64_t)off[q] << (16u * q);
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const uint32_t q = (qs[t >> 2] >> (8 * (t & 3))) & 0xFFu;
                if (q >= G) continue;
                const uint32_t f = (uint32_t)(op >> (16u * q)) & 0xFFFFu;
                op += 1ull << (16u * q);
                s_out[f] = ((uint64_t)(16u * lane + (uint32_t)t) << KEY_BITS) | hs[t];
            }
        } else {
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const uint32_t q = (qs[t >> 2] >> (8 * (t & 3))) & 0xFFu;
                if (q >= G) continue;
                uint32_t f = 0;
#pragma unroll
                for (uint32_t j = 0; j < G; ++j)
                    if (q == j) f = off[j]++;
                s_out[f] = ((uint64_t)(16u * lane + (uint32_t)t) << KEY_BITS) | hs[t];
            }
        }
        wave_sync();
        for (uint32_t j = lane; j < qa[G]; j += 64) {
            uint32_t q = 0;
#pragma unroll
            for (uint32_t k = 1; k < G; ++k) q += j >= qa[k] ? 1u : 0u;
            uint64_t o = 0;
#pragma unroll
            for (uint32_t k = 0; k < G; ++k)
                if (q == k) o = run[k] + (j - qa[k]);
            const uint64_t v = s_out[j];
            if (o < cap) pos[(uint64_t)q * cap + o] = ((t0 - a + (v >> KEY_BITS)) << KEY_BITS) | (v & H43_MASK);
        }
#pragma unroll
        for (uint32_t q = 0; q < G; ++q) run[q] += qa[q + 1] - qa[q];
        wave_sync();  // s_out is rewritten by the next tile
    }
}

// The level-1 histogram of each pass of a group from its entries' bucket bits: blockIdx.y = the
// pass within the group, blockIdx.x strides over its list; NB counters in LDS, merged once.
constexpr uint32_t PH_THREADS = 512;
__global__ __launch_bounds__(PH_THREADS) void k_pass_hist(const uint64_t* __restrict__ pos, uint64_t cap,
                                                          const unsigned long long* __restrict__ npos, uint32_t NB,
                                                          int rem_bits, uint32_t* __restrict__ hist) {
    extern __shared__ uint32_t s_h[];  // [NB]
    const uint32_t q = blockIdx.y;
    for (uint32_t k = threadIdx.x; k < NB; k += PH_THREADS) s_h[k] = 0;
    __syncthreads();
    const uint64_t n = min((uint64_t)npos[q], cap);
    const uint64_t* p = pos + (uint64_t)q * cap;
    constexpr uint32_t U = 4;
    for (uint64_t j0 = (uint64_t)blockIdx.x * PH_THREADS * U; j0 < n; j0 += (uint64_t)gridDim.x * PH_THREADS * U) {
        uint64_t v[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint64_t j = j0 + u * PH_THREADS + threadIdx.x;
            v[u] = j < n ? p[j] : ~0ull;
        }
#pragma unroll
        for (uint32_t u = 0; u < U; ++u)
            if (v[u] != ~0ull) atomicAdd(&s_h[(uint32_t)((v[u] & H43_MASK) >> rem_bits) & (NB - 1)], 1u);
    }
    __syncthreads();
    uint32_t* hq = hist + (uint64_t)q * NB;
    for (uint32_t k = threadIdx.x; k < NB; k += PH_THREADS)
        if (s_h[k]) atomicAdd(&hq[k], s_h[k]);
}

// Per-workgroup histogram of the level-1 buckets (count pass, one key-range pass = the whole
// key space).
__global__ __launch_bounds__(EX_THREADS) void k_extract(ExtractArgs X) {
    const uint8_t* __restrict__ res = X.res;
    const uint64_t rp = X.rp, span = X.span;
    extern __shared__ uint32_t s_cnt[];  // [NB]
    const int nbits = X.owner_bits + X.b1_bits;
    const uint32_t NB = 1u << nbits;
    const int rem_bits = KEY_BITS - nbits;
    const uint32_t wg = blockIdx.x;
    for (uint32_t b = threadIdx.x; b < NB; b += blockDim.x) s_cnt[b] = 0u;
    __syncthreads();
    const uint64_t begin = (uint64_t)wg * span;
    const uint64_t end = min(begin + span, rp);
    for (uint64_t base = begin + (uint64_t)threadIdx.x * EX_POS_PER_THREAD; base < end;
         base += (uint64_t)blockDim.x * EX_POS_PER_THREAD) {
        const uint4 v0 = *reinterpret_cast<const uint4*>(res + base);
        const uint4 v1 = *reinterpret_cast<const uint4*>(res + base + 16);
        const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        uint32_t code[24];
        uint32_t valid = 0;
#pragma unroll
        for (int j = 0; j < 24; ++j) {
            uint32_t c = (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            uint32_t cd = residue_code(c);
            valid |= (cd < 40u ? 1u : 0u) << j;
            code[j] = cd < 40u ? cd : 0u;
        }
        uint64_t k = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) k = k * 40u + code[j];
        constexpr uint64_t P7 = 6553600000000ull / 40u;  // 40^7
#pragma unroll
        for (int t = 0; t < EX_POS_PER_THREAD; ++t) {
            if (t > 0) k = (k - (uint64_t)code[t - 1] * P7) * 40u + code[t + 7];
            const uint64_t p = base + t;
            if (((valid >> t) & 0xFFu) == 0xFFu && p < end) {
                const uint64_t h = mix43(k);
                atomicAdd(&s_cnt[(uint32_t)(h >> rem_bits)], 1u);
            }
        }
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < NB; b += blockDim.x) X.hist[(uint64_t)wg * NB + b] = s_cnt[b];
}

// ------------------------------------------------------------------------------------------
// Two-pass LDS-staged scatter of the occurrence elements (replaces a direct 4096-way scatter,
// whose 16-byte stores from every workgroup into every bucket left partial lines in L2:
// ~4x write amplification measured).  Pass 1 partitions by the top 6 bucket bits (64-way) as
// the windows are extracted; pass 2 splits each of those ranges by the remaining bits.  Each
// pass stages 4096 elements per round in LDS, sorted by destination, reserves one global range
// per destination per round with one atomic, and writes runs of ~64 / ~32 contiguous elements.
// Element order inside a bucket is immaterial (elements carry their ordinal).  Between the
// passes the low 16 bits of lo hold the full bucket id instead of (len - i) mod 2^16, which
// pass 2 restores from len mod 2^16 (hi[63:48]) and i.
// ------------------------------------------------------------------------------------------
constexpr int SC_ROUND = 4096;        // elements staged per round (64 KB of LDS)
constexpr int SC_L0_BITS = 6;         // pass-1 fan-out
constexpr int SC_POS = SC_ROUND / EX_THREADS;  // windows per thread per round (8)
constexpr uint64_t SC_SLICE = 65536;  // pass-2 elements per workgroup

// Staged-scatter cursors, one per 128-byte line: every workgroup of a launch reserves from the
// same 64 level-0 cursors each round, and atomics on one line serialise.
constexpr uint32_t CUR_STRIDE = 16;

template <int R>
struct StageLdsT {
    uint64_t hi[R];
    uint64_t lo[R];
    uint8_t dst[R];
    uint32_t cnt[128];
    uint32_t off[129];
    unsigned long long base[128];
    uint32_t wave[48];
};
using StageLds = StageLdsT<SC_ROUND>;
// k_extract_stage_pos's half round (option stage_round = 1, the default): 2048 elements, ~37 KB
// of LDS, four workgroups per CU instead of two to hide the position -> sequence -> window gather
// chain (C3 step 2046 -> 1950 ms, the kernel 435 -> 320 ms per step)
constexpr int SC_ROUND_HALF = SC_ROUND / 2;

// The rank of a lane's element among its destination's elements (LDS counter cnt[d]), called by
// every lane of the wave (v: the lane has an element): the lanes that share the first live lane's
// destination reserve together with one atomic, the rest one each.  A heavy key crowds its
// elements into one destination, and same-address LDS atomics serialise lane by lane.
__device__ __forceinline__ uint32_t agg_rank(uint32_t* cnt, uint32_t d, bool v) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t act = __ballot(v);
    if (act == 0) return 0u;
    const uint32_t l0 = (uint32_t)__ffsll((long long)act) - 1u;
    const uint32_t d0 = (uint32_t)__builtin_amdgcn_readlane((int)d, (int)l0);
    const uint64_t same = __ballot(v && d == d0);
    uint32_t base = 0;
    if (lane == l0) base = atomicAdd(&cnt[d0], (uint32_t)__popcll(same));
    base = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)l0);
    if (v && d == d0) return base + (uint32_t)__popcll(same & ((1ull << lane) - 1ull));
    return v ? atomicAdd(&cnt[d], 1u) : 0u;
}
// the same aggregation for a count (no ranks)
__device__ __forceinline__ void agg_count(uint32_t* cnt, uint32_t d, bool v) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t act = __ballot(v);
    if (act == 0) return;
    const uint32_t l0 = (uint32_t)__ffsll((long long)act) - 1u;
    const uint32_t d0 = (uint32_t)__builtin_amdgcn_readlane((int)d, (int)l0);
    const uint64_t same = __ballot(v && d == d0);
    if (lane == l0) atomicAdd(&cnt[d0], (uint32_t)__popcll(same));
    if (v && d != d0) atomicAdd(&cnt[d], 1u);
}

// counts already in L.cnt[0..nd): exclusive offsets, then one global reservation per destination
template <class Lds>
__device__ __forceinline__ uint32_t stage_reserve(Lds& L, uint32_t nd, unsigned long long* __restrict__ cur,
                                                  uint32_t cur_base) {
    const uint32_t t = threadIdx.x;
    uint32_t tot;
    const uint32_t c = t < nd ? L.cnt[t] : 0u;
    const uint32_t ex = wg_exclusive_scan(c, L.wave, tot);
    if (t < nd) {
        L.off[t] = ex;
        L.base[t] = c ? atomicAdd(&cur[(uint64_t)(cur_base + t) * CUR_STRIDE], (unsigned long long)c) : 0ull;
    }
    if (t == 0) L.off[nd] = tot;
    __syncthreads();
    return tot;
}

__global__ __launch_bounds__(EX_THREADS, 2) void k_extract_stage(ExtractArgs X, unsigned long long* __restrict__ cur0,
                                                                 uint64_t* __restrict__ out_hi,
                                                                 uint64_t* __restrict__ out_lo) {
    __shared__ StageLds L;
    const uint8_t* __restrict__ res = X.res;
    const int nbits = X.owner_bits + X.b1_bits;
    const int rem_bits = KEY_BITS - nbits;
    const uint64_t rem_mask = (1ull << rem_bits) - 1;
    const int l0_shift = nbits - SC_L0_BITS;
    const uint64_t begin = (uint64_t)blockIdx.x * X.span;
    const uint64_t end = min(begin + X.span, X.rp);
    // the next round's residues and sequence record are loaded before this round's LDS work, so
    // their HBM latency (blk2seq -> meta is a dependent pair) overlaps the staging
    uint2 nv0 = make_uint2(0u, 0u), nv1 = make_uint2(0u, 0u);
    uint32_t ns = 0;
    SeqMeta nm{};
    auto fetch = [&](uint64_t b) {
        const uint64_t q = b + (uint64_t)threadIdx.x * SC_POS;
        nv0 = nv1 = make_uint2(0u, 0u);
        if (q < end) {  // the residue buffer is padded by 64 bytes past rp, not more
            nv0 = *reinterpret_cast<const uint2*>(res + q);
            nv1 = *reinterpret_cast<const uint2*>(res + q + 8);
            ns = X.blk2seq[q >> 6];
            nm = X.meta[ns];
        }
    };
    fetch(begin);
    for (uint64_t base = begin; base < end; base += SC_ROUND) {
        if (threadIdx.x < 128) L.cnt[threadIdx.x] = 0;
        __syncthreads();
        const uint64_t p0 = base + (uint64_t)threadIdx.x * SC_POS;
        const uint2 v0 = nv0, v1 = nv1;
        uint32_t s = ns;
        SeqMeta m = nm;
        if (base + SC_ROUND < end) fetch(base + SC_ROUND);
        const uint32_t w[4] = {v0.x, v0.y, v1.x, v1.y};
        uint32_t code[16];
        uint32_t valid = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t cd = residue_code((w[j >> 2] >> (8 * (j & 3))) & 0xFFu);
            valid |= (cd < 40u ? 1u : 0u) << j;
            code[j] = cd < 40u ? cd : 0u;
        }
        uint64_t k = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) k = k * 40u + code[j];
        constexpr uint64_t P7 = 6553600000000ull / 40u;  // 40^7
        uint64_t eh[SC_POS], el[SC_POS];
        uint32_t rk[SC_POS], l0[SC_POS];
        uint32_t ok = 0;
#pragma unroll
        for (int t = 0; t < SC_POS; ++t) {
            if (t > 0) k = (k - (uint64_t)code[t - 1] * P7) * 40u + code[t + 7];
            const uint64_t p = p0 + t;
            eh[t] = el[t] = 0;
            rk[t] = l0[t] = 0;
            if (((valid >> t) & 0xFFu) == 0xFFu && p < end) {
                while (p > m.pstart + m.len) m = X.meta[++s];  // valid windows never span a separator
                const uint64_t h = mix43(k);
                const uint32_t bucket = (uint32_t)(h >> rem_bits);
                make_elem(h & rem_mask, X.s_base + s, (uint32_t)(p - m.pstart), m, eh[t], el[t]);
                el[t] = (el[t] & ~0xFFFFull) | bucket;  // bucket id rides in the offset field until pass 2
                l0[t] = bucket >> l0_shift;
                rk[t] = atomicAdd(&L.cnt[l0[t]], 1u);
                ok |= 1u << t;
            }
        }
        __syncthreads();
        const uint32_t tot = stage_reserve(L, 1u << SC_L0_BITS, cur0, 0);
#pragma unroll
        for (int t = 0; t < SC_POS; ++t)
            if ((ok >> t) & 1u) {
                const uint32_t slot = L.off[l0[t]] + rk[t];
                L.hi[slot] = eh[t];
                L.lo[slot] = el[t];
                L.dst[slot] = (uint8_t)l0[t];
            }
        __syncthreads();
        for (uint32_t j = threadIdx.x; j < tot; j += blockDim.x) {
            const uint32_t d = L.dst[j];
            const uint64_t o = L.base[d] + (j - L.off[d]);
            out_hi[o] = L.hi[j];
            out_lo[o] = L.lo[j];
        }
        __syncthreads();
    }
}

// The staged level-0 scatter over a key-range pass's entries pos[0..n) (same staging rounds as
// k_extract_stage).  An entry carries the window's key hash (bucket and rem bits, no residue
// read) and its offset in its emission row's span; the row is found from the pass's row offsets
// sel[0..nrows] (k_sel_scan): each thread's entries ascend, so it walks its row forward -- one
// binary search per thread at the start, then a compare per entry.  Each position finds its
// sequence through blk2seq, reusing the previous one while it still contains the window.
template <int R, int MINB>
__global__ __launch_bounds__(EX_THREADS, MINB) void k_extract_stage_pos(ExtractArgs X, const uint64_t* __restrict__ pos,
                                                                        const unsigned long long* __restrict__ np,
                                                                        const uint64_t* __restrict__ sel, uint32_t nrows,
                                                                        uint64_t sel_span,
                                                                        unsigned long long* __restrict__ cur0,
                                                                        uint64_t* __restrict__ out_hi,
                                                                        uint64_t* __restrict__ out_lo) {
    constexpr int SC_POS = R / EX_THREADS;
    const uint64_t n = min((uint64_t)*np, X.pos_cap);
    __shared__ StageLdsT<R> L;
    const int nbits = X.owner_bits + X.b1_bits;
    const uint32_t NB = 1u << nbits;
    const int rem_bits = KEY_BITS - X.pass_bits - nbits;
    const uint64_t rem_mask = (1ull << rem_bits) - 1;
    const int l0_shift = nbits - SC_L0_BITS;
    const uint64_t begin = (uint64_t)blockIdx.x * X.span, end = min(begin + X.span, n);
    uint32_t s = 0xFFFFFFFFu;
    SeqMeta m{};
    // the emission row of this thread's first entry: the last row whose offset is <= it
    uint32_t row = 0;
    {
        const uint64_t j0 = begin + (uint64_t)threadIdx.x * SC_POS;
        uint32_t lo = 0, hi = nrows;  // sel[lo] <= j0 < sel[hi] (sel[nrows] = n)
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (sel[mid] <= j0)
                lo = mid;
            else
                hi = mid;
        }
        row = lo;
    }
    uint64_t row_end = sel[row + 1];
    // the next round's entries are loaded before this round's sequence gathers and LDS work
    uint64_t nxt[SC_POS];
#pragma unroll
    for (int t = 0; t < SC_POS; ++t) {
        const uint64_t j = begin + (uint64_t)threadIdx.x * SC_POS + t;
        nxt[t] = j < end ? pos[j] : ~0ull;
    }
    for (uint64_t base = begin; base < end; base += R) {
        if (threadIdx.x < 128) L.cnt[threadIdx.x] = 0;
        __syncthreads();
        uint64_t ent[SC_POS];
#pragma unroll
        for (int t = 0; t < SC_POS; ++t) ent[t] = nxt[t];
#pragma unroll
        for (int t = 0; t < SC_POS; ++t) {
            const uint64_t j = base + R + (uint64_t)threadIdx.x * SC_POS + t;
            nxt[t] = j < end ? pos[j] : ~0ull;
        }
        uint64_t eh[SC_POS], el[SC_POS];
        uint32_t rk[SC_POS], l0[SC_POS];
#pragma unroll
        for (int t = 0; t < SC_POS; ++t) {
            eh[t] = el[t] = 0;
            rk[t] = l0[t] = 0;
            if (ent[t] != ~0ull) {
                const uint64_t j = base + (uint64_t)threadIdx.x * SC_POS + t;
                while (j >= row_end) row_end = sel[++row + 1];  // rows without entries are skipped
                const uint64_t p = (uint64_t)row * sel_span + (ent[t] >> KEY_BITS);
                if (s == 0xFFFFFFFFu || p < m.pstart || p > m.pstart + m.len) {
                    s = X.blk2seq[p >> 6];
                    m = X.meta[s];
                }
                while (p > m.pstart + m.len) m = X.meta[++s];
                const uint64_t h = ent[t] & H43_MASK;
                const uint32_t bucket = (uint32_t)(h >> rem_bits) & (NB - 1);
                // a heavy key routed in from a later pass keeps (natural ^ this pass) above its rem
                const uint64_t route = (uint64_t)((uint32_t)(h >> (KEY_BITS - X.pass_bits)) ^ X.pass_id) << rem_bits;
                make_elem((h & rem_mask) | route, X.s_base + s, (uint32_t)(p - m.pstart), m, eh[t], el[t]);
                el[t] = (el[t] & ~0xFFFFull) | bucket;  // bucket id rides in the offset field until pass 2
                l0[t] = bucket >> l0_shift;
            }
        }
#pragma unroll
        for (int t = 0; t < SC_POS; ++t) rk[t] = agg_rank(L.cnt, l0[t], ent[t] != ~0ull);
        __syncthreads();
        const uint32_t tot = stage_reserve(L, 1u << SC_L0_BITS, cur0, 0);
#pragma unroll
        for (int t = 0; t < SC_POS; ++t)
            if (ent[t] != ~0ull) {
                const uint32_t slot = L.off[l0[t]] + rk[t];
                L.hi[slot] = eh[t];
                L.lo[slot] = el[t];
                L.dst[slot] = (uint8_t)l0[t];
            }
        __syncthreads();
        for (uint32_t j = threadIdx.x; j < tot; j += blockDim.x) {
            const uint32_t d = L.dst[j];
            const uint64_t o = L.base[d] + (j - L.off[d]);
            out_hi[o] = L.hi[j];
            out_lo[o] = L.lo[j];
        }
        __syncthreads();
    }
}

// cur0[b0] = start of pass-1 range b0; cur1[b] = start of bucket b; slice prefix for pass 2
__global__ void k_stage_init(const uint64_t* __restrict__ bstart, uint32_t NB, int l0_shift,
                             unsigned long long* __restrict__ cur0, unsigned long long* __restrict__ cur1,
                             uint32_t* __restrict__ slice_base) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < NB) cur1[(uint64_t)t * CUR_STRIDE] = bstart[t];
    if (blockIdx.x == 0) {
        __shared__ uint32_t s_n[(1 << SC_L0_BITS) + 1];
        const uint32_t n0 = 1u << SC_L0_BITS;
        if (threadIdx.x < n0) {
            const uint64_t a = bstart[(uint64_t)threadIdx.x << l0_shift];
            const uint64_t e = bstart[(uint64_t)(threadIdx.x + 1) << l0_shift];
            cur0[threadIdx.x * CUR_STRIDE] = a;
            s_n[threadIdx.x] = (uint32_t)((e - a + SC_SLICE - 1) / SC_SLICE);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t acc = 0;
            for (uint32_t b = 0; b < n0; ++b) {
                slice_base[b] = acc;
                acc += s_n[b];
            }
            slice_base[n0] = acc;
        }
    }
}

__global__ __launch_bounds__(EX_THREADS, 2) void k_split_stage(const uint64_t* __restrict__ in_hi,
                                                               const uint64_t* __restrict__ in_lo,
                                                               const uint64_t* __restrict__ bstart, int nbits,
                                                               const uint32_t* __restrict__ slice_base,
                                                               unsigned long long* __restrict__ cur1,
                                                               uint64_t* __restrict__ out_hi,
                                                               uint64_t* __restrict__ out_lo) {
    __shared__ StageLds L;
    const uint32_t n0 = 1u << SC_L0_BITS;
    const int sub_bits = nbits - SC_L0_BITS;
    const uint32_t nsub = 1u << sub_bits;
    const uint32_t w = blockIdx.x;
    if (w >= slice_base[n0]) return;
    uint32_t b0 = 0;
    while (b0 + 1 < n0 && slice_base[b0 + 1] <= w) ++b0;
    const uint64_t a0 = bstart[(uint64_t)b0 << sub_bits], e0 = bstart[(uint64_t)(b0 + 1) << sub_bits];
    const uint64_t begin = a0 + (uint64_t)(w - slice_base[b0]) * SC_SLICE;
    const uint64_t end = min(begin + SC_SLICE, e0);
    for (uint64_t base = begin; base < end; base += SC_ROUND) {
        if (threadIdx.x < 128) L.cnt[threadIdx.x] = 0;
        __syncthreads();
        uint64_t eh[SC_POS], el[SC_POS];
        uint32_t rk[SC_POS], sb[SC_POS];
#pragma unroll
        for (int t = 0; t < SC_POS; ++t) {
            const uint64_t j = base + threadIdx.x + (uint64_t)t * EX_THREADS;
            rk[t] = sb[t] = 0;
            eh[t] = el[t] = 0;
            if (j < end) {
                eh[t] = in_hi[j];
                el[t] = in_lo[j];
            }
        }
#pragma unroll
        for (int t = 0; t < SC_POS; ++t) {
            const uint64_t j = base + threadIdx.x + (uint64_t)t * EX_THREADS;
            if (j < end) {
                sb[t] = (uint32_t)(el[t] & 0xFFFFu) & (nsub - 1);
                const uint32_t i = (uint32_t)(el[t] >> 16) & ((1u << ELEM_I_BITS) - 1);
                el[t] = (el[t] & ~0xFFFFull) | (((uint32_t)(eh[t] >> 48) - i) & 0xFFFFu);  // restore (len - i) mod 2^16
            }
        }
#pragma unroll
        for (int t = 0; t < SC_POS; ++t)
            rk[t] = agg_rank(L.cnt, sb[t], base + threadIdx.x + (uint64_t)t * EX_THREADS < end);
        __syncthreads();
        const uint32_t tot = stage_reserve(L, nsub, cur1, b0 << sub_bits);
#pragma unroll
        for (int t = 0; t < SC_POS; ++t) {
            const uint64_t j = base + threadIdx.x + (uint64_t)t * EX_THREADS;
            if (j < end) {
                const uint32_t slot = L.off[sb[t]] + rk[t];
                L.hi[slot] = eh[t];
                L.lo[slot] = el[t];
                L.dst[slot] = (uint8_t)sb[t];
            }
        }
        __syncthreads();
        for (uint32_t j = threadIdx.x; j < tot; j += blockDim.x) {
            const uint32_t d = L.dst[j];
            const uint64_t o = L.base[d] + (j - L.off[d]);
            out_hi[o] = L.hi[j];
            out_lo[o] = L.lo[j];
        }
        __syncthreads();
    }
}

// partial[rb][b] = sum of hist[w][b] over rows w of row-block rb
__global__ void k_colsum(const uint32_t* __restrict__ hist, uint32_t nwg, uint32_t NB, uint32_t* __restrict__ partial) {
    uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t rb = blockIdx.y;
    if (b >= NB) return;
    uint32_t w0 = rb * SCAN_ROWS, w1 = min(nwg, w0 + SCAN_ROWS);
    uint32_t s = 0;
    for (uint32_t w = w0; w < w1; ++w) s += hist[(uint64_t)w * NB + b];
    partial[(uint64_t)rb * NB + b] = s;
}

// One workgroup: bucket totals -> owner-relative bucket starts; rbbase[rb][b] = start of the
// row-block's first row within the bucket (owner-relative); owner_start[o] absolute.
__global__ void k_bstart(const uint32_t* __restrict__ partial, uint32_t nrb, uint32_t NB, int b1_bits,
                         uint32_t* __restrict__ rbbase, uint32_t* __restrict__ bstart, uint64_t* __restrict__ owner_start,
                         uint32_t nowners) {
    __shared__ uint32_t s_wave[34];
    __shared__ unsigned long long s_tot[64];
    const uint32_t per = (NB + blockDim.x - 1) / blockDim.x;
    const uint32_t b0 = threadIdx.x * per;
    // per-thread totals over its bucket range
    uint32_t local = 0;
    for (uint32_t b = b0; b < min(NB, b0 + per); ++b) {
        uint32_t acc = 0;
        for (uint32_t rb = 0; rb < nrb; ++rb) {
            uint32_t v = partial[(uint64_t)rb * NB + b];
            rbbase[(uint64_t)rb * NB + b] = acc;
            acc += v;
        }
        bstart[b] = acc;  // temporarily the total
        local += acc;
    }
    uint32_t total;
    uint32_t ex = wg_exclusive_scan(local, s_wave, total);
    // absolute exclusive starts
    uint32_t run = ex;
    for (uint32_t b = b0; b < min(NB, b0 + per); ++b) {
        uint32_t t = bstart[b];
        bstart[b] = run;
        run += t;
    }
    __syncthreads();
    // owner starts (absolute), then make bucket starts owner-relative
    if (threadIdx.x < nowners) {
        uint32_t ob = threadIdx.x << b1_bits;
        s_tot[threadIdx.x] = bstart[ob];
    }
    if (threadIdx.x == 0) s_tot[nowners] = total;
    __syncthreads();
    if (threadIdx.x <= nowners) owner_start[threadIdx.x] = s_tot[threadIdx.x];
    for (uint32_t b = b0; b < min(NB, b0 + per); ++b) {
        uint32_t o = b >> b1_bits;
        uint32_t rel = bstart[b] - (uint32_t)s_tot[o];
        for (uint32_t rb = 0; rb < nrb; ++rb) rbbase[(uint64_t)rb * NB + b] += rel;
    }
    __syncthreads();
    for (uint32_t b = b0; b < min(NB, b0 + per); ++b) bstart[b] -= (uint32_t)s_tot[b >> b1_bits];
    if (threadIdx.x == 0) bstart[NB] = 0;  // sentinel unused
}

// offs[w][b] = rbbase[rb][b] + sum of hist rows before w inside the row-block
__global__ void k_coloffs(const uint32_t* __restrict__ hist, const uint32_t* __restrict__ rbbase, uint32_t nwg, uint32_t NB,
                          uint32_t* __restrict__ offs) {
    uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t rb = blockIdx.y;
    if (b >= NB) return;
    uint32_t w0 = rb * SCAN_ROWS, w1 = min(nwg, w0 + SCAN_ROWS);
    uint32_t run = rbbase[(uint64_t)rb * NB + b];
    for (uint32_t w = w0; w < w1; ++w) {
        uint64_t idx = (uint64_t)w * NB + b;
        uint32_t v = hist[idx];
        offs[idx] = run;
        run += v;
    }
}

struct BucketArgs {
    uint64_t* recs_hi;         // elements of this owner, level-1 bucket-major (SoA hi / lo)
    const uint64_t* recs_lo;
    uint64_t* tmp_hi;          // level-2 partition scratch, same indexing as recs
    uint64_t* tmp_lo;
    const uint64_t* bstart;    // [nbuckets+1] bucket starts (in recs when nsrc == 1; in tmp always)
    const uint64_t* seg_start; // nsrc > 1: [nsrc][nbuckets] start of each source rank's piece in recs
    const uint32_t* seg_len;   // nsrc > 1: [nsrc][nbuckets] its length
    uint32_t nsrc;             // 1, or the world size after the all-to-all exchange
    uint32_t* sub_tab;         // [nbuckets][SUB_TAB]: number of level-2 sub-buckets, then their offsets
    unsigned long long* kept_ctr;  // kept k-mer counter (shared by k_bucket_process and k_overflow)

    uint32_t nbuckets;
    uint32_t bucket_base;      // global bucket id of bucket 0 (owner << b1_bits)
    int rem_bits;
    const uint32_t* glen;      // protein length by global sequence index (read only for lengths >= 65536
                               // and by overflow sub-buckets)
    uint8_t* flags;
    unsigned long long* ctr;   // [0] kept [1] overflow entries [2] flagged seqs [3] jobs [4] lens
    uint64_t* out_keys;
    skm_stored_kmer_data* out_data;
    Job* jobs;
    uint32_t* lens;
    OvfEntry* ovf;
    uint32_t ovf_cap;
    unsigned long long* stamps;   // optional [32] per-phase cycle sums (diagnostics)
    uint64_t* big_desc;        // [big_cap][2] groups of > 64 members handed to k_big_groups
    uint32_t big_cap;
    int prio;                  // wave issue priority of the group-by (above the concurrent chains)
    int pshift;                // KEY_BITS - pass bits (key_h43)
    int flag_check;            // 1: a signature flag is stored only when it reads 0 (option flag_check)
    const uint32_t* skip;      // k_ovf_plan's verdict for the pass (nonzero: the run is being abandoned)
    uint32_t sub_target;       // k_partition: target elements per level-2 sub-bucket (0: SUB_TARGET)
    int diag;                  // option diag (diagnostics only)
    const uint32_t* order;     // k_partition: bucket of each workgroup (k_part_order; null: blockIdx.x)
    int part_class;            // k_partition: 0 all buckets, 1 the oversized ones (order[nb] of them), 2 the rest
};

#define SKM_STAMP(i)                                                          \
    do {                                                                      \
        if (A.stamps && threadIdx.x == 0) {                                   \
            const uint64_t _t = __builtin_amdgcn_s_memtime();                 \
            atomicAdd(&A.stamps[(i)], (unsigned long long)(_t - *L.tlast));   \
            *L.tlast = _t;                                                    \
        }                                                                     \
    } while (0)

constexpr uint32_t JOB_KEPT = 0x8000u;        // jobinfo flag: the representative's group is kept
constexpr uint32_t JOB_COUNT_MASK = 0x0FFFu;  // jobinfo: best-run length (<= CAP)

struct SubLds {
    uint64_t* hi;      // [CAP] element: rem<<16|func   (kept: 1<<63 | h43<<16 | avg)
    uint64_t* lo;      // [CAP] element: s<<36|i<<16|off (kept, no job: func|mean|median|var)
    uint32_t* tab;     // [TAB] hash slot: rep<<16 | count; later jobinfo[CAP] + func|mean[CAP]
    uint16_t* slot;    // [CAP] element -> hash slot
    uint16_t* rank;    // [CAP] element -> rank within its group (insertion order)
    uint16_t* goff;    // [CAP] representative -> first slot of its group in `order`
    uint16_t* glist;   // [CAP] group -> representative
    uint16_t* order;   // [CAP] multi-occurrence elements grouped by representative
    uint16_t* big;     // [CAP/2] wave-level group list
    uint32_t* wave;    // scan scratch (>= 40 words, 16-byte aligned)
    uint32_t* nbig;
    uint64_t* tlast;   // stamp scratch
    uint32_t* ccnt;    // [8] size-class counters
    uint32_t* lens32;  // the sub-bucket's consumed record slots viewed as u32 (chain lengths)
    uint64_t lens_sel; // selector | u32 offset of lens32 in its buffer
};

__device__ __forceinline__ uint64_t kept_hi(uint64_t h43, uint32_t avg) { return (1ull << 63) | (h43 << 16) | avg; }
__device__ __forceinline__ uint64_t kept_lo(uint32_t f, uint32_t mean, uint32_t med, uint32_t var) {
    return (uint64_t)f | ((uint64_t)mean << 16) | ((uint64_t)med << 32) | ((uint64_t)var << 48);
}

// The kept arena holds the k-mer's 43-bit hash until the run's last kernel over the arena
// (k_kept_finalize) decodes every key in one streaming pass, off the group-by's emit phase.
__device__ __forceinline__ void write_kept(const BucketArgs& A, uint64_t o, uint64_t H, uint64_t L) {
    A.out_keys[o] = (H >> 16) & KEY_MASK;
    skm_stored_kmer_data d;
    d.avg_from_end = (uint16_t)(H & 0xFFFFu);
    d.function_index = (uint16_t)(L & 0xFFFFu);
    d.mean = (uint16_t)(L >> 16);
    d.median = (uint16_t)(L >> 32);
    d.var = (uint16_t)(L >> 48);
    A.out_data[o] = d;
}


// Thread-level group (c <= N members at order[a..a+c)): members sorted in registers by
// (func, ordinal); the sorted member list is written back so the best run is contiguous.

// Wave-level group (c > SMALLC).  Best function by Boyer-Moore majority: if any function has
// >= 80 % of the occurrences it is the strict majority, otherwise the group is cut anyway.
// The best-function members are compacted to order[a..a+cbest) and sorted by ordinal.
__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
    return ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m, 64) << 32) |
           (uint32_t)__shfl_xor((int)(uint32_t)v, m, 64);
}


__device__ __forceinline__ void bm_combine(uint32_t& cand, uint32_t& cc) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t oc = xs(cand, d), on = xs(cc, d);
        if (oc == cand) {
            cc += on;
        } else if (cc >= on) {
            cc -= on;
        } else {
            cand = oc;
            cc = on - cc;
        }
    }
    cand = (uint32_t)__shfl((int)cand, 0, 64);
}


// ------------------------------------------------------------------------------------------
// Groups of 2..64 members, packed 64/S to a wave in aligned segments of S lanes (S = 2..64, the
// next power of two >= c), one member per lane.  Every step is a segment-local shuffle network,
// so a wave resolves up to 32 groups at once with one code path:
//   sort by (function, ordinal) -> function runs by ballot -> best run by segmented max (ties to
//   the lowest FunctionIndex) -> fp32 cut -> u16 mean over the run -> upper-median offset by a
//   second segment sort -> chain lengths of the best run in visit (reverse ordinal) order.
// ------------------------------------------------------------------------------------------
template <int S>
__device__ __forceinline__ uint64_t seg_bitonic64(uint64_t key, uint32_t& pay, uint32_t m) {
#pragma unroll
    for (int k = 2; k <= S; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const uint64_t ok = xs64(key, j);
            const uint32_t op = xs(pay, j);
            const bool take_min = ((m & (uint32_t)j) == 0) == ((m & (uint32_t)k) == 0);
            if (take_min ? (ok < key) : (ok > key)) {
                key = ok;
                pay = op;
            }
        }
    }
    return key;
}

template <int S>
__device__ __forceinline__ uint32_t seg_bitonic32(uint32_t key, uint32_t m) {
#pragma unroll
    for (int k = 2; k <= S; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const uint32_t ok = xs(key, j);
            const bool take_min = ((m & (uint32_t)j) == 0) == ((m & (uint32_t)k) == 0);
            key = take_min ? min(key, ok) : max(key, ok);
        }
    }
    return key;
}

template <int S>
__device__ __forceinline__ uint32_t seg_reduce_max(uint32_t x) {
#pragma unroll
    for (int d = 1; d < S; d <<= 1) x = max(x, xs(x, d));
    return x;
}

template <int S>
__device__ __forceinline__ uint32_t seg_reduce_sum(uint32_t x) {
#pragma unroll
    for (int d = 1; d < S; d <<= 1) x += xs(x, d);
    return x;
}

// One wave task: groups big[q0 .. q0 + 64/S) of the class with segment size S.
template <int S>
__device__ __forceinline__ void seg_groups(const SubLds& L, uint32_t q0, uint32_t qend, uint32_t G, uint32_t M,
                                           const BucketArgs& A, uint64_t hprefix, uint32_t* jobinfo,
                                           uint32_t* fmean) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t m = lane & (uint32_t)(S - 1);
    const uint32_t sbase = lane - m;
    const uint32_t q = q0 + lane / (uint32_t)S;
    const bool gv = q < qend;
    uint32_t rep = 0, a = 0, c = 0;
    if (gv) {
        const uint32_t g = L.big[q];
        rep = L.glist[g];
        a = L.goff[rep];
        c = (g + 1 < G ? L.goff[L.glist[g + 1]] : M) - a;
    }
    const bool real = gv && m < c;
    uint64_t key = ~0ull;
    uint32_t pay = 0;
    if (real) {
        const uint32_t j = L.order[a + m];
        const uint64_t hj = L.hi[j], lj = L.lo[j];
        key = ((hj & 0xFFFFull) << 48) | (lj >> 16);  // function, then ordinal (s << 20 | i)
        pay = (uint32_t)(hj >> 47);                    // len mod 2^16 << 1 | big-length flag
    }
    key = seg_bitonic64<S>(key, pay, m);
    // function runs (padding lanes are heads of empty runs)
    const uint32_t f = (uint32_t)(key >> 48);
    const uint32_t fprev = (uint32_t)__shfl_up((int)f, 1, 64);
    const bool head = !real || m == 0 || f != fprev;
    const uint64_t H = __ballot(head);
    const uint64_t above = lane == 63 ? 0ull : (H & ~((2ull << lane) - 1ull));
    const uint32_t nh = above ? (uint32_t)__ffsll((long long)above) - 1u : 64u;
    const uint32_t rlen = min(nh, sbase + c) - lane;
    const uint32_t v = (real && head) ? ((rlen << 16) | (0xFFFFu - f)) : 0u;
    const uint32_t best = seg_reduce_max<S>(v);
    const uint32_t cbest = best >> 16, bf = 0xFFFFu - (best & 0xFFFFu);
    const bool kept = gv && !((float)cbest < float(c) * 0.8f);
    const bool inrun = real && f == bf;
    const uint32_t len16 = pay >> 1;
    const uint32_t sum = seg_reduce_sum<S>(inrun ? len16 : 0u);
    // upper median of the offsets (len - i) mod 2^16 over all members
    const uint32_t i = (uint32_t)(key & ((1u << ELEM_I_BITS) - 1));
    const uint32_t off = real ? ((len16 - i) & 0xFFFFu) : 0x10000u;
    const uint32_t osort = seg_bitonic32<S>(off, m);
    const uint32_t avg = (uint32_t)__shfl((int)osort, (int)(sbase + (c >> 1)), 64);
    // best run: lanes [rs, rs + cbest), ascending ordinal
    const uint64_t R = __ballot(inrun);
    const uint64_t segmask = (S == 64) ? ~0ull : (((1ull << S) - 1ull) << sbase);
    const uint64_t Rs = R & segmask;
    const uint32_t rs = Rs ? (uint32_t)__ffsll((long long)Rs) - 1u : sbase;
    const uint32_t s = (uint32_t)(key >> ELEM_I_BITS) & ((1u << ELEM_S_BITS) - 1u);
    const uint32_t fl = (A.flag_check && real && A.flags) ? A.flags[s] : 0u;  // diag 1: no flags
    const uint32_t len = (pay & 1u) ? A.glen[s] : len16;
    if (kept && real && fl == 0 && A.flags) mark_seq(A.flags, s);
    const uint32_t x0 = (uint32_t)__shfl((int)len, (int)(rs + cbest - 1), 64);  // first visited
    const uint32_t x1 = (uint32_t)__shfl((int)len, (int)rs, 64);                // second when cbest == 2
    if (kept && inrun && cbest >= 3) L.lens32[2 * a + (rs + cbest - 1 - lane)] = len;  // visit order
    if (kept && m == 0) {
        GRes r;
        r.kept = true;
        r.best_f = bf;
        r.cbest = cbest;
        r.avg = avg;
        r.mean = d2u16((double)(uint16_t)sum / (double)cbest);
        stats_small(r, x0, cbest == 2 ? x1 : 0u, cbest);
        const uint64_t h43 = key_h43(hprefix, (L.hi[rep] >> 16) & REM_MASK, A.rem_bits, A.pshift);
        L.hi[rep] = kept_hi(h43, r.avg);
        if (cbest >= 3) {
            jobinfo[rep] = (a << 16) | JOB_KEPT | cbest;  // chain lengths at lens32[2a..2a+cbest)
            fmean[rep] = bf | ((uint32_t)r.mean << 16);
        } else {
            jobinfo[rep] = JOB_KEPT;
            L.lo[rep] = kept_lo(bf, r.mean, r.median, r.var);
        }
    }
}

// One sub-bucket of n <= CAP records: LDS hash grouping (ranks from the insert atomics give a
// counting sort by group), singletons resolved immediately, multi-occurrence groups by threads
// (small) or waves (large); no workgroup-wide sort.
constexpr uint32_t LPER = CAP / BPK_THREADS;  // elements per thread of one batch

// the batch's elements into registers, every load in flight at once (a rolled loop would wait for
// each pair before its LDS store)
__device__ __forceinline__ void load_batch(const uint64_t* __restrict__ src_hi, const uint64_t* __restrict__ src_lo,
                                           uint32_t n, uint64_t (&eh)[LPER], uint64_t (&el)[LPER]) {
#pragma unroll
    for (uint32_t u = 0; u < LPER; ++u) {
        const uint32_t j = threadIdx.x + u * BPK_THREADS;
        if (j < n) {
            eh[u] = __builtin_nontemporal_load(src_hi + j);
            el[u] = __builtin_nontemporal_load(src_lo + j);
        }
    }
}

// One batch of n <= CAP elements.  (Measured: issuing the next batch's loads here, to overlap their
// latency with this batch's work, gained nothing -- the other workgroup of the CU already hides
// it -- and cost register spills.)
__device__ __forceinline__ void process_sub(const uint64_t* __restrict__ src_hi, const uint64_t* __restrict__ src_lo,
                                            uint32_t n, const BucketArgs& A, uint64_t hprefix, const SubLds& L) {
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    const uint32_t EMPTY = 0xFFFFFFFFu;
    // 1. the elements into LDS
    uint64_t eh[LPER], el[LPER];
    load_batch(src_hi, src_lo, n, eh, el);
    for (uint32_t t = tid; t < (uint32_t)TAB; t += nt) L.tab[t] = EMPTY;
#pragma unroll
    for (uint32_t u = 0; u < LPER; ++u) {
        const uint32_t j = tid + u * BPK_THREADS;
        if (j < n) {
            L.hi[j] = eh[u];
            L.lo[j] = el[u];
        }
    }
    if (tid == 0) *L.nbig = 0;
    if (tid < 8) L.ccnt[tid] = 0;  // the size-class counters (last read before this batch's emit)
    __syncthreads();
    SKM_STAMP(2);
    // 2. hash insert: slot = representative << 16 | count; the pre-increment count is the rank
    for (uint32_t j = tid; j < n; j += nt) {
        const uint32_t rem = (uint32_t)(L.hi[j] >> 16) & REM_MASK;
        uint32_t slot = (rem * 0x9E3779B1u) >> (32 - TAB_BITS);
        uint32_t rk = 0;
        while (true) {
            const uint32_t cur = atomicCAS(&L.tab[slot], EMPTY, (j << 16) | 1u);
            if (cur == EMPTY) break;
            if (((uint32_t)(L.hi[cur >> 16] >> 16) & REM_MASK) == rem) {
                rk = atomicAdd(&L.tab[slot], 1u) & 0xFFFFu;
                break;
            }
            slot = (slot + 1) & (TAB - 1);
        }
        L.slot[j] = (uint16_t)slot;
        L.rank[j] = (uint16_t)rk;
    }
    __syncthreads();
    SKM_STAMP(3);
    // 3. singletons resolved in place; multi-occurrence groups get a slice of `order` (each thread
    //    owns LPER consecutive elements: one workgroup scan for the whole batch)
    uint32_t M = 0, G = 0;
    {
        const uint32_t j0 = tid * LPER;
        uint32_t ev[LPER], loc = 0;
#pragma unroll
        for (uint32_t u = 0; u < LPER; ++u) {
            const uint32_t j = j0 + u;
            ev[u] = j < n ? L.tab[L.slot[j]] : 0u;
            const uint32_t cnt = ev[u] & 0xFFFFu;
            loc += (cnt > 1 && (ev[u] >> 16) == j) ? ((cnt << 13) | 1u) : 0u;
        }
        uint32_t tot;
        uint32_t v = wg_exclusive_scan1(loc, L.wave, tot);  // L.wave next written by the emit scan
        uint32_t ms[LPER];  // the singletons' sequences, flagged after the loop
#pragma unroll
        for (uint32_t u = 0; u < LPER; ++u) {
            const uint32_t j = j0 + u;
            const uint32_t cnt = ev[u] & 0xFFFFu;
            ms[u] = 0xFFFFFFFFu;
            if (j < n && cnt > 1 && (ev[u] >> 16) == j) {
                L.goff[j] = (uint16_t)(v >> 13);
                L.glist[v & 0x1FFFu] = (uint16_t)j;
                v += (cnt << 13) | 1u;
            } else if (j < n && cnt == 1) {  // group of one: always kept (1 >= 0.8), median 0, var 0
                const uint64_t H = L.hi[j], Lo = L.lo[j];
                ms[u] = (uint32_t)(Lo >> 36);
                L.hi[j] = kept_hi(key_h43(hprefix, (H >> 16) & REM_MASK, A.rem_bits, A.pshift), (uint32_t)(Lo & 0xFFFFu));
                L.lo[j] = kept_lo((uint32_t)(H & 0xFFFFu), d2u16((double)(uint16_t)(H >> 48) / 1.0), 0, 0);
                L.rank[j] = 0xFFFFu;  // singleton marker
            }
        }
        if (A.flags) mark_seqs<LPER>(A.flags, A.flag_check, ms);
        M = tot >> 13;
        G = tot & 0x1FFFu;
    }
    __syncthreads();
    SKM_STAMP(4);
    // 4. counting-sort scatter of the multi-occurrence elements, and the groups' size classes:
    //    classes 0..5 = segment size 2,4,..,64 (packed 64/S per wave), class 6 = more than 64
    //    members (one wave per group).  `big` will hold the class-ordered list.
    for (uint32_t j = tid; j < n; j += nt) {
        const uint32_t e = L.tab[L.slot[j]];
        if ((e & 0xFFFFu) > 1) L.order[L.goff[e >> 16] + L.rank[j]] = (uint16_t)j;
    }
    uint32_t* ccnt = L.ccnt;
    auto cls_of = [](uint32_t c) -> uint32_t {
        return c > 64u ? 6u : 31u - (uint32_t)__clz(c - 1u) - 0u;  // c in [2,64]: ceil(log2 c) - 1
    };
    for (uint32_t g = tid; g < G; g += nt) {
        const uint32_t a = L.goff[L.glist[g]];
        const uint32_t c = g + 1 < G ? L.goff[L.glist[g + 1]] - a : M - a;
        atomicAdd(&ccnt[cls_of(c)], 1u);  // (a per-wave ballot version measured slower)
    }
    __syncthreads();
    SKM_STAMP(5);
    // 5. the job info (over the hash table, read for the last time above), the class offsets
    uint32_t* jobinfo = L.tab;        // per representative: best-run start << 16 | KEPT | best count
    uint32_t* fmean = L.tab + CAP;    // per representative: func | mean << 16
    for (uint32_t j = tid; j < n; j += nt) jobinfo[j] = L.rank[j] == 0xFFFFu ? JOB_KEPT : 0u;
    // ccnt[0..7]: cursors, [8..15]: class starts in big[], [16..23]: first wave task of each class
    uint32_t* cstart = ccnt + 8;
    uint32_t* tstart = ccnt + 16;
    if (tid == 0) {
        uint32_t run = 0, acc = 0;
        for (int q = 0; q < 7; ++q) {
            const uint32_t t = ccnt[q];
            ccnt[q] = run;
            cstart[q] = run;
            tstart[q] = acc;
            const uint32_t per = q < 6 ? (64u >> (q + 1)) : 1u;
            acc += (t + per - 1) / per;
            run += t;
        }
        cstart[7] = run;
        tstart[7] = acc;
    }
    // groups of more than 64 members go to k_big_groups: reserve their descriptors now, the
    // atomic's latency behind the class scatter
    unsigned long long big_base = 0;
    if (tid == 0 && cstart[7] > cstart[6]) big_base = atomicAdd(&A.ctr[5], (unsigned long long)(cstart[7] - cstart[6]));
    __syncthreads();
    for (uint32_t g = tid; g < G; g += nt) {
        const uint32_t a = L.goff[L.glist[g]];
        const uint32_t c = g + 1 < G ? L.goff[L.glist[g + 1]] - a : M - a;
        L.big[atomicAdd(&ccnt[cls_of(c)], 1u)] = (uint16_t)g;
    }
    if (tid == 0) *reinterpret_cast<unsigned long long*>(L.wave + 44) = big_base;
    __syncthreads();
    SKM_STAMP(6);
    {
        // one list of wave tasks: first the hand-off of each group of more than 64 members (its
        // members (func << 48 | ordinal) into the group's own consumed slots, protein length
        // beside it, one descriptor each; k_big_groups resolves them register-resident), then the
        // packed groups -- class k packs 64 >> (k + 1) groups per task
        const uint32_t ntask = tstart[6];
        const uint32_t nbig = cstart[7] - cstart[6];
        const uint64_t bbase = *reinterpret_cast<const unsigned long long*>(L.wave + 44);
        const uint32_t wave = tid >> 6, nwaves = nt >> 6, lane = tid & 63u;
        uint64_t* slots = reinterpret_cast<uint64_t*>(L.lens32);
        uint64_t* slots_lo = const_cast<uint64_t*>(src_lo);
        // tasks taken from an LDS counter (ccnt[7], zeroed with the class counters), longest first:
        // the hand-offs, then the packed classes from 64-lane segments down to pairs
        (void)wave;
        (void)nwaves;
        for (;;) {
            uint32_t t = 0;
            if (lane == 0) t = atomicAdd(&ccnt[7], 1u);
            t = (uint32_t)__builtin_amdgcn_readfirstlane((int)t);
            if (t >= nbig + ntask) break;
            if (t < nbig) {
                const uint32_t g = L.big[cstart[6] + t];
                const uint32_t rep = L.glist[g];
                const uint32_t a = L.goff[rep];
                const uint32_t c = g + 1 < G ? L.goff[L.glist[g + 1]] - a : M - a;
                for (uint32_t u = lane; u < c; u += 64) {
                    const uint32_t j = L.order[a + u];
                    const uint64_t hj = L.hi[j], lj = L.lo[j];
                    slots[a + u] = ((hj & 0xFFFFull) << 48) | (lj >> 16);
                    slots_lo[a + u] = elem_len(hj, lj, A.glen);  // no per-member gathers downstream
                }
                const uint64_t q = bbase + t;
                if (lane == 0 && q < A.big_cap) {
                    A.big_desc[2 * q] = key_h43(hprefix, (L.hi[rep] >> 16) & REM_MASK, A.rem_bits, A.pshift) |
                                        ((uint64_t)c << KEY_BITS);
                    A.big_desc[2 * q + 1] = L.lens_sel + 2 * a;
                }
                continue;
            }
            const uint32_t ts = ntask - 1u - (t - nbig);
            uint32_t k = 0;
            while (k < 5 && ts >= tstart[k + 1]) ++k;
            const uint32_t per = 64u >> (k + 1);
            const uint32_t q0 = cstart[k] + (ts - tstart[k]) * per, qe = cstart[k + 1];
            switch (k) {
                case 0: seg_groups<2>(L, q0, qe, G, M, A, hprefix, jobinfo, fmean); break;
                case 1: seg_groups<4>(L, q0, qe, G, M, A, hprefix, jobinfo, fmean); break;
                case 2: seg_groups<8>(L, q0, qe, G, M, A, hprefix, jobinfo, fmean); break;
                case 3: seg_groups<16>(L, q0, qe, G, M, A, hprefix, jobinfo, fmean); break;
                case 4: seg_groups<32>(L, q0, qe, G, M, A, hprefix, jobinfo, fmean); break;
                default: seg_groups<64>(L, q0, qe, G, M, A, hprefix, jobinfo, fmean); break;
            }
        }
    }
    __syncthreads();
    SKM_STAMP(11);
    SKM_STAMP(7);
    // 6. emit kept k-mers and chain jobs: one scan and one reservation per batch; the kept
    //    elements are first compacted in LDS (slot[] = kept list, order[] = job list, rank[] =
    //    a job's kept position) so consecutive lanes write consecutive records
    constexpr uint32_t EMIT_PER = CAP / BPK_THREADS;
    unsigned long long* s_base = reinterpret_cast<unsigned long long*>(L.wave + 36);
    const uint32_t j0 = tid * EMIT_PER;
    uint32_t cnt = 0;
#pragma unroll
    for (uint32_t u = 0; u < EMIT_PER; ++u) {
        const uint32_t j = j0 + u;
        const uint32_t jb = j < n ? jobinfo[j] : 0u;
        cnt += ((jb & JOB_KEPT) ? 1u : 0u) | ((jb & JOB_COUNT_MASK) ? 0x10000u : 0u);
    }
    uint32_t tot;
    const uint32_t pos = wg_exclusive_scan1(cnt, L.wave, tot);  // next written by the next batch's classify
    // the two reservations from two waves at once, their latency behind the LDS compaction
    unsigned long long rsv = 0;
    if (tid == 0 && (tot & 0xFFFFu)) rsv = atomicAdd(A.kept_ctr, (unsigned long long)(tot & 0xFFFFu));
    if (tid == 64 && (tot >> 16)) rsv = atomicAdd(&A.ctr[3], (unsigned long long)(tot >> 16));
    {
        uint32_t pk = pos & 0xFFFFu, pj = pos >> 16;
#pragma unroll
        for (uint32_t u = 0; u < EMIT_PER; ++u) {
            const uint32_t jb = j0 + u < n ? jobinfo[j0 + u] : 0u;
            if (!(jb & JOB_KEPT)) continue;
            L.slot[pk] = (uint16_t)(j0 + u);
            if (jb & JOB_COUNT_MASK) {
                L.order[pj++] = (uint16_t)(j0 + u);
                L.rank[j0 + u] = (uint16_t)pk;
            }
            ++pk;
        }
    }
    if (tid == 0 || tid == 64) s_base[tid >> 6] = rsv;
    __syncthreads();
    const uint32_t nkept = tot & 0xFFFFu, njob = tot >> 16;
    if (nkept) {
        const uint64_t ob = s_base[0];
#pragma unroll 1
        for (uint32_t t = tid; t < nkept; t += nt) {
            const uint32_t j = L.slot[t];
            const uint32_t jb = jobinfo[j];
            uint64_t lo;
            if (jb & JOB_COUNT_MASK) {
                const uint32_t fm = fmean[j];
                lo = kept_lo(fm & 0xFFFFu, fm >> 16, 0, 0);
            } else {
                lo = L.lo[j];
            }
            write_kept(A, ob + t, L.hi[j], lo);
        }
        const uint64_t jbase = njob ? s_base[1] : 0;
#pragma unroll 1
        for (uint32_t t = tid; t < njob; t += nt) {
            const uint32_t j = L.order[t];
            const uint32_t jb = jobinfo[j];
            Job jbr;
            jbr.lens_off = L.lens_sel + 2 * (jb >> 16);
            jbr.n = jb & JOB_COUNT_MASK;
            jbr.out_idx = (uint32_t)(ob + L.rank[j]);
            A.jobs[jbase + t] = jbr;
        }
    }
    __syncthreads();
    SKM_STAMP(8);
}

__global__ __launch_bounds__(BPK_THREADS, BPK_WAVES_EU) void k_bucket_process(BucketArgs A) {
    static_assert(CAP % BPK_THREADS == 0, "emit assigns CAP / BPK_THREADS elements per thread");
    __shared__ uint64_t s_hi[CAP];
    __shared__ uint64_t s_lo[CAP];
    __shared__ uint32_t s_tab[TAB];
    __shared__ uint32_t s_sub[(1 << MAX_B2) + 1];
    __align__(16) __shared__ uint16_t s_slot[CAP];
    __align__(16) __shared__ uint16_t s_rank[CAP];
    __align__(16) __shared__ uint16_t s_goff[CAP];
    __align__(16) __shared__ uint16_t s_glist[CAP];
    __align__(16) __shared__ uint16_t s_order[CAP];
    __align__(16) __shared__ uint16_t s_big[CAP / 2];
    __shared__ __align__(16) uint32_t s_wave[48];
    __shared__ uint32_t s_nbig;
    __shared__ uint64_t s_tlast;
    __shared__ uint32_t s_ccnt[24];
    if (A.skip && *A.skip) return;
    SubLds L;
    L.ccnt = s_ccnt;
    L.tlast = &s_tlast;
    if (threadIdx.x == 0) s_tlast = __builtin_amdgcn_s_memtime();
    L.hi = s_hi;
    L.lo = s_lo;
    L.tab = s_tab;
    L.slot = s_slot;
    L.rank = s_rank;
    L.goff = s_goff;
    L.glist = s_glist;
    L.order = s_order;
    L.big = s_big;
    L.wave = s_wave;
    L.nbig = &s_nbig;

    const uint32_t bucket = blockIdx.x;
    if (bucket >= A.nbuckets) return;
    const uint64_t r0 = A.bstart[bucket], r1 = A.bstart[bucket + 1];
    const uint64_t n = r1 - r0;
    if (n == 0) return;
    const uint64_t hprefix = (uint64_t)(A.bucket_base + bucket) << A.rem_bits;
    if (A.prio == 1) __builtin_amdgcn_s_setprio(1);
    if (A.prio == 2) __builtin_amdgcn_s_setprio(2);
    if (A.prio >= 3) __builtin_amdgcn_s_setprio(3);

    // a bucket that fits LDS is one batch straight from recs; otherwise the sub-buckets of the
    // partition pass (k_partition) in tmp: consecutive sub-buckets are contiguous and hold
    // disjoint keys, so as many as fit in LDS form one batch (the per-pass fixed costs -- load
    // latency, barriers, reservations -- are paid once per ~CAP elements).  One call site of
    // process_sub keeps the kernel's code footprint small.
    const bool direct = n <= (uint64_t)CAP && A.nsrc == 1;
    uint32_t nsub = 1;
    if (!direct) {
        const uint32_t* tab = A.sub_tab + (uint64_t)bucket * SUB_TAB;
        nsub = tab[0];
        for (uint32_t d = threadIdx.x; d <= nsub; d += blockDim.x) s_sub[d] = tab[1 + d];
        __syncthreads();
        SKM_STAMP(9);
    }
    // batches: the whole bucket (fits LDS), or runs of consecutive sub-buckets of <= CAP elements
    // in total (sub-buckets beyond CAP are k_overflow's)
    struct Batch {
        uint32_t a, cnt;  // first element (bucket-relative), elements; cnt == 0: none left
    };
    auto next_batch = [&](uint32_t& d) -> Batch {
        if (direct) {
            if (d >= 1) return Batch{0, 0};
            d = 1;
            return Batch{0, (uint32_t)n};
        }
        while (d < nsub) {
            const uint32_t a = s_sub[d];
            if (s_sub[d + 1] - a == 0 || s_sub[d + 1] - a > (uint32_t)CAP) {  // empty, or k_overflow's
                ++d;
                continue;
            }
            uint32_t d2 = d + 1;
            while (d2 < nsub && s_sub[d2 + 1] - a <= (uint32_t)CAP) ++d2;
            d = d2;
            return Batch{a, s_sub[d2] - a};
        }
        return Batch{0, 0};
    };
    const uint64_t* base_hi = direct ? A.recs_hi + r0 : A.tmp_hi + r0;
    const uint64_t* base_lo = direct ? A.recs_lo + r0 : A.tmp_lo + r0;
    const uint64_t sel = direct ? LENS_IN_RECS : LENS_IN_TMP;
    uint32_t d = 0;
    for (Batch cur = next_batch(d); cur.cnt; cur = next_batch(d)) {
        L.lens_sel = (sel << LENS_SEL_SHIFT) | (2 * (r0 + cur.a));
        L.lens32 = reinterpret_cast<uint32_t*>(const_cast<uint64_t*>(base_hi + cur.a));
        process_sub(base_hi + cur.a, base_lo + cur.a, cur.cnt, A, hprefix, L);
        __syncthreads();
        SKM_STAMP(10);
    }
}

// ------------------------------------------------------------------------------------------
// Groups of 65..CAP members (k_bucket_process hands them over as descriptors): one wave per group,
// no workgroup barriers, every member register-resident (E = 2..32 per lane).  Counting is done
// on ballots (v_cmp + s_bcnt1, no cross-lane latency): the best-function count and the
// upper-median offset by a 16-step radix select.  The best-function members are sorted by
// ordinal with a bitonic network over 64 E keys (compare-exchanges within a lane below distance
// E, DPP / swizzle / permlane exchanges above) and their lengths written in visit order into
// the group's own slots (the chain job's input).
// ------------------------------------------------------------------------------------------
struct BigOut {              // one per descriptor; n == 0: group cut
    uint64_t h43;            // hashed key
    uint64_t lens_off;       // chain input (selector | u32 offset)
    uint32_t n;              // best-function members (chain length)
    uint16_t avg, func, mean, pad0;
    uint32_t pad1;
};
static_assert(sizeof(BigOut) == 32, "BigOut layout");

struct BigArgs {
    const uint64_t* desc;
    const unsigned long long* ndesc;   // device counter (k_bucket_process)
    uint32_t cap;
    const uint64_t* recs_hi;
    const uint64_t* tmp_hi;
    const uint64_t* recs_lo;   // lo slots: the members' protein lengths
    const uint64_t* tmp_lo;
    uint8_t* flags;
    BigOut* out;
};

template <int E>
__device__ __forceinline__ uint32_t ballot_count(const bool (&p)[E]) {
    uint32_t n = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) n += (uint32_t)__popcll(__ballot(p[e]));
    return n;
}

template <int E, int D>
__device__ __forceinline__ void bitonic_cross(uint64_t (&ky)[E], bool take_min) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint64_t o = xshfl64<D>(ky[e]);
        ky[e] = take_min ? (o < ky[e] ? o : ky[e]) : (o > ky[e] ? o : ky[e]);
    }
}

template <int E>
__device__ __forceinline__ void big_group(const BigArgs& B, uint64_t g, uint64_t* mem, const uint64_t* mlen,
                                          uint32_t c, uint64_t h43, uint64_t lens_off) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t fo[E];  // func << 16 | offset (padding: 0xFFFFFFFF)
    uint64_t ky[E];  // ordinal (s << 20 | i) << 16 | member index
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t t = lane * E + (uint32_t)e;
        fo[e] = 0xFFFFFFFFu;
        ky[e] = ~0ull;
        if (t < c) {
            const uint64_t v = mem[t];
            const uint32_t len = (uint32_t)mlen[t];
            const uint32_t i = (uint32_t)v & ((1u << ELEM_I_BITS) - 1u);
            fo[e] = ((uint32_t)(v >> 48) << 16) | ((len - i) & 0xFFFFu);
            ky[e] = (v << 16) | t;
        }
    }
    // majority candidate (a function with >= 80 % of the members is the strict majority)
    uint32_t cand = 0xFFFFFFFFu, cc = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        if (fo[e] != 0xFFFFFFFFu) {
            const uint32_t f = fo[e] >> 16;
            if (cc == 0) {
                cand = f;
                cc = 1;
            } else if (f == cand) {
                ++cc;
            } else {
                --cc;
            }
        }
    }
    bm_combine(cand, cc);
    bool p[E];
#pragma unroll
    for (int e = 0; e < E; ++e) p[e] = (fo[e] >> 16) == cand;  // padding has func 0xFFFF != cand
    const uint32_t nb = ballot_count<E>(p);
    BigOut o;
    o.h43 = h43;
    o.lens_off = lens_off;
    o.n = 0;
    o.avg = o.func = o.mean = 0;
    o.pad0 = 0;
    o.pad1 = 0;
    if ((float)nb < float(c) * 0.8f) {
        if (lane == 0) B.out[g] = o;
        return;
    }
    // the members' flags, up to 8 reads in flight per lane before their atomics (one mark after
    // another waited a global round trip each: E of them per lane)
    if (B.flags) {
        constexpr int MC = E < 8 ? E : 8;
#pragma unroll
        for (int e0 = 0; e0 < E; e0 += MC) {
            uint32_t ms[MC];
#pragma unroll
            for (int u = 0; u < MC; ++u)
                ms[u] = fo[e0 + u] != 0xFFFFFFFFu ? (uint32_t)(ky[e0 + u] >> (16 + ELEM_I_BITS)) : 0xFFFFFFFFu;
            mark_seqs<MC>(B.flags, 0, ms);
        }
    }
    uint32_t sum = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        if (fo[e] != 0xFFFFFFFFu && p[e]) sum += (uint32_t)mlen[ky[e] & 0xFFFFu];  // L2-warm (read above)
        if (!p[e]) ky[e] = ~0ull;  // sort key: best-function members only
    }
    sum = wave_sum(sum);
    // upper median offset: the (c/2)-th smallest (0-based) by radix select, bit 15 down to 0
    uint32_t k = c / 2, pre = 0;
#pragma unroll 1
    for (int b = 15; b >= 0; --b) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const uint32_t v = fo[e] == 0xFFFFFFFFu ? 0x10000u : (fo[e] & 0xFFFFu);
            p[e] = ((v >> b) ^ (pre >> b)) == 0u;  // bits above b match the prefix, bit b clear
        }
        const uint32_t n0 = ballot_count<E>(p);
        if (k >= n0) {
            k -= n0;
            pre |= 1u << b;
        }
    }
    // ascending bitonic sort of the 64 E keys (blocked: lane holds keys lane*E .. lane*E+E-1)
#pragma unroll 1
    for (uint32_t kk = 2; kk <= 64u * E; kk <<= 1) {
        const bool asc_lane = ((lane * (uint32_t)E) & kk) == 0;  // valid when kk >= 2E
#pragma unroll 1
        for (uint32_t jj = kk >> 1; jj >= (uint32_t)E; jj >>= 1) {
            const uint32_t d = jj / (uint32_t)E;
            const bool take_min = ((lane & d) == 0) == asc_lane;
            switch (d) {  // wave-uniform
                case 1: bitonic_cross<E, 1>(ky, take_min); break;
                case 2: bitonic_cross<E, 2>(ky, take_min); break;
                case 4: bitonic_cross<E, 4>(ky, take_min); break;
                case 8: bitonic_cross<E, 8>(ky, take_min); break;
                case 16: bitonic_cross<E, 16>(ky, take_min); break;
                default: bitonic_cross<E, 32>(ky, take_min); break;
            }
        }
#pragma unroll
        for (int jj = E / 2; jj > 0; jj >>= 1) {
            if ((uint32_t)jj < kk) {
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const int l = e ^ jj;
                    if (l > e) {
                        const bool asc = (((lane * (uint32_t)E) + (uint32_t)e) & kk) == 0;
                        const uint64_t x = ky[e], y = ky[l];
                        const bool sw = asc ? (y < x) : (x < y);
                        ky[e] = sw ? y : x;
                        ky[l] = sw ? x : y;
                    }
                }
            }
        }
    }
    // chain input: best-function lengths in visit (reverse ordinal) order, over the group's own
    // slots (every member is in registers by now)
    uint32_t* lens = reinterpret_cast<uint32_t*>(mem);
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t t = lane * E + (uint32_t)e;
        if (t < nb) lens[nb - 1 - t] = (uint32_t)mlen[ky[e] & 0xFFFFu];
    }
    o.n = nb;
    o.avg = (uint16_t)pre;
    o.func = (uint16_t)cand;
    o.mean = d2u16((double)(uint16_t)sum / (double)nb);
    if (lane == 0) B.out[g] = o;
}

constexpr int BIG_WG = 256;

// LARGE = false: groups of 65..1024 members (E <= 16, 128 VGPRs, 2 waves per SIMD);
// LARGE = true: 1025..CAP (E = 32), a separate launch so the common case keeps its occupancy.
template <bool LARGE>
__global__ __launch_bounds__(BIG_WG, LARGE ? 3 : 4) void k_big_groups(BigArgs B) {
    const uint64_t nd = min((uint64_t)*B.ndesc, (uint64_t)B.cap);
    const uint64_t nw = (uint64_t)gridDim.x * (BIG_WG / 64);
    for (uint64_t g = (uint64_t)blockIdx.x * (BIG_WG / 64) + (threadIdx.x >> 6); g < nd; g += nw) {
        const uint64_t d0 = B.desc[2 * g], d1 = B.desc[2 * g + 1];
        const uint32_t c = (uint32_t)(d0 >> KEY_BITS);
        if (LARGE != (c > 1024u)) continue;
        const uint64_t h43 = d0 & KEY_MASK;
        const uint64_t sel = d1 >> LENS_SEL_SHIFT, off = d1 & LENS_OFF_MASK;
        uint64_t* mem = const_cast<uint64_t*>(sel == LENS_IN_RECS ? B.recs_hi : B.tmp_hi) + off / 2;
        const uint64_t* mlen = (sel == LENS_IN_RECS ? B.recs_lo : B.tmp_lo) + off / 2;
        if constexpr (LARGE) {
            big_group<32>(B, g, mem, mlen, c, h43, d1);
        } else {
            if (c <= 128u) big_group<2>(B, g, mem, mlen, c, h43, d1);
            else if (c <= 256u) big_group<4>(B, g, mem, mlen, c, h43, d1);
            else if (c <= 512u) big_group<8>(B, g, mem, mlen, c, h43, d1);
            else big_group<16>(B, g, mem, mlen, c, h43, d1);
        }
    }
}

// Kept big groups appended to the kept k-mers and chain jobs: one reservation per round of
// BIG_WG descriptors per workgroup.
__global__ __launch_bounds__(BIG_WG) void k_big_append(const BigOut* __restrict__ out, BigArgs B, BucketArgs A) {
    __shared__ __align__(16) uint32_t s_wave[48];
    __shared__ unsigned long long s_base[2];
    const uint64_t nd = min((uint64_t)*B.ndesc, (uint64_t)B.cap);
    const uint64_t per = (nd + gridDim.x - 1) / gridDim.x;
    const uint64_t g0 = (uint64_t)blockIdx.x * per, g1 = min(nd, g0 + per);
    for (uint64_t r = g0; r < g1; r += BIG_WG) {
        const uint64_t g = r + threadIdx.x;
        const bool kept = g < g1 && out[g].n != 0;
        uint32_t tot;
        const uint32_t pos = wg_exclusive_scan(kept ? 1u : 0u, s_wave, tot);
        if (tot == 0) continue;
        if (threadIdx.x == 0) {
            s_base[0] = atomicAdd(A.kept_ctr, (unsigned long long)tot);
            s_base[1] = atomicAdd(&A.ctr[3], (unsigned long long)tot);
            atomicAdd(&A.ctr[6], (unsigned long long)tot);  // kept big groups (diagnostics)
        }
        __syncthreads();
        if (kept) {
            const BigOut o = out[g];
            const uint64_t w = s_base[0] + pos;
            write_kept(A, w, kept_hi(o.h43, o.avg), kept_lo(o.func, o.mean, 0, 0));
            Job jb;
            jb.lens_off = o.lens_off;
            jb.n = o.n;
            jb.out_idx = (uint32_t)w;
            A.jobs[s_base[1] + pos] = jb;
        }
        __syncthreads();
    }
}

// Level-2 partition of every level-1 bucket that does not fit LDS (or arrives in pieces from
// several ranks): count by the next b2 bits of rem, exclusive scan, scatter into tmp.  Writes the
// sub-bucket table for k_bucket_process and queues sub-buckets larger than CAP for k_overflow,
// so the overflow path (and its long P^2 chains) can run concurrently with the group-by.
// PT_ROUND elements staged per round of the level-2 scatter.  LDS ~52 KB at 2048: three
// workgroups per CU (the sub-bucket of a staged element is recomputed from its key instead of
// staged, and the running write offsets double as the sub-bucket table); 4096 (option
// partition_round = 1, 2): one per CU, but each round's run per sub-bucket is twice as long, so
// fewer 128-byte lines leave L2 partly written.
// k_partition's workgroup order: the buckets of more than twice the mean size first, then the rest,
// each class in bucket order.  One workgroup walks a whole bucket, and a routed heavy k-mer makes
// its bucket several times the mean (C3: ~1 M occurrences beside a mean of ~230 K): started late in
// bucket order, those workgroups were the kernel's tail in the passes holding heavy keys.
__global__ __launch_bounds__(1024) void k_part_order(const uint64_t* __restrict__ bstart, uint32_t nb,
                                                     uint32_t* __restrict__ order) {
    __shared__ uint32_t s_wave[48];
    const uint64_t total = bstart[nb] - bstart[0];
    const uint64_t thr = 2 * (total / max(nb, 1u));
    const uint32_t per = (nb + blockDim.x - 1) / blockDim.x;
    const uint32_t b0 = min(nb, threadIdx.x * per), b1 = min(nb, b0 + per);
    uint32_t loc = 0;
    for (uint32_t b = b0; b < b1; ++b) loc += bstart[b + 1] - bstart[b] > thr ? 1u : 0u;
    uint32_t nbig;
    uint32_t pos = wg_exclusive_scan(loc, s_wave, nbig);
    uint32_t sp = b0 - pos;  // the small buckets before b0
    for (uint32_t b = b0; b < b1; ++b) {
        if (bstart[b + 1] - bstart[b] > thr)
            order[pos++] = b;
        else
            order[nbig + sp++] = b;
    }
    if (threadIdx.x == 0) order[nb] = nbig;  // the oversized buckets: order[0, nbig)
}

template <uint32_t PT_ROUND, uint32_t PT_THREADS, int MINB>
__global__ __launch_bounds__(PT_THREADS, MINB) void k_partition(BucketArgs A) {
    __shared__ uint32_t s_cur[(1 << MAX_B2) + 1];   // counts, then running write offsets
    __shared__ uint32_t s_rc[1 << MAX_B2];          // this round's count per sub-bucket
    __shared__ uint16_t s_ro[(1 << MAX_B2) + 1];    // ... and its staging offset (<= PT_ROUND)
    __shared__ uint64_t s_sh[PT_ROUND];
    __shared__ uint64_t s_sl[PT_ROUND];
    __shared__ __align__(16) uint32_t s_wave[48];
    if (blockIdx.x >= A.nbuckets) return;
    // part_class 1: the oversized buckets only (order[0, nbig)), 2: the others (order[nbig, nb))
    uint32_t slot = blockIdx.x;
    if (A.part_class) {
        const uint32_t nbig = A.order[A.nbuckets];
        if (A.part_class == 1 && slot >= nbig) return;
        if (A.part_class == 2) {
            slot += nbig;
            if (slot >= A.nbuckets) return;
        }
    }
    const uint32_t bucket = A.order ? A.order[slot] : slot;
    const uint64_t r0 = A.bstart[bucket], r1 = A.bstart[bucket + 1];
    const uint64_t n = r1 - r0;
    uint32_t* tab = A.sub_tab + (uint64_t)bucket * SUB_TAB;
    if (n == 0 || (n <= (uint64_t)CAP && A.nsrc == 1)) {  // processed in place by k_bucket_process
        if (threadIdx.x == 0) tab[0] = 0;
        return;
    }
    const uint64_t rem_mask = (1ull << A.rem_bits) - 1;
    int b2 = 0;
    const uint64_t target = A.sub_target ? A.sub_target : (uint32_t)SUB_TARGET;
    while (b2 < MAX_B2 && (n >> b2) > target) ++b2;
    const uint32_t nsub = 1u << b2;
    const int shift = A.rem_bits - b2;
    for (uint32_t d = threadIdx.x; d <= nsub; d += blockDim.x) s_cur[d] = 0;
    __syncthreads();
    // the bucket's elements: one contiguous range, or one piece per source rank after the exchange
    const uint32_t nseg = A.nsrc;
    auto seg = [&](uint32_t p, uint64_t& base, uint64_t& len) {
        if (nseg == 1) {
            base = r0;
            len = n;
        } else {
            base = A.seg_start[(uint64_t)p * A.nbuckets + bucket];
            len = A.seg_len[(uint64_t)p * A.nbuckets + bucket];
        }
    };
    for (uint32_t p = 0; p < nseg; ++p) {
        uint64_t base, len;
        seg(p, base, len);
        for (uint64_t j0 = 0; j0 < len; j0 += blockDim.x) {  // wave-uniform trip count (agg_count)
            const uint64_t j = j0 + threadIdx.x;
            const bool v = j < len;
            const uint64_t h = v ? A.recs_hi[base + j] : 0ull;
            agg_count(s_cur, (uint32_t)(((h >> 16) & rem_mask) >> shift), v);
        }
    }
    __syncthreads();
    {
        const uint32_t per = (nsub + blockDim.x - 1) / blockDim.x;
        const uint32_t d0 = threadIdx.x * per;
        uint32_t local = 0;
        for (uint32_t d = d0; d < min(nsub, d0 + per); ++d) local += s_cur[d];
        uint32_t tot;
        uint32_t run = wg_exclusive_scan(local, s_wave, tot);
        for (uint32_t d = d0; d < min(nsub, d0 + per); ++d) {
            const uint32_t t = s_cur[d];
            s_cur[d] = run;
            run += t;
        }
        __syncthreads();
        if (threadIdx.x == 0) s_cur[nsub] = tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) tab[0] = nsub;
    for (uint32_t d = threadIdx.x; d <= nsub; d += blockDim.x) tab[1 + d] = s_cur[d];
    __syncthreads();
    // staged scatter: each round sorts PT_ROUND elements by sub-bucket in LDS, then writes each
    // sub-bucket's run contiguously (whole lines instead of scattered 8-byte stores)
    // the next round's elements are loaded into registers before this round's LDS work, so the
    // HBM latency overlaps the staging instead of opening every round
    // (the register prefetch only in the 2048 form: the 4096 form would spill)
    constexpr uint32_t PER = PT_ROUND / PT_THREADS;
    constexpr bool PF = PER <= 4;
    constexpr uint32_t NPF = PF ? PER : 1;
    for (uint32_t p = 0; p < nseg; ++p) {
        uint64_t base, len;
        seg(p, base, len);
        uint64_t nh[NPF], nl[NPF];
        if constexpr (PF) {
#pragma unroll
            for (uint32_t u = 0; u < PER; ++u) {
                const uint64_t j = threadIdx.x + (uint64_t)u * PT_THREADS;
                if (j < len) {
                    nh[u] = A.recs_hi[base + j];
                    nl[u] = A.recs_lo[base + j];
                }
            }
        }
        for (uint64_t rb = 0; rb < len; rb += PT_ROUND) {
            for (uint32_t d = threadIdx.x; d < nsub; d += blockDim.x) s_rc[d] = 0;
            uint64_t eh[PER], el[PER];
            uint32_t sb[PER], rk[PER];
#pragma unroll
            for (uint32_t u = 0; u < PER; ++u) {
                sb[u] = 0xFFFFFFFFu;
                if constexpr (PF) {
                    eh[u] = nh[u];
                    el[u] = nl[u];
                    const uint64_t j = rb + PT_ROUND + threadIdx.x + (uint64_t)u * PT_THREADS;
                    if (j < len) {
                        nh[u] = A.recs_hi[base + j];
                        nl[u] = A.recs_lo[base + j];
                    }
                } else {
                    const uint64_t j = rb + threadIdx.x + (uint64_t)u * PT_THREADS;
                    if (j < len) {
                        eh[u] = A.recs_hi[base + j];
                        el[u] = A.recs_lo[base + j];
                    }
                }
            }
            __syncthreads();
#pragma unroll
            for (uint32_t u = 0; u < PER; ++u) {
                const uint64_t j = rb + threadIdx.x + (uint64_t)u * PT_THREADS;
                const bool v = j < len;
                if (v) sb[u] = (uint32_t)(((eh[u] >> 16) & rem_mask) >> shift);
                rk[u] = agg_rank(s_rc, v ? sb[u] : 0u, v);
            }
            __syncthreads();
            {   // exclusive scan of the round counts over the sub-buckets
                const uint32_t per = (nsub + blockDim.x - 1) / blockDim.x;
                const uint32_t d0 = threadIdx.x * per;
                uint32_t local = 0;
                for (uint32_t d = d0; d < min(nsub, d0 + per); ++d) local += s_rc[d];
                uint32_t tot;
                uint32_t run = wg_exclusive_scan(local, s_wave, tot);
                for (uint32_t d = d0; d < min(nsub, d0 + per); ++d) {
                    s_ro[d] = (uint16_t)run;
                    run += s_rc[d];
                }
                if (threadIdx.x == 0) s_ro[nsub] = (uint16_t)tot;
                __syncthreads();
            }
#pragma unroll
            for (uint32_t u = 0; u < PER; ++u)
                if (sb[u] != 0xFFFFFFFFu) {
                    const uint32_t slot = s_ro[sb[u]] + rk[u];
                    s_sh[slot] = eh[u];
                    s_sl[slot] = el[u];
                }
            __syncthreads();
            const uint32_t tot = s_ro[nsub];
            for (uint32_t k = threadIdx.x; k < tot; k += blockDim.x) {
                const uint64_t h = s_sh[k];
                const uint32_t d = (uint32_t)(((h >> 16) & rem_mask) >> shift);
                const uint64_t o = r0 + s_cur[d] + (k - s_ro[d]);
                A.tmp_hi[o] = h;
                A.tmp_lo[o] = s_sl[k];
            }
            __syncthreads();
            for (uint32_t d = threadIdx.x; d < nsub; d += blockDim.x) s_cur[d] += s_rc[d];
            __syncthreads();
        }
    }
    // s_cur[d] now ends sub-bucket d, i.e. starts d + 1
    for (uint32_t d = threadIdx.x; d < nsub; d += blockDim.x) {
        const uint32_t beg = d ? s_cur[d - 1] : 0u;
        const uint32_t cnt = s_cur[d] - beg;
        if (cnt > (uint32_t)CAP) {
            const unsigned int en = atomicAdd(reinterpret_cast<unsigned int*>(&A.ctr[1]), 1u);
            if (en < A.ovf_cap) {
                OvfEntry o;
                o.off = r0 + beg;
                o.n = cnt;
                o.bucket = bucket;
                o.scratch = 0;
                o.npad = 0;
                o.src = 1;
                A.ovf[en] = o;
            }
        }
    }
}

struct OvfScratch {
    uint64_t* hi;       // sorted elements
    uint64_t* lo;
    uint32_t* heads;    // group heads
    uint64_t* jobinfo;  // per head: best-run start << 32 | best count
    uint32_t* fmean;    // per head: func | mean << 16
};

// Overflow sub-buckets (n > CAP): global-memory bitonic sort (LDS for strides < CAP), then the
// same group processing on the global arrays.
// Chains of at least inline_min samples (the heaviest k-mers, the longest serial work of the whole
// build) run inside k_overflow as soon as their sub-bucket is grouped -- the host orders the
// overflow sub-buckets largest first -- instead of waiting for the whole overflow pass.
constexpr uint32_t OVF_INLINE_CAP = 32;   // inline chains per workgroup (more: ordinary jobs)
constexpr uint32_t OVF_BLOCK_GROUP = 1024;  // groups above this size: workgroup-cooperative statistics

__global__ __launch_bounds__(BP_THREADS) void k_overflow(BucketArgs A, OvfScratch S, uint32_t* plan, int lo_slot,
                                                          int hi_slot, int q_slot, uint32_t inline_min, int prio) {
    __shared__ uint64_t s_hi[CAP];
    __shared__ uint64_t s_lo[CAP];
    __shared__ __align__(16) uint32_t s_wave[48];
    __shared__ uint32_t s_nbig;
    __shared__ uint32_t s_big[BP_THREADS];
    __shared__ uint32_t s_ninl;
    __shared__ uint64_t s_inl[OVF_INLINE_CAP][2];  // lens offset, n << 32 | output index
    __shared__ uint32_t s_q;
    // entries [plan[lo_slot] (0 when < 0), plan[hi_slot]) of k_ovf_plan's list, taken one at a time
    // from the queue counter plan[q_slot] (largest first: the list is sorted by size class)
    const uint32_t q_lo = lo_slot < 0 ? 0u : plan[lo_slot], q_hi = plan[hi_slot];
    auto entry = [&](const OvfEntry e) {
        if (e.n == 0) return;  // every key of the sub-bucket went to k_heavy
        if ((A.diag & 32) && e.n <= (uint32_t)CAP) return;  // diagnostics: the entries of one LDS chunk
        if ((A.diag & 64) && e.n > (uint32_t)CAP) return;   //   / of the global network, skipped
        // src 2: the light remainder k_ovf_split compacted into this entry's own scratch (sorted in
        // place: each chunk is loaded whole before it is written back)
        const uint64_t* src_hi = (e.src == 2 ? S.hi : e.src ? A.tmp_hi : A.recs_hi) + e.off;
        const uint64_t* src_lo = (e.src == 2 ? S.lo : e.src ? A.tmp_lo : A.recs_lo) + e.off;
        uint64_t* ghi = S.hi + e.scratch;
        uint64_t* glo = S.lo + e.scratch;
        uint32_t* heads = S.heads + e.scratch;
        uint64_t* jobinfo = S.jobinfo + e.scratch;
        uint32_t* fmean = S.fmean + e.scratch;
        const uint32_t n = e.n;
        uint32_t N = CAP;  // the network size: pow2 >= n, at least one chunk (<= the entry's scratch)
        while (N < n) N <<= 1;
        const uint32_t tid = threadIdx.x, nt = blockDim.x;
        const uint64_t hprefix = (uint64_t)(A.bucket_base + e.bucket) << A.rem_bits;
        // phase 0: chunks of CAP sorted ascending in LDS.  The padding beyond n holds the maximum
        // key and the network is ascending-only, so no element ever moves into a chunk made only of
        // padding: those chunks are written once and skipped by every later step
        const uint32_t nch = (n + CAP - 1) / CAP * CAP;  // first all-padding chunk
        for (uint32_t c0 = nch; c0 < N; c0 += CAP)
            for (uint32_t j = tid; j < CAP; j += nt) {
                ghi[c0 + j] = ~0ull;
                glo[c0 + j] = ~0ull;
            }
        for (uint32_t c0 = 0; c0 < nch; c0 += CAP) {
            for (uint32_t j = tid; j < CAP; j += nt) {
                const uint32_t g = c0 + j;
                if (g < n) {
                    s_hi[j] = src_hi[g] & 0x00007FFFFFFFFFFFull;  // group key = rem | func (length bits dropped)
                    s_lo[j] = src_lo[g];
                } else {
                    s_hi[j] = ~0ull;
                    s_lo[j] = ~0ull;
                }
            }
            __syncthreads();
            bitonic_lds(s_hi, s_lo, CAP, 2, CAP, CAP);
            for (uint32_t j = tid; j < CAP; j += nt) {
                ghi[c0 + j] = s_hi[j];
                glo[c0 + j] = s_lo[j];
            }
            __threadfence_block();
            __syncthreads();
        }
        for (uint32_t k = 2 * CAP; k <= N; k <<= 1) {
            for (uint32_t j = k >> 1; j >= (uint32_t)CAP; j >>= 1) {
                for (uint32_t t = tid; t < N / 2; t += nt) {
                    const uint32_t i = 2 * t - (t & (j - 1));
                    if (i >= nch) continue;  // i and its partner above it are both maximum-key padding
                    const uint32_t l = j == (k >> 1) ? (i ^ (k - 1)) : i + j;
                    const uint64_t ah = ghi[i], al = glo[i], bh = ghi[l], bl = glo[l];
                    if (elem_less(bh, bl, ah, al)) {
                        ghi[i] = bh;
                        glo[i] = bl;
                        ghi[l] = ah;
                        glo[l] = al;
                    }
                }
                __threadfence_block();
                __syncthreads();
            }
            for (uint32_t c0 = 0; c0 < nch; c0 += CAP) {  // chunks above nch stay all padding
                for (uint32_t j = tid; j < CAP; j += nt) {
                    s_hi[j] = ghi[c0 + j];
                    s_lo[j] = glo[c0 + j];
                }
                __syncthreads();
                bitonic_lds(s_hi, s_lo, CAP, k, k, CAP >> 1);
                for (uint32_t j = tid; j < CAP; j += nt) {
                    ghi[c0 + j] = s_hi[j];
                    glo[c0 + j] = s_lo[j];
                }
                __threadfence_block();
                __syncthreads();
            }
        }
        // group heads
        uint32_t G = 0;
        for (uint32_t c0 = 0; c0 < n; c0 += nt) {
            const uint32_t t = c0 + tid;
            const bool head = t < n && (t == 0 || (ghi[t] >> 16) != (ghi[t - 1] >> 16));
            uint32_t tot;
            const uint32_t pos = wg_exclusive_scan(head ? 1u : 0u, s_wave, tot);
            if (head) {
                heads[G + pos] = t;
                jobinfo[t] = 0;
            }
            G += tot;
        }
        __threadfence_block();
        __syncthreads();
        const GlbView V{ghi, glo};
        auto stage = [&](const GRes& r, uint32_t a) {
            if (!r.kept) return;
            const uint64_t h43 = key_h43(hprefix, ghi[a] >> 16, A.rem_bits, A.pshift);
            if (r.cbest >= 3) {
                jobinfo[a] = ((uint64_t)(a + r.rb) << 32) | r.cbest;
                fmean[a] = r.best_f | ((uint32_t)r.mean << 16);
            } else {
                glo[a] = kept_lo(r.best_f, r.mean, r.median, r.var);
            }
            ghi[a] = kept_hi(h43, r.avg);
        };
        for (uint32_t g0 = 0; g0 < G; g0 += nt) {
            if (tid == 0) s_nbig = 0;
            __syncthreads();
            const uint32_t g = g0 + tid;
            if (g < G) {
                const uint32_t a = heads[g];
                const uint32_t b = g + 1 < G ? heads[g + 1] : n;
                const uint32_t c = b - a;
                if (c > (uint32_t)SMALLC) {
                    s_big[atomicAdd(&s_nbig, 1u)] = g;
                } else {
                    GRes r;
                    if (c <= 4)
                        r = group_thread<4>(V, a, c, A.glen, A.flags);
                    else if (c <= 8)
                        r = group_thread<8>(V, a, c, A.glen, A.flags);
                    else
                        r = group_thread<16>(V, a, c, A.glen, A.flags);
                    stage(r, a);
                }
            }
            __syncthreads();
            const uint32_t nbig = s_nbig;
            for (uint32_t bi = tid >> 6; bi < nbig; bi += nt >> 6) {
                const uint32_t gg = s_big[bi];
                const uint32_t a = heads[gg];
                const uint32_t b = gg + 1 < G ? heads[gg + 1] : n;
                if (b - a > OVF_BLOCK_GROUP) continue;  // the whole workgroup takes it below
                const GRes r = group_wave(V, a, b - a, A.glen, A.flags);
                if ((tid & 63u) == 0) stage(r, a);
            }
            // groups of more than OVF_BLOCK_GROUP members (the heaviest k-mers): one at a time by the
            // whole workgroup (a single wave would walk them ~20 times serially)
            for (uint32_t bi = 0; bi < nbig; ++bi) {
                const uint32_t gg = s_big[bi];
                const uint32_t a = heads[gg];
                const uint32_t b = gg + 1 < G ? heads[gg + 1] : n;
                if (b - a <= OVF_BLOCK_GROUP) continue;
                GRes r;
                if (!group_block(V, a, b - a, A.glen, A.flags, reinterpret_cast<uint32_t*>(s_hi), 2 * CAP, s_wave, r)) {
                    if (tid < 64) r = group_wave(V, a, b - a, A.glen, A.flags);  // > 2*CAP function runs
                }
                if (tid == 0) stage(r, a);
                __syncthreads();
            }
            __threadfence_block();
            __syncthreads();
        }
        // emit over groups
        unsigned long long* s_base = reinterpret_cast<unsigned long long*>(s_wave + 36);
        for (uint32_t g0 = 0; g0 < G; g0 += nt) {
            const uint32_t g = g0 + tid;
            const uint32_t a = g < G ? heads[g] : 0u;
            const uint64_t H = g < G ? ghi[a] : 0ull;
            const bool kept = (H >> 63) != 0;
            const uint64_t jb = kept ? jobinfo[a] : 0ull;
            const uint32_t jn = (uint32_t)(jb & 0xFFFFFFFFu);
            // an inline chain takes a slot of s_inl now (no job); without a free slot it is a job
            uint32_t islot = OVF_INLINE_CAP;
            if (jn >= inline_min) islot = atomicAdd(&s_ninl, 1u);
            const bool inl = islot < OVF_INLINE_CAP;
            uint32_t K, J, Lt;
            const uint32_t kpos = wg_exclusive_scan(kept ? 1u : 0u, s_wave, K);
            const uint32_t jpos = wg_exclusive_scan((jn && !inl) ? 1u : 0u, s_wave, J);
            const uint32_t lpos = wg_exclusive_scan(jn, s_wave, Lt);
            if (K == 0) continue;
            if (tid == 0) {
                s_base[0] = atomicAdd(A.kept_ctr, (unsigned long long)K);
                atomicAdd(&A.ctr[0], (unsigned long long)K);  // the overflow's own kept count
                if (J) {
                    s_base[1] = atomicAdd(&A.ctr[3], (unsigned long long)J);
                    s_base[2] = atomicAdd(&A.ctr[4], (unsigned long long)Lt);
                }
                s_nbig = 0;
            }
            __syncthreads();
            if (kept) {
                const uint64_t o = s_base[0] + kpos;
                if (jn) {
                    const uint32_t fm = fmean[a];
                    write_kept(A, o, H, kept_lo(fm & 0xFFFFu, fm >> 16, 0, 0));
                    Job jbr;
                    jbr.lens_off = s_base[2] + lpos;
                    jbr.n = jn;
                    jbr.out_idx = (uint32_t)o;
                    if (inl) {
                        s_inl[islot][0] = jbr.lens_off;
                        s_inl[islot][1] = ((uint64_t)jn << 32) | (uint32_t)o;
                    } else {
                        A.jobs[s_base[1] + jpos] = jbr;
                    }
                    if (jn <= 64) {
                        const uint64_t start = jb >> 32;
                        for (uint32_t t = 0; t < jn; ++t)
                            A.lens[jbr.lens_off + t] = A.glen[glo[start + jn - 1 - t] >> 36];
                    } else {
                        const uint32_t bi = atomicAdd(&s_nbig, 1u);
                        s_big[bi] = g;
                        s_lo[bi] = jbr.lens_off;
                    }
                } else {
                    write_kept(A, o, H, glo[a]);
                }
            }
            __syncthreads();
            // long chains: the whole workgroup writes their lengths
            const uint32_t nb = s_nbig;
            for (uint32_t q = 0; q < nb; ++q) {
                const uint32_t gg = s_big[q];
                const uint32_t aa = heads[gg];
                const uint64_t jbq = jobinfo[aa];
                const uint32_t nq = (uint32_t)(jbq & 0xFFFFFFFFu);
                const uint64_t start = jbq >> 32;
                const uint64_t loff = s_lo[q];
                for (uint32_t t = tid; t < nq; t += nt) A.lens[loff + t] = A.glen[glo[start + nq - 1 - t] >> 36];
            }
            __syncthreads();
        }
        // inline chains: a wave pair each (P^2 on the even wave, variance on the odd), raised issue
        // priority -- they are the critical path of the overflow stream
        __threadfence_block();
        __syncthreads();
        const uint32_t ninl = min(s_ninl, OVF_INLINE_CAP);
        const uint32_t wave = tid >> 6, pairs = (nt >> 6) / 2;
        if (ninl && prio == 1) __builtin_amdgcn_s_setprio(1);
        if (ninl && prio == 2) __builtin_amdgcn_s_setprio(2);
        if (ninl && prio >= 3) __builtin_amdgcn_s_setprio(3);
        for (uint32_t q = wave / 2; q < ninl; q += pairs) {
            const uint64_t off = s_inl[q][0], w = s_inl[q][1];
            const uint32_t cn = (uint32_t)(w >> 32), o = (uint32_t)w;
            const uint32_t* x = A.lens + off;
            if ((wave & 1u) == 0) {
                const double med = chain_long_p2(x, cn);
                if ((tid & 63u) == 0) A.out_data[o].median = d2u16(med);
            } else {
                const double v = chain_long_var(x, cn);
                if ((tid & 63u) == 0) A.out_data[o].var = d2u16(v);
            }
        }
    };
    for (;;) {
        if (threadIdx.x == 0) {
            s_q = q_lo + atomicAdd(&plan[q_slot], 1u);
            s_ninl = 0;
        }
        __syncthreads();
        const uint32_t q = s_q;
        if (q >= q_hi) break;
        entry(A.ovf[q]);
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------
// Heavy keys.  An overflow sub-bucket is oversized because a few k-mers occur thousands of times
// (at C3, single k-mers reach ~10^6 occurrences); sorting such a sub-bucket by (key, function,
// ordinal) with a one-workgroup global bitonic network costs O(n log^2 n) passes.  The large
// sub-buckets are split first (k_ovf_split): an LDS table counts each key's occurrences, keys of
// >= HEAVY_MIN occurrences are copied out to their own contiguous range (k_heavy), the rest (the
// "light" keys, ~SUB_TARGET elements) is compacted in place of the sub-bucket's scratch and runs
// through k_overflow as before, now mostly as a single LDS chunk.
//
// A heavy key needs no sort by (function, ordinal) (process_kmer_set, signature_build.tcc:219-293):
//   - best function: a function with >= 80 % of the occurrences is the strict majority, so the
//     Boyer-Moore candidate plus an exact count decides the cut (fp32, as everywhere);
//   - avg_from_end (upper median of the offsets), the u16 length sum, the signature flags: order-free;
//   - the P^2 median / variance samples are the best-function members' protein lengths in visit
//     (reverse ordinal) order; the ordinal is (sequence, window) and every member of one sequence
//     contributes the same length, so the samples are glen[s] over the members' sequence indices
//     sorted descending -- a u32 radix sort, not a 16-byte sort.
// ------------------------------------------------------------------------------------------
constexpr uint32_t HEAVY_MIN = 1024;        // occurrences that make a key heavy
// overflow sub-buckets of at least this size are split: every one beyond LDS (C3 A/B: 4096 ->
// 2049 takes k_overflow's global-network entries down, 1655 -> 1623 ms/step over two boxes)
constexpr uint32_t SPLIT_MIN = CAP + 1;
constexpr uint32_t SPLIT_TAB = 4096;        // LDS key table slots (load <= ~0.5 at SUB_TARGET)
constexpr uint32_t SPLIT_MAXH = 256;        // heavy keys taken out of one sub-bucket (more stay light)
constexpr uint32_t HEAVY_WG = 512;
constexpr uint32_t HEAVY_GRID = 1024;       // k_heavy: persistent workgroups taking keys from a queue

struct HeavyKey {
    uint64_t off;       // first element in the heavy arrays
    uint32_t n;         // occurrences
    uint32_t bucket;    // level-1 bucket of its sub-bucket
    uint32_t rem;       // the key's low hash bits (group key)
    uint32_t pad;
};

struct HeavyArgs {
    HeavyKey* keys;
    unsigned long long* nkeys;    // device counters (cleared per pass)
    unsigned long long* cursor;
    unsigned long long* queue;    // k_heavy's work queue (cleared per pass): keys are taken in list
                                  //   order, largest sub-buckets first (k_ovf_plan / k_ovf_split)
    uint64_t* rec;                // heavy members, key-contiguous: heavy_rec() (8 B) ...
    uint32_t* len;                //   ... and the protein length (4 B) -- 12 B per member instead
                                  //   of the 16-byte element; k_heavy's first read takes rec only
    uint32_t* s0;                 // radix-sort ping-pong of the best members' sequence indices
    uint32_t* s1;
    // giant chains (>= 2^giant_class samples): samples and jobs in this pass's slot buffers, run
    // by k_chain_dyn on a chain stream as soon as k_heavy ends (the pass's own lens buffer is
    // reused by the next pass; the slot's is not until its chains are done)
    uint32_t nosort;              // diagnostics (option diag & 2): the samples in member order
    uint32_t fast;                // n_functions <= HV_FT: function counts in LDS, bucketed sample order
    uint32_t n_total;             // sequences of the build (the bucket range of the sequence indices)
    uint32_t giant_min;           // 0: off
    uint32_t* gsamples;
    Job* gjobs;
    unsigned long long* gcount;   // [0] jobs, [1] samples
    uint64_t gcap;                // sample capacity
    unsigned long long* gstat;    // run totals: [0] giant chains, [1] longest
};

__device__ __forceinline__ uint32_t split_hash(uint32_t rem) { return (rem * 0x9E3779B1u) >> (32 - 12); }

// A heavy member as k_heavy reads it: everything but the key (one key per range) and the length:
//   s << 36 | (len - i) mod 2^16 << 16 | function     (s = global sequence index, 28 bits)
// bits 32..35 stay 0, so ~0 never is a record (the kernels' "no member" marker)
__device__ __forceinline__ uint64_t heavy_rec(uint64_t hi, uint64_t lo) {
    return (lo & ~((1ull << 36) - 1ull)) | ((lo & 0xFFFFull) << 16) | (hi & 0xFFFFull);
}
__device__ __forceinline__ uint32_t hr_func(uint64_t x) { return (uint32_t)x & 0xFFFFu; }
__device__ __forceinline__ uint32_t hr_off(uint64_t x) { return (uint32_t)(x >> 16) & 0xFFFFu; }
__device__ __forceinline__ uint32_t hr_seq(uint64_t x) { return (uint32_t)(x >> 36); }

constexpr uint32_t SPLIT_U = 8;   // elements per thread per iteration (loads issued together)

// One workgroup per overflow entry of >= SPLIT_MIN elements (the first entries of the sorted list).
__global__ __launch_bounds__(BP_THREADS) void k_ovf_split(BucketArgs A, OvfScratch S, HeavyArgs H, uint32_t heavy_min,
                                                           uint32_t* plan) {
    static_assert(SPLIT_TAB == 4096, "split_hash yields 12 bits");
    __shared__ uint32_t s_key[SPLIT_TAB];
    __shared__ uint32_t s_cnt[SPLIT_TAB];
    __shared__ uint16_t s_hid[SPLIT_TAB];
    __shared__ uint64_t s_hbase[SPLIT_MAXH];
    __shared__ uint32_t s_hcur[SPLIT_MAXH];
    __shared__ uint32_t s_nh, s_fail, s_lcur, s_heavy;
    const uint32_t tid = threadIdx.x, nt = blockDim.x, lane = tid & 63u;
    __shared__ uint32_t s_q;
    // entries [0, plan[PLAN_NSPLIT]) of k_ovf_plan's list (the largest), from queue plan[PLAN_Q_SPLIT]
    const uint32_t q_hi = plan[PLAN_NSPLIT];
    auto entry = [&](const uint32_t qe) {
        OvfEntry e = A.ovf[qe];
        const uint64_t* src_hi = (e.src ? A.tmp_hi : A.recs_hi) + e.off;
        const uint64_t* src_lo = (e.src ? A.tmp_lo : A.recs_lo) + e.off;
        const uint32_t n = e.n;
        constexpr uint32_t EMPTY = 0xFFFFFFFFu;
        for (uint32_t q = tid; q < SPLIT_TAB; q += nt) {
            s_key[q] = EMPTY;
            s_cnt[q] = 0;
            s_hid[q] = 0xFFFFu;
        }
        if (tid == 0) {
            s_nh = 0;
            s_fail = 0;
            s_lcur = 0;
            s_heavy = 0;
        }
        __syncthreads();
        const uint64_t lt = (1ull << lane) - 1ull;
        // ---- 1. occurrences per key (wave-aggregated for the lanes sharing lane 0's key) ----
        for (uint32_t j0 = 0; j0 < n; j0 += nt * SPLIT_U) {
            uint32_t rems[SPLIT_U];
    #pragma unroll
            for (uint32_t u = 0; u < SPLIT_U; ++u) {
                const uint32_t j = j0 + u * nt + tid;
                rems[u] = j < n ? (uint32_t)(src_hi[j] >> 16) & REM_MASK : EMPTY;
            }
    #pragma unroll
            for (uint32_t u = 0; u < SPLIT_U; ++u) {
                const uint32_t rem = rems[u];
                const bool v = rem != EMPTY;
                const uint32_t r0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)rem);
                const uint64_t same = __ballot(v && rem == r0);
                const bool lead = v && rem == r0 && (same & lt) == 0;
                if (v && (rem != r0 || lead)) {
                    uint32_t slot = split_hash(rem), probe = 0;
                    for (; probe < SPLIT_TAB; ++probe) {
                        const uint32_t k = s_key[slot];
                        if (k == rem) break;
                        if (k == EMPTY) {
                            const uint32_t old = atomicCAS(&s_key[slot], EMPTY, rem);
                            if (old == EMPTY || old == rem) break;
                        }
                        slot = (slot + 1) & (SPLIT_TAB - 1);
                    }
                    if (probe == SPLIT_TAB)
                        s_fail = 1;
                    else
                        atomicAdd(&s_cnt[slot], lead ? (uint32_t)__popcll(same) : 1u);
                }
            }
        }
        __syncthreads();
        if (s_fail) return;  // more distinct keys than the table holds: the entry keeps the sort path
        // ---- 2. heavy keys: their own ranges in the heavy arrays ----
        for (uint32_t q = tid; q < SPLIT_TAB; q += nt)
            if (s_cnt[q] >= heavy_min) {
                const uint32_t h = atomicAdd(&s_nh, 1u);
                if (h < SPLIT_MAXH) {
                    s_hid[q] = (uint16_t)h;
                    s_hcur[h] = 0;
                    const uint64_t hk = atomicAdd(H.nkeys, 1ull);
                    const uint64_t base = atomicAdd(H.cursor, (unsigned long long)s_cnt[q]);
                    s_hbase[h] = base;
                    HeavyKey K;
                    K.off = base;
                    K.n = s_cnt[q];
                    K.bucket = e.bucket;
                    K.rem = s_key[q];
                    K.pad = 0;
                    H.keys[hk] = K;
                    atomicAdd(&s_heavy, s_cnt[q]);
                }
            }
        __syncthreads();
        if (s_heavy == 0) return;  // nothing heavy: unchanged
        // ---- 3. scatter: heavy members to their key's range, the rest compacted into the scratch ----
        uint64_t* lhi = S.hi + e.scratch;
        uint64_t* llo = S.lo + e.scratch;
        for (uint32_t j0 = 0; j0 < n; j0 += nt * SPLIT_U) {
            uint64_t eh[SPLIT_U], el[SPLIT_U];
    #pragma unroll
            for (uint32_t u = 0; u < SPLIT_U; ++u) {
                const uint32_t j = j0 + u * nt + tid;
                eh[u] = j < n ? src_hi[j] : ~0ull;
                el[u] = j < n ? src_lo[j] : 0ull;
            }
    #pragma unroll
            for (uint32_t u = 0; u < SPLIT_U; ++u) {
                const bool v = eh[u] != ~0ull;
                uint32_t hid = 0xFFFFu;
                if (v) {
                    const uint32_t rem = (uint32_t)(eh[u] >> 16) & REM_MASK;
                    uint32_t slot = split_hash(rem);
                    while (s_key[slot] != rem) slot = (slot + 1) & (SPLIT_TAB - 1);
                    hid = s_hid[slot];
                }
                // light members: wave-aggregated cursor
                const uint64_t lm = __ballot(v && hid == 0xFFFFu);
                uint32_t lbase = 0;
                if (lm) {
                    const uint32_t leader = (uint32_t)(__ffsll((long long)lm) - 1);
                    if (lane == leader) lbase = atomicAdd(&s_lcur, (uint32_t)__popcll(lm));
                    lbase = (uint32_t)__shfl((int)lbase, (int)leader, 64);
                }
                if (v && hid == 0xFFFFu) {
                    const uint32_t pos = lbase + (uint32_t)__popcll(lm & lt);
                    lhi[pos] = eh[u];
                    llo[pos] = el[u];
                }
                // heavy members: aggregated for the lanes sharing lane 0's key
                const uint32_t h0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(v ? hid : 0xFFFFu));
                const uint64_t hm = __ballot(v && hid != 0xFFFFu && hid == h0);
                uint32_t hbase = 0;
                if (hm) {
                    const uint32_t leader = (uint32_t)(__ffsll((long long)hm) - 1);
                    if (lane == leader) hbase = atomicAdd(&s_hcur[h0], (uint32_t)__popcll(hm));
                    hbase = (uint32_t)__shfl((int)hbase, (int)leader, 64);
                }
                if (v && hid != 0xFFFFu) {
                    const uint32_t pos = hid == h0 ? hbase + (uint32_t)__popcll(hm & lt) : atomicAdd(&s_hcur[hid], 1u);
                    const uint64_t o = s_hbase[hid] + pos;
                    H.rec[o] = heavy_rec(eh[u], el[u]);
                    H.len[o] = elem_len(eh[u], el[u], A.glen);
                }
            }
        }
        __syncthreads();
        if (tid == 0) {  // the entry now names its light remainder (in place in its scratch)
            e.n = n - s_heavy;
            e.src = 2;
            e.off = e.scratch;
            A.ovf[qe] = e;
        }
    };
    for (;;) {
        if (tid == 0) s_q = atomicAdd(&plan[PLAN_Q_SPLIT], 1u);
        __syncthreads();
        const uint32_t q = s_q;
        if (q >= q_hi) break;
        entry(q);
        __syncthreads();
    }
}

// Stable LSD radix sort (ascending) of a[0..n) by one workgroup, RB-bit digits over `bits` bits,
// ping-ponging with b; returns the buffer holding the result.  Items go in rounds of one per
// thread, the next round's item loaded before the current one is ranked; a round's rank among
// equal digits is the wave ballot match plus the lower waves' counts (tagged with the round
// number, so the count table is never cleared: tag 0 is never live).
constexpr int RB = 9;
constexpr uint32_t RBINS = 1u << RB;
__device__ uint32_t* wg_radix_sort_u32(uint32_t* a, uint32_t* b, uint32_t n, int bits, uint32_t* s_hist,
                                       uint32_t (*s_wc)[RBINS], uint32_t* s_run, uint32_t& tag) {
    const uint32_t tid = threadIdx.x, nt = blockDim.x, lane = tid & 63u, wave = tid >> 6, nw = nt >> 6;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int shift = 0; shift < bits; shift += RB) {
        for (uint32_t d = tid; d < RBINS; d += nt) s_hist[d] = 0;
        __syncthreads();
        for (uint32_t j0 = 0; j0 < n; j0 += nt * SPLIT_U) {
            uint32_t x[SPLIT_U];
#pragma unroll
            for (uint32_t u = 0; u < SPLIT_U; ++u) {
                const uint32_t j = j0 + u * nt + tid;
                x[u] = j < n ? a[j] : 0u;
            }
#pragma unroll
            for (uint32_t u = 0; u < SPLIT_U; ++u)
                if (j0 + u * nt + tid < n) atomicAdd(&s_hist[(x[u] >> shift) & (RBINS - 1)], 1u);
        }
        __syncthreads();
        {   // exclusive scan of the bins (one bin per thread, RBINS <= blockDim)
            const uint32_t c = tid < RBINS ? s_hist[tid] : 0u;
            uint32_t tot;
            const uint32_t ex = wg_exclusive_scan(c, s_run + RBINS, tot);
            if (tid < RBINS) s_run[tid] = ex;
            __syncthreads();
        }
        uint32_t nk = tid < n ? a[tid] : 0u;
        for (uint32_t j0 = 0; j0 < n; j0 += nt) {
            ++tag;
            const uint32_t j = j0 + tid;
            const bool v = j < n;
            const uint32_t k = nk;
            if (j0 + nt + tid < n) nk = a[j0 + nt + tid];
            const uint32_t d = (k >> shift) & (RBINS - 1);
            uint64_t peers = __ballot(v);
#pragma unroll
            for (int q = 0; q < RB; ++q) {
                const uint64_t m = __ballot((d >> q) & 1u);
                peers &= ((d >> q) & 1u) ? m : ~m;
            }
            const uint32_t pre = (uint32_t)__popcll(peers & lt);
            const uint32_t tg = tag & 0x1FFFFFFu;
            if (v && pre == 0) s_wc[wave][d] = (tg << 7) | (uint32_t)__popcll(peers);
            __syncthreads();
            if (v) {
                uint32_t o = s_run[d] + pre;
                for (uint32_t w = 0; w < wave; ++w) {
                    const uint32_t c = s_wc[w][d];
                    if ((c >> 7) == tg) o += c & 127u;
                }
                b[o] = k;
            }
            __syncthreads();
            for (uint32_t dd = tid; dd < RBINS; dd += nt) {
                uint32_t add = 0;
                for (uint32_t w = 0; w < nw; ++w) {
                    const uint32_t c = s_wc[w][dd];
                    if ((c >> 7) == tg) add += c & 127u;
                }
                s_run[dd] += add;
            }
            __syncthreads();
        }
        uint32_t* t = a;
        a = b;
        b = t;
    }
    return a;
}

// k_heavy's one-read statistics and bucketed sample order (round 4): the per-function counts of a
// heavy key in an LDS table (exact best function, no Boyer-Moore + recount), and the best members'
// (sequence index, length) items scattered into HV_NBK-way sequence-index buckets of <= HV_BCAP
// items, each bucket sorted by one wave in registers -- instead of compacting sequence indices,
// LSD-sorting them in three barrier-bound passes and gathering each member's length at random.
constexpr uint32_t HV_FT = 4096;     // function table (n_functions <= HV_FT; else the Boyer-Moore path)
constexpr uint32_t HV_NBK = 4096;    // sequence-index buckets per key (power of two <= HV_NBK)
constexpr uint32_t HV_BCAP = 512;    // items one wave sorts (8 per lane); a larger bucket: the LSD path

// LDS histogram add of one value per lane into bins that few values share (the offset's high byte:
// (len - i) mod 2^16 of a family's members lands in a handful of bins, so per-lane atomics would
// serialise 64-deep on one address): one atomic per distinct bin per wave.
__device__ __forceinline__ void wave_hist_add(uint32_t* h, uint32_t bin, bool v) {
    const uint32_t lane = threadIdx.x & 63u;
    uint64_t act = __ballot(v);
    while (act) {
        const uint32_t l0 = (uint32_t)__ffsll((long long)act) - 1u;
        const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)bin, (int)l0);
        const uint64_t m = __ballot(v && bin == b0) & act;
        if (lane == l0) atomicAdd(&h[b0], (uint32_t)__popcll(m));
        act &= ~m;
    }
}

// Bitonic sort, descending, of 64 E items held E per lane (item i = e * 64 + lane).
template <int E>
__device__ __forceinline__ void wave_sort_desc(uint64_t (&v)[E]) {
    const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
    for (int k = 2; k <= 64 * E; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j >= 64) {
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const int pe = e ^ (j >> 6);
                    if (pe > e) {
                        const bool up = (((uint32_t)e * 64u + lane) & (uint32_t)k) == 0;
                        const uint64_t a = v[e], b = v[pe];
                        if (up ? a < b : a > b) {
                            v[e] = b;
                            v[pe] = a;
                        }
                    }
                }
            } else {
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const uint32_t i = (uint32_t)e * 64u + lane;
                    const uint64_t o = xs64(v[e], j);
                    const bool keep_max = ((i & (uint32_t)j) == 0) == ((i & (uint32_t)k) == 0);
                    v[e] = keep_max ? (v[e] > o ? v[e] : o) : (v[e] < o ? v[e] : o);
                }
            }
        }
    }
}

// one bucket [a, a + c) of (s + 1, length) items (0: not a best member): sorted descending by one
// wave, the first nb lengths out in visit order (sequence index descending) at out, the best
// members' signature flags set in that order
template <int E>
__device__ __forceinline__ void heavy_bucket_out(const uint32_t* __restrict__ ks, const uint32_t* __restrict__ ls,
                                                 uint32_t a, uint32_t c, uint32_t nb, uint32_t* __restrict__ out,
                                                 uint8_t* flags) {
    const uint32_t lane = threadIdx.x & 63u;
    uint64_t v[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t i = (uint32_t)e * 64u + lane;
        v[e] = i < c ? ((uint64_t)ks[a + i] << 32) | ls[a + i] : 0ull;
    }
    wave_sort_desc<E>(v);
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t i = (uint32_t)e * 64u + lane;
        if (i < nb) {
            out[i] = (uint32_t)v[e];
            if (flags) mark_seq(flags, (uint32_t)(v[e] >> 32) - 1u);
        }
    }
}

// One heavy key per workgroup iteration (persistent grid; the key count is read on the device).
__global__ __launch_bounds__(HEAVY_WG) void k_heavy(BucketArgs A, HeavyArgs H) {
    static_assert(RBINS <= HEAVY_WG, "one radix bin per thread in the scan");
    __shared__ uint32_t s_hist[RBINS], s_run[RBINS + 48];
    __shared__ uint32_t s_wc[HEAVY_WG / 64][RBINS];
    __shared__ __align__(16) uint32_t s_wave[48];
    __shared__ uint32_t s_bm[2 * (HEAVY_WG / 64)];
    __shared__ uint32_t s_cur, s_sel[3], s_key;
    __shared__ uint32_t s_fb[HV_FT];    // function counts (pass 1), then best members per bucket
    __shared__ uint32_t s_bk[HV_NBK];   // members per bucket -> bucket cursors -> bucket ends
    __shared__ uint32_t s_oh[256], s_ol[256];  // offset histograms: high byte, low byte
    static_assert(HV_FT == HV_NBK, "s_fb doubles as the per-bucket best counts");
    const uint32_t tid = threadIdx.x, nt = blockDim.x, lane = tid & 63u, wave = tid >> 6, nw = nt >> 6;
    const uint64_t lt = (1ull << lane) - 1ull;
    const uint32_t nkeys = (uint32_t)*H.nkeys;
    uint32_t tag = 0;  // round tags of s_wc: 0 is never a live round
    for (uint32_t q = tid; q < (HEAVY_WG / 64) * RBINS; q += nt) (&s_wc[0][0])[q] = 0;
    __syncthreads();
    constexpr uint32_t U = SPLIT_U;
    for (;;) {
        // dynamic queue: a workgroup that drew a giant key does not also own every 512th key after it
        __syncthreads();
        if (tid == 0) s_key = (uint32_t)min((unsigned long long)nkeys, atomicAdd(H.queue, 1ull));
        __syncthreads();
        const uint32_t q = s_key;
        if (q >= nkeys) break;
        const HeavyKey K = H.keys[q];
        const uint64_t* rec = H.rec + K.off;
        const uint32_t* rlen = H.len + K.off;
        const uint32_t n = K.n;
        uint32_t best_f = 0, cb = 0, NBK = 0;
        bool bucketed = false;
        if (H.fast) {
            // ---- one read: function counts, offset high byte, members per sequence bucket ----
            NBK = 1;
            while (NBK < HV_NBK && NBK * 256u < n) NBK <<= 1;
            for (uint32_t d = tid; d < HV_FT; d += nt) s_fb[d] = 0;
            for (uint32_t d = tid; d < NBK; d += nt) s_bk[d] = 0;
            for (uint32_t d = tid; d < 256; d += nt) s_oh[d] = 0;
            __syncthreads();
            for (uint32_t j0 = 0; j0 < n; j0 += nt * U) {
                uint64_t x[U];
#pragma unroll
                for (uint32_t u = 0; u < U; ++u) {
                    const uint32_t j = j0 + u * nt + tid;
                    x[u] = j < n ? rec[j] : ~0ull;
                }
#pragma unroll
                for (uint32_t u = 0; u < U; ++u) {
                    const bool v = x[u] != ~0ull;
                    const uint32_t f = v ? hr_func(x[u]) : 0xFFFFFFFFu;
                    // the lanes sharing lane 0's function add once (a heavy key is mostly one function)
                    const uint32_t f0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)f);
                    const uint64_t same = __ballot(v && f == f0);
                    if (v && f != f0) atomicAdd(&s_fb[f], 1u);
                    if (v && f == f0 && (same & lt) == 0) atomicAdd(&s_fb[f], (uint32_t)__popcll(same));
                    wave_hist_add(s_oh, hr_off(x[u]) >> 8, v);
                    if (v) atomicAdd(&s_bk[(uint32_t)(((uint64_t)hr_seq(x[u]) * NBK) / H.n_total)], 1u);
                }
            }
            __syncthreads();
            // the best function: the largest count, ties to the lowest FunctionIndex (the first
            // std::map entry wins and only a strictly greater count replaces it)
            uint32_t cm = 0;
            for (uint32_t d = tid; d < HV_FT; d += nt) cm = max(cm, s_fb[d]);
            cm = wg_max(cm, s_wave);
            uint32_t fm = 0;
            for (uint32_t d = tid; d < HV_FT; d += nt)
                if (s_fb[d] == cm) fm = max(fm, HV_FT - 1u - d);
            fm = wg_max(fm, s_wave);
            best_f = HV_FT - 1u - fm;
            cb = cm;
            uint32_t bm = 0;
            for (uint32_t d = tid; d < NBK; d += nt) bm = max(bm, s_bk[d]);
            bm = wg_max(bm, s_wave);
            bucketed = bm <= HV_BCAP && !H.nosort;
        } else {
            // ---- Boyer-Moore majority function, then its exact count ----
            uint32_t cand = 0xFFFFFFFFu, cc = 0;
            for (uint32_t j0 = 0; j0 < n; j0 += nt * U) {
                uint32_t f[U];
    #pragma unroll
                for (uint32_t u = 0; u < U; ++u) {
                    const uint32_t j = j0 + u * nt + tid;
                    f[u] = j < n ? hr_func(rec[j]) : 0xFFFFFFFFu;
                }
    #pragma unroll
                for (uint32_t u = 0; u < U; ++u) {
                    if (f[u] == 0xFFFFFFFFu) continue;
                    if (cc == 0) {
                        cand = f[u];
                        cc = 1;
                    } else if (f[u] == cand) {
                        ++cc;
                    } else {
                        --cc;
                    }
                }
            }
            bm_combine(cand, cc);  // over the wave (lane 0 broadcast)
            if (lane == 0) {
                s_bm[2 * wave] = cand;
                s_bm[2 * wave + 1] = cc;
            }
            __syncthreads();
            if (tid == 0) {
                uint32_t c0 = s_bm[0], n0 = s_bm[1];
                for (uint32_t w = 1; w < nw; ++w) {
                    const uint32_t c1 = s_bm[2 * w], n1 = s_bm[2 * w + 1];
                    if (c1 == c0) {
                        n0 += n1;
                    } else if (n0 >= n1) {
                        n0 -= n1;
                    } else {
                        c0 = c1;
                        n0 = n1 - n0;
                    }
                }
                s_sel[0] = c0;
            }
            __syncthreads();
            best_f = s_sel[0];
            cb = 0;
            for (uint32_t j0 = 0; j0 < n; j0 += nt * U) {
                uint32_t f[U];
    #pragma unroll
                for (uint32_t u = 0; u < U; ++u) {
                    const uint32_t j = j0 + u * nt + tid;
                    f[u] = j < n ? hr_func(rec[j]) : 0xFFFFFFFFu;
                }
    #pragma unroll
                for (uint32_t u = 0; u < U; ++u) cb += f[u] == best_f;
            }
            cb = wg_sum(cb, s_wave);
        }
        if ((float)cb < float(n) * 0.8f) continue;  // cut (uniform); the best run is the majority
        uint32_t pre = 0;         // avg_from_end: the (n/2)-th smallest offset
        uint16_t mean = 0;
        const uint32_t* sorted = nullptr;  // the LSD path: the best members' sequence indices, ascending
        if (bucketed) {
            // ---- bucket starts; the offset's high byte ----
            {
                const uint32_t per = (NBK + nt - 1) / nt, b0 = min(NBK, tid * per), b1 = min(NBK, b0 + per);
                uint32_t loc = 0;
                for (uint32_t d = b0; d < b1; ++d) loc += s_bk[d];
                uint32_t tot;
                uint32_t x = wg_exclusive_scan(loc, s_wave, tot);
                for (uint32_t d = b0; d < b1; ++d) {
                    const uint32_t c = s_bk[d];
                    s_bk[d] = x;  // cursor = start
                    x += c;
                }
            }
            for (uint32_t d = tid; d < NBK; d += nt) s_fb[d] = 0;  // best members per bucket
            for (uint32_t d = tid; d < 256; d += nt) s_ol[d] = 0;
            if (tid == 0) {
                uint32_t kk = n / 2, d = 0;
                while (kk >= s_oh[d]) kk -= s_oh[d++];
                s_sel[0] = d;
                s_sel[1] = kk;
            }
            __syncthreads();
            const uint32_t hb = s_sel[0], krem = s_sel[1];
            // ---- second read: flags of the other members, u16 length sum, the offset's low byte,
            //      every member's item into its bucket ((s + 1, length) for the best, 0 otherwise) ----
            uint32_t* ks = H.s0 + K.off;
            uint32_t* ls = H.s1 + K.off;
            uint32_t sum = 0;
            for (uint32_t j0 = 0; j0 < n; j0 += nt * U) {
                uint64_t x[U];
                uint32_t ln[U];
#pragma unroll
                for (uint32_t u = 0; u < U; ++u) {
                    const uint32_t j = j0 + u * nt + tid;
                    x[u] = j < n ? rec[j] : ~0ull;
                    ln[u] = j < n ? rlen[j] : 0u;
                }
#pragma unroll
                for (uint32_t u = 0; u < U; ++u) {
                    if (x[u] == ~0ull) continue;
                    const uint32_t sq = hr_seq(x[u]);
                    const uint32_t bk = (uint32_t)(((uint64_t)sq * NBK) / H.n_total);
                    const uint32_t off = hr_off(x[u]);
                    if ((off >> 8) == hb) atomicAdd(&s_ol[off & 255u], 1u);
                    const bool best = hr_func(x[u]) == best_f;
                    const uint32_t slot = atomicAdd(&s_bk[bk], 1u);
                    if (best) {
                        sum += ln[u] & 0xFFFFu;  // the u16 accumulator needs len mod 2^16 only
                        atomicAdd(&s_fb[bk], 1u);
                        ks[slot] = sq + 1u;
                        ls[slot] = ln[u];
                    } else {
                        ks[slot] = 0u;
                        ls[slot] = 0u;
                        if (A.flags) mark_seq(A.flags, sq);
                    }
                }
            }
            sum = wg_sum(sum, s_wave);  // its barriers also close the scatter
            mean = d2u16((double)(uint16_t)sum / (double)cb);
            if (tid == 0) {
                uint32_t kk = krem, d = 0;
                while (kk >= s_ol[d]) kk -= s_ol[d++];
                s_sel[0] = (hb << 8) | d;
            }
            // the buckets' output offsets in visit order (sequence index descending: the last
            // bucket first), in place of their best counts: s_fb[k] = best members of buckets > k
            {
                const uint32_t per = (NBK + nt - 1) / nt, r0 = min(NBK, tid * per), r1 = min(NBK, r0 + per);
                uint32_t loc = 0;
                for (uint32_t r = r0; r < r1; ++r) loc += s_fb[NBK - 1 - r];
                uint32_t tot;
                uint32_t x = wg_exclusive_scan(loc, s_wave, tot);
                for (uint32_t r = r0; r < r1; ++r) {
                    const uint32_t c = s_fb[NBK - 1 - r];
                    s_fb[NBK - 1 - r] = x;
                    x += c;
                }
            }
            __syncthreads();
            pre = s_sel[0];
        } else {
            // ---- flags, u16 length sum and the best members' sequence indices; offset histogram
            //      of the high byte for the upper-median select ----
            if (tid == 0) s_cur = 0;
            for (uint32_t d = tid; d < 256; d += nt) s_hist[d] = 0;
            __syncthreads();
            uint32_t* sa = H.s0 + K.off;
            uint32_t* sb = H.s1 + K.off;
            uint32_t sum = 0, smax = 0;
            for (uint32_t j0 = 0; j0 < n; j0 += nt * U) {
                uint64_t l[U];
                uint32_t f[U], gl[U];
    #pragma unroll
                for (uint32_t u = 0; u < U; ++u) {
                    const uint32_t j = j0 + u * nt + tid;
                    const uint64_t x = j < n ? rec[j] : ~0ull;
                    f[u] = j < n ? hr_func(x) : 0xFFFFFFFFu;
                    // the mean's accumulator is a u16: the length mod 2^16 is all it needs
                    gl[u] = j < n ? rlen[j] & 0xFFFFu : 0u;
                    l[u] = x;
                }
    #pragma unroll
                for (uint32_t u = 0; u < U; ++u) gl[u] = f[u] == best_f ? gl[u] : 0u;
    #pragma unroll
                for (uint32_t u = 0; u < U; ++u) {
                    const bool v = f[u] != 0xFFFFFFFFu;
                    const uint32_t s = hr_seq(l[u]);
                    const bool best = f[u] == best_f;
                    if (v && !best && A.flags) mark_seq(A.flags, s);  // the best members' flags go out in sorted order below
                    wave_hist_add(s_hist, hr_off(l[u]) >> 8, v);
                    if (best) {
                        sum += gl[u];
                        smax = max(smax, s);
                    }
                    const uint64_t bm = __ballot(best);
                    uint32_t base = 0;
                    if (bm) {
                        const uint32_t leader = (uint32_t)(__ffsll((long long)bm) - 1);
                        if (lane == leader) base = atomicAdd(&s_cur, (uint32_t)__popcll(bm));
                        base = (uint32_t)__shfl((int)base, (int)leader, 64);
                    }
                    if (best) sa[base + (uint32_t)__popcll(bm & lt)] = s;
                }
            }
            sum = wg_sum(sum, s_wave);
            smax = wg_max(smax, s_wave);
            mean = d2u16((double)(uint16_t)sum / (double)cb);
            // ---- avg_from_end: the (n/2)-th smallest offset, high byte then low byte ----
            uint32_t k = n / 2;
            for (int sh = 8; sh >= 0; sh -= 8) {
                if (sh == 0) {
                    for (uint32_t d = tid; d < 256; d += nt) s_hist[d] = 0;
                    __syncthreads();
                    for (uint32_t j0 = 0; j0 < n; j0 += nt * U) {
                        uint32_t o[U];
    #pragma unroll
                        for (uint32_t u = 0; u < U; ++u) {
                            const uint32_t j = j0 + u * nt + tid;
                            o[u] = j < n ? hr_off(rec[j]) : 0xFFFFFFFFu;
                        }
    #pragma unroll
                        for (uint32_t u = 0; u < U; ++u)
                            if (o[u] != 0xFFFFFFFFu && (o[u] >> 8) == (pre >> 8)) atomicAdd(&s_hist[o[u] & 255u], 1u);
                    }
                }
                __syncthreads();
                if (tid == 0) {
                    uint32_t d = 0;
                    while (k >= s_hist[d]) k -= s_hist[d++];
                    s_sel[0] = d;
                    s_sel[1] = k;
                }
                __syncthreads();
                pre |= s_sel[0] << sh;
                k = s_sel[1];
                __syncthreads();
            }
            // ---- samples in visit order: sequence indices descending ----
            int bits = 0;
            while (bits < 32 && (smax >> bits)) bits += RB;
            sorted = H.nosort ? sa : wg_radix_sort_u32(sa, sb, cb, bits, s_hist, s_wc, s_run, tag);
            __syncthreads();
        }
        if (tid == 0) {
            s_sel[0] = (uint32_t)atomicAdd(A.kept_ctr, 1ull);
            atomicAdd(&A.ctr[0], 1ull);
            // a giant chain's samples go to the pass's giant buffer while it has room (sized
            // before the run: a key that does not fit takes the ordinary job path)
            bool g = false;
            if (H.giant_min && cb >= H.giant_min) {
                const uint64_t c = atomicAdd(&H.gcount[1], (unsigned long long)cb);
                if (c + cb <= H.gcap) {
                    g = true;
                    s_cur = (uint32_t)c;
                    s_sel[1] = (uint32_t)atomicAdd(&H.gcount[0], 1ull);
                    atomicAdd(&H.gstat[0], 1ull);
                    atomicMax(&H.gstat[1], (unsigned long long)cb);
                }
            }
            if (!g) {
                s_sel[1] = (uint32_t)atomicAdd(&A.ctr[3], 1ull);
                s_cur = (uint32_t)atomicAdd(&A.ctr[4], (unsigned long long)cb);
            }
            s_sel[2] = g ? 1u : 0u;
        }
        __syncthreads();
        const uint32_t o = s_sel[0], jb = s_sel[1], loff = s_cur;
        const bool giant = s_sel[2] != 0;
        uint32_t* lens_out = giant ? H.gsamples : A.lens;
        if (bucketed) {
            // ---- each bucket sorted by one wave; its best members' lengths out in visit order ----
            const uint32_t* ks = H.s0 + K.off;
            const uint32_t* ls = H.s1 + K.off;
            for (uint32_t bk = wave; bk < NBK; bk += nw) {
                const uint32_t a = bk ? s_bk[bk - 1] : 0u, c = s_bk[bk] - a;
                const uint32_t nb = (bk ? s_fb[bk - 1] : cb) - s_fb[bk];
                if (nb == 0) continue;
                uint32_t* out = lens_out + (uint64_t)loff + s_fb[bk];
                if (c <= 64)
                    heavy_bucket_out<1>(ks, ls, a, c, nb, out, A.flags);
                else if (c <= 128)
                    heavy_bucket_out<2>(ks, ls, a, c, nb, out, A.flags);
                else if (c <= 256)
                    heavy_bucket_out<4>(ks, ls, a, c, nb, out, A.flags);
                else
                    heavy_bucket_out<8>(ks, ls, a, c, nb, out, A.flags);
            }
        } else {
            for (uint32_t t0 = 0; t0 < cb; t0 += nt * U) {
                uint32_t sv[U];
    #pragma unroll
                for (uint32_t u = 0; u < U; ++u) {
                    const uint32_t t = t0 + u * nt + tid;
                    sv[u] = t < cb ? sorted[cb - 1 - t] : 0u;
                }
    #pragma unroll
                for (uint32_t u = 0; u < U; ++u) {
                    const uint32_t t = t0 + u * nt + tid;
                    if (t < cb) {
                        // monotone sequence indices: the length gathers and the signature flags of the
                        // best members touch neighbouring lines instead of random ones
                        lens_out[(uint64_t)loff + t] = A.glen[sv[u]];
                        if (A.flags) mark_seq(A.flags, sv[u]);
                    }
                }
            }
        }
        if (tid == 0) {
            const uint64_t h43 = key_h43((uint64_t)(A.bucket_base + K.bucket) << A.rem_bits, K.rem, A.rem_bits, A.pshift);
            write_kept(A, o, kept_hi(h43, pre), kept_lo(best_f, mean, 0, 0));
            Job jbr;
            jbr.n = cb;
            jbr.out_idx = o;
            if (giant) {
                jbr.lens_off = reinterpret_cast<uint64_t>(H.gsamples + loff);  // device address
                H.gjobs[jb] = jbr;
            } else {
                jbr.lens_off = loff;
                A.jobs[jb] = jbr;
            }
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------
// Overflow plan, on the device (one workgroup, right after k_partition): the host used to read the
// overflow list back, sort it by size and size the scratch.  The entries are counting-sorted into
// descending size classes (tier by the split / heavy thresholds, then floor(log2 n)), so the split
// and heavy entries are prefixes and the persistent kernels take the largest first; each entry gets
// its scratch range (pow2 >= n elements); the totals are checked against the work buffers sized
// before the run (too small: the demand is recorded and the step redone with grown buffers) and the
// kept arena against the pass's element count (full: SKM_E_OOM at the step's end).
// ------------------------------------------------------------------------------------------
struct PlanArgs {
    const OvfEntry* in;                 // k_partition's list
    OvfEntry* out;                      // sorted by size class, descending, scratch assigned
    const unsigned long long* ctr;      // the pass's counters: [1] entries (low 32 bits)
    const unsigned long long* kept;     // [0]: the kept arena cursor
    const unsigned long long* nloc;     // elements the pass groups
    unsigned long long* run;
    uint32_t* plan;
    uint32_t ovf_cap, split_min, heavy_min;
    uint64_t kept_cap, tot_cap, split_cap;
};

constexpr uint32_t PLAN_BINS = 3 * 32;

__device__ __forceinline__ uint32_t plan_bin(uint32_t n, uint32_t split_min, uint32_t heavy_min) {
    const uint32_t tier = (n >= split_min ? 1u : 0u) + (n >= heavy_min ? 1u : 0u);
    return PLAN_BINS - 1u - (tier * 32u + (31u - (uint32_t)__clz(n | 1u)));  // 0: the largest
}

__global__ __launch_bounds__(1024) void k_ovf_plan(PlanArgs P) {
    __shared__ uint32_t s_cnt[PLAN_BINS];
    __shared__ unsigned long long s_part[1024];
    __shared__ unsigned long long s_tot, s_elems, s_split;
    __shared__ uint32_t s_nsplit, s_nheavy;
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    const uint64_t raw = P.ctr[1] & 0xFFFFFFFFull;
    const uint32_t n = (uint32_t)min<uint64_t>(raw, P.ovf_cap);
    for (uint32_t i = tid; i < PLAN_BINS; i += nt) s_cnt[i] = 0;
    if (tid == 0) {
        s_tot = s_elems = s_split = 0;
        s_nsplit = s_nheavy = 0;
    }
    __syncthreads();
    for (uint32_t i = tid; i < n; i += nt) atomicAdd(&s_cnt[plan_bin(P.in[i].n, P.split_min, P.heavy_min)], 1u);
    __syncthreads();
    if (tid == 0) {
        uint32_t r = 0;
        for (uint32_t b = 0; b < PLAN_BINS; ++b) {
            const uint32_t c = s_cnt[b];
            s_cnt[b] = r;
            r += c;
        }
    }
    __syncthreads();
    unsigned long long lt = 0, le = 0, ls = 0;
    uint32_t lns = 0, lnh = 0;
    for (uint32_t i = tid; i < n; i += nt) {
        OvfEntry e = P.in[i];
        const uint32_t pos = atomicAdd(&s_cnt[plan_bin(e.n, P.split_min, P.heavy_min)], 1u);
        uint64_t np = 1;
        while (np < e.n) np <<= 1;
        e.npad = (uint32_t)np;
        P.out[pos] = e;
        lt += np;
        le += e.n;
        if (e.n >= P.split_min) {
            ls += e.n;
            ++lns;
        }
        if (e.n >= P.heavy_min) ++lnh;
    }
    atomicAdd(&s_tot, lt);
    atomicAdd(&s_elems, le);
    atomicAdd(&s_split, ls);
    atomicAdd(&s_nsplit, lns);
    atomicAdd(&s_nheavy, lnh);
    __threadfence_block();
    __syncthreads();
    // scratch offsets in list order: a contiguous run of entries per thread
    const uint32_t per = (n + nt - 1) / nt;
    const uint32_t a = min(n, tid * per), e_ = min(n, a + per);
    unsigned long long sum = 0;
    for (uint32_t i = a; i < e_; ++i) sum += P.out[i].npad;
    s_part[tid] = sum;
    __syncthreads();
    if (tid == 0) {
        unsigned long long r = 0;
        for (uint32_t t = 0; t < nt; ++t) {
            const unsigned long long v = s_part[t];
            s_part[t] = r;
            r += v;
        }
    }
    __syncthreads();
    unsigned long long o = s_part[tid];
    for (uint32_t i = a; i < e_; ++i) {
        P.out[i].scratch = o;
        o += P.out[i].npad;
    }
    if (tid == 0) {
        unsigned long long* R = P.run;
        const uint64_t tot = s_tot, split = s_split, nl = *P.nloc;
        // demands are recorded for every pass, so one redo takes the whole run
        atomicMax(&R[RUN_DEM_TOT], (unsigned long long)tot);
        atomicMax(&R[RUN_DEM_SPLIT], (unsigned long long)split);
        if (raw > P.ovf_cap) atomicOr(&R[RUN_FLAGS], RUN_F_CAP);
        const bool over = tot > P.tot_cap || split > P.split_cap;
        if (over) atomicOr(&R[RUN_FLAGS], RUN_F_RERUN);
        if (P.kept[0] + nl > P.kept_cap) atomicOr(&R[RUN_FLAGS], RUN_F_ARENA);
        // a pass that does not fit is skipped (the step is redone); after an error every pass is.
        // The passes after a mere overrun still run, so their demands are known for the redo
        const bool skip = over || (atomicAdd(&R[RUN_FLAGS], 0ull) & (RUN_F_ARENA | RUN_F_CAP)) != 0;
        P.plan[PLAN_NOVF] = skip ? 0u : n;
        P.plan[PLAN_NSPLIT] = skip ? 0u : s_nsplit;
        P.plan[PLAN_NHEAVY] = skip ? 0u : s_nheavy;
        P.plan[PLAN_SKIP] = skip ? 1u : 0u;
        P.plan[PLAN_Q_SPLIT] = 0;
        P.plan[PLAN_Q_HEAVY] = 0;
        P.plan[PLAN_Q_REST] = 0;
        R[RUN_ACC_NOVF] += n;
        R[RUN_ACC_OVF_ELEMS] += s_elems;
        R[RUN_ACC_GROUPED] += nl;
        R[RUN_LAST_NOVF] = n;
    }
}

// end of a pass (one thread, after both overflow streams joined): run totals and the bounds the
// chain lists rely on
// tests (poison_jobs): every slot of the stashed long-job list holds a canary job whose output
// record is the arena's spare slot at index `idx` (past the kept capacity); k_chain_long reaching a
// slot k_long_stash did not write would overwrite the canary record, which phase_final checks
__global__ void k_poison_jobs(Job* __restrict__ jobs, uint64_t n, uint64_t samples, uint32_t idx,
                             skm_stored_kmer_data* __restrict__ out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (uint64_t j = t; j < n; j += (uint64_t)gridDim.x * blockDim.x) jobs[j] = Job{samples, 8u, idx};
    if (t == 0) out[idx] = skm_stored_kmer_data{0xC0DE, 0xC0DE, 0xC0DE, 0xC0DE, 0xC0DE};
}

__global__ void k_pass_account(const unsigned long long* __restrict__ ctr, unsigned long long* __restrict__ run,
                               uint64_t jobs_cap, uint64_t jobs2_cap, uint64_t big_cap, uint64_t lens_cap) {
    const unsigned long long j = ctr[3] + ctr[8 + 3];
    run[RUN_ACC_JOBS] += j;
    run[RUN_ACC_LENS] += ctr[8 + 4];
    run[RUN_ACC_OVF_KEPT] += ctr[8];
    run[RUN_ACC_BIG] += ctr[5];
    run[RUN_ACC_BIG_KEPT] += ctr[6];
    run[RUN_LAST_JOBS] = j;
    if (ctr[3] > jobs_cap || ctr[8 + 3] > jobs2_cap || ctr[5] > big_cap || ctr[8 + 4] > lens_cap)
        atomicOr(&run[RUN_FLAGS], RUN_F_CAP);
}

// distinct_functions[f] += kept k-mers with best function f (LDS privatised when it fits)
// Over the whole kept arena after the last pass: decode each key (43-bit hash -> unmix43 ->
// base-40 -> the 8 residue bytes, Kmer<8> as a little-endian u64) and count distinct_functions.
__global__ void k_kept_finalize(uint64_t* __restrict__ keys, const skm_stored_kmer_data* __restrict__ data,
                                const unsigned long long* __restrict__ n_p, uint32_t nf, uint32_t* __restrict__ dfunc) {
    extern __shared__ uint32_t s_h[];
    const uint64_t n = *n_p;  // the arena cursor after the last pass
    const bool lds = nf <= 16384;
    if (lds)
        for (uint32_t f = threadIdx.x; f < nf; f += blockDim.x) s_h[f] = 0;
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        keys[i] = decode_key(unmix43(keys[i]));
        uint32_t f = data[i].function_index;
        if (f < nf) {
            if (lds)
                atomicAdd(&s_h[f], 1u);
            else
                atomicAdd(&dfunc[f], 1u);
        }
    }
    __syncthreads();
    if (lds)
        for (uint32_t f = threadIdx.x; f < nf; f += blockDim.x)
            if (s_h[f]) atomicAdd(&dfunc[f], s_h[f]);
}

__global__ void k_func_hist_seqs(const SeqMeta* __restrict__ meta, uint32_t nseq, uint32_t nf, uint32_t* __restrict__ swf) {
    extern __shared__ uint32_t s_h[];
    const bool lds = nf <= 16384;
    if (lds)
        for (uint32_t f = threadIdx.x; f < nf; f += blockDim.x) s_h[f] = 0;
    __syncthreads();
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nseq; s += gridDim.x * blockDim.x) {
        uint32_t f = meta[s].func;
        if (f < nf) {
            if (lds)
                atomicAdd(&s_h[f], 1u);
            else
                atomicAdd(&swf[f], 1u);
        }
    }
    __syncthreads();
    if (lds)
        for (uint32_t f = threadIdx.x; f < nf; f += blockDim.x)
            if (s_h[f]) atomicAdd(&swf[f], s_h[f]);
}

// option flag_bits: the per-sequence bytes from the run's flag bits (one word of 32 flags per thread)
__global__ void k_flags_from_bits(const uint32_t* __restrict__ bits, uint32_t nseq, uint8_t* __restrict__ flags) {
    for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < (nseq + 31) / 32; w += gridDim.x * blockDim.x) {
        const uint32_t v = bits[w];
        const uint32_t n = min(32u, nseq - 32 * w);
        uint8_t* o = flags + 32 * (uint64_t)w;
        for (uint32_t t = 0; t < n; ++t) o[t] = (uint8_t)((v >> t) & 1u);
    }
}

__global__ void k_count_flags(const uint8_t* __restrict__ flags, uint32_t nseq, unsigned long long* __restrict__ out) {
    uint32_t local = 0;
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nseq; s += gridDim.x * blockDim.x) local += flags[s] ? 1u : 0u;
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) local += __shfl_down(local, d, 64);
    if ((threadIdx.x & 63) == 0 && local) atomicAdd(out, (unsigned long long)local);
}

// world > 1 exchange of one pass (exchange()): per-bucket element counts from the owner-major
// bucket starts; each peer's total is checked against the prepare-time count the transfer sizes
// were planned with (a mismatch fails the run with SKM_E_STATE instead of mis-sized transfers)
__global__ void k_send_counts(const uint64_t* __restrict__ bstart, uint32_t NB, uint32_t NB1, uint32_t W,
                              const unsigned long long* __restrict__ expect, unsigned long long* __restrict__ run,
                              uint32_t* __restrict__ out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < NB) out[t] = (uint32_t)(bstart[t + 1] - bstart[t]);
    if (t < W && bstart[(uint64_t)(t + 1) * NB1] - bstart[(uint64_t)t * NB1] != expect[t])
        atomicOr(&run[RUN_FLAGS], (unsigned long long)RUN_F_CAP);
}

// the receive layout from the received counts cnt[source][bucket] (one workgroup): source-major
// pieces (seg_start = exclusive scan of the flattened counts, seg_len = counts) and the bucket-major
// virtual numbering the partition kernel uses (vstart[k] = elements of buckets < k over all
// sources; vstart[NB1] = the pass's element count, read by the overflow plan)
__global__ __launch_bounds__(1024) void k_recv_plan(const uint32_t* __restrict__ cnt, uint32_t W, uint32_t NB1,
                                                    const unsigned long long* __restrict__ expect,
                                                    unsigned long long* __restrict__ run,
                                                    uint64_t* __restrict__ seg_start, uint32_t* __restrict__ seg_len,
                                                    uint64_t* __restrict__ vstart) {
    __shared__ uint32_t s_wave[17];
    __shared__ unsigned long long s_tot[64];
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    const uint32_t N = W * NB1;
    {   // flat exclusive scan (consecutive chunks per thread)
        const uint32_t per = (N + nt - 1) / nt, a = min(N, tid * per), e = min(N, a + per);
        uint32_t loc = 0;
        for (uint32_t i = a; i < e; ++i) loc += cnt[i];
        uint32_t tot;
        uint64_t run_ = wg_exclusive_scan(loc, s_wave, tot);
        for (uint32_t i = a; i < e; ++i) {
            seg_start[i] = run_;
            seg_len[i] = cnt[i];
            run_ += cnt[i];
        }
    }
    if (tid < 64) s_tot[tid] = 0;
    __syncthreads();
    for (uint32_t i = tid; i < N; i += nt) atomicAdd(&s_tot[i / NB1], (unsigned long long)cnt[i]);
    __syncthreads();
    if (tid < W && s_tot[tid] != expect[tid]) atomicOr(&run[RUN_FLAGS], (unsigned long long)RUN_F_CAP);
    {   // per-bucket sums over the sources, exclusive scan over the buckets
        const uint32_t per = (NB1 + nt - 1) / nt, a = min(NB1, tid * per), e = min(NB1, a + per);
        uint32_t loc = 0;
        for (uint32_t k = a; k < e; ++k)
            for (uint32_t p = 0; p < W; ++p) loc += cnt[(uint64_t)p * NB1 + k];
        uint32_t tot;
        uint64_t run_ = wg_exclusive_scan(loc, s_wave, tot);
        for (uint32_t k = a; k < e; ++k) {
            vstart[k] = run_;
            for (uint32_t p = 0; p < W; ++p) run_ += cnt[(uint64_t)p * NB1 + k];
        }
        if (tid == 0) vstart[NB1] = tot;
    }
}

// skm_build_finish_slice: kept k-mers of one output slice (top bits of slice_hash(key)), compacted
// in any order (the host sorts them); count first, then the copy into the slice's own buffers
__global__ __launch_bounds__(256) void k_slice_select(const uint64_t* __restrict__ keys,
                                                      const skm_stored_kmer_data* __restrict__ data, uint64_t n,
                                                      int bits, uint64_t slice, unsigned long long* __restrict__ cursor,
                                                      uint64_t* __restrict__ out_keys,
                                                      skm_stored_kmer_data* __restrict__ out_data) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t b0 = (uint64_t)blockIdx.x * blockDim.x; b0 < n; b0 += stride) {
        const uint64_t j = b0 + threadIdx.x;
        const uint64_t k = j < n ? keys[j] : 0ull;
        const bool in = j < n && (bits == 0 || (slice_hash(k) >> (64 - bits)) == slice);
        const uint64_t m = __ballot(in);
        if (!m) continue;
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(cursor, (unsigned long long)__popcll(m));
        base = __shfl(base, 0, 64);
        if (in && out_keys) {
            const uint64_t o = base + (uint64_t)__popcll(m & ((1ull << lane) - 1ull));
            out_keys[o] = k;
            out_data[o] = data[j];
        }
    }
}

// Build options beyond skm_build_opts: the key-range pass count and device-memory budget
// (skm_build_set_option), and diagnostic tunables kept at their tuned defaults in production.
struct Tune {
    int passes = 0;                  // key-range passes: 0 = automatic from the memory budget
    int64_t mem_budget_mb = 0;       // device memory the build may plan for (0 = free memory)
    int ovf_heavy = 8192;            // overflow sub-buckets >= this many elements go to stream 2
    int ovf_inline_min = 0x7FFFFFFF; // overflow chains of >= this many samples run inline
    int inline_prio = 3;
    int ovf_long_class = 14;         // chains of >= 2^class samples leave the pass (chain streams)
    int main_long_class = 14;
    int ovf_chain_wgs = 0;
    int chain_prio = 0;
    int bucket_prio = 0;
    int chain_lds_kb = 0;
    int host_timing = 0;
    int heavy_min = (int)HEAVY_MIN;  // occurrences that make a key heavy (k_ovf_split)
    int split_min = (int)SPLIT_MIN;  // overflow sub-buckets of at least this size are split
    // heavy chains of >= 2^class samples start right after k_heavy on rotating chain streams
    // (0: off; -1, the default: 14 with one pass, off with key-range passes -- measured at C3, the
    // FP64-bound chains running beside the pass kernels slow them by more than the tail they
    // would hide; giant_class())
    int giant_class = -1;
    int giant_passes = 0;            // giant chains only in the last N passes (0: all)
    int prefetch = 1;                // next pass group's positions (k_pass_emit) during this group-by
    int heavy_grid = (int)HEAVY_GRID; // persistent grids: k_heavy,
    int ovf_grid = 1024;             //   k_overflow (per stream),
    int split_grid = 512;            //   k_ovf_split,
    int chain_grid = 4096;           //   k_chains
    int stream_prio = 0;             // 1: the group-by stream at the highest priority
    // key-range passes: stashed long chains leave in this many batches.  Round 6 (C3, one box,
    // after the staging stopped re-reading the residues): 2 -> 1404-1426 ms/step, chain tail 11 ms;
    // 4 -> 1536-1541 ms, tail 92-105 ms (the batch flushed after pass 11 still ran when the last
    // pass ended); 1 -> 1835 ms; 8 -> 2464 ms
    int chain_batches = 2;
    int chain_streams = 1;           //   over this many streams (1..4)
    int poison_jobs = 0;             // tests: every slot of the run's long-job list starts as a canary job
    int route_vacate = 0;            // routing: the last this many passes hold no heavy key (0: half)
    // routing: pass 0 holds only the heavy keys, so their chains start a heavy-only pass into the
    // step (-1, the default: on at world > 1, where one or two passes per rank would otherwise
    // start the heaviest chain half a step in -- the pass count is doubled below four passes;
    // 0: off; 1: on)
    // key-range passes on one GPU: a pass's tail (k_big_groups, the group-by's chains, the pass
    // accounting) runs on its own stream beside the next pass's staging, which writes a buffer of
    // its own (the split waits for the tail: it overwrites the slots the tail reads)
    int tail_async = 1;
    int big_grid = 2048;             // k_big_groups' persistent grids: groups of 65..1024 members,
    int big_grid_large = 512;        //   and of 1025..CAP
    // tail_async: the 1025..CAP class on a second tail stream.  Measured slower at C3 (round 6,
    // one box: 1445 / 1474 vs 1391 / 1429 ms/step): the concurrent classes slow the chains after them
    int big_split = 0;
    // tail_async: the tail is issued after the next pass's scan kernels (k_colsum .. k_stage_init),
    // which otherwise wait ~2 ms per pass behind k_big_groups' persistent grid for their workgroups.
    // Within noise at C3 (round 6, one box: 1434 / 1387 vs 1414 / 1377 ms/step): the scan's 25 ms
    // per step go, the tail then slows the staging more
    int tail_defer = 0;
    int part_order = 1;              // k_partition: the buckets of > 2x the mean size first (k_part_order)
    // part_order: those buckets by 1024-thread workgroups on stream 2, beside the rest.  Within noise
    // at C3 (round 6, one box, three alternations: 1353 / 1378 / 1378 vs 1374 / 1371 / 1353 ms/step):
    // the heavy buckets' workgroups stay as long, now beside the rest
    int part_split = 0;
    // tail_async: the split writes the pass's elements into one of two element buffers by pass
    // parity, so the next pass's split no longer waits for this pass's tail (which reads them);
    // the wait moves to the partition.  Costs 16 B per element of the largest pass (when it fits
    // beside a kept arena of a quarter of the valid windows).  With tail_defer, within noise at C3
    // (1396 / 1405 vs 1414 / 1377 ms/step): the device is busy either way, the tail's work moves
    int recs_rot = 0;
    int emit_group = 0;              // key-range passes emitted per residue scan (0: 4; 1, 2, 4, 8 or 16)
    int route_first = -1;
    int route_first_min = 1 << 17;   // route_first: k-mers of >= this many occurrences make pass 0 (C3: ~4.5 %
                                     //   of the windows; those of >= 2^14 hold ~17 %, too many for a short pass)
    int route_heavy_min = 1 << 14;   // key-range passes: k-mers of >= this many occurrences are routed into
                                     //   the first half of the passes (0: off; k_pass_ids)
    int overlap = 0;                 // key-range passes, one GPU: pipelined passes (a second element set)
    int chain_cus = 0;               // CUs of the long-chain stream (0: all; set_option recreates it)
    int side_cus = 0;                // CUs of the overflow and selection streams (0: all)
    int serial_overflow = 0;         // diagnostics: 1 = the overflow path starts after the group-by kernel
    int flag_check = 0;              // 1: k_bucket_process reads a signature flag before storing it
    int partition_round = 0;         // k_partition staging rounds: 0 = 2048 elements (three 512-thread
                                     //   workgroups per CU), 1 = 4096 (one), 2 = 4096 (one of 1024 threads)
    int stage_round = 1;             // key-range passes: 1 = the staged position scatter in half rounds
                                     //   (2048 elements, four workgroups per CU); 0 = full rounds
    // key-range passes: stashed long chains below this many samples run one lane each (k_chains,
    // 64 chains per wave) instead of on a wave pair, except the batch after the last pass (0: off).
    // Measured at C3: 1.91 -> 1.70-1.73 s/step -- the wave pairs held ~4 k waves resident for the
    // whole batch, and a k_bucket_process workgroup needs half of a CU's registers and LDS
    int lane_long = 1 << 20;
    int lane_grid = 256;             //   their k_chains grid
    int chain_queue = 0;             // k_chains: waves take 64-job blocks from a queue (0: strided)
    int lane_streams = 1;            //   the streams their batches rotate over (1..4)
    int lane_tail = 1 << 16;         //   the last batch's threshold (its wave pairs are the tail's latency)
    int sub_target = 0;              // k_partition's target elements per level-2 sub-bucket (0: SUB_TARGET)
    int heavy_lsd = 0;               // 1: k_heavy's round-3 path (Boyer-Moore + recount, LSD sort, length
                                     //   gathers) for every key instead of the one-read bucketed path
    int flag_bits = 1;               // signature flags as bits, read before an atomic set (mark_seq);
                                     //   0: a byte store per kept occurrence (C3: +58 ms/step)
    int diag = 0;                    // diagnostics only (wrong results): 1 = no signature flag stores,
                                     //   2 = k_heavy without its sequence-index sort, 4 = no chain kernels,
                                     //   8 = no stashed long chains, 16 = no per-pass k_chains,
                                     //   32 / 64 = k_overflow skips its entries of <= / > CAP elements
    int handoff_index_limit = 0;     // tests: finish hand-offs of >= this many k-mers take u64 arena
                                     //   indices (0: 2^32, where they are needed)
    int handoff_max_chunk = 0;       // tests: cap on the hand-off's chunk size (0: memory-planned)
};

}  // namespace skm

// ==========================================================================================
// Host side
// ==========================================================================================
using namespace skm;

struct ChainSet {            // job sort scratch + sorted jobs of one chain launch
    DevBuf hist, offs, sorted, long_off;
};

struct skm_build {
    skm_build_opts opts{};
    int device = 0;
    hipStream_t stream = nullptr;
    // timing events, one set per key-range pass (read after the step's single host sync)
    struct EvSet {
        hipEvent_t ev[13] = {}, o[3] = {}, o3[3] = {};
    };
    std::deque<EvSet> evsets;
    hipEvent_t* ev = nullptr;           // the current pass's set
    hipEvent_t* ev_o = nullptr;
    hipEvent_t* ev_o3 = nullptr;
    float last_ms[15] = {};
    uint64_t ovf_elems = 0, ovf_kept = 0;

    // host staging (reference emission order, only sequences with a kept function)
    // residues stream to HBM as batches arrive: packed (one 0 separator after each sequence) into
    // two pinned staging buffers that alternate -- the host fills one while the DMA engine copies
    // the other (section 8(f)4); prepare only flushes the last one
    uint8_t* st_pin[2] = {};
    size_t st_fill[2] = {};
    hipEvent_t st_ev[2] = {};
    bool st_busy[2] = {};
    int st_cur = 0;
    uint64_t rp_total = 0;          // residues packed so far (incl. separators)
    uint64_t rp_dev = 0;            // bytes of them issued to the device
    uint64_t res_cap = 0;           // d_res capacity
    std::vector<SeqMeta> h_meta;
    std::vector<uint32_t> h_seqid;
    std::unique_ptr<HostPool> pool;     // host threads of the packing (add_batch) and the hand-off copies
    HandoffStats handoff;               // the last finish's kept-set hand-off (skm_output.hip)
    std::vector<uint32_t> h_keep;       // add_batch scratch: the batch's kept sequences, their offsets
    std::vector<uint64_t> h_cum;
    // host seconds in add_batch (all calls), and prepare's phases: the residue / metadata upload, the
    // pass plan (the pass tallies and the routing sketch: device work), the allocations and the rest
    double add_s = 0, add_pack_s = 0, add_wait_s = 0, prep_upload_s = 0, prep_plan_s = 0, prep_rest_s = 0;
    uint64_t n_windows = 0;
    bool seqid_strict = true;
    bool prepared = false, ran = false;

    // device input
    DevBuf d_res, d_meta, d_blk2seq, d_glen;
    uint64_t rp = 0;       // packed length
    uint32_t nseq = 0;
    // geometry / ranks
    int world = 1, rank = 0;
    int owner_bits = 0, b1_bits = 12;
    uint32_t s_base = 0;   // global index of this shard's first sequence
    uint32_t n_total = 0;  // sequences over all ranks
    std::vector<uint32_t> g_seqid;  // world > 1: all ranks' seq ids in global order (finish)
    bool g_strict = true;
    // device work
    DevBuf d_hist, d_offs, d_partial, d_rbbase, d_bstart32, d_bstart, d_owner_start;
    DevBuf d_recs_hi, d_recs_lo, d_tmp_hi, d_tmp_lo;
    DevBuf d_stg_hi, d_stg_lo;          // tail_async: the level-0 staging (else tmp holds it)
    DevBuf d_part_order;                // k_part_order's workgroup -> bucket map
    DevBuf d_cur0, d_cur1, d_slices;   // staged scatter cursors
    DevBuf d_flagbits;
    DevBuf d_chainq;              // k_chains work queues: two counters per launch of a run
    uint32_t chainq_next = 0;
    DevBuf d_keys, d_data, d_ctr, d_flags, d_dfunc, d_swf, d_ovf, d_ovf_hi, d_ovf_lo, d_ovf_heads, d_ovf_job, d_ovf_fm;
    DevBuf d_jobs, d_lens, d_stamps, d_big_desc, d_big_out;
    uint64_t big_cap = 0, n_big = 0, big_kept = 0;
    bool stamps = false;
    uint64_t jobs_cap = 0, lens_cap = 0, n_jobs = 0, n_lens = 0;
    uint32_t n_overflow = 0, n_overflow_last = 0;
    uint32_t nwg = 0;
    uint64_t span = 0;
    uint64_t n_kept = 0;
    uint64_t ovf_cap = 0;

    // world > 1: owner-partitioned exchange
    DevBuf d_rhi, d_rlo;                 // received elements, [source rank][level-1 bucket]
    DevBuf d_cnt_send, d_cnt_recv;       // [world][NB1] element counts
    DevBuf d_seg_start, d_seg_len, d_vstart;
    // elements this rank sends to / receives from each peer in each pass ([pass][peer], exchanged
    // at prepare: pass_peer_counts), their device copy (sends, then receives) for the checks
    std::vector<uint64_t> xs_send, xs_recv;
    DevBuf d_xs;
    uint64_t n_local_max = 0;            // the largest pass's received elements
    uint64_t n_local = 0;                // elements this rank groups (received, or extracted at world 1)
    uint64_t cap_local = 0;

    // transport: RCCL communicator, or the in-process rank group used by the tests
#if defined(SKM_WITH_RCCL)
    ncclComm_t comm = nullptr;
#endif
    std::vector<skm_build*> group;
    skm_transport tp{};                   // host transport (tp.alltoallv != nullptr)

    // second stream: overflow sub-buckets + their chains, concurrent with the group-by
    hipStream_t stream2 = nullptr, stream3 = nullptr;
    hipStream_t stream_tail = nullptr;  // tail_async: a pass's big groups, main chains and accounting
    hipStream_t stream_tail2 = nullptr; //   the groups of 1025..CAP members beside the smaller big groups
    hipEvent_t ev_tail_bp = nullptr, ev_tail_done = nullptr, ev_tail2 = nullptr;
    bool tail_pending = false;          // the last pass's tail is still in flight on stream_tail
    std::function<void()> tail_issue;   // tail_defer: the last pass's tail, not yet issued
    hipEvent_t ev_scan = nullptr;       // tail_defer: the next pass's scan kernels are done
    bool rot = false;                   // recs_rot: odd passes split into d_recs_*2
    uint64_t free_after_prepare = 0;    // device bytes free after prepare (counters [44])
    hipEvent_t ev_part = nullptr, ev_split = nullptr, ev_part_heavy = nullptr;
    DevBuf d_hv_keys, d_hv_rec, d_hv_len, d_hv_s0, d_hv_s1;   // heavy keys of the split overflow
    DevBuf d_sub_tab, d_jobs2, d_jobs3;

    // pinned host staging for the pipeline's small readbacks
    unsigned long long* h_pin = nullptr;   // [128] counters and run slots
    OvfEntry* h_ovf = nullptr;
    size_t h_ovf_cap = 0;
    unsigned long long* pinned_ctr() {
        if (!h_pin) SKM_HIP(hipHostMalloc(reinterpret_cast<void**>(&h_pin), 128 * 8, hipHostMallocDefault));
        return h_pin;
    }
    OvfEntry* pinned_ovf(size_t n) {
        if (n > h_ovf_cap) {
            if (h_ovf) SKM_HIP(hipHostFree(h_ovf));
            h_ovf = nullptr;
            h_ovf_cap = std::max<size_t>(n, 1024);
            SKM_HIP(hipHostMalloc(reinterpret_cast<void**>(&h_ovf), sizeof(OvfEntry) * h_ovf_cap, hipHostMallocDefault));
        }
        return h_ovf;
    }

    uint64_t jobs2_cap = 0;
    ChainSet cs_main, cs_ovf, cs_ovf3;
    uint32_t n_ovf_heavy = 0;

    // key-range passes (out-of-core build): P = 2^pass_bits passes over disjoint k-mer ranges
    int pass_bits = 0;
    uint64_t pass_max = 0;              // valid windows of the largest pass (this shard)
    uint64_t valid_total = 0;           // valid windows of this shard
    DevBuf d_ids;                       // per-window pass id (pass_bits > 0; k_pass_ids, once per run)
    DevBuf d_bloom;                     // heavy-key routing filter (route)
    std::vector<uint64_t> cnt64;        // valid windows by the top 6 hash bits (size_passes)
    bool route = false;
    bool route_first = false;           // routing into a heavy-only pass 0 (route_plan; every rank alike)
    uint64_t routed = 0;                // occurrences routed into the first half of the passes (or pass 0)
    // the window positions and level-1 histograms of a group of emit_g passes (k_pass_emit: one
    // residue scan per group), in emit_g slots; the next group's scan runs on stx once the group's
    // last pass has staged its elements (ev_staged), beside that pass's group-by
    DevBuf d_posg, d_histg, d_npos;      // d_npos: every pass's window count (k_sel_scan)
    uint32_t emit_g = 1;
    DevBuf d_selrows, d_seloff;          // per-workgroup windows of each pass, their scanned offsets
    uint64_t sel_span = 0;               // windows per k_pass_ids / k_pass_emit workgroup (< 2^REL_BITS)
    uint32_t sel_wg = SEL_WG;            // k_pass_ids / k_pass_emit workgroups (tally rows)
    hipStream_t stx = nullptr;
    hipEvent_t ev_staged = nullptr, ev_emit = nullptr;
    // pipelined passes (option overlap, one GPU, key-range passes): a second element buffer set,
    // so that a pass's overflow path (streams 2/3, reading its buffers) overlaps the next pass's
    // extract / split / partition instead of closing the pass; per-set counter blocks, plans and
    // overflow lists; ev_ovf_done[k] = the overflow path (and the pass accounting) of the last
    // pass that used set k is complete, ev_main_done[k] = its main-stream work is
    bool overlap = false;
    DevBuf d_recs_hi2, d_recs_lo2, d_tmp_hi2, d_tmp_lo2, d_ovf2b;
    hipEvent_t ev_ovf_done[2] = {}, ev_main_done[2] = {};
    bool ovf_pending[2] = {false, false};
    int64_t emit_q = -1;                // the group whose scan is queued on stx
    uint32_t pf_nwg = 1;                // count-kernel rows of the histogram matrix (pass mode)
    uint64_t pf_span = 0;
    uint64_t kept_cap = 0;              // kept k-mer arena (keys + records), shared by all passes
    hipEvent_t ev_start = nullptr;
    // run totals over the passes (counters(), timings)
    struct Acc {
        uint64_t novf, jobs, lens, ovf_elems, ovf_kept, big, big_kept, grouped;
    } acc{};
    float pass_ms[12] = {};
    skm::Tune tune;
    // key-range passes: the long chains leave their pass (stashed samples, run-level job list) and
    // run in batches on a fourth stream (mid-run and at the end), overlapping the later passes
    hipStream_t chain_st = nullptr;
    hipEvent_t chain_ev[3] = {};
    // stashed long chains below tune.lane_long samples: one lane each (k_chains) on their own stream
    static constexpr int LANE_ST = 4;  // batches rotate over tune.lane_streams of them
    hipStream_t lane_st[LANE_ST] = {};
    hipEvent_t lane_ev[LANE_ST] = {};
    bool lane_used[LANE_ST] = {};
    // giant chains of k_heavy: rotating slots (stream, sample / job buffers, counters, events)
    static constexpr int GSLOTS = 3;  // + st, st2, st3, chain_st, stx: 8 streams
    hipStream_t gst[GSLOTS] = {};
    hipEvent_t gev_ready[GSLOTS] = {}, gev_done[GSLOTS] = {};
    std::deque<DevBuf> gsamples, gjobs, gcount;   // per key-range pass (reused by the next run)
    bool gused[GSLOTS] = {};
    bool chain_used[GSLOTS + 1] = {};   // long-chain batches issued on chain_stream(k) this run
    DevBuf d_gstat;                      // run totals: giant chains, longest giant chain
    uint64_t giant_jobs = 0, giant_max = 0;
    DevBuf d_long_arena;                 // stashed samples of the run's long chains
    DevBuf d_long_jobs;                  // run-level list of stashed long jobs (device addresses)
    uint64_t long_jobs_cap = 0;
    // device-side pass control: the overflow plan (sorted list, per-pass plan) and the run slots
    DevBuf d_ovf2, d_plan, d_run;
    // capacities of the data-dependent work buffers (alloc_caps), grown to a run's demand
    uint64_t tot_cap = 0, split_cap = 0, long_cap = 0;
    uint64_t run_flags = 0, demand[4] = {}, n_jobs_last = 0, n_redo = 0;
    uint64_t long_samples = 0;          // samples of the stashed long chains (last run)
    // per-kernel device time (skm_build_set_kernel_timing): an event pair around every launch of
    // the run (or of one kernel), summed by kernel name after the step's host synchronisation
    int kt_mode = 0;
    std::string kt_only;
    std::vector<hipEvent_t> kt_pool;
    size_t kt_used = 0;
    struct KtRec {
        const char* name;
        size_t e0;
    };
    std::vector<KtRec> kt_recs;
    std::vector<std::string> kt_names;  // last run: kernel names, total ms, launches
    std::vector<double> kt_ms;
    std::vector<uint64_t> kt_n;
    // the long-chain tail: from the end of the last pass on the group-by stream to the last chain
    hipEvent_t ev_tail[2] = {};
    hipEvent_t ev_giant[2] = {};        // the run's first giant-chain launch: start, end (timings [13], [14])
    bool giant_timed = false;
};

namespace {

// SKM_LAUNCH: hipLaunchKernelGGL with the launch bracketed by an event pair when kernel timing is
// on for this kernel (skm_build_set_kernel_timing); otherwise exactly the launch
int kt_begin(skm_build* b, const char* name, hipStream_t st) {
    if (!b->kt_mode || (!b->kt_only.empty() && b->kt_only != name)) return -1;
    while (b->kt_pool.size() < b->kt_used + 2) {
        hipEvent_t e;
        SKM_HIP(hipEventCreate(&e));
        b->kt_pool.push_back(e);
    }
    const size_t e0 = b->kt_used;
    b->kt_used += 2;
    SKM_HIP(hipEventRecord(b->kt_pool[e0], st));
    b->kt_recs.push_back({name, e0});
    return (int)e0;
}
void kt_end(skm_build* b, int e0, hipStream_t st) {
    if (e0 >= 0) SKM_HIP(hipEventRecord(b->kt_pool[(size_t)e0 + 1], st));
}
#define SKM_LAUNCH(B, K, G, BL, LDS, ST, ...)                   \
    do {                                                        \
        const int _kt = kt_begin((B), #K, (ST));                \
        hipLaunchKernelGGL(K, G, BL, LDS, ST, __VA_ARGS__);     \
        kt_end((B), _kt, (ST));                                 \
    } while (0)
// the same, timed under an explicit name (template instantiations sharing one table row)
#define SKM_LAUNCH_AS(B, NAME, K, G, BL, LDS, ST, ...)          \
    do {                                                        \
        const int _kt = kt_begin((B), NAME, (ST));              \
        hipLaunchKernelGGL(K, G, BL, LDS, ST, __VA_ARGS__);     \
        kt_end((B), _kt, (ST));                                 \
    } while (0)

// after the step's synchronisation: per-kernel totals of the run
void kt_collect(skm_build* b) {
    b->kt_names.clear();
    b->kt_ms.clear();
    b->kt_n.clear();
    for (const auto& r : b->kt_recs) {
        float t = 0.f;
        SKM_HIP(hipEventElapsedTime(&t, b->kt_pool[r.e0], b->kt_pool[r.e0 + 1]));
        size_t k = 0;
        while (k < b->kt_names.size() && b->kt_names[k] != r.name) ++k;
        if (k == b->kt_names.size()) {
            b->kt_names.emplace_back(r.name);
            b->kt_ms.push_back(0.0);
            b->kt_n.push_back(0);
        }
        b->kt_ms[k] += t;
        b->kt_n[k] += 1;
    }
}

__global__ void k_abs_starts(const uint32_t* rel, const uint64_t* ost, uint32_t NB, int b1_bits, uint32_t nowners,
                             uint64_t* out) {
    uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < NB) out[k] = ost[k >> b1_bits] + rel[k];
    if (k == NB) out[NB] = ost[nowners];
}

// ------------------------------------------------------------------------------------------
// Collectives over the ranks of one build.  `bs` lists the handles this process drives: {b}
// with an RCCL communicator (one process per GPU), or every rank of an in-process group
// (skm_build_group_run; the exchange is then plain device copies).  All are stream-ordered on
// each handle's stream; the group form synchronises around each step.
// ------------------------------------------------------------------------------------------
using Ranks = std::vector<skm_build*>;

bool is_group(const Ranks& bs) { return bs.size() > 1 || (bs[0]->world > 1 && !bs[0]->group.empty()); }

void sync_all(const Ranks& bs) {
    for (auto* b : bs) SKM_HIP(hipStreamSynchronize(b->stream));
}

#if defined(SKM_WITH_RCCL)
#define SKM_NCCL(x)                                                                              \
    do {                                                                                         \
        ncclResult_t _r = (x);                                                                   \
        if (_r != ncclSuccess) throw skm::Error(SKM_E_COMM, std::string("RCCL: ") + ncclGetErrorString(_r)); \
    } while (0)
#endif

bool has_tp(const Ranks& bs) { return bs.size() == 1 && bs[0]->world > 1 && bs[0]->tp.alltoallv != nullptr; }

void tp_check(int rc, const char* what) {
    SKM_CHECK(rc == 0, SKM_E_COMM, std::string("host transport ") + what + " failed");
}

// Exchange planning of one pass (pure host arithmetic).  Send side: from the owner-major bucket
// starts, per-bucket counts (the all-to-all payload) and each peer's contiguous element range.
struct SendPlan {
    std::vector<uint32_t> cnt;        // [W * NB1]
    std::vector<uint64_t> off, n;     // [W] elements
};
SendPlan plan_send(const uint64_t* abs, int W, uint32_t NB1) {
    SendPlan p;
    const uint64_t NB = (uint64_t)NB1 * W;
    p.cnt.resize(NB);
    for (uint64_t k = 0; k < NB; ++k) p.cnt[k] = (uint32_t)(abs[k + 1] - abs[k]);
    p.off.assign(W, 0);
    p.n.assign(W, 0);
    for (int q = 0; q < W; ++q) {
        p.off[q] = abs[(uint64_t)q * NB1];
        p.n[q] = abs[(uint64_t)(q + 1) * NB1] - abs[(uint64_t)q * NB1];
    }
    return p;
}
// Receive side, from the received counts [source][bucket]: source-major pieces in the receive
// buffer, and the bucket-major virtual numbering the partition kernel uses for tmp.
struct RecvPlan {
    std::vector<uint64_t> off, n;         // [W] elements per source
    std::vector<uint64_t> seg_start;      // [W * NB1]
    std::vector<uint32_t> seg_len;        // [W * NB1]
    std::vector<uint64_t> vstart;         // [NB1 + 1]
    uint64_t total = 0;
};
RecvPlan plan_recv(const uint32_t* rc, int W, uint32_t NB1) {
    RecvPlan p;
    const uint64_t NB = (uint64_t)NB1 * W;
    p.off.assign(W, 0);
    p.n.assign(W, 0);
    p.seg_start.resize(NB);
    p.seg_len.resize(NB);
    p.vstart.assign(NB1 + 1, 0);
    std::vector<uint64_t> bucket_tot(NB1, 0);
    uint64_t run = 0;
    for (int s = 0; s < W; ++s) {
        p.off[s] = run;
        for (uint32_t k = 0; k < NB1; ++k) {
            const uint32_t c = rc[(uint64_t)s * NB1 + k];
            p.seg_start[(uint64_t)s * NB1 + k] = run;
            p.seg_len[(uint64_t)s * NB1 + k] = c;
            bucket_tot[k] += c;
            run += c;
        }
        p.n[s] = run - p.off[s];
    }
    for (uint32_t k = 0; k < NB1; ++k) p.vstart[k + 1] = p.vstart[k] + bucket_tot[k];
    p.total = run;
    return p;
}

// host-transport all-to-all of host buffers with byte offsets/counts per peer (packed staging)
void tp_alltoallv_host(const skm_transport& tp, int W, const uint8_t* send, const std::vector<uint64_t>& soff,
                       const std::vector<uint64_t>& scnt, uint8_t* recv, const std::vector<uint64_t>& roff,
                       const std::vector<uint64_t>& rcnt) {
    tp_check(tp.alltoallv(tp.ctx, send, scnt.data(), soff.data(), recv, rcnt.data(), roff.data()), "alltoallv");
    (void)W;
}

// all-to-all with variable counts: rank p sends send[p] + soff[p][q] (scnt[p][q] bytes) to rank q,
// which receives it at recv[q] + roff[q][p].
struct A2A {
    std::vector<const uint8_t*> send;
    std::vector<uint8_t*> recv;
    std::vector<std::vector<uint64_t>> soff, scnt, roff, rcnt;  // bytes, [local handle][peer]
};

void alltoallv(const Ranks& bs, const A2A& x) {
    if (has_tp(bs)) {  // device -> packed host staging -> caller's channel -> device
        skm_build* b = bs[0];
        const int W = b->world;
        std::vector<uint64_t> so(W), ro(W);
        uint64_t st = 0, rt = 0;
        for (int q = 0; q < W; ++q) {
            so[q] = st;
            st += x.scnt[0][q];
            ro[q] = rt;
            rt += x.rcnt[0][q];
        }
        std::vector<uint8_t> hs(std::max<uint64_t>(st, 1)), hr(std::max<uint64_t>(rt, 1));
        SKM_HIP(hipStreamSynchronize(b->stream));
        for (int q = 0; q < W; ++q)
            if (x.scnt[0][q]) SKM_HIP(hipMemcpy(hs.data() + so[q], x.send[0] + x.soff[0][q], x.scnt[0][q], hipMemcpyDeviceToHost));
        tp_alltoallv_host(b->tp, W, hs.data(), so, x.scnt[0], hr.data(), ro, x.rcnt[0]);
        for (int q = 0; q < W; ++q)
            if (x.rcnt[0][q]) SKM_HIP(hipMemcpy(x.recv[0] + x.roff[0][q], hr.data() + ro[q], x.rcnt[0][q], hipMemcpyHostToDevice));
        return;
    }
    if (is_group(bs)) {
        sync_all(bs);
        const size_t W = bs.size();
        for (size_t p = 0; p < W; ++p)
            for (size_t q = 0; q < W; ++q)
                if (x.scnt[p][q])
                    SKM_HIP(hipMemcpyAsync(x.recv[q] + x.roff[q][p], x.send[p] + x.soff[p][q], x.scnt[p][q],
                                           hipMemcpyDeviceToDevice, bs[q]->stream));
        sync_all(bs);
        return;
    }
#if defined(SKM_WITH_RCCL)
    skm_build* b = bs[0];
    const int W = b->world, me = b->rank;
    if (x.scnt[0][me])
        SKM_HIP(hipMemcpyAsync(x.recv[0] + x.roff[0][me], x.send[0] + x.soff[0][me], x.scnt[0][me],
                               hipMemcpyDeviceToDevice, b->stream));
    SKM_NCCL(ncclGroupStart());
    for (int q = 0; q < W; ++q) {
        if (q == me) continue;
        if (x.scnt[0][q]) SKM_NCCL(ncclSend(x.send[0] + x.soff[0][q], x.scnt[0][q], ncclUint8, q, b->comm, b->stream));
        if (x.rcnt[0][q]) SKM_NCCL(ncclRecv(x.recv[0] + x.roff[0][q], x.rcnt[0][q], ncclUint8, q, b->comm, b->stream));
    }
    SKM_NCCL(ncclGroupEnd());
#else
    throw Error(SKM_E_COMM, "libskm was built without RCCL");
#endif
}

// element-wise reduction of a device array across ranks (in place): u32 sum or u8 max
enum class Red { SumU32, MaxU8 };

void allreduce(const Ranks& bs, const std::vector<void*>& ptr, size_t count, Red op) {
    if (count == 0) return;
    if (has_tp(bs)) {
        skm_build* b = bs[0];
        const size_t es = op == Red::SumU32 ? 4 : 1;
        std::vector<uint8_t> h(count * es);
        SKM_HIP(hipStreamSynchronize(b->stream));
        SKM_HIP(hipMemcpy(h.data(), ptr[0], count * es, hipMemcpyDeviceToHost));
        tp_check(b->tp.allreduce(b->tp.ctx, h.data(), count, op == Red::SumU32 ? 0 : 1), "allreduce");
        SKM_HIP(hipMemcpy(ptr[0], h.data(), count * es, hipMemcpyHostToDevice));
        return;
    }
    if (is_group(bs)) {
        sync_all(bs);
        const size_t es = op == Red::SumU32 ? 4 : 1;
        std::vector<uint8_t> acc(count * es, 0), tmp(count * es);
        for (size_t r = 0; r < bs.size(); ++r) {
            SKM_HIP(hipMemcpy(tmp.data(), ptr[r], count * es, hipMemcpyDeviceToHost));
            if (op == Red::SumU32) {
                auto* a = reinterpret_cast<uint32_t*>(acc.data());
                auto* t = reinterpret_cast<const uint32_t*>(tmp.data());
                for (size_t i = 0; i < count; ++i) a[i] += t[i];
            } else {
                for (size_t i = 0; i < count; ++i) acc[i] = std::max(acc[i], tmp[i]);
            }
        }
        for (size_t r = 0; r < bs.size(); ++r) SKM_HIP(hipMemcpy(ptr[r], acc.data(), count * es, hipMemcpyHostToDevice));
        return;
    }
#if defined(SKM_WITH_RCCL)
    skm_build* b = bs[0];
    if (op == Red::SumU32)
        SKM_NCCL(ncclAllReduce(ptr[0], ptr[0], count, ncclUint32, ncclSum, b->comm, b->stream));
    else
        SKM_NCCL(ncclAllReduce(ptr[0], ptr[0], count, ncclUint8, ncclMax, b->comm, b->stream));
#else
    throw Error(SKM_E_COMM, "libskm was built without RCCL");
#endif
}

// gather one u64 per rank to every rank (host values)
std::vector<uint64_t> allgather_u64(const Ranks& bs, const std::vector<uint64_t>& mine) {
    if (has_tp(bs)) {
        skm_build* b = bs[0];
        std::vector<uint64_t> out(b->world), bytes(b->world, 8);
        tp_check(b->tp.allgatherv(b->tp.ctx, &mine[0], out.data(), bytes.data()), "allgatherv");
        return out;
    }
    if (is_group(bs)) return mine;  // one value per handle, already in rank order
#if defined(SKM_WITH_RCCL)
    skm_build* b = bs[0];
    DevBuf d;
    d.ensure(8 * (b->world + 1));
    SKM_HIP(hipMemcpyAsync(d.as<uint64_t>() + b->rank, &mine[0], 8, hipMemcpyHostToDevice, b->stream));
    SKM_NCCL(ncclAllGather(d.as<uint64_t>() + b->rank, d.p, 1, ncclUint64, b->comm, b->stream));
    std::vector<uint64_t> out(b->world);
    SKM_HIP(hipMemcpyAsync(out.data(), d.p, 8 * b->world, hipMemcpyDeviceToHost, b->stream));
    SKM_HIP(hipStreamSynchronize(b->stream));
    return out;
#else
    throw Error(SKM_E_COMM, "libskm was built without RCCL");
#endif
}

// every rank receives the rank-ordered concatenation of all ranks' device arrays
void allgatherv(const Ranks& bs, const std::vector<const void*>& src, const std::vector<void*>& dst,
                const std::vector<uint64_t>& bytes_per_rank) {
    const size_t W = bytes_per_rank.size();
    std::vector<uint64_t> off(W + 1, 0);
    for (size_t r = 0; r < W; ++r) off[r + 1] = off[r] + bytes_per_rank[r];
    if (has_tp(bs)) {
        skm_build* b = bs[0];
        std::vector<uint8_t> hs(std::max<uint64_t>(bytes_per_rank[b->rank], 1)), hr(std::max<uint64_t>(off[W], 1));
        SKM_HIP(hipStreamSynchronize(b->stream));
        if (bytes_per_rank[b->rank])
            SKM_HIP(hipMemcpy(hs.data(), src[0], bytes_per_rank[b->rank], hipMemcpyDeviceToHost));
        tp_check(b->tp.allgatherv(b->tp.ctx, hs.data(), hr.data(), bytes_per_rank.data()), "allgatherv");
        if (off[W]) SKM_HIP(hipMemcpy(dst[0], hr.data(), off[W], hipMemcpyHostToDevice));
        return;
    }
    if (is_group(bs)) {
        sync_all(bs);
        for (size_t q = 0; q < bs.size(); ++q)
            for (size_t r = 0; r < W; ++r)
                if (bytes_per_rank[r])
                    SKM_HIP(hipMemcpy(static_cast<uint8_t*>(dst[q]) + off[r], src[r], bytes_per_rank[r],
                                      hipMemcpyDeviceToDevice));
        return;
    }
#if defined(SKM_WITH_RCCL)
    skm_build* b = bs[0];
    SKM_NCCL(ncclGroupStart());
    for (int r = 0; r < b->world; ++r)
        if (bytes_per_rank[r])
            SKM_NCCL(ncclBroadcast(r == b->rank ? src[0] : nullptr, static_cast<uint8_t*>(dst[0]) + off[r],
                                   bytes_per_rank[r], ncclUint8, r, b->comm, b->stream));
    SKM_NCCL(ncclGroupEnd());
#else
    throw Error(SKM_E_COMM, "libskm was built without RCCL");
#endif
}

// ------------------------------------------------------------------------------------------
// prepare: pack + upload; with world > 1 also the global sequence numbering
// ------------------------------------------------------------------------------------------
void set_geometry(skm_build* b) {
    b->world = std::max(1, b->opts.world_size);
    b->rank = b->opts.rank;
    int ob = 0;
    while ((1 << ob) < b->world) ++ob;
    b->owner_bits = ob;
    // 4096 level-1 buckets in total (8192 from 4 ranks up); rem <= 31 bits leaves element bit 47
    // for the big-length flag
    const int total = 12 + (ob >= 2 ? 1 : 0);
    b->b1_bits = total - ob;
}

// ------------------------------------------------------------------------------------------
// Residue staging (pinned, double-buffered host -> HBM)
// ------------------------------------------------------------------------------------------
constexpr size_t STAGE_BYTES = 64ull << 20;

// d_res holds at least `need` bytes; growing keeps the bytes already uploaded (device copy)
void res_reserve(skm_build* b, uint64_t need) {
    if (need <= b->res_cap && b->d_res.p) return;
    const uint64_t cap = std::max<uint64_t>({need, b->res_cap + b->res_cap / 2, STAGE_BYTES});
    void* np = nullptr;
    SKM_HIP(hipMalloc(&np, cap));
    if (b->rp_dev) SKM_HIP(hipMemcpyAsync(np, b->d_res.p, b->rp_dev, hipMemcpyDeviceToDevice, b->stream));
    SKM_HIP(hipStreamSynchronize(b->stream));
    if (b->d_res.p) SKM_HIP(hipFree(b->d_res.p));
    b->d_res.p = np;
    b->d_res.bytes = cap;
    b->res_cap = cap;
}

// hand the current staging buffer to the DMA engine and switch to the other one (waiting only if
// its previous copy is still in flight)
void stage_flush(skm_build* b) {
    const int c = b->st_cur;
    if (b->st_fill[c]) {
        res_reserve(b, b->rp_dev + b->st_fill[c] + 64);
        SKM_HIP(hipMemcpyAsync(b->d_res.as<uint8_t>() + b->rp_dev, b->st_pin[c], b->st_fill[c], hipMemcpyHostToDevice,
                               b->stream));
        SKM_HIP(hipEventRecord(b->st_ev[c], b->stream));
        b->st_busy[c] = true;
        b->rp_dev += b->st_fill[c];
        b->st_fill[c] = 0;
    }
    b->st_cur ^= 1;
    const int n = b->st_cur;
    if (b->st_busy[n]) {
        const auto t0 = std::chrono::steady_clock::now();
        SKM_HIP(hipEventSynchronize(b->st_ev[n]));
        b->add_wait_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        b->st_busy[n] = false;
    }
    b->st_fill[n] = 0;
}

void prepare_local(skm_build* b) {
    SKM_HIP(hipSetDevice(b->device));
    set_geometry(b);
    stage_flush(b);  // the last staging buffer; the residues are then resident
    const uint64_t rp = b->rp_total;
    b->rp = rp;
    b->nseq = (uint32_t)b->h_meta.size();
    SKM_CHECK(b->h_meta.size() < (1ull << ELEM_S_BITS), SKM_E_ARG, "too many sequences in one build shard");
    res_reserve(b, rp + 64);
    SKM_HIP(hipMemsetAsync(b->d_res.as<uint8_t>() + rp, 0, 64, b->stream));  // window-load padding
    b->d_meta.ensure(sizeof(SeqMeta) * (b->nseq + 1));
    const SeqMeta sentinel{rp, 0, 0xFFFF, 0};  // the table, then its sentinel (no host copy of the table)
    if (b->nseq) SKM_HIP(hipMemcpy(b->d_meta.p, b->h_meta.data(), sizeof(SeqMeta) * b->nseq, hipMemcpyHostToDevice));
    SKM_HIP(hipMemcpy(b->d_meta.as<SeqMeta>() + b->nseq, &sentinel, sizeof(SeqMeta), hipMemcpyHostToDevice));
    const uint64_t nblk = (rp >> 6) + 1;
    b->d_blk2seq.ensure(sizeof(uint32_t) * nblk);
    SKM_HIP(hipMemsetAsync(b->d_blk2seq.p, 0, sizeof(uint32_t) * nblk, b->stream));
    if (b->nseq)
        hipLaunchKernelGGL(k_blk2seq, dim3((b->nseq + 255) / 256), dim3(256), 0, b->stream, b->d_meta.as<SeqMeta>(), b->nseq,
                           b->d_blk2seq.as<uint32_t>(), nblk);
    SKM_HIP(hipGetLastError());
    // extract geometry + work buffers
    const uint32_t NB = 1u << (b->owner_bits + b->b1_bits);
    uint64_t step = (uint64_t)EX_THREADS * EX_POS_PER_THREAD;
    uint64_t nwg = std::max<uint64_t>(1, std::min<uint64_t>(EX_MAX_WG, ceil_div(rp ? rp : 1, step)));
    b->span = ceil_div(ceil_div(rp ? rp : 1, nwg), step) * step;
    b->nwg = (uint32_t)ceil_div(rp ? rp : 1, b->span);
    const uint32_t nrb = (uint32_t)ceil_div(b->nwg, SCAN_ROWS);
    b->d_hist.ensure(sizeof(uint32_t) * (uint64_t)b->nwg * NB);
    b->d_offs.ensure(sizeof(uint32_t) * (uint64_t)b->nwg * NB);
    b->d_partial.ensure(sizeof(uint32_t) * (uint64_t)nrb * NB);
    b->d_rbbase.ensure(sizeof(uint32_t) * (uint64_t)nrb * NB);
    b->d_bstart32.ensure(sizeof(uint32_t) * (NB + 1));
    b->d_bstart.ensure(sizeof(uint64_t) * (NB + 1));
    b->d_owner_start.ensure(sizeof(uint64_t) * 80);
    b->d_ctr.ensure(3 * 256);
    b->d_dfunc.ensure(sizeof(uint32_t) * std::max<uint32_t>(b->opts.n_functions, 1));
    b->d_swf.ensure(sizeof(uint32_t) * std::max<uint32_t>(b->opts.n_functions, 1));
}

// Valid windows of this shard by the top 6 bits of mix43(key) (one scan), then the pass count:
// the smallest power of two whose largest pass fits the 32-bit element indexing and whose
// per-pass work buffers (~PASS_BYTES per element) leave room for the kept arena (18 B per kept
// k-mer, accumulated over all passes).
constexpr uint64_t PASS_BYTES = 104;   // recs 16 + tmp 16 + received 16 (world > 1) + chain lens/jobs ~10 + overflow scratch ~40
// HBM a shard's work buffers take for passes of at most m elements: PASS_BYTES per element, with
// key-range passes also the window-position slots of a pass group (8 B per element and slot,
// G = min(P, 4) slots, size_local) and the pass-id byte per residue.
// giant: giant chains on (giant_class), whose per-pass sample slots (alloc_caps: 4 B x giant_cap,
// giant_cap = min(split_cap ~ 5/16 of the pass, 2^28), and their job lists) count too.
inline uint64_t pass_work(uint64_t m, int pb, uint64_t rp, bool giant = false) {
    const uint64_t G = pb ? std::min<uint64_t>(1ull << pb, 4) : 0;
    const uint64_t gcap = std::min<uint64_t>(m / 16 * 5 + (1u << 15), 1ull << 28);
    const uint64_t gw = giant ? (1ull << pb) * (4 * gcap + sizeof(Job) * (gcap >> 10) + 4096) : 0;
    return m * (PASS_BYTES + 8 * G) + (pb ? rp : 0) + gw;
}
// the work buffers may take 5/8 of the budget; the kept arena (18 B per kept k-mer) and the
// grow-and-redo reserve share the rest
inline bool work_fits(uint64_t work, uint64_t budget) { return work <= budget / 8 * 5; }
// forced_pb >= 0: the pass count the ranks agreed on (prepare), which leaves the caller's
// key_range_passes option as it was set
void size_passes(skm_build* b, int forced_pb = -1) {
    DevBuf d_cnt;
    d_cnt.ensure(8 * 64);
    SKM_HIP(hipMemsetAsync(d_cnt.p, 0, 8 * 64, b->stream));
    if (b->rp)
        hipLaunchKernelGGL(k_pass_ids, dim3(1024), dim3(256), 4u * 64, b->stream, b->d_res.as<uint8_t>(), b->rp, 0, 0,
                           nullptr, d_cnt.as<unsigned long long>(), nullptr, 64u);
    SKM_HIP(hipGetLastError());
    uint64_t cnt[64];
    SKM_HIP(hipMemcpyAsync(cnt, d_cnt.p, sizeof(cnt), hipMemcpyDeviceToHost, b->stream));
    SKM_HIP(hipStreamSynchronize(b->stream));
    b->valid_total = 0;
    for (int i = 0; i < 64; ++i) b->valid_total += cnt[i];
    auto pass_max = [&](int pb) {
        uint64_t m = 0;
        const int per = 64 >> pb;
        for (int p = 0; p < (1 << pb); ++p) {
            uint64_t t = 0;
            for (int i = 0; i < per; ++i) t += cnt[p * per + i];
            m = std::max(m, t);
        }
        return m;
    };
    size_t fr = 0, tot = 0;
    SKM_HIP(hipMemGetInfo(&fr, &tot));
    const uint64_t budget = b->tune.mem_budget_mb > 0 ? (uint64_t)b->tune.mem_budget_mb << 20 : (uint64_t)fr;
    int pb = 0;
    if (forced_pb >= 0) {
        pb = forced_pb;
    } else if (b->tune.passes > 0) {
        while ((1 << pb) < b->tune.passes) ++pb;
    } else {
        // up to a quarter of the elements may sit in one pass's received buffer after the
        // exchange (skewed owners); 2^32 - 2^28 leaves the same slack for the 32-bit indexing
        while (pb < 6) {
            const uint64_t m = pass_max(pb);
            const bool giant = b->tune.giant_class > 0 || (b->tune.giant_class < 0 && (pb == 0 || b->world > 1));
            if (m < (1ull << 32) - (1ull << 28) && work_fits(pass_work(m, pb, b->rp, giant), budget)) break;
            ++pb;
        }
    }
    SKM_CHECK(pb <= 6, SKM_E_ARG, "key_range_passes must be a power of two <= 64");
    b->pass_bits = pb;
    b->pass_max = pass_max(pb);
    b->route = false;
    b->routed = 0;
    b->cnt64.assign(cnt, cnt + 64);
    SKM_CHECK(b->pass_max < (1ull << 32), SKM_E_ARG, "more than 2^32 occurrences in one pass of one GPU shard");
}

// buffers sized by the number of elements this rank groups in one pass
bool tail_async_on(const skm_build* b) { return b->tune.tail_async && b->world == 1 && b->pass_bits && !b->overlap; }

void ensure_local(skm_build* b, uint64_t n) {
    if (tail_async_on(b)) {  // within PASS_BYTES: the 16 B/element of the received set (world > 1) are free
        const uint64_t cs = std::max<uint64_t>(n + n / 16, 1);
        b->d_stg_hi.ensure(8 * cs);
        b->d_stg_lo.ensure(8 * cs);
    }
    if (n <= b->cap_local && b->cap_local) return;
    const uint64_t c = std::max<uint64_t>(n + n / 16, 1);
    if (b->world > 1) {
        b->d_rhi.ensure(8 * c);
        b->d_rlo.ensure(8 * c);
    }
    b->d_tmp_hi.ensure(8 * c);
    b->d_tmp_lo.ensure(8 * c);
    if (b->pass_bits == 0) {  // one pass: the kept arena never holds more than its elements
        b->d_keys.ensure(8 * c);
        b->d_data.ensure(sizeof(skm_stored_kmer_data) * c + 16);
        b->kept_cap = c;
    }
    const uint32_t NB1 = 1u << b->b1_bits;
    b->ovf_cap = c / CAP + NB1 + 16;
    b->jobs_cap = c / 3 + 16;
    b->lens_cap = c + 16;
    b->d_jobs.ensure(sizeof(Job) * b->jobs_cap);
    b->d_lens.ensure(sizeof(uint32_t) * b->lens_cap);
    b->d_ovf.ensure(sizeof(OvfEntry) * b->ovf_cap);
    b->big_cap = c / 65 + 64;  // groups of > 64 members
    b->d_big_desc.ensure(16 * b->big_cap);
    b->d_big_out.ensure(sizeof(BigOut) * b->big_cap);
    b->cap_local = c;
}

// extract buffers (one pass of this shard), the pass-id bytes, and with passes the kept arena
void size_local(skm_build* b) {
    const uint64_t W = std::max<uint64_t>(b->pass_max, 1);
    b->d_recs_hi.ensure(8 * W);
    b->d_recs_lo.ensure(8 * W);
    if (b->pass_bits > 0) {
        const uint32_t NB = 1u << (b->owner_bits + b->b1_bits);
        const uint32_t P = 1u << b->pass_bits;
        const uint32_t eg = b->tune.emit_group > 0 ? (uint32_t)b->tune.emit_group : 4u;
        b->emit_g = std::max<uint32_t>(1, std::min<uint32_t>(P, eg));
        b->d_posg.ensure(8 * W * b->emit_g);
        b->d_ids.ensure(((b->rp + 15) & ~15ull) + 64);
        SKM_HIP(hipMemsetAsync(b->d_ids.p, 0xFF, ((b->rp + 15) & ~15ull) + 64, b->stream));  // padding: no window
        b->d_histg.ensure(sizeof(uint32_t) * (uint64_t)NB * b->emit_g);
        b->d_npos.ensure(8ull * P);
        // rows of at most 2^REL_BITS - 16 residues: an entry keeps its window's offset in the row
        const uint64_t rmax = (1ull << REL_BITS) - 16;
        b->sel_wg = (uint32_t)std::max<uint64_t>(SEL_WG, ceil_div(std::max<uint64_t>(b->rp, 1), rmax));
        b->d_selrows.ensure(4ull * b->sel_wg * P);
        b->d_seloff.ensure(8ull * P * (b->sel_wg + 1));
        b->sel_span = ceil_div(ceil_div(std::max<uint64_t>(b->rp, 1), b->sel_wg), 16) * 16;
        SKM_CHECK(b->sel_span < (1ull << REL_BITS), SKM_E_STATE, "pass entry row span exceeds REL_BITS");
        // count-kernel geometry from the largest pass (the kernels read the pass's own count)
        // (the pass's histogram comes from k_pass_emit: this grid is the staged scatter's alone;
        // the half-round variant runs four workgroups per CU)
        const uint64_t stage_wg = b->tune.stage_round == 1 ? 4ull * EX_MAX_WG : EX_MAX_WG;
        uint32_t nwg = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(stage_wg, ceil_div(W, (uint64_t)SC_ROUND * 4)));
        b->pf_span = ceil_div(ceil_div(W, nwg), (uint64_t)SC_ROUND) * SC_ROUND;
        b->pf_nwg = (uint32_t)std::max<uint64_t>(1, ceil_div(W, b->pf_span));
        // the histogram matrix of a pass may use every extract workgroup row
        b->d_hist.ensure(sizeof(uint32_t) * (uint64_t)EX_MAX_WG * NB);
        b->d_offs.ensure(sizeof(uint32_t) * (uint64_t)EX_MAX_WG * NB);
        b->d_partial.ensure(sizeof(uint32_t) * (uint64_t)ceil_div(EX_MAX_WG, SCAN_ROWS) * NB);
        b->d_rbbase.ensure(sizeof(uint32_t) * (uint64_t)ceil_div(EX_MAX_WG, SCAN_ROWS) * NB);
    }
}

void size_arena(skm_build* b) {
    if (b->pass_bits == 0) return;
    size_t fr = 0, tot = 0;
    SKM_HIP(hipMemGetInfo(&fr, &tot));
    // the work buffers are allocated by now (alloc_caps); keep 32 B per element of the largest pass
    // in reserve for a redo that grows them (and for the received buffers at world > 1)
    const uint64_t reserve = b->pass_max * 32 + (1ull << 30);
    // a re-prepare (an option set after a run) reuses the arena it already holds: its bytes are
    // free for this plan too (counting them as used shrank the cap below the kept count)
    const uint64_t held = (uint64_t)b->d_keys.bytes + (uint64_t)b->d_data.bytes;
    const uint64_t avail = fr + held > reserve ? fr + held - reserve : 0;
    uint64_t cap = std::min<uint64_t>(b->valid_total + 16, avail / (8 + sizeof(skm_stored_kmer_data)));
    if (b->tune.mem_budget_mb > 0) {
        const uint64_t budget = (uint64_t)b->tune.mem_budget_mb << 20;
        const bool giant = b->tune.giant_class > 0 || (b->tune.giant_class < 0 && (b->pass_bits == 0 || b->world > 1));
        const uint64_t used = pass_work(b->pass_max, b->pass_bits, b->rp, giant);
        cap = std::min<uint64_t>(cap, budget > used ? (budget - used) / 18 : 0);
    }
    cap = std::max<uint64_t>(cap, b->pass_max + 16);
    b->d_keys.ensure(8 * cap);
    b->d_data.ensure(sizeof(skm_stored_kmer_data) * cap + 16);
    b->kept_cap = cap;
}

void alloc_caps(skm_build* b);
void pass_peer_counts(const Ranks& bs);

// the heavy-only first pass (option route_first): asked for by default at world > 1
bool route_first_on(const skm_build* b) {
    return b->tune.route_first > 0 || (b->tune.route_first < 0 && b->world > 1);
}
// k_pass_ids' routing argument: the vacated pass count, or ROUTE_FIRST (as route_plan agreed)
uint32_t route_arg(const skm_build* b) {
    return b->route_first ? ROUTE_FIRST : (uint32_t)std::max(0, b->tune.route_vacate);
}

// Heavy-key routing plan, after the ranks agreed on the pass count (one GPU: at least 4 passes;
// world > 1: at least 2).  Every rank sketches 1/64 of its windows into a count-min sketch; at
// world > 1 the sketches are summed over the ranks (all-reduce, 32 MB), so a key's estimate is
// its global occurrence count and every owner's first passes receive the same heavy keys.  The
// keys whose estimate reaches route_heavy_min / 64 (15 % slack) set their two filter bits; the
// ranks' filters are OR-ed (all-reduce max over bytes) and packed into the 64 KB bit filter
// k_pass_ids consults.  The routed pass sizes are then re-checked against the memory budget and
// the 32-bit slack the pass count was chosen for: a shard whose routed largest pass
// no longer fits turns routing off on every rank (the ranks must route alike).
void route_plan(const Ranks& bs) {
    skm_build* b0 = bs[0];
    int pb = b0->pass_bits;
    const int W = b0->world;
    for (auto* b : bs) {
        b->route = false;
        b->route_first = false;
        b->routed = 0;
    }
    // bit 0: route; bit 1: into a heavy-only pass 0 (from one pass up: the pass count is doubled)
    auto wish = [&](const skm_build* b) -> uint64_t {
        const bool first = route_first_on(b);
        if (b->tune.route_heavy_min <= 0 || pb < (first ? (W > 1 ? 1 : 0) : (W > 1 ? 1 : 2))) return 0u;
        return first ? 3u : 1u;
    };
    uint64_t want = 3u;
    {   // the options are per handle: route (first) only if every rank asks for it
        std::vector<uint64_t> mine(bs.size());
        for (size_t k = 0; k < bs.size(); ++k) mine[k] = wish(bs[k]);
        const std::vector<uint64_t> all = W > 1 ? allgather_u64(bs, mine) : mine;
        for (auto v : all) want &= v;
    }
    if (!(want & 1u)) return;
    const bool first = (want & 2u) != 0;
    const size_t ncms = 2ull << CMS_BITS, nbl = 1ull << BLOOM_BITS;
    std::vector<DevBuf> cms(bs.size()), bl8(bs.size());
    std::vector<void*> pc, pb8;
    for (size_t k = 0; k < bs.size(); ++k) {
        skm_build* b = bs[k];
        cms[k].ensure(4 * ncms);
        bl8[k].ensure(nbl);
        SKM_HIP(hipMemsetAsync(cms[k].p, 0, 4 * ncms, b->stream));
        SKM_HIP(hipMemsetAsync(bl8[k].p, 0, nbl, b->stream));
        if (b->rp)
            hipLaunchKernelGGL(k_route_sketch, dim3(2048), dim3(256), 0, b->stream, b->d_res.as<uint8_t>(), b->rp,
                               cms[k].as<uint32_t>(), 0u, nullptr);
        SKM_HIP(hipGetLastError());
        pc.push_back(cms[k].p);
        pb8.push_back(bl8[k].p);
    }
    if (W > 1) allreduce(bs, pc, ncms, Red::SumU32);
    for (size_t k = 0; k < bs.size(); ++k) {
        skm_build* b = bs[k];
        const uint64_t hmin = first ? (uint64_t)std::max(1, b->tune.route_first_min) : (uint64_t)b->tune.route_heavy_min;
        const uint32_t thresh = std::max<uint32_t>(8, (uint32_t)((hmin >> ROUTE_SAMPLE) * 85 / 100));
        if (b->rp)
            hipLaunchKernelGGL(k_route_sketch, dim3(2048), dim3(256), 0, b->stream, b->d_res.as<uint8_t>(), b->rp,
                               cms[k].as<uint32_t>(), thresh, bl8[k].as<uint8_t>());
        SKM_HIP(hipGetLastError());
    }
    if (W > 1) allreduce(bs, pb8, nbl, Red::MaxU8);
    for (size_t k = 0; k < bs.size(); ++k) {
        skm_build* b = bs[k];
        b->route_first = first;  // route_arg
        b->d_bloom.ensure(nbl / 8);
        hipLaunchKernelGGL(k_bloom_pack, dim3((uint32_t)(nbl / 32 + 255) / 256), dim3(256), 0, b->stream,
                           bl8[k].as<uint8_t>(), b->d_bloom.as<uint32_t>());
        SKM_HIP(hipGetLastError());
    }
    std::vector<uint64_t> ok(bs.size(), 1), heavy(bs.size(), 0);
    std::vector<uint64_t> routed_m(bs.size()), routed_n(bs.size());
    // the routed pass sizes of every shard at pass_bits pb
    auto count_routed = [&]() {
        for (size_t k = 0; k < bs.size(); ++k) {
            skm_build* b = bs[k];
            const uint32_t P = 1u << pb;
            DevBuf d_cnt;
            d_cnt.ensure(8 * 64);
            SKM_HIP(hipMemsetAsync(d_cnt.p, 0, 8 * 64, b->stream));
            if (b->rp)
                hipLaunchKernelGGL(k_pass_ids, dim3(1024), dim3(256), 4u * 64 + (uint32_t)(nbl / 8), b->stream,
                                   b->d_res.as<uint8_t>(), b->rp, pb, 0, nullptr, d_cnt.as<unsigned long long>(),
                                   b->d_bloom.as<uint32_t>(), 64u, nullptr, 0, route_arg(b));
            SKM_HIP(hipGetLastError());
            uint64_t cnt[64];
            SKM_HIP(hipMemcpyAsync(cnt, d_cnt.p, sizeof(cnt), hipMemcpyDeviceToHost, b->stream));
            SKM_HIP(hipStreamSynchronize(b->stream));
            const int R = b->tune.route_vacate > 0 ? std::min(b->tune.route_vacate, (int)P - 1) : (int)(P >> 1);
            uint64_t natural_late = 0, late = 0, m = 0;  // occurrences of the vacated passes before / after routing
            if (first) {
                natural_late = cnt[0];  // the heavy-only pass
            } else {
                for (int p = (int)P - R; p < (int)P; ++p) {
                    for (int i = 0; i < (64 >> pb); ++i) natural_late += b->cnt64[p * (64 >> pb) + i];
                    late += cnt[p];
                }
            }
            for (uint32_t p = 0; p < P; ++p) m = std::max<uint64_t>(m, cnt[p]);
            size_t fr = 0, tot = 0;
            SKM_HIP(hipMemGetInfo(&fr, &tot));
            const uint64_t budget = b->tune.mem_budget_mb > 0 ? (uint64_t)b->tune.mem_budget_mb << 20 : (uint64_t)fr;
            const bool forced = b->tune.passes > 0;
            const bool giant = b->tune.giant_class > 0 || (b->tune.giant_class < 0 && (pb == 0 || b->world > 1));
            ok[k] = m < (1ull << 32) - (1ull << 28) &&
                    (forced || m <= b->pass_max || work_fits(pass_work(m, pb, b->rp, giant), budget));
            routed_m[k] = m;
            routed_n[k] = natural_late - late;
            heavy[k] = first ? cnt[0] : 0;
        }
    };
    auto turn_off = [&]() {
        for (auto* b : bs) b->route_first = false;
    };
    count_routed();
    if (first) {
        // no heavy key on any rank: no heavy-only pass (and no routing)
        const std::vector<uint64_t> all = W > 1 ? allgather_u64(bs, heavy) : heavy;
        uint64_t any = 0;
        for (auto v : all) any |= v;
        if (!any) return turn_off();
        // below four passes the light keys of pass 0 would crowd one pass: twice the passes
        // (size_passes re-counts; the forced pass count of the option stands)
        if (pb < 2 && b0->tune.passes <= 0 && pb < 6) {
            ++pb;
            for (auto* b : bs) {
                size_passes(b, pb);
                b->route_first = true;
            }
            count_routed();
        }
        // a forced single pass stays one pass: with no pass bits k_pass_ids routes nothing, so
        // routing is off and the routed counter stays 0
        if (pb == 0) return turn_off();
    }
    {
        const std::vector<uint64_t> all = W > 1 ? allgather_u64(bs, ok) : ok;
        for (auto v : all)
            if (!v) return turn_off();  // routing off on every rank: the unrouted pass sizes stand
    }
    for (size_t k = 0; k < bs.size(); ++k) {
        bs[k]->pass_max = routed_m[k];
        bs[k]->routed = routed_n[k];
        bs[k]->route = true;
    }
}

void prepare(const Ranks& bs) {
    bool need = false;
    for (auto* b : bs) need |= !b->prepared;
    if (!need) return;
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    for (auto* b : bs) prepare_local(b);
    for (auto* b : bs) SKM_HIP(hipStreamSynchronize(b->stream));
    const auto t1 = clk::now();
    for (auto* b : bs) size_passes(b);
    {   // every rank runs the same passes
        std::vector<uint64_t> mine;
        for (auto* b : bs) mine.push_back((uint64_t)b->pass_bits);
        const std::vector<uint64_t> all = bs[0]->world > 1 ? allgather_u64(bs, mine) : mine;
        uint64_t pb = 0;
        for (auto v : all) pb = std::max(pb, v);
        for (auto* b : bs)
            if ((uint64_t)b->pass_bits != pb) size_passes(b, (int)pb);
        route_plan(bs);
        for (auto* b : bs) SKM_HIP(hipStreamSynchronize(b->stream));
    }
    const auto t2 = clk::now();
    for (auto* b : bs) {
        b->prep_upload_s = std::chrono::duration<double>(t1 - t0).count();
        b->prep_plan_s = std::chrono::duration<double>(t2 - t1).count();
    }
    for (auto* b : bs) size_local(b);
    skm_build* b0 = bs[0];
    if (b0->world == 1) {
        b0->s_base = 0;
        b0->n_total = b0->nseq;
        b0->d_glen.ensure(4 * (b0->nseq + 1));
        std::vector<uint32_t> len(b0->nseq);
        for (uint32_t s = 0; s < b0->nseq; ++s) len[s] = b0->h_meta[s].len;
        if (b0->nseq) SKM_HIP(hipMemcpyAsync(b0->d_glen.p, len.data(), 4 * b0->nseq, hipMemcpyHostToDevice, b0->stream));
        ensure_local(b0, b0->pass_max);
    } else {
        // global sequence numbering: ranks hold contiguous file ranges in rank order
        std::vector<uint64_t> mine;
        for (auto* b : bs) mine.push_back(b->nseq);
        const std::vector<uint64_t> ns = allgather_u64(bs, mine);
        uint64_t tot = 0;
        for (auto v : ns) tot += v;
        SKM_CHECK(tot < (1ull << ELEM_S_BITS), SKM_E_ARG, "too many sequences in one build");
        std::vector<uint64_t> bytes(ns.size());
        for (size_t r = 0; r < ns.size(); ++r) bytes[r] = 4 * ns[r];
        std::vector<DevBuf> lens_src(bs.size()), ids_src(bs.size()), ids_all(bs.size());
        std::vector<const void*> src_l, src_i;
        std::vector<void*> dst_l, dst_i;
        for (size_t k = 0; k < bs.size(); ++k) {
            skm_build* b = bs[k];
            uint64_t base = 0;
            for (int r = 0; r < b->rank; ++r) base += ns[r];
            b->s_base = (uint32_t)base;
            b->n_total = (uint32_t)tot;
            std::vector<uint32_t> len(b->nseq);
            for (uint32_t s = 0; s < b->nseq; ++s) len[s] = b->h_meta[s].len;
            lens_src[k].ensure(4 * (b->nseq + 1));
            ids_src[k].ensure(4 * (b->nseq + 1));
            ids_all[k].ensure(4 * (tot + 1));
            b->d_glen.ensure(4 * (tot + 1));
            SKM_HIP(hipMemcpy(lens_src[k].p, len.data(), 4 * b->nseq, hipMemcpyHostToDevice));
            SKM_HIP(hipMemcpy(ids_src[k].p, b->h_seqid.data(), 4 * b->nseq, hipMemcpyHostToDevice));
            src_l.push_back(lens_src[k].p);
            src_i.push_back(ids_src[k].p);
            dst_l.push_back(b->d_glen.p);
            dst_i.push_back(ids_all[k].p);
        }
        if (is_group(bs)) {  // allgatherv takes every rank's source in the group form
            allgatherv(bs, src_l, dst_l, bytes);
            allgatherv(bs, src_i, dst_i, bytes);
        } else {
            allgatherv(bs, {src_l[0]}, {dst_l[0]}, bytes);
            allgatherv(bs, {src_i[0]}, {dst_i[0]}, bytes);
        }
        sync_all(bs);
        pass_peer_counts(bs);  // every pass's send / receive sizes, known to the host from here on
        for (size_t k = 0; k < bs.size(); ++k) {
            skm_build* b = bs[k];
            b->g_seqid.resize(tot);
            if (tot) SKM_HIP(hipMemcpy(b->g_seqid.data(), ids_all[k].p, 4 * tot, hipMemcpyDeviceToHost));
            b->g_strict = true;
            for (uint64_t s = 1; s < tot; ++s)
                if (b->g_seqid[s] <= b->g_seqid[s - 1]) b->g_strict = false;
            ensure_local(b, std::max(b->pass_max, b->n_local_max));  // the largest pass's received elements
        }
    }
    for (auto* b : bs) {
        if (!b->tot_cap) {  // first guesses; a run that needs more grows them (run_ranks)
            b->tot_cap = b->cap_local / 8 * 5 + (1u << 16);
            b->split_cap = b->tot_cap / 2;
            b->long_cap = b->pass_bits ? b->valid_total / 8 + (1u << 16) : 0;
        }
        alloc_caps(b);
        // recs_rot: the second element buffer, before the kept arena takes the rest of the memory
        b->rot = false;
        if (b->tune.recs_rot && b->tune.tail_async && !b->tune.overlap && b->world == 1 && b->pass_bits > 0) {
            const uint64_t W = std::max<uint64_t>(b->pass_max, 1);
            if (b->d_recs_hi2.bytes >= 8 * W && b->d_recs_lo2.bytes >= 8 * W) {
                b->rot = true;
            } else {
                size_t fr = 0, tot = 0;
                SKM_HIP(hipMemGetInfo(&fr, &tot));
                const uint64_t held = (uint64_t)b->d_keys.bytes + (uint64_t)b->d_data.bytes;
                const uint64_t need = 16 * W + 32 * W + (1ull << 30) + 18 * (b->valid_total / 4);
                if ((uint64_t)fr + held > need) {
                    b->d_recs_hi2.ensure(8 * W);
                    b->d_recs_lo2.ensure(8 * W);
                    b->rot = true;
                }
            }
        }
        size_arena(b);
        b->d_flags.ensure(std::max<uint64_t>(b->n_total, 1));
        b->d_flagbits.ensure(4 * ((b->n_total + 31) / 32 + 1));
        // pipelined passes when the second element buffer set fits beside everything else with a
        // tenth of the memory to spare (the data-sized buffers may still grow on a redo)
        b->overlap = false;
        if (b->tune.overlap && b->world == 1 && b->pass_bits > 0) {
            size_t fr = 0, tot = 0;
            SKM_HIP(hipMemGetInfo(&fr, &tot));
            const uint64_t need = 16 * std::max<uint64_t>(b->pass_max, 1) + 16 * b->cap_local;
            if (b->d_recs_hi2.bytes >= 8 * std::max<uint64_t>(b->pass_max, 1) && b->d_tmp_hi2.bytes >= 8 * b->cap_local) {
                b->overlap = true;
            } else if ((uint64_t)fr > need + tot / 10) {
                b->d_recs_hi2.ensure(8 * std::max<uint64_t>(b->pass_max, 1));
                b->d_recs_lo2.ensure(8 * std::max<uint64_t>(b->pass_max, 1));
                b->d_tmp_hi2.ensure(8 * b->cap_local);
                b->d_tmp_lo2.ensure(8 * b->cap_local);
                b->overlap = true;
            }
            if (b->overlap) b->d_ovf2b.ensure(sizeof(OvfEntry) * std::max<uint64_t>(b->ovf_cap, 1));
        }
        {
            size_t fr = 0, tot = 0;
            SKM_HIP(hipMemGetInfo(&fr, &tot));
            b->free_after_prepare = fr;
        }
        SKM_HIP(hipStreamSynchronize(b->stream));
        b->prepared = true;
        b->ran = false;
    }
    for (auto* b : bs) b->prep_rest_s = std::chrono::duration<double>(clk::now() - t2).count();
}

// ------------------------------------------------------------------------------------------
// run: extract -> [exchange] -> group-by -> chains -> statistics [-> reductions]
// ------------------------------------------------------------------------------------------
// Key-range pass group g (passes g*G .. g*G+G-1): every pass's window positions and level-1
// histogram into the G slots (k_pass_emit), on stream `st` (no host round trip: the offsets and
// counts come from begin_run's tally and k_sel_scan on the device).
void emit_group(skm_build* b, uint32_t g, hipStream_t st) {
    const uint32_t G = b->emit_g;
    const uint32_t NB = 1u << (b->owner_bits + b->b1_bits);
    const int rem_bits = KEY_BITS - b->pass_bits - b->owner_bits - b->b1_bits;
    const uint64_t cap = std::max<uint64_t>(b->pass_max, 1);
#define SKM_EMIT(GG)                                                                                                    \
    SKM_LAUNCH_AS(b, "k_pass_emit", k_pass_emit<GG>, dim3(b->sel_wg), dim3(EMIT_THREADS), 0, st, b->d_res.as<uint8_t>(), \
                  b->d_ids.as<uint8_t>(), b->rp, g * G, b->sel_span, b->d_seloff.as<uint64_t>(), b->sel_wg, \
                  b->d_posg.as<uint64_t>(), cap)
    if (G == 16)
        SKM_EMIT(16);
    else if (G == 8)
        SKM_EMIT(8);
    else if (G == 4)
        SKM_EMIT(4);
    else if (G == 2)
        SKM_EMIT(2);
    else
        SKM_EMIT(1);
#undef SKM_EMIT
    // the group's histograms from the entries' bucket bits (8 B per window read, no residues)
    SKM_HIP(hipMemsetAsync(b->d_histg.p, 0, sizeof(uint32_t) * NB * G, st));
    SKM_LAUNCH(b, k_pass_hist, dim3(256, G), dim3(PH_THREADS), 4u * NB, st, b->d_posg.as<uint64_t>(), cap,
               b->d_npos.as<unsigned long long>() + (uint64_t)g * G, NB, rem_bits, b->d_histg.as<uint32_t>());
    SKM_HIP(hipGetLastError());
    if (st != b->stream) SKM_HIP(hipEventRecord(b->ev_emit, st));
}

// the element buffer set, counter block, plan and overflow list of a pass (set 0 unless overlap)
inline int pset(const skm_build* b, uint32_t pass) { return b->overlap ? (int)(pass & 1u) : 0; }
inline bool rset(const skm_build* b, uint32_t pass) { return pset(b, pass) || (b->rot && (pass & 1u)); }
inline uint64_t* recs_hi(skm_build* b, uint32_t pass) { return (rset(b, pass) ? b->d_recs_hi2 : b->d_recs_hi).as<uint64_t>(); }
inline uint64_t* recs_lo(skm_build* b, uint32_t pass) { return (rset(b, pass) ? b->d_recs_lo2 : b->d_recs_lo).as<uint64_t>(); }
inline uint64_t* tmp_hi(skm_build* b, uint32_t pass) { return (pset(b, pass) ? b->d_tmp_hi2 : b->d_tmp_hi).as<uint64_t>(); }
inline uint64_t* tmp_lo(skm_build* b, uint32_t pass) { return (pset(b, pass) ? b->d_tmp_lo2 : b->d_tmp_lo).as<uint64_t>(); }
// d_ctr: [0] the kept arena cursor, [2] the flag count (run-level); per-set pass counters at 32, 64
inline unsigned long long* pass_ctr(skm_build* b, uint32_t pass) {
    return b->d_ctr.as<unsigned long long>() + 32 * (1 + pset(b, pass));
}

// the main stream waits for the previous pass's tail (tail_async) before it overwrites what the tail
// reads (the split's recs, then the partition's tmp, the counters, the job lists) or reads what it
// writes (the stash cursors, the kept arena's totals)
// tail_defer: the last pass's tail is issued now (after_scan: behind the next pass's scan kernels)
void issue_tail(skm_build* b, bool after_scan) {
    if (!b->tail_issue) return;
    if (after_scan) {
        SKM_HIP(hipEventRecord(b->ev_scan, b->stream));
        SKM_HIP(hipStreamWaitEvent(b->stream_tail, b->ev_scan, 0));
    }
    std::function<void()> f;
    f.swap(b->tail_issue);
    f();
}

void join_tail(skm_build* b) {
    issue_tail(b, false);
    if (!b->tail_pending) return;
    SKM_HIP(hipStreamWaitEvent(b->stream, b->ev_tail_done, 0));
    b->tail_pending = false;
}

void phase_extract(skm_build* b, uint32_t pass) {
    hipStream_t st = b->stream;
    const int nbits = b->owner_bits + b->b1_bits;
    const uint32_t NB = 1u << nbits;
    const uint32_t nowners = 1u << b->owner_bits;
    SKM_HIP(hipEventRecord(b->ev[0], st));
    // ---- 1. count ----
    const size_t lds_cnt = sizeof(uint32_t) * NB;
    ExtractArgs X;
    X.res = b->d_res.as<uint8_t>();
    X.rp = b->rp;
    X.span = b->span;
    X.owner_bits = b->owner_bits;
    X.b1_bits = b->b1_bits;
    X.pass_bits = b->pass_bits;
    X.pass_id = pass;
    X.pos_cap = b->pass_max;
    X.ids = nullptr;
    X.hist = b->d_hist.as<uint32_t>();
    X.offs = b->d_offs.as<uint32_t>();
    X.owner_start = b->d_owner_start.as<uint64_t>();
    X.blk2seq = b->d_blk2seq.as<uint32_t>();
    X.meta = b->d_meta.as<SeqMeta>();
    X.s_base = b->s_base;
    X.out_hi = recs_hi(b, pass);
    X.out_lo = recs_lo(b, pass);
    uint32_t nwg = b->nwg, hist_rows = b->nwg;
    if (b->pass_bits) {
        // this pass's window positions and histogram: its group's scan, queued on stx during the
        // previous group's last group-by, or issued now (the run's first group)
        const uint32_t G = b->emit_g, q = pass % G;
        if (q == 0) {
            if (b->emit_q == (int64_t)(pass / G))
                SKM_HIP(hipStreamWaitEvent(st, b->ev_emit, 0));
            else
                emit_group(b, pass / G, st);
            b->emit_q = -1;
        }
        X.hist = b->d_histg.as<uint32_t>() + (uint64_t)q * NB;  // one row: the pass's histogram
        X.span = b->pf_span;
        nwg = b->pf_nwg;
        hist_rows = 1;
        (void)lds_cnt;
    } else {
        SKM_LAUNCH(b, k_extract, dim3(nwg), dim3(EX_THREADS), lds_cnt, st, X);
    }
    SKM_HIP(hipGetLastError());
    SKM_HIP(hipEventRecord(b->ev[1], st));
    // ---- 2. scan ----
    const uint32_t nrb = (uint32_t)ceil_div(hist_rows, SCAN_ROWS);
    dim3 gsc((NB + 255) / 256, nrb);
    SKM_LAUNCH(b, k_colsum, gsc, dim3(256), 0, st, X.hist, hist_rows, NB, b->d_partial.as<uint32_t>());
    SKM_LAUNCH(b, k_bstart, dim3(1), dim3(1024), 0, st, b->d_partial.as<uint32_t>(), nrb, NB, b->b1_bits,
                       b->d_rbbase.as<uint32_t>(), b->d_bstart32.as<uint32_t>(), b->d_owner_start.as<uint64_t>(), nowners);
    SKM_LAUNCH(b, k_coloffs, gsc, dim3(256), 0, st, X.hist, b->d_rbbase.as<uint32_t>(), hist_rows,
                       NB, b->d_offs.as<uint32_t>());
    SKM_LAUNCH(b, k_abs_starts, dim3((NB + 1 + 255) / 256), dim3(256), 0, st, b->d_bstart32.as<uint32_t>(),
                       b->d_owner_start.as<uint64_t>(), NB, b->b1_bits, nowners, b->d_bstart.as<uint64_t>());
    SKM_HIP(hipGetLastError());
    SKM_HIP(hipEventRecord(b->ev[2], st));
    // ---- 3. scatter: 64-way staged pass into tmp, then the split into the final buckets ----
    if (b->overlap && b->ovf_pending[pset(b, pass)]) {  // the set's previous pass still read it
        SKM_HIP(hipStreamWaitEvent(st, b->ev_ovf_done[pset(b, pass)], 0));
        b->ovf_pending[pset(b, pass)] = false;
    }
    const int l0_shift = nbits - SC_L0_BITS;
    b->d_cur0.ensure(8ull * 64 * CUR_STRIDE);
    b->d_cur1.ensure(8ull * NB * CUR_STRIDE);
    b->d_slices.ensure(4 * 80);
    SKM_LAUNCH(b, k_stage_init, dim3((NB + 255) / 256), dim3(256), 0, st, b->d_bstart.as<uint64_t>(), NB, l0_shift,
                       b->d_cur0.as<unsigned long long>(), b->d_cur1.as<unsigned long long>(), b->d_slices.as<uint32_t>());
    issue_tail(b, true);
    // the level-0 staging: tmp, or (tail_async) a buffer of its own, so it overlaps the previous
    // pass's tail, which still reads tmp and recs
    const bool sep = tail_async_on(b);
    uint64_t* stg_hi = sep ? b->d_stg_hi.as<uint64_t>() : tmp_hi(b, pass);
    uint64_t* stg_lo = sep ? b->d_stg_lo.as<uint64_t>() : tmp_lo(b, pass);
    if (!sep) join_tail(b);
    if (b->pass_bits && b->tune.stage_round == 1)
        SKM_LAUNCH_AS(b, "k_extract_stage_pos", (k_extract_stage_pos<SC_ROUND_HALF, 4>), dim3(nwg), dim3(EX_THREADS), 0, st, X,
                   b->d_posg.as<uint64_t>() + (uint64_t)(pass % b->emit_g) * std::max<uint64_t>(b->pass_max, 1),
                   b->d_npos.as<unsigned long long>() + pass,
                   b->d_seloff.as<uint64_t>() + (uint64_t)pass * (b->sel_wg + 1), b->sel_wg, b->sel_span,
                   b->d_cur0.as<unsigned long long>(), stg_hi, stg_lo);
    else if (b->pass_bits)
        SKM_LAUNCH_AS(b, "k_extract_stage_pos", (k_extract_stage_pos<SC_ROUND, 2>), dim3(nwg), dim3(EX_THREADS), 0, st, X,
                   b->d_posg.as<uint64_t>() + (uint64_t)(pass % b->emit_g) * std::max<uint64_t>(b->pass_max, 1),
                   b->d_npos.as<unsigned long long>() + pass,
                   b->d_seloff.as<uint64_t>() + (uint64_t)pass * (b->sel_wg + 1), b->sel_wg, b->sel_span,
                   b->d_cur0.as<unsigned long long>(), stg_hi, stg_lo);
    else
        SKM_LAUNCH(b, k_extract_stage, dim3(nwg), dim3(EX_THREADS), 0, st, X, b->d_cur0.as<unsigned long long>(),
                           stg_hi, stg_lo);
    // recs_rot: the split writes the other element buffer; the wait moves to the partition
    if (!b->rot) join_tail(b);
    const uint32_t nsl = (uint32_t)(ceil_div(b->pass_max, SC_SLICE) + (1u << SC_L0_BITS));
    SKM_LAUNCH(b, k_split_stage, dim3(nsl), dim3(EX_THREADS), 0, st, stg_hi,
                       stg_lo, b->d_bstart.as<uint64_t>(), nbits, b->d_slices.as<uint32_t>(),
                       b->d_cur1.as<unsigned long long>(), recs_hi(b, pass), recs_lo(b, pass));
    SKM_HIP(hipGetLastError());
    SKM_HIP(hipEventRecord(b->ev[3], st));
}

// world > 1, one key-range pass: the element counts of every (pass, peer) pair were exchanged at
// prepare (pass_peer_counts), so every size of the pass's all-to-alls is a host value already and
// the exchange issues without a host round trip: per-bucket counts (fixed size) and the elements
// (RCCL: stream-ordered grouped send/recv; the in-process group and the host transport stage and
// synchronise inside alltoallv), then the receive layout is planned on the device (k_recv_plan).
void exchange(const Ranks& bs, uint32_t pass) {
    const int W = bs[0]->world;
    const uint32_t NB1 = 1u << bs[0]->b1_bits;
    const uint32_t NB = NB1 * (uint32_t)W;
    A2A cx, ex_hi, ex_lo;
    for (auto* b : bs) {
        b->d_cnt_send.ensure(4ull * NB);
        b->d_cnt_recv.ensure(4ull * NB);
        SKM_LAUNCH(b, k_send_counts, dim3((NB + 255) / 256), dim3(256), 0, b->stream, b->d_bstart.as<uint64_t>(), NB, NB1,
                   (uint32_t)W, b->d_xs.as<unsigned long long>() + (uint64_t)pass * W, b->d_run.as<unsigned long long>(),
                   b->d_cnt_send.as<uint32_t>());
        cx.send.push_back(b->d_cnt_send.as<uint8_t>());
        cx.recv.push_back(b->d_cnt_recv.as<uint8_t>());
        std::vector<uint64_t> off(W), c(W, 4ull * NB1);
        for (int q = 0; q < W; ++q) off[q] = 4ull * NB1 * q;
        cx.soff.push_back(off);
        cx.scnt.push_back(c);
        cx.roff.push_back(off);
        cx.rcnt.push_back(c);
        std::vector<uint64_t> so(W), sc(W), ro(W), rcn(W);
        uint64_t s0 = 0, r0 = 0;
        for (int q = 0; q < W; ++q) {
            const uint64_t ns = b->xs_send[(uint64_t)pass * W + q], nr = b->xs_recv[(uint64_t)pass * W + q];
            so[q] = 8 * s0;
            sc[q] = 8 * ns;
            ro[q] = 8 * r0;
            rcn[q] = 8 * nr;
            s0 += ns;
            r0 += nr;
        }
        ex_hi.send.push_back(b->d_recs_hi.as<uint8_t>());
        ex_hi.recv.push_back(b->d_rhi.as<uint8_t>());
        ex_lo.send.push_back(b->d_recs_lo.as<uint8_t>());
        ex_lo.recv.push_back(b->d_rlo.as<uint8_t>());
        for (A2A* e : {&ex_hi, &ex_lo}) {
            e->soff.push_back(so);
            e->scnt.push_back(sc);
            e->roff.push_back(ro);
            e->rcnt.push_back(rcn);
        }
    }
    alltoallv(bs, cx);
    alltoallv(bs, ex_hi);
    alltoallv(bs, ex_lo);
    for (auto* b : bs) {
        b->d_seg_start.ensure(8ull * NB);
        b->d_seg_len.ensure(4ull * NB);
        b->d_vstart.ensure(8ull * (NB1 + 1));
        SKM_LAUNCH(b, k_recv_plan, dim3(1), dim3(1024), 0, b->stream, b->d_cnt_recv.as<uint32_t>(), (uint32_t)W, NB1,
                   b->d_xs.as<unsigned long long>() + (uint64_t)(b->xs_recv.size() / W + pass) * W,
                   b->d_run.as<unsigned long long>(), b->d_seg_start.as<uint64_t>(), b->d_seg_len.as<uint32_t>(),
                   b->d_vstart.as<uint64_t>());
        SKM_HIP(hipGetLastError());
    }
}

// world > 1, at prepare: every rank's valid windows by (pass, owner) -- one counting scan -- and
// one all-to-all of those counts, so each pass's send and receive sizes are known to the host up
// front; the received elements of the largest pass size this rank's work buffers
void pass_peer_counts(const Ranks& bs) {
    const int W = bs[0]->world;
    const uint32_t P = 1u << bs[0]->pass_bits;
    A2A x;
    std::vector<DevBuf> snd(bs.size()), rcv(bs.size());
    for (size_t k = 0; k < bs.size(); ++k) {
        skm_build* b = bs[k];
        DevBuf cnt;
        cnt.ensure(8ull * P * W);
        SKM_HIP(hipMemsetAsync(cnt.p, 0, 8ull * P * W, b->stream));
        if (b->rp)  // by routed pass id when routing (route_plan)
            hipLaunchKernelGGL(k_pass_ids, dim3(1024), dim3(256), 4u * P * W + (b->route ? (1u << BLOOM_BITS) / 8 : 0u),
                               b->stream, b->d_res.as<uint8_t>(), b->rp, b->pass_bits, b->owner_bits, nullptr,
                               cnt.as<unsigned long long>(), b->route ? b->d_bloom.as<uint32_t>() : nullptr, P * W,
                               nullptr, 0, route_arg(b));
        SKM_HIP(hipGetLastError());
        std::vector<uint64_t> c(P * W), t(P * W);
        SKM_HIP(hipMemcpyAsync(c.data(), cnt.p, 8ull * P * W, hipMemcpyDeviceToHost, b->stream));
        SKM_HIP(hipStreamSynchronize(b->stream));
        b->xs_send = c;  // [pass][peer]
        for (uint32_t p = 0; p < P; ++p)
            for (int q = 0; q < W; ++q) t[(uint64_t)q * P + p] = c[(uint64_t)p * W + q];  // [peer][pass]
        snd[k].ensure(8ull * P * W);
        rcv[k].ensure(8ull * P * W);
        SKM_HIP(hipMemcpy(snd[k].p, t.data(), 8ull * P * W, hipMemcpyHostToDevice));
        x.send.push_back(snd[k].as<uint8_t>());
        x.recv.push_back(rcv[k].as<uint8_t>());
        std::vector<uint64_t> off(W), n(W, 8ull * P);
        for (int q = 0; q < W; ++q) off[q] = 8ull * P * q;
        x.soff.push_back(off);
        x.scnt.push_back(n);
        x.roff.push_back(off);
        x.rcnt.push_back(n);
    }
    alltoallv(bs, x);
    sync_all(bs);
    for (size_t k = 0; k < bs.size(); ++k) {
        skm_build* b = bs[k];
        std::vector<uint64_t> t(P * W);
        SKM_HIP(hipMemcpy(t.data(), rcv[k].p, 8ull * P * W, hipMemcpyDeviceToHost));
        b->xs_recv.assign((uint64_t)P * W, 0);
        uint64_t most = 0;
        for (uint32_t p = 0; p < P; ++p) {
            uint64_t tot = 0;
            for (int q = 0; q < W; ++q) {
                b->xs_recv[(uint64_t)p * W + q] = t[(uint64_t)q * P + p];  // [pass][source]
                tot += t[(uint64_t)q * P + p];
            }
            most = std::max(most, tot);
        }
        SKM_CHECK(most < (1ull << 32) - (1ull << 28), SKM_E_ARG, "more than 2^32 occurrences in one pass of one GPU");
        b->n_local_max = most;
        // device copy for the exchange's checks: [pass][peer] sends, then [pass][source] receives
        b->d_xs.ensure(16ull * P * W);
        SKM_HIP(hipMemcpy(b->d_xs.p, b->xs_send.data(), 8ull * P * W, hipMemcpyHostToDevice));
        SKM_HIP(hipMemcpy(b->d_xs.as<uint64_t>() + (uint64_t)P * W, b->xs_recv.data(), 8ull * P * W, hipMemcpyHostToDevice));
    }
}

// Job sort by length class (longest first) + the chain kernels, for a job list whose length is on
// the device (nj_d, at most cap).  Chains of >= 2^long_class samples get a wave pair each
// (k_chain_long): in situ with one pass; with key-range passes their samples are stashed into the
// run's long arena and they run on the chain stream, overlapping the following passes.  The
// per-lane chains run on st (or st_short) within the pass.  Fixed grids that read the counts on
// the device: no host round trip.
// Giant chains (>= 2^class samples) start on their own streams right after k_heavy instead of
// waiting for the stash batches.  Default on with one pass, and at world > 1 (verdict r04 #4): the
// owner split leaves each rank few passes (two at 8 GPUs), routing puts the heaviest k-mers into
// the first, and their stashed chains would only start after that pass's group-by (~0.08 s of a
// ~0.2 s step) -- the multi-GPU step's floor.  Off on one GPU with key-range passes, where the
// stash batches overlap the later passes (C3: +60..80 ms, the FP64 chain waves slow the passes).
// samples a pass's giant-chain buffer holds (k_heavy: a key that no longer fits takes the job path):
// the split capacity, at most 2^28 (1 GB per pass: C3's heavy-only pass 0 holds ~7 * 10^8 samples
// of keys of >= 2^17 occurrences; the longest chains come first in k_heavy's list, mostly)
uint64_t giant_cap(const skm_build* b) { return std::min<uint64_t>(std::max<uint64_t>(b->split_cap, 1), 1ull << 28); }

int giant_class(const skm_build* b) {
    return b->tune.giant_class >= 0 ? b->tune.giant_class : (b->pass_bits == 0 || b->world > 1 ? 14 : 0);
}

constexpr uint32_t JOB_NWG = 256;      // k_job_count / k_job_scatter workgroups (one chunk each)
constexpr uint32_t LONG_GRID = 2048;   // k_chain_long / k_long_stash workgroups (one job at a time)

constexpr uint32_t CHAINQ_SLOTS = 256;  // k_chains launches per run (2 per pass + the stash batches)

// a zeroed pair of k_chains queue counters on stream st (distinct per launch of the run)
unsigned long long* chain_queue(skm_build* b, hipStream_t st) {
    if (!b->tune.chain_queue) return nullptr;
    b->d_chainq.ensure(16ull * CHAINQ_SLOTS);
    unsigned long long* q = b->d_chainq.as<unsigned long long>() + 2 * (b->chainq_next++ % CHAINQ_SLOTS);
    SKM_HIP(hipMemsetAsync(q, 0, 16, st));
    return q;
}

void launch_chains(skm_build* b, hipStream_t st, const Job* jobs, const unsigned long long* nj_d, uint64_t cap,
                   ChainSet& cs, const uint32_t* lens, const uint32_t* recs32, const uint32_t* tmp32,
                   const uint32_t* big32, skm_stored_kmer_data* out, uint32_t long_class,
                   hipStream_t st_short = nullptr, hipEvent_t ev_sorted = nullptr, uint32_t max_wgs = 0) {
    const Tune& tn = b->tune;
    SKM_LAUNCH(b, k_job_count, dim3(JOB_NWG), dim3(JOB_WG), 0, st, jobs, nj_d, cap, cs.hist.as<uint32_t>());
    SKM_LAUNCH(b, k_job_scan, dim3(1), dim3(64), 0, st, cs.hist.as<uint32_t>(), JOB_NWG, cs.offs.as<uint64_t>(),
                       long_class);
    SKM_LAUNCH(b, k_job_scatter, dim3(JOB_NWG), dim3(JOB_WG), 0, st, jobs, nj_d, cap, cs.offs.as<uint64_t>(),
                       cs.sorted.as<Job>());
    if (st_short && ev_sorted) SKM_HIP(hipEventRecord(ev_sorted, st));  // sorted jobs ready
    // k_job_scan leaves the long jobs' count after the offsets; they lead the sorted order
    const uint64_t* nlong_d = cs.offs.as<uint64_t>() + (uint64_t)JOB_NWG * JOB_CLASSES;
    const auto* nlong_u = reinterpret_cast<const unsigned long long*>(nlong_d);
    const bool run_chains = !(tn.diag & 4) && !(tn.diag & 16);
    if (b->pass_bits == 0) {
        // one pass: the long chains start on st as soon as their jobs are sorted
        const uint32_t lds = (uint32_t)tn.chain_lds_kb * 1024u;
        static bool attr = false;
        if (lds > 65536 && !attr) {
            SKM_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k_chain_long),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            attr = true;
        }
        if (run_chains)
            SKM_LAUNCH(b, k_chain_long, dim3(LONG_GRID), dim3(128), lds, st, cs.sorted.as<Job>(), nullptr, nlong_u,
                       lens, recs32, tmp32, big32, out, tn.chain_prio);
    } else {
        SKM_LAUNCH(b, k_long_plan, dim3(1), dim3(1024), 0, st, cs.sorted.as<Job>(), nlong_d,
                           cs.long_off.as<uint64_t>(), b->d_run.as<unsigned long long>(), b->long_cap,
                           b->long_jobs_cap);
        SKM_LAUNCH(b, k_long_stash, dim3(LONG_GRID), dim3(256), 0, st, cs.sorted.as<Job>(), nlong_d,
                           cs.long_off.as<uint64_t>(), lens, recs32, tmp32, big32, b->d_long_arena.as<uint32_t>(),
                           b->d_long_jobs.as<Job>());
    }
    // the per-lane chains on their own stream (when given): they do not wait for the long ones
    hipStream_t ss = st;
    if (st_short && ev_sorted) {
        SKM_HIP(hipStreamWaitEvent(st_short, ev_sorted, 0));
        ss = st_short;
    }
    if (run_chains) {
        unsigned long long* q = chain_queue(b, ss);
        SKM_LAUNCH(b, k_chains, dim3(max_wgs ? max_wgs : (uint32_t)std::max(1, tn.chain_grid)), dim3(256), 0, ss,
                   cs.sorted.as<Job>(), nlong_u, nj_d, cap, lens, recs32, tmp32, big32, out, 0u, q);
    }
    SKM_HIP(hipGetLastError());
}

// Group-by.  k_partition splits the oversized level-1 buckets and k_ovf_plan orders and sizes the
// overflow sub-buckets on the device; the overflow (the heaviest k-mers and their long P^2 chains)
// then runs on streams 2 and 3, concurrently with k_bucket_process on the first.  No host round
// trip: every launch is issued up front, the grids that depend on counts are persistent.
void phase_group(skm_build* b, uint32_t pass) {
    hipStream_t st = b->stream, st2 = b->stream2, st3 = b->stream3;
    const bool multi = b->world > 1;
    const uint32_t NB1 = 1u << b->b1_bits;
    join_tail(b);  // recs_rot: the previous pass's tail still read tmp, the counters and the job lists
    SKM_HIP(hipEventRecord(b->ev[4], st));
    // per-pass counters; [0] (kept k-mers: the arena cursor) and the signature flags run over
    // all passes (begin_run clears them)
    unsigned long long* ctr_d = pass_ctr(b, pass);
    SKM_HIP(hipMemsetAsync(ctr_d, 0, 256, st));
    unsigned long long* run_d = b->d_run.as<unsigned long long>();
    const int ks = pset(b, pass);
    uint32_t* plan_d = b->d_plan.as<uint32_t>() + PLAN_SLOTS * ks;
    OvfEntry* ovf2_d = (ks ? b->d_ovf2b : b->d_ovf2).as<OvfEntry>();
    BucketArgs A;
    A.recs_hi = multi ? b->d_rhi.as<uint64_t>() : recs_hi(b, pass);
    A.recs_lo = multi ? b->d_rlo.as<uint64_t>() : recs_lo(b, pass);
    A.tmp_hi = tmp_hi(b, pass);
    A.tmp_lo = tmp_lo(b, pass);
    A.bstart = multi ? b->d_vstart.as<uint64_t>() : b->d_bstart.as<uint64_t>();
    A.seg_start = multi ? b->d_seg_start.as<uint64_t>() : nullptr;
    A.seg_len = multi ? b->d_seg_len.as<uint32_t>() : nullptr;
    A.nsrc = multi ? (uint32_t)b->world : 1u;
    A.sub_tab = b->d_sub_tab.as<uint32_t>();
    A.kept_ctr = b->d_ctr.as<unsigned long long>();
    A.nbuckets = NB1;
    A.bucket_base = (pass << (b->owner_bits + b->b1_bits)) | ((uint32_t)b->rank << b->b1_bits);
    A.rem_bits = KEY_BITS - b->pass_bits - b->owner_bits - b->b1_bits;
    A.pshift = KEY_BITS - b->pass_bits;
    A.glen = b->d_glen.as<uint32_t>();
    A.flags = (b->tune.diag & 1) ? nullptr
              : b->tune.flag_bits ? reinterpret_cast<uint8_t*>(reinterpret_cast<uintptr_t>(b->d_flagbits.p) | 1u)
                                  : b->d_flags.as<uint8_t>();
    A.flag_check = b->tune.flag_bits ? 0 : b->tune.flag_check;  // reads the byte form only
    A.ctr = ctr_d;
    A.out_keys = b->d_keys.as<uint64_t>();
    A.out_data = b->d_data.as<skm_stored_kmer_data>();
    A.jobs = b->d_jobs.as<Job>();
    A.lens = b->d_lens.as<uint32_t>();
    A.ovf = b->d_ovf.as<OvfEntry>();
    A.ovf_cap = (uint32_t)b->ovf_cap;
    A.prio = b->tune.bucket_prio;
    A.stamps = nullptr;
    A.big_desc = b->d_big_desc.as<uint64_t>();
    A.big_cap = (uint32_t)std::min<uint64_t>(b->big_cap, 0xFFFFFFFFull);
    A.skip = nullptr;
    A.sub_target = (uint32_t)std::max(0, b->tune.sub_target);
    A.diag = b->tune.diag;
    if (b->stamps) {
        SKM_HIP(hipMemsetAsync(b->d_stamps.p, 0, 32 * 8, st));
        A.stamps = b->d_stamps.as<unsigned long long>();
    }
    // ---- 4a. level-2 partition (the oversized buckets' workgroups first) ----
    A.order = nullptr;
    A.part_class = 0;
    if (b->tune.part_order) {
        b->d_part_order.ensure(4ull * (NB1 + 1));
        SKM_LAUNCH(b, k_part_order, dim3(1), dim3(1024), 0, st, A.bstart, NB1, b->d_part_order.as<uint32_t>());
        A.order = b->d_part_order.as<uint32_t>();
    }
    if (A.order && b->tune.part_split && b->tune.partition_round == 0 && !b->overlap) {
        // part_split: the oversized buckets on stream 2 by 1024-thread workgroups (rounds of 4096),
        // beside the others on the main stream -- a heavy bucket's workgroup no longer sets the
        // kernel's length (stream 2's earlier work is joined: the split waited for the last tail)
        BucketArgs AH = A;
        AH.part_class = 1;
        SKM_HIP(hipEventRecord(b->ev_part, st));
        SKM_HIP(hipStreamWaitEvent(st2, b->ev_part, 0));
        SKM_LAUNCH_AS(b, "k_partition", (k_partition<4096, 1024, 1>), dim3(NB1), dim3(1024), 0, st2, AH);
        SKM_HIP(hipEventRecord(b->ev_part_heavy, st2));
        A.part_class = 2;
        SKM_LAUNCH_AS(b, "k_partition", (k_partition<2048, BP_THREADS, 3>), dim3(NB1), dim3(BP_THREADS), 0, st, A);
        SKM_HIP(hipStreamWaitEvent(st, b->ev_part_heavy, 0));
        A.part_class = 0;
    } else if (b->tune.partition_round == 1)
        SKM_LAUNCH_AS(b, "k_partition", (k_partition<4096, 512, 1>), dim3(NB1), dim3(512), 0, st, A);
    else if (b->tune.partition_round == 2)
        SKM_LAUNCH_AS(b, "k_partition", (k_partition<4096, 1024, 1>), dim3(NB1), dim3(1024), 0, st, A);
    else
        SKM_LAUNCH_AS(b, "k_partition", (k_partition<2048, BP_THREADS, 3>), dim3(NB1), dim3(BP_THREADS), 0, st, A);
    SKM_HIP(hipGetLastError());
    SKM_HIP(hipEventRecord(b->ev[10], st));
    // the group's position slots are free once its last pass has staged its elements; the next
    // group's scan waits until this pass's partition is done too, so that it overlaps the group-by
    // rather than the scatters on the step's critical path
    if (b->pass_bits && pass % b->emit_g == b->emit_g - 1) SKM_HIP(hipEventRecord(b->ev_staged, st));
    // ---- the overflow plan (the pass's element count: the last bucket start, or the exchange's) ----
    const unsigned long long* nloc_d;
    if (multi) {  // the received element count: k_recv_plan's vstart[NB1]
        nloc_d = reinterpret_cast<const unsigned long long*>(b->d_vstart.as<uint64_t>() + NB1);
    } else {
        nloc_d = reinterpret_cast<const unsigned long long*>(b->d_bstart.as<uint64_t>() + NB1);
    }
    const uint32_t split_min = (uint32_t)std::max(b->tune.split_min, CAP + 1);
    const uint32_t key_min = (uint32_t)std::max(b->tune.heavy_min, 2);
    PlanArgs P;
    P.in = b->d_ovf.as<OvfEntry>();
    P.out = ovf2_d;
    P.ctr = ctr_d;
    P.kept = b->d_ctr.as<unsigned long long>();
    P.nloc = nloc_d;
    P.run = run_d;
    P.plan = plan_d;
    P.ovf_cap = (uint32_t)b->ovf_cap;
    P.split_min = split_min;
    P.heavy_min = (uint32_t)b->tune.ovf_heavy;
    P.kept_cap = b->kept_cap;
    P.tot_cap = b->tot_cap;
    P.split_cap = b->split_cap;
    SKM_LAUNCH(b, k_ovf_plan, dim3(1), dim3(1024), 0, st, P);
    SKM_HIP(hipGetLastError());
    A.skip = plan_d + PLAN_SKIP;
    // ---- 5. overflow sub-buckets (> CAP elements), largest first, concurrent with the group-by:
    //      the split (heavy keys out to k_heavy) and the heavy entries on stream 2, whose chains
    //      start as soon as they are grouped; the rest on stream 3 ----
    BucketArgs A2 = A, A3 = A;
    OvfScratch S;
    S.hi = b->d_ovf_hi.as<uint64_t>();
    S.lo = b->d_ovf_lo.as<uint64_t>();
    S.heads = b->d_ovf_heads.as<uint32_t>();
    S.jobinfo = b->d_ovf_job.as<uint64_t>();
    S.fmean = b->d_ovf_fm.as<uint32_t>();
    // both parts append to one job list (own job / length counters of the overflow; the kept
    // counter stays shared); the chains start when both parts are grouped
    A2.ovf = ovf2_d;
    A2.ctr = ctr_d + 8;
    A2.jobs = b->d_jobs2.as<Job>();
    A2.lens = b->d_lens.as<uint32_t>();
    A3.ovf = A2.ovf;
    A3.ctr = A2.ctr;
    A3.jobs = A2.jobs;
    A3.lens = A2.lens;
    const uint32_t inline_min = (uint32_t)b->tune.ovf_inline_min;
    const int prio = b->tune.inline_prio;
    HeavyArgs H;
    H.keys = b->d_hv_keys.as<HeavyKey>();
    H.nkeys = ctr_d + 18;  // cleared with the pass's counters
    H.cursor = ctr_d + 19;
    H.queue = ctr_d + 20;
    H.rec = b->d_hv_rec.as<uint64_t>();
    H.len = b->d_hv_len.as<uint32_t>();
    H.s0 = b->d_hv_s0.as<uint32_t>();
    H.s1 = b->d_hv_s1.as<uint32_t>();
    H.nosort = (b->tune.diag & 2) ? 1u : 0u;
    H.fast = b->opts.n_functions <= HV_FT && !b->tune.heavy_lsd ? 1u : 0u;
    H.n_total = std::max<uint32_t>(b->n_total, 1);
    // giant chains: samples and jobs in this pass's own buffers, run on a rotating chain stream
    // (only in the last giant_passes passes: earlier passes' long chains overlap the later passes
    // from the stash batches anyway; the last pass's would form the tail)
    const int gs = (int)(pass % skm_build::GSLOTS);
    const uint32_t NP = 1u << b->pass_bits;
    const bool late = b->tune.giant_passes <= 0 || pass + (uint32_t)b->tune.giant_passes >= NP;
    const int gcls = giant_class(b);
    H.giant_min = gcls > 0 && late && pass < b->gsamples.size() ? 1u << gcls : 0u;
    H.gsamples = nullptr;
    H.gjobs = nullptr;
    H.gcount = nullptr;
    H.gcap = 0;
    H.gstat = nullptr;
    if (H.giant_min) {
        H.gsamples = b->gsamples[pass].as<uint32_t>();
        H.gjobs = b->gjobs[pass].as<Job>();
        H.gcount = b->gcount[pass].as<unsigned long long>();
        H.gcap = giant_cap(b);
        H.gstat = b->d_gstat.as<unsigned long long>();
    }
    // issued before the group-by (concurrent with it), or after it (option serial_overflow: the
    // group-by's time alone)
    auto launch_overflow = [&]() {
    SKM_HIP(hipEventRecord(b->ev_part, st));
    SKM_HIP(hipStreamWaitEvent(st2, b->ev_part, 0));
    SKM_HIP(hipStreamWaitEvent(st3, b->ev_part, 0));
    SKM_HIP(hipEventRecord(b->ev_o[0], st2));
    SKM_HIP(hipEventRecord(b->ev_o3[0], st3));
    if (H.giant_min) SKM_HIP(hipMemsetAsync(b->gcount[pass].p, 0, 16, st2));
    SKM_LAUNCH(b, k_ovf_split, dim3((uint32_t)std::max(1, b->tune.split_grid)), dim3(BP_THREADS), 0, st2, A2, S, H, key_min, plan_d);
    SKM_HIP(hipEventRecord(b->ev_split, st2));
    SKM_HIP(hipStreamWaitEvent(st3, b->ev_split, 0));
    SKM_LAUNCH(b, k_heavy, dim3((uint32_t)std::max(1, b->tune.heavy_grid)), dim3(HEAVY_WG), 0, st2, A2, H);
    SKM_HIP(hipGetLastError());
    if (H.giant_min) {
        SKM_HIP(hipEventRecord(b->gev_ready[gs], st2));
        SKM_HIP(hipStreamWaitEvent(b->gst[gs], b->gev_ready[gs], 0));
        SKM_LAUNCH(b, k_giant_order, dim3(1), dim3(1024), 0, b->gst[gs], H.gjobs, H.gcount);
        if (!b->giant_timed) SKM_HIP(hipEventRecord(b->ev_giant[0], b->gst[gs]));
        SKM_LAUNCH(b, k_chain_dyn, dim3(1024), dim3(128), 0, b->gst[gs], H.gjobs, H.gcount, A.out_data,
                           b->tune.chain_prio);
        SKM_HIP(hipGetLastError());
        if (!b->giant_timed) SKM_HIP(hipEventRecord(b->ev_giant[1], b->gst[gs]));
        b->giant_timed = true;
        SKM_HIP(hipEventRecord(b->gev_done[gs], b->gst[gs]));
        b->gused[gs] = true;
    }
    SKM_LAUNCH(b, k_overflow, dim3((uint32_t)std::max(1, b->tune.ovf_grid)), dim3(BP_THREADS), 0, st2, A2, S, plan_d, -1, (int)PLAN_NHEAVY,
                       (int)PLAN_Q_HEAVY, inline_min, prio);
    SKM_HIP(hipEventRecord(b->ev_o[1], st2));
    SKM_LAUNCH(b, k_overflow, dim3((uint32_t)std::max(1, b->tune.ovf_grid)), dim3(BP_THREADS), 0, st3, A3, S, plan_d, (int)PLAN_NHEAVY,
                       (int)PLAN_NOVF, (int)PLAN_Q_REST, inline_min, prio);
    SKM_HIP(hipGetLastError());
    };
    if (!b->tune.serial_overflow) launch_overflow();
    // ---- 4b. group-by of the sub-buckets that fit LDS; groups of > 64 members are handed to
    //      k_big_groups (one wave each) and appended ----
    BigArgs BA;
    BA.desc = A.big_desc;
    BA.ndesc = ctr_d + 5;
    BA.cap = A.big_cap;
    BA.recs_hi = A.recs_hi;
    BA.tmp_hi = A.tmp_hi;
    BA.recs_lo = A.recs_lo;
    BA.tmp_lo = A.tmp_lo;
    BA.flags = A.flags;
    BA.out = b->d_big_out.as<BigOut>();
    SKM_HIP(hipEventRecord(b->ev[11], st));
    SKM_LAUNCH(b, k_bucket_process, dim3(NB1), dim3(BPK_THREADS), 0, st, A);
    SKM_HIP(hipGetLastError());
    SKM_HIP(hipEventRecord(b->ev[5], st));
    if (b->tune.serial_overflow) launch_overflow();
    // the next group's positions overlap this pass's group-by on stx (the group's slots were
    // last read by this pass's staging; ev_staged is recorded after the partition)
    if (b->pass_bits && pass + 1 < NP && (pass + 1) % b->emit_g == 0 && b->tune.prefetch) {
        SKM_HIP(hipStreamWaitEvent(b->stx, b->ev_staged, 0));
        emit_group(b, (pass + 1) / b->emit_g, b->stx);
        b->emit_q = (pass + 1) / b->emit_g;
    }
    // the pass's tail: on the main stream, or (tail_async) on its own stream beside the next pass's
    // staging -- the next split waits for it (join_tail)
    const bool tail_async = tail_async_on(b);
    hipStream_t tt = tail_async ? b->stream_tail : st;
    if (tail_async) {
        SKM_HIP(hipEventRecord(b->ev_tail_bp, st));
        SKM_HIP(hipStreamWaitEvent(tt, b->ev_tail_bp, 0));
    }
    hipEvent_t* ev = b->ev;  // this pass's events (the deferred tail is issued after use_evset(pass + 1))
    auto big_tail = [=]() {
    if (tail_async && b->tune.big_split) {
        // the two size classes of big groups are independent (disjoint descriptors and outputs):
        // the large class on a stream of its own, joined before the append
        SKM_HIP(hipStreamWaitEvent(b->stream_tail2, b->ev_tail_bp, 0));
        SKM_LAUNCH(b, k_big_groups<true>, dim3((uint32_t)std::max(1, b->tune.big_grid_large)), dim3(BIG_WG), 0,
                   b->stream_tail2, BA);
        SKM_HIP(hipEventRecord(b->ev_tail2, b->stream_tail2));
        SKM_LAUNCH(b, k_big_groups<false>, dim3((uint32_t)std::max(1, b->tune.big_grid)), dim3(BIG_WG), 0, tt, BA);
        SKM_HIP(hipStreamWaitEvent(tt, b->ev_tail2, 0));
    } else {
        SKM_LAUNCH(b, k_big_groups<false>, dim3((uint32_t)std::max(1, b->tune.big_grid)), dim3(BIG_WG), 0, tt, BA);
        SKM_LAUNCH(b, k_big_groups<true>, dim3((uint32_t)std::max(1, b->tune.big_grid_large)), dim3(BIG_WG), 0, tt, BA);
    }
    SKM_LAUNCH(b, k_big_append, dim3(256), dim3(BIG_WG), 0, tt, BA.out, BA, A);
    SKM_HIP(hipGetLastError());
    SKM_HIP(hipEventRecord(ev[12], tt));
    };
    // ---- 6. deferred P^2 / variance chains: the overflow's as soon as both parts are grouped
    //      (the long ones on stream 2, the per-lane ones on stream 3), the group-by's on st ----
    SKM_HIP(hipEventRecord(b->ev_o3[0], st3));
    SKM_HIP(hipStreamWaitEvent(st2, b->ev_o3[0], 0));
    launch_chains(b, st2, A2.jobs, ctr_d + 8 + 3, b->jobs2_cap, b->cs_ovf, A2.lens, nullptr, nullptr, nullptr,
                  A.out_data, (uint32_t)b->tune.ovf_long_class, st3, b->ev_o3[2], (uint32_t)b->tune.ovf_chain_wgs);
    SKM_HIP(hipEventRecord(b->ev_o[2], st2));
    SKM_HIP(hipEventRecord(b->ev_o3[1], st3));
    hipEvent_t* ev_o = b->ev_o;
    hipEvent_t* ev_o3 = b->ev_o3;
    auto main_tail = [=]() {
    big_tail();
    launch_chains(b, tt, A.jobs, ctr_d + 3, b->jobs_cap, b->cs_main, A.lens, reinterpret_cast<const uint32_t*>(A.recs_hi),
                  reinterpret_cast<const uint32_t*>(A.tmp_hi), nullptr, A.out_data, (uint32_t)b->tune.main_long_class);
    if (b->overlap) {
        // the pass ends on the main stream here; its overflow path and accounting finish on
        // stream 2 beside the next pass, whose staging into this set waits for ev_ovf_done
        SKM_HIP(hipEventRecord(b->ev_main_done[ks], st));
        SKM_HIP(hipEventRecord(ev[6], st));
        SKM_HIP(hipStreamWaitEvent(st2, ev_o3[1], 0));
        SKM_HIP(hipStreamWaitEvent(st2, b->ev_main_done[ks], 0));
        SKM_LAUNCH(b, k_pass_account, dim3(1), dim3(1), 0, st2, ctr_d, run_d, b->jobs_cap, b->jobs2_cap, b->big_cap,
                   b->lens_cap);
        SKM_HIP(hipGetLastError());
        SKM_HIP(hipEventRecord(b->ev_ovf_done[ks], st2));
        b->ovf_pending[ks] = true;
        SKM_HIP(hipEventRecord(ev[7], st));
        return;
    }
    SKM_HIP(hipStreamWaitEvent(tt, ev_o[2], 0));
    SKM_HIP(hipStreamWaitEvent(tt, ev_o3[1], 0));
    SKM_HIP(hipEventRecord(ev[6], tt));
    // ---- 7. run totals and the chain lists' bounds ----
    SKM_LAUNCH(b, k_pass_account, dim3(1), dim3(1), 0, tt, ctr_d, run_d, b->jobs_cap, b->jobs2_cap, b->big_cap,
                       b->lens_cap);
    SKM_HIP(hipGetLastError());
    SKM_HIP(hipEventRecord(ev[7], tt));
    if (tail_async) {
        SKM_HIP(hipEventRecord(b->ev_tail_done, tt));
        b->tail_pending = true;
    }
    };
    // tail_defer: issued by the next pass's phase_extract after its scan kernels (or by join_tail)
    if (tail_async && b->tune.tail_defer && pass + 1 < NP && !b->overlap)
        b->tail_issue = main_tail;
    else
        main_tail();
}

// overlap: the main stream waits for every pass's overflow path still in flight
void drain_overflow(skm_build* b) {
    for (int k = 0; k < 2; ++k)
        if (b->ovf_pending[k]) {
            SKM_HIP(hipStreamWaitEvent(b->stream, b->ev_ovf_done[k], 0));
            b->ovf_pending[k] = false;
        }
}

// Work buffers whose size depends on the data (the overflow scratch, the split path, the chain
// lists, the stashed long chains, the giant slots): sized from the capacities before the run, so
// the passes need no host decisions.  A run that outgrows one records its demand; run_ranks grows
// the capacities and redoes the step (the first run on a new input at most).
void alloc_caps(skm_build* b) {
    const uint64_t T = std::max<uint64_t>(b->tot_cap, 1), Sp = std::max<uint64_t>(b->split_cap, 1);
    b->d_ovf_hi.ensure(8 * T);
    b->d_ovf_lo.ensure(8 * T);
    b->d_ovf_heads.ensure(4 * T);
    b->d_ovf_job.ensure(8 * T);
    b->d_ovf_fm.ensure(4 * T);
    b->jobs2_cap = T / 3 + 16;  // a job has >= 3 members
    b->d_jobs2.ensure(sizeof(Job) * b->jobs2_cap);
    const uint32_t key_min = (uint32_t)std::max(b->tune.heavy_min, 2);
    b->d_hv_keys.ensure(sizeof(HeavyKey) * (Sp / key_min + 16));
    b->d_hv_rec.ensure(8 * Sp);
    b->d_hv_len.ensure(4 * Sp);
    b->d_hv_s0.ensure(4 * Sp);
    b->d_hv_s1.ensure(4 * Sp);
    b->d_ovf2.ensure(sizeof(OvfEntry) * std::max<uint64_t>(b->ovf_cap, 1));
    if (b->overlap) b->d_ovf2b.ensure(sizeof(OvfEntry) * std::max<uint64_t>(b->ovf_cap, 1));
    b->d_plan.ensure(4 * PLAN_SLOTS * 2);
    b->d_run.ensure(8 * RUN_SLOTS);
    b->d_sub_tab.ensure(4ull * (1u << b->b1_bits) * SUB_TAB);
    b->d_stamps.ensure(32 * 8);
    // job sort scratch; the long jobs (>= 2^class samples each) bound the plan offsets
    const int cls = std::max(1, std::min(b->tune.main_long_class, b->tune.ovf_long_class));
    struct {
        ChainSet* cs;
        uint64_t cap, elems;
    } sets[2] = {{&b->cs_main, b->jobs_cap, b->cap_local}, {&b->cs_ovf, b->jobs2_cap, T}};
    for (auto& c : sets) {
        c.cs->hist.ensure(4ull * JOB_NWG * JOB_CLASSES);
        c.cs->offs.ensure(8ull * JOB_NWG * JOB_CLASSES + 16);
        c.cs->sorted.ensure(sizeof(Job) * c.cap);
        c.cs->long_off.ensure(8ull * (std::min(c.cap, (c.elems >> cls) + 16) + 8));
    }
    if (b->pass_bits) {
        // every long job has >= 2^class distinct samples of this shard's elements (received ones:
        // bounded by the world's)
        b->long_jobs_cap = std::max<uint64_t>(b->long_jobs_cap, b->world * (b->valid_total >> cls) + 4096);
        b->d_long_jobs.ensure(sizeof(Job) * b->long_jobs_cap);
        b->d_long_arena.ensure(4 * std::max<uint64_t>(b->long_cap, 1));
    }
    const uint32_t NP = 1u << b->pass_bits;
    if (giant_class(b) > 0) {
        while (b->gsamples.size() < NP) {
            b->gsamples.emplace_back();
            b->gjobs.emplace_back();
            b->gcount.emplace_back();
        }
        for (uint32_t p = 0; p < NP; ++p) {
            b->gsamples[p].ensure(4 * giant_cap(b));
            b->gjobs[p].ensure(sizeof(Job) * (giant_cap(b) / (1u << giant_class(b)) + 16));
            b->gcount[p].ensure(16);
        }
    }
}

// run start: arena cursor, signature flags, run slots; the pass ids (one residue scan)
void begin_run(skm_build* b) {
    hipStream_t st = b->stream;
    alloc_caps(b);
    b->chainq_next = 0;
    b->emit_q = -1;  // no pass group's positions are queued from an earlier (possibly aborted) run
    b->giant_timed = false;
    b->tail_pending = false;
    b->tail_issue = nullptr;
    SKM_HIP(hipEventRecord(b->ev_start, st));
    SKM_HIP(hipMemsetAsync(b->d_ctr.p, 0, 3 * 256, st));
    b->ovf_pending[0] = b->ovf_pending[1] = false;
    SKM_HIP(hipMemsetAsync(b->d_run.p, 0, 8 * RUN_SLOTS, st));
    SKM_HIP(hipMemsetAsync(b->d_flags.p, 0, b->n_total ? b->n_total : 1, st));
    if (b->tune.flag_bits) SKM_HIP(hipMemsetAsync(b->d_flagbits.p, 0, 4 * ((b->n_total + 31) / 32 + 1), st));
    b->d_gstat.ensure(16);
    SKM_HIP(hipMemsetAsync(b->d_gstat.p, 0, 16, st));
    if (b->tune.poison_jobs && b->pass_bits && b->long_jobs_cap)
        hipLaunchKernelGGL(k_poison_jobs, dim3(256), dim3(256), 0, st, b->d_long_jobs.as<Job>(), b->long_jobs_cap,
                           reinterpret_cast<uint64_t>(b->d_long_arena.p), (uint32_t)b->kept_cap,
                           b->d_data.as<skm_stored_kmer_data>());
    if (b->pass_bits) {
        const uint32_t P = 1u << b->pass_bits;
        // every window's pass id and every workgroup's windows per pass (k_pass_emit's input and offsets)
        SKM_LAUNCH(b, k_pass_ids, dim3(b->sel_wg), dim3(256), 4u * P + (b->route ? (1u << BLOOM_BITS) / 8 : 0u), st,
                   b->d_res.as<uint8_t>(), b->rp, b->pass_bits, 0, b->d_ids.as<uint8_t>(), nullptr,
                   b->route ? b->d_bloom.as<uint32_t>() : nullptr, P, b->d_selrows.as<uint32_t>(), b->sel_span,
                   route_arg(b));
        SKM_LAUNCH(b, k_sel_scan, dim3(P), dim3(1024), 0, st, b->d_selrows.as<uint32_t>(), b->sel_wg, P,
                   b->d_seloff.as<uint64_t>(), b->d_npos.as<unsigned long long>(), b->pass_max,
                   b->d_run.as<unsigned long long>());
    }
    SKM_HIP(hipGetLastError());
    b->acc = skm_build::Acc{};
    b->kt_used = 0;
    b->kt_recs.clear();
    std::memset(b->pass_ms, 0, sizeof(b->pass_ms));
    for (bool& g : b->gused) g = false;
    for (bool& g : b->chain_used) g = false;
    b->n_kept = 0;
}

// the pass's timing events (one set per pass: read once, after the step's single host sync)
void use_evset(skm_build* b, uint32_t pass) {
    while (b->evsets.size() <= pass) {
        b->evsets.emplace_back();
        skm_build::EvSet& e = b->evsets.back();
        for (auto& x : e.ev) SKM_HIP(hipEventCreate(&x));
        for (auto& x : e.o) SKM_HIP(hipEventCreate(&x));
        for (auto& x : e.o3) SKM_HIP(hipEventCreate(&x));
    }
    b->ev = b->evsets[pass].ev;
    b->ev_o = b->evsets[pass].o;
    b->ev_o3 = b->evsets[pass].o3;
}

// after the step's sync: phase times of every pass
void pass_times(skm_build* b, uint32_t npass) {
    // [0] extract-count [1] scan [2] extract-scatter [3] bucket [5] chains [8] exchange
    // [9] partition [10] group-by kernel [11] big groups; [4] overflow (own streams)
    const int idx[9] = {0, 1, 2, 3, 5, 8, 9, 10, 11};
    const int from[9] = {0, 1, 2, 4, 12, 3, 4, 11, 5}, to[9] = {1, 2, 3, 12, 6, 4, 10, 5, 12};
    for (uint32_t p = 0; p < npass && p < b->evsets.size(); ++p) {
        const skm_build::EvSet& e = b->evsets[p];
        for (int i = 0; i < 9; ++i) {
            float t = 0.f;
            SKM_HIP(hipEventElapsedTime(&t, e.ev[from[i]], e.ev[to[i]]));
            b->pass_ms[idx[i]] += t;
        }
        float t2 = 0.f, t3 = 0.f;  // the overflow path end to end (both parts, their chains included)
        SKM_HIP(hipEventElapsedTime(&t2, e.o[0], e.o[2]));
        SKM_HIP(hipEventElapsedTime(&t3, e.o[0], e.o3[1]));
        b->pass_ms[4] += std::max(t2, t3);
    }
}

// key-range passes: run the stashed long chains not yet launched, as one batch on the chain
// stream.  The batch's job range is taken on st (k_long_snap), in stream order after the passes so
// far -- whose overflow stashes st already waited for -- and before the next pass reserves more.
// Batches go to the chain stream, or rotate over it and the giant-chain streams (chain_streams
// option).  A batch lasts as long as its longest chain, so on one stream the batches queue behind
// each other -- which measured better at C3 (four batches: 2.46 s vs 2.50 s rotating over four
// streams): fewer FP64 chain waves compete with the pass kernels.
hipStream_t chain_stream(skm_build* b, int slot) {
    const int k = slot % std::max(1, std::min(b->tune.chain_streams, 1 + skm_build::GSLOTS));
    return k == 0 ? b->chain_st : b->gst[k - 1];
}

void flush_long_chains(skm_build* b, int slot) {
    join_tail(b);  // the stash of the last pass's chains (k_long_stash) is part of its tail
    unsigned long long* run_d = b->d_run.as<unsigned long long>();
    unsigned long long* rng = run_d + RUN_SNAP + 2 * slot;
    SKM_LAUNCH(b, k_long_snap, dim3(1), dim3(1), 0, b->stream, run_d, rng, b->long_jobs_cap);
    SKM_HIP(hipEventRecord(b->chain_ev[0], b->stream));
    hipStream_t cs = chain_stream(b, slot);
    SKM_HIP(hipStreamWaitEvent(cs, b->chain_ev[0], 0));
    b->chain_used[slot % std::max(1, std::min(b->tune.chain_streams, 1 + skm_build::GSLOTS))] = true;
    // the batch's chains below lane_long samples one lane each (k_chains: 64 chains per wave, ~50x
    // less wave time per sample than a wave pair, ~2.5x the latency), the rest on wave pairs; in
    // the last batch (slot 16, the tail after the last pass) only those below lane_tail -- and with
    // fewer than 8 passes in every batch (a batch then has at most a few passes to hide a lane
    // chain's latency behind: the multi-GPU shapes, 1-4 passes per rank)
    const bool few = (1 << b->pass_bits) < 8;
    const int lmax = slot < 16 && !few ? b->tune.lane_long : std::min(b->tune.lane_long, b->tune.lane_tail);
    const uint32_t lane_max = lmax > 0 ? (uint32_t)lmax : 0u;
    if (!(b->tune.diag & 4) && !(b->tune.diag & 8))
        SKM_LAUNCH(b, k_chain_long, dim3(LONG_GRID), dim3(128), 0, cs, b->d_long_jobs.as<Job>(), rng, rng + 1,
                   nullptr, nullptr, nullptr, nullptr, b->d_data.as<skm_stored_kmer_data>(), b->tune.chain_prio,
                   lane_max);
    if (lane_max && !(b->tune.diag & 4) && !(b->tune.diag & 8)) {
        // a batch lasts as long as its longest chain: batches rotate over lane_streams streams so a
        // batch of giant chains does not hold back the next one
        const int ls = slot % std::max(1, std::min(b->tune.lane_streams, (int)skm_build::LANE_ST));
        hipStream_t lst = b->lane_st[ls];
        SKM_HIP(hipStreamWaitEvent(lst, b->chain_ev[0], 0));
        unsigned long long* q = chain_queue(b, lst);
        SKM_LAUNCH(b, k_chains_stash, dim3((uint32_t)std::max(1, b->tune.lane_grid)), dim3(256), 0, lst,
                   b->d_long_jobs.as<Job>(), rng, rng + 1, b->long_jobs_cap, b->d_data.as<skm_stored_kmer_data>(),
                   lane_max, q);
        b->lane_used[ls] = true;
    }
    SKM_HIP(hipGetLastError());
}

// per-rank statistics over the whole arena (distinct_functions) and the shard (seqs_with_func)
void phase_stats(skm_build* b) {
    hipStream_t st = b->stream;
    const uint32_t F = b->opts.n_functions;
    SKM_HIP(hipEventRecord(b->ev_tail[0], st));  // the last pass is issued: the tail starts here
    join_tail(b);
    drain_overflow(b);
    if (b->tune.flag_bits && b->n_total)
        SKM_LAUNCH(b, k_flags_from_bits, dim3(1024), dim3(256), 0, st, b->d_flagbits.as<uint32_t>(),
                   (uint32_t)b->n_total, b->d_flags.as<uint8_t>());
    // the arena's keys decoded and distinct_functions counted while the last chains run: neither
    // reads what the chains write (the records' median / var), and every pass's kept k-mers are in
    // the arena once the main stream is here
    SKM_HIP(hipMemsetAsync(b->d_dfunc.p, 0, sizeof(uint32_t) * (F ? F : 1), st));
    SKM_HIP(hipMemsetAsync(b->d_swf.p, 0, sizeof(uint32_t) * (F ? F : 1), st));
    const size_t lds_f = F <= 16384 ? sizeof(uint32_t) * F : 0;
    if (b->pass_bits) flush_long_chains(b, 16);  // the last batch of long chains first, on the chain streams
    SKM_LAUNCH(b, k_kept_finalize, dim3(2048), dim3(256), lds_f, st, b->d_keys.as<uint64_t>(),
                       b->d_data.as<skm_stored_kmer_data>(), b->d_ctr.as<unsigned long long>(), F,
                       b->d_dfunc.as<uint32_t>());
    if (b->nseq)
        SKM_LAUNCH(b, k_func_hist_seqs, dim3(256), dim3(256), lds_f, st, b->d_meta.as<SeqMeta>(), b->nseq, F,
                           b->d_swf.as<uint32_t>());
    if (b->pass_bits) {  // the long chains of every pass (the last batch on the chain stream)
        for (int k = 0; k < skm_build::LANE_ST; ++k) {
            if (!b->lane_used[k]) continue;
            SKM_HIP(hipEventRecord(b->lane_ev[k], b->lane_st[k]));
            SKM_HIP(hipStreamWaitEvent(st, b->lane_ev[k], 0));
            b->lane_used[k] = false;
        }
        for (int k = 0; k <= skm_build::GSLOTS; ++k) {
            if (!b->chain_used[k]) continue;
            const hipStream_t cs = chain_stream(b, k);
            hipEvent_t e = k == 0 ? b->chain_ev[2] : b->gev_done[k - 1];
            SKM_HIP(hipEventRecord(e, cs));
            SKM_HIP(hipStreamWaitEvent(st, e, 0));
        }
    }
    for (int g = 0; g < skm_build::GSLOTS; ++g)  // the giant chains of every pass
        if (b->gused[g]) SKM_HIP(hipStreamWaitEvent(st, b->gev_done[g], 0));
    SKM_HIP(hipEventRecord(b->ev_tail[1], st));
    SKM_HIP(hipEventRecord(b->ev[7], st));
    SKM_HIP(hipGetLastError());
}

// the step's one host synchronisation: counters, run slots and timings come back together
void phase_final(skm_build* b) {
    hipStream_t st = b->stream;
    SKM_LAUNCH(b, k_count_flags, dim3(256), dim3(256), 0, st, b->d_flags.as<uint8_t>(), b->n_total,
                       b->d_ctr.as<unsigned long long>() + 2);
    SKM_HIP(hipGetLastError());
    unsigned long long* pin = b->pinned_ctr();
    SKM_HIP(hipMemcpyAsync(pin + 48, b->d_gstat.p, 16, hipMemcpyDeviceToHost, st));
    SKM_HIP(hipMemcpyAsync(pin + 56, b->d_ctr.p, 8, hipMemcpyDeviceToHost, st));
    SKM_HIP(hipMemcpyAsync(pin + 64, b->d_run.p, 8 * RUN_SLOTS, hipMemcpyDeviceToHost, st));
    const bool canary = b->tune.poison_jobs && b->pass_bits && b->long_jobs_cap;
    if (canary)
        SKM_HIP(hipMemcpyAsync(pin + 42, b->d_data.as<skm_stored_kmer_data>() + b->kept_cap,
                               sizeof(skm_stored_kmer_data), hipMemcpyDeviceToHost, st));
    SKM_HIP(hipEventRecord(b->ev[8], st));
    SKM_HIP(hipEventSynchronize(b->ev[8]));
    const unsigned long long* R = pin + 64;
    b->giant_jobs = pin[48];
    b->giant_max = pin[49];
    b->n_kept = pin[56];
    b->run_flags = R[RUN_FLAGS];
    if (canary) {  // a chain ran on a long-job slot that no stash wrote
        const auto* c = reinterpret_cast<const skm_stored_kmer_data*>(pin + 42);
        if (c->median != 0xC0DE || c->var != 0xC0DE) b->run_flags |= RUN_F_CAP;
    }
    for (int i = 0; i < 4; ++i) b->demand[i] = R[RUN_DEM_TOT + i];
    // what the passes asked of the long arena and job list (the reservations that did not fit included)
    b->demand[2] = std::max<uint64_t>(b->demand[2], R[RUN_LONG_WANT]);
    b->demand[3] = std::max<uint64_t>(b->demand[3], R[RUN_LONG_WANTJ]);
    pass_times(b, 1u << b->pass_bits);
    for (int i = 0; i < 12; ++i) b->last_ms[i] = b->pass_ms[i];
    SKM_HIP(hipEventElapsedTime(&b->last_ms[6], b->ev[7], b->ev[8]));      // stats (+ reductions)
    SKM_HIP(hipEventElapsedTime(&b->last_ms[7], b->ev_start, b->ev[8]));   // whole run
    SKM_HIP(hipEventElapsedTime(&b->last_ms[12], b->ev_tail[0], b->ev_tail[1]));  // long-chain tail
    b->last_ms[13] = b->last_ms[14] = -1.0f;  // the first giant chains' start / end from the run's start
    if (b->giant_timed) {
        SKM_HIP(hipEventElapsedTime(&b->last_ms[13], b->ev_start, b->ev_giant[0]));
        SKM_HIP(hipEventElapsedTime(&b->last_ms[14], b->ev_start, b->ev_giant[1]));
    }
    b->long_samples = R[RUN_LONG_CUR];
    kt_collect(b);
    // run totals for counters() / finish()
    b->n_overflow = (uint32_t)R[RUN_ACC_NOVF];
    b->n_overflow_last = (uint32_t)R[RUN_LAST_NOVF];
    b->n_jobs = R[RUN_ACC_JOBS];
    b->n_jobs_last = R[RUN_LAST_JOBS];
    b->n_lens = R[RUN_ACC_LENS];
    b->ovf_elems = R[RUN_ACC_OVF_ELEMS];
    b->ovf_kept = R[RUN_ACC_OVF_KEPT];
    b->n_big = R[RUN_ACC_BIG];
    b->big_kept = R[RUN_ACC_BIG_KEPT];
    b->n_local = R[RUN_ACC_GROUPED];
    b->ran = true;
}

// a redo: capacities grown to the recorded demands (with slack), buffers reallocated
void grow_caps(skm_build* b) {
    auto grow = [](uint64_t& cap, uint64_t dem) {
        if (dem > cap) cap = dem + dem / 8 + 1024;
    };
    grow(b->tot_cap, b->demand[0]);
    grow(b->split_cap, b->demand[1]);
    grow(b->long_cap, b->demand[2]);
    grow(b->long_jobs_cap, b->demand[3]);
    SKM_HIP(hipDeviceSynchronize());
    alloc_caps(b);
}

void run_once(const Ranks& bs) {
    for (auto* b : bs) begin_run(b);
    const uint32_t P = 1u << bs[0]->pass_bits;
    for (uint32_t pass = 0; pass < P; ++pass) {
        for (auto* b : bs) {
            use_evset(b, pass);
            phase_extract(b, pass);
        }
        if (bs[0]->world > 1) exchange(bs, pass);
        for (auto* b : bs) {
            phase_group(b, pass);
            // the stashed long chains leave in batches (default two: the first half's chains
            // overlap the second half); the last batch runs after the last pass (phase_stats)
            // (two passes -- the world > 1 shape with routing -- flush after the first: the routed
            // heavy keys' chains then run beside the second pass instead of after it)
            const uint32_t nb = std::min<uint32_t>(P >= 2 ? std::min<uint32_t>(P, (uint32_t)std::max(1, b->tune.chain_batches)) : 1u, 16u);
            const uint32_t per = std::max<uint32_t>(1u, P / nb);
            if (nb > 1 && (pass + 1) % per == 0 && pass + 1 < P) {
                drain_overflow(b);  // the snapshot takes every stash issued so far, complete
                flush_long_chains(b, (int)((pass + 1) / per - 1));
            }
        }
    }
    for (auto* b : bs) phase_stats(b);
    if (bs[0]->world > 1) {
        std::vector<void*> df, sw, fl;
        for (auto* b : bs) {
            df.push_back(b->d_dfunc.p);
            sw.push_back(b->d_swf.p);
            fl.push_back(b->d_flags.p);
        }
        const uint32_t F = bs[0]->opts.n_functions;
        allreduce(bs, df, F, Red::SumU32);
        allreduce(bs, sw, F, Red::SumU32);
        allreduce(bs, fl, bs[0]->n_total, Red::MaxU8);
    }
    for (auto* b : bs) phase_final(b);
}

void run_ranks(const Ranks& bs) {
    prepare(bs);
    for (int attempt = 0;; ++attempt) {
        run_once(bs);
        std::vector<uint64_t> mine;
        for (auto* b : bs) mine.push_back((b->run_flags & RUN_F_RERUN) ? 1u : 0u);
        const std::vector<uint64_t> all = bs[0]->world > 1 ? allgather_u64(bs, mine) : mine;
        bool redo = false;
        for (auto v : all) redo |= v != 0;
        if (!redo) break;
        SKM_CHECK(attempt < 3, SKM_E_STATE, "build work buffers did not converge");
        for (auto* b : bs) {
            grow_caps(b);
            ++b->n_redo;
        }
    }
    for (auto* b : bs) {
        SKM_CHECK(!(b->run_flags & RUN_F_ARENA), SKM_E_OOM,
                  "kept k-mer arena exhausted (raise the device memory budget or the key-range passes)");
        SKM_CHECK(!(b->run_flags & RUN_F_CAP), SKM_E_STATE, "build work list capacity exceeded");
    }
}

Ranks ranks_of(skm_build* b) {
    if (!b->group.empty()) return b->group;
    return Ranks{b};
}

}  // namespace

// A build drives up to 10 streams at once (group-by, two overflow streams, the pass tail, the
// next group's emission, the stashed-chain stream and the giant-chain slots).  HIP maps streams
// onto GPU_MAX_HW_QUEUES hardware queues (default 4); streams sharing a queue execute in order,
// which would serialise a pass behind the previous pass's long chains.  Ask for at least 16, as
// bench.py and the tests run with (read at HIP init, so this only takes effect when libskm is
// loaded before the first HIP call; the CLIs set it themselves).
__attribute__((constructor)) static void skm_hw_queues() {
    const char* q = getenv("GPU_MAX_HW_QUEUES");
    if (!q || atoi(q) < 16) setenv("GPU_MAX_HW_QUEUES", "16", 1);
}

extern "C" {

int skm_build_create(skm_build** out, const int* devices, int n_devices, const skm_build_opts* opts) {
    SKM_API_BEGIN
    SKM_CHECK(out && opts, SKM_E_ARG, "null argument");
    SKM_CHECK(opts->k == 8, SKM_E_ARG, "only k = 8 is supported (kmers-build-signatures.cc:17)");
    SKM_CHECK(opts->n_functions < 0xFFFFu, SKM_E_ARG, "n_functions must be < 65535");
    SKM_CHECK(n_devices == 1, SKM_E_ARG, "one device per process (multi-GPU: one process per GPU)");
    const int ws = std::max(1, opts->world_size);
    SKM_CHECK(ws <= 64 && (ws & (ws - 1)) == 0, SKM_E_ARG, "world_size must be a power of two <= 64");
    SKM_CHECK(opts->rank >= 0 && opts->rank < ws, SKM_E_ARG, "rank out of range");
    int ndev = 0;
    SKM_HIP(hipGetDeviceCount(&ndev));
    SKM_CHECK(ndev > 0, SKM_E_HIP, "no HIP device");
    auto* b = new skm_build();
    b->opts = *opts;
    b->opts.world_size = ws;
    b->device = devices ? devices[0] : 0;
    SKM_HIP(hipSetDevice(b->device));
    SKM_HIP(hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking));
    SKM_HIP(hipStreamCreateWithFlags(&b->stream2, hipStreamNonBlocking));
    SKM_HIP(hipStreamCreateWithFlags(&b->stream3, hipStreamNonBlocking));
    SKM_HIP(hipStreamCreateWithFlags(&b->stream_tail, hipStreamNonBlocking));
    SKM_HIP(hipStreamCreateWithFlags(&b->stream_tail2, hipStreamNonBlocking));
    SKM_HIP(hipEventCreateWithFlags(&b->ev_tail2, hipEventDisableTiming));
    SKM_HIP(hipEventCreateWithFlags(&b->ev_tail_bp, hipEventDisableTiming));
    SKM_HIP(hipEventCreateWithFlags(&b->ev_tail_done, hipEventDisableTiming));
    SKM_HIP(hipEventCreateWithFlags(&b->ev_scan, hipEventDisableTiming));
    use_evset(b, 0);
    SKM_HIP(hipEventCreate(&b->ev_start));
    SKM_HIP(hipStreamCreateWithFlags(&b->chain_st, hipStreamNonBlocking));
    for (int k = 0; k < skm_build::LANE_ST; ++k) {
        SKM_HIP(hipStreamCreateWithFlags(&b->lane_st[k], hipStreamNonBlocking));
        SKM_HIP(hipEventCreateWithFlags(&b->lane_ev[k], hipEventDisableTiming));
    }
    SKM_HIP(hipStreamCreateWithFlags(&b->stx, hipStreamNonBlocking));
    SKM_HIP(hipEventCreateWithFlags(&b->ev_staged, hipEventDisableTiming));
    SKM_HIP(hipEventCreateWithFlags(&b->ev_emit, hipEventDisableTiming));
    for (int g = 0; g < skm_build::GSLOTS; ++g) {
        SKM_HIP(hipStreamCreateWithFlags(&b->gst[g], hipStreamNonBlocking));
        SKM_HIP(hipEventCreateWithFlags(&b->gev_ready[g], hipEventDisableTiming));
        SKM_HIP(hipEventCreateWithFlags(&b->gev_done[g], hipEventDisableTiming));
    }
    for (auto& e : b->chain_ev) SKM_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    SKM_HIP(hipEventCreateWithFlags(&b->ev_part, hipEventDisableTiming));
    SKM_HIP(hipEventCreateWithFlags(&b->ev_part_heavy, hipEventDisableTiming));
    for (int k = 0; k < 2; ++k) {
        SKM_HIP(hipEventCreateWithFlags(&b->ev_ovf_done[k], hipEventDisableTiming));
        SKM_HIP(hipEventCreateWithFlags(&b->ev_main_done[k], hipEventDisableTiming));
    }
    for (auto& e : b->ev_tail) SKM_HIP(hipEventCreate(&e));
    for (auto& e : b->ev_giant) SKM_HIP(hipEventCreate(&e));
    for (int i = 0; i < 2; ++i) {
        SKM_HIP(hipHostMalloc(reinterpret_cast<void**>(&b->st_pin[i]), STAGE_BYTES, hipHostMallocDefault));
        SKM_HIP(hipEventCreateWithFlags(&b->st_ev[i], hipEventDisableTiming));
    }
    SKM_HIP(hipEventCreateWithFlags(&b->ev_split, hipEventDisableTiming));
    set_geometry(b);
    *out = b;
    SKM_API_END
}

int skm_build_add_batch(skm_build* b, const uint8_t* residues, const uint64_t* seq_off, const uint32_t* seq_len,
                        const uint16_t* seq_func, const uint32_t* seq_id, size_t n_seqs) {
    SKM_API_BEGIN
    SKM_CHECK(b, SKM_E_ARG, "null build");
    SKM_CHECK(n_seqs == 0 || (residues && seq_off && seq_len && seq_func), SKM_E_ARG, "null array");
    SKM_HIP(hipSetDevice(b->device));
    const auto t0 = std::chrono::steady_clock::now();
    // the batch's kept sequences (signature_build.tcc:155-158 skips the others), validated
    std::vector<uint32_t>& ks = b->h_keep;
    ks.clear();
    for (size_t s = 0; s < n_seqs; ++s) {
        const uint16_t f = seq_func[s];
        if (f == SKM_UNDEFINED_FUNCTION) continue;
        SKM_CHECK(f < b->opts.n_functions, SKM_E_ARG, "seq_func out of range");
        SKM_CHECK(seq_len[s] < (1u << ELEM_I_BITS), SKM_E_ARG, "protein longer than 1,048,575 residues");
        ks.push_back((uint32_t)s);
    }
    if (b->h_meta.capacity() < b->h_meta.size() + ks.size()) {  // geometric growth without skm_build_reserve
        b->h_meta.reserve(std::max(b->h_meta.size() + ks.size(), 2 * b->h_meta.capacity()));
        b->h_seqid.reserve(std::max(b->h_seqid.size() + ks.size(), 2 * b->h_seqid.capacity()));
    }
    // Segments that fit the current pinned staging buffer: their metadata and residues written by
    // the host pool in byte-balanced parts (the packing used to be one memcpy per sequence on one
    // thread, ~2 GB/s: 8 s of a C3 one-shot build); the DMA of the other staging buffer overlaps.
    if (!b->pool) b->pool.reset(new HostPool(HostPool::default_threads()));
    std::vector<uint64_t>& cum = b->h_cum;
    size_t i = 0;
    while (i < ks.size()) {
        const size_t room = STAGE_BYTES - b->st_fill[b->st_cur];
        size_t j = i;
        uint64_t bytes = 0;
        cum.clear();
        while (j < ks.size() && bytes + seq_len[ks[j]] + 1 <= room) {
            cum.push_back(bytes);
            bytes += seq_len[ks[j]] + 1;
            ++j;
        }
        if (j == i) {  // the buffer is full: hand it to the DMA engine
            stage_flush(b);
            continue;
        }
        cum.push_back(bytes);
        // the segment's metadata and residues, both by the pool over the same byte-balanced
        // sequence ranges (a serial metadata loop cost ~0.5 s of a C3 add at 50 M sequences)
        const size_t nseg = j - i, m0 = b->h_meta.size();
        b->h_meta.resize(m0 + nseg);
        b->h_seqid.resize(m0 + nseg);
        if (m0 && (seq_id ? seq_id[ks[i]] : (uint32_t)m0) <= b->h_seqid[m0 - 1]) b->seqid_strict = false;
        uint8_t* base = b->st_pin[b->st_cur] + b->st_fill[b->st_cur];
        const int parts = bytes >= (1u << 18) ? std::min<int>(4 * b->pool->threads(), (int)(bytes >> 16)) : 1;
        std::atomic<uint64_t> nwin{0};
        std::atomic<bool> strict{true};
        const auto tp = std::chrono::steady_clock::now();
        b->pool->run(parts, [&](int p) {
            const uint64_t lo = bytes * (uint64_t)p / (uint64_t)parts, hi = bytes * (uint64_t)(p + 1) / (uint64_t)parts;
            const size_t a = (size_t)(std::lower_bound(cum.begin(), cum.begin() + nseg, lo) - cum.begin());
            const size_t e = (size_t)(std::lower_bound(cum.begin(), cum.begin() + nseg, hi) - cum.begin());
            uint64_t w = 0;
            bool st = true;
            for (size_t k = a; k < e; ++k) {
                const uint32_t s = ks[i + k];
                SeqMeta& m = b->h_meta[m0 + k];
                m.pstart = b->rp_total + cum[k];
                m.len = seq_len[s];
                m.func = seq_func[s];
                m.pad = 0;
                const uint32_t sid = seq_id ? seq_id[s] : (uint32_t)(m0 + k);
                if (seq_id && k > 0 && sid <= seq_id[ks[i + k - 1]]) st = false;
                b->h_seqid[m0 + k] = sid;
                if (m.len >= 8) w += m.len - 7;
                uint8_t* dst = base + cum[k];
                std::memcpy(dst, residues + seq_off[s], seq_len[s]);
                dst[seq_len[s]] = 0;
            }
            nwin.fetch_add(w, std::memory_order_relaxed);
            if (!st) strict.store(false, std::memory_order_relaxed);
        });
        b->add_pack_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - tp).count();
        b->n_windows += nwin.load();
        if (!strict.load()) b->seqid_strict = false;
        b->st_fill[b->st_cur] += bytes;
        b->rp_total += bytes;
        i = j;
    }
    b->prepared = false;
    b->ran = false;
    b->add_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    SKM_API_END
}

int skm_build_reserve(skm_build* b, uint64_t n_residues, uint64_t n_seqs) {
    SKM_API_BEGIN
    SKM_CHECK(b, SKM_E_ARG, "null build");
    SKM_HIP(hipSetDevice(b->device));
    res_reserve(b, n_residues + n_seqs + 64);
    b->h_meta.reserve(n_seqs);
    b->h_seqid.reserve(n_seqs);
    SKM_API_END
}

static void check_transport(skm_build* b) {
#if defined(SKM_WITH_RCCL)
    const bool comm = b->comm != nullptr;
#else
    const bool comm = false;
#endif
    SKM_CHECK(b->world == 1 || comm || !b->group.empty() || b->tp.alltoallv, SKM_E_STATE,
              "world_size > 1 needs skm_build_set_comm, skm_build_set_transport or skm_build_group_run first");
}

int skm_build_prepare(skm_build* b) {
    SKM_API_BEGIN
    SKM_CHECK(b, SKM_E_ARG, "null build");
    check_transport(b);
    SKM_HIP(hipSetDevice(b->device));
    prepare(ranks_of(b));
    SKM_API_END
}

int skm_build_run(skm_build* b) {
    SKM_API_BEGIN
    SKM_CHECK(b, SKM_E_ARG, "null build");
    check_transport(b);
    SKM_HIP(hipSetDevice(b->device));
    run_ranks(ranks_of(b));
    SKM_API_END
}

int skm_build_group_run(skm_build* const* bs, int n) {
    SKM_API_BEGIN
    SKM_CHECK(bs && n >= 1, SKM_E_ARG, "null argument");
    Ranks g(bs, bs + n);
    for (int r = 0; r < n; ++r) {
        SKM_CHECK(g[r], SKM_E_ARG, "null build");
        SKM_CHECK(g[r]->world == n && g[r]->rank == r, SKM_E_ARG, "group member r must have rank r and world_size n");
    }
    for (auto* b : g) b->group = n > 1 ? g : Ranks{};
    SKM_HIP(hipSetDevice(g[0]->device));
    run_ranks(n > 1 ? g : Ranks{g[0]});
    SKM_API_END
}

int skm_comm_unique_id(uint8_t id[128]) {
    SKM_API_BEGIN
    SKM_CHECK(id, SKM_E_ARG, "null argument");
#if defined(SKM_WITH_RCCL)
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId must be 128 bytes");
    ncclUniqueId u;
    SKM_NCCL(ncclGetUniqueId(&u));
    std::memcpy(id, &u, 128);
#else
    std::memset(id, 0, 128);
    throw Error(SKM_E_COMM, "libskm was built without RCCL");
#endif
    SKM_API_END
}

int skm_build_set_transport(skm_build* b, const skm_transport* tp) {
    SKM_API_BEGIN
    SKM_CHECK(b && tp && tp->alltoallv && tp->allreduce && tp->allgatherv, SKM_E_ARG, "incomplete transport");
#if defined(SKM_WITH_RCCL)
    SKM_CHECK(b->comm == nullptr, SKM_E_STATE, "an RCCL communicator is already set");
#endif
    b->tp = *tp;
    SKM_API_END
}

int skm_debug_exchange_plan(const skm_transport* tp, int rank, int world, uint32_t nb1, const uint64_t* bucket_starts,
                            uint64_t* recv_off, uint64_t* recv_cnt, uint64_t* vstart) {
    SKM_API_BEGIN
    SKM_CHECK(tp && tp->alltoallv && bucket_starts && recv_off && recv_cnt && vstart && world >= 1 && rank >= 0 &&
                  rank < world && nb1 >= 1, SKM_E_ARG, "bad argument");
    const SendPlan sp = plan_send(bucket_starts, world, nb1);
    std::vector<uint64_t> off(world), c(world, 4ull * nb1);
    for (int q = 0; q < world; ++q) off[q] = 4ull * nb1 * q;
    std::vector<uint32_t> rc((uint64_t)world * nb1);
    tp_alltoallv_host(*tp, world, reinterpret_cast<const uint8_t*>(sp.cnt.data()), off, c,
                      reinterpret_cast<uint8_t*>(rc.data()), off, c);
    const RecvPlan rp = plan_recv(rc.data(), world, nb1);
    for (int q = 0; q < world; ++q) {
        recv_off[q] = rp.off[q];
        recv_cnt[q] = rp.n[q];
    }
    for (uint32_t k = 0; k <= nb1; ++k) vstart[k] = rp.vstart[k];
    SKM_API_END
}

int skm_debug_transport_check(const skm_transport* tp, int rank, int world) {
    SKM_API_BEGIN
    SKM_CHECK(tp && tp->alltoallv && tp->allreduce && tp->allgatherv && world >= 1 && rank >= 0 && rank < world,
              SKM_E_ARG, "bad argument");
    // allreduce: u32 sums wrap mod 2^32, u8 max
    std::vector<uint32_t> u(1000);
    for (uint32_t i = 0; i < u.size(); ++i) u[i] = 0x80000000u + (uint32_t)rank * 7u + i;
    tp_check(tp->allreduce(tp->ctx, u.data(), u.size(), 0), "allreduce");
    for (uint32_t i = 0; i < u.size(); ++i) {
        uint32_t want = 0;
        for (int r = 0; r < world; ++r) want += 0x80000000u + (uint32_t)r * 7u + i;
        SKM_CHECK(u[i] == want, SKM_E_COMM, "allreduce(u32 sum) mismatch");
    }
    std::vector<uint8_t> m(300);
    for (uint32_t i = 0; i < m.size(); ++i) m[i] = (uint8_t)((i * 31u + (uint32_t)rank * 101u) & 0xFFu);
    tp_check(tp->allreduce(tp->ctx, m.data(), m.size(), 1), "allreduce");
    for (uint32_t i = 0; i < m.size(); ++i) {
        uint8_t want = 0;
        for (int r = 0; r < world; ++r) want = std::max<uint8_t>(want, (uint8_t)((i * 31u + (uint32_t)r * 101u) & 0xFFu));
        SKM_CHECK(m[i] == want, SKM_E_COMM, "allreduce(u8 max) mismatch");
    }
    // allgatherv: rank r contributes 3r + 1 bytes of value r + 1
    std::vector<uint64_t> bytes(world), o(world + 1, 0);
    for (int r = 0; r < world; ++r) {
        bytes[r] = 3u * r + 1u;
        o[r + 1] = o[r] + bytes[r];
    }
    std::vector<uint8_t> mine(bytes[rank], (uint8_t)(rank + 1)), all(o[world]);
    tp_check(tp->allgatherv(tp->ctx, mine.data(), all.data(), bytes.data()), "allgatherv");
    for (int r = 0; r < world; ++r)
        for (uint64_t j = o[r]; j < o[r + 1]; ++j) SKM_CHECK(all[j] == (uint8_t)(r + 1), SKM_E_COMM, "allgatherv mismatch");
    // alltoallv: rank p sends p*16 + q + 1 bytes of value (p * world + q) & 0xFF to rank q
    std::vector<uint64_t> sc(world), so(world), rcn(world), ro(world);
    uint64_t st = 0, rt = 0;
    for (int q = 0; q < world; ++q) {
        sc[q] = (uint64_t)rank * 16 + q + 1;
        so[q] = st;
        st += sc[q];
        rcn[q] = (uint64_t)q * 16 + rank + 1;
        ro[q] = rt;
        rt += rcn[q];
    }
    std::vector<uint8_t> sb(st), rb(rt, 0xEE);
    for (int q = 0; q < world; ++q) std::memset(sb.data() + so[q], (rank * world + q) & 0xFF, sc[q]);
    tp_check(tp->alltoallv(tp->ctx, sb.data(), sc.data(), so.data(), rb.data(), rcn.data(), ro.data()), "alltoallv");
    for (int p = 0; p < world; ++p)
        for (uint64_t j = 0; j < rcn[p]; ++j)
            SKM_CHECK(rb[ro[p] + j] == (uint8_t)((p * world + rank) & 0xFF), SKM_E_COMM, "alltoallv mismatch");
    SKM_API_END
}

int skm_build_set_comm(skm_build* b, const uint8_t id[128]) {
    SKM_API_BEGIN
    SKM_CHECK(b && id, SKM_E_ARG, "null argument");
#if defined(SKM_WITH_RCCL)
    SKM_CHECK(b->comm == nullptr, SKM_E_STATE, "communicator already set");
    SKM_HIP(hipSetDevice(b->device));
    if (b->world == 1) return SKM_OK;
    ncclUniqueId u;
    std::memcpy(&u, id, 128);
    SKM_NCCL(ncclCommInitRank(&b->comm, b->world, u, b->rank));
#else
    throw Error(SKM_E_COMM, "libskm was built without RCCL");
#endif
    SKM_API_END
}

int skm_build_set_option(skm_build* b, const char* name, int64_t value) {
    SKM_API_BEGIN
    SKM_CHECK(b && name, SKM_E_ARG, "null argument");
    const std::string n(name);
    Tune& t = b->tune;
    if (n == "key_range_passes") {
        SKM_CHECK(value >= 0 && value <= 64 && (value & (value - 1)) == 0, SKM_E_ARG,
                  "key_range_passes must be 0 (automatic) or a power of two <= 64");
        t.passes = (int)value;
    } else if (n == "stream_priority") {
        // 1: the group-by stream (the step's critical path) at the device's highest priority, so
        // its workgroups are dispatched ahead of the overflow / chain / prefetch streams' work
        SKM_CHECK(value == 0 || value == 1, SKM_E_ARG, "stream_priority must be 0 or 1");
        SKM_HIP(hipSetDevice(b->device));
        SKM_HIP(hipStreamSynchronize(b->stream));
        SKM_HIP(hipStreamDestroy(b->stream));
        int least = 0, greatest = 0;
        SKM_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
        SKM_HIP(hipStreamCreateWithPriority(&b->stream, hipStreamNonBlocking, value ? greatest : least));
        t.stream_prio = (int)value;
    } else if (n == "chain_cus" || n == "side_cus") {
        // chain_cus: the long-chain stream confined to this many CUs (0: all) -- a batch of
        // stashed long chains is thousands of two-wave workgroups whose registers would otherwise
        // keep one of the two group-by workgroups off every CU while it runs; side_cus: the same
        // for the overflow streams and the next pass's selection.  The CUs taken are the last
        // value/8 of every 32 (spread over the XCDs).
        SKM_CHECK(value >= 0 && value <= 256 && value % 8 == 0, SKM_E_ARG, (n + " must be a multiple of 8 in [0, 256]").c_str());
        SKM_HIP(hipSetDevice(b->device));
        hipDeviceProp_t prop;
        SKM_HIP(hipGetDeviceProperties(&prop, b->device));
        const uint32_t ncu = (uint32_t)prop.multiProcessorCount;
        auto remake = [&](hipStream_t& x) {
            SKM_HIP(hipStreamSynchronize(x));
            SKM_HIP(hipStreamDestroy(x));
            if (value == 0 || (uint32_t)value >= ncu) {
                SKM_HIP(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
                return;
            }
            std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
            const uint32_t per = (uint32_t)value / 8;  // per block of 32 CUs
            uint32_t taken = 0;
            for (uint32_t c = 0; c < ncu && taken < (uint32_t)value; ++c)
                if (c % 32 >= 32 - per) {
                    mask[c / 32] |= 1u << (c % 32);
                    ++taken;
                }
            SKM_HIP(hipExtStreamCreateWithCUMask(&x, (uint32_t)mask.size(), mask.data()));
        };
        if (n == "chain_cus") {  // the wave-pair chains' stream and the per-lane stash streams
            remake(b->chain_st);
            for (int k = 0; k < skm_build::LANE_ST; ++k) remake(b->lane_st[k]);
            t.chain_cus = (int)value;
        } else {
            remake(b->stream2);
            remake(b->stream3);
            remake(b->stx);
            t.side_cus = (int)value;
        }
    } else if (n == "work_buffer_elements") {
        // capacities of the data-sized work buffers (tests: force the grow-and-redo path); 0 = the
        // automatic first guess
        SKM_CHECK(value >= 0, SKM_E_ARG, "work_buffer_elements must be >= 0");
        b->tot_cap = b->split_cap = b->long_cap = (uint64_t)value;
        b->long_jobs_cap = value ? 1 : 0;
    } else if (n == "device_memory_budget_mb") {
        SKM_CHECK(value >= 0, SKM_E_ARG, "device_memory_budget_mb must be >= 0");
        t.mem_budget_mb = value;
    } else {
        int* f = n == "overflow_heavy_min" ? &t.ovf_heavy
               : n == "overflow_inline_min" ? &t.ovf_inline_min
               : n == "overflow_inline_prio" ? &t.inline_prio
               : n == "overflow_long_class" ? &t.ovf_long_class
               : n == "main_long_class" ? &t.main_long_class
               : n == "overflow_chain_wgs" ? &t.ovf_chain_wgs
               : n == "chain_prio" ? &t.chain_prio
               : n == "bucket_prio" ? &t.bucket_prio
               : n == "chain_lds_kb" ? &t.chain_lds_kb
               : n == "host_timing" ? &t.host_timing
               : n == "heavy_min" ? &t.heavy_min
               : n == "split_min" ? &t.split_min
               : n == "giant_class" ? &t.giant_class
               : n == "giant_passes" ? &t.giant_passes
               : n == "heavy_lsd" ? &t.heavy_lsd
               : n == "prefetch" ? &t.prefetch
               : n == "overflow_grid" ? &t.ovf_grid
               : n == "split_grid" ? &t.split_grid
               : n == "chain_grid" ? &t.chain_grid
               : n == "chain_batches" ? &t.chain_batches
               : n == "chain_streams" ? &t.chain_streams
               : n == "poison_jobs" ? &t.poison_jobs
               : n == "route_heavy_min" ? &t.route_heavy_min
               : n == "stage_round" ? &t.stage_round
               : n == "partition_round" ? &t.partition_round
               : n == "flag_check" ? &t.flag_check
               : n == "diag" ? &t.diag
               : n == "flag_bits" ? &t.flag_bits
               : n == "sub_target" ? &t.sub_target
               : n == "lane_long" ? &t.lane_long
               : n == "lane_grid" ? &t.lane_grid
               : n == "lane_tail" ? &t.lane_tail
               : n == "lane_streams" ? &t.lane_streams
               : n == "chain_queue" ? &t.chain_queue
               : n == "serial_overflow" ? &t.serial_overflow
               : n == "overlap" ? &t.overlap
               : n == "heavy_grid" ? &t.heavy_grid
               : n == "route_vacate" ? &t.route_vacate
               : n == "route_first" ? &t.route_first
               : n == "tail_async" ? &t.tail_async
               : n == "big_grid" ? &t.big_grid
               : n == "big_grid_large" ? &t.big_grid_large
               : n == "big_split" ? &t.big_split
               : n == "tail_defer" ? &t.tail_defer
               : n == "part_order" ? &t.part_order
               : n == "part_split" ? &t.part_split
               : n == "recs_rot" ? &t.recs_rot
               : n == "emit_group" ? &t.emit_group
               : n == "handoff_index_limit" ? &t.handoff_index_limit
               : n == "handoff_max_chunk" ? &t.handoff_max_chunk
               : n == "route_first_min" ? &t.route_first_min : nullptr;
        SKM_CHECK(f != nullptr, SKM_E_ARG, "unknown build option: " + n);
        SKM_CHECK(value >= 0 && value <= 0x7FFFFFFF, SKM_E_ARG, "option value out of range");
        if (n == "overflow_long_class" || n == "main_long_class")
            SKM_CHECK(value >= 1 && value < 32, SKM_E_ARG, "long chain classes in [1, 32)");
        if (n == "giant_class") SKM_CHECK(value < 32, SKM_E_ARG, "giant_class in [0, 32)");
        if (n == "emit_group")
            SKM_CHECK(value == 0 || value == 1 || value == 2 || value == 4 || value == 8 || value == 16, SKM_E_ARG,
                      "emit_group must be 0, 1, 2, 4, 8 or 16");
        *f = (int)value;
    }
    b->prepared = false;  // pass geometry and buffers are re-planned on the next prepare/run
    b->ran = false;
    SKM_API_END
}

// Diagnostics: enable per-phase s_memtime sums in k_bucket_process (returned by the next call).
int skm_build_debug_stamps(skm_build* b, int enable, uint64_t* out, int cap) {
    SKM_API_BEGIN
    SKM_CHECK(b, SKM_E_ARG, "null build");
    if (out && cap > 0 && b->stamps && b->d_stamps.p) {
        uint64_t tmp[32];
        SKM_HIP(hipMemcpy(tmp, b->d_stamps.p, sizeof(tmp), hipMemcpyDeviceToHost));
        for (int i = 0; i < cap && i < 32; ++i) out[i] = tmp[i];
    }
    b->stamps = enable != 0;
    SKM_API_END
}

// Diagnostics: lengths of the first `cap` chain jobs of the last pass in execution order (longest
// class first; the overflow's, the longest, when the pass had an overflow).
int skm_build_debug_jobs(skm_build* b, uint32_t* out, int cap) {
    SKM_API_BEGIN
    SKM_CHECK(b && out, SKM_E_ARG, "null argument");
    SKM_HIP(hipDeviceSynchronize());
    const uint64_t n = std::min<uint64_t>((uint64_t)cap, b->n_jobs_last);
    std::vector<Job> j(n);
    const bool ovf = b->n_overflow_last && b->cs_ovf.sorted.p;
    const DevBuf& src = ovf ? b->cs_ovf.sorted : b->cs_main.sorted;
    const uint64_t m = std::min<uint64_t>(n, src.bytes / sizeof(Job));
    if (m) SKM_HIP(hipMemcpy(j.data(), src.p, sizeof(Job) * m, hipMemcpyDeviceToHost));
    for (uint64_t i = 0; i < (uint64_t)cap; ++i) out[i] = i < m ? j[i].n : 0u;
    SKM_API_END
}

// Diagnostics: element counts of the last pass's overflow sub-buckets as k_partition listed them
// (before k_ovf_split takes the heavy keys out); returns how many there were.
int skm_build_debug_overflow(skm_build* b, uint32_t* out, int cap) {
    if (!b || !out) return SKM_E_ARG;
    if (hipSetDevice(b->device) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return SKM_E_HIP;
    const uint32_t n = b->d_ovf.p ? (uint32_t)std::min<uint64_t>(b->n_overflow_last, b->d_ovf.bytes / sizeof(OvfEntry)) : 0u;
    std::vector<OvfEntry> e(n);
    if (n && hipMemcpy(e.data(), b->d_ovf.p, sizeof(OvfEntry) * n, hipMemcpyDeviceToHost) != hipSuccess) return SKM_E_HIP;
    for (int i = 0; i < cap; ++i) out[i] = (uint32_t)i < n ? e[i].n : 0u;
    return (int)n;
}

// Diagnostics: time k_chains on `njobs` synthetic jobs of length n (lengths 300 +- 60).
int skm_debug_chain_bench(uint32_t n, uint32_t njobs, int mode, float* ms) {
    SKM_API_BEGIN
    SKM_CHECK(ms && n && njobs, SKM_E_ARG, "bad argument");
    std::vector<uint32_t> lens((size_t)n * njobs);
    uint32_t x = 12345;
    for (auto& v : lens) {
        x = x * 1664525u + 1013904223u;
        v = 240 + (x >> 16) % 121;
    }
    std::vector<Job> jobs(njobs);
    for (uint32_t i = 0; i < njobs; ++i) jobs[i] = Job{(uint64_t)i * n, n, i};
    DevBuf dl, dj, dout;
    dl.ensure(4 * lens.size());
    dj.ensure(sizeof(Job) * njobs);
    dout.ensure(std::max(sizeof(skm_stored_kmer_data), sizeof(double)) * njobs);
    SKM_HIP(hipMemcpy(dl.p, lens.data(), 4 * lens.size(), hipMemcpyHostToDevice));
    SKM_HIP(hipMemcpy(dj.p, jobs.data(), sizeof(Job) * njobs, hipMemcpyHostToDevice));
    DevBuf dn;  // the job count, as the chain kernels read it
    dn.ensure(8);
    const unsigned long long nj64 = njobs;
    SKM_HIP(hipMemcpy(dn.p, &nj64, 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    SKM_HIP(hipEventCreate(&e0));
    SKM_HIP(hipEventCreate(&e1));
    const uint64_t threads = ceil_div(njobs, 64) * 128;
    for (int it = 0; it < 2; ++it) {
        SKM_HIP(hipEventRecord(e0, 0));
        if (mode == 3 || mode == 4 || mode == 5)
            hipLaunchKernelGGL(k_chain_long_half, dim3(njobs), dim3(64), 0, 0, dj.as<Job>(), dl.as<uint32_t>(),
                               mode - 3, reinterpret_cast<double*>(dout.p));
        else if (mode == 2 || (mode == 0 && n >= (1u << LONG_CLASS)))
            hipLaunchKernelGGL(k_chain_long, dim3(njobs), dim3(128), 0, 0, dj.as<Job>(), nullptr, dn.as<unsigned long long>(),
                               dl.as<uint32_t>(), dl.as<uint32_t>(), dl.as<uint32_t>(), dl.as<uint32_t>(),
                               dout.as<skm_stored_kmer_data>(), 0);
        else
            hipLaunchKernelGGL(k_chains, dim3((uint32_t)ceil_div(threads, 256)), dim3(256), 0, 0, dj.as<Job>(), nullptr,
                               dn.as<unsigned long long>(), (uint64_t)njobs, dl.as<uint32_t>(), dl.as<uint32_t>(),
                               dl.as<uint32_t>(), dl.as<uint32_t>(), dout.as<skm_stored_kmer_data>());
        SKM_HIP(hipEventRecord(e1, 0));
        SKM_HIP(hipEventSynchronize(e1));
        SKM_HIP(hipEventElapsedTime(ms, e0, e1));
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    SKM_API_END
}

// Diagnostics: one chain through the per-lane (mode 1) or wave-pair (mode 2) code, raw results.
int skm_debug_chain_eval(const uint32_t* samples, uint32_t n, int mode, double* median, double* var) {
    SKM_API_BEGIN
    SKM_CHECK(samples && n && median && var && (mode == 1 || mode == 2), SKM_E_ARG, "bad argument");
    DevBuf dx, dout;
    dx.ensure(4ull * n);
    dout.ensure(16);
    SKM_HIP(hipMemcpy(dx.p, samples, 4ull * n, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_chain_eval, dim3(1), dim3(128), 0, 0, dx.as<uint32_t>(), n, mode, dout.as<double>());
    SKM_HIP(hipGetLastError());
    double r[2];
    SKM_HIP(hipMemcpy(r, dout.p, 16, hipMemcpyDeviceToHost));
    *median = r[0];
    *var = r[1];
    SKM_API_END
}

// Diagnostics: device reciprocal / corrected-quotient check against IEEE division.
int skm_debug_div_check(uint64_t nm, uint32_t per, uint64_t* mismatches) {
    SKM_API_BEGIN
    SKM_CHECK(mismatches && nm, SKM_E_ARG, "bad argument");
    DevBuf d;
    d.ensure(8);
    SKM_HIP(hipMemset(d.p, 0, 8));
    hipLaunchKernelGGL(k_div_check, dim3((uint32_t)ceil_div(nm, 256)), dim3(256), 0, 0, nm, per,
                       d.as<unsigned long long>());
    SKM_HIP(hipGetLastError());
    SKM_HIP(hipMemcpy(mismatches, d.p, 8, hipMemcpyDeviceToHost));
    SKM_API_END
}

int skm_build_counters(skm_build* b, uint64_t* out, int cap) {
    if (!b || !out) return SKM_E_ARG;
    auto us = [](double sec) { return (uint64_t)(sec * 1e6); };
    const uint64_t v[46] = {b->n_windows, b->n_kept, b->n_overflow, b->n_jobs, b->n_lens, b->nseq, b->n_local,
                            b->ovf_elems, b->ovf_kept, b->n_big, b->big_kept, 1ull << b->pass_bits, b->valid_total,
                            b->giant_jobs, b->giant_max, b->n_redo, b->tot_cap, b->split_cap, b->long_cap,
                            b->long_jobs_cap, b->demand[0], b->demand[1], b->demand[2], b->demand[3],
                            b->long_samples, b->routed, us(b->add_s), us(b->prep_upload_s), us(b->prep_plan_s),
                            us(b->prep_rest_s), b->pass_bits ? (1ull << b->pass_bits) / b->emit_g : 0ull, us(b->add_pack_s),
                            us(b->add_wait_s), us(b->handoff.total_s), us(b->handoff.wait_s),
                            us(b->handoff.copy_s), b->handoff.chunks, (uint64_t)(1e3 * b->handoff.select_ms),
                            (uint64_t)(1e3 * b->handoff.sort_ms), (uint64_t)(1e3 * b->handoff.gather_ms),
                            (uint64_t)(1e3 * b->handoff.d2h_ms), b->handoff.max_chunk,
                            (uint64_t)b->handoff.wide_index, b->kept_cap, b->free_after_prepare,
                            (uint64_t)b->rot};
    int n = std::min(cap, 46);
    for (int i = 0; i < n; ++i) out[i] = v[i];
    return n;
}

int skm_build_set_kernel_timing(skm_build* b, int enable, const char* only) {
    SKM_API_BEGIN
    SKM_CHECK(b, SKM_E_ARG, "null build");
    b->kt_mode = enable ? 1 : 0;
    b->kt_only = only ? std::string(only) : std::string();
    SKM_API_END
}

int skm_build_kernel_timings(skm_build* b, char* names, size_t names_cap, float* ms, uint64_t* launches, int cap) {
    if (!b) return SKM_E_ARG;
    const int n = (int)b->kt_names.size();
    std::string all;
    for (int k = 0; k < n; ++k) {
        if (k < cap) {
            if (ms) ms[k] = (float)b->kt_ms[k];
            if (launches) launches[k] = b->kt_n[k];
        }
        all += b->kt_names[k];
        all += '\n';
    }
    if (names && names_cap) {
        const size_t c = std::min(names_cap - 1, all.size());
        std::memcpy(names, all.data(), c);
        names[c] = 0;
    }
    return n;
}

int skm_build_last_timings(skm_build* b, float* ms, int cap) {
    if (!b || !ms) return SKM_E_ARG;
    int n = std::min(cap, 15);
    for (int i = 0; i < n; ++i) ms[i] = b->last_ms[i];
    return n;
}

int skm_build_finish(skm_build* b, skm_kept* out) {
    SKM_API_BEGIN
    SKM_CHECK(b && out, SKM_E_ARG, "null argument");
    check_transport(b);
    SKM_HIP(hipSetDevice(b->device));
    const Ranks bs = ranks_of(b);
    bool need = false;
    for (auto* x : bs) need |= !x->prepared || !x->ran;
    if (need) run_ranks(bs);
    std::memset(out, 0, sizeof(*out));
    const uint32_t F = b->opts.n_functions;
    // kept k-mers: rank 0 gathers every rank's owned k-mers; other ranks return their own
    std::vector<uint64_t> mine;
    for (auto* x : bs) mine.push_back(x->n_kept);
    const std::vector<uint64_t> nk = b->world > 1 ? allgather_u64(bs, mine) : mine;
    uint64_t total = 0;
    for (auto v : nk) total += v;
    const bool gather = b->world > 1 && b->rank == 0;
    const uint64_t n = gather ? total : b->n_kept;
    // the arena the hand-off reads: this rank's own, or (rank 0 at world > 1) every rank's in rank
    // order on this device
    DevBuf gk, gd;
    const uint64_t* src_k = b->d_keys.as<uint64_t>();
    const skm_stored_kmer_data* src_d = b->d_data.as<skm_stored_kmer_data>();
    if (b->world > 1 && bs.size() > 1) {  // in-process group: device-to-device copies
        if (gather) {
            gk.ensure(8 * (total + 1));
            gd.ensure(sizeof(skm_stored_kmer_data) * (total + 1));
            uint64_t o = 0;
            for (auto* x : bs) {
                if (x->n_kept) {
                    SKM_HIP(hipMemcpy(gk.as<uint64_t>() + o, x->d_keys.p, 8 * x->n_kept, hipMemcpyDeviceToDevice));
                    SKM_HIP(hipMemcpy(gd.as<skm_stored_kmer_data>() + o, x->d_data.p,
                                      sizeof(skm_stored_kmer_data) * x->n_kept, hipMemcpyDeviceToDevice));
                }
                o += x->n_kept;
            }
            src_k = gk.as<uint64_t>();
            src_d = gd.as<skm_stored_kmer_data>();
        }
    } else if (b->world > 1) {  // RCCL / host transport: every rank sends its k-mers to rank 0
        const int W = b->world;
        A2A xk, xd;
        std::vector<uint64_t> so(W, 0), sck(W, 0), scd(W, 0), rok(W, 0), rod(W, 0), rck(W, 0), rcd(W, 0);
        sck[0] = 8 * b->n_kept;
        scd[0] = sizeof(skm_stored_kmer_data) * b->n_kept;
        if (gather) {
            gk.ensure(8 * (total + 1));
            gd.ensure(sizeof(skm_stored_kmer_data) * (total + 1));
            uint64_t o = 0;
            for (int r = 0; r < W; ++r) {
                rok[r] = 8 * o;
                rod[r] = sizeof(skm_stored_kmer_data) * o;
                rck[r] = 8 * nk[r];
                rcd[r] = sizeof(skm_stored_kmer_data) * nk[r];
                o += nk[r];
            }
        }
        xk.send = {b->d_keys.as<uint8_t>()};
        xk.recv = {gather ? gk.as<uint8_t>() : nullptr};
        xk.soff = {so};
        xk.scnt = {sck};
        xk.roff = {rok};
        xk.rcnt = {rck};
        xd.send = {b->d_data.as<uint8_t>()};
        xd.recv = {gather ? gd.as<uint8_t>() : nullptr};
        xd.soff = {so};
        xd.scnt = {scd};
        xd.roff = {rod};
        xd.rcnt = {rcd};
        alltoallv(bs, xk);
        alltoallv(bs, xd);
        SKM_HIP(hipStreamSynchronize(b->stream));
        if (gather) {
            src_k = gk.as<uint64_t>();
            src_d = gd.as<skm_stored_kmer_data>();
        }
    }
    out->distinct_functions = (uint32_t*)std::malloc(sizeof(uint32_t) * std::max<uint32_t>(F, 1));
    out->seqs_with_func = (uint32_t*)std::malloc(sizeof(uint32_t) * std::max<uint32_t>(F, 1));
    SKM_CHECK(out->distinct_functions && out->seqs_with_func, SKM_E_OOM, "host allocation failed");
    if (F) {
        SKM_HIP(hipMemcpyAsync(out->distinct_functions, b->d_dfunc.p, sizeof(uint32_t) * F, hipMemcpyDeviceToHost, b->stream));
        SKM_HIP(hipMemcpyAsync(out->seqs_with_func, b->d_swf.p, sizeof(uint32_t) * F, hipMemcpyDeviceToHost, b->stream));
    }
    unsigned long long ctr[3];
    SKM_HIP(hipMemcpyAsync(ctr, b->d_ctr.p, sizeof(ctr), hipMemcpyDeviceToHost, b->stream));
    const bool strict = b->world > 1 ? b->g_strict : b->seqid_strict;
    std::vector<uint8_t> flags;
    if (!strict) {
        flags.resize(b->n_total);
        if (b->n_total) SKM_HIP(hipMemcpyAsync(flags.data(), b->d_flags.p, b->n_total, hipMemcpyDeviceToHost, b->stream));
    }
    SKM_HIP(hipStreamSynchronize(b->stream));
    // keys ascending: device radix sort in chunks, streamed to the host arrays (skm_output.hip)
    if (!b->pool) b->pool.reset(new HostPool(HostPool::default_threads()));
    kept_handoff(src_k, src_d, n, b->stream, b->pool.get(), &out->keys, &out->data, &b->handoff,
                 (uint64_t)b->tune.handoff_index_limit, (uint64_t)b->tune.handoff_max_chunk);
    out->n = n;
    out->n_functions = F;
    out->distinct_signatures = total;
    if (strict) {
        out->n_seqs_with_signature = ctr[2];
    } else {  // colliding seq ids (files with > max_seqs_per_file sequences): count distinct ids
        const std::vector<uint32_t>& sid = b->world > 1 ? b->g_seqid : b->h_seqid;
        std::vector<uint32_t> ids;
        for (uint32_t s = 0; s < b->n_total; ++s)
            if (flags[s]) ids.push_back(sid[s]);
        std::sort(ids.begin(), ids.end());
        out->n_seqs_with_signature = (uint64_t)(std::unique(ids.begin(), ids.end()) - ids.begin());
    }
    out->n_windows = b->n_windows;
    out->n_records = b->n_local;
    SKM_API_END
}

int skm_build_finish_slice(skm_build* b, int slice_bits, uint32_t slice, skm_kept* out) {
    SKM_API_BEGIN
    SKM_CHECK(b && out, SKM_E_ARG, "null argument");
    SKM_CHECK(slice_bits >= 0 && slice_bits <= 16 && slice < (1u << slice_bits), SKM_E_ARG, "bad slice");
    check_transport(b);
    SKM_HIP(hipSetDevice(b->device));
    const Ranks bs = ranks_of(b);
    bool need = false;
    for (auto* x : bs) need |= !x->prepared || !x->ran;
    if (need) run_ranks(bs);
    std::memset(out, 0, sizeof(*out));
    hipStream_t st = b->stream;
    const uint32_t F = b->opts.n_functions;
    DevBuf cur, dk, dd;
    cur.ensure(8);
    SKM_HIP(hipMemsetAsync(cur.p, 0, 8, st));
    const uint64_t nk = b->n_kept;
    if (nk)
        hipLaunchKernelGGL(k_slice_select, dim3(2048), dim3(256), 0, st, b->d_keys.as<uint64_t>(),
                           b->d_data.as<skm_stored_kmer_data>(), nk, slice_bits, (uint64_t)slice,
                           cur.as<unsigned long long>(), nullptr, nullptr);
    SKM_HIP(hipGetLastError());
    uint64_t n = 0;
    SKM_HIP(hipMemcpyAsync(&n, cur.p, 8, hipMemcpyDeviceToHost, st));
    SKM_HIP(hipStreamSynchronize(st));
    if (n) {
        dk.ensure(8 * n);
        dd.ensure(sizeof(skm_stored_kmer_data) * n + 16);
        SKM_HIP(hipMemsetAsync(cur.p, 0, 8, st));
        hipLaunchKernelGGL(k_slice_select, dim3(2048), dim3(256), 0, st, b->d_keys.as<uint64_t>(),
                           b->d_data.as<skm_stored_kmer_data>(), nk, slice_bits, (uint64_t)slice,
                           cur.as<unsigned long long>(), dk.as<uint64_t>(), dd.as<skm_stored_kmer_data>());
        SKM_HIP(hipGetLastError());
    }
    out->distinct_functions = (uint32_t*)std::malloc(sizeof(uint32_t) * std::max<uint32_t>(F, 1));
    out->seqs_with_func = (uint32_t*)std::malloc(sizeof(uint32_t) * std::max<uint32_t>(F, 1));
    SKM_CHECK(out->distinct_functions && out->seqs_with_func, SKM_E_OOM, "host allocation failed");
    if (F) {
        SKM_HIP(hipMemcpyAsync(out->distinct_functions, b->d_dfunc.p, sizeof(uint32_t) * F, hipMemcpyDeviceToHost, st));
        SKM_HIP(hipMemcpyAsync(out->seqs_with_func, b->d_swf.p, sizeof(uint32_t) * F, hipMemcpyDeviceToHost, st));
    }
    unsigned long long ctr[3];
    SKM_HIP(hipMemcpyAsync(ctr, b->d_ctr.p, sizeof(ctr), hipMemcpyDeviceToHost, st));
    SKM_HIP(hipStreamSynchronize(st));
    // keys ascending: the slice sorted on the device and streamed out (skm_output.hip)
    if (!b->pool) b->pool.reset(new HostPool(HostPool::default_threads()));
    kept_handoff(dk.as<uint64_t>(), dd.as<skm_stored_kmer_data>(), n, st, b->pool.get(), &out->keys, &out->data,
                 &b->handoff, (uint64_t)b->tune.handoff_index_limit, (uint64_t)b->tune.handoff_max_chunk);
    out->n = n;
    out->n_functions = F;
    uint64_t total = b->n_kept;
    if (b->world > 1) {
        std::vector<uint64_t> mine;
        for (auto* x : bs) mine.push_back(x->n_kept);
        total = 0;
        for (auto v : allgather_u64(bs, mine)) total += v;
    }
    out->distinct_signatures = total;
    out->n_seqs_with_signature = ctr[2];  // per sequence (colliding seq ids counted per sequence)
    out->n_windows = b->n_windows;
    out->n_records = b->n_local;
    SKM_API_END
}

int skm_build_signature_flags(skm_build* b, uint8_t* out, uint64_t cap) {
    SKM_API_BEGIN
    SKM_CHECK(b && out, SKM_E_ARG, "null argument");
    SKM_CHECK(b->ran, SKM_E_STATE, "no completed run");
    SKM_HIP(hipSetDevice(b->device));
    const uint64_t n = std::min<uint64_t>(cap, b->n_total);
    if (n) SKM_HIP(hipMemcpy(out, b->d_flags.p, n, hipMemcpyDeviceToHost));
    SKM_API_END
}

void skm_kept_free(skm_kept* k) {
    if (!k) return;
    std::free(k->keys);
    std::free(k->data);
    std::free(k->distinct_functions);
    std::free(k->seqs_with_func);
    std::memset(k, 0, sizeof(*k));
}

void skm_build_destroy(skm_build* b) {
    if (!b) return;
    (void)hipSetDevice(b->device);
    if (b->stream) (void)hipStreamSynchronize(b->stream);
#if defined(SKM_WITH_RCCL)
    if (b->comm) (void)ncclCommDestroy(b->comm);
#endif
    for (auto* x : b->group)  // leave the other members usable on their own
        if (x != b) x->group.clear();
    if (b->stream2) (void)hipStreamSynchronize(b->stream2);
    if (b->stream3) (void)hipStreamSynchronize(b->stream3);
    if (b->stream_tail) (void)hipStreamSynchronize(b->stream_tail);
    if (b->stream_tail2) (void)hipStreamSynchronize(b->stream_tail2);
    if (b->chain_st) (void)hipStreamSynchronize(b->chain_st);
    for (auto& set : b->evsets) {
        for (auto& e : set.ev)
            if (e) (void)hipEventDestroy(e);
        for (auto& e : set.o)
            if (e) (void)hipEventDestroy(e);
        for (auto& e : set.o3)
            if (e) (void)hipEventDestroy(e);
    }
    if (b->ev_part) (void)hipEventDestroy(b->ev_part);
    if (b->ev_part_heavy) (void)hipEventDestroy(b->ev_part_heavy);
    for (int k = 0; k < 2; ++k) {
        if (b->ev_ovf_done[k]) (void)hipEventDestroy(b->ev_ovf_done[k]);
        if (b->ev_main_done[k]) (void)hipEventDestroy(b->ev_main_done[k]);
    }
    for (auto& e : b->ev_tail)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : b->ev_giant)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : b->kt_pool) (void)hipEventDestroy(e);
    for (int i = 0; i < 2; ++i) {
        if (b->st_busy[i] && b->st_ev[i]) (void)hipEventSynchronize(b->st_ev[i]);
        if (b->st_pin[i]) (void)hipHostFree(b->st_pin[i]);
        if (b->st_ev[i]) (void)hipEventDestroy(b->st_ev[i]);
    }
    if (b->ev_split) (void)hipEventDestroy(b->ev_split);
    if (b->ev_start) (void)hipEventDestroy(b->ev_start);
    for (int g = 0; g < skm_build::GSLOTS; ++g) {
        if (b->gst[g]) {
            (void)hipStreamSynchronize(b->gst[g]);
            (void)hipStreamDestroy(b->gst[g]);
        }
        if (b->gev_ready[g]) (void)hipEventDestroy(b->gev_ready[g]);
        if (b->gev_done[g]) (void)hipEventDestroy(b->gev_done[g]);
    }
    if (b->stx) {
        (void)hipStreamSynchronize(b->stx);
        (void)hipStreamDestroy(b->stx);
    }
    if (b->ev_staged) (void)hipEventDestroy(b->ev_staged);
    if (b->ev_emit) (void)hipEventDestroy(b->ev_emit);
    if (b->chain_st) {
        (void)hipStreamSynchronize(b->chain_st);
        (void)hipStreamDestroy(b->chain_st);
    }
    for (int k = 0; k < skm_build::LANE_ST; ++k) {
        if (b->lane_st[k]) {
            (void)hipStreamSynchronize(b->lane_st[k]);
            (void)hipStreamDestroy(b->lane_st[k]);
        }
        if (b->lane_ev[k]) (void)hipEventDestroy(b->lane_ev[k]);
    }
    for (auto& e : b->chain_ev)
        if (e) (void)hipEventDestroy(e);
    if (b->h_pin) (void)hipHostFree(b->h_pin);
    if (b->h_ovf) (void)hipHostFree(b->h_ovf);
    if (b->stream) (void)hipStreamDestroy(b->stream);
    if (b->stream2) (void)hipStreamDestroy(b->stream2);
    if (b->stream3) (void)hipStreamDestroy(b->stream3);
    if (b->stream_tail) (void)hipStreamDestroy(b->stream_tail);
    if (b->stream_tail2) (void)hipStreamDestroy(b->stream_tail2);
    if (b->ev_tail2) (void)hipEventDestroy(b->ev_tail2);
    if (b->ev_tail_bp) (void)hipEventDestroy(b->ev_tail_bp);
    if (b->ev_tail_done) (void)hipEventDestroy(b->ev_tail_done);
    if (b->ev_scan) (void)hipEventDestroy(b->ev_scan);
    delete b;
}

}  // extern "C"
