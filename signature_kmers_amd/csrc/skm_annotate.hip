// skm_annotate.hip -- function calling against a CMPH/BDZ signature DB resident in HBM.
//
// Replaces FunctionCaller<CmphKmerDb>::process_aa_seq (call_functions.tcc:259-338) with its
// window iterator for_each_kmer<8> (kmer_data.h:76-102), CmphKmerDb::fetch (cmph_kmer.h:139-147)
// and HitSet::process (call_functions.tcc:35-103).
//
//   k_lookup   one thread per 16 windows: window validity (no 'X'/'*' in the window or the byte
//              after it), jenkins lookup2 -> 3 vertices -> 2-bit g -> rank (popcount over u32
//              words of g) -> 10-byte record gather; writes func<<16|mean per window position
//   k_calls_scan   one thread per query sequence: the HitSet state machine over its window hits,
//              emitting one segment per HitSet::process
//   k_seg_process  one wave per segment: statistics (Boost.Math mean / median / MAD) in LDS,
//              the length test, the KmerCall
//   scan + k_gather   CSR compaction of the calls
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <memory>
#include <thread>
#include <cstring>
#include <cmath>
#include <fstream>
#include <random>
#include <string>
#include <vector>

#include "skm_bdz.h"
#include "skm_common.h"
#include "skm_lookup.h"
#include "skm_pool.h"
#include "skm_select.h"
#include "skm_util.h"

namespace skm {

// the kept keys into the 16-byte-slot table (exact_slot): the key by CAS on its slot's first 8
// bytes, then its record index and record word; bad |= 1 for a key 0, 2 for a duplicate key
__global__ void k_exact_insert(const uint64_t* __restrict__ keys, const uint16_t* __restrict__ dat, uint64_t n,
                               uint4* __restrict__ tab, uint64_t mask, uint32_t shift, uint32_t* __restrict__ bad) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned long long k = keys[i];
    if (k == 0) {
        atomicOr(bad, 1u);
        return;
    }
    uint64_t h = xmix(k) >> shift;
    for (;;) {
        unsigned long long* key = reinterpret_cast<unsigned long long*>(tab + h);
        const unsigned long long prev = atomicCAS(key, 0ull, k);
        if (prev == 0ull) {
            uint32_t* rest = reinterpret_cast<uint32_t*>(tab + h) + 2;
            rest[0] = (uint32_t)i;
            rest[1] = ((uint32_t)dat[5 * i + 1] << 16) | (uint32_t)dat[5 * i + 2];  // function_index, mean
            return;
        }
        if (prev == k) {
            atomicOr(bad, 2u);
            return;
        }
        h = (h + 1) & mask;
    }
}


// MODE: LK_BDZ7 = BDZ with rank blocks of 128 (cmph's default b = 7), LK_EXACT = kept-k-mer
// table, LK_BDZ = BDZ with any b (per-window search)
enum { LK_BDZ7 = 0, LK_EXACT = 1, LK_BDZ = 2 };
template <int MODE>
__global__ __launch_bounds__(LK_THREADS) __attribute__((amdgpu_waves_per_eu(4))) void k_lookup(const uint8_t* __restrict__ res, uint64_t rp, DevBdz D,
                                                      uint32_t* __restrict__ hits) {
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x * LK_POS;
    for (uint64_t base = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * LK_POS; base < rp; base += step) {
        const uint4 v0 = *reinterpret_cast<const uint4*>(res + base);
        const uint4 v1 = *reinterpret_cast<const uint4*>(res + base + 16);
        const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        // bad[j]: byte j is a separator (0) or ambiguous; amb[j]: byte j is 'X' or '*'
        uint32_t bad = 0, amb = 0;
#pragma unroll
        for (int j = 0; j < 25 && j < 32; ++j) {
            uint32_t c = (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            bool a = ambig(c);
            amb |= (a ? 1u : 0u) << j;
            bad |= ((a || c == 0) ? 1u : 0u) << j;
        }
        uint32_t out[LK_POS];
        if constexpr (MODE == LK_EXACT) {
            // the 16 windows' first probes issued together (one 16-byte slot each: key and record
            // word); the few that land on another key walk on (linear probing, load <= 1/2)
            uint4 sl[LK_POS];
            uint64_t hp[LK_POS];
            uint32_t live = 0;
#pragma unroll
            for (int t = 0; t < LK_POS; ++t) {
                const uint64_t p = base + t;
                uint32_t lo, hi;
                key_at(w, t, lo, hi);
                const bool ok = p < rp && ((bad >> t) & 0xFFu) == 0 && ((amb >> (t + 8)) & 1u) == 0;
                hp[t] = xmix(((uint64_t)hi << 32) | lo) >> D.xshift;
                sl[t] = ok ? D.xtab[hp[t]] : make_uint4(0u, 0u, 0u, 0u);
                live |= (ok ? 1u : 0u) << t;
            }
#pragma unroll
            for (int t = 0; t < LK_POS; ++t) {
                uint32_t lo, hi;
                key_at(w, t, lo, hi);
                uint4 q = sl[t];
                uint64_t h = hp[t];
                while (((live >> t) & 1u) && !(q.x == lo && q.y == hi) && (q.x | q.y) != 0u) {
                    h = (h + 1) & D.xmask;
                    q = D.xtab[h];
                }
                out[t] = ((live >> t) & 1u) && (q.x | q.y) != 0u ? q.w : NO_HIT;  // function_index << 16 | mean
            }
        } else if constexpr (MODE != LK_BDZ7) {
#pragma unroll
            for (int t = 0; t < LK_POS; ++t) {
                const uint64_t p = base + t;
                uint32_t o = NO_HIT;
                if (p < rp && ((bad >> t) & 0xFFu) == 0 && ((amb >> (t + 8)) & 1u) == 0) {
                    uint32_t lo, hi;
                    key_at(w, t, lo, hi);
                    const uint32_t idx = bdz_lookup(D, lo, hi);
                    if (idx < D.m) o = D.fm[idx];  // function_index << 16 | mean
                }
                out[t] = o;
            }
        } else {
            // BDZ search in phases over 8 windows at a time so every dependent level issues 8+
            // independent loads: (1) jenkins -> 3 (g word, rank word) pairs, one 8-byte load each,
            // (2) select vertex, one popcount -> .dat record
#pragma unroll
            for (int half = 0; half < LK_POS / 8; ++half) {
                uint32_t hl[8];  // the candidates' in-word positions (v & 15), 4 bits each
                uint2 gp[8][3];  // (g word, rank of its first vertex) of each candidate
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    uint32_t lo, hi;
                    key_at(w, half * 8 + u, lo, hi);
                    uint32_t a = 0x9e3779b9u + lo, b = 0x9e3779b9u + hi, c = D.seed + 8u;
                    jmix(a, b, c);
                    const uint32_t hv[3] = {fastmod(a, D.r_magic, D.r), fastmod(b, D.r_magic, D.r) + D.r,
                                            fastmod(c, D.r_magic, D.r) + 2u * D.r};
                    hl[u] = (hv[0] & 15u) | (hv[1] & 15u) << 4 | (hv[2] & 15u) << 8;
#pragma unroll
                    for (int j = 0; j < 3; ++j)
                        gp[u][j] = *reinterpret_cast<const uint2*>(D.blk + (hv[j] >> 7) * 16u + 2u * ((hv[j] & 127u) >> 4));
                }
                uint32_t rank[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    uint32_t sum = 0;
#pragma unroll
                    for (int j = 0; j < 3; ++j) sum += (gp[u][j].x >> (((hl[u] >> (4 * j)) & 15u) * 2)) & 3u;
                    const uint32_t sel = sum % 3u;
                    // v's own g word and the rank of its first vertex (b = 7, checked on open)
                    // (selected per component: a select of whole uint2 values becomes a
                    // dynamically indexed stack array)
                    const bool s0 = sel == 0, s1 = sel == 1;
                    const uint32_t qx = s0 ? gp[u][0].x : (s1 ? gp[u][1].x : gp[u][2].x);
                    const uint32_t qy = s0 ? gp[u][0].y : (s1 ? gp[u][1].y : gp[u][2].y);
                    const uint32_t pe = (hl[u] >> (4 * sel)) & 15u;
                    const uint32_t pmask = pe ? (0xFFFFFFFFu >> (32u - 2u * pe)) : 0u;
                    rank[u] = qy + pe - unassigned_in(qx & pmask);
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int t = half * 8 + u;
                    const uint64_t p = base + t;
                    uint32_t o = NO_HIT;
                    if (p < rp && ((bad >> t) & 0xFFu) == 0 && ((amb >> (t + 8)) & 1u) == 0 && rank[u] < D.m)
                        o = D.fm[rank[u]];  // function_index << 16 | mean
                    out[t] = o;
                }
            }
        }
        uint4* dst = reinterpret_cast<uint4*>(hits + base);
        dst[0] = make_uint4(out[0], out[1], out[2], out[3]);
        dst[1] = make_uint4(out[4], out[5], out[6], out[7]);
        dst[2] = make_uint4(out[8], out[9], out[10], out[11]);
        dst[3] = make_uint4(out[12], out[13], out[14], out[15]);
    }
}

struct CallArgs {
    const QMeta* meta;
    const uint32_t* hits;
    uint16_t* scratch;          // per-sequence value scratch (nwin entries)
    const uint64_t* scr_off;    // [nseq] scratch offsets (= window offsets)
    const uint64_t* cap_off;    // [nseq+1] call slot offsets
    skm_kmer_call* slots;
    uint32_t* counts;           // [nseq]
    uint32_t nseq;
    int min_hits, max_gap, ignore_hypo, mean_mode, mad_mode;
    uint32_t hypo;
};

__device__ __forceinline__ bool usable(uint32_t h, const CallArgs& A) {
    return h != NO_HIT && !(A.ignore_hypo && (h >> 16) == A.hypo);
}

__device__ void heap_sort_u16(uint16_t* a, uint32_t n) {
    auto sift = [&](uint32_t start, uint32_t end) {
        uint32_t root = start;
        while (2 * root + 1 < end) {
            uint32_t child = 2 * root + 1;
            if (child + 1 < end && a[child] < a[child + 1]) ++child;
            if (a[root] < a[child]) {
                uint16_t t = a[root];
                a[root] = a[child];
                a[child] = t;
                root = child;
            } else {
                return;
            }
        }
    };
    if (n < 2) return;
    for (uint32_t s = n / 2; s-- > 0;) sift(s, n);
    for (uint32_t end = n - 1; end > 0; --end) {
        uint16_t t = a[0];
        a[0] = a[end];
        a[end] = t;
        sift(0, end);
    }
}

// k-th smallest |2 v_j - C2| over sorted v[0..n) (two pointers from the centre outward)
__device__ uint32_t kth_dev(const uint16_t* v, uint32_t n, uint32_t C2, uint32_t k) {
    // split: first index with 2v > C2
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (2u * v[mid] > C2)
            hi = mid;
        else
            lo = mid + 1;
    }
    int64_t L = (int64_t)lo - 1;
    uint32_t R = lo;
    uint32_t d = 0;
    for (uint32_t t = 0; t <= k; ++t) {
        uint32_t dl = L >= 0 ? C2 - 2u * v[L] : 0xFFFFFFFFu;
        uint32_t dr = R < n ? 2u * v[R] - C2 : 0xFFFFFFFFu;
        if (dl <= dr) {
            d = dl;
            --L;
        } else {
            d = dr;
            ++R;
        }
    }
    return d;
}

// HitSet::process over window range [first, last] with current function cur.
template <bool LEGACY_MAD>
__device__ void hitset_process(const CallArgs& A, const uint32_t* hit, uint16_t* scr, uint32_t first, uint32_t last,
                               uint32_t cur, double seqlen, skm_kmer_call* slots, uint32_t& ncalls) {
    uint32_t n = 0, last_cur = first;
    for (uint32_t i = first; i <= last; ++i) {
        const uint32_t h = hit[i];
        if (!usable(h, A) || (h >> 16) != cur) continue;
        scr[n++] = (uint16_t)(h & 0xFFFFu);
        last_cur = i;
    }
    // Boost.Math mean over float(kdata.mean) in hit order
    float mean;
    if (A.mean_mode == 1) {
        float mu = 0, fi = 1;
        for (uint32_t j = 0; j < n; ++j) {
            mu = mu + ((float)scr[j] - mu) / fi;
            fi += 1;
        }
        mean = mu;
    } else {
        float mu[4] = {0, 0, 0, 0};
        float fi = 1;
        const uint32_t end = n - (n % 4);
        uint32_t j = 0;
        for (; j < end; j += 4) {
            const float inv = 1.0f / fi;
            float t0 = (float)scr[j] - mu[0], t1 = (float)scr[j + 1] - mu[1];
            float t2 = (float)scr[j + 2] - mu[2], t3 = (float)scr[j + 3] - mu[3];
            t0 *= inv;
            t1 *= inv;
            t2 *= inv;
            t3 *= inv;
            mu[0] += t0;
            mu[1] += t1;
            mu[2] += t2;
            mu[3] += t3;
            fi += 1;
        }
        const float num1 = float(n - (n % 4)) / float(4);
        const float num2 = num1 + float(n % 4);
        for (; j < n; ++j) {
            mu[3] += ((float)scr[j] - mu[3]) / fi;
            fi += 1;
        }
        mean = (num1 * (mu[0] + mu[1] + mu[2]) + num2 * mu[3]) / float(n);
    }
    float median, mad;
    if constexpr (LEGACY_MAD) {
        legacy_median_mad(scr, n, median, mad);
    } else {
        heap_sort_u16(scr, n);
        uint32_t C2;
        if (n & 1) {
            const uint32_t m = scr[(n - 1) / 2];
            median = (float)m;
            C2 = 2u * m;
        } else {
            const uint32_t a = scr[n / 2 - 1], b = scr[n / 2];
            median = ((float)a + (float)b) / 2;
            C2 = a + b;
        }
        if (n & 1) {
            mad = (float)kth_dev(scr, n, C2, (n - 1) / 2) * 0.5f;
        } else {
            const float d1 = (float)kth_dev(scr, n, C2, n / 2 - 1) * 0.5f;
            const float d2 = (float)kth_dev(scr, n, C2, n / 2) * 0.5f;
            mad = (d1 + d2) / 2.0f;
        }
    }
    if (mad == 0) mad = 30;
    const double cutoff_b = (double)mean - 2.0 * (double)mad;
    const double cutoff_t = (double)mean + 2.0 * (double)mad;
    if ((int)n >= A.min_hits && !(seqlen < cutoff_b || seqlen > cutoff_t)) {
        skm_kmer_call c;
        c.start = first;
        c.end = last_cur + 7u;
        c.count = (int32_t)n;
        c.function_index = (uint16_t)cur;
        c.pad = 0;
        c.protein_length_median = (uint32_t)median;
        c.protein_length_med_avg_dev = mad;
        slots[ncalls++] = c;
    }
}

// HitSet state machine (call_functions.tcc:259-338), thread per sequence.  Each HitSet::process
// event becomes a segment {sequence, first window, last window, current function}; the
// statistics of a segment never feed back into the state machine, so they run afterwards one
// wave per segment (k_seg_process) instead of divergently inside this loop.
__global__ void k_calls_scan(CallArgs A, uint4* __restrict__ segs) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= A.nseq) return;
    const QMeta m = A.meta[s];
    const uint32_t nwin = m.len >= 8 ? m.len - 7 : 0;
    uint4* out = segs + A.cap_off[s];
    uint32_t nseg = 0;
    // HitSet: all usable hits in window range [first, last_pos]; pair = (prev, last); ncur = the
    // hits of the current function (HitSet::process's fI_count).  A process() event with
    // ncur < min_hits emits no call (call_functions.tcc:60), so it yields no segment.
    uint32_t count = 0, ncur = 0, first = 0, last_pos = 0, prev_pos = 0, last_f = 0, prev_f = 0, cur = 0xFFFFu;
    auto process = [&]() {
        if ((int)ncur >= A.min_hits) out[nseg++] = make_uint4(s, first, last_pos, cur);
        if (prev_f != cur && prev_f == last_f) {
            cur = prev_f;
            first = prev_pos;
            count = 2;
            ncur = 2;  // the kept pair has the new current function
        } else {
            count = 0;
            ncur = 0;
        }
    };
    // the next 16 hits are loaded while these 16 are walked (the walk is a per-thread chain): four
    // 16-byte loads from the 16-byte aligned slot below the sequence's first hit (slots outside
    // [0, nwin) are skipped; the hit array is padded by 16 slots), so a wave's load instruction
    // covers 64 lines four times fewer times than with 16 dword loads
    const uint32_t mis = (uint32_t)(m.pstart & 3u);
    const uint4* h4 = reinterpret_cast<const uint4*>(A.hits + (m.pstart - mis));
    const uint32_t tot = nwin ? nwin + mis : 0u;
    uint4 nb[4];
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) nb[k] = 4u * k < tot ? h4[k] : make_uint4(NO_HIT, NO_HIT, NO_HIT, NO_HIT);
    for (uint32_t j0 = 0; j0 < tot; j0 += 16) {
        uint32_t hb[16];
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            hb[4 * k] = nb[k].x;
            hb[4 * k + 1] = nb[k].y;
            hb[4 * k + 2] = nb[k].z;
            hb[4 * k + 3] = nb[k].w;
        }
        if (j0 + 16 < tot) {
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) nb[k] = h4[(j0 >> 2) + 4 + k];
        }
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) {
            const uint32_t h = hb[k], i = j0 + k - mis;  // wraps above nwin before the first window
            if (i >= nwin || !usable(h, A)) continue;
            const uint32_t f = h >> 16;
            if (count > 0 && (uint64_t)last_pos + (uint64_t)A.max_gap < (uint64_t)i) {
                if ((int)count >= A.min_hits) {
                    process();
                } else {
                    count = 0;
                    ncur = 0;
                }
            }
            if (count == 0) {
                cur = f;
                first = i;
            }
            prev_pos = last_pos;
            prev_f = last_f;
            last_pos = i;
            last_f = f;
            ++count;
            ncur += f == cur;
            if (count > 1 && cur != f && prev_f == f) process();
        }
    }
    if ((int)count >= A.min_hits && (int)ncur >= A.min_hits) out[nseg++] = make_uint4(s, first, last_pos, cur);
    A.counts[s] = nseg;
}

// dense segment list: segments of sequence s at seg_off[s]..
__global__ void k_gather_segs(const uint4* __restrict__ segs, const uint64_t* __restrict__ cap_off,
                              const uint64_t* __restrict__ seg_off, uint32_t nseq, uint4* __restrict__ dense) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nseq) return;
    const uint64_t a = seg_off[s], e = seg_off[s + 1], src = cap_off[s];
    for (uint64_t j = a; j < e; ++j) dense[j] = segs[src + (j - a)];
}

// k-th smallest (0-based) |2 v_j - C2| over sorted v[0..n): the deviations left and right of
// C2/2 are two sorted runs; binary search on how many of the k+1 smallest come from the left.
__device__ uint32_t kth_dev_sorted(const uint32_t* v, uint32_t n, uint32_t C2, uint32_t k) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (2u * v[mid] > C2)
            hi = mid;
        else
            lo = mid + 1;
    }
    const uint32_t nL = lo, nR = n - lo, mm = k + 1;
    auto Ld = [&](uint32_t i) { return C2 - 2u * v[nL - 1 - i]; };
    auto Rd = [&](uint32_t i) { return 2u * v[nL + i] - C2; };
    uint32_t a = mm > nR ? mm - nR : 0u, b = mm < nL ? mm : nL;
    while (a < b) {  // first t where "take more from the left" is false
        const uint32_t t = (a + b) >> 1, u = mm - t;
        if (u > 0 && Rd(u - 1) > Ld(t))
            a = t + 1;
        else
            b = t;
    }
    const uint32_t t = a, u = mm - t;
    const uint32_t x = t > 0 ? Ld(t - 1) : 0u, y = u > 0 ? Rd(u - 1) : 0u;
    return x > y ? x : y;
}

constexpr int SEG_WAVES = 4;

// wave-wide min / max / inclusive sum on DPP (row_shr 1/2/4/8 within rows of 16, then row_bcast
// 15 / 31; lanes without a source keep the identity): no LDS round trips, unlike __shfl
template <int OP>  // 0: min, 1: max, 2: inclusive prefix sum
__device__ __forceinline__ uint32_t dpp_step(uint32_t x, uint32_t y) {
    return OP == 0 ? min(x, y) : OP == 1 ? max(x, y) : x + y;
}
template <int OP>
__device__ __forceinline__ uint32_t wave_dpp_scan(uint32_t x) {
    constexpr int id = OP == 0 ? -1 : 0;
    x = dpp_step<OP>(x, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)x, 0x111, 0xF, 0xF, false));
    x = dpp_step<OP>(x, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)x, 0x112, 0xF, 0xF, false));
    x = dpp_step<OP>(x, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)x, 0x114, 0xF, 0xF, false));
    x = dpp_step<OP>(x, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)x, 0x118, 0xF, 0xF, false));
    x = dpp_step<OP>(x, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)x, 0x142, 0xA, 0xF, false));
    x = dpp_step<OP>(x, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)x, 0x143, 0xC, 0xF, false));
    return x;
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_dpp_scan<0>(v), 63);
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_dpp_scan<1>(v), 63);
}

// k-th smallest (0-based) of a wave's n items x[e] (item e * 64 + lane; values < 2^bits): MSD
// radix select, one bit per step, counted on ballots (wave-uniform result)
template <int E>
__device__ __forceinline__ uint32_t wave_select(const uint32_t (&x)[E], uint32_t n, uint32_t k, int bits) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t pre = 0;
    for (int b = bits - 1; b >= 0; --b) {
        uint32_t c = 0;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            if ((uint32_t)e * 64u >= n) break;  // wave-uniform
            const bool v = (uint32_t)e * 64u + lane < n;
            c += (uint32_t)__popcll(__ballot(v && ((x[e] ^ pre) >> (b + 1)) == 0 && ((x[e] >> b) & 1u) == 0));
        }
        if (k >= c) {
            k -= c;
            pre |= 1u << b;
        }
    }
    return pre;
}
constexpr uint32_t SEG_CAP = 1024;  // 16 KB of LDS per 4-wave block: 8 blocks per CU (2048: 5)

// a wave's histogram h[0..R) of its n items x[e] (item e * 64 + lane, values < R) in its LDS
template <int E>
__device__ __forceinline__ void wave_hist(uint32_t* h, const uint32_t (&x)[E], uint32_t n, uint32_t R) {
    const uint32_t lane = threadIdx.x & 63u;
    wave_sync_lds();  // the previous reads of h are done
    for (uint32_t t = lane; t < R; t += 64) h[t] = 0u;
    wave_sync_lds();
#pragma unroll
    for (int e = 0; e < E; ++e) {
        if ((uint32_t)e * 64u >= n) break;  // wave-uniform
        if ((uint32_t)e * 64u + lane < n) atomicAdd(&h[x[e]], 1u);
    }
    wave_sync_lds();
}

// the k1-th and k2-th smallest (0-based) values of a wave histogram over [0, R), R <= SEG_CAP,
// whose bins [b0, b0 + B) lane l holds in c[] (b0 = l B): one DPP scan of the lanes' counts, the
// owner of rank k walks its bins
constexpr uint32_t HBMAX = SEG_CAP / 64;
__device__ __forceinline__ void hist_kth2(const uint32_t (&c)[HBMAX], uint32_t B, uint32_t k1, uint32_t k2,
                                          uint32_t& v1, uint32_t& v2) {
    const uint32_t b0 = (threadIdx.x & 63u) * B;
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t b = 0; b < HBMAX; ++b) {
        if (b >= B) break;  // wave-uniform
        sum += c[b];
    }
    const uint32_t inc = wave_dpp_scan<2>(sum);
    uint32_t acc = inc - sum, r1 = 0, r2 = 0;
    const uint64_t o1 = __ballot(acc <= k1 && k1 < inc), o2 = __ballot(acc <= k2 && k2 < inc);
#pragma unroll
    for (uint32_t b = 0; b < HBMAX; ++b) {
        if (b >= B) break;
        const uint32_t a2 = acc + c[b];
        if (acc <= k1 && k1 < a2) r1 = b0 + b;
        if (acc <= k2 && k2 < a2) r2 = b0 + b;
        acc = a2;
    }
    v1 = (uint32_t)__builtin_amdgcn_readlane((int)r1, __ffsll((long long)o1) - 1);
    v2 = (uint32_t)__builtin_amdgcn_readlane((int)r2, __ffsll((long long)o2) - 1);
}

// One wave per HitSet::process segment (call_functions.tcc:35-103): the hits of the current
// function in window order (ballot compaction into LDS), Boost.Math mean (four-lane Welford on
// lanes 0-3, or the single running mean), median by an LDS bitonic sort, MAD as the k-th
// deviation of the sorted run, the length window test, and the KmerCall (count = -1: none).
// Segments of more than SEG_CAP hits take the sequential path on a private global scratch.
template <bool LEGACY_MAD>  // mad_mode 1 in its own instantiation: no register cost for the default
__global__ __launch_bounds__(64 * SEG_WAVES) void k_seg_process(CallArgs A, const uint4* __restrict__ segs,
                                                                uint32_t nseg, skm_kmer_call* __restrict__ out,
                                                                uint16_t* __restrict__ pool,
                                                                unsigned long long* __restrict__ pool_ctr) {
    __shared__ uint32_t sv[SEG_WAVES][SEG_CAP];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t j = blockIdx.x * SEG_WAVES + wave;
    if (j >= nseg) return;  // wave-uniform
    const uint4 sg = segs[j];
    const uint32_t first = sg.y, last = sg.z, cur = sg.w;
    const QMeta m = A.meta[sg.x];
    const uint32_t* hit = A.hits + m.pstart;
    const double seqlen = (double)m.len;
    uint32_t* buf = sv[wave];
    uint32_t n = 0, last_cur = first;
    auto take64 = [&](uint32_t i0, uint32_t h) {  // the usable hits of cur among windows i0 + lane
        const bool take = usable(h, A) && (h >> 16) == cur;
        const uint64_t bal = __ballot(take);
        const uint32_t pos = n + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
        if (take && pos < SEG_CAP) buf[pos] = h & 0xFFFFu;
        if (bal) last_cur = i0 + 63u - (uint32_t)__clzll(bal);
        n += (uint32_t)__popcll(bal);
    };
    // the first SEG_CAP windows' hits loaded together (one memory latency per segment instead of
    // one per 64 windows); a longer window range walks the rest 64 at a time, the next in flight
    constexpr uint32_t SEG_PRE = SEG_CAP / 64;
    const uint32_t span = last - first + 1u;
    uint32_t hv[SEG_PRE];
#pragma unroll
    for (uint32_t e = 0; e < SEG_PRE; ++e) {
        const uint32_t i = first + e * 64u + lane;
        hv[e] = e * 64u < span && i <= last ? hit[i] : NO_HIT;
    }
#pragma unroll
    for (uint32_t e = 0; e < SEG_PRE; ++e) {
        if (e * 64u >= span) break;  // wave-uniform
        take64(first + e * 64u, hv[e]);
    }
    if (span > SEG_CAP) {
        uint32_t hn = first + SEG_CAP + lane <= last ? hit[first + SEG_CAP + lane] : NO_HIT;
        for (uint32_t i0 = first + SEG_CAP; i0 <= last; i0 += 64) {
            const uint32_t h = hn, i1 = i0 + 64u + lane;
            hn = i1 <= last ? hit[i1] : NO_HIT;
            take64(i0, h);
        }
    }
    if (n > SEG_CAP) {  // long run: the sequential restatement on a private scratch
        if (lane == 0) {
            uint16_t* scr = pool + atomicAdd(pool_ctr, (unsigned long long)n);
            uint32_t nc = 0;
            hitset_process<LEGACY_MAD>(A, hit, scr, first, last, cur, seqlen, out + j, nc);
            if (nc == 0) out[j].count = -1;
        }
        return;
    }
    wave_sync_lds();
    // Boost.Math mean over float(kdata.mean) in hit order
    float mean;
    if (A.mean_mode == 1) {
        float mu = 0, fi = 1;
        if (lane == 0)
            for (uint32_t q = 0; q < n; ++q) {
                mu = mu + ((float)buf[q] - mu) / fi;
                fi += 1;
            }
        mean = __shfl(mu, 0);
    } else {
        const uint32_t end = n - (n % 4);
        float mu = 0, fi = 1;
        // step i of the four running means (items 4 i .. 4 i + 3, one per lane 0-3) multiplies by
        // RN(1 / (i + 1)): the same correctly rounded division, done for 64 steps at once (one per
        // lane) and broadcast by readlane; the items of 8 steps are read from LDS ahead of their
        // chain (round 3's loop waited on one LDS read and one division per step, round 4's
        // first version on a global table load per step)
        const uint32_t nq = end >> 2;
        for (uint32_t i0 = 0; i0 < nq; i0 += 64) {
            const float r = 1.0f / (float)(i0 + lane + 1u);
            const uint32_t cnt = min(64u, nq - i0);
            for (uint32_t t0 = 0; t0 < cnt; t0 += 8) {
                float xv[8];  // 4 (i0 + t0 + u) + 3 <= 4 * 255 + 3 < SEG_CAP: in the wave's buffer
#pragma unroll
                for (int u = 0; u < 8; ++u) xv[u] = (float)buf[4u * (i0 + t0 + (uint32_t)u) + (lane & 3u)];
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (t0 + (uint32_t)u < cnt) {
                        const float inv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(r), (int)(t0 + (uint32_t)u)));
                        float t = xv[u] - mu;
                        t *= inv;
                        mu += t;
                    }
            }
        }
        fi += (float)nq;  // the tail's running count (exact: nq <= 256)
        if (lane == 3)
            for (uint32_t q = end; q < n; ++q) {
                mu += ((float)buf[q] - mu) / fi;
                fi += 1;
            }
        const float m0 = __shfl(mu, 0), m1 = __shfl(mu, 1), m2 = __shfl(mu, 2), m3 = __shfl(mu, 3);
        const float num1 = float(n - (n % 4)) / float(4);
        const float num2 = num1 + float(n % 4);
        mean = (num1 * (m0 + m1 + m2) + num2 * m3) / float(n);
    }
    auto emit = [&](float median, float mad) {
        if (mad == 0) mad = 30;
        const double cutoff_b = (double)mean - 2.0 * (double)mad;
        const double cutoff_t = (double)mean + 2.0 * (double)mad;
        skm_kmer_call c;
        c.start = first;
        c.end = last_cur + 7u;
        c.count = ((int)n >= A.min_hits && !(seqlen < cutoff_b || seqlen > cutoff_t)) ? (int32_t)n : -1;
        c.function_index = (uint16_t)cur;
        c.pad = 0;
        c.protein_length_median = (uint32_t)median;
        c.protein_length_med_avg_dev = mad;
        out[j] = c;
    };
    if constexpr (LEGACY_MAD) {  // the <= 1.75 MAD: libstdc++ selection order on the hit-order run
        if (lane != 0) return;
        float median, mad;
        legacy_median_mad(buf, n, median, mad);
        emit(median, mad);
        return;
    }
    // median and MAD from the run held in registers (E <= 16 items per lane, item e * 64 + lane):
    // the (n-1)/2-th (odd n) or the n/2-1-th and n/2-th smallest (even) of the u16 lengths, then
    // the same ranks of |2 v - C2| -- the order statistics the sorted run gives
    // (call_functions.tcc:51-53), without an LDS sort (round 3: a 512-element bitonic network per
    // segment).  A segment's lengths span a few hundred values, so both selects read a histogram of
    // x - min in the wave's LDS buffer (two per segment); a wider span takes MSD radix selects on
    // ballots.
    // (loops bounded by the wave-uniform item count, lane conditions as selects: the LDS reads
    // stay inside the buffer, so no exec-mask branches)
    uint32_t x[SEG_CAP / 64];
    uint32_t vmin = 0xFFFFu, vmax = 0u;
#pragma unroll
    for (int e = 0; e < (int)(SEG_CAP / 64); ++e) x[e] = 0u;
#pragma unroll
    for (int e = 0; e < (int)(SEG_CAP / 64); ++e) {
        if ((uint32_t)e * 64u >= n) break;  // wave-uniform
        const uint32_t i = (uint32_t)e * 64u + lane;
        const uint32_t v = buf[i];
        const bool in = i < n;
        x[e] = in ? v : 0u;
        vmin = min(vmin, in ? v : 0xFFFFu);
        vmax = max(vmax, in ? v : 0u);
    }
    vmin = wave_min_u32(vmin);
    vmax = wave_max_u32(vmax);
#pragma unroll
    for (int e = 0; e < (int)(SEG_CAP / 64); ++e) x[e] -= vmin;
    const uint32_t R = vmax - vmin + 1u;  // n == 0: wraps above SEG_CAP (the radix path)
    float median, mad;
    if (R <= SEG_CAP) {
        // the order statistics from histograms in the wave's (now free) LDS buffer: of x - min, then
        // of the deviations |2 x - C2| = 2 i + (C2 & 1), all of one parity, binned by i < R
        const uint32_t k1 = (n - 1) / 2, k2 = n / 2;  // odd n: the same rank twice
        const uint32_t B = (R + 63u) >> 6, b0 = lane * B;
        uint32_t a, b, c[HBMAX];
        wave_hist(buf, x, n, R);
#pragma unroll
        for (uint32_t t = 0; t < HBMAX; ++t) {
            if (t >= B) break;  // wave-uniform
            const uint32_t v = buf[min(b0 + t, SEG_CAP - 1u)];
            c[t] = b0 + t < R ? v : 0u;
        }
        hist_kth2(c, B, k1, k2, a, b);
        const uint32_t C2 = a + b;
        median = (n & 1) ? (float)(a + vmin) : ((float)(a + vmin) + (float)(b + vmin)) / 2;
        // the deviation histogram folded from the same one: bin i counts the values at
        // |2 v - C2| = 2 i + p, i.e. v = up + i and v = lo - i (lo = up once when p = 0)
        const uint32_t p = C2 & 1u, up = (C2 + p) >> 1, lo = (C2 - p) >> 1;
#pragma unroll
        for (uint32_t t = 0; t < HBMAX; ++t) {
            if (t >= B) break;
            const uint32_t i = b0 + t;
            const bool hi_in = up + i < R, lo_in = (i > 0 || p) && i <= lo;
            const uint32_t vu = buf[min(up + i, SEG_CAP - 1u)], vl = buf[lo_in ? lo - i : 0u];
            const uint32_t d = (hi_in ? vu : 0u) + (lo_in ? vl : 0u);
            c[t] = i < R ? d : 0u;
        }
        hist_kth2(c, B, k1, k2, a, b);
        if (n & 1)
            mad = (float)(2u * a + p) * 0.5f;
        else
            mad = ((float)(2u * a + p) * 0.5f + (float)(2u * b + p) * 0.5f) / 2.0f;
        if (lane == 0) emit(median, mad);
        return;
    }
    const int vbits = 32 - __clz(vmax - vmin);  // bits of the largest x - vmin
    uint32_t C2;  // 2 * (median - vmin): the deviations |2 v - C2| are shift-invariant
    if (n & 1) {
        const uint32_t md = wave_select(x, n, (n - 1) / 2, vbits);
        median = (float)(md + vmin);
        C2 = 2u * md;
    } else {
        const uint32_t a = wave_select(x, n, n / 2 - 1, vbits), b = wave_select(x, n, n / 2, vbits);
        median = ((float)(a + vmin) + (float)(b + vmin)) / 2;
        C2 = a + b;
    }
#pragma unroll
    for (int e = 0; e < (int)(SEG_CAP / 64); ++e) x[e] = 2u * x[e] > C2 ? 2u * x[e] - C2 : C2 - 2u * x[e];
    const int dbits = vbits + 1;  // |2 v - C2| <= 2 (vmax - vmin)
    if (n & 1) {
        mad = (float)wave_select(x, n, (n - 1) / 2, dbits) * 0.5f;
    } else {
        const float d1 = (float)wave_select(x, n, n / 2 - 1, dbits) * 0.5f;
        const float d2 = (float)wave_select(x, n, n / 2, dbits) * 0.5f;
        mad = (d1 + d2) / 2.0f;
    }
    if (lane == 0) emit(median, mad);
}

// calls kept per sequence (segment results with count >= 0)
__global__ void k_count_calls(const skm_kmer_call* __restrict__ res, const uint64_t* __restrict__ seg_off,
                              uint32_t nseq, uint32_t* __restrict__ counts) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nseq) return;
    uint32_t c = 0;
    for (uint64_t j = seg_off[s]; j < seg_off[s + 1]; ++j) c += res[j].count >= 0;
    counts[s] = c;
}

__global__ void k_gather_valid(const skm_kmer_call* __restrict__ res, const uint64_t* __restrict__ seg_off,
                               const uint64_t* __restrict__ call_off, uint32_t nseq, skm_kmer_call* __restrict__ out) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nseq) return;
    uint64_t o = call_off[s];
    for (uint64_t j = seg_off[s]; j < seg_off[s + 1]; ++j)
        if (res[j].count >= 0) out[o++] = res[j];
}

// capacity of the call slot range of sequence s
__global__ void k_caps(const QMeta* __restrict__ meta, uint32_t nseq, int min_hits, uint32_t* __restrict__ cap) {
    uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nseq) return;
    uint32_t len = meta[s].len;
    uint32_t nwin = len >= 8 ? len - 7 : 0;
    cap[s] = min_hits > 2 ? nwin / (uint32_t)(min_hits - 2) + 2u : 2u * nwin + 2u;
}

// ---- exclusive scan u32 -> u64 (out has n+1 entries) ----
constexpr int SC_THREADS = 256, SC_ITEMS = 8, SC_TILE = SC_THREADS * SC_ITEMS;

__global__ void k_scan_tiles(const uint32_t* __restrict__ in, uint64_t n, uint64_t* __restrict__ out,
                             uint64_t* __restrict__ tile_sums) {
    __shared__ uint64_t s_w[SC_THREADS / 64 + 1];
    const uint64_t t0 = (uint64_t)blockIdx.x * SC_TILE + (uint64_t)threadIdx.x * SC_ITEMS;
    uint64_t v[SC_ITEMS];
    uint64_t local = 0;
#pragma unroll
    for (int j = 0; j < SC_ITEMS; ++j) {
        v[j] = (t0 + j < n) ? in[t0 + j] : 0;
        local += v[j];
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t x = local;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) s_w[wave] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t acc = 0;
        for (int w = 0; w < SC_THREADS / 64; ++w) {
            uint64_t t = s_w[w];
            s_w[w] = acc;
            acc += t;
        }
        tile_sums[blockIdx.x] = acc;
    }
    __syncthreads();
    uint64_t run = s_w[wave] + x - local;
#pragma unroll
    for (int j = 0; j < SC_ITEMS; ++j) {
        if (t0 + j < n) out[t0 + j] = run;
        run += v[j];
    }
}

__global__ void k_scan_sums(uint64_t* __restrict__ sums, uint64_t nt, uint64_t* __restrict__ total) {
    // single workgroup, sequential over chunks of 1024
    __shared__ uint64_t s_w[17];
    uint64_t carry = 0;
    for (uint64_t c0 = 0; c0 < nt; c0 += blockDim.x) {
        uint64_t i = c0 + threadIdx.x;
        uint64_t v = i < nt ? sums[i] : 0;
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        uint64_t x = v;
        for (int d = 1; d < 64; d <<= 1) {
            uint64_t y = __shfl_up(x, d, 64);
            if (lane >= d) x += y;
        }
        if (lane == 63) s_w[wave] = x;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint64_t acc = 0;
            for (int w = 0; w < (int)(blockDim.x / 64); ++w) {
                uint64_t t = s_w[w];
                s_w[w] = acc;
                acc += t;
            }
            s_w[16] = acc;
        }
        __syncthreads();
        if (i < nt) sums[i] = carry + s_w[wave] + x - v;
        carry += s_w[16];
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = carry;
}

__global__ void k_scan_add(uint64_t* __restrict__ out, uint64_t n, const uint64_t* __restrict__ tile_sums,
                           const uint64_t* __restrict__ total) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] += tile_sums[i / SC_TILE];
    if (i == n) out[n] = *total;
}

__global__ void k_gather_calls(const skm_kmer_call* __restrict__ slots, const uint64_t* __restrict__ cap_off,
                               const uint64_t* __restrict__ call_off, uint32_t nseq, skm_kmer_call* __restrict__ out) {
    uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nseq) return;
    uint64_t a = call_off[s], e = call_off[s + 1], src = cap_off[s];
    for (uint64_t j = a; j < e; ++j) out[j] = slots[src + (j - a)];
}

void Scanner::run(const uint32_t* in, uint64_t n, uint64_t* out, hipStream_t st) {
    uint64_t nt = std::max<uint64_t>(1, ceil_div(n, SC_TILE));
    tiles.ensure(8 * nt);
    total.ensure(8);
    hipLaunchKernelGGL(k_scan_tiles, dim3((uint32_t)nt), dim3(SC_THREADS), 0, st, in, n, out, tiles.as<uint64_t>());
    hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(1024), 0, st, tiles.as<uint64_t>(), nt, total.as<uint64_t>());
    hipLaunchKernelGGL(k_scan_add, dim3((uint32_t)ceil_div(n + 1, 256)), dim3(256), 0, st, out, n,
                       tiles.as<uint64_t>(), total.as<uint64_t>());
    SKM_HIP(hipGetLastError());
}

// fm[i] = function_index << 16 | mean of .dat record i (u16 words 1 and 2 of its 10 bytes): the 4
// aligned bytes the call path reads per hit (one gather instead of two 2-byte loads)
__global__ void k_dat_fm(const uint16_t* __restrict__ dat, uint64_t n, uint32_t* __restrict__ fm) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fm[i] = ((uint32_t)dat[5 * i + 1] << 16) | (uint32_t)dat[5 * i + 2];
}

// the 0 after every query sequence of a batch uploaded as the caller packed it
__global__ void k_zero_seps(const QMeta* __restrict__ meta, uint32_t n, uint8_t* __restrict__ res) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < n) res[meta[s].pstart + meta[s].len] = 0;
}

// the b == 7 (g word, rank) pair lines from g and the rank table (defined with the BDZ builder)
__global__ void k_mph_blk(const uint32_t* __restrict__ g, uint64_t gwords, const uint32_t* __restrict__ rank,
                          uint64_t nrank, uint64_t nblk, uint32_t* __restrict__ blk);

}  // namespace skm

using namespace skm;

struct skm_query {
    skm_db* db = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t ev[5] = {};
    float last_ms[5] = {};
    uint32_t nseq = 0;
    uint64_t rp = 0, n_windows = 0;
    DevBuf d_res, d_meta, d_hits, d_scr, d_scr_off, d_caps, d_cap_off, d_slots, d_counts, d_call_off, d_calls;
    DevBuf d_seg_off, d_segs, d_segres, d_pool_ctr;
    Scanner scan;
    uint64_t n_calls = 0;
    bool ran = false;
    std::unique_ptr<HostPool> pool;  // packs the residues (created on first use)
};

namespace {

void db_upload(skm_db* db, const uint8_t* dat, size_t dat_len) {
    SKM_HIP(hipSetDevice(db->device));
    Bdz& h = db->bdz;
    SKM_CHECK(dat_len % 10 == 0, SKM_E_IO, "kmer_data.dat size is not a multiple of 10");
    db->dat_records = dat_len / 10;
    SKM_CHECK(db->dat_records >= h.m, SKM_E_IO, "kmer_data.dat has fewer records than the hash size");
    const size_t gbytes = ((h.g.size() + 63) / 64) * 64 + 64;
    std::vector<uint8_t> g(gbytes, 0xFF);
    std::memcpy(g.data(), h.g.data(), h.g.size());
    db->d_g.ensure(gbytes);
    SKM_HIP(hipMemcpy(db->d_g.p, g.data(), gbytes, hipMemcpyHostToDevice));
    db->d_rank.ensure(4 * std::max<size_t>(h.ranktable.size(), 1));
    if (!h.ranktable.empty()) SKM_HIP(hipMemcpy(db->d_rank.p, h.ranktable.data(), 4 * h.ranktable.size(), hipMemcpyHostToDevice));
    db->d_dat.ensure(std::max<size_t>(dat_len, 16));
    if (dat_len) SKM_HIP(hipMemcpy(db->d_dat.p, dat, dat_len, hipMemcpyHostToDevice));
    DevBdz& D = db->dev;
    D.g = db->d_g.as<uint32_t>();
    D.ranktable = db->d_rank.as<uint32_t>();
    D.dat = db->d_dat.as<uint16_t>();
    D.m = h.m;
    D.r = h.r;
    D.b = h.b;
    D.seed = h.seed;
    D.r_magic = h.r ? (~0ull / h.r + 1) : 0;
    db->m = h.m;
    // the record words from the uploaded records, on the device
    const uint64_t nrec = dat_len / 10;
    db->d_fm.ensure(4 * std::max<uint64_t>(nrec, 1));
    if (nrec)
        hipLaunchKernelGGL(k_dat_fm, dim3((uint32_t)ceil_div(nrec, 256)), dim3(256), 0, 0, db->d_dat.as<uint16_t>(), nrec,
                           db->d_fm.as<uint32_t>());
    D.fm = db->d_fm.as<uint32_t>();
    // b == 7: g and the rank table interleaved, one 64-byte line per 128 vertices -- pairs (g word
    // w, rank of its first vertex = rank table entry plus the assigned vertices of the words before
    // it), so one 8-byte load gives a vertex's g value and rank; built on the device from the
    // uploaded g (padded with 0xFF) and rank table
    D.blk = nullptr;
    if (h.b == 7) {
        const uint64_t nblk = (uint64_t)h.n / 128 + 2;
        db->d_blk.ensure(64 * nblk);
        hipLaunchKernelGGL(k_mph_blk, dim3((uint32_t)ceil_div(nblk, 256)), dim3(256), 0, 0, db->d_g.as<uint32_t>(),
                           (uint64_t)(gbytes / 4), db->d_rank.as<uint32_t>(), (uint64_t)h.ranktable.size(), nblk,
                           db->d_blk.as<uint32_t>());
        D.blk = db->d_blk.as<uint32_t>();
    }
    SKM_HIP(hipGetLastError());
    SKM_HIP(hipDeviceSynchronize());
}

void db_upload_kept(skm_db* db, const uint64_t* keys, const skm_stored_kmer_data* data, size_t n) {
    SKM_HIP(hipSetDevice(db->device));
    SKM_CHECK(n < 0xFFFFFFFFull, SKM_E_ARG, "too many kept k-mers for a u32 record index");
    db->exact = true;
    db->m = (uint32_t)n;
    db->dat_records = n;
    int lg = std::max(4, ilog2_ceil(2 * (uint64_t)std::max<size_t>(n, 1)));  // load factor <= 1/2
    const uint64_t T = 1ull << lg;
    db->d_xtab.ensure(16 * T);
    db->d_dat.ensure(std::max<size_t>(10 * n, 16));
    SKM_HIP(hipMemset(db->d_xtab.p, 0, 16 * T));
    if (n) SKM_HIP(hipMemcpy(db->d_dat.p, data, 10 * n, hipMemcpyHostToDevice));
    DevBdz& D = db->dev;
    D = DevBdz{};
    D.dat = db->d_dat.as<uint16_t>();
    D.m = (uint32_t)n;
    D.xtab = db->d_xtab.as<uint4>();
    D.xmask = T - 1;
    D.xshift = 64u - (uint32_t)lg;
    D.fm = nullptr;  // the exact path reads the record word from the slot
    if (n) {
        DevBuf dk, dbad;
        dk.ensure(8 * n);
        dbad.ensure(4);
        SKM_HIP(hipMemcpy(dk.p, keys, 8 * n, hipMemcpyHostToDevice));
        SKM_HIP(hipMemset(dbad.p, 0, 4));
        hipLaunchKernelGGL(k_exact_insert, dim3((uint32_t)ceil_div(n, 256)), dim3(256), 0, 0, dk.as<uint64_t>(),
                           db->d_dat.as<uint16_t>(), (uint64_t)n, db->d_xtab.as<uint4>(), T - 1, 64u - (uint32_t)lg,
                           dbad.as<uint32_t>());
        SKM_HIP(hipGetLastError());
        uint32_t bad = 0;
        SKM_HIP(hipMemcpy(&bad, dbad.p, 4, hipMemcpyDeviceToHost));
        SKM_CHECK(!(bad & 1u), SKM_E_ARG, "kept k-mer key 0 is not a valid k-mer");
        SKM_CHECK(!(bad & 2u), SKM_E_ARG, "duplicate kept k-mer keys");
    }
}

bool read_file(const char* path, std::vector<uint8_t>& out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    f.seekg(0, std::ios::end);
    std::streamoff n = f.tellg();
    f.seekg(0);
    out.resize((size_t)n);
    if (n) f.read((char*)out.data(), n);
    return (bool)f;
}

// a whole file into an uninitialised buffer, read by a few threads with pread (the C2 DB's .dat is
// 1.7 GB: one zero-filled vector and one stream read took half of skm_db_open)
bool read_file_par(const char* path, std::unique_ptr<uint8_t[]>& out, uint64_t& n) {
    const int fd = ::open(path, O_RDONLY);
    if (fd < 0) return false;
    struct stat sb;
    if (::fstat(fd, &sb) != 0) {
        ::close(fd);
        return false;
    }
    n = (uint64_t)sb.st_size;
    out.reset(new uint8_t[std::max<uint64_t>(n, 1)]);
    const uint64_t piece = std::max<uint64_t>(64ull << 20, (n + 7) / 8);
    const int nt = (int)std::max<uint64_t>(1, std::min<uint64_t>(8, (n + piece - 1) / piece));
    std::atomic<bool> ok{true};
    auto part = [&](int t) {
        const uint64_t a = (uint64_t)t * piece, b = std::min(n, a + piece);
        for (uint64_t o = a; o < b;) {
            const ssize_t r = ::pread(fd, out.get() + o, (size_t)std::min<uint64_t>(b - o, 1ull << 30), (off_t)o);
            if (r <= 0) {
                ok = false;
                return;
            }
            o += (uint64_t)r;
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(part, t);
    part(0);
    for (auto& x : th) x.join();
    ::close(fd);
    return ok.load();
}

void query_run(skm_query* q, const skm_annot_opts* o) {
    skm_db* db = q->db;
    SKM_HIP(hipSetDevice(db->device));
    hipStream_t st = q->stream;
    SKM_HIP(hipEventRecord(q->ev[0], st));
    if (q->rp && db->m) {
        uint64_t nthreads = ceil_div(q->rp, LK_POS);
        uint32_t grid = (uint32_t)std::min<uint64_t>(ceil_div(nthreads, LK_THREADS), 256ull * 16);
        if (db->exact)
            hipLaunchKernelGGL(k_lookup<LK_EXACT>, dim3(grid), dim3(LK_THREADS), 0, st, q->d_res.as<uint8_t>(),
                               q->rp, db->dev, q->d_hits.as<uint32_t>());
        else if (db->dev.b == 7)
            hipLaunchKernelGGL(k_lookup<LK_BDZ7>, dim3(grid), dim3(LK_THREADS), 0, st, q->d_res.as<uint8_t>(),
                               q->rp, db->dev, q->d_hits.as<uint32_t>());
        else
            hipLaunchKernelGGL(k_lookup<LK_BDZ>, dim3(grid), dim3(LK_THREADS), 0, st, q->d_res.as<uint8_t>(),
                               q->rp, db->dev, q->d_hits.as<uint32_t>());
    } else if (q->rp) {
        SKM_HIP(hipMemsetAsync(q->d_hits.p, 0xFF, 4 * q->rp, st));
    }
    SKM_HIP(hipGetLastError());
    SKM_HIP(hipEventRecord(q->ev[1], st));
    const uint32_t ns = q->nseq;
    if (ns) {
        hipLaunchKernelGGL(k_caps, dim3(ceil_div(ns, 256)), dim3(256), 0, st, q->d_meta.as<QMeta>(), ns, o->min_hits,
                           q->d_caps.as<uint32_t>());
        q->scan.run(q->d_caps.as<uint32_t>(), ns, q->d_cap_off.as<uint64_t>(), st);
        uint64_t cap_total = 0;
        SKM_HIP(hipMemcpyAsync(&cap_total, q->d_cap_off.as<uint64_t>() + ns, 8, hipMemcpyDeviceToHost, st));
        SKM_HIP(hipStreamSynchronize(st));
        q->d_slots.ensure(sizeof(skm_kmer_call) * std::max<uint64_t>(cap_total, 1));
        CallArgs A;
        A.meta = q->d_meta.as<QMeta>();
        A.hits = q->d_hits.as<uint32_t>();
        A.scratch = q->d_scr.as<uint16_t>();
        A.scr_off = q->d_scr_off.as<uint64_t>();
        A.cap_off = q->d_cap_off.as<uint64_t>();
        A.slots = q->d_slots.as<skm_kmer_call>();
        A.counts = q->d_counts.as<uint32_t>();
        A.nseq = ns;
        A.min_hits = o->min_hits;
        A.max_gap = o->max_gap;
        A.ignore_hypo = o->ignore_hypo && o->hypo_index >= 0;
        A.mean_mode = o->mean_mode;
        A.mad_mode = o->mad_mode;
        A.hypo = o->hypo_index >= 0 ? (uint32_t)o->hypo_index : 0xFFFFFFFFu;
        SKM_HIP(hipEventRecord(q->ev[2], st));
        hipLaunchKernelGGL(k_calls_scan, dim3(ceil_div(ns, 64)), dim3(64), 0, st, A, q->d_slots.as<uint4>());
        SKM_HIP(hipGetLastError());
        q->scan.run(q->d_counts.as<uint32_t>(), ns, q->d_seg_off.as<uint64_t>(), st);
        uint64_t nseg = 0;
        SKM_HIP(hipMemcpyAsync(&nseg, q->d_seg_off.as<uint64_t>() + ns, 8, hipMemcpyDeviceToHost, st));
        SKM_HIP(hipStreamSynchronize(st));
        q->d_segs.ensure(16 * std::max<uint64_t>(nseg, 1));
        q->d_segres.ensure(sizeof(skm_kmer_call) * std::max<uint64_t>(nseg, 1));
        q->d_scr.ensure(2 * (q->n_windows + 2 * nseg + 64));
        q->d_pool_ctr.ensure(8);
        SKM_HIP(hipMemsetAsync(q->d_pool_ctr.p, 0, 8, st));
        hipLaunchKernelGGL(k_gather_segs, dim3(ceil_div(ns, 256)), dim3(256), 0, st, q->d_slots.as<uint4>(),
                           q->d_cap_off.as<uint64_t>(), q->d_seg_off.as<uint64_t>(), ns, q->d_segs.as<uint4>());
        if (nseg) {
            auto kseg = A.mad_mode == 1 ? k_seg_process<true> : k_seg_process<false>;
            hipLaunchKernelGGL(kseg, dim3((uint32_t)ceil_div(nseg, SEG_WAVES)), dim3(64 * SEG_WAVES), 0, st, A,
                               q->d_segs.as<uint4>(), (uint32_t)nseg, q->d_segres.as<skm_kmer_call>(),
                               q->d_scr.as<uint16_t>(), q->d_pool_ctr.as<unsigned long long>());
        }
        SKM_HIP(hipGetLastError());
        SKM_HIP(hipEventRecord(q->ev[3], st));
        hipLaunchKernelGGL(k_count_calls, dim3(ceil_div(ns, 256)), dim3(256), 0, st, q->d_segres.as<skm_kmer_call>(),
                           q->d_seg_off.as<uint64_t>(), ns, q->d_counts.as<uint32_t>());
        q->scan.run(q->d_counts.as<uint32_t>(), ns, q->d_call_off.as<uint64_t>(), st);
        SKM_HIP(hipMemcpyAsync(&q->n_calls, q->d_call_off.as<uint64_t>() + ns, 8, hipMemcpyDeviceToHost, st));
        SKM_HIP(hipStreamSynchronize(st));
        q->d_calls.ensure(sizeof(skm_kmer_call) * std::max<uint64_t>(q->n_calls, 1));
        hipLaunchKernelGGL(k_gather_valid, dim3(ceil_div(ns, 256)), dim3(256), 0, st, q->d_segres.as<skm_kmer_call>(),
                           q->d_seg_off.as<uint64_t>(), q->d_call_off.as<uint64_t>(), ns, q->d_calls.as<skm_kmer_call>());
        SKM_HIP(hipGetLastError());
    } else {
        SKM_HIP(hipEventRecord(q->ev[2], st));
        SKM_HIP(hipEventRecord(q->ev[3], st));
        q->n_calls = 0;
    }
    SKM_HIP(hipEventRecord(q->ev[4], st));
    SKM_HIP(hipEventSynchronize(q->ev[4]));
    SKM_HIP(hipEventElapsedTime(&q->last_ms[0], q->ev[0], q->ev[1]));  // lookup
    SKM_HIP(hipEventElapsedTime(&q->last_ms[1], q->ev[2], q->ev[3]));  // hitset
    SKM_HIP(hipEventElapsedTime(&q->last_ms[2], q->ev[3], q->ev[4]));  // compaction
    SKM_HIP(hipEventElapsedTime(&q->last_ms[3], q->ev[0], q->ev[4]));  // total
    q->ran = true;
}

}  // namespace

extern "C" {

int skm_db_open_mem(skm_db** out, const uint8_t* mph, size_t mph_len, const uint8_t* dat, size_t dat_len, int device) {
    SKM_API_BEGIN
    SKM_CHECK(out && mph, SKM_E_ARG, "null argument");
    auto* db = new skm_db();
    db->device = device;
    std::string err;
    if (!bdz_parse(mph, mph_len, db->bdz, err)) {
        delete db;
        throw Error(SKM_E_IO, "kmer_data.mph: " + err);
    }
    try {
        db_upload(db, dat, dat_len);
    } catch (...) {
        delete db;
        throw;
    }
    *out = db;
    SKM_API_END
}

int skm_db_open(skm_db** out, const char* mph_path, const char* dat_path, int device) {
    SKM_API_BEGIN
    SKM_CHECK(out && mph_path && dat_path, SKM_E_ARG, "null argument");
    std::vector<uint8_t> mph;
    std::unique_ptr<uint8_t[]> dat;
    uint64_t dat_len = 0;
    SKM_CHECK(read_file(mph_path, mph), SKM_E_IO, std::string("cannot read ") + mph_path);
    SKM_CHECK(read_file_par(dat_path, dat, dat_len), SKM_E_IO, std::string("cannot read ") + dat_path);
    int rc = skm_db_open_mem(out, mph.data(), mph.size(), dat.get(), dat_len, device);
    if (rc) return rc;
    SKM_API_END
}

int skm_db_open_kept(skm_db** out, const uint64_t* keys, const skm_stored_kmer_data* data, size_t n, int device) {
    SKM_API_BEGIN
    SKM_CHECK(out && (n == 0 || (keys && data)), SKM_E_ARG, "null argument");
    auto* db = new skm_db();
    db->device = device;
    try {
        db_upload_kept(db, keys, data, n);
    } catch (...) {
        delete db;
        throw;
    }
    *out = db;
    SKM_API_END
}

int skm_db_size(skm_db* db, uint32_t* m) {
    if (!db || !m) return SKM_E_ARG;
    *m = db->m;
    return SKM_OK;
}

extern "C++" {
// mode 0: exact table; 1: generic bdz_search (any b); 2: the (g word, rank) pair lines (b == 7)
template <int MODE>
__global__ void k_lookup_keys(const uint64_t* __restrict__ keys, uint64_t n, DevBdz D, uint32_t* __restrict__ out) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t k = keys[i];
    const uint32_t lo = (uint32_t)k, hi = (uint32_t)(k >> 32);
    out[i] = MODE == 0 ? exact_lookup(D, lo, hi) : MODE == 1 ? bdz_lookup(D, lo, hi) : bdz7_lookup(D, lo, hi);
}
}  // extern "C++"

static int db_lookup(skm_db* db, const uint64_t* keys, size_t n, uint32_t* idx_out, bool generic) {
    SKM_API_BEGIN
    SKM_CHECK(db && (n == 0 || (keys && idx_out)), SKM_E_ARG, "null argument");
    if (n == 0) return SKM_OK;
    SKM_HIP(hipSetDevice(db->device));
    if (db->m == 0) {
        for (size_t i = 0; i < n; ++i) idx_out[i] = 0;  // empty hash: every key maps to rank 0 == size (miss)
        return SKM_OK;
    }
    DevBuf dk, dout;
    dk.ensure(8 * n);
    dout.ensure(4 * n);
    SKM_HIP(hipMemcpy(dk.p, keys, 8 * n, hipMemcpyHostToDevice));
    const dim3 grid((uint32_t)ceil_div(n, 256)), blk(256);
    // the same search the annotate / matrix kernels run: pair lines whenever the DB has them
    if (db->exact)
        hipLaunchKernelGGL(k_lookup_keys<0>, grid, blk, 0, 0, dk.as<uint64_t>(), (uint64_t)n, db->dev, dout.as<uint32_t>());
    else if (db->dev.blk && !generic)
        hipLaunchKernelGGL(k_lookup_keys<2>, grid, blk, 0, 0, dk.as<uint64_t>(), (uint64_t)n, db->dev, dout.as<uint32_t>());
    else
        hipLaunchKernelGGL(k_lookup_keys<1>, grid, blk, 0, 0, dk.as<uint64_t>(), (uint64_t)n, db->dev, dout.as<uint32_t>());
    SKM_HIP(hipGetLastError());
    SKM_HIP(hipMemcpy(idx_out, dout.p, 4 * n, hipMemcpyDeviceToHost));
    SKM_API_END
}

int skm_db_lookup(skm_db* db, const uint64_t* keys, size_t n, uint32_t* idx_out) {
    return db_lookup(db, keys, n, idx_out, false);
}

int skm_debug_db_lookup_generic(skm_db* db, const uint64_t* keys, size_t n, uint32_t* idx_out) {
    return db_lookup(db, keys, n, idx_out, true);
}

void skm_db_close(skm_db* db) {
    if (!db) return;
    skm_query_destroy(db->aq);
    delete db;
}

int skm_mph_build(const uint64_t* keys, const skm_stored_kmer_data* data, size_t n, uint32_t seed, const char* mph_path,
                  const char* dat_path) {
    SKM_API_BEGIN
    SKM_CHECK((n == 0 || (keys && data)) && mph_path && dat_path, SKM_E_ARG, "null argument");
    Bdz h;
    std::string err;
    SKM_CHECK(bdz_build(keys, n, seed, h, err), SKM_E_ARG, err);
    // dense record array indexed by the hash (perfect_hash.h:41-54): unwritten slots would keep the
    // StoredKmerData defaults, but a minimal perfect hash writes every slot.
    std::vector<skm_stored_kmer_data> kd(n);
    for (size_t i = 0; i < n; ++i) {
        uint8_t kb[8];
        std::memcpy(kb, &keys[i], 8);
        uint32_t idx = bdz_search(h, kb, 8);
        SKM_CHECK(idx < n, SKM_E_ARG, "BDZ construction produced an out-of-range slot");
        kd[idx] = data[i];
    }
    std::vector<uint8_t> img = bdz_dump(h);
    std::ofstream fm(mph_path, std::ios::binary);
    SKM_CHECK((bool)fm, SKM_E_IO, std::string("cannot write ") + mph_path);
    fm.write((const char*)img.data(), (std::streamsize)img.size());
    std::ofstream fd(dat_path, std::ios::binary);
    SKM_CHECK((bool)fd, SKM_E_IO, std::string("cannot write ") + dat_path);
    if (n) fd.write((const char*)kd.data(), (std::streamsize)(sizeof(skm_stored_kmer_data) * n));
    SKM_CHECK((bool)fm && (bool)fd, SKM_E_IO, "write failed");
    SKM_API_END
}

namespace {
// (Re)loads a query object with a batch of sequences: the packed residues (one 0 after each
// sequence) and the per-sequence tables on the device; the buffers only grow, so a reused query
// (skm_annotate's, one per DB) allocates nothing once it has seen its largest batch.  Input that is
// already packed (sequence s at sum_{t<s} (len_t + 1), a 0 after each) is uploaded as it is.
void query_setup(skm_query* q, const uint8_t* residues, const uint64_t* seq_off, const uint32_t* seq_len,
                 size_t n_seqs) {
    SKM_HIP(hipSetDevice(q->db->device));
    if (!q->stream) {
        SKM_HIP(hipStreamCreateWithFlags(&q->stream, hipStreamNonBlocking));
        for (auto& e : q->ev) SKM_HIP(hipEventCreate(&e));
    }
    q->ran = false;
    q->n_calls = 0;
    std::vector<QMeta> meta(n_seqs);
    std::vector<uint64_t> scr_off(n_seqs);
    uint64_t total = 0, nwin_tot = 0;
    // packed offsets: the caller's bytes [0, max_end) -- which hold every sequence, so the buffer
    // spans them -- go to the device as they are, and the separators are zeroed there (no byte
    // outside a sequence is relied on)
    bool packed = true;
    uint64_t max_end = 0;
    for (size_t s = 0; s < n_seqs; ++s) {
        meta[s].pstart = total;
        meta[s].len = seq_len[s];
        meta[s].pad = 0;
        packed = packed && seq_off[s] == total;
        if (seq_len[s]) max_end = std::max<uint64_t>(max_end, seq_off[s] + seq_len[s]);
        total += (uint64_t)seq_len[s] + 1;
        scr_off[s] = nwin_tot;
        nwin_tot += seq_len[s] >= 8 ? seq_len[s] - 7 : 0;
    }
    // otherwise the packed residues, copied by the host pool in byte-balanced sequence ranges
    // (10 M queries are ~3 GB)
    std::vector<uint8_t> res;
    const uint8_t* src = residues;
    if (!packed) {
        res.resize(total);
        if (!q->pool) q->pool.reset(new HostPool(n_seqs > 4096 ? HostPool::default_threads() : 1));
        const int parts = std::max(1, std::min<int>(4 * q->pool->threads(), (int)(total >> 20)));
        q->pool->run(parts, [&](int p) {
            const uint64_t lo = total * (uint64_t)p / (uint64_t)parts, hi = total * (uint64_t)(p + 1) / (uint64_t)parts;
            auto first_at = [&](uint64_t x) {  // first sequence starting at or after byte x
                size_t a = 0, e = n_seqs;
                while (a < e) {
                    const size_t mid = (a + e) / 2;
                    if (meta[mid].pstart < x) a = mid + 1; else e = mid;
                }
                return a;
            };
            for (size_t s = first_at(lo), e = first_at(hi); s < e; ++s) {
                std::memcpy(res.data() + meta[s].pstart, residues + seq_off[s], seq_len[s]);
                res[meta[s].pstart + seq_len[s]] = 0;
            }
        });
        src = res.data();
    }
    q->nseq = (uint32_t)n_seqs;
    q->rp = total;
    q->n_windows = nwin_tot;
    // hits are written in 16-window groups: pad to a multiple of 16 positions
    const uint64_t rp_pad = ceil_div(q->rp + 1, LK_POS) * LK_POS;
    q->d_res.ensure(rp_pad + 64);
    const uint64_t body = packed ? max_end : q->rp;
    SKM_HIP(hipMemsetAsync(q->d_res.as<uint8_t>() + body, 0, rp_pad + 64 - body, q->stream));
    if (body) SKM_HIP(hipMemcpyAsync(q->d_res.p, src, body, hipMemcpyHostToDevice, q->stream));
    q->d_meta.ensure(sizeof(QMeta) * std::max<size_t>(n_seqs, 1));
    if (n_seqs) SKM_HIP(hipMemcpyAsync(q->d_meta.p, meta.data(), sizeof(QMeta) * n_seqs, hipMemcpyHostToDevice, q->stream));
    if (packed && n_seqs)
        hipLaunchKernelGGL(k_zero_seps, dim3((uint32_t)ceil_div(n_seqs, 256)), dim3(256), 0, q->stream,
                           q->d_meta.as<QMeta>(), (uint32_t)n_seqs, q->d_res.as<uint8_t>());
    q->d_hits.ensure(4 * (rp_pad + 16));
    q->d_scr.ensure(2 * std::max<uint64_t>(nwin_tot, 1));
    q->d_scr_off.ensure(8 * std::max<size_t>(n_seqs, 1));
    if (n_seqs) SKM_HIP(hipMemcpyAsync(q->d_scr_off.p, scr_off.data(), 8 * n_seqs, hipMemcpyHostToDevice, q->stream));
    q->d_caps.ensure(4 * std::max<size_t>(n_seqs, 1));
    q->d_cap_off.ensure(8 * (n_seqs + 1));
    q->d_counts.ensure(4 * std::max<size_t>(n_seqs, 1));
    q->d_call_off.ensure(8 * (n_seqs + 1));
    q->d_seg_off.ensure(8 * (n_seqs + 1));
    SKM_HIP(hipStreamSynchronize(q->stream));  // the host arrays above go out of scope
}
}  // namespace

int skm_query_create(skm_query** out, skm_db* db, const uint8_t* residues, const uint64_t* seq_off,
                     const uint32_t* seq_len, size_t n_seqs) {
    SKM_API_BEGIN
    SKM_CHECK(out && db, SKM_E_ARG, "null argument");
    SKM_CHECK(n_seqs == 0 || (residues && seq_off && seq_len), SKM_E_ARG, "null array");
    SKM_CHECK(n_seqs < 0xFFFFFFFFull, SKM_E_ARG, "too many query sequences in one batch");
    auto* q = new skm_query();
    q->db = db;
    try {
        query_setup(q, residues, seq_off, seq_len, n_seqs);
    } catch (...) {
        skm_query_destroy(q);
        throw;
    }
    *out = q;
    SKM_API_END
}

int skm_query_run(skm_query* q, const skm_annot_opts* opts) {
    SKM_API_BEGIN
    SKM_CHECK(q && opts, SKM_E_ARG, "null argument");
    SKM_CHECK(opts->mean_mode == 0 || opts->mean_mode == 1, SKM_E_ARG, "mean_mode must be 0 or 1");
    SKM_CHECK(opts->mad_mode == 0 || opts->mad_mode == 1, SKM_E_ARG, "mad_mode must be 0 or 1");
    SKM_CHECK(opts->min_hits >= 1 && opts->max_gap >= 0, SKM_E_ARG, "invalid min_hits / max_gap");
    query_run(q, opts);
    SKM_API_END
}

int skm_query_last_timings(skm_query* q, float* ms, int cap) {
    if (!q || !ms) return SKM_E_ARG;
    int n = std::min(cap, 4);
    for (int i = 0; i < n; ++i) ms[i] = q->last_ms[i];
    return n;
}

int skm_query_calls(skm_query* q, skm_calls* out) {
    SKM_API_BEGIN
    SKM_CHECK(q && out, SKM_E_ARG, "null argument");
    SKM_CHECK(q->ran, SKM_E_STATE, "skm_query_run has not been called");
    SKM_HIP(hipSetDevice(q->db->device));
    std::memset(out, 0, sizeof(*out));
    out->n_seqs = q->nseq;
    out->n_calls = q->n_calls;
    out->n_windows = q->n_windows;
    out->call_off = (uint64_t*)std::malloc(8 * (q->nseq + 1));
    out->calls = (skm_kmer_call*)std::malloc(sizeof(skm_kmer_call) * std::max<uint64_t>(q->n_calls, 1));
    SKM_CHECK(out->call_off && out->calls, SKM_E_OOM, "host allocation failed");
    if (q->nseq)
        SKM_HIP(hipMemcpyAsync(out->call_off, q->d_call_off.p, 8 * (q->nseq + 1), hipMemcpyDeviceToHost, q->stream));
    else
        out->call_off[0] = 0;
    if (q->n_calls)
        SKM_HIP(hipMemcpyAsync(out->calls, q->d_calls.p, sizeof(skm_kmer_call) * q->n_calls, hipMemcpyDeviceToHost, q->stream));
    SKM_HIP(hipStreamSynchronize(q->stream));
    SKM_API_END
}

int skm_query_window_hits(skm_query* q, uint64_t* hit_off, uint32_t* pos, uint32_t* fm, uint64_t cap, uint64_t* n_out) {
    SKM_API_BEGIN
    SKM_CHECK(q && hit_off && n_out, SKM_E_ARG, "null argument");
    SKM_CHECK(q->ran, SKM_E_STATE, "skm_query_run has not been called");
    SKM_HIP(hipSetDevice(q->db->device));
    // the device hit words, one per packed residue position (sequence s starts at pstart(s) =
    // sum over t < s of len_t + 1): a window's word is its record's function_index << 16 | mean,
    // NO_HIT where k_lookup found no usable window or no record
    std::vector<uint32_t> h(q->rp);
    if (q->rp) SKM_HIP(hipMemcpyAsync(h.data(), q->d_hits.p, 4 * q->rp, hipMemcpyDeviceToHost, q->stream));
    std::vector<QMeta> meta(q->nseq);
    if (q->nseq) SKM_HIP(hipMemcpyAsync(meta.data(), q->d_meta.p, sizeof(QMeta) * q->nseq, hipMemcpyDeviceToHost, q->stream));
    SKM_HIP(hipStreamSynchronize(q->stream));
    uint64_t n = 0;
    for (uint32_t s = 0; s < q->nseq; ++s) {
        hit_off[s] = n;
        const uint64_t a = meta[s].pstart;
        for (uint32_t i = 0; i < meta[s].len; ++i) {
            const uint32_t w = h[a + i];
            if (w == NO_HIT) continue;
            if (n < cap) {
                if (pos) pos[n] = i;
                if (fm) fm[n] = w;
            }
            ++n;
        }
    }
    hit_off[q->nseq] = n;
    *n_out = n;
    SKM_API_END
}

void skm_query_destroy(skm_query* q) {
    if (!q) return;
    (void)hipSetDevice(q->db->device);
    if (q->stream) (void)hipStreamSynchronize(q->stream);
    for (auto& e : q->ev)
        if (e) (void)hipEventDestroy(e);
    if (q->stream) (void)hipStreamDestroy(q->stream);
    delete q;
}

namespace {
int annotate_setup(skm_db* db, const uint8_t* residues, const uint64_t* seq_off, const uint32_t* seq_len, size_t n_seqs) {
    SKM_API_BEGIN
    SKM_CHECK(db, SKM_E_ARG, "null argument");
    SKM_CHECK(n_seqs == 0 || (residues && seq_off && seq_len), SKM_E_ARG, "null array");
    SKM_CHECK(n_seqs < 0xFFFFFFFFull, SKM_E_ARG, "too many query sequences in one batch");
    if (!db->aq) {
        db->aq = new skm_query();
        db->aq->db = db;
    }
    query_setup(db->aq, residues, seq_off, seq_len, n_seqs);
    SKM_API_END
}
}  // namespace

// one batch through the DB's own reused query (its device buffers, stream and host pool persist
// from call to call: a batch of the annotate CLI used to create and free all of them)
int skm_annotate(skm_db* db, const uint8_t* residues, const uint64_t* seq_off, const uint32_t* seq_len, size_t n_seqs,
                 const skm_annot_opts* opts, skm_calls* out) {
    int rc = annotate_setup(db, residues, seq_off, seq_len, n_seqs);
    if (!rc) rc = skm_query_run(db->aq, opts);
    if (!rc) rc = skm_query_calls(db->aq, out);
    return rc;
}

void skm_calls_free(skm_calls* c) {
    if (!c) return;
    std::free(c->call_off);
    std::free(c->calls);
    std::memset(c, 0, sizeof(*c));
}

}  // extern "C"

// ------------------------------------------------------------------------------------------
// BDZ construction on the device (build_perfect_hash, perfect_hash.h:11-69, via cmph_new
// CMPH_BDZ): same parameters as the host builder (r = ceil(1.23 m / 3) made odd, n = 3r,
// jenkins seeds from mt19937(seed)), 3-hypergraph peeled in parallel rounds:
//   k_mph_edges     one thread per key: 3 vertices, (degree, incident edge-id sum) += (1, e) in
//                   one 64-bit atomic each
//   k_mph_frontier  vertices of degree 1 (one reservation per wave of 8 x 64 vertices)
//   k_mph_peel      a frontier vertex v peels its only edge e iff v is the first degree-1
//                   vertex of e (deterministic: one peeler per edge, no atomics on e)
//   k_mph_apply     the peeled edges leave their vertices; vertices that drop to degree 1 form
//                   the next frontier
//   k_mph_assign    rounds in reverse: the free vertex gets (position - g[u1] - g[u2]) mod 3
//                   (unassigned = 3 = 0 mod 3); edges of one round never share a free vertex
//                   and their other vertices were freed in later rounds, so a round is parallel
//   rank table on the host from g; records placed by the device lookup.
// Any acyclic peel order gives a valid minimal perfect hash; this one is deterministic (the
// frontier ORDER depends on atomics, the peeled SET of a round and the g values do not).
//
// Sized for the headline build's kept set (C3: 2.89 G keys, 3.55 G vertices): cmph's BDZ keeps
// m, n and r as cmph_uint32, so every key, edge and vertex index here is a u32 and the limit is
// n = 3r < 2^32 (MPH_MAX_KEYS).  An edge's vertices are recomputed from its key where they are
// needed (8 random bytes instead of a 12-byte edge array: 35 GB less HBM at C3); a peeled entry is
// the edge id plus its free position in a byte array beside it; the peel state (degrees, XORs,
// frontiers) is freed before the records are uploaded and placed.
// ------------------------------------------------------------------------------------------
namespace skm {

constexpr uint64_t MPH_MAX_KEYS = 3400000000ull;  // n = 3 * ceil(1.23 m / 3) (+ retries) < 2^32 - 2^12

struct MphDev {
    uint32_t r;
    uint64_t r_magic;
    uint32_t seed;
};

__device__ __forceinline__ void mph_verts(const MphDev& P, uint64_t k, uint32_t v[3]) {
    uint32_t a = 0x9e3779b9u + (uint32_t)k, b = 0x9e3779b9u + (uint32_t)(k >> 32), c = P.seed + 8u;
    jmix(a, b, c);
    v[0] = fastmod(a, P.r_magic, P.r);
    v[1] = fastmod(b, P.r_magic, P.r) + P.r;
    v[2] = fastmod(c, P.r_magic, P.r) + 2u * P.r;
}

// A vertex's peel state is one u64: its degree << 40 | the sum of its incident edge ids.  One
// 64-bit atomic adds or removes an edge (the degree and the id sum move together, half the
// atomics of separate degree and XOR words); at degree 1 the sum is the edge.  The sum stays below
// 2^40 while the degree is below 256: a vertex reaching MPH_DEG_MAX fails the attempt (never seen
// at 2.89 G keys: the degrees are ~Poisson(2.4)).
constexpr int MPH_SUM_BITS = 40;
constexpr uint64_t MPH_ONE = 1ull << MPH_SUM_BITS;
constexpr uint32_t MPH_DEG_MAX = 255;
__device__ __forceinline__ uint32_t vdeg(uint64_t x) { return (uint32_t)(x >> MPH_SUM_BITS); }

// (grids: m, n < 2^32 - 2^12, so a u32 global thread index never wraps)
__global__ void k_mph_edges(const uint64_t* __restrict__ keys, uint32_t m, MphDev P, unsigned long long* __restrict__ dx,
                            uint32_t* __restrict__ bad) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= m) return;
    uint32_t v[3];
    mph_verts(P, keys[e], v);
#pragma unroll
    for (int j = 0; j < 3; ++j)
        if (vdeg(atomicAdd(&dx[v[j]], MPH_ONE + e)) + 1u >= MPH_DEG_MAX) atomicOr(bad, 1u);
}

// MPH_FR_PER vertices per thread, one frontier reservation per wave (a single counter: at C3's
// 3.55 G vertices one atomic per 64 vertices was 55 M atomics on one address per attempt)
constexpr uint32_t MPH_FR_PER = 8;
__global__ __launch_bounds__(256) void k_mph_frontier(const unsigned long long* __restrict__ dx, uint32_t nv,
                                                      uint32_t* __restrict__ fr, uint32_t* __restrict__ nfr) {
    const uint64_t v0 = (uint64_t)blockIdx.x * (256u * MPH_FR_PER) + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t lt = (1ull << lane) - 1ull;
    uint64_t bal[MPH_FR_PER];
    uint32_t tot = 0;
#pragma unroll
    for (uint32_t j = 0; j < MPH_FR_PER; ++j) {
        const uint64_t v = v0 + 256u * j;
        bal[j] = __ballot(v < nv && vdeg(dx[v]) == 1u);
        tot += (uint32_t)__popcll(bal[j]);
    }
    if (tot == 0) return;  // wave-uniform
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(nfr, tot);
    base = (uint32_t)__shfl((int)base, 0);
#pragma unroll
    for (uint32_t j = 0; j < MPH_FR_PER; ++j) {
        if ((bal[j] >> lane) & 1ull) fr[base + (uint32_t)__popcll(bal[j] & lt)] = (uint32_t)(v0 + 256u * j);
        base += (uint32_t)__popcll(bal[j]);
    }
}

// peeled entry: the edge id in pe[], the position of its free vertex in pp[]
__global__ void k_mph_peel(const uint32_t* __restrict__ fr, uint32_t nf, const uint64_t* __restrict__ keys, MphDev P,
                           const unsigned long long* __restrict__ dx, uint32_t* __restrict__ pe,
                           uint8_t* __restrict__ pp, uint32_t* __restrict__ npeeled) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    bool take = false;
    uint32_t e = 0, pos = 0;
    if (i < nf) {
        const uint32_t v = fr[i];
        const uint64_t xv = dx[v];
        if (vdeg(xv) == 1u) {
            e = (uint32_t)xv;
            uint32_t u[3];
            mph_verts(P, keys[e], u);
            for (uint32_t p = 0; p < 3; ++p) {
                if (vdeg(dx[u[p]]) == 1u) {  // first degree-1 vertex of e peels it
                    take = u[p] == v;
                    pos = p;
                    break;
                }
            }
        }
    }
    const uint64_t bal = __ballot(take);
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t base = 0;
    if (lane == 0 && bal) base = atomicAdd(npeeled, (uint32_t)__popcll(bal));
    base = __shfl(base, 0);
    if (take) {
        const uint32_t o = base + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
        pe[o] = e;
        pp[o] = (uint8_t)pos;
    }
}

__global__ void k_mph_apply(const uint32_t* __restrict__ pe, uint32_t p0, uint32_t p1, const uint64_t* __restrict__ keys,
                            MphDev P, unsigned long long* __restrict__ dx, uint32_t* __restrict__ fr,
                            uint32_t* __restrict__ nfr) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = t < p1 - p0;
    const uint32_t e = live ? pe[p0 + t] : 0u;
    uint32_t u[3] = {0u, 0u, 0u};
    if (live) mph_verts(P, keys[e], u);
    bool add[3] = {false, false, false};
#pragma unroll
    for (int j = 0; j < 3; ++j)
        if (live) {
            add[j] = vdeg(atomicAdd(&dx[u[j]], 0ull - (MPH_ONE + e))) == 2u;
        }
    // the vertices that dropped to degree 1: one frontier reservation per wave (a single counter)
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t lt = (1ull << lane) - 1ull;
    uint64_t bal[3];
    uint32_t tot = 0;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        bal[j] = __ballot(add[j]);
        tot += (uint32_t)__popcll(bal[j]);
    }
    if (tot == 0) return;  // wave-uniform
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(nfr, tot);
    base = (uint32_t)__shfl((int)base, 0);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        if (add[j]) fr[base + (uint32_t)__popcll(bal[j] & lt)] = u[j];
        base += (uint32_t)__popcll(bal[j]);
    }
}

__device__ __forceinline__ uint32_t gmod3(const uint32_t* g, uint32_t i) {
    const uint32_t x = (g[i >> 4] >> ((i & 15u) * 2)) & 3u;
    return x == 3u ? 0u : x;
}

__global__ void k_mph_assign(const uint32_t* __restrict__ pe, const uint8_t* __restrict__ pp, uint32_t p0, uint32_t p1,
                             const uint64_t* __restrict__ keys, MphDev P, uint32_t* __restrict__ g) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= p1 - p0) return;
    const uint32_t e = pe[p0 + t], p = pp[p0 + t];
    uint32_t u[3];
    mph_verts(P, keys[e], u);
    uint32_t s = 0, fv = 0;
#pragma unroll
    for (uint32_t j = 0; j < 3; ++j) {
        if (j == p)
            fv = u[j];
        else
            s += gmod3(g, u[j]);
    }
    const uint32_t val = (p + 6u - s) % 3u;
    // entries start at 3 (0b11): clear the bits that are 0 in val
    atomicAnd(&g[fv >> 4], ~((3u & ~val) << ((fv & 15u) * 2)));
}

// bad: 1 = a key's slot >= m, 2 = two keys on one slot (the slot bitmap), 4 = the pair-line
// search disagrees with the generic one, 8 = a .dat record differs from its key's record
__global__ void k_mph_place(const uint64_t* __restrict__ keys, uint32_t m, DevBdz D, const uint16_t* __restrict__ data,
                            uint16_t* __restrict__ dat, uint32_t* __restrict__ bits, uint32_t* __restrict__ bad) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint64_t k = keys[i];
    const uint32_t idx = bdz_lookup(D, (uint32_t)k, (uint32_t)(k >> 32));
    if (idx >= m) {
        atomicOr(bad, 1u);
        return;
    }
    if (bits) {
        const uint32_t bit = 1u << (idx & 31u);
        if (atomicOr(&bits[idx >> 5], bit) & bit) atomicOr(bad, 2u);
    }
#pragma unroll
    for (int j = 0; j < 5; ++j) dat[5ull * idx + j] = data[5ull * i + j];
}

// the b == 7 (g word, rank) pair lines of the annotate lookup (db_upload's layout), built on the
// device from g and the rank table: one thread per 128-vertex block
__global__ void k_mph_blk(const uint32_t* __restrict__ g, uint64_t gwords, const uint32_t* __restrict__ rank,
                          uint64_t nrank, uint64_t nblk, uint32_t* __restrict__ blk) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nblk) return;
    uint32_t r = q < nrank ? rank[q] : 0u;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        const uint64_t gi = 8 * q + (uint64_t)w;
        const uint32_t x = gi < gwords ? g[gi] : 0xFFFFFFFFu;
        blk[16 * q + 2 * (uint64_t)w] = x;
        blk[16 * q + 2 * (uint64_t)w + 1] = r;
        r += 16u - (uint32_t)__popc(x & (x >> 1) & 0x55555555u);
    }
}

__global__ void k_mph_verify(const uint64_t* __restrict__ keys, uint32_t m, DevBdz D, const uint16_t* __restrict__ data,
                             const uint16_t* __restrict__ dat, uint32_t* __restrict__ bad) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint64_t k = keys[i];
    const uint32_t idx = bdz_lookup(D, (uint32_t)k, (uint32_t)(k >> 32));
    const uint32_t idx7 = bdz7_lookup(D, (uint32_t)k, (uint32_t)(k >> 32));
    if (idx7 != idx) atomicOr(bad, 4u);
    if (idx >= m) return;
    bool same = true;
#pragma unroll
    for (int j = 0; j < 5; ++j) same &= dat[5ull * idx + j] == data[5ull * i + j];
    if (!same) atomicOr(bad, 8u);
}

// keys ascending?  [0] |= 1 if some adjacent pair is out of order, 2 if some adjacent pair is equal
__global__ void k_mph_adjacent(const uint64_t* __restrict__ keys, uint32_t m, uint32_t* __restrict__ flags) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i + 1 >= m) return;
    const uint64_t a = keys[i], b = keys[i + 1];
    if (a > b) atomicOr(flags, 1u);
    if (a == b) atomicOr(flags, 2u);
}

}  // namespace skm

namespace {
double secs_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
}

// A device array written to a file by a few host threads, each copying its own range D2H into an
// uninitialised host buffer and pwrite-ing it at its offset: the copies of one range overlap the
// page-cache writes of another (the C2 CLI's .dat is 1.7 GB; one zero-filled vector, one copy and
// one ofstream write took most of its MPH phase).  Returns false on an I/O or HIP error.
bool write_device_file(const char* path, const void* dev, uint64_t bytes, int device) {
    const int fd = ::open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) return false;
    std::unique_ptr<uint8_t[]> host(new uint8_t[std::max<uint64_t>(bytes, 1)]);
    const uint64_t piece = std::max<uint64_t>(64ull << 20, (bytes + 7) / 8);
    const int nt = (int)std::min<uint64_t>(8, (bytes + piece - 1) / piece);
    std::atomic<bool> ok{true};
    auto part = [&](int t) {
        const uint64_t a = (uint64_t)t * piece, b = std::min(bytes, a + piece);
        if (a >= b) return;
        if (hipSetDevice(device) != hipSuccess ||
            hipMemcpy(host.get() + a, static_cast<const uint8_t*>(dev) + a, b - a, hipMemcpyDeviceToHost) != hipSuccess) {
            ok = false;
            return;
        }
        for (uint64_t o = a; o < b;) {
            const ssize_t w = ::pwrite(fd, host.get() + o, (size_t)std::min<uint64_t>(b - o, 1ull << 30), (off_t)o);
            if (w <= 0) {
                ok = false;
                return;
            }
            o += (uint64_t)w;
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(part, t);
    part(0);
    for (auto& x : th) x.join();
    return ::close(fd) == 0 && ok.load();
}
}  // namespace

extern "C" int skm_mph_build_device_ex(const uint64_t* keys, const skm_stored_kmer_data* data, size_t nkeys,
                                       uint32_t seed, const char* mph_path, const char* dat_path, int device, int verify,
                                       skm_mph_stats* stats) {
    SKM_API_BEGIN
    SKM_CHECK(nkeys == 0 || (keys && data), SKM_E_ARG, "null argument");
    const auto t_all = std::chrono::steady_clock::now();
    skm_mph_stats st{};
    st.n_keys = nkeys;
    if (device < 0 || nkeys < 1024) {
        SKM_CHECK(mph_path && dat_path, SKM_E_ARG, "the host builder writes both files");
        const int rc = skm_mph_build(keys, data, nkeys, seed, mph_path, dat_path);
        st.total_s = secs_since(t_all);
        if (stats) *stats = st;
        return rc;
    }
    SKM_CHECK(nkeys <= MPH_MAX_KEYS, SKM_E_ARG,
              "too many keys for one BDZ: cmph keeps m, n = 3r as 32-bit words (n = 1.23 m < 2^32)");
    SKM_HIP(hipSetDevice(device));
    const uint32_t m = (uint32_t)nkeys;
    Bdz h;
    h.m = m;
    h.r = (uint32_t)std::ceil((1.23 * m) / 3);
    if (h.r % 2 == 0) h.r += 1;
    h.b = 7;
    h.k = 1u << h.b;
    auto t = std::chrono::steady_clock::now();
    DevBuf dkeys, ddata, ddx, dfr0, dfr1, dpe, dpp, dcnt, dg;
    dkeys.ensure(8ull * m);
    SKM_HIP(hipMemcpy(dkeys.p, keys, 8ull * m, hipMemcpyHostToDevice));
    st.upload_s = secs_since(t);
    t = std::chrono::steady_clock::now();
    dpe.ensure(4ull * m);
    dpp.ensure(m);
    dcnt.ensure(64);
    uint32_t* cnt = dcnt.as<uint32_t>();  // [0] frontier A, [1] frontier B, [2] peeled, [3] bad, [4] order
    std::mt19937 rng(seed);
    bool ok = false;
    std::vector<uint32_t> rounds;  // peel-list boundaries
    MphDev P{};
    for (int attempt = 0; attempt < 1000 && !ok; ++attempt) {
        if (attempt > 0 && attempt % 20 == 0) h.r += 2;
        if (attempt == 1) {  // duplicate keys never give an acyclic graph: check once
            SKM_HIP(hipMemset(cnt + 4, 0, 4));
            hipLaunchKernelGGL(k_mph_adjacent, dim3(ceil_div(m, 256)), dim3(256), 0, 0, dkeys.as<uint64_t>(), m, cnt + 4);
            uint32_t order = 0;
            SKM_HIP(hipMemcpy(&order, cnt + 4, 4, hipMemcpyDeviceToHost));
            bool dup = (order & 2u) != 0;
            if (order & 1u) {  // not ascending: sort a host copy
                std::vector<uint64_t> sk(keys, keys + nkeys);
                std::sort(sk.begin(), sk.end());
                dup = std::adjacent_find(sk.begin(), sk.end()) != sk.end();
            }
            SKM_CHECK(!dup, SKM_E_ARG, "BDZ construction failed: duplicate keys");
        }
        h.n = 3 * h.r;
        SKM_CHECK((uint64_t)3 * h.r < 0xFFFFF000ull, SKM_E_ARG, "BDZ vertex count exceeds 32 bits");
        h.ranktablesize = (uint32_t)std::ceil(h.n / (double)h.k);
        h.seed = rng();
        P = MphDev{h.r, ~0ull / h.r + 1, h.seed};
        const uint32_t nv = h.n;
        ddx.ensure(8ull * nv);
        dfr0.ensure(4ull * nv);
        dfr1.ensure(4ull * nv);
        SKM_HIP(hipMemset(ddx.p, 0, 8ull * nv));
        SKM_HIP(hipMemset(dcnt.p, 0, 64));
        hipLaunchKernelGGL(k_mph_edges, dim3(ceil_div(m, 256)), dim3(256), 0, 0, dkeys.as<uint64_t>(), m, P,
                           ddx.as<unsigned long long>(), cnt + 3);
        hipLaunchKernelGGL(k_mph_frontier, dim3(ceil_div(nv, 256 * MPH_FR_PER)), dim3(256), 0, 0, ddx.as<unsigned long long>(), nv,
                           dfr0.as<uint32_t>(), cnt + 0);
        SKM_HIP(hipGetLastError());
        uint32_t hc[4] = {0, 0, 0, 0};
        SKM_HIP(hipMemcpy(hc, cnt, 16, hipMemcpyDeviceToHost));
        uint32_t nf = hc[3] ? 0u : hc[0], npeeled = 0;  // a vertex of degree >= MPH_DEG_MAX: next seed
        rounds.assign(1, 0);
        DevBuf* cur = &dfr0;
        DevBuf* nxt = &dfr1;
        int fcur = 0;
        while (nf > 0) {
            hipLaunchKernelGGL(k_mph_peel, dim3(ceil_div(nf, 256)), dim3(256), 0, 0, cur->as<uint32_t>(), nf,
                               dkeys.as<uint64_t>(), P, ddx.as<unsigned long long>(), dpe.as<uint32_t>(),
                               dpp.as<uint8_t>(), cnt + 2);
            SKM_HIP(hipMemset(cnt + (1 - fcur), 0, 4));
            uint32_t np = 0;
            SKM_HIP(hipMemcpy(&np, cnt + 2, 4, hipMemcpyDeviceToHost));
            if (np == npeeled) break;
            hipLaunchKernelGGL(k_mph_apply, dim3(ceil_div(np - npeeled, 256)), dim3(256), 0, 0, dpe.as<uint32_t>(),
                               npeeled, np, dkeys.as<uint64_t>(), P, ddx.as<unsigned long long>(),
                               nxt->as<uint32_t>(), cnt + (1 - fcur));
            SKM_HIP(hipGetLastError());
            rounds.push_back(np);
            npeeled = np;
            SKM_HIP(hipMemcpy(&nf, cnt + (1 - fcur), 4, hipMemcpyDeviceToHost));
            std::swap(cur, nxt);
            fcur = 1 - fcur;
        }
        ok = npeeled == m;
        st.attempts = (uint32_t)attempt + 1;
    }
    SKM_CHECK(ok, SKM_E_ARG, "BDZ construction failed: no acyclic 3-graph in 1000 attempts");
    st.peel_rounds = (uint32_t)rounds.size() - 1;
    st.n_vertices = h.n;
    ddx.release();
    dfr0.release();
    dfr1.release();
    st.peel_s = secs_since(t);
    // assignment, rounds in reverse
    t = std::chrono::steady_clock::now();
    const uint64_t gwords = ceil_div(h.n, 16) + 1;
    dg.ensure(4 * gwords);
    SKM_HIP(hipMemset(dg.p, 0xFF, 4 * gwords));
    for (size_t ri = rounds.size() - 1; ri >= 1; --ri) {
        const uint32_t p0 = rounds[ri - 1], p1 = rounds[ri];
        hipLaunchKernelGGL(k_mph_assign, dim3(ceil_div(p1 - p0, 256)), dim3(256), 0, 0, dpe.as<uint32_t>(),
                           dpp.as<uint8_t>(), p0, p1, dkeys.as<uint64_t>(), P, dg.as<uint32_t>());
    }
    SKM_HIP(hipGetLastError());
    dpe.release();
    dpp.release();
    std::vector<uint32_t> gw(gwords);
    SKM_HIP(hipMemcpy(gw.data(), dg.p, 4 * gwords, hipMemcpyDeviceToHost));
    st.assign_s = secs_since(t);
    t = std::chrono::steady_clock::now();
    h.g.assign((size_t)std::ceil(h.n / 4.0), 0xFF);
    std::memcpy(h.g.data(), gw.data(), h.g.size());
    h.ranktable.assign(h.ranktablesize, 0);
    {
        uint64_t count = 0;
        for (uint64_t i = 0; i < h.ranktablesize; ++i) {
            h.ranktable[i] = (uint32_t)count;
            const uint64_t v0 = i * h.k, v1 = std::min<uint64_t>(h.n, v0 + h.k);
            for (uint64_t v = v0; v < v1; v += 16) {  // k = 128: whole words; entries past n stay 3
                const uint32_t w = gw[v >> 4];
                count += 16u - (uint32_t)__builtin_popcount(w & (w >> 1) & 0x55555555u);
            }
        }
        SKM_CHECK(count == m, SKM_E_ARG, "BDZ construction: assigned vertex count != number of keys");
    }
    st.rank_s = secs_since(t);
    // place the records: dat[search(key)] = data
    t = std::chrono::steady_clock::now();
    DevBuf drank, ddat, dbits;
    drank.ensure(4ull * std::max<uint32_t>(h.ranktablesize, 1));
    SKM_HIP(hipMemcpy(drank.p, h.ranktable.data(), 4ull * h.ranktablesize, hipMemcpyHostToDevice));
    ddata.ensure(10ull * m);
    SKM_HIP(hipMemcpy(ddata.p, data, 10ull * m, hipMemcpyHostToDevice));
    ddat.ensure(10ull * m);
    if (verify) {
        dbits.ensure(4 * (ceil_div(m, 32) + 1));
        SKM_HIP(hipMemset(dbits.p, 0, 4 * (ceil_div(m, 32) + 1)));
    }
    DevBdz D{};
    D.g = dg.as<uint32_t>();
    D.ranktable = drank.as<uint32_t>();
    D.m = m;
    D.r = h.r;
    D.b = h.b;
    D.seed = h.seed;
    D.r_magic = ~0ull / h.r + 1;
    SKM_HIP(hipMemset(cnt + 3, 0, 4));
    hipLaunchKernelGGL(k_mph_place, dim3(ceil_div(m, 256)), dim3(256), 0, 0, dkeys.as<uint64_t>(), m, D,
                       ddata.as<uint16_t>(), ddat.as<uint16_t>(), verify ? dbits.as<uint32_t>() : nullptr, cnt + 3);
    SKM_HIP(hipGetLastError());
    uint32_t bad = 0;
    SKM_HIP(hipMemcpy(&bad, cnt + 3, 4, hipMemcpyDeviceToHost));
    SKM_CHECK(!(bad & 1u), SKM_E_ARG, "BDZ construction produced an out-of-range slot");
    SKM_CHECK(!(bad & 2u), SKM_E_STATE, "BDZ construction mapped two keys to one slot");
    st.place_s = secs_since(t);
    if (verify) {  // the annotate path's b == 7 pair-line search over every key, and the records
        t = std::chrono::steady_clock::now();
        dbits.release();
        const uint64_t nblk = (uint64_t)h.n / 128 + 2;
        DevBuf dblk;
        dblk.ensure(64 * nblk);
        hipLaunchKernelGGL(k_mph_blk, dim3(ceil_div(nblk, 256)), dim3(256), 0, 0, dg.as<uint32_t>(), gwords,
                           drank.as<uint32_t>(), (uint64_t)h.ranktablesize, nblk, dblk.as<uint32_t>());
        D.blk = dblk.as<uint32_t>();
        hipLaunchKernelGGL(k_mph_verify, dim3(ceil_div(m, 256)), dim3(256), 0, 0, dkeys.as<uint64_t>(), m, D,
                           ddata.as<uint16_t>(), ddat.as<uint16_t>(), cnt + 3);
        SKM_HIP(hipGetLastError());
        SKM_HIP(hipMemcpy(&bad, cnt + 3, 4, hipMemcpyDeviceToHost));
        SKM_CHECK(!(bad & 4u), SKM_E_STATE, "BDZ pair-line search differs from the generic search");
        SKM_CHECK(!(bad & 8u), SKM_E_STATE, "BDZ .dat record differs from its key's record");
        st.verified = 1;
        st.verify_s = secs_since(t);
    }
    t = std::chrono::steady_clock::now();
    if (mph_path) {
        std::vector<uint8_t> img = bdz_dump(h);
        std::ofstream fm(mph_path, std::ios::binary);
        SKM_CHECK((bool)fm, SKM_E_IO, std::string("cannot write ") + mph_path);
        fm.write((const char*)img.data(), (std::streamsize)img.size());
        SKM_CHECK((bool)fm, SKM_E_IO, "write failed");
    }
    if (dat_path)
        SKM_CHECK(write_device_file(dat_path, ddat.p, 10ull * m, device), SKM_E_IO, std::string("cannot write ") + dat_path);
    st.write_s = secs_since(t);
    st.total_s = secs_since(t_all);
    if (stats) *stats = st;
    SKM_API_END
}

extern "C" int skm_mph_build_device(const uint64_t* keys, const skm_stored_kmer_data* data, size_t nkeys, uint32_t seed,
                                    const char* mph_path, const char* dat_path, int device) {
    if (!mph_path || !dat_path) {
        skm::set_last_error("null argument");
        return SKM_E_ARG;
    }
    return skm_mph_build_device_ex(keys, data, nkeys, seed, mph_path, dat_path, device, 0, nullptr);
}
