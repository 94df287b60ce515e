// skm_matrix.hip -- kmers-matrix-distance on the device (BASELINE configs[4]).
//
// Replaces MatrixDistance::compute (matrix_distance.h:45-170) / the kmers-matrix-distance main
// (kmers-matrix-distance.cc:94-212): every query window of for_each_kmer<8> is looked up in the
// signature DB (CmphKmerDb::fetch, cmph_kmer.h:139-147), hits of "hypothetical protein" are
// dropped (ignore_hypothetical(true), :164 -> call_functions.tcc:285-289), hit_cb's length filter
// keeps a hit iff mean - 2 sd <= seqlen <= mean + 2 sd with sd = var ? sqrt(var) : 0.1 seqlen
// (:123-152), kmer_hit_map[kmer] collects the distinct sequence indices (SeqIdMap,
// seq_id_map.h:12-27) and every pair id1 < id2 of a k-mer's set adds one to seq_dist[id1][id2]
// (:176-196).
//
// Device pipeline (one GPU computes the rows [r0, r1) of the upper-triangle count matrix):
//   k_md_hits      one thread per 16 window positions of the packed queries: window validity,
//                  DB lookup, record, filters; surviving (kmer, index) records compacted with one
//                  atomic per wave
//   k_md_slot      kmer -> slot of an open-addressing table (atomicCAS); composite
//                  slot << idx_bits | index
//   k_rs_hist / k_rs_scatter   LSD radix sort of the composites, 8-bit digits (stable: per-round
//                  wave match by ballots + per-wave digit counts in LDS)
//   k_md_starts / k_md_segstart   k-mer group boundaries (composites with equal slot)
//   k_md_rowstat / k_md_rowfill   row lists: every distinct composite with partners after it in
//                  its group, bucketed by its index id1 (counting sort)
//   k_md_rows      one 1024-thread workgroup per row (work queue): the row's pair counts in an
//                  LDS histogram over its columns (u16 counters: 65536 columns per pass), short
//                  partner lists walked by a lane, long ones by a wave; nonzero columns compacted
//                  in column order -- no global atomics on the counts, no dense matrix in HBM
//   k_md_gather    (id1, id2, count) triples in row order
// Multi-GPU (skm_matrix_set_transport / skm_matrix_set_comm): rank r of W holds a
// contiguous range of the query sequences.  It looks up only those (k_md_hits), sends each hit to
// the k-mer's owner GPU (k_md_owner_*, one all-to-all), the owner groups its k-mers (slot table +
// radix sort) and sends every group's members to the GPUs whose row band (skm_matrix_tile_rows)
// the group has pairs in -- the suffix of members from the band's first row on (k_md_route_*,
// one all-to-all) -- and each GPU counts the pairs of its band from the groups it received.  The
// host concatenates the bands in row order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "skm_common.h"
#include "skm_lookup.h"
#include "skm_util.h"

#if defined(SKM_WITH_RCCL)
#include <rccl/rccl.h>
#endif

namespace skm {

constexpr int MD_THREADS = 256;

struct MdHitArgs {
    const uint8_t* res;        // packed residues, a 0 after each sequence
    uint64_t rp;               // packed length
    const QMeta* meta;         // [nseq]
    uint32_t nseq;
    const uint32_t* seq_idx;   // SeqIdMap index per sequence
    DevBdz D;
    int exact;                 // KeptKmerDB lookup
    uint32_t hypo;             // function index dropped by ignore_hypothetical (0xFFFFFFFF: none)
    unsigned long long* rec_key;
    uint32_t* rec_idx;
    unsigned long long* nrec;
};

__device__ __forceinline__ uint32_t md_rank(const DevBdz& D, int exact, uint32_t lo, uint32_t hi) {
    return exact ? exact_lookup(D, lo, hi) : (D.blk ? bdz7_lookup(D, lo, hi) : bdz_lookup(D, lo, hi));
}

// largest s with meta[s].pstart <= p
__device__ __forceinline__ uint32_t seq_of(const QMeta* meta, uint32_t nseq, uint64_t p) {
    uint32_t lo = 0, hi = nseq;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (meta[mid].pstart <= p)
            lo = mid;
        else
            hi = mid;
    }
    return lo;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    return x;
}

__global__ __launch_bounds__(MD_THREADS) void k_md_hits(MdHitArgs A) {
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x * LK_POS;
    const uint32_t lane = threadIdx.x & 63u;
    // every lane of a wave runs the same number of iterations (wave-wide compaction below)
    const uint64_t first = ((uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u)) * LK_POS;
    for (uint64_t wbase = first; wbase < A.rp; wbase += step) {
        const uint64_t base = wbase + (uint64_t)lane * LK_POS;
        uint64_t key[LK_POS];
        uint32_t idx[LK_POS];
        uint32_t keep = 0;  // bit t: window base + t is a surviving hit
        if (base < A.rp) {
            const uint4 v0 = *reinterpret_cast<const uint4*>(A.res + base);
            const uint4 v1 = *reinterpret_cast<const uint4*>(A.res + base + 16);
            const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
            uint32_t bad = 0, amb = 0;
#pragma unroll
            for (int j = 0; j < 25; ++j) {
                const uint32_t c = (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
                const bool a = ambig(c);
                amb |= (a ? 1u : 0u) << j;
                bad |= ((a || c == 0) ? 1u : 0u) << j;
            }
            uint32_t s = 0xFFFFFFFFu;
            uint64_t send = 0;
#pragma unroll
            for (int t = 0; t < LK_POS; ++t) {
                const uint64_t p = base + t;
                uint32_t lo, hi;
                key_at(w, t, lo, hi);
                key[t] = ((uint64_t)hi << 32) | lo;
                idx[t] = 0;
                if (p >= A.rp || ((bad >> t) & 0xFFu) != 0 || ((amb >> (t + 8)) & 1u) != 0) continue;
                if (s == 0xFFFFFFFFu || p >= send) {
                    s = seq_of(A.meta, A.nseq, p);
                    send = A.meta[s].pstart + A.meta[s].len;
                }
                const uint32_t r = md_rank(A.D, A.exact, lo, hi);
                if (r >= A.D.m) continue;  // fetch: no callback (cmph_kmer.h:143-146)
                const uint16_t* rec = A.D.dat + (uint64_t)r * 5;
                const uint32_t func = rec[1], mean_u = rec[2], var_u = rec[4];
                if (func == A.hypo) continue;  // ignore_hypothetical (call_functions.tcc:285-289)
                // hit_cb (kmers-matrix-distance.cc:132-149): reject seqlen outside mean -/+ 2 sd.
                // var != 0: |seqlen - mean| > 2 sqrt(var) exactly in integers (for an integer var
                // that is not a square, mean +/- 2 sqrt(var) is >= 1e-3 away from any integer, far
                // beyond the double roundings of the reference); var == 0: the reference's doubles.
                const uint32_t len = A.meta[s].len;
                bool ok;
                if (var_u == 0) {
                    const double seqlen = (double)len, mean = (double)mean_u;
                    const double sd = seqlen * 0.1;
                    const double cb = mean - sd * 2.0, ct = mean + sd * 2.0;
                    ok = !(seqlen < cb || seqlen > ct);
                } else {
                    const int64_t dl = (int64_t)len - (int64_t)mean_u;
                    ok = (uint64_t)(dl * dl) <= 4ull * var_u;
                }
                if (!ok) continue;
                idx[t] = A.seq_idx[s];
                keep |= 1u << t;
            }
        }
        const uint32_t cnt = (uint32_t)__popc(keep);
        const uint32_t incl = wave_incl_scan(cnt);
        const uint32_t total = __shfl(incl, 63, 64);
        if (total == 0) continue;
        unsigned long long wb = 0;
        if (lane == 63) wb = atomicAdd(A.nrec, (unsigned long long)total);
        wb = __shfl(wb, 63, 64);
        uint64_t o = wb + incl - cnt;
#pragma unroll
        for (int t = 0; t < LK_POS; ++t) {
            if (!((keep >> t) & 1u)) continue;
            A.rec_key[o] = key[t];
            A.rec_idx[o] = idx[t];
            ++o;
        }
    }
}

// kmer -> table slot (the table holds kmers; 0 = empty, a window never has a 0 byte)
__global__ void k_md_slot(const unsigned long long* __restrict__ keys, const uint32_t* __restrict__ idx,
                          const unsigned long long* __restrict__ nrec, unsigned long long* __restrict__ tab,
                          uint64_t mask, uint32_t shift, uint32_t idx_bits, uint64_t* __restrict__ comp) {
    const uint64_t n = *nrec;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long k = keys[i];
        uint64_t h = xmix(k) >> shift;
        for (;;) {
            const unsigned long long prev = atomicCAS(&tab[h], 0ull, k);
            if (prev == 0ull || prev == k) break;
            h = (h + 1) & mask;
        }
        comp[i] = (h << idx_bits) | idx[i];
    }
}

// ---- LSD radix sort of u64 keys, 8-bit digits ----
constexpr int RS_THREADS = 256, RS_ITEMS = 16, RS_TILE = RS_THREADS * RS_ITEMS;

__global__ __launch_bounds__(RS_THREADS) void k_rs_hist(const uint64_t* __restrict__ in, uint64_t n, int shift,
                                                        uint32_t nblocks, uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * RS_TILE;
#pragma unroll
    for (int j = 0; j < RS_ITEMS; ++j) {
        const uint64_t i = t0 + (uint64_t)j * RS_THREADS + threadIdx.x;
        if (i < n) atomicAdd(&h[(uint32_t)(in[i] >> shift) & 255u], 1u);
    }
    __syncthreads();
    hist[(uint64_t)threadIdx.x * nblocks + blockIdx.x] = h[threadIdx.x];
}

// Stable scatter: items in striped order (round j, thread t); within a round the rank among equal
// digits comes from a ballot match in the wave plus the counts of the lower waves.
__global__ __launch_bounds__(RS_THREADS) void k_rs_scatter(const uint64_t* __restrict__ in, uint64_t n, int shift,
                                                           uint32_t nblocks, const uint64_t* __restrict__ offs,
                                                           uint64_t* __restrict__ out) {
    constexpr int NW = RS_THREADS / 64;
    __shared__ uint64_t run[256];
    __shared__ uint32_t wcnt[NW][256];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    run[tid] = offs[(uint64_t)tid * nblocks + blockIdx.x];
    const uint64_t t0 = (uint64_t)blockIdx.x * RS_TILE;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (int j = 0; j < RS_ITEMS; ++j) {
        const uint64_t i = t0 + (uint64_t)j * RS_THREADS + tid;
        if (t0 + (uint64_t)j * RS_THREADS >= n) break;  // block-uniform
#pragma unroll
        for (int w = 0; w < NW; ++w) wcnt[w][tid] = 0;
        __syncthreads();
        const bool valid = i < n;
        const uint64_t k = valid ? in[i] : 0;
        const uint32_t d = (uint32_t)(k >> shift) & 255u;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const uint64_t m = __ballot((d >> b) & 1u);
            peers &= ((d >> b) & 1u) ? m : ~m;
        }
        const uint32_t pre = (uint32_t)__popcll(peers & lt);
        if (valid && pre == 0) wcnt[wave][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        if (valid) {
            uint64_t o = run[d] + pre;
            for (uint32_t w = 0; w < wave; ++w) o += wcnt[w][d];
            out[o] = k;
        }
        __syncthreads();
        uint32_t add = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) add += wcnt[w][tid];
        run[tid] += add;
        __syncthreads();
    }
}

// group starts: slot differs from the previous composite
__global__ void k_md_starts(const uint64_t* __restrict__ c, uint64_t n, uint32_t idx_bits, uint32_t* __restrict__ flag) {
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    flag[e] = (e == 0 || (c[e] >> idx_bits) != (c[e - 1] >> idx_bits)) ? 1u : 0u;
}

__global__ void k_md_segstart(const uint32_t* __restrict__ flag, const uint64_t* __restrict__ S, uint64_t n,
                              uint64_t* __restrict__ segstart) {
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    if (flag[e]) segstart[S[e]] = e;
    if (e == n - 1) segstart[S[n]] = n;
}

__host__ __device__ __forceinline__ uint64_t rowbase(uint64_t i, uint64_t n) { return i * (2 * n - i - 1) / 2; }

// Row lists: element e (a distinct (kmer, index) composite whose group has members after it)
// belongs to row id1 = index(e); its partners are the distinct composites after it in its group.
struct MdRowArgs {
    const uint64_t* comp;      // sorted composites
    const uint64_t* S;         // exclusive scan of group-start flags [n+1]
    const uint64_t* segstart;  // [nseg+1]
    uint64_t n;
    uint64_t idx_mask;
    uint32_t r0, rows;         // row tile [r0, r0 + rows)
    uint64_t nidx;
    uint32_t* rowlen;          // [rows] entries per row
    uint32_t* rowub;           // [rows] partner slots per row (upper bound of its nonzero pairs)
    uint32_t* cursor;          // [rows]
    const uint64_t* rowoff;    // [rows+1] scan of rowlen
    const uint64_t* ubo;       // [rows+1] scan of rowub
    uint32_t* rowlist;         // entries (element positions) by row
    uint32_t* rownnz;          // [rows] nonzero pairs per row
    uint32_t* scratch;         // per row, from ubo[row]: (id2, count) pairs
    unsigned int* rowctr;      // work queue
    unsigned long long* incs;  // pair increments (diagnostics / roofline)
};

__device__ __forceinline__ bool md_entry(const MdRowArgs& R, uint64_t e, uint32_t& row, uint64_t& ge) {
    const uint64_t c = R.comp[e];
    if (e > 0 && R.comp[e - 1] == c) return false;  // duplicate (kmer, index)
    const uint64_t id1 = c & R.idx_mask;
    if (id1 < R.r0 || id1 >= (uint64_t)R.r0 + R.rows) return false;
    ge = R.segstart[R.S[e + 1]];  // end of e's group (group id S[e+1] - 1)
    if (ge <= e + 1) return false;
    row = (uint32_t)(id1 - R.r0);
    return true;
}

__global__ void k_md_rowstat(MdRowArgs R) {
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < R.n; e += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t row;
        uint64_t ge;
        if (!md_entry(R, e, row, ge)) continue;
        atomicAdd(&R.rowlen[row], 1u);
        atomicAdd(&R.rowub[row], (uint32_t)min<uint64_t>(ge - e - 1, 0xFFFFFFFFull));
    }
}

__global__ void k_md_rowfill(MdRowArgs R) {
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < R.n; e += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t row;
        uint64_t ge;
        if (!md_entry(R, e, row, ge)) continue;
        R.rowlist[R.rowoff[row] + atomicAdd(&R.cursor[row], 1u)] = (uint32_t)e;
    }
}

// One workgroup per row at a time (work queue): the row's pair counts accumulate in an LDS
// histogram over its columns id2 = id1+1 .. nidx-1 (u16 counters, two per word: 65536 columns per
// pass; u32 counters, 32768 per pass, when the row has > 65535 entries and a u16 could wrap) with
// a bitmap of the touched words; the touched words are then compacted in column order into the
// row's scratch range and reset (the histogram is all-zero between rows, nothing is cleared).
// The walk is flattened over the whole workgroup: the partner ranges of up to 1024 entries are
// prefix-summed and every thread takes partners by index (4 independent loads in flight).  No
// global atomics on the counts and no dense matrix in HBM.
constexpr int MR_THREADS = 1024;
constexpr uint32_t MR_WORDS = 32768;              // 128 KB of LDS
constexpr uint32_t MR_BM = MR_WORDS / 32;         // bitmap words (== MR_THREADS)
constexpr uint32_t MR_UNROLL = 4;
static_assert(MR_BM == (uint32_t)MR_THREADS, "one bitmap word per thread in the compaction");

__device__ __forceinline__ uint32_t wg_scan_excl(uint32_t v, uint32_t* s_w, uint32_t& total) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) s_w[wave] = x;
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < MR_THREADS / 64; ++w) {
        const uint32_t t = s_w[w];
        before += w < wave ? t : 0u;
        tot += t;
    }
    total = tot;
    return before + x - v;
}

__global__ __launch_bounds__(MR_THREADS) void k_md_rows(MdRowArgs R) {
    __shared__ __align__(16) uint32_t h[MR_WORDS];
    __shared__ uint32_t bm[MR_BM];
    __shared__ uint32_t sp[MR_THREADS];   // partner prefix of the sweep's entries
    __shared__ uint64_t sq[MR_THREADS];   // first partner of each entry
    __shared__ uint32_t s_w[MR_THREADS / 64];
    __shared__ uint32_t s_row;
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    for (uint32_t w = tid * 4; w < MR_WORDS; w += MR_THREADS * 4) *reinterpret_cast<uint4*>(&h[w]) = make_uint4(0, 0, 0, 0);
    bm[tid] = 0;
    uint64_t incs = 0;
    for (;;) {
        __syncthreads();
        if (tid == 0) s_row = atomicAdd(R.rowctr, 1u);
        __syncthreads();
        const uint32_t row = s_row;
        if (row >= R.rows) break;
        const uint64_t l0 = R.rowoff[row], l1 = R.rowoff[row + 1];
        if (l0 == l1) {
            if (tid == 0) R.rownnz[row] = 0;
            continue;
        }
        const uint64_t id1 = (uint64_t)R.r0 + row;
        const uint64_t ncol = R.nidx - id1 - 1;
        const bool wide = l1 - l0 > 65535u;
        const uint32_t cpp = wide ? MR_WORDS : 2u * MR_WORDS;
        const bool multi = ncol > cpp;
        uint32_t* out = R.scratch + 2 * R.ubo[row];
        uint32_t nnz = 0;
        for (uint64_t cb = 0; cb < ncol; cb += cpp) {
            const uint32_t cc = (uint32_t)min<uint64_t>(cpp, ncol - cb);
            // this pass: id2 in [clo, chi); a group's composites are sorted by index, so each
            // entry's partners in the window are one range
            const uint64_t clo = id1 + 1 + cb, chi = clo + cc;
            for (uint64_t kb = l0; kb < l1; kb += MR_THREADS) {
                const uint64_t k = kb + tid;
                uint64_t qa = 0, qb = 0;
                if (k < l1) {
                    const uint64_t e = R.rowlist[k];
                    qa = e + 1;
                    qb = R.segstart[R.S[e + 1]];
                    if (multi) {
                        uint64_t lo = qa, hi = qb;
                        while (lo < hi) {
                            const uint64_t mid = (lo + hi) >> 1;
                            if ((R.comp[mid] & R.idx_mask) < clo) lo = mid + 1; else hi = mid;
                        }
                        const uint64_t qa2 = lo;
                        hi = qb;
                        while (lo < hi) {
                            const uint64_t mid = (lo + hi) >> 1;
                            if ((R.comp[mid] & R.idx_mask) < chi) lo = mid + 1; else hi = mid;
                        }
                        qa = qa2;
                        qb = lo;
                    }
                }
                const uint32_t pc = (uint32_t)(qb - qa);
                uint32_t T;
                const uint32_t pre = wg_scan_excl(pc, s_w, T);
                sp[tid] = pre;
                sq[tid] = qa;
                __syncthreads();
                const uint32_t ne = (uint32_t)min<uint64_t>(MR_THREADS, l1 - kb);
                for (uint32_t t0 = 0; t0 < T; t0 += MR_THREADS * MR_UNROLL) {
                    uint64_t cq[MR_UNROLL], cp[MR_UNROLL];
#pragma unroll
                    for (uint32_t u = 0; u < MR_UNROLL; ++u) {
                        const uint32_t t = t0 + u * MR_THREADS + tid;
                        cq[u] = 0;
                        cp[u] = 0;
                        if (t < T) {
                            // largest entry i with sp[i] <= t
                            uint32_t i = 0;
#pragma unroll
                            for (uint32_t st = MR_THREADS / 2; st >= 1; st >>= 1)
                                if (i + st < ne && sp[i + st] <= t) i += st;
                            const uint64_t q = sq[i] + (t - sp[i]);
                            cq[u] = R.comp[q];
                            cp[u] = R.comp[q - 1];
                        }
                    }
#pragma unroll
                    for (uint32_t u = 0; u < MR_UNROLL; ++u) {
                        if (cq[u] != cp[u]) {  // a partner, not a duplicate (kmer, index)
                            const uint32_t c = (uint32_t)((cq[u] & R.idx_mask) - clo);
                            const uint32_t w = wide ? c : (c >> 1);
                            atomicAdd(&h[w], wide ? 1u : (1u << (16 * (c & 1u))));
                            atomicOr(&bm[w >> 5], 1u << (w & 31u));
                            ++incs;
                        }
                    }
                }
                __syncthreads();
            }
            // compaction: thread tid owns bitmap word tid = histogram words 32 tid .. 32 tid + 31
            const uint32_t bits = bm[tid];
            uint32_t cnt = 0;
            for (uint32_t b = bits; b; b &= b - 1) {
                const uint32_t v = h[tid * 32 + (uint32_t)__ffs(b) - 1];
                cnt += wide ? 1u : ((v & 0xFFFFu) != 0) + ((v >> 16) != 0);
            }
            uint32_t tot;
            uint32_t o = nnz + wg_scan_excl(cnt, s_w, tot);
            for (uint32_t b = bits; b; b &= b - 1) {
                const uint32_t w = tid * 32 + (uint32_t)__ffs(b) - 1;
                const uint32_t v = h[w];
                h[w] = 0;
                if (wide) {
                    out[2 * o] = (uint32_t)(clo + w);
                    out[2 * o + 1] = v;
                    ++o;
                } else {
                    if (v & 0xFFFFu) {
                        out[2 * o] = (uint32_t)(clo + 2 * w);
                        out[2 * o + 1] = v & 0xFFFFu;
                        ++o;
                    }
                    if (v >> 16) {
                        out[2 * o] = (uint32_t)(clo + 2 * w + 1);
                        out[2 * o + 1] = v >> 16;
                        ++o;
                    }
                }
            }
            bm[tid] = 0;
            nnz += tot;
            __syncthreads();  // s_w / h / bm reuse by the next pass
        }
        if (tid == 0) R.rownnz[row] = nnz;
    }
    uint64_t x = incs;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    if (lane == 0 && x) atomicAdd(R.incs, (unsigned long long)x);
}

// rows in order: (id2, count) scratch pairs -> (id1, id2, count) triples at the row's final offset
__global__ void k_md_gather(const uint32_t* __restrict__ scratch, const uint64_t* __restrict__ ubo,
                            const uint64_t* __restrict__ fo, uint32_t r0, uint32_t rows, uint32_t* __restrict__ out) {
    for (uint32_t row = blockIdx.x; row < rows; row += gridDim.x) {
        const uint64_t a = fo[row], cnt = fo[row + 1] - a;
        const uint32_t* src = scratch + 2 * ubo[row];
        for (uint64_t j = threadIdx.x; j < cnt; j += blockDim.x) {
            out[3 * (a + j)] = r0 + row;
            out[3 * (a + j) + 1] = src[2 * j];
            out[3 * (a + j) + 2] = src[2 * j + 1];
        }
    }
}

// ---- multi-GPU: hits to the k-mer's owner, groups to the row bands they touch ----
__device__ __forceinline__ uint32_t md_owner(uint64_t k, uint32_t W) {
    return (uint32_t)(((xmix(k) >> 32) * (uint64_t)W) >> 32);
}

constexpr int OW_TILE = 4096;

// cnt[W]: hits per owner (LDS counts per tile, one global add per owner per tile)
__global__ __launch_bounds__(256) void k_md_owner_count(const unsigned long long* __restrict__ keys,
                                                        const unsigned long long* __restrict__ nrec, uint32_t W,
                                                        unsigned long long* __restrict__ cnt) {
    __shared__ uint32_t c[64];
    const uint64_t n = *nrec;
    if (threadIdx.x < 64) c[threadIdx.x] = 0;
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        atomicAdd(&c[md_owner(keys[i], W)], 1u);
    __syncthreads();
    if (threadIdx.x < W && c[threadIdx.x]) atomicAdd(&cnt[threadIdx.x], (unsigned long long)c[threadIdx.x]);
}

// owner-major send buffers: each tile reserves its owners' ranges once (cur[o] starts at the
// owner's offset), then places its hits (order within an owner is immaterial: the owner sorts)
__global__ __launch_bounds__(256) void k_md_owner_scatter(const unsigned long long* __restrict__ keys,
                                                          const uint32_t* __restrict__ idx,
                                                          const unsigned long long* __restrict__ nrec, uint32_t W,
                                                          unsigned long long* __restrict__ cur,
                                                          unsigned long long* __restrict__ skey,
                                                          uint32_t* __restrict__ sidx) {
    __shared__ uint32_t c[64];
    __shared__ unsigned long long base[64];
    const uint64_t n = *nrec;
    for (uint64_t t0 = (uint64_t)blockIdx.x * OW_TILE; t0 < n; t0 += (uint64_t)gridDim.x * OW_TILE) {
        if (threadIdx.x < 64) c[threadIdx.x] = 0;
        __syncthreads();
        for (uint32_t j = threadIdx.x; j < OW_TILE && t0 + j < n; j += blockDim.x) atomicAdd(&c[md_owner(keys[t0 + j], W)], 1u);
        __syncthreads();
        if (threadIdx.x < W) {
            base[threadIdx.x] = c[threadIdx.x] ? atomicAdd(&cur[threadIdx.x], (unsigned long long)c[threadIdx.x]) : 0ull;
            c[threadIdx.x] = 0;
        }
        __syncthreads();
        for (uint32_t j = threadIdx.x; j < OW_TILE && t0 + j < n; j += blockDim.x) {
            const unsigned long long k = keys[t0 + j];
            const uint32_t o = md_owner(k, W);
            const uint64_t at = base[o] + atomicAdd(&c[o], 1u);
            skey[at] = k;
            sidx[at] = idx[t0 + j];
        }
        __syncthreads();
    }
}

// first composite of the group [a, e) whose index is >= lo (the group is sorted by index)
__device__ __forceinline__ uint64_t md_first_ge(const uint64_t* __restrict__ comp, uint64_t a, uint64_t e,
                                                uint64_t idx_mask, uint64_t lo) {
    while (a < e) {
        const uint64_t mid = (a + e) >> 1;
        if ((comp[mid] & idx_mask) < lo) a = mid + 1; else e = mid;
    }
    return a;
}

// cnt[g]: members group g sends to band b -- its suffix from band b's first row, when a
// member of the band has a partner after it; 0 otherwise
__global__ void k_md_route_count(const uint64_t* __restrict__ comp, const uint64_t* __restrict__ segstart,
                                 uint64_t G, uint64_t idx_mask, const uint32_t* __restrict__ band, uint32_t b,
                                 uint32_t* __restrict__ cnt) {
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < G; g += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t a = segstart[g], e = segstart[g + 1];
        const uint64_t f = md_first_ge(comp, a, e, idx_mask, band[b]);
        const bool send = f + 1 < e && (comp[f] & idx_mask) < band[b + 1];
        cnt[g] = send ? (uint32_t)(e - f) : 0u;
    }
}

// the members of each group for band b, as (gid << idx_bits | index) with gid = gbase + g
// (globally increasing in source-rank order: the receiver's composites are already sorted)
__global__ void k_md_route_fill(const uint64_t* __restrict__ comp, const uint64_t* __restrict__ segstart, uint64_t G,
                                uint64_t idx_mask, uint32_t idx_bits, const uint32_t* __restrict__ cnt,
                                const uint64_t* __restrict__ off, uint64_t gbase, uint64_t* __restrict__ out) {
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < G; g += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t c = cnt[g];
        if (!c) continue;
        const uint64_t e = segstart[g + 1];
        uint64_t* dst = out + off[g];
        const uint64_t f = e - c;
        for (uint32_t j = 0; j < c; ++j) dst[j] = ((gbase + g) << idx_bits) | (comp[f + j] & idx_mask);
    }
}

}  // namespace skm

using namespace skm;

struct skm_matrix {
    skm_db* db = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t ev[6] = {};
    float last_ms[6] = {};
    uint32_t nseq = 0, nidx = 0;
    uint64_t rp = 0, n_windows = 0;
    DevBuf d_res, d_meta, d_idx, d_rkey, d_ridx, d_nrec, d_tab, d_comp, d_comp2, d_hist, d_hoff, d_flag, d_S,
        d_seg, d_rlen, d_rub, d_rcur, d_roff, d_ubo, d_rnnz, d_fo, d_rlist, d_scr, d_out, d_incs;
    Scanner scan;
    uint64_t n_hits = 0, n_incs = 0, n_pairs = 0, n_groups = 0;
    bool ran = false;
    // ranks: this handle's queries are rank `rank` of `world`; joined by a host transport or RCCL
    int rank = 0, world = 1;
    skm_transport tp{};
#if defined(SKM_WITH_RCCL)
    ncclComm_t comm = nullptr;
#endif
    DevBuf d_ocnt, d_skey, d_sidx, d_band, d_rtc, d_rto, d_send, d_xbuf;
    uint64_t n_local_hits = 0, n_routed = 0;
    uint32_t band_lo = 0, band_hi = 0;
};

namespace {

// ---- rank collectives of the multi-GPU matrix (host transport or RCCL) ----
#if defined(SKM_WITH_RCCL)
#define MX_NCCL(x)                                                                                          \
    do {                                                                                                    \
        ncclResult_t _r = (x);                                                                              \
        if (_r != ncclSuccess) throw skm::Error(SKM_E_COMM, std::string("RCCL: ") + ncclGetErrorString(_r)); \
    } while (0)
#endif

void mx_tp_check(int rc, const char* what) {
    SKM_CHECK(rc == 0, SKM_E_COMM, std::string("host transport ") + what + " failed");
}

// device all-to-all of bytes: send + soff[q] (scnt[q]) to rank q, received at recv + roff[p]
void mx_alltoallv(skm_matrix* M, const uint8_t* send, const std::vector<uint64_t>& soff,
                  const std::vector<uint64_t>& scnt, uint8_t* recv, const std::vector<uint64_t>& roff,
                  const std::vector<uint64_t>& rcnt) {
    const int W = M->world, me = M->rank;
    if (M->tp.alltoallv) {
        std::vector<uint64_t> so(W), ro(W);
        uint64_t st = 0, rt = 0;
        for (int q = 0; q < W; ++q) {
            so[q] = st;
            st += scnt[q];
            ro[q] = rt;
            rt += rcnt[q];
        }
        std::vector<uint8_t> hs(std::max<uint64_t>(st, 1)), hr(std::max<uint64_t>(rt, 1));
        SKM_HIP(hipStreamSynchronize(M->stream));
        for (int q = 0; q < W; ++q)
            if (scnt[q]) SKM_HIP(hipMemcpy(hs.data() + so[q], send + soff[q], scnt[q], hipMemcpyDeviceToHost));
        mx_tp_check(M->tp.alltoallv(M->tp.ctx, hs.data(), scnt.data(), so.data(), hr.data(), rcnt.data(), ro.data()),
                    "alltoallv");
        for (int q = 0; q < W; ++q)
            if (rcnt[q]) SKM_HIP(hipMemcpy(recv + roff[q], hr.data() + ro[q], rcnt[q], hipMemcpyHostToDevice));
        return;
    }
#if defined(SKM_WITH_RCCL)
    SKM_CHECK(M->comm, SKM_E_STATE, "matrix ranks joined by neither a transport nor a communicator");
    if (scnt[me]) SKM_HIP(hipMemcpyAsync(recv + roff[me], send + soff[me], scnt[me], hipMemcpyDeviceToDevice, M->stream));
    MX_NCCL(ncclGroupStart());
    for (int q = 0; q < W; ++q) {
        if (q == me) continue;
        if (scnt[q]) MX_NCCL(ncclSend(send + soff[q], scnt[q], ncclUint8, q, M->comm, M->stream));
        if (rcnt[q]) MX_NCCL(ncclRecv(recv + roff[q], rcnt[q], ncclUint8, q, M->comm, M->stream));
    }
    MX_NCCL(ncclGroupEnd());
#else
    (void)me;
    throw Error(SKM_E_COMM, "libskm was built without RCCL");
#endif
}

// every rank sends one u64 to every rank: out[p] = what rank p sent to this rank
std::vector<uint64_t> mx_exchange_u64(skm_matrix* M, const std::vector<uint64_t>& mine) {
    const int W = M->world;
    std::vector<uint64_t> out(W, 0);
    if (M->tp.alltoallv) {
        std::vector<uint64_t> c(W, 8), o(W);
        for (int q = 0; q < W; ++q) o[q] = 8ull * q;
        mx_tp_check(M->tp.alltoallv(M->tp.ctx, mine.data(), c.data(), o.data(), out.data(), c.data(), o.data()),
                    "alltoallv");
        return out;
    }
    M->d_xbuf.ensure(16ull * W);
    uint8_t* d = M->d_xbuf.as<uint8_t>();
    SKM_HIP(hipMemcpyAsync(d, mine.data(), 8ull * W, hipMemcpyHostToDevice, M->stream));
    std::vector<uint64_t> c(W, 8), o(W);
    for (int q = 0; q < W; ++q) o[q] = 8ull * q;
    mx_alltoallv(M, d, o, c, d + 8ull * W, o, c);
    SKM_HIP(hipMemcpyAsync(out.data(), d + 8ull * W, 8ull * W, hipMemcpyDeviceToHost, M->stream));
    SKM_HIP(hipStreamSynchronize(M->stream));
    return out;
}

// the composite group-by of n (kmer, index) hits (slot table + LSD radix sort): d_comp sorted,
// d_S / d_seg the group boundaries; returns the number of groups
uint64_t md_group(skm_matrix* M, const unsigned long long* keys, const uint32_t* idx, const unsigned long long* nrec,
                  uint64_t n, uint32_t idx_bits, hipStream_t st) {
    const int lg = std::max(4, ilog2_ceil(2 * std::max<uint64_t>(n, 1)));
    const uint32_t key_bits = (uint32_t)lg + idx_bits;
    SKM_CHECK(key_bits <= 64, SKM_E_ARG, "matrix distance: too many hits / sequences for 64-bit composites");
    if (!n) return 0;
    const uint64_t T = 1ull << lg;
    M->d_tab.ensure(8 * T);
    SKM_HIP(hipMemsetAsync(M->d_tab.p, 0, 8 * T, st));
    M->d_comp.ensure(8 * n);
    M->d_comp2.ensure(8 * n);
    const uint32_t g = (uint32_t)std::min<uint64_t>(ceil_div(n, 256), 256ull * 32);
    hipLaunchKernelGGL(k_md_slot, dim3(g), dim3(256), 0, st, keys, idx, nrec, M->d_tab.as<unsigned long long>(), T - 1,
                       64u - (uint32_t)lg, idx_bits, M->d_comp.as<uint64_t>());
    SKM_HIP(hipGetLastError());
    const uint32_t nb = (uint32_t)ceil_div(n, RS_TILE);
    M->d_hist.ensure(4ull * 256 * nb);
    M->d_hoff.ensure(8ull * (256 * (uint64_t)nb + 1));
    uint64_t* a = M->d_comp.as<uint64_t>();
    uint64_t* b = M->d_comp2.as<uint64_t>();
    for (uint32_t sh = 0; sh < key_bits; sh += 8) {
        hipLaunchKernelGGL(k_rs_hist, dim3(nb), dim3(RS_THREADS), 0, st, a, n, (int)sh, nb, M->d_hist.as<uint32_t>());
        M->scan.run(M->d_hist.as<uint32_t>(), 256ull * nb, M->d_hoff.as<uint64_t>(), st);
        hipLaunchKernelGGL(k_rs_scatter, dim3(nb), dim3(RS_THREADS), 0, st, a, n, (int)sh, nb, M->d_hoff.as<uint64_t>(), b);
        SKM_HIP(hipGetLastError());
        std::swap(a, b);
    }
    if (a != M->d_comp.as<uint64_t>()) {
        std::swap(M->d_comp.p, M->d_comp2.p);
        std::swap(M->d_comp.bytes, M->d_comp2.bytes);
    }
    return 1;  // groups: md_bounds
}

// group boundaries of the sorted composites d_comp[0..n): S (scan of group starts), segstart
uint64_t md_bounds(skm_matrix* M, uint64_t n, uint32_t idx_bits, hipStream_t st) {
    if (!n) return 0;
    M->d_flag.ensure(4 * n);
    M->d_S.ensure(8 * (n + 1));
    hipLaunchKernelGGL(k_md_starts, dim3((uint32_t)ceil_div(n, 256)), dim3(256), 0, st, M->d_comp.as<uint64_t>(), n,
                       idx_bits, M->d_flag.as<uint32_t>());
    M->scan.run(M->d_flag.as<uint32_t>(), n, M->d_S.as<uint64_t>(), st);
    M->d_seg.ensure(8 * (n + 1));
    hipLaunchKernelGGL(k_md_segstart, dim3((uint32_t)ceil_div(n, 256)), dim3(256), 0, st, M->d_flag.as<uint32_t>(),
                       M->d_S.as<uint64_t>(), n, M->d_seg.as<uint64_t>());
    SKM_HIP(hipGetLastError());
    uint64_t G = 0;
    SKM_HIP(hipMemcpyAsync(&G, M->d_S.as<uint64_t>() + n, 8, hipMemcpyDeviceToHost, st));
    SKM_HIP(hipStreamSynchronize(st));
    return G;
}

// world > 1: hits -> owners -> groups -> bands; leaves this band's received groups in d_comp /
// d_S / d_seg and returns their composite count
uint64_t md_exchange(skm_matrix* M, uint64_t n_local, uint32_t idx_bits, hipStream_t st) {
    const int W = M->world;
    // 1. hits to the k-mer owners
    M->d_ocnt.ensure(8ull * (2 * W));
    unsigned long long* ocnt = M->d_ocnt.as<unsigned long long>();
    SKM_HIP(hipMemsetAsync(ocnt, 0, 8ull * W, st));
    const uint32_t ge = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(n_local, 256), 256ull * 32));
    hipLaunchKernelGGL(k_md_owner_count, dim3(ge), dim3(256), 0, st, M->d_rkey.as<unsigned long long>(),
                       M->d_nrec.as<unsigned long long>(), (uint32_t)W, ocnt);
    SKM_HIP(hipGetLastError());
    std::vector<uint64_t> sc(W), so(W, 0);
    SKM_HIP(hipMemcpyAsync(sc.data(), ocnt, 8ull * W, hipMemcpyDeviceToHost, st));
    SKM_HIP(hipStreamSynchronize(st));
    for (int q = 1; q < W; ++q) so[q] = so[q - 1] + sc[q - 1];
    M->d_skey.ensure(8 * std::max<uint64_t>(n_local, 1));
    M->d_sidx.ensure(4 * std::max<uint64_t>(n_local, 1));
    SKM_HIP(hipMemcpyAsync(ocnt + W, so.data(), 8ull * W, hipMemcpyHostToDevice, st));
    const uint32_t gs = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(n_local, OW_TILE), 4096));
    hipLaunchKernelGGL(k_md_owner_scatter, dim3(gs), dim3(256), 0, st, M->d_rkey.as<unsigned long long>(),
                       M->d_ridx.as<uint32_t>(), M->d_nrec.as<unsigned long long>(), (uint32_t)W, ocnt + W,
                       M->d_skey.as<unsigned long long>(), M->d_sidx.as<uint32_t>());
    SKM_HIP(hipGetLastError());
    SKM_HIP(hipStreamSynchronize(st));  // the local hits are copied out before d_rkey / d_ridx are reused
    const std::vector<uint64_t> rc = mx_exchange_u64(M, sc);
    std::vector<uint64_t> ro(W, 0);
    for (int q = 1; q < W; ++q) ro[q] = ro[q - 1] + rc[q - 1];
    const uint64_t n_own = ro[W - 1] + rc[W - 1];
    M->d_rkey.ensure(8 * std::max<uint64_t>(n_own, 1));  // the local hits were copied out already
    M->d_ridx.ensure(4 * std::max<uint64_t>(n_own, 1));
    auto scaled = [](const std::vector<uint64_t>& v, uint64_t k) {
        std::vector<uint64_t> r(v.size());
        for (size_t i = 0; i < v.size(); ++i) r[i] = v[i] * k;
        return r;
    };
    SKM_HIP(hipStreamSynchronize(st));
    mx_alltoallv(M, M->d_skey.as<uint8_t>(), scaled(so, 8), scaled(sc, 8), M->d_rkey.as<uint8_t>(), scaled(ro, 8),
                 scaled(rc, 8));
    mx_alltoallv(M, M->d_sidx.as<uint8_t>(), scaled(so, 4), scaled(sc, 4), M->d_ridx.as<uint8_t>(), scaled(ro, 4),
                 scaled(rc, 4));
    SKM_HIP(hipMemcpyAsync(M->d_nrec.p, &n_own, 8, hipMemcpyHostToDevice, st));
    SKM_HIP(hipStreamSynchronize(st));
    // 2. the owned k-mers' groups
    md_group(M, M->d_rkey.as<unsigned long long>(), M->d_ridx.as<uint32_t>(), M->d_nrec.as<unsigned long long>(), n_own,
             idx_bits, st);
    const uint64_t G = md_bounds(M, n_own, idx_bits, st);
    // 3. group suffixes to the row bands (band b = skm_matrix_tile_rows(n_idx, b, W))
    std::vector<uint32_t> band(W + 1);
    for (int q = 0; q < W; ++q) skm_matrix_tile_rows(M->nidx, q, W, &band[q], &band[q + 1]);
    M->d_band.ensure(4ull * (W + 1));
    SKM_HIP(hipMemcpyAsync(M->d_band.p, band.data(), 4ull * (W + 1), hipMemcpyHostToDevice, st));
    SKM_HIP(hipStreamSynchronize(st));
    std::vector<uint64_t> mine(W, G);
    const std::vector<uint64_t> gall = mx_exchange_u64(M, mine);
    uint64_t gbase = 0, gtot = 0;
    for (int q = 0; q < W; ++q) {
        if (q < M->rank) gbase += gall[q];
        gtot += gall[q];
    }
    SKM_CHECK(gtot < (1ull << (64 - idx_bits)), SKM_E_ARG, "matrix distance: too many k-mer groups for 64-bit composites");
    const uint64_t idx_mask = (1ull << idx_bits) - 1;
    std::vector<uint64_t> bc(W, 0), bo(W, 0);
    if (G) {
        // one band at a time over G-sized count / offset buffers (a dense W x G table grew with the
        // world size times the owned groups -- ADVICE r03): the bands' totals first, then the fill
        M->d_rtc.ensure(4ull * G);
        M->d_rto.ensure(8ull * (G + 1));
        const uint32_t gg = (uint32_t)std::min<uint64_t>(ceil_div(G, 256), 256ull * 32);
        auto count_band = [&](int q) {
            hipLaunchKernelGGL(k_md_route_count, dim3(gg), dim3(256), 0, st, M->d_comp.as<uint64_t>(),
                               M->d_seg.as<uint64_t>(), G, idx_mask, M->d_band.as<uint32_t>(), (uint32_t)q,
                               M->d_rtc.as<uint32_t>());
            SKM_HIP(hipGetLastError());
            M->scan.run(M->d_rtc.as<uint32_t>(), G, M->d_rto.as<uint64_t>(), st);
        };
        // every band's count, scan and total copy queued back to back (stream order keeps band q's
        // total copy ahead of band q+1's scan); one host synchronisation for all W totals
        for (int q = 0; q < W; ++q) {
            count_band(q);
            SKM_HIP(hipMemcpyAsync(&bc[q], M->d_rto.as<uint64_t>() + G, 8, hipMemcpyDeviceToHost, st));
        }
        SKM_HIP(hipStreamSynchronize(st));
        for (int q = 1; q < W; ++q) bo[q] = bo[q - 1] + bc[q - 1];
        const uint64_t tot = bo[W - 1] + bc[W - 1];
        M->d_send.ensure(8 * std::max<uint64_t>(tot, 1));
        for (int q = 0; q < W; ++q) {
            if (!bc[q]) continue;
            count_band(q);
            hipLaunchKernelGGL(k_md_route_fill, dim3(gg), dim3(256), 0, st, M->d_comp.as<uint64_t>(),
                               M->d_seg.as<uint64_t>(), G, idx_mask, idx_bits, M->d_rtc.as<uint32_t>(),
                               M->d_rto.as<uint64_t>(), gbase, M->d_send.as<uint64_t>() + bo[q]);
            SKM_HIP(hipGetLastError());
        }
        SKM_HIP(hipStreamSynchronize(st));
    } else {
        M->d_send.ensure(8);
    }
    const std::vector<uint64_t> rbc = mx_exchange_u64(M, bc);
    std::vector<uint64_t> rbo(W, 0);
    for (int q = 1; q < W; ++q) rbo[q] = rbo[q - 1] + rbc[q - 1];
    const uint64_t n_band = rbo[W - 1] + rbc[W - 1];
    M->d_comp2.ensure(8 * std::max<uint64_t>(n_band, 1));
    mx_alltoallv(M, M->d_send.as<uint8_t>(), scaled(bo, 8), scaled(bc, 8), M->d_comp2.as<uint8_t>(), scaled(rbo, 8),
                 scaled(rbc, 8));
    SKM_HIP(hipStreamSynchronize(st));
    std::swap(M->d_comp.p, M->d_comp2.p);
    std::swap(M->d_comp.bytes, M->d_comp2.bytes);
    M->n_routed = n_band;
    M->band_lo = band[M->rank];
    M->band_hi = band[M->rank + 1];
    M->n_groups = G;
    md_bounds(M, n_band, idx_bits, st);
    return n_band;
}

void matrix_run(skm_matrix* M, const skm_matrix_opts* o) {
    skm_db* db = M->db;
    SKM_HIP(hipSetDevice(db->device));
    hipStream_t st = M->stream;
    const uint32_t r0_in = (o->row_begin == 0 && o->row_end == 0) ? 0u : o->row_begin;
    const uint32_t r1_in = (o->row_begin == 0 && o->row_end == 0) ? M->nidx : std::min(o->row_end, M->nidx);
    SKM_HIP(hipEventRecord(M->ev[0], st));
    // 1. hits
    SKM_HIP(hipMemsetAsync(M->d_nrec.p, 0, 16, st));
    if (M->rp && db->m) {
        MdHitArgs A;
        A.res = M->d_res.as<uint8_t>();
        A.rp = M->rp;
        A.meta = M->d_meta.as<QMeta>();
        A.nseq = M->nseq;
        A.seq_idx = M->d_idx.as<uint32_t>();
        A.D = db->dev;
        A.exact = db->exact ? 1 : 0;
        A.hypo = o->hypo_index >= 0 ? (uint32_t)o->hypo_index : 0xFFFFFFFFu;
        A.rec_key = M->d_rkey.as<unsigned long long>();
        A.rec_idx = M->d_ridx.as<uint32_t>();
        A.nrec = M->d_nrec.as<unsigned long long>();
        const uint64_t nthreads = ceil_div(M->rp, LK_POS);
        const uint32_t grid = (uint32_t)std::min<uint64_t>(ceil_div(nthreads, MD_THREADS), 256ull * 16);
        hipLaunchKernelGGL(k_md_hits, dim3(grid), dim3(MD_THREADS), 0, st, A);
        SKM_HIP(hipGetLastError());
    }
    SKM_HIP(hipEventRecord(M->ev[1], st));
    uint64_t n = 0;
    SKM_HIP(hipMemcpyAsync(&n, M->d_nrec.p, 8, hipMemcpyDeviceToHost, st));
    SKM_HIP(hipStreamSynchronize(st));
    M->n_hits = n;
    M->n_local_hits = n;
    M->n_incs = 0;
    M->n_pairs = 0;
    M->n_groups = 0;
    // 2. group: slot table + radix sort of (slot, index) composites + group boundaries
    const uint32_t idx_bits = (uint32_t)std::max(1, ilog2_ceil(std::max<uint64_t>(M->nidx, 2)));
    const bool multi = M->world > 1;
    uint32_t r0 = r0_in, r1 = r1_in;
    if (multi) {  // owner-partitioned hits, band-routed groups: this rank's band of rows
        n = md_exchange(M, n, idx_bits, st);
        r0 = M->band_lo;
        r1 = M->band_hi;
    }
    if (n && !multi) {
        md_group(M, M->d_rkey.as<unsigned long long>(), M->d_ridx.as<uint32_t>(), M->d_nrec.as<unsigned long long>(), n,
                 idx_bits, st);
        M->n_groups = md_bounds(M, n, idx_bits, st);
    }
    SKM_HIP(hipEventRecord(M->ev[2], st));
    // 3. pair counts: row lists, one LDS histogram per row, compaction in row order
    float pairs_ms = 0, emit_ms = 0;
    uint64_t out_n = 0;
    if (n && r1 > r0) {
        const uint32_t rows = r1 - r0;
        M->d_rlen.ensure(4ull * rows);
        M->d_rub.ensure(4ull * rows);
        M->d_rcur.ensure(4ull * rows);
        M->d_roff.ensure(8ull * (rows + 1));
        M->d_ubo.ensure(8ull * (rows + 1));
        M->d_rnnz.ensure(4ull * rows);
        M->d_fo.ensure(8ull * (rows + 1));
        M->d_incs.ensure(16);
        SKM_HIP(hipMemsetAsync(M->d_rlen.p, 0, 4ull * rows, st));
        SKM_HIP(hipMemsetAsync(M->d_rub.p, 0, 4ull * rows, st));
        SKM_HIP(hipMemsetAsync(M->d_rcur.p, 0, 4ull * rows, st));
        SKM_HIP(hipMemsetAsync(M->d_incs.p, 0, 16, st));
        MdRowArgs R;
        R.comp = M->d_comp.as<uint64_t>();
        R.S = M->d_S.as<uint64_t>();
        R.segstart = M->d_seg.as<uint64_t>();
        R.n = n;
        R.idx_mask = (1ull << idx_bits) - 1;
        R.r0 = r0;
        R.rows = rows;
        R.nidx = M->nidx;
        R.rowlen = M->d_rlen.as<uint32_t>();
        R.rowub = M->d_rub.as<uint32_t>();
        R.cursor = M->d_rcur.as<uint32_t>();
        R.rowoff = M->d_roff.as<uint64_t>();
        R.ubo = M->d_ubo.as<uint64_t>();
        R.rownnz = M->d_rnnz.as<uint32_t>();
        R.rowctr = reinterpret_cast<unsigned int*>(M->d_incs.as<unsigned long long>() + 1);
        R.incs = M->d_incs.as<unsigned long long>();
        const uint32_t ge = (uint32_t)std::min<uint64_t>(ceil_div(n, 256), 256ull * 32);
        hipLaunchKernelGGL(k_md_rowstat, dim3(ge), dim3(256), 0, st, R);
        M->scan.run(R.rowlen, rows, M->d_roff.as<uint64_t>(), st);
        M->scan.run(R.rowub, rows, M->d_ubo.as<uint64_t>(), st);
        uint64_t tot[2] = {0, 0};
        SKM_HIP(hipMemcpyAsync(&tot[0], M->d_roff.as<uint64_t>() + rows, 8, hipMemcpyDeviceToHost, st));
        SKM_HIP(hipMemcpyAsync(&tot[1], M->d_ubo.as<uint64_t>() + rows, 8, hipMemcpyDeviceToHost, st));
        SKM_HIP(hipStreamSynchronize(st));
        M->d_rlist.ensure(4 * std::max<uint64_t>(tot[0], 1));
        M->d_scr.ensure(8 * std::max<uint64_t>(tot[1], 1));
        R.rowlist = M->d_rlist.as<uint32_t>();
        R.scratch = M->d_scr.as<uint32_t>();
        hipLaunchKernelGGL(k_md_rowfill, dim3(ge), dim3(256), 0, st, R);
        SKM_HIP(hipGetLastError());
        hipEvent_t e0, e1;
        SKM_HIP(hipEventCreate(&e0));
        SKM_HIP(hipEventCreate(&e1));
        SKM_HIP(hipEventRecord(e0, st));
        int dev = 0, ncu = 256;
        SKM_HIP(hipGetDevice(&dev));
        SKM_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
        hipLaunchKernelGGL(k_md_rows, dim3((uint32_t)std::max(1, ncu)), dim3(MR_THREADS), 0, st, R);
        SKM_HIP(hipGetLastError());
        SKM_HIP(hipEventRecord(e1, st));
        M->scan.run(R.rownnz, rows, M->d_fo.as<uint64_t>(), st);
        SKM_HIP(hipMemcpyAsync(&out_n, M->d_fo.as<uint64_t>() + rows, 8, hipMemcpyDeviceToHost, st));
        SKM_HIP(hipStreamSynchronize(st));
        M->d_out.ensure(12 * std::max<uint64_t>(out_n, 1));
        hipLaunchKernelGGL(k_md_gather, dim3(std::min<uint32_t>(rows, 256u * 16u)), dim3(256), 0, st,
                           M->d_scr.as<uint32_t>(), M->d_ubo.as<uint64_t>(), M->d_fo.as<uint64_t>(), r0, rows,
                           M->d_out.as<uint32_t>());
        SKM_HIP(hipGetLastError());
        SKM_HIP(hipEventRecord(M->ev[3], st));
        SKM_HIP(hipEventSynchronize(M->ev[3]));
        SKM_HIP(hipEventElapsedTime(&pairs_ms, e0, e1));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        unsigned long long incs = 0;
        SKM_HIP(hipMemcpy(&incs, M->d_incs.p, 8, hipMemcpyDeviceToHost));
        M->n_incs = incs;
    }
    SKM_HIP(hipEventRecord(M->ev[3], st));
    SKM_HIP(hipEventSynchronize(M->ev[3]));
    M->n_pairs = out_n;
    SKM_HIP(hipEventElapsedTime(&M->last_ms[0], M->ev[0], M->ev[1]));  // hits
    SKM_HIP(hipEventElapsedTime(&M->last_ms[1], M->ev[1], M->ev[2]));  // group (slot + sort + bounds)
    M->last_ms[2] = pairs_ms;                                          // pair increments
    SKM_HIP(hipEventElapsedTime(&emit_ms, M->ev[2], M->ev[3]));
    M->last_ms[3] = emit_ms - pairs_ms;                                // row lists + compaction
    SKM_HIP(hipEventElapsedTime(&M->last_ms[4], M->ev[0], M->ev[3]));  // total
    M->ran = true;
}

}  // namespace

extern "C" {

int skm_matrix_tile_rows(uint32_t n_idx, int rank, int world, uint32_t* row_begin, uint32_t* row_end) {
    SKM_API_BEGIN
    SKM_CHECK(row_begin && row_end && world >= 1 && rank >= 0 && rank < world, SKM_E_ARG, "invalid tile request");
    const uint64_t N = n_idx, total = rowbase(N, N);
    auto bound = [&](int r) -> uint32_t {  // first row whose prefix area reaches r/world of the total
        if (r <= 0) return 0;
        if (r >= world) return n_idx;
        const long double target = (long double)total * r / world;
        uint32_t lo = 0, hi = n_idx;
        while (lo < hi) {
            const uint32_t mid = lo + (hi - lo) / 2;
            if ((long double)rowbase(mid, N) < target)
                lo = mid + 1;
            else
                hi = mid;
        }
        return lo;
    };
    *row_begin = bound(rank);
    *row_end = bound(rank + 1);
    SKM_API_END
}

int skm_matrix_create(skm_matrix** out, skm_db* db, const uint8_t* residues, const uint64_t* seq_off,
                      const uint32_t* seq_len, const uint32_t* seq_idx, size_t n_seqs, uint32_t n_idx) {
    SKM_API_BEGIN
    SKM_CHECK(out && db, SKM_E_ARG, "null argument");
    SKM_CHECK(n_seqs == 0 || (residues && seq_off && seq_len && seq_idx), SKM_E_ARG, "null array");
    SKM_CHECK(n_seqs < 0xFFFFFFFFull, SKM_E_ARG, "too many sequences in one batch");
    for (size_t s = 0; s < n_seqs; ++s) SKM_CHECK(seq_idx[s] < n_idx, SKM_E_ARG, "seq_idx out of range");
    SKM_HIP(hipSetDevice(db->device));
    auto* M = new skm_matrix();
    M->db = db;
    try {
        SKM_HIP(hipStreamCreateWithFlags(&M->stream, hipStreamNonBlocking));
        for (auto& e : M->ev) SKM_HIP(hipEventCreate(&e));
        std::vector<uint8_t> res;
        std::vector<QMeta> meta(n_seqs);
        uint64_t total = 0;
        for (size_t s = 0; s < n_seqs; ++s) total += (uint64_t)seq_len[s] + 1;
        res.reserve(total);
        for (size_t s = 0; s < n_seqs; ++s) {
            meta[s].pstart = res.size();
            meta[s].len = seq_len[s];
            meta[s].pad = 0;
            res.insert(res.end(), residues + seq_off[s], residues + seq_off[s] + seq_len[s]);
            res.push_back(0);
            M->n_windows += seq_len[s] >= 8 ? seq_len[s] - 7 : 0;
        }
        M->nseq = (uint32_t)n_seqs;
        M->nidx = n_idx;
        M->rp = res.size();
        const uint64_t rp_pad = ceil_div(M->rp + 1, LK_POS) * LK_POS;
        M->d_res.ensure(rp_pad + 64);
        SKM_HIP(hipMemsetAsync(M->d_res.p, 0, rp_pad + 64, M->stream));
        if (M->rp) SKM_HIP(hipMemcpyAsync(M->d_res.p, res.data(), M->rp, hipMemcpyHostToDevice, M->stream));
        M->d_meta.ensure(sizeof(QMeta) * std::max<size_t>(n_seqs, 1));
        if (n_seqs) SKM_HIP(hipMemcpyAsync(M->d_meta.p, meta.data(), sizeof(QMeta) * n_seqs, hipMemcpyHostToDevice, M->stream));
        M->d_idx.ensure(4 * std::max<size_t>(n_seqs, 1));
        if (n_seqs) SKM_HIP(hipMemcpyAsync(M->d_idx.p, seq_idx, 4 * n_seqs, hipMemcpyHostToDevice, M->stream));
        const uint64_t cap = std::max<uint64_t>(M->n_windows, 1);  // one record per window at most
        M->d_rkey.ensure(8 * cap);
        M->d_ridx.ensure(4 * cap);
        M->d_nrec.ensure(16);
        SKM_HIP(hipStreamSynchronize(M->stream));
    } catch (...) {
        skm_matrix_destroy(M);
        throw;
    }
    *out = M;
    SKM_API_END
}

int skm_matrix_set_transport(skm_matrix* m, int rank, int world, const skm_transport* tp) {
    SKM_API_BEGIN
    SKM_CHECK(m && tp && tp->alltoallv, SKM_E_ARG, "incomplete transport");
    SKM_CHECK(world >= 1 && world <= 64 && rank >= 0 && rank < world, SKM_E_ARG, "rank / world out of range");
    m->rank = rank;
    m->world = world;
    m->tp = *tp;
    SKM_API_END
}

int skm_matrix_set_comm(skm_matrix* m, int rank, int world, const uint8_t id[128]) {
    SKM_API_BEGIN
    SKM_CHECK(m && id, SKM_E_ARG, "null argument");
    SKM_CHECK(world >= 1 && world <= 64 && rank >= 0 && rank < world, SKM_E_ARG, "rank / world out of range");
#if defined(SKM_WITH_RCCL)
    SKM_CHECK(m->comm == nullptr, SKM_E_STATE, "communicator already set");
    SKM_HIP(hipSetDevice(m->db->device));
    m->rank = rank;
    m->world = world;
    if (world > 1) {
        ncclUniqueId u;
        std::memcpy(&u, id, 128);
        MX_NCCL(ncclCommInitRank(&m->comm, world, u, rank));
    }
#else
    throw Error(SKM_E_COMM, "libskm was built without RCCL");
#endif
    SKM_API_END
}

int skm_matrix_run(skm_matrix* m, const skm_matrix_opts* opts) {
    SKM_API_BEGIN
    SKM_CHECK(m && opts, SKM_E_ARG, "null argument");
    SKM_CHECK(opts->row_begin <= opts->row_end, SKM_E_ARG, "row_begin > row_end");
    matrix_run(m, opts);
    SKM_API_END
}

int skm_matrix_last_timings(skm_matrix* m, float* ms, int cap) {
    if (!m || !ms) return SKM_E_ARG;
    const int n = std::min(cap, 5);
    for (int i = 0; i < n; ++i) ms[i] = m->last_ms[i];
    return n;
}

int skm_matrix_counters(skm_matrix* m, uint64_t* out, int cap) {
    if (!m || !out) return SKM_E_ARG;
    const uint64_t v[7] = {m->n_windows, m->n_hits, m->n_incs, m->n_pairs, m->n_groups, m->n_local_hits, m->n_routed};
    const int n = std::min(cap, 7);
    for (int i = 0; i < n; ++i) out[i] = v[i];
    return n;
}

int skm_matrix_pairs(skm_matrix* m, skm_pairs* out) {
    SKM_API_BEGIN
    SKM_CHECK(m && out, SKM_E_ARG, "null argument");
    SKM_CHECK(m->ran, SKM_E_STATE, "skm_matrix_run has not been called");
    SKM_HIP(hipSetDevice(m->db->device));
    std::memset(out, 0, sizeof(*out));
    out->n = m->n_pairs;
    out->n_hits = m->n_hits;
    out->pairs = (uint32_t*)std::malloc(12 * std::max<uint64_t>(m->n_pairs, 1));
    SKM_CHECK(out->pairs, SKM_E_OOM, "host allocation failed");
    if (m->n_pairs) SKM_HIP(hipMemcpy(out->pairs, m->d_out.p, 12 * m->n_pairs, hipMemcpyDeviceToHost));
    SKM_API_END
}

void skm_pairs_free(skm_pairs* p) {
    if (!p) return;
    std::free(p->pairs);
    std::memset(p, 0, sizeof(*p));
}

void skm_matrix_destroy(skm_matrix* m) {
    if (!m) return;
    (void)hipSetDevice(m->db->device);
    if (m->stream) (void)hipStreamSynchronize(m->stream);
#if defined(SKM_WITH_RCCL)
    if (m->comm) (void)ncclCommDestroy(m->comm);
#endif
    for (auto& e : m->ev)
        if (e) (void)hipEventDestroy(e);
    if (m->stream) (void)hipStreamDestroy(m->stream);
    delete m;
}

}  // extern "C"
