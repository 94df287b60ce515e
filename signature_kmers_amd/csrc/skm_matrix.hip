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
// Device pipeline (one GPU holds the row tile [r0, r1) of the upper-triangle count matrix):
//   k_md_hits      one thread per 16 window positions of the packed queries: window validity,
//                  DB lookup, record, filters; surviving (kmer, index) records compacted with one
//                  atomic per wave
//   k_md_slot      kmer -> slot of an open-addressing table (atomicCAS); composite
//                  slot << idx_bits | index
//   k_rs_hist / k_rs_scatter   LSD radix sort of the composites, 8-bit digits (stable: per-round
//                  wave match by ballots + per-wave digit counts in LDS)
//   k_md_starts / k_md_segstart   k-mer group boundaries (composites with equal slot)
//   k_md_pairs     one wave per 64 consecutive composites; a lane walks its own short pair row,
//                  rows of > 16 partners are walked by the whole wave; one atomic add per pair
//                  increment into the dense tile (u32, row-major triangle)
//   k_md_rowcount / k_md_emit   stable compaction of the nonzero counts into sorted
//                  (id1, id2, count) triples; emitted cells are reset to 0 for the next run
// The hit records are identical on every GPU (each recomputes them: ~3 % of the time), so the
// row tiles need no collective; the host concatenates the tiles in row order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "skm_common.h"
#include "skm_lookup.h"
#include "skm_util.h"

namespace skm {

constexpr int MD_THREADS = 256;
constexpr uint32_t MD_LONG_ROW = 16;   // rows with more partners are walked by the whole wave

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
    return exact ? exact_lookup(D, lo, hi) : bdz_lookup(D, lo, hi);
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

struct MdPairArgs {
    const uint64_t* comp;      // sorted composites
    const uint64_t* S;         // exclusive scan of group-start flags [n+1]
    const uint64_t* segstart;  // [nseg+1]
    uint64_t n;
    uint64_t idx_mask;
    uint32_t r0, r1;           // row tile
    uint64_t nidx;             // matrix order
    uint64_t base0;            // rowbase(r0)
    uint32_t* tile;            // counts, row-major upper triangle of rows [r0, r1)
    unsigned long long* incs;  // pair increments (diagnostics / roofline)
};

__host__ __device__ __forceinline__ uint64_t rowbase(uint64_t i, uint64_t n) { return i * (2 * n - i - 1) / 2; }

__global__ __launch_bounds__(MD_THREADS) void k_md_pairs(MdPairArgs P) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nw = (uint64_t)gridDim.x * (MD_THREADS / 64);
    uint64_t incs = 0;
    for (uint64_t c0 = ((uint64_t)blockIdx.x * (MD_THREADS / 64) + (threadIdx.x >> 6)) * 64; c0 < P.n; c0 += nw * 64) {
        const uint64_t e = c0 + lane;
        uint64_t ge = 0, roff = 0;
        bool act = false;
        if (e < P.n) {
            const uint64_t c = P.comp[e];
            const uint64_t id1 = c & P.idx_mask;
            if ((e == 0 || P.comp[e - 1] != c) && id1 >= P.r0 && id1 < P.r1) {
                ge = P.segstart[P.S[e + 1]];  // end of e's group (group id S[e+1] - 1)
                act = ge > e + 1;
                roff = rowbase(id1, P.nidx) - P.base0 - id1 - 1;
            }
        }
        const bool is_long = act && ge - e - 1 > MD_LONG_ROW;
        if (act && !is_long) {
            for (uint64_t q = e + 1; q < ge; ++q) {
                const uint64_t cq = P.comp[q];
                if (cq == P.comp[q - 1]) continue;  // duplicate (kmer, index)
                atomicAdd(&P.tile[roff + (cq & P.idx_mask)], 1u);
                ++incs;
            }
        }
        uint64_t lm = __ballot(is_long);
        while (lm) {
            const int L = __ffsll((unsigned long long)lm) - 1;
            lm &= lm - 1;
            const uint64_t le = __shfl(e, L, 64), lge = __shfl(ge, L, 64), lro = __shfl(roff, L, 64);
            for (uint64_t q = le + 1 + lane; q < lge; q += 64) {
                const uint64_t cq = P.comp[q];
                if (cq == P.comp[q - 1]) continue;
                atomicAdd(&P.tile[lro + (cq & P.idx_mask)], 1u);
                ++incs;
            }
        }
    }
    // one atomic per wave
    uint64_t x = incs;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    if (lane == 0 && x) atomicAdd(P.incs, (unsigned long long)x);
}

// nonzero cells per row of the tile
__global__ __launch_bounds__(MD_THREADS) void k_md_rowcount(const uint32_t* __restrict__ tile, uint32_t r0, uint32_t r1,
                                                            uint64_t nidx, uint64_t base0, uint32_t* __restrict__ cnt) {
    __shared__ uint32_t s_w[MD_THREADS / 64];
    for (uint32_t r = r0 + blockIdx.x; r < r1; r += gridDim.x) {
        const uint64_t a = rowbase(r, nidx) - base0, len = nidx - r - 1;
        uint32_t c = 0;
        const uint32_t* row = tile + a;
        for (uint64_t j = threadIdx.x; j < len; j += MD_THREADS) c += row[j] != 0;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
        if ((threadIdx.x & 63u) == 0) s_w[threadIdx.x >> 6] = c;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t t = 0;
            for (int w = 0; w < MD_THREADS / 64; ++w) t += s_w[w];
            cnt[r - r0] = t;
        }
        __syncthreads();
    }
}

// stable compaction of each row's nonzero cells into (id1, id2, count); cells reset to 0
__global__ __launch_bounds__(MD_THREADS) void k_md_emit(uint32_t* __restrict__ tile, uint32_t r0, uint32_t r1, uint64_t nidx,
                                                        uint64_t base0, const uint64_t* __restrict__ roff,
                                                        uint32_t* __restrict__ out) {
    __shared__ uint32_t s_w[MD_THREADS / 64 + 1];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (uint32_t r = r0 + blockIdx.x; r < r1; r += gridDim.x) {
        const uint64_t a = rowbase(r, nidx) - base0, len = nidx - r - 1;
        uint32_t* row = tile + a;
        uint64_t o = roff[r - r0];
        for (uint64_t j0 = 0; j0 < len; j0 += MD_THREADS) {
            const uint64_t j = j0 + threadIdx.x;
            const uint32_t v = j < len ? row[j] : 0u;
            const uint64_t m = __ballot(v != 0);
            if (lane == 0) s_w[wave] = (uint32_t)__popcll(m);
            __syncthreads();
            uint32_t before = 0, tot = 0;
            for (uint32_t w = 0; w < MD_THREADS / 64; ++w) {
                before += w < wave ? s_w[w] : 0u;
                tot += s_w[w];
            }
            if (v) {
                const uint64_t p = o + before + (uint32_t)__popcll(m & lt);
                out[3 * p] = r;
                out[3 * p + 1] = (uint32_t)(r + 1 + j);
                out[3 * p + 2] = v;
                row[j] = 0;
            }
            o += tot;
            __syncthreads();
        }
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
        d_seg, d_tile, d_rcnt, d_roff, d_out, d_out2, d_incs;
    Scanner scan;
    uint64_t n_hits = 0, n_incs = 0, n_pairs = 0, n_groups = 0;
    bool ran = false;
};

namespace {

void matrix_run(skm_matrix* M, const skm_matrix_opts* o) {
    skm_db* db = M->db;
    SKM_HIP(hipSetDevice(db->device));
    hipStream_t st = M->stream;
    const uint32_t r0 = (o->row_begin == 0 && o->row_end == 0) ? 0u : o->row_begin;
    const uint32_t r1 = (o->row_begin == 0 && o->row_end == 0) ? M->nidx : std::min(o->row_end, M->nidx);
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
    M->n_incs = 0;
    M->n_pairs = 0;
    M->n_groups = 0;
    // 2. group: slot table + radix sort of (slot, index) composites + group boundaries
    const uint32_t idx_bits = (uint32_t)std::max(1, ilog2_ceil(std::max<uint64_t>(M->nidx, 2)));
    const int lg = std::max(4, ilog2_ceil(2 * std::max<uint64_t>(n, 1)));
    const uint32_t key_bits = (uint32_t)lg + idx_bits;
    SKM_CHECK(key_bits <= 64, SKM_E_ARG, "matrix distance: too many hits / sequences for 64-bit composites");
    if (n) {
        const uint64_t T = 1ull << lg;
        M->d_tab.ensure(8 * T);
        SKM_HIP(hipMemsetAsync(M->d_tab.p, 0, 8 * T, st));
        M->d_comp.ensure(8 * n);
        M->d_comp2.ensure(8 * n);
        const uint32_t g = (uint32_t)std::min<uint64_t>(ceil_div(n, 256), 256ull * 32);
        hipLaunchKernelGGL(k_md_slot, dim3(g), dim3(256), 0, st, M->d_rkey.as<unsigned long long>(),
                           M->d_ridx.as<uint32_t>(), M->d_nrec.as<unsigned long long>(),
                           M->d_tab.as<unsigned long long>(), T - 1, 64u - (uint32_t)lg, idx_bits, M->d_comp.as<uint64_t>());
        SKM_HIP(hipGetLastError());
        const uint32_t nb = (uint32_t)ceil_div(n, RS_TILE);
        M->d_hist.ensure(4ull * 256 * nb);
        M->d_hoff.ensure(8ull * (256 * (uint64_t)nb + 1));
        uint64_t* a = M->d_comp.as<uint64_t>();
        uint64_t* b = M->d_comp2.as<uint64_t>();
        for (uint32_t sh = 0; sh < key_bits; sh += 8) {
            hipLaunchKernelGGL(k_rs_hist, dim3(nb), dim3(RS_THREADS), 0, st, a, n, (int)sh, nb, M->d_hist.as<uint32_t>());
            M->scan.run(M->d_hist.as<uint32_t>(), 256ull * nb, M->d_hoff.as<uint64_t>(), st);
            hipLaunchKernelGGL(k_rs_scatter, dim3(nb), dim3(RS_THREADS), 0, st, a, n, (int)sh, nb,
                               M->d_hoff.as<uint64_t>(), b);
            SKM_HIP(hipGetLastError());
            std::swap(a, b);
        }
        if (a != M->d_comp.as<uint64_t>()) {
            std::swap(M->d_comp.p, M->d_comp2.p);
            std::swap(M->d_comp.bytes, M->d_comp2.bytes);
        }
        M->d_flag.ensure(4 * n);
        M->d_S.ensure(8 * (n + 1));
        hipLaunchKernelGGL(k_md_starts, dim3((uint32_t)ceil_div(n, 256)), dim3(256), 0, st, M->d_comp.as<uint64_t>(), n,
                           idx_bits, M->d_flag.as<uint32_t>());
        M->scan.run(M->d_flag.as<uint32_t>(), n, M->d_S.as<uint64_t>(), st);
        M->d_seg.ensure(8 * (n + 1));
        hipLaunchKernelGGL(k_md_segstart, dim3((uint32_t)ceil_div(n, 256)), dim3(256), 0, st, M->d_flag.as<uint32_t>(),
                           M->d_S.as<uint64_t>(), n, M->d_seg.as<uint64_t>());
        SKM_HIP(hipGetLastError());
        SKM_HIP(hipMemcpyAsync(&M->n_groups, M->d_S.as<uint64_t>() + n, 8, hipMemcpyDeviceToHost, st));
    }
    SKM_HIP(hipEventRecord(M->ev[2], st));
    // 3. pair counts, tile by tile (rows [r0, r1) cut into sub-tiles that fit the budget)
    float pairs_ms = 0, emit_ms = 0;
    uint64_t out_n = 0;
    if (n && r1 > r0) {
        const uint64_t N = M->nidx;
        size_t freeb = 0, totb = 0;
        SKM_HIP(hipMemGetInfo(&freeb, &totb));
        uint64_t budget = o->max_tile_bytes ? o->max_tile_bytes : (uint64_t)(0.6 * (double)(freeb + M->d_tile.bytes));
        budget = std::max<uint64_t>(budget, 4 * N + 64);
        std::vector<std::pair<uint32_t, uint32_t>> subs;
        for (uint32_t a = r0; a < r1;) {
            uint32_t b = a + 1;
            // grow b while the sub-tile fits (rows are contiguous in the triangle)
            uint32_t lo = a + 1, hi = r1;
            while (lo < hi) {
                const uint32_t mid = lo + (hi - lo + 1) / 2;
                if (4 * (rowbase(mid, N) - rowbase(a, N)) <= budget)
                    lo = mid;
                else
                    hi = mid - 1;
            }
            b = lo;
            subs.push_back({a, b});
            a = b;
        }
        uint64_t max_area = 0;
        for (auto& s : subs) max_area = std::max(max_area, rowbase(s.second, N) - rowbase(s.first, N));
        const bool fresh = M->d_tile.bytes < 4 * max_area + 16 || !M->d_tile.p;
        M->d_tile.ensure(4 * max_area + 16);
        if (fresh) SKM_HIP(hipMemsetAsync(M->d_tile.p, 0, M->d_tile.bytes, st));
        M->d_incs.ensure(8);
        SKM_HIP(hipMemsetAsync(M->d_incs.p, 0, 8, st));
        uint32_t max_rows = 0;
        for (auto& s : subs) max_rows = std::max(max_rows, s.second - s.first);
        M->d_rcnt.ensure(4ull * max_rows);
        M->d_roff.ensure(8ull * (max_rows + 1));
        hipEvent_t e0, e1, e2;
        SKM_HIP(hipEventCreate(&e0));
        SKM_HIP(hipEventCreate(&e1));
        SKM_HIP(hipEventCreate(&e2));
        for (auto& s : subs) {
            MdPairArgs P;
            P.comp = M->d_comp.as<uint64_t>();
            P.S = M->d_S.as<uint64_t>();
            P.segstart = M->d_seg.as<uint64_t>();
            P.n = n;
            P.idx_mask = (1ull << idx_bits) - 1;
            P.r0 = s.first;
            P.r1 = s.second;
            P.nidx = N;
            P.base0 = rowbase(s.first, N);
            P.tile = M->d_tile.as<uint32_t>();
            P.incs = M->d_incs.as<unsigned long long>();
            SKM_HIP(hipEventRecord(e0, st));
            const uint32_t gp = (uint32_t)std::min<uint64_t>(ceil_div(ceil_div(n, 64), MD_THREADS / 64), 256ull * 64);
            hipLaunchKernelGGL(k_md_pairs, dim3(gp), dim3(MD_THREADS), 0, st, P);
            SKM_HIP(hipGetLastError());
            SKM_HIP(hipEventRecord(e1, st));
            const uint32_t rows = s.second - s.first;
            const uint32_t gr = std::min<uint32_t>(rows, 256u * 16u);
            hipLaunchKernelGGL(k_md_rowcount, dim3(gr), dim3(MD_THREADS), 0, st, M->d_tile.as<uint32_t>(), s.first,
                               s.second, N, P.base0, M->d_rcnt.as<uint32_t>());
            M->scan.run(M->d_rcnt.as<uint32_t>(), rows, M->d_roff.as<uint64_t>(), st);
            uint64_t cnt = 0;
            SKM_HIP(hipMemcpyAsync(&cnt, M->d_roff.as<uint64_t>() + rows, 8, hipMemcpyDeviceToHost, st));
            SKM_HIP(hipStreamSynchronize(st));
            if (12 * (out_n + cnt) + 16 > M->d_out.bytes) {  // grow, keeping the earlier sub-tiles
                M->d_out2.ensure(12 * (out_n + cnt) + (12 * (out_n + cnt)) / 4 + 16);
                if (out_n) SKM_HIP(hipMemcpyAsync(M->d_out2.p, M->d_out.p, 12 * out_n, hipMemcpyDeviceToDevice, st));
                std::swap(M->d_out.p, M->d_out2.p);
                std::swap(M->d_out.bytes, M->d_out2.bytes);
            }
            hipLaunchKernelGGL(k_md_emit, dim3(gr), dim3(MD_THREADS), 0, st, M->d_tile.as<uint32_t>(), s.first, s.second,
                               N, P.base0, M->d_roff.as<uint64_t>(), M->d_out.as<uint32_t>() + 3 * out_n);
            SKM_HIP(hipGetLastError());
            SKM_HIP(hipEventRecord(e2, st));
            SKM_HIP(hipEventSynchronize(e2));
            float t1 = 0, t2 = 0;
            SKM_HIP(hipEventElapsedTime(&t1, e0, e1));
            SKM_HIP(hipEventElapsedTime(&t2, e1, e2));
            pairs_ms += t1;
            emit_ms += t2;
            out_n += cnt;
        }
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        (void)hipEventDestroy(e2);
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
    M->last_ms[3] = emit_ms;                                           // row counts + compaction
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
    const uint64_t v[5] = {m->n_windows, m->n_hits, m->n_incs, m->n_pairs, m->n_groups};
    const int n = std::min(cap, 5);
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
    for (auto& e : m->ev)
        if (e) (void)hipEventDestroy(e);
    if (m->stream) (void)hipStreamDestroy(m->stream);
    delete m;
}

}  // extern "C"
