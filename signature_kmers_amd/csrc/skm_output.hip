// skm_output.hip -- the kept-set hand-off: a build's kept k-mers from HBM to the caller's host
// arrays, in ascending key order (skm_build_finish / skm_build_finish_slice).
//
// The reference writes final.kmers and the .dat from one in-memory KeptKmers map in hash order
// (kmers-build-signatures.cc:198-264); this port hands the set back sorted (deterministic output).
// Round 4 downloaded the whole arena, then sorted an index permutation on ONE host thread
// (~30 s for C2's 168.7 M kept k-mers; C3's 2.89 G did not fit host memory twice over).  Now:
//
//   k_out_hist    one read of the arena's keys: a 16384-bin histogram of the sort code's top bits
//   host plan     consecutive bins into chunks of <= ~2^27 k-mers (any size works: a chunk's
//                 device scratch is sized to the largest)
//   per chunk     k_out_select (the chunk's (sort code, arena index) pairs, wave-aggregated
//                 compaction) -> rocPRIM radix sort of the pairs (43 bits) -> k_out_gather (the
//                 keys and 10-byte records in key order, double-buffered) -> D2H in 64 MB pieces
//                 through two pinned buffers, each piece copied out to the caller's arrays by the
//                 host pool while the next piece is in flight; chunk c+1 sorts while chunk c drains
//
// Sort code: the little-endian key's bytes are compared from byte 7 down (u64 order), and the 40
// residue codes of ok_prot_ (skm_common.h residue_code: upper case 0..19, lower case 20..39, each
// ascending in byte value) are monotone in the byte, so sum_j code(byte j) * 40^j (< 2^43) orders
// kept keys exactly as their u64 values do.
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <vector>

#include "skm_common.h"
#include "skm_output.h"
#include "skm_util.h"

namespace skm {

namespace {

constexpr int OUT_BIN_BITS = 14;                        // histogram bins: top bits of the 43-bit code
constexpr int OUT_BIN_SHIFT = KEY_BITS - OUT_BIN_BITS;  // 29
constexpr uint32_t OUT_BINS = 1u << OUT_BIN_BITS;
constexpr int OUT_THREADS = 256;

__device__ __forceinline__ uint64_t sort_code(uint64_t raw) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 7; j >= 0; --j) c = c * 40u + residue_code((uint32_t)(raw >> (8 * j)) & 0xFFu);
    return c;
}

__global__ __launch_bounds__(OUT_THREADS) void k_out_hist(const uint64_t* __restrict__ keys, uint64_t n,
                                                          uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[OUT_BINS];
    for (uint32_t i = threadIdx.x; i < OUT_BINS; i += OUT_THREADS) h[i] = 0;
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * OUT_THREADS + threadIdx.x; i < n; i += (uint64_t)gridDim.x * OUT_THREADS)
        atomicAdd(&h[sort_code(keys[i]) >> OUT_BIN_SHIFT], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < OUT_BINS; i += OUT_THREADS)
        if (h[i]) atomicAdd(&hist[i], h[i]);
}

// the (sort code, arena index) pairs of the keys whose bin lies in [lo, hi).  Tiles of 16
// elements per thread (coalesced, strided by the block); the block's selected count is scanned
// over its waves and reserved with ONE atomic per tile -- a chunk selects ~1/22 of the arena's
// keys, spread over it in hash order, so a per-wave reservation put ~40 M atomics on one address
// per chunk at C3 (0.5 s per chunk)
// per chunk -- the arena index is a u32 below 2^32 kept k-mers, a u64 from there (a multi-GPU
// build hands rank 0 the union of every rank's kept set)
constexpr int SEL_ITEMS = 16;
template <class IdxT>
__global__ __launch_bounds__(OUT_THREADS) void k_out_select(const uint64_t* __restrict__ keys, uint64_t n, uint32_t lo,
                                                            uint32_t hi, unsigned long long* __restrict__ cur,
                                                            uint64_t* __restrict__ code, IdxT* __restrict__ idx) {
    constexpr int NW = OUT_THREADS / 64;
    __shared__ uint32_t wsum[NW];
    __shared__ unsigned long long base_s;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint64_t TILE = (uint64_t)OUT_THREADS * SEL_ITEMS;
    for (uint64_t t0 = (uint64_t)blockIdx.x * TILE; t0 < n; t0 += (uint64_t)gridDim.x * TILE) {
        uint64_t c[SEL_ITEMS];
        uint32_t mask = 0;
#pragma unroll
        for (int j = 0; j < SEL_ITEMS; ++j) {
            const uint64_t i = t0 + (uint64_t)j * OUT_THREADS + tid;
            c[j] = i < n ? sort_code(keys[i]) : 0;
            const uint32_t bin = (uint32_t)(c[j] >> OUT_BIN_SHIFT);
            mask |= (i < n && bin >= lo && bin < hi) ? (1u << j) : 0u;
        }
        // exclusive prefix of the per-thread counts within the wave (shuffle scan), then over waves
        const uint32_t cnt = (uint32_t)__popc(mask);
        uint32_t incl = cnt;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t v = __shfl_up(incl, d);
            if (lane >= (uint32_t)d) incl += v;
        }
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        if (tid == 0) {
            uint32_t tot = 0;
            for (int w = 0; w < NW; ++w) tot += wsum[w];
            base_s = tot ? atomicAdd(cur, (unsigned long long)tot) : 0ull;
        }
        __syncthreads();
        uint64_t o = base_s + (incl - cnt);
        for (uint32_t w = 0; w < wave; ++w) o += wsum[w];
#pragma unroll
        for (int j = 0; j < SEL_ITEMS; ++j)
            if ((mask >> j) & 1u) {
                code[o] = c[j];
                idx[o] = (IdxT)(t0 + (uint64_t)j * OUT_THREADS + tid);
                ++o;
            }
        __syncthreads();  // wsum / base_s are rewritten by the next tile
    }
}

template <class IdxT>
__global__ __launch_bounds__(OUT_THREADS) void k_out_gather(const uint64_t* __restrict__ keys,
                                                            const skm_stored_kmer_data* __restrict__ data,
                                                            const IdxT* __restrict__ idx, uint64_t m,
                                                            uint64_t* __restrict__ okeys,
                                                            skm_stored_kmer_data* __restrict__ odata) {
    for (uint64_t j = (uint64_t)blockIdx.x * OUT_THREADS + threadIdx.x; j < m; j += (uint64_t)gridDim.x * OUT_THREADS) {
        const IdxT i = idx[j];
        okeys[j] = keys[i];
        odata[j] = data[i];
    }
}

struct Chunk {
    uint32_t lo, hi;     // bins [lo, hi)
    uint64_t n, at;      // k-mers, output offset
};

// host arrays for n records; large ones on 2 MB pages (fewer first-touch faults in the copy-out)
void* host_alloc(size_t bytes) {
    const size_t a = 1ull << 21;
    if (bytes < (64ull << 20)) return std::malloc(std::max<size_t>(bytes, 16));
    void* p = std::aligned_alloc(a, (bytes + a - 1) / a * a);
    if (p) (void)madvise(p, (bytes + a - 1) / a * a, MADV_HUGEPAGE);
    return p;
}

}  // namespace

namespace {

template <class IdxT>
void kept_handoff_t(const uint64_t* dkeys, const skm_stored_kmer_data* ddata, uint64_t n, hipStream_t st,
                    HostPool* pool, uint64_t** keys_out, skm_stored_kmer_data** data_out, HandoffStats* stats,
                    uint64_t max_chunk) {
    auto now = [] { return std::chrono::steady_clock::now(); };
    const auto t0 = now();
    uint64_t* hk = (uint64_t*)host_alloc(8 * n);
    skm_stored_kmer_data* hd = (skm_stored_kmer_data*)host_alloc(sizeof(skm_stored_kmer_data) * n);
    if (!hk || !hd) {
        std::free(hk);
        std::free(hd);
        throw Error(SKM_E_OOM, "host allocation failed");
    }
    *keys_out = hk;
    *data_out = hd;
    HandoffStats S;
    S.n = n;
    if (n == 0) {
        if (stats) *stats = S;
        return;
    }
    // 1. histogram and the chunk plan
    DevBuf d_hist, d_cur;
    d_hist.ensure(4ull * OUT_BINS);
    d_cur.ensure(8);
    SKM_HIP(hipMemsetAsync(d_hist.p, 0, 4ull * OUT_BINS, st));
    const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(n, OUT_THREADS), 2048));
    hipLaunchKernelGGL(k_out_hist, dim3(grid), dim3(OUT_THREADS), 0, st, dkeys, n, d_hist.as<uint32_t>());
    SKM_HIP(hipGetLastError());
    std::vector<uint32_t> hist(OUT_BINS);
    SKM_HIP(hipMemcpyAsync(hist.data(), d_hist.p, 4ull * OUT_BINS, hipMemcpyDeviceToHost, st));
    SKM_HIP(hipStreamSynchronize(st));
    // chunk target: <= 2^27 k-mers, and its device scratch (sort pairs in and out, the double-
    // buffered gather, the radix sort's temporary ~ one more pair array) within 3/4 of the memory
    // free now -- the builder's work buffers are still allocated at finish
    const uint64_t per = 2 * (8 + sizeof(IdxT)) + 2 * (8 + sizeof(skm_stored_kmer_data)) + (8 + sizeof(IdxT));
    size_t free_b = 0, total_b = 0;
    SKM_HIP(hipMemGetInfo(&free_b, &total_b));
    const uint64_t fit = std::max<uint64_t>(1ull << 16, (uint64_t)(0.75 * (double)free_b) / per);
    uint64_t target = std::max<uint64_t>(1ull << 22, std::min<uint64_t>(1ull << 27, ceil_div(n, 4)));
    target = std::min(target, std::min(fit, max_chunk));
    std::vector<Chunk> chunks;
    uint64_t tot = 0, cmax = 0;
    for (uint32_t b = 0; b < OUT_BINS;) {
        Chunk c{b, b, 0, tot};
        while (c.hi < OUT_BINS && (c.n == 0 || c.n + hist[c.hi] <= target)) c.n += hist[c.hi++];
        b = c.hi;
        if (c.n) {
            chunks.push_back(c);
            tot += c.n;
            cmax = std::max(cmax, c.n);
        }
    }
    SKM_CHECK(tot == n, SKM_E_STATE, "kept-set hand-off: histogram does not cover the arena");
    S.chunks = chunks.size();
    S.max_chunk = cmax;
    // 2. device scratch for the largest chunk; double-buffered gather output
    DevBuf kin, kout, vin, vout, tmp, gk[2], gd[2];
    kin.ensure(8 * cmax);
    kout.ensure(8 * cmax);
    vin.ensure(sizeof(IdxT) * cmax);
    vout.ensure(sizeof(IdxT) * cmax);
    size_t tmp_bytes = 0;
    SKM_HIP(rocprim::radix_sort_pairs(nullptr, tmp_bytes, kin.as<uint64_t>(), kout.as<uint64_t>(), vin.as<IdxT>(),
                                      vout.as<IdxT>(), (size_t)cmax, 0, KEY_BITS, st));
    tmp.ensure(std::max<size_t>(tmp_bytes, 16));
    for (int k = 0; k < 2; ++k) {
        gk[k].ensure(8 * cmax);
        gd[k].ensure(sizeof(skm_stored_kmer_data) * cmax + 16);
    }
    // pinned staging ring and the copy stream
    constexpr size_t PIECE = 64ull << 20;
    uint8_t* pin[2] = {nullptr, nullptr};
    hipStream_t cs = nullptr;
    hipEvent_t ev_g[2] = {}, ev_d[2] = {}, ev_p[2] = {};
    // timing: per chunk (start, selected, sorted, gathered) on st; per piece (start, end) on cs
    std::vector<hipEvent_t> tev;
    auto tmark = [&](hipStream_t s_) -> size_t {
        hipEvent_t e;
        SKM_HIP(hipEventCreate(&e));
        tev.push_back(e);
        SKM_HIP(hipEventRecord(e, s_));
        return tev.size() - 1;
    };
    std::vector<size_t> cmark, pmark;
    auto cleanup = [&]() {
        if (cs) (void)hipStreamSynchronize(cs);
        (void)hipStreamSynchronize(st);
        for (auto* p : pin)
            if (p) (void)hipHostFree(p);
        for (auto* set : {ev_g, ev_d, ev_p})
            for (int k = 0; k < 2; ++k)
                if (set[k]) (void)hipEventDestroy(set[k]);
        for (auto e : tev) (void)hipEventDestroy(e);
        if (cs) (void)hipStreamDestroy(cs);
    };
    try {
        const auto ta = now();
        for (int k = 0; k < 2; ++k) {
            SKM_HIP(hipHostMalloc(reinterpret_cast<void**>(&pin[k]), PIECE, hipHostMallocDefault));
            SKM_HIP(hipEventCreateWithFlags(&ev_g[k], hipEventDisableTiming));
            SKM_HIP(hipEventCreateWithFlags(&ev_d[k], hipEventDisableTiming));
            SKM_HIP(hipEventCreateWithFlags(&ev_p[k], hipEventDisableTiming));
        }
        SKM_HIP(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
        S.setup_s = std::chrono::duration<double>(now() - ta).count();
        auto enqueue_chunk = [&](size_t c) {  // select -> sort -> gather into buffer c & 1
            const Chunk& C = chunks[c];
            const int k = (int)(c & 1);
            if (c >= 2) SKM_HIP(hipStreamWaitEvent(st, ev_d[k], 0));  // chunk c-2 has left gk/gd[k]
            cmark.push_back(tmark(st));
            SKM_HIP(hipMemsetAsync(d_cur.p, 0, 8, st));
            hipLaunchKernelGGL(k_out_select<IdxT>, dim3(grid), dim3(OUT_THREADS), 0, st, dkeys, n, C.lo, C.hi,
                               d_cur.as<unsigned long long>(), kin.as<uint64_t>(), vin.as<IdxT>());
            SKM_HIP(hipGetLastError());
            tmark(st);
            size_t tb = tmp.bytes;
            SKM_HIP(rocprim::radix_sort_pairs(tmp.p, tb, kin.as<uint64_t>(), kout.as<uint64_t>(), vin.as<IdxT>(),
                                              vout.as<IdxT>(), (size_t)C.n, 0, KEY_BITS, st));
            tmark(st);
            const uint32_t gg = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(C.n, OUT_THREADS), 4096));
            hipLaunchKernelGGL(k_out_gather<IdxT>, dim3(gg), dim3(OUT_THREADS), 0, st, dkeys, ddata, vout.as<IdxT>(), C.n,
                               gk[k].as<uint64_t>(), gd[k].as<skm_stored_kmer_data>());
            SKM_HIP(hipGetLastError());
            tmark(st);
            SKM_HIP(hipEventRecord(ev_g[k], st));
        };
        // the pieces: each chunk's keys, then its records, in 64 MB pieces
        struct Piece {
            size_t chunk;
            const uint8_t* src;
            uint8_t* dst;
            size_t bytes;
            bool first, last;
        };
        std::vector<Piece> pieces;
        for (size_t c = 0; c < chunks.size(); ++c) {
            const int k = (int)(c & 1);
            const size_t first = pieces.size();
            const std::pair<const uint8_t*, uint8_t*> seg[2] = {
                {gk[k].as<uint8_t>(), reinterpret_cast<uint8_t*>(hk + chunks[c].at)},
                {gd[k].as<uint8_t>(), reinterpret_cast<uint8_t*>(hd + chunks[c].at)}};
            const size_t bytes[2] = {8 * chunks[c].n, sizeof(skm_stored_kmer_data) * chunks[c].n};
            for (int s = 0; s < 2; ++s)
                for (size_t o = 0; o < bytes[s]; o += PIECE)
                    pieces.push_back({c, seg[s].first + o, seg[s].second + o, std::min(PIECE, bytes[s] - o), false, false});
            pieces[first].first = true;
            pieces.back().last = true;
        }
        size_t enq = 0;
        auto issue = [&](size_t p) {  // D2H of piece p into pin[p & 1] on the copy stream
            const Piece& P = pieces[p];
            if (P.first) {
                while (enq <= P.chunk + 1 && enq < chunks.size()) enqueue_chunk(enq++);  // keep the sorter one ahead
                SKM_HIP(hipStreamWaitEvent(cs, ev_g[P.chunk & 1], 0));
            }
            pmark.push_back(tmark(cs));
            SKM_HIP(hipMemcpyAsync(pin[p & 1], P.src, P.bytes, hipMemcpyDeviceToHost, cs));
            tmark(cs);
            SKM_HIP(hipEventRecord(ev_p[p & 1], cs));
            if (P.last) SKM_HIP(hipEventRecord(ev_d[P.chunk & 1], cs));
        };
        const int T = pool ? pool->threads() : 1;
        issue(0);
        for (size_t p = 0; p < pieces.size(); ++p) {
            if (p + 1 < pieces.size()) issue(p + 1);  // pin[(p+1) & 1] was drained by the last iteration
            const auto tw = now();
            SKM_HIP(hipEventSynchronize(ev_p[p & 1]));
            S.wait_s += std::chrono::duration<double>(now() - tw).count();
            const auto tc = now();
            const Piece& P = pieces[p];
            const uint8_t* src = pin[p & 1];
            const int parts = (int)std::max<size_t>(1, std::min<size_t>((size_t)T * 2, P.bytes >> 20));
            auto cp = [&](int q) {
                const size_t a = P.bytes * (size_t)q / (size_t)parts, e = P.bytes * (size_t)(q + 1) / (size_t)parts;
                std::memcpy(P.dst + a, src + a, e - a);
            };
            if (pool)
                pool->run(parts, cp);
            else
                for (int q = 0; q < parts; ++q) cp(q);
            S.copy_s += std::chrono::duration<double>(now() - tc).count();
            S.bytes += P.bytes;
        }
        SKM_HIP(hipStreamSynchronize(cs));
        SKM_HIP(hipStreamSynchronize(st));
        float ms = 0;
        for (size_t m : cmark) {
            SKM_HIP(hipEventElapsedTime(&ms, tev[m], tev[m + 1]));
            S.select_ms += ms;
            SKM_HIP(hipEventElapsedTime(&ms, tev[m + 1], tev[m + 2]));
            S.sort_ms += ms;
            SKM_HIP(hipEventElapsedTime(&ms, tev[m + 2], tev[m + 3]));
            S.gather_ms += ms;
        }
        for (size_t m : pmark) {
            SKM_HIP(hipEventElapsedTime(&ms, tev[m], tev[m + 1]));
            S.d2h_ms += ms;
        }
    } catch (...) {
        cleanup();
        throw;
    }
    cleanup();
    S.total_s = std::chrono::duration<double>(now() - t0).count();
    if (stats) *stats = S;
}

}  // namespace

void kept_handoff(const uint64_t* dkeys, const skm_stored_kmer_data* ddata, uint64_t n, hipStream_t st,
                  HostPool* pool, uint64_t** keys_out, skm_stored_kmer_data** data_out, HandoffStats* stats,
                  uint64_t index_limit, uint64_t max_chunk) {
    // index_limit (test hook, 0 = 2^32): hand-offs of at least that many k-mers take u64 arena indices
    const uint64_t lim = index_limit ? index_limit : (1ull << 32);
    if (n < lim)
        kept_handoff_t<uint32_t>(dkeys, ddata, n, st, pool, keys_out, data_out, stats, max_chunk ? max_chunk : ~0ull);
    else
        kept_handoff_t<uint64_t>(dkeys, ddata, n, st, pool, keys_out, data_out, stats, max_chunk ? max_chunk : ~0ull);
    if (stats) stats->wide_index = n >= lim ? 1 : 0;
}

}  // namespace skm
