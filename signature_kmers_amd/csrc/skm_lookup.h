// skm_lookup.h -- device-side signature DB lookup shared by the annotate and matrix-distance
// paths: the HBM layout of a CmphKmerDb / KeptKmerDB (skm_db), the window iterator predicates of
// for_each_kmer<8> (kmer_data.h:76-102) and cmph's bdz_search (cmph_kmer.h:139-147).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "skm_bdz.h"
#include "skm_util.h"

namespace skm {

constexpr uint32_t NO_HIT = 0xFFFFFFFFu;
constexpr int LK_THREADS = 256;
constexpr int LK_POS = 16;

struct QMeta {
    uint64_t pstart;
    uint32_t len;
    uint32_t pad;
};

struct DevBdz {
    const uint32_t* g;          // g as little-endian u32 words (16 entries each), padded
    const uint32_t* ranktable;
    const uint16_t* dat;        // 5 u16 per record
    const uint32_t* fm;         // per record: function_index | mean << 16 (what the call path reads)
    // b == 7: 64-byte line per block of 128 vertices: 8 pairs (g word, rank of its first vertex =
    // rank table entry + assigned vertices before it), so the 8-byte load that fetches a
    // candidate vertex's g word for the selection also brings its rank
    const uint32_t* blk;
    uint32_t m, r, b, seed;
    uint64_t r_magic;           // fastmod: ceil(2^64 / r)
    // exact-key mode (KeptKmerDB, kept_kmer_db.h:20-27): open-addressing table of the kept keys,
    // 16-byte slots (x, y = the key's low / high word, 0 = empty: a k-mer key is never 0; z = its
    // record index; w = the record's function_index << 16 | mean), eight to a 128-byte line: a
    // probe and the call path's record word arrive in one load (round 5 had the keys, the record
    // indices and the records in three arrays: three lines per window)
    const uint4* xtab;                // [mask+1]
    uint64_t xmask;
    uint32_t xshift;
};

__device__ __forceinline__ uint64_t xmix(uint64_t k) {  // murmur3 fmix64 (bijective)
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

// KeptKmerDB::fetch: the slot of the key, or an empty slot (x == y == 0) on a miss
__device__ __forceinline__ uint4 exact_slot(const DevBdz& D, uint32_t lo, uint32_t hi) {
    const uint64_t k = ((uint64_t)hi << 32) | lo;
    uint64_t h = xmix(k) >> D.xshift;
    for (;;) {
        const uint4 t = D.xtab[h];
        if ((t.x == lo && t.y == hi) || (t.x | t.y) == 0u) return t;
        h = (h + 1) & D.xmask;
    }
}
// the record index of a kept k-mer; D.m on a miss
__device__ __forceinline__ uint32_t exact_lookup(const DevBdz& D, uint32_t lo, uint32_t hi) {
    const uint4 t = exact_slot(D, lo, hi);
    return (t.x | t.y) ? t.z : D.m;
}

__device__ __forceinline__ uint32_t fastmod(uint32_t a, uint64_t M, uint32_t d) {
    uint64_t low = M * a;
    return (uint32_t)__umul64hi(low, (uint64_t)d);
}

__device__ __forceinline__ void jmix(uint32_t& a, uint32_t& b, uint32_t& c) {
    a -= b; a -= c; a ^= (c >> 13);
    b -= c; b -= a; b ^= (a << 8);
    c -= a; c -= b; c ^= (b >> 13);
    a -= b; a -= c; a ^= (c >> 12);
    b -= c; b -= a; b ^= (a << 16);
    c -= a; c -= b; c ^= (b >> 5);
    a -= b; a -= c; a ^= (c >> 3);
    b -= c; b -= a; b ^= (a << 10);
    c -= a; c -= b; c ^= (b >> 15);
}

__device__ __forceinline__ uint32_t gval(const uint32_t* g, uint32_t i) { return (g[i >> 4] >> ((i & 15u) * 2)) & 3u; }

__device__ __forceinline__ uint32_t unassigned_in(uint32_t w) { return __popc(w & (w >> 1) & 0x55555555u); }

// cmph bdz_search for an 8-byte key given as two little-endian u32 words
__device__ __forceinline__ uint32_t bdz_lookup(const DevBdz& D, uint32_t lo, uint32_t hi) {
    uint32_t a = 0x9e3779b9u + lo, b = 0x9e3779b9u + hi, c = D.seed + 8u;
    jmix(a, b, c);
    const uint32_t h0 = fastmod(a, D.r_magic, D.r);
    const uint32_t h1 = fastmod(b, D.r_magic, D.r) + D.r;
    const uint32_t h2 = fastmod(c, D.r_magic, D.r) + 2u * D.r;
    const uint32_t sel = (gval(D.g, h0) + gval(D.g, h1) + gval(D.g, h2)) % 3u;
    const uint32_t v = sel == 0 ? h0 : (sel == 1 ? h1 : h2);
    // rank(v): ranktable[v >> b] + assigned entries in [ (v>>b)<<b, v )
    const uint32_t blk = v >> D.b;
    uint32_t rank = D.ranktable[blk];
    uint32_t i = blk << D.b;
    // head: up to the next 16-aligned entry
    while (i < v && (i & 15u)) {
        rank += gval(D.g, i) != 3u;
        ++i;
    }
    for (; i + 16 <= v; i += 16) rank += 16u - unassigned_in(D.g[i >> 4]);
    if (i < v) {
        const uint32_t nb = (v - i) * 2u;
        const uint32_t w = D.g[i >> 4] & ((1u << nb) - 1u);
        rank += (v - i) - unassigned_in(w);
    }
    return rank;
}

// the same search over the b == 7 (g word, rank) pair lines (D.blk): one 8-byte gather per
// candidate vertex, then the rank from the selected pair
__device__ __forceinline__ uint32_t bdz7_lookup(const DevBdz& D, uint32_t lo, uint32_t hi) {
    uint32_t a = 0x9e3779b9u + lo, b = 0x9e3779b9u + hi, c = D.seed + 8u;
    jmix(a, b, c);
    const uint32_t hv[3] = {fastmod(a, D.r_magic, D.r), fastmod(b, D.r_magic, D.r) + D.r,
                            fastmod(c, D.r_magic, D.r) + 2u * D.r};
    uint2 gp[3];
#pragma unroll
    for (int j = 0; j < 3; ++j)
        gp[j] = *reinterpret_cast<const uint2*>(D.blk + (hv[j] >> 7) * 16u + 2u * ((hv[j] & 127u) >> 4));
    uint32_t sum = 0;
#pragma unroll
    for (int j = 0; j < 3; ++j) sum += (gp[j].x >> ((hv[j] & 15u) * 2)) & 3u;
    const uint32_t sel = sum % 3u;
    const bool s0 = sel == 0, s1 = sel == 1;
    const uint32_t qx = s0 ? gp[0].x : (s1 ? gp[1].x : gp[2].x);
    const uint32_t qy = s0 ? gp[0].y : (s1 ? gp[1].y : gp[2].y);
    const uint32_t pe = (s0 ? hv[0] : (s1 ? hv[1] : hv[2])) & 15u;
    const uint32_t pmask = pe ? (0xFFFFFFFFu >> (32u - 2u * pe)) : 0u;
    return qy + pe - unassigned_in(qx & pmask);
}

__device__ __forceinline__ bool ambig(uint32_t c) { return c == 'X' || c == '*'; }

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// key bytes t..t+7 of the 32-byte window w[8]
__device__ __forceinline__ void key_at(const uint32_t (&w)[8], int t, uint32_t& lo, uint32_t& hi) {
    const int wi = t >> 2, sh = (t & 3) * 8;
    if (sh == 0) {
        lo = w[wi];
        hi = w[wi + 1];
    } else {
        lo = (w[wi] >> sh) | (w[wi + 1] << (32 - sh));
        hi = (w[wi + 1] >> sh) | (w[wi + 2] << (32 - sh));
    }
}

// exclusive scan of n u32 values into n+1 u64 offsets (out[n] = total), on stream st
struct Scanner {
    DevBuf tiles, total;
    void run(const uint32_t* in, uint64_t n, uint64_t* out, hipStream_t st);
};

}  // namespace skm

struct skm_query;

// CmphKmerDb<StoredKmerData,8> / KeptKmerDB<8> resident in HBM (skm_db_open*, skm_annotate.hip)
struct skm_db {
    skm_query* aq = nullptr;     // skm_annotate's query, reused call to call (its buffers, stream)
    int device = 0;
    bool exact = false;          // KeptKmerDB semantics (skm_db_open_kept)
    uint32_t m = 0;              // hash size (BDZ) or number of kept keys (exact)
    skm::Bdz bdz;
    uint64_t dat_records = 0;
    skm::DevBuf d_g, d_rank, d_dat, d_xtab, d_fm, d_blk;
    skm::DevBdz dev{};
};
