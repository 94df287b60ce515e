// skm_bdz.cpp -- CMPH-compatible BDZ image I/O, host search, and host construction.
//
// Construction follows the BDZ scheme the reference gets from cmph_new(CMPH_BDZ)
// (perfect_hash.h:29-33): r = ceil(1.23 m / 3) rounded up to odd, n = 3r vertices, one
// 3-edge per key from the jenkins hash, peel the 3-hypergraph, assign 2-bit g values in
// reverse peel order so that (g[h0]+g[h1]+g[h2]) % 3 selects the key's free vertex, then a rank
// table over blocks of k = 2^b vertices.  Any acyclic peel order yields a valid MPH; the bytes
// differ from cmph's (which depend on rand() and TBB iteration order), reading is exact.
#include "skm_bdz.h"

#include <cmath>
#include <cstring>
#include <random>

namespace skm {

static inline void jmix(uint32_t& a, uint32_t& b, uint32_t& c) {
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

void jenkins_hash_vector(uint32_t seed, const uint8_t* k, uint32_t keylen, uint32_t* hashes) {
    uint32_t len = keylen;
    uint32_t a = 0x9e3779b9u, b = 0x9e3779b9u, c = seed;
    while (len >= 12) {
        a += (uint32_t)k[0] | ((uint32_t)k[1] << 8) | ((uint32_t)k[2] << 16) | ((uint32_t)k[3] << 24);
        b += (uint32_t)k[4] | ((uint32_t)k[5] << 8) | ((uint32_t)k[6] << 16) | ((uint32_t)k[7] << 24);
        c += (uint32_t)k[8] | ((uint32_t)k[9] << 8) | ((uint32_t)k[10] << 16) | ((uint32_t)k[11] << 24);
        jmix(a, b, c);
        k += 12;
        len -= 12;
    }
    c += keylen;
    // tail bytes: byte j of the last block goes to a (j<4), b (4<=j<8), c (8<=j<11, shifted by 8)
    for (uint32_t j = 0; j < len; ++j) {
        uint32_t v = k[j];
        if (j < 4)
            a += v << (8 * j);
        else if (j < 8)
            b += v << (8 * (j - 4));
        else
            c += v << (8 * (j - 7));
    }
    jmix(a, b, c);
    hashes[0] = a;
    hashes[1] = b;
    hashes[2] = c;
}

static inline uint32_t gv(const std::vector<uint8_t>& g, uint32_t i) { return (g[i >> 2] >> ((i & 3u) << 1)) & 3u; }

bool bdz_parse(const uint8_t* buf, size_t len, Bdz& h, std::string& err) {
    size_t p = 0;
    auto rd32 = [&](uint32_t& v) {
        if (p + 4 > len) return false;
        std::memcpy(&v, buf + p, 4);
        p += 4;
        return true;
    };
    std::string algo;
    while (p < len && buf[p]) algo.push_back((char)buf[p++]);
    if (p >= len || algo != "bdz") {
        err = "not a cmph BDZ image (algorithm '" + algo + "')";
        return false;
    }
    ++p;
    uint32_t size = 0, buflen = 0;
    if (!rd32(size) || !rd32(buflen) || p + buflen > len) {
        err = "truncated header";
        return false;
    }
    if (buflen != 12 || std::strncmp((const char*)buf + p, "jenkins", 8) != 0) {
        err = "unsupported hash state (only jenkins)";
        return false;
    }
    std::memcpy(&h.seed, buf + p + 8, 4);
    p += buflen;
    if (!rd32(h.n) || !rd32(h.m) || !rd32(h.r)) {
        err = "truncated n/m/r";
        return false;
    }
    const size_t sizeg = (size_t)std::ceil(h.n / 4.0);
    if (p + sizeg > len) {
        err = "truncated g";
        return false;
    }
    h.g.assign(buf + p, buf + p + sizeg);
    p += sizeg;
    if (!rd32(h.k) || p + 1 > len) {
        err = "truncated k/b";
        return false;
    }
    h.b = buf[p++];
    if (!rd32(h.ranktablesize) || p + 4ull * h.ranktablesize > len) {
        err = "truncated rank table";
        return false;
    }
    h.ranktable.resize(h.ranktablesize);
    if (h.ranktablesize) std::memcpy(h.ranktable.data(), buf + p, 4ull * h.ranktablesize);
    // everything the searches index must be in range: g[v] for v < n = 3r, ranktable[v >> b]
    if (h.r == 0 || 3ull * h.r != (uint64_t)h.n || size != h.m || h.m > h.n) {
        err = "inconsistent BDZ parameters";
        return false;
    }
    if (h.b >= 32 || h.k != (1u << h.b) || (uint64_t)h.ranktablesize < ((uint64_t)h.n + h.k - 1) / h.k) {
        err = "inconsistent BDZ rank table (k, b, ranktablesize)";
        return false;
    }
    return true;
}

std::vector<uint8_t> bdz_dump(const Bdz& h) {
    std::vector<uint8_t> out;
    auto put = [&](const void* p, size_t n) {
        const uint8_t* c = (const uint8_t*)p;
        out.insert(out.end(), c, c + n);
    };
    auto put32 = [&](uint32_t v) { put(&v, 4); };
    put("bdz", 4);
    put32(h.m);
    put32(12);
    put("jenkins", 8);
    put32(h.seed);
    put32(h.n);
    put32(h.m);
    put32(h.r);
    put(h.g.data(), h.g.size());
    put32(h.k);
    put(&h.b, 1);
    put32(h.ranktablesize);
    put(h.ranktable.data(), 4ull * h.ranktable.size());
    return out;
}

uint32_t bdz_search(const Bdz& h, const uint8_t* key, uint32_t keylen) {
    uint32_t hl[3];
    jenkins_hash_vector(h.seed, key, keylen, hl);
    hl[0] = hl[0] % h.r;
    hl[1] = hl[1] % h.r + h.r;
    hl[2] = hl[2] % h.r + (h.r << 1);
    const uint32_t v = hl[(gv(h.g, hl[0]) + gv(h.g, hl[1]) + gv(h.g, hl[2])) % 3];
    const uint32_t idx = v >> h.b;
    uint32_t rank = h.ranktable[idx];
    for (uint32_t i = idx << h.b; i < v; ++i) rank += gv(h.g, i) != 3u;
    return rank;
}

bool bdz_build(const uint64_t* keys, size_t nkeys, uint32_t seed, Bdz& h, std::string& err) {
    const double c = 1.23;
    h.m = (uint32_t)nkeys;
    h.r = (uint32_t)std::ceil((c * nkeys) / 3);
    if (h.r % 2 == 0) h.r += 1;
    h.b = 7;
    h.k = 1u << h.b;
    {   // duplicate keys never give an acyclic 3-graph: report them instead of retrying
        std::vector<uint64_t> sk(keys, keys + nkeys);
        std::sort(sk.begin(), sk.end());
        if (std::adjacent_find(sk.begin(), sk.end()) != sk.end()) {
            err = "BDZ construction failed: duplicate keys";
            return false;
        }
    }
    std::mt19937 rng(seed);
    std::vector<uint32_t> ev((size_t)3 * nkeys);
    std::vector<uint32_t> deg, xor_edge, queue;
    std::vector<uint8_t> removed;
    for (int attempt = 0; attempt < 1000; ++attempt) {
        // tiny key sets (r = 1 or 3) can be cyclic for every seed: widen r (kept odd) every 20
        // failed attempts.  Readers take r from the image, so any odd r stays cmph-compatible.
        if (attempt > 0 && attempt % 20 == 0) h.r += 2;
        h.n = 3 * h.r;
        h.ranktablesize = (uint32_t)std::ceil(h.n / (double)h.k);
        deg.assign(h.n, 0);
        xor_edge.assign(h.n, 0);
        h.seed = rng();
        for (size_t e = 0; e < nkeys; ++e) {
            uint8_t kb[8];
            std::memcpy(kb, &keys[e], 8);
            uint32_t hl[3];
            jenkins_hash_vector(h.seed, kb, 8, hl);
            uint32_t v0 = hl[0] % h.r, v1 = hl[1] % h.r + h.r, v2 = hl[2] % h.r + (h.r << 1);
            ev[3 * e] = v0;
            ev[3 * e + 1] = v1;
            ev[3 * e + 2] = v2;
            deg[v0]++;
            deg[v1]++;
            deg[v2]++;
            xor_edge[v0] ^= (uint32_t)e;
            xor_edge[v1] ^= (uint32_t)e;
            xor_edge[v2] ^= (uint32_t)e;
        }
        // peel: vertices of degree 1 identify their only edge through the XOR of incident edges
        queue.clear();
        queue.reserve(nkeys);
        removed.assign(nkeys, 0);
        std::vector<uint32_t> free_vertex(nkeys, 0);
        std::vector<uint32_t> stack;
        for (uint32_t v = 0; v < h.n; ++v)
            if (deg[v] == 1) stack.push_back(v);
        while (!stack.empty()) {
            uint32_t v = stack.back();
            stack.pop_back();
            if (deg[v] != 1) continue;
            uint32_t e = xor_edge[v];
            if (removed[e]) continue;
            removed[e] = 1;
            queue.push_back(e);
            free_vertex[e] = v;
            for (int j = 0; j < 3; ++j) {
                uint32_t u = ev[3 * (size_t)e + j];
                deg[u]--;
                xor_edge[u] ^= e;
                if (deg[u] == 1) stack.push_back(u);
            }
        }
        if (queue.size() != nkeys) continue;  // cyclic: new seed
        // assign in reverse peel order: the free vertex gets the value that selects it
        h.g.assign((size_t)std::ceil(h.n / 4.0), 0xFF);
        std::vector<uint8_t> visited(h.n, 0);
        auto setv = [&](uint32_t i, uint32_t val) {
            h.g[i >> 2] = (uint8_t)((h.g[i >> 2] & ~(3u << ((i & 3u) << 1))) | (val << ((i & 3u) << 1)));
        };
        for (size_t qi = queue.size(); qi-- > 0;) {
            uint32_t e = queue[qi];
            uint32_t fv = free_vertex[e];
            int fj = 0;
            for (int j = 0; j < 3; ++j)
                if (ev[3 * (size_t)e + j] == fv) fj = j;
            uint32_t s = 0;
            for (int j = 0; j < 3; ++j) {
                uint32_t u = ev[3 * (size_t)e + j];
                if (j == fj) continue;
                if (!visited[u]) {
                    visited[u] = 1;  // stays UNASSIGNED (3)
                }
                s += gv(h.g, u);
            }
            setv(fv, (uint32_t)((fj + 9 - (s % 3)) % 3));
            visited[fv] = 1;
        }
        // rank table: assigned entries before each block of k vertices
        h.ranktable.assign(h.ranktablesize, 0);
        uint32_t count = 0;
        for (uint32_t i = 0; i < h.ranktablesize; ++i) {
            h.ranktable[i] = count;
            uint32_t v0 = i * h.k, v1 = std::min<uint32_t>(h.n, v0 + h.k);
            for (uint32_t v = v0; v < v1; ++v) count += gv(h.g, v) != 3u;
        }
        return true;
    }
    err = "BDZ construction failed: no acyclic 3-graph in 1000 attempts";
    return false;
}

}  // namespace skm
