// skm_bdz.h -- CMPH BDZ minimal perfect hash: cmph_dump-compatible image I/O, host search and
// host construction (3-hypergraph peeling).  The device lookup lives in skm_annotate.hip.
//
// Layout of a cmph 2.0 BDZ dump (what CmphKmerDb::load_hash reads via cmph_load,
// cmph_kmer.h:95-104, and what build_perfect_hash writes via cmph_dump, perfect_hash.h:66):
//   "bdz\0" | u32 size(m) | u32 buflen | "jenkins\0" u32 seed | u32 n | u32 m | u32 r |
//   u8 g[ceil(n/4)] | u32 k | u8 b | u32 ranktablesize | u32 ranktable[ranktablesize]
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace skm {

struct Bdz {
    uint32_t m = 0, n = 0, r = 0, k = 128, ranktablesize = 0, seed = 0;
    uint8_t b = 7;
    std::vector<uint8_t> g;
    std::vector<uint32_t> ranktable;
};

void jenkins_hash_vector(uint32_t seed, const uint8_t* k, uint32_t keylen, uint32_t* hashes);
bool bdz_parse(const uint8_t* buf, size_t len, Bdz& out, std::string& err);
std::vector<uint8_t> bdz_dump(const Bdz& h);
uint32_t bdz_search(const Bdz& h, const uint8_t* key, uint32_t keylen);
// Construct over n 8-byte keys (distinct).  Returns false if no acyclic graph was found.
bool bdz_build(const uint64_t* keys, size_t n, uint32_t seed, Bdz& out, std::string& err);

}  // namespace skm
