// ============================================================================================
//  oracle/skm_oracle.cpp  --  TEST INFRASTRUCTURE ONLY (the checker, never the product path)
// ============================================================================================
//
//  CPU restatement of the olsonanl/signature_kmers hot path (reference @ 2024-11-15, read from
//  /root/reference as text; nothing is copied).  Only tests/, __graft_entry__.smoke() and the
//  `cpu_baseline` leg of bench.py may load this library.  The product (signature_kmers_amd/,
//  libskm.so, the CLIs) never links or calls it.
//
//  PARITY STATUS: **partly pinned**.  The window iterator for_each_kmer<8> (kmer_data.h:76-102)
//  is pinned against the reference's own code: oracle/Makefile.ref compiles kmer_data.h and
//  fasta_parser.{h,cc} unchanged from /root/reference (std-only headers) into oracle/_ref/ref_pin,
//  whose outputs over adversarial inputs are tests/golden/ref_windows.npz / ref_fasta.npz
//  (tests/test_ref_pin_cpu.py checks oracle_kmer_windows against them).  Everything else is
//  **parity unpinned**: the rest of the reference cannot be compiled here (Boost, TBB<=2020
//  headers, CMPH and NuDB are absent; NuDB is git-cloned from the network by its Makefile) and
//  it ships no tests, fixtures or golden vectors.  That part is pinned
//  only by (a) known-answer tests derived from the reference source semantics
//  (tests/test_oracle_kat.py) and (b) the restated third-party algorithms below, whose versions
//  are unpinned by the reference Makefile:
//     * CMPH 2.0.x BDZ  (jenkins lookup2 hash, 2-bit g array, rank table)   -- cmph_kmer.h:85-147
//     * Boost.Accumulators mean / median(P^2) / variance (accumulator_set<unsigned short,..>)
//                                                                            -- signature_build.tcc:262-279
//     * Boost.Math statistics mean / median / median_absolute_deviation      -- call_functions.tcc:51-53
//     * TBB 2020 concurrent_unordered_multimap duplicate order (LIFO)        -- signature_build.tcc:186-208
//
//  Semantics follow `--n-threads 1` of the reference (the only deterministic mode).
//
//  Functions and the reference lines they restate:
//    oracle_build            signature_build.tcc:121-181 (load_kmers_from_sequence),
//                            :184-213 (process_kmers), :219-293 (process_kmer_set)
//    P2Median / SigAcc       Boost.Accumulators p_square_quantile / variance / mean (lazy)
//    oracle_bdz_*            cmph bdz.c search/rank + cmph_load layout (cmph_kmer.h:95-104,139-147)
//    oracle_process_aa_seq   call_functions.tcc:259-338 + HitSet::process :35-103,
//                            for_each_kmer kmer_data.h:76-102
//    oracle_find_best_call   call_functions.tcc:347-659
//    oracle_matrix_distance  kmers-matrix-distance.cc:94-212, matrix_distance.h:45-170
// ============================================================================================

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <regex>
#include <set>
#include <string>
#include <thread>
#include <vector>

extern "C" {

#pragma pack(push, 1)
struct oracle_stored {             // StoredKmerData, kmer_data.h:114-128 (5 x u16 = 10 B)
    uint16_t avg_from_end;
    uint16_t function_index;
    uint16_t mean;
    uint16_t median;
    uint16_t var;
};
#pragma pack(pop)

struct oracle_call {               // KmerCall, call_functions.h:23-48
    uint32_t start;
    uint32_t end;
    int32_t count;
    uint16_t function_index;
    uint16_t pad;
    uint32_t protein_length_median;
    float protein_length_med_avg_dev;
};

}  // extern "C"

namespace {

const uint16_t kUndefinedFunction = 0xFFFF;  // kmer_data.h:23

// ok_prot_ (signature_build.h:102-103): 20 amino acids, both cases.  std::set<unsigned char>::find
// of the reference as a 256-entry membership table (same answer for every byte).
struct OkProt {
    bool t[256] = {};
    OkProt() {
        for (const char* s = "ACDEFGHIKLMNPQRSTVWYacdefghiklmnpqrstvwy"; *s; ++s) t[(unsigned char)*s] = true;
    }
};
const OkProt kOkProt;
inline bool ok_prot(unsigned char c) { return kOkProt.t[c]; }

// double -> unsigned short as gcc/x86-64 emits it (cvttsd2si to a 32-bit int, keep 16 bits);
// out-of-range doubles give the integer-indefinite value 0x80000000 -> 0.  
uint16_t d2u16(double d) {
    if (!(d > -2147483649.0 && d < 2147483648.0)) return 0;
    return (uint16_t)(int32_t)d;
}

// --------------------------------------------------------------------------------------------
// Boost.Accumulators p_square_quantile (p = 0.5, the default median feature).
// --------------------------------------------------------------------------------------------
struct P2Median {
    double heights[5] = {0, 0, 0, 0, 0};
    double actual[5] = {1, 2, 3, 4, 5};
    double desired[5] = {1, 2, 3, 4, 5};   // 1, 1+2p, 1+4p, 3+2p, 5
    static constexpr double incr[5] = {0.0, 0.25, 0.5, 0.75, 1.0};  // 0, p/2, p, (1+p)/2, 1

    void add(uint32_t sample, size_t cnt) {
        const double x = (double)sample;
        if (cnt <= 5) {
            heights[cnt - 1] = x;
            if (cnt == 5) std::sort(heights, heights + 5);
            return;
        }
        size_t cell;
        if (x < heights[0]) {
            heights[0] = x;
            cell = 1;
        } else if (heights[4] <= x) {
            heights[4] = x;
            cell = 4;
        } else {
            cell = (size_t)(std::upper_bound(heights, heights + 5, x) - heights);
        }
        for (size_t i = cell; i < 5; ++i) actual[i] += 1.0;
        for (size_t i = 0; i < 5; ++i) desired[i] += incr[i];
        for (size_t i = 1; i <= 3; ++i) {
            double d = desired[i] - actual[i];
            double dp = actual[i + 1] - actual[i];
            double dm = actual[i - 1] - actual[i];
            double hp = (heights[i + 1] - heights[i]) / dp;
            double hm = (heights[i - 1] - heights[i]) / dm;
            if ((d >= 1. && dp > 1.) || (d <= -1. && dm < -1.)) {
                short sign_d = static_cast<short>(d / std::abs(d));
                double h = heights[i] + sign_d / (dp - dm) * ((sign_d - dm) * hp + (dp - sign_d) * hm);
                if (heights[i - 1] < h && h < heights[i + 1]) {
                    heights[i] = h;
                } else {
                    if (d > 0) heights[i] += hp;
                    if (d < 0) heights[i] -= hm;
                }
                actual[i] += sign_d;
            }
        }
    }
    double result() const { return heights[2]; }
};
constexpr double P2Median::incr[5];

// accumulator_set<unsigned short, stats<tag::mean, tag::median, tag::variance>>
// (signature_build.tcc:262-264).  sum is stored as the Sample type (u16, wraps); mean is the
// lazy sum/count; variance's mean dependency resolves to that lazy mean; features are updated in
// dependency order (count, sum, ..., variance).
struct SigAcc {
    size_t count = 0;
    uint16_t sum = 0;
    double variance = 0.0;
    P2Median median;

    void operator()(uint32_t x) {
        ++count;
        sum = (uint16_t)(sum + x);
        median.add(x, count);
        if (count > 1) {
            double mean = (double)sum / (double)count;
            double tmp = (double)x - mean;
            variance = variance * (double)(count - 1) / (double)count + tmp * tmp / (double)(count - 1);
        }
    }
    double mean() const { return (double)sum / (double)count; }
};

struct Occ {
    uint64_t key;       // 8 raw residue bytes, little-endian (byte 0 = first residue)
    uint32_t seq;       // index into the caller's sequence arrays
    uint32_t i;         // window start within the sequence
};

inline uint64_t load_key(const uint8_t* p) {
    uint64_t k;
    std::memcpy(&k, p, 8);
    return k;
}

}  // namespace

extern "C" {

// --------------------------------------------------------------------------------------------
//  Signature build: extract (A2) + group (A4) + cut/stats (A5).
//  Inputs are the per-sequence arrays the C-ABI skm_build_add_batch takes, in reference emission
//  order.  seq_func == 0xFFFF means "no kept function" (the reference returns before extracting,
//  signature_build.tcc:155-158).  Outputs are sorted by key.
// --------------------------------------------------------------------------------------------
int oracle_build(const uint8_t* residues, const uint64_t* seq_off, const uint32_t* seq_len,
                 const uint16_t* seq_func, const uint32_t* seq_id, uint64_t n_seqs,
                 uint32_t n_functions, uint64_t* out_keys, oracle_stored* out_data, uint64_t out_cap,
                 uint64_t* out_n, uint32_t* distinct_functions, uint32_t* seqs_with_func,
                 uint64_t* n_seqs_with_signature, uint64_t* distinct_signatures) {
    const int K = 8;
    std::vector<Occ> occ;
    for (uint32_t f = 0; f < n_functions; ++f) {
        distinct_functions[f] = 0;
        seqs_with_func[f] = 0;
    }
    // load_kmers_from_sequence: insertion order = sequence order, window order.
    for (uint64_t s = 0; s < n_seqs; ++s) {
        uint16_t f = seq_func[s];
        if (f == kUndefinedFunction) continue;
        if (f < n_functions) seqs_with_func[f]++;
        const uint8_t* seq = residues + seq_off[s];
        uint32_t len = seq_len[s];
        if (len < (uint32_t)K) continue;
        for (uint32_t i = 0; i + K <= len; ++i) {
            bool ok = true;
            for (int j = 0; j < K; ++j)
                if (!ok_prot(seq[i + j])) { ok = false; break; }
            if (ok) occ.push_back({load_key(seq + i), (uint32_t)s, i});
        }
    }
    // Group: equal keys contiguous; each group is visited in REVERSE insertion order
    // (TBB 2020 multimap inserts a duplicate before the first equal node).
    std::stable_sort(occ.begin(), occ.end(), [](const Occ& a, const Occ& b) { return a.key < b.key; });

    std::set<uint32_t> seqs_with_signature;
    uint64_t kept = 0, n_sig = 0;
    size_t a = 0;
    std::vector<uint16_t> offsets;
    while (a < occ.size()) {
        size_t b = a + 1;
        while (b < occ.size() && occ[b].key == occ[a].key) ++b;
        // KmerSet: func_count (std::map, ascending FunctionIndex), count, set (visit order)
        std::map<uint16_t, int> func_count;
        int count = 0;
        for (size_t j = b; j-- > a;) {
            func_count[seq_func[occ[j].seq]]++;
            count++;
        }
        // process_kmer_set (signature_build.tcc:219-293)
        uint16_t best_func_1 = kUndefinedFunction;
        int best_count_1 = -1, best_count_2 = -1;
        for (auto& x : func_count) {
            if (best_func_1 == kUndefinedFunction) {
                best_func_1 = x.first;
                best_count_1 = x.second;
            } else if (x.second > best_count_1) {
                best_count_2 = best_count_1;
                best_func_1 = x.first;
                best_count_1 = x.second;
            } else if (x.second > best_count_2) {
                best_count_2 = x.second;
            }
        }
        float thresh = float(count) * 0.8f;
        int best_count = best_count_1;
        uint16_t best_func = best_func_1;
        if (!((float)best_count < thresh)) {
            SigAcc acc;
            offsets.clear();
            for (size_t j = b; j-- > a;) {
                const Occ& o = occ[j];
                uint32_t len = seq_len[o.seq];
                if (seq_func[o.seq] == best_func) acc(len);
                offsets.push_back((uint16_t)(len - o.i));
                seqs_with_signature.insert(seq_id[o.seq]);
            }
            uint16_t mean = d2u16(acc.mean());
            uint16_t median = d2u16(acc.median.result());
            uint16_t var = d2u16(acc.variance);
            std::sort(offsets.begin(), offsets.end());
            uint16_t avg_from_end = offsets[offsets.size() / 2];
            n_sig++;
            if (best_func < n_functions) distinct_functions[best_func]++;
            if (kept < out_cap) {
                out_keys[kept] = occ[a].key;
                out_data[kept] = {avg_from_end, best_func, mean, median, var};
            }
            kept++;
        }
        a = b;
    }
    *out_n = kept;
    *n_seqs_with_signature = seqs_with_signature.size();
    *distinct_signatures = n_sig;
    return kept <= out_cap ? 0 : -1;
}

// --------------------------------------------------------------------------------------------
//  The same build on n_threads host threads (the CPU baseline of bench.py on all the node's
//  cores).  Same semantics as oracle_build (the --n-threads 1 results, not the
//  racy multithreaded reference): sequences are split into contiguous ranges, each thread
//  extracts its range into per-shard lists (shard = hash of the key), the lists of a shard are
//  concatenated in range order (so insertion order is kept) and each shard is grouped and cut
//  by one thread exactly like oracle_build.  Kept k-mers come out in shard order (the
//  reference's kept_kmers_ is a hash map, unordered); out_keys/out_data must hold every window.
// --------------------------------------------------------------------------------------------
// The build restricted to one slice of the key space (checks at sizes the whole build cannot be
// held in host memory, e.g. the 50M-protein proteome): only windows whose key passes
// slice_hash(key) >> (64 - sel_bits) == sel are grouped (sel_bits 0 = every window).  Every key's
// occurrences are all in or all out, so each selected group is exactly the reference's group.
// Besides the kept k-mers of the slice (at most out_cap; *out_n is the full count) it returns the
// valid windows of the WHOLE input (*valid_windows, all keys), the largest selected group
// (*max_group) and, if seq_flags != nullptr, the per-sequence flags of the slice's kept k-mers.
// slice_hash is MurmurHash3's 64-bit finalizer of the little-endian key (a public function; the
// product's skm_build_finish_slice selects with the same one).
static inline uint64_t slice_hash(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

int oracle_build_sel_mt(const uint8_t* residues, const uint64_t* seq_off, const uint32_t* seq_len,
                        const uint16_t* seq_func, const uint32_t* seq_id, uint64_t n_seqs, uint32_t n_functions,
                        int n_threads, int sel_bits, uint64_t sel, uint64_t* out_keys, oracle_stored* out_data,
                        uint64_t out_cap, uint64_t* out_n, uint32_t* distinct_functions, uint32_t* seqs_with_func,
                        uint64_t* n_seqs_with_signature, uint64_t* distinct_signatures, uint64_t* valid_windows,
                        uint64_t* max_group, uint8_t* seq_flags);

int oracle_build_mt(const uint8_t* residues, const uint64_t* seq_off, const uint32_t* seq_len,
                    const uint16_t* seq_func, const uint32_t* seq_id, uint64_t n_seqs, uint32_t n_functions,
                    int n_threads, uint64_t* out_keys, oracle_stored* out_data, uint64_t* out_n,
                    uint32_t* distinct_functions, uint32_t* seqs_with_func, uint64_t* n_seqs_with_signature,
                    uint64_t* distinct_signatures) {
    uint64_t valid = 0, mg = 0;
    return oracle_build_sel_mt(residues, seq_off, seq_len, seq_func, seq_id, n_seqs, n_functions, n_threads, 0, 0,
                               out_keys, out_data, ~0ull, out_n, distinct_functions, seqs_with_func,
                               n_seqs_with_signature, distinct_signatures, &valid, &mg, nullptr);
}

int oracle_build_sel_mt(const uint8_t* residues, const uint64_t* seq_off, const uint32_t* seq_len,
                        const uint16_t* seq_func, const uint32_t* seq_id, uint64_t n_seqs, uint32_t n_functions,
                        int n_threads, int sel_bits, uint64_t sel, uint64_t* out_keys, oracle_stored* out_data,
                        uint64_t out_cap, uint64_t* out_n, uint32_t* distinct_functions, uint32_t* seqs_with_func,
                        uint64_t* n_seqs_with_signature, uint64_t* distinct_signatures, uint64_t* valid_windows,
                        uint64_t* max_group, uint8_t* seq_flags) {
    const int K = 8;
    auto selected = [sel_bits, sel](uint64_t key) {
        return sel_bits == 0 || (slice_hash(key) >> (64 - sel_bits)) == sel;
    };
    const int T = std::max(1, n_threads);
    const int S = 8 * T;  // shards
    auto shard_of = [S](uint64_t k) {
        k ^= k >> 33;
        k *= 0xff51afd7ed558ccdull;
        k ^= k >> 33;
        return (int)(k % (uint64_t)S);
    };
    // contiguous sequence ranges of ~equal residue count
    uint64_t total = 0;
    for (uint64_t s = 0; s < n_seqs; ++s) total += seq_len[s];
    std::vector<uint64_t> cut(T + 1, n_seqs);
    cut[0] = 0;
    {
        uint64_t acc = 0;
        int t = 1;
        for (uint64_t s = 0; s < n_seqs && t < T; ++s) {
            acc += seq_len[s];
            while (t < T && acc >= total * (uint64_t)t / (uint64_t)T) cut[t++] = s + 1;
        }
    }
    std::vector<std::vector<std::vector<Occ>>> parts(T, std::vector<std::vector<Occ>>(S));
    std::vector<std::vector<uint32_t>> swf(T, std::vector<uint32_t>(n_functions, 0));
    std::vector<uint64_t> nvalid(T, 0);
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t]() {
            uint64_t nv = 0;
            for (uint64_t s = cut[t]; s < cut[t + 1]; ++s) {
                const uint16_t f = seq_func[s];
                if (f == kUndefinedFunction) continue;
                if (f < n_functions) swf[t][f]++;
                const uint8_t* seq = residues + seq_off[s];
                const uint32_t len = seq_len[s];
                if (len < (uint32_t)K) continue;
                uint32_t run = 0;  // valid residues ending at i
                for (uint32_t i = 0; i < len; ++i) {
                    run = ok_prot(seq[i]) ? run + 1 : 0;
                    if (i + 1 >= (uint32_t)K && run >= (uint32_t)K) {
                        const uint32_t w = i + 1 - K;
                        const uint64_t key = load_key(seq + w);
                        ++nv;
                        if (selected(key)) parts[t][shard_of(key)].push_back({key, (uint32_t)s, w});
                    }
                }
            }
            nvalid[t] = nv;
        });
    for (auto& x : th) x.join();
    th.clear();
    struct ShardOut {
        std::vector<uint64_t> keys;
        std::vector<oracle_stored> data;
        std::vector<uint32_t> df;
        uint64_t n_sig = 0, max_group = 0;
    };
    std::vector<ShardOut> outs(S);
    std::vector<uint8_t> flag(n_seqs, 0);  // sequence has a kept k-mer
    std::atomic<int> next(0);
    for (int t = 0; t < T; ++t)
        th.emplace_back([&]() {
            std::vector<uint16_t> offsets;
            for (int sh; (sh = next.fetch_add(1)) < S;) {
                std::vector<Occ> occ;
                size_t n = 0;
                for (int u = 0; u < T; ++u) n += parts[u][sh].size();
                occ.reserve(n);
                for (int u = 0; u < T; ++u) {
                    occ.insert(occ.end(), parts[u][sh].begin(), parts[u][sh].end());
                    std::vector<Occ>().swap(parts[u][sh]);
                }
                std::stable_sort(occ.begin(), occ.end(), [](const Occ& a, const Occ& b) { return a.key < b.key; });
                ShardOut& O = outs[sh];
                O.df.assign(n_functions, 0);
                size_t a = 0;
                while (a < occ.size()) {
                    size_t b = a + 1;
                    while (b < occ.size() && occ[b].key == occ[a].key) ++b;
                    O.max_group = std::max<uint64_t>(O.max_group, b - a);
                    std::map<uint16_t, int> func_count;
                    int count = 0;
                    for (size_t j = b; j-- > a;) {
                        func_count[seq_func[occ[j].seq]]++;
                        count++;
                    }
                    uint16_t best_func = kUndefinedFunction;
                    int best_count = -1;
                    for (auto& x : func_count)
                        if (best_func == kUndefinedFunction || x.second > best_count) {
                            best_func = x.first;
                            best_count = x.second;
                        }
                    if (!((float)best_count < float(count) * 0.8f)) {
                        SigAcc acc;
                        offsets.clear();
                        for (size_t j = b; j-- > a;) {
                            const Occ& o = occ[j];
                            const uint32_t len = seq_len[o.seq];
                            if (seq_func[o.seq] == best_func) acc(len);
                            offsets.push_back((uint16_t)(len - o.i));
                            __atomic_store_n(&flag[o.seq], (uint8_t)1, __ATOMIC_RELAXED);
                        }
                        std::sort(offsets.begin(), offsets.end());
                        O.keys.push_back(occ[a].key);
                        O.data.push_back({offsets[offsets.size() / 2], best_func, d2u16(acc.mean()),
                                          d2u16(acc.median.result()), d2u16(acc.variance)});
                        O.n_sig++;
                        if (best_func < n_functions) O.df[best_func]++;
                    }
                    a = b;
                }
            }
        });
    for (auto& x : th) x.join();
    uint64_t kept = 0, n_sig = 0;
    for (uint32_t f = 0; f < n_functions; ++f) {
        distinct_functions[f] = 0;
        seqs_with_func[f] = 0;
        for (int t = 0; t < T; ++t) seqs_with_func[f] += swf[t][f];
    }
    uint64_t mg = 0;
    for (int sh = 0; sh < S; ++sh) {
        ShardOut& O = outs[sh];
        const uint64_t room = kept < out_cap ? out_cap - kept : 0;
        const uint64_t c = std::min<uint64_t>(room, O.keys.size());
        std::copy(O.keys.begin(), O.keys.begin() + c, out_keys + kept);
        std::copy(O.data.begin(), O.data.begin() + c, out_data + kept);
        kept += O.keys.size();
        n_sig += O.n_sig;
        mg = std::max(mg, O.max_group);
        for (uint32_t f = 0; f < n_functions; ++f) distinct_functions[f] += O.df[f];
    }
    uint64_t nv = 0;
    for (int t = 0; t < T; ++t) nv += nvalid[t];
    *valid_windows = nv;
    *max_group = mg;
    if (seq_flags) std::copy(flag.begin(), flag.end(), seq_flags);
    std::vector<uint32_t> ids;  // seqs_with_a_signature is a set of seq_ids (colliding ids count once)
    for (uint64_t s = 0; s < n_seqs; ++s)
        if (flag[s]) ids.push_back(seq_id[s]);
    std::sort(ids.begin(), ids.end());
    *out_n = kept;
    *n_seqs_with_signature = (uint64_t)(std::unique(ids.begin(), ids.end()) - ids.begin());
    *distinct_signatures = n_sig;
    return kept <= out_cap ? 0 : -1;
}

// Number of windows the build examines (units of the k-mers/s metric): sum over sequences with
// a kept function of max(0, len-7).
uint64_t oracle_count_windows(const uint32_t* seq_len, const uint16_t* seq_func, uint64_t n_seqs) {
    uint64_t w = 0;
    for (uint64_t s = 0; s < n_seqs; ++s)
        if (seq_func[s] != kUndefinedFunction && seq_len[s] >= 8) w += seq_len[s] - 7;
    return w;
}

// --------------------------------------------------------------------------------------------
//  CMPH BDZ (restated from cmph 2.0.x bdz.c / jenkins_hash.c; file layout of cmph_dump).
// --------------------------------------------------------------------------------------------
struct oracle_bdz {
    uint32_t m, n, r, k, ranktablesize, seed;
    uint8_t b;
    std::vector<uint8_t>* g;
    std::vector<uint32_t>* ranktable;
};

static inline void jenkins_mix(uint32_t& a, uint32_t& b, uint32_t& c) {
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

void oracle_jenkins_hash_vector(uint32_t seed, const uint8_t* k, uint32_t keylen, uint32_t* hashes) {
    uint32_t len = keylen, length = keylen;
    uint32_t a = 0x9e3779b9, b = 0x9e3779b9, c = seed;
    while (len >= 12) {
        a += ((uint32_t)k[0] + ((uint32_t)k[1] << 8) + ((uint32_t)k[2] << 16) + ((uint32_t)k[3] << 24));
        b += ((uint32_t)k[4] + ((uint32_t)k[5] << 8) + ((uint32_t)k[6] << 16) + ((uint32_t)k[7] << 24));
        c += ((uint32_t)k[8] + ((uint32_t)k[9] << 8) + ((uint32_t)k[10] << 16) + ((uint32_t)k[11] << 24));
        jenkins_mix(a, b, c);
        k += 12;
        len -= 12;
    }
    c += length;
    switch (len) {  // all cases fall through
        case 11: c += ((uint32_t)k[10] << 24); [[fallthrough]];
        case 10: c += ((uint32_t)k[9] << 16); [[fallthrough]];
        case 9: c += ((uint32_t)k[8] << 8); [[fallthrough]];
        case 8: b += ((uint32_t)k[7] << 24); [[fallthrough]];
        case 7: b += ((uint32_t)k[6] << 16); [[fallthrough]];
        case 6: b += ((uint32_t)k[5] << 8); [[fallthrough]];
        case 5: b += (uint8_t)k[4]; [[fallthrough]];
        case 4: a += ((uint32_t)k[3] << 24); [[fallthrough]];
        case 3: a += ((uint32_t)k[2] << 16); [[fallthrough]];
        case 2: a += ((uint32_t)k[1] << 8); [[fallthrough]];
        case 1: a += (uint8_t)k[0]; [[fallthrough]];
        default: break;
    }
    jenkins_mix(a, b, c);
    hashes[0] = a;
    hashes[1] = b;
    hashes[2] = c;
}

static inline uint32_t gval(const uint8_t* g, uint32_t i) { return (g[i >> 2] >> ((i & 3u) << 1)) & 3u; }

static uint8_t bdz_lookup_table(uint8_t byte) {  // number of assigned (!= 3) entries in a g byte
    uint8_t n = 0;
    for (int j = 0; j < 4; ++j)
        if (((byte >> (2 * j)) & 3u) != 3u) n++;
    return n;
}

// Parse a cmph_dump() BDZ image: "bdz\0", u32 size, u32 buflen, "jenkins\0"+u32 seed,
// u32 n, u32 m, u32 r, u8 g[ceil(n/4)], u32 k, u8 b, u32 ranktablesize, u32 ranktable[].
oracle_bdz* oracle_bdz_load(const uint8_t* buf, uint64_t len) {
    uint64_t p = 0;
    auto need = [&](uint64_t n) { return p + n <= len; };
    auto rd32 = [&](uint32_t& v) { if (!need(4)) return false; std::memcpy(&v, buf + p, 4); p += 4; return true; };
    std::string algo;
    while (p < len && buf[p] != 0) algo.push_back((char)buf[p++]);
    if (p >= len || algo != "bdz") return nullptr;
    p++;
    uint32_t size, buflen;
    if (!rd32(size) || !rd32(buflen) || !need(buflen)) return nullptr;
    std::string hname((const char*)buf + p);
    if (hname != "jenkins" || buflen != 12) return nullptr;
    uint32_t seed;
    std::memcpy(&seed, buf + p + 8, 4);
    p += buflen;
    oracle_bdz* h = new oracle_bdz();
    h->seed = seed;
    if (!rd32(h->n) || !rd32(h->m) || !rd32(h->r)) { delete h; return nullptr; }
    uint32_t sizeg = (uint32_t)std::ceil(h->n / 4.0);
    if (!need(sizeg)) { delete h; return nullptr; }
    h->g = new std::vector<uint8_t>(buf + p, buf + p + sizeg);
    p += sizeg;
    if (!rd32(h->k) || !need(1)) { delete h->g; delete h; return nullptr; }
    h->b = buf[p++];
    if (!rd32(h->ranktablesize) || !need(4ull * h->ranktablesize)) { delete h->g; delete h; return nullptr; }
    h->ranktable = new std::vector<uint32_t>(h->ranktablesize);
    std::memcpy(h->ranktable->data(), buf + p, 4ull * h->ranktablesize);
    (void)size;
    return h;
}

void oracle_bdz_free(oracle_bdz* h) {
    if (!h) return;
    delete h->g;
    delete h->ranktable;
    delete h;
}

uint32_t oracle_bdz_size(const oracle_bdz* h) { return h->m; }

// bdz_search: jenkins -> 3 vertices -> (g0+g1+g2)%3 -> rank(vertex).
uint32_t oracle_bdz_search(const oracle_bdz* h, const uint8_t* key, uint32_t keylen) {
    uint32_t hl[3];
    oracle_jenkins_hash_vector(h->seed, key, keylen, hl);
    const uint8_t* g = h->g->data();
    hl[0] = hl[0] % h->r;
    hl[1] = hl[1] % h->r + h->r;
    hl[2] = hl[2] % h->r + (h->r << 1);
    uint32_t vertex = hl[(gval(g, hl[0]) + gval(g, hl[1]) + gval(g, hl[2])) % 3];
    // rank()
    uint32_t index = vertex >> h->b;
    uint32_t base_rank = (*h->ranktable)[index];
    uint32_t beg_idx_v = index << h->b;
    uint32_t beg_idx_b = beg_idx_v >> 2;
    uint32_t end_idx_b = vertex >> 2;
    while (beg_idx_b < end_idx_b) base_rank += bdz_lookup_table(g[beg_idx_b++]);
    beg_idx_v = beg_idx_b << 2;
    while (beg_idx_v < vertex) {
        if (gval(g, beg_idx_v) != 3u) base_rank++;
        beg_idx_v++;
    }
    return base_rank;
}

void oracle_bdz_search_keys(const oracle_bdz* h, const uint64_t* keys, uint64_t n, uint32_t* out) {
    for (uint64_t i = 0; i < n; ++i) {
        uint8_t kb[8];
        std::memcpy(kb, &keys[i], 8);
        out[i] = oracle_bdz_search(h, kb, 8);
    }
}

// --------------------------------------------------------------------------------------------
//  Function calling: for_each_kmer (kmer_data.h:76-102) + FunctionCaller::process_aa_seq
//  (call_functions.tcc:259-338) + HitSet::process (:35-103) against a CmphKmerDb
//  (cmph_kmer.h:139-147: idx = bdz_search; idx >= m is a miss; NO key verification).
// --------------------------------------------------------------------------------------------
struct oracle_annot_opts {
    int32_t min_hits;       // 5  (call_functions.h:66)
    int32_t max_gap;        // 200
    int32_t ignore_hypo;    // --ignore-hypo
    int32_t hypo_index;     // index of "hypothetical protein" in function.index
    int32_t mean_mode;      // 0: Boost.Math >=1.76 4-lane mean, 1: single running mean (<=1.75)
    int32_t mad_mode;       // 0: |x(mid) - median| (corrected MAD), 1: legacy abs(x(mid))
};

namespace {

struct Hit {
    oracle_stored kdata;
    unsigned long pos;
};

// Boost.Math statistics::mean(std::vector<float>)
float bm_mean(const std::vector<float>& v, int mode) {
    if (mode == 1) {
        float mu = 0, i = 1;
        for (float x : v) {
            mu = mu + (x - mu) / i;
            i += 1;
        }
        return mu;
    }
    const size_t elements = v.size();
    float mu[4] = {0, 0, 0, 0};
    float i = 1;
    size_t it = 0;
    const size_t end = elements - (elements % 4);
    while (it != end) {
        const float inv = 1.0f / i;
        float temp[4] = {v[it], v[it + 1], v[it + 2], v[it + 3]};
        for (int j = 0; j < 4; ++j) temp[j] -= mu[j];
        for (int j = 0; j < 4; ++j) temp[j] *= inv;
        for (int j = 0; j < 4; ++j) mu[j] += temp[j];
        i += 1;
        it += 4;
    }
    const float num1 = float(elements - (elements % 4)) / float(4);
    const float num2 = num1 + float(elements % 4);
    while (it != elements) {
        mu[3] += (v[it] - mu[3]) / i;
        i += 1;
        ++it;
    }
    return (num1 * (mu[0] + mu[1] + mu[2]) + num2 * mu[3]) / float(elements);
}

float bm_median(std::vector<float>& v) {
    size_t n = v.size();
    if (n & 1) {
        auto middle = v.begin() + (n - 1) / 2;
        std::nth_element(v.begin(), middle, v.end());
        return *middle;
    }
    auto middle = v.begin() + n / 2 - 1;
    std::nth_element(v.begin(), middle, v.end());
    std::nth_element(middle, middle + 1, v.end());
    return (*middle + *(middle + 1)) / 2;
}

float bm_mad(std::vector<float>& v, int mode) {
    float center = bm_median(v);
    size_t n = v.size();
    auto comparator = [&center](float a, float b) { return std::abs(a - center) < std::abs(b - center); };
    if (n & 1) {
        auto middle = v.begin() + (n - 1) / 2;
        std::nth_element(v.begin(), middle, v.end(), comparator);
        return mode == 1 ? std::abs(*middle) : std::abs(*middle - center);
    }
    auto middle = v.begin() + n / 2 - 1;
    std::nth_element(v.begin(), middle, v.end(), comparator);
    std::nth_element(middle, middle + 1, v.end(), comparator);
    if (mode == 1) return (std::abs(*middle) + std::abs(*(middle + 1))) / std::abs(2.0f);
    return (std::abs(*middle - center) + std::abs(*(middle + 1) - center)) / std::abs(2.0f);
}

void hitset_process(std::vector<Hit>& hits, double seqlen, uint16_t& current_fI,
                    std::vector<oracle_call>& calls, const oracle_annot_opts& o) {
    int fI_count = 0;
    size_t last_hit = 0;
    std::vector<float> protein_lengths;
    for (size_t h = 0; h < hits.size(); ++h) {
        if (hits[h].kdata.function_index == current_fI) {
            last_hit = h;
            fI_count++;
            protein_lengths.push_back(static_cast<float>(hits[h].kdata.mean));
        }
    }
    float mean_length = bm_mean(protein_lengths, o.mean_mode);
    float median_length = bm_median(protein_lengths);
    float mad_length = bm_mad(protein_lengths, o.mad_mode);
    if (mad_length == 0) mad_length = 30;
    double cutoff_b = mean_length - 2.0 * mad_length;
    double cutoff_t = mean_length + 2.0 * mad_length;
    if (fI_count >= o.min_hits) {
        if (!(seqlen < cutoff_b || seqlen > cutoff_t)) {
            calls.push_back({static_cast<unsigned int>(hits[0].pos),
                             static_cast<unsigned int>(hits[last_hit].pos + (8 - 1)), fI_count, current_fI, 0,
                             static_cast<unsigned int>(median_length), mad_length});
        }
    }
    auto end = hits.rbegin();
    if (end[1].kdata.function_index != current_fI && end[1].kdata.function_index == end[0].kdata.function_index) {
        current_fI = end[1].kdata.function_index;
        hits.erase(hits.begin(), hits.end() - 2);
    } else {
        hits.clear();
    }
}

}  // namespace

// One query sequence.  Returns the number of calls written (<= cap) or the needed count.
}  // extern "C"

// for_each_kmer<8> (kmer_data.h:76-102): only upper-case 'X' and '*' are ambiguous; a window is
// skipped when the next ambiguous byte lies inside it OR right after it (kend >= next_ambig,
// :90), then the scan restarts after that byte (:93).  cb(ptr, offset) per yielded window.
template <class CB>
static void for_each_kmer8(const uint8_t* seq, uint32_t len, CB cb) {
    const int N = 8;
    const uint8_t* ptr = seq;
    const uint8_t* end = seq + len;
    auto is_ambig = [](uint8_t c) { return c == '*' || c == 'X'; };
    auto find_ambig = [&](const uint8_t* from) {
        while (from < end && !is_ambig(*from)) ++from;
        return from;
    };
    const uint8_t* next_ambig = find_ambig(ptr);
    // last_kmer = end - N (pointer compare; no windows when len < N)
    while (len >= (uint32_t)N && ptr <= end - N) {
        const uint8_t* kend = ptr + N;
        if (next_ambig != end && kend >= next_ambig) {
            ptr = next_ambig + 1;
            next_ambig = find_ambig(ptr);
            continue;
        }
        cb(ptr, (size_t)(ptr - seq));
        ptr++;
    }
}

// fetch(ptr) -> const oracle_stored* or nullptr: CmphKmerDb::fetch (idx >= size -> no callback,
// cmph_kmer.h:139-147) or KeptKmerDB::fetch (exact key, kept_kmer_db.h:20-27).
template <class Fetch>
static int64_t process_aa_seq_impl(Fetch fetch, const uint8_t* seq, uint32_t len, const oracle_annot_opts* opts,
                                   oracle_call* out, uint64_t cap) {
    std::vector<Hit> hits;
    std::vector<oracle_call> calls;
    uint16_t current_fI = kUndefinedFunction;
    double seqlen = static_cast<double>(len);
    for_each_kmer8(seq, len, [&](const uint8_t* ptr, size_t offset) {
        const oracle_stored* kp = fetch(ptr);
        if (kp) {
            const oracle_stored& kdata = *kp;
            bool skip = opts->ignore_hypo && kdata.function_index == (uint16_t)opts->hypo_index &&
                        opts->hypo_index >= 0;
            if (!skip) {
                if (!hits.empty() && hits.back().pos + (unsigned long)opts->max_gap < offset) {
                    if ((int)hits.size() >= opts->min_hits)
                        hitset_process(hits, seqlen, current_fI, calls, *opts);
                    else
                        hits.clear();
                }
                if (hits.empty()) current_fI = kdata.function_index;
                hits.push_back({kdata, offset});
                if (hits.size() > 1 && current_fI != kdata.function_index) {
                    auto e = hits.rbegin();
                    if (e[1].kdata.function_index == e[0].kdata.function_index)
                        hitset_process(hits, seqlen, current_fI, calls, *opts);
                }
            }
        }
    });
    if ((int)hits.size() >= opts->min_hits) hitset_process(hits, seqlen, current_fI, calls, *opts);
    for (size_t i = 0; i < calls.size() && i < cap; ++i) out[i] = calls[i];
    return (int64_t)calls.size();
}

extern "C" {

// The offsets for_each_kmer8 yields over one sequence (out: room for len entries); returns the
// count.  Pinned against the reference's own for_each_kmer<8> (tests/golden/ref_windows.npz).
uint32_t oracle_kmer_windows(const uint8_t* seq, uint32_t len, uint32_t* out) {
    uint32_t n = 0;
    for_each_kmer8(seq, len, [&](const uint8_t*, size_t off) { out[n++] = (uint32_t)off; });
    return n;
}

int64_t oracle_process_aa_seq(const oracle_bdz* db, const oracle_stored* dat, const uint8_t* seq,
                              uint32_t len, const oracle_annot_opts* opts, oracle_call* out, uint64_t cap) {
    auto fetch = [&](const uint8_t* k) -> const oracle_stored* {
        uint32_t idx = oracle_bdz_search(db, k, 8);
        return idx < db->m ? &dat[idx] : nullptr;
    };
    return process_aa_seq_impl(fetch, seq, len, opts, out, cap);
}

// Recall pass against the exact kept-k-mer DB (kmers-build-signatures.cc:238-349): keys sorted
// ascending (as oracle_build returns them), data[i] the record of keys[i].
int64_t oracle_annotate_exact(const uint64_t* keys, const oracle_stored* data, uint64_t nkeys, const uint8_t* residues,
                              const uint64_t* seq_off, const uint32_t* seq_len, uint64_t n_seqs,
                              const oracle_annot_opts* opts, uint64_t* call_off, oracle_call* calls, uint64_t cap) {
    auto fetch = [&](const uint8_t* k) -> const oracle_stored* {
        uint64_t key = load_key(k);
        const uint64_t* it = std::lower_bound(keys, keys + nkeys, key);
        return (it != keys + nkeys && *it == key) ? &data[it - keys] : nullptr;
    };
    uint64_t total = 0;
    std::vector<oracle_call> tmp(1024);
    for (uint64_t s = 0; s < n_seqs; ++s) {
        call_off[s] = total;
        int64_t n = process_aa_seq_impl(fetch, residues + seq_off[s], seq_len[s], opts, tmp.data(), tmp.size());
        if ((uint64_t)n > tmp.size()) {
            tmp.resize(n);
            n = process_aa_seq_impl(fetch, residues + seq_off[s], seq_len[s], opts, tmp.data(), tmp.size());
        }
        for (int64_t i = 0; i < n; ++i) {
            if (total < cap) calls[total] = tmp[i];
            total++;
        }
    }
    call_off[n_seqs] = total;
    return total <= cap ? (int64_t)total : -1;
}

// Batch form: CSR output (call_off has n_seqs+1 entries).  Returns total calls or -1 if cap short.
int64_t oracle_annotate(const oracle_bdz* db, const oracle_stored* dat, const uint8_t* residues,
                        const uint64_t* seq_off, const uint32_t* seq_len, uint64_t n_seqs,
                        const oracle_annot_opts* opts, uint64_t* call_off, oracle_call* calls, uint64_t cap) {
    uint64_t total = 0;
    std::vector<oracle_call> tmp(1024);
    for (uint64_t s = 0; s < n_seqs; ++s) {
        call_off[s] = total;
        int64_t n = oracle_process_aa_seq(db, dat, residues + seq_off[s], seq_len[s], opts, tmp.data(), tmp.size());
        if ((uint64_t)n > tmp.size()) {
            tmp.resize(n);
            n = oracle_process_aa_seq(db, dat, residues + seq_off[s], seq_len[s], opts, tmp.data(), tmp.size());
        }
        for (int64_t i = 0; i < n; ++i) {
            if (total < cap) calls[total] = tmp[i];
            total++;
        }
    }
    call_off[n_seqs] = total;
    return total <= cap ? (int64_t)total : -1;
}

// The call path on n_threads host threads (bench.py's CPU baseline of the annotate leg): each
// thread runs process_aa_seq over a contiguous range of sequences (the reference parallelises
// over files, kmers-call-functions.cc:166-189; here one batch is split).  Returns the number of
// calls (the calls themselves are computed and dropped).
int64_t oracle_annotate_mt(const oracle_bdz* db, const oracle_stored* dat, const uint8_t* residues,
                           const uint64_t* seq_off, const uint32_t* seq_len, uint64_t n_seqs,
                           const oracle_annot_opts* opts, int n_threads) {
    const int T = std::max(1, n_threads);
    std::vector<int64_t> cnt(T, 0);
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t]() {
            std::vector<oracle_call> tmp(1024);
            const uint64_t s0 = n_seqs * (uint64_t)t / (uint64_t)T, s1 = n_seqs * (uint64_t)(t + 1) / (uint64_t)T;
            for (uint64_t s = s0; s < s1; ++s) {
                int64_t n = oracle_process_aa_seq(db, dat, residues + seq_off[s], seq_len[s], opts, tmp.data(), tmp.size());
                if ((uint64_t)n > tmp.size()) {
                    tmp.resize(n);
                    n = oracle_process_aa_seq(db, dat, residues + seq_off[s], seq_len[s], opts, tmp.data(), tmp.size());
                }
                cnt[t] += n;
            }
        });
    for (auto& x : th) x.join();
    int64_t total = 0;
    for (int64_t c : cnt) total += c;
    return total;
}

// --------------------------------------------------------------------------------------------
//  kmers-matrix-distance (kmers-matrix-distance.cc:94-212; MatrixDistance::compute,
//  matrix_distance.h:45-170).  process_fasta_stream_parallel (call_functions.tcc:157-215) runs
//  process_aa_seq with ignore_hypothetical(true) (:164), so hit_cb (:123-152) sees every window of
//  for_each_kmer whose record is not "hypothetical protein" (call_functions.tcc:285-291):
//     stddev = var == 0 ? seqlen * 0.1 : sqrt(var);  keep iff mean - 2 sd <= seqlen <= mean + 2 sd
//  and inserts the sequence's SeqIdMap index (seq_id_map.h:12-27) into kmer_hit_map[kmer] (a set:
//  one entry per (kmer, index)).  Then for every k-mer and every id1 < id2 of its set
//  seq_dist[id1][id2]++ (:176-196).  The HitSet / find_best_call results do not feed the matrix.
//  seq_idx[s]: the SeqIdMap index of sequence s (first occurrence of its id).  Output: (id1, id2,
//  count) triples sorted by (id1, id2) (the reference prints hash order; compare as sets).
//  Returns the number of pairs (writes at most cap).
// --------------------------------------------------------------------------------------------
int64_t oracle_matrix_distance(const oracle_bdz* db, const oracle_stored* dat, const uint8_t* residues,
                               const uint64_t* seq_off, const uint32_t* seq_len, const uint32_t* seq_idx,
                               uint64_t n_seqs, int32_t hypo_index, uint32_t* out, uint64_t cap) {
    std::map<uint64_t, std::vector<uint32_t>> hit_map;  // kmer -> indices (deduplicated below)
    for (uint64_t s = 0; s < n_seqs; ++s) {
        const double seqlen = static_cast<double>(seq_len[s]);
        for_each_kmer8(residues + seq_off[s], seq_len[s], [&](const uint8_t* ptr, size_t) {
            const uint32_t idx = oracle_bdz_search(db, ptr, 8);
            if (idx >= db->m) return;  // fetch: no callback on a miss (cmph_kmer.h:143-146)
            const oracle_stored& kd = dat[idx];
            if (hypo_index >= 0 && kd.function_index == (uint16_t)hypo_index) return;
            const double mean = static_cast<double>(kd.mean);
            const double stddev = kd.var == 0 ? seqlen * 0.1 : std::sqrt(static_cast<double>(kd.var));
            const double cutoff_b = mean - stddev * 2.0;
            const double cutoff_t = mean + stddev * 2.0;
            if (seqlen < cutoff_b || seqlen > cutoff_t) return;
            hit_map[load_key(ptr)].push_back(seq_idx[s]);
        });
    }
    std::map<std::pair<uint32_t, uint32_t>, uint32_t> dist;
    for (auto& kv : hit_map) {
        std::vector<uint32_t>& v = kv.second;
        std::sort(v.begin(), v.end());
        v.erase(std::unique(v.begin(), v.end()), v.end());
        for (size_t a = 0; a < v.size(); ++a)
            for (size_t b = a + 1; b < v.size(); ++b) dist[{v[a], v[b]}]++;
    }
    uint64_t n = 0;
    for (auto& kv : dist) {
        if (n < cap) {
            out[3 * n] = kv.first.first;
            out[3 * n + 1] = kv.first.second;
            out[3 * n + 2] = kv.second;
        }
        ++n;
    }
    return (int64_t)n;
}

// The same pair counts on n_threads host threads (bench.py's CPU baseline of the matrix leg; the
// reference fills kmer_hit_map from process_fasta_stream_parallel's TBB tasks, matrix_distance.h
// :130-143).  (1) threads over sequence ranges collect (kmer, index) hits; (2) threads over k-mer
// hash shards dedupe each k-mer's index set and emit its id1 < id2 pair keys; (3) threads over
// id1 shards sort and run-length count the pair keys.  out != nullptr: the pairs sorted by
// (id1, id2), as oracle_matrix_distance.  Returns the number of pairs (writes at most cap).
int64_t oracle_matrix_distance_mt(const oracle_bdz* db, const oracle_stored* dat, const uint8_t* residues,
                                  const uint64_t* seq_off, const uint32_t* seq_len, const uint32_t* seq_idx,
                                  uint64_t n_seqs, int32_t hypo_index, uint32_t* out, uint64_t cap, int n_threads) {
    const int T = std::max(1, n_threads);
    auto shard_of = [T](uint64_t k) { return (int)(((k * 0x9E3779B97F4A7C15ull) >> 40) % (uint64_t)T); };
    // (1) hits, bucketed by k-mer shard per producing thread
    std::vector<std::vector<std::vector<std::pair<uint64_t, uint32_t>>>> hits(T, std::vector<std::vector<std::pair<uint64_t, uint32_t>>>(T));
    {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t]() {
                const uint64_t s0 = n_seqs * (uint64_t)t / (uint64_t)T, s1 = n_seqs * (uint64_t)(t + 1) / (uint64_t)T;
                for (uint64_t s = s0; s < s1; ++s) {
                    const double seqlen = static_cast<double>(seq_len[s]);
                    for_each_kmer8(residues + seq_off[s], seq_len[s], [&](const uint8_t* ptr, size_t) {
                        const uint32_t idx = oracle_bdz_search(db, ptr, 8);
                        if (idx >= db->m) return;
                        const oracle_stored& kd = dat[idx];
                        if (hypo_index >= 0 && kd.function_index == (uint16_t)hypo_index) return;
                        const double mean = static_cast<double>(kd.mean);
                        const double stddev = kd.var == 0 ? seqlen * 0.1 : std::sqrt(static_cast<double>(kd.var));
                        if (seqlen < mean - stddev * 2.0 || seqlen > mean + stddev * 2.0) return;
                        const uint64_t k = load_key(ptr);
                        hits[t][shard_of(k)].emplace_back(k, seq_idx[s]);
                    });
                }
            });
        for (auto& x : th) x.join();
    }
    // (2) per k-mer shard: group, dedupe, emit pair keys bucketed by id1 shard
    std::vector<std::vector<std::vector<uint64_t>>> pairs(T, std::vector<std::vector<uint64_t>>(T));
    {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t]() {
                std::vector<std::pair<uint64_t, uint32_t>> v;
                for (int p = 0; p < T; ++p) v.insert(v.end(), hits[p][t].begin(), hits[p][t].end());
                for (int p = 0; p < T; ++p) std::vector<std::pair<uint64_t, uint32_t>>().swap(hits[p][t]);
                std::sort(v.begin(), v.end());
                v.erase(std::unique(v.begin(), v.end()), v.end());
                for (size_t a = 0; a < v.size();) {
                    size_t e = a;
                    while (e < v.size() && v[e].first == v[a].first) ++e;
                    for (size_t i = a; i < e; ++i)
                        for (size_t j = i + 1; j < e; ++j)
                            pairs[t][v[i].second % (uint32_t)T].push_back(((uint64_t)v[i].second << 32) | v[j].second);
                    a = e;
                }
            });
        for (auto& x : th) x.join();
    }
    // (3) per id1 shard: count
    std::vector<std::vector<std::pair<uint64_t, uint32_t>>> cnt(T);
    {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t]() {
                std::vector<uint64_t> v;
                for (int p = 0; p < T; ++p) {
                    v.insert(v.end(), pairs[p][t].begin(), pairs[p][t].end());
                    std::vector<uint64_t>().swap(pairs[p][t]);
                }
                std::sort(v.begin(), v.end());
                for (size_t a = 0; a < v.size();) {
                    size_t e = a;
                    while (e < v.size() && v[e] == v[a]) ++e;
                    cnt[t].emplace_back(v[a], (uint32_t)(e - a));
                    a = e;
                }
            });
        for (auto& x : th) x.join();
    }
    uint64_t n = 0;
    for (auto& c : cnt) n += c.size();
    if (out) {
        std::vector<std::pair<uint64_t, uint32_t>> all;
        all.reserve(n);
        for (auto& c : cnt) all.insert(all.end(), c.begin(), c.end());
        std::sort(all.begin(), all.end());
        for (uint64_t i = 0; i < n && i < cap; ++i) {
            out[3 * i] = (uint32_t)(all[i].first >> 32);
            out[3 * i + 1] = (uint32_t)all[i].first;
            out[3 * i + 2] = all[i].second;
        }
    }
    return (int64_t)n;
}

// --------------------------------------------------------------------------------------------
//  find_best_call (call_functions.tcc:347-659).  function_index: array of nfunc C strings
//  (function.index column 1).  Writes the called function string (NUL-terminated) into out_func.
// --------------------------------------------------------------------------------------------
static std::vector<std::string> split_str(const std::string& s, const std::string& delim) {
    std::vector<std::string> result;  // operators.h:183-194
    size_t start = 0;
    std::string::size_type e = 0;
    while (e != std::string::npos) {
        e = s.find(delim, start);
        result.push_back(s.substr(start, e - start));
        start = e + delim.length();
    }
    return result;
}

// split (operators.h:80-91) as the tests see it: the parts' [begin, end) byte ranges of s into
// se[2 * k], se[2 * k + 1] for k < cap; returns the number of parts (pinned by ref_split.npz)
extern "C" uint64_t oracle_split(const char* s, uint64_t n, const char* d, uint64_t dn, uint64_t* se, uint64_t cap) {
    const std::string str(s ? s : "", n), delim(d ? d : "", dn);
    const std::vector<std::string> parts = split_str(str, delim);
    uint64_t pos = 0;
    for (uint64_t k = 0; k < parts.size(); ++k) {
        if (k < cap) {
            se[2 * k] = pos;
            se[2 * k + 1] = pos + parts[k].size();
        }
        pos += parts[k].size() + delim.size();
    }
    return parts.size();
}

void oracle_find_best_call(const oracle_call* calls_in, uint64_t ncalls, const char* const* function_index,
                           uint64_t nfunc, uint16_t* out_fi, float* out_score, float* out_offset,
                           char* out_func, uint64_t out_func_cap) {
    auto function_at_index = [&](int idx) -> std::string {
        if (idx == kUndefinedFunction) return "";
        if (idx < 0 || (uint64_t)idx >= nfunc) return "";
        return function_index[idx];
    };
    uint16_t function_index_r = kUndefinedFunction;
    std::string function;
    float score = 0.0;
    float score_offset = 0.0;
    auto finish = [&]() {
        *out_fi = function_index_r;
        *out_score = score;
        *out_offset = score_offset;
        if (out_func_cap) {
            size_t n = std::min<size_t>(function.size(), out_func_cap - 1);
            std::memcpy(out_func, function.data(), n);
            out_func[n] = 0;
        }
    };
    std::vector<oracle_call> calls(calls_in, calls_in + ncalls);
    if (calls.empty()) { finish(); return; }
    std::vector<oracle_call> collapsed;
    auto comp = calls.begin();
    while (comp != calls.end()) {
        collapsed.push_back(*comp);
        comp++;
        oracle_call& cur = collapsed.back();
        while (comp != calls.end() && cur.function_index == comp->function_index) {
            cur.end = comp->end;
            cur.count += comp->count;
            comp++;
        }
    }
    std::vector<oracle_call> merged;
    const int merge_interior_thresh = 5, merge_exterior_thresh = 10;
    comp = collapsed.begin();
    while (comp != collapsed.end()) {
        merged.push_back(*comp);
        comp++;
        auto comp2 = comp + 1;
        oracle_call& cur = merged.back();
        while (comp != collapsed.end() && comp2 != collapsed.end() && cur.function_index == comp2->function_index &&
               comp->count < merge_interior_thresh && (cur.count + comp2->count) >= merge_exterior_thresh) {
            cur.end = comp2->end;
            cur.count += comp2->count;
            comp += 2;
            comp2 = comp + 1;
        }
    }
    if (merged.size() > 1) {
        char next_func_key = 'A';
        char next_fusion_key = 'W';
        std::map<std::string, char> func_map, fusion_map;
        std::map<char, std::pair<uint16_t, std::string>> key_to_function_info;
        struct FAcc { size_t n = 0; float sum = 0; };   // accumulator_set<float, mean, variance>
        std::map<char, FAcc> part_stats;
        std::string exp;
        int sum_scores = 0;
        for (auto c : merged) {
            sum_scores += c.count;
            std::string func = function_at_index(c.function_index);
            std::vector<std::string> parts = split_str(func, " / ");
            std::string fusion_key;
            for (auto& part : parts) {
                if (func_map.find(part) == func_map.end()) {
                    char f = next_func_key++;
                    func_map[part] = f;
                }
                fusion_key += func_map[part];
            }
            if (parts.size() > 1) {
                if (fusion_map.find(fusion_key) == fusion_map.end()) fusion_map[fusion_key] = next_fusion_key++;
                char fkey = fusion_map[fusion_key];
                exp += fkey;
                FAcc& fa = part_stats[fkey];
                fa.n++;
                fa.sum += static_cast<float>(c.protein_length_median);
                key_to_function_info[fkey] = std::make_pair(c.function_index, func);
            } else {
                exp += func_map[func];
                FAcc& fa = part_stats[func_map[func]];
                fa.n++;
                fa.sum += static_cast<float>(c.protein_length_median);
                key_to_function_info[func_map[func]] = std::make_pair(c.function_index, func);
            }
        }
        static const std::regex fusion_re("^W?A[A|W]*W[B|W]*BW?");
        if (std::regex_match(exp, fusion_re)) {
            auto accmean = [&](char k) { FAcc& f = part_stats[k]; return f.sum / (float)f.n; };
            float a_mean = accmean('A');
            float w_mean = accmean('W');
            float b_mean = accmean('B');
            float diff = (a_mean + b_mean) - w_mean;
            float frac_dif = std::abs(diff) / w_mean;
            if (frac_dif < 0.1) {
                function_index_r = key_to_function_info['W'].first;
                function = key_to_function_info['W'].second;
                score = (float)sum_scores;
                score_offset = 0.0;
                finish();
                return;
            }
        }
    }
    std::map<int, int> by_func;
    for (auto c : merged) {
        auto it = by_func.find(c.function_index);
        if (it == by_func.end())
            by_func.insert(std::make_pair((int)c.function_index, c.count));
        else
            it->second += c.count;
    }
    typedef std::pair<uint16_t, int> ent_t;
    std::vector<ent_t> vec;
    for (auto it = by_func.begin(); it != by_func.end(); it++) vec.push_back(*it);
    if (vec.size() > 1) {
        std::partial_sort(vec.begin(), vec.begin() + 2, vec.end(),
                          [](const ent_t& s1, const ent_t& s2) { return (s1.second > s2.second); });
    }
    if (vec.size() == 1)
        score_offset = (float)vec[0].second;
    else
        score_offset = (float)(vec[0].second - vec[1].second);
    if (score_offset >= 5.0) {
        auto best = vec[0];
        function_index_r = best.first;
        function = function_at_index(function_index_r);
        score = (float)best.second;
    } else {
        function_index_r = kUndefinedFunction;
        function = "";
        score = 0.0;
        if (vec.size() >= 2) {
            std::string f1 = function_at_index(vec[0].first);
            std::string f2 = function_at_index(vec[1].first);
            if (f2 > f1) std::swap(f1, f2);
            if (vec.size() == 2) {
                function = f1 + " ?? " + f2;
                score = (float)vec[0].second;
            } else if (vec.size() > 2) {
                float pair_offset = (float)(vec[1].second - vec[2].second);
                if (pair_offset > 2.0) {
                    function = f1 + " ?? " + f2;
                    score = (float)vec[0].second;
                    score_offset = pair_offset;
                }
            }
        }
    }
    finish();
}

}  // extern "C"
