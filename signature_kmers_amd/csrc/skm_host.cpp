// skm_host.cpp -- host-side pieces of libskm that stay on the CPU in the reference design:
// error state, version, and find_best_call (call_functions.tcc:347-659: collapse, F1-F2-F1 merge,
// fusion detection, best-vs-second margin, "f1 ?? f2" fallback).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "skm_strutil.h"
#include "skm_util.h"

namespace skm {

static thread_local std::string g_last_error;
void set_last_error(const std::string& msg) { g_last_error = msg; }

namespace {

// Matcher for boost::regex("^W?A[A|W]*W[B|W]*BW?") under regex_match (whole string).
// Character classes include '|'.  Implemented as the NFA it denotes.
bool fusion_pattern(const std::string& s) {
    // states: 0 start, 1 after optional W (pre-A), 2 in [A|W]* after A, 3 in [B|W]* after W,
    // 4 after B, 5 after trailing W (accepting: 4, 5)
    std::vector<int> cur = {0}, nxt;
    auto add = [&](std::vector<int>& v, int st) {
        if (std::find(v.begin(), v.end(), st) == v.end()) v.push_back(st);
    };
    // epsilon: state 0 can skip the optional W -> state 1
    add(cur, 1);
    for (char c : s) {
        nxt.clear();
        for (int st : cur) {
            switch (st) {
                case 0:
                    if (c == 'W') add(nxt, 1);
                    break;
                case 1:
                    if (c == 'A') add(nxt, 2);
                    break;
                case 2:  // [A|W]* then mandatory W
                    if (c == 'A' || c == '|' || c == 'W') add(nxt, 2);
                    if (c == 'W') add(nxt, 3);
                    break;
                case 3:  // [B|W]* then mandatory B
                    if (c == 'B' || c == '|' || c == 'W') add(nxt, 3);
                    if (c == 'B') add(nxt, 4);
                    break;
                case 4:
                    if (c == 'W') add(nxt, 5);
                    break;
                default:
                    break;
            }
        }
        std::swap(cur, nxt);
        if (cur.empty()) return false;
    }
    for (int st : cur)
        if (st == 4 || st == 5) return true;
    return false;
}

}  // namespace
}  // namespace skm

using namespace skm;

extern "C" {

const char* skm_last_error(void) { return g_last_error.c_str(); }
const char* skm_version(void) { return "signature_kmers_amd 0.1 (gfx950)"; }

int skm_device_count(int* n) {
    SKM_API_BEGIN
    SKM_CHECK(n, SKM_E_ARG, "null argument");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    *n = e == hipSuccess ? c : 0;
    SKM_API_END
}

int skm_find_best_call(const skm_kmer_call* calls_in, size_t ncalls, const char* const* function_index, size_t nfunc,
                       uint16_t* out_fi, float* out_score, float* out_offset, char* out_func, size_t out_func_cap) {
    SKM_API_BEGIN
    SKM_CHECK(out_fi && out_score && out_offset, SKM_E_ARG, "null output");
    auto fname = [&](uint32_t idx) -> std::string {
        if (idx == SKM_UNDEFINED_FUNCTION || idx >= nfunc || !function_index || !function_index[idx]) return "";
        return function_index[idx];
    };
    uint16_t fi = SKM_UNDEFINED_FUNCTION;
    std::string func;
    float score = 0.0f, score_offset = 0.0f;
    auto emit = [&]() {
        *out_fi = fi;
        *out_score = score;
        *out_offset = score_offset;
        if (out_func && out_func_cap) {
            size_t n = std::min(func.size(), out_func_cap - 1);
            std::memcpy(out_func, func.data(), n);
            out_func[n] = 0;
        }
    };
    if (ncalls == 0) {
        emit();
        return SKM_OK;
    }
    // 1. collapse runs of the same function (end and count accumulate)
    std::vector<skm_kmer_call> collapsed;
    for (size_t i = 0; i < ncalls; ++i) {
        if (!collapsed.empty() && collapsed.back().function_index == calls_in[i].function_index) {
            collapsed.back().end = calls_in[i].end;
            collapsed.back().count += calls_in[i].count;
        } else {
            collapsed.push_back(calls_in[i]);
        }
    }
    // 2. F1 F2 F1 with F2.count < 5 and F1+F1 >= 10: drop F2, merge the F1s
    std::vector<skm_kmer_call> merged;
    for (size_t i = 0; i < collapsed.size();) {
        merged.push_back(collapsed[i]);
        skm_kmer_call& cur = merged.back();
        size_t j = i + 1;
        while (j < collapsed.size() && j + 1 < collapsed.size() &&
               cur.function_index == collapsed[j + 1].function_index && collapsed[j].count < 5 &&
               cur.count + collapsed[j + 1].count >= 10) {
            cur.end = collapsed[j + 1].end;
            cur.count += collapsed[j + 1].count;
            j += 2;
        }
        i = j;
    }
    // 3. fusion calls
    if (merged.size() > 1) {
        char next_func_key = 'A', next_fusion_key = 'W';
        std::map<std::string, char> func_key, fusion_key_map;
        std::map<char, std::pair<uint16_t, std::string>> key_info;
        std::map<char, std::pair<size_t, float>> part;  // accumulator_set<float, mean>: (count, sum)
        std::string exp;
        int sum_scores = 0;
        for (const auto& c : merged) {
            sum_scores += c.count;
            std::string f = fname(c.function_index);
            std::vector<std::string> parts = skm_str::split(f, " / ");  // call_functions.tcc:487
            std::string fk;
            for (const auto& p : parts) {
                if (!func_key.count(p)) func_key[p] = next_func_key++;
                fk += func_key[p];
            }
            char key;
            if (parts.size() > 1) {
                if (!fusion_key_map.count(fk)) fusion_key_map[fk] = next_fusion_key++;
                key = fusion_key_map[fk];
            } else {
                key = func_key[f];
            }
            exp += key;
            auto& acc = part[key];
            acc.first += 1;
            acc.second += static_cast<float>(c.protein_length_median);
            key_info[key] = std::make_pair(c.function_index, f);
        }
        if (fusion_pattern(exp)) {
            auto mean = [&](char k) {
                auto& a = part[k];
                return a.second / (float)a.first;
            };
            const float a_mean = mean('A'), w_mean = mean('W'), b_mean = mean('B');
            const float diff = (a_mean + b_mean) - w_mean;
            const float frac_dif = std::fabs(diff) / w_mean;
            if (frac_dif < 0.1) {
                fi = key_info['W'].first;
                func = key_info['W'].second;
                score = (float)sum_scores;
                score_offset = 0.0f;
                emit();
                return SKM_OK;
            }
        }
    }
    // 4. per-function score sums, top two by partial_sort (libstdc++ semantics on ties)
    std::map<int, int> by_func;
    for (const auto& c : merged) by_func[c.function_index] += c.count;
    std::vector<std::pair<uint16_t, int>> vec(by_func.begin(), by_func.end());
    if (vec.size() > 1)
        std::partial_sort(vec.begin(), vec.begin() + 2, vec.end(),
                          [](const std::pair<uint16_t, int>& a, const std::pair<uint16_t, int>& b) { return a.second > b.second; });
    score_offset = vec.size() == 1 ? (float)vec[0].second : (float)(vec[0].second - vec[1].second);
    if (score_offset >= 5.0f) {
        fi = vec[0].first;
        func = fname(fi);
        score = (float)vec[0].second;
    } else if (vec.size() >= 2) {
        std::string f1 = fname(vec[0].first), f2 = fname(vec[1].first);
        if (f2 > f1) std::swap(f1, f2);
        if (vec.size() == 2) {
            func = f1 + " ?? " + f2;
            score = (float)vec[0].second;
        } else {
            const float pair_offset = (float)(vec[1].second - vec[2].second);
            if (pair_offset > 2.0f) {
                func = f1 + " ?? " + f2;
                score = (float)vec[0].second;
                score_offset = pair_offset;
            }
        }
    }
    emit();
    SKM_API_END
}

}  // extern "C"
