// skm_caller.cpp -- see skm_caller.h.
#include "skm_caller.h"

#include "../skm_strutil.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <fstream>
#include <memory>
#include <mutex>
#include <thread>

namespace skmf {

bool read_function_index(const std::string& path, std::vector<std::string>& table, std::string& err) {
    // call_functions.tcc:123-148: max id over the lines, then function_index_[stoi(parts[0])] =
    // parts[1] with parts = split(line, "\t") (operators.h:80-91).  One read instead of two; a
    // line without a tab (parts[1] out of range in the reference) names the empty string.
    std::ifstream f(path);
    if (!f) {
        err = "cannot read " + path;
        return false;
    }
    std::vector<std::pair<int, std::string>> rows;
    int max_id = 0;
    std::string line;
    while (std::getline(f, line, '\n')) {
        const std::vector<std::string> parts = skm_str::split(line, "\t");
        int id = 0;
        try {
            id = std::stoi(parts[0]);
        } catch (const std::exception&) {
            err = "bad function.index line in " + path + ": '" + line + "'";
            return false;
        }
        if (id < 0) {
            err = "negative function index in " + path + ": '" + line + "'";
            return false;
        }
        max_id = std::max(max_id, id);
        rows.emplace_back(id, parts.size() > 1 ? parts[1] : std::string());
    }
    table.assign((size_t)max_id + 1, std::string());
    for (auto& r : rows) table[(size_t)r.first] = r.second;
    return true;
}

namespace {
int g_mean_mode = 0, g_mad_mode = 0;
}

void set_boost_math_modes(int mean_mode, int mad_mode) {
    g_mean_mode = mean_mode;
    g_mad_mode = mad_mode;
}

bool annot_opts_for(const std::vector<std::string>& function_index, bool ignore_hypo, skm_annot_opts& o,
                    std::string& err) {
    auto hit = std::find(function_index.begin(), function_index.end(), "hypothetical protein");
    if (hit == function_index.end()) {  // process_aa_seq exits here (call_functions.tcc:269-274)
        err = "Cannot find hypothetical protein index";
        return false;
    }
    o = skm_annot_opts{};
    o.min_hits = 5;
    o.max_gap = 200;
    o.ignore_hypo = ignore_hypo ? 1 : 0;
    o.hypo_index = (int32_t)(hit - function_index.begin());
    o.mean_mode = g_mean_mode;
    o.mad_mode = g_mad_mode;
    return true;
}

int annotate_batch(skm_db* db, const std::vector<const FastaFile*>& files, const skm_annot_opts& o, int n_threads,
                   skm_calls* calls, std::string& err) {
    *calls = skm_calls{};
    // the batch packed as skm_annotate lays it out on the device (every sequence followed by a 0,
    // back to back), so the library uploads it as it is instead of packing a second copy; files
    // are copied by the host threads
    std::vector<uint64_t> rbase(files.size() + 1, 0), sbase(files.size() + 1, 0);
    for (size_t f = 0; f < files.size(); ++f) {
        uint64_t nb = 0;
        for (size_t r = 0; r < files[f]->size(); ++r) nb += (uint64_t)files[f]->len[r] + 1;
        rbase[f + 1] = rbase[f] + nb;
        sbase[f + 1] = sbase[f] + files[f]->size();
    }
    std::unique_ptr<uint8_t[]> res(new uint8_t[std::max<uint64_t>(rbase.back(), 1)]);
    std::vector<uint64_t> off(sbase.back());
    std::vector<uint32_t> len(sbase.back());
    std::atomic<size_t> nextf{0};
    auto cp = [&]() {
        for (size_t f; (f = nextf.fetch_add(1)) < files.size();) {
            const FastaFile& F = *files[f];
            uint64_t p = rbase[f];
            for (size_t r = 0; r < F.size(); ++r) {
                std::memcpy(res.get() + p, F.residues.data() + F.off[r], F.len[r]);
                res[p + F.len[r]] = 0;
                off[sbase[f] + r] = p;
                len[sbase[f] + r] = F.len[r];
                p += (uint64_t)F.len[r] + 1;
            }
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < std::max(1, std::min<int>(n_threads, (int)files.size())); ++t) th.emplace_back(cp);
    cp();
    for (auto& t : th) t.join();
    const int rc = skm_annotate(db, res.get(), off.data(), len.data(), off.size(), &o, calls);
    if (rc) err = skm_last_error();
    return rc;
}

int best_calls_batch(const skm_calls& calls, const std::vector<const FastaFile*>& files,
                     const std::vector<const char*>& fidx, int n_threads, const std::vector<std::vector<SeqCall>*>& out,
                     std::string& err) {
    std::vector<std::pair<size_t, size_t>> where;  // (file, record) per batch sequence
    for (size_t f = 0; f < files.size(); ++f)
        for (size_t r = 0; r < files[f]->size(); ++r) where.emplace_back(f, r);
    if (where.size() != calls.n_seqs) {
        err = "find_best_call: call list does not match the batch";
        return SKM_E_STATE;
    }
    std::atomic<size_t> next{0};
    std::atomic<int> first_rc{0};
    std::mutex err_mu;  // skm_last_error() is per thread: the failing worker records its own message
    std::string worker_err;
    auto work = [&]() {
        std::vector<char> fb(1 << 16);
        const size_t chunk = 4096;
        for (size_t s0; (s0 = next.fetch_add(chunk)) < where.size();) {
            for (size_t s = s0; s < std::min(where.size(), s0 + chunk); ++s) {
                SeqCall& c = (*out[where[s].first])[where[s].second];
                float offset = 0;
                int r = skm_find_best_call(calls.calls + calls.call_off[s], calls.call_off[s + 1] - calls.call_off[s],
                                           fidx.data(), fidx.size(), &c.fi, &c.score, &offset, fb.data(), fb.size());
                if (r) {
                    std::lock_guard<std::mutex> lk(err_mu);
                    if (!first_rc) {
                        first_rc = r;
                        worker_err = skm_last_error();
                    }
                }
                c.func = fb.data();
            }
        }
    };
    const int nt = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::max(1, n_threads), where.size() / 4096 + 1));
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work);
    work();
    for (auto& t : th) t.join();
    if (first_rc) err = worker_err.empty() ? std::string("find_best_call failed") : worker_err;
    return first_rc;
}

int call_files(skm_db* db, const std::vector<const FastaFile*>& files, const std::vector<std::string>& function_index,
               bool ignore_hypo, int n_threads, std::vector<std::vector<SeqCall>>& out, std::string& err,
               double* device_ms, uint64_t max_batch_residues, double* host_ms) {
    const auto t_begin = std::chrono::steady_clock::now();
    double dev_ms = 0;
    skm_annot_opts o{};
    if (!annot_opts_for(function_index, ignore_hypo, o, err)) return SKM_E_ARG;
    std::vector<const char*> fidx(function_index.size());
    for (size_t i = 0; i < function_index.size(); ++i) fidx[i] = function_index[i].c_str();
    out.assign(files.size(), std::vector<SeqCall>());
    for (size_t f = 0; f < files.size(); ++f) out[f].resize(files[f]->size());
    size_t f0 = 0;
    while (f0 < files.size()) {
        // one device batch: whole files up to max_batch_residues residues
        size_t f1 = f0;
        uint64_t nres = 0;
        while (f1 < files.size() && (f1 == f0 || nres + files[f1]->residues.size() <= max_batch_residues))
            nres += files[f1++]->residues.size();
        const std::vector<const FastaFile*> batch(files.begin() + f0, files.begin() + f1);
        skm_calls calls{};
        auto t0 = std::chrono::steady_clock::now();
        int rc = annotate_batch(db, batch, o, n_threads, &calls, err);
        dev_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (rc) return rc;
        std::vector<std::vector<SeqCall>*> outp;
        for (size_t f = f0; f < f1; ++f) outp.push_back(&out[f]);
        rc = best_calls_batch(calls, batch, fidx, n_threads, outp, err);
        skm_calls_free(&calls);
        if (rc) return rc;
        f0 = f1;
    }
    if (device_ms) *device_ms = dev_ms;
    if (host_ms)
        *host_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_begin).count() - dev_ms;
    return SKM_OK;
}

}  // namespace skmf
