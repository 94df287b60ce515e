// skm_caller.h -- FunctionCaller<KmerDb>::process_fasta_stream for the CLIs
// (call_functions.tcc:109-257): every record with a non-empty id is one query; the windows are
// looked up and the HitSet calls made on the GPU (skm_annotate), find_best_call runs on the host.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "skm.h"
#include "skm_front.h"

namespace skmf {

struct SeqCall {
    uint16_t fi = 0xFFFF;
    float score = 0.0f;
    std::string func;
};

// FunctionCaller::read_function_index (call_functions.tcc:123-148): column 0 = index, column 1 =
// name; the table is sized max index + 1.
bool read_function_index(const std::string& path, std::vector<std::string>& table, std::string& err);

// Boost.Math statistics the reference was compiled against (call_functions.tcc:51-53; SURVEY
// A.6): mean_mode 0 = the >= 1.76 four-lane mean, 1 = the single running mean; mad_mode 0 =
// |x(mid) - median|, 1 = the older median_absolute_deviation that returns |x(mid)|.  Process-wide
// setting for call_files (the CLIs' --boost-math-stats option); default 0 / 0.
void set_boost_math_modes(int mean_mode, int mad_mode);

// Query every sequence of every file (in order) against db.  out[f][r] is the call for record r
// of file f.  Files are batched so one device batch holds <= max_batch_residues residues.
// device_ms: wall ms in skm_annotate (packing, upload, device pipeline, calls download);
// host_ms: wall ms of the rest (batch assembly, find_best_call on n_threads host threads).
int call_files(skm_db* db, const std::vector<const FastaFile*>& files, const std::vector<std::string>& function_index,
               bool ignore_hypo, int n_threads, std::vector<std::vector<SeqCall>>& out, std::string& err,
               double* device_ms = nullptr, uint64_t max_batch_residues = 2000000000ull, double* host_ms = nullptr);

// The two halves of call_files, for callers that pipeline them (kmers-call-functions overlaps
// parsing, the device and find_best_call over groups of files, as the reference overlaps its
// per-file tasks with its writer thread, kmers-call-functions.cc:147-189).
// annot_opts_for: process_aa_seq's options (min_hits 5, max_gap 200, the hypothetical-protein
// index -- an error when the function index has none, call_functions.tcc:269-274).
bool annot_opts_for(const std::vector<std::string>& function_index, bool ignore_hypo, skm_annot_opts& o,
                    std::string& err);
// the device half for one batch of whole files: the windows looked up and the HitSet calls made
// (skm_annotate over their sequences, in file order); *calls is released with skm_calls_free
int annotate_batch(skm_db* db, const std::vector<const FastaFile*>& files, const skm_annot_opts& o, int n_threads,
                   skm_calls* calls, std::string& err);
// the host half: find_best_call per sequence on n_threads threads; out[f] is the call vector of
// files[f] (sized by the caller)
int best_calls_batch(const skm_calls& calls, const std::vector<const FastaFile*>& files,
                     const std::vector<const char*>& fidx, int n_threads, const std::vector<std::vector<SeqCall>*>& out,
                     std::string& err);

}  // namespace skmf
