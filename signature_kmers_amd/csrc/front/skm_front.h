// skm_front.h -- host front end of the signature-k-mer CLIs: FASTA parsing, the SEED function
// assignment rules and the per-sequence FunctionIndex table that feeds skm_build_add_batch.
//
// Restates (same observable behaviour, no Boost):
//   FastaParser            fasta_parser.h:38-164, fasta_parser.cc:17-36
//   seed_utils             seed_utils.h:10-62 (the Boost.Regex patterns are hand-coded matchers)
//   FunctionMap            function_map.h:44-465
//   populate_path_list...  path_utils.h:17-100 (readdir order, regular files only)
//   SignatureBuilder::load_kmers_from_fasta/_sequence  signature_build.tcc:84-181 (sequence
//                          selection, seq_id = file_number*max_seqs_per_file + k, u32 wrap)
// Files are parsed in parallel (one task per file) and applied to the FunctionMap in file order,
// so results equal the reference's --n-threads 1 run.
#pragma once
#include <cstdint>
#include <map>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

namespace skmf {

// One parsed FASTA file: records with a non-empty id, residues back to back.
struct FastaFile {
    std::string path;
    std::string filename;
    std::vector<std::string> ids;
    std::vector<std::string> defs;  // definition line incl. its leading blank (fasta_parser.h:65-68)
    std::vector<uint64_t> off;      // into residues
    std::vector<uint32_t> len;
    std::vector<uint8_t> residues;  // empty when parsed headers-only
    uint64_t n_residues = 0;        // residue count (also when headers-only)
    size_t size() const { return ids.size(); }
};

// FastaParser state machine over a whole file.  Parse errors are reported on stderr exactly as
// the reference prints them and the offending character is dropped.  Returns false if the file
// cannot be read.
// keep_residues = false: headers-only (ids, definitions, offsets and lengths as if the residues
// were kept, no residue bytes; same parse errors).
bool parse_fasta_file(const std::string& path, FastaFile& out, bool keep_residues = true);
void parse_fasta_buffer(const char* buf, size_t n, FastaFile& out, bool keep_residues = true);
// Parse several files on up to n_threads threads; result order = input order.  keep_residues
// (optional, one flag per path) selects the headers-only form for the files whose flag is 0.
bool parse_fasta_files(const std::vector<std::string>& paths, std::vector<FastaFile>& out, int n_threads,
                       std::string& err, const std::vector<char>* keep_residues = nullptr);

// path_utils.h: regular files of each directory in directory_iterator (readdir) order.
bool list_regular_files(const std::string& dir, std::vector<std::string>& out, std::string& err);
// load_strings / load_set_from_file: one entry per line (every line, empty ones too).
std::vector<std::string> load_lines(const std::string& path, bool* ok = nullptr);

// seed_utils.h
void split_func_comment(const std::string& s, std::string& func, std::string& sep, std::string& comment);
bool is_truncated_comment(const std::string& s);
std::string strip_func_comment(const std::string& s);
std::vector<std::string> roles_of_function(const std::string& function);
// function_map.h:123 regex_match(def, "\s+(.*)\s+\[([^]]+)\]$")
bool match_genome_defline(const std::string& def, std::string& func_part, std::string& genome);
// function_map.h:124 regex_search(id, "fig\|(\d+\.\d+)")
bool search_fig_genome(const std::string& id, std::string& genome);

// accumulator_set<float, stats<mean, median(P^2), variance, count>> (function_map.h:463)
struct FloatStats {
    uint64_t count = 0;
    float sum = 0.0f;
    float variance = 0.0f;
    float heights[5] = {0, 0, 0, 0, 0};
    float actual[5] = {1, 2, 3, 4, 5};
    float desired[5] = {1, 2, 3, 4, 5};
    void add(float x);
    float mean() const { return sum / (float)count; }
    float median() const { return heights[2]; }
};

class FunctionMap {
public:
    void add_good_functions(const std::vector<std::string>& v) { good_functions_.insert(v.begin(), v.end()); }
    void add_good_roles(const std::vector<std::string>& v) { good_roles_.insert(v.begin(), v.end()); }
    // function_map.h:62-104.  threads > 1: the lines are split on that many host threads, then
    // the three tables are filled in line order, one thread per table (same tables, same messages)
    void load_id_assignments(const std::string& path, int threads = 1);
    void load_id_assignments(const std::vector<std::string>& paths, int threads);  // in path order
    // function_map.h:119-238 over an already parsed file (keep flag: signature_build.tcc:32
    // always passes false)
    void load_fasta_file(const FastaFile& f, const std::set<std::string>& deleted_fids);
    // load_fasta_file over every file in order, the per-record parsing (definition line, function /
    // comment split, the file's genome) on `threads` host threads and the table updates in record
    // order on the caller's: the same tables, messages and first exception as the loop
    void load_fasta_files(const std::vector<FastaFile>& files, const std::set<std::string>& deleted_fids, int threads);
    // function_map.h:257-332; returns the number of kept functions ("kept N functions")
    unsigned process_kept_functions(int min_reps_required, const std::set<std::string>& ignored);
    // function_map.h:389-411
    bool write_function_index(const std::string& dir) const;

    std::string lookup_function_of_id(const std::string& id) const;
    uint16_t lookup_index(const std::string& func) const;
    std::string lookup_function(uint16_t idx) const;
    void lookup_original_assignment(const std::string& id, std::string& func, std::string& stripped) const;
    // FunctionIndex -> name table (function.index column 1), size = kept count
    std::vector<std::string> index_table() const;

private:
    std::map<std::string, std::set<std::string>> function_genome_map_;
    std::unordered_map<std::string, std::string> id_function_map_;
    std::map<std::string, uint16_t> function_index_map_;
    std::map<uint16_t, std::string> index_function_map_;
    std::set<std::string> good_roles_, good_functions_;
    std::unordered_map<std::string, std::string> original_assignment_, original_assignment_stripped_;
    mutable std::map<std::string, FloatStats> function_accumulators_;
};

// Per-sequence build input of one file in reference emission order (signature_build.tcc:84-181):
// sequences without an assigned function are skipped (no seq_id consumed), sequences whose
// function is not kept consume a seq_id and are skipped.
struct BuildBatch {
    std::vector<uint64_t> off;
    std::vector<uint32_t> len;
    std::vector<uint16_t> func;
    std::vector<uint32_t> seq_id;
};
void select_build_sequences(const FunctionMap& fm, const FastaFile& f, unsigned file_number,
                            unsigned max_seqs_per_file, const std::set<std::string>& deleted_fids,
                            BuildBatch& out);

// End the process with status `code` once its output is written: std::_Exit after flushing
// stdout / stderr, skipping the destructors of the host-side tables (FunctionMap, parsed files:
// millions of strings) and the HIP runtime's teardown (~1.4 s at C2 for kmers-build-signatures).
// SKM_CLI_FULL_EXIT=1 (e.g. under a profiler that writes its trace at exit) returns normally.
[[noreturn]] void fast_exit(int code);
// seconds since this process started (the CLIs' "startup" phase: loader, libskm, HIP runtime)
double process_age_s();
// ostream << float/double with the default format (precision 6, %g), incl. "-nan"/"inf".
std::string fmt_g(double v);

// Minimal Boost.program_options-style command line: --name value, --name=value, -x value,
// multitoken options consume values up to the next option, positional names fill in order.
struct Options {
    struct Spec {
        std::string name;
        char short_name;
        bool flag;        // bool_switch
        bool multi;       // multitoken / repeated
    };
    std::vector<Spec> specs;
    std::vector<std::string> positional;  // option names filled by positional arguments
    std::map<std::string, std::vector<std::string>> values;
    bool parse(int argc, char** argv, std::string& err);
    bool has(const std::string& n) const { return values.count(n) != 0; }
    std::string get(const std::string& n, const std::string& dflt = "") const;
    std::vector<std::string> all(const std::string& n) const;
};

std::string path_join(const std::string& dir, const std::string& name);
std::string path_filename(const std::string& p);
bool path_is_relative(const std::string& p);
bool ensure_directory(const std::string& dir);

}  // namespace skmf
