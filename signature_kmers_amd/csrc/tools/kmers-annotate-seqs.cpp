// kmers-annotate-seqs -- drop-in for the reference's main (kmers-annotate-seqs.cc:35-169).
//
//   kmers-annotate-seqs [options] kmer-data-dir genus-data-dir sequences-dir calls-file uncalled-ids-file
// Every regular file of sequences-dir (readdir order) is called against <kmer-data-dir>/kmer_data
// (CmphKmerDb in HBM).  Called ids go to calls-file as "id\tfunc\tfunc_index\tscore\n"; ids whose
// call has no function index (no call, or an "f1 ?? f2" call) go to uncalled-ids-file
// (kmers-annotate-seqs.cc:136-146,163-167).  genus-data-dir is accepted and unused, as upstream.
// Extra options: --device N; --boost-math-stats current|legacy (the Boost.Math mean / MAD the
// reference was compiled against, call_functions.tcc:51-53: current = >= 1.76, legacy = the older
// single running mean and |x(mid)| MAD).
#include <sys/stat.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <thread>

#include "skm.h"
#include "skm_caller.h"
#include "skm_front.h"

using namespace skmf;

namespace {
void die(const std::string& m) {
    std::cerr << m << "\n";
    std::exit(1);
}
}  // namespace

int main(int argc, char** argv) {
    {  // libskm runs up to 10 streams at once: 16 hardware queues (read at the first HIP call)
        const char* q = getenv("GPU_MAX_HW_QUEUES");
        if (!q || atoi(q) < 16) setenv("GPU_MAX_HW_QUEUES", "16", 1);
    }
    Options op;
    op.specs = {{"kmer-data-dir", 'd', false, false}, {"genus-data-dir", 'g', false, false},
                {"sequences-dir", 0, false, false},   {"calls-file", 0, false, false},
                {"uncalled-ids-file", 0, false, false}, {"parallel", 'j', false, false},
                {"ignore-hypo", 0, true, false},      {"help", 'h', true, false},
                {"device", 0, false, false}, {"boost-math-stats", 0, false, false}};
    op.positional = {"kmer-data-dir", "genus-data-dir", "sequences-dir", "calls-file", "uncalled-ids-file"};
    std::string err;
    if (!op.parse(argc, argv, err)) die(err);
    if (op.has("help")) {
        std::cout << "Usage: " << argv[0]
                  << " kmer-data-dir genus-data-dir sequences-dir calls-file uncalled-ids-file\nAllowed options:\n"
                  << "  -d [ --kmer-data-dir ] arg    Kmer data directory\n"
                  << "  -g [ --genus-data-dir ] arg   Genus data directory\n"
                  << "  --sequences-dir arg           Sequence directory\n"
                  << "  --calls-file arg              Output calls file\n"
                  << "  --uncalled-ids-file arg       Output uncalled IDs file\n"
                  << "  -j [ --parallel ] arg         Number of threads\n"
                  << "  --ignore-hypo                 Ignore hypothetical protein kmers when making calls\n"
                  << "  --device arg                  HIP device ordinal (default 0)\n"
                  << "  --boost-math-stats arg          current (default) | legacy Boost.Math mean/MAD\n"
                  << "  -h [ --help ]                 show this help message\n\n";
        return 0;
    }
    int n_threads = std::atoi(op.get("parallel", "0").c_str());
    if (n_threads < 2) n_threads = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    {
        const std::string bm = op.get("boost-math-stats", "current");
        if (bm != "current" && bm != "legacy") die("--boost-math-stats must be current or legacy");
        set_boost_math_modes(bm == "legacy", bm == "legacy");
    }
    const int device = std::atoi(op.get("device", "0").c_str());
    const std::string data_dir = op.get("kmer-data-dir");
    const std::string db_base = path_join(data_dir, "kmer_data");
    struct stat sb;
    if (stat((db_base + ".mph").c_str(), &sb) != 0) die("Database \"" + db_base + "\" does not exist");
    skm_db* db = nullptr;
    if (skm_db_open(&db, (db_base + ".mph").c_str(), (db_base + ".dat").c_str(), device)) die(skm_last_error());
    std::vector<std::string> fidx;
    if (!read_function_index(path_join(data_dir, "function.index"), fidx, err)) die(err);

    std::vector<std::string> inputs;
    if (!list_regular_files(op.get("sequences-dir"), inputs, err)) die(err);
    std::vector<FastaFile> files;
    if (!parse_fasta_files(inputs, files, n_threads, err)) die(err);
    std::vector<const FastaFile*> fptr;
    for (auto& f : files) fptr.push_back(&f);
    std::vector<std::vector<SeqCall>> calls;
    if (call_files(db, fptr, fidx, op.has("ignore-hypo"), n_threads, calls, err)) die(err);
    skm_db_close(db);

    std::ofstream anno(op.get("calls-file"));
    std::vector<std::string> uncalled;
    for (size_t f = 0; f < files.size(); ++f) {
        std::string buf;
        for (size_t r = 0; r < files[f].size(); ++r) {
            const SeqCall& c = calls[f][r];
            if (c.fi == 0xFFFF)
                uncalled.push_back(files[f].ids[r]);
            else
                buf += files[f].ids[r] + "\t" + c.func + "\t" + std::to_string((unsigned)c.fi) + "\t" + fmt_g(c.score) + "\n";
        }
        anno << buf;
    }
    std::ofstream un(op.get("uncalled-ids-file"));
    for (auto& id : uncalled) un << id << "\n";
    return 0;
}
