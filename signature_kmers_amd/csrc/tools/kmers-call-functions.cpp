// kmers-call-functions -- drop-in for the reference's main (kmers-call-functions.cc:34-197).
//
//   kmers-call-functions [options] data-dir input-file [input-file ...]
// Opens <data-dir>/kmer_data.mph + .dat (CmphKmerDb, cmph_kmer.h) into HBM, reads
// <data-dir>/function.index, and writes one line per query sequence
// "id\tfunc\tfunc_index\tscore\n" (kmers-call-functions.cc:178), files in input order, to -o or
// stdout.  Window lookups and HitSet calls run on the GPU (skm_annotate), find_best_call on host.
// --debug-hits prints the per-hit lines of the reference's debug hit callback
// (kmers-call-functions.cc:109-118) before each file's calls.
// Extra options: --device N; --boost-math-stats current|legacy (the Boost.Math mean / MAD the
// reference was compiled against, call_functions.tcc:51-53: current = >= 1.76, legacy = the older
// single running mean and |x(mid)| MAD).
#include <sys/stat.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <atomic>
#include <chrono>
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

bool file_exists(const std::string& p) {
    struct stat sb;
    return stat(p.c_str(), &sb) == 0;
}

// --debug-hits: hit stream of FunctionCaller::process_aa_seq (for_each_kmer + fetch + the hypo
// filter), printed as the reference's hit_cb does.  The windows and their DB hits are the device's
// (k_lookup's window iterator, skm_query_window_hits); the printed record fields come from the
// .dat slot of each hit window's key.
void debug_hits(skm_db* db, const std::vector<uint8_t>& dat, const FastaFile& f, const std::vector<std::string>& fidx,
                bool ignore_hypo, int hypo, std::ostream& os) {
    const size_t n = f.size();
    if (n == 0) return;
    std::vector<uint64_t> off(f.off.begin(), f.off.end());
    skm_query* q = nullptr;
    if (skm_query_create(&q, db, f.residues.data(), off.data(), f.len.data(), n)) die(skm_last_error());
    skm_annot_opts o{5, 200, 0, -1, 0, 0};
    std::vector<uint64_t> hoff(n + 1);
    uint64_t nh = 0;
    if (skm_query_run(q, &o) || skm_query_window_hits(q, hoff.data(), nullptr, nullptr, 0, &nh)) die(skm_last_error());
    std::vector<uint32_t> pos(std::max<uint64_t>(nh, 1));
    if (skm_query_window_hits(q, hoff.data(), pos.data(), nullptr, nh, &nh)) die(skm_last_error());
    skm_query_destroy(q);
    std::vector<uint64_t> keys(nh);
    for (size_t r = 0; r < n; ++r)
        for (uint64_t h = hoff[r]; h < hoff[r + 1]; ++h) std::memcpy(&keys[h], f.residues.data() + f.off[r] + pos[h], 8);
    std::vector<uint32_t> idx(nh);
    if (nh && skm_db_lookup(db, keys.data(), nh, idx.data())) die(skm_last_error());
    for (uint64_t i = 0; i < nh; ++i) {
        skm_stored_kmer_data kd;
        std::memcpy(&kd, dat.data() + 10ull * idx[i], 10);
        if (ignore_hypo && kd.function_index == hypo) continue;
        char kb[9];
        std::memcpy(kb, &keys[i], 8);
        kb[8] = 0;
        const std::string fn = kd.function_index < fidx.size() ? fidx[kd.function_index] : "";
        os << kb << "\t" << pos[i] << "\t" << fn << "\t" << kd.median << "\t" << kd.mean << "\t" << kd.var << "\t"
           << fmt_g(std::sqrt((double)kd.var)) << "\t" << "\n";
    }
}

}  // namespace

int main(int argc, char** argv) {
    {  // libskm runs up to 8 streams at once: at least 8 hardware queues (read at the first HIP call)
        const char* q = getenv("GPU_MAX_HW_QUEUES");
        if (!q || atoi(q) < 8) setenv("GPU_MAX_HW_QUEUES", "8", 1);
    }
    Options op;
    op.specs = {{"data-dir", 'd', false, false}, {"input-files", 'i', false, true}, {"output-files", 'o', false, false},
                {"n-threads", 'j', false, false}, {"ignore-hypo", 0, true, false},  {"debug-hits", 0, true, false},
                {"help", 'h', true, false},       {"device", 0, false, false}, {"boost-math-stats", 0, false, false}};
    op.positional = {"data-dir", "input-files"};
    std::string err;
    if (!op.parse(argc, argv, err)) die(err);
    auto usage = [&]() {
        std::cout << "Usage: " << argv[0] << " data-dir input-file [input-file, ...]\nAllowed options:\n"
                  << "  -d [ --data-dir ] arg       Data directory\n"
                  << "  -i [ --input-files ] arg    Input files\n"
                  << "  -o [ --output-files ] arg   Output file\n"
                  << "  -j [ --n-threads ] arg      Number of threads\n"
                  << "  --ignore-hypo               Ignore hypothetical protein kmers when making calls\n"
                  << "  --debug-hits                Debug kmer hits\n"
                  << "  --device arg                HIP device ordinal (default 0)\n"
                  << "  --boost-math-stats arg        current (default) | legacy Boost.Math mean/MAD\n"
                  << "  -h [ --help ]               show this help message\n\n";
    };
    if (op.has("help")) {
        usage();
        return 0;
    }
    std::vector<std::string> inputs = op.all("input-files");
    if (inputs.empty()) {
        usage();
        return 1;
    }
    std::cerr << "Data size " << sizeof(skm_stored_kmer_data) << "\n";
    int n_threads = std::atoi(op.get("n-threads", "0").c_str());
    if (n_threads < 2) n_threads = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    {
        const std::string bm = op.get("boost-math-stats", "current");
        if (bm != "current" && bm != "legacy") die("--boost-math-stats must be current or legacy");
        set_boost_math_modes(bm == "legacy", bm == "legacy");
    }
    const int device = std::atoi(op.get("device", "0").c_str());
    const std::string data_dir = op.get("data-dir");
    const std::string db_base = path_join(data_dir, "kmer_data");
    const std::string mph = db_base + ".mph", dat = db_base + ".dat";
    if (!file_exists(mph)) die("Database \"" + db_base + "\" does not exist");
    skm_db* db = nullptr;
    const auto t_open0 = std::chrono::steady_clock::now();
    if (skm_db_open(&db, mph.c_str(), dat.c_str(), device)) die(skm_last_error());
    const double t_open = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_open0).count();
    std::vector<std::string> fidx;
    if (!read_function_index(path_join(data_dir, "function.index"), fidx, err)) die(err);
    const bool ignore_hypo = op.has("ignore-hypo");

    auto now_s = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    double t0 = now_s();
    std::vector<FastaFile> files;
    if (!parse_fasta_files(inputs, files, n_threads, err)) die(err);
    const double t_parse = now_s() - t0;
    std::vector<const FastaFile*> fptr;
    for (auto& f : files) fptr.push_back(&f);
    std::vector<std::vector<SeqCall>> calls;
    double dev_ms = 0, host_ms = 0;
    if (call_files(db, fptr, fidx, ignore_hypo, n_threads, calls, err, &dev_ms, 2000000000ull, &host_ms)) die(err);
    t0 = now_s();

    std::ofstream ofs;
    std::ostream* out = &std::cout;
    if (op.has("output-files")) {
        ofs.open(op.get("output-files"));
        if (!ofs) die("cannot write " + op.get("output-files"));
        out = &ofs;
    }
    std::vector<uint8_t> datbuf;
    int hypo = -1;
    if (op.has("debug-hits")) {
        std::ifstream df(dat, std::ios::binary);
        datbuf.assign(std::istreambuf_iterator<char>(df), std::istreambuf_iterator<char>());
        for (size_t i = 0; i < fidx.size(); ++i)
            if (fidx[i] == "hypothetical protein") {
                hypo = (int)i;
                break;
            }
    }
    // each file's lines formatted on the host threads, written in file order
    std::vector<std::string> text(files.size());
    {
        std::atomic<size_t> next{0};
        auto fmt = [&]() {
            for (size_t f; (f = next.fetch_add(1)) < files.size();) {
                std::string& buf = text[f];
                for (size_t r = 0; r < files[f].size(); ++r) {
                    const SeqCall& c = calls[f][r];
                    buf += files[f].ids[r];
                    buf += '\t';
                    buf += c.func;
                    buf += '\t';
                    buf += std::to_string((unsigned)c.fi);
                    buf += '\t';
                    buf += fmt_g(c.score);
                    buf += '\n';
                }
            }
        };
        std::vector<std::thread> th;
        for (int t = 1; t < std::min<int>(n_threads, (int)files.size()); ++t) th.emplace_back(fmt);
        fmt();
        for (auto& t : th) t.join();
    }
    for (size_t f = 0; f < files.size(); ++f) {
        if (op.has("debug-hits")) debug_hits(db, datbuf, files[f], fidx, ignore_hypo, hypo, std::cout);
        out->write(text[f].data(), (std::streamsize)text[f].size());
        std::string().swap(text[f]);
    }
    out->flush();
    const double t_write = now_s() - t0;
    skm_db_close(db);
    uint64_t nrec = 0;
    for (auto& f : files) nrec += f.size();
    // one machine-readable line of the phases (bench.py's cli_call leg)
    std::cerr << "phases: sequences " << nrec << " db_open " << t_open << " parse " << t_parse << " device " << dev_ms / 1e3 << " best_call "
              << host_ms / 1e3 << " write " << t_write << "\n";
    return 0;
}
