// kmers-call-functions -- drop-in for the reference's main (kmers-call-functions.cc:34-197).
//
//   kmers-call-functions [options] data-dir input-file [input-file ...]
// Opens <data-dir>/kmer_data.mph + .dat (CmphKmerDb, cmph_kmer.h) into HBM, reads
// <data-dir>/function.index, and writes one line per query sequence
// "id\tfunc\tfunc_index\tscore\n" (kmers-call-functions.cc:178), files in input order, to -o or
// stdout.  Window lookups and HitSet calls run on the GPU (skm_annotate), find_best_call on host.
// --debug-hits prints the per-hit lines of the reference's debug hit callback
// (kmers-call-functions.cc:109-118) before each file's calls.  Parsing, the device, find_best_call
// and the writer run as a pipeline over groups of files (see main).
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
#include <condition_variable>
#include <mutex>
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
    const double t_startup = process_age_s();  // before main: loader, libskm, HIP runtime
    {  // libskm runs up to 10 streams at once: 16 hardware queues (read at the first HIP call)
        const char* q = getenv("GPU_MAX_HW_QUEUES");
        if (!q || atoi(q) < 16) setenv("GPU_MAX_HW_QUEUES", "16", 1);
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
    // the HIP runtime initialises on a thread of its own while the DB files are read (the first
    // HIP call of a process costs ~0.1-0.3 s; skm_db_open's uploads then find it done)
    std::thread hip_warm([] {
        int ndev = 0;
        (void)skm_device_count(&ndev);
    });
    const std::string data_dir = op.get("data-dir");
    const std::string db_base = path_join(data_dir, "kmer_data");
    const std::string mph = db_base + ".mph", dat = db_base + ".dat";
    if (!file_exists(mph)) die("Database \"" + db_base + "\" does not exist");
    std::vector<std::string> fidx;
    if (!read_function_index(path_join(data_dir, "function.index"), fidx, err)) die(err);
    const bool ignore_hypo = op.has("ignore-hypo");
    skm_annot_opts aopts{};
    if (!annot_opts_for(fidx, ignore_hypo, aopts, err)) die(err);
    std::vector<const char*> fptr_idx(fidx.size());
    for (size_t i = 0; i < fidx.size(); ++i) fptr_idx[i] = fidx[i].c_str();
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
        hypo = aopts.hypo_index;
    }
    // Pipelined over groups of input files, as the reference overlaps its per-file tasks with its
    // writer thread (kmers-call-functions.cc:147-189): a parse stage (the files of a group on the
    // host threads), the device stage (skm_annotate of the group), a host stage (find_best_call
    // and each file's lines) and this thread writing the groups in input order.  The DB is opened
    // (read + uploaded to HBM) while the first groups parse.  Output bytes are those of the
    // one-phase-at-a-time form.
    using clk = std::chrono::steady_clock;
    auto secs = [](clk::time_point a) { return std::chrono::duration<double>(clk::now() - a).count(); };
    const auto t_all = clk::now();
    const size_t per_group = std::max<size_t>(1, std::min<size_t>(128, (inputs.size() + 7) / 8));
    const size_t ng = (inputs.size() + per_group - 1) / per_group;
    struct Group {
        std::vector<FastaFile> files;
        std::vector<std::vector<SeqCall>> calls;
        skm_calls dev{};
        std::string text;
        int state = 0;  // 1 parsed, 2 on-device done, 3 calls + text ready; -1 failed
        std::string err;
    };
    std::vector<Group> groups(ng);
    std::mutex mu;
    std::condition_variable cv;
    auto set_state = [&](size_t g, int st, const std::string& e = std::string()) {
        std::lock_guard<std::mutex> lk(mu);
        groups[g].state = st;
        if (st < 0) groups[g].err = e;
        cv.notify_all();
    };
    auto wait_state = [&](size_t g, int st) {  // false: the group failed
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return groups[g].state >= st || groups[g].state < 0; });
        return groups[g].state >= 0;
    };
    skm_db* db = nullptr;
    double t_open = 0, t_parse = 0, t_dev = 0, t_best = 0, t_write = 0;
    std::string db_err;
    std::thread db_thread([&] {
        const auto t = clk::now();
        if (skm_db_open(&db, mph.c_str(), dat.c_str(), device)) db_err = skm_last_error();
        t_open = secs(t);
    });
    std::thread parser([&] {
        for (size_t g = 0; g < ng; ++g) {
            const auto t = clk::now();
            const std::vector<std::string> paths(inputs.begin() + g * per_group,
                                                 inputs.begin() + std::min(inputs.size(), (g + 1) * per_group));
            std::string e;
            if (!parse_fasta_files(paths, groups[g].files, n_threads, e)) {
                for (size_t h = g; h < ng; ++h) set_state(h, -1, e);
                return;
            }
            t_parse += secs(t);
            set_state(g, 1);
        }
    });
    std::thread device_stage([&] {
        db_thread.join();
        hip_warm.join();
        for (size_t g = 0; g < ng; ++g) {
            if (!db_err.empty()) {
                set_state(g, -1, db_err);
                continue;
            }
            if (!wait_state(g, 1)) continue;
            const auto t = clk::now();
            std::vector<const FastaFile*> fp;
            for (auto& f : groups[g].files) fp.push_back(&f);
            std::string e;
            if (annotate_batch(db, fp, aopts, n_threads, &groups[g].dev, e)) {
                set_state(g, -1, e);
                continue;
            }
            t_dev += secs(t);
            set_state(g, 2);
        }
    });
    std::thread host_stage([&] {
        for (size_t g = 0; g < ng; ++g) {
            if (!wait_state(g, 2)) continue;
            const auto t = clk::now();
            Group& G = groups[g];
            std::vector<const FastaFile*> fp;
            std::vector<std::vector<SeqCall>*> op_;
            G.calls.resize(G.files.size());
            for (size_t f = 0; f < G.files.size(); ++f) {
                fp.push_back(&G.files[f]);
                G.calls[f].resize(G.files[f].size());
                op_.push_back(&G.calls[f]);
            }
            std::string e;
            const int rc = best_calls_batch(G.dev, fp, fptr_idx, n_threads, op_, e);
            skm_calls_free(&G.dev);
            if (rc) {
                set_state(g, -1, e);
                continue;
            }
            // the group's lines, its files in order ("id\tfunc\tfunc_index\tscore\n", :178): each
            // file's lines formatted on the host threads, then joined in order
            std::vector<std::string> ftext(G.files.size());
            std::atomic<size_t> nextf{0};
            auto fmt = [&]() {
                for (size_t f; (f = nextf.fetch_add(1)) < G.files.size();) {
                    std::string& o = ftext[f];
                    for (size_t r = 0; r < G.files[f].size(); ++r) {
                        const SeqCall& c = G.calls[f][r];
                        o += G.files[f].ids[r];
                        o += '\t';
                        o += c.func;
                        o += '\t';
                        o += std::to_string((unsigned)c.fi);
                        o += '\t';
                        o += fmt_g(c.score);
                        o += '\n';
                    }
                }
            };
            {
                std::vector<std::thread> th;
                for (int t = 1; t < std::max(1, std::min<int>(n_threads, (int)G.files.size())); ++t) th.emplace_back(fmt);
                fmt();
                for (auto& x : th) x.join();
            }
            size_t tl = 0;
            for (auto& x : ftext) tl += x.size();
            G.text.reserve(tl);
            for (auto& x : ftext) G.text += x;
            std::vector<std::vector<SeqCall>>().swap(G.calls);
            t_best += secs(t);
            set_state(g, 3);
        }
    });
    uint64_t nrec = 0;
    std::string fail;
    for (size_t g = 0; g < ng; ++g) {
        if (!wait_state(g, 3)) {
            fail = groups[g].err;
            break;
        }
        const auto t = clk::now();
        Group& G = groups[g];
        if (op.has("debug-hits")) {  // per file: its hit lines, then its calls (the reference's order)
            size_t at = 0;
            for (auto& f : G.files) {
                debug_hits(db, datbuf, f, fidx, ignore_hypo, hypo, std::cout);
                size_t end = at;
                for (size_t r = 0; r < f.size(); ++r) end = G.text.find('\n', end) + 1;
                out->write(G.text.data() + at, (std::streamsize)(end - at));
                at = end;
            }
        } else {
            out->write(G.text.data(), (std::streamsize)G.text.size());
        }
        for (auto& f : G.files) nrec += f.size();
        std::string().swap(G.text);
        std::vector<FastaFile>().swap(G.files);
        t_write += secs(t);
    }
    parser.join();
    device_stage.join();
    host_stage.join();
    if (!fail.empty()) die(fail);
    out->flush();
    if (db) skm_db_close(db);
    // one machine-readable line of the phases (bench.py's cli_call leg): busy seconds per stage
    // (the stages overlap) and the pipeline's wall time
    std::cerr << "phases: sequences " << nrec << " db_open " << t_open << " parse " << t_parse << " device " << t_dev
              << " best_call " << t_best << " write " << t_write << " groups " << ng << " wall " << secs(t_all)
              << " startup " << t_startup << "\n";
    if (ofs.is_open()) ofs.close();
    fast_exit(0);
}
