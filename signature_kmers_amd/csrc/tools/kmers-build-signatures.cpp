// kmers-build-signatures -- drop-in for the reference's main (kmers-build-signatures.cc:126-373).
//
// Same options, same files in --kmer-data-dir (function.index, otu.index, genomes, final.kmers,
// distinct_functions, recall.report.d/<fasta>, kmer_data.mph/.dat with --perfect-hash) and the
// same stdout lines.  The k-mer extraction, group-by, 80 % cut and statistics run on one MI355X
// through libskm (skm_build_*); the recall pass runs the GPU annotate path against an exact-key
// DB of the kept k-mers (KeptKmerDB semantics, skm_db_open_kept); the perfect hash is built on a
// host thread while the recall runs (as the reference does, kmers-build-signatures.cc:268-276).
//
// Result order: final.kmers is written in ascending k-mer key order and distinct_functions in
// ascending function index; the reference writes both in TBB hash-table order, so compare them
// as sets.  --nudb-file is not supported (NuDB is out of scope).
// Extra options: --device N (HIP device), --dump-extract FILE (write the build input arrays and
// stop before touching the GPU; used by the CPU tests), --mph-seed N.
// Multi-GPU: --n-gpus N forks one process per GPU (rank r on device r) before
// any GPU or thread use; or, under an external launcher (RANK / WORLD_SIZE / LOCAL_RANK in the
// environment, e.g. torchrun --no-python), each launched process is one rank and rank 0 hands the
// RCCL unique id to the others through --comm-file (default <kmer-data-dir>/.skm_comm_id).
// Every rank parses every file's headers (the FunctionMap needs them all) but keeps residues only
// for the files it builds (rank 0, which runs the recall pass, keeps all); rank r builds the
// contiguous range of files r*F/N .. (r+1)*F/N, the ranks exchange occurrences by owner GPU (RCCL all-to-all) and
// rank 0 gathers the kept k-mers and writes every output, exactly as one process would.
// --comm host joins the forked ranks through socketpairs instead of RCCL (several ranks may then
// share one GPU: --device is every rank's device; used by the tests).
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <iostream>
#include <map>
#include <sstream>
#include <thread>
#include <vector>
#include <atomic>
#include <condition_variable>
#include <mutex>

#include "skm.h"
#include "skm_caller.h"
#include "skm_front.h"
#include "skm_mesh.h"

using namespace skmf;

namespace {

const int K = 8;
const unsigned MaxSequencesPerFile = 100000;

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void die(const std::string& m) {
    std::cerr << m << "\n";
    std::exit(1);
}

std::string quoted(const std::string& p) { return "\"" + p + "\""; }

// final.kmers (kmers-build-signatures.cc:212-216): "KMER\tavg_from_end\tfunction_index\t\n" per
// kept k-mer.  Blocks of lines are sized first (the decimal widths), then formatted and written
// at their offsets (pwrite) by `threads` threads, so formatting and writing overlap.
void write_final_kmers(const std::string& path, const skm_kept& kept, int threads) {
    const uint64_t B = 1u << 20;  // lines per block
    const uint64_t nb = (kept.n + B - 1) / B;
    const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)std::max(1, threads), nb));
    auto ndig = [](unsigned v) { return v < 10 ? 1 : v < 100 ? 2 : v < 1000 ? 3 : v < 10000 ? 4 : 5; };
    auto fmt_u = [](char* p, unsigned v) {  // decimal, returns the digits written
        char t[8];
        int n = 0;
        do {
            t[n++] = (char)('0' + v % 10);
            v /= 10;
        } while (v);
        for (int i = 0; i < n; ++i) p[i] = t[n - 1 - i];
        return n;
    };
    std::vector<uint64_t> off(nb + 1, 0);
    auto par = [&](const std::function<void(uint64_t)>& f) {
        std::atomic<uint64_t> next{0};
        auto work = [&] {
            for (uint64_t b; (b = next.fetch_add(1)) < nb;) f(b);
        };
        std::vector<std::thread> th;
        for (int t = 1; t < T; ++t) th.emplace_back(work);
        work();
        for (auto& x : th) x.join();
    };
    par([&](uint64_t b) {
        uint64_t n = 0;
        for (uint64_t i = b * B, e = std::min<uint64_t>(kept.n, i + B); i < e; ++i)
            n += 12 + ndig(kept.data[i].avg_from_end) + ndig(kept.data[i].function_index);
        off[b + 1] = n;
    });
    for (uint64_t b = 0; b < nb; ++b) off[b + 1] += off[b];
    const int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) die("cannot write " + path);
    std::atomic<bool> ok{true};
    par([&](uint64_t b) {
        std::string o(off[b + 1] - off[b], '\0');
        char* p = &o[0];
        for (uint64_t i = b * B, e = std::min<uint64_t>(kept.n, i + B); i < e; ++i) {
            std::memcpy(p, &kept.keys[i], 8);
            p[8] = '\t';
            p += 9;
            p += fmt_u(p, kept.data[i].avg_from_end);
            *p++ = '\t';
            p += fmt_u(p, kept.data[i].function_index);
            *p++ = '\t';
            *p++ = '\n';
        }
        for (uint64_t w = 0; w < o.size();) {
            const ssize_t r = ::pwrite(fd, o.data() + w, o.size() - w, (off_t)(off[b] + w));
            if (r <= 0) {
                ok = false;
                return;
            }
            w += (uint64_t)r;
        }
    });
    if (::close(fd) != 0 || !ok) die("cannot write " + path);
}

// binary dump of the build input (--dump-extract): u64 n_seqs, u64 n_residues, then
// residues[n_residues], off u64[n], len u32[n], func u16[n], seq_id u32[n]
void dump_extract(const std::string& path, const std::vector<FastaFile>& files, const std::vector<BuildBatch>& batches) {
    std::vector<uint8_t> res;
    std::vector<uint64_t> off;
    std::vector<uint32_t> len, sid;
    std::vector<uint16_t> fn;
    for (size_t f = 0; f < files.size(); ++f) {
        const BuildBatch& b = batches[f];
        for (size_t s = 0; s < b.off.size(); ++s) {
            off.push_back(res.size());
            res.insert(res.end(), files[f].residues.begin() + b.off[s], files[f].residues.begin() + b.off[s] + b.len[s]);
            len.push_back(b.len[s]);
            fn.push_back(b.func[s]);
            sid.push_back(b.seq_id[s]);
        }
    }
    std::ofstream o(path, std::ios::binary);
    uint64_t n = off.size(), nr = res.size();
    o.write((const char*)&n, 8);
    o.write((const char*)&nr, 8);
    o.write((const char*)res.data(), (std::streamsize)nr);
    o.write((const char*)off.data(), (std::streamsize)(8 * n));
    o.write((const char*)len.data(), (std::streamsize)(4 * n));
    o.write((const char*)fn.data(), (std::streamsize)(2 * n));
    o.write((const char*)sid.data(), (std::streamsize)(4 * n));
    if (!o) die("cannot write " + path);
}

}  // namespace

int main(int argc, char** argv) {
    {  // libskm runs up to 10 streams at once: 16 hardware queues (read at the first HIP call)
        const char* q = getenv("GPU_MAX_HW_QUEUES");
        if (!q || atoi(q) < 16) setenv("GPU_MAX_HW_QUEUES", "16", 1);
    }
    Options op;
    op.specs = {{"definition-dir", 'D', false, true},  {"fasta-dir", 'F', false, true},
                {"fasta-keep-functions-dir", 'K', false, true}, {"good-functions", 0, false, true},
                {"good-roles", 0, false, true},        {"deleted-features-file", 0, false, false},
                {"ignored-functions-file", 0, false, false}, {"kmer-data-dir", 0, false, false},
                {"nudb-file", 0, false, false},        {"min-reps-required", 0, false, false},
                {"final-kmers", 0, false, false},      {"n-threads", 0, false, false},
                {"perfect-hash", 0, false, false},     {"perfect-hash-data", 0, false, false},
                {"help", 'h', true, false},            {"device", 0, false, false},
                {"dump-extract", 0, false, false},     {"mph-seed", 0, false, false},
                {"n-gpus", 0, false, false},           {"comm", 0, false, false},
                {"comm-file", 0, false, false}};
    std::string err;
    if (!op.parse(argc, argv, err)) die(err);
    if (op.has("help")) {
        std::cout << "Usage: " << argv[0] << " [options]\nAllowed options:\n"
                  << "  -D [ --definition-dir ] arg          Directory of function definition files\n"
                  << "  -F [ --fasta-dir ] arg               Directory of fasta files of protein data\n"
                  << "  -K [ --fasta-keep-functions-dir ] arg Directory of fasta files of protein data (keep functions defined here)\n"
                  << "  --good-functions arg                 File containing list of functions to be kept\n"
                  << "  --good-roles arg                     File containing list of roles to be kept\n"
                  << "  --deleted-features-file arg          File containing list of deleted feature IDs\n"
                  << "  --ignored-functions-file arg         File containing list of functions for which we do not create signatures\n"
                  << "  --kmer-data-dir arg                  Write kmer data files to this directory\n"
                  << "  --min-reps-required arg              Minimum number of genomes a function must be seen in\n"
                  << "  --final-kmers arg                    Write final.kmers file\n"
                  << "  --n-threads arg                      Number of host threads (results do not depend on it)\n"
                  << "  --perfect-hash arg                   Compute perfect hash of signature kmers and store in this file\n"
                  << "  --perfect-hash-data arg              Kmer data stored by perfect hash\n"
                  << "  --device arg                         HIP device ordinal (default 0)\n"
                  << "  --n-gpus arg                         ranks (one process and GPU each, power of two)\n"
                  << "  --comm arg                           rccl (default) or host (socketpairs; ranks may share a GPU)\n"
                  << "  --comm-file arg                      RCCL id rendezvous file under an external launcher\n"
                  << "  -h [ --help ]                        show this help message\n";
        return 1;
    }
    const double t_start = now_s();
    const double t_startup = process_age_s();  // before main: loader, libskm, HIP runtime
    // ranks: forked here (before any thread or GPU use), or given by an external launcher
    Mesh mesh;
    const std::string comm = op.get("comm", "rccl");
    if (comm != "rccl" && comm != "host") die("--comm must be rccl or host");
    const char* env_ws = std::getenv("WORLD_SIZE");
    const bool launched = env_ws && std::atoi(env_ws) > 1 && !op.has("n-gpus");
    int local_rank = 0;
    if (launched) {
        if (comm == "host") die("--comm host needs --n-gpus (forked ranks)");
        mesh.world = std::atoi(env_ws);
        mesh.rank = std::atoi(std::getenv("RANK") ? std::getenv("RANK") : "0");
        local_rank = std::atoi(std::getenv("LOCAL_RANK") ? std::getenv("LOCAL_RANK") : "0");
    } else {
        const int ng = std::atoi(op.get("n-gpus", "1").c_str());
        if (ng < 1 || ng > 64 || (ng & (ng - 1))) die("--n-gpus must be a power of two in [1, 64]");
        if (!mesh_fork(ng, mesh, err)) die(err);
        mesh.watch_children();
        local_rank = mesh.rank;
    }
    const int rank = mesh.rank, world = mesh.world;
    if (rank != 0 && !std::freopen("/dev/null", "w", stdout)) die("cannot silence rank stdout");
    // host threads for parsing / find_best_call only: results never depend on it
    int n_threads = std::atoi(op.get("n-threads", "0").c_str());
    if (n_threads < 2) n_threads = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (world > 1) n_threads = std::max(1, n_threads / std::min(world, 8));
    const int device = std::atoi(op.get("device", "0").c_str()) + (world > 1 && comm == "rccl" ? local_rank : 0);
    const int min_reps_required = std::atoi(op.get("min-reps-required", "3").c_str());
    const std::string kmer_data_dir = op.get("kmer-data-dir");
    std::string final_kmers = op.get("final-kmers");
    std::string ph_file = op.get("perfect-hash"), ph_data = op.get("perfect-hash-data");

    // the HIP runtime initialises on a thread of its own while the host parses (the first HIP call
    // of a process costs ~0.3-0.5 s)
    double t_hip_init = 0;
    std::thread hip_warm([&] {
        const double th = now_s();
        int ndev = 0;
        (void)skm_device_count(&ndev);
        t_hip_init = now_s() - th;
    });
    std::vector<std::string> definition_files, fasta_files, keep_files;
    auto populate = [&](const std::vector<std::string>& dirs, std::vector<std::string>& out) {
        for (const auto& d : dirs)
            if (!list_regular_files(d, out, err)) die(err);
    };
    populate(op.all("definition-dir"), definition_files);
    populate(op.all("fasta-dir"), fasta_files);
    populate(op.all("fasta-keep-functions-dir"), keep_files);
    std::cout << "definitions: ";
    for (auto& x : op.all("definition-dir")) std::cout << x << " ";
    std::cout << std::endl << "fasta: ";
    for (auto& x : op.all("fasta-dir")) std::cout << x << " ";
    std::cout << std::endl << "keep: ";
    for (auto& x : op.all("fasta-keep-functions-dir")) std::cout << x << " ";
    std::cout << std::endl;

    std::vector<std::string> good_functions, good_roles;
    for (auto& f : op.all("good-functions")) {
        bool ok;
        auto v = load_lines(f, &ok);
        if (!ok) std::cerr << "could not open " << f << "\n";
        good_functions.insert(good_functions.end(), v.begin(), v.end());
    }
    for (auto& f : op.all("good-roles")) {
        bool ok;
        auto v = load_lines(f, &ok);
        if (!ok) std::cerr << "could not open " << f << "\n";
        good_roles.insert(good_roles.end(), v.begin(), v.end());
    }

    // the FASTA files parse on the host threads while this thread loads the definitions (the two are
    // independent until the FunctionMap reads the records, below)
    std::cerr << "load fasta\n";
    std::vector<std::string> all_paths = fasta_files;  // fasta-dir files, then keep-dir files (signature_build.tcc:26-35)
    all_paths.insert(all_paths.end(), keep_files.begin(), keep_files.end());
    std::vector<FastaFile> files;
    // this rank's contiguous range of files (global file numbering keeps seq_id = file*100000+k)
    const size_t f0 = all_paths.size() * (size_t)rank / (size_t)world,
                 f1 = all_paths.size() * (size_t)(rank + 1) / (size_t)world;
    const bool dump = op.has("dump-extract");
    // The FunctionMap needs every file's headers; residues are kept only for the files this rank
    // builds -- and on rank 0, whose recall pass reads every sequence, for all of them.
    std::vector<char> keep_res(all_paths.size(), 0);
    for (size_t f = 0; f < all_paths.size(); ++f) keep_res[f] = rank == 0 || dump || (f >= f0 && f < f1);
    double t0 = now_s();
    bool parsed_ok = true;
    std::string parse_err;
    double t_files = 0;  // the parser thread's own time
    std::thread parser([&] {
        parsed_ok = parse_fasta_files(all_paths, files, n_threads, parse_err, &keep_res);
        t_files = now_s() - t0;
    });
    const double td = now_s();
    FunctionMap fm;
    fm.add_good_roles(good_roles);
    fm.add_good_functions(good_functions);
    fm.load_id_assignments(definition_files, n_threads);
    const double t_defs = now_s() - td;

    std::set<std::string> deleted_fids, ignored_functions;
    if (op.has("deleted-features-file"))
        for (auto& l : load_lines(op.get("deleted-features-file"))) deleted_fids.insert(l);
    if (op.has("ignored-functions-file"))
        for (auto& l : load_lines(op.get("ignored-functions-file"))) ignored_functions.insert(l);

    if (!kmer_data_dir.empty() && !ensure_directory(kmer_data_dir)) die("Error creating " + quoted(kmer_data_dir));

    parser.join();
    if (!parsed_ok) die(parse_err);
    const double t_fm0 = now_s();
    try {
        fm.load_fasta_files(files, deleted_fids, n_threads);
    } catch (const std::exception& e) {
        die(std::string("terminate called after throwing an instance of 'std::out_of_range': ") + e.what());
    }
    const double t_parse = now_s() - t0, t_fm = now_s() - t_fm0;

    unsigned nkept_f = fm.process_kept_functions(min_reps_required, ignored_functions);
    std::cout << "kept " << nkept_f << " functions\n";
    if (!kmer_data_dir.empty()) {
        if (!fm.write_function_index(kmer_data_dir)) die("cannot write function.index");
        std::ofstream(path_join(kmer_data_dir, "otu.index")).close();
        std::ofstream g(path_join(kmer_data_dir, "genomes"));
        g << "empty genomes\n";
    }

    std::cerr << "extract kmers\n";
    std::vector<BuildBatch> batches(files.size());
    // Sequence selection runs on a worker pool, file by file, while this thread streams every
    // finished file (in order) into the build: skm_build_add_batch packs it into a pinned staging
    // buffer whose DMA to HBM overlaps the next file's packing and the workers' selection.
    const size_t s0 = dump ? 0 : f0, s1 = dump ? files.size() : f1;
    std::mutex sel_mu;
    std::condition_variable sel_cv;
    std::vector<char> sel_done(files.size(), 0);
    std::atomic<size_t> sel_next{s0};
    auto sel_work = [&]() {
        for (size_t f; (f = sel_next.fetch_add(1)) < s1;) {
            select_build_sequences(fm, files[f], (unsigned)f, MaxSequencesPerFile, deleted_fids, batches[f]);
            std::lock_guard<std::mutex> g(sel_mu);
            sel_done[f] = 1;
            sel_cv.notify_all();
        }
    };
    std::vector<std::thread> sel_pool;
    for (int t = 0; t < std::max(1, n_threads - 1); ++t) sel_pool.emplace_back(sel_work);
    auto join_selection = [&]() {
        for (auto& t : sel_pool)
            if (t.joinable()) t.join();
    };
    if (dump) {
        hip_warm.join();
        join_selection();
        if (rank != 0) return 0;
        dump_extract(op.get("dump-extract"), files, batches);
        std::cerr << "wrote build input to " << op.get("dump-extract") << "\n";
        std::cerr << "phases: parse " << t_parse << " parse_files " << t_files << " defs " << t_defs << " fm_load " << t_fm
                  << "\n";
        if (!mesh.wait_children(err)) die(err);
        return 0;
    }

    skm_build* b = nullptr;
    skm_build_opts bo{};
    bo.k = K;
    bo.max_seqs_per_file = MaxSequencesPerFile;
    bo.n_functions = std::max(1u, nkept_f);
    bo.canonical_order = 1;
    bo.rank = rank;
    bo.world_size = world;
    auto check = [](int rc, const char* what) {
        if (rc) die(std::string(what) + ": " + skm_last_error());
    };
    hip_warm.join();
    const double t_create0 = now_s();
    check(skm_build_create(&b, &device, 1, &bo), "skm_build_create");
    {
        uint64_t nres = 0, nseq = 0;
        for (size_t f = f0; f < f1; ++f) {
            nres += files[f].residues.size();
            nseq += files[f].size();
        }
        check(skm_build_reserve(b, nres, nseq), "skm_build_reserve");
    }
    // test hook (tests/test_gpu_cli.py): this rank fails before joining the communicator
    if (const char* fail = std::getenv("SKM_CLI_FAIL_RANK"))
        if (world > 1 && std::atoi(fail) == rank) die("injected failure (SKM_CLI_FAIL_RANK)");
    skm_transport tp = mesh.transport();
    if (world > 1 && comm == "host") {
        check(skm_build_set_transport(b, &tp), "skm_build_set_transport");
    } else if (world > 1) {
        uint8_t id[128] = {0};
        if (rank == 0) check(skm_comm_unique_id(id), "skm_comm_unique_id");
        if (launched) {
            const std::string cf = op.get("comm-file", path_join(kmer_data_dir.empty() ? "." : kmer_data_dir, ".skm_comm_id"));
            if (!file_rendezvous(cf, rank, id, 300.0, err)) die(err);
        } else if (!mesh.share_id(id, err)) {
            die(err);
        }
        check(skm_build_set_comm(b, id), "skm_build_set_comm");
    }
    const double t_create = now_s() - t_create0;
    const double t_add0 = now_s();
    for (size_t f = f0; f < f1; ++f) {
        {
            std::unique_lock<std::mutex> g(sel_mu);
            sel_cv.wait(g, [&] { return sel_done[f] != 0; });
        }
        const BuildBatch& bb = batches[f];
        if (bb.off.empty()) continue;
        check(skm_build_add_batch(b, files[f].residues.data(), bb.off.data(), bb.len.data(), bb.func.data(),
                                  bb.seq_id.data(), bb.off.size()),
              "skm_build_add_batch");
    }
    join_selection();
    const double t_add = now_s() - t_add0;
    std::cerr << "process kmers\n";
    t0 = now_s();
    check(skm_build_prepare(b), "skm_build_prepare");
    const double t_prepare = now_s() - t0;
    t0 = now_s();
    check(skm_build_run(b), "skm_build_run");
    const double t_run = now_s() - t0;
    t0 = now_s();
    skm_kept kept{};
    check(skm_build_finish(b, &kept), "skm_build_finish");
    const double t_finish = now_s() - t0;
    float ph[12] = {0};
    int nph = skm_build_last_timings(b, ph, 12);
    const double t_build = t_prepare + t_run + t_finish;
    skm_build_destroy(b);
    if (rank != 0) {  // rank 0 holds every kept k-mer and the all-reduced statistics
        skm_kept_free(&kept);
        return 0;
    }
    std::cout << "Kept " << kept.n << " kmers\n";
    std::cout << "distinct_signatures=" << kept.distinct_signatures << "\n";
    std::cout << "num_seqs_with_a_signature=" << kept.n_seqs_with_signature << "\n";

    std::thread final_kmers_thread;
    double t_final_kmers = 0, t_mph = 0;
    if (!final_kmers.empty()) {
        if (path_is_relative(final_kmers)) {
            final_kmers = path_join(kmer_data_dir, final_kmers);
            std::cerr << "Updated final_kmers to " << quoted(final_kmers) << "\n";
        }
        final_kmers_thread = std::thread([&]() {
            const double tk = now_s();
            std::cerr << "writing kmers to " << quoted(final_kmers) << "\n";
            write_final_kmers(final_kmers, kept, std::max(1, n_threads / 2));
            t_final_kmers = now_s() - tk;
            std::cerr << "writing kmers to " << quoted(final_kmers) << " complete\n";
        });
    }

    {
        std::ofstream df(path_join(kmer_data_dir, "distinct_functions"));
        for (uint32_t f = 0; f < kept.n_functions; ++f)
            if (kept.distinct_functions[f]) df << f << "\t" << fm.lookup_function((uint16_t)f) << "\t" << kept.distinct_functions[f] << "\n";
    }

    const std::string report_dir = path_join(kmer_data_dir, "recall.report.d");
    if (mkdir(report_dir.c_str(), 0777) != 0) std::cerr << "mkdir " << quoted(report_dir) << " failed\n";
    const std::string fi_file = path_join(kmer_data_dir, "function.index");

    std::thread perfect_hash_thread;
    int ph_rc = 0;
    std::string ph_err;
    if (!ph_file.empty()) {
        if (path_is_relative(ph_file)) ph_file = path_join(kmer_data_dir, ph_file);
        if (path_is_relative(ph_data)) ph_data = path_join(kmer_data_dir, ph_data);
        const uint32_t seed = (uint32_t)std::strtoul(op.get("mph-seed", "1").c_str(), nullptr, 10);
        perfect_hash_thread = std::thread([&, seed]() {
            const double tm = now_s();
            std::cerr << "build perfect hash into " << quoted(ph_file) << " with data in " << quoted(ph_data) << "\n";
            ph_rc = skm_mph_build_device(kept.keys, kept.data, kept.n, seed, ph_file.c_str(), ph_data.c_str(), device);
            t_mph = now_s() - tm;
            if (ph_rc)
                ph_err = skm_last_error();
            else
                std::cerr << "Wrote " << kept.n << " values\n";
        });
    }

    // recall of the training sequences with the new k-mers (kmers-build-signatures.cc:238-349)
    std::vector<std::string> fidx;
    if (!read_function_index(fi_file, fidx, err)) die(err);
    std::cerr << "Begin recall\n";
    t0 = now_s();
    skm_db* kdb = nullptr;
    check(skm_db_open_kept(&kdb, kept.keys, kept.data, kept.n, device), "skm_db_open_kept");
    std::vector<const FastaFile*> fptr;
    for (auto& f : files) fptr.push_back(&f);
    std::vector<std::vector<SeqCall>> calls;
    double recall_dev_ms = 0;
    if (call_files(kdb, fptr, fidx, false, n_threads, calls, err, &recall_dev_ms)) die(err);
    skm_db_close(kdb);
    {  // one report per file (kmers-build-signatures.cc:300-349), the files on the host threads
        std::atomic<size_t> next_f{0};
        auto report = [&]() {
            for (size_t f; (f = next_f.fetch_add(1)) < files.size();) {
                std::map<std::string, std::string> data;  // saver::data (first emplace wins), sorted by id
                for (size_t r = 0; r < files[f].size(); ++r) {
                    const std::string& id = files[f].ids[r];
                    const SeqCall& c = calls[f][r];
                    std::string orig, orig_stripped;
                    fm.lookup_original_assignment(id, orig, orig_stripped);
                    if (orig_stripped != c.func && !data.count(id))
                        data.emplace(id, id + "\t" + orig + "\t" + orig_stripped + "\t" + c.func + "\t" +
                                             std::to_string((int)c.fi) + "\t" + fmt_g(c.score) + "\n");
                }
                std::string text;
                for (auto& e : data) text += e.second;
                std::ofstream of(path_join(report_dir, files[f].filename));
                of.write(text.data(), (std::streamsize)text.size());
            }
        };
        std::vector<std::thread> th;
        for (int t = 1; t < std::min<int>(n_threads, (int)files.size()); ++t) th.emplace_back(report);
        report();
        for (auto& t : th) t.join();
    }
    const double t_recall = now_s() - t0;
    const double t_recall_dev = recall_dev_ms / 1000.0;

    if (op.has("nudb-file")) std::cerr << "--nudb-file: NuDB output is not supported by this build; skipped\n";
    if (perfect_hash_thread.joinable()) {
        std::cerr << "Awaiting completion of perfect hash creation\n";
        perfect_hash_thread.join();
        if (ph_rc) die("perfect hash: " + ph_err);
    }
    if (final_kmers_thread.joinable()) {
        std::cerr << "Awaiting completion of final kmers dump\n";
        final_kmers_thread.join();
    }
    skm_kept_free(&kept);
    if (!mesh.wait_children(err)) die(err);
    std::cerr << "timing: parse " << t_parse << " s, build " << t_build << " s (device pipeline "
              << (nph > 7 ? ph[7] : 0.0f) << " ms), recall " << t_recall << " s, total " << now_s() - t_start << " s\n";
    // one machine-readable line of the phases (bench.py's cli_build leg)
    std::cerr << "phases: parse " << t_parse << " add " << t_add << " prepare " << t_prepare << " run " << t_run
              << " finish " << t_finish << " final_kmers " << t_final_kmers << " mph " << t_mph << " recall "
              << t_recall << " recall_device " << t_recall_dev << " total " << now_s() - t_start << " startup "
              << t_startup << " defs " << t_defs << " hip_init " << t_hip_init << " create " << t_create
              << " parse_files " << t_files << " fm_load " << t_fm << "\n";
    std::cerr << "all done\n";
    fast_exit(0);  // every output file is closed by now
}
