// kmers-matrix-distance -- drop-in for the reference's main (kmers-matrix-distance.cc:94-212).
//
//   kmers-matrix-distance [options] data-dir input-file
// Opens <data-dir>/kmer_data.mph + .dat (CmphKmerDb) into HBM, reads <data-dir>/function.index,
// parses the FASTA file (process_fasta_stream_parallel's parse: records with an empty id are
// dropped, every other id gets its SeqIdMap index in file order, call_functions.tcc:169-181) and
// prints "seq1\tseq2\tcount\n" for every pair of sequences sharing count signature-k-mer hits
// (:199-211) to stdout, like the reference (which parses -o but never uses it).  The pair counts
// run on the GPU (skm_matrix_*): lookups, hit_cb's length filter (:123-152), k-mer grouping, pair
// increments, compaction.  Order: sorted by (seq1 index, seq2 index) (the reference prints the
// hash order of its concurrent maps).  --min-hits, --debug-hits, --verbose and -j are accepted
// and, as in the reference main, have no effect on the output.
// Extra options: --device N, --max-tile-bytes B (bound on the dense count tile in HBM).
// Multi-GPU: --n-gpus N forks one process per GPU before any GPU use, on
// device --device + r (all on --device with --same-device, as the tests do on one GPU).  Every rank
// parses the input (the SeqIdMap indices are global) and looks up only its contiguous range of the
// records; the (k-mer, index) hits go to the k-mer's owner GPU and each k-mer's index set to the
// GPUs whose row band of the pair triangle (skm_matrix_tile_rows: bands of equal area) it has pairs
// in -- two all-to-alls, over RCCL (--comm rccl, default) or the forked ranks' socketpairs
// (--comm host) -- and rank r counts the pairs of its band.  Each rank streams its band's lines to
// rank 0, which prints the bands in rank order: the same lines in the same (seq1, seq2) order as
// one GPU.
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <unordered_map>
#include <vector>

#include "skm.h"
#include "skm_caller.h"
#include "skm_front.h"
#include "skm_mesh.h"

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

}  // namespace

int main(int argc, char** argv) {
    {  // libskm runs up to 10 streams at once: 16 hardware queues (read at the first HIP call)
        const char* q = getenv("GPU_MAX_HW_QUEUES");
        if (!q || atoi(q) < 16) setenv("GPU_MAX_HW_QUEUES", "16", 1);
    }
    Options op;
    op.specs = {{"data-dir", 'd', false, false},   {"input-file", 'i', false, false}, {"output-file", 'o', false, false},
                {"min-hits", 0, false, false},    {"n-threads", 'j', false, false},  {"debug-hits", 0, true, false},
                {"verbose", 0, true, false},      {"help", 'h', true, false},        {"device", 0, false, false},
                {"max-tile-bytes", 0, false, false}, {"n-gpus", 0, false, false},
                {"same-device", 0, true, false},  {"comm", 0, false, false}};
    op.positional = {"data-dir", "input-file"};
    std::string err;
    if (!op.parse(argc, argv, err)) die(err);
    if (op.has("help")) {
        std::cout << "Usage: " << argv[0] << " data-dir input-file\nAllowed options:\n"
                  << "  -d [ --data-dir ] arg       Data directory\n"
                  << "  -i [ --input-file ] arg     Input fasta file\n"
                  << "  -o [ --output-file ] arg    Output file\n"
                  << "  --min-hits arg              Minimum shared kmer hits to emit a match\n"
                  << "  -j [ --n-threads ] arg      Number of threads\n"
                  << "  --debug-hits                Debug kmer hits\n"
                  << "  --verbose                   Verbose mode\n"
                  << "  --device arg                HIP device ordinal (default 0)\n"
                  << "  --max-tile-bytes arg        HBM bound of the dense pair-count tile (default: 60 % of free)\n"
                  << "  --n-gpus arg                ranks (one process and GPU each): query ranges, k-mer owners,\n"
                  << "                              row bands of the triangle\n"
                  << "  --comm arg                  rccl (default) or host (socketpairs; ranks may share a GPU)\n"
                  << "  --same-device               every rank on --device\n"
                  << "  -h [ --help ]               show this help message\n\n";
        return 0;
    }
    const int ng = std::atoi(op.get("n-gpus", "1").c_str());
    if (ng < 1 || ng > 64) die("--n-gpus must be in [1, 64]");
    Mesh mesh;
    if (!mesh_fork(ng, mesh, err)) die(err);  // before any GPU call
    mesh.watch_children();
    const int device = std::atoi(op.get("device", "0").c_str()) + (op.has("same-device") ? 0 : mesh.rank);
    const std::string data_dir = op.get("data-dir");
    const std::string db_base = path_join(data_dir, "kmer_data");
    const std::string mph = db_base + ".mph", dat = db_base + ".dat";
    if (!file_exists(mph)) die("Database \"" + db_base + "\" does not exist");
    skm_db* db = nullptr;
    if (skm_db_open(&db, mph.c_str(), dat.c_str(), device)) die(skm_last_error());
    std::vector<std::string> fidx;
    if (!read_function_index(path_join(data_dir, "function.index"), fidx, err)) die(err);

    FastaFile f;
    const std::string in = op.get("input-file");
    if (!in.empty()) parse_fasta_file(in, f);  // an unreadable file parses as empty (fs::ifstream)
    // SeqIdMap (seq_id_map.h:12-27): index of the first record with each id
    std::unordered_map<std::string, uint32_t> id_to_index;
    std::vector<const std::string*> index_to_id;
    std::vector<uint32_t> seq_idx(f.size());
    for (size_t r = 0; r < f.size(); ++r) {
        auto it = id_to_index.find(f.ids[r]);
        if (it == id_to_index.end()) {
            it = id_to_index.emplace(f.ids[r], (uint32_t)index_to_id.size()).first;
            index_to_id.push_back(&f.ids[r]);
        }
        seq_idx[r] = it->second;
    }
    int hypo = -1;
    for (size_t i = 0; i < fidx.size(); ++i)
        if (fidx[i] == "hypothetical protein") {
            hypo = (int)i;
            break;
        }
    if (hypo < 0 && f.size() > 0) die("Cannot find hypothetical protein index");  // call_functions.tcc:269-274

    // this rank's records: the r-th of ng contiguous ranges
    const size_t ra = f.size() * (size_t)mesh.rank / (size_t)ng, rb = f.size() * (size_t)(mesh.rank + 1) / (size_t)ng;
    const size_t nmine = rb - ra;
    skm_matrix* m = nullptr;
    if (skm_matrix_create(&m, db, f.residues.data(), nmine ? f.off.data() + ra : nullptr,
                          nmine ? f.len.data() + ra : nullptr, nmine ? seq_idx.data() + ra : nullptr, nmine,
                          (uint32_t)index_to_id.size()))
        die(skm_last_error());
    skm_transport tp = mesh.transport();
    if (ng > 1) {
        // RCCL cannot put several ranks on one GPU: --same-device defaults to the host transport
        const std::string comm = op.get("comm", op.has("same-device") ? "host" : "rccl");
        if (comm == "rccl" && op.has("same-device")) die("--comm rccl needs one GPU per rank (drop --same-device)");
        if (comm == "host") {
            if (skm_matrix_set_transport(m, mesh.rank, ng, &tp)) die(skm_last_error());
        } else if (comm == "rccl") {
            uint8_t id[128];
            if (mesh.rank == 0 && skm_comm_unique_id(id)) die(skm_last_error());
            if (!mesh.share_id(id, err)) die(err);
            if (skm_matrix_set_comm(m, mesh.rank, ng, id)) die(skm_last_error());
        } else {
            die("--comm must be rccl or host");
        }
    }
    skm_matrix_opts mo;
    std::memset(&mo, 0, sizeof(mo));
    mo.hypo_index = hypo;
    mo.max_tile_bytes = std::strtoull(op.get("max-tile-bytes", "0").c_str(), nullptr, 10);
    if (skm_matrix_run(m, &mo)) die(skm_last_error());
    uint64_t ctr[5] = {0, 0, 0, 0, 0};
    skm_matrix_counters(m, ctr, 5);
    // ctr[4] counts the k-mers this rank owns (each k-mer has one owner): the ranks send theirs to
    // rank 0 ahead of their pair bands, so the line prints the whole map's size as one process does
    // (kmers-matrix-distance.cc:169)
    uint64_t hit_map = ctr[4];
    if (mesh.rank != 0) {
        if (write(mesh.fd[0], &hit_map, 8) != 8) die("write to rank 0 failed");
    } else {
        for (int q = 1; q < ng; ++q) {
            uint64_t v = 0;
            size_t got = 0;
            while (got < 8) {
                const ssize_t r = read(mesh.fd[q], reinterpret_cast<char*>(&v) + got, 8 - got);
                if (r <= 0) die("read from rank " + std::to_string(q) + " failed");
                got += (size_t)r;
            }
            hit_map += v;
        }
        std::cerr << "kmer_hit_map size " << hit_map << "\n";
    }
    skm_pairs pairs;
    if (skm_matrix_pairs(m, &pairs)) die(skm_last_error());
    if (mesh.rank == 0) std::cerr << "write output\n";
    // rank 0 prints to stdout; the other ranks stream their band to rank 0
    const int out_fd = mesh.rank == 0 ? 1 : mesh.fd[0];
    auto flush = [&](std::string& b) {
        size_t o = 0;
        while (o < b.size()) {
            const ssize_t w = write(out_fd, b.data() + o, b.size() - o);
            if (w <= 0) die("write failed");
            o += (size_t)w;
        }
        b.clear();
    };
    std::fflush(stdout);
    std::string buf;
    buf.reserve(1 << 20);
    for (uint64_t i = 0; i < pairs.n; ++i) {
        const uint32_t* p = pairs.pairs + 3 * i;
        buf += *index_to_id[p[0]];
        buf += '\t';
        buf += *index_to_id[p[1]];
        buf += '\t';
        buf += std::to_string(p[2]);
        buf += '\n';
        if (buf.size() > (1u << 20)) flush(buf);
    }
    flush(buf);
    skm_pairs_free(&pairs);
    skm_matrix_destroy(m);
    skm_db_close(db);
    if (mesh.rank != 0) {
        close(mesh.fd[0]);
        return 0;
    }
    // the other bands, in rank (= row) order
    std::vector<char> chunk(1 << 20);
    for (int q = 1; q < ng; ++q) {
        for (;;) {
            const ssize_t r = read(mesh.fd[q], chunk.data(), chunk.size());
            if (r < 0) die("read from rank " + std::to_string(q) + " failed");
            if (r == 0) break;
            std::string part(chunk.data(), (size_t)r);
            flush(part);
        }
    }
    if (!mesh.wait_children(err)) die(err);
    return 0;
}
