// skm-front-probe -- test hook for the host front end's hand-coded Boost.Regex matchers.
// Reads hex-encoded strings, one per line, from stdin; prints one line per input with the
// hex-encoded results, tab separated:
//   split_func_comment: func sep comment | is_truncated_comment(s) | strip_func_comment(s) |
//   roles_of_function(s) joined by 0x01 | genome defline match (0/1) func genome | fig genome (0/1) genome
// skm-front-probe --fasta FILE KEEP: parse FILE (KEEP 1 = with residues, 0 = headers-only) and print
// one line per record (hex id, hex definition, offset, length), then "n_residues N residues R".
#include <cstdio>
#include <iostream>
#include <string>

#include "skm_front.h"

using namespace skmf;

static std::string unhex(const std::string& h) {
    std::string s;
    for (size_t i = 0; i + 1 < h.size(); i += 2) s.push_back((char)std::stoi(h.substr(i, 2), nullptr, 16));
    return s;
}
static std::string hex(const std::string& s) {
    static const char* d = "0123456789abcdef";
    std::string h;
    for (unsigned char c : s) {
        h.push_back(d[c >> 4]);
        h.push_back(d[c & 15]);
    }
    return h.empty() ? "-" : h;
}

int main(int argc, char** argv) {
    if (argc == 4 && std::string(argv[1]) == "--fasta") {
        FastaFile f;
        if (!parse_fasta_file(argv[2], f, std::string(argv[3]) == "1")) return 1;
        for (size_t r = 0; r < f.size(); ++r)
            std::cout << hex(f.ids[r]) << "\t" << hex(f.defs[r]) << "\t" << f.off[r] << "\t" << f.len[r] << "\n";
        std::cout << "n_residues " << f.n_residues << " residues " << f.residues.size() << "\n";
        return 0;
    }
    std::string line;
    while (std::getline(std::cin, line)) {
        std::string s = line == "-" ? std::string() : unhex(line);
        std::string f, sep, c;
        split_func_comment(s, f, sep, c);
        std::string roles;
        auto r = roles_of_function(s);
        for (size_t i = 0; i < r.size(); ++i) roles += (i ? "\x01" : "") + r[i];
        std::string gf, gg, fg;
        bool gm = match_genome_defline(s, gf, gg);
        bool fm = search_fig_genome(s, fg);
        std::cout << hex(f) << "\t" << hex(sep) << "\t" << hex(c) << "\t" << (is_truncated_comment(s) ? 1 : 0) << "\t"
                  << hex(strip_func_comment(s)) << "\t" << r.size() << "\t" << hex(roles) << "\t" << (gm ? 1 : 0)
                  << "\t" << hex(gf) << "\t" << hex(gg) << "\t" << (fm ? 1 : 0) << "\t" << hex(fg) << "\n";
    }
    return 0;
}
