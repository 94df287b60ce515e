// skm-front-probe -- test hook for the host front end's hand-coded Boost.Regex matchers.
// Reads hex-encoded strings, one per line, from stdin; prints one line per input with the
// hex-encoded results, tab separated:
//   split_func_comment: func sep comment | is_truncated_comment(s) | strip_func_comment(s) |
//   roles_of_function(s) joined by 0x01 | genome defline match (0/1) func genome | fig genome (0/1) genome
// skm-front-probe --fasta FILE KEEP: parse FILE (KEEP 1 = with residues, 0 = headers-only) and print
// one line per record (hex id, hex definition, offset, length), then "n_residues N residues R".
// skm-front-probe --fasta-hex: one hex-encoded FASTA file image per stdin line ("-" = empty); per
// image, one line per record "R <hex id> <hex def> <hex residues>" and one per parse error the
// parser reported "E <line> <hex message> <hex id>", in the order the parser produced them, then
// "END" (the shape of oracle/ref_pin's output, so tests compare with the reference's FastaParser).
// skm-front-probe --split: one "<hex s> <hex delim>" per stdin line -> "P <n> <hex part> ..." from
// the shared split (skm_strutil.h; oracle/ref_pin's P output shape).
// skm-front-probe --function-index FILE: read_function_index -> one "<index> <hex name>" per slot.
#include <cstdio>
#include <iostream>
#include <sstream>
#include <string>

#include "../skm_strutil.h"
#include "skm_caller.h"
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
    if (argc == 3 && std::string(argv[1]) == "--function-index") {
        std::vector<std::string> table;
        std::string err;
        if (!read_function_index(argv[2], table, err)) {
            std::cerr << err << "\n";
            return 1;
        }
        for (size_t i = 0; i < table.size(); ++i) std::cout << i << " " << hex(table[i]) << "\n";
        return 0;
    }
    std::string line;
    if (argc == 2 && std::string(argv[1]) == "--split") {
        while (std::getline(std::cin, line)) {
            const size_t sp = line.find(' ');
            const auto un = [](const std::string& h) { return h == "-" ? std::string() : unhex(h); };
            const auto parts = skm_str::split(un(line.substr(0, sp)), un(line.substr(sp + 1)));
            std::cout << "P " << parts.size();
            for (const auto& p : parts) std::cout << " " << hex(p);
            std::cout << "\n";
        }
        return 0;
    }
    if (argc == 2 && std::string(argv[1]) == "--fasta-hex") {
        while (std::getline(std::cin, line)) {
            const std::string img = line == "-" ? std::string() : unhex(line);
            std::ostringstream errs;
            std::streambuf* old = std::cerr.rdbuf(errs.rdbuf());
            FastaFile f;
            parse_fasta_buffer(img.data(), img.size(), f, true);
            std::cerr.rdbuf(old);
            // records and errors interleave in parse order: a record is emitted when the next
            // '>' (or the end) is read, so each error line precedes the records emitted after it;
            // the probe reports errors with the record they were found in (by the id shown)
            std::istringstream es(errs.str());
            std::string el;
            while (std::getline(es, el)) {
                // "Error found: <msg> at line <n> id='<id>'"
                const std::string pre = "Error found: ";
                const size_t at = el.rfind(" at line "), idq = el.rfind(" id='");
                if (el.compare(0, pre.size(), pre) != 0 || at == std::string::npos || idq == std::string::npos) {
                    std::cout << "X " << hex(el) << "\n";
                    continue;
                }
                const std::string msg = el.substr(pre.size(), at - pre.size());
                const std::string ln = el.substr(at + 9, idq - at - 9);
                const std::string id = el.substr(idq + 5, el.size() - idq - 6);
                std::cout << "E " << ln << " " << hex(msg) << " " << hex(id) << "\n";
            }
            for (size_t r = 0; r < f.size(); ++r)
                std::cout << "R " << hex(f.ids[r]) << " " << hex(f.defs[r]) << " "
                          << hex(std::string(f.residues.begin() + f.off[r], f.residues.begin() + f.off[r] + f.len[r]))
                          << "\n";
            std::cout << "END\n";
        }
        return 0;
    }
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
