// ============================================================================================
//  oracle/ref_pin.cpp  --  TEST INFRASTRUCTURE ONLY (generates golden vectors; never shipped)
// ============================================================================================
//
//  A driver around the parts of the reference that compile here UNCHANGED with the image's g++
//  (std-only headers, no Boost / TBB / CMPH):
//    kmer_data.h        for_each_kmer<N>  (kmer_data.h:76-102), the annotate window iterator, and
//                       the StoredKmerData / KmerAttributes records (kmer_data.h:105-128)
//    fasta_parser.h/.cc FastaParser       (fasta_parser.h:38-144, fasta_parser.cc:17-36)
//    operators.h        split()           (operators.h:80-91), used by read_function_index
//                       (call_functions.tcc:143) and find_best_call's fusion keys (:487)
//  They are compiled from where they lie under /root/reference/src by oracle/Makefile.ref into
//  oracle/_ref/ref_pin (git-ignored).  Nothing of the reference is copied into this repository:
//  this file only #includes the reference headers and calls them.
//
//  tests/golden/make_golden_ref.py feeds it adversarial inputs and stores what it prints in
//  tests/golden/ref_windows.npz / ref_fasta.npz, which pin the oracle restatement, the product
//  front end and the device window iterator against the reference itself.
//
//  Protocol (stdin, one request per line; "-" = empty blob):
//    W <hex seq>    for_each_kmer<8> over the bytes -> "W <offsets comma separated or ->"
//    F <hex file>   FastaParser as SignatureBuilder::load_kmers_from_fasta drives it
//                   (signature_build.tcc:87-101: set_def_callback, parse(istream), then the
//                   caller's own parse_complete() again) with an error callback that records and
//                   continues (signature_build sets none; the parser then prints and continues);
//                   prints one line per callback "R <hex id> <hex def> <hex seq>" and per error
//                   "E <line> <hex message> <hex id>" in call order, then "END"
//    S <hex file>   FastaParser as function_map.h:128-237 / call_functions.tcc:165-182 drive it
//                   (set_callback (id, seq) only), the same output with "-" for the definition
//    P <hex s> <hex delim>   split(s, delim) -> "P <n> <hex part> ..." (n parts, "-" = empty)
//    L -            the record layouts -> "L <sizeof StoredKmerData> <alignof> <offsetof
//                   avg_from_end function_index mean median var> <sizeof KmerAttributes>
//                   <alignof> <offsetof func_index otu_index offset seq_id protein_length>"
// ============================================================================================
#include <algorithm>
#include <cstddef>
#include <cstdio>
#include <iostream>
#include <iterator>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "fasta_parser.h"
#include "kmer_data.h"
#include "operators.h"  // needs <vector>, <map>, <algorithm> from the includer (as call_functions.h does)

namespace {

std::string unhex(const std::string& h) {
    std::string s;
    if (h == "-") return s;
    for (size_t i = 0; i + 1 < h.size(); i += 2) s.push_back((char)std::stoi(h.substr(i, 2), nullptr, 16));
    return s;
}

std::string hex(const std::string& s) {
    static const char* d = "0123456789abcdef";
    if (s.empty()) return "-";
    std::string h;
    for (unsigned char c : s) {
        h.push_back(d[c >> 4]);
        h.push_back(d[c & 15]);
    }
    return h;
}

void run_windows(const std::string& seq) {
    std::string offs;
    for_each_kmer<8>(seq, [&](const std::array<char, 8>&, size_t off) {
        if (!offs.empty()) offs += ",";
        offs += std::to_string(off);
    });
    std::cout << "W " << (offs.empty() ? "-" : offs) << "\n";
}

void run_fasta(const std::string& data, bool with_def) {
    std::vector<std::string> out;
    FastaParser parser;
    if (with_def)
        parser.set_def_callback([&](const std::string& id, const std::string& def, const std::string& seq) {
            out.push_back("R " + hex(id) + " " + hex(def) + " " + hex(seq));
        });
    else
        parser.set_callback([&](const std::string& id, const std::string& seq) {
            out.push_back("R " + hex(id) + " - " + hex(seq));
        });
    parser.set_error_callback([&](const std::string& err, int line, const std::string id) {
        out.push_back("E " + std::to_string(line) + " " + hex(err) + " " + hex(id));
        return true;
    });
    std::istringstream is(data);
    parser.parse(is);
    parser.parse_complete();
    for (auto& l : out) std::cout << l << "\n";
    std::cout << "END\n";
}

void run_split(const std::string& s, const std::string& delim) {
    const std::vector<std::string> parts = split(s, delim);
    std::cout << "P " << parts.size();
    for (const auto& p : parts) std::cout << " " << hex(p);
    std::cout << "\n";
}

void run_layout() {
    std::cout << "L " << sizeof(StoredKmerData) << " " << alignof(StoredKmerData) << " "
              << offsetof(StoredKmerData, avg_from_end) << " " << offsetof(StoredKmerData, function_index) << " "
              << offsetof(StoredKmerData, mean) << " " << offsetof(StoredKmerData, median) << " "
              << offsetof(StoredKmerData, var) << " " << sizeof(KmerAttributes) << " " << alignof(KmerAttributes)
              << " " << offsetof(KmerAttributes, func_index) << " " << offsetof(KmerAttributes, otu_index) << " "
              << offsetof(KmerAttributes, offset) << " " << offsetof(KmerAttributes, seq_id) << " "
              << offsetof(KmerAttributes, protein_length) << "\n";
}

}  // namespace

int main() {
    std::cerr.rdbuf(nullptr);  // the parser's own "Error found" prints; the callback records them
    std::string line;
    while (std::getline(std::cin, line)) {
        if (line.size() < 3) continue;
        const char op = line[0];
        if (op == 'P') {  // two hex fields
            const size_t sp = line.find(' ', 2);
            run_split(unhex(line.substr(2, sp - 2)), unhex(line.substr(sp + 1)));
            continue;
        }
        if (op == 'L') {
            run_layout();
            continue;
        }
        const std::string arg = unhex(line.substr(2));
        if (op == 'W')
            run_windows(arg);
        else if (op == 'F')
            run_fasta(arg, true);
        else if (op == 'S')
            run_fasta(arg, false);
    }
    return 0;
}
