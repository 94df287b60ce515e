// skm_front.cpp -- host front end (see skm_front.h for the reference mapping).
#include "skm_front.h"

#include <cerrno>
#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <emmintrin.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <cstdint>
#include <functional>
#include <iterator>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <thread>

namespace skmf {

namespace {

inline bool is_space(unsigned char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r'; }
inline bool is_digit(unsigned char c) { return c >= '0' && c <= '9'; }

struct CharClass {
    bool alpha[256];
    bool res[256];  // a residue byte inside a data line: a letter or '*'
    CharClass() {
        for (int c = 0; c < 256; ++c) {
            alpha[c] = (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z');
            res[c] = alpha[c] || c == '*';
        }
    }
};
const CharClass kCls;

// the first byte at or after q (< end) that is not a residue byte (letter or '*'): 16 bytes per
// step (SSE2 compares), then byte by byte
inline const unsigned char* residue_run_end(const unsigned char* q, const unsigned char* end) {
    const __m128i k20 = _mm_set1_epi8(0x20), ka = _mm_set1_epi8('a'), k25 = _mm_set1_epi8(25),
                  kst = _mm_set1_epi8('*');
    while (end - q >= 16) {
        const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(q));
        const __m128i t = _mm_sub_epi8(_mm_or_si128(v, k20), ka);  // 0..25 for a letter of either case
        const __m128i ok = _mm_or_si128(_mm_cmpeq_epi8(_mm_min_epu8(t, k25), t), _mm_cmpeq_epi8(v, kst));
        const unsigned m = (unsigned)_mm_movemask_epi8(ok);
        if (m != 0xFFFFu) return q + __builtin_ctz(~m);
        q += 16;
    }
    while (q < end && kCls.res[*q]) ++q;
    return q;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// FastaParser (fasta_parser.h:38-144).  The callback fires on '>' in s_id_or_data and once more
// from parse_complete(); callers ignore records with an empty id, so only non-empty ids are kept.
// ---------------------------------------------------------------------------------------------
// Keep = false is the headers-only form (ids, definitions, offsets and lengths, no residue
// bytes): what a rank needs of the files another rank builds.
namespace {
template <bool Keep>
void parse_fasta_impl(const char* buf, size_t n, FastaFile& out) {
    enum State { S_START, S_ID, S_DEF, S_DATA, S_ID_OR_DATA } st = S_START;
    int line = 1;
    std::string id, def;
    uint64_t nres = Keep ? out.residues.size() : out.n_residues;
    uint64_t seq_start = nres;
    auto emit = [&]() {
        if (!id.empty()) {
            out.ids.push_back(id);
            out.defs.push_back(def);
            out.off.push_back(seq_start);
            out.len.push_back((uint32_t)(nres - seq_start));
        } else {
            nres = seq_start;
            if (Keep) out.residues.resize(seq_start);
        }
        id.clear();
        def.clear();
        seq_start = nres;
    };
    // the file's reports, written to std::cerr in one piece at the end (one flushed write per
    // report serialised the parse threads on the stream: ~30 per genome file of the C4 input)
    std::string reports;
    auto error = [&](const std::string& msg) {
        reports += "Error found: " + msg + " at line " + std::to_string(line) + " id='" + id + "'\n";
    };
    const unsigned char* p = reinterpret_cast<const unsigned char*>(buf);
    const unsigned char* end = p + n;
    {  // the record tables sized once ('>' bytes bound the records)
        size_t recs = 0;
        for (const void* q = buf; (q = std::memchr(q, '>', (size_t)(end - static_cast<const unsigned char*>(q)))) != nullptr;
             q = static_cast<const unsigned char*>(q) + 1)
            ++recs;
        out.ids.reserve(out.ids.size() + recs);
        out.defs.reserve(out.defs.size() + recs);
        out.off.reserve(out.off.size() + recs);
        out.len.reserve(out.len.size() + recs);
    }
    while (p < end) {
        const unsigned char c = *p++;
        if (c == '\n') ++line;
        if (c == '\r') continue;
        switch (st) {
            case S_START:
                if (c != '>')
                    error("Missing >");
                else
                    st = S_ID;
                break;
            case S_ID:
                if (c == ' ' || c == '\t') {
                    def.push_back((char)c);
                    st = S_DEF;
                } else if (c == '\n') {
                    st = S_DATA;
                } else {
                    // the rest of the id in one append (the bytes the per-byte states would add)
                    const unsigned char* q = p;
                    while (q < end && *q != ' ' && *q != '\t' && *q != '\n' && *q != '\r') ++q;
                    id.push_back((char)c);
                    id.append(reinterpret_cast<const char*>(p), (size_t)(q - p));
                    p = q;
                }
                break;
            case S_DEF:
                if (c == '\n') {
                    st = S_DATA;
                } else {
                    const unsigned char* q = p;
                    while (q < end && *q != '\n' && *q != '\r') ++q;
                    def.push_back((char)c);
                    def.append(reinterpret_cast<const char*>(p), (size_t)(q - p));
                    p = q;
                }
                break;
            case S_DATA:
                if (c == '\n') {
                    st = S_ID_OR_DATA;
                } else if (kCls.res[c]) {
                    // fast path: the rest of the sequence body while it is residue lines -- each
                    // line's run, its '\n', and the next line's first byte when it is a letter
                    // (what S_DATA -> S_ID_OR_DATA -> S_DATA would do byte by byte); anything else
                    // goes back to the states above
                    const unsigned char* a = p - 1;
                    for (;;) {
                        const unsigned char* q = residue_run_end(p, end);
                        if (Keep) out.residues.insert(out.residues.end(), a, q);
                        nres += (uint64_t)(q - a);
                        p = q;
                        if (!(end - p >= 2 && p[0] == '\n' && kCls.alpha[p[1]])) break;
                        ++line;
                        a = p + 1;
                        p += 2;
                    }
                } else {
                    error(std::string("Bad data character '") + (char)c + "'");
                }
                break;
            case S_ID_OR_DATA:
                if (c == '>') {
                    emit();
                    st = S_ID;
                } else if (c == '\n') {
                } else if (kCls.alpha[c]) {
                    if (Keep) out.residues.push_back(c);
                    ++nres;
                    st = S_DATA;
                } else {
                    error(std::string("Bad id or data character '") + (char)c + "'");
                }
                break;
        }
    }
    emit();  // parse_complete()
    out.n_residues = nres;
    if (!reports.empty()) std::cerr << reports << std::flush;
}
}  // namespace

void parse_fasta_buffer(const char* buf, size_t n, FastaFile& out, bool keep_residues) {
    if (keep_residues)
        parse_fasta_impl<true>(buf, n, out);
    else
        parse_fasta_impl<false>(buf, n, out);
}

bool parse_fasta_file(const std::string& path, FastaFile& out, bool keep_residues) {
    out = FastaFile();
    out.path = path;
    out.filename = path_filename(path);
    // the whole file into an uninitialised buffer (no zero fill: ~1.3 MB per genome file)
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) return false;
    struct stat sb;
    if (::fstat(fd, &sb) != 0) {
        ::close(fd);
        return false;
    }
    const size_t n = (size_t)std::max<off_t>(sb.st_size, 0);
    std::unique_ptr<char[]> buf(new char[std::max<size_t>(n, 1)]);
    size_t got = 0;
    while (got < n) {
        const ssize_t r = ::read(fd, buf.get() + got, n - got);
        if (r <= 0) break;
        got += (size_t)r;
    }
    ::close(fd);
    if (keep_residues) out.residues.reserve(got);
    parse_fasta_buffer(buf.get(), got, out, keep_residues);
    out.residues.shrink_to_fit();
    return true;
}

bool parse_fasta_files(const std::vector<std::string>& paths, std::vector<FastaFile>& out, int n_threads,
                       std::string& err, const std::vector<char>* keep_residues) {
    out.assign(paths.size(), FastaFile());
    std::atomic<size_t> next{0};
    std::atomic<bool> ok{true};
    std::string bad;
    auto work = [&]() {
        for (size_t i; (i = next.fetch_add(1)) < paths.size();) {
            if (!parse_fasta_file(paths[i], out[i], !keep_residues || (*keep_residues)[i])) {
                ok = false;
                bad = paths[i];
            }
        }
    };
    int nt = std::max(1, std::min<int>(n_threads, (int)paths.size()));
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work);
    work();
    for (auto& t : th) t.join();
    if (!ok) err = "cannot read " + bad;
    return ok;
}

// ---------------------------------------------------------------------------------------------
// paths (path_utils.h)
// ---------------------------------------------------------------------------------------------
std::string path_join(const std::string& dir, const std::string& name) {
    if (dir.empty()) return name;
    if (dir.back() == '/') return dir + name;
    return dir + "/" + name;
}
std::string path_filename(const std::string& p) {
    size_t s = p.find_last_of('/');
    return s == std::string::npos ? p : p.substr(s + 1);
}
bool path_is_relative(const std::string& p) { return p.empty() || p[0] != '/'; }
bool ensure_directory(const std::string& dir) {
    if (dir.empty()) return true;
    struct stat sb;
    if (stat(dir.c_str(), &sb) == 0 && S_ISDIR(sb.st_mode)) return true;
    if (mkdir(dir.c_str(), 0777) == 0) return true;
    // forked ranks create the output directory concurrently: losing the race is success
    return errno == EEXIST && stat(dir.c_str(), &sb) == 0 && S_ISDIR(sb.st_mode);
}

bool list_regular_files(const std::string& dir, std::vector<std::string>& out, std::string& err) {
    DIR* d = opendir(dir.c_str());
    if (!d) {
        err = "cannot open directory " + dir;
        return false;
    }
    while (struct dirent* e = readdir(d)) {
        if (!std::strcmp(e->d_name, ".") || !std::strcmp(e->d_name, "..")) continue;
        std::string p = path_join(dir, e->d_name);
        struct stat sb;
        if (stat(p.c_str(), &sb) == 0 && S_ISREG(sb.st_mode)) out.push_back(p);
    }
    closedir(d);
    return true;
}

std::vector<std::string> load_lines(const std::string& path, bool* ok) {
    std::vector<std::string> v;
    std::ifstream f(path);
    if (ok) *ok = (bool)f;
    std::string line;
    while (std::getline(f, line, '\n')) v.push_back(line);
    return v;
}

// ---------------------------------------------------------------------------------------------
// seed_utils.h regexes as hand-coded matchers (Boost.Regex Perl semantics, leftmost match,
// \s = [ \t\n\v\f\r]).
// ---------------------------------------------------------------------------------------------

// regex_match(str, "(.*?)(?:\s+(\#+)\s+(.*))?"): the lazy prefix stops at the first position i
// where str[i..] = \s+ #+ \s+ .*  (the optional group is tried before the empty tail).
void split_func_comment(const std::string& s, std::string& func, std::string& sep, std::string& comment) {
    const size_t n = s.size();
    for (size_t i = 0; i < n; ++i) {
        if (!is_space((unsigned char)s[i])) continue;
        size_t j = i;
        while (j < n && is_space((unsigned char)s[j])) ++j;
        if (j < n && s[j] == '#') {
            size_t k = j;
            while (k < n && s[k] == '#') ++k;
            if (k < n && is_space((unsigned char)s[k])) {
                size_t c = k;
                while (c < n && is_space((unsigned char)s[c])) ++c;
                func = s.substr(0, i);
                sep = s.substr(j, k - j);
                comment = s.substr(c);
                return;
            }
        }
        i = j - 1;  // positions inside this blank run give the same outcome
    }
    func = s;
    sep.clear();
    comment.clear();
}

// regex_search(str, "^(?:frag|missing|trunc)"); '^' also matches after a newline (Perl mode)
bool is_truncated_comment(const std::string& s) {
    auto at = [&](size_t p) {
        return s.compare(p, 4, "frag") == 0 || s.compare(p, 7, "missing") == 0 || s.compare(p, 5, "trunc") == 0;
    };
    if (at(0)) return true;
    for (size_t p = 0; p + 1 < s.size(); ++p)
        if (s[p] == '\n' && at(p + 1)) return true;
    return false;
}

// regex_replace(str, "(\s*\#.*$)", ""): everything from the blank run before the first '#'.
std::string strip_func_comment(const std::string& s) {
    size_t h = s.find('#');
    if (h == std::string::npos) return s;
    size_t w = h;
    while (w > 0 && is_space((unsigned char)s[w - 1])) --w;
    return s.substr(0, w);
}

// sregex_token_iterator(stripped, "\s+[/@]\s+|\s*;\s+", -1)
std::vector<std::string> roles_of_function(const std::string& function) {
    const std::string s = strip_func_comment(function);
    const size_t n = s.size();
    std::vector<std::string> ret;
    auto match_at = [&](size_t i, size_t& e) -> bool {
        // alternative 1: \s+[/@]\s+
        size_t j = i;
        while (j < n && is_space((unsigned char)s[j])) ++j;
        if (j > i && j < n && (s[j] == '/' || s[j] == '@')) {
            size_t k = j + 1, k0 = k;
            while (k < n && is_space((unsigned char)s[k])) ++k;
            if (k > k0) {
                e = k;
                return true;
            }
        }
        // alternative 2: \s*;\s+
        if (j < n && s[j] == ';') {
            size_t k = j + 1, k0 = k;
            while (k < n && is_space((unsigned char)s[k])) ++k;
            if (k > k0) {
                e = k;
                return true;
            }
        }
        return false;
    };
    size_t last = 0;
    bool any = false;
    for (size_t i = 0; i < n; ++i) {
        size_t e;
        if (match_at(i, e)) {
            ret.push_back(s.substr(last, i - last));
            last = e;
            i = e - 1;
            any = true;
        }
    }
    if (!any) {
        if (n) ret.push_back(s);
    } else if (last != n) {
        ret.push_back(s.substr(last));
    }
    return ret;
}

// regex_match(def, "\s+(.*)\s+\[([^]]+)\]$"): the greedy (.*) ends at the blank right before the
// last '[' whose bracket content (no ']') runs to a final ']'.
bool match_genome_defline(const std::string& def, std::string& func_part, std::string& genome) {
    const size_t n = def.size();
    if (n < 4 || def[n - 1] != ']') return false;
    size_t q = std::string::npos;
    for (size_t i = n - 1; i-- > 0;) {
        if (def[i] == ']') break;
        if (def[i] == '[' && i + 1 < n - 1 && i >= 1 && is_space((unsigned char)def[i - 1])) {
            q = i;
            break;
        }
    }
    if (q == std::string::npos) return false;
    const size_t p = q - 1;  // the blank consumed by the second \s+
    if (p < 1 || !is_space((unsigned char)def[0])) return false;
    size_t R = 0;
    while (R < n && is_space((unsigned char)def[R])) ++R;
    const size_t start = std::min(R, p);
    func_part = def.substr(start, p - start);
    genome = def.substr(q + 1, n - 1 - (q + 1));
    return true;
}

bool search_fig_genome(const std::string& id, std::string& genome) {
    for (size_t pos = id.find("fig|"); pos != std::string::npos; pos = id.find("fig|", pos + 1)) {
        size_t a = pos + 4, b = a;
        while (b < id.size() && is_digit((unsigned char)id[b])) ++b;
        if (b == a || b >= id.size() || id[b] != '.') continue;
        size_t c = b + 1, d = c;
        while (d < id.size() && is_digit((unsigned char)id[d])) ++d;
        if (d == c) continue;
        genome = id.substr(a, d - a);
        return true;
    }
    return false;
}

static bool match_genome_id(const std::string& s) {  // regex_match(s, "\d+\.\d+")
    size_t b = 0;
    while (b < s.size() && is_digit((unsigned char)s[b])) ++b;
    if (b == 0 || b >= s.size() || s[b] != '.') return false;
    size_t d = b + 1;
    while (d < s.size() && is_digit((unsigned char)s[d])) ++d;
    return d > b + 1 && d == s.size();
}

// ---------------------------------------------------------------------------------------------
// accumulator_set<float, stats<mean, median, variance, count>>: float sum, P^2 (p = 0.5) in
// float, iterative variance over the lazy mean (features updated count, sum, median, variance).
// ---------------------------------------------------------------------------------------------
void FloatStats::add(float x) {
    ++count;
    sum += x;
    if (count <= 5) {
        heights[count - 1] = x;
        if (count == 5) std::sort(heights, heights + 5);
    } else {
        static const float incr[5] = {0.0f, 0.25f, 0.5f, 0.75f, 1.0f};
        size_t cell;
        if (x < heights[0]) {
            heights[0] = x;
            cell = 1;
        } else if (heights[4] <= x) {
            heights[4] = x;
            cell = 4;
        } else {
            cell = (size_t)(std::upper_bound(heights, heights + 5, x) - heights);
        }
        for (size_t i = cell; i < 5; ++i) actual[i] += 1.0f;
        for (size_t i = 0; i < 5; ++i) desired[i] += incr[i];
        for (size_t i = 1; i <= 3; ++i) {
            float d = desired[i] - actual[i];
            float dp = actual[i + 1] - actual[i];
            float dm = actual[i - 1] - actual[i];
            float hp = (heights[i + 1] - heights[i]) / dp;
            float hm = (heights[i - 1] - heights[i]) / dm;
            if ((d >= 1. && dp > 1) || (d <= -1. && dm < -1)) {
                short sign_d = static_cast<short>(d / std::abs(d));
                float h = heights[i] + sign_d / (dp - dm) * ((sign_d - dm) * hp + (dp - sign_d) * hm);
                if (heights[i - 1] < h && h < heights[i + 1]) {
                    heights[i] = h;
                } else {
                    if (d > 0) heights[i] += hp;
                    if (d < 0) heights[i] -= hm;
                }
                actual[i] += sign_d;
            }
        }
    }
    if (count > 1) {
        float mean = sum / (float)count;
        float tmp = x - mean;
        variance = variance * (float)(count - 1) / (float)count + tmp * tmp / (float)(count - 1);
    }
}

void fast_exit(int code) {
    std::cout.flush();
    std::cerr.flush();
    std::fflush(nullptr);
    const char* full = std::getenv("SKM_CLI_FULL_EXIT");
    if (full && std::atoi(full) != 0) std::exit(code);
    std::_Exit(code);
}

double process_age_s() {
    // /proc/self/stat field 22: start time in clock ticks after boot; /proc/uptime: seconds after boot
    std::ifstream st("/proc/self/stat"), up("/proc/uptime");
    std::string line;
    double uptime = 0;
    if (!std::getline(st, line) || !(up >> uptime)) return 0;
    const size_t rp = line.rfind(')');  // the command name may hold spaces
    if (rp == std::string::npos) return 0;
    std::istringstream is(line.substr(rp + 2));
    std::string tok;
    unsigned long long start = 0;
    for (int field = 3; field <= 22 && (is >> tok); ++field)
        if (field == 22) start = std::strtoull(tok.c_str(), nullptr, 10);
    const long hz = sysconf(_SC_CLK_TCK);
    return hz > 0 ? std::max(0.0, uptime - (double)start / (double)hz) : 0.0;
}

std::string fmt_g(double v) {
    char b[64];
    std::snprintf(b, sizeof b, "%g", v);
    return b;
}

// ---------------------------------------------------------------------------------------------
// FunctionMap
// ---------------------------------------------------------------------------------------------
namespace {
// one definition line's fields (load_id_assignments)
struct IdLine {
    std::string id, func, stripped;
    bool bad = false, truncated = false;
};
void parse_id_line(const char* b, const char* e, IdLine& x) {
    const std::string line(b, e);
    const size_t s = line.find('\t');
    if (s == std::string::npos) {
        x.bad = true;
        return;
    }
    const size_t s2 = line.find('\t', s + 1);
    x.id = line.substr(0, s);
    x.func = s2 == std::string::npos ? line.substr(s + 1) : line.substr(s + 1, s2 - s - 1);
    std::string delim, comment;
    split_func_comment(x.func, x.stripped, delim, comment);
    x.truncated = delim == "#" && is_truncated_comment(comment);
}
// f(0..n-1) on up to `threads` std::threads (the caller's included)
void par_for(int n, int threads, const std::function<void(int)>& f) {
    std::vector<std::thread> th;
    std::atomic<int> next{0};
    auto work = [&] {
        for (int i; (i = next.fetch_add(1)) < n;) f(i);
    };
    for (int t = 1; t < std::min(threads, n); ++t) th.emplace_back(work);
    work();
    for (auto& x : th) x.join();
}
}  // namespace

void FunctionMap::load_id_assignments(const std::string& path, int threads) {
    load_id_assignments(std::vector<std::string>{path}, threads);
}

void FunctionMap::load_id_assignments(const std::vector<std::string>& paths, int threads) {
    // every file's lines, split as std::getline returns them ('\n'; a last line without one
    // included) and parsed on the host threads, file by file
    std::vector<std::vector<IdLine>> lines(paths.size());
    par_for((int)paths.size(), std::max(1, threads), [&](int fi) {
        std::ifstream f(paths[(size_t)fi], std::ios::binary);
        if (!f) return;
        const std::string buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
        std::vector<IdLine>& out = lines[(size_t)fi];
        for (size_t p = 0; p < buf.size();) {
            const size_t q = buf.find('\n', p);
            const size_t e = q == std::string::npos ? buf.size() : q;
            out.emplace_back();
            parse_id_line(buf.data() + p, buf.data() + e, out.back());
            p = q == std::string::npos ? buf.size() : q + 1;
        }
    });
    size_t n = 0;
    for (size_t fi = 0; fi < paths.size(); ++fi) {
        n += lines[fi].size();
        for (size_t i = 0; i < lines[fi].size(); ++i)
            if (lines[fi][i].bad) std::cerr << "bad line " << i + 1 << " in file \"" << paths[fi] << "\"\n";
    }
    // the three tables are independent: one thread each, every one in file and line order (a
    // later assignment of an id replaces an earlier one, as operator[] = does)
    par_for(3, threads > 1 ? 3 : 1, [&](int k) {
        auto& tab = k == 0 ? original_assignment_stripped_ : k == 1 ? original_assignment_ : id_function_map_;
        tab.reserve(tab.size() + n);
        for (const auto& fl : lines)
            for (const IdLine& x : fl) {
                if (x.bad) continue;
                if (k == 0) tab[x.id] = x.stripped;
                if (k == 1) tab[x.id] = x.func;
                if (k == 2 && !x.truncated) tab[x.id] = x.stripped;
            }
    });
}

void FunctionMap::load_fasta_files(const std::vector<FastaFile>& files, const std::set<std::string>& deleted_fids,
                                   int threads) {
    // per file: the kept records' (index, function before the id table) and the file's genome --
    // set by its first record that passes the checks and never changed after (load_fasta_file)
    struct FileRecs {
        std::vector<uint32_t> rec;
        std::vector<std::string> func;
        std::string genome, msg;
        size_t bad = SIZE_MAX;  // the first blank definition line (load_fasta_file throws there)
    };
    std::vector<FileRecs> out(files.size());
    par_for((int)files.size(), std::max(1, threads), [&](int fi) {
        const FastaFile& f = files[(size_t)fi];
        FileRecs& o = out[(size_t)fi];
        o.rec.reserve(f.size());
        o.func.reserve(f.size());
        std::string genome;
        for (size_t r = 0; r < f.size(); ++r) {
            const std::string& id = f.ids[r];
            const std::string& def = f.defs[r];
            if (deleted_fids.count(id)) continue;
            std::string func;
            if (!def.empty()) {
                const size_t x = def.find_first_not_of(" \t");
                if (x == std::string::npos) {
                    o.bad = r;
                    break;
                }
                func = def.substr(x);
            }
            std::string genome_loc, fpart, g;
            if (match_genome_defline(def, fpart, g)) {
                std::string delim, comment;
                split_func_comment(fpart, func, delim, comment);
                if (delim == "#" && is_truncated_comment(comment)) continue;
                genome_loc = g;
            }
            if (genome.empty()) {
                if (def.empty())
                    search_fig_genome(id, genome);
                else if (!genome_loc.empty())
                    genome = genome_loc;
            }
            if (genome.empty()) {
                genome = f.filename;
                if (!match_genome_id(genome)) o.msg += "cannot determine genome from file \"" + f.path + "\"\n";
            }
            o.rec.push_back((uint32_t)r);
            o.func.push_back(std::move(func));
        }
        o.genome = genome;
    });
    size_t total = 0;
    for (const auto& o : out) total += o.rec.size();
    id_function_map_.reserve(id_function_map_.size() + total);
    // the ids' table entries found on the host threads (no writer yet; the entries an insert adds
    // below do not move the others); the ones not found are added in record order below
    std::vector<std::vector<std::string*>> cur_of(files.size());
    par_for((int)files.size(), std::max(1, threads), [&](int fi) {
        const FileRecs& o = out[(size_t)fi];
        auto& c = cur_of[(size_t)fi];
        c.resize(o.rec.size());
        for (size_t k = 0; k < o.rec.size(); ++k) {
            auto it = id_function_map_.find(files[(size_t)fi].ids[o.rec[k]]);
            c[k] = it == id_function_map_.end() ? nullptr : &it->second;
        }
    });
    // the function tables' entries of each function name, found once (std::map nodes are stable),
    // and the genome last added to its set (an equal insert is a no-op)
    struct FuncRef {
        std::set<std::string>* genomes;
        FloatStats* acc;
        const std::string* last;
    };
    std::unordered_map<std::string, FuncRef> fref;
    for (size_t fi = 0; fi < files.size(); ++fi) {
        const FastaFile& f = files[fi];
        FileRecs& o = out[fi];
        std::cerr << o.msg;
        for (size_t k = 0; k < o.rec.size(); ++k) {
            const uint32_t r = o.rec[k];
            std::string& func = o.func[k];
            std::string& cur = cur_of[fi][k] ? *cur_of[fi][k] : id_function_map_[f.ids[r]];
            if (cur.empty()) {
                if (!func.empty()) cur = func;
            } else {
                func = cur;
            }
            if (func.empty()) continue;
            auto it = fref.find(func);
            if (it == fref.end())
                it = fref.emplace(func, FuncRef{&function_genome_map_[func], &function_accumulators_[func], nullptr}).first;
            FuncRef& x = it->second;
            if (!x.last || *x.last != o.genome) x.last = &*x.genomes->insert(o.genome).first;
            x.acc->add((float)f.len[r]);
        }
        if (o.bad != SIZE_MAX)
            throw std::out_of_range("blank definition line for " + f.ids[o.bad] + " in " + f.path);
    }
}

void FunctionMap::load_fasta_file(const FastaFile& f, const std::set<std::string>& deleted_fids) {
    std::string genome;
    for (size_t r = 0; r < f.size(); ++r) {
        const std::string& id = f.ids[r];
        const std::string& def = f.defs[r];
        if (deleted_fids.count(id)) continue;
        std::string func;
        if (!def.empty()) {
            size_t x = def.find_first_not_of(" \t");
            if (x == std::string::npos)  // def.substr(npos) throws in the reference
                throw std::out_of_range("blank definition line for " + id + " in " + f.path);
            func = def.substr(x);
        }
        std::string genome_loc, fpart, g;
        if (match_genome_defline(def, fpart, g)) {
            std::string delim, comment;
            split_func_comment(fpart, func, delim, comment);
            if (delim == "#" && is_truncated_comment(comment)) continue;
            genome_loc = g;
        }
        if (genome.empty()) {
            if (def.empty())
                search_fig_genome(id, genome);
            else if (!genome_loc.empty())
                genome = genome_loc;
        }
        if (genome.empty()) {
            genome = f.filename;
            if (!match_genome_id(genome)) std::cerr << "cannot determine genome from file \"" << f.path << "\"\n";
        }
        std::string& cur = id_function_map_[id];
        if (cur.empty()) {
            if (!func.empty()) cur = func;
        } else {
            func = cur;
        }
        if (!func.empty()) {
            function_genome_map_[func].insert(genome);
            function_accumulators_[func].add((float)f.len[r]);
        }
    }
}

unsigned FunctionMap::process_kept_functions(int min_reps_required, const std::set<std::string>& ignored) {
    std::set<std::string> kept;
    for (const auto& e : function_genome_map_) {
        const std::string& function = e.first;
        bool ok = (int)e.second.size() >= min_reps_required || good_functions_.count(function);
        if (!ok) {
            for (const auto& role : roles_of_function(function))
                if (good_roles_.count(role)) {
                    ok = true;
                    break;
                }
        }
        if (ok) kept.insert(function);
    }
    kept.insert("hypothetical protein");
    for (const auto& fn : ignored) {
        std::cerr << "Ignore '" << fn << "'\n";
        kept.erase(fn);
    }
    unsigned short next = 0;
    function_index_map_.clear();
    index_function_map_.clear();
    for (const auto& f : kept) {
        unsigned short id = next++;
        function_index_map_[f] = id;
        index_function_map_[id] = f;
    }
    return next;
}

bool FunctionMap::write_function_index(const std::string& dir) const {
    std::ofstream of(path_join(dir, "function.index"));
    if (!of) return false;
    for (const auto& ent : index_function_map_) {
        FloatStats& a = function_accumulators_[ent.second];
        const double mean = a.mean(), median = a.median(), var = a.variance;
        const double dev = std::sqrt(var);
        of << ent.first << "\t" << ent.second << "\t" << (int)a.count << "\t" << fmt_g(mean) << "\t" << fmt_g(median)
           << "\t" << fmt_g(var) << "\t" << fmt_g(dev) << "\n";
    }
    return (bool)of;
}

std::string FunctionMap::lookup_function_of_id(const std::string& id) const {
    auto it = id_function_map_.find(id);
    return it == id_function_map_.end() ? std::string() : it->second;
}
uint16_t FunctionMap::lookup_index(const std::string& func) const {
    auto it = function_index_map_.find(func);
    return it == function_index_map_.end() ? (uint16_t)0xFFFF : it->second;
}
std::string FunctionMap::lookup_function(uint16_t idx) const {
    auto it = index_function_map_.find(idx);
    return it == index_function_map_.end() ? std::string() : it->second;
}
void FunctionMap::lookup_original_assignment(const std::string& id, std::string& func, std::string& stripped) const {
    auto x = original_assignment_.find(id);
    if (x != original_assignment_.end()) {
        func = x->second;
        stripped = original_assignment_stripped_.at(id);
    }
}
std::vector<std::string> FunctionMap::index_table() const {
    std::vector<std::string> t;
    for (const auto& e : index_function_map_) {
        if (t.size() <= e.first) t.resize((size_t)e.first + 1);
        t[e.first] = e.second;
    }
    return t;
}

void select_build_sequences(const FunctionMap& fm, const FastaFile& f, unsigned file_number,
                            unsigned max_seqs_per_file, const std::set<std::string>& deleted_fids,
                            BuildBatch& out) {
    out = BuildBatch();
    unsigned next_sequence_id = file_number * max_seqs_per_file;
    std::unordered_map<std::string, uint16_t> fi_cache;
    for (size_t r = 0; r < f.size(); ++r) {
        const std::string& id = f.ids[r];
        if (!deleted_fids.empty() && deleted_fids.count(id)) continue;
        std::string func = fm.lookup_function_of_id(id);
        if (func.empty()) continue;
        unsigned seq_id = next_sequence_id++;
        auto it = fi_cache.find(func);
        uint16_t fi = it != fi_cache.end() ? it->second : (fi_cache[func] = fm.lookup_index(func));
        if (fi == 0xFFFF) continue;
        out.off.push_back(f.off[r]);
        out.len.push_back(f.len[r]);
        out.func.push_back(fi);
        out.seq_id.push_back(seq_id);
    }
}

// ---------------------------------------------------------------------------------------------
// command line
// ---------------------------------------------------------------------------------------------
bool Options::parse(int argc, char** argv, std::string& err) {
    auto find_long = [&](const std::string& n) -> const Spec* {
        for (auto& s : specs)
            if (s.name == n) return &s;
        return nullptr;
    };
    auto find_short = [&](char c) -> const Spec* {
        for (auto& s : specs)
            if (s.short_name && s.short_name == c) return &s;
        return nullptr;
    };
    size_t pos_i = 0;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        const Spec* sp = nullptr;
        std::string inline_val;
        bool has_inline = false;
        if (a.size() > 2 && a[0] == '-' && a[1] == '-') {
            std::string nm = a.substr(2);
            size_t eq = nm.find('=');
            if (eq != std::string::npos) {
                inline_val = nm.substr(eq + 1);
                nm = nm.substr(0, eq);
                has_inline = true;
            }
            sp = find_long(nm);
            if (!sp) {
                err = "unrecognised option '" + a + "'";
                return false;
            }
        } else if (a.size() >= 2 && a[0] == '-' && a[1] != '-') {
            sp = find_short(a[1]);
            if (!sp) {
                err = "unrecognised option '" + a + "'";
                return false;
            }
            if (a.size() > 2) {
                inline_val = a.substr(2);
                has_inline = true;
            }
        } else {
            if (pos_i >= positional.size()) {
                err = "too many positional options";
                return false;
            }
            const std::string& pn = positional[pos_i];
            const Spec* ps = find_long(pn);
            values[pn].push_back(a);
            if (!(ps && ps->multi)) ++pos_i;
            continue;
        }
        auto& dst = values[sp->name];
        if (sp->flag) {
            dst.push_back("1");
            continue;
        }
        if (has_inline) {
            dst.push_back(inline_val);
            if (!sp->multi) continue;
        } else {
            if (i + 1 >= argc) {
                err = "option '--" + sp->name + "' requires an argument";
                return false;
            }
            dst.push_back(argv[++i]);
        }
        if (sp->multi)
            while (i + 1 < argc && argv[i + 1][0] != '-') dst.push_back(argv[++i]);
    }
    return true;
}

std::string Options::get(const std::string& n, const std::string& dflt) const {
    auto it = values.find(n);
    return it == values.end() || it->second.empty() ? dflt : it->second.back();
}
std::vector<std::string> Options::all(const std::string& n) const {
    auto it = values.find(n);
    return it == values.end() ? std::vector<std::string>() : it->second;
}

}  // namespace skmf
