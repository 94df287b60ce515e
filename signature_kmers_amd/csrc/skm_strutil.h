// skm_strutil.h -- the reference's string split, shared by libskm (find_best_call's fusion keys)
// and the host front end (read_function_index).  Header-only, std only.
#pragma once

#include <string>
#include <vector>

namespace skm_str {

// split(s, delim) of operators.h:80-91: the delimiter is a whole string; every field is kept,
// empty ones included (an empty s gives one empty field, a trailing delimiter a trailing empty
// field).  Pinned against the reference compiled unchanged (tests/golden/ref_split.npz).  An
// empty delimiter never terminates in the reference; here it yields s as one field.
inline std::vector<std::string> split(const std::string& s, const std::string& delim) {
    std::vector<std::string> out;
    if (delim.empty()) {
        out.push_back(s);
        return out;
    }
    std::string::size_type start = 0, end = 0;
    while (end != std::string::npos) {
        end = s.find(delim, start);
        out.push_back(s.substr(start, end == std::string::npos ? std::string::npos : end - start));
        start = end + delim.size();
    }
    return out;
}

}  // namespace skm_str
