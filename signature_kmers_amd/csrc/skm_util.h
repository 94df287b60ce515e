// skm_util.h -- error plumbing and small device helpers shared by libskm translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

#include "../../include/skm.h"

namespace skm {

// Internal errors are C++ exceptions carrying an SKM_E_* code; every extern "C" entry point
// catches them (SKM_API_BEGIN/END) so nothing crosses the C boundary.
struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void set_last_error(const std::string& msg);

#define SKM_HIP(call)                                                                               \
    do {                                                                                            \
        hipError_t _e = (call);                                                                     \
        if (_e != hipSuccess)                                                                       \
            throw ::skm::Error(_e == hipErrorOutOfMemory ? SKM_E_OOM : SKM_E_HIP,                   \
                               std::string(#call) + ": " + hipGetErrorString(_e));                  \
    } while (0)

#define SKM_CHECK(cond, code, msg)                           \
    do {                                                     \
        if (!(cond)) throw ::skm::Error((code), (msg));      \
    } while (0)

#define SKM_API_BEGIN try {
#define SKM_API_END                                          \
    }                                                        \
    catch (const ::skm::Error& e) {                          \
        ::skm::set_last_error(e.what());                     \
        return e.code;                                       \
    }                                                        \
    catch (const std::bad_alloc&) {                          \
        ::skm::set_last_error("host allocation failed");     \
        return SKM_E_OOM;                                    \
    }                                                        \
    catch (const std::exception& e) {                        \
        ::skm::set_last_error(e.what());                     \
        return SKM_E_ARG;                                    \
    }                                                        \
    return SKM_OK;

// RAII device buffer (hipMalloc).  Grows but never shrinks.
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    void ensure(size_t n) {
        if (n <= bytes && p) return;
        if (p) SKM_HIP(hipFree(p));
        p = nullptr;
        bytes = 0;
        size_t alloc = n ? n : 16;
        SKM_HIP(hipMalloc(&p, alloc));
        bytes = alloc;
    }
    void release() {
        if (p) SKM_HIP(hipFree(p));
        p = nullptr;
        bytes = 0;
    }
    template <typename T>
    T* as() const {
        return reinterpret_cast<T*>(p);
    }
};

inline uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }
inline int ilog2_ceil(uint64_t x) {
    int b = 0;
    while ((1ull << b) < x) ++b;
    return b;
}

}  // namespace skm
