// Shared helpers for liblgcn.so (gfx950). Error state is thread-local; the only other global
// state is the process-wide tuning struct (lgcn_set_tuning, set before work is issued), so every
// entry point is re-entrant across threads and devices.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "lgcn.h"

namespace lgcn {

inline char* err_buf() {
    static thread_local char buf[512] = {0};
    return buf;
}

inline int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(err_buf(), 512, fmt, ap);
    va_end(ap);
    return code;
}

inline int check_hip(hipError_t e, const char* what) {
    if (e == hipSuccess) return LGCN_OK;
    return fail(static_cast<int>(e), "%s: %s", what, hipGetErrorString(e));
}

// A kernel launch error is reported by hipGetLastError(); it never synchronises.
inline int check_launch(const char* what) { return check_hip(hipGetLastError(), what); }

// The process-wide tuning (csrc/lgcn_tuning.cpp; defaults = the measured choices).
const lgcn_tuning_t& tuning();

inline hipStream_t as_stream(lgcn_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Carve a caller-provided workspace into 256-byte aligned pieces.
struct Carver {
    char* base;
    size_t cap;
    size_t used = 0;
    bool ok = true;
    template <class T>
    T* take(size_t count) {
        size_t off = align_up(used, 256);
        size_t bytes = count * sizeof(T);
        if (base == nullptr || off + bytes > cap) {
            ok = false;
            used = off + bytes;
            return nullptr;
        }
        used = off + bytes;
        return reinterpret_cast<T*>(base + off);
    }
};

constexpr int kBlock = 256;  // 4 waves of 64

inline unsigned grid_for(int64_t n, int block = kBlock, int64_t cap = 1 << 20) {
    int64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return static_cast<unsigned>(g);
}

// Bits needed to radix-sort keys in [0, n).
inline int key_bits(int64_t n) {
    int b = 1;
    while ((int64_t(1) << b) < n) ++b;
    return b;
}

}  // namespace lgcn
