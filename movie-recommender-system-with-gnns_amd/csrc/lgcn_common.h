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

// ---- Adam element arithmetic shared by the row-lazy Adam (lgcn_rowadam.hip) and the catch-up
// that rides in block-split launches (lgcn_spmm.hip, lgcn_adam_ride_t) ----------------------------

struct AdamK {
    float omb1, beta2, omb2, eps;
    int markstein;  // the step-constant division by Markstein's correction (div_step)
};

// sqrt(v) / c with c = bc2_sqrt, the step's constant, and rc = 1 / c (both fp32, rc correctly
// rounded): Markstein's correction q0 = s * rc, r = fma(-c, q0, s) (exact), q = fma(r, rc, q0)
// gives the correctly rounded quotient — the value IEEE division gives — in 3 instructions instead
// of the division's 9 (v_div_scale x 2, v_rcp, 4 FMAs, v_div_fmas, v_div_fixup). Proven for the
// schedule of beta2 = 0.999 (the reference's Adam default): tools/markstein_check.c tries every
// significand of a binade — by scale invariance every normal s; s = sqrt(v) is never subnormal —
// for each of its 10,030 distinct step constants, 0 mismatches (profiles/r03x_adam/). The proof
// covers the constants built from the double beta2 = 0.999 exactly: lgcn_adam_consts records that in
// consts[0].x (kConstsMarkstein), and the replays take the shortcut only when it is set; any other
// beta2 — np.float32(0.999) passed as a double included — takes the IEEE division. That the device's
// constants equal the checker's host-libm ones is a GPU test (test_gpu_training.py).
__device__ __forceinline__ float div_step(float s, float c, float rc, int markstein) {
    if (markstein) {
        const float q0 = s * rc;
        return __builtin_fmaf(__builtin_fmaf(-c, q0, s), rc, q0);
    }
    return s / c;
}

// adam_elem (lgcn_rowadam.hip; the dense kernel's lgcn_optim.hip adam_elem) with g == 0 (a missed
// step), the same floats with fewer instructions: g * coef and g * g are +0, so v + omb2 * 0 ==
// v * beta2 (v >= 0 and omb2 finite: adding +0 changes nothing), and m + omb1 * (0 - m) ==
// m - omb1 * m (0 - m == -m exactly for m != 0, m is never -0).
__device__ __forceinline__ void adam_elem_zero(float& p, float& m, float& v, float step_size, float bc2_sqrt,
                                               float rc, const AdamK& k) {
    m = m - k.omb1 * m;
    v = v * k.beta2;
    const float denom = div_step(sqrtf(v), bc2_sqrt, rc, k.markstein) + k.eps;
    p = p + step_size * (m / denom);
}

// A row's zero-gradient replays from step `from` through `upto` on LPR lanes x NV float4 of a
// row of d = 4 * LPR * NV floats (P / M / V already offset to the lane's first float4).
template <int LPR, int NV>
__device__ __forceinline__ void adam_replay_row(float4* P, float4* M, float4* V, int64_t from, int64_t upto,
                                                const float4* __restrict__ consts, const AdamK& k) {
    float4 p[NV], m[NV], v[NV];
#pragma unroll
    for (int q = 0; q < NV; ++q) {
        p[q] = P[q * LPR];
        m[q] = M[q * LPR];
        v[q] = V[q * LPR];
    }
    for (int64_t s = from; s <= upto; ++s) {
        const float4 c = consts[s];
        const float rc = c.z;  // 1 / c.y, from lgcn_adam_consts
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            adam_elem_zero(p[q].x, m[q].x, v[q].x, c.x, c.y, rc, k);
            adam_elem_zero(p[q].y, m[q].y, v[q].y, c.x, c.y, rc, k);
            adam_elem_zero(p[q].z, m[q].z, v[q].z, c.x, c.y, rc, k);
            adam_elem_zero(p[q].w, m[q].w, v[q].w, c.x, c.y, rc, k);
        }
    }
#pragma unroll
    for (int q = 0; q < NV; ++q) {
        P[q * LPR] = p[q];
        M[q * LPR] = m[q];
        V[q * LPR] = v[q];
    }
}

// The riding catch-up (lgcn_adam_ride_t) as the device sees it.
struct AdamRide {
    const int32_t* rows;
    int64_t n_rows;
    const uint8_t* skip;
    float* p_lo;
    float* p_hi;
    float* m_lo;
    float* m_hi;
    float* v_lo;
    float* v_hi;
    int64_t split;
    int32_t* last;
    const int64_t* step;
    const float4* consts;
    AdamK k;
    int32_t max_replays;
};

// Ride entry i on lane l of its LPR-lane group: advance the row by at most max_replays
// zero-gradient steps, never past the step in progress (step[0] + 1).
template <int LPR, int NV>
__device__ __forceinline__ void adam_ride_entry(const AdamRide& R, int64_t i, int l) {
    if (i >= R.n_rows) return;
    const int64_t row = R.rows[i];
    if (R.skip && R.skip[row]) return;
    const int64_t from = int64_t(R.last[row]) + 1;
    int64_t upto = from - 1 + R.max_replays;
    const int64_t target = R.step[0] + 1;
    if (upto > target) upto = target;
    if (from > upto) return;
    AdamK k = R.k;
    if (R.consts[0].x != 1.0f) k.markstein = 0;  // constants not from the proven schedule
    constexpr int64_t d = int64_t(LPR) * NV * 4;
    const int64_t off = row < R.split ? row * d : (row - R.split) * d;
    float4* P = reinterpret_cast<float4*>((row < R.split ? R.p_lo : R.p_hi) + off) + l;
    float4* M = reinterpret_cast<float4*>((row < R.split ? R.m_lo : R.m_hi) + off) + l;
    float4* V = reinterpret_cast<float4*>((row < R.split ? R.v_lo : R.v_hi) + off) + l;
    adam_replay_row<LPR, NV>(P, M, V, from, upto, R.consts, k);
    if (l == 0) R.last[row] = static_cast<int32_t>(upto);
}

// Bits needed to radix-sort keys in [0, n).
inline int key_bits(int64_t n) {
    int b = 1;
    while ((int64_t(1) << b) < n) ++b;
    return b;
}

}  // namespace lgcn
