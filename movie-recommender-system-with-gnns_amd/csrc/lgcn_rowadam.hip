// Row-lazy Adam for the two embedding tables of the sparse Cluster-GCN batch step
// (reference utils/train_test.py:95-96: clip_grad_norm_(1) + optim.Adam(lr=1e-3), dense on
// [U, d] + [I, d] every step).
//
// A row with a zero gradient still moves under Adam (m and v decay, p steps by m/denom), but its
// update is a fixed function of (p, m, v, step constants): applied later, in order, it gives the
// same floats. So a row is brought up to date only when it is next touched — replaying its missed
// zero-gradient steps with exactly the arithmetic the dense kernel (lgcn_optim.hip adam_elem) uses
// — and the rows a batch never reaches are not streamed every step. lgcn_row_adam_flush replays
// every row up to the current step (epoch end / before parameters are read).
//
//   last[r]   the last step applied to row r (int32 per global row id)
//   consts[t] (step_size_t, bc2_sqrt_t, 1 / bc2_sqrt_t, 0), t = 1..T: the per-step constants, filled by
//             lgcn_adam_consts with the same double formulas as lgcn_adam_prologue
//   step      device int64: the number of completed steps (capturable; lgcn_row_adam_update
//             advances it)
//
// Rows live in two tables (r < split: lo[r], else hi[r - split]) like everywhere else.

#include <climits>
#include <cmath>

#include "lgcn_common.h"
#include "lgcn_exact.h"
#include "lgcn_reg.h"

using namespace lgcn;

namespace {

struct RowTables {
    float* p_lo;
    float* p_hi;
    float* g_lo;
    float* g_hi;
    float* m_lo;
    float* m_hi;
    float* v_lo;
    float* v_hi;
    int64_t split;
    int32_t d;
};

struct RowList {
    const int32_t* rows_a;   // row ids
    int64_t n_a;
    const int64_t* keys_b;   // rows keys_b[j] + off_b
    int64_t n_b;
    int64_t off_b;
    const uint8_t* first_b;  // nullable: entry j counts only if first_b[j] (its key's first occurrence)
    const uint8_t* skip_b;   // nullable: ... and !skip_b[row] (the row is already in list a)
};

struct AdamK {
    float omb1, beta2, omb2, eps;
    int markstein;  // the step-constant division by Markstein's correction (div_step)
    // zero-gradient replays in the exact shortened sqrt / division (fast_horizon) when set:
    // 1 / -log2 of the per-step decay bounds of |m| and v (rounding included), host-computed
    int fast;
    float inv_lm, inv_lv;
};

template <class T>
__device__ __forceinline__ T* trow(T* lo, T* hi, int64_t split, int64_t r, int64_t d) {
    return r < split ? lo + r * d : hi + (r - split) * d;
}

// sqrt(v) / c with c = bc2_sqrt, the step's constant, and rc = 1 / c (both fp32, rc correctly
// rounded): Markstein's correction q0 = s * rc, r = fma(-c, q0, s) (exact), q = fma(r, rc, q0)
// gives the correctly rounded quotient — the value IEEE division gives — in 3 instructions instead
// of the division's 9 (v_div_scale x 2, v_rcp, 4 FMAs, v_div_fmas, v_div_fixup). Proven for the
// schedule of beta2 = 0.999 (the reference's Adam default): tools/markstein_check.c tries every
// significand of a binade — by scale invariance every normal s; s = sqrt(v) is never subnormal —
// for each of its 10,030 distinct step constants, 0 mismatches (profiles/r03x_adam/). The proof
// covers the constants built from the double beta2 = 0.999 exactly: lgcn_adam_consts records that in
// consts[0].x (kConstsMarkstein), and k_row_adam takes the shortcut only when it is set; any other
// beta2 — np.float32(0.999) passed as a double included — takes the IEEE division. That the device's
// constants equal the checker's host-libm ones is a GPU test (test_gpu_training.py).
__device__ __forceinline__ float div_step(float s, float c, float rc, int markstein) {
    if (markstein) {
        const float q0 = s * rc;
        return __builtin_fmaf(__builtin_fmaf(-c, q0, s), rc, q0);
    }
    return s / c;
}

// the dense kernel's element update (lgcn_optim.hip adam_elem), verbatim
__device__ __forceinline__ void adam_elem(float& p, float& g, float& m, float& v, float coef, float step_size,
                                          float bc2_sqrt, float rc, const AdamK& k) {
    g = g * coef;
    m = m + k.omb1 * (g - m);
    v = v * k.beta2;
    v = v + k.omb2 * (g * g);
    const float denom = div_step(sqrtf(v), bc2_sqrt, rc, k.markstein) + k.eps;
    p = p + step_size * (m / denom);
}

// adam_elem with g == 0 (a missed step), the same floats with fewer instructions: g * coef and
// g * g are +0, so v + omb2 * 0 == v * beta2 (v >= 0 and omb2 finite: adding +0 changes nothing),
// and m + omb1 * (0 - m) == m - omb1 * m (0 - m == -m exactly for m != 0, m is never -0).
__device__ __forceinline__ void adam_elem_zero(float& p, float& m, float& v, float step_size, float bc2_sqrt,
                                               float rc, const AdamK& k) {
    m = m - k.omb1 * m;
    v = v * k.beta2;
    const float denom = div_step(sqrtf(v), bc2_sqrt, rc, k.markstein) + k.eps;
    p = p + step_size * (m / denom);
}

// adam_elem_zero with lgcn_exact.h's shortened sqrt and division: bitwise the same while every
// operand stays in their ranges — v == +0 or v >= 2^-96, m == +0 or 2^-40 <= |m| <= 2^40, and the
// denominator in [2^-40, 2^40] (eps >= 2^-40 and v <= 2^60 with c >= 2^-9, checked by the host and
// by fast_horizon).
__device__ __forceinline__ void adam_elem_zero_fast(float& p, float& m, float& v, float step_size, float bc2_sqrt,
                                                    float rc, const AdamK& k) {
    m = m - k.omb1 * m;
    v = v * k.beta2;
    const float denom = div_step(sqrt_normal(v), bc2_sqrt, rc, 1) + k.eps;
    p = p + step_size * div_window(m, denom);
}

// How many zero-gradient replays from (m, v) stay inside adam_elem_zero_fast's ranges. A replay
// multiplies |m| by at least f_m = (1 - omb1)(1 - 2^-22) and v by at least f_v = beta2 (1 - 2^-23)
// (the two roundings of m - omb1 * m, the one of v * beta2), and makes neither larger, so from
// |m| >= 2^e the first floor((e + 40) / -log2 f_m) replays keep |m| >= 2^-40 (inv_lm = 1 /
// -log2 f_m, rounded down), likewise v >= 2^-96; +0 stays +0. 0 (never fast) for anything else:
// |m| > 2^40, v > 2^60, a negative zero, NaN or inf.
__device__ __forceinline__ int64_t horizon_m(float m, float inv) {
    const uint32_t b = __float_as_uint(m);
    if (b == 0u) return INT64_MAX;
    const int e = static_cast<int>((b >> 23) & 0xffu) - 127;
    if (e > 39 || e < -40) return 0;
    return static_cast<int64_t>(static_cast<float>(e + 40) * inv);
}

__device__ __forceinline__ int64_t horizon_v(float v, float inv) {
    const uint32_t b = __float_as_uint(v);
    if (b == 0u) return INT64_MAX;
    const int e = static_cast<int>((b >> 23) & 0xffu) - 127;
    if ((b >> 31) || e > 59 || e < -96) return 0;
    return static_cast<int64_t>(static_cast<float>(e + 96) * inv);
}

constexpr int64_t kFastMinReplays = 3;

template <int NV>
__device__ __forceinline__ int64_t fast_horizon(const float4 (&m)[NV], const float4 (&v)[NV], const AdamK& k) {
    int64_t h = INT64_MAX;
#pragma unroll
    for (int q = 0; q < NV; ++q) {
        h = min(h, min(min(horizon_m(m[q].x, k.inv_lm), horizon_m(m[q].y, k.inv_lm)),
                       min(horizon_m(m[q].z, k.inv_lm), horizon_m(m[q].w, k.inv_lm))));
        h = min(h, min(min(horizon_v(v[q].x, k.inv_lv), horizon_v(v[q].y, k.inv_lv)),
                       min(horizon_v(v[q].z, k.inv_lv), horizon_v(v[q].w, k.inv_lv))));
    }
    return h;
}

// Entry i of the list: its row, and whether it passes the first_b filter. An entry that fails it
// may be padding (ids -1 in the exchange's slot arrays), so `row` must not be dereferenced for it.
__device__ __forceinline__ bool list_entry(const RowList& L, int64_t i, int64_t& row) {
    if (i < L.n_a) {
        row = L.rows_a[i];
        return true;
    }
    const int64_t j = i - L.n_a;
    row = L.keys_b[j] + L.off_b;
    return !L.first_b || L.first_b[j];
}

// ... and the skip_b filter (only for entries that passed list_entry: skip_b is indexed by row)
__device__ __forceinline__ bool list_skipped(const RowList& L, int64_t i, int64_t row) {
    return i >= L.n_a && L.skip_b && L.skip_b[row];
}

__device__ __forceinline__ bool list_row(const RowList& L, int64_t i, int64_t& row) {
    return list_entry(L, i, row) && !list_skipped(L, i, row);
}

// consts[0].x: 1 when the constants come from the double beta2 = 0.999 exactly (the schedule
// tools/markstein_check.c proves the div_step shortcut for), else 0. Set by a call starting at t = 1,
// cleared by any call with another beta2.
constexpr double kMarksteinBeta2 = 0.999;

__global__ void k_adam_consts(float4* __restrict__ consts, int64_t t0, int64_t t1, float lr, double beta1,
                              double beta2) {
    const int64_t t = t0 + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x == 0 && (t0 == 1 || beta2 != kMarksteinBeta2))
        consts[0] = make_float4(beta2 == kMarksteinBeta2 ? 1.0f : 0.0f, 0.0f, 0.0f, 0.0f);
    if (t > t1) return;
    const double bc1 = 1.0 - pow(beta1, double(t));
    const double bc2 = 1.0 - pow(beta2, double(t));
    const float c = static_cast<float>(sqrt(bc2));
    // z: 1 / c in fp32 (correctly rounded), the reciprocal div_step's shortcut multiplies by —
    // built once here instead of once per replayed step and lane
    consts[t] = make_float4(static_cast<float>(-(static_cast<double>(lr) / bc1)), c, 1.0f / c, 0.0f);
}

// One LPR-lane group per list entry (or per row for the flush). mode 0: catch the row up to
// step[0] with zero-gradient replays (duplicates skipped through claim stamps). mode 1: catch up
// to step[0] then apply step[0]+1 with the row's gradient (the list must be duplicate-free:
// first_b / skip_b). mode 2 (flush): every row in [0, n_rows) up to step[0].
template <int LPR, int NV>
__global__ __launch_bounds__(kBlock) void k_row_adam(RowTables T, RowList L, int64_t n_rows, int32_t* __restrict__ last,
                                                     int32_t* __restrict__ claim, const int64_t* __restrict__ step,
                                                     const float4* __restrict__ consts, AdamK k,
                                                     const float* __restrict__ clip, int mode, RegRows R) {
    constexpr int GPB = kBlock / LPR;
    const int g = threadIdx.x / LPR;
    const int l = threadIdx.x % LPR;
    const int64_t i = int64_t(blockIdx.x) * GPB + g;
    // mode 3: the update after lgcn_row_grad_norm already advanced the counter to t + 1
    const bool upd = mode == 1 || mode == 3;
    const int64_t t = step[0] - (mode == 3 ? 1 : 0);
    if (consts[0].x != 1.0f) k.markstein = 0;  // constants not from the proven schedule
    int64_t row;
    int32_t last_row;
    if (mode == 2) {
        if (i >= n_rows) return;
        row = i;
        last_row = last[row];
    } else {
        if (i >= L.n_a + L.n_b) return;
        if (!list_entry(L, i, row)) return;  // filtered (or padding: row may be -1)
        // issued beside the skip filter and the claim instead of after them: only this row's
        // winner ever writes last[row] (its lane 0, at the end), so the value is the same
        last_row = last[row];
        if (list_skipped(L, i, row)) return;
        if (mode == 0) {
            // duplicates in the catch-up list: the first claimer of this step's stamp does the work
            int won = 0;
            if (l == 0) won = atomicExch(claim + row, static_cast<int32_t>(2 * t)) != static_cast<int32_t>(2 * t);
            won = __shfl(won, 0, LPR);
            if (!won) return;
        }
    }
    const int64_t from = int64_t(last_row) + 1;
    const int64_t upto = t;  // zero-gradient replays through step t
    // a catch-up (or flush) of a row that is already current touches nothing (on the planted
    // graph ~95 % of a step's negative rows were updated the step before: no p/m/v traffic)
    if (!upd && from > upto) return;
    const float coef = (upd && clip) ? clip[1] : 1.0f;
    const int64_t d = T.d;
    // the step's reg-gradient rows (R.w_lo set, ABI 10): added to the gradient here, from the row's
    // parameters as the forward read them (before any replay below), instead of by passes after the
    // backward
    const bool reg = upd && R.w_lo != nullptr;
    int64_t nf = 0, nn = 0;
    if (reg) reg_counts(R, row, nf, nn);
    float4* P = reinterpret_cast<float4*>(trow(T.p_lo, T.p_hi, T.split, row, d)) + l;
    float4* M = reinterpret_cast<float4*>(trow(T.m_lo, T.m_hi, T.split, row, d)) + l;
    float4* V = reinterpret_cast<float4*>(trow(T.v_lo, T.v_hi, T.split, row, d)) + l;
    float4 p[NV], m[NV], v[NV];
#pragma unroll
    for (int q = 0; q < NV; ++q) {
        p[q] = P[q * LPR];
        m[q] = M[q * LPR];
        v[q] = V[q * LPR];
    }
    float4 w0[NV];  // (a copy: no wait on the counts before the replays)
    if (reg) {
#pragma unroll
        for (int q = 0; q < NV; ++q) w0[q] = p[q];
    }
    // replays [from, fast_end) in the shortened arithmetic (bitwise the same), the rest in full; a
    // row with fewer than kFastMinReplays to replay skips it (the range checks cost about what two
    // shortened replays save: the planted graph's rows are mostly one step behind)
    const int64_t fast_end = (k.fast && k.markstein && upto - from + 1 >= kFastMinReplays)
                                 ? from + min(fast_horizon<NV>(m, v, k), upto - from + 1)
                                 : from;
    for (int64_t s = from; s <= upto; ++s) {
        const float4 c = consts[s];
        const float rc = c.z;  // 1 / c.y, from lgcn_adam_consts
        if (s < fast_end) {
#pragma unroll
            for (int q = 0; q < NV; ++q) {
                adam_elem_zero_fast(p[q].x, m[q].x, v[q].x, c.x, c.y, rc, k);
                adam_elem_zero_fast(p[q].y, m[q].y, v[q].y, c.x, c.y, rc, k);
                adam_elem_zero_fast(p[q].z, m[q].z, v[q].z, c.x, c.y, rc, k);
                adam_elem_zero_fast(p[q].w, m[q].w, v[q].w, c.x, c.y, rc, k);
            }
            continue;
        }
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            adam_elem_zero(p[q].x, m[q].x, v[q].x, c.x, c.y, rc, k);
            adam_elem_zero(p[q].y, m[q].y, v[q].y, c.x, c.y, rc, k);
            adam_elem_zero(p[q].z, m[q].z, v[q].z, c.x, c.y, rc, k);
            adam_elem_zero(p[q].w, m[q].w, v[q].w, c.x, c.y, rc, k);
        }
    }
    int32_t now = static_cast<int32_t>(upto);
    if (upd) {
        const float4 c = consts[t + 1];
        const float rc = c.z;
        const float4* G = reinterpret_cast<const float4*>(trow(T.g_lo, T.g_hi, T.split, row, d)) + l;
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            float4 gv = G[q * LPR];
            if (reg && (nf > 0 || nn > 0)) gv = reg_apply(gv, w0[q], reg_scale(R.coeff, R.B, T.d), nf, nn);
            adam_elem(p[q].x, gv.x, m[q].x, v[q].x, coef, c.x, c.y, rc, k);
            adam_elem(p[q].y, gv.y, m[q].y, v[q].y, coef, c.x, c.y, rc, k);
            adam_elem(p[q].z, gv.z, m[q].z, v[q].z, coef, c.x, c.y, rc, k);
            adam_elem(p[q].w, gv.w, m[q].w, v[q].w, coef, c.x, c.y, rc, k);
        }
        now = static_cast<int32_t>(t + 1);
    }
    if (from <= upto || upd) {
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            P[q * LPR] = p[q];
            M[q * LPR] = m[q];
            V[q * LPR] = v[q];
        }
    }
    if (l == 0) last[row] = now;
}

// Sum of squares of the listed (duplicate-free) gradient rows: per-block partials, in a fixed
// assignment (deterministic), finished by the dense path's k_norm_finish.
template <int LPR, int NV>
__global__ __launch_bounds__(kBlock) void k_row_sqnorm(RowTables T, RowList L, float* __restrict__ partial, RegRows R) {
    constexpr int GPB = kBlock / LPR;
    __shared__ float red[kBlock / 64];
    const int g = threadIdx.x / LPR;
    const int l = threadIdx.x % LPR;
    const int64_t n = L.n_a + L.n_b;
    float acc = 0.f;
    for (int64_t i = int64_t(blockIdx.x) * GPB + g; i < n; i += int64_t(gridDim.x) * GPB) {
        int64_t row;
        if (!list_row(L, i, row)) continue;
        const float4* G = reinterpret_cast<const float4*>(trow(T.g_lo, T.g_hi, T.split, row, int64_t(T.d))) + l;
        // the reg rows (ABI 10): the norm of g + them; the counts and W issued beside G
        int64_t nf = 0, nn = 0;
        float4 w[NV];
        if (R.w_lo) {
            reg_counts(R, row, nf, nn);
            const float4* W = reinterpret_cast<const float4*>(trow(R.w_lo, R.w_hi, R.w_split, row, int64_t(T.d))) + l;
#pragma unroll
            for (int q = 0; q < NV; ++q) w[q] = W[q * LPR];
        }
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            float4 x = G[q * LPR];
            if (R.w_lo) x = reg_apply(x, w[q], reg_scale(R.coeff, R.B, T.d), nf, nn);
            acc += x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
        }
    }
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        float s = 0.f;
        for (int w = 0; w < kBlock / 64; ++w) s += red[w];
        partial[blockIdx.x] = s;
    }
}

__global__ __launch_bounds__(kBlock) void k_norm_finish_rows(const float* __restrict__ partial, int nparts,
                                                             float max_norm, float* __restrict__ out,
                                                             int64_t* __restrict__ step_advance) {
    __shared__ float red[kBlock / 64];
    float acc = 0.f;
    for (int i = threadIdx.x; i < nparts; i += blockDim.x) acc += partial[i];
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        float s = 0.f;
        for (int w = 0; w < kBlock / 64; ++w) s += red[w];
        const float norm = sqrtf(s);
        const float coef = max_norm / (norm + 1e-6f);
        out[0] = norm;
        out[1] = coef < 1.0f ? coef : 1.0f;
        if (step_advance) step_advance[0] += 1;  // the step the update (mode 3) then applies
    }
}

__global__ void k_step_advance(int64_t* step) {
    if (threadIdx.x == 0 && blockIdx.x == 0) step[0] += 1;
}

constexpr int kRowNormBlocks = 2048;

template <int LPR, int NV>
int launch_row_adam(const RowTables& T, const RowList& L, int64_t n_rows, int32_t* last, int32_t* claim,
                    const int64_t* step, const float4* consts, const AdamK& k, const float* clip, int mode,
                    const RegRows& R, hipStream_t s) {
    constexpr int GPB = kBlock / LPR;
    const int64_t n = mode == 2 ? n_rows : L.n_a + L.n_b;
    if (n <= 0) return LGCN_OK;
    k_row_adam<LPR, NV><<<dim3(static_cast<unsigned>((n + GPB - 1) / GPB)), kBlock, 0, s>>>(T, L, n_rows, last, claim,
                                                                                          step, consts, k, clip, mode, R);
    return check_launch("k_row_adam");
}

template <int LPR, int NV>
int launch_row_norm(const RowTables& T, const RowList& L, float max_norm, float* ws, float* out, int64_t* step,
                    const RegRows& R, hipStream_t s) {
    k_row_sqnorm<LPR, NV><<<kRowNormBlocks, kBlock, 0, s>>>(T, L, ws, R);
    if (int rc = check_launch("k_row_sqnorm")) return rc;
    if (!out) return LGCN_OK;  // partials only (lgcn_row_grad_sqnorm)
    k_norm_finish_rows<<<1, kBlock, 0, s>>>(ws, kRowNormBlocks, max_norm, out, step);
    return check_launch("k_norm_finish_rows");
}

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

int check_tables(const RowTables& T, bool need_grad) {
    if (!T.p_lo || !T.m_lo || !T.v_lo || T.d <= 0 || T.split < 0) return fail(LGCN_E_ARG, "lgcn_row_adam: bad tables");
    if (need_grad && !T.g_lo) return fail(LGCN_E_ARG, "lgcn_row_adam: null gradient table");
    const void* ps[] = {T.p_lo, T.p_hi, T.g_lo, T.g_hi, T.m_lo, T.m_hi, T.v_lo, T.v_hi};
    for (const void* p : ps)
        if (p && !al16(p)) return fail(LGCN_E_UNSUPPORTED, "lgcn_row_adam: tables must be 16-byte aligned");
    return LGCN_OK;
}

#define LGCN_ROW_DISPATCH(CALL)                                                     \
    switch (T.d) {                                                                  \
        case 8: return CALL(2, 1);                                                  \
        case 16: return CALL(4, 1);                                                 \
        case 32: return CALL(8, 1);                                                 \
        case 64: return CALL(16, 1);                                                \
        case 128: return CALL(32, 1);                                               \
        case 256: return CALL(64, 1);                                               \
        case 512: return CALL(64, 2);                                               \
        default: return fail(LGCN_E_UNSUPPORTED, "lgcn_row_adam: d=%d", T.d);     \
    }

int row_adam(float* p_lo, float* p_hi, float* g_lo, float* g_hi, float* m_lo, float* m_hi, float* v_lo,
                  float* v_hi, int64_t split, int32_t d, const int32_t* rows_a, int64_t n_a, const int64_t* keys_b,
                  int64_t n_b, int64_t off_b, const uint8_t* first_b, const uint8_t* skip_b, int64_t n_rows,
                  int32_t* last, int32_t* claim, int64_t* step, const float* consts, float one_minus_beta1,
                  float beta2, float one_minus_beta2, float eps, const float* clip, int32_t mode,
                  const RegRows& R, lgcn_stream_t stream) {
    RowTables T{p_lo, p_hi, g_lo, g_hi, m_lo, m_hi, v_lo, v_hi, split, d};
    if (int rc = check_tables(T, mode == 1 || mode == 3)) return rc;
    if (mode < 0 || mode > 3 || !last || !step || !consts || (mode == 0 && !claim) || n_a < 0 || n_b < 0 ||
        (n_a > 0 && !rows_a) || (n_b > 0 && !keys_b))
        return fail(LGCN_E_ARG, "lgcn_row_adam: bad args");
    RowList L{rows_a, n_a, keys_b, n_b, off_b, first_b, skip_b};
    AdamK k{one_minus_beta1, beta2, one_minus_beta2, eps, beta2 == 0.999f, 0, 0.0f, 0.0f};
    // the shortened replay (adam_elem_zero_fast) needs the Markstein schedule (c >= sqrt(0.001)),
    // a denominator floor eps in [2^-40, 2^30] and decays that shrink |m| and v
    if (k.markstein && eps >= 0x1p-40f && eps <= 0x1p30f && one_minus_beta1 > 0.0f && one_minus_beta1 <= 0.5f) {
        const double fm = (1.0 - static_cast<double>(one_minus_beta1)) * (1.0 - std::ldexp(1.0, -22));
        const double fv = static_cast<double>(beta2) * (1.0 - std::ldexp(1.0, -23));
        k.fast = 1;
        k.inv_lm = static_cast<float>(1.0 / -std::log2(fm) * (1.0 - 1e-6));
        k.inv_lv = static_cast<float>(1.0 / -std::log2(fv) * (1.0 - 1e-6));
    }
    hipStream_t s = as_stream(stream);
    if (!al16(consts)) return fail(LGCN_E_ARG, "lgcn_row_adam: consts must be 16-byte aligned");
    const auto* c2 = reinterpret_cast<const float4*>(consts);
    int rc = LGCN_OK;
#define LGCN_RA(LP, NVV) launch_row_adam<LP, NVV>(T, L, n_rows, last, claim, step, c2, k, clip, mode, R, s)
    auto run = [&]() -> int { LGCN_ROW_DISPATCH(LGCN_RA) };
#undef LGCN_RA
    rc = run();
    if (rc) return rc;
    if (mode == 1) {  // the step is done: advance the device counter
        k_step_advance<<<1, 64, 0, s>>>(step);
        return check_launch("k_step_advance");
    }
    return LGCN_OK;
}

int row_norm(const float* g_lo, const float* g_hi, int64_t split, int32_t d, const int32_t* rows_a,
                       int64_t n_a, const int64_t* keys_b, int64_t n_b, int64_t off_b, const uint8_t* first_b,
                       const uint8_t* skip_b, float max_norm, float* ws, float* out, int64_t* step_advance,
                       const RegRows& R, lgcn_stream_t stream) {
    RowTables T{nullptr, nullptr, const_cast<float*>(g_lo), const_cast<float*>(g_hi), nullptr, nullptr, nullptr,
                nullptr, split, d};
    if (!g_lo || !ws || n_a < 0 || n_b < 0 || (n_a > 0 && !rows_a) || (n_b > 0 && !keys_b))
        return fail(LGCN_E_ARG, "lgcn_row_grad_norm: bad args");
    if (!al16(g_lo) || (g_hi && !al16(g_hi))) return fail(LGCN_E_UNSUPPORTED, "lgcn_row_grad_norm: alignment");
    RowList L{rows_a, n_a, keys_b, n_b, off_b, first_b, skip_b};
    hipStream_t s = as_stream(stream);
#define LGCN_RN(LP, NVV) launch_row_norm<LP, NVV>(T, L, max_norm, ws, out, step_advance, R, s)
    LGCN_ROW_DISPATCH(LGCN_RN)
#undef LGCN_RN
}


// lgcn_reg_rows_t -> RegRows, checked (the norm reads W; the update uses its own parameter rows)
int to_reg(const lgcn_reg_rows_t* r, int32_t d, RegRows& R, const char* who) {
    if (!r || !r->w_lo || r->B < 1 || r->neg_off < 0 || r->neg_rows < 0 ||
        (r->neg_rows > 0 && (r->neg_rowptr == nullptr) == (r->neg_count == nullptr)))
        return fail(LGCN_E_ARG, "%s: bad reg rows (w_lo, B >= 1, and exactly one of neg_rowptr / neg_count "
                    "when neg_rows > 0)", who);
    if (!al16(r->w_lo) || (r->w_hi && !al16(r->w_hi)) || d % 4 != 0)
        return fail(LGCN_E_UNSUPPORTED, "%s: reg tables must be 16-byte aligned", who);
    R = RegRows{r->w_lo, r->w_hi, r->w_split, r->coeff, r->B, r->fixed_rowptr, r->neg_rowptr, r->neg_count,
                r->neg_off, r->neg_rows};
    return LGCN_OK;
}

}  // namespace

extern "C" {

int lgcn_adam_consts(float* consts, int64_t t0, int64_t t1, float lr, double beta1, double beta2,
                     lgcn_stream_t stream) {
    if (!consts || t0 < 1 || t1 < t0) return fail(LGCN_E_ARG, "lgcn_adam_consts: bad range");
    if (!al16(consts)) return fail(LGCN_E_ARG, "lgcn_adam_consts: consts must be 16-byte aligned");
    const int64_t n = t1 - t0 + 1;
    k_adam_consts<<<grid_for(n, kBlock, int64_t(1) << 30), kBlock, 0, as_stream(stream)>>>(
        reinterpret_cast<float4*>(consts), t0, t1, lr, beta1, beta2);
    return check_launch("k_adam_consts");
}

int lgcn_row_adam(float* p_lo, float* p_hi, float* g_lo, float* g_hi, float* m_lo, float* m_hi, float* v_lo,
                  float* v_hi, int64_t split, int32_t d, const int32_t* rows_a, int64_t n_a, const int64_t* keys_b,
                  int64_t n_b, int64_t off_b, const uint8_t* first_b, const uint8_t* skip_b, int64_t n_rows,
                  int32_t* last, int32_t* claim, int64_t* step, const float* consts, float one_minus_beta1,
                  float beta2, float one_minus_beta2, float eps, const float* clip, int32_t mode,
                  lgcn_stream_t stream) {
    return row_adam(p_lo, p_hi, g_lo, g_hi, m_lo, m_hi, v_lo, v_hi, split, d, rows_a, n_a, keys_b, n_b, off_b, first_b,
                    skip_b, n_rows, last, claim, step, consts, one_minus_beta1, beta2, one_minus_beta2, eps, clip, mode,
                    RegRows{}, stream);
}

int lgcn_row_adam_reg(float* p_lo, float* p_hi, float* g_lo, float* g_hi, float* m_lo, float* m_hi, float* v_lo,
                      float* v_hi, int64_t split, int32_t d, const int32_t* rows_a, int64_t n_a, const int64_t* keys_b,
                      int64_t n_b, int64_t off_b, const uint8_t* first_b, const uint8_t* skip_b, int32_t* last,
                      int64_t* step, const float* consts, float one_minus_beta1, float beta2, float one_minus_beta2,
                      float eps, const float* clip, int32_t mode, const lgcn_reg_rows_t* reg, lgcn_stream_t stream) {
    RegRows R{};
    if (int rc = to_reg(reg, d, R, "lgcn_row_adam_reg")) return rc;
    if (mode != 1 && mode != 3) return fail(LGCN_E_ARG, "lgcn_row_adam_reg: mode 1 or 3 (an update)");
    return row_adam(p_lo, p_hi, g_lo, g_hi, m_lo, m_hi, v_lo, v_hi, split, d, rows_a, n_a, keys_b, n_b, off_b, first_b,
                    skip_b, 0, last, nullptr, step, consts, one_minus_beta1, beta2, one_minus_beta2, eps, clip, mode, R,
                    stream);
}

int lgcn_row_grad_norm_workspace_floats(void) { return kRowNormBlocks; }

int lgcn_row_grad_norm(const float* g_lo, const float* g_hi, int64_t split, int32_t d, const int32_t* rows_a,
                       int64_t n_a, const int64_t* keys_b, int64_t n_b, int64_t off_b, const uint8_t* first_b,
                       const uint8_t* skip_b, float max_norm, float* ws, float* out, int64_t* step_advance,
                       lgcn_stream_t stream) {
    return row_norm(g_lo, g_hi, split, d, rows_a, n_a, keys_b, n_b, off_b, first_b, skip_b, max_norm, ws, out,
                    step_advance, RegRows{}, stream);
}

int lgcn_row_grad_norm_reg(const float* g_lo, const float* g_hi, int64_t split, int32_t d, const int32_t* rows_a,
                           int64_t n_a, const int64_t* keys_b, int64_t n_b, int64_t off_b, const uint8_t* first_b,
                           const uint8_t* skip_b, float max_norm, float* ws, float* out, int64_t* step_advance,
                           const lgcn_reg_rows_t* reg, lgcn_stream_t stream) {
    RegRows R{};
    if (int rc = to_reg(reg, d, R, "lgcn_row_grad_norm_reg")) return rc;
    if (!out) return fail(LGCN_E_ARG, "lgcn_row_grad_norm_reg: null out");
    return row_norm(g_lo, g_hi, split, d, rows_a, n_a, keys_b, n_b, off_b, first_b, skip_b, max_norm, ws, out,
                    step_advance, R, stream);
}

int lgcn_row_grad_sqnorm(const float* g_lo, const float* g_hi, int64_t split, int32_t d, const int32_t* rows_a,
                         int64_t n_a, const int64_t* keys_b, int64_t n_b, int64_t off_b, const uint8_t* first_b,
                         const uint8_t* skip_b, float* partials, lgcn_stream_t stream) {
    if (!partials) return fail(LGCN_E_ARG, "lgcn_row_grad_sqnorm: null partials");
    return lgcn_row_grad_norm(g_lo, g_hi, split, d, rows_a, n_a, keys_b, n_b, off_b, first_b, skip_b, 0.0f, partials,
                              nullptr, nullptr, stream);
}

int lgcn_row_grad_norm_finish(const float* partials, int64_t nparts, float max_norm, float* out, int64_t* step_advance,
                              lgcn_stream_t stream) {
    if (!partials || !out || nparts < 1 || nparts > INT32_MAX)
        return fail(LGCN_E_ARG, "lgcn_row_grad_norm_finish: bad args");
    k_norm_finish_rows<<<1, kBlock, 0, as_stream(stream)>>>(partials, static_cast<int>(nparts), max_norm, out,
                                                           step_advance);
    return check_launch("k_norm_finish_rows");
}

}  // extern "C"
