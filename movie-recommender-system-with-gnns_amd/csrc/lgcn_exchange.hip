// Row-sparse gradient exchange for data-parallel Cluster-GCN training (C4) with the row-lazy
// Adam. The reference's DP equivalent is one dense all_reduce of both embedding gradients per
// step (the single-GPU step is reference utils/train_test.py:86-96). A batch step
// writes a nonzero gradient only on its rows (touched rows + first-occurrence negatives), a few
// % of N, so each rank ships just those rows:
//
//   lgcn_rows_pack        rank r: its listed rows -> ids[cap] (int64, -1 = empty) + rows[cap, d]
//                         (lgcn_amd.distributed.RowExchange packs both into one record block:
//                         the ids as the first 2*cap words, then the rows)
//   (one all_gather over RCCL of the record blocks: [W, cap*(d+2)]; ids copied out contiguous)
//   lgcn_rows_mark_first  first[i] = entry i is the first occurrence of its row in the gathered
//                         list (deterministic: lowest index wins; claim[N] int32 = INT32_MAX
//                         between calls, restored on exit)
//   lgcn_rows_accumulate  per rank r = 0..W-1 in order (rank r's rows at rows + r*rank_stride):
//                         g[row] = first ? row_r : g[row] + row_r; then g[row] /= W on the first
//                         entries (div > 0)
//
// Every rank runs the same launches on the same gathered bytes, so the gradient rows, the clip
// norm over the union (lgcn_row_grad_norm with first_b) and the row Adam update are bitwise the
// same on every rank, and the replicas stay identical. The per-row sum is rank order
// (g0 + g1) + g2 ..., then / W, which is what a dense sum-then-divide computes for W = 2
// exactly (a + b == b + a).

#include <climits>

#include "lgcn_common.h"

using namespace lgcn;

namespace {

template <class T>
__device__ __forceinline__ T* trow(T* lo, T* hi, int64_t split, int64_t r, int64_t d) {
    return r < split ? lo + r * d : hi + (r - split) * d;
}

// One LPR-lane group per slot of the packed list (rows_a then keys_b, as lgcn_row_adam's list).
template <int LPR, int NV>
__global__ __launch_bounds__(kBlock) void k_rows_pack(const float* __restrict__ g_lo, const float* __restrict__ g_hi,
                                                      int64_t split, int32_t d, const int32_t* __restrict__ rows_a,
                                                      int64_t n_a, const int64_t* __restrict__ keys_b, int64_t n_b,
                                                      int64_t off_b, const uint8_t* __restrict__ first_b,
                                                      const uint8_t* __restrict__ skip_b, int64_t cap,
                                                      int64_t* __restrict__ ids, float* __restrict__ rows) {
    constexpr int GPB = kBlock / LPR;
    const int g = threadIdx.x / LPR;
    const int l = threadIdx.x % LPR;
    const int64_t i = int64_t(blockIdx.x) * GPB + g;
    if (i >= cap) return;
    int64_t row = -1;
    if (i < n_a) {
        row = rows_a[i];
    } else if (i < n_a + n_b) {
        const int64_t j = i - n_a;
        row = keys_b[j] + off_b;
        if ((first_b && !first_b[j]) || (skip_b && skip_b[row])) row = -1;
    }
    if (l == 0) ids[i] = row;
    if (row < 0) return;
    const float4* src = reinterpret_cast<const float4*>(trow(g_lo, g_hi, split, row, int64_t(d))) + l;
    float4* dst = reinterpret_cast<float4*>(rows + i * int64_t(d)) + l;
#pragma unroll
    for (int q = 0; q < NV; ++q) dst[q * LPR] = src[q * LPR];
}

__global__ void k_claim_min(const int64_t* __restrict__ ids, int64_t n, int32_t* __restrict__ claim) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t r = ids[i];
    if (r >= 0) atomicMin(claim + r, static_cast<int32_t>(i));
}

__global__ void k_claim_read(const int64_t* __restrict__ ids, int64_t n, const int32_t* __restrict__ claim,
                             uint8_t* __restrict__ first) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t r = ids[i];
    first[i] = (r >= 0 && claim[r] == static_cast<int32_t>(i)) ? 1 : 0;
}

__global__ void k_claim_reset(const int64_t* __restrict__ ids, int64_t n, int32_t* __restrict__ claim) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t r = ids[i];
    if (r >= 0) claim[r] = INT_MAX;
}

// mode 0: g[row] = first ? x : g[row] + x (one rank's slots: rows unique within them)
// mode 1: g[row] = g[row] / div on first entries
template <int LPR, int NV>
__global__ __launch_bounds__(kBlock) void k_rows_accumulate(const int64_t* __restrict__ ids,
                                                            const float* __restrict__ rows, int64_t n,
                                                            const uint8_t* __restrict__ first, float* g_lo,
                                                            float* g_hi, int64_t split, int32_t d, int mode,
                                                            float div) {
    constexpr int GPB = kBlock / LPR;
    const int g = threadIdx.x / LPR;
    const int l = threadIdx.x % LPR;
    const int64_t i = int64_t(blockIdx.x) * GPB + g;
    if (i >= n) return;
    const int64_t row = ids[i];
    if (row < 0) return;
    const bool f = first[i] != 0;
    if (mode == 1 && !f) return;
    float4* G = reinterpret_cast<float4*>(trow(g_lo, g_hi, split, row, int64_t(d))) + l;
    if (mode == 1) {
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            const float4 v = G[q * LPR];
            G[q * LPR] = make_float4(v.x / div, v.y / div, v.z / div, v.w / div);
        }
        return;
    }
    const float4* X = reinterpret_cast<const float4*>(rows + i * int64_t(d)) + l;
#pragma unroll
    for (int q = 0; q < NV; ++q) {
        const float4 x = X[q * LPR];
        if (f) {
            G[q * LPR] = x;
        } else {
            const float4 v = G[q * LPR];
            G[q * LPR] = make_float4(v.x + x.x, v.y + x.y, v.z + x.z, v.w + x.w);
        }
    }
}


// ---- owner-sharded exchange (lgcn_amd.owner.OwnerExchange) ----
// Rows are owned by rank row % W. A send buffer holds W destination blocks of block_floats floats:
//   [grad ids: 2*cap floats (int64) | grad rows: cap*d | request ids: 2*rcap floats (int64) | pad]
// Slots are taken with one atomic per entry (per-destination counters), so slot order varies run
// to run; nothing downstream depends on it (per-row sums are rank-ordered and a row appears at
// most once per rank block; the clip norm sweeps the owner's rows in row order).

__global__ void k_owner_reset(float* __restrict__ send, int64_t world, int64_t block_floats, int64_t cap,
                              int64_t req_off, int64_t rcap, int32_t* __restrict__ counts) {
    const int64_t per = cap + rcap;
    const int64_t n = world * per;
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int64_t o = i / per, j = i % per;
        int64_t* ids = reinterpret_cast<int64_t*>(send + o * block_floats + (j < cap ? 0 : req_off));
        ids[j < cap ? j : j - cap] = -1;
    }
    if (blockIdx.x == 0 && threadIdx.x < 2 * world) counts[threadIdx.x] = 0;
}

// One LPR-lane group per entry of the (rows_a, keys_b) list: the listed gradient row goes to
// destination row % W at the next free slot of that destination.
template <int LPR, int NV>
__global__ __launch_bounds__(kBlock) void k_owner_pack_rows(
    const float* __restrict__ g_lo, const float* __restrict__ g_hi, int64_t split, int32_t d,
    const int32_t* __restrict__ rows_a, int64_t n_a, const int64_t* __restrict__ keys_b, int64_t n_b, int64_t off_b,
    const uint8_t* __restrict__ first_b, const uint8_t* __restrict__ skip_b, int64_t world, int64_t cap,
    int64_t block_floats, int32_t* __restrict__ counts, float* __restrict__ send, int32_t* __restrict__ overflow) {
    constexpr int GPB = kBlock / LPR;
    const int g = threadIdx.x / LPR;
    const int l = threadIdx.x % LPR;
    const int64_t i = int64_t(blockIdx.x) * GPB + g;
    if (i >= n_a + n_b) return;
    int64_t row;
    if (i < n_a) {
        row = rows_a[i];
    } else {
        const int64_t j = i - n_a;
        row = keys_b[j] + off_b;
        if ((first_b && !first_b[j]) || (skip_b && skip_b[row])) return;
    }
    const int64_t o = row % world;
    int slot = 0;
    if (l == 0) slot = atomicAdd(counts + o, 1);
    slot = __shfl(slot, 0, LPR);
    if (slot >= cap) {
        if (l == 0) atomicOr(overflow, 1);
        return;
    }
    float* blk = send + o * block_floats;
    if (l == 0) reinterpret_cast<int64_t*>(blk)[slot] = row;
    const float4* src = reinterpret_cast<const float4*>(trow(g_lo, g_hi, split, row, int64_t(d))) + l;
    float4* dst = reinterpret_cast<float4*>(blk + 2 * cap + int64_t(slot) * d) + l;
#pragma unroll
    for (int q = 0; q < NV; ++q) dst[q * LPR] = src[q * LPR];
}

// Request ids (rows_a, then keys_b + off_b) to destination row % W; also mine[o*rcap + slot].
// claim (nullable): each distinct row is requested once — the entry whose exchange of the call's
// stamp into claim[row] finds another value packs it, the others skip (a row's copy is the same
// whichever entry requested it).
__global__ void k_owner_pack_requests(const int32_t* __restrict__ rows_a, int64_t n_a,
                                      const int64_t* __restrict__ keys_b, int64_t n_b, int64_t off_b, int64_t world,
                                      int64_t rcap, int64_t block_floats, int64_t req_off,
                                      int32_t* __restrict__ counts, float* __restrict__ send,
                                      int64_t* __restrict__ mine, int32_t* __restrict__ overflow,
                                      int32_t* __restrict__ claim, int32_t stamp) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n_a + n_b; i += stride) {
        const int64_t row = i < n_a ? int64_t(rows_a[i]) : keys_b[i - n_a] + off_b;
        if (claim && atomicExch(claim + row, stamp) == stamp) continue;  // already requested this call
        const int64_t o = row % world;
        const int slot = atomicAdd(counts + world + o, 1);
        if (slot >= rcap) {
            atomicOr(overflow, 2);
            continue;
        }
        reinterpret_cast<int64_t*>(send + o * block_floats + req_off)[slot] = row;
        mine[o * rcap + slot] = row;
    }
}

// out[i] = p[ids[i]] (ids[i] >= 0); rows of out are d floats apart, rank blocks of n floats
template <int LPR, int NV>
__global__ __launch_bounds__(kBlock) void k_rows_gather(const float* __restrict__ p_lo, const float* __restrict__ p_hi,
                                                        int64_t split, int32_t d, const int64_t* __restrict__ ids,
                                                        int64_t n, float* __restrict__ out, int scatter) {
    constexpr int GPB = kBlock / LPR;
    const int g = threadIdx.x / LPR;
    const int l = threadIdx.x % LPR;
    const int64_t i = int64_t(blockIdx.x) * GPB + g;
    if (i >= n) return;
    const int64_t row = ids[i];
    if (row < 0) return;
    float4* P = reinterpret_cast<float4*>(trow(const_cast<float*>(p_lo), const_cast<float*>(p_hi), split, row,
                                               int64_t(d))) + l;
    float4* X = reinterpret_cast<float4*>(out + i * int64_t(d)) + l;
#pragma unroll
    for (int q = 0; q < NV; ++q) {
        if (scatter) P[q * LPR] = X[q * LPR];
        else X[q * LPR] = P[q * LPR];
    }
}

__global__ void k_rows_mark(const int64_t* __restrict__ ids, const uint8_t* __restrict__ first, int64_t n,
                            uint8_t* __restrict__ mask, uint8_t value) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t r = ids[i];
    if (r >= 0 && (!first || first[i])) mask[r] = value;
}

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

#define LGCN_EX_DISPATCH(CALL, WHAT)                                              \
    switch (d) {                                                                  \
        case 8: CALL(2, 1); break;                                                \
        case 16: CALL(4, 1); break;                                               \
        case 32: CALL(8, 1); break;                                               \
        case 64: CALL(16, 1); break;                                              \
        case 128: CALL(32, 1); break;                                             \
        case 256: CALL(64, 1); break;                                             \
        case 512: CALL(64, 2); break;                                             \
        default: return fail(LGCN_E_UNSUPPORTED, WHAT ": d=%d unsupported", d); \
    }

}  // namespace

extern "C" {

int lgcn_rows_pack(const float* g_lo, const float* g_hi, int64_t split, int32_t d, const int32_t* rows_a,
                   int64_t n_a, const int64_t* keys_b, int64_t n_b, int64_t off_b, const uint8_t* first_b,
                   const uint8_t* skip_b, int64_t cap, int64_t* ids, float* rows, lgcn_stream_t stream) {
    if (!g_lo || !ids || !rows || n_a < 0 || n_b < 0 || cap < n_a + n_b || (n_a > 0 && !rows_a) ||
        (n_b > 0 && !keys_b))
        return fail(LGCN_E_ARG, "lgcn_rows_pack: bad args (n_a=%lld n_b=%lld cap=%lld)", (long long)n_a,
                    (long long)n_b, (long long)cap);
    if (!al16(g_lo) || (g_hi && !al16(g_hi)) || !al16(rows))
        return fail(LGCN_E_UNSUPPORTED, "lgcn_rows_pack: tables must be 16-byte aligned");
    if (cap == 0) return LGCN_OK;
    hipStream_t s = as_stream(stream);
#define LGCN_PK(LP, NVV)                                                                                       \
    k_rows_pack<LP, NVV><<<grid_for(cap * LP, kBlock, int64_t(1) << 30), kBlock, 0, s>>>(                       \
        g_lo, g_hi, split, d, rows_a, n_a, keys_b, n_b, off_b, first_b, skip_b, cap, ids, rows)
    LGCN_EX_DISPATCH(LGCN_PK, "lgcn_rows_pack")
#undef LGCN_PK
    return check_launch("k_rows_pack");
}

int lgcn_owner_reset(float* send, int64_t world, int64_t block_floats, int64_t cap, int64_t req_off, int64_t rcap,
                     int32_t* counts, lgcn_stream_t stream) {
    if (!send || !counts || world < 1 || world > 64 || cap < 0 || rcap < 0 || req_off < 2 * cap ||
        block_floats < req_off + 2 * rcap || (block_floats & 3) || (req_off & 1) || (cap & 1))
        return fail(LGCN_E_ARG, "lgcn_owner_reset: bad layout (world=%lld block=%lld cap=%lld req_off=%lld rcap=%lld)",
                    (long long)world, (long long)block_floats, (long long)cap, (long long)req_off, (long long)rcap);
    k_owner_reset<<<grid_for(world * (cap + rcap), kBlock, 4096), kBlock, 0, as_stream(stream)>>>(
        send, world, block_floats, cap, req_off, rcap, counts);
    return check_launch("k_owner_reset");
}

int lgcn_owner_pack_rows(const float* g_lo, const float* g_hi, int64_t split, int32_t d, const int32_t* rows_a,
                         int64_t n_a, const int64_t* keys_b, int64_t n_b, int64_t off_b, const uint8_t* first_b,
                         const uint8_t* skip_b, int64_t world, int64_t cap, int64_t block_floats, int32_t* counts,
                         float* send, int32_t* overflow, lgcn_stream_t stream) {
    if (!g_lo || !send || !counts || !overflow || world < 1 || cap < 0 || n_a < 0 || n_b < 0 ||
        (n_a > 0 && !rows_a) || (n_b > 0 && !keys_b) || block_floats < cap * (int64_t(d) + 2))
        return fail(LGCN_E_ARG, "lgcn_owner_pack_rows: bad args");
    if (!al16(g_lo) || (g_hi && !al16(g_hi)) || !al16(send) || (block_floats & 3) || (cap & 1))
        return fail(LGCN_E_UNSUPPORTED, "lgcn_owner_pack_rows: 16-byte alignment (block_floats %% 4, cap even)");
    const int64_t n = n_a + n_b;
    if (n == 0) return LGCN_OK;
    hipStream_t s = as_stream(stream);
#define LGCN_OP(LP, NVV)                                                                                     \
    k_owner_pack_rows<LP, NVV><<<grid_for(n * LP, kBlock, int64_t(1) << 30), kBlock, 0, s>>>(                 \
        g_lo, g_hi, split, d, rows_a, n_a, keys_b, n_b, off_b, first_b, skip_b, world, cap, block_floats, counts, \
        send, overflow)
    LGCN_EX_DISPATCH(LGCN_OP, "lgcn_owner_pack_rows")
#undef LGCN_OP
    return check_launch("k_owner_pack_rows");
}

int lgcn_owner_pack_requests(const int32_t* rows_a, int64_t n_a, const int64_t* keys_b, int64_t n_b, int64_t off_b,
                             int64_t world, int64_t rcap, int64_t block_floats, int64_t req_off, int32_t* counts,
                             float* send, int64_t* mine, int32_t* overflow, int32_t* claim, int32_t stamp,
                             lgcn_stream_t stream) {
    if (!send || !counts || !mine || !overflow || world < 1 || rcap < 0 || n_a < 0 || n_b < 0 ||
        (n_a > 0 && !rows_a) || (n_b > 0 && !keys_b) || block_floats < req_off + 2 * rcap || (req_off & 1) ||
        (claim && stamp < 0))
        return fail(LGCN_E_ARG, "lgcn_owner_pack_requests: bad args");
    if (n_a + n_b == 0) return LGCN_OK;
    k_owner_pack_requests<<<grid_for(n_a + n_b, kBlock, 4096), kBlock, 0, as_stream(stream)>>>(
        rows_a, n_a, keys_b, n_b, off_b, world, rcap, block_floats, req_off, counts, send, mine, overflow, claim,
        stamp);
    return check_launch("k_owner_pack_requests");
}

int lgcn_rows_gather(const float* p_lo, const float* p_hi, int64_t split, int32_t d, const int64_t* ids, int64_t n,
                     float* rows, int32_t scatter, lgcn_stream_t stream) {
    if (!p_lo || n < 0 || (n > 0 && (!ids || !rows)))
        return fail(LGCN_E_ARG, "lgcn_rows_gather: bad args");
    if (!al16(p_lo) || (p_hi && !al16(p_hi)) || !al16(rows))
        return fail(LGCN_E_UNSUPPORTED, "lgcn_rows_gather: 16-byte alignment");
    if (n == 0) return LGCN_OK;
    hipStream_t s = as_stream(stream);
#define LGCN_RG(LP, NVV)                                                                                     \
    k_rows_gather<LP, NVV><<<grid_for(n * LP, kBlock, int64_t(1) << 30), kBlock, 0, s>>>(                     \
        p_lo, p_hi, split, d, ids, n, rows, scatter)
    LGCN_EX_DISPATCH(LGCN_RG, "lgcn_rows_gather")
#undef LGCN_RG
    return check_launch("k_rows_gather");
}

int lgcn_rows_mark(const int64_t* ids, const uint8_t* first, int64_t n, uint8_t* mask, int32_t value,
                   lgcn_stream_t stream) {
    if (n < 0 || (n > 0 && (!ids || !mask))) return fail(LGCN_E_ARG, "lgcn_rows_mark: bad args");
    if (n == 0) return LGCN_OK;
    k_rows_mark<<<grid_for(n, kBlock, int64_t(1) << 30), kBlock, 0, as_stream(stream)>>>(ids, first, n, mask,
                                                                                         uint8_t(value));
    return check_launch("k_rows_mark");
}

int lgcn_rows_mark_first(const int64_t* ids, int64_t n, int32_t* claim, uint8_t* first, lgcn_stream_t stream) {
    if (n < 0 || (n > 0 && (!ids || !claim || !first)) || n > INT_MAX)
        return fail(LGCN_E_ARG, "lgcn_rows_mark_first: bad args (n=%lld)", (long long)n);
    if (n == 0) return LGCN_OK;
    hipStream_t s = as_stream(stream);
    const unsigned grid = grid_for(n, kBlock, int64_t(1) << 30);
    k_claim_min<<<grid, kBlock, 0, s>>>(ids, n, claim);
    if (int rc = check_launch("k_claim_min")) return rc;
    k_claim_read<<<grid, kBlock, 0, s>>>(ids, n, claim, first);
    if (int rc = check_launch("k_claim_read")) return rc;
    k_claim_reset<<<grid, kBlock, 0, s>>>(ids, n, claim);
    return check_launch("k_claim_reset");
}

int lgcn_rows_accumulate(const int64_t* ids, const float* rows, int64_t world, int64_t cap, int64_t rank_stride,
                         const uint8_t* first, float* g_lo, float* g_hi, int64_t split, int32_t d, float div,
                         lgcn_stream_t stream) {
    if (world < 1 || cap < 0 || !g_lo || (cap > 0 && (!ids || !rows || !first)) || rank_stride < cap * int64_t(d))
        return fail(LGCN_E_ARG, "lgcn_rows_accumulate: bad args (rank_stride=%lld < cap*d?)", (long long)rank_stride);
    if (!al16(g_lo) || (g_hi && !al16(g_hi)) || (rows && !al16(rows)) || rank_stride % 4)
        return fail(LGCN_E_UNSUPPORTED, "lgcn_rows_accumulate: tables and rank blocks must be 16-byte aligned");
    if (cap == 0) return LGCN_OK;
    hipStream_t s = as_stream(stream);
#define LGCN_AC(LP, NVV)                                                                                         \
    for (int64_t r = 0; r < world; ++r) {                                                                        \
        k_rows_accumulate<LP, NVV><<<grid_for(cap * LP, kBlock, int64_t(1) << 30), kBlock, 0, s>>>(                \
            ids + r * cap, rows + r * rank_stride, cap, first + r * cap, g_lo, g_hi, split, d, 0, 1.0f);            \
        if (int rc = check_launch("k_rows_accumulate")) return rc;                                               \
    }                                                                                                            \
    if (div > 0.f)                                                                                               \
        k_rows_accumulate<LP, NVV><<<grid_for(world * cap * LP, kBlock, int64_t(1) << 30), kBlock, 0, s>>>(        \
            ids, rows, world * cap, first, g_lo, g_hi, split, d, 1, div)
    LGCN_EX_DISPATCH(LGCN_AC, "lgcn_rows_accumulate")
#undef LGCN_AC
    return check_launch("k_rows_accumulate");
}

}  // extern "C"
