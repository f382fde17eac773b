// Plan construction for LightGCN propagation on gfx950: stable CSR build, gcn_norm edge
// weights and the load-balanced work schedule. Runs once per edge set (the reference
// recomputes gcn_norm on every layer call — reference models/light_gcn.py:33 via PyG 2.4.0
// LGConv.forward — but the result is identical each time, so one plan per edge_index is
// a legal cache).
//
// Everything is stream-ordered on the caller's stream, allocation-free and sync-free.

#include <hipcub/hipcub.hpp>

#include "lgcn_common.h"

using namespace lgcn;

namespace {

// key32[e] = key[e], eid[e] = e; count ids outside [0, N).
__global__ void k_prep_keys(const int64_t* __restrict__ key, const int64_t* __restrict__ other,
                            int64_t E, int64_t N, int32_t* __restrict__ key32,
                            int32_t* __restrict__ eid, unsigned long long* __restrict__ err) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    unsigned long long bad_local = 0;
    for (int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; e < E; e += stride) {
        const int64_t k = key[e];
        const int64_t o = other[e];
        const bool bad = (k < 0) | (k >= N) | (o < 0) | (o >= N);
        bad_local += bad;
        key32[e] = bad ? 0 : static_cast<int32_t>(k);
        eid[e] = static_cast<int32_t>(e);
    }
    if (bad_local) atomicAdd(err, bad_local);
}

// rowptr from sorted keys (all in [0, N)): rowptr[r] = the first slot whose key is >= r, by a
// binary search per row — one thread per row, so runs of empty rows (touched-only batch plans,
// segment plans built over max(N, M) rows) cost no serial loop.
__global__ void k_rowptr_from_sorted(const int32_t* __restrict__ keys, int64_t E, int64_t N,
                                     int64_t* __restrict__ rowptr) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t r = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; r <= N; r += stride) {
        int64_t lo = 0, hi = E;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (keys[mid] < r) lo = mid + 1;
            else hi = mid;
        }
        rowptr[r] = lo;
    }
}

// col[p] = other[eid[p]]; an out-of-range id (already counted in err) becomes 0 so no later
// pass of the build can read outside [0, N) before the caller sees the error.
__global__ void k_gather_col(const int64_t* __restrict__ other, const int32_t* __restrict__ eid,
                             int64_t E, int64_t N, int32_t* __restrict__ col) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t p = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; p < E; p += stride) {
        const int64_t o = other[eid[p]];
        col[p] = (o < 0 || o >= N) ? 0 : static_cast<int32_t>(o);
    }
}

// PyG gcn_norm: deg = scatter(ones, target, reduce='sum') in fp32 — a sequential fp32 sum of
// ones saturates at 2^24 — then deg.pow_(-0.5) (== 1/sqrt(deg), both correctly rounded, on
// CPU) and inf -> 0.
__global__ void k_inv_sqrt_degree(const int64_t* __restrict__ rowptr, int64_t N,
                                  float* __restrict__ dis) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < N; i += stride) {
        int64_t deg = rowptr[i + 1] - rowptr[i];
        if (deg > (int64_t(1) << 24)) deg = int64_t(1) << 24;
        const float degf = static_cast<float>(deg);
        dis[i] = (deg == 0) ? 0.0f : 1.0f / sqrtf(degf);
    }
}

__device__ __forceinline__ int64_t row_of_slot(const int64_t* __restrict__ rowptr, int64_t N,
                                               int64_t p) {
    // largest r in [0, N) with rowptr[r] <= p (then rowptr[r+1] > p)
    int64_t lo = 0, hi = N - 1;
    while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (rowptr[mid] <= p) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// w = dis[source] * 1 * dis[target]; (dis[a]*1)*dis[b] == dis[a]*dis[b] exactly.
__global__ void k_edge_norm(const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                            int64_t N, int64_t E, const float* __restrict__ dis,
                            float* __restrict__ val) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t p = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; p < E; p += stride) {
        const int64_t r = row_of_slot(rowptr, N, p);
        val[p] = dis[r] * dis[col[p]];
    }
}

// ---- schedule ----
__global__ void k_sched_count(const int64_t* __restrict__ rowptr, int64_t N, int32_t chunk,
                              const uint8_t* __restrict__ row_mask, int64_t* __restrict__ n_items,
                              int32_t* __restrict__ n_part, int32_t* __restrict__ n_split) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < N; i += stride) {
        const int64_t deg = rowptr[i + 1] - rowptr[i];
        const bool live = (row_mask == nullptr) || row_mask[i];
        const int64_t nch = !live ? 0 : (deg > chunk) ? (deg + chunk - 1) / chunk : 1;
        n_items[i] = nch;
        n_part[i] = (nch > 1) ? static_cast<int32_t>(nch) : 0;
        n_split[i] = (nch > 1) ? 1 : 0;
    }
}

__global__ void k_fill_u32(uint32_t* __restrict__ p, int64_t n, uint32_t v) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = v;
}

__global__ void k_sched_fill(const int64_t* __restrict__ rowptr, int64_t N, int32_t chunk, int64_t side_split,
                             const int64_t* __restrict__ n_items, const int64_t* __restrict__ item_off,
                             const int32_t* __restrict__ n_part, const int32_t* __restrict__ part_off,
                             const int32_t* __restrict__ n_split, const int32_t* __restrict__ split_off,
                             lgcn_item_t* __restrict__ raw, uint32_t* __restrict__ keys,
                             int32_t* __restrict__ idx, lgcn_split_t* __restrict__ splits,
                             int64_t* __restrict__ counts) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < N; i += stride) {
        const int64_t beg = rowptr[i];
        const int64_t deg = rowptr[i + 1] - beg;
        const int64_t nch = n_items[i];
        const int64_t off = item_off[i];
        for (int64_t c = 0; c < nch; ++c) {
            lgcn_item_t it;
            it.beg = beg + c * chunk;
            const int64_t rem = deg - c * chunk;
            it.len = static_cast<int32_t>(rem < chunk ? rem : chunk);
            it.dst = (nch > 1) ? -(part_off[i] + static_cast<int32_t>(c)) - 1 : static_cast<int32_t>(i);
            raw[off + c] = it;
            // rows [0, side_split) first, then the rest; longest first inside each side
            const uint32_t side = (i >= side_split) ? 1u : 0u;
            keys[off + c] = (side << 31) | static_cast<uint32_t>(chunk - it.len);
            idx[off + c] = static_cast<int32_t>(off + c);
        }
        if (nch > 1) {
            lgcn_split_t s;
            s.row = static_cast<int32_t>(i);
            s.pbeg = part_off[i];
            s.pcnt = static_cast<int32_t>(nch);
            s.pad = 0;
            splits[split_off[i]] = s;
        }
        if (i == N - 1) {
            counts[0] = off + nch;
            counts[1] = split_off[i] + n_split[i];
            counts[2] = part_off[i] + n_part[i];
        }
    }
}

__global__ void k_sched_gather(const lgcn_item_t* __restrict__ raw, const int32_t* __restrict__ idx,
                               int64_t n, lgcn_item_t* __restrict__ items) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t m = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; m < n; m += stride)
        items[m] = raw[idx[m]];
}

// ---- source-sliced schedule (lgcn_slice_schedule_build; see lgcn_amd/sliced.py) ----
constexpr int32_t kSliceFirst = 0x20000000;
constexpr int32_t kSliceLast = 0x40000000;

__device__ __forceinline__ int slice_of(int64_t c, const int64_t* __restrict__ bounds, int S) {
    // bounds[0] = 0 < bounds[1] < ... < bounds[S] = N: the s with bounds[s] <= c < bounds[s+1]
    int lo = 0, hi = S - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (bounds[mid] <= c) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// A row's slice segments: [start, end) runs of its CSR list whose neighbours fall in one source
// slice, visited in ascending slice order. Found by binary search of the slice bounds in the row's
// (ascending) neighbour list — O(segments * log deg) per row instead of a scan of every edge. On an
// unsorted row (flagged by k_slice_count; the host then discards the schedule) the searches still
// return positions inside [start, end), so every segment stays in bounds and count / fill agree.
template <class F>
__device__ __forceinline__ void for_each_segment(const int32_t* __restrict__ col, int64_t beg, int64_t end,
                                                 const int64_t* __restrict__ bounds, int S, F&& f) {
    int sl = slice_of(col[beg], bounds, S);
    int64_t start = beg;
    while (start < end) {
        int64_t stop = end;
        if (sl < S - 1) {  // lower bound of bounds[sl + 1] in col[start, end)
            const int64_t b = bounds[sl + 1];
            int64_t lo = start, hi = end;
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if (col[mid] < b) lo = mid + 1;
                else hi = mid;
            }
            stop = lo;
        }
        if (stop > start) f(start, stop, sl);
        start = stop;
        ++sl;
    }
}

// One wave per row: the lanes check that its neighbours ascend (coalesced), lane 0 counts its
// segments, chunks (hub: a segment longer than chunk) and items.
__global__ void k_slice_count(const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col, int64_t N,
                              const int64_t* __restrict__ bounds, int S, int32_t chunk,
                              const uint8_t* __restrict__ row_mask, int64_t* __restrict__ n_items, int32_t* __restrict__ n_part,
                              int32_t* __restrict__ n_split, int32_t* __restrict__ unsorted) {
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t(gridDim.x) * blockDim.x) >> 6;
    for (int64_t i = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6; i < N; i += nwaves) {
        const int64_t beg = rowptr[i], end = rowptr[i + 1];
        bool bad = false;
        for (int64_t e = beg + 1 + lane; e < end; e += 64) bad |= col[e] < col[e - 1];
        if (__any(bad) && lane == 0) atomicOr(unsorted, 1);
        if (lane != 0) continue;
        if (row_mask != nullptr && row_mask[i] == 0) {  // not scheduled (another rank's row)
            n_items[i] = 0;
            n_part[i] = 0;
            n_split[i] = 0;
            continue;
        }
        if (end == beg) {
            n_items[i] = 1;
            n_part[i] = 0;
            n_split[i] = 0;
            continue;
        }
        int64_t segs = 0, chunks = 0, maxlen = 0;
        for_each_segment(col, beg, end, bounds, S, [&](int64_t a, int64_t b, int) {
            const int64_t len = b - a;
            ++segs;
            chunks += (len + chunk - 1) / chunk;
            maxlen = len > maxlen ? len : maxlen;
        });
        const bool hub = maxlen > chunk;
        n_items[i] = hub ? chunks : segs;
        n_part[i] = hub ? static_cast<int32_t>(chunks) : 0;
        n_split[i] = hub ? 1 : 0;
    }
}

__global__ void k_slice_fill(const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col, int64_t N,
                             const int64_t* __restrict__ bounds, int S, int32_t chunk,
                             const uint8_t* __restrict__ row_mask,
                             const int64_t* __restrict__ n_items, const int64_t* __restrict__ item_off,
                             const int32_t* __restrict__ n_part, const int32_t* __restrict__ part_off,
                             const int32_t* __restrict__ n_split, const int32_t* __restrict__ split_off,
                             lgcn_item_t* __restrict__ raw, uint32_t* __restrict__ keys, int32_t* __restrict__ idx,
                             lgcn_split_t* __restrict__ splits, int64_t* __restrict__ counts) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < N; i += stride) {
        const int64_t beg = rowptr[i], end = rowptr[i + 1];
        int64_t o = item_off[i];
        auto emit = [&](int64_t b, int32_t lenflags, int32_t dst, int sl, int32_t len) {
            lgcn_item_t it;
            it.beg = b;
            it.len = lenflags;
            it.dst = dst;
            raw[o] = it;
            // slice-major, longest first inside a slice
            const uint32_t l24 = static_cast<uint32_t>(len < 0xFFFFFF ? len : 0xFFFFFF);
            keys[o] = (static_cast<uint32_t>(sl) << 24) | (0xFFFFFFu - l24);
            idx[o] = static_cast<int32_t>(o);
            ++o;
        };
        if (row_mask != nullptr && row_mask[i] == 0) {
            // no items
        } else if (end == beg) {
            emit(beg, kSliceFirst | kSliceLast, static_cast<int32_t>(i), 0, 0);
        } else {
            const bool hub = n_part[i] > 0;
            int32_t pk = 0;  // hub rows: next partial slot, in CSR order
            for_each_segment(col, beg, end, bounds, S, [&](int64_t sb, int64_t e, int sl) {
                const int64_t len = e - sb;
                if (hub) {
                    for (int64_t c0 = 0; c0 < len; c0 += chunk) {
                        const int32_t l = static_cast<int32_t>(len - c0 < chunk ? len - c0 : chunk);
                        emit(sb + c0, l, -(part_off[i] + pk) - 1, sl, l);
                        ++pk;
                    }
                } else {
                    const int32_t flags = (sb == beg ? kSliceFirst : 0) | (e == end ? kSliceLast : 0);
                    emit(sb, static_cast<int32_t>(len) | flags, static_cast<int32_t>(i), sl, static_cast<int32_t>(len));
                }
            });
            if (hub) {
                lgcn_split_t sp;
                sp.row = static_cast<int32_t>(i);
                sp.pbeg = part_off[i];
                sp.pcnt = n_part[i];
                sp.pad = 0;
                splits[split_off[i]] = sp;
            }
        }
        if (i == N - 1) {
            counts[0] = item_off[i] + n_items[i];
            counts[1] = split_off[i] + n_split[i];
            counts[2] = part_off[i] + n_part[i];
        }
    }
}

// offsets[s] = first sorted item of slice s (lower bound of s << 24), s = 0..S
__global__ void k_slice_offsets(const uint32_t* __restrict__ skeys, int64_t n, int S, int64_t* __restrict__ offsets) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s > S) return;
    const uint32_t key = static_cast<uint32_t>(s) << 24;
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (skeys[mid] < key) lo = mid + 1;
        else hi = mid;
    }
    offsets[s] = lo;  // offsets[S] = number of real items (padding keys sort after S << 24)
}

int64_t slice_items_cap(int64_t E, int64_t N, int S, int32_t chunk) {
    const int64_t segs = E < N * int64_t(S) ? E : N * int64_t(S);
    return segs + E / chunk + N + 1;
}

// ---- to_undirected / coalesce (reference data/dataset_handler.py:141, PyG 2.4.0) ----
__global__ void k_pair_keys(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int64_t P, int64_t N,
                            unsigned long long* __restrict__ keys, int32_t* __restrict__ bad) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < P; i += stride) {
        const int64_t a = src[i], b = dst[i];
        if (a < 0 || a >= N || b < 0 || b >= N) atomicOr(bad, 1);
        const int64_t ca = a < 0 ? 0 : (a >= N ? N - 1 : a);
        const int64_t cb = b < 0 ? 0 : (b >= N ? N - 1 : b);
        keys[i] = static_cast<unsigned long long>(ca) * static_cast<unsigned long long>(N) + static_cast<unsigned long long>(cb);
        keys[P + i] = static_cast<unsigned long long>(cb) * static_cast<unsigned long long>(N) + static_cast<unsigned long long>(ca);
    }
}

__global__ void k_unique_flags(const unsigned long long* __restrict__ k, int64_t n, int32_t* __restrict__ flag) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
        flag[i] = (i == 0 || k[i] != k[i - 1]) ? 1 : 0;
}

__global__ void k_unique_scatter(const unsigned long long* __restrict__ k, const int32_t* __restrict__ flag,
                                 const int32_t* __restrict__ pos, int64_t n, int64_t N, int64_t* __restrict__ row,
                                 int64_t* __restrict__ col, int64_t* __restrict__ count) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        if (flag[i]) {
            const unsigned long long v = k[i];
            row[pos[i]] = static_cast<int64_t>(v / static_cast<unsigned long long>(N));
            col[pos[i]] = static_cast<int64_t>(v % static_cast<unsigned long long>(N));
        }
        if (i == n - 1) count[0] = pos[i] + flag[i];
    }
}

size_t coalesce_cub_bytes(int64_t n, int bits) {
    size_t a = 0, b = 0;
    (void)hipcub::DeviceRadixSort::SortKeys(nullptr, a, (const unsigned long long*)nullptr,
                                            (unsigned long long*)nullptr, static_cast<int>(n), 0, bits);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (const int32_t*)nullptr, (int32_t*)nullptr, static_cast<int>(n));
    return a > b ? a : b;
}

int coalesce_bits(int64_t N) {
    int b = 1;
    while (b < 64 && (b >= 63 || (int64_t(1) << b) < N * N)) ++b;
    return b;
}

// sizes of the cub temp storage we need
size_t csr_cub_bytes(int64_t E, int64_t N) {
    size_t t = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, t, (const int32_t*)nullptr, (int32_t*)nullptr,
                                       (const int32_t*)nullptr, (int32_t*)nullptr,
                                       static_cast<int>(E), 0, key_bits(N));
    return t;
}

int64_t sched_items_cap(int64_t E, int64_t N, int32_t chunk) { return N + E / chunk + 1; }

size_t sched_cub_bytes(int64_t E, int64_t N, int32_t chunk) {
    const int64_t cap = sched_items_cap(E, N, chunk);
    size_t a = 0, b = 0, c = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, a, (const int64_t*)nullptr, (int64_t*)nullptr,
                                     static_cast<int>(N));
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (const int32_t*)nullptr, (int32_t*)nullptr,
                                     static_cast<int>(N));
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, c, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                       (const int32_t*)nullptr, (int32_t*)nullptr,
                                       static_cast<int>(cap), 0, 32);
    size_t m = a > b ? a : b;
    return m > c ? m : c;
}


// ---- key grouping (lgcn_group_keys): a counting sort in five stream-ordered steps ----
// Every index a kernel writes through is checked against the range it must fall in; a check
// that fails counts in err (and the write is dropped) instead of faulting.

__device__ __forceinline__ int64_t group_key(const int64_t* __restrict__ key, int64_t b, int64_t R, bool& bad) {
    const int64_t k = key[b];
    bad = (k < 0) | (k >= R);
    return bad ? 0 : k;  // lgcn_csr_build groups a bad key under 0
}

__global__ void k_group_count(const int64_t* __restrict__ key, int64_t B, int64_t R, int32_t* __restrict__ count,
                              unsigned long long* __restrict__ err) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    unsigned long long bad_local = 0;
    for (int64_t b = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; b < B; b += stride) {
        bool bad;
        const int64_t k = group_key(key, b, R, bad);
        bad_local += bad;
        atomicAdd(&count[k], 1);
    }
    if (bad_local) atomicAdd(err, bad_local);
}

// Exclusive scan of count[0..R) in two parallel passes over tiles of kScanTile keys (one key per
// thread, coalesced): k_group_tile_sums writes each tile's total to tsum[t]; k_group_scan then
// adds, per tile, the totals of the tiles before it to a block scan of its keys and writes
// rowptr[r] and cursor[r] = start of key r (cursor overwrites count in place); the last tile also
// writes rowptr[R]. (A one-workgroup scan serialises either its tiles' global round trips or
// uncoalesced segment loads on one CU: 42-50 us at R = 59,047.)
constexpr int kScanTile = 1024;
__global__ __launch_bounds__(kScanTile) void k_group_tile_sums(const int32_t* __restrict__ count, int64_t R,
                                                               int32_t* __restrict__ tsum) {
    using Reduce = hipcub::BlockReduce<int32_t, kScanTile>;
    __shared__ typename Reduce::TempStorage tmp;
    const int64_t i = int64_t(blockIdx.x) * kScanTile + threadIdx.x;
    const int32_t v = i < R ? count[i] : 0;
    const int32_t t = Reduce(tmp).Sum(v);
    if (threadIdx.x == 0) tsum[blockIdx.x] = t;
}

__global__ __launch_bounds__(kScanTile) void k_group_scan(int32_t* __restrict__ count_cursor, int64_t R,
                                                          const int32_t* __restrict__ tsum,
                                                          int64_t* __restrict__ rowptr, int64_t B,
                                                          unsigned long long* __restrict__ err) {
    using Scan = hipcub::BlockScan<int32_t, kScanTile>;
    using Reduce = hipcub::BlockReduce<int32_t, kScanTile>;
    __shared__ typename Scan::TempStorage tmp;
    __shared__ typename Reduce::TempStorage rtmp;
    // the totals of the tiles before this one (a few dozen values: one pass of the block)
    int32_t before = 0;
    for (int64_t t = threadIdx.x; t < blockIdx.x; t += kScanTile) before += tsum[t];
    const int32_t offset = Reduce(rtmp).Sum(before);  // valid in thread 0
    __shared__ int32_t s_off;
    if (threadIdx.x == 0) s_off = offset;
    const int64_t i = int64_t(blockIdx.x) * kScanTile + threadIdx.x;
    const int32_t v = i < R ? count_cursor[i] : 0;
    int32_t pre, total;
    Scan(tmp).ExclusiveSum(v, pre, total);
    __syncthreads();
    const int32_t run = s_off + pre;
    if (i < R) {
        rowptr[i] = run;
        count_cursor[i] = run;
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
        rowptr[R] = s_off + total;
        // the counts must add up to the B keys: anything else means the count array was not zero
        // on entry (the cursor contract broken), and every later index would be off
        if (s_off + total != B) atomicAdd(err, 1ull << 32);
    }
}

__global__ void k_group_place(const int64_t* __restrict__ key, int64_t B, int64_t R,
                              const int64_t* __restrict__ rowptr, int32_t* __restrict__ cursor,
                              int32_t* __restrict__ perm, unsigned long long* __restrict__ err) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t b = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; b < B; b += stride) {
        bool bad;
        const int64_t k = group_key(key, b, R, bad);
        const int32_t pos = atomicAdd(&cursor[k], 1);
        // cannot happen when count and key agree; pos < B also holds a corrupted rowptr to perm's size
        if (pos < rowptr[k] || pos >= rowptr[k + 1] || pos >= B) {
            atomicAdd(err, 1ull << 32);
            continue;
        }
        perm[pos] = static_cast<int32_t>(b);
    }
}

// Each key's positions in ascending order (insertion sort; groups are a few entries long); the
// cursor is zeroed for the next call (no memset node in a captured step).
__global__ void k_group_order(const int64_t* __restrict__ rowptr, int64_t R, int32_t* __restrict__ perm,
                              int32_t* __restrict__ cursor, int64_t B, unsigned long long* __restrict__ err) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t r = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; r < R; r += stride) {
        cursor[r] = 0;
        const int64_t beg = rowptr[r], end = rowptr[r + 1];
        if (beg < 0 || end < beg || end > B) {  // a corrupted rowptr: count it, write nothing
            atomicAdd(err, 1ull << 32);
            continue;
        }
        for (int64_t i = beg + 1; i < end; ++i) {
            const int32_t v = perm[i];
            int64_t j = i - 1;
            while (j >= beg && perm[j] > v) {
                perm[j + 1] = perm[j];
                --j;
            }
            perm[j + 1] = v;
        }
    }
}

// ---- content digest of a device buffer (lgcn_digest128) ---------------------------------------
// The per-batch caches find a batch's plans / captured graph by the CONTENT of its edge_index
// (lgcn_amd._cache). For a device tensor that was a copy to the host and XXH3 there, one sync per
// new tensor object; this is the on-device digest: two independent 64-bit lanes, each the sum
// mod 2^64 over the 8-byte words w_i of a keyed mix f(w_i, i) (murmur3's fmix64 finaliser), then
// the length folded in. Sums mod 2^64 associate exactly, so the digest is deterministic for any
// grid; the word index inside the mix makes it order-sensitive. Not cryptographic (nor is XXH3):
// an accidental collision needs two equal-shaped batches with equal 128-bit sums.
__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

__device__ __forceinline__ void digest_word(uint64_t w, uint64_t i, uint64_t& a, uint64_t& b) {
    a += fmix64(w ^ fmix64(i * 0x9e3779b97f4a7c15ull + 0x243f6a8885a308d3ull));
    b += fmix64((w + 0x632be59bd9b4e019ull) * 0xd6e8feb86659fd93ull ^ fmix64(i + 0x8cb92ba72f3d8dd7ull));
}

__device__ __forceinline__ void block_sum2(uint64_t& a, uint64_t& b) {
    __shared__ uint64_t red[kBlock / 64][2];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        a += __shfl_xor(a, off, 64);
        b += __shfl_xor(b, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        red[threadIdx.x >> 6][0] = a;
        red[threadIdx.x >> 6][1] = b;
    }
    __syncthreads();
    a = b = 0;
    if (threadIdx.x == 0)
        for (int w = 0; w < kBlock / 64; ++w) {
            a += red[w][0];
            b += red[w][1];
        }
}

__global__ __launch_bounds__(kBlock) void k_digest_partial(const uint64_t* __restrict__ words, int64_t nwords,
                                                           const uint8_t* __restrict__ tail, int32_t ntail,
                                                           uint64_t* __restrict__ ws) {
    uint64_t a = 0, b = 0;
    for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < nwords; i += int64_t(gridDim.x) * kBlock)
        digest_word(words[i], static_cast<uint64_t>(i), a, b);
    if (ntail > 0 && blockIdx.x == 0 && threadIdx.x == 0) {  // the last < 8 bytes as one word
        uint64_t w = 0;
        for (int j = 0; j < ntail; ++j) w |= static_cast<uint64_t>(tail[j]) << (8 * j);
        digest_word(w, static_cast<uint64_t>(nwords), a, b);
    }
    block_sum2(a, b);
    if (threadIdx.x == 0) {
        ws[2 * blockIdx.x] = a;
        ws[2 * blockIdx.x + 1] = b;
    }
}

__global__ __launch_bounds__(kBlock) void k_digest_final(const uint64_t* __restrict__ ws, int32_t nblocks,
                                                         int64_t nbytes, uint64_t* __restrict__ out) {
    uint64_t a = 0, b = 0;
    for (int i = threadIdx.x; i < nblocks; i += kBlock) {
        a += ws[2 * i];
        b += ws[2 * i + 1];
    }
    block_sum2(a, b);
    if (threadIdx.x == 0) {
        out[0] = fmix64(a ^ static_cast<uint64_t>(nbytes));
        out[1] = fmix64(b + static_cast<uint64_t>(nbytes) * 0x9e3779b97f4a7c15ull);
    }
}

}  // namespace

extern "C" {

const char* lgcn_last_error(void) { return err_buf(); }

int lgcn_digest128(const void* data, int64_t nbytes, uint64_t* ws, int64_t ws_words, uint64_t* out,
                   lgcn_stream_t stream) {
    if (nbytes < 0 || (nbytes > 0 && !data) || !ws || !out || (reinterpret_cast<uintptr_t>(data) & 7) ||
        ws_words < 2 * LGCN_DIGEST_BLOCKS)
        return fail(LGCN_E_ARG, "lgcn_digest128: bad args (nbytes=%lld ws_words=%lld, data 8-byte aligned)",
                    (long long)nbytes, (long long)ws_words);
    const int64_t nwords = nbytes / 8;
    int64_t blocks = (nwords + kBlock * 8 - 1) / (kBlock * 8);  // >= 8 words per thread
    if (blocks < 1) blocks = 1;
    if (blocks > LGCN_DIGEST_BLOCKS) blocks = LGCN_DIGEST_BLOCKS;
    hipStream_t s = as_stream(stream);
    const uint8_t* bytes = static_cast<const uint8_t*>(data);
    k_digest_partial<<<dim3(static_cast<unsigned>(blocks)), kBlock, 0, s>>>(
        static_cast<const uint64_t*>(data), nwords, bytes + nwords * 8, static_cast<int32_t>(nbytes & 7), ws);
    int rc = check_launch("k_digest_partial");
    if (rc != LGCN_OK) return rc;
    k_digest_final<<<1, kBlock, 0, s>>>(ws, static_cast<int32_t>(blocks), nbytes, out);
    return check_launch("k_digest_final");
}
int lgcn_abi_version(void) { return LGCN_ABI_VERSION; }

int lgcn_csr_workspace_size(int64_t E, int64_t N, size_t* bytes) {
    if (!bytes || E < 0 || N < 0) return fail(LGCN_E_ARG, "lgcn_csr_workspace_size: bad args");
    if (E > INT32_MAX || N > INT32_MAX)
        return fail(LGCN_E_UNSUPPORTED, "lgcn_csr_workspace_size: E=%lld N=%lld exceed int32",
                    (long long)E, (long long)N);
    Carver c{nullptr, 0};
    c.take<int32_t>(E);  // key32 in
    c.take<int32_t>(E);  // key32 out
    c.take<int32_t>(E);  // eid in
    c.take<char>(csr_cub_bytes(E, N > 0 ? N : 1));
    *bytes = c.used + 256;
    return LGCN_OK;
}

int lgcn_csr_build(const int64_t* key, const int64_t* other, int64_t E, int64_t N,
                   int64_t* rowptr, int32_t* col, int32_t* eid, int64_t* err_count, void* ws,
                   size_t ws_bytes, lgcn_stream_t stream) {
    if (E < 0 || N < 0 || !rowptr || !err_count || (E > 0 && (!key || !other || !col || !eid)))
        return fail(LGCN_E_ARG, "lgcn_csr_build: bad args");
    if (E > INT32_MAX || N > INT32_MAX)
        return fail(LGCN_E_UNSUPPORTED, "lgcn_csr_build: E=%lld N=%lld exceed int32",
                    (long long)E, (long long)N);
    hipStream_t s = as_stream(stream);
    if (E == 0) {
        int rc = check_hip(hipMemsetAsync(rowptr, 0, sizeof(int64_t) * (N + 1), s), "memset rowptr");
        return rc;
    }
    Carver c{static_cast<char*>(ws), ws_bytes};
    int32_t* k_in = c.take<int32_t>(E);
    int32_t* k_out = c.take<int32_t>(E);
    int32_t* e_in = c.take<int32_t>(E);
    size_t cub_bytes = csr_cub_bytes(E, N);
    void* cub_tmp = c.take<char>(cub_bytes);
    if (!c.ok) return fail(LGCN_E_WORKSPACE, "lgcn_csr_build: workspace %zu < %zu", ws_bytes, c.used);

    k_prep_keys<<<grid_for(E, kBlock, 8192), kBlock, 0, s>>>(
        key, other, E, N, k_in, e_in, reinterpret_cast<unsigned long long*>(err_count));
    if (int rc = check_launch("k_prep_keys")) return rc;
    // LSD radix sort is stable: equal keys keep input (edge) order.
    if (int rc = check_hip(hipcub::DeviceRadixSort::SortPairs(cub_tmp, cub_bytes, k_in, k_out, e_in,
                                                              eid, static_cast<int>(E), 0,
                                                              key_bits(N), s),
                           "SortPairs(csr)"))
        return rc;
    k_rowptr_from_sorted<<<grid_for(N + 1, kBlock, 8192), kBlock, 0, s>>>(k_out, E, N, rowptr);
    if (int rc = check_launch("k_rowptr_from_sorted")) return rc;
    k_gather_col<<<grid_for(E, kBlock, 8192), kBlock, 0, s>>>(other, eid, E, N, col);
    return check_launch("k_gather_col");
}

int64_t lgcn_group_keys_cursor_len(int64_t R) { return R + (R + kScanTile - 1) / kScanTile; }

int lgcn_group_keys(const int64_t* key, int64_t B, int64_t R, int64_t* rowptr, int32_t* perm, int32_t* cursor,
                    int64_t* err_count, lgcn_stream_t stream) {
    if (B < 0 || R < 1 || !rowptr || !err_count || !cursor || (B > 0 && (!key || !perm)))
        return fail(LGCN_E_ARG, "lgcn_group_keys: bad args");
    if (B > INT32_MAX || R > INT32_MAX)
        return fail(LGCN_E_UNSUPPORTED, "lgcn_group_keys: B=%lld R=%lld exceed int32", (long long)B, (long long)R);
    hipStream_t s = as_stream(stream);
    auto* err = reinterpret_cast<unsigned long long*>(err_count);
    if (B > 0) {
        k_group_count<<<grid_for(B, kBlock, 4096), kBlock, 0, s>>>(key, B, R, cursor, err);
        if (int rc = check_launch("k_group_count")) return rc;
    }
    const int64_t tiles = (R + kScanTile - 1) / kScanTile;
    int32_t* tsum = cursor + R;  // the tail of the caller's scratch: one total per tile
    k_group_tile_sums<<<static_cast<unsigned>(tiles), kScanTile, 0, s>>>(cursor, R, tsum);
    if (int rc = check_launch("k_group_tile_sums")) return rc;
    k_group_scan<<<static_cast<unsigned>(tiles), kScanTile, 0, s>>>(cursor, R, tsum, rowptr, B, err);
    if (int rc = check_launch("k_group_scan")) return rc;
    if (B > 0) {
        k_group_place<<<grid_for(B, kBlock, 4096), kBlock, 0, s>>>(key, B, R, rowptr, cursor, perm, err);
        if (int rc = check_launch("k_group_place")) return rc;
    }
    k_group_order<<<grid_for(R, kBlock, 4096), kBlock, 0, s>>>(rowptr, R, perm, cursor, B, err);
    return check_launch("k_group_order");
}

int lgcn_inv_sqrt_degree(const int64_t* rowptr_fwd, int64_t N, float* dis, lgcn_stream_t stream) {
    if (N < 0 || !rowptr_fwd || (N > 0 && !dis)) return fail(LGCN_E_ARG, "lgcn_inv_sqrt_degree: bad args");
    if (N == 0) return LGCN_OK;
    k_inv_sqrt_degree<<<grid_for(N, kBlock, 8192), kBlock, 0, as_stream(stream)>>>(rowptr_fwd, N, dis);
    return check_launch("k_inv_sqrt_degree");
}

int lgcn_edge_norm(const int64_t* rowptr, const int32_t* col, int64_t N, int64_t E,
                   const float* dis, float* val, lgcn_stream_t stream) {
    if (N < 0 || E < 0 || !rowptr || (E > 0 && (!col || !dis || !val)))
        return fail(LGCN_E_ARG, "lgcn_edge_norm: bad args");
    if (E == 0) return LGCN_OK;
    if (N == 0) return fail(LGCN_E_ARG, "lgcn_edge_norm: E > 0 with N == 0");
    k_edge_norm<<<grid_for(E, kBlock, 8192), kBlock, 0, as_stream(stream)>>>(rowptr, col, N, E, dis, val);
    return check_launch("k_edge_norm");
}

int lgcn_schedule_workspace_size(int64_t E, int64_t N, int32_t chunk, size_t* bytes) {
    if (!bytes || E < 0 || N < 0 || chunk < 1) return fail(LGCN_E_ARG, "lgcn_schedule_workspace_size: bad args");
    if (N > INT32_MAX || E > INT32_MAX) return fail(LGCN_E_UNSUPPORTED, "schedule: sizes exceed int32");
    const int64_t cap = sched_items_cap(E, N, chunk);
    Carver c{nullptr, 0};
    c.take<int64_t>(N);          // n_items
    c.take<int64_t>(N);          // item_off
    c.take<int32_t>(N);          // n_part
    c.take<int32_t>(N);          // part_off
    c.take<int32_t>(N);          // n_split
    c.take<int32_t>(N);          // split_off
    c.take<lgcn_item_t>(cap);    // raw items
    c.take<uint32_t>(cap);       // keys in
    c.take<uint32_t>(cap);       // keys out
    c.take<int32_t>(cap);        // idx in
    c.take<int32_t>(cap);        // idx out
    c.take<char>(sched_cub_bytes(E, N > 0 ? N : 1, chunk));
    *bytes = c.used + 256;
    return LGCN_OK;
}

int lgcn_schedule_build(const int64_t* rowptr, int64_t N, int64_t E, int32_t chunk, int64_t side_split,
                        const uint8_t* row_mask, lgcn_item_t* items, int64_t items_cap, lgcn_split_t* splits,
                        int64_t splits_cap, int64_t* counts, void* ws, size_t ws_bytes,
                        lgcn_stream_t stream) {
    if (!rowptr || !counts || N < 0 || E < 0 || chunk < 1 || chunk >= (1 << 30) || side_split < 0)
        return fail(LGCN_E_ARG, "lgcn_schedule_build: bad args");
    if (N > INT32_MAX || E > INT32_MAX) return fail(LGCN_E_UNSUPPORTED, "schedule: sizes exceed int32");
    hipStream_t s = as_stream(stream);
    if (N == 0) return check_hip(hipMemsetAsync(counts, 0, 3 * sizeof(int64_t), s), "memset counts");
    const int64_t cap = sched_items_cap(E, N, chunk);
    if (!items || items_cap < cap || !splits || splits_cap < N)
        return fail(LGCN_E_ARG, "lgcn_schedule_build: items_cap %lld < %lld or splits_cap %lld < %lld",
                    (long long)items_cap, (long long)cap, (long long)splits_cap, (long long)N);
    Carver c{static_cast<char*>(ws), ws_bytes};
    int64_t* n_items = c.take<int64_t>(N);
    int64_t* item_off = c.take<int64_t>(N);
    int32_t* n_part = c.take<int32_t>(N);
    int32_t* part_off = c.take<int32_t>(N);
    int32_t* n_split = c.take<int32_t>(N);
    int32_t* split_off = c.take<int32_t>(N);
    lgcn_item_t* raw = c.take<lgcn_item_t>(cap);
    uint32_t* k_in = c.take<uint32_t>(cap);
    uint32_t* k_out = c.take<uint32_t>(cap);
    int32_t* i_in = c.take<int32_t>(cap);
    int32_t* i_out = c.take<int32_t>(cap);
    size_t cub_bytes = sched_cub_bytes(E, N, chunk);
    void* cub_tmp = c.take<char>(cub_bytes);
    if (!c.ok) return fail(LGCN_E_WORKSPACE, "lgcn_schedule_build: workspace %zu < %zu", ws_bytes, c.used);

    const unsigned g = grid_for(N, kBlock, 8192);
    k_sched_count<<<g, kBlock, 0, s>>>(rowptr, N, chunk, row_mask, n_items, n_part, n_split);
    if (int rc = check_launch("k_sched_count")) return rc;
    size_t t = cub_bytes;
    if (int rc = check_hip(hipcub::DeviceScan::ExclusiveSum(cub_tmp, t, n_items, item_off, static_cast<int>(N), s), "scan items")) return rc;
    t = cub_bytes;
    if (int rc = check_hip(hipcub::DeviceScan::ExclusiveSum(cub_tmp, t, n_part, part_off, static_cast<int>(N), s), "scan parts")) return rc;
    t = cub_bytes;
    if (int rc = check_hip(hipcub::DeviceScan::ExclusiveSum(cub_tmp, t, n_split, split_off, static_cast<int>(N), s), "scan splits")) return rc;
    // padding slots [n_items, cap) sort last (key = chunk + 1) and are never read
    const uint32_t pad_key = 0xFFFFFFFFu;  // sorts after both sides
    k_fill_u32<<<grid_for(cap, kBlock, 8192), kBlock, 0, s>>>(k_in, cap, pad_key);
    if (int rc = check_launch("k_fill_u32")) return rc;
    k_fill_u32<<<grid_for(cap, kBlock, 8192), kBlock, 0, s>>>(reinterpret_cast<uint32_t*>(i_in), cap, 0u);
    if (int rc = check_launch("k_fill_u32")) return rc;
    k_sched_fill<<<g, kBlock, 0, s>>>(rowptr, N, chunk, side_split, n_items, item_off, n_part, part_off, n_split,
                                      split_off, raw, k_in, i_in, splits, counts);
    if (int rc = check_launch("k_sched_fill")) return rc;
    t = cub_bytes;
    if (int rc = check_hip(hipcub::DeviceRadixSort::SortPairs(cub_tmp, t, k_in, k_out, i_in, i_out,
                                                              static_cast<int>(cap), 0, 32, s),
                           "SortPairs(schedule)"))
        return rc;
    // gather all cap slots; the tail beyond n_items is padding the kernels never index
    k_sched_gather<<<grid_for(cap, kBlock, 8192), kBlock, 0, s>>>(raw, i_out, cap, items);
    return check_launch("k_sched_gather");
}


int lgcn_slice_schedule_workspace_size(int64_t E, int64_t N, int32_t S, int32_t chunk, size_t* bytes,
                                       int64_t* items_cap) {
    if (!bytes || E < 0 || N < 0 || S < 1 || S > 250 || chunk < 1)
        return fail(LGCN_E_ARG, "lgcn_slice_schedule_workspace_size: bad args");
    const int64_t cap = slice_items_cap(E, N, S, chunk);
    if (items_cap) *items_cap = cap;
    size_t a = 0, b = 0, c = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, a, (const int64_t*)nullptr, (int64_t*)nullptr,
                                           static_cast<int>(N > 0 ? N : 1));
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (const int32_t*)nullptr, (int32_t*)nullptr,
                                           static_cast<int>(N > 0 ? N : 1));
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, c, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (const int32_t*)nullptr, (int32_t*)nullptr, static_cast<int>(cap), 0,
                                             32);
    size_t m = a > b ? a : b;
    m = m > c ? m : c;
    Carver cv{nullptr, 0};
    cv.take<int64_t>(N);
    cv.take<int64_t>(N);
    cv.take<int32_t>(N);
    cv.take<int32_t>(N);
    cv.take<int32_t>(N);
    cv.take<int32_t>(N);
    cv.take<lgcn_item_t>(cap);
    cv.take<uint32_t>(cap);
    cv.take<uint32_t>(cap);
    cv.take<int32_t>(cap);
    cv.take<int32_t>(cap);
    cv.take<char>(m);
    *bytes = cv.used + 256;
    return LGCN_OK;
}

int lgcn_slice_schedule_build(const int64_t* rowptr, const int32_t* col, int64_t N, int64_t E,
                              const int64_t* bounds, int32_t S, int32_t chunk, const uint8_t* row_mask,
                              lgcn_item_t* items, int64_t items_cap,
                              int64_t* offsets, lgcn_split_t* splits, int64_t splits_cap, int64_t* counts,
                              void* ws, size_t ws_bytes, lgcn_stream_t stream) {
    if (!rowptr || !bounds || !counts || !offsets || N <= 0 || E < 0 || S < 1 || S > 250 || chunk < 1 ||
        chunk >= (1 << 24) || (E > 0 && !col))
        return fail(LGCN_E_ARG, "lgcn_slice_schedule_build: bad args");
    if (N > INT32_MAX || E > INT32_MAX) return fail(LGCN_E_UNSUPPORTED, "slice schedule: sizes exceed int32");
    hipStream_t s = as_stream(stream);
    const int64_t cap = slice_items_cap(E, N, S, chunk);
    if (!items || items_cap < cap || !splits || splits_cap < N)
        return fail(LGCN_E_ARG, "lgcn_slice_schedule_build: items_cap %lld < %lld or splits_cap %lld < %lld",
                    (long long)items_cap, (long long)cap, (long long)splits_cap, (long long)N);
    Carver c{static_cast<char*>(ws), ws_bytes};
    int64_t* n_items = c.take<int64_t>(N);
    int64_t* item_off = c.take<int64_t>(N);
    int32_t* n_part = c.take<int32_t>(N);
    int32_t* part_off = c.take<int32_t>(N);
    int32_t* n_split = c.take<int32_t>(N);
    int32_t* split_off = c.take<int32_t>(N);
    lgcn_item_t* raw = c.take<lgcn_item_t>(cap);
    uint32_t* k_in = c.take<uint32_t>(cap);
    uint32_t* k_out = c.take<uint32_t>(cap);
    int32_t* i_in = c.take<int32_t>(cap);
    int32_t* i_out = c.take<int32_t>(cap);
    size_t a = 0, b = 0, cb = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, a, (const int64_t*)nullptr, (int64_t*)nullptr, static_cast<int>(N));
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (const int32_t*)nullptr, (int32_t*)nullptr, static_cast<int>(N));
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, cb, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (const int32_t*)nullptr, (int32_t*)nullptr, static_cast<int>(cap), 0, 32);
    size_t cub_bytes = a > b ? a : b;
    cub_bytes = cub_bytes > cb ? cub_bytes : cb;
    void* cub_tmp = c.take<char>(cub_bytes);
    if (!c.ok) return fail(LGCN_E_WORKSPACE, "lgcn_slice_schedule_build: workspace %zu < %zu", ws_bytes, c.used);
    // counts[3] = 1 if some row's neighbours are not ascending (the caller falls back)
    if (int rc = check_hip(hipMemsetAsync(counts, 0, 4 * sizeof(int64_t), s), "memset counts")) return rc;
    const unsigned g = grid_for(N, kBlock, 8192);
    k_slice_count<<<grid_for(N * 64, kBlock, 8192), kBlock, 0, s>>>(rowptr, col, N, bounds, S, chunk, row_mask,
                                                                     n_items, n_part,
                                                                     n_split,
                                       reinterpret_cast<int32_t*>(counts + 3));
    if (int rc = check_launch("k_slice_count")) return rc;
    size_t t = cub_bytes;
    if (int rc = check_hip(hipcub::DeviceScan::ExclusiveSum(cub_tmp, t, n_items, item_off, static_cast<int>(N), s), "scan items")) return rc;
    t = cub_bytes;
    if (int rc = check_hip(hipcub::DeviceScan::ExclusiveSum(cub_tmp, t, n_part, part_off, static_cast<int>(N), s), "scan parts")) return rc;
    t = cub_bytes;
    if (int rc = check_hip(hipcub::DeviceScan::ExclusiveSum(cub_tmp, t, n_split, split_off, static_cast<int>(N), s), "scan splits")) return rc;
    k_fill_u32<<<grid_for(cap, kBlock, 8192), kBlock, 0, s>>>(k_in, cap, 0xFFFFFFFFu);
    if (int rc = check_launch("k_fill_u32")) return rc;
    k_fill_u32<<<grid_for(cap, kBlock, 8192), kBlock, 0, s>>>(reinterpret_cast<uint32_t*>(i_in), cap, 0u);
    if (int rc = check_launch("k_fill_u32")) return rc;
    k_slice_fill<<<g, kBlock, 0, s>>>(rowptr, col, N, bounds, S, chunk, row_mask, n_items, item_off, n_part, part_off, n_split,
                                      split_off, raw, k_in, i_in, splits, counts);
    if (int rc = check_launch("k_slice_fill")) return rc;
    t = cub_bytes;
    if (int rc = check_hip(hipcub::DeviceRadixSort::SortPairs(cub_tmp, t, k_in, k_out, i_in, i_out,
                                                              static_cast<int>(cap), 0, 32, s),
                           "SortPairs(slice schedule)"))
        return rc;
    k_sched_gather<<<grid_for(cap, kBlock, 8192), kBlock, 0, s>>>(raw, i_out, cap, items);
    if (int rc = check_launch("k_sched_gather")) return rc;
    // offsets over the sorted keys; padding keys (0xFFFFFFFF) sort after every real slice
    k_slice_offsets<<<1, 256, 0, s>>>(k_out, cap, S, offsets);
    return check_launch("k_slice_offsets");
}


int lgcn_coalesce_workspace_size(int64_t P, int64_t N, size_t* bytes) {
    if (!bytes || P < 0 || N < 0) return fail(LGCN_E_ARG, "lgcn_coalesce_workspace_size: bad args");
    if (2 * P > INT32_MAX || N > (int64_t(1) << 31)) return fail(LGCN_E_UNSUPPORTED, "coalesce: sizes exceed int32");
    const int64_t n = 2 * P > 0 ? 2 * P : 1;
    Carver c{nullptr, 0};
    c.take<unsigned long long>(n);
    c.take<unsigned long long>(n);
    c.take<int32_t>(n);
    c.take<int32_t>(n);
    c.take<int32_t>(1);
    c.take<char>(coalesce_cub_bytes(n, coalesce_bits(N > 1 ? N : 2)));
    *bytes = c.used + 256;
    return LGCN_OK;
}

int lgcn_coalesce_undirected(const int64_t* src, const int64_t* dst, int64_t P, int64_t N, int64_t* out_row,
                             int64_t* out_col, int64_t* out_count, int64_t* err_count, void* ws, size_t ws_bytes,
                             lgcn_stream_t stream) {
    if (P < 0 || N <= 0 || !out_count || !err_count || (P > 0 && (!src || !dst || !out_row || !out_col)))
        return fail(LGCN_E_ARG, "lgcn_coalesce_undirected: bad args");
    if (2 * P > INT32_MAX) return fail(LGCN_E_UNSUPPORTED, "coalesce: sizes exceed int32");
    hipStream_t s = as_stream(stream);
    if (int rc = check_hip(hipMemsetAsync(out_count, 0, sizeof(int64_t), s), "memset count")) return rc;
    if (int rc = check_hip(hipMemsetAsync(err_count, 0, sizeof(int64_t), s), "memset err")) return rc;
    if (P == 0) return LGCN_OK;
    const int64_t n = 2 * P;
    const int bits = coalesce_bits(N > 1 ? N : 2);
    Carver c{static_cast<char*>(ws), ws_bytes};
    auto* k_in = c.take<unsigned long long>(n);
    auto* k_out = c.take<unsigned long long>(n);
    int32_t* flag = c.take<int32_t>(n);
    int32_t* pos = c.take<int32_t>(n);
    c.take<int32_t>(1);
    const size_t cub_bytes = coalesce_cub_bytes(n, bits);
    void* cub_tmp = c.take<char>(cub_bytes);
    if (!c.ok) return fail(LGCN_E_WORKSPACE, "lgcn_coalesce_undirected: workspace %zu < %zu", ws_bytes, c.used);
    const unsigned g = grid_for(n, kBlock, 16384);
    k_pair_keys<<<grid_for(P, kBlock, 16384), kBlock, 0, s>>>(src, dst, P, N, k_in,
                                                              reinterpret_cast<int32_t*>(err_count));
    if (int rc = check_launch("k_pair_keys")) return rc;
    size_t t = cub_bytes;
    if (int rc = check_hip(hipcub::DeviceRadixSort::SortKeys(cub_tmp, t, k_in, k_out, static_cast<int>(n), 0, bits, s),
                           "SortKeys(coalesce)"))
        return rc;
    k_unique_flags<<<g, kBlock, 0, s>>>(k_out, n, flag);
    if (int rc = check_launch("k_unique_flags")) return rc;
    t = cub_bytes;
    if (int rc = check_hip(hipcub::DeviceScan::ExclusiveSum(cub_tmp, t, flag, pos, static_cast<int>(n), s), "scan unique"))
        return rc;
    k_unique_scatter<<<g, kBlock, 0, s>>>(k_out, flag, pos, n, N, out_row, out_col, out_count);
    return check_launch("k_unique_scatter");
}

}  // extern "C"
