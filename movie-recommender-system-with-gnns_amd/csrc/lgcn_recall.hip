// Recall@k of the reference's evaluate() (reference utils/train_test.py:165-212) on gfx950.
//
// The reference scores sample_size sampled "user" rows against every positive and negative row
// of the edge set (cosine = mm of L2-normalised rows), takes torch.topk(k) per user and counts
// the hits that are positives (index < P). Per user, that count is all we need, so nothing of
// the [Q, M] score matrix is kept:
//
//   k_normalize_rows  x[r] / ||x[r]|| (optionally gathered through an index list), written into a
//                     zero-padded [rows, D] image (D = the compiled width >= d);
//   k_score_filter    f32 MFMA (v_mfma_f32_32x32x2_f32, exact f32) scores of 32-query blocks
//                     against 32-candidate blocks; an epilogue keeps (key, index) of every score
//                     at or above the query's threshold key in a per-query list;
//   k_select_topk     one workgroup per query: radix select (4 x 8-bit passes) of the k-th
//                     largest key in its list, then either that key (a new threshold) or the
//                     hit count (positives above it, plus positives among the ties).
//
// Thresholds come from a strided candidate subset first: the k-th largest score of ANY subset is
// <= the k-th largest of all M, so the filtered list always holds the true top k, and it holds
// about k * M / |subset| entries. If a list overflows its capacity, its kept entries are real
// candidates too, so their k-th largest is again a valid (tighter) threshold and the caller
// re-runs the filter (lgcn_amd.recall does this; it never happens at the reference's sizes).
//
// Ties at the k-th score take the lowest candidate indices first, which are the positives
// (torch.topk leaves tie order unspecified). NaN scores (zero rows, normalised as 0/0 like the
// reference) rank first, as torch.topk ranks NaN above every number.

#include "lgcn_common.h"

using namespace lgcn;

namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;

__device__ __forceinline__ uint32_t score_key(float s) {
    if (s != s) return 0xFFFFFFFFu;
    const uint32_t u = __float_as_uint(s);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// inverse of score_key (the NaN key maps back to a NaN)
__device__ __forceinline__ float key_score(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k ^ 0x80000000u) : ~k);
}

// one 32-lane half-wave per row
__global__ __launch_bounds__(kBlock) void k_normalize_rows(const float* __restrict__ x, const int64_t* __restrict__ idx,
                                                           int64_t rows, int64_t ld, int32_t d,
                                                           float* __restrict__ out, int32_t D, int64_t out_rows) {
    const int64_t r = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / 32;
    const int l = threadIdx.x & 31;
    if (r >= out_rows) return;
    float* o = out + r * D;
    if (r >= rows) {  // padding rows: zeros
        for (int c = l; c < D; c += 32) o[c] = 0.f;
        return;
    }
    const float* src = x + (idx ? idx[r] : r) * ld;
    float ss = 0.f;
    for (int c = l; c < d; c += 32) {
        const float v = src[c];
        ss += v * v;
    }
#pragma unroll
    for (int off = 16; off > 0; off >>= 1) ss += __shfl_xor(ss, off, 32);
    const float n = sqrtf(ss);
    for (int c = l; c < D; c += 32) o[c] = (c < d) ? src[c] / n : 0.f;
}

constexpr int kStage = 512;  // staged accepted scores per wave

// Workgroup = 4 waves over the same candidate blocks; wave w owns the 32 queries
// [(qg*4 + w)*32, +32), held in registers for the whole launch. Lane l = (i = l&31, h = l>>5)
// holds, for MFMA step s, A = Q[i][h*D/2 + s] and B = C[j][h*D/2 + s], so each step's 2-wide k
// slice is columns s and D/2+s and the D/2 steps cover the row.
// Candidate blocks (32 rows) are staged through LDS, double-buffered: the global loads of block
// n+1 are in flight (in registers) while block n's MFMAs run, and land in the other buffer.
// Grid: 1-D, XCD-aware. Workgroup wid runs on XCD wid % 8; the query groups of one candidate
// chunk get consecutive slots of the SAME XCD, so they run together and share its L2 copy of the
// chunk's rows (the queries, not the candidates, are what differs between them).
// At <= 170 VGPRs two waves share each SIMD, so one wave's epilogue hides under the other's MFMAs.
// D = 256 asks for one: its two candidate buffers + staging (≈ 89 KB of LDS per workgroup) leave
// room for one workgroup (one wave per SIMD) per CU whatever the register count.
template <int D>
constexpr int score_filter_waves() { return D >= 256 ? 1 : 2; }

template <int D>
__global__ __launch_bounds__(kBlock, score_filter_waves<D>()) void k_score_filter(const float* __restrict__ Qn, int64_t Qvalid, int32_t nqg,
                                                            int32_t nchunk, const float* __restrict__ Cn, int64_t M,
                                                            int64_t stride, const uint32_t* __restrict__ thr,
                                                            uint32_t* __restrict__ list_key,
                                                            int32_t* __restrict__ list_idx,
                                                            int32_t* __restrict__ list_n, int32_t cap) {
    constexpr int H = D / 2;
    constexpr int ROWF = D + 4;               // padded LDS row: conflict-free ds_read_b128 down a column
    constexpr int NF4 = 32 * D / 4;           // float4s per candidate block
    constexpr int PER = (NF4 + kBlock - 1) / kBlock;
    __shared__ float cs[2][32 * ROWF];
    // wave-private staging of accepted scores: appended without atomics (ballot prefix), flushed
    // to the per-query lists with ONE returning global atomic per query per flush
    __shared__ uint32_t st_key[4][kStage];
    __shared__ int32_t st_idx[4][kStage];
    __shared__ uint8_t st_row[4][kStage];  // query row within the wave's 32
    __shared__ uint16_t st_rank[4][kStage];
    __shared__ int32_t st_cnt[4][32];
    __shared__ int32_t st_base[4][32];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int i = lane & 31;
    const int h = lane >> 5;
    const int wid = blockIdx.x;
    const int slot = wid >> 3;
    const int qg = slot % nqg;
    const int chunk = (slot / nqg) * 8 + (wid & 7);
    const int64_t q0 = (int64_t(qg) * 4 + wv) * 32;  // first query of this wave
    float a[H];
    {
        const float4* src = reinterpret_cast<const float4*>(Qn + (q0 + i) * D + h * H);
#pragma unroll
        for (int v = 0; v < H / 4; ++v) {
            const float4 t = src[v];
            a[4 * v] = t.x;
            a[4 * v + 1] = t.y;
            a[4 * v + 2] = t.z;
            a[4 * v + 3] = t.w;
        }
    }
    // this lane's 16 output rows: (r&3) + 8*(r>>2) + 4h. The test runs on floats, inclusively:
    // !(score < t) keeps every score whose key is >= the threshold key (and NaN, which ranks
    // first, and -0 beside +0 — extra entries are harmless, the selection works on exact keys).
    // Padding queries get +inf (their zero rows score 0).
    float th[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int64_t q = q0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        th[r] = (q < Qvalid) ? (thr ? key_score(thr[q]) : -__builtin_inff()) : __builtin_inff();
    }
    int scnt = 0;  // wave-uniform staged count
    const unsigned long long below = (1ull << lane) - 1ull;
    // flush (wave-uniform): ranks within each query row from LDS atomics (list order does not
    // matter: selection ranks keys), one global atomic per row, then the stores
    auto flush = [&]() {
        if (lane < 32) st_cnt[wv][lane] = 0;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        for (int e = lane; e < scnt; e += 64)
            st_rank[wv][e] = static_cast<uint16_t>(atomicAdd(&st_cnt[wv][st_row[wv][e]], 1));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane < 32) {
            const int c = st_cnt[wv][lane];
            st_base[wv][lane] = c > 0 ? atomicAdd(list_n + q0 + lane, c) : 0;
        }
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        for (int e = lane; e < scnt; e += 64) {
            const int row = st_row[wv][e];
            const int32_t pos = st_base[wv][row] + st_rank[wv][e];
            if (pos < cap) {
                const int64_t q = q0 + row;
                list_key[q * cap + pos] = st_key[wv][e];
                list_idx[q * cap + pos] = st_idx[wv][e];
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        scnt = 0;
    };
    const int64_t nblk = (M + 31) / 32;
    float4 pre[PER];
    auto fetch = [&](int64_t cb) {
#pragma unroll
        for (int p = 0; p < PER; ++p) {
            const int t = threadIdx.x + p * kBlock;
            const int r = t / (D / 4), c4 = t % (D / 4);
            const int64_t j = cb * 32 + r;
            pre[p] = (t < NF4 && j < M) ? reinterpret_cast<const float4*>(Cn + j * stride * D)[c4]
                                        : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto land = [&](int buf) {
#pragma unroll
        for (int p = 0; p < PER; ++p) {
            const int t = threadIdx.x + p * kBlock;
            if (t < NF4) *reinterpret_cast<float4*>(&cs[buf][(t / (D / 4)) * ROWF + (t % (D / 4)) * 4]) = pre[p];
        }
    };
    int64_t cb = chunk;
    if (cb < nblk) {
        fetch(cb);
        land(0);
    }
    __syncthreads();
    int buf = 0;
    for (; cb < nblk; cb += nchunk) {
        const int64_t nxt = cb + nchunk;
        if (nxt < nblk) fetch(nxt);  // in flight during this block's MFMAs
        f32x16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.f;
        const float* brow = &cs[buf][i * ROWF + h * H];
        // B in groups of G float4 per LDS wait (G*4 MFMAs behind each wait)
        constexpr int G = (H / 4) >= 4 ? 4 : (H / 4);
#pragma unroll
        for (int v0 = 0; v0 < H / 4; v0 += G) {
            float4 bv[G];
#pragma unroll
            for (int g = 0; g < G; ++g) bv[g] = *reinterpret_cast<const float4*>(brow + 4 * (v0 + g));
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const int v = v0 + g;
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * v], bv[g].x, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * v + 1], bv[g].y, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * v + 2], bv[g].z, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * v + 3], bv[g].w, acc, 0, 0, 0);
            }
        }
        // epilogue: column = candidate j (this lane's), rows = queries; branch-free test, and
        // a wave-uniform branch only for the (rare) slots where some lane passes
        const int64_t j = cb * 32 + i;
        const int32_t jj = static_cast<int32_t>(j * stride);
        const bool jok = j < M;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row0 = (r & 3) + 8 * (r >> 2);
            const int row = row0 + 4 * h;
            const bool take = jok & !(acc[r] < th[r]);
            if (thr == nullptr) {  // dense mode: every subset score at its subset slot
                const uint32_t key = score_key(acc[r]);
                if (take) {
                    const int64_t q = q0 + row;
                    list_key[q * cap + j] = key;
                    list_idx[q * cap + j] = jj;
                }
                continue;
            }
            const unsigned long long m = __ballot(take);
            if (m == 0ull) continue;
            const int n = __popcll(m);
            if (scnt + n > kStage) flush();
            if (take) {
                const int sl = scnt + __popcll(m & below);
                st_key[wv][sl] = score_key(acc[r]);
                st_idx[wv][sl] = jj;
                st_row[wv][sl] = static_cast<uint8_t>(row);
            }
            scnt += n;
        }
        if (nxt < nblk) land(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }
    if (thr != nullptr) flush();
}

// k-th largest key per query list (radix select), then the threshold or the hit count.
constexpr int kSelBlock = 1024;

__global__ __launch_bounds__(kSelBlock) void k_select_topk(const uint32_t* __restrict__ list_key,
                                                           const int32_t* __restrict__ list_idx,
                                                           const int32_t* __restrict__ list_n, int32_t dense_n,
                                                           int32_t cap, int32_t k, int64_t P, int64_t Qvalid,
                                                           uint32_t* __restrict__ thr_out, int32_t* __restrict__ hits_out) {
    __shared__ uint32_t hist[256];
    __shared__ uint32_t s_prefix, s_mask, s_k;
    __shared__ int32_t red[kSelBlock / 64][2];
    const int64_t q = blockIdx.x;
    if (q >= Qvalid) {
        if (threadIdx.x == 0) {
            if (thr_out) thr_out[q] = 0xFFFFFFFFu;
            if (hits_out) hits_out[q] = 0;
        }
        return;
    }
    int32_t n = list_n ? list_n[q] : dense_n;
    if (n > cap) n = cap;
    const uint32_t* keys = list_key + q * cap;
    const int32_t* idx = list_idx + q * cap;
    if (n < k) {  // cannot rank k: threshold "everything", hits invalid
        if (threadIdx.x == 0) {
            if (thr_out) thr_out[q] = 0u;
            if (hits_out) hits_out[q] = -1;
        }
        return;
    }
    if (threadIdx.x == 0) {
        s_prefix = 0u;
        s_mask = 0u;
        s_k = static_cast<uint32_t>(k);
    }
    for (int shift = 24; shift >= 0; shift -= 8) {
        for (int t = threadIdx.x; t < 256; t += kSelBlock) hist[t] = 0u;
        __syncthreads();
        const uint32_t prefix = s_prefix, mask = s_mask;
        for (int e = threadIdx.x; e < n; e += kSelBlock) {
            const uint32_t key = keys[e];
            if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t cum = 0, kk = s_k;
            int bsel = 0;
            for (int bin = 255; bin >= 0; --bin) {
                if (cum + hist[bin] >= kk) {
                    bsel = bin;
                    break;
                }
                cum += hist[bin];
            }
            s_k = kk - cum;
            s_prefix = prefix | (static_cast<uint32_t>(bsel) << shift);
            s_mask = mask | (255u << shift);
        }
        __syncthreads();
    }
    const uint32_t T = s_prefix;
    const int32_t need = static_cast<int32_t>(s_k);  // taken from the keys equal to T
    if (thr_out && threadIdx.x == 0) thr_out[q] = T;
    if (!hits_out) return;
    int32_t above = 0, ties = 0;
    for (int e = threadIdx.x; e < n; e += kSelBlock) {
        const uint32_t key = keys[e];
        const bool pos = idx[e] < P;
        above += (key > T && pos) ? 1 : 0;
        ties += (key == T && pos) ? 1 : 0;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        above += __shfl_xor(above, off, 64);
        ties += __shfl_xor(ties, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        red[threadIdx.x >> 6][0] = above;
        red[threadIdx.x >> 6][1] = ties;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int32_t A = 0, Ti = 0;
        for (int w = 0; w < kSelBlock / 64; ++w) {
            A += red[w][0];
            Ti += red[w][1];
        }
        hits_out[q] = A + (Ti < need ? Ti : need);
    }
}

// ---------------------------------------------------------------------------------------------
// CPU torch.topk's tie rule (lgcn_select_topk_stl). On CPU, the reference's torch.topk(scores, k)
// (utils/train_test.py:197) runs ATen's topk_impl_loop (TopKImpl.h): the row as (value, index)
// pairs, then std::partial_sort(k) when k * 64 <= M, else std::nth_element(k - 1), both with the
// comparator (isnan(x) && !isnan(y)) || x > y — libstdc++ (GCC 11) instantiated inside libtorch.
// Which of several EQUAL scores make the top k is therefore whatever those two algorithms leave
// in the first k slots; with duplicated candidate rows (an item that is a positive of one edge and
// a sampled negative of another scores identically) that decides hits. The kernels below run the
// same libstdc++ algorithms, step for step, on the same (key, index) sequence (checked against
// torch.topk on tie-heavy rows in tests/test_recall_stl.py's host model of these steps).
// Keys compare as the floats do: -0 is mapped onto +0's key (equal as floats), NaN is highest.
namespace stl {

struct El {
    uint32_t k;
    int32_t i;
};

__device__ __forceinline__ uint32_t canon(uint32_t k) { return k == 0x7FFFFFFFu ? 0x80000000u : k; }
__device__ __forceinline__ bool comp(const El& x, const El& y) { return x.k > y.k; }

// (key, index) arrays in LDS or global memory (flat addresses)
struct Arr {
    uint32_t* k;
    int32_t* i;
    __device__ __forceinline__ El get(int64_t p) const { return El{k[p], i[p]}; }
    __device__ __forceinline__ void set(int64_t p, const El& e) const {
        k[p] = e.k;
        i[p] = e.i;
    }
    __device__ __forceinline__ void swap(int64_t a, int64_t b) const {
        const El x = get(a), y = get(b);
        set(a, y);
        set(b, x);
    }
};

// std::__adjust_heap + std::__push_heap
__device__ void adjust_heap(const Arr& a, int64_t first, int64_t hole, int64_t len, El value) {
    const int64_t top = hole;
    int64_t second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (comp(a.get(first + second), a.get(first + second - 1))) --second;
        a.set(first + hole, a.get(first + second));
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        a.set(first + hole, a.get(first + second - 1));
        hole = second - 1;
    }
    int64_t parent = (hole - 1) / 2;
    while (hole > top && comp(a.get(first + parent), value)) {
        a.set(first + hole, a.get(first + parent));
        hole = parent;
        parent = (hole - 1) / 2;
    }
    a.set(first + hole, value);
}

// std::__make_heap
__device__ void make_heap(const Arr& a, int64_t first, int64_t last) {
    const int64_t len = last - first;
    if (len < 2) return;
    for (int64_t parent = (len - 2) / 2;; --parent) {
        adjust_heap(a, first, parent, len, a.get(first + parent));
        if (parent == 0) return;
    }
}

// std::__heap_select: the heap of [first, middle) keeps the best; an element replaces the heap's
// top (its worst) only if strictly better (std::__pop_heap into the element's slot)
__device__ void heap_select(const Arr& a, int64_t first, int64_t middle, int64_t last) {
    make_heap(a, first, middle);
    for (int64_t i = middle; i < last; ++i) {
        if (comp(a.get(i), a.get(first))) {
            const El v = a.get(i);
            a.set(i, a.get(first));
            adjust_heap(a, first, 0, middle - first, v);
        }
    }
}

// std::__move_median_to_first
__device__ void move_median_to_first(const Arr& a, int64_t r, int64_t x, int64_t y, int64_t z) {
    const El A = a.get(x), B = a.get(y), C = a.get(z);
    if (comp(A, B)) {
        if (comp(B, C)) a.swap(r, y);
        else if (comp(A, C)) a.swap(r, z);
        else a.swap(r, x);
    } else if (comp(A, C)) {
        a.swap(r, x);
    } else if (comp(B, C)) {
        a.swap(r, z);
    } else {
        a.swap(r, y);
    }
}

// std::__unguarded_partition around the pivot at `pivot`
__device__ int64_t unguarded_partition(const Arr& a, int64_t first, int64_t last, int64_t pivot) {
    const El pv = a.get(pivot);  // the pivot slot is outside [first, last): never swapped here
    while (true) {
        while (comp(a.get(first), pv)) ++first;
        --last;
        while (comp(pv, a.get(last))) --last;
        if (!(first < last)) return first;
        a.swap(first, last);
        ++first;
    }
}

// std::__insertion_sort (with __unguarded_linear_insert)
__device__ void insertion_sort(const Arr& a, int64_t first, int64_t last) {
    if (first == last) return;
    for (int64_t i = first + 1; i != last; ++i) {
        const El v = a.get(i);
        if (comp(v, a.get(first))) {
            for (int64_t j = i; j > first; --j) a.set(j, a.get(j - 1));  // std::move_backward
            a.set(first, v);
        } else {
            int64_t j = i, nx = i - 1;
            while (comp(v, a.get(nx))) {
                a.set(j, a.get(nx));
                j = nx;
                --nx;
            }
            a.set(j, v);
        }
    }
}

__device__ __forceinline__ int64_t lg(int64_t n) { return 63 - __clzll(static_cast<unsigned long long>(n)); }

// std::nth_element -> std::__introselect(first, nth, last, 2 * __lg(last - first))
__device__ void nth_element(const Arr& a, int64_t first, int64_t nth, int64_t last) {
    if (first == last || nth == last) return;
    int64_t depth = 2 * lg(last - first);
    while (last - first > 3) {
        if (depth == 0) {
            heap_select(a, first, nth + 1, last);
            a.swap(first, nth);  // the nth element to its final place
            return;
        }
        --depth;
        const int64_t mid = first + (last - first) / 2;
        move_median_to_first(a, first, first + 1, mid, last - 1);
        const int64_t cut = unguarded_partition(a, first + 1, last, first);
        if (cut <= nth) first = cut;
        else last = cut;
    }
    insertion_sort(a, first, last);
}

}  // namespace stl

constexpr int kStlHeapMax = 4096;  // k of the partial_sort path (k * 64 <= M): 32 KB of LDS

// partial_sort path: one wave per query streams its dense key row in index order; an element is
// compared with the heap's top in parallel (64 per step), and the few that beat it are inserted in
// index order by lane 0 (std::__heap_select's loop, with the heap in LDS).
__global__ __launch_bounds__(64) void k_select_stl_heap(const uint32_t* __restrict__ list_key, int64_t cap, int64_t M,
                                                        int32_t k, int64_t P, int64_t Qvalid,
                                                        int32_t* __restrict__ hits_out) {
    __shared__ uint32_t hk[kStlHeapMax];
    __shared__ int32_t hi[kStlHeapMax];
    const int64_t q = blockIdx.x;
    const int lane = threadIdx.x;
    if (q >= Qvalid) {
        if (lane == 0) hits_out[q] = 0;
        return;
    }
    const uint32_t* row = list_key + q * cap;
    for (int t = lane; t < k; t += 64) {
        hk[t] = stl::canon(row[t]);
        hi[t] = t;
    }
    __syncthreads();
    const stl::Arr heap{hk, hi};
    if (lane == 0) stl::make_heap(heap, 0, k);
    __syncthreads();
    constexpr int U = 8;  // 64-key steps loaded together
    for (int64_t base = k; base < M; base += 64 * U) {
        uint32_t v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = base + u * 64 + lane;
            v[u] = j < M ? stl::canon(row[j]) : 0u;  // key 0 is below every score's key
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            unsigned long long m = __ballot(v[u] > hk[0]);
            while (m) {
                const int l = __ffsll(static_cast<long long>(m)) - 1;
                m &= m - 1ull;
                const uint32_t vl = __shfl(v[u], l, 64);
                if (lane == 0 && vl > hk[0])
                    stl::adjust_heap(heap, 0, 0, k, stl::El{vl, static_cast<int32_t>(base + u * 64 + l)});
            }
            __syncthreads();  // lane 0's heap writes before the next top read
        }
    }
    int32_t h = 0;
    for (int t = lane; t < k; t += 64) h += hi[t] < P ? 1 : 0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) h += __shfl_xor(h, off, 64);
    if (lane == 0) hits_out[q] = h;
}

// nth_element path (k * 64 > M, so M < 64 k): lane 0 runs std::nth_element in place on the
// query's dense (key, index) row in global memory; the top k are then its first k slots.
__global__ __launch_bounds__(64) void k_select_stl_nth(uint32_t* __restrict__ list_key, int32_t* __restrict__ list_idx,
                                                       int64_t cap, int64_t M, int32_t k, int64_t P, int64_t Qvalid,
                                                       int32_t* __restrict__ hits_out) {
    const int64_t q = blockIdx.x;
    const int lane = threadIdx.x;
    if (q >= Qvalid) {
        if (lane == 0) hits_out[q] = 0;
        return;
    }
    uint32_t* kr = list_key + q * cap;
    int32_t* ir = list_idx + q * cap;
    for (int64_t t = lane; t < M; t += 64) {
        kr[t] = stl::canon(kr[t]);
        ir[t] = static_cast<int32_t>(t);
    }
    __syncthreads();
    if (lane == 0) stl::nth_element(stl::Arr{kr, ir}, 0, k - 1, M);
    __syncthreads();
    int32_t h = 0;
    for (int t = lane; t < k; t += 64) h += ir[t] < P ? 1 : 0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) h += __shfl_xor(h, off, 64);
    if (lane == 0) hits_out[q] = h;
}

template <int D>
int launch_filter(const float* Qn, int64_t Qpad, int64_t Qvalid, const float* Cn, int64_t M, int64_t stride,
                  const uint32_t* thr, uint32_t* lk, int32_t* li, int32_t* ln, int32_t cap, hipStream_t s) {
    constexpr int QW = 4 * 32;  // queries per workgroup
    if (Qpad % QW != 0) return fail(LGCN_E_ARG, "lgcn_score_filter: padded query count %lld not a multiple of %d",
                                    (long long)Qpad, QW);
    const int64_t nblk = (M + 31) / 32;
    const int64_t nqg = Qpad / QW;
    // candidate chunks: a multiple of 8 (the XCD mapping), ~2048 workgroups in all
    int64_t nchunk = (2048 / nqg + 7) / 8 * 8;
    const int64_t need = (nblk + 7) / 8 * 8;
    if (nchunk > need) nchunk = need;
    if (nchunk < 8) nchunk = 8;
    const int64_t grid = nqg * nchunk;
    if (grid > INT32_MAX || nqg > INT32_MAX) return fail(LGCN_E_ARG, "lgcn_score_filter: too many queries");
    k_score_filter<D><<<dim3(static_cast<unsigned>(grid)), kBlock, 0, s>>>(
        Qn, Qvalid, static_cast<int32_t>(nqg), static_cast<int32_t>(nchunk), Cn, M, stride, thr, lk, li, ln, cap);
    return check_launch("k_score_filter");
}

}  // namespace

extern "C" {

int lgcn_recall_width(int32_t d, int32_t* D_out, int32_t* qpad_multiple) {
    if (d <= 0 || d > 256 || !D_out) return fail(LGCN_E_UNSUPPORTED, "lgcn_recall_width: d=%d (max 256)", d);
    int D = 8;
    while (D < d) D <<= 1;
    *D_out = D;
    if (qpad_multiple) *qpad_multiple = 128;
    return LGCN_OK;
}

int lgcn_normalize_rows(const float* x, const int64_t* idx, int64_t rows, int64_t ld, int32_t d, float* out,
                        int32_t D, int64_t out_rows, lgcn_stream_t stream) {
    if (rows < 0 || out_rows < rows || d <= 0 || D < d || ld < d || (out_rows > 0 && !out) || (rows > 0 && !x))
        return fail(LGCN_E_ARG, "lgcn_normalize_rows: bad args");
    if (out_rows == 0) return LGCN_OK;
    const int64_t threads = out_rows * 32;
    k_normalize_rows<<<grid_for(threads, kBlock, int64_t(1) << 31), kBlock, 0, as_stream(stream)>>>(x, idx, rows, ld, d,
                                                                                                   out, D, out_rows);
    return check_launch("k_normalize_rows");
}

int lgcn_score_filter(const float* Qn, int64_t Qpad, int64_t Qvalid, const float* Cn, int64_t M, int64_t stride,
                      int32_t D, const uint32_t* thr, uint32_t* list_key, int32_t* list_idx, int32_t* list_n,
                      int32_t cap, lgcn_stream_t stream) {
    if (!Qn || Qpad <= 0 || Qvalid > Qpad || M < 0 || stride <= 0 || !list_key || !list_idx || cap <= 0 ||
        (thr && !list_n) || (M > 0 && !Cn) || (M - 1) * stride >= (int64_t(1) << 31))
        return fail(LGCN_E_ARG, "lgcn_score_filter: bad args");
    if (!thr && M > cap) return fail(LGCN_E_ARG, "lgcn_score_filter: dense mode needs M <= cap");
    if (M == 0) return LGCN_OK;
    hipStream_t s = as_stream(stream);
    switch (D) {
        case 8: return launch_filter<8>(Qn, Qpad, Qvalid, Cn, M, stride, thr, list_key, list_idx, list_n, cap, s);
        case 16: return launch_filter<16>(Qn, Qpad, Qvalid, Cn, M, stride, thr, list_key, list_idx, list_n, cap, s);
        case 32: return launch_filter<32>(Qn, Qpad, Qvalid, Cn, M, stride, thr, list_key, list_idx, list_n, cap, s);
        case 64: return launch_filter<64>(Qn, Qpad, Qvalid, Cn, M, stride, thr, list_key, list_idx, list_n, cap, s);
        case 128: return launch_filter<128>(Qn, Qpad, Qvalid, Cn, M, stride, thr, list_key, list_idx, list_n, cap, s);
        case 256: return launch_filter<256>(Qn, Qpad, Qvalid, Cn, M, stride, thr, list_key, list_idx, list_n, cap, s);
        default: return fail(LGCN_E_UNSUPPORTED, "lgcn_score_filter: D=%d (use lgcn_recall_width)", D);
    }
}

int lgcn_select_topk(const uint32_t* list_key, const int32_t* list_idx, const int32_t* list_n, int32_t dense_n,
                     int32_t cap, int32_t k, int64_t P, int64_t Qpad, int64_t Qvalid, uint32_t* thr_out,
                     int32_t* hits_out, lgcn_stream_t stream) {
    if (!list_key || !list_idx || cap <= 0 || k <= 0 || Qpad <= 0 || Qvalid > Qpad || (!thr_out && !hits_out) ||
        (!list_n && dense_n < 0))
        return fail(LGCN_E_ARG, "lgcn_select_topk: bad args");
    k_select_topk<<<dim3(static_cast<unsigned>(Qpad)), kSelBlock, 0, as_stream(stream)>>>(
        list_key, list_idx, list_n, dense_n, cap, k, P, Qvalid, thr_out, hits_out);
    return check_launch("k_select_topk");
}

int lgcn_select_topk_stl(uint32_t* list_key, int32_t* list_idx, int64_t cap, int64_t M, int32_t k, int64_t P,
                         int64_t Qpad, int64_t Qvalid, int32_t* hits_out, lgcn_stream_t stream) {
    if (!list_key || !list_idx || !hits_out || k <= 0 || M < k || cap < M || Qpad <= 0 || Qvalid > Qpad ||
        Qpad > INT32_MAX || M > INT32_MAX)
        return fail(LGCN_E_ARG, "lgcn_select_topk_stl: bad args");
    const bool heap = static_cast<int64_t>(k) * 64 <= M;  // ATen topk_impl_loop's use_partial_sort
    if (heap) {
        if (k > kStlHeapMax)
            return fail(LGCN_E_UNSUPPORTED, "lgcn_select_topk_stl: k=%d > %d on the partial_sort path", k, kStlHeapMax);
        k_select_stl_heap<<<dim3(static_cast<unsigned>(Qpad)), 64, 0, as_stream(stream)>>>(list_key, cap, M, k, P,
                                                                                           Qvalid, hits_out);
        return check_launch("k_select_stl_heap");
    }
    k_select_stl_nth<<<dim3(static_cast<unsigned>(Qpad)), 64, 0, as_stream(stream)>>>(list_key, list_idx, cap, M, k, P,
                                                                                      Qvalid, hits_out);
    return check_launch("k_select_stl_nth");
}

}  // extern "C"
