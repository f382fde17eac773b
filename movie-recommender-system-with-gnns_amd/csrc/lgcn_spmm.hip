// LightGCN propagation kernels for gfx950 (MI355X).
//
// One launch = one LGConv layer y = Â x over a plan's CSR (rows = destinations), fused with
// the LightGCN layer-stack epilogue (reference models/light_gcn.py:29-36; Â is PyG 2.4.0's
// gcn_norm-weighted adjacency, applied by LGConv.forward at :33).
//
// Mapping (d = 64 fp32, the headline config): a 256-thread workgroup = 4 waves = 16 groups of
// 16 lanes; one group owns one schedule item (a whole row, or a <= chunk-edge piece of a long
// row); each lane owns one float4 column slice, so one wave-instruction gathers 4 neighbour
// rows (1 KiB) with global_load_dwordx4. Items are ordered longest-first, so the 4 groups of a
// wave carry (nearly) equal work. Neighbour ids/weights are loaded once per 16-edge batch
// (prefetched one batch ahead), coalesced, and broadcast inside the group by cross-lane permute;
// UNROLL gathers are issued before the first add, so every wave keeps several KiB in flight.
// Measured alternatives that did not pay on C2 (tools/variants.py, profiles/r01c_final/):
// XCD-aware column split (each XCD one 128-B or 64-B slice of every row: +5% / +100% time),
// 16-deep unroll, non-temporal col/val loads (within 1%).
//
// Numerics: per row, v = (((0 + w0*x0) + w1*x1) + ...) in CSR order, mul then add (no FMA:
// this file is built with -ffp-contract=off), i.e. the order and rounding of PyG's CPU
// scatter_add_. Unsplit rows are therefore bit-identical to the reference CPU path; split rows
// add chunk partials in chunk order (deterministic, within 1e-6 relative).
// No atomics anywhere: every output row is written by exactly one group.

#include <cstdlib>

#include "lgcn_common.h"

using namespace lgcn;

namespace {

struct SpmmArgs {
    const lgcn_item_t* items;
    int64_t n_items;
    const lgcn_split_t* splits;
    int64_t n_splits;
    const int32_t* col;
    const float* val;
    const float* x_lo;
    const float* x_hi;
    int64_t x_split;
    const float* e_lo;
    const float* e_hi;
    int64_t e_split;
    float* y;
    float* acc_lo;
    float* acc_hi;
    int64_t acc_split;
    float* partial;
    int32_t d;
    int32_t mode;
    float div;
    float mul;
    float* run;  // sliced launches: running row sums between a row's source-slice segments
    const lgcn_item_t* chunks;  // block-split launches: split rows' chunk items, partial-slot order
    int32_t nt = 0;  // bit 0: non-temporal row stores, bit 1: non-temporal row loads (LGCN_SPMM_NT overrides)
    // combine launches: split rows [0, n_big) get a workgroup each; rows [n_big, n_splits) have at
    // most kVSums chunks and are combined one per lane group (lgcn_spmm_pair's n_split_big)
    int64_t n_big = -1;  // -1: every split row gets a workgroup
};

typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_row(float4* p, float4 v, int nt) {
    if (nt & 1) {
        f4v w = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(w, reinterpret_cast<f4v*>(p));
    } else {
        *p = v;
    }
}
__device__ __forceinline__ float4 ld_row(const float4* p, int nt) {
    if (nt & 2) {
        const f4v w = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
        return make_float4(w.x, w.y, w.z, w.w);
    }
    return *p;
}

// Sliced-schedule item flags, in the high bits of lgcn_item_t::len (rows, not partial chunks).
constexpr int32_t kItemFirst = 0x20000000;
constexpr int32_t kItemLast = 0x40000000;
constexpr int32_t kItemLenMask = 0x1FFFFFFF;

template <class T>
__device__ __forceinline__ T* split_row(T* lo, T* hi, int64_t split, int64_t r, int64_t stride) {
    return (r < split) ? lo + r * stride : hi + (r - split) * stride;
}

__device__ __forceinline__ float4 f4_add(float4 a, float4 b) {
    return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float4 f4_axpy(float4 acc, float w, float4 x) {
    // acc + (w * x): two roundings, never contracted (-ffp-contract=off)
    return make_float4(acc.x + w * x.x, acc.y + w * x.y, acc.z + w * x.z, acc.w + w * x.w);
}
__device__ __forceinline__ float4 f4_divmul(float4 a, float div, float mul) {
    return make_float4((a.x / div) * mul, (a.y / div) * mul, (a.z / div) * mul, (a.w / div) * mul);
}

// Epilogue for one finished row r; lane l owns float4 slots l, l+LPR, ... (NV of them).
template <int LPR, int NV>
__device__ __forceinline__ void finish_row_vec(const SpmmArgs& a, int64_t r, int l0, const float4 (&v)[NV]) {
    // lane slots are l0 + k*LPR (l0 = column-slice base + lane)
    const int l = l0;
    const int64_t d4 = a.d / 4;
    float4* acc = reinterpret_cast<float4*>(split_row(a.acc_lo, a.acc_hi, a.acc_split, r, a.d));
    if (a.mode == LGCN_EPI_INIT || a.mode == LGCN_EPI_FINAL_E) {
        const float4* e = reinterpret_cast<const float4*>(split_row(a.e_lo, a.e_hi, a.e_split, r, a.d));
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const float4 s = f4_add(ld_row(e + l + k * LPR, a.nt), v[k]);
            st_row(acc + l + k * LPR, (a.mode == LGCN_EPI_INIT) ? s : f4_divmul(s, a.div, a.mul), a.nt);
        }
    } else if (a.mode == LGCN_EPI_STORE) {
#pragma unroll
        for (int k = 0; k < NV; ++k) st_row(acc + l + k * LPR, v[k], a.nt);
    } else if (a.mode == LGCN_EPI_SCALE) {
#pragma unroll
        for (int k = 0; k < NV; ++k)
            acc[l + k * LPR] = make_float4((v[k].x * a.mul) / a.div, (v[k].y * a.mul) / a.div,
                                           (v[k].z * a.mul) / a.div, (v[k].w * a.mul) / a.div);
    } else {
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const float4 s = f4_add(ld_row(acc + l + k * LPR, a.nt), v[k]);
            st_row(acc + l + k * LPR, (a.mode == LGCN_EPI_ADD) ? s : f4_divmul(s, a.div, a.mul), a.nt);
        }
    }
    if (a.y != nullptr && (a.mode == LGCN_EPI_INIT || a.mode == LGCN_EPI_ADD)) {
        float4* y = reinterpret_cast<float4*>(a.y) + r * d4;
#pragma unroll
        for (int k = 0; k < NV; ++k) st_row(y + l + k * LPR, v[k], a.nt);
    }
}

// One batch of n <= LPR edges of an item, added to acc in CSR order: lane j of the group holds
// edge j's (col, val), broadcast with __shfl; UNROLL neighbour rows are gathered (one float4 per
// lane each) before the first add.
template <int LPR, int NV, int UNROLL, int TAIL>
__device__ __forceinline__ void sum_batch(const float4* __restrict__ xlo, const float4* __restrict__ xhi,
                                          int64_t x_split, int c, float w, int n, float4 (&acc)[NV]) {
    const int64_t d4 = int64_t(LPR) * NV;
    int j = 0;
    for (; j + UNROLL <= n; j += UNROLL) {
        float4 xv[UNROLL][NV];
        float wv[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const int cj = __shfl(c, j + u, LPR);
            wv[u] = __shfl(w, j + u, LPR);
            const float4* src = (cj < x_split) ? xlo + int64_t(cj) * d4 : xhi + (int64_t(cj) - x_split) * d4;
#pragma unroll
            for (int k = 0; k < NV; ++k) xv[u][k] = src[k * LPR];
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
#pragma unroll
            for (int k = 0; k < NV; ++k) acc[k] = f4_axpy(acc[k], wv[u], xv[u][k]);
    }
    if (TAIL == 1 && j < n) {
        // the batch's last n - j (< UNROLL) edges: all their gathers issued (exec-predicated)
        // before the first add, then added in CSR order — one memory latency instead of n - j
        const int rem = n - j;
        float4 xv[UNROLL - 1][NV];
        float wv[UNROLL - 1];
#pragma unroll
        for (int u = 0; u < UNROLL - 1; ++u) {
            const int ju = j + (u < rem ? u : 0);
            const int cj = __shfl(c, ju, LPR);
            wv[u] = __shfl(w, ju, LPR);
            const float4* src = (cj < x_split) ? xlo + int64_t(cj) * d4 : xhi + (int64_t(cj) - x_split) * d4;
            if (u < rem) {
#pragma unroll
                for (int k = 0; k < NV; ++k) xv[u][k] = src[k * LPR];
            }
        }
#pragma unroll
        for (int u = 0; u < UNROLL - 1; ++u)
            if (u < rem) {
#pragma unroll
                for (int k = 0; k < NV; ++k) acc[k] = f4_axpy(acc[k], wv[u], xv[u][k]);
            }
        j = n;
    }
    for (; j < n; ++j) {
        const int cj = __shfl(c, j, LPR);
        const float wj = __shfl(w, j, LPR);
        const float4* src = (cj < x_split) ? xlo + int64_t(cj) * d4 : xhi + (int64_t(cj) - x_split) * d4;
#pragma unroll
        for (int k = 0; k < NV; ++k) acc[k] = f4_axpy(acc[k], wj, src[k * LPR]);
    }
}

// Rows narrower than UNROLL lanes (LPR < UNROLL, d <= 16): one load round of SB = LPR * CM edges,
// UNROLL edges at a time across UNROLL / LPR batches (edge e of the round: lane e % LPR of batch
// slot e / LPR, both static), each group's gathers issued (exec-predicated on e < n) before its
// adds, which run in CSR order — UNROLL rows in flight per lane group instead of LPR.
template <int LPR, int NV, int UNROLL, int CM>
__device__ __forceinline__ void sum_round_narrow(const float4* __restrict__ xlo, const float4* __restrict__ xhi,
                                                 int64_t x_split, const int (&c)[CM], const float (&w)[CM], int n,
                                                 float4 (&acc)[NV]) {
    constexpr int SB = LPR * CM;
    constexpr int UG = UNROLL < SB ? UNROLL : SB;
    static_assert(SB % UG == 0, "load round must be a whole number of gather groups");
    const int64_t d4 = int64_t(LPR) * NV;
#pragma unroll
    for (int j = 0; j < SB; j += UG) {
        if (j >= n) break;
        float4 xv[UG][NV];
        float wv[UG];
#pragma unroll
        for (int u = 0; u < UG; ++u) {
            const int e = j + u;
            const int cj = __shfl(c[e / LPR], e % LPR, LPR);
            wv[u] = __shfl(w[e / LPR], e % LPR, LPR);
            if (e < n) {
                const float4* src = (cj < x_split) ? xlo + int64_t(cj) * d4 : xhi + (int64_t(cj) - x_split) * d4;
#pragma unroll
                for (int k = 0; k < NV; ++k) xv[u][k] = src[k * LPR];
            }
        }
#pragma unroll
        for (int u = 0; u < UG; ++u)
            if (j + u < n) {
#pragma unroll
                for (int k = 0; k < NV; ++k) acc[k] = f4_axpy(acc[k], wv[u], xv[u][k]);
            }
    }
}

// Sum of one item's edges into acc, in CSR order. The lanes load (col, val) coalesced, CM batches
// of LPR edges per load round (CM > 1 at narrow rows: one 128-B line of col per round instead of a
// fraction of one, which the gathers would evict from L1 before the next batch reads it) — the
// NEXT round's pairs are loaded before the current round's gathers are issued, so that latency
// overlaps them — then each batch goes through sum_batch in order.
template <int LPR, int NV, int UNROLL, int TAIL, int CM = 1>
__device__ __forceinline__ void sum_item(const SpmmArgs& a, const lgcn_item_t it, int l, float4 (&acc)[NV]) {
    const float4* __restrict__ xlo = reinterpret_cast<const float4*>(a.x_lo) + l;
    const float4* __restrict__ xhi = reinterpret_cast<const float4*>(a.x_hi) + l;
    constexpr int SB = LPR * CM;  // edges per load round
    int cn[CM];
    float wn[CM];
#pragma unroll
    for (int m = 0; m < CM; ++m) {
        cn[m] = 0;
        wn[m] = 0.f;
        if (m * LPR + l < it.len) {
            cn[m] = *(a.col + it.beg + m * LPR + l);
            wn[m] = *(a.val + it.beg + m * LPR + l);
        }
    }
    for (int b = 0; b < it.len; b += SB) {
        int c[CM];
        float w[CM];
#pragma unroll
        for (int m = 0; m < CM; ++m) {
            c[m] = cn[m];
            w[m] = wn[m];
        }
        if (b + SB < it.len) {  // prefetch the next round
#pragma unroll
            for (int m = 0; m < CM; ++m)
                if (b + SB + m * LPR + l < it.len) {
                    cn[m] = *(a.col + it.beg + b + SB + m * LPR + l);
                    wn[m] = *(a.val + it.beg + b + SB + m * LPR + l);
                }
        }
        if constexpr (LPR < UNROLL) {
            sum_round_narrow<LPR, NV, UNROLL, CM>(xlo, xhi, a.x_split, c, w, min(SB, it.len - b), acc);
        } else {
#pragma unroll
            for (int m = 0; m < CM; ++m)
                if (b + m * LPR < it.len)
                    sum_batch<LPR, NV, UNROLL, TAIL>(xlo, xhi, a.x_split, c[m], w[m], min(LPR, it.len - b - m * LPR),
                                                     acc);
        }
    }
}

// Split rows (chunked hubs) are summed with ONE association at every width: partial/chunk c goes
// to running sum v = c % kVSums (in c order), then the kVSums sums are added in v order. Lane
// group g of a workgroup owns sums g, g + GPB, ... (GPB = groups per block: 64 at d=16, 16 at
// d=64, 4 at d >= 256), so a row's result does not depend on d — a column share of a row (the
// column-split sharded forward, lgcn_amd.sharded) is bitwise that share of the full-width row.
constexpr int kVSums = 16;

// Block-split launches (lgcn_spmm_blocksplit): workgroup s < n_splits sums split row s whole:
// each chunk (from 0, in CSR order — the partial the item pass would have written) into its
// running sum, then the sums in order through LDS: the association of item pass + k_combine_vec,
// so bitwise the same result, without the partials' round trip or the second launch.
template <int LPR, int NV, int UNROLL, int TAIL, int CM>
__device__ __forceinline__ void split_row_block(const SpmmArgs& a, int64_t s, int g, int l) {
    constexpr int GPB = kBlock / LPR;
    constexpr int VPG = (kVSums + GPB - 1) / GPB;
    __shared__ float4 lds[kVSums][LPR * NV];
    const lgcn_split_t sp = a.splits[s];
#pragma unroll
    for (int j = 0; j < VPG; ++j) {
        const int v = g + j * GPB;
        if (v >= kVSums) break;
        float4 acc[NV];
#pragma unroll
        for (int k = 0; k < NV; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int c = v; c < sp.pcnt; c += kVSums) {
            float4 part[NV];
#pragma unroll
            for (int k = 0; k < NV; ++k) part[k] = make_float4(0.f, 0.f, 0.f, 0.f);
            sum_item<LPR, NV, UNROLL, TAIL, CM>(a, a.chunks[int64_t(sp.pbeg) + c], l, part);
#pragma unroll
            for (int k = 0; k < NV; ++k) acc[k] = f4_add(acc[k], part[k]);
        }
#pragma unroll
        for (int k = 0; k < NV; ++k) lds[v][l + k * LPR] = acc[k];
    }
    __syncthreads();
    if (g != 0) return;
    float4 acc[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] = lds[0][l + k * LPR];
    const int nv = sp.pcnt < kVSums ? sp.pcnt : kVSums;
    for (int h = 1; h < nv; ++h)
#pragma unroll
        for (int k = 0; k < NV; ++k) acc[k] = f4_add(acc[k], lds[h][l + k * LPR]);
    finish_row_vec<LPR, NV>(a, sp.row, l, acc);
}

// The item pass. Group g of the block owns item blockIdx*GPB + g (summed by sum_item).
// SLICED: one launch of a source-sliced schedule (lgcn_spmm_run). A row item continues the row's
// running sum from a.run unless it is the row's FIRST segment, and runs the epilogue only on its
// LAST one; the sum stays one sequential chain in CSR order across launches.
// BSPLIT: workgroups [0, n_splits) sum the split rows (split_row_block), the rest the items.
// blk: the workgroup's index within this pass (blockIdx.x, or its share of a paired launch).
template <int LPR, int NV, int UNROLL, bool SLICED, int TAIL, bool BSPLIT, int CM>
__device__ __forceinline__ void item_pass(const SpmmArgs& a, int64_t blk) {
    constexpr int GPB = kBlock / LPR;
    const int g = threadIdx.x / LPR;
    const int l = threadIdx.x % LPR;
    if (BSPLIT && blk < a.n_splits) {
        split_row_block<LPR, NV, UNROLL, TAIL, CM>(a, blk, g, l);
        return;
    }
    const int64_t item = (blk - (BSPLIT ? a.n_splits : 0)) * GPB + g;
    if (item >= a.n_items) return;
    lgcn_item_t it = a.items[item];
    int32_t flags = kItemFirst | kItemLast;
    if (SLICED && it.dst >= 0) {
        flags = it.len & (kItemFirst | kItemLast);
        it.len &= kItemLenMask;
    }
    const int64_t d4 = int64_t(LPR) * NV;
    float4 acc[NV];
    if (SLICED && !(flags & kItemFirst)) {
        const float4* r = reinterpret_cast<const float4*>(a.run) + int64_t(it.dst) * d4 + l;
#pragma unroll
        for (int k = 0; k < NV; ++k) acc[k] = ld_row(r + k * LPR, a.nt);
    } else {
#pragma unroll
        for (int k = 0; k < NV; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    sum_item<LPR, NV, UNROLL, TAIL, CM>(a, it, l, acc);
    if (it.dst < 0) {
        float4* p = reinterpret_cast<float4*>(a.partial) + int64_t(-it.dst - 1) * d4 + l;
#pragma unroll
        for (int k = 0; k < NV; ++k) p[k * LPR] = acc[k];
        return;
    }
    if (SLICED && !(flags & kItemLast)) {
        float4* r = reinterpret_cast<float4*>(a.run) + int64_t(it.dst) * d4 + l;
#pragma unroll
        for (int k = 0; k < NV; ++k) st_row(r + k * LPR, acc[k], a.nt);
        return;
    }
    finish_row_vec<LPR, NV>(a, it.dst, l, acc);
}

template <int LPR, int NV, int UNROLL, bool SLICED = false, int TAIL = 0, bool BSPLIT = false, int CM = 1>
__global__ __launch_bounds__(kBlock) void k_spmm_vec(SpmmArgs a) {
    item_pass<LPR, NV, UNROLL, SLICED, TAIL, BSPLIT, CM>(a, blockIdx.x);
}

// Two independent plain item passes of one width in one launch (lgcn_spmm_pair): workgroups
// [0, blocks_a) run pass a, the rest pass b. Each pass keeps its own longest-first order, and b's
// longest items start while a's last workgroups drain, so the pair pays one launch gap and one
// drain instead of two. Per row the arithmetic is the single pass's (bitwise).
// xcd_a (1..7, default 4): workgroups are dealt to the 8 XCDs round-robin (workgroup i on XCD
// i % 8), so while both passes have blocks left, pass a takes the slots of XCDs [0, xcd_a) and
// pass b those of XCDs [xcd_a, 8) — each XCD's L2 then caches one pass's gather table instead of
// both — and the longer pass's remaining blocks follow on every XCD. xcd_a = 0: a's blocks, then
// b's, on every XCD.
template <int LPR, int NV, int UNROLL, int TAIL, int CM>
__global__ __launch_bounds__(kBlock) void k_spmm_pair(SpmmArgs a, SpmmArgs b, int64_t blocks_a, int64_t blocks_b,
                                                      int xcd_a) {
    const int64_t blk = blockIdx.x;
    if (xcd_a > 0) {
        const int64_t sa = xcd_a, sb = 8 - xcd_a;
        const int64_t ra = blocks_a / sa, rb = blocks_b / sb;
        const int64_t rounds = ra < rb ? ra : rb;  // rounds of 8 with both passes present
        if (blk < 8 * rounds) {
            const int64_t k = blk >> 3, x = blk & 7;
            if (x < sa)
                item_pass<LPR, NV, UNROLL, false, TAIL, false, CM>(a, k * sa + x);
            else
                item_pass<LPR, NV, UNROLL, false, TAIL, false, CM>(b, k * sb + x - sa);
            return;
        }
        const int64_t r = blk - 8 * rounds, left_a = blocks_a - rounds * sa;  // the rest, a's first
        if (r < left_a)
            item_pass<LPR, NV, UNROLL, false, TAIL, false, CM>(a, rounds * sa + r);
        else
            item_pass<LPR, NV, UNROLL, false, TAIL, false, CM>(b, rounds * sb + r - left_a);
        return;
    }
    if (blk < blocks_a)
        item_pass<LPR, NV, UNROLL, false, TAIL, false, CM>(a, blk);
    else
        item_pass<LPR, NV, UNROLL, false, TAIL, false, CM>(b, blk - blocks_a);
}

// lgcn_spmm_pair's XCDs for pass a: 4 by default (reduce-mode 4 x 2 rank step, K=3, C2: 0.193 ->
// 0.176 ms against a's blocks then b's; 8 x 1 0.182 vs 0.184, profiles/r04a_pair/);
// lgcn_tuning_t.pair_xcds_a = 0 (sequential) or 1..7 overrides.
int pair_xcd_a() { return tuning().pair_xcds_a; }

// Split rows: one workgroup per split row. Running sum v (of kVSums, owned by lane group v % GPB)
// adds partials v, v + kVSums, ... in that order; the kVSums sums are then added in v order through
// LDS. The association is fixed by the code and the same at every width, so results are
// deterministic run to run and a column share is bitwise the full row's share.
// The partials of a sum are loaded kCombineBatch at a time, all issued (predicated past pcnt) before
// the first add, so a sum of n partials waits ceil(n / kCombineBatch) memory round trips instead of
// one per partial — the combine launch is a chain of dependent loads, not a bandwidth problem.
constexpr int kCombineBatch = 8;

template <int LPR, int NV>
__device__ __forceinline__ void combine_row(const SpmmArgs& a, int64_t s) {
    constexpr int GPB = kBlock / LPR;
    constexpr int VPG = (kVSums + GPB - 1) / GPB;
    __shared__ float4 lds[kVSums][LPR * NV];
    const int g = threadIdx.x / LPR;
    const int l = threadIdx.x % LPR;
    if (s >= a.n_splits) return;  // whole block
    const lgcn_split_t sp = a.splits[s];
    const int64_t d4 = int64_t(LPR) * NV;
    const float4* p = reinterpret_cast<const float4*>(a.partial) + int64_t(sp.pbeg) * d4;
#pragma unroll
    for (int j = 0; j < VPG; ++j) {
        const int v = g + j * GPB;
        if (v >= kVSums) break;
        float4 acc[NV];
#pragma unroll
        for (int k = 0; k < NV; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int c = v; c < sp.pcnt; c += kCombineBatch * kVSums) {
            float4 t[kCombineBatch][NV];
#pragma unroll
            for (int u = 0; u < kCombineBatch; ++u)
                if (c + u * kVSums < sp.pcnt)
#pragma unroll
                    for (int k = 0; k < NV; ++k) t[u][k] = p[int64_t(c + u * kVSums) * d4 + l + k * LPR];
#pragma unroll
            for (int u = 0; u < kCombineBatch; ++u)
                if (c + u * kVSums < sp.pcnt)
#pragma unroll
                    for (int k = 0; k < NV; ++k) acc[k] = f4_add(acc[k], t[u][k]);
        }
#pragma unroll
        for (int k = 0; k < NV; ++k) lds[v][l + k * LPR] = acc[k];
    }
    __syncthreads();
    if (g != 0) return;
    float4 acc[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] = lds[0][l + k * LPR];
    const int nv = sp.pcnt < kVSums ? sp.pcnt : kVSums;
    for (int h = 1; h < nv; ++h)
#pragma unroll
        for (int k = 0; k < NV; ++k) acc[k] = f4_add(acc[k], lds[h][l + k * LPR]);
    finish_row_vec<LPR, NV>(a, sp.row, l, acc);
}

template <int LPR, int NV>
__global__ __launch_bounds__(kBlock) void k_combine_vec(SpmmArgs a) {
    combine_row<LPR, NV>(a, blockIdx.x);
}

// A split row of at most kVSums chunks, combined by one lane group: running sum v holds partial v
// alone (0 + p_v), and the sums are added in v order — combine_row's association for such a row,
// so bitwise its result — without a workgroup, LDS or a barrier per row. All of the row's partials
// are loaded (predicated past pcnt) before the first add: one memory round trip, not pcnt.
template <int LPR, int NV>
__device__ __forceinline__ void combine_small_row(const SpmmArgs& a, int64_t s, int l) {
    constexpr int B = NV == 1 ? kVSums : kCombineBatch;  // partials in flight (registers: B * NV float4)
    const lgcn_split_t sp = a.splits[s];
    const int64_t d4 = int64_t(LPR) * NV;
    const float4* p = reinterpret_cast<const float4*>(a.partial) + int64_t(sp.pbeg) * d4 + l;
    const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 acc[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] = zero;
    if (sp.pcnt > kVSums) {
        // outside the packed-row contract (pack_split_rows / ride_layout put only rows of <=
        // kVSums chunks here): still combine_row's association — running sum v = 0 + p_v +
        // p_{v+kVSums} + ..., the sums added in v order — one sum at a time (2 x NV registers)
        for (int v = 0; v < kVSums; ++v) {
            float4 s[NV];
#pragma unroll
            for (int k = 0; k < NV; ++k) s[k] = zero;
            for (int c = v; c < sp.pcnt; c += kVSums)
#pragma unroll
                for (int k = 0; k < NV; ++k) s[k] = f4_add(s[k], p[int64_t(c) * d4 + k * LPR]);
#pragma unroll
            for (int k = 0; k < NV; ++k) acc[k] = v == 0 ? s[k] : f4_add(acc[k], s[k]);
        }
        finish_row_vec<LPR, NV>(a, sp.row, l, acc);
        return;
    }
    for (int c0 = 0; c0 < sp.pcnt; c0 += B) {
        float4 t[B][NV];
#pragma unroll
        for (int u = 0; u < B; ++u)
            if (c0 + u < sp.pcnt)
#pragma unroll
                for (int k = 0; k < NV; ++k) t[u][k] = p[int64_t(c0 + u) * d4 + k * LPR];
#pragma unroll
        for (int u = 0; u < B; ++u)
            if (c0 + u < sp.pcnt)
#pragma unroll
                for (int k = 0; k < NV; ++k) acc[k] = c0 + u == 0 ? f4_add(zero, t[u][k]) : f4_add(acc[k], f4_add(zero, t[u][k]));
    }
    finish_row_vec<LPR, NV>(a, sp.row, l, acc);
}

// Workgroups of one pass's combine: a.n_big whole-workgroup rows, then the small rows GPB per block.
template <int LPR, int NV>
__host__ __device__ __forceinline__ int64_t combine_blocks(const SpmmArgs& a) {
    constexpr int GPB = kBlock / LPR;
    const int64_t big = a.n_big < 0 ? a.n_splits : a.n_big;
    return big + (a.n_splits - big + GPB - 1) / GPB;
}

template <int LPR, int NV>
__device__ __forceinline__ void combine_block(const SpmmArgs& a, int64_t blk) {
    constexpr int GPB = kBlock / LPR;
    const int64_t big = a.n_big < 0 ? a.n_splits : a.n_big;
    if (blk < big) {
        combine_row<LPR, NV>(a, blk);
        return;
    }
    const int64_t s = big + (blk - big) * GPB + threadIdx.x / LPR;
    if (s < a.n_splits) combine_small_row<LPR, NV>(a, s, threadIdx.x % LPR);
}

// The split rows of one pass, packed (a.n_big >= 0: lgcn_spmm_pass).
template <int LPR, int NV>
__global__ __launch_bounds__(kBlock) void k_combine_packed(SpmmArgs a) {
    combine_block<LPR, NV>(a, blockIdx.x);
}

// One source-slice launch of a sliced schedule (a, SLICED item pass) carrying another pass's split
// rows (r: combine only) as its first rb workgroups (lgcn_spmm_run_slices_ride): the combine of one
// side's split rows of the layer before, or of the other slice group of this layer, rides in a
// launch that neither reads nor writes those rows or their partials, instead of a launch of its own.
template <int LPR, int NV, int UNROLL, int TAIL, int CM>
__global__ __launch_bounds__(kBlock) void k_spmm_ride(SpmmArgs a, SpmmArgs r, int64_t rb) {
    const int64_t blk = blockIdx.x;
    if (blk < rb) {
        combine_block<LPR, NV>(r, blk);
        return;
    }
    item_pass<LPR, NV, UNROLL, true, TAIL, false, CM>(a, blk - rb);
}

// The split rows of two passes in one launch: a's workgroups first, then b's.
template <int LPR, int NV>
__global__ __launch_bounds__(kBlock) void k_combine_pair(SpmmArgs a, SpmmArgs b, int64_t blocks_a) {
    const int64_t blk = blockIdx.x;
    if (blk < blocks_a)
        combine_block<LPR, NV>(a, blk);
    else
        combine_block<LPR, NV>(b, blk - blocks_a);
}

// ---- generic path: any d <= 64*KMAX, one wave per item, scalar columns ----
constexpr int KMAX = 16;

__device__ __forceinline__ void finish_row_scalar(const SpmmArgs& a, int64_t r, int l, const float (&v)[KMAX]) {
    float* acc = split_row(a.acc_lo, a.acc_hi, a.acc_split, r, a.d);
    const float* e = (a.mode == LGCN_EPI_INIT || a.mode == LGCN_EPI_FINAL_E)
                         ? split_row(a.e_lo, a.e_hi, a.e_split, r, a.d)
                         : nullptr;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
        const int cidx = l + 64 * k;
        if (cidx < a.d) {
            float s;
            if (a.mode == LGCN_EPI_STORE) s = v[k];
            else if (a.mode == LGCN_EPI_SCALE) s = (v[k] * a.mul) / a.div;
            else if (e) s = e[cidx] + v[k];
            else s = acc[cidx] + v[k];
            if (a.mode == LGCN_EPI_FINAL_ACC || a.mode == LGCN_EPI_FINAL_E) s = (s / a.div) * a.mul;
            acc[cidx] = s;
            if (a.y != nullptr && (a.mode == LGCN_EPI_INIT || a.mode == LGCN_EPI_ADD))
                a.y[r * a.d + cidx] = v[k];
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_spmm_scalar(SpmmArgs a) {
    const int g = threadIdx.x / 64;
    const int l = threadIdx.x % 64;
    const int64_t item = int64_t(blockIdx.x) * (kBlock / 64) + g;
    if (item >= a.n_items) return;
    const lgcn_item_t it = a.items[item];
    float acc[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) acc[k] = 0.f;
    for (int e = 0; e < it.len; ++e) {
        const int cj = a.col[it.beg + e];
        const float w = a.val[it.beg + e];
        const float* src = split_row(a.x_lo, a.x_hi, a.x_split, int64_t(cj), a.d);
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
            const int cidx = l + 64 * k;
            if (cidx < a.d) acc[k] = acc[k] + w * src[cidx];
        }
    }
    if (it.dst < 0) {
        float* p = a.partial + int64_t(-it.dst - 1) * a.d;
#pragma unroll
        for (int k = 0; k < KMAX; ++k)
            if (l + 64 * k < a.d) p[l + 64 * k] = acc[k];
        return;
    }
    finish_row_scalar(a, it.dst, l, acc);
}

__global__ __launch_bounds__(kBlock) void k_combine_scalar(SpmmArgs a) {
    const int g = threadIdx.x / 64;
    const int l = threadIdx.x % 64;
    const int64_t s = int64_t(blockIdx.x) * (kBlock / 64) + g;
    if (s >= a.n_splits) return;
    const lgcn_split_t sp = a.splits[s];
    float acc[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) acc[k] = 0.f;
    for (int c = 0; c < sp.pcnt; ++c) {
        const float* p = a.partial + int64_t(sp.pbeg + c) * a.d;
#pragma unroll
        for (int k = 0; k < KMAX; ++k)
            if (l + 64 * k < a.d) acc[k] = acc[k] + p[l + 64 * k];
    }
    finish_row_scalar(a, sp.row, l, acc);
}

enum { PASS_ITEMS = 1, PASS_COMBINE = 2, PASS_BOTH = 3, PASS_BSPLIT = 4, PASS_RIDE = 8 };

template <int LPR, int NV, int UNROLL, int TAIL = 0, int CM = 1>
int launch_vec(const SpmmArgs& a, hipStream_t s, int pass, const SpmmArgs* b = nullptr) {
    constexpr int GPB = kBlock / LPR;
    if (pass == PASS_RIDE) {  // lgcn_spmm_run_slices_ride: a's slice items + b's split-row combine
        const int64_t blocks = (a.n_items + GPB - 1) / GPB, rb = b->n_splits > 0 ? combine_blocks<LPR, NV>(*b) : 0;
        if (blocks + rb > 0) {
            k_spmm_ride<LPR, NV, UNROLL, TAIL, CM><<<dim3(static_cast<unsigned>(blocks + rb)), kBlock, 0, s>>>(a, *b, rb);
            return check_launch("k_spmm_ride");
        }
        return LGCN_OK;
    }
    if (b != nullptr) {  // lgcn_spmm_pair: two plain passes, one launch per half
        if (pass & PASS_ITEMS) {
            const int64_t ba = (a.n_items + GPB - 1) / GPB, bb = (b->n_items + GPB - 1) / GPB;
            if (ba + bb > 0) {
                k_spmm_pair<LPR, NV, UNROLL, TAIL, CM><<<dim3(static_cast<unsigned>(ba + bb)), kBlock, 0, s>>>(
                    a, *b, ba, bb, pair_xcd_a());
                if (int rc = check_launch("k_spmm_pair")) return rc;
            }
        }
        if ((pass & PASS_COMBINE) && a.n_splits + b->n_splits > 0) {
            const int64_t ca = combine_blocks<LPR, NV>(a), cb = combine_blocks<LPR, NV>(*b);
            k_combine_pair<LPR, NV><<<dim3(static_cast<unsigned>(ca + cb)), kBlock, 0, s>>>(a, *b, ca);
            if (int rc = check_launch("k_combine_pair")) return rc;
        }
        return LGCN_OK;
    }
    if (pass == PASS_BSPLIT) {  // split rows (one workgroup each) and items in one launch
        const int64_t blocks = a.n_splits + (a.n_items + GPB - 1) / GPB;
        if (blocks > 0) {
            k_spmm_vec<LPR, NV, UNROLL, false, TAIL, true, CM><<<dim3(static_cast<unsigned>(blocks)), kBlock, 0, s>>>(a);
            if (int rc = check_launch("k_spmm_vec")) return rc;
        }
        return LGCN_OK;
    }
    if ((pass & PASS_ITEMS) && a.n_items > 0) {
        const int64_t blocks = (a.n_items + GPB - 1) / GPB;
        if (a.run != nullptr)
            k_spmm_vec<LPR, NV, UNROLL, true, TAIL, false, CM><<<dim3(static_cast<unsigned>(blocks)), kBlock, 0, s>>>(a);
        else
            k_spmm_vec<LPR, NV, UNROLL, false, TAIL, false, CM><<<dim3(static_cast<unsigned>(blocks)), kBlock, 0, s>>>(a);
        if (int rc = check_launch("k_spmm_vec")) return rc;
    }
    if ((pass & PASS_COMBINE) && a.n_splits > 0) {
        if (a.n_big >= 0) {  // lgcn_spmm_pass with n_split_big: the small rows one per lane group
            k_combine_packed<LPR, NV><<<dim3(static_cast<unsigned>(combine_blocks<LPR, NV>(a))), kBlock, 0, s>>>(a);
            return check_launch("k_combine_packed");
        }
        k_combine_vec<LPR, NV><<<dim3(static_cast<unsigned>(a.n_splits)), kBlock, 0, s>>>(a);
        if (int rc = check_launch("k_combine_vec")) return rc;
    }
    return LGCN_OK;
}


int launch_scalar(const SpmmArgs& a, hipStream_t s, int pass) {
    constexpr int GPB = kBlock / 64;
    if ((pass & PASS_ITEMS) && a.n_items > 0) {
        const int64_t blocks = (a.n_items + GPB - 1) / GPB;
        k_spmm_scalar<<<dim3(static_cast<unsigned>(blocks)), kBlock, 0, s>>>(a);
        if (int rc = check_launch("k_spmm_scalar")) return rc;
    }
    if ((pass & PASS_COMBINE) && a.n_splits > 0) {
        const int64_t blocks = (a.n_splits + GPB - 1) / GPB;
        k_combine_scalar<<<dim3(static_cast<unsigned>(blocks)), kBlock, 0, s>>>(a);
        if (int rc = check_launch("k_combine_scalar")) return rc;
    }
    return LGCN_OK;
}


bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

__global__ void k_scale(const float* __restrict__ in, float* __restrict__ out, int64_t n, float mul, float div) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
        out[i] = (in[i] * mul) / div;
}

// out[r] = (((e[r] + y0[r]) + y1[r]) + ... + y_{K-1}[r]) / div * mul (K == 1: (e + y0) / div * mul):
// the same roundings in the same order as the INIT / ADD / FINAL_ACC (FINAL_E) epilogues.
struct StackRows {
    const float* y[8];
};
__global__ void k_stack_mean(const float4* __restrict__ e, StackRows ys, int32_t K, int64_t n4, float4* __restrict__ out,
                             float div, float mul) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n4; i += stride) {
        float4 acc = e[i];
        for (int k = 0; k < K; ++k) acc = f4_add(acc, reinterpret_cast<const float4*>(ys.y[k])[i]);
        out[i] = f4_divmul(acc, div, mul);
    }
}

__global__ void k_copy_scale(const float* __restrict__ lo, const float* __restrict__ hi, int64_t split,
                             int64_t N, int32_t d, float* __restrict__ out, float div, float mul) {
    const int64_t n = N * d;
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int64_t r = i / d;
        const int64_t c = i - r * d;
        const float x = (r < split) ? lo[r * d + c] : hi[(r - split) * d + c];
        out[i] = (x / div) * mul;
    }
}

// Argument checks of one pass (everything but the empty-pass shortcut); LGCN_OK or the failure.
int check_pass(const lgcn_item_t* items, int64_t n_items, const lgcn_split_t* splits, int64_t n_splits, int64_t N,
               int32_t d, const float* x_lo, const float* x_hi, int64_t x_split, const float* e_lo, const float* e_hi,
               int64_t e_split, const float* acc_lo, const float* acc_hi, int64_t acc_split, const float* partial,
               int32_t mode, int pass, const lgcn_item_t* chunks) {
    if (N < 0 || d <= 0 || n_items < 0 || n_splits < 0)
        return fail(LGCN_E_ARG, "lgcn_spmm: bad sizes (N=%lld d=%d)", (long long)N, d);
    if (mode < LGCN_EPI_INIT || mode > LGCN_EPI_SCALE) return fail(LGCN_E_ARG, "lgcn_spmm: bad mode %d", mode);
    if (N == 0 || (n_items == 0 && n_splits == 0)) return LGCN_OK;
    // col/val may be NULL for an edge-free plan (every item then has len 0)
    if ((n_items > 0 && !items) || !x_lo || !acc_lo) return fail(LGCN_E_ARG, "lgcn_spmm: null items/x/acc");
    if (x_split < N && !x_hi) return fail(LGCN_E_ARG, "lgcn_spmm: x_hi required (x_split < N)");
    if (acc_split < N && !acc_hi) return fail(LGCN_E_ARG, "lgcn_spmm: acc_hi required (acc_split < N)");
    const bool needs_e = (mode == LGCN_EPI_INIT || mode == LGCN_EPI_FINAL_E);
    if (needs_e && (!e_lo || (e_split < N && !e_hi)))
        return fail(LGCN_E_ARG, "lgcn_spmm: mode %d needs the e table", mode);
    if (pass == PASS_BSPLIT) {
        if (n_splits > 0 && (!splits || !chunks))
            return fail(LGCN_E_ARG, "lgcn_spmm_blocksplit: splits need their chunk items");
    } else if (n_splits > 0 && (!splits || !partial)) {
        return fail(LGCN_E_ARG, "lgcn_spmm: splits need partial scratch");
    }
    if (d > 64 * KMAX && d % 4 != 0)
        return fail(LGCN_E_UNSUPPORTED, "lgcn_spmm: d=%d unsupported (d > %d needs d %% 4 == 0)", d, 64 * KMAX);
    return LGCN_OK;
}

bool vec_aligned(const SpmmArgs& a) {
    return (a.d % 4 == 0) && aligned16(a.x_lo) && aligned16(a.acc_lo) && aligned16(a.partial) &&
           (a.x_hi == nullptr || aligned16(a.x_hi)) && (a.acc_hi == nullptr || aligned16(a.acc_hi)) &&
           (a.e_lo == nullptr || aligned16(a.e_lo)) && (a.e_hi == nullptr || aligned16(a.e_hi)) &&
           (a.y == nullptr || aligned16(a.y));
}

int dispatch(SpmmArgs& a, int64_t N, hipStream_t s, int pass, float* run, const SpmmArgs* b);

int spmm_impl(const lgcn_item_t* items, int64_t n_items, const lgcn_split_t* splits, int64_t n_splits,
              const int32_t* col, const float* val, int64_t N, int32_t d, const float* x_lo,
              const float* x_hi, int64_t x_split, const float* e_lo, const float* e_hi, int64_t e_split,
              float* y, float* acc_lo, float* acc_hi, int64_t acc_split, float* partial, int32_t mode,
              float div, float mul, lgcn_stream_t stream, int pass, float* run = nullptr,
              const lgcn_item_t* chunks = nullptr) {
    if (int rc = check_pass(items, n_items, splits, n_splits, N, d, x_lo, x_hi, x_split, e_lo, e_hi, e_split, acc_lo,
                            acc_hi, acc_split, partial, mode, pass, chunks))
        return rc;
    if (N == 0 || (n_items == 0 && n_splits == 0)) return LGCN_OK;
    SpmmArgs a{items, n_items, splits, n_splits, col, val, x_lo, x_hi, x_split, e_lo, e_hi, e_split,
               y, acc_lo, acc_hi, acc_split, partial, d, mode, div, mul, run, chunks};
    return dispatch(a, N, as_stream(stream), pass, run, nullptr);
}

// The kernel instance for width d (and the launch's kind), launched for pass a — or for the pair
// (a, b) of lgcn_spmm_pair, which share d, N and the instance.
int dispatch(SpmmArgs& a, int64_t N, hipStream_t s, int pass, float* run, const SpmmArgs* b) {
    const int32_t d = a.d;
    const int64_t n_items = a.n_items + (b ? b->n_items : 0);
    // Non-temporal row traffic (epilogue e/acc/y and running-sum loads and stores): those rows are
    // touched once per launch, so they stream past the L2 and leave it to the gathered rows.
    // Measured (profiles/r02z_nt/): sliced C2 K=3 d=64 1.274 -> 1.241 ms, d=32 0.747 -> 0.698. On
    // for sliced launches and for tables beyond the Infinity Cache (C5); off for plain launches
    // over cache-resident tables — the sharded ranks' plain schedule measured +2-3 % with it (their
    // y is the next layer's gathered table) — and for block-split Cluster-GCN launches (+2.6 %).
    // (Re-checked on the round-4 sliced schedule: 3 / 0 / 1 / 2 -> 1.217 / 1.226 / 1.233 / 1.218 ms,
    // profiles/r04zk_nt/ — settled, so no longer a knob.)
    a.nt = (pass != PASS_BSPLIT && (run != nullptr || N * int64_t(d) * 4 > (int64_t(512) << 20))) ? 3 : 0;
    SpmmArgs bb;
    if (b != nullptr) {
        bb = *b;
        bb.nt = pass == PASS_RIDE ? 0 : a.nt;  // a riding combine keeps the standalone combine's stores
        b = &bb;
    }

    const bool vec_ok = vec_aligned(a) && (b == nullptr || vec_aligned(*b));
    if (b != nullptr && !vec_ok)
        return fail(LGCN_E_UNSUPPORTED, "%s: needs d in {4,8,...,1024} and aligned rows",
                    pass == PASS_RIDE ? "lgcn_spmm_run_slices_ride" : "lgcn_spmm_pair");
    if (vec_ok) {
        // Predicated tail (TAIL = 1): a row's last < UNROLL edges of each batch are gathered
        // together instead of one at a time. It costs VGPRs (occupancy 6-7 -> 4 waves/SIMD at
        // d >= 32), so it is on where latency, not loads in flight, bounds the pass: d <= 64, and
        // small plain-schedule launches (Cluster-GCN batch plans). Measured (profiles/r01k_tail/):
        // C2 d=32 -6 %, d=64 -2 %, C3 training step -5 %; C2 d=128 / d=256 +3 % (kept off there).
        // lgcn_tuning_t.spmm_tail: -1 = this choice, 0 / 1 = forced off / on. (The 16-deep
        // unroll at d = 64, once variant 1 of this knob, measured within 1 % or slower in every
        // round: removed.)
        const int tv = tuning().spmm_tail;
        const bool tail = tv == 1 || (tv < 0 && (d <= 64 || (run == nullptr && n_items <= 65536)));
        // Index load rounds (CM batches of LPR edges per col/val load): one or two 128-B lines of
        // col per round at narrow rows, on every launch but the block-split Cluster-GCN batch plans
        // (at d = 128 the C3 step measured +11 % with CM = 4, so d >= 128 keeps one batch per round).
        // Measured (profiles/r02x_cm/): C2 K=3 d=64 1.317 -> 1.269 ms (CM 4), d=32 0.791 -> 0.742
        // (CM 4), d=16 0.859 -> 0.610 (CM 16), d=8 1.354 -> 0.773 (CM 32); d=128/256 slower (kept at 1).
        // The narrow-row round path at d=32 measured the same as per-batch (0.739 vs 0.743 ms), at d=64
        // +5 %. lgcn_tuning_t.spmm_index_rounds overrides.
        const bool rounds = pass != PASS_BSPLIT;
        const int cm = tuning().spmm_index_rounds;
        if (tail) {
            switch (d) {
                case 4: return (cm ? cm : rounds ? 32 : 8) == 32 ? launch_vec<1, 1, 8, 1, 32>(a, s, pass, b)
                                                                : launch_vec<1, 1, 8, 1, 8>(a, s, pass, b);
                case 8: {
                    const int c = cm ? cm : rounds ? 32 : 4;
                    return c == 16 ? launch_vec<2, 1, 8, 1, 16>(a, s, pass, b)
                         : c == 32 ? launch_vec<2, 1, 8, 1, 32>(a, s, pass, b) : launch_vec<2, 1, 8, 1, 4>(a, s, pass, b);
                }
                case 16: {
                    const int c = cm ? cm : rounds ? 16 : 2;
                    return c == 8 ? launch_vec<4, 1, 8, 1, 8>(a, s, pass, b)
                         : c == 16 ? launch_vec<4, 1, 8, 1, 16>(a, s, pass, b) : launch_vec<4, 1, 8, 1, 2>(a, s, pass, b);
                }
                case 32: {
                    const int c = cm ? cm : rounds ? 4 : 1;
                    return c == 4 ? launch_vec<8, 1, 8, 1, 4>(a, s, pass, b)
                         : c == 8 ? launch_vec<8, 1, 8, 1, 8>(a, s, pass, b) : launch_vec<8, 1, 8, 1>(a, s, pass, b);
                }
                case 64: {
                    const int c = cm ? cm : rounds ? 4 : 1;
                    return c == 4 ? launch_vec<16, 1, 8, 1, 4>(a, s, pass, b)
                         : c == 2 ? launch_vec<16, 1, 8, 1, 2>(a, s, pass, b) : launch_vec<16, 1, 8, 1>(a, s, pass, b);
                }
                case 128: return launch_vec<32, 1, 8, 1>(a, s, pass, b);
                case 256: return launch_vec<64, 1, 8, 1>(a, s, pass, b);
                case 512: return launch_vec<64, 2, 4, 1>(a, s, pass, b);
                case 1024: return launch_vec<64, 4, 2, 1>(a, s, pass, b);
                default: break;
            }
        }
        switch (d) {
            case 4: return launch_vec<1, 1, 8, 0, 8>(a, s, pass, b);
            case 8: return launch_vec<2, 1, 8, 0, 4>(a, s, pass, b);
            case 16: return launch_vec<4, 1, 8, 0, 2>(a, s, pass, b);
            case 32: return launch_vec<8, 1, 8>(a, s, pass, b);
            case 64: return launch_vec<16, 1, 8>(a, s, pass, b);
            case 128: return launch_vec<32, 1, 8>(a, s, pass, b);
            case 256: return launch_vec<64, 1, 8>(a, s, pass, b);
            case 512: return launch_vec<64, 2, 4>(a, s, pass, b);
            case 1024: return launch_vec<64, 4, 2>(a, s, pass, b);
            default: break;
        }
    }
    if (run != nullptr) return fail(LGCN_E_UNSUPPORTED, "lgcn_spmm_run: needs d in {4,8,...,1024} and aligned rows");
    if (pass == PASS_BSPLIT)
        return fail(LGCN_E_UNSUPPORTED, "lgcn_spmm_blocksplit: needs d in {4,8,...,1024} and aligned rows");
    if (d > 64 * KMAX) return fail(LGCN_E_UNSUPPORTED, "lgcn_spmm: d=%d unsupported", d);
    return launch_scalar(a, s, pass);
}

}  // namespace

extern "C" {

#define LGCN_SPMM_PARAMS                                                                             \
    const lgcn_item_t *items, int64_t n_items, const lgcn_split_t *splits, int64_t n_splits,        \
        const int32_t *col, const float *val, int64_t N, int32_t d, const float *x_lo,              \
        const float *x_hi, int64_t x_split, const float *e_lo, const float *e_hi, int64_t e_split,  \
        float *y, float *acc_lo, float *acc_hi, int64_t acc_split, float *partial, int32_t mode,     \
        float div, float mul, lgcn_stream_t stream
#define LGCN_SPMM_ARGS                                                                              \
    items, n_items, splits, n_splits, col, val, N, d, x_lo, x_hi, x_split, e_lo, e_hi, e_split, y, \
        acc_lo, acc_hi, acc_split, partial, mode, div, mul, stream

int lgcn_spmm(LGCN_SPMM_PARAMS) { return spmm_impl(LGCN_SPMM_ARGS, PASS_BOTH); }
int lgcn_spmm_items(LGCN_SPMM_PARAMS) { return spmm_impl(LGCN_SPMM_ARGS, PASS_ITEMS); }
int lgcn_spmm_combine(LGCN_SPMM_PARAMS) { return spmm_impl(LGCN_SPMM_ARGS, PASS_COMBINE); }
int lgcn_spmm_run(LGCN_SPMM_PARAMS, float* run) {
    if (!run) return fail(LGCN_E_ARG, "lgcn_spmm_run: null running-sum buffer");
    return spmm_impl(LGCN_SPMM_ARGS, PASS_ITEMS, run);
}
int lgcn_spmm_run_slices(const lgcn_item_t* items, const int64_t* slice_offsets, int32_t S, const int32_t* col,
                         const float* val, int64_t N, int32_t d, const float* x_lo, const float* x_hi,
                         int64_t x_split, const float* e_lo, const float* e_hi, int64_t e_split, float* y,
                         float* acc_lo, float* acc_hi, int64_t acc_split, float* partial, int32_t mode, float div,
                         float mul, lgcn_stream_t stream, float* run) {
    if (!run || S < 0 || (S > 0 && (!items || !slice_offsets)))
        return fail(LGCN_E_ARG, "lgcn_spmm_run_slices: bad args");
    for (int32_t sl = 0; sl < S; ++sl) {
        const int64_t b = slice_offsets[sl], n = slice_offsets[sl + 1] - b;
        if (b < 0 || n < 0) return fail(LGCN_E_ARG, "lgcn_spmm_run_slices: offsets not ascending at slice %d", sl);
        if (n == 0) continue;
        if (int rc = spmm_impl(items + b, n, nullptr, 0, col, val, N, d, x_lo, x_hi, x_split, e_lo, e_hi, e_split, y,
                               acc_lo, acc_hi, acc_split, partial, mode, div, mul, stream, PASS_ITEMS, run))
            return rc;
    }
    return LGCN_OK;
}
int lgcn_spmm_blocksplit(LGCN_SPMM_PARAMS, const lgcn_item_t* chunks) {
    return spmm_impl(LGCN_SPMM_ARGS, PASS_BSPLIT, nullptr, chunks);
}

// lgcn_pass_t -> SpmmArgs, validated as a plain pass of width d over N rows.
static int pass_args(const lgcn_pass_t& p, int64_t N, int32_t d, const char* who, SpmmArgs& out) {
    if (int rc = check_pass(p.items, p.n_items, p.splits, p.n_splits, N, d, p.x_lo, p.x_hi, p.x_split, p.e_lo,
                            p.e_hi, p.e_split, p.acc_lo, p.acc_hi, p.acc_split, p.partial, p.mode, PASS_BOTH, nullptr))
        return rc;
    if (p.n_split_big > p.n_splits)
        return fail(LGCN_E_ARG, "%s: n_split_big %lld > n_splits %lld", who, (long long)p.n_split_big,
                    (long long)p.n_splits);
    out = SpmmArgs{p.items, p.n_items, p.splits, p.n_splits, p.col, p.val, p.x_lo, p.x_hi, p.x_split,
                   p.e_lo, p.e_hi, p.e_split, p.y, p.acc_lo, p.acc_hi, p.acc_split, p.partial, d, p.mode,
                   p.div, p.mul, nullptr, nullptr};
    out.n_big = p.n_split_big < 0 ? -1 : p.n_split_big;
    return LGCN_OK;
}

int lgcn_spmm_pair(const lgcn_pass_t* a, const lgcn_pass_t* b, int64_t N, int32_t d, int32_t what,
                   lgcn_stream_t stream) {
    if (!a || !b || what < 1 || what > 3) return fail(LGCN_E_ARG, "lgcn_spmm_pair: bad args");
    SpmmArgs args[2];
    if (int rc = pass_args(*a, N, d, "lgcn_spmm_pair", args[0])) return rc;
    if (int rc = pass_args(*b, N, d, "lgcn_spmm_pair", args[1])) return rc;
    if (N == 0) return LGCN_OK;
    return dispatch(args[0], N, as_stream(stream), what, nullptr, &args[1]);
}

int lgcn_spmm_pass(const lgcn_pass_t* p, int64_t N, int32_t d, int32_t what, lgcn_stream_t stream) {
    if (!p || what < 1 || what > 3) return fail(LGCN_E_ARG, "lgcn_spmm_pass: bad args");
    SpmmArgs a;
    if (int rc = pass_args(*p, N, d, "lgcn_spmm_pass", a)) return rc;
    if (N == 0) return LGCN_OK;
    return dispatch(a, N, as_stream(stream), what, nullptr, nullptr);
}

int lgcn_spmm_run_slices_ride(const lgcn_item_t* items, const int64_t* slice_offsets, int32_t S, const int32_t* col,
                              const float* val, int64_t N, int32_t d, const float* x_lo, const float* x_hi,
                              int64_t x_split, const float* e_lo, const float* e_hi, int64_t e_split, float* y,
                              float* acc_lo, float* acc_hi, int64_t acc_split, float* partial, int32_t mode,
                              float div, float mul, lgcn_stream_t stream, float* run, const lgcn_pass_t* ride,
                              int32_t ride_slice) {
    if (!run || S < 0 || (S > 0 && (!items || !slice_offsets)))
        return fail(LGCN_E_ARG, "lgcn_spmm_run_slices_ride: bad args");
    SpmmArgs r{};
    const bool riding = ride != nullptr && ride->n_splits > 0;
    if (riding) {
        if (ride_slice < 0 || ride_slice >= S)
            return fail(LGCN_E_ARG, "lgcn_spmm_run_slices_ride: ride_slice %d outside [0, %d)", ride_slice, S);
        if (int rc = pass_args(*ride, N, d, "lgcn_spmm_run_slices_ride", r)) return rc;
    }
    for (int32_t sl = 0; sl < S; ++sl) {
        const int64_t b = slice_offsets[sl], n = slice_offsets[sl + 1] - b;
        if (b < 0 || n < 0) return fail(LGCN_E_ARG, "lgcn_spmm_run_slices_ride: offsets not ascending at slice %d", sl);
        const bool here = riding && sl == ride_slice;
        if (here && n == 0) {  // nothing to ride in: the combine alone
            if (int rc = dispatch(r, N, as_stream(stream), PASS_COMBINE, nullptr, nullptr)) return rc;
            continue;
        }
        if (n == 0) continue;
        if (!here) {
            if (int rc = spmm_impl(items + b, n, nullptr, 0, col, val, N, d, x_lo, x_hi, x_split, e_lo, e_hi, e_split,
                                   y, acc_lo, acc_hi, acc_split, partial, mode, div, mul, stream, PASS_ITEMS, run))
                return rc;
            continue;
        }
        if (int rc = check_pass(items + b, n, nullptr, 0, N, d, x_lo, x_hi, x_split, e_lo, e_hi, e_split, acc_lo,
                                acc_hi, acc_split, partial, mode, PASS_ITEMS, nullptr))
            return rc;
        SpmmArgs a{items + b, n, nullptr, 0, col, val, x_lo, x_hi, x_split, e_lo, e_hi, e_split,
                   y, acc_lo, acc_hi, acc_split, partial, d, mode, div, mul, run, nullptr};
        if (int rc = dispatch(a, N, as_stream(stream), PASS_RIDE, run, &r)) return rc;
    }
    return LGCN_OK;
}

int lgcn_stack_mean_rows(const float* e, const float* const* ys, int32_t K, int64_t rows, int32_t d, float* out,
                         float div, float mul, lgcn_stream_t stream) {
    if (K < 1 || K > 8 || rows < 0 || d <= 0 || d % 4 != 0 || (rows > 0 && (!e || !ys || !out)))
        return fail(LGCN_E_ARG, "lgcn_stack_mean_rows: bad args (K=%d rows=%lld d=%d)", K, (long long)rows, d);
    if (rows == 0) return LGCN_OK;
    StackRows st{};
    for (int k = 0; k < K; ++k) {
        if (!ys[k] || !aligned16(ys[k])) return fail(LGCN_E_ARG, "lgcn_stack_mean_rows: layer %d table", k);
        st.y[k] = ys[k];
    }
    if (!aligned16(e) || !aligned16(out)) return fail(LGCN_E_UNSUPPORTED, "lgcn_stack_mean_rows: alignment");
    const int64_t n4 = rows * d / 4;
    k_stack_mean<<<grid_for(n4, kBlock, 16384), kBlock, 0, as_stream(stream)>>>(
        reinterpret_cast<const float4*>(e), st, K, n4, reinterpret_cast<float4*>(out), div, mul);
    return check_launch("k_stack_mean");
}

int lgcn_scale(const float* in, float* out, int64_t n, float mul, float div, lgcn_stream_t stream) {
    if (n < 0 || (n > 0 && (!in || !out))) return fail(LGCN_E_ARG, "lgcn_scale: bad args");
    if (n == 0) return LGCN_OK;
    k_scale<<<grid_for(n, kBlock, 16384), kBlock, 0, as_stream(stream)>>>(in, out, n, mul, div);
    return check_launch("k_scale");
}

int lgcn_copy_scale(const float* x_lo, const float* x_hi, int64_t x_split, int64_t N, int32_t d,
                    float* out, float div, float mul, lgcn_stream_t stream) {
    if (N < 0 || d <= 0 || (N > 0 && (!x_lo || !out)) || (x_split < N && !x_hi))
        return fail(LGCN_E_ARG, "lgcn_copy_scale: bad args");
    if (N == 0) return LGCN_OK;
    k_copy_scale<<<grid_for(N * d, kBlock, 16384), kBlock, 0, as_stream(stream)>>>(x_lo, x_hi, x_split, N, d,
                                                                                   out, div, mul);
    return check_launch("k_copy_scale");
}

}  // extern "C"
