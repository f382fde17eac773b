// Fused cosine-BPR loss and its gradient for the Cluster-GCN training step (gfx950).
//
// Reference utils/train_test.py:105-134 (compute_embeddings: six row gathers) and :18-64
// (bpr_loss: L2 reg on layer-0 rows, row-normalised cosines, softplus(10 * margin)):
//   loss = -mean_b softplus(10 (cos(u_b, p_b) - cos(u_b, n_b))) / 10
//          + coeff * mean_{b,c} (eu_bc^2 + ep_bc^2 + en_bc^2)
// PyTorch runs this as ~25 elementwise/reduction launches forward, ~30 backward, and scatters
// the row gradients with a sort-based index_put_. Here:
//   k_bpr_fused   one lane group per triplet: loads the 6 rows once (propagated F rows for the
//                 cosines, layer-0 W rows for the reg term), reduces the 6 dot products inside
//                 the group, and writes the per-triplet gradient rows (dF for u, p, n and the
//                 reg gradient for W) plus the two loss terms — no atomics;
//   k_bpr_loss    deterministic sum of the loss terms (one block, or 256 shares + one block);
//   k_segment_rows  adds the gradient rows into their destination rows in a fixed (stable
//                 sorted) order using the CSR lgcn_csr_build makes of the 3B row keys.
// The gradient is the analytic derivative of the same expression (not bitwise torch autograd).

#include <climits>

#include "lgcn_common.h"
#include "lgcn_reg.h"

using namespace lgcn;

namespace {

template <class T>
__device__ __forceinline__ T* srow(T* lo, T* hi, int64_t split, int64_t r, int64_t stride) {
    return (r < split) ? lo + r * stride : hi + (r - split) * stride;
}

// The reg-gradient rows of the BPR loss (reference utils/train_test.py:38-41: reg = coeff *
// mean(eu^2 + ep^2 + en^2) over the layer-0 rows) are kreg * W[row] for every occurrence of a row,
// kreg = coeff * 2 / (B * d): all the rows summed into one output row are the SAME row. So their
// sum needs no materialised [3B, d] table: it is n copies of kreg * W[row] added in sequence.
struct RegSrc {
    const float* w_lo;  // nullptr: no reg rows
    const float* w_hi;
    int64_t w_split;
    float coeff;
    int64_t B;
};

// acc = (((0 + v) + v) + ...) n times, v = kreg * W[row] (lgcn_reg.h): lane l's NV float4 slots
template <int LPR, int NV>
__device__ __forceinline__ void reg_sum(const RegSrc& r, int64_t row, int32_t d, int64_t n, int l, float4 (&acc)[NV]) {
    const float kreg = reg_scale(r.coeff, r.B, d);
    const float4* w = reinterpret_cast<const float4*>(row < r.w_split ? r.w_lo + row * d : r.w_hi + (row - r.w_split) * d) + l;
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] = reg_copies(w[k * LPR], kreg, n);
}

template <int LPR>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
    for (int off = LPR / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, LPR);
    return v;
}

__device__ __forceinline__ float dot4(float4 a, float4 b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }

struct BprArgs {
    const float* f_lo;
    const float* f_hi;
    int64_t f_split;
    const float* w_lo;
    const float* w_hi;
    int64_t w_split;
    int64_t U;
    const int64_t* u;
    const int64_t* p;
    const int64_t* n;
    int64_t B;
    int32_t d;
    const uint8_t* touched;  // nullable: rows not propagated use (W / div) * mul
    float div;
    float mul;
    float coeff;
    float* cf;     // [3B, d] dF rows (u | p | n)
    float* cw;     // [3B, d] reg-gradient rows for W (u | p | n)
    float* terms;  // [2B]: softplus terms | reg row sums
    // column-sharded training (lgcn_bpr_fused_cols): the rows are one rank's d of d_full columns
    float* sums;     // [B, 6] per-triplet (|u|^2, |p|^2, |n|^2, u.p, u.n, reg squares)
    int32_t d_full;  // the full width (reg mean); == d unsharded
};

// phase 0: fused (the sums reduced inside the lane group); 1: write this rank's column partials
// of the six sums to a.sums and stop; 2: read the six full sums from a.sums (all-reduced over the
// column groups) and finish with them.
constexpr int kBprFused = 0, kBprPartials = 1, kBprFromSums = 2;

// SPEC: the propagated rows of u, p and n are loaded beside the touched flags and the W rows, and
// the flag then picks F or (W / div) * mul (one dependent load level fewer per triplet; the same
// values). It pays on small batches, whose negatives mostly hit propagated rows; on large ones
// (most negatives untouched) the extra F reads cost more (profiles/r06q_bpr_speculative/).
constexpr int64_t kBprSpecMaxB = 49152;

template <int LPR, int NV, int PHASE, bool SPEC = false>
__global__ __launch_bounds__(kBlock) void k_bpr_fused(BprArgs a) {
    constexpr int GPB = kBlock / LPR;
    const int g = threadIdx.x / LPR;
    const int l = threadIdx.x % LPR;
    const int64_t b = int64_t(blockIdx.x) * GPB + g;
    if (b >= a.B) return;
    const int64_t d = a.d;
    const int64_t ru = a.u[b];
    const int64_t rp = a.U + a.p[b];
    const int64_t rn = a.U + a.n[b];
    const float4* wu = reinterpret_cast<const float4*>(srow(a.w_lo, a.w_hi, a.w_split, ru, d)) + l;
    const float4* wp = reinterpret_cast<const float4*>(srow(a.w_lo, a.w_hi, a.w_split, rp, d)) + l;
    const float4* wn = reinterpret_cast<const float4*>(srow(a.w_lo, a.w_hi, a.w_split, rn, d)) + l;
    // a row the sparse batch never reached is (x0 / div) * mul: read it from W instead of F
    const bool tu = a.touched == nullptr || a.touched[ru];
    const bool tp = a.touched == nullptr || a.touched[rp];
    const bool tn = a.touched == nullptr || a.touched[rn];
    const float4* fu = (SPEC || tu) ? reinterpret_cast<const float4*>(srow(a.f_lo, a.f_hi, a.f_split, ru, d)) + l : wu;
    const float4* fp = (SPEC || tp) ? reinterpret_cast<const float4*>(srow(a.f_lo, a.f_hi, a.f_split, rp, d)) + l : wp;
    const float4* fn = (SPEC || tn) ? reinterpret_cast<const float4*>(srow(a.f_lo, a.f_hi, a.f_split, rn, d)) + l : wn;
    float4 U_[NV], P_[NV], N_[NV], WU[NV], WP[NV], WN[NV];
    float suu = 0.f, spp = 0.f, snn = 0.f, sup = 0.f, sun = 0.f, sreg = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        U_[k] = fu[k * LPR];
        P_[k] = fp[k * LPR];
        N_[k] = fn[k * LPR];
        WU[k] = wu[k * LPR];
        WP[k] = wp[k * LPR];
        WN[k] = wn[k * LPR];
        if constexpr (SPEC) {  // an untouched row's F is not the propagated value: take it from W
            if (!tu) U_[k] = WU[k];
            if (!tp) P_[k] = WP[k];
            if (!tn) N_[k] = WN[k];
        }
        if (!tu) U_[k] = make_float4((U_[k].x / a.div) * a.mul, (U_[k].y / a.div) * a.mul, (U_[k].z / a.div) * a.mul, (U_[k].w / a.div) * a.mul);
        if (!tp) P_[k] = make_float4((P_[k].x / a.div) * a.mul, (P_[k].y / a.div) * a.mul, (P_[k].z / a.div) * a.mul, (P_[k].w / a.div) * a.mul);
        if (!tn) N_[k] = make_float4((N_[k].x / a.div) * a.mul, (N_[k].y / a.div) * a.mul, (N_[k].z / a.div) * a.mul, (N_[k].w / a.div) * a.mul);
        suu += dot4(U_[k], U_[k]);
        spp += dot4(P_[k], P_[k]);
        snn += dot4(N_[k], N_[k]);
        sup += dot4(U_[k], P_[k]);
        sun += dot4(U_[k], N_[k]);
        sreg += dot4(WU[k], WU[k]) + dot4(WP[k], WP[k]) + dot4(WN[k], WN[k]);
    }
    suu = group_sum<LPR>(suu);
    spp = group_sum<LPR>(spp);
    snn = group_sum<LPR>(snn);
    sup = group_sum<LPR>(sup);
    sun = group_sum<LPR>(sun);
    sreg = group_sum<LPR>(sreg);
    if constexpr (PHASE == kBprPartials) {
        if (l == 0) {
            float* o = a.sums + b * 6;
            o[0] = suu, o[1] = spp, o[2] = snn, o[3] = sup, o[4] = sun, o[5] = sreg;
        }
        return;
    }
    if constexpr (PHASE == kBprFromSums) {
        const float* o = a.sums + b * 6;
        suu = o[0], spp = o[1], snn = o[2], sup = o[3], sun = o[4], sreg = o[5];
    }
    const float nu = sqrtf(suu), np = sqrtf(spp), nn = sqrtf(snn);
    const float cp = sup / (nu * np);
    const float cn = sun / (nu * nn);
    const float z = 10.0f * (cp - cn);
    // F.softplus(beta=1, threshold=20) and its derivative
    const float sp = (z > 20.0f) ? z : log1pf(expf(z));
    const float sg = (z > 20.0f) ? 1.0f : 1.0f / (1.0f + expf(-z));
    const float inv_b = 1.0f / static_cast<float>(a.B);
    const float dcp = -sg * inv_b;  // d loss / d cos(u,p)
    const float dcn = sg * inv_b;   // d loss / d cos(u,n)
    const float kreg = a.coeff * 2.0f / (static_cast<float>(a.B) * static_cast<float>(a.d_full));
    const float inu = 1.0f / nu, inp = 1.0f / np, inn = 1.0f / nn;
    float4* cfu = reinterpret_cast<float4*>(a.cf + b * d) + l;
    float4* cfp = reinterpret_cast<float4*>(a.cf + (a.B + b) * d) + l;
    float4* cfn = reinterpret_cast<float4*>(a.cf + (2 * a.B + b) * d) + l;
    float4* cwu = a.cw ? reinterpret_cast<float4*>(a.cw + b * d) + l : nullptr;
    float4* cwp = a.cw ? reinterpret_cast<float4*>(a.cw + (a.B + b) * d) + l : nullptr;
    float4* cwn = a.cw ? reinterpret_cast<float4*>(a.cw + (2 * a.B + b) * d) + l : nullptr;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        float4 du, dp, dn;
#define LGCN_BPR_LANE(c)                                                                 \
    {                                                                                    \
        const float av = U_[k].c * inu, bv = P_[k].c * inp, cv = N_[k].c * inn;           \
        du.c = (dcp * (bv - cp * av) + dcn * (cv - cn * av)) * inu;                      \
        dp.c = dcp * (av - cp * bv) * inp;                                               \
        dn.c = dcn * (av - cn * cv) * inn;                                               \
    }
        LGCN_BPR_LANE(x) LGCN_BPR_LANE(y) LGCN_BPR_LANE(z) LGCN_BPR_LANE(w)
#undef LGCN_BPR_LANE
        cfu[k * LPR] = du;
        cfp[k * LPR] = dp;
        cfn[k * LPR] = dn;
        if (a.cw != nullptr) {  // materialised reg rows (else the scatters form them, RegSrc)
            cwu[k * LPR] = make_float4(kreg * WU[k].x, kreg * WU[k].y, kreg * WU[k].z, kreg * WU[k].w);
            cwp[k * LPR] = make_float4(kreg * WP[k].x, kreg * WP[k].y, kreg * WP[k].z, kreg * WP[k].w);
            cwn[k * LPR] = make_float4(kreg * WN[k].x, kreg * WN[k].y, kreg * WN[k].z, kreg * WN[k].w);
        }
    }
    if (l == 0) {
        a.terms[b] = sp;
        a.terms[a.B + b] = sreg;
    }
}

constexpr int kLossBlock = 1024;
constexpr int kLossPartBlock = 256;

// Sums of t[0..n) and t[stride..stride+n) by one block of kLossBlock threads (each thread its
// strided terms in index order, loads issued 8 at a time, then the fixed wave/LDS tree), into the
// loss of B triplets. Run as its own launch (k_bpr_loss) or as the extra workgroup of the range
// scatter (k_range_scatter has the same block size): the same association either way.
__device__ __forceinline__ void bpr_loss_block(const float* __restrict__ t, int64_t n, int64_t stride, int64_t B,
                                               int32_t d, float coeff, float* __restrict__ loss,
                                               double* __restrict__ acc = nullptr, double w = 0.0) {
    __shared__ float r0[kLossBlock / 64], r1[kLossBlock / 64];
    float s0 = 0.f, s1 = 0.f;
    constexpr int kU = 8;
    int64_t i = threadIdx.x;
    for (; i + (kU - 1) * int64_t(kLossBlock) < n; i += kU * int64_t(kLossBlock)) {
        float a[kU], c[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            a[u] = t[i + u * int64_t(kLossBlock)];
            c[u] = t[stride + i + u * int64_t(kLossBlock)];
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            s0 += a[u];
            s1 += c[u];
        }
    }
    for (; i < n; i += kLossBlock) {
        s0 += t[i];
        s1 += t[stride + i];
    }
    for (int off = 32; off > 0; off >>= 1) {
        s0 += __shfl_down(s0, off, 64);
        s1 += __shfl_down(s1, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        r0[threadIdx.x >> 6] = s0;
        r1[threadIdx.x >> 6] = s1;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float a = 0.f, c = 0.f;
        for (int w = 0; w < kLossBlock / 64; ++w) {
            a += r0[w];
            c += r1[w];
        }
        const float bf = static_cast<float>(B);
        // -(mean softplus) / 10 + coeff * mean(squares); B == 0 gives NaN, as torch's empty mean
        const float l = -((a / bf) / 10.0f) + coeff * (c / (bf * static_cast<float>(d)));
        loss[0] = l;
        if (acc) {  // the harness's epoch sum, as k_loss_accumulate adds it (ABI 10)
            const double cw = static_cast<double>(l) * w;
            acc[0] = acc[0] + cw;
        }
    }
}

__global__ __launch_bounds__(kLossBlock) void k_bpr_loss(const float* __restrict__ t, int64_t n, int64_t stride,
                                                         int64_t B, int32_t d, float coeff, float* __restrict__ loss) {
    bpr_loss_block(t, n, stride, B, d, coeff, loss);
}

// the single-block loss sum as an extra workgroup of the range scatter (lgcn_range_scatter_add_loss)
struct LossArgs {
    const float* terms;
    int64_t B;
    int32_t d;
    float coeff;
    float* loss;
    double* acc;  // nullable: acc[0] += double(loss) * w in the same workgroup
    double w;
};

// First stage of the two-stage sum: block p sums its contiguous share of each term array (threads
// strided in index order, then the fixed wave/LDS tree) into part[p] and part[P + p].
__global__ __launch_bounds__(kLossPartBlock) void k_bpr_loss_part(const float* __restrict__ terms, int64_t B,
                                                                  float* __restrict__ part) {
    __shared__ float r0[kLossPartBlock / 64], r1[kLossPartBlock / 64];
    const int64_t P = gridDim.x;
    const int64_t per = (B + P - 1) / P;
    const int64_t lo = int64_t(blockIdx.x) * per;
    const int64_t hi = lo + per < B ? lo + per : B;
    float s0 = 0.f, s1 = 0.f;
    constexpr int kU = 4;
    int64_t i = lo + threadIdx.x;
    for (; i + (kU - 1) * int64_t(kLossPartBlock) < hi; i += kU * int64_t(kLossPartBlock)) {
        float a[kU], c[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            a[u] = terms[i + u * int64_t(kLossPartBlock)];
            c[u] = terms[B + i + u * int64_t(kLossPartBlock)];
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            s0 += a[u];
            s1 += c[u];
        }
    }
    for (; i < hi; i += kLossPartBlock) {
        s0 += terms[i];
        s1 += terms[B + i];
    }
    for (int off = 32; off > 0; off >>= 1) {
        s0 += __shfl_down(s0, off, 64);
        s1 += __shfl_down(s1, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        r0[threadIdx.x >> 6] = s0;
        r1[threadIdx.x >> 6] = s1;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float a = 0.f, c = 0.f;
        for (int w = 0; w < kLossPartBlock / 64; ++w) {
            a += r0[w];
            c += r1[w];
        }
        part[blockIdx.x] = a;
        part[P + blockIdx.x] = c;
    }
}

// out[r] = sum of C rows perm[rowptr[r] .. rowptr[r+1]) in order (add == 0: every row written,
// 0 for empty rows); add != 0: out[r] += that sum, rows without contributions untouched.
template <int LPR, int NV>
__global__ __launch_bounds__(kBlock) void k_segment_rows(const int64_t* __restrict__ rowptr,
                                                         const int32_t* __restrict__ perm,
                                                         const float* __restrict__ C, int64_t N, int32_t d,
                                                         float* out_lo, float* out_hi, int64_t split, int add,
                                                         float mul, float div) {
    constexpr int GPB = kBlock / LPR;
    const int g = threadIdx.x / LPR;
    const int l = threadIdx.x % LPR;
    const int64_t r = int64_t(blockIdx.x) * GPB + g;
    if (r >= N) return;
    const int64_t beg = rowptr[r], end = rowptr[r + 1];
    if (add && beg == end) return;
    float4 acc[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t e = beg; e < end; ++e) {
        const float4* c = reinterpret_cast<const float4*>(C + int64_t(perm[e]) * d) + l;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const float4 v = c[k * LPR];
            acc[k] = make_float4(acc[k].x + v.x, acc[k].y + v.y, acc[k].z + v.z, acc[k].w + v.w);
        }
    }
    float4* o = reinterpret_cast<float4*>(srow(out_lo, out_hi, split, r, int64_t(d))) + l;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        if (add) {
            const float4 v = o[k * LPR];
            acc[k] = make_float4(v.x + (acc[k].x * mul) / div, v.y + (acc[k].y * mul) / div,
                                 v.z + (acc[k].z * mul) / div, v.w + (acc[k].w * mul) / div);
        } else {
            acc[k] = make_float4((acc[k].x * mul) / div, (acc[k].y * mul) / div, (acc[k].z * mul) / div,
                                 (acc[k].w * mul) / div);
        }
        o[k * LPR] = acc[k];
    }
}

// ---- per-step scatter of the negatives' gradient rows (deterministic, no atomics) ----
// Range-owner scatter: workgroup w owns output rows [key_offset + w*span, ... + span). It streams
// all B keys in index order, keeps the ones in its range through an ORDERED block compaction
// (wave ballot + per-wave prefix), so its list is in b order, then every first occurrence of a row
// sums that row's C rows in list (= b) order and adds (sum * mul) / div to it. One launch,
// deterministic, no atomics; each workgroup reads the B keys once (L2-resident).
constexpr int kRangeCap = 4096;

constexpr int kRSBlock = 1024;          // 16 waves: more lane groups for the per-row sums
constexpr int kRSSpanTable = 2048;      // spans up to this many rows keep per-row tables in LDS
constexpr int kRSWaves = kRSBlock / 64;
constexpr int kRSChunks = 4;            // 64-key chunks per wave per round (coalesced)

template <int LPR, int NV>
__global__ __launch_bounds__(kRSBlock) void k_range_scatter(const int64_t* __restrict__ keys, int64_t B, int64_t nrows,
                                                            int64_t span, int64_t key_offset, const float* __restrict__ C,
                                                            int32_t d, float* out_lo, float* out_hi, int64_t split,
                                                            float mul, float div, const float* __restrict__ C2,
                                                            RegSrc reg,
                                                            float* __restrict__ c2buf, uint8_t* __restrict__ c2flag,
                                                            int* __restrict__ overflow,
                                                            const uint8_t* __restrict__ store_unless,
                                                            int32_t* __restrict__ reg_count, LossArgs la) {
    static_assert(kRSBlock == kLossBlock, "the loss workgroup needs the loss block's size (its association)");
    if (la.loss != nullptr && blockIdx.x == gridDim.x - 1) {
        bpr_loss_block(la.terms, la.B, la.B, la.B, la.d, la.coeff, la.loss, la.acc, la.w);
        return;
    }
    constexpr int GPB = kRSBlock / LPR;
    const bool second = C2 != nullptr || reg.w_lo != nullptr;  // a second (parked) sum per row
    // reg_count (ABI 10): each row's occurrence count instead of a parked sum (the clip norm and
    // the update form the reg rows from it); the flags are written either way
    const bool flags = second || reg_count != nullptr;
    __shared__ int lkey[kRangeCap];
    __shared__ int lidx[kRangeCap];
    __shared__ int wave_cnt[kRSWaves];
    __shared__ int list_n;
    // per row of the span (span <= kRSSpanTable): its first list entry and its entry count, so an
    // entry knows whether it is its row's first and, for the common single-occurrence row, needs
    // no scan of the list (the scans were the launch's critical path: profiles/r05zv_range_scatter/)
    __shared__ int lfirst[kRSSpanTable];
    __shared__ int lcount[kRSSpanTable];
    const bool tables = span <= kRSSpanTable;
    const int64_t lo = int64_t(blockIdx.x) * span;
    const int64_t hi = lo + span < nrows ? lo + span : nrows;
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int g = threadIdx.x / LPR;
    const int l = threadIdx.x % LPR;
    const unsigned long long below = (1ull << lane) - 1ull;
    if (reg_count)  // every row of the range: 0 unless it has keys (the barrier below orders the stores)
        for (int64_t i = lo + threadIdx.x; i < hi; i += kRSBlock) reg_count[i] = 0;
    if (threadIdx.x == 0) list_n = 0;
    __syncthreads();
    int64_t base = 0;
    constexpr int64_t kPerRound = int64_t(kRSBlock) * kRSChunks;  // <= kRangeCap: a round always fits an empty list
    static_assert(kPerRound <= kRangeCap, "a round must fit an empty list");
    // this round's keys (kv) are in registers before the round starts: the next round's are loaded
    // right after this round's ballots, so their latency overlaps the round's barriers and stores
    int64_t kv[kRSChunks];
    auto load_round = [&](int64_t b0, int64_t (&dst)[kRSChunks]) {
#pragma unroll
        for (int j = 0; j < kRSChunks; ++j) {
            const int64_t bj = b0 + (int64_t(wv) * kRSChunks + j) * 64 + lane;
            dst[j] = bj < B ? keys[bj] : -1;
        }
    };
    load_round(base, kv);
    while (true) {
        // fill the list in b order until full or all keys seen: wave w owns keys
        // [base + w*64*kRSChunks, +64*kRSChunks) of the round, chunk j at + j*64 + lane (coalesced);
        // order inside a wave comes from the ballot masks, across waves from the wave counts
        for (; base < B; base += kPerRound) {
            unsigned long long m[kRSChunks];
            int c = 0;
#pragma unroll
            for (int j = 0; j < kRSChunks; ++j) {
                const int64_t bj = base + (int64_t(wv) * kRSChunks + j) * 64 + lane;
                // keys no workgroup owns (outside [0, nrows)): workgroup 0 clears their flag
                if (flags && blockIdx.x == 0 && bj < B && (kv[j] < 0 || kv[j] >= nrows)) c2flag[bj] = 0;
            }
#pragma unroll
            for (int j = 0; j < kRSChunks; ++j) {
                m[j] = __ballot(kv[j] >= lo && kv[j] < hi);
                c += __popcll(m[j]);
            }
            int64_t kn[kRSChunks];
            load_round(base + kPerRound, kn);  // the next round's keys, in flight across the barriers
            if (lane == 0) wave_cnt[wv] = c;
            __syncthreads();
            int off = list_n;
            int total = list_n;
            for (int w = 0; w < kRSWaves; ++w) {
                const int cw = wave_cnt[w];
                if (w < wv) off += cw;
                total += cw;
            }
            if (total > kRangeCap) {  // this round does not fit: flush first, redo it (kv still holds it)
                if (threadIdx.x == 0 && overflow) *overflow = 1;  // C2 rows would then be split: report
                __syncthreads();
                break;
            }
#pragma unroll
            for (int j = 0; j < kRSChunks; ++j) {
                if ((m[j] >> lane) & 1ull) {
                    const int pos = off + __popcll(m[j] & below);
                    lkey[pos] = static_cast<int>(kv[j] - lo);
                    lidx[pos] = static_cast<int>(base + (int64_t(wv) * kRSChunks + j) * 64 + lane);
                }
                off += __popcll(m[j]);
            }
            __syncthreads();
            if (threadIdx.x == 0) list_n = total;
            __syncthreads();
#pragma unroll
            for (int j = 0; j < kRSChunks; ++j) kv[j] = kn[j];
        }
        // sum every row of the list in list order
        const int n = list_n;
        if (tables) {
            for (int i = threadIdx.x; i < span; i += kRSBlock) {
                lfirst[i] = INT_MAX;
                lcount[i] = 0;
            }
            __syncthreads();
            for (int e = threadIdx.x; e < n; e += kRSBlock) {
                atomicMin(&lfirst[lkey[e]], e);
                atomicAdd(&lcount[lkey[e]], 1);
            }
            __syncthreads();
        }
        for (int e = g; e < n; e += GPB) {
            const int key = lkey[e];
            bool first = true;
            if (tables) {
                first = lfirst[key] == e;
            } else {
                for (int q = 0; q < e; ++q)
                    if (lkey[q] == key) {
                        first = false;
                        break;
                    }
            }
            // every b is in exactly one list: its flag is written here (1 = the row's parked C2 sum)
            if (flags && l == 0) c2flag[lidx[e]] = first ? 1 : 0;
            if (!first) continue;
            float4 acc[NV], acc2[NV];
#pragma unroll
            for (int k = 0; k < NV; ++k) {
                acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
                acc2[k] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
            int64_t occ = 0;
            // a row with one entry sums just it; else the entries from e on, in list order
            const int q_end = (tables && lcount[key] == 1) ? e + 1 : n;
            for (int q = e; q < q_end; ++q) {
                if (lkey[q] != key) continue;
                ++occ;
                const float4* c = reinterpret_cast<const float4*>(C + int64_t(lidx[q]) * d) + l;
#pragma unroll
                for (int k = 0; k < NV; ++k) {
                    const float4 v = c[k * LPR];
                    acc[k] = make_float4(acc[k].x + v.x, acc[k].y + v.y, acc[k].z + v.z, acc[k].w + v.w);
                }
                if (C2) {
                    const float4* c2 = reinterpret_cast<const float4*>(C2 + int64_t(lidx[q]) * d) + l;
#pragma unroll
                    for (int k = 0; k < NV; ++k) {
                        const float4 v = c2[k * LPR];
                        acc2[k] = make_float4(acc2[k].x + v.x, acc2[k].y + v.y, acc2[k].z + v.z, acc2[k].w + v.w);
                    }
                }
            }
            const int64_t row = lo + key + key_offset;
            if (reg_count && l == 0) reg_count[lo + key] = static_cast<int32_t>(occ);
            if (second) {  // second source: park the row's sum in the slot of its first occurrence
                if (!C2) reg_sum<LPR, NV>(reg, row, d, occ, l, acc2);
                float4* cb = reinterpret_cast<float4*>(c2buf + int64_t(lidx[e]) * d) + l;
#pragma unroll
                for (int k = 0; k < NV; ++k) cb[k * LPR] = acc2[k];
            }
            float4* o = reinterpret_cast<float4*>(srow(out_lo, out_hi, split, row, int64_t(d))) + l;
            if (store_unless && !store_unless[row]) {  // row not written before: store
#pragma unroll
                for (int k = 0; k < NV; ++k)
                    o[k * LPR] = make_float4((acc[k].x * mul) / div, (acc[k].y * mul) / div, (acc[k].z * mul) / div,
                                             (acc[k].w * mul) / div);
            } else {
#pragma unroll
                for (int k = 0; k < NV; ++k) {
                    const float4 v = o[k * LPR];
                    o[k * LPR] = make_float4(v.x + (acc[k].x * mul) / div, v.y + (acc[k].y * mul) / div,
                                             v.z + (acc[k].z * mul) / div, v.w + (acc[k].w * mul) / div);
                }
            }
        }
        __syncthreads();
        if (base >= B) break;
        if (threadIdx.x == 0) list_n = 0;
        __syncthreads();
    }
}

// The same per-row work as k_range_scatter for large B (a structured graph's big Cluster-GCN
// batches: every k_range_scatter workgroup streams all B keys, so its cost grows as B^2): the keys
// come grouped by row, in b order, from one stable radix sort (lgcn_csr_build over the keys:
// rowptr[nrows+1], perm[B] = b). One lane group per row: flags (1 at the row's first b), the C and
// C2 sums in b order — the range scatter's association, so bitwise its result — the parked C2
// sum, and the (sum * mul) / div store or add.
template <int LPR, int NV>
__global__ __launch_bounds__(kBlock) void k_sorted_scatter(const int64_t* __restrict__ rowptr,
                                                           const int32_t* __restrict__ perm, int64_t nrows,
                                                           int64_t key_offset, const float* __restrict__ C, int32_t d,
                                                           float* out_lo, float* out_hi, int64_t split, float mul,
                                                           float div, const float* __restrict__ C2, RegSrc reg,
                                                           float* __restrict__ c2buf, uint8_t* __restrict__ c2flag,
                                                           const uint8_t* __restrict__ store_unless) {
    constexpr int GPB = kBlock / LPR;
    const bool second = C2 != nullptr || reg.w_lo != nullptr;
    const int g = threadIdx.x / LPR;
    const int l = threadIdx.x % LPR;
    const int64_t r = int64_t(blockIdx.x) * GPB + g;
    if (r >= nrows) return;
    const int64_t q0 = rowptr[r], q1 = rowptr[r + 1];
    if (q0 == q1) return;
    const int64_t first = perm[q0];
    if (c2flag)  // 1 at the row's first b (with or without a parked second sum)
        for (int64_t q = q0 + l; q < q1; q += LPR) c2flag[perm[q]] = (q == q0) ? 1 : 0;
    float4 acc[NV], acc2[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        acc2[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    int64_t q = q0;
    if (!C2) {
        // the row's C rows four at a time: loads issued together, added in b order (same sums)
        for (; q + 4 <= q1; q += 4) {
            float4 v[4][NV];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const float4* c = reinterpret_cast<const float4*>(C + int64_t(perm[q + u]) * d) + l;
#pragma unroll
                for (int k = 0; k < NV; ++k) v[u][k] = c[k * LPR];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int k = 0; k < NV; ++k)
                    acc[k] = make_float4(acc[k].x + v[u][k].x, acc[k].y + v[u][k].y, acc[k].z + v[u][k].z,
                                         acc[k].w + v[u][k].w);
        }
    }
    for (; q < q1; ++q) {
        const int64_t b = perm[q];
        const float4* c = reinterpret_cast<const float4*>(C + b * d) + l;
        float4 v[NV], v2[NV];
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k] = c[k * LPR];
        if (C2) {
            const float4* c2 = reinterpret_cast<const float4*>(C2 + b * d) + l;
#pragma unroll
            for (int k = 0; k < NV; ++k) v2[k] = c2[k * LPR];
        }
#pragma unroll
        for (int k = 0; k < NV; ++k) acc[k] = make_float4(acc[k].x + v[k].x, acc[k].y + v[k].y, acc[k].z + v[k].z, acc[k].w + v[k].w);
        if (C2) {
#pragma unroll
            for (int k = 0; k < NV; ++k)
                acc2[k] = make_float4(acc2[k].x + v2[k].x, acc2[k].y + v2[k].y, acc2[k].z + v2[k].z, acc2[k].w + v2[k].w);
        }
    }
    const int64_t row = r + key_offset;
    if (second) {
        if (!C2) reg_sum<LPR, NV>(reg, row, d, q1 - q0, l, acc2);
        float4* cb = reinterpret_cast<float4*>(c2buf + first * d) + l;
#pragma unroll
        for (int k = 0; k < NV; ++k) cb[k * LPR] = acc2[k];
    }
    float4* o = reinterpret_cast<float4*>(srow(out_lo, out_hi, split, row, int64_t(d))) + l;
    if (store_unless && !store_unless[row]) {
#pragma unroll
        for (int k = 0; k < NV; ++k)
            o[k * LPR] = make_float4((acc[k].x * mul) / div, (acc[k].y * mul) / div, (acc[k].z * mul) / div,
                                     (acc[k].w * mul) / div);
    } else {
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const float4 v = o[k * LPR];
            o[k * LPR] = make_float4(v.x + (acc[k].x * mul) / div, v.y + (acc[k].y * mul) / div,
                                     v.z + (acc[k].z * mul) / div, v.w + (acc[k].w * mul) / div);
        }
    }
}

// acc[0] += double(loss[0]) * w: the harness's epoch-loss sum (reference utils/train_test.py:101-103,
// total_loss += loss.item() * edges, in Python floats) with the same two double roundings (product,
// then sum; built without contraction), as one node of the batch's captured step.
__global__ void k_loss_accumulate(const float* __restrict__ loss, double w, double* __restrict__ acc) {
    if (threadIdx.x == 0) {
        const double c = static_cast<double>(loss[0]) * w;
        acc[0] = acc[0] + c;
    }
}

// Second pass for the parked sums: each flagged slot b adds c2buf[b] to row keys[b] + key_offset.
// Every row owns at most one flagged slot (its first occurrence) unless the scatter overflowed.
template <int LPR, int NV>
__global__ __launch_bounds__(kBlock) void k_flagged_rows_add(const int64_t* __restrict__ keys, int64_t B,
                                                             int64_t key_offset, const float* __restrict__ c2buf,
                                                             const uint8_t* __restrict__ c2flag, int32_t d,
                                                             float* out_lo, float* out_hi, int64_t split) {
    constexpr int GPB = kBlock / LPR;
    const int g = threadIdx.x / LPR;
    const int l = threadIdx.x % LPR;
    const int64_t b = int64_t(blockIdx.x) * GPB + g;
    if (b >= B || !c2flag[b]) return;
    const float4* c = reinterpret_cast<const float4*>(c2buf + b * d) + l;
    float4* o = reinterpret_cast<float4*>(srow(out_lo, out_hi, split, keys[b] + key_offset, int64_t(d))) + l;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const float4 v = o[k * LPR], a = c[k * LPR];
        o[k * LPR] = make_float4(v.x + a.x, v.y + a.y, v.z + a.z, v.w + a.w);
    }
}

template <int LPR, int NV>
int launch_rs(const int64_t* keys, int64_t B, int64_t nrows, int64_t key_offset, const float* C, int32_t d, float* lo,
              float* hi, int64_t split, float mul, float div, const float* C2, RegSrc reg, float* c2buf,
              uint8_t* c2flag, int* overflow, const uint8_t* store_unless, int32_t* reg_count, const LossArgs& la,
              hipStream_t s) {
    // every workgroup streams all B keys once; enough workgroups that each keeps ~<= 256 entries
    // on average (the list holds kRangeCap), at least 256 (one per CU)
    int64_t wgs = B / 256 + 1;
    if (wgs < 256) wgs = 256;
    if (wgs > 65535) wgs = 65535;
    if (wgs > nrows) wgs = nrows > 0 ? nrows : 1;
    const int64_t span = (nrows + wgs - 1) / wgs;
    const int64_t grid = (nrows + span - 1) / span + (la.loss != nullptr ? 1 : 0);  // + the loss workgroup
    k_range_scatter<LPR, NV><<<dim3(static_cast<unsigned>(grid)), kRSBlock, 0, s>>>(keys, B, nrows, span, key_offset, C, d,
                                                                                 lo, hi, split, mul, div, C2, reg,
                                                                                 c2buf, c2flag, overflow, store_unless,
                                                                                 reg_count, la);
    return check_launch("k_range_scatter");
}

template <int LPR, int NV>
int launch_ss(const int64_t* rowptr, const int32_t* perm, int64_t nrows, int64_t key_offset, const float* C, int32_t d,
              float* lo, float* hi, int64_t split, float mul, float div, const float* C2, RegSrc reg, float* c2buf,
              uint8_t* c2flag, const uint8_t* store_unless, hipStream_t s) {
    constexpr int GPB = kBlock / LPR;
    const int64_t blocks = (nrows + GPB - 1) / GPB;
    k_sorted_scatter<LPR, NV><<<dim3(static_cast<unsigned>(blocks)), kBlock, 0, s>>>(
        rowptr, perm, nrows, key_offset, C, d, lo, hi, split, mul, div, C2, reg, c2buf, c2flag, store_unless);
    return check_launch("k_sorted_scatter");
}

// Rows of a segment plan (rowptr over N rows, n contributions to row r): out[r] += n copies of
// kreg * W[r] summed in sequence — the fixed (user, positive) reg-gradient rows, added after the
// backward (reference utils/train_test.py:38-41 through autograd), without a [2B, d] table.
template <int LPR, int NV>
__global__ __launch_bounds__(kBlock) void k_reg_rows(const int64_t* __restrict__ rowptr, const int32_t* __restrict__ rows,
                                                     int64_t n_rows, RegSrc reg, int32_t d, float* out_lo,
                                                     float* out_hi, int64_t split, int64_t key_offset) {
    constexpr int GPB = kBlock / LPR;
    const int64_t i = int64_t(blockIdx.x) * GPB + threadIdx.x / LPR;
    const int l = threadIdx.x % LPR;
    if (i >= n_rows) return;
    const int64_t r = rows ? rows[i] : i;
    const int64_t n = rowptr[r + 1] - rowptr[r];
    if (n == 0) return;
    float4 acc[NV];
    reg_sum<LPR, NV>(reg, r + key_offset, d, n, l, acc);
    float4* o = reinterpret_cast<float4*>(srow(out_lo, out_hi, split, r + key_offset, int64_t(d))) + l;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const float4 v = o[k * LPR];
        o[k * LPR] = make_float4(v.x + acc[k].x, v.y + acc[k].y, v.z + acc[k].z, v.w + acc[k].w);
    }
}

template <int LPR, int NV>
int launch_reg(const int64_t* rowptr, const int32_t* rows, int64_t n_rows, RegSrc reg, int32_t d, float* lo, float* hi,
               int64_t split, hipStream_t s, int64_t key_offset = 0) {
    constexpr int GPB = kBlock / LPR;
    const int64_t blocks = (n_rows + GPB - 1) / GPB;
    if (blocks == 0) return LGCN_OK;
    k_reg_rows<LPR, NV><<<dim3(static_cast<unsigned>(blocks)), kBlock, 0, s>>>(rowptr, rows, n_rows, reg, d, lo, hi,
                                                                              split, key_offset);
    return check_launch("k_reg_rows");
}

template <int LPR, int NV>
int launch_fra(const int64_t* keys, int64_t B, int64_t key_offset, const float* c2buf, const uint8_t* c2flag, int32_t d,
               float* lo, float* hi, int64_t split, hipStream_t s) {
    constexpr int GPB = kBlock / LPR;
    const int64_t blocks = (B + GPB - 1) / GPB;
    if (blocks > 0)
        k_flagged_rows_add<LPR, NV><<<dim3(static_cast<unsigned>(blocks)), kBlock, 0, s>>>(keys, B, key_offset, c2buf,
                                                                                         c2flag, d, lo, hi, split);
    return check_launch("k_flagged_rows_add");
}

template <int LPR, int NV>
int launch_bpr(const BprArgs& a, int phase, hipStream_t s) {
    constexpr int GPB = kBlock / LPR;
    const int64_t blocks = (a.B + GPB - 1) / GPB;
    if (blocks > 0) {
        const dim3 grid(static_cast<unsigned>(blocks));
        const bool spec = a.touched != nullptr && a.B < kBprSpecMaxB;
        if (phase == kBprPartials) {
            if (spec) k_bpr_fused<LPR, NV, kBprPartials, true><<<grid, kBlock, 0, s>>>(a);
            else k_bpr_fused<LPR, NV, kBprPartials><<<grid, kBlock, 0, s>>>(a);
        } else if (phase == kBprFromSums) {
            if (spec) k_bpr_fused<LPR, NV, kBprFromSums, true><<<grid, kBlock, 0, s>>>(a);
            else k_bpr_fused<LPR, NV, kBprFromSums><<<grid, kBlock, 0, s>>>(a);
        } else {
            if (spec) k_bpr_fused<LPR, NV, kBprFused, true><<<grid, kBlock, 0, s>>>(a);
            else k_bpr_fused<LPR, NV, kBprFused><<<grid, kBlock, 0, s>>>(a);
        }
    }
    return check_launch("k_bpr_fused");
}

int bpr_dispatch(const BprArgs& a, int phase, hipStream_t s) {
    switch (a.d) {
        case 8: return launch_bpr<2, 1>(a, phase, s);
        case 16: return launch_bpr<4, 1>(a, phase, s);
        case 32: return launch_bpr<8, 1>(a, phase, s);
        case 64: return launch_bpr<16, 1>(a, phase, s);
        case 128: return launch_bpr<32, 1>(a, phase, s);
        case 256: return launch_bpr<64, 1>(a, phase, s);
        case 512: return launch_bpr<64, 2>(a, phase, s);
        default: return fail(LGCN_E_UNSUPPORTED, "lgcn_bpr_fused: d=%d (supported 8..512, powers of two)", a.d);
    }
}

template <int LPR, int NV>
int launch_seg(const int64_t* rowptr, const int32_t* perm, const float* C, int64_t N, int32_t d, float* lo, float* hi,
               int64_t split, int add, float mul, float div, hipStream_t s) {
    constexpr int GPB = kBlock / LPR;
    const int64_t blocks = (N + GPB - 1) / GPB;
    k_segment_rows<LPR, NV><<<dim3(static_cast<unsigned>(blocks)), kBlock, 0, s>>>(rowptr, perm, C, N, d, lo, hi,
                                                                                  split, add, mul, div);
    return check_launch("k_segment_rows");
}

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// lgcn_range_scatter_add(_loss): argument checks, then the width dispatch
int range_scatter(const int64_t* keys, int64_t B, int64_t nrows, int64_t key_offset, const float* C, int32_t d,
                  float* out_lo, float* out_hi, int64_t split, float mul, float div, const float* C2,
                  const float* reg_w_lo, const float* reg_w_hi, int64_t reg_w_split, float reg_coeff, int64_t reg_B,
                  float* c2buf, uint8_t* c2flag, int32_t* overflow, const uint8_t* store_unless, int32_t* reg_count,
                  const LossArgs& la, lgcn_stream_t stream) {
    const bool second = C2 != nullptr || reg_w_lo != nullptr;
    if (B < 0 || d <= 0 || nrows < 0 || (B > 0 && (!keys || !C || !out_lo)) || (second && (!c2buf || !c2flag)) ||
        (C2 && reg_w_lo) || (reg_count && (second || !c2flag)))
        return fail(LGCN_E_ARG, "lgcn_range_scatter_add: bad args");
    if (B == 0) return LGCN_OK;
    if (nrows == 0)  // no key is in range: nothing to add, every flag 0
        return (second || reg_count) ? check_hip(hipMemsetAsync(c2flag, 0, static_cast<size_t>(B), as_stream(stream)),
                                                 "memset c2flag")
                                     : LGCN_OK;
    if (d % 4 != 0 || !al16(C) || !al16(out_lo) || (out_hi && !al16(out_hi)) || (C2 && !al16(C2)) ||
        (second && !al16(c2buf)) || (reg_w_lo && (!al16(reg_w_lo) || (reg_w_hi && !al16(reg_w_hi)))))
        return fail(LGCN_E_UNSUPPORTED, "lgcn_range_scatter_add: needs d %% 4 == 0 and aligned rows");
    hipStream_t s = as_stream(stream);
    const RegSrc reg{reg_w_lo, reg_w_hi, reg_w_split, reg_coeff, reg_B};
#define LGCN_RS(L, V) launch_rs<L, V>(keys, B, nrows, key_offset, C, d, out_lo, out_hi, split, mul, div, C2, reg, c2buf, c2flag, overflow, store_unless, reg_count, la, s)
    switch (d) {
        case 8: return LGCN_RS(2, 1);
        case 16: return LGCN_RS(4, 1);
        case 32: return LGCN_RS(8, 1);
        case 64: return LGCN_RS(16, 1);
        case 128: return LGCN_RS(32, 1);
        case 256: return LGCN_RS(64, 1);
        case 512: return LGCN_RS(64, 2);
        default: return fail(LGCN_E_UNSUPPORTED, "lgcn_range_scatter_add: d=%d", d);
    }
#undef LGCN_RS
}
}  // namespace

extern "C" {

int lgcn_bpr_fused(const float* f_lo, const float* f_hi, int64_t f_split, const float* w_lo, const float* w_hi,
                   int64_t w_split, int64_t U, const int64_t* u, const int64_t* p, const int64_t* n, int64_t B,
                   int32_t d, const uint8_t* touched, float div, float mul, float coeff, float* cf, float* cw,
                   float* terms, lgcn_stream_t stream) {
    if (B < 0 || d <= 0 || U < 0) return fail(LGCN_E_ARG, "lgcn_bpr_fused: bad sizes");
    if (B == 0) return LGCN_OK;
    if (!f_lo || !w_lo || !u || !p || !n || !cf || !terms)
        return fail(LGCN_E_ARG, "lgcn_bpr_fused: null pointer");
    if (d % 4 != 0 || !al16(f_lo) || !al16(w_lo) || (f_hi && !al16(f_hi)) || (w_hi && !al16(w_hi)) || !al16(cf) ||
        (cw && !al16(cw)))
        return fail(LGCN_E_UNSUPPORTED, "lgcn_bpr_fused: needs d %% 4 == 0 and 16-byte aligned rows (d=%d)", d);
    BprArgs a{f_lo, f_hi, f_split, w_lo, w_hi, w_split, U, u, p, n, B, d, touched, div, mul, coeff, cf, cw, terms,
              nullptr, d};
    return bpr_dispatch(a, kBprFused, as_stream(stream));
}

int lgcn_bpr_fused_cols(const float* f_lo, const float* f_hi, int64_t f_split, const float* w_lo, const float* w_hi,
                        int64_t w_split, int64_t U, const int64_t* u, const int64_t* p, const int64_t* n, int64_t B,
                        int32_t d, int32_t d_full, const uint8_t* touched, float div, float mul, float coeff, float* sums,
                        int32_t phase, float* cf, float* cw, float* terms, lgcn_stream_t stream) {
    if (B < 0 || d <= 0 || d_full < d || U < 0 || (phase != kBprPartials && phase != kBprFromSums))
        return fail(LGCN_E_ARG, "lgcn_bpr_fused_cols: bad sizes or phase");
    if (B == 0) return LGCN_OK;
    if (!f_lo || !w_lo || !u || !p || !n || !sums || (phase == kBprFromSums && (!cf || !terms)))
        return fail(LGCN_E_ARG, "lgcn_bpr_fused_cols: null pointer");
    if (d % 4 != 0 || !al16(f_lo) || !al16(w_lo) || (f_hi && !al16(f_hi)) || (w_hi && !al16(w_hi)) ||
        (cf && !al16(cf)) || (cw && !al16(cw)))
        return fail(LGCN_E_UNSUPPORTED, "lgcn_bpr_fused_cols: needs d %% 4 == 0 and 16-byte aligned rows (d=%d)", d);
    BprArgs a{f_lo, f_hi, f_split, w_lo, w_hi, w_split, U, u, p, n, B, d, touched, div, mul, coeff, cf, cw, terms,
              sums, d_full};
    return bpr_dispatch(a, phase, as_stream(stream));
}

int lgcn_range_scatter_add(const int64_t* keys, int64_t B, int64_t nrows, int64_t key_offset, const float* C,
                           int32_t d, float* out_lo, float* out_hi, int64_t split, float mul, float div,
                           const float* C2, const float* reg_w_lo, const float* reg_w_hi, int64_t reg_w_split,
                           float reg_coeff, int64_t reg_B, float* c2buf, uint8_t* c2flag, int32_t* overflow,
                           const uint8_t* store_unless, lgcn_stream_t stream) {
    return range_scatter(keys, B, nrows, key_offset, C, d, out_lo, out_hi, split, mul, div, C2, reg_w_lo, reg_w_hi,
                         reg_w_split, reg_coeff, reg_B, c2buf, c2flag, overflow, store_unless, nullptr,
                         LossArgs{nullptr, 0, 0, 0.f, nullptr, nullptr, 0.0}, stream);
}

int lgcn_range_scatter_add_loss(const int64_t* keys, int64_t B, int64_t nrows, int64_t key_offset, const float* C,
                                int32_t d, float* out_lo, float* out_hi, int64_t split, float mul, float div,
                                const float* C2, const float* reg_w_lo, const float* reg_w_hi, int64_t reg_w_split,
                                float reg_coeff, int64_t reg_B, float* c2buf, uint8_t* c2flag, int32_t* overflow,
                                const uint8_t* store_unless, const float* terms, int64_t loss_B, int32_t loss_d,
                                float loss_coeff, float* loss, lgcn_stream_t stream) {
    if (!terms || !loss || loss_B < 1 || loss_d <= 0 || loss_B >= LGCN_LOSS_FUSED_MAX_B || B <= 0 || nrows <= 0)
        return fail(LGCN_E_ARG, "lgcn_range_scatter_add_loss: bad loss args (B=%lld; the single-block sum needs "
                    "1 <= B < %d, and a scatter with work)", (long long)loss_B, LGCN_LOSS_FUSED_MAX_B);
    return range_scatter(keys, B, nrows, key_offset, C, d, out_lo, out_hi, split, mul, div, C2, reg_w_lo, reg_w_hi,
                         reg_w_split, reg_coeff, reg_B, c2buf, c2flag, overflow, store_unless, nullptr,
                         LossArgs{terms, loss_B, loss_d, loss_coeff, loss, nullptr, 0.0}, stream);
}

int lgcn_range_scatter_add_counts(const int64_t* keys, int64_t B, int64_t nrows, int64_t key_offset, const float* C,
                                  int32_t d, float* out_lo, float* out_hi, int64_t split, float mul, float div,
                                  uint8_t* c2flag, int32_t* overflow, const uint8_t* store_unless, int32_t* reg_count,
                                  const float* terms, int64_t loss_B, int32_t loss_d, float loss_coeff, float* loss,
                                  double* loss_acc, double loss_w, lgcn_stream_t stream) {
    if (!c2flag || !reg_count) return fail(LGCN_E_ARG, "lgcn_range_scatter_add_counts: null c2flag / reg_count");
    if ((loss_acc && !terms) ||
        (terms && (!loss || loss_B < 1 || loss_d <= 0 || loss_B >= LGCN_LOSS_FUSED_MAX_B || B <= 0 || nrows <= 0)))
        return fail(LGCN_E_ARG, "lgcn_range_scatter_add_counts: bad loss args (B=%lld; the single-block sum needs "
                    "1 <= B < %d, and a scatter with work)", (long long)loss_B, LGCN_LOSS_FUSED_MAX_B);
    return range_scatter(keys, B, nrows, key_offset, C, d, out_lo, out_hi, split, mul, div, nullptr, nullptr, nullptr,
                         0, 0.f, 0, nullptr, c2flag, overflow, store_unless, reg_count,
                         terms ? LossArgs{terms, loss_B, loss_d, loss_coeff, loss, loss_acc, loss_w}
                               : LossArgs{nullptr, 0, 0, 0.f, nullptr, nullptr, 0.0},
                         stream);
}


int lgcn_sorted_scatter_add(const int64_t* rowptr, const int32_t* perm, int64_t nrows, int64_t key_offset,
                            const float* C, int32_t d, float* out_lo, float* out_hi, int64_t split, float mul,
                            float div, const float* C2, const float* reg_w_lo, const float* reg_w_hi,
                            int64_t reg_w_split, float reg_coeff, int64_t reg_B, float* c2buf, uint8_t* c2flag,
                            const uint8_t* store_unless, lgcn_stream_t stream) {
    const bool second = C2 != nullptr || reg_w_lo != nullptr;
    if (nrows < 0 || d <= 0 || (nrows > 0 && (!rowptr || !perm || !C || !out_lo)) || (second && (!c2buf || !c2flag)) ||
        (C2 && reg_w_lo))
        return fail(LGCN_E_ARG, "lgcn_sorted_scatter_add: bad args");
    if (nrows == 0) return LGCN_OK;
    if (d % 4 != 0 || !al16(C) || !al16(out_lo) || (out_hi && !al16(out_hi)) || (C2 && !al16(C2)) ||
        (second && !al16(c2buf)) || (reg_w_lo && (!al16(reg_w_lo) || (reg_w_hi && !al16(reg_w_hi)))))
        return fail(LGCN_E_UNSUPPORTED, "lgcn_sorted_scatter_add: needs d %% 4 == 0 and aligned rows");
    hipStream_t s = as_stream(stream);
    const RegSrc reg{reg_w_lo, reg_w_hi, reg_w_split, reg_coeff, reg_B};
#define LGCN_SS(L, V) launch_ss<L, V>(rowptr, perm, nrows, key_offset, C, d, out_lo, out_hi, split, mul, div, C2, reg, c2buf, c2flag, store_unless, s)
    switch (d) {
        case 8: return LGCN_SS(2, 1);
        case 16: return LGCN_SS(4, 1);
        case 32: return LGCN_SS(8, 1);
        case 64: return LGCN_SS(16, 1);
        case 128: return LGCN_SS(32, 1);
        case 256: return LGCN_SS(64, 1);
        case 512: return LGCN_SS(64, 2);
        default: return fail(LGCN_E_UNSUPPORTED, "lgcn_sorted_scatter_add: d=%d", d);
    }
#undef LGCN_SS
}

int lgcn_grouped_reg_add(const int64_t* rowptr, int64_t nrows, int64_t key_offset, const float* w_lo,
                         const float* w_hi, int64_t w_split, int32_t d, float coeff, int64_t B, float* out_lo,
                         float* out_hi, int64_t split, lgcn_stream_t stream) {
    if (nrows < 0 || d <= 0 || B < 0 || key_offset < 0 || (nrows > 0 && (!rowptr || !w_lo || !out_lo)))
        return fail(LGCN_E_ARG, "lgcn_grouped_reg_add: bad args");
    if (nrows == 0) return LGCN_OK;
    if (d % 4 != 0 || !al16(w_lo) || (w_hi && !al16(w_hi)) || !al16(out_lo) || (out_hi && !al16(out_hi)))
        return fail(LGCN_E_UNSUPPORTED, "lgcn_grouped_reg_add: needs d %% 4 == 0 and aligned rows");
    hipStream_t s = as_stream(stream);
    const RegSrc reg{w_lo, w_hi, w_split, coeff, B};
#define LGCN_GR(L, V) launch_reg<L, V>(rowptr, nullptr, nrows, reg, d, out_lo, out_hi, split, s, key_offset)
    switch (d) {
        case 8: return LGCN_GR(2, 1);
        case 16: return LGCN_GR(4, 1);
        case 32: return LGCN_GR(8, 1);
        case 64: return LGCN_GR(16, 1);
        case 128: return LGCN_GR(32, 1);
        case 256: return LGCN_GR(64, 1);
        case 512: return LGCN_GR(64, 2);
        default: return fail(LGCN_E_UNSUPPORTED, "lgcn_grouped_reg_add: d=%d", d);
    }
#undef LGCN_GR
}

int lgcn_reg_rows_add(const int64_t* rowptr, const int32_t* rows, int64_t n_rows, const float* w_lo, const float* w_hi,
                      int64_t w_split, int32_t d, float coeff, int64_t B, float* out_lo, float* out_hi, int64_t split,
                      lgcn_stream_t stream) {
    if (n_rows < 0 || d <= 0 || B < 0 || (n_rows > 0 && (!rowptr || !w_lo || !out_lo)))
        return fail(LGCN_E_ARG, "lgcn_reg_rows_add: bad args");
    if (n_rows == 0) return LGCN_OK;
    if (d % 4 != 0 || !al16(w_lo) || (w_hi && !al16(w_hi)) || !al16(out_lo) || (out_hi && !al16(out_hi)))
        return fail(LGCN_E_UNSUPPORTED, "lgcn_reg_rows_add: needs d %% 4 == 0 and aligned rows");
    hipStream_t s = as_stream(stream);
    const RegSrc reg{w_lo, w_hi, w_split, coeff, B};
    switch (d) {
        case 8: return launch_reg<2, 1>(rowptr, rows, n_rows, reg, d, out_lo, out_hi, split, s);
        case 16: return launch_reg<4, 1>(rowptr, rows, n_rows, reg, d, out_lo, out_hi, split, s);
        case 32: return launch_reg<8, 1>(rowptr, rows, n_rows, reg, d, out_lo, out_hi, split, s);
        case 64: return launch_reg<16, 1>(rowptr, rows, n_rows, reg, d, out_lo, out_hi, split, s);
        case 128: return launch_reg<32, 1>(rowptr, rows, n_rows, reg, d, out_lo, out_hi, split, s);
        case 256: return launch_reg<64, 1>(rowptr, rows, n_rows, reg, d, out_lo, out_hi, split, s);
        case 512: return launch_reg<64, 2>(rowptr, rows, n_rows, reg, d, out_lo, out_hi, split, s);
        default: return fail(LGCN_E_UNSUPPORTED, "lgcn_reg_rows_add: d=%d", d);
    }
}

int lgcn_flagged_rows_add(const int64_t* keys, int64_t B, int64_t key_offset, const float* c2buf, const uint8_t* c2flag,
                          int32_t d, float* out_lo, float* out_hi, int64_t split, lgcn_stream_t stream) {
    if (B < 0 || d <= 0 || (B > 0 && (!keys || !c2buf || !c2flag || !out_lo))) return fail(LGCN_E_ARG, "lgcn_flagged_rows_add: bad args");
    if (B == 0) return LGCN_OK;
    hipStream_t s = as_stream(stream);
#define LGCN_FRA(L, V) launch_fra<L, V>(keys, B, key_offset, c2buf, c2flag, d, out_lo, out_hi, split, s)
    switch (d) {
        case 8: return LGCN_FRA(2, 1);
        case 16: return LGCN_FRA(4, 1);
        case 32: return LGCN_FRA(8, 1);
        case 64: return LGCN_FRA(16, 1);
        case 128: return LGCN_FRA(32, 1);
        case 256: return LGCN_FRA(64, 1);
        case 512: return LGCN_FRA(64, 2);
        default: return fail(LGCN_E_UNSUPPORTED, "lgcn_flagged_rows_add: d=%d", d);
    }
#undef LGCN_FRA
}

int lgcn_bpr_loss(const float* terms, int64_t B, int32_t d, float coeff, float* loss, float* partial,
                  lgcn_stream_t stream) {
    if (B < 0 || !loss || (B > 0 && !terms)) return fail(LGCN_E_ARG, "lgcn_bpr_loss: bad args");
    hipStream_t s = as_stream(stream);
    // large batches: LGCN_LOSS_PARTS blocks sum contiguous shares, one block sums the shares
    // (a single block over 2B terms is latency-bound: 26 us at B = 180k)
    static_assert(LGCN_LOSS_FUSED_MAX_B == 16 * LGCN_LOSS_PARTS * kLossPartBlock / 64,
                  "the fused loss covers exactly the single-block sizes");
    if (partial != nullptr && B >= LGCN_LOSS_FUSED_MAX_B) {
        k_bpr_loss_part<<<LGCN_LOSS_PARTS, kLossPartBlock, 0, s>>>(terms, B, partial);
        if (int rc = check_launch("k_bpr_loss_part")) return rc;
        k_bpr_loss<<<1, kLossBlock, 0, s>>>(partial, LGCN_LOSS_PARTS, LGCN_LOSS_PARTS, B, d, coeff, loss);
        return check_launch("k_bpr_loss");
    }
    k_bpr_loss<<<1, kLossBlock, 0, s>>>(terms, B, B, B, d, coeff, loss);
    return check_launch("k_bpr_loss");
}

int lgcn_loss_accumulate(const float* loss, double w, double* acc, lgcn_stream_t stream) {
    if (!loss || !acc) return fail(LGCN_E_ARG, "lgcn_loss_accumulate: null pointer");
    k_loss_accumulate<<<1, 64, 0, as_stream(stream)>>>(loss, w, acc);
    return check_launch("k_loss_accumulate");
}

int lgcn_segment_rows(const int64_t* rowptr, const int32_t* perm, const float* C, int64_t N, int32_t d,
                      float* out_lo, float* out_hi, int64_t split, int32_t add, float mul, float div,
                      lgcn_stream_t stream) {
    if (N < 0 || d <= 0 || !rowptr || !out_lo || (split < N && !out_hi)) return fail(LGCN_E_ARG, "lgcn_segment_rows: bad args");
    if (N == 0) return LGCN_OK;
    if (d % 4 != 0 || !al16(out_lo) || (out_hi && !al16(out_hi)) || (C && !al16(C)))
        return fail(LGCN_E_UNSUPPORTED, "lgcn_segment_rows: needs d %% 4 == 0 and aligned rows");
    hipStream_t s = as_stream(stream);
    switch (d) {
        case 8: return launch_seg<2, 1>(rowptr, perm, C, N, d, out_lo, out_hi, split, add, mul, div, s);
        case 16: return launch_seg<4, 1>(rowptr, perm, C, N, d, out_lo, out_hi, split, add, mul, div, s);
        case 32: return launch_seg<8, 1>(rowptr, perm, C, N, d, out_lo, out_hi, split, add, mul, div, s);
        case 64: return launch_seg<16, 1>(rowptr, perm, C, N, d, out_lo, out_hi, split, add, mul, div, s);
        case 128: return launch_seg<32, 1>(rowptr, perm, C, N, d, out_lo, out_hi, split, add, mul, div, s);
        case 256: return launch_seg<64, 1>(rowptr, perm, C, N, d, out_lo, out_hi, split, add, mul, div, s);
        case 512: return launch_seg<64, 2>(rowptr, perm, C, N, d, out_lo, out_hi, split, add, mul, div, s);
        default: return fail(LGCN_E_UNSUPPORTED, "lgcn_segment_rows: d=%d (supported 16..512, powers of two)", d);
    }
}

}  // extern "C"
