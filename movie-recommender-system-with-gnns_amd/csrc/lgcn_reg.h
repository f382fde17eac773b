// The BPR loss's reg-gradient rows (reference utils/train_test.py:38-41: reg = coeff * mean(eu^2 +
// ep^2 + en^2) over the layer-0 rows, differentiated by autograd) — one definition for every kernel
// that forms them, so every path adds the same floats:
//   every occurrence of row r in a batch's 3B (user, positive, negative) keys contributes
//   kreg * W[r], kreg = coeff * 2 / (B * d) (the k_bpr_fused expression), and a row's n
//   occurrences are summed in sequence from 0; the (user, positive) copies are added to the row's
//   gradient first, the negatives' copies after them.
// lgcn_bpr.hip's scatters park or add them after the backward; lgcn_rowadam.hip's clip norm and
// update form them on the fly from the row counts (RegRows) instead (ABI 10).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace lgcn {

__device__ __forceinline__ float reg_scale(float coeff, int64_t B, int32_t d) {
    return coeff * 2.0f / (static_cast<float>(B) * static_cast<float>(d));
}

// ((0 + v) + v) + ... n times, v = kreg * x
__device__ __forceinline__ float4 reg_copies(float4 x, float kreg, int64_t n) {
    const float4 v = make_float4(kreg * x.x, kreg * x.y, kreg * x.z, kreg * x.w);
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t i = 0; i < n; ++i) s = make_float4(s.x + v.x, s.y + v.y, s.z + v.z, s.w + v.w);
    return s;
}

// A step's reg rows by their occurrence counts (lgcn_reg_rows_t of include/lgcn.h).
struct RegRows {
    const float* w_lo;  // nullptr: no reg rows
    const float* w_hi;
    int64_t w_split;
    float coeff;
    int64_t B;
    const int64_t* fixed_rowptr;  // [N + 1] (user, positive) occurrences per global row, or nullptr
    const int64_t* neg_rowptr;    // [neg_rows + 1] grouped negatives, or nullptr ...
    const int32_t* neg_count;     // ... [neg_rows] occurrences per row
    int64_t neg_off;
    int64_t neg_rows;
};

__device__ __forceinline__ void reg_counts(const RegRows& R, int64_t row, int64_t& nf, int64_t& nn) {
    nf = R.fixed_rowptr ? R.fixed_rowptr[row + 1] - R.fixed_rowptr[row] : 0;
    nn = 0;
    const int64_t r = row - R.neg_off;
    if (r >= 0 && r < R.neg_rows) nn = R.neg_rowptr ? R.neg_rowptr[r + 1] - R.neg_rowptr[r] : R.neg_count[r];
}

// g + (nf copies) + (nn copies), each sum added only when it has copies: the additions the
// separate after-backward passes made, in their order
__device__ __forceinline__ float4 reg_apply(float4 g, float4 w, float kreg, int64_t nf, int64_t nn) {
    if (nf > 0) {
        const float4 s = reg_copies(w, kreg, nf);
        g = make_float4(g.x + s.x, g.y + s.y, g.z + s.z, g.w + s.w);
    }
    if (nn > 0) {
        const float4 s = reg_copies(w, kreg, nn);
        g = make_float4(g.x + s.x, g.y + s.y, g.z + s.z, g.w + s.w);
    }
    return g;
}

}  // namespace lgcn
