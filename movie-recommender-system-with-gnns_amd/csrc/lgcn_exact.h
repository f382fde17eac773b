// Shortened forms of the correctly rounded fp32 sqrt and division that hipcc emits for sqrtf(x)
// and a / b on gfx950 (fp32 denormals on), exact on stated input ranges: the instructions they
// drop are the ones that only act outside those ranges, so inside them the results are bitwise
// the full sequences' — checked exhaustively for sqrt_normal (every fp32 input in its range) and
// on 2^32 random + boundary pairs for div_window by tools/exact_math_check.hip
// (profiles/r05t_adam_fast/).
//
// Used by the row-lazy Adam's zero-gradient replays (lgcn_rowadam.hip), which are bound by VALU
// issue: per element and replayed step the full sqrt is 16 instructions and the division 11, of
// about 30 (tools/adam_replay_probe.hip).
#pragma once

#include <hip/hip_runtime.h>

namespace lgcn {

// sqrtf(x) for x == +0 or 2^-96 <= x <= FLT_MAX. The full sequence first scales x < 2^-96 by 2^32
// (and the root back by 2^-16) and finally returns +-0 / +inf unchanged (v_cmp_class 0x260); in
// this range neither acts. What remains: v_sqrt_f32's estimate s, moved to s - 1 ulp if the
// residual x - (s - 1ulp) s <= 0, or to s + 1 ulp if x - (s + 1ulp) s > 0. For x = +0: s = 0, the
// first residual is NaN (s - 1ulp is a NaN pattern), the second +0, so +0 is returned.
__device__ __forceinline__ float sqrt_normal(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sd = __int_as_float(__float_as_int(s) - 1), su = __int_as_float(__float_as_int(s) + 1);
    const float t = __builtin_fmaf(-sd, s, x) <= 0.0f ? sd : s;
    return __builtin_fmaf(-su, s, x) > 0.0f ? su : t;
}

// a / b for a == +0 or 2^-40 <= |a| <= 2^40, and 2^-40 <= b <= 2^40. v_div_scale leaves such
// operands unscaled (no denormal operand, reciprocal or quotient; exponent gap < 96; numerator
// exponent > 23), so v_div_fmas is a plain FMA, and v_div_fixup returns its input for a finite
// normal (or +0) quotient. What remains: v_rcp_f32, one Newton step on the reciprocal, the
// quotient and two residual corrections.
__device__ __forceinline__ float div_window(float a, float b) {
    const float r = __builtin_amdgcn_rcpf(b);
    const float r1 = __builtin_fmaf(__builtin_fmaf(-b, r, 1.0f), r, r);
    const float q = a * r1;
    const float q1 = __builtin_fmaf(__builtin_fmaf(-b, q, a), r1, q);
    return __builtin_fmaf(__builtin_fmaf(-b, q1, a), r1, q1);
}

}  // namespace lgcn
