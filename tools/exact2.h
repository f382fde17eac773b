// Two-element (packed) forms of the correctly rounded fp32 sqrt and division that hipcc emits for
// sqrtf(x) and a / b on gfx950 (fp32 denormals on, -ffp-contract=off): the same instruction
// sequences, with the two elements' independent multiplies and FMAs issued as one v_pk_mul_f32 /
// v_pk_fma_f32 each. Every packed op is the same IEEE operation per element, so the results are
// bitwise the compiler's — checked exhaustively for sqrt (all 2^32 inputs) and on 2^32 random,
// 16k special and 2^29 Adam-range pairs for the division by tools/exact_math_check.hip.
//
// Written for the row-lazy Adam's zero-gradient replays (csrc/lgcn_rowadam.hip) and measured there
// by tools/adam_replay_probe.hip: no faster than the scalar code (profiles/r05s_adam_replay/), so
// the library keeps the scalar element update; this header serves the two tools only.
#pragma once

#include <hip/hip_runtime.h>

namespace lgcn {

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 f2_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

__device__ __forceinline__ f2 f2_step_ulp(f2 s, int k) {
    return f2{__int_as_float(__float_as_int(s.x) + k), __int_as_float(__float_as_int(s.y) + k)};
}

// sqrtf(x) per element: inputs below 2^-96 are scaled by 2^32 (result by 2^-16), v_sqrt_f32's
// estimate s is moved to s - 1 ulp if the residual x - (s - 1ulp) * s <= 0, or to s + 1 ulp if
// x - (s + 1ulp) * s > 0, and +-0 / +inf return themselves (v_cmp_class mask 0x260).
__device__ __forceinline__ f2 sqrt2(f2 x) {
    const bool sx = x.x < 0x1p-96f, sy = x.y < 0x1p-96f;
    const f2 xs = x * 0x1p32f;
    const f2 xp{sx ? xs.x : x.x, sy ? xs.y : x.y};
    const f2 s{__builtin_amdgcn_sqrtf(xp.x), __builtin_amdgcn_sqrtf(xp.y)};
    const f2 sd = f2_step_ulp(s, -1), su = f2_step_ulp(s, 1);
    const f2 rd = f2_fma(-sd, s, xp);
    const f2 ru = f2_fma(-su, s, xp);
    f2 t{rd.x <= 0.0f ? sd.x : s.x, rd.y <= 0.0f ? sd.y : s.y};
    t = f2{ru.x > 0.0f ? su.x : t.x, ru.y > 0.0f ? su.y : t.y};
    const f2 ts = t * 0x1p-16f;
    t = f2{sx ? ts.x : t.x, sy ? ts.y : t.y};
    return f2{__builtin_amdgcn_classf(xp.x, 0x260) ? xp.x : t.x, __builtin_amdgcn_classf(xp.y, 0x260) ? xp.y : t.y};
}

// a / b per element: v_div_scale of both operands, v_rcp_f32, two Newton steps on the reciprocal
// and the quotient, v_div_fmas (undoes the scaling), v_div_fixup (specials).
__device__ __forceinline__ f2 div2(f2 a, f2 b) {
    bool fx, fy, qx, qy;
    const f2 ds{__builtin_amdgcn_div_scalef(a.x, b.x, false, &fx), __builtin_amdgcn_div_scalef(a.y, b.y, false, &fy)};
    const f2 ns{__builtin_amdgcn_div_scalef(a.x, b.x, true, &qx), __builtin_amdgcn_div_scalef(a.y, b.y, true, &qy)};
    const f2 r{__builtin_amdgcn_rcpf(ds.x), __builtin_amdgcn_rcpf(ds.y)};
    const f2 e = f2_fma(-ds, r, f2{1.0f, 1.0f});
    const f2 r1 = f2_fma(e, r, r);
    const f2 q = ns * r1;
    const f2 e2 = f2_fma(-ds, q, ns);
    const f2 q1 = f2_fma(e2, r1, q);
    const f2 e3 = f2_fma(-ds, q1, ns);
    const f2 fm{__builtin_amdgcn_div_fmasf(e3.x, r1.x, q1.x, qx), __builtin_amdgcn_div_fmasf(e3.y, r1.y, q1.y, qy)};
    return f2{__builtin_amdgcn_div_fixupf(fm.x, b.x, a.x), __builtin_amdgcn_div_fixupf(fm.y, b.y, a.y)};
}

}  // namespace lgcn
