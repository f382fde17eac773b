// What bounds the row-lazy Adam's zero-gradient replays (k_row_adam's catch-up loop): the replay
// of R missed steps on n rows of d = 128, timed for the scalar element code (round 4), the packed
// pairs of tools/exact2.h, the packed code with two float4 per lane (twice the independent chains),
// and the packed code with a division that skips v_div_scale / v_div_fmas / v_div_fixup inside an
// exponent window. Every variant's output is checked bitwise against the scalar one. Result
// (profiles/r05s_adam_replay/): all four run at the same 0.9-1.15e12 element-steps/s, so none of
// instruction count, packing, ILP or the division's helper instructions is what bounds the loop.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off \
//       -Itools tools/adam_replay_probe.hip -o tools/_bin/adam_replay_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

#include "exact2.h"

using lgcn::f2;

struct K {
    float omb1, beta2, eps;
};

__device__ __forceinline__ float div_step(float s, float c, float rc) {
    const float q0 = s * rc;
    return __builtin_fmaf(__builtin_fmaf(-c, q0, s), rc, q0);
}

__device__ __forceinline__ void zero1(float& p, float& m, float& v, float ss, float c, float rc, const K& k) {
    m = m - k.omb1 * m;
    v = v * k.beta2;
    const float denom = div_step(sqrtf(v), c, rc) + k.eps;
    p = p + ss * (m / denom);
}

__device__ __forceinline__ void zero2(f2& p, f2& m, f2& v, float ss, float c, float rc, const K& k) {
    m = m - k.omb1 * m;
    v = v * k.beta2;
    const f2 s = lgcn::sqrt2(v);
    const f2 q0 = s * rc;
    const f2 denom = lgcn::f2_fma(lgcn::f2_fma(f2{-c, -c}, q0, s), f2{rc, rc}, q0) + k.eps;
    p = p + ss * lgcn::div2(m, denom);
}

// the division without v_div_scale / v_div_fmas / v_div_fixup where they change nothing: every
// operand's exponent within 2^+-40 of 1 (no operand scaling, a normal quotient, no special case);
// other lanes take the full sequence
__device__ __forceinline__ bool window2(f2 a, f2 b) {
    const unsigned e0 = __builtin_amdgcn_ubfe(__float_as_uint(a.x), 23, 8), e1 = __builtin_amdgcn_ubfe(__float_as_uint(a.y), 23, 8);
    const unsigned e2 = __builtin_amdgcn_ubfe(__float_as_uint(b.x), 23, 8), e3 = __builtin_amdgcn_ubfe(__float_as_uint(b.y), 23, 8);
    const unsigned lo = min(min(e0, e1), min(e2, e3)), hi = max(max(e0, e1), max(e2, e3));
    return lo >= 87u && hi <= 167u;
}

__device__ __forceinline__ f2 div2_fast(f2 a, f2 b) {
    if (!window2(a, b)) return lgcn::div2(a, b);
    const f2 r{__builtin_amdgcn_rcpf(b.x), __builtin_amdgcn_rcpf(b.y)};
    const f2 e = lgcn::f2_fma(-b, r, f2{1.0f, 1.0f});
    const f2 r1 = lgcn::f2_fma(e, r, r);
    const f2 q = a * r1;
    const f2 e2 = lgcn::f2_fma(-b, q, a);
    const f2 q1 = lgcn::f2_fma(e2, r1, q);
    const f2 e3 = lgcn::f2_fma(-b, q1, a);
    return lgcn::f2_fma(e3, r1, q1);
}

__device__ __forceinline__ void zero3(f2& p, f2& m, f2& v, float ss, float c, float rc, const K& k) {
    m = m - k.omb1 * m;
    v = v * k.beta2;
    const f2 s = lgcn::sqrt2(v);
    const f2 q0 = s * rc;
    const f2 denom = lgcn::f2_fma(lgcn::f2_fma(f2{-c, -c}, q0, s), f2{rc, rc}, q0) + k.eps;
    p = p + ss * div2_fast(m, denom);
}

// diagnostics (not exact): 4 = scalar without the sqrt (denominator from v itself), 5 = scalar
// without the division (p += ss * m * denom), 6 = scalar with v_sqrt_f32's estimate and its two
// residual corrections only (no scaling or class fix-ups)
__device__ __forceinline__ float sqrt_lite(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sd = __int_as_float(__float_as_int(s) - 1), su = __int_as_float(__float_as_int(s) + 1);
    float t = __builtin_fmaf(-sd, s, x) <= 0.0f ? sd : s;
    return __builtin_fmaf(-su, s, x) > 0.0f ? su : t;
}

template <int D>
__device__ __forceinline__ void zero_diag(float& p, float& m, float& v, float ss, float c, float rc, const K& k) {
    m = m - k.omb1 * m;
    v = v * k.beta2;
    const float sq = D == 4 ? v : D == 6 ? sqrt_lite(v) : sqrtf(v);
    const float denom = div_step(sq, c, rc) + k.eps;
    p = p + ss * (D == 5 ? m * denom : m / denom);
}

// VARIANT 0: scalar, one float4 per lane (32 lanes per row); 1: packed pairs, one float4 per lane;
// 2: packed pairs, two float4 per lane (16 lanes per row, 2x the independent chains per lane);
// 3: packed pairs with the windowed division
template <int VARIANT>
__global__ __launch_bounds__(256) void k_replay(float4* P, float4* M, float4* V, const float4* consts, int n, int R,
                                                K k) {
    constexpr int NV = VARIANT == 2 ? 2 : 1;
    constexpr int LPR = 32 / NV;
    const int row = (blockIdx.x * 256 + threadIdx.x) / LPR;
    const int l = threadIdx.x % LPR;
    if (row >= n) return;
    float4* pp = P + int64_t(row) * 32 + l;
    float4* mm = M + int64_t(row) * 32 + l;
    float4* vv = V + int64_t(row) * 32 + l;
    float4 p[NV], m[NV], v[NV];
#pragma unroll
    for (int q = 0; q < NV; ++q) {
        p[q] = pp[q * LPR];
        m[q] = mm[q * LPR];
        v[q] = vv[q * LPR];
    }
    for (int s = 1; s <= R; ++s) {
        const float4 c = consts[s];
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            if constexpr (VARIANT >= 4) {
                zero_diag<VARIANT>(p[q].x, m[q].x, v[q].x, c.x, c.y, c.z, k);
                zero_diag<VARIANT>(p[q].y, m[q].y, v[q].y, c.x, c.y, c.z, k);
                zero_diag<VARIANT>(p[q].z, m[q].z, v[q].z, c.x, c.y, c.z, k);
                zero_diag<VARIANT>(p[q].w, m[q].w, v[q].w, c.x, c.y, c.z, k);
            } else if constexpr (VARIANT == 0) {
                zero1(p[q].x, m[q].x, v[q].x, c.x, c.y, c.z, k);
                zero1(p[q].y, m[q].y, v[q].y, c.x, c.y, c.z, k);
                zero1(p[q].z, m[q].z, v[q].z, c.x, c.y, c.z, k);
                zero1(p[q].w, m[q].w, v[q].w, c.x, c.y, c.z, k);
            } else {
                f2 p0{p[q].x, p[q].y}, p1{p[q].z, p[q].w}, m0{m[q].x, m[q].y}, m1{m[q].z, m[q].w};
                f2 v0{v[q].x, v[q].y}, v1{v[q].z, v[q].w};
                if constexpr (VARIANT == 3) {
                    zero3(p0, m0, v0, c.x, c.y, c.z, k);
                    zero3(p1, m1, v1, c.x, c.y, c.z, k);
                } else {
                    zero2(p0, m0, v0, c.x, c.y, c.z, k);
                    zero2(p1, m1, v1, c.x, c.y, c.z, k);
                }
                p[q] = make_float4(p0.x, p0.y, p1.x, p1.y);
                m[q] = make_float4(m0.x, m0.y, m1.x, m1.y);
                v[q] = make_float4(v0.x, v0.y, v1.x, v1.y);
            }
        }
    }
#pragma unroll
    for (int q = 0; q < NV; ++q) {
        pp[q * LPR] = p[q];
        mm[q * LPR] = m[q];
        vv[q * LPR] = v[q];
    }
}

int main(int argc, char** argv) {
    const int n_max = 200000;
    const size_t elems = size_t(n_max) * 128;
    std::vector<float> h0(elems), hm(elems), hv(elems);
    uint64_t x = 88172645463325252ull;
    auto rnd = [&]() {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        return float((x >> 40) & 0xffffff) / float(1 << 24);
    };
    for (size_t i = 0; i < elems; ++i) {
        h0[i] = (rnd() - 0.5f) * 0.2f;
        hm[i] = (rnd() - 0.5f) * 1e-3f;
        hv[i] = rnd() * 1e-6f;
    }
    const int T = 64;
    std::vector<float> hc(4 * (T + 1));
    for (int t = 1; t <= T; ++t) {
        const double bc1 = 1.0 - std::pow(0.9, t), bc2 = 1.0 - std::pow(0.999, t);
        const float c = static_cast<float>(std::sqrt(bc2));
        hc[4 * t] = static_cast<float>(-(1e-3 / bc1));
        hc[4 * t + 1] = c;
        hc[4 * t + 2] = 1.0f / c;
    }
    float *P, *M, *V, *C, *P0;
    (void)hipMalloc(&P, elems * 4);
    (void)hipMalloc(&M, elems * 4);
    (void)hipMalloc(&V, elems * 4);
    (void)hipMalloc(&P0, elems * 4);
    (void)hipMalloc(&C, hc.size() * 4);
    (void)hipMemcpy(C, hc.data(), hc.size() * 4, hipMemcpyHostToDevice);
    const K k{0.1f, 0.999f, 1e-8f};
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int ns[] = {17000, 170000};
    const int Rs[] = {4, 16, 32};
    for (int n : ns)
        for (int R : Rs) {
            float ms[7];
            for (int var = 0; var < 7; ++var) {
                (void)hipMemcpy(P, h0.data(), size_t(n) * 512, hipMemcpyHostToDevice);
                (void)hipMemcpy(M, hm.data(), size_t(n) * 512, hipMemcpyHostToDevice);
                (void)hipMemcpy(V, hv.data(), size_t(n) * 512, hipMemcpyHostToDevice);
                const int lpr = var == 2 ? 16 : 32;
                const int blocks = (n * lpr + 255) / 256;
                auto launch = [&]() {
                    if (var == 0)
                        k_replay<0><<<blocks, 256>>>((float4*)P, (float4*)M, (float4*)V, (const float4*)C, n, R, k);
                    else if (var == 1)
                        k_replay<1><<<blocks, 256>>>((float4*)P, (float4*)M, (float4*)V, (const float4*)C, n, R, k);
                    else if (var == 4)
                        k_replay<4><<<blocks, 256>>>((float4*)P, (float4*)M, (float4*)V, (const float4*)C, n, R, k);
                    else if (var == 5)
                        k_replay<5><<<blocks, 256>>>((float4*)P, (float4*)M, (float4*)V, (const float4*)C, n, R, k);
                    else if (var == 6)
                        k_replay<6><<<blocks, 256>>>((float4*)P, (float4*)M, (float4*)V, (const float4*)C, n, R, k);
                    else if (var == 3)
                        k_replay<3><<<blocks, 256>>>((float4*)P, (float4*)M, (float4*)V, (const float4*)C, n, R, k);
                    else
                        k_replay<2><<<blocks, 256>>>((float4*)P, (float4*)M, (float4*)V, (const float4*)C, n, R, k);
                };
                launch();  // one replay for the bitwise check, then timed repeats (values keep moving)
                if (var >= 4) {
                } else if (var == 0)
                    (void)hipMemcpy(P0, P, size_t(n) * 512, hipMemcpyDeviceToDevice);
                else {
                    std::vector<float> x0(size_t(n) * 128), x1(size_t(n) * 128);
                    (void)hipMemcpy(x0.data(), P0, size_t(n) * 512, hipMemcpyDeviceToHost);
                    (void)hipMemcpy(x1.data(), P, size_t(n) * 512, hipMemcpyDeviceToHost);
                    if (std::memcmp(x0.data(), x1.data(), x0.size() * 4) != 0) {
                        std::printf("variant %d differs from the scalar replay (n=%d R=%d)\n", var, n, R);
                        return 1;
                    }
                }
                (void)hipEventRecord(a);
                for (int it = 0; it < 20; ++it) launch();
                (void)hipEventRecord(b);
                (void)hipEventSynchronize(b);
                (void)hipEventElapsedTime(&ms[var], a, b);
                ms[var] /= 20;
            }
            const double el = double(n) * 128 * R;
            std::printf("n=%6d R=%2d: scalar %7.2f us, packed %7.2f us, packed 2xILP %7.2f us, windowed div %7.2f us "
                        "(%.0f / %.0f / %.0f / %.0f G element-steps/s)\n",
                        n, R, ms[0] * 1e3, ms[1] * 1e3, ms[2] * 1e3, ms[3] * 1e3, el / ms[0] / 1e6, el / ms[1] / 1e6,
                        el / ms[2] / 1e6, el / ms[3] / 1e6);
            std::printf("            diagnostics: no sqrt %7.2f us, no division %7.2f us, sqrt estimate + corrections only %7.2f us\n",
                        ms[4] * 1e3, ms[5] * 1e3, ms[6] * 1e3);
        }
    return 0;
}
