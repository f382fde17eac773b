// Bitwise checks of the library's shortened exact sqrt / division (csrc/lgcn_exact.h, used by the
// row-lazy Adam) and of the packed forms in tools/exact2.h against the compiler's own sqrtf and
// '/' on gfx950, built with the library's flags:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off \
//       -Imovie-recommender-system-with-gnns_amd/csrc tools/exact_math_check.hip -o tools/_bin/exact_math_check
// sqrt_normal: every fp32 input in its range ({+0} and [2^-96, FLT_MAX]). div_window: 2^32
// quotients of operands drawn log-uniformly over its ranges (either sign, +0 numerators) and the
// cross product of its boundary values. sqrt2: every one of the 2^32 bit patterns. div2: 2^32
// random bit patterns (every exponent, denormals, inf and NaN included), the 128 x 128 cross
// product of special and boundary values, and 2^29 pairs from the Adam's ranges. A NaN result must
// be NaN on both sides; every other result must have the same bits. Exit 1 on any mismatch.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdint>

#include "exact2.h"
#include "lgcn_exact.h"

using lgcn::f2;

__device__ __forceinline__ uint32_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return static_cast<uint32_t>(x);
}

__device__ __forceinline__ bool same(float a, float b) {
    if (a != a) return b != b;
    return __float_as_uint(a) == __float_as_uint(b);
}

__global__ void k_sqrt(unsigned long long* bad) {
    unsigned long long n = 0;
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < (1ull << 31); i += stride) {
        const float x = __uint_as_float(static_cast<uint32_t>(i));
        const float y = __uint_as_float(static_cast<uint32_t>(i | (1ull << 31)));
        const f2 r = lgcn::sqrt2(f2{x, y});
        n += !same(r.x, sqrtf(x)) + !same(r.y, sqrtf(y));
    }
    if (n) atomicAdd(bad, n);
}

// every fp32 bit pattern in sqrt_normal's range: +0 and [2^-96, FLT_MAX]
__global__ void k_sqrt_normal(unsigned long long* bad) {
    unsigned long long n = 0;
    const uint32_t lo = 0x0f800000u, hi = 0x7f7fffffu;  // 2^-96, FLT_MAX
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i <= uint64_t(hi - lo) + 1; i += stride) {
        const float x = i == uint64_t(hi - lo) + 1 ? 0.0f : __uint_as_float(lo + static_cast<uint32_t>(i));
        n += !same(lgcn::sqrt_normal(x), sqrtf(x));
    }
    if (n) atomicAdd(bad, n);
}

// div_window: mode 0 operands log-uniform in the window (a: either sign, 1/64 of them +0), mode 1
// the cross product of boundary values (+-2^-40, +-2^40 and their in-range neighbours, +0, 1, ...)
__device__ float window_edge(int k) {
    const float v[8] = {0x1p-40f, 0x1.000002p-40f, 0x1.fffffep39f, 0x1p39f, 1.0f, 0x1.fffffep-1f, 3.0f, 0x1.8p-20f};
    return v[k & 7];
}

__global__ void k_div_window(unsigned long long* bad, uint64_t n, int mode, uint64_t seed) {
    unsigned long long cnt = 0;
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        float a, b;
        if (mode == 0) {
            const uint32_t ra = mix(seed + 2 * i), rb = mix(seed + 2 * i + 1);
            // 2^u with u in [-40, 40), significand from the low bits: every exponent, continuous
            a = __uint_as_float(((static_cast<uint32_t>(87 + (ra >> 25) % 80)) << 23) | (ra & 0x7fffffu));
            b = __uint_as_float(((static_cast<uint32_t>(87 + (rb >> 25) % 80)) << 23) | (rb & 0x7fffffu));
            if ((ra >> 23) & 1u) a = -a;
            if (((ra >> 24) & 63u) == 0u) a = 0.0f;
        } else {
            a = (i & 64) ? -window_edge(static_cast<int>(i >> 3)) : window_edge(static_cast<int>(i >> 3));
            if ((i & 56) == 56) a = 0.0f;
            b = window_edge(static_cast<int>(i));
        }
        cnt += !same(lgcn::div_window(a, b), a / b);
    }
    if (cnt) atomicAdd(bad, cnt);
}

__device__ float special(int k) {
    const float v[16] = {0.0f, 1.0f, 0x1p-149f, 0x1p-126f, 0x1.fffffep-127f, 0x1.fffffep127f, INFINITY, NAN,
                         0x1p-96f, 0x1p-64f, 0x1p64f, 0x1p96f, 3.0f, 0x1.800002p0f, 1e-8f, 0.999f};
    const float s = v[k & 15];
    const int e = (k >> 4) & 3;  // scaled around the special value
    const float t = e == 0 ? s : e == 1 ? s * 0x1.000002p0f : e == 2 ? s * 0x1.fffffep-1f : s * 0x1p-24f;
    return (k >> 6) & 1 ? -t : t;
}

// mode 0: random bit patterns; 1: special x special (n = 128 * 128 / 2 pairs); 2: Adam ranges
__global__ void k_div(unsigned long long* bad, uint64_t n, int mode, uint64_t seed) {
    unsigned long long cnt = 0;
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        float a0, b0, a1, b1;
        if (mode == 0) {
            a0 = __uint_as_float(mix(seed + 4 * i));
            b0 = __uint_as_float(mix(seed + 4 * i + 1));
            a1 = __uint_as_float(mix(seed + 4 * i + 2));
            b1 = __uint_as_float(mix(seed + 4 * i + 3));
        } else if (mode == 1) {
            const int p = static_cast<int>(2 * i);
            a0 = special(p >> 7);
            b0 = special(p & 127);
            a1 = special((p + 1) >> 7);
            b1 = special((p + 1) & 127);
        } else {
            // |m| = 2^u with u uniform in [-100, 0] (continuous significand), denominator 2^w, w in [-26.6, 4]
            auto draw = [&](uint64_t k, float lo, float hi) {
                const float u = lo + (hi - lo) * (mix(seed + k) * 0x1p-32f);
                return exp2f(u);
            };
            a0 = draw(4 * i, -100.0f, 0.0f) * ((mix(seed ^ i) & 1) ? -1.0f : 1.0f);
            b0 = draw(4 * i + 1, -26.6f, 4.0f);
            a1 = draw(4 * i + 2, -100.0f, 0.0f);
            b1 = draw(4 * i + 3, -26.6f, 4.0f);
        }
        const f2 r = lgcn::div2(f2{a0, a1}, f2{b0, b1});
        cnt += !same(r.x, a0 / b0) + !same(r.y, a1 / b1);
    }
    if (cnt) atomicAdd(bad, cnt);
}

int main() {
    unsigned long long* bad;
    if (hipMalloc(&bad, 8 * sizeof(unsigned long long)) != hipSuccess) return 2;
    (void)hipMemset(bad, 0, 8 * sizeof(unsigned long long));
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    k_sqrt<<<8192, 256>>>(bad);
    k_div<<<8192, 256>>>(bad + 1, 1ull << 30, 0, 0x9e3779b97f4a7c15ULL);
    k_div<<<8192, 256>>>(bad + 1, 1ull << 30, 0, 0x2545f4914f6cdd1dULL);
    k_div<<<64, 128>>>(bad + 2, 128 * 128 / 2, 1, 0);
    k_div<<<8192, 256>>>(bad + 3, 1ull << 27, 2, 0x853c49e6748fea9bULL);
    k_div<<<8192, 256>>>(bad + 3, 1ull << 27, 2, 0xda3e39cb94b95bdbULL);
    k_sqrt_normal<<<8192, 256>>>(bad + 4);
    k_div_window<<<8192, 256>>>(bad + 5, 1ull << 32, 0, 0x5851f42d4c957f2dULL);
    k_div_window<<<8, 64>>>(bad + 6, 512, 1, 0);
    (void)hipEventRecord(b);
    if (hipEventSynchronize(b) != hipSuccess) return 2;
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    unsigned long long h[8];
    (void)hipMemcpy(h, bad, sizeof(h), hipMemcpyDeviceToHost);
    std::printf("sqrt2: %llu mismatches of 4294967296 inputs\n", h[0]);
    std::printf("div2 random bits: %llu mismatches of 4294967296 quotients\n", h[1]);
    std::printf("div2 specials: %llu mismatches of 16384 quotients\n", h[2]);
    std::printf("div2 Adam ranges: %llu mismatches of 536870912 quotients\n", h[3]);
    std::printf("sqrt_normal: %llu mismatches of %u inputs (+0, [2^-96, FLT_MAX])\n", h[4], 0x7f7fffffu - 0x0f800000u + 2u);
    std::printf("div_window random: %llu mismatches of 4294967296 quotients\n", h[5]);
    std::printf("div_window boundaries: %llu mismatches of 512 quotients\n", h[6]);
    std::printf("%.1f ms\n", ms);
    return (h[0] | h[1] | h[2] | h[3] | h[4] | h[5] | h[6]) ? 1 : 0;
}
