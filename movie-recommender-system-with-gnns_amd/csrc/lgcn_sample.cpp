// Host-side user sampling for Recall@k (reference utils/train_test.py:187:
// np.random.choice(num_users, sample_size, replace=False), once per sample).
//
// numpy's legacy RandomState draws that as permutation(n)[:size]: a Fisher–Yates shuffle of
// arange(n) from i = n-1 down to 1 with j = random_interval(i) (smallest all-ones mask >= i,
// MT19937 32-bit draws rejected while > i). That shuffle of the whole population is what costs
// the reference's Recall@k its time (≈5–12 ms per sample at 6e5 users). This file runs the same
// algorithm on the same MT19937 state, so the picks AND the generator state afterwards are
// numpy's bit for bit (tests/test_sample.py), but keeps only what the prefix needs: position i
// is dead after step i, so a step past the prefix is one draw and one store.

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <thread>
#include <vector>

#include "lgcn_common.h"

using lgcn::fail;

namespace {

// MT19937 over its own copy of the 624-word key (numpy get_state()[1]) and position.
struct MT19937 {
    uint32_t mt[624];
    int pos;
    uint32_t tb[624];  // tempered outputs of the current key, made a whole block at a time

    __attribute__((always_inline)) inline void twist() {
        constexpr uint32_t kUpper = 0x80000000u, kLower = 0x7fffffffu, kMatrix = 0x9908b0dfu;
        int k = 0;
        for (; k < 624 - 397; ++k) {
            const uint32_t y = (mt[k] & kUpper) | (mt[k + 1] & kLower);
            mt[k] = mt[k + 397] ^ (y >> 1) ^ ((y & 1u) ? kMatrix : 0u);
        }
        for (; k < 623; ++k) {
            const uint32_t y = (mt[k] & kUpper) | (mt[k + 1] & kLower);
            mt[k] = mt[k + 397 - 624] ^ (y >> 1) ^ ((y & 1u) ? kMatrix : 0u);
        }
        const uint32_t y = (mt[623] & kUpper) | (mt[0] & kLower);
        mt[623] = mt[396] ^ (y >> 1) ^ ((y & 1u) ? kMatrix : 0u);
        pos = 0;
    }

    __attribute__((always_inline)) inline void temper_all() {
        for (int k = 0; k < 624; ++k) {
            uint32_t y = mt[k];
            y ^= (y >> 11);
            y ^= (y << 7) & 0x9d2c5680u;
            y ^= (y << 15) & 0xefc60000u;
            y ^= (y >> 18);
            tb[k] = y;
        }
    }

    __attribute__((always_inline)) inline void refill() {
        twist();
        temper_all();
    }

    __attribute__((always_inline)) inline uint32_t next() {
        if (pos >= 624) refill();
        return tb[pos++];
    }

    // numpy random_interval(max) for max <= 0xffffffff
    __attribute__((always_inline)) inline uint32_t interval(uint32_t max) {
        if (max == 0) return 0;
        const uint32_t mask = 0xffffffffu >> __builtin_clz(max);
        uint32_t v;
        while ((v = (next() & mask)) > max) {
        }
        return v;
    }
};

// The draws one shuffle of arange(n) consumes, without the shuffle: i = n-1 .. 1, each step
// taking MT outputs until one masked output is <= i (numpy's rejection rule). Only the accept
// test is on the loop-carried path; the mask is fixed while i stays above half of it.
// Eight outputs at a time where that is unambiguous: within a group i falls by at most 8, so the
// group's accepts are its count of masked values <= i - 7 whenever no value lies in (i - 7, i]
// (rare while i >> 8); such a group runs one output at a time. Two counts per group vectorise
// (AVX2 where the host has it: 2x the SSE2 build's rate on this loop).
template <int G>
__attribute__((always_inline)) inline void skip_shuffle_impl(MT19937& g, int64_t n) {
    uint32_t ii = static_cast<uint32_t>(n - 1);
    while (ii >= 1) {
        if (g.pos >= 624) g.refill();
        const uint32_t mask = 0xffffffffu >> __builtin_clz(ii);
        const uint32_t lo = mask >> 1;  // the mask holds while ii > lo
        int p = g.pos;
        while (p + G <= 624 && ii > lo + G) {
            const uint32_t thr = ii - (G - 1);
            uint32_t ca = 0, cb = 0;
            for (int k = 0; k < G; ++k) {
                const uint32_t v = g.tb[p + k] & mask;
                ca += static_cast<uint32_t>(v <= thr);
                cb += static_cast<uint32_t>(v <= ii);
            }
            if (__builtin_expect(ca == cb, 1)) {
                ii -= ca;
            } else {
                for (int k = 0; k < G; ++k) ii -= static_cast<uint32_t>((g.tb[p + k] & mask) <= ii);
            }
            p += G;
        }
        while (p < 624 && ii > lo) ii -= static_cast<uint32_t>((g.tb[p++] & mask) <= ii);
        g.pos = p;
    }
}

// One draw: numpy's shuffle of arange(n) from the state in g, keeping the first `size` entries.
// x: n + 1 int32 scratch (one spare slot).
__attribute__((always_inline)) inline void one_choice_impl(MT19937& g, int64_t n, int64_t size, int32_t* xs,
                                                           int64_t* o) {
    for (int64_t t = 0; t < n; ++t) xs[t] = static_cast<int32_t>(t);
    int64_t i = n - 1;
    // past the prefix: x[i] is dead after its swap, so a step is x[j] = x[i]. One loop
    // iteration per MT draw, branch-free: a rejected draw stores into a dummy slot and leaves
    // i unchanged (the rejections are random, so a branch on them mispredicts ~1 in 4).
    {
        uint32_t ii = static_cast<uint32_t>(i);
        const uint32_t stop = static_cast<uint32_t>(size > 1 ? size : 1);
        const uint32_t dummy = static_cast<uint32_t>(n);
        int p = g.pos;
        while (ii >= stop) {
            if (p >= 624) {
                g.refill();
                p = 0;
            }
            // draws left in this block, each iteration consumes exactly one
            const int avail = 624 - p;
            for (int t = 0; t < avail && ii >= stop; ++t) {
                const uint32_t mask = 0xffffffffu >> __builtin_clz(ii);  // smallest all-ones >= ii (ii >= 1)
                const uint32_t v = g.tb[p++] & mask;
                const uint32_t okm = 0u - static_cast<uint32_t>(v <= ii);  // all ones if accepted
                xs[(v & okm) | (dummy & ~okm)] = xs[ii];
                ii -= okm & 1u;
            }
        }
        g.pos = p;
        i = static_cast<int64_t>(ii);
    }
    for (; i >= 1; --i) {  // inside the prefix: out[i] is final after step i
        const uint32_t j = g.interval(static_cast<uint32_t>(i));
        const int32_t vj = xs[j];
        xs[j] = xs[i];
        o[i] = vj;
    }
    if (size > 0) o[0] = xs[0];
}

// Both loops (and the MT refills inlined into them) built twice: for AVX2 hosts (the two counts
// per group and the block twist/temper vectorise 8-wide: ≈ 2x the baseline build's rate) and for
// the x86-64 baseline, picked once at run time.
__attribute__((target("avx2"))) void skip_shuffle_avx2(MT19937& g, int64_t n) { skip_shuffle_impl<8>(g, n); }
__attribute__((target("avx2"))) void one_choice_avx2(MT19937& g, int64_t n, int64_t size, int32_t* xs, int64_t* o) {
    one_choice_impl(g, n, size, xs, o);
}
void skip_shuffle_base(MT19937& g, int64_t n) { skip_shuffle_impl<8>(g, n); }
void one_choice_base(MT19937& g, int64_t n, int64_t size, int32_t* xs, int64_t* o) {
    one_choice_impl(g, n, size, xs, o);
}
bool host_avx2() {
    static const bool yes = __builtin_cpu_supports("avx2");
    return yes;
}
void skip_shuffle(MT19937& g, int64_t n) {
    if (host_avx2()) skip_shuffle_avx2(g, n);
    else skip_shuffle_base(g, n);
}
void one_choice(MT19937& g, int64_t n, int64_t size, int32_t* xs, int64_t* o) {
    if (host_avx2()) one_choice_avx2(g, n, size, xs, o);
    else one_choice_base(g, n, size, xs, o);
}

int choice_threads(int64_t n, int64_t draws) {
    if (draws < 2 || n < 65536) return 1;
    int t = lgcn::tuning().choice_threads;
    const unsigned hw = std::thread::hardware_concurrency();
    if (hw > 0 && static_cast<unsigned>(t) > hw) t = static_cast<int>(hw);
    if (t > draws) t = static_cast<int>(draws);
    return t < 1 ? 1 : t;
}

}  // namespace

// The draws run in parallel: the main thread walks the MT stream through each draw's accept
// tests only (skip_shuffle: where draw d+1 starts does not depend on the shuffle itself) and
// hands each draw's starting state to a worker, which replays that draw's shuffle; the picks
// and the final state are the sequential loop's.
extern "C" int lgcn_legacy_choice(uint32_t* key, int32_t* pos, int64_t n, int64_t size, int64_t draws, int64_t* out) {
    if (!key || !pos || *pos < 0 || *pos > 624 || n <= 0 || size < 0 || size > n || draws < 0 ||
        (size > 0 && draws > 0 && !out) || n - 1 > int64_t(0xffffffffLL) || n > int64_t(INT32_MAX))
        return LGCN_E_ARG;
    MT19937 g;
    std::memcpy(g.mt, key, sizeof(g.mt));
    g.pos = *pos;
    g.temper_all();  // outputs pos..623 of the caller's current block
    const int T = choice_threads(n, draws);
    if (T == 1) {
        std::vector<int32_t> x(static_cast<size_t>(n) + 1);
        for (int64_t d = 0; d < draws; ++d) one_choice(g, n, size, x.data(), out + d * size);
    } else {
        std::vector<std::vector<int32_t>> xs(static_cast<size_t>(T));  // one scratch per worker slot
        std::vector<std::thread> workers;
        try {
            workers.reserve(static_cast<size_t>(draws));
            for (auto& x : xs) x.resize(static_cast<size_t>(n) + 1);
            for (int64_t d = 0; d < draws; ++d) {
                if (static_cast<int64_t>(workers.size()) >= T) workers[static_cast<size_t>(d - T)].join();
                // a worker slot is reused once the draw that held it has been joined
                int32_t* x = xs[static_cast<size_t>(d % T)].data();
                workers.emplace_back([g, n, size, x, o = out + d * size]() mutable { one_choice(g, n, size, x, o); });
                skip_shuffle(g, n);
            }
        } catch (const std::exception& e) {  // no thread / no memory: the caller's state is untouched
            for (auto& w : workers)
                if (w.joinable()) w.join();
            return fail(LGCN_E_UNSUPPORTED, "lgcn_legacy_choice: %s", e.what());
        }
        for (auto& w : workers)
            if (w.joinable()) w.join();
    }
    std::memcpy(key, g.mt, sizeof(g.mt));
    *pos = g.pos;
    return LGCN_OK;
}
