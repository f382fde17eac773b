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
#include <cstring>
#include <vector>

#include "lgcn.h"

namespace {

struct MT19937 {
    uint32_t* mt;  // caller's 624-word key (numpy get_state()[1]), updated in place
    int pos;

    void twist() {
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

    // tempered outputs of the current key, made a whole block at a time (vectorisable) instead
    // of one dependent chain per draw
    uint32_t tb[624];
    void temper_all() {
        for (int k = 0; k < 624; ++k) {
            uint32_t y = mt[k];
            y ^= (y >> 11);
            y ^= (y << 7) & 0x9d2c5680u;
            y ^= (y << 15) & 0xefc60000u;
            y ^= (y >> 18);
            tb[k] = y;
        }
    }

    inline uint32_t next() {
        if (pos >= 624) {
            twist();
            temper_all();
        }
        return tb[pos++];
    }

    // numpy random_interval(max) for max <= 0xffffffff
    inline uint32_t interval(uint32_t max) {
        if (max == 0) return 0;
        uint32_t mask = max;
        mask |= mask >> 1;
        mask |= mask >> 2;
        mask |= mask >> 4;
        mask |= mask >> 8;
        mask |= mask >> 16;
        uint32_t v;
        while ((v = (next() & mask)) > max) {
        }
        return v;
    }
};

}  // namespace

extern "C" int lgcn_legacy_choice(uint32_t* key, int32_t* pos, int64_t n, int64_t size, int64_t draws, int64_t* out) {
    if (!key || !pos || *pos < 0 || *pos > 624 || n <= 0 || size < 0 || size > n || draws < 0 ||
        (size > 0 && draws > 0 && !out) || n - 1 > int64_t(0xffffffffLL) || n > int64_t(INT32_MAX))
        return LGCN_E_ARG;
    MT19937 g{key, *pos, {}};
    g.temper_all();  // outputs pos..623 of the caller's current block
    std::vector<int32_t> x(static_cast<size_t>(n) + 1);
    for (int64_t d = 0; d < draws; ++d) {
        for (int64_t t = 0; t < n; ++t) x[t] = static_cast<int32_t>(t);
        int64_t* o = out + d * size;
        int64_t i = n - 1;
        // past the prefix: x[i] is dead after its swap, so a step is x[j] = x[i]. One loop
        // iteration per MT draw, branch-free: a rejected draw stores into a dummy slot and leaves
        // i unchanged (the rejections are random, so a branch on them mispredicts ~1 in 4).
        {
            uint32_t ii = static_cast<uint32_t>(i);
            const uint32_t stop = static_cast<uint32_t>(size > 1 ? size : 1);
            int32_t* xs = x.data();
            const uint32_t dummy = static_cast<uint32_t>(n);  // x has one spare slot
            int p = g.pos;
            while (ii >= stop) {
                if (p >= 624) {
                    g.pos = p;
                    g.twist();
                    g.temper_all();
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
            const int32_t vj = x[j];
            x[j] = x[i];
            o[i] = vj;
        }
        if (size > 0) o[0] = x[0];
    }
    *pos = g.pos;
    return LGCN_OK;
}
