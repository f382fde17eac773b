// Process-wide tuning of liblgcn.so (include/lgcn.h, ABI 7): the schedule choices that earlier
// builds read from environment variables on every dispatch. Defaults are the measured choices
// (DESIGN.md §5); lgcn_set_tuning validates and replaces the whole struct.
#include <cstring>

#include "lgcn_common.h"

namespace lgcn {

namespace {

lgcn_tuning_t defaults() {
    lgcn_tuning_t t;
    std::memset(&t, 0, sizeof t);
    t.spmm_tail = -1;
    t.spmm_index_rounds = 0;
    t.pair_xcds_a = 4;
    t.partition_refine_rounds = 16;
    t.partition_cluster_rounds = 8;
    t.choice_threads = 16;
    return t;
}

lgcn_tuning_t g_tuning = defaults();

}  // namespace

const lgcn_tuning_t& tuning() { return g_tuning; }

}  // namespace lgcn

extern "C" {

int lgcn_tuning_defaults(lgcn_tuning_t* t) {
    if (t == nullptr) return lgcn::fail(LGCN_E_ARG, "lgcn_tuning_defaults: null");
    *t = lgcn::defaults();
    return LGCN_OK;
}

int lgcn_get_tuning(lgcn_tuning_t* t) {
    if (t == nullptr) return lgcn::fail(LGCN_E_ARG, "lgcn_get_tuning: null");
    *t = lgcn::g_tuning;
    return LGCN_OK;
}

int lgcn_set_tuning(const lgcn_tuning_t* t) {
    using lgcn::fail;
    if (t == nullptr) return fail(LGCN_E_ARG, "lgcn_set_tuning: null");
    if (t->spmm_tail < -1 || t->spmm_tail > 1) return fail(LGCN_E_ARG, "lgcn_set_tuning: spmm_tail %d", t->spmm_tail);
    const int r = t->spmm_index_rounds;
    if (!(r == 0 || r == 1 || r == 2 || r == 4 || r == 8 || r == 16 || r == 32))
        return fail(LGCN_E_ARG, "lgcn_set_tuning: spmm_index_rounds %d not in {0,1,2,4,8,16,32}", r);
    if (t->pair_xcds_a < 0 || t->pair_xcds_a > 7)
        return fail(LGCN_E_ARG, "lgcn_set_tuning: pair_xcds_a %d not in [0, 7]", t->pair_xcds_a);
    if (t->partition_refine_rounds < 0 || t->partition_refine_rounds > 1024 || t->partition_cluster_rounds < 0 ||
        t->partition_cluster_rounds > 1024)
        return fail(LGCN_E_ARG, "lgcn_set_tuning: partition rounds %d / %d not in [0, 1024]",
                    t->partition_refine_rounds, t->partition_cluster_rounds);
    if (t->choice_threads < 1 || t->choice_threads > 256)
        return fail(LGCN_E_ARG, "lgcn_set_tuning: choice_threads %d not in [1, 256]", t->choice_threads);
    for (int i = 0; i < 10; ++i)
        if (t->reserved[i] != 0) return fail(LGCN_E_ARG, "lgcn_set_tuning: reserved[%d] != 0", i);
    lgcn::g_tuning = *t;
    return LGCN_OK;
}

}  // extern "C"
