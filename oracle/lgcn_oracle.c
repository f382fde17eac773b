/*
 * ORACLE — test infrastructure, not product code. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg load liboracle.so, and only as the checker / CPU baseline.
 *
 * Plain-C restatement (fp32, scalar, single thread, no FMA contraction: built with
 * -ffp-contract=off) of the reference's propagation path at sizes numpy cannot reach quickly:
 *   - gcn_norm (PyG 2.4.0, add_self_loops=False; called via LGConv.forward at reference
 *     models/light_gcn.py:33): deg = fp32 sum of ones at edge_index[1] (saturates at 2^24),
 *     dis = 1/sqrt(deg) (inf -> 0), w_e = (dis[src]*1)*dis[dst];
 *   - LGConv propagate: out = 0; for e in edge order: out[dst_e] += w_e * x[src_e]
 *     (index_select -> mul -> CPU scatter_add_, which adds in edge order);
 *   - its autograd transpose: out = 0; for e in edge order: out[src_e] += w_e * dy[dst_e];
 *   - LightGCN.forward (reference models/light_gcn.py:28-40): stack-sum / (K+1) * fp32(1/(K+1));
 *   - stable CSR grouping by a key (the order the two loops above add in).
 * Mirrors oracle/lgconv_ref.py (numpy) bit for bit; tests/test_oracle.py checks that.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

int64_t oracle_csr_build(const int64_t* key, const int64_t* other, int64_t E, int64_t N,
                         int64_t* rowptr, int32_t* col, int32_t* eid) {
    int64_t bad = 0;
    memset(rowptr, 0, sizeof(int64_t) * (size_t)(N + 1));
    for (int64_t e = 0; e < E; ++e) {
        int64_t k = key[e], o = other[e];
        if (k < 0 || k >= N || o < 0 || o >= N) { ++bad; continue; }
        rowptr[k + 1]++;
    }
    if (bad) return bad;
    for (int64_t i = 0; i < N; ++i) rowptr[i + 1] += rowptr[i];
    int64_t* fill = (int64_t*)malloc(sizeof(int64_t) * (size_t)(N > 0 ? N : 1));
    memcpy(fill, rowptr, sizeof(int64_t) * (size_t)N);
    for (int64_t e = 0; e < E; ++e) {
        int64_t p = fill[key[e]]++;
        col[p] = (int32_t)other[e];
        eid[p] = (int32_t)e;
    }
    free(fill);
    return 0;
}

void oracle_inv_sqrt_degree(const int64_t* dst, int64_t E, int64_t N, float* dis) {
    float* deg = (float*)calloc((size_t)(N > 0 ? N : 1), sizeof(float));
    for (int64_t e = 0; e < E; ++e) deg[dst[e]] += 1.0f; /* sequential fp32 sum of ones */
    for (int64_t i = 0; i < N; ++i) {
        float v = 1.0f / sqrtf(deg[i]);
        dis[i] = isinf(v) ? 0.0f : v;
    }
    free(deg);
}

void oracle_gcn_norm(const int64_t* src, const int64_t* dst, int64_t E, int64_t N, float* dis, float* w) {
    oracle_inv_sqrt_degree(dst, E, N, dis);
    for (int64_t e = 0; e < E; ++e) w[e] = (dis[src[e]] * 1.0f) * dis[dst[e]];
}

/* out[N,d] = scatter_add over edges in order of w_e * x[from_e] at to_e */
void oracle_scatter_layer(const float* x, const int64_t* from, const int64_t* to, const float* w, int64_t E,
                          int64_t N, int32_t d, float* out) {
    memset(out, 0, sizeof(float) * (size_t)N * (size_t)d);
    for (int64_t e = 0; e < E; ++e) {
        const float* xs = x + from[e] * d;
        float* o = out + to[e] * d;
        const float we = w[e];
        for (int32_t c = 0; c < d; ++c) {
            float m = we * xs[c];
            o[c] = o[c] + m;
        }
    }
}

void oracle_lgconv(const float* x, const int64_t* src, const int64_t* dst, const float* w, int64_t E, int64_t N,
                   int32_t d, float* out) {
    oracle_scatter_layer(x, src, dst, w, E, N, d, out);
}

void oracle_lgconv_transposed(const float* dy, const int64_t* src, const int64_t* dst, const float* w, int64_t E,
                              int64_t N, int32_t d, float* out) {
    oracle_scatter_layer(dy, dst, src, w, E, N, d, out);
}

/* out[N,d] (users first). scratch: 2*N*d floats. */
void oracle_lightgcn_forward(const float* uw, const float* iw, int64_t U, int64_t I, const int64_t* src,
                             const int64_t* dst, int64_t E, int32_t d, int32_t K, float* out, float* scratch) {
    const int64_t N = U + I;
    const size_t nd = (size_t)N * (size_t)d;
    float* dis = (float*)malloc(sizeof(float) * (size_t)(N > 0 ? N : 1));
    float* w = (float*)malloc(sizeof(float) * (size_t)(E > 0 ? E : 1));
    oracle_gcn_norm(src, dst, E, N, dis, w);
    float* x = scratch;
    float* y = scratch + nd;
    memcpy(x, uw, sizeof(float) * (size_t)U * (size_t)d);
    memcpy(x + (size_t)U * d, iw, sizeof(float) * (size_t)I * (size_t)d);
    memcpy(out, x, sizeof(float) * nd); /* running stack sum, starts at x0 */
    for (int32_t k = 0; k < K; ++k) {
        oracle_scatter_layer(x, src, dst, w, E, N, d, y);
        for (size_t i = 0; i < nd; ++i) out[i] = out[i] + y[i];
        float* t = x; x = y; y = t;
    }
    const float div = (float)(K + 1);
    const float mul = (float)(1.0 / (double)(K + 1));
    for (size_t i = 0; i < nd; ++i) out[i] = (out[i] / div) * mul;
    free(dis);
    free(w);
}

/* grad[N,d] of the forward above given dout[N,d]. scratch: 2*N*d floats. */
void oracle_lightgcn_backward(const float* dout, int64_t N, const int64_t* src, const int64_t* dst, int64_t E,
                              int32_t d, int32_t K, float* grad, float* scratch) {
    const size_t nd = (size_t)N * (size_t)d;
    float* dis = (float*)malloc(sizeof(float) * (size_t)(N > 0 ? N : 1));
    float* w = (float*)malloc(sizeof(float) * (size_t)(E > 0 ? E : 1));
    oracle_gcn_norm(src, dst, E, N, dis, w);
    float* g = scratch;
    float* t = scratch + nd;
    const float div = (float)(K + 1);
    const float mul = (float)(1.0 / (double)(K + 1));
    for (size_t i = 0; i < nd; ++i) g[i] = (dout[i] * mul) / div;
    memcpy(grad, g, sizeof(float) * nd);
    for (int32_t k = 0; k < K; ++k) {
        oracle_scatter_layer(grad, dst, src, w, E, N, d, t);
        for (size_t i = 0; i < nd; ++i) grad[i] = g[i] + t[i];
    }
    free(dis);
    free(w);
}
