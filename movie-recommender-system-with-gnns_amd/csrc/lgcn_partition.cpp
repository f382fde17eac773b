// Host-side graph partitioner for Cluster-GCN batching — the METIS replacement.
//
// Reference: data/dataset_handler.py:273 ClusterData(train_dataset, num_parts) (PyG 2.4.0) runs
// METIS_PartGraphKway (via torch_sparse.partition, CPU) on the training graph and keeps only the
// edges whose two endpoints fall in the same part. METIS is not available here, so this file
// provides a deterministic balanced k-way partitioner with the same contract (node -> part id in
// [0, k), parts balanced on node count) that runs in O(passes * E):
//
//   two initial phases, the better kept (more edges intra-part after refinement + fix-up):
//   (a) the nodes streamed as below; (b) size-constrained label-propagation clustering (KaHIP's
//   SCLaP: a node joins the neighbouring cluster holding strictly more of its neighbours, clusters
//   capped at a part's capacity), the clusters contracted into a node- and edge-weighted graph and
//   streamed the same way. (b) finds communities where the graph has them (planted ML-25M-sized
//   graph, 1024 parts: 0.514 of the train edges intra-part vs 0.463 for (a), truth 0.527);
//   (a) wins on the unstructured ML-25M-shaped graph.
//   restreaming Linear Deterministic Greedy (Stanton & Kliot 2012; Nishimura & Ugander 2013):
//   nodes are streamed in BFS order over the undirected adjacency; node v goes to the part i
//   maximising  |N(v) ∩ P_i| * (1 - |P_i| / C),  C = ceil(N/k * (1 + imbalance)), ties to the
//   smaller part then the lower id, parts at capacity skipped. Passes after the first re-stream the
//   same order, reading the previous pass's labels for neighbours not yet placed in this pass.
//   Then size-constrained label propagation refines the labels (moves that strictly raise a
//   node's intra-part neighbours, under the capacity), and a final fix-up makes the part sizes
//   exactly floor/ceil(N/k) (no empty part, hence no empty training batch), moving the nodes
//   that lose the fewest intra-part edges. On a planted 256-community user-item graph this keeps
//   0.756 of the edges intra-part against the ground truth's 0.781 (tools/partition_quality.py).
//
// Quality is reported as the fraction of edges kept intra-part (what Cluster-GCN trains on).
// Pure host code: no HIP calls, callable without a GPU.

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "lgcn_common.h"

namespace {

thread_local char g_perr[256];


// lgcn_tuning_t.partition_refine_rounds: the refinement rounds (default 16; 0 = LDG only)
int refine_rounds() { return lgcn::tuning().partition_refine_rounds; }


// lgcn_tuning_t.partition_cluster_rounds: the clustering rounds of the initial phase (default
// 8; 0 = stream the nodes themselves, the round-1 partitioner)
int cluster_rounds() { return lgcn::tuning().partition_cluster_rounds; }

// Size-constrained label-propagation clustering (KaHIP's SCLaP, used there for coarsening):
// every node starts alone; in `order`, a node joins the neighbouring cluster holding strictly more
// of its neighbours than its own, if that cluster stays within `ucap` nodes. Returns cluster ids
// compacted to 0 .. C-1 (in order of first appearance along `order`) and their sizes.
int64_t sclap_clusters(const std::vector<int64_t>& rowptr, const std::vector<int32_t>& adj,
                       const std::vector<int32_t>& order, int64_t N, int64_t ucap, int rounds,
                       std::vector<int32_t>& cl, std::vector<int64_t>& csz) {
    cl.resize(N);
    std::vector<int64_t> sz(N, 1);
    for (int64_t v = 0; v < N; ++v) cl[v] = static_cast<int32_t>(v);
    std::vector<int64_t> cnt(N, 0);
    std::vector<int32_t> touched;
    for (int r = 0; r < rounds; ++r) {
        int64_t moved = 0;
        for (const int32_t v : order) {
            const int32_t own = cl[v];
            touched.clear();
            for (int64_t p = rowptr[v]; p < rowptr[v + 1]; ++p) {
                const int32_t c = cl[adj[p]];
                if (cnt[c]++ == 0) touched.push_back(c);
            }
            int32_t best = own;
            int64_t bc = cnt[own];
            for (const int32_t c : touched) {
                if (c == own || sz[c] + 1 > ucap) continue;
                if (cnt[c] > bc || (cnt[c] == bc && best != own && c < best)) {
                    best = c;
                    bc = cnt[c];
                }
            }
            for (const int32_t c : touched) cnt[c] = 0;
            if (best != own) {
                cl[v] = best;
                sz[own]--;
                sz[best]++;
                ++moved;
            }
        }
        if (moved * 1000 < N) break;
    }
    std::vector<int32_t> id(N, -1);
    int64_t C = 0;
    for (const int32_t v : order)
        if (id[cl[v]] < 0) id[cl[v]] = static_cast<int32_t>(C++);
    csz.assign(C, 0);
    for (int64_t v = 0; v < N; ++v) {
        cl[v] = id[cl[v]];
        csz[cl[v]]++;
    }
    return C;
}

int perr(int code, const char* msg) {
    std::strncpy(g_perr, msg, sizeof(g_perr) - 1);
    return code;
}

}  // namespace

extern "C" {

const char* lgcn_partition_last_error(void) { return g_perr; }

int lgcn_partition_edges(const int64_t* src, const int64_t* dst, int64_t E, int64_t N, int32_t num_parts,
                         int32_t passes, float imbalance, int32_t* part_out) {
    if (N < 0 || E < 0 || num_parts < 1 || passes < 1 || imbalance < 0.f || !part_out || (E > 0 && (!src || !dst)))
        return perr(LGCN_E_ARG, "lgcn_partition_edges: bad args");
    if (N == 0) return LGCN_OK;
    if (num_parts == 1) {
        std::fill(part_out, part_out + N, 0);
        return LGCN_OK;
    }
    // undirected adjacency (both directions, self loops dropped; duplicates kept: they weigh a
    // neighbour as the number of edges to it, as METIS edge weights would)
    std::vector<int64_t> rowptr(N + 1, 0);
    for (int64_t e = 0; e < E; ++e) {
        const int64_t a = src[e], b = dst[e];
        if (a < 0 || a >= N || b < 0 || b >= N) return perr(LGCN_E_ARG, "lgcn_partition_edges: node id out of range");
        if (a == b) continue;
        rowptr[a + 1]++;
        rowptr[b + 1]++;
    }
    for (int64_t i = 0; i < N; ++i) rowptr[i + 1] += rowptr[i];
    std::vector<int32_t> adj(static_cast<size_t>(rowptr[N]));
    {
        std::vector<int64_t> fill(rowptr.begin(), rowptr.end() - 1);
        for (int64_t e = 0; e < E; ++e) {
            const int64_t a = src[e], b = dst[e];
            if (a == b) continue;
            adj[fill[a]++] = static_cast<int32_t>(b);
            adj[fill[b]++] = static_cast<int32_t>(a);
        }
    }
    // BFS stream order (restart at the lowest unvisited id for each component)
    std::vector<int32_t> order;
    order.reserve(N);
    {
        std::vector<uint8_t> seen(N, 0);
        for (int64_t s = 0; s < N; ++s) {
            if (seen[s]) continue;
            seen[s] = 1;
            size_t head = order.size();
            order.push_back(static_cast<int32_t>(s));
            while (head < order.size()) {
                const int32_t v = order[head++];
                for (int64_t p = rowptr[v]; p < rowptr[v + 1]; ++p) {
                    const int32_t u = adj[p];
                    if (!seen[u]) {
                        seen[u] = 1;
                        order.push_back(u);
                    }
                }
            }
        }
    }
    const int64_t cap = static_cast<int64_t>((static_cast<double>(N) / num_parts) * (1.0 + imbalance)) + 1;
    std::vector<int64_t> size(num_parts, 0);
    std::vector<int64_t> cnt(num_parts, 0);
    std::vector<int32_t> touched;
    touched.reserve(1024);
    // Initial phase. With clustering (default): size-constrained label propagation groups nodes
    // into clusters of at most a part's capacity (communities, where the graph has them), the
    // clusters are contracted into a node-weighted graph, and LDG streams the clusters; without:
    // LDG streams the nodes (unit weights). Either way the labels land on every node.
    // One full run (initial phase, refinement, balance fix-up) with `crounds` clustering rounds
    // (0 = stream the nodes); returns the labels.
    auto run = [&](const int crounds) {
        std::vector<int32_t> prev(N, -1);
        {
            std::vector<int32_t> cl;
            std::vector<int64_t> w;
            int64_t C = N;
            std::vector<int64_t> crp;
            std::vector<int32_t> cadj;
            std::vector<int64_t> cew;
            if (crounds > 0) {
                C = sclap_clusters(rowptr, adj, order, N, cap, crounds, cl, w);
                // contracted graph: cluster adjacency with edge weights (fine edge counts)
                std::vector<uint64_t> keys;
                keys.reserve(adj.size());
                for (int64_t v = 0; v < N; ++v)
                    for (int64_t p = rowptr[v]; p < rowptr[v + 1]; ++p) {
                        const int32_t a = cl[v], b = cl[adj[p]];
                        if (a != b) keys.push_back((static_cast<uint64_t>(a) << 32) | static_cast<uint32_t>(b));
                    }
                std::sort(keys.begin(), keys.end());
                crp.assign(C + 1, 0);
                for (size_t i = 0; i < keys.size();) {
                    size_t j = i;
                    while (j < keys.size() && keys[j] == keys[i]) ++j;
                    const int64_t a = static_cast<int64_t>(keys[i] >> 32);
                    cadj.push_back(static_cast<int32_t>(keys[i] & 0xFFFFFFFFu));
                    cew.push_back(static_cast<int64_t>(j - i));
                    crp[a + 1]++;
                    i = j;
                }
                for (int64_t i = 0; i < C; ++i) crp[i + 1] += crp[i];
            } else {
                cl.resize(N);
                for (int64_t v = 0; v < N; ++v) cl[v] = static_cast<int32_t>(v);
                w.assign(N, 1);
            }
            const std::vector<int64_t>& R_ = crounds > 0 ? crp : rowptr;
            const std::vector<int32_t>& A_ = crounds > 0 ? cadj : adj;
            // stream order of the units: BFS over their graph, heaviest-first start per component
            std::vector<int32_t> corder;
            if (crounds > 0) {
                corder.reserve(C);
                std::vector<int32_t> byw(C);
                for (int64_t i = 0; i < C; ++i) byw[i] = static_cast<int32_t>(i);
                std::stable_sort(byw.begin(), byw.end(), [&](int32_t a, int32_t b) { return w[a] > w[b]; });
                std::vector<uint8_t> seen(C, 0);
                for (const int32_t s0 : byw) {
                    if (seen[s0]) continue;
                    seen[s0] = 1;
                    size_t head = corder.size();
                    corder.push_back(s0);
                    while (head < corder.size()) {
                        const int32_t v = corder[head++];
                        for (int64_t p = R_[v]; p < R_[v + 1]; ++p) {
                            const int32_t u = A_[p];
                            if (!seen[u]) {
                                seen[u] = 1;
                                corder.push_back(u);
                            }
                        }
                    }
                }
            }
            const std::vector<int32_t>& O_ = crounds > 0 ? corder : order;
            std::vector<int64_t> conn(num_parts, 0);
            std::vector<int32_t> cprev(C, -1), ccur(C, -1);
            for (int32_t pass = 0; pass < passes; ++pass) {
                std::fill(size.begin(), size.end(), 0);
                std::fill(ccur.begin(), ccur.end(), -1);
                for (const int32_t v : O_) {
                    touched.clear();
                    for (int64_t p = R_[v]; p < R_[v + 1]; ++p) {
                        const int32_t u = A_[p];
                        const int32_t lab = ccur[u] >= 0 ? ccur[u] : cprev[u];
                        if (lab < 0) continue;
                        if (conn[lab] == 0) touched.push_back(lab);
                        conn[lab] += crounds > 0 ? cew[p] : 1;
                    }
                    int32_t best = -1;
                    double best_score = -1.0;
                    for (const int32_t i : touched) {
                        if (size[i] + w[v] > cap) continue;
                        const double score = static_cast<double>(conn[i]) * (1.0 - static_cast<double>(size[i]) / cap);
                        if (score > best_score || (score == best_score && (size[i] < size[best] ||
                                                                           (size[i] == size[best] && i < best)))) {
                            best = i;
                            best_score = score;
                        }
                    }
                    for (const int32_t i : touched) conn[i] = 0;
                    if (best < 0 || best_score <= 0.0) {
                        // no placed neighbour (or all their parts full): least loaded part, lowest id
                        best = static_cast<int32_t>(std::min_element(size.begin(), size.end()) - size.begin());
                    }
                    ccur[v] = best;
                    size[best] += w[v];
                }
                cprev.swap(ccur);
            }
            for (int64_t v = 0; v < N; ++v) prev[v] = cprev[cl[v]];
        }
        // Refinement: size-constrained label propagation (in the spirit of KaHIP's SCLaP). In stream
        // order, a node moves to the part holding most of its neighbours if that part is under the
        // capacity and strictly more of its neighbours are there than in its own part (so the number
        // of intra-part edges never decreases); labels update in place. Rounds stop when fewer than
        // N/1000 nodes move.
        {
            std::fill(size.begin(), size.end(), 0);
            for (int64_t v = 0; v < N; ++v) size[prev[v]]++;
            for (int round = 0, rounds = refine_rounds(); round < rounds; ++round) {
                int64_t moved = 0;
                for (const int32_t v : order) {
                    const int32_t own = prev[v];
                    touched.clear();
                    for (int64_t p = rowptr[v]; p < rowptr[v + 1]; ++p) {
                        const int32_t lab = prev[adj[p]];
                        if (cnt[lab]++ == 0) touched.push_back(lab);
                    }
                    int32_t best = own;
                    int64_t best_cnt = cnt[own];
                    for (const int32_t i : touched) {
                        if (i == own || size[i] >= cap) continue;
                        if (cnt[i] > best_cnt || (cnt[i] == best_cnt && best != own && i < best)) {
                            best = i;
                            best_cnt = cnt[i];
                        }
                    }
                    for (const int32_t i : touched) cnt[i] = 0;
                    if (best != own) {
                        prev[v] = best;
                        size[own]--;
                        size[best]++;
                        ++moved;
                    }
                }
                if (moved * 1000 < N) break;
            }
        }
        // Balance fix-up: parts end with exactly floor(N/k) or ceil(N/k) nodes (the first N % k parts
        // get the extra node), so no part is empty. The nodes of over-full parts leave in ascending
        // order of their neighbours inside their part (ties: latest-streamed first), each to the
        // under-full part holding most of its neighbours (ties: lowest id; none: the lowest-id
        // under-full part).
        {
            std::vector<int64_t> target(num_parts, N / num_parts);
            for (int64_t i = 0; i < N % num_parts; ++i) target[i]++;
            std::fill(size.begin(), size.end(), 0);
            for (int64_t v = 0; v < N; ++v) size[prev[v]]++;
            std::vector<int64_t> pos(N);
            for (int64_t i = 0; i < N; ++i) pos[order[i]] = i;
            std::vector<std::pair<int64_t, int64_t>> cand;  // (intra neighbours, -stream position)
            for (int64_t v = 0; v < N; ++v) {
                if (size[prev[v]] <= target[prev[v]]) continue;
                int64_t in = 0;
                for (int64_t p = rowptr[v]; p < rowptr[v + 1]; ++p) in += prev[adj[p]] == prev[v];
                cand.emplace_back(in, -pos[v]);
            }
            std::sort(cand.begin(), cand.end());
            int32_t fill_part = 0;
            for (const auto& c : cand) {
                const int32_t v = order[-c.second];
                const int32_t own = prev[v];
                if (size[own] <= target[own]) continue;
                while (fill_part < num_parts && size[fill_part] >= target[fill_part]) ++fill_part;
                if (fill_part >= num_parts) break;
                touched.clear();
                for (int64_t p = rowptr[v]; p < rowptr[v + 1]; ++p) {
                    const int32_t lab = prev[adj[p]];
                    if (cnt[lab]++ == 0) touched.push_back(lab);
                }
                int32_t best = fill_part;
                int64_t best_cnt = 0;
                for (const int32_t i : touched) {
                    if (size[i] >= target[i]) continue;
                    if (cnt[i] > best_cnt || (cnt[i] == best_cnt && i < best)) {
                        best = i;
                        best_cnt = cnt[i];
                    }
                }
                for (const int32_t i : touched) cnt[i] = 0;
                prev[v] = best;
                size[own]--;
                size[best]++;
            }
        }
        return prev;
    };
    // Clustering finds communities where the graph has them (planted ML-25M-sized graph, 1024
    // parts: 0.514 intra vs 0.463 streaming nodes) and loses where it has none (ML-25M-shaped
    // random graph: 0.023 vs 0.027), so both initial phases run and the labels keeping more
    // edges intra-part win (ties: the node-streaming run).
    auto intra = [&](const std::vector<int32_t>& lab) {
        int64_t k = 0;
        for (int64_t v = 0; v < N; ++v)
            for (int64_t q = rowptr[v]; q < rowptr[v + 1]; ++q) k += lab[v] == lab[adj[q]];
        return k;
    };
    std::vector<int32_t> prev = run(0);
    const int crounds = cluster_rounds();
    if (crounds > 0) {
        std::vector<int32_t> alt = run(crounds);
        if (intra(alt) > intra(prev)) prev.swap(alt);
    }
    std::memcpy(part_out, prev.data(), sizeof(int32_t) * static_cast<size_t>(N));
    return LGCN_OK;
}

}  // extern "C"
