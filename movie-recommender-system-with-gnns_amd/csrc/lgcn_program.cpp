// Launch programs (include/lgcn.h, ABI 11): a captured hipGraph issued as plain stream launches.
//
// A Cluster-GCN training step is captured once per batch (lgcn_amd.train_step) so the host does
// not re-issue its ~14 launches through Python every step. Replaying the captured graph costs the
// GPU ~8 us per hipGraphLaunch of its own (the idle gap before each step), while the
// same kernels issued eagerly run back to back: the eager step was measured faster on the GPU (C3
// 0.143 vs 0.151 ms) but its Python issue (0.130 ms per step) is nearly as long as the step. A
// launch program keeps both wins: the graph's nodes are read once (kernel function, grid, block,
// argument buffers, dynamic LDS; memsets) in a dependency order and each run issues them with
// hipLaunchKernel / hipMemset*Async on the caller's stream from one C call. The argument buffers
// are the graph's own (kernelParams of each node), so the graph must outlive the program; the
// step's device buffers are the capture's (its private memory pool).
#include <algorithm>
#include <new>
#include <vector>

#include "lgcn_common.h"

namespace lgcn {

namespace {

struct Op {
    hipGraphNodeType type;
    hipKernelNodeParams k;
    hipMemsetParams m;
};

struct Program {
    std::vector<Op> ops;
    int launches = 0;
};

int issue(const Op& op, hipStream_t s) {
    switch (op.type) {
        case hipGraphNodeTypeKernel:
            return check_hip(hipLaunchKernel(op.k.func, op.k.gridDim, op.k.blockDim, op.k.kernelParams,
                                             op.k.sharedMemBytes, s),
                             "lgcn_program_run: hipLaunchKernel");
        case hipGraphNodeTypeMemset: {
            const hipMemsetParams& m = op.m;
            if (m.height <= 1) {
                hipDeviceptr_t dst = reinterpret_cast<hipDeviceptr_t>(m.dst);
                if (m.elementSize == 1)
                    return check_hip(hipMemsetD8Async(dst, static_cast<unsigned char>(m.value), m.width, s),
                                     "lgcn_program_run: memset");
                if (m.elementSize == 2)
                    return check_hip(hipMemsetD16Async(dst, static_cast<unsigned short>(m.value), m.width, s),
                                     "lgcn_program_run: memset");
                return check_hip(hipMemsetD32Async(dst, static_cast<int>(m.value), m.width, s),
                                 "lgcn_program_run: memset");
            }
            return check_hip(hipMemset2DAsync(m.dst, m.pitch, static_cast<int>(m.value), m.width, m.height, s),
                             "lgcn_program_run: memset2d");
        }
        default:
            return fail(LGCN_E_UNSUPPORTED, "lgcn_program_run: node type %d", static_cast<int>(op.type));
    }
}

}  // namespace

}  // namespace lgcn

extern "C" {

int lgcn_program_from_graph(void* graph, void** prog_out) {
    using namespace lgcn;
    if (graph == nullptr || prog_out == nullptr) return fail(LGCN_E_ARG, "lgcn_program_from_graph: null");
    *prog_out = nullptr;
    hipGraph_t g = reinterpret_cast<hipGraph_t>(graph);
    size_t n = 0;
    if (int rc = check_hip(hipGraphGetNodes(g, nullptr, &n), "hipGraphGetNodes")) return rc;
    std::vector<hipGraphNode_t> nodes(n);
    if (n)
        if (int rc = check_hip(hipGraphGetNodes(g, nodes.data(), &n), "hipGraphGetNodes")) return rc;
    nodes.resize(n);
    // dependency order (Kahn; among ready nodes the lowest index first, so a one-stream capture
    // keeps its issue order): every node is issued after all of its dependencies, on one stream
    std::vector<std::vector<size_t>> succ(n);
    std::vector<size_t> indeg(n, 0);
    for (size_t i = 0; i < n; ++i) {
        size_t nd = 0;
        if (int rc = check_hip(hipGraphNodeGetDependencies(nodes[i], nullptr, &nd), "hipGraphNodeGetDependencies"))
            return rc;
        std::vector<hipGraphNode_t> deps(nd);
        if (nd)
            if (int rc = check_hip(hipGraphNodeGetDependencies(nodes[i], deps.data(), &nd),
                                   "hipGraphNodeGetDependencies"))
                return rc;
        for (size_t j = 0; j < nd; ++j) {
            auto it = std::find(nodes.begin(), nodes.end(), deps[j]);
            if (it == nodes.end()) return fail(LGCN_E_ARG, "lgcn_program_from_graph: dependency outside the graph");
            succ[static_cast<size_t>(it - nodes.begin())].push_back(i);
            ++indeg[i];
        }
    }
    Program* p = new (std::nothrow) Program;
    if (p == nullptr) return fail(LGCN_E_ARG, "lgcn_program_from_graph: out of host memory");
    std::vector<bool> done(n, false);
    for (size_t emitted = 0; emitted < n; ++emitted) {
        size_t pick = n;
        for (size_t i = 0; i < n; ++i)
            if (!done[i] && indeg[i] == 0) {
                pick = i;
                break;
            }
        if (pick == n) {
            delete p;
            return fail(LGCN_E_ARG, "lgcn_program_from_graph: cycle");
        }
        done[pick] = true;
        for (size_t s : succ[pick]) --indeg[s];
        Op op{};
        if (int rc = check_hip(hipGraphNodeGetType(nodes[pick], &op.type), "hipGraphNodeGetType")) {
            delete p;
            return rc;
        }
        int rc = LGCN_OK;
        switch (op.type) {
            case hipGraphNodeTypeKernel:
                rc = check_hip(hipGraphKernelNodeGetParams(nodes[pick], &op.k), "hipGraphKernelNodeGetParams");
                if (rc == LGCN_OK && (op.k.extra != nullptr || op.k.func == nullptr))
                    rc = fail(LGCN_E_UNSUPPORTED, "lgcn_program_from_graph: kernel node without kernelParams");
                ++p->launches;
                break;
            case hipGraphNodeTypeMemset:
                rc = check_hip(hipGraphMemsetNodeGetParams(nodes[pick], &op.m), "hipGraphMemsetNodeGetParams");
                if (rc == LGCN_OK && op.m.elementSize != 1 && op.m.elementSize != 2 && op.m.elementSize != 4)
                    rc = fail(LGCN_E_UNSUPPORTED, "lgcn_program_from_graph: memset of %u-byte elements",
                              op.m.elementSize);
                if (rc == LGCN_OK && op.m.height > 1 && op.m.elementSize != 1)
                    rc = fail(LGCN_E_UNSUPPORTED, "lgcn_program_from_graph: 2-D memset of wide elements");
                ++p->launches;
                break;
            case hipGraphNodeTypeEmpty:
                continue;  // a join point: the one-stream issue order already orders it
            default:
                // copies too: a captured 1-D copy's node reads back as 3-D parameters that
                // hipMemcpy3DAsync refuses (measured), and no API returns its 1-D form
                rc = fail(LGCN_E_UNSUPPORTED, "lgcn_program_from_graph: node type %d (copies, events, host "
                          "or child graphs) has no stream-launch form here", static_cast<int>(op.type));
        }
        if (rc != LGCN_OK) {
            delete p;
            return rc;
        }
        p->ops.push_back(op);
    }
    *prog_out = p;
    return LGCN_OK;
}

int lgcn_program_launches(const void* prog) {
    if (prog == nullptr) return lgcn::fail(LGCN_E_ARG, "lgcn_program_launches: null");
    return static_cast<const lgcn::Program*>(prog)->launches;
}

int lgcn_program_run(const void* prog, lgcn_stream_t stream) {
    using namespace lgcn;
    if (prog == nullptr) return fail(LGCN_E_ARG, "lgcn_program_run: null");
    hipStream_t s = as_stream(stream);
    for (const Op& op : static_cast<const Program*>(prog)->ops)
        if (int rc = issue(op, s)) return rc;
    return LGCN_OK;
}

int lgcn_program_free(void* prog) {
    delete static_cast<lgcn::Program*>(prog);
    return LGCN_OK;
}

}  // extern "C"
