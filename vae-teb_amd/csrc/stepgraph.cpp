// Native multi-stream executor for a captured training step.
//
// The eager step enqueues ~500 kernels across 3-4 HIP streams from Python
// (~10 ms of host dispatch per step, as long as the GPU work itself).  A
// captured hipGraph replays with almost no host cost, but ROCm's graph launch
// runs the step's independent branches with far less overlap than the eager
// streams do (measured: 21 % of the replay with no kernel running, 28 % with
// two, vs 2 % / 61 % eager), so the replay is slower on the GPU.  This
// executor takes the captured graph (torch.cuda.CUDAGraph(keep_graph=True)
// .raw_cuda_graph()), topologically orders its nodes in capture order, assigns
// them to N streams (greedy: a node follows its most recent dependency's
// stream when that stream has not moved on, else the least-recently-used
// stream), and keeps only the cross-stream dependencies that no earlier wait
// already implies (transitive per-stream frontiers) as event waits.  A launch
// is then one C++ loop of hipLaunchKernel / memcpy / memset calls and event
// record / waits on the caller's stream plus N-1 internal streams, bracketed
// by a fork from and a join back into the caller's stream (the other streams
// are the caller's too, e.g. the side streams the eager step uses: each HIP
// stream is bound to one of the process's 4 hardware queues at creation, and
// two of the executor's streams sharing a queue would serialise): stream-ordered like
// any other launch, the same kernels with the same arguments (the graph's
// private memory pool fixes every address), so a replay is bit-identical to
// the eager step.  Kernel arguments point into the graph's node storage: the
// CUDAGraph object must outlive the executor.
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <queue>
#include <vector>

#include "common.h"

namespace vt {
namespace {

enum OpKind { OP_KERNEL = 0, OP_MEMCPY = 1, OP_MEMSET = 2, OP_MARK = 3 };

struct Op {
    int kind = OP_KERNEL;
    hipKernelNodeParams kp{};
    void* cdst = nullptr;     // 1-D memcpy
    const void* csrc = nullptr;
    size_t cbytes = 0;
    hipMemcpyKind ckind = hipMemcpyDefault;
    hipMemsetParams sp{};
    int stream = 0;
    int bucket = -1;          // OP_MARK: the gradient bucket whose writers it joins
    int record = -1;          // event recorded after this op (-1: none)
    std::vector<int> waits;   // events this op's stream waits on before it
};

struct StepGraph {
    int n_streams = 0;        // compute streams; markers run on one more (index n_streams)
    bool has_comm = false;
    std::vector<Op> ops;
    std::vector<hipEvent_t> events;
    hipEvent_t fork = nullptr;
    std::vector<hipEvent_t> join;
    int n_kernel = 0, n_memcpy = 0, n_memset = 0, n_waits = 0;
};

#define SG_TRY(expr, msg)                                                \
    do {                                                                 \
        hipError_t e_ = (expr);                                          \
        if (e_ != hipSuccess) {                                          \
            set_error("vt_stepgraph: %s: %s", msg, hipGetErrorString(e_)); \
            return VT_ERR_HIP;                                           \
        }                                                                \
    } while (0)

int build(hipGraph_t g, int n_streams, StepGraph* sg) {
    size_t n = 0;
    SG_TRY(hipGraphGetNodes(g, nullptr, &n), "hipGraphGetNodes");
    std::vector<hipGraphNode_t> nodes(n);
    if (n) SG_TRY(hipGraphGetNodes(g, nodes.data(), &n), "hipGraphGetNodes");
    std::vector<int> type(n);
    std::vector<std::vector<int>> deps(n);
    auto index_of = [&](hipGraphNode_t x) {
        // nodes are few hundred: a linear scan per dependency is cheap at build time
        for (size_t i = 0; i < n; ++i)
            if (nodes[i] == x) return (int)i;
        return -1;
    };
    for (size_t i = 0; i < n; ++i) {
        hipGraphNodeType t;
        SG_TRY(hipGraphNodeGetType(nodes[i], &t), "hipGraphNodeGetType");
        type[i] = (int)t;
        if (t != hipGraphNodeTypeKernel && t != hipGraphNodeTypeMemcpy && t != hipGraphNodeTypeMemset &&
            t != hipGraphNodeTypeEmpty) {
            set_error("vt_stepgraph: unsupported graph node type %d", (int)t);
            return VT_ERR_ARG;
        }
        size_t nd = 0;
        SG_TRY(hipGraphNodeGetDependencies(nodes[i], nullptr, &nd), "hipGraphNodeGetDependencies");
        std::vector<hipGraphNode_t> d(nd);
        if (nd) SG_TRY(hipGraphNodeGetDependencies(nodes[i], d.data(), &nd), "hipGraphNodeGetDependencies");
        for (auto x : d) {
            const int j = index_of(x);
            if (j < 0) {
                set_error("vt_stepgraph: dependency outside the graph");
                return VT_ERR_ARG;
            }
            deps[i].push_back(j);
        }
    }
    // topological order, ties by capture (node) order
    std::vector<int> indeg(n, 0);
    std::vector<std::vector<int>> succ(n);
    for (size_t i = 0; i < n; ++i)
        for (int d : deps[i]) {
            succ[d].push_back((int)i);
            ++indeg[i];
        }
    std::priority_queue<int, std::vector<int>, std::greater<int>> ready;
    for (size_t i = 0; i < n; ++i)
        if (!indeg[i]) ready.push((int)i);
    std::vector<int> order;
    while (!ready.empty()) {
        const int i = ready.top();
        ready.pop();
        order.push_back(i);
        for (int s : succ[i])
            if (--indeg[s] == 0) ready.push(s);
    }
    if (order.size() != n) {
        set_error("vt_stepgraph: graph has a cycle");
        return VT_ERR_ARG;
    }
    if (getenv("VAETEB_STEPGRAPH_DEBUG")) {  // the non-kernel nodes and their capture-order neighbours
        auto kname = [&](int k) -> const char* {
            if (k < 0 || k >= (int)n || type[k] != hipGraphNodeTypeKernel) return "-";
            hipKernelNodeParams kp{};
            if (hipGraphKernelNodeGetParams(nodes[k], &kp) != hipSuccess) return "?";
            const char* nm = hipKernelNameRefByPtr(kp.func, nullptr);
            return nm ? nm : "?";
        };
        for (size_t k = 0; k < order.size(); ++k) {
            const int i = order[k];
            if (type[i] == hipGraphNodeTypeKernel || type[i] == hipGraphNodeTypeEmpty) continue;
            fprintf(stderr, "stepgraph node %d type %d after [%.90s] before [%.90s]\n", i, type[i],
                    kname(k > 0 ? order[k - 1] : -1), kname(k + 1 < order.size() ? order[k + 1] : -1));
        }
    }
    // empty nodes: replace by their (resolved) dependencies
    std::vector<std::vector<int>> rdeps(n);
    for (int i : order) {
        std::vector<int> r;
        for (int d : deps[i]) {
            if (type[d] == hipGraphNodeTypeEmpty)
                r.insert(r.end(), rdeps[d].begin(), rdeps[d].end());
            else
                r.push_back(d);
        }
        std::sort(r.begin(), r.end());
        r.erase(std::unique(r.begin(), r.end()), r.end());
        rdeps[i] = r;
    }
    // gradient-bucket markers (vt_bucket_marker): not launched; they go to an extra
    // stream (index n_streams) that only waits for the bucket's writers
    const void* mark_fn = bucket_marker_kernel();
    std::vector<int> mark_bucket(n, -1);
    bool any_mark = false;
    for (size_t i = 0; i < n; ++i) {
        if (type[i] != hipGraphNodeTypeKernel) continue;
        hipKernelNodeParams kp{};
        SG_TRY(hipGraphKernelNodeGetParams(nodes[i], &kp), "hipGraphKernelNodeGetParams");
        if (kp.func == mark_fn && kp.kernelParams && kp.kernelParams[0]) {
            mark_bucket[i] = *(const int*)kp.kernelParams[0];
            any_mark = true;
        }
    }
    // stream assignment with per-stream frontiers: seen[s][x] = number of ops of
    // stream x known complete before the next op of stream s (transitively)
    const int S = n_streams + (any_mark ? 1 : 0);
    const int SC = n_streams;   // streams a compute op may take
    std::vector<int> op_of(n, -1), pos(n, 0), cnt(S, 0), tail(S, -1), last_use(S, -1);
    std::vector<std::vector<int>> seen(S, std::vector<int>(S, 0));
    std::vector<std::vector<int>> snap(n);
    std::vector<int> event_of(n, -1);
    int n_events = 0;
    sg->ops.clear();
    int tick = 0;
    for (int i : order) {
        if (type[i] == hipGraphNodeTypeEmpty) continue;
        int s = -1, best_d = -1;
        if (mark_bucket[i] >= 0) {
            s = SC;
        } else {
            for (int d : rdeps[i]) {  // follow the most recent dependency whose stream has not moved on
                const int x = sg->ops[op_of[d]].stream;
                if (x < SC && tail[x] == d && d > best_d) {
                    best_d = d;
                    s = x;
                }
            }
        }
        if (s < 0) {  // the least recently used stream (an unused one first)
            s = 0;
            for (int x = 1; x < SC; ++x)
                if (last_use[x] < last_use[s]) s = x;
        }
        Op op;
        op.stream = s;
        // waits, latest dependency first per stream
        std::vector<int> ds = rdeps[i];
        std::sort(ds.begin(), ds.end(), [&](int a, int b) { return pos[a] > pos[b]; });
        for (int d : ds) {
            const int x = sg->ops[op_of[d]].stream;
            if (x == s || seen[s][x] >= pos[d]) continue;
            if (event_of[d] < 0) {
                event_of[d] = n_events++;
                sg->ops[op_of[d]].record = event_of[d];
            }
            op.waits.push_back(event_of[d]);
            for (int y = 0; y < S; ++y) seen[s][y] = std::max(seen[s][y], snap[d][y]);
        }
        const hipGraphNode_t nd = nodes[i];
        if (mark_bucket[i] >= 0) {
            op.kind = OP_MARK;
            op.bucket = mark_bucket[i];
        } else if (type[i] == hipGraphNodeTypeKernel) {
            op.kind = OP_KERNEL;
            SG_TRY(hipGraphKernelNodeGetParams(nd, &op.kp), "hipGraphKernelNodeGetParams");
            if (op.kp.kernelParams == nullptr || op.kp.func == nullptr) {
                set_error("vt_stepgraph: kernel node without kernelParams");
                return VT_ERR_ARG;
            }
            ++sg->n_kernel;
        } else if (type[i] == hipGraphNodeTypeMemcpy) {
            op.kind = OP_MEMCPY;
            // hipMemcpyAsync captures as a 1-D node: read back through the driver-style
            // getter (hipGraphMemcpyNodeGetParams does not describe 1-D nodes)
            HIP_MEMCPY3D dp{};
            SG_TRY(hipDrvGraphMemcpyNodeGetParams(nd, &dp), "hipDrvGraphMemcpyNodeGetParams");
            const void* src = dp.srcMemoryType == hipMemoryTypeHost ? dp.srcHost : (const void*)dp.srcDevice;
            void* dst = dp.dstMemoryType == hipMemoryTypeHost ? dp.dstHost : (void*)dp.dstDevice;
            if (dp.srcArray || dp.dstArray || dp.Height > 1 || dp.Depth > 1 || dp.srcY || dp.srcZ || dp.dstY ||
                dp.dstZ || !src || !dst || !dp.WidthInBytes) {
                set_error("vt_stepgraph: memcpy node is not a 1-D linear copy (width %zu height %zu depth %zu, "
                          "src %p type %d, dst %p type %d)", dp.WidthInBytes, dp.Height, dp.Depth, src,
                          (int)dp.srcMemoryType, dst, (int)dp.dstMemoryType);
                return VT_ERR_ARG;
            }
            op.cdst = (char*)dst + dp.dstXInBytes;
            op.csrc = (const char*)src + dp.srcXInBytes;
            op.cbytes = dp.WidthInBytes;
            op.ckind = hipMemcpyDefault;
            ++sg->n_memcpy;
        } else {
            op.kind = OP_MEMSET;
            SG_TRY(hipGraphMemsetNodeGetParams(nd, &op.sp), "hipGraphMemsetNodeGetParams");
            if (op.sp.height > 1 || (op.sp.elementSize != 1 && op.sp.elementSize != 2 && op.sp.elementSize != 4)) {
                set_error("vt_stepgraph: 2-D memset node");
                return VT_ERR_ARG;
            }
            ++sg->n_memset;
        }
        sg->n_waits += (int)op.waits.size();
        pos[i] = ++cnt[s];
        seen[s][s] = pos[i];
        snap[i] = seen[s];
        tail[s] = i;
        last_use[s] = tick++;
        op_of[i] = (int)sg->ops.size();
        sg->ops.push_back(op);
    }
    sg->n_streams = SC;
    sg->has_comm = any_mark;
    sg->events.assign(n_events, nullptr);
    for (auto& e : sg->events) SG_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    SG_TRY(hipEventCreateWithFlags(&sg->fork, hipEventDisableTiming), "hipEventCreate");
    sg->join.assign(S, nullptr);   // S includes the marker stream
    for (auto& e : sg->join) SG_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    return VT_OK;
}

void destroy(StepGraph* sg) {
    for (auto e : sg->events) (void)hipEventDestroy(e);
    for (auto e : sg->join) (void)hipEventDestroy(e);
    if (sg->fork) (void)hipEventDestroy(sg->fork);
    delete sg;
}

int launch(StepGraph* sg, const hipStream_t* st, int begin, int end, int flags) {
    const hipStream_t caller = st[0];
    const int S = sg->n_streams + (sg->has_comm ? 1 : 0);
    if (flags & 1) {
        SG_TRY(hipEventRecord(sg->fork, caller), "fork record");
        for (int s = 1; s < S; ++s) SG_TRY(hipStreamWaitEvent(st[s], sg->fork, 0), "fork wait");
    }
    for (int k = begin; k < end; ++k) {
        const Op& op = sg->ops[k];
        hipStream_t q = st[op.stream];
        for (int e : op.waits) SG_TRY(hipStreamWaitEvent(q, sg->events[e], 0), "wait");
        if (op.kind == OP_MARK) {
            // not launched: the stream has now joined the bucket's writers
        } else if (op.kind == OP_KERNEL) {
            SG_TRY(hipLaunchKernel(op.kp.func, op.kp.gridDim, op.kp.blockDim, op.kp.kernelParams,
                                   op.kp.sharedMemBytes, q),
                   "hipLaunchKernel");
        } else if (op.kind == OP_MEMCPY) {
            SG_TRY(hipMemcpyAsync(op.cdst, op.csrc, op.cbytes, op.ckind, q), "hipMemcpyAsync");
        } else if (op.sp.elementSize == 1) {
            SG_TRY(hipMemsetAsync(op.sp.dst, (int)op.sp.value, op.sp.width, q), "hipMemsetAsync");
        } else if (op.sp.elementSize == 2) {
            SG_TRY(hipMemsetD16Async((hipDeviceptr_t)op.sp.dst, (unsigned short)op.sp.value, op.sp.width, q),
                   "hipMemsetD16Async");
        } else {
            SG_TRY(hipMemsetD32Async((hipDeviceptr_t)op.sp.dst, (int)op.sp.value, op.sp.width, q),
                   "hipMemsetD32Async");
        }
        if (op.record >= 0) SG_TRY(hipEventRecord(sg->events[op.record], q), "record");
    }
    if (flags & 2) {
        for (int s = 1; s < S; ++s) {
            SG_TRY(hipEventRecord(sg->join[s], st[s]), "join record");
            SG_TRY(hipStreamWaitEvent(caller, sg->join[s], 0), "join wait");
        }
    }
    return VT_OK;
}

}  // namespace
}  // namespace vt

using namespace vt;

extern "C" {

int vt_stepgraph_build(void* graph, int n_streams, void** handle) {
    VT_CHECK_ARG(graph && handle && n_streams >= 1 && n_streams <= 8, "vt_stepgraph_build: args (1..8 streams)");
    StepGraph* sg = new StepGraph();
    const int rc = build((hipGraph_t)graph, n_streams, sg);
    if (rc != VT_OK) {
        destroy(sg);
        return rc;
    }
    *handle = sg;
    return VT_OK;
}

int vt_stepgraph_launch(void* handle, void* const* streams) {
    VT_CHECK_ARG(handle != nullptr && streams != nullptr, "vt_stepgraph_launch: null handle / streams");
    const StepGraph* sg = (const StepGraph*)handle;
    const int S = sg->n_streams + (sg->has_comm ? 1 : 0);
    for (int s = 1; s < S; ++s)
        VT_CHECK_ARG(streams[s] != streams[0], "vt_stepgraph_launch: stream %d is the caller's stream", s);
    return launch((StepGraph*)handle, (const hipStream_t*)streams, 0, (int)sg->ops.size(), 3);
}

int vt_stepgraph_launch_range(void* handle, void* const* streams, int begin, int end, int flags) {
    VT_CHECK_ARG(handle != nullptr && streams != nullptr, "vt_stepgraph_launch_range: null handle / streams");
    const StepGraph* sg = (const StepGraph*)handle;
    VT_CHECK_ARG(begin >= 0 && begin <= end && end <= (int)sg->ops.size() && flags >= 0 && flags <= 3,
                 "vt_stepgraph_launch_range: range [%d, %d) of %d ops, flags %d", begin, end, (int)sg->ops.size(),
                 flags);
    const int S = sg->n_streams + (sg->has_comm ? 1 : 0);
    for (int s = 1; s < S; ++s)
        VT_CHECK_ARG(streams[s] != streams[0], "vt_stepgraph_launch_range: stream %d is the caller's stream", s);
    return launch((StepGraph*)handle, (const hipStream_t*)streams, begin, end, flags);
}

int vt_stepgraph_markers(void* handle, int* n_ops, int* n_markers, int* ends, int* buckets, int cap) {
    VT_CHECK_ARG(handle && n_ops && n_markers && cap >= 0 && (cap == 0 || (ends && buckets)),
                 "vt_stepgraph_markers: args");
    const StepGraph* sg = (const StepGraph*)handle;
    *n_ops = (int)sg->ops.size();
    int m = 0;
    for (int k = 0; k < (int)sg->ops.size(); ++k) {
        if (sg->ops[k].kind != OP_MARK) continue;
        if (m < cap) {
            ends[m] = k + 1;
            buckets[m] = sg->ops[k].bucket;
        }
        ++m;
    }
    *n_markers = m;
    return VT_OK;
}

int vt_stepgraph_info(void* handle, int* n_kernel, int* n_memcpy, int* n_memset, int* n_waits) {
    VT_CHECK_ARG(handle && n_kernel && n_memcpy && n_memset && n_waits, "vt_stepgraph_info: args");
    const StepGraph* sg = (const StepGraph*)handle;
    *n_kernel = sg->n_kernel;
    *n_memcpy = sg->n_memcpy;
    *n_memset = sg->n_memset;
    *n_waits = sg->n_waits;
    return VT_OK;
}

int vt_stepgraph_destroy(void* handle) {
    if (handle) destroy((StepGraph*)handle);
    return VT_OK;
}

}  // extern "C"
