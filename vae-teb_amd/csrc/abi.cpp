// Error channel and version of the VAE-TEB C ABI (include/vaeteb.h).
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <utility>
#include <vector>

#include "common.h"

namespace vt {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

unsigned arrive_slots(unsigned n, hipStream_t st) {
    static std::atomic<unsigned> next[2];
    constexpr unsigned HALF = ARRIVE_POOL / 2;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    const int cap = (st && hipStreamIsCapturing(st, &cs) == hipSuccess && cs == hipStreamCaptureStatusActive) ? 1 : 0;
    for (;;) {
        const unsigned b = next[cap].fetch_add(n) % HALF;
        if (b + n <= HALF) return b + cap * HALF;
    }
}

static std::vector<std::pair<const void*, size_t>>& arrive_pools() {
    static std::vector<std::pair<const void*, size_t>> v;
    return v;
}
int register_arrive_pool(const void* sym, size_t bytes) {
    arrive_pools().emplace_back(sym, bytes);
    return (int)arrive_pools().size();
}

static std::atomic<int> g_h16{0};   // 16-bit MFMA operand format (h16.h): 0 bf16, 1 fp16
int h16_format() { return g_h16.load(std::memory_order_relaxed); }
}  // namespace vt

extern "C" {
const char* vt_last_error(void) { return vt::g_err; }

int vt_arrive_reset(void* stream) {
    for (const auto& [sym, bytes] : vt::arrive_pools()) {
        void* p = nullptr;
        if (hipGetSymbolAddress(&p, sym) != hipSuccess || hipMemsetAsync(p, 0, bytes, vt::S(stream)) != hipSuccess) {
            vt::set_error("vt_arrive_reset: cannot clear a counter pool");
            return VT_ERR_HIP;
        }
    }
    return VT_OK;
}
int vt_abi_version(void) { return 1; }
int vt_set_h16_format(int fp16) { return vt::g_h16.exchange(fp16 ? 1 : 0); }
int vt_get_h16_format(void) { return vt::h16_format(); }
}

// ------------------------------------------------------------ stream forks
// `to` waits for everything enqueued on `from` so far: hipEventRecord of a pooled
// (timing-disabled) event + hipStreamWaitEvent — what torch's Stream.wait_stream
// does, without creating a Python Event per fork (~2 us instead of ~15 us on the
// host; the model forks / joins its side streams ~60 times per training step).
// The wait captures the event's state when it is enqueued, so an event may be
// re-recorded once its waits are enqueued; the ring is far larger than the forks
// of one step.  Under hipGraph capture both calls become graph dependencies.
namespace {
constexpr int kForkEvents = 1024, kMaxDevices = 16;
// one ring per device (an event is created on, and may only be recorded on streams of,
// the device current at its creation); the index advances atomically, so marks from
// several host threads take distinct slots.  slot = device * kForkEvents + index.
hipEvent_t g_fork_ev[kMaxDevices][kForkEvents];
std::atomic<unsigned> g_fork_next[kMaxDevices];

// Capture bookkeeping of every slot: the capture sequence id of the
// stream that last recorded the slot (0: recorded outside any capture) and that stream.  A
// wait is legal only inside the capture that recorded the slot (or, outside captures, on a
// slot recorded outside one); anything else is reported as VT_ERR_HIP with the slot's
// history instead of reaching the runtime.  VAETEB_EVENT_TRACE=1 also prints every mark /
// wait to stderr.
struct SlotRec {
    unsigned long long cap;
    void* stream;
};
SlotRec g_slot[kMaxDevices][kForkEvents];
int g_trace = -1;

unsigned long long capture_id(void* stream, bool* capturing) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    if (hipStreamGetCaptureInfo((hipStream_t)stream, &st, &id) != hipSuccess) {
        (void)hipGetLastError();
        st = hipStreamCaptureStatusNone;
    }
    *capturing = st == hipStreamCaptureStatusActive;
    return *capturing ? id : 0ull;
}

bool trace() {
    if (g_trace < 0) {
        const char* e = getenv("VAETEB_EVENT_TRACE");
        g_trace = e && e[0] == '1';
    }
    return g_trace;
}
}  // namespace

extern "C" int vt_stream_mark(void* stream, int* slot) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) {
        vt::set_error("vt_stream_mark: device %d (at most %d devices)", dev, kMaxDevices);
        return VT_ERR_ARG;
    }
    const int i = (int)(g_fork_next[dev].fetch_add(1, std::memory_order_relaxed) % kForkEvents);
    hipEvent_t& ev = g_fork_ev[dev][i];
    if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
        vt::set_error("vt_stream_mark: hipEventCreateWithFlags failed");
        return VT_ERR_HIP;
    }
    bool capturing = false;
    const unsigned long long cap = capture_id(stream, &capturing);
    if (hipEventRecord(ev, (hipStream_t)stream) != hipSuccess) {
        vt::set_error("vt_stream_mark: %s", hipGetErrorString(hipGetLastError()));
        return VT_ERR_HIP;
    }
    g_slot[dev][i] = SlotRec{cap, stream};
    if (trace()) fprintf(stderr, "[vt_event] mark slot %d event %p stream %p capture %llu\n", dev * kForkEvents + i,
                         (void*)ev, stream, cap);
    *slot = dev * kForkEvents + i;
    return VT_OK;
}

extern "C" int vt_stream_wait_mark(void* stream, int slot) {
    const int dev = slot / kForkEvents, i = slot % kForkEvents;
    if (slot < 0 || dev >= kMaxDevices || !g_fork_ev[dev][i]) {
        vt::set_error("vt_stream_wait_mark: bad slot %d", slot);
        return VT_ERR_ARG;
    }
    bool capturing = false;
    const unsigned long long cap = capture_id(stream, &capturing);
    const SlotRec& r = g_slot[dev][i];
    if (trace()) fprintf(stderr, "[vt_event] wait slot %d event %p stream %p capture %llu (recorded on %p capture %llu)\n",
                         slot, (void*)g_fork_ev[dev][i], stream, cap, r.stream, r.cap);
    // legal: the same capture; a non-capturing stream joining the capture the slot was recorded
    // in (while that capture is active); a capturing stream waiting on a slot recorded outside
    // any capture (an external dependency).  Not: a slot recorded in ANOTHER capture, or in a
    // capture that has ended.
    bool bad = cap != 0 && r.cap != 0 && r.cap != cap;
    if (cap == 0 && r.cap != 0) {
        bool rec_capturing = false;
        bad = capture_id(r.stream, &rec_capturing) != r.cap;
    }
    if (bad) {
        vt::set_error("vt_stream_wait_mark: slot %d was recorded on stream %p in capture %llu; the wait on stream %p "
                      "is in capture %llu (0 = none): not the recording capture, or that capture has ended",
                      slot, r.stream, r.cap, stream, cap);
        return VT_ERR_HIP;
    }
    if (hipStreamWaitEvent((hipStream_t)stream, g_fork_ev[dev][i], 0) != hipSuccess) {
        vt::set_error("vt_stream_wait_mark: %s", hipGetErrorString(hipGetLastError()));
        return VT_ERR_HIP;
    }
    return VT_OK;
}

extern "C" int vt_stream_fork(void* from, void* to) {
    int slot;
    const int rc = vt_stream_mark(from, &slot);
    return rc != VT_OK ? rc : vt_stream_wait_mark(to, slot);
}

// ------------------------------------------------------------ capture inspection
// Diagnostic (tools/capture_probe.py model_head_info): the capture state of
// `stream` — status, capture id, the captured graph's node count by type, the stream's current
// dependency set (the nodes its next captured operation would depend on: type, and for kernel
// nodes the grid / block / dynamic LDS), and every kernel node of the graph with an empty grid or
// block — written as text into buf.  Reads the graph under capture, never modifies it.
extern "C" int vt_capture_info(void* stream, char* buf, int len) {
    if (!buf || len <= 0) return VT_ERR_ARG;
    int o = 0;
    auto put = [&](const char* fmt, auto... a) {
        if (o < len) o += snprintf(buf + o, (size_t)(len - o), fmt, a...);
    };
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    hipGraph_t g = nullptr;
    const hipGraphNode_t* deps = nullptr;
    size_t nd = 0;
    const hipError_t e = hipStreamGetCaptureInfo_v2((hipStream_t)stream, &st, &id, &g, &deps, &nd);
    put("stream %p: %s status %d capture %llu", stream, hipGetErrorString(e), (int)st, id);
    if (e != hipSuccess || st != hipStreamCaptureStatusActive || !g) return VT_OK;
    auto kern = [&](hipGraphNode_t n) {
        hipKernelNodeParams p{};
        if (hipGraphKernelNodeGetParams(n, &p) == hipSuccess)
            put(" kernel fn %p grid %ux%ux%u block %ux%ux%u lds %u", p.func, p.gridDim.x, p.gridDim.y, p.gridDim.z,
                p.blockDim.x, p.blockDim.y, p.blockDim.z, p.sharedMemBytes);
    };
    size_t nn = 0;
    (void)hipGraphGetNodes(g, nullptr, &nn);
    std::vector<hipGraphNode_t> nodes(nn);
    if (nn) (void)hipGraphGetNodes(g, nodes.data(), &nn);
    int count[32] = {0}, empty_kernels = 0;
    for (size_t i = 0; i < nn; ++i) {
        hipGraphNodeType t = hipGraphNodeTypeEmpty;
        (void)hipGraphNodeGetType(nodes[i], &t);
        count[(int)t & 31]++;
        if (t == hipGraphNodeTypeKernel) {
            hipKernelNodeParams p{};
            if (hipGraphKernelNodeGetParams(nodes[i], &p) == hipSuccess &&
                (p.gridDim.x * p.gridDim.y * p.gridDim.z == 0 || p.blockDim.x * p.blockDim.y * p.blockDim.z == 0)) {
                ++empty_kernels;
                put("\n  EMPTY-GRID node %zu:", i);
                kern(nodes[i]);
            }
        }
    }
    put("\n  graph %p: %zu nodes; by type:", (void*)g, nn);
    for (int t = 0; t < 32; ++t)
        if (count[t]) put(" [%d]=%d", t, count[t]);
    put(" (0 kernel, 1 memcpy, 2 memset, 3 host, 4 graph, 5 empty, 6 wait-event, 7 event-record); empty grids %d",
        empty_kernels);
    put("\n  dependencies of the next captured op: %zu", nd);
    for (size_t i = 0; i < nd; ++i) {
        hipGraphNodeType t = hipGraphNodeTypeEmpty;
        (void)hipGraphNodeGetType(deps[i], &t);
        size_t ndep = 0, nchild = 0;
        (void)hipGraphNodeGetDependencies(deps[i], nullptr, &ndep);
        (void)hipGraphNodeGetDependentNodes(deps[i], nullptr, &nchild);
        put("\n   dep %zu: node %p type %d (%zu deps, %zu dependents)", i, (void*)deps[i], (int)t, ndep, nchild);
        if (t == hipGraphNodeTypeKernel) kern(deps[i]);
    }
    return VT_OK;
}
