// Error channel and version of the VAE-TEB C ABI (include/vaeteb.h).
#include <stdarg.h>
#include <stdio.h>

#include <atomic>

#include "common.h"

namespace vt {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
}  // namespace vt

extern "C" {
const char* vt_last_error(void) { return vt::g_err; }
int vt_abi_version(void) { return 1; }
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
    if (hipEventRecord(ev, (hipStream_t)stream) != hipSuccess) {
        vt::set_error("vt_stream_mark: %s", hipGetErrorString(hipGetLastError()));
        return VT_ERR_HIP;
    }
    *slot = dev * kForkEvents + i;
    return VT_OK;
}

extern "C" int vt_stream_wait_mark(void* stream, int slot) {
    const int dev = slot / kForkEvents, i = slot % kForkEvents;
    if (slot < 0 || dev >= kMaxDevices || !g_fork_ev[dev][i]) {
        vt::set_error("vt_stream_wait_mark: bad slot %d", slot);
        return VT_ERR_ARG;
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
