// Error channel and version of the VAE-TEB C ABI (include/vaeteb.h).
#include <stdarg.h>
#include <stdio.h>

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
constexpr int kForkEvents = 1024;
hipEvent_t g_fork_ev[kForkEvents];
int g_fork_next = 0;
}  // namespace

extern "C" int vt_stream_mark(void* stream, int* slot) {
    const int i = g_fork_next;
    g_fork_next = (i + 1) % kForkEvents;
    if (!g_fork_ev[i] && hipEventCreateWithFlags(&g_fork_ev[i], hipEventDisableTiming) != hipSuccess) {
        vt::set_error("vt_stream_mark: hipEventCreateWithFlags failed");
        return VT_ERR_HIP;
    }
    if (hipEventRecord(g_fork_ev[i], (hipStream_t)stream) != hipSuccess) {
        vt::set_error("vt_stream_mark: %s", hipGetErrorString(hipGetLastError()));
        return VT_ERR_HIP;
    }
    *slot = i;
    return VT_OK;
}

extern "C" int vt_stream_wait_mark(void* stream, int slot) {
    if (slot < 0 || slot >= kForkEvents || !g_fork_ev[slot]) {
        vt::set_error("vt_stream_wait_mark: bad slot %d", slot);
        return VT_ERR_ARG;
    }
    if (hipStreamWaitEvent((hipStream_t)stream, g_fork_ev[slot], 0) != hipSuccess) {
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
