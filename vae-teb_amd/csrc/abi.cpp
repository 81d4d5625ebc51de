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
