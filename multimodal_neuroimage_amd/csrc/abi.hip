// ABI bookkeeping of libmmni.so: version and the thread-local last-error message.
#include "mmni_common.h"

namespace mmni {
static thread_local char g_last_error[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
    va_end(ap);
}
}  // namespace mmni

extern "C" int mmni_version(void) { return MMNI_ABI_VERSION; }
extern "C" const char* mmni_last_error(void) { return mmni::g_last_error; }
