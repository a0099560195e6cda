// Error reporting and version for libdgc_hip.so. The per-kernel entry points live
// next to their kernels (compensate.hip, select.hip, decompress.hip).
#include <cstdarg>

#include "dgc_common.hpp"

namespace dgc {

static thread_local char g_last_error[1024] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
    va_end(ap);
}

}  // namespace dgc

extern "C" const char* dgc_last_error(void) { return dgc::g_last_error; }

extern "C" const char* dgc_version(void) { return "dgc_hip 0.1 gfx950"; }
