// Error channel and version of the pis_* C-ABI (include/pis_capi.h).
#include <cstdarg>

#include "common.h"

namespace pis {
static thread_local char g_last_error[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
}
}  // namespace pis

extern "C" const char* pis_last_error(void) { return pis::g_last_error; }
extern "C" int pis_version(void) { return 1; }
