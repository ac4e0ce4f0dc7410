// C ABI utilities: error reporting and version (include/d2d_hip.h).
#include <cstdarg>
#include <cstdio>

#include "d2d_hip.h"

static thread_local char g_err[512] = "";

void d2d_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

extern "C" const char* d2d_last_error(void) { return g_err; }

extern "C" int d2d_abi_version(void) { return D2D_ABI_VERSION; }
