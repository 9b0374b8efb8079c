// Error reporting and version entry points of the C ABI.
#include <cstdarg>
#include <cstdio>

#include "sa_internal.h"

namespace sa {
static thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int check_hip(hipError_t e, const char* what) {
  if (e == hipSuccess) return SA_OK;
  return fail(SA_EHIP, "%s: %s", what, hipGetErrorString(e));
}

int check_launch(const char* what) { return check_hip(hipGetLastError(), what); }
}  // namespace sa

extern "C" int sa_abi_version(void) { return SA_ABI_VERSION; }
extern "C" const char* sa_last_error(void) { return sa::g_err; }
