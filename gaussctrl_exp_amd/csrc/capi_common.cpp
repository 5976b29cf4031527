// capi_common.cpp -- error plumbing and version for the C ABI (include/gsplat_mi355x.h).
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

namespace gs {

int g_quirks = GSPLAT_QUIRKS_ALL;

static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

static thread_local hipError_t g_noted = hipSuccess;
static thread_local const char *g_noted_what = "";

void note(hipError_t e, const char *what) {
  if (e != hipSuccess && g_noted == hipSuccess) {
    g_noted = e;
    g_noted_what = what;
  }
}

int check_launch(const char *what) {
  hipError_t e = hipGetLastError();
  if (g_noted != hipSuccess) {
    set_error("%s: %s failed: %s", what, g_noted_what, hipGetErrorString(g_noted));
    g_noted = hipSuccess;
    return 1;
  }
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return 1;
  }
  return 0;
}

}  // namespace gs

extern "C" int gsplat_abi_version(void) { return GSPLAT_MI355X_ABI_VERSION; }
extern "C" const char *gsplat_last_error(void) { return gs::g_err; }

extern "C" int gsplat_set_quirks(int mask) {
  if (mask & ~GSPLAT_QUIRKS_ALL) {
    gs::set_error("gsplat_set_quirks: unknown bits 0x%x", mask & ~GSPLAT_QUIRKS_ALL);
    return 1;
  }
  gs::g_quirks = mask;
  return 0;
}
extern "C" int gsplat_get_quirks(void) { return gs::g_quirks; }
