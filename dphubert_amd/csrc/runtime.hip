// Error reporting and ABI version for the DPHuBERT gfx950 kernel library.
#include "common.h"

#include <stdarg.h>
#include <stdio.h>

namespace dph {
namespace {
thread_local char g_err[1024] = {0};
}

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return DPH_ELAUNCH;
  }
  return DPH_OK;
}
}  // namespace dph

extern "C" const char* dph_last_error(void) { return dph::g_err; }
extern "C" int dph_abi_version(void) { return 2; }
