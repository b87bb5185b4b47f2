// ABI housekeeping: version, thread-local last-error message, launch status.
#include <stdarg.h>
#include <stdio.h>

#include "vm_common.h"

namespace {
thread_local char g_err[512] = "";
}

namespace vmhost {
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: HIP launch failed: %s", what, hipGetErrorString(e));
    return VM_E_LAUNCH;
  }
  return VM_OK;
}
}  // namespace vmhost

extern "C" int vm_abi_version(void) { return VM_ABI_VERSION; }
extern "C" const char* vm_last_error(void) { return g_err; }
