// ABI housekeeping: version, thread-local last-error message, launch status.
#include <stdarg.h>
#include <stdio.h>

#include <atomic>

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

int device_cus(hipStream_t stream) {
  static std::atomic<int> cached[64];
  int dev = 0;
  if (stream) {
    if (hipStreamGetDevice(stream, &dev) != hipSuccess) return 0;
  } else if (hipGetDevice(&dev) != hipSuccess) {
    return 0;
  }
  if (dev < 0 || dev >= 64) return 0;
  int n = cached[dev].load(std::memory_order_relaxed);
  if (!n) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    cached[dev].store(n, std::memory_order_relaxed);
  }
  return n;
}
}  // namespace vmhost

extern "C" int vm_abi_version(void) { return VM_ABI_VERSION; }
extern "C" const char* vm_last_error(void) { return g_err; }
