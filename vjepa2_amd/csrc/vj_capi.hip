// C ABI plumbing of libvjepa_hip.so: version, thread-local last-error string.
// Every entry point returns 0 (VJ_OK) or an error code and never exits the process.
#include <stdarg.h>
#include "vj_common.h"

static thread_local char g_err[1024] = {0};

void vj_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

extern "C" int vj_version(void) { return 1; }

// CRC-32 of include/vjepa_hip.h when this library was built (build.py passes it): the Python binding
// compares it with the header it types the entry points from, so a library left stale after a
// signature change fails loudly instead of taking misplaced arguments.
#ifndef VJ_HEADER_CRC
#define VJ_HEADER_CRC 0
#endif
extern "C" int vj_header_crc(void) { return (int)(unsigned)VJ_HEADER_CRC; }

extern "C" int vj_get_last_error(char* buf, size_t n) {
  if (!buf || n == 0) return VJ_ERR_ARG;
  strncpy(buf, g_err, n - 1);
  buf[n - 1] = 0;
  return VJ_OK;
}

extern "C" int vj_device_sync(void) {
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    vj_set_error("hipDeviceSynchronize: %s", hipGetErrorString(e));
    return VJ_ERR_LAUNCH;
  }
  return VJ_OK;
}
