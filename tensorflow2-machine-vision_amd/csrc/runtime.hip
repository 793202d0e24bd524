// Library-level entry points: error reporting, ABI version, async memset.
#include <stdarg.h>
#include <stdio.h>
#include "common.hpp"

namespace edet {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return EDET_EHIP;
  }
  return EDET_OK;
}

}  // namespace edet

extern "C" {

const char* edet_last_error(void) { return edet::g_err; }

int edet_abi_version(void) { return 2; }

int edet_memset_async(void* p, int value, size_t bytes, edet_stream_t stream) {
  if (bytes == 0) return EDET_OK;
  EDET_REQUIRE(p != nullptr, "edet_memset_async: null pointer");
  hipError_t e = hipMemsetAsync(p, value, bytes, (hipStream_t)stream);
  if (e != hipSuccess) {
    edet::set_error("hipMemsetAsync: %s", hipGetErrorString(e));
    return EDET_EHIP;
  }
  return EDET_OK;
}

int edet_memcpy_async(void* dst, const void* src, size_t bytes, edet_stream_t stream) {
  if (bytes == 0) return EDET_OK;
  EDET_REQUIRE(dst && src, "edet_memcpy_async: null pointer");
  hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream);
  if (e != hipSuccess) {
    edet::set_error("hipMemcpyAsync: %s", hipGetErrorString(e));
    return EDET_EHIP;
  }
  return EDET_OK;
}

}  // extern "C"
