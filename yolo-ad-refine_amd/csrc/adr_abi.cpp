// Error plumbing and ABI version for libadr_hip.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include "../../include/adr.h"

namespace adr {
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
    set_error("%s: HIP launch failed: %s", what, hipGetErrorString(e));
    return ADR_ERR_LAUNCH;
  }
  return ADR_OK;
}
}  // namespace adr

extern "C" int adr_abi_version(void) { return ADR_ABI_VERSION; }
extern "C" const char* adr_last_error(void) { return adr::g_err; }

extern "C" int adr_memset_zero(void* ptr, size_t bytes, void* stream) {
  if (!ptr || !bytes) return ADR_OK;
  hipError_t e = hipMemsetAsync(ptr, 0, bytes, (hipStream_t)stream);
  if (e != hipSuccess) {
    adr::set_error("adr_memset_zero: %s", hipGetErrorString(e));
    return ADR_ERR_LAUNCH;
  }
  return ADR_OK;
}
