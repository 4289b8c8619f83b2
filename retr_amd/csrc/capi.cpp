// Error plumbing of the C-ABI (thread-local last-error message).
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include "../../include/retr_hip.h"

static thread_local char g_err[512] = "";

void retr_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int retr_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    retr_set_error("%s: %s", what, hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}

extern "C" const char* retr_last_error(void) { return g_err; }
extern "C" int retr_abi_version(void) { return 1; }
