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

// device-resident step seed used by every dropout mask (see common.hpp make_dp)
static const unsigned long long* g_seed_base = nullptr;
const unsigned long long* retr_seed_base() { return g_seed_base; }
extern "C" void retr_set_seed_base(const unsigned long long* p) { g_seed_base = p; }

static int g_deterministic = 0;
int retr_deterministic() { return g_deterministic; }
extern "C" void retr_set_deterministic(int on) { g_deterministic = on ? 1 : 0; }
extern "C" int retr_get_deterministic(void) { return g_deterministic; }

static int g_tune[RETR_TUNE_COUNT] = {0};
int retr_tune_get(int knob) { return knob >= 0 && knob < RETR_TUNE_COUNT ? g_tune[knob] : 0; }
extern "C" int retr_tune(int knob, int value) {
  if (knob < 0 || knob >= RETR_TUNE_COUNT) return -1;
  const int old = g_tune[knob];
  g_tune[knob] = value;
  return old;
}

__global__ void seed_bump_kernel(unsigned long long* p, unsigned long long d) { *p += d; }
extern "C" int retr_seed_bump(unsigned long long* p, unsigned long long delta, void* stream) {
  hipLaunchKernelGGL(seed_bump_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, p, delta);
  return retr_check_launch("seed_bump");
}

// Measurement helper (bench.py probe): one wave that busy-waits `us` microseconds on the device
// clock (s_memrealtime, 100 MHz).  Launched just before a probe's start event so the host has
// already queued the timed kernel when the event executes: the event pair then brackets only
// device execution, not host launch latency.
__global__ void spin_kernel(unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}
extern "C" int retr_spin_us(float us, void* stream) {
  unsigned long long ticks = us > 0.f ? (unsigned long long)(us * 100.f) : 0ull;
  if (ticks > 100000000ull) ticks = 100000000ull;   // <= 1 s
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, ticks);
  return retr_check_launch("spin");
}
