// Device bounds checks of the debug build (SURVEY.md §5 "HIP debug build plus bounds asserts in
// kernels under a flag").  Built with -DSA_DEBUG=1 (`python -m socceraction_amd.build --debug`,
// libsocceraction_amd_debug.so); the default build compiles every check away.
//
// A failing check does not trap (a device trap aborts the queue): it records the first failure
// -- source file, line and the offending value -- in a per-translation-unit device word and lets
// the kernel carry on with the access clamped or skipped where the caller says so.
// sa_debug_check() (C ABI) synchronises the device, collects the record of every translation
// unit, clears it and returns SA_EDATA with the location in sa_last_error().
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdio>

#ifndef SA_DEBUG
#define SA_DEBUG 0
#endif

namespace sa {

// host: one poll function per translation unit (registered at load time)
typedef int (*debug_poll_fn)(char* msg, int cap);
bool register_debug_poll(debug_poll_fn fn);

#if SA_DEBUG
// [0] = failing line (0: none), [1] = low word of the value, [2] = high word
static __device__ int32_t g_dbg_rec[3];

__device__ __noinline__ __attribute__((unused)) static void debug_report(int line, long long v) {
  if (atomicCAS(&g_dbg_rec[0], 0, line) == 0) {
    atomicExch(&g_dbg_rec[1], (int32_t)(v & 0xFFFFFFFFll));
    atomicExch(&g_dbg_rec[2], (int32_t)(v >> 32));
  }
}

static int debug_poll_this_tu(char* msg, int cap) {
  int32_t rec[3] = {0, 0, 0};
  if (hipMemcpyFromSymbol(rec, HIP_SYMBOL(g_dbg_rec), sizeof(rec), 0, hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  if (rec[0] == 0) return 0;
  const int32_t zero[3] = {0, 0, 0};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_rec), zero, sizeof(zero), 0, hipMemcpyHostToDevice);
  const long long v = (long long)(((uint64_t)(uint32_t)rec[2] << 32) | (uint32_t)rec[1]);
  snprintf(msg, cap, "device bounds check failed: %s:%d (value %lld)", __BASE_FILE__, rec[0], v);
  return 1;
}

static const bool g_dbg_registered = register_debug_poll(&debug_poll_this_tu);

// SA_DCHECK(cond, value): record a failure of `cond`; the statement that follows must not rely
// on it (callers clamp or skip the access themselves).
#define SA_DCHECK(cond, val)                                   \
  do {                                                         \
    if (!(cond)) ::sa::debug_report(__LINE__, (long long)(val)); \
  } while (0)
// SA_DGUARD(cond, val, action): as SA_DCHECK, then `action` (e.g. return / break) on failure.
#define SA_DGUARD(cond, val, action)                             \
  if (!(cond)) {                                                 \
    ::sa::debug_report(__LINE__, (long long)(val));              \
    action;                                                      \
  }
#else
#define SA_DCHECK(cond, val) ((void)0)
#define SA_DGUARD(cond, val, action) ((void)0)
#endif

}  // namespace sa
