// Host-side helpers shared by the C-ABI entry points (error reporting, launch checks, scratch).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/socceraction_amd.h"
#include "sa_debug.h"

namespace sa {
// Records a printf-style message in the thread-local error slot and returns `code`.
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
// Maps a pending launch error (hipGetLastError) to SA_EHIP.
int check_launch(const char* what);
int check_hip(hipError_t e, const char* what);
inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// Library-owned device scratch (the cached per-device arena of sa_api.hip).  acquire returns a
// slot of at least `bytes` that no other call is using; release hands it back once the work
// enqueued on `st` is done with it (stream-ordered reuse).
struct Scratch {
  void* ptr = nullptr;
  int slot = -1;
};
int scratch_acquire(size_t bytes, hipStream_t st, Scratch* out);
void scratch_release(const Scratch& s, hipStream_t st);
}  // namespace sa
