// Host-side helpers shared by the C-ABI entry points (error reporting, launch checks).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/socceraction_amd.h"

namespace sa {
// Records a printf-style message in the thread-local error slot and returns `code`.
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
// Maps a pending launch error (hipGetLastError) to SA_EHIP.
int check_launch(const char* what);
int check_hip(hipError_t e, const char* what);
inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }
}  // namespace sa
