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
// Compute units and LDS bytes per workgroup of device `dev`, queried once per device (256 /
// 64 KiB when the query fails).
int device_cus(int dev);
int device_lds_max(int dev);
// The current device (0 when the query fails).
int current_device();

// Library-owned device scratch (the cached per-device arena of sa_api.hip).  acquire returns a
// slot of at least `bytes` that no other call is using; release hands it back once the work
// enqueued on `st` is done with it (stream-ordered reuse).
struct Scratch {
  void* ptr = nullptr;
  int slot = -1;
};
int scratch_acquire(size_t bytes, hipStream_t st, Scratch* out);
void scratch_release(const Scratch& s, hipStream_t st);

// Large-grid xT (sa_xt_large.hip).  xt_band_ok: the band-owned count holds a grid of C cells;
// xt_count_bands: that count of one batch, added into the caller's counts.  xt_compact_*: the
// compact form of count rows and one value iteration over it (C <= 9472).
bool xt_band_ok(int C);
int xt_count_bands(const sa_actions& A, const uint32_t* cells, int64_t n, int l, int w, int64_t* shot,
                   int64_t* goal, int64_t* move, int32_t* trans, int32_t* err, uint32_t* codes, hipStream_t st);
bool xt_compact_ok(int C);
size_t xt_compact_bytes(int C, int nrows);
int xt_compact_build(const int32_t* cnt_rows, int C, int nrows, uint32_t* ell, int32_t* row_len, hipStream_t st);
int xt_compact_iterate(const uint32_t* ell, const int32_t* row_len, const int32_t* cnt_rows, const int64_t* move,
                       const double* gs, const double* pmove, int C, int rb, int nrows, const double* x, double eps,
                       double* xo, const int32_t* flag_prev, int32_t* flag_out, hipStream_t st);
// The whole value iteration over the compact form of every row (sa_xt_solve_compact):
// reordered sums under an error bound, or the reference's order (SA_XT_SOLVE_EXACT, or when the
// bound cannot decide); *path = SA_XT_PATH_*.  xt_out (optional): the reordered path also
// writes the final iterate there (the surface).  Synchronises the stream.
// hook (optional): work enqueued right after the one-launch reordered solve, before the host
// waits for its status (sa_xt_fit_rate_interp_codes: the rate of the surface the solve writes);
// hook->ran says whether it was.
struct SolveHook {
  int (*fn)(void* ctx);
  void* ctx;
  bool ran;
};
int xt_compact_solve(const uint32_t* ell, const int32_t* row_len, const int32_t* cnt_rows, const int64_t* move,
                     const double* gs, const double* pmove, int C, double eps, int max_iter, int flags,
                     double* heat, int* n_iter, int* path, hipStream_t st, double* xt_out = nullptr,
                     SolveHook* hook = nullptr);
}  // namespace sa
