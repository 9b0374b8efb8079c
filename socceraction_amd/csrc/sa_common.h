// Shared device helpers and vocabulary constants for the gfx950 kernels.
//
// Vocabulary ids follow reference spadl/config.py:24-57 and
// atomic/spadl/config.py:25-36 (ids are list positions).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>

#include "../../include/socceraction_amd.h"
#include "sa_debug.h"

namespace sa {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef long long i64x2 __attribute__((ext_vector_type(2)));

// SPADL action types / results used by the path
constexpr int T_PASS = 0, T_CROSS = 1, T_CORNER_CROSSED = 5, T_CORNER_SHORT = 6, T_SHOT = 11,
              T_SHOT_PENALTY = 12, T_SHOT_FREEKICK = 13, T_DRIBBLE = 21;
constexpr int R_SUCCESS = 1, R_OWNGOAL = 3;
// Atomic-SPADL
constexpr int AT_INTERCEPTION2 = 24, AT_GOAL = 27, AT_OWNGOAL = 28;
constexpr int N_TYPES = 23, N_RESULTS = 6, N_BODYPARTS = 4, N_ATOMIC_NAMES = 32;

constexpr double FIELD_L = 105.0;
constexpr double FIELD_W = 68.0;
constexpr double GOAL_Y = 34.0;  // field_width / 2 (vaep/features.py:351-352)

// -------------------------------------------------------------------------------------
// SWAR byte compare: returns 0x01 in every byte of `w` equal to `v` (exact, no false hits)
__device__ __forceinline__ uint32_t bytes_eq(uint32_t w, uint32_t v) {
  uint32_t x = w ^ (v * 0x01010101u);
  uint32_t t = ((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x;  // high bit set <=> byte != 0
  return (~t >> 7) & 0x01010101u;
}

__device__ __forceinline__ uint32_t byte_of(uint32_t w, int b) { return (w >> (8 * b)) & 0xFFu; }

// Funnel shift: bytes [s, s+4) of the 8-byte little-endian pair (lo, hi), s in 0..3.
__device__ __forceinline__ uint32_t funnel_bytes(uint32_t lo, uint32_t hi, int s) {
  return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)s);
}

// Segment lookup: largest g with seg_off[g] <= j (seg_off sorted, seg_off[0] = 0).
__device__ __forceinline__ int64_t find_segment(const int64_t* __restrict__ seg_off, int64_t nseg,
                                                int64_t j) {
  int64_t lo = 0, hi = nseg;  // invariant: seg_off[lo] <= j < seg_off[hi]
  while (hi - lo > 1) {
    int64_t mid = (lo + hi) >> 1;
    if (seg_off[mid] <= j)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

// Guarded scalar loads (rows outside [0, n) read as 0).
template <typename T>
__device__ __forceinline__ T ld_or0(const T* __restrict__ p, int64_t i, int64_t n) {
  return (i >= 0 && i < n) ? p[i] : T(0);
}

// Load 4 bytes [4*wi, 4*wi+4) of a length-n u8 array into one word (zero padded).
__device__ __forceinline__ uint32_t ld_u8x4(const uint8_t* __restrict__ p, int64_t wi, int64_t n) {
  int64_t b = wi * 4;
  if (b >= 0 && b + 4 <= n) return *reinterpret_cast<const uint32_t*>(p + b);
  uint32_t w = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) w |= (uint32_t)ld_or0(p, b + q, n) << (8 * q);
  return w;
}

// -------------------------------------------------------------------------------------
// xT binning (reference xthreat.py:25-37): numpy float64 -> int64 cast (x86 cvttsd2si: NaN /
// out of range -> INT64_MIN), then clip; (x / 105) * l in f64, divide THEN multiply.
__device__ __forceinline__ int cell_index(double v, int l) {
  long long c = (v >= -9.2233720368547758e18 && v < 9.2233720368547758e18) ? (long long)v
                                                                             : (long long)INT64_MIN;
  return c < 0 ? 0 : (c > l - 1 ? l - 1 : (int)c);
}

__device__ __forceinline__ int flat_index(double x, double y, int l, int w) {
  int xi = cell_index(x / FIELD_L * (double)l, l);
  int yj = cell_index(y / FIELD_W * (double)w, w);
  return (w - 1 - yj) * l + xi;
}

__device__ __forceinline__ bool is_move(int t) { return t == T_PASS || t == T_DRIBBLE || t == T_CROSS; }

// xT cell code of one SPADL action for a fit + rate of the same actions on an (l, w) grid with
// l * w <= SA_XT_CELLS_MAX_C (include/socceraction_amd.h): written once per action where the
// coordinates are already in registers (the VAEP feature pass, or sa_xt_cells), read by the
// count and rate passes instead of the 34 B of coordinates and ids.
//   bits 0-11 start cell, 12-23 end cell (0 when not binned), 24-25 class (1 shot = type 11,
//   2 move = pass / dribble / cross), 26 result == success, 27 start has a NaN, 28 start not
//   finite, 29 end not finite.
constexpr uint32_t XT_CELL_SHOT = 1u, XT_CELL_MOVE = 2u;

__device__ __forceinline__ uint32_t xt_cell_code(int t, int r, double sx, double sy, double ex,
                                                 double ey, int l, int w) {
  const uint32_t cls = t == T_SHOT ? XT_CELL_SHOT : (is_move(t) ? XT_CELL_MOVE : 0u);
  const bool snan = isnan(sx) || isnan(sy);
  const bool sfin = isfinite(sx) && isfinite(sy);
  const bool efin = isfinite(ex) && isfinite(ey);
  uint32_t c = (cls << 24) | ((uint32_t)(r == R_SUCCESS) << 26) | ((uint32_t)snan << 27) |
               ((uint32_t)!sfin << 28) | ((uint32_t)!efin << 29);
  if (cls != 0 && sfin) c |= (uint32_t)flat_index(sx, sy, l, w);
  if (cls == XT_CELL_MOVE && efin) c |= (uint32_t)flat_index(ex, ey, l, w) << 12;
  return c;
}

}  // namespace sa
