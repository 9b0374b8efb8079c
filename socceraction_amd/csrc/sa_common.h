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
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
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
// The cast + clip without the int64 conversion (gfx950 has none: ~10 f64 instructions per cast,
// most of K1's VALU time): NaN and v >= 2^63 cast to INT64_MIN (cell 0), every other v clips to
// [0, l - 1] before the truncation -- trunc(min(max(v, 0), l - 1)) == clip(trunc(v), 0, l - 1),
// incl. v < -2^63 (INT64_MIN -> 0) -- so one v_cvt_i32_f64 of a value in [0, l - 1] remains.
__device__ __forceinline__ int cell_index(double v, int l) {
  const bool inr = v < 9.2233720368547758e18;  // false for NaN
  return inr ? (int)__builtin_fmin(__builtin_fmax(v, 0.0), (double)(l - 1)) : 0;
}

__device__ __forceinline__ int flat_index(double x, double y, int l, int w) {
  int xi = cell_index(x / FIELD_L * (double)l, l);
  int yj = cell_index(y / FIELD_W * (double)w, w);
  return (w - 1 - yj) * l + xi;
}

__device__ __forceinline__ bool is_move(int t) { return t == T_PASS || t == T_DRIBBLE || t == T_CROSS; }

// The binning's quotients x / 105 and y / 68 without a division: y = x * r, r = RN(1 / b), then
// Markstein's correction y + r * (x - y * b) by two fmas -- the correctly rounded quotient for
// every x whose quotient is a normal number (scripts/check_quotient.c; 1e9 random doubles over
// 2^-960..2^960 and [0, 128) against x / b, no mismatch).  Elsewhere it may differ from x / b
// only where the int64 cast cannot tell (|q| < 2^-1000: cell 0 either way; x = +-inf gives NaN
// instead of +-inf: both cast to INT64_MIN), so flat_index_q(bin_q...) == flat_index for every
// double input.
struct BinQ {
  double sx, sy, ex, ey;  // start / end coordinates over the field's extent
};
__device__ __forceinline__ double bin_quot(double x, double b, double rb) {
  const double y = x * rb;
  return __builtin_fma(__builtin_fma(-y, b, x), rb, y);
}
__device__ __forceinline__ BinQ bin_q(double sx, double sy, double ex, double ey) {
  constexpr double RL = 1.0 / FIELD_L, RW = 1.0 / FIELD_W;
  return BinQ{bin_quot(sx, FIELD_L, RL), bin_quot(sy, FIELD_W, RW), bin_quot(ex, FIELD_L, RL),
              bin_quot(ey, FIELD_W, RW)};
}
__device__ __forceinline__ int flat_index_q(double qx, double qy, int l, int w) {
  int xi = cell_index(qx * (double)l, l);
  int yj = cell_index(qy * (double)w, w);
  return (w - 1 - yj) * l + xi;
}

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


// Grids of C <= SA_XT_CELLS16_MAX_C cells (the small-grid count; 16 x 12) carry a 16-bit cell
// code (include/socceraction_amd.h): s * C + e for a successful move with finite coordinates,
// then the ranges below -- 2 B per action written by the feature pass and read by the count and
// the rate instead of 4 (the bench step: 2.951 -> 2.935 ms, profiles/r05ap).  SA_XT_CELLS16=0
// (A/B builds) keeps the u32 code for every grid.
#ifndef SA_XT_CELLS16
#define SA_XT_CELLS16 1
#endif
__host__ __device__ constexpr bool xt_c16(int C) { return SA_XT_CELLS16 && C <= SA_XT_CELLS16_MAX_C; }
constexpr uint32_t XT_C16_NONE = 0xFFFFu;
// ranges (C <= 202 < 256, so no division decodes them): successful move with finite
// coordinates s << 8 | e; shot with a finite start XT_C16_SHOT + 2 s + goal; a move with a finite
// start that is unsuccessful XT_C16_MISS + s, has a non-finite end XT_C16_EEND + s (unsuccessful)
// or XT_C16_EEND_S + s (successful); XT_C16_SPEC + {0 shot NaN start, 1 shot infinite start,
// 2 / 3 move NaN start unsuccessful / successful, 4 / 5 move infinite start unsuccessful /
// successful}; XT_C16_NONE any other action
constexpr uint32_t XT_C16_SHOT = 202u << 8, XT_C16_MISS = XT_C16_SHOT + 512u, XT_C16_EEND = XT_C16_MISS + 256u,
                   XT_C16_EEND_S = XT_C16_EEND + 256u, XT_C16_SPEC = XT_C16_EEND_S + 256u;
static_assert(XT_C16_SPEC + 6u < XT_C16_NONE, "16-bit cell code ranges");
__device__ __forceinline__ uint32_t xt_cell_code16(int t, int r, double sx, double sy, double ex, double ey,
                                                   int l, int w) {
  const bool shot = t == T_SHOT, mv = is_move(t), succ = r == R_SUCCESS;
  if (!shot && !mv) return XT_C16_NONE;
  const bool snan = isnan(sx) || isnan(sy), sfin = isfinite(sx) && isfinite(sy);
  const bool efin = isfinite(ex) && isfinite(ey);
  if (shot) {
    if (snan) return XT_C16_SPEC;
    if (!sfin) return XT_C16_SPEC + 1u;
    return XT_C16_SHOT + 2u * (uint32_t)flat_index(sx, sy, l, w) + (succ ? 1u : 0u);
  }
  if (snan) return XT_C16_SPEC + 2u + (succ ? 1u : 0u);
  if (!sfin) return XT_C16_SPEC + 4u + (succ ? 1u : 0u);
  const uint32_t cs = (uint32_t)flat_index(sx, sy, l, w);
  if (!efin) return (succ ? XT_C16_EEND_S : XT_C16_EEND) + cs;
  if (!succ) return XT_C16_MISS + cs;
  return (cs << 8) | (uint32_t)flat_index(ex, ey, l, w);
}

// ---- shared by the xT count passes (sa_xt.hip, sa_xt_large.hip) ----
// Rate operand of one action for a later rate() on the same (l, w) grid, written by the count
// pass so the rate pass reads 4 B instead of the 34 B of coordinates and ids again
// (xthreat.py:440-465 without interpolation): start cell | end cell << 16 for a successful
// move with finite coordinates, XT_CODE_BAD for a successful move with a non-finite one (the
// reference's int64 cast raises), XT_CODE_NAN for every other action (rated NaN).
constexpr uint32_t XT_CODE_NAN = 0xFFFFFFFFu, XT_CODE_BAD = 0xFFFFFFFEu;

__device__ __forceinline__ uint32_t rate_code(int t, int r, double sx, double sy, double ex, double ey,
                                              int l, int w) {
  if (!is_move(t) || r != R_SUCCESS) return XT_CODE_NAN;
  if (!isfinite(sx) || !isfinite(sy) || !isfinite(ex) || !isfinite(ey)) return XT_CODE_BAD;
  return (uint32_t)flat_index(sx, sy, l, w) | ((uint32_t)flat_index(ex, ey, l, w) << 16);
}

// The operand of a rate(use_interpolation=True) of the same action on the L x W node grid
// (xthreat.py:443-464: the start and end node of a successful move), u64 so that L * W up to 2^31
// fits: start node | end node << 32; markers as rate_code.
constexpr uint64_t XT_ICODE_NAN = ~0ull, XT_ICODE_BAD = ~0ull - 1;

__device__ __forceinline__ uint64_t rate_icode(int t, int r, double sx, double sy, double ex, double ey,
                                               int L, int W) {
  if (!is_move(t) || r != R_SUCCESS) return XT_ICODE_NAN;
  if (!isfinite(sx) || !isfinite(sy) || !isfinite(ex) || !isfinite(ey)) return XT_ICODE_BAD;
  return (uint64_t)(uint32_t)flat_index(sx, sy, L, W) | ((uint64_t)(uint32_t)flat_index(ex, ey, L, W) << 32);
}

// One action's part of the count pass: shot/goal/move histograms and the successful-move
// transition count, with the reference's non-finite rules (xthreat.py:40-67: _count drops rows
// with a NaN start, casts the rest; :177-218: move_transition_matrix casts every move
// coordinate).  Error flags, one byte each so that a sum all-reduce of the ranks' flags keeps
// them apart: 0x1 = infinite shot start, 0x100 = infinite move start, 0x10000 = NaN move start
// or non-finite move end (see sa_xt_count).
constexpr int32_t XT_ERRB_SHOT = 0x1, XT_ERRB_MOVE_START = 0x100, XT_ERRB_MOVE_OTHER = 0x10000;

struct XtAct {
  uint32_t cls;            // 0, XT_CELL_SHOT, XT_CELL_MOVE
  bool succ, snan, sfin, efin;
  int cs, ce;              // start / end cell (valid when binned)
};

// branch-free (selects only: the codes of a wave are of every kind)
__device__ __forceinline__ XtAct decode_cell16(uint32_t c, int C) {
  (void)C;
  const uint32_t dB = c - XT_C16_SHOT, dR = c - XT_C16_MISS, kS = c - XT_C16_SPEC;
  const bool A = c < XT_C16_SHOT, Bq = c >= XT_C16_SHOT && c < XT_C16_MISS;
  const bool R = c >= XT_C16_MISS && c < XT_C16_SPEC, S = c >= XT_C16_SPEC && c != XT_C16_NONE;
  const uint32_t kR = dR >> 8;
  XtAct a;
  a.cls = (A || R || (S && kS >= 2u)) ? XT_CELL_MOVE : ((Bq || (S && kS < 2u)) ? XT_CELL_SHOT : 0u);
  a.succ = A || (Bq && (dB & 1u)) || (R && kR == 2u) || (S && kS >= 2u && (kS & 1u));
  a.snan = S && (kS == 0u || kS == 2u || kS == 3u);
  a.sfin = !S;
  a.efin = !(R && kR != 0u);
  a.cs = A ? (int)(c >> 8) : (Bq ? (int)(dB >> 1) : (R ? (int)(dR & 0xFFu) : 0));
  a.ce = A ? (int)(c & 0xFFu) : 0;
  return a;
}

__device__ __forceinline__ XtAct decode_cell(uint32_t c) {
  XtAct a;
  a.cls = (c >> 24) & 3u;
  a.succ = (c >> 26) & 1u;
  a.snan = (c >> 27) & 1u;
  a.sfin = !((c >> 28) & 1u);
  a.efin = !((c >> 29) & 1u);
  a.cs = (int)(c & 0xFFFu);
  a.ce = (int)((c >> 12) & 0xFFFu);
  return a;
}


// rate_code / rate_icode from the binning quotients (bin_q of the same coordinates).
__device__ __forceinline__ uint32_t rate_code_q(int t, int r, double sx, double sy, double ex, double ey,
                                                const BinQ& q, int l, int w) {
  if (!is_move(t) || r != R_SUCCESS) return XT_CODE_NAN;
  if (!isfinite(sx) || !isfinite(sy) || !isfinite(ex) || !isfinite(ey)) return XT_CODE_BAD;
  return (uint32_t)flat_index_q(q.sx, q.sy, l, w) | ((uint32_t)flat_index_q(q.ex, q.ey, l, w) << 16);
}
__device__ __forceinline__ uint64_t rate_icode_q(int t, int r, double sx, double sy, double ex, double ey,
                                                 const BinQ& q, int L, int W) {
  if (!is_move(t) || r != R_SUCCESS) return XT_ICODE_NAN;
  if (!isfinite(sx) || !isfinite(sy) || !isfinite(ex) || !isfinite(ey)) return XT_ICODE_BAD;
  return (uint64_t)(uint32_t)flat_index_q(q.sx, q.sy, L, W) | ((uint64_t)(uint32_t)flat_index_q(q.ex, q.ey, L, W) << 32);
}

// The XtAct of one action from its row (the coordinate form of decode_cell; t < 0: not counted).
__device__ __forceinline__ XtAct act_from_row(int t, int r, double sx, double sy, double ex, double ey, int l,
                                              int w) {
  XtAct a;
  a.cls = t == T_SHOT ? XT_CELL_SHOT : (is_move(t) ? XT_CELL_MOVE : 0u);
  a.succ = r == R_SUCCESS;
  a.snan = isnan(sx) || isnan(sy);
  a.sfin = isfinite(sx) && isfinite(sy);
  a.efin = isfinite(ex) && isfinite(ey);
  a.cs = (a.cls && a.sfin) ? flat_index(sx, sy, l, w) : 0;
  a.ce = (a.cls == XT_CELL_MOVE && a.succ && a.efin) ? flat_index(ex, ey, l, w) : 0;
  return a;
}

// act_from_row from the binning quotients (bin_q of the same coordinates).
__device__ __forceinline__ XtAct act_from_row_q(int t, int r, double sx, double sy, double ex, double ey,
                                                const BinQ& q, int l, int w) {
  XtAct a;
  a.cls = t == T_SHOT ? XT_CELL_SHOT : (is_move(t) ? XT_CELL_MOVE : 0u);
  a.succ = r == R_SUCCESS;
  a.snan = isnan(sx) || isnan(sy);
  a.sfin = isfinite(sx) && isfinite(sy);
  a.efin = isfinite(ex) && isfinite(ey);
  a.cs = (a.cls && a.sfin) ? flat_index_q(q.sx, q.sy, l, w) : 0;
  a.ce = (a.cls == XT_CELL_MOVE && a.succ && a.efin) ? flat_index_q(q.ex, q.ey, l, w) : 0;
  return a;
}

}  // namespace sa
