// VAEP / Atomic-VAEP hot-path kernels for gfx950 (MI355X).
//
//   bool_colgroup_kernel     one-hot + team features (gamestates + flip fused in), bool block
//   num_features_kernel      time / location / polar / movement / deltas / ids, f64 + i64 blocks
//   goalscore_wave16_kernel  segmented exclusive scan (one wave per segment)
//   labels_kernel            scores / concedes / goal_from_shot look-ahead
//   formula_kernel           offensive / defensive / vaep value (f64 or f32)
//
// All of it is HBM-bound byte/int/f64 streaming; nothing here is GEMM-shaped.  The output
// is ~94 % of the traffic, so the kernels are built around full-width stores:
//  * bool columns: a lane owns 16 consecutive actions and writes one 16-B word per column,
//    so one store instruction writes 1 KiB of one column;
//  * f64 / i64 columns: a lane owns 2 consecutive actions (one 16-B store), so one store
//    instruction writes 1 KiB of one column.
// Long runs per column per wave matter (see bool_colgroup_kernel).  Game-state windows
// never leave registers: window i of action j is row j - min(i, j - segment_start)
// (vaep/features.py:83-88), built with funnel shifts from the lane's rows j0-8 .. j0+15.
//
// Compile-time knobs (the default build is the measured configuration; variants are built
// with `python -m socceraction_amd.build -DNAME=V --variant=tag`): SA_NT_STORES (non-temporal
// stores), SA_XCD_REMAP (XCD-contiguous block order), SA_CG_COLS (bool columns per wave),
// SA_DEBUG (device bounds checks, sa_debug.h).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "sa_common.h"
#include "sa_internal.h"

#ifndef SA_NT_STORES
#define SA_NT_STORES 1
#endif
#ifndef SA_XCD_REMAP
#define SA_XCD_REMAP 1  // block -> output range mapping that gives each XCD a contiguous part
#endif

namespace sa {

constexpr int WAVE = 64;
constexpr int LANE_ACTS = 16;
#ifndef SA_CG_COLS
#define SA_CG_COLS 32  // bool_colgroup_kernel: target columns per wave
#endif
#ifndef SA_NUM_BLOCK_WAVES
#define SA_NUM_BLOCK_WAVES 4  // numeric-pass workgroup in waves (A/B knob; 3 waves per SIMD fit 12 per CU)
#endif
constexpr int BLOCK_WAVES = SA_NUM_BLOCK_WAVES;
constexpr int NUM_PAIRS = 1;                    // 2-action pairs per lane in num_features_kernel
constexpr int WAVE_ACTS = 128 * NUM_PAIRS;      // actions per wave in num_features_kernel
constexpr int BLOCK_ACTS = WAVE_ACTS * BLOCK_WAVES;

struct FeatArgs {
  sa_actions a;
  sa_feature_plan p;
  uint8_t* bout;
  double* fout;
  int64_t* iout;
  int64_t Cb, Cf, Ci;  // columns of each block
  int64_t Rb, Rf, Ri;  // rows per tile of each block (include/socceraction_amd.h)
  uint32_t* xt_cells;  // optional: xT cell code of every action (sa_vaep_features_xt)
  int32_t xt_l, xt_w;
  uint16_t* bbits;     // optional: bool features as bitmaps instead of bout (sa_vaep_features_bits)
  int64_t bstride;     // u16 per bitmap
  // optional tail (sa_vaep_step_f64): labels + f64 formula of the same rows, computed by the
  // numeric pass (num_features_kernel<..., TAIL>)
  int32_t nr;
  uint8_t *sc, *co, *gfs;
  const double *ps, *pc;
  double *off, *def, *val;
  bool vec_ok;
  // optional (sa_vaep_features_conditions): the numeric columns become split-condition bitmaps
  const int32_t *cond_fstart, *cond_istart;  // [Cf + 1], [Ci + 1]: conditions of each column
  const float* cond_thr;                     // per condition: float32 threshold (`x < thr` goes left)
  const int32_t* cond_dl;                    // per condition: NaN goes left
  int32_t cond_row0;                         // bitmap row of condition 0 (after the bool columns)
  int32_t cond_n;                             // conditions (num_cond_lds_kernel stages the tables)
  // the numeric pass over rows [row0, row_end) only (row_end 0: to n); row0 a multiple of
  // BLOCK_ACTS (sa_vaep_step_f64_chunked: one launch per chunk of the batch)
  int64_t row0, row_end;
};
typedef float f32x2 __attribute__((ext_vector_type(2)));

// COND mode of the numeric pass: a store of column `col` (rows jb, jb+1 of the lane) evaluates
// that column's split conditions of a learner instead -- bit = goes right, xgboost's float32
// compare (`x < thr` left, NaN -> default) -- and the wave's 128 bits of each condition go to
// bitmap row cond_row0 + c (Arrow layout).  Both learners of VAEP.rate read these bitmaps like
// bool features, so the numeric values never reach HBM.
// The wave's outcome of condition c is two ballots (rows wb + 2l and wb + 2l + 1 of lane l); lane
// c % 64 of the wave keeps them until the wave moves to another chunk of 64 conditions, then
// every holding lane interleaves its pair into the 128-bit run of its bitmap row and stores it
// in one 16-B store: one store instruction per chunk instead of one per condition.
struct CondAcc {
  uint64_t even, odd;  // this lane's condition (chunk + lane): ballots over even / odd rows
  uint64_t held;       // uniform: lanes holding a condition of the chunk
  int32_t chunk;       // uniform: first condition of the chunk
  float tv;            // threshold of condition chunk + lane (loaded when the chunk changes)
  uint64_t dlm;        // uniform: the chunk's conditions whose NaN goes left
};

// the sinks take the wave's first row (wb) and the ok / NaN masks from wave_base: one 128-row
// pair per lane.  More pairs per lane would need a flush and a new wb per pair.
static_assert(NUM_PAIRS == 1, "COND sinks assume one 2-row pair per lane (CondSink::wb)");

struct CondSink {
  const int32_t* start;
  const float* thr;
  const int32_t* dl;
  uint16_t* bits;
  int64_t stride16;  // u16 per bitmap row
  int32_t row0;
  int64_t wb, n;
  CondAcc* acc;
  int32_t n_start;   // entries of start (columns + 1)
  int32_t n_cond;
  int32_t sv;        // start[lane] (lanes < n_start): a column's starts by v_readlane, no load
  uint64_t ok0, ok1; // uniform: the wave's rows present (even / odd)
};

__device__ __forceinline__ CondSink cond_sink(const int32_t* start, int32_t n_start, const FeatArgs& args,
                                              int64_t wb, int64_t n, CondAcc* acc) {
  const int lane = threadIdx.x & 63;
  const int64_t jb = wb + 2 * lane;
  CondSink k{start, args.cond_thr, args.cond_dl, args.bbits, args.bstride, args.cond_row0, wb, n, acc,
             n_start, args.cond_n, lane < n_start ? start[lane] : 0, __ballot(jb < n), __ballot(jb + 1 < n)};
  return k;
}

__device__ __forceinline__ uint64_t spread32(uint32_t v) {  // bit i -> bit 2i
  uint64_t x = v;
  x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
  x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
  x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
  x = (x | (x << 2)) & 0x3333333333333333ull;
  x = (x | (x << 1)) & 0x5555555555555555ull;
  return x;
}

__device__ __forceinline__ void cond_flush(const CondSink* s) {
  CondAcc* a = s->acc;
  const int lane = threadIdx.x & 63;
  if ((a->held >> lane) & 1) {
    const uint64_t lo = spread32((uint32_t)a->even) | (spread32((uint32_t)a->odd) << 1);
    const uint64_t hi = spread32((uint32_t)(a->even >> 32)) | (spread32((uint32_t)(a->odd >> 32)) << 1);
    uint4* dst = reinterpret_cast<uint4*>(s->bits + (int64_t)(s->row0 + a->chunk + lane) * s->stride16 + s->wb / 16);
    *dst = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
  }
  a->held = 0;
}

// old with lane k's value replaced by the uniform v: v_writelane_b32 on both halves, the lane
// select in M0 (gfx9's constant bus takes one SGPR besides M0); one instruction per dword instead
// of a lane compare, two moves and two selects
__device__ __forceinline__ uint64_t writelane64(uint64_t old, uint64_t v, int k) {
  uint32_t lo = (uint32_t)old, hi = (uint32_t)(old >> 32);
  const uint32_t vlo = __builtin_amdgcn_readfirstlane((uint32_t)v), vhi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  asm volatile("v_writelane_b32 %0, %1, m0" : "+v"(lo) : "s"(vlo), "{m0}"(k));
  asm volatile("v_writelane_b32 %0, %1, m0" : "+v"(hi) : "s"(vhi), "{m0}"(k));
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ void cond_store(const CondSink* s, int64_t col, float x0, float x1) {
  CondAcc* a = s->acc;
  const int lane = threadIdx.x & 63;
  // per column: the NaN rows as wave masks (the rows present: per wave, in the sink); per
  // condition two compares, the rest is scalar (`!(x < thr)` is true for NaN: right unless NaN
  // goes left)
  const uint64_t ok0 = s->ok0, ok1 = s->ok1;
  const uint64_t nan0 = __ballot(isnan(x0)), nan1 = __ballot(isnan(x1));
  // the column's first / end condition from the lane-resident starts (n_start <= 64: checked by
  // sa_vaep_features_conditions; k <= 3 plans have at most 47 f64 / 15 i64 columns)
  SA_DCHECK(col + 1 < s->n_start, col);
  const int c0 = __builtin_amdgcn_readlane(s->sv, (int)col);
  const int c1 = __builtin_amdgcn_readlane(s->sv, (int)col + 1);
  // the column's conditions in segments inside one 64-condition chunk; a chunk's thresholds and
  // NaN directions are loaded (one per lane) when the wave enters it and read back by
  // v_readlane, so a segment costs no load and no wait (the COND pass with a threshold load and
  // chunk test per condition cost 0.9 ms over the plain numeric pass, with a load per segment
  // 0.8, r06t / r06i)
  for (int cb = c0; cb < c1;) {  // wave-uniform
    const int chunk = cb & ~63;
    if (chunk != a->chunk) {
      if (a->held) cond_flush(s);
      a->chunk = chunk;
      const int cl = chunk + lane;
      a->tv = cl < s->n_cond ? s->thr[cl] : 0.0f;
      a->dlm = __ballot(cl < s->n_cond && s->dl[cl] != 0);  // NaN goes left, per condition
    }
    const int ce = c1 < chunk + 64 ? c1 : chunk + 64;
    for (int c = cb; c < ce; ++c) {
      const int q = c & 63;
      const float thr = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(a->tv), q));
      uint64_t m0 = __ballot(!(x0 < thr)) & ok0, m1 = __ballot(!(x1 < thr)) & ok1;
      if ((a->dlm >> q) & 1ull) {
        m0 &= ~nan0;
        m1 &= ~nan1;
      }
      const int k = c & 63;  // the holding lane takes the two masks
      a->even = writelane64(a->even, m0, k);
      a->odd = writelane64(a->odd, m1, k);
    }
    const int k0 = cb & 63, nk = ce - cb;  // lanes k0 .. k0 + nk - 1 now hold conditions
    a->held |= (nk == 64 ? ~0ull : ((1ull << nk) - 1ull)) << k0;
    cb = ce;
  }
}

// Workgroups are dispatched round-robin over the 8 XCDs (XCD = blockIdx % 8).  Writing the
// output front to back in blockIdx order leaves every XCD's concurrent stores scattered over
// the whole active window; remapped, XCD x owns the contiguous logical blocks
// [x*per, (x+1)*per) and sweeps them in order, which keeps each XCD's open DRAM rows
// together (scripts/probe_store_colgroup.hip: 6.1 -> 6.9 TB/s for the bool image).  The grid
// must be a multiple of 8 blocks; logical blocks past the real count exit.
__device__ __forceinline__ int64_t xcd_logical_block() {
#if SA_XCD_REMAP
  const int64_t b = blockIdx.x, per = gridDim.x / 8;
  return (b % 8) * per + b / 8;
#else
  return blockIdx.x;
#endif
}

static inline unsigned xcd_grid(int64_t blocks) {
  return (unsigned)((blocks + 7) / 8 * 8);
}

// Element offset of (row j, column c) in a tiled column-major block with C columns.  A
// lane's 16 (or 2) rows never straddle a tile because R % 16 == 0.
__device__ __forceinline__ int64_t tile_off(int64_t j, int64_t c, int64_t C, int64_t R) {
  SA_DCHECK(j >= 0 && c >= 0 && c < C && R > 0 && R % 16 == 0, j);
  const int64_t t = j / R;
  return t * C * R + c * R + (j - t * R);
}

// ------------------------------------------------------------------------------ helpers
struct SegCursor {
  int64_t g, s, e;  // segment index, start, end (exclusive)
};

__device__ __forceinline__ SegCursor seg_at(const sa_actions& A, int64_t j) {
  SegCursor c;
  if (A.seg_of_block) {  // the segment of the row's block start, then forward to the row
    c.g = A.seg_of_block[j / SA_SEG_BLOCK];
    SA_DCHECK(c.g >= 0 && c.g < A.n_segments, c.g);
    c.s = A.seg_off[c.g];
    c.e = A.seg_off[c.g + 1];
    while (j >= c.e) {
      ++c.g;
      SA_DGUARD(c.g < A.n_segments, j, --c.g; break);
      c.s = c.e;
      c.e = A.seg_off[c.g + 1];
    }
    return c;
  }
  c.g = find_segment(A.seg_off, A.n_segments, j);
  c.s = A.seg_off[c.g];
  c.e = A.seg_off[c.g + 1];
  SA_DCHECK(c.g >= 0 && c.g < A.n_segments && c.s <= j && j < c.e, j);
  return c;
}

__device__ __forceinline__ void seg_advance(const sa_actions& A, SegCursor& c, int64_t j) {
  while (j >= c.e) {
    ++c.g;
    SA_DGUARD(c.g < A.n_segments, j, --c.g; break);
    c.s = c.e;
    c.e = A.seg_off[c.g + 1];
  }
}

// Wave-uniform segment cursor of row jw: one search per wave (scalar loads); lanes then advance
// from it to their own rows -- a per-lane binary search was ~14 dependent divergent loads.
__device__ __forceinline__ SegCursor wave_cursor(const sa_actions& A, int64_t jw) {
  const int lo = __builtin_amdgcn_readfirstlane((int)(jw & 0xFFFFFFFF));
  const int hi = __builtin_amdgcn_readfirstlane((int)(jw >> 32));
  return seg_at(A, ((int64_t)hi << 32) | (uint32_t)lo);
}

// Game-state windows of a lane's 16 actions, kept as 16 bytes (4 words) per id column.
// R[0..5] holds rows j0-8 .. j0+15 (byte 8 = row j0).  Window i+1 is the window-i rows
// shifted by one row, except for actions whose row already reached the segment start
// (d = j - seg_start < i+1): they keep their window-i byte (vaep/features.py:83-88 clamps
// the shifted frames at the first row).  Everything stays in registers (static indices).
__device__ __forceinline__ void shift_rows(uint32_t (&R)[6]) {
#pragma unroll
  for (int k = 5; k > 0; --k) R[k] = funnel_bytes(R[k - 1], R[k], 3);  // (R[k] << 8) | R[k-1] >> 24
  R[0] <<= 8;
}

// 0xFF in every byte whose d (0..15) is >= i (1..15); all-ones when i == 0
__device__ __forceinline__ uint32_t ge_mask(uint32_t dw, int i) {
  const uint32_t x = (dw + (uint32_t)(16 - i) * 0x01010101u) & 0x10101010u;
  return (x >> 4) * 0xFFu;
}

template <typename V, typename P>
__device__ __forceinline__ void st16(P* p, V v) {
#if SA_NT_STORES
  __builtin_nontemporal_store(v, reinterpret_cast<V*>(p));
#else
  *reinterpret_cast<V*>(p) = v;
#endif
}

// 0x01-per-byte mask -> 4 bits
__device__ __forceinline__ uint32_t pack4(uint32_t x) {
  return (x & 1u) | ((x >> 7) & 2u) | ((x >> 14) & 4u) | ((x >> 21) & 8u);
}

// 4 x 4 byte transpose: word q byte k of the result = word k byte q of the input.  The bitmap
// mode of the bool pass keeps a lane's 16 rows in this STRIDED order (word q byte k = row
// 4k + q), so that the four compare words of a column combine into one word whose byte k holds
// rows 4k .. 4k+3 as a nibble in row order (bits_of_strided).
__device__ __forceinline__ void transpose_bytes4(uint32_t (&w)[4]) {
  const uint32_t t0 = __builtin_amdgcn_perm(w[1], w[0], 0x05010400u);  // a0 b0 a1 b1
  const uint32_t t1 = __builtin_amdgcn_perm(w[1], w[0], 0x07030602u);  // a2 b2 a3 b3
  const uint32_t t2 = __builtin_amdgcn_perm(w[3], w[2], 0x05010400u);  // c0 d0 c1 d1
  const uint32_t t3 = __builtin_amdgcn_perm(w[3], w[2], 0x07030602u);  // c2 d2 c3 d3
  w[0] = __builtin_amdgcn_perm(t2, t0, 0x05040100u);                   // a0 b0 c0 d0
  w[1] = __builtin_amdgcn_perm(t2, t0, 0x07060302u);                   // a1 b1 c1 d1
  w[2] = __builtin_amdgcn_perm(t3, t1, 0x05040100u);                   // a2 b2 c2 d2
  w[3] = __builtin_amdgcn_perm(t3, t1, 0x07060302u);                   // a3 b3 c3 d3
}

// 16 row bits (bit r = row r) of four 0x01-per-byte compare words in the strided order
__device__ __forceinline__ uint32_t bits_of_strided(uint32_t e0, uint32_t e1, uint32_t e2, uint32_t e3) {
  const uint32_t x = e0 | (e1 << 1) | (e2 << 2) | (e3 << 3);  // byte k: rows 4k .. 4k+3
  const uint32_t y = x | (x >> 4);                             // bytes 0, 2: rows 0-7, 8-15
  return (y & 0xFFu) | ((y >> 8) & 0xFF00u);
}

// Stores into tiled blocks: `base` already points at the lane's (tile, row) position of
// column 0, so column c is c * R elements further.
__device__ __forceinline__ void st_bool16(uint8_t* __restrict__ base, int64_t col, int64_t C, int64_t R,
                                          uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
  u32x4 v = {w0, w1, w2, w3};
  SA_DGUARD(col >= 0 && col < C, col, return);
  st16(base + col * R, v);
}

// The 16 bool values (0x01 bytes) of a lane's rows j0 .. j0+15 of column `col`: 16 bytes into
// the tiled bool block (row order), or -- bitmap mode, words in the strided order -- 16 bits
// into bitmap `col` (rows >= n cleared).
template <bool BITS>
__device__ __forceinline__ void st_bool_out(const FeatArgs& a, uint8_t* __restrict__ bb, int64_t col, int64_t j0,
                                            uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
  if (BITS) {
    SA_DGUARD(col >= 0 && col < a.Cb, col, return);
    uint32_t b = bits_of_strided(w0, w1, w2, w3);
    if (a.a.n - j0 < 16) b &= (1u << (a.a.n - j0)) - 1u;
    a.bbits[col * a.bstride + j0 / 16] = (uint16_t)b;
  } else {
    st_bool16(bb, col, a.Cb, a.Rb, w0, w1, w2, w3);
  }
}

__device__ __forceinline__ void st_f64x2(double* __restrict__ base, int64_t col, int64_t C, int64_t R,
                                         double v0, double v1) {
  f64x2 v = {v0, v1};
  SA_DGUARD(col >= 0 && col < C, col, return);
#if SA_NUM_PROBE & 8  // probe: the f64 block is not written (wrong outputs)
  if (v0 == 1.2345e300) st16(base + col * R, v);
#else
  st16(base + col * R, v);
#endif
}

__device__ __forceinline__ void st_i64x2(int64_t* __restrict__ base, int64_t col, int64_t C, int64_t R,
                                         int64_t v0, int64_t v1) {
  i64x2 v = {(long long)v0, (long long)v1};
  SA_DGUARD(col >= 0 && col < C, col, return);
  st16(base + col * R, v);
}

__device__ __forceinline__ void st_f64x2(CondSink* s, int64_t col, int64_t, int64_t, double v0, double v1) {
  cond_store(s, col, (float)v0, (float)v1);
}

__device__ __forceinline__ void st_i64x2(CondSink* s, int64_t col, int64_t, int64_t, int64_t v0, int64_t v1) {
  cond_store(s, col, (float)v0, (float)v1);
}

// float32 form of the numeric blocks (sa_vaep_features_bits_f32: what xgboost learners compare,
// values rounded to nearest like xgboost's own float32 conversion): 8-B stores, 512 B per wave
// instruction
__device__ __forceinline__ void st_f64x2(float* __restrict__ base, int64_t col, int64_t C, int64_t R,
                                         double v0, double v1) {
  f32x2 v = {(float)v0, (float)v1};
  SA_DGUARD(col >= 0 && col < C, col, return);
  st16(base + col * R, v);
}

__device__ __forceinline__ void st_i64x2(float* __restrict__ base, int64_t col, int64_t C, int64_t R,
                                         int64_t v0, int64_t v1) {
  f32x2 v = {(float)v0, (float)v1};
  SA_DGUARD(col >= 0 && col < C, col, return);
  st16(base + col * R, v);
}

// SA_NUM_PROBE (diagnostic builds only, wrong values): bit 0 = no transcendental math in the
// numeric pass (sqrt / atan / division replaced by an add), bit 1 = no goalscore carry pass,
// bit 2 = no coordinate / time reads, bit 3 = no f64-block stores, bit 7 = coordinate / time
// reads from the first 8192 rows (L2 hits), bit 5 = no goalscore /
// label / formula stores (the stores that precede the main row loads).
#ifndef SA_NUM_PROBE
#define SA_NUM_PROBE 0
#endif
#ifndef SA_COND_FAMILY
#define SA_COND_FAMILY 1  // the COND pass in family-major column order (0: window-major, A/B)
#endif
#ifndef SA_NUM_FAMILY_MAJOR
#define SA_NUM_FAMILY_MAJOR 0  // numeric pass store order (num_features_kernel, KF = 3)
#endif
#if SA_NUM_PROBE & 1
#define NUM_SQRT(x) (x)
#else
#define NUM_SQRT(x) sqrt(x)
#endif

// nan_to_num(arctan(dy / dx)) of vaep/features.py:376 (atan(+-inf) = +-pi/2, 0/0 -> 0)
__device__ __forceinline__ double polar_angle(double dy, double dx) {
#if SA_NUM_PROBE & 1
  return dy + dx;
#else
  const double a = atan(dy / dx);
  return isnan(a) ? 0.0 : a;
#endif
}


// goal / owngoal bytes of a word of type / result bytes (vaep/labels.py:28-33;
// atomic/vaep/labels.py:27-28)
__device__ __forceinline__ void goal_bytes(uint32_t tw, uint32_t rw, bool atomic, uint32_t& g,
                                           uint32_t& o) {
  if (atomic) {
    g = bytes_eq(tw, AT_GOAL);
    o = bytes_eq(tw, AT_OWNGOAL);
  } else {
    const uint32_t shot = bytes_eq(tw, T_SHOT) | bytes_eq(tw, T_SHOT_PENALTY) |
                          bytes_eq(tw, T_SHOT_FREEKICK);
    g = shot & bytes_eq(rw, R_SUCCESS);
    o = shot & bytes_eq(rw, R_OWNGOAL);
  }
}

struct Gs16In {
  u32x4 ty, rs;
  int32_t tm[16];
};

template <bool ATOMIC>
__device__ __forceinline__ void gs16_load(const sa_frame& F, int64_t j0, int64_t n, Gs16In& v) {
  if (j0 >= 0 && j0 + 16 <= n) {
    v.ty = *reinterpret_cast<const u32x4*>(F.type_id + j0);
    v.rs = ATOMIC ? u32x4{0, 0, 0, 0} : *reinterpret_cast<const u32x4*>(F.result_id + j0);
    const int4* tp = reinterpret_cast<const int4*>(F.team + j0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int4 t = tp[q];
      v.tm[4 * q] = t.x;
      v.tm[4 * q + 1] = t.y;
      v.tm[4 * q + 2] = t.z;
      v.tm[4 * q + 3] = t.w;
    }
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v.ty[q] = ld_u8x4(F.type_id, j0 / 4 + q, n);
      v.rs[q] = ATOMIC ? 0u : ld_u8x4(F.result_id, j0 / 4 + q, n);
    }
#pragma unroll
    for (int m = 0; m < 16; ++m) v.tm[m] = ld_or0(F.team, j0 + m, n);
  }
}

constexpr int GS_LDS_PITCH = 18;  // i64 per lane: 16 rows + pad (144 B: 16-B aligned)

__device__ __forceinline__ void wave_sync() {  // LDS hand-off between the lanes of one wave
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ------------------------------------------------------------------------------ bool block
// actiontype_onehot, result_onehot, actiontype_result_onehot, bodypart_onehot, team.
constexpr int BOOL_TILE = 1024;  // rows per tile of the bool block image

// Column-group form (default): the bool image is swept front to back like a fill.  A wave
// owns one column group -- `gcols` consecutive block columns -- of one 1024-row tile, so a
// tile is written by `ngroups` short waves whose 1-KiB column runs follow each other in
// memory, and logical blocks are laid out per XCD (xcd_logical_block) so each XCD streams
// through its own contiguous eighth of the image.  Every wave rebuilds the tile's game-state
// windows from the id columns (L2 hits: a tile's groups run back to back on one XCD) and
// writes only the (family, window, value) columns inside its range.
constexpr int CG_WAVES = 4;  // waves per workgroup
#ifndef SA_BOOL_PROBE
#define SA_BOOL_PROBE 0
#endif
#define CG_EQ(w, v) bytes_eq((w), (v))

// WIDE (windowed mode, nb_prev_actions > 9: windows reach past the 8-row halo): each window's
// rows are gathered per action, row j - min(i, j - segment start), with the uncapped distance.
constexpr int BOOL_HALO = 8;  // rows before j0 held in registers: windows i <= 8 (k <= 9)
constexpr int WIDE_D_MAX = 1 << 30;

// The pass over logical workgroup `lblock` (bool_colgroup_kernel; and the bool workgroups of the
// SA_FUSED_STEP probe's one-launch step).
template <bool ATOMIC, bool EXPLICIT, bool BITS, bool WIDE>
__device__ __forceinline__ void bool_colgroup_body(const FeatArgs& args, int ngroups, int gcols,
                                                   int64_t lblock) {
  const int lane = threadIdx.x & (WAVE - 1);
  const int wv = threadIdx.x / WAVE;
  const sa_actions& A = args.a;
  const sa_feature_plan& P = args.p;
  const int64_t n = A.n;
  const int K = P.nb_prev_actions;
  const int64_t R = args.Rb;
  const int64_t w = lblock * CG_WAVES + wv;
  const int64_t tile0 = (w / ngroups) * BOOL_TILE;
  const int c_lo = (int)(w % ngroups) * gcols;
  const int c_hi = c_lo + gcols < (int)args.Cb ? c_lo + gcols : (int)args.Cb;
  const int64_t j0 = tile0 + (int64_t)lane * LANE_ACTS;
  const sa_frame& F0 = A.frames[0];
  const int tcol = P.bool_col[SA_XFN_TEAM];
  // team_1 .. team_{K-1} columns inside [c_lo, c_hi)?
  const bool need_team = tcol >= 0 && K > 1 && tcol < c_hi && tcol + K - 1 > c_lo;
  if (tile0 >= n || c_lo >= c_hi) return;
  uint8_t* bb = BITS ? nullptr : args.bout + tile_off(j0 < n ? j0 : tile0, 0, args.Cb, R);
  if (j0 >= n) return;
  // d = min(j - seg_start, 15) per action: segment of the tile start (same for all lanes),
  // then each lane advances to its own rows
  uint32_t dw[4] = {0, 0, 0, 0};
  int32_t dm[WIDE ? LANE_ACTS : 1];  // WIDE: j - seg_start per action, uncapped (up to 2^30)
#pragma unroll
  for (int m = 0; m < (WIDE ? LANE_ACTS : 1); ++m) dm[m] = 0;
  if (!EXPLICIT && K > 1) {
    SegCursor c = seg_at(A, tile0);
#pragma unroll
    for (int m = 0; m < LANE_ACTS; ++m) {
      const int64_t j = j0 + m;
      if (j < n) {
        seg_advance(A, c, j);
        const int64_t dd = j - c.s;
        if (WIDE) {
          dm[m] = dd > WIDE_D_MAX ? WIDE_D_MAX : (int32_t)dd;
        } else {
          const int d = dd > 15 ? 15 : (int)dd;
          dw[m >> 2] |= (uint32_t)d << (8 * (m & 3));
        }
      }
    }
  }
  uint32_t TR[6], RR[6], BR[6];  // rows j0-8 .. j0+15 (windowed mode)
  uint32_t tw[4], rw[4], bw[4];  // window i of the lane's 16 actions
  if (!EXPLICIT && !WIDE) {
#if SA_BOOL_PROBE & 1  // probe: the id words from the first 8K rows (L2 hits; wrong values)
    const int64_t wbase = ((j0 / 4) & 2047) + 2 - 2;
#else
    const int64_t wbase = j0 / 4 - 2;
#endif
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      TR[k] = ld_u8x4(F0.type_id, wbase + k, n);
      RR[k] = ATOMIC ? 0u : ld_u8x4(F0.result_id, wbase + k, n);
      BR[k] = ld_u8x4(F0.bodypart_id, wbase + k, n);
    }
  }
  const int c_type = P.bool_col[SA_XFN_ACTIONTYPE_ONEHOT];
  const int c_res = ATOMIC ? -1 : P.bool_col[SA_XFN_RESULT_ONEHOT];
  const int c_tr = ATOMIC ? -1 : P.bool_col[SA_XFN_ACTIONTYPE_RESULT_ONEHOT];
  const int c_bp = P.bool_col[SA_XFN_BODYPART_ONEHOT];
  const int ntypes = ATOMIC ? N_ATOMIC_NAMES : N_TYPES;
  // [v0, v1): values v of a family whose column base + v lies in [c_lo, c_hi)
  auto range = [&](int base, int nv, int& v0, int& v1) {
    v0 = c_lo - base > 0 ? c_lo - base : 0;
    v1 = c_hi - base < nv ? c_hi - base : nv;
  };
  for (int i = 0; i < K; ++i) {
    if (EXPLICIT) {
      const sa_frame& Fi = A.frames[i];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        tw[q] = ld_u8x4(Fi.type_id, j0 / 4 + q, n);
        rw[q] = ATOMIC ? 0u : ld_u8x4(Fi.result_id, j0 / 4 + q, n);
        bw[q] = ld_u8x4(Fi.bodypart_id, j0 / 4 + q, n);
      }
    } else if (WIDE) {  // window i gathered per action: row j - min(i, d) (features.py:83-88)
#pragma unroll
      for (int q = 0; q < 4; ++q) tw[q] = rw[q] = bw[q] = 0;
#pragma unroll
      for (int m = 0; m < LANE_ACTS; ++m) {
        const int64_t j = j0 + m;
        if (j < n) {
          const int64_t r = j - (dm[m] < i ? dm[m] : i);
          SA_DCHECK(r >= 0 && r <= j, r);
          tw[m >> 2] |= (uint32_t)F0.type_id[r] << (8 * (m & 3));
          if (!ATOMIC) rw[m >> 2] |= (uint32_t)F0.result_id[r] << (8 * (m & 3));
          bw[m >> 2] |= (uint32_t)F0.bodypart_id[r] << (8 * (m & 3));
        }
      }
    } else if (i == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        tw[q] = TR[2 + q];
        rw[q] = RR[2 + q];
        bw[q] = BR[2 + q];
      }
    } else {  // window i = window i-1 shifted one row, clamped bytes kept
      shift_rows(TR);
      if (!ATOMIC) shift_rows(RR);
      shift_rows(BR);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t mk = ge_mask(dw[q], i);
        tw[q] = (TR[2 + q] & mk) | (tw[q] & ~mk);
        rw[q] = (RR[2 + q] & mk) | (rw[q] & ~mk);
        bw[q] = (BR[2 + q] & mk) | (bw[q] & ~mk);
      }
    }
    // the compare operands: row order (byte block), strided order (bitmaps)
    uint32_t xt[4], xr[4], xb[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      xt[q] = tw[q];
      xr[q] = rw[q];
      xb[q] = bw[q];
    }
    if (BITS) {
      transpose_bytes4(xt);
      if (!ATOMIC) transpose_bytes4(xr);
      transpose_bytes4(xb);
    }
    int v0, v1;
    if (c_type >= 0) {
      const int base = c_type + i * ntypes;
      range(base, ntypes, v0, v1);
      for (int u = v0; u < v1; ++u) {
        if (!ATOMIC) {
          st_bool_out<BITS>(args, bb, base + u, j0, CG_EQ(xt[0], u), CG_EQ(xt[1], u), CG_EQ(xt[2], u),
                    CG_EQ(xt[3], u));
        } else {
          // 33 atomic names, 32 unique: 'interception' (ids 10 and 24) is ONE column true for
          // both ids (atomic/vaep/features.py:114-132 + atomic/spadl/config.py:25-36)
          const uint32_t id = u <= 23 ? (uint32_t)u : (uint32_t)u + 1;
          uint32_t m0 = CG_EQ(xt[0], id), m1 = CG_EQ(xt[1], id), m2 = CG_EQ(xt[2], id),
                   m3 = CG_EQ(xt[3], id);
          if (u == 10) {
            m0 |= CG_EQ(xt[0], AT_INTERCEPTION2);
            m1 |= CG_EQ(xt[1], AT_INTERCEPTION2);
            m2 |= CG_EQ(xt[2], AT_INTERCEPTION2);
            m3 |= CG_EQ(xt[3], AT_INTERCEPTION2);
          }
          st_bool_out<BITS>(args, bb, base + u, j0, m0, m1, m2, m3);
        }
      }
    }
    if (c_res >= 0) {
      const int base = c_res + i * N_RESULTS;
      range(base, N_RESULTS, v0, v1);
      for (int r = v0; r < v1; ++r)
        st_bool_out<BITS>(args, bb, base + r, j0, CG_EQ(xr[0], r), CG_EQ(xr[1], r), CG_EQ(xr[2], r),
                  CG_EQ(xr[3], r));
    }
    if (c_tr >= 0) {
      const int base = c_tr + i * N_TYPES * N_RESULTS;
      range(base, N_TYPES * N_RESULTS, v0, v1);
      if (v0 < v1) {
        // code = type*6 + result per byte (type <= 22, result <= 5: no carry between bytes)
        uint32_t cw[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) cw[q] = (xt[q] << 2) + (xt[q] << 1) + xr[q];
        for (int code = v0; code < v1; ++code)
          st_bool_out<BITS>(args, bb, base + code, j0, CG_EQ(cw[0], code), CG_EQ(cw[1], code),
                    CG_EQ(cw[2], code), CG_EQ(cw[3], code));
      }
    }
    if (c_bp >= 0) {
      const int base = c_bp + i * N_BODYPARTS;
      range(base, N_BODYPARTS, v0, v1);
      for (int b = v0; b < v1; ++b)
        st_bool_out<BITS>(args, bb, base + b, j0, CG_EQ(xb[0], b), CG_EQ(xb[1], b), CG_EQ(xb[2], b),
                  CG_EQ(xb[3], b));
    }
    const int tc = tcol + i - 1;
    if (need_team && i >= 1 && tc >= c_lo && tc < c_hi) {  // team_i (features.py:448-452)
      uint32_t m[4] = {0, 0, 0, 0};
#pragma unroll
      for (int mm = 0; mm < LANE_ACTS; ++mm) {
        int32_t t0, ti;
        if (EXPLICIT) {
          t0 = ld_or0(A.frames[0].team, j0 + mm, n);
          ti = ld_or0(A.frames[i].team, j0 + mm, n);
        } else {
          const int d = WIDE ? dm[mm] : (int)byte_of(dw[mm >> 2], mm & 3);
          const int s = d < i ? d : i;
          SA_DCHECK(s >= 0 && (WIDE || s <= BOOL_HALO), s);
          // team codes straight from L1/L2 (a few waves per tile need them): the kernel keeps
          // no LDS, so xT workgroups with large LDS footprints co-reside with it
#if SA_BOOL_PROBE & 1
          t0 = ld_or0(F0.team, ((j0 + mm) & 8191) + 16, n);
          ti = ld_or0(F0.team, ((j0 + mm) & 8191) + 16 - s, n);
#else
          t0 = ld_or0(F0.team, j0 + mm, n);
          ti = ld_or0(F0.team, j0 + mm - s, n);
#endif
        }
        if (BITS)  // strided order: word mm & 3, byte mm >> 2
          m[mm & 3] |= (uint32_t)(t0 == ti) << (8 * (mm >> 2));
        else
          m[mm >> 2] |= (uint32_t)(t0 == ti) << (8 * (mm & 3));
      }
      st_bool_out<BITS>(args, bb, tc, j0, m[0], m[1], m[2], m[3]);
    }
  }
}

template <bool ATOMIC, bool EXPLICIT, bool BITS, bool WIDE = false>
__global__ __launch_bounds__(64 * CG_WAVES) void bool_colgroup_kernel(FeatArgs args, int ngroups,
                                                                      int gcols) {
  bool_colgroup_body<ATOMIC, EXPLICIT, BITS, WIDE>(args, ngroups, gcols, xcd_logical_block());
}

// ------------------------------------------------------------------------------ f64/i64 block
// A lane owns 2 consecutive actions (jb, jb+1); one store instruction writes 1 KiB of one
// column, and with 128-row tiles (SA_NUM_TILE_QUANTUM) a wave's pass over 128 rows writes
// one contiguous [C x 128] slab.
struct NumCols {  // first column of each transformer in the f64 / i64 blocks (-1 = absent)
  int at, re, bi, ti, tf, sl, el, sp, ep, mv, td, sd, lo, po, mp, di;
  int nf, ni;  // column counts of the f64 / i64 blocks (bounds checks of the debug build)
};

struct Win {  // one game-state window of the lane's 2 actions (flipped coordinates)
  double c0[2], c1[2], c2[2], c3[2], ts[2];
  int32_t per[2], typ[2], res[2], bp[2];
};

// Column families of the numeric pass (emit_window's `fam`): FAM_ALL = every family of window
// i; otherwise one family, so a caller can write the columns family by family (each family's
// windows are adjacent block columns).
enum { FAM_ALL = -1, FAM_IDS = 0, FAM_TIME, FAM_SL, FAM_EL, FAM_SP, FAM_EP, FAM_MV, FAM_TD, FAM_SD,
       FAM_LO, FAM_PO, FAM_MP, FAM_DI };
#define FAM_ON(f) (fam == FAM_ALL || fam == (f))

// Every f64 / i64 column of window i (features.py:151-499, atomic/vaep/features.py:135-226), or
// only family `fam`'s.
template <bool ATOMIC, typename FT, typename IT>
__device__ __forceinline__ void emit_window(const NumCols& C, int i, const Win& w,
                                            const double (&sx0)[2], const double (&sy0)[2],
                                            const double (&t0)[2], FT* __restrict__ fb,
                                            IT* __restrict__ ib, int64_t Rf, int64_t Ri, int fam = FAM_ALL) {
  if (FAM_ON(FAM_IDS)) {
    if (C.at >= 0) st_i64x2(ib, C.at + i, C.ni, Ri, w.typ[0], w.typ[1]);
    if (C.re >= 0) st_i64x2(ib, C.re + i, C.ni, Ri, w.res[0], w.res[1]);
    if (C.bi >= 0) st_i64x2(ib, C.bi + i, C.ni, Ri, w.bp[0], w.bp[1]);
  }
  if (FAM_ON(FAM_TIME) && C.ti >= 0) st_i64x2(ib, C.ti + i, C.ni, Ri, w.per[0], w.per[1]);
  if (FAM_ON(FAM_TIME) && C.tf >= 0) {
    st_f64x2(fb, C.tf + 2 * i, C.nf, Rf, w.ts[0], w.ts[1]);
    // ((period_id - 1) * 45 * 60) + time_seconds   (features.py:313)
    st_f64x2(fb, C.tf + 2 * i + 1, C.nf, Rf, (double)((w.per[0] - 1) * 2700) + w.ts[0],
             (double)((w.per[1] - 1) * 2700) + w.ts[1]);
  }
  if (!ATOMIC) {
    if (FAM_ON(FAM_SL) && C.sl >= 0) {
      st_f64x2(fb, C.sl + 2 * i, C.nf, Rf, w.c0[0], w.c0[1]);
      st_f64x2(fb, C.sl + 2 * i + 1, C.nf, Rf, w.c1[0], w.c1[1]);
    }
    if (FAM_ON(FAM_EL) && C.el >= 0) {
      st_f64x2(fb, C.el + 2 * i, C.nf, Rf, w.c2[0], w.c2[1]);
      st_f64x2(fb, C.el + 2 * i + 1, C.nf, Rf, w.c3[0], w.c3[1]);
    }
    if (FAM_ON(FAM_SP) && C.sp >= 0) {
      double dist[2], ang[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const double dx = fabs(FIELD_L - w.c0[e]), dy = fabs(GOAL_Y - w.c1[e]);
        dist[e] = NUM_SQRT(dx * dx + dy * dy);
        ang[e] = polar_angle(dy, dx);
      }
      st_f64x2(fb, C.sp + 2 * i, C.nf, Rf, dist[0], dist[1]);
      st_f64x2(fb, C.sp + 2 * i + 1, C.nf, Rf, ang[0], ang[1]);
    }
    if (FAM_ON(FAM_EP) && C.ep >= 0) {
      double dist[2], ang[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const double dx = fabs(FIELD_L - w.c2[e]), dy = fabs(GOAL_Y - w.c3[e]);
        dist[e] = NUM_SQRT(dx * dx + dy * dy);
        ang[e] = polar_angle(dy, dx);
      }
      st_f64x2(fb, C.ep + 2 * i, C.nf, Rf, dist[0], dist[1]);
      st_f64x2(fb, C.ep + 2 * i + 1, C.nf, Rf, ang[0], ang[1]);
    }
    if (FAM_ON(FAM_MV) && C.mv >= 0) {
      double mdx[2], mdy[2], mv[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        mdx[e] = w.c2[e] - w.c0[e];
        mdy[e] = w.c3[e] - w.c1[e];
        mv[e] = NUM_SQRT(mdx[e] * mdx[e] + mdy[e] * mdy[e]);
      }
      st_f64x2(fb, C.mv + 3 * i, C.nf, Rf, mdx[0], mdx[1]);
      st_f64x2(fb, C.mv + 3 * i + 1, C.nf, Rf, mdy[0], mdy[1]);
      st_f64x2(fb, C.mv + 3 * i + 2, C.nf, Rf, mv[0], mv[1]);
    }
    if (FAM_ON(FAM_SD) && i >= 1 && C.sd >= 0) {  // space_delta: a_i end - a0 start (features.py:491-499)
      double sdx[2], sdy[2], sm[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        sdx[e] = w.c2[e] - sx0[e];
        sdy[e] = w.c3[e] - sy0[e];
        sm[e] = NUM_SQRT(sdx[e] * sdx[e] + sdy[e] * sdy[e]);
      }
      st_f64x2(fb, C.sd + 3 * (i - 1), C.nf, Rf, sdx[0], sdx[1]);
      st_f64x2(fb, C.sd + 3 * (i - 1) + 1, C.nf, Rf, sdy[0], sdy[1]);
      st_f64x2(fb, C.sd + 3 * (i - 1) + 2, C.nf, Rf, sm[0], sm[1]);
    }
  } else {
    if (FAM_ON(FAM_LO) && C.lo >= 0) {
      st_f64x2(fb, C.lo + 2 * i, C.nf, Rf, w.c0[0], w.c0[1]);
      st_f64x2(fb, C.lo + 2 * i + 1, C.nf, Rf, w.c1[0], w.c1[1]);
    }
    if (FAM_ON(FAM_PO) && C.po >= 0) {
      double dist[2], ang[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const double dx = fabs(FIELD_L - w.c0[e]), dy = fabs(GOAL_Y - w.c1[e]);
        dist[e] = NUM_SQRT(dx * dx + dy * dy);
        ang[e] = polar_angle(dy, dx);
      }
      st_f64x2(fb, C.po + 2 * i, C.nf, Rf, dist[0], dist[1]);
      st_f64x2(fb, C.po + 2 * i + 1, C.nf, Rf, ang[0], ang[1]);
    }
    if (FAM_ON(FAM_MP) && C.mp >= 0) {  // atomic/vaep/features.py:196-199
      double md[2], ma[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        md[e] = sqrt(w.c2[e] * w.c2[e] + w.c3[e] * w.c3[e]);
        ma[e] = (w.c3[e] == 0.0) ? 0.0 : atan2(w.c3[e], w.c2[e]);
      }
      st_f64x2(fb, C.mp + 2 * i, C.nf, Rf, md[0], md[1]);
      st_f64x2(fb, C.mp + 2 * i + 1, C.nf, Rf, ma[0], ma[1]);
    }
    if (FAM_ON(FAM_DI) && C.di >= 0) {  // atomic/vaep/features.py:219-224
      double ox[2], oy[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const double td = sqrt(w.c2[e] * w.c2[e] + w.c3[e] * w.c3[e]);
        ox[e] = td > 0.0 ? w.c2[e] / td : w.c2[e];
        oy[e] = td > 0.0 ? w.c3[e] / td : w.c3[e];
      }
      st_f64x2(fb, C.di + 2 * i, C.nf, Rf, ox[0], ox[1]);
      st_f64x2(fb, C.di + 2 * i + 1, C.nf, Rf, oy[0], oy[1]);
    }
  }
  if (FAM_ON(FAM_TD) && i >= 1 && C.td >= 0)  // time_delta: a0 time - a_i time (features.py:469-473)
    st_f64x2(fb, C.td + (i - 1), C.nf, Rf, t0[0] - w.ts[0], t0[1] - w.ts[1]);
}

// play_left_to_right of one window value pair, keyed on the CURRENT action (features.py:109-115)
template <bool ATOMIC>
__device__ __forceinline__ void flip(Win& w, int e) {
  w.c0[e] = FIELD_L - w.c0[e];
  w.c1[e] = FIELD_W - w.c1[e];
  if (ATOMIC) {
    w.c2[e] = -w.c2[e];
    w.c3[e] = -w.c3[e];
  } else {
    w.c2[e] = FIELD_L - w.c2[e];
    w.c3[e] = FIELD_W - w.c3[e];
  }
}

__device__ __forceinline__ void load_row(const sa_frame& F, int64_t r, bool atomic, Win& w, int e) {
  w.c0[e] = F.c0[r];
  w.c1[e] = F.c1[r];
  w.c2[e] = F.c2[r];
  w.c3[e] = F.c3[r];
  w.ts[e] = F.time_seconds[r];
  w.per[e] = F.period_id[r];
  w.typ[e] = F.type_id[r];
  w.res[e] = atomic ? 0 : F.result_id[r];
  w.bp[e] = F.bodypart_id[r];
}

struct Row {  // one action row, raw: 5 f64 + the 4 u8 ids packed in one word
  double c0, c1, c2, c3, ts;
  uint32_t ids;  // period | type << 8 | result << 16 | bodypart << 24
};

__device__ __forceinline__ void load_row1(const sa_frame& F, int64_t r, bool atomic, Row& o) {
  o.c0 = F.c0[r];
  o.c1 = F.c1[r];
  o.c2 = F.c2[r];
  o.c3 = F.c3[r];
  o.ts = F.time_seconds[r];
  o.ids = (uint32_t)F.period_id[r] | ((uint32_t)F.type_id[r] << 8) |
          ((uint32_t)(atomic ? 0 : F.result_id[r]) << 16) | ((uint32_t)F.bodypart_id[r] << 24);
}

// SA_NUM_NTL: the numeric pass's streamed inputs -- bit 0 the coordinates and times, bit 1 the
// probabilities -- loaded non-temporally, so the ~1 GB they stream per pass does not push the
// id / team columns (7 B/action) the bool pass reads next out of the Infinity Cache.  Every
// streamed byte is loaded once (the pool rows come from the neighbour lane), so nothing is
// lost by not caching them.  Pair A/B (profiles/r03_numeric_pass_ab.md): numeric step pass +
// bool pass 3.035 -> 2.940 ms (slow box), 2.591 -> 2.541 ms (fast box); coordinates or
// probabilities alone keep the columns only partly resident
#ifndef SA_NUM_NTL
#define SA_NUM_NTL 3
#endif
template <int BIT = 1, typename V>
__device__ __forceinline__ V ld_stream(const V* p) {  // BIT 1: coordinates / time, 2: probabilities
  if constexpr ((SA_NUM_NTL & BIT) != 0) return __builtin_nontemporal_load(p);
  return *p;
}

// rows r, r+1 (r even: 16-B aligned f64 pairs, 2-B aligned id pairs)
__device__ __forceinline__ void load_pair(const sa_frame& F, int64_t r, bool atomic, Row& a, Row& b) {
#if SA_NUM_PROBE & 4  // probe: no coordinate / time reads (wrong values)
  const double q = (double)(r & 1023);
  const f64x2 x0 = {q, q + 1}, x1 = {q * 0.5, q}, x2 = {q + 3, q}, x3 = {q, q * 0.25}, x4 = {q, q + 2};
#elif SA_NUM_PROBE & 128  // probe: coordinate / time reads from the first 8192 rows (L2 hits; wrong values)
  const int64_t rq = r & 8190;
  const f64x2 x0 = *reinterpret_cast<const f64x2*>(F.c0 + rq);
  const f64x2 x1 = *reinterpret_cast<const f64x2*>(F.c1 + rq);
  const f64x2 x2 = *reinterpret_cast<const f64x2*>(F.c2 + rq);
  const f64x2 x3 = *reinterpret_cast<const f64x2*>(F.c3 + rq);
  const f64x2 x4 = *reinterpret_cast<const f64x2*>(F.time_seconds + rq);
#else
  const f64x2 x0 = ld_stream(reinterpret_cast<const f64x2*>(F.c0 + r));
  const f64x2 x1 = ld_stream(reinterpret_cast<const f64x2*>(F.c1 + r));
  const f64x2 x2 = ld_stream(reinterpret_cast<const f64x2*>(F.c2 + r));
  const f64x2 x3 = ld_stream(reinterpret_cast<const f64x2*>(F.c3 + r));
  const f64x2 x4 = ld_stream(reinterpret_cast<const f64x2*>(F.time_seconds + r));
#endif
  const uint32_t pe = *reinterpret_cast<const uint16_t*>(F.period_id + r);
  const uint32_t ty = *reinterpret_cast<const uint16_t*>(F.type_id + r);
  const uint32_t rs = atomic ? 0u : *reinterpret_cast<const uint16_t*>(F.result_id + r);
  const uint32_t bo = *reinterpret_cast<const uint16_t*>(F.bodypart_id + r);
  a = Row{x0[0], x1[0], x2[0], x3[0], x4[0],
          (pe & 0xFF) | ((ty & 0xFF) << 8) | ((rs & 0xFF) << 16) | ((bo & 0xFF) << 24)};
  b = Row{x0[1], x1[1], x2[1], x3[1], x4[1],
          (pe >> 8) | ((ty >> 8) << 8) | ((rs >> 8) << 16) | ((bo >> 8) << 24)};
}

__device__ __forceinline__ Row shfl_up_row(const Row& r) {  // lane l gets lane l-1's row
  Row o;
  o.c0 = __shfl_up(r.c0, 1, WAVE);
  o.c1 = __shfl_up(r.c1, 1, WAVE);
  o.c2 = __shfl_up(r.c2, 1, WAVE);
  o.c3 = __shfl_up(r.c3, 1, WAVE);
  o.ts = __shfl_up(r.ts, 1, WAVE);
  o.ids = __shfl_up(r.ids, 1, WAVE);
  return o;
}

__device__ __forceinline__ void row_to_win(const Row& r, Win& w, int e) {
  w.c0[e] = r.c0;
  w.c1[e] = r.c1;
  w.c2[e] = r.c2;
  w.c3[e] = r.c3;
  w.ts[e] = r.ts;
  w.per[e] = r.ids & 0xFF;
  w.typ[e] = (r.ids >> 8) & 0xFF;
  w.res[e] = (r.ids >> 16) & 0xFF;
  w.bp[e] = r.ids >> 24;
}

// ------------------------------------------------------------------------------ goalscore,
// fused into the numeric pass (windowed mode).  features.py:505-539 /
// atomic/vaep/features.py:229-260: per segment, A = team of the segment's first row; for each
// action the goals of its own team and of the other team before it (exclusive cumsum of the
// goal / owngoal credits) and their difference.  A wave's 128 rows need (1) the goals of the
// segment of its first row between that segment's start and the wave's first row -- counted
// by the whole wave, 16 rows per lane per pass, from L2 (the neighbouring tiles of the same
// game run on the same XCD) -- and (2) the exclusive counts inside the wave: four 64-bit
// ballots (credits of A and of B on even and on odd rows) and a popcount of the lanes between
// the row's segment start and the row.  No inter-wave dependency, no extra launch.

// (goals of A, goals of B) in rows [s, e) of one segment whose first-row team is `ta`, packed
// as low / high 32 bits; every lane of the wave must call it and gets the total.
template <bool ATOMIC>
__device__ __forceinline__ uint64_t wave_goals(const sa_frame& F, int64_t n, int64_t s, int64_t e,
                                               int32_t ta) {
  const int lane = threadIdx.x & (WAVE - 1);
  uint64_t acc = 0;
  for (int64_t base = s & ~(int64_t)15; base < e; base += 16 * WAVE) {  // wave-uniform
    const int64_t j0 = base + 16 * lane;
    if (j0 < e) {
      Gs16In v;
      gs16_load<ATOMIC>(F, j0, n, v);
      uint32_t gm = 0, om = 0, am = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t gb, ob;
        goal_bytes(v.ty[q], v.rs[q], ATOMIC, gb, ob);
        gm |= pack4(gb) << (4 * q);
        om |= pack4(ob) << (4 * q);
      }
#pragma unroll
      for (int m = 0; m < 16; ++m) am |= (uint32_t)(v.tm[m] == ta) << m;
      const int lo = s > j0 ? (int)(s - j0) : 0;
      const int hi = e < j0 + 16 ? (int)(e - j0) : 16;
      const uint32_t vm = lo >= hi ? 0u : (0xFFFFu >> (16 - (hi - lo))) << lo;
      const uint32_t gA = ((gm & am) | (om & ~am)) & vm, gB = ((gm & ~am) | (om & am)) & vm;
      acc += (uint64_t)__popc(gA) | ((uint64_t)__popc(gB) << 32);
    }
  }
#pragma unroll
  for (int off = WAVE / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, WAVE);
  return acc;
}

// lanes [a, b) of a 64-bit ballot (0 <= a, b <= 64)
__device__ __forceinline__ uint64_t lane_range(int a, int b) {
  const uint64_t below_b = b >= 64 ? ~0ull : ((1ull << b) - 1ull);
  const uint64_t below_a = a >= 64 ? ~0ull : ((1ull << a) - 1ull);
  return a >= b ? 0ull : (below_b & ~below_a);
}

// goalscore_team / _opponent / _diff of the lane's rows jb, jb+1 (wave rows wb .. wb+127, rows
// >= n get don't-care padding like the other columns) into v[column][row].  Loads only: the
// caller stores after the wave's last load (see num_features_kernel).  Every lane of the wave
// must call it; `c` = a segment cursor at or before row jb (clamped to n - 1).
template <bool ATOMIC>
__device__ __forceinline__ void goalscore_pair(const sa_actions& A, int64_t wb, int64_t jb, SegCursor c,
                                               int64_t (&v)[3][2]) {
  const int64_t n = A.n;
  const sa_frame& F = A.frames[0];
  const int lane = threadIdx.x & (WAVE - 1);
  const SegCursor c0 = wave_cursor(A, wb);  // segment of the wave's first row (uniform)
  uint64_t carry = 0;
  if (c0.s < wb && !(SA_NUM_PROBE & 2)) carry = wave_goals<ATOMIC>(F, n, c0.s, wb, F.team[c0.s]);
  bool gA[2], gB[2], isA[2];
  int64_t s[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int64_t j = jb + e < n ? jb + e : n - 1;
    seg_advance(A, c, j);
    s[e] = c.s;
    const int t = F.type_id[j];
    bool goal, og;
    if (ATOMIC) {
      goal = t == AT_GOAL;
      og = t == AT_OWNGOAL;
    } else {
      const bool shot = t == T_SHOT || t == T_SHOT_PENALTY || t == T_SHOT_FREEKICK;
      const int r = F.result_id[j];
      goal = shot && r == R_SUCCESS;
      og = shot && r == R_OWNGOAL;
    }
    isA[e] = F.team[j] == F.team[c.s];
    const bool valid = jb + e < n;
    gA[e] = valid && ((goal && isA[e]) || (og && !isA[e]));
    gB[e] = valid && ((goal && !isA[e]) || (og && isA[e]));
  }
  const uint64_t EA = __ballot(gA[0]), OA = __ballot(gA[1]);
  const uint64_t EB = __ballot(gB[0]), OB = __ballot(gB[1]);
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int t = 2 * lane + e;                           // row offset in the wave
    const int lo = s[e] > wb ? (int)(s[e] - wb) : 0;      // first row of the segment in the wave
    const uint64_t me = lane_range((lo + 1) >> 1, (t + 1) >> 1);  // even rows in [lo, t)
    const uint64_t mo = lane_range(lo >> 1, t >> 1);              // odd rows in [lo, t)
    int64_t cA = __popcll(EA & me) + __popcll(OA & mo);
    int64_t cB = __popcll(EB & me) + __popcll(OB & mo);
    if (s[e] < wb) {
      cA += (int64_t)(carry & 0xFFFFFFFFull);
      cB += (int64_t)(carry >> 32);
    }
    const int64_t tm = isA[e] ? cA : cB, op = isA[e] ? cB : cA;
    v[0][e] = tm;
    v[1][e] = op;
    v[2][e] = tm - op;
  }
}

// ------------------------------------------------------------------------------ tail in the
// numeric pass (sa_vaep_step_f64): labels + f64 formula of the lane's rows jb, jb+1.
template <bool ATOMIC, typename T>
__device__ __forceinline__ void formula_rows(const sa_actions& A, const T* __restrict__ ps,
                                             const T* __restrict__ pc, T* __restrict__ off,
                                             T* __restrict__ def, T* __restrict__ val, bool vec_ok,
                                             int64_t j0, SegCursor& cur);
template <bool ATOMIC, typename T, typename V>
__device__ __forceinline__ bool formula_vals(const sa_actions& A, const T* __restrict__ ps,
                                             const T* __restrict__ pc, bool vec_ok, int64_t j0, SegCursor& cur,
                                             V& vo, V& vd, V& vv, const double* t_in = nullptr);

// goal (bit 0) / owngoal (bit 1) / shot (bit 2, atomic goal_from_shot) of row j
template <bool ATOMIC>
__device__ __forceinline__ uint32_t label_bits(const sa_frame& F, int64_t j) {
  const int t = F.type_id[j];
  if (ATOMIC) return (uint32_t)(t == AT_GOAL) | ((uint32_t)(t == AT_OWNGOAL) << 1) | ((uint32_t)(t == T_SHOT) << 2);
  const bool shot = t == T_SHOT || t == T_SHOT_PENALTY || t == T_SHOT_FREEKICK;
  const int r = F.result_id[j];
  return (uint32_t)(shot && r == R_SUCCESS) | ((uint32_t)(shot && r == R_OWNGOAL) << 1);
}

// labels.scores / concedes / goal_from_shot (vaep/labels.py:9-116, atomic/vaep/labels.py:9-107)
// of the lane's rows jb, jb+1 in the numeric pass's layout (lane l = rows wb + 2l, +1): the
// look-ahead rows jb+2 .. jb+11 come from lanes l+1 .. l+5 by shuffles, the last five lanes load
// the rows after the wave themselves.  nr_actions <= SA_STEP_MAX_NR.  Every lane of the wave
// must call it; `c` = a segment cursor at or before row jb (clamped to n - 1).
constexpr int SA_STEP_MAX_NR = 11;
template <bool ATOMIC>
__device__ __forceinline__ void labels_pair(const sa_actions& A, int nr, int64_t jb, SegCursor c,
                                            uint32_t& so, uint32_t& cout, uint32_t& go) {
  const int64_t n = A.n;
  const sa_frame& F = A.frames[0];
  const int lane = threadIdx.x & (WAVE - 1);
  uint32_t bits[6];   // rows jb + 2k (low nibble), jb + 2k + 1 (high nibble)
  int32_t tm[6][2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int64_t j = jb + q < n ? jb + q : n - 1;
    tm[0][q] = F.team[j];
    bits[0] = q ? bits[0] | (label_bits<ATOMIC>(F, j) << 4) : label_bits<ATOMIC>(F, j);
  }
#pragma unroll
  for (int k = 1; k < 6; ++k) {
    bits[k] = __shfl_down(bits[0], k, WAVE);
    tm[k][0] = __shfl_down(tm[0][0], k, WAVE);
    tm[k][1] = __shfl_down(tm[0][1], k, WAVE);
    if (lane + k >= WAVE) {  // rows after the wave
      uint32_t b = 0;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int64_t j = jb + 2 * k + q < n ? jb + 2 * k + q : n - 1;
        tm[k][q] = F.team[j];
        b |= label_bits<ATOMIC>(F, j) << (4 * q);
      }
      bits[k] = b;
    }
  }
  so = cout = go = 0;
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int64_t j = jb + e;
    if (j < n) {
      seg_advance(A, c, j);
      const int64_t last = c.e - 1;
      const int64_t hj = j + nr - 1 < last ? j + nr - 1 : last;
      const int hi = (int)(hj - jb);  // largest look-ahead offset from jb
      const int32_t tj = tm[0][e];
      const uint32_t bj = bits[0] >> (4 * e);
      bool s = bj & 1u, cc = (bj >> 1) & 1u;
#pragma unroll
      for (int d = e + 1; d <= SA_STEP_MAX_NR; ++d) {
        if (d <= hi) {
          const uint32_t b = bits[d >> 1] >> (4 * (d & 1));
          const bool same = tm[d >> 1][d & 1] == tj;
          s |= ((b & 1u) && same) || ((b & 2u) && !same);
          cc |= ((b & 1u) && !same) || ((b & 2u) && same);
        }
      }
      bool gf;
      if (ATOMIC)  // shot followed by a goal; the segment's last row compares NaN -> False
        gf = ((bj >> 2) & 1u) && j < last && ((bits[(e + 1) >> 1] >> (4 * ((e + 1) & 1))) & 1u);
      else
        gf = bj & 1u;
      so |= (uint32_t)s << (8 * e);
      cout |= (uint32_t)cc << (8 * e);
      go |= (uint32_t)gf << (8 * e);
    }
  }
}

// the labels of rows jb, jb+1 (labels_pair's bytes) into the label columns
__device__ __forceinline__ void labels_store(int64_t n, uint8_t* __restrict__ sc, uint8_t* __restrict__ co,
                                             uint8_t* __restrict__ gfs, int64_t jb, uint32_t so, uint32_t cout,
                                             uint32_t go) {
  if (jb < n && !(SA_NUM_PROBE & 32)) {
    if (jb + 1 < n) {
      if (sc) *reinterpret_cast<uint16_t*>(sc + jb) = (uint16_t)so;
      if (co) *reinterpret_cast<uint16_t*>(co + jb) = (uint16_t)cout;
      if (gfs) *reinterpret_cast<uint16_t*>(gfs + jb) = (uint16_t)go;
    } else {
      if (sc) sc[jb] = (uint8_t)so;
      if (co) co[jb] = (uint8_t)cout;
      if (gfs) gfs[jb] = (uint8_t)go;
    }
  }
}

// KF = 3: windowed mode with nb_prev_actions <= 3.  The pair's rows jb-2 .. jb+1 are read
// once (16-B loads) and the windows are formed in registers (see the loop below).
// KF = 0: any mode / any k (explicit frames: k <= SA_MAX_FRAMES; windowed: any k): per-window
// row loads.
// Waves per SIMD the compiler must leave room for (a VGPR cap; SA_NUM_WAVES, A/B builds).  The
// SPADL step form fits 128 VGPRs without spills at 4 waves (its pool rows come by shuffles),
// but whether that helps depends on the box: the step's pair 1.336 vs 1.389 ms on a fast box,
// 1.592 vs 1.549 ms on a slow one (profiles/r03_numeric_pass_ab.md), so no form is capped.
#ifndef SA_NUM_WAVES
#define SA_NUM_WAVES 0
#endif
template <bool ATOMIC, bool TAIL>
constexpr int num_min_waves() {
  return SA_NUM_WAVES > 0 ? SA_NUM_WAVES : 1;
}
// The pass over the wave's 128 rows from wave_base.  F0: frames[0] with the streamed columns
// (coordinates, time) where the caller wants them read from; ps / pc: the probabilities (TAIL).
template <bool ATOMIC, bool EXPLICIT, int KF, bool TAIL = false, bool N32 = false, bool COND = false>
__device__ __forceinline__ void num_features_body(const FeatArgs& args, int64_t wave_base, const sa_frame& F0,
                                                  const double* ps_in, const double* pc_in) {
  // N32: the f64 and i64 blocks hold float32 values (sa_vaep_features_bits_f32); COND: no blocks,
  // the columns' split conditions as bitmaps (sa_vaep_features_conditions)
  using FT = typename std::conditional<COND, CondSink, typename std::conditional<N32, float, double>::type>::type;
  using IT = typename std::conditional<COND, CondSink, typename std::conditional<N32, float, int64_t>::type>::type;
  const int lane = threadIdx.x & (WAVE - 1);
  const sa_actions& A = args.a;
  const sa_feature_plan& P = args.p;
  const int64_t n = A.n;
  const int K = P.nb_prev_actions;
  const int64_t Rf = args.Rf, Ri = args.Ri;
  // whole wave past the end (uniform: the goalscore ballots need every lane)
  if (wave_base >= n || (args.row_end > 0 && wave_base >= args.row_end)) return;
  CondAcc acc{0, 0, 0, -64, 0.0f, 0};
  CondSink sink_f, sink_i;
  if constexpr (COND) {
    sink_f = cond_sink(args.cond_fstart, (int)args.Cf + 1, args, wave_base, n, &acc);
    sink_i = cond_sink(args.cond_istart, (int)args.Ci + 1, args, wave_base, n, &acc);
  }
  auto fblock = [&](int64_t j) -> FT* {
    if constexpr (COND) return &sink_f;
    else return reinterpret_cast<FT*>(args.fout) + tile_off(j, 0, args.Cf, Rf);
  };
  auto iblock = [&](int64_t j) -> IT* {
    if constexpr (COND) return &sink_i;
    else return reinterpret_cast<IT*>(args.iout) + tile_off(j, 0, args.Ci, Ri);
  };
  SegCursor cur = {0, 0, 0};
  const int gcol = EXPLICIT ? -1 : P.i64_col[SA_XFN_GOALSCORE];
  // A lane owns rows jb, jb+1 (NUM_PAIRS == 1).  Every load of the wave -- its rows, the goal
  // credits, the label look-ahead, the probabilities -- is issued before its first store: on
  // gfx950 a wait for a load also waits for every store issued before it (one vmcnt), so a
  // store-then-load order made each wave sit out several write round trips.
  const int64_t jw = wave_base + 2 * lane;  // this lane's first row (may be >= n in the last wave)
  int64_t jb = jw;
  if (COND && jb >= n) jb = (n - 1) & ~(int64_t)1;
  const int64_t jq = jb < n ? jb : ((n - 1) & ~(int64_t)1);  // rows this lane loads (clamped)
  int64_t jr[2];
  jr[0] = jq;
  jr[1] = jq + 1 < n ? jq + 1 : n - 1;  // padded tail rows recompute row n-1
  Row cand[2], pool[2];
  if (KF == 3) {
    // the pair's window rows: cand = rows jb, jb+1 (each input row is loaded by ONE lane:
    // streamed, read once from HBM), pool = the older rows jb-1, jb-2 = the previous lane's
    // cand rows, by shuffles; lane 0 loads its own (the previous tile's last rows).  Lanes
    // clamped past the batch end (jw >= n) get don't-care pool rows: their outputs are not
    // stored (COND: masked off in cond_store)
    if (jq + 2 <= n) {
      load_pair(F0, jq, ATOMIC, cand[0], cand[1]);
    } else {  // the batch's last row: guarded scalar loads
      load_row1(F0, jr[0], ATOMIC, cand[0]);
      load_row1(F0, jr[1], ATOMIC, cand[1]);
    }
    pool[0] = shfl_up_row(cand[1]);
    pool[1] = shfl_up_row(cand[0]);
    if (lane == 0) {
      if (jq >= 2) {
        load_pair(F0, jq - 2, ATOMIC, pool[1], pool[0]);
      } else {  // the batch's first rows: windows clamp to row 0
        load_row1(F0, jq - 1 < 0 ? 0 : jq - 1, ATOMIC, pool[0]);
        load_row1(F0, 0, ATOMIC, pool[1]);
      }
    }
  }
  // the block addresses of rows jb, jb+1 (column 0; COND: the condition sinks), before any store
  // so that no address arithmetic waits behind one
  FT* fb = fblock(jq);
  IT* ib = iblock(jq);
  IT* gib = iblock((jw < n ? jw : n - 1) & ~(int64_t)1);
  int64_t gs[3][2];
  uint32_t lso = 0, lco = 0, lgo = 0;
  f64x2 fo, fd, fv;
  bool fok = false;
  int dd[2] = {0, 0};
  bool away[2] = {false, false};
  if (!EXPLICIT) {
    const int64_t jl = jw < n ? jw : n - 1;
    cur = wave_cursor(A, wave_base);
    seg_advance(A, cur, jl);
    if (gcol >= 0) goalscore_pair<ATOMIC>(A, wave_base, jw, cur, gs);
    if (TAIL) {  // labels + formula of the same rows (every lane of the wave present)
      labels_pair<ATOMIC>(A, args.nr, jw, cur, lso, lco, lgo);
      if (args.ps) {  // uniform: labels only when no probabilities are given
        SegCursor fc = cur;
        const double t_rows[2] = {cand[0].ts, cand[1].ts};  // rows jw, jw+1 (KF = 3)
        fok = formula_vals<ATOMIC, double>(A, ps_in, pc_in, args.vec_ok, jw, fc, fo, fd, fv,
                                           KF == 3 ? t_rows : nullptr);
      }
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int64_t j = jr[e];
      seg_advance(A, cur, j);
      const int64_t d = j - cur.s;
      dd[e] = d > WIDE_D_MAX ? WIDE_D_MAX : (int)d;  // compared with the window index only
      away[e] = A.home_team != nullptr && F0.team[j] != A.home_team[cur.g];
    }
    // -- every load is out; the stores follow
    if (gcol >= 0 && (jw < n || COND) && !(SA_NUM_PROBE & 32)) {  // condition sinks: whole wave, tail masked
#pragma unroll
      for (int k = 0; k < 3; ++k) st_i64x2(gib, gcol + k, (int)args.Ci, Ri, gs[k][0], gs[k][1]);
    }
    if (TAIL) {
      labels_store(n, args.sc, args.co, args.gfs, jw, lso, lco, lgo);
      if (fok && !(SA_NUM_PROBE & 32)) {
#if SA_NUM_PROBE & 64  // probe: the formula values into the f64 tile's last three columns
        if constexpr (!COND && !N32) {
          st16(fb + (args.Cf - 3) * Rf, fo);
          st16(fb + (args.Cf - 2) * Rf, fd);
          st16(fb + (args.Cf - 1) * Rf, fv);
        }
#else
        st16(args.off + jw, fo);
        st16(args.def + jw, fd);
        st16(args.val + jw, fv);
#endif
      }
    }
  }
  // COND: every lane stays (the ballots and the chunk stores need the whole wave); lanes past the
  // end recompute the last pair and their bits are masked off in cond_store
  if (!COND && jw >= n) return;
  NumCols C;
  C.at = P.i64_col[SA_XFN_ACTIONTYPE];
  C.re = P.i64_col[SA_XFN_RESULT];
  C.bi = P.i64_col[SA_XFN_BODYPART];
  C.ti = P.i64_col[SA_XFN_TIME];
  C.tf = P.f64_col[SA_XFN_TIME];
  C.sl = P.f64_col[SA_XFN_STARTLOCATION];
  C.el = P.f64_col[SA_XFN_ENDLOCATION];
  C.sp = P.f64_col[SA_XFN_STARTPOLAR];
  C.ep = P.f64_col[SA_XFN_ENDPOLAR];
  C.mv = P.f64_col[SA_XFN_MOVEMENT];
  C.td = P.f64_col[SA_XFN_TIME_DELTA];
  C.sd = P.f64_col[SA_XFN_SPACE_DELTA];
  C.lo = P.f64_col[SA_XFN_LOCATION];
  C.po = P.f64_col[SA_XFN_POLAR];
  C.mp = P.f64_col[SA_XFN_MOVEMENT_POLAR];
  C.di = P.f64_col[SA_XFN_DIRECTION];
  C.nf = (int)args.Cf;
  C.ni = (int)args.Ci;

  {
    double sx0[2], sy0[2], t0[2];
    if (KF == 3) {
      // Moving from window i-1 to i, action 1 takes action 0's previous row and action 0 takes
      // the next pool row, unless the action's window already reached its segment start
      // (d < i): then it keeps its row.  (If action 0 is clamped so is action 1, whose d is at
      // most d0 + 1.)
      if (!ATOMIC && args.xt_cells) {  // the raw (unflipped) rows jb, jb+1: xT cell codes
        uint32_t cc[2];
        const bool c16 = xt_c16(args.xt_l * args.xt_w);
#pragma unroll
        for (int e = 0; e < 2; ++e)
          cc[e] = c16 ? xt_cell_code16((cand[e].ids >> 8) & 0xFF, (cand[e].ids >> 16) & 0xFF, cand[e].c0,
                                       cand[e].c1, cand[e].c2, cand[e].c3, args.xt_l, args.xt_w)
                      : xt_cell_code((cand[e].ids >> 8) & 0xFF, (cand[e].ids >> 16) & 0xFF, cand[e].c0,
                                     cand[e].c1, cand[e].c2, cand[e].c3, args.xt_l, args.xt_w);
        if (c16) {
          uint16_t* c2 = reinterpret_cast<uint16_t*>(args.xt_cells);
          if (jb + 2 <= n)
            *reinterpret_cast<uint32_t*>(c2 + jb) = cc[0] | (cc[1] << 16);
          else
            c2[jb] = (uint16_t)cc[0];
        } else if (jb + 2 <= n) {
          *reinterpret_cast<uint2*>(args.xt_cells + jb) = make_uint2(cc[0], cc[1]);
        } else {
          args.xt_cells[jb] = cc[0];
        }
      }
      // COND: the family-major order too -- the condition tables are numbered by column, so
      // visiting the columns in block order moves through each 64-condition chunk once (a chunk
      // change flushes the held bitmaps: window-major order changed chunks ~12 times per wave)
      if constexpr (SA_NUM_FAMILY_MAJOR || (COND && SA_COND_FAMILY)) {
      // family by family, each family's windows back to back: the block columns are
      // family-major with the windows adjacent, so the wave writes its [C x 128] slab front to
      // back instead of jumping by the family width for every window.  Window i of action e
      // is row jb + e - min(i, d_e) of the four held rows jb-2 .. jb+1 (selected, not shifted).
      // the three windows' rows (the shift of the window-major loop below, unrolled): window 1
      // of action 0 is row jb-1 unless d0 < 1, of action 1 row jb unless d1 < 1; and so on
      Win w0, w1, w2;
      {
        const Row y0 = dd[0] >= 1 ? pool[0] : cand[0], y1 = dd[1] >= 1 ? cand[0] : cand[1];
        const Row z0 = dd[0] >= 2 ? pool[1] : y0, z1 = dd[1] >= 2 ? y0 : y1;
        row_to_win(cand[0], w0, 0);
        row_to_win(cand[1], w0, 1);
        row_to_win(y0, w1, 0);
        row_to_win(y1, w1, 1);
        row_to_win(z0, w2, 0);
        row_to_win(z1, w2, 1);
      }
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        if (!EXPLICIT && away[e]) {
          flip<ATOMIC>(w0, e);
          flip<ATOMIC>(w1, e);
          flip<ATOMIC>(w2, e);
        }
        sx0[e] = w0.c0[e];
        sy0[e] = w0.c1[e];
        t0[e] = w0.ts[e];
      }
      auto family = [&](int fam) __attribute__((always_inline)) {
        emit_window<ATOMIC, FT, IT>(C, 0, w0, sx0, sy0, t0, fb, ib, Rf, Ri, fam);
        if (K > 1) emit_window<ATOMIC, FT, IT>(C, 1, w1, sx0, sy0, t0, fb, ib, Rf, Ri, fam);
        if (K > 2) emit_window<ATOMIC, FT, IT>(C, 2, w2, sx0, sy0, t0, fb, ib, Rf, Ri, fam);
      };
      // the default plans' block order (catalog.py: xfns order)
      family(FAM_IDS);
      family(FAM_TIME);
      if (ATOMIC) {
        family(FAM_TD);
        family(FAM_LO);
        family(FAM_PO);
        family(FAM_MP);
        family(FAM_DI);
      } else {
        family(FAM_SL);
        family(FAM_EL);
        family(FAM_SP);
        family(FAM_EP);
        family(FAM_MV);
        family(FAM_TD);
        family(FAM_SD);
      }
      } else {
#pragma unroll 1
      for (int i = 0; i < K; ++i) {
        if (i > 0) {
          const Row prev0 = cand[0];
          if (dd[1] >= i) cand[1] = prev0;
          if (dd[0] >= i) cand[0] = pool[0];
          pool[0] = pool[1];
        }
        Win wf;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          row_to_win(cand[e], wf, e);
          if (!EXPLICIT && away[e]) flip<ATOMIC>(wf, e);
        }
        if (i == 0) {
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            sx0[e] = wf.c0[e];
            sy0[e] = wf.c1[e];
            t0[e] = wf.ts[e];
          }
        }
        emit_window<ATOMIC, FT, IT>(C, i, wf, sx0, sy0, t0, fb, ib, Rf, Ri);
      }
      }
    } else {
      for (int i = 0; i < K; ++i) {
        const sa_frame& Fi = EXPLICIT ? A.frames[i] : F0;
        Win w;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int64_t r = EXPLICIT ? jr[e] : jr[e] - (dd[e] < i ? dd[e] : i);
          load_row(Fi, r, ATOMIC, w, e);
          if (!ATOMIC && !EXPLICIT && i == 0 && args.xt_cells && jb + e < n)  // raw row jb+e
          {
            if (xt_c16(args.xt_l * args.xt_w))
              reinterpret_cast<uint16_t*>(args.xt_cells)[jb + e] = (uint16_t)xt_cell_code16(
                  w.typ[e], w.res[e], w.c0[e], w.c1[e], w.c2[e], w.c3[e], args.xt_l, args.xt_w);
            else
              args.xt_cells[jb + e] = xt_cell_code(w.typ[e], w.res[e], w.c0[e], w.c1[e], w.c2[e],
                                                   w.c3[e], args.xt_l, args.xt_w);
          }
          if (!EXPLICIT && away[e]) flip<ATOMIC>(w, e);
          if (i == 0) {
            sx0[e] = w.c0[e];
            sy0[e] = w.c1[e];
            t0[e] = w.ts[e];
          }
        }
        emit_window<ATOMIC, FT, IT>(C, i, w, sx0, sy0, t0, fb, ib, Rf, Ri);
      }
    }
  }
  if constexpr (COND) {
    if (acc.held) cond_flush(&sink_f);
  }
}

template <bool ATOMIC, bool EXPLICIT, int KF, bool TAIL = false, bool N32 = false, bool COND = false>
__global__ __launch_bounds__(64 * BLOCK_WAVES) __attribute__((amdgpu_waves_per_eu(num_min_waves<ATOMIC, TAIL>(), 8)))
void num_features_kernel(FeatArgs args) {
  const int wv = threadIdx.x / WAVE;
  const int64_t wave_base = args.row0 + (xcd_logical_block() * BLOCK_WAVES + wv) * WAVE_ACTS;
  num_features_body<ATOMIC, EXPLICIT, KF, TAIL, N32, COND>(args, wave_base, args.a.frames[0], args.ps, args.pc);
}

// sa_vaep_features_conditions' numeric pass with the condition tables (column starts,
// thresholds, NaN directions: 4 (Cf + Ci + 2) + 8 n_cond bytes) staged in LDS once per
// workgroup.  Read from global memory, each column's starts and each segment's thresholds cost
// a vmcnt(0) wait -- on gfx950 also a wait for every store the wave issued before (the bitmap
// flushes) -- in the middle of the pass; from LDS an lgkmcnt wait on a ds_read.
constexpr int COND_LDS_MAX = 32 * 1024;  // bytes of staged tables per workgroup (else global)
__host__ __device__ inline int64_t cond_lds_bytes(int64_t cf, int64_t ci, int64_t n_cond) {
  return 4 * (cf + ci + 2) + 8 * n_cond;
}
template <bool ATOMIC>
__global__ __launch_bounds__(64 * BLOCK_WAVES) __attribute__((amdgpu_waves_per_eu(num_min_waves<ATOMIC, false>(), 8)))
void num_cond_lds_kernel(FeatArgs args) {
  extern __shared__ __attribute__((aligned(16))) int32_t ctab[];
  const int nf = (int)args.Cf + 1, ni = (int)args.Ci + 1, nc = args.cond_n;
  int32_t* fs = ctab;
  int32_t* is = fs + nf;
  float* th = reinterpret_cast<float*>(is + ni);
  int32_t* dl = reinterpret_cast<int32_t*>(th + nc);
  for (int i = threadIdx.x; i < nf; i += 64 * BLOCK_WAVES) fs[i] = args.cond_fstart[i];
  for (int i = threadIdx.x; i < ni; i += 64 * BLOCK_WAVES) is[i] = args.cond_istart[i];
  for (int i = threadIdx.x; i < nc; i += 64 * BLOCK_WAVES) {
    th[i] = args.cond_thr[i];
    dl[i] = args.cond_dl[i];
  }
  __syncthreads();
  FeatArgs a = args;
  a.cond_fstart = fs;
  a.cond_istart = is;
  a.cond_thr = th;
  a.cond_dl = dl;
  const int wv = threadIdx.x / WAVE;
  const int64_t wave_base = args.row0 + (xcd_logical_block() * BLOCK_WAVES + wv) * WAVE_ACTS;
  num_features_body<ATOMIC, false, 3, false, false, true>(a, wave_base, a.a.frames[0], a.ps, a.pc);
}

// SA_FUSED_STEP = 1 (probe builds): the SPADL step's bool pass and numeric step pass as ONE
// launch, their workgroups interleaved in proportion (logical workgroup L is a bool one when
// floor((L + 1) nb / T) > floor(L nb / T)), so each CU mixes the pure-store bool tiles with the
// read-heavy numeric tiles of the same rows, whose inputs the two then share in L2.  The A/B of
// the headline's one bounded experiment (scripts/fused_step_ab.py).
#ifndef SA_COND_LDS
#define SA_COND_LDS 1  // 0: the COND pass reads its condition tables from global memory (A/B)
#endif
#ifndef SA_FUSED_STEP
#define SA_FUSED_STEP 0
#endif
#if SA_FUSED_STEP
static_assert(CG_WAVES == BLOCK_WAVES, "one workgroup shape for both passes");
__global__ __launch_bounds__(64 * BLOCK_WAVES) void step_fused_kernel(FeatArgs args, int ngroups, int gcols,
                                                                      int64_t nb, int64_t total) {
  const int64_t L = xcd_logical_block();
  if (L >= total) return;
  const int64_t bi = L * nb / total;
  if ((L + 1) * nb / total > bi) {
    bool_colgroup_body<false, false, false, false>(args, ngroups, gcols, bi);
  } else {
    const int wv = threadIdx.x / WAVE;
    const int64_t wave_base = args.row0 + ((L - bi) * BLOCK_WAVES + wv) * WAVE_ACTS;
    num_features_body<false, false, 3, true, false, false>(args, wave_base, args.a.frames[0], args.ps, args.pc);
  }
}
#endif

// SA_NUM_STAGE = T > 0 (probe builds): the SPADL step pass with each workgroup's streamed inputs
// -- coordinates, time and the two probabilities of T x 512 rows (56 B per row) plus the two rows
// before -- loaded into LDS in one burst before any of the T tiles' stores; the tiles then read
// those columns from LDS.  The experiment on the read / write turnaround of the numeric pass
// (profiles/r03_numeric_pass_ab.md): does separating a CU's reads from its stores in time help?
#ifndef SA_NUM_STAGE
#define SA_NUM_STAGE 0
#endif
#if SA_NUM_STAGE > 0
constexpr int STG_T = SA_NUM_STAGE;
constexpr int STG_ROWS = STG_T * BLOCK_ACTS + 2;
constexpr int STG_NP = (STG_ROWS / 2 + 255) / 256;  // row pairs per thread per column
__global__ __launch_bounds__(256) void num_staged_kernel(FeatArgs args) {
  extern __shared__ __attribute__((aligned(16))) double stg[];  // [7][STG_ROWS]
  const sa_frame& G = args.a.frames[0];
  const int64_t n = args.a.n;
  const int64_t row0 = xcd_logical_block() * (int64_t)(STG_T * BLOCK_ACTS);
  if (row0 >= n) return;
  const int64_t lo = row0 - 2;  // LDS row i = row lo + i
  const int64_t hi = min(n, row0 + (int64_t)STG_T * BLOCK_ACTS);
  const double* src[7] = {G.c0, G.c1, G.c2, G.c3, G.time_seconds, args.ps, args.pc};
  const int ncol = args.ps ? 7 : 5;
  for (int c = 0; c < ncol; ++c) {  // every load of the column before its LDS stores
    f64x2 v[STG_NP];
#pragma unroll
    for (int q = 0; q < STG_NP; ++q) {
      const int pr = q * 256 + threadIdx.x;
      const int64_t r = lo + 2 * (int64_t)pr;
      v[q] = f64x2{0.0, 0.0};
      if (pr < STG_ROWS / 2 && r >= 0) {
        if (r + 1 < hi) v[q] = ld_stream(reinterpret_cast<const f64x2*>(src[c] + r));
        else if (r < hi) v[q][0] = src[c][r];
      }
    }
#pragma unroll
    for (int q = 0; q < STG_NP; ++q) {
      const int pr = q * 256 + threadIdx.x;
      if (pr < STG_ROWS / 2) *reinterpret_cast<f64x2*>(stg + c * STG_ROWS + 2 * pr) = v[q];
    }
  }
  __syncthreads();
  sa_frame F = G;
  F.c0 = stg - lo;
  F.c1 = stg + STG_ROWS - lo;
  F.c2 = stg + 2 * STG_ROWS - lo;
  F.c3 = stg + 3 * STG_ROWS - lo;
  F.time_seconds = stg + 4 * STG_ROWS - lo;
  const double* ps = args.ps ? stg + 5 * STG_ROWS - lo : nullptr;
  const double* pc = args.ps ? stg + 6 * STG_ROWS - lo : nullptr;
  const int wv = threadIdx.x / WAVE;
#pragma unroll 1
  for (int t = 0; t < STG_T; ++t)
    num_features_body<false, false, 3, true>(args, row0 + (int64_t)t * BLOCK_ACTS + wv * WAVE_ACTS, F, ps, pc);
}
#endif

// ------------------------------------------------------------------------------ goalscore
// features.py:505-539 / atomic/vaep/features.py:229-260: per segment, teamA = team of the
// segment's first row, exclusive cumsum of goals for A and for B.  One wave per segment.

// 16-rows-per-lane form: passes of 1024 rows, so a ~1,600-row game is 2 passes instead of 13
// and each pass issues all of its loads at once (16 type + 16 result bytes, 64 B of team codes
// per lane; the next pass's loads go out before this pass is scanned).  A lane sums its 16
// (goals A, goals B) increments as one packed u64, the wave scans the 64 lane totals, and the
// lane then walks its rows with the exclusive count: 8 i64x2 stores per column per lane.
template <bool ATOMIC>
__global__ __launch_bounds__(256) void goalscore_wave16_kernel(sa_actions A,
                                                               int64_t* __restrict__ block,
                                                               int64_t C, int64_t col, int64_t R) {
  __shared__ __align__(16) int64_t gs_lds[4][WAVE * GS_LDS_PITCH];
  const int lane = threadIdx.x & (WAVE - 1);
  const int64_t g = (int64_t)blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE;
  if (g >= A.n_segments) return;
  const int64_t s = A.seg_off[g], e = A.seg_off[g + 1];
  if (s >= e) return;
  const int64_t n = A.n;
  const sa_frame& F = A.frames[0];
  const int32_t teamA = F.team[s];
  const int64_t base0 = s & ~(int64_t)127;  // 128-row aligned: whole 1-KiB column runs  // 16-row aligned: vector loads, whole 16-row runs
  uint64_t carry = 0;  // low 32 bits: goals of team A before this pass; high: team B
  Gs16In cur, nxt;
  gs16_load<ATOMIC>(F, base0 + 16 * lane, n, cur);
  for (int64_t base = base0; base < e; base += 16 * WAVE) {
    const int64_t j0 = base + 16 * lane;
    if (base + 16 * WAVE < e) gs16_load<ATOMIC>(F, j0 + 16 * WAVE, n, nxt);
    uint32_t gm = 0, om = 0, am = 0;  // goal / owngoal / team-A row bits (valid rows only)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t gb, ob;
      goal_bytes(cur.ty[q], cur.rs[q], ATOMIC, gb, ob);
      gm |= pack4(gb) << (4 * q);
      om |= pack4(ob) << (4 * q);
    }
#pragma unroll
    for (int m = 0; m < 16; ++m) am |= (uint32_t)(cur.tm[m] == teamA) << m;
    const int lo = s > j0 ? (int)(s - j0) : 0;                // first valid row of the lane
    const int hi = e < j0 + 16 ? (int)(e - j0) : 16;           // one past the last
    const uint32_t vm = lo >= hi ? 0u : (0xFFFFu >> (16 - (hi - lo))) << lo;
    const uint32_t gA = ((gm & am) | (om & ~am)) & vm, gB = ((gm & ~am) | (om & am)) & vm;
    const uint64_t x = (uint64_t)__popc(gA) | ((uint64_t)__popc(gB) << 32);
    uint64_t incl = x;
#pragma unroll
    for (int off = 1; off < WAVE; off <<= 1) {
      const uint64_t y = __shfl_up(incl, off, WAVE);
      if (lane >= off) incl += y;
    }
    const uint64_t ex = carry + incl - x;  // goals before row j0
    carry += __shfl(incl, WAVE - 1, WAVE);
    // the lane's 16 rows -> LDS one column at a time, then back out in pass-of-128 order
    // (lane l: rows 2l, 2l+1 of each 128-row run), so every store instruction writes 1 KiB
    // contiguous of one column (the lane's own 128-B run per instruction was 2.3x slower)
    const int64_t cA0 = (int64_t)(ex & 0xFFFFFFFFull), cB0 = (int64_t)(ex >> 32);
    int64_t* xl = gs_lds[threadIdx.x / WAVE];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      wave_sync();
#pragma unroll
      for (int m = 0; m < 16; m += 2) {
        int64_t v[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const uint32_t below = (1u << (m + q)) - 1u;  // rows of this lane before m+q
          const int64_t cA = cA0 + __popc(gA & below), cB = cB0 + __popc(gB & below);
          const bool isA = (am >> (m + q)) & 1;
          const int64_t tm = isA ? cA : cB, op = isA ? cB : cA;
          v[q] = k == 0 ? tm : (k == 1 ? op : tm - op);
        }
        *reinterpret_cast<i64x2*>(xl + lane * GS_LDS_PITCH + m) = i64x2{(long long)v[0], (long long)v[1]};
      }
      wave_sync();
#pragma unroll
      for (int p = 0; p < 8; ++p) {
        const int r = 128 * p + 2 * lane;  // row offset from `base`
        const int64_t jr = base + r;
        const i64x2 v = *reinterpret_cast<const i64x2*>(xl + (r / 16) * GS_LDS_PITCH + (r % 16));
        int64_t* o = block + tile_off(jr, col + k, C, R);
        if (jr >= s && jr + 1 < e) {
          st16(o, v);
        } else {
          if (jr >= s && jr < e) o[0] = v[0];
          if (jr + 1 >= s && jr + 1 < e) o[1] = v[1];
        }
      }
    }
    cur = nxt;
  }
}

// ------------------------------------------------------------------------------ labels
// vaep/labels.py:9-116, atomic/vaep/labels.py:9-107.  A lane owns 16 consecutive actions
// and holds rows j0 .. j0+31 as goal / owngoal bit masks plus team codes, so a look-ahead of
// nr_actions <= 17 needs no further loads.  The look-ahead clamps at the segment's last row,
// which only repeats a row already in the window, so the window is rows j+1 .. min(j+nr-1,
// last).
// Rows j0 .. j0+15 of one lane (j0 < n); `cur` = a segment cursor at or before row j0.
template <bool ATOMIC>
__device__ __forceinline__ void labels_rows(const sa_actions& A, int nr, uint8_t* __restrict__ sc,
                                            uint8_t* __restrict__ co, uint8_t* __restrict__ gfs,
                                            int64_t j0, SegCursor cur) {
  const int64_t n = A.n;
  const sa_frame& F = A.frames[0];
  uint32_t gm = 0, om = 0, shm = 0;  // goal / owngoal / shot(type 11) row bits
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint32_t tw = ld_u8x4(F.type_id, j0 / 4 + q, n);
    const uint32_t rw = ATOMIC ? 0u : ld_u8x4(F.result_id, j0 / 4 + q, n);
    uint32_t g, o;
    goal_bytes(tw, rw, ATOMIC, g, o);
    gm |= pack4(g) << (4 * q);
    om |= pack4(o) << (4 * q);
    if (ATOMIC) shm |= pack4(bytes_eq(tw, T_SHOT)) << (4 * q);
  }
  int32_t tm[32];
  if (j0 + 32 <= n) {
    const int4* tp = reinterpret_cast<const int4*>(F.team + j0);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int4 v = tp[q];
      tm[4 * q] = v.x;
      tm[4 * q + 1] = v.y;
      tm[4 * q + 2] = v.z;
      tm[4 * q + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int r = 0; r < 32; ++r) tm[r] = ld_or0(F.team, j0 + r, n);
  }
  const int32_t t0 = tm[0];
  int32_t t1 = t0;
  uint32_t e0 = 0;
#pragma unroll
  for (int r = 0; r < 32; ++r) {
    e0 |= (uint32_t)(tm[r] == t0) << r;
    if (t1 == t0 && tm[r] != t0) t1 = tm[r];
  }
  uint32_t e1 = 0;
#pragma unroll
  for (int r = 0; r < 32; ++r) e1 |= (uint32_t)(tm[r] == t1) << r;
  uint32_t s_out[4] = {0, 0, 0, 0}, c_out[4] = {0, 0, 0, 0}, g_out[4] = {0, 0, 0, 0};
#pragma unroll
  for (int m = 0; m < LANE_ACTS; ++m) {
    const int64_t j = j0 + m;
    if (j < n) {
      seg_advance(A, cur, j);
      const int64_t last = cur.e - 1;
      bool scores, concedes;
      const bool goal_j = (gm >> m) & 1, og_j = (om >> m) & 1;
      if (nr <= 17) {
        const int64_t hi = j + nr - 1 < last ? j + nr - 1 : last;
        const int span = (int)(hi - j);  // 0 .. 16
        const uint32_t win = span > 0 ? (((1u << span) - 1u) << (m + 1)) : 0u;
        // equality masks of the window's first two team codes cover every row whose team is
        // one of them (two teams per game); a third code takes the full compare
        uint32_t same;
        if (tm[m] == t0)
          same = e0;
        else if (tm[m] == t1)
          same = e1;
        else {
          same = 0;
#pragma unroll
          for (int r = 0; r < 32; ++r) same |= (uint32_t)(tm[r] == tm[m]) << r;
        }
        scores = goal_j || (((gm & same) | (om & ~same)) & win) != 0;
        concedes = og_j || (((gm & ~same) | (om & same)) & win) != 0;
      } else {
        scores = goal_j;
        concedes = og_j;
        const int32_t tj = tm[m];
        for (int i = 1; i < nr; ++i) {
          const int64_t c = j + i < last ? j + i : last;
          const int t = F.type_id[c];
          bool goal, og;
          if (ATOMIC) {
            goal = t == AT_GOAL;
            og = t == AT_OWNGOAL;
          } else {
            const bool shot = t == T_SHOT || t == T_SHOT_PENALTY || t == T_SHOT_FREEKICK;
            const int res = F.result_id[c];
            goal = shot && res == R_SUCCESS;
            og = shot && res == R_OWNGOAL;
          }
          const bool same = F.team[c] == tj;
          scores |= (goal && same) || (og && !same);
          concedes |= (goal && !same) || (og && same);
        }
      }
      bool gf;
      if (ATOMIC)  // shot followed by goal; the segment's last row compares NaN -> False
        gf = ((shm >> m) & 1) && j < last && ((gm >> (m + 1)) & 1);
      else
        gf = goal_j;
      s_out[m >> 2] |= (uint32_t)scores << (8 * (m & 3));
      c_out[m >> 2] |= (uint32_t)concedes << (8 * (m & 3));
      g_out[m >> 2] |= (uint32_t)gf << (8 * (m & 3));
    }
  }
  if (sc) st16(sc + j0, u32x4{s_out[0], s_out[1], s_out[2], s_out[3]});
  if (co) st16(co + j0, u32x4{c_out[0], c_out[1], c_out[2], c_out[3]});
  if (gfs) st16(gfs + j0, u32x4{g_out[0], g_out[1], g_out[2], g_out[3]});
}

template <bool ATOMIC>
__global__ __launch_bounds__(256) void labels_kernel(sa_actions A, int nr, uint8_t* __restrict__ sc,
                                                     uint8_t* __restrict__ co,
                                                     uint8_t* __restrict__ gfs) {
  const int64_t j0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * LANE_ACTS;
  if (j0 >= A.n) return;
  labels_rows<ATOMIC>(A, nr, sc, co, gfs, j0, wave_cursor(A, j0));  // first active lane's row
}

// ------------------------------------------------------------------------------ formula
// vaep/formula.py:8-151, atomic/vaep/formula.py:8-141.  Arithmetic stays in the probability
// dtype and mirrors the pandas expression tree operation by operation.  A lane owns V
// consecutive actions (16-B stores); the previous row's values come from the same lane or,
// for the lane's first action, from the neighbouring lane by a wave shuffle.
// Rows j0 .. j0+V-1 of one lane (V = 16 / sizeof(T)); every lane of the wave calls it with
// consecutive j0 (the previous row comes from the neighbouring lane); `cur` = a segment cursor
// at or before row j0, advanced by the call.
// t_in (optional, vector path): the rows' time_seconds the caller already holds (the numeric
// step pass loaded them with its window rows), so they are not read a second time
template <bool ATOMIC, typename T, typename VT>
__device__ __forceinline__ bool formula_vals(const sa_actions& A, const T* __restrict__ ps,
                                             const T* __restrict__ pc, bool vec_ok, int64_t j0, SegCursor& cur,
                                             VT& vo, VT& vd, VT& vv, const double* t_in) {
  constexpr int V = 16 / sizeof(T);
  const int64_t n = A.n;
  const int lane = threadIdx.x & (WAVE - 1);
  const bool active = j0 < n;
  const sa_frame& F = A.frames[0];
  T s_[V], c_[V];
  double t_[V];
  int32_t tm_[V], ty_[V], rs_[V];
  typedef T vec_t __attribute__((ext_vector_type(V)));
  if (vec_ok && active && j0 + V <= n) {  // whole 16-B vectors (vec_ok: 16-B aligned probabilities)
    const vec_t vs = ld_stream<2>(reinterpret_cast<const vec_t*>(ps + j0));
    const vec_t vc = ld_stream<2>(reinterpret_cast<const vec_t*>(pc + j0));
#pragma unroll
    for (int q = 0; q < V; q += 2) {
      if (t_in) {
        t_[q] = t_in[q];
        t_[q + 1] = t_in[q + 1];
      } else {
        const f64x2 tv = *reinterpret_cast<const f64x2*>(F.time_seconds + j0 + q);
        t_[q] = tv[0];
        t_[q + 1] = tv[1];
      }
    }
    uint32_t tyw, rsw = 0;
    if (V == 4) {
      const int4 tv = *reinterpret_cast<const int4*>(F.team + j0);
      tm_[0] = tv.x;
      tm_[1 % V] = tv.y;
      tm_[2 % V] = tv.z;
      tm_[3 % V] = tv.w;
      tyw = *reinterpret_cast<const uint32_t*>(F.type_id + j0);
      if (!ATOMIC) rsw = *reinterpret_cast<const uint32_t*>(F.result_id + j0);
    } else {
      const int2 tv = *reinterpret_cast<const int2*>(F.team + j0);
      tm_[0] = tv.x;
      tm_[1 % V] = tv.y;
      tyw = *reinterpret_cast<const uint16_t*>(F.type_id + j0);
      if (!ATOMIC) rsw = *reinterpret_cast<const uint16_t*>(F.result_id + j0);
    }
#pragma unroll
    for (int q = 0; q < V; ++q) {
      s_[q] = vs[q];
      c_[q] = vc[q];
      ty_[q] = (int32_t)byte_of(tyw, q);
      rs_[q] = (int32_t)byte_of(rsw, q);
    }
  } else {
#pragma unroll
    for (int q = 0; q < V; ++q) {  // own rows j0 .. j0+V-1 (clamped to n-1 in the tail)
      const int64_t j = active ? (j0 + q < n ? j0 + q : n - 1) : 0;
      s_[q] = ps[j];
      c_[q] = pc[j];
      t_[q] = F.time_seconds[j];
      tm_[q] = F.team[j];
      ty_[q] = F.type_id[j];
      rs_[q] = ATOMIC ? 0 : F.result_id[j];
    }
  }
  // row j0-1 comes from the previous lane (lane 0 loads it itself)
  T sp = __shfl_up(s_[V - 1], 1, WAVE), cp = __shfl_up(c_[V - 1], 1, WAVE);
  double tp = __shfl_up(t_[V - 1], 1, WAVE);
  int32_t tmp = __shfl_up(tm_[V - 1], 1, WAVE), typ = __shfl_up(ty_[V - 1], 1, WAVE),
          rsp = __shfl_up(rs_[V - 1], 1, WAVE);
  if (!active) return false;
  if (lane == 0 && j0 > 0) {
    const int64_t p = j0 - 1;
    sp = ps[p];
    cp = pc[p];
    tp = F.time_seconds[p];
    tmp = F.team[p];
    typ = F.type_id[p];
    rsp = ATOMIC ? 0 : F.result_id[p];
  }
#pragma unroll
  for (int q = 0; q < V; ++q) {
    const int64_t j = j0 + q < n ? j0 + q : n - 1;
    seg_advance(A, cur, j);
    const bool first = j == cur.s;  // _prev of a segment's first row is the row itself
    T Sp = q ? s_[q - 1] : sp, Cp = q ? c_[q - 1] : cp;
    double Tp = q ? t_[q - 1] : tp;
    int32_t TMp = q ? tm_[q - 1] : tmp, TYp = q ? ty_[q - 1] : typ, RSp = q ? rs_[q - 1] : rsp;
    if (first) {
      Sp = s_[q];
      Cp = c_[q];
      Tp = t_[q];
      TMp = tm_[q];
      TYp = ty_[q];
      RSp = rs_[q];
    }
    const T one = T(1), zero = T(0);
    const bool same = TMp == tm_[q];
    const T fs = same ? one : zero, fn = same ? zero : one;
    T prev_s = Sp * fs + Cp * fn;  // _prev(scores) * sameteam + _prev(concedes) * ~sameteam
    T prev_c = Cp * fs + Sp * fn;
    bool prevgoal;
    if (ATOMIC) {
      prevgoal = TYp == AT_GOAL || TYp == AT_OWNGOAL;
    } else {
      if (fabs(t_[q] - Tp) > 10.0) {  // _samephase_nb
        prev_s = zero;
        prev_c = zero;
      }
      prevgoal = (TYp == T_SHOT || TYp == T_SHOT_PENALTY || TYp == T_SHOT_FREEKICK) &&
                 RSp == R_SUCCESS;
    }
    if (prevgoal) {
      prev_s = zero;
      prev_c = zero;
    }
    if (!ATOMIC) {
      if (ty_[q] == T_SHOT_PENALTY) prev_s = T(0.792453);
      if (ty_[q] == T_CORNER_CROSSED || ty_[q] == T_CORNER_SHORT) prev_s = T(0.046500);
    }
    const T o = s_[q] - prev_s;
    const T d = -(c_[q] - prev_c);
    vo[q] = o;
    vd[q] = d;
    vv[q] = o + d;
  }
  return true;
}

// formula_vals of rows j0 .. j0+V-1, stored (one 16-B store per output column)
template <bool ATOMIC, typename T>
__device__ __forceinline__ void formula_rows(const sa_actions& A, const T* __restrict__ ps,
                                             const T* __restrict__ pc, T* __restrict__ off,
                                             T* __restrict__ def, T* __restrict__ val, bool vec_ok,
                                             int64_t j0, SegCursor& cur) {
  constexpr int V = 16 / sizeof(T);
  typedef T vec_t __attribute__((ext_vector_type(V)));
  vec_t vo, vd, vv;
  if (!formula_vals<ATOMIC, T>(A, ps, pc, vec_ok, j0, cur, vo, vd, vv)) return;
  st16(off + j0, vo);
  st16(def + j0, vd);
  st16(val + j0, vv);
}

template <bool ATOMIC, typename T>
__global__ __launch_bounds__(256) void formula_kernel(sa_actions A, const T* __restrict__ ps,
                                                      const T* __restrict__ pc, T* __restrict__ off,
                                                      T* __restrict__ def, T* __restrict__ val,
                                                      bool vec_ok) {
  constexpr int V = 16 / sizeof(T);
  const int64_t j0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * V;
  const int64_t jw = ((int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~(WAVE - 1))) * V;
  if (jw >= A.n) return;  // whole wave past the end (the shuffles need every lane of a live wave)
  SegCursor cur = wave_cursor(A, jw);
  formula_rows<ATOMIC, T>(A, ps, pc, off, def, val, vec_ok, j0, cur);
}

// Labels and formula of the same 1024 rows in one wave (the step's tail: one launch, the ids
// and team codes read once): the labels part as labels_kernel (a lane owns 16 rows), then the
// formula part in passes of 64 * V rows as formula_kernel (a lane owns V rows), both lanes'
// segment cursors advancing from one wave-uniform search.
template <bool ATOMIC, typename T>
__global__ __launch_bounds__(256) void labels_formula_kernel(sa_actions A, int nr, uint8_t* __restrict__ sc,
                                                             uint8_t* __restrict__ co,
                                                             uint8_t* __restrict__ gfs,
                                                             const T* __restrict__ ps,
                                                             const T* __restrict__ pc, T* __restrict__ off,
                                                             T* __restrict__ def, T* __restrict__ val,
                                                             bool vec_ok) {
  constexpr int V = 16 / sizeof(T);
  const int lane = threadIdx.x & (WAVE - 1);
  const int64_t jw = ((int64_t)blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE) * (WAVE * LANE_ACTS);
  if (jw >= A.n) return;
  const SegCursor wc = wave_cursor(A, jw);
  const int64_t jl = jw + (int64_t)lane * LANE_ACTS;
  if (jl < A.n) labels_rows<ATOMIC>(A, nr, sc, co, gfs, jl, wc);
  SegCursor fc = wc;
#pragma unroll 1
  for (int p = 0; p < LANE_ACTS / V; ++p) {
    const int64_t base = jw + (int64_t)p * WAVE * V;
    if (base >= A.n) break;  // uniform
    formula_rows<ATOMIC, T>(A, ps, pc, off, def, val, vec_ok, base + (int64_t)lane * V, fc);
  }
}

}  // namespace sa

// ================================== C ABI =================================================
using namespace sa;

static int check_actions(const sa_actions* a, bool allow_explicit) {
  if (!a) return fail(SA_EINVAL, "null sa_actions");
  if (a->n < 0) return fail(SA_EINVAL, "n < 0");
  if (a->n_frames < 1 || a->n_frames > SA_MAX_FRAMES)
    return fail(SA_EINVAL, "n_frames must be in [1, %d]", SA_MAX_FRAMES);
  if (!allow_explicit && a->n_frames != 1) return fail(SA_EINVAL, "explicit frames not allowed here");
  if (a->n_frames > 1 && a->n_segments != 1)
    return fail(SA_EINVAL, "explicit-frame mode requires exactly one segment");
  if (a->n > 0 && (a->n_segments < 1 || !a->seg_off))
    return fail(SA_EINVAL, "n_segments must be >= 1 with seg_off");
  for (int f = 0; f < a->n_frames; ++f) {
    const sa_frame& F = a->frames[f];
    if (!F.type_id || !F.team || !F.bodypart_id || !F.period_id || !F.time_seconds || !F.c0 ||
        !F.c1 || !F.c2 || !F.c3 || (!a->atomic && !F.result_id))
      return fail(SA_EINVAL, "frame %d has a null column", f);
    if (!aligned16(F.type_id) || !aligned16(F.result_id) || !aligned16(F.bodypart_id) ||
        !aligned16(F.team))
      return fail(SA_EINVAL, "frame %d: id and team columns must be 16-byte aligned", f);
    if (!aligned16(F.c0) || !aligned16(F.c1) || !aligned16(F.c2) || !aligned16(F.c3) ||
        !aligned16(F.time_seconds))
      return fail(SA_EINVAL, "frame %d: coordinate and time columns must be 16-byte aligned", f);
  }
  return SA_OK;
}

static int check_block(const sa_block* b, int64_t n, int64_t quantum, const char* what) {
  const int64_t n16 = ((n + 15) / 16) * 16;
  if (!b || !b->data) return fail(SA_EINVAL, "%s block is null", what);
  if (!aligned16(b->data)) return fail(SA_EINVAL, "%s block must be 16-byte aligned", what);
  if (b->n_cols < 0) return fail(SA_EINVAL, "%s block has a negative column count", what);
  const int64_t R = b->tile_rows;
  if (R <= 0 || R % 16 != 0 || (R < n16 && R % quantum != 0))
    return fail(SA_EINVAL,
                "%s block: tile_rows must be a multiple of 16 and either >= round_up(n, 16) or a "
                "multiple of %lld", what, (long long)quantum);
  return SA_OK;
}

struct TailArgs {  // labels + f64 formula riding in the numeric pass (sa_vaep_step_f64)
  int32_t nr;
  uint8_t *sc, *co, *gfs;
  const double *ps, *pc;
  double *off, *def, *val;
  int64_t chunk;     // > 0: the numeric pass in launches of `chunk` rows (sa_vaep_step_f64_chunked)
  int32_t prefetch;  // each chunk's inputs read into the Infinity Cache first
};

// sa_vaep_step_f64_chunked's probe of the numeric pass's read / write turnaround: rows [r0, r1)'s
// inputs (coordinates, time, ids, team codes, probabilities: 64 B per row) read once with the
// default cache policy, so the Infinity Cache holds them when the pass over the chunk runs --
// the chunk's HBM reads happen in one pure-read burst instead of inside the pass's write stream.
// 4 rows per thread; the values only feed a compare that never stores.
__global__ __launch_bounds__(256) void prefetch_rows_kernel(sa_actions A, const double* __restrict__ ps,
                                                            const double* __restrict__ pc, int64_t r0, int64_t r1,
                                                            uint32_t* __restrict__ sink) {
  const int64_t j = r0 + 4 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (j + 4 > r1) return;  // r0, r1 multiples of 4 (or r1 = n: the tail rows stay out)
  const sa_frame& F = A.frames[0];
  uint64_t h = 0;
  auto f2 = [&](const double* c) {
    if (!c) return;
    const f64x2 a = *reinterpret_cast<const f64x2*>(c + j), b = *reinterpret_cast<const f64x2*>(c + j + 2);
    h ^= (uint64_t)__double_as_longlong(a[0] + a[1] + b[0] + b[1]);
  };
  f2(F.c0);
  f2(F.c1);
  f2(F.c2);
  f2(F.c3);
  f2(F.time_seconds);
  f2(ps);
  f2(pc);
  h ^= *reinterpret_cast<const uint32_t*>(F.type_id + j) ^ *reinterpret_cast<const uint32_t*>(F.result_id + j) ^
       *reinterpret_cast<const uint32_t*>(F.bodypart_id + j) ^ *reinterpret_cast<const uint32_t*>(F.period_id + j);
  const i32x4 tm = *reinterpret_cast<const i32x4*>(F.team + j);
  h ^= (uint32_t)(tm[0] ^ tm[1] ^ tm[2] ^ tm[3]);
  if (h == 0x5A5A5A5A5A5A5A5Aull) sink[0] = (uint32_t)h;  // never in practice: keeps the loads
}

static int launch_features(const sa_actions* a, const sa_feature_plan* plan, const sa_block* bool_out,
                           const sa_block* f64_out, const sa_block* i64_out, int32_t xt_l,
                           int32_t xt_w, uint32_t* xt_cells, void* stream, uint8_t* bits = nullptr,
                           int64_t bits_stride = 0, int32_t n_bits = 0, const TailArgs* tail = nullptr,
                           bool num32 = false, const FeatArgs* cond = nullptr);

extern "C" int sa_vaep_features(const sa_actions* a, const sa_feature_plan* plan,
                                const sa_block* bool_out, const sa_block* f64_out,
                                const sa_block* i64_out, void* stream) {
  return launch_features(a, plan, bool_out, f64_out, i64_out, 0, 0, nullptr, stream);
}

extern "C" int sa_vaep_features_xt(const sa_actions* a, const sa_feature_plan* plan,
                                   const sa_block* bool_out, const sa_block* f64_out,
                                   const sa_block* i64_out, int32_t xt_l, int32_t xt_w,
                                   uint32_t* xt_cells, void* stream) {
  if (!a) return fail(SA_EINVAL, "null sa_actions");
  if (a->atomic || a->n_frames != 1) return fail(SA_EINVAL, "xT cells need SPADL actions in windowed mode");
  if (xt_l < 1 || xt_w < 1 || (int64_t)xt_l * xt_w > SA_XT_CELLS_MAX_C)
    return fail(SA_EINVAL, "xT cell codes need 1 <= l * w <= %d", SA_XT_CELLS_MAX_C);
  if (!xt_cells || !aligned16(xt_cells)) return fail(SA_EINVAL, "xt_cells must be 16-byte aligned");
  return launch_features(a, plan, bool_out, f64_out, i64_out, xt_l, xt_w, xt_cells, stream);
}

extern "C" int sa_vaep_features_bits(const sa_actions* a, const sa_feature_plan* plan, uint8_t* bool_bits,
                                     int64_t bits_stride, int32_t n_bool_cols, const sa_block* f64_out,
                                     const sa_block* i64_out, void* stream) {
  if (!a) return fail(SA_EINVAL, "null sa_actions");
  if (!bool_bits || n_bool_cols < 1 || bits_stride < 2 * ((a->n + 15) / 16) || bits_stride % 2 ||
      ((uintptr_t)bool_bits & 1u))
    return fail(SA_EINVAL, "bool bitmaps: even stride of at least ceil(n/16)*2 bytes, 2-byte aligned");
  if (a->n_frames != 1) return fail(SA_EINVAL, "bool bitmaps: windowed mode only");
  return launch_features(a, plan, nullptr, f64_out, i64_out, 0, 0, nullptr, stream, bool_bits, bits_stride,
                         n_bool_cols);
}

extern "C" int sa_vaep_features_bits_f32(const sa_actions* a, const sa_feature_plan* plan, uint8_t* bool_bits,
                                         int64_t bits_stride, int32_t n_bool_cols, const sa_block* f32_out,
                                         const sa_block* i32f_out, void* stream) {
  if (!a) return fail(SA_EINVAL, "null sa_actions");
  if (!bool_bits || n_bool_cols < 1 || bits_stride < 2 * ((a->n + 15) / 16) || bits_stride % 2 ||
      ((uintptr_t)bool_bits & 1u))
    return fail(SA_EINVAL, "bool bitmaps: even stride of at least ceil(n/16)*2 bytes, 2-byte aligned");
  if (a->n_frames != 1) return fail(SA_EINVAL, "bool bitmaps: windowed mode only");
  if (!plan || plan->nb_prev_actions > 3)
    return fail(SA_EINVAL, "float32 numeric blocks: nb_prev_actions <= 3 (use sa_vaep_features_bits)");
  return launch_features(a, plan, nullptr, f32_out, i32f_out, 0, 0, nullptr, stream, bool_bits, bits_stride,
                         n_bool_cols, nullptr, true);
}

extern "C" int sa_vaep_features_conditions(const sa_actions* a, const sa_feature_plan* plan, uint8_t* bits,
                                           int64_t bits_stride, int32_t n_bool_cols, int32_t n_f64_cols,
                                           int32_t n_i64_cols, const int32_t* cond_fstart,
                                           const int32_t* cond_istart, const float* cond_thr,
                                           const int32_t* cond_dl, int32_t n_cond, void* stream) {
  if (!a) return fail(SA_EINVAL, "null sa_actions");
  if (a->n_frames != 1) return fail(SA_EINVAL, "condition bitmaps: windowed mode only");
  if (!plan || plan->nb_prev_actions > 3) return fail(SA_EINVAL, "condition bitmaps: nb_prev_actions <= 3");
  if (!bits || n_bool_cols < 0 || n_cond < 0 || n_f64_cols < 0 || n_i64_cols < 0 || bits_stride % 16 ||
      bits_stride < 16 * ((a->n + 127) / 128) || !aligned16(bits))
    return fail(SA_EINVAL, "condition bitmaps: 16-byte aligned rows of at least ceil(n/128)*16 bytes");
  if (!cond_fstart || !cond_istart || (n_cond > 0 && (!cond_thr || !cond_dl)))
    return fail(SA_EINVAL, "null condition table");
  if (n_f64_cols >= WAVE || n_i64_cols >= WAVE)  // the starts are held one per lane
    return fail(SA_EINVAL, "condition bitmaps: at most %d f64 and %d i64 columns", WAVE - 1, WAVE - 1);
  // stand-in descriptors: the numeric pass writes no block in this mode, only the bitmaps
  const sa_block fz{bits, n_f64_cols, 0, 128}, iz{bits, n_i64_cols, 0, 128};
  FeatArgs c{};
  c.cond_fstart = cond_fstart;
  c.cond_istart = cond_istart;
  c.cond_thr = cond_thr;
  c.cond_dl = cond_dl;
  c.cond_row0 = n_bool_cols;
  c.cond_n = n_cond;
  return launch_features(a, plan, nullptr, &fz, &iz, 0, 0, nullptr, stream, bits, bits_stride, n_bool_cols, nullptr,
                         false, &c);
}

extern "C" int sa_vaep_step_f64(const sa_actions* a, const sa_feature_plan* plan, const sa_block* bool_out,
                                const sa_block* f64_out, const sa_block* i64_out, int32_t xt_l, int32_t xt_w,
                                uint32_t* xt_cells, int32_t nr_actions, uint8_t* scores, uint8_t* concedes,
                                uint8_t* goal_from_shot, int64_t ld, const double* p_scores,
                                const double* p_concedes, double* off, double* def, double* val,
                                void* stream) {
  int rc = check_actions(a, false);
  if (rc) return rc;
  if (!plan) return fail(SA_EINVAL, "null plan");
  if (nr_actions < 1) return fail(SA_EINVAL, "nr_actions must be >= 1");
  if (ld % 16 != 0 || ld < ((a->n + 15) / 16) * 16)
    return fail(SA_EINVAL, "ld must be a multiple of 16 and >= round_up(n, 16)");
  if (!aligned16(scores) || !aligned16(concedes) || !aligned16(goal_from_shot))
    return fail(SA_EINVAL, "label outputs must be 16-byte aligned");
  const bool formula = p_scores || p_concedes || off || def || val;  // all NULL: labels only
  if (formula && (!p_scores || !p_concedes || !off || !def || !val))
    return fail(SA_EINVAL, "null probability/output pointer");
  if (!aligned16(off) || !aligned16(def) || !aligned16(val))
    return fail(SA_EINVAL, "formula outputs must be 16-byte aligned (length >= round_up(n, 16))");
  if (xt_cells) {
    if (a->atomic) return fail(SA_EINVAL, "xT cells need SPADL actions");
    if (xt_l < 1 || xt_w < 1 || (int64_t)xt_l * xt_w > SA_XT_CELLS_MAX_C)
      return fail(SA_EINVAL, "xT cell codes need 1 <= l * w <= %d", SA_XT_CELLS_MAX_C);
    if (!aligned16(xt_cells)) return fail(SA_EINVAL, "xt_cells must be 16-byte aligned");
  }
  // no fused form: the separate launches.  Atomic actions always take them: their numeric pass
  // (136 VGPRs, 3 waves per SIMD) loses more to the tail's registers than the tail's launch
  // costs (cfg3, 4.0e7 atomic actions: 3.89 ms separate vs 4.35 ms fused, scripts/atomic_ab.py,
  // profiles/r03_atomic_ab.json)
  if (a->atomic || plan->nb_prev_actions > 3 || nr_actions > SA_STEP_MAX_NR) {
    if ((rc = launch_features(a, plan, bool_out, f64_out, i64_out, xt_l, xt_w, xt_cells, stream))) return rc;
    if (!formula) return sa_vaep_labels(a, nr_actions, scores, concedes, goal_from_shot, ld, stream);
    return sa_vaep_labels_formula_f64(a, nr_actions, scores, concedes, goal_from_shot, ld, p_scores,
                                      p_concedes, off, def, val, stream);
  }
  const TailArgs t{nr_actions, scores, concedes, goal_from_shot, p_scores, p_concedes, off, def, val, 0, 0};
  return launch_features(a, plan, bool_out, f64_out, i64_out, xt_l, xt_w, xt_cells, stream, nullptr, 0, 0, &t);
}

extern "C" int sa_vaep_step_f64_chunked(const sa_actions* a, const sa_feature_plan* plan, const sa_block* bool_out,
                                        const sa_block* f64_out, const sa_block* i64_out, int32_t xt_l, int32_t xt_w,
                                        uint32_t* xt_cells, int32_t nr_actions, uint8_t* scores, uint8_t* concedes,
                                        uint8_t* goal_from_shot, int64_t ld, const double* p_scores,
                                        const double* p_concedes, double* off, double* def, double* val,
                                        int64_t chunk_rows, int32_t prefetch, void* stream) {
  if (chunk_rows < 0 || chunk_rows % BLOCK_ACTS != 0)
    return fail(SA_EINVAL, "chunk_rows must be a non-negative multiple of %d", BLOCK_ACTS);
  if (!a || a->atomic || !plan || plan->nb_prev_actions > 3 || nr_actions < 1 || nr_actions > SA_STEP_MAX_NR ||
      !p_scores || !p_concedes)
    return fail(SA_EINVAL, "the chunked step takes the fused SPADL step form with probabilities");
  if (bool_out && bool_out->n_cols > 0) {
    for (int x = 0; x < SA_XFN_COUNT; ++x)
      if (plan->bool_col[x] >= 0) return fail(SA_EINVAL, "the chunked step is the numeric pass only");
  }
  if (chunk_rows == 0)
    return sa_vaep_step_f64(a, plan, bool_out, f64_out, i64_out, xt_l, xt_w, xt_cells, nr_actions, scores, concedes,
                            goal_from_shot, ld, p_scores, p_concedes, off, def, val, stream);
  int rc = check_actions(a, false);
  if (rc) return rc;
  if (ld % 16 != 0 || ld < ((a->n + 15) / 16) * 16)
    return fail(SA_EINVAL, "ld must be a multiple of 16 and >= round_up(n, 16)");
  if (!aligned16(scores) || !aligned16(concedes) || !aligned16(goal_from_shot) || !off || !def || !val ||
      !aligned16(off) || !aligned16(def) || !aligned16(val))
    return fail(SA_EINVAL, "label / formula outputs: non-null, 16-byte aligned");
  if (xt_cells && (xt_l < 1 || xt_w < 1 || (int64_t)xt_l * xt_w > SA_XT_CELLS_MAX_C || !aligned16(xt_cells)))
    return fail(SA_EINVAL, "bad xT cell code arguments");
  const TailArgs t{nr_actions, scores, concedes, goal_from_shot, p_scores, p_concedes, off, def, val, chunk_rows,
                   prefetch};
  return launch_features(a, plan, bool_out, f64_out, i64_out, xt_l, xt_w, xt_cells, stream, nullptr, 0, 0, &t);
}

static int launch_features(const sa_actions* a, const sa_feature_plan* plan, const sa_block* bool_out,
                           const sa_block* f64_out, const sa_block* i64_out, int32_t xt_l,
                           int32_t xt_w, uint32_t* xt_cells, void* stream, uint8_t* bits,
                           int64_t bits_stride, int32_t n_bits, const TailArgs* tail, bool num32,
                           const FeatArgs* cond) {
  int rc = check_actions(a, true);
  if (rc) return rc;
  if (!plan) return fail(SA_EINVAL, "null plan");
  const int K = plan->nb_prev_actions;
  if (K < 1) return fail(SA_EINVAL, "nb_prev_actions must be >= 1");
  if (a->n_frames > 1 && a->n_frames != K)
    return fail(SA_EINVAL, "explicit mode needs n_frames == nb_prev_actions");
  bool wb = false, wf = false, wi = false, wn = false;
  for (int x = 0; x < SA_XFN_COUNT; ++x) {
    wb |= plan->bool_col[x] >= 0;
    wf |= plan->f64_col[x] >= 0;
    wi |= plan->i64_col[x] >= 0;
    wn |= plan->f64_col[x] >= 0 || (plan->i64_col[x] >= 0 && x != SA_XFN_GOALSCORE);
  }
  if (wb && !bits && (rc = check_block(bool_out, a->n, SA_BOOL_TILE_QUANTUM, "bool"))) return rc;
  if (wf && (rc = check_block(f64_out, a->n, SA_NUM_TILE_QUANTUM, "f64"))) return rc;
  if (wi && (rc = check_block(i64_out, a->n, SA_NUM_TILE_QUANTUM, "i64"))) return rc;
  for (int x = 0; x < SA_XFN_COUNT; ++x) {
    if ((wb && plan->bool_col[x] >= (bits ? n_bits : bool_out->n_cols)) || (wf && plan->f64_col[x] >= f64_out->n_cols) ||
        (wi && plan->i64_col[x] >= i64_out->n_cols))
      return fail(SA_EINVAL, "plan column offset beyond the block's column count");
  }
  if (a->atomic) {
    const int spadl_only[] = {SA_XFN_RESULT, SA_XFN_RESULT_ONEHOT, SA_XFN_ACTIONTYPE_RESULT_ONEHOT,
                              SA_XFN_STARTLOCATION, SA_XFN_ENDLOCATION, SA_XFN_STARTPOLAR,
                              SA_XFN_ENDPOLAR, SA_XFN_MOVEMENT, SA_XFN_SPACE_DELTA};
    for (int x : spadl_only)
      if (plan->bool_col[x] >= 0 || plan->f64_col[x] >= 0 || plan->i64_col[x] >= 0)
        return fail(SA_EINVAL, "transformer %d is not defined for atomic actions", x);
  } else {
    const int atomic_only[] = {SA_XFN_LOCATION, SA_XFN_POLAR, SA_XFN_MOVEMENT_POLAR, SA_XFN_DIRECTION};
    for (int x : atomic_only)
      if (plan->bool_col[x] >= 0 || plan->f64_col[x] >= 0 || plan->i64_col[x] >= 0)
        return fail(SA_EINVAL, "transformer %d is only defined for atomic actions", x);
  }
  if (a->n == 0) return SA_OK;
  hipStream_t st = (hipStream_t)stream;
  FeatArgs args{*a,
                *plan,
                wb && !bits ? (uint8_t*)bool_out->data : nullptr,
                wf ? (double*)f64_out->data : nullptr,
                wi ? (int64_t*)i64_out->data : nullptr,
                wb ? (bits ? (int64_t)n_bits : bool_out->n_cols) : 0,
                wf ? f64_out->n_cols : 0,
                wi ? i64_out->n_cols : 0,
                wb && !bits ? bool_out->tile_rows : BOOL_TILE,
                wf ? f64_out->tile_rows : 16,
                wi ? i64_out->tile_rows : 16,
                xt_cells,
                xt_l,
                xt_w,
                (wb || cond) ? (uint16_t*)bits : nullptr,  // COND: the condition rows even with no bool column
                bits_stride / 2,
                tail ? tail->nr : 0,
                tail ? tail->sc : nullptr,
                tail ? tail->co : nullptr,
                tail ? tail->gfs : nullptr,
                tail ? tail->ps : nullptr,
                tail ? tail->pc : nullptr,
                tail ? tail->off : nullptr,
                tail ? tail->def : nullptr,
                tail ? tail->val : nullptr,
                tail ? (aligned16(tail->ps) && aligned16(tail->pc)) : false,
                cond ? cond->cond_fstart : nullptr,
                cond ? cond->cond_istart : nullptr,
                cond ? cond->cond_thr : nullptr,
                cond ? cond->cond_dl : nullptr,
                cond ? cond->cond_row0 : 0};
  args.cond_n = cond ? cond->cond_n : 0;
  const dim3 grid(xcd_grid((a->n + BLOCK_ACTS - 1) / BLOCK_ACTS)), block(BLOCK_WAVES * WAVE);
  const bool expl = a->n_frames > 1;
  if (wb) {  // one wave per (tile, group of ~32 columns), XCD-contiguous sweep order
    const int ng = (int)((args.Cb + SA_CG_COLS - 1) / SA_CG_COLS);
    const int gc = (int)((args.Cb + ng - 1) / ng);
    const int64_t waves = (a->n + BOOL_TILE - 1) / BOOL_TILE * ng;
    const dim3 cgrid(xcd_grid((waves + CG_WAVES - 1) / CG_WAVES)), cblock(WAVE * CG_WAVES);
    const bool wide = !expl && K > BOOL_HALO + 1;  // windows past the register halo
#if SA_FUSED_STEP
    if (!bits && !wide && !expl && !a->atomic && tail && tail->chunk == 0 && !cond && !num32) {
      const int64_t nb = cgrid.x, nn = (a->n + BLOCK_ACTS - 1) / BLOCK_ACTS;
      hipLaunchKernelGGL(step_fused_kernel, dim3(xcd_grid(nb + nn)), cblock, 0, st, args, ng, gc, nb, nb + nn);
      return check_launch("step_fused_kernel");
    }
#endif
    if (bits) {  // the on-device VAEP.rate: SPADL or atomic, windowed, as bitmaps
      if (wide) {
        if (a->atomic)
          hipLaunchKernelGGL((bool_colgroup_kernel<true, false, true, true>), cgrid, cblock, 0, st, args, ng, gc);
        else
          hipLaunchKernelGGL((bool_colgroup_kernel<false, false, true, true>), cgrid, cblock, 0, st, args, ng, gc);
      } else if (a->atomic) {
        hipLaunchKernelGGL((bool_colgroup_kernel<true, false, true>), cgrid, cblock, 0, st, args, ng, gc);
      } else {
        hipLaunchKernelGGL((bool_colgroup_kernel<false, false, true>), cgrid, cblock, 0, st, args, ng, gc);
      }
    } else if (a->atomic) {
      if (expl)
        hipLaunchKernelGGL((bool_colgroup_kernel<true, true, false>), cgrid, cblock, 0, st, args, ng, gc);
      else if (wide)
        hipLaunchKernelGGL((bool_colgroup_kernel<true, false, false, true>), cgrid, cblock, 0, st, args, ng, gc);
      else
        hipLaunchKernelGGL((bool_colgroup_kernel<true, false, false>), cgrid, cblock, 0, st, args, ng, gc);
    } else {
      if (expl)
        hipLaunchKernelGGL((bool_colgroup_kernel<false, true, false>), cgrid, cblock, 0, st, args, ng, gc);
      else if (wide)
        hipLaunchKernelGGL((bool_colgroup_kernel<false, false, false, true>), cgrid, cblock, 0, st, args, ng, gc);
      else
        hipLaunchKernelGGL((bool_colgroup_kernel<false, false, false>), cgrid, cblock, 0, st, args, ng, gc);
    }
    rc = check_launch("bool_colgroup_kernel");
    if (rc) return rc;
  }
  const int gc = plan->i64_col[SA_XFN_GOALSCORE];
  if (wn || xt_cells || tail || (gc >= 0 && !expl)) {  // windowed mode: goalscore fused into this pass
    const bool fast = !expl && K <= 3;  // register-resident windows (KF = 3)
    if (cond && SA_COND_LDS && cond_lds_bytes(args.Cf, args.Ci, args.cond_n) <= COND_LDS_MAX) {
      const size_t lds = (size_t)cond_lds_bytes(args.Cf, args.Ci, args.cond_n);
      if (a->atomic)
        hipLaunchKernelGGL(num_cond_lds_kernel<true>, grid, block, lds, st, args);
      else
        hipLaunchKernelGGL(num_cond_lds_kernel<false>, grid, block, lds, st, args);
    } else if (cond) {  // windowed, K <= 3 (checked by sa_vaep_features_conditions)
      if (a->atomic)
        hipLaunchKernelGGL((num_features_kernel<true, false, 3, false, false, true>), grid, block, 0, st, args);
      else
        hipLaunchKernelGGL((num_features_kernel<false, false, 3, false, false, true>), grid, block, 0, st, args);
    } else if (num32) {  // windowed, K <= 3 (checked by sa_vaep_features_bits_f32)
      if (a->atomic)
        hipLaunchKernelGGL((num_features_kernel<true, false, 3, false, true>), grid, block, 0, st, args);
      else
        hipLaunchKernelGGL((num_features_kernel<false, false, 3, false, true>), grid, block, 0, st, args);
    } else if (tail && tail->chunk > 0 && !a->atomic) {  // sa_vaep_step_f64_chunked (probe)
      for (int64_t c0 = 0; c0 < a->n; c0 += tail->chunk) {
        const int64_t c1 = c0 + tail->chunk < a->n ? c0 + tail->chunk : a->n;
        if (tail->prefetch) {
          const int64_t th = (c1 - c0 + 3) / 4;
          hipLaunchKernelGGL(prefetch_rows_kernel, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, st, *a,
                             tail->ps, tail->pc, c0, c1, xt_cells);
        }
        args.row0 = c0;
        args.row_end = c1;
        const dim3 cg(xcd_grid((c1 - c0 + BLOCK_ACTS - 1) / BLOCK_ACTS));
        hipLaunchKernelGGL((num_features_kernel<false, false, 3, true>), cg, block, 0, st, args);
      }
    } else if (tail) {  // windowed, K <= 3 (checked by sa_vaep_step_f64)
#if SA_NUM_STAGE > 0
      if (!a->atomic && (!tail->ps || (aligned16(tail->ps) && aligned16(tail->pc)))) {
        const dim3 sg(xcd_grid((a->n + STG_T * BLOCK_ACTS - 1) / (STG_T * BLOCK_ACTS)));
        hipLaunchKernelGGL(num_staged_kernel, sg, block, sizeof(double) * 7 * STG_ROWS, st, args);
      } else
#endif
      if (a->atomic)
        hipLaunchKernelGGL((num_features_kernel<true, false, 3, true>), grid, block, 0, st, args);
      else
        hipLaunchKernelGGL((num_features_kernel<false, false, 3, true>), grid, block, 0, st, args);
    } else if (a->atomic) {
      if (expl)
        hipLaunchKernelGGL((num_features_kernel<true, true, 0>), grid, block, 0, st, args);
      else if (fast)
        hipLaunchKernelGGL((num_features_kernel<true, false, 3>), grid, block, 0, st, args);
      else
        hipLaunchKernelGGL((num_features_kernel<true, false, 0>), grid, block, 0, st, args);
    } else {
      if (expl)
        hipLaunchKernelGGL((num_features_kernel<false, true, 0>), grid, block, 0, st, args);
      else if (fast)
        hipLaunchKernelGGL((num_features_kernel<false, false, 3>), grid, block, 0, st, args);
      else
        hipLaunchKernelGGL((num_features_kernel<false, false, 0>), grid, block, 0, st, args);
    }
    rc = check_launch("num_features_kernel");
    if (rc) return rc;
  }
  if (gc >= 0 && expl) rc = sa_vaep_goalscore(a, i64_out, gc, stream);  // explicit frames: own scan
  return rc;
}

extern "C" int sa_vaep_goalscore(const sa_actions* a, const sa_block* i64_out, int32_t col,
                                 void* stream) {
  int rc = check_actions(a, true);
  if (rc) return rc;
  if ((rc = check_block(i64_out, a->n, SA_NUM_TILE_QUANTUM, "i64"))) return rc;
  if (col < 0 || col + 3 > i64_out->n_cols) return fail(SA_EINVAL, "goalscore columns outside the block");
  if (a->n == 0) return SA_OK;
  hipStream_t st = (hipStream_t)stream;
  int64_t* blk = (int64_t*)i64_out->data;
  const dim3 g4((unsigned)((a->n_segments + 3) / 4));  // one wave per segment
  if (a->atomic)
    hipLaunchKernelGGL((goalscore_wave16_kernel<true>), g4, dim3(256), 0, st, *a, blk,
                       (int64_t)i64_out->n_cols, (int64_t)col, i64_out->tile_rows);
  else
    hipLaunchKernelGGL((goalscore_wave16_kernel<false>), g4, dim3(256), 0, st, *a, blk,
                       (int64_t)i64_out->n_cols, (int64_t)col, i64_out->tile_rows);
  return check_launch("goalscore_wave16_kernel");
}

extern "C" int sa_vaep_labels(const sa_actions* a, int32_t nr_actions, uint8_t* scores,
                              uint8_t* concedes, uint8_t* goal_from_shot, int64_t ld, void* stream) {
  int rc = check_actions(a, false);
  if (rc) return rc;
  if (nr_actions < 1) return fail(SA_EINVAL, "nr_actions must be >= 1");
  if (ld % 16 != 0 || ld < ((a->n + 15) / 16) * 16)
    return fail(SA_EINVAL, "ld must be a multiple of 16 and >= round_up(n, 16)");
  if (!aligned16(scores) || !aligned16(concedes) || !aligned16(goal_from_shot))
    return fail(SA_EINVAL, "label outputs must be 16-byte aligned");
  if (a->n == 0) return SA_OK;
  const int64_t lanes = (a->n + LANE_ACTS - 1) / LANE_ACTS;
  const dim3 grid((unsigned)((lanes + 255) / 256)), block(256);
  hipStream_t st = (hipStream_t)stream;
  if (a->atomic)
    hipLaunchKernelGGL((labels_kernel<true>), grid, block, 0, st, *a, nr_actions, scores, concedes,
                       goal_from_shot);
  else
    hipLaunchKernelGGL((labels_kernel<false>), grid, block, 0, st, *a, nr_actions, scores, concedes,
                       goal_from_shot);
  return check_launch("labels_kernel");
}

template <typename T>
static int launch_formula(const sa_actions* a, const T* ps, const T* pc, T* off, T* def, T* val,
                          void* stream) {
  int rc = check_actions(a, false);
  if (rc) return rc;
  if (!ps || !pc || !off || !def || !val) return fail(SA_EINVAL, "null probability/output pointer");
  if (!aligned16(off) || !aligned16(def) || !aligned16(val))
    return fail(SA_EINVAL, "formula outputs must be 16-byte aligned (length >= round_up(n, 4))");
  if (a->n == 0) return SA_OK;
  constexpr int V = 16 / sizeof(T);
  const int64_t lanes = (a->n + V - 1) / V;
  const dim3 grid((unsigned)((lanes + 255) / 256)), block(256);
  const bool vec_ok = aligned16(ps) && aligned16(pc);
  hipStream_t st = (hipStream_t)stream;
  if (a->atomic)
    hipLaunchKernelGGL((formula_kernel<true, T>), grid, block, 0, st, *a, ps, pc, off, def, val, vec_ok);
  else
    hipLaunchKernelGGL((formula_kernel<false, T>), grid, block, 0, st, *a, ps, pc, off, def, val, vec_ok);
  return check_launch("formula_kernel");
}

extern "C" int sa_vaep_formula_f64(const sa_actions* a, const double* p_scores,
                                   const double* p_concedes, double* off, double* def, double* val,
                                   void* stream) {
  return launch_formula<double>(a, p_scores, p_concedes, off, def, val, stream);
}

extern "C" int sa_vaep_formula_f32(const sa_actions* a, const float* p_scores, const float* p_concedes,
                                   float* off, float* def, float* val, void* stream) {
  return launch_formula<float>(a, p_scores, p_concedes, off, def, val, stream);
}

template <typename T>
static int launch_labels_formula(const sa_actions* a, int32_t nr_actions, uint8_t* scores,
                                 uint8_t* concedes, uint8_t* goal_from_shot, int64_t ld, const T* ps,
                                 const T* pc, T* off, T* def, T* val, void* stream) {
  int rc = check_actions(a, false);
  if (rc) return rc;
  if (nr_actions < 1) return fail(SA_EINVAL, "nr_actions must be >= 1");
  if (ld % 16 != 0 || ld < ((a->n + 15) / 16) * 16)
    return fail(SA_EINVAL, "ld must be a multiple of 16 and >= round_up(n, 16)");
  if (!aligned16(scores) || !aligned16(concedes) || !aligned16(goal_from_shot))
    return fail(SA_EINVAL, "label outputs must be 16-byte aligned");
  if (!ps || !pc || !off || !def || !val) return fail(SA_EINVAL, "null probability/output pointer");
  if (!aligned16(off) || !aligned16(def) || !aligned16(val))
    return fail(SA_EINVAL, "formula outputs must be 16-byte aligned (length >= round_up(n, 16))");
  if (a->n == 0) return SA_OK;
  const int64_t waves = (a->n + WAVE * LANE_ACTS - 1) / (WAVE * LANE_ACTS);
  const dim3 grid((unsigned)((waves + 3) / 4)), block(256);
  const bool vec_ok = aligned16(ps) && aligned16(pc);
  hipStream_t st = (hipStream_t)stream;
  if (a->atomic)
    hipLaunchKernelGGL((labels_formula_kernel<true, T>), grid, block, 0, st, *a, nr_actions, scores,
                       concedes, goal_from_shot, ps, pc, off, def, val, vec_ok);
  else
    hipLaunchKernelGGL((labels_formula_kernel<false, T>), grid, block, 0, st, *a, nr_actions, scores,
                       concedes, goal_from_shot, ps, pc, off, def, val, vec_ok);
  return check_launch("labels_formula_kernel");
}

extern "C" int sa_vaep_labels_formula_f64(const sa_actions* a, int32_t nr_actions, uint8_t* scores,
                                          uint8_t* concedes, uint8_t* goal_from_shot, int64_t ld,
                                          const double* p_scores, const double* p_concedes, double* off,
                                          double* def, double* val, void* stream) {
  return launch_labels_formula<double>(a, nr_actions, scores, concedes, goal_from_shot, ld, p_scores,
                                       p_concedes, off, def, val, stream);
}

extern "C" int sa_vaep_labels_formula_f32(const sa_actions* a, int32_t nr_actions, uint8_t* scores,
                                          uint8_t* concedes, uint8_t* goal_from_shot, int64_t ld,
                                          const float* p_scores, const float* p_concedes, float* off,
                                          float* def, float* val, void* stream) {
  return launch_labels_formula<float>(a, nr_actions, scores, concedes, goal_from_shot, ld, p_scores,
                                      p_concedes, off, def, val, stream);
}
