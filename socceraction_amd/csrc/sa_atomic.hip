// SPADL -> Atomic-SPADL conversion on gfx950 (reference: socceraction/atomic/spadl/base.py).
//
// The reference runs four insertion passes, each a concat + stable sort on (game_id,
// period_id, action_id) + action_id reset.  Every inserted row carries its parent's
// action_id + 0.1 (and, for a dribble, the successor's game / period, which equal the
// parent's position in sorted order), so it always lands directly after its parent.  Hence
// row r of the (sorted) input expands into the fixed sequence
//
//     r, x4(r)?, x3(r)?, dA(r)?, e1(r)?, dB(r)?
//
//   e1  _extra_from_passes  (base.py:38-112)   r and its INPUT-order successor q
//   dA  _add_dribbles        (spadl/base.py:54-93) r -> r'   (only without e1: e1 starts
//                            where r ends, so r -> e1 is never far enough for a dribble)
//   dB  _add_dribbles        e1 -> r'
//   x3  _extra_from_shots    (base.py:115-165)  goal / owngoal / shot followed by a corner or
//                            goalkick (the row after r is dA, e1 or r'; only r' can be one)
//   x4  _extra_from_fouls    (base.py:168-196)  yellow / red card
//
// where r' is r's successor in sorted order.  Inserted rows never qualify for a later pass
// (results -1 / success, non-shot types), which is why the sequence stops at five.  One
// kernel counts each block's output rows, one scans the block totals, one writes the rows
// (block scan + the block's prefix).  Everything is exact: the only arithmetic is the
// reference's own (midpoint times, squared distances, end - start) in f64 with
// -ffp-contract=off.
#include <hip/hip_runtime.h>

#include "sa_common.h"
#include "sa_internal.h"

namespace sa {

constexpr int AC_THREADS = 256;
constexpr int AC_PER_THREAD = 1;
constexpr int AC_BLOCK_ROWS = AC_THREADS * AC_PER_THREAD;  // 256 sorted rows per block
constexpr int AC_MAX_OUT = AC_BLOCK_ROWS * 5;              // worst-case output rows per block

// atomic/spadl/config.py:25-36 ids; `actiontypes.index('interception')` is the FIRST
// position, 10 (base.py:96-99)
constexpr int A_DRIBBLE = 21, A_RECEIVAL = 23, A_INTERCEPTION = 10, A_OUT = 25, A_OFFSIDE = 26,
              A_GOAL = 27, A_OWNGOAL = 28, A_YELLOW = 29, A_RED = 30, A_CORNER = 31,
              A_FREEKICK = 32;
constexpr int T_THROW_IN = 2, T_GOALKICK = 22;

struct SRow {
  double t, sx, sy, ex, ey;
  int32_t game, team, player, event;
  int per, type, res, bp;
};

__device__ __forceinline__ SRow load_srow(const sa_spadl_frame& F, int64_t r) {
  SRow o;
  o.t = F.time_seconds[r];
  o.sx = F.start_x[r];
  o.sy = F.start_y[r];
  o.ex = F.end_x[r];
  o.ey = F.end_y[r];
  o.game = F.game[r];
  o.team = F.team[r];
  o.player = F.player[r];
  o.event = F.event[r];
  o.per = F.period_id[r];
  o.type = F.type_id[r];
  o.res = F.result_id[r];
  o.bp = F.bodypart_id[r];
  return o;
}

__device__ __forceinline__ bool is_passlike(int t) {  // base.py:42-53
  return t == 0 || t == 1 || t == 2 || t == 3 || t == 4 || t == 5 || t == 6 || t == 18 || t == 22;
}
__device__ __forceinline__ bool is_interceptionlike(int t) {  // base.py:55-63
  return t == 10 || t == 9 || t == 16 || t == 14 || t == 15 || t == 17;
}
__device__ __forceinline__ bool is_shot(int t) { return t == 11 || t == 12 || t == 13; }

// _add_dribbles predicate for an action ending at (ex, ey) by `team` at time t in period
// `per`, followed by row n (spadl/base.py:57-69)
__device__ __forceinline__ bool dribble(double ex, double ey, int32_t team, double t, int per,
                                        const SRow& n) {
  const double dx = ex - n.sx, dy = ey - n.sy;
  const double d2 = dx * dx + dy * dy;
  const double dt = n.t - t;
  return team == n.team && d2 >= 9.0 && d2 <= 3600.0 && dt < 10.0 && per == n.per;
}

enum { G_X4 = 1, G_X3 = 2, G_DA = 4, G_E1 = 8, G_DB = 16 };

struct Group {
  SRow r, rp;  // the row and its sorted successor
  uint32_t mask;
  int x4_type, x3_type, e1_type;
  int32_t e1_team, e1_player;
  double e1_t;
};

// e1 of row R followed in INPUT order by Q (base.py:65-107): a pass-like action followed by a
// non-interception in the same game and period gets a receival / interception / out / offside
// row at its end; false when it gets none
__device__ __forceinline__ bool e1_of(const SRow& R, const SRow& Q, int& type, int32_t& team, int32_t& player,
                                      double& t) {
  if (!is_passlike(R.type) || Q.game != R.game || Q.per != R.per || is_interceptionlike(Q.type)) return false;
  const bool st = Q.team == R.team;
  const bool out = (Q.type == T_GOALKICK && !st) || Q.type == T_THROW_IN;
  const bool offside = R.res == 2;
  int ty = st ? A_RECEIVAL : A_INTERCEPTION;
  if (out) ty = A_OUT;
  if (offside) ty = A_OFFSIDE;
  type = ty;
  team = ty == A_INTERCEPTION ? Q.team : R.team;
  player = (out || offside) ? R.player : Q.player;
  t = (R.t + Q.t) / 2;
  return true;
}

// PASSES = false: the frame already went through _extra_from_passes (the general first pass,
// sa_atomic_passes_emit), so no row gets an e1 here
template <bool PASSES = true>
__device__ __forceinline__ Group group_at(const sa_spadl_frame& F, int64_t p) {
  const int64_t n = F.n;
  Group G;
  const int64_t r = F.order ? F.order[p] : p;
  G.r = load_srow(F, r);
  const bool has_rp = p + 1 < n;
  if (has_rp) G.rp = load_srow(F, F.order ? F.order[p + 1] : p + 1);
  const SRow& R = G.r;
  G.mask = 0;
  // e1: pass-like action followed (in INPUT order) by a non-interception in the same game
  // and period
  if (PASSES && r + 1 < n && is_passlike(R.type)) {
    const SRow Q = (F.order == nullptr && has_rp) ? G.rp : load_srow(F, r + 1);
    if (e1_of(R, Q, G.e1_type, G.e1_team, G.e1_player, G.e1_t)) G.mask |= G_E1;
  }
  if (has_rp) {
    if (G.mask & G_E1) {
      if (dribble(R.ex, R.ey, G.e1_team, G.e1_t, R.per, G.rp)) G.mask |= G_DB;
    } else if (dribble(R.ex, R.ey, R.team, R.t, R.per, G.rp)) {
      G.mask |= G_DA;
    }
  }
  const bool shot = is_shot(R.type);
  const bool goal = shot && R.res == 1;
  const bool owngoal = R.res == 3;
  const bool out3 = shot && has_rp && !(G.mask & (G_DA | G_E1)) &&
                    (G.rp.type == 5 || G.rp.type == 6 || G.rp.type == T_GOALKICK) &&
                    G.rp.game == R.game && G.rp.per == R.per;
  if (goal || owngoal || out3) {
    G.mask |= G_X3;
    G.x3_type = owngoal ? A_OWNGOAL : (goal ? A_GOAL : A_OUT);
  }
  if (R.res == 4 || R.res == 5) {
    G.mask |= G_X4;
    G.x4_type = R.res == 5 ? A_RED : A_YELLOW;
  }
  return G;
}

__device__ __forceinline__ int group_size(uint32_t mask) { return 1 + __popc(mask); }

__device__ __forceinline__ int simplify(int t) {  // base.py:223-235
  if (t == 5 || t == 6) return A_CORNER;
  if (t == 3 || t == 4 || t == 13) return A_FREEKICK;
  return t;
}

// One output row (after _convert_columns / _simplify).  `kind` is the position in the group
// sequence r, x4, x3, dA, e1, dB.
struct Elem {
  double t, x, y, dx, dy;
  int32_t game, team, player, event;
  int per, type, bp;
};

enum { K_R = 0, K_X4, K_X3, K_DA, K_E1, K_DB, K_COUNT };

__device__ __forceinline__ bool has_kind(uint32_t mask, int k) {
  return k == K_R || (mask & (1u << (k == K_X4 ? 0 : k == K_X3 ? 1 : k == K_DA ? 2 : k == K_E1 ? 3 : 4)));
}

__device__ __forceinline__ Elem elem_of(const Group& G, int kind) {
  const SRow& R = G.r;
  const SRow& N = G.rp;
  Elem e;
  switch (kind) {
    case K_R:  // r itself: x, y = start; dx, dy = end - start
      e = Elem{R.t, R.sx, R.sy, R.ex - R.sx, R.ey - R.sy, R.game, R.team, R.player, R.event, R.per,
               simplify(R.type), R.bp};
      break;
    case K_X4:  // card: start = end = r's end; r's time, bodypart, team, player
      e = Elem{R.t, R.ex, R.ey, R.ex - R.ex, R.ey - R.ey, R.game, R.team, R.player, R.event, R.per,
               G.x4_type, R.bp};
      break;
    case K_X3:  // out / goal / owngoal: same shape
      e = Elem{R.t, R.ex, R.ey, R.ex - R.ex, R.ey - R.ey, R.game, R.team, R.player, R.event, R.per,
               G.x3_type, R.bp};
      break;
    case K_DA:  // dribble r -> r': the successor's game, period, team, player; no event
      e = Elem{(R.t + N.t) / 2, R.ex, R.ey, N.sx - R.ex, N.sy - R.ey, N.game, N.team, N.player, -1,
               N.per, A_DRIBBLE, 0};
      break;
    case K_E1:  // receival / interception / out / offside at r's end, foot
      e = Elem{G.e1_t, R.ex, R.ey, R.ex - R.ex, R.ey - R.ey, R.game, G.e1_team, G.e1_player, R.event,
               R.per, G.e1_type, 0};
      break;
    default:  // dribble e1 -> r'
      e = Elem{(G.e1_t + N.t) / 2, R.ex, R.ey, N.sx - R.ex, N.sy - R.ey, N.game, N.team, N.player, -1,
               N.per, A_DRIBBLE, 0};
      break;
  }
  return e;
}

// exclusive block scan of one int per thread (256 threads = 4 waves)
__device__ __forceinline__ int64_t block_excl_scan(int64_t v, int64_t* wsum, int64_t& total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int64_t incl = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  int64_t pre = 0;
  total = 0;
#pragma unroll
  for (int k = 0; k < AC_THREADS / 64; ++k) {
    pre += k < wv ? wsum[k] : 0;
    total += wsum[k];
  }
  return pre + incl - v;
}

template <bool PASSES>
__global__ __launch_bounds__(AC_THREADS) void atomic_count_kernel(sa_spadl_frame F, int64_t* __restrict__ bsum) {
  __shared__ int64_t wsum[AC_THREADS / 64];
  const int64_t p = (int64_t)blockIdx.x * AC_BLOCK_ROWS + threadIdx.x;
  const int64_t c = p < F.n ? group_size(group_at<PASSES>(F, p).mask) : 0;
  int64_t total;
  block_excl_scan(c, wsum, total);
  if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

// exclusive prefix of the block totals, in place; bsum[nb] = grand total (one workgroup of
// 1024 threads).  Tiles of SC_THREADS * SC_K entries are staged through LDS with coalesced
// loads (block totals are <= 5 * 256, so int32 holds them), each thread scans SC_K
// consecutive entries serially, and ONE block scan per tile combines the threads.
constexpr int SC_THREADS = 1024, SC_K = 16, SC_TILE = SC_THREADS * SC_K;

__global__ __launch_bounds__(SC_THREADS) void atomic_scan_kernel(int64_t* __restrict__ bsum, int64_t nb) {
  __shared__ int32_t tile[SC_TILE];  // 64 KiB
  __shared__ int64_t ws[SC_THREADS / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int64_t carry = 0;
  for (int64_t c0 = 0; c0 < nb; c0 += SC_TILE) {
#pragma unroll
    for (int k = 0; k < SC_K; ++k) {
      const int64_t i = c0 + (int64_t)k * SC_THREADS + threadIdx.x;
      tile[k * SC_THREADS + threadIdx.x] = i < nb ? (int32_t)bsum[i] : 0;
    }
    __syncthreads();
    int32_t loc[SC_K];
    int64_t acc = 0;
#pragma unroll
    for (int k = 0; k < SC_K; ++k) {
      loc[k] = tile[threadIdx.x * SC_K + k];
      acc += loc[k];
    }
    int64_t incl = acc;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int64_t y = __shfl_up(incl, off, 64);
      if (lane >= off) incl += y;
    }
    if (lane == 63) ws[wv] = incl;
    __syncthreads();
    int64_t pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < SC_THREADS / 64; ++w) {
      const int64_t x = ws[w];
      pre += w < wv ? x : 0;
      tot += x;
    }
    int64_t run = carry + pre + incl - acc;
#pragma unroll
    for (int k = 0; k < SC_K; ++k) {
      const int64_t i = c0 + (int64_t)threadIdx.x * SC_K + k;
      if (i < nb) bsum[i] = run;
      run += loc[k];
    }
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) bsum[nb] = carry;
}

// Each block's output rows form one contiguous range [bpre[b], bpre[b+1]).  The rows are
// built in LDS (5 f64 columns, then -- reusing the same bytes -- the 4 int32 and 3 u8
// columns) and copied out with consecutive threads on consecutive rows, so every global
// store instruction is a contiguous run instead of 64 scattered 8-B writes (16M SPADL rows:
// 4.2 -> 0.61 ms).
template <bool PASSES>
__global__ __launch_bounds__(AC_THREADS) void atomic_emit_kernel(sa_spadl_frame F, const int64_t* __restrict__ bpre,
                                                                sa_atomic_frame O) {
  __shared__ double lds[5 * AC_MAX_OUT];  // 51,200 B
  __shared__ int64_t wsum[AC_THREADS / 64];
  const int64_t p = (int64_t)blockIdx.x * AC_BLOCK_ROWS + threadIdx.x;
  const bool live = p < F.n;
  Group G;
  int c = 0;
  if (live) {
    G = group_at<PASSES>(F, p);
    c = group_size(G.mask);
  }
  int64_t total;
  const int lo = (int)block_excl_scan(c, wsum, total);
  const int tot = (int)total;
  const int64_t base = bpre[blockIdx.x];
  if (live) {
    int o = lo;
#pragma unroll
    for (int k = 0; k < K_COUNT; ++k) {
      if (!has_kind(G.mask, k)) continue;
      const Elem e = elem_of(G, k);
      lds[0 * AC_MAX_OUT + o] = e.t;
      lds[1 * AC_MAX_OUT + o] = e.x;
      lds[2 * AC_MAX_OUT + o] = e.y;
      lds[3 * AC_MAX_OUT + o] = e.dx;
      lds[4 * AC_MAX_OUT + o] = e.dy;
      ++o;
    }
  }
  __syncthreads();
  double* const fo[5] = {O.time_seconds, O.x, O.y, O.dx, O.dy};
#pragma unroll
  for (int col = 0; col < 5; ++col)
    for (int k = threadIdx.x; k < tot; k += AC_THREADS) fo[col][base + k] = lds[col * AC_MAX_OUT + k];
  __syncthreads();
  int32_t* li = reinterpret_cast<int32_t*>(lds);
  uint8_t* lu = reinterpret_cast<uint8_t*>(li + 4 * AC_MAX_OUT);
  if (live) {
    int o = lo;
#pragma unroll
    for (int k = 0; k < K_COUNT; ++k) {
      if (!has_kind(G.mask, k)) continue;
      const Elem e = elem_of(G, k);
      li[0 * AC_MAX_OUT + o] = e.game;
      li[1 * AC_MAX_OUT + o] = e.team;
      li[2 * AC_MAX_OUT + o] = e.player;
      li[3 * AC_MAX_OUT + o] = e.event;
      lu[0 * AC_MAX_OUT + o] = (uint8_t)e.per;
      lu[1 * AC_MAX_OUT + o] = (uint8_t)e.type;
      lu[2 * AC_MAX_OUT + o] = (uint8_t)e.bp;
      ++o;
    }
  }
  __syncthreads();
  int32_t* const io[4] = {O.game, O.team, O.player, O.event};
#pragma unroll
  for (int col = 0; col < 4; ++col)
    for (int k = threadIdx.x; k < tot; k += AC_THREADS) io[col][base + k] = li[col * AC_MAX_OUT + k];
  uint8_t* const uo[3] = {O.period_id, O.type_id, O.bodypart_id};
#pragma unroll
  for (int col = 0; col < 3; ++col)
    for (int k = threadIdx.x; k < tot; k += AC_THREADS) uo[col][base + k] = lu[col * AC_MAX_OUT + k];
}

// ---- _add_dribbles as an operator of its own (spadl/base.py:54-93) -----------------------
// Row j is compared with its INPUT-order successor (shift(-1, fill_value=0): the last row meets
// an all-zero row whose period 0 never matches).  A dribble row j' carries the successor's
// game / period / team / player, the midpoint time, start = j's end and end = the successor's
// start, foot / dribble / success.  Output order: when the (game, period, action_id) keys of
// the input increase strictly and every dribble's key (successor's game and period, action_id
// + 0.1) falls below its successor's key (host-checked), the reference's sort puts j' directly
// after j, so rows are written at j + (dribbles before j) (+1 for j'); otherwise the host's
// stable lexsort of the concatenated keys gives every row's position in `dest` (first the n
// input rows, then the dribbles in input order -- the reference's concat order).
struct DribbleRule {
  double min2, max2, max_dt;  // min_dribble_length**2, max_dribble_length**2, max_dribble_duration
};

__device__ __forceinline__ bool dribble_after(const sa_spadl_frame& F, int64_t j, const DribbleRule& D,
                                              SRow& R, SRow& Q) {
  R = load_srow(F, j);
  if (j + 1 >= F.n) return false;
  Q = load_srow(F, j + 1);
  const double dx = R.ex - Q.sx, dy = R.ey - Q.sy;
  const double d2 = dx * dx + dy * dy;
  const double dt = Q.t - R.t;
  return R.team == Q.team && d2 >= D.min2 && d2 <= D.max2 && dt < D.max_dt && R.per == Q.per;
}

// Also counts (into *misplaced) the rows that rule out the fast layout: input keys (game code,
// period, action_id) not strictly above the previous row's, or a dribble whose key
// (action_id + 0.1) does not fall strictly between its row's and its successor's.
__global__ __launch_bounds__(AC_THREADS) void dribble_count_kernel(sa_spadl_frame F, DribbleRule D,
                                                                  const double* __restrict__ aid,
                                                                  int64_t* __restrict__ bsum,
                                                                  unsigned long long* __restrict__ misplaced,
                                                                  uint8_t* __restrict__ flags) {
  __shared__ int64_t wsum[AC_THREADS / 64];
  const int64_t p = (int64_t)blockIdx.x * AC_BLOCK_ROWS + threadIdx.x;
  int64_t c = 0;
  bool bad = false;
  if (p < F.n) {
    SRow R, Q;
    const bool d = dribble_after(F, p, D, R, Q);
    if (flags) flags[p] = d;
    c = 1 + d;
    if (aid) {
      const double a = aid[p];
      if (p > 0) {
        const int32_t g0 = F.game[p - 1];
        const int p0 = F.period_id[p - 1];
        const double a0 = aid[p - 1];
        bad = !(g0 < R.game || (g0 == R.game && (p0 < R.per || (p0 == R.per && a0 < a))));
      }
      if (d) {
        const double da = a + 0.1;
        bad |= !(da > a && da < aid[p + 1]);
      }
    }
  }
  const uint64_t m = __ballot(bad);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(misplaced, (unsigned long long)__popcll(m));
  int64_t total;
  block_excl_scan(c, wsum, total);
  if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

__device__ __forceinline__ void put_spadl_row(const sa_spadl_out& O, int64_t o, double t, double sx, double sy,
                                              double ex, double ey, int32_t game, int32_t team,
                                              int32_t player, int32_t event, int per, int type, int res,
                                              int bp, int64_t src) {
  O.time_seconds[o] = t;
  O.start_x[o] = sx;
  O.start_y[o] = sy;
  O.end_x[o] = ex;
  O.end_y[o] = ey;
  O.game[o] = game;
  O.team[o] = team;
  O.player[o] = player;
  O.event[o] = event;
  O.period_id[o] = (uint8_t)per;
  O.type_id[o] = (uint8_t)type;
  O.result_id[o] = (uint8_t)res;
  O.bodypart_id[o] = (uint8_t)bp;
  O.src[o] = src;
}

// Fast layout (dest == NULL): a block's rows form one contiguous output range; they are built
// in LDS (the 5 f64 + src columns, then the 4 int32 + 4 u8 columns in the same bytes) and
// copied out by consecutive threads, like atomic_emit_kernel.  With dest the rows scatter.
constexpr int DE_MAX_OUT = 2 * AC_BLOCK_ROWS;

__global__ __launch_bounds__(AC_THREADS) void dribble_emit_kernel(sa_spadl_frame F, DribbleRule D,
                                                                 const int64_t* __restrict__ bpre,
                                                                 const int64_t* __restrict__ dest,
                                                                 sa_spadl_out O) {
  __shared__ double lds[6 * DE_MAX_OUT];  // 24 KiB
  __shared__ int64_t wsum[AC_THREADS / 64];
  const int64_t p = (int64_t)blockIdx.x * AC_BLOCK_ROWS + threadIdx.x;
  const bool live = p < F.n;
  SRow R, Q;
  bool d = false;
  if (live) d = dribble_after(F, p, D, R, Q);
  int64_t total;
  const int64_t lo = block_excl_scan(live ? 1 + d : 0, wsum, total);
  const int64_t g = bpre[blockIdx.x] + lo;  // row p's position in the fast layout
  if (dest) {
    if (!live) return;
    put_spadl_row(O, dest[p], R.t, R.sx, R.sy, R.ex, R.ey, R.game, R.team, R.player, R.event, R.per, R.type,
                  R.res, R.bp, p);
    if (d)  // g - p = dribbles before row p
      put_spadl_row(O, dest[F.n + (g - p)], (R.t + Q.t) / 2, R.ex, R.ey, Q.sx, Q.sy, Q.game, Q.team, Q.player,
                    -1, Q.per, A_DRIBBLE, 1, 0, ~(p + 1));
    return;
  }
  const int tot = (int)total;
  const int o = (int)lo;
  const int64_t base = bpre[blockIdx.x];
  int64_t* lsrc = reinterpret_cast<int64_t*>(lds + 5 * DE_MAX_OUT);
  if (live) {
    lds[0 * DE_MAX_OUT + o] = R.t;
    lds[1 * DE_MAX_OUT + o] = R.sx;
    lds[2 * DE_MAX_OUT + o] = R.sy;
    lds[3 * DE_MAX_OUT + o] = R.ex;
    lds[4 * DE_MAX_OUT + o] = R.ey;
    lsrc[o] = p;
    if (d) {
      lds[0 * DE_MAX_OUT + o + 1] = (R.t + Q.t) / 2;
      lds[1 * DE_MAX_OUT + o + 1] = R.ex;
      lds[2 * DE_MAX_OUT + o + 1] = R.ey;
      lds[3 * DE_MAX_OUT + o + 1] = Q.sx;
      lds[4 * DE_MAX_OUT + o + 1] = Q.sy;
      lsrc[o + 1] = ~(p + 1);
    }
  }
  __syncthreads();
  double* const fo[5] = {O.time_seconds, O.start_x, O.start_y, O.end_x, O.end_y};
#pragma unroll
  for (int col = 0; col < 5; ++col)
    for (int k = threadIdx.x; k < tot; k += AC_THREADS) fo[col][base + k] = lds[col * DE_MAX_OUT + k];
  for (int k = threadIdx.x; k < tot; k += AC_THREADS) O.src[base + k] = lsrc[k];
  __syncthreads();
  int32_t* li = reinterpret_cast<int32_t*>(lds);
  uint8_t* lu = reinterpret_cast<uint8_t*>(li + 4 * DE_MAX_OUT);
  if (live) {
    li[0 * DE_MAX_OUT + o] = R.game;
    li[1 * DE_MAX_OUT + o] = R.team;
    li[2 * DE_MAX_OUT + o] = R.player;
    li[3 * DE_MAX_OUT + o] = R.event;
    lu[0 * DE_MAX_OUT + o] = (uint8_t)R.per;
    lu[1 * DE_MAX_OUT + o] = (uint8_t)R.type;
    lu[2 * DE_MAX_OUT + o] = (uint8_t)R.res;
    lu[3 * DE_MAX_OUT + o] = (uint8_t)R.bp;
    if (d) {
      li[0 * DE_MAX_OUT + o + 1] = Q.game;
      li[1 * DE_MAX_OUT + o + 1] = Q.team;
      li[2 * DE_MAX_OUT + o + 1] = Q.player;
      li[3 * DE_MAX_OUT + o + 1] = -1;
      lu[0 * DE_MAX_OUT + o + 1] = (uint8_t)Q.per;
      lu[1 * DE_MAX_OUT + o + 1] = (uint8_t)A_DRIBBLE;
      lu[2 * DE_MAX_OUT + o + 1] = 1;
      lu[3 * DE_MAX_OUT + o + 1] = 0;
    }
  }
  __syncthreads();
  int32_t* const io[4] = {O.game, O.team, O.player, O.event};
#pragma unroll
  for (int col = 0; col < 4; ++col)
    for (int k = threadIdx.x; k < tot; k += AC_THREADS) io[col][base + k] = li[col * DE_MAX_OUT + k];
  uint8_t* const uo[4] = {O.period_id, O.type_id, O.result_id, O.bodypart_id};
#pragma unroll
  for (int col = 0; col < 4; ++col)
    for (int k = threadIdx.x; k < tot; k += AC_THREADS) uo[col][base + k] = lu[col * DE_MAX_OUT + k];
}

// ---- the general first pass (base.py:38-112) ---------------------------------------------
// For frames whose (game, period, action_id) keys repeat, or lie less than 0.1 apart, the e1
// rows do not all land right after their parents, so the first pass runs on its own: flags of
// the rows that get one (INPUT-order successor, as the reference's shift(-1)), then every row of
// the reference's concat [inputs, e1 rows in input order] is written at its position in the
// stable sort (dest, from the host).  After it the keys are 0..n+m-1 (the reference resets
// action_id), and the remaining passes run as the single expansion without e1 (PASSES = false).
__global__ __launch_bounds__(AC_THREADS) void atomic_passes_flags_kernel(sa_spadl_frame F,
                                                                        uint8_t* __restrict__ flags) {
  const int64_t j = (int64_t)blockIdx.x * AC_THREADS + threadIdx.x;
  if (j >= F.n) return;
  bool on = false;
  if (j + 1 < F.n) {
    const SRow R = load_srow(F, j);
    if (is_passlike(R.type)) {
      int ty;
      int32_t tm, pl;
      double t;
      on = e1_of(R, load_srow(F, j + 1), ty, tm, pl, t);
    }
  }
  flags[j] = on;
}

__global__ __launch_bounds__(AC_THREADS) void atomic_passes_emit_kernel(sa_spadl_frame F,
                                                                       const int64_t* __restrict__ parents,
                                                                       int64_t m, const int64_t* __restrict__ dest,
                                                                       sa_spadl_out O) {
  const int64_t i = (int64_t)blockIdx.x * AC_THREADS + threadIdx.x;
  if (i >= F.n + m) return;
  if (i < F.n) {
    const SRow R = load_srow(F, i);
    put_spadl_row(O, dest[i], R.t, R.sx, R.sy, R.ex, R.ey, R.game, R.team, R.player, R.event, R.per, R.type,
                  R.res, R.bp, i);
    return;
  }
  const int64_t p = parents[i - F.n];
  SA_DGUARD(p >= 0 && p + 1 < F.n, p, return);
  const SRow R = load_srow(F, p);
  int ty = 0;
  int32_t tm = 0, pl = 0;
  double t = 0.0;
  e1_of(R, load_srow(F, p + 1), ty, tm, pl, t);
  // start = end = the parent's end; bodypart foot; result -1 (kept as 255: no later pass reads
  // it as a result the reference would match); the parent's event
  put_spadl_row(O, dest[i], t, R.ex, R.ey, R.ex, R.ey, R.game, tm, pl, R.event, R.per, ty, 255, 0, ~p);
}

// seg_off[key[k]] = k at every run start of the sorted keys 0..n_seg-1 (each present)
__global__ __launch_bounds__(256) void segment_offsets_kernel(const int32_t* __restrict__ key, int64_t n,
                                                              int64_t n_seg, int64_t* __restrict__ seg_off) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k == 0) seg_off[n_seg] = n;
  if (k >= n) return;
  const int32_t g = key[k];
  if ((k == 0 || key[k - 1] != g) && g >= 0 && g < n_seg) seg_off[g] = k;
}

}  // namespace sa

// ================================== C ABI =================================================
using namespace sa;

static int64_t n_blocks(int64_t n) { return (n + AC_BLOCK_ROWS - 1) / AC_BLOCK_ROWS; }

extern "C" int64_t sa_atomic_scratch_bytes(int64_t n) {
  return n < 0 ? 0 : (n_blocks(n) + 2) * (int64_t)sizeof(int64_t);
}

static int check_spadl_frame(const sa_spadl_frame* F) {
  if (!F || F->n < 0) return fail(SA_EINVAL, "bad sa_spadl_frame");
  if (F->n > 0 && (!F->time_seconds || !F->start_x || !F->start_y || !F->end_x || !F->end_y ||
                   !F->game || !F->team || !F->player || !F->event || !F->period_id ||
                   !F->type_id || !F->result_id || !F->bodypart_id))
    return fail(SA_EINVAL, "sa_spadl_frame has a null column");
  return SA_OK;
}

template <bool PASSES>
static int atomic_count(const sa_spadl_frame* in, void* scratch, int64_t* n_out, void* stream) {
  int rc = check_spadl_frame(in);
  if (rc) return rc;
  if (!n_out || (in->n > 0 && !scratch)) return fail(SA_EINVAL, "null scratch or n_out");
  *n_out = 0;
  if (in->n == 0) return SA_OK;
  hipStream_t st = (hipStream_t)stream;
  const int64_t nb = n_blocks(in->n);
  int64_t* bsum = (int64_t*)scratch;
  hipLaunchKernelGGL(atomic_count_kernel<PASSES>, dim3((unsigned)nb), dim3(AC_THREADS), 0, st, *in, bsum);
  if ((rc = check_launch("atomic_count_kernel"))) return rc;
  hipLaunchKernelGGL(atomic_scan_kernel, dim3(1), dim3(SC_THREADS), 0, st, bsum, nb);
  if ((rc = check_launch("atomic_scan_kernel"))) return rc;
  if ((rc = check_hip(hipMemcpyAsync(n_out, bsum + nb, sizeof(int64_t), hipMemcpyDeviceToHost, st),
                      "copy n_out")))
    return rc;
  return check_hip(hipStreamSynchronize(st), "hipStreamSynchronize");
}

template <bool PASSES>
static int atomic_emit(const sa_spadl_frame* in, const void* scratch, const sa_atomic_frame* out, void* stream) {
  int rc = check_spadl_frame(in);
  if (rc) return rc;
  if (in->n == 0) return SA_OK;
  if (!scratch || !out || !out->time_seconds || !out->x || !out->y || !out->dx || !out->dy ||
      !out->game || !out->team || !out->player || !out->event || !out->period_id || !out->type_id ||
      !out->bodypart_id)
    return fail(SA_EINVAL, "null scratch or output column");
  const int64_t nb = n_blocks(in->n);
  hipLaunchKernelGGL(atomic_emit_kernel<PASSES>, dim3((unsigned)nb), dim3(AC_THREADS), 0, (hipStream_t)stream,
                     *in, (const int64_t*)scratch, *out);
  return check_launch("atomic_emit_kernel");
}

extern "C" int sa_atomic_count(const sa_spadl_frame* in, void* scratch, int64_t* n_out, void* stream) {
  return atomic_count<true>(in, scratch, n_out, stream);
}

extern "C" int sa_atomic_emit(const sa_spadl_frame* in, const void* scratch, const sa_atomic_frame* out,
                              void* stream) {
  return atomic_emit<true>(in, scratch, out, stream);
}

extern "C" int sa_atomic_count_after_passes(const sa_spadl_frame* in, void* scratch, int64_t* n_out,
                                            void* stream) {
  if (in && in->order) return fail(SA_EINVAL, "the first pass's output is sorted: order must be NULL");
  return atomic_count<false>(in, scratch, n_out, stream);
}

extern "C" int sa_atomic_emit_after_passes(const sa_spadl_frame* in, const void* scratch,
                                           const sa_atomic_frame* out, void* stream) {
  if (in && in->order) return fail(SA_EINVAL, "the first pass's output is sorted: order must be NULL");
  return atomic_emit<false>(in, scratch, out, stream);
}

static bool spadl_out_ok(const sa_spadl_out* out) {
  return out && out->time_seconds && out->start_x && out->start_y && out->end_x && out->end_y && out->game &&
         out->team && out->player && out->event && out->period_id && out->type_id && out->result_id &&
         out->bodypart_id && out->src;
}

extern "C" int sa_atomic_passes_flags(const sa_spadl_frame* in, uint8_t* flags, void* stream) {
  int rc = check_spadl_frame(in);
  if (rc) return rc;
  if (in->order) return fail(SA_EINVAL, "_extra_from_passes reads rows in input order: order must be NULL");
  if (in->n == 0) return SA_OK;
  if (!flags) return fail(SA_EINVAL, "null flags");
  hipLaunchKernelGGL(atomic_passes_flags_kernel, dim3((unsigned)n_blocks(in->n)), dim3(AC_THREADS), 0,
                     (hipStream_t)stream, *in, flags);
  return check_launch("atomic_passes_flags_kernel");
}

extern "C" int sa_atomic_passes_emit(const sa_spadl_frame* in, const int64_t* parents, int64_t m,
                                     const int64_t* dest, const sa_spadl_out* out, void* stream) {
  int rc = check_spadl_frame(in);
  if (rc) return rc;
  if (in->order) return fail(SA_EINVAL, "_extra_from_passes reads rows in input order: order must be NULL");
  if (m < 0 || m > in->n || (m > 0 && !parents)) return fail(SA_EINVAL, "bad parents");
  if (in->n == 0) return SA_OK;
  if (!dest || !spadl_out_ok(out)) return fail(SA_EINVAL, "null dest or output column");
  hipLaunchKernelGGL(atomic_passes_emit_kernel, dim3((unsigned)n_blocks(in->n + m)), dim3(AC_THREADS), 0,
                     (hipStream_t)stream, *in, parents, m, dest, *out);
  return check_launch("atomic_passes_emit_kernel");
}

static int check_dribble_rule(double min2, double max2, double max_dt) {
  if (!(min2 >= 0) || !(max2 >= 0) || max_dt != max_dt) return fail(SA_EINVAL, "bad dribble thresholds");
  return SA_OK;
}

extern "C" int sa_dribble_count(const sa_spadl_frame* in, double min_len2, double max_len2, double max_dt,
                                const double* action_id, void* scratch, uint8_t* flags, int64_t* n_out,
                                int64_t* n_misplaced, void* stream) {
  int rc = check_spadl_frame(in);
  if (rc || (rc = check_dribble_rule(min_len2, max_len2, max_dt))) return rc;
  if (in->order) return fail(SA_EINVAL, "_add_dribbles reads rows in input order: order must be NULL");
  if (!n_out || (in->n > 0 && !scratch)) return fail(SA_EINVAL, "null scratch or n_out");
  *n_out = 0;
  if (n_misplaced) *n_misplaced = action_id ? 0 : -1;
  if (in->n == 0) return SA_OK;
  hipStream_t st = (hipStream_t)stream;
  const int64_t nb = n_blocks(in->n);
  int64_t* bsum = (int64_t*)scratch;  // [nb] block counts -> prefix, [nb] total, [nb + 1] misplaced
  if ((rc = check_hip(hipMemsetAsync(bsum + nb + 1, 0, sizeof(int64_t), st), "memset"))) return rc;
  hipLaunchKernelGGL(dribble_count_kernel, dim3((unsigned)nb), dim3(AC_THREADS), 0, st, *in,
                     DribbleRule{min_len2, max_len2, max_dt}, action_id, bsum,
                     (unsigned long long*)(bsum + nb + 1), flags);
  if ((rc = check_launch("dribble_count_kernel"))) return rc;
  hipLaunchKernelGGL(atomic_scan_kernel, dim3(1), dim3(SC_THREADS), 0, st, bsum, nb);
  if ((rc = check_launch("atomic_scan_kernel"))) return rc;
  int64_t res[2] = {0, 0};
  if ((rc = check_hip(hipMemcpyAsync(res, bsum + nb, sizeof(res), hipMemcpyDeviceToHost, st), "copy n_out")))
    return rc;
  if ((rc = check_hip(hipStreamSynchronize(st), "hipStreamSynchronize"))) return rc;
  *n_out = res[0];
  if (n_misplaced && action_id) *n_misplaced = res[1];
  return SA_OK;
}

extern "C" int sa_dribble_emit(const sa_spadl_frame* in, double min_len2, double max_len2, double max_dt,
                               const void* scratch, const int64_t* dest, const sa_spadl_out* out,
                               void* stream) {
  int rc = check_spadl_frame(in);
  if (rc || (rc = check_dribble_rule(min_len2, max_len2, max_dt))) return rc;
  if (in->order) return fail(SA_EINVAL, "_add_dribbles reads rows in input order: order must be NULL");
  if (in->n == 0) return SA_OK;
  if (!scratch || !out || !out->time_seconds || !out->start_x || !out->start_y || !out->end_x ||
      !out->end_y || !out->game || !out->team || !out->player || !out->event || !out->period_id ||
      !out->type_id || !out->result_id || !out->bodypart_id || !out->src)
    return fail(SA_EINVAL, "null scratch or output column");
  const int64_t nb = n_blocks(in->n);
  hipLaunchKernelGGL(dribble_emit_kernel, dim3((unsigned)nb), dim3(AC_THREADS), 0, (hipStream_t)stream, *in,
                     DribbleRule{min_len2, max_len2, max_dt}, (const int64_t*)scratch, dest, *out);
  return check_launch("dribble_emit_kernel");
}

extern "C" int sa_segment_offsets(const int32_t* key, int64_t n, int64_t n_segments, int64_t* seg_off,
                                  void* stream) {
  if (n < 0 || n_segments < 0 || !seg_off || (n > 0 && !key)) return fail(SA_EINVAL, "bad segment offsets args");
  const int64_t threads = n > 0 ? n : 1;
  hipLaunchKernelGGL(segment_offsets_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, key, n, n_segments, seg_off);
  return check_launch("segment_offsets_kernel");
}
