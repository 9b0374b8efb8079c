// Expected Threat (xT) kernels for gfx950: binning + counts, normalisation, value
// iteration, interpolated surface and rate.  Reference: socceraction/xthreat.py.
//
// Binning reproduces `_get_cell_indexes` bit for bit: (x / 105) * l in f64 (divide
// THEN multiply), truncation toward zero like numpy's int64 cast, clip to [0, l-1].
// The value iteration keeps the reference's summation order exactly: for each cell r
// total = sum_{c=0}^{C-1} T[r,c] * x[c], accumulated left to right in f64 with
// separate multiply and add (xthreat.py:306-312), so iterates and the iteration count
// are bit-identical to the pandas path.  T is kept transposed (Tt[c*C + r]) so that at
// step c the lanes of a wave read one contiguous run of rows (coalesced).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <vector>

#include "sa_common.h"
#include "sa_internal.h"

#ifndef SA_XC_UC
#define SA_XC_UC 8  // count pass from cell codes: codes per thread per pass, all loaded first
#endif
#ifndef SA_XT_BANDS
#define SA_XT_BANDS 1  // grids the band-owned count holds (sa_xt_large.hip); 0: XC_VEC / XC_GLOBAL atomics
#endif
#ifndef SA_XT_COMPACT
#define SA_XT_COMPACT 1  // large-grid solve over the compact count rows (0: xt_iter_kernel on the dense rows)
#endif
#ifndef SA_XT_WIDE
#define SA_XT_WIDE 1  // C <= 197: XC_WIDE count pass (0: the 32k-action XC_SMALL workgroups)
#endif

namespace sa {

// ---------------------------------------------------------------------------------------------
// Count pass.  XC_SMALL: per-workgroup LDS histograms (u32 for the three C-vectors, the C x C
// transition counts packed two u16 per word), flushed with one global atomic per non-zero
// bin; a workgroup handles <= 65535 actions so a u16 bin cannot overflow.  XC_VEC (C up to
// ~10k, e.g. 105 x 68): only the three C-vectors in LDS -- every move hits move[start], so
// global atomics there serialise on a few thousand hot addresses -- and the sparse C x C
// transition counts as global atomics.  XC_GLOBAL: global atomics for everything.
// XC_WIDE (C <= 197, e.g. 16 x 12): all 3C + C*C bins as u32 in one 1024-thread workgroup's LDS
// (150 KB at C = 192, one workgroup per CU), each workgroup counting one contiguous chunk of
// the actions -- 16 waves per CU keep the loads in flight, and the C*C flush happens once per
// CU instead of once per 32k actions (16M actions: 472 -> see DESIGN.md).
constexpr int XT_THREADS = 256;
constexpr int XT_WIDE_THREADS = 1024;
constexpr int XT_SMALL_ACTS = 32768;  // actions per workgroup in XC_SMALL / XC_VEC
enum { XC_GLOBAL = 0, XC_VEC = 1, XC_SMALL = 2, XC_WIDE = 3 };

template <int MODE>
__device__ __forceinline__ void count_one(const XtAct& a, int C, uint32_t* hs, uint32_t* hg, uint32_t* hm,
                                          uint32_t* ht, unsigned long long* shot,
                                          unsigned long long* goal, unsigned long long* move,
                                          int32_t* trans, int32_t& bad) {
  constexpr bool SMALL = MODE == XC_SMALL, WIDE = MODE == XC_WIDE, VEC = MODE != XC_GLOBAL;
  if (a.cls == XT_CELL_SHOT) {
    if (a.snan) return;  // _count drops NaN rows (xthreat.py:60-61)
    if (!a.sfin) {
      bad |= XT_ERRB_SHOT;
      return;
    }
    SA_DGUARD(a.cs >= 0 && a.cs < C, a.cs, return);
    if (VEC) {
      atomicAdd(&hs[a.cs], 1u);
      if (a.succ) atomicAdd(&hg[a.cs], 1u);
    } else {
      atomicAdd(&shot[a.cs], 1ull);
      if (a.succ) atomicAdd(&goal[a.cs], 1ull);
    }
  } else if (a.cls == XT_CELL_MOVE) {
    if (a.snan) {  // dropped by action_prob's _count; move_transition_matrix's cast raises
      bad |= XT_ERRB_MOVE_OTHER;
      return;
    }
    if (!a.sfin) {
      bad |= XT_ERRB_MOVE_START;
      return;
    }
    SA_DGUARD(a.cs >= 0 && a.cs < C, a.cs, return);
    if (VEC)
      atomicAdd(&hm[a.cs], 1u);
    else
      atomicAdd(&move[a.cs], 1ull);
    if (!a.efin) {
      bad |= XT_ERRB_MOVE_OTHER;  // only move_transition_matrix reads the end coordinates
      return;
    }
    if (a.succ) {
      SA_DGUARD(a.ce >= 0 && a.ce < C, a.ce, return);
      const int64_t k = (int64_t)a.cs * C + a.ce;
      if (SMALL)
        atomicAdd(&ht[k >> 1], (k & 1) ? 0x10000u : 1u);
      else if (WIDE)
        atomicAdd(&ht[k], 1u);
      else
        atomicAdd(&trans[k], 1);
    }
  }
}

// CELLS = false: reads the actions' coordinates and ids (34 B per action) and may write each
// action's rate operand (`codes`, sa_xt_count_codes).  CELLS = true: reads the 4-B cell codes a
// producer wrote (sa_xt_count_cells).
template <int MODE, bool CELLS>
__global__ __launch_bounds__(XT_WIDE_THREADS) void xt_count_kernel(sa_actions A, const uint32_t* __restrict__ cells,
                                                                  int64_t n, int l, int w,
                                                                  unsigned long long* __restrict__ shot,
                                                                  unsigned long long* __restrict__ goal,
                                                                  unsigned long long* __restrict__ move,
                                                                  int32_t* __restrict__ trans,
                                                                  int32_t* __restrict__ err, int64_t chunk,
                                                                  uint32_t* __restrict__ codes) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const int C = l * w;
  const sa_frame& F = A.frames[0];
  uint32_t* hs = lds;          // [C]
  uint32_t* hg = lds + C;      // [C]
  uint32_t* hm = lds + 2 * C;  // [C]
  uint32_t* ht = lds + 3 * C;  // SMALL: [(C*C+1)/2] packed u16 pairs; WIDE: [C*C] u32
  constexpr bool SMALL = MODE == XC_SMALL, WIDE = MODE == XC_WIDE, VEC = MODE != XC_GLOBAL;
  int64_t begin, end, stride;
  if (VEC) {
    const int tw = SMALL ? (C * C + 1) / 2 : (WIDE ? C * C : 0);
    for (int k = threadIdx.x; k < 3 * C + tw; k += blockDim.x) lds[k] = 0;
    __syncthreads();
    begin = (int64_t)blockIdx.x * chunk + threadIdx.x;
    end = min(n, (int64_t)(blockIdx.x + 1) * chunk);
    stride = blockDim.x;
  } else {
    begin = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    end = n;
    stride = (int64_t)gridDim.x * blockDim.x;
  }
  int32_t bad = 0;
  // XC_U actions per thread per pass, every load issued before any is used (the loop is
  // otherwise one HBM round trip per action); rows past `end` are clamped and skipped
  constexpr int XC_U = CELLS ? SA_XC_UC : 4;
  for (int64_t j0 = begin; j0 < end; j0 += XC_U * stride) {
    XtAct act[XC_U];
    if (CELLS) {
      uint32_t cv[XC_U];
      const bool c16 = xt_c16(C);  // 16-bit codes (grids of <= SA_XT_CELLS16_MAX_C cells)
#pragma unroll
      for (int u = 0; u < XC_U; ++u) {
        const int64_t j = j0 + u * stride < end ? j0 + u * stride : end - 1;
        cv[u] = c16 ? (uint32_t)reinterpret_cast<const uint16_t*>(cells)[j] : cells[j];
      }
#pragma unroll
      for (int u = 0; u < XC_U; ++u) {
        act[u] = c16 ? decode_cell16(cv[u], C) : decode_cell(cv[u]);
        if (j0 + u * stride >= end) act[u].cls = 0;
      }
    } else {
      int tt[XC_U], rr[XC_U];
      double sx[XC_U], sy[XC_U], ex[XC_U], ey[XC_U];
#pragma unroll
      for (int u = 0; u < XC_U; ++u) {
        const int64_t j = j0 + u * stride < end ? j0 + u * stride : end - 1;
        tt[u] = j0 + u * stride < end ? F.type_id[j] : -1;
        rr[u] = F.result_id[j];
        sx[u] = F.c0[j];
        sy[u] = F.c1[j];
        ex[u] = F.c2[j];
        ey[u] = F.c3[j];
      }
#pragma unroll
      for (int u = 0; u < XC_U; ++u) {
        const int t = tt[u], r = rr[u];
        if (codes && t >= 0) codes[j0 + u * stride] = rate_code(t, r, sx[u], sy[u], ex[u], ey[u], l, w);
        XtAct& a = act[u];
        a.cls = t == T_SHOT ? XT_CELL_SHOT : (is_move(t) ? XT_CELL_MOVE : 0u);
        a.succ = r == R_SUCCESS;
        a.snan = isnan(sx[u]) || isnan(sy[u]);
        a.sfin = isfinite(sx[u]) && isfinite(sy[u]);
        a.efin = isfinite(ex[u]) && isfinite(ey[u]);
        a.cs = (a.cls && a.sfin) ? flat_index(sx[u], sy[u], l, w) : 0;
        a.ce = (a.cls == XT_CELL_MOVE && a.succ && a.efin) ? flat_index(ex[u], ey[u], l, w) : 0;
      }
    }
#pragma unroll
    for (int u = 0; u < XC_U; ++u) count_one<MODE>(act[u], C, hs, hg, hm, ht, shot, goal, move, trans, bad);
  }
  if (bad) atomicOr(err, bad);
  if (VEC) {
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      if (hs[c]) atomicAdd(&shot[c], (unsigned long long)hs[c]);
      if (hg[c]) atomicAdd(&goal[c], (unsigned long long)hg[c]);
      if (hm[c]) atomicAdd(&move[c], (unsigned long long)hm[c]);
    }
  }
  if (WIDE) {
    for (int k = threadIdx.x; k < C * C; k += blockDim.x) {
      const uint32_t v = ht[k];
      if (v) atomicAdd(&trans[k], (int32_t)v);
    }
  }
  if (SMALL) {
    const int tw = (C * C + 1) / 2;
    for (int k = threadIdx.x; k < tw; k += blockDim.x) {
      const uint32_t v = ht[k];
      if (v & 0xFFFFu) atomicAdd(&trans[2 * k], (int32_t)(v & 0xFFFFu));
      if (v >> 16) atomicAdd(&trans[2 * k + 1], (int32_t)(v >> 16));
    }
  }
}

// Cell codes alone (the binning of the count pass): one thread per 4 actions, 16-B stores.
__global__ __launch_bounds__(256) void xt_cells_kernel(sa_actions A, int l, int w, uint32_t* __restrict__ cells) {
  const int64_t j0 = 4 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (j0 >= A.n) return;
  const sa_frame& F = A.frames[0];
  u32x4 v = {0, 0, 0, 0};
  const bool c16 = xt_c16(l * w);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t j = j0 + q < A.n ? j0 + q : A.n - 1;
    v[q] = c16 ? xt_cell_code16(F.type_id[j], F.result_id[j], F.c0[j], F.c1[j], F.c2[j], F.c3[j], l, w)
               : xt_cell_code(F.type_id[j], F.result_id[j], F.c0[j], F.c1[j], F.c2[j], F.c3[j], l, w);
  }
  if (c16) {
    uint16_t* c2 = reinterpret_cast<uint16_t*>(cells);
    for (int q = 0; j0 + q < A.n && q < 4; ++q) c2[j0 + q] = (uint16_t)v[q];
  } else if (j0 + 4 <= A.n) {
    *reinterpret_cast<u32x4*>(cells + j0) = v;
  } else {
    for (int q = 0; j0 + q < A.n; ++q) cells[j0 + q] = v[q];
  }
}

// ---------------------------------------------------------------------------------------------
// Normalisation (xthreat.py:70-98, 144-174, 177-218).
__global__ void xt_prob_kernel(const unsigned long long* __restrict__ shot,
                               const unsigned long long* __restrict__ goal,
                               const unsigned long long* __restrict__ move, int C,
                               double* __restrict__ mats, double* __restrict__ gs,
                               double* __restrict__ pmove) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double s = (double)shot[c], g = (double)goal[c], m = (double)move[c];
  const double tot = m + s;
  const double ps = s != 0.0 ? g / s : 0.0;  // _safe_divide
  const double pshot = tot != 0.0 ? s / tot : 0.0;
  const double pm = tot != 0.0 ? m / tot : 0.0;
  mats[c] = ps;
  mats[C + c] = pshot;
  mats[2 * C + c] = pm;
  gs[c] = ps * pshot;
  pmove[c] = pm;
}

// Tt[e*C + s] = trans[s*C + e] / move[s]  (32x32 LDS-tiled transpose; rows with no moves stay 0)
__global__ __launch_bounds__(256) void xt_transpose_kernel(const int32_t* __restrict__ trans,
                                                           const unsigned long long* __restrict__ move,
                                                           int C, double* __restrict__ Tt) {
  __shared__ double tile[32][33];
  const int s0 = blockIdx.y * 32, e0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int k = ty; k < 32; k += 8) {
    const int s = s0 + k, e = e0 + tx;
    double v = 0.0;
    if (s < C && e < C) {
      const int32_t cnt = trans[(int64_t)s * C + e];
      v = cnt != 0 ? (double)cnt / (double)move[s] : 0.0;
    }
    tile[k][tx] = v;
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int e = e0 + k, s = s0 + tx;
    if (s < C && e < C) Tt[(int64_t)e * C + s] = tile[tx][k];
  }
}

// One value-iteration step for C rows; row r = one lane, sequential sum over c in runs of 8
// loads (~5.4 us per iteration at C = 192; see xt_solve_small_kernel for what was tried).
__device__ __forceinline__ double row_payoff(const double* __restrict__ Tt, const double* __restrict__ x,
                                             int C, int r) {
  double acc = 0.0;
  int c = 0;
  for (; c + 8 <= C; c += 8) {
    double tv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) tv[u] = Tt[(int64_t)(c + u) * C + r];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const double p = tv[u] * x[c + u];
      acc = acc + p;
    }
  }
  for (; c < C; ++c) {
    const double p = Tt[(int64_t)c * C + r] * x[c];
    acc = acc + p;
  }
  return acc;
}

constexpr int XT_SOLVE_MAX_C = SA_XT_SOLVE_MAX_C;

// Small grids (C <= XT_SOLVE_MAX_C, e.g. 16 x 12): one persistent workgroup runs every
// iteration, row r = one lane, x in LDS; Tt is the exact transposed matrix of
// xt_transpose_kernel (L2-resident).  Measured at C = 192 (scripts/xt_solve_time.py, isolated,
// 26 iterations incl. normalisation and the host sync): runs of 8 loads 0.181 ms; 32 / 64
// columns software-pipelined ahead 0.347 / 0.367 ms (more registers, fewer resident waves); all
// 16 waves streaming Tt through LDS 0.453 ms; the counts in LDS with one division per element
// 0.469 ms; the whole matrix in the registers of 512 threads 0.343 ms (and it waits for a whole
// idle CU next to the VAEP kernels: 1.49 ms in the step).
__global__ __launch_bounds__(1024) void xt_solve_small_kernel(const double* __restrict__ Tt,
                                                                 const double* __restrict__ gs,
                                                                 const double* __restrict__ pmove, int C,
                                                                 double eps, int max_iter,
                                                                 double* __restrict__ heat,
                                                                 double* __restrict__ xT_out,
                                                                 int32_t* __restrict__ n_iter) {
  __shared__ double xs[XT_SOLVE_MAX_C];
  const int r = threadIdx.x;
  if (r < C) {
    xs[r] = 0.0;
    heat[r] = 0.0;
  }
  __syncthreads();
  int it = 0;
  bool cont = true;
  while (cont && it < max_iter) {
    double nx = 0.0;
    int flag = 0;
    if (r < C) {
      const double tot = row_payoff(Tt, xs, C, r);
      const double mv = pmove[r] * tot;
      nx = gs[r] + mv;
      const double diff = nx - xs[r];
      flag = diff > eps;  // np.any(diff > eps): NaN compares False
      heat[(int64_t)(it + 1) * C + r] = nx;
    }
    cont = __syncthreads_or(flag);
    if (r < C) xs[r] = nx;
    __syncthreads();
    ++it;
  }
  if (r < C) xT_out[r] = xs[r];
  if (r == 0) *n_iter = cont ? -1 : it;
}

// Grids up to 16 x 12 (C <= XR_MAX_C = 192, the default grid): the transition matrix lives in
// registers for all iterations.  Each row is split into H parts of 192 / H columns; lane (row r,
// part h) holds T[r][h*192/H .. (h+1)*192/H) (loaded once from the exact transposed matrix;
// columns >= C and rows >= C hold +0), so a wave covers 64 / H rows.  Per iteration the part-0
// lanes run the first terms of the row's sequential sum, hand the partial sum to their part-1
// lane (a wave shuffle), which continues, and so on: the reference's left-to-right order
// (xthreat.py:306-312), each product rounded before its add (-ffp-contract=off).  Padded terms
// are +0 * +0 = +0 and leave the (non-negative) running sum unchanged, so any C <= 192 runs the
// same 192 steps.  x is double-buffered in LDS; one barrier (which also ORs the convergence
// flags) per iteration.  Nothing is read from memory after the first iteration's loads.
// SA_XR_PARTS = H: 2 (default, 96 doubles per lane, 224 VGPRs, no spills): 71 us for 26
// iterations (rocprofv3), 0.110 ms incl. normalisation + host sync; H = 1 (192 doubles, 256
// VGPRs + 150 AGPRs) 0.144 ms, H = 4 0.134 ms (profiles/r02_step_ab.md).
constexpr int XR_MAX_C = 192;
#ifndef SA_XR_PARTS
#define SA_XR_PARTS 2
#endif

template <int H>
__global__ __launch_bounds__(H * XR_MAX_C) void xt_solve_reg_kernel(const double* __restrict__ Tt,
                                                                    const double* __restrict__ gs,
                                                                    const double* __restrict__ pmove, int C,
                                                                    double eps, int max_iter,
                                                                    double* __restrict__ heat,
                                                                    double* __restrict__ xT_out,
                                                                    int32_t* __restrict__ n_iter) {
  static_assert(H == 1 || H == 2 || H == 4, "parts per row");
  constexpr int NP = XR_MAX_C / H, RW = 64 / H;  // columns per part, rows per wave
  __shared__ __attribute__((aligned(16))) double xs[2][XR_MAX_C];
  const int lane = threadIdx.x & 63;
  const int h = lane / RW;
  const int r = (int)(threadIdx.x >> 6) * RW + lane % RW;
  const bool own = h == H - 1 && r < C;  // the lane that finishes row r
  double t[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const int c = h * NP + k;
    t[k] = (r < C && c < C) ? Tt[(int64_t)c * C + r] : 0.0;
  }
  const double g = own ? gs[r] : 0.0, pm = own ? pmove[r] : 0.0;
  for (int c = threadIdx.x; c < 2 * XR_MAX_C; c += blockDim.x) (&xs[0][0])[c] = 0.0;
  if (own) heat[r] = 0.0;
  __syncthreads();
  int it = 0;
  bool cont = true;
  while (cont && it < max_iter) {
    const double* __restrict__ x = xs[it & 1] + h * NP;
    double acc = 0.0;
#pragma unroll
    for (int q = 0; q < H; ++q) {
      if (h == q) {
#pragma unroll
        for (int k = 0; k < NP; ++k) {
          const double p = t[k] * x[k];
          acc = acc + p;
        }
      }
      if (q + 1 < H) acc = __shfl(acc, q * RW + lane % RW);  // part q+1 continues part q's sum
    }
    int flag = 0;
    if (own) {
      const double mv = pm * acc;
      const double nx = g + mv;
      const double diff = nx - xs[it & 1][r];
      flag = diff > eps;  // np.any(diff > eps): NaN compares False
      heat[(int64_t)(it + 1) * C + r] = nx;
      xs[(it + 1) & 1][r] = nx;
    }
    cont = __syncthreads_or(flag);
    ++it;
  }
  if (own) xT_out[r] = xs[it & 1][r];
  if (threadIdx.x == 0) *n_iter = cont ? -1 : it;
}

// Large grids (C > XT_SOLVE_MAX_C, e.g. 105 x 68 = 7140 cells): one launch per iteration.
// The dense transition matrix is never materialised for the iteration: a workgroup owns
// XI_ROWS rows r and streams their int32 count rows trans[r*C + c] (4 B per element instead
// of 8 B of f64 T: 204 MB instead of 408 MB per iteration at 7140 cells, which then also
// stays resident in the 256 MB Infinity Cache across iterations).  T[r,c] * x[c] is formed
// exactly as the reference rounds it -- one correctly rounded division cnt / move[r], one
// multiply -- and cnt == 0 gives +0, which leaves a non-negative running sum unchanged.  So
// each loader wave compacts the non-zero columns of its rows (ballot + mbcnt, in column
// order), divides only those, and the chain lanes add each row's compacted products strictly
// left to right: the reference's sequential rounding, over nnz instead of C terms.
// 8 loader waves (2 rows each) keep XI_DEPTH chunks of XI_CH columns in flight (unconditional loads from
// clamped addresses); a fifth wave runs the 16 chains, one chunk behind the loaders (two LDS
// buffers, one barrier per chunk).  Measured at 7140 cells (profiles/r01_xt_iteration.md):
// 62 us per iteration; 4 loader waves 71 us, chains inside each loader wave without barriers
// 98 us, dense division of every element +10 us, an uncompacted chain +45 us.  flags[it] != 0 <=>
// some cell of iteration it moved by more than eps; a launch whose predecessor converged is
// a no-op.
#ifndef SA_XI_DEPTH
#define SA_XI_DEPTH 2
#endif
#ifndef SA_XI_LOADERS
#define SA_XI_LOADERS 8
#endif
#ifndef SA_XI_ROWS
#define SA_XI_ROWS 16  // rows per workgroup = chain lanes (16, 32 or 64)
#endif
#ifndef SA_XI_CH
#define SA_XI_CH 128  // columns per chunk (64 or 128)
#endif
constexpr int XI_ROWS = SA_XI_ROWS;
constexpr int XI_LOADERS = SA_XI_LOADERS;        // loader waves; one more wave runs the chains
constexpr int XI_RQ = XI_ROWS / XI_LOADERS;      // rows per loader wave
constexpr int XI_THREADS = (XI_LOADERS + 1) * 64;
constexpr int XI_CH = SA_XI_CH;        // columns per chunk = XI_NI per loader lane per row
constexpr int XI_NI = XI_CH / 64;
static_assert(XI_RQ >= 1 && XI_RQ * XI_LOADERS == XI_ROWS && XI_NI >= 1 && XI_NI * 64 == XI_CH &&
                  (XI_ROWS & (XI_ROWS - 1)) == 0 && XI_ROWS <= 64,
              "xt_iter_kernel shape");
static_assert(XI_THREADS <= 1024, "xt_iter_kernel: SA_XI_LOADERS + 1 waves must fit one workgroup");
constexpr int XI_DEPTH = SA_XI_DEPTH;  // chunks in flight per loader lane
constexpr int XI_LST = XI_CH + 1;      // list row stride (doubles): chain reads hit 16 banks

struct XiChunk {
  int32_t cnt[XI_RQ][XI_NI];  // [row q][column i]
  double xv[XI_NI];           // x[c] of column i
};

// Rows [rb, rb + nrows) of the system: `trans` points at the count row of row rb (row rb + i
// at trans + i*C), x is the full current vector, xo[i] receives the new value of row rb + i
// and *flag_out |= (some row moved by more than eps).  A non-null flag_prev == 0 (the
// previous iteration converged) makes the launch a no-op.
__global__ __launch_bounds__(XI_THREADS) void xt_iter_kernel(const int32_t* __restrict__ trans,
                                                             const unsigned long long* __restrict__ move,
                                                             const double* __restrict__ gs,
                                                             const double* __restrict__ pmove, int C,
                                                             int rb, int nrows, double eps,
                                                             const double* __restrict__ x,
                                                             double* __restrict__ xo,
                                                             const int32_t* flag_prev,
                                                             int32_t* __restrict__ flag_out) {
  if (flag_prev && __hip_atomic_load(flag_prev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
    return;
  __shared__ double list[2][XI_ROWS * XI_LST];       // compacted x, then products, per row
  __shared__ int32_t cbuf[XI_LOADERS][XI_RQ][XI_CH];  // compacted counts (loader-wave private)
  __shared__ int32_t lens[2][XI_ROWS];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r0 = blockIdx.x * XI_ROWS;  // local row index of the block's first row
  const int nch = (C + XI_CH - 1) / XI_CH;
  const int nchp = (nch + XI_DEPTH - 1) / XI_DEPTH * XI_DEPTH;
  if (wv < XI_LOADERS) {  // ---- loader waves: rows r0 + RQ*wv + q, columns k*XI_CH + 64*i + lane
    const int32_t* rowp[XI_RQ];
    double mvq[XI_RQ];
    bool rowok[XI_RQ];
#pragma unroll
    for (int q = 0; q < XI_RQ; ++q) {
      const int r = r0 + XI_RQ * wv + q;
      rowok[q] = r < nrows;
      const int rc = rowok[q] ? r : nrows - 1;
      rowp[q] = trans + (int64_t)rc * C;
      mvq[q] = (double)move[rb + rc];
    }
    auto issue = [&](XiChunk& R, int k) {  // unconditional loads from clamped addresses
#pragma unroll
      for (int i = 0; i < XI_NI; ++i) {
        const int c = k * XI_CH + 64 * i + lane;
        const int cc = c < C ? c : C - 1;
        R.xv[i] = x[cc];
#pragma unroll
        for (int q = 0; q < XI_RQ; ++q) R.cnt[q][i] = rowp[q][cc];
      }
    };
    auto stage = [&](const XiChunk& R, int k, int par) {
      double* lst = list[par];
#pragma unroll
      for (int q = 0; q < XI_RQ; ++q) {
        const int row = XI_RQ * wv + q;
        int base = 0;
#pragma unroll
        for (int i = 0; i < XI_NI; ++i) {  // compact the non-zero columns, in column order
          const bool cok = k * XI_CH + 64 * i + lane < C;
          const int32_t cnt = (cok && rowok[q]) ? R.cnt[q][i] : 0;
          const uint64_t m = __ballot(cnt != 0);
          const int pos = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
          if (cnt != 0) {
            lst[row * XI_LST + pos] = R.xv[i];
            cbuf[wv][q][pos] = cnt;
          }
          base += __popcll(m);
        }
        for (int e = lane; e < base; e += 64) {  // T[r, c] * x[c] on the compacted entries
          const double tv = (double)cbuf[wv][q][e] / mvq[q];
          lst[row * XI_LST + e] = tv * lst[row * XI_LST + e];
        }
        if (lane == 0) lens[par][row] = base;
      }
    };
    // a multiple of XI_DEPTH chunks with no data-dependent branches around the loads; the empty
    // asm keeps each prefetch where it is issued (the compiler otherwise sinks it next to its
    // use and the wait counts drain every load); chunks past C are empty
    XiChunk R[XI_DEPTH];
#pragma unroll
    for (int d = 0; d < XI_DEPTH; ++d) issue(R[d], d);
    asm volatile("" ::: "memory");
    for (int k0 = 0; k0 < nchp; k0 += XI_DEPTH) {
#pragma unroll
      for (int d = 0; d < XI_DEPTH; ++d) {
        const int k = k0 + d;
        stage(R[d], k, k & 1);
        issue(R[d], k + XI_DEPTH);  // past the end: clamped, harmless re-reads of column C-1
        asm volatile("" ::: "memory");
        __syncthreads();
      }
    }
  } else {  // ---- chain wave: lane r adds its row's compacted products strictly left to right
    double acc = 0.0;
    const int r = lane & (XI_ROWS - 1);
    for (int k = 0; k < nchp; ++k) {
      __syncthreads();
      const int par = k & 1;
      const int len = lens[par][r];
      int mx = 0;
#pragma unroll
      for (int u = 0; u < XI_ROWS; ++u) mx = max(mx, lens[par][u]);
      const double* lst = list[par] + r * XI_LST;
      for (int j = 0; j < mx; j += 8) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = lst[(j + u) & (XI_CH - 1)];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const double p = (j + u < len) ? v[u] : 0.0;
          acc = acc + p;
        }
      }
    }
    if (lane < XI_ROWS && r0 + r < nrows) {
      const int rr = rb + r0 + r;  // global row
      const double mv = pmove[rr] * acc;
      const double nx = gs[rr] + mv;
      xo[r0 + r] = nx;
      if ((nx - x[rr]) > eps) atomicOr(flag_out, 1);  // np.any(diff > eps): NaN is False
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Interpolated surface: grid[r*L + h] = B(xs[h], ys[r]) — piecewise bilinear through the cell
// centres (interp2d kind='linear' on a regular grid), clamped to the centre hull.
__device__ __forceinline__ void bracket(const double* __restrict__ c, int m, double q, int& i, double& t) {
  q = q < c[0] ? c[0] : (q > c[m - 1] ? c[m - 1] : q);
  int lo = 0, hi = m - 1;  // c[lo] <= q <= c[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (c[mid] <= q)
      lo = mid;
    else
      hi = mid;
  }
  i = lo;
  t = (q - c[lo]) / (c[lo + 1] - c[lo]);
}

__global__ void xt_interp_kernel(const double* __restrict__ xT, const double* __restrict__ cx,
                                 const double* __restrict__ cy, int l, int w,
                                 const double* __restrict__ xs, int L, const double* __restrict__ ys,
                                 int W, double* __restrict__ grid) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= (int64_t)L * W) return;
  const int r = (int)(k / L), h = (int)(k % L);
  const double xq = xs[h], yq = ys[r];
  int i, j;
  double tx, ty;
  bracket(cx, l, xq, i, tx);
  bracket(cy, w, yq, j, ty);
  const double z00 = xT[j * l + i], z01 = xT[j * l + i + 1];
  const double z10 = xT[(j + 1) * l + i], z11 = xT[(j + 1) * l + i + 1];
  const double ux = 1.0 - tx, uy = 1.0 - ty;
  grid[k] = (ux * z00 + tx * z01) * uy + (ux * z10 + tx * z11) * ty;
}

// The interpolated surface's node brackets, one table entry per node column h (x axis, entries
// [0, L)) and node row r (y axis, entries [L, L + W)): the (i, tx) / (j, ty) xt_interp_kernel
// computes for that node, by the same bracket().  With them the rate evaluates a node's value
// in the same operations as the grid -- bit for bit -- without the L x W grid.
__global__ void xt_axes_kernel(const double* __restrict__ cx, const double* __restrict__ cy, int l, int w,
                               const double* __restrict__ xs, int L, const double* __restrict__ ys, int W,
                               int32_t* __restrict__ idx, double* __restrict__ frac) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= L + W) return;
  int i;
  double t;
  if (k < L)
    bracket(cx, l, xs[k], i, t);
  else
    bracket(cy, w, ys[k - L], i, t);
  idx[k] = i;
  frac[k] = t;
}

// B(xs[h], ys[r]) of node k = r * L + h: xt_interp_kernel's expression on the (w x l) surface
__device__ __forceinline__ double node_value(const double* __restrict__ xT, int l, int L, int k,
                                             const int32_t* __restrict__ idx, const double* __restrict__ frac) {
  const int r = k / L, h = k - r * L;
  const int i = idx[h], j = idx[L + r];
  const double tx = frac[h], ty = frac[L + r];
  const double z00 = xT[j * l + i], z01 = xT[j * l + i + 1];
  const double z10 = xT[(j + 1) * l + i], z11 = xT[(j + 1) * l + i + 1];
  const double ux = 1.0 - tx, uy = 1.0 - ty;
  return (ux * z00 + tx * z01) * uy + (ux * z10 + tx * z11) * ty;
}

// rate (xthreat.py:408-465): successful moves get grid[end] - grid[start], others NaN.
__device__ __forceinline__ double rate_one(int t, int r, double sx, double sy, double ex, double ey,
                                           const double* __restrict__ grid, int L, int W, int32_t& bad) {
  double v = __builtin_nan("");
  if (is_move(t) && r == R_SUCCESS) {
    if (!isfinite(sx) || !isfinite(sy) || !isfinite(ex) || !isfinite(ey)) {
      bad = 4;
    } else {
      const int s = flat_index(sx, sy, L, W), e = flat_index(ex, ey, L, W);
      SA_DGUARD(s >= 0 && s < L * W && e >= 0 && e < L * W, s, return v);
      v = grid[e] - grid[s];
    }
  }
  return v;
}

// A thread rates 2 consecutive actions: 16-B loads of each coordinate column, 2-B loads of the
// ids and one 16-B store (vec: host-checked alignment), so a wave moves 1 KiB per instruction
// instead of 512 B (f64) or 64 B (ids).
__global__ __launch_bounds__(256) void xt_rate_kernel(sa_actions A, const double* __restrict__ grid,
                                                      int L, int W, double* __restrict__ out,
                                                      int32_t* __restrict__ err, int vec) {
  const int64_t j0 = 2 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (j0 >= A.n) return;
  const sa_frame& F = A.frames[0];
  int32_t bad = 0;
  if (vec && j0 + 1 < A.n) {
    const f64x2 sx = *reinterpret_cast<const f64x2*>(F.c0 + j0);
    const f64x2 sy = *reinterpret_cast<const f64x2*>(F.c1 + j0);
    const f64x2 ex = *reinterpret_cast<const f64x2*>(F.c2 + j0);
    const f64x2 ey = *reinterpret_cast<const f64x2*>(F.c3 + j0);
    const uint32_t ty = *reinterpret_cast<const uint16_t*>(F.type_id + j0);
    const uint32_t rs = *reinterpret_cast<const uint16_t*>(F.result_id + j0);
    f64x2 v;
    v[0] = rate_one(ty & 0xFF, rs & 0xFF, sx[0], sy[0], ex[0], ey[0], grid, L, W, bad);
    v[1] = rate_one(ty >> 8, rs >> 8, sx[1], sy[1], ex[1], ey[1], grid, L, W, bad);
    __builtin_nontemporal_store(v, reinterpret_cast<f64x2*>(out + j0));
  } else {
    for (int64_t j = j0; j < j0 + 2 && j < A.n; ++j)
      out[j] = rate_one(F.type_id[j], F.result_id[j], F.c0[j], F.c1[j], F.c2[j], F.c3[j], grid, L, W, bad);
  }
  if (bad && err) atomicOr(err, bad);
}

// rate(use_interpolation=True) from the (w x l) surface and the node tables (sa_xt_rate_interp):
// xt_rate_kernel's layout (2 actions per thread, 16-B loads and store), each node value evaluated
// in place (node_value) instead of gathered from the 5.7 MB L x W grid.
__device__ __forceinline__ double rate_interp_one(int t, int r, double sx, double sy, double ex, double ey,
                                                  const double* __restrict__ xT, int l, int L, int W,
                                                  const int32_t* __restrict__ idx,
                                                  const double* __restrict__ frac, int32_t& bad) {
  double v = __builtin_nan("");
  if (is_move(t) && r == R_SUCCESS) {
    if (!isfinite(sx) || !isfinite(sy) || !isfinite(ex) || !isfinite(ey)) {
      bad = 4;
    } else {
      const int s = flat_index(sx, sy, L, W), e = flat_index(ex, ey, L, W);
      SA_DGUARD(s >= 0 && s < L * W && e >= 0 && e < L * W, s, return v);
      v = node_value(xT, l, L, e, idx, frac) - node_value(xT, l, L, s, idx, frac);
    }
  }
  return v;
}

__global__ __launch_bounds__(256) void xt_rate_interp_kernel(sa_actions A, const double* __restrict__ xT, int l,
                                                             int L, int W, const int32_t* __restrict__ idx,
                                                             const double* __restrict__ frac,
                                                             double* __restrict__ out, int32_t* __restrict__ err,
                                                             int vec) {
  const int64_t j0 = 2 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (j0 >= A.n) return;
  const sa_frame& F = A.frames[0];
  int32_t bad = 0;
  if (vec && j0 + 1 < A.n) {
    const f64x2 sx = *reinterpret_cast<const f64x2*>(F.c0 + j0);
    const f64x2 sy = *reinterpret_cast<const f64x2*>(F.c1 + j0);
    const f64x2 ex = *reinterpret_cast<const f64x2*>(F.c2 + j0);
    const f64x2 ey = *reinterpret_cast<const f64x2*>(F.c3 + j0);
    const uint32_t ty = *reinterpret_cast<const uint16_t*>(F.type_id + j0);
    const uint32_t rs = *reinterpret_cast<const uint16_t*>(F.result_id + j0);
    f64x2 v;
    v[0] = rate_interp_one(ty & 0xFF, rs & 0xFF, sx[0], sy[0], ex[0], ey[0], xT, l, L, W, idx, frac, bad);
    v[1] = rate_interp_one(ty >> 8, rs >> 8, sx[1], sy[1], ex[1], ey[1], xT, l, L, W, idx, frac, bad);
    __builtin_nontemporal_store(v, reinterpret_cast<f64x2*>(out + j0));
  } else {
    for (int64_t j = j0; j < j0 + 2 && j < A.n; ++j)
      out[j] = rate_interp_one(F.type_id[j], F.result_id[j], F.c0[j], F.c1[j], F.c2[j], F.c3[j], xT, l, L, W,
                               idx, frac, bad);
  }
  if (bad && err) atomicOr(err, bad);
}

// The same rate with the (w x l) surface and the node tables staged in LDS (the 105 x 68 surface
// and its 1050 + 680 node brackets: 78 KB): persistent workgroups load them once, then stream the
// actions two pairs per thread per pass (every load before the first store), so every node value
// is eight LDS reads instead of a chain of L2 gathers.  Same node_value operations: bit-identical.
// 16M actions: 0.145 ms (42 B/action: 4.6 TB/s) vs 0.32 ms for L2 gathers of the node tables and
// 0.235 ms for gathers from the materialised 1050 x 680 grid; a software-pipelined loop (next
// pass's loads before this pass's node values) and 4 pairs per pass were not faster
// (profiles/r03_xt_rate_interp_ab.md).
#ifndef SA_XRI_THREADS
#define SA_XRI_THREADS 1024  // 16 waves per CU (82 VGPRs); 512: 0.157 ms, 1024: 0.145 ms per 16M actions
#endif
#ifndef SA_XRI_U
#define SA_XRI_U 2
#endif
#ifndef SA_XRI_BPC
#define SA_XRI_BPC 4  // workgroups per CU in the grid (one resident at a time): 1 / 2 / 4 / 8 / 16: 0.156 / 0.150 / 0.147 / 0.160 / 0.185 ms
#endif
constexpr int XRI_THREADS = SA_XRI_THREADS;
static_assert(XRI_THREADS % 64 == 0 && XRI_THREADS <= 1024 && SA_XRI_U >= 1 && SA_XRI_BPC >= 1,
              "xt_rate_interp_lds_kernel shape (SA_XRI_THREADS / SA_XRI_U / SA_XRI_BPC)");
constexpr size_t XRI_LDS_MAX = 78 * 1024;

__device__ __forceinline__ void rate_interp_pair(const sa_frame& F, int64_t n, int64_t j0, int vec,
                                                 const double* __restrict__ xT, int l, int L, int W,
                                                 const int32_t* __restrict__ idx, const double* __restrict__ frac,
                                                 double* __restrict__ out, int32_t& bad) {
  if (vec && j0 + 1 < n) {
    const f64x2 sx = *reinterpret_cast<const f64x2*>(F.c0 + j0);
    const f64x2 sy = *reinterpret_cast<const f64x2*>(F.c1 + j0);
    const f64x2 ex = *reinterpret_cast<const f64x2*>(F.c2 + j0);
    const f64x2 ey = *reinterpret_cast<const f64x2*>(F.c3 + j0);
    const uint32_t ty = *reinterpret_cast<const uint16_t*>(F.type_id + j0);
    const uint32_t rs = *reinterpret_cast<const uint16_t*>(F.result_id + j0);
    f64x2 v;
    v[0] = rate_interp_one(ty & 0xFF, rs & 0xFF, sx[0], sy[0], ex[0], ey[0], xT, l, L, W, idx, frac, bad);
    v[1] = rate_interp_one(ty >> 8, rs >> 8, sx[1], sy[1], ex[1], ey[1], xT, l, L, W, idx, frac, bad);
    __builtin_nontemporal_store(v, reinterpret_cast<f64x2*>(out + j0));
  } else {
    for (int64_t j = j0; j < j0 + 2 && j < n; ++j)
      out[j] = rate_interp_one(F.type_id[j], F.result_id[j], F.c0[j], F.c1[j], F.c2[j], F.c3[j], xT, l, L, W, idx,
                               frac, bad);
  }
}

__global__ __launch_bounds__(XRI_THREADS) void xt_rate_interp_lds_kernel(sa_actions A, const double* __restrict__ xT,
                                                                        int l, int w, int L, int W,
                                                                        const int32_t* __restrict__ idx,
                                                                        const double* __restrict__ frac,
                                                                        double* __restrict__ out,
                                                                        int32_t* __restrict__ err, int vec) {
  extern __shared__ __attribute__((aligned(16))) double xri_lds[];
  double* sxT = xri_lds;                                        // [w * l]
  double* sfrac = sxT + w * l;                                  // [L + W]
  int32_t* sidx = reinterpret_cast<int32_t*>(sfrac + (L + W));  // [L + W]
  for (int k = threadIdx.x; k < w * l; k += blockDim.x) sxT[k] = xT[k];
  for (int k = threadIdx.x; k < L + W; k += blockDim.x) {
    sfrac[k] = frac[k];
    sidx[k] = idx[k];
  }
  __syncthreads();
  const sa_frame& F = A.frames[0];
  const int64_t n = A.n, pairs = (n + 1) / 2, stride = (int64_t)gridDim.x * blockDim.x;
  int32_t bad = 0;
  constexpr int U = SA_XRI_U;  // pairs per thread per pass, every load issued before the first store
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < pairs; p += U * stride) {
    if (vec && 2 * (p + (U - 1) * stride) + 1 < n) {
      f64x2 sx[U], sy[U], ex[U], ey[U];
      uint32_t ty[U], rs[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t j0 = 2 * (p + u * stride);
        sx[u] = *reinterpret_cast<const f64x2*>(F.c0 + j0);
        sy[u] = *reinterpret_cast<const f64x2*>(F.c1 + j0);
        ex[u] = *reinterpret_cast<const f64x2*>(F.c2 + j0);
        ey[u] = *reinterpret_cast<const f64x2*>(F.c3 + j0);
        ty[u] = *reinterpret_cast<const uint16_t*>(F.type_id + j0);
        rs[u] = *reinterpret_cast<const uint16_t*>(F.result_id + j0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        f64x2 v;
        v[0] = rate_interp_one(ty[u] & 0xFF, rs[u] & 0xFF, sx[u][0], sy[u][0], ex[u][0], ey[u][0], sxT, l, L, W,
                               sidx, sfrac, bad);
        v[1] = rate_interp_one(ty[u] >> 8, rs[u] >> 8, sx[u][1], sy[u][1], ex[u][1], ey[u][1], sxT, l, L, W, sidx,
                               sfrac, bad);
        __builtin_nontemporal_store(v, reinterpret_cast<f64x2*>(out + 2 * (p + u * stride)));
      }
    } else {
      for (int u = 0; u < U && p + u * stride < pairs; ++u)
        rate_interp_pair(F, n, 2 * (p + u * stride), vec, sxT, l, L, W, sidx, sfrac, out, bad);
    }
  }
  if (bad && err) atomicOr(err, bad);
}

// rate(use_interpolation=True) from the u64 node operands the count pass wrote (rate_icode,
// sa_xt_count_bucket): xt_rate_interp_lds_kernel's LDS-staged surface and node tables and its
// node_value operations -- bit-identical values, NaN pattern and error bit 4 -- reading 8 B per
// action instead of the 34 B of coordinates and ids.  A thread rates 2 consecutive actions per
// pass (one 16-B code load, one 16-B store), U pairs per pass, every load before the stores.
// The sets (a fit's device batches, XRI_MAX_SETS per launch) are rated one after the other by
// the whole grid, the surface staged once: one launch per fit instead of one per batch.
constexpr int XRI_MAX_SETS = 16;
struct XriSets {
  int n;
  const uint64_t* codes[XRI_MAX_SETS];
  double* out[XRI_MAX_SETS];
  int64_t cnt[XRI_MAX_SETS];
};

__global__ __launch_bounds__(XRI_THREADS) void xt_rate_icodes_lds_kernel(XriSets sets, const double* __restrict__ xT,
                                                                        int l, int w, int L, int W,
                                                                        const int32_t* __restrict__ idx,
                                                                        const double* __restrict__ frac,
                                                                        int32_t* __restrict__ err) {
  extern __shared__ __attribute__((aligned(16))) double xri_lds[];
  double* sxT = xri_lds;                                        // [w * l]
  double* sfrac = sxT + w * l;                                  // [L + W]
  int32_t* sidx = reinterpret_cast<int32_t*>(sfrac + (L + W));  // [L + W]
  for (int k = threadIdx.x; k < w * l; k += blockDim.x) sxT[k] = xT[k];
  for (int k = threadIdx.x; k < L + W; k += blockDim.x) {
    sfrac[k] = frac[k];
    sidx[k] = idx[k];
  }
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int32_t bad = 0;
  auto one = [&](uint64_t c) -> double {
    if (c == XT_ICODE_NAN) return __builtin_nan("");
    if (c == XT_ICODE_BAD) {
      bad = 4;
      return __builtin_nan("");
    }
    const int s = (int)(uint32_t)c, e = (int)(c >> 32);
    SA_DGUARD(s >= 0 && s < L * W && e >= 0 && e < L * W, s, return __builtin_nan(""));
    return node_value(sxT, l, L, e, sidx, sfrac) - node_value(sxT, l, L, s, sidx, sfrac);
  };
  constexpr int U = SA_XRI_U;
  for (int q = 0; q < sets.n; ++q) {
    const uint64_t* __restrict__ icodes = sets.codes[q];
    double* __restrict__ out = sets.out[q];
    const int64_t n = sets.cnt[q], pairs = (n + 1) / 2;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < pairs; p += U * stride) {
      if (2 * (p + (U - 1) * stride) + 1 < n) {
        u64x2 c[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
          c[u] = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(icodes + 2 * (p + u * stride)));
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const f64x2 v = {one(c[u][0]), one(c[u][1])};
          __builtin_nontemporal_store(v, reinterpret_cast<f64x2*>(out + 2 * (p + u * stride)));
        }
      } else {
        for (int u = 0; u < U && p + u * stride < pairs; ++u)
          for (int64_t j = 2 * (p + u * stride); j < 2 * (p + u * stride) + 2 && j < n; ++j) out[j] = one(icodes[j]);
      }
    }
  }
  if (bad && err) atomicOr(err, bad);
}

// rate() from the count pass's codes: a thread rates 4 actions (one 16-B code load, two 16-B
// stores) -- 12 B per action instead of 42.
__global__ __launch_bounds__(256) void xt_rate_codes_kernel(const uint32_t* __restrict__ codes, int64_t n,
                                                            const double* __restrict__ grid,
                                                            double* __restrict__ out,
                                                            int32_t* __restrict__ err) {
  const int64_t j0 = 4 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (j0 >= n) return;
  int32_t bad = 0;
  auto one = [&](uint32_t c) -> double {
    if (c == XT_CODE_NAN) return __builtin_nan("");
    if (c == XT_CODE_BAD) {
      bad = 4;
      return __builtin_nan("");
    }
    return grid[c >> 16] - grid[c & 0xFFFFu];
  };
  if (j0 + 4 <= n) {
    const u32x4 c = *reinterpret_cast<const u32x4*>(codes + j0);
    const f64x2 a = {one(c[0]), one(c[1])}, b = {one(c[2]), one(c[3])};
    __builtin_nontemporal_store(a, reinterpret_cast<f64x2*>(out + j0));
    __builtin_nontemporal_store(b, reinterpret_cast<f64x2*>(out + j0 + 2));
  } else {
    for (int64_t j = j0; j < n; ++j) out[j] = one(codes[j]);
  }
  if (bad && err) atomicOr(err, bad);
}

// rate() from the cell codes (grid = the fitted (w, l) surface): a thread rates 4 actions
// (one 16-B code load, two 16-B stores) -- 12 B per action.
__global__ __launch_bounds__(256) void xt_rate_cells_kernel(const uint32_t* __restrict__ cells, int64_t n,
                                                            int C, const double* __restrict__ grid,
                                                            double* __restrict__ out,
                                                            int32_t* __restrict__ err) {
  const int64_t j0 = 4 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (j0 >= n) return;
  int32_t bad = 0;
  const bool c16 = xt_c16(C);
  auto one = [&](uint32_t c) -> double {
    const XtAct a = c16 ? decode_cell16(c, C) : decode_cell(c);
    if (a.cls != XT_CELL_MOVE || !a.succ) return __builtin_nan("");
    if (!a.sfin || !a.efin) {
      bad = 4;  // the reference's int64 cast of a non-finite coordinate raises
      return __builtin_nan("");
    }
    SA_DGUARD(a.cs < C && a.ce < C, c, return __builtin_nan(""));
    return grid[a.ce] - grid[a.cs];
  };
  if (c16) {
    const uint16_t* c2 = reinterpret_cast<const uint16_t*>(cells);
    if (j0 + 4 <= n) {
      const uint2 q = *reinterpret_cast<const uint2*>(c2 + j0);
      const f64x2 x = {one(q.x & 0xFFFFu), one(q.x >> 16)}, y = {one(q.y & 0xFFFFu), one(q.y >> 16)};
      __builtin_nontemporal_store(x, reinterpret_cast<f64x2*>(out + j0));
      __builtin_nontemporal_store(y, reinterpret_cast<f64x2*>(out + j0 + 2));
    } else {
      for (int64_t j = j0; j < n; ++j) out[j] = one(c2[j]);
    }
    if (bad && err) atomicOr(err, bad);
    return;
  }
  if (j0 + 4 <= n) {
    const u32x4 c = *reinterpret_cast<const u32x4*>(cells + j0);
    const f64x2 x = {one(c[0]), one(c[1])}, y = {one(c[2]), one(c[3])};
    __builtin_nontemporal_store(x, reinterpret_cast<f64x2*>(out + j0));
    __builtin_nontemporal_store(y, reinterpret_cast<f64x2*>(out + j0 + 2));
  } else {
    for (int64_t j = j0; j < n; ++j) out[j] = one(cells[j]);
  }
  if (bad && err) atomicOr(err, bad);
}

}  // namespace sa

// ================================== C ABI =================================================
using namespace sa;

extern "C" int sa_xt_count(const sa_actions* a, int32_t l, int32_t w, int64_t* shot, int64_t* goal,
                           int64_t* move, int32_t* trans, int32_t* err_flags, void* stream) {
  return sa_xt_count_codes(a, l, w, shot, goal, move, trans, err_flags, nullptr, 0, stream);
}

// Count-pass launcher shared by the coordinate path (cells == nullptr) and the cell-code path.
static int launch_count(const sa_actions& A, const uint32_t* cells, int64_t n, int32_t l, int32_t w,
                        int64_t* shot, int64_t* goal, int64_t* move, int32_t* trans, int32_t* err_flags,
                        uint32_t* codes, int32_t flags, hipStream_t st) {
  const int C = l * w;
  const size_t small_lds = (size_t)(3 * C + (C * C + 1) / 2) * 4;
  auto* us = reinterpret_cast<unsigned long long*>(shot);
  auto* ug = reinterpret_cast<unsigned long long*>(goal);
  auto* um = reinterpret_cast<unsigned long long*>(move);
  const size_t vec_lds = (size_t)3 * C * 4;
  const unsigned wg_blocks = (unsigned)((n + XT_SMALL_ACTS - 1) / XT_SMALL_ACTS);
  const size_t wide_lds = (size_t)(3 * C + C * C) * 4;
  const bool cl = cells != nullptr;
  // SA_XT_COUNT_SHARED: the pass runs next to other kernels (bench.py's side stream), so use the
  // 80-KB-LDS workgroups that co-reside with them instead of one 150-KB workgroup per CU, which
  // waits for whole CUs to drain (in-process A/B: 3.35 vs 3.40 ms per step)
  const bool shared = (flags & SA_XT_COUNT_SHARED) != 0;
#define SA_COUNT_LAUNCH(MODE, GRID, BLOCK, LDS, CHUNK)                                                   \
  do {                                                                                                  \
    if (cl)                                                                                             \
      hipLaunchKernelGGL((xt_count_kernel<MODE, true>), GRID, BLOCK, LDS, st, A, cells, n, l, w, us, ug,  \
                         um, trans, err_flags, (int64_t)(CHUNK), nullptr);                              \
    else                                                                                                \
      hipLaunchKernelGGL((xt_count_kernel<MODE, false>), GRID, BLOCK, LDS, st, A, nullptr, n, l, w, us,   \
                         ug, um, trans, err_flags, (int64_t)(CHUNK), codes);                            \
  } while (0)
  if (SA_XT_WIDE && wide_lds <= 150 * 1024 && !shared) {
    // one workgroup per CU (or fewer when there are few actions: >= 4096 actions each)
    const int cus = device_cus(current_device());
    int64_t blocks = (n + 4095) / 4096;
    if (blocks > cus) blocks = cus;
    const int64_t chunk = (n + blocks - 1) / blocks;
    SA_COUNT_LAUNCH(XC_WIDE, dim3((unsigned)blocks), dim3(XT_WIDE_THREADS), wide_lds, chunk);
  } else if (small_lds <= 80 * 1024) {
    SA_COUNT_LAUNCH(XC_SMALL, dim3(wg_blocks), dim3(XT_THREADS), small_lds, XT_SMALL_ACTS);
  } else if (SA_XT_BANDS && xt_band_ok(C) && n <= INT32_MAX) {
    // band-owned count (sa_xt_large.hip): no global atomics into the C x C table
    return xt_count_bands(A, cells, n, l, w, shot, goal, move, trans, err_flags, codes, st);
  } else if (vec_lds <= 120 * 1024) {
    SA_COUNT_LAUNCH(XC_VEC, dim3(wg_blocks), dim3(XT_THREADS), vec_lds, XT_SMALL_ACTS);
  } else {
    int64_t blocks = (n + XT_THREADS - 1) / XT_THREADS;
    if (blocks > 4096) blocks = 4096;
    SA_COUNT_LAUNCH(XC_GLOBAL, dim3((unsigned)blocks), dim3(XT_THREADS), 0, 0);
  }
#undef SA_COUNT_LAUNCH
  return check_launch("xt_count_kernel");
}

extern "C" int sa_xt_count_codes(const sa_actions* a, int32_t l, int32_t w, int64_t* shot,
                                 int64_t* goal, int64_t* move, int32_t* trans, int32_t* err_flags,
                                 uint32_t* codes, int32_t flags, void* stream) {
  if (!a || a->n < 0) return fail(SA_EINVAL, "bad sa_actions");
  if (l < 1 || w < 1) return fail(SA_EINVAL, "l and w must be >= 1");
  if ((int64_t)l * w > 46340) return fail(SA_EINVAL, "grid too large (C*C must fit int32 indexing)");
  if (!shot || !goal || !move || !trans || !err_flags) return fail(SA_EINVAL, "null output");
  const sa_frame& F = a->frames[0];
  if (a->n > 0 && (!F.type_id || !F.result_id || !F.c0 || !F.c1 || !F.c2 || !F.c3))
    return fail(SA_EINVAL, "null input column");
  if (codes && !aligned16(codes)) return fail(SA_EINVAL, "codes must be 16-byte aligned");
  if (codes && (int64_t)l * w > 65535) return fail(SA_EINVAL, "rate codes need l * w <= 65535");
  if (a->n == 0) return SA_OK;
  return launch_count(*a, nullptr, a->n, l, w, shot, goal, move, trans, err_flags, codes, flags,
                      (hipStream_t)stream);
}

extern "C" int sa_xt_cells(const sa_actions* a, int32_t l, int32_t w, uint32_t* cells, void* stream) {
  if (!a || a->n < 0 || a->atomic) return fail(SA_EINVAL, "bad sa_actions (SPADL actions required)");
  if (l < 1 || w < 1 || (int64_t)l * w > SA_XT_CELLS_MAX_C)
    return fail(SA_EINVAL, "cell codes need 1 <= l * w <= %d", SA_XT_CELLS_MAX_C);
  if (a->n == 0) return SA_OK;
  const sa_frame& F = a->frames[0];
  if (!F.type_id || !F.result_id || !F.c0 || !F.c1 || !F.c2 || !F.c3 || !cells)
    return fail(SA_EINVAL, "null input column or output");
  if (!aligned16(cells)) return fail(SA_EINVAL, "cells must be 16-byte aligned");
  const int64_t threads = (a->n + 3) / 4;
  hipLaunchKernelGGL(xt_cells_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, *a, l, w, cells);
  return check_launch("xt_cells_kernel");
}

extern "C" int sa_xt_count_cells(const uint32_t* cells, int64_t n, int32_t l, int32_t w, int64_t* shot,
                                 int64_t* goal, int64_t* move, int32_t* trans, int32_t* err_flags,
                                 int32_t flags, void* stream) {
  if (n < 0 || l < 1 || w < 1 || (int64_t)l * w > SA_XT_CELLS_MAX_C)
    return fail(SA_EINVAL, "cell codes need n >= 0 and 1 <= l * w <= %d", SA_XT_CELLS_MAX_C);
  if (!shot || !goal || !move || !trans || !err_flags || (n > 0 && !cells))
    return fail(SA_EINVAL, "null pointer");
  if (n == 0) return SA_OK;
  sa_actions none;
  memset(&none, 0, sizeof(none));
  return launch_count(none, cells, n, l, w, shot, goal, move, trans, err_flags, nullptr, flags,
                      (hipStream_t)stream);
}

extern "C" int sa_xt_solve_async(const int64_t* shot, const int64_t* goal, const int64_t* move,
                                 const int32_t* trans, int32_t l, int32_t w, double eps, int32_t max_iter,
                                 double* mats, double* trans_t, double* heatmaps, int32_t* n_iter_dev,
                                 void* stream) {
  if (l < 1 || w < 1 || max_iter < 0) return fail(SA_EINVAL, "bad l, w or max_iter");
  const int C = l * w;
  if (C > XT_SOLVE_MAX_C) return fail(SA_EINVAL, "the asynchronous solve takes grids of <= %d cells", XT_SOLVE_MAX_C);
  if (!shot || !goal || !move || !trans || !mats || !trans_t || !heatmaps || !n_iter_dev)
    return fail(SA_EINVAL, "null pointer");
  hipStream_t st = (hipStream_t)stream;
  auto* us = reinterpret_cast<const unsigned long long*>(shot);
  auto* ug = reinterpret_cast<const unsigned long long*>(goal);
  auto* um = reinterpret_cast<const unsigned long long*>(move);
  Scratch sc;  // gs[C] | pmove[C]
  int rc = scratch_acquire(sizeof(double) * 2 * C, st, &sc);
  if (rc) return rc;
  double* gs = static_cast<double*>(sc.ptr);
  double* pm = gs + C;
  hipLaunchKernelGGL(xt_prob_kernel, dim3((C + 255) / 256), dim3(256), 0, st, us, ug, um, C, mats, gs, pm);
  const dim3 tgrid((C + 31) / 32, (C + 31) / 32);
  hipLaunchKernelGGL(xt_transpose_kernel, tgrid, dim3(256), 0, st, trans, um, C, trans_t);
  rc = check_launch("xt normalise");
  if (!rc && C <= XR_MAX_C) {
    hipLaunchKernelGGL(xt_solve_reg_kernel<SA_XR_PARTS>, dim3(1), dim3(SA_XR_PARTS * XR_MAX_C), 0, st, trans_t, gs,
                       pm, C, eps, max_iter, heatmaps, mats + 3 * C, n_iter_dev);
    rc = check_launch("xt_solve_reg_kernel");
  } else if (!rc) {
    hipLaunchKernelGGL(xt_solve_small_kernel, dim3(1), dim3(((C + 63) / 64) * 64), 0, st, trans_t, gs, pm, C, eps,
                       max_iter, heatmaps, mats + 3 * C, n_iter_dev);
    rc = check_launch("xt_solve_small_kernel");
  }
  scratch_release(sc, st);
  return rc;
}

extern "C" int sa_xt_solve(const int64_t* shot, const int64_t* goal, const int64_t* move,
                           const int32_t* trans, int32_t l, int32_t w, double eps, int32_t max_iter,
                           double* mats, double* trans_t, double* heatmaps, int32_t* n_iter,
                           void* stream) {
  return sa_xt_solve_ex(shot, goal, move, trans, l, w, eps, max_iter, 0, mats, trans_t, heatmaps, n_iter, nullptr,
                        nullptr, nullptr, stream);
}

static int solve_ex(const int64_t* shot, const int64_t* goal, const int64_t* move, const int32_t* trans, int32_t l,
                    int32_t w, double eps, int32_t max_iter, int32_t flags, double* mats, double* trans_t,
                    double* heatmaps, int32_t* n_iter, int32_t* path, const uint32_t* ell_in,
                    const int32_t* row_len_in, void* stream, SolveHook* hook);

extern "C" int sa_xt_solve_ex(const int64_t* shot, const int64_t* goal, const int64_t* move,
                              const int32_t* trans, int32_t l, int32_t w, double eps, int32_t max_iter,
                              int32_t flags, double* mats, double* trans_t, double* heatmaps, int32_t* n_iter,
                              int32_t* path, const uint32_t* ell_in, const int32_t* row_len_in, void* stream) {
  return solve_ex(shot, goal, move, trans, l, w, eps, max_iter, flags, mats, trans_t, heatmaps, n_iter, path, ell_in,
                  row_len_in, stream, nullptr);
}

static int solve_ex(const int64_t* shot, const int64_t* goal, const int64_t* move, const int32_t* trans, int32_t l,
                    int32_t w, double eps, int32_t max_iter, int32_t flags, double* mats, double* trans_t,
                    double* heatmaps, int32_t* n_iter, int32_t* path, const uint32_t* ell_in,
                    const int32_t* row_len_in, void* stream, SolveHook* hook) {
  if (l < 1 || w < 1 || max_iter < 0) return fail(SA_EINVAL, "bad l, w or max_iter");
  const int C = l * w;
  if (!shot || !goal || !move || !trans || !mats || (!trans_t && C <= XT_SOLVE_MAX_C) || !heatmaps || !n_iter)
    return fail(SA_EINVAL, "null pointer");
  if (flags & ~SA_XT_SOLVE_EXACT) return fail(SA_EINVAL, "unknown flags");
  if (!ell_in != !row_len_in) return fail(SA_EINVAL, "ell and row_len come together");
  if (ell_in && (C <= XT_SOLVE_MAX_C || !SA_XT_COMPACT || !xt_compact_ok(C) || !aligned16(ell_in)))
    return fail(SA_EINVAL, "a prebuilt compact form is for %d < C <= the compact limit (16-byte aligned)",
                XT_SOLVE_MAX_C);
  if (path) *path = SA_XT_PATH_SEQUENTIAL;
  hipStream_t st = (hipStream_t)stream;
  auto* us = reinterpret_cast<const unsigned long long*>(shot);
  auto* ug = reinterpret_cast<const unsigned long long*>(goal);
  auto* um = reinterpret_cast<const unsigned long long*>(move);
  // scratch: gs[C] | pmove[C] | n_iter | convergence flags[max_iter + 1]
  Scratch sc;
  int rc = scratch_acquire(sizeof(double) * 2 * C + sizeof(int32_t) * (max_iter + 2), st, &sc);
  if (rc) return rc;
  double* gs = static_cast<double*>(sc.ptr);
  double* pm = gs + C;
  int32_t* dn = reinterpret_cast<int32_t*>(pm + C);
  int32_t* dflags = dn + 1;
  int32_t iters = -1;
  hipLaunchKernelGGL(xt_prob_kernel, dim3((C + 255) / 256), dim3(256), 0, st, us, ug, um, C, mats, gs, pm);
  if (trans_t) {  // the dense transposed matrix: read by the small-grid solve, optional above
    const dim3 tgrid((C + 31) / 32, (C + 31) / 32);
    hipLaunchKernelGGL(xt_transpose_kernel, tgrid, dim3(256), 0, st, trans, um, C, trans_t);
  }
  rc = check_launch("xt normalise");
  if (!rc && C <= XT_SOLVE_MAX_C) {
    if (C <= XR_MAX_C) {
      hipLaunchKernelGGL(xt_solve_reg_kernel<SA_XR_PARTS>, dim3(1), dim3(SA_XR_PARTS * XR_MAX_C), 0, st, trans_t, gs, pm, C, eps,
                         max_iter, heatmaps, mats + 3 * C, dn);
      rc = check_launch("xt_solve_reg_kernel");
    } else {
      hipLaunchKernelGGL(xt_solve_small_kernel, dim3(1), dim3(((C + 63) / 64) * 64), 0, st, trans_t, gs, pm, C,
                         eps, max_iter, heatmaps, mats + 3 * C, dn);
      rc = check_launch("xt_solve_small_kernel");
    }
    if (!rc) rc = check_hip(hipMemcpyAsync(&iters, dn, sizeof(int32_t), hipMemcpyDeviceToHost, st),
                            "copy n_iter");
    if (!rc) rc = check_hip(hipStreamSynchronize(st), "hipStreamSynchronize");
  } else if (!rc) {
    // the compact form of the count rows, built once (sa_xt_large.hip): [ell | row_len]
    const bool compact = SA_XT_COMPACT && xt_compact_ok(C);
    rc = check_hip(hipMemsetAsync(heatmaps, 0, sizeof(double) * C, st), "memset");
    if (!rc && !compact)  // the dense loop's flags (the compact solve keeps its own)
      rc = check_hip(hipMemsetAsync(dflags, 0, sizeof(int32_t) * (max_iter + 1), st), "memset");
    Scratch ce;
    const uint32_t* ell = ell_in;  // prebuilt by the count (sa_xt_count_from_buckets_ex), or built here
    const int32_t* slen = row_len_in;
    if (!rc && compact && !ell) {
      const size_t eb = (xt_compact_bytes(C, C) + 255) & ~(size_t)255;
      rc = scratch_acquire(eb + sizeof(int32_t) * (size_t)C, st, &ce);
      if (!rc) {
        uint32_t* e = static_cast<uint32_t*>(ce.ptr);
        int32_t* sl = reinterpret_cast<int32_t*>(static_cast<char*>(ce.ptr) + eb);
        rc = xt_compact_build(trans, C, C, e, sl, st);
        ell = e;
        slen = sl;
      }
    }
    bool surface_done = false;  // the reordered solve wrote the surface itself
    if (compact && !rc) {  // reordered under the error bound, or the reference's order
      int p = SA_XT_PATH_SEQUENTIAL;
      rc = xt_compact_solve(ell, slen, trans, move, gs, pm, C, eps, max_iter, flags, heatmaps, &iters, &p, st,
                            mats + 3 * C, hook);
      if (path) *path = p;
      surface_done = p == SA_XT_PATH_REORDERED;
    }
    std::vector<int32_t> hflags(max_iter + 1, 0);
    const int batch = 8;
    for (int it0 = 0; !compact && !rc && it0 < max_iter && iters < 0; it0 += batch) {
      const int it1 = it0 + batch < max_iter ? it0 + batch : max_iter;
      for (int it = it0; it < it1 && !rc; ++it) {  // above the compact form's C: the dense rows
        double* xi = heatmaps + (int64_t)it * C;
        const int32_t* fp = it > 0 ? dflags + it - 1 : nullptr;
        hipLaunchKernelGGL(xt_iter_kernel, dim3((C + XI_ROWS - 1) / XI_ROWS), dim3(XI_THREADS), 0, st, trans, um,
                           gs, pm, C, 0, C, eps, xi, xi + C, fp, dflags + it);
        rc = check_launch("xt_iter_kernel");
      }
      if (!rc) rc = check_hip(hipMemcpyAsync(hflags.data() + it0, dflags + it0,
                                             sizeof(int32_t) * (it1 - it0), hipMemcpyDeviceToHost, st),
                              "copy flags");
      if (!rc) rc = check_hip(hipStreamSynchronize(st), "hipStreamSynchronize");
      for (int it = it0; !rc && it < it1; ++it)
        if (hflags[it] == 0) {
          iters = it + 1;
          break;
        }
    }
    if (!rc && !surface_done) {
      const int last = iters < 0 ? max_iter : iters;
      rc = check_hip(hipMemcpyAsync(mats + 3 * C, heatmaps + (int64_t)last * C, sizeof(double) * C,
                                    hipMemcpyDeviceToDevice, st),
                     "copy xT");
      if (!rc) rc = check_hip(hipStreamSynchronize(st), "hipStreamSynchronize");
    }
    if (compact && !ell_in) scratch_release(ce, st);
  }
  scratch_release(sc, st);
  *n_iter = iters;
  return rc;
}

extern "C" int sa_xt_interp_grid(const double* xT, const double* cx, const double* cy, int32_t l,
                                 int32_t w, const double* xs, int32_t L, const double* ys, int32_t W,
                                 double* grid, void* stream) {
  if (l < 2 || w < 2) return fail(SA_EINVAL, "interpolation needs at least 2 cells per axis");
  if (L < 1 || W < 1 || !xT || !cx || !cy || !xs || !ys || !grid)
    return fail(SA_EINVAL, "bad interpolation args");
  const int64_t total = (int64_t)L * W;
  hipLaunchKernelGGL(xt_interp_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, xT, cx, cy, l, w, xs, L, ys, W, grid);
  return check_launch("xt_interp_kernel");
}

extern "C" int sa_xt_normalize(const int64_t* shot, const int64_t* goal, const int64_t* move,
                               const int32_t* trans, int32_t l, int32_t w, double* mats,
                               double* trans_t, void* stream) {
  if (l < 1 || w < 1) return fail(SA_EINVAL, "bad l or w");
  if (!shot || !goal || !move || !trans || !mats || !trans_t) return fail(SA_EINVAL, "null pointer");
  const int C = l * w;
  hipStream_t st = (hipStream_t)stream;
  auto* us = reinterpret_cast<const unsigned long long*>(shot);
  auto* ug = reinterpret_cast<const unsigned long long*>(goal);
  auto* um = reinterpret_cast<const unsigned long long*>(move);
  Scratch sc;  // gs[C] | pmove[C] (not returned by this entry point)
  int rc = scratch_acquire(sizeof(double) * 2 * C, st, &sc);
  if (rc) return rc;
  double* gs = static_cast<double*>(sc.ptr);
  hipLaunchKernelGGL(xt_prob_kernel, dim3((C + 255) / 256), dim3(256), 0, st, us, ug, um, C, mats, gs,
                     gs + C);
  const dim3 tgrid((C + 31) / 32, (C + 31) / 32);
  hipLaunchKernelGGL(xt_transpose_kernel, tgrid, dim3(256), 0, st, trans, um, C, trans_t);
  rc = check_launch("xt normalise");
  scratch_release(sc, st);
  return rc;
}

extern "C" int sa_xt_rate(const sa_actions* a, const double* grid, int32_t L, int32_t W, double* out,
                          int32_t* err_flags, void* stream) {
  if (!a || a->n < 0 || !grid || !out || L < 1 || W < 1) return fail(SA_EINVAL, "bad xt_rate args");
  if (a->n == 0) return SA_OK;
  const sa_frame& F = a->frames[0];
  const int vec = aligned16(F.c0) && aligned16(F.c1) && aligned16(F.c2) && aligned16(F.c3) && aligned16(out) &&
                  ((uintptr_t)F.type_id & 1u) == 0 && ((uintptr_t)F.result_id & 1u) == 0;
  const int64_t threads = (a->n + 1) / 2;
  hipLaunchKernelGGL(xt_rate_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, *a, grid, L, W, out, err_flags, vec);
  return check_launch("xt_rate_kernel");
}

extern "C" int sa_xt_rate_interp(const sa_actions* a, const double* xT, const double* cx, const double* cy,
                                 int32_t l, int32_t w, const double* xs, int32_t L, const double* ys, int32_t W,
                                 double* out, int32_t* err_flags, void* stream) {
  if (!a || a->n < 0 || !xT || !cx || !cy || !xs || !ys || !out || L < 1 || W < 1)
    return fail(SA_EINVAL, "bad xt_rate_interp args");
  if (l < 2 || w < 2) return fail(SA_EINVAL, "interpolation needs at least 2 cells per axis");
  if ((int64_t)L * W > INT32_MAX) return fail(SA_EINVAL, "interpolated grid too large");
  if (a->n == 0) return SA_OK;
  hipStream_t st = (hipStream_t)stream;
  Scratch sc;  // frac[L + W] | idx[L + W]
  int rc = scratch_acquire((sizeof(double) + sizeof(int32_t)) * (size_t)(L + W), st, &sc);
  if (rc) return rc;
  double* frac = static_cast<double*>(sc.ptr);
  int32_t* idx = reinterpret_cast<int32_t*>(frac + (L + W));
  hipLaunchKernelGGL(xt_axes_kernel, dim3((unsigned)((L + W + 255) / 256)), dim3(256), 0, st, cx, cy, l, w, xs, L,
                     ys, W, idx, frac);
  const sa_frame& F = a->frames[0];
  const int vec = aligned16(F.c0) && aligned16(F.c1) && aligned16(F.c2) && aligned16(F.c3) && aligned16(out) &&
                  ((uintptr_t)F.type_id & 1u) == 0 && ((uintptr_t)F.result_id & 1u) == 0;
  const int64_t threads = (a->n + 1) / 2;
  const size_t lds = sizeof(double) * ((size_t)l * w + L + W) + sizeof(int32_t) * (size_t)(L + W);
  const int dev = current_device();
  if (lds <= XRI_LDS_MAX && lds <= (size_t)device_lds_max(dev)) {  // surface + node tables in LDS
    const int cus = device_cus(dev);
    const int64_t need = (threads + XRI_THREADS - 1) / XRI_THREADS;
    const int64_t most = (int64_t)cus * SA_XRI_BPC;
    const unsigned blocks = (unsigned)(need < most ? need : most);
    hipLaunchKernelGGL(xt_rate_interp_lds_kernel, dim3(blocks), dim3(XRI_THREADS), lds, st, *a, xT, l, w, L, W, idx,
                       frac, out, err_flags, vec);
    rc = check_launch("xt_rate_interp_lds_kernel");
  } else {
    hipLaunchKernelGGL(xt_rate_interp_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, *a, xT, l,
                       L, W, idx, frac, out, err_flags, vec);
    rc = check_launch("xt_rate_interp_kernel");
  }
  scratch_release(sc, st);
  return rc;
}

extern "C" int sa_xt_rate_interp_codes_many(int32_t nsets, const uint64_t* const* interp_codes, const int64_t* n,
                                            const double* xT, const double* cx, const double* cy, int32_t l, int32_t w,
                                            const double* xs, int32_t L, const double* ys, int32_t W,
                                            double* const* out, int32_t* err_flags, void* stream) {
  if (nsets < 0 || (nsets > 0 && (!interp_codes || !n || !out)) || !xT || !cx || !cy || !xs || !ys || L < 1 || W < 1)
    return fail(SA_EINVAL, "bad xt_rate_interp_codes args");
  if (l < 2 || w < 2) return fail(SA_EINVAL, "interpolation needs at least 2 cells per axis");
  if ((int64_t)L * W > INT32_MAX) return fail(SA_EINVAL, "interpolated grid too large");
  int64_t most_n = 0;
  for (int q = 0; q < nsets; ++q) {
    if (n[q] < 0) return fail(SA_EINVAL, "set %d: negative action count", q);
    if (n[q] > 0 && (!interp_codes[q] || !out[q])) return fail(SA_EINVAL, "set %d: null codes or out", q);
    if (n[q] > 0 && (!aligned16(interp_codes[q]) || !aligned16(out[q])))
      return fail(SA_EINVAL, "codes and out must be 16-byte aligned");
    most_n = n[q] > most_n ? n[q] : most_n;
  }
  const size_t lds = sizeof(double) * ((size_t)l * w + L + W) + sizeof(int32_t) * (size_t)(L + W);
  const int dev = current_device();
  if (lds > XRI_LDS_MAX || lds > (size_t)device_lds_max(dev))
    return fail(SA_EINVAL, "surface and node tables exceed the LDS");
  if (most_n == 0) return SA_OK;
  hipStream_t st = (hipStream_t)stream;
  Scratch sc;  // frac[L + W] | idx[L + W]
  int rc = scratch_acquire((sizeof(double) + sizeof(int32_t)) * (size_t)(L + W), st, &sc);
  if (rc) return rc;
  double* frac = static_cast<double*>(sc.ptr);
  int32_t* idx = reinterpret_cast<int32_t*>(frac + (L + W));
  hipLaunchKernelGGL(xt_axes_kernel, dim3((unsigned)((L + W + 255) / 256)), dim3(256), 0, st, cx, cy, l, w, xs, L,
                     ys, W, idx, frac);
  const int64_t threads = (most_n + 1) / 2;
  const int64_t need = (threads + XRI_THREADS - 1) / XRI_THREADS;
  const int64_t most = (int64_t)device_cus(dev) * SA_XRI_BPC;
  for (int q0 = 0; q0 < nsets && !rc; q0 += XRI_MAX_SETS) {
    XriSets S{};
    for (int q = q0; q < nsets && q < q0 + XRI_MAX_SETS; ++q) {
      if (n[q] == 0) continue;
      S.codes[S.n] = interp_codes[q];
      S.out[S.n] = out[q];
      S.cnt[S.n] = n[q];
      ++S.n;
    }
    if (!S.n) continue;
    hipLaunchKernelGGL(xt_rate_icodes_lds_kernel, dim3((unsigned)(need < most ? need : most)), dim3(XRI_THREADS),
                       lds, st, S, xT, l, w, L, W, idx, frac, err_flags);
    rc = check_launch("xt_rate_icodes_lds_kernel");
  }
  scratch_release(sc, st);
  return rc;
}

// ExpectedThreat.fit + rate(use_interpolation=True) of the same actions in one call: sa_xt_solve_ex
// (no transposed matrix) then sa_xt_rate_interp_codes_many over the surface it wrote.  Above the
// small-grid limit the rate is queued right behind the one-launch reordered solve, before the
// host waits for the solve's status -- no host round trip between the two; when the status
// sends the solve to another path (the reference's order: a decision inside the bound, a
// barrier timeout, an escaped count) the surface is rewritten and the rate runs again.
extern "C" int sa_xt_fit_rate_interp_codes(const int64_t* shot, const int64_t* goal, const int64_t* move,
                                           const int32_t* trans, int32_t l, int32_t w, double eps, int32_t max_iter,
                                           int32_t flags, double* mats, double* heatmaps, int32_t* n_iter,
                                           int32_t* path, const uint32_t* ell, const int32_t* row_len, int32_t nsets,
                                           const uint64_t* const* interp_codes, const int64_t* n, const double* cx,
                                           const double* cy, const double* xs, int32_t L, const double* ys,
                                           int32_t W, double* const* out, int32_t* err_flags, void* stream) {
  if (l < 1 || w < 1 || !mats || !path) return fail(SA_EINVAL, "bad l, w or null mats / path");
  if (l * w <= XT_SOLVE_MAX_C) return fail(SA_EINVAL, "the fused fit + rate is for grids above %d cells", XT_SOLVE_MAX_C);
  // the rate's arguments checked before anything is launched (sa_xt_rate_interp_codes_many's own
  // checks would first run behind the solve)
  if (nsets < 0 || (nsets > 0 && (!interp_codes || !n || !out)) || !cx || !cy || !xs || !ys || L < 1 || W < 1 ||
      l < 2 || w < 2 || (int64_t)L * W > INT32_MAX)
    return fail(SA_EINVAL, "bad rate arguments");
  for (int q = 0; q < nsets; ++q)
    if (n[q] < 0 || (n[q] > 0 && (!interp_codes[q] || !out[q] || !aligned16(interp_codes[q]) || !aligned16(out[q]))))
      return fail(SA_EINVAL, "set %d: bad count, codes or out", q);
  struct Rate {
    int32_t nsets;
    const uint64_t* const* codes;
    const int64_t* n;
    const double *xT, *cx, *cy, *xs, *ys;
    int32_t l, w, L, W;
    double* const* out;
    int32_t* err;
    void* stream;
  } r{nsets, interp_codes, n, mats + 3 * (int64_t)(l * w), cx, cy, xs, ys, l, w, L, W, out, err_flags, stream};
  auto rate = [](void* p) -> int {
    const Rate& q = *static_cast<const Rate*>(p);
    return sa_xt_rate_interp_codes_many(q.nsets, q.codes, q.n, q.xT, q.cx, q.cy, q.l, q.w, q.xs, q.L, q.ys, q.W,
                                        q.out, q.err, q.stream);
  };
  SolveHook hook{rate, &r, false};
  int rc = solve_ex(shot, goal, move, trans, l, w, eps, max_iter, flags, mats, nullptr, heatmaps, n_iter, path, ell,
                    row_len, stream, &hook);
  if (rc) return rc;
  if (!hook.ran || *path != SA_XT_PATH_REORDERED) rc = rate(&r);  // the surface the solve returned
  return rc;
}

extern "C" int sa_xt_rate_interp_codes(const uint64_t* interp_codes, int64_t n, const double* xT, const double* cx,
                                       const double* cy, int32_t l, int32_t w, const double* xs, int32_t L,
                                       const double* ys, int32_t W, double* out, int32_t* err_flags, void* stream) {
  if (n < 0 || (n > 0 && (!interp_codes || !out))) return fail(SA_EINVAL, "bad xt_rate_interp_codes args");
  return sa_xt_rate_interp_codes_many(1, &interp_codes, &n, xT, cx, cy, l, w, xs, L, ys, W, &out, err_flags, stream);
}

extern "C" int sa_xt_probabilities(const int64_t* shot, const int64_t* goal, const int64_t* move, int32_t C,
                                   double* mats, double* gs, double* pmove, void* stream) {
  if (C < 1 || !shot || !goal || !move || !mats || !gs || !pmove) return fail(SA_EINVAL, "bad xt probability args");
  hipLaunchKernelGGL(xt_prob_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const unsigned long long*>(shot),
                     reinterpret_cast<const unsigned long long*>(goal),
                     reinterpret_cast<const unsigned long long*>(move), C, mats, gs, pmove);
  return check_launch("xt_prob_kernel");
}

extern "C" int sa_xt_iterate_rows(const int32_t* cnt_rows, const int64_t* move, const double* gs,
                                  const double* pmove, int32_t C, int32_t r0, int32_t nrows, const double* x,
                                  double eps, double* x_next_rows, const int32_t* flag_prev, int32_t* flag_out,
                                  void* stream) {
  if (C < 1 || r0 < 0 || nrows < 0 || r0 + nrows > C) return fail(SA_EINVAL, "row range outside [0, C)");
  if (!move || !gs || !pmove || !x || !flag_out || (nrows > 0 && (!cnt_rows || !x_next_rows)))
    return fail(SA_EINVAL, "null xt iteration pointer");
  if (nrows == 0) return SA_OK;
  hipLaunchKernelGGL(xt_iter_kernel, dim3((nrows + XI_ROWS - 1) / XI_ROWS), dim3(XI_THREADS), 0,
                     (hipStream_t)stream, cnt_rows, reinterpret_cast<const unsigned long long*>(move), gs,
                     pmove, C, r0, nrows, eps, x, x_next_rows, flag_prev, flag_out);
  return check_launch("xt_iter_kernel");
}

extern "C" int sa_xt_rate_codes(const uint32_t* codes, int64_t n, const double* grid, double* out,
                                int32_t* err_flags, void* stream) {
  if (n < 0 || (n > 0 && (!codes || !grid || !out))) return fail(SA_EINVAL, "bad xt_rate_codes args");
  if (n == 0) return SA_OK;
  if (!aligned16(codes) || !aligned16(out)) return fail(SA_EINVAL, "codes and out must be 16-byte aligned");
  const int64_t threads = (n + 3) / 4;
  hipLaunchKernelGGL(xt_rate_codes_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, codes, n, grid, out, err_flags);
  return check_launch("xt_rate_codes_kernel");
}

extern "C" int sa_xt_rate_cells(const uint32_t* cells, int64_t n, int32_t l, int32_t w, const double* grid,
                                double* out, int32_t* err_flags, void* stream) {
  if (n < 0 || l < 1 || w < 1 || (int64_t)l * w > SA_XT_CELLS_MAX_C)
    return fail(SA_EINVAL, "cell codes need n >= 0 and 1 <= l * w <= %d", SA_XT_CELLS_MAX_C);
  if (n > 0 && (!cells || !grid || !out)) return fail(SA_EINVAL, "null pointer");
  if (n == 0) return SA_OK;
  if (!aligned16(cells) || !aligned16(out)) return fail(SA_EINVAL, "cells and out must be 16-byte aligned");
  const int64_t threads = (n + 3) / 4;
  hipLaunchKernelGGL(xt_rate_cells_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, cells, n, l * w, grid, out, err_flags);
  return check_launch("xt_rate_cells_kernel");
}
