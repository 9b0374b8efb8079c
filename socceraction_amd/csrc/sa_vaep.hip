// VAEP / Atomic-VAEP hot-path kernels for gfx950 (MI355X).
//
//   features_kernel   gamestates + play_left_to_right + every known transformer,
//                     fused; writes column-major bool / f64 / i64 blocks.
//   goalscore_kernel  segmented exclusive scan (one workgroup per segment).
//   labels_kernel     scores / concedes / goal_from_shot look-ahead.
//   formula_kernel    offensive / defensive / vaep value (f64 or f32).
//
// All of it is HBM-bound byte/int/f64 streaming: nothing here is GEMM-shaped.
// Layout: one wave owns 1024 consecutive actions.  Bool columns
// are written with lane-owns-16-actions (one 16-B store per lane = 1 KiB per wave
// instruction); f64/i64 columns with lane-owns-2-actions (again 1 KiB per wave
// instruction).  Per-action window metadata passes between the two phases in LDS.
#include <hip/hip_runtime.h>

#include <cmath>

#include "sa_common.h"
#include "sa_internal.h"

namespace sa {

constexpr int WAVE = 64;
constexpr int LANE_ACTS = 16;
constexpr int WAVE_ACTS = WAVE * LANE_ACTS;  // 1024
constexpr int BLOCK_WAVES = 4;

struct FeatArgs {
  sa_actions a;
  sa_feature_plan p;
  uint8_t* bout;
  double* fout;
  int64_t* iout;
  int64_t ld;
};

__device__ __forceinline__ uint32_t pick6(const uint32_t (&W)[6], int idx) {
  uint32_t r = W[0];
#pragma unroll
  for (int k = 1; k < 6; ++k) r = (idx == k) ? W[k] : r;
  return r;
}

// byte at position B (0..23) of the 24-byte window W
__device__ __forceinline__ uint32_t byte24(const uint32_t (&W)[6], int B) {
  return (pick6(W, B >> 2) >> (8 * (B & 3))) & 0xFFu;
}

__device__ __forceinline__ int32_t pick24(const int32_t (&T)[24], int idx) {
  int32_t r = T[0];
#pragma unroll
  for (int k = 1; k < 24; ++k) r = (idx == k) ? T[k] : r;
  return r;
}

// Word q (bytes 4q..4q+3 of the lane's 16 actions) of game-state window i, where the
// lane's rows j0-8 .. j0+15 sit in W (byte 8 = row j0) and d[m] = min(j - seg_start, 15).
__device__ __forceinline__ uint32_t window_word(const uint32_t (&W)[6], const uint32_t (&dw)[4],
                                                int q, int i, bool slow) {
  int B = 8 + 4 * q - i;  // 0 <= B <= 20
  uint32_t v = funnel_bytes(pick6(W, B >> 2), pick6(W, (B >> 2) + 1), B & 3);
  if (slow) {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      int d = (int)byte_of(dw[q], b);
      if (d < i) {  // window row clamps to the segment start: row j - d
        uint32_t x = byte24(W, 8 + 4 * q + b - d);
        v = (v & ~(0xFFu << (8 * b))) | (x << (8 * b));
      }
    }
  }
  return v;
}

__device__ __forceinline__ void st_bool16(uint8_t* __restrict__ base, int64_t col, int64_t ld,
                                          int64_t j0, uint32_t w0, uint32_t w1, uint32_t w2,
                                          uint32_t w3) {
  u32x4 v = {w0, w1, w2, w3};
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(base + col * ld + j0));
}

__device__ __forceinline__ void st_f64x2(double* __restrict__ base, int64_t col, int64_t ld,
                                         int64_t j, double v0, double v1) {
  f64x2 v = {v0, v1};
  __builtin_nontemporal_store(v, reinterpret_cast<f64x2*>(base + col * ld + j));
}

__device__ __forceinline__ void st_i64x2(int64_t* __restrict__ base, int64_t col, int64_t ld,
                                         int64_t j, int64_t v0, int64_t v1) {
  i64x2 v = {(long long)v0, (long long)v1};
  __builtin_nontemporal_store(v, reinterpret_cast<i64x2*>(base + col * ld + j));
}

// nan_to_num(arctan(dy / dx)) of vaep/features.py:376 (atan of +-inf is +-pi/2, 0/0 -> 0)
__device__ __forceinline__ double polar_angle(double dy, double dx) {
  double a = atan(dy / dx);
  return isnan(a) ? 0.0 : a;
}

template <bool ATOMIC, bool EXPLICIT>
__global__ __launch_bounds__(256) void features_kernel(FeatArgs args) {
  __shared__ __attribute__((aligned(16))) uint8_t info[BLOCK_WAVES][WAVE_ACTS];
  const int lane = threadIdx.x & (WAVE - 1);
  const int wv = threadIdx.x / WAVE;
  const sa_actions& A = args.a;
  const sa_feature_plan& P = args.p;
  const int64_t n = A.n;
  const int K = P.nb_prev_actions;
  const int64_t wave_base = ((int64_t)blockIdx.x * BLOCK_WAVES + wv) * WAVE_ACTS;
  const int64_t j0 = wave_base + (int64_t)lane * LANE_ACTS;
  const int64_t ld = args.ld;
  const sa_frame& F0 = A.frames[0];

  // ---------------- per-action window metadata: d = min(j - seg_start, 15), away -------------
  uint32_t dw[4] = {0, 0, 0, 0};  // rows >= n keep d = 0 (window rows stay in range)
  uint32_t aw[4] = {0, 0, 0, 0};
  int dmin = 15;
  if (!EXPLICIT && j0 < n) {
    int64_t g = find_segment(A.seg_off, A.n_segments, j0);
    int64_t s = A.seg_off[g], e = A.seg_off[g + 1];
#pragma unroll
    for (int m = 0; m < LANE_ACTS; ++m) {
      int64_t j = j0 + m;
      if (j < n) {
        while (j >= e) {
          ++g;
          s = e;
          e = A.seg_off[g + 1];
        }
        int64_t dd = j - s;
        int d = dd > 15 ? 15 : (int)dd;
        dmin = d < dmin ? d : dmin;
        uint32_t away = (A.home_team != nullptr && F0.team[j] != A.home_team[g]) ? 1u : 0u;
        dw[m >> 2] = (dw[m >> 2] & ~(0xFFu << (8 * (m & 3)))) | ((uint32_t)d << (8 * (m & 3)));
        aw[m >> 2] |= away << (8 * (m & 3));
      }
    }
  }
  {  // publish (d | away << 4) for phase B of this wave
    u32x4 v = {dw[0] | (aw[0] << 4), dw[1] | (aw[1] << 4), dw[2] | (aw[2] << 4),
               dw[3] | (aw[3] << 4)};
    *reinterpret_cast<u32x4*>(&info[wv][lane * LANE_ACTS]) = v;
  }

  // ---------------- phase A: bool columns, lane owns 16 consecutive actions -------------------
  const bool any_bool = P.bool_col[SA_XFN_ACTIONTYPE_ONEHOT] >= 0 ||
                        P.bool_col[SA_XFN_RESULT_ONEHOT] >= 0 ||
                        P.bool_col[SA_XFN_ACTIONTYPE_RESULT_ONEHOT] >= 0 ||
                        P.bool_col[SA_XFN_BODYPART_ONEHOT] >= 0 || P.bool_col[SA_XFN_TEAM] >= 0;
  if (any_bool && j0 < n) {
    const int64_t wbase = j0 / 4 - 2;  // word index of row j0-8
    uint32_t TW[6], RW[6], BW[6];
    int32_t TM[24];
    const bool need_team = P.bool_col[SA_XFN_TEAM] >= 0;
    if (!EXPLICIT) {
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        TW[k] = ld_u8x4(F0.type_id, wbase + k, n);
        RW[k] = ATOMIC ? 0u : ld_u8x4(F0.result_id, wbase + k, n);
        BW[k] = ld_u8x4(F0.bodypart_id, wbase + k, n);
      }
      if (need_team) {
#pragma unroll
        for (int k = 0; k < 24; ++k) TM[k] = ld_or0(F0.team, j0 - 8 + k, n);
      }
    }
    const bool slow = dmin < K - 1;
    for (int i = 0; i < K; ++i) {
      uint32_t tw[4], rw[4], bw[4];
      if (EXPLICIT) {
        const sa_frame& Fi = A.frames[i];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          tw[q] = ld_u8x4(Fi.type_id, j0 / 4 + q, n);
          rw[q] = ATOMIC ? 0u : ld_u8x4(Fi.result_id, j0 / 4 + q, n);
          bw[q] = ld_u8x4(Fi.bodypart_id, j0 / 4 + q, n);
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          tw[q] = window_word(TW, dw, q, i, slow);
          rw[q] = ATOMIC ? 0u : window_word(RW, dw, q, i, slow);
          bw[q] = window_word(BW, dw, q, i, slow);
        }
      }
      int c = P.bool_col[SA_XFN_ACTIONTYPE_ONEHOT];
      if (c >= 0) {
        if (!ATOMIC) {
          for (int t = 0; t < N_TYPES; ++t)
            st_bool16(args.bout, c + i * N_TYPES + t, ld, j0, bytes_eq(tw[0], t), bytes_eq(tw[1], t),
                      bytes_eq(tw[2], t), bytes_eq(tw[3], t));
        } else {
          // 33 atomic names, 32 unique: 'interception' (ids 10 and 24) is one column that is
          // true for both ids (atomic/vaep/features.py:114-132 + atomic/spadl/config.py:25-36)
          for (int u = 0; u < N_ATOMIC_NAMES; ++u) {
            uint32_t id = u <= 23 ? (uint32_t)u : (uint32_t)u + 1;
            uint32_t m0 = bytes_eq(tw[0], id), m1 = bytes_eq(tw[1], id), m2 = bytes_eq(tw[2], id),
                     m3 = bytes_eq(tw[3], id);
            if (u == 10) {
              m0 |= bytes_eq(tw[0], AT_INTERCEPTION2);
              m1 |= bytes_eq(tw[1], AT_INTERCEPTION2);
              m2 |= bytes_eq(tw[2], AT_INTERCEPTION2);
              m3 |= bytes_eq(tw[3], AT_INTERCEPTION2);
            }
            st_bool16(args.bout, c + i * N_ATOMIC_NAMES + u, ld, j0, m0, m1, m2, m3);
          }
        }
      }
      c = P.bool_col[SA_XFN_RESULT_ONEHOT];
      if (!ATOMIC && c >= 0) {
        for (int r = 0; r < N_RESULTS; ++r)
          st_bool16(args.bout, c + i * N_RESULTS + r, ld, j0, bytes_eq(rw[0], r), bytes_eq(rw[1], r),
                    bytes_eq(rw[2], r), bytes_eq(rw[3], r));
      }
      c = P.bool_col[SA_XFN_ACTIONTYPE_RESULT_ONEHOT];
      if (!ATOMIC && c >= 0) {
        // code = type*6 + result per byte (type <= 22, result <= 5: no carries between bytes)
        uint32_t cw[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) cw[q] = (tw[q] << 2) + (tw[q] << 1) + rw[q];
        const int64_t cb = c + (int64_t)i * N_TYPES * N_RESULTS;
        for (int code = 0; code < N_TYPES * N_RESULTS; ++code)
          st_bool16(args.bout, cb + code, ld, j0, bytes_eq(cw[0], code), bytes_eq(cw[1], code),
                    bytes_eq(cw[2], code), bytes_eq(cw[3], code));
      }
      c = P.bool_col[SA_XFN_BODYPART_ONEHOT];
      if (c >= 0) {
        for (int b = 0; b < N_BODYPARTS; ++b)
          st_bool16(args.bout, c + i * N_BODYPARTS + b, ld, j0, bytes_eq(bw[0], b),
                    bytes_eq(bw[1], b), bytes_eq(bw[2], b), bytes_eq(bw[3], b));
      }
      c = P.bool_col[SA_XFN_TEAM];
      if (c >= 0 && i >= 1) {  // team_i = team[a_i] == team[a0] (features.py:430-452)
        uint32_t m[4] = {0, 0, 0, 0};
#pragma unroll
        for (int mm = 0; mm < LANE_ACTS; ++mm) {
          int32_t t0, ti;
          if (EXPLICIT) {
            t0 = ld_or0(A.frames[0].team, j0 + mm, n);
            ti = ld_or0(A.frames[i].team, j0 + mm, n);
          } else {
            int d = (int)byte_of(dw[mm >> 2], mm & 3);
            int s = d < i ? d : i;
            t0 = TM[8 + mm];
            ti = pick24(TM, 8 + mm - s);
          }
          m[mm >> 2] |= (uint32_t)(t0 == ti) << (8 * (mm & 3));
        }
        st_bool16(args.bout, c + (i - 1), ld, j0, m[0], m[1], m[2], m[3]);
      }
    }
  }
  __syncthreads();

  // ---------------- phase B: f64 / i64 columns, lane owns 2 consecutive actions ---------------
  const bool any_num =
      P.i64_col[SA_XFN_ACTIONTYPE] >= 0 || P.i64_col[SA_XFN_RESULT] >= 0 ||
      P.i64_col[SA_XFN_BODYPART] >= 0 || P.i64_col[SA_XFN_TIME] >= 0 ||
      P.f64_col[SA_XFN_TIME] >= 0 || P.f64_col[SA_XFN_STARTLOCATION] >= 0 ||
      P.f64_col[SA_XFN_ENDLOCATION] >= 0 || P.f64_col[SA_XFN_STARTPOLAR] >= 0 ||
      P.f64_col[SA_XFN_ENDPOLAR] >= 0 || P.f64_col[SA_XFN_MOVEMENT] >= 0 ||
      P.f64_col[SA_XFN_TIME_DELTA] >= 0 || P.f64_col[SA_XFN_SPACE_DELTA] >= 0 ||
      P.f64_col[SA_XFN_LOCATION] >= 0 || P.f64_col[SA_XFN_POLAR] >= 0 ||
      P.f64_col[SA_XFN_MOVEMENT_POLAR] >= 0 || P.f64_col[SA_XFN_DIRECTION] >= 0;
  if (!any_num || wave_base >= n) return;

  for (int pr = 0; pr < LANE_ACTS / 2; ++pr) {
    const int rel = pr * 2 * WAVE + 2 * lane;  // 0..1022, even
    const int64_t jb = wave_base + rel;
    if (jb >= n) break;
    int64_t jr[2];
    int dd[2];
    bool away[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      int64_t j = jb + e;
      jr[e] = j < n ? j : n - 1;  // padded tail rows recompute the last row
      uint32_t inf = info[wv][rel + e];
      dd[e] = (int)(inf & 0x0F);
      away[e] = (inf >> 4) & 1;
    }
    // a0 values kept for the state features
    double sx0[2], sy0[2], t0[2];
    for (int i = 0; i < K; ++i) {
      const sa_frame& Fi = EXPLICIT ? A.frames[i] : F0;
      double c0[2], c1[2], c2[2], c3[2], ts[2];
      int32_t per[2], typ[2], res[2], bp[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        int64_t r = EXPLICIT ? jr[e] : jr[e] - (dd[e] < i ? dd[e] : i);
        c0[e] = Fi.c0[r];
        c1[e] = Fi.c1[r];
        c2[e] = Fi.c2[r];
        c3[e] = Fi.c3[r];
        ts[e] = Fi.time_seconds[r];
        per[e] = Fi.period_id[r];
        typ[e] = Fi.type_id[r];
        res[e] = ATOMIC ? 0 : Fi.result_id[r];
        bp[e] = Fi.bodypart_id[r];
        if (!EXPLICIT && away[e]) {  // play_left_to_right, keyed on the current action
          c0[e] = FIELD_L - c0[e];
          c1[e] = FIELD_W - c1[e];
          if (ATOMIC) {
            c2[e] = -c2[e];
            c3[e] = -c3[e];
          } else {
            c2[e] = FIELD_L - c2[e];
            c3[e] = FIELD_W - c3[e];
          }
        }
        if (i == 0) {
          sx0[e] = c0[e];
          sy0[e] = c1[e];
          t0[e] = ts[e];
        }
      }
      int c;
      if ((c = P.i64_col[SA_XFN_ACTIONTYPE]) >= 0) st_i64x2(args.iout, c + i, ld, jb, typ[0], typ[1]);
      if ((c = P.i64_col[SA_XFN_RESULT]) >= 0) st_i64x2(args.iout, c + i, ld, jb, res[0], res[1]);
      if ((c = P.i64_col[SA_XFN_BODYPART]) >= 0) st_i64x2(args.iout, c + i, ld, jb, bp[0], bp[1]);
      if ((c = P.i64_col[SA_XFN_TIME]) >= 0) st_i64x2(args.iout, c + i, ld, jb, per[0], per[1]);
      if ((c = P.f64_col[SA_XFN_TIME]) >= 0) {
        st_f64x2(args.fout, c + 2 * i, ld, jb, ts[0], ts[1]);
        // ((period_id - 1) * 45 * 60) + time_seconds   (features.py:313)
        st_f64x2(args.fout, c + 2 * i + 1, ld, jb, (double)((per[0] - 1) * 2700) + ts[0],
                 (double)((per[1] - 1) * 2700) + ts[1]);
      }
      if (!ATOMIC) {
        if ((c = P.f64_col[SA_XFN_STARTLOCATION]) >= 0) {
          st_f64x2(args.fout, c + 2 * i, ld, jb, c0[0], c0[1]);
          st_f64x2(args.fout, c + 2 * i + 1, ld, jb, c1[0], c1[1]);
        }
        if ((c = P.f64_col[SA_XFN_ENDLOCATION]) >= 0) {
          st_f64x2(args.fout, c + 2 * i, ld, jb, c2[0], c2[1]);
          st_f64x2(args.fout, c + 2 * i + 1, ld, jb, c3[0], c3[1]);
        }
        if ((c = P.f64_col[SA_XFN_STARTPOLAR]) >= 0) {
          double dist[2], ang[2];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            double dx = fabs(FIELD_L - c0[e]), dy = fabs(GOAL_Y - c1[e]);
            dist[e] = sqrt(dx * dx + dy * dy);
            ang[e] = polar_angle(dy, dx);
          }
          st_f64x2(args.fout, c + 2 * i, ld, jb, dist[0], dist[1]);
          st_f64x2(args.fout, c + 2 * i + 1, ld, jb, ang[0], ang[1]);
        }
        if ((c = P.f64_col[SA_XFN_ENDPOLAR]) >= 0) {
          double dist[2], ang[2];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            double dx = fabs(FIELD_L - c2[e]), dy = fabs(GOAL_Y - c3[e]);
            dist[e] = sqrt(dx * dx + dy * dy);
            ang[e] = polar_angle(dy, dx);
          }
          st_f64x2(args.fout, c + 2 * i, ld, jb, dist[0], dist[1]);
          st_f64x2(args.fout, c + 2 * i + 1, ld, jb, ang[0], ang[1]);
        }
        if ((c = P.f64_col[SA_XFN_MOVEMENT]) >= 0) {
          double mdx[2], mdy[2], mv[2];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            mdx[e] = c2[e] - c0[e];
            mdy[e] = c3[e] - c1[e];
            mv[e] = sqrt(mdx[e] * mdx[e] + mdy[e] * mdy[e]);
          }
          st_f64x2(args.fout, c + 3 * i, ld, jb, mdx[0], mdx[1]);
          st_f64x2(args.fout, c + 3 * i + 1, ld, jb, mdy[0], mdy[1]);
          st_f64x2(args.fout, c + 3 * i + 2, ld, jb, mv[0], mv[1]);
        }
        if (i >= 1 && (c = P.f64_col[SA_XFN_SPACE_DELTA]) >= 0) {
          double sdx[2], sdy[2], sm[2];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            sdx[e] = c2[e] - sx0[e];
            sdy[e] = c3[e] - sy0[e];
            sm[e] = sqrt(sdx[e] * sdx[e] + sdy[e] * sdy[e]);
          }
          st_f64x2(args.fout, c + 3 * (i - 1), ld, jb, sdx[0], sdx[1]);
          st_f64x2(args.fout, c + 3 * (i - 1) + 1, ld, jb, sdy[0], sdy[1]);
          st_f64x2(args.fout, c + 3 * (i - 1) + 2, ld, jb, sm[0], sm[1]);
        }
      } else {
        if ((c = P.f64_col[SA_XFN_LOCATION]) >= 0) {
          st_f64x2(args.fout, c + 2 * i, ld, jb, c0[0], c0[1]);
          st_f64x2(args.fout, c + 2 * i + 1, ld, jb, c1[0], c1[1]);
        }
        if ((c = P.f64_col[SA_XFN_POLAR]) >= 0) {
          double dist[2], ang[2];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            double dx = fabs(FIELD_L - c0[e]), dy = fabs(GOAL_Y - c1[e]);
            dist[e] = sqrt(dx * dx + dy * dy);
            ang[e] = polar_angle(dy, dx);
          }
          st_f64x2(args.fout, c + 2 * i, ld, jb, dist[0], dist[1]);
          st_f64x2(args.fout, c + 2 * i + 1, ld, jb, ang[0], ang[1]);
        }
        if ((c = P.f64_col[SA_XFN_MOVEMENT_POLAR]) >= 0) {
          double md[2], ma[2];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            md[e] = sqrt(c2[e] * c2[e] + c3[e] * c3[e]);
            ma[e] = (c3[e] == 0.0) ? 0.0 : atan2(c3[e], c2[e]);  // atomic/vaep/features.py:181-200
          }
          st_f64x2(args.fout, c + 2 * i, ld, jb, md[0], md[1]);
          st_f64x2(args.fout, c + 2 * i + 1, ld, jb, ma[0], ma[1]);
        }
        if ((c = P.f64_col[SA_XFN_DIRECTION]) >= 0) {
          double ox[2], oy[2];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            double td = sqrt(c2[e] * c2[e] + c3[e] * c3[e]);
            ox[e] = td > 0.0 ? c2[e] / td : c2[e];  // atomic/vaep/features.py:203-226
            oy[e] = td > 0.0 ? c3[e] / td : c3[e];
          }
          st_f64x2(args.fout, c + 2 * i, ld, jb, ox[0], ox[1]);
          st_f64x2(args.fout, c + 2 * i + 1, ld, jb, oy[0], oy[1]);
        }
      }
      if (i >= 1 && (c = P.f64_col[SA_XFN_TIME_DELTA]) >= 0)
        st_f64x2(args.fout, c + (i - 1), ld, jb, t0[0] - ts[0], t0[1] - ts[1]);
    }
  }
}

// ------------------------------------------------------------------------------------------
// goalscore (features.py:505-539 / atomic/vaep/features.py:313-344): per segment, teamA =
// team of the segment's first row, exclusive cumsum of goals for A and B.
constexpr int GS_THREADS = 256;

template <bool ATOMIC>
__global__ __launch_bounds__(GS_THREADS) void goalscore_kernel(sa_actions A, int64_t* __restrict__ out,
                                                               int64_t ld) {
  __shared__ uint64_t wsum[GS_THREADS / WAVE];
  const int64_t g = blockIdx.x;
  const int64_t s = A.seg_off[g], e = A.seg_off[g + 1];
  if (s >= e) return;
  const sa_frame& F = A.frames[0];
  const int32_t teamA = F.team[s];
  const int lane = threadIdx.x & (WAVE - 1), wv = threadIdx.x / WAVE;
  uint64_t carry = 0;  // low 32: goals team A so far, high 32: goals team B so far
  for (int64_t base = s; base < e; base += 2 * GS_THREADS) {
    int64_t jj[2];
    uint64_t inc[2];
    bool isA[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      int64_t j = base + 2 * threadIdx.x + q;
      jj[q] = j;
      inc[q] = 0;
      isA[q] = false;
      if (j < e) {
        int t = F.type_id[j];
        bool goal, og;
        if (ATOMIC) {
          goal = t == AT_GOAL;
          og = t == AT_OWNGOAL;
        } else {
          bool shot = t == T_SHOT || t == T_SHOT_PENALTY || t == T_SHOT_FREEKICK;
          int r = F.result_id[j];
          goal = shot && r == R_SUCCESS;
          og = shot && r == R_OWNGOAL;
        }
        isA[q] = F.team[j] == teamA;
        bool gA = (goal && isA[q]) || (og && !isA[q]);
        bool gB = (goal && !isA[q]) || (og && isA[q]);
        inc[q] = (uint64_t)gA | ((uint64_t)gB << 32);
      }
    }
    // block exclusive scan of (inc0 + inc1)
    uint64_t x = inc[0] + inc[1];
    uint64_t incl = x;
#pragma unroll
    for (int off = 1; off < WAVE; off <<= 1) {
      uint64_t y = __shfl_up(incl, off, WAVE);
      if (lane >= off) incl += y;
    }
    if (lane == WAVE - 1) wsum[wv] = incl;
    __syncthreads();
    uint64_t wpre = 0, total = 0;
#pragma unroll
    for (int k = 0; k < GS_THREADS / WAVE; ++k) {
      uint64_t v = wsum[k];
      if (k < wv) wpre += v;
      total += v;
    }
    __syncthreads();
    uint64_t excl = carry + wpre + incl - x;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      if (jj[q] < e) {
        int64_t cA = (int64_t)(excl & 0xFFFFFFFFull), cB = (int64_t)(excl >> 32);
        int64_t tm = isA[q] ? cA : cB, op = isA[q] ? cB : cA;
        out[jj[q]] = tm;
        out[ld + jj[q]] = op;
        out[2 * ld + jj[q]] = tm - op;
      }
      excl += inc[q];
    }
    carry += total;
  }
}

// ------------------------------------------------------------------------------------------
// labels (vaep/labels.py:9-116, atomic/vaep/labels.py:9-107).  Lane owns 16 consecutive
// actions; rows j0 .. j0+31 are held as goal/owngoal bit masks + team codes, so the
// look-ahead of nr_actions <= 17 needs no further loads.
template <bool ATOMIC>
__global__ __launch_bounds__(256) void labels_kernel(sa_actions A, int nr, uint8_t* __restrict__ sc,
                                                     uint8_t* __restrict__ co,
                                                     uint8_t* __restrict__ gfs) {
  const int64_t n = A.n;
  const int64_t j0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * LANE_ACTS;
  if (j0 >= n) return;
  const sa_frame& F = A.frames[0];
  int64_t g = find_segment(A.seg_off, A.n_segments, j0);
  int64_t e = A.seg_off[g + 1];
  uint32_t gm = 0, om = 0, sm = 0;  // goal / owngoal / shot(type 11, atomic gfs) bits
  int32_t tm[32];
  uint32_t t27 = 0;                 // atomic: type == goal bits
#pragma unroll
  for (int r = 0; r < 32; ++r) {
    int64_t j = j0 + r;
    int t = 0, res = 0;
    int32_t te = 0;
    if (j < n) {
      t = F.type_id[j];
      res = ATOMIC ? 0 : F.result_id[j];
      te = F.team[j];
    }
    bool goal, og;
    if (ATOMIC) {
      goal = t == AT_GOAL;
      og = t == AT_OWNGOAL;
    } else {
      bool shot = t == T_SHOT || t == T_SHOT_PENALTY || t == T_SHOT_FREEKICK;
      goal = shot && res == R_SUCCESS;
      og = shot && res == R_OWNGOAL;
    }
    gm |= (uint32_t)goal << r;
    om |= (uint32_t)og << r;
    sm |= (uint32_t)(t == T_SHOT) << r;
    t27 |= (uint32_t)(t == AT_GOAL) << r;
    tm[r] = te;
  }
  uint32_t s_out[4] = {0, 0, 0, 0}, c_out[4] = {0, 0, 0, 0}, g_out[4] = {0, 0, 0, 0};
#pragma unroll
  for (int m = 0; m < LANE_ACTS; ++m) {
    int64_t j = j0 + m;
    if (j >= n) break;
    while (j >= e) {
      ++g;
      e = A.seg_off[g + 1];
    }
    const int64_t last = e - 1;  // segment's last row: look-ahead clamps here
    bool scores, concedes;
    const bool goal_j = (gm >> m) & 1, og_j = (om >> m) & 1;
    if (nr <= 17) {
      int64_t hi = j + nr - 1 < last ? j + nr - 1 : last;  // rows j+1 .. hi
      int span = (int)(hi - j);                            // 0 .. 16
      uint32_t win = span > 0 ? (((1u << span) - 1u) << (m + 1)) : 0u;
      uint32_t same = 0;
#pragma unroll
      for (int r = 0; r < 32; ++r) same |= (uint32_t)(tm[r] == tm[m]) << r;
      scores = goal_j || (((gm & same) | (om & ~same)) & win) != 0;
      concedes = og_j || (((gm & ~same) | (om & same)) & win) != 0;
    } else {
      scores = goal_j;
      concedes = og_j;
      const int32_t tj = tm[m];
      for (int i = 1; i < nr; ++i) {
        int64_t c = j + i < last ? j + i : last;
        int t = F.type_id[c];
        bool goal, og;
        if (ATOMIC) {
          goal = t == AT_GOAL;
          og = t == AT_OWNGOAL;
        } else {
          bool shot = t == T_SHOT || t == T_SHOT_PENALTY || t == T_SHOT_FREEKICK;
          int res = F.result_id[c];
          goal = shot && res == R_SUCCESS;
          og = shot && res == R_OWNGOAL;
        }
        bool same = F.team[c] == tj;
        scores |= (goal && same) || (og && !same);
        concedes |= (goal && !same) || (og && same);
      }
    }
    bool gf;
    if (ATOMIC)  // shot followed by goal; the segment's last row compares with NaN -> False
      gf = ((sm >> m) & 1) && j < last && ((t27 >> (m + 1)) & 1);
    else
      gf = goal_j;
    s_out[m >> 2] |= (uint32_t)scores << (8 * (m & 3));
    c_out[m >> 2] |= (uint32_t)concedes << (8 * (m & 3));
    g_out[m >> 2] |= (uint32_t)gf << (8 * (m & 3));
  }
  if (sc) *reinterpret_cast<uint4*>(sc + j0) = make_uint4(s_out[0], s_out[1], s_out[2], s_out[3]);
  if (co) *reinterpret_cast<uint4*>(co + j0) = make_uint4(c_out[0], c_out[1], c_out[2], c_out[3]);
  if (gfs) *reinterpret_cast<uint4*>(gfs + j0) = make_uint4(g_out[0], g_out[1], g_out[2], g_out[3]);
}

// ------------------------------------------------------------------------------------------
// formula (vaep/formula.py:8-151, atomic/vaep/formula.py:8-141).  Arithmetic stays in the
// probability dtype and mirrors the reference's pandas expression tree operation by operation.
template <bool ATOMIC, typename T>
__global__ __launch_bounds__(256) void formula_kernel(sa_actions A, const T* __restrict__ ps,
                                                      const T* __restrict__ pc, T* __restrict__ off,
                                                      T* __restrict__ def, T* __restrict__ val) {
  constexpr int V = 16 / sizeof(T);
  const int64_t n = A.n;
  const int64_t j0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * V;
  if (j0 >= n) return;
  const sa_frame& F = A.frames[0];
  int64_t g = find_segment(A.seg_off, A.n_segments, j0);
  int64_t s = A.seg_off[g], e = A.seg_off[g + 1];
  T vo[V], vd[V], vv[V];
#pragma unroll
  for (int q = 0; q < V; ++q) {
    int64_t j = j0 + q;
    if (j >= n) j = n - 1;
    while (j >= e) {
      ++g;
      s = e;
      e = A.seg_off[g + 1];
    }
    const int64_t p = j > s ? j - 1 : j;  // _prev: shift(1) with row 0 = itself
    const T one = T(1), zero = T(0);
    const bool same = F.team[p] == F.team[j];
    const T fs = same ? one : zero, fn = same ? zero : one;
    T prev_s = ps[p] * fs + pc[p] * fn;
    T prev_c = pc[p] * fs + ps[p] * fn;
    const int tp = F.type_id[p], tj = F.type_id[j];
    bool prevgoal;
    if (ATOMIC) {
      prevgoal = tp == AT_GOAL || tp == AT_OWNGOAL;
    } else {
      const bool toolong = fabs(F.time_seconds[j] - F.time_seconds[p]) > 10.0;  // _samephase_nb
      if (toolong) {
        prev_s = zero;
        prev_c = zero;
      }
      prevgoal = (tp == T_SHOT || tp == T_SHOT_PENALTY || tp == T_SHOT_FREEKICK) &&
                 F.result_id[p] == R_SUCCESS;
    }
    if (prevgoal) {
      prev_s = zero;
      prev_c = zero;
    }
    if (!ATOMIC) {
      if (tj == T_SHOT_PENALTY) prev_s = T(0.792453);
      if (tj == T_CORNER_CROSSED || tj == T_CORNER_SHORT) prev_s = T(0.046500);
    }
    vo[q] = ps[j] - prev_s;
    vd[q] = -(pc[j] - prev_c);
    vv[q] = vo[q] + vd[q];
  }
  if (sizeof(T) == 8) {
    *reinterpret_cast<double2*>(off + j0) = *reinterpret_cast<double2*>(vo);
    *reinterpret_cast<double2*>(def + j0) = *reinterpret_cast<double2*>(vd);
    *reinterpret_cast<double2*>(val + j0) = *reinterpret_cast<double2*>(vv);
  } else {
    *reinterpret_cast<float4*>(off + j0) = *reinterpret_cast<float4*>(vo);
    *reinterpret_cast<float4*>(def + j0) = *reinterpret_cast<float4*>(vd);
    *reinterpret_cast<float4*>(val + j0) = *reinterpret_cast<float4*>(vv);
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
    if (!aligned16(F.type_id) || !aligned16(F.result_id) || !aligned16(F.bodypart_id))
      return fail(SA_EINVAL, "frame %d: id columns must be 16-byte aligned", f);
  }
  return SA_OK;
}

extern "C" int sa_vaep_features(const sa_actions* a, const sa_feature_plan* plan, uint8_t* bool_out,
                                double* f64_out, int64_t* i64_out, int64_t ld, void* stream) {
  int rc = check_actions(a, true);
  if (rc) return rc;
  if (!plan) return fail(SA_EINVAL, "null plan");
  const int K = plan->nb_prev_actions;
  if (K < 1 || K > SA_MAX_FRAMES) return fail(SA_EINVAL, "nb_prev_actions must be in [1, 8]");
  if (a->n_frames > 1 && a->n_frames != K)
    return fail(SA_EINVAL, "explicit mode needs n_frames == nb_prev_actions");
  if (ld % 16 != 0 || ld < ((a->n + 15) / 16) * 16)
    return fail(SA_EINVAL, "ld must be a multiple of 16 and >= round_up(n, 16)");
  bool wb = false, wf = false, wi = false;
  for (int x = 0; x < SA_XFN_COUNT; ++x) {
    wb |= plan->bool_col[x] >= 0;
    wf |= plan->f64_col[x] >= 0;
    wi |= plan->i64_col[x] >= 0;
  }
  if ((wb && !bool_out) || (wf && !f64_out) || (wi && !i64_out))
    return fail(SA_EINVAL, "plan writes a block whose pointer is null");
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
  FeatArgs args{*a, *plan, bool_out, f64_out, i64_out, ld};
  const int64_t waves = (a->n + WAVE_ACTS - 1) / WAVE_ACTS;
  const dim3 grid((unsigned)((waves + BLOCK_WAVES - 1) / BLOCK_WAVES)), block(BLOCK_WAVES * WAVE);
  const bool expl = a->n_frames > 1;
  if (a->atomic) {
    if (expl)
      hipLaunchKernelGGL((features_kernel<true, true>), grid, block, 0, st, args);
    else
      hipLaunchKernelGGL((features_kernel<true, false>), grid, block, 0, st, args);
  } else {
    if (expl)
      hipLaunchKernelGGL((features_kernel<false, true>), grid, block, 0, st, args);
    else
      hipLaunchKernelGGL((features_kernel<false, false>), grid, block, 0, st, args);
  }
  rc = check_launch("features_kernel");
  if (rc) return rc;
  const int gc = plan->i64_col[SA_XFN_GOALSCORE];
  if (gc >= 0) rc = sa_vaep_goalscore(a, i64_out + (int64_t)gc * ld, ld, stream);
  return rc;
}

extern "C" int sa_vaep_goalscore(const sa_actions* a, int64_t* out, int64_t ld, void* stream) {
  int rc = check_actions(a, true);
  if (rc) return rc;
  if (!out) return fail(SA_EINVAL, "null goalscore output");
  if (ld < a->n) return fail(SA_EINVAL, "ld < n");
  if (a->n == 0) return SA_OK;
  hipStream_t st = (hipStream_t)stream;
  if (a->atomic)
    hipLaunchKernelGGL((goalscore_kernel<true>), dim3((unsigned)a->n_segments), dim3(GS_THREADS), 0, st,
                       *a, out, ld);
  else
    hipLaunchKernelGGL((goalscore_kernel<false>), dim3((unsigned)a->n_segments), dim3(GS_THREADS), 0,
                       st, *a, out, ld);
  return check_launch("goalscore_kernel");
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
  if (a->atomic)
    hipLaunchKernelGGL((labels_kernel<true>), grid, block, 0, (hipStream_t)stream, *a, nr_actions,
                       scores, concedes, goal_from_shot);
  else
    hipLaunchKernelGGL((labels_kernel<false>), grid, block, 0, (hipStream_t)stream, *a, nr_actions,
                       scores, concedes, goal_from_shot);
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
  if (a->atomic)
    hipLaunchKernelGGL((formula_kernel<true, T>), grid, block, 0, (hipStream_t)stream, *a, ps, pc, off,
                       def, val);
  else
    hipLaunchKernelGGL((formula_kernel<false, T>), grid, block, 0, (hipStream_t)stream, *a, ps, pc,
                       off, def, val);
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
