// Expected Threat (xT) fit on large grids -- e.g. the 105 x 68 grid of BASELINE cfg5: C = 7140
// cells, 51M transition bins -- for gfx950.  Reference: socceraction/xthreat.py.
//
// 1. Band-owned transition count (xthreat.py:40-67 `_count`, :177-218 `move_transition_matrix`)
//    without global atomics.  Random int32 atomics into the 204 MB transition table execute at
//    the memory side, one uncached request per lane (MI355X_MICROARCH.md "Global float atomics":
//    64 lanes in 64 rows ~0.08 TB/s); the round-3 XC_VEC pass sat on that ceiling (0.446 ms per
//    16M actions).  Here the start cells are cut into bands of R consecutive cells and every
//    counted action becomes one 4-B key (start cell << 16 | slot), bucketed as a 16-bit bin:
//      K1 xt_keys_kernel        reads the actions once, writes each workgroup's keys contiguously
//                               (wave ballots) and the keys per band;
//      K3 xt_keys_scatter_kernel  the band offsets (every workgroup scans the band counts
//                               itself; the first one also writes them out), a counting sort of
//                               each workgroup's keys by band in LDS, then runs of keys into the
//                               band buckets;
//      K4 xt_band_count_kernel  one workgroup per band: its R rows x (C + 3) bins as u32 in LDS
//                               (143 KB at 105 x 68), filled from the band's bucket(s), flushed
//                               once with coalesced stores -- the shot / goal / move counts of
//                               the band's cells come from the same bins (slots C, C + 1, C + 2).
//    K1-K3 run per batch of actions (sa_xt_count_bucket); K4 runs once over the buckets of every
//    batch (sa_xt_count_from_buckets), so the 204 MB table is written once per fit.
// 2. Value iteration (xthreat.py:278-320) over a compact form of the counts built once per solve
//    (sa_xt_compact_rows): each row's non-zero counts in column order, 4 B each (column | count
//    << 16), chunk-interleaved per row.  Per iteration (xt_iter_ell_kernel) eight product waves
//    form T[r, c] * x[c] = (cnt / move[r]) * x[c] -- the correctly rounded quotient from the
//    row's reciprocal and one fma correction -- and one chain wave adds each row's products
//    strictly left to right (the reference's loop order; zero terms add +0 to a non-negative sum,
//    so skipping them keeps every bit).  62.5 MB per cfg5 iteration instead of the 204 MB dense
//    int32 rows.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "sa_common.h"
#include "sa_internal.h"

namespace sa {

// ============================================================================ band-owned count
#ifndef SA_XK_PROBE
#define SA_XK_PROBE 0  // diagnostic builds (wrong counts): 1 = no band histogram, 2 = no key stores
#endif
#ifndef SA_XK_THREADS
#define SA_XK_THREADS 1024  // K1 workgroup (118 VGPRs with the rate operands: one per CU, 16 waves; 512: the same, r04ae)
#endif
constexpr int XK_THREADS = SA_XK_THREADS;
#ifndef SA_XK_U
#define SA_XK_U 2  // K1 actions per thread per pass (coordinates; even; 4: 146.5 vs 143.4 us per 16M, r06k2)
#endif
static_assert(SA_XK_U >= 2 && SA_XK_U % 2 == 0 && SA_XK_U <= 16, "SA_XK_U");
#ifndef SA_XK_PIPE
#define SA_XK_PIPE 0  // 1: K1's coordinate passes software-pipelined (the next pass's loads issued
#endif                //    before this pass's arithmetic; two register buffers, alternating)
#ifndef SA_XK_BALANCE
#define SA_XK_BALANCE 1  // K1 regions per batch rounded up to whole rounds of the CUs (shorter regions)
#endif
#ifndef SA_XK_NT
#define SA_XK_NT 3  // bit 0: non-temporal coordinate / id loads in K1, bit 1: non-temporal operand stores
                    // (read once per fit; cfg5 batch 0.263 -> 0.251 ms, profiles/r04_xt_count_ab.md)
#endif
template <typename T>
__device__ __forceinline__ T xk_ld(const T* p) {
  if constexpr ((SA_XK_NT & 1) != 0) return __builtin_nontemporal_load(p);
  return *p;
}
template <typename T>
__device__ __forceinline__ void xk_st(T* p, T v) {
  if constexpr ((SA_XK_NT & 2) != 0) __builtin_nontemporal_store(v, p);
  else *p = v;
}
constexpr int XK_CHUNK = 32768;     // actions per K1 workgroup = key capacity of its region
constexpr int XS_THREADS = 1024;    // K3 workgroup
#ifndef SA_XS_SPLIT
#define SA_XS_SPLIT 1  // K3 workgroups per K1 region (2 / 4 parts: two per CU, slower; r04_xt_count_ab.md)
#endif
constexpr int XS_SPLIT = SA_XS_SPLIT;
constexpr int XS_PART = XK_CHUNK / XS_SPLIT;  // keys per K3 workgroup
constexpr int XS_PER = XS_PART / XS_THREADS;
constexpr int XB_THREADS = 1024;    // K4 workgroup
#ifndef SA_XB_RMAX
#define SA_XB_RMAX 8  // start cells per band at most (105 x 68: 5 = the most 160 KB of LDS holds)
#endif
constexpr int XB_MAX_ROWS = 8;      // start cells per band (LDS row sums)
static_assert(SA_XB_RMAX >= 1 && SA_XB_RMAX <= XB_MAX_ROWS, "SA_XB_RMAX");
constexpr int XB_NB_MAX = 4000;     // bands (K3 holds 2 words per band + a region's keys in LDS)
constexpr size_t XB_LDS_MAX = 160 * 1024;
constexpr int XB_MAX_SETS = 24;     // buckets per K4 launch
// K4's static LDS (row sums, set pointers and bounds), reserved out of XB_LDS_MAX before the
// dynamic R x P bins are sized (100 x 68 at R = 6 would ask 163,296 + 640 B of 163,840)
// + the compact-row staging rings (xe_emit: 256 entries per row)
constexpr size_t XB_LDS_STATIC = 1024 + (size_t)XB_MAX_ROWS * 256 * 4;
static_assert(XB_MAX_ROWS * 8 + XB_MAX_SETS * 24 + XB_MAX_ROWS * 256 * 4 <= XB_LDS_STATIC, "K4 static LDS");
constexpr uint32_t XB_NONE = 0xFFFFFFFFu;
// A bucketed key (K3's output, K4's and the band exchange's input) is 16 bits: the key's bin in
// its band's LDS histogram, (start cell - band * R) * P + slot -- K4 adds 1 at h[key] with no
// decode.  R * P <= (160 KB - static) / 4 < 65535 for every band shape (static_assert below), so
// 0xFFFF never is a bin.  Half the bytes of the 4-B keys K3 wrote before round 6 (K3's stores,
// K4's loads and the multi-GPU all-to-all).
typedef uint16_t xb_key_t;
static_assert((XB_LDS_MAX - XB_LDS_STATIC) / 4 < 0xFFFFu, "a band's bins fit 16-bit bucket keys");
constexpr uint32_t XE_CNT_ESC_K4 = 0xFFFFu;  // = XE_CNT_ESC: a count >= 65535 is read from the dense row
static_assert(XS_PER * XS_THREADS * XS_SPLIT == XK_CHUNK && XS_PER >= 1, "K3 holds one part of a K1 region");
static_assert(XS_PART * 4 + 2 * XB_NB_MAX * 4 + 256 <= XB_LDS_MAX, "K3 LDS");

struct XbShape {
  int C;           // cells
  int R;           // start cells per band
  int NB;          // bands
  int P;           // LDS pitch of a band row in K4 (>= C + 3, multiple of 4)
  uint64_t magic;  // band of start cell cs = (cs * magic) >> 32 = cs / R for cs < 2^16
};

__device__ __forceinline__ uint32_t band_of(uint32_t key, uint64_t magic) {
  return (uint32_t)(((uint64_t)(key >> 16) * magic) >> 32);
}

// One action -> its key (false: not counted).  Slots: the end cell of a successful move with
// finite coordinates (a transition; also counted in move), C = shot, C + 1 = scored shot,
// C + 2 = a move without a transition.  Same non-finite rules and error bytes as count_one
// (sa_xt.hip): a NaN start drops the action from _count, a cast of a non-finite coordinate
// raises in the reference.
__device__ __forceinline__ bool band_key(const XtAct& a, int C, uint32_t& key, int32_t& bad) {
  uint32_t slot;
  if (a.cls == XT_CELL_SHOT) {
    if (a.snan) return false;
    if (!a.sfin) {
      bad |= XT_ERRB_SHOT;
      return false;
    }
    slot = (uint32_t)C + (a.succ ? 1u : 0u);
  } else if (a.cls == XT_CELL_MOVE) {
    if (a.snan) {
      bad |= XT_ERRB_MOVE_OTHER;
      return false;
    }
    if (!a.sfin) {
      bad |= XT_ERRB_MOVE_START;
      return false;
    }
    if (!a.efin) {
      bad |= XT_ERRB_MOVE_OTHER;
      slot = (uint32_t)C + 2u;
    } else {
      slot = a.succ ? (uint32_t)a.ce : (uint32_t)C + 2u;
    }
  } else {
    return false;
  }
  // only a malformed cell code fails these: never an LDS bin past the bands or a band row
  if ((uint32_t)a.cs >= (uint32_t)C || slot > (uint32_t)C + 2u) return false;
  key = ((uint32_t)a.cs << 16) | slot;
  return true;
}

__device__ __forceinline__ uint32_t lane_rank(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Per-action rate operands the coordinate pass can write while it holds the coordinates:
// codes = sa_xt_count_codes' u32 operand of a rate on the (l, w) grid; icodes = the u64 operand
// of a rate(use_interpolation=True) on the L x W node grid (start node | end node << 32 of a
// successful move, XT_ICODE_BAD / XT_ICODE_NAN as rate_code's markers).
struct XkRate {
  uint32_t* codes;
  uint64_t* icodes;
  int L, W;
};

// K1: region r = actions [r * XK_CHUNK, (r + 1) * XK_CHUNK) -> keys[r * XK_CHUNK + i], i <
// region_cnt[r]; band_cnt[b] += the region's keys of band b.  CELLS: 4-B cell codes
// (sa_xt_cells, C <= SA_XT_CELLS_MAX_C) instead of the coordinates (no rate operands then).
// vec (coordinates): the columns are 16-byte (f64) / 2-byte (ids) aligned, so a lane loads two
// consecutive actions per column instruction (16-B and 2-B loads, half the load instructions).
template <bool CELLS>
__global__ __launch_bounds__(XK_THREADS) void xt_keys_kernel(sa_actions A, const uint32_t* __restrict__ cells,
                                                             int64_t n, int l, int w, XbShape S,
                                                             uint32_t* __restrict__ keys,
                                                             uint32_t* __restrict__ region_cnt,
                                                             uint32_t* __restrict__ band_cnt,
                                                             int32_t* __restrict__ err, XkRate RO, int vec,
                                                             int64_t chunk) {
  extern __shared__ uint32_t bh[];  // [NB]
  __shared__ uint32_t cursor;
  for (int b = threadIdx.x; b < S.NB; b += XK_THREADS) bh[b] = 0;
  if (threadIdx.x == 0) cursor = 0;
  __syncthreads();
  const int64_t begin = (int64_t)blockIdx.x * chunk;  // chunk <= XK_CHUNK, even
  const int64_t end = min(n, begin + chunk);
  uint32_t* out = keys + (int64_t)blockIdx.x * XK_CHUNK;
  const sa_frame& F = A.frames[0];
  const int lane = threadIdx.x & 63;
  int32_t bad = 0;
  constexpr int U = CELLS ? 8 : SA_XK_U;  // actions per thread per pass, every load issued first
  // the keys of one pass's actions: ballot ranks into the region, band histogram in LDS
  auto emit_keys = [&](const XtAct (&act)[U]) {
    uint32_t key[U];
    bool has[U];
    uint64_t m[U];
    uint32_t tot = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      has[u] = band_key(act[u], S.C, key[u], bad);
      m[u] = __ballot(has[u]);
      tot += (uint32_t)__popcll(m[u]);
    }
    uint32_t wbase = 0;
    if (lane == 0 && tot) wbase = atomicAdd(&cursor, tot);
    wbase = __shfl(wbase, 0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (has[u]) {
        const uint32_t pos = wbase + lane_rank(m[u]);
        SA_DGUARD(pos < XK_CHUNK, pos, continue);
        if (!(SA_XK_PROBE & 2)) out[pos] = key[u];
        if (!(SA_XK_PROBE & 1)) atomicAdd(&bh[band_of(key[u], S.magic)], 1u);
      }
      wbase += (uint32_t)__popcll(m[u]);
    }
  };
  if constexpr (!CELLS && SA_XK_PIPE) {
    if (vec) {  // wave-uniform
      constexpr int Q = U / 2;  // pairs per thread per pass
      struct Raw {
        f64x2 a[Q], b[Q], c[Q], d[Q];
        uint32_t ty[Q], rs[Q];
      };
      auto load = [&](Raw& R, int64_t base) {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          const int64_t j = base + 2 * ((int64_t)q * XK_THREADS + threadIdx.x);
          const int64_t jc = j + 1 < end ? j : ((end - 2) & ~(int64_t)1);  // a whole aligned pair
          R.a[q] = xk_ld(reinterpret_cast<const f64x2*>(F.c0 + jc));
          R.b[q] = xk_ld(reinterpret_cast<const f64x2*>(F.c1 + jc));
          R.c[q] = xk_ld(reinterpret_cast<const f64x2*>(F.c2 + jc));
          R.d[q] = xk_ld(reinterpret_cast<const f64x2*>(F.c3 + jc));
          R.ty[q] = xk_ld(reinterpret_cast<const uint16_t*>(F.type_id + jc));
          R.rs[q] = xk_ld(reinterpret_cast<const uint16_t*>(F.result_id + jc));
        }
      };
      auto pass = [&](const Raw& R, int64_t base) {
        int tt[U], rr[U];
        double sx[U], sy[U], ex[U], ey[U];
        int64_t jj[U];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          const int64_t j = base + 2 * ((int64_t)q * XK_THREADS + threadIdx.x);
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int u = 2 * q + e;
            jj[u] = j + e;
            sx[u] = R.a[q][e];
            sy[u] = R.b[q][e];
            ex[u] = R.c[q][e];
            ey[u] = R.d[q][e];
            tt[u] = (int)((R.ty[q] >> (8 * e)) & 0xFF);
            rr[u] = (int)((R.rs[q] >> (8 * e)) & 0xFF);
          }
          if (j + 1 >= end) {  // the batch's odd last action (or none): scalar, the rest not counted
            const int64_t k = j < end ? j : end - 1;
            sx[2 * q] = F.c0[k];
            sy[2 * q] = F.c1[k];
            ex[2 * q] = F.c2[k];
            ey[2 * q] = F.c3[k];
            tt[2 * q] = j < end ? (int)F.type_id[k] : -1;
            rr[2 * q] = F.result_id[k];
            tt[2 * q + 1] = -1;
          }
        }
        BinQ bq[U];
#pragma unroll
        for (int u = 0; u < U; ++u) bq[u] = bin_q(sx[u], sy[u], ex[u], ey[u]);
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          const int u = 2 * q;
          const int64_t j = jj[u];
          if (RO.codes && tt[u] >= 0) {
            const uint32_t c0 = rate_code_q(tt[u], rr[u], sx[u], sy[u], ex[u], ey[u], bq[u], l, w);
            if (tt[u + 1] >= 0)
              *reinterpret_cast<uint2*>(RO.codes + j) = make_uint2(
                  c0, rate_code_q(tt[u + 1], rr[u + 1], sx[u + 1], sy[u + 1], ex[u + 1], ey[u + 1], bq[u + 1], l, w));
            else
              RO.codes[j] = c0;
          }
          if (RO.icodes && tt[u] >= 0) {
            const uint64_t c0 = rate_icode_q(tt[u], rr[u], sx[u], sy[u], ex[u], ey[u], bq[u], RO.L, RO.W);
            if (tt[u + 1] >= 0)
              xk_st(reinterpret_cast<u64x2*>(RO.icodes + j),
                    u64x2{c0, rate_icode_q(tt[u + 1], rr[u + 1], sx[u + 1], sy[u + 1], ex[u + 1], ey[u + 1], bq[u + 1],
                                           RO.L, RO.W)});
            else
              RO.icodes[j] = c0;
          }
        }
        XtAct act[U];
#pragma unroll
        for (int u = 0; u < U; ++u) act[u] = act_from_row_q(tt[u], rr[u], sx[u], sy[u], ex[u], ey[u], bq[u], l, w);
        emit_keys(act);
      };
      const int64_t step = (int64_t)U * XK_THREADS;
      Raw ra, rb;  // alternate: no register copy of a load in flight
      load(ra, begin);
      for (int64_t base = begin; base < end; base += 2 * step) {  // wave-uniform bounds
        if (base + step < end) load(rb, base + step);
        pass(ra, base);
        if (base + step >= end) break;
        if (base + 2 * step < end) load(ra, base + 2 * step);
        pass(rb, base + step);
      }
    }
  }
  for (int64_t base = begin; base < end && !(!CELLS && SA_XK_PIPE && vec); base += (int64_t)U * XK_THREADS) {
    XtAct act[U];
    if (CELLS) {
      uint32_t cv[U];
      const bool c16 = xt_c16(S.C);  // 16-bit codes (grids of <= SA_XT_CELLS16_MAX_C cells), as xt_count_kernel
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t j = base + u * XK_THREADS + threadIdx.x, jc = j < end ? j : end - 1;
        cv[u] = c16 ? (uint32_t)reinterpret_cast<const uint16_t*>(cells)[jc] : cells[jc];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        act[u] = c16 ? decode_cell16(cv[u], S.C) : decode_cell(cv[u]);
        if (base + u * XK_THREADS + threadIdx.x >= end) act[u].cls = 0;
      }
    } else {
      // action u of the pass: j = base + 2 (p * XK_THREADS + tid) + e, u = 2 p + e (vec), or
      // j = base + u * XK_THREADS + tid; rows past `end` are clamped and not counted
      int tt[U], rr[U];
      double sx[U], sy[U], ex[U], ey[U];
      int64_t jj[U];
      if (vec) {
#pragma unroll
        for (int q = 0; q < U / 2; ++q) {
          const int64_t j = base + 2 * ((int64_t)q * XK_THREADS + threadIdx.x);
          const int64_t jc = j + 1 < end ? j : ((end - 2) & ~(int64_t)1);  // a whole aligned pair
          const f64x2 a = xk_ld(reinterpret_cast<const f64x2*>(F.c0 + jc)), b = xk_ld(reinterpret_cast<const f64x2*>(F.c1 + jc));
          const f64x2 c = xk_ld(reinterpret_cast<const f64x2*>(F.c2 + jc)), d = xk_ld(reinterpret_cast<const f64x2*>(F.c3 + jc));
          const uint32_t ty = xk_ld(reinterpret_cast<const uint16_t*>(F.type_id + jc));
          const uint32_t rs = xk_ld(reinterpret_cast<const uint16_t*>(F.result_id + jc));
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int u = 2 * q + e;
            jj[u] = j + e;
            sx[u] = a[e];
            sy[u] = b[e];
            ex[u] = c[e];
            ey[u] = d[e];
            tt[u] = (int)((ty >> (8 * e)) & 0xFF);
            rr[u] = (int)((rs >> (8 * e)) & 0xFF);
          }
          if (j + 1 >= end) {  // the batch's odd last action (or none): scalar, the rest not counted
            const int64_t k = j < end ? j : end - 1;
            sx[2 * q] = F.c0[k];
            sy[2 * q] = F.c1[k];
            ex[2 * q] = F.c2[k];
            ey[2 * q] = F.c3[k];
            tt[2 * q] = j < end ? (int)F.type_id[k] : -1;
            rr[2 * q] = F.result_id[k];
            tt[2 * q + 1] = -1;
          }
        }
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t j = base + u * XK_THREADS + threadIdx.x;
          const int64_t jc = j < end ? j : end - 1;
          jj[u] = j;
          tt[u] = j < end ? F.type_id[jc] : -1;
          rr[u] = F.result_id[jc];
          sx[u] = F.c0[jc];
          sy[u] = F.c1[jc];
          ex[u] = F.c2[jc];
          ey[u] = F.c3[jc];
        }
      }
      BinQ bq[U];  // the binning's quotients, once per action for the count and the rate operands
#pragma unroll
      for (int u = 0; u < U; ++u) bq[u] = bin_q(sx[u], sy[u], ex[u], ey[u]);
      if (vec) {  // a pair's two operands in one store (16 B: whole lines per instruction)
#pragma unroll
        for (int q = 0; q < U / 2; ++q) {
          const int u = 2 * q;
          const int64_t j = jj[u];
          if (RO.codes && tt[u] >= 0) {
            const uint32_t c0 = rate_code_q(tt[u], rr[u], sx[u], sy[u], ex[u], ey[u], bq[u], l, w);
            if (tt[u + 1] >= 0)
              *reinterpret_cast<uint2*>(RO.codes + j) = make_uint2(
                  c0, rate_code_q(tt[u + 1], rr[u + 1], sx[u + 1], sy[u + 1], ex[u + 1], ey[u + 1], bq[u + 1], l, w));
            else
              RO.codes[j] = c0;
          }
          if (RO.icodes && tt[u] >= 0) {
            const uint64_t c0 = rate_icode_q(tt[u], rr[u], sx[u], sy[u], ex[u], ey[u], bq[u], RO.L, RO.W);
            if (tt[u + 1] >= 0)
              xk_st(reinterpret_cast<u64x2*>(RO.icodes + j),
                    u64x2{c0, rate_icode_q(tt[u + 1], rr[u + 1], sx[u + 1], sy[u + 1], ex[u + 1], ey[u + 1], bq[u + 1],
                                           RO.L, RO.W)});
            else
              RO.icodes[j] = c0;
          }
        }
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t j = jj[u];
          if (RO.codes && tt[u] >= 0) RO.codes[j] = rate_code_q(tt[u], rr[u], sx[u], sy[u], ex[u], ey[u], bq[u], l, w);
          if (RO.icodes && tt[u] >= 0)
            RO.icodes[j] = rate_icode_q(tt[u], rr[u], sx[u], sy[u], ex[u], ey[u], bq[u], RO.L, RO.W);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) act[u] = act_from_row_q(tt[u], rr[u], sx[u], sy[u], ex[u], ey[u], bq[u], l, w);
    }
    emit_keys(act);
  }
  if (bad) atomicOr(err, bad);
  __syncthreads();
  for (int b = threadIdx.x; b < S.NB; b += XK_THREADS)
    if (bh[b]) atomicAdd(&band_cnt[b], bh[b]);
  if (threadIdx.x == 0) region_cnt[blockIdx.x] = cursor;
}

// Exclusive scan of a[0, n) in place by one NT-thread workgroup; returns the total (to every
// thread).  ws: NT / 64 + 1 words of LDS.
template <int NT>
__device__ uint32_t block_scan(uint32_t* a, int n, uint32_t* ws) {
  constexpr int NW = NT / 64;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int per = (n + NT - 1) / NT;
  const int lo = min(n, t * per), hi = min(n, lo + per);
  uint32_t s = 0;
  for (int i = lo; i < hi; ++i) s += a[i];
  uint32_t inc = s;  // inclusive wave scan
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t v = __shfl_up(inc, d);
    if (lane >= d) inc += v;
  }
  if (lane == 63) ws[wv] = inc;
  __syncthreads();
  if (t == 0) {
    uint32_t run = 0;
    for (int k = 0; k < NW; ++k) {
      const uint32_t v = ws[k];
      ws[k] = run;
      run += v;
    }
    ws[NW] = run;
  }
  __syncthreads();
  uint32_t run = ws[wv] + inc - s;
  for (int i = lo; i < hi; ++i) {
    const uint32_t v = a[i];
    a[i] = run;
    run += v;
  }
  const uint32_t total = ws[NW];
  __syncthreads();
  return total;
}
__device__ uint32_t block_scan_1024(uint32_t* a, int n, uint32_t* ws) { return block_scan<1024>(a, n, ws); }


// K3: XS_SPLIT workgroups per K1 region, one per part of its keys (<= XS_PART, XS_PER per thread in registers), ranked
// within their band by LDS atomics, each band's run gets its place in the band's bucket by ONE
// global atomic on the band cursor, the keys are sorted by band in LDS, and thread i writes the
// sorted key i -- consecutive threads of a run write consecutive words.
__global__ __launch_bounds__(XS_THREADS) void xt_keys_scatter_kernel(const uint32_t* __restrict__ keys,
                                                                     const uint32_t* __restrict__ region_cnt,
                                                                     XbShape S, const uint32_t* __restrict__ band_cnt,
                                                                     int64_t* __restrict__ band_off,
                                                                     uint32_t* __restrict__ cursor,
                                                                     xb_key_t* __restrict__ buckets) {
  extern __shared__ uint32_t sm[];
  uint32_t* bh = sm;              // [NB] keys per band, then the local run offsets
  uint32_t* bb = sm + S.NB;       // [NB] the bands' offsets, then the runs' places in the buckets
  uint32_t* sorted = sm + 2 * S.NB;  // [XS_PART]
  __shared__ uint32_t ws[17];
  // the band offsets: every workgroup scans K1's band counts itself (5.7 KB at cfg5, from L2)
  // instead of waiting for a one-workgroup scan launch; the first writes them out for K4
  for (int b = threadIdx.x; b < S.NB; b += XS_THREADS) bb[b] = band_cnt[b];
  __syncthreads();
  const uint32_t total = block_scan_1024(bb, S.NB, ws);
  if (blockIdx.x == 0) {
    for (int b = threadIdx.x; b < S.NB; b += XS_THREADS) band_off[b] = bb[b];
    if (threadIdx.x == 0) band_off[S.NB] = total;
  }
  const int region = blockIdx.x / XS_SPLIT, part = blockIdx.x % XS_SPLIT;
  const uint32_t rc = region_cnt[region], p0 = (uint32_t)part * XS_PART;
  const uint32_t cnt = rc > p0 ? min(rc - p0, (uint32_t)XS_PART) : 0u;
  const uint32_t* in = keys + (int64_t)region * XK_CHUNK + p0;
  for (int b = threadIdx.x; b < S.NB; b += XS_THREADS) bh[b] = 0;
  uint32_t k[XS_PER], rk[XS_PER];
#pragma unroll
  for (int u = 0; u < XS_PER; ++u) {
    const uint32_t i = u * XS_THREADS + threadIdx.x;
    k[u] = i < cnt ? in[i] : XB_NONE;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < XS_PER; ++u) {
    rk[u] = 0;
    if (k[u] != XB_NONE) {
      const uint32_t b = band_of(k[u], S.magic);
      SA_DGUARD(b < (uint32_t)S.NB, b, continue);
      rk[u] = atomicAdd(&bh[b], 1u);
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < S.NB; b += XS_THREADS) {  // cursor: zeroed with the band counts
    const uint32_t c = bh[b];
    bb[b] = c ? bb[b] + atomicAdd(&cursor[b], c) : 0u;
  }
  __syncthreads();
  block_scan_1024(bh, S.NB, ws);
#pragma unroll
  for (int u = 0; u < XS_PER; ++u)
    if (k[u] != XB_NONE) {
      const uint32_t b = band_of(k[u], S.magic);
      SA_DGUARD(b < (uint32_t)S.NB, b, continue);
      sorted[bh[b] + rk[u]] = k[u];
    }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < cnt; i += XS_THREADS) {
    const uint32_t key = sorted[i];
    const uint32_t b = band_of(key, S.magic);
    SA_DGUARD(b < (uint32_t)S.NB, b, continue);
    // the key's bin in its band's histogram (K4's LDS index): row within the band, slot
    buckets[bb[b] + (i - bh[b])] = (xb_key_t)(((key >> 16) - b * (uint32_t)S.R) * (uint32_t)S.P + (key & 0xFFFFu));
  }
}

struct XbSets {
  const xb_key_t* keys[XB_MAX_SETS];
  const int64_t* off[XB_MAX_SETS];
  int n;
};

// K4: workgroup lb = band b = band0 + lb = start cells [b R, b R + R).  Bins h[i][slot] (i < R,
// slot < C + 3) as u32 in LDS, filled by LDS atomics from every set's bucket of the band (set s:
// keys[s][off[s][lb] .. off[s][lb + 1])), then flushed: the transition rows with coalesced 16-B
// stores (vec) or 4-B stores, the shot / goal / move counts of each cell from slots C, C + 1,
// C + 2 and the row sum.  The outputs hold rows from band0 * R on (a rank's row block, or the
// whole table with band0 = 0).  overwrite: the rows and counts are written, not added to (a
// fresh accumulator: no read of the old rows).
// One wave writes a row's compact form (xt_ell_build_kernel's layout: the k-th non-zero count
// of the row, column | min(count, 0xFFFF) << 16, at slot (k & ~127) | (k & 31) << 2 | (k >> 5) & 3)
// 512 columns at a time (v[u] = the count at column c0 + 64 u + lane, 0 past the row): entries
// are ranked by ballot + mbcnt into a 256-entry LDS ring S, and every complete chunk of 128 goes
// out as 32 lanes x 16 B -- whole 512-B runs.  (Scattered 4-B stores left lines half written when
// L2 evicted them: each partial line cost the memory a read-modify-write, 60 us per cfg5 table.)
// Call with base = done = 0; after the last group, xe_emit_tail.
__device__ __forceinline__ void xe_emit_group(const uint32_t (&v)[8], int c0, uint32_t* __restrict__ E,
                                              uint32_t* S, int lane, int& base, int& done) {
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const uint64_t m = __ballot(v[u] != 0);
    if (v[u] != 0) {
      const uint32_t cnt = v[u] < XE_CNT_ESC_K4 ? v[u] : XE_CNT_ESC_K4;
      S[(base + (int)lane_rank(m)) & 255] = (uint32_t)(c0 + 64 * u + lane) | (cnt << 16);
    }
    base += (int)__popcll(m);
    if (base - done >= 128) {  // wave-uniform: a whole chunk is staged
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the ring writes land before the reads
      if (lane < 32) {
        const int o = done & 255;
        const uint4 q = {S[o + lane], S[o + lane + 32], S[o + lane + 64], S[o + lane + 96]};
        *reinterpret_cast<uint4*>(E + done + 4 * lane) = q;
      }
      done += 128;
    }
  }
}
__device__ __forceinline__ void xe_emit_tail(uint32_t* __restrict__ E, const uint32_t* S, int lane, int base, int done) {
  __builtin_amdgcn_s_waitcnt(0xc07f);
  if (lane < 32)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = done + lane + 32 * j;
      if (k < base) E[done + 4 * lane + j] = S[k & 255];
    }
}

// ell (optional, with overwrite): the band's rows also in the compact form of
// xt_ell_build_kernel, emitted from the bins (ell + row * pe, row_len[row]) -- the solve then
// skips its build pass and its 204 MB read of the table.  dense = 0 (with ell): the dense rows
// are written only for a band that holds a transition count >= 65535 (the one entry the compact
// form escapes to its dense row); every other band's dense rows stay unwritten -- 204 MB of
// stores a fit that reads only the compact rows does not need (sa_xt_count_from_buckets_ex
// with SA_XT_COUNT_COMPACT_ONLY).
__device__ __forceinline__ int xe_slot(int k);
__global__ __launch_bounds__(XB_THREADS) void xt_band_count_kernel(XbSets sets, XbShape S, int band0,
                                                                   unsigned long long* __restrict__ shot,
                                                                   unsigned long long* __restrict__ goal,
                                                                   unsigned long long* __restrict__ move,
                                                                   int32_t* __restrict__ trans, int overwrite,
                                                                   int vec, uint32_t* __restrict__ ell,
                                                                   int32_t* __restrict__ row_len, int pe,
                                                                   int dense) {
  extern __shared__ __attribute__((aligned(16))) uint32_t h[];  // [R][P]
  __shared__ unsigned long long msum[XB_MAX_ROWS];
  __shared__ uint32_t esc;  // dense = 0: the band holds a transition count >= 65535
  const int lb = blockIdx.x, b = band0 + lb, C = S.C, P = S.P;
  const int r0 = b * S.R, nr = min(S.R, C - r0);
  const int orow = r0 - band0 * S.R;  // the band's first row in the outputs
  for (int e = 4 * threadIdx.x; e < nr * P; e += 4 * XB_THREADS) *reinterpret_cast<u32x4*>(h + e) = u32x4{0, 0, 0, 0};
  if (threadIdx.x < XB_MAX_ROWS) msum[threadIdx.x] = 0;
  if (threadIdx.x == 0) esc = 0;
  // the band's keys, set after set, in tiles of XB_U keys per thread, two tiles in flight (the
  // next tile's loads are issued before the current tile's LDS atomics; one tile at a time
  // waited out a memory latency per 4 keys and per set: 148 us per cfg5 table pass).  Set
  // bounds and key pointers in LDS (global address space: no FLAT loads, whose lgkmcnt would
  // tie them to the LDS reads)
  typedef const xb_key_t __attribute__((address_space(1)))* gkeys;
  __shared__ gkeys kb[XB_MAX_SETS];
  __shared__ int64_t klo[XB_MAX_SETS], khi[XB_MAX_SETS];
  const int ns = sets.n;
  if (threadIdx.x < ns) {
    kb[threadIdx.x] = (gkeys)sets.keys[threadIdx.x];
    klo[threadIdx.x] = sets.off[threadIdx.x][lb];
    khi[threadIdx.x] = sets.off[threadIdx.x][lb + 1];
  }
  __syncthreads();
  constexpr int XB_U = 16;
  constexpr int64_t XB_TILE = (int64_t)XB_U * XB_THREADS;
  auto skip_empty = [&](int& ts, int64_t& ti) {  // (ts, ti): a tile of set ts from key ti; ts == ns: none
    while (ts < ns && klo[ts] >= khi[ts]) ++ts;
    if (ts < ns) ti = klo[ts];
  };
  auto next_tile = [&](int& ts, int64_t& ti) {
    if (ts >= ns) return;
    ti += XB_TILE;
    if (ti >= khi[ts]) {
      ++ts;
      skip_empty(ts, ti);
    }
  };
  auto load = [&](uint32_t (&v)[XB_U], int ts, int64_t ti) {
    if (ts >= ns) {
#pragma unroll
      for (int u = 0; u < XB_U; ++u) v[u] = XB_NONE;
      return;
    }
    const gkeys kp = kb[ts];
    const int64_t hi = khi[ts];
#pragma unroll
    for (int u = 0; u < XB_U; ++u) {
      const int64_t j = ti + u * XB_THREADS + threadIdx.x;
      v[u] = j < hi ? (uint32_t)kp[j] : XB_NONE;
    }
  };
  auto count = [&](const uint32_t (&v)[XB_U]) {
#pragma unroll
    for (int u = 0; u < XB_U; ++u)
      if (v[u] != XB_NONE) {  // the key is the bin (K3: row within the band * P + slot)
          SA_DGUARD(v[u] < (uint32_t)(nr * P) && (int)(v[u] % (uint32_t)P) < C + 3, v[u], continue);
          atomicAdd(&h[v[u]], 1u);
        }
  };
  int sa = 0, sb;
  int64_t ia = 0, ib;
  skip_empty(sa, ia);
  sb = sa;
  ib = ia;
  next_tile(sb, ib);
  uint32_t va[XB_U], vb[XB_U];
  load(va, sa, ia);
  load(vb, sb, ib);
  for (;;) {  // slots a / b alternate (no register copy of a load in flight)
    if (sa >= ns) break;
    count(va);
    sa = sb;
    ia = ib;
    next_tile(sa, ia);
    load(va, sa, ia);
    if (sb >= ns) break;
    count(vb);
    sb = sa;
    ib = ia;
    next_tile(sb, ib);
    load(vb, sb, ib);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  // with ell, the first nr waves emit the compact rows (one row each) WHILE the others flush the
  // dense rows: the emission is a chain of dependent LDS steps (~9 us per band) that would
  // otherwise idle the CU after the flush
  const int f0 = ell ? 64 * nr : 0, fth = XB_THREADS - f0;
  if ((int)threadIdx.x >= f0) {
    const int ft = threadIdx.x - f0;
    uint32_t big = 0;  // dense = 0: the largest transition count this thread saw
    for (int i = 0; i < nr; ++i) {
      const uint32_t* hr = h + i * P;
      int32_t* dst = trans + (int64_t)(orow + i) * C;
      unsigned long long ms = 0;
      if (!dense) {  // the row sums (and the escape test) only: no dense stores
        if (vec)
          for (int c = 4 * ft; c < C; c += 4 * fth) {
            const u32x4 v = *reinterpret_cast<const u32x4*>(hr + c);
            ms += (unsigned long long)v[0] + v[1] + v[2] + v[3];
            big = max(big, max(max(v[0], v[1]), max(v[2], v[3])));
          }
        else
          for (int c = ft; c < C; c += fth) {
            ms += hr[c];
            big = max(big, hr[c]);
          }
      } else if (vec) {  // C % 4 == 0 and trans 16-byte aligned: every row starts 16-byte aligned
        for (int c = 4 * ft; c < C; c += 4 * fth) {
          const u32x4 v = *reinterpret_cast<const u32x4*>(hr + c);
          ms += (unsigned long long)v[0] + v[1] + v[2] + v[3];
          i32x4 o = {(int32_t)v[0], (int32_t)v[1], (int32_t)v[2], (int32_t)v[3]};
          if (!overwrite) {
            const i32x4 old = *reinterpret_cast<const i32x4*>(dst + c);
            o += old;
          }
          *reinterpret_cast<i32x4*>(dst + c) = o;
        }
      } else {
        for (int c = ft; c < C; c += fth) {
          const uint32_t v = hr[c];
          ms += v;
          dst[c] = overwrite ? (int32_t)v : dst[c] + (int32_t)v;
        }
      }
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) ms += __shfl_xor(ms, d);
      if (lane == 0 && ms) atomicAdd(&msum[i], ms);
    }
    if (big >= XE_CNT_ESC_K4) esc = 1u;  // benign race: every writer stores 1
  } else {  // ell: wave i emits row i (xe_emit_group)
    __shared__ uint32_t ring[XB_MAX_ROWS][256];
    const int i = threadIdx.x >> 6;
    const uint32_t* hr = h + i * P;
    uint32_t* E = ell + (int64_t)(orow + i) * pe;
    int base = 0, done = 0;
    for (int c0 = 0; c0 < C; c0 += 64 * 8) {
      uint32_t v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int c = c0 + 64 * u + lane;
        v[u] = c < C ? hr[c] : 0u;
      }
      xe_emit_group(v, c0, E, ring[i], lane, base, done);
    }
    xe_emit_tail(E, ring[i], lane, base, done);
    if (lane == 0) row_len[orow + i] = base;
  }
  __syncthreads();
  if (!dense && esc) {  // workgroup-uniform: an escaped count's dense row is read by the solve
    for (int i = 0; i < nr; ++i) {  // (dense = 0 comes with ell, so with overwrite)
      const uint32_t* hr = h + i * P;
      int32_t* dst = trans + (int64_t)(orow + i) * C;
      for (int c = threadIdx.x; c < C; c += XB_THREADS) dst[c] = (int32_t)hr[c];
    }
  }
  if (threadIdx.x < nr) {
    const int i = threadIdx.x, r = orow + i;
    const uint32_t* hr = h + i * P;
    const unsigned long long sh = (unsigned long long)hr[C] + hr[C + 1], gl = hr[C + 1];
    const unsigned long long mv = msum[i] + hr[C + 2];
    if (overwrite) {
      shot[r] = sh;
      goal[r] = gl;
      move[r] = mv;
    } else {
      shot[r] += sh;
      goal[r] += gl;
      move[r] += mv;
    }
  }
}

// ============================================================================ compact iteration
constexpr int XE_S = 32;                     // rows per workgroup (slice) = chain lanes
constexpr int XE_P = 8;                      // product waves: rows p, p + 8, p + 16, p + 24
constexpr int XE_RPW = XE_S / XE_P;          // rows per product wave
constexpr int XE_KC = 128;                   // entries per row per chunk
constexpr int XE_PAIRS = XE_RPW / 2;         // row pairs per product wave (a 16-B load per pair)
constexpr int XE_PITCH = XE_KC + 2;          // prod row pitch (doubles): 16-B aligned rows whose
                                             // 16-B chain reads hit every bank once per 16 lanes
constexpr int XE_CT_MAX = 256;               // counts whose quotient is tabulated: CT = the largest
                                             // power of two <= 256 whose table fits next to x
#ifndef SA_XE_DEPTH
#define SA_XE_DEPTH 4                        // chunks of entries in flight per product lane
#endif
#ifndef SA_XE_NTL
#define SA_XE_NTL 0                          // 1: non-temporal entry loads
#endif
constexpr int XE_DEPTH = SA_XE_DEPTH;
#ifndef SA_XE_QDIV
#define SA_XE_QDIV 1                         // 1: quotients cnt / move by a corrected product with
#endif                                       //    the row's reciprocal; 0: per-row LDS table
constexpr int XE_THREADS = (XE_P + 1) * 64;  // + the chain wave
constexpr int XE_XMAX = 9472;                // x (C doubles) staged in LDS
constexpr int XE_BUILD_ROWS = 16;            // build: rows per workgroup (one wave each)
constexpr uint32_t XE_CNT_ESC = 0xFFFFu;     // count >= 65535: read from the dense row
#ifndef SA_XE_PROBE
#define SA_XE_PROBE 0  // diagnostic builds (wrong values): 1 = no products,
#endif                 // 4 = idle product waves (no loads, no LDS writes; the chain then reads LDS
                       // nobody wrote and may be folded away: no chain timing), 8 = no division path,
                       // 16 = workgroup 0's phase times (wall clock ticks) in x_next[0..3],
                       // 32 = its work / barrier clocks per wave in x_next[40..43], 64 = product
                       // waves without LDS traffic (x = the column, no product stores)
static_assert(XE_KC == 128 && XE_PAIRS * 2 * XE_P == XE_S, "xt_iter_ell_kernel shape: 32 lanes x 4 entries per row chunk");
static_assert(XE_THREADS <= 1024 && XE_S <= 64, "xt_iter_ell_kernel shape");
constexpr size_t XE_LDS_STATIC = (size_t)XE_S * (2 * XE_PITCH + 2) * 8 + XE_S * 4;
constexpr size_t XE_LDS_MAX = 160 * 1024;
static_assert((size_t)XE_XMAX * 8 + (size_t)XE_S * 16 * 8 + XE_LDS_STATIC <= XE_LDS_MAX,
              "xt_iter_ell_kernel LDS: x and a 16-count quotient table");
static_assert(XE_DEPTH >= 1 && XE_DEPTH <= 8, "SA_XE_DEPTH");

// A compact row's pitch in entries: C rounded up to whole chunks (room for a dense row).
__host__ __device__ constexpr int xe_pitch(int C) { return (C + XE_KC - 1) / XE_KC * XE_KC; }
// Storage slot of a row's k-th entry: chunk-interleaved, so the 16-B group at slot 4 l of a chunk
// holds its entries l, l + 32, l + 64, l + 96 -- one 16-B load per lane, yet each LDS instruction
// of the products (x at the columns, the product stores) spans 32 consecutive entries: columns
// close together, distinct banks (entries 4 apart would put a dense row's columns 32 B apart,
// eight lanes on a bank pair).
__device__ __forceinline__ int xe_slot(int k) { return (k & ~(XE_KC - 1)) | ((k & 31) << 2) | ((k >> 5) & 3); }
static_assert(XE_CNT_ESC_K4 == XE_CNT_ESC, "K4's compact rows escape counts like xt_ell_build_kernel");

// Compact form of rows [0, nrows) of a count block (row i at cnt_rows + i*C): row i's non-zero
// counts in column order, column | min(count, 0xFFFF) << 16, the k-th at ell[i*pe + xe_slot(k)]
// (pe = xe_pitch(C)), and their number at row_len[i].  One wave per row: 8 loads of 64 columns
// in flight, ballot + mbcnt for each entry's rank.
__global__ __launch_bounds__(XE_BUILD_ROWS * 64) void xt_ell_build_kernel(const int32_t* __restrict__ cnt_rows, int C,
                                                                          int nrows, uint32_t* __restrict__ ell,
                                                                          int32_t* __restrict__ row_len) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * XE_BUILD_ROWS + (threadIdx.x >> 6);
  if (r >= nrows) return;  // whole wave
  const int32_t* row = cnt_rows + (int64_t)r * C;
  uint32_t* E = ell + (int64_t)r * xe_pitch(C);
  __shared__ uint32_t ring[XE_BUILD_ROWS][256];
  int base = 0, done = 0;
  for (int c0 = 0; c0 < C; c0 += 64 * 8) {
    uint32_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int c = c0 + 64 * u + lane;
      v[u] = c < C ? (uint32_t)__builtin_nontemporal_load(row + c) : 0u;
    }
    xe_emit_group(v, c0, E, ring[threadIdx.x >> 6], lane, base, done);
  }
  xe_emit_tail(E, ring[threadIdx.x >> 6], lane, base, done);
  if (lane == 0) row_len[r] = base;
}

// One iteration of rows [rb, rb + nrows) from their compact form (xt_ell_build_kernel of the same
// rows; cnt_rows: the dense rows, read only for counts >= 65535): xo[i] = gs + pmove * sum over
// the row's non-zero columns c, in column order, of (cnt / move[r]) * x[c] -- xt_iter_kernel's
// operations (sa_xt.hip), without its per-chunk compaction of the dense rows.  One workgroup per
// slice of 32 rows.  Per chunk of KC entries per row, each product wave loads its 4 rows'
// entries (256 contiguous bytes per load; DEPTH - 1 chunks ahead), forms the products -- the
// quotient cnt / move[row] (QDIV: y = cnt * r, r = 1 / move[row] rounded; then
// y + r * (cnt - y * move) by two fmas, Markstein's correction: the correctly rounded quotient, the
// division's own bits -- scripts/check_quotient.c checks it exhaustively for cnt < 65536 against
// 6000 + 6001 divisors and on 4e8 random pairs up to 2^53; no LDS read, no table), times x at
// the column -- and writes them to prod[row][k]; the chain wave (lane = row) then adds its row's products strictly in order.  One barrier per
// chunk, two buffers; a row shorter than the slice's longest costs nothing past its end (its
// product lanes and its chain lane skip those chunks).
__global__ __launch_bounds__(XE_THREADS) void xt_iter_ell_kernel(const uint32_t* __restrict__ ell,
                                                                 const int32_t* __restrict__ row_len,
                                                                 const int32_t* __restrict__ cnt_rows,
                                                                 const unsigned long long* __restrict__ move,
                                                                 const double* __restrict__ gs,
                                                                 const double* __restrict__ pmove, int C, int rb,
                                                                 int nrows, int ct, double eps,
                                                                 const double* __restrict__ x,
                                                                 double* __restrict__ xo, const int32_t* flag_prev,
                                                                 int32_t* __restrict__ flag_out) {
  if (flag_prev && __hip_atomic_load(flag_prev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
#if SA_XE_PROBE & 16
  const long long t_entry = wall_clock64();
#endif
  extern __shared__ __attribute__((aligned(16))) double xs[];  // [C] x, then tq [S][ct]
  [[maybe_unused]] double* tq = xs + C;                        // tq[i * ct + q] = q / move[row i]
  __shared__ double prod[2][XE_S * XE_PITCH];
  __shared__ double mvs[XE_S], rcp[XE_S];
  __shared__ int lens[XE_S];
  const int row0 = blockIdx.x * XE_S, nr = min(XE_S, nrows - row0);
  const int pe = xe_pitch(C);
  // staging: every global load of x, move and row_len issued before the first LDS store (a
  // load-store loop would wait out one memory latency per 576 elements: ~13 at C = 7140)
  constexpr int XR = (XE_XMAX + XE_THREADS - 1) / XE_THREADS;
  double xr[XR];
#pragma unroll
  for (int u = 0; u < XR; ++u) xr[u] = x[min((int)threadIdx.x + u * XE_THREADS, C - 1)];
  const int t = threadIdx.x;
  const double mv0 = t < nr ? (double)move[rb + row0 + min(t, nr - 1)] : 1.0;
  const int len0 = t < nr ? row_len[row0 + min(t, nr - 1)] : 0;
#pragma unroll
  for (int u = 0; u < XR; ++u)
    if (t + u * XE_THREADS < C) xs[t + u * XE_THREADS] = xr[u];
  if (t < XE_S) {
    mvs[t] = mv0;
    rcp[t] = 1.0 / mv0;
    lens[t] = len0;
  }
  __syncthreads();
#if !SA_XE_QDIV
  const int lct = __builtin_ctz(ct);  // ct: a power of two
  for (int e = t; e < XE_S * ct; e += XE_THREADS) {
    const int q = e & (ct - 1);
    tq[e] = q == 0 ? 0.0 : (double)q / mvs[e >> lct];  // a count of 0 is a zero term (T = 0)
  }
  __syncthreads();
#endif
  int len = 0;
#pragma unroll
  for (int i = 0; i < XE_S; ++i) len = max(len, lens[i]);
#if SA_XE_PROBE & 16
  const long long t_setup = wall_clock64();
#endif
  const int nch = (len + XE_KC - 1) / XE_KC;
  const int nchp = (nch + XE_DEPTH - 1) / XE_DEPTH * XE_DEPTH;  // chunks past nch: +0 terms
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (wv < XE_P) {  // ---- product waves
#if SA_XE_PROBE & 4
    for (int j = 0; j < nchp; ++j) __syncthreads();
    return;
#endif
    // wave wv owns rows wv + 8 q (q < 4) as two pairs: half = lane / 32 takes row
    // wv + 8 (2 p + half) of pair p, lane l = lane % 32 its entries l + 32 u (u < 4) of each
    // chunk (one 16-B load of slots 4 l..4 l + 3: a wave instruction fetches 1 KiB, two rows'
    // chunks)
    const int half = lane >> 5, l32 = lane & 31;
    const uint32_t* Er[XE_PAIRS];
    int lr[XE_PAIRS], ir[XE_PAIRS];
    double mq[XE_PAIRS], rq[XE_PAIRS];  // the rows' move count and its rounded reciprocal
#pragma unroll
    for (int p = 0; p < XE_PAIRS; ++p) {
      const int i = wv + XE_P * (2 * p + half);
      ir[p] = i;
      mq[p] = mvs[i];
      rq[p] = rcp[i];
      Er[p] = ell + (int64_t)(row0 + min(i, nr - 1)) * pe;
      lr[p] = lens[i];
    }
    // DEPTH register slots of entries, slot d holding chunk j with j % DEPTH == d: the loop is
    // unrolled by DEPTH so a slot's loads are refilled right after its products are formed and
    // no register is copied while its load is in flight (a copy waits for the load); loads are
    // unconditional from addresses clamped to the row's last entries (a slice's HBM / Infinity
    // Cache bytes are its rows' entries only: one CU pulls ~30-70 GB/s, so the slice holding the
    // longest row would otherwise stream every row to that length), entries past a row's end
    // zeroed at their use
    u32x4 e[XE_DEPTH][XE_PAIRS];
    int jmax[XE_PAIRS];  // each row's last chunk: an ended row's loads re-read it (cache hits)
#pragma unroll
    for (int p = 0; p < XE_PAIRS; ++p) jmax[p] = lr[p] > 0 ? (lr[p] - 1) / XE_KC : 0;
    auto ld = [&](u32x4 (&d)[XE_PAIRS], int j) {
#pragma unroll
      for (int p = 0; p < XE_PAIRS; ++p) {
        const int k = min(j, jmax[p]) * XE_KC + 4 * l32;
#if SA_XE_NTL
        d[p] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(Er[p] + k));
#else  // default policy: the compact rows (~70 MB at cfg5) stay in the Infinity Cache across iterations
        d[p] = *reinterpret_cast<const u32x4*>(Er[p] + k);
#endif
      }
    };
    auto products = [&](const u32x4 (&E)[XE_PAIRS], int j) {
      double* pr = prod[j & 1];
      // every LDS read of the chunk first (x at the column; without QDIV the quotient from the
      // table at min(cnt, ct - 1); entries past a row's end are 0: T = 0, x[0]), then the rare
      // escaped counts (without QDIV: counts >= ct), then the products: no branch between a read
      // and its use, so the reads overlap
      double tv[XE_PAIRS][4], xv[XE_PAIRS][4];
      uint32_t en[XE_PAIRS][4];
      bool big = false, live[XE_PAIRS];
#pragma unroll
      for (int p = 0; p < XE_PAIRS; ++p) live[p] = j * XE_KC < lr[p];  // the row has entries in chunk j
#pragma unroll
      for (int p = 0; p < XE_PAIRS; ++p)
        if (live[p])  // an ended row costs no LDS traffic: its chain lane skips the chunk
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          en[p][u] = j * XE_KC + 32 * u + l32 < lr[p] ? E[p][u] : 0u;
          const uint32_t cnt = en[p][u] >> 16, col = en[p][u] & 0xFFFFu;
          SA_DCHECK((int)col < C, col);
#if SA_XE_PROBE & 64
          xv[p][u] = (double)col;
#else
          xv[p][u] = xs[col < (uint32_t)C ? col : 0u];
#endif
#if SA_XE_QDIV
          const double q = (double)cnt, y = q * rq[p];  // a count of 0 is a zero term (T = 0)
          tv[p][u] = __builtin_fma(__builtin_fma(-y, mq[p], q), rq[p], y);
          big |= cnt == XE_CNT_ESC;
#else
          tv[p][u] = tq[ir[p] * ct + min(cnt, (uint32_t)ct - 1u)];
          big |= cnt >= (uint32_t)ct;
#endif
        }
      if (__builtin_expect(__ballot(big) != 0, 0) && !(SA_XE_PROBE & 8)) {
#pragma unroll
        for (int p = 0; p < XE_PAIRS; ++p)
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const uint32_t cnt = en[p][u] >> 16, col = en[p][u] & 0xFFFFu;
            if (live[p] && cnt >= (uint32_t)(SA_XE_QDIV ? XE_CNT_ESC : ct)) {
              const int32_t c32 = cnt == XE_CNT_ESC ? cnt_rows[(int64_t)(row0 + ir[p]) * C + col] : (int32_t)cnt;
              tv[p][u] = (double)c32 / mq[p];
            }
          }
      }
#pragma unroll
      for (int p = 0; p < XE_PAIRS; ++p) {
        if (!live[p]) continue;
        double* dst = pr + ir[p] * XE_PITCH + l32;
#pragma unroll
        for (int u = 0; u < 4; ++u)
#if SA_XE_PROBE & 64
          if (tv[p][u] * xv[p][u] == -1.0) dst[32 * u] = 0.0;
#elif SA_XE_PROBE & 1
          dst[32 * u] = 0.0 * tv[p][u];
#else
          dst[32 * u] = tv[p][u] * xv[p][u];
#endif
      }
    };
#pragma unroll
    for (int d = 0; d < XE_DEPTH; ++d) ld(e[d], d);
    asm volatile("" ::: "memory");
#if SA_XE_PROBE & 32
    long long pw_work = 0, pw_bar = 0, pw_t = clock64();
#endif
    for (int j0 = 0; j0 < nchp; j0 += XE_DEPTH) {
#pragma unroll
      for (int d = 0; d < XE_DEPTH; ++d) {
        products(e[d], j0 + d);
        ld(e[d], j0 + d + XE_DEPTH);  // past the last chunk: harmless clamped re-reads
        asm volatile("" ::: "memory");
#if SA_XE_PROBE & 32
        const long long t1 = clock64();
        pw_work += t1 - pw_t;
#endif
        __syncthreads();
#if SA_XE_PROBE & 32
        pw_t = clock64();
        pw_bar += pw_t - t1;
#endif
      }
    }
#if SA_XE_PROBE & 32
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      xo[40] = (double)pw_work;
      xo[41] = (double)pw_bar;
    }
#endif
#if SA_XE_PROBE & 16
    if (blockIdx.x == 0 && threadIdx.x == 0) xo[3] = (double)(wall_clock64() - t_entry);
#endif
  } else {  // ---- chain wave: lane i adds row i's products strictly left to right
    // the critical path of the launch (the longest row's adds): first claim on its SIMD's issue
    // slots over the two product waves sharing it (MI355X_MICROARCH.md: priority, then age)
    __builtin_amdgcn_s_setprio(3);
    const int i = lane & (XE_S - 1), li = lane < XE_S ? lens[i] : 0;  // lanes >= S idle
    // the adds are LDS-fed: each 16-B read (2 products) costs the wave ~5 clocks of issue
    // whatever its active lanes and however far ahead it is issued, on top of the ~5-clock
    // dependent f64 add (scratch microbenchmarks: 10.35 clocks per add fed from LDS, 5.2 from
    // registers) -- the longest row's ~6000 adds bound the launch
    double acc = 0.0;
#if SA_XE_PROBE & 32
    long long cw_work = 0, cw_bar = 0, cw_t = clock64();
#endif
    for (int j = 0; j < nchp; ++j) {
#if SA_XE_PROBE & 32
      {
        const long long t1 = clock64();
        cw_work += t1 - cw_t;
        __syncthreads();
        cw_t = clock64();
        cw_bar += cw_t - t1;
      }
#else
      __syncthreads();
#endif
      if (j * XE_KC >= li) continue;  // row ended (or idle lane): no reads, no +0 adds
      const f64x2* pr = reinterpret_cast<const f64x2*>(prod[j & 1] + i * XE_PITCH);
      constexpr int G = 16;  // 16-B reads (two products each) issued a group ahead of their adds
      f64x2 v[G];
#pragma unroll
      for (int k = 0; k < G; ++k) v[k] = pr[k];
#pragma unroll
      for (int k0 = 0; k0 < XE_KC / 2; k0 += G) {
        f64x2 nx[G];
#pragma unroll
        for (int k = 0; k < G; ++k) nx[k] = k0 + G + k < XE_KC / 2 ? pr[k0 + G + k] : f64x2{0.0, 0.0};
#pragma unroll
        for (int k = 0; k < G; ++k) {
          acc = acc + v[k][0];
          acc = acc + v[k][1];
        }
#pragma unroll
        for (int k = 0; k < G; ++k) v[k] = nx[k];
      }
    }
    if (lane < nr) {
      const int rr = rb + row0 + lane;
      const double mv = pmove[rr] * acc;
      const double nx = gs[rr] + mv;
      xo[row0 + lane] = nx;
      if ((nx - x[rr]) > eps) atomicOr(flag_out, 1);  // np.any(diff > eps): NaN is False
    }
#if SA_XE_PROBE & 32  // shader clocks of work / barrier wait, chain wave (42, 43), product wave 0 (40, 41)
    if (blockIdx.x == 0 && lane == 0) {
      xo[42] = (double)(cw_work + (clock64() - cw_t));
      xo[43] = (double)cw_bar;
    }
#endif
#if SA_XE_PROBE & 16  // wall clock (100 MHz) ticks from entry: setup done, chain done, (3) products done
    if (blockIdx.x == 0 && lane == 0) {
      xo[0] = (double)nchp;
      xo[1] = (double)(t_setup - t_entry);
      xo[2] = (double)(wall_clock64() - t_entry);
    }
#endif
  }
}

// ============================================================================ reordered solve
// The whole value iteration in ONE launch with the row sums reordered (xthreat.py:303-317 fixes
// a left-to-right order; north_star allows 1e-6 relative on xT surfaces, only the iteration count
// must be the reference's).  One 512-thread workgroup per CU holds its rows' compact entries in
// REGISTERS (and LDS for the few that do not fit) for every iteration -- 62.5 MB at cfg5 = 244 KB
// per CU of a 512 KB register file -- so an iteration reads no count from memory: it stages x
// (C doubles) into LDS, forms its rows' sums and hands its new x values to every other workgroup
// through a grid barrier.
//
// Sum order (fixed, so every run gives the same bits): a row's 128-entry chunk ("unit") is summed
// by a half-wave -- each lane its 4 entries in order by fmas of the count and x, then a fixed
// 32-lane tree (recursive halving over 8 units at a time) -- and the row's unit sums by 8 lanes
// (lane j: units j, j + 8, ... in order; then a fixed 8-lane tree); the row sum is divided by the
// row's move count once.  Against the reference's sequential sum of the correctly rounded
// (cnt / m) * x[c] terms, both are sums of the same non-negative terms in some order, so with
// n <= C terms each differs from the exact sum S by at most (n + 2) u S (u = 2^-53), and the two
// by (2 C + 8) u S.  Across iterations a relative difference e_t of x becomes at most
// e_t + (2 C + 16) u in the next x (T substochastic, everything non-negative).  The decision
// `diff > eps` of a cell is therefore the reference's whenever |diff - eps| exceeds
// e_{t+1} (x_{t+1} + x_t) plus the subtraction's rounding; a cell inside that margin flags the
// solve as ambiguous and the caller re-solves it in the reference's order (xt_iter_ell_kernel).
// Without an ambiguous cell every decision, and so the iteration count, is the reference's; the
// iterates differ from the reference's by at most e_t relative (26 iterations at 105 x 68:
// <= 4e-11; measured 7e-15).
//
// Hand-off (MI355X_MICROARCH.md, visibility, Valid forms row 1): each workgroup stores its new x
// values write-through (agent-scope atomic stores) into a FRESH 128-B aligned row of a scratch
// history (a line is never read before it is written), every storing wave drains its stores,
// one lane arrives at the barrier; every load of handed-off words is an sc1 load (16-B buffer
// loads).  The barrier is XCD-hierarchical (workgroups b and b + 8 share an XCD): one counter per
// group, the group's last arriver adds to the top counter, the last group's last arriver writes
// every group's generation word, which the group's workgroups poll.  Every poll is bounded (1 s
// of the wall clock): a workgroup that times out sets the abort word and every workgroup leaves
// at its next barrier; the host then re-solves in the reference's order.
constexpr int XF_THREADS = 512;   // 2 waves per SIMD: 256 VGPRs each, half of them entries
constexpr int XF_HALVES = XF_THREADS / 32;  // half-waves per workgroup
constexpr int XF_G = 8;                     // units reduced together by a half-wave
#ifndef SA_XF_PAIR
#define SA_XF_PAIR 2  // units per pipeline stage: the next stage's x reads are in flight meanwhile
#endif
constexpr int XF_PAIR = SA_XF_PAIR;
static_assert(XF_G % XF_PAIR == 0, "SA_XF_PAIR");
#ifndef SA_XF_KREG
#define SA_XF_KREG 32  // units per half-wave held in registers
#endif
constexpr int XF_KREG = SA_XF_KREG;
static_assert(XF_KREG % XF_G == 0 && XF_KREG >= XF_G && XF_KREG <= 48, "SA_XF_KREG");
constexpr int XF_KOV_MAX = 16;  // units per half-wave held in LDS past the registers (the rest
                                // are re-read from the compact rows every iteration)
constexpr int XF_UNIT_BYTES = 32 * 16;      // a unit: 32 lanes x 16 B
constexpr int XF_X16 = (XE_XMAX / 2 + XF_THREADS - 1) / XF_THREADS;  // 16-B loads of x per thread
constexpr int XF_ROWL = 8;                  // lanes per row in the row phase
constexpr long long XF_SPIN_TICKS = 100000000;  // 1 s of the 100 MHz wall clock
// the first barrier: every workgroup of a resident grid arrives within microseconds of the
// launch; one that waits 50 ms shares the GPU with another persistent grid (two processes on
// one device: each may hold some CUs and wait for the rest) and gives up early
constexpr long long XF_SPIN_TICKS_FIRST = 5000000;
// control words (int32, zeroed before the launch), each counter on a 128-B line of its own:
// timeout, ambiguous, iterations (line 0), the top arrival counter (line 1), per group g & 7 its
// arrival counter (lines 2..9) and generation (lines 10..17), then one flag per iteration (some
// cell moved by more than eps)
constexpr int XF_ABORT = 1, XF_AMB = 2, XF_NITER = 3, XF_TOP = 32, XF_GRP = 64, XF_GEN = 64 + 8 * 32,
              XF_FLAGS = 64 + 16 * 32;
#ifndef SA_XF_PROBE
#define SA_XF_PROBE 0  // 1: workgroup 0's wall-clock ticks per phase in control words 4..7 (stderr);
#endif                 // diagnostic builds (wrong values): 2 = conflict-free x reads, 4 = no lane tree
__device__ __forceinline__ uint32_t xf_col(uint32_t e, int q) {
#if SA_XF_PROBE & 2
  return (uint32_t)((threadIdx.x & 63) + 64 * q) + (e & 0x10000u ? 1u : 0u);
#else
  (void)q;
  return e & 0xFFFFu;
#endif
}
typedef uint32_t __attribute__((address_space(1))) xf_gu32;
typedef unsigned long long __attribute__((address_space(1))) xf_gu64;

__device__ __forceinline__ uint32_t xf_ld32(const int32_t* p) {
  return __hip_atomic_load((xf_gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void xf_st32(int32_t* p, uint32_t v) {
  __hip_atomic_store((xf_gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t xf_add32(int32_t* p, uint32_t v) {
  return __hip_atomic_fetch_add((xf_gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Poll *p (relaxed sc1 loads, s_sleep between) until >= target; false on the abort word or the
// wall-clock bound (which then sets it).
__device__ bool xf_wait(int32_t* ctrl, int32_t* p, uint32_t target, long long limit) {
  const long long t0 = wall_clock64();
  while (xf_ld32(p) < target) {
    if (xf_ld32(ctrl + XF_ABORT)) return false;
    if (wall_clock64() - t0 > limit) {
      xf_st32(ctrl + XF_ABORT, 1u);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

// Largest i in [0, nrl) with luo[i] <= gu (luo ascending, luo[0] <= gu < luo[nrl]).
__device__ __forceinline__ int xf_locate(const int32_t* luo, int nrl, int gu) {
  int lo = 0, hi = nrl;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (luo[mid] <= gu)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

// Lane l32's 4 entries (l32 + 32 q, q < 4) of global unit gu: row ra + i, chunk gu - luo[i];
// entries past the row's end read as 0 (count 0, column 0: a +0 term).
__device__ __forceinline__ u32x4 xf_unit(const uint32_t* __restrict__ ell, const int32_t* __restrict__ row_len,
                                         const int32_t* luo, int nrl, int ra, int pe, int gu, int l32) {
  const int i = xf_locate(luo, nrl, gu);
  const int j = gu - luo[i];
  const int len = row_len[ra + i];
  u32x4 e = *reinterpret_cast<const u32x4*>(ell + (int64_t)(ra + i) * pe + j * XE_KC + 4 * l32);
  const int k = j * XE_KC + l32;
  e[0] = k < len ? e[0] : 0u;
  e[1] = k + 32 < len ? e[1] : 0u;
  e[2] = k + 64 < len ? e[2] : 0u;
  e[3] = k + 96 < len ? e[3] : 0u;
  return e;
}

__device__ __forceinline__ bool xf_has_esc(const u32x4& e) {
  return (e[0] >> 16) == XE_CNT_ESC || (e[1] >> 16) == XE_CNT_ESC || (e[2] >> 16) == XE_CNT_ESC ||
         (e[3] >> 16) == XE_CNT_ESC;
}

// Cross-lane moves without LDS (DPP and gfx950's v_permlane16_swap): a reduction through
// ds_bpermute paid the LDS latency at every one of its dependent levels (5.3 of 8.7 us per
// iteration at cfg5, probe build SA_XF_PROBE & 4).
template <int CTRL>
__device__ __forceinline__ double xf_dpp(double v) {  // DPP row op on both dwords
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
constexpr int XF_DPP_QUAD_XOR1 = 0xB1, XF_DPP_QUAD_XOR2 = 0x4E, XF_DPP_ROW_MIRROR = 0x140,
              XF_DPP_ROW_HALF_MIRROR = 0x141;
// a's lanes 16-31 <-> b's lanes 0-15 (and 48-63 <-> 32-47): each 32-lane half with itself
__device__ __forceinline__ void xf_swap16(double& a, double& b) {
  const long long x = __double_as_longlong(a), y = __double_as_longlong(b);
  const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)x, (unsigned)y, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(x >> 32), (unsigned)(y >> 32), false, false);
  a = __longlong_as_double((long long)(((unsigned long long)hi[0] << 32) | lo[0]));
  b = __longlong_as_double((long long)(((unsigned long long)hi[1] << 32) | lo[1]));
}

// 8 unit values per lane -> the sum over the half-wave's 32 lanes of unit (l32 >> 2) & 7, in
// lanes with l32 % 4 == 0 (and their 3 neighbours), by a fixed tree: recursive halving over the
// lane pairs (l, l + 16) (row swap), (l, 15 - l) within 16 (row mirror), (l, 7 - l) within 8
// (half mirror), then a butterfly within the quad (a + b and b + a are the same double: the 4
// copies agree).  Every pair stays inside its 32-lane half.
__device__ __forceinline__ double xf_reduce8(double (&v)[XF_G], int l32) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // lanes 0-15 keep units 0-3, lanes 16-31 units 4-7
    xf_swap16(v[i], v[i + 4]);
    v[i] = v[i] + v[i + 4];
  }
  const bool b3 = (l32 & 8) != 0, b2 = (l32 & 4) != 0;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const double send = b3 ? v[i] : v[i + 2];
    const double keep = b3 ? v[i + 2] : v[i];
    v[i] = keep + xf_dpp<XF_DPP_ROW_MIRROR>(send);
  }
  {
    const double send = b2 ? v[0] : v[1];
    const double keep = b2 ? v[1] : v[0];
    v[0] = keep + xf_dpp<XF_DPP_ROW_HALF_MIRROR>(send);
  }
  double s = v[0];
  s = s + xf_dpp<XF_DPP_QUAD_XOR1>(s);
  return s + xf_dpp<XF_DPP_QUAD_XOR2>(s);
}

// 8 units' sums (registers e[8]): per lane its 4 entries of each unit, count * x by fmas in entry
// order, software-pipelined by XF_PAIR units (the next stage's LDS reads of x issued before this
// stage's arithmetic); then xf_reduce8.
__device__ __forceinline__ double xf_group(const u32x4 (&e)[XF_G], const double* xs, int l32) {
  double v[XF_G];
  double xa[XF_PAIR][4], xb[XF_PAIR][4];
#pragma unroll
  for (int p = 0; p < XF_PAIR; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) xa[p][q] = xs[xf_col(e[p][q], q)];
#pragma unroll
  for (int s = 0; s < XF_G / XF_PAIR; ++s) {
    double(&cur)[XF_PAIR][4] = (s & 1) ? xb : xa;
    double(&nxt)[XF_PAIR][4] = (s & 1) ? xa : xb;
    if (s + 1 < XF_G / XF_PAIR) {
#pragma unroll
      for (int p = 0; p < XF_PAIR; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) nxt[p][q] = xs[xf_col(e[(s + 1) * XF_PAIR + p][q], q)];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int p = 0; p < XF_PAIR; ++p) {
      const u32x4& u = e[s * XF_PAIR + p];
      double a = (double)(u[0] >> 16) * cur[p][0];
      a = __builtin_fma((double)(u[1] >> 16), cur[p][1], a);
      a = __builtin_fma((double)(u[2] >> 16), cur[p][2], a);
      v[s * XF_PAIR + p] = __builtin_fma((double)(u[3] >> 16), cur[p][3], a);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
#if SA_XF_PROBE & 4
  double z = 0.0;
#pragma unroll
  for (int k = 0; k < XF_G; ++k) z += v[k];
  return z;
#else
  return xf_reduce8(v, l32);
#endif
}

__global__ __launch_bounds__(XF_THREADS) void xt_solve_reordered_kernel(
    const uint32_t* __restrict__ ell, const int32_t* __restrict__ row_len, const unsigned long long* __restrict__ move,
    const double* __restrict__ gs, const double* __restrict__ pmove, int C, int hp, double eps, int max_iter,
    int pmax, int kov, double* xb, double* __restrict__ heat, double* __restrict__ xt_out, int32_t* ctrl,
    int force_abort) {
  // LDS: ov [XF_HALVES][kov] units | xs [C] x_t | part [pmax] unit sums | luo [pmax + 1]
  extern __shared__ __attribute__((aligned(16))) u32x4 xf_lds[];
  u32x4* ov = xf_lds;
  double* xs = reinterpret_cast<double*>(xf_lds + (size_t)XF_HALVES * kov * 32);
  double* part = xs + ((C + 1) & ~1);
  int32_t* luo = reinterpret_cast<int32_t*>(part + pmax);
  uint32_t* scan = reinterpret_cast<uint32_t*>(xs);  // prologue: units of every row, scanned
  __shared__ uint32_t ws[XF_THREADS / 64 + 1];
  __shared__ int s_ra, s_rb;
#if SA_XF_PROBE
  const long long k_entry = wall_clock64();
#endif
  const int t = threadIdx.x, G = gridDim.x, g = blockIdx.x;
  const int l32 = t & 31, hw = t >> 5;
  const int pe = xe_pitch(C);

  // ---- rows of this workgroup: weight of row r = its units + 1, cut at multiples of total / G
  for (int r = t; r < C; r += XF_THREADS) scan[r] = (uint32_t)((row_len[r] + XE_KC - 1) / XE_KC);
  __syncthreads();
  const uint32_t U = block_scan<XF_THREADS>(scan, C, ws);
  if (t == 0) scan[C] = U;
  __syncthreads();
  const uint64_t K = (uint64_t)U + (uint64_t)C;
  auto owner = [&](int r) -> uint64_t {  // non-decreasing in r; owner(C) = G
    return r >= C ? (uint64_t)G : ((uint64_t)scan[r] + (uint64_t)r) * (uint64_t)G / K;
  };
  if (t < 2) {  // first row with owner >= g + t
    int lo = -1, hi = C;  // owner(lo) < g + t <= owner(hi)
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (owner(mid) >= (uint64_t)(g + t))
        hi = mid;
      else
        lo = mid;
    }
    if (t == 0)
      s_ra = hi;
    else
      s_rb = hi;
  }
  __syncthreads();
  const int ra = s_ra, nrl = s_rb - s_ra;
  const int ua = (int)scan[ra], nu = (int)scan[ra + nrl] - ua;
  // the host's bounds on units and rows per workgroup (never exceeded): the others leave at
  // their first barrier
  if (nu > pmax || nrl > pmax) {
    if (t == 0) xf_st32(ctrl + XF_ABORT, 2u);
    return;
  }
  for (int i = t; i <= nrl; i += XF_THREADS) luo[i] = (int32_t)scan[ra + i];
  __syncthreads();  // the scan's words are x's from here on
  const int hb = (int)((int64_t)nu * hw / XF_HALVES), he = (int)((int64_t)nu * (hw + 1) / XF_HALVES);
  const int hn = he - hb;  // this half-wave's units: local [hb, he)

  // ---- the half-wave's units: the first XF_KREG in registers for the whole solve, the next kov
  // in LDS, any further ones re-read from the compact rows every iteration
  u32x4 E[XF_KREG];
  bool esc = false;
#pragma unroll
  for (int k = 0; k < XF_KREG; ++k) {
    E[k] = k < hn ? xf_unit(ell, row_len, luo, nrl, ra, pe, ua + hb + k, l32) : u32x4{0u, 0u, 0u, 0u};
    esc |= xf_has_esc(E[k]);
  }
  u32x4* my_ov = ov + (size_t)hw * kov * 32 + l32;
  for (int k = XF_KREG; k < XF_KREG + kov; ++k) {
    const u32x4 e = k < hn ? xf_unit(ell, row_len, luo, nrl, ra, pe, ua + hb + k, l32) : u32x4{0u, 0u, 0u, 0u};
    esc |= xf_has_esc(e);
    my_ov[(k - XF_KREG) * 32] = e;
  }
  for (int k = XF_KREG + kov; k < hn; ++k) esc |= xf_has_esc(xf_unit(ell, row_len, luo, nrl, ra, pe, ua + hb + k, l32));
  if (__syncthreads_or(esc)) {  // a count >= 65535 (its value is in the dense row only): the host
    if (t == 0)                 // re-solves in order; the others leave at their first barrier
      xf_st32(ctrl + XF_ABORT, 4u);
    return;
  }

#if SA_XF_PROBE
  long long pt[5] = {0, 0, 0, 0, 0}, pc = k_entry;  // prologue, stage, units, rows, barrier
  auto tick = [&](int ph) {
    const long long n = wall_clock64();
    pt[ph] += n - pc;
    pc = n;
  };
  tick(0);
#else
  auto tick = [](int) {};
#endif
  constexpr double u = 0x1p-53;
  const double delta = (2.0 * (double)C + 16.0) * u;
  double ebound = 0.0;  // relative distance of x_t from the reference's x_t (bound)
  int n_iter = -1;
  const int grp = g & 7, ngrp = G < 8 ? G : 8, nq = (G - grp + 7) >> 3;  // barrier groups
  const int n16 = (C + 1) >> 1;                                         // 16-B words of x
  for (int it = 0; it < max_iter; ++it) {
    // the entries as the loop's own values: derived words (LDS addresses, counts as doubles)
    // hoisted out of the loop would take three times their registers
#pragma unroll
    for (int k = 0; k < XF_KREG; ++k) asm volatile("" : "+v"(E[k]));
    // ---- stage x_t: every 16-B word of the row loaded (sc1) before any LDS store
    if (it == 0) {
      for (int c = t; c < C; c += XF_THREADS) xs[c] = 0.0;
    } else {
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(xb + (int64_t)it * hp, 0, hp * 8, 0x00020000);
      u32x4 xr[XF_X16];  // past the row: the descriptor's range check returns 0, no memory access
#pragma unroll
      for (int q = 0; q < XF_X16; ++q) xr[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, (t + q * XF_THREADS) * 16, 0, 16);
#pragma unroll
      for (int q = 0; q < XF_X16; ++q) {
        const int w = t + q * XF_THREADS;
        if (w < n16) reinterpret_cast<u32x4*>(xs)[w] = xr[q];
      }
    }
    __syncthreads();
    tick(1);
    // ---- unit sums of the half-wave: registers, LDS, then re-read ones
#pragma unroll
    for (int k0 = 0; k0 < XF_KREG; k0 += XF_G) {
      if (k0 < hn) {  // half-wave uniform
        u32x4 e8[XF_G];
#pragma unroll
        for (int k = 0; k < XF_G; ++k) e8[k] = E[k0 + k];
        const double s = xf_group(e8, xs, l32);
        const int k = k0 + ((l32 >> 2) & 7);
        if ((l32 & 3) == 0 && k < hn) part[hb + k] = s;
      }
    }
    for (int k0 = XF_KREG; k0 < hn; k0 += XF_G) {
      u32x4 e8[XF_G];
#pragma unroll
      for (int k = 0; k < XF_G; ++k) {
        const int kk = k0 + k;
        e8[k] = kk >= hn ? u32x4{0u, 0u, 0u, 0u}
                         : (kk < XF_KREG + kov ? my_ov[(kk - XF_KREG) * 32]
                                                : xf_unit(ell, row_len, luo, nrl, ra, pe, ua + hb + kk, l32));
      }
      const double s = xf_group(e8, xs, l32);
      const int k = k0 + ((l32 >> 2) & 7);
      if ((l32 & 3) == 0 && k < hn) part[hb + k] = s;
    }
    __syncthreads();
    tick(2);
    // ---- rows, 8 lanes each: lane j sums units j, j + 8, ... in order, a fixed 8-lane tree; / move,
    // the reference's gs + pmove * (.) and its decision
    const double enext = (ebound + delta) * (1.0 + 0x1p-20);
    bool up = false, amb = false;
    xf_gu64* dst = (xf_gu64*)(xb + (int64_t)(it + 1) * hp);
    const int sub = t & (XF_ROWL - 1);
    for (int i0 = 0; i0 < nrl; i0 += XF_THREADS / XF_ROWL) {  // workgroup-uniform bound
      const int i = i0 + t / XF_ROWL;
      const bool live = i < nrl;
      const int r = ra + (live ? i : 0);
      double m = 1.0, gr = 0.0, pr = 0.0, xo = 0.0;
      int u0 = 0, u1 = 0;
      if (live) {
        if (sub == 0) {
          m = (double)move[r];
          gr = gs[r];
          pr = pmove[r];
          xo = xs[r];
        }
        u0 = luo[i] - ua;
        u1 = luo[i + 1] - ua;
      }
      double s = 0.0;
      for (int q = u0 + sub; q < u1; q += XF_ROWL) s = s + part[q];
      // a fixed 8-lane tree, lane 0's result used: pairs (l, 7 - l), then the quad's butterfly
      s = s + xf_dpp<XF_DPP_ROW_HALF_MIRROR>(s);
      s = s + xf_dpp<XF_DPP_QUAD_XOR1>(s);
      s = s + xf_dpp<XF_DPP_QUAD_XOR2>(s);
      if (live && sub == 0) {
        const double v = u1 > u0 ? s / m : 0.0;  // a row without entries sums +0 terms: 0
        const double xn = gr + pr * v;
        const double d = xn - xo;
        up |= d > eps;  // np.any(diff > eps)
        const double margin = enext * (xn + xo) * (1.0 + 0x1p-20) + 8.0 * u * (fabs(d) + fabs(eps));
        amb |= fabs(d - eps) <= margin;
        __hip_atomic_store(dst + r, (unsigned long long)__double_as_longlong(xn), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        heat[(int64_t)(it + 1) * C + r] = xn;
        if (xt_out) xt_out[r] = xn;  // the surface: the last iterate when the loop ends
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
    const int any_up = __syncthreads_or(up), any_amb = __syncthreads_or(amb);
    tick(3);
#if SA_DEBUG
    // sa_debug_xt_solve_abort: the last workgroup leaves without arriving (workgroup-uniform),
    // as if it never got a CU; the others' bounded polls time out and take the abort exit
    if (it == force_abort && g == G - 1) return;
#else
    (void)force_abort;
#endif
    if (t == 0) {  // ---- grid barrier, XCD-hierarchical; one lane per workgroup
      if (any_up) __hip_atomic_fetch_or((xf_gu32*)(ctrl + XF_FLAGS + it), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (any_amb) __hip_atomic_fetch_or((xf_gu32*)(ctrl + XF_AMB), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint32_t epoch = (uint32_t)it + 1;
      const uint32_t old = xf_add32(ctrl + XF_GRP + 32 * grp, 1u);
      bool go = true;
      if (old == epoch * (uint32_t)nq - 1) {  // the group's last arriver
        const uint32_t ot = xf_add32(ctrl + XF_TOP, 1u);
        if (ot == epoch * (uint32_t)ngrp - 1) {  // the last group: release every group
          for (int q = 0; q < ngrp; ++q) xf_st32(ctrl + XF_GEN + 32 * q, epoch);
          go = false;
        }
      }
      if (go) xf_wait(ctrl, ctrl + XF_GEN + 32 * grp, epoch, it == 0 ? XF_SPIN_TICKS_FIRST : XF_SPIN_TICKS);
    }
    __syncthreads();
    tick(4);
    const uint32_t flag = xf_ld32(ctrl + XF_FLAGS + it);
    const uint32_t stop = xf_ld32(ctrl + XF_ABORT) | xf_ld32(ctrl + XF_AMB);
    if (stop) break;  // every workgroup reads the same words behind the same barrier
    ebound = enext;
    if (!flag) {
      n_iter = it + 1;
      break;
    }
  }
#if SA_XF_PROBE
  if (t == 0) {  // the slowest workgroup's unit phase and the most units of one workgroup
    atomicMax(ctrl + XF_FLAGS + max_iter + 1, (int32_t)pt[2]);
    atomicMax(ctrl + XF_FLAGS + max_iter + 2, nu);
    atomicMax(ctrl + XF_FLAGS + max_iter + 3, (int32_t)pt[1]);
  }
#endif
  if (g == 0 && t == 0) {
    ctrl[XF_NITER] = n_iter;
#if SA_XF_PROBE
    for (int q = 0; q < 4; ++q) ctrl[4 + q] = (int32_t)pt[q + 1];
    ctrl[XF_FLAGS + max_iter] = (int32_t)pt[0];
#endif
  }
}

}  // namespace sa

// ================================== C ABI =================================================
using namespace sa;

namespace sa {
// The band shape of a grid, false when the band path cannot hold it (then the caller counts with
// the global-atomic pass).  R = C / 256 (>= 256 bands to fill the chip), at most what 160 KB of
// LDS holds and at most 8.
static bool xt_band_shape(int C, XbShape* s);
bool xt_band_ok(int C) {
  XbShape s;
  return xt_band_shape(C, &s);
}

static bool xt_band_shape(int C, XbShape* s) {
  if (C < 1 || C + 3 > 65536) return false;
  const int P = (C + 3 + 3) & ~3;
  int rmax = (int)((XB_LDS_MAX - XB_LDS_STATIC) / ((size_t)P * 4));
  if (rmax > SA_XB_RMAX) rmax = SA_XB_RMAX;
  if (rmax < 1) return false;
  int r = C / 256;
  if (r < 1) r = 1;
  if (r > rmax) r = rmax;
  const int nb = (C + r - 1) / r;
  if (nb > XB_NB_MAX) return false;
  s->C = C;
  s->R = r;
  s->NB = nb;
  s->P = P;
  s->magic = ((1ull << 32) + (uint64_t)r - 1) / (uint64_t)r;
  return true;
}

// K1 -> K2 -> K3 of one batch: its keys sorted into buckets[] by band, band_off[NB + 1].
static int bucket_batch(const sa_actions& A, const uint32_t* cells, int64_t n, int l, int w, const XbShape& S,
                        xb_key_t* buckets, int64_t* band_off, int32_t* err, const XkRate& RO, hipStream_t st) {
  // K1 runs one workgroup per CU: a batch's regions in whole rounds of the CUs (16M actions:
  // 489 regions of 32768 -> 512 of 31,488; a 4M tail: 123 -> 256), regions of >= 4096 actions
  int64_t regions = (n + XK_CHUNK - 1) / XK_CHUNK, chunk = XK_CHUNK;
  if (SA_XK_BALANCE && n > 0) {
    const int64_t G = device_cus(current_device());
    const int64_t r = (regions + G - 1) / G * G;
    chunk = ((n + r - 1) / r + 255) & ~(int64_t)255;
    if (chunk < 4096) chunk = 4096;
    if (chunk > XK_CHUNK) chunk = XK_CHUNK;
    regions = (n + chunk - 1) / chunk;
  }
  // scratch: band_cnt [NB] | cursor [NB] | region_cnt [regions] | keys [regions * XK_CHUNK], each
  // part on 256-B boundaries: the band counts and cursors are zeroed by ONE aligned fill (an
  // unaligned start split it into three fill kernels, ~9 us more per batch)
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t nbb = al((size_t)S.NB * 4), rcb = al((size_t)regions * 4);
  const size_t bytes = 2 * nbb + rcb + (size_t)regions * XK_CHUNK * 4;
  Scratch sc;
  int rc = scratch_acquire(bytes, st, &sc);
  if (rc) return rc;
  char* base = static_cast<char*>(sc.ptr);
  uint32_t* band_cnt = reinterpret_cast<uint32_t*>(base);
  uint32_t* cursor = reinterpret_cast<uint32_t*>(base + nbb);
  uint32_t* region_cnt = reinterpret_cast<uint32_t*>(base + 2 * nbb);
  uint32_t* keys = reinterpret_cast<uint32_t*>(base + 2 * nbb + rcb);
  rc = check_hip(hipMemsetAsync(band_cnt, 0, 2 * nbb, st), "memset band counts and cursors");
  if (!rc) {
    sa_actions none;
    memset(&none, 0, sizeof(none));
    const sa_frame& F = A.frames[0];
    const int vec = !cells && n >= 2 && aligned16(F.c0) && aligned16(F.c1) && aligned16(F.c2) && aligned16(F.c3) &&
                    ((uintptr_t)F.type_id & 1u) == 0 && ((uintptr_t)F.result_id & 1u) == 0;
    if (cells)
      hipLaunchKernelGGL((xt_keys_kernel<true>), dim3((unsigned)regions), dim3(XK_THREADS), (size_t)S.NB * 4, st, none,
                         cells, n, l, w, S, keys, region_cnt, band_cnt, err, XkRate{nullptr, nullptr, 0, 0}, 0, chunk);
    else
      hipLaunchKernelGGL((xt_keys_kernel<false>), dim3((unsigned)regions), dim3(XK_THREADS), (size_t)S.NB * 4, st, A,
                         nullptr, n, l, w, S, keys, region_cnt, band_cnt, err, RO, vec, chunk);
    rc = check_launch("xt_keys_kernel");
  }
  if (!rc) {
    const size_t lds = ((size_t)2 * S.NB + XS_PART) * 4;
    hipLaunchKernelGGL(xt_keys_scatter_kernel, dim3((unsigned)(regions * XS_SPLIT)), dim3(XS_THREADS), lds, st, keys,
                       region_cnt, S, band_cnt, band_off, cursor, buckets);
    rc = check_launch("xt_keys_scatter_kernel");
  }
  scratch_release(sc, st);
  return rc;
}

static int count_from_buckets(int nsets, const xb_key_t* const* buckets, const int64_t* const* band_off,
                              const XbShape& S, int band0, int nbands, int64_t* shot, int64_t* goal, int64_t* move,
                              int32_t* trans, int overwrite, hipStream_t st, uint32_t* ell = nullptr,
                              int32_t* row_len = nullptr, int dense = 1) {
  if (nbands <= 0) return SA_OK;
  // the compact rows come from the bins only when one launch writes the final counts
  if (ell && (!overwrite || nsets > XB_MAX_SETS)) return fail(SA_EINVAL, "compact rows need one overwriting launch");
  if (!dense && !ell) return fail(SA_EINVAL, "the dense rows may be skipped only beside the compact rows");
  const int vec = (S.C % 4 == 0) && aligned16(trans);
  const size_t lds = (size_t)S.R * S.P * 4;
  for (int s0 = 0; s0 < nsets || (s0 == 0 && nsets == 0); s0 += XB_MAX_SETS) {
    XbSets sets;
    memset(&sets, 0, sizeof(sets));
    sets.n = nsets - s0 < XB_MAX_SETS ? nsets - s0 : XB_MAX_SETS;
    for (int k = 0; k < sets.n; ++k) {
      sets.keys[k] = buckets[s0 + k];
      sets.off[k] = band_off[s0 + k];
    }
    // later launches add to what the first one wrote
    hipLaunchKernelGGL(xt_band_count_kernel, dim3((unsigned)nbands), dim3(XB_THREADS), lds, st, sets, S, band0,
                       reinterpret_cast<unsigned long long*>(shot), reinterpret_cast<unsigned long long*>(goal),
                       reinterpret_cast<unsigned long long*>(move), trans, (overwrite && s0 == 0) ? 1 : 0, vec,
                       ell, row_len, xe_pitch(S.C), dense);
    int rc = check_launch("xt_band_count_kernel");
    if (rc) return rc;
    if (nsets == 0) break;
  }
  return SA_OK;
}

// The whole band-owned count of one batch (sa_xt_count / sa_xt_count_codes / sa_xt_count_cells
// for grids the band path holds): buckets in scratch, added into the caller's counts.
int xt_count_bands(const sa_actions& A, const uint32_t* cells, int64_t n, int l, int w, int64_t* shot,
                   int64_t* goal, int64_t* move, int32_t* trans, int32_t* err, uint32_t* codes, hipStream_t st) {
  XbShape S;
  if (!xt_band_shape(l * w, &S)) return fail(SA_EINVAL, "grid outside the band-owned count");
  Scratch sc;  // buckets [n] | band_off [NB + 1]
  const size_t bb = ((size_t)n * sizeof(xb_key_t) + 255) & ~(size_t)255;
  int rc = scratch_acquire(bb + ((size_t)S.NB + 1) * 8, st, &sc);
  if (rc) return rc;
  xb_key_t* buckets = static_cast<xb_key_t*>(sc.ptr);
  int64_t* band_off = reinterpret_cast<int64_t*>(static_cast<char*>(sc.ptr) + bb);
  rc = bucket_batch(A, cells, n, l, w, S, buckets, band_off, err, XkRate{codes, nullptr, 0, 0}, st);
  if (!rc) {
    const xb_key_t* bk[1] = {buckets};
    const int64_t* bo[1] = {band_off};
    rc = count_from_buckets(1, bk, bo, S, 0, S.NB, shot, goal, move, trans, 0, st);
  }
  scratch_release(sc, st);
  return rc;
}

// Compact form + iteration used by sa_xt_solve for C > SA_XT_SOLVE_MAX_C.
bool xt_compact_ok(int C) { return C >= 1 && C <= XE_XMAX; }
size_t xt_compact_bytes(int C, int nrows) { return (size_t)(nrows > 0 ? nrows : 0) * (size_t)xe_pitch(C) * 4; }
int xt_compact_build(const int32_t* cnt_rows, int C, int nrows, uint32_t* ell, int32_t* row_len, hipStream_t st) {
  if (nrows <= 0) return SA_OK;
  hipLaunchKernelGGL(xt_ell_build_kernel, dim3((unsigned)((nrows + XE_BUILD_ROWS - 1) / XE_BUILD_ROWS)),
                     dim3(XE_BUILD_ROWS * 64), 0, st, cnt_rows, C, nrows, ell, row_len);
  return check_launch("xt_ell_build_kernel");
}
int xt_compact_iterate(const uint32_t* ell, const int32_t* row_len, const int32_t* cnt_rows, const int64_t* move,
                       const double* gs, const double* pmove, int C, int rb, int nrows, const double* x, double eps,
                       double* xo, const int32_t* flag_prev, int32_t* flag_out, hipStream_t st) {
  const int ns = (nrows + XE_S - 1) / XE_S;
  if (ns == 0) return SA_OK;
  int ct = SA_XE_QDIV ? 0 : XE_CT_MAX;  // the quotient table: as many counts as fit next to x
  while (ct > 16 && (size_t)C * 8 + (size_t)XE_S * ct * 8 + XE_LDS_STATIC > XE_LDS_MAX) ct >>= 1;
  hipLaunchKernelGGL(xt_iter_ell_kernel, dim3((unsigned)ns), dim3(XE_THREADS), ((size_t)C + (size_t)XE_S * ct) * 8, st,
                     ell, row_len, cnt_rows, reinterpret_cast<const unsigned long long*>(move), gs, pmove, C, rb,
                     nrows, ct, eps, x, xo, flag_prev, flag_out);
  return check_launch("xt_iter_ell_kernel");
}

// The reordered solve of the compact rows (xt_solve_reordered_kernel): *status 0 = solved
// (*n_iter the reference's count, -1: max_iter reached), 1 = a decision fell inside the error
// bound, 2 = not launched (grid, LDS, residency or scratch size), 3 = a barrier timed out.
// heat: [(max_iter + 1) * C] f64, rows 1.. written.  Synchronises the stream.
// A small pinned host buffer for the solve's control words (a pageable destination made the
// copy a staged, synchronous one: ~70 us of the call at cfg5).
static int32_t* pinned_ctrl() {
  static thread_local int32_t* p = nullptr;
  if (!p && hipHostMalloc(reinterpret_cast<void**>(&p), 64, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    p = nullptr;
  }
  return p;
}

// sa_debug_xt_solve_abort (debug builds): the iteration at which the reordered solve's last
// workgroup skips the grid barrier, -1 none
static int g_xf_force_abort = -1;

static int xt_solve_reordered(const uint32_t* ell, const int32_t* row_len, const int32_t* cnt_rows,
                              const int64_t* move, const double* gs, const double* pmove, int C, double eps,
                              int max_iter, double* heat, double* xt_out, int* n_iter, int* status, hipStream_t st,
                              SolveHook* hook) {
  *status = 2;
  *n_iter = -1;
  if (!xt_compact_ok(C) || max_iter < 1) return SA_OK;
  const int dev = current_device();
  const int G = device_cus(dev);
  const int upr = (C + XE_KC - 1) / XE_KC;                 // units of a dense row
  const int64_t kmax = (int64_t)C * upr + C;               // row weights (units + 1), at most
  const int pmax = (int)((kmax + G - 1) / G) + upr + 2;    // units (or rows) of one workgroup, at most
  const size_t fixed = (size_t)((C + 1) & ~1) * 8 + (size_t)pmax * 8 + ((size_t)pmax + 1) * 4;
  const size_t lmax = (size_t)device_lds_max(dev) - 1024;  // the kernel's static LDS
  if (fixed + (size_t)C * 4 > lmax || (size_t)(C + 1) * 4 > (size_t)((C + 1) & ~1) * 8) return SA_OK;
  int kov = (int)((lmax - fixed) / ((size_t)XF_HALVES * XF_UNIT_BYTES));
  if (kov > XF_KOV_MAX) kov = XF_KOV_MAX;
  const size_t lds = fixed + (size_t)XF_HALVES * kov * XF_UNIT_BYTES;
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void*>(xt_solve_reordered_kernel),
                                                   XF_THREADS, lds) != hipSuccess) {
    (void)hipGetLastError();
    return SA_OK;
  }
  if (nb < 1) return SA_OK;  // one resident workgroup per CU is what the grid barrier needs
  const int hp = (C + 15) & ~15;  // x history rows on whole 128-B lines
  const size_t xbytes = (size_t)(max_iter + 1) * (size_t)hp * 8;
  if (xbytes > ((size_t)512 << 20)) return SA_OK;
  const size_t cbytes = ((size_t)(XF_FLAGS + max_iter + 4) * 4 + 255) & ~(size_t)255;
  Scratch sc;
  int rc = scratch_acquire(cbytes + xbytes, st, &sc);
  if (rc) return rc;
  int32_t* ctrl = static_cast<int32_t*>(sc.ptr);
  double* xb = reinterpret_cast<double*>(static_cast<char*>(sc.ptr) + cbytes);
  int32_t hl[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int32_t* pin = pinned_ctrl();
  int32_t* h = pin ? pin : hl;
  rc = check_hip(hipMemsetAsync(ctrl, 0, cbytes, st), "memset solve control");
  if (!rc) {
    hipLaunchKernelGGL(xt_solve_reordered_kernel, dim3((unsigned)G), dim3(XF_THREADS), lds, st, ell, row_len,
                       reinterpret_cast<const unsigned long long*>(move), gs, pmove, C, hp, eps, max_iter, pmax, kov,
                       xb, heat, xt_out, ctrl, SA_DEBUG ? g_xf_force_abort : -1);
    rc = check_launch("xt_solve_reordered_kernel");
  }
  if (!rc) rc = check_hip(hipMemcpyAsync(h, ctrl, 8 * sizeof(int32_t), hipMemcpyDeviceToHost, st), "copy solve control");
  if (!rc && hook) {  // queued behind the solve: no host round trip between the two
    rc = hook->fn(hook->ctx);
    hook->ran = true;
  }
  if (!rc) rc = check_hip(hipStreamSynchronize(st), "hipStreamSynchronize");
#if SA_XF_PROBE
  int32_t pro[4] = {0, 0, 0, 0};
  if (!rc) rc = check_hip(hipMemcpy(pro, ctrl + XF_FLAGS + max_iter, 16, hipMemcpyDeviceToHost), "copy probe");
  fprintf(stderr,
          "xf_probe C=%d G=%d kreg=%d iters=%d ticks(10ns) wg0: prologue %d stage %d units %d rows %d barrier %d; "
          "max over wgs: units %d stage %d, units per wg %d (register capacity %d)\n",
          C, G, XF_KREG, h[XF_NITER], pro[0], h[4], h[5], h[6], h[7], pro[1], pro[3], pro[2], XF_HALVES * XF_KREG);
#endif
  scratch_release(sc, st);
  if (rc) return rc;
  if (h[XF_ABORT])  // 1: a barrier timed out; 2 / 4: a bound or an escaped count (not launchable)
    *status = h[XF_ABORT] == 1 ? 3 : 2;
  else if (h[XF_AMB])
    *status = 1;
  else {
    *status = 0;
    *n_iter = h[XF_NITER];
  }
  return SA_OK;
}

// The value iteration over the compact rows of the whole grid (heat row 0 already zero): the
// reordered solve unless `flags` asks for the reference's order, the sequential-order kernel
// (one launch per iteration, flags read back every 8) when asked or when the reordered solve
// cannot decide.  *path: SA_XT_PATH_*.  Synchronises the stream.
int xt_compact_solve(const uint32_t* ell, const int32_t* row_len, const int32_t* cnt_rows, const int64_t* move,
                     const double* gs, const double* pmove, int C, double eps, int max_iter, int flags,
                     double* heat, int* n_iter, int* path, hipStream_t st, double* xt_out, SolveHook* hook) {
  *n_iter = -1;
  *path = SA_XT_PATH_SEQUENTIAL;
  if (!(flags & SA_XT_SOLVE_EXACT)) {
    int status = 2, it = -1;
    int rc = xt_solve_reordered(ell, row_len, cnt_rows, move, gs, pmove, C, eps, max_iter, heat, xt_out, &it,
                                &status, st, xt_out ? hook : nullptr);
    if (rc) return rc;
    if (status == 0) {
      *n_iter = it;
      *path = SA_XT_PATH_REORDERED;
      return SA_OK;
    }
    *path = status == 1 ? SA_XT_PATH_INSIDE_BOUND : status == 3 ? SA_XT_PATH_TIMEOUT : SA_XT_PATH_UNAVAILABLE;
  }
  Scratch sc;  // convergence flags [max_iter + 1]
  int rc = scratch_acquire(sizeof(int32_t) * ((size_t)max_iter + 1), st, &sc);
  if (rc) return rc;
  int32_t* dflags = static_cast<int32_t*>(sc.ptr);
  rc = check_hip(hipMemsetAsync(dflags, 0, sizeof(int32_t) * ((size_t)max_iter + 1), st), "memset");
  std::vector<int32_t> hflags(max_iter + 1, 0);
  const int batch = 8;
  int iters = -1;
  for (int it0 = 0; !rc && it0 < max_iter && iters < 0; it0 += batch) {
    const int it1 = it0 + batch < max_iter ? it0 + batch : max_iter;
    for (int it = it0; it < it1 && !rc; ++it) {
      double* xi = heat + (int64_t)it * C;
      rc = xt_compact_iterate(ell, row_len, cnt_rows, move, gs, pmove, C, 0, C, xi, eps, xi + C,
                              it > 0 ? dflags + it - 1 : nullptr, dflags + it, st);
    }
    if (!rc)
      rc = check_hip(hipMemcpyAsync(hflags.data() + it0, dflags + it0, sizeof(int32_t) * (it1 - it0),
                                    hipMemcpyDeviceToHost, st),
                     "copy flags");
    if (!rc) rc = check_hip(hipStreamSynchronize(st), "hipStreamSynchronize");
    for (int it = it0; !rc && it < it1; ++it)
      if (hflags[it] == 0) {
        iters = it + 1;
        break;
      }
  }
  scratch_release(sc, st);
  *n_iter = iters;
  return rc;
}
}  // namespace sa

extern "C" int sa_debug_xt_solve_abort(int32_t iteration) {
#if SA_DEBUG
  if (iteration < -1) return fail(SA_EINVAL, "iteration must be >= -1");
  g_xf_force_abort = iteration;
  return SA_OK;
#else
  (void)iteration;
  return fail(SA_EINVAL, "sa_debug_xt_solve_abort: debug builds only (libsocceraction_amd_debug.so)");
#endif
}

extern "C" int sa_xt_band_shape(int32_t l, int32_t w, int32_t* rows_per_band, int32_t* n_bands) {
  if (l < 1 || w < 1 || (int64_t)l * w > 46340) return fail(SA_EINVAL, "bad l or w");
  XbShape S;
  if (!xt_band_shape(l * w, &S)) return fail(SA_EINVAL, "the band-owned count does not hold %d cells", l * w);
  if (rows_per_band) *rows_per_band = S.R;
  if (n_bands) *n_bands = S.NB;
  return SA_OK;
}

extern "C" int sa_xt_count_bucket(const sa_actions* a, const uint32_t* cells, int64_t n, int32_t l, int32_t w,
                                  uint16_t* buckets, int64_t* band_off, int32_t* err_flags, uint32_t* codes,
                                  uint64_t* interp_codes, int32_t L, int32_t W, void* stream) {
  if (l < 1 || w < 1 || (int64_t)l * w > 46340) return fail(SA_EINVAL, "bad l or w");
  XbShape S;
  if (!xt_band_shape(l * w, &S)) return fail(SA_EINVAL, "the band-owned count does not hold %d cells", l * w);
  if (!band_off || !err_flags) return fail(SA_EINVAL, "null output");
  if (cells) {
    if (n < 0 || (int64_t)l * w > SA_XT_CELLS_MAX_C) return fail(SA_EINVAL, "cell codes need l * w <= %d", SA_XT_CELLS_MAX_C);
    if (codes || interp_codes) return fail(SA_EINVAL, "rate codes come from the coordinate pass");
  } else {
    if (!a || a->n < 0 || a->atomic) return fail(SA_EINVAL, "bad sa_actions (SPADL actions required)");
    n = a->n;
    const sa_frame& F = a->frames[0];
    if (n > 0 && (!F.type_id || !F.result_id || !F.c0 || !F.c1 || !F.c2 || !F.c3))
      return fail(SA_EINVAL, "null input column");
    if (codes && !aligned16(codes)) return fail(SA_EINVAL, "codes must be 16-byte aligned");
    if (codes && (int64_t)l * w > 65535) return fail(SA_EINVAL, "rate codes need l * w <= 65535");
    if (interp_codes && (!aligned16(interp_codes) || L < 1 || W < 1 || (int64_t)L * W > INT32_MAX))
      return fail(SA_EINVAL, "interp_codes: 16-byte aligned, 1 <= L * W < 2^31");
  }
  if (n > INT32_MAX) return fail(SA_EINVAL, "at most 2^31 - 1 actions per batch");
  if (n > 0 && !buckets) return fail(SA_EINVAL, "null buckets");
  hipStream_t st = (hipStream_t)stream;
  if (n == 0)
    return check_hip(hipMemsetAsync(band_off, 0, sizeof(int64_t) * ((size_t)S.NB + 1), st), "memset band offsets");
  sa_actions none;
  memset(&none, 0, sizeof(none));
  return bucket_batch(cells ? none : *a, cells, n, l, w, S, buckets, band_off, err_flags,
                      XkRate{codes, interp_codes, L, W}, st);
}

extern "C" int sa_xt_count_from_buckets(int32_t nsets, const uint16_t* const* buckets, const int64_t* const* band_off,
                                        int32_t l, int32_t w, int64_t* shot, int64_t* goal, int64_t* move,
                                        int32_t* trans, int32_t flags, void* stream) {
  return sa_xt_count_from_buckets_ex(nsets, buckets, band_off, l, w, shot, goal, move, trans, flags, nullptr, nullptr,
                                     stream);
}

extern "C" int sa_xt_count_from_buckets_ex(int32_t nsets, const uint16_t* const* buckets,
                                           const int64_t* const* band_off, int32_t l, int32_t w, int64_t* shot,
                                           int64_t* goal, int64_t* move, int32_t* trans, int32_t flags,
                                           uint32_t* ell, int32_t* row_len, void* stream) {
  if (l < 1 || w < 1 || (int64_t)l * w > 46340) return fail(SA_EINVAL, "bad l or w");
  XbShape S;
  if (!xt_band_shape(l * w, &S)) return fail(SA_EINVAL, "the band-owned count does not hold %d cells", l * w);
  if (nsets < 0 || (nsets > 0 && (!buckets || !band_off))) return fail(SA_EINVAL, "bad bucket sets");
  for (int k = 0; k < nsets; ++k)
    if (!band_off[k]) return fail(SA_EINVAL, "null band offsets");
  if (!shot || !goal || !move || !trans) return fail(SA_EINVAL, "null count buffer");
  if (flags & ~(SA_XT_COUNT_OVERWRITE | SA_XT_COUNT_COMPACT_ONLY)) return fail(SA_EINVAL, "unknown flags");
  if (!ell != !row_len) return fail(SA_EINVAL, "ell and row_len come together");
  if ((flags & SA_XT_COUNT_COMPACT_ONLY) && !ell) return fail(SA_EINVAL, "SA_XT_COUNT_COMPACT_ONLY needs ell");
  if (ell) {
    if (!xt_compact_ok(l * w)) return fail(SA_EINVAL, "the compact form takes 1 <= C <= %d", XE_XMAX);
    if (!(flags & SA_XT_COUNT_OVERWRITE) || nsets > XB_MAX_SETS)
      return fail(SA_EINVAL, "compact rows need SA_XT_COUNT_OVERWRITE and at most %d bucket sets", XB_MAX_SETS);
    if (!aligned16(ell)) return fail(SA_EINVAL, "ell must be 16-byte aligned");
  }
  if (nsets == 0 && !(flags & SA_XT_COUNT_OVERWRITE)) return SA_OK;
  return count_from_buckets(nsets, buckets, band_off, S, 0, S.NB, shot, goal, move, trans,
                            (flags & SA_XT_COUNT_OVERWRITE) != 0, (hipStream_t)stream, ell, row_len,
                            (flags & SA_XT_COUNT_COMPACT_ONLY) ? 0 : 1);
}

extern "C" int sa_xt_count_band_rows(int32_t nsets, const uint16_t* const* buckets, const int64_t* const* band_off,
                                     int32_t l, int32_t w, int32_t band0, int32_t nbands, int64_t* shot_rows,
                                     int64_t* goal_rows, int64_t* move_rows, int32_t* trans_rows, int32_t flags,
                                     void* stream) {
  if (l < 1 || w < 1 || (int64_t)l * w > 46340) return fail(SA_EINVAL, "bad l or w");
  XbShape S;
  if (!xt_band_shape(l * w, &S)) return fail(SA_EINVAL, "the band-owned count does not hold %d cells", l * w);
  if (band0 < 0 || nbands < 0 || band0 + nbands > S.NB) return fail(SA_EINVAL, "band range outside [0, %d)", S.NB);
  if (nsets < 0 || (nsets > 0 && (!buckets || !band_off))) return fail(SA_EINVAL, "bad bucket sets");
  for (int k = 0; k < nsets; ++k)
    if (!band_off[k]) return fail(SA_EINVAL, "null band offsets");
  if (nbands > 0 && (!shot_rows || !goal_rows || !move_rows || !trans_rows))
    return fail(SA_EINVAL, "null count buffer");
  if (flags & ~SA_XT_COUNT_OVERWRITE) return fail(SA_EINVAL, "unknown flags");
  if (nsets == 0 && !(flags & SA_XT_COUNT_OVERWRITE)) return SA_OK;
  return count_from_buckets(nsets, buckets, band_off, S, band0, nbands, shot_rows, goal_rows, move_rows, trans_rows,
                            (flags & SA_XT_COUNT_OVERWRITE) != 0, (hipStream_t)stream);
}

extern "C" int sa_xt_compact_rows(const int32_t* cnt_rows, int32_t C, int32_t nrows, uint32_t* ell,
                                  int32_t* row_len, void* stream) {
  if (!xt_compact_ok(C) || nrows < 0) return fail(SA_EINVAL, "the compact form takes 1 <= C <= %d", XE_XMAX);
  if (nrows > 0 && (!cnt_rows || !ell || !row_len)) return fail(SA_EINVAL, "null pointer");
  if (nrows > 0 && !aligned16(ell)) return fail(SA_EINVAL, "ell must be 16-byte aligned");
  return xt_compact_build(cnt_rows, C, nrows, ell, row_len, (hipStream_t)stream);
}

extern "C" int sa_xt_iterate_compact(const uint32_t* ell, const int32_t* row_len, const int32_t* cnt_rows,
                                     const int64_t* move, const double* gs, const double* pmove, int32_t C, int32_t r0,
                                     int32_t nrows, const double* x, double eps, double* x_next_rows,
                                     const int32_t* flag_prev, int32_t* flag_out, void* stream) {
  if (!xt_compact_ok(C)) return fail(SA_EINVAL, "the compact form takes 1 <= C <= %d", XE_XMAX);
  if (r0 < 0 || nrows < 0 || r0 + nrows > C) return fail(SA_EINVAL, "row range outside [0, C)");
  if (!move || !gs || !pmove || !x || !flag_out ||
      (nrows > 0 && (!ell || !row_len || !cnt_rows || !x_next_rows)))
    return fail(SA_EINVAL, "null xt iteration pointer");
  if (nrows > 0 && !aligned16(ell)) return fail(SA_EINVAL, "ell must be 16-byte aligned");
  return xt_compact_iterate(ell, row_len, cnt_rows, move, gs, pmove, C, r0, nrows, x, eps, x_next_rows, flag_prev,
                            flag_out, (hipStream_t)stream);
}

extern "C" int sa_xt_solve_compact(const uint32_t* ell, const int32_t* row_len, const int32_t* cnt_rows,
                                   const int64_t* move, const double* gs, const double* pmove, int32_t C, double eps,
                                   int32_t max_iter, int32_t flags, double* heatmaps, int32_t* n_iter, int32_t* path,
                                   void* stream) {
  if (!xt_compact_ok(C)) return fail(SA_EINVAL, "the compact form takes 1 <= C <= %d", XE_XMAX);
  if (max_iter < 0) return fail(SA_EINVAL, "bad max_iter");
  if (!ell || !row_len || !cnt_rows || !move || !gs || !pmove || !heatmaps || !n_iter)
    return fail(SA_EINVAL, "null pointer");
  if (!aligned16(ell)) return fail(SA_EINVAL, "ell must be 16-byte aligned");
  if (flags & ~SA_XT_SOLVE_EXACT) return fail(SA_EINVAL, "unknown flags");
  hipStream_t st = (hipStream_t)stream;
  int rc = check_hip(hipMemsetAsync(heatmaps, 0, sizeof(double) * C, st), "memset");
  int it = -1, p = SA_XT_PATH_SEQUENTIAL;
  if (!rc) rc = xt_compact_solve(ell, row_len, cnt_rows, move, gs, pmove, C, eps, max_iter, flags, heatmaps, &it, &p, st);
  *n_iter = it;
  if (path) *path = p;
  return rc;
}

extern "C" int64_t sa_xt_compact_bytes(int32_t C, int32_t nrows) {
  if (!xt_compact_ok(C) || nrows < 0) return -1;
  return (int64_t)xt_compact_bytes(C, nrows);
}
