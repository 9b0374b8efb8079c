// Gradient-boosted tree inference on the VAEP feature blocks (gfx950): the `predict_proba`
// between `compute_features` and `formula.value` in VAEP.rate (reference vaep/base.py:284-333,
// SURVEY.md §8(f) row 3), evaluated where the features already are -- in HBM -- instead of
// copying ~940 B/action of features to a host learner.
//
// One thread per action; every tree is walked from its root in model order and the leaf
// values are summed onto the base margin in that order, then the logistic link is applied.
// The split rule and the arithmetic follow the producing library:
//   xgboost (binary:logistic, JSON model): float32 feature values, thresholds and sums;
//     `x < threshold` goes left; a missing (NaN) value follows default_left;
//     p = 1 / (1 + exp(-margin)) in float32.
//   scikit-learn HistGradientBoostingClassifier: float64; `x <= threshold` goes left; NaN
//     follows missing_go_to_left; p = expit(margin) in float64.
// The model's nodes are staged in LDS when they fit (a default 100-tree depth-3 model is 36 KB),
// sized to the model and shared by 16 waves per workgroup (occupancy), so the per-node loads of
// divergent lanes are LDS reads; feature values are read from the
// tiled blocks (row j of a column is contiguous across lanes: coalesced at the root, L2-resident
// afterwards).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <type_traits>

#include "sa_common.h"
#include "sa_internal.h"

namespace sa {

struct TNode {  // 24 B
  double thr_or_value;  // split threshold, or the leaf value
  int32_t feature;      // -1 = leaf
  int32_t left;         // child indices are absolute node indices; bit 31 of `right` = default_left
  int32_t right;
  int32_t pad;
};

constexpr int TR_THREADS = 1024;  // 16 waves share one LDS copy of the model
constexpr int TR_LDS_NODES = 2048;  // 48 KB
constexpr int TR_LDS_SLOTS = 2048;  // 8 KB
#ifndef SA_TREE_SCALED
#define SA_TREE_SCALED 1  // staged walk: condition byte offsets in the staged nodes (0: indices)
#endif
#ifndef SA_TREE_PERSIST
#define SA_TREE_PERSIST 0  // staged walk grid: N x the resident workgroups looping over tiles (A/B: 1.19 ms vs 1.12 per learner at N = 1, r06i; 0: one per tile)
#endif
#ifndef SA_TREE_TG
#define SA_TREE_TG 8
#endif
#ifndef SA_TREE_FIXED
#define SA_TREE_FIXED 1  // tree_depth given: fixed-depth walk over self-looping leaves
#endif
constexpr int TG = SA_TREE_TG;      // trees walked together per thread
static_assert(TG >= 1 && TG <= 32, "SA_TREE_TG: trees per thread");

// Row j's element of column `col` in each tiled block is base[kind] + col * R[kind]; the
// per-row bases are computed once (one division per block) instead of per feature read.
struct RowBases {
  const uint8_t* b;
  const double* f;
  const int64_t* i;
  int64_t Rb, Rf, Ri;
};

__device__ __forceinline__ RowBases row_bases(const sa_block& Bb, const sa_block& Bf, const sa_block& Bi,
                                              int64_t j) {
  RowBases r;
  const int64_t tb = j / Bb.tile_rows, tf = j / Bf.tile_rows, ti = j / Bi.tile_rows;
  r.Rb = Bb.tile_rows;
  r.Rf = Bf.tile_rows;
  r.Ri = Bi.tile_rows;
  r.b = (const uint8_t*)Bb.data + (tb * Bb.n_cols * r.Rb + (j - tb * r.Rb));
  r.f = (const double*)Bf.data + (tf * Bf.n_cols * r.Rf + (j - tf * r.Rf));
  r.i = (const int64_t*)Bi.data + (ti * Bi.n_cols * r.Ri + (j - ti * r.Ri));
  return r;
}

__device__ __forceinline__ double feature_value(const RowBases& r, int32_t slot) {
  const int kind = slot >> 24;
  const int64_t col = slot & 0xFFFFFF;
  if (kind == 0) return (double)r.b[col * r.Rb];
  if (kind == 1) return r.f[col * r.Rf];
  return (double)r.i[col * r.Ri];
}

template <bool F32, bool STAGED>
__global__ __launch_bounds__(TR_THREADS) void tree_predict_kernel(const TNode* __restrict__ nodes, int n_nodes,
                                                                   const int32_t* __restrict__ roots, int n_trees,
                                                                   const int32_t* __restrict__ slots, int n_slots,
                                                                   sa_block Bb, sa_block Bf, sa_block Bi,
                                                                   int64_t n, double base, int le,
                                                                   void* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char tr_lds[];  // nodes, then slots
  TNode* lds = reinterpret_cast<TNode*>(tr_lds);
  int32_t* lslots = reinterpret_cast<int32_t*>(tr_lds + (size_t)n_nodes * sizeof(TNode));
  // STAGED (host-checked: nodes and slots fit): every node / slot read is an LDS read; the
  // pointers must not be a runtime select between LDS and global, which compiles to flat
  // loads on the memory path
  if (STAGED) {
    for (int k = threadIdx.x; k < n_nodes; k += blockDim.x) lds[k] = nodes[k];
    for (int k = threadIdx.x; k < n_slots; k += blockDim.x) lslots[k] = slots[k];
    __syncthreads();
  }
  const TNode* __restrict__ N = STAGED ? lds : nodes;
  const int32_t* __restrict__ S = STAGED ? lslots : slots;
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const RowBases rb = row_bases(Bb, Bf, Bi, j);
  // TG trees walked together: their feature reads are independent, so a wave keeps TG loads
  // in flight instead of one dependent load per level; leaf values are added in tree order.
  using A = typename std::conditional<F32, float, double>::type;
  A m = (A)base;
  for (int t0 = 0; t0 < n_trees; t0 += TG) {
    int k[TG];
    A leafv[TG];
    uint32_t live = 0;
#pragma unroll
    for (int u = 0; u < TG; ++u) {
      k[u] = t0 + u < n_trees ? roots[t0 + u] : 0;
      leafv[u] = A(0);
      if (t0 + u < n_trees) live |= 1u << u;
    }
    while (live) {
#pragma unroll
      for (int u = 0; u < TG; ++u) {
        if (!(live & (1u << u))) continue;
        const TNode nd = N[k[u]];
        if (nd.feature < 0) {
          leafv[u] = (A)nd.thr_or_value;
          live &= ~(1u << u);
          continue;
        }
        const A v = (A)feature_value(rb, S[nd.feature]);
        const A thr = (A)nd.thr_or_value;
        const int right = nd.right & 0x7FFFFFFF;
        if (isnan(v))
          k[u] = nd.right < 0 ? nd.left : right;
        else
          k[u] = (le ? v <= thr : v < thr) ? nd.left : right;
      }
    }
#pragma unroll
    for (int u = 0; u < TG; ++u)
      if (t0 + u < n_trees) m = m + leafv[u];
  }
  if (F32)
    ((float*)out)[j] = 1.0f / (1.0f + expf(-(float)m));
  else
    ((double*)out)[j] = 1.0 / (1.0 + exp(-(double)m));
}

// Fixed-depth walk (tree_depth given, the model staged in LDS): leaves become self-loops (left =
// right = the leaf, a valid feature slot), so every tree of a TG-group is walked exactly the
// group's depth levels with no per-lane "still walking" state -- straight-line code instead of
// the divergent while-loop above, whose exec-mask juggling cost as many scalar as vector
// instructions.  Nodes are restaged with the feature slot in the node (one LDS read per level
// instead of two dependent ones) and the threshold in the model's arithmetic type.
template <typename A>
struct LNode {
  A thr;  // threshold (or the leaf value)
  int32_t slot, left, right;  // right: bit 31 = default_left
};

template <bool F32, bool LE>
__global__ __launch_bounds__(TR_THREADS) void tree_fixed_kernel(const TNode* __restrict__ nodes, int n_nodes,
                                                                 const int32_t* __restrict__ roots,
                                                                 const int32_t* __restrict__ depth, int n_trees,
                                                                 const int32_t* __restrict__ slots, sa_block Bb,
                                                                 sa_block Bf, sa_block Bi, int64_t n, double base,
                                                                 void* __restrict__ out) {
  using A = typename std::conditional<F32, float, double>::type;
  extern __shared__ __attribute__((aligned(16))) unsigned char tr_lds[];
  LNode<A>* L = reinterpret_cast<LNode<A>*>(tr_lds);
  __shared__ int32_t dummy_slot;
  if (threadIdx.x == 0) {  // the slot of the first split node: leaves read a feature that exists
    int32_t ds = 0;
    for (int k = 0; k < n_nodes; ++k)
      if (nodes[k].feature >= 0) {
        ds = slots[nodes[k].feature];
        break;
      }
    dummy_slot = ds;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < n_nodes; k += blockDim.x) {
    const TNode nd = nodes[k];
    LNode<A> o;
    o.thr = (A)nd.thr_or_value;
    if (nd.feature < 0) {
      o.slot = dummy_slot;
      o.left = k;
      o.right = k;
    } else {
      o.slot = slots[nd.feature];
      o.left = nd.left;
      o.right = nd.right;
    }
    L[k] = o;
  }
  __syncthreads();
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const RowBases rb = row_bases(Bb, Bf, Bi, j);
  A m = (A)base;
  for (int t0 = 0; t0 < n_trees; t0 += TG) {
    int k[TG];
    int D = 0;
#pragma unroll
    for (int u = 0; u < TG; ++u) {
      const int t = t0 + u < n_trees ? t0 + u : n_trees - 1;
      k[u] = roots[t];
      D = max(D, depth[t]);
    }
    for (int d = 0; d < D; ++d) {
#pragma unroll
      for (int u = 0; u < TG; ++u) {
        const LNode<A> nd = L[k[u]];
        const A v = (A)feature_value(rb, nd.slot);
        const bool left = isnan(v) ? nd.right < 0 : (LE ? v <= nd.thr : v < nd.thr);
        k[u] = left ? nd.left : (nd.right & 0x7FFFFFFF);
      }
    }
#pragma unroll
    for (int u = 0; u < TG; ++u)
      if (t0 + u < n_trees) m = m + L[k[u]].thr;
  }
  if (F32)
    ((float*)out)[j] = 1.0f / (1.0f + expf(-(float)m));
  else
    ((double*)out)[j] = 1.0 / (1.0 + exp(-(double)m));
}

// Staged condition walk (default when the model fits LDS).  Every split of the model is turned
// into a CONDITION whose outcome per row is one bit:
//   * a bool split: its column's value (a bool column whose threshold sends 0 and 1 the same
//     way is a constant split: condition 0, never set);
//   * a numeric split: (column, threshold, default direction) -- `x < thr` (xgboost, float32)
//     or `x <= thr` (scikit-learn, float64) goes left, NaN follows the default direction.
// Nodes are renumbered host-side so that each split's two children are adjacent, ordered (child
// on a clear bit, child on a set bit); a node is then 4 bytes {condition | first child << 16}
// and one level of the walk is child = first + bit.  A workgroup of 512 rows first evaluates
// every condition for its rows into LDS (64 B per condition: one bit per row; the used bool
// columns with one 16-B load per 16 rows, the distinct numeric columns with one coalesced 8-B
// load per row, TS_B columns in flight, each threshold a ballot), then walks the trees from
// LDS: per level a 4-B node read and a 1-B bit read, no branches, no float compares, no
// divergent global gathers.  Leaves are self-loops (condition 0, first child = the leaf), so
// an 8-tree group is walked exactly its depth; leaf values are summed in tree order: the
// gather walk's probabilities bit for bit.  Measured per 100-tree model on 16M actions
// (scripts/tree_probe.py): previous staged walk (bools staged, numeric splits gathered per
// level) 3.75 ms; a wave-uniform evaluation of every split by 64-bit lane masks 5.4 ms (its
// scalar instructions issue at the vector rate).
constexpr int TS_ROWS = 512;               // rows per tile
constexpr int TS_PIECES = TS_ROWS / 16;    // 16-row pieces per condition
constexpr int TS_CSTRIDE = TS_ROWS / 8 + 4;  // bytes per condition (+4: conditions start in different banks)
constexpr int TS_B = 8;                    // loads in flight per staging thread

template <typename A>
struct CondSet {  // the model's conditions
  const int32_t* bool_cols;
  const int32_t* num_cols;
  const int32_t* col_start;
  const A* num_thr;
  const int32_t* num_dl;
  int n_bool, n_ncol, n_num;
};

template <typename A>
struct CondModel {  // the model's walk
  const uint32_t* nodes;
  const A* leaf;
  const int32_t* roots;
  const int32_t* depth;
  int n_nodes, n_trees;
  double base;
  void* out;
};


// One value per lane against the thresholds of conditions [c0, c1): each condition's outcome over
// the wave's 64 rows as one 64-bit ballot into its LDS row (lane 0 writes it at M8w).  (Loading
// the thresholds 64 at a time and reading each back by v_readlane was slower here: 2.26 vs
// 1.97 ms per model, profiles/r06d -- the readlane -> compare chain serialises.)
template <typename A, bool LE>
__device__ __forceinline__ void ballot_conditions(const CondSet<A>& P, A x, int c0, int c1, int lane,
                                                  uint8_t* __restrict__ M8w) {
  for (int c = c0; c < c1; ++c) {
    const A thr = P.num_thr[c];
    const bool right = isnan(x) ? !P.num_dl[c] : !(LE ? x <= thr : x < thr);
    const uint64_t word = __ballot(right);
    if (lane == 0) {
      uint32_t* dst = reinterpret_cast<uint32_t*>(M8w + (1 + P.n_bool + c) * TS_CSTRIDE);
      dst[0] = (uint32_t)word;
      dst[1] = (uint32_t)(word >> 32);
    }
  }
}

// Condition bits of the TS_ROWS rows from R0 into M8 (TS_ROWS threads, s = 0 .. TS_ROWS-1; row
// R0 + s belongs to thread s, whole waves).
template <typename A, bool LE, bool N32>
__device__ __forceinline__ void stage_conditions(const CondSet<A>& P, const int32_t* __restrict__ BC,
                                                 const sa_block& Bb, const uint8_t* __restrict__ bits,
                                                 int64_t bstride, const sa_block& Bf, const sa_block& Bi, int64_t n,
                                                 int64_t R0, int s, uint8_t* __restrict__ M8) {
  const int wv = s >> 6, lane = s & 63;
  if (s < TS_CSTRIDE / 4) reinterpret_cast<uint32_t*>(M8)[s] = 0;  // condition 0: never set
  if (bits) {
    // bool conditions from bitmaps: item it = (column u, 64-row word q): one 8-B load
    constexpr int WQ = TS_ROWS / 64;
    const int nwi = P.n_bool * WQ;
    for (int i0 = 0; i0 < nwi; i0 += TS_ROWS * TS_B) {
      uint64_t w[TS_B];
#pragma unroll
      for (int b = 0; b < TS_B; ++b) {
        const int it = i0 + b * TS_ROWS + s;
        const int64_t r = R0 + 64 * (it % WQ);
        w[b] = it < nwi && r < n ? *reinterpret_cast<const uint64_t*>(bits + (int64_t)BC[it / WQ] * bstride + r / 8)
                                  : 0ull;
      }
#pragma unroll
      for (int b = 0; b < TS_B; ++b) {
        const int it = i0 + b * TS_ROWS + s;
        if (it < nwi) {
          uint32_t* dst = reinterpret_cast<uint32_t*>(M8 + (1 + it / WQ) * TS_CSTRIDE + 8 * (it % WQ));
          dst[0] = (uint32_t)w[b];
          dst[1] = (uint32_t)(w[b] >> 32);
        }
      }
    }
  }
  // bool conditions from the bool block: item it = (column u, 16-row piece p) -> 16 bits
  const int nbi = bits ? 0 : P.n_bool * TS_PIECES;
  for (int i0 = 0; i0 < nbi; i0 += TS_ROWS * TS_B) {
    u32x4 w[TS_B];
#pragma unroll
    for (int b = 0; b < TS_B; ++b) {
      const int it = i0 + b * TS_ROWS + s;
      w[b] = u32x4{0, 0, 0, 0};
      const int64_t r = R0 + 16 * (it % TS_PIECES);
      if (it < nbi && r < n) {
        const int64_t col = BC[it / TS_PIECES];
        SA_DCHECK(col >= 0 && col < Bb.n_cols, col);
        const int64_t t = r / Bb.tile_rows;
        w[b] = *reinterpret_cast<const u32x4*>((const uint8_t*)Bb.data + (t * Bb.n_cols + col) * Bb.tile_rows +
                                               (r - t * Bb.tile_rows));
      }
    }
#pragma unroll
    for (int b = 0; b < TS_B; ++b) {
      const int it = i0 + b * TS_ROWS + s;
      uint32_t bits = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) bits |= (((w[b][q] & 0x01010101u) * 0x01020408u) >> 24) << (4 * q);
      if (it < nbi)
        *reinterpret_cast<uint16_t*>(M8 + (1 + it / TS_PIECES) * TS_CSTRIDE + 2 * (it % TS_PIECES)) = (uint16_t)bits;
    }
  }
  // numeric conditions: the distinct numeric columns num_cols[q] are read TS_B at a time (one
  // 8-B load per row and column, all in flight before use), then column q's thresholds
  // (conditions col_start[q] .. col_start[q+1]) are balloted into the wave's 64-bit words
  const int64_t j = R0 + s < n ? R0 + s : n - 1;
  if (N32) {  // float32 numeric blocks (sa_vaep_features_bits_f32): one 4-B load per row and column
    const int64_t tf = j / Bf.tile_rows, ti = j / Bi.tile_rows;
    const float* pf = (const float*)Bf.data + (tf * Bf.n_cols * Bf.tile_rows + (j - tf * Bf.tile_rows));
    const float* pi = (const float*)Bi.data + (ti * Bi.n_cols * Bi.tile_rows + (j - ti * Bi.tile_rows));
    for (int q0 = 0; q0 < P.n_ncol; q0 += TS_B) {
      float raw[TS_B];
#pragma unroll
      for (int b = 0; b < TS_B; ++b) {
        const int32_t slot = P.num_cols[q0 + b < P.n_ncol ? q0 + b : P.n_ncol - 1];
        const bool f = (slot >> 24) == 1;
        raw[b] = f ? pf[(int64_t)(slot & 0xFFFFFF) * Bf.tile_rows] : pi[(int64_t)(slot & 0xFFFFFF) * Bi.tile_rows];
      }
#pragma unroll
      for (int b = 0; b < TS_B; ++b) {
        const int q = q0 + b;
        if (q >= P.n_ncol) break;
        const A x = (A)raw[b];
        ballot_conditions<A, LE>(P, x, P.col_start[q], P.col_start[q + 1], lane, M8 + 8 * wv);
      }
    }
    return;
  }
  const RowBases rb = row_bases(Bb, Bf, Bi, j);
  for (int q0 = 0; q0 < P.n_ncol; q0 += TS_B) {
    uint64_t raw[TS_B];
#pragma unroll
    for (int b = 0; b < TS_B; ++b) {
      const int32_t slot = P.num_cols[q0 + b < P.n_ncol ? q0 + b : P.n_ncol - 1];
      const bool f = (slot >> 24) == 1;
      const uint64_t* base = f ? reinterpret_cast<const uint64_t*>(rb.f) : reinterpret_cast<const uint64_t*>(rb.i);
      raw[b] = base[(int64_t)(slot & 0xFFFFFF) * (f ? rb.Rf : rb.Ri)];
    }
#pragma unroll
    for (int b = 0; b < TS_B; ++b) {
      const int q = q0 + b;
      if (q >= P.n_ncol) break;
      const A x = (P.num_cols[q] >> 24) == 1 ? (A)__longlong_as_double((long long)raw[b]) : (A)(double)(int64_t)raw[b];
      ballot_conditions<A, LE>(P, x, P.col_start[q], P.col_start[q + 1], lane, M8 + 8 * wv);
    }
  }
}

// Row R0 + s (s = 0 .. TS_ROWS-1) through every tree from the staged conditions M8.
// RD: the roots (RD[t]) and depths (RD[TSP + t]) staged in LDS, padded to whole groups of TG
// (TSP = n_trees rounded up to TG): a group's roots and depths are uniform LDS reads.  Loaded
// per tree from global memory they cost ~90 scalar instructions per group of 8 trees (address
// arithmetic and serialised waits), the walk's whole scalar budget (SQ_INSTS_SALU 1,159 per
// wave of 2,523 VALU, profiles/r06t).
// SCALED: the nodes' condition halves hold the condition's byte offset in M8 (condition x
// TS_CSTRIDE, staged so when it fits 16 bits): the bit's address is then one add of the node's
// low half, not a mask and a multiply-add (the walk is bound by VALU issue: 5 -> 4 per level).
template <typename A, bool SCALED = false>
__device__ __forceinline__ A walk_conditions(const CondModel<A>& P, const uint32_t* __restrict__ N,
                                             const A* __restrict__ LV, const uint8_t* __restrict__ M8,
                                             const int32_t* __restrict__ RD, int TSP, int s) {
  const uint8_t* Mrow = M8 + (s >> 3);  // this row's byte of every condition
  const int rbit = s & 7;
  A m = (A)P.base;
  for (int t0 = 0; t0 < P.n_trees; t0 += TG) {
    int k[TG];
    int D = 0;
#pragma unroll
    for (int u = 0; u < TG; ++u) {
      k[u] = RD[t0 + u];
      D = max(D, RD[TSP + t0 + u]);
    }
    for (int d = 0; d < D; ++d) {
      uint32_t nd[TG];
#pragma unroll
      for (int u = 0; u < TG; ++u) nd[u] = N[k[u]];
#pragma unroll
      for (int u = 0; u < TG; ++u) {
        const uint32_t bit = (Mrow[SCALED ? (nd[u] & 0xFFFFu) : (nd[u] & 0xFFFFu) * TS_CSTRIDE] >> rbit) & 1u;
        k[u] = (int)(nd[u] >> 16) + (int)bit;
      }
    }
    A lv[TG];
#pragma unroll
    for (int u = 0; u < TG; ++u) lv[u] = LV[k[u]];
#pragma unroll
    for (int u = 0; u < TG; ++u)
      if (t0 + u < P.n_trees) m = m + lv[u];
  }
  return m;
}

// One workgroup per tile: its 512 threads stage the tile's conditions, then walk its rows.
// Measured alternatives (scripts/tree_probe.py, 100-tree depth-3 model, 16M actions): persistent
// workgroups of 16 waves in two roles -- 8 staging tile i+1 while 8 walk tile i -- 7.6 ms (one
// such workgroup per CU leaves the staging too few loads in flight); both VAEP.rate learners in
// one launch over the union of their conditions 6.8 ms vs 2 x 2.9 (the larger LDS footprint
// halves the resident workgroups); 256- / 1024-row tiles 3.0 / 3.7 ms.
template <bool F32, bool LE, bool N32 = false>
__global__ __launch_bounds__(TS_ROWS) void tree_cond_kernel(CondSet<typename std::conditional<F32, float, double>::type> C,
                                                            CondModel<typename std::conditional<F32, float, double>::type> P,
                                                            sa_block Bb, const uint8_t* __restrict__ bits, int64_t bstride,
                                                            sa_block Bf, sa_block Bi, int64_t n) {
  using A = typename std::conditional<F32, float, double>::type;
  extern __shared__ __attribute__((aligned(16))) unsigned char ts_lds[];
  // LDS carved by integer offsets from ts_lds (a pointer cast through uintptr_t would make
  // every access a flat one): conditions, nodes, leaf values
  const int n_cond = 1 + C.n_bool + C.n_num;
  const size_t moff = ((size_t)n_cond * TS_CSTRIDE + 15) / 16 * 16;
  uint8_t* M8 = ts_lds;
  uint32_t* N = reinterpret_cast<uint32_t*>(ts_lds + moff);
  A* LV = reinterpret_cast<A*>(ts_lds + moff + (size_t)(P.n_nodes + (P.n_nodes & 1)) * 4);
  const int TSP = (P.n_trees + TG - 1) / TG * TG;
  int32_t* RD = reinterpret_cast<int32_t*>(ts_lds + moff + (size_t)(P.n_nodes + (P.n_nodes & 1)) * 4 +
                                           (size_t)(P.n_nodes + (P.n_nodes & 1)) * sizeof(A));
  int32_t* BC = RD + 2 * TSP;  // the bool conditions' columns / bitmap rows
  const int tid = threadIdx.x;
  const bool scaled = SA_TREE_SCALED && (int64_t)n_cond * TS_CSTRIDE <= 0x10000;  // uniform
  for (int k = tid; k < P.n_nodes; k += TS_ROWS) {
    const uint32_t nd = P.nodes[k];
    N[k] = scaled ? (nd & 0xFFFF0000u) | ((nd & 0xFFFFu) * TS_CSTRIDE) : nd;
    LV[k] = P.leaf[k];
  }
  for (int t = tid; t < TSP; t += TS_ROWS) {  // padding: the last tree again, depth 0 (not summed)
    RD[t] = P.roots[t < P.n_trees ? t : P.n_trees - 1];
    RD[TSP + t] = t < P.n_trees ? P.depth[t] : 0;
  }
  for (int k = tid; k < C.n_bool; k += TS_ROWS) BC[k] = C.bool_cols[k];
  __syncthreads();
  // tiles blockIdx.x, + gridDim.x, ...: the model's tables above are staged once per workgroup
  // (the grid is sized to the resident workgroups when SA_TREE_PERSIST, else one per tile)
  const int64_t tiles = (n + TS_ROWS - 1) / TS_ROWS;
  for (int64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const int64_t R0 = tile * TS_ROWS;
    stage_conditions<A, LE, N32>(C, BC, Bb, bits, bstride, Bf, Bi, n, R0, tid, M8);
    __syncthreads();
    const int64_t j = R0 + tid;
    if (j < n) {
      const A m = scaled ? walk_conditions<A, true>(P, N, LV, M8, RD, TSP, tid)
                         : walk_conditions<A, false>(P, N, LV, M8, RD, TSP, tid);
      if (F32)
        ((float*)P.out)[j] = 1.0f / (1.0f + expf(-(float)m));
      else
        ((double*)P.out)[j] = 1.0 / (1.0 + exp(-(double)m));
    }
    __syncthreads();  // every row walked before the next tile's conditions overwrite M8
  }
}

}  // namespace sa

using namespace sa;

extern "C" int sa_tree_predict(const void* nodes, int32_t n_nodes, const int32_t* roots, const int32_t* tree_depth,
                               int32_t n_trees, const int32_t* feature_slots, int32_t n_features,
                               const sa_block* bool_blk, const sa_block* f64_blk, const sa_block* i64_blk,
                               int64_t n, double base_margin, int32_t le, int32_t f32, void* p_out,
                               void* stream) {
  if (n < 0 || n_nodes < 1 || n_trees < 0 || n_features < 0 || !nodes || !roots || !p_out ||
      (n_features > 0 && !feature_slots))
    return fail(SA_EINVAL, "bad tree model arguments");
  sa_block z{nullptr, 0, 0, 16};  // absent block: never read (no slot refers to it)
  const sa_block Bb = bool_blk ? *bool_blk : z, Bf = f64_blk ? *f64_blk : z, Bi = i64_blk ? *i64_blk : z;
  if (n == 0) return SA_OK;
  const dim3 grid((unsigned)((n + TR_THREADS - 1) / TR_THREADS)), block(TR_THREADS);
  hipStream_t st = (hipStream_t)stream;
  const TNode* nd = (const TNode*)nodes;
  const bool staged = n_nodes <= TR_LDS_NODES && n_features <= TR_LDS_SLOTS;
  const size_t lds_bytes = (size_t)n_nodes * sizeof(TNode) + (size_t)n_features * sizeof(int32_t);
  if (SA_TREE_FIXED && tree_depth && n_nodes <= TR_LDS_NODES && n_trees > 0) {
    const size_t fb = (size_t)n_nodes * (f32 ? sizeof(LNode<float>) : sizeof(LNode<double>));
#define SA_TREE_FIXED_LAUNCH(F, LEQ)                                                                    \
  hipLaunchKernelGGL((tree_fixed_kernel<F, LEQ>), grid, block, fb, st, nd, n_nodes, roots, tree_depth, n_trees, \
                     feature_slots, Bb, Bf, Bi, n, base_margin, p_out)
    if (f32 && le)
      SA_TREE_FIXED_LAUNCH(true, true);
    else if (f32)
      SA_TREE_FIXED_LAUNCH(true, false);
    else if (le)
      SA_TREE_FIXED_LAUNCH(false, true);
    else
      SA_TREE_FIXED_LAUNCH(false, false);
#undef SA_TREE_FIXED_LAUNCH
    return check_launch("tree_fixed_kernel");
  }
#define SA_TREE_LAUNCH(F, S)                                                                       \
  hipLaunchKernelGGL((tree_predict_kernel<F, S>), grid, block, S ? lds_bytes : 0, st, nd, n_nodes, roots, n_trees, \
                     feature_slots, n_features, Bb, Bf, Bi, n, base_margin, le, p_out)
  if (f32 && staged)
    SA_TREE_LAUNCH(true, true);
  else if (f32)
    SA_TREE_LAUNCH(true, false);
  else if (staged)
    SA_TREE_LAUNCH(false, true);
  else
    SA_TREE_LAUNCH(false, false);
#undef SA_TREE_LAUNCH
  return check_launch("tree_predict_kernel");
}

// The staged walk's LDS: conditions, nodes, leaf values, then the roots and depths padded to
// whole tree groups.
static int64_t staged_lds_bytes(int32_t n_nodes, int32_t n_cond, int32_t f32, int32_t n_trees) {
  const int64_t np = n_nodes + (n_nodes & 1);
  return ((int64_t)n_cond * TS_CSTRIDE + 15) / 16 * 16 + np * 4 + np * (f32 ? 4 : 8) +
         (int64_t)(n_trees + TG - 1) / TG * TG * 8 + (int64_t)n_cond * 4;
}
// (a model has at most n_nodes trees: the bound a caller without the tree count can use)
extern "C" int64_t sa_tree_staged_lds_bytes(int32_t n_nodes, int32_t n_cond, int32_t f32) {
  return staged_lds_bytes(n_nodes, n_cond, f32, n_nodes);
}

extern "C" int sa_tree_predict_staged(const sa_tree_model* model, const int32_t* bool_cols, int32_t n_bool,
                                      const int32_t* num_cols, const int32_t* col_start, int32_t n_ncol,
                                      const void* num_thr, const int32_t* num_dl, int32_t n_num,
                                      const sa_block* bool_blk, const uint8_t* bool_bits, int64_t bits_stride,
                                      const sa_block* f64_blk, const sa_block* i64_blk, int64_t n, int32_t le,
                                      int32_t f32, void* stream) {
  if (!model || n < 0 || 1 + n_bool + n_num > 65536 || n_bool < 0 || n_num < 0 ||
      (n_bool > 0 && (!bool_cols || (!bool_blk && !bool_bits))) || n_ncol < 0 ||
      (bool_bits && (bits_stride % 8 || bits_stride < 8 * ((n + 63) / 64) || ((uintptr_t)bool_bits & 7u))) ||
      (n_num > 0 && (n_ncol < 1 || !num_cols || !col_start || !num_thr || !num_dl)))
    return fail(SA_EINVAL, "bad staged tree arguments");
  const sa_tree_model& m = *model;
  if (m.n_nodes < 1 || m.n_nodes > 65535 || m.n_trees < 1 || !m.nodes || !m.leaf || !m.roots || !m.tree_depth ||
      !m.p_out)
    return fail(SA_EINVAL, "bad staged tree model");
  const int64_t lds = staged_lds_bytes(m.n_nodes, 1 + n_bool + n_num, f32 & 1, m.n_trees);
  if (lds > 160 * 1024) return fail(SA_EINVAL, "staged tree model needs %lld B of LDS", (long long)lds);
  sa_block z{nullptr, 0, 0, 16};
  const sa_block Bb = bool_blk ? *bool_blk : z, Bf = f64_blk ? *f64_blk : z, Bi = i64_blk ? *i64_blk : z;
  if (n_bool > 0 && !bool_bits && (Bb.tile_rows % 16 != 0 || !aligned16(Bb.data)))
    return fail(SA_EINVAL, "bool block: 16-row tiles, 16-byte aligned");
  if (n == 0) return SA_OK;
  const int64_t tiles = (n + TS_ROWS - 1) / TS_ROWS;
  const dim3 block(TS_ROWS);
  hipStream_t st = (hipStream_t)stream;
  // SA_TREE_PERSIST: as many workgroups as are resident at once (each stages the model's tables
  // once and loops over tiles); else one workgroup per tile
#define SA_TS_LAUNCH(F, LEQ, A, N32)                                                                     \
  do {                                                                                                  \
    CondSet<A> C{bool_cols, num_cols, col_start, (const A*)num_thr, num_dl, n_bool, n_num > 0 ? n_ncol : 0, \
                 n_num};                                                                                \
    CondModel<A> P{(const uint32_t*)m.nodes, (const A*)m.leaf, m.roots, m.tree_depth, m.n_nodes,        \
                   m.n_trees,                m.base_margin,    m.p_out};                                \
    int64_t g = tiles;                                                                                  \
    if (SA_TREE_PERSIST) {                                                                              \
      int per_cu = 0;                                                                                   \
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, tree_cond_kernel<F, LEQ, N32>, TS_ROWS, \
                                                       (size_t)lds) != hipSuccess || per_cu < 1)        \
        per_cu = 1;                                                                                     \
      g = std::min<int64_t>(tiles, (int64_t)per_cu * device_cus(current_device()) * SA_TREE_PERSIST);   \
    }                                                                                                   \
    hipLaunchKernelGGL((tree_cond_kernel<F, LEQ, N32>), dim3((unsigned)g), block, (size_t)lds, st, C, P, Bb, \
                       bool_bits, bits_stride, Bf, Bi, n);                                               \
  } while (0)
  const bool n32 = (f32 & 2) != 0;  // float32 numeric blocks
  if (n32 && !(f32 & 1)) return fail(SA_EINVAL, "float32 numeric blocks need float32 (xgboost) arithmetic");
  if (n32 && le)
    SA_TS_LAUNCH(true, true, float, true);
  else if (n32)
    SA_TS_LAUNCH(true, false, float, true);
  else if (f32 && le)
    SA_TS_LAUNCH(true, true, float, false);
  else if (f32)
    SA_TS_LAUNCH(true, false, float, false);
  else if (le)
    SA_TS_LAUNCH(false, true, double, false);
  else
    SA_TS_LAUNCH(false, false, double, false);
#undef SA_TS_LAUNCH
  return check_launch("tree_cond_kernel");
}
