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
#ifndef SA_TREE_TG
#define SA_TREE_TG 8
#endif
#ifndef SA_TREE_FIXED
#define SA_TREE_FIXED 1  // tree_depth given: fixed-depth walk over self-looping leaves
#endif
constexpr int TG = SA_TREE_TG;      // trees walked together per thread

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

// Staged walk: the model's used BOOL feature columns of the workgroup's rows are copied into LDS
// once, packed to one bit per row, and every tree is walked from LDS.  The gathers of
// tree_fixed_kernel are divergent loads -- one per lane, level and tree, ~582 B/action for a
// 100-tree model, served a few lanes at a time by the memory pipeline.  Here a workgroup of
// 512 rows first reads the used bool columns of its rows with coalesced 16-B loads (515 of the
// 568 default features are bool; a column's 512 rows become 8 u64, one per wave, and a level
// reads the wave's u64 and shifts by the lane); the few numeric features stay gathers from the
// f64 / i64 blocks (row bases computed once per thread).  Nodes are restaged (host-prepared,
// `SNode`) with the feature as a compact reference: bit 30 = numeric, the rest = index into
// the bool column list or the numeric slot list; leaves are self-loops, so every tree of a
// group is walked exactly the group's depth (tree_fixed_kernel's fixed-depth walk).  Values,
// split rule and summation order equal tree_fixed_kernel's bit for bit.
constexpr int TS_ROWS = 512;              // rows (threads) per workgroup
constexpr int TS_WAVES = TS_ROWS / 64;
constexpr int TS_PIECES = TS_ROWS / 16;   // 16-row pieces per column
constexpr int32_t TS_NUM = 1 << 30;

template <typename A>
struct SNode {
  A thr;                      // threshold, or the leaf value
  int32_t ref, left, right;   // right: bit 31 = default_left
};

template <bool F32, bool LE>
__global__ __launch_bounds__(TS_ROWS) void tree_staged_kernel(const SNode<typename std::conditional<F32, float, double>::type>* __restrict__ nodes,
                                                              int n_nodes, const int32_t* __restrict__ roots,
                                                              const int32_t* __restrict__ depth, int n_trees,
                                                              const int32_t* __restrict__ bool_cols, int n_bool,
                                                              const int32_t* __restrict__ num_slots, int n_num,
                                                              sa_block Bb, sa_block Bf, sa_block Bi, int64_t n,
                                                              double base, void* __restrict__ out) {
  using A = typename std::conditional<F32, float, double>::type;
  extern __shared__ __attribute__((aligned(16))) unsigned char ts_lds[];
  SNode<A>* L = reinterpret_cast<SNode<A>*>(ts_lds);
  const size_t node_bytes = ((size_t)n_nodes * sizeof(SNode<A>) + 15) / 16 * 16;
  const int nb = n_bool > 0 ? n_bool : 1, nn = n_num > 0 ? n_num : 1;
  uint16_t* M16 = reinterpret_cast<uint16_t*>(ts_lds + node_bytes);            // [nb][TS_PIECES]
  const uint64_t* M = reinterpret_cast<const uint64_t*>(M16);                  // [nb][TS_WAVES]
  int32_t* NS = reinterpret_cast<int32_t*>(ts_lds + node_bytes + (size_t)nb * TS_ROWS / 8);  // [nn]
  int32_t* BC = NS + nn;                                                       // [nb]
  const int tid = threadIdx.x;
  const int64_t R0 = (int64_t)blockIdx.x * TS_ROWS;
  for (int k = tid; k < n_num; k += TS_ROWS) NS[k] = num_slots[k];
  for (int k = tid; k < n_bool; k += TS_ROWS) BC[k] = bool_cols[k];
  if (n_num == 0 && tid == 0) NS[0] = 1 << 24;
  if (n_bool == 0 && tid < TS_PIECES) M16[tid] = 0;
  // every load of a staging pass is issued before any is used (TS_B per thread in flight)
  constexpr int TS_B = 8;
  for (int k0 = 0; k0 < n_nodes; k0 += TS_ROWS * TS_B) {
#pragma unroll
    for (int b = 0; b < TS_B; ++b) {
      const int k = k0 + b * TS_ROWS + tid;
      if (k < n_nodes) L[k] = nodes[k];
    }
  }
  __syncthreads();  // BC
  {
    // bool columns: item it = (column u = it / TS_PIECES, 16-row piece p): one 16-B load of the
    // piece -> 16 bits at M16[it]
    const int nbi = n_bool * TS_PIECES;
    for (int i0 = 0; i0 < nbi; i0 += TS_ROWS * TS_B) {
      u32x4 w[TS_B];
#pragma unroll
      for (int b = 0; b < TS_B; ++b) {
        const int it = i0 + b * TS_ROWS + tid;
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
        const int it = i0 + b * TS_ROWS + tid;
        uint32_t bits = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) bits |= (((w[b][q] & 0x01010101u) * 0x01020408u) >> 24) << (4 * q);
        if (it < nbi) M16[it] = (uint16_t)bits;
      }
    }
  }
  __syncthreads();
  const int64_t j = R0 + tid;
  if (j >= n) return;
  const int wv = tid >> 6, lane = tid & 63;
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
      // the TG trees' node reads, then all their feature reads (the numeric gathers of the
      // lanes that need one go out together: one memory latency per level, not TG), then the
      // decisions
      SNode<A> nd[TG];
#pragma unroll
      for (int u = 0; u < TG; ++u) nd[u] = L[k[u]];
      A v[TG];
#pragma unroll
      for (int u = 0; u < TG; ++u) {
        const int idx = nd[u].ref & (TS_NUM - 1);
        SA_DCHECK((nd[u].ref & TS_NUM) ? idx < nn : idx < nb, nd[u].ref);
        if (nd[u].ref & TS_NUM) v[u] = (A)feature_value(rb, NS[idx]);
      }
#pragma unroll
      for (int u = 0; u < TG; ++u) {
        const int idx = nd[u].ref & (TS_NUM - 1);
        if (!(nd[u].ref & TS_NUM)) v[u] = (A)((M[idx * TS_WAVES + wv] >> lane) & 1ull);
        const bool left = isnan(v[u]) ? nd[u].right < 0 : (LE ? v[u] <= nd[u].thr : v[u] < nd[u].thr);
        k[u] = left ? nd[u].left : (nd[u].right & 0x7FFFFFFF);
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

extern "C" int64_t sa_tree_staged_lds_bytes(int32_t n_nodes, int32_t n_bool, int32_t n_num, int32_t f32) {
  const size_t node = f32 ? sizeof(SNode<float>) : sizeof(SNode<double>);
  const size_t nb = n_bool > 0 ? n_bool : 1, nn = n_num > 0 ? n_num : 1;
  return (int64_t)(((size_t)n_nodes * node + 15) / 16 * 16 + nb * TS_ROWS / 8 + (nn + nb) * 4);
}

extern "C" int sa_tree_predict_staged(const void* snodes, int32_t n_nodes, const int32_t* roots,
                                      const int32_t* tree_depth, int32_t n_trees, const int32_t* bool_cols,
                                      int32_t n_bool, const int32_t* num_slots, int32_t n_num,
                                      const sa_block* bool_blk, const sa_block* f64_blk,
                                      const sa_block* i64_blk, int64_t n, double base_margin, int32_t le,
                                      int32_t f32, void* p_out, void* stream) {
  if (n < 0 || n_nodes < 1 || n_trees < 1 || n_bool < 0 || n_num < 0 || !snodes || !roots ||
      !tree_depth || !p_out || (n_bool > 0 && (!bool_cols || !bool_blk)) || (n_num > 0 && !num_slots))
    return fail(SA_EINVAL, "bad staged tree model arguments");
  const int64_t lds = sa_tree_staged_lds_bytes(n_nodes, n_bool, n_num, f32);
  if (lds > 160 * 1024) return fail(SA_EINVAL, "staged tree model needs %lld B of LDS", (long long)lds);
  sa_block z{nullptr, 0, 0, 16};
  const sa_block Bb = bool_blk ? *bool_blk : z, Bf = f64_blk ? *f64_blk : z, Bi = i64_blk ? *i64_blk : z;
  if (n_bool > 0 && (Bb.tile_rows % 16 != 0 || !aligned16(Bb.data)))
    return fail(SA_EINVAL, "bool block: 16-row tiles, 16-byte aligned");
  if (n == 0) return SA_OK;
  const dim3 grid((unsigned)((n + TS_ROWS - 1) / TS_ROWS)), block(TS_ROWS);
  hipStream_t st = (hipStream_t)stream;
#define SA_TS_LAUNCH(F, LEQ, A)                                                                         \
  hipLaunchKernelGGL((tree_staged_kernel<F, LEQ>), grid, block, (size_t)lds, st,                         \
                     (const SNode<A>*)snodes, n_nodes, roots, tree_depth, n_trees, bool_cols, n_bool,       \
                     num_slots, n_num, Bb, Bf, Bi, n, base_margin, p_out)
  if (f32 && le)
    SA_TS_LAUNCH(true, true, float);
  else if (f32)
    SA_TS_LAUNCH(true, false, float);
  else if (le)
    SA_TS_LAUNCH(false, true, double);
  else
    SA_TS_LAUNCH(false, false, double);
#undef SA_TS_LAUNCH
  return check_launch("tree_staged_kernel");
}
