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
// The model's nodes are staged in LDS when they fit (a default 100-tree depth-3 model is 36 KB)
// so the per-node loads of divergent lanes are LDS reads; feature values are read from the
// tiled blocks (row j of a column is contiguous across lanes: coalesced at the root, L2-resident
// afterwards).
#include <hip/hip_runtime.h>

#include <cmath>

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

constexpr int TR_THREADS = 256;
constexpr int TR_LDS_NODES = 2048;  // 48 KB

__device__ __forceinline__ double feature_value(const sa_block& Bb, const sa_block& Bf,
                                                const sa_block& Bi, int32_t slot, int64_t j) {
  const int kind = slot >> 24, col = slot & 0xFFFFFF;
  if (kind == 0) {
    const int64_t R = Bb.tile_rows, t = j / R;
    return (double)((const uint8_t*)Bb.data)[t * Bb.n_cols * R + (int64_t)col * R + (j - t * R)];
  }
  if (kind == 1) {
    const int64_t R = Bf.tile_rows, t = j / R;
    return ((const double*)Bf.data)[t * Bf.n_cols * R + (int64_t)col * R + (j - t * R)];
  }
  const int64_t R = Bi.tile_rows, t = j / R;
  return (double)((const int64_t*)Bi.data)[t * Bi.n_cols * R + (int64_t)col * R + (j - t * R)];
}

template <bool F32>
__global__ __launch_bounds__(TR_THREADS) void tree_predict_kernel(const TNode* __restrict__ nodes, int n_nodes,
                                                                   const int32_t* __restrict__ roots, int n_trees,
                                                                   const int32_t* __restrict__ slots,
                                                                   sa_block Bb, sa_block Bf, sa_block Bi,
                                                                   int64_t n, double base, int le,
                                                                   void* __restrict__ out) {
  __shared__ TNode lds[TR_LDS_NODES];
  const bool staged = n_nodes <= TR_LDS_NODES;
  if (staged) {
    for (int k = threadIdx.x; k < n_nodes; k += blockDim.x) lds[k] = nodes[k];
    __syncthreads();
  }
  const TNode* __restrict__ N = staged ? lds : nodes;
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  if (F32) {
    float m = (float)base;
    for (int t = 0; t < n_trees; ++t) {
      int k = roots[t];
      for (;;) {
        const TNode nd = N[k];
        if (nd.feature < 0) {
          m = m + (float)nd.thr_or_value;
          break;
        }
        const float v = (float)feature_value(Bb, Bf, Bi, slots[nd.feature], j);
        const bool dl = nd.right < 0;
        const int right = nd.right & 0x7FFFFFFF;
        if (isnan(v))
          k = dl ? nd.left : right;
        else
          k = (le ? v <= (float)nd.thr_or_value : v < (float)nd.thr_or_value) ? nd.left : right;
      }
    }
    ((float*)out)[j] = 1.0f / (1.0f + expf(-m));
  } else {
    double m = base;
    for (int t = 0; t < n_trees; ++t) {
      int k = roots[t];
      for (;;) {
        const TNode nd = N[k];
        if (nd.feature < 0) {
          m = m + nd.thr_or_value;
          break;
        }
        const double v = feature_value(Bb, Bf, Bi, slots[nd.feature], j);
        const bool dl = nd.right < 0;
        const int right = nd.right & 0x7FFFFFFF;
        if (isnan(v))
          k = dl ? nd.left : right;
        else
          k = (le ? v <= nd.thr_or_value : v < nd.thr_or_value) ? nd.left : right;
      }
    }
    ((double*)out)[j] = 1.0 / (1.0 + exp(-m));
  }
}

}  // namespace sa

using namespace sa;

extern "C" int sa_tree_predict(const void* nodes, int32_t n_nodes, const int32_t* roots, int32_t n_trees,
                               const int32_t* feature_slots, int32_t n_features, const sa_block* bool_blk,
                               const sa_block* f64_blk, const sa_block* i64_blk, int64_t n, double base_margin,
                               int32_t le, int32_t f32, void* p_out, void* stream) {
  if (n < 0 || n_nodes < 1 || n_trees < 0 || n_features < 0 || !nodes || !roots || !p_out ||
      (n_features > 0 && !feature_slots))
    return fail(SA_EINVAL, "bad tree model arguments");
  sa_block z{nullptr, 0, 0, 16};
  const sa_block Bb = bool_blk ? *bool_blk : z, Bf = f64_blk ? *f64_blk : z, Bi = i64_blk ? *i64_blk : z;
  if (n == 0) return SA_OK;
  const dim3 grid((unsigned)((n + TR_THREADS - 1) / TR_THREADS)), block(TR_THREADS);
  hipStream_t st = (hipStream_t)stream;
  const TNode* nd = (const TNode*)nodes;
  if (f32)
    hipLaunchKernelGGL(tree_predict_kernel<true>, grid, block, 0, st, nd, n_nodes, roots, n_trees, feature_slots,
                       Bb, Bf, Bi, n, base_margin, le, p_out);
  else
    hipLaunchKernelGGL(tree_predict_kernel<false>, grid, block, 0, st, nd, n_nodes, roots, n_trees,
                       feature_slots, Bb, Bf, Bi, n, base_margin, le, p_out);
  return check_launch("tree_predict_kernel");
}
