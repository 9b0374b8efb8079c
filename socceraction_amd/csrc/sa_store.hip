// Arrow export of the bool blocks (the per-game feature / label stores
// the notebooks write, public-notebooks/2-compute-features-and-labels.ipynb `X.to_hdf(...)`).
//
// Arrow (and Parquet's in-memory form) keeps a bool column as a validity-free bitmap, least
// significant bit first. The feature blocks hold one byte per value (the reference's numpy
// bool), so packing on the host costs a pass over 515 B/action and ships 8x the bytes over
// PCIe; here the bitmaps are built where the bytes are: one thread turns 16 consecutive rows of
// one column (one 16-B load from the tiled block) into 2 bitmap bytes, so the loads of a wave
// are 1 KiB contiguous and its stores 128 B contiguous. Rows >= n are zero bits.
#include <hip/hip_runtime.h>

#include "sa_common.h"
#include "sa_internal.h"

namespace sa {

constexpr int PB_THREADS = 256;

__global__ __launch_bounds__(PB_THREADS) void pack_bits_kernel(const uint8_t* __restrict__ src, int32_t C,
                                                               int64_t R, int64_t n, int64_t groups,
                                                               uint8_t* __restrict__ bits, int64_t stride) {
  const int64_t gid = (int64_t)blockIdx.x * PB_THREADS + threadIdx.x;  // 16-row group of column y
  const int col = blockIdx.y;
  if (gid >= groups) return;
  const int64_t r0 = gid * 16;
  const int64_t tile = r0 / R, off = r0 - tile * R;
  const uint4 v = *reinterpret_cast<const uint4*>(src + (tile * C + col) * R + off);
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t b = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int k = 0; k < 4; ++k) b |= (uint32_t)(((w[q] >> (8 * k)) & 0xFFu) != 0) << (q * 4 + k);
  const int64_t valid = n - r0;
  if (valid < 16) b &= (1u << valid) - 1u;
  *reinterpret_cast<uint16_t*>(bits + col * stride + gid * 2) = (uint16_t)b;
}

}  // namespace sa

using namespace sa;

extern "C" int sa_pack_bits(const sa_block* blk, int64_t n, uint8_t* bits, int64_t col_stride, void* stream) {
  if (!blk || n < 0 || blk->n_cols < 0) return fail(SA_EINVAL, "bad sa_pack_bits arguments");
  if (n == 0 || blk->n_cols == 0) return SA_OK;
  const int64_t groups = (n + 15) / 16;
  if (!blk->data || !bits) return fail(SA_EINVAL, "null block or bitmap");
  if (blk->tile_rows < 16 || blk->tile_rows % 16 || !aligned16(blk->data))
    return fail(SA_EINVAL, "bool block tiles must be multiples of 16 rows, 16-byte aligned");
  if (col_stride < 2 * groups || col_stride % 2 || ((uintptr_t)bits & 1u))
    return fail(SA_EINVAL, "bitmap column stride must be even and hold ceil(n/16)*2 bytes");
  if (blk->n_cols > 65535) return fail(SA_EINVAL, "too many columns");
  const dim3 grid((unsigned)((groups + PB_THREADS - 1) / PB_THREADS), (unsigned)blk->n_cols);
  hipLaunchKernelGGL(pack_bits_kernel, grid, dim3(PB_THREADS), 0, (hipStream_t)stream, (const uint8_t*)blk->data,
                     blk->n_cols, blk->tile_rows, n, groups, bits, col_stride);
  return check_launch("pack_bits_kernel");
}
