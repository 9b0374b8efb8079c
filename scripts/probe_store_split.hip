// Store-granularity probe for the bool block.  Question: is the bool kernel's gap to a
// plain fill the layout, or the wave granularity (each wave owns a whole 515-column x
// 1024-row tile = 515 KiB, so a 16M-action launch is only ~2.5 waves per resident slot and
// the drain at the end runs the chip part empty)?  Every variant writes the same tiled
// [tiles][C][1024] image with 16-B non-temporal stores:
//   tile16      one wave per tile, all C columns (the round-1 bool_features_kernel shape)
//   split<S>    S waves per tile, wave s writes the contiguous column range s*C/S ..
//   *_occ24     LDS padding limits residency to 24 waves/CU (the real kernel's 73 VGPRs)
//   x4          the same at 4x the actions (a tail effect shrinks with the launch size)
//   hipcc -O3 --offload-arch=gfx950 -o scripts/probe_store_split scripts/probe_store_split.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int64_t N = 15992832;  // cfg2 actions rounded up to 1024
constexpr int C = 515;           // bool columns of the default k=3 VAEP

__global__ __launch_bounds__(256) void fill16(u32x4* p, int64_t n16) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
    __builtin_nontemporal_store(u32x4{(uint32_t)i, 1u, 2u, 3u}, p + i);
}

template <int S, int LDS_BYTES>
__global__ __launch_bounds__(256) void split16(uint8_t* out, int64_t tiles) {
  __shared__ uint32_t pad[LDS_BYTES / 4 > 256 ? LDS_BYTES / 4 : 256];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t g = (int64_t)blockIdx.x * 4 + wv;
  const int64_t t = g / S;
  const int s = (int)(g % S);
  uint32_t seed = (uint32_t)g;
  if (LDS_BYTES > 0) {
    pad[threadIdx.x] = lane;
    __syncthreads();
    seed ^= pad[(threadIdx.x + 1) & 255];
  }
  if (t >= tiles) return;
  const int c0 = s * C / S, c1 = (s + 1) * C / S;
  uint8_t* base = out + t * (int64_t)C * 1024 + lane * 16;
  for (int c = c0; c < c1; ++c)
    __builtin_nontemporal_store(u32x4{seed + c, seed ^ c, (uint32_t)c, seed},
                                (u32x4*)(base + (int64_t)c * 1024));
}

template <typename F>
static int timeit(const char* name, F launch, double bytes) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  launch();
  launch();
  CHECK(hipDeviceSynchronize());
  const int reps = 10;
  CHECK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) launch();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  printf("{\"pattern\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f}\n", name, ms, bytes / (ms * 1e-3) / 1e12);
  fflush(stdout);
  CHECK(hipGetLastError());
  return 0;
}

template <int S, int L>
static int run(const char* name, uint8_t* out, int64_t n) {
  const int64_t tiles = n / 1024;
  const int blocks = (int)((tiles * S + 3) / 4);
  return timeit(name, [&] { split16<S, L><<<blocks, 256>>>(out, tiles); }, (double)n * C);
}

int main() {
  const int64_t n4 = 4 * N;
  uint8_t* out = nullptr;
  CHECK(hipMalloc(&out, (size_t)n4 * C));
  int rc = 0;
  rc |= timeit("fill16 nt 16384x256", [&] { fill16<<<16384, 256>>>((u32x4*)out, N * C / 16); },
               (double)N * C);
  rc |= run<1, 0>("tile16", out, N);
  rc |= run<1, 26000>("tile16_occ24", out, N);
  rc |= run<2, 0>("split2", out, N);
  rc |= run<2, 26000>("split2_occ24", out, N);
  rc |= run<3, 0>("split3", out, N);
  rc |= run<3, 26000>("split3_occ24", out, N);
  rc |= run<4, 26000>("split4_occ24", out, N);
  rc |= run<8, 26000>("split8_occ24", out, N);
  rc |= run<1, 26000>("tile16_occ24 x4", out, n4);
  rc |= run<3, 26000>("split3_occ24 x4", out, n4);
  CHECK(hipFree(out));
  return rc;
}
