// Store-order probe for the bool block image ([tiles][515][1024] bytes, 31-column groups per
// wave, nt stores: the bool_colgroup_kernel's shape without its compute). The kernel's
// XCD-contiguous order (each XCD sweeps its own eighth of the image, 8 write fronts ~1 GB
// apart) runs 5.8 - 7.0 TB/s depending on the allocation, while a fill (one front) holds
// ~7.0. Here each XCD instead takes runs of S consecutive blocks, the runs dealt round-robin
// over the 8 XCDs, so the 8 fronts stay within 8*S blocks of each other:
//   S = 0   XCD-contiguous eighths (the kernel today)
//   S = -1  linear block order (no remap)
//   hipcc -O3 --offload-arch=gfx950 -o scripts/probe_store_xcdgroups scripts/probe_store_xcdgroups.hip
//   ./scripts/probe_store_xcdgroups TRIALS [KEEP_ALL]
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int64_t N = 15992832;
constexpr int C = 515;
constexpr int G = 31;
constexpr int NG = (C + G - 1) / G;

__global__ __launch_bounds__(256) void fill1(u32x4* p, int64_t n16) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n16) p[i] = u32x4{(uint32_t)i, 1u, 2u, 3u};
}

__device__ __forceinline__ int64_t remap(int64_t b, int64_t nb, int S) {
  if (S < 0) return b;
  const int64_t x = b % 8, k = b / 8;
  if (S == 0) return x * ((nb + 7) / 8) + k;
  return ((k / S) * 8 + x) * S + (k % S);
}

__global__ __launch_bounds__(256) void colgroup(uint8_t* out, int64_t tiles, int S) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t b = remap(blockIdx.x, gridDim.x, S);
  const int64_t w = b * 4 + wv;
  const int64_t t = w / NG;
  const int g = (int)(w % NG);
  if (t >= tiles) return;
  uint8_t* base = out + t * (int64_t)C * 1024 + lane * 16;
  const int c1 = (g + 1) * G < C ? (g + 1) * G : C;
  for (int c = g * G; c < c1; ++c) {
    const u32x4 v = {(uint32_t)t + c, 1u, 2u, (uint32_t)c};
    __builtin_nontemporal_store(v, (u32x4*)(base + (int64_t)c * 1024));
  }
}

// Interleaved columns: a workgroup of WG waves owns WG consecutive column groups of one tile
// (WG * 31 columns, the tile's last group shorter) and wave v writes columns base + WG*c + v,
// so at each step the workgroup's stores form one WG-KiB contiguous run.
template <int WG>
__global__ __launch_bounds__(64 * WG) void colinter(uint8_t* out, int64_t tiles, int S) {
  constexpr int CPB = WG * G;                  // columns per workgroup
  constexpr int BPT = (C + CPB - 1) / CPB;     // workgroups per tile
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t b = remap(blockIdx.x, gridDim.x, S);
  const int64_t t = b / BPT;
  const int q = (int)(b % BPT);
  if (t >= tiles) return;
  uint8_t* base = out + t * (int64_t)C * 1024 + lane * 16;
  const int c0 = q * CPB;
  for (int c = c0 + wv; c < c0 + CPB && c < C; c += WG) {
    const u32x4 v = {(uint32_t)t + c, 1u, 2u, (uint32_t)c};
    __builtin_nontemporal_store(v, (u32x4*)(base + (int64_t)c * 1024));
  }
}

template <typename L>
static int timeit(const char* name, int S, L launch, double bytes) {
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
  printf("{\"pattern\": \"%s\", \"S\": %d, \"ms\": %.4f, \"TBps\": %.3f}\n", name, S, ms,
         bytes / (ms * 1e-3) / 1e12);
  fflush(stdout);
  CHECK(hipGetLastError());
  return 0;
}

int main(int argc, char** argv) {
  const double bytes = (double)N * C;
  const int64_t n16 = N * C / 16, tiles = N / 1024;
  const int trials = argc > 1 ? atoi(argv[1]) : 1;
  const bool keep_all = argc > 2 && atoi(argv[2]) != 0;
  uint8_t* prev = nullptr;
  int rc = 0;
  const int Ss[] = {0, -1};
  for (int t = 0; t < trials; ++t) {
    uint8_t* out = nullptr;
    CHECK(hipMalloc(&out, (size_t)bytes));
    printf("{\"trial\": %d, \"ptr_GB\": %.2f}\n", t, (double)(uintptr_t)out / (1 << 30));
    rc |= timeit("fill", 0, [&] { fill1<<<(unsigned)((n16 + 255) / 256), 256>>>((u32x4*)out, n16); }, bytes);
    const unsigned blocks = (unsigned)((tiles * NG + 3) / 4);
    const unsigned nb = (blocks + 7) / 8 * 8;
    for (int S : Ss) {
      // every S needs a grid that covers all blocks after the remap: round up to 8*S
      unsigned g = nb;
      if (S > 0) g = (unsigned)((nb + 8 * S - 1) / (8 * S) * (8 * S));
      rc |= timeit("col31_nt", S, [&] { colgroup<<<g, 256>>>(out, tiles, S); }, bytes);
    }
    {
      constexpr int BPT4 = (C + 4 * G - 1) / (4 * G), BPT16 = (C + 16 * G - 1) / (16 * G);
      const unsigned g4 = (unsigned)((tiles * BPT4 + 7) / 8 * 8), g16 = (unsigned)((tiles * BPT16 + 7) / 8 * 8);
      rc |= timeit("inter4_nt", 0, [&] { colinter<4><<<g4, 256>>>(out, tiles, 0); }, bytes);
      rc |= timeit("inter4_nt", -1, [&] { colinter<4><<<g4, 256>>>(out, tiles, -1); }, bytes);
      rc |= timeit("inter16_nt", 0, [&] { colinter<16><<<g16, 1024>>>(out, tiles, 0); }, bytes);
      rc |= timeit("inter16_nt", -1, [&] { colinter<16><<<g16, 1024>>>(out, tiles, -1); }, bytes);
    }
    if (!keep_all) {
      if (prev) CHECK(hipFree(prev));
      prev = out;
    }
  }
  return rc;
}
