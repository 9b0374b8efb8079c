// Store-locality probe: the 1-store-per-thread fill (every resident wave writing inside one
// compact, advancing window) ran at ~7.0 TB/s where the bool block's tile pattern (each wave
// sweeping its own 515-KiB tile, ~6000 tiles open at once) ran at ~6.1 TB/s.  This probe
// writes the same tiled [tiles][515][1024] image with short waves: wave w writes G
// consecutive 1-KiB column runs of one tile, and waves are ordered so consecutive waves
// write consecutive addresses (the image is swept front to back like a fill).
//   colG      linear order (tile = w / groups, group = w % groups)
//   colG_xcd  each XCD (blockIdx % 8) sweeps its own contiguous eighth of the image
//   hipcc -O3 --offload-arch=gfx950 -o scripts/probe_store_colgroup scripts/probe_store_colgroup.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int64_t N = 15992832;
constexpr int C = 515;

__global__ __launch_bounds__(256) void fill1(u32x4* p, int64_t n16) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n16) p[i] = u32x4{(uint32_t)i, 1u, 2u, 3u};
}

template <int G, bool XCD, bool NT = false>
__global__ __launch_bounds__(256) void colgroup(uint8_t* out, int64_t tiles) {
  constexpr int NG = (C + G - 1) / G;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int64_t b = blockIdx.x;
  if (XCD) {  // block b runs on XCD b % 8: give each XCD a contiguous range of blocks
    const int64_t nb = gridDim.x, per = (nb + 7) / 8;
    b = (b % 8) * per + b / 8;
  }
  const int64_t w = b * 4 + wv;
  const int64_t t = w / NG;
  const int g = (int)(w % NG);
  if (t >= tiles) return;
  uint8_t* base = out + t * (int64_t)C * 1024 + lane * 16;
  const int c1 = (g + 1) * G < C ? (g + 1) * G : C;
  for (int c = g * G; c < c1; ++c) {
    const u32x4 v = {(uint32_t)t + c, 1u, 2u, (uint32_t)c};
    if (NT)
      __builtin_nontemporal_store(v, (u32x4*)(base + (int64_t)c * 1024));
    else
      *(u32x4*)(base + (int64_t)c * 1024) = v;
  }
}

template <typename L>
static int timeit(const char* name, L launch, double bytes) {
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

template <int G, bool X, bool NT = false>
static int run(const char* name, uint8_t* out, int64_t tiles) {
  constexpr int NG = (C + G - 1) / G;
  const unsigned blocks = (unsigned)((tiles * NG + 3) / 4);
  const unsigned nb = X ? (blocks + 7) / 8 * 8 : blocks;
  return timeit(name, [&] { colgroup<G, X, NT><<<nb, 256>>>(out, tiles); }, (double)tiles * 1024 * C);
}

int main(int argc, char** argv) {
  const double bytes = (double)N * C;
  const int64_t n16 = N * C / 16, tiles = N / 1024;
  const int trials = argc > 1 ? atoi(argv[1]) : 1;
  // argv[2] = 1: keep every allocation alive (each trial lands further into HBM)
  const bool keep_all = argc > 2 && atoi(argv[2]) != 0;
  uint8_t* keep[3] = {nullptr, nullptr, nullptr};
  int rc = 0;
  for (int t = 0; t < trials; ++t) {
    uint8_t* out = nullptr;
    CHECK(hipMalloc(&out, (size_t)bytes));
    printf("{\"trial\": %d, \"ptr_GB\": %.2f}\n", t, (double)(uintptr_t)out / (1 << 30));
    rc |= timeit("fill 1 store/thread", [&] { fill1<<<(unsigned)((n16 + 255) / 256), 256>>>((u32x4*)out, n16); }, bytes);
    rc |= run<515, false>("col515 (= tile)", out, tiles);
    rc |= run<16, false>("col16", out, tiles);
    rc |= run<32, false>("col32", out, tiles);
    rc |= run<16, true>("col16_xcd", out, tiles);
    rc |= run<32, true>("col32_xcd", out, tiles);
    rc |= run<26, true, true>("col26_xcd_nt", out, tiles);
    rc |= run<26, true, false>("col26_xcd", out, tiles);
    rc |= run<515, true>("col515_xcd", out, tiles);
    if (!keep_all) {
      if (keep[t % 3]) CHECK(hipFree(keep[t % 3]));
      keep[t % 3] = out;
    }
  }
  return rc;
}
