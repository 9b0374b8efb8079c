// Store-run-length probe for the bool block image ([tiles][515][1024] bytes, nt stores).
// A wave writes G consecutive 1-KiB column chunks of one tile (one 16-B store per lane per
// chunk); waves enumerate (tile, group) tile-major, so G = 1 in linear order IS the
// one-store-per-thread fill of this image.  The question: is the allocation-dependent
// spread of the bool kernel (G ~ 31, XCD-contiguous order) a property of the run length a
// wave writes (the active window = waves in flight x G KiB) or of the order?
//   hipcc -O3 --offload-arch=gfx950 -o scripts/probe_store_runlen scripts/probe_store_runlen.hip
//   ./scripts/probe_store_runlen ALLOCATIONS
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int64_t N = 15992832;
constexpr int C = 515;

__device__ __forceinline__ int64_t remap(int64_t b, int64_t nb, int xcd) {
  if (!xcd) return b;
  return (b % 8) * (nb / 8) + b / 8;
}

// wave -> (tile, group of G columns); WPB waves per block
template <int WPB>
__global__ __launch_bounds__(64 * WPB) void runs(uint8_t* out, int64_t tiles, int G, int xcd) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ng = (C + G - 1) / G;
  const int64_t w = remap(blockIdx.x, gridDim.x, xcd) * WPB + wv;
  const int64_t t = w / ng;
  const int g = (int)(w % ng);
  if (t >= tiles) return;
  uint8_t* base = out + t * (int64_t)C * 1024 + lane * 16;
  const int c1 = (g + 1) * G < C ? (g + 1) * G : C;
  for (int c = g * G; c < c1; ++c) {
    const u32x4 v = {(uint32_t)t + c, 1u, 2u, (uint32_t)c};
    __builtin_nontemporal_store(v, (u32x4*)(base + (int64_t)c * 1024));
  }
}

// Persistent form: W waves in flight (grid = 256 CUs x B blocks), wave w writes the 1-KiB
// chunks w, w + W, w + 2W, ... of the image in order (a moving front W KiB wide).
__global__ __launch_bounds__(256) void front(uint8_t* out, int64_t chunks) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t W = (int64_t)gridDim.x * 4;
  for (int64_t ch = (int64_t)blockIdx.x * 4 + wv; ch < chunks; ch += W) {
    const u32x4 v = {(uint32_t)ch, 1u, 2u, 3u};
    __builtin_nontemporal_store(v, (u32x4*)(out + ch * 1024 + lane * 16));
  }
}

// G = 1 with a per-wave prologue: `deps` dependent 16-B loads from a small (L2-resident)
// code image before the store, the latency the real kernel's code lookup would add
template <int WPB>
__global__ __launch_bounds__(64 * WPB) void runs_lat(uint8_t* out, const u32x4* codes,
                                                     int64_t tiles, int deps, int xcd) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t w = remap(blockIdx.x, gridDim.x, xcd) * WPB + wv;
  const int64_t t = w / C;
  const int c = (int)(w % C);
  if (t >= tiles) return;
  u32x4 v = {(uint32_t)t + c, 1u, 2u, (uint32_t)c};
  int idx = (int)((t * 16 + (c & 15)) & 4095) * 64 + lane;
  for (int d = 0; d < deps; ++d) {
    const u32x4 x = codes[idx];
    v ^= x;
    idx = (idx + (int)(x.x & 1u) * 64 + 64 * 17) & (4096 * 64 - 1);
  }
  __builtin_nontemporal_store(v, (u32x4*)(out + t * (int64_t)C * 1024 + (int64_t)c * 1024 + lane * 16));
}

template <typename L>
static int timeit(const char* name, int G, int xcd, L launch, double bytes) {
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
  printf("{\"pattern\": \"%s\", \"G\": %d, \"xcd\": %d, \"ms\": %.4f, \"TBps\": %.3f}\n", name, G,
         xcd, ms, bytes / (ms * 1e-3) / 1e12);
  fflush(stdout);
  CHECK(hipGetLastError());
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return 0;
}

// allocation flavours: 0 hipMalloc, 1 hipExtMallocWithFlags(hipDeviceMallocContiguous),
// 2 one VMM physical handle of the whole size mapped at a reserved range
static int alloc(uint8_t** out, size_t bytes, int how) {
  if (how == 0) return hipMalloc(out, bytes) != hipSuccess;
  if (how == 1) return hipExtMallocWithFlags((void**)out, bytes, hipDeviceMallocContiguous) != hipSuccess;
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  size_t gran = 0;
  CHECK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
  const size_t sz = (bytes + gran - 1) / gran * gran;
  hipMemGenericAllocationHandle_t h;
  CHECK(hipMemCreate(&h, sz, &prop, 0));
  void* va = nullptr;
  CHECK(hipMemAddressReserve(&va, sz, 0, nullptr, 0));
  CHECK(hipMemMap(va, sz, 0, h, 0));
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  CHECK(hipMemSetAccess(va, sz, &acc, 1));
  printf("{\"vmm_granularity\": %zu}\n", gran);
  *out = (uint8_t*)va;
  return 0;
}

int main(int argc, char** argv) {
  const double bytes = (double)N * C;
  const int64_t tiles = N / 1024, chunks = tiles * C;
  const int trials = argc > 1 ? atoi(argv[1]) : 1;
  const int how = argc > 2 ? atoi(argv[2]) : 0;
  const bool quick = argc > 3 && atoi(argv[3]) != 0;
  int rc = 0;
  const int Gs[] = {1, 2, 4, 31};
  u32x4* codes = nullptr;
  CHECK(hipMalloc(&codes, 4096 * 64 * sizeof(u32x4)));
  CHECK(hipMemset(codes, 0, 4096 * 64 * sizeof(u32x4)));
  for (int t = 0; t < trials; ++t) {
    uint8_t* out = nullptr;  // kept alive: every trial lands somewhere else
    if (alloc(&out, (size_t)bytes, how)) { fprintf(stderr, "allocation %d failed\n", how); return 1; }
    printf("{\"trial\": %d, \"ptr_GB\": %.2f}\n", t, (double)(uintptr_t)out / (1 << 30));
    if (quick) {
      for (int G : {1, 31}) {
        const int64_t ng = (C + G - 1) / G;
        const unsigned nb = (unsigned)(((tiles * ng + 3) / 4 + 7) / 8 * 8);
        rc |= timeit("runs4", G, 1, [&] { runs<4><<<nb, 256>>>(out, tiles, G, 1); }, bytes);
      }
      continue;
    }
    for (int G : Gs) {
      const int64_t ng = (C + G - 1) / G;
      const unsigned blocks = (unsigned)((tiles * ng + 3) / 4);
      const unsigned nb = (blocks + 7) / 8 * 8;
      for (int xcd = 0; xcd < 2; ++xcd)
        rc |= timeit("runs4", G, xcd, [&] { runs<4><<<nb, 256>>>(out, tiles, G, xcd); }, bytes);
    }
    for (int xcd = 0; xcd < 2; ++xcd) {
      const unsigned b1 = (unsigned)((chunks + 7) / 8 * 8), b16 = (unsigned)(((chunks + 15) / 16 + 7) / 8 * 8);
      const unsigned b1_2 = (unsigned)(((chunks + 1) / 2 + 7) / 8 * 8);
      rc |= timeit("runs1", 1, xcd, [&] { runs<1><<<b1, 64>>>(out, tiles, 1, xcd); }, bytes);
      rc |= timeit("runs1", 2, xcd, [&] { runs<1><<<b1_2, 64>>>(out, tiles, 2, xcd); }, bytes);
      rc |= timeit("runs16", 1, xcd, [&] { runs<16><<<b16, 1024>>>(out, tiles, 1, xcd); }, bytes);
      const unsigned b4 = (unsigned)(((chunks + 3) / 4 + 7) / 8 * 8);
      for (int deps : {1, 2, 4})
        rc |= timeit(deps == 1 ? "lat1" : deps == 2 ? "lat2" : "lat4", 1, xcd,
                     [&] { runs_lat<4><<<b4, 256>>>(out, codes, tiles, deps, xcd); }, bytes);
    }
  }
  return rc;
}
