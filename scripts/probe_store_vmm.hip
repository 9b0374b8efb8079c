// Placement probe: does the way the 8.2-GB bool image is allocated change the store rate of
// the bool kernel's pattern?  (profiles/r01d_placement.md: with hipMalloc the XCD-ordered
// column-group pattern runs 5.8 - 7.1 TB/s depending on the allocation, the 1-store-per-thread
// fill a constant ~7.0.)  Modes, each allocation kept alive so every trial lands elsewhere:
//   malloc      hipMalloc
//   vmm         hipMemCreate of ONE physical handle of the whole size, mapped with hipMemMap
//   vmm_chunks  the same address range backed by 256-MiB physical handles
//   hipcc -O3 --offload-arch=gfx950 -o scripts/probe_store_vmm scripts/probe_store_vmm.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int64_t N = 15992832;
constexpr int C = 515;
constexpr int G = 26;

__global__ __launch_bounds__(256) void fill1(u32x4* p, int64_t n16) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n16) p[i] = u32x4{(uint32_t)i, 1u, 2u, 3u};
}

// the bool kernel's store pattern: a wave writes G consecutive 1-KiB column runs of one
// 1024-row tile, each XCD (blockIdx % 8) sweeping its own contiguous eighth, nt stores
// V: 0 = eighths; 1 = eighths, odd XCDs sweep theirs backwards; 2 = eighths, XCD x starts at
// x/8 of its eighth (wrapping), so the 8 fronts are never a fixed distance apart; 3 = sixteenths
// (two fronts per XCD)
template <int V>
__global__ __launch_bounds__(256) void colgroup_xcd(uint8_t* out, int64_t tiles) {
  constexpr int NG = (C + G - 1) / G;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t nb = gridDim.x, per = nb / 8;  // nb is a multiple of 16
  const int64_t x = blockIdx.x % 8, i = blockIdx.x / 8;
  int64_t b;
  if (V == 0) b = x * per + i;
  else if (V == 1) b = x * per + ((x & 1) ? per - 1 - i : i);
  else if (V == 2) b = x * per + (i + x * (per / 8)) % per;
  else b = (int64_t)(blockIdx.x % 16) * (nb / 16) + blockIdx.x / 16;
  const int64_t w = b * 4 + wv;
  const int64_t t = w / NG;
  const int g = (int)(w % NG);
  if (t >= tiles) return;
  uint8_t* base = out + t * (int64_t)C * 1024 + lane * 16;
  const int c1 = (g + 1) * G < C ? (g + 1) * G : C;
  for (int c = g * G; c < c1; ++c)
    __builtin_nontemporal_store(u32x4{(uint32_t)t + c, 1u, 2u, (uint32_t)c}, (u32x4*)(base + (int64_t)c * 1024));
}

template <typename L>
static int timeit(const char* mode, int trial, const char* name, L launch, double bytes) {
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
  printf("{\"mode\": \"%s\", \"trial\": %d, \"pattern\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f}\n", mode, trial, name,
         ms, bytes / (ms * 1e-3) / 1e12);
  fflush(stdout);
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  CHECK(hipGetLastError());
  return 0;
}

static int vmm_alloc(size_t bytes, size_t chunk, uint8_t** out) {
  hipMemAllocationProp prop;
  memset(&prop, 0, sizeof(prop));
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  size_t gran = 0;
  CHECK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
  const size_t total = (bytes + gran - 1) / gran * gran;
  if (chunk == 0 || chunk > total) chunk = total;
  chunk = (chunk + gran - 1) / gran * gran;
  const size_t mapped = (total + chunk - 1) / chunk * chunk;
  void* va = nullptr;
  CHECK(hipMemAddressReserve(&va, mapped, 0, nullptr, 0));
  for (size_t off = 0; off < mapped; off += chunk) {
    hipMemGenericAllocationHandle_t h;
    CHECK(hipMemCreate(&h, chunk, &prop, 0));
    CHECK(hipMemMap((char*)va + off, chunk, 0, h, 0));
  }
  hipMemAccessDesc desc;
  memset(&desc, 0, sizeof(desc));
  desc.location = prop.location;
  desc.flags = hipMemAccessFlagsProtReadWrite;
  CHECK(hipMemSetAccess(va, mapped, &desc, 1));
  *out = (uint8_t*)va;
  printf("{\"vmm_granularity\": %zu, \"chunk\": %zu, \"mapped\": %zu}\n", gran, chunk, mapped);
  return 0;
}

int main(int argc, char** argv) {
  const double bytes = (double)N * C;
  const int64_t n16 = N * C / 16, tiles = N / 1024;
  const int trials = argc > 1 ? atoi(argv[1]) : 3;
  const char* modes[] = {"malloc", "vmm", "vmm_chunks"};
  const int n_modes = argc > 2 ? atoi(argv[2]) : 3;
  int rc = 0;
  for (int t = 0; t < trials; ++t) {
    for (int m = 0; m < n_modes; ++m) {
      uint8_t* out = nullptr;
      if (m == 0)
        CHECK(hipMalloc(&out, (size_t)bytes));
      else if (vmm_alloc((size_t)bytes, m == 1 ? 0 : ((size_t)256 << 20), &out))
        return 1;
      const unsigned nb = (unsigned)(((tiles * ((C + G - 1) / G) + 3) / 4 + 15) / 16 * 16);
      rc |= timeit(modes[m], t, "fill", [&] { fill1<<<(unsigned)((n16 + 255) / 256), 256>>>((u32x4*)out, n16); }, bytes);
      rc |= timeit(modes[m], t, "col26_xcd_nt", [&] { colgroup_xcd<0><<<nb, 256>>>(out, tiles); }, bytes);
      rc |= timeit(modes[m], t, "xcd_oddrev", [&] { colgroup_xcd<1><<<nb, 256>>>(out, tiles); }, bytes);
      rc |= timeit(modes[m], t, "xcd_phase", [&] { colgroup_xcd<2><<<nb, 256>>>(out, tiles); }, bytes);
      rc |= timeit(modes[m], t, "xcd_16ths", [&] { colgroup_xcd<3><<<nb, 256>>>(out, tiles); }, bytes);
      if (rc) return rc;
      // allocations stay alive (3 modes x trials x 8.2 GB, well inside 288 GB)
    }
  }
  return rc;
}
