// Store-flavour probe: which cache policy on a 16-B-per-lane vector store lets MI355X absorb
// a pure write stream fastest?  torch's fill_ has been measured at ~6.85 TB/s on these
// boxes while a grid-stride fill with `nt` stores reached ~5.6 TB/s, and the bool feature
// block (515 B of output per action) is store-bound.  Patterns (8.2 GB each):
//   fill   grid-stride 16-B stores, G blocks x 256 threads
//   tile   the bool block image: one wave per 1024-row tile, 515 column runs of 1 KiB
// flavours: plain (write-back in L2), nt, sc1 (write-through), sc0 sc1, nt sc1
//   hipcc -O3 --offload-arch=gfx950 -o scripts/probe_store_flavours scripts/probe_store_flavours.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int64_t N = 15992832;  // cfg2 actions rounded up to 1024
constexpr int C = 515;

enum { PLAIN = 0, NT = 1, SC1 = 2, SC01 = 3, NTSC1 = 4, CPP = 5, CPPNT = 6 };

template <int F>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
  if (F == PLAIN) asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(p), "v"(v) : "memory");
  if (F == NT) asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
  if (F == SC1) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  if (F == SC01) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
  if (F == NTSC1) asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
  if (F == CPP) *p = v;
  if (F == CPPNT) __builtin_nontemporal_store(v, p);
}

template <int F>
__global__ __launch_bounds__(256) void fill(u32x4* p, int64_t n16) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
    st<F>(p + i, u32x4{(uint32_t)i, 1u, 2u, 3u});
}

template <int F>
__global__ __launch_bounds__(256) void tile(uint8_t* out, int64_t tiles) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t t = (int64_t)blockIdx.x * 4 + wv;
  if (t >= tiles) return;
  uint8_t* base = out + t * (int64_t)C * 1024 + lane * 16;
  for (int c = 0; c < C; ++c)
    st<F>((u32x4*)(base + (int64_t)c * 1024), u32x4{(uint32_t)t + c, 1u, 2u, (uint32_t)c});
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

int main() {
  const double bytes = (double)N * C;
  const int64_t n16 = N * C / 16, tiles = N / 1024;
  uint8_t* out = nullptr;
  CHECK(hipMalloc(&out, (size_t)bytes));
  u32x4* p = (u32x4*)out;
  const int tb = (int)((tiles + 3) / 4);
  int rc = 0;
  rc |= timeit("fill cpp 16384", [&] { fill<CPP><<<16384, 256>>>(p, n16); }, bytes);
  rc |= timeit("fill cpp-nt 16384", [&] { fill<CPPNT><<<16384, 256>>>(p, n16); }, bytes);
  rc |= timeit("fill plain 16384", [&] { fill<PLAIN><<<16384, 256>>>(p, n16); }, bytes);
  rc |= timeit("fill nt 16384", [&] { fill<NT><<<16384, 256>>>(p, n16); }, bytes);
  rc |= timeit("fill sc1 16384", [&] { fill<SC1><<<16384, 256>>>(p, n16); }, bytes);
  rc |= timeit("fill sc0sc1 16384", [&] { fill<SC01><<<16384, 256>>>(p, n16); }, bytes);
  rc |= timeit("fill ntsc1 16384", [&] { fill<NTSC1><<<16384, 256>>>(p, n16); }, bytes);
  rc |= timeit("fill plain 2048", [&] { fill<PLAIN><<<2048, 256>>>(p, n16); }, bytes);
  rc |= timeit("fill plain 65536", [&] { fill<PLAIN><<<65536, 256>>>(p, n16); }, bytes);
  rc |= timeit("fill plain 1 pass", [&] { fill<PLAIN><<<(unsigned)((n16 + 255) / 256), 256>>>(p, n16); }, bytes);
  rc |= timeit("tile cpp", [&] { tile<CPP><<<tb, 256>>>(out, tiles); }, bytes);
  rc |= timeit("tile cpp-nt", [&] { tile<CPPNT><<<tb, 256>>>(out, tiles); }, bytes);
  rc |= timeit("tile plain", [&] { tile<PLAIN><<<tb, 256>>>(out, tiles); }, bytes);
  rc |= timeit("tile nt", [&] { tile<NT><<<tb, 256>>>(out, tiles); }, bytes);
  rc |= timeit("tile sc1", [&] { tile<SC1><<<tb, 256>>>(out, tiles); }, bytes);
  rc |= timeit("tile sc0sc1", [&] { tile<SC01><<<tb, 256>>>(out, tiles); }, bytes);
  rc |= timeit("tile ntsc1", [&] { tile<NTSC1><<<tb, 256>>>(out, tiles); }, bytes);
  CHECK(hipFree(out));
  return rc;
}
