// Store-pattern probe: how fast can MI355X absorb the bool block's write pattern, with no
// feature compute at all?  Separates "the layout / wave mapping caps us" from "the kernel's
// structure costs us".  Build + run (GPU box):
//   hipcc -O3 --offload-arch=gfx950 -o gpurun_out/probe scripts/probe_store_pattern.hip
//   gpurun_out/probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int64_t N = 15992832;  // cfg2 actions rounded up to 1024
constexpr int C = 515;           // bool columns of the default k=3 VAEP

// P0: grid-stride 16-B stores over the whole buffer (a fill).
__global__ __launch_bounds__(256) void fill16(u32x4* p, int64_t n16) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
    p[i] = u32x4{(uint32_t)i, 1u, 2u, 3u};
}

// P1: the bool kernel's pattern: wave w owns rows [1024w, 1024w+1024) = one tile [C][1024];
// lane l stores 16 B at column c, offset c*1024 + 16l.  LDS_PAD limits waves per CU.
template <int LDS_BYTES, bool NT>
__global__ __launch_bounds__(256) void tile16(uint8_t* out, int64_t n) {
  __shared__ uint32_t pad[LDS_BYTES / 4 > 0 ? LDS_BYTES / 4 : 1];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t w = (int64_t)blockIdx.x * 4 + wv;
  if (w * 1024 >= n) return;
  if (LDS_BYTES > 0) { pad[threadIdx.x] = lane; __syncthreads(); }
  uint8_t* base = out + w * (int64_t)C * 1024 + lane * 16;
  uint32_t seed = (uint32_t)w ^ (LDS_BYTES > 0 ? pad[(threadIdx.x + 1) & 255] : 0u);
  for (int c = 0; c < C; ++c) {
    u32x4 v = {seed + c, seed ^ c, (uint32_t)c, seed};
    if (NT) __builtin_nontemporal_store(v, (u32x4*)(base + (int64_t)c * 1024));
    else *(u32x4*)(base + (int64_t)c * 1024) = v;
  }
}

// P2: 512-row tiles, lane stores 8 B (two waves' worth of tiles per 1024 rows).
__global__ __launch_bounds__(256) void tile8(uint8_t* out, int64_t n) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t w = (int64_t)blockIdx.x * 4 + wv;
  if (w * 512 >= n) return;
  uint8_t* base = out + w * (int64_t)C * 512 + lane * 8;
  for (int c = 0; c < C; ++c) *(u32x2*)(base + (int64_t)c * 512) = u32x2{(uint32_t)w + c, (uint32_t)c};
}

// P3: plain column-major [C][N]: wave w writes rows [1024w, +1024) of every column.
__global__ __launch_bounds__(256) void colmajor16(uint8_t* out, int64_t n) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t w = (int64_t)blockIdx.x * 4 + wv;
  if (w * 1024 >= n) return;
  uint8_t* base = out + w * 1024 + lane * 16;
  for (int c = 0; c < C; ++c) *(u32x4*)(base + (int64_t)c * n) = u32x4{(uint32_t)w + c, 1u, 2u, (uint32_t)c};
}

// P4: tile pattern, but each wave writes its tile in 4 interleaved column groups -- two
// waves of a workgroup share one tile (2048-B per column per WG pair).
// P5: persistent: grid = 256 CUs x 8 WGs, waves loop over tiles w += total waves.
__global__ __launch_bounds__(256) void tile16_persistent(uint8_t* out, int64_t n) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t nt = n / 1024;
  for (int64_t w = (int64_t)blockIdx.x * 4 + wv; w < nt; w += (int64_t)gridDim.x * 4) {
    uint8_t* base = out + w * (int64_t)C * 1024 + lane * 16;
    for (int c = 0; c < C; ++c) *(u32x4*)(base + (int64_t)c * 1024) = u32x4{(uint32_t)w + c, 1u, 2u, (uint32_t)c};
  }
}

template <typename F>
static int timeit(const char* name, F launch, double bytes) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  launch(); launch();
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
  uint8_t* out = nullptr;
  CHECK(hipMalloc(&out, (size_t)bytes));
  const int64_t waves = N / 1024;
  const int blocks = (int)((waves + 3) / 4);
  int rc = 0;
  rc |= timeit("fill16 grid-stride 2048x256", [&] { fill16<<<2048, 256>>>((u32x4*)out, (int64_t)bytes / 16); }, bytes);
  rc |= timeit("fill16 grid-stride 16384x256", [&] { fill16<<<16384, 256>>>((u32x4*)out, (int64_t)bytes / 16); }, bytes);
  rc |= timeit("tile16 (bool pattern)", [&] { tile16<0, false><<<blocks, 256>>>(out, N); }, bytes);
  rc |= timeit("tile16 nt", [&] { tile16<0, true><<<blocks, 256>>>(out, N); }, bytes);
  rc |= timeit("tile16 lds16K (<=40 waves/CU)", [&] { tile16<16384, false><<<blocks, 256>>>(out, N); }, bytes);
  rc |= timeit("tile16 lds32K (<=20 waves/CU)", [&] { tile16<32768, false><<<blocks, 256>>>(out, N); }, bytes);
  rc |= timeit("tile16 lds54K (<=8..12 waves/CU)", [&] { tile16<54000, false><<<blocks, 256>>>(out, N); }, bytes);
  rc |= timeit("tile8 (512-row tiles)", [&] { tile8<<<(int)((N / 512 + 3) / 4), 256>>>(out, N); }, bytes);
  rc |= timeit("colmajor16", [&] { colmajor16<<<blocks, 256>>>(out, N); }, bytes);
  rc |= timeit("tile16 persistent 256x8", [&] { tile16_persistent<<<2048, 256>>>(out, N); }, bytes);
  rc |= timeit("tile16 persistent 256x4", [&] { tile16_persistent<<<1024, 256>>>(out, N); }, bytes);
  rc |= timeit("tile16 persistent 256x16", [&] { tile16_persistent<<<4096, 256>>>(out, N); }, bytes);
  CHECK(hipFree(out));
  return rc;
}
