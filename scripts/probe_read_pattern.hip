// Read-pattern probe for the xT iteration: how fast can the chip stream the C x C int32
// count matrix (C = 7140, 204 MB) in the access order the iteration kernel uses, with no
// compute?  hipcc -O3 --offload-arch=gfx950 -o scripts/probe_read_pattern scripts/probe_read_pattern.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int C = 7140;
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));

// (a) linear grid-stride 16-B loads
__global__ __launch_bounds__(256) void linear16(const i32x4* p, int64_t n16, int* out) {
  int acc = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    const i32x4 v = p[i];
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x7fffffff) out[0] = acc;
}

// (b) the iteration kernel's order: 16 rows per workgroup, wave w reads rows 4w..4w+3,
// lane reads column 128k + 64i + lane (dword), chunks k sequential, DEPTH chunks unrolled
template <int CH>
__global__ __launch_bounds__(256) void rows16(const int32_t* t, int* out) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r0 = blockIdx.x * 16;
  int acc = 0;
  const int32_t* rp[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) rp[q] = t + (int64_t)min(r0 + 4 * wv + q, C - 1) * C;
  for (int c0 = 0; c0 < C; c0 += CH) {
#pragma unroll
    for (int i = 0; i < CH / 64; ++i) {
      const int c = min(c0 + 64 * i + lane, C - 1);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc += rp[q][c];
    }
  }
  if (acc == 0x7fffffff) out[0] = acc;
}

// (c) blocked [C/16][C][16] layout: each workgroup streams its own contiguous 457 KB block
__global__ __launch_bounds__(256) void blocked(const i32x4* t, int* out) {
  const int64_t base = (int64_t)blockIdx.x * C * 16 / 4;  // in i32x4 units
  int acc = 0;
  for (int e = threadIdx.x; e < C * 16 / 4; e += 256) {
    const i32x4 v = t[base + e];
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x7fffffff) out[0] = acc;
}

// (d) rows16 but each wave streams ONE row at a time (4 rows in sequence), 256-B dword runs
__global__ __launch_bounds__(256) void rowseq(const int32_t* t, int* out) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r0 = blockIdx.x * 16;
  int acc = 0;
  for (int q = 0; q < 4; ++q) {
    const int32_t* rp = t + (int64_t)min(r0 + 4 * wv + q, C - 1) * C;
    for (int c = lane; c < C; c += 64) acc += rp[c];
  }
  if (acc == 0x7fffffff) out[0] = acc;
}

template <typename F>
static int timeit(const char* name, F launch, double bytes) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  launch(); launch();
  CHECK(hipDeviceSynchronize());
  const int reps = 20;
  CHECK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) launch();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  printf("{\"pattern\": \"%s\", \"us\": %.1f, \"TBps\": %.3f}\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
  fflush(stdout);
  return 0;
}

int main() {
  const int64_t n = (int64_t)C * C + 16 * C;  // room for the padded blocked layout
  int32_t* t = nullptr;
  int* out = nullptr;
  CHECK(hipMalloc(&t, n * 4));
  CHECK(hipMalloc(&out, 4));
  CHECK(hipMemset(t, 1, n * 4));
  const double bytes = (double)C * C * 4;
  const int wgs = (C + 15) / 16;
  timeit("linear16 2048x256", [&] { linear16<<<2048, 256>>>((const i32x4*)t, (int64_t)C * C / 4, out); }, bytes);
  timeit("linear16 8192x256", [&] { linear16<<<8192, 256>>>((const i32x4*)t, (int64_t)C * C / 4, out); }, bytes);
  timeit("rows16 CH128 (iteration order)", [&] { rows16<128><<<wgs, 256>>>(t, out); }, bytes);
  timeit("rows16 CH512", [&] { rows16<512><<<wgs, 256>>>(t, out); }, bytes);
  timeit("blocked [C/16][C][16]", [&] { blocked<<<wgs, 256>>>((const i32x4*)t, out); }, bytes);
  timeit("rowseq (wave streams one row at a time)", [&] { rowseq<<<wgs, 256>>>(t, out); }, bytes);
  CHECK(hipFree(t));
  return 0;
}
