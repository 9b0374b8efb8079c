// Runtime pieces of the C ABI: error reporting, version / build id, the per-device scratch
// arena (SURVEY.md §8(b) conventions) and the debug-build check collector.
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

#include "sa_internal.h"

#ifndef SA_BUILD_ID
#define SA_BUILD_ID "unversioned"
#endif

namespace sa {
static thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int check_hip(hipError_t e, const char* what) {
  if (e == hipSuccess) return SA_OK;
  return fail(SA_EHIP, "%s: %s", what, hipGetErrorString(e));
}

int check_launch(const char* what) { return check_hip(hipGetLastError(), what); }

// ------------------------------------------------------------------------ scratch arena
// Library-owned device scratch, cached per device.  A slot is handed to one call at a time;
// when the call releases it, an event recorded on the call's stream marks when the device is
// done with it, so the slot is reused immediately by the same stream (stream order) and by
// another stream once that event has completed.  Guarded by one mutex; freed by sa_shutdown().
namespace {
struct Slot {
  int dev;
  void* ptr;
  size_t bytes;
  hipStream_t last;
  hipEvent_t done;
  bool busy;
};
std::mutex g_arena_mu;
std::vector<Slot> g_slots;
}  // namespace

int scratch_acquire(size_t bytes, hipStream_t st, Scratch* out) {
  int dev = 0;
  int rc = check_hip(hipGetDevice(&dev), "hipGetDevice");
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_arena_mu);
  for (size_t i = 0; i < g_slots.size(); ++i) {
    Slot& s = g_slots[i];
    if (s.dev != dev || s.busy || s.bytes < bytes) continue;
    if (s.last != st && hipEventQuery(s.done) != hipSuccess) continue;  // still in use elsewhere
    s.busy = true;
    out->ptr = s.ptr;
    out->slot = (int)i;
    return SA_OK;
  }
  size_t cap = 64 * 1024;
  while (cap < bytes) cap *= 2;
  Slot s{dev, nullptr, cap, st, nullptr, true};
  if (hipMalloc(&s.ptr, cap) != hipSuccess) {
    (void)hipGetLastError();
    return fail(SA_ENOMEM, "scratch arena: hipMalloc of %zu bytes failed", cap);
  }
  if ((rc = check_hip(hipEventCreateWithFlags(&s.done, hipEventDisableTiming | hipEventDisableSystemFence), "hipEventCreate"))) {
    (void)hipFree(s.ptr);
    return rc;
  }
  g_slots.push_back(s);
  out->ptr = s.ptr;
  out->slot = (int)g_slots.size() - 1;
  return SA_OK;
}

void scratch_release(const Scratch& s, hipStream_t st) {
  if (s.slot < 0) return;
  std::lock_guard<std::mutex> lk(g_arena_mu);
  Slot& sl = g_slots[(size_t)s.slot];
  (void)hipEventRecord(sl.done, st);
  sl.last = st;
  sl.busy = false;
}

// ------------------------------------------------------------------------ device attributes
namespace {
constexpr int MAX_DEVICES = 64;
std::mutex g_attr_mu;
int g_cus[MAX_DEVICES], g_lds[MAX_DEVICES];
}  // namespace

int current_device() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return dev;
}

static int device_attr(int dev, int* cache, hipDeviceAttribute_t attr, int fallback) {
  if (dev < 0 || dev >= MAX_DEVICES) return fallback;
  std::lock_guard<std::mutex> lk(g_attr_mu);
  if (!cache[dev]) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, attr, dev) != hipSuccess || v < 1) {
      (void)hipGetLastError();
      v = fallback;
    }
    cache[dev] = v;
  }
  return cache[dev];
}

int device_cus(int dev) { return device_attr(dev, g_cus, hipDeviceAttributeMultiprocessorCount, 256); }
int device_lds_max(int dev) { return device_attr(dev, g_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, 64 * 1024); }

// ------------------------------------------------------------------------ debug collector
namespace {
std::mutex g_dbg_mu;
std::vector<debug_poll_fn>& polls() {
  static std::vector<debug_poll_fn> v;
  return v;
}
}  // namespace

bool register_debug_poll(debug_poll_fn fn) {
  std::lock_guard<std::mutex> lk(g_dbg_mu);
  polls().push_back(fn);
  return true;
}
}  // namespace sa

using namespace sa;

extern "C" int sa_device_alloc(int64_t bytes, int32_t flags, void** out) {
  if (!out || bytes <= 0 || (flags & ~1)) return fail(SA_EINVAL, "bad allocation request");
  *out = nullptr;
  if (flags & 1)
    return check_hip(hipExtMallocWithFlags(out, (size_t)bytes, hipDeviceMallocContiguous),
                     "sa_device_alloc: hipExtMallocWithFlags(contiguous)");
  return check_hip(hipMalloc(out, (size_t)bytes), "sa_device_alloc: hipMalloc");
}

extern "C" int sa_device_free(void* p) {
  return p ? check_hip(hipFree(p), "sa_device_free: hipFree") : SA_OK;
}

extern "C" int sa_copy2d_async(void* dst, int64_t dpitch, const void* src, int64_t spitch, int64_t width,
                               int64_t height, void* stream) {
  if (height == 0 || width == 0) return SA_OK;
  if (!dst || !src || width < 0 || height < 0 || dpitch < width || spitch < width)
    return fail(SA_EINVAL, "sa_copy2d_async: bad pitched copy");
  return check_hip(hipMemcpy2DAsync(dst, (size_t)dpitch, src, (size_t)spitch, (size_t)width, (size_t)height,
                                    hipMemcpyDefault, (hipStream_t)stream),
                   "sa_copy2d_async: hipMemcpy2DAsync");
}

extern "C" int sa_event_create(int32_t timing, void** ev) {
  if (!ev) return fail(SA_EINVAL, "sa_event_create: null output");
  *ev = nullptr;
  const unsigned flags = hipEventDisableSystemFence | (timing ? 0u : (unsigned)hipEventDisableTiming);
  return check_hip(hipEventCreateWithFlags(reinterpret_cast<hipEvent_t*>(ev), flags), "sa_event_create");
}

extern "C" int sa_event_destroy(void* ev) {
  return ev ? check_hip(hipEventDestroy((hipEvent_t)ev), "sa_event_destroy") : SA_OK;
}

extern "C" int sa_event_record(void* ev, void* stream) {
  if (!ev) return fail(SA_EINVAL, "sa_event_record: null event");
  return check_hip(hipEventRecord((hipEvent_t)ev, (hipStream_t)stream), "sa_event_record");
}

extern "C" int sa_stream_wait_event(void* stream, void* ev) {
  if (!ev) return fail(SA_EINVAL, "sa_stream_wait_event: null event");
  return check_hip(hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)ev, 0), "sa_stream_wait_event");
}

extern "C" int sa_event_synchronize(void* ev) {
  if (!ev) return fail(SA_EINVAL, "sa_event_synchronize: null event");
  return check_hip(hipEventSynchronize((hipEvent_t)ev), "sa_event_synchronize");
}

extern "C" int sa_event_elapsed(void* start, void* end, float* ms) {
  if (!start || !end || !ms) return fail(SA_EINVAL, "sa_event_elapsed: null argument");
  return check_hip(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)end), "sa_event_elapsed");
}

extern "C" int sa_abi_version(void) { return SA_ABI_VERSION; }

// one thread per segment: the blocks whose first row lies in [seg_off[g], seg_off[g+1])
__global__ void segment_blocks_kernel(const int64_t* __restrict__ seg_off, int64_t nseg,
                                      int32_t* __restrict__ seg_of_block) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nseg) return;
  const int64_t s = seg_off[g], e = seg_off[g + 1];
  for (int64_t b = (s + SA_SEG_BLOCK - 1) / SA_SEG_BLOCK; b * SA_SEG_BLOCK < e; ++b) seg_of_block[b] = (int32_t)g;
}

extern "C" int sa_segment_blocks(const int64_t* seg_off, int64_t n_segments, int64_t n, int32_t* seg_of_block,
                                 void* stream) {
  if (!seg_off || !seg_of_block || n_segments < 1 || n < 0 || n_segments > INT32_MAX)
    return fail(SA_EINVAL, "bad segment block args");
  if (n == 0) return SA_OK;
  hipLaunchKernelGGL(segment_blocks_kernel, dim3((unsigned)((n_segments + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, seg_off, n_segments, seg_of_block);
  return check_launch("segment_blocks_kernel");
}
extern "C" const char* sa_last_error(void) { return sa::g_err; }

// The build id is also kept as a plain marker string, so a build script can tell which sources
// a library file came from without loading it.
static const char kBuildMarker[] = "sa-build-id:" SA_BUILD_ID;
extern "C" const char* sa_build_id(void) { return kBuildMarker + 12; }

extern "C" int sa_debug_enabled(void) { return SA_DEBUG; }

extern "C" int sa_debug_check(void) {
#if SA_DEBUG
  int rc = check_hip(hipDeviceSynchronize(), "hipDeviceSynchronize");
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_dbg_mu);
  char msg[400];
  for (debug_poll_fn fn : polls()) {
    const int r = fn(msg, (int)sizeof(msg));
    if (r < 0) return fail(SA_EHIP, "sa_debug_check: reading the device record failed");
    if (r > 0) return fail(SA_EDATA, "%s", msg);
  }
#endif
  return SA_OK;
}

extern "C" int sa_shutdown(void) {
  std::lock_guard<std::mutex> lk(g_arena_mu);
  int rc = SA_OK;
  int cur = 0;
  (void)hipGetDevice(&cur);
  for (Slot& s : g_slots) {
    (void)hipSetDevice(s.dev);
    if (s.done) {
      if (!rc) rc = check_hip(hipEventSynchronize(s.done), "sa_shutdown: hipEventSynchronize");
      (void)hipEventDestroy(s.done);
    }
    if (s.ptr && !rc) rc = check_hip(hipFree(s.ptr), "sa_shutdown: hipFree");
  }
  (void)hipSetDevice(cur);
  g_slots.clear();
  return rc;
}
