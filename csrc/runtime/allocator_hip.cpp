// HIP backend of the auto-growth best-fit allocator (allocator.h) as a PyTorch pluggable allocator
// (torch.cuda.memory.CUDAPluggableAllocator: pa_malloc / pa_free) plus stats / release entry points for
// paddle.device.cuda.memory_* (paddlepaddle_amd/device/allocator.py). Host code only: hipMalloc / hipFree /
// events; built with hipcc into paddlepaddle_amd/_C_alloc.so.
#include <hip/hip_runtime.h>
#include <sys/types.h>

#include <cstdlib>
#include <mutex>

#include "allocator.h"

namespace {

constexpr int kMaxDev = 16;
pa_alloc::BestFitAllocator* g_alloc[kMaxDev] = {nullptr};
std::mutex g_mu;
size_t g_min_chunk = size_t(64) << 20;

struct DevGuard {
  int prev = -1;
  explicit DevGuard(int d) {
    (void)hipGetDevice(&prev);
    if (prev != d) (void)hipSetDevice(d);
  }
  ~DevGuard() {
    int cur = -1;
    (void)hipGetDevice(&cur);
    if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
  }
};

void* raw_alloc(size_t n, int dev) {
  DevGuard g(dev);
  void* p = nullptr;
  if (hipMalloc(&p, n) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return p;
}

void raw_free(void* p, int dev) {
  DevGuard g(dev);
  (void)hipFree(p);
}

void cross_stream_wait(uintptr_t owner, uintptr_t user, int dev) {
  DevGuard g(dev);
  hipEvent_t ev;
  if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
    (void)hipDeviceSynchronize();
    return;
  }
  (void)hipEventRecord(ev, reinterpret_cast<hipStream_t>(owner));
  (void)hipStreamWaitEvent(reinterpret_cast<hipStream_t>(user), ev, 0);
  (void)hipEventDestroy(ev);
}

void sync_device(int dev) {
  DevGuard g(dev);
  (void)hipDeviceSynchronize();
}

pa_alloc::BestFitAllocator* get(int dev) {
  if (dev < 0 || dev >= kMaxDev) return nullptr;
  pa_alloc::BestFitAllocator* a = g_alloc[dev];
  if (a != nullptr) return a;
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_alloc[dev] == nullptr) {
    const char* env = std::getenv("PADDLE_AMD_ALLOC_MIN_CHUNK_MB");
    if (env != nullptr) g_min_chunk = size_t(std::atoll(env)) << 20;
    g_alloc[dev] = new pa_alloc::BestFitAllocator({raw_alloc, raw_free, cross_stream_wait, sync_device}, dev,
                                                  g_min_chunk);
  }
  return g_alloc[dev];
}

}  // namespace

extern "C" __attribute__((visibility("default"))) void* pa_malloc(ssize_t size, int device, hipStream_t stream) {
  pa_alloc::BestFitAllocator* a = get(device);
  return a == nullptr ? nullptr : a->allocate(static_cast<size_t>(size), reinterpret_cast<uintptr_t>(stream));
}

extern "C" __attribute__((visibility("default"))) void pa_free(void* ptr, ssize_t size, int device, hipStream_t stream) {
  (void)size;
  (void)stream;
  pa_alloc::BestFitAllocator* a = get(device);
  if (a != nullptr) a->deallocate(ptr);
}

// out[11]: allocated, reserved, peak_allocated, peak_reserved, n_alloc, n_free, n_chunks, n_raw_alloc,
//          n_raw_free, n_cross_stream, n_oom_release
extern "C" __attribute__((visibility("default"))) int pa_alloc_stats(int device, int64_t* out) {
  pa_alloc::BestFitAllocator* a = (device >= 0 && device < kMaxDev) ? g_alloc[device] : nullptr;
  pa_alloc::Stats s;
  if (a != nullptr) s = a->stats();
  const int64_t v[11] = {s.allocated, s.reserved, s.peak_allocated, s.peak_reserved, s.n_alloc, s.n_free,
                         s.n_chunks, s.n_raw_alloc, s.n_raw_free, s.n_cross_stream, s.n_oom_release};
  for (int i = 0; i < 11; ++i) out[i] = v[i];
  return a != nullptr ? 0 : 1;
}

extern "C" __attribute__((visibility("default"))) int64_t pa_alloc_empty_cache(int device) {
  pa_alloc::BestFitAllocator* a = (device >= 0 && device < kMaxDev) ? g_alloc[device] : nullptr;
  return a == nullptr ? 0 : static_cast<int64_t>(a->release_free_chunks());
}

extern "C" __attribute__((visibility("default"))) void pa_alloc_reset_peak(int device) {
  pa_alloc::BestFitAllocator* a = (device >= 0 && device < kMaxDev) ? g_alloc[device] : nullptr;
  if (a != nullptr) a->reset_peaks();
}

extern "C" __attribute__((visibility("default"))) void pa_alloc_set_min_chunk(int64_t bytes) { g_min_chunk = bytes; }

// ---- graph-capture memory pools
extern "C" __attribute__((visibility("default"))) void pa_alloc_begin_pool(int device, hipStream_t stream,
                                                                          uint64_t pool) {
  pa_alloc::BestFitAllocator* a = get(device);
  if (a != nullptr) a->begin_pool(reinterpret_cast<uintptr_t>(stream), pool);
}

extern "C" __attribute__((visibility("default"))) void pa_alloc_end_pool(int device, hipStream_t stream) {
  pa_alloc::BestFitAllocator* a = get(device);
  if (a != nullptr) a->end_pool(reinterpret_cast<uintptr_t>(stream));
}

extern "C" __attribute__((visibility("default"))) void pa_alloc_release_pool(int device, uint64_t pool) {
  pa_alloc::BestFitAllocator* a = get(device);
  if (a != nullptr) a->release_pool(pool);
}

// ---- hipGraph capture / instantiate / launch (paddlepaddle_amd/device/cuda/graphs.py)
// mode: 0 global, 1 thread-local, 2 relaxed (hipStreamCaptureMode)
extern "C" __attribute__((visibility("default"))) int pa_graph_begin(hipStream_t stream, int mode) {
  const hipStreamCaptureMode m = mode == 0 ? hipStreamCaptureModeGlobal
                                           : (mode == 1 ? hipStreamCaptureModeThreadLocal : hipStreamCaptureModeRelaxed);
  return static_cast<int>(hipStreamBeginCapture(stream, m));
}

extern "C" __attribute__((visibility("default"))) int pa_graph_end(hipStream_t stream, void** graph_out,
                                                                  void** exec_out) {
  hipGraph_t g = nullptr;
  hipError_t e = hipStreamEndCapture(stream, &g);
  if (e != hipSuccess) return static_cast<int>(e);
  hipGraphExec_t x = nullptr;
  e = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
  if (e != hipSuccess) {
    (void)hipGraphDestroy(g);
    return static_cast<int>(e);
  }
  *graph_out = g;
  *exec_out = x;
  return 0;
}

extern "C" __attribute__((visibility("default"))) int pa_graph_launch(void* exec, hipStream_t stream) {
  return static_cast<int>(hipGraphLaunch(static_cast<hipGraphExec_t>(exec), stream));
}

extern "C" __attribute__((visibility("default"))) int pa_graph_num_nodes(void* graph, size_t* n) {
  return static_cast<int>(hipGraphGetNodes(static_cast<hipGraph_t>(graph), nullptr, n));
}

extern "C" __attribute__((visibility("default"))) int pa_graph_dot(void* graph, const char* path) {
  return static_cast<int>(hipGraphDebugDotPrint(static_cast<hipGraph_t>(graph), path, 0));
}

extern "C" __attribute__((visibility("default"))) void pa_graph_destroy(void* graph, void* exec) {
  if (exec != nullptr) (void)hipGraphExecDestroy(static_cast<hipGraphExec_t>(exec));
  if (graph != nullptr) (void)hipGraphDestroy(static_cast<hipGraph_t>(graph));
}
