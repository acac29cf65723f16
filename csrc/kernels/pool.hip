// Max pooling over channels-last (NHWC) activations, forward + backward, gfx950.
// Reference behaviour: paddle/phi/kernels/funcs/pooling.cu (max pool with padding as -inf, the first maximum
// of the window wins) and the mask-based backward of max_pool2d_with_index.
//
// Forward: a thread owns 8 channels of one output pixel (16-byte loads / stores); the value follows the
// reference's compare order (y = y > x ? y : x, so NaN behaves as in paddle/phi/kernels/funcs/pooling.h
// MaxPool), and the gradient slot is the first in-bounds element equal to the output (pooling.cu
// KernelMaxPool2DGrad's ele == input test; a NaN output gets no gradient), stored as a uint8 window offset
// (kernel <= 15x15, 255 = none). Backward is a gather, not a scatter: a
// thread owns 8 channels of one INPUT pixel, visits the <= ceil(K/s)^2 outputs whose windows contain it and
// adds dy where the stored offset points at this pixel — every dx element is written once, no atomics and
// no zero-fill pass (ATen's NHWC max_pool backward scatters into a zeroed dx).
#include "common.h"

using namespace pa;

namespace {

constexpr int kNoGrad = 255;  // window offsets are < 15 * 15

template <typename T>
__global__ __launch_bounds__(256) void maxpool_nhwc_fwd_k(const T* __restrict__ x, T* __restrict__ y,
                                                          uint8_t* __restrict__ arg, int N, int H, int W, int C,
                                                          int Ho, int Wo, int K, int s, int p) {
  const int cv = C / 8;
  const int64_t n_items = (int64_t)N * Ho * Wo * cv;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_items; i += (int64_t)gridDim.x * 256) {
    const int c8 = (int)(i % cv);
    int64_t t = i / cv;
    const int ow = (int)(t % Wo); t /= Wo;
    const int oh = (int)(t % Ho);
    const int n = (int)(t / Ho);
    float best[8];
    int bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = kNoGrad; }
    const int h0 = oh * s - p, w0 = ow * s - p;
    // value: the reference's running compare y = y > x ? y : x over the in-bounds window (a NaN is taken
    // when met and replaced by any later element)
    for (int kh = 0; kh < K; ++kh) {
      const int h = h0 + kh;
      if (h < 0 || h >= H) continue;
      for (int kw = 0; kw < K; ++kw) {
        const int w = w0 + kw;
        if (w < 0 || w >= W) continue;
        float v[8];
        load8<T>(x + (((int64_t)n * H + h) * W + w) * C + c8 * 8, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) best[j] = best[j] > v[j] ? best[j] : v[j];
      }
    }
    // gradient slot: the first in-bounds element equal to the output (the reference's ele == input test);
    // none for a NaN output (kNoGrad)
    for (int kh = 0; kh < K; ++kh) {
      const int h = h0 + kh;
      if (h < 0 || h >= H) continue;
      for (int kw = 0; kw < K; ++kw) {
        const int w = w0 + kw;
        if (w < 0 || w >= W) continue;
        float v[8];
        load8<T>(x + (((int64_t)n * H + h) * W + w) * C + c8 * 8, v);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (bi[j] == kNoGrad && v[j] == best[j]) bi[j] = kh * K + kw;
      }
    }
    store8<T>(y + i * 8, best);
    uint2 packed;
    packed.x = (uint32_t)bi[0] | ((uint32_t)bi[1] << 8) | ((uint32_t)bi[2] << 16) | ((uint32_t)bi[3] << 24);
    packed.y = (uint32_t)bi[4] | ((uint32_t)bi[5] << 8) | ((uint32_t)bi[6] << 16) | ((uint32_t)bi[7] << 24);
    *reinterpret_cast<uint2*>(arg + i * 8) = packed;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void maxpool_nhwc_bwd_k(const T* __restrict__ dy, const uint8_t* __restrict__ arg,
                                                          T* __restrict__ dx, int N, int H, int W, int C, int Ho,
                                                          int Wo, int K, int s, int p) {
  const int cv = C / 8;
  const int64_t n_items = (int64_t)N * H * W * cv;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_items; i += (int64_t)gridDim.x * 256) {
    const int c8 = (int)(i % cv);
    int64_t t = i / cv;
    const int w = (int)(t % W); t /= W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // outputs whose window [o*s - p, o*s - p + K) contains h: o in [ceil((h + p - K + 1) / s), floor((h + p) / s)]
    const int oh_lo = max(0, (h + p - K + s) / s), oh_hi = min(Ho - 1, (h + p) / s);
    const int ow_lo = max(0, (w + p - K + s) / s), ow_hi = min(Wo - 1, (w + p) / s);
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int kh = h - (oh * s - p);
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int kw = w - (ow * s - p);
        const int64_t o = (((int64_t)n * Ho + oh) * Wo + ow) * C + c8 * 8;
        const uint2 packed = *reinterpret_cast<const uint2*>(arg + o);
        const int me = kh * K + kw;
        bool hit = false;
#pragma unroll
        for (int j = 0; j < 8; ++j) hit |= (int)(((j < 4 ? packed.x : packed.y) >> (8 * (j & 3))) & 0xff) == me;
        if (!hit) continue;
        float g[8];
        load8<T>(dy + o, g);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if ((int)(((j < 4 ? packed.x : packed.y) >> (8 * (j & 3))) & 0xff) == me) acc[j] += g[j];
      }
    }
    store8<T>(dx + i * 8, acc);
  }
}

inline unsigned pool_grid(int64_t items) {
  int64_t g = (items + 255) / 256;
  if (g > 16384) g = 16384;
  return (unsigned)(g < 1 ? 1 : g);
}

}  // namespace

// x [N, H, W, C] -> y [N, Ho, Wo, C] and arg [N, Ho, Wo, C] uint8 (window offset kh*K + kw of the max)
PA_EXPORT int pa_maxpool_nhwc_fwd(const void* x, void* y, void* arg, int N, int H, int W, int C, int Ho, int Wo, int K,
                                  int s, int p, int dtype, hipStream_t st) {
  if (C % 8 || K < 1 || K * K > 255 || s < 1 || p < 0 || 2 * p > K) return 2;
  const int64_t items = (int64_t)N * Ho * Wo * (C / 8);
  PA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((maxpool_nhwc_fwd_k<T>), dim3(pool_grid(items)), dim3(256), 0, st,
                                                 (const T*)x, (T*)y, (uint8_t*)arg, N, H, W, C, Ho, Wo, K, s, p));
  PA_CHECK_LAUNCH();
  return 0;
}

PA_EXPORT int pa_maxpool_nhwc_bwd(const void* dy, const void* arg, void* dx, int N, int H, int W, int C, int Ho, int Wo,
                                  int K, int s, int p, int dtype, hipStream_t st) {
  if (C % 8 || K < 1 || K * K > 255 || s < 1 || p < 0) return 2;
  const int64_t items = (int64_t)N * H * W * (C / 8);
  PA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((maxpool_nhwc_bwd_k<T>), dim3(pool_grid(items)), dim3(256), 0, st,
                                                 (const T*)dy, (const uint8_t*)arg, (T*)dx, N, H, W, C, Ho, Wo, K, s,
                                                 p));
  PA_CHECK_LAUNCH();
  return 0;
}
