// Elementwise activation kernels + fused rotary embedding for gfx950.
// Reference behaviour: paddle/phi/kernels/gpu/gelu_kernel.cu, fusion/gpu/fused_bias_act_kernel.cu,
// incubate swiglu, fusion/gpu/fused_rope_kernel.cu.
// All kernels: 16-byte vectors per thread, grid-stride, grid capped at 256 CUs x 8 workgroups.
#include "common.h"

#include <algorithm>

using namespace pa;

namespace {

constexpr float kSqrt2OverPi = 0.7978845608028654f;
constexpr float kCoeff = 0.044715f;
constexpr float kInvSqrt2 = 0.7071067811865476f;
constexpr float kInvSqrt2Pi = 0.3989422804014327f;

__device__ __forceinline__ float gelu_f(float x, bool approx) {
  if (approx) return gelu_tanh_fast(x);
  return 0.5f * x * (1.f + erff(x * kInvSqrt2));
}

__device__ __forceinline__ float gelu_grad_f(float x, bool approx) {
  if (approx) return gelu_tanh_grad_fast(x);
  return 0.5f * (1.f + erff(x * kInvSqrt2)) + x * kInvSqrt2Pi * __expf(-0.5f * x * x);
}

__device__ __forceinline__ float silu_f(float x) { return x / (1.f + __expf(-x)); }

inline unsigned grid_for(int64_t nvec) {
  int64_t g = cdiv(nvec, 256);
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (unsigned)g;
}

template <typename T>
__global__ __launch_bounds__(256) void gelu_fwd_k(const T* __restrict__ x, T* __restrict__ y, int64_t nvec, bool approx) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    float v[8];
    load8<T>(x + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = gelu_f(v[j], approx);
    store8<T>(y + i * 8, v);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void gelu_bwd_k(const T* __restrict__ x, const T* __restrict__ dy, T* __restrict__ dx,
                                                  int64_t nvec, bool approx) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    float v[8], g[8];
    load8<T>(x + i * 8, v);
    load8<T>(dy + i * 8, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = g[j] * gelu_grad_f(v[j], approx);
    store8<T>(dx + i * 8, v);
  }
}

// y[r, c] = gelu_tanh(x[r, c] + b[c])
template <typename T>
// 2-D grid: blockIdx.x = 2048-column strip (a thread's 8 columns and their bias are fixed), blockIdx.y strides
// over the rows — no per-element index division.
__global__ __launch_bounds__(256) void bias_gelu_fwd_k(const T* __restrict__ x, const T* __restrict__ b,
                                                       T* __restrict__ y, int64_t rows, int64_t cols) {
  const int64_t c = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= cols) return;
  float bv[8];
  load8<T>(b + c, bv);
#pragma unroll 4
  for (int64_t r = blockIdx.y; r < rows; r += gridDim.y) {
    float v[8];
    load8<T>(x + r * cols + c, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = gelu_tanh_fast(v[j] + bv[j]);
    store8<T>(y + r * cols + c, v);
  }
}

// y = silu(a) * b over [rows, cols]; a, b have row stride `ld` (halves of a [rows, 2*cols] buffer allowed)
template <typename T>
__global__ __launch_bounds__(256) void swiglu_fwd_k(const T* __restrict__ a, const T* __restrict__ b, T* __restrict__ y,
                                                    int64_t rows, int64_t cols, int64_t ld) {
  const int64_t vpr = cols / 8, nvec = rows * vpr;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / vpr, c = (i % vpr) * 8;
    float av[8], bv[8];
    load8<T>(a + r * ld + c, av);
    load8<T>(b + r * ld + c, bv);
#pragma unroll
    for (int j = 0; j < 8; ++j) av[j] = silu_f(av[j]) * bv[j];
    store8<T>(y + r * cols + c, av);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void swiglu_bwd_k(const T* __restrict__ a, const T* __restrict__ b,
                                                    const T* __restrict__ dy, T* __restrict__ da, T* __restrict__ db,
                                                    int64_t rows, int64_t cols, int64_t ld, int64_t ldo) {
  const int64_t vpr = cols / 8, nvec = rows * vpr;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / vpr, c = (i % vpr) * 8;
    float av[8], bv[8], g[8], oa[8], ob[8];
    load8<T>(a + r * ld + c, av);
    load8<T>(b + r * ld + c, bv);
    load8<T>(dy + r * cols + c, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float s = 1.f / (1.f + __expf(-av[j]));
      ob[j] = g[j] * av[j] * s;
      oa[j] = g[j] * bv[j] * s * (1.f + av[j] * (1.f - s));
    }
    store8<T>(da + r * ldo + c, oa);
    store8<T>(db + r * ldo + c, ob);
  }
}

// Rotary embedding on x [B,S,H,D]; cos/sin fp32 [>=S, D].
// neox: rotate halves (d, d+D/2); else interleaved pairs (2i, 2i+1). inverse: use -sin (backward).
template <typename T, bool NEOX>
__global__ __launch_bounds__(256) void rope_k(const T* __restrict__ x, const float* __restrict__ cs,
                                              const float* __restrict__ sn, T* __restrict__ out, int64_t B, int64_t S,
                                              int64_t H, int64_t D, float sgn) {
  // NEOX: one thread handles 8 elements of the first half and the matching 8 of the second half
  const int64_t per_row = NEOX ? D / 16 : D / 8;
  const int64_t n = B * S * H * per_row;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t row = i / per_row;          // (b, s, h)
    const int64_t k = i % per_row;
    const int64_t s = (row / H) % S;
    const T* xr = x + row * D;
    T* orow = out + row * D;
    if (NEOX) {
      const int64_t d0 = k * 8, d1 = d0 + D / 2;
      float a[8], b[8], oa[8], ob[8];
      load8<T>(xr + d0, a);
      load8<T>(xr + d1, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float c0 = cs[s * D + d0 + j], s0 = sn[s * D + d0 + j] * sgn;
        const float c1 = cs[s * D + d1 + j], s1 = sn[s * D + d1 + j] * sgn;
        oa[j] = a[j] * c0 - b[j] * s0;
        ob[j] = b[j] * c1 + a[j] * s1;
      }
      store8<T>(orow + d0, oa);
      store8<T>(orow + d1, ob);
    } else {
      const int64_t d0 = k * 8;
      float a[8], o[8];
      load8<T>(xr + d0, a);
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const float c0 = cs[s * D + d0 + j], s0 = sn[s * D + d0 + j] * sgn;
        const float c1 = cs[s * D + d0 + j + 1], s1 = sn[s * D + d0 + j + 1] * sgn;
        o[j] = a[j] * c0 - a[j + 1] * s0;
        o[j + 1] = a[j + 1] * c1 + a[j] * s1;
      }
      store8<T>(orow + d0, o);
    }
  }
}

// RoPE over the first NH heads of token rows with their own leading dims: the fused QKV projection layout
// [B*S, ld] = [q heads | k heads | v heads]. Forward rotates q|k out of the projection into a packed buffer;
// backward rotates dq|dk in place inside the one qkv-gradient buffer (each thread reads its elements before
// writing them, so x == out is allowed: no __restrict__ on x / out).
template <typename T, bool NEOX>
__global__ __launch_bounds__(256) void rope_rows_k(const T* x, int64_t ldx, const float* __restrict__ cs,
                                                   const float* __restrict__ sn, T* out, int64_t ldo, int64_t rows,
                                                   int64_t S, int64_t NH, int64_t D, float sgn) {
  const int64_t per_head = NEOX ? D / 16 : D / 8;
  const int64_t per_row = NH * per_head;
  const int64_t n = rows * per_row;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t tok = i / per_row;
    const int64_t rem = i - tok * per_row;
    const int64_t h = rem / per_head, k = rem - h * per_head;
    const int64_t s = tok % S;
    const T* xr = x + tok * ldx + h * D;
    T* orow = out + tok * ldo + h * D;
    const float* cr = cs + s * D;
    const float* sr = sn + s * D;
    if (NEOX) {
      const int64_t d0 = k * 8, d1 = d0 + D / 2;
      float a[8], b[8], oa[8], ob[8];
      load8<T>(xr + d0, a);
      load8<T>(xr + d1, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        oa[j] = a[j] * cr[d0 + j] - b[j] * sr[d0 + j] * sgn;
        ob[j] = b[j] * cr[d1 + j] + a[j] * sr[d1 + j] * sgn;
      }
      store8<T>(orow + d0, oa);
      store8<T>(orow + d1, ob);
    } else {
      const int64_t d0 = k * 8;
      float a[8], o[8];
      load8<T>(xr + d0, a);
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        o[j] = a[j] * cr[d0 + j] - a[j + 1] * sr[d0 + j] * sgn;
        o[j + 1] = a[j + 1] * cr[d0 + j + 1] + a[j] * sr[d0 + j + 1] * sgn;
      }
      store8<T>(orow + d0, o);
    }
  }
}

}  // namespace

PA_EXPORT int pa_gelu_fwd(const void* x, void* y, int64_t n, int approx, int dtype, hipStream_t st) {
  const int64_t nvec = n / 8;
  PA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((gelu_fwd_k<T>), dim3(grid_for(nvec)), dim3(256), 0, st,
                                                 (const T*)x, (T*)y, nvec, approx != 0));
  PA_CHECK_LAUNCH();
  return 0;
}

PA_EXPORT int pa_gelu_bwd(const void* x, const void* dy, void* dx, int64_t n, int approx, int dtype, hipStream_t st) {
  const int64_t nvec = n / 8;
  PA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((gelu_bwd_k<T>), dim3(grid_for(nvec)), dim3(256), 0, st,
                                                 (const T*)x, (const T*)dy, (T*)dx, nvec, approx != 0));
  PA_CHECK_LAUNCH();
  return 0;
}

PA_EXPORT int pa_bias_gelu_fwd(const void* x, const void* b, void* y, int64_t rows, int64_t cols, int dtype,
                               hipStream_t st) {
  const unsigned gx = (unsigned)cdiv(cols / 8, 256);
  const unsigned gy = (unsigned)std::max<int64_t>(1, std::min<int64_t>(rows, 2048 / gx));
  PA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((bias_gelu_fwd_k<T>), dim3(gx, gy), dim3(256), 0, st,
                                                 (const T*)x, (const T*)b, (T*)y, rows, cols));
  PA_CHECK_LAUNCH();
  return 0;
}

PA_EXPORT int pa_swiglu_fwd(const void* a, const void* b, void* y, int64_t rows, int64_t cols, int64_t ld, int dtype,
                            hipStream_t st) {
  const int64_t nvec = rows * cols / 8;
  PA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((swiglu_fwd_k<T>), dim3(grid_for(nvec)), dim3(256), 0, st,
                                                 (const T*)a, (const T*)b, (T*)y, rows, cols, ld));
  PA_CHECK_LAUNCH();
  return 0;
}

PA_EXPORT int pa_swiglu_bwd(const void* a, const void* b, const void* dy, void* da, void* db, int64_t rows,
                            int64_t cols, int64_t ld_packed, int dtype, hipStream_t st) {
  const int64_t ld = ld_packed & 0xffffffffLL, ldo = (ld_packed >> 32) & 0xffffffffLL;
  const int64_t nvec = rows * cols / 8;
  PA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((swiglu_bwd_k<T>), dim3(grid_for(nvec)), dim3(256), 0, st,
                                                 (const T*)a, (const T*)b, (const T*)dy, (T*)da, (T*)db, rows, cols,
                                                 ld, ldo));
  PA_CHECK_LAUNCH();
  return 0;
}

PA_EXPORT int pa_rope_fwd(const void* x, const float* cs, const float* sn, void* out, int64_t B, int64_t S, int64_t H,
                          int64_t D, int flags, int dtype, hipStream_t st) {
  const bool neox = flags & 1;
  const float sgn = (flags & 2) ? -1.f : 1.f;
  const int64_t n = B * S * H * (neox ? D / 16 : D / 8);
  if (neox) {
    PA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((rope_k<T, true>), dim3(grid_for(n)), dim3(256), 0, st,
                                                   (const T*)x, cs, sn, (T*)out, B, S, H, D, sgn));
  } else {
    PA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((rope_k<T, false>), dim3(grid_for(n)), dim3(256), 0, st,
                                                   (const T*)x, cs, sn, (T*)out, B, S, H, D, sgn));
  }
  PA_CHECK_LAUNCH();
  return 0;
}

PA_EXPORT int pa_rope_rows(const void* x, int64_t ldx, const float* cs, const float* sn, void* out, int64_t ldo,
                           int64_t rows, int64_t S, int64_t NH, int64_t D, int flags, int dtype, hipStream_t st) {
  const bool neox = flags & 1;
  const float sgn = (flags & 2) ? -1.f : 1.f;
  const int64_t n = rows * NH * (neox ? D / 16 : D / 8);
  if (neox) {
    PA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((rope_rows_k<T, true>), dim3(grid_for(n)), dim3(256), 0, st,
                                                   (const T*)x, ldx, cs, sn, (T*)out, ldo, rows, S, NH, D, sgn));
  } else {
    PA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((rope_rows_k<T, false>), dim3(grid_for(n)), dim3(256), 0, st,
                                                   (const T*)x, ldx, cs, sn, (T*)out, ldo, rows, S, NH, D, sgn));
  }
  PA_CHECK_LAUNCH();
  return 0;
}
