// GEMM-epilogue companions for gfx950: bias-gradient column reduction, fused bias+GELU backward,
// fused dropout + residual add with a counter-based RNG (mask regenerated in backward, never stored).
// Reference behaviour: paddle/phi/kernels/fusion/gpu/fused_gemm_epilogue_kernel.cu (bias grad),
// fused_bias_act_kernel.cu, fused_dropout_add_kernel.cu.
//
// Column reductions use a 2-D grid: x = 2048-column stripe (256 threads x 8 columns, 16-byte loads,
// so one row of a stripe is a 4 KB coalesced read), y = row partition; fp32 partials go to a
// workspace [nparts, cols] and a second launch folds them (no atomics, deterministic).
#include "common.h"

using namespace pa;

namespace {

constexpr float kSqrt2OverPi = 0.7978845608028654f;
constexpr float kCoeff = 0.044715f;

__device__ __forceinline__ float gelu_tanh_grad(float x) { return gelu_tanh_grad_fast(x); }

// ---- counter-based RNG (64-bit mix, splitmix/murmur finaliser) -> uniform [0,1)
__device__ __forceinline__ uint32_t hash32(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}
__device__ __forceinline__ bool keep(uint64_t seed, uint64_t i, uint32_t thresh) { return hash32(seed, i) >= thresh; }

template <typename T>
__global__ __launch_bounds__(256) void colsum_partial_k(const T* __restrict__ x, float* __restrict__ part, int64_t rows,
                                                        int64_t cols, int nparts) {
  const int64_t c = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= cols) return;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t r = blockIdx.y; r < rows; r += nparts) {
    float v[8];
    load8<T>(x + r * cols + c, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += v[j];
  }
  store8<float>(part + (int64_t)blockIdx.y * cols + c, acc);
}

// Fold [nparts, cols] fp32 partials: a block owns 64 columns (8 x 8-column vectors) and spreads the
// partitions over 32 row groups, then reduces the groups through LDS — cols/64 blocks instead of one
// serial 256-deep loop per thread (which left all but ~10 CUs idle on a 20480-column bias).
template <typename T>
__global__ __launch_bounds__(256) void fold_partials_k(const float* __restrict__ part, T* __restrict__ out,
                                                       int64_t cols, int nparts, int accumulate) {
  __shared__ float red[32][65];
  const int cv = threadIdx.x & 7, rg = threadIdx.x >> 3;
  const int64_t c = (int64_t)blockIdx.x * 64 + cv * 8;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c < cols) {
    for (int p = rg; p < nparts; p += 32) {
      float v[8];
      load8<float>(part + (int64_t)p * cols + c, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rg][cv * 8 + j] = acc[j];
  __syncthreads();
  if (threadIdx.x < 64) {
    float sum = 0.f;
#pragma unroll 8
    for (int g = 0; g < 32; ++g) sum += red[g][threadIdx.x];
    red[0][threadIdx.x] = sum;
  }
  __syncthreads();
  if (rg == 0 && c < cols) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = red[0][cv * 8 + j];
    if (accumulate) {  // gradient-accumulation fusion: out += column sums (the parameter's .grad buffer)
      float o[8];
      load8<T>(out + c, o);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += o[j];
    }
    store8<T>(out + c, v);
  }
}

// dh = dy * gelu'(h + b) ; part[p, c] += dh   (h = pre-bias GEMM output)
template <typename T>
__global__ __launch_bounds__(256) void bias_gelu_bwd_k(const T* __restrict__ h, const T* __restrict__ b,
                                                       const T* __restrict__ dy, T* __restrict__ dh,
                                                       float* __restrict__ part, int64_t rows, int64_t cols,
                                                       int nparts) {
  const int64_t c = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= cols) return;
  float bv[8], acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  load8<T>(b + c, bv);
  for (int64_t r = blockIdx.y; r < rows; r += nparts) {
    float hv[8], g[8];
    load8<T>(h + r * cols + c, hv);
    load8<T>(dy + r * cols + c, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      g[j] *= gelu_tanh_grad(hv[j] + bv[j]);
      acc[j] += g[j];
    }
    store8<T>(dh + r * cols + c, g);
  }
  store8<float>(part + (int64_t)blockIdx.y * cols + c, acc);
}

// out = residual + keep(i) * x / (1-p)
template <typename T>
__global__ __launch_bounds__(256) void dropout_add_k(const T* __restrict__ x, const T* __restrict__ res,
                                                     T* __restrict__ out, int64_t nvec, uint64_t seed, uint32_t thresh,
                                                     float scale) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    float a[8], r[8];
    load8<T>(x + i * 8, a);
    if (res) load8<T>(res + i * 8, r); else {
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] += keep(seed, i * 8 + j, thresh) ? a[j] * scale : 0.f;
    store8<T>(out + i * 8, r);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void dropout_bwd_k(const T* __restrict__ dy, T* __restrict__ dx, int64_t nvec,
                                                     uint64_t seed, uint32_t thresh, float scale) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    float g[8];
    load8<T>(dy + i * 8, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = keep(seed, i * 8 + j, thresh) ? g[j] * scale : 0.f;
    store8<T>(dx + i * 8, g);
  }
}

// dropout backward of a [rows, cols] gradient that also writes the column partials of dx (the bias gradient of the
// linear whose output was dropped out: out-proj / FFN2 of a transformer block), laid out like colsum_partial_k's.
// The keep mask is indexed by the flat element index r * cols + c, as in dropout_add_k.
template <typename T>
__global__ __launch_bounds__(256) void dropout_bwd_colsum_k(const T* __restrict__ dy, T* __restrict__ dx,
                                                            float* __restrict__ part, int64_t rows, int64_t cols,
                                                            int nparts, uint64_t seed, uint32_t thresh, float scale) {
  const int64_t c = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= cols) return;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t r = blockIdx.y; r < rows; r += nparts) {
    float g[8];
    const int64_t e = r * cols + c;
    load8<T>(dy + e, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      g[j] = keep(seed, e + j, thresh) ? g[j] * scale : 0.f;
      acc[j] += g[j];
    }
    store8<T>(dx + e, g);
  }
  store8<float>(part + (int64_t)blockIdx.y * cols + c, acc);
}

inline int nparts_for(int64_t rows) {
  int64_t p = rows / 32;
  if (p < 1) p = 1;
  if (p > 256) p = 256;
  return (int)p;
}

inline unsigned grid_ew(int64_t nvec) {
  int64_t g = cdiv(nvec, 256);
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (unsigned)g;
}

}  // namespace

// workspace: fp32 [256 * cols] (caller-provided, reused)
// dtype bit 8: accumulate into `out` instead of overwriting it
PA_EXPORT int pa_colsum(const void* x, void* out, float* ws, int64_t rows, int64_t cols, int dtype_acc, hipStream_t st) {
  const int dtype = dtype_acc & 0xff, acc = (dtype_acc >> 8) & 1;
  const int np = nparts_for(rows);
  dim3 g1((unsigned)cdiv(cols, 2048), (unsigned)np), g2((unsigned)cdiv(cols, 64));
  PA_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((colsum_partial_k<T>), g1, dim3(256), 0, st, (const T*)x, ws, rows, cols, np);
    hipLaunchKernelGGL((fold_partials_k<T>), g2, dim3(256), 0, st, ws, (T*)out, cols, np, acc);
  });
  PA_CHECK_LAUNCH();
  return 0;
}

// dtype bit 8: accumulate the bias gradient into `db`
PA_EXPORT int pa_bias_gelu_bwd(const void* h, const void* b, const void* dy, void* dh, void* db, float* ws,
                               int64_t rows, int64_t cols, int dtype_acc, hipStream_t st) {
  const int dtype = dtype_acc & 0xff, acc = (dtype_acc >> 8) & 1;
  const int np = nparts_for(rows);
  dim3 g1((unsigned)cdiv(cols, 2048), (unsigned)np), g2((unsigned)cdiv(cols, 64));
  PA_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL((bias_gelu_bwd_k<T>), g1, dim3(256), 0, st, (const T*)h, (const T*)b, (const T*)dy, (T*)dh,
                       ws, rows, cols, np);
    hipLaunchKernelGGL((fold_partials_k<T>), g2, dim3(256), 0, st, ws, (T*)db, cols, np, acc);
  });
  PA_CHECK_LAUNCH();
  return 0;
}

PA_EXPORT int pa_dropout_add_fwd(const void* x, const void* res, void* out, int64_t n, float p, uint64_t seed,
                                 int dtype, hipStream_t st) {
  const int64_t nvec = n / 8;
  const uint32_t thresh = (uint32_t)fminf(p * 4294967296.0f, 4294967295.0f);
  const float scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  PA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((dropout_add_k<T>), dim3(grid_ew(nvec)), dim3(256), 0, st,
                                                 (const T*)x, (const T*)res, (T*)out, nvec, seed, thresh, scale));
  PA_CHECK_LAUNCH();
  return 0;
}

PA_EXPORT int pa_dropout_bwd(const void* dy, void* dx, int64_t n, float p, uint64_t seed, int dtype, hipStream_t st) {
  const int64_t nvec = n / 8;
  const uint32_t thresh = (uint32_t)fminf(p * 4294967296.0f, 4294967295.0f);
  const float scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  PA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((dropout_bwd_k<T>), dim3(grid_ew(nvec)), dim3(256), 0, st,
                                                 (const T*)dy, (T*)dx, nvec, seed, thresh, scale));
  PA_CHECK_LAUNCH();
  return 0;
}

// dropout backward over a [rows, cols] gradient + the column partials of dx into ws [nparts, cols] (fp32, nparts =
// pa_colsum_nparts(rows)); pa_fold_partials turns them into the column sums later (bias gradient)
PA_EXPORT int pa_dropout_bwd_colsum(const void* dy, void* dx, float* ws, int64_t rows, int64_t cols, float p,
                                    uint64_t seed, int dtype, hipStream_t st) {
  if (cols % 8) return 1;
  const uint32_t thresh = (uint32_t)fminf(p * 4294967296.0f, 4294967295.0f);
  const float scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  const int np = nparts_for(rows);
  dim3 g1((unsigned)cdiv(cols, 2048), (unsigned)np);
  PA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((dropout_bwd_colsum_k<T>), g1, dim3(256), 0, st, (const T*)dy, (T*)dx,
                                                 ws, rows, cols, np, seed, thresh, scale));
  PA_CHECK_LAUNCH();
  return 0;
}

PA_EXPORT int64_t pa_colsum_nparts(int64_t rows) { return nparts_for(rows); }

// dtype bit 8: accumulate into `out`
PA_EXPORT int pa_fold_partials(const float* ws, void* out, int64_t cols, int64_t nparts, int dtype_acc,
                               hipStream_t st) {
  const int dtype = dtype_acc & 0xff, acc = (dtype_acc >> 8) & 1;
  dim3 g2((unsigned)cdiv(cols, 64));
  PA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((fold_partials_k<T>), g2, dim3(256), 0, st, ws, (T*)out, cols,
                                                 (int)nparts, acc));
  PA_CHECK_LAUNCH();
  return 0;
}
