// Softmax and fused softmax-cross-entropy for gfx950.
// Reference behaviour: paddle/phi/kernels/gpu/softmax_kernel.cu, cross_entropy_kernel.cu
// (softmax_with_cross_entropy, hard labels, ignore_index).
//
// Rows up to 64K wide, cols % 8 == 0. One 256-thread workgroup per row, 16-byte vector loads,
// online (max, sum) merge in one pass: the logits row is read once for the statistics and once
// more for the output (second read is usually an L2 hit: a 50K-vocab bf16 row is 100 KB).
#include "common.h"

using namespace pa;

namespace {

struct MS { float m, s; };

__device__ __forceinline__ MS ms_merge(MS a, MS b) {
  const float m = fmaxf(a.m, b.m);
  if (m == -INFINITY) return {m, 0.f};
  return {m, a.s * __expf(a.m - m) + b.s * __expf(b.m - m)};
}

__device__ __forceinline__ MS wave_ms(MS v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    MS u{__shfl_xor(v.m, o, 64), __shfl_xor(v.s, o, 64)};
    v = ms_merge(v, u);
  }
  return v;
}

__device__ __forceinline__ MS block_ms(MS v, float* sm, float* ss) {
  v = wave_ms(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) { sm[w] = v.m; ss[w] = v.s; }
  __syncthreads();
  MS r{sm[0], ss[0]};
#pragma unroll
  for (int i = 1; i < 4; ++i) r = ms_merge(r, MS{sm[i], ss[i]});
  return r;
}

template <typename T>
__device__ __forceinline__ MS row_stats(const T* xr, int64_t cols) {
  MS acc{-INFINITY, 0.f};
  for (int64_t e = (int64_t)threadIdx.x * 8; e < cols; e += 2048) {
    float v[8];
    load8<T>(xr + e, v);
    float m = v[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) m = fmaxf(m, v[j]);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += __expf(v[j] - m);
    acc = ms_merge(acc, MS{m, s});
  }
  return acc;
}

template <typename T>
__global__ __launch_bounds__(256) void softmax_fwd_k(const T* __restrict__ x, T* __restrict__ y, int64_t cols) {
  __shared__ float sm[4], ss[4];
  const int64_t row = blockIdx.x;
  const T* xr = x + row * cols;
  MS st = block_ms(row_stats<T>(xr, cols), sm, ss);
  const float inv = 1.0f / st.s;
  T* yr = y + row * cols;
  for (int64_t e = (int64_t)threadIdx.x * 8; e < cols; e += 2048) {
    float v[8];
    load8<T>(xr + e, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = __expf(v[j] - st.m) * inv;
    store8<T>(yr + e, v);
  }
}

// dx = y * (dy - sum(dy*y))
template <typename T>
__global__ __launch_bounds__(256) void softmax_bwd_k(const T* __restrict__ y, const T* __restrict__ dy,
                                                     T* __restrict__ dx, int64_t cols) {
  __shared__ float red[4];
  const int64_t row = blockIdx.x;
  float s = 0.f;
  for (int64_t e = (int64_t)threadIdx.x * 8; e < cols; e += 2048) {
    float a[8], b[8];
    load8<T>(y + row * cols + e, a);
    load8<T>(dy + row * cols + e, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j] * b[j];
  }
  s = block_sum<256>(s, red);
  for (int64_t e = (int64_t)threadIdx.x * 8; e < cols; e += 2048) {
    float a[8], b[8], o[8];
    load8<T>(y + row * cols + e, a);
    load8<T>(dy + row * cols + e, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = a[j] * (b[j] - s);
    store8<T>(dx + row * cols + e, o);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void softmax_ce_fwd_k(const T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                        float* __restrict__ loss, float* __restrict__ lse_out,
                                                        int64_t cols, int64_t ignore_index) {
  __shared__ float sm[4], ss[4];
  const int64_t row = blockIdx.x;
  const T* xr = logits + row * cols;
  MS st = block_ms(row_stats<T>(xr, cols), sm, ss);
  if (threadIdx.x == 0) {
    const float lse = st.m + __logf(st.s);
    lse_out[row] = lse;
    const int64_t lb = labels[row];
    if (lb == ignore_index || lb < 0 || lb >= cols) {
      loss[row] = 0.f;
    } else {
      loss[row] = lse - to_f(xr[lb]);
    }
  }
}

// dlogits = (softmax - onehot(label)) * dloss[row]; ignored rows -> 0
template <typename T>
__global__ __launch_bounds__(256) void softmax_ce_bwd_k(const T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                        const float* __restrict__ lse, const float* __restrict__ dloss,
                                                        T* __restrict__ dlogits, int64_t cols, int64_t ignore_index) {
  const int64_t row = blockIdx.x;
  const int64_t lb = labels[row];
  const bool ign = (lb == ignore_index || lb < 0 || lb >= cols);
  const float g = ign ? 0.f : dloss[row];
  const float l = lse[row];
  const T* xr = logits + row * cols;
  T* dr = dlogits + row * cols;
  for (int64_t e = (int64_t)threadIdx.x * 8; e < cols; e += 2048) {
    float v[8];
    load8<T>(xr + e, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float p = __expf(v[j] - l);
      if (e + j == lb) p -= 1.f;
      v[j] = p * g;
    }
    store8<T>(dr + e, v);
  }
}

// ---- vocabulary-slice cross entropy (vocab-parallel CE over the mp group, vocab-chunked fused LM head):
// the kernels see columns [v0, v0 + cols) of the full vocabulary.
// fwd: lse_out[row] = logsumexp of the slice, tgt_out[row] = logit of the row's label when it falls in the slice
//      (else 0); the caller combines the slices (one small collective / torch op).
// bwd: dlogits = (exp(x - lse[row]) - [label == v0 + j]) * dloss[row] with the GLOBAL lse; a label outside the slice
//      only drops the one-hot term, rows whose label is ignore_index get 0. May run in place (dlogits == logits).
template <typename T>
__global__ __launch_bounds__(256) void ce_slice_fwd_k(const T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                      float* __restrict__ lse_out, float* __restrict__ tgt_out,
                                                      int64_t cols, int64_t v0) {
  __shared__ float sm[4], ss[4];
  const int64_t row = blockIdx.x;
  const T* xr = logits + row * cols;
  MS st = block_ms(row_stats<T>(xr, cols), sm, ss);
  if (threadIdx.x == 0) {
    lse_out[row] = st.m + __logf(st.s);
    const int64_t lb = labels[row] - v0;
    tgt_out[row] = (lb >= 0 && lb < cols) ? to_f(xr[lb]) : 0.f;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void ce_slice_bwd_k(const T* logits, const int64_t* __restrict__ labels,
                                                      const float* __restrict__ lse, const float* __restrict__ dloss,
                                                      T* dlogits, int64_t cols, int64_t v0, int64_t ignore_index) {
  const int64_t row = blockIdx.x;
  const int64_t lab = labels[row];
  const float g = lab == ignore_index ? 0.f : dloss[row];
  const int64_t lb = lab - v0;
  const float l = lse[row];
  const T* xr = logits + row * cols;
  T* dr = dlogits + row * cols;
  for (int64_t e = (int64_t)threadIdx.x * 8; e < cols; e += 2048) {
    float v[8];
    load8<T>(xr + e, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float pr = __expf(v[j] - l);
      if (e + j == lb) pr -= 1.f;
      v[j] = pr * g;
    }
    store8<T>(dr + e, v);
  }
}

}  // namespace

PA_EXPORT int pa_softmax_fwd(const void* x, void* y, int64_t rows, int64_t cols, int dtype, hipStream_t st) {
  PA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((softmax_fwd_k<T>), dim3((unsigned)rows), dim3(256), 0, st,
                                                 (const T*)x, (T*)y, cols));
  PA_CHECK_LAUNCH();
  return 0;
}

PA_EXPORT int pa_softmax_bwd(const void* y, const void* dy, void* dx, int64_t rows, int64_t cols, int dtype,
                             hipStream_t st) {
  PA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((softmax_bwd_k<T>), dim3((unsigned)rows), dim3(256), 0, st,
                                                 (const T*)y, (const T*)dy, (T*)dx, cols));
  PA_CHECK_LAUNCH();
  return 0;
}

PA_EXPORT int pa_softmax_ce_fwd(const void* logits, const int64_t* labels, float* loss, float* lse, int64_t rows,
                                int64_t cols, int64_t ignore_index, int dtype, hipStream_t st) {
  PA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((softmax_ce_fwd_k<T>), dim3((unsigned)rows), dim3(256), 0, st,
                                                 (const T*)logits, labels, loss, lse, cols, ignore_index));
  PA_CHECK_LAUNCH();
  return 0;
}

PA_EXPORT int pa_softmax_ce_bwd(const void* logits, const int64_t* labels, const float* lse, const float* dloss,
                                void* dlogits, int64_t rows, int64_t cols, int64_t ignore_index, int dtype,
                                hipStream_t st) {
  PA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((softmax_ce_bwd_k<T>), dim3((unsigned)rows), dim3(256), 0, st,
                                                 (const T*)logits, labels, lse, dloss, (T*)dlogits, cols,
                                                 ignore_index));
  PA_CHECK_LAUNCH();
  return 0;
}

PA_EXPORT int pa_ce_slice_fwd(const void* logits, const int64_t* labels, float* lse, float* tgt, int64_t rows,
                              int64_t cols, int64_t v0, int dtype, hipStream_t st) {
  if (rows <= 0) return 0;
  PA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((ce_slice_fwd_k<T>), dim3((unsigned)rows), dim3(256), 0, st,
                                                 (const T*)logits, labels, lse, tgt, cols, v0));
  PA_CHECK_LAUNCH();
  return 0;
}

PA_EXPORT int pa_ce_slice_bwd(const void* logits, const int64_t* labels, const float* lse, const float* dloss,
                              void* dlogits, int64_t rows, int64_t cols, int64_t v0, int64_t ignore_index, int dtype,
                              hipStream_t st) {
  if (rows <= 0) return 0;
  PA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((ce_slice_bwd_k<T>), dim3((unsigned)rows), dim3(256), 0, st,
                                                 (const T*)logits, labels, lse, dloss, (T*)dlogits, cols, v0,
                                                 ignore_index));
  PA_CHECK_LAUNCH();
  return 0;
}
