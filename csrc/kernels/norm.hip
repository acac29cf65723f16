// RMSNorm / LayerNorm forward + backward for gfx950.
// Reference behaviour: paddle/phi/kernels/gpu/{rms_norm,layer_norm}_kernel.cu (+_grad).
//
// Layout: x [rows, cols] row-major, cols % 8 == 0. fp32 statistics (mean / rstd per row).
// Row kernels: one 64-lane wave per row, 4 rows per 256-thread workgroup, each lane keeps VPL
// 16-byte vectors of its row in registers (so the row is read from HBM exactly once);
// rows of more than 3072 columns use a workgroup-per-row two-pass kernel (faster in the step, see norm_fwd_wide).
// Weight/bias gradients are column reductions done by a separate coalesced kernel that writes
// fp32 partials [nparts, cols] (summed on the host side by one tiny reduction) — no atomics.
#include "common.h"

using namespace pa;

namespace {

template <typename T, int VPL, bool LN>
__global__ __launch_bounds__(256) void norm_fwd_rows(const T* __restrict__ x, const T* __restrict__ w,
                                                     const T* __restrict__ b, T* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int64_t rows, int64_t cols, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* xr = x + row * cols;
  // LayerNorm: the mean is summed about the row's first element, so rows with a large mean keep their digits
  const float sh = LN ? to_f(xr[0]) : 0.f;
  float v[VPL][8];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    const int64_t e = ((int64_t)k * 64 + lane) * 8;
    if (e < cols) {
      load8<T>(xr + e, v[k]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[k][j] = LN ? sh : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += LN ? v[k][j] - sh : v[k][j] * v[k][j];
  }
  s = wave_sum(s);
  const float inv_n = 1.0f / (float)cols;
  float mu = 0.f, rstd;
  if (LN) {
    mu = sh + s * inv_n;
    float s2 = 0.f;
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
      const int64_t e = ((int64_t)k * 64 + lane) * 8;
      if (e < cols) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { float d = v[k][j] - mu; s2 += d * d; }
      }
    }
    s2 = wave_sum(s2);
    rstd = rsqrtf(s2 * inv_n + eps);
  } else {
    rstd = rsqrtf(s * inv_n + eps);
  }
  if (lane == 0) {
    if (LN) mean_out[row] = mu;
    rstd_out[row] = rstd;
  }
  T* yr = y + row * cols;
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    const int64_t e = ((int64_t)k * 64 + lane) * 8;
    if (e < cols) {
      float o[8], wv[8], bv[8];
      if (w) load8<T>(w + e, wv); else {
#pragma unroll
        for (int j = 0; j < 8; ++j) wv[j] = 1.f;
      }
      if (LN && b) load8<T>(b + e, bv); else {
#pragma unroll
        for (int j = 0; j < 8; ++j) bv[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[k][j] - mu) * rstd * wv[j] + bv[j];
      store8<T>(yr + e, o);
    }
  }
}

// wide rows (>= 4096 columns): one 256-thread workgroup per row, two passes over global (the second hits L2).
// Measured in the GPT-3 13B step (5120 columns, operands from HBM): forward 19.5 vs 22.5 us, data gradient 38.8 vs
// 48.0 us for the wave-per-row kernels (`profiles/norm_rows_vs_wide_r4.md`): a whole workgroup's loads per row in
// flight instead of one wave's. LayerNorm sums are taken about the row's first element (shifted moments) so the
// one-pass variance does not cancel for rows with a large mean.
template <typename T, bool LN>
__global__ __launch_bounds__(256) void norm_fwd_wide(const T* __restrict__ x, const T* __restrict__ w,
                                                     const T* __restrict__ b, T* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int64_t rows, int64_t cols, float eps) {
  __shared__ float red[4];
  const int64_t row = blockIdx.x;
  const T* xr = x + row * cols;
  const float sh = LN ? to_f(xr[0]) : 0.f;
  float s = 0.f, s2 = 0.f;
  for (int64_t e = (int64_t)threadIdx.x * 8; e < cols; e += 256 * 8) {
    float v[8];
    load8<T>(xr + e, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) { const float d = v[j] - sh; s += d; s2 += d * d; }
  }
  const float inv_n = 1.0f / (float)cols;
  float mu = 0.f, rstd;
  if (LN) {
    s = block_sum<256>(s, red);
    s2 = block_sum<256>(s2, red);
    const float md = s * inv_n;
    mu = sh + md;
    rstd = rsqrtf(fmaxf(s2 * inv_n - md * md, 0.f) + eps);
  } else {
    s2 = block_sum<256>(s2, red);
    rstd = rsqrtf(s2 * inv_n + eps);
  }
  if (threadIdx.x == 0) {
    if (LN) mean_out[row] = mu;
    rstd_out[row] = rstd;
  }
  T* yr = y + row * cols;
  for (int64_t e = (int64_t)threadIdx.x * 8; e < cols; e += 256 * 8) {
    float v[8], wv[8], bv[8], o[8];
    load8<T>(xr + e, v);
    if (w) load8<T>(w + e, wv); else for (int j = 0; j < 8; ++j) wv[j] = 1.f;
    if (LN && b) load8<T>(b + e, bv); else for (int j = 0; j < 8; ++j) bv[j] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (v[j] - mu) * rstd * wv[j] + bv[j];
    store8<T>(yr + e, o);
  }
}

// dx for one row per wave. LN: dx = rstd*(g - mean(g) - xhat*mean(g*xhat)); RMS: drop mean(g).
template <typename T, int VPL, bool LN>
__global__ __launch_bounds__(256) void norm_bwd_dx_rows(const T* __restrict__ dy, const T* __restrict__ x,
                                                        const T* __restrict__ w, const float* __restrict__ mean,
                                                        const float* __restrict__ rstd, T* __restrict__ dx,
                                                        int64_t rows, int64_t cols, const T* __restrict__ res) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float mu = LN ? mean[row] : 0.f;
  const float rs = rstd[row];
  float xh[VPL][8], g[VPL][8];
  float sg = 0.f, sgx = 0.f;
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    const int64_t e = ((int64_t)k * 64 + lane) * 8;
    if (e < cols) {
      float xv[8], dv[8], wv[8];
      load8<T>(x + row * cols + e, xv);
      load8<T>(dy + row * cols + e, dv);
      if (w) load8<T>(w + e, wv); else for (int j = 0; j < 8; ++j) wv[j] = 1.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        xh[k][j] = (xv[j] - mu) * rs;
        g[k][j] = dv[j] * wv[j];
        sg += g[k][j];
        sgx += g[k][j] * xh[k][j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) { xh[k][j] = 0.f; g[k][j] = 0.f; }
    }
  }
  const float inv_n = 1.0f / (float)cols;
  sgx = wave_sum(sgx) * inv_n;
  sg = LN ? wave_sum(sg) * inv_n : 0.f;
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    const int64_t e = ((int64_t)k * 64 + lane) * 8;
    if (e < cols) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = rs * (g[k][j] - sg - xh[k][j] * sgx);
      if (res) {  // + the residual branch's gradient of the same input (fused residual add)
        float rv[8];
        load8<T>(res + row * cols + e, rv);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] += rv[j];
      }
      store8<T>(dx + row * cols + e, o);
    }
  }
}

template <typename T, bool LN>
__global__ __launch_bounds__(256) void norm_bwd_dx_wide(const T* __restrict__ dy, const T* __restrict__ x,
                                                        const T* __restrict__ w, const float* __restrict__ mean,
                                                        const float* __restrict__ rstd, T* __restrict__ dx,
                                                        int64_t rows, int64_t cols, const T* __restrict__ res) {
  __shared__ float red[4];
  const int64_t row = blockIdx.x;
  const float mu = LN ? mean[row] : 0.f;
  const float rs = rstd[row];
  float sg = 0.f, sgx = 0.f;
  for (int64_t e = (int64_t)threadIdx.x * 8; e < cols; e += 2048) {
    float xv[8], dv[8], wv[8];
    load8<T>(x + row * cols + e, xv);
    load8<T>(dy + row * cols + e, dv);
    if (w) load8<T>(w + e, wv); else for (int j = 0; j < 8; ++j) wv[j] = 1.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) { float gg = dv[j] * wv[j]; sg += gg; sgx += gg * (xv[j] - mu) * rs; }
  }
  const float inv_n = 1.0f / (float)cols;
  sgx = block_sum<256>(sgx, red) * inv_n;
  sg = LN ? block_sum<256>(sg, red) * inv_n : 0.f;
  for (int64_t e = (int64_t)threadIdx.x * 8; e < cols; e += 2048) {
    float xv[8], dv[8], wv[8], o[8];
    load8<T>(x + row * cols + e, xv);
    load8<T>(dy + row * cols + e, dv);
    if (w) load8<T>(w + e, wv); else for (int j = 0; j < 8; ++j) wv[j] = 1.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = rs * (dv[j] * wv[j] - sg - (xv[j] - mu) * rs * sgx);
    if (res) {
      float rv[8];
      load8<T>(res + row * cols + e, rv);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] += rv[j];
    }
    store8<T>(dx + row * cols + e, o);
  }
}

// column partial sums: dw_part[p, c] = sum_{rows r ≡ p mod nparts} dy*xhat ; db_part likewise with dy.
template <typename T, bool LN>
__global__ __launch_bounds__(256) void norm_bwd_wb(const T* __restrict__ dy, const T* __restrict__ x,
                                                   const float* __restrict__ mean, const float* __restrict__ rstd,
                                                   float* __restrict__ dw_part, float* __restrict__ db_part,
                                                   int64_t rows, int64_t cols, int nparts) {
  const int64_t c = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  const int p = blockIdx.y;
  if (c >= cols) return;
  float aw[8] = {0, 0, 0, 0, 0, 0, 0, 0}, ab[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t r = p; r < rows; r += nparts) {
    float xv[8], dv[8];
    load8<T>(x + r * cols + c, xv);
    load8<T>(dy + r * cols + c, dv);
    const float mu = LN ? mean[r] : 0.f;
    const float rs = rstd[r];
#pragma unroll
    for (int j = 0; j < 8; ++j) { aw[j] += dv[j] * (xv[j] - mu) * rs; ab[j] += dv[j]; }
  }
  store8<float>(dw_part + (int64_t)p * cols + c, aw);
  if (db_part) store8<float>(db_part + (int64_t)p * cols + c, ab);
}

template <typename T, bool LN>
int launch_fwd(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd, int64_t rows,
               int64_t cols, float eps, hipStream_t st) {
  const int64_t vpl = cdiv(cols, 512);
  dim3 grid((unsigned)cdiv(rows, 4)), block(256);
  auto X = (const T*)x; auto W = (const T*)w; auto B = (const T*)b; auto Y = (T*)y;
#define PA_FWD(V) hipLaunchKernelGGL((norm_fwd_rows<T, V, LN>), grid, block, 0, st, X, W, B, Y, mean, rstd, rows, cols, eps)
  if (vpl <= 1) PA_FWD(1);
  else if (vpl <= 2) PA_FWD(2);
  else if (vpl <= 3) PA_FWD(3);
  else if (vpl <= 4) PA_FWD(4);
  else if (vpl <= 6) PA_FWD(6);
  else hipLaunchKernelGGL((norm_fwd_wide<T, LN>), dim3((unsigned)rows), block, 0, st, X, W, B, Y, mean, rstd, rows, cols, eps);
#undef PA_FWD
  PA_CHECK_LAUNCH();
  return 0;
}

template <typename T, bool LN>
int launch_bwd(const void* dy, const void* x, const void* w, const float* mean, const float* rstd, void* dx,
               float* dw_part, float* db_part, int64_t rows, int64_t cols, int nparts, hipStream_t st,
               const void* res = nullptr) {
  const int64_t vpl = cdiv(cols, 512);
  dim3 grid((unsigned)cdiv(rows, 4)), block(256);
  auto DY = (const T*)dy; auto X = (const T*)x; auto W = (const T*)w; auto DX = (T*)dx; auto RES = (const T*)res;
#define PA_BWD(V) hipLaunchKernelGGL((norm_bwd_dx_rows<T, V, LN>), grid, block, 0, st, DY, X, W, mean, rstd, DX, rows, cols, RES)
  if (vpl <= 1) PA_BWD(1);
  else if (vpl <= 2) PA_BWD(2);
  else if (vpl <= 3) PA_BWD(3);
  else if (vpl <= 4) PA_BWD(4);
  else if (vpl <= 6) PA_BWD(6);
  else hipLaunchKernelGGL((norm_bwd_dx_wide<T, LN>), dim3((unsigned)rows), block, 0, st, DY, X, W, mean, rstd, DX, rows, cols,
                          RES);
#undef PA_BWD
  PA_CHECK_LAUNCH();
  if (dw_part) {
    dim3 g2((unsigned)cdiv(cols, 2048), (unsigned)nparts);
    hipLaunchKernelGGL((norm_bwd_wb<T, LN>), g2, block, 0, st, DY, X, mean, rstd, dw_part, db_part, rows, cols, nparts);
    PA_CHECK_LAUNCH();
  }
  return 0;
}

}  // namespace

PA_EXPORT int pa_rms_norm_fwd(const void* x, const void* w, void* y, float* rstd, int64_t rows, int64_t cols,
                              float eps, int dtype, hipStream_t st) {
  PA_DISPATCH_DTYPE(dtype, T, return (launch_fwd<T, false>(x, w, nullptr, y, nullptr, rstd, rows, cols, eps, st)));
  return 0;
}

PA_EXPORT int pa_rms_norm_bwd(const void* dy, const void* x, const void* w, const float* rstd, void* dx,
                              float* dw_part, int64_t rows, int64_t cols, int dtype_np, hipStream_t st) {
  const int dtype = dtype_np & 0xff, nparts = dtype_np >> 8;
  PA_DISPATCH_DTYPE(dtype, T,
                    return (launch_bwd<T, false>(dy, x, w, nullptr, rstd, dx, w ? dw_part : nullptr, nullptr, rows,
                                                 cols, nparts > 0 ? nparts : 1, st)));
  return 0;
}

// RMSNorm backward with the residual branch's gradient summed into dx (dx = d rms_norm / dx + res): the pre-norm
// block's x feeds both the norm and the residual add, so this replaces autograd's separate accumulation add.
PA_EXPORT int pa_rms_norm_bwd_res(const void* dy, const void* x, const void* w, const float* rstd, void* dx,
                                  float* dw_part, void* res, int64_t rows, int64_t cols, int dtype_np,
                                  hipStream_t st) {
  const int dtype = dtype_np & 0xff, nparts = dtype_np >> 8;
  PA_DISPATCH_DTYPE(dtype, T,
                    return (launch_bwd<T, false>(dy, x, w, nullptr, rstd, dx, w ? dw_part : nullptr, nullptr, rows,
                                                 cols, nparts > 0 ? nparts : 1, st, res)));
  return 0;
}

PA_EXPORT int pa_layer_norm_fwd(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd,
                                int64_t rows, int64_t cols, float eps, int dtype, hipStream_t st) {
  PA_DISPATCH_DTYPE(dtype, T, return (launch_fwd<T, true>(x, w, b, y, mean, rstd, rows, cols, eps, st)));
  return 0;
}

// res (nullable): [rows, cols] gradient of the same input from a residual branch, added into dx in the pass.
PA_EXPORT int pa_layer_norm_bwd(const void* dy, const void* x, const void* w, const float* mean, const float* rstd,
                                void* dx, float* dw_part, float* db_part, void* res, int64_t rows, int64_t cols,
                                int dtype_np, hipStream_t st) {
  const int dtype = dtype_np & 0xff, nparts = dtype_np >> 8;
  PA_DISPATCH_DTYPE(dtype, T,
                    return (launch_bwd<T, true>(dy, x, w, mean, rstd, dx, dw_part, db_part, rows, cols,
                                                nparts > 0 ? nparts : 1, st, res)));
  return 0;
}

// Weight / bias gradient finalize of the norm backwards in one launch: out_a[c] = sum_p part_a[p][c],
// out_b[c] = sum_p part_b[p][c] (part_b / out_b may be null), written in the parameters' dtypes. Bit 8 of a
// dtype code accumulates into that output (out += sum: the parameter's .grad buffer) instead of overwriting it.
// Block = 64 columns x 4 part groups, folded through LDS; grid (cols / 64, 2).
__global__ __launch_bounds__(256) void reduce_parts_k(const float* __restrict__ pa, const float* __restrict__ pb,
                                                      void* oa, void* ob, int nparts, int64_t cols, int dta, int dtb) {
  const float* part = blockIdx.y == 0 ? pa : pb;
  void* out = blockIdx.y == 0 ? oa : ob;
  const int dtc = blockIdx.y == 0 ? dta : dtb;
  const int dt = dtc & 0xff;
  const bool accum = (dtc >> 8) & 1;
  if (part == nullptr || out == nullptr) return;
  const int cx = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 64 + cx;
  float acc = 0.f;
  if (c < cols) {
#pragma unroll 8
    for (int p = g; p < nparts; p += 4) acc += part[(int64_t)p * cols + c];
  }
  __shared__ float sm[4][64];
  sm[g][cx] = acc;
  __syncthreads();
  if (g == 0 && c < cols) {
    float v = sm[0][cx] + sm[1][cx] + sm[2][cx] + sm[3][cx];
    if (dt == kF32) {
      float* o = reinterpret_cast<float*>(out);
      o[c] = accum ? o[c] + v : v;
    } else if (dt == kBF16) {
      bf16* o = reinterpret_cast<bf16*>(out);
      o[c] = from_f<bf16>(accum ? to_f(o[c]) + v : v);
    } else {
      f16* o = reinterpret_cast<f16*>(out);
      o[c] = from_f<f16>(accum ? to_f(o[c]) + v : v);
    }
  }
}

PA_EXPORT int pa_reduce_parts(const float* pa, const float* pb, void* oa, void* ob, int nparts, int64_t cols, int dta,
                              int dtb, hipStream_t st) {
  hipLaunchKernelGGL(reduce_parts_k, dim3((unsigned)((cols + 63) / 64), 2), dim3(256), 0, st, pa, pb, oa, ob, nparts,
                     cols, dta, dtb);
  PA_CHECK_LAUNCH();
  return 0;
}

PA_EXPORT int pa_version() { return 1; }
