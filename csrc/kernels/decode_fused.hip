// Fused inference kernels for the decoder step (LLaMA family), gfx950.
//
// Reference behaviour: paddle/phi/kernels/fusion/gpu/fused_bias_residual_layernorm (residual add + RMSNorm
// in one pass: incubate.nn.functional.fused_rms_norm with `residual`), fusion/gpu/fused_rope_kernel.cu and
// the cache write of masked_multihead_attention / block_multihead_attention (write_cache_kv).
//
// add_rms_norm_k: s = x + r (rounded to the storage type, as the unfused add would), y = s * rstd(s) * w.
//   One 64-lane wave per row, the row held in registers (read once, written twice). s may alias x.
// decode_rope_cache_k: the QKV projection output of one token per sequence, [B, (H + 2*Hkv) * D], is
//   rotated (NeoX halves) and split in one pass: rotated Q -> q_out [B, H, D]; rotated K and V -> the dense
//   caches [Bc, Hkv, Lc, D] at the device-side position *pos (no host read: hipGraph-capturable).
#include "common.h"

using namespace pa;

namespace {

inline unsigned launch_grid(int64_t items) {
  const int64_t g = (items + 255) / 256;
  return (unsigned)(g < 8192 ? (g > 0 ? g : 1) : 8192);
}

template <typename T, int VPL>
__global__ __launch_bounds__(256) void add_rms_norm_k(const T* x, const T* __restrict__ r,
                                                      const T* __restrict__ w, T* s_out, T* __restrict__ y,
                                                      int64_t rows, int64_t cols, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float v[VPL][8];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    const int64_t e = ((int64_t)k * 64 + lane) * 8;
    if (e < cols) {
      float a[8], b[8];
      load8<T>(x + row * cols + e, a);
      load8<T>(r + row * cols + e, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[k][j] = to_f(from_f<T>(a[j] + b[j]));  // the rounded sum, as add-then-norm
      store8<T>(s_out + row * cols + e, v[k]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[k][j] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += v[k][j] * v[k][j];
  }
  ss = wave_sum(ss);
  const float rstd = rsqrtf(ss / (float)cols + eps);
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    const int64_t e = ((int64_t)k * 64 + lane) * 8;
    if (e < cols) {
      float wv[8], o[8];
      load8<T>(w + e, wv);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[k][j] * rstd * wv[j];
      store8<T>(y + row * cols + e, o);
    }
  }
}

// Few rows (a decode step: one row per sequence): one 256-thread workgroup per row, so a 32-row call
// spreads over 32 CUs instead of 8 and each lane has at most 4 vectors in flight.
template <typename T, int VPT>
__global__ __launch_bounds__(256) void add_rms_norm_wg_k(const T* x, const T* __restrict__ r,
                                                         const T* __restrict__ w, T* s_out, T* __restrict__ y,
                                                         int64_t cols, float eps) {
  const int64_t row = blockIdx.x;
  const int tid = threadIdx.x;
  float v[VPT][8];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int64_t e = ((int64_t)k * 256 + tid) * 8;
    if (e < cols) {
      float a[8], b[8];
      load8<T>(x + row * cols + e, a);
      load8<T>(r + row * cols + e, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[k][j] = to_f(from_f<T>(a[j] + b[j]));
      store8<T>(s_out + row * cols + e, v[k]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[k][j] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += v[k][j] * v[k][j];
  }
  __shared__ float part[4];
  ss = wave_sum(ss);
  if ((tid & 63) == 0) part[tid >> 6] = ss;
  __syncthreads();
  const float rstd = rsqrtf((part[0] + part[1] + part[2] + part[3]) / (float)cols + eps);
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int64_t e = ((int64_t)k * 256 + tid) * 8;
    if (e < cols) {
      float wv[8], o[8];
      load8<T>(w + e, wv);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[k][j] * rstd * wv[j];
      store8<T>(y + row * cols + e, o);
    }
  }
}

// work item: (b, head, 8-lane chunk). Q and K heads: NeoX rotation of 8 elements of the first half and the
// matching 8 of the second half; V heads: a copy of 8 elements.
template <typename T>
__global__ __launch_bounds__(256) void decode_rope_cache_k(const T* __restrict__ qkv, int64_t ld,
                                                           const float* __restrict__ cs, const float* __restrict__ sn,
                                                           const int64_t* __restrict__ pos, T* __restrict__ q_out,
                                                           T* __restrict__ kc, T* __restrict__ vc, int B, int H,
                                                           int Hkv, int D, int64_t Lc) {
  const int rot = D / 16, cp = D / 8;
  const int per_b = (H + Hkv) * rot + Hkv * cp;
  const int64_t n = (int64_t)B * per_b;
  const int64_t p = *pos;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int b = (int)(i / per_b);
    int t = (int)(i % per_b);
    const T* row = qkv + (int64_t)b * ld;
    if (t < (H + Hkv) * rot) {
      const int head = t / rot, k = t % rot;
      const int d0 = k * 8, d1 = d0 + D / 2;
      const T* src = row + (int64_t)head * D;  // q heads then k heads are contiguous in the row
      float a[8], c[8], oa[8], ob[8];
      load8<T>(src + d0, a);
      load8<T>(src + d1, c);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        oa[j] = a[j] * cs[d0 + j] - c[j] * sn[d0 + j];
        ob[j] = c[j] * cs[d1 + j] + a[j] * sn[d1 + j];
      }
      T* dst;
      if (head < H) {
        dst = q_out + ((int64_t)b * H + head) * D;
      } else {
        dst = kc + (((int64_t)b * Hkv + (head - H)) * Lc + p) * D;
      }
      store8<T>(dst + d0, oa);
      store8<T>(dst + d1, ob);
    } else {
      t -= (H + Hkv) * rot;
      const int head = t / cp, k = t % cp;
      float a[8];
      load8<T>(row + (int64_t)(H + Hkv + head) * D + k * 8, a);
      store8<T>(vc + (((int64_t)b * Hkv + head) * Lc + p) * D + k * 8, a);
    }
  }
}

}  // namespace

PA_EXPORT int pa_add_rms_norm_fwd(const void* x, const void* r, const void* w, void* s_out, void* y, int64_t rows,
                                  int64_t cols, float eps, int dtype, hipStream_t st) {
  if (cols % 8 != 0 || cols > 64 * 8 * 16) return 2;
  if (rows < 256) {
    const int vpt = (int)((cols / 8 + 255) / 256);
#define PA_ARNW(V) hipLaunchKernelGGL((add_rms_norm_wg_k<T, V>), dim3((unsigned)rows), dim3(256), 0, st, (const T*)x, \
                                      (const T*)r, (const T*)w, (T*)s_out, (T*)y, cols, eps)
    if (vpt <= 1) {
      PA_DISPATCH_DTYPE(dtype, T, PA_ARNW(1));
    } else if (vpt <= 2) {
      PA_DISPATCH_DTYPE(dtype, T, PA_ARNW(2));
    } else {
      PA_DISPATCH_DTYPE(dtype, T, PA_ARNW(4));
    }
#undef PA_ARNW
    PA_CHECK_LAUNCH();
    return 0;
  }
  const dim3 grid((unsigned)((rows + 3) / 4)), block(256);
#define PA_ARN(V) hipLaunchKernelGGL((add_rms_norm_k<T, V>), grid, block, 0, st, (const T*)x, (const T*)r, \
                                     (const T*)w, (T*)s_out, (T*)y, rows, cols, eps)
  const int vpl = (int)((cols / 8 + 63) / 64);
  if (vpl <= 2) {
    PA_DISPATCH_DTYPE(dtype, T, PA_ARN(2));
  } else if (vpl <= 4) {
    PA_DISPATCH_DTYPE(dtype, T, PA_ARN(4));
  } else if (vpl <= 8) {
    PA_DISPATCH_DTYPE(dtype, T, PA_ARN(8));
  } else {
    PA_DISPATCH_DTYPE(dtype, T, PA_ARN(16));
  }
#undef PA_ARN
  PA_CHECK_LAUNCH();
  return 0;
}

PA_EXPORT int pa_decode_rope_cache(const void* qkv, int64_t ld, const float* cs, const float* sn, const int64_t* pos,
                                   void* q_out, void* kc, void* vc, int B, int H, int Hkv, int D, int64_t Lc, int dtype,
                                   hipStream_t st) {
  if (D % 16 != 0) return 2;
  const int64_t n = (int64_t)B * ((H + Hkv) * (D / 16) + Hkv * (D / 8));
  PA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((decode_rope_cache_k<T>), dim3(launch_grid(n)), dim3(256), 0, st,
                                                 (const T*)qkv, ld, cs, sn, pos, (T*)q_out, (T*)kc, (T*)vc, B, H, Hkv,
                                                 D, Lc));
  PA_CHECK_LAUNCH();
  return 0;
}
