// Batch norm over channels-last (NHWC / [rows, C]) activations with the activation and residual add
// fused in, for gfx950. Reference behaviour: paddle/phi/kernels/gpu/batch_norm_kernel.cu (training
// statistics, biased variance in the running average with factor 1 - momentum),
// batch_norm_grad_kernel.cu, and fusion/gpu/fused_bn_add_activation (bn + add + relu).
//
// A ResNet BN layer is three HBM passes in each direction, so the design is purely about bytes:
//   fwd: stats (read x) -> tiny finalize -> apply (read x [+ residual], write y = act(bn(x) [+ r]))
//   bwd: reduce (read dy, x [, y for the relu mask]) -> tiny finalize -> apply (read dy, x [, y],
//        write dx [and d_residual = masked dy])
// The relu mask is recomputed from the saved output y (the next conv keeps y alive anyway), so no
// mask tensor is stored and the separate relu / add kernels disappear.
//
// Reductions are channel-parallel: a workgroup owns CB channels (8 per lane, one 16-byte load) and a
// contiguous row range; lanes along the rows keep fp32 partials, folded through LDS into per-(row
// chunk, channel) partials; the finalize kernel folds the chunks in fp64.
#include "common.h"

using namespace pa;

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ void ld8(const uint16_t* p, float* f) { load8<bf16>(reinterpret_cast<const bf16*>(p), f); }
__device__ __forceinline__ void st8(uint16_t* p, const float* f) { store8<bf16>(reinterpret_cast<bf16*>(p), f); }

// MODE 0: acc1 = sum x, acc2 = sum x^2.
// MODE 1: dyp = relu ? (y > 0 ? dy : 0) : dy; acc1 = sum dyp, acc2 = sum dyp * (x - mean).
// MASKX (with RELU, no residual in the forward): the relu mask is recomputed from x as
// x * scale + shift > 0 with the forward's scale / shift (ss), the same expression the forward applied,
// so y is not read (one tensor fewer in both backward passes).
// MASKB (with RELU): the relu mask comes from the forward's bit mask (one byte per 8 channels of a row,
// bn_apply_k WMASK) instead of y: 1/16 of y's bytes.
template <int MODE, bool RELU, bool MASKX = false, bool MASKB = false>
__global__ __launch_bounds__(kThreads) void bn_reduce_k(const uint16_t* __restrict__ x, const uint16_t* __restrict__ dy,
                                                        const uint16_t* __restrict__ y, const float* __restrict__ mean,
                                                        float* __restrict__ partial, int64_t R, int C, int CB,
                                                        int64_t rows_per_chunk, const float* __restrict__ ss = nullptr,
                                                        const uint8_t* __restrict__ mbits = nullptr) {
  const int tcx = CB >> 3;               // lanes along channels
  const int rpi = kThreads / tcx;        // rows per iteration
  const int tx = threadIdx.x % tcx, ty = threadIdx.x / tcx;
  const int c0 = blockIdx.x * CB + tx * 8;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
  const int64_t r1 = min(R, r0 + rows_per_chunk);
  float a1[8], a2[8], mu[8], sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { a1[j] = 0.f; a2[j] = 0.f; mu[j] = 0.f; sc[j] = 0.f; sh[j] = 0.f; }
  if (MODE == 1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) mu[j] = mean[c0 + j];
  }
  if (MASKX) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { sc[j] = ss[c0 + j]; sh[j] = ss[C + c0 + j]; }
  }
  // U rows per trip keep U 16-byte loads per tensor in flight (the stats pass reads one tensor)
  constexpr int U = MODE == 0 ? 4 : 2;
  int64_t r = r0 + ty;
  for (; r + (U - 1) * rpi < r1; r += U * rpi) {
    float xs[U][8], gs[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) ld8(x + (r + u * rpi) * C + c0, xs[u]);
    if (MODE == 1) {
#pragma unroll
      for (int u = 0; u < U; ++u) ld8(dy + (r + u * rpi) * C + c0, gs[u]);
      if (RELU && MASKX) {
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int j = 0; j < 8; ++j) gs[u][j] = xs[u][j] * sc[j] + sh[j] > 0.f ? gs[u][j] : 0.f;
      } else if (RELU && MASKB) {
        uint32_t mb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) mb[u] = mbits[((r + u * rpi) * C + c0) >> 3];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int j = 0; j < 8; ++j) gs[u][j] = (mb[u] >> j) & 1u ? gs[u][j] : 0.f;
      } else if (RELU) {
        float ys[U][8];
#pragma unroll
        for (int u = 0; u < U; ++u) ld8(y + (r + u * rpi) * C + c0, ys[u]);
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int j = 0; j < 8; ++j) gs[u][j] = ys[u][j] > 0.f ? gs[u][j] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (MODE == 0) {
          a1[j] += xs[u][j];
          a2[j] += xs[u][j] * xs[u][j];
        } else {
          a1[j] += gs[u][j];
          a2[j] += gs[u][j] * (xs[u][j] - mu[j]);
        }
      }
  }
  for (; r < r1; r += rpi) {
    float xa[8];
    ld8(x + r * C + c0, xa);
    if (MODE == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { a1[j] += xa[j]; a2[j] += xa[j] * xa[j]; }
    } else {
      float ga[8];
      ld8(dy + r * C + c0, ga);
      if (RELU && MASKX) {
#pragma unroll
        for (int j = 0; j < 8; ++j) ga[j] = xa[j] * sc[j] + sh[j] > 0.f ? ga[j] : 0.f;
      } else if (RELU && MASKB) {
        const uint32_t mb = mbits[(r * C + c0) >> 3];
#pragma unroll
        for (int j = 0; j < 8; ++j) ga[j] = (mb >> j) & 1u ? ga[j] : 0.f;
      } else if (RELU) {
        float ya[8];
        ld8(y + r * C + c0, ya);
#pragma unroll
        for (int j = 0; j < 8; ++j) ga[j] = ya[j] > 0.f ? ga[j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) { a1[j] += ga[j]; a2[j] += ga[j] * (xa[j] - mu[j]); }
    }
  }
  // fold the rpi row-lanes: sm[ty][channel] for each accumulator
  __shared__ float sm[2][kThreads * 8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sm[0][ty * CB + tx * 8 + j] = a1[j];
    sm[1][ty * CB + tx * 8 + j] = a2[j];
  }
  __syncthreads();
  for (int cc = threadIdx.x; cc < 2 * CB; cc += kThreads) {
    const int which = cc / CB, c = cc % CB;
    float s = 0.f;
    for (int t = 0; t < rpi; ++t) s += sm[which][t * CB + c];
    partial[((int64_t)which * gridDim.y + blockIdx.y) * C + blockIdx.x * CB + c] = s;
  }
}

// fold the chunk partials of 64 channels per 1024-thread block: lane (c, k) sums chunks k, k+16, ...
// (8 independent loads per trip — the fold is latency-bound, not bandwidth-bound) in fp64, then the
// 16 chunk-lanes combine through LDS. Result valid in threads with k == 0.
constexpr int kFoldLanes = 16;
__device__ __forceinline__ bool fold_chunks(const float* __restrict__ partial, int chunks, int C, double* s1,
                                            double* s2, int* c_out) {
  __shared__ double sm1[kFoldLanes][64], sm2[kFoldLanes][64];
  const int cl = threadIdx.x & 63, k = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  double a = 0.0, b = 0.0;
  if (c < C) {
    const float* p1 = partial + c;
    const float* p2 = partial + (int64_t)chunks * C + c;
    int j = k;
    for (; j + 7 * kFoldLanes < chunks; j += 8 * kFoldLanes) {
      float u[8], v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        u[q] = p1[(int64_t)(j + q * kFoldLanes) * C];
        v[q] = p2[(int64_t)(j + q * kFoldLanes) * C];
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) { a += u[q]; b += v[q]; }
    }
    for (; j < chunks; j += kFoldLanes) {
      a += p1[(int64_t)j * C];
      b += p2[(int64_t)j * C];
    }
  }
  sm1[k][cl] = a;
  sm2[k][cl] = b;
  __syncthreads();
  double t1 = 0.0, t2 = 0.0;
  if (k == 0) {
#pragma unroll
    for (int q = 0; q < kFoldLanes; ++q) { t1 += sm1[q][cl]; t2 += sm2[q][cl]; }
  }
  *s1 = t1;
  *s2 = t2;
  *c_out = c;
  return k == 0 && c < C;
}

// forward finalize: batch mean / rstd, running stats, fused scale / shift
__global__ __launch_bounds__(1024) void bn_fwd_finalize_k(const float* __restrict__ partial, int chunks, int C, int64_t R,
                                                         const float* __restrict__ w, const float* __restrict__ b,
                                                         float* __restrict__ run_mean, float* __restrict__ run_var,
                                                         float momentum, float eps, float* __restrict__ save_mean,
                                                         float* __restrict__ save_rstd, float* __restrict__ ss) {
  double s1, s2;
  int c;
  if (!fold_chunks(partial, chunks, C, &s1, &s2, &c)) return;
  const double m = s1 / (double)R;
  double var = s2 / (double)R - m * m;
  var = var > 0.0 ? var : 0.0;
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  save_mean[c] = (float)m;
  save_rstd[c] = rstd;
  if (run_mean) run_mean[c] = momentum * run_mean[c] + (1.f - momentum) * (float)m;
  if (run_var) run_var[c] = momentum * run_var[c] + (1.f - momentum) * (float)var;
  const float sc = (w ? w[c] : 1.f) * rstd;
  ss[c] = sc;
  ss[C + c] = (b ? b[c] : 0.f) - (float)m * sc;
}

// backward finalize: dweight / dbias and the per-channel dx coefficients
//   dx = a * dyp - bc * x + d0 with a = w * rstd, bc = a * rstd^2 * sum(dyp (x - mean)) / R,
//   d0 = bc * mean - a * sum(dyp) / R   (use_global_stats: bc = 0, d0 = 0)
__global__ __launch_bounds__(1024) void bn_bwd_finalize_k(const float* __restrict__ partial, int chunks, int C, int64_t R,
                                                         const float* __restrict__ w, const float* __restrict__ mean,
                                                         const float* __restrict__ rstd, float* __restrict__ dw,
                                                         float* __restrict__ db, float* __restrict__ coef,
                                                         int global_stats) {
  double s1, s2;
  int c;
  if (!fold_chunks(partial, chunks, C, &s1, &s2, &c)) return;
  const float rs = rstd[c];
  if (dw) dw[c] = (float)s2 * rs;
  if (db) db[c] = (float)s1;
  const float a = (w ? w[c] : 1.f) * rs;
  float bc = 0.f, d0 = 0.f;
  if (!global_stats) {
    bc = (float)((double)a * rs * rs * s2 / (double)R);
    d0 = bc * mean[c] - (float)((double)a * s1 / (double)R);
  }
  coef[c] = a;
  coef[C + c] = bc;
  coef[2 * C + c] = d0;
}

// The apply passes are grid-strided over 16-byte vectors (8 channels of one row). With the grid stride a multiple
// of C / 8 — kThreads = 256 is, for every C / 8 that divides 256 (C <= 2048, power of two) — a thread keeps the
// same 8 channels for its whole loop: the per-channel constants are loaded once into registers instead of with
// every vector (they were half the memory instructions of the loop), and two vectors per trip keep two 16-byte
// loads per stream in flight. Other C take the general loop.

// y = act(x * scale + shift [+ res]); WMASK: also the relu mask, bit j of byte i = (y[8i + j] > 0)
template <bool RELU, bool RES, bool WMASK>
__device__ __forceinline__ void bn_apply_vec(const float* f, const float* r, const float* sc, const float* sh,
                                             uint16_t* __restrict__ y, uint8_t* __restrict__ mbits, int64_t i) {
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float t = f[j] * sc[j] + sh[j];
    if (RES) t += r[j];
    if (RELU) t = fmaxf(t, 0.f);
    v[j] = t;
  }
  uint4 o;
  o.x = pack_bf16(v[0], v[1]); o.y = pack_bf16(v[2], v[3]); o.z = pack_bf16(v[4], v[5]); o.w = pack_bf16(v[6], v[7]);
  *reinterpret_cast<uint4*>(y + i * 8) = o;
  if (WMASK) {
    // the mask of the stored (bf16-rounded) value, the same test the y-reading backward applies
    const uint32_t ww[4] = {o.x, o.y, o.z, o.w};
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bits |= (lo_bf16(ww[j]) > 0.f ? 1u : 0u) << (2 * j);
      bits |= (hi_bf16(ww[j]) > 0.f ? 1u : 0u) << (2 * j + 1);
    }
    mbits[i] = (uint8_t)bits;
  }
}

template <bool RELU, bool RES, bool WMASK = false>
__global__ __launch_bounds__(kThreads) void bn_apply_k(const uint16_t* __restrict__ x, const uint16_t* __restrict__ res,
                                                       const float* __restrict__ ss, uint16_t* __restrict__ y,
                                                       int64_t nvec, int C, uint8_t* __restrict__ mbits = nullptr) {
  const int cv = C >> 3;
  const int64_t T = (int64_t)gridDim.x * kThreads;
  const int64_t i0 = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  float sc[8], sh[8], f0[8], f1[8], r0[8], r1[8];
  if (T % cv == 0) {
    const int c0 = (int)(i0 % cv) * 8;
    load8<float>(ss + c0, sc);
    load8<float>(ss + C + c0, sh);
    for (int64_t i = i0; i < nvec; i += 2 * T) {
      const bool two = i + T < nvec;
      ld8(x + i * 8, f0);
      if (two) ld8(x + (i + T) * 8, f1);
      if (RES) {
        ld8(res + i * 8, r0);
        if (two) ld8(res + (i + T) * 8, r1);
      }
      bn_apply_vec<RELU, RES, WMASK>(f0, r0, sc, sh, y, mbits, i);
      if (two) bn_apply_vec<RELU, RES, WMASK>(f1, r1, sc, sh, y, mbits, i + T);
    }
    return;
  }
  for (int64_t i = i0; i < nvec; i += T) {
    const int c0 = (int)(i % cv) * 8;
    ld8(x + i * 8, f0);
    if (RES) ld8(res + i * 8, r0);
    load8<float>(ss + c0, sc);
    load8<float>(ss + C + c0, sh);
    bn_apply_vec<RELU, RES, WMASK>(f0, r0, sc, sh, y, mbits, i);
  }
}

// dx = a * dyp - bc * x + d0; dres = dyp   (MASKX: relu mask from x * scale + shift, see bn_reduce_k)
template <bool RELU, bool DRES, bool MASKX, bool MASKB>
__device__ __forceinline__ void bn_bwd_vec(float* g, const float* f, const uint16_t* __restrict__ y,
                                           const uint8_t* __restrict__ mbits, const float* sc, const float* sh,
                                           const float* a, const float* bc, const float* d0,
                                           uint16_t* __restrict__ dx, uint16_t* __restrict__ dres, int64_t i) {
  if (RELU && MASKX) {
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = f[j] * sc[j] + sh[j] > 0.f ? g[j] : 0.f;
  } else if (RELU && MASKB) {
    const uint32_t mb = mbits[i];
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = (mb >> j) & 1u ? g[j] : 0.f;
  } else if (RELU) {
    float yy[8];
    ld8(y + i * 8, yy);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = yy[j] > 0.f ? g[j] : 0.f;
  }
  if (DRES) st8(dres + i * 8, g);
  float o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = a[j] * g[j] - bc[j] * f[j] + d0[j];
  st8(dx + i * 8, o);
}

template <bool RELU, bool DRES, bool MASKX = false, bool MASKB = false>
__global__ __launch_bounds__(kThreads) void bn_bwd_apply_k(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x,
                                                           const uint16_t* __restrict__ y, const float* __restrict__ coef,
                                                           uint16_t* __restrict__ dx, uint16_t* __restrict__ dres,
                                                           int64_t nvec, int C, const float* __restrict__ ss = nullptr,
                                                           const uint8_t* __restrict__ mbits = nullptr) {
  const int cv = C >> 3;
  const int64_t T = (int64_t)gridDim.x * kThreads;
  const int64_t i0 = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  float sc[8], sh[8], a[8], bc[8], d0[8], g0[8], g1[8], f0[8], f1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sc[j] = 0.f; sh[j] = 0.f; }
  if (T % cv == 0) {
    const int c0 = (int)(i0 % cv) * 8;
    if (RELU && MASKX) {
      load8<float>(ss + c0, sc);
      load8<float>(ss + C + c0, sh);
    }
    load8<float>(coef + c0, a);
    load8<float>(coef + C + c0, bc);
    load8<float>(coef + 2 * C + c0, d0);
    for (int64_t i = i0; i < nvec; i += 2 * T) {
      const bool two = i + T < nvec;
      ld8(dy + i * 8, g0);
      ld8(x + i * 8, f0);
      if (two) {
        ld8(dy + (i + T) * 8, g1);
        ld8(x + (i + T) * 8, f1);
      }
      bn_bwd_vec<RELU, DRES, MASKX, MASKB>(g0, f0, y, mbits, sc, sh, a, bc, d0, dx, dres, i);
      if (two) bn_bwd_vec<RELU, DRES, MASKX, MASKB>(g1, f1, y, mbits, sc, sh, a, bc, d0, dx, dres, i + T);
    }
    return;
  }
  for (int64_t i = i0; i < nvec; i += T) {
    const int c0 = (int)(i % cv) * 8;
    ld8(dy + i * 8, g0);
    ld8(x + i * 8, f0);
    if (RELU && MASKX) {
      load8<float>(ss + c0, sc);
      load8<float>(ss + C + c0, sh);
    }
    load8<float>(coef + c0, a);
    load8<float>(coef + C + c0, bc);
    load8<float>(coef + 2 * C + c0, d0);
    bn_bwd_vec<RELU, DRES, MASKX, MASKB>(g0, f0, y, mbits, sc, sh, a, bc, d0, dx, dres, i);
  }
}

int pick_cb(int C) {
  if (C % 512 == 0) return 512;
  if (C % 256 == 0) return 256;
  if (C % 128 == 0) return 128;
  if (C % 64 == 0) return 64;
  if (C % 32 == 0) return 32;
  if (C % 16 == 0) return 16;
  return 8;
}

// row chunking: ~512 workgroups over the chip (2 per CU, each lane with two 16-byte loads in
// flight per tensor), each at least 8 row-iterations deep; fewer chunks keep the fold cheap
int g_target_wgs = 512;  // reduction workgroups over the chip (pa_bn_set_target_wgs)

void plan(int64_t R, int C, int* CB, int* chunks, int64_t* rows_per_chunk) {
  *CB = pick_cb(C);
  const int rpi = kThreads / (*CB / 8);
  const int gx = C / *CB;
  int64_t want = g_target_wgs / gx;
  if (want < 1) want = 1;
  int64_t rpc = (R + want - 1) / want;
  const int64_t min_rows = 8 * rpi;
  if (rpc < min_rows) rpc = min_rows;
  rpc = (rpc + rpi - 1) / rpi * rpi;
  *rows_per_chunk = rpc;
  *chunks = (int)((R + rpc - 1) / rpc);
}

unsigned apply_grid(int64_t nvec) {
  int64_t g = (nvec + kThreads * 4 - 1) / (kThreads * 4);
  if (g > 8192) g = 8192;
  return (unsigned)(g < 1 ? 1 : g);
}

}  // namespace

// Tuning knob for the reduction grid (microbenchmarks); returns the previous value.
PA_EXPORT int pa_bn_set_target_wgs(int n) {
  const int old = g_target_wgs;
  if (n > 0) g_target_wgs = n;
  return old;
}

// Number of row chunks (partial workspace = 2 * chunks * C floats) for a reduction over [R, C].
PA_EXPORT int pa_bn_chunks(int64_t R, int C) {
  int CB, chunks;
  int64_t rpc;
  plan(R, C, &CB, &chunks, &rpc);
  return chunks;
}

// Training forward. x, res, y: [R, C] bf16 (res may be null); w, b, run_mean, run_var fp32 [C] (any
// may be null); partial: 2 * chunks * C fp32; save_mean, save_rstd: [C]; ss: [2, C] scale / shift.
// training = 0: save_mean / save_rstd are inputs (running stats already turned into mean / rstd).
PA_EXPORT int pa_bn_fwd_nhwc(const void* x, const void* res, void* y, const float* w, const float* b, float* run_mean,
                             float* run_var, float* save_mean, float* save_rstd, float* partial, float* ss, int64_t R,
                             int C, float momentum, float eps, int relu, int training, hipStream_t st) {
  if (C % 8 != 0 || R < 1) return 3;
  int CB, chunks;
  int64_t rpc;
  plan(R, C, &CB, &chunks, &rpc);
  if (training) {
    hipLaunchKernelGGL((bn_reduce_k<0, false>), dim3(C / CB, chunks), dim3(kThreads), 0, st, (const uint16_t*)x,
                       nullptr, nullptr, nullptr, partial, R, C, CB, rpc);
    PA_CHECK_LAUNCH();
    hipLaunchKernelGGL(bn_fwd_finalize_k, dim3((C + 63) / 64), dim3(1024), 0, st, partial, chunks, C, R, w, b,
                       run_mean, run_var, momentum, eps, save_mean, save_rstd, ss);
    PA_CHECK_LAUNCH();
  }
  const int64_t nvec = R * C / 8;
  const unsigned g = apply_grid(nvec);
#define PA_BN_APPLY(RL, RS)                                                                                      \
  hipLaunchKernelGGL((bn_apply_k<RL, RS>), dim3(g), dim3(kThreads), 0, st, (const uint16_t*)x, (const uint16_t*)res, \
                     ss, (uint16_t*)y, nvec, C)
  if (relu && res) PA_BN_APPLY(true, true);
  else if (relu) PA_BN_APPLY(true, false);
  else if (res) PA_BN_APPLY(false, true);
  else PA_BN_APPLY(false, false);
#undef PA_BN_APPLY
  PA_CHECK_LAUNCH();
  return 0;
}

// Backward. dy, x, y: [R, C] bf16 (y only read when relu); dx out; dres out (null: no residual
// gradient); dw, db fp32 [C] out (nullable); coef: [3, C] workspace; partial: 2 * chunks * C.
// ss: the forward's [2, C] scale / shift, given for relu without residual (mask from x, y not read).
PA_EXPORT int pa_bn_bwd_nhwc(const void* dy, const void* x, const void* y, void* dx, void* dres, const float* w,
                             const float* mean, const float* rstd, float* dw, float* db, float* partial, float* coef,
                             int64_t R, int C, int relu, int global_stats, const float* ss, hipStream_t st) {
  if (C % 8 != 0 || R < 1) return 3;
  int CB, chunks;
  int64_t rpc;
  plan(R, C, &CB, &chunks, &rpc);
  const bool maskx = relu && ss != nullptr;  // relu mask from x and the forward's scale / shift, y unused
  if (maskx)
    hipLaunchKernelGGL((bn_reduce_k<1, true, true>), dim3(C / CB, chunks), dim3(kThreads), 0, st, (const uint16_t*)x,
                       (const uint16_t*)dy, nullptr, mean, partial, R, C, CB, rpc, ss);
  else if (relu)
    hipLaunchKernelGGL((bn_reduce_k<1, true>), dim3(C / CB, chunks), dim3(kThreads), 0, st, (const uint16_t*)x,
                       (const uint16_t*)dy, (const uint16_t*)y, mean, partial, R, C, CB, rpc);
  else
    hipLaunchKernelGGL((bn_reduce_k<1, false>), dim3(C / CB, chunks), dim3(kThreads), 0, st, (const uint16_t*)x,
                       (const uint16_t*)dy, nullptr, mean, partial, R, C, CB, rpc);
  PA_CHECK_LAUNCH();
  hipLaunchKernelGGL(bn_bwd_finalize_k, dim3((C + 63) / 64), dim3(1024), 0, st, partial, chunks, C, R, w, mean, rstd,
                     dw, db, coef, global_stats);
  PA_CHECK_LAUNCH();
  const int64_t nvec = R * C / 8;
  const unsigned g = apply_grid(nvec);
#define PA_BN_BWD(RL, DR)                                                                                         \
  hipLaunchKernelGGL((bn_bwd_apply_k<RL, DR>), dim3(g), dim3(kThreads), 0, st, (const uint16_t*)dy,                \
                     (const uint16_t*)x, (const uint16_t*)y, coef, (uint16_t*)dx, (uint16_t*)dres, nvec, C)
  if (maskx) {
    hipLaunchKernelGGL((bn_bwd_apply_k<true, false, true>), dim3(g), dim3(kThreads), 0, st, (const uint16_t*)dy,
                       (const uint16_t*)x, nullptr, coef, (uint16_t*)dx, nullptr, nvec, C, ss);
  } else if (relu && dres) PA_BN_BWD(true, true);
  else if (relu) PA_BN_BWD(true, false);
  else if (dres) PA_BN_BWD(false, true);
  else PA_BN_BWD(false, false);
#undef PA_BN_BWD
  PA_CHECK_LAUNCH();
  return 0;
}

// Residual + relu variants that keep a bit mask of the relu instead of re-reading y in the backward
// (mbits: R * C / 8 bytes). Forward: bn_apply writes y and the mask; backward: both passes read the mask.
PA_EXPORT int pa_bn_fwd_nhwc_mask(const void* x, const void* res, void* y, const float* w, const float* b,
                                  float* run_mean, float* run_var, float* save_mean, float* save_rstd, float* partial,
                                  float* ss, void* mbits, int64_t R, int C, float momentum, float eps, int training,
                                  hipStream_t st) {
  if (C % 8 != 0 || R < 1 || !mbits) return 3;
  int CB, chunks;
  int64_t rpc;
  plan(R, C, &CB, &chunks, &rpc);
  if (training) {
    hipLaunchKernelGGL((bn_reduce_k<0, false>), dim3(C / CB, chunks), dim3(kThreads), 0, st, (const uint16_t*)x,
                       nullptr, nullptr, nullptr, partial, R, C, CB, rpc);
    PA_CHECK_LAUNCH();
    hipLaunchKernelGGL(bn_fwd_finalize_k, dim3((C + 63) / 64), dim3(1024), 0, st, partial, chunks, C, R, w, b,
                       run_mean, run_var, momentum, eps, save_mean, save_rstd, ss);
    PA_CHECK_LAUNCH();
  }
  const int64_t nvec = R * C / 8;
  if (res)
    hipLaunchKernelGGL((bn_apply_k<true, true, true>), dim3(apply_grid(nvec)), dim3(kThreads), 0, st,
                       (const uint16_t*)x, (const uint16_t*)res, ss, (uint16_t*)y, nvec, C, (uint8_t*)mbits);
  else
    hipLaunchKernelGGL((bn_apply_k<true, false, true>), dim3(apply_grid(nvec)), dim3(kThreads), 0, st,
                       (const uint16_t*)x, nullptr, ss, (uint16_t*)y, nvec, C, (uint8_t*)mbits);
  PA_CHECK_LAUNCH();
  return 0;
}

PA_EXPORT int pa_bn_bwd_nhwc_mask(const void* dy, const void* x, const void* mbits, void* dx, void* dres,
                                  const float* w, const float* mean, const float* rstd, float* dw, float* db,
                                  float* partial, float* coef, int64_t R, int C, int global_stats, hipStream_t st) {
  if (C % 8 != 0 || R < 1 || !mbits) return 3;
  int CB, chunks;
  int64_t rpc;
  plan(R, C, &CB, &chunks, &rpc);
  const uint8_t* mb = (const uint8_t*)mbits;
  hipLaunchKernelGGL((bn_reduce_k<1, true, false, true>), dim3(C / CB, chunks), dim3(kThreads), 0, st,
                     (const uint16_t*)x, (const uint16_t*)dy, nullptr, mean, partial, R, C, CB, rpc, nullptr, mb);
  PA_CHECK_LAUNCH();
  hipLaunchKernelGGL(bn_bwd_finalize_k, dim3((C + 63) / 64), dim3(1024), 0, st, partial, chunks, C, R, w, mean, rstd,
                     dw, db, coef, global_stats);
  PA_CHECK_LAUNCH();
  const int64_t nvec = R * C / 8;
  const unsigned g = apply_grid(nvec);
  if (dres)
    hipLaunchKernelGGL((bn_bwd_apply_k<true, true, false, true>), dim3(g), dim3(kThreads), 0, st, (const uint16_t*)dy,
                       (const uint16_t*)x, nullptr, coef, (uint16_t*)dx, (uint16_t*)dres, nvec, C, nullptr, mb);
  else
    hipLaunchKernelGGL((bn_bwd_apply_k<true, false, false, true>), dim3(g), dim3(kThreads), 0, st,
                       (const uint16_t*)dy, (const uint16_t*)x, nullptr, coef, (uint16_t*)dx, nullptr, nvec, C,
                       nullptr, mb);
  PA_CHECK_LAUNCH();
  return 0;
}

// ---- conv -> BN fusion: the producing convolution wrote the forward partials (csrc/kernels/gemm.hip
// kEpiStats: stats[2][chunks][C], one chunk per 64/128 output rows), so the statistics pass over x is skipped.

namespace {
// first-level fold of a long chunk list: block (cx, g) folds chunks [g * per, (g + 1) * per) of 64 channels
// into out[2][gridDim.y][C] (fp64 lane sums, as fold_chunks)
__global__ __launch_bounds__(1024) void bn_fold_range_k(const float* __restrict__ partial, int chunks, int C, int per,
                                                        float* __restrict__ out) {
  __shared__ double sm1[kFoldLanes][64], sm2[kFoldLanes][64];
  const int cl = threadIdx.x & 63, k = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int j0 = blockIdx.y * per, j1 = min(chunks, j0 + per);
  double a = 0.0, b = 0.0;
  if (c < C) {
    const float* p1 = partial + c;
    const float* p2 = partial + (int64_t)chunks * C + c;
    int j = j0 + k;
    for (; j + 3 * kFoldLanes < j1; j += 4 * kFoldLanes) {
      float u[4], v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        u[q] = p1[(int64_t)(j + q * kFoldLanes) * C];
        v[q] = p2[(int64_t)(j + q * kFoldLanes) * C];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) { a += u[q]; b += v[q]; }
    }
    for (; j < j1; j += kFoldLanes) {
      a += p1[(int64_t)j * C];
      b += p2[(int64_t)j * C];
    }
  }
  sm1[k][cl] = a;
  sm2[k][cl] = b;
  __syncthreads();
  if (k == 0 && c < C) {
    double t1 = 0.0, t2 = 0.0;
#pragma unroll
    for (int q = 0; q < kFoldLanes; ++q) { t1 += sm1[q][cl]; t2 += sm2[q][cl]; }
    out[(int64_t)blockIdx.y * C + c] = (float)t1;
    out[((int64_t)gridDim.y + blockIdx.y) * C + c] = (float)t2;
  }
}
constexpr int kFoldPer = 256;  // chunks per first-level block
}  // namespace

// Workspace floats pa_bn_fwd_nhwc_pre needs for `chunks` producer chunks (0: folded directly).
PA_EXPORT int64_t pa_bn_pre_ws(int chunks, int C) {
  if (chunks <= kFoldPer) return 0;
  return 2 * (int64_t)((chunks + kFoldPer - 1) / kFoldPer) * C;
}

// Training forward from precomputed partials (stats[2][chunks][C] written by the convolution): fold ->
// finalize (mean / rstd / running stats / scale-shift) -> apply, as pa_bn_fwd_nhwc / _mask without the
// statistics pass. mbits (relu only): also the relu bit mask. ws: pa_bn_pre_ws floats (may be null if 0).
PA_EXPORT int pa_bn_fwd_nhwc_pre(const void* x, const void* res, void* y, const float* w, const float* b,
                                 float* run_mean, float* run_var, float* save_mean, float* save_rstd,
                                 const float* stats, int chunks, float* ws, float* ss, void* mbits, int64_t R, int C,
                                 float momentum, float eps, int relu, hipStream_t st) {
  if (C % 8 != 0 || R < 1 || chunks < 1 || !stats) return 3;
  if (mbits && !relu) return 3;
  const float* part = stats;
  int nch = chunks;
  if (chunks > kFoldPer) {
    if (!ws) return 3;
    const int groups = (chunks + kFoldPer - 1) / kFoldPer;
    hipLaunchKernelGGL(bn_fold_range_k, dim3((C + 63) / 64, groups), dim3(1024), 0, st, stats, chunks, C, kFoldPer,
                       ws);
    PA_CHECK_LAUNCH();
    part = ws;
    nch = groups;
  }
  hipLaunchKernelGGL(bn_fwd_finalize_k, dim3((C + 63) / 64), dim3(1024), 0, st, part, nch, C, R, w, b, run_mean,
                     run_var, momentum, eps, save_mean, save_rstd, ss);
  PA_CHECK_LAUNCH();
  const int64_t nvec = R * C / 8;
  const unsigned g = apply_grid(nvec);
  const uint16_t* xp = (const uint16_t*)x;
  const uint16_t* rp = (const uint16_t*)res;
  uint16_t* yp = (uint16_t*)y;
  if (mbits && res)
    hipLaunchKernelGGL((bn_apply_k<true, true, true>), dim3(g), dim3(kThreads), 0, st, xp, rp, ss, yp, nvec, C,
                       (uint8_t*)mbits);
  else if (mbits)
    hipLaunchKernelGGL((bn_apply_k<true, false, true>), dim3(g), dim3(kThreads), 0, st, xp, nullptr, ss, yp, nvec, C,
                       (uint8_t*)mbits);
  else if (relu && res)
    hipLaunchKernelGGL((bn_apply_k<true, true>), dim3(g), dim3(kThreads), 0, st, xp, rp, ss, yp, nvec, C, nullptr);
  else if (relu)
    hipLaunchKernelGGL((bn_apply_k<true, false>), dim3(g), dim3(kThreads), 0, st, xp, nullptr, ss, yp, nvec, C, nullptr);
  else if (res)
    hipLaunchKernelGGL((bn_apply_k<false, true>), dim3(g), dim3(kThreads), 0, st, xp, rp, ss, yp, nvec, C, nullptr);
  else
    hipLaunchKernelGGL((bn_apply_k<false, false>), dim3(g), dim3(kThreads), 0, st, xp, nullptr, ss, yp, nvec, C,
                       nullptr);
  PA_CHECK_LAUNCH();
  return 0;
}

// Backward from precomputed partials ([sum dyp, sum dyp * (x - mean)] written by the producing data-gradient
// convolution, gemm.hip kEpiStatsBwd) for the relu-without-residual form (mask from x * ss[0] + ss[1]):
// fold -> finalize (dweight / dbias / dx coefficients) -> apply.
PA_EXPORT int pa_bn_bwd_nhwc_pre(const void* dy, const void* x, void* dx, const float* w, const float* mean,
                                 const float* rstd, float* dw, float* db, const float* stats, int chunks, float* ws,
                                 float* coef, int64_t R, int C, int global_stats, const float* ss, hipStream_t st) {
  if (C % 8 != 0 || R < 1 || chunks < 1 || !stats || !ss) return 3;
  const float* part = stats;
  int nch = chunks;
  if (chunks > kFoldPer) {
    if (!ws) return 3;
    const int groups = (chunks + kFoldPer - 1) / kFoldPer;
    hipLaunchKernelGGL(bn_fold_range_k, dim3((C + 63) / 64, groups), dim3(1024), 0, st, stats, chunks, C, kFoldPer,
                       ws);
    PA_CHECK_LAUNCH();
    part = ws;
    nch = groups;
  }
  hipLaunchKernelGGL(bn_bwd_finalize_k, dim3((C + 63) / 64), dim3(1024), 0, st, part, nch, C, R, w, mean, rstd, dw, db,
                     coef, global_stats);
  PA_CHECK_LAUNCH();
  const int64_t nvec = R * C / 8;
  hipLaunchKernelGGL((bn_bwd_apply_k<true, false, true>), dim3(apply_grid(nvec)), dim3(kThreads), 0, st,
                     (const uint16_t*)dy, (const uint16_t*)x, nullptr, coef, (uint16_t*)dx, nullptr, nvec, C, ss);
  PA_CHECK_LAUNCH();
  return 0;
}

// ---- split-phase entry points (cross-rank SyncBatchNorm: the per-channel sums are all-reduced between
// the reduction and the apply; reference: sync_batch_norm_utils.h:575 all-reduces the backward stats)

namespace {
__global__ __launch_bounds__(1024) void bn_fold_k(const float* __restrict__ partial, int chunks, int C,
                                                  float* __restrict__ sums) {
  double s1, s2;
  int c;
  if (!fold_chunks(partial, chunks, C, &s1, &s2, &c)) return;
  sums[c] = (float)s1;
  sums[C + c] = (float)s2;
}
}  // namespace

// mode 0: sums = [sum x, sum x^2]; mode 1: sums = [sum dyp, sum dyp * (x - mean)] with dyp the relu-masked
// dy (mask from y, or from x * ss[0] + ss[1] when ss is given). sums: [2, C] fp32; partial as above.
PA_EXPORT int pa_bn_reduce_nhwc(int mode, const void* x, const void* dy, const void* y, const float* mean,
                                const float* ss, float* partial, float* sums, int64_t R, int C, int relu,
                                hipStream_t st) {
  if (C % 8 != 0 || R < 1) return 3;
  int CB, chunks;
  int64_t rpc;
  plan(R, C, &CB, &chunks, &rpc);
  const dim3 grid(C / CB, chunks);
  const uint16_t *xp = (const uint16_t*)x, *dp = (const uint16_t*)dy, *yp = (const uint16_t*)y;
  if (mode == 0)
    hipLaunchKernelGGL((bn_reduce_k<0, false>), grid, dim3(kThreads), 0, st, xp, nullptr, nullptr, nullptr, partial,
                       R, C, CB, rpc);
  else if (relu && ss)
    hipLaunchKernelGGL((bn_reduce_k<1, true, true>), grid, dim3(kThreads), 0, st, xp, dp, nullptr, mean, partial, R,
                       C, CB, rpc, ss);
  else if (relu)
    hipLaunchKernelGGL((bn_reduce_k<1, true>), grid, dim3(kThreads), 0, st, xp, dp, yp, mean, partial, R, C, CB, rpc);
  else
    hipLaunchKernelGGL((bn_reduce_k<1, false>), grid, dim3(kThreads), 0, st, xp, dp, nullptr, mean, partial, R, C, CB,
                       rpc);
  PA_CHECK_LAUNCH();
  hipLaunchKernelGGL(bn_fold_k, dim3((C + 63) / 64), dim3(1024), 0, st, partial, chunks, C, sums);
  PA_CHECK_LAUNCH();
  return 0;
}

// dx = coef[0] * dyp - coef[1] * x + coef[2] (coef: [3, C] fp32, computed by the caller from global sums);
// dres = dyp when given.
PA_EXPORT int pa_bn_bwd_apply_nhwc(const void* dy, const void* x, const void* y, const float* coef, void* dx,
                                   void* dres, int64_t R, int C, int relu, const float* ss, hipStream_t st) {
  if (C % 8 != 0 || R < 1) return 3;
  const int64_t nvec = R * C / 8;
  const unsigned g = apply_grid(nvec);
  const uint16_t *dp = (const uint16_t*)dy, *xp = (const uint16_t*)x, *yp = (const uint16_t*)y;
  uint16_t *dxp = (uint16_t*)dx, *drp = (uint16_t*)dres;
  if (relu && ss && !dres)
    hipLaunchKernelGGL((bn_bwd_apply_k<true, false, true>), dim3(g), dim3(kThreads), 0, st, dp, xp, nullptr, coef,
                       dxp, nullptr, nvec, C, ss);
  else if (relu && dres)
    hipLaunchKernelGGL((bn_bwd_apply_k<true, true>), dim3(g), dim3(kThreads), 0, st, dp, xp, yp, coef, dxp, drp, nvec, C,
                       nullptr);
  else if (relu)
    hipLaunchKernelGGL((bn_bwd_apply_k<true, false>), dim3(g), dim3(kThreads), 0, st, dp, xp, yp, coef, dxp, nullptr,
                       nvec, C, nullptr);
  else if (dres)
    hipLaunchKernelGGL((bn_bwd_apply_k<false, true>), dim3(g), dim3(kThreads), 0, st, dp, xp, nullptr, coef, dxp, drp,
                       nvec, C, nullptr);
  else
    hipLaunchKernelGGL((bn_bwd_apply_k<false, false>), dim3(g), dim3(kThreads), 0, st, dp, xp, nullptr, coef, dxp,
                       nullptr, nvec, C, nullptr);
  PA_CHECK_LAUNCH();
  return 0;
}
