// Multi-tensor AdamW (+ master weights) and multi-tensor sum-of-squares for gfx950.
// Reference behaviour: paddle/phi/kernels/gpu/fused_adam_kernel.cu, adamw_kernel.cu.
//
// One launch per parameter group. Device table row (9 x int64):
//   [param_fp32*, grad*, m*, v*, lowp_param* (or 0), numel, gdtype | (ldtype<<8), wd (f32 bits), lr_mult (f32 bits)]
// Work items (2 x int64): [tensor index, start element]; each item covers kChunk elements.
// A persistent grid walks the items; per element: fp32 math, decoupled weight decay,
// bias-corrected update, optional low-precision shadow write in the same pass.
#include "common.h"

using namespace pa;

namespace {

constexpr int64_t kChunk = 16384;

struct Row {
  float* p; const void* g; float* m; float* v; void* lp; int64_t n; int64_t dt; int64_t wd; int64_t lrm;
};

__device__ __forceinline__ float ld_any(const void* p, int64_t i, int dt) {
  if (dt == kF32) return ((const float*)p)[i];
  if (dt == kBF16) return to_f(((const bf16*)p)[i]);
  return to_f(((const f16*)p)[i]);
}

__device__ __forceinline__ void st_any(void* p, int64_t i, int dt, float x) {
  if (dt == kF32) ((float*)p)[i] = x;
  else if (dt == kBF16) ((bf16*)p)[i] = from_f<bf16>(x);
  else ((f16*)p)[i] = from_f<f16>(x);
}

__global__ __launch_bounds__(256) void adamw_multi_k(const int64_t* __restrict__ table, const int64_t* __restrict__ items,
                                                     int64_t n_items, const float* __restrict__ inv_scale_p, float lr,
                                                     float b1, float b2, float eps, float bc1, float bc2,
                                                     const float* __restrict__ hyper) {
  const float inv_scale = inv_scale_p ? *inv_scale_p : 1.f;
  if (hyper) {  // device-resident {lr, beta1^t, beta2^t}: a captured step keeps following the schedule on replay
    lr = hyper[0];
    bc1 = 1.f - hyper[1];
    bc2 = 1.f - hyper[2];
  }
  const float rbc2 = 1.f / bc2;
  for (int64_t it = blockIdx.x; it < n_items; it += gridDim.x) {
    const int64_t ti = items[it * 2], s = items[it * 2 + 1];
    const int64_t* r = table + ti * 9;
    float* __restrict__ P = (float*)r[0];
    const void* G = (const void*)r[1];
    float* __restrict__ M = (float*)r[2];
    float* __restrict__ V = (float*)r[3];
    void* LP = (void*)r[4];
    const int64_t n = r[5];
    const int gdt = (int)(r[6] & 0xff), ldt = (int)((r[6] >> 8) & 0xff);
    const float wd = __int_as_float((int)r[7]);
    const float plr = lr * __int_as_float((int)r[8]);
    const float decay = 1.f - plr * wd;
    const float step = plr / bc1;
    const int64_t e = s + kChunk < n ? s + kChunk : n;
    // vector path: 4 elements per thread per iteration when everything is aligned
    const bool vec = ((((uintptr_t)P | (uintptr_t)M | (uintptr_t)V) & 15) == 0) &&
                     ((((uintptr_t)G) & (gdt == kF32 ? 15 : 7)) == 0) &&
                     (ldt == 3 || ((((uintptr_t)LP) & (ldt == kF32 ? 15 : 7)) == 0)) && (s % 4 == 0);
    int64_t i0 = s;
    if (vec) {
      const int64_t ev = s + ((e - s) / 4) * 4;
      for (int64_t i = s + (int64_t)threadIdx.x * 4; i < ev; i += 256 * 4) {
        float4 p = *(float4*)(P + i), m = *(float4*)(M + i), v = *(float4*)(V + i);
        float g[4];
        if (gdt == kF32) {
          float4 gg = *(const float4*)((const float*)G + i);
          g[0] = gg.x; g[1] = gg.y; g[2] = gg.z; g[3] = gg.w;
        } else {
          uint2 gg = *(const uint2*)((const uint16_t*)G + i);
          if (gdt == kBF16) { g[0] = lo_bf16(gg.x); g[1] = hi_bf16(gg.x); g[2] = lo_bf16(gg.y); g[3] = hi_bf16(gg.y); }
          else { g[0] = lo_f16(gg.x); g[1] = hi_f16(gg.x); g[2] = lo_f16(gg.y); g[3] = hi_f16(gg.y); }
        }
        float pa_[4] = {p.x, p.y, p.z, p.w}, ma[4] = {m.x, m.y, m.z, m.w}, va[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float gj = g[j] * inv_scale;
          ma[j] = b1 * ma[j] + (1.f - b1) * gj;
          va[j] = b2 * va[j] + (1.f - b2) * gj * gj;
          pa_[j] = pa_[j] * decay - step * ma[j] / (sqrtf(va[j] * rbc2) + eps);
        }
        *(float4*)(P + i) = make_float4(pa_[0], pa_[1], pa_[2], pa_[3]);
        *(float4*)(M + i) = make_float4(ma[0], ma[1], ma[2], ma[3]);
        *(float4*)(V + i) = make_float4(va[0], va[1], va[2], va[3]);
        if (ldt == kBF16) {
          *(uint2*)((uint16_t*)LP + i) = make_uint2(pack_bf16(pa_[0], pa_[1]), pack_bf16(pa_[2], pa_[3]));
        } else if (ldt == kF16) {
          *(uint2*)((uint16_t*)LP + i) = make_uint2(pack_f16(pa_[0], pa_[1]), pack_f16(pa_[2], pa_[3]));
        } else if (ldt == kF32) {
          *(float4*)((float*)LP + i) = make_float4(pa_[0], pa_[1], pa_[2], pa_[3]);
        }
      }
      i0 = ev;
    }
    for (int64_t i = i0 + threadIdx.x; i < e; i += 256) {
      const float gj = ld_any(G, i, gdt) * inv_scale;
      float m = b1 * M[i] + (1.f - b1) * gj;
      float v = b2 * V[i] + (1.f - b2) * gj * gj;
      float p = P[i] * decay - step * m / (sqrtf(v * rbc2) + eps);
      M[i] = m; V[i] = v; P[i] = p;
      if (ldt != 3) st_any(LP, i, ldt, p);
    }
  }
}

// table rows (3 x int64): [ptr, numel, dtype]; items as above. partial[blockIdx] = sum of squares
__global__ __launch_bounds__(256) void sq_norm_multi_k(const int64_t* __restrict__ table, const int64_t* __restrict__ items,
                                                       int64_t n_items, float* __restrict__ partial) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int64_t it = blockIdx.x; it < n_items; it += gridDim.x) {
    const int64_t ti = items[it * 2], s = items[it * 2 + 1];
    const void* X = (const void*)table[ti * 3];
    const int64_t n = table[ti * 3 + 1];
    const int dt = (int)table[ti * 3 + 2];
    const int64_t e = s + kChunk < n ? s + kChunk : n;
    int64_t i0 = s;
    if ((((uintptr_t)X) & 15) == 0) {  // 16-byte vector path
      const int per = dt == kF32 ? 4 : 8;
      const int64_t ev = s + ((e - s) / per) * per;
      for (int64_t i = s + (int64_t)threadIdx.x * per; i < ev; i += 256 * per) {
        if (dt == kF32) {
          const float4 v = *reinterpret_cast<const float4*>((const float*)X + i);
          acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
        } else {
          float v[8];
          if (dt == kBF16) load8<bf16>((const bf16*)X + i, v); else load8<f16>((const f16*)X + i, v);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc += v[j] * v[j];
        }
      }
      i0 = ev;
    }
    for (int64_t i = i0 + threadIdx.x; i < e; i += 256) {
      const float x = ld_any(X, i, dt);
      acc += x * x;
    }
  }
  acc = block_sum<256>(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = acc;
}

// Multi-tensor Momentum (paddle/phi/kernels/gpu/momentum_kernel.cu semantics): same table rows as
// AdamW with m* = velocity (fp32) and v* unused; wd = L2 coefficient folded into the gradient.
//   g = grad * rescale * inv_scale + wd * p;  vel = mu * vel + g;  p -= lr * (nesterov ? g + mu * vel : vel)
__global__ __launch_bounds__(256) void momentum_multi_k(const int64_t* __restrict__ table,
                                                        const int64_t* __restrict__ items, int64_t n_items,
                                                        const float* __restrict__ inv_scale_p, float lr, float mu,
                                                        float rescale, int nesterov) {
  const float gs = rescale * (inv_scale_p ? *inv_scale_p : 1.f);
  for (int64_t it = blockIdx.x; it < n_items; it += gridDim.x) {
    const int64_t ti = items[it * 2], s = items[it * 2 + 1];
    const int64_t* r = table + ti * 9;
    float* __restrict__ P = (float*)r[0];
    const void* G = (const void*)r[1];
    float* __restrict__ VEL = (float*)r[2];
    void* LP = (void*)r[4];
    const int64_t n = r[5];
    const int gdt = (int)(r[6] & 0xff), ldt = (int)((r[6] >> 8) & 0xff);
    const float wd = __int_as_float((int)r[7]);
    const float plr = lr * __int_as_float((int)r[8]);
    const int64_t e = s + kChunk < n ? s + kChunk : n;
    const bool vec = ((((uintptr_t)P | (uintptr_t)VEL) & 15) == 0) &&
                     ((((uintptr_t)G) & (gdt == kF32 ? 15 : 7)) == 0) &&
                     (ldt == 3 || ((((uintptr_t)LP) & (ldt == kF32 ? 15 : 7)) == 0)) && (s % 4 == 0);
    int64_t i0 = s;
    if (vec) {
      const int64_t ev = s + ((e - s) / 4) * 4;
      for (int64_t i = s + (int64_t)threadIdx.x * 4; i < ev; i += 256 * 4) {
        float4 p = *(float4*)(P + i), v = *(float4*)(VEL + i);
        float g[4];
        if (gdt == kF32) {
          float4 gg = *(const float4*)((const float*)G + i);
          g[0] = gg.x; g[1] = gg.y; g[2] = gg.z; g[3] = gg.w;
        } else {
          uint2 gg = *(const uint2*)((const uint16_t*)G + i);
          if (gdt == kBF16) { g[0] = lo_bf16(gg.x); g[1] = hi_bf16(gg.x); g[2] = lo_bf16(gg.y); g[3] = hi_bf16(gg.y); }
          else { g[0] = lo_f16(gg.x); g[1] = hi_f16(gg.x); g[2] = lo_f16(gg.y); g[3] = hi_f16(gg.y); }
        }
        float pa_[4] = {p.x, p.y, p.z, p.w}, va[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float gj = g[j] * gs + wd * pa_[j];
          va[j] = mu * va[j] + gj;
          pa_[j] -= plr * (nesterov ? gj + mu * va[j] : va[j]);
        }
        *(float4*)(P + i) = make_float4(pa_[0], pa_[1], pa_[2], pa_[3]);
        *(float4*)(VEL + i) = make_float4(va[0], va[1], va[2], va[3]);
        if (ldt == kBF16) {
          *(uint2*)((uint16_t*)LP + i) = make_uint2(pack_bf16(pa_[0], pa_[1]), pack_bf16(pa_[2], pa_[3]));
        } else if (ldt == kF16) {
          *(uint2*)((uint16_t*)LP + i) = make_uint2(pack_f16(pa_[0], pa_[1]), pack_f16(pa_[2], pa_[3]));
        } else if (ldt == kF32) {
          *(float4*)((float*)LP + i) = make_float4(pa_[0], pa_[1], pa_[2], pa_[3]);
        }
      }
      i0 = ev;
    }
    for (int64_t i = i0 + threadIdx.x; i < e; i += 256) {
      const float p = P[i];
      const float gj = ld_any(G, i, gdt) * gs + wd * p;
      const float v = mu * VEL[i] + gj;
      const float np = p - plr * (nesterov ? gj + mu * v : v);
      VEL[i] = v; P[i] = np;
      if (ldt != 3) st_any(LP, i, ldt, np);
    }
  }
}

// Values carried as kernel arguments (copied into the launch / the captured graph node at launch time), so a
// pointer table written inside a hipGraph capture does not reference any host buffer on replay.
constexpr int kArgVals = 248;
struct ArgVals {
  int64_t v[kArgVals];
};

__global__ __launch_bounds__(256) void write_i64_k(int64_t* __restrict__ dst, ArgVals a, int n) {
  if ((int)threadIdx.x < n) dst[threadIdx.x] = a.v[threadIdx.x];
}

}  // namespace

PA_EXPORT int pa_adamw_multi(const int64_t* table, const int64_t* items, int64_t n_items, const float* inv_scale,
                             float lr, float b1, float b2, float eps, float wd_unused, float bc1, float bc2,
                             const float* hyper, hipStream_t st) {
  if (n_items <= 0) return 0;
  int64_t g = n_items < 4096 ? n_items : 4096;
  hipLaunchKernelGGL(adamw_multi_k, dim3((unsigned)g), dim3(256), 0, st, table, items, n_items, inv_scale, lr, b1, b2,
                     eps, bc1, bc2, hyper);
  PA_CHECK_LAUNCH();
  return 0;
}

// One optimizer step of the device-resident Adam hyper-parameters {lr, beta1^t, beta2^t}: the beta powers advance
// on the device (reference: the beta1_pow / beta2_pow accumulators updated inside adam_kernel), so a hipGraph that
// captured the step applies the right bias correction on every replay; lr is written by the LR scheduler.
__global__ void adam_hyper_step_k(float* hyper, float b1, float b2) {
  if (threadIdx.x == 0) {
    hyper[1] *= b1;
    hyper[2] *= b2;
  }
}

PA_EXPORT int pa_adam_hyper_step(float* hyper, float b1, float b2, hipStream_t st) {
  hipLaunchKernelGGL(adam_hyper_step_k, dim3(1), dim3(64), 0, st, hyper, b1, b2);
  PA_CHECK_LAUNCH();
  return 0;
}

// partial must hold 1024 floats; caller sums it.
PA_EXPORT int pa_sq_norm_multi(const int64_t* table, const int64_t* items, int64_t n_items, float* partial,
                               hipStream_t st) {
  (void)hipMemsetAsync(partial, 0, 1024 * sizeof(float), st);
  if (n_items <= 0) return 0;
  int64_t g = n_items < 1024 ? n_items : 1024;
  hipLaunchKernelGGL(sq_norm_multi_k, dim3((unsigned)g), dim3(256), 0, st, table, items, n_items, partial);
  PA_CHECK_LAUNCH();
  return 0;
}

PA_EXPORT int pa_momentum_multi(const int64_t* table, const int64_t* items, int64_t n_items, const float* inv_scale,
                                float lr, float mu, float rescale, int nesterov, hipStream_t st) {
  if (n_items <= 0) return 0;
  int64_t g = n_items < 4096 ? n_items : 4096;
  hipLaunchKernelGGL(momentum_multi_k, dim3((unsigned)g), dim3(256), 0, st, table, items, n_items, inv_scale, lr, mu,
                     rescale, nesterov);
  PA_CHECK_LAUNCH();
  return 0;
}

// dst[0:n] (device) = src[0:n] (host int64), as kernel-argument payloads of <= 248 values per launch.
PA_EXPORT int pa_write_i64(int64_t* dst, const int64_t* src, int64_t n, hipStream_t st) {
  for (int64_t o = 0; o < n; o += kArgVals) {
    ArgVals a;
    const int m = (int)(n - o < kArgVals ? n - o : kArgVals);
    for (int i = 0; i < m; ++i) a.v[i] = src[o + i];
    hipLaunchKernelGGL(write_i64_k, dim3(1), dim3(256), 0, st, dst + o, a, m);
    PA_CHECK_LAUNCH();
  }
  return 0;
}
