// Shared helpers for the gfx950 (CDNA4) kernels of paddlepaddle_amd.
// Wave = 64 lanes; vectorised 16-byte global accesses (8 x bf16/fp16 or 4 x fp32);
// fp32 math; bf16 rounding through the hardware cvt (NaN-preserving, see MI355X_MICROARCH.md).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#define PA_EXPORT extern "C" __attribute__((visibility("default")))

namespace pa {

constexpr int kWave = 64;

enum DType : int { kF32 = 0, kF16 = 1, kBF16 = 2 };

using bf16 = __hip_bfloat16;
using f16 = __half;

template <typename T> struct Vec8;   // 8 elements = 16 bytes for 16-bit types
template <> struct Vec8<bf16> { using type = uint4; };
template <> struct Vec8<f16> { using type = uint4; };

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16 x) { return __bfloat162float(x); }
__device__ __forceinline__ float to_f(f16 x) { return __half2float(x); }

template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return __float2bfloat16(x); }
template <> __device__ __forceinline__ f16 from_f<f16>(float x) { return __float2half(x); }

// bf16 <-> fp32 on raw 16-bit patterns
__device__ __forceinline__ float bf16_bits_to_f(uint32_t b) { return __uint_as_float(b << 16); }
__device__ __forceinline__ float lo_bf16(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi_bf16(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// one v_cvt_pk_bf16_f32 (RNE, NaN-preserving) for the pair; the scalar __float2bfloat16 form costs
// two converts + a shift + an OR per pair
typedef float pa_f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 pa_bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack_bf16(float a, float b) {
  const pa_f32x2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, pa_bf16x2));
}
__device__ __forceinline__ uint32_t pack_f16(float a, float b) {
  f16 x = __float2half(a), y = __float2half(b);
  return (uint32_t)(*reinterpret_cast<uint16_t*>(&x)) | ((uint32_t)(*reinterpret_cast<uint16_t*>(&y)) << 16);
}
__device__ __forceinline__ float lo_f16(uint32_t w) {
  uint16_t u = (uint16_t)(w & 0xffff); return __half2float(*reinterpret_cast<f16*>(&u));
}
__device__ __forceinline__ float hi_f16(uint32_t w) {
  uint16_t u = (uint16_t)(w >> 16); return __half2float(*reinterpret_cast<f16*>(&u));
}

// ---- 8-element vector load/store into float[8] (16-bit types: one 16-byte access; fp32: two)
template <typename T> __device__ __forceinline__ void load8(const T* p, float* f);
template <> __device__ __forceinline__ void load8<bf16>(const bf16* p, float* f) {
  uint4 v = *reinterpret_cast<const uint4*>(p);
  f[0] = lo_bf16(v.x); f[1] = hi_bf16(v.x); f[2] = lo_bf16(v.y); f[3] = hi_bf16(v.y);
  f[4] = lo_bf16(v.z); f[5] = hi_bf16(v.z); f[6] = lo_bf16(v.w); f[7] = hi_bf16(v.w);
}
template <> __device__ __forceinline__ void load8<f16>(const f16* p, float* f) {
  uint4 v = *reinterpret_cast<const uint4*>(p);
  f[0] = lo_f16(v.x); f[1] = hi_f16(v.x); f[2] = lo_f16(v.y); f[3] = hi_f16(v.y);
  f[4] = lo_f16(v.z); f[5] = hi_f16(v.z); f[6] = lo_f16(v.w); f[7] = hi_f16(v.w);
}
template <> __device__ __forceinline__ void load8<float>(const float* p, float* f) {
  float4 a = *reinterpret_cast<const float4*>(p);
  float4 b = *reinterpret_cast<const float4*>(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

template <typename T> __device__ __forceinline__ void store8(T* p, const float* f);
template <> __device__ __forceinline__ void store8<bf16>(bf16* p, const float* f) {
  uint4 v;
  v.x = pack_bf16(f[0], f[1]); v.y = pack_bf16(f[2], f[3]); v.z = pack_bf16(f[4], f[5]); v.w = pack_bf16(f[6], f[7]);
  *reinterpret_cast<uint4*>(p) = v;
}
template <> __device__ __forceinline__ void store8<f16>(f16* p, const float* f) {
  uint4 v;
  v.x = pack_f16(f[0], f[1]); v.y = pack_f16(f[2], f[3]); v.z = pack_f16(f[4], f[5]); v.w = pack_f16(f[6], f[7]);
  *reinterpret_cast<uint4*>(p) = v;
}
template <> __device__ __forceinline__ void store8<float>(float* p, const float* f) {
  *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(f[4], f[5], f[6], f[7]);
}

// ---- tanh-approximated GELU without tanhf: with s = sigmoid(2u) = 1 / (1 + 2^(-2u log2 e)),
// u = sqrt(2/pi) (x + 0.044715 x^3):  gelu(x) = x s,  gelu'(x) = s + 2 x s (1 - s) sqrt(2/pi) (1 + 3 * 0.044715 x^2).
// One v_exp_f32 + one v_rcp_f32 per element (tanhf is a long VALU sequence; these epilogue / elementwise
// passes are VALU-bound with it). Saturates correctly: 2^(+inf) -> s = 0, 2^(-inf) -> s = 1.
__device__ __forceinline__ float gelu_sig2u(float x) {
  const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-2.8853900817779268f * u));  // 2 log2(e)
}
__device__ __forceinline__ float gelu_tanh_fast(float x) { return x * gelu_sig2u(x); }
__device__ __forceinline__ float gelu_tanh_grad_fast(float x) {
  const float s = gelu_sig2u(x);
  return s + 2.f * x * s * (1.f - s) * 0.7978845608028654f * (1.f + 0.134145f * x * x);
}

// ---- wave / block reductions (wave64)
// sum over the 16 lanes of a DPP row (lanes 16r .. 16r + 15); every lane of the row ends with the total
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, true));   // quad_perm 1,0,3,2
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, true));   // quad_perm 2,3,0,1
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, true));  // row_half_mirror
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, true));  // row_mirror
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block reduce for blockDim.x == NT (multiple of 64); smem holds NT/64 floats
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* smem) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) smem[w] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += smem[i];
  return r;
}
template <int NT>
__device__ __forceinline__ float block_max(float v, float* smem) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) smem[w] = v;
  __syncthreads();
  float r = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r = fmaxf(r, smem[i]);
  return r;
}

__host__ __device__ inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace pa

#define PA_DISPATCH_DTYPE(code, T, ...)                   \
  switch (code) {                                         \
    case pa::kF32: { using T = float; __VA_ARGS__; break; } \
    case pa::kF16: { using T = pa::f16; __VA_ARGS__; break; } \
    case pa::kBF16: { using T = pa::bf16; __VA_ARGS__; break; } \
    default: return 2;                                    \
  }

#define PA_CHECK_LAUNCH() do { hipError_t e_ = hipGetLastError(); if (e_ != hipSuccess) return 1; } while (0)
