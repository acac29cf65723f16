// Weight-only quantized GEMM (int8 / packed int4, per-channel or group-64/128 scales) and LLM.int8 for decode
// shapes (M <= 64 activation rows), with the dequantisation done in registers on the way into the MFMA.
//
// Reference behaviour: paddle/phi/kernels/gpu/weight_only_linear_kernel.cu, llm_int8_linear_kernel.cu,
// python/paddle/nn/quant/quantized_linear.py:56 (weight_quantize layout: int8 [N][K]; int4 [N/2][K] with the two
// output channels 2j / 2j+1 of a byte in its low / high nibble, stored +8 on ROCm; scales [N] or [K/G][N]).
//
// y[M, N] = x[M, K] . dequant(Wq)^T (+ bias). Decode GEMMs are bound by the weight bytes, so the kernel is
// built to stream Wq once at full width:
//   * a workgroup = 4 waves owns 16 x NT output channels (NT = 1 / 2 / 4 for M <= 16 / 32 / 64: each activation
//     fragment then feeds NT weight fragments) and every activation row (M <= 64: up to four 16-row MFMA tiles);
//     its waves take interleaved 64-deep K chunks (adjacent waves read adjacent weight bytes), and the K range
//     may be split over gridDim.y workgroups as well so that narrow layers still fill the chip;
//   * per chunk each lane loads 16 weight bytes of one channel (one 16-byte load: 16 int8 k-values, or for int4
//     the byte pair-row shared by channels 2j / 2j+1) and 16 activations per row tile, converts the integers to
//     exact bf16 integers and runs two v_mfma_f32_16x16x32_bf16 per row tile. A and B use the same permuted
//     k order inside the chunk (lane group q holds k = 16q .. 16q + 15: the first MFMA takes 0..7, the second
//     8..15), which is legal because the product sums over k;
//   * per-channel scales multiply the finished sums; group scales multiply each chunk's partial sum (a chunk
//     never straddles a group: G is 64 or 128);
//   * LLM.int8: the rows arrive split in two bf16 operands, the row-quantised inlier part xq (integers) with a
//     per-row scale and the outlier columns xo (zero elsewhere): acc = xq.Wq and acco = xo.Wq run on the same
//     weight fragment, y = sw[n] * (sx[m] * acc + acco);
//   * the four waves' sums meet in LDS; without a K split the workgroup writes bf16 (+ bias), with one it adds
//     fp32 partials into a zeroed slab that pa_wo_finalize turns into bf16 (+ bias).
#include "common.h"

#include <algorithm>

namespace {

using bf16x8 = __attribute__((ext_vector_type(8))) short;
using f32x4 = __attribute__((ext_vector_type(4))) float;

struct WoArgs {
  const uint16_t* x;    // [M][ldx] bf16 (LLM.int8: the inlier integers)
  const uint16_t* xo;   // LLM.int8 outlier operand [M][ldx] bf16, or null
  const float* sx;      // LLM.int8 per-row scale [M], or null
  const int8_t* w;      // int8 [N][K] or int4 pairs [N/2][K]
  const float* scale;   // [N] (per channel) or [K/G][N] (groups)
  const uint16_t* bias; // [N] bf16 or null
  uint16_t* y;          // [M][ldy] bf16 (no split)
  float* ws;            // [M][N] fp32 partial slab (split)
  int M, N, K, ldx, ldy, kchunks_per_split, split;
};

__device__ __forceinline__ short bf16_of_int(int v) {
  // |v| <= 127: exactly representable; bf16 bits of the float
  return (short)(__float_as_uint((float)v) >> 16);
}

template <int BITS>
__device__ __forceinline__ void dequant16(uint4 raw, int nibble_hi, bf16x8& lo, bf16x8& hi) {
  const uint32_t wd[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint32_t byte = (wd[i >> 2] >> (8 * (i & 3))) & 0xffu;
    int v;
    if constexpr (BITS == 8) {
      v = (int)(int8_t)byte;
    } else {
      v = (int)((nibble_hi ? (byte >> 4) : byte) & 0xfu) - 8;
    }
    if (i < 8) lo[i] = bf16_of_int(v);
    else hi[i - 8] = bf16_of_int(v);
  }
}

__device__ __forceinline__ void load_x16(const uint16_t* row, bool ok, bf16x8& lo, bf16x8& hi) {
  if (ok) {
    const uint4 a = *reinterpret_cast<const uint4*>(row);
    const uint4 b = *reinterpret_cast<const uint4*>(row + 8);
    lo = __builtin_bit_cast(bf16x8, a);
    hi = __builtin_bit_cast(bf16x8, b);
  } else {
    lo = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    hi = lo;
  }
}

// BITS: 8 / 4; G: 0 = per-channel scale, else group size (64 / 128); MT: 16-row tiles (ceil(M / 16)); NT: 16-column
// tiles per wave (the workgroup covers 16 * NT channels: more rows re-read the activations more often, so larger M
// gives each activation fragment more channels to feed); LLM: int8 mode
template <int BITS, int G, int MT, int NT, bool LLM>
__global__ __launch_bounds__(256) void wo_gemm_k(WoArgs p) {
  constexpr int TILE = MT * 256;                       // floats of one 16-column tile's partial sums
  __shared__ float red[4][NT * TILE * (LLM ? 2 : 1)];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int col = lane & 15, q = lane >> 4;
  const int n0 = blockIdx.x * 16 * NT;
  const int chunk0 = blockIdx.y * p.kchunks_per_split;
  const int nch = min(p.kchunks_per_split, p.K / 64 - chunk0);
  const int8_t* wrow[NT];
  int nib[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int n = n0 + j * 16 + col;
    wrow[j] = BITS == 8 ? p.w + (int64_t)n * p.K : p.w + (int64_t)(n >> 1) * p.K;
    nib[j] = n & 1;
  }
  f32x4 acc[MT][NT], acco[MT][NT];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      acc[t][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      acco[t][j] = acc[t][j];
    }
  // weight stream two chunks ahead of the MFMAs (the only HBM operand; activations are L2-resident)
  uint4 raw0[NT], raw1[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    raw0[j] = wave < nch ? *reinterpret_cast<const uint4*>(wrow[j] + (chunk0 + wave) * 64 + q * 16)
                         : make_uint4(0, 0, 0, 0);
    raw1[j] = wave + 4 < nch ? *reinterpret_cast<const uint4*>(wrow[j] + (chunk0 + wave + 4) * 64 + q * 16)
                             : make_uint4(0, 0, 0, 0);
  }
  for (int c = wave; c < nch; c += 4) {
    const int kc = (chunk0 + c) * 64 + q * 16;
    bf16x8 blo[NT], bhi[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      dequant16<BITS>(raw0[j], nib[j], blo[j], bhi[j]);
      raw0[j] = raw1[j];
      raw1[j] = c + 8 < nch ? *reinterpret_cast<const uint4*>(wrow[j] + (chunk0 + c + 8) * 64 + q * 16)
                            : make_uint4(0, 0, 0, 0);
    }
    float s[NT];
    if constexpr (G != 0) {
#pragma unroll
      for (int j = 0; j < NT; ++j) s[j] = p.scale[(int64_t)(((chunk0 + c) * 64) / G) * p.N + n0 + j * 16 + col];
    }
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int m = t * 16 + col;
      const bool ok = m < p.M;
      bf16x8 alo, ahi;
      load_x16(p.x + (int64_t)(ok ? m : 0) * p.ldx + kc, ok, alo, ahi);
      bf16x8 olo, ohi;
      if constexpr (LLM) load_x16(p.xo + (int64_t)(ok ? m : 0) * p.ldx + kc, ok, olo, ohi);
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        f32x4 z = G ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[t][j];
        z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo, blo[j], z, 0, 0, 0);
        z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, bhi[j], z, 0, 0, 0);
        if constexpr (G != 0) acc[t][j] += z * s[j];
        else acc[t][j] = z;
        if constexpr (LLM) {
          acco[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(olo, blo[j], acco[t][j], 0, 0, 0);
          acco[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ohi, bhi[j], acco[t][j], 0, 0, 0);
        }
      }
    }
  }
  // D layout: col = lane & 15 (the channel), rows (lane >> 4) * 4 + r of each 16-row tile
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        red[wave][j * TILE + (t * 16 + q * 4 + r) * 16 + col] = acc[t][j][r];
        if constexpr (LLM) red[wave][NT * TILE + j * TILE + (t * 16 + q * 4 + r) * 16 + col] = acco[t][j][r];
      }
  __syncthreads();
  for (int e = tid; e < NT * TILE; e += 256) {
    const int j = e / TILE, w = e % TILE;
    const int m = w >> 4, nn = n0 + j * 16 + (w & 15);
    if (m >= p.M) continue;
    float v = red[0][e] + red[1][e] + red[2][e] + red[3][e];
    if constexpr (LLM) {
      const int eo = NT * TILE + e;
      const float o = red[0][eo] + red[1][eo] + red[2][eo] + red[3][eo];
      v = (v * p.sx[m] + o) * p.scale[nn];
    } else if constexpr (G == 0) {
      v *= p.scale[nn];
    }
    if (p.split > 1) {
      atomicAdd(p.ws + (int64_t)m * p.N + nn, v);
    } else {
      if (p.bias) v += pa::bf16_bits_to_f(p.bias[nn]);
      p.y[(int64_t)m * p.ldy + nn] = (uint16_t)(pa::pack_bf16(v, 0.f) & 0xffffu);
    }
  }
}

__global__ void wo_finalize_k(const float* ws, const uint16_t* bias, uint16_t* y, int M, int N, int ldy) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)M * N) return;
  const int m = (int)(i / N), nn = (int)(i % N);
  float v = ws[i];
  if (bias) v += pa::bf16_bits_to_f(bias[nn]);
  y[(int64_t)m * ldy + nn] = (uint16_t)(pa::pack_bf16(v, 0.f) & 0xffffu);
}

// dequantisation to a bf16 [N][K] image (prefill shapes run the bf16 GEMM on it, B K-major)
template <int BITS, int G>
__global__ void wo_dequant_k(const int8_t* w, const float* scale, uint16_t* out, int N, int K) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;  // 8 consecutive k of one channel
  if (i >= (int64_t)N * K) return;
  const int n = (int)(i / K), k = (int)(i % K);
  uint32_t packed[4];
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    float f[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int kk = k + j + h;
      int v;
      if constexpr (BITS == 8) {
        v = (int)w[(int64_t)n * K + kk];
      } else {
        const uint32_t byte = (uint8_t)w[(int64_t)(n >> 1) * K + kk];
        v = (int)(((n & 1) ? (byte >> 4) : byte) & 0xfu) - 8;
      }
      const float s = G ? scale[(int64_t)(kk / G) * N + n] : scale[n];
      f[h] = (float)v * s;
    }
    packed[j / 2] = pa::pack_bf16(f[0], f[1]);
  }
  *reinterpret_cast<uint4*>(out + i) = make_uint4(packed[0], packed[1], packed[2], packed[3]);
}

// column tiles per wave by row count (more rows: more channels per activation fragment)
inline int nt_for(int M) { return M <= 16 ? 1 : (M <= 32 ? 2 : 4); }

template <int BITS, int G, bool LLM, int NT>
int launch_nt(const WoArgs& a, dim3 grid, hipStream_t st) {
  const int mt = (a.M + 15) / 16;
  switch (mt) {
    case 1: hipLaunchKernelGGL((wo_gemm_k<BITS, G, 1, NT, LLM>), grid, dim3(256), 0, st, a); break;
    case 2: hipLaunchKernelGGL((wo_gemm_k<BITS, G, 2, NT, LLM>), grid, dim3(256), 0, st, a); break;
    case 3: hipLaunchKernelGGL((wo_gemm_k<BITS, G, 3, NT, LLM>), grid, dim3(256), 0, st, a); break;
    case 4: hipLaunchKernelGGL((wo_gemm_k<BITS, G, 4, NT, LLM>), grid, dim3(256), 0, st, a); break;
    default: return 1;
  }
  return 0;
}

template <int BITS, int G, bool LLM>
int launch_mt(const WoArgs& a, dim3 grid, hipStream_t st) {
  const int nt = LLM ? std::min(nt_for(a.M), 2) : nt_for(a.M);
  if (nt == 1) return launch_nt<BITS, G, LLM, 1>(a, grid, st);
  if (nt == 2) return launch_nt<BITS, G, LLM, 2>(a, grid, st);
  if constexpr (!LLM) return launch_nt<BITS, G, LLM, 4>(a, grid, st);
  return 1;
}

}  // namespace

// Splits of K so that (N / (16 * NT)) x splits workgroups fill the chip (>= 2 per CU), each split a multiple of
// 4 chunks of 64.
PA_EXPORT int pa_wo_gemm_splits(int64_t M, int64_t N, int64_t K, int llm) {
  int nt = nt_for((int)M);
  if (llm && nt > 2) nt = 2;
  const int64_t wgs = N / (16 * nt), chunks = K / 64;
  int s = 1;
  while (wgs * s < 512 && chunks % (s * 2 * 4) == 0) s *= 2;
  return s;
}

// bits: 8 / 4; group: -1 (per channel), 64, 128; llm: 1 = LLM.int8 (xo / sx given, per-channel scales).
// Requirements (checked by ops/quant.py too): M <= 64, K % 64 == 0, N % 16 == 0, 16-byte aligned rows.
// ws: M * N fp32, zeroed here, when splits > 1.
PA_EXPORT int pa_wo_gemm(const void* x, const void* xo, const float* sx, const void* w, const float* scale,
                         const void* bias, void* y, float* ws, int M, int N, int K, int ldx, int ldy, int bits,
                         int group, int splits, hipStream_t st) {
  if (M <= 0 || M > 64 || K % 64 != 0 || ldx % 8 != 0) return 1;
  const int nt_req = xo != nullptr ? std::min(nt_for(M), 2) : nt_for(M);
  if (N % (16 * nt_req) != 0) return 1;
  if (bits != 8 && bits != 4) return 2;
  if (group != -1 && group != 64 && group != 128) return 3;
  const bool llm = xo != nullptr;
  if (llm && (bits != 8 || group != -1 || sx == nullptr)) return 4;
  if (splits < 1 || (K / 64) % splits != 0) return 5;
  if (splits > 1 && ws == nullptr) return 6;
  WoArgs a{};
  a.x = (const uint16_t*)x; a.xo = (const uint16_t*)xo; a.sx = sx; a.w = (const int8_t*)w; a.scale = scale;
  a.bias = (const uint16_t*)bias; a.y = (uint16_t*)y; a.ws = ws;
  a.M = M; a.N = N; a.K = K; a.ldx = ldx; a.ldy = ldy; a.split = splits; a.kchunks_per_split = K / 64 / splits;
  if (splits > 1 && hipMemsetAsync(ws, 0, sizeof(float) * (size_t)M * N, st) != hipSuccess) return 7;
  dim3 grid((unsigned)(N / (16 * nt_req)), (unsigned)splits);
  int rc;
  if (llm) rc = launch_mt<8, 0, true>(a, grid, st);
  else if (bits == 8 && group == -1) rc = launch_mt<8, 0, false>(a, grid, st);
  else if (bits == 8 && group == 64) rc = launch_mt<8, 64, false>(a, grid, st);
  else if (bits == 8) rc = launch_mt<8, 128, false>(a, grid, st);
  else if (group == -1) rc = launch_mt<4, 0, false>(a, grid, st);
  else if (group == 64) rc = launch_mt<4, 64, false>(a, grid, st);
  else rc = launch_mt<4, 128, false>(a, grid, st);
  if (rc) return rc;
  if (splits > 1) {
    const int64_t tot = (int64_t)M * N;
    hipLaunchKernelGGL(wo_finalize_k, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, ws,
                       (const uint16_t*)bias, (uint16_t*)y, M, N, ldy);
  }
  PA_CHECK_LAUNCH();
  return 0;
}

// out [N][K] bf16 = dequant(w) (K % 8 == 0)
PA_EXPORT int pa_wo_dequant(const void* w, const float* scale, void* out, int N, int K, int bits, int group,
                            hipStream_t st) {
  if (K % 8 != 0 || (bits != 8 && bits != 4) || (group != -1 && group != 64 && group != 128)) return 1;
  const int64_t threads = (int64_t)N * K / 8;
  dim3 grid((unsigned)((threads + 255) / 256));
  const int8_t* wp = (const int8_t*)w;
  uint16_t* op = (uint16_t*)out;
#define PA_DQ(B, G) hipLaunchKernelGGL((wo_dequant_k<B, G>), grid, dim3(256), 0, st, wp, scale, op, N, K)
  if (bits == 8) {
    if (group == -1) PA_DQ(8, 0); else if (group == 64) PA_DQ(8, 64); else PA_DQ(8, 128);
  } else {
    if (group == -1) PA_DQ(4, 0); else if (group == 64) PA_DQ(4, 64); else PA_DQ(4, 128);
  }
#undef PA_DQ
  PA_CHECK_LAUNCH();
  return 0;
}
