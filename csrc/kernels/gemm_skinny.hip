// Memory-bound "skinny" GEMM: C[M, N] = A[M, K] . B[K, N] (+ bias, or accumulated onto C) for a very tall M and a
// small N x K (N <= 256, K <= 256) — the 1x1 convolutions of ResNet's 56x56 / 28x28 stages as forward
// (Y = X . W^T) and data-gradient (dX = dY . W) GEMMs over the N*H*W pixel rows. At these shapes the 256x256-tile
// kernels of gemm.hip run at half the HBM roofline: one workgroup per CU serialises load -> MFMA -> store, and a
// 256-wide tile wastes 3/4 of its MFMAs when N = 64. Here:
//   * B^T (N x K, <= 132 KB) is staged once per workgroup into LDS (transposed on the way in when B is N-major);
//   * each wave owns 16-row blocks of A, strided over the grid; the next block's A fragments (16 B per lane per
//     32-deep K step, straight from HBM into registers in the MFMA operand layout) are in flight while the current
//     block's MFMAs and stores run, and 4 waves per workgroup x several workgroups per CU keep HBM busy;
//   * the product is computed transposed (D = B^T . A^T on v_mfma_f32_16x16x32_bf16) with the B^T rows of two
//     16-column tiles interleaved, so each lane ends up holding 8 consecutive output columns of one row and writes
//     them as one 16-byte store (no LDS round trip for the epilogue).
// Reference role: the cuDNN 1x1-convolution kernels behind paddle/phi/kernels/gpu/conv_kernel.cu.
#include "common.h"

#include <cstdlib>

namespace {
using namespace pa;

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;

union Frag8 {
  bf16x8_t v;
  uint4 u;
  u32x4 w;
};

constexpr int kSkEpiBias = 1;
constexpr int kSkEpiAccum = 2;
constexpr int kSkEpiRelu = 4;

struct SkArgs {
  const uint16_t* a;
  const uint16_t* b;
  uint16_t* c;
  const uint16_t* bias;
  int64_t M, lda, ldb, ldc;
  int b_kmajor;  // 1: B^T given row-major [N][K] (ldb = its row stride); 0: B row-major [K][N]
  int flags;
  float* stats;  // STATS: batch-norm partials [2][chunks][N] of the stored C, chunk = global wave id (conv -> BN)
};

// Batch-norm partials of a wave (conv -> BN fusion): s1 / s2 hold a lane's sums over its rows of the 8 consecutive
// columns c0 = 32 q + 8 g; the 16 lanes of a DPP row (same g) are folded and lane r = 0 stores the wave's chunk.
template <int NQ>
__device__ __forceinline__ void sk_stats_store(float* stats, int64_t chunk, int64_t chunks, int ncols, int lane,
                                               float (&s1)[NQ][8], float (&s2)[NQ][8]) {
  const int g = lane >> 4;
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s1[q][j] = row16_sum(s1[q][j]);
      s2[q][j] = row16_sum(s2[q][j]);
    }
  if ((lane & 15) == 0) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      float* d1 = stats + chunk * ncols + 32 * q + 8 * g;
      float* d2 = stats + (chunks + chunk) * ncols + 32 * q + 8 * g;
      *reinterpret_cast<float4*>(d1) = make_float4(s1[q][0], s1[q][1], s1[q][2], s1[q][3]);
      *reinterpret_cast<float4*>(d1 + 4) = make_float4(s1[q][4], s1[q][5], s1[q][6], s1[q][7]);
      *reinterpret_cast<float4*>(d2) = make_float4(s2[q][0], s2[q][1], s2[q][2], s2[q][3]);
      *reinterpret_cast<float4*>(d2 + 4) = make_float4(s2[q][4], s2[q][5], s2[q][6], s2[q][7]);
    }
  }
}

__device__ __forceinline__ void sk_stats_add(const uint4& o, float* s1, float* s2) {
  const uint32_t w[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float a = lo_bf16(w[j]), b = hi_bf16(w[j]);
    s1[2 * j] += a; s2[2 * j] += a * a;
    s1[2 * j + 1] += b; s2[2 * j + 1] += b * b;
  }
}

template <int NT, int KS, int R, bool STATS = false>
__global__ __launch_bounds__(256) void skinny_gemm_k(SkArgs p) {
  constexpr int N = 16 * NT, K = 32 * KS, LDK = K + 8;  // LDS row of B^T padded by 16 bytes
  extern __shared__ __attribute__((aligned(16))) uint16_t bt[];
  const int tid = threadIdx.x;
  // ---- B^T -> LDS [N][LDK]
  if (p.b_kmajor) {
    for (int idx = tid; idx < N * (K / 8); idx += 256) {
      const int n = idx / (K / 8), kc = idx % (K / 8);
      *reinterpret_cast<uint4*>(bt + n * LDK + kc * 8) =
          *reinterpret_cast<const uint4*>(p.b + (int64_t)n * p.ldb + kc * 8);
    }
  } else {
    for (int idx = tid; idx < K * (N / 8); idx += 256) {
      const int k = idx / (N / 8), nc = idx % (N / 8);
      const uint4 v = *reinterpret_cast<const uint4*>(p.b + (int64_t)k * p.ldb + nc * 8);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bt[(nc * 8 + 2 * j) * LDK + k] = (uint16_t)(w[j] & 0xffffu);
        bt[(nc * 8 + 2 * j + 1) * LDK + k] = (uint16_t)(w[j] >> 16);
      }
    }
  }
  __syncthreads();

  const int wave = tid >> 6, lane = tid & 63, r = lane & 15, g = lane >> 4;
  // a wave iteration covers R 16-row blocks: every B^T fragment read from LDS feeds R MFMAs
  const int64_t nb = (p.M + 16 * R - 1) / (16 * R);
  const int64_t stride = (int64_t)gridDim.x * 4;
  int64_t blk = (int64_t)blockIdx.x * 4 + wave;
  constexpr int NQ = STATS ? NT / 2 : 1;
  float s1[NQ][8], s2[NQ][8];
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) { s1[q][j] = 0.f; s2[q][j] = 0.f; }
  if (blk >= nb) {  // wave-uniform; no barrier follows
    if constexpr (STATS) sk_stats_store<NQ>(p.stats, (int64_t)blockIdx.x * 4 + wave, stride, N, lane, s1, s2);
    return;
  }

  // B^T operand of tile t, K step ks: MFMA row r of tile t is output column 32(t/2) + 8(r/4) + 4(t%2) + r%4
  // (two tiles interleaved so a lane's 8 results are 8 consecutive columns)
  const int brow = 8 * (r >> 2) + (r & 3);
  auto bfrag = [&](int t, int ks) {
    Frag8 f;
    f.u = *reinterpret_cast<const uint4*>(bt + (32 * (t >> 1) + 4 * (t & 1) + brow) * LDK + 32 * ks + 8 * g);
    return f;
  };
  auto load_a = [&](int64_t b, Frag8 (&fr)[R][KS]) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      int64_t row = b * 16 * R + 16 * i + r;
      row = row < p.M ? row : p.M - 1;
      const uint16_t* src = p.a + row * p.lda + 8 * g;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        fr[i][ks].w = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + 32 * ks));
    }
  };

  Frag8 acur[R][KS], anext[R][KS];
  load_a(blk, acur);
  for (; blk < nb; blk += stride) {
    const bool more = blk + stride < nb;
    if (more) load_a(blk + stride, anext);
    f32x4 acc[R][NT];
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const Frag8 bf = bfrag(t, ks);
#pragma unroll
        for (int i = 0; i < R; ++i)
          acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf.v, acur[i][ks].v, acc[i][t], 0, 0, 0);
        if ((t & 1) == 1) __builtin_amdgcn_sched_barrier(0);  // bound the B^T reads in flight (registers)
      }
#pragma unroll
    for (int i = 0; i < R; ++i) {
      // lane: output row (blk*R + i)*16 + r, columns 32q + 8g .. +7 of tile pair q
      const int64_t row = blk * 16 * R + 16 * i + r;
      if (row < p.M) {
        uint16_t* dst = p.c + row * p.ldc;
#pragma unroll
        for (int q = 0; q < NT / 2; ++q) {
          const int c0 = 32 * q + 8 * g;
          float v[8];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[j] = acc[i][2 * q][j];
            v[4 + j] = acc[i][2 * q + 1][j];
          }
          if (p.flags & kSkEpiBias) {
            const uint4 bb = *reinterpret_cast<const uint4*>(p.bias + c0);
            const uint32_t w[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              v[2 * j] += lo_bf16(w[j]);
              v[2 * j + 1] += hi_bf16(w[j]);
            }
          }
          if (p.flags & kSkEpiAccum) {
            const uint4 cc = *reinterpret_cast<const uint4*>(dst + c0);
            const uint32_t w[4] = {cc.x, cc.y, cc.z, cc.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              v[2 * j] += lo_bf16(w[j]);
              v[2 * j + 1] += hi_bf16(w[j]);
            }
          }
          if (p.flags & kSkEpiRelu) {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j], 0.f);
          }
          uint4 o;
          o.x = pack_bf16(v[0], v[1]);
          o.y = pack_bf16(v[2], v[3]);
          o.z = pack_bf16(v[4], v[5]);
          o.w = pack_bf16(v[6], v[7]);
          *reinterpret_cast<uint4*>(dst + c0) = o;
          if constexpr (STATS) sk_stats_add(o, s1[q], s2[q]);
        }
      }
    }
    if (more) {
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) acur[i][ks] = anext[i][ks];
    }
  }
  if constexpr (STATS) sk_stats_store<NQ>(p.stats, (int64_t)blockIdx.x * 4 + wave, stride, N, lane, s1, s2);
}

// Opt a kernel into 160 KB of dynamic LDS once per device (the attribute is per device; one process may drive
// several GPUs). Bit d of `done` marks device d.
__host__ inline void sk_lds_attr(const void* fn, unsigned long long& done) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  const unsigned long long bit = 1ull << (dev & 63);
  if (done & bit) return;
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  done |= bit;
}

// workgroups of a skinny_gemm_k launch (the statistics variant writes 4 chunks per workgroup)
inline int64_t sk_grid(int64_t M, int64_t N, int64_t K) {
  const int R = N <= 128 ? 2 : 1;
  const size_t lds = (size_t)N * (K + 8) * 2;
  const int per_cu = (int)std::min<size_t>(8, (160 * 1024) / lds);
  const int64_t nb = (M + 16 * R - 1) / (16 * R);
  return std::min<int64_t>((nb + 3) / 4, (int64_t)256 * per_cu);
}

template <int NT, int KS, bool STATS = false>
int launch_sk(const SkArgs& a, hipStream_t st) {
  // two 16-row blocks per wave iteration, except N = 256 (its 128 accumulators would leave one wave per SIMD)
  constexpr int R = NT <= 8 ? 2 : 1;
  constexpr int N = 16 * NT, K = 32 * KS;
  const size_t lds = (size_t)N * (K + 8) * 2;
  if (lds > 160 * 1024) return 2;
  const int64_t grid = sk_grid(a.M, N, K);
  static unsigned long long attr_done = 0;  // devices whose LDS limit this instantiation raised
  sk_lds_attr(reinterpret_cast<const void*>(&skinny_gemm_k<NT, KS, R, STATS>), attr_done);
  hipLaunchKernelGGL((skinny_gemm_k<NT, KS, R, STATS>), dim3((unsigned)grid), dim3(256), lds, st, a);
  PA_CHECK_LAUNCH();
  return 0;
}

template <int NT, bool STATS = false>
int launch_sk_k(const SkArgs& a, int64_t K, hipStream_t st) {
  switch (K) {
    case 32: return launch_sk<NT, 1, STATS>(a, st);
    case 64: return launch_sk<NT, 2, STATS>(a, st);
    case 128: return launch_sk<NT, 4, STATS>(a, st);
    case 256: return launch_sk<NT, 8, STATS>(a, st);
    default: return 2;
  }
}

// ---- implicit-GEMM convolution on the same scheme: Y[p, co] = sum_{tap, c} X[pixel(p, tap), c] . W[co, tap, c] for the
// small-channel KxK layers (C = 64, Cout = 64: ResNet-50's 56x56 3x3, forward and — with the flipped, in/out-swapped
// filter — stride-1 data gradient), where the 256-wide tile of the general implicit kernel wastes 3/4 of its MFMAs.
// The filter [Cout][KH][KW][C] is B^T (K = KH*KW*C = 576: 74 KB of LDS, 2 workgroups per CU); a lane's A fragment of
// K step (tap, 32-channel slice) is 16 B of one input pixel, fetched by a raw buffer load whose offset is pushed past
// the buffer's end for taps in the padding (the hardware returns zeros: no branches, no zero page). Neighbouring
// output pixels re-read the same input pixels across taps from L1 / L2; HBM sees X about once.
struct SkConvArgs {
  const uint16_t* x;
  const uint16_t* w;  // [Cout][KH][KW][C]
  uint16_t* y;
  const uint16_t* bias;
  int64_t M;  // N * Ho * Wo
  int H, W, Ho, Wo, stride, pad;
  uint32_t x_bytes;
  int flags;
};

// Per wave iteration: a super-block of R x 16 output pixels, so every B^T fragment read from LDS feeds R MFMAs
// (LDS traffic / R); A moves through a ring of S tap-groups of fragments, the loads of tap g + S - 1 issued while
// tap g's MFMAs run (crossing into the next super-block at the end), so the loop never waits on a whole block.
template <int NT, int C, int KH, int KW, int R, int NW>
__global__ __launch_bounds__(NW * 64) void skinny_conv_k(SkConvArgs p) {
  constexpr int NOUT = 16 * NT, KG = KH * KW, CS = C / 32, K = KG * C, LDK = K + 8, S = 3;
  static_assert(KG % S == 0, "tap count must be a multiple of the ring depth");
  extern __shared__ __attribute__((aligned(16))) uint16_t bt[];
  const int tid = threadIdx.x;
  for (int idx = tid; idx < NOUT * (K / 8); idx += NW * 64) {
    const int n = idx / (K / 8), kc = idx % (K / 8);
    *reinterpret_cast<uint4*>(bt + n * LDK + kc * 8) = *reinterpret_cast<const uint4*>(p.w + (int64_t)n * K + kc * 8);
  }
  __syncthreads();
  const int wave = tid >> 6, lane = tid & 63, r = lane & 15, g = lane >> 4;
  const int64_t nsb = (p.M + 16 * R - 1) / (16 * R);
  const int64_t stride = (int64_t)gridDim.x * NW;
  int64_t sb = (int64_t)blockIdx.x * NW + wave;
  if (sb >= nsb) return;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(p.x), 0, (int)p.x_bytes,
                                                                       0x00020000);
  const int brow = 8 * (r >> 2) + (r & 3);
  // lane's output pixel of block i of super-block s: image base (n*H*W), top-left input row / column of its window
  auto rows = [&](int64_t s, int* rb, int* rh, int* rw) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      int64_t row = s * 16 * R + 16 * i + r;
      row = row < p.M ? row : p.M - 1;
      const int wo = (int)(row % p.Wo);
      const int64_t t1 = row / p.Wo;
      const int ho = (int)(t1 % p.Ho);
      rb[i] = (int)(t1 / p.Ho) * p.H * p.W;
      rh[i] = ho * p.stride - p.pad;
      rw[i] = wo * p.stride - p.pad;
    }
  };
  auto load_tap = [&](const int* rb, const int* rh, const int* rw, int tap, Frag8 (&dst)[R][CS]) {
    const int kh = tap / KW, kw = tap % KW;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int hi = rh[i] + kh, wi = rw[i] + kw;
      const bool ok = (unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W;
      const int off = ok ? ((rb[i] + hi * p.W + wi) * C + 8 * g) * 2 : 0x7ff00000;
#pragma unroll
      for (int cs = 0; cs < CS; ++cs)
        dst[i][cs].w = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, off + 64 * cs, 0, 0));
    }
  };
  Frag8 ring[S][R][CS];
  int cb[R], ch[R], cw[R], nbs[R], nh[R], nw[R];
  rows(sb, cb, ch, cw);
#pragma unroll
  for (int j = 0; j < S - 1; ++j) load_tap(cb, ch, cw, j, ring[j]);
  for (; sb < nsb; sb += stride) {
    const bool more = sb + stride < nsb;
    if (more) rows(sb + stride, nbs, nh, nw);
    f32x4 acc[R][NT];
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kg = 0; kg < KG; ++kg) {
      const int g2 = kg + S - 1;
      if (g2 < KG) load_tap(cb, ch, cw, g2, ring[g2 % S]);
      else if (more) load_tap(nbs, nh, nw, g2 - KG, ring[g2 % S]);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        Frag8 bf[CS];
#pragma unroll
        for (int cs = 0; cs < CS; ++cs)
          bf[cs].u = *reinterpret_cast<const uint4*>(bt + (32 * (t >> 1) + 4 * (t & 1) + brow) * LDK +
                                                     kg * C + 32 * cs + 8 * g);
#pragma unroll
        for (int i = 0; i < R; ++i)
#pragma unroll
          for (int cs = 0; cs < CS; ++cs)
            acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[cs].v, ring[kg % S][i][cs].v, acc[i][t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);  // one tile's B^T fragments live at a time (register budget)
      }
    }
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int64_t row = sb * 16 * R + 16 * i + r;
      if (row < p.M) {
        uint16_t* dst = p.y + row * NOUT;
#pragma unroll
        for (int q = 0; q < NT / 2; ++q) {
          const int c0 = 32 * q + 8 * g;
          float v[8];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[j] = acc[i][2 * q][j];
            v[4 + j] = acc[i][2 * q + 1][j];
          }
          if (p.flags & kSkEpiBias) {
            const uint4 bb = *reinterpret_cast<const uint4*>(p.bias + c0);
            const uint32_t w[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              v[2 * j] += lo_bf16(w[j]);
              v[2 * j + 1] += hi_bf16(w[j]);
            }
          }
          uint4 o;
          o.x = pack_bf16(v[0], v[1]);
          o.y = pack_bf16(v[2], v[3]);
          o.z = pack_bf16(v[4], v[5]);
          o.w = pack_bf16(v[6], v[7]);
          *reinterpret_cast<uint4*>(dst + c0) = o;
        }
      }
    }
    if (more) {
#pragma unroll
      for (int i = 0; i < R; ++i) {
        cb[i] = nbs[i];
        ch[i] = nh[i];
        cw[i] = nw[i];
      }
    }
  }
}

template <int NT, int C, int KH, int KW, int R, int NW>
int launch_skconv(const SkConvArgs& a, hipStream_t st) {
  constexpr int K = KH * KW * C;
  const size_t lds = (size_t)16 * NT * (K + 8) * 2;
  const int per_cu = (int)std::max<size_t>(1, std::min<size_t>(8, (160 * 1024) / lds));
  const int64_t nb = (a.M + 16 * R - 1) / (16 * R);
  const int64_t grid = std::min<int64_t>((nb + NW - 1) / NW, (int64_t)256 * per_cu);
  static unsigned long long attr_done = 0;  // devices whose LDS limit this instantiation raised
  sk_lds_attr(reinterpret_cast<const void*>(&skinny_conv_k<NT, C, KH, KW, R, NW>), attr_done);
  hipLaunchKernelGGL((skinny_conv_k<NT, C, KH, KW, R, NW>), dim3((unsigned)grid), dim3(NW * 64), lds, st, a);
  PA_CHECK_LAUNCH();
  return 0;
}

// ---- 3x3, stride 1, pad 1, C = Cout = 64 on a per-wave LDS halo tile. A wave owns a segment of 16 output pixels of
// one image row; its input window (3 rows x 18 pixels x 64 channels = 6.75 KB) arrives in 7 LDS-DMA instructions
// (global_load_lds_dwordx4, padding pixels fetched from a zero page), so the 9 taps' A fragments are LDS reads
// instead of 18 per-tap HBM / L2 gathers. The 16-byte channel chunks of a pixel are XOR-swizzled by the pixel
// index (conflict-free 16-lane row reads). All 18 A fragments are read into registers before the MFMAs, and the
// next segment's DMA is issued right then, so the window load overlaps this segment's 72 MFMAs.
__device__ __forceinline__ void sk_glds16(const void* g, char* lds_wave_base) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uintptr_t>(lds_wave_base));
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m0) : "memory", "m0");
}

struct SkHaloArgs {
  const uint16_t* x;
  const uint16_t* w;   // [64][3][3][64]
  const uint16_t* zero;  // >= 128 zero bytes
  uint16_t* y;
  const uint16_t* bias;
  int N, H, W;  // output = input size (stride 1, pad 1)
  int flags;
  float* stats;  // STATS: batch-norm partials [2][gridDim.x * NW][64] of y (conv -> BN fusion)
};

template <int NW, int R, bool STATS = false>
__global__ __launch_bounds__(NW * 64) void skinny_conv_halo_k(SkHaloArgs p) {
  // R: segments of 16 R output pixels (R = 2: every B^T fragment read feeds 2 MFMAs, half the LDS B traffic)
  constexpr int C = 64, NT = 4, K = 9 * C, LDK = K + 8, WPX = 16 * R + 2, SLOTS = 3 * WPX * 8;
  constexpr int NI = (SLOTS + 63) / 64, TILE = NI * 1024;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* bt = smem;
  char* tiles = reinterpret_cast<char*>(smem + 16 * NT * LDK);
  const int tid = threadIdx.x;
  for (int idx = tid; idx < 16 * NT * (K / 8); idx += NW * 64) {
    const int n = idx / (K / 8), kc = idx % (K / 8);
    *reinterpret_cast<uint4*>(bt + n * LDK + kc * 8) = *reinterpret_cast<const uint4*>(p.w + (int64_t)n * K + kc * 8);
  }
  __syncthreads();
  const int wave = tid >> 6, lane = tid & 63, r = lane & 15, g = lane >> 4;
  char* tile = tiles + wave * TILE;
  const int segs_row = (p.W + 16 * R - 1) / (16 * R);
  const int64_t nseg = (int64_t)p.N * p.H * segs_row;
  const int64_t stride = (int64_t)gridDim.x * NW;
  int64_t sg = (int64_t)blockIdx.x * NW + wave;
  constexpr int NQ = STATS ? NT / 2 : 1;
  float s1[NQ][8], s2[NQ][8];
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) { s1[q][j] = 0.f; s2[q][j] = 0.f; }
  if (sg >= nseg) {
    if constexpr (STATS) sk_stats_store<NQ>(p.stats, (int64_t)blockIdx.x * NW + wave, stride, 16 * NT, lane, s1, s2);
    return;
  }
  // DMA of segment s's window: slot q = 64 i + lane (q < SLOTS) -> LDS byte 16 q = (row, px, swizzled chunk)
  auto load_window = [&](int64_t s) {
    const int seg = (int)(s % segs_row);
    const int64_t t1 = s / segs_row;
    const int ho = (int)(t1 % p.H);
    const int n = (int)(t1 / p.H);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = 64 * i + lane;
      const int row = q / (8 * WPX), px = (q % (8 * WPX)) >> 3, chs = q & 7;
      const int hi = ho - 1 + row, wi = 16 * R * seg - 1 + px;
      const int ch = chs ^ (px & 7);
      const bool ok = q < SLOTS && (unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W;
      const uint16_t* src = ok ? p.x + (((int64_t)n * p.H + hi) * p.W + wi) * C + 8 * ch : p.zero + 8 * (q & 7);
      sk_glds16(src, tile + 1024 * i);
    }
  };
  const int brow = 8 * (r >> 2) + (r & 3);
  load_window(sg);
  for (; sg < nseg; sg += stride) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's window has landed (its own DMA only)
    Frag8 af[R][9][2];
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int kh = tap / 3, kw = tap % 3, px = 16 * i + r + kw;
#pragma unroll
        for (int cs = 0; cs < 2; ++cs) {
          const int ch = (4 * cs + g) ^ (px & 7);
          af[i][tap][cs].u = *reinterpret_cast<const uint4*>(tile + ((kh * WPX + px) * 8 + ch) * 16);
        }
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // window consumed: the next DMA may overwrite it
    const int64_t cur = sg;
    if (sg + stride < nseg) load_window(sg + stride);
    f32x4 acc[R][NT];
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
#pragma unroll
        for (int cs = 0; cs < 2; ++cs) {
          Frag8 bf;
          bf.u = *reinterpret_cast<const uint4*>(bt + (32 * (t >> 1) + 4 * (t & 1) + brow) * LDK + tap * C + 32 * cs +
                                                 8 * g);
#pragma unroll
          for (int i = 0; i < R; ++i)
            acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf.v, af[i][tap][cs].v, acc[i][t], 0, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    const int seg = (int)(cur % segs_row);
    const int64_t t1 = cur / segs_row;  // n * H + ho
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int wo = 16 * R * seg + 16 * i + r;
      if (wo < p.W) {
        uint16_t* dst = p.y + (t1 * p.W + wo) * (16 * NT);
#pragma unroll
        for (int q = 0; q < NT / 2; ++q) {
          const int c0 = 32 * q + 8 * g;
          float v[8];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[j] = acc[i][2 * q][j];
            v[4 + j] = acc[i][2 * q + 1][j];
          }
          if (p.flags & kSkEpiBias) {
            const uint4 bb = *reinterpret_cast<const uint4*>(p.bias + c0);
            const uint32_t w[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              v[2 * j] += lo_bf16(w[j]);
              v[2 * j + 1] += hi_bf16(w[j]);
            }
          }
          uint4 o;
          o.x = pack_bf16(v[0], v[1]);
          o.y = pack_bf16(v[2], v[3]);
          o.z = pack_bf16(v[4], v[5]);
          o.w = pack_bf16(v[6], v[7]);
          *reinterpret_cast<uint4*>(dst + c0) = o;
          if constexpr (STATS) sk_stats_add(o, s1[q], s2[q]);
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (STATS) sk_stats_store<NQ>(p.stats, (int64_t)blockIdx.x * NW + wave, stride, 16 * NT, lane, s1, s2);
}

template <int NW, int R>
int64_t halo_grid(int64_t N, int64_t H, int64_t W) {
  constexpr int NI = (3 * (16 * R + 2) * 8 + 63) / 64;
  const size_t lds = (size_t)64 * (9 * 64 + 8) * 2 + (size_t)NW * NI * 1024;
  const int64_t nseg = N * H * ((W + 16 * R - 1) / (16 * R));
  const int per_cu = (int)std::max<size_t>(1, (160 * 1024) / lds);
  return std::min<int64_t>((nseg + NW - 1) / NW, (int64_t)256 * per_cu);
}

template <int NW, int R, bool STATS = false>
int launch_halo(const SkHaloArgs& a, hipStream_t st) {
  constexpr int NI = (3 * (16 * R + 2) * 8 + 63) / 64;
  const size_t lds = (size_t)64 * (9 * 64 + 8) * 2 + (size_t)NW * NI * 1024;
  if (lds > 160 * 1024) return 2;
  const int64_t grid = halo_grid<NW, R>(a.N, a.H, a.W);
  static unsigned long long attr_done = 0;
  sk_lds_attr(reinterpret_cast<const void*>(&skinny_conv_halo_k<NW, R, STATS>), attr_done);
  hipLaunchKernelGGL((skinny_conv_halo_k<NW, R, STATS>), dim3((unsigned)grid), dim3(NW * 64), lds, st, a);
  PA_CHECK_LAUNCH();
  return 0;
}

// ---- 3x3 stride-1 pad-1 weight gradient, C = Cout = 64: dW[co][kh][kw][c] = sum_px dY[px][co] X[px + tap][c].
// A workgroup of 9 waves (one per tap) walks 32-pixel row pieces of its share of the image rows: the piece's dY tile
// [32 px][64 co] and input window [3 rows][34 px][64 c] (16.75 KB) arrive by LDS-DMA into a double buffer; both MFMA
// operands are pixel-contiguous columns of those row-major tiles, read with ds_read_b64_tr_b16 (the hardware
// transpose). Each wave accumulates its tap's 64 x 64 block (16 tiles of 16x16) over the pieces and writes an fp32
// slab per workgroup; the slabs are summed afterwards (split over pixels).
typedef short s16x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ s16x4_t sk_lds_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4_t*)(reinterpret_cast<uintptr_t>(p)));
}

// 16-byte chunk swizzle of a 128-byte pixel row of the weight-gradient tiles: pixels 4 apart (the rows of one
// transposed read) and 8 apart (the two 16-lane groups of a half-wave) land on different banks
__device__ __forceinline__ int wg_swz(int px) { return (px & 3) ^ (((px >> 3) & 1) << 2); }  // conflict-free (bank model)

struct SkWgArgs {
  const uint16_t* x;
  const uint16_t* dy;
  const uint16_t* zero;
  float* ws;  // [gridDim.x][64][9][64]
  int N, H, W;
};

__global__ __launch_bounds__(576) void skinny_wgrad3_k(SkWgArgs p) {
  // 1152 DMA slots of 16 B per stage; NST stages: pieces s+1 .. s+NST-1 are in flight while piece s is multiplied
  // (the DMA latency under load, ~2 us, is several pieces' worth of MFMA work)
  constexpr int C = 64, DY_B = 32 * 128, WIN_B = 3 * 34 * 128, STAGE = 18 * 1024, NST = 4;
  __shared__ __attribute__((aligned(16))) char lds[NST * STAGE];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int l16 = lane & 15, g = lane >> 4, q = l16 >> 2, pp = l16 & 3;
  const int pieces_row = (p.W + 31) / 32;
  const int64_t npieces = (int64_t)p.N * p.H * pieces_row;
  const int64_t per = (npieces + gridDim.x - 1) / gridDim.x;
  const int64_t p0 = (int64_t)blockIdx.x * per;
  const int64_t p1 = p0 + per < npieces ? p0 + per : npieces;
  // DMA of piece s into stage st: slots 0..255 = dY tile (px, chunk), 256..1071 = window (row, px, chunk); the
  // remaining slots load the zero page into the stage's tail
  auto load_piece = [&](int64_t s, int st) {
    const int pc = (int)(s % pieces_row);
    const int64_t t1 = s / pieces_row;
    const int ho = (int)(t1 % p.H);
    const int n = (int)(t1 / p.H);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int slot = 576 * i + tid;  // wave-contiguous 1 KB pieces: slot = 64 * (9 i + wave) + lane
      const uint16_t* src = p.zero + 8 * (slot & 7);
      if (slot < 256) {
        const int px = slot >> 3, ch = (slot & 7) ^ wg_swz(px), wo = 32 * pc + px;
        if (wo < p.W) src = p.dy + (((int64_t)n * p.H + ho) * p.W + wo) * C + 8 * ch;
      } else if (slot < 256 + 816) {
        const int u = slot - 256, row = u / 272, px = (u % 272) >> 3, ch = (u & 7) ^ wg_swz(px);
        const int hi = ho - 1 + row, wi = 32 * pc - 1 + px;
        if ((unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W)
          src = p.x + (((int64_t)n * p.H + hi) * p.W + wi) * C + 8 * ch;
      }
      sk_glds16(src, lds + st * STAGE + 1024 * (9 * i + wave));
    }
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int kh = wave / 3, kw = wave % 3;
#pragma unroll
  for (int j = 0; j < NST - 1; ++j)
    if (p0 + j < p1) load_piece(p0 + j, j);
  for (int64_t s = p0; s < p1; ++s) {
    const int st = (int)((s - p0) % NST);
    // this wave's DMA of piece s has landed once at most 2 per younger piece in flight remain outstanding
    const int64_t younger = p1 - 1 - s < NST - 2 ? p1 - 1 - s : NST - 2;
    if (younger >= 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every wave's DMA of piece s landed; stage (s - 1) % NST was read in the last step
    if (s + NST - 1 < p1) load_piece(s + NST - 1, (int)((s + NST - 1 - p0) % NST));
    const char* dyt = lds + st * STAGE;
    const char* win = dyt + DY_B;
    // k (pixel) = 8 g + 4 h + element; A = dY^T (row co), B = window pixels (column c)
    Frag8 af[4], bfr[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int pa = 8 * g + 4 * h + q, pb = pa + kw;  // dY tile pixel, window pixel of this lane's row
        const s16x4_t va = sk_lds_tr(dyt + pa * 128 + (((2 * t + (pp >> 1)) ^ wg_swz(pa)) << 4) + 8 * (pp & 1));
        const s16x4_t vb = sk_lds_tr(win + (kh * 34 + pb) * 128 + (((2 * t + (pp >> 1)) ^ wg_swz(pb)) << 4) +
                                     8 * (pp & 1));
        af[t].u = h == 0 ? make_uint4(__builtin_bit_cast(uint2, va).x, __builtin_bit_cast(uint2, va).y, af[t].u.z,
                                      af[t].u.w)
                         : make_uint4(af[t].u.x, af[t].u.y, __builtin_bit_cast(uint2, va).x,
                                      __builtin_bit_cast(uint2, va).y);
        bfr[t].u = h == 0 ? make_uint4(__builtin_bit_cast(uint2, vb).x, __builtin_bit_cast(uint2, vb).y, bfr[t].u.z,
                                       bfr[t].u.w)
                          : make_uint4(bfr[t].u.x, bfr[t].u.y, __builtin_bit_cast(uint2, vb).x,
                                       __builtin_bit_cast(uint2, vb).y);
      }
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b)
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a].v, bfr[b].v, acc[a][b], 0, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // slab [64 co][9 taps][64 c]: lane holds rows co = 16 a + 4 g + i, column c = 16 b + l16
  float* slab = p.ws + (int64_t)blockIdx.x * (64 * 9 * 64);
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        slab[((16 * a + 4 * g + i) * 9 + wave) * 64 + 16 * b + l16] = acc[a][b][i];
}

}  // namespace

// 1 if (N, K) has an instantiation (N in {32, 64, 128, 256}, K in {32, 64, 128, 256}).
PA_EXPORT int pa_gemm_skinny_ok(int64_t N, int64_t K) {
  return (N == 32 || N == 64 || N == 128 || N == 256) && (K == 32 || K == 64 || K == 128 || K == 256);
}

// C[M, N] (+)= A[M, K] . B (+ bias) (relu). A row-major (lda), C row-major (ldc), 16-byte aligned rows;
// b_kmajor = 1: b is B^T row-major [N][K] (ldb); 0: b is B row-major [K][N] (ldb). flags: 1 bias, 2 accumulate
// onto C, 4 relu. Returns 2 for an unsupported (N, K).
PA_EXPORT int pa_gemm_skinny(const void* a, const void* b, void* c, const void* bias, int64_t M, int64_t N, int64_t K,
                             int64_t lda, int64_t ldb, int64_t ldc, int b_kmajor, int flags, void* stream) {
  if (M <= 0) return 0;
  if (!pa_gemm_skinny_ok(N, K)) return 2;
  SkArgs g{static_cast<const uint16_t*>(a), static_cast<const uint16_t*>(b), static_cast<uint16_t*>(c),
           static_cast<const uint16_t*>(bias), M, lda, ldb, ldc, b_kmajor, flags};
  hipStream_t st = static_cast<hipStream_t>(stream);
  switch (N) {
    case 32: return launch_sk_k<2>(g, K, st);
    case 64: return launch_sk_k<4>(g, K, st);
    case 128: return launch_sk_k<8>(g, K, st);
    case 256: return launch_sk_k<16>(g, K, st);
    default: return 2;
  }
}

// Statistics chunks of pa_gemm_skinny_stats for (M, N, K) (0: no statistics variant, N > 128).
PA_EXPORT int64_t pa_gemm_skinny_stats_chunks(int64_t M, int64_t N, int64_t K) {
  if (!pa_gemm_skinny_ok(N, K) || N > 128 || M <= 0) return 0;
  return sk_grid(M, N, K) * 4;
}

// pa_gemm_skinny (no accumulate / relu) that also writes the batch-norm partials of the stored C to stats
// ([2][chunks][N] fp32, chunks = pa_gemm_skinny_stats_chunks) for the following BN (conv -> BN fusion).
PA_EXPORT int pa_gemm_skinny_stats(const void* a, const void* b, void* c, const void* bias, int64_t M, int64_t N,
                                   int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int b_kmajor, float* stats,
                                   void* stream) {
  if (M <= 0) return 0;
  if (!pa_gemm_skinny_ok(N, K) || N > 128 || !stats) return 2;
  SkArgs g{static_cast<const uint16_t*>(a), static_cast<const uint16_t*>(b), static_cast<uint16_t*>(c),
           static_cast<const uint16_t*>(bias), M, lda, ldb, ldc, b_kmajor, bias ? kSkEpiBias : 0, stats};
  hipStream_t st = static_cast<hipStream_t>(stream);
  switch (N) {
    case 32: return launch_sk_k<2, true>(g, K, st);
    case 64: return launch_sk_k<4, true>(g, K, st);
    case 128: return launch_sk_k<8, true>(g, K, st);
    default: return 2;
  }
}

// 1 if the skinny implicit convolution has an instantiation for (C, Cout, KH, KW).
PA_EXPORT int pa_conv_skinny_ok(int64_t C, int64_t Cout, int64_t KH, int64_t KW) {
  return C == 64 && Cout == 64 && KH == 3 && KW == 3;
}

// NHWC convolution y[N, Ho, Wo, Cout] = conv(x[N, H, W, C], w[Cout][KH][KW][C]) (+ bias), symmetric padding, no
// dilation, on the skinny implicit-GEMM kernels (stride 1 / pad 1: the LDS halo-tile kernel; zero_page: >= 128 zero
// bytes it reads for padding pixels). x must be below 2 GB (32-bit buffer offsets). Returns 2 if the
// shape has no instantiation.
PA_EXPORT int pa_conv_skinny(const void* x, const void* w, const void* bias, void* y, const void* zero_page, int64_t N,
                             int64_t H, int64_t W, int64_t C, int64_t Cout, int64_t KH, int64_t KW, int64_t stride,
                             int64_t pad, int64_t Ho, int64_t Wo, void* stream) {
  if (!pa_conv_skinny_ok(C, Cout, KH, KW)) return 2;
  const int64_t xb = N * H * W * C * 2;
  if (xb >= ((int64_t)1 << 31) - (1 << 21)) return 2;
  SkConvArgs a{static_cast<const uint16_t*>(x), static_cast<const uint16_t*>(w), static_cast<uint16_t*>(y),
               static_cast<const uint16_t*>(bias), N * Ho * Wo, (int)H, (int)W, (int)Ho, (int)Wo, (int)stride, (int)pad,
               (uint32_t)xb, bias ? kSkEpiBias : 0};
  if (a.M <= 0) return 0;
  if (stride == 1 && pad == 1 && Ho == H && Wo == W && zero_page != nullptr) {
    // PA_SKCONV_HALO (measurement): 0 = the per-tap gather kernel below, 8 = 8 waves per workgroup; default 12 waves
    // (3 per SIMD, 160 KB of LDS: 89.7 vs 96.3 us with 8, profiles/conv3x3_skinny_sweep_r3.log)
    static const int halo = [] {
      const char* e = getenv("PA_SKCONV_HALO");
      return e ? atoi(e) : 12;
    }();
    if (halo) {
      SkHaloArgs h{static_cast<const uint16_t*>(x), static_cast<const uint16_t*>(w),
                   static_cast<const uint16_t*>(zero_page), static_cast<uint16_t*>(y),
                   static_cast<const uint16_t*>(bias), (int)N, (int)H, (int)W, bias ? kSkEpiBias : 0};
      hipStream_t hs = static_cast<hipStream_t>(stream);
      if (halo == 8) return launch_halo<8, 1>(h, hs);
      if (halo == 2) return launch_halo<6, 2>(h, hs);  // 32-pixel segments, 6 waves (measurement)
      return launch_halo<12, 1>(h, hs);
    }
  }
  static const int cfg = [] {  // PA_SKCONV_CFG (measurement): 0 = R2 x 4 waves, 1 = R1 x 8, 2 = R2 x 8, 3 = R1 x 4
    const char* e = getenv("PA_SKCONV_CFG");
    return e ? atoi(e) : 0;
  }();
  hipStream_t st = static_cast<hipStream_t>(stream);
  switch (cfg) {
    case 1: return launch_skconv<4, 64, 3, 3, 1, 8>(a, st);
    case 2: return launch_skconv<4, 64, 3, 3, 2, 8>(a, st);
    case 3: return launch_skconv<4, 64, 3, 3, 1, 4>(a, st);
    default: return launch_skconv<4, 64, 3, 3, 2, 4>(a, st);
  }
}

// Statistics chunks of pa_conv_skinny_stats (the 3x3 stride-1 pad-1 halo kernel, 12 waves per workgroup).
PA_EXPORT int64_t pa_conv_skinny_stats_chunks(int64_t N, int64_t H, int64_t W) { return halo_grid<12, 1>(N, H, W) * 12; }

// 3x3 stride-1 pad-1 C = Cout = 64 convolution on the halo kernel that also writes the batch-norm partials of y
// ([2][chunks][64], chunks = pa_conv_skinny_stats_chunks) for the following BN (conv -> BN fusion).
PA_EXPORT int pa_conv_skinny_stats(const void* x, const void* w, const void* bias, void* y, const void* zero_page,
                                   int64_t N, int64_t H, int64_t W, float* stats, void* stream) {
  if (!zero_page || !stats || N <= 0) return 2;
  if (N * H * W * 64 * 2 >= ((int64_t)1 << 31) - (1 << 21)) return 2;
  SkHaloArgs h{static_cast<const uint16_t*>(x), static_cast<const uint16_t*>(w),
               static_cast<const uint16_t*>(zero_page), static_cast<uint16_t*>(y),
               static_cast<const uint16_t*>(bias), (int)N, (int)H, (int)W, bias ? kSkEpiBias : 0, stats};
  return launch_halo<12, 1, true>(h, static_cast<hipStream_t>(stream));
}

// dW partial slabs of the 3x3 stride-1 pad-1 C = Cout = 64 weight gradient (skinny_wgrad3_k): ws holds `splits`
// fp32 [64][3][3][64] slabs (sum them for dW in [Cout][KH][KW][C]). Returns 2 for other shapes.
PA_EXPORT int pa_conv_skinny_wgrad(const void* x, const void* dy, const void* zero_page, float* ws, int64_t N, int64_t H,
                                   int64_t W, int64_t C, int64_t Cout, int64_t splits, void* stream) {
  if (C != 64 || Cout != 64 || splits < 1 || zero_page == nullptr) return 2;
  SkWgArgs a{static_cast<const uint16_t*>(x), static_cast<const uint16_t*>(dy), static_cast<const uint16_t*>(zero_page),
             ws, (int)N, (int)H, (int)W};
  hipLaunchKernelGGL(skinny_wgrad3_k, dim3((unsigned)splits), dim3(576), 0, static_cast<hipStream_t>(stream), a);
  PA_CHECK_LAUNCH();
  return 0;
}
