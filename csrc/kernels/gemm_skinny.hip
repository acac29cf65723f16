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
};

template <int NT, int KS>
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
  const int64_t nb = (p.M + 15) / 16;
  const int64_t stride = (int64_t)gridDim.x * 4;
  int64_t blk = (int64_t)blockIdx.x * 4 + wave;
  if (blk >= nb) return;  // wave-uniform; no barrier follows

  // B^T operand of tile t, K step ks: MFMA row r of tile t is output column 32(t/2) + 8(r/4) + 4(t%2) + r%4
  // (two tiles interleaved so a lane's 8 results are 8 consecutive columns)
  const int brow = 8 * (r >> 2) + (r & 3);
  auto bfrag = [&](int t, int ks) {
    Frag8 f;
    f.u = *reinterpret_cast<const uint4*>(bt + (32 * (t >> 1) + 4 * (t & 1) + brow) * LDK + 32 * ks + 8 * g);
    return f;
  };
  auto load_a = [&](int64_t b, Frag8* fr) {
    int64_t row = b * 16 + r;
    row = row < p.M ? row : p.M - 1;
    const uint16_t* src = p.a + row * p.lda + 8 * g;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) fr[ks].w = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + 32 * ks));
  };

  Frag8 acur[KS], anext[KS];
  load_a(blk, acur);
  for (; blk < nb; blk += stride) {
    const bool more = blk + stride < nb;
    if (more) load_a(blk + stride, anext);
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfrag(t, ks).v, acur[ks].v, acc[t], 0, 0, 0);
        if ((t & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // bound the B^T reads in flight (registers)
      }
    // lane: output row blk*16 + r, columns 32q + 8g .. +7 of tile pair q
    const int64_t row = blk * 16 + r;
    if (row < p.M) {
      uint16_t* dst = p.c + row * p.ldc;
#pragma unroll
      for (int q = 0; q < NT / 2; ++q) {
        const int c0 = 32 * q + 8 * g;
        float v[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[i] = acc[2 * q][i];
          v[4 + i] = acc[2 * q + 1][i];
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
      }
    }
    if (more) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) acur[ks] = anext[ks];
    }
  }
}

template <int NT, int KS>
int launch_sk(const SkArgs& a, hipStream_t st) {
  constexpr int N = 16 * NT, K = 32 * KS;
  const size_t lds = (size_t)N * (K + 8) * 2;
  if (lds > 160 * 1024) return 2;
  const int per_cu = (int)std::min<size_t>(8, (160 * 1024) / lds);
  const int64_t nb = (a.M + 15) / 16;
  const int64_t grid = std::min<int64_t>((nb + 3) / 4, (int64_t)256 * per_cu);
  static bool attr_set = false;  // dynamic LDS above 64 KB needs the attribute
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&skinny_gemm_k<NT, KS>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  hipLaunchKernelGGL((skinny_gemm_k<NT, KS>), dim3((unsigned)grid), dim3(256), lds, st, a);
  PA_CHECK_LAUNCH();
  return 0;
}

template <int NT>
int launch_sk_k(const SkArgs& a, int64_t K, hipStream_t st) {
  switch (K) {
    case 32: return launch_sk<NT, 1>(a, st);
    case 64: return launch_sk<NT, 2>(a, st);
    case 128: return launch_sk<NT, 4>(a, st);
    case 256: return launch_sk<NT, 8>(a, st);
    default: return 2;
  }
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
