// OCP fp8 GEMM on the gfx950 block-scaled MFMA (v_mfma_scale_f32_16x16x128_f8f6f4) with a fused
// epilogue: C[M,N] = act(alpha * A[M,K] . B[N,K]^T + bias[N]), C in fp16 or bf16.
// Reference behaviour: python/paddle/tensor/linalg.py fp8_fp8_half_gemm_fused and
// paddle/phi/kernels/fusion/fp8_gemm/ (cutlass fp8 GEMM with bias + identity / relu / gelu epilogue).
//
// A and B are both K-major (x [M][K] and the weight stored [N][K], transpose_y=True in the reference);
// the Python wrapper makes other layouts K-major first. Either operand may be e4m3 or e5m2
// (cbsz / blgp format codes 0 / 1). The per-tensor scale of the reference is `alpha`, applied in the
// epilogue; the MFMA's per-32-element E8M0 block scales are all 1.0 (exponent 127), so the
// instruction runs the MX-fp8 rate (2x bf16 per clock) on plain per-tensor-scaled data.
//
// Structure: the bf16 generic kernel's (gemm.hip gemm_bf16_kernel) at the same bytes: 256 x 256 tiles,
// 128 k (= 128 bytes) per stage, 8 waves as 2 (M) x 4 (N) with a 128 x 64 wave tile, two LDS stages of
// 64 KiB fed by global_load_lds_dwordx4, 16-B chunk XOR swizzle on 128-B rows. Fragments: lane l holds row
// (l & 15) and the 32 k-bytes [32 (l >> 4), 32 (l >> 4) + 32) for A and for B alike, so any k permutation
// the instruction applies inside its 128-k block is the same on both operands (and with unit block scales
// no scale placement matters). Operands are swapped (D = B-frag x A-frag) so a lane ends with 4
// consecutive columns of one output row.
#include "common.h"

using namespace pa;

namespace {

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int kTile = 256;
constexpr int kKB = 128;  // bytes (= fp8 elements) of k per stage
constexpr int kOpBytes = kTile * kKB;
constexpr int kStage = 2 * kOpBytes;

struct Fp8Args {
  const uint8_t* a;
  const uint8_t* b;
  void* c;
  const uint16_t* bias;
  int64_t lda, ldb, ldc;
  int M, N, K;
  int tiles_m, tiles_n;
  float alpha;
  int act;  // 0 identity, 1 gelu (erf), 2 relu
};

__device__ __forceinline__ void glds16(const void* g, char* lds_wave_base) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uintptr_t>(lds_wave_base));
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m0) : "memory", "m0");
}

// one operand tile: 256 rows x 128 k-bytes -> LDS image [256][128 B], chunk c of row r at c ^ ((r >> 1) & 7)
__device__ __forceinline__ void stage_op(const uint8_t* __restrict__ g, int64_t ld, int r0, int rmax, int k0,
                                         char* img, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = i * 8 + wave;  // 8 rows x 128 B per wave instruction
    const int row = q * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ ((row >> 1) & 7);
    int gr = r0 + row;
    gr = gr < rmax ? gr : rmax - 1;
    glds16(g + (int64_t)gr * ld + k0 + lc * 16, img + q * 1024);
  }
}

__device__ __forceinline__ i32x8 frag(const char* img, int rbase, int lane) {
  const int row = rbase + (lane & 15);
  const int c0 = 2 * (lane >> 4), sw = (row >> 1) & 7;
  const uint4 lo = *reinterpret_cast<const uint4*>(img + row * 128 + ((c0 ^ sw) << 4));
  const uint4 hi = *reinterpret_cast<const uint4*>(img + row * 128 + (((c0 + 1) ^ sw) << 4));
  i32x8 f;
  f[0] = (int)lo.x; f[1] = (int)lo.y; f[2] = (int)lo.z; f[3] = (int)lo.w;
  f[4] = (int)hi.x; f[5] = (int)hi.y; f[6] = (int)hi.z; f[7] = (int)hi.w;
  return f;
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

__device__ __forceinline__ float act_f(float v, int act) {
  if (act == 1) return 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
  if (act == 2) return v > 0.f ? v : 0.f;
  return v;
}

template <int FA, int FB, bool OUT_F16>
__global__ __launch_bounds__(512, 1) void gemm_fp8_kernel(Fp8Args p) {
  constexpr int MR = 8, NR = 4;  // wave tile 128 x 64
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 2, wn = wave & 3;

  const int nwg = p.tiles_m * p.tiles_n;
  const int pid = xcd_remap((int)blockIdx.x, nwg);
  constexpr int GM = 8;
  const int per_group = GM * p.tiles_n;
  const int first_m = (pid / per_group) * GM;
  const int gsz = min(p.tiles_m - first_m, GM);
  const int tm = first_m + (pid % per_group) % gsz;
  const int tn = (pid % per_group) / gsz;
  const int m0 = tm * kTile, n0 = tn * kTile;

  f32x4 acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto stage_tile = [&](int t, int buf) {
    char* base = smem + buf * kStage;
    stage_op(p.a, p.lda, m0, p.M, t * kKB, base, wave, lane);
    stage_op(p.b, p.ldb, n0, p.N, t * kKB, base + kOpBytes, wave, lane);
  };

  const int nk = p.K / kKB;
  stage_tile(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    if (t + 1 < nk) stage_tile(t + 1, cur ^ 1);
    const char* aimg = smem + cur * kStage;
    const char* bimg = aimg + kOpBytes;
    i32x8 bf[NR];
#pragma unroll
    for (int j = 0; j < NR; ++j) bf[j] = frag(bimg, wn * 64 + j * 16, lane);
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      const i32x8 af = frag(aimg, wm * 128 + i * 16, lane);
#pragma unroll
      for (int j = 0; j < NR; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bf[j], af, acc[i][j], FB, FA, 0, 127, 0, 127);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // lane holds C[m = mrow0 + i*16][n = ncol0 + j*16 + 0..3]
  const int mrow0 = m0 + wm * 128 + (lane & 15);
  const int ncol0 = n0 + wn * 64 + 4 * (lane >> 4);
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const int n = ncol0 + j * 16;
    if (n >= p.N) continue;  // N % 4 == 0 (launcher)
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (p.bias) {
      const uint2 braw = *reinterpret_cast<const uint2*>(p.bias + n);
      if (OUT_F16) {
        bv[0] = lo_f16(braw.x); bv[1] = hi_f16(braw.x); bv[2] = lo_f16(braw.y); bv[3] = hi_f16(braw.y);
      } else {
        bv[0] = lo_bf16(braw.x); bv[1] = hi_bf16(braw.x); bv[2] = lo_bf16(braw.y); bv[3] = hi_bf16(braw.y);
      }
    }
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      const int m = mrow0 + i * 16;
      if (m >= p.M) continue;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = act_f(acc[i][j][e] * p.alpha + bv[e], p.act);
      uint2* cp = reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(p.c) + (int64_t)m * p.ldc + n);
      *cp = OUT_F16 ? make_uint2(pack_f16(v[0], v[1]), pack_f16(v[2], v[3]))
                    : make_uint2(pack_bf16(v[0], v[1]), pack_bf16(v[2], v[3]));
    }
  }
}

template <int FA, int FB, bool F16>
int launch(const Fp8Args& g, hipStream_t st) {
  static bool attr = false;
  constexpr int smem = 2 * kStage;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_fp8_kernel<FA, FB, F16>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              smem);
    attr = true;
  }
  hipLaunchKernelGGL((gemm_fp8_kernel<FA, FB, F16>), dim3(g.tiles_m * g.tiles_n), dim3(512), smem, st, g);
  return (int)hipGetLastError();
}

template <int FA, int FB>
int launch_out(const Fp8Args& g, int out_f16, hipStream_t st) {
  return out_f16 ? launch<FA, FB, true>(g, st) : launch<FA, FB, false>(g, st);
}

}  // namespace

// fmt_a / fmt_b: 0 = e4m3fn, 1 = e5m2. act: 0 identity, 1 gelu, 2 relu. bias: [N] in the output dtype or null.
// Returns 1 for an unsupported shape / stride (K % 128, N % 4, leading dims % 16 bytes).
PA_EXPORT int pa_gemm_fp8(const void* a, const void* b, void* c, const void* bias, int64_t M, int64_t N, int64_t K,
                          int64_t lda, int64_t ldb, int64_t ldc, int fmt_a, int fmt_b, float alpha, int act,
                          int out_f16, hipStream_t st) {
  if (K % kKB != 0 || N % 4 != 0 || lda % 16 != 0 || ldb % 16 != 0 || ldc % 4 != 0) return 1;
  if (fmt_a < 0 || fmt_a > 1 || fmt_b < 0 || fmt_b > 1 || act < 0 || act > 2) return 1;
  if (M <= 0 || N <= 0) return 0;
  Fp8Args g{};
  g.a = (const uint8_t*)a; g.b = (const uint8_t*)b; g.c = c; g.bias = (const uint16_t*)bias;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.M = (int)M; g.N = (int)N; g.K = (int)K;
  g.tiles_m = (int)((M + kTile - 1) / kTile);
  g.tiles_n = (int)((N + kTile - 1) / kTile);
  g.alpha = alpha; g.act = act;
  if (fmt_a == 0 && fmt_b == 0) return launch_out<0, 0>(g, out_f16, st);
  if (fmt_a == 0 && fmt_b == 1) return launch_out<0, 1>(g, out_f16, st);
  if (fmt_a == 1 && fmt_b == 0) return launch_out<1, 0>(g, out_f16, st);
  return launch_out<1, 1>(g, out_f16, st);
}
