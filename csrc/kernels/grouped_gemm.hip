// Grouped (MoE) GEMM and token routing for gfx950 — every expert in ONE launch, no host sync.
// Reference behaviour: paddle/phi/kernels/fusion/cutlass/fused_moe_kernel.cu (grouped GEMM over experts),
// python/paddle/incubate/nn/functional/fused_moe.py:20, incubate/distributed/models/moe/moe_layer.py
// (tokens dispatched to experts, outputs combined with the gate weights).
//
// Tokens are sorted by expert (pa_moe_route below): rows offs[e] .. offs[e+1] of the sorted activations
// belong to expert e. The three products of a per-expert linear layer y_e = x_e . W_e (W_e [K, N]) are
//   MODE 0  forward  Y[rows_e]  = X[rows_e] . W_e        A K-major (rows = tokens), B MN-major
//   MODE 1  dgrad    dX[rows_e] = dY[rows_e] . W_e^T     A K-major, B K-major (W_e read as [K rows][N])
//   MODE 2  wgrad    dW_e = X[rows_e]^T . dY[rows_e]     A MN-major, B MN-major, reduction over the
//                                                         expert's tokens (its own length)
// Forward / dgrad launch an upper bound of M tiles (ceil(T / BM) + E for T routed tokens, no count on the
// host); every workgroup finds its expert by walking the device offsets and the ones past the last tile
// exit at once. Wgrad launches E x tiles(K) x tiles(N) workgroups; the token tail of each expert is read
// from a 16-byte zero page so the reduction needs no masking.
//
// Tiles: 128 x 128 x 64 with 4 waves (2 x 2, 64 x 64 per wave) for small experts, 256 x 256 x 64 with 8
// waves (2 x 4, 128 x 64 per wave) when the experts hold >= 1024 rows on average; v_mfma_f32_16x16x32_bf16
// with operands swapped so a lane ends with 4 consecutive output columns of one row. Both operands go
// global -> LDS with global_load_lds_dwordx4 into two stages, K-major images XOR-swizzled per 16-B chunk,
// MN-major images read with ds_read_b64_tr_b16.
#include "common.h"

using namespace pa;

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;

union Frag8 {
  bf16x8_t v;
  uint4 u;
  s16x4 h[2];
};

constexpr int kK = 64;  // k per stage
enum : int { kGBias = 1, kGAccum = 2, kGOutF32 = 4 };

struct GGArgs {
  const uint16_t* a;
  const uint16_t* b;
  void* c;
  const uint16_t* bias;
  const uint16_t* zero;  // 16 zero bytes (wgrad token tail)
  const int* offs;       // [E + 1] row offsets of the sorted tokens
  int64_t lda, ldb, ldc;
  int64_t b_es, c_es, bias_es;  // per-expert strides (elements) of B, C (wgrad) and bias
  int E, M, N, K;               // C is M x N (forward / dgrad: M = rows of the expert), reduction K
  int tiles_m, tiles_n;
  int flags;
};

__device__ __forceinline__ void glds16(const void* g, char* lds_wave_base) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uintptr_t>(lds_wave_base));
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m0) : "memory", "m0");
}

__device__ __forceinline__ s16x4 lds_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(reinterpret_cast<uintptr_t>(p)));
}

// MN-major image swizzle (chunk XOR within a 256-B k-row of 16 chunks)
__device__ __forceinline__ int mn_swz(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 1; }

// K-major tile: R rows from r0 (clamped to rmax - 1; clamped rows are never stored) x 64 k from k0
template <int R, int NW>
__device__ __forceinline__ void stage_k(const uint16_t* __restrict__ g, int64_t ld, int r0, int rmax, int k0,
                                        char* img, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < R / (8 * NW); ++i) {
    const int q = i * NW + wave;
    const int row = q * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ ((row >> 1) & 7);
    int gr = r0 + row;
    gr = gr < rmax ? gr : rmax - 1;
    glds16(g + (int64_t)gr * ld + k0 + lc * 8, img + q * 1024);
  }
}

// MN-major tile: 64 k-rows from k0 (rows >= kend read the zero page) x R columns from c0 (clamped)
template <int R, int NW>
__device__ __forceinline__ void stage_mn(const uint16_t* __restrict__ g, int64_t ld, int c0, int cmax, int k0,
                                         int kend, const uint16_t* zero, char* img, int wave, int lane) {
  constexpr int CPR = R / 8;
#pragma unroll
  for (int i = 0; i < R / (8 * NW); ++i) {
    const int q = i * NW + wave;
    const int lin = q * 64 + lane;
    const int row = lin / CPR;
    const int lc = (lin % CPR) ^ (mn_swz(row) & (CPR - 1));
    int gc = c0 + lc * 8;
    gc = gc < cmax ? gc : cmax - 8;
    const int kr = k0 + row;
    const uint16_t* src = kr < kend ? g + (int64_t)kr * ld + gc : zero;
    glds16(src, img + q * 1024);
  }
}

template <int R, bool KMAJ>
__device__ __forceinline__ bf16x8_t frag(const char* img, int rbase, int s, int lane) {
  Frag8 f;
  if constexpr (KMAJ) {
    const int row = rbase + (lane & 15);
    const int c = s * 4 + (lane >> 4);
    f.u = *reinterpret_cast<const uint4*>(img + row * 128 + ((c ^ ((row >> 1) & 7)) << 4));
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
    const int col = rbase + pp * 4;
    const int lc = col >> 3, sub = (col & 7) * 2;
    const int k1 = s * 32 + g * 8 + q, k2 = k1 + 4;
    f.h[0] = lds_tr(img + k1 * (R * 2) + ((lc ^ (mn_swz(k1) & (R / 8 - 1))) << 4) + sub);
    f.h[1] = lds_tr(img + k2 * (R * 2) + ((lc ^ (mn_swz(k2) & (R / 8 - 1))) << 4) + sub);
  }
  return f.v;
}

// BM x BN tile, NW waves as 2 (M) x NW/2 (N); per wave (BM/2) x (2 BN/NW) = MR x NR fragments of 16 x 16
template <int MODE, int BM, int BN, int NW>
__global__ __launch_bounds__(NW * 64, (BM * BN > 128 * 128 ? 1 : 2)) void grouped_gemm_kernel(GGArgs p) {
  constexpr bool AK = MODE != 2;
  constexpr bool BK = MODE == 1;
  constexpr int WN = NW / 2;
  constexpr int MR = BM / 2 / 16, NR = BN / WN / 16;
  constexpr int A_BYTES = BM * kK * 2;
  constexpr int STAGE = (BM + BN) * kK * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;

  int e = -1, m0 = 0, mend = 0, n0 = 0, kbeg = 0, kend = 0, nk = 0;
  if constexpr (MODE != 2) {
    const int tn = (int)blockIdx.x % p.tiles_n;
    const int mt = (int)blockIdx.x / p.tiles_n;
    int cum = 0;
    for (int i = 0; i < p.E; ++i) {
      const int s = p.offs[i], t = p.offs[i + 1];
      const int nt = (t - s + BM - 1) / BM;
      if (mt < cum + nt) {
        e = i; m0 = s + (mt - cum) * BM; mend = t;
        break;
      }
      cum += nt;
    }
    if (e < 0) return;  // past the last tile of the last expert (uniform over the workgroup)
    n0 = tn * BN;
    kbeg = 0; kend = p.K; nk = p.K / kK;
  } else {
    const int per = p.tiles_m * p.tiles_n;
    e = (int)blockIdx.x / per;
    const int r = (int)blockIdx.x % per;
    m0 = (r / p.tiles_n) * BM; mend = p.M;
    n0 = (r % p.tiles_n) * BN;
    kbeg = p.offs[e]; kend = p.offs[e + 1];
    nk = (kend - kbeg + kK - 1) / kK;
  }
  const uint16_t* bptr = p.b + (MODE != 2 ? (int64_t)e * p.b_es : 0);

  f32x4 acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto stage_tile = [&](int t, int buf) {
    char* base = smem + buf * STAGE;
    const int k0 = kbeg + t * kK;
    if constexpr (AK) stage_k<BM, NW>(p.a, p.lda, m0, mend, k0, base, wave, lane);
    else stage_mn<BM, NW>(p.a, p.lda, m0, mend, k0, kend, p.zero, base, wave, lane);
    if constexpr (BK) stage_k<BN, NW>(bptr, p.ldb, n0, p.N, k0, base + A_BYTES, wave, lane);
    else stage_mn<BN, NW>(bptr, p.ldb, n0, p.N, k0, MODE == 2 ? kend : k0 + kK, p.zero, base + A_BYTES, wave, lane);
  };

  if (nk > 0) {
    stage_tile(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    if (t + 1 < nk) stage_tile(t + 1, cur ^ 1);
    const char* aimg = smem + cur * STAGE;
    const char* bimg = aimg + A_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8_t bf[NR];
#pragma unroll
      for (int j = 0; j < NR; ++j) bf[j] = frag<BN, BK>(bimg, wn * (BN / WN) + j * 16, s, lane);
#pragma unroll
      for (int i = 0; i < MR; ++i) {
        const bf16x8_t af = frag<BM, AK>(aimg, wm * (BM / 2) + i * 16, s, lane);
#pragma unroll
        for (int j = 0; j < NR; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af, acc[i][j], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: lane holds C[m0 + wm*BM/2 + i*16 + (lane & 15)][n0 + wn*BN/WN + j*16 + 4*(lane >> 4) + 0..3]
  void* cbase = p.c;
  if constexpr (MODE == 2) {
    cbase = (p.flags & kGOutF32) ? (void*)(reinterpret_cast<float*>(p.c) + (int64_t)e * p.c_es)
                                 : (void*)(reinterpret_cast<uint16_t*>(p.c) + (int64_t)e * p.c_es);
  }
  const int mrow0 = m0 + wm * (BM / 2) + (lane & 15);
  const int ncol0 = n0 + wn * (BN / WN) + 4 * (lane >> 4);
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const int n = ncol0 + j * 16;
    if (n >= p.N) continue;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (MODE == 0 && (p.flags & kGBias)) {
      const uint2 braw = *reinterpret_cast<const uint2*>(p.bias + (int64_t)e * p.bias_es + n);
      bv[0] = lo_bf16(braw.x); bv[1] = hi_bf16(braw.x); bv[2] = lo_bf16(braw.y); bv[3] = hi_bf16(braw.y);
    }
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      const int m = mrow0 + i * 16;
      if (m >= mend) continue;
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = acc[i][j][q] + bv[q];
      const int64_t off = (int64_t)m * p.ldc + n;
      if (p.flags & kGOutF32) {
        float4* cp = reinterpret_cast<float4*>(reinterpret_cast<float*>(cbase) + off);
        if (p.flags & kGAccum) {
          const float4 o = *cp;
          v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
        }
        *cp = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        uint2* cp = reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(cbase) + off);
        if (p.flags & kGAccum) {
          const uint2 o = *cp;
          v[0] += lo_bf16(o.x); v[1] += hi_bf16(o.x); v[2] += lo_bf16(o.y); v[3] += hi_bf16(o.y);
        }
        *cp = make_uint2(pack_bf16(v[0], v[1]), pack_bf16(v[2], v[3]));
      }
    }
  }
}

template <int MODE, int BM, int BN, int NW>
int launch_gg(const GGArgs& a, int grid, hipStream_t st) {
  constexpr int smem = 2 * (BM + BN) * kK * 2;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)grouped_gemm_kernel<MODE, BM, BN, NW>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr_set = true;
  }
  if (grid <= 0) return 0;
  hipLaunchKernelGGL((grouped_gemm_kernel<MODE, BM, BN, NW>), dim3((unsigned)grid), dim3(NW * 64), smem, st, a);
  return (int)hipGetLastError();
}

// ---- routing: expert id per (token, slot) entry -> counts, offsets, stable permutation.
// One workgroup per expert scans all entries in order; a wave ballot + popcount gives every matching entry
// its rank, so the order inside an expert is the entry order (deterministic, no atomics).
__global__ __launch_bounds__(256) void moe_count_kernel(const int* __restrict__ eid, int n, int* __restrict__ counts) {
  const int e = blockIdx.x;
  __shared__ int part[4];
  int c = 0;
  for (int i = threadIdx.x; i < n; i += 256) c += eid[i] == e;
  c = (int)wave_sum((float)c);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) counts[e] = part[0] + part[1] + part[2] + part[3];
}

__global__ __launch_bounds__(256) void moe_scatter_kernel(const int* __restrict__ eid, int n, int E,
                                                          const int* __restrict__ counts, int* __restrict__ offs,
                                                          int* __restrict__ perm) {
  const int e = blockIdx.x;
  __shared__ int wcount[4];
  __shared__ int base_s;
  if (threadIdx.x == 0) {
    int b = 0;
    for (int i = 0; i < e; ++i) b += counts[i];
    base_s = b;
    offs[e] = b;
    if (e == E - 1) offs[E] = b + counts[e];
  }
  __syncthreads();
  int base = base_s;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int i0 = 0; i0 < n; i0 += 256) {
    const int i = i0 + threadIdx.x;
    const bool hit = i < n && eid[i] == e;
    const uint64_t m = __ballot(hit);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wcount[wave] = __popcll(m);
    __syncthreads();
    int wb = base;
    for (int w = 0; w < wave; ++w) wb += wcount[w];
    if (hit) perm[wb + before] = i;
    base += wcount[0] + wcount[1] + wcount[2] + wcount[3];
    __syncthreads();
  }
}

}  // namespace

// mode 0 forward: x [T, K] (sorted rows), w [E, K, N], bias [E, N] or null -> y [T, N] (bf16)
// mode 1 dgrad:   dy [T, N], w [E, K, N] -> dx [T, K]   (here "N" of the call = K of the layer)
// mode 2 wgrad:   x [T, K], dy [T, N] -> dw [E, K, N] (bf16, or fp32 / accumulate by flags)
// rows: T (the allocated rows; the launch covers ceil(T / 128) + E tiles). zero: >= 16 zero bytes.
// big: 256 x 256 tiles (8 waves) when the experts hold many rows on average (forward / dgrad: rows / E
// >= 1024, wgrad: a large output per expert), else 128 x 128 (4 waves) so small experts waste little.
template <int BM, int BN, int NW>
static int dispatch_gg(int mode, GGArgs& p, int64_t rows, hipStream_t st) {
  p.tiles_n = (p.N + BN - 1) / BN;
  if (mode == 0 || mode == 1) {
    const int64_t mt = (rows + BM - 1) / BM + p.E;
    const int grid = (int)(mt * p.tiles_n);
    return mode == 0 ? launch_gg<0, BM, BN, NW>(p, grid, st) : launch_gg<1, BM, BN, NW>(p, grid, st);
  }
  p.tiles_m = (p.M + BM - 1) / BM;
  return launch_gg<2, BM, BN, NW>(p, p.E * p.tiles_m * p.tiles_n, st);
}

PA_EXPORT int pa_grouped_gemm(int mode, const void* a, const void* b, void* c, const void* bias, const int* offs,
                              const void* zero, int E, int64_t rows, int M, int N, int K, int64_t lda, int64_t ldb,
                              int64_t ldc, int flags, hipStream_t st) {
  if (mode < 0 || mode > 2) return 4;
  if (N % 8 != 0 || (mode != 2 && K % kK != 0) || (mode == 2 && M % 8 != 0)) return 3;
  GGArgs p;
  p.a = (const uint16_t*)a; p.b = (const uint16_t*)b; p.c = c; p.bias = (const uint16_t*)bias;
  p.zero = (const uint16_t*)zero; p.offs = offs;
  p.lda = lda; p.ldb = ldb; p.ldc = ldc;
  p.E = E; p.M = M; p.N = N; p.K = K; p.flags = flags;
  p.tiles_m = 0;
  // forward: w_e is [K, N]; dgrad: w_e is [N(call), K(call)] = [K_layer, N_layer]; wgrad: C_e is [M, N]
  p.b_es = (int64_t)K * N;
  p.bias_es = N;
  p.c_es = (int64_t)M * N;
  bool big;
  if (mode == 2) big = (int64_t)M * N >= (int64_t)2048 * 2048 && rows / E >= 256;
  else big = rows / E >= 1024 && N >= 1024;
  return big ? dispatch_gg<256, 256, 8>(mode, p, rows, st) : dispatch_gg<128, 128, 4>(mode, p, rows, st);
}

// eid [n] int32 expert per entry (negative = dropped) -> counts [E], offs [E + 1], perm [n] (entries of
// expert 0 in order, then expert 1, ...; the tail past offs[E] is left untouched)
PA_EXPORT int pa_moe_route(const int* eid, int n, int E, int* counts, int* offs, int* perm, hipStream_t st) {
  if (E <= 0) return 3;
  hipLaunchKernelGGL(moe_count_kernel, dim3(E), dim3(256), 0, st, eid, n, counts);
  PA_CHECK_LAUNCH();
  hipLaunchKernelGGL(moe_scatter_kernel, dim3(E), dim3(256), 0, st, eid, n, E, counts, offs, perm);
  PA_CHECK_LAUNCH();
  return 0;
}
