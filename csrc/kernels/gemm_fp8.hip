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
  // balanced tail (ping-pong kernel, as gemm.hip's): tiles [full_tiles, tiles) are cut along K into tail_split
  // slices that write fp32 256 x 256 partials to tail_ws; gemm_fp8_tail_reduce_k sums them and applies the epilogue
  int full_tiles, tail_split;
  float* tail_ws;
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
  // chunks c0, c0 + 1 (c0 even) sit at (c0 ^ sw) and (c0 ^ sw) ^ 1: the second address is the first XOR 16
  const int off = row * 128 + ((c0 ^ sw) << 4);
  const uint4 lo = *reinterpret_cast<const uint4*>(img + off);
  const uint4 hi = *reinterpret_cast<const uint4*>(img + (off ^ 16));
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

// ---------------------------------------------------------------------------------------------
// Ping-pong fp8 kernel: gemm.hip's 256x256 8-phase schedule (gemm256_kernel) at the fp8 byte geometry. A K-tile
// of 128 fp8 is 128 bytes per row — the bf16 kernel's 64-element tile byte for byte — so the staging (four 16-KiB
// half-tiles per K-tile, each issued six phases ahead by global_load_lds), the counted vmcnt waits, the barrier
// stagger of the wm == 1 waves (one wave per SIMD in its MFMA cluster while the other reads LDS) and the LDS
// swizzle are unchanged; per phase a wave runs 8 v_mfma_scale_f32_16x16x128_f8f6f4 (= the 16 bf16 16x16x32
// MFMAs' cycles at twice the FLOPs). Fragments: lane l holds row (l & 15) and k-bytes [32 (l >> 4), +32) of the
// 128-byte row (chunks 2g, 2g + 1). Wave (wm, wn) owns rows {wm*64.., 128+wm*64..} x cols {wn*32.., 128+wn*32..}.
// Epilogue: alpha, bias, activation in registers, the 16-bit tile staged through LDS, 16-byte row stores
// (N % 8 == 0).
__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void vm_wait(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// one half-tile: 128 rows x 128 k-bytes -> LDS [128][128 B], chunk c of row r at c ^ ((r >> 1) & 7); 2 glds / lane
__device__ __forceinline__ void stage_half8(const uint8_t* __restrict__ g, int64_t ld, int r0, int rmax, int k0,
                                            char* img, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = i * 8 + wave;
    const int row = q * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ ((row >> 1) & 7);
    int gr = r0 + row;
    gr = gr < rmax ? gr : rmax - 1;
    glds16(g + (int64_t)gr * ld + k0 + lc * 16, img + q * 1024);
  }
}

// C += B-frag x A-frag on the unscaled v_mfma_f32_16x16x128_f8f6f4 (formats in cbsz / blgp); PA_FP8_SCALED_MFMA
// selects the block-scaled form with unit E8M0 scales instead (the builtin: an extra scale operand pair).
template <int FA, int FB>
__device__ __forceinline__ f32x4 mfma8(const i32x8& b, const i32x8& a, f32x4 c) {
#ifdef PA_FP8_SCALED_MFMA
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(b, a, c, FB, FA, 0, 127, 0, 127);
#else
  if constexpr (FB == 0 && FA == 0) {
    asm("v_mfma_f32_16x16x128_f8f6f4 %0, %1, %2, %0" : "+v"(c) : "v"(b), "v"(a));
  } else if constexpr (FB == 1 && FA == 0) {
    asm("v_mfma_f32_16x16x128_f8f6f4 %0, %1, %2, %0 cbsz:1" : "+v"(c) : "v"(b), "v"(a));
  } else if constexpr (FB == 0 && FA == 1) {
    asm("v_mfma_f32_16x16x128_f8f6f4 %0, %1, %2, %0 blgp:1" : "+v"(c) : "v"(b), "v"(a));
  } else {
    asm("v_mfma_f32_16x16x128_f8f6f4 %0, %1, %2, %0 cbsz:1 blgp:1" : "+v"(c) : "v"(b), "v"(a));
  }
  return c;
#endif
}

template <int V>
struct IntC {
  static constexpr int value = V;
};

// grouped tile order (8 m-tiles per group), as gemm.hip tile_coords
__device__ __forceinline__ void tile_coords8(int pid, int tiles_m, int tiles_n, int* tm, int* tn) {
  constexpr int GM = 8;
  const int per_group = GM * tiles_n;
  const int first_m = (pid / per_group) * GM;
  const int gsz = min(tiles_m - first_m, GM);
  *tm = first_m + (pid % per_group) % gsz;
  *tn = (pid % per_group) / gsz;
}

// balanced-tail reduction: tail tile b = tile full_tiles + b; a thread sums the slices' partials of 4 columns and
// applies the epilogue
template <bool OUT_F16>
__global__ __launch_bounds__(256) void gemm_fp8_tail_reduce_k(Fp8Args p) {
  const int b = blockIdx.x;
  int tm, tn;
  tile_coords8(p.full_tiles + b, p.tiles_m, p.tiles_n, &tm, &tn);
  const int e = (blockIdx.y * 256 + threadIdx.x) * 4;
  const int r = e >> 8, c = e & 255;
  const int m = tm * 256 + r, n = tn * 256 + c;
  if (m >= p.M || n >= p.N) return;
  const float* src = p.tail_ws + (int64_t)b * p.tail_split * 65536 + e;
  float4 a = *reinterpret_cast<const float4*>(src);
  for (int k = 1; k < p.tail_split; ++k) {
    const float4 v = *reinterpret_cast<const float4*>(src + (int64_t)k * 65536);
    a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
  }
  float bq[4] = {0.f, 0.f, 0.f, 0.f};
  if (p.bias) {
    const uint2 braw = *reinterpret_cast<const uint2*>(p.bias + n);
    if (OUT_F16) {
      bq[0] = lo_f16(braw.x); bq[1] = hi_f16(braw.x); bq[2] = lo_f16(braw.y); bq[3] = hi_f16(braw.y);
    } else {
      bq[0] = lo_bf16(braw.x); bq[1] = hi_bf16(braw.x); bq[2] = lo_bf16(braw.y); bq[3] = hi_bf16(braw.y);
    }
  }
  const float av[4] = {a.x, a.y, a.z, a.w};
  float v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = act_f(av[q] * p.alpha + bq[q], p.act);
  *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(p.c) + (int64_t)m * p.ldc + n) =
      OUT_F16 ? make_uint2(pack_f16(v[0], v[1]), pack_f16(v[2], v[3]))
              : make_uint2(pack_bf16(v[0], v[1]), pack_bf16(v[2], v[3]));
}

int device_cus8() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  return cus;
}

// tail plan: the remainder of the last whole wave of tiles is cut along K so the last wave fills the chip (only
// when it covers at most half of it and every slice keeps at least 4 K-tiles of 128)
void pp_plan8(int64_t M, int64_t N, int64_t K, int cus, int* full, int* split) {
  const int64_t T = ((M + 255) / 256) * ((N + 255) / 256);
  const int64_t nk = K / kKB;
  *full = (int)T;
  *split = 0;
  if (T <= cus) return;
  const int64_t r = T % cus;
  if (r == 0 || 2 * r > cus) return;
  int sp = 1;
  while (r * sp * 2 <= cus && nk % (sp * 2) == 0 && nk / (sp * 2) >= 4) sp *= 2;
  if (sp == 1) return;
  *full = (int)(T - r);
  *split = sp;
}

constexpr int kPPThreads = 512;
constexpr int kEpiRS = 264;  // 16-bit values per row of the epilogue image (528-byte rows)

template <int FA, int FB, bool OUT_F16>
__global__ __launch_bounds__(kPPThreads, 1) void gemm_fp8_pp_kernel(Fp8Args p) {
  constexpr int HALF = 128 * kKB;  // 16 KiB
  constexpr int STAGE = 4 * HALF;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 2, wn = wave & 3;

  const int bid = (int)blockIdx.x;
  int pid;
  float* tail_out = nullptr;
  if (p.tail_split > 0 && bid >= p.full_tiles) {  // K slice of a tail tile
    const int u = bid - p.full_tiles;
    const int ks = u % p.tail_split;
    pid = p.full_tiles + u / p.tail_split;
    p.K /= p.tail_split;
    p.a += (int64_t)ks * p.K;
    p.b += (int64_t)ks * p.K;
    tail_out = p.tail_ws + (int64_t)u * 65536;
  } else {
    pid = xcd_remap(bid, p.tail_split > 0 ? p.full_tiles : p.tiles_m * p.tiles_n);
  }
  int tm, tn;
  tile_coords8(pid, p.tiles_m, p.tiles_n, &tm, &tn);
  const int m0 = tm * kTile, n0 = tn * kTile;
  const int nk = p.K / kKB;

  auto stage_h = [&](int t, int h, char* dst) {
    const int k0 = t * kKB;
    if (h == 0 || h == 2) stage_half8(p.a, p.lda, m0 + (h == 2 ? 128 : 0), p.M, k0, dst, wave, lane);
    else stage_half8(p.b, p.ldb, n0 + (h == 3 ? 128 : 0), p.N, k0, dst, wave, lane);
  };
  auto issue = [&](int j) {
    const int t = j >> 2, h = j & 3;
    stage_h(t, h, smem + (t & 1) * STAGE + h * HALF);
  };
  auto issue_h = [&](int t, auto hc) {
    constexpr int h = decltype(hc)::value;
    stage_h(t, h, smem + (t & 1) * STAGE + h * HALF);
  };

  f32x4 acc[2][4][2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][i][b][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int last_j = 4 * nk - 1;
  auto wait_for = [&](int phase, int jstar) {
    const int issued = min(phase + 6, last_j);
    vm_wait(2 * max(issued - jstar, 0));
  };
  const int npro = min(6, 4 * nk);
#pragma unroll 1
  for (int j = 0; j < npro; ++j) issue(j);
  vm_wait(2 * max(min(5, last_j) - 1, 0));
  bar();
  const bool lag = __builtin_amdgcn_readfirstlane(wm) == 1;
  if (lag) bar();

  i32x8 af[4], bl[2], br[2];
  const int ar = wm * 64, bc = wn * 32;

  auto ktile = [&](int t, auto steady) {
    constexpr bool S = decltype(steady)::value;
    const char* buf = smem + (t & 1) * STAGE;
    const int ph = 4 * t;
    // phase 0: read A-top + B-left; MFMA (top, L)
#pragma unroll
    for (int j = 0; j < 2; ++j) bl[j] = frag(buf + HALF, bc + j * 16, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = frag(buf, ar + i * 16, lane);
    if (S) {
      issue_h(t + 1, IntC<2>{});
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      if (ph + 6 <= last_j) issue(ph + 6);
      wait_for(ph, ph + 3);
    }
    bar();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[0][i][0][j] =
            mfma8<FA, FB>(bl[j], af[i], acc[0][i][0][j]);
    __builtin_amdgcn_s_setprio(0);
    bar();
    // phase 1: read B-right; MFMA (top, R)
#pragma unroll
    for (int j = 0; j < 2; ++j) br[j] = frag(buf + 3 * HALF, bc + j * 16, lane);
    if (S) {
      issue_h(t + 1, IntC<3>{});
      asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    } else {
      if (ph + 7 <= last_j) issue(ph + 7);
      wait_for(ph + 1, ph + 2);
    }
    bar();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[0][i][1][j] =
            mfma8<FA, FB>(br[j], af[i], acc[0][i][1][j]);
    __builtin_amdgcn_s_setprio(0);
    bar();
    // phase 2: read A-bottom; MFMA (bottom, L)
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = frag(buf + 2 * HALF, ar + i * 16, lane);
    if (S) issue_h(t + 2, IntC<0>{});
    else if (ph + 8 <= last_j) issue(ph + 8);
    bar();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[1][i][0][j] =
            mfma8<FA, FB>(bl[j], af[i], acc[1][i][0][j]);
    __builtin_amdgcn_s_setprio(0);
    bar();
    // phase 3: wait for H0 / H1 of tile t + 1; MFMA (bottom, R)
    if (S) {
      issue_h(t + 2, IntC<1>{});
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      if (ph + 9 <= last_j) issue(ph + 9);
      if (t + 1 < nk) wait_for(ph + 3, ph + 5);
    }
    bar();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[1][i][1][j] =
            mfma8<FA, FB>(br[j], af[i], acc[1][i][1][j]);
    __builtin_amdgcn_s_setprio(0);
    bar();
  };
  const int nsteady = max(nk - 2, 0);
  int t = 0;
#pragma unroll 1
  for (; t < nsteady; ++t) ktile(t, IntC<1>{});
#pragma unroll 1
  for (; t < nk; ++t) ktile(t, IntC<0>{});
  if (!lag) bar();

  if (tail_out) {  // raw fp32 partial of this K slice, row-major 256 x 256
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
    for (int bh = 0; bh < 2; ++bh)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ah = 0; ah < 2; ++ah)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = ah * 128 + ar + i * 16 + (lane & 15);
            const int c = bh * 128 + bc + j * 16 + 4 * (lane >> 4);
            const f32x4 v = acc[ah][i][bh][j];
            *reinterpret_cast<float4*>(tail_out + r * 256 + c) = make_float4(v[0], v[1], v[2], v[3]);
          }
    return;
  }

  // epilogue: alpha, bias, activation in registers; the 16-bit tile through LDS ([256][264]); row stores.
  // The MFMAs are inline asm, so the compiler's hazard tracking does not see their results: wait out the
  // MFMA -> VALU read latency of the last accumulators explicitly.
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  uint16_t* im = reinterpret_cast<uint16_t*>(smem);
  bar();
#pragma unroll
  for (int bh = 0; bh < 2; ++bh)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = bh * 128 + bc + j * 16 + 4 * (lane >> 4);
      float bq[4] = {0.f, 0.f, 0.f, 0.f};
      if (p.bias && n0 + c < p.N) {
        const uint2 braw = *reinterpret_cast<const uint2*>(p.bias + n0 + c);
        if (OUT_F16) {
          bq[0] = lo_f16(braw.x); bq[1] = hi_f16(braw.x); bq[2] = lo_f16(braw.y); bq[3] = hi_f16(braw.y);
        } else {
          bq[0] = lo_bf16(braw.x); bq[1] = hi_bf16(braw.x); bq[2] = lo_bf16(braw.y); bq[3] = hi_bf16(braw.y);
        }
      }
#pragma unroll
      for (int ah = 0; ah < 2; ++ah)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = ah * 128 + ar + i * 16 + (lane & 15);
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = act_f(acc[ah][i][bh][j][e] * p.alpha + bq[e], p.act);
          *reinterpret_cast<uint2*>(im + r * kEpiRS + c) =
              OUT_F16 ? make_uint2(pack_f16(v[0], v[1]), pack_f16(v[2], v[3]))
                      : make_uint2(pack_bf16(v[0], v[1]), pack_bf16(v[2], v[3]));
        }
    }
  bar();
  const int ecb = (tid & 31) * 8, erb = tid >> 5;
  const int nb_ = n0 + ecb;
  if (nb_ < p.N) {
#pragma unroll 4
    for (int step = 0; step < 16; ++step) {
      const int r = step * 16 + erb;
      const int m = m0 + r;
      if (m >= p.M) break;
      *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(p.c) + (int64_t)m * p.ldc + nb_) =
          *reinterpret_cast<const uint4*>(im + r * kEpiRS + ecb);
    }
  }
}

template <int FA, int FB, bool F16>
int launch_pp(const Fp8Args& g, hipStream_t st) {
  static bool attr = false;
  // two 64-KiB stages; the epilogue image [256][264] x 2 B (132 KiB) reuses them and is the larger
  constexpr int smem = (2 * 4 * 128 * kKB) > (kTile * kEpiRS * 2) ? (2 * 4 * 128 * kKB) : (kTile * kEpiRS * 2);
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_fp8_pp_kernel<FA, FB, F16>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  const int T = g.tiles_m * g.tiles_n;
  const int grid = g.tail_split ? g.full_tiles + (T - g.full_tiles) * g.tail_split : T;
  hipLaunchKernelGGL((gemm_fp8_pp_kernel<FA, FB, F16>), dim3(grid), dim3(kPPThreads), smem, st, g);
  int rc = (int)hipGetLastError();
  if (rc || !g.tail_split) return rc;
  hipLaunchKernelGGL((gemm_fp8_tail_reduce_k<F16>), dim3(T - g.full_tiles, 64), dim3(256), 0, st, g);
  return (int)hipGetLastError();
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
int launch_out(const Fp8Args& g, int out_f16, bool pp, hipStream_t st) {
  if (pp) return out_f16 ? launch_pp<FA, FB, true>(g, st) : launch_pp<FA, FB, false>(g, st);
  return out_f16 ? launch<FA, FB, true>(g, st) : launch<FA, FB, false>(g, st);
}

// kernel choice: 0 auto (ping-pong when N % 8 == 0 and ldc % 8 == 0), 1 generic, 2 ping-pong (as auto)
int g_fp8_kernel = 0;

}  // namespace

// fmt_a / fmt_b: 0 = e4m3fn, 1 = e5m2. act: 0 identity, 1 gelu, 2 relu. bias: [N] in the output dtype or null.
// Returns 1 for an unsupported shape / stride (K % 128, N % 4, leading dims % 16 bytes).
// Workspace (bytes) the ping-pong fp8 GEMM's balanced tail needs (0: none).
PA_EXPORT int64_t pa_gemm_fp8_ws_bytes(int64_t M, int64_t N, int64_t K) {
  int full, split;
  pp_plan8(M, N, K, device_cus8(), &full, &split);
  if (!split) return 0;
  const int64_t T = ((M + 255) / 256) * ((N + 255) / 256);
  return (T - full) * split * 65536 * 4;
}

static int fp8_impl(const void* a, const void* b, void* c, const void* bias, int64_t M, int64_t N, int64_t K,
                    int64_t lda, int64_t ldb, int64_t ldc, int fmt_a, int fmt_b, float alpha, int act, int out_f16,
                    void* ws, hipStream_t st);

PA_EXPORT int pa_gemm_fp8(const void* a, const void* b, void* c, const void* bias, int64_t M, int64_t N, int64_t K,
                          int64_t lda, int64_t ldb, int64_t ldc, int fmt_a, int fmt_b, float alpha, int act,
                          int out_f16, hipStream_t st) {
  return fp8_impl(a, b, c, bias, M, N, K, lda, ldb, ldc, fmt_a, fmt_b, alpha, act, out_f16, nullptr, st);
}

// the same with the balanced-tail workspace (pa_gemm_fp8_ws_bytes(M, N, K) bytes; may be null when that is 0)
PA_EXPORT int pa_gemm_fp8_ws(const void* a, const void* b, void* c, const void* bias, int64_t M, int64_t N, int64_t K,
                             int64_t lda, int64_t ldb, int64_t ldc, int fmt_a, int fmt_b, float alpha, int act,
                             int out_f16, void* ws, hipStream_t st) {
  return fp8_impl(a, b, c, bias, M, N, K, lda, ldb, ldc, fmt_a, fmt_b, alpha, act, out_f16, ws, st);
}

static int fp8_impl(const void* a, const void* b, void* c, const void* bias, int64_t M, int64_t N, int64_t K,
                    int64_t lda, int64_t ldb, int64_t ldc, int fmt_a, int fmt_b, float alpha, int act, int out_f16,
                    void* ws, hipStream_t st) {
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
  const bool pp = g_fp8_kernel != 1 && N % 8 == 0 && ldc % 8 == 0;
  g.full_tiles = g.tiles_m * g.tiles_n;
  g.tail_split = 0;
  if (pp && ws) {
    int full, split;
    pp_plan8(M, N, K, device_cus8(), &full, &split);
    if (split) {
      g.full_tiles = full;
      g.tail_split = split;
      g.tail_ws = (float*)ws;
    }
  }
  if (fmt_a == 0 && fmt_b == 0) return launch_out<0, 0>(g, out_f16, pp, st);
  if (fmt_a == 0 && fmt_b == 1) return launch_out<0, 1>(g, out_f16, pp, st);
  if (fmt_a == 1 && fmt_b == 0) return launch_out<1, 0>(g, out_f16, pp, st);
  return launch_out<1, 1>(g, out_f16, pp, st);
}

// 0 auto, 1 generic kernel only (A/B and tests)
PA_EXPORT int pa_gemm_fp8_set_kernel(int k) {
  g_fp8_kernel = k;
  return 0;
}
