// Hand-written bf16 GEMM with fused epilogues for gfx950 (CDNA4 MFMA).
// Reference behaviour: paddle/phi/kernels/gpu/matmul_kernel.cu (cuBLAS) and
// paddle/phi/kernels/fusion/gpu/fused_gemm_epilogue_kernel.cu (cublasLt bias / GELU epilogues,
// the pre-activation "reserve space" kept for the backward).
//
//   C[M,N] = epilogue( A[M,K] . B[K,N] )
//
// Operand layouts (template): each operand is either K-major (A stored [M][K], B stored [N][K]) or
// MN-major (A stored [K][M], B stored [K][N]); this covers the three linear-layer products
//   forward  y  = x  . W      (A K-major, B MN-major: paddle's W is [in, out])
//   dgrad    dx = dy . W^T    (A K-major, B K-major)
//   wgrad    dW = x^T . dy    (A MN-major, B MN-major)
// without any transpose copies.
//
// Structure (CDNA4 playbook, cdna_hip_programming.md section 5):
//   * 256 x BN x 64 tiles, 8 waves (512 threads) as 2 (M) x 4 (N); per wave 128 x BN/4;
//     v_mfma_f32_16x16x32_bf16, operands swapped (D = B^T-frag x A-frag) so each lane ends with
//     4 consecutive output columns of one row -> 8/16-byte epilogue stores.
//   * global -> LDS with global_load_lds_dwordx4 (no VGPR staging), two LDS stages (128 KiB for
//     256x256): tile t+1 is in flight while tile t is consumed.
//   * K-major images: [rows][64 k] with 128-B rows, 16-B chunk XOR-swizzle chunk ^ ((row>>1)&7):
//     the ds_read_b128 of 16 rows x one chunk hits 16 distinct bank slots.
//   * MN-major images: [64 k][R] rows, read with ds_read_b64_tr_b16 (hardware transpose) and
//     swizzled chunk ^ 2*((k&3) | ((k>>3)&1)<<2) so each 32-lane half reads 8 distinct 32-B slots.
//   * glds writes LDS lane-linearly, so the swizzle is applied to the per-lane GLOBAL source address
//     and undone on the LDS read (both sides or neither).
//   * XCD-aware bijective block remap + grouped tile order so the blocks of one XCD share A / B
//     panels in their private L2.
//   * epilogue: + bias[N], tanh-GELU (optionally storing the pre-activation for the backward),
//     accumulate into an existing C (gradient-accumulation fusion), bf16 or fp32 output.
#include "common.h"

#include <climits>

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

constexpr int kBM = 256;
constexpr int kBK = 64;
constexpr int kThreads = 512;

enum EpiFlags : int {
  kEpiBias = 1,       // + bias[n]
  kEpiGelu = 2,       // tanh-GELU after the bias
  kEpiAux = 4,        // store the pre-activation (x.W + b) to aux (bf16, ldc)
  kEpiAccum = 8,      // C += result (read-modify-write)
  kEpiOutF32 = 16,    // C is fp32
  kEpiStats = 32,     // per-column batch-norm partials of the stored C (sum, sum of squares) to stats
  kEpiStatsBwd = 64,  // with kEpiStats: BN-backward partials instead (C is the BN's output gradient):
                      // sum dyp, sum dyp * (x - mean), dyp = relu mask (x * scale + shift > 0) of the stored C
  kEpiGeluBwd = 128,  // C = result * gelu'(aux): aux holds the GELU's pre-activation (the data gradient of the
                      // linear after a GELU, fused with the GELU backward; 256x256 kernels, staged epilogue)
  kEpiColSum = 256,   // column sums of the result per 256-row tile to stats[tiles_m][N] (fp32; bias gradient)
  kEpiResid = 512,    // C = result + res (bf16 [M][ldc]): the residual add after an output projection
};
constexpr int kEpiStaged = kEpiAux | kEpiAccum | kEpiOutF32 | kEpiGeluBwd | kEpiColSum | kEpiResid;

struct GemmArgs {
  const uint16_t* a;
  const uint16_t* b;
  void* c;
  const uint16_t* bias;
  uint16_t* aux;
  int64_t lda, ldb, ldc;
  int M, N, K;
  int tiles_m, tiles_n;
  int flags;
  float alpha;
  int64_t c_split;  // split-K: blockIdx.y = K slice of p.K elements; output slab stride (fp32 elements)
  // implicit-GEMM convolution (NHWC): A[p][k] = x[n, ho*s - pad + kh*dil, wo*s - pad + kw*dil, c],
  // p = (n, ho, wo), k = (kh * KW + kw) * C + c; out-of-image taps read the 128-byte zero page
  const uint16_t* zero;
  int cH, cW, cC, cHo, cWo, cKW, cStride, cPadH, cPadW, cDil;
  // 3-D (NDHWC) forward: depth, output depth, taps per depth slice (KH * KW) and depth padding; 2-D: 1, 1, KH*KW, 0
  int cD, cDo, cKHW, cPadD;
  // balanced tail (ping-pong kernel): tiles [full_tiles, tiles) are split over K into tail_split slices
  // (workgroups full_tiles + u, u = local tile * tail_split + slice) that write fp32 256x256 partials to
  // tail_ws; gemm_tail_reduce_k sums them and applies the epilogue. tail_split == 0: no tail.
  int full_tiles, tail_split;
  float* tail_ws;
  // operand segments (ping-pong kernel), nseg = 0 / 1: none. seg_k = 1: the K range is split, K-tiles
  // [seg_end[s-1], seg_end[s]) read A = seg_a[s] (lda seg_lda[s]) and B = seg_b[s] (ldb seg_ldb[s]) from their own
  // k = 0: C = sum_s A_s . B_s in one launch (the data gradient of sibling linears, the weight gradient of two
  // accumulation micro-batches) without concatenated copies. seg_k = 0: the N range is split (seg_end in columns,
  // multiples of 128), columns of segment s read B = seg_b[s] from its own column 0: C = A . [B_0 | B_1 | ...] (one
  // GEMM for the q / k / v or gate / up projections of one input).
  int nseg, seg_k;
  int seg_end[4];
  const uint16_t* seg_a[4];
  const uint16_t* seg_b[4];
  int64_t seg_lda[4], seg_ldb[4];
  // kEpiStats: stats[2][chunks][N] fp32, chunk = m-tile * (waves along M) + wave row; each (chunk, column) is
  // written by exactly one lane (no atomics, deterministic), folded by bn.hip (pa_bn_fwd_nhwc_pre)
  float* stats;
  // kEpiStatsBwd: the BN's input x ([M][ldc] bf16), its forward scale / shift ss [2][N] and batch mean [N]
  const uint16_t* bn_x;
  const float* bn_ss;
  const float* bn_mean;
  // kEpiResid: the residual read by the epilogue (bf16, leading dimension ldc)
  const uint16_t* res;
};

// split-K view: slice blockIdx.y of K (p.K elements each) and its own fp32 output slab
template <bool AK, bool BKM>
__device__ __forceinline__ GemmArgs split_view(const GemmArgs& p0) {
  GemmArgs p = p0;
  const int64_t ks = blockIdx.y;
  if (ks) {
    p.a += ks * (int64_t)p.K * (AK ? 1 : p.lda);
    p.b += ks * (int64_t)p.K * (BKM ? 1 : p.ldb);
    p.c = reinterpret_cast<float*>(p.c) + ks * p.c_split;
  }
  return p;
}

__device__ __forceinline__ float gelu_tanh(float x) { return gelu_tanh_fast(x); }

// Batch-norm statistics of the fragment epilogue (conv -> BN fusion, reference:
// fusion/gpu/fused_scale_bias_relu_conv_bn_kernel.cu computes the BN sums of the conv output in the conv):
// s1 / s2 are a lane's sums of its rows for 4 consecutive columns n..n+3; the 16 lanes of the DPP row are
// folded and lane 0 of the row writes chunk `chunk` of stats[2][chunks][N].
__device__ __forceinline__ void stats_store(const GemmArgs& p, int chunk, int chunks, int n, int lane, float* s1,
                                            float* s2) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    s1[e] = row16_sum(s1[e]);
    s2[e] = row16_sum(s2[e]);
  }
  if ((lane & 15) == 0) {
    *reinterpret_cast<float4*>(p.stats + (int64_t)chunk * p.N + n) = make_float4(s1[0], s1[1], s1[2], s1[3]);
    *reinterpret_cast<float4*>(p.stats + ((int64_t)chunks + chunk) * p.N + n) = make_float4(s2[0], s2[1], s2[2], s2[3]);
  }
}

// BN-backward partials of 4 stored gradient values (packed pair o.x, o.y) against the BN input at the same
// element (conv dgrad -> relu' -> BN backward, reference fusion/gpu/fused_dconv_drelu_dbn_kernel.cu)
__device__ __forceinline__ void stats_add_bwd(const GemmArgs& p, int64_t off, uint2 o, const float* sc,
                                              const float* sh, const float* mu, float* s1, float* s2) {
  const uint2 xr = *reinterpret_cast<const uint2*>(p.bn_x + off);
  const float g[4] = {lo_bf16(o.x), hi_bf16(o.x), lo_bf16(o.y), hi_bf16(o.y)};
  const float x[4] = {lo_bf16(xr.x), hi_bf16(xr.x), lo_bf16(xr.y), hi_bf16(xr.y)};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float d = x[e] * sc[e] + sh[e] > 0.f ? g[e] : 0.f;
    s1[e] += d;
    s2[e] += d * (x[e] - mu[e]);
  }
}

// per-column BN constants of the backward statistics for columns n..n+3
__device__ __forceinline__ void bn_cols(const GemmArgs& p, int n, float* sc, float* sh, float* mu) {
  const float4 a = *reinterpret_cast<const float4*>(p.bn_ss + n);
  const float4 b = *reinterpret_cast<const float4*>(p.bn_ss + p.N + n);
  const float4 m = *reinterpret_cast<const float4*>(p.bn_mean + n);
  sc[0] = a.x; sc[1] = a.y; sc[2] = a.z; sc[3] = a.w;
  sh[0] = b.x; sh[1] = b.y; sh[2] = b.z; sh[3] = b.w;
  mu[0] = m.x; mu[1] = m.y; mu[2] = m.z; mu[3] = m.w;
}

// stored bf16 pair -> the two rounded values accumulated into the statistics
__device__ __forceinline__ void stats_add2(uint32_t packed, float* s1, float* s2, int e) {
  const float a = lo_bf16(packed), b = hi_bf16(packed);
  s1[e] += a; s2[e] += a * a;
  s1[e + 1] += b; s2[e + 1] += b * b;
}

// global_load_lds_dwordx4 issued from inline asm: hipcc treats a builtin LDS-DMA as a pending write to
// every LDS object and puts s_waitcnt vmcnt(0) in front of the next ds_read, which would drain the
// prefetch pipeline each phase. The kernels retire the DMA themselves with counted vmcnt + barrier.
// M0 holds the wave-uniform LDS destination (lane i writes base + 16 i).
__device__ __forceinline__ void glds16(const void* g, char* lds_wave_base) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uintptr_t>(lds_wave_base));
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m0) : "memory", "m0");
}

__device__ __forceinline__ s16x4 lds_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(reinterpret_cast<uintptr_t>(p)));
}

// swizzle of an MN-major image row (even chunk XOR so 32-B pairs stay together)
__device__ __forceinline__ int mn_swz(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 1; }
// the swizzle restricted to a k-row of R columns (R / 8 chunks): a no-op for R >= 128; for R = 64 it keeps
// the chunk inside its row (slot <-> global chunk stays a bijection)
template <int R>
__device__ __forceinline__ int mn_swz_r(int k) { return mn_swz(k) & (R / 8 - 1); }

// ---- staging of one operand tile (R rows of the output dimension x 64 k) into LDS
// K-major: image [R][64] (128-B rows).  MN-major: image [64][R] (2R-byte rows).
template <int R, bool KMAJ, int NW = 8>
__device__ __forceinline__ void stage(const uint16_t* __restrict__ g, int64_t ld, int r0, int rmax, int k0,
                                      char* img, int wave, int lane) {
  constexpr int NQ = R / (8 * NW);  // glds instructions per thread (R*64*2 bytes / (NW * 64 * 16))
  if constexpr (KMAJ) {
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      const int q = i * NW + wave;              // wave-instruction id: 8 rows x 128 B
      const int row = q * 8 + (lane >> 3);
      const int lc = (lane & 7) ^ ((row >> 1) & 7);
      int gr = r0 + row;
      gr = gr < rmax ? gr : rmax - 1;
      glds16(g + (int64_t)gr * ld + k0 + lc * 8, img + q * 1024);
    }
  } else {
    constexpr int CPR = R / 8;  // 16-B chunks per k-row
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      const int q = i * NW + wave;
      const int lin = q * 64 + lane;
      const int row = lin / CPR;                // k
      const int lc = (lin % CPR) ^ mn_swz_r<R>(row);
      int gc = r0 + lc * 8;
      gc = gc < rmax ? gc : rmax - 8;
      glds16(g + (int64_t)(k0 + row) * ld + gc, img + q * 1024);
    }
  }
}

// Weight gradient of a KxK NHWC convolution as a GEMM: dW^T[m = (kh*KW + kw)*C + c][n = co] =
//   sum_p x[n_img, ho*s - pad + kh*dil, wo*s - pad + kw*dil, c] * dy[p][co],  p = (n_img, ho, wo).
// A (M x K, MN-major: 8 consecutive m are 8 channels of one tap) is gathered per (pixel, tap) here; the
// image is the one stage<256, false> builds (chunk lc of k-row `row` at slot lc ^ mn_swz(row)).
// kglob = first pixel of the K tile (split-K slices included); taps outside the image read the zero page.
// Per-lane gather state for the NQ pieces a lane stages per K tile: the (tap, channel) of its m chunk is
// fixed for the whole K loop; the pixel (n, ho, wo) of its k-row advances by 64 pixels per K tile, updated
// incrementally (no integer division inside the loop).
template <int NW>
struct ConvWState {
  static constexpr int NQ = kBM / (8 * NW);
  int c[NQ], hoff[NQ], woff[NQ];  // channel, kh*dil - pad, kw*dil - pad  (hoff = INT_MIN: m past M)
  int n[NQ], ho[NQ], wo[NQ];
};

template <int NW>
__device__ __forceinline__ void convw_init(const GemmArgs& p, int m0, int64_t kglob, ConvWState<NW>& st, int wave,
                                           int lane) {
  constexpr int CPR = kBM / 8;
  const int hw = p.cHo * p.cWo;
#pragma unroll
  for (int i = 0; i < ConvWState<NW>::NQ; ++i) {
    const int q = i * NW + wave;
    const int lin = q * 64 + lane;
    const int row = lin / CPR;
    const int lc = (lin % CPR) ^ mn_swz(row);
    const int m = m0 + lc * 8;
    const int tap = m / p.cC, kh = tap / p.cKW, kw = tap - kh * p.cKW;
    st.c[i] = m - tap * p.cC;
    st.hoff[i] = m < p.M ? kh * p.cDil - p.cPadH : INT_MIN / 2;
    st.woff[i] = kw * p.cDil - p.cPadW;
    const int pix = (int)(kglob + row);
    st.n[i] = pix / hw;
    const int rem = pix - st.n[i] * hw;
    st.ho[i] = rem / p.cWo;
    st.wo[i] = rem - st.ho[i] * p.cWo;
  }
}

template <int NW>
__device__ __forceinline__ void convw_advance(const GemmArgs& p, ConvWState<NW>& st, int dho, int dwo) {
#pragma unroll
  for (int i = 0; i < ConvWState<NW>::NQ; ++i) {
    st.wo[i] += dwo;
    st.ho[i] += dho;
    if (st.wo[i] >= p.cWo) { st.wo[i] -= p.cWo; st.ho[i] += 1; }
    while (st.ho[i] >= p.cHo) { st.ho[i] -= p.cHo; st.n[i] += 1; }
  }
}

template <int NW>
__device__ __forceinline__ void stage_convw(const GemmArgs& p, const ConvWState<NW>& st, char* img, int wave) {
#pragma unroll
  for (int i = 0; i < ConvWState<NW>::NQ; ++i) {
    const int q = i * NW + wave;
    const int hi = st.ho[i] * p.cStride + st.hoff[i], wi = st.wo[i] * p.cStride + st.woff[i];
    const bool ok = hi >= 0 && hi < p.cH && wi >= 0 && wi < p.cW;
    const uint16_t* src = ok ? p.a + (((int64_t)st.n[i] * p.cH + hi) * p.cW + wi) * p.cC + st.c[i] : p.zero;
    glds16(src, img + q * 1024);
  }
}

// ---- fragment read: 16 rows (output dim) x 8 k for k-substep s (32 k) -> mfma operand
template <int R, bool KMAJ>
__device__ __forceinline__ bf16x8_t frag(const char* img, int rbase, int s, int lane) {
  Frag8 f;
  if constexpr (KMAJ) {
    const int row = rbase + (lane & 15);
    const int c = s * 4 + (lane >> 4);
    f.u = *reinterpret_cast<const uint4*>(img + row * 128 + ((c ^ ((row >> 1) & 7)) << 4));
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
    const int col = rbase + pp * 4;           // first of 4 columns supplied by this lane
    const int lc = col >> 3, sub = (col & 7) * 2;
    const int k1 = s * 32 + g * 8 + q, k2 = k1 + 4;
    f.h[0] = lds_tr(img + k1 * (R * 2) + ((lc ^ mn_swz_r<R>(k1)) << 4) + sub);
    f.h[1] = lds_tr(img + k2 * (R * 2) + ((lc ^ mn_swz_r<R>(k2)) << 4) + sub);
  }
  return f.v;
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// segment of a K-tile / column index v (wave-uniform: constant-index selects, no dynamic kernel-argument indexing)
__device__ __forceinline__ int seg_of(const GemmArgs& p, int v) {
  int s = 0;
#pragma unroll
  for (int i = 0; i < 3; ++i) s += (i + 1 < p.nseg && v >= p.seg_end[i]) ? 1 : 0;
  return s;
}
template <class T>
__device__ __forceinline__ T pick4(int s, T v0, T v1, T v2, T v3) {
  return s == 0 ? v0 : (s == 1 ? v1 : (s == 2 ? v2 : v3));
}

// NW = 8: waves 2 (M) x 4 (N), wave tile 128 x BN/4, 2 waves per SIMD.
// NW = 4: waves 2 (M) x 2 (N), wave tile 128 x BN/2 (256 accumulator registers, 1 wave per SIMD):
//         a third less LDS read traffic per MFMA than the 8-wave form.
template <int BN, bool AK, bool BKM, int NW = 8, bool CONVW = false>
__global__ __launch_bounds__(NW * 64, 1) void gemm_bf16_kernel(GemmArgs p0) {
  const GemmArgs p = split_view<AK, BKM>(p0);
  const int64_t kslice = CONVW ? (int64_t)blockIdx.y * p0.K : 0;  // first pixel of this split (conv wgrad)
  (void)kslice;
  constexpr int WN = NW / 2;
  constexpr int A_BYTES = kBM * kBK * 2;
  constexpr int B_BYTES = BN * kBK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int MR = (kBM / 2) / 16;  // 8 m-fragments per wave
  constexpr int NR = (BN / WN) / 16;  // n-fragments per wave
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WN, wn = wave % WN;

  // tile order: XCD-contiguous chunks, grouped by 8 m-tiles so neighbours share B panels
  const int nwg = p.tiles_m * p.tiles_n;
  const int pid = xcd_remap((int)blockIdx.x, nwg);
  constexpr int GM = 8;
  const int per_group = GM * p.tiles_n;
  const int gid = pid / per_group;
  const int first_m = gid * GM;
  const int gsz = min(p.tiles_m - first_m, GM);
  const int tm = first_m + (pid % per_group) % gsz;
  const int tn = (pid % per_group) / gsz;
  const int m0 = tm * kBM, n0 = tn * BN;

  f32x4 acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / kBK;
  ConvWState<NW> cw;  // conv weight gradient: gather state of the A operand (tiles staged in order t = 0, 1, ..)
  int cw_dho = 0, cw_dwo = 0;
  if constexpr (CONVW) {
    convw_init<NW>(p0, m0, kslice, cw, wave, lane);
    cw_dho = kBK / p0.cWo;
    cw_dwo = kBK - cw_dho * p0.cWo;
  }
  auto stage_tile = [&](int t, int buf) {
    char* base = smem + buf * STAGE;
    if constexpr (CONVW) {
      stage_convw<NW>(p0, cw, base, wave);
      convw_advance<NW>(p0, cw, cw_dho, cw_dwo);
    } else {
      stage<kBM, AK, NW>(p.a, p.lda, m0, p.M, t * kBK, base, wave, lane);
    }
    stage<BN, BKM, NW>(p.b, p.ldb, n0, p.N, t * kBK, base + A_BYTES, wave, lane);
  };

  stage_tile(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    if (t + 1 < nk) stage_tile(t + 1, cur ^ 1);
    const char* aimg = smem + cur * STAGE;
    const char* bimg = aimg + A_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8_t bf[NR];
#pragma unroll
      for (int j = 0; j < NR; ++j) bf[j] = frag<BN, BKM>(bimg, wn * (BN / WN) + j * 16, s, lane);
#pragma unroll
      for (int i = 0; i < MR; ++i) {
        const bf16x8_t af = frag<kBM, AK>(aimg, wm * (kBM / 2) + i * 16, s, lane);
#pragma unroll
        for (int j = 0; j < NR; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af, acc[i][j], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: lane holds C[m = mb + i*16 + (lane&15)][n = nb + j*16 + 4*(lane>>4) + 0..3]
  const int flags = p.flags;
  const int mrow0 = m0 + wm * (kBM / 2) + (lane & 15);
  const int ncol0 = n0 + wn * (BN / WN) + 4 * (lane >> 4);
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const int n = ncol0 + j * 16;
    if (n >= p.N) continue;  // N % 4 == 0 is required by the launcher
    float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
    float bsc[4] = {0.f, 0.f, 0.f, 0.f}, bsh[4] = {0.f, 0.f, 0.f, 0.f}, bmu[4] = {0.f, 0.f, 0.f, 0.f};
    if (flags & kEpiStatsBwd) bn_cols(p, n, bsc, bsh, bmu);
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (flags & kEpiBias) {
      const uint2 braw = *reinterpret_cast<const uint2*>(p.bias + n);
      bv[0] = lo_bf16(braw.x); bv[1] = hi_bf16(braw.x); bv[2] = lo_bf16(braw.y); bv[3] = hi_bf16(braw.y);
    }
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      const int m = mrow0 + i * 16;
      if (m >= p.M) continue;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] * p.alpha + bv[e];
      const int64_t off = (int64_t)m * p.ldc + n;
      if (flags & kEpiAux) {
        *reinterpret_cast<uint2*>(p.aux + off) = make_uint2(pack_bf16(v[0], v[1]), pack_bf16(v[2], v[3]));
      }
      if (flags & kEpiGelu) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = gelu_tanh(v[e]);
      }
      if (flags & kEpiOutF32) {
        float4* cp = reinterpret_cast<float4*>(reinterpret_cast<float*>(p.c) + off);
        if (flags & kEpiAccum) {
          const float4 o = *cp;
          v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
        }
        *cp = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        uint2* cp = reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(p.c) + off);
        if (flags & kEpiAccum) {
          const uint2 o = *cp;
          v[0] += lo_bf16(o.x); v[1] += hi_bf16(o.x); v[2] += lo_bf16(o.y); v[3] += hi_bf16(o.y);
        }
        const uint2 o = make_uint2(pack_bf16(v[0], v[1]), pack_bf16(v[2], v[3]));
        *cp = o;
        if (flags & kEpiStatsBwd) {
          stats_add_bwd(p, off, o, bsc, bsh, bmu, s1, s2);
        } else if (flags & kEpiStats) {
          stats_add2(o.x, s1, s2, 0);
          stats_add2(o.y, s1, s2, 2);
        }
      }
    }
    if (flags & kEpiStats) stats_store(p, tm * 2 + wm, p.tiles_m * 2, n, lane, s1, s2);
  }
}

// ---------------------------------------------------------------------------------------------
// 256x256x64 8-wave kernel with the 4-phase-per-K-tile interleave (cdna_hip_programming.md 5,
// "256^2 8-phase template"): every K-tile is split into four 16-KiB half-tiles
//   H0 = A rows 0..127, H1 = B cols 0..127, H2 = A rows 128..255, H3 = B cols 128..255
// and each phase {ds_read a register subtile ; issue ONE half-tile of glds ; barrier ; 16 MFMA ;
// barrier}. Reads: phase 0 H0+H1, phase 1 H3, phase 2 H2. Half-tile j (= 4 * tile + h) is issued in
// phase j - 6, so 5-6 phases of load latency are hidden, and each read is preceded by a counted vmcnt
// in the phase before it. The wm == 1 waves run one barrier behind the wm == 0 waves (ping-pong:
// per SIMD one wave is in its MFMA cluster while the other reads LDS / issues glds); because of the
// stagger a half-tile is restaged at least two phases after its last ds_read (WAR), and a read
// happens at least one barrier after the wait that retires it in both wave groups (RAW).
// Wave (wm, wn) owns rows {wm*64.., 128+wm*64..} x cols {wn*32.., 128+wn*32..}: the four phases
// compute its quadrants (top,L) (top,R) (bottom,L) (bottom,R).
__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (the immediate must be a literal)
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

// grouped tile order (8 m-tiles per group, so neighbouring workgroups share B panels)
__device__ __forceinline__ void tile_coords(int pid, int tiles_m, int tiles_n, int* tm, int* tn) {
  constexpr int GM = 8;
  const int per_group = GM * tiles_n;
  const int first_m = (pid / per_group) * GM;
  const int gsz = min(tiles_m - first_m, GM);
  *tm = first_m + (pid % per_group) % gsz;
  *tn = (pid % per_group) / gsz;
}

constexpr int kEpiRowStride = 260;      // fp32 per row of the epilogue image (256 + 4 padding)
constexpr int kEpiRowStrideBf16 = 264;  // bf16 per row of the one-pass bf16 epilogue image (528-byte rows)

template <int V>
struct IntC {
  static constexpr int value = V;
};
using H0_ = IntC<0>;
using H1_ = IntC<1>;
using H2_ = IntC<2>;
using H3_ = IntC<3>;
using True_ = IntC<1>;
using False_ = IntC<0>;

// Coalesced epilogue pass over 128 rows of a 256-column tile from the fp32 LDS image (kEpiRowStride floats per
// row): each thread owns 8 consecutive columns and walks the rows NT / 32 at a time. Epilogues that read global
// memory (accumulate into C, the GELU backward's pre-activation) issue the reads of 8 row steps before the first
// is used: one memory latency per 8 steps instead of one per step (the loop-carried form left each step waiting
// on its own read). kEpiGeluBwd excludes kEpiAccum and kEpiResid; kEpiResid excludes kEpiAccum.
template <int NT>
__device__ __forceinline__ void epi_rows(const GemmArgs& p, const float* img, int m_base, int n0, int tid,
                                         const float* bv, float* cs) {
  constexpr int RS = kEpiRowStride;
  constexpr int RSTEP = NT / 32;
  constexpr int NSTEP = 128 / RSTEP;
  constexpr int G = 4;  // reads in flight per thread: register room next to the live accumulators
  const int ec = (tid & 31) * 8, er = tid / 32;
  const int n = n0 + ec;
  if (n >= p.N) return;
  const int flags = p.flags;
  const bool f32 = flags & kEpiOutF32;
  const bool rd_pre = flags & kEpiGeluBwd, rd_res = (flags & kEpiResid) && !rd_pre;
  const bool rd_c = (flags & kEpiAccum) && !rd_pre && !rd_res;
#pragma unroll 1
  for (int g0 = 0; g0 < NSTEP; g0 += G) {
    uint4 rd[G][2];
    if (rd_pre || rd_res || rd_c) {
#pragma unroll
      for (int s = 0; s < G; ++s) {
        const int m = m_base + (g0 + s) * RSTEP + er;
        rd[s][0] = rd[s][1] = make_uint4(0u, 0u, 0u, 0u);
        if (m < p.M) {
          const int64_t off = (int64_t)m * p.ldc + n;
          if (rd_pre) {
            rd[s][0] = *reinterpret_cast<const uint4*>(p.aux + off);
          } else if (rd_res) {
            rd[s][0] = *reinterpret_cast<const uint4*>(p.res + off);
          } else if (f32) {
            rd[s][0] = *reinterpret_cast<const uint4*>(reinterpret_cast<const float*>(p.c) + off);
            rd[s][1] = *reinterpret_cast<const uint4*>(reinterpret_cast<const float*>(p.c) + off + 4);
          } else {
            rd[s][0] = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(p.c) + off);
          }
        }
      }
    }
#pragma unroll
    for (int s = 0; s < G; ++s) {
      const int r = (g0 + s) * RSTEP + er;
      const int m = m_base + r;
      if (m >= p.M) break;
      float v[8];
      const f32x4 lo = *reinterpret_cast<const f32x4*>(img + r * RS + ec);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(img + r * RS + ec + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = lo[e] * p.alpha + bv[e];
        v[4 + e] = hi[e] * p.alpha + bv[4 + e];
      }
      const int64_t off = (int64_t)m * p.ldc + n;
      if (flags & kEpiAux) store8<bf16>(reinterpret_cast<bf16*>(p.aux + off), v);
      if (flags & kEpiGelu) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = gelu_tanh(v[e]);
      }
      // the 8 bf16 (or fp32) values this step read ahead
      float o[8];
      if (rd_pre || rd_res || (rd_c && !f32)) {
        const uint4 u = rd[s][0];
        o[0] = lo_bf16(u.x); o[1] = hi_bf16(u.x); o[2] = lo_bf16(u.y); o[3] = hi_bf16(u.y);
        o[4] = lo_bf16(u.z); o[5] = hi_bf16(u.z); o[6] = lo_bf16(u.w); o[7] = hi_bf16(u.w);
      } else if (rd_c) {
        const uint4 u0 = rd[s][0], u1 = rd[s][1];
        o[0] = __uint_as_float(u0.x); o[1] = __uint_as_float(u0.y); o[2] = __uint_as_float(u0.z);
        o[3] = __uint_as_float(u0.w); o[4] = __uint_as_float(u1.x); o[5] = __uint_as_float(u1.y);
        o[6] = __uint_as_float(u1.z); o[7] = __uint_as_float(u1.w);
      }
      if (rd_pre) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] *= gelu_tanh_grad_fast(o[e]);
      } else if (rd_c || rd_res) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += o[e];
      }
      if (flags & kEpiColSum) {
#pragma unroll
        for (int e = 0; e < 8; ++e) cs[e] += v[e];
      }
      if (f32) store8<float>(reinterpret_cast<float*>(p.c) + off, v);
      else store8<bf16>(reinterpret_cast<bf16*>(reinterpret_cast<uint16_t*>(p.c) + off), v);
    }
  }
}

// kEpiColSum: the per-thread column sums of epi_rows (8 columns, its rows of the tile) folded over the NT / 32
// threads that share those columns through LDS; one fp32 store per column of the tile (no atomics, deterministic).
template <int NT>
__device__ __forceinline__ void colsum_finish(const GemmArgs& p, float* red, const float* cs, int tid, int m0,
                                              int n0) {
  constexpr int R = NT / 32;
  const int ec = (tid & 31) * 8, er = tid / 32;
  __syncthreads();  // every thread is done reading the epilogue image
  *reinterpret_cast<float4*>(red + er * 256 + ec) = make_float4(cs[0], cs[1], cs[2], cs[3]);
  *reinterpret_cast<float4*>(red + er * 256 + ec + 4) = make_float4(cs[4], cs[5], cs[6], cs[7]);
  __syncthreads();
  for (int c = tid; c < 256; c += NT) {
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < R; ++r) s += red[r * 256 + c];
    if (n0 + c < p.N) p.stats[(int64_t)(m0 >> 8) * p.N + n0 + c] = s;
  }
}

// SEG: 0 plain operands; 1 K-segmented, 2 N-segmented operands (GemmArgs::nseg, pa_gemm_bf16_pp_segs). The
// segment selection is compiled only into the segmented instantiations: the plain kernel's staging code (and its
// register allocation) is the unsegmented ping-pong loop.
template <bool AK, bool BKM, int SEG = 0>
__global__ __launch_bounds__(kThreads, 1) void gemm256_kernel(GemmArgs p0) {
  GemmArgs p = split_view<AK, BKM>(p0);
  constexpr int HALF = 128 * kBK * 2;  // 16 KiB
  constexpr int STAGE = 4 * HALF;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 2, wn = wave & 3;

  // Balanced tail: the first full_tiles workgroups (a whole number of waves over the CUs) own whole
  // tiles; the remaining tiles are cut along K so the last wave is as wide as the chip (320 tiles of a
  // 4096 x 5120 output on 256 CUs: 256 whole + 64 x 4 quarter tiles = 1.25 tile-times instead of 2).
  const int bid = (int)blockIdx.x;
  int pid;
  float* tail_out = nullptr;
  int kt0 = 0;  // first global K-tile of this workgroup (tail slices start inside K)
  if (p.tail_split > 0 && bid >= p.full_tiles) {
    const int u = bid - p.full_tiles;
    const int ks = u % p.tail_split;
    pid = p.full_tiles + u / p.tail_split;
    p.K /= p.tail_split;
    if constexpr (SEG == 0) {  // plain operands: the slice's operand bases move (the round-4 kernel)
      p.a += (int64_t)ks * p.K * (AK ? 1 : p.lda);
      p.b += (int64_t)ks * p.K * (BKM ? 1 : p.ldb);
    } else {  // segmented operands: the slice's first global K-tile selects the segment
      kt0 = ks * (p.K / kBK);
    }
    tail_out = p.tail_ws + (int64_t)u * 65536;
  } else {
    pid = xcd_remap(bid, p.tail_split > 0 ? p.full_tiles : p.tiles_m * p.tiles_n);
  }
  int tm, tn;
  tile_coords(pid, p.tiles_m, p.tiles_n, &tm, &tn);
  const int m0 = tm * 256, n0 = tn * 256;
  const int nk = p.K / kBK;

  // Staging of the A (h = 0, 2: rows m0, m0 + 128) or B (h = 1, 3: columns n0, n0 + 128) half of local K-tile t,
  // through the operand segments when there are any (wave-uniform selects).
  auto stage_half = [&](int t, int h, char* dst) {
    const int tg = SEG == 0 ? t : kt0 + t;
    int k0 = tg * kBK;
    const uint16_t* a = p.a;
    const uint16_t* b = p.b;
    int64_t lda = p.lda, ldb = p.ldb;
    if constexpr (SEG == 1) {
      const int s = seg_of(p, tg);
      k0 = (tg - pick4(s, 0, p.seg_end[0], p.seg_end[1], p.seg_end[2])) * kBK;
      a = pick4(s, p.seg_a[0], p.seg_a[1], p.seg_a[2], p.seg_a[3]);
      b = pick4(s, p.seg_b[0], p.seg_b[1], p.seg_b[2], p.seg_b[3]);
      lda = pick4(s, p.seg_lda[0], p.seg_lda[1], p.seg_lda[2], p.seg_lda[3]);
      ldb = pick4(s, p.seg_ldb[0], p.seg_ldb[1], p.seg_ldb[2], p.seg_ldb[3]);
    }
    if (h == 0 || h == 2) {
      stage<128, AK>(a, lda, m0 + (h == 2 ? 128 : 0), p.M, k0, dst, wave, lane);
    } else {
      int c0 = n0 + (h == 3 ? 128 : 0), cmax = p.N;
      if constexpr (SEG == 2) {  // column segments: segment s owns columns [seg_end[s-1], seg_end[s]) of C
        const int s = seg_of(p, c0);
        const int start = pick4(s, 0, p.seg_end[0], p.seg_end[1], p.seg_end[2]);
        b = pick4(s, p.seg_b[0], p.seg_b[1], p.seg_b[2], p.seg_b[3]);
        ldb = pick4(s, p.seg_ldb[0], p.seg_ldb[1], p.seg_ldb[2], p.seg_ldb[3]);
        cmax = pick4(s, p.seg_end[0], p.seg_end[1], p.seg_end[2], p.seg_end[3]) - start;
        c0 -= start;
      }
      stage<128, BKM>(b, ldb, c0, cmax, k0, dst, wave, lane);
    }
  };
  // issue half-tile j (tile j>>2, half j&3) into buffer (j>>2)&1
  auto issue = [&](int j) {
    const int t = j >> 2, h = j & 3;
    stage_half(t, h, smem + (t & 1) * STAGE + h * HALF);
  };
  // the same with the half known at compile time (steady-state body: no branch on h)
  auto issue_h = [&](int t, auto hc) {
    constexpr int h = decltype(hc)::value;
    stage_half(t, h, smem + (t & 1) * STAGE + h * HALF);
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

  // Half-tile j is issued in phase j - 6 (phase = 4 * tile + p). Before each phase that reads a
  // half-tile the waves wait (in the previous phase, before its first barrier) until that half-tile
  // is retired: vmcnt = 2 * (half-tiles issued after it).
  const int last_j = 4 * nk - 1;
  auto wait_for = [&](int phase, int jstar) {
    const int issued = min(phase + 6, last_j);
    vm_wait(2 * max(issued - jstar, 0));
  };
  const int npro = min(6, 4 * nk);
#pragma unroll 1
  for (int j = 0; j < npro; ++j) issue(j);
  vm_wait(2 * max(min(5, last_j) - 1, 0));  // H0, H1 of tile 0
  bar();
  // ping-pong: the wm == 1 waves run one barrier behind, so on every SIMD one wave issues its
  // MFMA cluster while the other does its ds_reads / glds (+1 barrier at the end for wm == 0).
  const bool lag = __builtin_amdgcn_readfirstlane(wm) == 1;
  if (lag) bar();

  bf16x8_t af[4][2], bl[2][2], br[2][2];
  const int ar = wm * 64, bc = wn * 32;

  // One K-tile = 4 phases. STEADY (t <= nk - 3): every issue happens and every wait count is the
  // constant of the formula above (issued - jstar = 3, 5, 4 half-tiles -> vmcnt 6, 10, 8), so the body
  // has no branches; the last two tiles run the generic body with clamped counts.
  auto ktile = [&](int t, auto steady) {
    constexpr bool S = decltype(steady)::value;
    const char* buf = smem + (t & 1) * STAGE;
    const int ph = 4 * t;
    // ---- phase 0: read A-top + B-left; issue j = ph + 6; MFMA (top, L)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j) bl[j][ks] = frag<128, BKM>(buf + HALF, bc + j * 16, ks, lane);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i][ks] = frag<128, AK>(buf, ar + i * 16, ks, lane);
    if (S) {
      issue_h(t + 1, H2_{});
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // B-right of this tile, read in phase 1
    } else {
      if (ph + 6 <= last_j) issue(ph + 6);
      wait_for(ph, ph + 3);
    }
    bar();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[0][i][0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl[j][ks], af[i][ks], acc[0][i][0][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    bar();
    // ---- phase 1: read B-right; issue j = ph + 7; MFMA (top, R)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j) br[j][ks] = frag<128, BKM>(buf + 3 * HALF, bc + j * 16, ks, lane);
    if (S) {
      issue_h(t + 1, H3_{});
      asm volatile("s_waitcnt vmcnt(10)" ::: "memory");  // A-bottom of this tile, read in phase 2
    } else {
      if (ph + 7 <= last_j) issue(ph + 7);
      wait_for(ph + 1, ph + 2);
    }
    bar();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[0][i][1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(br[j][ks], af[i][ks], acc[0][i][1][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    bar();
    // ---- phase 2: read A-bottom; issue j = ph + 8; MFMA (bottom, L)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i][ks] = frag<128, AK>(buf + 2 * HALF, ar + i * 16, ks, lane);
    if (S) issue_h(t + 2, H0_{});
    else if (ph + 8 <= last_j) issue(ph + 8);
    bar();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[1][i][0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl[j][ks], af[i][ks], acc[1][i][0][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    bar();
    // ---- phase 3: issue j = ph + 9; wait for H0/H1 of tile t+1; MFMA (bottom, R)
    if (S) {
      issue_h(t + 2, H1_{});
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      if (ph + 9 <= last_j) issue(ph + 9);
      if (t + 1 < nk) wait_for(ph + 3, ph + 5);
    }
    bar();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[1][i][1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(br[j][ks], af[i][ks], acc[1][i][1][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    bar();
  };
  const int nsteady = max(nk - 2, 0);
  int t = 0;
#pragma unroll 1
  for (; t < nsteady; ++t) ktile(t, True_{});
#pragma unroll 1
  for (; t < nk; ++t) ktile(t, False_{});
  if (!lag) bar();

  if (tail_out) {  // K-slice of a tail tile: raw fp32 partial, row-major 256 x 256
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

  // ---- epilogue, staged through LDS in two 128-row halves: the accumulators go to a row-major fp32 image
  // (1040-byte rows: the 16 rows of a ds_write_b128 lane group land on distinct banks), then every thread
  // owns 8 consecutive columns and walks 8 row steps of 16 rows, so each wave instruction moves whole
  // 512-byte (bf16) / 1 KiB (fp32) row segments — bias / alpha / pre-activation / GELU / accumulate are
  // applied in that coalesced phase. The scattered 8-byte fragment stores left the tile wave's final burst
  // (aux / accumulate read-modify-write) far below the HBM rate.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int flags = p.flags;
  if (!(flags & kEpiStaged)) {
    // bf16 output without aux / accumulate: alpha, bias and GELU applied in registers, the finished bf16 tile
    // staged through LDS in one pass ([256][264] bf16, 528-byte rows) instead of two fp32 halves
    uint16_t* im = reinterpret_cast<uint16_t*>(smem);
    constexpr int RSB = kEpiRowStrideBf16;
    bar();
#pragma unroll
    for (int bh = 0; bh < 2; ++bh)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = bh * 128 + bc + j * 16 + 4 * (lane >> 4);
        float bq[4] = {0.f, 0.f, 0.f, 0.f};
        if ((flags & kEpiBias) && n0 + c < p.N) {
          const uint2 braw = *reinterpret_cast<const uint2*>(p.bias + n0 + c);
          bq[0] = lo_bf16(braw.x); bq[1] = hi_bf16(braw.x); bq[2] = lo_bf16(braw.y); bq[3] = hi_bf16(braw.y);
        }
#pragma unroll
        for (int ah = 0; ah < 2; ++ah)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = ah * 128 + ar + i * 16 + (lane & 15);
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v[e] = acc[ah][i][bh][j][e] * p.alpha + bq[e];
              if (flags & kEpiGelu) v[e] = gelu_tanh(v[e]);
            }
            *reinterpret_cast<uint2*>(im + r * RSB + c) = make_uint2(pack_bf16(v[0], v[1]), pack_bf16(v[2], v[3]));
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
            *reinterpret_cast<const uint4*>(im + r * RSB + ecb);
      }
    }
    return;
  }
  float* img = reinterpret_cast<float*>(smem);
  constexpr int RS = kEpiRowStride;  // floats per image row
  float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  {
    const int n = n0 + (tid & 31) * 8;
    if ((flags & kEpiBias) && n < p.N) load8<bf16>(reinterpret_cast<const bf16*>(p.bias + n), bv);
  }
#pragma unroll
  for (int ah = 0; ah < 2; ++ah) {
    bar();
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int bh = 0; bh < 2; ++bh)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int r = ar + i * 16 + (lane & 15);
          const int c = bh * 128 + bc + j * 16 + 4 * (lane >> 4);
          *reinterpret_cast<f32x4*>(img + r * RS + c) = acc[ah][i][bh][j];
        }
    bar();
    epi_rows<kThreads>(p, img, m0 + ah * 128, n0, tid, bv, cs);
  }
  if (flags & kEpiColSum) colsum_finish<kThreads>(p, img, cs, tid, m0, n0);
}

// ---------------------------------------------------------------------------------------------
// 256x256 tile, 4 waves (one per SIMD), 128x128 outputs per wave held in the accumulator file.
// The 8-wave ping-pong kernel above hides latency by pairing two waves on each SIMD; PMC showed 31 % of its
// wave cycles parked (barriers every phase, each wave reading its fragments from LDS while its partner
// computes). This form keeps one wave per SIMD and hides latency inside the wave instead:
//   * 8 x 8 MFMA 16x16x32 fragments per wave = 256 fp32 accumulators -> AGPRs (launch bounds 256 x 1 give the
//     wave the whole 512-entry register file); a third less LDS read traffic per MFMA than 128x64 wave tiles.
//   * K-tiles of 32 in a 4-slot LDS ring (4 x 32 KiB): tile t+1 is read into the second fragment register set
//     while the 64 MFMAs of tile t run; tiles t+2, t+3 (+ t+4 issued after the barrier) stay in flight, so a
//     glds has three K-tiles (~3k cycles) to land. One barrier per K-tile.
//   * K-major images [256][32] (64-B rows) with the chunk swizzle c ^ 2*((row >> 3) & 1): the 16 rows x 4 chunks
//     of one fragment ds_read_b128 hit 16 distinct 16-B bank slots in each lane group. MN-major images [32][256]
//     (512-B rows) use the mn_swz swizzle and ds_read_b64_tr_b16 like the kernels above.
__device__ __forceinline__ int k32_swz(int row) { return ((row >> 3) & 1) << 1; }

typedef int i32x4 __attribute__((ext_vector_type(4)));

// LDS-DMA staging of one operand's 256 x 32 tile through buffer_load_dwordx4 ... lds: the buffer descriptor
// holds the tile's base address (advanced by scalar adds per K-tile), each lane's byte offset inside the tile
// window is loop-invariant (4 pieces per wave), M0 the wave-uniform LDS destination: no VALU per load.
template <bool KMAJ>
struct Loader32 {
  uint64_t base;    // wave-uniform address of (first row / column of the tile, k = 0)
  uint64_t kstep;   // bytes per K-tile of 32
  int voff[4];      // per-lane byte offsets of this wave's 4 pieces

  __device__ __forceinline__ void init(const uint16_t* g, int64_t ld, int r0, int rmax, int wave, int lane) {
    base = reinterpret_cast<uint64_t>(g) + (KMAJ ? (uint64_t)r0 * ld * 2 : (uint64_t)r0 * 2);
    kstep = KMAJ ? 64 : (uint64_t)ld * 64;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = i * 4 + wave;  // 1-KiB piece of the 16-KiB operand image
      if constexpr (KMAJ) {
        const int row = q * 16 + (lane >> 2);
        const int c = (lane & 3) ^ k32_swz(row);
        const int gr = min(r0 + row, rmax - 1) - r0;
        voff[i] = gr * (int)ld * 2 + c * 16;
      } else {
        const int lin = q * 64 + lane;
        const int row = lin >> 5;  // k
        const int lc = (lin & 31) ^ mn_swz(row);
        const int gc = min(r0 + lc * 8, rmax - 8) - r0;
        voff[i] = row * (int)ld * 2 + gc * 2;
      }
    }
  }
  // piece i of K-tile t into the operand image at LDS byte address img (wave-uniform)
  __device__ __forceinline__ void load(int t, int i, uint32_t img, int wave) const {
    const uint64_t b = base + (uint64_t)t * kstep;
    i32x4 srd;
    srd[0] = (int)(uint32_t)b;
    srd[1] = (int)((uint32_t)(b >> 32) & 0xffff);
    srd[2] = -1;
    srd[3] = 0x00020000;
    const uint32_t m0 = img + (uint32_t)(i * 4 + wave) * 1024u;
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff[i]), "s"(srd),
                 "s"(m0)
                 : "memory");
  }
};

template <bool KMAJ>
__device__ __forceinline__ bf16x8_t frag32(const char* img, int rbase, int lane) {
  if constexpr (KMAJ) {
    const int row = rbase + (lane & 15);
    const int c = (lane >> 4) ^ k32_swz(row);
    Frag8 f;
    f.u = *reinterpret_cast<const uint4*>(img + row * 64 + (c << 4));
    return f.v;
  } else {
    return frag<256, false>(img, rbase, 0, lane);
  }
}

// acc += a . b with the accumulator pinned to the AGPR file ("+a"): the builtin lets the register allocator
// move accumulators between the AGPR and VGPR halves of the unified file across the unrolled K-loop (hundreds
// of v_accvgpr moves per K-tile). Operands come straight from ds_read (the compiler's lgkmcnt covers them); the
// accumulator is re-read by the next MFMA on it 64 MFMAs later, so no MFMA->MFMA hazard arises.
__device__ __forceinline__ void mfma_acc(f32x4& acc, const bf16x8_t& a, const bf16x8_t& b) {
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// vmcnt for "tile t+1 has landed" at the top of K-iteration t: the tiles issued after it stay in flight
__device__ __forceinline__ void wait_tiles_after(int n_after) {
  if (n_after >= 3) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else if (n_after == 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if (n_after == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ABL (diagnostic ablations, timing only, wrong results): 1 = no global loads in the K-loop, 2 = no global
// loads and no fragment reads, 3 = 2 without the per-tile barrier, 5 = loads issued but never waited for in the
// K-loop (load latency taken out, issue cost and bandwidth kept)
template <bool AK, bool BKM, int ABL = 0, int NSLOT = 4>
__global__ __launch_bounds__(256, 1) void gemm4w_kernel(GemmArgs p) {
  constexpr int BK = 32;
  constexpr int OPB = 256 * BK * 2;  // 16 KiB per operand image
  constexpr int SLOT = 2 * OPB;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;

  // balanced tail as in gemm256_kernel
  const int bid = (int)blockIdx.x;
  int pid;
  float* tail_out = nullptr;
  if (p.tail_split > 0 && bid >= p.full_tiles) {
    const int u = bid - p.full_tiles;
    const int ks = u % p.tail_split;
    pid = p.full_tiles + u / p.tail_split;
    p.K /= p.tail_split;
    p.a += (int64_t)ks * p.K * (AK ? 1 : p.lda);
    p.b += (int64_t)ks * p.K * (BKM ? 1 : p.ldb);
    tail_out = p.tail_ws + (int64_t)u * 65536;
  } else {
    pid = xcd_remap(bid, p.tail_split > 0 ? p.full_tiles : p.tiles_m * p.tiles_n);
  }
  int tm, tn;
  tile_coords(pid, p.tiles_m, p.tiles_n, &tm, &tn);
  const int m0 = tm * 256, n0 = tn * 256;
  const int nk = p.K / BK;

  const int wv = __builtin_amdgcn_readfirstlane(wave);
  Loader32<AK> la;
  Loader32<BKM> lb;
  la.init(p.a, p.lda, m0, p.M, wv, lane);
  lb.init(p.b, p.ldb, n0, p.N, wv, lane);
  const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>(smem);
  // piece g (0..3: A, 4..7: B) of this wave's share of K-tile t
  auto piece = [&](int t, int g) {
    const uint32_t slot = lds0 + (uint32_t)(t % NSLOT) * SLOT;
    if (g < 4) la.load(t, g, slot, wv);
    else lb.load(t, g - 4, slot + OPB, wv);
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  asm volatile("s_nop 4" ::: "memory");  // v_accvgpr_write of the zeros -> first MFMA reading them as C
  bf16x8_t fa0[8], fb0[8], fa1[8], fb1[8];
  const int ar = wm * 128, bc = wn * 128;
  // K-iteration t: F(t) = (fc, gc) is in registers. Wait for tile t+1, barrier (every wave has read F(t) out of
  // slot t % 4, and tile t+1 is visible), then 8 groups of {one LDS-DMA piece of tile t+4 into slot t % 4,
  // two fragment reads of F(t+1), the 8 MFMAs of fragment row g}: the loads issue in the MFMA gaps.
  auto step = [&](int t, const bf16x8_t(&fc)[8], const bf16x8_t(&gc)[8], bf16x8_t(&fn)[8], bf16x8_t(&gn)[8],
                  auto full) {
    constexpr bool F = decltype(full)::value;
    if (ABL != 5) {
      if (F) wait_tiles_after(NSLOT - 2);
      else if (t + 1 < nk) wait_tiles_after(min(t + NSLOT - 1, nk - 1) - (t + 1));
    }
    if (ABL < 3 || ABL == 5) bar();
    const bool iss = (F || t + NSLOT < nk) && ABL == 0;
    const bool rd = (F || t + 1 < nk) && ABL < 2;
    const char* nb = smem + ((t + 1) % NSLOT) * SLOT;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      // fillers spread over the MFMA gaps (a wave alone on its SIMD issues nothing else while an MFMA holds the
      // issue port, so fillers bunched ahead of the MFMAs would all be exposed): after MFMA 0 the LDS-DMA piece;
      // the 16 fragment reads of F(t+1) early in the step (groups 0..5), so the next step's first MFMAs never
      // wait on a read issued a few MFMAs before them (lgkmcnt counts in order)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        mfma_acc(acc[g][k], gc[k], fc[g]);
        if (k == 0 && iss) piece(t + NSLOT, g);
        const int r = 3 * g + (k - 1) / 2;  // fragment read r of F(t+1) after MFMAs 1, 3, 5 of groups 0..5
        if ((k & 1) && k < 6 && r < 16 && rd) {
          if (r < 8) gn[r] = frag32<BKM>(nb + OPB, bc + r * 16, lane);
          else fn[r - 8] = frag32<AK>(nb, ar + (r - 8) * 16, lane);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };

  const int npro = min(NSLOT, nk);
#pragma unroll 1
  for (int t = 0; t < npro; ++t)
#pragma unroll
    for (int g = 0; g < 8; ++g) piece(t, g);
  if (npro == 5) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");  // tile 0 landed, tiles 1.. in flight
  else wait_tiles_after(npro - 1);
  bar();
#pragma unroll
  for (int j = 0; j < 8; ++j) fb0[j] = frag32<BKM>(smem + OPB, bc + j * 16, lane);
#pragma unroll
  for (int i = 0; i < 8; ++i) fa0[i] = frag32<AK>(smem, ar + i * 16, lane);
  int t = 0;
#pragma unroll 1
  for (; t + 1 + NSLOT < nk; t += 2) {  // steady state: every load is issued, constant wait counts
    step(t, fa0, fb0, fa1, fb1, True_{});
    step(t + 1, fa1, fb1, fa0, fb0, True_{});
  }
#pragma unroll 1
  for (; t + 1 < nk; t += 2) {
    step(t, fa0, fb0, fa1, fb1, False_{});
    step(t + 1, fa1, fb1, fa0, fb0, False_{});
  }
  if (t < nk) step(t, fa0, fb0, fa1, fb1, False_{});
  // the last MFMAs' results -> v_accvgpr_read by compiler code (hipcc pads nothing after an asm MFMA)
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 15\n\ts_nop 7" ::: "memory");

  if (tail_out) {  // K-slice of a tail tile: raw fp32 partial, row-major 256 x 256
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int r = ar + i * 16 + (lane & 15);
        const int c = bc + j * 16 + 4 * (lane >> 4);
        const f32x4 v = acc[i][j];
        *reinterpret_cast<float4*>(tail_out + r * 256 + c) = make_float4(v[0], v[1], v[2], v[3]);
      }
    return;
  }

  // epilogue through LDS, one 128-row half at a time (the two waves with wm == half write their accumulators)
  float* img = reinterpret_cast<float*>(smem);
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  {
    const int n = n0 + (tid & 31) * 8;
    if ((p.flags & kEpiBias) && n < p.N) load8<bf16>(reinterpret_cast<const bf16*>(p.bias + n), bv);
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    bar();
    if (wm == h) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int r = i * 16 + (lane & 15);
          const int c = bc + j * 16 + 4 * (lane >> 4);
          *reinterpret_cast<f32x4*>(img + r * kEpiRowStride + c) = acc[i][j];
        }
    }
    bar();
    epi_rows<256>(p, img, m0 + h * 128, n0, tid, bv, cs);
  }
  if (p.flags & kEpiColSum) colsum_finish<256>(p, img, cs, tid, m0, n0);
}

// ---------------------------------------------------------------------------------------------
// 256 x 160 x 64 tiles in a 3-stage LDS ring (3 x 52 KiB = 156 KiB of the 160 KiB LDS): two K-tiles
// of glds stay in flight while one is consumed, so the global->LDS latency is hidden by two K-tiles of
// MFMA work instead of one (PMC on the 256x256 two-stage kernel: 36 % of wave cycles waiting on
// vmcnt / barrier). 160 columns also give whole waves of tiles on the GPT shapes (N = 5120 / 15360 /
// 20480 -> 32 / 96 / 128 column tiles; 256x256 leaves 1.25 waves at N = 5120).
// 8 waves as 4 (M) x 2 (N), wave tile 64 x 80 (4 x 5 MFMA fragments).
// B images of 160 columns: K-major [160][64] (as above); MN-major [64][160] with 320-B rows, which
// already rotate by 64 B per row, plus a 32-B XOR on rows with bit 3 set so the 8 rows of one
// ds_read_b64_tr_b16 half-wave land on 8 distinct 32-B slots.
constexpr int kBN3 = 160;

template <int R, bool KMAJ>
__device__ __forceinline__ void stage_r(const uint16_t* __restrict__ g, int64_t ld, int r0, int rmax, int k0,
                                        char* img, int wave, int lane) {
  constexpr int NI = R / 8;               // wave-instructions (1 KiB each) per operand tile
  constexpr int PER = (NI + 7) / 8;       // per wave; the overflow slots repeat an existing instruction
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    int q = i * 8 + wave;
    if (q >= NI) q -= 8 * PER - NI;       // same bytes to the same LDS place: a benign duplicate
    if constexpr (KMAJ) {
      const int row = q * 8 + (lane >> 3);
      const int lc = (lane & 7) ^ ((row >> 1) & 7);
      int gr = r0 + row;
      gr = gr < rmax ? gr : rmax - 1;
      glds16(g + (int64_t)gr * ld + k0 + lc * 8, img + q * 1024);
    } else {
      constexpr int CPR = R / 8;
      const int lin = q * 64 + lane;
      const int row = lin / CPR;
      const int sw = (R == 160) ? (((row >> 3) & 1) << 1) : mn_swz(row);
      const int lc = (lin % CPR) ^ sw;
      int gc = r0 + lc * 8;
      gc = gc < rmax ? gc : rmax - 8;
      glds16(g + (int64_t)(k0 + row) * ld + gc, img + q * 1024);
    }
  }
}

template <int R, bool KMAJ>
__device__ __forceinline__ bf16x8_t frag_r(const char* img, int rbase, int s, int lane) {
  if constexpr (KMAJ || R != 160) {
    return frag<R, KMAJ>(img, rbase, s, lane);
  } else {
    Frag8 f;
    const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
    const int col = rbase + pp * 4;
    const int lc = col >> 3, sub = (col & 7) * 2;
    const int k1 = s * 32 + g * 8 + q, k2 = k1 + 4;
    f.h[0] = lds_tr(img + k1 * (R * 2) + ((lc ^ (((k1 >> 3) & 1) << 1)) << 4) + sub);
    f.h[1] = lds_tr(img + k2 * (R * 2) + ((lc ^ (((k2 >> 3) & 1) << 1)) << 4) + sub);
    return f.v;
  }
}

// Per-thread precomputed output pixels of the 4 A rows this thread stages (implicit-GEMM conv).
struct ConvRows {
  int pix[4];  // n * D * H * W (first pixel of the image), or -1 for rows past M
  int db[4], hb[4], wb[4];
};

__device__ __forceinline__ ConvRows conv_rows(const GemmArgs& p, int m0, int wave, int lane) {
  ConvRows r;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (i * 8 + wave) * 8 + (lane >> 3);
    const int m = m0 + row;
    if (m < p.M) {
      const int hw = p.cHo * p.cWo, dhw = p.cDo * hw;
      const int n = m / dhw, r1 = m - n * dhw;
      const int dd = r1 / hw, rem = r1 - dd * hw;
      const int ho = rem / p.cWo, wo = rem - ho * p.cWo;
      r.pix[i] = n * p.cD * p.cH * p.cW;
      r.db[i] = dd * p.cStride - p.cPadD;
      r.hb[i] = ho * p.cStride - p.cPadH;
      r.wb[i] = wo * p.cStride - p.cPadW;
    } else {
      r.pix[i] = -1; r.db[i] = 0; r.hb[i] = 0; r.wb[i] = 0;
    }
  }
  return r;
}

// A tile (256 pixels x 64 channels of one filter tap) of K-tile k0, same LDS image as stage_r<256, true>
__device__ __forceinline__ void stage_conv(const GemmArgs& p, const ConvRows& cr, int k0, char* img, int wave,
                                           int lane) {
  const int tap = k0 / p.cC, c0 = k0 - tap * p.cC;
  const int kd = tap / p.cKHW, t2 = tap - kd * p.cKHW;
  const int kh = t2 / p.cKW, kw = t2 - kh * p.cKW;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = i * 8 + wave;
    const int row = q * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ ((row >> 1) & 7);
    const int di = cr.db[i] + kd * p.cDil, hi = cr.hb[i] + kh * p.cDil, wi = cr.wb[i] + kw * p.cDil;
    const bool ok = cr.pix[i] >= 0 && di >= 0 && di < p.cD && hi >= 0 && hi < p.cH && wi >= 0 && wi < p.cW;
    const uint16_t* src =
        ok ? p.a + ((int64_t)(cr.pix[i] + (di * p.cH + hi) * p.cW + wi) * p.cC + c0 + lc * 8) : p.zero + lc * 8;
    glds16(src, img + q * 1024);
  }
}

template <bool AK, bool BKM, bool CONV = false>
__global__ __launch_bounds__(kThreads, 1) void gemm3s_kernel(GemmArgs p0) {
  const GemmArgs p = split_view<AK, BKM>(p0);
  constexpr int BN = kBN3;
  constexpr int A_BYTES = kBM * kBK * 2;
  constexpr int B_BYTES = BN * kBK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int MR = 4, NR = 5;
  constexpr int NL = (kBM / 8 + 7) / 8 + (BN / 8 + 7) / 8;  // glds per thread per K-tile (4 + 3)
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;

  const int nwg = p.tiles_m * p.tiles_n;
  const int pid = xcd_remap((int)blockIdx.x, nwg);
  constexpr int GM = 8;
  const int per_group = GM * p.tiles_n;
  const int gid = pid / per_group;
  const int first_m = gid * GM;
  const int gsz = min(p.tiles_m - first_m, GM);
  const int tm = first_m + (pid % per_group) % gsz;
  const int tn = (pid % per_group) / gsz;
  const int m0 = tm * kBM, n0 = tn * BN;

  f32x4 acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / kBK;
  ConvRows cr;
  if constexpr (CONV) cr = conv_rows(p, m0, wave, lane);
  auto stage_tile = [&](int t) {
    char* base = smem + (t % 3) * STAGE;
    if constexpr (CONV) stage_conv(p, cr, t * kBK, base, wave, lane);
    else stage_r<kBM, AK>(p.a, p.lda, m0, p.M, t * kBK, base, wave, lane);
    stage_r<BN, BKM>(p.b, p.ldb, n0, p.N, t * kBK, base + A_BYTES, wave, lane);
  };

  stage_tile(0);
  if (nk > 1) {
    stage_tile(1);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NL) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  bar();

#pragma unroll 1
  for (int t = 0; t < nk; ++t) {
    const bool pre = t + 2 < nk;
    if (pre) stage_tile(t + 2);
    const char* aimg = smem + (t % 3) * STAGE;
    const char* bimg = aimg + A_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8_t bf[NR];
#pragma unroll
      for (int j = 0; j < NR; ++j) bf[j] = frag_r<BN, BKM>(bimg, wn * 80 + j * 16, s, lane);
#pragma unroll
      for (int i = 0; i < MR; ++i) {
        const bf16x8_t af = frag_r<kBM, AK>(aimg, wm * 64 + i * 16, s, lane);
#pragma unroll
        for (int j = 0; j < NR; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af, acc[i][j], 0, 0, 0);
      }
    }
    if (pre) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NL) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();
  }

  const int flags = p.flags;
  const int mrow0 = m0 + wm * 64 + (lane & 15);
  const int ncol0 = n0 + wn * 80 + 4 * (lane >> 4);
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const int n = ncol0 + j * 16;
    if (n >= p.N) continue;
    float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
    float bsc[4] = {0.f, 0.f, 0.f, 0.f}, bsh[4] = {0.f, 0.f, 0.f, 0.f}, bmu[4] = {0.f, 0.f, 0.f, 0.f};
    if (flags & kEpiStatsBwd) bn_cols(p, n, bsc, bsh, bmu);
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (flags & kEpiBias) {
      const uint2 braw = *reinterpret_cast<const uint2*>(p.bias + n);
      bv[0] = lo_bf16(braw.x); bv[1] = hi_bf16(braw.x); bv[2] = lo_bf16(braw.y); bv[3] = hi_bf16(braw.y);
    }
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      const int m = mrow0 + i * 16;
      if (m >= p.M) continue;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] * p.alpha + bv[e];
      const int64_t off = (int64_t)m * p.ldc + n;
      if (flags & kEpiAux)
        *reinterpret_cast<uint2*>(p.aux + off) = make_uint2(pack_bf16(v[0], v[1]), pack_bf16(v[2], v[3]));
      if (flags & kEpiGelu) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = gelu_tanh(v[e]);
      }
      if (flags & kEpiOutF32) {
        float4* cp = reinterpret_cast<float4*>(reinterpret_cast<float*>(p.c) + off);
        if (flags & kEpiAccum) {
          const float4 o = *cp;
          v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
        }
        *cp = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        uint2* cp = reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(p.c) + off);
        if (flags & kEpiAccum) {
          const uint2 o = *cp;
          v[0] += lo_bf16(o.x); v[1] += hi_bf16(o.x); v[2] += lo_bf16(o.y); v[3] += hi_bf16(o.y);
        }
        const uint2 o = make_uint2(pack_bf16(v[0], v[1]), pack_bf16(v[2], v[3]));
        *cp = o;
        if (flags & kEpiStatsBwd) {
          stats_add_bwd(p, off, o, bsc, bsh, bmu, s1, s2);
        } else if (flags & kEpiStats) {
          stats_add2(o.x, s1, s2, 0);
          stats_add2(o.y, s1, s2, 2);
        }
      }
    }
    if (flags & kEpiStats) stats_store(p, tm * 4 + wm, p.tiles_m * 4, n, lane, s1, s2);
  }
}

template <bool AK, bool BKM, bool CONV = false>
int launch3s(const GemmArgs& a0, int splits, hipStream_t st) {
  GemmArgs a = a0;
  a.tiles_m = (a.M + kBM - 1) / kBM;
  a.tiles_n = (a.N + kBN3 - 1) / kBN3;
  const int smem = 3 * (kBM + kBN3) * kBK * 2;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm3s_kernel<AK, BKM, CONV>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              smem);
    attr_set = true;
  }
  hipLaunchKernelGGL((gemm3s_kernel<AK, BKM, CONV>), dim3(a.tiles_m * a.tiles_n, splits), dim3(kThreads), smem, st,
                     a);
  return (int)hipGetLastError();
}

template <bool AK, bool BKM, int SEG>
int launch256_seg(const GemmArgs& a0, int splits, hipStream_t st, int grid) {
  GemmArgs a = a0;
  a.tiles_m = (a.M + 255) / 256;
  a.tiles_n = (a.N + 255) / 256;
  if (!grid) {
    grid = a.tiles_m * a.tiles_n;
    a.tail_split = 0;
  }
  constexpr int kLoop = 2 * 4 * 128 * kBK * 2, kEpi0 = 128 * kEpiRowStride * 4, kEpi1 = 256 * kEpiRowStrideBf16 * 2;
  constexpr int kEpi = kEpi0 > kEpi1 ? kEpi0 : kEpi1;
  const int smem = kLoop > kEpi ? kLoop : kEpi;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm256_kernel<AK, BKM, SEG>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              smem);
    attr_set = true;
  }
  hipLaunchKernelGGL((gemm256_kernel<AK, BKM, SEG>), dim3(grid, splits), dim3(kThreads), smem, st, a);
  return (int)hipGetLastError();
}

template <bool AK, bool BKM>
int launch256(const GemmArgs& a0, int splits, hipStream_t st, int grid = 0, int seg = 0) {
  if (seg == 1) return launch256_seg<AK, BKM, 1>(a0, splits, st, grid);
  if (seg == 2) return launch256_seg<AK, BKM, 2>(a0, splits, st, grid);
  return launch256_seg<AK, BKM, 0>(a0, splits, st, grid);
}

template <int BN, bool AK, bool BKM>
int launch(const GemmArgs& a0, int splits, hipStream_t st) {
  if constexpr (BN == 0) return launch256<AK, BKM>(a0, splits, st);
  if constexpr (BN == 160) return launch3s<AK, BKM>(a0, splits, st);
  GemmArgs a = a0;
  constexpr int NW = BN == 4 ? 4 : 8;                  // BN code 4: 256x256 tile with 4 waves
  constexpr int BNk = (BN == 0 || BN == 4) ? 256 : BN;
  a.tiles_m = (a.M + kBM - 1) / kBM;
  a.tiles_n = (a.N + BNk - 1) / BNk;
  const int smem = 2 * (kBM + BNk) * kBK * 2;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm_bf16_kernel<BNk, AK, BKM, NW>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr_set = true;
  }
  hipLaunchKernelGGL((gemm_bf16_kernel<BNk, AK, BKM, NW>), dim3(a.tiles_m * a.tiles_n, splits), dim3(NW * 64), smem,
                     st, a);
  return (int)hipGetLastError();
}

template <int BN>
int dispatch_layout(const GemmArgs& a, int a_kmajor, int b_kmajor, int splits, hipStream_t st) {
  if (a_kmajor && !b_kmajor) return launch<BN, true, false>(a, splits, st);
  if (a_kmajor && b_kmajor) return launch<BN, true, true>(a, splits, st);
  if (!a_kmajor && !b_kmajor) return launch<BN, false, false>(a, splits, st);
  return launch<BN, false, true>(a, splits, st);
}

// ---------------------------------------------------------------------------------------------
// Small-M GEMM for decode (serving): C[M <= 64, N] = A[M, K] . B[K, N] with A K-major (activations,
// a few rows) and B MN-major (paddle's [in, out] weights, streamed once). The work is bandwidth-bound
// on B, so the kernel is built around keeping many weight bytes in flight: 4 waves, tile 64 x 128, K
// split over gridDim.y, a 4-deep LDS ring filled by glds (3 K-tiles = 72 KiB per CU in flight), one
// barrier per K-tile. Rows >= M are clamped reads whose results are never stored. Each split writes an
// fp32 slab; pa_gemm_small_m_reduce sums the slabs (+ bias) into bf16. Without a split the accumulators
// go straight to C. (A last-arriving-split reduction inside the kernel measured 2-3x slower: the agent-scope
// release fence it needs writes back the whole XCD L2 in every workgroup.)
constexpr int kSmBM = 64, kSmBN = 128, kSmNW = 4;

template <int kSmStages>
__global__ __launch_bounds__(kSmNW * 64, 1) void gemm_small_m_kernel(const uint16_t* __restrict__ a, int64_t lda,
                                                                    const uint16_t* __restrict__ b, int64_t ldb,
                                                                    float* __restrict__ ws, int M, int N, int k_per,
                                                                    const uint16_t* __restrict__ bias,
                                                                    uint16_t* __restrict__ c, int64_t ldc) {
  constexpr int A_BYTES = kSmBM * kBK * 2, B_BYTES = kSmBN * kBK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int NL = kSmBM / (8 * kSmNW) + kSmBN / (8 * kSmNW);  // glds per thread per K-tile (2 + 4)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int n0 = blockIdx.x * kSmBN;
  const int ks = blockIdx.y;
  const uint16_t* ap = a + (int64_t)ks * k_per;
  const uint16_t* bp = b + (int64_t)ks * k_per * ldb;
  const int nk = k_per / kBK;

  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto stage_tile = [&](int t) {
    char* base = smem + (t % kSmStages) * STAGE;
    stage<kSmBM, true, kSmNW>(ap, lda, 0, M, t * kBK, base, wave, lane);
    stage<kSmBN, false, kSmNW>(bp, ldb, n0, N, t * kBK, base + A_BYTES, wave, lane);
  };
  const int pro = min(kSmStages - 1, nk);
  for (int t = 0; t < pro; ++t) stage_tile(t);
  // wait for tile 0: (pro - 1) tiles may stay in flight
  if (pro >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NL) : "memory");
  else if (pro == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NL) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bar();

#pragma unroll 1
  for (int t = 0; t < nk; ++t) {
    if (t + kSmStages - 1 < nk) stage_tile(t + kSmStages - 1);
    const char* aimg = smem + (t % kSmStages) * STAGE;
    const char* bimg = aimg + A_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8_t bf[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j] = frag<kSmBN, false>(bimg, wave * 32 + j * 16, s, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bf16x8_t af = frag<kSmBM, true>(aimg, i * 16, s, lane);
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af, acc[i][j], 0, 0, 0);
      }
    }
    // retire tile t+1 (tiles issued after it may stay in flight)
    const int after = min(nk - 1, t + kSmStages - 1) - (t + 1);
    if (after >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NL) : "memory");
    else if (after == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NL) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();
  }
  // lane holds C[m = i*16 + (lane&15)][n = n0 + wave*32 + j*16 + 4*(lane>>4) + 0..3]
  if (gridDim.y == 1) {  // no split: bias + bf16 straight from the accumulators, no reduction pass
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = i * 16 + (lane & 15);
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = n0 + wave * 32 + j * 16 + 4 * (lane >> 4);
        if (n >= N) continue;
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if (bias) {
          const uint2 braw = *reinterpret_cast<const uint2*>(bias + n);
          v[0] += lo_bf16(braw.x); v[1] += hi_bf16(braw.x); v[2] += lo_bf16(braw.y); v[3] += hi_bf16(braw.y);
        }
        *reinterpret_cast<uint2*>(c + (int64_t)m * ldc + n) = make_uint2(pack_bf16(v[0], v[1]), pack_bf16(v[2], v[3]));
      }
    }
    return;
  }
  float* out = ws + (int64_t)ks * M * N;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = i * 16 + (lane & 15);
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wave * 32 + j * 16 + 4 * (lane >> 4);
      if (n < N)
        *reinterpret_cast<float4*>(out + (int64_t)m * N + n) =
            make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    }
  }
}

__global__ __launch_bounds__(256) void gemm_small_m_reduce_k(const float* __restrict__ ws, const uint16_t* __restrict__ bias,
                                                            uint16_t* __restrict__ c, int64_t ldc, int M, int N,
                                                            int splits) {
  const int64_t i4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i4 >= (int64_t)M * N) return;
  const int m = (int)(i4 / N), n = (int)(i4 % N);
  float4 acc = *reinterpret_cast<const float4*>(ws + i4);
  for (int s = 1; s < splits; ++s) {
    const float4 v = *reinterpret_cast<const float4*>(ws + (int64_t)s * M * N + i4);
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  if (bias) {
    const uint2 braw = *reinterpret_cast<const uint2*>(bias + n);
    acc.x += lo_bf16(braw.x); acc.y += hi_bf16(braw.x); acc.z += lo_bf16(braw.y); acc.w += hi_bf16(braw.y);
  }
  *reinterpret_cast<uint2*>(c + (int64_t)m * ldc + n) = make_uint2(pack_bf16(acc.x, acc.y), pack_bf16(acc.z, acc.w));
}

// Balanced-tail reduction: tail tile b (blockIdx.x) = tile full_tiles + b; each thread sums the
// tail_split fp32 partials of 4 consecutive columns and applies the epilogue of the main kernel.
__global__ __launch_bounds__(256) void gemm_tail_reduce_k(GemmArgs p) {
  const int b = blockIdx.x;
  int tm, tn;
  tile_coords(p.full_tiles + b, p.tiles_m, p.tiles_n, &tm, &tn);
  const int e = (blockIdx.y * 256 + threadIdx.x) * 4;  // element of the 256 x 256 tile
  const int r = e >> 8, c = e & 255;
  const int m = tm * 256 + r, n = tn * 256 + c;
  if (m >= p.M || n >= p.N) return;
  const float* src = p.tail_ws + (int64_t)b * p.tail_split * 65536 + e;
  float4 a = *reinterpret_cast<const float4*>(src);
  for (int k = 1; k < p.tail_split; ++k) {
    const float4 v = *reinterpret_cast<const float4*>(src + (int64_t)k * 65536);
    a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
  }
  const int flags = p.flags;
  float bv[4] = {0.f, 0.f, 0.f, 0.f};
  if (flags & kEpiBias) {
    const uint2 braw = *reinterpret_cast<const uint2*>(p.bias + n);
    bv[0] = lo_bf16(braw.x); bv[1] = hi_bf16(braw.x); bv[2] = lo_bf16(braw.y); bv[3] = hi_bf16(braw.y);
  }
  float v[4] = {a.x * p.alpha + bv[0], a.y * p.alpha + bv[1], a.z * p.alpha + bv[2], a.w * p.alpha + bv[3]};
  const int64_t off = (int64_t)m * p.ldc + n;
  if (flags & kEpiAux)
    *reinterpret_cast<uint2*>(p.aux + off) = make_uint2(pack_bf16(v[0], v[1]), pack_bf16(v[2], v[3]));
  if (flags & kEpiGelu) {
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = gelu_tanh(v[q]);
  }
  if (flags & kEpiResid) {
    const uint2 rr = *reinterpret_cast<const uint2*>(p.res + off);
    v[0] += lo_bf16(rr.x); v[1] += hi_bf16(rr.x); v[2] += lo_bf16(rr.y); v[3] += hi_bf16(rr.y);
  }
  if (flags & kEpiOutF32) {
    float4* cp = reinterpret_cast<float4*>(reinterpret_cast<float*>(p.c) + off);
    if (flags & kEpiAccum) {
      const float4 o = *cp;
      v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
    }
    *cp = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    uint2* cp = reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(p.c) + off);
    if (flags & kEpiAccum) {
      const uint2 o = *cp;
      v[0] += lo_bf16(o.x); v[1] += hi_bf16(o.x); v[2] += lo_bf16(o.y); v[3] += hi_bf16(o.y);
    }
    *cp = make_uint2(pack_bf16(v[0], v[1]), pack_bf16(v[2], v[3]));
  }
}

int device_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  return cus;
}

// Tail plan of the ping-pong kernel: tiles beyond the last whole wave are split along K so the last wave
// has about one workgroup per CU. Only when the remainder covers at most half the chip and every slice
// keeps at least 4 K-tiles.
void pp_plan(int64_t M, int64_t N, int64_t K, int cus, int* full, int* split) {
  const int64_t T = ((M + 255) / 256) * ((N + 255) / 256);
  const int64_t nk = K / kBK;
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

}  // namespace

// Workspace (bytes) the ping-pong GEMM needs for its balanced tail (0: none).
PA_EXPORT int64_t pa_gemm_pp_ws_bytes(int64_t M, int64_t N, int64_t K) {
  int full, split;
  pp_plan(M, N, K, device_cus(), &full, &split);
  if (!split) return 0;
  const int64_t T = ((M + 255) / 256) * ((N + 255) / 256);
  return (T - full) * split * 65536 * 4;
}

namespace {
template <bool AK, bool BKM>
int launch4w(const GemmArgs& g, int grid, hipStream_t st) {
  constexpr int kLoop = 4 * 2 * 256 * 32 * 2, kEpi = 128 * kEpiRowStride * 4;
  constexpr int smem = kLoop > kEpi ? kLoop : kEpi;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm4w_kernel<AK, BKM>, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr_set = true;
  }
  hipLaunchKernelGGL((gemm4w_kernel<AK, BKM>), dim3(grid), dim3(256), smem, st, g);
  return (int)hipGetLastError();
}

// One 256x256-tile GEMM on kernel `kern` (1 8-wave ping-pong, 2 4-wave K32 ring) with the balanced tail when ws is given (pp_plan); g holds operands, sizes and epilogue fields.
int run_tile256(int kern, GemmArgs g, int a_kmajor, int b_kmajor, void* ws, hipStream_t st) {
  const int64_t M = g.M, N = g.N, K = g.K;
  if (K % kBK != 0 || N % 8 != 0 || g.lda % 8 != 0 || g.ldb % 8 != 0 || g.ldc % 4 != 0) return 1;
  if (!a_kmajor && M % 8 != 0) return 1;
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  g.c_split = M * g.ldc;
  int full, split;
  pp_plan(M, N, K, device_cus(), &full, &split);
  if (split && !ws) split = 0;
  g.tiles_m = (int)((M + 255) / 256);
  g.tiles_n = (int)((N + 255) / 256);
  const int T = g.tiles_m * g.tiles_n;
  g.full_tiles = split ? full : T;
  g.tail_split = split;
  g.tail_ws = (float*)ws;
  const int grid = split ? full + (T - full) * split : T;
  const int lay = (a_kmajor ? 0 : 2) + (b_kmajor ? 1 : 0);
  int rc;
  if (kern == 1) {
    rc = lay == 0 ? launch256<true, false>(g, 1, st, grid) : lay == 1 ? launch256<true, true>(g, 1, st, grid)
       : lay == 2 ? launch256<false, false>(g, 1, st, grid) : launch256<false, true>(g, 1, st, grid);
  } else {
    rc = lay == 0 ? launch4w<true, false>(g, grid, st) : lay == 1 ? launch4w<true, true>(g, grid, st)
       : lay == 2 ? launch4w<false, false>(g, grid, st) : launch4w<false, true>(g, grid, st);
  }
  if (rc || !split) return rc;
  hipLaunchKernelGGL(gemm_tail_reduce_k, dim3(T - full, 64), dim3(256), 0, st, g);
  return (int)hipGetLastError();
}

GemmArgs tile256_args(const void* a, const void* b, void* c, const void* bias, void* aux, int64_t M, int64_t N,
                      int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int flags, float alpha) {
  GemmArgs g{};
  g.a = (const uint16_t*)a; g.b = (const uint16_t*)b; g.c = c;
  g.bias = (const uint16_t*)bias; g.aux = (uint16_t*)aux;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.M = (int)M; g.N = (int)N; g.K = (int)K;
  g.flags = flags; g.alpha = alpha;
  return g;
}
}  // namespace

// Ping-pong 256x256 GEMM (same operands / flags as pa_gemm_bf16, no split-K) with the balanced tail;
// ws: pa_gemm_pp_ws_bytes(M, N, K) bytes (may be null when that is 0).
PA_EXPORT int pa_gemm_bf16_pp(const void* a, const void* b, void* c, const void* bias, void* aux, int64_t M, int64_t N,
                              int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int a_kmajor, int b_kmajor, int flags,
                              float alpha, void* ws, hipStream_t st) {
  return run_tile256(1, tile256_args(a, b, c, bias, aux, M, N, K, lda, ldb, ldc, flags, alpha), a_kmajor, b_kmajor,
                     ws, st);
}

// Split-K on the ping-pong kernel: every tile cut into `splits` K slices (the balanced-tail machinery with no
// whole tiles), fp32 256 x 256 partials in ws (tiles x splits x 256 KiB), summed with the epilogue by
// gemm_tail_reduce_k — for products with few output tiles and a long K (the weight gradients of convolutions over
// all pixels of a batch). Requires (K / 64) % splits == 0.
PA_EXPORT int64_t pa_gemm_pp_splitk_ws_bytes(int64_t M, int64_t N, int splits) {
  return ((M + 255) / 256) * ((N + 255) / 256) * (int64_t)splits * 65536 * 4;
}

PA_EXPORT int pa_gemm_bf16_pp_splitk(const void* a, const void* b, void* c, int64_t M, int64_t N, int64_t K,
                                     int64_t lda, int64_t ldb, int64_t ldc, int a_kmajor, int b_kmajor, int flags,
                                     float alpha, int splits, void* ws, hipStream_t st) {
  if (K % kBK != 0 || N % 8 != 0 || lda % 8 != 0 || ldb % 8 != 0 || ldc % 4 != 0 || splits < 1) return 1;
  if ((K / kBK) % splits != 0 || !ws || (flags & ~(kEpiOutF32 | kEpiAccum))) return 1;
  if (!a_kmajor && M % 8 != 0) return 1;
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  GemmArgs g{};
  g.a = (const uint16_t*)a; g.b = (const uint16_t*)b; g.c = c;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.M = (int)M; g.N = (int)N; g.K = (int)K;
  g.flags = flags; g.alpha = alpha;
  g.tiles_m = (int)((M + 255) / 256);
  g.tiles_n = (int)((N + 255) / 256);
  const int T = g.tiles_m * g.tiles_n;
  g.full_tiles = 0;
  g.tail_split = splits;
  g.tail_ws = (float*)ws;
  const int grid = T * splits;
  int rc;
  if (a_kmajor && !b_kmajor) rc = launch256<true, false>(g, 1, st, grid);
  else if (a_kmajor && b_kmajor) rc = launch256<true, true>(g, 1, st, grid);
  else if (!a_kmajor && !b_kmajor) rc = launch256<false, false>(g, 1, st, grid);
  else rc = launch256<false, true>(g, 1, st, grid);
  if (rc) return rc;
  hipLaunchKernelGGL(gemm_tail_reduce_k, dim3(T, 64), dim3(256), 0, st, g);
  return (int)hipGetLastError();
}

// Segmented operands on the ping-pong kernel (GemmArgs::nseg): seg = [nseg][5] int64 host array of
// {a_ptr, b_ptr, lda, ldb, end} per segment (end: K-tiles x 64 = K elements for seg_k = 1, columns for seg_k = 0),
// same operand layouts in every segment. K = total K (seg_k) or the A operand's K; N = total columns. a / b in
// the call are unused for the segmented operand. Workspace as pa_gemm_bf16_pp(M, N, K).
PA_EXPORT int pa_gemm_bf16_pp_segs(const int64_t* seg, int nseg, int seg_k, const void* a, const void* b, void* c,
                                   const void* bias, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
                                   int64_t ldc, int a_kmajor, int b_kmajor, int flags, float alpha, void* ws,
                                   hipStream_t st) {
  if (nseg < 1 || nseg > 4 || K % kBK != 0 || N % 8 != 0 || ldc % 4 != 0) return 1;
  if (!a_kmajor && M % 8 != 0) return 1;
  if (flags & (kEpiAux | kEpiStats)) return 1;
  if (M <= 0 || N <= 0) return 0;
  GemmArgs g{};
  g.a = (const uint16_t*)a; g.b = (const uint16_t*)b; g.c = c; g.bias = (const uint16_t*)bias;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.nseg = nseg; g.seg_k = seg_k;
  int64_t prev = 0;
  for (int s = 0; s < 4; ++s) {
    const int64_t* e = seg + 5 * (s < nseg ? s : nseg - 1);
    g.seg_a[s] = (const uint16_t*)e[0];
    g.seg_b[s] = (const uint16_t*)e[1];
    g.seg_lda[s] = e[2];
    g.seg_ldb[s] = e[3];
    if (s < nseg) {
      const int64_t end = e[4];
      if (end <= prev || e[2] % 8 != 0 || e[3] % 8 != 0) return 1;
      if (seg_k ? (end % kBK != 0) : (end % 128 != 0 && s + 1 < nseg)) return 1;
      g.seg_end[s] = (int)(seg_k ? end / kBK : end);
      prev = end;
    } else {
      g.seg_end[s] = g.seg_end[nseg - 1];
    }
  }
  if (seg_k ? prev != K : prev != N) return 1;
  if (!seg_k && (lda % 8 != 0)) return 1;
  if (seg_k && (flags & kEpiBias)) return 1;
  g.M = (int)M; g.N = (int)N; g.K = (int)K;
  g.flags = flags; g.alpha = alpha;
  g.c_split = M * ldc;
  int full, split;
  pp_plan(M, N, K, device_cus(), &full, &split);
  if (split && !ws) split = 0;
  g.tiles_m = (int)((M + 255) / 256);
  g.tiles_n = (int)((N + 255) / 256);
  const int T = g.tiles_m * g.tiles_n;
  g.full_tiles = split ? full : T;
  g.tail_split = split;
  g.tail_ws = (float*)ws;
  const int grid = split ? full + (T - full) * split : T;
  int rc;
  const int sg = nseg > 1 ? (seg_k ? 1 : 2) : 0;
  if (a_kmajor && !b_kmajor) rc = launch256<true, false>(g, 1, st, grid, sg);
  else if (a_kmajor && b_kmajor) rc = launch256<true, true>(g, 1, st, grid, sg);
  else if (!a_kmajor && !b_kmajor) rc = launch256<false, false>(g, 1, st, grid, sg);
  else rc = launch256<false, true>(g, 1, st, grid, sg);
  if (rc || !split) return rc;
  hipLaunchKernelGGL(gemm_tail_reduce_k, dim3(T - full, 64), dim3(256), 0, st, g);
  return (int)hipGetLastError();
}

// 4-wave 256x256 GEMM (gemm4w_kernel; same operands / flags / workspace as pa_gemm_bf16_pp).
PA_EXPORT int pa_gemm_bf16_4w(const void* a, const void* b, void* c, const void* bias, void* aux, int64_t M, int64_t N,
                              int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int a_kmajor, int b_kmajor, int flags,
                              float alpha, void* ws, hipStream_t st) {
  return run_tile256(2, tile256_args(a, b, c, bias, aux, M, N, K, lda, ldb, ldc, flags, alpha), a_kmajor, b_kmajor,
                     ws, st);
}

// Output projection with the residual add in its epilogue: C = a . b (+ bias) + res (bf16, [M][ldc]; may not alias
// C). Ping-pong kernel with the balanced tail (ws as pa_gemm_bf16_pp). Replaces the separate elementwise add after
// the attention / MLP output projections of a pre-norm decoder layer (one read of the residual instead of a
// read of both summands and a write).
PA_EXPORT int pa_gemm_bf16_res(const void* a, const void* b, void* c, const void* bias, const void* res, int64_t M,
                               int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int a_kmajor, int b_kmajor,
                               void* ws, hipStream_t st) {
  if (!res || res == c) return 1;
  GemmArgs g = tile256_args(a, b, c, bias, nullptr, M, N, K, lda, ldb, ldc, (bias ? kEpiBias : 0) | kEpiResid, 1.f);
  g.res = (const uint16_t*)res;
  return run_tile256(1, g, a_kmajor, b_kmajor, ws, st);
}

// Data gradient of the linear after a tanh-GELU, fused with the GELU backward and the first linear's bias gradient
// (reference fusion/gpu/fused_feedforward_grad: the dropout/activation backward runs as its own pass there):
// dh = (a . b) * gelu'(pre) (bf16, [M][ldc]) and colsum[tiles_m][N] = per-256-row-tile column sums of dh (fp32,
// folded into the bias gradient by pa_fold_partials with nparts = tiles_m). kern: as run_tile256; no balanced tail
// (the column sums are per whole tile). pre: the forward's stored pre-activation (x . W1 + b1), same layout as dh.
PA_EXPORT int pa_gemm_bf16_dgelu(const void* a, const void* b, void* dh, const void* pre, float* colsum, int64_t M,
                                 int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int a_kmajor,
                                 int b_kmajor, int kern, hipStream_t st) {
  if (!pre || !colsum || kern < 1 || kern > 2) return 1;
  GemmArgs g = tile256_args(a, b, dh, nullptr, const_cast<void*>(pre), M, N, K, lda, ldb, ldc,
                            kEpiGeluBwd | kEpiColSum, 1.f);
  g.stats = colsum;
  return run_tile256(kern, g, a_kmajor, b_kmajor, nullptr, st);
}

// Diagnostic ablations of gemm4w_kernel (A K-major, B MN-major, no tail): timing only.
PA_EXPORT int pa_gemm_bf16_4w_abl(const void* a, const void* b, void* c, int64_t M, int64_t N, int64_t K, int abl,
                                  hipStream_t st) {
  if (K % kBK || N % 256 || M % 256) return 1;
  GemmArgs g{};
  g.a = (const uint16_t*)a; g.b = (const uint16_t*)b; g.c = c;
  g.lda = K; g.ldb = N; g.ldc = N; g.M = (int)M; g.N = (int)N; g.K = (int)K; g.alpha = 1.f;
  g.tiles_m = (int)(M / 256); g.tiles_n = (int)(N / 256);
  g.full_tiles = g.tiles_m * g.tiles_n;
  constexpr int smem = 128 * kEpiRowStride * 4;
#define PA_G4A(V)                                                                                              \
  do {                                                                                                         \
    (void)hipFuncSetAttribute((const void*)gemm4w_kernel<true, false, V>,                                      \
                              hipFuncAttributeMaxDynamicSharedMemorySize, smem);                               \
    hipLaunchKernelGGL((gemm4w_kernel<true, false, V>), dim3(g.full_tiles), dim3(256), smem, st, g);           \
  } while (0)
  if (abl == 1) PA_G4A(1);
  else if (abl == 2) PA_G4A(2);
  else if (abl == 3) PA_G4A(3);
  else if (abl == 5) PA_G4A(5);
  else if (abl >= 6 && abl <= 8) {  // operand footprint ablations: 6 both, 7 B, 8 A read from one L2-resident row
    if (abl != 7) g.lda = 0;
    if (abl != 8) g.ldb = 0;
    PA_G4A(0);
  }
  else if (abl == 4) {
    (void)hipFuncSetAttribute((const void*)gemm4w_kernel<true, false, 0, 5>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              5 * 32768);
    hipLaunchKernelGGL((gemm4w_kernel<true, false, 0, 5>), dim3(g.full_tiles), dim3(256), 5 * 32768, st, g);
  } else PA_G4A(0);
#undef PA_G4A
  return (int)hipGetLastError();
}

// C = epi(alpha * A.B). A: [M][K] (a_kmajor) or [K][M]; B: [N][K] (b_kmajor) or [K][N].
// Requirements (checked by the Python wrapper too): K % 64 == 0, 16-byte aligned rows
// (lda, ldb % 8 == 0), M % 8 == 0 if A is MN-major, N % 8 == 0, ldc % 4 == 0.
PA_EXPORT int pa_gemm_bf16(const void* a, const void* b, void* c, const void* bias, void* aux, int64_t M, int64_t N,
                           int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int a_kmajor, int b_kmajor, int flags,
                           float alpha, int bn, int splits, hipStream_t st) {
  // split-K (splits > 1): K is split into `splits` slices of K / splits elements; slice s writes fp32
  // partials to c + s * M * ldc (no bias / activation / accumulate); the caller reduces the slabs.
  if (splits < 1) splits = 1;
  if (K % splits != 0) return 1;
  const int64_t Kc = K / splits;
  if (Kc % kBK != 0 || N % 8 != 0 || lda % 8 != 0 || ldb % 8 != 0 || ldc % 4 != 0) return 1;
  if (!a_kmajor && M % 8 != 0) return 1;
  if (splits > 1 && (flags & (kEpiBias | kEpiGelu | kEpiAux | kEpiAccum))) return 1;
  if (splits > 1 && !(flags & kEpiOutF32)) return 1;
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  GemmArgs g{};
  g.a = (const uint16_t*)a; g.b = (const uint16_t*)b; g.c = c;
  g.bias = (const uint16_t*)bias; g.aux = (uint16_t*)aux;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.M = (int)M; g.N = (int)N; g.K = (int)Kc;
  g.flags = flags; g.alpha = alpha;
  g.c_split = M * ldc;
  // bn: 160 = three-stage 256x160 kernel; 256 / 128 = two-stage kernel with 256x256 / 256x128 tiles;
  // 1 = 4-phase ping-pong 256x256 kernel
  if (bn == 160) return dispatch_layout<160>(g, a_kmajor, b_kmajor, splits, st);
  if (bn == 128) return dispatch_layout<128>(g, a_kmajor, b_kmajor, splits, st);
  if (bn == 1) return dispatch_layout<0>(g, a_kmajor, b_kmajor, splits, st);
  if (bn == 4) return dispatch_layout<4>(g, a_kmajor, b_kmajor, splits, st);
  return dispatch_layout<256>(g, a_kmajor, b_kmajor, splits, st);
}

// Implicit-GEMM NDHWC 3-D convolution forward: out[N*Do*Ho*Wo, Cout] = im2col3d(x) . W^T (+ bias), x [N, D, H, W, C]
// bf16 (C % 64 == 0), w [Cout, KD, KH, KW, C] (channels-last filter); every 64-deep K tile is one (kd, kh, kw) tap.
// Same 256x160 kernel as the 2-D forward (a 2-D convolution is the D = KD = 1 case).
PA_EXPORT int pa_conv3d_ndhwc_fwd(const void* x, const void* w, const void* bias, void* out, const void* zero, int N,
                                  int D, int H, int W, int C, int Cout, int KD, int KH, int KW, int stride, int pad_d,
                                  int pad_h, int pad_w, int dil, int Do, int Ho, int Wo, hipStream_t st) {
  if (C % kBK != 0 || Cout % 8 != 0 || N <= 0) return 1;
  GemmArgs g{};
  g.a = (const uint16_t*)x; g.b = (const uint16_t*)w; g.c = out; g.bias = (const uint16_t*)bias;
  g.M = N * Do * Ho * Wo; g.N = Cout; g.K = KD * KH * KW * C;
  g.lda = C; g.ldb = (int64_t)KD * KH * KW * C; g.ldc = Cout;
  g.flags = bias ? kEpiBias : 0; g.alpha = 1.f;
  g.zero = (const uint16_t*)zero;
  g.cD = D; g.cDo = Do; g.cKHW = KH * KW; g.cPadD = pad_d;
  g.cH = H; g.cW = W; g.cC = C; g.cHo = Ho; g.cWo = Wo; g.cKW = KW; g.cStride = stride; g.cPadH = pad_h;
  g.cPadW = pad_w; g.cDil = dil;
  return launch3s<true, true, true>(g, 1, st);
}

// Statistics chunks of a kEpiStats launch (stats: [2][chunks][N] fp32): 256-row tiles x waves along M
// (4 for the 256x160 kernel, 2 for the two-stage kernels).
PA_EXPORT int pa_gemm_stats_chunks(int64_t M, int bn) { return (int)((M + kBM - 1) / kBM) * (bn == 160 ? 4 : 2); }

// pa_gemm_bf16 (bf16 output, no split) that also writes the per-column batch-norm partials of the stored C
// (sum, sum of squares of the bf16-rounded values) to stats. bn: 160, 256, 128 or 4 (two-stage 4-wave).
PA_EXPORT int pa_gemm_bf16_stats(const void* a, const void* b, void* c, const void* bias, int64_t M, int64_t N,
                                 int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int a_kmajor, int b_kmajor,
                                 int flags, int bn, float* stats, hipStream_t st) {
  if (K % kBK != 0 || N % 8 != 0 || lda % 8 != 0 || ldb % 8 != 0 || ldc % 4 != 0 || !stats) return 1;
  if (!a_kmajor && M % 8 != 0) return 1;
  if (flags & (kEpiOutF32 | kEpiGelu | kEpiAux)) return 1;
  if (bn != 160 && bn != 256 && bn != 128 && bn != 4) return 1;
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  GemmArgs g{};
  g.a = (const uint16_t*)a; g.b = (const uint16_t*)b; g.c = c;
  g.bias = (const uint16_t*)bias;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.M = (int)M; g.N = (int)N; g.K = (int)K;
  g.flags = flags | kEpiStats; g.alpha = 1.f;
  g.c_split = M * ldc;
  g.stats = stats;
  if (bn == 160) return dispatch_layout<160>(g, a_kmajor, b_kmajor, 1, st);
  if (bn == 128) return dispatch_layout<128>(g, a_kmajor, b_kmajor, 1, st);
  if (bn == 4) return dispatch_layout<4>(g, a_kmajor, b_kmajor, 1, st);
  return dispatch_layout<256>(g, a_kmajor, b_kmajor, 1, st);
}

// pa_gemm_bf16_stats in BN-backward form: C is the gradient of a relu'd BN's output (a 1x1 convolution's data
// gradient); stats receives [sum dyp, sum dyp * (x - mean)] per column with x / ss / mean the BN's forward input,
// scale-shift and batch mean (bn.hip pa_bn_bwd_nhwc_pre consumes them).
PA_EXPORT int pa_gemm_bf16_bnbwd(const void* a, const void* b, void* c, int64_t M, int64_t N, int64_t K, int64_t lda,
                                 int64_t ldb, int64_t ldc, int a_kmajor, int b_kmajor, int bn, const void* bn_x,
                                 const float* bn_ss, const float* bn_mean, float* stats, hipStream_t st) {
  if (K % kBK != 0 || N % 8 != 0 || lda % 8 != 0 || ldb % 8 != 0 || ldc % 4 != 0 || !stats) return 1;
  if (!bn_x || !bn_ss || !bn_mean) return 1;
  if (!a_kmajor && M % 8 != 0) return 1;
  if (bn != 160 && bn != 256 && bn != 128 && bn != 4) return 1;
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  GemmArgs g{};
  g.a = (const uint16_t*)a; g.b = (const uint16_t*)b; g.c = c;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.M = (int)M; g.N = (int)N; g.K = (int)K;
  g.flags = kEpiStats | kEpiStatsBwd; g.alpha = 1.f;
  g.c_split = M * ldc;
  g.stats = stats;
  g.bn_x = (const uint16_t*)bn_x; g.bn_ss = bn_ss; g.bn_mean = bn_mean;
  if (bn == 160) return dispatch_layout<160>(g, a_kmajor, b_kmajor, 1, st);
  if (bn == 128) return dispatch_layout<128>(g, a_kmajor, b_kmajor, 1, st);
  if (bn == 4) return dispatch_layout<4>(g, a_kmajor, b_kmajor, 1, st);
  return dispatch_layout<256>(g, a_kmajor, b_kmajor, 1, st);
}

// Implicit-GEMM NHWC convolution forward: out[N*Ho*Wo, Cout] = im2col(x) . W^T (+ bias), with
// x [N, H, W, C] bf16 (C % 64 == 0), w [Cout, KH, KW, C] bf16 (channels-last filter), out NHWC bf16.
// Runs on the 3-stage 256x160 kernel; `zero` is a >= 128-byte zeroed device buffer for padding taps.
PA_EXPORT int pa_conv2d_nhwc_fwd(const void* x, const void* w, const void* bias, void* out, const void* zero, int N,
                                 int H, int W, int C, int Cout, int KH, int KW, int stride, int pad_h, int pad_w,
                                 int dil, int Ho, int Wo, hipStream_t st) {
  if (C % kBK != 0 || Cout % 8 != 0 || N <= 0) return 1;
  GemmArgs g{};
  g.a = (const uint16_t*)x; g.b = (const uint16_t*)w; g.c = out; g.bias = (const uint16_t*)bias;
  g.M = N * Ho * Wo; g.N = Cout; g.K = KH * KW * C;
  g.lda = C; g.ldb = (int64_t)KH * KW * C; g.ldc = Cout;
  g.flags = bias ? kEpiBias : 0; g.alpha = 1.f;
  g.zero = (const uint16_t*)zero;
  g.cD = 1; g.cDo = 1; g.cKHW = KH * KW; g.cPadD = 0;
  g.cH = H; g.cW = W; g.cC = C; g.cHo = Ho; g.cWo = Wo; g.cKW = KW; g.cStride = stride; g.cPadH = pad_h;
  g.cPadW = pad_w; g.cDil = dil;
  return launch3s<true, true, true>(g, 1, st);
}

// pa_conv2d_nhwc_fwd that also writes the batch-norm partials of the output (stats: [2][chunks][Cout],
// chunks = pa_gemm_stats_chunks(N * Ho * Wo, 160)) for the following BN layer (conv -> BN fusion).
PA_EXPORT int pa_conv2d_nhwc_fwd_stats(const void* x, const void* w, const void* bias, void* out, const void* zero,
                                       int N, int H, int W, int C, int Cout, int KH, int KW, int stride, int pad_h,
                                       int pad_w, int dil, int Ho, int Wo, float* stats, hipStream_t st) {
  if (C % kBK != 0 || Cout % 8 != 0 || N <= 0 || !stats) return 1;
  GemmArgs g{};
  g.a = (const uint16_t*)x; g.b = (const uint16_t*)w; g.c = out; g.bias = (const uint16_t*)bias;
  g.M = N * Ho * Wo; g.N = Cout; g.K = KH * KW * C;
  g.lda = C; g.ldb = (int64_t)KH * KW * C; g.ldc = Cout;
  g.flags = (bias ? kEpiBias : 0) | kEpiStats; g.alpha = 1.f;
  g.stats = stats;
  g.zero = (const uint16_t*)zero;
  g.cD = 1; g.cDo = 1; g.cKHW = KH * KW; g.cPadD = 0;
  g.cH = H; g.cW = W; g.cC = C; g.cHo = Ho; g.cWo = Wo; g.cKW = KW; g.cStride = stride; g.cPadH = pad_h;
  g.cPadW = pad_w; g.cDil = dil;
  return launch3s<true, true, true>(g, 1, st);
}

// pa_conv2d_nhwc_fwd in BN-backward form (the stride-1 data gradient of a KxK convolution, run as the convolution
// of dY with the flipped filter): out is the gradient of a relu'd BN's output, stats as pa_gemm_bf16_bnbwd.
PA_EXPORT int pa_conv2d_nhwc_fwd_bnbwd(const void* x, const void* w, void* out, const void* zero, int N, int H, int W,
                                       int C, int Cout, int KH, int KW, int stride, int pad_h, int pad_w, int dil,
                                       int Ho, int Wo, const void* bn_x, const float* bn_ss, const float* bn_mean,
                                       float* stats, hipStream_t st) {
  if (C % kBK != 0 || Cout % 8 != 0 || N <= 0 || !stats || !bn_x || !bn_ss || !bn_mean) return 1;
  GemmArgs g{};
  g.a = (const uint16_t*)x; g.b = (const uint16_t*)w; g.c = out;
  g.M = N * Ho * Wo; g.N = Cout; g.K = KH * KW * C;
  g.lda = C; g.ldb = (int64_t)KH * KW * C; g.ldc = Cout;
  g.flags = kEpiStats | kEpiStatsBwd; g.alpha = 1.f;
  g.stats = stats;
  g.bn_x = (const uint16_t*)bn_x; g.bn_ss = bn_ss; g.bn_mean = bn_mean;
  g.zero = (const uint16_t*)zero;
  g.cD = 1; g.cDo = 1; g.cKHW = KH * KW; g.cPadD = 0;
  g.cH = H; g.cW = W; g.cC = C; g.cHo = Ho; g.cWo = Wo; g.cKW = KW; g.cStride = stride; g.cPadH = pad_h;
  g.cPadW = pad_w; g.cDil = dil;
  return launch3s<true, true, true>(g, 1, st);
}

// Weight gradient of a KxK NHWC convolution, transposed: ws[splits][KH*KW*C][Cout] fp32 slabs (summed by the
// caller) of dW^T = im2col(x)^T . dy, the im2col rows gathered on the fly (stage_convw). x [N, H, W, C],
// dy [N, Ho, Wo, Cout] bf16; C % 8 == 0, Cout % 8 == 0, (N*Ho*Wo) % (64 * splits) == 0.
PA_EXPORT int pa_conv2d_nhwc_wgrad(const void* x, const void* dy, float* ws, const void* zero, int N, int H, int W,
                                   int C, int Cout, int KH, int KW, int stride, int pad_h, int pad_w, int dil, int Ho,
                                   int Wo, int splits, int bn, hipStream_t st) {
  const int64_t P = (int64_t)N * Ho * Wo;
  if (C % 8 || Cout % 8 || splits < 1 || P % (64 * splits) || P / splits > 0x7fffffff) return 1;
  if (bn != 64 && bn != 128 && bn != 256) return 2;
  GemmArgs g{};
  g.a = (const uint16_t*)x; g.b = (const uint16_t*)dy; g.c = ws;
  g.lda = 0; g.ldb = Cout; g.ldc = Cout;
  g.M = KH * KW * C; g.N = Cout; g.K = (int)(P / splits);
  g.flags = kEpiOutF32; g.alpha = 1.f;
  g.c_split = (int64_t)g.M * Cout;
  g.zero = (const uint16_t*)zero;
  g.cD = 1; g.cDo = 1; g.cKHW = KH * KW; g.cPadD = 0;
  g.cH = H; g.cW = W; g.cC = C; g.cHo = Ho; g.cWo = Wo; g.cKW = KW; g.cStride = stride; g.cPadH = pad_h;
  g.cPadW = pad_w; g.cDil = dil;
  g.tiles_m = (g.M + kBM - 1) / kBM;
  g.tiles_n = (g.N + bn - 1) / bn;
  const int smem = 2 * (kBM + bn) * kBK * 2;
  static bool attr_set[3] = {false, false, false};
#define PA_WG(BNV, I)                                                                                           \
  do {                                                                                                          \
    if (!attr_set[I]) {                                                                                         \
      (void)hipFuncSetAttribute((const void*)gemm_bf16_kernel<BNV, false, false, 8, true>,                      \
                                hipFuncAttributeMaxDynamicSharedMemorySize, smem);                              \
      attr_set[I] = true;                                                                                       \
    }                                                                                                           \
    hipLaunchKernelGGL((gemm_bf16_kernel<BNV, false, false, 8, true>), dim3(g.tiles_m * g.tiles_n, splits),     \
                       dim3(512), smem, st, g);                                                                 \
  } while (0)
  if (bn == 256) PA_WG(256, 1);
  else if (bn == 64) PA_WG(64, 2);
  else PA_WG(128, 0);
#undef PA_WG
  return (int)hipGetLastError();
}

// Decode-shape GEMM: c[M, N] (bf16, row stride ldc) = a[M, K] (K-major) . b[K, N] (N-major) (+ bias),
// M <= 64, K % (64 * splits) == 0, N % 8 == 0; `ws` = fp32 workspace of splits * M * N floats.
PA_EXPORT int pa_gemm_small_m(const void* a, int64_t lda, const void* b, int64_t ldb, void* c, int64_t ldc,
                              const void* bias, float* ws, int M, int N, int K, int splits, int stages, hipStream_t st) {
  if (M < 1 || M > kSmBM || N % 8 != 0 || splits < 1 || K % (kBK * splits) != 0 || lda % 8 || ldb % 8) return 1;
  if (stages != 3 && stages != 4) return 2;
  // 4 stages: 96 KiB LDS, one workgroup per CU; 3 stages: 72 KiB, two per CU
  const int smem = stages * (kSmBM + kSmBN) * kBK * 2;
  static bool attr_set[2] = {false, false};
  const dim3 grid((N + kSmBN - 1) / kSmBN, splits), block(kSmNW * 64);
#define PA_SMM(S)                                                                                                \
  do {                                                                                                          \
    if (!attr_set[S - 3]) {                                                                                     \
      (void)hipFuncSetAttribute((const void*)gemm_small_m_kernel<S>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                smem);                                                                          \
      attr_set[S - 3] = true;                                                                                   \
    }                                                                                                           \
    hipLaunchKernelGGL(gemm_small_m_kernel<S>, grid, block, smem, st, (const uint16_t*)a, lda, (const uint16_t*)b, \
                       ldb, ws, M, N, K / splits, (const uint16_t*)bias, (uint16_t*)c, ldc);                    \
  } while (0)
  if (stages == 3) PA_SMM(3);
  else PA_SMM(4);
#undef PA_SMM
  if (splits == 1) return (int)hipGetLastError();
  const int64_t n4 = (int64_t)M * N / 4;
  hipLaunchKernelGGL(gemm_small_m_reduce_k, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, ws,
                     (const uint16_t*)bias, (uint16_t*)c, ldc, M, N, splits);
  return (int)hipGetLastError();
}

namespace {
// Slab sum with the split dimension spread over the block: 16 lanes of float4 columns x 16 split groups; each
// thread sums every 16th slab of its 4 columns (several loads in flight), the 16 groups fold through LDS. A
// weight gradient has few outputs and many slabs (64 x 64 x 128 splits), which a one-thread-per-output loop
// walks serially.
__global__ __launch_bounds__(256) void slab_reduce_k(const float* __restrict__ ws, uint16_t* __restrict__ c,
                                                     int64_t ldc, int64_t M, int64_t N, int splits) {
  __shared__ float4 red[16][16];
  const int cl = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int64_t i4 = ((int64_t)blockIdx.x * 16 + cl) * 4;
  const int64_t MN = M * N;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i4 < MN) {
    int s = g;
    for (; s + 48 < splits; s += 64) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(ws + (int64_t)(s + 16 * u) * MN + i4);
#pragma unroll
      for (int u = 0; u < 4; ++u) { acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w; }
    }
    for (; s < splits; s += 16) {
      const float4 v = *reinterpret_cast<const float4*>(ws + (int64_t)s * MN + i4);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  red[g][cl] = acc;
  __syncthreads();
  if (g == 0 && i4 < MN) {
    float4 t = red[0][cl];
#pragma unroll
    for (int q = 1; q < 16; ++q) { t.x += red[q][cl].x; t.y += red[q][cl].y; t.z += red[q][cl].z; t.w += red[q][cl].w; }
    const int64_t m = i4 / N, n = i4 % N;
    *reinterpret_cast<uint2*>(c + m * ldc + n) = make_uint2(pack_bf16(t.x, t.y), pack_bf16(t.z, t.w));
  }
}
}  // namespace

// Sum of `splits` fp32 slabs [splits][M][N] (split-K partials) into bf16 C [M][ldc] in one pass (the weight
// gradients of convolutions: replaces a separate reduction and cast). N % 4 == 0.
PA_EXPORT int pa_slab_reduce_bf16(const float* ws, void* c, int64_t ldc, int64_t M, int64_t N, int splits,
                                  hipStream_t st) {
  if (N % 4 != 0 || ldc % 4 != 0 || splits < 1 || M <= 0) return 1;
  const int64_t n4 = M * N / 4;
  hipLaunchKernelGGL(slab_reduce_k, dim3((unsigned)((n4 + 15) / 16)), dim3(256), 0, st, ws, (uint16_t*)c, ldc, M, N,
                     splits);
  return (int)hipGetLastError();
}
