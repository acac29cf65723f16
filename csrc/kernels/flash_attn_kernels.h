// Flash attention forward + backward for gfx950 (CDNA4), bf16 / fp16 in, fp32 accumulate.
// Reference behaviour: paddle/phi/kernels/gpu/flash_attn_kernel.cu / flash_attn_grad_kernel.cu
// (layout [batch, seq, heads, head_dim], causal = bottom-right aligned, GQA, LSE output, dropout,
// variable-length batches by cu_seqlens), python/paddle/nn/functional/flash_attention.py:1145
// (scaled_dot_product_attention with attn_mask) and :1306 (flashmask_attention row bounds).
//
// MFMA: v_mfma_f32_32x32x16_{bf16,f16} (lane l: r = l&31, h = l>>5;
//   A[row r][k 8h+j], B[k 8h+j][col r], D[row (i&3)+8(i>>2)+4h][col r]).
//
// Forward (per workgroup: 4 waves x 32 queries = 128-query block; K/V tiles of 64 keys in LDS):
//   S^T = K Q^T        -> the query is the MFMA column, so each lane owns one query and the row
//                         max / sum are in-lane (+ one xor-32 exchange), no LDS for P;
//   O^T += V^T P^T     -> the S^T accumulator is re-used directly as the B operand (packed),
//                         V^T comes from ds_read_b64_tr_b16 transposed LDS reads; O^T keeps the
//                         query on the lane, so the online-softmax rescale is per lane.
//   K/V tiles go global -> LDS by global_load_lds in two stages (tile t+1 in flight while t computes);
//   the rescale of O is deferred until a tile's max exceeds the running reference by 2^8.
// Backward (per workgroup: NW waves x 32 keys; loop over 32-query blocks and, for GQA, over the query
//   heads that share this KV head, so dK / dV are summed per KV head in registers):
//   S = Q K^T, P = exp(S - LSE), dP = dO V^T, dS = P (dP - delta);
//   dV^T += dO^T P and dK^T += Q^T dS with P / dS as B operands (no lane movement),
//   dQ += dS K via a dS^T tile in LDS, accumulated into fp32 with global atomics.
//
// Optional per-element terms, identical in both passes:
//   * dense mask [B|1, H|1, Sq, Sk]: bool (False = masked) or additive (bf16 / fp32, added to scale*QK^T);
//   * flashmask row bounds [B|1, H|1, Sk, 1|2|4] int32 (LTS[, LTE | UTE][, UTS, UTE]) per key column;
//   * dropout on P with a counter-based hash of (seed, batch*head, query, key): the backward regenerates
//     the same keep mask; P's row sum (softmax normaliser) is taken before dropout.
//   * varlen: cu_seqlens_q / _k [B+1] on the device; sequence b occupies rows cu[b]..cu[b+1] of packed
//     [total, H, D] tensors; LSE / delta are [H, total_q].
#pragma once
#include "common.h"

using namespace pa;

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_t;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

namespace pa_fa {

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

union Frag {
  bf16x8_t v;
  f16x8_t f;
  uint4 u;
  s16x4 h[2];
};

template <bool F16>
__device__ __forceinline__ f32x16 mfma32(const Frag& a, const Frag& b, f32x16 c) {
  if constexpr (F16) return __builtin_amdgcn_mfma_f32_32x32x16_f16(a.f, b.f, c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.v, b.v, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

template <bool F16>
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  if constexpr (F16) return pack_f16(a, b);
  else return pack_bf16(a, b);
}

template <bool F16>
__device__ __forceinline__ Frag pack8(const float* f) {
  Frag x;
  x.u.x = pack2<F16>(f[0], f[1]);
  x.u.y = pack2<F16>(f[2], f[3]);
  x.u.z = pack2<F16>(f[4], f[5]);
  x.u.w = pack2<F16>(f[6], f[7]);
  return x;
}

template <bool F16>
__device__ __forceinline__ float half_lo(uint32_t w) {
  if constexpr (F16) return lo_f16(w);
  else return lo_bf16(w);
}
template <bool F16>
__device__ __forceinline__ float half_hi(uint32_t w) {
  if constexpr (F16) return hi_f16(w);
  else return hi_bf16(w);
}

// LDS byte offset of 16-byte chunk `ch` of row `row` in a [rows][NCH*8] 16-bit image that serves
// both ds_read_b128 row reads and ds_read_b64_tr_b16 transposed reads without bank conflicts.
template <int NCH>
__device__ __forceinline__ int img_off(int row, int ch) {
  int sw;
  if (NCH >= 16) sw = ((row & 3) << 2) | ((row >> 2) & 3);
  else if (NCH == 8) sw = ((row & 3) << 1) | ((row >> 2) & 1);
  else sw = (row & 3);
  return row * (NCH * 16) + 16 * (ch ^ (sw & (NCH - 1)));
}

// Workgroup barrier that orders LDS only: waits for this wave's LDS ops (lgkmcnt) but leaves global
// memory ops in flight.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Global loads the compiler does not track: the caller retires them with an explicit counted vmcnt.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4 gload16_async(const void* p) {
  u32x4 r;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return r;
}
__device__ __forceinline__ uint2 gload8_async(const void* p) {
  uint2 r;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return r;
}
__device__ __forceinline__ uint32_t gload4_async(const void* p) {
  uint32_t r;
  asm volatile("global_load_dword %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return r;
}
__device__ __forceinline__ uint32_t gload2_async(const void* p) {
  uint32_t r;
  asm volatile("global_load_ushort %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return r;
}
__device__ __forceinline__ uint32_t gload1_async(const void* p) {
  uint32_t r;
  asm volatile("global_load_ubyte %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return r;
}

__device__ __forceinline__ uint4 lds_b128(const char* smem, int off) {
  return *reinterpret_cast<const uint4*>(smem + off);
}

__device__ __forceinline__ s16x4 lds_tr(const char* smem, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(reinterpret_cast<uintptr_t>(smem + off)));
}

__device__ __forceinline__ void glds16_fa(const void* g, const char* lds) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uintptr_t>(lds));
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m0) : "memory", "m0");
}

__device__ __forceinline__ void glds4_fa(const void* g, const char* lds) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uintptr_t>(lds));
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(g), "s"(m0) : "memory", "m0");
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// 1-D grid of nb * BH workgroups -> (head bh, block rank). Dispatch is round-robin over the 8 XCDs
// (workgroup id mod 8). With grp > 0 (BH % 8 == 0): XCD x owns heads x, x+8, ...; it walks them in groups
// of `grp` heads, and inside a group rank-major (rank 0 = heaviest block under the causal mask first),
// head-minor. So every XCD gets the same mix of block sizes, the heavy blocks go first, and the
// workgroups in flight on one XCD touch only ~grp heads' K/V (L2 reuse).
__device__ __forceinline__ void block_map(int L, int BH, int nb, int grp, int& bh, int& rank) {
  if (grp > 0) {
    const int xcd = L & 7, i = L >> 3;
    const int hpx = BH >> 3;
    const int gi = i / (grp * nb);
    const int g_eff = min(grp, hpx - gi * grp);
    const int j = i - gi * grp * nb;
    rank = j / g_eff;
    bh = xcd + 8 * (gi * grp + j % g_eff);
  } else {
    bh = L % BH;
    rank = L / BH;
  }
}

// ---- dropout: Philox-style 2x32 rounds keyed by the seed; one 32-bit word per (query, key pair),
// the low half decides the even key and the high half the odd key (keep if < keep16).
__device__ __forceinline__ uint32_t drop_hash(uint32_t s0, uint32_t s1, uint32_t a, uint32_t b) {
  uint32_t x = a, y = b, k = s0;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint32_t lo = x * 0xD256D193u;
    const uint32_t hi = __umulhi(x, 0xD256D193u);
    x = hi ^ k ^ y;
    y = lo;
    k += 0x9E3779B9u ^ s1;
  }
  return x ^ y;
}
__device__ __forceinline__ bool drop_keep(uint32_t word, int key, uint32_t keep16) {
  return ((word >> ((key & 1) * 16)) & 0xFFFFu) < keep16;
}

// mask kinds
enum MaskKind : int { kMaskNone = 0, kMaskBool = 1, kMaskBF16 = 2, kMaskF32 = 3 };

struct FwdArgs {
  const uint16_t* q; const uint16_t* k; const uint16_t* v; uint16_t* o; float* lse;
  int64_t qs[3], ks[3], vs[3], os[3];  // strides (batch, seq, head) in elements
  int B, Sq, Sk, H, Hk;                // Sq / Sk: max sequence lengths when varlen
  float scale_log2, inv_scale;
  int causal;
  int grp;  // heads per dispatch group (block_map)
  const int* cu_q; const int* cu_k;
  const void* mask; int mask_kind; int64_t ms[3];   // mask strides (b, h, q) in elements, key stride 1
  const int* fm; int fm_cols; int64_t fms[2];       // flashmask (b, h) strides in elements
  const int* fm_stats; int64_t fmst[2];              // per 64-key tile bound extrema (b, h strides in tiles)
  int dropout; uint32_t keep16; float rkeep; uint32_t seed0, seed1;
  int64_t lse_s[2];                                  // lse strides (b, h); row index = q_start + q
};

// flashmask: masked iff q in [lo0, lo1) or q in [up0, up1)
struct FmBounds {
  int lo0, lo1, up0, up1;
};
__device__ __forceinline__ FmBounds fm_canon(const int* v, int cols, int causal) {
  FmBounds b;
  b.lo0 = v[0];
  b.lo1 = 0x7fffffff;
  b.up0 = 0;
  b.up1 = 0;
  if (cols == 2) {
    if (causal) b.lo1 = v[1];
    else b.up1 = v[1];
  } else if (cols == 4) {
    b.lo1 = v[1];
    b.up0 = v[2];
    b.up1 = v[3];
  }
  return b;
}
__device__ __forceinline__ bool fm_masked(const FmBounds& b, int q) {
  return (q >= b.lo0 && q < b.lo1) || (q >= b.up0 && q < b.up1);
}

// Extrema of the canonical bounds over each 64-key tile: {min lo0, max lo0, min lo1, max lo1, min up0, max up0,
// min up1, max up1}; one wave per (b, h, tile). Lets the attention kernels skip tiles that are masked for every
// row of a block and drop the per-element test on tiles no bound touches.
static __global__ __launch_bounds__(64) void fa_fm_tile_stats(const int* __restrict__ fm, int cols, int causal, int Sk,
                                                       int ntiles, int64_t fm_sb, int64_t fm_sh, int Hm,
                                                       int* __restrict__ stats) {
  const int tile = blockIdx.x % ntiles, bh = blockIdx.x / ntiles;
  const int b = bh / Hm, h = bh % Hm;
  const int key = tile * 64 + threadIdx.x;
  int v[8];
  if (key < Sk) {
    const FmBounds fb = fm_canon(fm + b * fm_sb + h * fm_sh + (int64_t)key * cols, cols, causal);
    v[0] = v[1] = fb.lo0; v[2] = v[3] = fb.lo1; v[4] = v[5] = fb.up0; v[6] = v[7] = fb.up1;
  } else {
    for (int i = 0; i < 8; i += 2) { v[i] = 0x7fffffff; v[i + 1] = -0x7fffffff; }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
      v[i] = min(v[i], __shfl_xor(v[i], off, 64));
      v[i + 1] = max(v[i + 1], __shfl_xor(v[i + 1], off, 64));
    }
  if (threadIdx.x < 8) stats[(int64_t)blockIdx.x * 8 + threadIdx.x] = v[threadIdx.x];
}

// rows [q_lo, q_hi] against a tile's extrema: 2 = masked for every (row, key), 0 = no bound touches any row,
// 1 = test per element
__device__ __forceinline__ int fm_tile_class(const int* st, int q_lo, int q_hi) {
  const bool dead = (q_lo >= st[1] && q_hi < st[2]) || (q_lo >= st[5] && q_hi < st[6]);
  if (dead) return 2;
  const bool clean = (q_hi < st[0] || q_lo >= st[3]) && (q_hi < st[4] || q_lo >= st[7]);
  return clean ? 0 : 1;
}

// ------------------------------------------------------------------------------------- forward
// Same math and lane layout for every variant; the data movement:
//   * K/V tiles by global_load_lds (lane-linear LDS writes, swizzle applied to the per-lane source chunk).
//   * Two LDS stages, one barrier per tile; the flashmask bounds of the tile ride along (one more piece).
//   * dense mask values of tile t+1 are loaded into registers next to the tile's LDS-DMA (untracked asm
//     loads retired by the same vmcnt(0) at the loop top).
//   * Deferred rescale; the softmax scale folded into the exp2 argument.
// FEAT: compile-time feature set (1 bool mask, 8 additive bf16 mask, 16 additive fp32 mask, 2 flashmask,
// 4 dropout), so every path keeps only the registers it needs (the plain path is unchanged).
template <int D, bool F16, int MINW, int FEAT>
__global__ __launch_bounds__(256, MINW) void fa_fwd_kernel(FwdArgs p) {
  constexpr bool kMask = (FEAT & 25) != 0, kFm = FEAT & 2, kDrop = FEAT & 4;
  constexpr int kMk = (FEAT & 1) ? kMaskBool : ((FEAT & 8) ? kMaskBF16 : ((FEAT & 16) ? kMaskF32 : kMaskNone));
  constexpr int NCH = D / 8;
  constexpr int KS = D / 16;
  constexpr int NDT = D / 32;
  constexpr int BN = 64;
  constexpr int TILE_BYTES = BN * D * 2;
  constexpr int NI = TILE_BYTES / 1024 / 4;  // glds per wave per tensor per tile
  constexpr float kDefer = 8.f;              // log2 of the largest accepted P before a rescale
  constexpr int FM_BYTES = 1024;             // flashmask bounds of one tile: 64 keys x up to 4 int32
  __shared__ __attribute__((aligned(1024))) char smem[4 * TILE_BYTES + 2 * FM_BYTES];
  char* fm_lds = smem + 4 * TILE_BYTES;

  const int nqb = (p.Sq + 127) / 128;
  int bh, rank;
  block_map((int)blockIdx.x, p.B * p.H, nqb, p.grp, bh, rank);
  const int qb = p.causal ? (nqb - 1 - rank) : rank;
  const int b = bh / p.H, h = bh % p.H;
  const int hk = h / (p.H / p.Hk);
  int q_start = 0, k_start = 0, Sq = p.Sq, Sk = p.Sk;
  if (p.cu_q != nullptr) {
    q_start = p.cu_q[b];
    Sq = p.cu_q[b + 1] - q_start;
    k_start = p.cu_k[b];
    Sk = p.cu_k[b + 1] - k_start;
  }
  if (qb * 128 >= Sq) return;  // varlen: this sequence is shorter than the longest (uniform exit)
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 31, hf = lane >> 5;
  const int qi = qb * 128 + w * 32 + r;
  const int shift = Sk - Sq;
  const float c = p.scale_log2;
  const bool varlen = p.cu_q != nullptr;

  Frag qf[KS];
  {
    const uint16_t* qrow = p.q + (varlen ? (int64_t)q_start * p.qs[1] : (int64_t)b * p.qs[0]) +
                           (int64_t)(qi < Sq ? qi : 0) * p.qs[1] + (int64_t)h * p.qs[2];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (qi < Sq) qf[ks].u = *reinterpret_cast<const uint4*>(qrow + ks * 16 + hf * 8);
      else qf[ks].u = make_uint4(0, 0, 0, 0);
    }
  }

  f32x16 oacc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) oacc[dt] = zero16();
  float m_run = -INFINITY, l_run = 0.f;

  int kv_end = Sk;
  if (p.causal) {
    const int last_q = min(qb * 128 + 127, Sq - 1);
    kv_end = min(Sk, last_q + shift + 1);
  }
  const int n_tiles = kv_end > 0 ? (kv_end + BN - 1) / BN : 0;

  const uint16_t* kbase = p.k + (varlen ? (int64_t)k_start * p.ks[1] : (int64_t)b * p.ks[0]) + (int64_t)hk * p.ks[2];
  const uint16_t* vbase = p.v + (varlen ? (int64_t)k_start * p.vs[1] : (int64_t)b * p.vs[0]) + (int64_t)hk * p.vs[2];
  constexpr int mk = kMk;
  const char* mrow = nullptr;  // this lane's mask row (bytes)
  if (kMask) {
    const int esz = mk == kMaskBool ? 1 : (mk == kMaskBF16 ? 2 : 4);
    mrow = reinterpret_cast<const char*>(p.mask) +
           ((int64_t)b * p.ms[0] + (int64_t)h * p.ms[1] + (int64_t)(qi < Sq ? qi : 0) * p.ms[2]) * esz;
  }
  const int* fmb = kFm ? p.fm + (int64_t)b * p.fms[0] + (int64_t)h * p.fms[1] : nullptr;

  // dense-mask values of one tile for this lane: 8 groups of 4 consecutive keys (group g = 4 kt + m:
  // keys kv0 + 32 kt + 8 m + 4 hf + 0..3), as raw 32-bit words (bool: 1 word, bf16: 2, fp32: 4 per group)
  constexpr int kMw = kMk == kMaskF32 ? 4 : (kMk == kMaskBF16 ? 2 : 1);
  uint32_t mv[8][kMw];
  auto mask_load = [&](int tile) {
    const int kv0 = tile * BN;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      int key = kv0 + 32 * (g >> 2) + 8 * (g & 3) + 4 * hf;
      key = key < Sk ? key : 0;  // keys past the end are masked by the bounds check
      if constexpr (kMk == kMaskBool) {
        mv[g][0] = gload4_async(mrow + key);
      } else if constexpr (kMk == kMaskBF16) {
        const uint2 t2 = gload8_async(mrow + 2 * key);
        mv[g][0] = t2.x; mv[g][1] = t2.y;
      } else if constexpr (kMk == kMaskF32) {
        const u32x4 t4 = gload16_async(mrow + 4 * key);
        mv[g][0] = t4[0]; mv[g][1] = t4[1]; mv[g][2] = t4[2]; mv[g][3] = t4[3];
      }
    }
  };

  auto issue = [&](int tile, int stage) {
    const char* kdst = smem + stage * 2 * TILE_BYTES;
    const char* vdst = kdst + TILE_BYTES;
    const int kv0 = tile * BN;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int qq = w * NI + i;
      const int o = qq * 1024 + lane * 16;
      const int row = o / (NCH * 16), slot = (o % (NCH * 16)) / 16;
      const int ch = (img_off<NCH>(row, slot) - row * (NCH * 16)) / 16;  // slot ^ swizzle(row)
      int key = kv0 + row;
      key = key < Sk ? key : Sk - 1;  // rows past the end are masked to -inf below
      glds16_fa(kbase + (int64_t)key * p.ks[1] + ch * 8, kdst + qq * 1024);
      glds16_fa(vbase + (int64_t)key * p.vs[1] + ch * 8, vdst + qq * 1024);
    }
    if (kFm && w == 0) {
      // 64 keys x fm_cols int32 = 16 * fm_cols 16-byte pieces: lanes < 16 * fm_cols
      const int nl = 16 * p.fm_cols;
      if (lane < nl) {
        int key = kv0 + (lane * 4) / p.fm_cols;
        const int part = (lane * 4) % p.fm_cols;
        key = key < Sk ? key : 0;  // (the host pads the key dim to a multiple of 4: a group never crosses it)
        glds16_fa(fmb + (int64_t)key * p.fm_cols + part, fm_lds + stage * FM_BYTES);
      }
    }
  };

  const int gi = lane & 15, qq = gi >> 2, pp = gi & 3, G1 = (lane >> 4) & 1;
  // The mask words of tile t are loaded right after the barrier (no asm result is carried around the loop: a
  // register copy at the back edge could read a destination before its load returned) and retired by a
  // counted vmcnt that leaves tile t+1's LDS-DMA in flight.
  const int dma_per_tile = 2 * NI;
  if (n_tiles > 0) issue(0, 0);
  for (int t = 0; t < n_tiles; ++t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of tile t are in LDS
    raw_barrier();                                     // ... everyone's, and stage (t+1)&1 is free
    if (kMask) mask_load(t);
    const bool more = t + 1 < n_tiles;
    if (more) issue(t + 1, (t + 1) & 1);
    const char* ks_lds = smem + (t & 1) * 2 * TILE_BYTES;
    const char* vs_lds = ks_lds + TILE_BYTES;
    const int kv0 = t * BN;
    int fm_cls = 1;
    if constexpr (kFm) {
      if (p.fm_stats != nullptr) {
        const int* st = p.fm_stats + (int64_t)b * p.fmst[0] + (int64_t)h * p.fmst[1] + (int64_t)t * 8;
        fm_cls = fm_tile_class(st, qb * 128, min(qb * 128 + 127, Sq - 1));
        if (fm_cls == 2) continue;  // uniform: every row of the block is masked for every key of the tile
      }
    }

    f32x16 sacc[2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      sacc[kt] = zero16();
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        Frag a;
        a.u = lds_b128(ks_lds, img_off<NCH>(kt * 32 + r, 2 * ks + hf));
        sacc[kt] = mfma32<F16>(a, qf[ks], sacc[kt]);
      }
    }
    if (kMask) {
      switch (more ? dma_per_tile : 0) {
        case 4: asm volatile("s_waitcnt vmcnt(4)" : "+v"(mv[0][0]), "+v"(mv[7][0]) :: "memory"); break;
        case 8: asm volatile("s_waitcnt vmcnt(8)" : "+v"(mv[0][0]), "+v"(mv[7][0]) :: "memory"); break;
        case 16: asm volatile("s_waitcnt vmcnt(16)" : "+v"(mv[0][0]), "+v"(mv[7][0]) :: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(0)" : "+v"(mv[0][0]), "+v"(mv[7][0]) :: "memory"); break;
      }
#pragma unroll
      for (int g = 0; g < 8; ++g)
#pragma unroll
        for (int j = 0; j < kMw; ++j) asm volatile("" : "+v"(mv[g][j]));
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int g = 4 * kt + (i >> 2), e = i & 3;
          if constexpr (kMk == kMaskBool) {
            if (((mv[g][0] >> (8 * e)) & 0xFFu) == 0u) sacc[kt][i] = -INFINITY;
          } else if constexpr (kMk == kMaskBF16) {
            const uint32_t wd = mv[g][e >> 1];
            sacc[kt][i] += ((e & 1) ? hi_bf16(wd) : lo_bf16(wd)) * p.inv_scale;
          } else if constexpr (kMk == kMaskF32) {
            sacc[kt][i] += __uint_as_float(mv[g][e]) * p.inv_scale;
          }
        }
    }
    const bool need_mask = (kv0 + BN > Sk) || (p.causal && (kv0 + BN - 1 > qb * 128 + shift)) || (kFm && fm_cls);
    if (need_mask) {
      const int* fmt = reinterpret_cast<const int*>(fm_lds + (t & 1) * FM_BYTES);
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int kl = kt * 32 + (i & 3) + 8 * (i >> 2) + 4 * hf;
          const int kj = kv0 + kl;
          bool dead = kj >= Sk || (p.causal && kj > qi + shift);
          if (kFm && fm_cls) dead = dead || fm_masked(fm_canon(fmt + kl * p.fm_cols, p.fm_cols, p.causal), qi);
          if (dead) sacc[kt][i] = -INFINITY;
        }
    }
    float mloc = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 16; ++i) mloc = fmaxf(mloc, sacc[kt][i]);
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
    const float m_new = fmaxf(m_run, mloc);
    // (m_new - m_run) * c: +inf on a row's first live tile, NaN while the row is all -inf (no rescale)
    if (__ballot((m_new - m_run) * c > kDefer)) {
      const float alpha = (m_run == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f((m_run - m_new) * c);
      m_run = m_new;
      l_run *= alpha;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) oacc[dt][i] *= alpha;
    }
    const float mc = (m_run == -INFINITY) ? 0.f : m_run * c;
    float psum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float e = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[kt][i], c, -mc));
        sacc[kt][i] = e;
        psum += e;
      }
    l_run += psum;
    if (kDrop) {
      // keep mask on the PV operand only (the normaliser l uses the undropped P)
      const uint32_t qa = (uint32_t)qi ^ ((uint32_t)bh * 0x9E3779B1u);
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int k0 = kv0 + kt * 32 + 8 * m + 4 * hf;  // multiple of 4: pairs k0/2 and k0/2 + 1
          const uint32_t w0 = drop_hash(p.seed0, p.seed1, qa, (uint32_t)(k0 >> 1));
          const uint32_t w1 = drop_hash(p.seed0, p.seed1, qa, (uint32_t)(k0 >> 1) + 1u);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const uint32_t wd = e < 2 ? w0 : w1;
            const int i = 4 * m + e;
            sacc[kt][i] = drop_keep(wd, k0 + e, p.keep16) ? sacc[kt][i] * p.rkeep : 0.f;
          }
        }
    }

    Frag pf[2][2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float tmp[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) tmp[j] = sacc[kt][8 * s + j];
        pf[kt][s] = pack8<F16>(tmp);
      }

#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      const int cch = (dt * 32 + 16 * G1) / 8 + (pp >> 1);
      const int cb = 8 * (pp & 1);
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int R0 = kt * 32 + 16 * s + 4 * hf;
          Frag a;
          a.h[0] = lds_tr(vs_lds, img_off<NCH>(R0 + qq, cch) + cb);
          a.h[1] = lds_tr(vs_lds, img_off<NCH>(R0 + 8 + qq, cch) + cb);
          oacc[dt] = mfma32<F16>(a, pf[kt][s], oacc[dt]);
        }
      }
    }
  }

  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if (qi < Sq) {
    uint16_t* orow = p.o + (varlen ? (int64_t)q_start * p.os[1] : (int64_t)b * p.os[0]) + (int64_t)qi * p.os[1] +
                     (int64_t)h * p.os[2];
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d0 = dt * 32 + 8 * g + 4 * hf;
        uint2 v2;
        v2.x = pack2<F16>(oacc[dt][4 * g + 0] * inv, oacc[dt][4 * g + 1] * inv);
        v2.y = pack2<F16>(oacc[dt][4 * g + 2] * inv, oacc[dt][4 * g + 3] * inv);
        *reinterpret_cast<uint2*>(orow + d0) = v2;
      }
    }
    if (hf == 0) {
      const float lse = (m_run == -INFINITY) ? INFINITY : (m_run * c * kLn2 + __logf(l_tot));
      p.lse[(int64_t)b * p.lse_s[0] + (int64_t)h * p.lse_s[1] + q_start + qi] = lse;
    }
  }
}

// ------------------------------------------------------------------------------------- backward
struct BwdArgs {
  const uint16_t* q; const uint16_t* k; const uint16_t* v; const uint16_t* o; const uint16_t* dout;
  const float* lse; float* dq_acc; const float* delta; uint16_t* dk; uint16_t* dv;
  int64_t qs[3], ks[3], vs[3], dos[3], dks[3], dvs[3];
  int B, Sq, Sk, H, Hk;
  float scale, scale_log2, inv_scale;
  int causal;
  int grp;
  const int* cu_q; const int* cu_k;
  const void* mask; int mask_kind; int64_t ms[3];
  const int* fm; int fm_cols; int64_t fms[2];
  const int* fm_stats; int64_t fmst[2];
  int dropout; uint32_t keep16; float rkeep; uint32_t seed0, seed1;
  int64_t lse_s[2];
  int abl;  // measurement ablations (0 in normal runs): 1 dQ atomics dropped, 2 dQ step skipped, 4 dK/dV GEMMs skipped
  int k16;  // 1: the 8-wave 16-keys-per-wave kernel (fa_bwd16_kernel) for D = 128 without mask / dropout
  // dS route (fa_bwd16_kernel<.., true> + fa_bwd_dq_kernel): unscaled dS^T tiles [B*H][ds_rows keys][ds_ld queries]
  // (16-bit) instead of fp32 dQ atomics; ds == nullptr: the atomics kernels
  uint16_t* ds; int64_t ds_ld; int ds_rows;
  uint16_t* dq; int64_t dqs[3];
  int dq_grp;  // block_map group of the dQ kernel's grid
};

// delta[b,h,q] = sum_d dO * O   (delta / lse index = b * lse_s0 + h * lse_s1 + q)
template <bool F16>
__global__ __launch_bounds__(256) void fa_bwd_delta(const uint16_t* __restrict__ o, const uint16_t* __restrict__ dout,
                                                    float* __restrict__ delta, int64_t o_sb, int64_t o_ss, int64_t o_sh,
                                                    int64_t d_sb, int64_t d_ss, int64_t d_sh, int B, int Sq, int H, int D,
                                                    int64_t l_sb, int64_t l_sh) {
  const int per_row = D / 8;  // lanes per (b,q,h) row
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t row = gid / per_row;
  const int c = (int)(gid % per_row);
  const int64_t nrows = (int64_t)B * Sq * H;
  float s = 0.f;
  int bb = 0, qq = 0, hh = 0;
  if (row < nrows) {
    hh = (int)(row % H);
    qq = (int)((row / H) % Sq);
    bb = (int)(row / ((int64_t)H * Sq));
    const uint4 a = *reinterpret_cast<const uint4*>(o + bb * o_sb + qq * o_ss + hh * o_sh + c * 8);
    const uint4 g = *reinterpret_cast<const uint4*>(dout + bb * d_sb + qq * d_ss + hh * d_sh + c * 8);
    const uint32_t aw[4] = {a.x, a.y, a.z, a.w}, gw[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) s += half_lo<F16>(aw[j]) * half_lo<F16>(gw[j]) + half_hi<F16>(aw[j]) * half_hi<F16>(gw[j]);
  }
  for (int off = per_row / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (row < nrows && c == 0) delta[(int64_t)bb * l_sb + (int64_t)hh * l_sh + qq] = s;
}

// dq[b,q,h,:] (16-bit, strided) = dq_acc[b,q,h,:] (fp32, contiguous [B,Sq,H,D])
template <bool F16>
__global__ __launch_bounds__(256) void fa_bwd_dq_convert(const float* __restrict__ acc, uint16_t* __restrict__ dq,
                                                         int64_t s_b, int64_t s_s, int64_t s_h, int B, int Sq, int H,
                                                         int D) {
  const int64_t n = (int64_t)B * Sq * H * D / 8;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t e = i * 8;
    const int d = (int)(e % D);
    const int64_t row = e / D;
    const int hh = (int)(row % H), qq = (int)((row / H) % Sq), bb = (int)(row / ((int64_t)H * Sq));
    float v[8];
    load8<float>(acc + e, v);
    uint4 w;
    w.x = pack2<F16>(v[0], v[1]); w.y = pack2<F16>(v[2], v[3]); w.z = pack2<F16>(v[4], v[5]); w.w = pack2<F16>(v[6], v[7]);
    *reinterpret_cast<uint4*>(dq + bb * s_b + qq * s_s + hh * s_h + d) = w;
  }
}

// NW waves x 32 keys per workgroup; CACHE_KV keeps this lane's K / V rows as MFMA B fragments in registers.
template <int D, bool F16, int NW, bool CACHE_KV, int FEAT>
__global__ __launch_bounds__(NW * 64, 1) void fa_bwd_kernel(BwdArgs p) {
  constexpr bool kMask = (FEAT & 25) != 0, kFm = FEAT & 2, kDrop = FEAT & 4;
  constexpr int kMk = (FEAT & 1) ? kMaskBool : ((FEAT & 8) ? kMaskBF16 : ((FEAT & 16) ? kMaskF32 : kMaskNone));
  constexpr int NCH = D / 8;
  constexpr int KS = D / 16;
  constexpr int NDT = D / 32;
  constexpr int NT = NW * 64;
  constexpr int BK = NW * 32;  // keys per workgroup
  constexpr int BM = 32;       // queries per inner step
  constexpr int KT_BYTES = BK * D * 2;
  constexpr int QT_BYTES = BM * D * 2;
  constexpr int DST_BYTES = BK * BM * 2;  // dS^T [BK keys][32 q], 64-byte rows
  constexpr int DT_PER_WAVE = (NDT + NW - 1) / NW;
  constexpr int ATOMICS = 16 * DT_PER_WAVE;  // fire-and-forget dQ atomics per wave per block
  __shared__ __attribute__((aligned(16))) char smem[2 * KT_BYTES + 2 * QT_BYTES + 2 * DST_BYTES + 2 * BM * 4];
  char* k_lds = smem;
  char* v_lds = smem + KT_BYTES;
  char* q_lds = v_lds + KT_BYTES;
  char* do_lds = q_lds + QT_BYTES;
  char* ds_lds = do_lds + QT_BYTES;
  float* lse_s = reinterpret_cast<float*>(ds_lds + 2 * DST_BYTES);  // ds_lds: two dS^T buffers
  float* dlt_s = lse_s + BM;

  const int nkb0 = (p.Sk + BK - 1) / BK;
  int kb, bhk;  // key block 0 is the heaviest under the causal mask: rank order
  block_map((int)blockIdx.x, p.B * p.Hk, nkb0, p.grp, bhk, kb);
  const int b = bhk / p.Hk, hk = bhk % p.Hk;
  const int G = p.H / p.Hk;
  int q_start = 0, k_start = 0, Sq = p.Sq, Sk = p.Sk;
  const bool varlen = p.cu_q != nullptr;
  if (varlen) {
    q_start = p.cu_q[b];
    Sq = p.cu_q[b + 1] - q_start;
    k_start = p.cu_k[b];
    Sk = p.cu_k[b + 1] - k_start;
  }
  if (kb * BK >= Sk) return;  // uniform exit
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 31, hf = lane >> 5;
  const int gi = lane & 15, qq = gi >> 2, pp = gi & 3, G1 = (lane >> 4) & 1;
  const int shift = Sk - Sq;
  const int kj = kb * BK + w * 32 + r;  // this lane's key (MFMA column)

  // K / V tile -> LDS (row image, also read transposed for dQ)
  const uint16_t* kbase = p.k + (varlen ? (int64_t)k_start * p.ks[1] : (int64_t)b * p.ks[0]) + (int64_t)hk * p.ks[2];
  const uint16_t* vbase = p.v + (varlen ? (int64_t)k_start * p.vs[1] : (int64_t)b * p.vs[0]) + (int64_t)hk * p.vs[2];
#pragma unroll
  for (int i = 0; i < BK * NCH / NT; ++i) {
    const int idx = tid + NT * i;
    const int row = idx / NCH, ch = idx % NCH;
    const int key = kb * BK + row;
    uint4 val = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
    if (key < Sk) {
      val = *reinterpret_cast<const uint4*>(kbase + (int64_t)key * p.ks[1] + ch * 8);
      vv = *reinterpret_cast<const uint4*>(vbase + (int64_t)key * p.vs[1] + ch * 8);
    }
    *reinterpret_cast<uint4*>(k_lds + img_off<NCH>(row, ch)) = val;
    *reinterpret_cast<uint4*>(v_lds + img_off<NCH>(row, ch)) = vv;
  }

  f32x16 dk_acc[NDT], dv_acc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) { dk_acc[dt] = zero16(); dv_acc[dt] = zero16(); }

  __syncthreads();
  Frag kfr[CACHE_KV ? KS : 1], vfr[CACHE_KV ? KS : 1];
  if constexpr (CACHE_KV) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      kfr[ks].u = lds_b128(k_lds, img_off<NCH>(w * 32 + r, 2 * ks + hf));
      vfr[ks].u = lds_b128(v_lds, img_off<NCH>(w * 32 + r, 2 * ks + hf));
    }
  }

  // query range of head h that sees any key of this block: the causal start, narrowed by flashmask bounds that
  // hold for every key of the block (rows >= max LTS when no key has an LTE, rows < min UTE when no key has a
  // UTS) — whole masked stretches (other documents, outside a sliding window) are never visited
  int q_begin0 = 0;
  if (p.causal) q_begin0 = max(0, kb * BK - shift);
  const int h0 = hk * G;
  const int64_t dq_row0 = varlen ? (int64_t)q_start : (int64_t)b * p.Sq;
  auto head_range = [&](int h, int& qa, int& qe) {
    qa = q_begin0;
    qe = Sq;
    if constexpr (kFm) {
      if (p.fm_stats != nullptr) {
        const int* st = p.fm_stats + (int64_t)b * p.fmst[0] + (int64_t)h * p.fmst[1] + (int64_t)(kb * (BK / 64)) * 8;
        int mx_lo0 = st[1], mn_lo1 = st[2], mx_up0 = st[5], mn_up1 = st[6];
#pragma unroll
        for (int tt = 1; tt < BK / 64; ++tt) {
          mx_lo0 = max(mx_lo0, st[tt * 8 + 1]); mn_lo1 = min(mn_lo1, st[tt * 8 + 2]);
          mx_up0 = max(mx_up0, st[tt * 8 + 5]); mn_up1 = min(mn_up1, st[tt * 8 + 6]);
        }
        if (mn_lo1 == 0x7fffffff) qe = min(qe, max(mx_lo0, 0));
        if (mx_up0 <= 0) qa = max(qa, min(mn_up1, Sq));
      }
    }
    qa = (qa / BM) * BM;
  };

  constexpr int QLOADS = BM * NCH / NT;
  u32x4 qreg[QLOADS], dreg[QLOADS];
  constexpr int mk = kMk;
  constexpr bool has_fm = kFm;
  // per-iteration prefetch (untracked asm loads, retired by the counted vmcnt at the loop top):
  // Q / dO rows, the row constants, this lane's 16 mask values and (flashmask) this key's row bounds
  float lse_raw = 0.f, dlt_raw = 0.f;
  uint32_t mreg[16];
  bool row_ok = false;
  bool q_ok[QLOADS];
  auto prefetch = [&](int h, int q0) {
    const uint16_t* qbase = p.q + (varlen ? (int64_t)q_start * p.qs[1] : (int64_t)b * p.qs[0]) + (int64_t)h * p.qs[2];
    const uint16_t* dobase =
        p.dout + (varlen ? (int64_t)q_start * p.dos[1] : (int64_t)b * p.dos[0]) + (int64_t)h * p.dos[2];
#pragma unroll
    for (int i = 0; i < QLOADS; ++i) {
      const int idx = tid + NT * i;
      const int row = idx / NCH, ch = idx % NCH;
      const int qx = q0 + row;
      q_ok[i] = qx < Sq;
      const int qc = q_ok[i] ? qx : Sq - 1;
      qreg[i] = gload16_async(qbase + (int64_t)qc * p.qs[1] + ch * 8);
      dreg[i] = gload16_async(dobase + (int64_t)qc * p.dos[1] + ch * 8);
    }
    const int qx = q0 + (tid & (BM - 1));
    row_ok = qx < Sq;
    const int qc = row_ok ? qx : Sq - 1;
    const int64_t lrow = (int64_t)b * p.lse_s[0] + (int64_t)h * p.lse_s[1] + q_start + qc;
    lse_raw = __uint_as_float(gload4_async(p.lse + lrow));
    dlt_raw = __uint_as_float(gload4_async(p.delta + lrow));
  };
  // this lane's 16 dense-mask values for (h, q0): issued after the iteration's barriers, retired by a counted
  // vmcnt before use (never carried around the loop in flight)
  auto mask_load = [&](int h, int q0) {
    if constexpr (kMask) {
      constexpr int esz = kMk == kMaskBool ? 1 : (kMk == kMaskBF16 ? 2 : 4);
      const char* mb = reinterpret_cast<const char*>(p.mask) + ((int64_t)b * p.ms[0] + (int64_t)h * p.ms[1]) * esz;
      const int kc = kj < Sk ? kj : 0;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        int qr = q0 + (i & 3) + 8 * (i >> 2) + 4 * hf;
        qr = qr < Sq ? qr : 0;
        const char* ad = mb + ((int64_t)qr * p.ms[2] + kc) * esz;
        if constexpr (kMk == kMaskBool) mreg[i] = gload1_async(ad);
        else if constexpr (kMk == kMaskBF16) mreg[i] = gload2_async(ad);
        else mreg[i] = gload4_async(ad);
      }
    }
  };
  const bool has_atomics = w < NDT;
  const float inv_scale = 1.f / p.scale;

  // dQ[q][d] += sum_key dS[q][key] K[key][d] for the (head, query block) whose dS^T is in `dsb`; wave w handles
  // d tiles dt = w, w+NW, ... Software-pipelined by one iteration (runs after the next iteration's second barrier).
  auto dq_step = [&](const char* dsb, int h, int qb0) {
    float* dqb = p.dq_acc + dq_row0 * p.H * D + (int64_t)h * D;
    const __amdgpu_buffer_rsrc_t dq_rsrc = __builtin_amdgcn_make_buffer_rsrc(
        dqb, 0, (int)((int64_t)(Sq - 1) * p.H * D * 4 + D * 4), 0x00020000);
    for (int dt = w; dt < NDT; dt += NW) {
      f32x16 qacc = zero16();
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        Frag a, bb;
        // A = dS[q=r][key = 16ks + 8hf + j]: transposed read of the dS^T image (rows = keys)
        const int kr0 = 16 * ks + 8 * hf;
        const int ra = kr0 + qq, rb = kr0 + 4 + qq;
        a.h[0] = lds_tr(dsb, ra * (BM * 2) + (((16 * G1 + 4 * pp) * 2) ^ (((ra >> 2) & 3) << 3)));
        a.h[1] = lds_tr(dsb, rb * (BM * 2) + (((16 * G1 + 4 * pp) * 2) ^ (((rb >> 2) & 3) << 3)));
        // B = K[key = 16ks + 8hf + j][d = dt*32 + r]: transposed read of the K image
        const int cch = (dt * 32 + 16 * G1) / 8 + (pp >> 1);
        bb.h[0] = lds_tr(k_lds, img_off<NCH>(kr0 + qq, cch) + 8 * (pp & 1));
        bb.h[1] = lds_tr(k_lds, img_off<NCH>(kr0 + 4 + qq, cch) + 8 * (pp & 1));
        qacc = mfma32<F16>(a, bb, qacc);
      }
      // byte offsets into this (b, h)'s dQ rows (row stride H*D floats); out-of-range rows (ragged last
      // block) fall outside the buffer resource and are dropped by the hardware
      const int rs = p.H * D * 4;
      const int base = qb0 * rs + (dt * 32 + r) * 4;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qr = (i & 3) + 8 * (i >> 2) + 4 * hf;
        const int off = (qb0 + qr < Sq && !(p.abl & 1)) ? base + qr * rs : 0x7ffffff0;
        __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(qacc[i] * p.scale, dq_rsrc, off, 0, 0);
      }
    }
  };


  // heads of this KV group one after another (dK / dV summed in registers), query blocks pipelined per head:
  // Q / dO / row constants of block i+1 load during block i, block i's dQ runs during block i+1
  for (int hi = 0; hi < G; ++hi) {
    const int h = h0 + hi;
    int qa, qe;
    head_range(h, qa, qe);
    const int n_qb = qa < qe ? (qe - qa + BM - 1) / BM : 0;
    if (n_qb == 0) continue;
    FmBounds fbk{0, 0, 0, 0};  // flashmask bounds of this lane's key for head h (plain loads)
    if constexpr (kFm) {
      const int* fbp = p.fm + (int64_t)b * p.fms[0] + (int64_t)h * p.fms[1] + (int64_t)(kj < Sk ? kj : 0) * p.fm_cols;
      int v4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v4[j] = fbp[j < p.fm_cols ? j : 0];
      fbk = fm_canon(v4, p.fm_cols, p.causal);
    }
    prefetch(h, qa);
    for (int it = 0; it < n_qb; ++it) {
      const int q0 = qa + it * BM;
      if (it == 0 || !has_atomics || ATOMICS > 63) {
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(qreg[0]), "+v"(dreg[0]), "+v"(lse_raw), "+v"(dlt_raw)::"memory");
      } else {
        asm volatile("s_waitcnt vmcnt(%4)" : "+v"(qreg[0]), "+v"(dreg[0]), "+v"(lse_raw), "+v"(dlt_raw)
                     : "n"(ATOMICS > 63 ? 0 : ATOMICS) : "memory");
      }
      if constexpr (QLOADS > 1) asm volatile("" : "+v"(qreg[QLOADS - 1]), "+v"(dreg[QLOADS - 1]));
#pragma unroll
      for (int i = 0; i < QLOADS; ++i) {
        if (!q_ok[i]) {
          qreg[i] = u32x4{0u, 0u, 0u, 0u};
          dreg[i] = u32x4{0u, 0u, 0u, 0u};
        }
      }
      // row constants enter the S / dP accumulators as their initial values:
      // S' = Q K^T - LSE/scale  ->  P = exp2(scale*log2e * S');   dP' = dO V^T - delta  ->  dS = P * dP'
      const float lse_r = row_ok ? -lse_raw * inv_scale : -INFINITY;
      const float dlt_r = row_ok ? -dlt_raw : 0.f;
      lds_barrier();  // previous iteration's LDS reads done
#pragma unroll
      for (int i = 0; i < QLOADS; ++i) {
        const int idx = tid + NT * i;
        const int row = idx / NCH, ch = idx % NCH;
        *reinterpret_cast<u32x4*>(q_lds + img_off<NCH>(row, ch)) = qreg[i];
        *reinterpret_cast<u32x4*>(do_lds + img_off<NCH>(row, ch)) = dreg[i];
      }
      if (tid < BM) {
        lse_s[tid] = lse_r;
        dlt_s[tid] = dlt_r;
      }
      lds_barrier();
      if (kMask) mask_load(h, q0);
      if (it + 1 < n_qb) prefetch(h, q0 + BM);
      if (it > 0 && !(p.abl & 2)) dq_step(ds_lds + (((it - 1) & 1) * DST_BYTES), h, q0 - BM);
      const bool dq_ran = it > 0 && has_atomics;

      // S' and dP' : rows q (registers), cols = this lane's key.
      f32x16 sacc, pacc;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 l4 = *reinterpret_cast<const float4*>(lse_s + 8 * g + 4 * hf);
        const float4 d4 = *reinterpret_cast<const float4*>(dlt_s + 8 * g + 4 * hf);
        sacc[4 * g + 0] = l4.x; sacc[4 * g + 1] = l4.y; sacc[4 * g + 2] = l4.z; sacc[4 * g + 3] = l4.w;
        pacc[4 * g + 0] = d4.x; pacc[4 * g + 1] = d4.y; pacc[4 * g + 2] = d4.z; pacc[4 * g + 3] = d4.w;
      }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        Frag qa, da;
        qa.u = lds_b128(q_lds, img_off<NCH>(r, 2 * ks + hf));
        da.u = lds_b128(do_lds, img_off<NCH>(r, 2 * ks + hf));
        if constexpr (CACHE_KV) {
          sacc = mfma32<F16>(qa, kfr[ks], sacc);
          pacc = mfma32<F16>(da, vfr[ks], pacc);
        } else {
          Frag kk, vv;
          kk.u = lds_b128(k_lds, img_off<NCH>(w * 32 + r, 2 * ks + hf));
          vv.u = lds_b128(v_lds, img_off<NCH>(w * 32 + r, 2 * ks + hf));
          sacc = mfma32<F16>(qa, kk, sacc);
          pacc = mfma32<F16>(da, vv, pacc);
        }
      }
      if constexpr (kMask) {
        // retire the mask values: the prefetch (2 * QLOADS + 2 loads) and the dQ atomics were issued after them
        const int n_after = (it + 1 < n_qb ? 2 * QLOADS + 2 : 0) + (dq_ran ? ATOMICS : 0);
        switch (n_after) {
          case 4: asm volatile("s_waitcnt vmcnt(4)" : "+v"(mreg[0]), "+v"(mreg[15]) :: "memory"); break;
          case 6: asm volatile("s_waitcnt vmcnt(6)" : "+v"(mreg[0]), "+v"(mreg[15]) :: "memory"); break;
          case 16: asm volatile("s_waitcnt vmcnt(16)" : "+v"(mreg[0]), "+v"(mreg[15]) :: "memory"); break;
          case 18: asm volatile("s_waitcnt vmcnt(18)" : "+v"(mreg[0]), "+v"(mreg[15]) :: "memory"); break;
          case 20: asm volatile("s_waitcnt vmcnt(20)" : "+v"(mreg[0]), "+v"(mreg[15]) :: "memory"); break;
          case 22: asm volatile("s_waitcnt vmcnt(22)" : "+v"(mreg[0]), "+v"(mreg[15]) :: "memory"); break;
          case 34: asm volatile("s_waitcnt vmcnt(34)" : "+v"(mreg[0]), "+v"(mreg[15]) :: "memory"); break;
          default: asm volatile("s_waitcnt vmcnt(0)" : "+v"(mreg[0]), "+v"(mreg[15]) :: "memory"); break;
        }
#pragma unroll
        for (int i = 1; i < 15; ++i) asm volatile("" : "+v"(mreg[i]));
      }
      if (kMask && (mk == kMaskBF16 || mk == kMaskF32)) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float madd = mk == kMaskBF16 ? lo_bf16(mreg[i]) : __uint_as_float(mreg[i]);
          sacc[i] += madd * inv_scale;
        }
      }
      // P and dS computed in place, then packed straight into MFMA fragments.
      const bool need_mask = kj >= Sk || (p.causal && kb * BK + BK - 1 > q0 + shift) || mk == kMaskBool || kFm;
      const uint32_t ka = (uint32_t)(kj >> 1);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qr = (i & 3) + 8 * (i >> 2) + 4 * hf;
        float pr = __builtin_amdgcn_exp2f(sacc[i] * p.scale_log2);
        if (need_mask) {
          bool dead = kj >= Sk || (p.causal && kj > q0 + qr + shift);
          if (kMask && mk == kMaskBool) dead = dead || (mreg[i] & 0xFFu) == 0u;
          if (kFm) dead = dead || fm_masked(fbk, q0 + qr);
          if (dead) pr = 0.f;
        }
        if (kDrop) {
          const uint32_t qa = (uint32_t)(q0 + qr) ^ ((uint32_t)(b * p.H + h) * 0x9E3779B1u);
          const bool keep = drop_keep(drop_hash(p.seed0, p.seed1, qa, ka), kj, p.keep16);
          const float ndelta = dlt_s[qr];  // -delta of this row (the dP accumulator's initial value)
          const float dp = pacc[i] - ndelta;
          pacc[i] = pr * ((keep ? dp * p.rkeep : 0.f) + ndelta);
          sacc[i] = keep ? pr * p.rkeep : 0.f;
        } else {
          sacc[i] = pr;
          pacc[i] = pr * pacc[i];
        }
      }
      Frag pf[2], sf[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float a[8], cc[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) { a[j] = sacc[8 * s + j]; cc[j] = pacc[8 * s + j]; }
        pf[s] = pack8<F16>(a);
        sf[s] = pack8<F16>(cc);
      }

      // dV^T += dO^T P ; dK^T += Q^T dS  (A via transposed reads of the dO / Q images)
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        if (p.abl & 4) break;
        const int cch = (dt * 32 + 16 * G1) / 8 + (pp >> 1);
        const int cb = 8 * (pp & 1);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int R0 = 16 * s + 4 * hf;
          Frag a, cfr;
          a.h[0] = lds_tr(do_lds, img_off<NCH>(R0 + qq, cch) + cb);
          a.h[1] = lds_tr(do_lds, img_off<NCH>(R0 + 8 + qq, cch) + cb);
          dv_acc[dt] = mfma32<F16>(a, pf[s], dv_acc[dt]);
          cfr.h[0] = lds_tr(q_lds, img_off<NCH>(R0 + qq, cch) + cb);
          cfr.h[1] = lds_tr(q_lds, img_off<NCH>(R0 + 8 + qq, cch) + cb);
          dk_acc[dt] = mfma32<F16>(cfr, sf[s], dk_acc[dt]);
        }
      }

      // dS^T tile [BK keys][32 q]: lane writes its key row, 4 consecutive q per 8-byte store.
      // 64-byte rows: the 8-byte column slot is XORed with (row >> 2) & 3 so that the 16 rows of a
      // store's lane group land on distinct banks (rows r, r+4, r+8, r+12 would collide otherwise).
      {
        const int row = w * 32 + r;
        char* rowp = ds_lds + (it & 1) * DST_BYTES + row * (BM * 2);
        const int sw = ((row >> 2) & 3) << 3;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const Frag f = sf[s];
          *reinterpret_cast<uint2*>(rowp + (((16 * s + 4 * hf) * 2) ^ sw)) = make_uint2(f.u.x, f.u.y);
          *reinterpret_cast<uint2*>(rowp + (((16 * s + 8 + 4 * hf) * 2) ^ sw)) = make_uint2(f.u.z, f.u.w);
        }
      }
    }
    // dQ of the head's last block
    lds_barrier();
    if (!(p.abl & 2)) dq_step(ds_lds + (((n_qb - 1) & 1) * DST_BYTES), h, qa + (n_qb - 1) * BM);
  }

  // write dK = scale * (dK^T)^T, dV = (dV^T)^T : lane = key, 4 consecutive d per 8-byte store
  if (kj < Sk) {
    uint16_t* dkrow = p.dk + (varlen ? (int64_t)k_start * p.dks[1] : (int64_t)b * p.dks[0]) + (int64_t)kj * p.dks[1] +
                      (int64_t)hk * p.dks[2];
    uint16_t* dvrow = p.dv + (varlen ? (int64_t)k_start * p.dvs[1] : (int64_t)b * p.dvs[0]) + (int64_t)kj * p.dvs[1] +
                      (int64_t)hk * p.dvs[2];
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d0 = dt * 32 + 8 * g + 4 * hf;
        uint2 a, cc;
        a.x = pack2<F16>(dk_acc[dt][4 * g] * p.scale, dk_acc[dt][4 * g + 1] * p.scale);
        a.y = pack2<F16>(dk_acc[dt][4 * g + 2] * p.scale, dk_acc[dt][4 * g + 3] * p.scale);
        cc.x = pack2<F16>(dv_acc[dt][4 * g], dv_acc[dt][4 * g + 1]);
        cc.y = pack2<F16>(dv_acc[dt][4 * g + 2], dv_acc[dt][4 * g + 3]);
        *reinterpret_cast<uint2*>(dkrow + d0) = a;
        *reinterpret_cast<uint2*>(dvrow + d0) = cc;
      }
    }
  }
}



// ---------------------------------------------------------------------------------------------------------------
// Backward, 16 keys per wave (D = 128, no mask / flashmask / dropout): 8 waves x 16 keys = the same 128-key block
// per workgroup as fa_bwd_kernel<128, .., 4, ..>, but on v_mfma_f32_16x16x32 tiles, so a wave's dK^T / dV^T
// accumulators are 2 x 8 x 4 fp32 registers (not 2 x 4 x 16) and its cached K / V fragments 2 x 16: the kernel fits
// 256 registers and runs 2 waves per SIMD (the 4-wave kernel holds one, and its S / dP / softmax / LDS phases
// serialise on it). Same math and pipeline:
//   S = Q K^T and dP = dO V^T as [16 q][16 key] tiles (2 query tiles of a 32-query block), initialised with the
//   row constants (-LSE/scale, -delta); P = exp2(scale*log2e*S), dS = P dP. A 16x16x32 accumulator is the B operand
//   of the next product with the k (query) index permuted: element j of lane group g is query 4g+j (j < 4) of tile 0
//   and 16+4g+j-4 of tile 1 — so P / dS feed dV^T += dO^T P and dK^T += Q^T dS with no lane movement; the A operands
//   dO^T / Q^T come from ds_read_b64_tr_b16 reads of the row images at those query rows.
//   dQ += dS K over the workgroup's 128 keys through a dS^T LDS image (rows = key, 64-byte rows), wave w owning
//   d columns 16w..16w+15, fp32 atomics into dq_acc; software-pipelined one block behind like the 4-wave kernel.
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <bool F16>
__device__ __forceinline__ f32x4 mfma16(const Frag& a, const Frag& b, f32x4 c) {
  if constexpr (F16) return __builtin_amdgcn_mfma_f32_16x16x32_f16(a.f, b.f, c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, c, 0, 0, 0);
}

// [rows][128 x 16-bit] image as 8-row x 32-column subtiles of 512 B (cdna_hip_programming.md T10 image (a)), the
// 16-byte chunk of a 64-byte subtile row XOR-swizzled by s(row) = {0, 2, 3, 1}[(row >> 2) & 3]. Under the LDS lane
// groups of MI355X_MICROARCH.md (ds_read_b128: 4 x 16 lanes {0-3,12-15,20-27} ..., ds_read_b64_tr_b16: 2 x 32) every
// read below is conflict-free: the Q / dO / K fragment reads (b128), the Q / dO transposed reads of dV / dK and the K
// transposed reads of dQ (the previous s(row) = (row >> 2) & 3 left the first two 2-way conflicted: PMC showed 44 %
// of the kernel's LDS cycles as bank conflicts). The reads of one loop stay a per-lane base plus immediates (a chunk
// step of 4 or a row step of 8 is a constant), so few address registers stay live.
__device__ __forceinline__ int fa_swz(int row) { return (0x78 >> (2 * ((row >> 2) & 3))) & 3; }
__device__ __forceinline__ int img_a(int row, int ch) {
  return 2048 * (row >> 3) + 512 * (ch >> 2) + 64 * (row & 7) + 16 * ((ch & 3) ^ fa_swz(row));
}

// byte offset of the 8-byte unit (row, col4) of a [rows][32 x 16-bit] image with 64-byte rows (col4 = column / 4),
// swizzled by (row >> 1) & 7: the 16-lane groups of the ds_write_b64 stores (16 consecutive rows) and the 32-lane
// groups of the transposed reads (rows r, r + 8 of one bank quarter) hit distinct banks. The second query tile's
// columns (col4 + 4) are the base XOR 32.
__device__ __forceinline__ int dst_off(int row, int col4) {
  return row * 64 + ((col4 ^ ((row >> 1) & 7)) << 3);
}

// DSQ (the dS route): the pipelined dQ step is replaced by a coalesced copy of the block's dS^T image
// [128 keys][32 queries] to p.ds (one 16-byte store per thread); fa_bwd_dq_kernel computes dQ = scale * dS K from
// it. No fp32 dQ buffer, no atomics (they held the kernel at the chip's atomic rate: 4096 fp32 adds per block
// per workgroup), no convert pass. Query blocks start at a 128-aligned row so every dS^T tile the dQ kernel
// reads below the causal diagonal has been written (zeros where masked).
template <bool F16, bool DSQ>
__global__ __launch_bounds__(512, 1) void fa_bwd16_kernel(BwdArgs p) {
  constexpr int D = 128, NCH = 16, NW = 8, NT = NW * 64, BK = 128, BM = 32;
  constexpr int KT_BYTES = BK * D * 2;
  constexpr int QT_BYTES = BM * D * 2;
  constexpr int DST_BYTES = BK * BM * 2;
  // K, V | Q, dO (two stages each, filled by global_load_lds) | dS^T (two stages) | row constants (two stages:
  // 32 LSE then 32 delta values)
  __shared__ __attribute__((aligned(16))) char smem[2 * KT_BYTES + 4 * QT_BYTES + 2 * DST_BYTES + 2 * 2 * BM * 4];
  char* k_lds = smem;
  char* v_lds = smem + KT_BYTES;
  char* q_st = v_lds + KT_BYTES;          // stage s: q_st + s * QT_BYTES
  char* do_st = q_st + 2 * QT_BYTES;
  char* ds_lds = do_st + 2 * QT_BYTES;
  char* rc_st = ds_lds + 2 * DST_BYTES;   // stage s: rc_st + s * 256

  const int nkb0 = (p.Sk + BK - 1) / BK;
  int kb, bhk;
  block_map((int)blockIdx.x, p.B * p.Hk, nkb0, p.grp, bhk, kb);
  const int b = bhk / p.Hk, hk = bhk % p.Hk;
  const int G = p.H / p.Hk;
  int q_start = 0, k_start = 0, Sq = p.Sq, Sk = p.Sk;
  const bool varlen = p.cu_q != nullptr;
  if (varlen) {
    q_start = p.cu_q[b];
    Sq = p.cu_q[b + 1] - q_start;
    k_start = p.cu_k[b];
    Sk = p.cu_k[b + 1] - k_start;
  }
  if (kb * BK >= Sk) return;  // uniform exit
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r16 = lane & 15, kg = lane >> 4;
  const int tq = r16 >> 2, tp = r16 & 3;  // transposed reads: block row and column quad this lane addresses
  const int shift = Sk - Sq;
  const int kj = kb * BK + w * 16 + r16;  // this lane's key (MFMA column of S / dP, of dK^T / dV^T)

  const uint16_t* kbase = p.k + (varlen ? (int64_t)k_start * p.ks[1] : (int64_t)b * p.ks[0]) + (int64_t)hk * p.ks[2];
  const uint16_t* vbase = p.v + (varlen ? (int64_t)k_start * p.vs[1] : (int64_t)b * p.vs[0]) + (int64_t)hk * p.vs[2];
#pragma unroll
  for (int i = 0; i < BK * NCH / NT; ++i) {
    const int idx = tid + NT * i;
    const int row = idx / NCH, ch = idx % NCH;
    const int key = kb * BK + row;
    uint4 val = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
    if (key < Sk) {
      val = *reinterpret_cast<const uint4*>(kbase + (int64_t)key * p.ks[1] + ch * 8);
      vv = *reinterpret_cast<const uint4*>(vbase + (int64_t)key * p.vs[1] + ch * 8);
    }
    *reinterpret_cast<uint4*>(k_lds + img_a(row, ch)) = val;
    *reinterpret_cast<uint4*>(v_lds + img_a(row, ch)) = vv;
  }
  f32x4 dk_acc[8], dv_acc[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt)
#pragma unroll
    for (int i = 0; i < 4; ++i) { dk_acc[dt][i] = 0.f; dv_acc[dt][i] = 0.f; }
  __syncthreads();
  // K^T / V^T B fragments of this wave's 16 keys: element j of group kg = d 32ks + 8kg + j
  Frag kfr[4], vfr[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    kfr[ks].u = lds_b128(k_lds, img_a(w * 16 + r16, 4 * ks + kg));
    vfr[ks].u = lds_b128(v_lds, img_a(w * 16 + r16, 4 * ks + kg));
  }

  int q_begin0 = 0;
  if (p.causal) q_begin0 = max(0, kb * BK - shift);
  q_begin0 = DSQ ? (q_begin0 / 128) * 128 : (q_begin0 / BM) * BM;
  const int h0 = hk * G;
  const int64_t dq_row0 = varlen ? (int64_t)q_start : (int64_t)b * p.Sq;

  // Q / dO block q0 of head h -> stage sl by global_load_lds (no registers in flight: at 254 VGPRs an asm load's
  // destination could be moved by the allocator before the data lands). The LDS write is lane-linear (wave w:
  // bytes 1024w .. 1024w + 1023 of the tile), so each lane fetches the chunk (row, ch) that img_a puts at its
  // destination. Wave 0 also fetches the 32 LSE (lanes 0..31) and delta (lanes 32..63) values of the block.
  const int o_dst = 1024 * w + 16 * lane;
  const int pf_row = 8 * (o_dst >> 11) + ((o_dst & 511) >> 6);
  const int pf_ch = 4 * ((o_dst & 2047) >> 9) + (((o_dst & 63) >> 4) ^ fa_swz(pf_row));
  auto prefetch = [&](int h, int q0, int sl) {
    const uint16_t* qbase = p.q + (varlen ? (int64_t)q_start * p.qs[1] : (int64_t)b * p.qs[0]) + (int64_t)h * p.qs[2];
    const uint16_t* dobase =
        p.dout + (varlen ? (int64_t)q_start * p.dos[1] : (int64_t)b * p.dos[0]) + (int64_t)h * p.dos[2];
    const int qx = q0 + pf_row;
    const int qc = qx < Sq ? qx : Sq - 1;
    glds16_fa(qbase + (int64_t)qc * p.qs[1] + pf_ch * 8, q_st + sl * QT_BYTES + 1024 * w);
    glds16_fa(dobase + (int64_t)qc * p.dos[1] + pf_ch * 8, do_st + sl * QT_BYTES + 1024 * w);
    if (w == 0) {
      const int qr = q0 + (lane & 31);
      const int qrc = qr < Sq ? qr : Sq - 1;
      const int64_t lrow = (int64_t)b * p.lse_s[0] + (int64_t)h * p.lse_s[1] + q_start + qrc;
      glds4_fa(lane < 32 ? (const void*)(p.lse + lrow) : (const void*)(p.delta + lrow), rc_st + sl * 256);
    }
  };
  const float inv_scale = 1.f / p.scale;

  auto dq_step = [&](const char* dsb, int h, int qb0) {
    float* dqb = p.dq_acc + dq_row0 * p.H * D + (int64_t)h * D;
    const __amdgpu_buffer_rsrc_t dq_rsrc = __builtin_amdgcn_make_buffer_rsrc(
        dqb, 0, (int)((int64_t)(Sq - 1) * p.H * D * 4 + D * 4), 0x00020000);
    f32x4 qacc[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int i = 0; i < 4; ++i) qacc[qt][i] = 0.f;
    // per-lane bases; the key block 32ks is +8192 (K image) / +2048 (dS^T image) and query tile 1 is +32 bytes
    const int kb0 = img_a(8 * kg + tq, 2 * w + (tp >> 1)) + 8 * (tp & 1);
    const int kb4 = img_a(8 * kg + 4 + tq, 2 * w + (tp >> 1)) + 8 * (tp & 1);
    const int sb0 = dst_off(8 * kg + tq, tp), sb4 = dst_off(8 * kg + 4 + tq, tp);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      Frag bb;  // K[key 32ks + 8kg + j][d 16w + r16]
      bb.h[0] = lds_tr(k_lds, kb0 + 8192 * ks);
      bb.h[1] = lds_tr(k_lds, kb4 + 8192 * ks);
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        Frag a;  // dS[q 16qt + r16][key 32ks + 8kg + j] from the dS^T image
        a.h[0] = lds_tr(dsb, (sb0 ^ (32 * qt)) + 2048 * ks);
        a.h[1] = lds_tr(dsb, (sb4 ^ (32 * qt)) + 2048 * ks);
        qacc[qt] = mfma16<F16>(a, bb, qacc[qt]);
      }
      if (ks & 1) __builtin_amdgcn_sched_barrier(0);
    }
    const int rs = p.H * D * 4;
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int qr = 16 * qt + 4 * kg + i;
        const int off = (qb0 + qr < Sq) ? (qb0 + qr) * rs + (16 * w + r16) * 4 : 0x7ffffff0;
        __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(qacc[qt][i] * p.scale, dq_rsrc, off, 0, 0);
      }
  };
  // DSQ: the block's dS [32 q][128 keys] goes to the scratch in key groups of 32: group g (keys 32g..32g+31) is a
  // row-major [ds_ld queries][32 keys] matrix, so a dQ key step reads 128 contiguous 64-byte rows (one 8 KiB run)
  // and this store writes 4 runs of 2 KiB. Wave w reads the fragment (keys 32ks.., queries 16qt..) of the dS^T image
  // transposed (the dQ operand read of the atomics kernel): lane (r16, kg) holds keys 8kg..8kg+7 of query 16qt + r16
  // = 16 contiguous bytes; one global_store_dwordx4 per lane (inline asm: exactly one vector-memory op, which the
  // counted vmcnt at the loop top relies on), 1 KiB contiguous per wave instruction.
  const int st_ks = w >> 1, st_qt = w & 1;
  const int st_o0 = (dst_off(8 * kg + tq, tp) ^ (32 * st_qt)) + 2048 * st_ks;
  const int st_o1 = (dst_off(8 * kg + 4 + tq, tp) ^ (32 * st_qt)) + 2048 * st_ks;
  const int64_t nkg = p.ds_rows / 32;
  auto ds_store = [&](const char* dsb, int h, int qb0) {
    Frag a;
    a.h[0] = lds_tr(dsb, st_o0);
    a.h[1] = lds_tr(dsb, st_o1);
    const u32x4 v = {a.u.x, a.u.y, a.u.z, a.u.w};
    uint16_t* dst = p.ds + (((int64_t)(b * p.H + h) * nkg + kb * 4 + st_ks) * p.ds_ld + qb0 + 16 * st_qt + r16) * 32 +
                    8 * kg;
    asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(dst), "v"(v) : "memory");
  };

  for (int hi = 0; hi < G; ++hi) {
    const int h = h0 + hi;
    const int qa = q_begin0;
    const int n_qb = qa < Sq ? (Sq - qa + BM - 1) / BM : 0;
    if (n_qb == 0) continue;
    prefetch(h, qa, 0);
    // n_qb + 1 passes: the last one only runs the pipelined dQ step of the last block (one dq_step call site:
    // a second inlined copy after the loop pushed the kernel past 256 registers)
    for (int it = 0; it <= n_qb; ++it) {
      const int q0 = qa + it * BM;
      const bool last = it == n_qb;
      const int sl = it & 1;
      // this block's stage has landed: the loads were issued in the previous pass, before its 8 dQ atomics
      if (!last) {
        if (it >= 2) {
          if constexpr (DSQ) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
      lds_barrier();  // every wave's stage data visible; the previous pass's reads of the other stage done
      if (!last && it + 1 < n_qb) prefetch(h, q0 + BM, sl ^ 1);
      if constexpr (DSQ) {
        if (it > 0) ds_store(ds_lds + (((it - 1) & 1) * DST_BYTES), h, q0 - BM);
      } else {
        if (it > 0 && p.k16 == 1) dq_step(ds_lds + (((it - 1) & 1) * DST_BYTES), h, q0 - BM);
      }
      if (last) break;

      const char* q_lds = q_st + sl * QT_BYTES;
      const char* do_lds = do_st + sl * QT_BYTES;
      const float* lse_s = reinterpret_cast<const float*>(rc_st + sl * 256);
      const float* dlt_s = lse_s + BM;
      // S' and dP' tiles: rows = queries 16qt + 4kg + i, column = this lane's key; the row constants enter as the
      // accumulators' initial values (-LSE/scale, -delta; rows past Sq: -inf, 0)
      f32x4 sacc[2], pacc[2];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const float4 l4 = *reinterpret_cast<const float4*>(lse_s + 16 * qt + 4 * kg);
        const float4 d4 = *reinterpret_cast<const float4*>(dlt_s + 16 * qt + 4 * kg);
        const float lv[4] = {l4.x, l4.y, l4.z, l4.w}, dv4[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bool ok = q0 + 16 * qt + 4 * kg + i < Sq;
          sacc[qt][i] = ok ? -lv[i] * inv_scale : -INFINITY;
          pacc[qt][i] = ok ? -dv4[i] : 0.f;
        }
      }
      const int rb = img_a(r16, kg);  // query tile qt: +4096, d block 32ks: +512
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          Frag qf, df;
          qf.u = lds_b128(q_lds, rb + 4096 * qt + 512 * ks);
          df.u = lds_b128(do_lds, rb + 4096 * qt + 512 * ks);
          sacc[qt] = mfma16<F16>(qf, kfr[ks], sacc[qt]);
          pacc[qt] = mfma16<F16>(df, vfr[ks], pacc[qt]);
        }
        if (ks & 1) __builtin_amdgcn_sched_barrier(0);
      }
      const bool need_mask = kj >= Sk || (p.causal && kb * BK + BK - 1 > q0 + shift);
      float pv[8], sv[8];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int qr = 16 * qt + 4 * kg + i;
          float pr = __builtin_amdgcn_exp2f(sacc[qt][i] * p.scale_log2);
          if (need_mask && (kj >= Sk || (p.causal && kj > q0 + qr + shift))) pr = 0.f;
          pv[4 * qt + i] = pr;
          sv[4 * qt + i] = pr * pacc[qt][i];
          if (p.k16 >= 3) {  // debug levels (tools/fa16_diag.py): 3 = P := 1, 4 = P := S' (raw accumulator)
            pv[4 * qt + i] = p.k16 == 3 ? 1.f : sacc[qt][i];
            sv[4 * qt + i] = pacc[qt][i];
          }
        }
      const Frag pf = pack8<F16>(pv), sf = pack8<F16>(sv);

      // dV^T += dO^T P ; dK^T += Q^T dS  (A: transposed reads at query rows 4kg+tq and 16+4kg+tq)
      // transposed-read bases for even / odd d tiles; d tiles 2m, 2m+1: +512m; query rows 16..: +4096
      const int tb0 = img_a(4 * kg + tq, tp >> 1) + 8 * (tp & 1);
      const int tb1 = img_a(4 * kg + tq, 2 + (tp >> 1)) + 8 * (tp & 1);
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) {
        const int tb = ((dt & 1) ? tb1 : tb0) + 512 * (dt >> 1);
        Frag a, c;
        a.h[0] = lds_tr(do_lds, tb);
        a.h[1] = lds_tr(do_lds, tb + 4096);
        dv_acc[dt] = mfma16<F16>(a, pf, dv_acc[dt]);
        c.h[0] = lds_tr(q_lds, tb);
        c.h[1] = lds_tr(q_lds, tb + 4096);
        dk_acc[dt] = mfma16<F16>(c, sf, dk_acc[dt]);
        if (dt & 1) __builtin_amdgcn_sched_barrier(0);  // bound the reads in flight (register budget: 2 waves/SIMD)
      }
      // dS^T [128 keys][32 q]: this lane's key row, queries 4kg..4kg+3 and 16+4kg..16+4kg+3
      {
        char* dsb = ds_lds + (it & 1) * DST_BYTES;
        const int row = w * 16 + r16;
        *reinterpret_cast<uint2*>(dsb + dst_off(row, kg)) = make_uint2(sf.u.x, sf.u.y);
        *reinterpret_cast<uint2*>(dsb + dst_off(row, 4 + kg)) = make_uint2(sf.u.z, sf.u.w);
      }
    }
  }

  if (kj < Sk) {
    uint16_t* dkrow = p.dk + (varlen ? (int64_t)k_start * p.dks[1] : (int64_t)b * p.dks[0]) + (int64_t)kj * p.dks[1] +
                      (int64_t)hk * p.dks[2];
    uint16_t* dvrow = p.dv + (varlen ? (int64_t)k_start * p.dvs[1] : (int64_t)b * p.dvs[0]) + (int64_t)kj * p.dvs[1] +
                      (int64_t)hk * p.dvs[2];
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      const int d0 = 16 * dt + 4 * kg;
      uint2 a, cc;
      a.x = pack2<F16>(dk_acc[dt][0] * p.scale, dk_acc[dt][1] * p.scale);
      a.y = pack2<F16>(dk_acc[dt][2] * p.scale, dk_acc[dt][3] * p.scale);
      cc.x = pack2<F16>(dv_acc[dt][0], dv_acc[dt][1]);
      cc.y = pack2<F16>(dv_acc[dt][2], dv_acc[dt][3]);
      *reinterpret_cast<uint2*>(dkrow + d0) = a;
      *reinterpret_cast<uint2*>(dvrow + d0) = cc;
    }
  }
}

// ---------------------------------------------------------------------------------------------------------------
// dQ of the dS route: dQ[b, q, h, :] = scale * sum_key dS[q][key] K[b, key, hk, :] from the dS tiles written by
// fa_bwd16_kernel<.., true> (key groups of 32: [ds_ld queries][32 keys] row-major each). One workgroup = 4 waves =
// 128 queries x 128 d of one (batch, head); key steps of 32 = one key group: the A operand is one contiguous 8 KiB
// run ([128 q][32 keys], K-major: ds_read_b128 fragments, 16-byte chunks swizzled by ((row >> 3) & 1) << 1), the B
// operand K [32 keys][128 d] an MN-major image read with ds_read_b64_tr_b16 (the MN-major fragment read of
// gemm.hip). Both filled by LDS-DMA with the swizzle on the source address. Waves 2 x 2, 64 x 64 outputs each
// (4 x 4 MFMA 16x16x32 tiles). The dS stream is read once from HBM, so the loop is load-latency bound: a 4-slot LDS
// ring (64 KiB) keeps three key steps in flight per workgroup and two workgroups share a CU. Causal: key steps up to
// the block's last visible key; heaviest blocks first.
__device__ __forceinline__ int dq_swz(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 1; }

__device__ __forceinline__ Frag dq_frag(const char* img, int rbase, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
  const int col = rbase + pp * 4;
  const int lc = col >> 3, sub = (col & 7) * 2;
  const int k1 = g * 8 + q, k2 = k1 + 4;
  Frag f;
  f.h[0] = lds_tr(img, k1 * 256 + ((lc ^ dq_swz(k1)) << 4) + sub);
  f.h[1] = lds_tr(img, k2 * 256 + ((lc ^ dq_swz(k2)) << 4) + sub);
  return f;
}

__device__ __forceinline__ void dq_wait_after(int n) {  // "all but the 4 n youngest loads" (4 glds per lane per step)
  if (n >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (n == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <bool F16>
__global__ __launch_bounds__(256, 2) void fa_bwd_dq_kernel(BwdArgs p) {
  constexpr int TB = 32 * 128 * 2;  // one operand image: 8 KiB
  constexpr int NS = 4;             // ring slots
  __shared__ __attribute__((aligned(1024))) char smem[NS * 2 * TB];
  const int nqb = (p.Sq + 127) / 128;
  int bh, rank;
  block_map((int)blockIdx.x, p.B * p.H, nqb, p.dq_grp, bh, rank);
  const int qb = p.causal ? (nqb - 1 - rank) : rank;
  const int b = bh / p.H, h = bh % p.H, hk = h / (p.H / p.Hk);
  const int q0 = qb * 128;
  const int shift = p.Sk - p.Sq;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int wm = w >> 1, wn = w & 1;
  int kend = p.Sk;
  if (p.causal) kend = min(p.Sk, min(q0 + 127, p.Sq - 1) + shift + 1);
  const int nkt = kend > 0 ? (kend + 31) / 32 : 0;

  const uint16_t* ds = p.ds + ((int64_t)bh * (p.ds_rows / 32) * p.ds_ld + q0) * 32;  // key group 0, query q0
  const int64_t ds_grp = p.ds_ld * 32;                                               // elements per key group
  const uint16_t* kb = p.k + (int64_t)b * p.ks[0] + (int64_t)hk * p.ks[2];
  // per-lane staging geometry: 2 pieces of 1 KiB per operand per wave. A (K-major): piece = 16 query rows of 64 B;
  // B (MN-major): piece = 4 key rows of 256 B
  int aoff[2], srow[2], scol[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int lin = (i * 4 + w) * 64 + lane;
    const int arow = lin >> 2;
    aoff[i] = arow * 32 + (((lin & 3) ^ (((arow >> 3) & 1) << 1)) * 8);
    srow[i] = lin >> 4;
    scol[i] = ((lin & 15) ^ dq_swz(srow[i])) * 8;
  }
  auto issue = [&](int t) {
    char* a_img = smem + (t % NS) * 2 * TB;
    char* b_img = a_img + TB;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      glds16_fa(ds + t * ds_grp + aoff[i], a_img + (i * 4 + w) * 1024);
      const int key = t * 32 + srow[i];
      const int kc = key < p.Sk ? key : p.Sk - 1;
      glds16_fa(kb + (int64_t)kc * p.ks[1] + scol[i], b_img + (i * 4 + w) * 1024);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int t = 0; t < min(nkt, NS - 1); ++t) issue(t);
  for (int t = 0; t < nkt; ++t) {
    dq_wait_after(min(nkt - 1 - t, NS - 2));  // step t landed (this wave's part); later steps stay in flight
    lds_barrier();                            // ... for every wave; slot (t - 1) % NS no longer read
    if (t + NS - 1 < nkt) issue(t + NS - 1);
    const char* a_img = smem + (t % NS) * 2 * TB;
    const char* b_img = a_img + TB;
    Frag af[4], bf[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // A[q = row][keys 8c..8c+7], c = lane >> 4
      const int row = wm * 64 + i * 16 + (lane & 15);
      af[i].u = lds_b128(a_img, row * 64 + (((lane >> 4) ^ (((row >> 3) & 1) << 1)) << 4));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = dq_frag(b_img, wn * 64 + j * 16, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16<F16>(bf[j], af[i], acc[i][j]);
  }
  // lane: query q0 + 64wm + 16i + (lane & 15), d = 64wn + 16j + 4(lane >> 4) .. +3
  uint16_t* dqb = p.dq + (int64_t)b * p.dqs[0] + (int64_t)h * p.dqs[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = q0 + wm * 64 + i * 16 + (lane & 15);
    if (q >= p.Sq) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int d = wn * 64 + j * 16 + 4 * (lane >> 4);
      uint2 o;
      o.x = pack2<F16>(acc[i][j][0] * p.scale, acc[i][j][1] * p.scale);
      o.y = pack2<F16>(acc[i][j][2] * p.scale, acc[i][j][3] * p.scale);
      *reinterpret_cast<uint2*>(dqb + (int64_t)q * p.dqs[1] + d) = o;
    }
  }
}

// ---- launch helpers (one instantiation set per 16-bit type: flash_attn.hip = bf16, flash_attn_f16.hip = fp16)
template <int D, bool F16, int MW>
void fa_fwd_feat(const FwdArgs& a, int feat, dim3 grid, hipStream_t st) {
  switch (feat) {
    case 0: hipLaunchKernelGGL((fa_fwd_kernel<D, F16, MW, 0>), grid, dim3(256), 0, st, a); break;
    case 1: hipLaunchKernelGGL((fa_fwd_kernel<D, F16, MW, 1>), grid, dim3(256), 0, st, a); break;
    case 2: hipLaunchKernelGGL((fa_fwd_kernel<D, F16, MW, 2>), grid, dim3(256), 0, st, a); break;
    case 4: hipLaunchKernelGGL((fa_fwd_kernel<D, F16, MW, 4>), grid, dim3(256), 0, st, a); break;
    case 5: hipLaunchKernelGGL((fa_fwd_kernel<D, F16, MW, 5>), grid, dim3(256), 0, st, a); break;
    case 6: hipLaunchKernelGGL((fa_fwd_kernel<D, F16, MW, 6>), grid, dim3(256), 0, st, a); break;
    case 8: hipLaunchKernelGGL((fa_fwd_kernel<D, F16, MW, 8>), grid, dim3(256), 0, st, a); break;
    case 12: hipLaunchKernelGGL((fa_fwd_kernel<D, F16, MW, 12>), grid, dim3(256), 0, st, a); break;
    case 16: hipLaunchKernelGGL((fa_fwd_kernel<D, F16, MW, 16>), grid, dim3(256), 0, st, a); break;
    case 20: hipLaunchKernelGGL((fa_fwd_kernel<D, F16, MW, 20>), grid, dim3(256), 0, st, a); break;
    default: break;
  }
}

template <bool F16>
void fa_fwd_dispatch(const FwdArgs& a, int D, int feat, dim3 grid, hipStream_t st) {
  if (D == 128) fa_fwd_feat<128, F16, 2>(a, feat, grid, st);
  else if (D == 64) fa_fwd_feat<64, F16, 2>(a, feat, grid, st);
  else fa_fwd_feat<256, F16, 1>(a, feat, grid, st);
}

template <int D, bool F16, int NW, bool CK>
void fa_bwd_feat(const BwdArgs& a, int feat, dim3 grid, hipStream_t st) {
  switch (feat) {
    case 0: hipLaunchKernelGGL((fa_bwd_kernel<D, F16, NW, CK, 0>), grid, dim3(NW * 64), 0, st, a); break;
    case 1: hipLaunchKernelGGL((fa_bwd_kernel<D, F16, NW, CK, 1>), grid, dim3(NW * 64), 0, st, a); break;
    case 2: hipLaunchKernelGGL((fa_bwd_kernel<D, F16, NW, CK, 2>), grid, dim3(NW * 64), 0, st, a); break;
    case 4: hipLaunchKernelGGL((fa_bwd_kernel<D, F16, NW, CK, 4>), grid, dim3(NW * 64), 0, st, a); break;
    case 5: hipLaunchKernelGGL((fa_bwd_kernel<D, F16, NW, CK, 5>), grid, dim3(NW * 64), 0, st, a); break;
    case 6: hipLaunchKernelGGL((fa_bwd_kernel<D, F16, NW, CK, 6>), grid, dim3(NW * 64), 0, st, a); break;
    case 8: hipLaunchKernelGGL((fa_bwd_kernel<D, F16, NW, CK, 8>), grid, dim3(NW * 64), 0, st, a); break;
    case 12: hipLaunchKernelGGL((fa_bwd_kernel<D, F16, NW, CK, 12>), grid, dim3(NW * 64), 0, st, a); break;
    case 16: hipLaunchKernelGGL((fa_bwd_kernel<D, F16, NW, CK, 16>), grid, dim3(NW * 64), 0, st, a); break;
    case 20: hipLaunchKernelGGL((fa_bwd_kernel<D, F16, NW, CK, 20>), grid, dim3(NW * 64), 0, st, a); break;
    default: break;
  }
}

template <bool F16>
void fa_bwd_dispatch(const BwdArgs& a, int D, int feat, dim3 grid, hipStream_t st) {
  if (D == 128 && feat == 0 && a.ds != nullptr) {  // dS route (the caller checked eligibility)
    hipLaunchKernelGGL((fa_bwd16_kernel<F16, true>), grid, dim3(512), 0, st, a);
    const int nqb = (a.Sq + 127) / 128;
    hipLaunchKernelGGL((fa_bwd_dq_kernel<F16>), dim3((unsigned)(a.B * a.H * nqb)), dim3(256), 0, st, a);
    return;
  }
  if (D == 128 && feat == 0 && a.k16 && a.abl == 0) {
    hipLaunchKernelGGL((fa_bwd16_kernel<F16, false>), grid, dim3(512), 0, st, a);
    return;
  }
  if (D == 128) fa_bwd_feat<128, F16, 4, true>(a, feat, grid, st);
  else if (D == 64) fa_bwd_feat<64, F16, 4, true>(a, feat, grid, st);
  else fa_bwd_feat<256, F16, 2, false>(a, feat, grid, st);
}

template <bool F16>
void fa_bwd_aux(int which, const BwdArgs& a, const uint16_t* o, const uint16_t* dout, float* delta, const int64_t* os,
                const int64_t* dos, const float* dq_acc, uint16_t* dq, const int64_t* dqs, int DB, int DS, int H, int D,
                hipStream_t st) {
  if (which == 0) {
    const int64_t threads = (int64_t)DB * DS * H * (D / 8);
    hipLaunchKernelGGL(fa_bwd_delta<F16>, dim3((unsigned)cdiv(threads, 256)), dim3(256), 0, st, o, dout, delta, os[0],
                       os[1], os[2], dos[0], dos[1], dos[2], DB, DS, H, D, a.lse_s[0], a.lse_s[1]);
  } else {
    const int64_t nvec = (int64_t)DB * DS * H * D / 8;
    int64_t g = cdiv(nvec, 256);
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(fa_bwd_dq_convert<F16>, dim3((unsigned)g), dim3(256), 0, st, dq_acc, dq, dqs[0], dqs[1], dqs[2],
                       DB, DS, H, D);
  }
}

}  // namespace pa_fa
using namespace pa_fa;

// fp16 instantiations live in flash_attn_f16.hip
void pa_fa_fwd_f16(const FwdArgs& a, int D, int feat, dim3 grid, hipStream_t st);
void pa_fa_bwd_f16(const BwdArgs& a, int D, int feat, dim3 grid, hipStream_t st);
void pa_fa_bwd_aux_f16(int which, const BwdArgs& a, const uint16_t* o, const uint16_t* dout, float* delta,
                       const int64_t* os, const int64_t* dos, const float* dq_acc, uint16_t* dq, const int64_t* dqs,
                       int DB, int DS, int H, int D, hipStream_t st);
