// Flash attention forward + backward for gfx950 (CDNA4), bf16 in / fp32 accumulate.
// Reference behaviour: paddle/phi/kernels/gpu/flash_attn_kernel.cu / flash_attn_grad_kernel.cu
// (layout [batch, seq, heads, head_dim], causal = bottom-right aligned, GQA, LSE output).
//
// MFMA: v_mfma_f32_32x32x16_bf16 (lane l: r = l&31, h = l>>5;
//   A[row r][k 8h+j], B[k 8h+j][col r], D[row (i&3)+8(i>>2)+4h][col r]).
//
// Forward (per workgroup: 4 waves x 32 queries = 128-query block; K/V tiles of 64 keys in LDS):
//   S^T = K Q^T        -> the query is the MFMA column, so each lane owns one query and the row
//                         max / sum are in-lane (+ one xor-32 exchange), no LDS for P;
//   O^T += V^T P^T     -> the S^T accumulator is re-used directly as the B operand (bf16-packed),
//                         V^T comes from ds_read_b64_tr_b16 transposed LDS reads; O^T keeps the
//                         query on the lane, so the online-softmax rescale is per lane.
//   K/V of tile j+1 are prefetched into registers while tile j computes (async-stage split).
// Backward (per workgroup: 4 waves x 32 keys = 128-key block, loop over 32-query blocks):
//   S = Q K^T, P = exp(S - LSE), dP = dO V^T, dS = P (dP - delta);
//   dV^T += dO^T P and dK^T += Q^T dS with P / dS as B operands (no lane movement),
//   dQ += dS K via a bf16 dS^T tile in LDS, accumulated into fp32 with global atomics.
#include "common.h"

using namespace pa;

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

namespace {

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

__device__ __forceinline__ f32x16 mfma32(bf16x8_t a, bf16x8_t b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

union Frag {
  bf16x8_t v;
  uint4 u;
  s16x4 h[2];
};

// LDS byte offset of 16-byte chunk `ch` of row `row` in a [rows][NCH*8] bf16 image that serves
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
// memory ops in flight. __syncthreads() would also drain vmcnt, i.e. wait for the fire-and-forget dQ
// atomics of the previous query block at every step (they have no consumer inside the kernel).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Global loads the compiler does not track (see fa_bwd_kernel): the caller waits with a counted vmcnt.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4 gload16_async(const void* p) {
  u32x4 r;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return r;
}
__device__ __forceinline__ float gload4_async(const float* p) {
  float r;
  asm volatile("global_load_dword %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return r;
}

__device__ __forceinline__ uint4 lds_b128(const char* smem, int off) {
  return *reinterpret_cast<const uint4*>(smem + off);
}

__device__ __forceinline__ s16x4 lds_tr(const char* smem, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(reinterpret_cast<uintptr_t>(smem + off)));
}

__device__ __forceinline__ bf16x8_t pack8(const float* f) {
  Frag x;
  x.u.x = pack_bf16(f[0], f[1]);
  x.u.y = pack_bf16(f[2], f[3]);
  x.u.z = pack_bf16(f[4], f[5]);
  x.u.w = pack_bf16(f[6], f[7]);
  return x.v;
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

struct FwdArgs {
  const uint16_t* q; const uint16_t* k; const uint16_t* v; uint16_t* o; float* lse;
  int64_t qs[3], ks[3], vs[3], os[3];  // strides (batch, seq, head) in elements
  int B, Sq, Sk, H, Hk;
  float scale_log2;
  int causal;
  int grp;  // heads per dispatch group (block_map)
};

// ------------------------------------------------------------------------------------- forward
template <int D>
__global__ __launch_bounds__(256, 2) void fa_fwd_kernel(FwdArgs p) {
  constexpr int NCH = D / 8;       // 16-byte chunks per row
  constexpr int KS = D / 16;       // k-steps over head dim
  constexpr int NDT = D / 32;      // 32-wide output d tiles
  constexpr int BN = 64;           // keys per tile
  constexpr int TILE_BYTES = BN * D * 2;
  constexpr int LOADS = BN * NCH / 256;  // 16-byte chunks per thread per tensor
  __shared__ __attribute__((aligned(16))) char smem[2 * TILE_BYTES];
  char* ks_lds = smem;
  char* vs_lds = smem + TILE_BYTES;

  const int nqb = (p.Sq + 127) / 128;
  int bh, rank;
  block_map((int)blockIdx.x, p.B * p.H, nqb, p.grp, bh, rank);
  const int qb = p.causal ? (nqb - 1 - rank) : rank;
  const int b = bh / p.H, h = bh % p.H;
  const int hk = h / (p.H / p.Hk);
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 31, hf = lane >> 5;
  const int qi = qb * 128 + w * 32 + r;
  const int shift = p.Sk - p.Sq;

  // Q fragments (B operand of S^T = K Q^T): lane holds Q[qi][16ks + 8hf + j]
  bf16x8_t qf[KS];
  {
    const uint16_t* qrow = p.q + (int64_t)b * p.qs[0] + (int64_t)(qi < p.Sq ? qi : 0) * p.qs[1] + (int64_t)h * p.qs[2];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      Frag f;
      if (qi < p.Sq) f.u = *reinterpret_cast<const uint4*>(qrow + ks * 16 + hf * 8);
      else f.u = make_uint4(0, 0, 0, 0);
      qf[ks] = f.v;
    }
  }

  f32x16 oacc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) oacc[dt] = zero16();
  float m_run = -INFINITY, l_run = 0.f;

  int kv_end = p.Sk;
  if (p.causal) {
    const int last_q = min(qb * 128 + 127, p.Sq - 1);
    kv_end = min(p.Sk, last_q + shift + 1);
  }
  const int n_tiles = kv_end > 0 ? (kv_end + BN - 1) / BN : 0;

  const uint16_t* kbase = p.k + (int64_t)b * p.ks[0] + (int64_t)hk * p.ks[2];
  const uint16_t* vbase = p.v + (int64_t)b * p.vs[0] + (int64_t)hk * p.vs[2];

  uint4 kreg[LOADS], vreg[LOADS];
  auto gload = [&](int tile) {
    const int kv0 = tile * BN;
#pragma unroll
    for (int i = 0; i < LOADS; ++i) {
      const int idx = tid + 256 * i;
      const int row = idx / NCH, ch = idx % NCH;
      const int key = kv0 + row;
      if (key < p.Sk) {
        kreg[i] = *reinterpret_cast<const uint4*>(kbase + (int64_t)key * p.ks[1] + ch * 8);
        vreg[i] = *reinterpret_cast<const uint4*>(vbase + (int64_t)key * p.vs[1] + ch * 8);
      } else {
        kreg[i] = make_uint4(0, 0, 0, 0);
        vreg[i] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int i = 0; i < LOADS; ++i) {
      const int idx = tid + 256 * i;
      const int row = idx / NCH, ch = idx % NCH;
      *reinterpret_cast<uint4*>(ks_lds + img_off<NCH>(row, ch)) = kreg[i];
      *reinterpret_cast<uint4*>(vs_lds + img_off<NCH>(row, ch)) = vreg[i];
    }
  };

  if (n_tiles > 0) gload(0);
  for (int t = 0; t < n_tiles; ++t) {
    __syncthreads();  // previous tile's LDS reads are done
    lstore();
    __syncthreads();
    if (t + 1 < n_tiles) gload(t + 1);  // overlaps with the MFMA work below
    const int kv0 = t * BN;

    // ---- S^T = K Q^T for two 32-key sub-tiles
    f32x16 sacc[2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      sacc[kt] = zero16();
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        Frag a;
        a.u = lds_b128(ks_lds, img_off<NCH>(kt * 32 + r, 2 * ks + hf));
        sacc[kt] = mfma32(a.v, qf[ks], sacc[kt]);
      }
    }
    // ---- scale, mask, online softmax (log2 domain)
    float mloc = -INFINITY;
    const bool need_mask = (kv0 + BN > p.Sk) || (p.causal && (kv0 + BN - 1 > qb * 128 + shift));
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float s = sacc[kt][i] * p.scale_log2;
        if (need_mask) {
          const int kj = kv0 + kt * 32 + (i & 3) + 8 * (i >> 2) + 4 * hf;
          if (kj >= p.Sk || (p.causal && kj > qi + shift)) s = -INFINITY;
        }
        sacc[kt][i] = s;
        mloc = fmaxf(mloc, s);
      }
    }
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
    const float m_new = fmaxf(m_run, mloc);
    const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_use);
    float psum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float e = __builtin_amdgcn_exp2f(sacc[kt][i] - m_use);
        sacc[kt][i] = e;
        psum += e;
      }
    }
    l_run = l_run * alpha + psum;
    m_run = m_new;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) oacc[dt][i] *= alpha;

    // ---- P^T as bf16 B fragments: fragment s of sub-tile kt = regs 8s..8s+7
    bf16x8_t pf[2][2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float tmp[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) tmp[j] = sacc[kt][8 * s + j];
        pf[kt][s] = pack8(tmp);
      }

    // ---- O^T += V^T P^T (A = V^T via transposed LDS reads)
    const int gi = lane & 15, qq = gi >> 2, pp = gi & 3, G1 = (lane >> 4) & 1;
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
          oacc[dt] = mfma32(a.v, pf[kt][s], oacc[dt]);
        }
      }
    }
  }

  // ---- epilogue
  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if (qi < p.Sq) {
    uint16_t* orow = p.o + (int64_t)b * p.os[0] + (int64_t)qi * p.os[1] + (int64_t)h * p.os[2];
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d0 = dt * 32 + 8 * g + 4 * hf;
        uint2 v2;
        v2.x = pack_bf16(oacc[dt][4 * g + 0] * inv, oacc[dt][4 * g + 1] * inv);
        v2.y = pack_bf16(oacc[dt][4 * g + 2] * inv, oacc[dt][4 * g + 3] * inv);
        *reinterpret_cast<uint2*>(orow + d0) = v2;
      }
    }
    if (hf == 0) {
      const float lse = (m_run == -INFINITY) ? INFINITY : (m_run * kLn2 + __logf(l_tot));
      p.lse[((int64_t)b * p.H + h) * p.Sq + qi] = lse;
    }
  }
}

// ------------------------------------------------------------------------------------- forward v2
// Same math and lane layout as fa_fwd_kernel; the data movement and softmax bookkeeping differ:
//   * K/V tiles go global -> LDS by global_load_lds (no register round trip, no VALU for the LDS
//     writes). glds writes LDS lane-linearly, so the image swizzle is applied to the per-lane global
//     source chunk (ch = slot ^ swizzle(row)); the image is the same one img_off() addresses.
//   * Two LDS stages: tile t+1 is fetched while tile t computes, one barrier per tile.
//   * Deferred rescale: the running max (reference for exp2) is only raised when a tile's max exceeds
//     it by more than 2^8 (in exp2 units); otherwise P values up to 256 are accumulated against the
//     stale reference. The 64 O-accumulator multiplies then run on a few tiles per row, not all.
//   * The softmax scale is folded into the exp2 argument: p = exp2(s * c - m * c), one FMA per score,
//     and the max is taken on raw scores.
__device__ __forceinline__ void glds16_fa(const void* g, const char* lds) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uintptr_t>(lds));
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m0) : "memory", "m0");
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int D>
__global__ __launch_bounds__(256, 2) void fa_fwd2_kernel(FwdArgs p) {
  constexpr int NCH = D / 8;
  constexpr int KS = D / 16;
  constexpr int NDT = D / 32;
  constexpr int BN = 64;
  constexpr int TILE_BYTES = BN * D * 2;
  constexpr int NI = TILE_BYTES / 1024 / 4;  // glds per wave per tensor per tile
  constexpr float kDefer = 8.f;              // log2 of the largest accepted P before a rescale
  __shared__ __attribute__((aligned(1024))) char smem[4 * TILE_BYTES];  // [stage][K | V]

  const int nqb = (p.Sq + 127) / 128;
  int bh, rank;
  block_map((int)blockIdx.x, p.B * p.H, nqb, p.grp, bh, rank);
  const int qb = p.causal ? (nqb - 1 - rank) : rank;
  const int b = bh / p.H, h = bh % p.H;
  const int hk = h / (p.H / p.Hk);
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 31, hf = lane >> 5;
  const int qi = qb * 128 + w * 32 + r;
  const int shift = p.Sk - p.Sq;
  const float c = p.scale_log2;

  bf16x8_t qf[KS];
  {
    const uint16_t* qrow = p.q + (int64_t)b * p.qs[0] + (int64_t)(qi < p.Sq ? qi : 0) * p.qs[1] + (int64_t)h * p.qs[2];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      Frag f;
      if (qi < p.Sq) f.u = *reinterpret_cast<const uint4*>(qrow + ks * 16 + hf * 8);
      else f.u = make_uint4(0, 0, 0, 0);
      qf[ks] = f.v;
    }
  }

  f32x16 oacc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) oacc[dt] = zero16();
  float m_run = -INFINITY, l_run = 0.f;

  int kv_end = p.Sk;
  if (p.causal) {
    const int last_q = min(qb * 128 + 127, p.Sq - 1);
    kv_end = min(p.Sk, last_q + shift + 1);
  }
  const int n_tiles = kv_end > 0 ? (kv_end + BN - 1) / BN : 0;

  const uint16_t* kbase = p.k + (int64_t)b * p.ks[0] + (int64_t)hk * p.ks[2];
  const uint16_t* vbase = p.v + (int64_t)b * p.vs[0] + (int64_t)hk * p.vs[2];

  // this lane's (row, chunk) in each of its NI 1-KiB pieces (tile independent)
  auto issue = [&](int tile, int stage) {
    const char* kdst = smem + stage * 2 * TILE_BYTES;
    const char* vdst = kdst + TILE_BYTES;
    const int kv0 = tile * BN;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = w * NI + i;
      const int o = q * 1024 + lane * 16;
      const int row = o / (NCH * 16), slot = (o % (NCH * 16)) / 16;
      const int ch = (img_off<NCH>(row, slot) - row * (NCH * 16)) / 16;  // slot ^ swizzle(row)
      int key = kv0 + row;
      key = key < p.Sk ? key : p.Sk - 1;  // rows past the end are masked to -inf below
      glds16_fa(kbase + (int64_t)key * p.ks[1] + ch * 8, kdst + q * 1024);
      glds16_fa(vbase + (int64_t)key * p.vs[1] + ch * 8, vdst + q * 1024);
    }
  };

  const int gi = lane & 15, qq = gi >> 2, pp = gi & 3, G1 = (lane >> 4) & 1;
  if (n_tiles > 0) issue(0, 0);
  for (int t = 0; t < n_tiles; ++t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of tile t are in LDS
    raw_barrier();                                     // ... everyone's, and stage (t+1)&1 is free
    if (t + 1 < n_tiles) issue(t + 1, (t + 1) & 1);
    const char* ks_lds = smem + (t & 1) * 2 * TILE_BYTES;
    const char* vs_lds = ks_lds + TILE_BYTES;
    const int kv0 = t * BN;

    f32x16 sacc[2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      sacc[kt] = zero16();
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        Frag a;
        a.u = lds_b128(ks_lds, img_off<NCH>(kt * 32 + r, 2 * ks + hf));
        sacc[kt] = mfma32(a.v, qf[ks], sacc[kt]);
      }
    }
    float mloc = -INFINITY;
    const bool need_mask = (kv0 + BN > p.Sk) || (p.causal && (kv0 + BN - 1 > qb * 128 + shift));
    if (need_mask) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int kj = kv0 + kt * 32 + (i & 3) + 8 * (i >> 2) + 4 * hf;
          if (kj >= p.Sk || (p.causal && kj > qi + shift)) sacc[kt][i] = -INFINITY;
        }
    }
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

    bf16x8_t pf[2][2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float tmp[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) tmp[j] = sacc[kt][8 * s + j];
        pf[kt][s] = pack8(tmp);
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
          oacc[dt] = mfma32(a.v, pf[kt][s], oacc[dt]);
        }
      }
    }
  }

  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if (qi < p.Sq) {
    uint16_t* orow = p.o + (int64_t)b * p.os[0] + (int64_t)qi * p.os[1] + (int64_t)h * p.os[2];
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d0 = dt * 32 + 8 * g + 4 * hf;
        uint2 v2;
        v2.x = pack_bf16(oacc[dt][4 * g + 0] * inv, oacc[dt][4 * g + 1] * inv);
        v2.y = pack_bf16(oacc[dt][4 * g + 2] * inv, oacc[dt][4 * g + 3] * inv);
        *reinterpret_cast<uint2*>(orow + d0) = v2;
      }
    }
    if (hf == 0) {
      const float lse = (m_run == -INFINITY) ? INFINITY : (m_run * c * kLn2 + __logf(l_tot));
      p.lse[((int64_t)b * p.H + h) * p.Sq + qi] = lse;
    }
  }
}

// ------------------------------------------------------------------------------------- backward
struct BwdArgs {
  const uint16_t* q; const uint16_t* k; const uint16_t* v; const uint16_t* o; const uint16_t* dout;
  const float* lse; float* dq_acc; const float* delta; uint16_t* dk; uint16_t* dv;
  int64_t qs[3], ks[3], vs[3], dos[3], dks[3], dvs[3];
  int B, Sq, Sk, H, Hk;
  float scale, scale_log2;
  int causal;
  int grp;
};

// delta[b,h,q] = sum_d dO * O
__global__ __launch_bounds__(256) void fa_bwd_delta(const uint16_t* __restrict__ o, const uint16_t* __restrict__ dout,
                                                    float* __restrict__ delta, int64_t o_sb, int64_t o_ss, int64_t o_sh,
                                                    int64_t d_sb, int64_t d_ss, int64_t d_sh, int B, int Sq, int H, int D) {
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
    float a[8], g[8];
    load8<bf16>((const bf16*)(o + bb * o_sb + qq * o_ss + hh * o_sh + c * 8), a);
    load8<bf16>((const bf16*)(dout + bb * d_sb + qq * d_ss + hh * d_sh + c * 8), g);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j] * g[j];
  }
  for (int off = per_row / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (row < nrows && c == 0) delta[((int64_t)bb * H + hh) * Sq + qq] = s;
}

// dq[b,q,h,:] (bf16, strided) = dq_acc[b,q,h,:] (fp32, contiguous [B,Sq,H,D])
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
    store8<bf16>((bf16*)(dq + bb * s_b + qq * s_s + hh * s_h + d), v);
  }
}

template <int D>
__global__ __launch_bounds__(256, 1) void fa_bwd_kernel(BwdArgs p) {
  constexpr int NCH = D / 8;
  constexpr int KS = D / 16;
  constexpr int NDT = D / 32;
  constexpr int BK = 128;  // keys per workgroup (4 waves x 32)
  constexpr int BM = 32;   // queries per inner step
  constexpr int KT_BYTES = BK * D * 2;
  constexpr int QT_BYTES = BM * D * 2;
  constexpr int DST_BYTES = BK * BM * 2;  // dS^T [128 keys][32 q] bf16, 64-byte rows
  __shared__ __attribute__((aligned(16))) char smem[2 * KT_BYTES + 2 * QT_BYTES + 2 * DST_BYTES + 2 * BM * 4];
  char* k_lds = smem;
  char* v_lds = smem + KT_BYTES;
  char* q_lds = v_lds + KT_BYTES;
  char* do_lds = q_lds + QT_BYTES;
  char* ds_lds = do_lds + QT_BYTES;
  float* lse_s = reinterpret_cast<float*>(ds_lds + 2 * DST_BYTES);  // ds_lds: two dS^T buffers
  float* dlt_s = lse_s + BM;

  int kb, bh;  // key block 0 is the heaviest under the causal mask: rank order
  block_map((int)blockIdx.x, p.B * p.H, (p.Sk + 127) / 128, p.grp, bh, kb);
  const int b = bh / p.H, h = bh % p.H;
  const int hk = h / (p.H / p.Hk);
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 31, hf = lane >> 5;
  const int gi = lane & 15, qq = gi >> 2, pp = gi & 3, G1 = (lane >> 4) & 1;
  const int shift = p.Sk - p.Sq;
  const int kj = kb * BK + w * 32 + r;  // this lane's key (MFMA column)

  // K tile -> LDS (row image, also read transposed for dQ)
  const uint16_t* kbase = p.k + (int64_t)b * p.ks[0] + (int64_t)hk * p.ks[2];
  const uint16_t* vbase = p.v + (int64_t)b * p.vs[0] + (int64_t)hk * p.vs[2];
#pragma unroll
  for (int i = 0; i < BK * NCH / 256; ++i) {
    const int idx = tid + 256 * i;
    const int row = idx / NCH, ch = idx % NCH;
    const int key = kb * BK + row;
    uint4 val = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
    if (key < p.Sk) {
      val = *reinterpret_cast<const uint4*>(kbase + (int64_t)key * p.ks[1] + ch * 8);
      vv = *reinterpret_cast<const uint4*>(vbase + (int64_t)key * p.vs[1] + ch * 8);
    }
    *reinterpret_cast<uint4*>(k_lds + img_off<NCH>(row, ch)) = val;
    *reinterpret_cast<uint4*>(v_lds + img_off<NCH>(row, ch)) = vv;
  }

  f32x16 dk_acc[NDT], dv_acc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) { dk_acc[dt] = zero16(); dv_acc[dt] = zero16(); }

  // This lane's K / V rows as MFMA B fragments, loaded once: they are the same for every query
  // block, so the S / dP chains below read only Q / dO from LDS (half the LDS traffic of that phase).
  __syncthreads();
  bf16x8_t kfr[KS], vfr[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    Frag kb8, vb8;
    kb8.u = lds_b128(k_lds, img_off<NCH>(w * 32 + r, 2 * ks + hf));
    vb8.u = lds_b128(v_lds, img_off<NCH>(w * 32 + r, 2 * ks + hf));
    kfr[ks] = kb8.v;
    vfr[ks] = vb8.v;
  }

  // query range that sees any key of this block
  int q_begin = 0;
  if (p.causal) q_begin = max(0, kb * BK - shift);
  q_begin = (q_begin / BM) * BM;
  const uint16_t* qbase = p.q + (int64_t)b * p.qs[0] + (int64_t)h * p.qs[2];
  const uint16_t* dobase = p.dout + (int64_t)b * p.dos[0] + (int64_t)h * p.dos[2];
  const float* lse_b = p.lse + ((int64_t)b * p.H + h) * p.Sq;
  const float* dlt_b = p.delta + ((int64_t)b * p.H + h) * p.Sq;
  float* dqb = p.dq_acc + (int64_t)b * p.Sq * p.H * D + (int64_t)h * D;  // contiguous [B,Sq,H,D]

  // Q / dO / LSE / delta of the next query block are prefetched into registers while the current
  // block computes (async-stage split): the HBM latency is hidden behind ~40 MFMAs per wave.
  constexpr int QLOADS = BM * NCH / 256;
  u32x4 qreg[QLOADS], dreg[QLOADS];
  float lse_r = -INFINITY, dlt_r = 0.f;
  const float inv_scale = 1.f / p.scale;
  // dQ accumulator of this (b, h) as a buffer resource: 32-bit offsets, no 64-bit address math per atomic
  const __amdgpu_buffer_rsrc_t dq_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      dqb, 0, (int)((int64_t)(p.Sq - 1) * p.H * D * 4 + D * 4), 0x00020000);
  // The prefetch loads are issued from inline asm so that hipcc does not track them: at the loop top the
  // kernel waits with a counted vmcnt that leaves the previous block's 16 fire-and-forget dQ atomics
  // (issued after these loads) in flight, instead of the vmcnt(0) the compiler would emit.
  // Loads are unconditional (rows clamped into range, zeroed after the wait): an asm result written
  // under a divergent branch could be merged by a register copy before the data has arrived.
  float lse_raw = 0.f, dlt_raw = 0.f;
  bool row_ok = false;
  bool q_ok[QLOADS];
  auto prefetch = [&](int q0) {
#pragma unroll
    for (int i = 0; i < QLOADS; ++i) {
      const int idx = tid + 256 * i;
      const int row = idx / NCH, ch = idx % NCH;
      const int qx = q0 + row;
      q_ok[i] = qx < p.Sq;
      const int qc = q_ok[i] ? qx : p.Sq - 1;
      qreg[i] = gload16_async(qbase + (int64_t)qc * p.qs[1] + ch * 8);
      dreg[i] = gload16_async(dobase + (int64_t)qc * p.dos[1] + ch * 8);
    }
    const int qx = q0 + (tid & (BM - 1));
    row_ok = qx < p.Sq;
    const int qc = row_ok ? qx : p.Sq - 1;
    lse_raw = gload4_async(lse_b + qc);
    dlt_raw = gload4_async(dlt_b + qc);
  };
  if (q_begin < p.Sq) prefetch(q_begin);
  const bool has_atomics = w < NDT;  // waves that own a dQ d-tile issue 16 atomics per block

  // dQ[q][d] += sum_key dS[q][key] K[key][d] for the query block whose dS^T is in `dsb`; wave w handles
  // d tiles dt = w, w+4, ... Software-pipelined by one block: block i's dQ runs in iteration i+1 (after
  // that iteration's second barrier), so no barrier is needed between the dS^T store and its reads.
  auto dq_step = [&](const char* dsb, int qb0) {
    for (int dt = w; dt < NDT; dt += 4) {
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
        qacc = mfma32(a.v, bb.v, qacc);
      }
      if (p.causal >= 0) {
        // byte offsets into this (b, h)'s dQ rows (row stride H*D floats); out-of-range rows
        // (ragged last block) fall outside the buffer resource and are dropped by the hardware
        const int rs = p.H * D * 4;
        const int base = qb0 * rs + (dt * 32 + r) * 4;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int qr = (i & 3) + 8 * (i >> 2) + 4 * hf;
          const int off = (qb0 + qr < p.Sq) ? base + qr * rs : 0x7ffffff0;
          __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(qacc[i] * p.scale, dq_rsrc, off, 0, 0);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) asm volatile("" ::"v"(qacc[i]));
      }
    }
    };

  for (int q0 = q_begin; q0 < p.Sq; q0 += BM) {
    if (q0 == q_begin || !has_atomics) {
      asm volatile("s_waitcnt vmcnt(0)" : "+v"(qreg[0]), "+v"(dreg[0]), "+v"(lse_raw), "+v"(dlt_raw)::"memory");
    } else {
      asm volatile("s_waitcnt vmcnt(16)" : "+v"(qreg[0]), "+v"(dreg[0]), "+v"(lse_raw), "+v"(dlt_raw)::"memory");
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
    lse_r = row_ok ? -lse_raw * inv_scale : -INFINITY;
    dlt_r = row_ok ? -dlt_raw : 0.f;
    lds_barrier();  // previous iteration's LDS reads done
#pragma unroll
    for (int i = 0; i < QLOADS; ++i) {
      const int idx = tid + 256 * i;
      const int row = idx / NCH, ch = idx % NCH;
      *reinterpret_cast<u32x4*>(q_lds + img_off<NCH>(row, ch)) = qreg[i];
      *reinterpret_cast<u32x4*>(do_lds + img_off<NCH>(row, ch)) = dreg[i];
    }
    if (tid < BM) {
      lse_s[tid] = lse_r;
      dlt_s[tid] = dlt_r;
    }
    lds_barrier();
    if (q0 + BM < p.Sq) prefetch(q0 + BM);
    if (q0 > q_begin) dq_step(ds_lds + ((((q0 - q_begin) / BM - 1) & 1) * DST_BYTES), q0 - BM);

    // S' = Q K^T - LSE/scale and dP' = dO V^T - delta : rows q (registers), cols = this lane's key.
    // Row constants for this lane's 16 query rows (8g + 4hf + 0..3): 4 x 16-byte LDS reads each.
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
      sacc = mfma32(qa.v, kfr[ks], sacc);
      pacc = mfma32(da.v, vfr[ks], pacc);
    }
    // P and dS computed in place, then packed straight into bf16 MFMA fragments.
    const bool need_mask = kj >= p.Sk || (p.causal && kb * BK + BK - 1 > q0 + shift);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int qr = (i & 3) + 8 * (i >> 2) + 4 * hf;
      float pr = __builtin_amdgcn_exp2f(sacc[i] * p.scale_log2);
      if (need_mask && (kj >= p.Sk || (p.causal && kj > q0 + qr + shift))) pr = 0.f;
      sacc[i] = pr;
      pacc[i] = pr * pacc[i];
    }
    bf16x8_t pf[2], sf[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float a[8], c[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { a[j] = sacc[8 * s + j]; c[j] = pacc[8 * s + j]; }
      pf[s] = pack8(a);
      sf[s] = pack8(c);
    }

    // dV^T += dO^T P ; dK^T += Q^T dS  (A via transposed reads of the dO / Q images)
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      const int cch = (dt * 32 + 16 * G1) / 8 + (pp >> 1);
      const int cb = 8 * (pp & 1);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int R0 = 16 * s + 4 * hf;
        Frag a, c;
        a.h[0] = lds_tr(do_lds, img_off<NCH>(R0 + qq, cch) + cb);
        a.h[1] = lds_tr(do_lds, img_off<NCH>(R0 + 8 + qq, cch) + cb);
        dv_acc[dt] = mfma32(a.v, pf[s], dv_acc[dt]);
        c.h[0] = lds_tr(q_lds, img_off<NCH>(R0 + qq, cch) + cb);
        c.h[1] = lds_tr(q_lds, img_off<NCH>(R0 + 8 + qq, cch) + cb);
        dk_acc[dt] = mfma32(c.v, sf[s], dk_acc[dt]);
      }
    }

    // dS^T tile [128 keys][32 q] bf16: lane writes its key row, 4 consecutive q per 8-byte store.
    // 64-byte rows: the 8-byte column slot is XORed with (row >> 2) & 3 so that the 16 rows of a
    // store's lane group land on distinct banks (rows r, r+4, r+8, r+12 would collide otherwise).
    {
      // fragment s, elements 0..3 = q 16s+4hf+0..3, elements 4..7 = q 16s+8+4hf+0..3
      const int row = w * 32 + r;
      char* rowp = ds_lds + (((q0 - q_begin) / BM) & 1) * DST_BYTES + row * (BM * 2);
      const int sw = ((row >> 2) & 3) << 3;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        Frag f;
        f.v = sf[s];
        *reinterpret_cast<uint2*>(rowp + (((16 * s + 4 * hf) * 2) ^ sw)) = make_uint2(f.u.x, f.u.y);
        *reinterpret_cast<uint2*>(rowp + (((16 * s + 8 + 4 * hf) * 2) ^ sw)) = make_uint2(f.u.z, f.u.w);
      }
    }
  }
  // dQ of the last query block
  if (q_begin < p.Sq) {
    lds_barrier();
    const int q_last = q_begin + ((p.Sq - 1 - q_begin) / BM) * BM;
    dq_step(ds_lds + ((((q_last - q_begin) / BM) & 1) * DST_BYTES), q_last);
  }

  // write dK = scale * (dK^T)^T, dV = (dV^T)^T : lane = key, 4 consecutive d per 8-byte store
  if (kj < p.Sk) {
    uint16_t* dkrow = p.dk + (int64_t)b * p.dks[0] + (int64_t)kj * p.dks[1] + (int64_t)h * p.dks[2];
    uint16_t* dvrow = p.dv + (int64_t)b * p.dvs[0] + (int64_t)kj * p.dvs[1] + (int64_t)h * p.dvs[2];
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d0 = dt * 32 + 8 * g + 4 * hf;
        uint2 a, c;
        a.x = pack_bf16(dk_acc[dt][4 * g] * p.scale, dk_acc[dt][4 * g + 1] * p.scale);
        a.y = pack_bf16(dk_acc[dt][4 * g + 2] * p.scale, dk_acc[dt][4 * g + 3] * p.scale);
        c.x = pack_bf16(dv_acc[dt][4 * g], dv_acc[dt][4 * g + 1]);
        c.y = pack_bf16(dv_acc[dt][4 * g + 2], dv_acc[dt][4 * g + 3]);
        *reinterpret_cast<uint2*>(dkrow + d0) = a;
        *reinterpret_cast<uint2*>(dvrow + d0) = c;
      }
    }
  }
}

}  // namespace

// heads per dispatch group for block_map: all of an XCD's heads at once (global heaviest-first) while that
// is at most 512 workgroups per XCD, else groups that keep ~`inflight` workgroups (2 per CU forward, 1
// backward) on a few heads for L2 reuse of their K/V (or Q/dO); 0 (plain head-fastest order) when B*H is
// not a multiple of 8.
static int fa_group(int BH, int nb, int inflight) {
  if (BH % 8 != 0) return 0;
  const int hpx = BH / 8;
  if (hpx * nb <= 512) return hpx;
  return std::max(1, (inflight + nb - 1) / nb);
}

static int g_fwd_variant = 2;  // 1: register-staged single-buffer kernel, 2: fa_fwd2_kernel

// A/B switch for the microbenchmarks
PA_EXPORT int pa_flash_attn_set_fwd_variant(int v) {
  g_fwd_variant = v;
  return 0;
}

// strides: host array of 12 int64 = q(b,s,h), k(b,s,h), v(b,s,h), o(b,s,h)
PA_EXPORT int pa_flash_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse,
                                const int64_t* strides, int B, int Sq, int Sk, int H, int Hk, int D, float scale,
                                int causal, hipStream_t st) {
  if (H % Hk != 0) return 3;
  FwdArgs a;
  a.q = (const uint16_t*)q; a.k = (const uint16_t*)k; a.v = (const uint16_t*)v; a.o = (uint16_t*)o; a.lse = lse;
  for (int i = 0; i < 3; ++i) {
    a.qs[i] = strides[i]; a.ks[i] = strides[3 + i]; a.vs[i] = strides[6 + i]; a.os[i] = strides[9 + i];
  }
  a.B = B; a.Sq = Sq; a.Sk = Sk; a.H = H; a.Hk = Hk;
  a.scale_log2 = scale * kLog2e;
  a.causal = causal;
  const int nqb = (Sq + 127) / 128;
  a.grp = fa_group(B * H, nqb, 64);
  dim3 grid((unsigned)(B * H * nqb));
  if (D != 128 && D != 64) return 4;
  if (g_fwd_variant == 2) {
    if (D == 128) hipLaunchKernelGGL(fa_fwd2_kernel<128>, grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(fa_fwd2_kernel<64>, grid, dim3(256), 0, st, a);
  } else {
    if (D == 128) hipLaunchKernelGGL(fa_fwd_kernel<128>, grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(fa_fwd_kernel<64>, grid, dim3(256), 0, st, a);
  }
  PA_CHECK_LAUNCH();
  return 0;
}

// strides: host array of 24 int64 = q, k, v, o, do, dq, dk, dv  (each b,s,h)
PA_EXPORT int pa_flash_attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout,
                                const float* lse, void* dq, void* dk, void* dv, float* dq_acc, float* delta,
                                const int64_t* strides, int B, int Sq, int Sk, int H, int Hk, int D, float scale,
                                int causal, hipStream_t st) {
  if (H % Hk != 0) return 3;
  if (D != 128 && D != 64) return 4;
  const int64_t* qs = strides; const int64_t* ks = strides + 3; const int64_t* vs = strides + 6;
  const int64_t* os = strides + 9; const int64_t* dos = strides + 12; const int64_t* dqs = strides + 15;
  const int64_t* dks = strides + 18; const int64_t* dvs = strides + 21;
  // delta = rowsum(dO * O)
  {
    const int64_t threads = (int64_t)B * Sq * H * (D / 8);
    hipLaunchKernelGGL(fa_bwd_delta, dim3((unsigned)cdiv(threads, 256)), dim3(256), 0, st, (const uint16_t*)o,
                       (const uint16_t*)dout, delta, os[0], os[1], os[2], dos[0], dos[1], dos[2], B, Sq, H, D);
    PA_CHECK_LAUNCH();
  }
  hipMemsetAsync(dq_acc, 0, (size_t)B * Sq * H * D * sizeof(float), st);
  BwdArgs a;
  a.q = (const uint16_t*)q; a.k = (const uint16_t*)k; a.v = (const uint16_t*)v; a.o = (const uint16_t*)o;
  a.dout = (const uint16_t*)dout; a.lse = lse; a.dq_acc = dq_acc; a.delta = delta;
  a.dk = (uint16_t*)dk; a.dv = (uint16_t*)dv;
  for (int i = 0; i < 3; ++i) {
    a.qs[i] = qs[i]; a.ks[i] = ks[i]; a.vs[i] = vs[i]; a.dos[i] = dos[i]; a.dks[i] = dks[i]; a.dvs[i] = dvs[i];
  }
  a.B = B; a.Sq = Sq; a.Sk = Sk; a.H = H; a.Hk = Hk;
  a.scale = scale; a.scale_log2 = scale * kLog2e; a.causal = causal;
  const int nkb = (Sk + 127) / 128;
  a.grp = fa_group(B * H, nkb, 32);
  dim3 grid((unsigned)(B * H * nkb));
  if (D == 128) hipLaunchKernelGGL(fa_bwd_kernel<128>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(fa_bwd_kernel<64>, grid, dim3(256), 0, st, a);
  PA_CHECK_LAUNCH();
  {
    const int64_t nvec = (int64_t)B * Sq * H * D / 8;
    int64_t g = cdiv(nvec, 256);
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(fa_bwd_dq_convert, dim3((unsigned)g), dim3(256), 0, st, dq_acc, (uint16_t*)dq, dqs[0], dqs[1],
                       dqs[2], B, Sq, H, D);
    PA_CHECK_LAUNCH();
  }
  return 0;
}

// ablation hook (timing only): causal flag -1/-2 skips the dQ atomics
PA_EXPORT int pa_flash_attn_bwd_ablate(const void* q, const void* k, const void* v, const void* o, const void* dout,
                                       const float* lse, void* dq, void* dk, void* dv, float* dq_acc, float* delta,
                                       const int64_t* strides, int B, int Sq, int Sk, int H, int Hk, int D,
                                       float scale, int causal, hipStream_t st) {
  return pa_flash_attn_bwd(q, k, v, o, dout, lse, dq, dk, dv, dq_acc, delta, strides, B, Sq, Sk, H, Hk, D, scale,
                           causal, st);
}
