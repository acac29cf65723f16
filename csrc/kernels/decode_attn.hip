// Paged-KV decode attention (one new query token per sequence) for gfx950, bf16 cache / fp32 math.
// Reference behaviour: paddle/phi/kernels/fusion/gpu/block_attn.h (block_multihead_attention decode
// path) and masked_multihead_attention_kernel.cu.
//
// Decode is a KV-cache stream: per (sequence, kv head) the kernel reads every cached key and value
// once. To fill 256 CUs even at small batch, the key range is split across workgroups
// (flash-decoding): grid = (seq, kv head, split); each workgroup runs an online softmax over its
// blocks for ALL query heads of the GQA group (K/V bytes are read once for the group), writes a
// partial (m, l, o); a second tiny kernel merges the splits.
//
// Work split inside a workgroup (256 threads = 4 waves): the split's keys go to the waves in 16-key
// chunks, round-robin; within the wave 16 lanes cover one key's D = 128 elements (8 bf16 each, one
// 16-byte load), so a wave-instruction covers 4 keys and a chunk is 4 of them (8 loads in flight per
// lane). Dot products reduce over the 16 lanes with 4 xor-shuffles.
#include "common.h"

using namespace pa;

namespace {

constexpr int kLanesPerKey = 16;

template <int D, int G>
__global__ __launch_bounds__(256) void paged_decode_k(const uint16_t* __restrict__ q,      // [N, H, D]
                                                       const uint16_t* __restrict__ kc,     // [nb, Hkv, bs, D]
                                                       const uint16_t* __restrict__ vc,
                                                       const int* __restrict__ tables,     // [N, max_blocks]
                                                       const int* __restrict__ lens,       // [N]
                                                       float* __restrict__ part_o,         // [N, H, S, D]
                                                       float* __restrict__ part_ml,        // [N, H, S, 2]
                                                       uint16_t* __restrict__ out,         // [N, H, D] (splits 1)
                                                       int H, int Hkv, int bs, int max_blocks, int splits,
                                                       int64_t blk_stride, int64_t head_stride,
                                                       float scale_log2) {
  static_assert(D == 128, "decode kernel is specialised for head_dim 128");
  constexpr int EPL = D / kLanesPerKey;  // 8 elements per lane
  const int n = blockIdx.x, hk = blockIdx.y, sp = blockIdx.z;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int sub = lane >> 4;            // which of the wave's 4 keys
  const int li = lane & 15;             // position inside the key's 16 lanes
  const int len = lens[n];
  const int nblk = (len + bs - 1) / bs;
  const int per = (nblk + splits - 1) / splits;
  const int b0 = sp * per, b1 = min(nblk, b0 + per);

  // query rows of the group: lane holds elements [8 li, 8 li + 8) of each head
  float qv[G][EPL];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float f[8];
    load8<bf16>(reinterpret_cast<const bf16*>(q + ((int64_t)n * H + hk * G + g) * D + li * EPL), f);
#pragma unroll
    for (int j = 0; j < EPL; ++j) qv[g][j] = f[j] * scale_log2;
  }
  float m[G], l[G], o[G][EPL];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = -INFINITY;
    l[g] = 0.f;
#pragma unroll
    for (int j = 0; j < EPL; ++j) o[g][j] = 0.f;
  }

  // Keys of this split in 16-key chunks dealt round-robin to the 4 waves (balanced to one chunk); 4 keys
  // per 16-lane group per chunk, all 8 loads issued before the first use, and the online softmax rescales
  // once per 4 keys. A key's cache row comes from its block-table entry (any block size). Keys past the end
  // read the last valid row (finite data) and are masked to -inf.
  const int kbeg = b0 * bs, kfin = min(b1 * bs, len);
  const int64_t trow = (int64_t)n * max_blocks;
  for (int c0 = kbeg + 16 * w; c0 < kfin; c0 += 64) {
    float kf[4][8], vf[4][8];
    bool valid[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int key = c0 + 4 * u + sub;
      valid[u] = key < kfin;
      const int kk = valid[u] ? key : kfin - 1;
      const int blk = kk / bs;
      const int64_t off = (int64_t)tables[trow + blk] * blk_stride + (int64_t)hk * head_stride +
                          (int64_t)(kk - blk * bs) * D + li * EPL;
      load8<bf16>(reinterpret_cast<const bf16*>(kc + off), kf[u]);
      load8<bf16>(reinterpret_cast<const bf16*>(vc + off), vf[u]);
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float sc[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float t = 0.f;
#pragma unroll
        for (int j = 0; j < EPL; ++j) t += qv[g][j] * kf[u][j];
        t += __shfl_xor(t, 1, 64);
        t += __shfl_xor(t, 2, 64);
        t += __shfl_xor(t, 4, 64);
        t += __shfl_xor(t, 8, 64);
        sc[u] = valid[u] ? t : -INFINITY;
      }
      const float mx = fmaxf(fmaxf(sc[0], sc[1]), fmaxf(sc[2], sc[3]));
      const float mn = fmaxf(m[g], mx);
      if (mn == -INFINITY) continue;  // nothing valid yet in this lane group
      const float a = (m[g] == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(m[g] - mn);
      float pe[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) pe[u] = __builtin_amdgcn_exp2f(sc[u] - mn);  // exp2(-inf) = 0
      l[g] = l[g] * a + (pe[0] + pe[1]) + (pe[2] + pe[3]);
#pragma unroll
      for (int j = 0; j < EPL; ++j)
        o[g][j] = o[g][j] * a + pe[0] * vf[0][j] + pe[1] * vf[1][j] + pe[2] * vf[2][j] + pe[3] * vf[3][j];
      m[g] = mn;
    }
  }

  // merge the 4 key groups of the wave, then the 4 waves, through LDS
  __shared__ float sm_m[16][G], sm_l[16][G];
  __shared__ float sm_o[16][G][D];
  const int slot = w * 4 + sub;  // 16 partial states per workgroup
#pragma unroll
  for (int g = 0; g < G; ++g) {
    if (li == 0) { sm_m[slot][g] = m[g]; sm_l[slot][g] = l[g]; }
#pragma unroll
    for (int j = 0; j < EPL; ++j) sm_o[slot][g][li * EPL + j] = o[g][j];
  }
  __syncthreads();
  // thread t handles (g, d) pairs: G * D outputs, 256 threads
  for (int idx = tid; idx < G * D; idx += 256) {
    const int g = idx / D, d = idx % D;
    float mm = -INFINITY;
#pragma unroll
    for (int s = 0; s < 16; ++s) mm = fmaxf(mm, sm_m[s][g]);
    float ll = 0.f, oo = 0.f;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const float ms = sm_m[s][g];
      const float f = (ms == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(ms - mm);
      ll += sm_l[s][g] * f;
      oo += sm_o[s][g][d] * f;
    }
    if (splits == 1) {  // the whole key range is here: write the normalised output, no combine pass
      const float v = ll > 0.f ? oo / ll : 0.f;
      bf16 x = __float2bfloat16(v);
      out[((int64_t)n * H + hk * G + g) * D + d] = *reinterpret_cast<uint16_t*>(&x);
      continue;
    }
    const int64_t row = ((int64_t)n * H + hk * G + g) * splits + sp;
    part_o[row * D + d] = oo;
    if (d == 0) {
      part_ml[row * 2] = mm;
      part_ml[row * 2 + 1] = ll;
    }
  }
}

// merge split partials: out[n, h, :] = sum_s o_s * 2^(m_s - M) / sum_s l_s * 2^(m_s - M)
__global__ __launch_bounds__(128) void paged_decode_combine_k(const float* __restrict__ part_o,
                                                              const float* __restrict__ part_ml,
                                                              uint16_t* __restrict__ out, int splits, int D) {
  const int64_t row = blockIdx.x;  // n * H + h
  const int d = threadIdx.x;
  float mm = -INFINITY;
  for (int s = 0; s < splits; ++s) mm = fmaxf(mm, part_ml[(row * splits + s) * 2]);
  float ll = 0.f, oo = 0.f;
  for (int s = 0; s < splits; ++s) {
    const float ms = part_ml[(row * splits + s) * 2];
    const float f = (ms == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(ms - mm);
    ll += part_ml[(row * splits + s) * 2 + 1] * f;
    if (d < D) oo += part_o[(row * splits + s) * D + d] * f;
  }
  if (d < D) {
    const float v = ll > 0.f ? oo / ll : 0.f;
    bf16 x = __float2bfloat16(v);
    out[row * D + d] = *reinterpret_cast<uint16_t*>(&x);
  }
}

}  // namespace

// q [N, H, 128] bf16; caches bf16, key t of block pb / kv head h at pb*blk_stride + h*head_stride + t*128
// (paged [num_blocks, Hkv, block_size, 128]: blk_stride = Hkv*bs*128, head_stride = bs*128; a dense
// [B, H, max_len, 128] cache is viewed as virtual blocks with head_stride = max_len*128);
// tables [N, max_blocks] int32; lens [N] int32 (tokens in cache incl. the current one);
// part_o [N*H*splits*128] f32 and part_ml [N*H*splits*2] f32 workspaces; out [N, H, 128] bf16.
PA_EXPORT int pa_paged_decode_attn(const void* q, const void* kc, const void* vc, const int* tables, const int* lens,
                                   float* part_o, float* part_ml, void* out, int N, int H, int Hkv, int D, int bs,
                                   int max_blocks, int splits, int64_t blk_stride, int64_t head_stride, float scale,
                                   hipStream_t st) {
  if (D != 128 || H % Hkv != 0 || splits < 1) return 3;
  const int G = H / Hkv;
  const float sl2 = scale * 1.4426950408889634f;
  dim3 grid((unsigned)N, (unsigned)Hkv, (unsigned)splits);
#define PA_DEC(GG)                                                                                                  \
  hipLaunchKernelGGL((paged_decode_k<128, GG>), grid, dim3(256), 0, st, (const uint16_t*)q, (const uint16_t*)kc,   \
                     (const uint16_t*)vc, tables, lens, part_o, part_ml, (uint16_t*)out, H, Hkv, bs, max_blocks, splits, blk_stride,      \
                     head_stride, sl2)
  switch (G) {
    case 1: PA_DEC(1); break;
    case 2: PA_DEC(2); break;
    case 4: PA_DEC(4); break;
    case 8: PA_DEC(8); break;
    default: return 4;
  }
#undef PA_DEC
  PA_CHECK_LAUNCH();
  if (splits == 1) return 0;
  hipLaunchKernelGGL(paged_decode_combine_k, dim3((unsigned)(N * H)), dim3(128), 0, st, part_o, part_ml,
                     (uint16_t*)out, splits, D);
  PA_CHECK_LAUNCH();
  return 0;
}
