// Flash attention launchers (C ABI) and the bf16 kernel instantiations; kernels: flash_attn_kernels.h,
// fp16 instantiations: flash_attn_f16.hip.
#include "flash_attn_kernels.h"

#include <algorithm>
#include <cstdlib>

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

// Optional arguments (mirrors paddlepaddle_amd/ops/attention.py:_AttnExtra, all 8-byte fields).
struct PaAttnExtra {
  const int* cu_q; const int* cu_k;
  const void* mask; int64_t mask_kind; int64_t ms[3];
  const int* fm; int64_t fm_cols; int64_t fms[2];
  const int* fm_stats; int64_t fmst[2];
  double drop_p; uint64_t seed;
  int64_t lse_s[2];  // 0, 0 -> dense [B, H, Sq]
  int64_t dtype;     // 0 bf16, 1 fp16
};

template <typename A>
static void fill_extra(A& a, const PaAttnExtra* ex, int B, int Sq, int H) {
  a.cu_q = nullptr; a.cu_k = nullptr; a.mask = nullptr; a.mask_kind = 0; a.fm = nullptr; a.fm_cols = 0;
  a.dropout = 0; a.keep16 = 65536u; a.rkeep = 1.f; a.seed0 = 0; a.seed1 = 0;
  for (int i = 0; i < 3; ++i) a.ms[i] = 0;
  a.fms[0] = a.fms[1] = 0;
  a.fm_stats = nullptr; a.fmst[0] = a.fmst[1] = 0;
  a.lse_s[0] = (int64_t)H * Sq; a.lse_s[1] = Sq;
  if (ex == nullptr) return;
  a.cu_q = ex->cu_q; a.cu_k = ex->cu_k;
  a.mask = ex->mask; a.mask_kind = (int)ex->mask_kind;
  for (int i = 0; i < 3; ++i) a.ms[i] = ex->ms[i];
  a.fm = ex->fm; a.fm_cols = (int)ex->fm_cols; a.fms[0] = ex->fms[0]; a.fms[1] = ex->fms[1];
  a.fm_stats = ex->fm_stats; a.fmst[0] = ex->fmst[0]; a.fmst[1] = ex->fmst[1];
  if (ex->drop_p > 0.0) {
    a.dropout = 1;
    const double keep = 1.0 - ex->drop_p;
    a.keep16 = (uint32_t)(keep * 65536.0 + 0.5);
    a.rkeep = (float)(1.0 / keep);
    a.seed0 = (uint32_t)ex->seed;
    a.seed1 = (uint32_t)(ex->seed >> 32);
  }
  if (ex->lse_s[0] != 0 || ex->lse_s[1] != 0) { a.lse_s[0] = ex->lse_s[0]; a.lse_s[1] = ex->lse_s[1]; }
}

// compile-time feature set of a launch: 1 / 8 / 16 bool / bf16 / fp32 mask, 2 flashmask, 4 dropout (mask +
// flashmask together is not instantiated)
static int fa_features(int mask_kind, const int* fm, int dropout) {
  if (mask_kind != 0 && fm != nullptr) return -1;
  const int m = mask_kind == 1 ? 1 : (mask_kind == 2 ? 8 : (mask_kind == 3 ? 16 : 0));
  return m | (fm != nullptr ? 2 : 0) | (dropout ? 4 : 0);
}

static int g_fwd_variant = 2;

// A/B switch kept for the microbenchmarks (one forward kernel now)
PA_EXPORT int pa_flash_attn_set_fwd_variant(int v) {
  g_fwd_variant = v;
  return 0;
}

// strides: host array of 12 int64 = q(b,s,h), k(b,s,h), v(b,s,h), o(b,s,h). Sq / Sk: max lengths when varlen.
PA_EXPORT int pa_flash_attn_fwd_ex(const void* q, const void* k, const void* v, void* o, float* lse,
                                   const int64_t* strides, int B, int Sq, int Sk, int H, int Hk, int D, float scale,
                                   int causal, const PaAttnExtra* ex, hipStream_t st) {
  if (H % Hk != 0) return 3;
  if (D != 128 && D != 64 && D != 256) return 4;
  if (ex != nullptr && ex->fm != nullptr && ex->fm_cols != 1 && ex->fm_cols != 2 && ex->fm_cols != 4) return 5;
  FwdArgs a;
  a.q = (const uint16_t*)q; a.k = (const uint16_t*)k; a.v = (const uint16_t*)v; a.o = (uint16_t*)o; a.lse = lse;
  for (int i = 0; i < 3; ++i) {
    a.qs[i] = strides[i]; a.ks[i] = strides[3 + i]; a.vs[i] = strides[6 + i]; a.os[i] = strides[9 + i];
  }
  a.B = B; a.Sq = Sq; a.Sk = Sk; a.H = H; a.Hk = Hk;
  a.scale_log2 = scale * kLog2e;
  a.inv_scale = 1.f / scale;
  a.causal = causal;
  fill_extra(a, ex, B, Sq, H);
  const int nqb = (Sq + 127) / 128;
  a.grp = fa_group(B * H, nqb, 64);
  dim3 grid((unsigned)(B * H * nqb));
  const bool f16 = ex != nullptr && ex->dtype == 1;
  const int feat = fa_features(a.mask_kind, a.fm, a.dropout);
  if (feat < 0) return 6;
  if (f16) pa_fa_fwd_f16(a, D, feat, grid, st);
  else fa_fwd_dispatch<false>(a, D, feat, grid, st);
  PA_CHECK_LAUNCH();
  return 0;
}

PA_EXPORT int pa_flash_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse,
                                const int64_t* strides, int B, int Sq, int Sk, int H, int Hk, int D, float scale,
                                int causal, hipStream_t st) {
  return pa_flash_attn_fwd_ex(q, k, v, o, lse, strides, B, Sq, Sk, H, Hk, D, scale, causal, nullptr, st);
}

// strides: host array of 24 int64 = q, k, v, o, do, dq, dk, dv  (each b,s,h). dk / dv are [.., Hk, D] (summed
// over the query heads of each KV head in-kernel). dq_acc: fp32 [rows, H, D] contiguous, rows = B*Sq
// (dense) or total_q (varlen, `q_rows`); delta: same layout as lse.
// dS route eligibility (fa_bwd16_kernel<.., true> + fa_bwd_dq_kernel): D = 128, no mask / flashmask / dropout,
// dense batches. The caller allocates the dS^T scratch [B*H][ceil128(Sk)][ceil128(Sq)] 16-bit elements.
PA_EXPORT int pa_flash_attn_bwd_ds_ok(int D, int has_mask, int has_fm, int dropout, int varlen) {
  const char* env = getenv("PA_FA_BWD_DS");
  if (env != nullptr && atoi(env) == 0) return 0;
  const char* k16_env = getenv("PA_FA_BWD16");
  if (k16_env != nullptr && atoi(k16_env) != 1) return 0;
  const char* abl_env = getenv("PA_FA_BWD_ABL");
  if (abl_env != nullptr && atoi(abl_env) != 0) return 0;
  return D == 128 && !has_mask && !has_fm && !dropout && !varlen;
}

static int flash_attn_bwd_impl(const void* q, const void* k, const void* v, const void* o, const void* dout,
                               const float* lse, void* dq, void* dk, void* dv, float* dq_acc, float* delta,
                               const int64_t* strides, int B, int Sq, int Sk, int H, int Hk, int D, float scale,
                               int causal, int64_t q_rows, const PaAttnExtra* ex, void* ds, hipStream_t st) {
  if (H % Hk != 0) return 3;
  if (D != 128 && D != 64 && D != 256) return 4;
  const int64_t* qs = strides; const int64_t* ks = strides + 3; const int64_t* vs = strides + 6;
  const int64_t* os = strides + 9; const int64_t* dos = strides + 12; const int64_t* dqs = strides + 15;
  const int64_t* dks = strides + 18; const int64_t* dvs = strides + 21;
  const bool varlen = ex != nullptr && ex->cu_q != nullptr;
  const bool f16 = ex != nullptr && ex->dtype == 1;
  BwdArgs a;
  a.B = B; a.Sq = Sq; a.Sk = Sk; a.H = H; a.Hk = Hk;
  fill_extra(a, ex, B, Sq, H);
  // delta = rowsum(dO * O), in the lse layout; varlen: rows of the packed tensors ([H, total_q])
  const int DB = varlen ? 1 : B;
  const int DS = varlen ? (int)q_rows : Sq;
  if (f16) pa_fa_bwd_aux_f16(0, a, (const uint16_t*)o, (const uint16_t*)dout, delta, os, dos, nullptr, nullptr, nullptr,
                             DB, DS, H, D, st);
  else fa_bwd_aux<false>(0, a, (const uint16_t*)o, (const uint16_t*)dout, delta, os, dos, nullptr, nullptr, nullptr, DB,
                         DS, H, D, st);
  PA_CHECK_LAUNCH();
  const int64_t rows = varlen ? q_rows : (int64_t)B * Sq;
  a.ds = nullptr;
  a.ds_ld = 0;
  a.ds_rows = 0;
  a.dq = (uint16_t*)dq;
  for (int i = 0; i < 3; ++i) a.dqs[i] = dqs[i];
  a.dq_grp = 0;
  if (ds != nullptr) {
    if (varlen || D != 128) return 7;
    a.ds = (uint16_t*)ds;
    a.ds_ld = (Sq + 127) / 128 * 128;
    a.ds_rows = (Sk + 127) / 128 * 128;
    a.dq_grp = fa_group(B * H, (Sq + 127) / 128, 64);
  } else {
    hipMemsetAsync(dq_acc, 0, (size_t)rows * H * D * sizeof(float), st);
  }
  a.q = (const uint16_t*)q; a.k = (const uint16_t*)k; a.v = (const uint16_t*)v; a.o = (const uint16_t*)o;
  a.dout = (const uint16_t*)dout; a.lse = lse; a.dq_acc = dq_acc; a.delta = delta;
  a.dk = (uint16_t*)dk; a.dv = (uint16_t*)dv;
  for (int i = 0; i < 3; ++i) {
    a.qs[i] = qs[i]; a.ks[i] = ks[i]; a.vs[i] = vs[i]; a.dos[i] = dos[i]; a.dks[i] = dks[i]; a.dvs[i] = dvs[i];
  }
  a.scale = scale; a.scale_log2 = scale * kLog2e; a.inv_scale = 1.f / scale; a.causal = causal;
  const char* abl_env = getenv("PA_FA_BWD_ABL");  // measurement ablations only (tools/bench_fa_bwd_abl.py)
  a.abl = abl_env ? atoi(abl_env) : 0;
  // 16-keys-per-wave backward (D = 128, no mask / dropout): the default (1.04-1.06x the 4-wave kernel,
  // profiles/flash_attn_bwd_ablations_r3.md); PA_FA_BWD16=0 selects the 4-wave kernel
  const char* k16_env = getenv("PA_FA_BWD16");
  a.k16 = k16_env ? atoi(k16_env) : 1;
  const int BK = D == 256 ? 64 : 128;
  const int nkb = (Sk + BK - 1) / BK;
  a.grp = fa_group(B * Hk, nkb, 32);
  dim3 grid((unsigned)(B * Hk * nkb));
  const int feat = fa_features(a.mask_kind, a.fm, a.dropout);
  if (feat < 0) return 6;
  if (ds != nullptr && feat != 0) return 7;
  if (f16) pa_fa_bwd_f16(a, D, feat, grid, st);
  else fa_bwd_dispatch<false>(a, D, feat, grid, st);
  PA_CHECK_LAUNCH();
  if (ds != nullptr) return 0;  // dQ written by fa_bwd_dq_kernel
  if (f16) pa_fa_bwd_aux_f16(1, a, nullptr, nullptr, nullptr, nullptr, nullptr, dq_acc, (uint16_t*)dq, dqs, DB, DS, H, D,
                             st);
  else fa_bwd_aux<false>(1, a, nullptr, nullptr, nullptr, nullptr, nullptr, dq_acc, (uint16_t*)dq, dqs, DB, DS, H, D, st);
  PA_CHECK_LAUNCH();
  return 0;
}

PA_EXPORT int pa_flash_attn_bwd_ex(const void* q, const void* k, const void* v, const void* o, const void* dout,
                                   const float* lse, void* dq, void* dk, void* dv, float* dq_acc, float* delta,
                                   const int64_t* strides, int B, int Sq, int Sk, int H, int Hk, int D, float scale,
                                   int causal, int64_t q_rows, const PaAttnExtra* ex, hipStream_t st) {
  return flash_attn_bwd_impl(q, k, v, o, dout, lse, dq, dk, dv, dq_acc, delta, strides, B, Sq, Sk, H, Hk, D, scale,
                             causal, q_rows, ex, nullptr, st);
}

// the dS route: ds = scratch of pa_flash_attn_bwd_ds_bytes bytes; dq_acc unused (may be null)
PA_EXPORT int64_t pa_flash_attn_bwd_ds_bytes(int B, int Sq, int Sk, int H) {
  return (int64_t)B * H * ((Sk + 127) / 128 * 128) * ((Sq + 127) / 128 * 128) * 2;
}

PA_EXPORT int pa_flash_attn_bwd_ds(const void* q, const void* k, const void* v, const void* o, const void* dout,
                                   const float* lse, void* dq, void* dk, void* dv, void* ds, float* delta,
                                   const int64_t* strides, int B, int Sq, int Sk, int H, int Hk, int D, float scale,
                                   int causal, const PaAttnExtra* ex, hipStream_t st) {
  return flash_attn_bwd_impl(q, k, v, o, dout, lse, dq, dk, dv, nullptr, delta, strides, B, Sq, Sk, H, Hk, D, scale,
                             causal, (int64_t)B * Sq, ex, ds, st);
}

PA_EXPORT int pa_flash_attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout,
                                const float* lse, void* dq, void* dk, void* dv, float* dq_acc, float* delta,
                                const int64_t* strides, int B, int Sq, int Sk, int H, int Hk, int D, float scale,
                                int causal, hipStream_t st) {
  return pa_flash_attn_bwd_ex(q, k, v, o, dout, lse, dq, dk, dv, dq_acc, delta, strides, B, Sq, Sk, H, Hk, D, scale,
                              causal, (int64_t)B * Sq, nullptr, st);
}

// Flashmask tile extrema for block skipping: stats [Bm * Hm * ntiles * 8] int32, ntiles = ceil(Sk / 64) rounded
// up to even (tiles past Sk get identity extrema). fm [Bm, Hm, Sk(+pad), cols] with (b, h) strides in elements.
PA_EXPORT int pa_fa_fm_stats(const int* fm, int cols, int causal, int Sk, int Bm, int Hm, int64_t sb, int64_t sh,
                             int ntiles, int* stats, hipStream_t st) {
  if (cols != 1 && cols != 2 && cols != 4) return 5;
  hipLaunchKernelGGL(fa_fm_tile_stats, dim3((unsigned)(Bm * Hm * ntiles)), dim3(64), 0, st, fm, cols, causal, Sk,
                     ntiles, sb, sh, Hm, stats);
  PA_CHECK_LAUNCH();
  return 0;
}
