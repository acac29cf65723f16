// Native training executor: runs a traced static training program — forward, backward and the optimizer update —
// as one C++ call, with no Python between operations.
//
// Reference behaviour: paddle/fluid/framework/new_executor/pir_interpreter.cc (BuildInstruction :805: one
// instruction per op; BuildInstructionDependences :1078 and the last-use GC of program_interpreter.cc:142,231) —
// the reference executes a program that already holds its backward and optimizer ops. Here the forward program is
// traced (static/program.py) and lowered by static/native_train.py into instructions of three kinds:
//   * hot ops on this framework's hand-written CDNA4 kernels, each a C++ autograd node whose backward launches the
//     matching kernels: linear / linear_nt on the MFMA GEMMs (dgrad and wgrad read the transposed operands in
//     place), layer_norm / rms_norm, flash attention (fwd + bwd), softmax cross entropy, NHWC implicit-GEMM
//     convolution (forward, stride-1 data gradient as the flipped-filter forward, split-K weight gradient) and the
//     fused NHWC batch norm (+ReLU, + residual);
//   * every other op as the ATen operator(s) it dispatched to at trace time (captured below autograd on meta
//     tensors, so each instruction is one dispatcher call whose autograd formula records the backward);
//   * one optimizer instruction (AdamW / Adam / Momentum multi-tensor kernels over a pointer table built here;
//     global-norm clipping as a device scalar folded into the update).
// run(): feeds -> forward instructions (slots released after their last reader: only what autograd saved stays
// alive) -> torch autograd engine backward from the loss (the C++ engine, in-place accumulation into the
// persistent gradient buffers) -> optimizer kernels -> fetches.
#include <torch/extension.h>
#include <torch/csrc/autograd/custom_function.h>
#include <torch/csrc/autograd/autograd.h>
#include <torch/csrc/jit/python/pybind_utils.h>
#include <torch/csrc/autograd/python_variable.h>
#include <ATen/core/dispatch/Dispatcher.h>
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPGuard.h>
#include <hip/hip_runtime_api.h>

#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace py = pybind11;
using torch::autograd::AutogradContext;
using torch::autograd::variable_list;

extern "C" {
struct PaAttnExtra {  // mirror of csrc/kernels/flash_attn.hip
  const int* cu_q;
  const int* cu_k;
  const void* mask;
  int64_t mask_kind;
  int64_t ms[3];
  const int* fm;
  int64_t fm_cols;
  int64_t fms[2];
  const int* fm_stats;
  int64_t fmst[2];
  double drop_p;
  uint64_t seed;
  int64_t lse_s[2];
  int64_t dtype;
};
int pa_gemm_bf16(const void* a, const void* b, void* c, const void* bias, void* aux, int64_t M, int64_t N, int64_t K,
                 int64_t lda, int64_t ldb, int64_t ldc, int a_kmajor, int b_kmajor, int flags, float alpha, int bn,
                 int splits, hipStream_t st);
int pa_gemm_bf16_pp(const void* a, const void* b, void* c, const void* bias, void* aux, int64_t M, int64_t N,
                    int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int a_kmajor, int b_kmajor, int flags,
                    float alpha, void* ws, hipStream_t st);
int64_t pa_gemm_pp_ws_bytes(int64_t M, int64_t N, int64_t K);
int pa_layer_norm_fwd(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd, int64_t rows,
                      int64_t cols, float eps, int dtype, hipStream_t st);
int pa_layer_norm_bwd(const void* dy, const void* x, const void* w, const float* mean, const float* rstd, void* dx,
                      float* dw_part, float* db_part, void* res, int64_t rows, int64_t cols, int dtype_np,
                      hipStream_t st);
int pa_rms_norm_fwd(const void* x, const void* w, void* y, float* rstd, int64_t rows, int64_t cols, float eps,
                    int dtype, hipStream_t st);
int pa_rms_norm_bwd(const void* dy, const void* x, const void* w, const float* rstd, void* dx, float* dw_part,
                    int64_t rows, int64_t cols, int dtype_np, hipStream_t st);
int pa_flash_attn_fwd_ex(const void* q, const void* k, const void* v, void* o, float* lse, const int64_t* strides,
                         int B, int Sq, int Sk, int H, int Hk, int D, float scale, int causal, const PaAttnExtra* ex,
                         hipStream_t st);
int pa_flash_attn_bwd_ex(const void* q, const void* k, const void* v, const void* o, const void* dout,
                         const float* lse, void* dq, void* dk, void* dv, float* dq_acc, float* delta,
                         const int64_t* strides, int B, int Sq, int Sk, int H, int Hk, int D, float scale, int causal,
                         int64_t q_rows, const PaAttnExtra* ex, hipStream_t st);
int pa_softmax_ce_fwd(const void* logits, const int64_t* labels, float* loss, float* lse, int64_t rows, int64_t cols,
                      int64_t ignore_index, int dtype, hipStream_t st);
int pa_softmax_ce_bwd(const void* logits, const int64_t* labels, const float* lse, const float* dloss, void* dlogits,
                      int64_t rows, int64_t cols, int64_t ignore_index, int dtype, hipStream_t st);
int pa_conv2d_nhwc_fwd(const void* x, const void* w, const void* bias, void* out, const void* zero, int N, int H,
                       int W, int C, int Cout, int KH, int KW, int stride, int pad_h, int pad_w, int dil, int Ho,
                       int Wo, hipStream_t st);
int pa_conv2d_nhwc_wgrad(const void* x, const void* dy, float* ws, const void* zero, int N, int H, int W, int C,
                         int Cout, int KH, int KW, int stride, int pad_h, int pad_w, int dil, int Ho, int Wo,
                         int splits, int bn, hipStream_t st);
int pa_bn_chunks(int64_t R, int C);
int pa_bn_fwd_nhwc(const void* x, const void* res, void* y, const float* w, const float* b, float* run_mean,
                   float* run_var, float* save_mean, float* save_rstd, float* partial, float* ss, int64_t R, int C,
                   float momentum, float eps, int relu, int training, hipStream_t st);
int pa_bn_bwd_nhwc(const void* dy, const void* x, const void* y, void* dx, void* dres, const float* w,
                   const float* mean, const float* rstd, float* dw, float* db, float* partial, float* coef, int64_t R,
                   int C, int relu, int global_stats, const float* ss, hipStream_t st);
int pa_adamw_multi(const int64_t* table, const int64_t* items, int64_t n_items, const float* inv_scale, float lr,
                   float b1, float b2, float eps, float wd_unused, float bc1, float bc2, const float* hyper,
                   hipStream_t st);
int pa_momentum_multi(const int64_t* table, const int64_t* items, int64_t n_items, const float* inv_scale, float lr,
                      float mu, float rescale, int nesterov, hipStream_t st);
}

namespace {

std::unordered_map<std::string, int64_t> g_calls;  // hand-written kernel launches per kind (tests assert on them)
inline void count(const char* k) { ++g_calls[k]; }

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

int dcode(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return 0;
    case at::kHalf: return 1;
    case at::kBFloat16: return 2;
    default: return -1;
  }
}

bool al16(const at::Tensor& t) { return (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0; }

void chk(int rc, const char* what) {
  if (rc != 0) throw std::runtime_error(std::string("native train executor: ") + what + " launch failed (" +
                                        std::to_string(rc) + ")");
}

const void* ptr_or_null(const at::Tensor& t) { return t.defined() && t.numel() > 0 ? t.data_ptr() : nullptr; }

// custom autograd functions take absent optional operands as empty placeholders (an undefined tensor argument has
// no device for the autograd input metadata); inside, an empty operand means "absent"
at::Tensor opt_in(const at::Tensor& t, const at::Tensor& like) {
  return t.defined() ? t : at::empty({0}, like.options().requires_grad(false));
}
at::Tensor present(const at::Tensor& t) { return t.defined() && t.numel() > 0 ? t : at::Tensor(); }

// ------------------------------------------------------------------------------------------------ GEMM
constexpr int kEpiBias = 1, kEpiGelu = 2, kEpiAux = 4, kEpiAccum = 8, kEpiF32 = 16;

struct Lay {
  int64_t ld = 0;
  bool kmajor = false;
  bool ok = false;
};

// (leading dim, K-major) of a 2-D operand view whose K dimension is 1 - outer (ops/gemm.py _layout)
Lay lay(const at::Tensor& t, int outer) {
  const int kd = 1 - outer;
  Lay l;
  if (t.stride(kd) == 1 && t.size(kd) >= 1) {
    l.ld = t.size(outer) > 1 ? t.stride(outer) : t.size(kd);
    l.kmajor = true;
    l.ok = true;
  } else if (t.stride(outer) == 1) {
    l.ld = t.size(kd) > 1 ? t.stride(kd) : t.size(outer);
    l.kmajor = false;
    l.ok = true;
  }
  return l;
}

// the MFMA GEMM's operand conditions for C = a @ b (ops/gemm.py supported)
bool mm_ok(const at::Tensor& a, const at::Tensor& b) {
  if (!a.is_cuda() || a.dim() != 2 || b.dim() != 2 || a.scalar_type() != at::kBFloat16 ||
      b.scalar_type() != at::kBFloat16)
    return false;
  const int64_t M = a.size(0), K = a.size(1), N = b.size(1);
  if (K == 0 || M == 0 || K % 64 != 0 || N % 8 != 0 || b.size(0) != K) return false;
  const Lay la = lay(a, 0), lb = lay(b, 1);
  if (!la.ok || !lb.ok || la.ld % 8 != 0 || lb.ld % 8 != 0) return false;
  if (!la.kmajor && M % 8 != 0) return false;
  return al16(a) && al16(b);
}

// out = epilogue(a @ b) on the hand-written kernels: the 256x256 ping-pong kernel once the output fills a wave of
// tiles, else the 2-stage kernels (tile width as ops/gemm.py _pick_bn)
at::Tensor mm(const at::Tensor& a, const at::Tensor& b, const at::Tensor& bias, bool gelu, at::Tensor aux,
              at::Tensor out, bool accumulate) {
  const int64_t M = a.size(0), K = a.size(1), N = b.size(1);
  const Lay la = lay(a, 0), lb = lay(b, 1);
  if (!out.defined()) out = at::empty({M, N}, a.options());
  int flags = 0;
  if (bias.defined()) flags |= kEpiBias;
  if (gelu) flags |= kEpiGelu;
  if (aux.defined()) flags |= kEpiAux;
  if (accumulate) flags |= kEpiAccum;
  if (out.scalar_type() == at::kFloat) flags |= kEpiF32;
  const int64_t tiles = ((M + 255) / 256) * ((N + 255) / 256);
  int rc;
  if (M >= 1024 && N >= 1024 && tiles >= 256) {
    const int64_t nb = pa_gemm_pp_ws_bytes(M, N, K);
    at::Tensor ws = nb > 0 ? at::empty({(nb + 3) / 4}, a.options().dtype(at::kFloat)) : at::Tensor();
    rc = pa_gemm_bf16_pp(a.data_ptr(), b.data_ptr(), out.data_ptr(), ptr_or_null(bias),
                         aux.defined() ? aux.data_ptr() : nullptr, M, N, K, la.ld, lb.ld, out.stride(0),
                         la.kmajor ? 1 : 0, lb.kmajor ? 1 : 0, flags, 1.f, ws.defined() ? ws.data_ptr() : nullptr,
                         stream());
  } else {
    int bn = 160;
    if (!lb.kmajor) {
      auto eff = [&](int64_t w) {
        const int64_t t = ((M + 255) / 256) * ((N + w - 1) / w);
        const int64_t waves = (t + 255) / 256;
        return static_cast<double>(t) / static_cast<double>(waves * 256) * (w == 256 ? 1.0 : 0.9);
      };
      bn = eff(256) >= eff(128) ? 256 : 128;
    }
    rc = pa_gemm_bf16(a.data_ptr(), b.data_ptr(), out.data_ptr(), ptr_or_null(bias),
                      aux.defined() ? aux.data_ptr() : nullptr, M, N, K, la.ld, lb.ld, out.stride(0),
                      la.kmajor ? 1 : 0, lb.kmajor ? 1 : 0, flags, 1.f, bn, 1, stream());
  }
  chk(rc, "gemm");
  count("gemm");
  return out;
}

at::Tensor matmul2d(const at::Tensor& a, const at::Tensor& b) {
  if (mm_ok(a, b)) return mm(a, b, at::Tensor(), false, at::Tensor(), at::Tensor(), false);
  return at::mm(a, b);
}

std::vector<int64_t> with_last(at::IntArrayRef s, int64_t n) {
  std::vector<int64_t> v(s.begin(), s.end());
  v.back() = n;
  return v;
}

// ------------------------------------------------------------------------------------------------ linear
// y = act(x @ W + b), W [in, out] (paddle layout); act 0 none, 1 tanh-GELU (epilogue of the GEMM, pre-activation
// kept for the backward), 2 relu
// The function's output reshaped to ``sizes`` over the same storage, WITHOUT autograd view tracking: a view returned
// from a custom Function may not be modified in place (the program's in-place collectives write these outputs); used
// only where the function saves nothing that aliases the output.
inline at::Tensor out_alias(const at::Tensor& y, at::IntArrayRef sizes) {
  at::Tensor v = y.view(sizes);
  at::Tensor t = at::empty({0}, y.options());
  t.set_(v.storage(), v.storage_offset(), v.sizes(), v.strides());
  return t;
}

struct LinearFn : public torch::autograd::Function<LinearFn> {
  static at::Tensor forward(AutogradContext* ctx, at::Tensor x, at::Tensor w, at::Tensor b, int64_t act) {
    b = present(b);
    const int64_t K = x.size(-1), N = w.size(1);
    at::Tensor x2 = x.reshape({-1, K});
    if (!x2.is_contiguous()) x2 = x2.contiguous();
    at::Tensor y, pre;
    const bool bias_ok = !b.defined() || (b.scalar_type() == at::kBFloat16 && b.is_contiguous() && al16(b));
    if (mm_ok(x2, w) && bias_ok && (act != 1 || b.defined())) {
      if (act == 1) {
        pre = at::empty({x2.size(0), N}, x2.options());
        y = mm(x2, w, b, true, pre, at::Tensor(), false);
      } else {
        y = mm(x2, w, b, false, at::Tensor(), at::Tensor(), false);
      }
    } else {
      at::Tensor h = at::mm(x2, w);
      if (b.defined()) h = h + b;
      if (act == 1) {
        pre = h;
        y = at::gelu(h, "tanh");
      } else {
        y = h;
      }
    }
    if (act == 2) {
      y = at::relu(y);
      pre = y;  // the relu mask
    }
    ctx->save_for_backward({x2, w, pre});
    ctx->saved_data["act"] = act;
    ctx->saved_data["has_b"] = b.defined();
    ctx->saved_data["shape"] = x.sizes().vec();
    if (act == 2) return y.view(with_last(x.sizes(), N));  // y is the saved relu mask: keep autograd's view checks
    return out_alias(y, with_last(x.sizes(), N));
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto sv = ctx->get_saved_variables();
    at::Tensor x2 = sv[0], w = sv[1], pre = sv[2];
    const int64_t act = ctx->saved_data["act"].toInt();
    const int64_t N = w.size(1);
    at::Tensor dy = grads[0].reshape({-1, N}).to(x2.scalar_type());
    if (!dy.is_contiguous()) dy = dy.contiguous();
    if (act == 1) dy = at::gelu_backward(dy, pre, "tanh");
    if (act == 2) dy = dy * (pre > 0);
    at::Tensor dx, dw, db;
    if (ctx->needs_input_grad(0)) dx = matmul2d(dy, w.t()).view(ctx->saved_data["shape"].toIntVector());
    if (ctx->needs_input_grad(1)) dw = matmul2d(x2.t(), dy);
    if (ctx->saved_data["has_b"].toBool() && ctx->needs_input_grad(2))
      db = dy.to(at::kFloat).sum(0).to(dy.scalar_type());
    return {dx, dw, db, at::Tensor()};
  }
};

// y = x @ W^T with W [out, in] (the tied LM head)
struct LinearNTFn : public torch::autograd::Function<LinearNTFn> {
  static at::Tensor forward(AutogradContext* ctx, at::Tensor x, at::Tensor w) {
    const int64_t K = x.size(-1), N = w.size(0);
    at::Tensor x2 = x.reshape({-1, K});
    if (!x2.is_contiguous()) x2 = x2.contiguous();
    at::Tensor y = matmul2d(x2, w.t());
    ctx->save_for_backward({x2, w});
    ctx->saved_data["shape"] = x.sizes().vec();
    return out_alias(y, with_last(x.sizes(), N));
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto sv = ctx->get_saved_variables();
    at::Tensor x2 = sv[0], w = sv[1];
    at::Tensor dy = grads[0].reshape({-1, w.size(0)}).to(x2.scalar_type());
    if (!dy.is_contiguous()) dy = dy.contiguous();
    at::Tensor dx, dw;
    if (ctx->needs_input_grad(0)) dx = matmul2d(dy, w).view(ctx->saved_data["shape"].toIntVector());
    if (ctx->needs_input_grad(1)) dw = matmul2d(dy.t(), x2);
    return {dx, dw};
  }
};

// ------------------------------------------------------------------------------------------------ norms
int64_t norm_parts(int64_t rows) { return std::min<int64_t>(std::max<int64_t>((rows + 15) / 16, 1), 512); }

bool norm_ok(const at::Tensor& x, const at::Tensor& w) {
  return x.is_cuda() && dcode(x) >= 0 && x.size(-1) % 8 == 0 && (!w.defined() || w.numel() == x.size(-1));
}

// layer_norm (rms = false) / rms_norm over the last dimension
struct NormFn : public torch::autograd::Function<NormFn> {
  static at::Tensor forward(AutogradContext* ctx, at::Tensor x, at::Tensor w, at::Tensor b, double eps, bool rms) {
    w = present(w);
    b = present(b);
    const int64_t cols = x.size(-1);
    at::Tensor x2 = x.reshape({-1, cols}).contiguous();
    const int64_t rows = x2.size(0);
    at::Tensor wc = w.defined() ? w.to(x2.scalar_type()).contiguous() : at::Tensor();
    at::Tensor bc = b.defined() ? b.to(x2.scalar_type()).contiguous() : at::Tensor();
    at::Tensor y = at::empty_like(x2);
    at::Tensor stats = at::empty({2, rows}, x2.options().dtype(at::kFloat));
    float* mean = stats.data_ptr<float>();
    float* rstd = mean + rows;
    if (rms) {
      chk(pa_rms_norm_fwd(x2.data_ptr(), ptr_or_null(wc), y.data_ptr(), rstd, rows, cols, static_cast<float>(eps),
                          dcode(x2), stream()),
          "rms_norm");
      count("rms_norm");
    } else {
      chk(pa_layer_norm_fwd(x2.data_ptr(), ptr_or_null(wc), ptr_or_null(bc), y.data_ptr(), mean, rstd, rows, cols,
                            static_cast<float>(eps), dcode(x2), stream()),
          "layer_norm");
      count("layer_norm");
    }
    ctx->save_for_backward({x2, wc, stats});
    ctx->saved_data["rms"] = rms;
    ctx->saved_data["has_w"] = w.defined();
    ctx->saved_data["has_b"] = b.defined();
    ctx->saved_data["wdt"] = static_cast<int64_t>(w.defined() ? w.scalar_type() : x2.scalar_type());
    ctx->saved_data["bdt"] = static_cast<int64_t>(b.defined() ? b.scalar_type() : x2.scalar_type());
    return out_alias(y, x.sizes());
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto sv = ctx->get_saved_variables();
    at::Tensor x2 = sv[0], wc = sv[1], stats = sv[2];
    const int64_t rows = x2.size(0), cols = x2.size(1);
    at::Tensor dy = grads[0].reshape({rows, cols}).to(x2.scalar_type()).contiguous();
    at::Tensor dx = at::empty_like(x2);
    const int64_t np = norm_parts(rows);
    at::Tensor dwp = at::empty({np, cols}, x2.options().dtype(at::kFloat));
    at::Tensor dbp = at::empty({np, cols}, x2.options().dtype(at::kFloat));
    const float* mean = stats.data_ptr<float>();
    const float* rstd = mean + rows;
    const bool rms = ctx->saved_data["rms"].toBool();
    const int dnp = dcode(x2) | static_cast<int>(np << 8);
    if (rms) {
      chk(pa_rms_norm_bwd(dy.data_ptr(), x2.data_ptr(), ptr_or_null(wc), rstd, dx.data_ptr(),
                          wc.defined() ? dwp.data_ptr<float>() : nullptr, rows, cols, dnp, stream()),
          "rms_norm_bwd");
    } else {
      chk(pa_layer_norm_bwd(dy.data_ptr(), x2.data_ptr(), ptr_or_null(wc), mean, rstd, dx.data_ptr(),
                            dwp.data_ptr<float>(), dbp.data_ptr<float>(), nullptr, rows, cols, dnp, stream()),
          "layer_norm_bwd");
    }
    at::Tensor dw, db;
    if (ctx->saved_data["has_w"].toBool())
      dw = dwp.sum(0).to(static_cast<at::ScalarType>(ctx->saved_data["wdt"].toInt()));
    if (ctx->saved_data["has_b"].toBool())
      db = dbp.sum(0).to(static_cast<at::ScalarType>(ctx->saved_data["bdt"].toInt()));
    return {dx.view(grads[0].sizes()), dw, db, at::Tensor(), at::Tensor()};
  }
};

// ------------------------------------------------------------------------------------------------ attention
void strides3(const at::Tensor& t, std::vector<int64_t>& v) {
  v.push_back(t.stride(0));
  v.push_back(t.stride(1));
  v.push_back(t.stride(2));
}

PaAttnExtra extra_for(const at::Tensor& q) {
  PaAttnExtra ex;
  std::memset(&ex, 0, sizeof(ex));
  ex.dtype = q.scalar_type() == at::kHalf ? 1 : 0;
  return ex;
}

bool attn_ok(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v) {
  auto lastdim = [](const at::Tensor& t) {
    if (t.stride(3) != 1 || !al16(t)) return false;
    for (int d = 0; d < 3; ++d)
      if (t.stride(d) % 8 != 0) return false;
    return true;
  };
  if (!q.is_cuda() || q.dim() != 4 || k.dim() != 4 || v.dim() != 4) return false;
  if ((q.scalar_type() != at::kBFloat16 && q.scalar_type() != at::kHalf) || k.scalar_type() != q.scalar_type() ||
      v.scalar_type() != q.scalar_type())
    return false;
  const int64_t D = q.size(3);
  if ((D != 64 && D != 128 && D != 256) || k.size(3) != D || v.size(3) != D || q.size(2) % k.size(2) != 0)
    return false;
  return lastdim(q) && lastdim(k) && lastdim(v);
}

at::Tensor lastdim_contig(const at::Tensor& t) {
  bool ok = t.stride(-1) == 1 && al16(t);
  for (int64_t d = 0; d + 1 < t.dim() && ok; ++d) ok = t.stride(d) % 8 == 0;
  return ok ? t : t.contiguous();
}

void fa_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, at::Tensor& o, at::Tensor& lse,
            bool causal, double scale) {
  const int64_t B = q.size(0), Sq = q.size(1), H = q.size(2), D = q.size(3), Sk = k.size(1), Hk = k.size(2);
  o = at::empty({B, Sq, H, D}, q.options());
  lse = at::empty({B, H, Sq}, q.options().dtype(at::kFloat));
  std::vector<int64_t> st;
  strides3(q, st);
  strides3(k, st);
  strides3(v, st);
  strides3(o, st);
  PaAttnExtra ex = extra_for(q);
  chk(pa_flash_attn_fwd_ex(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr<float>(), st.data(),
                           (int)B, (int)Sq, (int)Sk, (int)H, (int)Hk, (int)D, static_cast<float>(scale),
                           causal ? 1 : 0, &ex, stream()),
      "flash_attn");
  count("flash_attn");
}

void fa_bwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, const at::Tensor& o, const at::Tensor& lse,
            const at::Tensor& dout, const at::Tensor& dq, const at::Tensor& dk, const at::Tensor& dv, bool causal,
            double scale) {
  const int64_t B = q.size(0), Sq = q.size(1), H = q.size(2), D = q.size(3), Sk = k.size(1), Hk = k.size(2);
  at::Tensor dq_acc = at::empty({B * Sq, H, D}, q.options().dtype(at::kFloat));
  at::Tensor delta = at::empty({B, H, Sq}, q.options().dtype(at::kFloat));
  std::vector<int64_t> st;
  for (const at::Tensor* t : {&q, &k, &v, &o, &dout, &dq, &dk, &dv}) strides3(*t, st);
  PaAttnExtra ex = extra_for(q);
  chk(pa_flash_attn_bwd_ex(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), dout.data_ptr(),
                           lse.data_ptr<float>(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(),
                           dq_acc.data_ptr<float>(), delta.data_ptr<float>(), st.data(), (int)B, (int)Sq, (int)Sk,
                           (int)H, (int)Hk, (int)D, static_cast<float>(scale), causal ? 1 : 0, B * Sq, &ex, stream()),
      "flash_attn_bwd");
  count("flash_attn_bwd");
}

// q [B, Sq, H, D], k / v [B, Sk, Hk, D] -> o [B, Sq, H, D]
struct FlashAttnFn : public torch::autograd::Function<FlashAttnFn> {
  static at::Tensor forward(AutogradContext* ctx, at::Tensor q, at::Tensor k, at::Tensor v, bool causal,
                            double scale) {
    q = lastdim_contig(q);
    k = lastdim_contig(k);
    v = lastdim_contig(v);
    at::Tensor o, lse;
    fa_fwd(q, k, v, o, lse, causal, scale);
    ctx->save_for_backward({q, k, v, o, lse});
    ctx->saved_data["causal"] = causal;
    ctx->saved_data["scale"] = scale;
    return o;
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto sv = ctx->get_saved_variables();
    at::Tensor q = sv[0], k = sv[1], v = sv[2], o = sv[3], lse = sv[4];
    at::Tensor d = lastdim_contig(grads[0].to(q.scalar_type()));
    at::Tensor dq = at::empty_like(q), dk = at::empty_like(k), dv = at::empty_like(v);
    fa_bwd(q, k, v, o, lse, d, dq, dk, dv, ctx->saved_data["causal"].toBool(), ctx->saved_data["scale"].toDouble());
    return {dq, dk, dv, at::Tensor(), at::Tensor()};
  }
};

// qkv [B, S, H, 3, D] -> o [B, S, H, D]; the gradient is one dqkv buffer
struct FlashAttnQKVFn : public torch::autograd::Function<FlashAttnQKVFn> {
  static at::Tensor forward(AutogradContext* ctx, at::Tensor qkv, bool causal, double scale) {
    at::Tensor o, lse;
    fa_fwd(qkv.select(3, 0), qkv.select(3, 1), qkv.select(3, 2), o, lse, causal, scale);
    ctx->save_for_backward({qkv, o, lse});
    ctx->saved_data["causal"] = causal;
    ctx->saved_data["scale"] = scale;
    return o;
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto sv = ctx->get_saved_variables();
    at::Tensor qkv = sv[0], o = sv[1], lse = sv[2];
    at::Tensor d = lastdim_contig(grads[0].to(qkv.scalar_type()));
    at::Tensor g = at::empty_like(qkv);
    fa_bwd(qkv.select(3, 0), qkv.select(3, 1), qkv.select(3, 2), o, lse, d, g.select(3, 0), g.select(3, 1),
           g.select(3, 2), ctx->saved_data["causal"].toBool(), ctx->saved_data["scale"].toDouble());
    return {g, at::Tensor(), at::Tensor()};
  }
};

// ------------------------------------------------------------------------------------------------ cross entropy
// per-row loss (fp32, labels' shape) = logsumexp(logits) - logits[label]; 0 where label == ignore_index
struct SoftmaxCEFn : public torch::autograd::Function<SoftmaxCEFn> {
  static at::Tensor forward(AutogradContext* ctx, at::Tensor logits, at::Tensor labels, int64_t ignore) {
    const int64_t V = logits.size(-1);
    at::Tensor lg = logits.reshape({-1, V}).contiguous();
    at::Tensor lb = labels.reshape({-1}).to(at::kLong).contiguous();
    const int64_t rows = lg.size(0);
    at::Tensor loss = at::empty({rows}, lg.options().dtype(at::kFloat));
    at::Tensor lse = at::empty({rows}, lg.options().dtype(at::kFloat));
    chk(pa_softmax_ce_fwd(lg.data_ptr(), lb.data_ptr<int64_t>(), loss.data_ptr<float>(), lse.data_ptr<float>(), rows,
                          V, ignore, dcode(lg), stream()),
        "softmax_ce");
    count("softmax_ce");
    ctx->save_for_backward({lg, lb, lse});
    ctx->saved_data["ignore"] = ignore;
    ctx->saved_data["shape"] = logits.sizes().vec();
    std::vector<int64_t> out(logits.sizes().begin(), logits.sizes().end() - 1);
    return out_alias(loss, out);
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto sv = ctx->get_saved_variables();
    at::Tensor lg = sv[0], lb = sv[1], lse = sv[2];
    const int64_t rows = lg.size(0), V = lg.size(1);
    at::Tensor dl = grads[0].reshape({-1}).to(at::kFloat).contiguous();
    at::Tensor dlog = at::empty_like(lg);
    chk(pa_softmax_ce_bwd(lg.data_ptr(), lb.data_ptr<int64_t>(), lse.data_ptr<float>(), dl.data_ptr<float>(),
                          dlog.data_ptr(), rows, V, ctx->saved_data["ignore"].toInt(), dcode(lg), stream()),
        "softmax_ce_bwd");
    return {dlog.view(ctx->saved_data["shape"].toIntVector()), at::Tensor(), at::Tensor()};
  }
};

// ------------------------------------------------------------------------------------------------ convolution
at::Tensor zero_page(const at::Tensor& like) {
  static std::unordered_map<int, at::Tensor> pages;
  const int dev = like.get_device();
  auto it = pages.find(dev);
  if (it == pages.end())
    it = pages.emplace(dev, at::zeros({128}, like.options().dtype(at::kBFloat16))).first;
  return it->second;
}

// NHWC implicit-GEMM forward: x [N, H, W, C], wk [Cout, KH, KW, C] -> [N, Ho, Wo, Cout]
at::Tensor implicit_fwd(const at::Tensor& x, const at::Tensor& wk, const at::Tensor& b, int64_t Cout, int64_t KH,
                        int64_t KW, int64_t stride, int64_t ph, int64_t pw, int64_t dil) {
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int64_t Ho = (H + 2 * ph - dil * (KH - 1) - 1) / stride + 1;
  const int64_t Wo = (W + 2 * pw - dil * (KW - 1) - 1) / stride + 1;
  at::Tensor out = at::empty({N, Ho, Wo, Cout}, x.options());
  chk(pa_conv2d_nhwc_fwd(x.data_ptr(), wk.data_ptr(), ptr_or_null(b), out.data_ptr(), zero_page(x).data_ptr(),
                         (int)N, (int)H, (int)W, (int)C, (int)Cout, (int)KH, (int)KW, (int)stride, (int)ph, (int)pw,
                         (int)dil, (int)Ho, (int)Wo, stream()),
      "conv2d");
  count("conv2d");
  return out;
}

int wgrad_splits(int64_t P, int64_t M, int64_t N, int64_t bn) {
  const int64_t tiles = ((M + 255) / 256) * ((N + bn - 1) / bn);
  int64_t s = 1;
  while (tiles * s * 2 <= 2 * 256 && P % (64 * s * 2) == 0 && (s * 2) * M * N * 4 <= (256LL << 20)) s *= 2;
  return static_cast<int>(s);
}

// the NHWC convolution for an NCHW *view* of channels-last storage (how a traced NHWC model hands its activations
// to conv2d): x_nchw = x_nhwc.permute(0, 3, 1, 2); the output is returned the same way
bool conv_ok(const at::Tensor& x, const at::Tensor& w, int64_t groups) {
  if (!x.is_cuda() || x.dim() != 4 || w.dim() != 4 || groups != 1) return false;
  if (x.scalar_type() != at::kBFloat16 || w.scalar_type() != at::kBFloat16) return false;
  if (!x.permute({0, 2, 3, 1}).is_contiguous() || x.numel() == 0) return false;
  return x.size(1) % 64 == 0 && w.size(0) % 8 == 0;
}

struct ConvNHWCFn : public torch::autograd::Function<ConvNHWCFn> {
  static at::Tensor forward(AutogradContext* ctx, at::Tensor x, at::Tensor w, at::Tensor b, int64_t stride,
                            int64_t ph, int64_t pw, int64_t dil) {
    b = present(b);
    at::Tensor xh = x.permute({0, 2, 3, 1});
    at::Tensor wk = w.permute({0, 2, 3, 1}).contiguous();
    at::Tensor bb = b.defined() ? b.to(x.scalar_type()).contiguous() : at::Tensor();
    at::Tensor y = implicit_fwd(xh, wk, bb, w.size(0), w.size(2), w.size(3), stride, ph, pw, dil);
    ctx->save_for_backward({xh, w});
    ctx->saved_data["cfg"] = std::vector<int64_t>{stride, ph, pw, dil, b.defined() ? 1 : 0};
    ctx->saved_data["bdt"] = static_cast<int64_t>(b.defined() ? b.scalar_type() : x.scalar_type());
    return y.permute({0, 3, 1, 2});
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto sv = ctx->get_saved_variables();
    at::Tensor xh = sv[0], w = sv[1];
    auto cfg = ctx->saved_data["cfg"].toIntVector();
    const int64_t stride = cfg[0], ph = cfg[1], pw = cfg[2], dil = cfg[3];
    const int64_t N = xh.size(0), H = xh.size(1), W = xh.size(2), C = xh.size(3);
    const int64_t Cout = w.size(0), KH = w.size(2), KW = w.size(3);
    at::Tensor dyh = grads[0].permute({0, 2, 3, 1}).to(xh.scalar_type()).contiguous();
    const int64_t Ho = dyh.size(1), Wo = dyh.size(2);
    at::Tensor dx, dw, db;
    const bool own_dx = ctx->needs_input_grad(0) && stride == 1 && dil == 1 && Cout % 64 == 0 && C % 8 == 0 &&
                        KH == KW && ph == pw && ph <= KH - 1;
    if (own_dx) {  // the transposed convolution: flipped filter, channel axes swapped, padding KH - 1 - pad
      at::Tensor wt = w.flip({2, 3}).permute({1, 2, 3, 0}).contiguous();
      dx = implicit_fwd(dyh, wt, at::Tensor(), C, KH, KW, 1, KH - 1 - ph, KW - 1 - pw, 1);
    }
    const int64_t P = N * Ho * Wo;
    const bool own_dw = ctx->needs_input_grad(1) && C % 8 == 0 && Cout % 8 == 0 && P % 64 == 0;
    if (own_dw) {  // split-K implicit GEMM gathering the im2col rows of x on the fly
      const int64_t M = KH * KW * C;
      const int64_t bn = Cout % 256 == 0 ? 256 : (Cout <= 64 ? 64 : 128);
      const int splits = wgrad_splits(P, M, Cout, bn);
      at::Tensor ws = at::empty({splits, M, Cout}, xh.options().dtype(at::kFloat));
      chk(pa_conv2d_nhwc_wgrad(xh.data_ptr(), dyh.data_ptr(), ws.data_ptr<float>(), zero_page(xh).data_ptr(), (int)N,
                               (int)H, (int)W, (int)C, (int)Cout, (int)KH, (int)KW, (int)stride, (int)ph, (int)pw,
                               (int)dil, (int)Ho, (int)Wo, splits, (int)bn, stream()),
          "conv2d_wgrad");
      count("conv2d_wgrad");
      dw = ws.sum(0).view({KH, KW, C, Cout}).permute({3, 2, 0, 1}).to(w.scalar_type()).contiguous();
    }
    const bool need_dx = ctx->needs_input_grad(0) && !own_dx, need_dw = ctx->needs_input_grad(1) && !own_dw;
    if (need_dx || need_dw) {
      auto r = at::convolution_backward(dyh.permute({0, 3, 1, 2}), xh.permute({0, 3, 1, 2}), w, c10::nullopt,
                                        {stride, stride}, {ph, pw}, {dil, dil}, false, {0, 0}, 1,
                                        {need_dx, need_dw, false});
      if (need_dx) dx = std::get<0>(r).permute({0, 2, 3, 1}).contiguous();
      if (need_dw) dw = std::get<1>(r);
    }
    if (cfg[4] && ctx->needs_input_grad(2))
      db = dyh.to(at::kFloat).sum({0, 1, 2}).to(static_cast<at::ScalarType>(ctx->saved_data["bdt"].toInt()));
    return {dx.defined() ? dx.permute({0, 3, 1, 2}) : dx, dw, db, at::Tensor(), at::Tensor(), at::Tensor(),
            at::Tensor()};
  }
};

// ------------------------------------------------------------------------------------------------ batch norm
// y = act(bn(x) [+ residual]) over the channel (last) dim of x2 [R, C] bf16; weight / bias / running stats fp32
struct BNActFn : public torch::autograd::Function<BNActFn> {
  static at::Tensor forward(AutogradContext* ctx, at::Tensor x2, at::Tensor w, at::Tensor b, at::Tensor res,
                            at::Tensor rm, at::Tensor rv, bool training, double momentum, double eps, bool relu) {
    w = present(w);
    b = present(b);
    res = present(res);
    rm = present(rm);
    rv = present(rv);
    const int64_t R = x2.size(0);
    const int C = static_cast<int>(x2.size(1));
    at::Tensor y = at::empty_like(x2);
    at::Tensor ss = at::empty({2, C}, x2.options().dtype(at::kFloat));
    at::Tensor mean, rstd, partial;
    if (training) {
      mean = at::empty({C}, x2.options().dtype(at::kFloat));
      rstd = at::empty({C}, x2.options().dtype(at::kFloat));
      partial = at::empty({2 * static_cast<int64_t>(pa_bn_chunks(R, C)) * C}, x2.options().dtype(at::kFloat));
    } else {
      mean = rm.to(at::kFloat).contiguous();
      rstd = at::rsqrt(rv.to(at::kFloat) + eps);
      at::Tensor wf = w.defined() ? w.to(at::kFloat) : at::ones_like(mean);
      at::Tensor bf = b.defined() ? b.to(at::kFloat) : at::zeros_like(mean);
      ss[0].copy_(wf * rstd);
      ss[1].copy_(bf - mean * wf * rstd);
    }
    chk(pa_bn_fwd_nhwc(x2.data_ptr(), ptr_or_null(res), y.data_ptr(), w.defined() ? w.data_ptr<float>() : nullptr,
                       b.defined() ? b.data_ptr<float>() : nullptr, training ? rm.data_ptr<float>() : nullptr,
                       training ? rv.data_ptr<float>() : nullptr, mean.data_ptr<float>(), rstd.data_ptr<float>(),
                       training ? partial.data_ptr<float>() : nullptr, ss.data_ptr<float>(), R, C,
                       static_cast<float>(momentum), static_cast<float>(eps), relu ? 1 : 0, training ? 1 : 0,
                       stream()),
        "batch_norm");
    count("batch_norm");
    ctx->save_for_backward({x2, relu ? y : at::Tensor(), w, mean, rstd});
    ctx->saved_data["flags"] = std::vector<int64_t>{relu, training, res.defined(), w.defined(), b.defined()};
    return y;
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto sv = ctx->get_saved_variables();
    at::Tensor x2 = sv[0], y = sv[1], w = sv[2], mean = sv[3], rstd = sv[4];
    auto f = ctx->saved_data["flags"].toIntVector();
    const int64_t R = x2.size(0);
    const int C = static_cast<int>(x2.size(1));
    at::Tensor dy = grads[0].to(x2.scalar_type()).contiguous();
    at::Tensor dx = at::empty_like(x2);
    at::Tensor dres = f[2] ? at::empty_like(x2) : at::Tensor();
    at::Tensor dw = f[3] ? at::empty({C}, x2.options().dtype(at::kFloat)) : at::Tensor();
    at::Tensor db = f[4] ? at::empty({C}, x2.options().dtype(at::kFloat)) : at::Tensor();
    at::Tensor partial = at::empty({2 * static_cast<int64_t>(pa_bn_chunks(R, C)) * C}, x2.options().dtype(at::kFloat));
    at::Tensor coef = at::empty({3, C}, x2.options().dtype(at::kFloat));
    chk(pa_bn_bwd_nhwc(dy.data_ptr(), x2.data_ptr(), ptr_or_null(y), dx.data_ptr(),
                       dres.defined() ? dres.data_ptr() : nullptr, w.defined() ? w.data_ptr<float>() : nullptr,
                       mean.data_ptr<float>(), rstd.data_ptr<float>(), dw.defined() ? dw.data_ptr<float>() : nullptr,
                       db.defined() ? db.data_ptr<float>() : nullptr, partial.data_ptr<float>(),
                       coef.data_ptr<float>(), R, C, (int)f[0], f[1] ? 0 : 1, nullptr, stream()),
        "batch_norm_bwd");
    count("batch_norm_bwd");
    return {dx, dw, db, dres, at::Tensor(), at::Tensor(), at::Tensor(), at::Tensor(), at::Tensor(), at::Tensor()};
  }
};

bool bn_ok(const at::Tensor& x2, const at::Tensor& w, const at::Tensor& b, const at::Tensor& res,
           const at::Tensor& rm, const at::Tensor& rv) {
  if (!x2.is_cuda() || x2.scalar_type() != at::kBFloat16 || x2.size(1) % 8 != 0 || !x2.is_contiguous()) return false;
  for (const at::Tensor* t : {&w, &b, &rm, &rv})
    if (t->defined() && (t->scalar_type() != at::kFloat || !t->is_contiguous())) return false;
  return !res.defined() || (res.scalar_type() == at::kBFloat16 && res.is_contiguous());
}

// ------------------------------------------------------------------------------------------------ program
enum Kind : int { kAten = 0, kLinear, kLinearNT, kNorm, kFlash, kFlashQKV, kSoftmaxCE, kConv, kBN, kAlias, kComm, kPy };

enum ArgKind : int { kSlot = 0, kSlotList = 1, kConst = 2, kRunDevice = 3, kOptSlotList = 4 };

struct Arg {
  int kind = kConst;
  int slot = -1;
  std::vector<int> slots;
  c10::IValue value;
};

struct Instr {
  int kind = kAten;
  std::string name;
  c10::optional<c10::OperatorHandle> op;
  std::vector<Arg> args;
  std::vector<std::vector<int>> outs;  // per return: its slot (or the slots of a tensor-list return)
  std::vector<int> in;                 // native instructions: operand slots (-1 = absent)
  std::vector<int64_t> ia;             // native instructions: int attributes
  std::vector<double> fa;              // native instructions: float attributes
};

struct OptGroup {  // one optimizer instruction
  int kind = 0;    // 1 adam(w), 2 momentum
  std::vector<at::Tensor> params, masters, m1, m2, lowp;  // m1: moment1 / velocity; m2 adam only
  std::vector<double> coeff, lr_mult;
  at::Tensor table, items;
  int64_t n_items = 0;
  std::vector<void*> table_key;
};

constexpr int64_t kChunk = 65536;  // elements per (tensor, chunk) work item (optimizer/optimizer.py _CHUNK)

int32_t f2i(double x) {
  float f = static_cast<float>(x);
  int32_t i;
  std::memcpy(&i, &f, 4);
  return i;
}

class TrainProgram {
 public:
  TrainProgram(int n_slots, std::string device) : slots_(n_slots), device_(std::move(device)) {}

  int grow(int n) {
    if (n > static_cast<int>(slots_.size())) slots_.resize(n);
    return static_cast<int>(slots_.size());
  }

  void add_aten(const std::string& name, const std::string& overload, py::list args, py::list outs) {
    Instr I;
    I.kind = kAten;
    I.name = name + "." + overload;
    I.op = c10::Dispatcher::singleton().findSchemaOrThrow(name.c_str(), overload.c_str());
    const auto& schema = I.op->schema();
    if (args.size() != schema.arguments().size())
      throw std::runtime_error("native train executor: " + I.name + " expects " +
                               std::to_string(schema.arguments().size()) + " arguments, got " +
                               std::to_string(args.size()));
    for (size_t i = 0; i < args.size(); ++i) {
      py::tuple a = args[i].cast<py::tuple>();
      Arg x;
      x.kind = a[0].cast<int>();
      if (x.kind == kSlot) {
        x.slot = a[1].cast<int>();
      } else if (x.kind == kSlotList || x.kind == kOptSlotList) {
        for (auto s : a[1]) x.slots.push_back(py::cast<int>(s));
      } else if (x.kind == kConst) {
        x.value = torch::jit::toIValue(a[1], schema.arguments()[i].type());
      }
      I.args.push_back(std::move(x));
    }
    for (auto o : outs) {
      std::vector<int> v;
      if (py::isinstance<py::list>(o)) {
        for (auto s : o) v.push_back(py::cast<int>(s));
      } else {
        v.push_back(py::cast<int>(o));
      }
      I.outs.push_back(std::move(v));
    }
    code_.push_back(std::move(I));
  }

  void add_native(const std::string& kind, std::vector<int> in, std::vector<int> outs, std::vector<int64_t> ia,
                  std::vector<double> fa) {
    static const std::unordered_map<std::string, int> kinds = {
        {"linear", kLinear}, {"linear_nt", kLinearNT}, {"norm", kNorm},     {"flash_attention", kFlash},
        {"flash_attention_qkvpacked", kFlashQKV},      {"softmax_ce", kSoftmaxCE},
        {"conv2d", kConv},   {"batch_norm_act", kBN},  {"alias", kAlias}};
    auto it = kinds.find(kind);
    if (it == kinds.end()) throw std::runtime_error("native train executor: unknown native op " + kind);
    Instr I;
    I.kind = it->second;
    I.name = kind;
    I.in = std::move(in);
    for (int s : outs) I.outs.push_back({s});
    I.ia = std::move(ia);
    I.fa = std::move(fa);
    code_.push_back(std::move(I));
  }

  // a collective of the program (in place on its operand slots): run on the program's communication stream, after
  // the compute stream's work so far (its inputs exist); a later instruction reading a slot it wrote waits for it
  // with an event (reference new_executor/interpreter/stream_analyzer.cc: communication ops on their own stream,
  // cross-stream dependencies as events; dependency_builder.cc: read-after-write edges on the written vars)
  void add_comm(py::object fn, std::vector<int> slots, const std::string& name) {
    Instr I;
    I.kind = kComm;
    I.name = name;
    I.in = std::move(slots);
    I.ia = {static_cast<int64_t>(comm_fns_.size())};
    comm_fns_.push_back(std::move(fn));
    code_.push_back(std::move(I));
  }

  // an op run through Python (an op of this framework the native kinds do not cover, a collective with autograd
  // semantics of a partitioned program): fn(*operand tensors) -> tensor / sequence of tensors into ``outs``;
  // autograd records whatever the op records
  void add_py(py::object fn, std::vector<int> in, std::vector<int> outs, const std::string& name) {
    Instr I;
    I.kind = kPy;
    I.name = name;
    I.in = std::move(in);
    for (int o : outs) I.outs.push_back({o});
    I.ia = {static_cast<int64_t>(comm_fns_.size())};
    comm_fns_.push_back(std::move(fn));
    code_.push_back(std::move(I));
  }

  // parameters (leaf tensors requiring grad), buffers and constants: persistent slots
  void bind(int slot, at::Tensor t) {
    grow(slot + 1);
    slots_.at(slot) = std::move(t);
    persistent_.push_back(slot);
  }

  void set_loss(int slot) { loss_ = slot; }

  // called with the optimizer parameters' gradients after the backward, before clipping / the update (static
  // collective data parallelism: the gradient all-reduce over the data-parallel group)
  void set_grad_hook(py::object fn) { grad_hook_ = std::move(fn); }

  // one optimizer group: masters[i] is read only where has_master[i] (fp32 master weights of low-precision params)
  void add_optimizer(const std::string& kind, std::vector<at::Tensor> params, std::vector<at::Tensor> masters,
                     std::vector<int64_t> has_master, std::vector<at::Tensor> m1, std::vector<at::Tensor> m2,
                     std::vector<double> coeff, std::vector<double> lr_mult) {
    OptGroup g;
    if (kind == "adam") g.kind = 1;
    else if (kind == "momentum") g.kind = 2;
    else throw std::runtime_error("native train executor: unknown optimizer " + kind);
    g.params = std::move(params);
    g.masters = std::move(masters);
    for (size_t i = 0; i < g.masters.size(); ++i)
      if (!has_master.at(i)) g.masters[i] = at::Tensor();
    g.m1 = std::move(m1);
    g.m2 = std::move(m2);
    g.coeff = std::move(coeff);
    g.lr_mult = std::move(lr_mult);
    opt_.push_back(std::move(g));
  }

  // last readers of every slot: a non-persistent slot is released right after it (autograd keeps what it saved)
  void finalize(std::vector<int> fetch) {
    fetch_ = std::move(fetch);
    std::vector<char> keep(slots_.size(), 0);
    for (int s : persistent_) keep.at(s) = 1;
    for (int s : fetch_) keep.at(s) = 1;
    if (loss_ >= 0) keep.at(loss_) = 1;
    std::vector<int> last(slots_.size(), -1);
    auto reads = [&](const Instr& I, auto&& fn) {
      for (const Arg& a : I.args) {
        if (a.kind == kSlot && a.slot >= 0) fn(a.slot);
        if (a.kind == kSlotList || a.kind == kOptSlotList)
          for (int s : a.slots)
            if (s >= 0) fn(s);
      }
      for (int s : I.in)
        if (s >= 0) fn(s);
    };
    for (size_t n = 0; n < code_.size(); ++n) reads(code_[n], [&](int s) { last.at(s) = static_cast<int>(n); });
    reads_.assign(code_.size(), {});
    for (size_t n = 0; n < code_.size(); ++n) reads(code_[n], [&](int s) { reads_[n].push_back(s); });
    release_.assign(code_.size(), {});
    for (size_t s = 0; s < last.size(); ++s)
      if (last[s] >= 0 && !keep[s]) release_[last[s]].push_back(static_cast<int>(s));
    for (size_t n = 0; n < code_.size(); ++n)
      for (const auto& o : code_[n].outs)
        for (int s : o)
          if (s >= 0 && last.at(s) < 0 && !keep[s]) release_[n].push_back(s);
  }

  // scalars: per optimizer group {lr, b1, b2, eps, bc1, bc2} (adam) or {lr, mu, rescale, nesterov} (momentum);
  // clip_norm > 0: global-norm clipping folded into the update
  std::vector<at::Tensor> run(const std::vector<std::pair<int, at::Tensor>>& feeds, bool backward,
                              std::vector<std::vector<double>> scalars, double clip_norm) {
    for (const auto& f : feeds) slots_.at(f.first) = f.second;
    at::Tensor loss;
    // progress of this run, read by the executor when it raised: a failed step may be replayed elsewhere only if
    // it failed in the forward before any instruction with device side effects completed
    phase_ = 0;
    done_ = 0;
    {
      at::AutoGradMode grad_mode(backward);
      for (size_t n = 0; n < code_.size(); ++n) {
        if (code_[n].kind == kComm) {
          exec_comm(code_[n]);
        } else {
          wait_pending(n);
          exec(code_[n]);
        }
        done_ = static_cast<int64_t>(n) + 1;
        for (int s : release_[n]) slots_[s] = at::Tensor();
      }
      join_comm();
      if (backward) {
        phase_ = 1;
        loss = slots_.at(loss_);
        zero_grads();
        torch::autograd::backward({loss});
      }
    }
    if (backward && !opt_.empty() && grad_hook_ && !grad_hook_.is_none()) {
      phase_ = 2;
      std::vector<at::Tensor> gs;
      for (auto& g : opt_)
        for (auto& p : g.params)
          if (p.grad().defined()) gs.push_back(p.grad());
      py::gil_scoped_acquire gil;  // run() is bound with the GIL released
      grad_hook_(gs);
    }
    if (backward && !opt_.empty()) {
      phase_ = 3;
      at::NoGradGuard ng;
      at::Tensor inv_scale = clip_norm > 0 ? clip_coef(clip_norm) : at::Tensor();
      for (size_t g = 0; g < opt_.size(); ++g) step(opt_[g], g < scalars.size() ? scalars[g] : std::vector<double>{},
                                                     inv_scale);
    }
    std::vector<at::Tensor> out;
    for (int s : fetch_) out.push_back(slots_[s].defined() ? slots_[s].detach() : slots_[s]);
    for (const auto& f : feeds) slots_[f.first] = at::Tensor();
    for (int s : fetch_) {
      bool persistent = false;
      for (int p : persistent_) persistent |= p == s;
      if (!persistent) slots_[s] = at::Tensor();
    }
    if (loss_ >= 0) slots_[loss_] = at::Tensor();
    return out;
  }

  int64_t num_instructions() const { return static_cast<int64_t>(code_.size()); }
  // forward only, autograd recording (a pipeline stage's micro-batch: the caller runs the backward): the fetch slots'
  // values with their autograd history; intermediates released after their last reader
  std::vector<at::Tensor> forward(const std::vector<std::pair<int, at::Tensor>>& feeds) {
    for (const auto& f : feeds) slots_.at(f.first) = f.second;
    phase_ = 0;
    done_ = 0;
    {
      at::AutoGradMode grad_mode(true);
      for (size_t n = 0; n < code_.size(); ++n) {
        if (code_[n].kind == kComm) {
          exec_comm(code_[n]);
        } else {
          wait_pending(n);
          exec(code_[n]);
        }
        done_ = static_cast<int64_t>(n) + 1;
        for (int s : release_[n]) slots_[s] = at::Tensor();
      }
      join_comm();
    }
    std::vector<at::Tensor> out;
    for (int s : fetch_) out.push_back(slots_[s]);
    for (const auto& f : feeds) slots_[f.first] = at::Tensor();
    for (int s : fetch_) {
      bool persistent = false;
      for (int p : persistent_) persistent |= p == s;
      if (!persistent) slots_[s] = at::Tensor();
    }
    return out;
  }

  int64_t num_comm() const {
    int64_t n = 0;
    for (const auto& I : code_) n += I.kind == kComm;
    return n;
  }

  ~TrainProgram() {
    for (hipEvent_t e : events_) (void)hipEventDestroy(e);
    py::gil_scoped_acquire gil;
    comm_fns_.clear();
  }
  // phase of the last run when it stopped (0 forward, 1 backward, 2 gradient hook, 3 update) and the number of
  // forward instructions it completed
  int64_t phase() const { return phase_; }
  int64_t done() const { return done_; }
  int64_t num_native() const {
    int64_t n = 0;
    for (const auto& I : code_) n += I.kind != kAten && I.kind != kAlias && I.kind != kComm && I.kind != kPy;
    return n;
  }

 private:
  // persistent gradient buffers: zeroed in place each step, so autograd accumulates into the same storage and the
  // optimizer's pointer table stays valid
  void zero_grads() {
    for (auto& g : opt_)
      for (auto& p : g.params) {
        at::Tensor gr = p.mutable_grad();
        if (gr.defined()) gr.zero_();
      }
  }

  at::Tensor clip_coef(double clip) {
    std::vector<at::Tensor> gs;
    for (auto& g : opt_)
      for (auto& p : g.params)
        if (p.grad().defined()) gs.push_back(p.grad());
    if (gs.empty()) return at::Tensor();
    auto norms = at::_foreach_norm(gs, 2);
    at::Tensor total = at::stack(norms).to(at::kFloat).square().sum().sqrt();
    return (clip / at::clamp_min(total, clip)).reshape({1}).contiguous();
  }

  void build_table(OptGroup& g) {
    std::vector<void*> key;
    for (auto& p : g.params) key.push_back(p.grad().defined() ? p.grad().data_ptr() : nullptr);
    if (g.table.defined() && key == g.table_key) return;
    std::vector<int64_t> rows, items;
    for (size_t i = 0; i < g.params.size(); ++i) {
      at::Tensor p = g.params[i];
      at::Tensor gr = p.grad();
      if (!gr.defined()) throw std::runtime_error("native train executor: a parameter got no gradient");
      at::Tensor w = g.masters[i].defined() ? g.masters[i] : p;
      const int64_t n = w.numel();
      const int64_t gdt = dcode(gr), ldt = g.masters[i].defined() ? dcode(p) : 3;
      if (g.kind == 1) {
        rows.insert(rows.end(), {reinterpret_cast<int64_t>(w.data_ptr()), reinterpret_cast<int64_t>(gr.data_ptr()),
                                 reinterpret_cast<int64_t>(g.m1[i].data_ptr()),
                                 reinterpret_cast<int64_t>(g.m2[i].data_ptr()),
                                 g.masters[i].defined() ? reinterpret_cast<int64_t>(p.data_ptr()) : 0, n,
                                 gdt | (ldt << 8), f2i(g.coeff[i]), f2i(g.lr_mult[i])});
      } else {
        rows.insert(rows.end(), {reinterpret_cast<int64_t>(w.data_ptr()), reinterpret_cast<int64_t>(gr.data_ptr()),
                                 reinterpret_cast<int64_t>(g.m1[i].data_ptr()), 0,
                                 g.masters[i].defined() ? reinterpret_cast<int64_t>(p.data_ptr()) : 0, n,
                                 gdt | (ldt << 8), f2i(g.coeff[i]), f2i(g.lr_mult[i])});
      }
      for (int64_t s = 0; s < n; s += kChunk) items.insert(items.end(), {static_cast<int64_t>(i), s});
    }
    auto opts = at::TensorOptions().dtype(at::kLong);
    at::Tensor dev_opts = g.params[0];
    g.table = at::tensor(rows, opts).to(dev_opts.device());
    g.items = at::tensor(items, opts).to(dev_opts.device());
    g.n_items = static_cast<int64_t>(items.size() / 2);
    g.table_key = std::move(key);
  }

  void step(OptGroup& g, const std::vector<double>& s, const at::Tensor& inv_scale) {
    if (g.params.empty()) return;
    if (!g.params[0].is_cuda()) throw std::runtime_error("native train executor: optimizer kernels need a GPU");
    build_table(g);
    const float* inv = inv_scale.defined() ? inv_scale.data_ptr<float>() : nullptr;
    if (g.kind == 1) {
      if (s.size() != 6) throw std::runtime_error("native train executor: adam needs {lr, b1, b2, eps, bc1, bc2}");
      chk(pa_adamw_multi(g.table.data_ptr<int64_t>(), g.items.data_ptr<int64_t>(), g.n_items, inv, (float)s[0],
                         (float)s[1], (float)s[2], (float)s[3], 0.f, (float)s[4], (float)s[5], nullptr, stream()),
          "adamw");
      count("adamw");
    } else {
      if (s.size() != 4) throw std::runtime_error("native train executor: momentum needs {lr, mu, rescale, nesterov}");
      chk(pa_momentum_multi(g.table.data_ptr<int64_t>(), g.items.data_ptr<int64_t>(), g.n_items, inv, (float)s[0],
                            (float)s[1], (float)s[2], (int)s[3], stream()),
          "momentum");
      count("momentum");
    }
  }

  at::Tensor slot(int s) const { return s >= 0 ? slots_.at(s) : at::Tensor(); }

  // ---- communication stream
  hipEvent_t next_event() {
    if (ev_next_ == events_.size()) {
      hipEvent_t e;
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
        throw std::runtime_error("native train executor: hipEventCreate failed");
      events_.push_back(e);
    }
    return events_[ev_next_++];
  }

  void exec_comm(const Instr& I) {
    std::vector<at::Tensor> ts;
    for (int s : I.in) ts.push_back(slots_.at(s));
    const bool gpu = !ts.empty() && ts[0].is_cuda();
    if (!gpu) {  // host collectives (gloo on CPU tensors): in program order on the caller's thread
      py::gil_scoped_acquire gil;
      py::tuple args(ts.size());
      for (size_t i = 0; i < ts.size(); ++i) args[i] = py::cast(ts[i]);
      comm_fns_.at(I.ia[0])(*args);
      count("comm");
      return;
    }
    const c10::DeviceIndex dev = ts[0].device().index();
    if (!comm_stream_) comm_stream_ = c10::hip::getStreamFromPool(false, dev);
    hipStream_t comp = c10::hip::getCurrentHIPStream(dev).stream();
    hipEvent_t ready = next_event();  // the collective's inputs: everything issued on the compute stream so far
    if (hipEventRecord(ready, comp) != hipSuccess || hipStreamWaitEvent(comm_stream_->stream(), ready, 0) != hipSuccess)
      throw std::runtime_error("native train executor: stream dependency failed");
    {
      c10::hip::HIPStreamGuard guard(*comm_stream_);
      py::gil_scoped_acquire gil;
      py::tuple args(ts.size());
      for (size_t i = 0; i < ts.size(); ++i) args[i] = py::cast(ts[i]);
      comm_fns_.at(I.ia[0])(*args);
    }
    hipEvent_t done = next_event();
    if (hipEventRecord(done, comm_stream_->stream()) != hipSuccess)
      throw std::runtime_error("native train executor: hipEventRecord failed");
    for (int s : I.in) pending_[s] = done;
    for (auto& t : ts) comm_keep_.push_back(t);  // alive (not reused by the compute stream) until join_comm
    count("comm");
  }

  // a compute instruction reading a slot a collective wrote: the compute stream waits for that collective
  void wait_pending(size_t n) {
    if (pending_.empty()) return;
    for (int s : reads_[n]) {
      auto it = pending_.find(s);
      if (it == pending_.end()) continue;
      hipStream_t comp = c10::hip::getCurrentHIPStream().stream();
      if (hipStreamWaitEvent(comp, it->second, 0) != hipSuccess)
        throw std::runtime_error("native train executor: hipStreamWaitEvent failed");
      pending_.erase(it);
    }
  }

  // end of the forward: the compute stream waits for every outstanding collective; their operands may be freed
  void join_comm() {
    if (comm_stream_ && ev_next_ > 0) {
      hipEvent_t all = next_event();
      hipStream_t comp = c10::hip::getCurrentHIPStream().stream();
      if (hipEventRecord(all, comm_stream_->stream()) != hipSuccess || hipStreamWaitEvent(comp, all, 0) != hipSuccess)
        throw std::runtime_error("native train executor: stream join failed");
    }
    pending_.clear();
    comm_keep_.clear();
    ev_next_ = 0;
  }
  void put(const Instr& I, size_t k, const at::Tensor& t) {
    if (k < I.outs.size() && !I.outs[k].empty() && I.outs[k][0] >= 0) slots_[I.outs[k][0]] = t;
  }

  void exec(Instr& I) {
    switch (I.kind) {
      case kAten: {
        torch::jit::Stack stack;
        stack.reserve(I.args.size());
        for (const Arg& a : I.args) {
          switch (a.kind) {
            case kSlot: stack.emplace_back(a.slot >= 0 ? c10::IValue(slots_.at(a.slot)) : c10::IValue()); break;
            case kSlotList: {
              std::vector<at::Tensor> v;
              for (int s : a.slots) v.push_back(slots_.at(s));
              stack.emplace_back(v);
              break;
            }
            case kOptSlotList: {
              c10::List<c10::optional<at::Tensor>> v;
              for (int s : a.slots) v.push_back(s >= 0 ? c10::optional<at::Tensor>(slots_.at(s)) : c10::nullopt);
              stack.emplace_back(v);
              break;
            }
            case kRunDevice: stack.emplace_back(c10::Device(device_)); break;
            default: stack.push_back(a.value);
          }
        }
        I.op->callBoxed(&stack);
        for (size_t r = 0; r < I.outs.size() && r < stack.size(); ++r) {
          const c10::IValue& v = stack[r];
          if (v.isTensor()) {
            if (!I.outs[r].empty() && I.outs[r][0] >= 0) slots_[I.outs[r][0]] = v.toTensor();
          } else if (v.isTensorList()) {
            auto lst = v.toTensorVector();
            for (size_t j = 0; j < lst.size() && j < I.outs[r].size(); ++j)
              if (I.outs[r][j] >= 0) slots_[I.outs[r][j]] = lst[j];
          }
        }
        break;
      }
      case kAlias: put(I, 0, slot(I.in[0])); break;
      case kLinear: {  // in: x, w, b; ia: act
        at::Tensor x = slot(I.in[0]), w = slot(I.in[1]), b = slot(I.in[2]);
        put(I, 0, LinearFn::apply(x, w, opt_in(b, x), I.ia[0]));
        break;
      }
      case kLinearNT: put(I, 0, LinearNTFn::apply(slot(I.in[0]), slot(I.in[1]))); break;
      case kNorm: {  // in: x, w, b; ia: rms; fa: eps
        at::Tensor x = slot(I.in[0]), w = slot(I.in[1]), b = slot(I.in[2]);
        if (norm_ok(x, w)) {
          put(I, 0, NormFn::apply(x, opt_in(w, x), opt_in(b, x), I.fa[0], I.ia[0] != 0));
        } else if (I.ia[0]) {
          at::Tensor xf = x.to(at::kFloat);
          at::Tensor y = (xf * at::rsqrt(xf.pow(2).mean({-1}, true) + I.fa[0])).to(x.scalar_type());
          put(I, 0, w.defined() ? y * w : y);
        } else {
          put(I, 0, at::layer_norm(x, {x.size(-1)}, w, b, I.fa[0]));
        }
        break;
      }
      case kFlash: {  // in: q, k, v; ia: causal; fa: scale
        at::Tensor q = slot(I.in[0]), k = slot(I.in[1]), v = slot(I.in[2]);
        if (!attn_ok(q, k, v))
          throw std::runtime_error("native train executor: flash_attention operands outside the kernel");
        put(I, 0, FlashAttnFn::apply(q, k, v, I.ia[0] != 0, I.fa[0]));
        break;
      }
      case kFlashQKV: {
        at::Tensor qkv = slot(I.in[0]);
        if (!attn_ok(qkv.select(3, 0), qkv.select(3, 1), qkv.select(3, 2)))
          throw std::runtime_error("native train executor: flash_attention_qkvpacked operands outside the kernel");
        put(I, 0, FlashAttnQKVFn::apply(qkv, I.ia[0] != 0, I.fa[0]));
        break;
      }
      case kSoftmaxCE: put(I, 0, SoftmaxCEFn::apply(slot(I.in[0]), slot(I.in[1]), I.ia[0])); break;
      case kConv: {  // in: x (NCHW view), w, b; ia: stride, ph, pw, dil, groups
        at::Tensor x = slot(I.in[0]), w = slot(I.in[1]), b = slot(I.in[2]);
        if (conv_ok(x, w, I.ia[4])) {
          put(I, 0, ConvNHWCFn::apply(x, w, opt_in(b, x), I.ia[0], I.ia[1], I.ia[2], I.ia[3]));
        } else {
          put(I, 0, at::conv2d(x, w, b.defined() ? c10::optional<at::Tensor>(b) : c10::nullopt, {I.ia[0], I.ia[0]},
                               {I.ia[1], I.ia[2]}, {I.ia[3], I.ia[3]}, I.ia[4]));
        }
        break;
      }
      case kBN: {  // in: x, w, b, rm, rv, res; ia: training, relu; fa: momentum, eps
        at::Tensor x = slot(I.in[0]), w = slot(I.in[1]), b = slot(I.in[2]), rm = slot(I.in[3]), rv = slot(I.in[4]),
                   res = slot(I.in[5]);
        const int64_t C = x.size(-1);
        at::Tensor x2 = x.reshape({-1, C});
        at::Tensor r2 = res.defined() ? res.reshape({-1, C}) : res;
        if (!bn_ok(x2, w, b, r2, rm, rv))
          throw std::runtime_error("native train executor: batch_norm_act operands outside the kernel");
        put(I, 0, BNActFn::apply(x2, opt_in(w, x2), opt_in(b, x2), opt_in(r2, x2), opt_in(rm, x2), opt_in(rv, x2),
                                 I.ia[0] != 0, I.fa[0], I.fa[1], I.ia[1] != 0)
                      .view(x.sizes()));
        break;
      }
      case kPy: {
        py::gil_scoped_acquire gil;
        py::tuple args(I.in.size());
        for (size_t i = 0; i < I.in.size(); ++i)
          args[i] = I.in[i] >= 0 && slots_.at(I.in[i]).defined() ? py::cast(slots_.at(I.in[i])) : py::none();
        py::object r = comm_fns_.at(I.ia[0])(*args);
        if (THPVariable_Check(r.ptr())) {
          put(I, 0, THPVariable_Unpack(r.ptr()));
        } else if (py::isinstance<py::tuple>(r) || py::isinstance<py::list>(r)) {
          auto seq = r.cast<py::sequence>();
          for (size_t k = 0; k < seq.size() && k < I.outs.size(); ++k) {
            py::object e = seq[k];
            if (THPVariable_Check(e.ptr())) put(I, k, THPVariable_Unpack(e.ptr()));
          }
        }
        count("py");
        break;
      }
      default: throw std::runtime_error("native train executor: bad instruction " + I.name);
    }
  }

  std::vector<at::Tensor> slots_;
  std::string device_;
  std::vector<Instr> code_;
  std::vector<int> persistent_, fetch_;
  std::vector<std::vector<int>> release_;
  std::vector<OptGroup> opt_;
  py::object grad_hook_;
  int64_t phase_ = 0, done_ = 0;
  std::vector<std::vector<int>> reads_;  // per instruction: slots it reads (event waits)
  std::vector<py::object> comm_fns_;
  c10::optional<c10::hip::HIPStream> comm_stream_;
  std::unordered_map<int, hipEvent_t> pending_;  // slot -> event of the collective that wrote it
  std::vector<hipEvent_t> events_;
  size_t ev_next_ = 0;
  std::vector<at::Tensor> comm_keep_;
  int loss_ = -1;
};

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "native training executor (forward instructions, C++ autograd backward, fused optimizer update)";
  m.def("kernel_calls", []() { return g_calls; });
  m.def("reset_kernel_calls", []() { g_calls.clear(); });
  py::class_<TrainProgram>(m, "TrainProgram")
      .def(py::init<int, std::string>())
      .def("grow", &TrainProgram::grow)
      .def("add_aten", &TrainProgram::add_aten)
      .def("add_native", &TrainProgram::add_native)
      .def("add_comm", &TrainProgram::add_comm)
      .def("add_py", &TrainProgram::add_py)
      .def("forward", &TrainProgram::forward, py::arg("feeds"), py::call_guard<py::gil_scoped_release>())
      .def("bind", &TrainProgram::bind)
      .def("set_loss", &TrainProgram::set_loss)
      .def("set_grad_hook", &TrainProgram::set_grad_hook)
      .def("add_optimizer", &TrainProgram::add_optimizer)
      .def("finalize", &TrainProgram::finalize)
      .def("run", &TrainProgram::run, py::arg("feeds"), py::arg("backward"), py::arg("scalars"), py::arg("clip_norm"),
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("num_instructions", &TrainProgram::num_instructions)
      .def_property_readonly("num_native", &TrainProgram::num_native)
      .def_property_readonly("num_comm", &TrainProgram::num_comm)
      .def_property_readonly("phase", &TrainProgram::phase)
      .def_property_readonly("done", &TrainProgram::done);
}
