// Native program interpreter: executes a static / inference program as a flat instruction list in C++.
// Reference behaviour: paddle/fluid/framework/new_executor/program_interpreter.cc (Build: instruction list from
// the program, BuildOperatorDependences / last-use analysis for eager garbage collection; Run: execute the
// instructions in order, release every intermediate after its last reader).
//
// Here the program is the reference PIR format lowered by framework/native_interp.py: every value is a slot
// index, mutable attributes (full / full_int_array operands) are folded into per-instruction attributes at
// compile time, and each instruction is one call on the current HIP stream — no Python between operations.
// Device instructions run this framework's hand-written CDNA4 kernels (csrc/kernels, linked from _C_hip.so)
// where the operands fit them: matmul / fused linear (bias + GELU epilogue) on the MFMA GEMMs, layer_norm /
// rms_norm / softmax on the row kernels, flash_attn / flash_attn_qkvpacked on the flash-attention forward;
// everything else (and host tensors) is one ATen call. Slots whose last reader has run are released
// immediately (feeds, parameters and fetch targets excepted), so peak memory follows the live set.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>

#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

// hand-written kernels (csrc/kernels/*.hip, exported by _C_hip.so)
extern "C" {
int pa_gemm_bf16(const void* a, const void* b, void* c, const void* bias, void* aux, int64_t M, int64_t N, int64_t K,
                 int64_t lda, int64_t ldb, int64_t ldc, int a_kmajor, int b_kmajor, int flags, float alpha, int bn,
                 int splits, hipStream_t st);
int pa_gemm_bf16_pp(const void* a, const void* b, void* c, const void* bias, void* aux, int64_t M, int64_t N,
                    int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int a_kmajor, int b_kmajor, int flags,
                    float alpha, void* ws, hipStream_t st);
int64_t pa_gemm_pp_ws_bytes(int64_t M, int64_t N, int64_t K);
int pa_layer_norm_fwd(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd, int64_t rows,
                      int64_t cols, float eps, int dtype, hipStream_t st);
int pa_rms_norm_fwd(const void* x, const void* w, void* y, float* rstd, int64_t rows, int64_t cols, float eps,
                    int dtype, hipStream_t st);
int pa_softmax_fwd(const void* x, void* y, int64_t rows, int64_t cols, int dtype, hipStream_t st);
int pa_flash_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, const int64_t* strides, int B,
                      int Sq, int Sk, int H, int Hk, int D, float scale, int causal, hipStream_t st);
}

namespace {

// launches of the hand-written kernels by the interpreter (what the Predictor's GPU tests assert)
std::unordered_map<std::string, int64_t> g_kernel_calls;
constexpr int kEpiBias = 1, kEpiGelu = 2;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

int kdtype(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return 0;
    case at::kHalf: return 1;
    case at::kBFloat16: return 2;
    default: return -1;
  }
}

bool aligned16(const at::Tensor& t) { return (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0; }

// One guard for every hand-written kernel launched from the interpreter (the Python paths enforce the same:
// ops/activation.py softmax, ops/attention.py _lastdim_contig, ops/gemm.py supported): the kernels use 16-byte
// vector loads / stores, so each operand pointer must be 16-byte aligned and every leading stride (elements) a
// multiple of 8 (16 bytes of bf16). Optional operands (nullptr) are skipped. Failing it means "use ATen".
bool vec16_ok(std::initializer_list<const at::Tensor*> ts) {
  for (const at::Tensor* t : ts) {
    if (t == nullptr || !t->defined()) continue;
    if (!aligned16(*t)) return false;
    for (int64_t d = 0; d + 1 < t->dim(); ++d)
      if (t->size(d) > 1 && t->stride(d) % 8 != 0) return false;
  }
  return true;
}

void check_launch(int rc, const char* what) {
  if (rc != 0) throw std::runtime_error(std::string("interpreter: ") + what + " kernel launch failed (" +
                                        std::to_string(rc) + ")");
}

// y[M, N] = x[M, K] . W (+ bias, GELU) on the MFMA GEMM; W is [K, N] rows (paddle layout) or, with trans_w,
// [N, K] rows. Returns an undefined tensor when the operands do not fit the kernel (the caller uses ATen).
at::Tensor hip_linear(const at::Tensor& x_in, const at::Tensor& w, const at::Tensor* bias, bool trans_w, bool gelu) {
  if (!x_in.is_cuda() || x_in.scalar_type() != at::kBFloat16 || w.scalar_type() != at::kBFloat16 || w.dim() != 2 ||
      x_in.dim() < 2)
    return at::Tensor();
  if (bias != nullptr && (bias->scalar_type() != at::kBFloat16 || bias->dim() != 1 || !bias->is_contiguous()))
    return at::Tensor();
  const int64_t K = x_in.size(-1);
  const int64_t N = trans_w ? w.size(0) : w.size(1);
  if ((trans_w ? w.size(1) : w.size(0)) != K || K % 64 != 0 || N % 8 != 0) return at::Tensor();
  at::Tensor x = x_in.reshape({-1, K});
  if (!x.is_contiguous() || !w.is_contiguous() || !vec16_ok({&x, &w, bias})) return at::Tensor();
  const int64_t M = x.size(0);
  std::vector<int64_t> oshape(x_in.sizes().begin(), x_in.sizes().end());
  oshape.back() = N;
  at::Tensor y = at::empty({M, N}, x.options());
  const int flags = (bias != nullptr ? kEpiBias : 0) | (gelu ? kEpiGelu : 0);
  const void* bp = bias != nullptr ? bias->data_ptr() : nullptr;
  const int64_t ldb = trans_w ? K : N;
  const int64_t tiles = ((M + 255) / 256) * ((N + 255) / 256);
  int rc;
  if (M >= 1024 && N >= 1024 && tiles >= 256) {
    const int64_t nb = pa_gemm_pp_ws_bytes(M, N, K);
    at::Tensor ws = nb > 0 ? at::empty({nb / 4}, x.options().dtype(at::kFloat)) : at::Tensor();
    rc = pa_gemm_bf16_pp(x.data_ptr(), w.data_ptr(), y.data_ptr(), bp, nullptr, M, N, K, K, ldb, N, 1, trans_w ? 1 : 0,
                         flags, 1.f, nb > 0 ? ws.data_ptr() : nullptr, cur_stream());
  } else {
    rc = pa_gemm_bf16(x.data_ptr(), w.data_ptr(), y.data_ptr(), bp, nullptr, M, N, K, K, ldb, N, 1, trans_w ? 1 : 0,
                      flags, 1.f, trans_w ? 160 : 256, 1, cur_stream());
  }
  check_launch(rc, "gemm");
  ++g_kernel_calls["gemm"];
  return y.view(oshape);
}

// layer_norm / rms_norm over the trailing `cols` elements with same-dtype weight / bias
at::Tensor hip_norm(const at::Tensor& x, const at::Tensor* w, const at::Tensor* b, int64_t begin, double eps,
                    bool rms) {
  const int dt = kdtype(x);
  if (!x.is_cuda() || dt < 0 || !x.is_contiguous() || !vec16_ok({&x, w, b})) return at::Tensor();
  int64_t cols = 1;
  for (int64_t d = begin; d < x.dim(); ++d) cols *= x.size(d);
  if (cols % 8 != 0) return at::Tensor();
  for (const at::Tensor* p : {w, b})
    if (p != nullptr && (p->scalar_type() != x.scalar_type() || !p->is_contiguous() || p->numel() != cols))
      return at::Tensor();
  const int64_t rows = x.numel() / cols;
  at::Tensor y = at::empty_like(x);
  at::Tensor stats = at::empty({2, rows}, x.options().dtype(at::kFloat));
  float* mean = stats.data_ptr<float>();
  float* rstd = mean + rows;
  int rc;
  if (rms) {
    rc = pa_rms_norm_fwd(x.data_ptr(), w ? w->data_ptr() : nullptr, y.data_ptr(), rstd, rows, cols,
                         static_cast<float>(eps), dt, cur_stream());
  } else {
    rc = pa_layer_norm_fwd(x.data_ptr(), w ? w->data_ptr() : nullptr, b ? b->data_ptr() : nullptr, y.data_ptr(), mean,
                           rstd, rows, cols, static_cast<float>(eps), dt, cur_stream());
  }
  check_launch(rc, rms ? "rms_norm" : "layer_norm");
  ++g_kernel_calls[rms ? "rms_norm" : "layer_norm"];
  return y;
}

at::Tensor hip_softmax_lastdim(const at::Tensor& x) {
  const int dt = kdtype(x);
  if (!x.is_cuda() || dt < 0 || !x.is_contiguous() || x.dim() < 1) return at::Tensor();
  const int64_t cols = x.size(-1);
  // softmax.hip reads / writes rows in 8-element vectors and keeps a row in one workgroup: cols % 8 == 0,
  // 0 < cols <= 65536, 16-byte aligned rows (ops/activation.py applies the same conditions)
  if (cols <= 0 || cols % 8 != 0 || cols > 65536 || !vec16_ok({&x})) return at::Tensor();
  at::Tensor y = at::empty_like(x);
  if (!aligned16(y)) return at::Tensor();
  check_launch(pa_softmax_fwd(x.data_ptr(), y.data_ptr(), x.numel() / cols, cols, dt, cur_stream()), "softmax");
  ++g_kernel_calls["softmax"];
  return y;
}

// q / k / v [B, S, H(k), D] views with a unit last stride (any batch / sequence / head strides)
at::Tensor hip_flash_attn(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, bool causal, double scale) {
  if (!q.is_cuda() || q.scalar_type() != at::kBFloat16 || k.scalar_type() != at::kBFloat16 ||
      v.scalar_type() != at::kBFloat16 || q.dim() != 4 || k.dim() != 4 || v.dim() != 4)
    return at::Tensor();
  const int64_t B = q.size(0), Sq = q.size(1), H = q.size(2), D = q.size(3), Sk = k.size(1), Hk = k.size(2);
  if ((D != 64 && D != 128 && D != 256) || q.stride(3) != 1 || k.stride(3) != 1 || v.stride(3) != 1 || H % Hk != 0)
    return at::Tensor();
  if (!vec16_ok({&q, &k, &v})) return at::Tensor();
  at::Tensor o = at::empty({B, Sq, H, D}, q.options());
  at::Tensor lse = at::empty({B, H, Sq}, q.options().dtype(at::kFloat));
  const int64_t st[12] = {q.stride(0), q.stride(1), q.stride(2), k.stride(0), k.stride(1), k.stride(2),
                          v.stride(0), v.stride(1), v.stride(2), o.stride(0), o.stride(1), o.stride(2)};
  const double sc = scale > 0 ? scale : 1.0 / std::sqrt(static_cast<double>(D));
  check_launch(pa_flash_attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr<float>(), st,
                                 (int)B, (int)Sq, (int)Sk, (int)H, (int)Hk, (int)D, static_cast<float>(sc),
                                 causal ? 1 : 0, cur_stream()),
               "flash_attn");
  ++g_kernel_calls["flash_attn"];
  return o;
}

at::Tensor ref_attention(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, bool causal, double scale) {
  // [B, S, H, D] -> ATen SDPA over [B, H, S, D] (GQA by repeating K / V heads)
  at::Tensor qq = q.transpose(1, 2), kk = k.transpose(1, 2), vv = v.transpose(1, 2);
  if (kk.size(1) != qq.size(1)) {
    const int64_t rep = qq.size(1) / kk.size(1);
    kk = kk.repeat_interleave(rep, 1);
    vv = vv.repeat_interleave(rep, 1);
  }
  c10::optional<double> sc;
  if (scale > 0) sc = scale;
  return at::scaled_dot_product_attention(qq, kk, vv, {}, 0.0, causal, sc).transpose(1, 2);
}

enum Op : int {
  kMatmul, kAdd, kSub, kMul, kDiv, kMaximum, kMinimum, kPowT, kPowS, kRelu, kRelu6, kSigmoid, kTanh, kSilu, kExp,
  kSqrt, kRsqrt, kAbs, kLog, kSquare, kHardswish, kHardsigmoid, kLeakyRelu, kElu, kGelu, kSoftmax, kLogSoftmax,
  kLayerNorm, kBatchNorm, kScale, kReshape, kTranspose, kUnsqueeze, kSqueeze, kFlatten, kConcat, kStack, kSplit,
  kSplitNum, kSlice, kCast, kConv2d, kPool2d, kMean, kSum, kMax, kMin, kArgmax, kEmbedding, kGather, kExpand, kTile,
  kWhere, kClip, kIdentity, kFull, kFullLike, kShape, kFullIntArray, kRmsNorm, kLinear, kFlashAttn, kFlashAttnQKV,
  kArange, kLess, kLessEq, kGreater, kGreaterEq, kEqual, kNotEqual, kLogicalAnd, kLogicalOr, kLogicalNot,
  kIncrement,
  // control flow (structured pd_op.if / pd_op.while lowered to branches by framework/native_interp.py):
  kJump,         // pc = target
  kJumpIfFalse,  // pc = target unless in[0] (a scalar bool tensor) is true
  kMove          // out[k] = in[k] for every k, all inputs read before any output is written (yield / block args)
};

const std::unordered_map<std::string, int>& op_table() {
  static const std::unordered_map<std::string, int> t = {
      {"matmul", kMatmul}, {"add", kAdd}, {"subtract", kSub}, {"multiply", kMul}, {"divide", kDiv},
      {"maximum", kMaximum}, {"minimum", kMinimum}, {"elementwise_pow", kPowT}, {"pow", kPowS}, {"relu", kRelu},
      {"relu6", kRelu6}, {"sigmoid", kSigmoid}, {"tanh", kTanh}, {"silu", kSilu}, {"swish", kSilu}, {"exp", kExp},
      {"sqrt", kSqrt}, {"rsqrt", kRsqrt}, {"abs", kAbs}, {"log", kLog}, {"square", kSquare},
      {"hardswish", kHardswish}, {"hardsigmoid", kHardsigmoid}, {"leaky_relu", kLeakyRelu}, {"elu", kElu},
      {"gelu", kGelu}, {"softmax", kSoftmax}, {"log_softmax", kLogSoftmax}, {"layer_norm", kLayerNorm},
      {"batch_norm", kBatchNorm}, {"batch_norm_", kBatchNorm}, {"scale", kScale}, {"reshape", kReshape},
      {"transpose", kTranspose}, {"unsqueeze", kUnsqueeze}, {"squeeze", kSqueeze}, {"flatten", kFlatten},
      {"concat", kConcat}, {"stack", kStack}, {"split", kSplit}, {"split_with_num", kSplitNum}, {"slice", kSlice},
      {"cast", kCast}, {"conv2d", kConv2d}, {"depthwise_conv2d", kConv2d}, {"pool2d", kPool2d}, {"mean", kMean},
      {"sum", kSum}, {"max", kMax}, {"min", kMin}, {"argmax", kArgmax}, {"embedding", kEmbedding},
      {"gather", kGather}, {"expand", kExpand}, {"tile", kTile}, {"where", kWhere}, {"clip", kClip},
      {"assign", kIdentity}, {"dropout", kIdentity}, {"full", kFull}, {"full_like", kFullLike}, {"shape", kShape},
      {"full_int_array", kFullIntArray}, {"rms_norm", kRmsNorm}, {"fused_linear", kLinear},
      {"flash_attn", kFlashAttn}, {"flash_attn_qkvpacked", kFlashAttnQKV}, {"arange", kArange},
      {"less_than", kLess}, {"less_equal", kLessEq}, {"greater_than", kGreater}, {"greater_equal", kGreaterEq},
      {"equal", kEqual}, {"not_equal", kNotEqual}, {"logical_and", kLogicalAnd}, {"logical_or", kLogicalOr},
      {"logical_not", kLogicalNot}, {"increment", kIncrement}, {"increment_", kIncrement},
      {"__jump", kJump}, {"__jump_if_false", kJumpIfFalse}, {"__move", kMove}};
  return t;
}

struct Attr {
  std::vector<int64_t> ints;
  double f = 0.0;
  std::string s;
  int kind = 0;  // 1 int list / int, 2 float, 3 string
};

struct Instr {
  int op;
  std::string name;
  std::vector<int> in, out;
  std::unordered_map<std::string, Attr> a;

  bool has(const char* k) const { return a.count(k) != 0; }
  int64_t i(const char* k, int64_t d) const {
    auto it = a.find(k);
    if (it == a.end()) return d;
    if (it->second.kind == 2) return static_cast<int64_t>(it->second.f);
    return it->second.ints.empty() ? d : it->second.ints[0];
  }
  double f(const char* k, double d) const {
    auto it = a.find(k);
    if (it == a.end()) return d;
    if (it->second.kind == 1) return it->second.ints.empty() ? d : static_cast<double>(it->second.ints[0]);
    return it->second.f;
  }
  std::vector<int64_t> v(const char* k) const {
    auto it = a.find(k);
    return it == a.end() ? std::vector<int64_t>{} : it->second.ints;
  }
  std::string s(const char* k, const std::string& d) const {
    auto it = a.find(k);
    return it == a.end() ? d : it->second.s;
  }
};

at::ScalarType dtype_of(const std::string& s) {
  if (s == "float32" || s == "float") return at::kFloat;
  if (s == "float16") return at::kHalf;
  if (s == "bfloat16") return at::kBFloat16;
  if (s == "float64") return at::kDouble;
  if (s == "int64") return at::kLong;
  if (s == "int32") return at::kInt;
  if (s == "int16") return at::kShort;
  if (s == "int8") return at::kChar;
  if (s == "uint8") return at::kByte;
  if (s == "bool") return at::kBool;
  throw std::runtime_error("interpreter: unknown dtype " + s);
}

int64_t norm_axis(int64_t ax, int64_t nd) { return ax < 0 ? ax + nd : ax; }

std::vector<int64_t> paddle_shape(const at::Tensor& x, std::vector<int64_t> shape) {
  for (size_t k = 0; k < shape.size(); ++k)
    if (shape[k] == 0 && static_cast<int64_t>(k) < x.dim()) shape[k] = x.size(k);  // 0 copies the input dim
  return shape;
}

at::Tensor nchw(const at::Tensor& x, bool nhwc) { return nhwc ? x.permute({0, 3, 1, 2}) : x; }
at::Tensor back(const at::Tensor& y, bool nhwc) { return nhwc ? y.permute({0, 2, 3, 1}).contiguous() : y; }

std::vector<int64_t> axes_or_all(const Instr& ins, const at::Tensor& x) {
  std::vector<int64_t> ax = ins.v("axis");
  if (ax.empty()) {
    for (int64_t d = 0; d < x.dim(); ++d) ax.push_back(d);
  }
  for (auto& a : ax) a = norm_axis(a, x.dim());
  return ax;
}

class Interpreter {
 public:
  explicit Interpreter(int n_slots, std::string device) : slots_(n_slots), device_(std::move(device)) {}

  void add(const std::string& op, std::vector<int> in, std::vector<int> out, py::dict attrs) {
    auto it = op_table().find(op);
    if (it == op_table().end()) throw std::runtime_error("interpreter: unsupported op " + op);
    Instr ins;
    ins.op = it->second;
    ins.name = op;
    ins.in = std::move(in);
    ins.out = std::move(out);
    for (auto kv : attrs) {
      Attr a;
      py::handle v = kv.second;
      if (py::isinstance<py::bool_>(v)) {
        a.kind = 1;
        a.ints = {v.cast<bool>() ? 1 : 0};
      } else if (py::isinstance<py::int_>(v)) {
        a.kind = 1;
        a.ints = {v.cast<int64_t>()};
      } else if (py::isinstance<py::float_>(v)) {
        a.kind = 2;
        a.f = v.cast<double>();
      } else if (py::isinstance<py::str>(v)) {
        a.kind = 3;
        a.s = v.cast<std::string>();
      } else if (py::isinstance<py::list>(v) || py::isinstance<py::tuple>(v)) {
        a.kind = 1;
        for (auto e : v) a.ints.push_back(py::cast<int64_t>(e));
      } else {
        continue;  // attributes the kernels never read
      }
      ins.a[kv.first.cast<std::string>()] = std::move(a);
    }
    code_.push_back(std::move(ins));
  }

  // slots that live across runs (parameters) and the fetch targets; computes each slot's last reader
  void finalize(std::vector<int> keep, std::vector<int> fetch) {
    keep_.assign(slots_.size(), 0);
    for (int k : keep) keep_.at(k) = 1;
    for (int k : fetch) keep_.at(k) = 1;
    fetch_ = std::move(fetch);
    std::vector<int> last(slots_.size(), -1);
    for (size_t n = 0; n < code_.size(); ++n)
      for (int s : code_[n].in)
        if (s >= 0) last[s] = static_cast<int>(n);
    // loops (a backward jump at b to t <= b, the loop exit at b + 1): a slot read inside [t, b] but written outside
    // it (defined before the loop, a feed or a parameter) is read again by the next iteration, so it is released
    // only once the loop has exited
    for (size_t b = 0; b < code_.size(); ++b) {
      if (code_[b].op != kJump) continue;
      const int t = static_cast<int>(code_[b].i("target", 0));
      if (t > static_cast<int>(b)) continue;
      std::vector<char> inside_w(slots_.size(), 0);
      for (size_t n = t; n <= b; ++n)
        for (int s : code_[n].out)
          if (s >= 0) inside_w[s] = 1;
      for (size_t n = t; n <= b; ++n)
        for (int s : code_[n].in)
          if (s >= 0 && !inside_w[s]) last[s] = std::max(last[s], static_cast<int>(b) + 1);
    }
    release_.assign(code_.size(), {});
    for (size_t s = 0; s < last.size(); ++s)
      if (last[s] >= 0 && last[s] < static_cast<int>(code_.size()) && !keep_[s])
        release_[last[s]].push_back(static_cast<int>(s));
    // outputs never read (e.g. a dropout mask) are dropped right after their producer
    for (size_t n = 0; n < code_.size(); ++n)
      for (int s : code_[n].out)
        if (s >= 0 && last[s] < 0 && !keep_[s]) release_[n].push_back(s);
  }

  void bind(int slot, at::Tensor t) {
    slots_.at(slot) = std::move(t);
    persistent_.push_back(slot);
  }

  std::vector<at::Tensor> run(const std::vector<std::pair<int, at::Tensor>>& feeds) {
    at::NoGradGuard ng;
    for (const auto& f : feeds) slots_.at(f.first) = f.second;
    peak_live_ = 0;
    int64_t live = 0;
    for (const auto& s : slots_) live += s.defined() ? 1 : 0;
    const size_t ncode = code_.size();
    int64_t steps = 0;
    for (size_t n = 0; n < ncode;) {
      const Instr& I = code_[n];
      size_t next = n + 1;
      if (I.op == kJump) {
        next = static_cast<size_t>(I.i("target", 0));
      } else if (I.op == kJumpIfFalse) {
        const at::Tensor& c = in(I, 0);
        if (!c.defined() || c.numel() != 1)
          throw std::runtime_error("interpreter: control-flow condition is not a one-element tensor");
        if (!c.item().toBool()) next = static_cast<size_t>(I.i("target", 0));
      } else {
        exec(I);
      }
      for (int s : I.out) live += (s >= 0 && slots_[s].defined()) ? 1 : 0;
      peak_live_ = std::max(peak_live_, live);
      for (int s : release_[n]) {
        if (slots_[s].defined()) --live;
        slots_[s] = at::Tensor();
      }
      if (++steps > max_steps_) throw std::runtime_error("interpreter: instruction budget exceeded (endless loop?)");
      n = next;
    }
    std::vector<at::Tensor> out;
    out.reserve(fetch_.size());
    for (int s : fetch_) out.push_back(slots_[s]);
    // branches not taken / loops leave slots whose last reader did not run: drop every non-persistent slot
    for (size_t s = 0; s < slots_.size(); ++s)
      if (!keep_[s]) slots_[s] = at::Tensor();
    return out;
  }

  int64_t num_instructions() const { return static_cast<int64_t>(code_.size()); }
  int64_t peak_live() const { return peak_live_; }
  int64_t releases() const {
    int64_t n = 0;
    for (const auto& r : release_) n += static_cast<int64_t>(r.size());
    return n;
  }

 private:
  const at::Tensor& in(const Instr& ins, size_t k) const { return slots_.at(ins.in.at(k)); }
  void put(const Instr& ins, size_t k, at::Tensor t) {
    if (k < ins.out.size() && ins.out[k] >= 0) slots_[ins.out[k]] = std::move(t);
  }

  void exec(const Instr& I) {
    switch (I.op) {
      case kMatmul: {
        at::Tensor x = in(I, 0), y = in(I, 1);
        if (!I.i("transpose_x", 0) && y.dim() == 2) {
          at::Tensor r = hip_linear(x, y, nullptr, I.i("transpose_y", 0) != 0, false);
          if (r.defined()) {
            put(I, 0, r);
            break;
          }
        }
        if (I.i("transpose_x", 0) && x.dim() >= 2) x = x.transpose(-1, -2);
        if (I.i("transpose_y", 0) && y.dim() >= 2) y = y.transpose(-1, -2);
        put(I, 0, at::matmul(x, y));
        break;
      }
      case kAdd: put(I, 0, in(I, 0) + in(I, 1)); break;
      case kSub: put(I, 0, in(I, 0) - in(I, 1)); break;
      case kMul: put(I, 0, in(I, 0) * in(I, 1)); break;
      case kDiv: put(I, 0, in(I, 0) / in(I, 1)); break;
      case kMaximum: put(I, 0, at::maximum(in(I, 0), in(I, 1))); break;
      case kMinimum: put(I, 0, at::minimum(in(I, 0), in(I, 1))); break;
      case kPowT: put(I, 0, at::pow(in(I, 0), in(I, 1))); break;
      case kPowS: put(I, 0, at::pow(in(I, 0), I.f("y", 1.0))); break;
      case kRelu: put(I, 0, at::relu(in(I, 0))); break;
      case kRelu6: put(I, 0, at::hardtanh(in(I, 0), 0.0, 6.0)); break;
      case kSigmoid: put(I, 0, at::sigmoid(in(I, 0))); break;
      case kTanh: put(I, 0, at::tanh(in(I, 0))); break;
      case kSilu: put(I, 0, at::silu(in(I, 0))); break;
      case kExp: put(I, 0, at::exp(in(I, 0))); break;
      case kSqrt: put(I, 0, at::sqrt(in(I, 0))); break;
      case kRsqrt: put(I, 0, at::rsqrt(in(I, 0))); break;
      case kAbs: put(I, 0, at::abs(in(I, 0))); break;
      case kLog: put(I, 0, at::log(in(I, 0))); break;
      case kSquare: put(I, 0, in(I, 0) * in(I, 0)); break;
      case kHardswish: put(I, 0, at::hardswish(in(I, 0))); break;
      case kHardsigmoid:
        put(I, 0, at::clamp(in(I, 0) * I.f("slope", 0.1666667) + I.f("offset", 0.5), 0.0, 1.0));
        break;
      case kLeakyRelu: put(I, 0, at::leaky_relu(in(I, 0), I.f("negative_slope", 0.02))); break;
      case kElu: put(I, 0, at::elu(in(I, 0), I.f("alpha", 1.0))); break;
      case kGelu: put(I, 0, at::gelu(in(I, 0), I.i("approximate", 0) ? "tanh" : "none")); break;
      case kSoftmax: {
        const at::Tensor& x = in(I, 0);
        if (norm_axis(I.i("axis", -1), x.dim()) == x.dim() - 1) {
          at::Tensor r = hip_softmax_lastdim(x);
          if (r.defined()) {
            put(I, 0, r);
            break;
          }
        }
        put(I, 0, at::softmax(x, I.i("axis", -1)));
        break;
      }
      case kLogSoftmax: put(I, 0, at::log_softmax(in(I, 0), I.i("axis", -1))); break;
      case kLayerNorm: {
        const at::Tensor& x = in(I, 0);
        const int64_t ax = norm_axis(I.i("begin_norm_axis", 1), x.dim());
        std::vector<int64_t> shp(x.sizes().begin() + ax, x.sizes().end());
        c10::optional<at::Tensor> w, b;
        if (I.in.size() > 1 && I.in[1] >= 0) w = in(I, 1);
        if (I.in.size() > 2 && I.in[2] >= 0) b = in(I, 2);
        at::Tensor r = hip_norm(x, w ? &*w : nullptr, b ? &*b : nullptr, ax, I.f("epsilon", 1e-5), false);
        put(I, 0, r.defined() ? r : at::layer_norm(x, shp, w, b, I.f("epsilon", 1e-5)));
        break;
      }
      case kRmsNorm: {  // reference rms_norm operands: x, bias, residual, norm_weight, norm_bias
        const at::Tensor& x = in(I, 0);
        if ((I.in.size() > 1 && I.in[1] >= 0) || (I.in.size() > 2 && I.in[2] >= 0) || (I.in.size() > 4 && I.in[4] >= 0))
          throw std::runtime_error("interpreter: rms_norm with bias / residual / norm_bias operands is not lowered");
        const int64_t ax = norm_axis(I.i("begin_norm_axis", x.dim() - 1), x.dim());
        c10::optional<at::Tensor> w;
        if (I.in.size() > 3 && I.in[3] >= 0) w = in(I, 3);
        at::Tensor r = hip_norm(x, w ? &*w : nullptr, nullptr, ax, I.f("epsilon", 1e-6), true);
        if (!r.defined()) {
          std::vector<int64_t> dims;
          for (int64_t d = ax; d < x.dim(); ++d) dims.push_back(d);
          at::Tensor xf = x.to(at::kFloat);
          r = (xf * at::rsqrt(xf.pow(2).mean(dims, true) + I.f("epsilon", 1e-6))).to(x.scalar_type());
          if (w) r = r * *w;
        }
        put(I, 0, r);
        break;
      }
      case kLinear: {  // fused_linear: x . W (+ bias) (GELU): the GEMM with its epilogue
        const at::Tensor& x = in(I, 0);
        const at::Tensor& w = in(I, 1);
        const bool has_b = I.in.size() > 2 && I.in[2] >= 0;
        const bool gelu = I.s("activation", "none") == "gelu";
        const bool tw = I.i("transpose_y", 0) != 0;
        at::Tensor r = hip_linear(x, w, has_b ? &in(I, 2) : nullptr, tw, gelu);
        if (!r.defined()) {
          r = at::matmul(x, tw ? w.t() : w);
          if (has_b) r = r + in(I, 2);
          if (gelu) r = at::gelu(r, I.i("approximate", 0) ? "tanh" : "none");
        }
        put(I, 0, r);
        break;
      }
      case kFlashAttn:
      case kFlashAttnQKV: {
        at::Tensor q, k, v;
        if (I.op == kFlashAttn) {
          q = in(I, 0);
          k = in(I, 1);
          v = in(I, 2);
        } else {  // reference qkvpacked layout [B, S, G + 2, Hk, D]: G query groups, then K and V
          const at::Tensor& qkv = in(I, 0);
          const int64_t g = qkv.size(2) - 2;
          q = qkv.narrow(2, 0, g).flatten(2, 3);
          k = qkv.select(2, g);
          v = qkv.select(2, g + 1);
          if (g > 1) q = qkv.narrow(2, 0, g).transpose(2, 3).flatten(2, 3);
        }
        const int mask_in = I.op == kFlashAttn ? 4 : 2;
        if (I.in.size() > static_cast<size_t>(mask_in) && I.in[mask_in] >= 0)
          throw std::runtime_error("interpreter: flash_attn with an attn_mask operand is not lowered");
        const bool causal = I.i("causal", 0) != 0;
        const double scale = I.f("scale", -1.0);
        at::Tensor o = hip_flash_attn(q, k, v, causal, scale);
        put(I, 0, o.defined() ? o : ref_attention(q, k, v, causal, scale));
        break;
      }
      case kArange: {
        auto opts = at::TensorOptions().dtype(dtype_of(I.s("dtype", "int64"))).device(device_);
        put(I, 0, at::arange(I.f("start", 0.0), I.f("end", 0.0), I.f("step", 1.0), opts));
        break;
      }
      case kBatchNorm: {  // inputs: x, mean, variance, scale, bias (inference statistics)
        const bool nhwc = I.s("data_format", "NCHW") == "NHWC";
        at::Tensor x = nchw(in(I, 0), nhwc);
        c10::optional<at::Tensor> w, b;
        if (I.in.size() > 3 && I.in[3] >= 0) w = in(I, 3);
        if (I.in.size() > 4 && I.in[4] >= 0) b = in(I, 4);
        at::Tensor y = at::batch_norm(x, w, b, in(I, 1), in(I, 2), false, 0.0, I.f("epsilon", 1e-5), true);
        put(I, 0, back(y, nhwc));
        break;
      }
      case kScale: {
        const double s = I.f("scale", 1.0), b = I.f("bias", 0.0);
        put(I, 0, I.i("bias_after_scale", 1) ? in(I, 0) * s + b : (in(I, 0) + b) * s);
        break;
      }
      case kReshape: put(I, 0, in(I, 0).reshape(paddle_shape(in(I, 0), I.v("shape")))); break;
      case kTranspose: put(I, 0, in(I, 0).permute(I.v("perm"))); break;
      case kUnsqueeze: {
        at::Tensor x = in(I, 0);
        std::vector<int64_t> ax = I.v("axis");
        for (int64_t a : ax) x = x.unsqueeze(a < 0 ? a + x.dim() + 1 : a);
        put(I, 0, x);
        break;
      }
      case kSqueeze: {
        at::Tensor x = in(I, 0);
        std::vector<int64_t> ax = I.v("axis");
        if (ax.empty()) {
          x = x.squeeze();
        } else {
          for (auto& a : ax) a = norm_axis(a, x.dim());
          std::sort(ax.rbegin(), ax.rend());
          for (int64_t a : ax)
            if (x.size(a) == 1) x = x.squeeze(a);
        }
        put(I, 0, x);
        break;
      }
      case kFlatten: {
        const at::Tensor& x = in(I, 0);
        put(I, 0, at::flatten(x, norm_axis(I.i("start_axis", 1), x.dim()), norm_axis(I.i("stop_axis", -1), x.dim())));
        break;
      }
      case kConcat:
      case kStack: {
        std::vector<at::Tensor> xs;
        for (size_t k = 0; k < I.in.size(); ++k) xs.push_back(in(I, k));
        put(I, 0, I.op == kConcat ? at::cat(xs, I.i("axis", 0)) : at::stack(xs, I.i("axis", 0)));
        break;
      }
      case kSplit:
      case kSplitNum: {
        const at::Tensor& x = in(I, 0);
        const int64_t ax = norm_axis(I.i("axis", 0), x.dim());
        std::vector<at::Tensor> parts;
        if (I.op == kSplitNum) {
          parts = at::chunk(x, I.i("num", 1), ax);
        } else {
          std::vector<int64_t> sec = I.v("sections");
          int64_t known = 0, neg = -1;
          for (size_t k = 0; k < sec.size(); ++k) {
            if (sec[k] < 0) neg = static_cast<int64_t>(k);
            else known += sec[k];
          }
          if (neg >= 0) sec[neg] = x.size(ax) - known;
          parts = at::split_with_sizes(x, sec, ax);
        }
        for (size_t k = 0; k < parts.size(); ++k) put(I, k, parts[k]);
        break;
      }
      case kSlice: {
        at::Tensor x = in(I, 0);
        std::vector<int64_t> axes = I.v("axes"), st = I.v("starts"), en = I.v("ends"), dec = I.v("decrease_axis");
        for (size_t k = 0; k < axes.size(); ++k) {
          const int64_t ax = norm_axis(axes[k], x.dim()), n = x.size(ax);
          int64_t s = st[k] < 0 ? st[k] + n : st[k], e = en[k] < 0 ? en[k] + n : en[k];
          s = std::max<int64_t>(0, std::min(s, n));
          e = std::max<int64_t>(s, std::min(e, n));
          x = x.slice(ax, s, e);
        }
        if (!dec.empty()) {
          for (auto& a : dec) a = norm_axis(a, x.dim());
          std::sort(dec.rbegin(), dec.rend());
          for (int64_t a : dec) x = x.squeeze(a);
        }
        put(I, 0, x);
        break;
      }
      case kCast: put(I, 0, in(I, 0).to(dtype_of(I.s("dtype", "float32")))); break;
      case kConv2d: {
        const bool nhwc = I.s("data_format", "NCHW") == "NHWC";
        at::Tensor x = nchw(in(I, 0), nhwc);
        std::vector<int64_t> st = I.v("strides"), pd = I.v("paddings"), dl = I.v("dilations");
        if (st.empty()) st = {1, 1};
        if (dl.empty()) dl = {1, 1};
        if (pd.empty()) pd = {0, 0};
        if (pd.size() == 4) {
          if (pd[0] == pd[1] && pd[2] == pd[3]) {
            pd = {pd[0], pd[2]};
          } else {  // asymmetric: explicit pad (left, right, top, bottom), then no padding in the conv
            x = at::constant_pad_nd(x, {pd[2], pd[3], pd[0], pd[1]}, 0);
            pd = {0, 0};
          }
        }
        c10::optional<at::Tensor> b;
        if (I.in.size() > 2 && I.in[2] >= 0) b = in(I, 2);
        put(I, 0, back(at::conv2d(x, in(I, 1), b, st, pd, dl, I.i("groups", 1)), nhwc));
        break;
      }
      case kPool2d: {
        const bool nhwc = I.s("data_format", "NCHW") == "NHWC";
        at::Tensor x = nchw(in(I, 0), nhwc);
        const bool mx = I.s("pooling_type", "max") == "max";
        std::vector<int64_t> ks = I.v("kernel_size");
        if (I.i("global_pooling", 0) || (I.i("adaptive", 0) && ks == std::vector<int64_t>{1, 1})) {
          put(I, 0, back(mx ? std::get<0>(at::adaptive_max_pool2d(x, {1, 1})) : at::adaptive_avg_pool2d(x, {1, 1}),
                         nhwc));
          break;
        }
        if (I.i("adaptive", 0)) {
          put(I, 0, back(mx ? std::get<0>(at::adaptive_max_pool2d(x, ks)) : at::adaptive_avg_pool2d(x, ks), nhwc));
          break;
        }
        std::vector<int64_t> st = I.v("strides"), pd = I.v("paddings");
        if (pd.size() == 4) pd = {pd[0], pd[2]};
        if (pd.empty()) pd = {0, 0};
        const bool ceil = I.i("ceil_mode", 0) != 0;
        at::Tensor y = mx ? at::max_pool2d(x, ks, st, pd, {1, 1}, ceil)
                          : at::avg_pool2d(x, ks, st, pd, ceil, !I.i("exclusive", 1));
        put(I, 0, back(y, nhwc));
        break;
      }
      case kMean: put(I, 0, at::mean(in(I, 0), axes_or_all(I, in(I, 0)), I.i("keepdim", 0) != 0)); break;
      case kSum: put(I, 0, at::sum(in(I, 0), axes_or_all(I, in(I, 0)), I.i("keepdim", 0) != 0)); break;
      case kMax: put(I, 0, at::amax(in(I, 0), axes_or_all(I, in(I, 0)), I.i("keepdim", 0) != 0)); break;
      case kMin: put(I, 0, at::amin(in(I, 0), axes_or_all(I, in(I, 0)), I.i("keepdim", 0) != 0)); break;
      case kArgmax: {
        const at::Tensor& x = in(I, 0);
        at::Tensor r = I.i("flatten", 0) ? at::argmax(x.reshape({-1}), 0, false)
                                        : at::argmax(x, I.i("axis", -1), I.i("keepdims", 0) != 0);
        put(I, 0, r);
        break;
      }
      case kEmbedding: put(I, 0, at::embedding(in(I, 1), in(I, 0))); break;
      case kGather: put(I, 0, at::index_select(in(I, 0), I.i("axis", 0), in(I, 1).reshape({-1}))); break;
      case kExpand: put(I, 0, in(I, 0).expand(I.v("shape"))); break;
      case kTile: put(I, 0, in(I, 0).repeat(I.v("repeat_times"))); break;
      case kWhere: put(I, 0, at::where(in(I, 0), in(I, 1), in(I, 2))); break;
      case kClip: put(I, 0, at::clamp(in(I, 0), I.f("min", -3.4e38), I.f("max", 3.4e38))); break;
      case kIdentity: put(I, 0, in(I, 0)); break;
      case kLess: put(I, 0, at::lt(in(I, 0), in(I, 1))); break;
      case kLessEq: put(I, 0, at::le(in(I, 0), in(I, 1))); break;
      case kGreater: put(I, 0, at::gt(in(I, 0), in(I, 1))); break;
      case kGreaterEq: put(I, 0, at::ge(in(I, 0), in(I, 1))); break;
      case kEqual: put(I, 0, at::eq(in(I, 0), in(I, 1))); break;
      case kNotEqual: put(I, 0, at::ne(in(I, 0), in(I, 1))); break;
      case kLogicalAnd: put(I, 0, at::logical_and(in(I, 0), in(I, 1))); break;
      case kLogicalOr: put(I, 0, at::logical_or(in(I, 0), in(I, 1))); break;
      case kLogicalNot: put(I, 0, at::logical_not(in(I, 0))); break;
      case kIncrement: put(I, 0, at::add(in(I, 0), I.f("value", 1.0))); break;  // out of place (no aliasing)
      case kMove: {
        std::vector<at::Tensor> vals;
        vals.reserve(I.in.size());
        for (size_t k = 0; k < I.in.size(); ++k) vals.push_back(in(I, k));
        for (size_t k = 0; k < vals.size(); ++k) put(I, k, std::move(vals[k]));
        break;
      }
      case kFull: {
        auto opts = at::TensorOptions().dtype(dtype_of(I.s("dtype", "float32"))).device(device_);
        put(I, 0, at::full(I.v("shape"), I.f("value", 0.0), opts));
        break;
      }
      case kFullIntArray: {
        std::vector<int64_t> v = I.v("value");
        auto opts = at::TensorOptions().dtype(dtype_of(I.s("dtype", "int64"))).device(device_);
        put(I, 0, at::tensor(v, at::TensorOptions().dtype(at::kLong)).to(opts));
        break;
      }
      case kFullLike: {
        const at::Tensor& x = in(I, 0);
        const std::string dt = I.s("dtype", "");
        auto opts = x.options();
        if (!dt.empty() && dt != "undefined") opts = opts.dtype(dtype_of(dt));
        put(I, 0, at::full(x.sizes(), I.f("value", 0.0), opts));
        break;
      }
      case kShape: {
        std::vector<int64_t> s(in(I, 0).sizes().begin(), in(I, 0).sizes().end());
        put(I, 0, at::tensor(s, at::TensorOptions().dtype(at::kLong)).to(at::kInt).to(in(I, 0).device()));
        break;
      }
      default:
        throw std::runtime_error("interpreter: op not implemented: " + I.name);
    }
  }

  std::vector<at::Tensor> slots_;
  std::string device_;
  std::vector<Instr> code_;
  std::vector<int> keep_, fetch_, persistent_;
  std::vector<std::vector<int>> release_;
  int64_t max_steps_ = int64_t(1) << 40;
  int64_t peak_live_ = 0;
};

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "native program interpreter (instruction list + last-use GC; hand-written HIP kernels, ATen otherwise)";
  m.def("kernel_calls", []() { return g_kernel_calls; }, "launches of the hand-written kernels per kind");
  m.def("reset_kernel_calls", []() { g_kernel_calls.clear(); });
  m.def("supported_ops", []() {
    std::vector<std::string> v;
    for (const auto& kv : op_table()) v.push_back(kv.first);
    return v;
  });
  py::class_<Interpreter>(m, "Interpreter")
      .def(py::init<int, std::string>())
      .def("add", &Interpreter::add)
      .def("finalize", &Interpreter::finalize)
      .def("bind", &Interpreter::bind)
      .def("run", &Interpreter::run)
      .def_property_readonly("num_instructions", &Interpreter::num_instructions)
      .def_property_readonly("peak_live", &Interpreter::peak_live)
      .def_property_readonly("releases", &Interpreter::releases);
}
