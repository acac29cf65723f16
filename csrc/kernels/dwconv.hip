// Depthwise 2-D convolution, NHWC (groups == C_in == C_out), forward + data gradient + weight gradient.
// Reference behaviour: paddle/phi/kernels/gpu/depthwise_conv.h (depthwise_conv2d / _grad: stride, padding,
// dilation, per-channel KHxKW filter, optional bias).
//
// Memory-bound direct convolution: one lane owns 8 consecutive channels of one pixel (16-byte loads for 16-bit
// types), the filter is pre-transposed on the host to [KH*KW, C] so a tap's 8 weights are one vector load, and
// the tap loop reads the input rows through L1/L2 (neighbouring output pixels of a wave share them). fp32 math.
//   forward  y[n,oh,ow,c]  = b[c] + sum_{kh,kw} x[n, oh*s-p+kh*d, ow*s-p+kw*d, c] * w[kh,kw,c]
//   dgrad    dx[n,ih,iw,c] = sum_{kh,kw: (ih+p-kh*d) % s == 0, ...} dy[n, oh, ow, c] * w[kh,kw,c]
//   wgrad    dw[kh,kw,c]   = sum_{n,oh,ow} dy[n,oh,ow,c] * x[n, oh*s-p+kh*d, ow*s-p+kw*d, c]
//            -> per-lane fp32 partials [nparts, KT, C] over pixel stripes (up to 9 taps per pass), folded by
//               pa_reduce_parts (norm.hip) on the host side.
// Pre-activation ReLU (reference fuse_relu_depthwise_conv_pass / depthwise_conv2d fuse_relu_before_depthwise_conv,
// shape[14] = 1): the convolution reads relu(x) — forward and weight gradient clamp x on load, the data gradient
// is masked by x > 0 — so the ReLU output is never written or re-read.
#include "common.h"

using namespace pa;

namespace {

struct DwArgs {
  int N, H, W, C, Ho, Wo, KH, KW, sh, sw, ph, pw, dh, dw, relu;
};

template <typename T>
__global__ __launch_bounds__(256) void dw_fwd_k(const T* __restrict__ x, const T* __restrict__ wt,
                                                const T* __restrict__ bias, T* __restrict__ y, DwArgs a) {
  const int cg = a.C / 8;
  const int64_t total = (int64_t)a.N * a.Ho * a.Wo * cg;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c0 = (int)(i % cg) * 8;
    int64_t pix = i / cg;
    const int ow = (int)(pix % a.Wo);
    pix /= a.Wo;
    const int oh = (int)(pix % a.Ho);
    const int n = (int)(pix / a.Ho);
    float acc[8];
    if (bias != nullptr) load8<T>(bias + c0, acc);
    else
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int kh = 0; kh < a.KH; ++kh) {
      const int ih = oh * a.sh - a.ph + kh * a.dh;
      if (ih < 0 || ih >= a.H) continue;
      const T* xrow = x + (((int64_t)n * a.H + ih) * a.W) * a.C + c0;
      for (int kw = 0; kw < a.KW; ++kw) {
        const int iw = ow * a.sw - a.pw + kw * a.dw;
        if (iw < 0 || iw >= a.W) continue;
        float xv[8], wv[8];
        load8<T>(xrow + (int64_t)iw * a.C, xv);
        load8<T>(wt + (int64_t)(kh * a.KW + kw) * a.C + c0, wv);
        if (a.relu)
#pragma unroll
          for (int j = 0; j < 8; ++j) xv[j] = fmaxf(xv[j], 0.f);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(xv[j], wv[j], acc[j]);
      }
    }
    store8<T>(y + (((int64_t)n * a.Ho + oh) * a.Wo + ow) * a.C + c0, acc);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void dw_dgrad_k(const T* __restrict__ dy, const T* __restrict__ wt,
                                                  const T* __restrict__ x, T* __restrict__ dx, DwArgs a) {
  const int cg = a.C / 8;
  const int64_t total = (int64_t)a.N * a.H * a.W * cg;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c0 = (int)(i % cg) * 8;
    int64_t pix = i / cg;
    const int iw = (int)(pix % a.W);
    pix /= a.W;
    const int ih = (int)(pix % a.H);
    const int n = (int)(pix / a.H);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int kh = 0; kh < a.KH; ++kh) {
      const int th = ih + a.ph - kh * a.dh;
      if (th < 0 || th % a.sh) continue;
      const int oh = th / a.sh;
      if (oh >= a.Ho) continue;
      const T* drow = dy + (((int64_t)n * a.Ho + oh) * a.Wo) * a.C + c0;
      for (int kw = 0; kw < a.KW; ++kw) {
        const int tw = iw + a.pw - kw * a.dw;
        if (tw < 0 || tw % a.sw) continue;
        const int ow = tw / a.sw;
        if (ow >= a.Wo) continue;
        float gv[8], wv[8];
        load8<T>(drow + (int64_t)ow * a.C, gv);
        load8<T>(wt + (int64_t)(kh * a.KW + kw) * a.C + c0, wv);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(gv[j], wv[j], acc[j]);
      }
    }
    const int64_t o = (((int64_t)n * a.H + ih) * a.W + iw) * a.C + c0;
    if (a.relu) {  // d relu(x) / dx: the gradient passes where x > 0
      float xv[8];
      load8<T>(x + o, xv);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = xv[j] > 0.f ? acc[j] : 0.f;
    }
    store8<T>(dx + o, acc);
  }
}

// block = 256 lanes = CGB channel groups x TY pixel lanes; grid = (pixel stripes, channel blocks, tap passes).
// Lane (cgl, ty) of stripe s sums pixels s*TY*PPL + ty, + TY, ... for taps [tap0, tap0 + KT) and writes its fp32
// partial to part[(s * TY + ty), t, c].
constexpr int kMaxTaps = 9;

template <typename T>
__global__ __launch_bounds__(256) void dw_wgrad_k(const T* __restrict__ x, const T* __restrict__ dy,
                                                  float* __restrict__ part, DwArgs a, int CGB, int ppl) {
  const int TY = 256 / CGB;
  const int cgl = threadIdx.x % CGB, ty = threadIdx.x / CGB;
  const int cg = blockIdx.y * CGB + cgl;
  const int ntaps = a.KH * a.KW;
  const int tap0 = blockIdx.z * kMaxTaps;
  const int KT = min(kMaxTaps, ntaps - tap0);
  if (ty >= TY) return;
  const bool live = cg * 8 < a.C;
  const int c0 = live ? cg * 8 : 0;
  float acc[kMaxTaps][8];
#pragma unroll
  for (int t = 0; t < kMaxTaps; ++t)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[t][j] = 0.f;
  const int64_t P = (int64_t)a.N * a.Ho * a.Wo;
  const int64_t p_begin = (int64_t)blockIdx.x * TY * ppl;
  for (int k = 0; k < ppl && live; ++k) {
    const int64_t p = p_begin + (int64_t)k * TY + ty;
    if (p >= P) break;
    const int ow = (int)(p % a.Wo);
    const int oh = (int)((p / a.Wo) % a.Ho);
    const int n = (int)(p / ((int64_t)a.Wo * a.Ho));
    float gv[8];
    load8<T>(dy + p * a.C + c0, gv);
#pragma unroll
    for (int t = 0; t < kMaxTaps; ++t) {  // fully unrolled: acc stays in registers (static indices)
      const int tap = tap0 + t;
      const int kh = tap / a.KW, kw = tap % a.KW;
      const int ih = oh * a.sh - a.ph + kh * a.dh, iw = ow * a.sw - a.pw + kw * a.dw;
      if (t < KT && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W) {
        float xv[8];
        load8<T>(x + (((int64_t)n * a.H + ih) * a.W + iw) * a.C + c0, xv);
        if (a.relu)
#pragma unroll
          for (int j = 0; j < 8; ++j) xv[j] = fmaxf(xv[j], 0.f);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[t][j] = fmaf(gv[j], xv[j], acc[t][j]);
      }
    }
  }
  if (!live) return;
  const int64_t row = (int64_t)blockIdx.x * TY + ty;
  float* dst = part + row * (int64_t)ntaps * a.C;
#pragma unroll
  for (int t = 0; t < kMaxTaps; ++t) {
    if (t < KT) {
      float* q = dst + (int64_t)(tap0 + t) * a.C + c0;
      store8<float>(q, acc[t]);
    }
  }
}

unsigned grid_for(int64_t total) {
  int64_t g = cdiv(total, 256);
  if (g > 65536) g = 65536;
  return (unsigned)(g < 1 ? 1 : g);
}

DwArgs make_args(const int* s) {
  DwArgs a;
  a.N = s[0]; a.H = s[1]; a.W = s[2]; a.C = s[3]; a.Ho = s[4]; a.Wo = s[5]; a.KH = s[6]; a.KW = s[7];
  a.sh = s[8]; a.sw = s[9]; a.ph = s[10]; a.pw = s[11]; a.dh = s[12]; a.dw = s[13];
  a.relu = s[14];
  return a;
}

}  // namespace

// shape: int32[15] = N, H, W, C, Ho, Wo, KH, KW, sh, sw, ph, pw, dh, dw, pre-ReLU; wt: filter as [KH*KW, C]
PA_EXPORT int pa_dwconv_fwd(const void* x, const void* wt, const void* bias, void* y, const int* shape, int dtype,
                            hipStream_t st) {
  const DwArgs a = make_args(shape);
  if (a.C % 8) return 3;
  const unsigned g = grid_for((int64_t)a.N * a.Ho * a.Wo * (a.C / 8));
  PA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((dw_fwd_k<T>), dim3(g), dim3(256), 0, st, (const T*)x,
                                                 (const T*)wt, (const T*)bias, (T*)y, a));
  PA_CHECK_LAUNCH();
  return 0;
}

// x: the forward input (read only with the pre-ReLU flag, for the mask; may be null otherwise)
PA_EXPORT int pa_dwconv_dgrad(const void* dy, const void* wt, const void* x, void* dx, const int* shape, int dtype,
                              hipStream_t st) {
  const DwArgs a = make_args(shape);
  if (a.C % 8) return 3;
  if (a.relu && x == nullptr) return 4;
  const unsigned g = grid_for((int64_t)a.N * a.H * a.W * (a.C / 8));
  PA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((dw_dgrad_k<T>), dim3(g), dim3(256), 0, st, (const T*)dy,
                                                 (const T*)wt, (const T*)x, (T*)dx, a));
  PA_CHECK_LAUNCH();
  return 0;
}

// Layout of the partials the caller allocates: fp32 [nparts, KH*KW, C] with nparts from pa_dwconv_wgrad_parts.
PA_EXPORT int pa_dwconv_wgrad_parts(const int* shape, int* out /* nparts, stripes, CGB, ppl */) {
  const DwArgs a = make_args(shape);
  const int cg = a.C / 8;
  const int CGB = cg >= 64 ? 64 : (cg >= 32 ? 32 : (cg >= 16 ? 16 : (cg >= 8 ? 8 : (cg >= 4 ? 4 : (cg >= 2 ? 2 : 1)))));
  const int TY = 256 / CGB;
  const int64_t P = (int64_t)a.N * a.Ho * a.Wo;
  const int cblocks = (int)cdiv(cg, CGB);
  // ~4 workgroups per CU over the stripes x channel blocks, at least 16 pixels per lane
  int64_t stripes = cdiv(1024, cblocks);
  int ppl = (int)cdiv(P, stripes * TY);
  if (ppl < 16) ppl = 16;
  stripes = cdiv(P, (int64_t)TY * ppl);
  out[0] = (int)(stripes * TY);
  out[1] = (int)stripes;
  out[2] = CGB;
  out[3] = ppl;
  return 0;
}

PA_EXPORT int pa_dwconv_wgrad(const void* x, const void* dy, float* part, const int* shape, int dtype,
                              hipStream_t st) {
  const DwArgs a = make_args(shape);
  if (a.C % 8) return 3;
  int pp[4];
  pa_dwconv_wgrad_parts(shape, pp);
  const int cg = a.C / 8;
  dim3 grid((unsigned)pp[1], (unsigned)cdiv(cg, pp[2]), (unsigned)cdiv(a.KH * a.KW, kMaxTaps));
  PA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((dw_wgrad_k<T>), grid, dim3(256), 0, st, (const T*)x,
                                                 (const T*)dy, part, a, pp[2], pp[3]));
  PA_CHECK_LAUNCH();
  return 0;
}
