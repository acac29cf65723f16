// Standalone check of the 16x16x32 MFMA operand maps and ds_read_b64_tr_b16 on gfx950 as used by fa_bwd16_kernel:
// one wave computes S = Q K^T (16x16, K = 32) from row reads and dV-style X^T P (A from transposed reads of a
// [32 rows][16 cols] row image) and writes them out; the host compares with a plain loop.
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <cstdio>
#include <cstring>
#include <cmath>
#include <vector>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef float f32x4 __attribute__((ext_vector_type(4)));
union Frag { bf16x8 v; uint4 u; s16x4 h[2]; };

__device__ s16x4 tr(const char* smem, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(reinterpret_cast<uintptr_t>(smem + off)));
}

// A: [16][32] row-major bf16 (rows m, cols k); B: [16][32] (rows n, cols k) -> S[m][n] = sum_k A[m][k] B[n][k]
// X: [32][16] (rows k, cols m) -> T[m][n] = sum_k X[k][m] P[k][n] with P[k][n] = B[n][k]
__global__ void k(const uint16_t* A, const uint16_t* B, const uint16_t* X, float* S, float* T) {
  __shared__ __attribute__((aligned(16))) char a_img[16 * 64], b_img[16 * 64], x_img[32 * 32];
  const int l = threadIdx.x, r16 = l & 15, kg = l >> 4, tq = r16 >> 2, tp = r16 & 3;
  for (int i = l; i < 16 * 32; i += 64) {
    reinterpret_cast<uint16_t*>(a_img)[i] = A[i];
    reinterpret_cast<uint16_t*>(b_img)[i] = B[i];
    reinterpret_cast<uint16_t*>(x_img)[i] = X[i];
  }
  __syncthreads();
  Frag a, b;
  a.u = *reinterpret_cast<const uint4*>(a_img + r16 * 64 + kg * 16);  // A[m = r16][k = 8kg + j]
  b.u = *reinterpret_cast<const uint4*>(b_img + r16 * 64 + kg * 16);  // B^T[k = 8kg + j][n = r16]
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, acc, 0, 0, 0);
  for (int i = 0; i < 4; ++i) S[(4 * kg + i) * 16 + r16] = acc[i];
  // T = X^T P with the permuted k: element j of group kg <-> k = 4kg + j (j < 4), 16 + 4kg + j - 4
  Frag x, pf;
  x.h[0] = tr(x_img, (4 * kg + tq) * 32 + 4 * tp * 2);
  x.h[1] = tr(x_img, (16 + 4 * kg + tq) * 32 + 4 * tp * 2);
  // P[k][n] for this lane's column n = r16 at those k: B[n][k]
  const uint16_t* brow = reinterpret_cast<const uint16_t*>(b_img + r16 * 64);
  uint16_t pv[8];
  for (int j = 0; j < 4; ++j) { pv[j] = brow[4 * kg + j]; pv[4 + j] = brow[16 + 4 * kg + j]; }
  pf.u = make_uint4(pv[0] | (pv[1] << 16), pv[2] | (pv[3] << 16), pv[4] | (pv[5] << 16), pv[6] | (pv[7] << 16));
  f32x4 t = {0.f, 0.f, 0.f, 0.f};
  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x.v, pf.v, t, 0, 0, 0);
  for (int i = 0; i < 4; ++i) T[(4 * kg + i) * 16 + r16] = t[i];
}

static uint16_t bf(float f) { uint32_t u; std::memcpy(&u, &f, 4); return (uint16_t)(u >> 16); }
static float fb(uint16_t h) { uint32_t u = (uint32_t)h << 16; float f; std::memcpy(&f, &u, 4); return f; }

int main() {
  std::vector<uint16_t> A(512), B(512), X(512);
  for (int i = 0; i < 512; ++i) { A[i] = bf((i * 7 % 13) - 6); B[i] = bf((i * 5 % 11) - 5); X[i] = bf((i * 3 % 7) - 3); }
  uint16_t *dA, *dB, *dX; float *dS, *dT;
  hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dX, 1024); hipMalloc(&dS, 1024); hipMalloc(&dT, 1024);
  hipMemcpy(dA, A.data(), 1024, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), 1024, hipMemcpyHostToDevice);
  hipMemcpy(dX, X.data(), 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dX, dS, dT);
  std::vector<float> S(256), T(256);
  hipMemcpy(S.data(), dS, 1024, hipMemcpyDeviceToHost);
  hipMemcpy(T.data(), dT, 1024, hipMemcpyDeviceToHost);
  double es = 0, et = 0;
  for (int m = 0; m < 16; ++m)
    for (int n = 0; n < 16; ++n) {
      double s = 0, t = 0;
      for (int kk = 0; kk < 32; ++kk) { s += fb(A[m * 32 + kk]) * fb(B[n * 32 + kk]); t += fb(X[kk * 16 + m]) * fb(B[n * 32 + kk]); }
      es = fmax(es, fabs(s - S[m * 16 + n])); et = fmax(et, fabs(t - T[m * 16 + n]));
    }
  printf("S max err %g  T (transposed-read operand, permuted k) max err %g\n", es, et);
  printf("S[0][0..3] %g %g %g %g\n", S[0], S[1], S[2], S[3]);
  return 0;
}
