// fp16 instantiations of the flash attention kernels (csrc/kernels/flash_attn_kernels.h); compiled as a
// separate translation unit so the two 16-bit types build in parallel.
#include "flash_attn_kernels.h"

void pa_fa_fwd_f16(const FwdArgs& a, int D, int feat, dim3 grid, hipStream_t st) {
  fa_fwd_dispatch<true>(a, D, feat, grid, st);
}

void pa_fa_bwd_f16(const BwdArgs& a, int D, int feat, dim3 grid, hipStream_t st) {
  fa_bwd_dispatch<true>(a, D, feat, grid, st);
}

void pa_fa_bwd_aux_f16(int which, const BwdArgs& a, const uint16_t* o, const uint16_t* dout, float* delta,
                       const int64_t* os, const int64_t* dos, const float* dq_acc, uint16_t* dq, const int64_t* dqs,
                       int DB, int DS, int H, int D, hipStream_t st) {
  fa_bwd_aux<true>(which, a, o, dout, delta, os, dos, dq_acc, dq, dqs, DB, DS, H, D, st);
}
