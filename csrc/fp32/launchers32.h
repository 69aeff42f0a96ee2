// Host launch entry points of the fp32 kernels (csrc/fp32/*.hip, namespace pva_f32).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "f32_params.h"

namespace pva_f32 {
int igemm32_tile(int N);
int igemm32_bm(int N);   // output-position rows per workgroup (= rows per statistics partial)
void igemm32_launch(const Conv32& p, int np, hipStream_t s);   // np: bf16 pieces per fp32 operand (2 or 3)
void wgrad32_tile(int K, int Cout, int* bm, int* bn);
void wgrad32_launch(Wgrad32 p, int np, hipStream_t s);
void wpack32_launch(int mode, const float* src, void* dst, int Cout, int Cin, int taps, int cip, float beta,
                    hipStream_t s);
int chan_reduce32_blocks(int64_t M, int C);
void chan_reduce32_launch(const float* y, int ldy, const float* d, int ldd, const float* o, int ldo, const float* mean,
                          int mode, int relu, int64_t M, int C, int blocks, float* part, hipStream_t s);
void bn32_finalize_launch(const float* part, int R, int C, int64_t count, int mode, const float* gamma,
                          const float* beta, float* rmean, float* rvar, int64_t* nbt, float momentum, float eps,
                          float* stat, const float* fstat, float* dgamma, float* dbeta, float* coef, float gbeta,
                          hipStream_t s);
void bn32_apply_launch(const float* y, int ldy, const float* stat, const float* add, int lda, int relu, float* out,
                       int ldo, int64_t M, int C, hipStream_t s);
void bn32_bwd_apply_launch(const float* d, int ldd, const float* o, int ldo, int relu, const float* y, int ldy,
                           const float* fstat, const float* coef, float* dy, int lddy, float* gout, int ldg, int64_t M,
                           int C, hipStream_t s);
void copy32_launch(const float* src, int lds, float* dst, int ldd, int64_t M, int C, int acc, hipStream_t s);
void maxpool32_launch(int bwd, const float* a, float* b, uint8_t* arg, int N, int T, int H, int W, int To, int Ho,
                      int Wo, int C, const int* k, const int* st, const int* pd, hipStream_t s);
void avgpool32_launch(int bwd, const float* a, float* b, int N, int T, int H, int W, int C, int kt, int kh, int kw,
                      int ldf, int coff, hipStream_t s);
void to_ndhwc32_launch(const float* x, float* y, int N, int Cin, int64_t S, int Cp, hipStream_t s);
}  // namespace pva_f32
