// Skinny fp32-MFMA linear kernels (mlp.hip), dispatched from the vt_linear_*
// entry points of gemm.hip for widths <= 256.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vt {

constexpr int SK_MAX_N = 256;   // output columns of k_sk_gemm (16 tiles)
constexpr int SK_MAX_K1 = 144;  // K (+1 bias column) of k_sk_dw (9 tiles)

int sk_linear_fwd(const float* X, int64_t R, int K, const float* W, int N, const float* bias, float* Y,
                  hipStream_t st);
int sk_linear_ln_fwd(const float* X, int64_t R, int K, const float* W, int N, const float* bias, const float* g,
                     const float* beta, int act, float eps, float* Y, float* XH, float* RS, hipStream_t st);
int sk_linear_bwd_data(const float* dY, int64_t R, int N, const float* W, int K, float* dX, int accumulate,
                       hipStream_t st);
int64_t sk_dw_blocks(int64_t R);
int64_t sk_dw_workspace(int64_t R, int N, int K);
int sk_linear_bwd_weight(const float* dY, int64_t R, int N, const float* X, int K, float* dW, float* db,
                         int accumulate, float* ws, int64_t ws_floats, hipStream_t st);
// dW (+)= dY^T X, dW2 (+)= dY^T X2, db (and db2) (+)= column sums of dY, in one pass over dY
int sk_linear_bwd_weight2(const float* dY, int64_t R, int N, const float* X, int K, const float* X2, int K2,
                          float* dW, float* dW2, float* db, float* db2, int accumulate, float* ws, int64_t ws_floats,
                          hipStream_t st, int x2_shift = 0);
// the fixed-order sum of k_sk_dw's per-workgroup partial slabs part[blocks][N][K1] into dW / dW2 / db / db2
void sk_sum_launch(const float* part, int blocks, int N, int K, int K2, int K1, float* dW, float* dW2, float* db,
                   float* db2, int accumulate, hipStream_t st);
// skdw16.hip: the 16-bit LSTM's parameter gradients on bf16 MFMA (dG, x, h_{t-1} rounded to bf16,
// fp32 accumulation); VT_ERR_ARG when the shape / alignment is not supported
int sk_lstm16_dw(const float* dG, const float* x, int In, const float* h, int S, int64_t R, float* dW_ih,
                 float* dW_hh, float* db_ih, float* db_hh, int accumulate, float* ws, int64_t ws_floats,
                 hipStream_t st);

}  // namespace vt
