// Skinny fp32 GEMMs of the ResidualMLP / LSTM-projection layers
// (ref/model/vae_teb_model.py:336-403 Linear -> LN -> act; :474-480, :647-653
// nn.LSTM input projections): rows = B*S = 65,536, widths <= 256, on the
// exact-fp32 matrix cores (v_mfma_f32_16x16x4_f32 = an fmaf chain at the
// 157 TF fp32 rate).  These layers are HBM-bound (a 64-wide activation is
// 16.8 MB), so the kernels are organised around one pass over the rows:
//
//  k_sk_gemm  C[R, Nc] = A[R, Kd] op(B): forward (B = W^T) and input gradient
//             (B = W).  A workgroup owns 16*PM*4 rows and ALL Nc columns, so
//             the forward can finish LayerNorm + activation in its epilogue
//             (row statistics by 16-lane shuffles over the accumulator layout)
//             and write y, xhat and rstd without re-reading the linear output.
//  k_sk_dw    dW[N, K] (+ db) = dY^T X over the rows: a workgroup streams a
//             contiguous row range through LDS and its 8 waves own the
//             16x16 (n, k) tile pairs (db as an extra ones-column of X);
//             per-workgroup slabs are summed in fixed order (k_sk_sum).
#include <stdlib.h>

#include "common.h"
#include "skinny.h"

namespace vt {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float sk_act(float z, int act) {
    switch (act) {
        case 1: return z > 0.f ? z : 0.f;
        case 2: return 0.5f * z * (1.f + erff(z * 0.70710678118654752f));
        case 3: return tanhf(z);
        default: return z;
    }
}

// sum over the 16 lanes of a row group (lanes l with equal l >> 4)
__device__ __forceinline__ float sum16(float v) {
    v += __shfl_xor(v, 1, 16);
    v += __shfl_xor(v, 2, 16);
    v += __shfl_xor(v, 4, 16);
    v += __shfl_xor(v, 8, 16);
    return v;
}

static constexpr int SK_KC = 32;  // reduction chunk staged per step
static constexpr int SK_AS = 50;  // A row stride in LDS (>= 32, == 18 mod 32: conflict-free fragments)

template <int NT>
struct SkCfg {
    static constexpr int PM = NT <= 8 ? 2 : 1;                     // 16-row tiles per wave
    static constexpr int ROWS = 4 * 16 * PM;                        // rows per workgroup (4 waves)
    static constexpr int BS = 16 * NT + ((NT & 1) ? 0 : 16);        // B row stride (== 16 mod 32)
};

// C[r][n] = sum_k A[r][k] B[k][n] (+ bias[n]).
// BT = true : B[k][n] = W[n][k], W is [Nc][Kd] (forward, W = nn.Linear.weight)
// BT = false: B[k][n] = W[k][n], W is [Kd][Nc] (input gradient, dX = dY W)
// EPI 0: C (+)= result.  EPI 1: z = result + bias -> LayerNorm(eps) -> gamma, beta
// -> act: C = y, XH = xhat, RS = rstd (any of them may be null).
template <int NT, bool BT, int EPI>
__global__ __launch_bounds__(256) void k_sk_gemm(const float* __restrict__ A, int64_t R, int Kd,
                                                 const float* __restrict__ W, int Nc, const float* __restrict__ bias,
                                                 float* __restrict__ C, int accumulate, const float* __restrict__ lg,
                                                 const float* __restrict__ lb, int act, float eps,
                                                 float* __restrict__ XH, float* __restrict__ RS) {
    using Cf = SkCfg<NT>;
    constexpr int PM = Cf::PM, ROWS = Cf::ROWS, BS = Cf::BS;
    __shared__ float As[ROWS * SK_AS];
    __shared__ float Bs[SK_KC * BS];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lr = lane & 15, lc = lane >> 4;
    const int64_t r0 = (int64_t)blockIdx.x * ROWS;
    f32x4 acc[PM][NT];
#pragma unroll
    for (int m = 0; m < PM; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int k0 = 0; k0 < Kd; k0 += SK_KC) {
        // A chunk: ROWS x 32, rows of 128 B (coalesced); all loads before the stores
        {
            constexpr int U = ROWS * SK_KC / 256;
            float v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = tid + 256 * u, row = i >> 5, col = i & 31;
                const int64_t gr = r0 + row;
                v[u] = (gr < R && k0 + col < Kd) ? A[gr * Kd + k0 + col] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = tid + 256 * u, row = i >> 5, col = i & 31;
                As[row * SK_AS + col] = v[u];
            }
        }
        // B chunk: 32 x 16*NT as Bs[k][n]
        {
            constexpr int U = (SK_KC * 16 * NT + 255) / 256;
            float v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = tid + 256 * u;
                float x = 0.f;
                if (i < SK_KC * 16 * NT) {
                    if (BT) {  // read along k (contiguous in W[n][.])
                        const int n = i >> 5, k = i & 31;
                        if (n < Nc && k0 + k < Kd) x = W[(int64_t)n * Kd + k0 + k];
                    } else {  // read along n (contiguous in W[k][.])
                        const int k = i / (16 * NT), n = i - k * (16 * NT);
                        if (n < Nc && k0 + k < Kd) x = W[(int64_t)(k0 + k) * Nc + n];
                    }
                }
                v[u] = x;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = tid + 256 * u;
                if (i < SK_KC * 16 * NT) {
                    int k, n;
                    if (BT) { n = i >> 5; k = i & 31; }
                    else { k = i / (16 * NT); n = i - k * (16 * NT); }
                    Bs[k * BS + n] = v[u];
                }
            }
        }
        __syncthreads();
        const int steps = (Kd - k0 < SK_KC ? Kd - k0 + 3 : SK_KC) >> 2;
        const float* ap = As + (16 * PM * wv + lr) * SK_AS + lc;
        const float* bp = Bs + lc * BS + lr;
        for (int s = 0; s < steps; ++s) {
            float a[PM], b[NT];
#pragma unroll
            for (int m = 0; m < PM; ++m) a[m] = ap[16 * m * SK_AS + 4 * s];
#pragma unroll
            for (int n = 0; n < NT; ++n) b[n] = bp[4 * s * BS + 16 * n];
#pragma unroll
            for (int m = 0; m < PM; ++m)
#pragma unroll
                for (int n = 0; n < NT; ++n) acc[m][n] = mfma4(a[m], b[n], acc[m][n]);
        }
        __syncthreads();
    }

    // D layout: col = 16 n + lr, row = 16 (PM wv + m) + 4 lc + r
    float bcol[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) {
        const int col = 16 * n + lr;
        bcol[n] = (bias && col < Nc) ? bias[col] : 0.f;
    }
#pragma unroll
    for (int m = 0; m < PM; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t row = r0 + 16 * (PM * wv + m) + 4 * lc + r;
            if (EPI == 0) {
                if (row >= R) continue;
#pragma unroll
                for (int n = 0; n < NT; ++n) {
                    const int col = 16 * n + lr;
                    if (col >= Nc) continue;
                    float o = acc[m][n][r] + bcol[n];
                    if (accumulate) o += C[row * Nc + col];
                    C[row * Nc + col] = o;
                }
            } else {
                // LayerNorm over the Nc columns of this row (all 16 lanes of the row group
                // take part in the shuffles, so the row guard comes after them)
                float z[NT], s = 0.f;
#pragma unroll
                for (int n = 0; n < NT; ++n) {
                    const int col = 16 * n + lr;
                    z[n] = col < Nc ? acc[m][n][r] + bcol[n] : 0.f;
                    s += z[n];
                }
                const float mean = sum16(s) / (float)Nc;
                float v = 0.f;
#pragma unroll
                for (int n = 0; n < NT; ++n) {
                    const int col = 16 * n + lr;
                    const float d = col < Nc ? z[n] - mean : 0.f;
                    v += d * d;
                }
                const float rstd = rsqrtf(sum16(v) / (float)Nc + eps);
                if (row >= R) continue;
#pragma unroll
                for (int n = 0; n < NT; ++n) {
                    const int col = 16 * n + lr;
                    if (col >= Nc) continue;
                    const float h = (z[n] - mean) * rstd;
                    if (XH) XH[row * Nc + col] = h;
                    if (C) C[row * Nc + col] = sk_act(h * lg[col] + lb[col], act);
                }
                if (RS && lr == 0) RS[row] = rstd;
            }
        }
}

// ---------------------------------------------------------------- weight grad
static constexpr int DW_ROWS = 32;   // rows per LDS chunk
static constexpr int DW_THREADS = 512;

// part[blk][n][k'] = sum over the workgroup's rows of dY[r][n] * X1[r][k'], where
// X1 = [X | X2 | 1] (X2 [R, K2] optional, K2 = 0 without; k' = K + K2 is the
// bias column when with_bias).  x2_shift > 0: X2's row r is the given matrix's row r - 1,
// zero where r % x2_shift == 0 (an LSTM's h_{t-1} read from h, x2_shift = S).  NTN x NTK tile pairs over 8 waves, PPW pairs
// per wave: when PPW is a multiple of NTK a wave owns PPW / NTK whole tile rows
// (its A fragments are read once per k-step for all NTK pairs of a row), else
// pairs are dealt round-robin.  The next 64-row chunk is loaded into registers
// while the MFMAs consume the current one from LDS.
template <int NTN, int NTK>
__global__ __launch_bounds__(DW_THREADS) void k_sk_dw(const float* __restrict__ dY, const float* __restrict__ X,
                                                      int64_t R, int N, int K, const float* __restrict__ X2, int K2,
                                                      int with_bias, int64_t rows_per_block,
                                                      float* __restrict__ part, int x2_shift) {
    constexpr int HS = 16 * NTN + ((NTN & 1) ? 0 : 16);  // == 16 mod 32
    constexpr int XS2 = 16 * NTK + ((NTK & 1) ? 0 : 16);
    constexpr int PAIRS = NTN * NTK, PPW = (PAIRS + 7) / 8;
    constexpr bool ROWS_OWNED = PAIRS % 8 == 0 && PPW % NTK == 0;
    constexpr int HT = DW_ROWS * 16 * NTN, UH = (HT + DW_THREADS - 1) / DW_THREADS;
    constexpr int XT = DW_ROWS * 16 * NTK, UX = (XT + DW_THREADS - 1) / DW_THREADS;
    __shared__ float Hs[DW_ROWS * HS];
    __shared__ float Xs[DW_ROWS * XS2];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lr = lane & 15, lc = lane >> 4;
    const int KX = K + K2, K1 = KX + (with_bias ? 1 : 0);
    auto pair_tn = [&](int j) { return ROWS_OWNED ? wv * (PPW / NTK) + j / NTK : (wv + 8 * j) / NTK; };
    auto pair_tk = [&](int j) { return ROWS_OWNED ? j % NTK : (wv + 8 * j) % NTK; };
    f32x4 acc[PPW];
#pragma unroll
    for (int j = 0; j < PPW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int64_t rb = (int64_t)blockIdx.x * rows_per_block;
    const int64_t re = rb + rows_per_block < R ? rb + rows_per_block : R;
    float vh[UH], vx[UX];
    auto load = [&](int64_t c0) {  // dY rows [t][n] and X1 rows [t][k'] of the chunk at c0
        const int n = re - c0 < DW_ROWS ? (int)(re - c0) : DW_ROWS;
        const int rm0 = x2_shift > 0 ? (int)(c0 % x2_shift) : 0;   // the chunk's first row within its sample
#pragma unroll
        for (int u = 0; u < UH; ++u) {
            const int i = tid + DW_THREADS * u;
            const int t = i / (16 * NTN), c = i - t * (16 * NTN);
            vh[u] = (i < HT && t < n && c < N) ? dY[(c0 + t) * N + c] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < UX; ++u) {
            const int i = tid + DW_THREADS * u;
            const int t = i / (16 * NTK), c = i - t * (16 * NTK);
            float x = 0.f;
            if (i < XT && t < n) {
                if (c < K) {
                    x = X[(c0 + t) * K + c];
                } else if (c < KX) {
                    if (x2_shift > 0) {   // R < 2^31 rows (checked by the caller)
                        int rm = rm0 + t;   // (c0 + t) mod x2_shift: one subtraction when x2_shift >= DW_ROWS
                        if (x2_shift >= DW_ROWS) rm = rm >= x2_shift ? rm - x2_shift : rm;
                        else rm %= x2_shift;
                        x = rm ? X2[(c0 + t - 1) * K2 + (c - K)] : 0.f;
                    } else {
                        x = X2[(c0 + t) * K2 + (c - K)];
                    }
                } else {
                    x = c == KX && with_bias ? 1.f : 0.f;
                }
            }
            vx[u] = x;
        }
    };
    if (rb < re) load(rb);
    for (int64_t c0 = rb; c0 < re; c0 += DW_ROWS) {
        const int n = re - c0 < DW_ROWS ? (int)(re - c0) : DW_ROWS;
#pragma unroll
        for (int u = 0; u < UH; ++u) {
            const int i = tid + DW_THREADS * u;
            const int t = i / (16 * NTN), c = i - t * (16 * NTN);
            if (i < HT) Hs[t * HS + c] = vh[u];
        }
#pragma unroll
        for (int u = 0; u < UX; ++u) {
            const int i = tid + DW_THREADS * u;
            const int t = i / (16 * NTK), c = i - t * (16 * NTK);
            if (i < XT) Xs[t * XS2 + c] = vx[u];
        }
        __syncthreads();
        if (c0 + DW_ROWS < re) load(c0 + DW_ROWS);  // in flight during this chunk's MFMAs
        const int groups = (n + 3) >> 2;
        for (int q = 0; q < groups; ++q) {
            const float* hp = Hs + (4 * q + lc) * HS + lr;
            const float* xp = Xs + (4 * q + lc) * XS2 + lr;
            if (ROWS_OWNED) {
                float xa[NTK];
#pragma unroll
                for (int tk = 0; tk < NTK; ++tk) xa[tk] = xp[16 * tk];
#pragma unroll
                for (int jr = 0; jr < PPW / NTK; ++jr) {
                    const float ha = hp[16 * (wv * (PPW / NTK) + jr)];
#pragma unroll
                    for (int tk = 0; tk < NTK; ++tk) acc[jr * NTK + tk] = mfma4(ha, xa[tk], acc[jr * NTK + tk]);
                }
            } else {
#pragma unroll
                for (int j = 0; j < PPW; ++j) {
                    if (PAIRS % 8 != 0 && wv + 8 * j >= PAIRS) continue;
                    acc[j] = mfma4(hp[16 * pair_tn(j)], xp[16 * pair_tk(j)], acc[j]);
                }
            }
        }
        __syncthreads();
    }
    // D: col (k') = 16 tk + lr, row (n) = 16 tn + 4 lc + r
    float* pb = part + (int64_t)blockIdx.x * N * K1;
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
        if (!ROWS_OWNED && wv + 8 * j >= PAIRS) continue;
        const int tn = pair_tn(j), tk = pair_tk(j);
        const int k = 16 * tk + lr;
        if (k >= K1) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int nn = 16 * tn + 4 * lc + r;
            if (nn < N) pb[nn * K1 + k] = acc[j][r];
        }
    }
}

// dW[n][k] (+)= sum_b part[b][n][k] (k < K), dW2[n][k - K] (k < K + K2), db[n]
// (and db2[n], when given) (+)= sum_b part[b][n][K + K2].  Fixed order: 64
// outputs per workgroup, wave w sums blocks w, w + 4, w + 8, ... in sequence
// (coalesced 256-byte rows, 16 loads in flight), then (w0 + w1) + (w2 + w3).
__global__ __launch_bounds__(256) void k_sk_sum(const float* __restrict__ part, int blocks, int N, int K, int K2,
                                                int K1, float* __restrict__ dW, float* __restrict__ dW2,
                                                float* __restrict__ db, float* __restrict__ db2, int accumulate) {
    __shared__ float red[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t total = (int64_t)N * K1;
    const int64_t i = (int64_t)blockIdx.x * 64 + lane;
    float a = 0.f;
    if (i < total) {
        const float* p = part + i;
        int b = w;
        for (; b + 60 < blocks; b += 64) {
            float v[16];
#pragma unroll
            for (int m = 0; m < 16; ++m) v[m] = p[(int64_t)(b + 4 * m) * total];
#pragma unroll
            for (int m = 0; m < 16; ++m) a += v[m];
        }
        for (; b < blocks; b += 4) a += p[(int64_t)b * total];
    }
    red[w][lane] = a;
    __syncthreads();
    if (w != 0 || i >= total) return;
    const float t = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    const int n = (int)(i / K1), k = (int)(i - (int64_t)n * K1);
    float* dst = k < K ? dW + (int64_t)n * K + k : (k < K + K2 ? dW2 + (int64_t)n * K2 + (k - K) : db + n);
    *dst = accumulate ? *dst + t : t;
    if (k == K + K2 && db2) db2[n] = accumulate ? db2[n] + t : t;
}

// ------------------------------------------------------------------- launchers
template <bool BT, int EPI>
static int sk_gemm_launch(const float* A, int64_t R, int Kd, const float* W, int Nc, const float* bias, float* C,
                          int accumulate, const float* lg, const float* lb, int act, float eps, float* XH, float* RS,
                          hipStream_t st) {
    const int NT = (Nc + 15) / 16;
#define VT_SK(NTV)                                                                                                 \
    case NTV: {                                                                                                    \
        const unsigned blocks = (unsigned)((R + SkCfg<NTV>::ROWS - 1) / SkCfg<NTV>::ROWS);                          \
        hipLaunchKernelGGL((k_sk_gemm<NTV, BT, EPI>), dim3(blocks), dim3(256), 0, st, A, R, Kd, W, Nc, bias, C,     \
                           accumulate, lg, lb, act, eps, XH, RS);                                                  \
        break;                                                                                                     \
    }
    switch (NT) {
        VT_SK(1) VT_SK(2) VT_SK(3) VT_SK(4) VT_SK(5) VT_SK(6) VT_SK(7) VT_SK(8) VT_SK(9) VT_SK(10) VT_SK(11)
        VT_SK(12) VT_SK(13) VT_SK(14) VT_SK(15) VT_SK(16)
        default: return VT_ERR_ARG;
    }
#undef VT_SK
    return VT_OK;
}

int sk_linear_fwd(const float* X, int64_t R, int K, const float* W, int N, const float* bias, float* Y,
                  hipStream_t st) {
    return sk_gemm_launch<true, 0>(X, R, K, W, N, bias, Y, 0, nullptr, nullptr, 0, 0.f, nullptr, nullptr, st);
}

int sk_linear_ln_fwd(const float* X, int64_t R, int K, const float* W, int N, const float* bias, const float* g,
                     const float* beta, int act, float eps, float* Y, float* XH, float* RS, hipStream_t st) {
    return sk_gemm_launch<true, 1>(X, R, K, W, N, bias, Y, 0, g, beta, act, eps, XH, RS, st);
}

int sk_linear_bwd_data(const float* dY, int64_t R, int N, const float* W, int K, float* dX, int accumulate,
                       hipStream_t st) {
    return sk_gemm_launch<false, 0>(dY, R, N, W, K, nullptr, dX, accumulate, nullptr, nullptr, 0, 0.f, nullptr,
                                    nullptr, st);
}

template <int NTN>
static void sk_dw_k(int NTK, dim3 grid, hipStream_t st, const float* dY, const float* X, int64_t R, int N, int K,
                    const float* X2, int K2, int wb, int64_t rpb, float* part, int x2_shift) {
#define VT_DWK(K_)                                                                                                 \
    case K_:                                                                                                       \
        hipLaunchKernelGGL((k_sk_dw<NTN, K_>), grid, dim3(DW_THREADS), 0, st, dY, X, R, N, K, X2, K2, wb, rpb,     \
                           part, x2_shift);                                                                        \
        break;
    switch (NTK) {
        VT_DWK(1) VT_DWK(2) VT_DWK(3) VT_DWK(4) VT_DWK(5) VT_DWK(6) VT_DWK(7) VT_DWK(8) VT_DWK(9)
    }
#undef VT_DWK
}

static int g_sk_dw_cap = 0;   // workgroup cap of k_sk_dw (VAETEB_SKDW_BLOCKS, default 256)

int64_t sk_dw_blocks(int64_t R) {
    if (g_sk_dw_cap == 0) {
        const char* e = getenv("VAETEB_SKDW_BLOCKS");
        g_sk_dw_cap = e ? atoi(e) : 256;
        if (g_sk_dw_cap < 1) g_sk_dw_cap = 256;
    }
    int64_t blocks = (R + 255) / 256;  // >= 256 rows each, at most g_sk_dw_cap workgroups
    return blocks > g_sk_dw_cap ? g_sk_dw_cap : (blocks < 1 ? 1 : blocks);
}

int64_t sk_dw_workspace(int64_t R, int N, int K) { return sk_dw_blocks(R) * N * (K + 1); }

int sk_linear_bwd_weight2(const float* dY, int64_t R, int N, const float* X, int K, const float* X2, int K2,
                          float* dW, float* dW2, float* db, float* db2, int accumulate, float* ws, int64_t ws_floats,
                          hipStream_t st, int x2_shift) {
    const int K1 = K + K2 + (db ? 1 : 0);
    if (x2_shift > 0 && R >= ((int64_t)1 << 31)) return VT_ERR_ARG;
    const int NTN = (N + 15) / 16, NTK = (K1 + 15) / 16;
    if (NTN > 16 || NTK > 9) return VT_ERR_ARG;
    int64_t blocks = sk_dw_blocks(R);
    if (blocks * N * K1 > ws_floats) blocks = ws_floats / ((int64_t)N * K1);
    if (blocks < 1) return VT_ERR_ARG;
    int64_t rpb = (R + blocks - 1) / blocks;
    rpb = (rpb + 3) / 4 * 4;
    blocks = (R + rpb - 1) / rpb;
    dim3 grid((unsigned)blocks);
    const int wb = db != nullptr;
    switch (NTN) {
        case 1: sk_dw_k<1>(NTK, grid, st, dY, X, R, N, K, X2, K2, wb, rpb, ws, x2_shift); break;
        case 2: sk_dw_k<2>(NTK, grid, st, dY, X, R, N, K, X2, K2, wb, rpb, ws, x2_shift); break;
        case 3: sk_dw_k<3>(NTK, grid, st, dY, X, R, N, K, X2, K2, wb, rpb, ws, x2_shift); break;
        case 4: sk_dw_k<4>(NTK, grid, st, dY, X, R, N, K, X2, K2, wb, rpb, ws, x2_shift); break;
        case 5: sk_dw_k<5>(NTK, grid, st, dY, X, R, N, K, X2, K2, wb, rpb, ws, x2_shift); break;
        case 6: sk_dw_k<6>(NTK, grid, st, dY, X, R, N, K, X2, K2, wb, rpb, ws, x2_shift); break;
        case 7: sk_dw_k<7>(NTK, grid, st, dY, X, R, N, K, X2, K2, wb, rpb, ws, x2_shift); break;
        case 8: sk_dw_k<8>(NTK, grid, st, dY, X, R, N, K, X2, K2, wb, rpb, ws, x2_shift); break;
        case 9: sk_dw_k<9>(NTK, grid, st, dY, X, R, N, K, X2, K2, wb, rpb, ws, x2_shift); break;
        default: sk_dw_k<16>(NTK, grid, st, dY, X, R, N, K, X2, K2, wb, rpb, ws, x2_shift); break;
    }
    const int64_t total = (int64_t)N * K1;
    hipLaunchKernelGGL(k_sk_sum, dim3((unsigned)((total + 63) / 64)), dim3(256), 0, st, ws, (int)blocks, N, K, K2, K1,
                       dW, dW2, db, db2, accumulate);
    return VT_OK;
}

void sk_sum_launch(const float* part, int blocks, int N, int K, int K2, int K1, float* dW, float* dW2, float* db,
                   float* db2, int accumulate, hipStream_t st) {
    const int64_t total = (int64_t)N * K1;
    hipLaunchKernelGGL(k_sk_sum, dim3((unsigned)((total + 63) / 64)), dim3(256), 0, st, part, blocks, N, K, K2, K1,
                       dW, dW2, db, db2, accumulate);
}

int sk_linear_bwd_weight(const float* dY, int64_t R, int N, const float* X, int K, float* dW, float* db,
                         int accumulate, float* ws, int64_t ws_floats, hipStream_t st) {
    return sk_linear_bwd_weight2(dY, R, N, X, K, nullptr, 0, dW, nullptr, db, nullptr, accumulate, ws, ws_floats, st);
}

}  // namespace vt
