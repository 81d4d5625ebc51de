// fp32 tiled GEMM engine for the model's small dense layers and 1-D conv
// stacks (SURVEY.md §8(a) a10, a11, a13, a15 and the LSTM input projections).
//
// C[M,N] = sum_k A(m,k) * B(k,n), A and B supplied by loader functors, so one
// kernel covers: Linear fwd (X W^T), Linear bwd-data (dY W), Linear bwd-weight
// (dY^T X, split-K over the 65k rows), and the conv blocks as implicit GEMMs
// whose A-loader gathers the im2col window straight from the (B, L, C)
// activation — fusing kymatio-style reflect padding, replicate fallback,
// causal left padding and the x2 linear upsample of
// ref/model/vae_teb_model.py:182-253 into the operand load (no padded or
// upsampled copy ever hits HBM).
//
// Tile 64x64x16, 256 threads (4 waves), 4x4 fp32 accumulators per thread;
// LDS operand images [k][m] / [k][n] padded by one float4 to keep the 16
// distinct float4 reads per wave conflict free.  Split-K partials go to a
// caller workspace and are reduced in fixed order (bit-reproducible).
#include <algorithm>

#include "common.h"
#include "skinny.h"

namespace vt {

static constexpr int TM = 64, TN = 64, TK = 16, GT = 256;

// ------------------------------------------------------------------ loaders
// Each loader: float at(m, k) for in-range indices; M_FAST/K_FAST tell the
// kernel which index is contiguous in memory (for coalesced tile loads).
struct RowMajor {            // P[r * ld + c]; (r, c) = (first, second) index
    const float* p;
    int64_t ld;
    __device__ float at(int64_t r, int64_t c) const { return p[r * ld + c]; }
};
struct ColMajor {            // P[c * ld + r]
    const float* p;
    int64_t ld;
    __device__ float at(int64_t r, int64_t c) const { return p[c * ld + r]; }
};

// Conv geometry shared by the gather loaders.  Activations are (B, L, C).
struct ConvGeom {
    int B, L_in, Cin, Cout, K;
    int up;       // 1: x2 linear upsample (align_corners=False) before padding
    int mode;     // 0: causal (left K-1 zeros); 1: reflect (p = (K-1)/2), replicate if L_up <= p
    int L_up;     // L_in * (up ? 2 : 1)
    int pad;      // left pad in the upsampled domain
    int L_out;    // output length
};

// value of the padded / upsampled input at padded position tp (channel ci)
__device__ __forceinline__ float conv_src(const float* __restrict__ x, const ConvGeom& g, int b, int tp, int ci) {
    int t = tp - g.pad;  // position in the upsampled signal
    if (g.mode == 0) {
        if (t < 0) return 0.f;
    } else if (g.L_up <= g.pad) {
        t = t < 0 ? 0 : (t >= g.L_up ? g.L_up - 1 : t);  // replicate
    } else {
        t = t < 0 ? -t : t;
        t = t >= g.L_up ? 2 * (g.L_up - 1) - t : t;        // reflect
    }
    const float* xb = x + (int64_t)b * g.L_in * g.Cin + ci;
    if (!g.up) return xb[(int64_t)t * g.Cin];
    // F.interpolate(scale 2, linear, align_corners=False)
    float src = (t + 0.5f) * 0.5f - 0.5f;
    src = src < 0.f ? 0.f : src;
    const int i0 = (int)src;
    const int i1 = i0 + 1 < g.L_in ? i0 + 1 : g.L_in - 1;
    const float l1 = src - (float)i0, l0 = 1.f - l1;
    return l0 * xb[(int64_t)i0 * g.Cin] + l1 * xb[(int64_t)i1 * g.Cin];
}

// A(m = b*L_out + t, kk = k*Cin + ci) = xpad[b, t + k, ci]
struct Im2col {
    const float* x;
    ConvGeom g;
    __device__ float at(int64_t m, int64_t kk) const {
        const int b = (int)(m / g.L_out), t = (int)(m - (int64_t)b * g.L_out);
        const int k = (int)(kk / g.Cin), ci = (int)(kk - (int64_t)k * g.Cin);
        return conv_src(x, g, b, t + k, ci);
    }
};
// B(kk = k*Cin + ci, co) = W[co, ci, k]   (torch Conv1d weight layout)
struct ConvW {
    const float* w;
    int Cin, K;
    __device__ float at(int64_t kk, int64_t co) const {
        const int k = (int)(kk / Cin), ci = (int)(kk - (int64_t)k * Cin);
        return w[(co * Cin + ci) * K + k];
    }
};
// bwd-data: A(m = b*Lp + tp, kk = k*Cout + co) = dY[b, tp - k, co] (0 outside)
struct Col2imA {
    const float* dy;
    int L_out, Lp, Cout;
    __device__ float at(int64_t m, int64_t kk) const {
        const int b = (int)(m / Lp), tp = (int)(m - (int64_t)b * Lp);
        const int k = (int)(kk / Cout), co = (int)(kk - (int64_t)k * Cout);
        const int t = tp - k;
        return (t >= 0 && t < L_out) ? dy[((int64_t)b * L_out + t) * Cout + co] : 0.f;
    }
};
// B(kk = k*Cout + co, ci) = W[co, ci, k]
struct ConvWT {
    const float* w;
    int Cin, Cout, K;
    __device__ float at(int64_t kk, int64_t ci) const {
        const int k = (int)(kk / Cout), co = (int)(kk - (int64_t)k * Cout);
        return w[((int64_t)co * Cin + ci) * K + k];
    }
};

// ------------------------------------------------------------------ kernel
// Output: if ws != nullptr, raw partial sums ws[z][m][n]; else
// C[m*ldc + n] = (accumulate ? C : 0) + acc + (bias ? bias[n] : 0).
template <class LA, class LB, bool A_M_FAST, bool B_N_FAST>
__global__ __launch_bounds__(GT) void k_gemm(LA la, LB lb, int64_t M, int N, int64_t K, int64_t k_chunk,
                                             float* __restrict__ C, int64_t ldc, const float* __restrict__ bias,
                                             int accumulate, float* __restrict__ ws) {
    __shared__ __attribute__((aligned(16))) float As[TK][TM + 4];
    __shared__ __attribute__((aligned(16))) float Bs[TK][TN + 4];
    const int tid = threadIdx.x;
    const int ty = tid >> 4, tx = tid & 15;
    const int64_t m0 = (int64_t)blockIdx.x * TM;
    const int n0 = blockIdx.y * TN;
    const int64_t kb = (int64_t)blockIdx.z * k_chunk;
    const int64_t ke = kb + k_chunk < K ? kb + k_chunk : K;
    float acc[4][4] = {};
    // register prefetch: the global loads of tile k0+TK are issued before the
    // FMAs of tile k0, so their latency hides under the compute
    float ra[4], rb[4];
    auto fetch = [&](int64_t k0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int idx = tid + GT * i;
            int mm, kk;
            if (A_M_FAST) { kk = idx >> 6; mm = idx & 63; } else { mm = idx >> 4; kk = idx & 15; }
            const int64_t gm = m0 + mm, gk = k0 + kk;
            ra[i] = (gm < M && gk < ke) ? la.at(gm, gk) : 0.f;
            int nn, kb2;
            if (B_N_FAST) { kb2 = idx >> 6; nn = idx & 63; } else { nn = idx >> 4; kb2 = idx & 15; }
            const int gn = n0 + nn;
            const int64_t gk2 = k0 + kb2;
            rb[i] = (gn < N && gk2 < ke) ? lb.at(gk2, gn) : 0.f;
        }
    };
    if (kb < ke) fetch(kb);
    for (int64_t k0 = kb; k0 < ke; k0 += TK) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int idx = tid + GT * i;
            int mm, kk;
            if (A_M_FAST) { kk = idx >> 6; mm = idx & 63; } else { mm = idx >> 4; kk = idx & 15; }
            As[kk][mm] = ra[i];
            int nn, kb2;
            if (B_N_FAST) { kb2 = idx >> 6; nn = idx & 63; } else { nn = idx >> 4; kb2 = idx & 15; }
            Bs[kb2][nn] = rb[i];
        }
        __syncthreads();
        if (k0 + TK < ke) fetch(k0 + TK);
#pragma unroll
        for (int kk = 0; kk < TK; ++kk) {
            const float4 a = *reinterpret_cast<const float4*>(&As[kk][ty * 4]);
            const float4 b = *reinterpret_cast<const float4*>(&Bs[kk][tx * 4]);
            const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(av[i], bv[j], acc[i][j]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int64_t m = m0 + ty * 4 + i;
        if (m >= M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n0 + tx * 4 + j;
            if (n >= N) continue;
            if (ws) {
                ws[((int64_t)blockIdx.z * M + m) * N + n] = acc[i][j];
            } else {
                float v = acc[i][j] + (bias ? bias[n] : 0.f);
                if (accumulate) v += C[m * ldc + n];
                C[m * ldc + n] = v;
            }
        }
    }
}

// out[m, n] (+)= sum_z ws[z, m, n] + bias; layout 0 row-major (ldc), 1 conv
// weight (m = co, n = k*Cin + ci -> C[(co*Cin + ci)*K + k]), 2 row-major with
// the last column (the fused ones-column = bias gradient) written to col_out[m].
__global__ void k_splitk_reduce(const float* __restrict__ ws, int splits, int64_t M, int N, float* __restrict__ C,
                                int64_t ldc, const float* __restrict__ bias, int accumulate, int layout, int Cin,
                                int Kw, float* __restrict__ col_out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M * N) return;
    const int64_t m = i / N;
    const int n = (int)(i - m * N);
    float v = 0.f;
#pragma unroll 8
    for (int z = 0; z < splits; ++z) v += ws[(int64_t)z * M * N + i];
    if (bias) v += bias[n];
    float* o;
    if (layout == 1) {
        const int k = n / Cin, ci = n - k * Cin;
        o = C + (m * Cin + ci) * Kw + k;
    } else if (layout == 2 && n == N - 1) {
        o = col_out + m;
    } else {
        o = C + m * ldc + n;
    }
    if (accumulate) v += *o;
    *o = v;
}

struct RowMajorOnes {        // X[r * ld + c] for c < K, 1 for c == K (fused bias-gradient column)
    const float* p;
    int64_t ld;
    int K;
    __device__ float at(int64_t r, int64_t c) const { return c < K ? p[r * ld + c] : 1.f; }
};

// column sums: out[n] (+)= sum_m X[m, n] over a row-major (M, N) matrix.
// Two-stage, fixed order: partial[block][n] then reduction.
// 256 threads cover rpi = 256/N rows x N columns per iteration (coalesced rows);
// columns wider than 256 loop.  Partials combined per column in LDS.
__global__ __launch_bounds__(256) void k_colsum_partial(const float* __restrict__ X, int64_t M, int N,
                                                        int64_t rows_per_block, float* __restrict__ partial) {
    __shared__ float red[256];
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = r0 + rows_per_block < M ? r0 + rows_per_block : M;
    if (N <= 256) {
        const int rpi = 256 / N;
        const int c = threadIdx.x % N, ro = threadIdx.x / N;
        // four independent accumulators: four loads in flight per thread
        float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
        if (ro < rpi) {
            int64_t r = r0 + ro;
            for (; r + 3 * rpi < r1; r += 4 * rpi) {
                a0 += X[r * N + c];
                a1 += X[(r + rpi) * N + c];
                a2 += X[(r + 2 * rpi) * N + c];
                a3 += X[(r + 3 * rpi) * N + c];
            }
            for (; r < r1; r += rpi) a0 += X[r * N + c];
        }
        const float a = (a0 + a1) + (a2 + a3);
        red[threadIdx.x] = a;
        __syncthreads();
        if (threadIdx.x < N) {
            float s = 0.f;
            for (int i = 0; i < rpi; ++i) s += red[i * N + threadIdx.x];
            partial[(int64_t)blockIdx.x * N + threadIdx.x] = s;
        }
    } else {  // one column per thread, grid.y over 256-column chunks
        const int n = blockIdx.y * 256 + threadIdx.x;
        if (n >= N) return;
        float a = 0.f;
        for (int64_t r = r0; r < r1; ++r) a += X[r * N + n];
        partial[(int64_t)blockIdx.x * N + n] = a;
    }
}
// one workgroup per column
__global__ __launch_bounds__(256) void k_colsum_final(const float* __restrict__ partial, int blocks, int N,
                                                      float* __restrict__ out, int accumulate) {
    __shared__ float red[16];
    const int n = blockIdx.x;
    float a = 0.f;
#pragma unroll 8
    for (int b = threadIdx.x; b < blocks; b += 256) a += partial[(int64_t)b * N + n];   // 8 loads in flight, same order
    a = block_sum(a, red);
    if (threadIdx.x == 0) out[n] = accumulate ? out[n] + a : a;
}

// conv bwd-data fold: gradient of the padded / upsampled input (B, Lp, Cin)
// back onto the real input (B, L_in, Cin): sum over the padded positions that
// read each upsampled sample, then through the linear-interpolation weights.
// One sample per grid row (blockIdx.y), 32-bit position / channel arithmetic
// within it (host check: Lp * Cin < 2^31); (s, ci) through a float reciprocal
// while positions are exact in fp32 (rcin = 0: integer division).
template <bool UP>
__global__ void k_conv_fold(const float* __restrict__ gpad, ConvGeom g, float rcin, float* __restrict__ dx,
                            int accumulate) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;  // s * Cin + ci within sample b
    if (i >= g.L_in * g.Cin) return;
    const int b = blockIdx.y;
    const int Lp = g.L_out + g.K - 1;  // padded length the bwd-data GEMM produced
    const float* gb0 = gpad + (int64_t)b * Lp * g.Cin;
    float out;
    if (!UP && g.mode == 0) {
        out = gb0[g.pad * g.Cin + i];  // causal: padded rows [pad, pad + L) are the input rows, a flat copy
    } else {
        // (s, ci) = divmod(i, Cin) through the reciprocal, corrected by one either way
        int s = rcin != 0.f ? (int)((float)i * rcin) : i / g.Cin;
        if (s * g.Cin > i) --s;
        else if ((s + 1) * g.Cin <= i) ++s;
        const int ci = i - s * g.Cin;
        const float* gb = gb0 + ci;
        // gradient of upsampled position t: sum of padded positions tp with map(tp) == t
        auto gup = [&](int t) -> float {
            float v = gb[(t + g.pad) * g.Cin];  // the direct copy
            if (g.mode == 0) return v;
            if (g.L_up <= g.pad) {  // replicate: edges collect the pads
                if (t == 0)
                    for (int tp = 0; tp < g.pad; ++tp) v += gb[tp * g.Cin];
                if (t == g.L_up - 1)
                    for (int tp = g.pad + g.L_up; tp < Lp; ++tp) v += gb[tp * g.Cin];
                return v;
            }
            if (t >= 1 && t <= g.pad) v += gb[(g.pad - t) * g.Cin];                        // left mirror
            const int tr = g.pad + 2 * (g.L_up - 1) - t;                                   // right mirror
            if (t <= g.L_up - 2 && tr < Lp && tr >= g.pad + g.L_up) v += gb[tr * g.Cin];
            return v;
        };
        if (!UP) {
            out = gup(s);
        } else {
            // adjoint of the x2 linear upsample (align_corners=False): upsampled t reads
            // i0 = floor(max((t + .5) / 2 - .5, 0)) with 1 - l and i1 = min(i0 + 1, L - 1) with l, so input s
            // collects t = 2s - 1 (1/4), 2s (3/4; 1 at s = 0), 2s + 1 (3/4; 1 at s = L - 1), 2s + 2 (1/4),
            // summed in increasing t
            out = 0.f;
            if (s >= 1) out = fmaf(0.25f, gup(2 * s - 1), out);
            out = fmaf(s == 0 ? 1.f : 0.75f, gup(2 * s), out);
            out = fmaf(s == g.L_in - 1 ? 1.f : 0.75f, gup(2 * s + 1), out);
            if (2 * s + 2 <= g.L_up - 1) out = fmaf(0.25f, gup(2 * s + 2), out);
        }
    }
    float* o = dx + (int64_t)b * g.L_in * g.Cin + i;
    *o = accumulate ? *o + out : out;
}

static int fold_launch(const float* gpad, const ConvGeom& g, float* dX, int accumulate, hipStream_t st) {
    VT_CHECK_ARG((int64_t)(g.L_out + g.K - 1) * g.Cin < (1ll << 31) && g.B <= 65535, "conv fold: shape");
    const dim3 grid((unsigned)((g.L_in * g.Cin + 255) / 256), (unsigned)g.B);
    const float rcin = (int64_t)g.L_in * g.Cin < (1 << 24) ? 1.f / (float)g.Cin : 0.f;
    if (g.up)
        hipLaunchKernelGGL(k_conv_fold<true>, grid, dim3(256), 0, st, gpad, g, rcin, dX, accumulate);
    else
        hipLaunchKernelGGL(k_conv_fold<false>, grid, dim3(256), 0, st, gpad, g, rcin, dX, accumulate);
    return VT_OK;
}

static inline dim3 gemm_grid(int64_t M, int N, int splits) {
    return dim3((unsigned)((M + TM - 1) / TM), (unsigned)((N + TN - 1) / TN), (unsigned)splits);
}

template <class LA, class LB, bool AM, bool BN>
static int launch(const char* name, LA la, LB lb, int64_t M, int N, int64_t K, float* C, int64_t ldc,
                  const float* bias, int accumulate, float* ws, int64_t ws_floats, int splits_wanted, int layout,
                  int Cin, int Kw, hipStream_t st, float* col_out = nullptr) {
    int splits = 1;
    if (splits_wanted > 1 && ws) {
        int64_t cap = ws_floats / (M * (int64_t)N);
        int64_t maxs = (K + TK - 1) / TK;
        splits = (int)std::min<int64_t>(std::min<int64_t>(splits_wanted, cap), maxs);
        if (splits < 1) splits = 1;
    }
    if (splits == 1 && layout == 0) {
        hipLaunchKernelGGL((k_gemm<LA, LB, AM, BN>), gemm_grid(M, N, 1), dim3(GT), 0, st, la, lb, M, N, K, K, C, ldc,
                           bias, accumulate, (float*)nullptr);
    } else {
        if (!ws || ws_floats < M * (int64_t)N * splits) {
            set_error("%s: workspace too small (%lld floats needed)", name, (long long)(M * (int64_t)N * splits));
            return VT_ERR_ARG;
        }
        int64_t chunk = (K + splits - 1) / splits;
        chunk = (chunk + TK - 1) / TK * TK;
        splits = (int)((K + chunk - 1) / chunk);
        hipLaunchKernelGGL((k_gemm<LA, LB, AM, BN>), gemm_grid(M, N, splits), dim3(GT), 0, st, la, lb, M, N, K, chunk,
                           C, ldc, bias, accumulate, ws);
        const int64_t tot = M * (int64_t)N;
        hipLaunchKernelGGL(k_splitk_reduce, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, ws, splits, M, N, C,
                           ldc, bias, accumulate, layout, Cin, Kw, col_out);
    }
    VT_LAUNCH_CHECK(name);
    return VT_OK;
}

static ConvGeom make_geom(int B, int L_in, int Cin, int Cout, int K, int mode, int up) {
    ConvGeom g;
    g.B = B; g.L_in = L_in; g.Cin = Cin; g.Cout = Cout; g.K = K; g.mode = mode; g.up = up;
    g.L_up = L_in * (up ? 2 : 1);
    g.pad = mode == 0 ? K - 1 : (K - 1) / 2;
    g.L_out = mode == 0 ? g.L_up : g.L_up + 2 * g.pad - K + 1;
    return g;
}

}  // namespace vt

using namespace vt;

extern "C" {

int vt_gemm_splits_hint(int64_t M, int N, int64_t K) {
    const int64_t tiles = ((M + TM - 1) / TM) * ((N + TN - 1) / TN);
    // ~4 workgroups per CU (latency hiding), >= 256 reduction rows per split,
    // <= 256 splits so the fixed-order split reduction stays short
    int64_t s = 1024 / (tiles > 0 ? tiles : 1);
    int64_t maxs = (K + 255) / 256;
    if (maxs > 256) maxs = 256;
    if (s > maxs) s = maxs;
    return (int)(s < 1 ? 1 : s);
}

// Y[R,N] = X[R,K] W[N,K]^T + b   (nn.Linear)
int vt_linear_fwd(const float* X, int64_t R, int K, const float* W, int N, const float* bias, float* Y,
                  void* stream) {
    VT_CHECK_ARG(R > 0 && K > 0 && N > 0, "vt_linear_fwd: shape");
    if (N <= SK_MAX_N) {
        sk_linear_fwd(X, R, K, W, N, bias, Y, S(stream));
        VT_LAUNCH_CHECK("vt_linear_fwd");
        return VT_OK;
    }
    return launch<RowMajor, ColMajor, false, false>("vt_linear_fwd", RowMajor{X, K}, ColMajor{W, K}, R, N, K, Y, N,
                                                    bias, 0, nullptr, 0, 1, 0, 0, 0, S(stream));
}

// dX[R,K] (+)= dY[R,N] W[N,K]
int vt_linear_bwd_data(const float* dY, int64_t R, int N, const float* W, int K, float* dX, int accumulate,
                       void* stream) {
    VT_CHECK_ARG(R > 0 && K > 0 && N > 0, "vt_linear_bwd_data: shape");
    if (K <= SK_MAX_N) {
        sk_linear_bwd_data(dY, R, N, W, K, dX, accumulate, S(stream));
        VT_LAUNCH_CHECK("vt_linear_bwd_data");
        return VT_OK;
    }
    return launch<RowMajor, RowMajor, false, true>("vt_linear_bwd_data", RowMajor{dY, N}, RowMajor{W, K}, R, K, N, dX,
                                                   K, nullptr, accumulate, nullptr, 0, 1, 0, 0, 0, S(stream));
}

// dW[N,K] (+)= dY[R,N]^T X[R,K]  (split-K over R through `ws`)
int vt_linear_bwd_weight(const float* dY, int64_t R, int N, const float* X, int K, float* dW, float* db,
                         int accumulate, float* ws, int64_t ws_floats, void* stream) {
    VT_CHECK_ARG(R > 0 && K > 0 && N > 0, "vt_linear_bwd_weight: shape");
    if (N <= SK_MAX_N && K + 1 <= SK_MAX_K1 && sk_dw_workspace(R, N, K) <= ws_floats) {
        int rc = sk_linear_bwd_weight(dY, R, N, X, K, dW, db, accumulate, ws, ws_floats, S(stream));
        VT_CHECK_ARG(rc == VT_OK, "vt_linear_bwd_weight: workspace too small");
        VT_LAUNCH_CHECK("vt_linear_bwd_weight");
        return VT_OK;
    }
    if (db) {  // bias gradient fused as an extra ones-column of X
        const int K1 = K + 1;
        int splits = vt_gemm_splits_hint(N, K1, R);
        return launch<ColMajor, RowMajorOnes, true, true>("vt_linear_bwd_weight", ColMajor{dY, N},
                                                          RowMajorOnes{X, K, K}, N, K1, R, dW, K, nullptr, accumulate,
                                                          ws, ws_floats, splits, 2, 0, 0, S(stream), db);
    }
    return launch<ColMajor, RowMajor, true, true>("vt_linear_bwd_weight", ColMajor{dY, N}, RowMajor{X, K}, N, K, R, dW,
                                                  K, nullptr, accumulate, ws, ws_floats, vt_gemm_splits_hint(N, K, R),
                                                  0, 0, 0, S(stream));
}

// fold of a padded / upsampled input gradient gpad (B, L_out+K-1, Cin) onto dX (B, L_in, Cin)
int vt_conv1d_fold(const float* gpad, int B, int L_in, int Cin, int Cout, int K, int mode, int up, float* dX,
                   int accumulate, void* stream) {
    VT_CHECK_ARG(B > 0 && L_in > 0 && Cin > 0, "vt_conv1d_fold: shape");
    ConvGeom g = make_geom(B, L_in, Cin, Cout, K, mode, up);
    const int rc = fold_launch(gpad, g, dX, accumulate, S(stream));
    if (rc) return rc;
    VT_LAUNCH_CHECK("vt_conv1d_fold");
    return VT_OK;
}

// Y = act(LayerNorm(X W^T + b)) fused (ResidualMLP hidden layer), also xhat / rstd
int vt_linear_ln_fwd(const float* X, int64_t R, int K, const float* W, int N, const float* bias, const float* gamma,
                     const float* beta, int act, float eps, float* Y, float* xhat, float* rstd, void* stream) {
    VT_CHECK_ARG(R > 0 && K > 0 && N > 0 && N <= SK_MAX_N && gamma && beta && act >= 0 && act <= 3,
                 "vt_linear_ln_fwd: shape (N <= %d)", SK_MAX_N);
    sk_linear_ln_fwd(X, R, K, W, N, bias, gamma, beta, act, eps, Y, xhat, rstd, S(stream));
    VT_LAUNCH_CHECK("vt_linear_ln_fwd");
    return VT_OK;
}

// out[N] (+)= column sums of X[R,N]  (bias / BN-beta gradients)
int vt_colsum(const float* X, int64_t R, int N, float* out, int accumulate, float* ws, int64_t ws_floats,
              void* stream) {
    VT_CHECK_ARG(R > 0 && N > 0, "vt_colsum: shape");
    // narrow N: 64 rows per block (1024 blocks at 65,536 rows); wide N: a thread per
    // column and 8 rows per block (512 workgroups for the 256 x 4096 head gradients)
    const int64_t rows = N <= 256 ? 64 : 8;
    int64_t blocks = (R + rows - 1) / rows;
    if (blocks > 1024) blocks = 1024;
    if (blocks * N > ws_floats) blocks = ws_floats / N;
    VT_CHECK_ARG(blocks >= 1, "vt_colsum: workspace too small");
    const int64_t rpb = (R + blocks - 1) / blocks;
    blocks = (R + rpb - 1) / rpb;
    hipLaunchKernelGGL(k_colsum_partial, dim3((unsigned)blocks, N <= 256 ? 1 : (unsigned)((N + 255) / 256)),
                       dim3(256), 0, S(stream), X, R, N, rpb, ws);
    hipLaunchKernelGGL(k_colsum_final, dim3(N), dim3(256), 0, S(stream), ws, (int)blocks, N, out,
                       accumulate);
    VT_LAUNCH_CHECK("vt_colsum");
    return VT_OK;
}

// 1-D conv over (B, L, C) activations, no bias (the reference's blocks use bias=False).
// mode 0: CausalMultiChannelConvBlock (left pad K-1, vae_teb_model.py:198-203)
// mode 1: MultiChannelConvBlock (reflect pad (K-1)/2 or replicate when L <= p,
//         optional x2 linear upsample first, vae_teb_model.py:232-251)
int vt_conv1d_out_len(int L_in, int K, int mode, int up) { return make_geom(1, L_in, 1, 1, K, mode, up).L_out; }

int vt_conv1d_fwd(const float* X, int B, int L_in, int Cin, const float* W, int Cout, int K, int mode, int up,
                  float* Y, void* stream) {
    VT_CHECK_ARG(B > 0 && L_in > 0 && Cin > 0 && Cout > 0 && K > 0 && (mode == 0 || mode == 1),
                 "vt_conv1d_fwd: shape");
    ConvGeom g = make_geom(B, L_in, Cin, Cout, K, mode, up);
    VT_CHECK_ARG(mode == 0 || g.L_up > 1, "vt_conv1d_fwd: length");
    const int64_t M = (int64_t)B * g.L_out;
    return launch<Im2col, ConvW, false, false>("vt_conv1d_fwd", Im2col{X, g}, ConvW{W, Cin, K}, M, Cout,
                                               (int64_t)K * Cin, Y, Cout, nullptr, 0, nullptr, 0, 1, 0, 0, 0,
                                               S(stream));
}

// dX (+)= conv1d input gradient.  gpad: caller scratch of B*(L_out+K-1)*Cin floats.
int vt_conv1d_bwd_data(const float* dY, int B, int L_in, int Cin, const float* W, int Cout, int K, int mode, int up,
                       float* dX, int accumulate, float* gpad, void* stream) {
    VT_CHECK_ARG(B > 0 && L_in > 0 && Cin > 0 && Cout > 0 && K > 0, "vt_conv1d_bwd_data: shape");
    ConvGeom g = make_geom(B, L_in, Cin, Cout, K, mode, up);
    const int Lp = g.L_out + K - 1;
    const int64_t M = (int64_t)B * Lp;
    int rc = launch<Col2imA, ConvWT, false, false>("vt_conv1d_bwd_data", Col2imA{dY, g.L_out, Lp, Cout},
                                                   ConvWT{W, Cin, Cout, K}, M, Cin, (int64_t)K * Cout, gpad, Cin,
                                                   nullptr, 0, nullptr, 0, 1, 0, 0, 0, S(stream));
    if (rc) return rc;
    rc = fold_launch(gpad, g, dX, accumulate, S(stream));
    if (rc) return rc;
    VT_LAUNCH_CHECK("vt_conv1d_bwd_data(fold)");
    return VT_OK;
}

// dW[Cout, Cin, K] (+)= sum_{b,t} dY[b,t,co] * xpad[b, t+k, ci]  (split-K over B*L_out)
int vt_conv1d_bwd_weight(const float* dY, const float* X, int B, int L_in, int Cin, int Cout, int K, int mode, int up,
                         float* dW, int accumulate, float* ws, int64_t ws_floats, void* stream) {
    VT_CHECK_ARG(B > 0 && L_in > 0 && Cin > 0 && Cout > 0 && K > 0, "vt_conv1d_bwd_weight: shape");
    ConvGeom g = make_geom(B, L_in, Cin, Cout, K, mode, up);
    const int64_t Mrows = (int64_t)B * g.L_out;
    const int N = K * Cin;
    // C[co, kk] = sum_m dY[m, co] * im2col[m, kk]
    return launch<ColMajor, Im2col, true, true>("vt_conv1d_bwd_weight", ColMajor{dY, Cout}, Im2col{X, g}, Cout, N,
                                                 Mrows, dW, 0, nullptr, accumulate, ws, ws_floats,
                                                 std::max(2, vt_gemm_splits_hint(Cout, N, Mrows)), 1, Cin, K,
                                                 S(stream));
}

}  // extern "C"
