// Direct 1-D convolution kernels for the encoder / decoder conv stacks
// (ref/model/vae_teb_model.py:128-253), on (B, L, C)
// activations.
//
// Forward: a workgroup owns (sample b, 64 output positions, 64 output
// channels).  For each chunk of 16 input channels it stages, in LDS, the input
// window [t0 - pad, t0 + 64 + K - 1 - pad) — reflect / replicate / causal-zero
// padding and the x2 linear upsample applied while staging, so no padded copy
// exists in HBM — and the filter taps W[co][ci][k] of the chunk; each thread
// then accumulates a 4 (positions) x 4 (channels) register tile over
// (k, ci) reading both operands from LDS (every staged input sample is reused
// K times, every tap 64 times).
// Backward-data is the same kernel on dY with transposed, flipped taps and
// causal padding (a "full" correlation over the padded input), followed by
// the fold of the padded/upsampled gradient (gemm.hip k_conv_fold).
// Backward-weight: a workgroup accumulates dW[64 co][16 ci][K] over a slice of
// the B*L_out rows from LDS-staged dY rows and input windows; slices are
// summed in fixed order.
#include "common.h"

namespace vt {

static constexpr int CT = 64;   // output positions per workgroup
static constexpr int CC = 64;   // output channels per workgroup
static constexpr int CI = 16;   // input-channel chunk
static constexpr int KMAX = 11;

struct Geo {
    int B, L_in, Cin, Cout, K, up, mode, L_up, pad, L_out;
};

// input value at padded position tp (upsampled domain) — see gemm.hip conv_src
__device__ __forceinline__ float src_val(const float* __restrict__ xb, const Geo& g, int tp, int ci) {
    int t = tp - g.pad;
    if (g.mode == 0) {
        if (t < 0 || t >= g.L_up) return 0.f;
    } else if (g.L_up <= g.pad) {
        t = t < 0 ? 0 : (t >= g.L_up ? g.L_up - 1 : t);
    } else {
        t = t < 0 ? -t : t;
        t = t >= g.L_up ? 2 * (g.L_up - 1) - t : t;
    }
    if (!g.up) return xb[(int64_t)t * g.Cin + ci];
    float s = (t + 0.5f) * 0.5f - 0.5f;
    s = s < 0.f ? 0.f : s;
    const int i0 = (int)s;
    const int i1 = i0 + 1 < g.L_in ? i0 + 1 : g.L_in - 1;
    const float l1 = s - (float)i0;
    return (1.f - l1) * xb[(int64_t)i0 * g.Cin + ci] + l1 * xb[(int64_t)i1 * g.Cin + ci];
}

// flip_t: use W[ci][co][K-1-k] (transposed, flipped) instead of W[co][ci][k]
template <bool FLIP_T>
__global__ __launch_bounds__(256) void k_conv_fwd(const float* __restrict__ x, Geo g, const float* __restrict__ w,
                                                  float* __restrict__ y) {
    __shared__ float xs[(CT + KMAX - 1) * CI];
    __shared__ __attribute__((aligned(16))) float ws[KMAX * CI * CC];
    const int tid = threadIdx.x;
    const int tx = tid & 15, ty = tid >> 4;     // tx: channel group (4), ty: position group (4)
    const int b = blockIdx.z;
    const int t0 = blockIdx.x * CT;
    const int co0 = blockIdx.y * CC;
    const int K = g.K;
    const int win = CT + K - 1;
    const float* xb = x + (int64_t)b * g.L_in * g.Cin;
    float acc[4][4] = {};
    for (int c0 = 0; c0 < g.Cin; c0 += CI) {
        const int cn = g.Cin - c0 < CI ? g.Cin - c0 : CI;
        for (int i = tid; i < win * CI; i += 256) {
            const int r = i / CI, c = i - r * CI;
            const int tp = t0 + r;
            xs[i] = (c < cn && tp < g.L_out + K - 1) ? src_val(xb, g, tp, c0 + c) : 0.f;
        }
        for (int i = tid; i < K * CI * CC; i += 256) {
            const int co = i % CC, rest = i / CC;
            const int c = rest % CI, k = rest / CI;
            float v = 0.f;
            if (c < cn && co0 + co < g.Cout) {
                const int gco = co0 + co, gci = c0 + c;
                v = FLIP_T ? w[((int64_t)gci * g.Cout + gco) * K + (K - 1 - k)]
                           : w[((int64_t)gco * g.Cin + gci) * K + k];
            }
            ws[(k * CI + c) * CC + co] = v;
        }
        __syncthreads();
        for (int k = 0; k < K; ++k) {
#pragma unroll 4
            for (int c = 0; c < CI; ++c) {
                const float4 wv = *reinterpret_cast<const float4*>(&ws[(k * CI + c) * CC + tx * 4]);
                const float wa[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float a = xs[(ty * 4 + i + k) * CI + c];
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a, wa[j], acc[i][j]);
                }
            }
        }
        __syncthreads();
    }
    const int Lo = FLIP_T ? g.L_out + K - 1 : g.L_out;  // bwd-data writes the padded length
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int t = t0 + ty * 4 + i;
        if (t >= Lo) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int co = co0 + tx * 4 + j;
            if (co < g.Cout) y[((int64_t)b * Lo + t) * g.Cout + co] = acc[i][j];
        }
    }
}

// dW partial: ws_out[split][co][ci][k] = sum over the split's rows of
// dY[b,t,co] * xpad[b, t+k, ci].  Workgroup: 64 co x 16 ci x K, rows in chunks of CT.
__global__ __launch_bounds__(256) void k_conv_dw(const float* __restrict__ dy, const float* __restrict__ x, Geo g,
                                                 int64_t rows_per_split, float* __restrict__ part) {
    __shared__ float ds[CT * CC];                       // dY chunk [t][co]
    __shared__ float xs[(CT + KMAX - 1) * CI];          // input window [tp][ci]
    const int tid = threadIdx.x;
    const int cg = tid & 15;        // co group of 4
    const int cil = tid >> 4;       // ci within chunk (0..15)
    const int co0 = blockIdx.x * CC;
    const int c0 = blockIdx.y * CI;
    const int K = g.K;
    const int64_t rows = (int64_t)g.B * g.L_out;
    const int64_t r0 = (int64_t)blockIdx.z * rows_per_split;
    const int64_t r1 = r0 + rows_per_split < rows ? r0 + rows_per_split : rows;
    float acc[4][KMAX];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < KMAX; ++k) acc[j][k] = 0.f;
    // rows are processed in chunks that never cross a sample boundary
    for (int64_t r = r0; r < r1;) {
        const int b = (int)(r / g.L_out);
        const int t0 = (int)(r - (int64_t)b * g.L_out);
        int n = g.L_out - t0;
        if (n > CT) n = CT;
        if (r + n > r1) n = (int)(r1 - r);
        const float* xb = x + (int64_t)b * g.L_in * g.Cin;
        const float* dyb = dy + ((int64_t)b * g.L_out + t0) * g.Cout;
        for (int i = tid; i < CT * CC; i += 256) {
            const int t = i / CC, co = i - t * CC;
            ds[i] = (t < n && co0 + co < g.Cout) ? dyb[(int64_t)t * g.Cout + co0 + co] : 0.f;
        }
        for (int i = tid; i < (CT + K - 1) * CI; i += 256) {
            const int tp = i / CI, c = i - tp * CI;
            xs[i] = (tp < n + K - 1 && c0 + c < g.Cin) ? src_val(xb, g, t0 + tp, c0 + c) : 0.f;
        }
        __syncthreads();
        for (int t = 0; t < n; ++t) {
            const float d0 = ds[t * CC + cg * 4 + 0], d1 = ds[t * CC + cg * 4 + 1];
            const float d2 = ds[t * CC + cg * 4 + 2], d3 = ds[t * CC + cg * 4 + 3];
#pragma unroll
            for (int k = 0; k < KMAX; ++k) {
                if (k < K) {
                    const float xv = xs[(t + k) * CI + cil];
                    acc[0][k] = fmaf(d0, xv, acc[0][k]);
                    acc[1][k] = fmaf(d1, xv, acc[1][k]);
                    acc[2][k] = fmaf(d2, xv, acc[2][k]);
                    acc[3][k] = fmaf(d3, xv, acc[3][k]);
                }
            }
        }
        __syncthreads();
        r += n;
    }
    const int ci = c0 + cil;
    if (ci >= g.Cin) return;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int co = co0 + cg * 4 + j;
        if (co >= g.Cout) continue;
#pragma unroll
        for (int k = 0; k < KMAX; ++k)
            if (k < K) part[(((int64_t)blockIdx.z * g.Cout + co) * g.Cin + ci) * K + k] = acc[j][k];
    }
}

// out[i] (+)= sum_s part[s][i], i < n (fixed order)
__global__ void k_sum_splits(const float* __restrict__ part, int splits, int64_t n, float* __restrict__ out,
                             int accumulate) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float a = 0.f;
#pragma unroll 8
    for (int s = 0; s < splits; ++s) a += part[(int64_t)s * n + i];
    out[i] = accumulate ? out[i] + a : a;
}

static Geo geo(int B, int L_in, int Cin, int Cout, int K, int mode, int up) {
    Geo g;
    g.B = B; g.L_in = L_in; g.Cin = Cin; g.Cout = Cout; g.K = K; g.mode = mode; g.up = up;
    g.L_up = L_in * (up ? 2 : 1);
    g.pad = mode == 0 ? K - 1 : (K - 1) / 2;
    g.L_out = mode == 0 ? g.L_up : g.L_up + 2 * g.pad - K + 1;
    return g;
}

}  // namespace vt

using namespace vt;

extern "C" {

int vt_conv1d_direct_fwd(const float* X, int B, int L_in, int Cin, const float* W, int Cout, int K, int mode, int up,
                         float* Y, void* stream) {
    VT_CHECK_ARG(B > 0 && L_in > 0 && Cin > 0 && Cout > 0 && K > 0 && K <= KMAX && (mode == 0 || mode == 1),
                 "vt_conv1d_direct_fwd: shape (K <= %d)", KMAX);
    Geo g = geo(B, L_in, Cin, Cout, K, mode, up);
    dim3 grid((g.L_out + CT - 1) / CT, (Cout + CC - 1) / CC, B);
    hipLaunchKernelGGL(k_conv_fwd<false>, grid, dim3(256), 0, S(stream), X, g, W, Y);
    VT_LAUNCH_CHECK("vt_conv1d_direct_fwd");
    return VT_OK;
}

// gpad[b, tp, ci] = sum_{k,co} dY[b, tp-k, co] W[co, ci, k], tp < L_out + K - 1:
// the forward kernel on dY (channels Cout -> Cin) with causal padding K-1 and
// transposed / flipped taps.
int vt_conv1d_direct_bwd_gpad(const float* dY, int B, int L_in, int Cin, const float* W, int Cout, int K, int mode,
                              int up, float* gpad, void* stream) {
    VT_CHECK_ARG(B > 0 && K <= KMAX, "vt_conv1d_direct_bwd_gpad: shape");
    Geo f = geo(B, L_in, Cin, Cout, K, mode, up);
    // geometry of the "full" correlation: input = dY (L_out x Cout), causal pad K-1
    Geo g = geo(B, f.L_out, Cout, Cin, K, 0, 0);
    g.L_out = f.L_out;  // kernel writes L_out + K - 1 rows (FLIP_T)
    dim3 grid((f.L_out + K - 1 + CT - 1) / CT, (Cin + CC - 1) / CC, B);
    hipLaunchKernelGGL(k_conv_fwd<true>, grid, dim3(256), 0, S(stream), dY, g, W, gpad);
    VT_LAUNCH_CHECK("vt_conv1d_direct_bwd_gpad");
    return VT_OK;
}

int vt_conv1d_direct_bwd_weight(const float* dY, const float* X, int B, int L_in, int Cin, int Cout, int K, int mode,
                                int up, float* dW, int accumulate, float* ws, int64_t ws_floats, void* stream) {
    VT_CHECK_ARG(B > 0 && K <= KMAX, "vt_conv1d_direct_bwd_weight: shape");
    Geo g = geo(B, L_in, Cin, Cout, K, mode, up);
    const int64_t rows = (int64_t)B * g.L_out;
    const int tiles = ((Cout + CC - 1) / CC) * ((Cin + CI - 1) / CI);
    const int64_t nout = (int64_t)Cout * Cin * K;
    int64_t splits = 1024 / tiles;
    if (splits < 1) splits = 1;
    if (splits > rows / CT) splits = rows / CT > 0 ? rows / CT : 1;
    if (splits * nout > ws_floats) splits = ws_floats / nout;
    VT_CHECK_ARG(splits >= 1, "vt_conv1d_direct_bwd_weight: workspace too small");
    int64_t rps = (rows + splits - 1) / splits;
    splits = (rows + rps - 1) / rps;
    dim3 grid((Cout + CC - 1) / CC, (Cin + CI - 1) / CI, (unsigned)splits);
    hipLaunchKernelGGL(k_conv_dw, grid, dim3(256), 0, S(stream), dY, X, g, rps, ws);
    hipLaunchKernelGGL(k_sum_splits, dim3((unsigned)((nout + 255) / 256)), dim3(256), 0, S(stream), ws, (int)splits,
                       nout, dW, accumulate);
    VT_LAUNCH_CHECK("vt_conv1d_direct_bwd_weight");
    return VT_OK;
}

}  // extern "C"
