// 1-D convolution kernels for the encoder / decoder conv stacks
// (ref/model/vae_teb_model.py:128-253), on (B, L, C)
// activations, as implicit GEMMs on the exact-fp32 matrix cores
// (v_mfma_f32_16x16x4_f32: bit-for-bit an fmaf chain, at the 157 TF fp32 rate,
// ~2x what the VALU reaches on the same tiles).
//
// Forward: out[t][co] = sum_{k, ci} xpad[t + k][ci] W[co][ci][k].  A workgroup
// (4 waves) owns (sample b, TP output positions, TC = 16*NT output channels,
// NT fitted to Cout so the 77/66/55/.../1-channel layers carry little
// padding); per chunk of CI input channels it stages in LDS the input window
// [t0 - pad, t0 + TP + K - 1 - pad) — reflect / replicate / causal-zero padding
// and the x2 linear upsample applied while staging, so no padded copy exists
// in HBM — and the taps of the chunk.  Each wave multiplies PM x NT 16x16
// tiles: per (4 input channels, tap) it reads one A fragment per position
// tile (the window shifted by the tap) and one B fragment per channel tile.
// Backward-data is the same kernel on dY with transposed, flipped taps and
// causal padding (a "full" correlation over the padded input), followed by
// the fold of the padded/upsampled gradient (gemm.hip k_conv_fold).
// Backward-weight: dW[co][ci][k] = sum_rows dY[row][co] xpad[row + k][ci]; a
// workgroup stages a chunk of dY rows and input rows (all channels) and its 8
// waves each own up to PPW (16 co x 16 ci) tile pairs with K accumulators,
// reducing over rows 4 at a time (A = dY rows, B = the input rows shifted by
// each tap).  Rows are split over workgroups; the partial slabs are summed in
// fixed order.
#include "common.h"
#include "conv.h"

namespace vt {

typedef float f32x4 __attribute__((ext_vector_type(4)));

static constexpr int KMAX = 11;
static constexpr int XS = 18;               // forward window row stride: conflict-free A fragments
static constexpr int FWD_LDS = 16384;       // forward LDS budget (floats, 64 KB)
static constexpr int DR = 64;               // dW rows per chunk
static constexpr int SS = 112;              // dW LDS row stride (== 16 mod 32), max channels
static constexpr int DW_CMAX = 96;
static constexpr int SB = 8;                // staging batch (loads in flight per thread)

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int K, int NT>
struct FwdCfg {
    static constexpr int PM = NT <= 3 ? 4 : (NT == 4 ? 3 : 2);         // position tiles per wave
    static constexpr int TC = 16 * NT, TP = 64 * PM;                     // workgroup tile
    static constexpr int WIN = TP + K - 1;
    static constexpr int WS = (K * TC) % 32 == 0 ? K * TC + 16 : K * TC; // tap row stride (== 16 mod 32)
    static constexpr int XF = (WIN * XS + 3) & ~3;
    static constexpr int CI = XF + 16 * WS <= FWD_LDS ? 16 : 8;          // input channels per chunk
    static constexpr int LDS_BYTES = (XF + CI * WS) * 4;
};

// FLIP_T: taps W[ci][co][K-1-k] (transposed, flipped) instead of W[co][ci][k].
template <int K, int NT, bool FLIP_T>
// stats != null: also the BatchNorm statistics of this tile's outputs,
// stats[0][co][tile] = sum_t y, stats[1][co][tile] = sum_t (y - tile mean)^2 (channel-major)
// (tile = b * gridDim.x + blockIdx.x), combined by k_bn_stats_finalize.
__global__ __launch_bounds__(256) void k_conv_fwd(const float* __restrict__ x, Geo g, const float* __restrict__ w,
                                                  float* __restrict__ y, int Lo, float* __restrict__ stats) {
    using C = FwdCfg<K, NT>;
    constexpr int PM = C::PM, TC = C::TC, TP = C::TP, WIN = C::WIN, WS = C::WS, CI = C::CI;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* xs = lds;            // [WIN][XS]   window, channel-fastest
    float* ws = lds + C::XF;    // [CI][K][TC] taps (row stride WS)
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lr = lane & 15, lc = lane >> 4;
    const int t0 = blockIdx.x * TP, co0 = blockIdx.y * TC, b = blockIdx.z;
    const float* xb = x + (int64_t)b * g.L_in * g.Cin;
    f32x4 acc[PM][NT];
#pragma unroll
    for (int m = 0; m < PM; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int c0 = 0; c0 < g.Cin; c0 += CI) {
        const int cn = g.Cin - c0 < CI ? g.Cin - c0 : CI;
        // staging in batches of SB elements per thread: a batch's loads are all in
        // flight before its LDS stores (not one L2 round trip per element)
        constexpr int UX = (WIN * CI + 255) / 256, UW = (CI * K * TC + 255) / 256;
#pragma unroll 1
        for (int u0 = 0; u0 < UX; u0 += SB) {
            float v[SB];
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                const int i = tid + 256 * (u0 + u);
                const int r = i / CI, c = i - r * CI;
                const int tp = t0 + r;
                v[u] = (i < WIN * CI && c < cn && tp < Lo + K - 1) ? src_val(xb, g, tp, c0 + c) : 0.f;
            }
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                const int i = tid + 256 * (u0 + u);
                const int r = i / CI, c = i - r * CI;
                if (i < WIN * CI) xs[r * XS + c] = v[u];
            }
        }
        // taps, read in global order (contiguous (ci, k) runs per co; (co, k) per ci when flipped)
        auto tap_idx = [&](int i, int& co, int& c, int& k) {
            if (FLIP_T) {
                c = i / (TC * K);
                const int rest = i - c * (TC * K);
                co = rest / K;
                k = rest - co * K;
            } else {
                co = i / (CI * K);
                const int rest = i - co * (CI * K);
                c = rest / K;
                k = rest - c * K;
            }
        };
#pragma unroll 1
        for (int u0 = 0; u0 < UW; u0 += SB) {
            float v[SB];
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                const int i = tid + 256 * (u0 + u);
                int co, c, k;
                tap_idx(i, co, c, k);
                float val = 0.f;
                if (i < CI * K * TC && c < cn && co0 + co < g.Cout) {
                    const int gco = co0 + co, gci = c0 + c;
                    val = FLIP_T ? w[((int64_t)gci * g.Cout + gco) * K + (K - 1 - k)]
                                 : w[((int64_t)gco * g.Cin + gci) * K + k];
                }
                v[u] = val;
            }
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                const int i = tid + 256 * (u0 + u);
                int co, c, k;
                tap_idx(i, co, c, k);
                if (i < CI * K * TC) ws[c * WS + k * TC + co] = v[u];
            }
        }
        __syncthreads();
        const int ng = (cn + 3) >> 2;
        for (int q = 0; q < ng; ++q) {
            const float* xq = xs + (PM * 16 * wv + lr) * XS + 4 * q + lc;
            const float* wq = ws + (4 * q + lc) * WS + lr;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                float af[PM], bf[NT];
#pragma unroll
                for (int m = 0; m < PM; ++m) af[m] = xq[(16 * m + k) * XS];
#pragma unroll
                for (int n = 0; n < NT; ++n) bf[n] = wq[k * TC + 16 * n];
#pragma unroll
                for (int m = 0; m < PM; ++m)
#pragma unroll
                    for (int n = 0; n < NT; ++n) acc[m][n] = mfma4(af[m], bf[n], acc[m][n]);
            }
        }
        __syncthreads();
    }
    // D layout: col (channel) = lane & 15, row (position) = 4 * (lane >> 4) + r
#pragma unroll
    for (int m = 0; m < PM; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int t = t0 + PM * 16 * wv + 16 * m + 4 * lc + r;
            if (t >= Lo) continue;
            float* yr = y + ((int64_t)b * Lo + t) * g.Cout;
#pragma unroll
            for (int n = 0; n < NT; ++n) {
                const int co = co0 + 16 * n + lr;
                if (co < g.Cout) yr[co] = acc[m][n][r];
            }
        }
    if (stats) {
        // per-column sum, then sum of squared deviations from the tile mean, over
        // the tile's valid positions (lanes -> wave via shuffles, waves via LDS)
        float* red1 = lds;           // [4][TC]
        float* red2 = lds + 4 * TC;  // [4][TC]
        const int nrow = Lo - t0 < TP ? Lo - t0 : TP;
        float cs[NT];
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            float a = 0.f;
#pragma unroll
            for (int m = 0; m < PM; ++m)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (t0 + PM * 16 * wv + 16 * m + 4 * lc + r < Lo) a += acc[m][n][r];
            a += __shfl_xor(a, 16);
            a += __shfl_xor(a, 32);
            cs[n] = a;
        }
        if (lc == 0)
#pragma unroll
            for (int n = 0; n < NT; ++n) red1[wv * TC + 16 * n + lr] = cs[n];
        __syncthreads();
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            const int c = 16 * n + lr;
            const float mu = (((red1[c] + red1[TC + c]) + red1[2 * TC + c]) + red1[3 * TC + c]) / (float)nrow;
            float q = 0.f;
#pragma unroll
            for (int m = 0; m < PM; ++m)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (t0 + PM * 16 * wv + 16 * m + 4 * lc + r < Lo) {
                        const float dlt = acc[m][n][r] - mu;
                        q += dlt * dlt;
                    }
            q += __shfl_xor(q, 16);
            q += __shfl_xor(q, 32);
            if (lc == 0) red2[wv * TC + c] = q;
        }
        __syncthreads();
        if (tid < TC && co0 + tid < g.Cout) {
            const int64_t tile = (int64_t)b * gridDim.x + blockIdx.x;
            // channel-major [2][Cout][tiles] (k_bn_stats_finalize reads a channel as one run)
            const int64_t ntile = (int64_t)gridDim.z * gridDim.x;
            float* sp = stats + (int64_t)(co0 + tid) * ntile + tile;
            sp[0] = ((red1[tid] + red1[TC + tid]) + red1[2 * TC + tid]) + red1[3 * TC + tid];
            sp[(int64_t)g.Cout * ntile] = ((red2[tid] + red2[TC + tid]) + red2[2 * TC + tid]) + red2[3 * TC + tid];
        }
    }
}

// The fixed pairwise tree over a 256-thread workgroup's values (level o: v[t] += v[t + o],
// o = 128 .. 1) with the levels below 64 as wave-0 shuffles instead of LDS round trips and
// barriers: the same additions in the same order (the same bits); every thread gets the sum.
// red: 256 doubles of LDS, reusable on return.
__device__ __forceinline__ double tree256(double v, double* red) {
    const int tid = threadIdx.x;
    red[tid] = v;
    __syncthreads();
    if (tid < 128) red[tid] += red[tid + 128];
    __syncthreads();
    if (tid < 64) {
        double x = red[tid] + red[tid + 64];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o);
        if (tid == 0) red[0] = x;
    }
    __syncthreads();
    const double r = red[0];
    __syncthreads();
    return r;
}

// BatchNorm batch statistics from the conv tiles' (sum, M2) partials (Chan's
// parallel combination in double, fixed order): mean, rstd and the running
// statistics (torch momentum semantics, unbiased running variance).
// One workgroup per channel.
__global__ __launch_bounds__(256) void k_bn_stats_finalize(const float* __restrict__ stats, int tiles_per_sample,
                                                           int B, int TP, int Lo, int C, float eps, float momentum,
                                                           float* __restrict__ mean, float* __restrict__ rstd,
                                                           float* __restrict__ run_mean, float* __restrict__ run_var) {
    __shared__ double red[256];
    const int c = blockIdx.x, tid = threadIdx.x;
    const int ntile = B * tiles_per_sample;
    const double M = (double)B * Lo;
    const float* s0p = stats + (int64_t)c * ntile;        // channel-major [2][C][tiles]
    const float* s1p = stats + (int64_t)(C + c) * ntile;
    double a = 0.0;
    int i = tid;
    for (; i + 1792 < ntile; i += 2048) {   // eight coalesced loads in flight, same order
        float u[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) u[k] = s0p[i + 256 * k];
#pragma unroll
        for (int k = 0; k < 8; ++k) a += (double)u[k];
    }
    for (; i < ntile; i += 256) a += (double)s0p[i];
    const double mu = tree256(a, red) / M;
    double q = 0.0;
    auto m2 = [&](int i, float sv, float mv) {
        const int tx = i % tiles_per_sample;
        const int n = Lo - tx * TP < TP ? Lo - tx * TP : TP;
        const double s1 = (double)sv;
        const double dm = s1 / n - mu;
        q += (double)mv + n * dm * dm;
    };
    i = tid;
    for (; i + 1792 < ntile; i += 2048) {   // the same order, eight tiles' loads in flight
        float u[8], v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            u[k] = s0p[i + 256 * k];
            v[k] = s1p[i + 256 * k];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) m2(i + 256 * k, u[k], v[k]);
    }
    for (; i < ntile; i += 256) m2(i, s0p[i], s1p[i]);
    const double var = tree256(q, red) / M;
    if (tid != 0) return;
    mean[c] = (float)mu;
    rstd[c] = (float)(1.0 / sqrt(var + (double)eps));
    if (run_mean) {
        const double unb = M > 1 ? var * M / (M - 1) : var;
        run_mean[c] = (float)((1.0 - momentum) * run_mean[c] + momentum * mu);
        run_var[c] = (float)((1.0 - momentum) * run_var[c] + momentum * unb);
    }
}

// dW partial slabs: part[split][co][ci][k] over the split's rows.
// 8 waves; each wave owns PPW (16 co x 16 ci) tile pairs with K accumulators
// each.  When a layer has fewer pairs than waves, wpp waves share a pair and
// interleave its row groups.
template <int K, int PPW>
__global__ __launch_bounds__(512) void k_conv_dw(const float* __restrict__ dy, const float* __restrict__ x, Geo g,
                                                 int64_t rows_per_split, int NTc, int npairs, int wpp,
                                                 float* __restrict__ part) {
    __shared__ float ds[(DR + 4) * SS];             // dY chunk [row][co]
    __shared__ float xs[(DR + 4 + KMAX - 1) * SS];  // input window [row][ci]
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lr = lane & 15, lc = lane >> 4;
    const int ngroups = 8 / wpp, grp = wv / wpp, sub = wv % wpp;
    int mt[PPW], nt[PPW];
    bool act[PPW];
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
        const int p = blockIdx.x * (ngroups * PPW) + grp + ngroups * j;
        act[j] = grp < ngroups && p < npairs;
        mt[j] = p / NTc;
        nt[j] = p - mt[j] * NTc;
    }
    const int64_t rows = (int64_t)g.B * g.L_out;
    const int64_t r0 = (int64_t)blockIdx.y * rows_per_split;
    const int64_t r1 = r0 + rows_per_split < rows ? r0 + rows_per_split : rows;
    f32x4 acc[PPW][K];
#pragma unroll
    for (int j = 0; j < PPW; ++j)
#pragma unroll
        for (int k = 0; k < K; ++k) acc[j][k] = f32x4{0.f, 0.f, 0.f, 0.f};
    // rows are processed in chunks that never cross a sample boundary
    for (int64_t r = r0; r < r1;) {
        const int b = (int)(r / g.L_out);
        const int t0 = (int)(r - (int64_t)b * g.L_out);
        int n = g.L_out - t0;
        if (n > DR) n = DR;
        if (r + n > r1) n = (int)(r1 - r);
        const int n4 = (n + 3) & ~3;  // rows n .. n4-1 are zero (partial last row group)
        const float* xb = x + (int64_t)b * g.L_in * g.Cin;
        const float* dyb = dy + ((int64_t)b * g.L_out + t0) * g.Cout;
        // staging in batches of SB elements per thread (loads in flight before the
        // LDS stores).  Flat element index -> (row, channel) by a float reciprocal
        // (exact here: indices < 2^13, the fraction is >= 0.5 / C from an integer).
        const int nd = n4 * g.Cout, nx = (n4 + K - 1) * g.Cin;
        const float icout = 1.f / g.Cout, icin = 1.f / g.Cin;
#pragma unroll 1
        for (int i0 = 0; i0 < nd; i0 += 512 * SB) {
            float v[SB];
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                const int i = i0 + tid + 512 * u;
                const int t = (int)((i + 0.5f) * icout);
                v[u] = (i < nd && t < n) ? dyb[i] : 0.f;  // rows of dY are contiguous
            }
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                const int i = i0 + tid + 512 * u;
                const int t = (int)((i + 0.5f) * icout), c = i - t * g.Cout;
                if (i < nd) ds[t * SS + c] = v[u];
            }
        }
#pragma unroll 1
        for (int i0 = 0; i0 < nx; i0 += 512 * SB) {
            float v[SB];
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                const int i = i0 + tid + 512 * u;
                const int tp = (int)((i + 0.5f) * icin), c = i - tp * g.Cin;
                v[u] = (i < nx && tp < n + K - 1) ? src_val(xb, g, t0 + tp, c) : 0.f;
            }
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                const int i = i0 + tid + 512 * u;
                const int tp = (int)((i + 0.5f) * icin), c = i - tp * g.Cin;
                if (i < nx) xs[tp * SS + c] = v[u];
            }
        }
        __syncthreads();
        for (int q = sub; q < (n4 >> 2); q += wpp) {
            const float* dq = ds + (4 * q + lc) * SS + lr;
            const float* xq = xs + (4 * q + lc) * SS + lr;
#pragma unroll
            for (int j = 0; j < PPW; ++j) {
                if (!act[j]) continue;
                const float a = dq[16 * mt[j]];
#pragma unroll
                for (int k = 0; k < K; ++k) acc[j][k] = mfma4(a, xq[k * SS + 16 * nt[j]], acc[j][k]);
            }
        }
        __syncthreads();
        r += n;
    }
    // waves sharing a pair (wpp > 1) combine their accumulators through LDS in
    // fixed order, one tap at a time; the sub-0 wave then holds the pair's sum
    if (wpp > 1) {
        float* red = ds;  // 8 waves x 256 floats
#pragma unroll
        for (int k = 0; k < K; ++k) {
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) red[wv * 256 + rr * 64 + lane] = acc[0][k][rr];
            __syncthreads();
            if (sub == 0)
                for (int s2 = 1; s2 < wpp; ++s2)
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) acc[0][k][rr] += red[(wv + s2) * 256 + rr * 64 + lane];
            __syncthreads();
        }
        if (sub != 0) return;
    }
    // D: col (ci) = lane & 15, row (co) = 4 * (lane >> 4) + rr
    const int64_t slot = blockIdx.y;
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
        if (!act[j]) continue;
        const int ci = 16 * nt[j] + lr;
        if (ci >= g.Cin) continue;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int co = 16 * mt[j] + 4 * lc + rr;
            if (co >= g.Cout) continue;
            float* p = part + ((slot * g.Cout + co) * g.Cin + ci) * K;
#pragma unroll
            for (int k = 0; k < K; ++k) p[k] = acc[j][k][rr];
        }
    }
}

// output position of slab element i: identity, or (SumPerm) slab order [k][o][i] -> [o][i][k]
struct SumPerm {
    int K, Co, Ci;   // K == 0: identity
};
__device__ __forceinline__ int64_t perm_out(int64_t i, SumPerm p) {
    if (p.K == 0) return i;
    const int64_t ci = i % p.Ci, r = i / p.Ci, o = r % p.Co, k = r / p.Co;
    return (o * p.Ci + ci) * p.K + k;
}

// out[i] (+)= sum_s part[s][i] (fixed order): 64 outputs x 4 split lanes per workgroup
__global__ __launch_bounds__(256) void k_sum_splits(const float* __restrict__ part, int splits, int64_t n,
                                                    float* __restrict__ out, int accumulate, SumPerm pm) {
    __shared__ float red[4][64];
    const int o = threadIdx.x & 63, sl = threadIdx.x >> 6;
    const int64_t i = (int64_t)blockIdx.x * 64 + o;
    float a = 0.f;
    if (i < n) {
#pragma unroll 8
        for (int s = sl; s < splits; s += 4) a += part[(int64_t)s * n + i];   // 8 loads in flight, same order
    }
    red[sl][o] = a;
    __syncthreads();
    if (sl == 0 && i < n) {
        const float s = (red[0][o] + red[1][o]) + (red[2][o] + red[3][o]);
        const int64_t q = perm_out(i, pm);
        out[q] = accumulate ? out[q] + s : s;
    }
}


// launches the forward kernel (stats optional) and returns its position tile TP
template <int K, int NT, bool FLIP_T>
static int fwd_nt(const float* x, const Geo& g, const float* w, float* y, int Lo, float* stats, hipStream_t st) {
    using C = FwdCfg<K, NT>;
    dim3 grid(cdiv(Lo, C::TP), cdiv(g.Cout, C::TC), g.B);
    if (x) hipLaunchKernelGGL((k_conv_fwd<K, NT, FLIP_T>), grid, dim3(256), C::LDS_BYTES, st, x, g, w, y, Lo, stats);
    return C::TP;
}

template <int K, bool FLIP_T>
static int fwd_k(const float* x, const Geo& g, const float* w, float* y, int Lo, float* stats, hipStream_t st) {
    switch (cdiv(g.Cout, 16) < 6 ? cdiv(g.Cout, 16) : 6) {
        case 1: return fwd_nt<K, 1, FLIP_T>(x, g, w, y, Lo, stats, st);
        case 2: return fwd_nt<K, 2, FLIP_T>(x, g, w, y, Lo, stats, st);
        case 3: return fwd_nt<K, 3, FLIP_T>(x, g, w, y, Lo, stats, st);
        case 4: return fwd_nt<K, 4, FLIP_T>(x, g, w, y, Lo, stats, st);
        case 5: return fwd_nt<K, 5, FLIP_T>(x, g, w, y, Lo, stats, st);
        default: return fwd_nt<K, 6, FLIP_T>(x, g, w, y, Lo, stats, st);
    }
}

// x == nullptr: no launch, only the position tile TP of this geometry
template <bool FLIP_T>
static int launch_fwd(const float* x, const Geo& g, const float* w, float* y, int Lo, hipStream_t st,
                      float* stats = nullptr) {
    switch (g.K) {
        case 1: return fwd_k<1, FLIP_T>(x, g, w, y, Lo, stats, st);
        case 2: return fwd_k<2, FLIP_T>(x, g, w, y, Lo, stats, st);
        case 3: return fwd_k<3, FLIP_T>(x, g, w, y, Lo, stats, st);
        case 4: return fwd_k<4, FLIP_T>(x, g, w, y, Lo, stats, st);
        case 5: return fwd_k<5, FLIP_T>(x, g, w, y, Lo, stats, st);
        case 6: return fwd_k<6, FLIP_T>(x, g, w, y, Lo, stats, st);
        case 7: return fwd_k<7, FLIP_T>(x, g, w, y, Lo, stats, st);
        case 8: return fwd_k<8, FLIP_T>(x, g, w, y, Lo, stats, st);
        case 9: return fwd_k<9, FLIP_T>(x, g, w, y, Lo, stats, st);
        case 10: return fwd_k<10, FLIP_T>(x, g, w, y, Lo, stats, st);
        default: return fwd_k<11, FLIP_T>(x, g, w, y, Lo, stats, st);
    }
}

// Two-stage fixed-order reduction for many splits: stage 1 sums groups of SG_GRP
// consecutive slabs per output (one thread per output, coalesced across
// outputs, grid (outputs / 256, groups) — enough workgroups for the
// 2-6 K-output conv gradients whose one-stage sum ran on ~30 workgroups) and
// leaves each group's sum in place in the group's first slab; stage 2 sums the
// groups in order.
static constexpr int SG_GRP = 32;
VT_ARRIVE_POOL(g_arrive_splits);

// stage 1 per workgroup; the workgroup that arrives last among a column block's groups runs
// stage 2 for that block (the same fixed tree over the group sums as a separate pass would:
// the same bits, one launch)
__global__ __launch_bounds__(256) void k_sum_splits_grp(float* __restrict__ part, int splits, int64_t n,
                                                        float* __restrict__ out, int accumulate, unsigned slot0,
                                                        SumPerm pm) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int s0 = blockIdx.y * SG_GRP;
    const int s1 = s0 + SG_GRP < splits ? s0 + SG_GRP : splits;
    float a[SG_GRP];
    const __amdgpu_buffer_rsrc_t pr = agent_rsrc(part, (int64_t)splits * n * 4);   // splits * n < 2^29 (bwd_weight)
    if (i < n) {
        // every load of the group in flight at once, then a fixed pairwise tree
#pragma unroll
        for (int u = 0; u < SG_GRP; ++u) a[u] = s0 + u < s1 ? part[(int64_t)(s0 + u) * n + i] : 0.f;
#pragma unroll
        for (int w = SG_GRP / 2; w >= 1; w /= 2)
#pragma unroll
            for (int u = 0; u < w; ++u) a[u] += a[u + w];
        st_agent(pr, (unsigned)(((int64_t)s0 * n + i) * 4), a[0]);
    }
    if (!last_arrival(&g_arrive_splits[slot0 + blockIdx.x], gridDim.y) || i >= n) return;
    // the group sums (<= SG_GRP of them: splits <= SG_GRP^2) in flight at once, fixed tree
#pragma unroll
    for (int u = 0; u < SG_GRP; ++u) a[u] = ld_agent(pr, u * SG_GRP < splits ? (unsigned)(((int64_t)u * SG_GRP * n + i) * 4) : 0x80000000u);   // past the array: 0
#pragma unroll
    for (int w = SG_GRP / 2; w >= 1; w /= 2)
#pragma unroll
        for (int u = 0; u < w; ++u) a[u] += a[u + w];
    const int64_t q = perm_out(i, pm);
    out[q] = accumulate ? out[q] + a[0] : a[0];
}

// part is scratch: the two-stage path overwrites it
int sum_splits_launch(const float* part, int splits, int64_t n, float* out, int accumulate, hipStream_t st,
                      int pK, int pCo, int pCi) {
    const SumPerm pm{pK, pCo, pCi};
    // one stage only for few splits: with many (e.g. 330 slabs of the 74k-weight K = 11 layer) a
    // thread's serial loop over the slabs was latency-bound (80 us); the group stage keeps
    // SG_GRP loads in flight per thread at any n
    if (splits <= 2 * SG_GRP) {
        hipLaunchKernelGGL(k_sum_splits, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, st, part, splits, n, out,
                           accumulate, pm);
        return VT_OK;
    }
    if (splits > SG_GRP * SG_GRP) return VT_ERR_ARG;
    float* p = const_cast<float*>(part);
    const unsigned bx = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(k_sum_splits_grp, dim3(bx, (unsigned)((splits + SG_GRP - 1) / SG_GRP)), dim3(256), 0, st, p,
                       splits, n, out, accumulate, arrive_slots(bx, st), pm);
    return VT_OK;
}

int bn_stats_finalize_launch(const float* stats, int tiles_per_sample, int B, int TP, int Lo, int C, float eps,
                             float momentum, float* mean, float* rstd, float* run_mean, float* run_var,
                             hipStream_t st) {
    hipLaunchKernelGGL(k_bn_stats_finalize, dim3(C), dim3(256), 0, st, stats, tiles_per_sample, B, TP, Lo, C, eps,
                       momentum, mean, rstd, run_mean, run_var);
    return VT_OK;
}


}  // namespace vt

using namespace vt;

extern "C" {

int vt_conv1d_bn_workspace_floats(int B, int L_in, int Cin, int Cout, int K, int mode, int up, int64_t* floats) {
    VT_CHECK_ARG(B > 0 && L_in > 0 && Cin > 0 && Cout > 0 && K > 0 && K <= KMAX, "vt_conv1d_bn_workspace_floats");
    Geo g = geo(B, L_in, Cin, Cout, K, mode, up);
    *floats = (int64_t)B * cdiv(g.L_out, 64) * 2 * Cout;  // any position tile >= 64 (fp32 and bf16 kernels)
    return VT_OK;
}

int vt_conv1d_bn_fwd(const float* X, int B, int L_in, int Cin, const float* W, int Cout, int K, int mode, int up,
                     const float* gamma, const float* beta, int act, float eps, float momentum, float* conv_out,
                     float* Y, float* mean, float* rstd, float* run_mean, float* run_var, float* ws,
                     int64_t ws_floats, void* stream) {
    VT_CHECK_ARG(B > 0 && L_in > 0 && Cin > 0 && Cout > 0 && K > 0 && K <= KMAX && (mode == 0 || mode == 1),
                 "vt_conv1d_bn_fwd: shape (K <= %d)", KMAX);
    Geo g = geo(B, L_in, Cin, Cout, K, mode, up);
    const int TP = launch_fwd<false>(nullptr, g, nullptr, nullptr, g.L_out, nullptr);
    const int tps = cdiv(g.L_out, TP);
    VT_CHECK_ARG(ws && ws_floats >= (int64_t)B * tps * 2 * Cout, "vt_conv1d_bn_fwd: workspace too small");
    hipStream_t st = S(stream);
    launch_fwd<false>(X, g, W, conv_out, g.L_out, st, ws);
    hipLaunchKernelGGL(k_bn_stats_finalize, dim3(Cout), dim3(256), 0, st, ws, tps, B, TP, g.L_out, Cout, eps,
                       momentum, mean, rstd, run_mean, run_var);
    const int rc = bn_apply_launch(conv_out, (int64_t)B * g.L_out, Cout, mean, rstd, gamma, beta, act, Y, st);
    if (rc) return rc;
    VT_LAUNCH_CHECK("vt_conv1d_bn_fwd");
    return VT_OK;
}

int vt_conv1d_direct_fwd(const float* X, int B, int L_in, int Cin, const float* W, int Cout, int K, int mode, int up,
                         float* Y, void* stream) {
    VT_CHECK_ARG(B > 0 && L_in > 0 && Cin > 0 && Cout > 0 && K > 0 && K <= KMAX && (mode == 0 || mode == 1),
                 "vt_conv1d_direct_fwd: shape (K <= %d)", KMAX);
    Geo g = geo(B, L_in, Cin, Cout, K, mode, up);
    launch_fwd<false>(X, g, W, Y, g.L_out, S(stream));
    VT_LAUNCH_CHECK("vt_conv1d_direct_fwd");
    return VT_OK;
}

// gpad[b, tp, ci] = sum_{k,co} dY[b, tp-k, co] W[co, ci, k], tp < L_out + K - 1:
// the forward kernel on dY (channels Cout -> Cin) with causal padding K-1 and
// transposed / flipped taps.
int vt_conv1d_direct_bwd_gpad(const float* dY, int B, int L_in, int Cin, const float* W, int Cout, int K, int mode,
                              int up, float* gpad, void* stream) {
    VT_CHECK_ARG(B > 0 && L_in > 0 && Cin > 0 && Cout > 0 && K > 0 && K <= KMAX, "vt_conv1d_direct_bwd_gpad: shape");
    Geo f = geo(B, L_in, Cin, Cout, K, mode, up);
    // geometry of the "full" correlation: input = dY (L_out x Cout), causal pad K-1
    Geo g = geo(B, f.L_out, Cout, Cin, K, 0, 0);
    launch_fwd<true>(dY, g, W, gpad, f.L_out + K - 1, S(stream));
    VT_LAUNCH_CHECK("vt_conv1d_direct_bwd_gpad");
    return VT_OK;
}

int vt_conv1d_direct_bwd_weight(const float* dY, const float* X, int B, int L_in, int Cin, int Cout, int K, int mode,
                                int up, float* dW, int accumulate, float* ws, int64_t ws_floats, void* stream) {
    VT_CHECK_ARG(B > 0 && L_in > 0 && K > 0 && K <= KMAX && Cin > 0 && Cout > 0 && Cin <= DW_CMAX &&
                     Cout <= DW_CMAX,
                 "vt_conv1d_direct_bwd_weight: shape (K <= %d, channels <= %d)", KMAX, DW_CMAX);
    Geo g = geo(B, L_in, Cin, Cout, K, mode, up);
    const int NTc = cdiv(Cin, 16), npairs = cdiv(Cout, 16) * NTc;
    const int ppw = K <= 5 ? 4 : (K == 6 || K == 7 ? 3 : 2);  // pairs per wave (K accumulators each)
    const int wpp = npairs >= 8 ? 1 : 8 / npairs;               // waves per pair for narrow layers
    const int per_block = (8 / wpp) * (wpp > 1 ? 1 : ppw);
    const int bx = cdiv(npairs, per_block);
    const int64_t rows = (int64_t)B * g.L_out;
    const int64_t nout = (int64_t)Cout * Cin * K;
    // ~512 workgroups, >= 4 row chunks each, partial slabs <= 8M floats and within the workspace
    int64_t splits = 512 / bx;
    if (splits * nout > (int64_t)8 << 20) splits = ((int64_t)8 << 20) / nout;
    if (splits > rows / (4 * DR)) splits = rows / (4 * DR);
    if (splits < 1) splits = 1;
    if (splits * nout > ws_floats) splits = ws_floats / nout;
    VT_CHECK_ARG(splits >= 1, "vt_conv1d_direct_bwd_weight: workspace too small");
    int64_t rps = (rows + splits - 1) / splits;
    splits = (rows + rps - 1) / rps;
    dim3 grid(bx, (unsigned)splits);
    hipStream_t st = S(stream);
    const int P = wpp > 1 ? 1 : ppw;
#define VT_CONV_DW(KK, PP) \
    if (K == KK && P == PP) \
        hipLaunchKernelGGL((k_conv_dw<KK, PP>), grid, dim3(512), 0, st, dY, X, g, rps, NTc, npairs, wpp, ws);
    VT_CONV_DW(1, 1) VT_CONV_DW(1, 4) VT_CONV_DW(2, 1) VT_CONV_DW(2, 4) VT_CONV_DW(3, 1) VT_CONV_DW(3, 4)
    VT_CONV_DW(4, 1) VT_CONV_DW(4, 4) VT_CONV_DW(5, 1) VT_CONV_DW(5, 4) VT_CONV_DW(6, 1) VT_CONV_DW(6, 3)
    VT_CONV_DW(7, 1) VT_CONV_DW(7, 3) VT_CONV_DW(8, 1) VT_CONV_DW(8, 2) VT_CONV_DW(9, 1) VT_CONV_DW(9, 2)
    VT_CONV_DW(10, 1) VT_CONV_DW(10, 2) VT_CONV_DW(11, 1) VT_CONV_DW(11, 2)
#undef VT_CONV_DW
    if (const int rc = sum_splits_launch(ws, (int)splits, nout, dW, accumulate, st)) {
        set_error("vt_conv1d_direct_bwd_weight: %d weight-gradient slabs exceed the split sum's limit", (int)splits);
        return rc;
    }
    VT_LAUNCH_CHECK("vt_conv1d_direct_bwd_weight");
    return VT_OK;
}

}  // extern "C"
