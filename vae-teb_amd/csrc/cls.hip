// Classifier kernels for config 4: FHRInceptionTimeClassifier
// (ref/model/inception_time.py:9-333) trained jointly with SeqVaeTeb
// (SeqVaeTebClassifier.compute_loss, ref/model/vae_teb_model.py:1440-1498).
//
// Activations are (B, L, C) row-major matrices with an explicit row stride, so
// the inception concatenation torch.concat([x1, x2, x3, x4], dim=1) is four
// column slices of one (B*L, 128) buffer written in place by the branch
// kernels, and the reference's (B, C, L) <-> (B, L, C) transposes vanish.
//
//  k_zconv_fwd   zero-padded conv (K 1/5/15/40) as an implicit GEMM on the
//                exact-fp32 matrix cores (v_mfma_f32_16x16x4_f32): a workgroup
//                owns 128 positions x all output channels of one sample; per
//                chunk of input channels it stages the zero-padded window and
//                the taps in LDS; each wave multiplies 2 x NT 16x16 tiles.  The
//                backward-data is the same kernel over dY with the transposed,
//                flipped taps.
//  k_zconv_dw    dW[o][i][k] = sum_rows dY[row][o] X[row+k-pad][i]: one
//                workgroup per group of samples, 8 waves each owning up to 20
//                (16 o x 16 i x tap) tiles, rows 4 at a time from LDS; slabs
//                summed in fixed order (k_sum_splits).
//  k_attn_fwd    softmax(Q K^T) V per (sample, head, 64 queries): K / V of the
//                head in LDS, S^T = K Q^T in registers (so the column softmax
//                is lane-local plus two shuffles and P^T is already the B
//                operand of O^T = V^T P^T: no LDS round trip for P).
//  k_attn_bwd    one workgroup per (sample, head), a wave per 64 keys, query
//                tiles of 16: P recomputed from the saved log-sum-exp, dV / dK
//                accumulated in registers, dQ through a fixed-order LDS sum.
// Everything is deterministic (no atomics).
#include <math.h>

#include "common.h"
#include "conv.h"

namespace vt {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mma(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ------------------------------------------------------------ zero-pad conv
constexpr int ZT = 256;           // threads per forward workgroup (4 waves)
constexpr int ZPM = 2;            // 16-position tiles per wave
constexpr int ZTP = 64 * ZPM;     // positions per workgroup

template <int K, int NT>
struct ZCfg {
    static constexpr int TC = 16 * NT;
    static constexpr int CI = K * TC * 16 <= 12288 ? 16 : 8;      // input channels per LDS chunk
    static constexpr int XS = CI + 2;                              // window row stride
    static constexpr int WIN = ZTP + K - 1;
    static constexpr int XF = (WIN * XS + 3) & ~3;
    static constexpr int WS = (K * TC) % 32 == 0 ? K * TC + 16 : K * TC;  // tap row stride
    static constexpr int LDS_BYTES = (XF + CI * WS) * 4;
};

// FLIP: taps W[i][o][K-1-k] of a weight stored [Ci_orig = Cout][Co_orig = Cin][K]
// (the backward-data of a conv whose input had Cout channels).
template <int K, int NT, bool FLIP>
__global__ __launch_bounds__(ZT) void k_zconv_fwd(const float* __restrict__ X, int ldx, int L, int Cin,
                                                  const float* __restrict__ W, int Cout, int pad,
                                                  float* __restrict__ Y, int ldy, int accumulate) {
    using C = ZCfg<K, NT>;
    constexpr int TC = C::TC, CI = C::CI, XS = C::XS, WIN = C::WIN, WS = C::WS;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* xs = lds;           // [WIN][XS]
    float* ws = lds + C::XF;   // [CI][K][TC] (row stride WS)
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lr = lane & 15, lc = lane >> 4;
    const int t0 = blockIdx.x * ZTP, b = blockIdx.y;
    const float* xb = X + (int64_t)b * L * ldx;
    f32x4 acc[ZPM][NT];
#pragma unroll
    for (int m = 0; m < ZPM; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int c0 = 0; c0 < Cin; c0 += CI) {
        const int cn = Cin - c0 < CI ? Cin - c0 : CI;
#pragma unroll 4
        for (int i = tid; i < WIN * CI; i += ZT) {
            const int r = i / CI, c = i - r * CI;
            const int t = t0 + r - pad;
            xs[r * XS + c] = (c < cn && t >= 0 && t < L) ? xb[(int64_t)t * ldx + c0 + c] : 0.f;
        }
#pragma unroll 4
        for (int i = tid; i < CI * K * TC; i += ZT) {
            int o, c, k;
            if (FLIP) {  // global order (i_orig = o, o_orig = c): contiguous k runs per (c, o)
                c = i / (TC * K);
                const int rest = i - c * TC * K;
                o = rest / K;
                k = rest - o * K;
            } else {     // contiguous (c, k) runs per o
                o = i / (CI * K);
                const int rest = i - o * CI * K;
                c = rest / K;
                k = rest - c * K;
            }
            float v = 0.f;
            if (c < cn && o < Cout)
                v = FLIP ? W[((int64_t)(c0 + c) * Cout + o) * K + (K - 1 - k)]
                         : W[((int64_t)o * Cin + c0 + c) * K + k];
            ws[c * WS + k * TC + o] = v;
        }
        __syncthreads();
        const int ng = (cn + 3) >> 2;
        for (int q = 0; q < ng; ++q) {
            const float* xq = xs + (ZPM * 16 * wv + lr) * XS + 4 * q + lc;
            const float* wq = ws + (4 * q + lc) * WS + lr;
#pragma unroll 5
            for (int k = 0; k < K; ++k) {
                float af[ZPM], bf[NT];
#pragma unroll
                for (int m = 0; m < ZPM; ++m) af[m] = xq[(16 * m + k) * XS];
#pragma unroll
                for (int n = 0; n < NT; ++n) bf[n] = wq[k * TC + 16 * n];
#pragma unroll
                for (int m = 0; m < ZPM; ++m)
#pragma unroll
                    for (int n = 0; n < NT; ++n) acc[m][n] = mma(af[m], bf[n], acc[m][n]);
            }
        }
        __syncthreads();
    }
    // D layout: channel = 16 n + lr, position = 4 lc + r
#pragma unroll
    for (int m = 0; m < ZPM; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int t = t0 + ZPM * 16 * wv + 16 * m + 4 * lc + r;
            if (t >= L) continue;
            float* yr = Y + ((int64_t)b * L + t) * ldy;
#pragma unroll
            for (int n = 0; n < NT; ++n) {
                const int o = 16 * n + lr;
                if (o < Cout) yr[o] = accumulate ? yr[o] + acc[m][n][r] : acc[m][n][r];
            }
        }
}

template <int K, bool FLIP>
int zconv_launch_k(const float* X, int ldx, int B, int L, int Cin, const float* W, int Cout, int pad, float* Y,
                   int ldy, int acc, hipStream_t st) {
    dim3 grid(cdiv(L, ZTP), B);
    if (Cout <= 32) {
        hipLaunchKernelGGL((k_zconv_fwd<K, 2, FLIP>), grid, dim3(ZT), (ZCfg<K, 2>::LDS_BYTES), st, X, ldx, L, Cin, W,
                           Cout, pad, Y, ldy, acc);
        return VT_OK;
    }
    if constexpr (K == 1) {  // wide outputs only for the 1x1 convs (residual bottleneck, its bwd-data)
        hipLaunchKernelGGL((k_zconv_fwd<K, 8, FLIP>), grid, dim3(ZT), (ZCfg<K, 8>::LDS_BYTES), st, X, ldx, L, Cin, W,
                           Cout, pad, Y, ldy, acc);
        return VT_OK;
    }
    return VT_ERR_ARG;
}

template <bool FLIP>
int zconv_launch(const float* X, int ldx, int B, int L, int Cin, const float* W, int Cout, int K, int pad, float* Y,
                 int ldy, int acc, hipStream_t st) {
    switch (K) {
        case 1: return zconv_launch_k<1, FLIP>(X, ldx, B, L, Cin, W, Cout, pad, Y, ldy, acc, st);
        case 5: return zconv_launch_k<5, FLIP>(X, ldx, B, L, Cin, W, Cout, pad, Y, ldy, acc, st);
        case 15: return zconv_launch_k<15, FLIP>(X, ldx, B, L, Cin, W, Cout, pad, Y, ldy, acc, st);
        default: return zconv_launch_k<40, FLIP>(X, ldx, B, L, Cin, W, Cout, pad, Y, ldy, acc, st);
    }
}

// Cin / Cout multiples of 16 up to 128; channels > 32 on either side only for 1x1 convs
bool zconv_shape_ok(int B, int L, int Cin, int Cout, int K, int pad) {
    return B > 0 && L > 0 && Cin > 0 && Cin % 16 == 0 && Cin <= 128 && Cout > 0 && Cout % 16 == 0 &&
           Cout <= 128 && (K == 1 || K == 5 || K == 15 || K == 40) && pad >= 0 && pad < K &&
           (K == 1 || (Cin <= 32 && Cout <= 32));
}

// ------------------------------------------------------------- conv weight grad
constexpr int DT = 512;           // 8 waves
constexpr int DRC = 64;           // rows per staged chunk
constexpr int DMAXT = 20;         // tiles per wave (K 40, 32 x 32 channels: 160 tiles / 8 waves)
constexpr int DX_FLOATS = 8448;   // X window LDS budget: (DRC + K - 1) * (Cin + 4)

int zdw_groups(int B) { return B < 256 ? B : 256; }

__global__ __launch_bounds__(DT) void k_zconv_dw(const float* __restrict__ dY, int ldy, const float* __restrict__ X,
                                                 int ldx, int B, int L, int Cin, int Cout, int K, int pad,
                                                 float* __restrict__ part) {
    __shared__ float dys[DRC * (128 + 4)];
    __shared__ float xs[DX_FLOATS];
    const int DS = Cout + 4, XS = Cin + 4;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lr = lane & 15, lc = lane >> 4;
    const int nIt = Cin >> 4, nT = (Cout >> 4) * nIt * K;
    const int tpw = (nT + 7) >> 3;
    const int j0 = wv * tpw;
    int tot[DMAXT], tit[DMAXT], tk[DMAXT];
#pragma unroll
    for (int j = 0; j < DMAXT; ++j) {
        const int jj = j0 + j;
        tk[j] = jj % K;
        const int rest = jj / K;
        tit[j] = rest % nIt;
        tot[j] = rest / nIt;
    }
    f32x4 acc[DMAXT];
#pragma unroll
    for (int j = 0; j < DMAXT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int b = blockIdx.x; b < B; b += gridDim.x) {
        const float* dyb = dY + (int64_t)b * L * ldy;
        const float* xb = X + (int64_t)b * L * ldx;
        for (int t0 = 0; t0 < L; t0 += DRC) {
            __syncthreads();
            for (int i = tid; i < DRC * Cout; i += DT) {
                const int r = i / Cout, o = i - r * Cout;
                dys[r * DS + o] = t0 + r < L ? dyb[(int64_t)(t0 + r) * ldy + o] : 0.f;
            }
            const int win = DRC + K - 1;
            for (int i = tid; i < win * Cin; i += DT) {
                const int r = i / Cin, c = i - r * Cin;
                const int t = t0 + r - pad;
                xs[r * XS + c] = (t >= 0 && t < L) ? xb[(int64_t)t * ldx + c] : 0.f;
            }
            __syncthreads();
            for (int s = 0; s < DRC / 4; ++s) {
                const int row = 4 * s + lc;
#pragma unroll
                for (int j = 0; j < DMAXT; ++j) {
                    if (j < tpw && j0 + j < nT) {
                        const float a = dys[row * DS + 16 * tot[j] + lr];
                        const float bb = xs[(row + tk[j]) * XS + 16 * tit[j] + lr];
                        acc[j] = mma(a, bb, acc[j]);
                    }
                }
            }
        }
    }
    float* slab = part + (int64_t)blockIdx.x * Cout * Cin * K;
#pragma unroll
    for (int j = 0; j < DMAXT; ++j) {
        if (j < tpw && j0 + j < nT) {
            const int i = 16 * tit[j] + lr;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int o = 16 * tot[j] + 4 * lc + r;
                slab[((int64_t)o * Cin + i) * K + tk[j]] = acc[j][r];
            }
        }
    }
}

// ------------------------------------------------------------- elementwise
__global__ void k_maxpool3_fwd(const float* __restrict__ X, int B, int L, int C, float* __restrict__ Y) {
    const int64_t n = (int64_t)B * L * C;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t row = i / C;
        const int t = (int)(row % L);
        float m = t > 0 ? X[i - C] : -INFINITY;
        const float v0 = X[i];
        m = (v0 > m || t == 0) ? v0 : m;
        if (t + 1 < L) {
            const float v1 = X[i + C];
            m = v1 > m ? v1 : m;
        }
        Y[i] = m;
    }
}

// position (-1, 0, +1 relative to t) of the first maximum of the window at t
__device__ __forceinline__ int argmax3(const float* __restrict__ X, int64_t i, int t, int L, int C) {
    int best = 0;
    float m;
    if (t > 0) {
        m = X[i - C];
        best = -1;
        const float v0 = X[i];
        if (v0 > m) { m = v0; best = 0; }
    } else {
        m = X[i];
    }
    if (t + 1 < L && X[i + C] > m) best = 1;
    return best;
}

__global__ void k_maxpool3_bwd(const float* __restrict__ dY, const float* __restrict__ X, int B, int L, int C,
                               float* __restrict__ dX, int accumulate) {
    const int64_t n = (int64_t)B * L * C;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int s = (int)((i / C) % L);
        float g = 0.f;
        // windows centred at s-1, s, s+1 whose first maximum is at s (fixed order)
        if (s > 0 && argmax3(X, i - C, s - 1, L, C) == 1) g += dY[i - C];
        if (argmax3(X, i, s, L, C) == 0) g += dY[i];
        if (s + 1 < L && argmax3(X, i + C, s + 1, L, C) == -1) g += dY[i + C];
        dX[i] = accumulate ? dX[i] + g : g;
    }
}

__global__ void k_add_act(const float* __restrict__ A, const float* __restrict__ Bm, int64_t n, int act,
                          float* __restrict__ Y) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float v = A[i] + Bm[i];
        Y[i] = act == 1 ? fmaxf(v, 0.f) : v;
    }
}

__device__ __forceinline__ uint32_t mix_hash(uint64_t seed, uint64_t idx) {
    uint64_t z = seed + 0x9E3779B97F4A7C15ull * (idx + 1ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (uint32_t)(z >> 32);
}

__device__ __forceinline__ uint32_t drop_threshold(float p) {
    const double t = (double)p * 4294967296.0;
    return t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
}

// Device-side seed offset (the seed_offset argument of the dropout / attention calls): added to every dropout seed, advanced
// once per training step on the device (vt_dropout_seed_advance), so a captured step replayed
// by the native executor draws new masks each replay (its host seeds are frozen at capture).
__device__ __forceinline__ uint64_t eff_seed(uint64_t seed, const uint64_t* __restrict__ soff) {
    return soff ? seed + soff[0] : seed;
}

__global__ void k_seed_advance(uint64_t* off) {
    if (threadIdx.x == 0) off[0] += 0xD1B54A32D192ED03ull;
}

__global__ void k_dropout(const float* __restrict__ X, int64_t n, int C, int L, float p, uint64_t seed,
                          const uint64_t* __restrict__ soff, float* __restrict__ Y) {
    seed = eff_seed(seed, soff);
    const uint32_t th = drop_threshold(p);
    const float sc = 1.f / (1.f - p);
    const int64_t LC = (int64_t)L * C;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t m = L > 0 ? (uint64_t)((i / LC) * C + i % C) : (uint64_t)i;
        Y[i] = mix_hash(seed, m) >= th ? X[i] * sc : 0.f;
    }
}

__global__ __launch_bounds__(256) void k_time_mean(const float* __restrict__ X, int L, int C, float* __restrict__ Y) {
    const int b = blockIdx.x;
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        const float* xb = X + (int64_t)b * L * C + c;
        float s = 0.f;
        for (int t = 0; t < L; ++t) s += xb[(int64_t)t * C];
        Y[(int64_t)b * C + c] = s / (float)L;
    }
}

__global__ void k_time_mean_bwd(const float* __restrict__ dY, int B, int L, int C, float* __restrict__ dX,
                                int accumulate) {
    const int64_t n = (int64_t)B * L * C;
    const float inv = 1.f / (float)L;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = i / ((int64_t)L * C);
        const float g = dY[b * C + i % C] * inv;
        dX[i] = accumulate ? dX[i] + g : g;
    }
}

__global__ __launch_bounds__(256) void k_ce_fwd(const float* __restrict__ logits, const int64_t* __restrict__ labels,
                                                int B, int C, float* __restrict__ loss, float* __restrict__ probs) {
    __shared__ float red[16];
    float s = 0.f;
    for (int b = threadIdx.x; b < B; b += blockDim.x) {
        const float* l = logits + (int64_t)b * C;
        float m = l[0];
        for (int c = 1; c < C; ++c) m = fmaxf(m, l[c]);
        float z = 0.f;
        for (int c = 0; c < C; ++c) z += expf(l[c] - m);
        const float lz = m + logf(z);
        for (int c = 0; c < C; ++c) probs[(int64_t)b * C + c] = expf(l[c] - lz);
        const int64_t y = labels[b];
        s += (y >= 0 && y < C) ? lz - l[y] : NAN;
    }
    s = block_sum(s, red);
    if (threadIdx.x == 0) loss[0] = s / (float)B;
}

__global__ void k_ce_bwd(const float* __restrict__ probs, const int64_t* __restrict__ labels, int B, int C,
                         const float* __restrict__ g, float* __restrict__ dl) {
    const int64_t n = (int64_t)B * C;
    const float sc = g[0] / (float)B;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = i / C, c = i % C;
        dl[i] = sc * (probs[i] - (labels[b] == c ? 1.f : 0.f));
    }
}

int ew_blocks(int64_t n) {
    const int64_t b = (n + 255) / 256;
    return (int)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

// --------------------------------------------------------------- attention
constexpr int DH = 32;            // head dim (embed 128 / 4 heads)
constexpr int AKS = DH + 1;       // LDS row stride of K / V
constexpr int AMAXKT = 16;        // S <= 256

__global__ __launch_bounds__(256) void k_attn_fwd(const float* __restrict__ qkv, int S, int H, float scale, float p,
                                                  uint64_t seed, const uint64_t* __restrict__ soff,
                                                  float* __restrict__ out, float* __restrict__ lse) {
    seed = eff_seed(seed, soff);
    __shared__ float Ks[256 * AKS];
    __shared__ float Vs[256 * AKS];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lr = lane & 15, lc = lane >> 4;
    const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
    const int E = H * DH, E3 = 3 * E;
    const float* base = qkv + (int64_t)b * S * E3 + h * DH;
    for (int i = tid; i < S * DH; i += 256) {
        const int r = i / DH, d = i - r * DH;
        Ks[r * AKS + d] = base[(int64_t)r * E3 + E + d];
        Vs[r * AKS + d] = base[(int64_t)r * E3 + 2 * E + d];
    }
    __syncthreads();
    const int q0 = blockIdx.x * 64 + 16 * wv;
    if (q0 >= S) return;
    const int nkt = S >> 4;
    // B operand Q^T[dim = 4 s + lc][query = lr]
    float qf[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) qf[s] = base[(int64_t)(q0 + lr) * E3 + 4 * s + lc];
    f32x4 st[AMAXKT];
#pragma unroll
    for (int kt = 0; kt < AMAXKT; ++kt) {
        st[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (kt < nkt) {
#pragma unroll
            for (int s = 0; s < 8; ++s) st[kt] = mma(Ks[(16 * kt + lr) * AKS + 4 * s + lc], qf[s], st[kt]);
        }
    }
    // column softmax: S^T[key = 16 kt + 4 lc + r][query = lr]
    float m = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < AMAXKT; ++kt)
        if (kt < nkt)
#pragma unroll
            for (int r = 0; r < 4; ++r) m = fmaxf(m, st[kt][r] * scale);
    m = fmaxf(m, __shfl_xor(m, 16));
    m = fmaxf(m, __shfl_xor(m, 32));
    float l = 0.f;
#pragma unroll
    for (int kt = 0; kt < AMAXKT; ++kt)
        if (kt < nkt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float e = expf(st[kt][r] * scale - m);
                st[kt][r] = e;
                l += e;
            }
    l += __shfl_xor(l, 16);
    l += __shfl_xor(l, 32);
    const float inv = 1.f / l;
    const int q = q0 + lr;
    if (lc == 0) lse[(int64_t)bh * S + q] = m + logf(l);
    const uint32_t th = drop_threshold(p);
    const float dsc = p > 0.f ? 1.f / (1.f - p) : 1.f;
#pragma unroll
    for (int kt = 0; kt < AMAXKT; ++kt)
        if (kt < nkt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float pv = st[kt][r] * inv;
                if (p > 0.f) {
                    const uint64_t id = ((uint64_t)bh * S + q) * S + 16 * kt + 4 * lc + r;
                    pv = mix_hash(seed, id) >= th ? pv * dsc : 0.f;
                }
                st[kt][r] = pv;
            }
    // O^T[dim][query] = sum_key V^T[dim][key] P^T[key][query]; step (kt, j) covers keys 16 kt + 4 g + j
    float* ob = out + ((int64_t)b * S + q) * E + h * DH;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
        f32x4 o = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kt = 0; kt < AMAXKT; ++kt)
            if (kt < nkt)
#pragma unroll
                for (int j = 0; j < 4; ++j) o = mma(Vs[(16 * kt + 4 * lc + j) * AKS + 16 * dt + lr], st[kt][j], o);
        // D: O^T[dim = 16 dt + 4 lc + r][query = lr]
#pragma unroll
        for (int r = 0; r < 4; ++r) ob[16 * dt + 4 * lc + r] = o[r];
    }
}

__global__ __launch_bounds__(256) void k_attn_bwd(const float* __restrict__ qkv, const float* __restrict__ O,
                                                  const float* __restrict__ dO, const float* __restrict__ lse, int S,
                                                  int H, float scale, float p, uint64_t seed,
                                                  const uint64_t* __restrict__ soff, float* __restrict__ dqkv) {
    seed = eff_seed(seed, soff);
    __shared__ float Ks[256 * AKS];
    __shared__ float Qs[16 * AKS], dOs[16 * AKS];
    __shared__ float dSs[4][16 * 17];
    __shared__ float dqp[4][16 * DH];
    __shared__ float lses[16], Dq[16];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lr = lane & 15, lc = lane >> 4;
    const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
    const int E = H * DH, E3 = 3 * E;
    const float* base = qkv + (int64_t)b * S * E3 + h * DH;
    const int nkt = S >> 4;
    for (int i = tid; i < S * DH; i += 256) {
        const int r = i / DH, d = i - r * DH;
        Ks[r * AKS + d] = base[(int64_t)r * E3 + E + d];
    }
    // this wave's key tiles: kt = wv + 4 u
    float vf[4][8];
    f32x4 dv[4][2], dk[4][2];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int kt = wv + 4 * u;
#pragma unroll
        for (int s = 0; s < 8; ++s)
            vf[u][s] = kt < nkt ? base[(int64_t)(16 * kt + lr) * E3 + 2 * E + 4 * s + lc] : 0.f;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) dv[u][dt] = dk[u][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const uint32_t th = drop_threshold(p);
    const float dsc = p > 0.f ? 1.f / (1.f - p) : 1.f;
    for (int qt = 0; qt < nkt; ++qt) {
        const int q0 = 16 * qt;
        __syncthreads();
        for (int i = tid; i < 16 * DH; i += 256) {
            const int r = i / DH, d = i - r * DH;
            const int64_t row = (int64_t)b * S + q0 + r;
            Qs[r * AKS + d] = base[(int64_t)(q0 + r) * E3 + d];
            dOs[r * AKS + d] = dO[row * E + h * DH + d];
        }
        if (tid < 16) {
            const int64_t row = (int64_t)b * S + q0 + tid;
            const float* orow = O + row * E + h * DH;
            const float* drow = dO + row * E + h * DH;
            float s = 0.f;
            for (int d = 0; d < DH; ++d) s += drow[d] * orow[d];
            Dq[tid] = s;
            lses[tid] = lse[(int64_t)bh * S + q0 + tid];
        }
        __syncthreads();
        f32x4 dq[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int kt = wv + 4 * u;
            if (kt >= nkt) break;
            // S[q = 4 lc + r][key = lr] = Q K^T ; dP = dO V^T (same layout)
            f32x4 sc = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                sc = mma(Qs[lr * AKS + 4 * s + lc], Ks[(16 * kt + lr) * AKS + 4 * s + lc], sc);
                dp = mma(dOs[lr * AKS + 4 * s + lc], vf[u][s], dp);
            }
            float pd[4], ds[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int ql = 4 * lc + r;
                const float pr = expf(sc[r] * scale - lses[ql]);
                float keep = 1.f;
                if (p > 0.f) {
                    const uint64_t id = ((uint64_t)bh * S + q0 + ql) * S + 16 * kt + lr;
                    keep = mix_hash(seed, id) >= th ? dsc : 0.f;
                }
                pd[r] = pr * keep;                       // dropped probabilities (used by O)
                ds[r] = pr * (dp[r] * keep - Dq[ql]);    // dS = P (dP - D)
            }
            // dV^T[dim][key] += dO^T[dim][q] Pd[q][key];  dK^T[dim][key] += Q^T[dim][q] dS[q][key]
#pragma unroll
            for (int dt = 0; dt < 2; ++dt)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    dv[u][dt] = mma(dOs[(4 * lc + j) * AKS + 16 * dt + lr], pd[j], dv[u][dt]);
                    dk[u][dt] = mma(Qs[(4 * lc + j) * AKS + 16 * dt + lr], ds[j], dk[u][dt]);
                }
            // dQ[q][dim] += dS[q][key] K[key][dim]: dS to A layout through LDS
            float* dsw = dSs[wv];
#pragma unroll
            for (int r = 0; r < 4; ++r) dsw[(4 * lc + r) * 17 + lr] = ds[r];
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): wave-local LDS exchange
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int dt = 0; dt < 2; ++dt)
#pragma unroll
                for (int s = 0; s < 4; ++s)
                    dq[dt] = mma(dsw[lr * 17 + 4 * s + lc], Ks[(16 * kt + 4 * s + lc) * AKS + 16 * dt + lr], dq[dt]);
            __builtin_amdgcn_wave_barrier();
        }
        // fixed-order sum of the 4 waves' dQ partials: D layout [q = 4 lc + r][dim = 16 dt + lr]
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int r = 0; r < 4; ++r) dqp[wv][(4 * lc + r) * DH + 16 * dt + lr] = dq[dt][r];
        __syncthreads();
        for (int i = tid; i < 16 * DH; i += 256) {
            const int r = i / DH, d = i - r * DH;
            const float s = ((dqp[0][i] + dqp[1][i]) + dqp[2][i]) + dqp[3][i];
            dqkv[((int64_t)b * S + q0 + r) * E3 + h * DH + d] = s * scale;
        }
    }
    // dK^T / dV^T D layout: [dim = 16 dt + 4 lc + r][key = 16 kt + lr]
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int kt = wv + 4 * u;
        if (kt >= nkt) break;
        float* row = dqkv + ((int64_t)b * S + 16 * kt + lr) * E3 + h * DH;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                row[E + 16 * dt + 4 * lc + r] = dk[u][dt][r] * scale;
                row[2 * E + 16 * dt + 4 * lc + r] = dv[u][dt][r];
            }
    }
}

}  // namespace

}  // namespace vt

using namespace vt;

extern "C" {

int vt_zconv_fwd(const float* X, int ldx, int B, int L, int Cin, const float* W, int Cout, int K, int pad_left,
                 float* Y, int ldy, int accumulate, void* stream) {
    VT_CHECK_ARG(zconv_shape_ok(B, L, Cin, Cout, K, pad_left) && ldx >= Cin && ldy >= Cout,
                 "vt_zconv_fwd: shape (Cin/Cout multiples of 16 <= 128, K in {1,5,15,40}, 0 <= pad < K)");
    VT_CHECK_ARG(zconv_launch<false>(X, ldx, B, L, Cin, W, Cout, K, pad_left, Y, ldy, accumulate, S(stream)) == VT_OK,
                 "vt_zconv_fwd: unsupported configuration");
    VT_LAUNCH_CHECK("vt_zconv_fwd");
    return VT_OK;
}

int vt_zconv_bwd_data(const float* dY, int ldy, int B, int L, int Cin, const float* W, int Cout, int K, int pad_left,
                      float* dX, int ldx, int accumulate, void* stream) {
    VT_CHECK_ARG(zconv_shape_ok(B, L, Cin, Cout, K, pad_left) && ldx >= Cin && ldy >= Cout,
                 "vt_zconv_bwd_data: shape");
    // conv of dY (Cout channels) with taps W[o][i][K-1-k] into Cin channels, pad K-1-pad_left
    VT_CHECK_ARG(zconv_launch<true>(dY, ldy, B, L, Cout, W, Cin, K, K - 1 - pad_left, dX, ldx, accumulate,
                                    S(stream)) == VT_OK,
                 "vt_zconv_bwd_data: unsupported configuration");
    VT_LAUNCH_CHECK("vt_zconv_bwd_data");
    return VT_OK;
}

int vt_zconv_bwd_weight_ws_floats(int B, int Cin, int Cout, int K, int64_t* floats) {
    VT_CHECK_ARG(B > 0 && floats, "vt_zconv_bwd_weight_ws_floats: args");
    *floats = (int64_t)zdw_groups(B) * Cout * Cin * K;
    return VT_OK;
}

int vt_zconv_bwd_weight(const float* dY, int ldy, const float* X, int ldx, int B, int L, int Cin, int Cout, int K,
                        int pad_left, float* dW, int accumulate, float* ws, int64_t ws_floats, void* stream) {
    VT_CHECK_ARG(zconv_shape_ok(B, L, Cin, Cout, K, pad_left) && ldx >= Cin && ldy >= Cout,
                 "vt_zconv_bwd_weight: shape");
    VT_CHECK_ARG(((Cout / 16) * (Cin / 16) * K + 7) / 8 <= DMAXT && (DRC + K - 1) * (Cin + 4) <= DX_FLOATS,
                 "vt_zconv_bwd_weight: too many (channel, tap) tiles");
    const int G = zdw_groups(B);
    const int64_t n = (int64_t)Cout * Cin * K;
    VT_CHECK_ARG(ws_floats >= G * n, "vt_zconv_bwd_weight: workspace too small");
    hipStream_t st = S(stream);
    hipLaunchKernelGGL(k_zconv_dw, dim3(G), dim3(DT), 0, st, dY, ldy, X, ldx, B, L, Cin, Cout, K, pad_left, ws);
    sum_splits_launch(ws, G, n, dW, accumulate, st);
    VT_LAUNCH_CHECK("vt_zconv_bwd_weight");
    return VT_OK;
}

int vt_maxpool3_fwd(const float* X, int B, int L, int C, float* Y, void* stream) {
    VT_CHECK_ARG(B > 0 && L > 0 && C > 0, "vt_maxpool3_fwd: shape");
    const int64_t n = (int64_t)B * L * C;
    hipLaunchKernelGGL(k_maxpool3_fwd, dim3(ew_blocks(n)), dim3(256), 0, S(stream), X, B, L, C, Y);
    VT_LAUNCH_CHECK("vt_maxpool3_fwd");
    return VT_OK;
}

int vt_maxpool3_bwd(const float* dY, const float* X, int B, int L, int C, float* dX, int accumulate, void* stream) {
    VT_CHECK_ARG(B > 0 && L > 0 && C > 0, "vt_maxpool3_bwd: shape");
    const int64_t n = (int64_t)B * L * C;
    hipLaunchKernelGGL(k_maxpool3_bwd, dim3(ew_blocks(n)), dim3(256), 0, S(stream), dY, X, B, L, C, dX, accumulate);
    VT_LAUNCH_CHECK("vt_maxpool3_bwd");
    return VT_OK;
}

int vt_add_act_fwd(const float* A, const float* Bm, int64_t n, int act, float* Y, void* stream) {
    VT_CHECK_ARG(n > 0 && (act == 0 || act == 1), "vt_add_act_fwd: n > 0, act none/relu");
    hipLaunchKernelGGL(k_add_act, dim3(ew_blocks(n)), dim3(256), 0, S(stream), A, Bm, n, act, Y);
    VT_LAUNCH_CHECK("vt_add_act_fwd");
    return VT_OK;
}

// the seed offset is read only when something is dropped (p > 0): a caller without one, or an
// eval / p = 0 call, passes nothing the kernels would dereference
static inline const uint64_t* seed_off(const void* off, float p) {
    return p > 0.f ? reinterpret_cast<const uint64_t*>(off) : nullptr;
}

int vt_dropout_seed_advance(void* offset, void* stream) {
    VT_CHECK_ARG(offset != nullptr, "vt_dropout_seed_advance: null offset");
    hipLaunchKernelGGL(k_seed_advance, dim3(1), dim3(64), 0, S(stream), reinterpret_cast<uint64_t*>(offset));
    VT_LAUNCH_CHECK("vt_dropout_seed_advance");
    return VT_OK;
}

int vt_dropout_apply(const float* X, int64_t n, int C, int L, float p, int64_t seed, const void* seed_offset, float* Y,
                     void* stream) {
    VT_CHECK_ARG(n > 0 && C > 0 && L >= 0 && p >= 0.f && p < 1.f, "vt_dropout_apply: args (0 <= p < 1)");
    hipLaunchKernelGGL(k_dropout, dim3(ew_blocks(n)), dim3(256), 0, S(stream), X, n, C, L, p, (uint64_t)seed,
                       seed_off(seed_offset, p), Y);
    VT_LAUNCH_CHECK("vt_dropout_apply");
    return VT_OK;
}

int vt_time_mean_fwd(const float* X, int B, int L, int C, float* Y, void* stream) {
    VT_CHECK_ARG(B > 0 && L > 0 && C > 0, "vt_time_mean_fwd: shape");
    hipLaunchKernelGGL(k_time_mean, dim3(B), dim3(C < 256 ? C : 256), 0, S(stream), X, L, C, Y);
    VT_LAUNCH_CHECK("vt_time_mean_fwd");
    return VT_OK;
}

int vt_time_mean_bwd(const float* dY, int B, int L, int C, float* dX, int accumulate, void* stream) {
    VT_CHECK_ARG(B > 0 && L > 0 && C > 0, "vt_time_mean_bwd: shape");
    const int64_t n = (int64_t)B * L * C;
    hipLaunchKernelGGL(k_time_mean_bwd, dim3(ew_blocks(n)), dim3(256), 0, S(stream), dY, B, L, C, dX, accumulate);
    VT_LAUNCH_CHECK("vt_time_mean_bwd");
    return VT_OK;
}

int vt_attn_fwd(const float* qkv, int B, int S_, int H, float scale, float p, int64_t seed, const void* seed_offset,
                float* out, float* lse, void* stream) {
    VT_CHECK_ARG(B > 0 && H > 0 && S_ > 0 && S_ % 16 == 0 && S_ <= 256 && p >= 0.f && p < 1.f,
                 "vt_attn_fwd: S multiple of 16 <= 256, 0 <= p < 1");
    hipLaunchKernelGGL(k_attn_fwd, dim3(cdiv(S_, 64), B * H), dim3(256), 0, S(stream), qkv, S_, H, scale, p,
                       (uint64_t)seed, seed_off(seed_offset, p), out, lse);
    VT_LAUNCH_CHECK("vt_attn_fwd");
    return VT_OK;
}

int vt_attn_bwd(const float* qkv, const float* out, const float* dout, const float* lse, int B, int S_, int H,
                float scale, float p, int64_t seed, const void* seed_offset, float* dqkv, void* stream) {
    VT_CHECK_ARG(B > 0 && H > 0 && S_ > 0 && S_ % 16 == 0 && S_ <= 256 && p >= 0.f && p < 1.f,
                 "vt_attn_bwd: S multiple of 16 <= 256, 0 <= p < 1");
    hipLaunchKernelGGL(k_attn_bwd, dim3(B * H), dim3(256), 0, S(stream), qkv, out, dout, lse, S_, H, scale, p,
                       (uint64_t)seed, seed_off(seed_offset, p), dqkv);
    VT_LAUNCH_CHECK("vt_attn_bwd");
    return VT_OK;
}

int vt_cross_entropy_fwd(const float* logits, const int64_t* labels, int B, int C, float* loss, float* probs,
                         void* stream) {
    VT_CHECK_ARG(B > 0 && C > 0, "vt_cross_entropy_fwd: shape");
    hipLaunchKernelGGL(k_ce_fwd, dim3(1), dim3(256), 0, S(stream), logits, labels, B, C, loss, probs);
    VT_LAUNCH_CHECK("vt_cross_entropy_fwd");
    return VT_OK;
}

int vt_cross_entropy_bwd(const float* probs, const int64_t* labels, int B, int C, const float* g, float* dlogits,
                         void* stream) {
    VT_CHECK_ARG(B > 0 && C > 0, "vt_cross_entropy_bwd: shape");
    const int64_t n = (int64_t)B * C;
    hipLaunchKernelGGL(k_ce_bwd, dim3(ew_blocks(n)), dim3(256), 0, S(stream), probs, labels, B, C, g, dlogits);
    VT_LAUNCH_CHECK("vt_cross_entropy_bwd");
    return VT_OK;
}

}  // extern "C"
