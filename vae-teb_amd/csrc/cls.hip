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
//  k_attn_fwd    softmax(Q K^T) V per (sample, head), 8 waves over the 16-query
//                tiles: K / V of the head staged in LDS once, S^T = K Q^T in registers (so the column softmax
//                is lane-local plus two shuffles and P^T is already the B
//                operand of O^T = V^T P^T: no LDS round trip for P).
//  k_attn_bwd    one workgroup per (sample, head), a wave per 64 keys, query
//                tiles of 16: P recomputed from the saved log-sum-exp, dV / dK
//                accumulated in registers, dQ through a fixed-order LDS sum.
// Everything is deterministic (no atomics).
#include <math.h>

#include "common.h"
#include "conv.h"
#include "dropout.h"

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

// ------------------------------------------------------- zero-pad conv, bf16 MFMA
// The same implicit GEMM on v_mfma_f32_16x16x32_bf16 (round 5; the
// reference trains the classifier in 16-bit autocast as well, ref/model/graph_model.py:510):
// operands rounded to bf16 while they are staged, fp32 accumulation.  Per chunk of 32 input
// channels the zero-padded window is staged as bf16 rows of 32 channels (RS16-element stride:
// 16 consecutive rows hit distinct 4-bank groups) and the taps as [tap][out][32 in] rows, in
// groups of KG taps (the 40-tap conv: 4 groups, 39 KB of LDS instead of 115); one MFMA k-step
// per (tap, position tile, output tile) contracts the chunk's 32 channels (16-channel inputs
// padded with zeros), lane group lc taking channels 8 lc .. 8 lc + 7 — so a fragment is one
// 16-byte LDS read of a window row shifted by the tap, or of a tap row.
constexpr int RS16 = 40;

template <int K, int NT>
struct Z16Cfg {
    static constexpr int TC = 16 * NT;
    static constexpr int WIN = ZTP + K - 1;
    static constexpr int KG = K <= 15 ? K : 10;
    static constexpr int XB = WIN * RS16, WB = KG * TC * RS16;   // bf16 elements
    static constexpr int LDS_BYTES = (XB + WB) * 2;
};

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// the bf16 tap image of one call: T[k][o][c] = W[o][c][k] (FLIP: W[c][o][K-1-k], the
// backward-data taps of a weight stored [Cin][Cout][K] in kernel terms), o < TC, c < cin32,
// zero padded — written once per call instead of every workgroup gathering fp32 taps
__global__ void k_zconv16_taps(const float* __restrict__ W, int Cin, int Cout, int K, int TC, int cin32, int flip,
                               __bf16* __restrict__ T) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (int64_t)K * TC * cin32) return;
    const int c = (int)(e % cin32), ko = (int)(e / cin32), o = ko % TC, k = ko / TC;
    float v = 0.f;
    if (o < Cout && c < Cin)
        v = flip ? W[((int64_t)c * Cout + o) * K + (K - 1 - k)] : W[((int64_t)o * Cin + c) * K + k];
    T[e] = (__bf16)v;
}

// the tap images of up to ZTB_MAX weights in one launch (an inception block's five convolutions)
constexpr int ZTB_MAX = 8;
struct ZTapBatch {
    int n, flip;
    const float* W[ZTB_MAX];
    __bf16* T[ZTB_MAX];
    int Cin[ZTB_MAX], Cout[ZTB_MAX], K[ZTB_MAX], TC[ZTB_MAX], cin32[ZTB_MAX];
    int prefix[ZTB_MAX + 1];   // workgroups before weight h
};
__global__ void k_zconv16_taps_batch(ZTapBatch tb) {
    int h = 0;
    while (h + 1 < tb.n && (int)blockIdx.x >= tb.prefix[h + 1]) ++h;
    const int64_t e = (int64_t)(blockIdx.x - tb.prefix[h]) * blockDim.x + threadIdx.x;
    const int K = tb.K[h], TC = tb.TC[h], cin32 = tb.cin32[h], Cin = tb.Cin[h], Cout = tb.Cout[h];
    if (e >= (int64_t)K * TC * cin32) return;
    const int c = (int)(e % cin32), ko = (int)(e / cin32), o = ko % TC, k = ko / TC;
    const float* W = tb.W[h];
    float v = 0.f;
    if (o < Cout && c < Cin)
        v = tb.flip ? W[((int64_t)c * Cout + o) * K + (K - 1 - k)] : W[((int64_t)o * Cin + c) * K + k];
    tb.T[h][e] = (__bf16)v;
}

template <int K, int NT, bool FLIP>
__global__ __launch_bounds__(ZT) void k_zconv16_fwd(const float* __restrict__ X, int ldx, int L, int Cin,
                                                    const __bf16* __restrict__ T, int Cout, int pad,
                                                    float* __restrict__ Y, int ldy, int accumulate) {
    using C = Z16Cfg<K, NT>;
    constexpr int TC = C::TC, WIN = C::WIN, KG = C::KG;
    const int cin32 = (Cin + 31) & ~31;
    extern __shared__ __attribute__((aligned(16))) __bf16 lb16[];
    __bf16* xs = lb16;            // [WIN][RS16]
    __bf16* ws = lb16 + C::XB;    // [KG][TC][RS16]
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lr = lane & 15, lc = lane >> 4;
    const int t0 = blockIdx.x * ZTP, b = blockIdx.y;
    const float* xb = X + (int64_t)b * L * ldx;
    f32x4 acc[ZPM][NT];
#pragma unroll
    for (int m = 0; m < ZPM; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int c0 = 0; c0 < Cin; c0 += 32) {
        const int cn = Cin - c0 < 32 ? Cin - c0 : 32;
        __syncthreads();   // the previous chunk's MFMAs are done with xs
        // window: WIN rows x 4 octets of 8 channels (zero outside [0, L) and past cn)
        for (int i = tid; i < WIN * 4; i += ZT) {
            const int r = i >> 2, oct = i & 3;
            const int t = t0 + r - pad;
            const bool ok = t >= 0 && t < L && 8 * oct < cn;
            float v[8];
            if (ok) {
                const float4 a = *reinterpret_cast<const float4*>(xb + (int64_t)t * ldx + c0 + 8 * oct);
                const float4 q = *reinterpret_cast<const float4*>(xb + (int64_t)t * ldx + c0 + 8 * oct + 4);
                v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = q.x; v[5] = q.y; v[6] = q.z; v[7] = q.w;
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = 0.f;
            }
            bf16x8 h;
#pragma unroll
            for (int j = 0; j < 8; ++j) h[j] = (__bf16)v[j];
            *reinterpret_cast<bf16x8*>(xs + r * RS16 + 8 * oct) = h;
        }
        for (int kg0 = 0; kg0 < K; kg0 += KG) {
            if (kg0) __syncthreads();   // the previous tap group's MFMAs are done with ws
            // taps kg0 .. kg0 + KG - 1: rows (tap, out) x 4 octets of 8 input channels, 16-byte
            // copies from the call's bf16 tap image (k_zconv16_taps: [K][TC][cin32], zero padded)
            for (int i = tid; i < KG * TC * 4; i += ZT) {
                const int oct = i & 3, r = i >> 2, kk = r / TC, o = r - kk * TC;
                const int k = kg0 + kk;
                bf16x8 h;
                if (k < K) {
                    h = *reinterpret_cast<const bf16x8*>(T + ((int64_t)k * TC + o) * cin32 + c0 + 8 * oct);
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) h[j] = (__bf16)0.f;
                }
                *reinterpret_cast<bf16x8*>(ws + (kk * TC + o) * RS16 + 8 * oct) = h;
            }
            __syncthreads();
            const __bf16* xq = xs + (ZPM * 16 * wv + lr + kg0) * RS16 + 8 * lc;
            const __bf16* wq = ws + lr * RS16 + 8 * lc;
            const int kn = K - kg0 < KG ? K - kg0 : KG;
#pragma unroll 2
            for (int kk = 0; kk < kn; ++kk) {
                bf16x8 af[ZPM], bfr[NT];
#pragma unroll
                for (int m = 0; m < ZPM; ++m) af[m] = *reinterpret_cast<const bf16x8*>(xq + (16 * m + kk) * RS16);
#pragma unroll
                for (int n = 0; n < NT; ++n) bfr[n] = *reinterpret_cast<const bf16x8*>(wq + (kk * TC + 16 * n) * RS16);
#pragma unroll
                for (int m = 0; m < ZPM; ++m)
#pragma unroll
                    for (int n = 0; n < NT; ++n)
                        acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr[n], acc[m][n], 0, 0, 0);
            }
        }
    }
    // D layout: channel = 16 n + lr, position = 4 lc + r (as k_zconv_fwd)
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

// bf16 elements of the tap image of a call (the workspace of vt_zconv16_fwd / _bwd_data)
int64_t zconv16_taps_elems(int Cin, int Cout, int K) {
    const int TC = Cout <= 32 ? 32 : 128;
    return (int64_t)K * TC * ((Cin + 31) & ~31);
}

// W == nullptr: T already holds the call's tap image (vt_zconv16_taps)
template <int K, bool FLIP>
int zconv16_launch_k(const float* X, int ldx, int B, int L, int Cin, const float* W, int Cout, int pad, float* Y,
                     int ldy, int acc, __bf16* T, hipStream_t st) {
    if ((ldx & 3) || (reinterpret_cast<uintptr_t>(X) & 15)) return VT_ERR_ARG;   // float4 row segments
    dim3 grid(cdiv(L, ZTP), B);
    const int cin32 = (Cin + 31) & ~31;
    auto taps = [&](int TC) {
        if (!W) return;
        const int64_t n = (int64_t)K * TC * cin32;
        // FLIP: the kernel's (Cin, Cout) are the weight's (Cout, Cin)
        hipLaunchKernelGGL(k_zconv16_taps, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, W, Cin, Cout, K, TC,
                           cin32, FLIP ? 1 : 0, T);
    };
    if (Cout <= 32) {
        taps(32);
        hipLaunchKernelGGL((k_zconv16_fwd<K, 2, FLIP>), grid, dim3(ZT), (Z16Cfg<K, 2>::LDS_BYTES), st, X, ldx, L, Cin,
                           T, Cout, pad, Y, ldy, acc);
        return VT_OK;
    }
    if constexpr (K == 1) {
        taps(128);
        hipLaunchKernelGGL((k_zconv16_fwd<K, 8, FLIP>), grid, dim3(ZT), (Z16Cfg<K, 8>::LDS_BYTES), st, X, ldx, L, Cin,
                           T, Cout, pad, Y, ldy, acc);
        return VT_OK;
    }
    return VT_ERR_ARG;
}

template <bool FLIP>
int zconv16_launch(const float* X, int ldx, int B, int L, int Cin, const float* W, int Cout, int K, int pad, float* Y,
                   int ldy, int acc, __bf16* T, hipStream_t st) {
    switch (K) {
        case 1: return zconv16_launch_k<1, FLIP>(X, ldx, B, L, Cin, W, Cout, pad, Y, ldy, acc, T, st);
        case 5: return zconv16_launch_k<5, FLIP>(X, ldx, B, L, Cin, W, Cout, pad, Y, ldy, acc, T, st);
        case 15: return zconv16_launch_k<15, FLIP>(X, ldx, B, L, Cin, W, Cout, pad, Y, ldy, acc, T, st);
        default: return zconv16_launch_k<40, FLIP>(X, ldx, B, L, Cin, W, Cout, pad, Y, ldy, acc, T, st);
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

// ------------------------------------------------------ conv weight grad, bf16 MFMA
// dW[o][i][k] = sum_rows dY[row][o] X[row + k - pad][i] on v_mfma_f32_16x16x32_bf16 (round 5):
// the 64-row chunk of dY and its input window are staged as bf16 row images (rows the
// contraction), both operands read with the gfx950 transposed LDS read (ds_read_b64_tr_b16:
// 8 rows x 16 channels per lane group), so one MFMA contracts 32 rows of one (16 o x 16 i x
// tap) tile — the fp32 kernel above needs 8 MFMAs and 16 scalar LDS reads for the same rows.
// Tiles (o, i, tap) with the tap fastest, D16W waves x <= D16MAXT tiles; per-workgroup slabs
// summed in fixed order (k_sum_splits).  16 waves of <= 10 tiles (round 5; was 8 x 20 at 256
// VGPRs + spills, one wave per SIMD pair-issuing): the same tiles and per-tile accumulation order.
typedef short zv4i16 __attribute__((ext_vector_type(4)));
constexpr int D16W = 16, D16T = 64 * D16W, D16R = 128, D16MAXT = 10;   // 128-row chunks: half the staging round trips of 64
constexpr int D16_DS = 136 * D16R;                  // dY image: 128 rows x (<= 128 + 8) channels
constexpr int D16_XS = (D16R + 40 + 8) * 40;        // window image, K <= 40 at <= 32 channels ...
constexpr int D16_XS1 = D16R * 136;                 // ... or K 1 at <= 128 channels

__device__ __forceinline__ bf16x8 ztr_frag(const __bf16* img, int row0, int col0, int stride) {
    // lane 4q + p of each 16-lane group: row row0 + 8 g + q (+ 4), columns col0 + 4p .. +3
    const int lane = threadIdx.x & 63, g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const __bf16* a0 = img + (row0 + 8 * g + q) * stride + col0 + 4 * p;
    const zv4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) zv4i16*)a0);
    const zv4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) zv4i16*)(a0 + 4 * stride));
    typedef short v8i16 __attribute__((ext_vector_type(8)));
    const v8i16 r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, r);
}

__global__ __launch_bounds__(D16T) void k_zconv16_dw(const float* __restrict__ dY, int ldy, const float* __restrict__ X,
                                                     int ldx, int B, int L, int Cin, int Cout, int K, int pad,
                                                     float* __restrict__ part) {
    __shared__ __attribute__((aligned(16))) __bf16 dys[D16_DS];
    __shared__ __attribute__((aligned(16))) __bf16 xs[D16_XS > D16_XS1 ? D16_XS : D16_XS1];
    const int DS = Cout + 8, XS = Cin + 8;   // Cin / Cout multiples of 16: rows 16 B apart mod 64 banks
    const int tid = threadIdx.x, lane = tid & 63, lr = lane & 15, lc = lane >> 4;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: the tile indices in SGPRs
    const int nIt = Cin >> 4, nT = (Cout >> 4) * nIt * K;
    const int tpw = (nT + D16W - 1) / D16W;
    const int j0 = wv * tpw;
    int tot[D16MAXT], tit[D16MAXT], tk[D16MAXT];
#pragma unroll
    for (int j = 0; j < D16MAXT; ++j) {
        const int jj = j0 + j;
        tk[j] = jj % K;
        const int rest = jj / K;
        tit[j] = rest % nIt;
        tot[j] = rest / nIt;
    }
    f32x4 acc[D16MAXT];
#pragma unroll
    for (int j = 0; j < D16MAXT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int win = D16R + K - 1;
    for (int b = blockIdx.x; b < B; b += gridDim.x) {
        const float* dyb = dY + (int64_t)b * L * ldy;
        const float* xb = X + (int64_t)b * L * ldx;
        for (int t0 = 0; t0 < L; t0 += D16R) {
            __syncthreads();   // the previous chunk's MFMAs are done with both images
            // dY rows t0 .. t0 + 63 (zero past L), 8 channels per item
            const int og = Cout >> 3;
            for (int i = tid; i < D16R * og; i += D16T) {
                const int r = i / og, o8 = i - r * og;
                const bool ok = t0 + r < L;
                const float* src = dyb + (int64_t)(ok ? t0 + r : 0) * ldy + 8 * o8;
                const float4 a = *reinterpret_cast<const float4*>(src), c = *reinterpret_cast<const float4*>(src + 4);
                const float v[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
                bf16x8 h;
#pragma unroll
                for (int j = 0; j < 8; ++j) h[j] = (__bf16)(ok ? v[j] : 0.f);
                *reinterpret_cast<bf16x8*>(dys + r * DS + 8 * o8) = h;
            }
            // the window: rows t0 - pad .. t0 - pad + win - 1 (zero outside [0, L))
            const int ig = Cin >> 3;
            for (int i = tid; i < win * ig; i += D16T) {
                const int r = i / ig, i8 = i - r * ig;
                const int t = t0 + r - pad;
                const bool ok = t >= 0 && t < L;
                const float* src = xb + (int64_t)(ok ? t : 0) * ldx + 8 * i8;
                const float4 a = *reinterpret_cast<const float4*>(src), c = *reinterpret_cast<const float4*>(src + 4);
                const float v[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
                bf16x8 h;
#pragma unroll
                for (int j = 0; j < 8; ++j) h[j] = (__bf16)(ok ? v[j] : 0.f);
                *reinterpret_cast<bf16x8*>(xs + r * XS + 8 * i8) = h;
            }
            __syncthreads();
#pragma unroll
            for (int s = 0; s < D16R / 32; ++s) {
                if (j0 >= nT) break;   // wave-uniform: a wave without tiles only stages
                int ot_prev = -1;
                bf16x8 a;
#pragma unroll
                for (int j = 0; j < D16MAXT; ++j) {
                    // no per-lane early-out: the transposed reads need all 64 lanes
                    if (j < tpw && j0 + j < nT) {
                        if (tot[j] != ot_prev) {
                            a = ztr_frag(dys, 32 * s, 16 * tot[j], DS);
                            ot_prev = tot[j];
                        }
                        const bf16x8 bb = ztr_frag(xs, 32 * s + tk[j], 16 * tit[j], XS);
                        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bb, acc[j], 0, 0, 0);
                    }
                }
            }
        }
    }
    // D: col (i) = lane & 15, row (o) = 4 (lane >> 4) + r.  Slab layout [tap][o][i] (i fastest:
    // 64-byte row segments per store instead of a K-float stride between lanes); the [o][i][tap]
    // weight layout is restored by the slab sum's output permutation (conv.hip sum_splits_launch)
    float* slab = part + (int64_t)blockIdx.x * Cout * Cin * K;
#pragma unroll
    for (int j = 0; j < D16MAXT; ++j) {
        if (j < tpw && j0 + j < nT) {
            const int i = 16 * tit[j] + lr;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int o = 16 * tot[j] + 4 * lc + r;
                slab[((int64_t)tk[j] * Cout + o) * Cin + i] = acc[j][r];
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

// channel-vectorised forms (C % 4 == 0): a thread owns 4 channels of MP_TR consecutive steps of
// one sequence, so each X / dY row is read once per run instead of three (fwd) / nine (bwd)
// times, with 32-bit index math.  Same comparisons and the same s-1, s, s+1 summation order as
// the scalar kernels above, hence bit-identical results.
constexpr int MP_TR = 4;

__device__ __forceinline__ float mp_max3(float a, float b, float c, bool ha, bool hc) {
    float m = ha ? a : -INFINITY;
    m = (b > m || !ha) ? b : m;
    if (hc) m = c > m ? c : m;
    return m;
}

__device__ __forceinline__ int mp_arg3(float a, float b, float c, bool ha, bool hc) {
    int best = 0;
    float m;
    if (ha) {
        m = a;
        best = -1;
        if (b > m) { m = b; best = 0; }
    } else {
        m = b;
    }
    if (hc && c > m) best = 1;
    return best;
}

__global__ __launch_bounds__(256) void k_maxpool3_fwd4(const float4* __restrict__ X, int B, int L, int C4,
                                                       float4* __restrict__ Y) {
    const int nrun = (L + MP_TR - 1) / MP_TR;
    const int n = B * nrun * C4;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int c = i % C4, r = i / C4;
        const int t0 = (r % nrun) * MP_TR, b = r / nrun;
        const float4* xb = X + (int64_t)b * L * C4 + c;
        float4* yb = Y + (int64_t)b * L * C4 + c;
        float4 v[MP_TR + 2];
#pragma unroll
        for (int j = 0; j < MP_TR + 2; ++j) {
            const int t = t0 - 1 + j;
            v[j] = (t >= 0 && t < L) ? xb[(int64_t)t * C4] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int j = 0; j < MP_TR; ++j) {
            const int t = t0 + j;
            if (t >= L) continue;
            const bool ha = t > 0, hc = t + 1 < L;
            float4 m;
            m.x = mp_max3(v[j].x, v[j + 1].x, v[j + 2].x, ha, hc);
            m.y = mp_max3(v[j].y, v[j + 1].y, v[j + 2].y, ha, hc);
            m.z = mp_max3(v[j].z, v[j + 1].z, v[j + 2].z, ha, hc);
            m.w = mp_max3(v[j].w, v[j + 1].w, v[j + 2].w, ha, hc);
            yb[(int64_t)t * C4] = m;
        }
    }
}

__device__ __forceinline__ float f4c(const float4& v, int q) {   // q: a compile-time constant
    return q == 0 ? v.x : (q == 1 ? v.y : (q == 2 ? v.z : v.w));
}

__global__ __launch_bounds__(256) void k_maxpool3_bwd4(const float4* __restrict__ dY, const float4* __restrict__ X,
                                                       int B, int L, int C4, float4* __restrict__ dX,
                                                       int accumulate) {
    const int nrun = (L + MP_TR - 1) / MP_TR;
    const int n = B * nrun * C4;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int c = i % C4, r = i / C4;
        const int t0 = (r % nrun) * MP_TR, b = r / nrun;
        const int64_t base = (int64_t)b * L * C4 + c;
        // X rows t0-2 .. t0+MP_TR+1, dY rows t0-1 .. t0+MP_TR
        float4 v[MP_TR + 4], g[MP_TR + 2];
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int j = 0; j < MP_TR + 4; ++j) {
            const int t = t0 - 2 + j;
            v[j] = z;
            if (t >= 0 && t < L) v[j] = X[base + (int64_t)t * C4];
        }
#pragma unroll
        for (int j = 0; j < MP_TR + 2; ++j) {
            const int t = t0 - 1 + j;
            g[j] = z;
            if (t >= 0 && t < L) g[j] = dY[base + (int64_t)t * C4];
        }
        // first-maximum position of the windows centred at t0-1 .. t0+MP_TR, 4 channels packed
        int a[MP_TR + 2][4];
#pragma unroll
        for (int j = 0; j < MP_TR + 2; ++j) {
            const int w = t0 - 1 + j;
            const bool ha = w > 0, hc = w + 1 < L;
            a[j][0] = mp_arg3(v[j].x, v[j + 1].x, v[j + 2].x, ha, hc);
            a[j][1] = mp_arg3(v[j].y, v[j + 1].y, v[j + 2].y, ha, hc);
            a[j][2] = mp_arg3(v[j].z, v[j + 1].z, v[j + 2].z, ha, hc);
            a[j][3] = mp_arg3(v[j].w, v[j + 1].w, v[j + 2].w, ha, hc);
        }
#pragma unroll
        for (int j = 1; j <= MP_TR; ++j) {
            const int s = t0 - 1 + j;
            if (s >= L) continue;
            float o[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float acc = 0.f;
                if (s > 0 && a[j - 1][q] == 1) acc += f4c(g[j - 1], q);
                if (a[j][q] == 0) acc += f4c(g[j], q);
                if (s + 1 < L && a[j + 1][q] == -1) acc += f4c(g[j + 1], q);
                o[q] = acc;
            }
            float4* dp = dX + base + (int64_t)s * C4;
            float4 r4 = make_float4(o[0], o[1], o[2], o[3]);
            if (accumulate) {
                const float4 d = *dp;
                r4 = make_float4(d.x + r4.x, d.y + r4.y, d.z + r4.z, d.w + r4.w);
            }
            *dp = r4;
        }
    }
}

__global__ void k_add_act(const float* __restrict__ A, const float* __restrict__ Bm, int64_t n, int act,
                          float* __restrict__ Y) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float v = A[i] + Bm[i];
        Y[i] = act == 1 ? fmaxf(v, 0.f) : v;
    }
}

// FHRResidual's tail in one pass each way (ref/model/inception_time.py:152-170): forward
// s = act(a + b) (saved for the backward) and y = Dropout1d(s); backward dx = Dropout1d(dy) act'(s)
// — each element the value of k_add_act + k_dropout / k_dropout + k_act_bwd (the same mask index,
// hash, scale and products).  act: 0 none, 1 ReLU.  F4: four channels of one row per thread.
template <bool F4>
__global__ void k_add_act_drop(const float* __restrict__ A, const float* __restrict__ Bm, int64_t n, int C, int act,
                               int L, float p, uint64_t seed, const uint64_t* __restrict__ soff,
                               float* __restrict__ S, float* __restrict__ Y) {
    seed = eff_seed(seed, soff);
    const uint32_t th = drop_threshold(p);
    const float sc = 1.f / (1.f - p);
    const int64_t LC = (int64_t)L * C;
    constexpr int V = F4 ? 4 : 1;
    for (int64_t i0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) * V; i0 < n;
         i0 += (int64_t)gridDim.x * blockDim.x * V) {
        const uint64_t m = L > 0 ? (uint64_t)((i0 / LC) * C + i0 % C) : (uint64_t)i0;
        float a[V], b[V], sv[V], yv[V];
        if constexpr (F4) {
            const float4 a4 = *reinterpret_cast<const float4*>(A + i0), b4 = *reinterpret_cast<const float4*>(Bm + i0);
            a[0] = a4.x; a[1] = a4.y; a[2] = a4.z; a[3] = a4.w;
            b[0] = b4.x; b[1] = b4.y; b[2] = b4.z; b[3] = b4.w;
        } else {
            a[0] = A[i0];
            b[0] = Bm[i0];
        }
#pragma unroll
        for (int e = 0; e < V; ++e) {
            const float v = a[e] + b[e];
            sv[e] = act == 1 ? fmaxf(v, 0.f) : v;
            yv[e] = mix_hash(seed, m + e) >= th ? sv[e] * sc : 0.f;
        }
        if constexpr (F4) {
            *reinterpret_cast<float4*>(S + i0) = make_float4(sv[0], sv[1], sv[2], sv[3]);
            *reinterpret_cast<float4*>(Y + i0) = make_float4(yv[0], yv[1], yv[2], yv[3]);
        } else {
            S[i0] = sv[0];
            Y[i0] = yv[0];
        }
    }
}

template <bool F4>
__global__ void k_act_drop_bwd(const float* __restrict__ dY, const float* __restrict__ S, int64_t n, int C, int act,
                               int L, float p, uint64_t seed, const uint64_t* __restrict__ soff,
                               float* __restrict__ dX) {
    seed = eff_seed(seed, soff);
    const uint32_t th = drop_threshold(p);
    const float sc = 1.f / (1.f - p);
    const int64_t LC = (int64_t)L * C;
    constexpr int V = F4 ? 4 : 1;
    for (int64_t i0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) * V; i0 < n;
         i0 += (int64_t)gridDim.x * blockDim.x * V) {
        const uint64_t m = L > 0 ? (uint64_t)((i0 / LC) * C + i0 % C) : (uint64_t)i0;
        float g[V], sv[V], o[V];
        if constexpr (F4) {
            const float4 g4 = *reinterpret_cast<const float4*>(dY + i0), s4 = *reinterpret_cast<const float4*>(S + i0);
            g[0] = g4.x; g[1] = g4.y; g[2] = g4.z; g[3] = g4.w;
            sv[0] = s4.x; sv[1] = s4.y; sv[2] = s4.z; sv[3] = s4.w;
        } else {
            g[0] = dY[i0];
            sv[0] = S[i0];
        }
#pragma unroll
        for (int e = 0; e < V; ++e) {
            const float gd = mix_hash(seed, m + e) >= th ? g[e] * sc : 0.f;
            o[e] = gd * (act == 1 ? (sv[e] > 0.f ? 1.f : 0.f) : 1.f);
        }
        if constexpr (F4) {
            *reinterpret_cast<float4*>(dX + i0) = make_float4(o[0], o[1], o[2], o[3]);
        } else {
            dX[i0] = o[0];
        }
    }
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

// C % 4 == 0: four channels of one row per thread (one index split per float4, 16-byte accesses);
// the same per-element mask index and hash as k_dropout.
__global__ void k_dropout4(const float4* __restrict__ X, int64_t n4, int C, int L, float p, uint64_t seed,
                           const uint64_t* __restrict__ soff, float4* __restrict__ Y) {
    seed = eff_seed(seed, soff);
    const uint32_t th = drop_threshold(p);
    const float sc = 1.f / (1.f - p);
    const int64_t LC = (int64_t)L * C;
    for (int64_t i4 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i4 < n4;
         i4 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = 4 * i4;
        const uint64_t m = L > 0 ? (uint64_t)((i / LC) * C + i % C) : (uint64_t)i;
        const float4 x = X[i4];
        float4 y;
        y.x = mix_hash(seed, m) >= th ? x.x * sc : 0.f;
        y.y = mix_hash(seed, m + 1) >= th ? x.y * sc : 0.f;
        y.z = mix_hash(seed, m + 2) >= th ? x.z * sc : 0.f;
        y.w = mix_hash(seed, m + 3) >= th ? x.w * sc : 0.f;
        Y[i4] = y;
    }
}

__global__ __launch_bounds__(256) void k_time_mean(const float* __restrict__ X, int L, int C, float* __restrict__ Y) {
    const int b = blockIdx.x;
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        const float* xb = X + (int64_t)b * L * C + c;
        float s = 0.f;
        int t = 0;
        // 16 rows' loads in flight, then added in row order (the same sum as the one-at-a-time
        // loop, which waited out a load per row: 85 us per launch at L = 256)
        for (; t + 16 <= L; t += 16) {
            float v[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) v[u] = xb[(int64_t)(t + u) * C];
#pragma unroll
            for (int u = 0; u < 16; ++u) s += v[u];
        }
        for (; t < L; ++t) s += xb[(int64_t)t * C];
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

constexpr int AFW = 8;            // waves per forward workgroup (query tiles wv, wv + AFW)

__global__ __launch_bounds__(64 * AFW, 4) void k_attn_fwd(const float* __restrict__ qkv, int S, int H, float scale,
                                                       float p, uint64_t seed, const uint64_t* __restrict__ soff,
                                                       float* __restrict__ out, float* __restrict__ lse) {
    seed = eff_seed(seed, soff);
    __shared__ float Ks[256 * AKS];
    __shared__ float Vs[256 * AKS];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lr = lane & 15, lc = lane >> 4;
    const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
    const int E = H * DH, E3 = 3 * E;
    const float* base = qkv + (int64_t)b * S * E3 + h * DH;
    for (int i = tid; i < S * DH; i += 64 * AFW) {
        const int r = i / DH, d = i - r * DH;
        Ks[r * AKS + d] = base[(int64_t)r * E3 + E + d];
        Vs[r * AKS + d] = base[(int64_t)r * E3 + 2 * E + d];
    }
    __syncthreads();
    const int nkt = S >> 4;
    for (int qt = wv; qt < nkt; qt += AFW) {
        const int q0 = 16 * qt;
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
                    // fused as written (fmaf): the contraction is not left to the compiler, whose
                    // choice moved with the launch bounds (a separate product rounds once more)
                    const float e = expf(fmaf(st[kt][r], scale, -m));
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
}

__global__ __launch_bounds__(256, 2) void k_attn_bwd(const float* __restrict__ qkv, const float* __restrict__ O,
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
                const float pr = expf(fmaf(sc[r], scale, -lses[ql]));   // fused as written (as the forward)
                float keep = 1.f;
                if (p > 0.f) {
                    const uint64_t id = ((uint64_t)bh * S + q0 + ql) * S + 16 * kt + lr;
                    keep = mix_hash(seed, id) >= th ? dsc : 0.f;
                }
                pd[r] = pr * keep;                       // dropped probabilities (used by O)
                ds[r] = pr * fmaf(dp[r], keep, -Dq[ql]);   // dS = P (dP - D)
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

int vt_zconv16_ws_floats(int Cin, int Cout, int K, int64_t* floats) {
    VT_CHECK_ARG(floats && Cin > 0 && Cout > 0 && K > 0, "vt_zconv16_ws_floats: args");
    const int64_t a = zconv16_taps_elems(Cin, Cout, K), b = zconv16_taps_elems(Cout, Cin, K);   // fwd / bwd-data
    *floats = ((a > b ? a : b) + 1) / 2;
    return VT_OK;
}

int vt_zconv16_taps_elems(int Cin, int Cout, int K, int64_t* elems) {
    VT_CHECK_ARG(elems && Cin > 0 && Cout > 0 && K > 0, "vt_zconv16_taps_elems: args");
    *elems = zconv16_taps_elems(Cin, Cout, K);
    return VT_OK;
}

int vt_zconv16_taps(int n, const int64_t* W, const int* Cin, const int* Cout, const int* K, int flip,
                    const int64_t* T, void* stream) {
    VT_CHECK_ARG(n >= 1 && n <= ZTB_MAX && W && Cin && Cout && K && T, "vt_zconv16_taps: %d weights (1..%d)", n,
                 ZTB_MAX);
    ZTapBatch tb{};
    tb.n = n;
    tb.flip = flip ? 1 : 0;
    tb.prefix[0] = 0;
    for (int h = 0; h < n; ++h) {
        VT_CHECK_ARG(W[h] && T[h] && !(T[h] & 15) && Cin[h] > 0 && Cout[h] > 0 && K[h] > 0,
                     "vt_zconv16_taps: weight %d", h);
        // the image of the convolution that reads it: forward (Cin -> Cout) or, flip, the
        // backward-data conv (Cout -> Cin) of the same weight
        const int ci = flip ? Cout[h] : Cin[h], co = flip ? Cin[h] : Cout[h];
        tb.W[h] = reinterpret_cast<const float*>(W[h]);
        tb.T[h] = reinterpret_cast<__bf16*>(T[h]);
        tb.Cin[h] = ci;
        tb.Cout[h] = co;
        tb.K[h] = K[h];
        tb.TC[h] = co <= 32 ? 32 : 128;
        tb.cin32[h] = (ci + 31) & ~31;
        const int64_t e = (int64_t)K[h] * tb.TC[h] * tb.cin32[h];
        tb.prefix[h + 1] = tb.prefix[h] + (int)((e + 255) / 256);
    }
    hipLaunchKernelGGL(k_zconv16_taps_batch, dim3((unsigned)tb.prefix[n]), dim3(256), 0, S(stream), tb);
    VT_LAUNCH_CHECK("vt_zconv16_taps");
    return VT_OK;
}

int vt_zconv16_fwd_t(const float* X, int ldx, int B, int L, int Cin, const void* T, int Cout, int K, int pad_left,
                     float* Y, int ldy, int accumulate, void* stream) {
    VT_CHECK_ARG(zconv_shape_ok(B, L, Cin, Cout, K, pad_left) && ldx >= Cin && ldy >= Cout && T &&
                     !(reinterpret_cast<uintptr_t>(T) & 15),
                 "vt_zconv16_fwd_t: shape / tap image");
    VT_CHECK_ARG(zconv16_launch<false>(X, ldx, B, L, Cin, nullptr, Cout, K, pad_left, Y, ldy, accumulate,
                                       reinterpret_cast<__bf16*>(const_cast<void*>(T)), S(stream)) == VT_OK,
                 "vt_zconv16_fwd_t: unsupported configuration (X 16-B aligned, ldx a multiple of 4)");
    VT_LAUNCH_CHECK("vt_zconv16_fwd_t");
    return VT_OK;
}

int vt_zconv16_bwd_data_t(const float* dY, int ldy, int B, int L, int Cin, const void* T, int Cout, int K,
                          int pad_left, float* dX, int ldx, int accumulate, void* stream) {
    VT_CHECK_ARG(zconv_shape_ok(B, L, Cin, Cout, K, pad_left) && ldx >= Cin && ldy >= Cout && T &&
                     !(reinterpret_cast<uintptr_t>(T) & 15),
                 "vt_zconv16_bwd_data_t: shape / tap image");
    VT_CHECK_ARG(zconv16_launch<true>(dY, ldy, B, L, Cout, nullptr, Cin, K, K - 1 - pad_left, dX, ldx, accumulate,
                                      reinterpret_cast<__bf16*>(const_cast<void*>(T)), S(stream)) == VT_OK,
                 "vt_zconv16_bwd_data_t: unsupported configuration (dY 16-B aligned, ldy a multiple of 4)");
    VT_LAUNCH_CHECK("vt_zconv16_bwd_data_t");
    return VT_OK;
}

int vt_zconv16_fwd(const float* X, int ldx, int B, int L, int Cin, const float* W, int Cout, int K, int pad_left,
                   float* Y, int ldy, int accumulate, float* ws, int64_t ws_floats, void* stream) {
    VT_CHECK_ARG(zconv_shape_ok(B, L, Cin, Cout, K, pad_left) && ldx >= Cin && ldy >= Cout,
                 "vt_zconv16_fwd: shape (Cin/Cout multiples of 16 <= 128, K in {1,5,15,40}, 0 <= pad < K)");
    VT_CHECK_ARG(ws && 2 * ws_floats >= zconv16_taps_elems(Cin, Cout, K) && !(reinterpret_cast<uintptr_t>(ws) & 15),
                 "vt_zconv16_fwd: workspace (vt_zconv16_ws_floats, 16-B aligned)");
    VT_CHECK_ARG(zconv16_launch<false>(X, ldx, B, L, Cin, W, Cout, K, pad_left, Y, ldy, accumulate,
                                       reinterpret_cast<__bf16*>(ws), S(stream)) == VT_OK,
                 "vt_zconv16_fwd: unsupported configuration (X 16-B aligned, ldx a multiple of 4)");
    VT_LAUNCH_CHECK("vt_zconv16_fwd");
    return VT_OK;
}

int vt_zconv16_bwd_data(const float* dY, int ldy, int B, int L, int Cin, const float* W, int Cout, int K, int pad_left,
                        float* dX, int ldx, int accumulate, float* ws, int64_t ws_floats, void* stream) {
    VT_CHECK_ARG(zconv_shape_ok(B, L, Cin, Cout, K, pad_left) && ldx >= Cin && ldy >= Cout,
                 "vt_zconv16_bwd_data: shape");
    VT_CHECK_ARG(ws && 2 * ws_floats >= zconv16_taps_elems(Cout, Cin, K) && !(reinterpret_cast<uintptr_t>(ws) & 15),
                 "vt_zconv16_bwd_data: workspace (vt_zconv16_ws_floats, 16-B aligned)");
    VT_CHECK_ARG(zconv16_launch<true>(dY, ldy, B, L, Cout, W, Cin, K, K - 1 - pad_left, dX, ldx, accumulate,
                                      reinterpret_cast<__bf16*>(ws), S(stream)) == VT_OK,
                 "vt_zconv16_bwd_data: unsupported configuration (dY 16-B aligned, ldy a multiple of 4)");
    VT_LAUNCH_CHECK("vt_zconv16_bwd_data");
    return VT_OK;
}

int vt_zconv16_bwd_weight(const float* dY, int ldy, const float* X, int ldx, int B, int L, int Cin, int Cout, int K,
                          int pad_left, float* dW, int accumulate, float* ws, int64_t ws_floats, void* stream) {
    VT_CHECK_ARG(zconv_shape_ok(B, L, Cin, Cout, K, pad_left) && ldx >= Cin && ldy >= Cout && !(ldx & 3) &&
                     !(ldy & 3) && !(reinterpret_cast<uintptr_t>(dY) & 15) && !(reinterpret_cast<uintptr_t>(X) & 15),
                 "vt_zconv16_bwd_weight: shape / alignment (16-B rows)");
    VT_CHECK_ARG(((Cout / 16) * (Cin / 16) * K + D16W - 1) / D16W <= D16MAXT, "vt_zconv16_bwd_weight: too many tiles");
    // one sample per workgroup up to 256 (the chunks' staging round trips, not the MFMAs, bound
    // a workgroup: 128 slabs took 25-44 us per launch whatever K)
    const int G = zdw_groups(B);
    const int64_t n = (int64_t)Cout * Cin * K;
    VT_CHECK_ARG(ws_floats >= G * n, "vt_zconv16_bwd_weight: workspace too small");
    hipStream_t st = S(stream);
    hipLaunchKernelGGL(k_zconv16_dw, dim3(G), dim3(D16T), 0, st, dY, ldy, X, ldx, B, L, Cin, Cout, K, pad_left, ws);
    const int rc = sum_splits_launch(ws, G, n, dW, accumulate, st, K, Cout, Cin);   // slab order [k][o][i] -> dW [o][i][k]
    if (rc) {
        set_error("vt_zconv16_bwd_weight: %d weight-gradient slabs exceed the split sum's limit", G);
        return rc;
    }
    VT_LAUNCH_CHECK("vt_zconv16_bwd_weight");
    return VT_OK;
}

int vt_zconv_bwd_weight_ws_floats(int B, int Cin, int Cout, int K, int64_t* floats) {
    VT_CHECK_ARG(B > 0 && floats, "vt_zconv_bwd_weight_ws_floats: args");
    *floats = (int64_t)zdw_groups(B) * Cout * Cin * K;   // both weight-gradient kernels: one slab per group
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
    const int rc = sum_splits_launch(ws, G, n, dW, accumulate, st);
    if (rc) {
        set_error("vt_zconv_bwd_weight: %d weight-gradient slabs exceed the split sum's limit", G);
        return rc;
    }
    VT_LAUNCH_CHECK("vt_zconv_bwd_weight");
    return VT_OK;
}

int vt_maxpool3_fwd(const float* X, int B, int L, int C, float* Y, void* stream) {
    VT_CHECK_ARG(B > 0 && L > 0 && C > 0, "vt_maxpool3_fwd: shape");
    const int64_t n = (int64_t)B * L * C;
    if (C % 4 == 0 && n < (int64_t)1 << 31) {
        const int64_t nv = (int64_t)B * ((L + MP_TR - 1) / MP_TR) * (C / 4);
        hipLaunchKernelGGL(k_maxpool3_fwd4, dim3(ew_blocks(nv)), dim3(256), 0, S(stream),
                           reinterpret_cast<const float4*>(X), B, L, C / 4, reinterpret_cast<float4*>(Y));
    } else {
        hipLaunchKernelGGL(k_maxpool3_fwd, dim3(ew_blocks(n)), dim3(256), 0, S(stream), X, B, L, C, Y);
    }
    VT_LAUNCH_CHECK("vt_maxpool3_fwd");
    return VT_OK;
}

int vt_maxpool3_bwd(const float* dY, const float* X, int B, int L, int C, float* dX, int accumulate, void* stream) {
    VT_CHECK_ARG(B > 0 && L > 0 && C > 0, "vt_maxpool3_bwd: shape");
    const int64_t n = (int64_t)B * L * C;
    if (C % 4 == 0 && n < (int64_t)1 << 31) {
        const int64_t nv = (int64_t)B * ((L + MP_TR - 1) / MP_TR) * (C / 4);
        hipLaunchKernelGGL(k_maxpool3_bwd4, dim3(ew_blocks(nv)), dim3(256), 0, S(stream),
                           reinterpret_cast<const float4*>(dY), reinterpret_cast<const float4*>(X), B, L, C / 4,
                           reinterpret_cast<float4*>(dX), accumulate);
    } else {
        hipLaunchKernelGGL(k_maxpool3_bwd, dim3(ew_blocks(n)), dim3(256), 0, S(stream), dY, X, B, L, C, dX,
                           accumulate);
    }
    VT_LAUNCH_CHECK("vt_maxpool3_bwd");
    return VT_OK;
}

static bool f4_ok(int64_t n, int C, const void* a, const void* b, const void* c, const void* d) {
    const uintptr_t o = reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) |
                        reinterpret_cast<uintptr_t>(c) | reinterpret_cast<uintptr_t>(d);
    return C % 4 == 0 && n % 4 == 0 && (o & 15) == 0;
}

int vt_add_act_dropout_fwd(const float* A, const float* Bm, int64_t n, int C, int act, int L, float p, int64_t seed,
                           const void* seed_offset, float* S_out, float* Y, void* stream) {
    VT_CHECK_ARG(n > 0 && C > 0 && L >= 0 && (act == 0 || act == 1) && p >= 0.f && p < 1.f && n % C == 0,
                 "vt_add_act_dropout_fwd: args (act none/relu, 0 <= p < 1, n a multiple of C)");
    const uint64_t* so = seed_off(seed_offset, p);
    if (f4_ok(n, C, A, Bm, S_out, Y))
        hipLaunchKernelGGL(k_add_act_drop<true>, dim3(ew_blocks(n / 4)), dim3(256), 0, S(stream), A, Bm, n, C, act, L,
                           p, (uint64_t)seed, so, S_out, Y);
    else
        hipLaunchKernelGGL(k_add_act_drop<false>, dim3(ew_blocks(n)), dim3(256), 0, S(stream), A, Bm, n, C, act, L, p,
                           (uint64_t)seed, so, S_out, Y);
    VT_LAUNCH_CHECK("vt_add_act_dropout_fwd");
    return VT_OK;
}

int vt_act_dropout_bwd(const float* dY, const float* S_in, int64_t n, int C, int act, int L, float p, int64_t seed,
                       const void* seed_offset, float* dX, void* stream) {
    VT_CHECK_ARG(n > 0 && C > 0 && L >= 0 && (act == 0 || act == 1) && p >= 0.f && p < 1.f && n % C == 0,
                 "vt_act_dropout_bwd: args (act none/relu, 0 <= p < 1, n a multiple of C)");
    const uint64_t* so = seed_off(seed_offset, p);
    if (f4_ok(n, C, dY, S_in, dX, dX))
        hipLaunchKernelGGL(k_act_drop_bwd<true>, dim3(ew_blocks(n / 4)), dim3(256), 0, S(stream), dY, S_in, n, C, act,
                           L, p, (uint64_t)seed, so, dX);
    else
        hipLaunchKernelGGL(k_act_drop_bwd<false>, dim3(ew_blocks(n)), dim3(256), 0, S(stream), dY, S_in, n, C, act, L,
                           p, (uint64_t)seed, so, dX);
    VT_LAUNCH_CHECK("vt_act_dropout_bwd");
    return VT_OK;
}

int vt_add_act_fwd(const float* A, const float* Bm, int64_t n, int act, float* Y, void* stream) {
    VT_CHECK_ARG(n > 0 && (act == 0 || act == 1), "vt_add_act_fwd: n > 0, act none/relu");
    hipLaunchKernelGGL(k_add_act, dim3(ew_blocks(n)), dim3(256), 0, S(stream), A, Bm, n, act, Y);
    VT_LAUNCH_CHECK("vt_add_act_fwd");
    return VT_OK;
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
    if (C % 4 == 0 && n % 4 == 0 && ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(Y)) & 15) == 0) {
        hipLaunchKernelGGL(k_dropout4, dim3(ew_blocks(n / 4)), dim3(256), 0, S(stream),
                           reinterpret_cast<const float4*>(X), n / 4, C, L, p, (uint64_t)seed,
                           seed_off(seed_offset, p), reinterpret_cast<float4*>(Y));
    } else {
        hipLaunchKernelGGL(k_dropout, dim3(ew_blocks(n)), dim3(256), 0, S(stream), X, n, C, L, p, (uint64_t)seed,
                           seed_off(seed_offset, p), Y);
    }
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
    hipLaunchKernelGGL(k_attn_fwd, dim3(B * H), dim3(64 * AFW), 0, S(stream), qkv, S_, H, scale, p,
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
