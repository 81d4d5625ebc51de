// Conv-block backward-data on a bf16 operand (SURVEY.md §8(a) a11, a15;
// ref/model/vae_teb_model.py:128-253 under autograd, in the reference's 16-bit
// training precision: DESIGN.md §5).
//
// Two launches replace the fused-staging kernel of conv_bf16.hip (k_conv_bf16<.., BNB>)
// and, for the x2-upsample layers, its gpad round trip + k_conv_fold:
//
//  1. k_bn_bwd_x16: the BatchNorm input gradient gamma rstd (dz - dbeta/M - xhat dgamma/M)
//     (bnbwd.h, the same element function and bits as every other path) streamed once
//     from (dy, pre-BN conv output) into bf16 rows of ceil32(C) channels (zero padding):
//     flat float4 reads of the odd-width fp32 rows, an LDS row image, 16-byte stores.
//     The rows are the operand of both the backward-data conv below and the weight
//     gradient (vt_conv1d_bwd_weight_bf16_dy16s), which stage them with aligned 16-byte
//     loads and no conversion.
//  2. k_cbd16: the transposed conv (implicit GEMM on v_mfma_f32_16x16x32_bf16, fp32
//     accumulation) over that operand.  A workgroup stages its whole operand window (all
//     channel chunks: one contiguous block of rows in HBM) once, then walks the 32-channel
//     chunks with the next chunk's taps prefetched into registers during the current
//     chunk's MFMAs.  Accumulation order (chunks ascending, taps ascending inside a chunk,
//     the same 8-channel lane groups) is that of k_conv_bf16, so the padded gradient rows
//     are bit-identical; the output is written
//       - without upsampling: straight into dX (crop; reflect mirror rows through the edge
//         buffer + k_conv_fold_edges, as vt_conv1d_bwd_dx_bf16_bn);
//       - with the x2 upsample (UPF): the tile's padded rows go to LDS and the fold (reflect
//         mirrors, then the adjoint of the linear upsample with its four fixed weights, in
//         k_conv_fold's order: the same bits) is applied there; each workgroup owns TS input
//         rows and computes the 2 TS + pad + 2 padded rows they read.
#include <stdlib.h>

#include "conv.h"
#include "h16.h"

namespace vt {

namespace {


constexpr int RS = 40;   // bf16 row stride of the staged window / tap rows (as conv_bf16.hip)
// rows per k_bn_bwd_x16 block (XRB): 64, or 256 for C <= 4 (vt_batchnorm_bwd_x16; every element's
// value is computed the same way for any block height: the same bits)

// ------------------------------------------------------------------ 1. BN backward -> bf16
template <typename H, int ACT, int XRB = 64>
__global__ __launch_bounds__(256) void k_bn_bwd_x16(const float* __restrict__ dy, const float* __restrict__ x2,
                                                    const float* __restrict__ bnp, int64_t M, int C, int c32,
                                                    float invM, H* __restrict__ d16) {
    extern __shared__ __attribute__((aligned(16))) float xl[];
    float* prm = xl;                                                // [C][8]: mean rstd gamma beta dgamma dbeta
    H* img = reinterpret_cast<H*>(xl + 8 * ((C + 3) & ~3));   // [XRB][c32]
    const int tid = threadIdx.x;
    for (int i = tid; i < 6 * C; i += 256) {
        const int k = i / C, c = i - k * C;
        prm[8 * c + k] = bnp[i];
    }
    __syncthreads();
    for (int64_t r0 = (int64_t)blockIdx.x * XRB; r0 < M; r0 += (int64_t)gridDim.x * XRB) {
        const int nr = M - r0 < XRB ? (int)(M - r0) : XRB;
        const int n = nr * C;                 // flat elements of this row block
        const float* a = dy + r0 * C;          // r0 * C * 4 bytes: 16-byte aligned (XRB % 4 == 0)
        const float* q = x2 + r0 * C;
        // flat float4 items (the tail of a ragged last block element by element)
        for (int i = tid; 4 * i < n; i += 256) {
            float va[4], vq[4];
            if (4 * i + 4 <= n) {
                const float4 fa = *reinterpret_cast<const float4*>(a + 4 * i);
                const float4 fq = *reinterpret_cast<const float4*>(q + 4 * i);
                va[0] = fa.x; va[1] = fa.y; va[2] = fa.z; va[3] = fa.w;
                vq[0] = fq.x; vq[1] = fq.y; vq[2] = fq.z; vq[3] = fq.w;
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    va[j] = 4 * i + j < n ? a[4 * i + j] : 0.f;
                    vq[j] = 4 * i + j < n ? q[4 * i + j] : 0.f;
                }
            }
            int r = (4 * i) / C, c = 4 * i - r * C;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (4 * i + j < n) {
                    const float4 p0 = *reinterpret_cast<const float4*>(prm + 8 * c);
                    const float2 p1 = *reinterpret_cast<const float2*>(prm + 8 * c + 4);
                    const float v = bn_bwd_val_r(va[j], vq[j], p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, ACT, invM);
                    img[r * c32 + c] = (H)v;
                }
                if (++c == C) {
                    c = 0;
                    ++r;
                }
            }
        }
        __syncthreads();
        // rows out as 16-byte segments, channels >= C zero
        const int segs = c32 / 8;
        for (int i = tid; i < nr * segs; i += 256) {
            const int r = i / segs, s = i - r * segs;
            hv8<H> v = *reinterpret_cast<const hv8<H>*>(img + r * c32 + 8 * s);
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (8 * s + j >= C) v[j] = (H)0.f;
            *reinterpret_cast<hv8<H>*>(d16 + (r0 + r) * c32 + 8 * s) = v;
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------ 2. backward-data conv
// geometry of one launch (bwd terms: the conv's input is the forward's output gradient)
struct BdGeo {
    int Lf;       // rows of d16 per sample (forward L_out)
    int Ci;       // channels of d16 (forward Cout); c32 = nch * 32 its row stride
    int nch;
    int Co;       // output channels (forward Cin)
    int Lp;       // padded gradient rows per sample: Lf + K - 1
    // output
    int pad;      // forward padding
    int L;        // dX rows per sample (forward L_in)
    int L_up;     // upsampled length (UPF)
    int TS;       // UPF: input rows owned per workgroup
    float* edge;  // non-UPF reflect: mirrored rows [B][2 pad][Co] (nullable: crop only)
    int p_first;  // non-UPF: first padded row computed (causal crop: pad; reflect: 0)
    int p_end;    // non-UPF: one past the last padded row computed
};

template <int K, int NT, int PMX = 0>
struct DCfg {
    // position blocks per wave: taller tiles for the narrow layers (more MFMA work per staged window);
    // PMX overrides (short rows: the encoders' 256 positions fill only half of a 512-row tile)
    static constexpr int PM = PMX ? PMX : (NT <= 2 ? 8 : 2);
    static constexpr int TC = 16 * NT, TP = 64 * PM, WIN = TP + K - 1;
    static constexpr int WB = K * TC * RS;                       // bf16 elements of one tap chunk
    static constexpr int NWI = (K * TC * 4 + 255) / 256;         // 16-byte tap items per thread
    static int lds_bytes(int nch, bool upf) {
        const int stage = (nch * WIN * RS + WB) * 2;
        const int fold = upf ? TP * (TC + 1) * 4 : 0;
        return stage > fold ? stage : fold;
    }
};

template <typename H, int K, int NT>
__device__ __forceinline__ void load_taps(hv8<H>* wt, const H* __restrict__ w16t, int co0,
                                          int Co, int c32, int c0) {
    using C = DCfg<K, NT>;
    const int tid = threadIdx.x;
#pragma unroll
    for (int it = 0; it < C::NWI; ++it) {
        const int i = tid + 256 * it;
        const int ic = i < K * C::TC * 4 ? i : K * C::TC * 4 - 1;
        const int oct = ic & 3, r = ic >> 2, k = r / C::TC, co = r - k * C::TC;
        const int coc = co0 + co < Co ? co0 + co : Co - 1;
        wt[it] = *(const hv8<H>*)(w16t + ((int64_t)coc * K + k) * c32 + c0 + 8 * oct);
    }
}

template <typename H, int K, int NT>
__device__ __forceinline__ void store_taps(const hv8<H>* wt, H* __restrict__ ws, int co0,
                                           int Co) {
    using C = DCfg<K, NT>;
    const int tid = threadIdx.x;
#pragma unroll
    for (int it = 0; it < C::NWI; ++it) {
        const int i = tid + 256 * it;
        if (i >= K * C::TC * 4) continue;
        const int oct = i & 3, r = i >> 2, k = r / C::TC, co = r - k * C::TC;
        hv8<H> v = wt[it];
        if (co0 + co >= Co) {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = (H)0.f;
        }
        *(hv8<H>*)(ws + (k * C::TC + co) * RS + 8 * oct) = v;
    }
}

// gradient of upsampled (unpadded) row t from the padded rows in LDS (local row = p - p0):
// k_conv_fold's gup for reflect padding with L_up > pad, same additions in the same order
__device__ __forceinline__ float fold_gup(const float* __restrict__ gp, int gs, int co, int t, int p0, int pad,
                                          int L_up, int Lp) {
    float v = gp[(t + pad - p0) * gs + co];
    if (t >= 1 && t <= pad) v += gp[(pad - t - p0) * gs + co];   // left mirror
    const int tr = pad + 2 * (L_up - 1) - t;                      // right mirror
    if (t <= L_up - 2 && tr < Lp && tr >= pad + L_up) v += gp[(tr - p0) * gs + co];
    return v;
}

template <typename H, int K, int NT, bool UPF, int PMX = 0>
__global__ __launch_bounds__(256) void k_cbd16(const H* __restrict__ d16, BdGeo g,
                                               const H* __restrict__ w16t, float* __restrict__ dx) {
    using C = DCfg<K, NT, PMX>;
    constexpr int PM = C::PM, TC = C::TC, TP = C::TP, WIN = C::WIN;
    extern __shared__ __attribute__((aligned(16))) char lb_raw[];
    H* const lb = reinterpret_cast<H*>(lb_raw);
    const int nch = g.nch, c32 = 32 * nch;
    H* xs = lb;                     // [nch][WIN][RS]
    H* ws = lb + nch * WIN * RS;    // [K][TC][RS]
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lr = lane & 15, lc = lane >> 4;
    const int co0 = blockIdx.y * TC, b = blockIdx.z;
    int p0, s0 = 0, s1 = 0;
    if constexpr (UPF) {
        s0 = blockIdx.x * g.TS;
        s1 = s0 + g.TS < g.L ? s0 + g.TS : g.L;
        p0 = s0 == 0 ? 0 : 2 * s0 - 1 + g.pad;
    } else {
        p0 = g.p_first + blockIdx.x * TP;   // causal: only the rows the crop keeps (p_first = pad)
    }
    hv8<H> wt[C::NWI];
    load_taps<H, K, NT>(wt, w16t, co0, g.Co, c32, 0);   // in flight during the window staging
    // the operand window: d16 rows p0 - (K - 1) .. p0 - (K - 1) + WIN - 1 of sample b, all chunks
    // (one contiguous run of rows in HBM), 16-byte items, zero outside [0, Lf)
    {
        const int segs = 4 * nch;
        const H* db = d16 + (int64_t)b * g.Lf * c32;
        const int rbase = p0 - (K - 1);
        constexpr int U = 8;
        for (int i0 = tid; i0 < WIN * segs; i0 += 256 * U) {
            hv8<H> v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = i0 + 256 * u;
                const int r = i / segs, s = i - r * segs;
                const int dr = rbase + r;
                const bool ok = i < WIN * segs && dr >= 0 && dr < g.Lf;
                v[u] = *(const hv8<H>*)(db + (int64_t)(ok ? dr : 0) * c32 + (ok ? 8 * s : 0));
                if (!ok) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) v[u][j] = (H)0.f;
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = i0 + 256 * u;
                if (i >= WIN * segs) continue;
                const int r = i / segs, s = i - r * segs;
                *(hv8<H>*)(xs + ((s >> 2) * WIN + r) * RS + 8 * (s & 3)) = v[u];
            }
        }
    }
    store_taps<H, K, NT>(wt, ws, co0, g.Co);
    __syncthreads();
    f32x4 acc[PM][NT];
#pragma unroll
    for (int m = 0; m < PM; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int ch = 0; ch < nch; ++ch) {
        const bool more = ch + 1 < nch;
        if (more) load_taps<H, K, NT>(wt, w16t, co0, g.Co, c32, 32 * (ch + 1));   // in flight during the MFMAs
        const H* xq = xs + (ch * WIN + PM * 16 * wv + lr) * RS + 8 * lc;
        const H* wq = ws + lr * RS + 8 * lc;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            hv8<H> af[PM], bf[NT];
#pragma unroll
            for (int m = 0; m < PM; ++m) af[m] = *(const hv8<H>*)(xq + (16 * m + k) * RS);
#pragma unroll
            for (int n = 0; n < NT; ++n) bf[n] = *(const hv8<H>*)(wq + (k * TC + 16 * n) * RS);
#pragma unroll
            for (int m = 0; m < PM; ++m)
#pragma unroll
                for (int n = 0; n < NT; ++n)
                    acc[m][n] = mfma16(af[m], bf[n], acc[m][n]);
        }
        __syncthreads();
        if (more) {
            store_taps<H, K, NT>(wt, ws, co0, g.Co);
            __syncthreads();
        }
    }
    // D layout: col (channel) = lane & 15, row (position) = 4 * (lane >> 4) + r
    if constexpr (!UPF) {
#pragma unroll
        for (int m = 0; m < PM; ++m)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int p = p0 + PM * 16 * wv + 16 * m + 4 * lc + r;
                if (p >= g.p_end) continue;
                const int sx = p - g.pad;
                float* yr;
                if (sx >= 0 && sx < g.L) yr = dx + ((int64_t)b * g.L + sx) * g.Co;
                else if (g.edge) yr = g.edge + ((int64_t)b * 2 * g.pad + (sx < 0 ? p : p - g.L)) * g.Co;
                else continue;
#pragma unroll
                for (int n = 0; n < NT; ++n) {
                    const int co = co0 + 16 * n + lr;
                    if (co < g.Co) yr[co] = acc[m][n][r];
                }
            }
    } else {
        // padded rows p0 .. p0 + TP - 1 to LDS (the staging buffers are free after the last barrier)
        constexpr int GS = TC + 1;
        float* gp = reinterpret_cast<float*>(lb);
#pragma unroll
        for (int m = 0; m < PM; ++m)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int lrow = PM * 16 * wv + 16 * m + 4 * lc + r;
#pragma unroll
                for (int n = 0; n < NT; ++n) gp[lrow * GS + 16 * n + lr] = acc[m][n][r];
            }
        __syncthreads();
        // input rows s0 .. s1 - 1, channels co0 .. co0 + TC - 1: k_conv_fold<true>'s arithmetic
        const int nco = g.Co - co0 < TC ? g.Co - co0 : TC;
        const int n = (s1 - s0) * nco;
        int sl = tid / nco, cl = tid - sl * nco;
        const int ds = 256 / nco, dc = 256 - ds * nco;
        for (int i = tid; i < n; i += 256) {
            const int s = s0 + sl;
            float out = 0.f;
            if (s >= 1) out = fmaf(0.25f, fold_gup(gp, GS, cl, 2 * s - 1, p0, g.pad, g.L_up, g.Lp), out);
            out = fmaf(s == 0 ? 1.f : 0.75f, fold_gup(gp, GS, cl, 2 * s, p0, g.pad, g.L_up, g.Lp), out);
            out = fmaf(s == g.L - 1 ? 1.f : 0.75f, fold_gup(gp, GS, cl, 2 * s + 1, p0, g.pad, g.L_up, g.Lp), out);
            if (2 * s + 2 <= g.L_up - 1)
                out = fmaf(0.25f, fold_gup(gp, GS, cl, 2 * s + 2, p0, g.pad, g.L_up, g.Lp), out);
            dx[((int64_t)b * g.L + s) * g.Co + co0 + cl] = out;
            sl += ds;
            cl += dc;
            if (cl >= nco) {
                cl -= nco;
                ++sl;
            }
        }
    }
}

// UPF: input rows per workgroup.  A tile computes TP padded rows, enough for 2 TS + pad + 2;
// a tile other than the last must not reach the right mirror rows (the last one has >= pad/2 + 1
// rows), and a single tile holds every padded row (2 L + 2 pad <= TP).  -1: no such TS.
static int ups_rows(int L, int pad, int TP) {
    for (int ts = (TP - pad - 2) / 2; ts > pad; --ts) {
        if (L <= ts) {
            if (2 * L + 2 * pad <= TP) return ts;
            continue;
        }
        const int r = L % ts == 0 ? ts : L % ts;
        if (2 * r >= pad + 2) return ts;
    }
    return -1;
}

template <typename H, int K, int NT>
int cbd_nt(const H* d16, BdGeo g, int B, const H* w16t, float* dx, bool upf, hipStream_t st) {
    using C = DCfg<K, NT>;
    const int lds = C::lds_bytes(g.nch, upf);
    if (upf) {
        g.TS = ups_rows(g.L, g.pad, C::TP);
        if (g.TS < 1) return VT_ERR_ARG;
        dim3 grid(cdiv(g.L, g.TS), cdiv(g.Co, C::TC), B);
        hipLaunchKernelGGL((k_cbd16<H, K, NT, true>), grid, dim3(256), lds, st, d16, g, w16t, dx);
    } else if (NT <= 2 && g.p_end - g.p_first <= 256) {
        // short rows (the encoders' L = 256): 128-position tiles, two per sample, every wave
        // busy (a 512-position tile left half of its waves without rows).  Each output's sum
        // over chunks and taps is one lane's, in the same order: the same bits
        using C2 = DCfg<K, NT, 2>;
        dim3 grid(cdiv(g.p_end - g.p_first, C2::TP), cdiv(g.Co, C2::TC), B);
        hipLaunchKernelGGL((k_cbd16<H, K, NT, false, 2>), grid, dim3(256), C2::lds_bytes(g.nch, false), st, d16, g, w16t,
                           dx);
    } else {
        dim3 grid(cdiv(g.p_end - g.p_first, C::TP), cdiv(g.Co, C::TC), B);
        hipLaunchKernelGGL((k_cbd16<H, K, NT, false>), grid, dim3(256), lds, st, d16, g, w16t, dx);
    }
    return VT_OK;
}

template <typename H, int K>
int cbd_k(const H* d16, const BdGeo& g, int B, const H* w16t, float* dx, bool upf, hipStream_t st) {
    switch (cdiv(g.Co, 16) < 6 ? cdiv(g.Co, 16) : 6) {
        case 1: return cbd_nt<H, K, 1>(d16, g, B, w16t, dx, upf, st);
        case 2: return cbd_nt<H, K, 2>(d16, g, B, w16t, dx, upf, st);
        case 3: return cbd_nt<H, K, 3>(d16, g, B, w16t, dx, upf, st);
        case 4: return cbd_nt<H, K, 4>(d16, g, B, w16t, dx, upf, st);
        case 5: return cbd_nt<H, K, 5>(d16, g, B, w16t, dx, upf, st);
        default: return cbd_nt<H, K, 6>(d16, g, B, w16t, dx, upf, st);
    }
}

constexpr int KMAX = 11;

}  // namespace
}  // namespace vt

using namespace vt;

extern "C" {

int vt_batchnorm_bwd_x16(const float* dY, const float* Xc, const float* bnp, int act, int64_t M, int C, void* d16,
                         void* stream) {
    VT_CHECK_ARG(dY && Xc && bnp && d16 && M > 0 && C > 0 && C <= 1024 && act >= 0 && act <= 3,
                 "vt_batchnorm_bwd_x16: arguments");
    const int c32 = cdiv(C, 32) * 32;
    // rows per block: 256 for the narrowest layers (C <= 4: one 64-row block is only 1 KB per
    // stream; measured C = 1, M = 1 M: 19.9 -> 15.1 us), 64 otherwise (C = 32: 5.4 vs 9.4 us);
    // VAETEB_BNX16_ROWS = 64 / 256 forces one (tools/bn_micro.py; the same bits either way)
    static const int xrb_env = getenv("VAETEB_BNX16_ROWS") ? atoi(getenv("VAETEB_BNX16_ROWS")) : 0;
    const int xrb = xrb_env == 256 || xrb_env == 64 ? xrb_env : (C <= 4 ? 256 : 64);
    const size_t lds = (size_t)8 * ((C + 3) & ~3) * 4 + (size_t)xrb * c32 * 2;
    VT_CHECK_ARG(lds <= 160 * 1024, "vt_batchnorm_bwd_x16: C too large");
    // at most 8 workgroups per CU of 64-row blocks, each walking several blocks: the per-workgroup
    // parameter staging (6 C loads + a barrier) is paid once per workgroup, not per block
    // (the same element computation: the same bits)
    const int64_t blocks = (M + xrb - 1) / xrb;
    static const int cap = getenv("VAETEB_BNX16_GRID") ? atoi(getenv("VAETEB_BNX16_GRID")) : 2048;
    const dim3 grid((unsigned)(blocks < cap ? blocks : cap));
    const float invM = 1.f / (float)M;
    hipStream_t st = S(stream);
#define VT_BNX(A, R) hipLaunchKernelGGL((k_bn_bwd_x16<H, A, R>), grid, dim3(256), lds, st, dY, Xc, bnp, M, C, c32, invM, (H*)d16)
    VT_H16(if (xrb == 256) {
        switch (act) {
            case 0: VT_BNX(0, 256); break;
            case 1: VT_BNX(1, 256); break;
            case 2: VT_BNX(2, 256); break;
            default: VT_BNX(3, 256); break;
        }
    } else {
        switch (act) {
            case 0: VT_BNX(0, 64); break;
            case 1: VT_BNX(1, 64); break;
            case 2: VT_BNX(2, 64); break;
            default: VT_BNX(3, 64); break;
        }
    });
#undef VT_BNX
    VT_LAUNCH_CHECK("vt_batchnorm_bwd_x16");
    return VT_OK;
}

int vt_conv1d_bwd_dx16(const void* d16, int B, int L_in, int Cin, const void* w16t, int Cout, int K, int mode, int up,
                       float* dX, float* edge, void* stream) {
    VT_CHECK_ARG(d16 && w16t && dX && B > 0 && B <= 65535 && L_in > 0 && Cin > 0 && Cout > 0 && K > 0 && K <= KMAX &&
                     (mode == 0 || mode == 1) && (up == 0 || up == 1),
                 "vt_conv1d_bwd_dx16: shape (K <= %d)", KMAX);
    const Geo f = geo(B, L_in, Cin, Cout, K, mode, up);
    VT_CHECK_ARG(mode == 1 ? f.L_up > f.pad : !up,
                 "vt_conv1d_bwd_dx16: geometry (reflect needs L_up > pad; causal without upsample)");
    VT_CHECK_ARG(up || mode == 0 || f.pad == 0 || edge, "vt_conv1d_bwd_dx16: reflect padding needs an edge buffer");
    BdGeo g;
    g.Lf = f.L_out;
    g.Ci = Cout;
    g.nch = cdiv(Cout, 32);
    g.Co = Cin;
    g.Lp = f.L_out + K - 1;
    g.pad = f.pad;
    g.L = L_in;
    g.L_up = f.L_up;
    g.TS = 0;
    g.edge = mode == 0 ? nullptr : edge;
    g.p_first = mode == 0 ? f.pad : 0;                 // causal: dX row s = padded row s + pad
    g.p_end = mode == 0 ? f.pad + L_in : g.Lp;
    hipStream_t st = S(stream);
    int rc = VT_ERR_ARG;
    VT_H16(const H* a = (const H*)d16; const H* w = (const H*)w16t;
           switch (K) {
               case 1: rc = cbd_k<H, 1>(a, g, B, w, dX, up, st); break;
               case 2: rc = cbd_k<H, 2>(a, g, B, w, dX, up, st); break;
               case 3: rc = cbd_k<H, 3>(a, g, B, w, dX, up, st); break;
               case 4: rc = cbd_k<H, 4>(a, g, B, w, dX, up, st); break;
               case 5: rc = cbd_k<H, 5>(a, g, B, w, dX, up, st); break;
               case 6: rc = cbd_k<H, 6>(a, g, B, w, dX, up, st); break;
               case 7: rc = cbd_k<H, 7>(a, g, B, w, dX, up, st); break;
               case 8: rc = cbd_k<H, 8>(a, g, B, w, dX, up, st); break;
               case 9: rc = cbd_k<H, 9>(a, g, B, w, dX, up, st); break;
               case 10: rc = cbd_k<H, 10>(a, g, B, w, dX, up, st); break;
               default: rc = cbd_k<H, 11>(a, g, B, w, dX, up, st); break;
           });
    VT_CHECK_ARG(rc == VT_OK, "vt_conv1d_bwd_dx16: tile too small for the upsample fold");
    VT_LAUNCH_CHECK("vt_conv1d_bwd_dx16");
    if (!up && mode == 1 && f.pad > 0) {
        fold_edges_launch(dX, edge, B, L_in, f.pad, Cin, st);
        VT_LAUNCH_CHECK("vt_conv1d_bwd_dx16");
    }
    return VT_OK;
}

}  // extern "C"
