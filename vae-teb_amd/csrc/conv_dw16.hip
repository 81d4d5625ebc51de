// bf16-MFMA weight gradient of the conv blocks (SURVEY.md §8(a) a11, a15;
// ref/model/vae_teb_model.py:128-253 under autograd), split out of conv_bf16.hip (round 5:
// one translation unit per kernel family, so the builds run in parallel).  The staging
// conventions (window padding / x2 upsample via conv.h, the previous block's BatchNorm via
// bnbwd.h for the conv-stack fold) are shared with the forward kernels.
#include <stdlib.h>

#include "conv.h"
#include "h16.h"

namespace vt {

extern int g_conv_kern;   // conv_bf16.hip (vt_conv_bf16_set_kernels)

namespace {

constexpr int KMAXB = 11;

// ------------------------------------------------------------ weight grad
// dW[co][ci][k] = sum_rows dY[row][co] xpad[row + k][ci] on bf16 MFMA: rows
// are the MFMA reduction (32 per k-step).  dY rows and the input window are
// staged row-major in bf16 (fp32 -> bf16 while staging; padding / upsample as
// in the forward) and both operands are read with the gfx950 transposed read
// ds_read_b64_tr_b16 (4 rows x 16 channels per 16-lane group, delivered
// column-major), so the tap shift k is a plain row offset of the window.
// Each wave owns PPW (16 co x 16 ci) tile pairs with K accumulators; NWV waves
// per workgroup (4 or 8: 8 halves the workgroups that stage the same rows when 4
// waves do not cover every pair); rows are split over workgroups
// (blockIdx.y), per-split partial slabs are summed in fixed order by conv.hip's
// k_sum_splits.
typedef short v4i16 __attribute__((ext_vector_type(4)));
constexpr int DWR = 64;  // rows per staged chunk (2 MFMA k-steps)
constexpr int KMAXB_DW = 11;

template <typename H>
__device__ __forceinline__ hv8<H> tr_frag(const H* img, int row0, int col0, int stride) {
    // lane 4q+p of each 16-lane group addresses row (row0 + q), columns col0 + 4p .. +3; two reads
    // (rows +0..3 and +4..7 of the lane group's 8-row block)
    const int lane = threadIdx.x & 63, g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const H* a0 = img + (row0 + 8 * g + q) * stride + col0 + 4 * p;
    const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)a0);
    const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) v4i16*)(a0 + 4 * stride));
    // whole-vector concatenation + bit_cast: element-wise bit_casts of the v4i16 results are
    // miscompiled (each lane's element 0 replicated by v_perm_b32)
    typedef short v8i16 __attribute__((ext_vector_type(8)));
    const v8i16 r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(hv8<H>, r);
}

// DYB: dY given in bf16 (dyb16, row stride dys = ceil8(Cout)), e.g. the BN input
// gradient written by the fused backward-data kernel (k_conv_bf16 BNB + dbf).
// IBN: x is the previous block's pre-BN conv output, its BatchNorm + activation (bi) applied
// while the window is staged (parameters in LDS at byte ipo, channel stride ceil16(Cin))
template <int K, int PPW, bool DYB = false, int NWV = 4, bool IBN = false, typename H = __bf16>
__global__ __launch_bounds__(64 * NWV) void k_conv_dw_bf16(const float* __restrict__ dy, const float* __restrict__ x, Geo g,
                                                      int64_t rows_per_split, int NTc, int npairs, int dstride,
                                                      int xstride, float* __restrict__ part,
                                                      const H* __restrict__ dyb16, int dys, BnIn bi, int ipo) {
    extern __shared__ __attribute__((aligned(16))) char lb_raw[];
    H* const lb = reinterpret_cast<H*>(lb_raw);
    float* ip = reinterpret_cast<float*>(reinterpret_cast<char*>(lb) + ipo);
    const int ics = (g.Cin + 15) / 16 * 16;
    if constexpr (IBN) {
        stage_bn_in(bi, g.Cin, ip, ics);
        __syncthreads();
    }
    H* ds = lb;                          // [DWR][dstride]   dY rows
    H* xs = lb + DWR * dstride;          // [DWR + K - 1 (+pad)][xstride] input window
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lr = lane & 15, lc = lane >> 4;
    int mt[PPW], nt[PPW];
    bool act[PPW];
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
        const int p = blockIdx.x * (NWV * PPW) + wv + NWV * j;
        act[j] = p < npairs;
        mt[j] = act[j] ? p / NTc : 0;
        nt[j] = act[j] ? p - mt[j] * NTc : 0;
    }
    const int64_t rows = (int64_t)g.B * g.L_out;
    const int64_t r0 = (int64_t)blockIdx.y * rows_per_split;
    const int64_t r1 = r0 + rows_per_split < rows ? r0 + rows_per_split : rows;
    f32x4 acc[PPW][K];
#pragma unroll
    for (int j = 0; j < PPW; ++j)
#pragma unroll
        for (int k = 0; k < K; ++k) acc[j][k] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int cout16 = (g.Cout + 15) / 16 * 16, cin16 = (g.Cin + 15) / 16 * 16;
    for (int64_t r = r0; r < r1;) {
        const int b = (int)(r / g.L_out);
        const int t0 = (int)(r - (int64_t)b * g.L_out);
        int n = g.L_out - t0;
        if (n > DWR) n = DWR;
        if (r + n > r1) n = (int)(r1 - r);
        const float* xb = x + (int64_t)b * g.L_in * g.Cin;
        const float* dyb = DYB ? nullptr : dy + ((int64_t)b * g.L_out + t0) * g.Cout;
        // dY rows (zero rows past n, zero channels past Cout), 4 channels per thread-item,
        // and the input window rows t0 .. t0 + DWR + K - 2 (padding / upsample applied,
        // zero past n + K - 1): items in rounds of 4 per thread, every load of a round
        // issued before its stores (clamped addresses, masked values)
        constexpr int UR = K <= 3 ? 1 : (IBN ? 2 : 4);   // small K, input BN: registers (occupancy) first
        const int nd = DWR * (cout16 / 4), nx = (DWR + K - 1) * (cin16 / 4);
        if constexpr (DYB) {
            const H* db16 = dyb16 + ((int64_t)b * g.L_out + t0) * dys;
            typedef short v4s __attribute__((ext_vector_type(4)));
            for (int i0 = tid; i0 < nd; i0 += 64 * NWV * UR) {
                v4s v[UR];
#pragma unroll
                for (int u = 0; u < UR; ++u) {
                    const int i = i0 + 64 * NWV * u;
                    const int t = i / (cout16 / 4), c = 4 * (i - t * (cout16 / 4));
                    const bool ok = i < nd && t < n && c < dys;   // pad channels are 0
                    v[u] = *(const v4s*)(db16 + (int64_t)(ok ? t : 0) * dys + (ok ? c : 0));
                    if (!ok) v[u] = v4s{0, 0, 0, 0};
                }
#pragma unroll
                for (int u = 0; u < UR; ++u) {
                    const int i = i0 + 64 * NWV * u;
                    const int t = i / (cout16 / 4), c = 4 * (i - t * (cout16 / 4));
                    if (i < nd) *(v4s*)(ds + t * dstride + c) = v[u];
                }
            }
        } else {
            for (int i0 = tid; i0 < nd; i0 += 64 * NWV * UR) {
                float v[UR][4];
#pragma unroll
                for (int u = 0; u < UR; ++u) {
                    const int i = i0 + 64 * NWV * u;
                    const int t = i / (cout16 / 4), c = 4 * (i - t * (cout16 / 4));
                    const bool ok = i < nd && t < n;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int cc = c + j < g.Cout ? c + j : g.Cout - 1;
                        v[u][j] = dyb[(int64_t)(ok ? t : 0) * g.Cout + cc];
                        v[u][j] = (ok && c + j < g.Cout) ? v[u][j] : 0.f;
                    }
                }
#pragma unroll
                for (int u = 0; u < UR; ++u) {
                    const int i = i0 + 64 * NWV * u;
                    const int t = i / (cout16 / 4), c = 4 * (i - t * (cout16 / 4));
                    if (i < nd)
#pragma unroll
                        for (int j = 0; j < 4; ++j) ds[t * dstride + c + j] = (H)v[u][j];
                }
            }
        }
        for (int i0 = tid; i0 < nx; i0 += 64 * NWV * UR) {
            float v[UR][4];
#pragma unroll
            for (int u = 0; u < UR; ++u) {
                const int i = i0 + 64 * NWV * u;
                const int t = i / (cin16 / 4), c = 4 * (i - t * (cin16 / 4));
                src_vec<4, IBN>(xb, g, t0 + t, c, i < nx && t < n + K - 1, v[u], ip, ics, bi.act);
            }
#pragma unroll
            for (int u = 0; u < UR; ++u) {
                const int i = i0 + 64 * NWV * u;
                const int t = i / (cin16 / 4), c = 4 * (i - t * (cin16 / 4));
                if (i < nx)
#pragma unroll
                    for (int j = 0; j < 4; ++j) xs[t * xstride + c + j] = (H)v[u][j];
            }
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < DWR / 32; ++s) {
            if (!act[0]) break;  // wave-uniform: a wave without pairs only stages
#pragma unroll
            for (int j = 0; j < PPW; ++j) {
                // no early-out on inactive pairs: the transposed read needs all 64 lanes (EXEC all ones)
                const hv8<H> a = tr_frag<H>(ds, 32 * s, 16 * mt[j], dstride);
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const hv8<H> bb = tr_frag<H>(xs, 32 * s + k, 16 * nt[j], xstride);
                    acc[j][k] = mfma16(a, bb, acc[j][k]);
                }
            }
        }
        __syncthreads();
        r += n;
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
            float* pp = part + ((slot * g.Cout + co) * g.Cin + ci) * K;
#pragma unroll
            for (int k = 0; k < K; ++k) pp[k] = acc[j][k][rr];
        }
    }
}

// The weight gradient with flat staging and a register-prefetched next chunk (round 3;
// vt_conv_bf16_set_kernels bit 1): the MFMA body, pair assignment, splits and 64-row
// chunks of k_conv_dw_bf16<.., DYB = true> (bit-identical partial slabs), the operands
// staged as in conv_fwd16.hip — dY from its bf16 rows by 16-byte loads, the input window's
// source rows copied with float4 loads into LDS (F) and formed into the bf16 image there
// (padding / x2 interpolation by up_lerp, the values of src_vec).  The next chunk's dY
// segments and F rows are loaded into registers before the current chunk's MFMAs.
constexpr int CDW_UD = 4;    // dY 16-byte segments per thread and chunk (256 threads)
constexpr int CDW_UF = 8;    // F float4 per thread and chunk (256 threads)
constexpr int CDW_UF_WIDE = 12;   // ... for the 256-row chunks

// CR: rows per chunk — 64 (DWR), or 256 for the narrow layers (dY <= 32 channels: four times
// the MFMA work per staged chunk, the same k-step order, so the same bits)
// IBN: as k_conv_dw_bf16 (the previous block's BatchNorm + act applied as the window is formed)
template <int K, int PPW, int NWV, int CR = DWR, bool IBN = false, typename H = __bf16>
__global__ __launch_bounds__(64 * NWV) void k_cdw16(const H* __restrict__ dyb16, int dys,
                                                   const float* __restrict__ x, Geo g, int64_t rows_per_split,
                                                   int NTc, int npairs, int dstride, int xstride,
                                                   float* __restrict__ part, int64_t total, BnIn bi, int ipo) {
    constexpr int NT = 64 * NWV;
    constexpr int UD = CR == DWR ? CDW_UD * 256 / NT : CR * 4 / NT;   // CR 256: dY rows of <= 4 segments
    constexpr int UF = CR == DWR ? CDW_UF * 256 / NT : CDW_UF_WIDE * 256 / NT;
    extern __shared__ __attribute__((aligned(16))) char lb_raw[];
    H* const lb = reinterpret_cast<H*>(lb_raw);
    H* ds = lb;                          // [CR][dstride]   dY rows
    H* xs = lb + CR * dstride;           // [CR + K - 1 (+pad)][xstride] input window
    float* F = reinterpret_cast<float*>(lb + CR * dstride + (CR + KMAXB_DW + 8) * xstride);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    int mt[PPW], nt[PPW];
    bool act[PPW];
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
        const int p = blockIdx.x * (NWV * PPW) + wv + NWV * j;
        act[j] = p < npairs;
        mt[j] = act[j] ? p / NTc : 0;
        nt[j] = act[j] ? p - mt[j] * NTc : 0;
    }
    const int64_t rows = (int64_t)g.B * g.L_out;
    const int64_t r0 = (int64_t)blockIdx.y * rows_per_split;
    const int64_t r1 = r0 + rows_per_split < rows ? r0 + rows_per_split : rows;
    f32x4 acc[PPW][K];
#pragma unroll
    for (int j = 0; j < PPW; ++j)
#pragma unroll
        for (int k = 0; k < K; ++k) acc[j][k] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int cout16 = (g.Cout + 15) / 16 * 16, cin16 = (g.Cin + 15) / 16 * 16;
    const int dsegs = cout16 / 8;
    float* ip = reinterpret_cast<float*>(reinterpret_cast<char*>(lb) + ipo);
    if constexpr (IBN) stage_bn_in(bi, g.Cin, ip, cin16);   // read after the first chunk's barrier
    // one chunk's operands into registers: dY segments and the F rows (float4 from the
    // boundary at or below the source run)
    hv8<H> dv[UD];
    float4 fv[UF];
    struct Chunk {
        int b, t0, n, lo, hi, off, nv;
    };
    auto load = [&](int64_t r, Chunk& c) {
        c.b = (int)(r / g.L_out);
        c.t0 = (int)(r - (int64_t)c.b * g.L_out);
        c.n = g.L_out - c.t0 < CR ? g.L_out - c.t0 : CR;
        if (r + c.n > r1) c.n = (int)(r1 - r);
        const H* db = dyb16 + ((int64_t)c.b * g.L_out + c.t0) * dys;
#pragma unroll
        for (int u = 0; u < UD; ++u) {
            const int i = tid + NT * u;
            const int t = i / dsegs, sg = i - t * dsegs;
            const bool ok = i < CR * dsegs && t < c.n && 8 * sg < dys;
            dv[u] = *(const hv8<H>*)(db + (int64_t)(ok ? t : 0) * dys + (ok ? 8 * sg : 0));
            if (!ok) {
#pragma unroll
                for (int j = 0; j < 8; ++j) dv[u][j] = (H)0.f;
            }
        }
        src_span(g, c.t0, c.n + K - 1, c.lo, c.hi);
        const int64_t f0 = ((int64_t)c.b * g.L_in + c.lo) * g.Cin;
        const int64_t fa = f0 & ~(int64_t)3;
        c.off = (int)(f0 - fa);
        const int nf = c.hi >= c.lo ? (int)(((int64_t)c.b * g.L_in + c.hi + 1) * g.Cin - fa) : 0;
        const int nv = (nf + 3) >> 2;
        c.nv = nv;
#pragma unroll
        for (int u = 0; u < UF; ++u) {
            const int i = tid + NT * u;
            const int64_t e = fa + 4 * (int64_t)i;
            if (i < nv && e + 3 < total) {
                fv[u] = *reinterpret_cast<const float4*>(x + e);
            } else {
                fv[u].x = i < nv && e < total ? x[e] : 0.f;
                fv[u].y = i < nv && e + 1 < total ? x[e + 1] : 0.f;
                fv[u].z = i < nv && e + 2 < total ? x[e + 2] : 0.f;
                fv[u].w = 0.f;
            }
        }
    };
    Chunk cur;
    if (r0 < r1) load(r0, cur);
    for (int64_t r = r0; r < r1;) {
        // registers -> LDS: dY rows, F
#pragma unroll
        for (int u = 0; u < UD; ++u) {
            const int i = tid + NT * u;
            if (i < CR * dsegs) {
                const int t = i / dsegs, sg = i - t * dsegs;
                *(hv8<H>*)(ds + t * dstride + 8 * sg) = dv[u];
            }
        }
#pragma unroll
        for (int u = 0; u < UF; ++u)
            if (tid + NT * u < cur.nv) reinterpret_cast<float4*>(F)[tid + NT * u] = fv[u];
        __syncthreads();
        // F -> the bf16 window image (rows t0 .. t0 + CR + K - 2, zero past n + K - 1), 8 channels
        // of one row per item
        {
            const int osegs = cin16 / 8;
            for (int i = tid; i < (CR + K - 1) * osegs; i += NT) {
                const int t = i / osegs, o = i - t * osegs;
                const int tp = cur.t0 + t, cb = 8 * o;
                int i0 = 0, i1 = 0;
                float l1 = 0.f;
                const bool in = t < cur.n + K - 1 && src_row(g, tp, i0, i1, l1);
                const float* p0 = F + cur.off + (in ? i0 - cur.lo : 0) * g.Cin;
                const float* p1 = F + cur.off + (in ? i1 - cur.lo : 0) * g.Cin;
                hv8<H> v;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int c = cb + j < g.Cin ? cb + j : g.Cin - 1;
                    float a = p0[c];
                    float q = g.up ? p1[c] : 0.f;
                    if constexpr (IBN) {
                        a = bn_relu_at(ip, cin16, cb + j, a);
                        q = g.up ? bn_relu_at(ip, cin16, cb + j, q) : 0.f;
                    }
                    v[j] = (H)((in && cb + j < g.Cin) ? (g.up ? up_lerp(a, q, l1) : a) : 0.f);
                }
                *(hv8<H>*)(xs + t * xstride + cb) = v;
            }
        }
        __syncthreads();
        const int64_t rn = r + cur.n;
        Chunk nxt = cur;
        if (rn < r1) load(rn, nxt);   // in flight during the MFMAs
#pragma unroll
        for (int s = 0; s < CR / 32; ++s) {
            if (!act[0]) break;  // wave-uniform: a wave without pairs only stages
#pragma unroll
            for (int j = 0; j < PPW; ++j) {
                const hv8<H> a = tr_frag<H>(ds, 32 * s, 16 * mt[j], dstride);
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const hv8<H> bb = tr_frag<H>(xs, 32 * s + k, 16 * nt[j], xstride);
                    acc[j][k] = mfma16(a, bb, acc[j][k]);
                }
            }
        }
        __syncthreads();
        cur = nxt;
        r = rn;
    }
    const int lr = lane & 15, lc = lane >> 4;
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
            float* pp = part + ((slot * g.Cout + co) * g.Cin + ci) * K;
#pragma unroll
            for (int k = 0; k < K; ++k) pp[k] = acc[j][k][rr];
        }
    }
}

}  // namespace
}  // namespace vt

using namespace vt;

extern "C" {

static int bwd_weight(const float* dY, const float* X, int B, int L_in, int Cin, int Cout, int K, int mode, int up,
                      float* dW, int accumulate, float* ws, int64_t ws_floats, hipStream_t st, const void* dy16,
                      int dys = 0, const BnIn* ibn = nullptr) {
    VT_CHECK_ARG(B > 0 && L_in > 0 && K > 0 && K <= KMAXB && Cin > 0 && Cout > 0 && Cin <= 128 && Cout <= 128,
                 "vt_conv1d_bwd_weight_bf16: shape (K <= %d, channels <= 128)", KMAXB);
    Geo g = geo(B, L_in, Cin, Cout, K, mode, up);
    const int NTc = cdiv(Cin, 16), npairs = cdiv(Cout, 16) * NTc;
    // pairs per wave: at most what the accumulators allow, and no more than the
    // 4 waves of one workgroup need (small layers: no MFMAs on empty pairs)
    const int ppw_max = K <= 3 ? 6 : (K <= 5 ? 4 : (K <= 7 ? 3 : 2));
    const int ppw = cdiv(npairs, 4) < ppw_max ? cdiv(npairs, 4) : ppw_max;
    // waves per workgroup (dy16 path): 8 when 4 do not own every pair, so each row is
    // staged by half as many workgroups (16 waves would cap the accumulators at 128 VGPRs)
    const int need = cdiv(npairs, ppw);
    const int nwv = !dy16 || need <= 4 ? 4 : 8;
    const int bx = cdiv(npairs, nwv * ppw);
    const int64_t rows = (int64_t)B * g.L_out;
    const int64_t nout = (int64_t)Cout * Cin * K;
    // workgroup budget of the row splits (VAETEB_CONVDW_WG, default 8192; measured 4096 -> 8192:
    // 8.80-8.85 -> 8.78-8.79 ms, 1024: 9.2 ms — the weight gradients join the step's end)
    static const int wg_budget = getenv("VAETEB_CONVDW_WG") ? atoi(getenv("VAETEB_CONVDW_WG")) : 8192;
    int64_t splits = (wg_budget > 0 ? wg_budget : 4096) / (nwv * bx);
    if (splits > 1024) splits = 1024;   // the two-stage split sum handles <= 32^2
    if (splits * nout > (int64_t)8 << 20) splits = ((int64_t)8 << 20) / nout;
    if (splits > rows / (4 * DWR)) splits = rows / (4 * DWR);
    if (splits < 1) splits = 1;
    if (splits * nout > ws_floats) splits = ws_floats / nout;
    VT_CHECK_ARG(splits >= 1, "vt_conv1d_bwd_weight_bf16: workspace too small");
    int64_t rps = (rows + splits - 1) / splits;
    splits = (rows + rps - 1) / rps;
    // row strides (bf16): channels rounded to 16, + 8 (rows start 16 B apart mod 64 banks)
    const int dstride = 16 * cdiv(Cout, 16) + 8, xstride = 16 * cdiv(Cin, 16) + 8;
    const size_t lds = (size_t)(DWR * dstride + (DWR + KMAXB + 8) * xstride) * 2;
    if (dys == 0) dys = (Cout + 7) & ~7;
    dim3 grid(bx, (unsigned)splits);
    // flat-staged kernel: F rows of a chunk fit the per-thread prefetch and LDS
    const int f_rows = (up ? (DWR + K - 1) / 2 + 3 : DWR + K - 1);
    const int64_t f_floats = (int64_t)f_rows * Cin + 8;
    // flat-staged weight gradient where it measured faster (K 9 / 7: 176 -> 111, 184 -> 118 us;
    // K <= 5 slower: 85 -> 108 us)
    const bool flat_ok = dy16 && ((uintptr_t)X & 15) == 0 && ((uintptr_t)dy16 & 15) == 0 && dys % 8 == 0;
    const bool flat = flat_ok && (g_conv_kern & 2) && (K >= 7 || (g_conv_kern & 4)) &&
                      f_floats <= (int64_t)4 * CDW_UF * 256 && 16 * cdiv(Cout, 16) <= 8 * CDW_UD * 32;
    const size_t lds_flat = lds + (size_t)f_floats * 4 + 64;
    const int64_t total_x = (int64_t)B * L_in * Cin;
    // 256-row chunks for the narrow layers (dY <= 32 channels, the window's source rows in
    // the wide prefetch): four times the MFMA work per staged chunk (measured: see DESIGN §9)
    const int fw_rows = up ? (256 + K - 1) / 2 + 3 : 256 + K - 1;
    const int64_t fw_floats = (int64_t)fw_rows * Cin + 8;
    const bool wide = flat_ok && (g_conv_kern & 8) && cdiv(Cout, 16) <= 2 &&
                      fw_floats <= (int64_t)4 * CDW_UF_WIDE * 256 && rps >= 256;
    const size_t lds_wide = (size_t)(256 * dstride + (256 + KMAXB + 8) * xstride) * 2 + (size_t)fw_floats * 4 + 64;
    // IBN: the input BatchNorm's parameters after each kernel's LDS ([4][ceil16(Cin)] floats)
    const BnIn bi = ibn ? *ibn : BnIn{};
    const int ib = ibn ? 16 * (16 * cdiv(Cin, 16)) : 0;
    const int ipo_w = ((int)lds_wide + 15) & ~15, ipo_f = ((int)lds_flat + 15) & ~15, ipo_d = ((int)lds + 15) & ~15;
#define VT_DWB_ONE(IB, HT)                                                                                      \
    if (wide && nwv == 8)                                                                                       \
        hipLaunchKernelGGL((k_cdw16<KK, PP, 8, 256, IB, HT>), grid, dim3(512), ipo_w + ib, st, (const HT*)dy16,   \
                           dys, X, g, rps, NTc, npairs, dstride, xstride, ws, total_x, bi, ipo_w);             \
    else if (wide)                                                                                              \
        hipLaunchKernelGGL((k_cdw16<KK, PP, 4, 256, IB, HT>), grid, dim3(256), ipo_w + ib, st, (const HT*)dy16,   \
                           dys, X, g, rps, NTc, npairs, dstride, xstride, ws, total_x, bi, ipo_w);             \
    else if (flat && nwv == 8)                                                                                  \
        hipLaunchKernelGGL((k_cdw16<KK, PP, 8, DWR, IB, HT>), grid, dim3(512), ipo_f + ib, st, (const HT*)dy16,   \
                           dys, X, g, rps, NTc, npairs, dstride, xstride, ws, total_x, bi, ipo_f);             \
    else if (flat)                                                                                              \
        hipLaunchKernelGGL((k_cdw16<KK, PP, 4, DWR, IB, HT>), grid, dim3(256), ipo_f + ib, st, (const HT*)dy16,   \
                           dys, X, g, rps, NTc, npairs, dstride, xstride, ws, total_x, bi, ipo_f);             \
    else if (dy16 && nwv == 8)                                                                                  \
        hipLaunchKernelGGL((k_conv_dw_bf16<KK, PP, true, 8, IB, HT>), grid, dim3(512), ipo_d + ib, st, dY, X, g,  \
                           rps, NTc, npairs, dstride, xstride, ws, (const HT*)dy16, dys, bi, ipo_d);           \
    else if (dy16)                                                                                              \
        hipLaunchKernelGGL((k_conv_dw_bf16<KK, PP, true, 4, IB, HT>), grid, dim3(256), ipo_d + ib, st, dY, X, g,  \
                           rps, NTc, npairs, dstride, xstride, ws, (const HT*)dy16, dys, bi, ipo_d);           \
    else if (!IB)                                                                                               \
        hipLaunchKernelGGL((k_conv_dw_bf16<KK, PP, false, 4, false, HT>), grid, dim3(256), ipo_d, st, dY, X, g,   \
                           rps, NTc, npairs, dstride, xstride, ws, (const HT*)nullptr, 0, bi, ipo_d);
    // fp16 operands (h16.h): the default kernel set; the conv-stack fold (ibn) is bf16-only
    const bool f16 = h16_format() != 0;
    VT_CHECK_ARG(!(f16 && ibn), "vt_conv1d_bwd_weight_bf16_in: the conv-stack fold has no fp16 form");
#define VT_DWB(KK_, PP_)                    \
    if (K == KK_ && ppw == PP_) {           \
        constexpr int KK = KK_, PP = PP_;   \
        if (f16) {                          \
            VT_DWB_ONE(false, _Float16)     \
        } else if (ibn) {                   \
            VT_DWB_ONE(true, __bf16)        \
        } else {                            \
            VT_DWB_ONE(false, __bf16)       \
        }                                   \
    }
#define VT_DWB6(KK) VT_DWB(KK, 1) VT_DWB(KK, 2) VT_DWB(KK, 3) VT_DWB(KK, 4) VT_DWB(KK, 5) VT_DWB(KK, 6)
#define VT_DWB4(KK) VT_DWB(KK, 1) VT_DWB(KK, 2) VT_DWB(KK, 3) VT_DWB(KK, 4)
#define VT_DWB3(KK) VT_DWB(KK, 1) VT_DWB(KK, 2) VT_DWB(KK, 3)
#define VT_DWB2(KK) VT_DWB(KK, 1) VT_DWB(KK, 2)
    VT_DWB6(1) VT_DWB6(2) VT_DWB6(3) VT_DWB4(4) VT_DWB4(5) VT_DWB3(6) VT_DWB3(7)
    VT_DWB2(8) VT_DWB2(9) VT_DWB2(10) VT_DWB2(11)
#undef VT_DWB6
#undef VT_DWB4
#undef VT_DWB3
#undef VT_DWB2
#undef VT_DWB
#undef VT_DWB_ONE
    const int rc = sum_splits_launch(ws, (int)splits, nout, dW, accumulate, st);
    if (rc) return rc;
    VT_LAUNCH_CHECK("vt_conv1d_bwd_weight_bf16");
    return VT_OK;
}

int vt_conv1d_bwd_weight_bf16(const float* dY, const float* X, int B, int L_in, int Cin, int Cout, int K, int mode,
                              int up, float* dW, int accumulate, float* ws, int64_t ws_floats, void* stream) {
    return bwd_weight(dY, X, B, L_in, Cin, Cout, K, mode, up, dW, accumulate, ws, ws_floats, S(stream), nullptr);
}

int vt_conv1d_bwd_weight_bf16_dy16(const void* dY16, const float* X, int B, int L_in, int Cin, int Cout, int K,
                                   int mode, int up, float* dW, int accumulate, float* ws, int64_t ws_floats,
                                   void* stream) {
    VT_CHECK_ARG(dY16 != nullptr, "vt_conv1d_bwd_weight_bf16_dy16: null dY16");
    return bwd_weight(nullptr, X, B, L_in, Cin, Cout, K, mode, up, dW, accumulate, ws, ws_floats, S(stream), dY16);
}

int vt_conv1d_bwd_weight_bf16_dy16s(const void* dY16, int dys, const float* X, int B, int L_in, int Cin, int Cout,
                                    int K, int mode, int up, float* dW, int accumulate, float* ws, int64_t ws_floats,
                                    void* stream) {
    VT_CHECK_ARG(dY16 != nullptr && dys >= ((Cout + 7) & ~7) && dys % 8 == 0,
                 "vt_conv1d_bwd_weight_bf16_dy16s: null dY16 or row stride %d (a multiple of 8 >= ceil8(Cout))", dys);
    return bwd_weight(nullptr, X, B, L_in, Cin, Cout, K, mode, up, dW, accumulate, ws, ws_floats, S(stream),
                      dY16, dys);
}

// the weight gradient of a block whose input is the previous block's pre-BN conv output X
// (its BatchNorm + activation applied as the window is staged); dY16 (bf16, row stride dys)
// or dY (fp32, dY16 == nullptr)
int vt_conv1d_bwd_weight_bf16_in(const float* dY, const void* dY16, int dys, const float* X, const float* in_mean,
                                 const float* in_rstd, const float* in_gamma, const float* in_beta, int in_act, int B,
                                 int L_in, int Cin, int Cout, int K, int mode, int up, float* dW, int accumulate,
                                 float* ws, int64_t ws_floats, void* stream) {
    VT_CHECK_ARG(in_mean && in_rstd && in_gamma && in_beta && in_act == 1,
                 "vt_conv1d_bwd_weight_bf16_in: input BatchNorm parameters (ReLU blocks only)");
    VT_CHECK_ARG(dY16 && dys >= ((Cout + 7) & ~7) && dys % 8 == 0,
                 "vt_conv1d_bwd_weight_bf16_in: bf16 dY16 (row stride %d) required", dys);
    (void)dY;
    const BnIn bi{in_mean, in_rstd, in_gamma, in_beta, in_act};
    return bwd_weight(dY, X, B, L_in, Cin, Cout, K, mode, up, dW, accumulate, ws, ws_floats, S(stream),
                      dY16, dY16 ? dys : 0, &bi);
}

}  // extern "C"
