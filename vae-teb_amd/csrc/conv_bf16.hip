// bf16-MFMA 1-D convolution for the conv blocks (SURVEY.md §8(a) a11, a15;
// ref/model/vae_teb_model.py:128-253) in the reference's training precision:
// the reference trains in fp16 autocast (bf16 here: DESIGN.md §5; Lightning precision="16-mixed",
// ref/model/graph_model.py:510; torch.amp.autocast, :709-711), i.e. conv
// operands in 16 bits with fp32 accumulation.  Here: bf16 operands on
// v_mfma_f32_16x16x32_bf16 (16x the fp32 MFMA rate), fp32 accumulation, fp32
// activations in HBM (the window is converted while it is staged), BatchNorm
// statistics / apply in fp32 exactly as on the fp32 path.
//
// Same implicit GEMM as conv.hip's k_conv_fwd: a workgroup (4 waves) owns
// (sample, TP output positions, TC = 16*NT output channels); per chunk of 32
// input channels it stages the input window (padding / x2 upsample applied,
// -> bf16) and the chunk's taps (from a bf16 weight shadow laid out
// [out][K][in32], one 16-byte row segment per load), then one MFMA k-step per
// tap: lane group lc takes input channels 8*lc .. 8*lc+7 of the chunk, so a
// fragment is one ds_read_b128 of a window row (shifted by the tap) or a tap
// row.  Rows are 40 bf16 (20 dwords) apart: 16 consecutive rows hit 16
// distinct 4-bank groups.  Backward-data is the same kernel on dY with the
// transposed / flipped shadow (causal padding K-1), as in conv.hip.
#include <stdlib.h>

#include "conv.h"
#include "h16.h"

namespace vt {

// kernel selection (vt_conv_bf16_set_kernels): bit 0 the flat-staged forward (conv_fwd16.hip),
// bit 1 the flat-staged weight gradient (k_cdw16, conv_dw16.hip), bit 2 both at every K, bit 3
// 256-row chunks in the flat weight gradient for dY <= 32 channels
int g_conv_kern = 11;

namespace {

constexpr int CB = 32;   // input channels per staged chunk (= one MFMA k-step)
constexpr int RS = 40;   // bf16 row stride of window and tap rows

template <int K, int NT>
struct BCfg {
    static constexpr int PM = NT <= 2 ? 4 : 2;                  // position tiles per wave
    static constexpr int TC = 16 * NT, TP = 64 * PM, WIN = TP + K - 1;
    static constexpr int XB = WIN * RS, WB = K * TC * RS;       // bf16 elements
    static constexpr int LDS_BYTES = (XB + WB) * 2 > 8 * TC * 4 ? (XB + WB) * 2 : 8 * TC * 4;
};

// Backward-data output written straight into dX (no padded gpad pass + fold):
// padded row t goes to dX row t - pad when it lies in [0, L), to edge row t (t < pad)
// or t - L (t >= pad + L) otherwise (reflect padding: k_conv_fold_edges adds those
// back); pad < 0: the plain [B][Lo] output.
struct FoldOut {
    int pad, L;
    float* edge;   // nullable: the edge rows are dropped (causal padding)
};

template <typename H>
__device__ __forceinline__ hv8<H> pack8(const float (&v)[8]) {
    hv8<H> r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (H)v[j];
    return r;
}

// Window staging with lanes along channels (the default; g_conv_cl): thread t stages
// channel c0 + (t & 31) of rows (t >> 5) + 8 i, so a wave-instruction reads two
// 128-B row segments (2-4 cache lines) instead of 4 channels in each of 16 rows, and
// the BatchNorm-backward parameters of its one channel sit in registers.  U rows per
// round, all their loads issued before the first use.  Same values and the same bf16
// roundings as the octet staging below (bit-identical results).
template <typename H, int K, int WIN, bool BNB, bool IBN = false>
__device__ __forceinline__ void stage_window_cl(H* __restrict__ xs, const float* __restrict__ xb,
                                                const float* __restrict__ x2b, const Geo& g, int t0, int TP, int Lo,
                                                int c0, const float* __restrict__ bp, int act, float invM,
                                                H* __restrict__ dbf, int b, bool write_dbf,
                                                const float* ip = nullptr, int ics = 0, int iact = 0) {
    constexpr int NR = (WIN + 7) / 8, U = K <= 3 ? 3 : 6;
    const int tid = threadIdx.x, cl = tid & 31, rg = tid >> 5;
    const int c = c0 + cl;
    const bool cok = c < g.Cin;
    const int cc = cok ? c : 0;
    float pm = 0.f, prs = 0.f, pga = 0.f, pbe = 0.f, pdg = 0.f, pdb = 0.f;
    if constexpr (BNB) {
        pm = bp[cc];
        prs = bp[g.Cin + cc];
        pga = bp[2 * g.Cin + cc];
        pbe = bp[3 * g.Cin + cc];
        pdg = bp[4 * g.Cin + cc];
        pdb = bp[5 * g.Cin + cc];
    }
    const int cpad = (g.Cin + 7) & ~7;
#pragma unroll
    for (int i0 = 0; i0 < NR; i0 += U) {
        float a[U], q[U], l1[U];
        bool ok[U], rok[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int r = rg + 8 * (i0 + u);
            const int tp = t0 + r;
            const bool rin = i0 + u < NR && r < WIN && tp < Lo + K - 1 && cok;
            if constexpr (BNB) {
                const int t = tp - g.pad;   // causal geometry: zero outside [0, L_in)
                rok[u] = i0 + u < NR && r < WIN && tp < Lo + K - 1 && t >= 0 && t < g.L_in;
                ok[u] = rin && t >= 0 && t < g.L_in;
                const int64_t off = ok[u] ? (int64_t)t * g.Cin + c : 0;
                a[u] = xb[off];
                q[u] = x2b[off];
                l1[u] = 0.f;
            } else {
                int i0r = 0, i1r = 0;
                float w1 = 0.f;
                rok[u] = false;
                ok[u] = rin && src_row(g, tp, i0r, i1r, w1);
                a[u] = xb[ok[u] ? (int64_t)i0r * g.Cin + c : 0];
                q[u] = g.up ? xb[ok[u] ? (int64_t)i1r * g.Cin + c : 0] : 0.f;
                l1[u] = w1;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int r = rg + 8 * (i0 + u);
            if (i0 + u >= NR || r >= WIN) continue;
            float v = 0.f;
            if (ok[u]) {
                if constexpr (BNB) {
                    v = bn_bwd_val_r(a[u], q[u], pm, prs, pga, pbe, pdg, pdb, act, invM);
                } else if constexpr (IBN) {
                    const float av = bn_relu_at(ip, ics, cc, a[u]);
                    v = g.up ? up_lerp(av, bn_relu_at(ip, ics, cc, q[u]), l1[u]) : av;
                } else {
                    v = g.up ? up_lerp(a[u], q[u], l1[u]) : a[u];
                }
            }
            xs[r * RS + cl] = (H)v;
            if constexpr (BNB) {
                // the bf16 side output: the row's channels and its zero channel padding up to cpad
                const int t = t0 + r - g.pad;
                if (write_dbf && rok[u] && c < cpad && t >= t0 && t < t0 + TP)
                    dbf[((int64_t)b * g.L_in + t) * cpad + c] = (H)v;
            }
        }
    }
}

// window staging (vt_conv_bf16_set_staging): 0 octets per lane, 2 lanes along channels everywhere,
// 1 (default) lanes along channels for the fused-BN backward-data kernels with K >= 7 only —
// measured in isolation (tools/conv_micro.py): K 11 / 9 / 7 BNB 98 / 91 / 105 -> 82 / 82 / 92 us,
// but the forward and every K = 3 instance slower (K 3 BNB 32 -> 260 us: 11-33 channel rows
// leave most of the 32 channel lanes idle)
int g_conv_cl = 1;

// x: fp32 (B, L_in, g.Cin) activations; w16: [g.Cout][K][cin32] bf16 shadow.
// BNB (backward-data only: causal geometry, no upsample): x is the block output
// gradient dy and the staged operand is the BatchNorm input gradient computed on
// the fly from dy, the pre-BN conv output x2 and bnp (conv.h bn_bwd_val).
// dbf (BNB, nullable): the staged BN input gradient, bf16, is also written to
// dbf[(b L_in + t) cpad + c] (cpad = ceil8(Cin)) by the blockIdx.y == 0 workgroups
// for their own rows t0 .. t0 + TP - 1 (each row once) — the weight gradient's operand.
// IBN (not with BNB): x is the previous block's pre-BN conv output, its BatchNorm + activation
// (bi, staged into LDS at byte ipo) applied to the source samples while the window is staged.
template <int K, int NT, bool BNB = false, bool CL = true, bool IBN = false, typename H = __bf16>
__global__ __launch_bounds__(256) void k_conv_bf16(const float* __restrict__ x, Geo g, const H* __restrict__ w16,
                                                   int cin32, float* __restrict__ y, int Lo,
                                                   float* __restrict__ stats, const float* __restrict__ x2,
                                                   const float* __restrict__ bnp, int act, float invM,
                                                   H* __restrict__ dbf, FoldOut fo, BnIn bi, int ipo) {
    static_assert(!(BNB && IBN), "k_conv_bf16: BNB and IBN exclusive");
    using C = BCfg<K, NT>;
    constexpr int PM = C::PM, TC = C::TC, TP = C::TP, WIN = C::WIN;
    extern __shared__ __attribute__((aligned(16))) char lb_raw[];
    H* const lb = reinterpret_cast<H*>(lb_raw);
    H* xs = lb;           // [WIN][RS]
    H* ws = lb + C::XB;   // [K][TC][RS]
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lr = lane & 15, lc = lane >> 4;
    const int t0 = blockIdx.x * TP, co0 = blockIdx.y * TC, b = blockIdx.z;
    const float* xb = x + (int64_t)b * g.L_in * g.Cin;
    float* bp = reinterpret_cast<float*>(reinterpret_cast<char*>(lb) + C::LDS_BYTES);  // BNB: 6 x Cin params
    if constexpr (BNB) {
        for (int i = tid; i < 6 * g.Cin; i += 256) bp[i] = bnp[i];
        __syncthreads();
    }
    float* ip = reinterpret_cast<float*>(reinterpret_cast<char*>(lb) + ipo);
    if constexpr (IBN) {
        stage_bn_in(bi, g.Cin, ip, cin32);
        __syncthreads();
    }
    const float* x2b = BNB ? x2 + (int64_t)b * g.L_in * g.Cin : nullptr;
    f32x4 acc[PM][NT];
#pragma unroll
    for (int m = 0; m < PM; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int c0 = 0; c0 < g.Cin; c0 += CB) {
        if constexpr (CL) {
            // taps (K x TC rows x 4 octets, 16 B each from the shadow): loads first, stores
            // after the window
            constexpr int NWI = (K * TC * 4 + 255) / 256;
            hv8<H> wt[NWI];
#pragma unroll
            for (int it = 0; it < NWI; ++it) {
                const int i = tid + 256 * it;
                const int ic = i < K * TC * 4 ? i : K * TC * 4 - 1;
                const int oct = ic & 3, r = ic >> 2, k = r / TC, co = r - k * TC;
                const int coc = co0 + co < g.Cout ? co0 + co : g.Cout - 1;
                wt[it] = *(const hv8<H>*)(w16 + ((int64_t)coc * K + k) * cin32 + c0 + 8 * oct);
            }
            stage_window_cl<H, K, WIN, BNB, IBN>(xs, xb, x2b, g, t0, TP, Lo, c0, bp, act, invM, dbf, b,
                                              BNB && dbf && blockIdx.y == 0, ip, cin32, bi.act);
#pragma unroll
            for (int it = 0; it < NWI; ++it) {
                const int i = tid + 256 * it;
                if (i >= K * TC * 4) continue;
                const int oct = i & 3, r = i >> 2, k = r / TC, co = r - k * TC;
                hv8<H> val = wt[it];
                if (co0 + co >= g.Cout) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) val[j] = (H)0.f;
                }
                *(hv8<H>*)(ws + (k * TC + co) * RS + 8 * oct) = val;
            }
        } else if constexpr (K <= 3) {
            // small K (few taps, little MFMA work per staged row): the per-element staging
            // keeps the register count, and with it the occupancy, low (measured faster)
            for (int i = tid; i < WIN * 4; i += 256) {
                const int row = i >> 2, oct = i & 3;
                const int tp = t0 + row, cb = c0 + 8 * oct;
                float v[8];
                const bool ok = tp < Lo + K - 1;
                if constexpr (BNB) {
                    const int t = tp - g.pad;   // causal geometry: zero outside [0, L_in)
                    const bool in = ok && t >= 0 && t < g.L_in;
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int c = cb + j;
                        v[j] = (in && c < g.Cin) ? bn_bwd_val(xb[(int64_t)t * g.Cin + c], x2b[(int64_t)t * g.Cin + c],
                                                               bp, g.Cin, c, act, invM)
                                                 : 0.f;
                    }
                    if (dbf && blockIdx.y == 0 && in && t >= t0 && t < t0 + TP && cb < g.Cin) {
                        const int cpad = (g.Cin + 7) & ~7;
                        *(hv8<H>*)(dbf + ((int64_t)b * g.L_in + t) * cpad + cb) = pack8<H>(v);
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        v[j] = (ok && cb + j < g.Cin) ? src_val<IBN>(xb, g, tp, cb + j, ip, cin32, bi.act) : 0.f;
                }
                *(hv8<H>*)(xs + row * RS + 8 * oct) = pack8<H>(v);
            }
            for (int i = tid; i < K * TC * 4; i += 256) {
                const int oct = i & 3, r = i >> 2, k = r / TC, co = r - k * TC;
                hv8<H> val;
                if (co0 + co < g.Cout) {
                    val = *(const hv8<H>*)(w16 + ((int64_t)(co0 + co) * K + k) * cin32 + c0 + 8 * oct);
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) val[j] = (H)0.f;
                }
                *(hv8<H>*)(ws + (k * TC + co) * RS + 8 * oct) = val;
            }
        } else {
            // window: WIN rows x 4 octets of 8 channels, fp32 -> bf16, and the chunk's taps
            // (K x TC rows x 4 octets, 16 B each from the shadow): every load of the thread
            // issued before the first store (clamped addresses, masked values)
            constexpr int NI = (WIN * 4 + 255) / 256, NWI = (K * TC * 4 + 255) / 256;
            hv8<H> wt[NWI];
    #pragma unroll
            for (int it = 0; it < NWI; ++it) {
                const int i = tid + 256 * it;
                const int ic = i < K * TC * 4 ? i : K * TC * 4 - 1;
                const int oct = ic & 3, r = ic >> 2, k = r / TC, co = r - k * TC;
                const int coc = co0 + co < g.Cout ? co0 + co : g.Cout - 1;
                wt[it] = *(const hv8<H>*)(w16 + ((int64_t)coc * K + k) * cin32 + c0 + 8 * oct);
            }
            // window items in rounds of NB (all loads of a round in flight together)
            constexpr int NB = BNB ? (NI < 2 ? NI : 2) : (NI < 3 ? NI : 3);
    #pragma unroll
            for (int r0 = 0; r0 < NI; r0 += NB) {
            float v[NB][8];
    #pragma unroll
            for (int it = 0; it < NB; ++it) {
                const int i = tid + 256 * (r0 + it);
                const int row = i >> 2, oct = i & 3;
                const int tp = t0 + row, cb = c0 + 8 * oct;
                const bool ok = r0 + it < NI && i < WIN * 4 && tp < Lo + K - 1;
                if constexpr (BNB) {
                    const int t = tp - g.pad;   // causal geometry: zero outside [0, L_in)
                    const bool in = ok && t >= 0 && t < g.L_in;
                    const int64_t ro = (int64_t)(in ? t : 0) * g.Cin;
                    float xa[8], xq[8];
    #pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int c = cb + j < g.Cin ? cb + j : g.Cin - 1;
                        xa[j] = xb[ro + c];
                        xq[j] = x2b[ro + c];
                    }
    #pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int c = cb + j < g.Cin ? cb + j : g.Cin - 1;
                        v[it][j] = (in && cb + j < g.Cin) ? bn_bwd_val(xa[j], xq[j], bp, g.Cin, c, act, invM) : 0.f;
                    }
                    if (dbf && blockIdx.y == 0 && in && t >= t0 && t < t0 + TP && cb < g.Cin) {
                        const int cpad = (g.Cin + 7) & ~7;   // cb < Cin and cb % 8 == 0: the octet fits the padded row
                        *(hv8<H>*)(dbf + ((int64_t)b * g.L_in + t) * cpad + cb) = pack8<H>(v[it]);
                    }
                } else {
                    src_vec<8, IBN>(xb, g, tp, cb, ok, v[it], ip, cin32, bi.act);
                }
            }
    #pragma unroll
            for (int it = 0; it < NB; ++it) {
                const int i = tid + 256 * (r0 + it);
                if (r0 + it < NI && i < WIN * 4) *(hv8<H>*)(xs + (i >> 2) * RS + 8 * (i & 3)) = pack8<H>(v[it]);
            }
            }
    #pragma unroll
            for (int it = 0; it < NWI; ++it) {
                const int i = tid + 256 * it;
                if (i >= K * TC * 4) continue;
                const int oct = i & 3, r = i >> 2, k = r / TC, co = r - k * TC;
                hv8<H> val = wt[it];
                if (co0 + co >= g.Cout) {
    #pragma unroll
                    for (int j = 0; j < 8; ++j) val[j] = (H)0.f;
                }
                *(hv8<H>*)(ws + (k * TC + co) * RS + 8 * oct) = val;
            }
        }
        __syncthreads();
        const H* xq = xs + (PM * 16 * wv + lr) * RS + 8 * lc;
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
    }
    // D layout: col (channel) = lane & 15, row (position) = 4 * (lane >> 4) + r
#pragma unroll
    for (int m = 0; m < PM; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int t = t0 + PM * 16 * wv + 16 * m + 4 * lc + r;
            if (t >= Lo) continue;
            float* yr = y + ((int64_t)b * Lo + t) * g.Cout;
            if (fo.pad >= 0) {
                const int sx = t - fo.pad;
                if (sx >= 0 && sx < fo.L) yr = y + ((int64_t)b * fo.L + sx) * g.Cout;
                else if (fo.edge) yr = fo.edge + ((int64_t)b * 2 * fo.pad + (sx < 0 ? t : t - fo.L)) * g.Cout;
                else continue;
            }
#pragma unroll
            for (int n = 0; n < NT; ++n) {
                const int co = co0 + 16 * n + lr;
                if (co < g.Cout) yr[co] = acc[m][n][r];
            }
        }
    if (stats) {
        // BatchNorm tile statistics, as conv.hip k_conv_fwd
        float* red1 = reinterpret_cast<float*>(lb);  // [4][TC]
        float* red2 = red1 + 4 * TC;                 // [4][TC]
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

// bf16 shadows of W [Cout][Cin][K]: w16 [Cout][K][cin32] (forward) and
// w16t [Cin][K][cout32] = W[co][ci][K-1-k] (backward-data), zero-padded.
template <typename H>
__global__ void k_conv_shadow(const float* __restrict__ W, int Cout, int Cin, int K, int cin32, int cout32,
                              H* __restrict__ w16, H* __restrict__ w16t) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n1 = (int64_t)Cout * K * cin32;
    if (i < n1) {
        const int ci = (int)(i % cin32);
        const int64_t r = i / cin32;
        const int k = (int)(r % K), co = (int)(r / K);
        w16[i] = (H)(ci < Cin ? W[((int64_t)co * Cin + ci) * K + k] : 0.f);
    } else if (i < n1 + (int64_t)Cin * K * cout32) {
        const int64_t j = i - n1;
        const int co = (int)(j % cout32);
        const int64_t r = j / cout32;
        const int k = (int)(r % K), ci = (int)(r / K);
        w16t[j] = (H)(co < Cout ? W[((int64_t)co * Cin + ci) * K + (K - 1 - k)] : 0.f);
    }
}

// Every bf16 conv weight's shadows in one launch (after the optimizer step, off the next
// forward's chain): workgroup b -> (weight, 256-element block) by prefix sums; the same
// element mapping as k_conv_shadow (the same bits).
constexpr int CSB_MAX = 24;
struct ConvShadowBatch {
    int n;
    const float* W[CSB_MAX];
    int Cout[CSB_MAX], Cin[CSB_MAX], K[CSB_MAX];
    void* w16[CSB_MAX];
    void* w16t[CSB_MAX];
    int prefix[CSB_MAX + 1];   // workgroups
};
template <typename H>
__global__ __launch_bounds__(256) void k_conv_shadow_batch(ConvShadowBatch cb) {
    int h = 0;
    while (h + 1 < cb.n && (int)blockIdx.x >= cb.prefix[h + 1]) ++h;
    const int Cout = cb.Cout[h], Cin = cb.Cin[h], K = cb.K[h];
    const int cin32 = (Cin + 31) / 32 * 32, cout32 = (Cout + 31) / 32 * 32;
    const int64_t i = (int64_t)(blockIdx.x - cb.prefix[h]) * 256 + threadIdx.x;
    const float* W = cb.W[h];
    const int64_t n1 = (int64_t)Cout * K * cin32;
    if (i < n1) {
        const int ci = (int)(i % cin32);
        const int64_t r = i / cin32;
        const int k = (int)(r % K), co = (int)(r / K);
        reinterpret_cast<H*>(cb.w16[h])[i] = (H)(ci < Cin ? W[((int64_t)co * Cin + ci) * K + k] : 0.f);
    } else if (i < n1 + (int64_t)Cin * K * cout32) {
        const int64_t j = i - n1;
        const int co = (int)(j % cout32);
        const int64_t r = j / cout32;
        const int k = (int)(r % K), ci = (int)(r / K);
        reinterpret_cast<H*>(cb.w16t[h])[j] = (H)(co < Cout ? W[((int64_t)co * Cin + ci) * K + (K - 1 - k)] : 0.f);
    }
}

// BatchNorm-backward staging (k_conv_bf16 / k_conv_dw_bf16 BNB): dy, the pre-BN
// conv output, the packed per-channel parameters (6 x C), activation and 1/M
struct BnB {
    const float* x2;
    const float* bnp;
    int act;
    float invM;
    void* dbf;     // nullable: bf16 copy of the BN input gradient (the weight gradient's operand)
};

template <int K, int NT>
int bf_nt(const float* x, const Geo& g, const void* w16v, int cin32, float* y, int Lo, float* stats,
          hipStream_t st, const BnB* bn, FoldOut fo, const BnIn* ibn) {
    using C = BCfg<K, NT>;
    if (x && h16_format()) {
        // fp16 operands (h16.h): the default kernel set only — the plain forward / backward-data
        // conv; the fused-BN backward staging and the conv-stack fold are bf16-only A/B paths
        if (bn || ibn) {
            set_error("conv bf16: the fused BatchNorm staging / conv-stack fold paths have no fp16 form");
            return VT_ERR_ARG;
        }
        if ((g_conv_kern & 1) && (K <= 5 || (g_conv_kern & 4)) && fo.pad < 0 && ((uintptr_t)x & 15) == 0) {
            const int tp = cfw16_launch(x, g, w16v, y, Lo, stats, st, nullptr);
            if (tp > 0) return tp;
        }
        dim3 grid(cdiv(Lo, C::TP), cdiv(g.Cout, C::TC), g.B);
        const _Float16* w16 = (const _Float16*)w16v;
        if (g_conv_cl == 2)
            hipLaunchKernelGGL((k_conv_bf16<K, NT, false, true, false, _Float16>), grid, dim3(256), C::LDS_BYTES, st, x,
                               g, w16, cin32, y, Lo, stats, nullptr, nullptr, 0, 0.f, nullptr, fo, BnIn{}, 0);
        else
            hipLaunchKernelGGL((k_conv_bf16<K, NT, false, false, false, _Float16>), grid, dim3(256), C::LDS_BYTES, st,
                               x, g, w16, cin32, y, Lo, stats, nullptr, nullptr, 0, 0.f, nullptr, fo, BnIn{}, 0);
        return C::TP;
    }
    const __bf16* w16 = (const __bf16*)w16v;
    // flat-staged forward where it measured faster than k_conv_bf16 (isolated, decoder
    // geometry: K 5 / 3 layers 60 -> 52, 102 -> 60 us; K >= 7 slower: 30 -> 43 us at K 11)
    if (x && !bn && (g_conv_kern & 1) && (K <= 5 || (g_conv_kern & 4)) && fo.pad < 0 && ((uintptr_t)x & 15) == 0) {
        const int tp = cfw16_launch(x, g, w16, y, Lo, stats, st, ibn);
        if (tp > 0) return tp;
    }
    dim3 grid(cdiv(Lo, C::TP), cdiv(g.Cout, C::TC), g.B);
    const bool cl = g_conv_cl == 2 || (g_conv_cl == 1 && bn && K >= 7);
    const BnIn bi = ibn ? *ibn : BnIn{};
    const int ipo = C::LDS_BYTES, ilds = C::LDS_BYTES + 16 * cin32;   // IBN: [4][cin32] parameters
    if (x && bn && cl)
        hipLaunchKernelGGL((k_conv_bf16<K, NT, true, true, false, __bf16>), grid, dim3(256), C::LDS_BYTES + 24 * g.Cin, st, x, g, w16,
                           cin32, y, Lo, stats, bn->x2, bn->bnp, bn->act, bn->invM, (__bf16*)bn->dbf, fo, bi, 0);
    else if (x && bn)
        hipLaunchKernelGGL((k_conv_bf16<K, NT, true, false, false, __bf16>), grid, dim3(256), C::LDS_BYTES + 24 * g.Cin, st, x, g,
                           w16, cin32, y, Lo, stats, bn->x2, bn->bnp, bn->act, bn->invM, (__bf16*)bn->dbf, fo, bi, 0);
    else if (x && cl && ibn)
        hipLaunchKernelGGL((k_conv_bf16<K, NT, false, true, true, __bf16>), grid, dim3(256), ilds, st, x, g, w16, cin32, y,
                           Lo, stats, nullptr, nullptr, 0, 0.f, nullptr, fo, bi, ipo);
    else if (x && cl)
        hipLaunchKernelGGL((k_conv_bf16<K, NT, false, true, false, __bf16>), grid, dim3(256), C::LDS_BYTES, st, x, g, w16, cin32, y,
                           Lo, stats, nullptr, nullptr, 0, 0.f, nullptr, fo, bi, 0);
    else if (x && ibn)
        hipLaunchKernelGGL((k_conv_bf16<K, NT, false, false, true, __bf16>), grid, dim3(256), ilds, st, x, g, w16, cin32, y,
                           Lo, stats, nullptr, nullptr, 0, 0.f, nullptr, fo, bi, ipo);
    else if (x)
        hipLaunchKernelGGL((k_conv_bf16<K, NT, false, false, false, __bf16>), grid, dim3(256), C::LDS_BYTES, st, x, g, w16, cin32, y,
                           Lo, stats, nullptr, nullptr, 0, 0.f, nullptr, fo, bi, 0);
    return C::TP;
}

template <int K>
int bf_k(const float* x, const Geo& g, const void* w16, int cin32, float* y, int Lo, float* stats, hipStream_t st,
         const BnB* bn, FoldOut fo, const BnIn* ibn) {
    switch (cdiv(g.Cout, 16) < 6 ? cdiv(g.Cout, 16) : 6) {
        case 1: return bf_nt<K, 1>(x, g, w16, cin32, y, Lo, stats, st, bn, fo, ibn);
        case 2: return bf_nt<K, 2>(x, g, w16, cin32, y, Lo, stats, st, bn, fo, ibn);
        case 3: return bf_nt<K, 3>(x, g, w16, cin32, y, Lo, stats, st, bn, fo, ibn);
        case 4: return bf_nt<K, 4>(x, g, w16, cin32, y, Lo, stats, st, bn, fo, ibn);
        case 5: return bf_nt<K, 5>(x, g, w16, cin32, y, Lo, stats, st, bn, fo, ibn);
        default: return bf_nt<K, 6>(x, g, w16, cin32, y, Lo, stats, st, bn, fo, ibn);
    }
}

// x == nullptr: no launch, only the position tile of this geometry
int bf_launch(const float* x, const Geo& g, const void* w16, int cin32, float* y, int Lo, float* stats,
              hipStream_t st, const BnB* bn = nullptr, FoldOut fo = FoldOut{-1, 0, nullptr},
              const BnIn* ibn = nullptr) {
    switch (g.K) {
        case 1: return bf_k<1>(x, g, w16, cin32, y, Lo, stats, st, bn, fo, ibn);
        case 2: return bf_k<2>(x, g, w16, cin32, y, Lo, stats, st, bn, fo, ibn);
        case 3: return bf_k<3>(x, g, w16, cin32, y, Lo, stats, st, bn, fo, ibn);
        case 4: return bf_k<4>(x, g, w16, cin32, y, Lo, stats, st, bn, fo, ibn);
        case 5: return bf_k<5>(x, g, w16, cin32, y, Lo, stats, st, bn, fo, ibn);
        case 6: return bf_k<6>(x, g, w16, cin32, y, Lo, stats, st, bn, fo, ibn);
        case 7: return bf_k<7>(x, g, w16, cin32, y, Lo, stats, st, bn, fo, ibn);
        case 8: return bf_k<8>(x, g, w16, cin32, y, Lo, stats, st, bn, fo, ibn);
        case 9: return bf_k<9>(x, g, w16, cin32, y, Lo, stats, st, bn, fo, ibn);
        case 10: return bf_k<10>(x, g, w16, cin32, y, Lo, stats, st, bn, fo, ibn);
        default: return bf_k<11>(x, g, w16, cin32, y, Lo, stats, st, bn, fo, ibn);
    }
}

// reflect padding without upsampling: the mirrored padded rows (edge, see FoldOut)
// added onto dX rows 1 .. pad and max(0, L - 1 - pad) .. L - 2, in the order of gemm.hip's
// k_conv_fold (direct, left mirror, right mirror: the same bits)
__global__ void k_conv_fold_edges(float* __restrict__ dx, const float* __restrict__ edge, int L, int pad, int C) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;   // (row slot, channel) within sample blockIdx.y
    if (i >= 2 * pad * C) return;
    const int r = i / C, c = i - r * C, b = blockIdx.y;
    const int s = r < pad ? 1 + r : L - 1 - pad + (r - pad);
    // left set: rows 1 .. pad; right set: rows L - 1 - pad .. L - 2 (row 0 included when L <= pad + 1),
    // its rows inside 1 .. pad already handled by the left set
    if (s < 0 || s > L - 1 || (r < pad && s < 1) || (r >= pad && s >= 1 && s <= pad)) return;
    const float* eb = edge + (int64_t)b * 2 * pad * C + c;
    float* o = dx + ((int64_t)b * L + s) * C + c;
    float v = *o;
    if (s >= 1 && s <= pad) v += eb[(pad - s) * C];              // left mirror: padded row pad - s
    const int tr = pad + 2 * (L - 1) - s;                        // right mirror: padded row tr
    if (s <= L - 2 && tr < L + 2 * pad && tr >= pad + L) v += eb[(tr - L) * C];
    *o = v;
}

constexpr int KMAXB = 11;

}  // namespace

void fold_edges_launch(float* dx, const float* edge, int B, int L, int pad, int C, hipStream_t st) {
    hipLaunchKernelGGL(k_conv_fold_edges, dim3((unsigned)((2 * pad * C + 255) / 256), (unsigned)B), dim3(256), 0, st,
                       dx, edge, L, pad, C);
}
}  // namespace vt

using namespace vt;

extern "C" {

int vt_conv_bf16_set_staging(int mode) {
    VT_CHECK_ARG(mode >= 0 && mode <= 2, "vt_conv_bf16_set_staging: mode %d not in 0..2", mode);
    g_conv_cl = mode;
    return VT_OK;
}

int vt_conv_bf16_set_kernels(int flags) {
    VT_CHECK_ARG(flags >= 0 && flags <= 15, "vt_conv_bf16_set_kernels: flags %d not in 0..15", flags);
    g_conv_kern = flags;
    return VT_OK;
}

int vt_conv1d_bf16_shadow(const float* W, int Cout, int Cin, int K, void* w16, void* w16t, void* stream) {
    VT_CHECK_ARG(Cout > 0 && Cin > 0 && K > 0 && K <= KMAXB, "vt_conv1d_bf16_shadow: shape");
    const int cin32 = cdiv(Cin, 32) * 32, cout32 = cdiv(Cout, 32) * 32;
    const int64_t n = (int64_t)Cout * K * cin32 + (int64_t)Cin * K * cout32;
    VT_H16(hipLaunchKernelGGL(k_conv_shadow<H>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, S(stream), W, Cout,
                              Cin, K, cin32, cout32, (H*)w16, (H*)w16t));
    VT_LAUNCH_CHECK("vt_conv1d_bf16_shadow");
    return VT_OK;
}

int vt_conv1d_bf16_shadow_batch(int n, const int64_t* W, const int* Cout, const int* Cin, const int* K,
                                const int64_t* w16, const int64_t* w16t, void* stream) {
    VT_CHECK_ARG(n >= 0 && n <= CSB_MAX, "vt_conv1d_bf16_shadow_batch: %d weights (at most %d)", n, CSB_MAX);
    if (n == 0) return VT_OK;
    ConvShadowBatch cb{};
    cb.n = n;
    cb.prefix[0] = 0;
    for (int h = 0; h < n; ++h) {
        VT_CHECK_ARG(W[h] && w16[h] && w16t[h] && Cout[h] > 0 && Cin[h] > 0 && K[h] > 0 && K[h] <= KMAXB,
                     "vt_conv1d_bf16_shadow_batch: weight %d", h);
        cb.W[h] = reinterpret_cast<const float*>(W[h]);
        cb.Cout[h] = Cout[h];
        cb.Cin[h] = Cin[h];
        cb.K[h] = K[h];
        cb.w16[h] = reinterpret_cast<void*>(w16[h]);
        cb.w16t[h] = reinterpret_cast<void*>(w16t[h]);
        const int64_t e = (int64_t)Cout[h] * K[h] * (cdiv(Cin[h], 32) * 32) + (int64_t)Cin[h] * K[h] * (cdiv(Cout[h], 32) * 32);
        cb.prefix[h + 1] = cb.prefix[h] + (int)((e + 255) / 256);
    }
    VT_H16(hipLaunchKernelGGL(k_conv_shadow_batch<H>, dim3((unsigned)cb.prefix[n]), dim3(256), 0, S(stream), cb));
    VT_LAUNCH_CHECK("vt_conv1d_bf16_shadow_batch");
    return VT_OK;
}

static int bn_fwd_bf16(const float* X, int B, int L_in, int Cin, const void* w16, int Cout, int K, int mode, int up,
                       const float* gamma, const float* beta, int act, float eps, float momentum, float* conv_out,
                       float* Y, float* mean, float* rstd, float* run_mean, float* run_var, float* ws,
                       int64_t ws_floats, hipStream_t st, const BnIn* ibn, const char* who) {
    VT_CHECK_ARG(B > 0 && L_in > 0 && Cin > 0 && Cout > 0 && K > 0 && K <= KMAXB && (mode == 0 || mode == 1),
                 "%s: shape (K <= %d)", who, KMAXB);
    Geo g = geo(B, L_in, Cin, Cout, K, mode, up);
    const int cin32 = cdiv(Cin, 32) * 32;
    const int TP = bf_launch(nullptr, g, nullptr, cin32, nullptr, g.L_out, nullptr, nullptr);
    const int tps = cdiv(g.L_out, TP);
    VT_CHECK_ARG(ws && ws_floats >= (int64_t)B * tps * 2 * Cout, "%s: workspace too small", who);
    if (bf_launch(X, g, w16, cin32, conv_out, g.L_out, ws, st, nullptr, FoldOut{-1, 0, nullptr}, ibn) < 0) return VT_ERR_ARG;
    bn_stats_finalize_launch(ws, tps, B, TP, g.L_out, Cout, eps, momentum, mean, rstd, run_mean, run_var, st);
    if (Y) bn_apply_launch(conv_out, (int64_t)B * g.L_out, Cout, mean, rstd, gamma, beta, act, Y, st);
    VT_LAUNCH_CHECK(who);
    return VT_OK;
}

int vt_conv1d_bn_fwd_bf16(const float* X, int B, int L_in, int Cin, const void* w16, int Cout, int K, int mode,
                          int up, const float* gamma, const float* beta, int act, float eps, float momentum,
                          float* conv_out, float* Y, float* mean, float* rstd, float* run_mean, float* run_var,
                          float* ws, int64_t ws_floats, void* stream) {
    return bn_fwd_bf16(X, B, L_in, Cin, w16, Cout, K, mode, up, gamma, beta, act, eps, momentum, conv_out, Y, mean,
                       rstd, run_mean, run_var, ws, ws_floats, S(stream), nullptr, "vt_conv1d_bn_fwd_bf16");
}

int vt_conv1d_bn_fwd_bf16_in(const float* X, const float* in_mean, const float* in_rstd, const float* in_gamma,
                             const float* in_beta, int in_act, int B, int L_in, int Cin, const void* w16, int Cout,
                             int K, int mode, int up, const float* gamma, const float* beta, int act, float eps,
                             float momentum, float* conv_out, float* Y, float* mean, float* rstd, float* run_mean,
                             float* run_var, float* ws, int64_t ws_floats, void* stream) {
    VT_CHECK_ARG(in_mean && in_rstd && in_gamma && in_beta && in_act == 1,
                 "vt_conv1d_bn_fwd_bf16_in: input BatchNorm parameters (ReLU blocks only)");
    const BnIn bi{in_mean, in_rstd, in_gamma, in_beta, in_act};
    return bn_fwd_bf16(X, B, L_in, Cin, w16, Cout, K, mode, up, gamma, beta, act, eps, momentum, conv_out, Y, mean,
                       rstd, run_mean, run_var, ws, ws_floats, S(stream), &bi, "vt_conv1d_bn_fwd_bf16_in");
}

int vt_conv1d_fwd_bf16(const float* X, int B, int L_in, int Cin, const void* w16, int Cout, int K, int mode, int up,
                       float* Y, void* stream) {
    VT_CHECK_ARG(B > 0 && L_in > 0 && Cin > 0 && Cout > 0 && K > 0 && K <= KMAXB && (mode == 0 || mode == 1),
                 "vt_conv1d_fwd_bf16: shape (K <= %d)", KMAXB);
    Geo g = geo(B, L_in, Cin, Cout, K, mode, up);
    if (bf_launch(X, g, w16, cdiv(Cin, 32) * 32, Y, g.L_out, nullptr, S(stream)) < 0) return VT_ERR_ARG;
    VT_LAUNCH_CHECK("vt_conv1d_fwd_bf16");
    return VT_OK;
}

static int bwd_gpad(const float* dY, int B, int L_in, int Cin, const void* w16t, int Cout, int K, int mode, int up,
                    float* gpad, hipStream_t st, const BnB* bn, const char* who,
                    FoldOut fo = FoldOut{-1, 0, nullptr}) {
    VT_CHECK_ARG(B > 0 && L_in > 0 && Cin > 0 && Cout > 0 && K > 0 && K <= KMAXB, "%s: shape", who);
    Geo f = geo(B, L_in, Cin, Cout, K, mode, up);
    Geo g = geo(B, f.L_out, Cout, Cin, K, 0, 0);  // input dY (L_out x Cout), causal pad K-1
    if (bf_launch(dY, g, w16t, cdiv(Cout, 32) * 32, gpad, f.L_out + K - 1, nullptr, st, bn, fo) < 0) return VT_ERR_ARG;
    VT_LAUNCH_CHECK(who);
    return VT_OK;
}

int vt_conv1d_bwd_gpad_bf16(const float* dY, int B, int L_in, int Cin, const void* w16t, int Cout, int K, int mode,
                            int up, float* gpad, void* stream) {
    return bwd_gpad(dY, B, L_in, Cin, w16t, Cout, K, mode, up, gpad, S(stream), nullptr, "vt_conv1d_bwd_gpad_bf16");
}

int vt_conv1d_bwd_gpad_bf16_bn(const float* dY, const float* Xc, const float* bnp, int act, int64_t M, int B,
                               int L_in, int Cin, const void* w16t, int Cout, int K, int mode, int up, float* gpad,
                               void* dxbn16, void* stream) {
    VT_CHECK_ARG(Xc && bnp && act >= 0 && act <= 3 && M > 0, "vt_conv1d_bwd_gpad_bf16_bn: BatchNorm arguments");
    const BnB bn{Xc, bnp, act, 1.f / (float)M, dxbn16};
    return bwd_gpad(dY, B, L_in, Cin, w16t, Cout, K, mode, up, gpad, S(stream), &bn, "vt_conv1d_bwd_gpad_bf16_bn");
}

int vt_conv1d_bwd_dx_bf16_bn(const float* dY, const float* Xc, const float* bnp, int act, int64_t M, int B, int L_in,
                             int Cin, const void* w16t, int Cout, int K, int mode, int up, float* dX, float* edge,
                             void* dxbn16, void* stream) {
    VT_CHECK_ARG(Xc && bnp && act >= 0 && act <= 3 && M > 0, "vt_conv1d_bwd_dx_bf16_bn: BatchNorm arguments");
    const Geo f = geo(B, L_in, Cin, Cout, K, mode, up);
    VT_CHECK_ARG(!up && (mode == 0 || f.L_up > f.pad) && (mode == 0 || f.pad == 0 || edge),
                 "vt_conv1d_bwd_dx_bf16_bn: geometry (no upsample, reflect needs L > pad and an edge buffer)");
    const BnB bn{Xc, bnp, act, 1.f / (float)M, dxbn16};
    const FoldOut fo{f.pad, L_in, mode == 0 ? nullptr : edge};
    const int rc = bwd_gpad(dY, B, L_in, Cin, w16t, Cout, K, mode, up, dX, S(stream), &bn,
                            "vt_conv1d_bwd_dx_bf16_bn", fo);
    if (rc) return rc;
    if (mode == 1 && f.pad > 0) {
        VT_CHECK_ARG(B <= 65535, "vt_conv1d_bwd_dx_bf16_bn: batch");
        fold_edges_launch(dX, edge, B, L_in, f.pad, Cin, S(stream));
        VT_LAUNCH_CHECK("vt_conv1d_bwd_dx_bf16_bn");
    }
    return VT_OK;
}

}  // extern "C"
