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

namespace vt {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

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

__device__ __forceinline__ bf16x8 pack8(const float (&v)[8]) {
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (__bf16)v[j];
    return r;
}

// Window staging with lanes along channels (the default; g_conv_cl): thread t stages
// channel c0 + (t & 31) of rows (t >> 5) + 8 i, so a wave-instruction reads two
// 128-B row segments (2-4 cache lines) instead of 4 channels in each of 16 rows, and
// the BatchNorm-backward parameters of its one channel sit in registers.  U rows per
// round, all their loads issued before the first use.  Same values and the same bf16
// roundings as the octet staging below (bit-identical results).
template <int K, int WIN, bool BNB>
__device__ __forceinline__ void stage_window_cl(__bf16* __restrict__ xs, const float* __restrict__ xb,
                                                const float* __restrict__ x2b, const Geo& g, int t0, int TP, int Lo,
                                                int c0, const float* __restrict__ bp, int act, float invM,
                                                __bf16* __restrict__ dbf, int b, bool write_dbf) {
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
                if constexpr (BNB) v = bn_bwd_val_r(a[u], q[u], pm, prs, pga, pbe, pdg, pdb, act, invM);
                else v = g.up ? up_lerp(a[u], q[u], l1[u]) : a[u];
            }
            xs[r * RS + cl] = (__bf16)v;
            if constexpr (BNB) {
                // the bf16 side output: the row's channels and its zero channel padding up to cpad
                const int t = t0 + r - g.pad;
                if (write_dbf && rok[u] && c < cpad && t >= t0 && t < t0 + TP)
                    dbf[((int64_t)b * g.L_in + t) * cpad + c] = (__bf16)v;
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
// kernel selection (vt_conv_bf16_set_kernels): bit 0 the flat-staged forward (conv_fwd16.hip)
int g_conv_kern = 11;   // bit 3: 256-row chunks in the flat weight gradient for dY <= 32 channels   // bit 1: the flat-staged weight gradient (k_cdw16); bit 2: both at every K

// x: fp32 (B, L_in, g.Cin) activations; w16: [g.Cout][K][cin32] bf16 shadow.
// BNB (backward-data only: causal geometry, no upsample): x is the block output
// gradient dy and the staged operand is the BatchNorm input gradient computed on
// the fly from dy, the pre-BN conv output x2 and bnp (conv.h bn_bwd_val).
// dbf (BNB, nullable): the staged BN input gradient, bf16, is also written to
// dbf[(b L_in + t) cpad + c] (cpad = ceil8(Cin)) by the blockIdx.y == 0 workgroups
// for their own rows t0 .. t0 + TP - 1 (each row once) — the weight gradient's operand.
template <int K, int NT, bool BNB = false, bool CL = true>
__global__ __launch_bounds__(256) void k_conv_bf16(const float* __restrict__ x, Geo g, const __bf16* __restrict__ w16,
                                                   int cin32, float* __restrict__ y, int Lo,
                                                   float* __restrict__ stats, const float* __restrict__ x2,
                                                   const float* __restrict__ bnp, int act, float invM,
                                                   __bf16* __restrict__ dbf, FoldOut fo) {
    using C = BCfg<K, NT>;
    constexpr int PM = C::PM, TC = C::TC, TP = C::TP, WIN = C::WIN;
    extern __shared__ __attribute__((aligned(16))) __bf16 lb[];
    __bf16* xs = lb;           // [WIN][RS]
    __bf16* ws = lb + C::XB;   // [K][TC][RS]
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lr = lane & 15, lc = lane >> 4;
    const int t0 = blockIdx.x * TP, co0 = blockIdx.y * TC, b = blockIdx.z;
    const float* xb = x + (int64_t)b * g.L_in * g.Cin;
    float* bp = reinterpret_cast<float*>(reinterpret_cast<char*>(lb) + C::LDS_BYTES);  // BNB: 6 x Cin params
    if constexpr (BNB) {
        for (int i = tid; i < 6 * g.Cin; i += 256) bp[i] = bnp[i];
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
            bf16x8 wt[NWI];
#pragma unroll
            for (int it = 0; it < NWI; ++it) {
                const int i = tid + 256 * it;
                const int ic = i < K * TC * 4 ? i : K * TC * 4 - 1;
                const int oct = ic & 3, r = ic >> 2, k = r / TC, co = r - k * TC;
                const int coc = co0 + co < g.Cout ? co0 + co : g.Cout - 1;
                wt[it] = *(const bf16x8*)(w16 + ((int64_t)coc * K + k) * cin32 + c0 + 8 * oct);
            }
            stage_window_cl<K, WIN, BNB>(xs, xb, x2b, g, t0, TP, Lo, c0, bp, act, invM, dbf, b,
                                         BNB && dbf && blockIdx.y == 0);
#pragma unroll
            for (int it = 0; it < NWI; ++it) {
                const int i = tid + 256 * it;
                if (i >= K * TC * 4) continue;
                const int oct = i & 3, r = i >> 2, k = r / TC, co = r - k * TC;
                bf16x8 val = wt[it];
                if (co0 + co >= g.Cout) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) val[j] = (__bf16)0.f;
                }
                *(bf16x8*)(ws + (k * TC + co) * RS + 8 * oct) = val;
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
                        *(bf16x8*)(dbf + ((int64_t)b * g.L_in + t) * cpad + cb) = pack8(v);
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) v[j] = (ok && cb + j < g.Cin) ? src_val(xb, g, tp, cb + j) : 0.f;
                }
                *(bf16x8*)(xs + row * RS + 8 * oct) = pack8(v);
            }
            for (int i = tid; i < K * TC * 4; i += 256) {
                const int oct = i & 3, r = i >> 2, k = r / TC, co = r - k * TC;
                bf16x8 val;
                if (co0 + co < g.Cout) {
                    val = *(const bf16x8*)(w16 + ((int64_t)(co0 + co) * K + k) * cin32 + c0 + 8 * oct);
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) val[j] = (__bf16)0.f;
                }
                *(bf16x8*)(ws + (k * TC + co) * RS + 8 * oct) = val;
            }
        } else {
            // window: WIN rows x 4 octets of 8 channels, fp32 -> bf16, and the chunk's taps
            // (K x TC rows x 4 octets, 16 B each from the shadow): every load of the thread
            // issued before the first store (clamped addresses, masked values)
            constexpr int NI = (WIN * 4 + 255) / 256, NWI = (K * TC * 4 + 255) / 256;
            bf16x8 wt[NWI];
    #pragma unroll
            for (int it = 0; it < NWI; ++it) {
                const int i = tid + 256 * it;
                const int ic = i < K * TC * 4 ? i : K * TC * 4 - 1;
                const int oct = ic & 3, r = ic >> 2, k = r / TC, co = r - k * TC;
                const int coc = co0 + co < g.Cout ? co0 + co : g.Cout - 1;
                wt[it] = *(const bf16x8*)(w16 + ((int64_t)coc * K + k) * cin32 + c0 + 8 * oct);
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
                        *(bf16x8*)(dbf + ((int64_t)b * g.L_in + t) * cpad + cb) = pack8(v[it]);
                    }
                } else {
                    src_vec<8>(xb, g, tp, cb, ok, v[it]);
                }
            }
    #pragma unroll
            for (int it = 0; it < NB; ++it) {
                const int i = tid + 256 * (r0 + it);
                if (r0 + it < NI && i < WIN * 4) *(bf16x8*)(xs + (i >> 2) * RS + 8 * (i & 3)) = pack8(v[it]);
            }
            }
    #pragma unroll
            for (int it = 0; it < NWI; ++it) {
                const int i = tid + 256 * it;
                if (i >= K * TC * 4) continue;
                const int oct = i & 3, r = i >> 2, k = r / TC, co = r - k * TC;
                bf16x8 val = wt[it];
                if (co0 + co >= g.Cout) {
    #pragma unroll
                    for (int j = 0; j < 8; ++j) val[j] = (__bf16)0.f;
                }
                *(bf16x8*)(ws + (k * TC + co) * RS + 8 * oct) = val;
            }
        }
        __syncthreads();
        const __bf16* xq = xs + (PM * 16 * wv + lr) * RS + 8 * lc;
        const __bf16* wq = ws + lr * RS + 8 * lc;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            bf16x8 af[PM], bf[NT];
#pragma unroll
            for (int m = 0; m < PM; ++m) af[m] = *(const bf16x8*)(xq + (16 * m + k) * RS);
#pragma unroll
            for (int n = 0; n < NT; ++n) bf[n] = *(const bf16x8*)(wq + (k * TC + 16 * n) * RS);
#pragma unroll
            for (int m = 0; m < PM; ++m)
#pragma unroll
                for (int n = 0; n < NT; ++n)
                    acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bf[n], acc[m][n], 0, 0, 0);
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
__global__ void k_conv_shadow(const float* __restrict__ W, int Cout, int Cin, int K, int cin32, int cout32,
                              __bf16* __restrict__ w16, __bf16* __restrict__ w16t) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n1 = (int64_t)Cout * K * cin32;
    if (i < n1) {
        const int ci = (int)(i % cin32);
        const int64_t r = i / cin32;
        const int k = (int)(r % K), co = (int)(r / K);
        w16[i] = (__bf16)(ci < Cin ? W[((int64_t)co * Cin + ci) * K + k] : 0.f);
    } else if (i < n1 + (int64_t)Cin * K * cout32) {
        const int64_t j = i - n1;
        const int co = (int)(j % cout32);
        const int64_t r = j / cout32;
        const int k = (int)(r % K), ci = (int)(r / K);
        w16t[j] = (__bf16)(co < Cout ? W[((int64_t)co * Cin + ci) * K + (K - 1 - k)] : 0.f);
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
    __bf16* w16[CSB_MAX];
    __bf16* w16t[CSB_MAX];
    int prefix[CSB_MAX + 1];   // workgroups
};
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
        cb.w16[h][i] = (__bf16)(ci < Cin ? W[((int64_t)co * Cin + ci) * K + k] : 0.f);
    } else if (i < n1 + (int64_t)Cin * K * cout32) {
        const int64_t j = i - n1;
        const int co = (int)(j % cout32);
        const int64_t r = j / cout32;
        const int k = (int)(r % K), ci = (int)(r / K);
        cb.w16t[h][j] = (__bf16)(co < Cout ? W[((int64_t)co * Cin + ci) * K + (K - 1 - k)] : 0.f);
    }
}

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

__device__ __forceinline__ bf16x8 tr_frag(const __bf16* img, int row0, int col0, int stride) {
    // lane 4q+p of each 16-lane group addresses row (row0 + q), columns col0 + 4p .. +3; two reads
    // (rows +0..3 and +4..7 of the lane group's 8-row block)
    const int lane = threadIdx.x & 63, g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const __bf16* a0 = img + (row0 + 8 * g + q) * stride + col0 + 4 * p;
    const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)a0);
    const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) v4i16*)(a0 + 4 * stride));
    // whole-vector concatenation + bit_cast: element-wise bit_casts of the v4i16 results are
    // miscompiled (each lane's element 0 replicated by v_perm_b32)
    typedef short v8i16 __attribute__((ext_vector_type(8)));
    const v8i16 r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, r);
}

// DYB: dY given in bf16 (dyb16, row stride dys = ceil8(Cout)), e.g. the BN input
// gradient written by the fused backward-data kernel (k_conv_bf16 BNB + dbf).
template <int K, int PPW, bool DYB = false, int NWV = 4>
__global__ __launch_bounds__(64 * NWV) void k_conv_dw_bf16(const float* __restrict__ dy, const float* __restrict__ x, Geo g,
                                                      int64_t rows_per_split, int NTc, int npairs, int dstride,
                                                      int xstride, float* __restrict__ part,
                                                      const __bf16* __restrict__ dyb16, int dys) {
    extern __shared__ __attribute__((aligned(16))) __bf16 lb[];
    __bf16* ds = lb;                          // [DWR][dstride]   dY rows
    __bf16* xs = lb + DWR * dstride;          // [DWR + K - 1 (+pad)][xstride] input window
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
        constexpr int UR = K <= 3 ? 1 : 4;   // small K: registers (occupancy) first
        const int nd = DWR * (cout16 / 4), nx = (DWR + K - 1) * (cin16 / 4);
        if constexpr (DYB) {
            const __bf16* db16 = dyb16 + ((int64_t)b * g.L_out + t0) * dys;
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
                        for (int j = 0; j < 4; ++j) ds[t * dstride + c + j] = (__bf16)v[u][j];
                }
            }
        }
        for (int i0 = tid; i0 < nx; i0 += 64 * NWV * UR) {
            float v[UR][4];
#pragma unroll
            for (int u = 0; u < UR; ++u) {
                const int i = i0 + 64 * NWV * u;
                const int t = i / (cin16 / 4), c = 4 * (i - t * (cin16 / 4));
                src_vec<4>(xb, g, t0 + t, c, i < nx && t < n + K - 1, v[u]);
            }
#pragma unroll
            for (int u = 0; u < UR; ++u) {
                const int i = i0 + 64 * NWV * u;
                const int t = i / (cin16 / 4), c = 4 * (i - t * (cin16 / 4));
                if (i < nx)
#pragma unroll
                    for (int j = 0; j < 4; ++j) xs[t * xstride + c + j] = (__bf16)v[u][j];
            }
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < DWR / 32; ++s) {
            if (!act[0]) break;  // wave-uniform: a wave without pairs only stages
#pragma unroll
            for (int j = 0; j < PPW; ++j) {
                // no early-out on inactive pairs: the transposed read needs all 64 lanes (EXEC all ones)
                const bf16x8 a = tr_frag(ds, 32 * s, 16 * mt[j], dstride);
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const bf16x8 bb = tr_frag(xs, 32 * s + k, 16 * nt[j], xstride);
                    acc[j][k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bb, acc[j][k], 0, 0, 0);
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
template <int K, int PPW, int NWV, int CR = DWR>
__global__ __launch_bounds__(64 * NWV) void k_cdw16(const __bf16* __restrict__ dyb16, int dys,
                                                   const float* __restrict__ x, Geo g, int64_t rows_per_split,
                                                   int NTc, int npairs, int dstride, int xstride,
                                                   float* __restrict__ part, int64_t total) {
    constexpr int NT = 64 * NWV;
    constexpr int UD = CR == DWR ? CDW_UD * 256 / NT : CR * 4 / NT;   // CR 256: dY rows of <= 4 segments
    constexpr int UF = CR == DWR ? CDW_UF * 256 / NT : CDW_UF_WIDE * 256 / NT;
    extern __shared__ __attribute__((aligned(16))) __bf16 lb[];
    __bf16* ds = lb;                          // [CR][dstride]   dY rows
    __bf16* xs = lb + CR * dstride;           // [CR + K - 1 (+pad)][xstride] input window
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
    // one chunk's operands into registers: dY segments and the F rows (float4 from the
    // boundary at or below the source run)
    bf16x8 dv[UD];
    float4 fv[UF];
    struct Chunk {
        int b, t0, n, lo, hi, off, nv;
    };
    auto load = [&](int64_t r, Chunk& c) {
        c.b = (int)(r / g.L_out);
        c.t0 = (int)(r - (int64_t)c.b * g.L_out);
        c.n = g.L_out - c.t0 < CR ? g.L_out - c.t0 : CR;
        if (r + c.n > r1) c.n = (int)(r1 - r);
        const __bf16* db = dyb16 + ((int64_t)c.b * g.L_out + c.t0) * dys;
#pragma unroll
        for (int u = 0; u < UD; ++u) {
            const int i = tid + NT * u;
            const int t = i / dsegs, sg = i - t * dsegs;
            const bool ok = i < CR * dsegs && t < c.n && 8 * sg < dys;
            dv[u] = *(const bf16x8*)(db + (int64_t)(ok ? t : 0) * dys + (ok ? 8 * sg : 0));
            if (!ok) {
#pragma unroll
                for (int j = 0; j < 8; ++j) dv[u][j] = (__bf16)0.f;
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
                *(bf16x8*)(ds + t * dstride + 8 * sg) = dv[u];
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
                bf16x8 v;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int c = cb + j < g.Cin ? cb + j : g.Cin - 1;
                    const float a = p0[c];
                    const float q = g.up ? p1[c] : 0.f;
                    v[j] = (__bf16)((in && cb + j < g.Cin) ? (g.up ? up_lerp(a, q, l1) : a) : 0.f);
                }
                *(bf16x8*)(xs + t * xstride + cb) = v;
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
                const bf16x8 a = tr_frag(ds, 32 * s, 16 * mt[j], dstride);
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const bf16x8 bb = tr_frag(xs, 32 * s + k, 16 * nt[j], xstride);
                    acc[j][k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bb, acc[j][k], 0, 0, 0);
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

// BatchNorm-backward staging (k_conv_bf16 / k_conv_dw_bf16 BNB): dy, the pre-BN
// conv output, the packed per-channel parameters (6 x C), activation and 1/M
struct BnB {
    const float* x2;
    const float* bnp;
    int act;
    float invM;
    __bf16* dbf;   // nullable: bf16 copy of the BN input gradient (the weight gradient's operand)
};

template <int K, int NT>
int bf_nt(const float* x, const Geo& g, const __bf16* w16, int cin32, float* y, int Lo, float* stats,
          hipStream_t st, const BnB* bn, FoldOut fo) {
    using C = BCfg<K, NT>;
    // flat-staged forward where it measured faster than k_conv_bf16 (isolated, decoder
    // geometry: K 5 / 3 layers 60 -> 52, 102 -> 60 us; K >= 7 slower: 30 -> 43 us at K 11)
    if (x && !bn && (g_conv_kern & 1) && (K <= 5 || (g_conv_kern & 4)) && fo.pad < 0 && ((uintptr_t)x & 15) == 0) {
        const int tp = cfw16_launch(x, g, w16, y, Lo, stats, st);
        if (tp > 0) return tp;
    }
    dim3 grid(cdiv(Lo, C::TP), cdiv(g.Cout, C::TC), g.B);
    const bool cl = g_conv_cl == 2 || (g_conv_cl == 1 && bn && K >= 7);
    if (x && bn && cl)
        hipLaunchKernelGGL((k_conv_bf16<K, NT, true, true>), grid, dim3(256), C::LDS_BYTES + 24 * g.Cin, st, x, g, w16,
                           cin32, y, Lo, stats, bn->x2, bn->bnp, bn->act, bn->invM, bn->dbf, fo);
    else if (x && bn)
        hipLaunchKernelGGL((k_conv_bf16<K, NT, true, false>), grid, dim3(256), C::LDS_BYTES + 24 * g.Cin, st, x, g,
                           w16, cin32, y, Lo, stats, bn->x2, bn->bnp, bn->act, bn->invM, bn->dbf, fo);
    else if (x && cl)
        hipLaunchKernelGGL((k_conv_bf16<K, NT, false, true>), grid, dim3(256), C::LDS_BYTES, st, x, g, w16, cin32, y,
                           Lo, stats, nullptr, nullptr, 0, 0.f, nullptr, fo);
    else if (x)
        hipLaunchKernelGGL((k_conv_bf16<K, NT, false, false>), grid, dim3(256), C::LDS_BYTES, st, x, g, w16, cin32, y,
                           Lo, stats, nullptr, nullptr, 0, 0.f, nullptr, fo);
    return C::TP;
}

template <int K>
int bf_k(const float* x, const Geo& g, const __bf16* w16, int cin32, float* y, int Lo, float* stats, hipStream_t st,
         const BnB* bn, FoldOut fo) {
    switch (cdiv(g.Cout, 16) < 6 ? cdiv(g.Cout, 16) : 6) {
        case 1: return bf_nt<K, 1>(x, g, w16, cin32, y, Lo, stats, st, bn, fo);
        case 2: return bf_nt<K, 2>(x, g, w16, cin32, y, Lo, stats, st, bn, fo);
        case 3: return bf_nt<K, 3>(x, g, w16, cin32, y, Lo, stats, st, bn, fo);
        case 4: return bf_nt<K, 4>(x, g, w16, cin32, y, Lo, stats, st, bn, fo);
        case 5: return bf_nt<K, 5>(x, g, w16, cin32, y, Lo, stats, st, bn, fo);
        default: return bf_nt<K, 6>(x, g, w16, cin32, y, Lo, stats, st, bn, fo);
    }
}

// x == nullptr: no launch, only the position tile of this geometry
int bf_launch(const float* x, const Geo& g, const __bf16* w16, int cin32, float* y, int Lo, float* stats,
              hipStream_t st, const BnB* bn = nullptr, FoldOut fo = FoldOut{-1, 0, nullptr}) {
    switch (g.K) {
        case 1: return bf_k<1>(x, g, w16, cin32, y, Lo, stats, st, bn, fo);
        case 2: return bf_k<2>(x, g, w16, cin32, y, Lo, stats, st, bn, fo);
        case 3: return bf_k<3>(x, g, w16, cin32, y, Lo, stats, st, bn, fo);
        case 4: return bf_k<4>(x, g, w16, cin32, y, Lo, stats, st, bn, fo);
        case 5: return bf_k<5>(x, g, w16, cin32, y, Lo, stats, st, bn, fo);
        case 6: return bf_k<6>(x, g, w16, cin32, y, Lo, stats, st, bn, fo);
        case 7: return bf_k<7>(x, g, w16, cin32, y, Lo, stats, st, bn, fo);
        case 8: return bf_k<8>(x, g, w16, cin32, y, Lo, stats, st, bn, fo);
        case 9: return bf_k<9>(x, g, w16, cin32, y, Lo, stats, st, bn, fo);
        case 10: return bf_k<10>(x, g, w16, cin32, y, Lo, stats, st, bn, fo);
        default: return bf_k<11>(x, g, w16, cin32, y, Lo, stats, st, bn, fo);
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
    hipLaunchKernelGGL(k_conv_shadow, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, S(stream), W, Cout, Cin, K,
                       cin32, cout32, (__bf16*)w16, (__bf16*)w16t);
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
        cb.w16[h] = reinterpret_cast<__bf16*>(w16[h]);
        cb.w16t[h] = reinterpret_cast<__bf16*>(w16t[h]);
        const int64_t e = (int64_t)Cout[h] * K[h] * (cdiv(Cin[h], 32) * 32) + (int64_t)Cin[h] * K[h] * (cdiv(Cout[h], 32) * 32);
        cb.prefix[h + 1] = cb.prefix[h] + (int)((e + 255) / 256);
    }
    hipLaunchKernelGGL(k_conv_shadow_batch, dim3((unsigned)cb.prefix[n]), dim3(256), 0, S(stream), cb);
    VT_LAUNCH_CHECK("vt_conv1d_bf16_shadow_batch");
    return VT_OK;
}

int vt_conv1d_bn_fwd_bf16(const float* X, int B, int L_in, int Cin, const void* w16, int Cout, int K, int mode,
                          int up, const float* gamma, const float* beta, int act, float eps, float momentum,
                          float* conv_out, float* Y, float* mean, float* rstd, float* run_mean, float* run_var,
                          float* ws, int64_t ws_floats, void* stream) {
    VT_CHECK_ARG(B > 0 && L_in > 0 && Cin > 0 && Cout > 0 && K > 0 && K <= KMAXB && (mode == 0 || mode == 1),
                 "vt_conv1d_bn_fwd_bf16: shape (K <= %d)", KMAXB);
    Geo g = geo(B, L_in, Cin, Cout, K, mode, up);
    const int cin32 = cdiv(Cin, 32) * 32;
    const int TP = bf_launch(nullptr, g, nullptr, cin32, nullptr, g.L_out, nullptr, nullptr);
    const int tps = cdiv(g.L_out, TP);
    VT_CHECK_ARG(ws && ws_floats >= (int64_t)B * tps * 2 * Cout, "vt_conv1d_bn_fwd_bf16: workspace too small");
    hipStream_t st = S(stream);
    bf_launch(X, g, (const __bf16*)w16, cin32, conv_out, g.L_out, ws, st);
    bn_stats_finalize_launch(ws, tps, B, TP, g.L_out, Cout, eps, momentum, mean, rstd, run_mean, run_var, st);
    bn_apply_launch(conv_out, (int64_t)B * g.L_out, Cout, mean, rstd, gamma, beta, act, Y, st);
    VT_LAUNCH_CHECK("vt_conv1d_bn_fwd_bf16");
    return VT_OK;
}

int vt_conv1d_fwd_bf16(const float* X, int B, int L_in, int Cin, const void* w16, int Cout, int K, int mode, int up,
                       float* Y, void* stream) {
    VT_CHECK_ARG(B > 0 && L_in > 0 && Cin > 0 && Cout > 0 && K > 0 && K <= KMAXB && (mode == 0 || mode == 1),
                 "vt_conv1d_fwd_bf16: shape (K <= %d)", KMAXB);
    Geo g = geo(B, L_in, Cin, Cout, K, mode, up);
    bf_launch(X, g, (const __bf16*)w16, cdiv(Cin, 32) * 32, Y, g.L_out, nullptr, S(stream));
    VT_LAUNCH_CHECK("vt_conv1d_fwd_bf16");
    return VT_OK;
}

static int bwd_gpad(const float* dY, int B, int L_in, int Cin, const void* w16t, int Cout, int K, int mode, int up,
                    float* gpad, hipStream_t st, const BnB* bn, const char* who,
                    FoldOut fo = FoldOut{-1, 0, nullptr}) {
    VT_CHECK_ARG(B > 0 && L_in > 0 && Cin > 0 && Cout > 0 && K > 0 && K <= KMAXB, "%s: shape", who);
    Geo f = geo(B, L_in, Cin, Cout, K, mode, up);
    Geo g = geo(B, f.L_out, Cout, Cin, K, 0, 0);  // input dY (L_out x Cout), causal pad K-1
    bf_launch(dY, g, (const __bf16*)w16t, cdiv(Cout, 32) * 32, gpad, f.L_out + K - 1, nullptr, st, bn, fo);
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
    const BnB bn{Xc, bnp, act, 1.f / (float)M, (__bf16*)dxbn16};
    return bwd_gpad(dY, B, L_in, Cin, w16t, Cout, K, mode, up, gpad, S(stream), &bn, "vt_conv1d_bwd_gpad_bf16_bn");
}

int vt_conv1d_bwd_dx_bf16_bn(const float* dY, const float* Xc, const float* bnp, int act, int64_t M, int B, int L_in,
                             int Cin, const void* w16t, int Cout, int K, int mode, int up, float* dX, float* edge,
                             void* dxbn16, void* stream) {
    VT_CHECK_ARG(Xc && bnp && act >= 0 && act <= 3 && M > 0, "vt_conv1d_bwd_dx_bf16_bn: BatchNorm arguments");
    const Geo f = geo(B, L_in, Cin, Cout, K, mode, up);
    VT_CHECK_ARG(!up && (mode == 0 || f.L_up > f.pad) && (mode == 0 || f.pad == 0 || edge),
                 "vt_conv1d_bwd_dx_bf16_bn: geometry (no upsample, reflect needs L > pad and an edge buffer)");
    const BnB bn{Xc, bnp, act, 1.f / (float)M, (__bf16*)dxbn16};
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

static int bwd_weight(const float* dY, const float* X, int B, int L_in, int Cin, int Cout, int K, int mode, int up,
                      float* dW, int accumulate, float* ws, int64_t ws_floats, hipStream_t st, const __bf16* dy16,
                      int dys = 0) {
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
#define VT_DWB(KK, PP)                                                                                         \
    if (K == KK && ppw == PP) {                                                                                \
        if (wide && nwv == 8)                                                                                  \
            hipLaunchKernelGGL((k_cdw16<KK, PP, 8, 256>), grid, dim3(512), lds_wide, st, dy16, dys, X, g, rps,   \
                               NTc, npairs, dstride, xstride, ws, total_x);                                   \
        else if (wide)                                                                                         \
            hipLaunchKernelGGL((k_cdw16<KK, PP, 4, 256>), grid, dim3(256), lds_wide, st, dy16, dys, X, g, rps,   \
                               NTc, npairs, dstride, xstride, ws, total_x);                                   \
        else if (flat && nwv == 8)                                                                             \
            hipLaunchKernelGGL((k_cdw16<KK, PP, 8>), grid, dim3(512), lds_flat, st, dy16, dys, X, g, rps, NTc,   \
                               npairs, dstride, xstride, ws, total_x);                                        \
        else if (flat)                                                                                         \
            hipLaunchKernelGGL((k_cdw16<KK, PP, 4>), grid, dim3(256), lds_flat, st, dy16, dys, X, g, rps, NTc,   \
                               npairs, dstride, xstride, ws, total_x);                                        \
        else if (dy16 && nwv == 8)                                                                             \
            hipLaunchKernelGGL((k_conv_dw_bf16<KK, PP, true, 8>), grid, dim3(512), lds, st, dY, X, g, rps, NTc,  \
                               npairs, dstride, xstride, ws, dy16, dys);                                      \
        else if (dy16)                                                                                         \
            hipLaunchKernelGGL((k_conv_dw_bf16<KK, PP, true>), grid, dim3(256), lds, st, dY, X, g, rps, NTc, npairs, \
                               dstride, xstride, ws, dy16, dys);                                              \
        else                                                                                                   \
            hipLaunchKernelGGL((k_conv_dw_bf16<KK, PP>), grid, dim3(256), lds, st, dY, X, g, rps, NTc, npairs, \
                               dstride, xstride, ws, nullptr, 0);                                             \
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
    return bwd_weight(nullptr, X, B, L_in, Cin, Cout, K, mode, up, dW, accumulate, ws, ws_floats, S(stream),
                      (const __bf16*)dY16);
}

int vt_conv1d_bwd_weight_bf16_dy16s(const void* dY16, int dys, const float* X, int B, int L_in, int Cin, int Cout,
                                    int K, int mode, int up, float* dW, int accumulate, float* ws, int64_t ws_floats,
                                    void* stream) {
    VT_CHECK_ARG(dY16 != nullptr && dys >= ((Cout + 7) & ~7) && dys % 8 == 0,
                 "vt_conv1d_bwd_weight_bf16_dy16s: null dY16 or row stride %d (a multiple of 8 >= ceil8(Cout))", dys);
    return bwd_weight(nullptr, X, B, L_in, Cin, Cout, K, mode, up, dW, accumulate, ws, ws_floats, S(stream),
                      (const __bf16*)dY16, dys);
}

}  // extern "C"
