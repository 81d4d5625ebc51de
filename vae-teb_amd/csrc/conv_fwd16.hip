// bf16-MFMA conv-block forward with flat operand staging (SURVEY.md §8(a) a11, a15;
// ref/model/vae_teb_model.py:128-253: Conv1d(bias=False) on the causal / reflect-padded,
// optionally x2 linearly upsampled input, in the reference's 16-bit autocast precision:
// DESIGN.md §5).
//
// The same implicit GEMM, tile shapes, accumulation order and BatchNorm tile statistics
// as conv_bf16.hip's k_conv_bf16 (so the outputs and statistics are bit-identical), with
// the operand window staged differently.  The fp32 activations have odd widths (87, 77,
// 33 ... channels), so a row is not 16-byte aligned and the element-wise staging of
// k_conv_bf16 issues one 4-byte load per element and lane.  Here a workgroup copies the
// source rows its window reads — one contiguous run of B*L_in*Cin floats — with float4
// loads into LDS (F), forms the whole bf16 window of every 32-channel chunk from F
// (padding and the x2 interpolation applied exactly as conv.h src_vec: the same
// arithmetic, rounded to bf16 afterwards, as the reference's autocast rounds the
// interpolated input of the next Conv1d), then walks the chunks with the next chunk's
// taps prefetched into registers during the current chunk's MFMAs (F's LDS is reused
// for the taps).
#include "conv.h"
#include "h16.h"

namespace vt {

namespace {


constexpr int RS = 40;   // bf16 row stride of window / tap rows (as conv_bf16.hip)

template <int K, int NT>
struct FCfg {
    static constexpr int PM = NT <= 2 ? 4 : 2;                  // as conv_bf16.hip BCfg (tile statistics)
    static constexpr int TC = 16 * NT, TP = 64 * PM, WIN = TP + K - 1;
    static constexpr int NWI = (K * TC * 4 + 255) / 256;
    static constexpr int WBYTES = K * TC * RS * 2;
};

// IBN: x is the previous block's pre-BN conv output; its BatchNorm + activation (bi, staged
// into LDS at byte ipo) are applied to the source samples as the window is formed
template <int K, int NT, bool IBN = false, typename H = __bf16>
__global__ __launch_bounds__(256) void k_cfw16(const float* __restrict__ x, Geo g, int nch,
                                               const H* __restrict__ w16, float* __restrict__ y, int Lo,
                                               float* __restrict__ stats, int64_t total, BnIn bi, int ipo) {
    using C = FCfg<K, NT>;
    constexpr int PM = C::PM, TC = C::TC, TP = C::TP, WIN = C::WIN;
    extern __shared__ __attribute__((aligned(16))) char lb_raw[];
    H* const lb = reinterpret_cast<H*>(lb_raw);
    const int cin32 = 32 * nch;
    H* xs = lb;                                              // [nch][WIN][RS]
    char* rest = reinterpret_cast<char*>(lb + nch * WIN * RS);   // F (fp32 source rows), then the taps
    float* F = reinterpret_cast<float*>(rest);
    H* ws = reinterpret_cast<H*>(rest);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lr = lane & 15, lc = lane >> 4;
    const int t0 = blockIdx.x * TP, co0 = blockIdx.y * TC, b = blockIdx.z;
    hv8<H> wt[C::NWI];
    auto load_taps = [&](int c0) {
#pragma unroll
        for (int it = 0; it < C::NWI; ++it) {
            const int i = tid + 256 * it;
            const int ic = i < K * TC * 4 ? i : K * TC * 4 - 1;
            const int oct = ic & 3, r = ic >> 2, k = r / TC, co = r - k * TC;
            const int coc = co0 + co < g.Cout ? co0 + co : g.Cout - 1;
            wt[it] = *(const hv8<H>*)(w16 + ((int64_t)coc * K + k) * cin32 + c0 + 8 * oct);
        }
    };
    load_taps(0);   // in flight during the window staging
    float* ip = reinterpret_cast<float*>(reinterpret_cast<char*>(lb) + ipo);
    if constexpr (IBN) stage_bn_in(bi, g.Cin, ip, cin32);   // visible after stage 1's barrier
    int lo, hi;
    src_span(g, t0, WIN < Lo + K - 1 - t0 ? WIN : Lo + K - 1 - t0, lo, hi);
    // 1. source rows lo .. hi: flat float4 copy (from the float4 boundary at or below the run)
    const int64_t f0 = ((int64_t)b * g.L_in + lo) * g.Cin;
    const int64_t fa = f0 & ~(int64_t)3;
    const int nf = hi >= lo ? (int)(((int64_t)b * g.L_in + hi + 1) * g.Cin - fa) : 0;
    const int nv = (nf + 3) >> 2;
    {
        constexpr int U = 12;
        for (int i0 = tid; i0 < nv; i0 += 256 * U) {
            float4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = i0 + 256 * u;
                const int64_t e = fa + 4 * (int64_t)i;
                if (i < nv && e + 3 < total) {
                    v[u] = *reinterpret_cast<const float4*>(x + e);
                } else {
                    v[u].x = i < nv && e < total ? x[e] : 0.f;
                    v[u].y = i < nv && e + 1 < total ? x[e + 1] : 0.f;
                    v[u].z = i < nv && e + 2 < total ? x[e + 2] : 0.f;
                    v[u].w = 0.f;
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = i0 + 256 * u;
                if (i < nv) reinterpret_cast<float4*>(F)[i] = v[u];
            }
        }
    }
    __syncthreads();
    // 2. the bf16 window of every chunk from F (rows relative to lo, offset f0 - fa): 8 channels
    // of one row per item, one row mapping per item
    {
        const int segs = 4 * nch;
        const int off = (int)(f0 - fa);
        for (int i = tid; i < WIN * segs; i += 256) {
            const int r = i / segs, s = i - r * segs;
            const int tp = t0 + r, cb = 8 * s;
            int i0 = 0, i1 = 0;
            float l1 = 0.f;
            const bool in = tp < Lo + K - 1 && src_row(g, tp, i0, i1, l1);
            const float* p0 = F + off + (in ? i0 - lo : 0) * g.Cin;
            const float* p1 = F + off + (in ? i1 - lo : 0) * g.Cin;
            hv8<H> v;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int c = cb + j < g.Cin ? cb + j : g.Cin - 1;
                float a = p0[c];
                float q = g.up ? p1[c] : 0.f;
                if constexpr (IBN) {
                    a = bn_relu_at(ip, cin32, cb + j, a);
                    q = g.up ? bn_relu_at(ip, cin32, cb + j, q) : 0.f;
                }
                // conv.h src_vec's values
                v[j] = (H)((in && cb + j < g.Cin) ? (g.up ? up_lerp(a, q, l1) : a) : 0.f);
            }
            *(hv8<H>*)(xs + ((s >> 2) * WIN + r) * RS + 8 * (s & 3)) = v;
        }
    }
    __syncthreads();   // F is dead: the taps take its place
    auto store_taps = [&]() {
#pragma unroll
        for (int it = 0; it < C::NWI; ++it) {
            const int i = tid + 256 * it;
            if (i >= K * TC * 4) continue;
            const int oct = i & 3, r = i >> 2, k = r / TC, co = r - k * TC;
            hv8<H> v = wt[it];
            if (co0 + co >= g.Cout) {
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = (H)0.f;
            }
            *(hv8<H>*)(ws + (k * TC + co) * RS + 8 * oct) = v;
        }
    };
    store_taps();
    __syncthreads();
    f32x4 acc[PM][NT];
#pragma unroll
    for (int m = 0; m < PM; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int ch = 0; ch < nch; ++ch) {
        const bool more = ch + 1 < nch;
        if (more) load_taps(32 * (ch + 1));
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
            store_taps();
            __syncthreads();
        }
    }
    // output (D: col (channel) = lane & 15, row (position) = 4 (lane >> 4) + r), as k_conv_bf16
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
        // BatchNorm tile statistics: k_conv_bf16's epilogue, the same order
        float* red1 = reinterpret_cast<float*>(lb);
        float* red2 = red1 + 4 * TC;
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
            const int64_t ntile = (int64_t)gridDim.z * gridDim.x;
            float* sp = stats + (int64_t)(co0 + tid) * ntile + tile;
            sp[0] = ((red1[tid] + red1[TC + tid]) + red1[2 * TC + tid]) + red1[3 * TC + tid];
            sp[(int64_t)g.Cout * ntile] = ((red2[tid] + red2[TC + tid]) + red2[2 * TC + tid]) + red2[3 * TC + tid];
        }
    }
}

// source rows a window of WIN padded positions can read: WIN + 2 (x2 upsample: half, + 2)
template <int K, int NT>
int cfw_nt(const float* x, const Geo& g, const void* w16, float* y, int Lo, float* stats, hipStream_t st,
           const BnIn* ibn) {
    using C = FCfg<K, NT>;
    const int nch = cdiv(g.Cin, 32);
    const int src_rows = g.up ? C::WIN / 2 + 3 : C::WIN;
    const int fbytes = (src_rows * g.Cin + 8) * 4;
    const int rest = fbytes > C::WBYTES ? fbytes : C::WBYTES;
    int lds = nch * C::WIN * RS * 2 + rest;
    if (lds < 8 * C::TC * 4) lds = 8 * C::TC * 4;
    const int ipo = (lds + 15) & ~15;   // the input BatchNorm's parameters (IBN): [4][32 nch] floats
    if (ibn) lds = ipo + 4 * 32 * nch * 4;
    if (lds > 160 * 1024) return VT_ERR_ARG;
    dim3 grid(cdiv(Lo, C::TP), cdiv(g.Cout, C::TC), g.B);
    const int64_t total = (int64_t)g.B * g.L_in * g.Cin;
    const BnIn bi = ibn ? *ibn : BnIn{};
    if (h16_format()) {   // fp16 operands (h16.h); the conv-stack fold (ibn) is bf16-only
        if (ibn) return VT_ERR_ARG;
        hipLaunchKernelGGL((k_cfw16<K, NT, false, _Float16>), grid, dim3(256), lds, st, x, g, nch,
                           (const _Float16*)w16, y, Lo, stats, total, bi, ipo);
    } else if (ibn)
        hipLaunchKernelGGL((k_cfw16<K, NT, true, __bf16>), grid, dim3(256), lds, st, x, g, nch, (const __bf16*)w16, y, Lo, stats,
                           total, bi, ipo);
    else
        hipLaunchKernelGGL((k_cfw16<K, NT, false, __bf16>), grid, dim3(256), lds, st, x, g, nch, (const __bf16*)w16, y, Lo, stats,
                           total, bi, ipo);
    return C::TP;
}

template <int K>
int cfw_k(const float* x, const Geo& g, const void* w16, float* y, int Lo, float* stats, hipStream_t st,
          const BnIn* ibn) {
    switch (cdiv(g.Cout, 16) < 6 ? cdiv(g.Cout, 16) : 6) {
        case 1: return cfw_nt<K, 1>(x, g, w16, y, Lo, stats, st, ibn);
        case 2: return cfw_nt<K, 2>(x, g, w16, y, Lo, stats, st, ibn);
        case 3: return cfw_nt<K, 3>(x, g, w16, y, Lo, stats, st, ibn);
        case 4: return cfw_nt<K, 4>(x, g, w16, y, Lo, stats, st, ibn);
        case 5: return cfw_nt<K, 5>(x, g, w16, y, Lo, stats, st, ibn);
        default: return cfw_nt<K, 6>(x, g, w16, y, Lo, stats, st, ibn);
    }
}

}  // namespace

// the flat-staged forward for geometry g (conv_bf16.hip dispatches here when enabled):
// returns the position tile (> 0, the statistics' tile height), or VT_ERR_ARG when the
// window's source rows do not fit in LDS (the caller uses k_conv_bf16)
int cfw16_launch(const float* x, const Geo& g, const void* w16, float* y, int Lo, float* stats, hipStream_t st,
                 const BnIn* ibn) {
    switch (g.K) {
        case 1: return cfw_k<1>(x, g, w16, y, Lo, stats, st, ibn);
        case 2: return cfw_k<2>(x, g, w16, y, Lo, stats, st, ibn);
        case 3: return cfw_k<3>(x, g, w16, y, Lo, stats, st, ibn);
        case 4: return cfw_k<4>(x, g, w16, y, Lo, stats, st, ibn);
        case 5: return cfw_k<5>(x, g, w16, y, Lo, stats, st, ibn);
        case 6: return cfw_k<6>(x, g, w16, y, Lo, stats, st, ibn);
        case 7: return cfw_k<7>(x, g, w16, y, Lo, stats, st, ibn);
        case 8: return cfw_k<8>(x, g, w16, y, Lo, stats, st, ibn);
        case 9: return cfw_k<9>(x, g, w16, y, Lo, stats, st, ibn);
        case 10: return cfw_k<10>(x, g, w16, y, Lo, stats, st, ibn);
        default: return cfw_k<11>(x, g, w16, y, Lo, stats, st, ibn);
    }
}

}  // namespace vt
