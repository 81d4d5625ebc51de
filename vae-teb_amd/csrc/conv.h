// Conv1d geometry shared by the fp32 (conv.hip) and bf16 (conv_bf16.hip)
// kernels: padding / x2 linear upsampling applied while an operand window is
// staged (ref/model/vae_teb_model.py:128-253).
#pragma once
#include "bnbwd.h"
#include "common.h"

namespace vt {

struct Geo {
    int B, L_in, Cin, Cout, K, up, mode, L_up, pad, L_out;
};

// the x2 linear upsample's value between source samples a, b (weight l1 on b): one
// definition with contraction off, so every kernel that stages an upsampled window
// (bf16 forward / weight gradient, the flat-staged forward) rounds it identically
__device__ __forceinline__ float up_lerp(float a, float b, float l1) {
#pragma clang fp contract(off)
    return (1.f - l1) * a + l1 * b;
}

// input value at padded position tp (upsampled domain) — see gemm.hip conv_src.  IBN: x holds
// the previous block's pre-BN conv output, its BatchNorm + activation (LDS parameters ip, channel
// stride cs) applied to each source sample before the interpolation (zero padding stays 0)
template <bool IBN = false>
__device__ __forceinline__ float src_val(const float* __restrict__ xb, const Geo& g, int tp, int ci,
                                         const float* ip = nullptr, int cs = 0, int iact = 0) {
    int t = tp - g.pad;
    if (g.mode == 0) {
        if (t < 0 || t >= g.L_up) return 0.f;
    } else if (g.L_up <= g.pad) {
        t = t < 0 ? 0 : (t >= g.L_up ? g.L_up - 1 : t);
    } else {
        t = t < 0 ? -t : t;
        t = t >= g.L_up ? 2 * (g.L_up - 1) - t : t;
    }
    if (!g.up) {
        const float v = xb[(int64_t)t * g.Cin + ci];
        return IBN ? bn_relu_at(ip, cs, ci, v) : v;
    }
    float s = (t + 0.5f) * 0.5f - 0.5f;
    s = s < 0.f ? 0.f : s;
    const int i0 = (int)s;
    const int i1 = i0 + 1 < g.L_in ? i0 + 1 : g.L_in - 1;
    const float l1 = s - (float)i0;
    float a = xb[(int64_t)i0 * g.Cin + ci], b = xb[(int64_t)i1 * g.Cin + ci];
    if constexpr (IBN) {
        a = bn_relu_at(ip, cs, ci, a);
        b = bn_relu_at(ip, cs, ci, b);
    }
    return up_lerp(a, b, l1);
}


// Source row(s) of padded position tp, the per-row part of src_val: false for
// a zero-padded position; else x row i0 (and i1 with weight l1 when
// upsampling: value = (1 - l1) x[i0] + l1 x[i1], as src_val).
__device__ __forceinline__ bool src_row(const Geo& g, int tp, int& i0, int& i1, float& l1) {
    int t = tp - g.pad;
    if (g.mode == 0) {
        if (t < 0 || t >= g.L_up) return false;
    } else if (g.L_up <= g.pad) {
        t = t < 0 ? 0 : (t >= g.L_up ? g.L_up - 1 : t);
    } else {
        t = t < 0 ? -t : t;
        t = t >= g.L_up ? 2 * (g.L_up - 1) - t : t;
    }
    if (!g.up) {
        i0 = i1 = t;
        l1 = 0.f;
        return true;
    }
    float s = (t + 0.5f) * 0.5f - 0.5f;
    s = s < 0.f ? 0.f : s;
    i0 = (int)s;
    i1 = i0 + 1 < g.L_in ? i0 + 1 : g.L_in - 1;
    l1 = s - (float)i0;
    return true;
}

// source rows [lo, hi] of input x (B, L_in, Cin) that padded positions [t0, t0 + n) read
// (conv.h src_row over the range): the up-domain rows t = tp - pad map monotonically in the
// interior, reflect (mode 1, L_up > pad) folds t < 0 onto [1, pad] and t >= L_up onto
// [L_up - 1 - pad, L_up - 2], replicate (L_up <= pad) stays within [0, L_up), zero padding
// (mode 0) reads nothing outside; the x2 upsample reads rows i0(t) .. i1(t) around t / 2
__device__ __forceinline__ void src_span(const Geo& g, int t0, int n, int& lo, int& hi) {
    const int ta = t0 - g.pad, tz = t0 + n - 1 - g.pad;
    int a = 0x7fffffff, z = -1;
    if (g.mode == 0) {
        a = ta > 0 ? ta : 0;
        z = tz < g.L_up - 1 ? tz : g.L_up - 1;
    } else if (g.L_up <= g.pad) {
        a = 0;
        z = g.L_up - 1;
    } else {
        if (tz >= 0 && ta <= g.L_up - 1) {
            a = ta > 0 ? ta : 0;
            z = tz < g.L_up - 1 ? tz : g.L_up - 1;
        }
        if (ta < 0) {
            const int l = -tz > 1 ? -tz : 1;
            a = l < a ? l : a;
            z = -ta > z ? -ta : z;
        }
        if (tz >= g.L_up) {
            const int l = 2 * (g.L_up - 1) - tz;
            const int h = 2 * (g.L_up - 1) - (ta > g.L_up ? ta : g.L_up);
            a = l < a ? l : a;
            z = h > z ? h : z;
        }
    }
    if (z < a) {
        lo = 0;
        hi = -1;
        return;
    }
    if (!g.up) {
        lo = a;
        hi = z;
        return;
    }
    float sa = (a + 0.5f) * 0.5f - 0.5f, sz = (z + 0.5f) * 0.5f - 0.5f;
    sa = sa < 0.f ? 0.f : sa;
    sz = sz < 0.f ? 0.f : sz;
    lo = (int)sa;
    hi = (int)sz + 1 < g.L_in ? (int)sz + 1 : g.L_in - 1;
}

// NC consecutive channels cb .. cb + NC - 1 of padded position tp (src_val for each,
// 0 where !ok or past Cin) with every load issued before any use: the row mapping
// is computed once, addresses are clamped into the sample and the values masked
// afterwards, so a staging loop keeps all its loads in flight instead of waiting
// on each element.
template <int NC, bool IBN = false>
__device__ __forceinline__ void src_vec(const float* __restrict__ xb, const Geo& g, int tp, int cb, bool ok,
                                        float (&v)[NC], const float* ip = nullptr, int cs = 0, int iact = 0) {
    int i0 = 0, i1 = 0;
    float l1 = 0.f;
    const bool in = ok && src_row(g, tp, i0, i1, l1);
    const float* p0 = xb + (int64_t)(in ? i0 : 0) * g.Cin;
    const float* p1 = xb + (int64_t)(in ? i1 : 0) * g.Cin;
    float a[NC], b[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        const int c = cb + j < g.Cin ? cb + j : g.Cin - 1;
        a[j] = p0[c];
        b[j] = g.up ? p1[c] : 0.f;
    }
    if constexpr (IBN) {   // channels past Cin: padding parameters, masked below
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            a[j] = bn_relu_at(ip, cs, cb + j, a[j]);
            b[j] = g.up ? bn_relu_at(ip, cs, cb + j, b[j]) : 0.f;
        }
    }
#pragma unroll
    for (int j = 0; j < NC; ++j)
        v[j] = (in && cb + j < g.Cin) ? (g.up ? up_lerp(a[j], b[j], l1) : a[j]) : 0.f;
}

static inline Geo geo(int B, int L_in, int Cin, int Cout, int K, int mode, int up) {
    Geo g;
    g.B = B; g.L_in = L_in; g.Cin = Cin; g.Cout = Cout; g.K = K; g.mode = mode; g.up = up;
    g.L_up = L_in * (up ? 2 : 1);
    g.pad = mode == 0 ? K - 1 : (K - 1) / 2;
    g.L_out = mode == 0 ? g.L_up : g.L_up + 2 * g.pad - K + 1;
    return g;
}


static inline int cdiv(int a, int b) { return (a + b - 1) / b; }

int bn_stats_finalize_launch(const float* stats, int tiles_per_sample, int B, int TP, int Lo, int C, float eps,
                             float momentum, float* mean, float* rstd, float* run_mean, float* run_var,
                             hipStream_t st);
// out (+)= the fixed-order sum of `splits` slabs of n floats; (pK, pCo, pCi) != 0: the slabs are
// in [k][o][i] order and out in [o][i][k] (the classifier's bf16 weight gradient)
int sum_splits_launch(const float* part, int splits, int64_t n, float* out, int accumulate, hipStream_t st,
                      int pK = 0, int pCo = 0, int pCi = 0);
// conv_fwd16.hip: the flat-staged bf16 forward (returns its position tile, or VT_ERR_ARG);
// ibn (nullable): x is the previous block's pre-BN output, its BatchNorm + act applied in staging
int cfw16_launch(const float* x, const Geo& g, const void* w16, float* y, int Lo, float* stats, hipStream_t st,
                 const BnIn* ibn = nullptr);
// conv_bf16.hip: the reflect mirror rows of a direct-dX backward-data conv added back (k_conv_fold_edges)
void fold_edges_launch(float* dx, const float* edge, int B, int L, int pad, int C, hipStream_t st);
int bn_apply_launch(const float* x, int64_t M, int C, const float* mean, const float* rstd, const float* gamma,
                    const float* beta, int act, float* y, hipStream_t st);

}  // namespace vt
