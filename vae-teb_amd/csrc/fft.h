// LDS-resident complex FFT for one workgroup (gfx950, wave64).
//
// Stockham autosort, radix-4 DIF with a final radix-2 stage: ping-pongs
// between two LDS buffers of n float2 (n = 8192 -> 2 x 64 KiB of the 160 KiB
// LDS), output in natural order, no bit reversal.  Butterfly index
// idx = p*s + q makes every stage's four reads unit-stride across lanes
// (addresses idx + k*n/4), so reads are bank-conflict free.
// Twiddles come from a host-built fp64-accurate table W_N^k = exp(-2*pi*i*k/N)
// (global, L2-resident); an FFT of length n = N/stride reads it with `stride`.
#pragma once
#include "common.h"

namespace vt {

template <bool INV>
__device__ __forceinline__ float2 twiddle(const float2* __restrict__ tw, int k) {
    float2 w = tw[k];
    return INV ? make_float2(w.x, -w.y) : w;
}

// In: x holds the sequence.  Returns the buffer holding the (unscaled) result.
// Must be called by all threads of the block; ends with a barrier.
template <bool INV>
__device__ float2* fft_lds(float2* x, float2* y, int n, const float2* __restrict__ tw, int tw_stride) {
    int s = 1, log2s = 0, len = n;
    const int quarter = n >> 2;
    while (len >= 4) {
        const int n1 = len >> 2;
        for (int idx = threadIdx.x; idx < quarter; idx += blockDim.x) {
            const int q = idx & (s - 1);
            const int p = idx >> log2s;
            const int base = q + s * p;
            const float2 a = x[base], b = x[base + s * n1], c = x[base + 2 * s * n1], d = x[base + 3 * s * n1];
            const int k = p * s * tw_stride;
            const float2 w1 = twiddle<INV>(tw, k), w2 = twiddle<INV>(tw, 2 * k), w3 = twiddle<INV>(tw, 3 * k);
            const float2 apc = cadd(a, c), amc = csub(a, c), bpd = cadd(b, d), bmd = csub(b, d);
            const float2 jbmd = make_float2(-bmd.y, bmd.x);  // i * (b - d)
            const int o = q + 4 * s * p;
            y[o] = cadd(apc, bpd);
            y[o + 2 * s] = cmul(w2, csub(apc, bpd));
            if (!INV) {
                y[o + s] = cmul(w1, csub(amc, jbmd));
                y[o + 3 * s] = cmul(w3, cadd(amc, jbmd));
            } else {
                y[o + s] = cmul(w1, cadd(amc, jbmd));
                y[o + 3 * s] = cmul(w3, csub(amc, jbmd));
            }
        }
        __syncthreads();
        float2* t = x; x = y; y = t;
        s <<= 2; log2s += 2; len >>= 2;
    }
    if (len == 2) {
        const int h = n >> 1;
        for (int q = threadIdx.x; q < h; q += blockDim.x) {
            const float2 a = x[q], b = x[q + h];
            y[q] = cadd(a, b);
            y[q + h] = csub(a, b);
        }
        __syncthreads();
        float2* t = x; x = y; y = t;
    }
    return x;
}

// Batched variant: nb independent length-n sequences at x + c * pitch
// (c < nb), for the four-step FFT's column / row passes (an odd pitch in
// float2 keeps the column-major staging reads and writes conflict-free).
template <bool INV>
__device__ float2* fft_lds_batch(float2* x, float2* y, int n, int nb, int pitch, const float2* __restrict__ tw,
                                 int tw_stride) {
    int s = 1, log2s = 0, len = n;
    const int quarter = n >> 2, lq = __builtin_ctz(quarter > 0 ? quarter : 1);
    while (len >= 4) {
        const int n1 = len >> 2;
        for (int it = threadIdx.x; it < nb * quarter; it += blockDim.x) {
            const int c = it >> lq, idx = it & (quarter - 1);
            const float2* xc = x + c * pitch;
            float2* yc = y + c * pitch;
            const int q = idx & (s - 1);
            const int p = idx >> log2s;
            const int base = q + s * p;
            const float2 a = xc[base], b = xc[base + s * n1], cc = xc[base + 2 * s * n1], d = xc[base + 3 * s * n1];
            const int k = p * s * tw_stride;
            const float2 w1 = twiddle<INV>(tw, k), w2 = twiddle<INV>(tw, 2 * k), w3 = twiddle<INV>(tw, 3 * k);
            const float2 apc = cadd(a, cc), amc = csub(a, cc), bpd = cadd(b, d), bmd = csub(b, d);
            const float2 jbmd = make_float2(-bmd.y, bmd.x);
            const int o = q + 4 * s * p;
            yc[o] = cadd(apc, bpd);
            yc[o + 2 * s] = cmul(w2, csub(apc, bpd));
            if (!INV) {
                yc[o + s] = cmul(w1, csub(amc, jbmd));
                yc[o + 3 * s] = cmul(w3, cadd(amc, jbmd));
            } else {
                yc[o + s] = cmul(w1, cadd(amc, jbmd));
                yc[o + 3 * s] = cmul(w3, csub(amc, jbmd));
            }
        }
        __syncthreads();
        float2* t = x; x = y; y = t;
        s <<= 2; log2s += 2; len >>= 2;
    }
    if (len == 2) {
        const int h = n >> 1, lh = __builtin_ctz(h);
        for (int it = threadIdx.x; it < nb * h; it += blockDim.x) {
            const int c = it >> lh, q = it & (h - 1);
            const float2 a = x[c * pitch + q], b = x[c * pitch + q + h];
            y[c * pitch + q] = cadd(a, b);
            y[c * pitch + q + h] = csub(a, b);
        }
        __syncthreads();
        float2* t = x; x = y; y = t;
    }
    return x;
}

}  // namespace vt
