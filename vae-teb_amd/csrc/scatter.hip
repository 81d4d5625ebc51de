// Batched Scattering1D cascade (orders 1 and 2, average=True): the
// reference's per-filter loop (ref/kymatio/kymatio/scattering1d/core/
// scattering1d.py:197-399: cdgmm -> subsample_fourier -> ifft -> modulus ->
// rfft -> cdgmm(phi) -> subsample_fourier -> irfft -> unpad, one small op per
// filter and per filter pair) regrouped by subsampling level so that one
// launch serves every (sample, filter) row of a level:
//
//   k_scat_filter_sub   Y[b,p,m]  = mean_c A[b, a_idx[p], m + c L] * psi_p[m + c L]
//                       (cdgmm + subsample_fourier fused; A = U0^ or U1^ of the
//                       level, gathered per row; L = n / k)
//   k_scat_mod_spec     U^[row]   = fft(| ifft(Y[row]) |)       (one LDS image;
//                       ifft -> modulus -> rfft of the reference, no HBM
//                       round trip in between)
//   k_scat_lowpass      S[b, ch[p], :] = real(ifft(subsample(U^ . phi, k)))[i0:i1]
//                       (cdgmm + subsample + irfft + unpad, written straight
//                       into the (B, C, S) output at the row's channel)
//
// One workgroup per output row: the fold (cdgmm + subsample) reads the whole
// source row unit-stride across the workgroup, so a level launches B x P
// workgroups whatever its subsampling.  Rows of length <= VT_FFT_MAX_LDS stay
// in LDS from the fold to the spectrum; longer rows (config 5: n_pad = 32768)
// are folded to HBM and go through vt_fft_large + k_modulus_cplx.
#include "fft.h"

namespace vt {

namespace {

constexpr int SC_THREADS = 512;

// One workgroup folds one row: dst[m] = (1/k) sum_c src[m + c L] f[m + c L],
// m < L (cdgmm + subsample_fourier).  L >= SC_THREADS: a thread per bin, c
// serial; L < SC_THREADS: G = SC_THREADS / L threads per bin take every G-th c
// and their partials are summed in fixed order through `red` (LDS, SC_THREADS
// float2).  Reads are unit-stride across the workgroup either way.  Ends with
// a barrier when dst is LDS.
template <bool DST_LDS>
__device__ __forceinline__ void fold_row(const float2* __restrict__ src, const float* __restrict__ f, int L, int k,
                                         float2* dst, float2* red) {
    const int t = threadIdx.x;
    const float sc = 1.0f / (float)k;
    if (L >= SC_THREADS) {
        for (int m = t; m < L; m += SC_THREADS) {
            float2 s = make_float2(0.f, 0.f);
            for (int c = 0; c < k; ++c) s = cadd(s, cscale(src[(int64_t)c * L + m], f[(int64_t)c * L + m]));
            dst[m] = cscale(s, sc);
        }
        if (DST_LDS) __syncthreads();
        return;
    }
    const int G = SC_THREADS / L;   // L, SC_THREADS powers of two
    const int m = t % L, g = t / L;
    float2 s = make_float2(0.f, 0.f);
    for (int c = g; c < k; c += G) s = cadd(s, cscale(src[(int64_t)c * L + m], f[(int64_t)c * L + m]));
    red[t] = s;
    __syncthreads();
    if (t < L) {
        float2 a = red[t];
        for (int gg = 1; gg < G; ++gg) a = cadd(a, red[gg * L + t]);
        dst[t] = cscale(a, sc);
    }
    __syncthreads();
}

// row r = (b, p): fold A[b, a_idx[p]] (length n) with filter p into out[r] (length n / k)
__global__ __launch_bounds__(SC_THREADS) void k_scat_filter_sub(const float2* __restrict__ A, int64_t a_rows, int n,
                                                                const int* __restrict__ a_idx,
                                                                const float* __restrict__ pool,
                                                                const int64_t* __restrict__ f_off, int P, int k,
                                                                float2* __restrict__ out) {
    __shared__ float2 red[SC_THREADS];
    const int64_t r = blockIdx.x, b = r / P;
    const int p = (int)(r - b * P), L = n / k;
    fold_row<false>(A + (b * a_rows + a_idx[p]) * n, pool + f_off[p], L, k, out + r * L, red);
}

// row r = (b, p): fold as above into LDS (L = n / k <= VT_FFT_MAX_LDS), ifft (1/L) -> |.| -> fft
__global__ __launch_bounds__(SC_THREADS) void k_scat_mod_spec(const float2* __restrict__ A, int64_t a_rows, int n,
                                                              const int* __restrict__ a_idx,
                                                              const float* __restrict__ pool,
                                                              const int64_t* __restrict__ f_off, int P, int k,
                                                              const float2* __restrict__ tw,
                                                              float2* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    const int L = n / k;
    float2* red = sm;
    float2* X = sm + SC_THREADS;
    float2* Y = X + L;
    const int64_t r = blockIdx.x, b = r / P;
    const int p = (int)(r - b * P);
    fold_row<true>(A + (b * a_rows + a_idx[p]) * n, pool + f_off[p], L, k, X, red);
    float2* R = fft_lds<true>(X, Y, L, tw, 1);
    float2* T = R == X ? Y : X;
    const float sc = 1.0f / (float)L;
    for (int i = threadIdx.x; i < L; i += SC_THREADS) {
        const float2 z = R[i];
        R[i] = make_float2(sqrtf(z.x * z.x + z.y * z.y) * sc, 0.f);   // |z / L| = |z| / L
    }
    __syncthreads();
    R = fft_lds<false>(R, T, L, tw, 1);
    float2* dst = out + r * L;
    for (int i = threadIdx.x; i < L; i += SC_THREADS) dst[i] = R[i];
}

// row r = (b, p): fold U[r] (length n) with phi into LDS (Lp = n / k), ifft (1/Lp),
// real part of [i0, i1) -> out[b][ch[p]][:]
__global__ __launch_bounds__(SC_THREADS) void k_scat_lowpass(const float2* __restrict__ U, int P, int n,
                                                             const float* __restrict__ phi, int k, int i0, int i1,
                                                             const int* __restrict__ ch, int out_C,
                                                             const float2* __restrict__ tw, float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    const int Lp = n / k;
    float2* red = sm;
    float2* X = sm + SC_THREADS;
    float2* Y = X + Lp;
    const int64_t r = blockIdx.x, b = r / P;
    const int p = (int)(r - b * P);
    fold_row<true>(U + r * n, phi, Lp, k, X, red);
    const float2* R = fft_lds<true>(X, Y, Lp, tw, 1);
    const int S = i1 - i0;
    const float sc = 1.0f / (float)Lp;
    float* dst = out + (b * out_C + ch[p]) * S;
    for (int t = threadIdx.x; t < S; t += SC_THREADS) dst[t] = R[i0 + t].x * sc;
}

__global__ void k_modulus_cplx(const float2* __restrict__ in, float2* __restrict__ out, int64_t total) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < total) {
        const float2 z = in[i];
        out[i] = make_float2(sqrtf(z.x * z.x + z.y * z.y), 0.f);
    }
}

inline bool pow2i(int64_t v) { return v > 0 && (v & (v - 1)) == 0; }

}  // namespace
}  // namespace vt

using namespace vt;

extern "C" {

int vt_scat_filter_sub(const void* A, int B, int64_t a_rows, int n, const int* a_idx, const float* pool,
                       const int64_t* f_off, int P, int k, void* out, void* stream) {
    VT_CHECK_ARG(B > 0 && a_rows > 0 && P > 0 && pow2i(n) && pow2i(k) && k <= n, "vt_scat_filter_sub: n=%d k=%d", n,
                 k);
    hipLaunchKernelGGL(k_scat_filter_sub, dim3((unsigned)((int64_t)B * P)), dim3(SC_THREADS), 0, S(stream),
                       (const float2*)A, a_rows, n, a_idx, pool, f_off, P, k, (float2*)out);
    VT_LAUNCH_CHECK("vt_scat_filter_sub");
    return VT_OK;
}

int vt_scat_mod_spec(const void* A, int B, int64_t a_rows, int n, const int* a_idx, const float* pool,
                     const int64_t* f_off, int P, int k, const void* tw, void* out, void* stream) {
    VT_CHECK_ARG(B > 0 && a_rows > 0 && P > 0 && pow2i(n) && pow2i(k) && n / k >= 4 && n / k <= VT_FFT_MAX_LDS,
                 "vt_scat_mod_spec: n=%d k=%d", n, k);
    const int L = n / k;
    hipLaunchKernelGGL(k_scat_mod_spec, dim3((unsigned)((int64_t)B * P)), dim3(SC_THREADS),
                       (size_t)(SC_THREADS + 2 * L) * sizeof(float2), S(stream), (const float2*)A, a_rows, n, a_idx,
                       pool, f_off, P, k, (const float2*)tw, (float2*)out);
    VT_LAUNCH_CHECK("vt_scat_mod_spec");
    return VT_OK;
}

int vt_scat_lowpass(const void* U, int B, int P, int n, const float* phi, int k, int i0, int i1, const int* ch,
                    int out_C, const void* tw, float* out, void* stream) {
    VT_CHECK_ARG(B > 0 && P > 0 && pow2i(n) && pow2i(k) && n / k >= 4 && n / k <= VT_FFT_MAX_LDS && 0 <= i0 &&
                     i0 < i1 && i1 <= n / k && out_C > 0,
                 "vt_scat_lowpass: n=%d k=%d [%d, %d)", n, k, i0, i1);
    const int Lp = n / k;
    hipLaunchKernelGGL(k_scat_lowpass, dim3((unsigned)((int64_t)B * P)), dim3(SC_THREADS),
                       (size_t)(SC_THREADS + 2 * Lp) * sizeof(float2), S(stream), (const float2*)U, P, n, phi, k, i0,
                       i1, ch, out_C, (const float2*)tw, out);
    VT_LAUNCH_CHECK("vt_scat_lowpass");
    return VT_OK;
}

int vt_modulus_cplx(const void* in, void* out, int64_t count, void* stream) {
    VT_CHECK_ARG(count > 0, "vt_modulus_cplx: empty");
    hipLaunchKernelGGL(k_modulus_cplx, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, S(stream),
                       (const float2*)in, (float2*)out, count);
    VT_LAUNCH_CHECK("vt_modulus_cplx");
    return VT_OK;
}

}  // extern "C"
