// Scattering1D + phase-harmonic front-end on gfx950.
//
// Data path for one training batch (x: B x 2 x N, ch0 = fhr, ch1 = up):
//   vt_fe_spectrum  reflect-pad + forward FFT (n_pad) per (sample, channel)
//                   -> xhat (B, 2, n_pad) complex64, L2/HBM resident
//   vt_fe_lowpass   S0 = phi-lowpass of the padded signal, decimated by 2^log2T
//   vt_fe_wavelet   one workgroup per (sample, wavelet item): xhat * psi_f ->
//                   inverse FFT in LDS -> (a) the analytic signal slice the
//                   phase path needs, (b) |U1| -> phi-lowpass -> S1 row
//   vt_fe_pairs     one workgroup per (sample, selected pair): accelerated
//                   product, reflect-pad, FFT, x phi, crop, 512-pt iFFT, real
//   vt_fe_normalize log/asinh + per-channel z-score, (B,C,S) -> (B,S,C)
// Reference: ref/kymatio/kymatio/scattering1d/core/scattering1d.py:197-399,
// ref/hdf5_dataset/kymatio_phase_scattering.py:211-301 (+ :303-360 cross),
// ref/hdf5_dataset/hdf5_dataset.py:18-137 (normalisation).
//
// Lowpass identity used for S0/S1 (exact up to an l1 tail < 1e-9 of the
// Gaussian h0 = ifft(phi_0)): kymatio's
//   unpad(irfft(periodize_K(fft_M(U) * phi_k)))  with phi_k = periodize_2^k(phi_0)
// equals the circular correlation of U with h0 sampled on the 2^k grid,
// evaluated every 2^log2T full-rate samples; h0 is even and decays like a
// Gaussian (sigma ~ 25 samples at T = 16), so each output is a short dot
// product read straight from the inverse-FFT result already in LDS.  The phase
// path's crop-to-n_pad/dec low-pass is NOT Gaussian in time (one-sided
// spectrum -> slowly decaying imaginary tail), so it stays in the FFT domain.
#include <math.h>
#include <stdlib.h>

#include <mutex>
#include <vector>

#include "common.h"
#include "cfft.h"
#include "fft.h"

namespace vt {

static constexpr int FE_THREADS = 512;

// ---------------------------------------------------------------- spectrum
__global__ __launch_bounds__(FE_THREADS) void k_fe_spectrum(const float* __restrict__ x, int N, int n_pad,
                                                            int pad_left, int pad_mode,
                                                            const float2* __restrict__ tw,
                                                            float2* __restrict__ xhat) {
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    float2* X = sm;
    float2* Y = sm + n_pad;
    const int64_t row = blockIdx.x;
    const float* xr = x + row * N;
    for (int n = threadIdx.x; n < n_pad; n += blockDim.x) {
        const int s = pad_src(n - pad_left, N, pad_mode);
        X[n] = make_float2(s < 0 ? 0.f : xr[s], 0.f);
    }
    __syncthreads();
    float2* R = fft_lds<false>(X, Y, n_pad, tw, 1);
    float2* o = xhat + row * n_pad;
    for (int n = threadIdx.x; n < n_pad; n += blockDim.x) o[n] = R[n];
}

// ---------------------------------------------------------------- S0 lowpass
// One workgroup per row (and 256 outputs): the padded row (reflect / zero / circular, as
// reflect_idx over [0, n_pad)) is staged once in LDS, then each output's 2 radius + 1 taps
// are read from LDS in the order of k_fe_lowpass (d = -radius .. radius: the same sums and
// bits); the taps h0[|d|] are wave-uniform (scalar loads).  The per-tap modulo and
// reflection of k_fe_lowpass made it latency-bound at ~67 us per launch.
__global__ __launch_bounds__(256) void k_fe_lowpass_lds(const float* __restrict__ x, int64_t x_row_stride, int N,
                                                        int n_pad, int pad_left, const float* __restrict__ h0,
                                                        int radius, int step, int start, int S,
                                                        float* __restrict__ out, int64_t out_row_stride) {
    extern __shared__ float xp[];   // n_pad
    const int64_t row = blockIdx.y;
    const float* xr = x + row * x_row_stride;
    // one reflection at most (the training geometry): no modulo; eight loads in flight
    const bool single = pad_left <= N - 1 && n_pad - pad_left - N <= N - 1;
    for (int n0 = threadIdx.x; n0 < n_pad; n0 += 256 * 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int n = n0 + 256 * u;
            const int i = n - pad_left;
            const int src = single ? (i < 0 ? -i : (i >= N ? 2 * N - 2 - i : i)) : reflect_idx(i, N);
            v[u] = n < n_pad ? xr[src] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (n0 + 256 * u < n_pad) xp[n0 + 256 * u] = v[u];
    }
    __syncthreads();
    const int m = blockIdx.x * 256 + threadIdx.x;
    if (m >= S) return;
    const int c = step * (m + start);
    float acc = 0.f;
    if (c - radius >= 0 && c + radius < n_pad) {
        // unrolled (eight LDS reads and scalar weight loads in flight, not one round trip per
        // tap) with the fma spelled out, as the one-at-a-time loop compiled it: the same bits
#pragma unroll 8
        for (int d = -radius; d <= radius; ++d) acc = fmaf(xp[c - d], h0[d < 0 ? -d : d], acc);
    } else {
        for (int d = -radius; d <= radius; ++d) {
            int n = (c - d) % n_pad;
            if (n < 0) n += n_pad;
            acc += xp[n] * h0[d < 0 ? -d : d];
        }
    }
    out[row * out_row_stride + m] = acc;
}

__global__ void k_fe_lowpass(const float* __restrict__ x, int64_t x_row_stride, int N, int n_pad, int pad_left,
                             const float* __restrict__ h0, int radius, int step, int start, int S,
                             float* __restrict__ out, int64_t out_row_stride) {
    const int64_t row = blockIdx.y;
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= S) return;
    const float* xr = x + row * x_row_stride;
    const int c = step * (m + start);
    float acc = 0.f;
    for (int d = -radius; d <= radius; ++d) {
        int n = c - d;
        n %= n_pad;
        if (n < 0) n += n_pad;
        acc += xr[reflect_idx(n - pad_left, N)] * h0[d < 0 ? -d : d];
    }
    out[row * out_row_stride + m] = acc;
}

// ---------------------------------------------------------------- wavelets
// items: n_items x 5 ints {chan, filter, analytic_slot|-1, s1_channel|-1, k1}
__global__ __launch_bounds__(FE_THREADS) void k_fe_wavelet(
    const float2* __restrict__ xhat, int C, int n_pad, const float* __restrict__ psi, int n_items,
    const int* __restrict__ items, const float2* __restrict__ tw, int N, int pad_left, float2* __restrict__ analytic,
    int n_slots, const float* __restrict__ h0, int radius, int step, int start, int S, float* __restrict__ s1,
    int s1_channels) {
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    float2* X = sm;
    float2* Y = sm + n_pad;
    const int item = blockIdx.x;
    const int64_t b = blockIdx.y;
    const int chan = items[item * 5 + 0], filt = items[item * 5 + 1], slot = items[item * 5 + 2];
    const int s1ch = items[item * 5 + 3], k1 = items[item * 5 + 4];
    const float2* xh = xhat + (b * C + chan) * n_pad;
    const float* ps = psi + (int64_t)filt * n_pad;
    for (int n = threadIdx.x; n < n_pad; n += blockDim.x) X[n] = cscale(xh[n], ps[n]);
    __syncthreads();
    float2* R = fft_lds<true>(X, Y, n_pad, tw, 1);
    const float inv_n = 1.0f / (float)n_pad;
    if (slot >= 0) {
        float2* a = analytic + (b * n_slots + slot) * (int64_t)N;
        for (int i = threadIdx.x; i < N; i += blockDim.x) a[i] = cscale(R[pad_left + i], inv_n);
    }
    if (s1ch >= 0) {
        float* U = reinterpret_cast<float*>(R == X ? Y : X);
        const int M = n_pad >> k1;
        for (int n = threadIdx.x; n < M; n += blockDim.x) {
            const float2 v = cscale(R[n << k1], inv_n);
            U[n] = sqrtf(v.x * v.x + v.y * v.y);
        }
        __syncthreads();
        for (int m = threadIdx.x; m < S; m += blockDim.x) {
            const int c = step * (m + start);
            // n' such that |c - (n' << k1)| <= radius
            const int lo = (c - radius + (1 << k1) - 1) >> k1;  // c - radius >= 0 assumed by host check
            const int hi = (c + radius) >> k1;
            float acc = 0.f;
            for (int n = lo; n <= hi; ++n) {
                int d = c - (n << k1);
                d = d < 0 ? -d : d;
                int nn = n % M;
                if (nn < 0) nn += M;
                acc += U[nn] * h0[d];
            }
            s1[(b * s1_channels + s1ch) * S + m] = acc;
        }
    }
}

// ---------------------------------------------------------------- phase pairs
// Polar analytic slots (round 4): the wavelet kernel stores each analytic
// sample of the 8192-point geometry as {arg(a) / 2 pi, |a|} — accel()'s angle and magnitude,
// computed once per slot sample instead of once per pair — and a pair's accelerated product
// accel(a_i, p) conj(a_j) = |a_i| |a_j| e^{2 pi i (p arg_i - arg_j)} is then one fused angle,
// one range reduction, one cos / sin and a product of magnitudes (no atan polynomial, no
// square root in the pair kernel).
__device__ __forceinline__ float2 polar_rev(float2 a) {
    const float ax = fabsf(a.x), ay = fabsf(a.y);
    const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    const float t = mx > 0.f ? mn * __builtin_amdgcn_rcpf(mx) : 0.f;
    const float s = t * t;
    float r = 0.000390918023f;
    r = fmaf(r, s, -0.00229176274f);
    r = fmaf(r, s, 0.00633099675f);
    r = fmaf(r, s, -0.0115143927f);
    r = fmaf(r, s, 0.016709527f);
    r = fmaf(r, s, -0.0225382969f);
    r = fmaf(r, s, 0.0318085626f);
    r = fmaf(r, s, -0.0530504771f);
    r = fmaf(r, s, 0.159154922f);
    r *= t;
    if (ay > ax) r = 0.25f - r;
    if (a.x < 0.f) r = 0.5f - r;
    r = copysignf(r, a.y);
    return make_float2(r, __builtin_amdgcn_sqrtf(a.x * a.x + a.y * a.y));
}
__device__ __forceinline__ float2 pair_polar(float2 pi, float2 pj, float p) {
    float v = fmaf(pi.x, p, -pj.x);   // revolutions
    v -= rintf(v);
    const float m = pi.y * pj.y;
    return make_float2(m * __builtin_amdgcn_cosf(v), m * __builtin_amdgcn_sinf(v));
}
template <bool POLAR>
__global__ __launch_bounds__(FE_THREADS) void k_fe_pairs(
    const float2* __restrict__ analytic, int n_slots, int N, int n_pad, int pad_left, int n_pairs,
    const int* __restrict__ slot_i, const int* __restrict__ slot_j, const float* __restrict__ power,
    const float2* __restrict__ tw, const float* __restrict__ phi0, int dec, int start, int S, int pad_mode,
    float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    float2* X = sm;
    float2* Y = sm + n_pad;
    const int pair = blockIdx.x;
    const int64_t b = blockIdx.y;
    const float2* ai = analytic + (b * n_slots + slot_i[pair]) * (int64_t)N;
    const float2* aj = analytic + (b * n_slots + slot_j[pair]) * (int64_t)N;
    const float pw = power[pair];
    float* o = out + (b * n_pairs + pair) * (int64_t)S;
    // accelerated product (kymatio_phase_scattering.py:211-218, :282-283)
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
        const float2 u = ai[i], v = aj[i];
        if constexpr (POLAR) {
            Y[i] = pair_polar(u, v, pw);
        } else {
            const float mag = sqrtf(u.x * u.x + u.y * u.y);
            const float ph = atan2f(u.y, u.x) * pw;
            float sn, cs;
            sincosf(ph, &sn, &cs);
            const float2 acc = make_float2(mag * cs, mag * sn);
            Y[i] = cmul(acc, cconj(v));
        }
        if (dec == 0) o[i] = Y[i].x;  // cross_phase_low_pass=False (:356-360): raw real part
    }
    if (dec == 0) return;
    __syncthreads();
    for (int n = threadIdx.x; n < n_pad; n += blockDim.x) {
        const int s = pad_src(n - pad_left, N, pad_mode);
        X[n] = s < 0 ? make_float2(0.f, 0.f) : Y[s];
    }
    __syncthreads();
    float2* R = fft_lds<false>(X, Y, n_pad, tw, 1);
    float2* Z = (R == X) ? Y : X;
    const int nb = n_pad / dec;
    for (int k = threadIdx.x; k < nb; k += blockDim.x) Z[k] = cscale(R[k], phi0[k]);
    __syncthreads();
    float2* Rs = fft_lds<true>(Z, R, nb, tw, dec);
    const float inv = 1.0f / (float)nb;
    for (int m = threadIdx.x; m < S; m += blockDim.x) o[m] = Rs[start + m].x * inv;
}

// ------------------------------------------- pairs, pruned 8192-point FFT
// The low-pass keeps only bins [0, 512) of the 8192-point FFT of the padded
// product (dec = 16), so the transform is decomposed 8192 = 16 x 16 x 32 in
// place (decimation in frequency) and pruned:
//   pass 1  radix-16 over n2 (stride 512), twiddle W_8192^{n1 k2}   (all data)
//   pass 2  radix-16 over n1b (stride 32) inside each 512-block,
//           twiddle W_512^{n1a k'b}                                  (all data)
//   pass 3  only outputs k'a in {0, 1} of the last radix-32 stage   (2/32 of it)
// giving X[k2 + 16 k'b + 256 k'a] = X[k], k < 512 — 3 register-DFT passes over
// LDS instead of 6.5 Stockham passes, in ONE 66 KB buffer (no ping-pong), so
// two workgroups share a CU.  The LDS image pads every 32 elements by one
// (index k2*512 + 32 n1b + n1a -> k2*528 + 33 n1b + n1a): passes 2 and 3 read
// it along n1a and along n1b without bank conflicts.
static constexpr int PR_N = 8192, PR_NB = 512, PR_IMG = 16 * 16 * 33;
static constexpr int PR_T = 512;  // threads of the pair kernel (8 waves: latency hiding at 2 workgroups / CU)

__device__ __forceinline__ int pr_pos(int idx) {  // natural index -> padded LDS position
    return (idx >> 5) * 33 + (idx & 31);
}

// |a| e^{i p arg(a)} for the phase acceleration, in revolutions: atan2 by an
// odd minimax polynomial of atan on [0, 1] (max error 1.3e-7 rad, fp32), the
// angle times p reduced to [-1/2, 1/2] revolution, then the hardware
// v_sin_f32 / v_cos_f32 (sin(2 pi x)).  Same branch convention as atan2f
// (torch.angle): (-1, -0) -> -pi.
__device__ __forceinline__ float2 accel(float2 a, float p) {
    const float ax = fabsf(a.x), ay = fabsf(a.y);
    const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    const float t = mx > 0.f ? mn * __builtin_amdgcn_rcpf(mx) : 0.f;
    const float s = t * t;
    float r = 0.000390918023f;
    r = fmaf(r, s, -0.00229176274f);
    r = fmaf(r, s, 0.00633099675f);
    r = fmaf(r, s, -0.0115143927f);
    r = fmaf(r, s, 0.016709527f);
    r = fmaf(r, s, -0.0225382969f);
    r = fmaf(r, s, 0.0318085626f);
    r = fmaf(r, s, -0.0530504771f);
    r = fmaf(r, s, 0.159154922f);
    r *= t;                                  // atan(t) / (2 pi)
    if (ay > ax) r = 0.25f - r;
    if (a.x < 0.f) r = 0.5f - r;
    r = copysignf(r, a.y);
    float v = r * p;
    v -= rintf(v);
    const float mag = __builtin_amdgcn_sqrtf(a.x * a.x + a.y * a.y);  // v_sqrt_f32 (1 ulp), no IEEE fix-up
    return make_float2(mag * __builtin_amdgcn_cosf(v), mag * __builtin_amdgcn_sinf(v));
}

// the product of a pair's two analytic samples in either storage form
template <bool POLAR>
__device__ __forceinline__ float2 pair_prod(float2 ai, float2 aj, float p) {
    if constexpr (POLAR) return pair_polar(ai, aj, p);
    else return F2(pmulc(C2(accel(ai, p)), C2(aj)));
}

// XCD-aware workgroup order: the hardware deals consecutive workgroups round-robin
// to the 8 XCDs, so the linear id is remapped to give each XCD a contiguous run of
// (sample, pair) items — the pairs of one sample then share that XCD's L2 copy of
// the sample's analytic signals instead of every XCD fetching them.
__device__ __forceinline__ int xcd_item(int L, int total) {
    return (total & 7) == 0 ? (L & 7) * (total >> 3) + (L >> 3) : L;
}

// G: the training geometry (N 4096, reflect pad 2048 each side) with every
// length and pad index a compile-time constant (no bounds checks, the reflection
// of each radix-16 column is known per n2); otherwise the runtime arguments.
// D: product columns formed straight from HBM / L2 (no LDS staging pass).
// P: diagnostic build stamping wave 0's wall clock at each phase boundary into
// stamps[(b * n_pairs + pair) * 8 + phase] (vt_fe_set_pairs_stamps).
// tab: the TW8K_* tables (cfft.h).  One (sample, pair) per workgroup, 1-D grid.
#define PR_STAMP(i)                                                                           \
    do {                                                                                      \
        if constexpr (P) {                                                                    \
            if (t == 0) stamps[((int64_t)b * n_pairs + pair) * 8 + (i)] = wall_clock64();    \
        }                                                                                     \
    } while (0)
static constexpr int PR_ZP = PR_NB + PR_NB / 8;  // padded 512-point buffer (z512_pos)
template <bool G, bool D = false, bool P = false, bool POLAR = true>
__global__ __launch_bounds__(PR_T) void k_fe_pairs8k(
    const float2* __restrict__ analytic, int n_slots, int N_, int pad_left_, int n_pairs, int B,
    const int* __restrict__ slot_i, const int* __restrict__ slot_j, const float* __restrict__ power,
    const float2* __restrict__ tab, const float* __restrict__ phi0, int start, int S, int pad_mode_,
    float* __restrict__ out, unsigned long long* __restrict__ stamps) {
    static_assert(PR_T == 512, "one padded column per thread");
    const int N = G ? 4096 : N_, pad_left = G ? 2048 : pad_left_, pad_mode = G ? 0 : pad_mode_;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    float2* img = sm;               // PR_IMG
    float2* Z = sm + PR_IMG;        // PR_ZP
    const int t = threadIdx.x;
    const int item = xcd_item(blockIdx.x, n_pairs * B);
    const int pair = item % n_pairs;
    const int64_t b = item / n_pairs;
    const float2* ai = analytic + (b * n_slots + slot_i[pair]) * (int64_t)N;
    const float2* aj = analytic + (b * n_slots + slot_j[pair]) * (int64_t)N;
    const float pw = power[pair];
    // pass-3 output bin of this thread and its low-pass weight (loaded up front)
    const int j3 = t & 255, ka = t >> 8, k2_3 = j3 >> 4, kb_3 = j3 & 15;
    const int k3 = k2_3 + 16 * kb_3 + 256 * ka;
    const float ph3 = phi0[k3];
    PR_STAMP(0);
    c2 v[16], w[15];
    // the pass-1 twiddles W_8192^{t k2}: issued before the barriers of the column formation
    // (no dependence on it), so their L2 latency overlaps the waits instead of following them
    auto load_w1 = [&]() {
#pragma unroll
        for (int k2 = 1; k2 < 16; ++k2) w[k2 - 1] = C2(tab[TW8K_T1 + 512 * (k2 - 1) + t]);
    };
    if constexpr (D) {
        load_w1();
        // 0+1 fused (training geometry only): column n1 = t of the reflect-padded product
        // straight from HBM / L2, the product formed in registers (each sample of the
        // signal is visited twice, once per reflection), first radix-16 pass, no staging
        static_assert(G, "direct columns: training geometry");
        float2 xa[16], xb[16];
#pragma unroll
        for (int n2 = 0; n2 < 16; ++n2) {
            const int i = t + 512 * n2 - 2048;
            const int s = n2 < 4 ? -i : (n2 < 12 ? i : 2 * 4096 - 2 - i);
            xa[n2] = ai[s];
            xb[n2] = aj[s];
        }
#pragma unroll
        for (int n2 = 0; n2 < 16; ++n2) v[n2] = C2(pair_prod<POLAR>(xa[n2], xb[n2], pw));
    } else {
        // 0: accelerated product c[u], u < N (kymatio_phase_scattering.py:211-218, :282-283), compact;
        // loads in batches of 8 per thread (all in flight before the first use)
        for (int u0 = t; u0 < N; u0 += PR_T * 8) {
            float2 xa[8], xb[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int u = u0 + PR_T * k;
                xa[k] = (G || u < N) ? ai[u] : make_float2(0.f, 0.f);
                xb[k] = (G || u < N) ? aj[u] : make_float2(0.f, 0.f);
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int u = u0 + PR_T * k;
                if (G || u < N) img[u] = pair_prod<POLAR>(xa[k], xb[k], pw);
            }
        }
        PR_STAMP(1);
        load_w1();
        __syncthreads();
        // 1: column n1 = t of the padded signal (reflect / zero / circular); one
        // reflection at most on the training geometry (no modulo)
        const bool single = pad_mode == 0 && pad_left <= N - 1 && PR_N - pad_left - N <= N - 1;
#pragma unroll
        for (int n2 = 0; n2 < 16; ++n2) {
            const int i = t + 512 * n2 - pad_left;
            const int s = G ? (n2 < 4 ? -i : (n2 < 12 ? i : 2 * N - 2 - i))
                            : single ? (i < 0 ? -i : (i >= N ? 2 * N - 2 - i : i)) : pad_src(i, N, pad_mode);
            v[n2] = s < 0 ? c2{0.f, 0.f} : C2(img[s]);
        }
        __syncthreads();
    }
    {
        pdft16(v);
        img[pr_pos(t)] = F2(v[0]);
#pragma unroll
        for (int k2 = 1; k2 < 16; ++k2) img[pr_pos(t + 512 * k2)] = F2(pmul(v[k2], w[k2 - 1]));
    }
    PR_STAMP(2);
    // the pass-2 twiddles W_512^{n1a kb}, likewise in flight across the barrier
#pragma unroll
    for (int kb = 1; kb < 16; ++kb) w[kb - 1] = C2(tab[TW8K_T2 + 32 * (kb - 1) + (t & 31)]);
    __syncthreads();
    // 2: job (k2, n1a) = (t >> 5, t & 31): radix-16 over n1b inside block k2, in place
    {
        const int k2 = t >> 5, n1a = t & 31;
        float2* base = img + k2 * 528 + n1a;
        c2 x[16];
#pragma unroll
        for (int n1b = 0; n1b < 16; ++n1b) x[n1b] = C2(base[33 * n1b]);
        pdft16(x);
        base[0] = F2(x[0]);
#pragma unroll
        for (int kb = 1; kb < 16; ++kb) base[33 * kb] = F2(pmul(x[kb], w[kb - 1]));
    }
    PR_STAMP(3);
    __syncthreads();
    // 3: (k2, k'b) = (j >> 4, j & 15), j = t & 255: output k'a = t >> 8 (0 or 1) of the
    // radix-32 stage; Z holds conj(X phi0) so that the 512-point inverse below is a
    // forward transform whose real part is the result
    {
        const float2* row = img + k2_3 * 528 + 33 * kb_3;
        c2 x = C2(row[0]);
        if (ka == 0) {
#pragma unroll
            for (int n1a = 1; n1a < 32; ++n1a) x += C2(row[n1a]);
        } else {
#pragma unroll
            for (int n1a = 1; n1a < 32; ++n1a) x = pmac(x, C2(row[n1a]), w32(n1a));  // W_32^{n1a}
        }
        Z[z512_pos(k3)] = make_float2(x.x * ph3, -x.y * ph3);
    }
    PR_STAMP(4);
    // wave 0's 512-point twiddles in flight across the barrier
    c2 w5[7], wb5[7];
    if (t < 64) fft512_twiddles(tab, w5, wb5);
    __syncthreads();
    // 4: inverse FFT of length 512 by wave 0, keep the real part of [start, start + S)
    if (t < 64) {
        c2 r[8];
        wave_fft512(Z, w5, wb5, r);
        PR_STAMP(5);
        float* o = out + (b * n_pairs + pair) * (int64_t)S;
        const float inv = 1.0f / (float)PR_NB;
        const int k0 = (t >> 3) + 8 * (t & 7);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int m = k0 + 64 * j - start;
            if (m >= 0 && m < S) o[m] = r[j].x * inv;
        }
        PR_STAMP(6);
    }
}
#undef PR_STAMP

// Persistent form of k_fe_pairs8k<true> (the training geometry): a grid of 2 workgroups per CU,
// each walking the items L = blockIdx.x, + gridDim.x, ... (gridDim a multiple of 8, so every
// workgroup stays on one XCD and the XCD-aware order keeps each XCD on consecutive items).
// The one-wave 512-point inverse (phase 4) of item i runs on wave 0 while waves 1-7 form item
// i+1's accelerated product (phase 0) in the image, which phase 3 has finished reading — the
// seven other waves no longer idle through the inverse.  Phases 1-4 are k_fe_pairs8k's, the
// product's elements are the same: bit-identical outputs.
static constexpr int PRP_T7 = PR_T - 64;   // threads of waves 1-7
template <bool POLAR>
__device__ __forceinline__ void pr_product_w17(float2* img, const float2* __restrict__ ai,
                                               const float2* __restrict__ aj, float pw, int t7) {
#pragma unroll
    for (int bt = 0; bt < 2; ++bt) {
        float2 xa[5], xb[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const int u = t7 + PRP_T7 * (5 * bt + k);
            if (bt == 0 || u < 4096) {
                xa[k] = ai[u];
                xb[k] = aj[u];
            }
        }
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const int u = t7 + PRP_T7 * (5 * bt + k);
            if (bt == 0 || u < 4096) img[u] = pair_prod<POLAR>(xa[k], xb[k], pw);
        }
    }
}

// (at most 128 VGPRs: two 8-wave workgroups per CU, as the per-item kernel; unconstrained, the
// compiler hoists the twiddle tables out of the item loop and needs 228)
template <bool POLAR>
__global__ __launch_bounds__(PR_T) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_fe_pairs8k_p(
    const float2* __restrict__ analytic, int n_slots, int n_pairs, int B, const int* __restrict__ slot_i,
    const int* __restrict__ slot_j, const float* __restrict__ power, const float2* __restrict__ tab,
    const float* __restrict__ phi0, int start, int S, float* __restrict__ out) {
    constexpr int N = 4096;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    float2* img = sm;               // PR_IMG
    float2* Z = sm + PR_IMG;        // PR_ZP
    const int t = threadIdx.x, total = n_pairs * B;
    const int j3 = t & 255, ka = t >> 8, k2_3 = j3 >> 4, kb_3 = j3 & 15;
    const int k3 = k2_3 + 16 * kb_3 + 256 * ka;
    const float ph3 = phi0[k3];
    auto item_of = [&](int L, int& pair, int64_t& b) {
        const int item = xcd_item(L, total);
        pair = item % n_pairs;
        b = item / n_pairs;
    };
    int L = blockIdx.x;
    int pair;
    int64_t b;
    item_of(L, pair, b);
    if (t >= 64)   // the first item's product (wave 0 has no inverse to run yet)
        pr_product_w17<POLAR>(img, analytic + (b * n_slots + slot_i[pair]) * (int64_t)N,
                       analytic + (b * n_slots + slot_j[pair]) * (int64_t)N, power[pair], t - 64);
    for (; L < total; L += gridDim.x) {
        __syncthreads();   // the product of item L is in img; Z is free (previous inverse done)
        // an opaque copy of the table pointer per item: the twiddle loads stay inside the loop
        // (hoisted, they would hold ~60 VGPRs across it and spill)
        const float2* tb = tab;
        asm volatile("" : "+s"(tb));
        c2 v[16];
#pragma unroll
        for (int n2 = 0; n2 < 16; ++n2) {
            const int i = t + 512 * n2 - 2048;
            const int s = n2 < 4 ? -i : (n2 < 12 ? i : 2 * N - 2 - i);
            v[n2] = C2(img[s]);
        }
        __syncthreads();
        {
            c2 w[15];
#pragma unroll
            for (int k2 = 1; k2 < 16; ++k2) w[k2 - 1] = C2(tb[TW8K_T1 + 512 * (k2 - 1) + t]);
            pdft16(v);
            img[pr_pos(t)] = F2(v[0]);
#pragma unroll
            for (int k2 = 1; k2 < 16; ++k2) img[pr_pos(t + 512 * k2)] = F2(pmul(v[k2], w[k2 - 1]));
        }
        __syncthreads();
        {
            const int k2 = t >> 5, n1a = t & 31;
            float2* base = img + k2 * 528 + n1a;
            c2 w[15], x[16];
#pragma unroll
            for (int kb = 1; kb < 16; ++kb) w[kb - 1] = C2(tb[TW8K_T2 + 32 * (kb - 1) + n1a]);
#pragma unroll
            for (int n1b = 0; n1b < 16; ++n1b) x[n1b] = C2(base[33 * n1b]);
            pdft16(x);
            base[0] = F2(x[0]);
#pragma unroll
            for (int kb = 1; kb < 16; ++kb) base[33 * kb] = F2(pmul(x[kb], w[kb - 1]));
        }
        __syncthreads();
        {
            const float2* row = img + k2_3 * 528 + 33 * kb_3;
            c2 x = C2(row[0]);
            if (ka == 0) {
#pragma unroll
                for (int n1a = 1; n1a < 32; ++n1a) x += C2(row[n1a]);
            } else {
#pragma unroll
                for (int n1a = 1; n1a < 32; ++n1a) x = pmac(x, C2(row[n1a]), w32(n1a));
            }
            Z[z512_pos(k3)] = make_float2(x.x * ph3, -x.y * ph3);
        }
        __syncthreads();   // img is free: waves 1-7 start the next item while wave 0 inverts this one
        const int Ln = L + (int)gridDim.x;
        if (t < 64) {   // wave 0 (wave-uniform branches: the register need is the larger, not the sum)
            c2 r[8];
            wave_fft512(Z, tb, r);
            int st_ = start, S_ = S;
            asm volatile("" : "+s"(st_), "+s"(S_));   // per-item output indices (not hoisted, spilled)
            float* o = out + (b * n_pairs + pair) * (int64_t)S_;
            const float inv = 1.0f / (float)PR_NB;
            const int k0 = (t >> 3) + 8 * (t & 7);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int m = k0 + 64 * j - st_;
                if (m >= 0 && m < S_) o[m] = r[j].x * inv;
            }
        } else if (Ln < total) {
            int np;
            int64_t nb;
            item_of(Ln, np, nb);
            pr_product_w17<POLAR>(img, analytic + (nb * n_slots + slot_i[np]) * (int64_t)N,
                           analytic + (nb * n_slots + slot_j[np]) * (int64_t)N, power[np], t - 64);
        }
        if (Ln < total) item_of(Ln, pair, b);
    }
}

// ------------------------------------------- pairs, half-image form (round 6)
// The same pruned 8192-point transform through HALF the LDS image, so that three 8-wave
// workgroups share a CU (6 waves per SIMD instead of 4: k_fe_pairs8k is issue / latency
// bound at two workgroups per CU, 0.46 of its wave cycles in issue stalls).
//   pass 1  the radix-16 over n2 begins with its radix-2 step: s[n] = v[n] + v[n + 8]
//           feeds the even blocks k2 = 2m, d[n] = (v[n] - v[n + 8]) W_16^n the odd ones
//           (a DFT-8 each).  Passes 2 and 3 never mix blocks, so the 8 blocks of one
//           parity run through ONE 8-block image (34 KB, which first holds the staged
//           product) while the other parity's d[] waits in registers.
//   pass 2  each radix-16 job (block, n1a) split over two waves by output parity (the
//           same radix-2 step, then a DFT-8); the pair reads before a barrier, writes after.
//   pass 3  each (block, k'b) row summed by four lanes, 8 terms each, both outputs
//           k'a = 0, 1 at once, the partials combined by DPP.
// Another DFT-16 factorisation and summation order than k_fe_pairs8k (other rounding);
// held to the same fp64 oracle (kymatio_phase_scattering.py:211-218, :233-273, :275-360).
static constexpr int PRH_IMG = 8 * 528;                           // one parity's 8 blocks, 33-padded
static constexpr int PRH_BUF = PRH_IMG > 4096 ? PRH_IMG : 4096;  // ... aliasing the staged product
static constexpr int PRH_LDS = (PRH_BUF + PR_ZP) * (int)sizeof(float2);

__device__ __forceinline__ c2 w16c(int n) { return w32(2 * n); }  // W_16^n (n a compile-time constant)

// quad butterflies by DPP: lane l receives lane l ^ 1 / l ^ 2 of its quad
__device__ __forceinline__ float qx1(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float qx2(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
}

// reflect-padded source index of column n1 = t, row n2 (training geometry: one reflection)
__device__ __forceinline__ int prh_src(int t, int n2) {
    const int i = t + 512 * n2 - 2048;
    return n2 < 4 ? -i : (n2 < 12 ? i : 2 * 4096 - 2 - i);
}

// blocks k2 = 2m + H (m < 8) from y (pass 1's output of that parity: the DFT-8 and the twiddles
// W_8192^{t k2} already applied in registers, ahead of the barrier that frees the image) to their
// 512 outputs X[k2 + 16 k'b + 256 k'a] (k'a < 2) in Z (conj(X phi), as k_fe_pairs8k).  Enters
// with img free, leaves with pass 3's reads of img possibly still in flight in waves 0-1 (the
// caller's barrier).
// P3: pass-3 form (1: one lane per row on waves 0-1, the default; 0: four lanes per row).  Measured
// and dropped: pass 2 as one thread per radix-16 job on waves 0-3 (no pair split, no middle barrier,
// fewer VALU): 0.78 vs 0.67 ms per launch in the step — four waves cannot hide its 16 LDS reads.
template <int H, int OCC, int P3>
__device__ __forceinline__ void prh_parity(float2* img, float2* Z, const c2 (&y)[8],
                                           const float2* __restrict__ tab, const float* __restrict__ phi0) {
    const int t = threadIdx.x, lane = t & 63;
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
    // phi at this lane's pass-3 outputs (loaded ahead, consumed after two barriers)
    float ph, ph1 = 0.f;
    if constexpr (P3 == 1) {
        const int k3 = (2 * (t >> 4) + H) + 16 * (t & 15);
        ph = t < 128 ? phi0[k3] : 0.f;
        ph1 = t < 128 ? phi0[k3 + 256] : 0.f;
    } else {
        ph = phi0[(2 * (t >> 6) + H) + 16 * ((t >> 2) & 15) + 256 * (t & 1)];
    }
#pragma unroll
    for (int m = 0; m < 8; ++m) img[528 * m + pr_pos(t)] = F2(y[m]);
    {
        // pass 2: wave wv -> output parity p2 = wv & 1 of blocks 2 (wv >> 1) + (lane >> 5), n1a = lane & 31
        const int p2 = wv & 1, n1a = lane & 31;
        float2* base = img + 528 * (2 * (wv >> 1) + (lane >> 5)) + n1a;
        c2 tw[8];
        auto load_tw = [&]() {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int kb = 2 * q + p2;
                if (kb > 0) tw[q] = C2(tab[TW8K_T2 + 32 * (kb - 1) + n1a]);
            }
        };
        if constexpr (OCC == 6) load_tw();   // in flight across the barrier (at 8 waves / SIMD: after it, registers)
        __syncthreads();
        if constexpr (OCC != 6) load_tw();
        c2 x[8];
        if (p2 == 0) {
#pragma unroll
            for (int n = 0; n < 8; ++n) x[n] = C2(base[33 * n]) + C2(base[33 * (n + 8)]);
        } else {
#pragma unroll
            for (int n = 0; n < 8; ++n) {
                const c2 e = C2(base[33 * n]) - C2(base[33 * (n + 8)]);
                x[n] = n == 0 ? e : (n == 4 ? mul_mi(e) : pmul(e, w16c(n)));
            }
        }
        __syncthreads();   // the other parity's wave has read the column too: write in place
        pdft8(x);
        if (p2 == 0) {
            base[0] = F2(x[0]);
#pragma unroll
            for (int q = 1; q < 8; ++q) base[33 * 2 * q] = F2(pmul(x[q], tw[q]));
        } else {
#pragma unroll
            for (int q = 0; q < 8; ++q) base[33 * (2 * q + 1)] = F2(pmul(x[q], tw[q]));
        }
    }
    __syncthreads();
    if constexpr (P3 == 1) {
        // pass 3: one lane per row (block m = t >> 4, k'b = t & 15), waves 0-1 only (the kernel is
        // issue bound: idle waves cost nothing, a row's work split over lanes costs the combine).
        // The two outputs of the 32-point DFT over n1a by two radix-2 folds:
        //   X0 = sum_n x_n,  X1 = sum_{n<8} ((x_n - x_{n+16}) - i (x_{n+8} - x_{n+24})) W_32^n
        if (t < 128) {
            const int m3 = t >> 4, kb3 = t & 15;
            const float2* row = img + 528 * m3 + 33 * kb3;
            c2 x0 = c2{0.f, 0.f}, x1 = c2{0.f, 0.f};
#pragma unroll
            for (int n = 0; n < 8; ++n) {
                const c2 a = C2(row[n]), b = C2(row[n + 8]), c = C2(row[n + 16]), e = C2(row[n + 24]);
                x0 += (a + c) + (b + e);
                const c2 f = add_mi(a - c, b - e);
                x1 = n == 0 ? f : pmac(x1, f, w32(n));
            }
            const int k3 = (2 * m3 + H) + 16 * kb3;
            Z[z512_pos(k3)] = make_float2(x0.x * ph, -x0.y * ph);
            Z[z512_pos(k3 + 256)] = make_float2(x1.x * ph1, -x1.y * ph1);
        }
    } else {
        // pass 3: row (block m = wv, k'b = (t >> 2) & 15), quarter q3 = t & 3 (n1a = 8 q3 + j)
        const int q3 = t & 3, kb3 = (t >> 2) & 15;
        const float2* row = img + 528 * wv + 33 * kb3 + 8 * q3;
        c2 e0 = C2(row[0]), e1 = e0;
#pragma unroll
        for (int j = 1; j < 8; ++j) {
            const c2 v = C2(row[j]);
            e0 += v;
            e1 = pmac(e1, v, w32(j));                // W_32^j
        }
        // W_32^{8 q3} = (-i)^q3
        float rx = (q3 & 1) ? e1.y : e1.x, ry = (q3 & 1) ? -e1.x : e1.y;
        const float sg = (q3 & 2) ? -1.f : 1.f;
        rx *= sg;
        ry *= sg;
        float a0 = e0.x + qx1(e0.x), a1 = e0.y + qx1(e0.y), b0 = rx + qx1(rx), b1 = ry + qx1(ry);
        a0 += qx2(a0);
        a1 += qx2(a1);
        b0 += qx2(b0);
        b1 += qx2(b1);
        if (q3 < 2) {
            const int k3 = (2 * wv + H) + 16 * kb3 + 256 * q3;
            const float xr = q3 ? b0 : a0, xi = q3 ? b1 : a1;
            Z[z512_pos(k3)] = make_float2(xr * ph, -xi * ph);
        }
    }
}

// OCC: waves per SIMD the registers are fitted to (6: three workgroups per CU, 80 VGPRs; 8: four, 64)
template <bool POLAR, int OCC, int P3 = 1>
__global__ __launch_bounds__(PR_T) __attribute__((amdgpu_waves_per_eu(OCC, OCC))) void k_fe_pairs8k_h(
    const float2* __restrict__ analytic, int n_slots, int n_pairs, int B, const int* __restrict__ slot_i,
    const int* __restrict__ slot_j, const float* __restrict__ power, const float2* __restrict__ tab,
    const float* __restrict__ phi0, int start, int S, float* __restrict__ out) {
    constexpr int N = 4096;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    float2* img = sm;              // the staged product (4096), then one parity's blocks (PRH_IMG)
    float2* Z = sm + PRH_BUF;      // PR_ZP
    const int t = threadIdx.x;
    const int item = xcd_item(blockIdx.x, n_pairs * B);
    const int pair = item % n_pairs;
    const int64_t b = item / n_pairs;
    const float2* ai = analytic + (b * n_slots + slot_i[pair]) * (int64_t)N;
    const float2* aj = analytic + (b * n_slots + slot_j[pair]) * (int64_t)N;
    const float pw = power[pair];
    // 0: accelerated product c[u], u < N (kymatio_phase_scattering.py:211-218, :282-283)
    constexpr int LB = OCC == 6 ? 8 : 4;   // loads in flight per batch
#pragma unroll
    for (int k0 = 0; k0 < 8; k0 += LB) {
        float2 xa[LB], xb[LB];
#pragma unroll
        for (int k = 0; k < LB; ++k) {
            xa[k] = ai[t + PR_T * (k0 + k)];
            xb[k] = aj[t + PR_T * (k0 + k)];
        }
#pragma unroll
        for (int k = 0; k < LB; ++k) img[t + PR_T * (k0 + k)] = pair_prod<POLAR>(xa[k], xb[k], pw);
    }
    __syncthreads();
    // 1: column n1 = t of the reflect-padded product, radix-2 step over n2
    c2 s[8], d[8], w[8];
#pragma unroll
    for (int n = 0; n < 8; ++n) {
        const c2 va = C2(img[prh_src(t, n)]), vb = C2(img[prh_src(t, n + 8)]);
        s[n] = va + vb;
        d[n] = va - vb;
    }
#pragma unroll
    for (int n = 1; n < 8; ++n) d[n] = n == 4 ? mul_mi(d[n]) : pmul(d[n], w16c(n));
    // pass 1 of the even blocks in registers while other waves may still read the product
#pragma unroll
    for (int m = 1; m < 8; ++m) w[m] = C2(tab[TW8K_T1 + 512 * (2 * m - 1) + t]);   // W_8192^{t 2m}
    pdft8(s);
#pragma unroll
    for (int m = 1; m < 8; ++m) s[m] = pmul(s[m], w[m]);
    __syncthreads();   // the product is consumed: the image overwrites it
    prh_parity<0, OCC, P3>(img, Z, s, tab, phi0);
    // pass 1 of the odd blocks in registers: waves 2-7 run it while waves 0-1 finish pass 3
#pragma unroll
    for (int m = 0; m < 8; ++m) w[m] = C2(tab[TW8K_T1 + 512 * (2 * m) + t]);       // W_8192^{t (2m + 1)}
    pdft8(d);
#pragma unroll
    for (int m = 0; m < 8; ++m) d[m] = pmul(d[m], w[m]);
    __syncthreads();   // the even blocks' pass 3 has read the image
    prh_parity<1, OCC, P3>(img, Z, d, tab, phi0);
    c2 w5[7], wb5[7];
    if (t < 64) fft512_twiddles(tab, w5, wb5);
    __syncthreads();
    // 4: inverse FFT of length 512 by wave 0, keep the real part of [start, start + S)
    if (t < 64) {
        c2 r[8];
        wave_fft512(Z, w5, wb5, r);
        float* o = out + (b * n_pairs + pair) * (int64_t)S;
        const float inv = 1.0f / (float)PR_NB;
        const int k0 = (t >> 3) + 8 * (t & 7);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int m = k0 + 64 * j - start;
            if (m >= 0 && m < S) o[m] = r[j].x * inv;
        }
    }
}

// ------------------------------------------- wavelets, 8192-point register FFT
// Inverse FFT of xhat * psi for the training geometry (n_pad = 8192) as the
// forward 16 x 16 x 32 decomposition of the pair kernel on conj(input)
// (ifft(X) = conj(fft(conj X))), all three passes full: pass 1 reads the
// spectrum straight from HBM into registers (no LDS staging), passes 2 / 3
// run on the 33-padded LDS image, the result goes back to LDS in natural order
// (padded every 32) for the coalesced analytic-signal copy and the S1
// low-pass.  One 66 KB image: two workgroups per CU (the generic Stockham
// path ping-pongs two 64 KB buffers: one).
__device__ __forceinline__ int nat_pos(int k) { return k + (k >> 5); }  // natural order, padded every 32

template <bool POLAR, bool LP = true>
__global__ __launch_bounds__(PR_T) void k_fe_wavelet8k(
    const float2* __restrict__ xhat, int C, const float* __restrict__ psi, const int* __restrict__ items, int n_items,
    int B, const float2* __restrict__ tab, int N, int pad_left, float2* __restrict__ analytic, int n_slots,
    const float* __restrict__ h0, int radius, int step, int start, int S, float* __restrict__ s1, int s1_channels,
    int nowrap) {
    static_assert(PR_T == 512, "one column per thread");
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    float2* img = sm;  // PR_IMG
    const int t = threadIdx.x;
    const int L = xcd_item(blockIdx.x, n_items * B);  // XCD-aware: one sample's items share an L2
    const int item = L % n_items;
    const int64_t b = L / n_items;
    const int chan = items[item * 5 + 0], filt = items[item * 5 + 1], slot = items[item * 5 + 2];
    const int s1ch = items[item * 5 + 3], k1 = items[item * 5 + 4];
    const float2* xh = xhat + (b * C + chan) * (int64_t)PR_N;
    const float* ps = psi + (int64_t)filt * PR_N;
    // pass 1: column n1 = t of conj(xhat * psi), straight from HBM
    {
        c2 v[16], w[15];
#pragma unroll
        for (int n2 = 0; n2 < 16; ++n2) {
            const int n = t + 512 * n2;
            const float2 x = xh[n];
            const float p = ps[n];
            v[n2] = c2{x.x * p, -x.y * p};
        }
#pragma unroll
        for (int k2 = 1; k2 < 16; ++k2) w[k2 - 1] = C2(tab[TW8K_T1 + 512 * (k2 - 1) + t]);
        pdft16(v);
        img[pr_pos(t)] = F2(v[0]);
#pragma unroll
        for (int k2 = 1; k2 < 16; ++k2) img[pr_pos(t + 512 * k2)] = F2(pmul(v[k2], w[k2 - 1]));
    }
    // the pass-2 twiddles in flight across the barrier (as k_fe_pairs8k)
    c2 w2[15];
#pragma unroll
    for (int kb = 1; kb < 16; ++kb) w2[kb - 1] = C2(tab[TW8K_T2 + 32 * (kb - 1) + (t & 31)]);
    __syncthreads();
    // pass 2: radix-16 over n1b inside block k2 (as k_fe_pairs8k)
    {
        const int k2 = t >> 5, n1a = t & 31;
        float2* base = img + k2 * 528 + n1a;
        c2 x[16];
        const c2* w = w2;
#pragma unroll
        for (int n1b = 0; n1b < 16; ++n1b) x[n1b] = C2(base[33 * n1b]);
        pdft16(x);
        base[0] = F2(x[0]);
#pragma unroll
        for (int kb = 1; kb < 16; ++kb) base[33 * kb] = F2(pmul(x[kb], w[kb - 1]));
    }
    __syncthreads();
    // pass 3: full radix-32 over n1a: X[k2 + 16 kb + 256 ka] (256 jobs)
    const int k2 = (t & 255) >> 4, kb = t & 15;
    c2 r[32];
    if (t < 256) {
        const float2* row = img + k2 * 528 + 33 * kb;
#pragma unroll
        for (int n1a = 0; n1a < 32; ++n1a) r[n1a] = C2(row[n1a]);
        pdft32(r);
    }
    __syncthreads();
    const float inv_n = 1.0f / (float)PR_N;
    if (t < 256) {
#pragma unroll
        for (int ka = 0; ka < 32; ++ka) {
            const int k = k2 + 16 * kb + 256 * ka;
            img[nat_pos(k)] = make_float2(r[ka].x * inv_n, -r[ka].y * inv_n);
        }
    }
    __syncthreads();
    if (slot >= 0) {
        float2* a = analytic + (b * n_slots + slot) * (int64_t)N;
        for (int i = t; i < N; i += PR_T) {
            const float2 v = img[nat_pos(pad_left + i)];
            a[i] = POLAR ? polar_rev(v) : v;
        }
    }
    if (LP && s1ch >= 0) {
        // the S1 low-pass with h0 staged in LDS and |u| of every sample the taps read formed
        // once, in place (the .x of its image entry), instead of a global h0 load and a square
        // root per tap (313 taps at k1 = 0, each sample read by ~20 outputs): the same
        // products summed in the same order as the else branch (the same bits).  Measured
        // 539 -> 419 us per launch, 372 us with the uniform-offset loop below; a residue-major
        // copy of |u| for conflict-free lane reads was slower (431 vs 419 us: its extra pass and
        // barrier cost more than the conflicts)
        const int M = PR_N >> k1;
        float* hl = reinterpret_cast<float*>(img + PR_IMG);
        for (int i = t; i <= radius; i += PR_T) hl[i] = h0[i];
        __syncthreads();   // the analytic copy above is done with the complex values
        for (int n = t; n < M; n += PR_T) {
            const float2 u = img[nat_pos(n << k1)];
            img[nat_pos(n << k1)].x = sqrtf(u.x * u.x + u.y * u.y);
        }
        __syncthreads();
        auto taps = [&](int c, int n0, int n1) {
            float acc = 0.f;
            for (int n = n0; n <= n1; ++n) {
                int d = c - (n << k1);
                d = d < 0 ? -d : d;
                int nn = n;
                if (!nowrap) {
                    nn %= M;
                    if (nn < 0) nn += M;
                }
                acc += img[nat_pos(nn << k1)].x * hl[d];
            }
            return acc;
        };
        if (nowrap && (step >> k1 << k1) == step) {
            // every output's centre c is a multiple of 2^k1: tap n = c / 2^k1 + j, j = -jr .. jr,
            // weight h0[|j| 2^k1] the same for every lane (a scalar load) — the same n order and
            // products as taps() (lo = c / 2^k1 - jr, hi = c / 2^k1 + jr)
            const int jr = radius >> k1;
            for (int m = t; m < S; m += PR_T) {
                const int c0 = (step >> k1) * (m + start);
                float acc = 0.f;
#pragma unroll 8
                for (int j = -jr; j <= jr; ++j) {
                    const int nn = c0 + j;
                    // fmaf spelled out: the unrolled body would otherwise be vectorised into
                    // packed multiplies + adds (two roundings, other bits than taps()'s fma)
                    acc = fmaf(img[nat_pos(nn << k1)].x, h0[(j < 0 ? -j : j) << k1], acc);
                }
                s1[(b * s1_channels + s1ch) * S + m] = acc;
            }
        } else {
            for (int m = t; m < S; m += PR_T) {
                const int c = step * (m + start);
                const int lo = (c - radius + (1 << k1) - 1) >> k1;
                const int hi = (c + radius) >> k1;
                s1[(b * s1_channels + s1ch) * S + m] = taps(c, lo, hi);
            }
        }
    } else if (s1ch >= 0) {
        const int M = PR_N >> k1;
        for (int m = t; m < S; m += PR_T) {
            const int c = step * (m + start);
            const int lo = (c - radius + (1 << k1) - 1) >> k1;
            const int hi = (c + radius) >> k1;
            float acc = 0.f;
            for (int n = lo; n <= hi; ++n) {
                int d = c - (n << k1);
                d = d < 0 ? -d : d;
                int nn = n;
                if (!nowrap) {
                    nn %= M;
                    if (nn < 0) nn += M;
                }
                const float2 u = img[nat_pos(nn << k1)];
                acc += sqrtf(u.x * u.x + u.y * u.y) * h0[d];
            }
            s1[(b * s1_channels + s1ch) * S + m] = acc;
        }
    }
}

// ---------------------------------------------------------------- normalise
// in (B, C, S) raw -> out[b, s, off + c] with row width out_C.
// kind: 0 = z-score only, 1 = log(max(x,0)+eps) then z, 2 = asinh then z.
__global__ void k_fe_normalize(const float* __restrict__ in, int C, int in_C, int in_S, int s0, int S,
                               const int* __restrict__ kind, const float* __restrict__ mean,
                               const float* __restrict__ stdv, float log_eps, float* __restrict__ out, int out_C,
                               int out_off) {
    const int64_t b = blockIdx.y;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= C * S) return;
    const int c = idx % C, s = idx / C;  // consecutive threads -> consecutive output channels
    float v = in[(b * in_C + c) * in_S + s0 + s];
    const int k = kind[c];
    if (k == 1) v = logf(fmaxf(v, 0.f) + log_eps);
    else if (k == 2) v = asinhf(v);
    out[(b * S + s) * out_C + out_off + c] = (v - mean[c]) / (stdv[c] + 1e-8f);
}

__global__ void k_normalize_raw(const float* __restrict__ x, int64_t row_stride, int N, float mean, float stdv,
                                float* __restrict__ out) {
    const int64_t r = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < N) out[r * N + i] = (x[r * row_stride + i] - mean) / (stdv + 1e-8f);
}

// ---------------------------------------------------------------- backend plugin ops
__global__ __launch_bounds__(FE_THREADS) void k_fft_rows(const float2* __restrict__ in, float2* __restrict__ out,
                                                         int n, const float2* __restrict__ tw, int tw_stride,
                                                         int inverse) {
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    float2* X = sm;
    float2* Y = sm + n;
    const int64_t r = blockIdx.x;
    for (int i = threadIdx.x; i < n; i += blockDim.x) X[i] = in[r * n + i];
    __syncthreads();
    float2* R = inverse ? fft_lds<true>(X, Y, n, tw, tw_stride) : fft_lds<false>(X, Y, n, tw, tw_stride);
    const float sc = inverse ? 1.0f / (float)n : 1.0f;
    for (int i = threadIdx.x; i < n; i += blockDim.x) out[r * n + i] = cscale(R[i], sc);
}

// Four-step FFT for n > VT_FFT_MAX_LDS (config 5: Scattering1D J=8 Q=12 on
// N = 16384 -> n_pad = 32768), n = n1 * n2 with n1 = 256 "rows" of n2 columns:
//   pass 1 (k_fft4_cols): 16 adjacent columns j2 per workgroup (128-byte row
//     segments from HBM), length-n1 FFTs over j1 in LDS, twiddle W_n^(j2 k1),
//     write A[k1][j2] (128-byte segments);
//   pass 2 (k_fft4_rows): RB rows k1 per workgroup, length-n2 FFTs over j2,
//     write X[k1 + n1 k2] (RB adjacent k1 per k2 -> RB * 8-byte segments), 1/n
//     for the inverse.
// LDS images are column-major with an odd float2 pitch: the staging writes /
// reads (one element per column across lanes) hit distinct banks and the
// butterflies stay unit-stride within a column.  tw: W_n^k, k < n.
constexpr int F4_N1 = 256, F4_COLS = 16;

__global__ __launch_bounds__(FE_THREADS) void k_fft4_cols(const float2* __restrict__ in, float2* __restrict__ ws,
                                                          int n, int n2, const float2* __restrict__ tw, int inverse) {
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    constexpr int P = F4_N1 + 1;
    float2* X = sm;
    float2* Y = sm + F4_COLS * P;
    const int64_t r = blockIdx.y;
    const int c0 = blockIdx.x * F4_COLS;
    const float2* src = in + r * n + c0;
    for (int i = threadIdx.x; i < F4_N1 * F4_COLS; i += blockDim.x) {
        const int j1 = i / F4_COLS, c = i % F4_COLS;
        X[c * P + j1] = src[(int64_t)j1 * n2 + c];
    }
    __syncthreads();
    float2* R = inverse ? fft_lds_batch<true>(X, Y, F4_N1, F4_COLS, P, tw, n2)
                        : fft_lds_batch<false>(X, Y, F4_N1, F4_COLS, P, tw, n2);
    float2* dst = ws + r * n + c0;
    for (int i = threadIdx.x; i < F4_N1 * F4_COLS; i += blockDim.x) {
        const int k1 = i / F4_COLS, c = i % F4_COLS;
        const int e = (int)(((int64_t)(c0 + c) * k1) & (n - 1));
        const float2 w = inverse ? twiddle<true>(tw, e) : twiddle<false>(tw, e);
        dst[(int64_t)k1 * n2 + c] = cmul(R[c * P + k1], w);
    }
}

__global__ __launch_bounds__(FE_THREADS) void k_fft4_rows(const float2* __restrict__ ws, float2* __restrict__ out,
                                                          int n, int n2, int rb, const float2* __restrict__ tw,
                                                          int inverse) {
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    const int P = n2 + 1;
    float2* X = sm;
    float2* Y = sm + rb * P;
    const int64_t r = blockIdx.y;
    const int k10 = blockIdx.x * rb;
    const float2* src = ws + r * n + (int64_t)k10 * n2;
    for (int i = threadIdx.x; i < rb * n2; i += blockDim.x) {
        const int rr = i / n2, j2 = i - rr * n2;
        X[rr * P + j2] = src[i];
    }
    __syncthreads();
    float2* R = inverse ? fft_lds_batch<true>(X, Y, n2, rb, P, tw, F4_N1)
                        : fft_lds_batch<false>(X, Y, n2, rb, P, tw, F4_N1);
    const float sc = inverse ? 1.0f / (float)n : 1.0f;
    float2* dst = out + r * n + k10;
    for (int i = threadIdx.x; i < rb * n2; i += blockDim.x) {
        const int k2 = i / rb, rr = i - k2 * rb;
        dst[(int64_t)k2 * F4_N1 + rr] = cscale(R[rr * P + k2], sc);
    }
}

__global__ void k_cdgmm(const float2* __restrict__ A, const float* __restrict__ Bf, int b_real,
                        float2* __restrict__ C, int64_t total, int n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int k = (int)(i % n);
    const float2 a = A[i];
    C[i] = b_real ? cscale(a, Bf[k]) : cmul(a, reinterpret_cast<const float2*>(Bf)[k]);
}

__global__ void k_modulus(const float2* __restrict__ in, float* __restrict__ out, int64_t total) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < total) {
        const float2 v = in[i];
        out[i] = sqrtf(v.x * v.x + v.y * v.y);
    }
}

// ModulusStable backward (ref/kymatio/kymatio/backend/torch_backend.py:63-96)
__global__ void k_modulus_bwd(const float2* __restrict__ in, const float* __restrict__ mod,
                              const float* __restrict__ g, float2* __restrict__ gin, int64_t total) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < total) {
        const float m = mod[i];
        gin[i] = m == 0.f ? make_float2(0.f, 0.f) : cscale(in[i], g[i] / m);
    }
}

// mean over k chunks (ref/kymatio/kymatio/scattering1d/backend/torch_backend.py:18-48)
__global__ void k_subsample_fourier(const float2* __restrict__ in, float2* __restrict__ out, int64_t rows, int n,
                                    int k) {
    const int m = n / k;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows * m) return;
    const int64_t r = i / m;
    const int j = (int)(i % m);
    float2 acc = make_float2(0.f, 0.f);
    for (int c = 0; c < k; ++c) acc = cadd(acc, in[r * n + c * m + j]);
    out[i] = cscale(acc, 1.0f / (float)k);
}

__global__ void k_pad_reflect(const float* __restrict__ in, float* __restrict__ out, int64_t rows, int N,
                              int pad_left, int n_out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows * n_out) return;
    const int64_t r = i / n_out;
    const int j = (int)(i % n_out);
    out[i] = in[r * N + reflect_idx(j - pad_left, N)];
}

static inline bool pow2(int n) { return n > 0 && (n & (n - 1)) == 0; }

// The TW8K_* twiddle tables (cfft.h) of the current device, built in fp64 on the
// first training-geometry call (69 KB, synchronous copy: that call must not be
// under stream capture — the first front-end call of a run is eager).
static const float2* tw8k_tables(hipStream_t st) {
    static std::mutex mu;
    static float2* tabs[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    if (tabs[dev] == nullptr) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
        std::vector<float2> h(TW8K_N);
        auto w = [](long m, long n) {
            const double a = -2.0 * M_PI * (double)(m % n) / (double)n;
            return make_float2((float)cos(a), (float)sin(a));
        };
        for (int k = 1; k < 16; ++k)
            for (int n = 0; n < 512; ++n) h[TW8K_T1 + 512 * (k - 1) + n] = w((long)n * k, 8192);
        for (int k = 1; k < 16; ++k)
            for (int n = 0; n < 32; ++n) h[TW8K_T2 + 32 * (k - 1) + n] = w((long)n * k, 512);
        for (int q = 1; q < 8; ++q)
            for (int l = 0; l < 64; ++l) h[TW8K_TA + 64 * (q - 1) + l] = w((long)l * q, 512);
        for (int r = 1; r < 8; ++r)
            for (int l = 0; l < 8; ++l) h[TW8K_TB + 8 * (r - 1) + l] = w((long)l * r, 64);
        float2* d = nullptr;
        if (hipMalloc(&d, sizeof(float2) * TW8K_N) != hipSuccess) return nullptr;
        if (hipMemcpy(d, h.data(), sizeof(float2) * TW8K_N, hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(d);
            return nullptr;
        }
        tabs[dev] = d;
    }
    return tabs[dev];
}
static inline size_t fft_lds_bytes(int n) { return (size_t)2 * n * sizeof(float2); }

}  // namespace vt

using namespace vt;

extern "C" {

int vt_fe_spectrum(const float* x, int64_t rows, int N, int n_pad, int pad_left, int pad_mode, const void* tw,
                   void* xhat, void* stream) {
    VT_CHECK_ARG(pow2(n_pad) && n_pad <= VT_FFT_MAX_LDS && n_pad >= N, "vt_fe_spectrum: n_pad=%d", n_pad);
    VT_CHECK_ARG(rows > 0 && N > 1 && pad_mode >= 0 && pad_mode <= 2, "vt_fe_spectrum: rows/N/pad_mode");
    hipLaunchKernelGGL(k_fe_spectrum, dim3((unsigned)rows), dim3(FE_THREADS), fft_lds_bytes(n_pad), S(stream), x, N,
                       n_pad, pad_left, pad_mode, (const float2*)tw, (float2*)xhat);
    VT_LAUNCH_CHECK("vt_fe_spectrum");
    return VT_OK;
}

int vt_fe_lowpass(const float* x, int64_t rows, int64_t x_row_stride, int N, int n_pad, int pad_left,
                  const float* h0, int radius, int step, int start, int S_out, float* out, int64_t out_row_stride,
                  void* stream) {
    VT_CHECK_ARG(rows > 0 && S_out > 0 && radius >= 0, "vt_fe_lowpass: shape");
    dim3 grid((S_out + 255) / 256, (unsigned)rows);
    if ((size_t)n_pad * sizeof(float) <= 64 * 1024)
        hipLaunchKernelGGL(k_fe_lowpass_lds, grid, dim3(256), (size_t)n_pad * sizeof(float), S(stream), x, x_row_stride,
                           N, n_pad, pad_left, h0, radius, step, start, S_out, out, out_row_stride);
    else
        hipLaunchKernelGGL(k_fe_lowpass, grid, dim3(256), 0, S(stream), x, x_row_stride, N, n_pad, pad_left, h0,
                           radius, step, start, S_out, out, out_row_stride);
    VT_LAUNCH_CHECK("vt_fe_lowpass");
    return VT_OK;
}

// polar analytic slots on the 8192-point geometry (default on; VAETEB_ANALYTIC_POLAR=0 /
// vt_fe_set_analytic_polar(0) keeps the complex form, as every other geometry — DESIGN.md §9); the
// wavelet and the pair entry points decide the form from the same predicate, so a pair launch
// always reads what the wavelet launch wrote
static int g_polar = -1;
static bool analytic_polar(int n_pad, int N, int pad_left) {
    if (g_polar < 0) {
        const char* e = getenv("VAETEB_ANALYTIC_POLAR");
        g_polar = e && e[0] == '0' ? 0 : 1;
    }
    return g_polar && n_pad == PR_N && pad_left + N <= PR_N;
}

int vt_fe_set_analytic_polar(int on) {
    (void)analytic_polar(PR_N, 0, 0);
    const int prev = g_polar;
    g_polar = on ? 1 : 0;
    return prev;
}

int vt_fe_wavelet(const void* xhat, int64_t B, int C, int n_pad, const float* psi, int n_items, const int* items,
                  const void* tw, int N, int pad_left, void* analytic, int n_slots, const float* h0, int radius,
                  int step, int start, int S_out, float* s1, int s1_channels, void* stream) {
    VT_CHECK_ARG(pow2(n_pad) && n_pad <= VT_FFT_MAX_LDS, "vt_fe_wavelet: n_pad=%d", n_pad);
    VT_CHECK_ARG(B > 0 && n_items > 0, "vt_fe_wavelet: empty");
    VT_CHECK_ARG(step * start - radius >= 0, "vt_fe_wavelet: lowpass window leaves the padded support");
    if (n_pad == PR_N && pad_left + N <= PR_N) {
        // the training geometry: register FFT, one 66 KB image
        const int nowrap = step * (start + S_out - 1) + radius < n_pad ? 1 : 0;
        const float2* tab = tw8k_tables(S(stream));
        VT_CHECK_ARG(tab != nullptr, "vt_fe_wavelet: twiddle tables unavailable (first call under stream capture?)");
        VT_CHECK_ARG((int64_t)n_items * B < (1ll << 31), "vt_fe_wavelet: grid");
        // VAETEB_WAVELET_LP=0: the S1 low-pass with a global h0 load and a square root per tap (A/B)
        // (two threads per output with the taps summed in two halves: 411 -> 380 us, but other
        // bits, and the J = 6 end-to-end gradient bound failed on them: not kept)
        static const bool lp_env = !(getenv("VAETEB_WAVELET_LP") && getenv("VAETEB_WAVELET_LP")[0] == '0');
        const bool lp = lp_env && radius < 2048;
        const bool pol = analytic_polar(n_pad, N, pad_left);
        auto kern = pol ? (lp ? k_fe_wavelet8k<true, true> : k_fe_wavelet8k<true, false>)
                        : (lp ? k_fe_wavelet8k<false, true> : k_fe_wavelet8k<false, false>);
        const size_t lds = PR_IMG * sizeof(float2) + (lp ? (size_t)((radius + 4) / 4 * 4) * 4 : 0);
        hipLaunchKernelGGL(kern, dim3((unsigned)(n_items * B)), dim3(PR_T), lds,
                           S(stream), (const float2*)xhat, C, psi, items, n_items, (int)B, tab, N, pad_left,
                           (float2*)analytic, n_slots, h0, radius, step, start, S_out, s1, s1_channels, nowrap);
    } else {
        hipLaunchKernelGGL(k_fe_wavelet, dim3(n_items, (unsigned)B), dim3(FE_THREADS), fft_lds_bytes(n_pad),
                           S(stream), (const float2*)xhat, C, n_pad, psi, n_items, items, (const float2*)tw, N,
                           pad_left, (float2*)analytic, n_slots, h0, radius, step, start, S_out, s1, s1_channels);
    }
    VT_LAUNCH_CHECK("vt_fe_wavelet");
    return VT_OK;
}

static unsigned long long* g_pairs_stamps = nullptr;  // diagnostic phase stamps (nullptr: off)
// persistent pair kernel grid (k_fe_pairs8k_p): VAETEB_PAIRS_PERSIST workgroups (a multiple of 8;
// -1: 2 per CU).  Default 0 = the one-item-per-workgroup kernel: measured in the bench step,
// the persistent form is slower (0.932 vs 0.844 ms per launch, round 4) — bit-identical, kept
// as an option
static int g_pairs_persist = -1;
static int pairs_persist_grid() {
    if (g_pairs_persist < 0) {
        const char* e = getenv("VAETEB_PAIRS_PERSIST");
        int v = e ? atoi(e) : 0;
        if (v < 0) {
            int dev = 0, cus = 256;
            if (hipGetDevice(&dev) == hipSuccess)
                (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
            v = 2 * cus;
        }
        g_pairs_persist = v / 8 * 8;
    }
    return g_pairs_persist;
}
static int g_pairs_direct = -1;  // -1: not yet read from VAETEB_PAIRS_DIRECT
static int pairs_direct() {
    if (g_pairs_direct < 0) {
        const char* e = getenv("VAETEB_PAIRS_DIRECT");
        g_pairs_direct = e != nullptr && e[0] == '1';
    }
    return g_pairs_direct;
}

// Select the pair kernel's product staging on the training geometry (0: LDS-staged
// product, the default; 1: direct columns).  Returns the previous setting.
int vt_fe_set_pairs_persist(int grid) {
    const int prev = pairs_persist_grid();
    if (grid < 0) {
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        grid = 2 * cus;
    }
    g_pairs_persist = grid / 8 * 8;
    return prev;
}

// half-image pair kernel (k_fe_pairs8k_h, three workgroups per CU) on the training geometry:
// VAETEB_PAIRS_HALF=0 selects the full-image k_fe_pairs8k (the form of rounds 2-5)
static int g_pairs_half = -1;
static int pairs_half() {
    if (g_pairs_half < 0) {
        const char* e = getenv("VAETEB_PAIRS_HALF");
        g_pairs_half = e != nullptr ? atoi(e) : 1;
    }
    return g_pairs_half;
}

int vt_fe_set_pairs_half(int on) {
    const int prev = pairs_half();
    g_pairs_half = on < 0 ? 0 : on;   // 2: the 64-VGPR form (four workgroups per CU)
    return prev;
}

int vt_fe_set_pairs_direct(int on) {
    const int prev = pairs_direct();
    g_pairs_direct = on ? 1 : 0;
    return prev;
}

// Diagnostic: stamp the phase boundaries of the training-geometry pair kernel
// (LDS-staged variant) into buf, 8 uint64 per (sample, pair), successive launches
// one after the other; nullptr turns it off.
int vt_fe_set_pairs_stamps(void* buf) {
    g_pairs_stamps = (unsigned long long*)buf;
    return VT_OK;
}

int vt_fe_pairs(const void* analytic, int64_t B, int n_slots, int N, int n_pad, int pad_left, int n_pairs,
                const int* slot_i, const int* slot_j, const float* power, const void* tw, const float* phi0, int dec,
                int start, int S_out, int pad_mode, float* out, void* stream) {
    VT_CHECK_ARG(pow2(n_pad) && n_pad <= VT_FFT_MAX_LDS, "vt_fe_pairs: n_pad=%d", n_pad);
    VT_CHECK_ARG(dec == 0 ? S_out == N : (dec >= 1 && pow2(dec) && n_pad / dec >= start + S_out),
                 "vt_fe_pairs: dec/start (decimation must be a power of two)");
    VT_CHECK_ARG(B > 0 && n_pairs > 0 && pad_mode >= 0 && pad_mode <= 2, "vt_fe_pairs: empty/pad_mode");
    if (dec == PR_N / PR_NB && n_pad == PR_N && start + S_out <= PR_NB && N <= PR_IMG) {
        // the training configuration (n_pad 8192, 512 low-pass bins): pruned transform
        const bool geo = N == 4096 && pad_left == 2048 && pad_mode == 0;
        // direct product columns: faster alone (front-end 2.27 -> 2.10 ms per batch) but
        // slower in the training step, where the phase and cross launches run concurrently
        // and the doubled L2 reads compete (1.19 -> 1.32 ms per launch): opt-in
        const bool direct = pairs_direct() != 0;
        const bool pol = analytic_polar(n_pad, N, pad_left);
        auto kern = pol ? (geo ? (direct ? k_fe_pairs8k<true, true, false, true> : k_fe_pairs8k<true, false, false, true>)
                               : k_fe_pairs8k<false, false, false, true>)
                        : (geo ? (direct ? k_fe_pairs8k<true, true, false, false> : k_fe_pairs8k<true, false, false, false>)
                               : k_fe_pairs8k<false, false, false, false>);
        if (g_pairs_stamps != nullptr && geo && !direct)
            kern = pol ? k_fe_pairs8k<true, false, true, true> : k_fe_pairs8k<true, false, true, false>;
        const float2* tab = tw8k_tables(S(stream));
        VT_CHECK_ARG(tab != nullptr, "vt_fe_pairs: twiddle tables unavailable (first call under stream capture?)");
        VT_CHECK_ARG((int64_t)n_pairs * B < (1ll << 31), "vt_fe_pairs: grid");
        const int64_t total = (int64_t)n_pairs * B;
        const int pgrid = pairs_persist_grid();
        if (geo && !direct && g_pairs_stamps == nullptr && pgrid > 0 && total >= 2 * pgrid) {
            hipLaunchKernelGGL(pol ? k_fe_pairs8k_p<true> : k_fe_pairs8k_p<false>, dim3((unsigned)pgrid), dim3(PR_T),
                               (PR_IMG + PR_ZP) * sizeof(float2),
                               S(stream), (const float2*)analytic, n_slots, n_pairs, (int)B, slot_i, slot_j, power, tab,
                               phi0, start, S_out, out);
            VT_LAUNCH_CHECK("vt_fe_pairs");
            return VT_OK;
        }
        if (geo && !direct && g_pairs_stamps == nullptr && pairs_half()) {
            // 1: 3 workgroups / CU; 2: 4 (64 VGPRs, spills: slower); 3: 3 with the four-lane pass 3
            const int hf = pairs_half();
            hipLaunchKernelGGL(pol ? (hf == 2   ? k_fe_pairs8k_h<true, 8>
                                      : hf == 3 ? k_fe_pairs8k_h<true, 6, 0>
                                                : k_fe_pairs8k_h<true, 6>)
                                   : (hf == 2   ? k_fe_pairs8k_h<false, 8>
                                      : hf == 3 ? k_fe_pairs8k_h<false, 6, 0>
                                                : k_fe_pairs8k_h<false, 6>),
                               dim3((unsigned)total), dim3(PR_T),
                               PRH_LDS, S(stream), (const float2*)analytic, n_slots, n_pairs, (int)B, slot_i, slot_j,
                               power, tab, phi0, start, S_out, out);
            VT_LAUNCH_CHECK("vt_fe_pairs");
            return VT_OK;
        }
        hipLaunchKernelGGL(kern, dim3((unsigned)(n_pairs * B)), dim3(PR_T), (PR_IMG + PR_ZP) * sizeof(float2),
                           S(stream), (const float2*)analytic, n_slots, N, pad_left, n_pairs, (int)B, slot_i, slot_j,
                           power, tab, phi0, start, S_out, pad_mode, out, g_pairs_stamps);
        if (g_pairs_stamps != nullptr && geo && !direct) g_pairs_stamps += (size_t)B * n_pairs * 8;  // next launch after
    } else {
        hipLaunchKernelGGL(analytic_polar(n_pad, N, pad_left) ? k_fe_pairs<true> : k_fe_pairs<false>,
                           dim3(n_pairs, (unsigned)B), dim3(FE_THREADS), fft_lds_bytes(n_pad), S(stream),
                           (const float2*)analytic, n_slots, N, n_pad, pad_left, n_pairs, slot_i, slot_j, power,
                           (const float2*)tw, phi0, dec, start, S_out, pad_mode, out);
    }
    VT_LAUNCH_CHECK("vt_fe_pairs");
    return VT_OK;
}

int vt_fe_normalize_window(const float* in, int64_t B, int C, int in_C, int in_S, int s0, int S_len,
                           const int* kind, const float* mean, const float* stdv, float log_eps, float* out,
                           int out_C, int out_off, void* stream) {
    VT_CHECK_ARG(B > 0 && C > 0 && S_len > 0 && out_off + C <= out_C && in_C >= C && s0 >= 0 && s0 + S_len <= in_S,
                 "vt_fe_normalize_window: shape");
    dim3 grid((C * S_len + 255) / 256, (unsigned)B);
    hipLaunchKernelGGL(k_fe_normalize, grid, dim3(256), 0, S(stream), in, C, in_C, in_S, s0, S_len, kind, mean, stdv,
                       log_eps, out, out_C, out_off);
    VT_LAUNCH_CHECK("vt_fe_normalize_window");
    return VT_OK;
}

int vt_fe_normalize(const float* in, int64_t B, int C, int in_C, int S_len, const int* kind, const float* mean,
                    const float* stdv, float log_eps, float* out, int out_C, int out_off, void* stream) {
    return vt_fe_normalize_window(in, B, C, in_C, S_len, 0, S_len, kind, mean, stdv, log_eps, out, out_C, out_off,
                                  stream);
}

int vt_normalize_raw(const float* x, int64_t rows, int64_t row_stride, int N, float mean, float stdv, float* out,
                     void* stream) {
    VT_CHECK_ARG(rows > 0 && N > 0, "vt_normalize_raw: shape");
    dim3 grid((N + 255) / 256, (unsigned)rows);
    hipLaunchKernelGGL(k_normalize_raw, grid, dim3(256), 0, S(stream), x, row_stride, N, mean, stdv, out);
    VT_LAUNCH_CHECK("vt_normalize_raw");
    return VT_OK;
}

int vt_fft(const void* in, void* out, int64_t rows, int n, int inverse, const void* tw, int tw_stride,
           void* stream) {
    VT_CHECK_ARG(pow2(n) && n <= VT_FFT_MAX_LDS && rows > 0, "vt_fft: n=%d rows=%lld", n, (long long)rows);
    hipLaunchKernelGGL(k_fft_rows, dim3((unsigned)rows), dim3(FE_THREADS), fft_lds_bytes(n), S(stream),
                       (const float2*)in, (float2*)out, n, (const float2*)tw, tw_stride, inverse);
    VT_LAUNCH_CHECK("vt_fft");
    return VT_OK;
}

int vt_fft_large(const void* in, void* out, void* ws, int64_t rows, int n, int inverse, const void* tw,
                 void* stream) {
    VT_CHECK_ARG(pow2(n) && n > VT_FFT_MAX_LDS && n <= (1 << 21) && rows > 0 && rows <= 65535,
                 "vt_fft_large: n=%d rows=%lld (pow2, %d < n <= 2^21)", n, (long long)rows, VT_FFT_MAX_LDS);
    VT_CHECK_ARG(ws != in && ws != out, "vt_fft_large: workspace aliases in/out");
    const int n2 = n / F4_N1;
    int rb = 8192 / n2;
    if (rb > 16) rb = 16;
    hipStream_t st = S(stream);
    hipLaunchKernelGGL(k_fft4_cols, dim3(n2 / F4_COLS, (unsigned)rows), dim3(FE_THREADS),
                       (size_t)2 * F4_COLS * (F4_N1 + 1) * sizeof(float2), st, (const float2*)in, (float2*)ws, n, n2,
                       (const float2*)tw, inverse);
    hipLaunchKernelGGL(k_fft4_rows, dim3(F4_N1 / rb, (unsigned)rows), dim3(FE_THREADS),
                       (size_t)2 * rb * (n2 + 1) * sizeof(float2), st, (const float2*)ws, (float2*)out, n, n2, rb,
                       (const float2*)tw, inverse);
    VT_LAUNCH_CHECK("vt_fft_large");
    return VT_OK;
}

int vt_cdgmm(const void* A, const void* Bf, int b_is_real, void* Cout, int64_t rows, int n, void* stream) {
    VT_CHECK_ARG(rows > 0 && n > 0, "vt_cdgmm: shape");
    const int64_t total = rows * n;
    hipLaunchKernelGGL(k_cdgmm, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, S(stream), (const float2*)A,
                       (const float*)Bf, b_is_real, (float2*)Cout, total, n);
    VT_LAUNCH_CHECK("vt_cdgmm");
    return VT_OK;
}

int vt_modulus(const void* in, float* out, int64_t count, void* stream) {
    VT_CHECK_ARG(count > 0, "vt_modulus: empty");
    hipLaunchKernelGGL(k_modulus, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, S(stream), (const float2*)in,
                       out, count);
    VT_LAUNCH_CHECK("vt_modulus");
    return VT_OK;
}

int vt_modulus_bwd(const void* in, const float* mod, const float* grad, void* grad_in, int64_t count, void* stream) {
    VT_CHECK_ARG(count > 0, "vt_modulus_bwd: empty");
    hipLaunchKernelGGL(k_modulus_bwd, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, S(stream),
                       (const float2*)in, mod, grad, (float2*)grad_in, count);
    VT_LAUNCH_CHECK("vt_modulus_bwd");
    return VT_OK;
}

int vt_subsample_fourier(const void* in, void* out, int64_t rows, int n, int k, void* stream) {
    VT_CHECK_ARG(rows > 0 && k >= 1 && n % k == 0, "vt_subsample_fourier: n=%d k=%d", n, k);
    const int64_t total = rows * (n / k);
    hipLaunchKernelGGL(k_subsample_fourier, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, S(stream),
                       (const float2*)in, (float2*)out, rows, n, k);
    VT_LAUNCH_CHECK("vt_subsample_fourier");
    return VT_OK;
}

int vt_pad_reflect(const float* in, float* out, int64_t rows, int N, int pad_left, int pad_right, void* stream) {
    VT_CHECK_ARG(rows > 0 && N > 1 && pad_left >= 0 && pad_right >= 0, "vt_pad_reflect: shape");
    const int n_out = N + pad_left + pad_right;
    const int64_t total = rows * n_out;
    hipLaunchKernelGGL(k_pad_reflect, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, S(stream), in, out, rows, N,
                       pad_left, n_out);
    VT_LAUNCH_CHECK("vt_pad_reflect");
    return VT_OK;
}

}  // extern "C"
