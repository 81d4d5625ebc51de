#include <stdlib.h>
// LSTM recurrence for the encoders' nn.LSTM(in, 64, 4 layers, batch_first)
// (ref/model/vae_teb_model.py:474-480, :647-653).
//
// Per layer the time-parallel parts are GEMMs (gemm.hip): the input
// projection G = X W_ih^T + b_ih for all t before the recurrence, and after
// the backward recurrence dW_ih = dG^T X, dW_hh = dG^T H_prev, db = sum dG,
// dX = dG W_ih.  Only the true recurrence runs here: one workgroup of 4H = 256
// threads per sample walks t = 0..S-1 with its W_hh row (forward) or W_hh
// column slice (backward) held in 64 VGPRs, h in LDS, one barrier pair per
// step; B = 256 samples fill the 256 CUs.  Gate order i, f, g, o (PyTorch).
#include <math.h>

#include "common.h"
#include "lstm_cell.h"
#include "skinny.h"

namespace vt {

static constexpr int H = 64;
static constexpr int G4 = 4 * H;

// The cell's transcendentals: the hardware forms of lstm_cell.h by default; built with
// -DVT_LSTM_LIBM=1 the libm forms (sigm_ieee / tanh_ieee).  Round 6 measured both against the
// fp64 oracle: the libm forms are not closer — the fp32 step at B = 256 and the
// S = 256 / 300 goldens scatter with the LSTM's last-bit rounding as the oracle's own one-ulp
// perturbed fp32 runs do — so the faster hardware forms stay.
#ifndef VT_LSTM_LIBM
#define VT_LSTM_LIBM 0
#endif
__device__ __forceinline__ float c_sigm(float x) { return VT_LSTM_LIBM ? sigm_ieee(x) : sigm(x); }
__device__ __forceinline__ float c_tanh(float x) { return VT_LSTM_LIBM ? tanh_ieee(x) : ftanh(x); }

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS traffic,
// not for its global stores / prefetch loads (__syncthreads() would drain
// vmcnt every time step and put an HBM round trip on the recurrence's
// critical path).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

static constexpr int TS = 16;  // time steps per staged chunk

typedef float f2 __attribute__((ext_vector_type(2)));

// DPP quad broadcast: every lane of a 4-lane quad receives lane Q's value
template <int Q>
__device__ __forceinline__ float quad_bcast(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), Q * 0x55, 0xF, 0xF,
                                                                 false));
}

// fixed-order quad sum ((l0 + l1) + (l2 + l3)), the same value in all 4 lanes
__device__ __forceinline__ float quad_sum(float v) {
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
    return v;
}

// h / dg vectors in LDS are stored in 16-float segments padded to 20 floats,
// so float4 reads of different segments by the lanes of a wave hit distinct
// banks (at most 2-way on 16 segments).
__device__ __forceinline__ int seg_pos(int k) { return k + ((k >> 4) << 2); }

// Forward.  Thread j = 4u + q computes, for the 4 gate rows of unit u, the
// partial dot products over k in [16q, 16q + 16) (W_hh[g*H + u][16q .. +16) in
// 32 packed VGPR pairs): only 4 float4 LDS reads of h per thread and step (the
// LDS return path, not the FMAs, bounded the full 64-long per-thread dots).  A
// DPP quad all-reduce completes the 4 gate pre-activations in every lane of
// the quad; each lane then has all gates of its unit (c is carried in every
// lane) and lane 0 publishes h (double-buffered: ONE barrier per time step).
// gin:   [B, S, 4H]  x W_ih^T + b_ih (precomputed)
// out_h: [B, S, H]; out_hprev: [B, S, H] (h_{t-1}, zeros at t = 0)
// out_c: [B, S, H] cell states; gates: [B, S, 4H] post-activation (i, f, g~, o)
// gin is loaded a chunk of TS steps ahead into registers and a chunk's outputs
// are staged in LDS and written in one coalesced burst.
__global__ __launch_bounds__(G4) void k_lstm_fwd(const float* __restrict__ gin, const float* __restrict__ whh,
                                                 const float* __restrict__ bhh, int S, float* __restrict__ out_h,
                                                 float* __restrict__ out_hprev, float* __restrict__ out_c,
                                                 float* __restrict__ gates) {
    __shared__ __attribute__((aligned(16))) float hbuf[2][80];
    __shared__ float og[TS * G4];                      // gates of the chunk
    __shared__ float oh[TS * H], ohp[TS * H], oc[TS * H];
    const int j = threadIdx.x, u = j >> 2, q = j & 3;
    const int row = q * H + u;                         // this lane's gate row (gin / gates column)
    const int64_t b = blockIdx.x;
    f2 w[4][8];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int k = 0; k < 8; ++k)
            w[g][k] = f2{whh[(g * H + u) * H + 16 * q + 2 * k], whh[(g * H + u) * H + 16 * q + 2 * k + 1]};
    const float bias = bhh[row];
    if (j < 80) hbuf[0][j] = 0.f;
    float c = 0.f, hprev = 0.f;  // h_{t-1} of unit u, kept in the publishing lane (no LDS read back)
    const float* g_in = gin + b * (int64_t)S * G4;
    float* gt = gates + b * (int64_t)S * G4;
    const int64_t hb = b * (int64_t)S * H;
    float cur[TS], nxt[TS];
#pragma unroll
    for (int i = 0; i < TS; ++i) cur[i] = g_in[(int64_t)(i < S ? i : S - 1) * G4 + row];
    lds_barrier();
    for (int t0 = 0; t0 < S; t0 += TS) {
#pragma unroll
        for (int i = 0; i < TS; ++i) {  // unconditional (clamped) loads: no per-step waits
            const int t = t0 + TS + i;
            nxt[i] = g_in[(int64_t)(t < S ? t : S - 1) * G4 + row];
        }
        const int n = S - t0 < TS ? S - t0 : TS;
#pragma unroll
        for (int i = 0; i < TS; ++i) {
            if (i >= n) continue;  // block-uniform
            const float* hc = hbuf[i & 1];   // TS even: parity of i == parity of t
            const float* hq = hc + 20 * q;
            const float x = cur[i] + bias;
            f2 a[4];
#pragma unroll
            for (int g = 0; g < 4; ++g) a[g] = f2{g == q ? x : 0.f, 0.f};
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const float4 hv = *reinterpret_cast<const float4*>(&hq[4 * m]);
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    a[g] = __builtin_elementwise_fma(w[g][2 * m], f2{hv.x, hv.y}, a[g]);
                    a[g] = __builtin_elementwise_fma(w[g][2 * m + 1], f2{hv.z, hv.w}, a[g]);
                }
            }
            const float pi = quad_sum(a[0].x + a[0].y), pf = quad_sum(a[1].x + a[1].y);
            const float pg = quad_sum(a[2].x + a[2].y), po = quad_sum(a[3].x + a[3].y);
            const float gi = c_sigm(pi), gf = c_sigm(pf), gg = c_tanh(pg), go = c_sigm(po);
            og[i * G4 + row] = q == 0 ? gi : (q == 1 ? gf : (q == 2 ? gg : go));
            c = cell_fwd_c(c, gi, gf, gg);
            if (q == 0) {
                const float hn = go * c_tanh(c);
                ohp[i * H + u] = hprev;
                hprev = hn;
                hbuf[(i + 1) & 1][seg_pos(u)] = hn;
                oh[i * H + u] = hn;
                oc[i * H + u] = c;
            }
            lds_barrier();
        }
        // flush the chunk: contiguous rows of gates / h / h_prev / c
        for (int idx = j; idx < n * G4; idx += G4) gt[(int64_t)t0 * G4 + idx] = og[idx];
        for (int idx = j; idx < n * H; idx += G4) {
            out_h[hb + (int64_t)t0 * H + idx] = oh[idx];
            out_hprev[hb + (int64_t)t0 * H + idx] = ohp[idx];
            out_c[hb + (int64_t)t0 * H + idx] = oc[idx];
        }
        lds_barrier();
#pragma unroll
        for (int i = 0; i < TS; ++i) cur[i] = nxt[i];
    }
}

static constexpr int TB = 8;   // backward steps per staged chunk (TB * H == 2 * G4 for the staging)

// row all-reduce over the 16 lanes of a DPP row (quad sums, then row_ror 4 and 8)
__device__ __forceinline__ float row16_sum(float v) {
    v = quad_sum(v);
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x124, 0xF, 0xF, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x128, 0xF, 0xF, false));
    return v;
}

// Backward.  dh_rec[u] = sum over the 256 gate rows of W_hh[row][u] dg[row]:
// thread j = 16 ug + rg computes the partial sums of units 4ug .. 4ug+3 over
// rows [16 rg, 16 rg + 16) (W_hh slice in 32 packed VGPR pairs, 4 float4 LDS
// reads of dg), a 16-lane DPP row all-reduce completes them, and lane rg < 4
// of the row owns unit u = 4ug + rg: it computes the unit's cell / gate
// derivatives (dc carried in that lane) and publishes the 4 gate derivatives
// (double-buffered: ONE barrier per time step).
// dh_out: [B, S, H] gradient arriving at this layer's outputs.
// dgates: [B, S, 4H] gradient w.r.t. the gate pre-activations.
// Chunks of TB steps (walking t downwards) of gates / c / dh_out are loaded
// into registers one chunk ahead and handed to LDS at the chunk boundary;
// dgates of a chunk are staged in LDS and written in a burst.
__global__ __launch_bounds__(G4) void k_lstm_bwd(const float* __restrict__ dh_out, const float* __restrict__ gates,
                                                 const float* __restrict__ cst, const float* __restrict__ whh, int S,
                                                 float* __restrict__ dgates) {
    __shared__ __attribute__((aligned(16))) float dg[2][320];
    __shared__ float sg[TB * G4], sc[(TB + 1) * H], sdh[TB * H];  // chunk inputs
    __shared__ float odg[TB * G4];                                 // chunk outputs
    const int j = threadIdx.x;
    const int ug = j >> 4, rg = j & 15;
    const int u = 4 * ug + (rg & 3);                               // the unit of lanes rg < 4
    const bool owner = rg < 4;
    const int64_t b = blockIdx.x;
    f2 wc[4][8];  // W_hh[16 rg + r][4 ug + m]
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int r = 0; r < 8; ++r)
            wc[m][r] = f2{whh[(16 * rg + 2 * r) * H + 4 * ug + m], whh[(16 * rg + 2 * r + 1) * H + 4 * ug + m]};
    float dhr = 0.f, dc = 0.f;
    const int64_t hb = b * (int64_t)S * H;
    const float* gt = gates + b * (int64_t)S * G4;
    float* dgo = dgates + b * (int64_t)S * G4;
    // chunk with steps [lo, lo + TB) (lo may be < 0 at the start of the sequence)
    float rgv[TB], rc[3], rdh[2];
    auto fetch = [&](int lo) {
#pragma unroll
        for (int i = 0; i < TB; ++i) {
            const int t = lo + i;
            rgv[i] = gt[(int64_t)(t >= 0 ? t : 0) * G4 + j];
        }
#pragma unroll
        for (int m = 0; m < 3; ++m) {  // (TB + 1) x H cells (t = lo-1 .. lo+TB-1)
            const int e = j + G4 * m;
            const int ee = e < (TB + 1) * H ? e : 0;
            const int tc = lo - 1 + ee / H;
            rc[m] = cst[hb + (int64_t)(tc >= 0 ? tc : 0) * H + (ee % H)];
        }
#pragma unroll
        for (int m = 0; m < 2; ++m) {  // TB x H output gradients
            const int e = j + G4 * m;
            const int td = lo + e / H;
            rdh[m] = dh_out[hb + (int64_t)(td >= 0 ? td : 0) * H + (e % H)];
        }
    };
    auto stash = [&]() {
#pragma unroll
        for (int i = 0; i < TB; ++i) sg[i * G4 + j] = rgv[i];
#pragma unroll
        for (int m = 0; m < 3; ++m) {
            const int e = j + G4 * m;
            if (e < (TB + 1) * H) sc[e] = rc[m];
        }
#pragma unroll
        for (int m = 0; m < 2; ++m) sdh[j + G4 * m] = rdh[m];
    };
    int lo = S - TB;
    fetch(lo);
    for (; lo > -TB; lo -= TB) {
        stash();
        lds_barrier();
        fetch(lo - TB);  // next chunk in flight during this one
        // the owner lanes' step inputs (gates, c_t, c_{t-1}, dh_out) are read from LDS one
        // step ahead, during the previous step's matvec: no LDS round trip on the recurrence
        float gi = 0.f, gf = 0.f, gg = 0.f, go = 0.f, c = 0.f, cp = 0.f, dho = 0.f;
        auto load_in = [&](int i) {
            gi = sg[i * G4 + u];
            gf = sg[i * G4 + H + u];
            gg = sg[i * G4 + 2 * H + u];
            go = sg[i * G4 + 3 * H + u];
            c = sc[(i + 1) * H + u];
            cp = lo + i > 0 ? sc[i * H + u] : 0.f;
            dho = sdh[i * H + u];
        };
        if (owner) load_in(TB - 1);
        for (int i = TB - 1; i >= 0; --i) {
            const int t = lo + i;
            if (t < 0) break;
            float* dgb = dg[t & 1];
            if (owner) {
                const float dh = dho + dhr;
                float v0, v1, v2, v3;
                cell_bwd<VT_LSTM_LIBM>(dh, gi, gf, gg, go, c, cp, dc, v0, v1, v2, v3);
                dgb[seg_pos(u)] = v0;
                dgb[seg_pos(H + u)] = v1;
                dgb[seg_pos(2 * H + u)] = v2;
                dgb[seg_pos(3 * H + u)] = v3;
                float* o = odg + i * G4;
                o[u] = v0; o[H + u] = v1; o[2 * H + u] = v2; o[3 * H + u] = v3;
            }
            lds_barrier();
            const float* dq = dgb + 20 * rg;
            f2 a[4] = {f2{0.f, 0.f}, f2{0.f, 0.f}, f2{0.f, 0.f}, f2{0.f, 0.f}};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float4 d = *reinterpret_cast<const float4*>(&dq[4 * r]);
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    a[m] = __builtin_elementwise_fma(wc[m][2 * r], f2{d.x, d.y}, a[m]);
                    a[m] = __builtin_elementwise_fma(wc[m][2 * r + 1], f2{d.z, d.w}, a[m]);
                }
            }
            if (owner && i > 0) load_in(i - 1);   // queued behind this step's dg reads
            const float s0 = row16_sum(a[0].x + a[0].y), s1 = row16_sum(a[1].x + a[1].y);
            const float s2 = row16_sum(a[2].x + a[2].y), s3 = row16_sum(a[3].x + a[3].y);
            const int m = rg & 3;
            dhr = m == 0 ? s0 : (m == 1 ? s1 : (m == 2 ? s2 : s3));
        }
        // flush dgates of the chunk's valid steps
        lds_barrier();
        const int t_first = lo < 0 ? 0 : lo;
        const int i0 = t_first - lo;
        for (int idx = i0 * G4 + j; idx < TB * G4; idx += G4) dgo[(int64_t)lo * G4 + idx] = odg[idx];
        lds_barrier();
    }
}


// ------------------------------------------------ fused input projections
// The same recurrences with the layer's input projections done inside on the
// exact-fp32 matrix cores, so neither G = X W_ih^T nor dX = dG W_ih exists as a
// separate GEMM launch on the layer-to-layer chain (nor G as a [B, S, 4H] HBM
// round trip).  Each MFMA output tile is the same v_mfma_f32_16x16x4_f32 chain
// over k, in the same order, from the same zero start as the skinny GEMMs
// (mlp.hip k_sk_gemm), so the results are bitwise those of the unfused path.

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// LDS hand-off between lanes of one wave (in-order LDS queue, no s_barrier)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

static constexpr int XSS = 68;  // row stride of a staged input chunk (== 4 mod 64: conflict-free A fragments)

// Forward with G computed in-kernel.  x: [B, S, In], In <= 4 KS; w_ih [4H][In].
// Wave wv owns the gate rows q H + 16 wv + (0..15) of all four gates, which are
// exactly the rows its own recurrence lanes consume: the projection of the
// NEXT chunk of TS steps (4 KS MFMAs per wave) is issued a few per time step
// behind each step's barrier, off the recurrence chain, from an input chunk
// staged in LDS one chunk ahead (double-buffered, loaded from HBM two ahead),
// and handed to the lanes through this wave's slice of the gates staging.
template <int KS>
__global__ __launch_bounds__(G4) __attribute__((amdgpu_waves_per_eu(2))) void k_lstm_fwd_x(const float* __restrict__ x, int In, const float* __restrict__ wih,
                                                   const float* __restrict__ bih, const float* __restrict__ whh,
                                                   const float* __restrict__ bhh, int S, float* __restrict__ out_h,
                                                   float* __restrict__ out_hprev, float* __restrict__ out_c,
                                                   float* __restrict__ gates) {
    constexpr int NX = (TS * 4 * KS + G4 - 1) / G4;  // staged input floats per thread
    constexpr int NM = 4 * KS;                        // projection MFMAs per wave and chunk
    __shared__ __attribute__((aligned(16))) float hbuf[2][80];
    __shared__ float og[TS * G4];
    __shared__ float oh[TS * H], ohp[TS * H], oc[TS * H];
    __shared__ float xs[2][TS * XSS];
    const int j = threadIdx.x, u = j >> 2, q = j & 3;
    const int lane = j & 63, wv = j >> 6, lr = lane & 15, lc = lane >> 4;
    const int row = q * H + u;
    const int64_t b = blockIdx.x;
    f2 w[4][8];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int k = 0; k < 8; ++k)
            w[g][k] = f2{whh[(g * H + u) * H + 16 * q + 2 * k], whh[(g * H + u) * H + 16 * q + 2 * k + 1]};
    const float bias = bhh[row];
    // B fragments of W_ih^T: tile g = gate g, column (gate row) g H + 16 wv + lr, k = 4 s + lc
    float wf[4][KS], bf[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int r = g * H + 16 * wv + lr;
        bf[g] = bih[r];
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
            const int k = 4 * s2 + lc;
            wf[g][s2] = k < In ? wih[(int64_t)r * In + k] : 0.f;
        }
    }
    for (int i = j; i < 2 * TS * XSS; i += G4) (&xs[0][0])[i] = 0.f;  // columns >= In stay zero
    if (j < 80) hbuf[0][j] = 0.f;
    // this thread's share of a TS x In input chunk (contiguous in x)
    const int CH = TS * In;
    int xo[NX];
#pragma unroll
    for (int m = 0; m < NX; ++m) {
        const int idx = j + G4 * m, t = idx / In;
        xo[m] = idx < CH ? t * XSS + (idx - t * In) : -1;
    }
    const float* xb = x + b * (int64_t)S * In;
    float xr[NX];
    auto xload = [&](int t0) {
#pragma unroll
        for (int m = 0; m < NX; ++m) {
            const int idx = j + G4 * m;
            xr[m] = (xo[m] >= 0 && t0 * In + idx < S * In) ? xb[(int64_t)t0 * In + idx] : 0.f;
        }
    };
    auto xstore = [&](int buf) {
#pragma unroll
        for (int m = 0; m < NX; ++m)
            if (xo[m] >= 0) xs[buf][xo[m]] = xr[m];
    };
    f32x4 acc[4];
    // G of the chunk from acc (+ b_ih) into this wave's rows of og: each lane reads
    // its own G[t][row] at step t (alongside h) and overwrites it with the gate
    auto publish = [&]() {
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int r = 0; r < 4; ++r) og[(4 * lc + r) * G4 + g * H + 16 * wv + lr] = acc[g][r] + bf[g];
        wave_lds_sync();
    };
    float c = 0.f, hprev = 0.f;
    float* gt = gates + b * (int64_t)S * G4;
    const int64_t hb = b * (int64_t)S * H;
    xload(0);
    xstore(0);
    xload(TS);
    xstore(1);
    xload(2 * TS);
    lds_barrier();
#pragma unroll
    for (int g = 0; g < 4; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int mm = 0; mm < NM; ++mm) acc[mm / KS] = mfma4(xs[0][lr * XSS + 4 * (mm % KS) + lc], wf[mm / KS][mm % KS], acc[mm / KS]);
    publish();
    int cb = 1;  // buffer holding the next chunk's input
    for (int t0 = 0; t0 < S; t0 += TS) {
        const int n = S - t0 < TS ? S - t0 : TS;
        const bool more = t0 + TS < S;
        const float* xn = xs[cb];
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
        // the next chunk's projection, a few MFMAs behind each step's barrier (measured:
        // as fast as, or faster than, interleaving them into the step's FMA chain or
        // issuing all of them at the chunk's end)
#pragma unroll
        for (int i = 0; i < TS; ++i) {
            if (i >= n) continue;  // block-uniform
            const float* hq = hbuf[i & 1] + 20 * q;
            const float xv = og[i * G4 + row] + bias;
            f2 a[4];
#pragma unroll
            for (int g = 0; g < 4; ++g) a[g] = f2{g == q ? xv : 0.f, 0.f};
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const float4 hv = *reinterpret_cast<const float4*>(&hq[4 * m]);
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    a[g] = __builtin_elementwise_fma(w[g][2 * m], f2{hv.x, hv.y}, a[g]);
                    a[g] = __builtin_elementwise_fma(w[g][2 * m + 1], f2{hv.z, hv.w}, a[g]);
                }
            }
            const float pi = quad_sum(a[0].x + a[0].y), pf = quad_sum(a[1].x + a[1].y);
            const float pg = quad_sum(a[2].x + a[2].y), po = quad_sum(a[3].x + a[3].y);
            const float gi = c_sigm(pi), gf = c_sigm(pf), gg = c_tanh(pg), go = c_sigm(po);
            og[i * G4 + row] = q == 0 ? gi : (q == 1 ? gf : (q == 2 ? gg : go));
            c = cell_fwd_c(c, gi, gf, gg);
            if (q == 0) {
                const float hn = go * c_tanh(c);
                ohp[i * H + u] = hprev;
                hprev = hn;
                hbuf[(i + 1) & 1][seg_pos(u)] = hn;
                oh[i * H + u] = hn;
                oc[i * H + u] = c;
            }
            lds_barrier();
            if (more) {
#pragma unroll
                for (int mm = i * NM / TS; mm < (i + 1) * NM / TS; ++mm)
                    acc[mm / KS] = mfma4(xn[lr * XSS + 4 * (mm % KS) + lc], wf[mm / KS][mm % KS], acc[mm / KS]);
            }
        }
        for (int idx = j; idx < n * G4; idx += G4) gt[(int64_t)t0 * G4 + idx] = og[idx];
        for (int idx = j; idx < n * H; idx += G4) {
            out_h[hb + (int64_t)t0 * H + idx] = oh[idx];
            out_hprev[hb + (int64_t)t0 * H + idx] = ohp[idx];
            out_c[hb + (int64_t)t0 * H + idx] = oc[idx];
        }
        lds_barrier();
        if (more) {
            publish();
            xstore(cb ^ 1);        // chunk + 2 into the buffer this chunk's input used
            xload(t0 + 3 * TS);
            cb ^= 1;
        }
    }
}

static constexpr int TB2 = 16;          // backward steps per chunk (one 16-row MFMA tile of dX)
static constexpr int ODS = G4 + 4;      // row stride of the staged dgates (== 4 mod 64)

// Backward with dX = dG W_ih computed in-kernel (dx may be null) and dG still
// written for the weight gradients (dgates may be null).  w_ih [4H][In],
// In <= 16 NTX; wave wv < NTX owns dX columns [16 wv, 16 wv + 16) and holds
// W_ih[:, its columns] as 64 B fragments.  A chunk's dG rows are staged in
// LDS (double-buffered) and its dX tile is accumulated (64 MFMAs, 4 per time
// step) during the NEXT chunk's steps, behind each step's barrier.
template <int NTX>
__global__ __launch_bounds__(G4) __attribute__((amdgpu_waves_per_eu(2))) void k_lstm_bwd_x(const float* __restrict__ dh_out, const float* __restrict__ gates,
                                                   const float* __restrict__ cst, const float* __restrict__ whh,
                                                   const float* __restrict__ wih, int In, int S,
                                                   float* __restrict__ dgates, float* __restrict__ dx) {
    __shared__ __attribute__((aligned(16))) float dg[2][320];
    __shared__ float sg[TB2 * G4], sc[(TB2 + 1) * H], sdh[TB2 * H];
    __shared__ float odg[2][TB2 * ODS];
    const int j = threadIdx.x;
    const int ug = j >> 4, rg = j & 15;
    const int u = 4 * ug + (rg & 3);
    const bool owner = rg < 4;
    const int lane = j & 63, wv = j >> 6, lr = lane & 15, lc = lane >> 4;
    const bool dxw = dx != nullptr && wv < NTX;   // wave-uniform
    const int64_t b = blockIdx.x;
    f2 wc[4][8];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int r = 0; r < 8; ++r)
            wc[m][r] = f2{whh[(16 * rg + 2 * r) * H + 4 * ug + m], whh[(16 * rg + 2 * r + 1) * H + 4 * ug + m]};
    // B fragments of W_ih: k (gate row) = 4 s + lc, column 16 wv + lr
    float wx[64];
    {
        const int col = 16 * wv + lr;
#pragma unroll
        for (int s2 = 0; s2 < 64; ++s2) wx[s2] = (wv < NTX && col < In) ? wih[(4 * s2 + lc) * In + col] : 0.f;
    }
    float dhr = 0.f, dc = 0.f;
    const int64_t hb = b * (int64_t)S * H;
    const float* gt = gates + b * (int64_t)S * G4;
    float* dgo = dgates ? dgates + b * (int64_t)S * G4 : nullptr;
    float* dxb = dx ? dx + b * (int64_t)S * In : nullptr;
    constexpr int NC = ((TB2 + 1) * H + G4 - 1) / G4, ND = TB2 * H / G4;
    float rgv[TB2], rc[NC], rdh[ND];
    auto fetch = [&](int lo) {
#pragma unroll
        for (int i = 0; i < TB2; ++i) {
            const int t = lo + i;
            rgv[i] = gt[(int64_t)(t >= 0 ? t : 0) * G4 + j];
        }
#pragma unroll
        for (int m = 0; m < NC; ++m) {
            const int e = j + G4 * m;
            const int ee = e < (TB2 + 1) * H ? e : 0;
            const int tc = lo - 1 + ee / H;
            rc[m] = cst[hb + (int64_t)(tc >= 0 ? tc : 0) * H + (ee % H)];
        }
#pragma unroll
        for (int m = 0; m < ND; ++m) {
            const int e = j + G4 * m;
            const int td = lo + e / H;
            rdh[m] = dh_out[hb + (int64_t)(td >= 0 ? td : 0) * H + (e % H)];
        }
    };
    auto stash = [&]() {
#pragma unroll
        for (int i = 0; i < TB2; ++i) sg[i * G4 + j] = rgv[i];
#pragma unroll
        for (int m = 0; m < NC; ++m) {
            const int e = j + G4 * m;
            if (e < (TB2 + 1) * H) sc[e] = rc[m];
        }
#pragma unroll
        for (int m = 0; m < ND; ++m) sdh[j + G4 * m] = rdh[m];
    };
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    auto dx_write = [&](int plo) {  // rows plo + 4 lc + r of the accumulated tile
        const int col = 16 * wv + lr;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int t = plo + 4 * lc + r;
            if (t >= 0 && col < In) dxb[(int64_t)t * In + col] = acc[r] + 0.f;
        }
    };
    int lo = S - TB2, cbuf = 0, plo = 0;
    bool prev = false;
    fetch(lo);
    for (; lo > -TB2; lo -= TB2) {
        stash();
        lds_barrier();
        fetch(lo - TB2);
        float gi = 0.f, gf = 0.f, gg = 0.f, go = 0.f, c = 0.f, cp = 0.f, dho = 0.f;
        auto load_in = [&](int i) {
            gi = sg[i * G4 + u];
            gf = sg[i * G4 + H + u];
            gg = sg[i * G4 + 2 * H + u];
            go = sg[i * G4 + 3 * H + u];
            c = sc[(i + 1) * H + u];
            cp = lo + i > 0 ? sc[i * H + u] : 0.f;
            dho = sdh[i * H + u];
        };
        load_in(TB2 - 1);
        float* ob = odg[cbuf];
        const float* op = odg[cbuf ^ 1];
        acc = f32x4{0.f, 0.f, 0.f, 0.f};
        float pa[4];  // A operands of the previous chunk's dX tile, one step ahead
#pragma unroll
        for (int k = 0; k < 4; ++k) pa[k] = op[lr * ODS + 4 * k + lc];
        // Straight-line steps (no per-step branches: the scheduler slots the dX MFMAs
        // into the recurrence's latency gaps).  Steps with t < 0 (last chunk) run on
        // finite clamped inputs after t = 0 and are not stored; in the first chunk the
        // MFMAs consume stale LDS and their tile is not stored either.
#pragma unroll
        for (int i = TB2 - 1; i >= 0; --i) {
            const int t = lo + i;
            float* dgb = dg[t & 1];
            const float dh = dho + dhr;
            float v0, v1, v2, v3;
            cell_bwd<VT_LSTM_LIBM>(dh, gi, gf, gg, go, c, cp, dc, v0, v1, v2, v3);
            if (owner) {
                dgb[seg_pos(u)] = v0;
                dgb[seg_pos(H + u)] = v1;
                dgb[seg_pos(2 * H + u)] = v2;
                dgb[seg_pos(3 * H + u)] = v3;
                float* o = ob + i * ODS;
                o[u] = v0; o[H + u] = v1; o[2 * H + u] = v2; o[3 * H + u] = v3;
            }
            const int p = TB2 - 1 - i;  // the previous chunk's dX tile, k-steps 4 p .. 4 p + 3
#pragma unroll
            for (int k = 0; k < 4; ++k) acc = mfma4(pa[k], wx[4 * p + k], acc);
            lds_barrier();
            const float* dq = dgb + 20 * rg;
            float4 dv[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) dv[r] = *reinterpret_cast<const float4*>(&dq[4 * r]);
            if (p + 1 < TB2) {
#pragma unroll
                for (int k = 0; k < 4; ++k) pa[k] = op[lr * ODS + 4 * (4 * (p + 1) + k) + lc];
            }
            if (i > 0) load_in(i - 1);
            f2 a[4] = {f2{0.f, 0.f}, f2{0.f, 0.f}, f2{0.f, 0.f}, f2{0.f, 0.f}};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    a[m] = __builtin_elementwise_fma(wc[m][2 * r], f2{dv[r].x, dv[r].y}, a[m]);
                    a[m] = __builtin_elementwise_fma(wc[m][2 * r + 1], f2{dv[r].z, dv[r].w}, a[m]);
                }
            }
            const float s0 = row16_sum(a[0].x + a[0].y), s1 = row16_sum(a[1].x + a[1].y);
            const float s2 = row16_sum(a[2].x + a[2].y), s3 = row16_sum(a[3].x + a[3].y);
            const int m = rg & 3;
            dhr = m == 0 ? s0 : (m == 1 ? s1 : (m == 2 ? s2 : s3));
        }
        if (dgo) {
            const int t_first = lo < 0 ? 0 : lo;
            for (int idx = (t_first - lo) * G4 + j; idx < TB2 * G4; idx += G4)
                dgo[(int64_t)lo * G4 + idx] = ob[(idx >> 8) * ODS + (idx & (G4 - 1))];
        }
        if (prev && dxw) dx_write(plo);
        lds_barrier();
        prev = true;
        plo = lo;
        cbuf ^= 1;
    }
    if (dxw && prev) {  // the last chunk's tile (its rows are in odg[cbuf ^ 1])
        const float* op = odg[cbuf ^ 1];
        acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 64; ++k) acc = mfma4(op[lr * ODS + 4 * k + lc], wx[k], acc);
        dx_write(plo);
    }
}

}  // namespace vt

using namespace vt;

extern "C" {

int vt_lstm_layer_fwd(const float* gin, const float* w_hh, const float* b_hh, int B, int seq, int hidden,
                      float* out_h, float* out_hprev, float* out_c, float* gates, void* stream) {
    VT_CHECK_ARG(hidden == H, "vt_lstm_layer_fwd: hidden size %d (kernel built for %d)", hidden, H);
    VT_CHECK_ARG(B > 0 && seq > 0, "vt_lstm_layer_fwd: shape");
    hipLaunchKernelGGL(k_lstm_fwd, dim3(B), dim3(G4), 0, S(stream), gin, w_hh, b_hh, seq, out_h, out_hprev, out_c,
                       gates);
    VT_LAUNCH_CHECK("vt_lstm_layer_fwd");
    return VT_OK;
}

int vt_lstm_layer_bwd(const float* dh_out, const float* gates, const float* cst, const float* w_hh, int B, int seq,
                      int hidden, float* dgates, void* stream) {
    VT_CHECK_ARG(hidden == H, "vt_lstm_layer_bwd: hidden size %d (kernel built for %d)", hidden, H);
    VT_CHECK_ARG(B > 0 && seq > 0, "vt_lstm_layer_bwd: shape");
    hipLaunchKernelGGL(k_lstm_bwd, dim3(B), dim3(G4), 0, S(stream), dh_out, gates, cst, w_hh, seq, dgates);
    VT_LAUNCH_CHECK("vt_lstm_layer_bwd");
    return VT_OK;
}

int vt_lstm_layer_fwd_x(const float* x, int In, const float* w_ih, const float* b_ih, const float* w_hh,
                        const float* b_hh, int B, int seq, int hidden, float* out_h, float* out_hprev, float* out_c,
                        float* gates, void* stream) {
    VT_CHECK_ARG(hidden == H, "vt_lstm_layer_fwd_x: hidden size %d (kernel built for %d)", hidden, H);
    VT_CHECK_ARG(B > 0 && seq > 0 && In > 0 && In <= 64, "vt_lstm_layer_fwd_x: shape (input size %d, at most 64)", In);
    VT_CHECK_ARG(x && w_ih && b_ih && w_hh && b_hh && out_h && out_hprev && out_c && gates,
                 "vt_lstm_layer_fwd_x: null pointer");
    const int ks = (In + 3) / 4;
#define VT_LFX(K_)                                                                                                 \
    hipLaunchKernelGGL((k_lstm_fwd_x<K_>), dim3(B), dim3(G4), 0, S(stream), x, In, w_ih, b_ih, w_hh, b_hh, seq,    \
                       out_h, out_hprev, out_c, gates)
    if (ks == 5) VT_LFX(5);        // encoder y layer 0 (In = 20)
    else if (ks == 8) VT_LFX(8);   // encoder x layer 0 (In = 32)
    else if (ks <= 4) VT_LFX(4);   // others: zero k-steps appended (an fma with 0 * 0)
    else if (ks <= 8) VT_LFX(8);
    else if (ks <= 12) VT_LFX(12);
    else VT_LFX(16);
#undef VT_LFX
    VT_LAUNCH_CHECK("vt_lstm_layer_fwd_x");
    return VT_OK;
}

int vt_lstm_layer_bwd_x(const float* dh_out, const float* gates, const float* cst, const float* w_hh,
                        const float* w_ih, int In, int B, int seq, int hidden, float* dgates, float* dx,
                        void* stream) {
    VT_CHECK_ARG(hidden == H, "vt_lstm_layer_bwd_x: hidden size %d (kernel built for %d)", hidden, H);
    VT_CHECK_ARG(B > 0 && seq > 0 && In > 0 && In <= 64, "vt_lstm_layer_bwd_x: shape (input size %d, at most 64)", In);
    VT_CHECK_ARG(dh_out && gates && cst && w_hh && (w_ih || !dx), "vt_lstm_layer_bwd_x: null pointer");
    const int ntx = (In + 15) / 16;
#define VT_LBX(N_)                                                                                                 \
    case N_:                                                                                                       \
        hipLaunchKernelGGL((k_lstm_bwd_x<N_>), dim3(B), dim3(G4), 0, S(stream), dh_out, gates, cst, w_hh, w_ih, In, \
                           seq, dgates, dx);                                                                       \
        break;
    switch (ntx) { VT_LBX(1) VT_LBX(2) VT_LBX(3) VT_LBX(4) }
#undef VT_LBX
    VT_LAUNCH_CHECK("vt_lstm_layer_bwd_x");
    return VT_OK;
}

int vt_lstm_layer_bwd_weight(const float* dgates, const float* x, int In, const float* hprev, int B, int seq,
                             int hidden, float* dw_ih, float* dw_hh, float* db_ih, float* db_hh, int accumulate,
                             float* ws, int64_t ws_floats, void* stream) {
    VT_CHECK_ARG(hidden == H, "vt_lstm_layer_bwd_weight: hidden size %d (kernel built for %d)", hidden, H);
    VT_CHECK_ARG(B > 0 && seq > 0 && In > 0 && In + H + 1 <= SK_MAX_K1, "vt_lstm_layer_bwd_weight: shape (In %d)", In);
    VT_CHECK_ARG(dgates && x && hprev && dw_ih && dw_hh && db_ih, "vt_lstm_layer_bwd_weight: null pointer");
    const int64_t R = (int64_t)B * seq;
    const int rc = sk_linear_bwd_weight2(dgates, R, G4, x, In, hprev, H, dw_ih, dw_hh, db_ih, db_hh, accumulate, ws,
                                         ws_floats, S(stream));
    VT_CHECK_ARG(rc == VT_OK, "vt_lstm_layer_bwd_weight: workspace too small");
    VT_LAUNCH_CHECK("vt_lstm_layer_bwd_weight");
    return VT_OK;
}

int vt_lstm16_layer_bwd_weight(const float* dgates, const float* x, int In, const float* h, int B, int seq,
                               int hidden, float* dw_ih, float* dw_hh, float* db_ih, float* db_hh, int accumulate,
                               float* ws, int64_t ws_floats, void* stream) {
    VT_CHECK_ARG(hidden == H, "vt_lstm16_layer_bwd_weight: hidden size %d (kernel built for %d)", hidden, H);
    VT_CHECK_ARG(B > 0 && seq > 0 && In > 0 && In + H + 1 <= SK_MAX_K1 && (int64_t)B * seq < ((int64_t)1 << 31),
                 "vt_lstm16_layer_bwd_weight: shape (In %d)", In);
    VT_CHECK_ARG(dgates && x && h && dw_ih && dw_hh && db_ih, "vt_lstm16_layer_bwd_weight: null pointer");
    const int64_t R = (int64_t)B * seq;
    // bf16 operands on bf16 MFMA (skdw16.hip, the 16-bit model's precision: dG / x / h rounded to
    // bf16, fp32 accumulation); VAETEB_L16_DW16=0 or an unsupported shape: the exact-fp32 kernel
    static const int dw16 = getenv("VAETEB_L16_DW16") ? atoi(getenv("VAETEB_L16_DW16")) : 1;
    if (dw16 && sk_lstm16_dw(dgates, x, In, h, seq, R, dw_ih, dw_hh, db_ih, db_hh, accumulate, ws, ws_floats,
                             S(stream)) == VT_OK) {
        VT_LAUNCH_CHECK("vt_lstm16_layer_bwd_weight");
        return VT_OK;
    }
    const int rc = sk_linear_bwd_weight2(dgates, R, G4, x, In, h, H, dw_ih, dw_hh, db_ih, db_hh, accumulate, ws,
                                         ws_floats, S(stream), seq);
    VT_CHECK_ARG(rc == VT_OK, "vt_lstm16_layer_bwd_weight: workspace too small");
    VT_LAUNCH_CHECK("vt_lstm16_layer_bwd_weight");
    return VT_OK;
}

}  // extern "C"
