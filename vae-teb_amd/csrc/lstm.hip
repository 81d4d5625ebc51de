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

namespace vt {

static constexpr int H = 64;
static constexpr int G4 = 4 * H;

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

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

// gin:   [B, S, 4H]  x W_ih^T + b_ih (precomputed)
// out_h: [B, S, H]; out_hprev: [B, S, H] (h_{t-1}, zeros at t = 0)
// out_c: [B, S, H] cell states; gates: [B, S, 4H] post-activation (i, f, g~, o)
// The recurrence only touches LDS and registers: gin is loaded a chunk of TS
// steps ahead into registers and the outputs of a chunk are staged in LDS and
// written in one coalesced burst, so no global round trip sits between steps.
__global__ __launch_bounds__(G4) void k_lstm_fwd(const float* __restrict__ gin, const float* __restrict__ whh,
                                                 const float* __restrict__ bhh, int S, float* __restrict__ out_h,
                                                 float* __restrict__ out_hprev, float* __restrict__ out_c,
                                                 float* __restrict__ gates) {
    __shared__ __attribute__((aligned(16))) float h[H];
    __shared__ float gb[G4];
    __shared__ float og[TS * G4];                      // gates of the chunk
    __shared__ float oh[TS * H], ohp[TS * H], oc[TS * H];
    const int j = threadIdx.x;
    const int64_t b = blockIdx.x;
    float w[H];
#pragma unroll
    for (int k = 0; k < H; ++k) w[k] = whh[j * H + k];
    const float bias = bhh[j];
    if (j < H) h[j] = 0.f;
    float c = 0.f;
    const float* g_in = gin + b * (int64_t)S * G4;
    float* gt = gates + b * (int64_t)S * G4;
    const int64_t hb = b * (int64_t)S * H;
    float cur[TS], nxt[TS];
#pragma unroll
    for (int i = 0; i < TS; ++i) cur[i] = g_in[(int64_t)(i < S ? i : S - 1) * G4 + j];
    lds_barrier();
    for (int t0 = 0; t0 < S; t0 += TS) {
#pragma unroll
        for (int i = 0; i < TS; ++i) {  // unconditional (clamped) loads: no per-step waits
            const int t = t0 + TS + i;
            nxt[i] = g_in[(int64_t)(t < S ? t : S - 1) * G4 + j];
        }
        const int n = S - t0 < TS ? S - t0 : TS;
#pragma unroll
        for (int i = 0; i < TS; ++i) {
            if (i >= n) continue;  // block-uniform
            float a0 = cur[i] + bias, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
            for (int k = 0; k < H; k += 4) {
                const float4 hv = *reinterpret_cast<const float4*>(&h[k]);
                a0 = fmaf(w[k], hv.x, a0);
                a1 = fmaf(w[k + 1], hv.y, a1);
                a2 = fmaf(w[k + 2], hv.z, a2);
                a3 = fmaf(w[k + 3], hv.w, a3);
            }
            const float a = (a0 + a1) + (a2 + a3);
            const float v = (j >= 2 * H && j < 3 * H) ? tanhf(a) : sigm(a);
            gb[j] = v;
            og[i * G4 + j] = v;
            lds_barrier();
            if (j < H) {
                c = gb[H + j] * c + gb[j] * gb[2 * H + j];
                const float hn = gb[3 * H + j] * tanhf(c);
                ohp[i * H + j] = h[j];
                h[j] = hn;
                oh[i * H + j] = hn;
                oc[i * H + j] = c;
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

static constexpr int TB = 8;  // backward steps per staged chunk (TB * H == 2 * G4 for the staging)

// dh_out: [B, S, H] gradient arriving at this layer's outputs.
// dgates: [B, S, 4H] gradient w.r.t. the gate pre-activations.
// Chunks of TB steps (walking t downwards) of gates / c / dh_out are loaded
// into registers one chunk ahead by all 256 threads and handed to LDS at the
// chunk boundary; dgates of a chunk are staged in LDS and written in a burst.
__global__ __launch_bounds__(G4) void k_lstm_bwd(const float* __restrict__ dh_out, const float* __restrict__ gates,
                                                 const float* __restrict__ cst, const float* __restrict__ whh, int S,
                                                 float* __restrict__ dgates) {
    __shared__ __attribute__((aligned(16))) float dg[G4];
    __shared__ float part[G4];
    __shared__ float dhr[H];
    __shared__ float sg[TB * G4], sc[(TB + 1) * H], sdh[TB * H];  // chunk inputs
    __shared__ float odg[TB * G4];                                 // chunk outputs
    const int j = threadIdx.x;
    const int q = j >> 6, k = j & 63;
    const int64_t b = blockIdx.x;
    float wc[H];  // W_hh[q*64 + r][k], r = 0..63
#pragma unroll
    for (int r = 0; r < H; ++r) wc[r] = whh[(q * H + r) * H + k];
    if (j < H) dhr[j] = 0.f;
    float dc = 0.f;
    const int64_t hb = b * (int64_t)S * H;
    const float* gt = gates + b * (int64_t)S * G4;
    float* dgo = dgates + b * (int64_t)S * G4;
    // chunk with steps [lo, lo + TB) (lo may be < 0 at the start of the sequence)
    float rg[TB], rc[3], rdh[2];
    auto fetch = [&](int lo) {
#pragma unroll
        for (int i = 0; i < TB; ++i) {
            const int t = lo + i;
            rg[i] = gt[(int64_t)(t >= 0 ? t : 0) * G4 + j];
        }
#pragma unroll
        for (int u = 0; u < 3; ++u) {  // (TB + 1) x H cells (t = lo-1 .. lo+TB-1)
            const int e = j + G4 * u;
            const int ee = e < (TB + 1) * H ? e : 0;
            const int tc = lo - 1 + ee / H;
            rc[u] = cst[hb + (int64_t)(tc >= 0 ? tc : 0) * H + (ee % H)];
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {  // TB x H output gradients
            const int e = j + G4 * u;
            const int td = lo + e / H;
            rdh[u] = dh_out[hb + (int64_t)(td >= 0 ? td : 0) * H + (e % H)];
        }
    };
    auto stash = [&]() {
#pragma unroll
        for (int i = 0; i < TB; ++i) sg[i * G4 + j] = rg[i];
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int e = j + G4 * u;
            if (e < (TB + 1) * H) sc[e] = rc[u];
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) sdh[j + G4 * u] = rdh[u];
    };
    int lo = S - TB;
    fetch(lo);
    for (; lo > -TB; lo -= TB) {
        stash();
        lds_barrier();
        fetch(lo - TB);  // next chunk in flight during this one
        for (int i = TB - 1; i >= 0; --i) {
            const int t = lo + i;
            if (t < 0) break;
            if (j < H) {
                const float gi = sg[i * G4 + j], gf = sg[i * G4 + H + j], gg = sg[i * G4 + 2 * H + j];
                const float go = sg[i * G4 + 3 * H + j];
                const float c = sc[(i + 1) * H + j], cp = t > 0 ? sc[i * H + j] : 0.f;
                const float dh = sdh[i * H + j] + dhr[j];
                const float tc = tanhf(c);
                const float d_o = dh * tc;
                dc = dc + dh * go * (1.f - tc * tc);
                const float di = dc * gg, dgg = dc * gi, df = dc * cp;
                dc = dc * gf;
                const float v0 = di * gi * (1.f - gi), v1 = df * gf * (1.f - gf);
                const float v2 = dgg * (1.f - gg * gg), v3 = d_o * go * (1.f - go);
                dg[j] = v0; dg[H + j] = v1; dg[2 * H + j] = v2; dg[3 * H + j] = v3;
                float* o = odg + i * G4;
                o[j] = v0; o[H + j] = v1; o[2 * H + j] = v2; o[3 * H + j] = v3;
            }
            lds_barrier();
            float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
            for (int r = 0; r < H; r += 4) {
                const float4 d = *reinterpret_cast<const float4*>(&dg[q * H + r]);
                a0 = fmaf(wc[r], d.x, a0);
                a1 = fmaf(wc[r + 1], d.y, a1);
                a2 = fmaf(wc[r + 2], d.z, a2);
                a3 = fmaf(wc[r + 3], d.w, a3);
            }
            part[j] = (a0 + a1) + (a2 + a3);
            lds_barrier();
            if (j < H) dhr[j] = (part[j] + part[H + j]) + (part[2 * H + j] + part[3 * H + j]);
            lds_barrier();
        }
        // flush dgates of the chunk's valid steps
        const int t_first = lo < 0 ? 0 : lo;
        const int i0 = t_first - lo;
        for (int idx = i0 * G4 + j; idx < TB * G4; idx += G4) dgo[(int64_t)lo * G4 + idx] = odg[idx];
        lds_barrier();
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

}  // extern "C"
