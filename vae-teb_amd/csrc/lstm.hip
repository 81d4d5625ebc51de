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

// gin:   [B, S, 4H]  x W_ih^T + b_ih (precomputed)
// out_h: [B, S, H]; out_hprev: [B, S, H] (h_{t-1}, zeros at t = 0)
// out_c: [B, S, H] cell states; gates: [B, S, 4H] post-activation (i, f, g~, o)
__global__ __launch_bounds__(G4) void k_lstm_fwd(const float* __restrict__ gin, const float* __restrict__ whh,
                                                 const float* __restrict__ bhh, int S, float* __restrict__ out_h,
                                                 float* __restrict__ out_hprev, float* __restrict__ out_c,
                                                 float* __restrict__ gates) {
    __shared__ __attribute__((aligned(16))) float h[H];
    __shared__ float gb[G4];
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
    float pre_next = g_in[j];
    __syncthreads();
    for (int t = 0; t < S; ++t) {
        const float pre = pre_next;
        if (t + 1 < S) pre_next = g_in[(int64_t)(t + 1) * G4 + j];
        float a0 = pre + bias, a1 = 0.f, a2 = 0.f, a3 = 0.f;
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
        gt[(int64_t)t * G4 + j] = v;
        __syncthreads();
        if (j < H) {
            c = gb[H + j] * c + gb[j] * gb[2 * H + j];
            const float hn = gb[3 * H + j] * tanhf(c);
            out_hprev[hb + (int64_t)t * H + j] = h[j];
            h[j] = hn;
            out_h[hb + (int64_t)t * H + j] = hn;
            out_c[hb + (int64_t)t * H + j] = c;
        }
        __syncthreads();
    }
}

// dh_out: [B, S, H] gradient arriving at this layer's outputs.
// dgates: [B, S, 4H] gradient w.r.t. the gate pre-activations.
__global__ __launch_bounds__(G4) void k_lstm_bwd(const float* __restrict__ dh_out, const float* __restrict__ gates,
                                                 const float* __restrict__ cst, const float* __restrict__ whh, int S,
                                                 float* __restrict__ dgates) {
    __shared__ __attribute__((aligned(16))) float dg[G4];
    __shared__ float part[G4];
    __shared__ float dhr[H];
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
    __syncthreads();
    for (int t = S - 1; t >= 0; --t) {
        if (j < H) {
            const float* g = gt + (int64_t)t * G4;
            const float gi = g[j], gf = g[H + j], gg = g[2 * H + j], go = g[3 * H + j];
            const float c = cst[hb + (int64_t)t * H + j];
            const float cp = t > 0 ? cst[hb + (int64_t)(t - 1) * H + j] : 0.f;
            const float dh = dh_out[hb + (int64_t)t * H + j] + dhr[j];
            const float tc = tanhf(c);
            const float d_o = dh * tc;
            dc = dc + dh * go * (1.f - tc * tc);
            const float di = dc * gg, dgg = dc * gi, df = dc * cp;
            dc = dc * gf;
            const float v0 = di * gi * (1.f - gi), v1 = df * gf * (1.f - gf);
            const float v2 = dgg * (1.f - gg * gg), v3 = d_o * go * (1.f - go);
            dg[j] = v0; dg[H + j] = v1; dg[2 * H + j] = v2; dg[3 * H + j] = v3;
            float* o = dgo + (int64_t)t * G4;
            o[j] = v0; o[H + j] = v1; o[2 * H + j] = v2; o[3 * H + j] = v3;
        }
        __syncthreads();
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
        __syncthreads();
        if (j < H) dhr[j] = (part[j] + part[H + j]) + (part[2 * H + j] + part[3 * H + j]);
        __syncthreads();
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
