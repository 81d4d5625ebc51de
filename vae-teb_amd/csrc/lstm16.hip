// LSTM recurrences on 16-bit MFMA over 4-sample tiles: the encoders'
// nn.LSTM(in, 64, 4 layers, batch_first) (ref/model/vae_teb_model.py:474-480,
// :647-653) at the reference's 16-bit autocast width (graph_model.py:510,
// :709-711: cuDNN runs the LSTM with fp16 operands and fp32 accumulation).
// SURVEY.md §8(a) a12, §8(f) 1.
//
// The fp32 kernels (lstm.hip) give every sample its own workgroup and do the
// 64 x 256 recurrent matvec on packed-fp32 FMAs: ~105 VALU per step and wave,
// issue-bound at ~570-650 ns per step.  Here one workgroup of 4 waves carries
// FOUR samples, and the matvec is a v_mfma_f32_16x16x32 with the 4 samples as
// the A rows {0-3, 4-7, 8-11, 12-15} (each sample's h broadcast into its 4 rows:
// every lane reads, no masks, and element 0 of each lane's accumulator is its
// own sample's result).  Wave w owns units 16w .. 16w+15 of all four gates, so
// lane (s = lane>>4, u = 16w + (lane&15)) receives exactly the four gate
// pre-activations of (sample s, unit u): the cell is lane-local, each lane
// evaluates 5 activations per step (not 4 gates in every lane of a quad), and
// one LDS barrier per step hands h (16-bit) to the next step's A operand.
//
// Forward: f16 operands (h in [-1, 1], layer inputs O(1): the reference's own
// fp16), fp32 accumulate, fp32 cell state, gates and h written in fp32.  The
// input projection x W_ih^T + b of the NEXT 16-step chunk is a dense chunk GEMM
// (rows (sample, step) = 4 x 4 per M-tile, laid out so that its accumulator
// lands in the lanes that consume it: no LDS round trip), KX MFMAs per step
// issued under the step's LDS latency.
// Backward: bf16 operands (gradients need fp32's exponent range: the
// reference scales fp16 gradients with GradScaler, bf16 needs no scale), dh_rec
// = dg_{t+1} W_hh as 8 MFMAs per wave and step; dX = dG W_ih of the previous
// chunk as a dense chunk GEMM (2 MFMAs per step) from the chunk's bf16 dg image.
// dgates are written in fp32 for the weight gradients (vt_lstm_layer_bwd_weight).
#include <stdlib.h>

#include "common.h"
#include "lstm_cell.h"

namespace vt {
namespace l16 {

static constexpr int H = 64;
static constexpr int G4 = 4 * H;
static constexpr int NS = 4;    // samples per workgroup
static constexpr int TC = 16;   // steps per chunk (4 M-tiles of 4 steps x 4 samples)

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mma16(f16x8 a, f16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mmab(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// LDS hand-off barrier (waits for LDS traffic only, not for global stores/prefetches)
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// DIAG & 2 (timing probe only): shader-clock stamps of lane 0 of every wave of workgroup 0
// at three points of each step, vector-stored to dbg[(t * 4 + wave) * 3 + k]
__device__ __forceinline__ void stamp(unsigned long long* dbg, int t, int k) {
    const unsigned long long v = __builtin_amdgcn_s_memtime();
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) dbg[((int64_t)t * 4 + (threadIdx.x >> 6)) * 3 + k] = v;
}

__device__ __forceinline__ f16x8 to_f16(float4 a, float4 b) {
    return f16x8{(_Float16)a.x, (_Float16)a.y, (_Float16)a.z, (_Float16)a.w,
                 (_Float16)b.x, (_Float16)b.y, (_Float16)b.z, (_Float16)b.w};
}

static constexpr int HS = H + 8;   // f16 row stride of the h image (144 B)

// Activations on exponent-ready pre-activations.  The forward's weights and biases are
// pre-scaled (gate rows i, f, o by -log2 e, g by -2 log2 e) so the MFMA yields
// p = -x log2 e (or -2 x log2 e) directly:
//   sigmoid(x) = 1 / (1 + 2^p),   tanh(x) = 2 / (1 + 2^p) - 1.
// tanh's absolute error is ~1e-7 (relative accuracy near 0 is not kept, unlike lstm_cell.h's
// ftanh: h and g~ enter a 16-bit matvec and an fp32 LayerNorm, where absolute error counts).
static constexpr float NL2E = -1.44269504088896341f;
__device__ __forceinline__ float sg2(float p) { return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(p)); }
__device__ __forceinline__ float th2(float p) { return fmaf(2.f, sg2(p), -1.f); }
__device__ __forceinline__ float gate_scale(int g) { return g == 2 ? 2.f * NL2E : NL2E; }

// x [B, S, In] (In % 4 == 0, In <= 32 KX), w_ih [4H][In], w_hh [4H][H];
// out_h / out_hprev / out_c [B, S, H]; gates [B, S, H, 4]: post-activation (i, f, g~, o) of
// each unit contiguous (one 16-B store per lane and step; private to vt_lstm16_layer_bwd).
template <int KX, int DIAG = 0>
__global__ __launch_bounds__(G4) void k_lstm16_fwd(const float* __restrict__ x, int In, const float* __restrict__ wih,
                                                   const float* __restrict__ bih, const float* __restrict__ whh,
                                                   const float* __restrict__ bhh, int B, int S,
                                                   float* __restrict__ out_h, float* __restrict__ out_hprev,
                                                   float* __restrict__ out_c, float* __restrict__ gates) {
    __shared__ __attribute__((aligned(16))) _Float16 hs[2][NS][HS];
    const int j = threadIdx.x, lane = j & 63, w = j >> 6, ln = lane & 15, lg = lane >> 4;
    const int u = 16 * w + ln;                 // this lane's unit; its sample is lg
    const int b0 = blockIdx.x * NS;
    // output row base of (sample lg); lanes of samples past B compute the clamped sample's
    // values bit for bit (same inputs, same instructions) and store them unmasked
    const int64_t ob = (int64_t)(b0 + lg < B ? b0 + lg : B - 1) * S;
    // recurrence B fragments: B[k][n] = W_hh[g H + u][k], k = 32 ks + 8 lg + e
    f16x8 bh[4][2];
    // input-projection B fragments: W_ih[g H + u][k] (zero for k >= In)
    f16x8 bx[4][KX];
    float bias[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const float sc = gate_scale(g);
        const float* wr = whh + (int64_t)(g * H + u) * H;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const float4 p = *reinterpret_cast<const float4*>(wr + 32 * ks + 8 * lg);
            const float4 q = *reinterpret_cast<const float4*>(wr + 32 * ks + 8 * lg + 4);
            bh[g][ks] = to_f16(p * sc, q * sc);
        }
        const float* xr = wih + (int64_t)(g * H + u) * In;
#pragma unroll
        for (int ks = 0; ks < KX; ++ks) {
            const int k = 32 * ks + 8 * lg;
            float4 p = make_float4(0.f, 0.f, 0.f, 0.f), q = p;   // (a select of pointers would go through scratch)
            if (k < In) p = *reinterpret_cast<const float4*>(xr + k);
            if (k + 4 < In) q = *reinterpret_cast<const float4*>(xr + k + 4);
            bx[g][ks] = to_f16(p * sc, q * sc);
        }
        bias[g] = (bih[g * H + u] + bhh[g * H + u]) * sc;
    }
    // chunk-GEMM A operand: M-tile m, row rho = ln -> (sample ln >> 2, step 4 m + (ln & 3)),
    // k = 32 ks + 8 lg + e; its accumulator element r is (sample lg, step 4 m + r) of this
    // lane's unit — exactly the value this lane consumes at that step
    const int xs = b0 + (ln >> 2) < B ? b0 + (ln >> 2) : B - 1;
    const float* xb = x + (int64_t)xs * S * In;
    float4 xr[4][KX][2];
    f16x8 xa[4][KX];
    auto xload = [&](int t0) {
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int t = t0 + 4 * m + (ln & 3);
#pragma unroll
            for (int ks = 0; ks < KX; ++ks)
#pragma unroll
                for (int h2 = 0; h2 < 2; ++h2) {
                    const int k = 32 * ks + 8 * lg + 4 * h2;
                    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (t < S && k < In) v = *reinterpret_cast<const float4*>(xb + (int64_t)t * In + k);
                    xr[m][ks][h2] = v;
                }
        }
    };
    auto xcvt = [&]() {
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int ks = 0; ks < KX; ++ks) xa[m][ks] = to_f16(xr[m][ks][0], xr[m][ks][1]);
    };
    f32x4 gc[4][4], gn[4][4];   // [m][g]: x W_ih^T + b of the current / next chunk
    auto xtile = [&](int m, int g) {
        f32x4 acc = f32x4{bias[g], bias[g], bias[g], bias[g]};
#pragma unroll
        for (int ks = 0; ks < KX; ++ks) acc = mma16(xa[m][ks], bx[g][ks], acc);
        return acc;
    };
    for (int i = j; i < 2 * NS * HS; i += G4) (&hs[0][0][0])[i] = (_Float16)0.f;
    xload(0);
    xcvt();
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int g = 0; g < 4; ++g) gc[m][g] = xtile(m, g);
    xload(TC);
    xcvt();
    xload(2 * TC);
    lds_barrier();
    float c = 0.f, hprev = 0.f;
    for (int t0 = 0; t0 < S; t0 += TC) {
        const int n = S - t0 < TC ? S - t0 : TC;
        const bool more = t0 + TC < S;
#pragma unroll
        for (int i = 0; i < TC; ++i) {
            if (i >= n) continue;   // block-uniform
            const int t = t0 + i;
            if constexpr ((DIAG & 2) != 0) stamp(reinterpret_cast<unsigned long long*>(out_hprev), t, 0);
            const _Float16* hp = &hs[i & 1][ln >> 2][8 * lg];
            const f16x8 a0 = *reinterpret_cast<const f16x8*>(hp);
            const f16x8 a1 = *reinterpret_cast<const f16x8*>(hp + 32);
            if (more) gn[i >> 2][i & 3] = xtile(i >> 2, i & 3);   // next chunk, under the LDS latency
            // C operand = the chunk GEMM's whole accumulator: every row of this lane's
            // 4-row group is its sample, so element r is step 4 m + r's pre-activation
            f32x4 p[4];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                p[g] = mma16(a0, bh[g][0], gc[i >> 2][g]);
                p[g] = mma16(a1, bh[g][1], p[g]);
            }
            const int r = i & 3;
            const float gi = sg2(p[0][r]), gf = sg2(p[1][r]), gg = th2(p[2][r]), go = sg2(p[3][r]);
            if constexpr ((DIAG & 2) != 0) {
                asm volatile("" ::"v"(gi), "v"(gf), "v"(gg), "v"(go));
                stamp(reinterpret_cast<unsigned long long*>(out_hprev), t, 1);
            }
            c = cell_fwd_c(c, gi, gf, gg);
            const float hn = go * th2(2.f * NL2E * c);
            hs[(i + 1) & 1][lg][u] = (_Float16)hn;
            if constexpr ((DIAG & 2) != 0) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                stamp(reinterpret_cast<unsigned long long*>(out_hprev), t, 2);
            }
            if constexpr (!(DIAG & 3)) {
                *reinterpret_cast<float4*>(gates + ((ob + t) * H + u) * 4) = make_float4(gi, gf, gg, go);
                out_h[(ob + t) * H + u] = hn;
                out_hprev[(ob + t) * H + u] = hprev;
                out_c[(ob + t) * H + u] = c;
            }
            hprev = hn;
            lds_barrier();
        }
        if (more) {
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int g = 0; g < 4; ++g) gc[m][g] = gn[m][g];
            xcvt();
            xload(t0 + 3 * TC);
        }
    }
}

static constexpr int DS = G4 + 8;   // bf16 row stride of the dg image (528 B)

// gate row of dg-image column k' (k' = 4 u + g: a lane's 4 gate derivatives are one 8-B store)
__device__ __forceinline__ int krow(int k) { return (k & 3) * H + (k >> 2); }

// tanh with relative accuracy ~1e-7 only in absolute terms (see th2)
__device__ __forceinline__ float tanh16(float x) { return th2(2.f * NL2E * x); }

// dh_out [B, S, H] (gradient at the layer's outputs), gates [B, S, H, 4] / cst from the
// forward; dgates [B, S, 4H] fp32 (may be null), dx [B, S, In] (may be null), In <= 16 NTX.
// the cell derivatives of one step (lstm_cell.h cell_bwd with tanh(c_t) given)
__device__ __forceinline__ void cell_bwd16(float dh, float gi, float gf, float gg, float go, float tc, float cp,
                                           float& dc, float& v0, float& v1, float& v2, float& v3) {
    const float d_o = dh * tc;
    dc = fmaf(dh * go, fmaf(-tc, tc, 1.f), dc);
    const float di = dc * gg, dgg = dc * gi, df = dc * cp;
    dc = dc * gf;
    v0 = di * gi * (1.f - gi);
    v1 = df * gf * (1.f - gf);
    v2 = dgg * fmaf(-gg, gg, 1.f);
    v3 = d_o * go * (1.f - go);
}

template <int NTX, bool WD, int DIAG = 0>
__global__ __launch_bounds__(G4) void k_lstm16_bwd(const float* __restrict__ dh_out, const float* __restrict__ gates,
                                                   const float* __restrict__ cst, const float* __restrict__ whh,
                                                   const float* __restrict__ wih, int In, int B, int S,
                                                   float* __restrict__ dgates, float* __restrict__ dx) {
    // the chunk's dg images (rows (step, sample), bf16), double-buffered: the recurrence
    // reads step t+1's rows, the dX chunk GEMM reads the previous chunk's
    __shared__ __attribute__((aligned(16))) __bf16 dgs[2][TC][NS][DS];
    const int j = threadIdx.x, lane = j & 63, w = j >> 6, ln = lane & 15, lg = lane >> 4;
    const int u = 16 * w + ln;
    const int b0 = blockIdx.x * NS;
    const int64_t ob = (int64_t)(b0 + lg < B ? b0 + lg : B - 1) * S;
    // recurrence B fragments: B[k'][n] = W_hh[krow(k')][u], k' = 32 ks + 8 lg + e
    bf16x8 bw[8];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
#pragma unroll
        for (int e = 0; e < 8; ++e) bw[ks][e] = (__bf16)whh[(int64_t)krow(32 * ks + 8 * lg + e) * H + u];
    // dX B fragments: W_ih[k][col], col = 16 w + ln
    const bool dxw = dx != nullptr && w < NTX;   // wave-uniform
    const int col = 16 * w + ln;
    bf16x8 bxw[8];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
#pragma unroll
        for (int e = 0; e < 8; ++e)
            bxw[ks][e] = (__bf16)((dxw && col < In) ? wih[(int64_t)krow(32 * ks + 8 * lg + e) * In + col] : 0.f);
    for (int i = j; i < 2 * TC * NS * DS; i += G4) (&dgs[0][0][0][0])[i] = (__bf16)0.f;
    // step inputs of this lane's (sample, unit) in registers by half chunks of 8 steps: the
    // current half and the next one in flight (loads issued 8 steps before their use; every
    // global access of a step unconditional, so the compiler's vmcnt waits count exactly)
    float4 cg[8], ng[8];
    float cc[9], nc[9], cd[8], nd[8];
    auto load_half = [&](int tb) {   // steps tb .. tb + 7 (clamped), c from tb - 1
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            int t = tb + k;
            t = t < S ? t : S - 1;
            t = t > 0 ? t : 0;
            ng[k] = *reinterpret_cast<const float4*>(gates + ((ob + t) * H + u) * 4);
            nd[k] = dh_out[(ob + t) * H + u];
            nc[k + 1] = cst[(ob + t) * H + u];
        }
        const int tp = tb > 0 ? (tb - 1 < S ? tb - 1 : S - 1) : 0;
        nc[0] = cst[(ob + tp) * H + u];
        if (tb <= 0) nc[0] = 0.f;
    };
    auto take = [&]() {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            cg[k] = ng[k];
            cd[k] = nd[k];
        }
#pragma unroll
        for (int k = 0; k < 9; ++k) cc[k] = nc[k];
    };
    f32x4 ax[4];
    float* dxb = dx ? dx + ob * In : nullptr;
    // dX tile m of the chunk at p0 from image buffer pb: k-steps [ks0, ks0 + nk)
    auto dx_mma = [&](int pb, int m, int ks0, int nk) {
        const __bf16* ap = &dgs[pb][4 * m + (ln & 3)][ln >> 2][8 * lg];
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (q >= ks0 && q < ks0 + nk) ax[m] = mmab(*reinterpret_cast<const bf16x8*>(ap + 32 * q), bxw[q], ax[m]);
    };
    // rows of samples past B hold the clamped sample's values bit for bit: stored unmasked
    auto dx_store = [&](int p0, int m) {
        if (col >= In) return;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int t = p0 + 4 * m + r;
            if (t < S) dxb[(int64_t)t * In + col] = ax[m][r];
        }
    };
    const int tl0 = ((S - 1) / TC) * TC;   // first chunk processed (the last in time)
    load_half(tl0 + 8);
    lds_barrier();
    float dc = 0.f;
    int cur = 0;
    int p0 = -1;   // start step of the previous (time-later) chunk, whose dX is pending
    for (int t0 = tl0; t0 >= 0; t0 -= TC) {
        const int n = S - t0 < TC ? S - t0 : TC;
        const bool pend = p0 >= 0 && dxw;   // block-uniform
#pragma unroll
        for (int m = 0; m < 4; ++m) ax[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = TC - 1; i >= 0; --i) {
            if (i == 15) {   // upper half in hand, the lower half in flight
                take();
                load_half(t0);
            }
            if (i == 7) {    // lower half in hand, the next chunk's upper half in flight
                take();
                load_half(t0 - 8);
            }
            if (i >= n) continue;   // block-uniform (first processed chunk only)
            const int t = t0 + i, k8 = i & 7;
            if constexpr ((DIAG & 2) != 0) stamp(reinterpret_cast<unsigned long long*>(dx), t, 0);
            // dh_rec = dg_{t+1} W_hh: A rows are the 4 samples' dg at t + 1 (zero at t = S - 1);
            // all 8 A fragments read before the first MFMA
            const __bf16* ap = (i + 1 < TC) ? &dgs[cur][i + 1][ln >> 2][8 * lg] : &dgs[cur ^ 1][0][ln >> 2][8 * lg];
            bf16x8 af[8];
#pragma unroll
            for (int ks = 0; ks < 8; ++ks) af[ks] = *reinterpret_cast<const bf16x8*>(ap + 32 * ks);
            f32x4 a0 = f32x4{0.f, 0.f, 0.f, 0.f}, a1 = a0;
#pragma unroll
            for (int ks = 0; ks < 8; ks += 2) {
                a0 = mmab(af[ks], bw[ks], a0);
                a1 = mmab(af[ks + 1], bw[ks + 1], a1);
            }
            // the 8 LDS reads in flight together, then the 8 MFMAs (the scheduler otherwise
            // pairs them one read ahead: 4 LDS round trips per step)
            __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
            // the previous chunk's dX: tile q >> 2, k-steps 2 (q & 3) .. +1 (q = processing order)
            const int q = TC - 1 - i;
            if (pend) dx_mma(cur ^ 1, q >> 2, 2 * (q & 3), 2);
            const float dh = cd[k8] + (a0[0] + a1[0]);
            if constexpr ((DIAG & 2) != 0) {
                asm volatile("" ::"v"(dh));
                stamp(reinterpret_cast<unsigned long long*>(dx), t, 1);
            }
            float v0, v1, v2, v3;
            cell_bwd16(dh, cg[k8].x, cg[k8].y, cg[k8].z, cg[k8].w, tanh16(cc[k8 + 1]), cc[k8], dc, v0, v1, v2, v3);
            typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
            *reinterpret_cast<bf16x4*>(&dgs[cur][i][lg][4 * u]) = bf16x4{(__bf16)v0, (__bf16)v1, (__bf16)v2, (__bf16)v3};
            if constexpr ((DIAG & 2) != 0) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                stamp(reinterpret_cast<unsigned long long*>(dx), t, 2);
            }
            if constexpr (WD && !(DIAG & 3)) {
                float* o = dgates + (ob + t) * G4 + u;
                o[0] = v0;
                o[H] = v1;
                o[2 * H] = v2;
                o[3 * H] = v3;
            }
            if (pend && (q & 3) == 3 && !(DIAG & 2)) dx_store(p0, q >> 2);
            lds_barrier();
        }
        p0 = t0;
        cur ^= 1;
    }
    if (dxw && !(DIAG & 2)) {   // chunk 0's dX (its image is in dgs[cur ^ 1])
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            ax[m] = f32x4{0.f, 0.f, 0.f, 0.f};
            dx_mma(cur ^ 1, m, 0, 8);
            dx_store(0, m);
        }
    }
}

}  // namespace l16
}  // namespace vt

using namespace vt::l16;

extern "C" {

int vt_lstm16_layer_fwd(const float* x, int In, const float* w_ih, const float* b_ih, const float* w_hh,
                        const float* b_hh, int B, int seq, int hidden, float* out_h, float* out_hprev, float* out_c,
                        float* gates, void* stream) {
    VT_CHECK_ARG(hidden == H, "vt_lstm16_layer_fwd: hidden size %d (kernel built for %d)", hidden, H);
    VT_CHECK_ARG(B > 0 && seq > 0 && In > 0 && In <= 64 && In % 4 == 0,
                 "vt_lstm16_layer_fwd: shape (input size %d: a multiple of 4, at most 64)", In);
    VT_CHECK_ARG(x && w_ih && b_ih && w_hh && b_hh && out_h && out_hprev && out_c && gates,
                 "vt_lstm16_layer_fwd: null pointer");
    const dim3 grid((B + NS - 1) / NS);
    static const int diag = getenv("VAETEB_L16_DIAG") ? atoi(getenv("VAETEB_L16_DIAG")) : 0;   // timing probes only
#define VT_L16F(K_, D_)                                                                                        \
    hipLaunchKernelGGL((k_lstm16_fwd<K_, D_>), grid, dim3(G4), 0, vt::S(stream), x, In, w_ih, b_ih, w_hh, b_hh, B, \
                       seq, out_h, out_hprev, out_c, gates)
    if (diag == 1) {
        if (In <= 32) VT_L16F(1, 1); else VT_L16F(2, 1);
    } else if (diag == 2) {
        if (In <= 32) VT_L16F(1, 2); else VT_L16F(2, 2);
    } else {
        if (In <= 32) VT_L16F(1, 0); else VT_L16F(2, 0);
    }
#undef VT_L16F
    VT_LAUNCH_CHECK("vt_lstm16_layer_fwd");
    return VT_OK;
}

int vt_lstm16_layer_bwd(const float* dh_out, const float* gates, const float* cst, const float* w_hh,
                        const float* w_ih, int In, int B, int seq, int hidden, float* dgates, float* dx,
                        void* stream) {
    VT_CHECK_ARG(hidden == H, "vt_lstm16_layer_bwd: hidden size %d (kernel built for %d)", hidden, H);
    VT_CHECK_ARG(B > 0 && seq > 0 && In > 0 && In <= 64, "vt_lstm16_layer_bwd: shape (input size %d, at most 64)",
                 In);
    VT_CHECK_ARG(dh_out && gates && cst && w_hh && (w_ih || !dx), "vt_lstm16_layer_bwd: null pointer");
    const dim3 grid((B + NS - 1) / NS);
    const int ntx = (In + 15) / 16;
    static const int diag = getenv("VAETEB_L16_DIAG") ? atoi(getenv("VAETEB_L16_DIAG")) : 0;   // timing probes only
#define VT_L16B_(N_, W_, D_)                                                                                    \
    hipLaunchKernelGGL((k_lstm16_bwd<N_, W_, D_>), grid, dim3(G4), 0, vt::S(stream), dh_out, gates, cst, w_hh, w_ih, \
                       In, B, seq, dgates, dx)
#define VT_L16B(N_)                                 \
    case N_:                                        \
        if (diag == 1) VT_L16B_(N_, true, 1);       \
        else if (diag == 2) VT_L16B_(N_, true, 2);  \
        else if (dgates) VT_L16B_(N_, true, 0);     \
        else VT_L16B_(N_, false, 0);                \
        break;
    switch (ntx) { VT_L16B(1) VT_L16B(2) VT_L16B(3) VT_L16B(4) }
#undef VT_L16B_
#undef VT_L16B
    VT_LAUNCH_CHECK("vt_lstm16_layer_bwd");
    return VT_OK;
}

}  // extern "C"
