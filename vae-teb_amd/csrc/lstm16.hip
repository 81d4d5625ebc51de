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
// input projection x W_ih^T + b of a 16-step chunk is a dense chunk GEMM (rows
// (sample, step) = 4 x 4 per M-tile, laid out so that its accumulator lands in
// the lanes that consume it: no LDS round trip), one burst per chunk.
// Backward: bf16 operands (gradients need fp32's exponent range: the
// reference scales fp16 gradients with GradScaler, bf16 needs no scale), dh_rec
// = dg_{t+1} W_hh as 8 MFMAs per wave and step; dX = dG W_ih of a chunk as a
// dense chunk GEMM from the chunk's bf16 dg image, one burst per chunk.
// dgates are written in fp32 for the weight gradients (vt_lstm_layer_bwd_weight).
#include <stdlib.h>

#include "common.h"
#include "lstm_cell.h"

namespace vt {
namespace l16 {

static constexpr int H = 64;
static constexpr int G4 = 4 * H;
static constexpr int TC = 16;   // steps per chunk

// flags of the chained launches (k_lstm16_fwd4 / _bwd4): T x nch words per launch from a pool
// (arrive_slots: launches on different streams never share them), and the bounded waits'
// timeout counter (vt_lstm16_chain_errors)
VT_ARRIVE_POOL(g_chain_flags);
static __device__ unsigned g_chain_err[1];

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
// out_h / out_c [B, S, H], out_hprev [B, S, H] (HP only); gates [B, S, H, 4]: post-activation
// (i, f, g~, o) of each unit contiguous (one 16-B store per lane and step; private to
// vt_lstm16_layer_bwd).  NS samples per workgroup (4 or 2): the 4 row groups of the MFMA
// tiles hold samples lg & (NS - 1) — with NS = 2 the lanes of groups 2, 3 repeat groups 0, 1
// and only groups 0, 1 store (half the per-CU store traffic, twice the workgroups).
template <int NS, int KX, bool HP, int DIAG = 0>
__global__ __launch_bounds__(G4) void k_lstm16_fwd(const float* __restrict__ x, int In, const float* __restrict__ wih,
                                                   const float* __restrict__ bih, const float* __restrict__ whh,
                                                   const float* __restrict__ bhh, int B, int S,
                                                   float* __restrict__ out_h, float* __restrict__ out_hprev,
                                                   float* __restrict__ out_c, float* __restrict__ gates) {
    __shared__ __attribute__((aligned(16))) _Float16 hs[2][NS][HS];
    const int j = threadIdx.x, lane = j & 63, w = j >> 6, ln = lane & 15, lg = lane >> 4;
    const int u = 16 * w + ln;                 // this lane's unit; its sample is sl
    const int sl = lg & (NS - 1), sa = (ln >> 2) & (NS - 1);   // the A row's sample: sa
    const bool wr = NS == 4 || lg < NS;        // the lanes that store
    const int b0 = blockIdx.x * NS;
    // output row base of (sample sl); lanes of samples past B compute the clamped sample's
    // values bit for bit (same inputs, same instructions) and store them unmasked
    const int64_t ob = (int64_t)(b0 + sl < B ? b0 + sl : B - 1) * S;
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
    // chunk-GEMM A operand: M-tile m, row rho = ln -> (sample sa, step 4 m + (ln & 3)),
    // k = 32 ks + 8 lg + e; its accumulator element r is (sample sl, step 4 m + r) of this
    // lane's unit — exactly the value this lane consumes at that step.  Computed at the start of
// each chunk (x converted a chunk ahead, loaded two ahead).
    const int xs = b0 + sa < B ? b0 + sa : B - 1;
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
    f32x4 gc[4][4];   // [m][g]: x W_ih^T + b of the current chunk
    auto xtile = [&](int m, int g) {
        f32x4 acc = f32x4{bias[g], bias[g], bias[g], bias[g]};
#pragma unroll
        for (int ks = 0; ks < KX; ++ks) acc = mma16(xa[m][ks], bx[g][ks], acc);
        return acc;
    };
    for (int i = j; i < 2 * NS * HS; i += G4) (&hs[0][0][0])[i] = (_Float16)0.f;
    xload(0);
    xcvt();
    xload(TC);
    lds_barrier();
    float c = 0.f, hprev = 0.f;
    for (int t0 = 0; t0 < S; t0 += TC) {
        const int n = S - t0 < TC ? S - t0 : TC;
        // the chunk's input projection as one burst of 16 KX MFMAs (issued per step beside the
        // recurrence's MFMAs it cost ~130 ns per step), then the next chunk's x converted and
        // the one after it loaded
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int g = 0; g < 4; ++g) gc[m][g] = xtile(m, g);
        xcvt();
        xload(t0 + 2 * TC);
#pragma unroll
        for (int i = 0; i < TC; ++i) {
            if (i >= n) continue;   // block-uniform
            const int t = t0 + i;
            if constexpr ((DIAG & 2) != 0) stamp(reinterpret_cast<unsigned long long*>(out_hprev), t, 0);
            const _Float16* hp = &hs[i & 1][sa][8 * lg];
            const f16x8 a0 = *reinterpret_cast<const f16x8*>(hp);
            const f16x8 a1 = *reinterpret_cast<const f16x8*>(hp + 32);
            // C operand = the chunk GEMM's whole accumulator: every row of this lane's
            // 4-row group is its sample, so element r is step 4 m + r's pre-activation
            f32x4 p[4];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                p[g] = mma16(a0, bh[g][0], gc[i >> 2][g]);
                p[g] = mma16(a1, bh[g][1], p[g]);
            }
            const int r = i & 3;
            float gi, gf, gg, go;
            if constexpr ((DIAG & 16) != 0) {   // probe: no activations
                gi = p[0][r] * 0.1f, gf = p[1][r] * 0.1f, gg = p[2][r] * 0.1f, go = p[3][r] * 0.1f;
            } else {
                gi = sg2(p[0][r]), gf = sg2(p[1][r]), gg = th2(p[2][r]), go = sg2(p[3][r]);
            }
            if constexpr ((DIAG & 2) != 0) {
                asm volatile("" ::"v"(gi), "v"(gf), "v"(gg), "v"(go));
                stamp(reinterpret_cast<unsigned long long*>(out_hprev), t, 1);
            }
            c = cell_fwd_c(c, gi, gf, gg);
            const float hn = (DIAG & 16) ? go * c : go * th2(2.f * NL2E * c);
            hs[(i + 1) & 1][sl][u] = (_Float16)hn;
            if constexpr ((DIAG & 2) != 0) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                stamp(reinterpret_cast<unsigned long long*>(out_hprev), t, 2);
            }
            if (!(DIAG & 3) && wr) {
                *reinterpret_cast<float4*>(gates + ((ob + t) * H + u) * 4) = make_float4(gi, gf, gg, go);
                out_h[(ob + t) * H + u] = hn;
                if constexpr (HP) out_hprev[(ob + t) * H + u] = hprev;
                out_c[(ob + t) * H + u] = c;
            }
            hprev = hn;
            lds_barrier();
        }
    }
}

// ---------------------------------------------------------------- two layers per workgroup
// Wavefront pipelining of a layer pair.  The recurrence is a latency
// chain (~50 instructions per wave and step against ~900 cycles of dependent latency), so one
// wave per SIMD leaves most issue slots idle.  Here one workgroup of 8 waves carries layers
// l (role A, waves 0-3) and l + 1 (role B, waves 4-7) of the same NS samples: B runs one
// 16-step chunk behind A, both step in lockstep under one barrier per step, and each SIMD
// interleaves an A wave with a B wave.  A's h of a chunk goes to B through an LDS image
// (16-bit, the A-operand layout of B's input-projection MFMAs) instead of HBM; A's whole
// input sequence is staged into LDS once, at the start, by coalesced loads (no global loads
// inside the step loop, so no wait there on the outstanding output stores).  The pair takes
// S + 16 steps where two layer launches take 2 S; per role the arithmetic is k_lstm16_fwd's
// (same operands, same MFMA chains, same activation code), so the outputs are bit-identical
// to two vt_lstm16_layer_fwd calls.
static constexpr int HX = H + 8;   // f16 row stride of the input images (144 B)
static constexpr int64_t L16_PAIR_STAGE_MAX = 120 * 1024;   // + ~20 KB static: within 160 KB

// LDS bytes of the staged input of one workgroup (dynamic shared memory)
__host__ __device__ constexpr int64_t fwd2_stage_bytes(int ns, int S) {
    return (int64_t)ns * ((S + TC - 1) / TC) * TC * HX * 2;
}

// Chained layer pairs (round 6): the four layers of an encoder in ONE
// launch, pair 0 (layers 0, 1) in workgroups [0, T) and pair 1 (layers 2, 3) in [T, 2T), tile b's
// consumer at b + T.  Pair 0's upper layer publishes each finished 16-step chunk of its h —
// agent-coherent (sc1) stores, a wait for them, then a per-(tile, chunk) flag — and pair 1's lower
// layer stages that chunk into its input image when the flag is up (sc1 loads), instead of waiting
// for the whole first launch: 4 layers in S + 4 chunks of steps instead of 2 (S + 1 chunk).  A
// consumer only waits on a workgroup of LOWER index (in-order dispatch: resident or finished,
// and with T a multiple of 8 on the same XCD), producers never wait: no deadlock whatever the
// occupancy; the waits are bounded anyway (a timeout counts an error, vt_lstm16_chain_errors).
// CH: 0 an independent pair, 1 producer, 2 consumer.
constexpr unsigned CHAIN_SPIN_MAX = 1u << 23;   // ~0.5 s of polling, then give up (counted)

__device__ __forceinline__ void chain_wait(unsigned* flag, unsigned* err) {
    unsigned n = 0;
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
        __builtin_amdgcn_s_sleep(2);
        if (++n > CHAIN_SPIN_MAX) {
            if ((threadIdx.x & 63) == 0) atomicAdd(err, 1u);
            break;
        }
    }
}

template <int NS, int KX, int ROLE, int CH = 0>
__device__ __forceinline__ void fwd2_role(int In, const float* __restrict__ wih, const float* __restrict__ bih,
                                          const float* __restrict__ whh, const float* __restrict__ bhh, int B, int S,
                                          float* __restrict__ out_h, float* __restrict__ out_c,
                                          float* __restrict__ gates, _Float16 (*hs)[NS][HS], _Float16* ximg,
                                          _Float16 (*himg)[NS][TC][HX], int tile = 0, unsigned* flags = nullptr,
                                          unsigned* err = nullptr, const float* __restrict__ xin = nullptr) {
    const int j = threadIdx.x & (G4 - 1), lane = j & 63, w = j >> 6, ln = lane & 15, lg = lane >> 4;
    const int u = 16 * w + ln;
    const int sl = lg & (NS - 1), sa = (ln >> 2) & (NS - 1);
    const bool wr = NS == 4 || lg < NS;
    const int b0 = (CH ? tile : (int)blockIdx.x) * NS;
    // producer's upper layer: h through the coherence point (the consumer may sit on another XCD)
    const __amdgpu_buffer_rsrc_t hrs = agent_rsrc(out_h, (int64_t)B * S * H * 4);
    const int64_t ob = (int64_t)(b0 + sl < B ? b0 + sl : B - 1) * S;
    f16x8 bh[4][2];
    f16x8 bx[4][KX];
    float bias[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const float sc = gate_scale(g);
        const float* wr_ = whh + (int64_t)(g * H + u) * H;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const float4 p = *reinterpret_cast<const float4*>(wr_ + 32 * ks + 8 * lg);
            const float4 q = *reinterpret_cast<const float4*>(wr_ + 32 * ks + 8 * lg + 4);
            bh[g][ks] = to_f16(p * sc, q * sc);
        }
        const float* xr = wih + (int64_t)(g * H + u) * In;
#pragma unroll
        for (int ks = 0; ks < KX; ++ks) {
            const int k = 32 * ks + 8 * lg;
            float4 p = make_float4(0.f, 0.f, 0.f, 0.f), q = p;
            if (k < In) p = *reinterpret_cast<const float4*>(xr + k);
            if (k + 4 < In) q = *reinterpret_cast<const float4*>(xr + k + 4);
            bx[g][ks] = to_f16(p * sc, q * sc);
        }
        bias[g] = (bih[g * H + u] + bhh[g * H + u]) * sc;
    }
    const int nch = (S + TC - 1) / TC;
    f32x4 gc[4][4];
    float c = 0.f;
    for (int k = 0; k <= nch; ++k) {
        const int ch = ROLE == 0 ? k : k - 1;   // this role's chunk in period k
        const bool act = ch >= 0 && ch < nch;   // block-uniform per role
        const int n = act ? (S - TC * ch < TC ? S - TC * ch : TC) : 0;
        if constexpr (CH == 2) {
            // consumer: this chunk of the producer's h (its input), f16 as the staging of the
            // independent pair converts it, once its flag is up
            if (ROLE == 0 && act) {
                unsigned* fl = flags + tile * nch + ch;
                chain_wait(fl, err);
                typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
                const __amdgpu_buffer_rsrc_t xr = agent_rsrc(xin, (int64_t)B * S * In * 4);
                const int i4 = In >> 2, per = TC * i4;
                for (int q = j; q < NS * per; q += G4) {
                    const int s_ = q / per, rem = q - s_ * per, tt = rem / i4, k4 = rem - tt * i4, t = TC * ch + tt;
                    const int bs = b0 + s_ < B ? b0 + s_ : B - 1;
                    if (t < S) {
                        const float4 v = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                            xr, (int)((((int64_t)bs * S + t) * In + 4 * k4) * 4), 0, CPOL_SC1));
                        *reinterpret_cast<f16x4*>(ximg + ((int64_t)s_ * nch * TC + t) * HX + 4 * k4) =
                            f16x4{(_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
                    }
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            lds_barrier();   // the chunk's input image complete (both roles: one barrier more per period)
            if (ROLE == 0 && act && j == 0) atomicExch(flags + tile * nch + ch, 0u);   // every wave saw it
        }
        if (act) {
            // the chunk's input projection from its 16-bit image: A rows (sample sa, step
            // 4 m + (ln & 3)), k = 32 ks + 8 lg + e (zero columns past In)
            const _Float16* im = ROLE == 0 ? ximg + ((int64_t)sa * nch * TC + TC * ch) * HX : &himg[ch & 1][sa][0][0];
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                f16x8 xa[KX];
#pragma unroll
                for (int ks = 0; ks < KX; ++ks)
                    xa[ks] = *reinterpret_cast<const f16x8*>(im + (4 * m + (ln & 3)) * HX + 32 * ks + 8 * lg);
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    f32x4 acc = f32x4{bias[g], bias[g], bias[g], bias[g]};
#pragma unroll
                    for (int ks = 0; ks < KX; ++ks) acc = mma16(xa[ks], bx[g][ks], acc);
                    gc[m][g] = acc;
                }
            }
        }
#pragma unroll
        for (int i = 0; i < TC; ++i) {
            if (i < n) {
                const int t = TC * ch + i;
                const _Float16* hp = &hs[i & 1][sa][8 * lg];
                const f16x8 a0 = *reinterpret_cast<const f16x8*>(hp);
                const f16x8 a1 = *reinterpret_cast<const f16x8*>(hp + 32);
                f32x4 p[4];
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    p[g] = mma16(a0, bh[g][0], gc[i >> 2][g]);
                    p[g] = mma16(a1, bh[g][1], p[g]);
                }
                const int r = i & 3;
                const float gi = sg2(p[0][r]), gf = sg2(p[1][r]), gg = th2(p[2][r]), go = sg2(p[3][r]);
                c = cell_fwd_c(c, gi, gf, gg);
                const float hn = go * th2(2.f * NL2E * c);
                // (as in k_lstm16_fwd the compiler rounds go * tanh to f16 once, v_fma_mixlo_f16)
                hs[(i + 1) & 1][sl][u] = (_Float16)hn;
                if (ROLE == 0) {
                    // the layer above reads h as the fp32 out_h rounded to f16 (twice rounded):
                    // an opaque fp32 copy keeps the product from being fused into the conversion
                    float hq = hn;
                    asm volatile("" : "+v"(hq));
                    himg[ch & 1][sl][i][u] = (_Float16)hq;
                }
                if (wr) {
                    *reinterpret_cast<float4*>(gates + ((ob + t) * H + u) * 4) = make_float4(gi, gf, gg, go);
                    if (CH == 1 && ROLE == 1)
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, hn), hrs,
                                                              (int)(((ob + t) * H + u) * 4), 0, CPOL_SC1);
                    else
                        out_h[(ob + t) * H + u] = hn;
                    out_c[(ob + t) * H + u] = c;
                }
            }
            lds_barrier();
        }
        if constexpr (CH == 1) {
            // producer: the chunk's h stores have reached the coherence point, then its flag
            if (ROLE == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            lds_barrier();
            if (ROLE == 1 && act && j == 0) atomicAdd(flags + tile * nch + ch, 1u);
        }
    }
}

// x [B, S, In] (In % 4 == 0, In <= 32 KXA); layer A's outputs hA / cA / gA, layer B's (input
// size H) hB / cB / gB, as k_lstm16_fwd's (no h_{t-1} output).  Dynamic LDS:
// fwd2_stage_bytes(NS, S), A's input [NS][ceil16(S)][HX] in f16.
template <int NS, int KXA>
__global__ __launch_bounds__(2 * G4) void k_lstm16_fwd2(const float* __restrict__ x, int In,
                                                        const float* __restrict__ wihA, const float* __restrict__ bihA,
                                                        const float* __restrict__ whhA, const float* __restrict__ bhhA,
                                                        const float* __restrict__ wihB, const float* __restrict__ bihB,
                                                        const float* __restrict__ whhB, const float* __restrict__ bhhB,
                                                        int B, int S, float* __restrict__ hA, float* __restrict__ cA,
                                                        float* __restrict__ gA, float* __restrict__ hB,
                                                        float* __restrict__ cB, float* __restrict__ gB) {
    __shared__ __attribute__((aligned(16))) _Float16 hsA[2][NS][HS];
    __shared__ __attribute__((aligned(16))) _Float16 hsB[2][NS][HS];
    __shared__ __attribute__((aligned(16))) _Float16 himg[2][NS][TC][HX];
    extern __shared__ __attribute__((aligned(16))) _Float16 ximg[];
    const int nch = (S + TC - 1) / TC, rows = NS * nch * TC;
    // zero: the recurrence images (h_{-1} = 0), the staged input (columns past In, steps
    // past S, samples past B), then the input itself in f16 (the same conversion as
    // k_lstm16_fwd's operand)
    for (int i = threadIdx.x; i < 2 * NS * HS; i += 2 * G4) {
        (&hsA[0][0][0])[i] = (_Float16)0.f;
        (&hsB[0][0][0])[i] = (_Float16)0.f;
    }
    typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
    for (int i = threadIdx.x; i < rows * HX / 4; i += 2 * G4)
        reinterpret_cast<f16x4*>(ximg)[i] = f16x4{(_Float16)0.f, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f};
    lds_barrier();
    {
        const int i4 = In >> 2, b0 = blockIdx.x * NS;
        const int per = S * i4, total = NS * per;
        constexpr int U = 8;
        for (int q0 = threadIdx.x; q0 < total; q0 += U * 2 * G4) {
            float4 v[U];
#pragma unroll
            for (int r = 0; r < U; ++r) {
                const int q = q0 + r * 2 * G4;
                const int s = q / per, rem = q - s * per, t = rem / i4, k4 = rem - t * i4;
                const int bs = b0 + s < B ? b0 + s : B - 1;
                v[r] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (q < total) v[r] = *reinterpret_cast<const float4*>(x + ((int64_t)bs * S + t) * In + 4 * k4);
            }
#pragma unroll
            for (int r = 0; r < U; ++r) {
                const int q = q0 + r * 2 * G4;
                const int s = q / per, rem = q - s * per, t = rem / i4, k4 = rem - t * i4;
                if (q < total)
                    *reinterpret_cast<f16x4*>(ximg + ((int64_t)s * nch * TC + t) * HX + 4 * k4) =
                        f16x4{(_Float16)v[r].x, (_Float16)v[r].y, (_Float16)v[r].z, (_Float16)v[r].w};
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    if (threadIdx.x < G4)
        fwd2_role<NS, KXA, 0>(In, wihA, bihA, whhA, bhhA, B, S, hA, cA, gA, hsA, ximg, himg);
    else
        fwd2_role<NS, 2, 1>(H, wihB, bihB, whhB, bhhB, B, S, hB, cB, gB, hsB, ximg, himg);
}

// the four layers' parameters [w_ih, w_hh, b_ih, b_hh] x 4 (the Python flat list's order) and
// outputs [h, c, gates] x 4 of a chained launch
struct Quad {
    const float* p[16];
    float* o[12];
};

// zero the recurrence images and the staged input image, then (stage) the tile's whole input
// x [B, S, In] in f16 (k_lstm16_fwd2's prologue)
template <int NS>
__device__ __forceinline__ void fwd2_prologue(const float* __restrict__ x, int In, int B, int S, int b0, bool stage,
                                              _Float16 (*hsA)[NS][HS], _Float16 (*hsB)[NS][HS], _Float16* ximg) {
    const int nch = (S + TC - 1) / TC, rows = NS * nch * TC;
    for (int i = threadIdx.x; i < 2 * NS * HS; i += 2 * G4) {
        (&hsA[0][0][0])[i] = (_Float16)0.f;
        (&hsB[0][0][0])[i] = (_Float16)0.f;
    }
    typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
    for (int i = threadIdx.x; i < rows * HX / 4; i += 2 * G4)
        reinterpret_cast<f16x4*>(ximg)[i] = f16x4{(_Float16)0.f, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f};
    lds_barrier();
    if (stage) {
        const int i4 = In >> 2;
        const int per = S * i4, total = NS * per;
        constexpr int U = 8;
        for (int q0 = threadIdx.x; q0 < total; q0 += U * 2 * G4) {
            float4 v[U];
#pragma unroll
            for (int r = 0; r < U; ++r) {
                const int q = q0 + r * 2 * G4;
                const int s = q / per, rem = q - s * per, t = rem / i4, k4 = rem - t * i4;
                const int bs = b0 + s < B ? b0 + s : B - 1;
                v[r] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (q < total) v[r] = *reinterpret_cast<const float4*>(x + ((int64_t)bs * S + t) * In + 4 * k4);
            }
#pragma unroll
            for (int r = 0; r < U; ++r) {
                const int q = q0 + r * 2 * G4;
                const int s = q / per, rem = q - s * per, t = rem / i4, k4 = rem - t * i4;
                if (q < total)
                    *reinterpret_cast<f16x4*>(ximg + ((int64_t)s * nch * TC + t) * HX + 4 * k4) =
                        f16x4{(_Float16)v[r].x, (_Float16)v[r].y, (_Float16)v[r].z, (_Float16)v[r].w};
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    lds_barrier();
}

// four layers in one launch (see fwd2_role): workgroups [0, T) run layers 0, 1 of tile b (the
// producer: the staged input x [B, S, In], In <= 32 KXA), [T, 2T) layers 2, 3 of tile b - T (the
// consumer: its input, layer 1's h, staged chunk by chunk as published).  slot0: T x nch zeroed
// words of g_chain_flags (left zero by the consumers).  Same arithmetic
// per role as two k_lstm16_fwd2 launches: the same bits.
template <int NS, int KXA>
__global__ __launch_bounds__(2 * G4) void k_lstm16_fwd4(const float* __restrict__ x, int In, Quad q, int B, int S,
                                                        int T, unsigned slot0) {
    unsigned* flags = g_chain_flags + slot0;
    unsigned* err = g_chain_err;
    __shared__ __attribute__((aligned(16))) _Float16 hsA[2][NS][HS];
    __shared__ __attribute__((aligned(16))) _Float16 hsB[2][NS][HS];
    __shared__ __attribute__((aligned(16))) _Float16 himg[2][NS][TC][HX];
    extern __shared__ __attribute__((aligned(16))) _Float16 ximg[];
    const bool cons = (int)blockIdx.x >= T;
    const int tile = cons ? (int)blockIdx.x - T : (int)blockIdx.x;
    fwd2_prologue<NS>(x, In, B, S, tile * NS, !cons, hsA, hsB, ximg);
    const bool A = threadIdx.x < G4;
    if (!cons) {
        if (A)
            fwd2_role<NS, KXA, 0, 1>(In, q.p[0], q.p[2], q.p[1], q.p[3], B, S, q.o[0], q.o[1], q.o[2], hsA, ximg,
                                     himg, tile, flags, err);
        else
            fwd2_role<NS, 2, 1, 1>(H, q.p[4], q.p[6], q.p[5], q.p[7], B, S, q.o[3], q.o[4], q.o[5], hsB, ximg, himg,
                                   tile, flags, err);
    } else {
        if (A)
            fwd2_role<NS, 2, 0, 2>(H, q.p[8], q.p[10], q.p[9], q.p[11], B, S, q.o[6], q.o[7], q.o[8], hsA, ximg,
                                   himg, tile, flags, err, q.o[3]);
        else
            fwd2_role<NS, 2, 1, 2>(H, q.p[12], q.p[14], q.p[13], q.p[15], B, S, q.o[9], q.o[10], q.o[11], hsB, ximg,
                                   himg, tile, flags, err);
    }
}

static constexpr int DS = G4 + 8;   // bf16 row stride of the dg image (528 B)

// gate row of dg-image column k' (k' = 4 u + g: a lane's 4 gate derivatives are one 8-B store)
__device__ __forceinline__ int krow(int k) { return (k & 3) * H + (k >> 2); }

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

// NS samples per workgroup as in the forward.  The dX chunk GEMM's M-tiles hold RPS = 16 / NS
// steps of each sample (row rho = RPS s + tl), TC NS / 16 tiles per chunk.
template <int NS, int NTX, bool WD, int DIAG = 0>
__global__ __launch_bounds__(G4) void k_lstm16_bwd(const float* __restrict__ dh_out, const float* __restrict__ gates,
                                                   const float* __restrict__ cst, const float* __restrict__ whh,
                                                   const float* __restrict__ wih, int In, int B, int S,
                                                   float* __restrict__ dgates, float* __restrict__ dx) {
    // the chunk's dg images (rows (step, sample), bf16), double-buffered: the recurrence
    // reads step t+1's rows, the dX chunk GEMM reads the previous chunk's
    __shared__ __attribute__((aligned(16))) __bf16 dgs[2][TC][NS][DS];
    const int j = threadIdx.x, lane = j & 63, w = j >> 6, ln = lane & 15, lg = lane >> 4;
    const int u = 16 * w + ln;
    const int sl = lg & (NS - 1), sa = (ln >> 2) & (NS - 1);
    const bool wr = NS == 4 || lg < NS;
    constexpr int RPS = 16 / NS, MT = TC * NS / 16;
    const int b0 = blockIdx.x * NS;
    const int64_t ob = (int64_t)(b0 + sl < B ? b0 + sl : B - 1) * S;
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
    f32x4 ax[MT];
    // dX tile m of a chunk from image buffer pb: A row rho = ln -> (sample ln / RPS, step
    // m RPS + ln % RPS); accumulator row 4 lg + r -> (sample (4 lg + r) / RPS, step ...)
    auto dx_mma = [&](int pb, int m) {
        const __bf16* ap = &dgs[pb][m * RPS + ln % RPS][ln / RPS][8 * lg];
#pragma unroll
        for (int q = 0; q < 8; ++q) ax[m] = mmab(*reinterpret_cast<const bf16x8*>(ap + 32 * q), bxw[q], ax[m]);
    };
    // rows of samples past B hold the clamped sample's values bit for bit: stored unmasked
    auto dx_store = [&](int p0, int m) {
        if (col >= In || !dx) return;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = 4 * lg + r, sr = row / RPS, t = p0 + m * RPS + row % RPS;
            const int64_t b = b0 + sr < B ? b0 + sr : B - 1;
            if (t < S) dx[(b * S + t) * In + col] = ax[m][r];
        }
    };
    const int tl0 = ((S - 1) / TC) * TC;   // first chunk processed (the last in time)
    load_half(tl0 + 8);
    lds_barrier();
    float dc = 0.f;
    int cur = 0;
    for (int t0 = tl0; t0 >= 0; t0 -= TC) {
        const int n = S - t0 < TC ? S - t0 : TC;
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
            const __bf16* ap = (i + 1 < TC) ? &dgs[cur][i + 1][sa][8 * lg] : &dgs[cur ^ 1][0][sa][8 * lg];
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
            const float dh = cd[k8] + (a0[0] + a1[0]);
            if constexpr ((DIAG & 2) != 0) {
                asm volatile("" ::"v"(dh));
                stamp(reinterpret_cast<unsigned long long*>(dx), t, 1);
            }
            float v0, v1, v2, v3;
            // tanh(c_t) with lstm_cell.h's relative accuracy near 0 (dg_o is proportional to it;
            // it depends on loaded c only, off the recurrence chain)
            cell_bwd16(dh, cg[k8].x, cg[k8].y, cg[k8].z, cg[k8].w, ftanh(cc[k8 + 1]), cc[k8], dc, v0, v1, v2, v3);
            typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
            *reinterpret_cast<bf16x4*>(&dgs[cur][i][sl][4 * u]) = bf16x4{(__bf16)v0, (__bf16)v1, (__bf16)v2, (__bf16)v3};
            if constexpr ((DIAG & 2) != 0) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                stamp(reinterpret_cast<unsigned long long*>(dx), t, 2);
            }
            if (WD && !(DIAG & 3) && wr) {
                float* o = dgates + (ob + t) * G4 + u;
                o[0] = v0;
                o[H] = v1;
                o[2 * H] = v2;
                o[3 * H] = v3;
            }
            lds_barrier();
        }
        // the chunk's dX = dG W_ih as one burst of 32 MFMAs per column tile from the complete
        // image (spread over the steps beside the recurrence's MFMAs it cost more than it hid)
        if (dxw && !(DIAG & 2)) {
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                ax[m] = f32x4{0.f, 0.f, 0.f, 0.f};
                dx_mma(cur, m);
            }
#pragma unroll
            for (int m = 0; m < MT; ++m) dx_store(t0, m);
        }
        cur ^= 1;
    }
}

// Backward of a layer pair: role U (waves 0-3) runs layer l + 1's backward recurrence,
// role L (waves 4-7) layer l's one chunk behind it (both walk the chunks from the last in
// time to the first).  U's dX = dG W_ih of a chunk — the gradient at layer l's outputs — goes
// to L through an LDS image (fp32, [NS][TC][H]) instead of HBM; L reads it one step at a
// time.  Per role the arithmetic is k_lstm16_bwd's instruction for instruction, so dgates of
// both layers and L's dX are bit-identical to two vt_lstm16_layer_bwd calls.
// CH (chained backward, k_lstm16_bwd4): 1 = the upper pair (layers 3, 2), whose lower role publishes
// its dX chunk by chunk (sc1 stores, a wait, the chunk's flag); 2 = the lower pair (layers 1, 0),
// whose upper role reads dh_out (= that dX) with sc1 loads, each chunk after its flag is up.
template <int NS, int NTX, int ROLE, int CH = 0>
__device__ __forceinline__ void bwd2_role(const float* __restrict__ dh_out, const float* __restrict__ gates,
                                          const float* __restrict__ cst, const float* __restrict__ whh,
                                          const float* __restrict__ wih, int In, int B, int S,
                                          float* __restrict__ dgates, float* __restrict__ dx,
                                          __bf16 (*dgs)[TC][NS][DS], float (*dximg)[NS][TC][H],
                                          __bf16 (*wT)[DS], int tile = 0, unsigned* flags = nullptr,
                                          unsigned* err = nullptr) {
    const int j = threadIdx.x & (G4 - 1), lane = j & 63, w = j >> 6, ln = lane & 15, lg = lane >> 4;
    const int u = 16 * w + ln;
    const int sl = lg & (NS - 1), sa = (ln >> 2) & (NS - 1);
    const bool wr = NS == 4 || lg < NS;
    constexpr int RPS = 16 / NS, MT = TC * NS / 16;
    const int b0 = (CH ? tile : (int)blockIdx.x) * NS;
    const int nchk = (S + TC - 1) / TC;
    const __amdgpu_buffer_rsrc_t drs = agent_rsrc(CH == 2 ? dh_out : dx, (int64_t)B * S * (CH == 2 ? H : In) * 4);
    const int64_t ob = (int64_t)(b0 + sl < B ? b0 + sl : B - 1) * S;
    bf16x8 bw[8];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
#pragma unroll
        for (int e = 0; e < 8; ++e) bw[ks][e] = (__bf16)whh[(int64_t)krow(32 * ks + 8 * lg + e) * H + u];
    // U's dX always (it is L's dh); L's only into a given dx.  The dX B operand (W_ih by
    // column, bf16, rows k' of the dg image) lives in LDS, not in 32 registers per lane: it is
    // read once per chunk, and two roles' registers must fit 256 per lane
    const bool dxw = (ROLE == 0 || dx != nullptr) && w < NTX;   // wave-uniform
    const int col = 16 * w + ln;
    for (int e = j; e < H * G4; e += G4) {
        const int cc_ = e / G4, kk = e - cc_ * G4;
        wT[cc_][kk] = (__bf16)(cc_ < In && (ROLE == 0 || dx != nullptr) ? wih[(int64_t)krow(kk) * In + cc_] : 0.f);
    }
    // step inputs of this lane's (sample, unit) by half chunks, in two fixed register sets:
    // A holds a chunk's upper half (steps 15..8), B its lower half; each is reloaded right
    // after its last use, 8 steps before its next one (no copies: a register hand-over across
    // the chunk loop's back edge would wait for the loads in flight)
    float4 gA[8], gB[8];
    float cA[9], cB[9], dA[8], dB[8];
    auto load_half = [&](int tb, float4(&g)[8], float(&c)[9], float(&d)[8]) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            int t = tb + k;
            t = t < S ? t : S - 1;
            t = t > 0 ? t : 0;
            g[k] = *reinterpret_cast<const float4*>(gates + ((ob + t) * H + u) * 4);
            if (ROLE == 0 && CH == 2)
                d[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                     drs, (int)(((ob + t) * H + u) * 4), 0, CPOL_SC1));
            else if (ROLE == 0)
                d[k] = dh_out[(ob + t) * H + u];
            c[k + 1] = cst[(ob + t) * H + u];
        }
        // c_{tb-1} (c_{-1} = 0 is applied at the use: a select here would wait for the load)
        const int tp = tb > 0 ? (tb - 1 < S ? tb - 1 : S - 1) : 0;
        c[0] = cst[(ob + tp) * H + u];
    };
    f32x4 ax[MT];
    const int tl0 = ((S - 1) / TC) * TC;
    const int nch = tl0 / TC + 1;
    if (CH == 2 && ROLE == 0) chain_wait(flags + tile * nchk + (nch - 1), err);   // the last chunk's dh
    load_half(tl0 + 8, gA, cA, dA);
    float dc = 0.f;
    int cur = 0;
    for (int k = 0; k <= nch; ++k) {
        const int t0 = ROLE == 0 ? tl0 - TC * k : tl0 - TC * (k - 1);
        const bool act = t0 >= 0 && t0 <= tl0;   // block-uniform per role
        const int n = act ? (S - t0 < TC ? S - t0 : TC) : 0;
        const int xb = (t0 / TC) & 1;             // dX image of this chunk (U writes, L reads)
#pragma unroll
        for (int i = TC - 1; i >= 0; --i) {
            // unconditional (indices clamped; an idle period's values are never used)
            // the consumer leaves the chunk's flag zero for the next launch once every wave has
            // passed its wait (at i == 7 of the previous period, or before the loop: a barrier since)
            if (CH == 2 && ROLE == 0 && i == 14 && act && j == 0) atomicExch(flags + tile * nchk + t0 / TC, 0u);
            if (i == 15) load_half(t0, gB, cB, dB);
            if (i == 7) {
                if (CH == 2 && ROLE == 0 && act && t0 >= TC) chain_wait(flags + tile * nchk + t0 / TC - 1, err);
                load_half(t0 - 8, gA, cA, dA);
            }
            if (i < n) {
                const int t = t0 + i, k8 = i & 7;
                const float4 gq = i >= 8 ? gA[k8] : gB[k8];
                const float c1 = i >= 8 ? cA[k8 + 1] : cB[k8 + 1], c0 = t > 0 ? (i >= 8 ? cA[k8] : cB[k8]) : 0.f;
                const float dho = ROLE == 0 ? (i >= 8 ? dA[k8] : dB[k8]) : dximg[xb][sl][i][u];
                const __bf16* ap = (i + 1 < TC) ? &dgs[cur][i + 1][sa][8 * lg] : &dgs[cur ^ 1][0][sa][8 * lg];
                bf16x8 af[8];
#pragma unroll
                for (int ks = 0; ks < 8; ++ks) af[ks] = *reinterpret_cast<const bf16x8*>(ap + 32 * ks);
                f32x4 a0 = f32x4{0.f, 0.f, 0.f, 0.f}, a1 = a0;
#pragma unroll
                for (int ks = 0; ks < 8; ks += 2) {
                    a0 = mmab(af[ks], bw[ks], a0);
                    a1 = mmab(af[ks + 1], bw[ks + 1], a1);
                }
                __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
                const float dh = dho + (a0[0] + a1[0]);
                float v0, v1, v2, v3;
                cell_bwd16(dh, gq.x, gq.y, gq.z, gq.w, ftanh(c1), c0, dc, v0, v1, v2, v3);
                typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
                *reinterpret_cast<bf16x4*>(&dgs[cur][i][sl][4 * u]) = bf16x4{(__bf16)v0, (__bf16)v1, (__bf16)v2, (__bf16)v3};
                if (wr) {
                    float* o = dgates + (ob + t) * G4 + u;
                    o[0] = v0;
                    o[H] = v1;
                    o[2 * H] = v2;
                    o[3 * H] = v3;
                }
            }
            lds_barrier();
        }
        if (dxw) {   // an idle period's burst stores nothing (t >= S) or into an unread image
            bf16x8 bxw[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) bxw[q] = *reinterpret_cast<const bf16x8*>(&wT[col][32 * q + 8 * lg]);
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                ax[m] = f32x4{0.f, 0.f, 0.f, 0.f};
                const __bf16* ap = &dgs[cur][m * RPS + ln % RPS][ln / RPS][8 * lg];
#pragma unroll
                for (int q = 0; q < 8; ++q) ax[m] = mmab(*reinterpret_cast<const bf16x8*>(ap + 32 * q), bxw[q], ax[m]);
            }
#pragma unroll
            for (int m = 0; m < MT; ++m)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = 4 * lg + r, sr = row / RPS, tt = m * RPS + row % RPS, t = t0 + tt;
                    if (ROLE == 0) {
                        dximg[xb][sr][tt][col] = ax[m][r];
                    } else if (col < In) {
                        const int64_t b = b0 + sr < B ? b0 + sr : B - 1;
                        if (t < S) {
                            if (CH == 1) {
                                // (a bit_cast of the vector element itself stored element 0 for every r:
                                // clang / ROCm 7.2, seen in the ISA — the value goes through a scalar first)
                                const float v = ax[m][r];
                                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), drs,
                                                                      (int)(((b * S + t) * In + col) * 4), 0, CPOL_SC1);
                            }
                            else
                                dx[(b * S + t) * In + col] = ax[m][r];
                        }
                    }
                }
        }
        cur ^= 1;   // (both images start zero: L's first chunk may start on either)
        if (CH == 1 && ROLE == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the chunk's dX landed
        lds_barrier();
        if (CH == 1 && ROLE == 1 && act && j == 0) atomicAdd(flags + tile * nchk + t0 / TC, 1u);
    }
}

// dh_out [B, S, H] at layer l + 1's outputs; gatesU / cU from layer l + 1's forward, gatesL /
// cL from layer l's; W_hh / W_ih of both; dgU / dgL [B, S, 4H] fp32; dx [B, S, InL] (layer l's
// input gradient; may be null)
template <int NS, int NTXL>
__global__ __launch_bounds__(2 * G4) void k_lstm16_bwd2(const float* __restrict__ dh_out,
                                                        const float* __restrict__ gatesU, const float* __restrict__ cU,
                                                        const float* __restrict__ whhU, const float* __restrict__ wihU,
                                                        const float* __restrict__ gatesL, const float* __restrict__ cL,
                                                        const float* __restrict__ whhL, const float* __restrict__ wihL,
                                                        int InL, int B, int S, float* __restrict__ dgU,
                                                        float* __restrict__ dgL, float* __restrict__ dx) {
    __shared__ __attribute__((aligned(16))) __bf16 dgsU[2][TC][NS][DS];
    __shared__ __attribute__((aligned(16))) __bf16 dgsL[2][TC][NS][DS];
    __shared__ __attribute__((aligned(16))) float dximg[2][NS][TC][H];
    __shared__ __attribute__((aligned(16))) __bf16 wTU[H][DS];   // W_ih by column (k' = 4 u + g)
    __shared__ __attribute__((aligned(16))) __bf16 wTL[H][DS];
    for (int i = threadIdx.x; i < 2 * TC * NS * DS; i += 2 * G4) {
        (&dgsU[0][0][0][0])[i] = (__bf16)0.f;
        (&dgsL[0][0][0][0])[i] = (__bf16)0.f;
    }
    lds_barrier();
    if (threadIdx.x < G4)
        bwd2_role<NS, 4, 0>(dh_out, gatesU, cU, whhU, wihU, H, B, S, dgU, nullptr, dgsU, dximg, wTU);
    else
        bwd2_role<NS, NTXL, 1>(nullptr, gatesL, cL, whhL, wihL, InL, B, S, dgL, dx, dgsL, dximg, wTL);
}

// four layers' backward in one launch: workgroups [0, T) run layers 3, 2 of tile b (the producer:
// layer 2's dX, the gradient at layer 1's outputs, published chunk by chunk into dmid [B, S, H]),
// [T, 2T) layers 1, 0 of tile b - T (the consumer, reading dmid as each chunk's flag comes up).
// p: [w_ih, w_hh] x 4 layers; gc: [gates, c] x 4 layers; dg[4]: dgates of each layer; dx: layer
// 0's input gradient (may be null).  Per role the arithmetic of two k_lstm16_bwd2 launches.
struct QuadB {
    const float* w_ih[4];
    const float* w_hh[4];
    const float* gates[4];
    const float* c[4];
    float* dg[4];
};
template <int NS, int NTXL>
__global__ __launch_bounds__(2 * G4) void k_lstm16_bwd4(const float* __restrict__ dh_out, QuadB q, int In0, int B,
                                                        int S, int T, float* __restrict__ dmid, float* __restrict__ dx,
                                                        unsigned slot0) {
    unsigned* flags = g_chain_flags + slot0;
    unsigned* err = g_chain_err;
    __shared__ __attribute__((aligned(16))) __bf16 dgsU[2][TC][NS][DS];
    __shared__ __attribute__((aligned(16))) __bf16 dgsL[2][TC][NS][DS];
    __shared__ __attribute__((aligned(16))) float dximg[2][NS][TC][H];
    __shared__ __attribute__((aligned(16))) __bf16 wTU[H][DS];
    __shared__ __attribute__((aligned(16))) __bf16 wTL[H][DS];
    for (int i = threadIdx.x; i < 2 * TC * NS * DS; i += 2 * G4) {
        (&dgsU[0][0][0][0])[i] = (__bf16)0.f;
        (&dgsL[0][0][0][0])[i] = (__bf16)0.f;
    }
    lds_barrier();
    const bool cons = (int)blockIdx.x >= T;
    const int tile = cons ? (int)blockIdx.x - T : (int)blockIdx.x;
    if (!cons) {
        if (threadIdx.x < G4)
            bwd2_role<NS, 4, 0, 1>(dh_out, q.gates[3], q.c[3], q.w_hh[3], q.w_ih[3], H, B, S, q.dg[3], nullptr, dgsU,
                                   dximg, wTU, tile, flags, err);
        else
            bwd2_role<NS, 4, 1, 1>(nullptr, q.gates[2], q.c[2], q.w_hh[2], q.w_ih[2], H, B, S, q.dg[2], dmid, dgsL,
                                   dximg, wTL, tile, flags, err);
    } else {
        if (threadIdx.x < G4)
            bwd2_role<NS, 4, 0, 2>(dmid, q.gates[1], q.c[1], q.w_hh[1], q.w_ih[1], H, B, S, q.dg[1], nullptr, dgsU,
                                   dximg, wTU, tile, flags, err);
        else
            bwd2_role<NS, NTXL, 1, 2>(nullptr, q.gates[0], q.c[0], q.w_hh[0], q.w_ih[0], In0, B, S, q.dg[0], dx, dgsL,
                                      dximg, wTL, tile, flags, err);
    }
}

}  // namespace l16
}  // namespace vt

using namespace vt::l16;

namespace {

// samples per workgroup: VAETEB_L16_NS (2 or 4; default 2)
static int l16_ns() {
    static const int ns = getenv("VAETEB_L16_NS") ? atoi(getenv("VAETEB_L16_NS")) : 2;
    return ns == 4 ? 4 : 2;
}
// samples per workgroup of the layer-pair kernels: VAETEB_L16_PAIR_NS (2 or 4; default 2)
static int l16_pair_ns() {
    static const int ns = getenv("VAETEB_L16_PAIR_NS") ? atoi(getenv("VAETEB_L16_PAIR_NS")) : 2;
    return ns == 4 ? 4 : 2;
}
// timing probes only (outputs not valid): 1 no stores, 2 in-kernel stamps
static int l16_diag() {
    static const int d = getenv("VAETEB_L16_DIAG") ? atoi(getenv("VAETEB_L16_DIAG")) : 0;
    return d == 1 || d == 2 ? d : 0;
}

template <int NS, int KX>
static void fwd_launch(dim3 grid, hipStream_t st, const float* x, int In, const float* w_ih, const float* b_ih,
                       const float* w_hh, const float* b_hh, int B, int seq, float* h, float* hp, float* c,
                       float* gates) {
#define VT_L16F(HP_, D_) \
    hipLaunchKernelGGL((k_lstm16_fwd<NS, KX, HP_, D_>), grid, dim3(G4), 0, st, x, In, w_ih, b_ih, w_hh, b_hh, B, seq, \
                       h, hp, c, gates)
    switch (l16_diag()) {
        case 1: VT_L16F(false, 1); break;
        case 2: VT_L16F(true, 2); break;
        default:
            if (hp) VT_L16F(true, 0);
            else VT_L16F(false, 0);
    }
#undef VT_L16F
}

template <int NS, int NTX>
static void bwd_launch(dim3 grid, hipStream_t st, const float* dh_out, const float* gates, const float* cst,
                       const float* w_hh, const float* w_ih, int In, int B, int seq, float* dgates, float* dx) {
#define VT_L16B(W_, D_)                                                                                            \
    hipLaunchKernelGGL((k_lstm16_bwd<NS, NTX, W_, D_>), grid, dim3(G4), 0, st, dh_out, gates, cst, w_hh, w_ih, In, \
                       B, seq, dgates, dx)
    switch (l16_diag()) {
        case 1: VT_L16B(true, 1); break;
        case 2: VT_L16B(true, 2); break;
        default:
            if (dgates) VT_L16B(true, 0);
            else VT_L16B(false, 0);
    }
#undef VT_L16B
}

}  // namespace

extern "C" {

int vt_lstm16_layer_fwd(const float* x, int In, const float* w_ih, const float* b_ih, const float* w_hh,
                        const float* b_hh, int B, int seq, int hidden, float* out_h, float* out_hprev, float* out_c,
                        float* gates, void* stream) {
    VT_CHECK_ARG(hidden == H, "vt_lstm16_layer_fwd: hidden size %d (kernel built for %d)", hidden, H);
    VT_CHECK_ARG(B > 0 && seq > 0 && In > 0 && In <= 64 && In % 4 == 0,
                 "vt_lstm16_layer_fwd: shape (input size %d: a multiple of 4, at most 64)", In);
    VT_CHECK_ARG(x && w_ih && b_ih && w_hh && b_hh && out_h && out_c && gates, "vt_lstm16_layer_fwd: null pointer");
    VT_CHECK_ARG(l16_diag() != 2 || out_hprev, "vt_lstm16_layer_fwd: the stamp probe writes into out_hprev");
    const int ns = l16_ns();
    const dim3 grid((B + ns - 1) / ns);
    hipStream_t st = vt::S(stream);
    if (ns == 4) {
        if (In <= 32) fwd_launch<4, 1>(grid, st, x, In, w_ih, b_ih, w_hh, b_hh, B, seq, out_h, out_hprev, out_c, gates);
        else fwd_launch<4, 2>(grid, st, x, In, w_ih, b_ih, w_hh, b_hh, B, seq, out_h, out_hprev, out_c, gates);
    } else {
        if (In <= 32) fwd_launch<2, 1>(grid, st, x, In, w_ih, b_ih, w_hh, b_hh, B, seq, out_h, out_hprev, out_c, gates);
        else fwd_launch<2, 2>(grid, st, x, In, w_ih, b_ih, w_hh, b_hh, B, seq, out_h, out_hprev, out_c, gates);
    }
    VT_LAUNCH_CHECK("vt_lstm16_layer_fwd");
    return VT_OK;
}

int vt_lstm16_pair_fwd(const float* x, int In, const float* w_ih0, const float* b_ih0, const float* w_hh0,
                       const float* b_hh0, const float* w_ih1, const float* b_ih1, const float* w_hh1,
                       const float* b_hh1, int B, int seq, int hidden, float* h0, float* c0, float* gates0, float* h1,
                       float* c1, float* gates1, void* stream) {
    VT_CHECK_ARG(hidden == H, "vt_lstm16_pair_fwd: hidden size %d (kernel built for %d)", hidden, H);
    VT_CHECK_ARG(B > 0 && seq > 0 && In > 0 && In <= 64 && In % 4 == 0,
                 "vt_lstm16_pair_fwd: shape (input size %d: a multiple of 4, at most 64)", In);
    VT_CHECK_ARG(x && w_ih0 && b_ih0 && w_hh0 && b_hh0 && w_ih1 && b_ih1 && w_hh1 && b_hh1 && h0 && c0 && gates0 &&
                     h1 && c1 && gates1,
                 "vt_lstm16_pair_fwd: null pointer");
    const int ns = l16_pair_ns();
    const int64_t lds = fwd2_stage_bytes(ns, seq);
    VT_CHECK_ARG(lds <= L16_PAIR_STAGE_MAX, "vt_lstm16_pair_fwd: sequence length %d too long for the staged input", seq);
    const dim3 grid((B + ns - 1) / ns);
    hipStream_t st = vt::S(stream);
#define VT_L16F2(NS_, KX_)                                                                                          \
    hipLaunchKernelGGL((k_lstm16_fwd2<NS_, KX_>), grid, dim3(2 * G4), lds, st, x, In, w_ih0, b_ih0, w_hh0, b_hh0, \
                       w_ih1, b_ih1, w_hh1, b_hh1, B, seq, h0, c0, gates0, h1, c1, gates1)
    if (ns == 4) {
        if (In <= 32) VT_L16F2(4, 1);
        else VT_L16F2(4, 2);
    } else {
        if (In <= 32) VT_L16F2(2, 1);
        else VT_L16F2(2, 2);
    }
#undef VT_L16F2
    VT_LAUNCH_CHECK("vt_lstm16_pair_fwd");
    return VT_OK;
}

int vt_lstm16_pair_bwd(const float* dh_out, const float* gates1, const float* c1, const float* w_hh1,
                       const float* w_ih1, const float* gates0, const float* c0, const float* w_hh0,
                       const float* w_ih0, int In0, int B, int seq, int hidden, float* dgates1, float* dgates0,
                       float* dx, void* stream) {
    VT_CHECK_ARG(hidden == H, "vt_lstm16_pair_bwd: hidden size %d (kernel built for %d)", hidden, H);
    VT_CHECK_ARG(B > 0 && seq > 0 && In0 > 0 && In0 <= 64, "vt_lstm16_pair_bwd: shape (input size %d, at most 64)",
                 In0);
    VT_CHECK_ARG(dh_out && gates1 && c1 && w_hh1 && w_ih1 && gates0 && c0 && w_hh0 && (w_ih0 || !dx) && dgates1 &&
                     dgates0,
                 "vt_lstm16_pair_bwd: null pointer");
    const dim3 grid((B + 1) / 2);
    hipStream_t st = vt::S(stream);
    if (In0 <= 32)
        hipLaunchKernelGGL((k_lstm16_bwd2<2, 2>), grid, dim3(2 * G4), 0, st, dh_out, gates1, c1, w_hh1, w_ih1, gates0,
                           c0, w_hh0, w_ih0, In0, B, seq, dgates1, dgates0, dx);
    else
        hipLaunchKernelGGL((k_lstm16_bwd2<2, 4>), grid, dim3(2 * G4), 0, st, dh_out, gates1, c1, w_hh1, w_ih1, gates0,
                           c0, w_hh0, w_ih0, In0, B, seq, dgates1, dgates0, dx);
    VT_LAUNCH_CHECK("vt_lstm16_pair_bwd");
    return VT_OK;
}

// the chained launches need T (workgroups per pair) a multiple of 8 — tile b's producer and
// consumer then sit on the same XCD of the round-robin workgroup placement — and flags within the
// pool; otherwise (or VAETEB_L16_CHAIN=0) the two pair launches run one after the other (the same
// kernels' arithmetic: the same bits either way)
static bool l16_chain_ok(int T, int seq) {
    static const bool on = !getenv("VAETEB_L16_CHAIN") || atoi(getenv("VAETEB_L16_CHAIN")) != 0;
    return on && T % 8 == 0 && (int64_t)T * ((seq + TC - 1) / TC) <= (int64_t)vt::ARRIVE_POOL / 8;
}

int vt_lstm16_quad_fwd(const float* x, int In, const float* const* params, int B, int seq, int hidden,
                       float* const* outs, void* stream) {
    VT_CHECK_ARG(hidden == H, "vt_lstm16_quad_fwd: hidden size %d (kernel built for %d)", hidden, H);
    VT_CHECK_ARG(B > 0 && seq > 0 && In > 0 && In <= 64 && In % 4 == 0,
                 "vt_lstm16_quad_fwd: shape (input size %d: a multiple of 4, at most 64)", In);
    VT_CHECK_ARG(x && params && outs, "vt_lstm16_quad_fwd: null pointer");
    Quad q;
    for (int i = 0; i < 16; ++i) {
        VT_CHECK_ARG(params[i], "vt_lstm16_quad_fwd: null parameter %d", i);
        q.p[i] = params[i];
    }
    for (int i = 0; i < 12; ++i) {
        VT_CHECK_ARG(outs[i], "vt_lstm16_quad_fwd: null output %d", i);
        q.o[i] = outs[i];
    }
    const int ns = l16_pair_ns(), T = (B + ns - 1) / ns;
    const int64_t lds = fwd2_stage_bytes(ns, seq);
    VT_CHECK_ARG(lds <= L16_PAIR_STAGE_MAX, "vt_lstm16_quad_fwd: sequence length %d too long for the staged input", seq);
    if (!l16_chain_ok(T, seq)) {
        int rc = vt_lstm16_pair_fwd(x, In, q.p[0], q.p[2], q.p[1], q.p[3], q.p[4], q.p[6], q.p[5], q.p[7], B, seq, H,
                                    q.o[0], q.o[1], q.o[2], q.o[3], q.o[4], q.o[5], stream);
        if (rc) return rc;
        return vt_lstm16_pair_fwd(q.o[3], H, q.p[8], q.p[10], q.p[9], q.p[11], q.p[12], q.p[14], q.p[13], q.p[15], B,
                                  seq, H, q.o[6], q.o[7], q.o[8], q.o[9], q.o[10], q.o[11], stream);
    }
    hipStream_t st = vt::S(stream);
    const unsigned slot0 = vt::arrive_slots((unsigned)(T * ((seq + TC - 1) / TC)), st);
    const dim3 grid(2 * T);
#define VT_L16F4(NS_, KX_) \
    hipLaunchKernelGGL((k_lstm16_fwd4<NS_, KX_>), grid, dim3(2 * G4), lds, st, x, In, q, B, seq, T, slot0)
    if (ns == 4) {
        if (In <= 32) VT_L16F4(4, 1);
        else VT_L16F4(4, 2);
    } else {
        if (In <= 32) VT_L16F4(2, 1);
        else VT_L16F4(2, 2);
    }
#undef VT_L16F4
    VT_LAUNCH_CHECK("vt_lstm16_quad_fwd");
    return VT_OK;
}

int vt_lstm16_quad_bwd(const float* dh_out, const float* const* w, const float* const* gc, int In0, int B, int seq,
                       int hidden, float* const* dg, float* dmid, float* dx, void* stream) {
    VT_CHECK_ARG(hidden == H, "vt_lstm16_quad_bwd: hidden size %d (kernel built for %d)", hidden, H);
    VT_CHECK_ARG(B > 0 && seq > 0 && In0 > 0 && In0 <= 64, "vt_lstm16_quad_bwd: shape (input size %d, at most 64)",
                 In0);
    VT_CHECK_ARG(dh_out && w && gc && dg && dmid, "vt_lstm16_quad_bwd: null pointer");
    QuadB q;
    for (int l = 0; l < 4; ++l) {
        q.w_ih[l] = w[2 * l];
        q.w_hh[l] = w[2 * l + 1];
        q.gates[l] = gc[2 * l];
        q.c[l] = gc[2 * l + 1];
        q.dg[l] = dg[l];
        VT_CHECK_ARG(q.w_hh[l] && q.gates[l] && q.c[l] && q.dg[l] && (q.w_ih[l] || (l == 0 && !dx)),
                     "vt_lstm16_quad_bwd: null pointer (layer %d)", l);
    }
    const int T = (B + 1) / 2;
    if (!l16_chain_ok(T, seq)) {
        int rc = vt_lstm16_pair_bwd(dh_out, q.gates[3], q.c[3], q.w_hh[3], q.w_ih[3], q.gates[2], q.c[2], q.w_hh[2],
                                    q.w_ih[2], H, B, seq, H, q.dg[3], q.dg[2], dmid, stream);
        if (rc) return rc;
        return vt_lstm16_pair_bwd(dmid, q.gates[1], q.c[1], q.w_hh[1], q.w_ih[1], q.gates[0], q.c[0], q.w_hh[0],
                                  q.w_ih[0], In0, B, seq, H, q.dg[1], q.dg[0], dx, stream);
    }
    hipStream_t st = vt::S(stream);
    const unsigned slot0 = vt::arrive_slots((unsigned)(T * ((seq + TC - 1) / TC)), st);
    if (In0 <= 32)
        hipLaunchKernelGGL((k_lstm16_bwd4<2, 2>), dim3(2 * T), dim3(2 * G4), 0, st, dh_out, q, In0, B, seq, T, dmid,
                           dx, slot0);
    else
        hipLaunchKernelGGL((k_lstm16_bwd4<2, 4>), dim3(2 * T), dim3(2 * G4), 0, st, dh_out, q, In0, B, seq, T, dmid,
                           dx, slot0);
    VT_LAUNCH_CHECK("vt_lstm16_quad_bwd");
    return VT_OK;
}

int vt_lstm16_chain_errors(int* count, int reset) {
    VT_CHECK_ARG(count, "vt_lstm16_chain_errors: null pointer");
    unsigned v = 0;
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_chain_err), sizeof(v)) != hipSuccess) return VT_ERR_HIP;
    *count = (int)v;
    if (reset) {
        v = 0;
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_chain_err), &v, sizeof(v)) != hipSuccess) return VT_ERR_HIP;
    }
    return VT_OK;
}

int vt_lstm16_layer_bwd(const float* dh_out, const float* gates, const float* cst, const float* w_hh,
                        const float* w_ih, int In, int B, int seq, int hidden, float* dgates, float* dx,
                        void* stream) {
    VT_CHECK_ARG(hidden == H, "vt_lstm16_layer_bwd: hidden size %d (kernel built for %d)", hidden, H);
    VT_CHECK_ARG(B > 0 && seq > 0 && In > 0 && In <= 64, "vt_lstm16_layer_bwd: shape (input size %d, at most 64)",
                 In);
    VT_CHECK_ARG(dh_out && gates && cst && w_hh && (w_ih || !dx), "vt_lstm16_layer_bwd: null pointer");
    VT_CHECK_ARG(l16_diag() != 2 || dx, "vt_lstm16_layer_bwd: the stamp probe writes into dx");
    const int ns = l16_ns();
    const dim3 grid((B + ns - 1) / ns);
    hipStream_t st = vt::S(stream);
    // column tiles of dX: 2 cover In <= 32 (the encoders' first layers: 20 / 32), 4 the rest
    if (ns == 4) {
        if (In <= 32) bwd_launch<4, 2>(grid, st, dh_out, gates, cst, w_hh, w_ih, In, B, seq, dgates, dx);
        else bwd_launch<4, 4>(grid, st, dh_out, gates, cst, w_hh, w_ih, In, B, seq, dgates, dx);
    } else {
        if (In <= 32) bwd_launch<2, 2>(grid, st, dh_out, gates, cst, w_hh, w_ih, In, B, seq, dgates, dx);
        else bwd_launch<2, 4>(grid, st, dh_out, gates, cst, w_hh, w_ih, In, B, seq, dgates, dx);
    }
    VT_LAUNCH_CHECK("vt_lstm16_layer_bwd");
    return VT_OK;
}

}  // extern "C"
