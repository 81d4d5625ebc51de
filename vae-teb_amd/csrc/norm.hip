// Normalisation + activation kernels on (rows, C) row-major activations.
//
// LayerNorm (+ activation) fused: every ResidualMLP layer is Linear -> LN ->
// act (ref/model/vae_teb_model.py:336-403), the encoders' fused/lstm norms and
// the decoder heads' LN(4096) (:882-896).  One wave per row, two-pass mean /
// variance in registers, affine + activation in the same pass; the backward
// recomputes z = xhat*gamma + beta for the activation derivative and keeps
// the gamma/beta column sums in registers per wave (no atomics, fixed order).
//
// BatchNorm1d in training mode (batch statistics over B*L per channel,
// momentum 0.9, eps 1e-5) + ReLU/tanh for the conv blocks
// (ref/model/vae_teb_model.py:175, :206-210, :230, :252-253).
#include <math.h>
#include <stdlib.h>

#include "bnbwd.h"
#include "common.h"
#include "dropout.h"

namespace vt {

enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2, ACT_TANH = 3 };

__device__ __forceinline__ float act_f(float z, int act) {
    switch (act) {
        case ACT_RELU: return z > 0.f ? z : 0.f;
        case ACT_GELU: return 0.5f * z * (1.f + erff(z * 0.70710678118654752f));
        case ACT_TANH: return tanhf(z);
        default: return z;
    }
}
// d act / dz
__device__ __forceinline__ float act_d(float z, int act) {
    switch (act) {
        case ACT_RELU: return z > 0.f ? 1.f : 0.f;
        case ACT_GELU: {
            const float cdf = 0.5f * (1.f + erff(z * 0.70710678118654752f));
            const float pdf = 0.39894228040143268f * expf(-0.5f * z * z);
            return cdf + z * pdf;
        }
        case ACT_TANH: {
            const float t = tanhf(z);
            return 1.f - t * t;
        }
        default: return 1.f;
    }
}

static constexpr int NT = 256;  // 4 waves

// ------------------------------------------------------------- LayerNorm fwd
__global__ __launch_bounds__(NT) void k_ln_fwd(const float* __restrict__ x, int64_t R, int C,
                                               const float* __restrict__ gamma, const float* __restrict__ beta,
                                               int act, float eps, float* __restrict__ y, float* __restrict__ xhat,
                                               float* __restrict__ rstd_out) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
    if (row >= R) return;
    const float* xr = x + row * C;
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s += xr[c];
    const float mean = wave_sum(s) / (float)C;
    float v = 0.f;
    for (int c = lane; c < C; c += 64) {
        const float d = xr[c] - mean;
        v += d * d;
    }
    const float rstd = rsqrtf(wave_sum(v) / (float)C + eps);
    float* yr = y + row * C;
    float* hr = xhat ? xhat + row * C : nullptr;
    for (int c = lane; c < C; c += 64) {
        const float h = (xr[c] - mean) * rstd;
        if (hr) hr[c] = h;
        yr[c] = act_f(h * gamma[c] + beta[c], act);
    }
    if (lane == 0 && rstd_out) rstd_out[row] = rstd;
}

// Wide rows (C >= 1024, the decoder heads' 4096): one workgroup per row, the row
// held in registers (V4 float4 per thread, one HBM read), block reductions via
// LDS — the wave-per-row kernel above ran 3 dependent 64-step loops per wave on
// only R/4 workgroups (74 us for 256 x 4096).
template <int V4>
__global__ __launch_bounds__(NT) void k_ln_fwd_wide(const float* __restrict__ x, int C, const float* __restrict__ gamma,
                                                    const float* __restrict__ beta, int act, float eps,
                                                    float* __restrict__ y, float* __restrict__ xhat,
                                                    float* __restrict__ rstd_out) {
    __shared__ float red[16];
    const int64_t row = blockIdx.x;
    const float4* xr = reinterpret_cast<const float4*>(x + row * C);
    const int C4 = C >> 2;
    float4 v[V4];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < V4; ++j) {
        const int c4 = threadIdx.x + NT * j;
        v[j] = c4 < C4 ? xr[c4] : make_float4(0.f, 0.f, 0.f, 0.f);
        s += (v[j].x + v[j].y) + (v[j].z + v[j].w);
    }
    const float mean = block_sum(s, red) / (float)C;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < V4; ++j) {
        const int c4 = threadIdx.x + NT * j;
        if (c4 < C4) {
            const float a = v[j].x - mean, b = v[j].y - mean, c = v[j].z - mean, d = v[j].w - mean;
            q += (a * a + b * b) + (c * c + d * d);
        }
    }
    const float rstd = rsqrtf(block_sum(q, red) / (float)C + eps);
    const float4* g4 = reinterpret_cast<const float4*>(gamma);
    const float4* b4 = reinterpret_cast<const float4*>(beta);
    float4* yr = reinterpret_cast<float4*>(y + row * C);
    float4* hr = xhat ? reinterpret_cast<float4*>(xhat + row * C) : nullptr;
#pragma unroll
    for (int j = 0; j < V4; ++j) {
        const int c4 = threadIdx.x + NT * j;
        if (c4 >= C4) continue;
        const float4 h = make_float4((v[j].x - mean) * rstd, (v[j].y - mean) * rstd, (v[j].z - mean) * rstd,
                                     (v[j].w - mean) * rstd);
        if (hr) hr[c4] = h;
        const float4 g = g4[c4], bb = b4[c4];
        yr[c4] = make_float4(act_f(h.x * g.x + bb.x, act), act_f(h.y * g.y + bb.y, act), act_f(h.z * g.z + bb.z, act),
                             act_f(h.w * g.w + bb.w, act));
    }
    if (threadIdx.x == 0 && rstd_out) rstd_out[row] = rstd;
}

// ------------------------------------------------------------- LayerNorm bwd
// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dy * act'(z) * gamma.
// gamma/beta column partials per block: part[block][0:C] = sum dz*xhat,
// part[block][C:2C] = sum dz.  Small-C path (C <= 512): per-lane registers.
template <int CPL>  // columns per lane (C <= 64*CPL)
__global__ __launch_bounds__(NT) void k_ln_bwd(const float* __restrict__ dy, const float* __restrict__ xhat,
                                               const float* __restrict__ rstd, int64_t R, int C,
                                               const float* __restrict__ gamma, const float* __restrict__ beta,
                                               int act, int64_t rows_per_block, float* __restrict__ dx,
                                               float* __restrict__ part) {
    __shared__ float red[NT / 64][2][64 * CPL];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float dg[CPL], db[CPL];
#pragma unroll
    for (int j = 0; j < CPL; ++j) dg[j] = db[j] = 0.f;
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = r0 + rows_per_block < R ? r0 + rows_per_block : R;
    for (int64_t row = r0 + w; row < r1; row += NT / 64) {
        const float* dyr = dy + row * C;
        const float* hr = xhat + row * C;
        float gv[CPL], hv[CPL];
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int j = 0; j < CPL; ++j) {
            const int c = lane + 64 * j;
            gv[j] = 0.f;
            hv[j] = 0.f;
            if (c < C) {
                const float h = hr[c];
                const float dz = dyr[c] * act_d(h * gamma[c] + beta[c], act);
                dg[j] += dz * h;
                db[j] += dz;
                gv[j] = dz * gamma[c];
                hv[j] = h;
                s1 += gv[j];
                s2 += gv[j] * h;
            }
        }
        const float m1 = wave_sum(s1) / (float)C, m2 = wave_sum(s2) / (float)C;
        const float rs = rstd[row];
        float* dxr = dx + row * C;
#pragma unroll
        for (int j = 0; j < CPL; ++j) {
            const int c = lane + 64 * j;
            if (c < C) dxr[c] = rs * (gv[j] - m1 - hv[j] * m2);
        }
    }
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
        red[w][0][lane + 64 * j] = dg[j];
        red[w][1][lane + 64 * j] = db[j];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += NT) {
        float a = 0.f, b = 0.f;
#pragma unroll
        for (int i = 0; i < NT / 64; ++i) {
            a += red[i][0][c];
            b += red[i][1][c];
        }
        part[(int64_t)blockIdx.x * 2 * C + c] = a;
        part[(int64_t)blockIdx.x * 2 * C + C + c] = b;
    }
}

// Large-C path (C > 512, few rows, e.g. the LN(4096) of the decoder heads):
// one block per row; per-row (dz*xhat, dz) written to scratch and reduced by
// k_rows_to_cols afterwards.
__global__ __launch_bounds__(NT) void k_ln_bwd_wide(const float* __restrict__ dy, const float* __restrict__ xhat,
                                                    const float* __restrict__ rstd, int C,
                                                    const float* __restrict__ gamma, const float* __restrict__ beta,
                                                    int act, float* __restrict__ dx, float* __restrict__ rowpart) {
    __shared__ float red[16];
    const int64_t row = blockIdx.x;
    const float* dyr = dy + row * C;
    const float* hr = xhat + row * C;
    float s1 = 0.f, s2 = 0.f;
    for (int c = threadIdx.x; c < C; c += NT) {
        const float h = hr[c];
        const float dz = dyr[c] * act_d(h * gamma[c] + beta[c], act);
        const float g = dz * gamma[c];
        s1 += g;
        s2 += g * h;
        rowpart[row * 2 * C + c] = dz * h;
        rowpart[row * 2 * C + C + c] = dz;
    }
    const float m1 = block_sum(s1, red) / (float)C;
    const float m2 = block_sum(s2, red) / (float)C;
    const float rs = rstd[row];
    for (int c = threadIdx.x; c < C; c += NT) {
        const float h = hr[c];
        const float dz = dyr[c] * act_d(h * gamma[c] + beta[c], act);
        dx[row * C + c] = rs * (dz * gamma[c] - m1 - h * m2);
    }
}

// ---------------------------------------------- narrow LayerNorm (C <= 256)
// 16 lanes per row (4 rows per wave, 16 per workgroup), lane l owns columns
// l&15 + 16 j: the 64-wide ResidualMLP rows of 256 B are covered by one
// instruction for 4 rows at once instead of a whole wave per row.
// butterfly sum over a row's 16 lanes, v + lane (l ^ m) for m = 1, 2, 4, 8 — the same
// values as the __shfl_xor(., m, 16) chain, with DPP moves instead of ds_bpermute.
// xor 4: the row rotated by 4 and by 12, both moved with every lane active (a DPP
// under a divergent branch would read inactive source lanes), then selected by lane bit 2
// (bit 2 clear: lane l + 4 = rotation by 12; set: lane l - 4 = rotation by 4).
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float sum16(float v) {
    v += dppf<0xB1>(v);                        // quad_perm [1,0,3,2]: l ^ 1
    v += dppf<0x4E>(v);                        // quad_perm [2,3,0,1]: l ^ 2
    const float r4 = dppf<0x124>(v), r12 = dppf<0x12C>(v);
    v += (threadIdx.x & 4) ? r4 : r12;         // row_ror:N reads lane (l - N) mod 16: l ^ 4
    v += dppf<0x128>(v);                       // row_ror 8: l ^ 8
    return v;
}

template <int CPL>  // columns per lane, C <= 16 * CPL
__global__ __launch_bounds__(NT) void k_ln_fwd16(const float* __restrict__ x, int64_t R, int C,
                                                 const float* __restrict__ gamma, const float* __restrict__ beta,
                                                 int act, float eps, float* __restrict__ y, float* __restrict__ xhat,
                                                 float* __restrict__ rstd_out) {
    const int lr = threadIdx.x & 15;
    const int64_t row = (int64_t)blockIdx.x * (NT / 16) + (threadIdx.x >> 4);
    const bool ok = row < R;
    const float* xr = x + (ok ? row : 0) * C;
    float v[CPL], s = 0.f;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
        const int c = lr + 16 * j;
        v[j] = (ok && c < C) ? xr[c] : 0.f;
        s += v[j];
    }
    const float mean = sum16(s) / (float)C;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
        const int c = lr + 16 * j;
        const float d = c < C ? v[j] - mean : 0.f;
        q += d * d;
    }
    const float rstd = rsqrtf(sum16(q) / (float)C + eps);
    if (!ok) return;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
        const int c = lr + 16 * j;
        if (c >= C) continue;
        const float h = (v[j] - mean) * rstd;
        if (xhat) xhat[row * C + c] = h;
        y[row * C + c] = act_f(h * gamma[c] + beta[c], act);
    }
    if (lr == 0 && rstd_out) rstd_out[row] = rstd;
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dy * act'(z) * gamma;
// part[block][0:C] = sum dz*xhat, part[block][C:2C] = sum dz over the block's rows.
template <int CPL>
__global__ __launch_bounds__(NT) void k_ln_bwd16(const float* __restrict__ dy, const float* __restrict__ xhat,
                                                 const float* __restrict__ rstd, int64_t R, int C,
                                                 const float* __restrict__ gamma, const float* __restrict__ beta,
                                                 int act, int64_t rows_per_block, float* __restrict__ dx,
                                                 float* __restrict__ part) {
    __shared__ float red[NT / 64][2][16 * CPL];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lr = lane & 15, grp = threadIdx.x >> 4;
    float gam[CPL], bet[CPL], dg[CPL], db[CPL];
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
        const int c = lr + 16 * j;
        gam[j] = c < C ? gamma[c] : 0.f;
        bet[j] = c < C ? beta[c] : 0.f;
        dg[j] = db[j] = 0.f;
    }
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = r0 + rows_per_block < R ? r0 + rows_per_block : R;
    for (int64_t rb = r0; rb < r1; rb += NT / 16) {
        const int64_t row = rb + grp;
        const bool ok = row < r1;
        const float* dyr = dy + (ok ? row : 0) * C;
        const float* hr = xhat + (ok ? row : 0) * C;
        float gv[CPL], hv[CPL], s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int j = 0; j < CPL; ++j) {
            const int c = lr + 16 * j;
            gv[j] = hv[j] = 0.f;
            if (ok && c < C) {
                const float h = hr[c];
                const float dz = dyr[c] * act_d(h * gam[j] + bet[j], act);
                dg[j] += dz * h;
                db[j] += dz;
                gv[j] = dz * gam[j];
                hv[j] = h;
                s1 += gv[j];
                s2 += gv[j] * h;
            }
        }
        const float m1 = sum16(s1) / (float)C, m2 = sum16(s2) / (float)C;
        if (!ok) continue;
        const float rs = rstd[row];
        float* dxr = dx + row * C;
#pragma unroll
        for (int j = 0; j < CPL; ++j) {
            const int c = lr + 16 * j;
            if (c < C) dxr[c] = rs * (gv[j] - m1 - hv[j] * m2);
        }
    }
    // column partials: the 4 row groups of a wave (lanes l, l^16, l^32), then the 4 waves
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
        dg[j] += __shfl_xor(dg[j], 16);
        dg[j] += __shfl_xor(dg[j], 32);
        db[j] += __shfl_xor(db[j], 16);
        db[j] += __shfl_xor(db[j], 32);
        if (lane < 16) {
            red[w][0][lr + 16 * j] = dg[j];
            red[w][1][lr + 16 * j] = db[j];
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += NT) {
        part[(int64_t)blockIdx.x * 2 * C + c] = (red[0][0][c] + red[1][0][c]) + (red[2][0][c] + red[3][0][c]);
        part[(int64_t)blockIdx.x * 2 * C + C + c] = (red[0][1][c] + red[1][1][c]) + (red[2][1][c] + red[3][1][c]);
    }
}

// out0[c] / out1[c - split] (+)= sum_b part[b][c], c < n.  A workgroup owns 16 columns; thread
// (l0, cc) forms the lane partials s_l = sum_k part[l + 64 k][c0 + cc], l = l0 + 16 q, k in order
// (16 adjacent columns of a partial row are one 64-B segment — a wave per column striding the
// rows with its lanes read 4 B per row, up to 132 us per launch at 2 C = 512), then a wave per
// column applies wave_sum's shuffle tree to the 64 s_l (round 5: the same bits as before)
constexpr int CR_C = 16;
__global__ __launch_bounds__(NT) void k_colred16(const float* __restrict__ part, int blocks, int n,
                                                  float* __restrict__ out0, float* __restrict__ out1, int split,
                                                  int accumulate) {
    static_assert(NT == 256, "16 columns x 16 lane groups");
    __shared__ float sl[CR_C][64 + 1];
    const int c0 = blockIdx.x * CR_C, cc = threadIdx.x & (CR_C - 1), l0 = threadIdx.x >> 4;
    const int c = c0 + cc;
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    if (c < n) {
        int k = 0;
        for (; 64 * (k + 4) <= blocks; k += 4) {   // 16 loads in flight, each a[q] in row order
            float v[4][4];
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                for (int q = 0; q < 4; ++q) v[kk][q] = part[(int64_t)(l0 + 16 * q + 64 * (k + kk)) * n + c];
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                for (int q = 0; q < 4; ++q) a[q] += v[kk][q];
        }
        for (; 64 * k < blocks; ++k) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int b = l0 + 16 * q + 64 * k;
                if (b < blocks) a[q] += part[(int64_t)b * n + c];
            }
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) sl[cc][l0 + 16 * q] = a[q];
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int j = w; j < CR_C; j += NT / 64) {
        if (c0 + j >= n) break;
        const float v = wave_sum(sl[j][lane]);
        if (lane == 0) {
            float* dst = c0 + j < split ? out0 + c0 + j : out1 + (c0 + j - split);
            *dst = accumulate ? *dst + v : v;
        }
    }
}

// out[c] (+)= sum_b part[b][c] for c < n: one workgroup per column, threads
// stride over the partials, fixed-order tree -> deterministic.
__global__ __launch_bounds__(NT) void k_reduce_parts(const float* __restrict__ part, int blocks, int n,
                                                     float* __restrict__ out0, float* __restrict__ out1, int split,
                                                     int accumulate) {
    __shared__ float red[16];
    const int c = blockIdx.x;
    float a = 0.f;
#pragma unroll 8
    for (int b = threadIdx.x; b < blocks; b += NT) a += part[(int64_t)b * n + c];   // 8 loads in flight, same order
    a = block_sum(a, red);
    if (threadIdx.x == 0) {
        float* o = c < split ? out0 + c : out1 + (c - split);
        *o = accumulate ? *o + a : a;
    }
}

// ------------------------------------------------------------- BatchNorm
// mode 0: mean[c] = S/M.  mode 1: var = S/M -> rstd, running stats update.
// mode 2: dbeta = S0, dgamma = S1 (+ the packed coefficients of vt_batchnorm_bwd_coef).
struct BnFin {
    int mode;   // < 0: the column-partial kernel only writes its partials (a separate finaliser)
    int64_t M;
    float eps, momentum;
    float *mean, *rstd, *run_mean, *run_var, *dgamma, *dbeta;
    int accumulate;
    float* bnp;
    const float *gamma, *beta;
    float *pg, *pb;
    int pacc;
    double* gpart;    // in-kernel finalize: the group sums ([2C][groups] doubles)
    unsigned slot0;   // its arrival counters (groups + 1)
};

__device__ __forceinline__ void bn_fin_channel(int c, int C, double s0, double s1, const BnFin& f) {
    const int64_t M = f.M;
    if (f.mode == 0) {
        f.mean[c] = (float)(s0 / (double)M);
    } else if (f.mode == 1) {
        const double var = s0 / (double)M;
        f.rstd[c] = (float)(1.0 / sqrt(var + (double)f.eps));
        if (f.run_mean) {
            const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
            f.run_mean[c] = (float)((1.0 - f.momentum) * f.run_mean[c] + f.momentum * f.mean[c]);
            f.run_var[c] = (float)((1.0 - f.momentum) * f.run_var[c] + f.momentum * unb);
        }
    } else {
        f.dbeta[c] = f.accumulate ? f.dbeta[c] + (float)s0 : (float)s0;
        f.dgamma[c] = f.accumulate ? f.dgamma[c] + (float)s1 : (float)s1;
        if (f.bnp) {   // vt_batchnorm_bwd_coef: the packed parameters
            f.bnp[c] = f.mean[c];
            f.bnp[C + c] = f.rstd[c];
            f.bnp[2 * C + c] = f.gamma[c];
            f.bnp[3 * C + c] = f.beta[c];
        }
        if (f.pg) {    // the parameter gradients (+)= the same float sums (no separate pass)
            f.pb[c] = f.pacc ? f.pb[c] + (float)s0 : (float)s0;
            f.pg[c] = f.pacc ? f.pg[c] + (float)s1 : (float)s1;
        }
    }
}

// The separate finaliser (channels > 128: past the in-kernel finalize's one thread per sum):
// one workgroup per channel; double accumulation, fixed-order tree.  part is channel-major
// ([2][C][blocks], k_col_partial4): thread t sums blocks t, t + NT, ... in that order with
// eight coalesced loads in flight.
__global__ __launch_bounds__(NT) void k_bn_finalize(const float* __restrict__ part, int blocks, int C, BnFin f) {
    __shared__ double r0[NT], r1[NT];
    const int c = blockIdx.x;
    double a0 = 0.0, a1 = 0.0;
    const float* p0 = part + (int64_t)c * blocks;
    const float* p1 = part + (int64_t)(C + c) * blocks;
    int b = threadIdx.x;
    for (; b + 7 * NT < blocks; b += 8 * NT) {
        float u[8], v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            u[k] = p0[b + k * NT];
            v[k] = p1[b + k * NT];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            a0 += (double)u[k];
            a1 += (double)v[k];
        }
    }
    for (; b < blocks; b += NT) {
        a0 += (double)p0[b];
        a1 += (double)p1[b];
    }
    static_assert(NT == 256, "k_bn_finalize: 256-thread tree");
    const int t = threadIdx.x;
    r0[t] = a0;
    r1[t] = a1;
    __syncthreads();
    if (t < 128) {
        r0[t] += r0[t + 128];
        r1[t] += r1[t + 128];
    }
    __syncthreads();
    if (t >= 64) return;
    double x0 = r0[t] + r0[t + 64], x1 = r1[t] + r1[t + 64];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        x0 += __shfl_down(x0, o);
        x1 += __shfl_down(x1, o);
    }
    if (t == 0) bn_fin_channel(c, C, x0, x1, f);
}

// In-kernel finalize of the column partials (round 5; replaces the k_bn_finalize launch for
// C <= 128): blocks form groups of BN_GB; the last-arriving block of a group sums its
// group's partials per (kind, channel) in block order, in double; the last group to finish
// sums the group sums in group order and applies bn_fin_channel.  Fixed order throughout.
constexpr int BN_GB = 64;
VT_ARRIVE_POOL(g_arrive_bn);
static int g_bn_fold = getenv("VAETEB_BN_FOLD") ? atoi(getenv("VAETEB_BN_FOLD")) : 1;
static int g_bn_fold_blocks = getenv("VAETEB_BN_BLOCKS") ? atoi(getenv("VAETEB_BN_BLOCKS")) : 512;
#define BN_FOLD_BLOCKS ((int64_t)(g_bn_fold_blocks > 0 && g_bn_fold_blocks <= 2048 ? g_bn_fold_blocks : 512))

__device__ __forceinline__ int bn_groups(int blocks) { return (blocks + BN_GB - 1) / BN_GB; }

__device__ void bn_fold_finalize(const float* part, int C, const BnFin& f) {
    __shared__ double fin[2 * 128];
    const int blocks = gridDim.x, ng = bn_groups(blocks), g = blockIdx.x / BN_GB;
    const int members = blocks - g * BN_GB < BN_GB ? blocks - g * BN_GB : BN_GB;
    if (!last_arrival(&g_arrive_bn[f.slot0 + g], (unsigned)members)) return;
    const int tid = threadIdx.x;
    const __amdgpu_buffer_rsrc_t pr = agent_rsrc(part, (int64_t)2 * C * blocks * 4);
    const __amdgpu_buffer_rsrc_t gr = agent_rsrc(f.gpart, (int64_t)2 * C * ng * 8);
    if (tid < 2 * C) {
        const int b0 = g * BN_GB;
        float v[BN_GB];
#pragma unroll
        for (int u = 0; u < BN_GB; ++u)
            v[u] = ld_agent(pr, u < members ? (unsigned)(((int64_t)tid * blocks + b0 + u) * 4) : 0x80000000u);
        double a = 0.0;
#pragma unroll
        for (int u = 0; u < BN_GB; ++u) a += (double)v[u];
        st_agent(gr, (unsigned)(((int64_t)tid * ng + g) * 8), a);
    }
    if (!last_arrival(&g_arrive_bn[f.slot0 + ng], (unsigned)ng)) return;
    if (tid < 2 * C) {
        constexpr int GMAX = 2048 / BN_GB;
        double v[GMAX];
#pragma unroll
        for (int q = 0; q < GMAX; ++q)
            v[q] = ld_agent_d(gr, q < ng ? (unsigned)(((int64_t)tid * ng + q) * 8) : 0x80000000u);
        double a = 0.0;
#pragma unroll
        for (int q = 0; q < GMAX; ++q) a += v[q];
        fin[tid] = a;
    }
    __syncthreads();
    if (tid < C) bn_fin_channel(tid, C, fin[tid], fin[C + tid], f);
}

__global__ void k_bn_apply(const float* __restrict__ x, int64_t M, int C, const float* __restrict__ mean,
                           const float* __restrict__ rstd, const float* __restrict__ gamma,
                           const float* __restrict__ beta, int act, float* __restrict__ y) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M * C) return;
    const int c = (int)(i % C);
    y[i] = bn_fwd_val(x[i], mean[c], rstd[c], gamma[c], beta[c], act);
}

// eval-mode BatchNorm: running statistics
__global__ void k_bn_eval(const float* __restrict__ x, int64_t M, int C, const float* __restrict__ run_mean,
                          const float* __restrict__ run_var, float eps, const float* __restrict__ gamma,
                          const float* __restrict__ beta, int act, float* __restrict__ y) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M * C) return;
    const int c = (int)(i % C);
    y[i] = act_f((x[i] - run_mean[c]) * (1.f / sqrtf(run_var[c] + eps)) * gamma[c] + beta[c], act);
}

__global__ void k_act_fwd(const float* __restrict__ x, int64_t n, int act, float* __restrict__ y) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = act_f(x[i], act);
}
__global__ void k_act_bwd(const float* __restrict__ dy, const float* __restrict__ x, int64_t n, int act,
                          float* __restrict__ dx) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dx[i] = dy[i] * act_d(x[i], act);
}

// ---------------------------------------------- BatchNorm, vectorised paths
// The element-wise BatchNorm passes over the conv blocks' (B*L, C) activations
// (C = 1..87 channels, up to 23 M elements) are HBM streams: 16-byte loads and
// stores, four elements per thread-step, the per-channel parameters staged once
// per workgroup in LDS, the activation a template parameter, 32-bit channel
// arithmetic (the flat index's channel advances by a fixed step per thread-step
// instead of a 64-bit modulo per element).
//   apply: y = act((x - mean) rstd gamma + beta)
//   dx:    dx = gamma rstd (dz - dbeta/M - xhat dgamma/M), dz = dy act'(xhat gamma + beta)
//   column partials, kind 0: x; 1: (x - mean)^2; 2: (dz, dz xhat)
static constexpr int BNV_C = 1024;  // max channels of the vectorised paths (LDS staging)
static constexpr int BNV_V = 4;     // float4 per thread per workgroup

__device__ __forceinline__ int wrapc(int c, int C) { return c >= C ? c - C : c; }

// channels of the 4 elements starting at channel c (C >= 4: one wrap at most)
__device__ __forceinline__ void chan4(int c, int C, int (&ce)[4]) {
    if (C >= 4) {
        ce[0] = c;
        ce[1] = wrapc(c + 1, C);
        ce[2] = wrapc(ce[1] + 1, C);
        ce[3] = wrapc(ce[2] + 1, C);
    } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) ce[e] = (c + e) % C;
    }
}

template <int ACT>
__global__ __launch_bounds__(NT) void k_bn_apply4(const float* __restrict__ x, int64_t n, int C,
                                                  const float* __restrict__ mean, const float* __restrict__ rstd,
                                                  const float* __restrict__ gamma, const float* __restrict__ beta,
                                                  float* __restrict__ y) {
    __shared__ float4 p[BNV_C];   // (mean, rstd, gamma, beta) per channel
    for (int c = threadIdx.x; c < C; c += NT) p[c] = make_float4(mean[c], rstd[c], gamma[c], beta[c]);
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * (NT * 4 * BNV_V);
    const int step = (NT * 4) % C;
    int c = (int)((base + 4 * threadIdx.x) % C);
#pragma unroll
    for (int v = 0; v < BNV_V; ++v, c = wrapc(c + step, C)) {
        const int64_t j = base + 4 * (threadIdx.x + NT * v);
        if (j >= n) break;
        int ce[4];
        chan4(c, C, ce);
        if (j + 4 <= n) {
            const float4 xv = *(const float4*)(x + j);
            const float xs[4] = {xv.x, xv.y, xv.z, xv.w};
            float o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float4 q = p[ce[e]];
                o[e] = bn_fwd_val(xs[e], q.x, q.y, q.z, q.w, ACT);
            }
            *(float4*)(y + j) = make_float4(o[0], o[1], o[2], o[3]);
        } else {
            for (int e = 0; e < (int)(n - j); ++e) {
                const float4 q = p[ce[e]];
                y[j + e] = bn_fwd_val(x[j + e], q.x, q.y, q.z, q.w, ACT);
            }
        }
    }
}

// Dropout1d of the BatchNorm backward's incoming gradient (vt_batchnorm_bwd_dropout): the
// kernels read dy through dmask, i.e. the value cls.hip's k_dropout would have written
struct DropArg {
    int L;
    float p;
    uint64_t seed;                // the effective seed (eff_seed applied in the kernel)
    const uint64_t* soff;
};
__device__ __forceinline__ float dmask(const DropArg& d, uint64_t seed, uint32_t th, float sc, int64_t i, int C,
                                       int ch, float g) {
    const uint64_t m = d.L > 0 ? (uint64_t)((i / ((int64_t)d.L * C)) * C + ch) : (uint64_t)i;
    return mix_hash(seed, m) >= th ? g * sc : 0.f;
}

// k_bn_apply4 followed by Dropout1d over (sample, channel) columns of L rows (L = 0: element-wise
// dropout): each element the value cls.hip's k_dropout writes from the applied output (the same
// hash of index b C + c, threshold and scale) — one pass over the activations instead of two
template <int ACT>
__global__ __launch_bounds__(NT) void k_bn_apply4d(const float* __restrict__ x, int64_t n, int C,
                                                   const float* __restrict__ mean, const float* __restrict__ rstd,
                                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                                   float* __restrict__ y, int L, float p, uint64_t seed,
                                                   const uint64_t* __restrict__ soff) {
    __shared__ float4 q4[BNV_C];   // (mean, rstd, gamma, beta) per channel
    for (int c = threadIdx.x; c < C; c += NT) q4[c] = make_float4(mean[c], rstd[c], gamma[c], beta[c]);
    __syncthreads();
    seed = eff_seed(seed, soff);
    const uint32_t th = drop_threshold(p);
    const float sc = 1.f / (1.f - p);
    const int64_t LC = (int64_t)L * C;
    auto drop = [&](int64_t i, int ch, float v) {
        const uint64_t m = L > 0 ? (uint64_t)((i / LC) * C + ch) : (uint64_t)i;
        return mix_hash(seed, m) >= th ? v * sc : 0.f;
    };
    const int64_t base = (int64_t)blockIdx.x * (NT * 4 * BNV_V);
    const int step = (NT * 4) % C;
    int c = (int)((base + 4 * threadIdx.x) % C);
#pragma unroll
    for (int v = 0; v < BNV_V; ++v, c = wrapc(c + step, C)) {
        const int64_t j = base + 4 * (threadIdx.x + NT * v);
        if (j >= n) break;
        int ce[4];
        chan4(c, C, ce);
        if (j + 4 <= n) {
            const float4 xv = *(const float4*)(x + j);
            const float xs[4] = {xv.x, xv.y, xv.z, xv.w};
            float o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float4 q = q4[ce[e]];
                o[e] = drop(j + e, ce[e], bn_fwd_val(xs[e], q.x, q.y, q.z, q.w, ACT));
            }
            *(float4*)(y + j) = make_float4(o[0], o[1], o[2], o[3]);
        } else {
            for (int e = 0; e < (int)(n - j); ++e) {
                const float4 q = q4[ce[e]];
                y[j + e] = drop(j + e, ce[e], bn_fwd_val(x[j + e], q.x, q.y, q.z, q.w, ACT));
            }
        }
    }
}

template <int ACT, bool DROP = false>
__global__ __launch_bounds__(NT) void k_bn_dx4(const float* __restrict__ dy, const float* __restrict__ x, int64_t n,
                                               int64_t M, int C, const float* __restrict__ mean,
                                               const float* __restrict__ rstd, const float* __restrict__ gamma,
                                               const float* __restrict__ beta, const float* __restrict__ dgamma,
                                               const float* __restrict__ dbeta, float* __restrict__ dx,
                                               DropArg dr = DropArg{}) {
    __shared__ float p[6][BNV_C];
    for (int c = threadIdx.x; c < C; c += NT) {
        p[0][c] = mean[c];
        p[1][c] = rstd[c];
        p[2][c] = gamma[c];
        p[3][c] = beta[c];
        p[4][c] = dgamma[c];
        p[5][c] = dbeta[c];
    }
    __syncthreads();
    const float inv = 1.f / (float)M;
    const int64_t base = (int64_t)blockIdx.x * (NT * 4 * BNV_V);
    const int step = (NT * 4) % C;
    int c = (int)((base + 4 * threadIdx.x) % C);
    auto one = [&](float xe, float dye, int cc) { return bn_bwd_val(dye, xe, &p[0][0], BNV_C, cc, ACT, inv); };
    const uint64_t dseed = DROP ? eff_seed(dr.seed, dr.soff) : 0;
    const uint32_t th = DROP ? drop_threshold(dr.p) : 0u;
    const float dsc = DROP ? 1.f / (1.f - dr.p) : 1.f;
    auto gm = [&](int64_t i, int cc, float g) { return DROP ? dmask(dr, dseed, th, dsc, i, C, cc, g) : g; };
#pragma unroll
    for (int v = 0; v < BNV_V; ++v, c = wrapc(c + step, C)) {
        const int64_t j = base + 4 * (threadIdx.x + NT * v);
        if (j >= n) break;
        int ce[4];
        chan4(c, C, ce);
        if (j + 4 <= n) {
            const float4 xv = *(const float4*)(x + j), gv = *(const float4*)(dy + j);
            *(float4*)(dx + j) = make_float4(one(xv.x, gm(j, ce[0], gv.x), ce[0]), one(xv.y, gm(j + 1, ce[1], gv.y), ce[1]),
                                             one(xv.z, gm(j + 2, ce[2], gv.z), ce[2]),
                                             one(xv.w, gm(j + 3, ce[3], gv.w), ce[3]));
        } else {
            for (int e = 0; e < (int)(n - j); ++e) dx[j + e] = one(x[j + e], gm(j + e, ce[e], dy[j + e]), ce[e]);
        }
    }
}

// Column partial sums (kinds as k_col_partial) over rows [r0, r1) of block b,
// r0 a multiple of 4: thread tid < T' reads the float4s at flat offsets
// r0*C + 4 tid + 4T' k, 4T' a multiple of C, so its four channels never change;
// the per-thread sums are combined in LDS in fixed order.
template <int KIND, int ACT, bool DROP = false, int U = 4>
__global__ __launch_bounds__(NT) void k_col_partial4(const float* __restrict__ x, const float* __restrict__ dy,
                                                     int64_t M, int C, int64_t rows_per_block, int Tp,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     float* __restrict__ part, BnFin fin, DropArg dr = DropArg{}) {
    __shared__ float red0[4 * NT], red1[4 * NT];
    // partials: plain stores for a separate finaliser, agent-coherent for the in-kernel one
    const __amdgpu_buffer_rsrc_t pr = agent_rsrc(part, (int64_t)2 * C * gridDim.x * 4);
    auto put = [&](int cc, float s0, float s1) {
        const int64_t o0 = (int64_t)cc * gridDim.x + blockIdx.x, o1 = (int64_t)(C + cc) * gridDim.x + blockIdx.x;
        if (fin.mode < 0) {
            part[o0] = s0;
            part[o1] = s1;
        } else {
            st_agent(pr, (unsigned)(o0 * 4), s0);
            st_agent(pr, (unsigned)(o1 * 4), s1);
        }
    };
    const int tid = threadIdx.x;
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = r0 + rows_per_block < M ? r0 + rows_per_block : M;
    float a0[4] = {0.f, 0.f, 0.f, 0.f}, a1[4] = {0.f, 0.f, 0.f, 0.f};
    if (tid < Tp) {
        int ce[4];
        chan4((4 * tid) % C, C, ce);
        const uint64_t dseed = DROP ? eff_seed(dr.seed, dr.soff) : 0;
        const uint32_t th = DROP ? drop_threshold(dr.p) : 0u;
        const float dsc = DROP ? 1.f / (1.f - dr.p) : 1.f;
        auto gm = [&](int64_t i, int cc, float g) { return DROP ? dmask(dr, dseed, th, dsc, i, C, cc, g) : g; };
        float mu[4], rs[4], ga[4], be[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            mu[e] = KIND >= 1 ? mean[ce[e]] : 0.f;
            rs[e] = KIND == 2 ? rstd[ce[e]] : 0.f;
            ga[e] = KIND == 2 ? gamma[ce[e]] : 0.f;
            be[e] = KIND == 2 ? beta[ce[e]] : 0.f;
        }
        const int64_t end = r1 * C;
        auto acc = [&](int e, float v, float g) {
            if (KIND == 0) {
                a0[e] += v;
            } else if (KIND == 1) {
                const float d = v - mu[e];
                a0[e] += d * d;
            } else {
                const float h = (v - mu[e]) * rs[e];
                const float dz = g * act_d(h * ga[e] + be[e], ACT);
                a0[e] += dz;
                a1[e] += dz * h;
            }
        };
        // KIND < 2 or ACT <= 1: the arithmetic spelled out (contraction off, fmaf where the
        // one-at-a-time loop compiled to an fma: KIND 1 d*d + a0; KIND 2 g act' + a0 and
        // h (g act') + a1 — act' is 0 or 1 for ACT <= 1, so every product there is exact),
        // four float4 of each stream in flight per thread over the same sequence of f: the
        // sums and their bits do not depend on the unrolling or on the compiler's choices
        constexpr bool PIN = KIND < 2 || ACT <= 1;
        auto acc4 = [&](int e, float v, float g) {
#pragma clang fp contract(off)
            if (KIND == 0) {
                a0[e] = a0[e] + v;
            } else if (KIND == 1) {
                const float d = v - mu[e];
                a0[e] = fmaf(d, d, a0[e]);
            } else {
                const float h = (v - mu[e]) * rs[e];
                const float ad = act_d(fmaf(h, ga[e], be[e]), ACT);
                a0[e] = fmaf(g, ad, a0[e]);
                a1[e] = fmaf(h, g * ad, a1[e]);
            }
        };
        auto accx = [&](int e, float v, float g) {
            if constexpr (PIN) acc4(e, v, g);
            else acc(e, v, g);
        };
        // U float4 of each stream in flight per thread (the same f sequence for any U: the same sums)
        int64_t f = r0 * C + 4 * tid;
        if constexpr (PIN) {
            for (; f + 4 * (U - 1) * (int64_t)Tp + 4 <= end; f += 4 * U * (int64_t)Tp) {
                float4 xv[U], gv[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    xv[u] = *(const float4*)(x + f + 4 * (int64_t)Tp * u);
                    gv[u] = KIND == 2 ? *(const float4*)(dy + f + 4 * (int64_t)Tp * u) : make_float4(0.f, 0.f, 0.f, 0.f);
                }
                if constexpr (DROP) {
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int64_t i0 = f + 4 * (int64_t)Tp * u;
                        gv[u] = make_float4(gm(i0, ce[0], gv[u].x), gm(i0 + 1, ce[1], gv[u].y),
                                            gm(i0 + 2, ce[2], gv[u].z), gm(i0 + 3, ce[3], gv[u].w));
                    }
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    acc4(0, xv[u].x, gv[u].x);
                    acc4(1, xv[u].y, gv[u].y);
                    acc4(2, xv[u].z, gv[u].z);
                    acc4(3, xv[u].w, gv[u].w);
                }
            }
        }
        for (; f < end; f += 4 * Tp) {
            if (f + 4 <= end) {
                const float4 xv = *(const float4*)(x + f);
                float4 gv = make_float4(0.f, 0.f, 0.f, 0.f);
                if (KIND == 2) gv = *(const float4*)(dy + f);
                if constexpr (DROP)
                    gv = make_float4(gm(f, ce[0], gv.x), gm(f + 1, ce[1], gv.y), gm(f + 2, ce[2], gv.z),
                                     gm(f + 3, ce[3], gv.w));
                accx(0, xv.x, gv.x);
                accx(1, xv.y, gv.y);
                accx(2, xv.z, gv.z);
                accx(3, xv.w, gv.w);
            } else {
                for (int e = 0; e < (int)(end - f); ++e) accx(e, x[f + e], KIND == 2 ? gm(f + e, ce[e], dy[f + e]) : 0.f);
            }
        }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        red0[4 * tid + e] = a0[e];
        red1[4 * tid + e] = a1[e];
    }
    __syncthreads();
    const int groups = 4 * Tp / C;
    if (groups >= 256) {
        // very narrow rows (C <= 4: 256 to 1024 thread groups per channel): one wave per
        // channel, lane l sums groups l, l + 64, ... in order, then a fixed shuffle tree — the
        // one-thread loop over 1024 LDS values was the kernel's tail (C = 1, M = 1M rows:
        // 46 -> 8.5 us; at C = 11 / 16 the one-thread loop is not slower, and keeps its bits)
        const int lane = tid & 63;
        for (int cc = tid >> 6; cc < C; cc += NT / 64) {
            float s0 = 0.f, s1 = 0.f;
            for (int q = lane; q < groups; q += 64) {
                s0 += red0[q * C + cc];
                s1 += red1[q * C + cc];
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                s0 += __shfl_down(s0, o);
                s1 += __shfl_down(s1, o);
            }
            if (lane == 0) put(cc, s0, s1);
        }
    } else {
        for (int cc = tid; cc < C; cc += NT) {
            float s0 = 0.f, s1 = 0.f;
            for (int q = 0; q < groups; ++q) {
                s0 += red0[q * C + cc];
                s1 += red1[q * C + cc];
            }
            // channel-major (part[k][c][block]): a channel's partials are one contiguous run
            put(cc, s0, s1);
        }
    }
    if (fin.mode >= 0) bn_fold_finalize(part, C, fin);
}

// active threads of k_col_partial4: the largest multiple of C / gcd(C, 4) within NT
static inline int colp_threads(int C) {
    const int g = C % 4 == 0 ? 4 : (C % 2 == 0 ? 2 : 1);
    const int P = C / g;
    return P <= NT ? NT / P * P : 0;
}

#define VT_ACT_SWITCH(act, F) \
    switch (act) {            \
        case ACT_RELU: F(ACT_RELU); break; \
        case ACT_GELU: F(ACT_GELU); break; \
        case ACT_TANH: F(ACT_TANH); break; \
        default: F(ACT_NONE); break;       \
    }

static inline unsigned bnv_blocks(int64_t n) { return (unsigned)((n + NT * 4 * BNV_V - 1) / (NT * 4 * BNV_V)); }

static void bn_apply_vec(const float* x, int64_t M, int C, const float* mean, const float* rstd, const float* gamma,
                         const float* beta, int act, float* y, hipStream_t st) {
    const int64_t n = M * C;
#define VT_F(A) hipLaunchKernelGGL(k_bn_apply4<A>, dim3(bnv_blocks(n)), dim3(NT), 0, st, x, n, C, mean, rstd, gamma, beta, y)
    VT_ACT_SWITCH(act, VT_F)
#undef VT_F
}

static void bn_dx_vec(const float* dy, const float* x, int64_t M, int C, const float* mean, const float* rstd,
                      const float* gamma, const float* beta, int act, const float* dgamma, const float* dbeta,
                      float* dx, hipStream_t st, const DropArg* dr = nullptr) {
    const int64_t n = M * C;
#define VT_F(A)                                                                                                   \
    if (dr)                                                                                                       \
        hipLaunchKernelGGL((k_bn_dx4<A, true>), dim3(bnv_blocks(n)), dim3(NT), 0, st, dy, x, n, M, C, mean, rstd,  \
                           gamma, beta, dgamma, dbeta, dx, *dr);                                                    \
    else                                                                                                          \
        hipLaunchKernelGGL((k_bn_dx4<A>), dim3(bnv_blocks(n)), dim3(NT), 0, st, dy, x, n, M, C, mean, rstd, gamma,  \
                           beta, dgamma, dbeta, dx, DropArg{})
    VT_ACT_SWITCH(act, VT_F)
#undef VT_F
}

// float4 of each stream in flight per thread of k_col_partial4 (VAETEB_COLP_U: 4 or 8; same bits)
static int g_colp_u = getenv("VAETEB_COLP_U") ? atoi(getenv("VAETEB_COLP_U")) : 4;

static void col_partial_vec(int kind, const float* x, const float* dy, int64_t M, int C, int64_t rpb, int blocks,
                            const float* mean, const float* rstd, const float* gamma, const float* beta, int act,
                            float* part, hipStream_t st, BnFin fin, const DropArg* dr = nullptr) {
    const int Tp = colp_threads(C);
    if (kind == 2 && !dr && g_colp_u == 8) {
#define VT_F(A)                                                                                                    \
        hipLaunchKernelGGL((k_col_partial4<2, A, false, 8>), dim3(blocks), dim3(NT), 0, st, x, dy, M, C, rpb, Tp,   \
                           mean, rstd, gamma, beta, part, fin, DropArg{})
        VT_ACT_SWITCH(act, VT_F)
#undef VT_F
        return;
    }
    if (kind == 0) {
        hipLaunchKernelGGL((k_col_partial4<0, ACT_NONE>), dim3(blocks), dim3(NT), 0, st, x, dy, M, C, rpb, Tp, mean,
                           rstd, gamma, beta, part, fin, DropArg{});
    } else if (kind == 1) {
        hipLaunchKernelGGL((k_col_partial4<1, ACT_NONE>), dim3(blocks), dim3(NT), 0, st, x, dy, M, C, rpb, Tp, mean,
                           rstd, gamma, beta, part, fin, DropArg{});
    } else {
#define VT_F(A)                                                                                                      \
    if (dr)                                                                                                          \
        hipLaunchKernelGGL((k_col_partial4<2, A, true>), dim3(blocks), dim3(NT), 0, st, x, dy, M, C, rpb, Tp, mean,   \
                           rstd, gamma, beta, part, fin, *dr);                                                         \
    else                                                                                                             \
        hipLaunchKernelGGL((k_col_partial4<2, A>), dim3(blocks), dim3(NT), 0, st, x, dy, M, C, rpb, Tp, mean, rstd,   \
                           gamma, beta, part, fin, DropArg{})
        VT_ACT_SWITCH(act, VT_F)
#undef VT_F
    }
}

static BnFin no_fin() {
    BnFin f{};
    f.mode = -1;
    return f;
}

// column partials + their finalize: in the partial kernel's last-arriving workgroups when the
// channels allow one thread per sum (C <= 128; the group sums after the block partials in
// ws), else the separate k_bn_finalize launch
static void col_partial_fin(int kind, const float* x, const float* dy, int64_t M, int C, int64_t rpb, int blocks,
                            const float* mean, const float* rstd, const float* gamma, const float* beta, int act,
                            float* ws, hipStream_t st, BnFin f, const DropArg* dr = nullptr) {
    if (C <= 128 && g_bn_fold) {
        const int ng = (blocks + BN_GB - 1) / BN_GB;
        f.gpart = reinterpret_cast<double*>(ws + (((int64_t)2 * C * blocks + 1) & ~(int64_t)1));
        f.slot0 = arrive_slots((unsigned)ng + 1, st);
        col_partial_vec(kind, x, dy, M, C, rpb, blocks, mean, rstd, gamma, beta, act, ws, st, f, dr);
    } else {
        col_partial_vec(kind, x, dy, M, C, rpb, blocks, mean, rstd, gamma, beta, act, ws, st, no_fin(), dr);
        hipLaunchKernelGGL(k_bn_finalize, dim3(C), dim3(NT), 0, st, ws, blocks, C, f);
    }
}

static inline unsigned blocks_for(int64_t n, int t = 256) { return (unsigned)((n + t - 1) / t); }

// ----------------------------------------------------- synchronised BatchNorm
// The per-rank halves of a cross-rank (SyncBatchNorm) train-mode BatchNorm: per-channel
// sums in double from the same column partials (k_col_partial4) and the same
// fixed-order combine as k_bn_finalize, written as [2][C] doubles + the row count at
// [2C], so the caller can all-reduce them (SUM) between the launches.
__global__ __launch_bounds__(NT) void k_sbn_sums(const float* __restrict__ part, int blocks, int C, int64_t M,
                                                 double* __restrict__ sums) {
    __shared__ double r0[NT], r1[NT];
    const int c = blockIdx.x;
    double a0 = 0.0, a1 = 0.0;
    const float* p0 = part + (int64_t)c * blocks;
    const float* p1 = part + (int64_t)(C + c) * blocks;
    for (int b = threadIdx.x; b < blocks; b += NT) {
        a0 += (double)p0[b];
        a1 += (double)p1[b];
    }
    r0[threadIdx.x] = a0;
    r1[threadIdx.x] = a1;
    __syncthreads();
    for (int o = NT / 2; o > 0; o >>= 1) {
        if (threadIdx.x < o) {
            r0[threadIdx.x] += r0[threadIdx.x + o];
            r1[threadIdx.x] += r1[threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        sums[c] = r0[0];
        sums[C + c] = r1[0];
        if (c == 0) sums[2 * C] = (double)M;
    }
}

// which 0: mean = S0 / M_total.  which 1: var = S0 / M_total -> rstd, running statistics
// (unbiased with the global count, as torch's SyncBatchNorm).  which 2: the LOCAL column
// sums of the backward -> dbeta (+)= S0, dgamma (+)= S1 (this rank's parameter gradients,
// averaged by the data-parallel all-reduce like any other gradient).
__global__ void k_sbn_stats(const double* __restrict__ sums, int C, int which, float eps, float momentum,
                            float* __restrict__ mean, float* __restrict__ rstd, float* __restrict__ run_mean,
                            float* __restrict__ run_var, float* __restrict__ dgamma, float* __restrict__ dbeta,
                            int accumulate) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const double M = sums[2 * C];
    if (which == 0) {
        mean[c] = (float)(sums[c] / M);
    } else if (which == 1) {
        const double var = sums[c] / M;
        rstd[c] = (float)(1.0 / sqrt(var + (double)eps));
        if (run_mean) {
            const double unb = M > 1 ? var * M / (M - 1) : var;
            run_mean[c] = (float)((1.0 - momentum) * run_mean[c] + momentum * mean[c]);
            run_var[c] = (float)((1.0 - momentum) * run_var[c] + momentum * unb);
        }
    } else {
        dbeta[c] = accumulate ? dbeta[c] + (float)sums[c] : (float)sums[c];
        dgamma[c] = accumulate ? dgamma[c] + (float)sums[C + c] : (float)sums[C + c];
    }
}

// the global column sums of the backward, divided by the global row count (read on the
// device: no host synchronisation), as the dgamma / dbeta arrays of k_bn_dx4 with M = 1
__global__ void k_sbn_dsum(const double* __restrict__ sums, int C, float* __restrict__ dg, float* __restrict__ db) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const double M = sums[2 * C];
    db[c] = (float)(sums[c] / M);
    dg[c] = (float)(sums[C + c] / M);
}

// y = act(BN(x)) for conv.hip's fused conv + BatchNorm forward
int bn_apply_launch(const float* x, int64_t M, int C, const float* mean, const float* rstd, const float* gamma,
                    const float* beta, int act, float* y, hipStream_t st) {
    if (C <= BNV_C)
        bn_apply_vec(x, M, C, mean, rstd, gamma, beta, act, y, st);
    else
        hipLaunchKernelGGL(k_bn_apply, dim3(blocks_for(M * C)), dim3(256), 0, st, x, M, C, mean, rstd, gamma, beta,
                           act, y);
    return VT_OK;
}

}  // namespace vt

using namespace vt;

extern "C" {

int vt_layernorm_fwd(const float* x, int64_t R, int C, const float* gamma, const float* beta, int act, float eps,
                     float* y, float* xhat, float* rstd, void* stream) {
    VT_CHECK_ARG(R > 0 && C > 0 && act >= 0 && act <= 3, "vt_layernorm_fwd: shape/act");
    if (C <= 256) {
        const dim3 grid((unsigned)((R + NT / 16 - 1) / (NT / 16)));
        hipStream_t st = S(stream);
        if (C <= 32)
            hipLaunchKernelGGL(k_ln_fwd16<2>, grid, dim3(NT), 0, st, x, R, C, gamma, beta, act, eps, y, xhat, rstd);
        else if (C <= 64)
            hipLaunchKernelGGL(k_ln_fwd16<4>, grid, dim3(NT), 0, st, x, R, C, gamma, beta, act, eps, y, xhat, rstd);
        else if (C <= 128)
            hipLaunchKernelGGL(k_ln_fwd16<8>, grid, dim3(NT), 0, st, x, R, C, gamma, beta, act, eps, y, xhat, rstd);
        else
            hipLaunchKernelGGL(k_ln_fwd16<16>, grid, dim3(NT), 0, st, x, R, C, gamma, beta, act, eps, y, xhat, rstd);
        VT_LAUNCH_CHECK("vt_layernorm_fwd");
        return VT_OK;
    }
    if (C >= 1024 && C % 4 == 0 && C <= 4 * 4 * NT && ((uintptr_t)x | (uintptr_t)y | (uintptr_t)gamma |
                                                       (uintptr_t)beta | (uintptr_t)xhat) % 16 == 0) {
        const int v4 = (C / 4 + NT - 1) / NT;
        hipStream_t st = S(stream);
#define VT_LNW(V)                                                                                              \
    if (v4 == V) hipLaunchKernelGGL(k_ln_fwd_wide<V>, dim3((unsigned)R), dim3(NT), 0, st, x, C, gamma, beta, act, eps, \
                                    y, xhat, rstd);
        VT_LNW(1) VT_LNW(2) VT_LNW(3) VT_LNW(4)
#undef VT_LNW
        VT_LAUNCH_CHECK("vt_layernorm_fwd");
        return VT_OK;
    }
    hipLaunchKernelGGL(k_ln_fwd, dim3(blocks_for(R, NT / 64)), dim3(NT), 0, S(stream), x, R, C, gamma, beta, act, eps,
                       y, xhat, rstd);
    VT_LAUNCH_CHECK("vt_layernorm_fwd");
    return VT_OK;
}

// workspace: small C (<=512): 2*C*min(1024, ceil(R/64)) floats; wide C: 2*R*C floats.
int vt_layernorm_bwd(const float* dy, const float* xhat, const float* rstd, int64_t R, int C, const float* gamma,
                     const float* beta, int act, float* dx, float* dgamma, float* dbeta, int accumulate_params,
                     float* ws, int64_t ws_floats, void* stream) {
    VT_CHECK_ARG(R > 0 && C > 0, "vt_layernorm_bwd: shape");
    hipStream_t st = S(stream);
    if (C <= 256) {
        int64_t blocks = (R + 63) / 64;  // 64 rows per workgroup (4 passes of 16 rows)
        if (blocks > 1024) blocks = 1024;
        if (blocks * 2 * C > ws_floats) blocks = ws_floats / (2 * C);
        VT_CHECK_ARG(blocks >= 1, "vt_layernorm_bwd: workspace too small");
        const int64_t rpb = (R + blocks - 1) / blocks;
        blocks = (R + rpb - 1) / rpb;
        const dim3 grid((unsigned)blocks);
#define VT_LNB(CPL) hipLaunchKernelGGL(k_ln_bwd16<CPL>, grid, dim3(NT), 0, st, dy, xhat, rstd, R, C, gamma, beta, act, \
                                       rpb, dx, ws)
        if (C <= 32) VT_LNB(2);
        else if (C <= 64) VT_LNB(4);
        else if (C <= 128) VT_LNB(8);
        else VT_LNB(16);
#undef VT_LNB
        hipLaunchKernelGGL(k_colred16, dim3((unsigned)((2 * C + CR_C - 1) / CR_C)), dim3(NT), 0, st, ws, (int)blocks,
                           2 * C, dgamma, dbeta, C, accumulate_params);
    } else if (C <= 512) {
        int64_t blocks = (R + 63) / 64;
        if (blocks > 1024) blocks = 1024;
        if (blocks * 2 * C > ws_floats) blocks = ws_floats / (2 * C);
        VT_CHECK_ARG(blocks >= 1, "vt_layernorm_bwd: workspace too small");
        const int64_t rpb = (R + blocks - 1) / blocks;
        blocks = (R + rpb - 1) / rpb;
        hipLaunchKernelGGL(k_ln_bwd<8>, dim3((unsigned)blocks), dim3(NT), 0, st, dy, xhat, rstd, R, C, gamma, beta,
                           act, rpb, dx, ws);
        hipLaunchKernelGGL(k_reduce_parts, dim3(2 * C), dim3(NT), 0, st, ws, (int)blocks, 2 * C, dgamma,
                           dbeta, C, accumulate_params);
    } else {
        VT_CHECK_ARG(ws_floats >= 2 * R * C, "vt_layernorm_bwd: workspace too small (wide)");
        hipLaunchKernelGGL(k_ln_bwd_wide, dim3((unsigned)R), dim3(NT), 0, st, dy, xhat, rstd, C, gamma, beta, act, dx,
                           ws);
        hipLaunchKernelGGL(k_reduce_parts, dim3(2 * C), dim3(NT), 0, st, ws, (int)R, 2 * C, dgamma, dbeta,
                           C, accumulate_params);
    }
    VT_LAUNCH_CHECK("vt_layernorm_bwd");
    return VT_OK;
}

// column-partial blocks of an M-row BatchNorm within ws_floats: the block partials [2][C][blocks]
// + (in-kernel finalize) the group sums [2C][ceil(blocks / BN_GB)] doubles after them
static int bn_blocks(int64_t M, int64_t ws_floats, int C, int64_t* rpb) {
    auto need = [&](int64_t b) { return ((2 * C * b + 1) & ~(int64_t)1) + 4 * C * ((b + BN_GB - 1) / BN_GB); };
    int64_t blocks = (M + 255) / 256;
    // in-kernel finalize (C <= 128): fewer, longer blocks — every block's arrival (an atomic round
    // trip) lengthens it, and at 2048 blocks those waits stacked up over the block rounds
    const int64_t cap = C <= 128 && g_bn_fold ? BN_FOLD_BLOCKS : 2048;
    if (blocks > cap) blocks = cap;
    while (blocks > 1 && need(blocks) > ws_floats) blocks = blocks * 15 / 16 < blocks - 1 ? blocks * 15 / 16 : blocks - 1;
    if (need(blocks) > ws_floats) return 0;
    *rpb = ((M + blocks - 1) / blocks + 3) / 4 * 4;  // a multiple of 4 (k_col_partial4's float4 rows)
    return (int)((M + *rpb - 1) / *rpb);
}

static BnFin fin_of(int mode, int64_t M) {
    BnFin f{};
    f.mode = mode;
    f.M = M;
    return f;
}

// Train-mode BatchNorm1d over x (M = B*L rows, C channels) + activation.
// Writes y, the batch mean / rstd (saved for backward) and updates the
// running statistics in place (nullable) with PyTorch's momentum semantics.
int vt_batchnorm_fwd(const float* x, int64_t M, int C, const float* gamma, const float* beta, int act, float eps,
                     float momentum, float* y, float* mean, float* rstd, float* run_mean, float* run_var, float* ws,
                     int64_t ws_floats, void* stream) {
    VT_CHECK_ARG(M > 0 && C > 0 && C <= 256, "vt_batchnorm_fwd: shape (C <= 256)");
    int64_t rpb;
    const int blocks = bn_blocks(M, ws_floats, C, &rpb);
    VT_CHECK_ARG(blocks >= 1, "vt_batchnorm_fwd: workspace too small");
    hipStream_t st = S(stream);
    BnFin f0 = fin_of(0, M);
    f0.mean = mean;
    col_partial_fin(0, x, nullptr, M, C, rpb, blocks, nullptr, nullptr, nullptr, nullptr, 0, ws, st, f0);
    BnFin f1 = fin_of(1, M);
    f1.eps = eps;
    f1.momentum = momentum;
    f1.mean = mean;
    f1.rstd = rstd;
    f1.run_mean = run_mean;
    f1.run_var = run_var;
    col_partial_fin(1, x, nullptr, M, C, rpb, blocks, mean, nullptr, nullptr, nullptr, 0, ws, st, f1);
    bn_apply_vec(x, M, C, mean, rstd, gamma, beta, act, y, st);
    VT_LAUNCH_CHECK("vt_batchnorm_fwd");
    return VT_OK;
}

int vt_batchnorm_fwd_dropout(const float* x, int64_t M, int C, const float* gamma, const float* beta, int act,
                             float eps, float momentum, float* y, float* mean, float* rstd, float* run_mean,
                             float* run_var, int L, float p, int64_t seed, const void* seed_offset, float* ws,
                             int64_t ws_floats, void* stream) {
    VT_CHECK_ARG(M > 0 && C > 0 && C <= 256 && L >= 0 && (L == 0 || M % L == 0) && p >= 0.f && p < 1.f,
                 "vt_batchnorm_fwd_dropout: shape (C <= 256, M a multiple of L) / 0 <= p < 1");
    int64_t rpb;
    const int blocks = bn_blocks(M, ws_floats, C, &rpb);
    VT_CHECK_ARG(blocks >= 1, "vt_batchnorm_fwd_dropout: workspace too small");
    hipStream_t st = S(stream);
    BnFin f0 = fin_of(0, M);
    f0.mean = mean;
    col_partial_fin(0, x, nullptr, M, C, rpb, blocks, nullptr, nullptr, nullptr, nullptr, 0, ws, st, f0);
    BnFin f1 = fin_of(1, M);
    f1.eps = eps;
    f1.momentum = momentum;
    f1.mean = mean;
    f1.rstd = rstd;
    f1.run_mean = run_mean;
    f1.run_var = run_var;
    col_partial_fin(1, x, nullptr, M, C, rpb, blocks, mean, nullptr, nullptr, nullptr, 0, ws, st, f1);
    const int64_t n = M * C;
    const uint64_t* so = seed_off(seed_offset, p);
#define VT_F(A)                                                                                                  \
    hipLaunchKernelGGL(k_bn_apply4d<A>, dim3(bnv_blocks(n)), dim3(NT), 0, st, x, n, C, mean, rstd, gamma, beta, y, \
                       L, p, (uint64_t)seed, so)
    VT_ACT_SWITCH(act, VT_F)
#undef VT_F
    VT_LAUNCH_CHECK("vt_batchnorm_fwd_dropout");
    return VT_OK;
}

int vt_batchnorm_bwd(const float* dy, const float* x, int64_t M, int C, const float* mean, const float* rstd,
                     const float* gamma, const float* beta, int act, float* dx, float* dgamma, float* dbeta,
                     int accumulate_params, float* ws, int64_t ws_floats, void* stream) {
    VT_CHECK_ARG(M > 0 && C > 0 && C <= 256, "vt_batchnorm_bwd: shape");
    int64_t rpb;
    const int blocks = bn_blocks(M, ws_floats - 2 * C, C, &rpb);
    VT_CHECK_ARG(blocks >= 1, "vt_batchnorm_bwd: workspace too small");
    hipStream_t st = S(stream);
    // fresh sums for the dx formula live at the end of ws; params may accumulate
    float* dg_now = ws + (ws_floats - 2 * C);
    float* db_now = dg_now + C;
    BnFin f = fin_of(2, M);
    f.dgamma = dg_now;
    f.dbeta = db_now;
    f.pg = dgamma;   // the parameter gradients written by the same finalize (round 5: was a
    f.pb = dbeta;    // k_reduce_parts launch over the one fresh sum per channel)
    f.pacc = accumulate_params;
    col_partial_fin(2, x, dy, M, C, rpb, blocks, mean, rstd, gamma, beta, act, ws, st, f);
    bn_dx_vec(dy, x, M, C, mean, rstd, gamma, beta, act, dg_now, db_now, dx, st);
    VT_LAUNCH_CHECK("vt_batchnorm_bwd");
    return VT_OK;
}

int vt_batchnorm_bwd_dropout(const float* dy, const float* x, int64_t M, int C, const float* mean, const float* rstd,
                             const float* gamma, const float* beta, int act, int L, float p, int64_t seed,
                             const void* seed_offset, float* dx, float* dgamma, float* dbeta, int accumulate_params,
                             float* ws, int64_t ws_floats, void* stream) {
    VT_CHECK_ARG(M > 0 && C > 0 && C <= 256 && L >= 0 && (L == 0 || M % L == 0) && p >= 0.f && p < 1.f,
                 "vt_batchnorm_bwd_dropout: shape (C <= 256, M a multiple of L) / 0 <= p < 1");
    if (p == 0.f)
        return vt_batchnorm_bwd(dy, x, M, C, mean, rstd, gamma, beta, act, dx, dgamma, dbeta, accumulate_params, ws,
                                ws_floats, stream);
    int64_t rpb;
    const int blocks = bn_blocks(M, ws_floats - 2 * C, C, &rpb);
    VT_CHECK_ARG(blocks >= 1, "vt_batchnorm_bwd_dropout: workspace too small");
    hipStream_t st = S(stream);
    const DropArg dr{L, p, (uint64_t)seed, seed_off(seed_offset, p)};
    float* dg_now = ws + (ws_floats - 2 * C);
    float* db_now = dg_now + C;
    BnFin f = fin_of(2, M);
    f.dgamma = dg_now;
    f.dbeta = db_now;
    f.pg = dgamma;
    f.pb = dbeta;
    f.pacc = accumulate_params;
    col_partial_fin(2, x, dy, M, C, rpb, blocks, mean, rstd, gamma, beta, act, ws, st, f, &dr);
    bn_dx_vec(dy, x, M, C, mean, rstd, gamma, beta, act, dg_now, db_now, dx, st, &dr);
    VT_LAUNCH_CHECK("vt_batchnorm_bwd_dropout");
    return VT_OK;
}

// The column sums of the BatchNorm backward without the element-wise pass: dgamma /
// dbeta (+)= the sums, and bnp = [mean | rstd | gamma | beta | dgamma_now | dbeta_now]
// (6 x C) for the bf16 conv backward kernels that apply the BN input gradient while
// staging their operand (vt_conv1d_bwd_*_bf16_bn).
int vt_batchnorm_bwd_coef(const float* dy, const float* x, int64_t M, int C, const float* mean, const float* rstd,
                          const float* gamma, const float* beta, int act, float* dgamma, float* dbeta,
                          int accumulate_params, float* bnp, float* ws, int64_t ws_floats, void* stream) {
    VT_CHECK_ARG(M > 0 && C > 0 && C <= 256 && bnp, "vt_batchnorm_bwd_coef: shape");
    int64_t rpb;
    const int blocks = bn_blocks(M, ws_floats, C, &rpb);
    VT_CHECK_ARG(blocks >= 1, "vt_batchnorm_bwd_coef: workspace too small");
    hipStream_t st = S(stream);
    float* dg_now = bnp + 4 * C;
    float* db_now = bnp + 5 * C;
    BnFin f = fin_of(2, M);
    f.mean = const_cast<float*>(mean);
    f.rstd = const_cast<float*>(rstd);
    f.dgamma = dg_now;
    f.dbeta = db_now;
    f.bnp = bnp;
    f.gamma = gamma;
    f.beta = beta;
    f.pg = dgamma;
    f.pb = dbeta;
    f.pacc = accumulate_params;
    col_partial_fin(2, x, dy, M, C, rpb, blocks, mean, rstd, gamma, beta, act, ws, st, f);
    VT_LAUNCH_CHECK("vt_batchnorm_bwd_coef");
    return VT_OK;
}

int vt_batchnorm_eval(const float* x, int64_t M, int C, const float* run_mean, const float* run_var, float eps,
                      const float* gamma, const float* beta, int act, float* y, void* stream) {
    VT_CHECK_ARG(M > 0 && C > 0, "vt_batchnorm_eval: shape");
    hipLaunchKernelGGL(k_bn_eval, dim3(blocks_for(M * C)), dim3(256), 0, S(stream), x, M, C, run_mean, run_var, eps,
                       gamma, beta, act, y);
    VT_LAUNCH_CHECK("vt_batchnorm_eval");
    return VT_OK;
}

int vt_syncbn_sums(const float* x, const float* dy, int64_t M, int C, int which, const float* mean,
                   const float* rstd, const float* gamma, const float* beta, int act, double* sums, float* ws,
                   int64_t ws_floats, void* stream) {
    VT_CHECK_ARG(M > 0 && C > 0 && C <= 256 && which >= 0 && which <= 2 && sums, "vt_syncbn_sums: shape");
    VT_CHECK_ARG(which == 0 || mean, "vt_syncbn_sums: mean needed");
    VT_CHECK_ARG(which < 2 || (dy && rstd && gamma && beta), "vt_syncbn_sums: backward arguments");
    int64_t rpb;
    const int blocks = bn_blocks(M, ws_floats, C, &rpb);
    VT_CHECK_ARG(blocks >= 1, "vt_syncbn_sums: workspace too small");
    hipStream_t st = S(stream);
    col_partial_vec(which, x, dy, M, C, rpb, blocks, mean, rstd, gamma, beta, act, ws, st, no_fin());
    hipLaunchKernelGGL(k_sbn_sums, dim3(C), dim3(NT), 0, st, ws, blocks, C, M, sums);
    VT_LAUNCH_CHECK("vt_syncbn_sums");
    return VT_OK;
}

int vt_syncbn_stats(const double* sums, int C, int which, float eps, float momentum, float* mean, float* rstd,
                    float* run_mean, float* run_var, float* dgamma, float* dbeta, int accumulate, void* stream) {
    VT_CHECK_ARG(sums && C > 0 && which >= 0 && which <= 2, "vt_syncbn_stats: arguments");
    VT_CHECK_ARG((which == 0 && mean) || (which == 1 && mean && rstd) || (which == 2 && dgamma && dbeta),
                 "vt_syncbn_stats: outputs");
    hipLaunchKernelGGL(k_sbn_stats, dim3(blocks_for(C)), dim3(256), 0, S(stream), sums, C, which, eps, momentum, mean,
                       rstd, run_mean, run_var, dgamma, dbeta, accumulate);
    VT_LAUNCH_CHECK("vt_syncbn_stats");
    return VT_OK;
}

int vt_batchnorm_apply(const float* x, int64_t M, int C, const float* mean, const float* rstd, const float* gamma,
                       const float* beta, int act, float* y, void* stream) {
    VT_CHECK_ARG(M > 0 && C > 0 && C <= BNV_C, "vt_batchnorm_apply: shape");
    bn_apply_vec(x, M, C, mean, rstd, gamma, beta, act, y, S(stream));
    VT_LAUNCH_CHECK("vt_batchnorm_apply");
    return VT_OK;
}

int vt_syncbn_bwd_dx(const float* dy, const float* x, int64_t M, int C, const float* mean, const float* rstd,
                     const float* gamma, const float* beta, int act, const double* sums, float* dx, float* ws,
                     void* stream) {
    VT_CHECK_ARG(M > 0 && C > 0 && C <= BNV_C && sums && ws, "vt_syncbn_bwd_dx: arguments");
    hipStream_t st = S(stream);
    float* dg = ws;
    float* db = ws + C;
    hipLaunchKernelGGL(k_sbn_dsum, dim3(blocks_for(C)), dim3(256), 0, st, sums, C, dg, db);
    const int64_t n = M * C;
#define VT_F(A)                                                                                                   \
    hipLaunchKernelGGL(k_bn_dx4<A>, dim3(bnv_blocks(n)), dim3(NT), 0, st, dy, x, n, (int64_t)1, C, mean, rstd, \
                       gamma, beta, dg, db, dx)
    VT_ACT_SWITCH(act, VT_F)
#undef VT_F
    VT_LAUNCH_CHECK("vt_syncbn_bwd_dx");
    return VT_OK;
}

int vt_act_fwd(const float* x, int64_t n, int act, float* y, void* stream) {
    VT_CHECK_ARG(n > 0, "vt_act_fwd: n");
    hipLaunchKernelGGL(k_act_fwd, dim3(blocks_for(n)), dim3(256), 0, S(stream), x, n, act, y);
    VT_LAUNCH_CHECK("vt_act_fwd");
    return VT_OK;
}

int vt_act_bwd(const float* dy, const float* x, int64_t n, int act, float* dx, void* stream) {
    VT_CHECK_ARG(n > 0, "vt_act_bwd: n");
    hipLaunchKernelGGL(k_act_bwd, dim3(blocks_for(n)), dim3(256), 0, S(stream), dy, x, n, act, dx);
    VT_LAUNCH_CHECK("vt_act_bwd");
    return VT_OK;
}

}  // extern "C"
