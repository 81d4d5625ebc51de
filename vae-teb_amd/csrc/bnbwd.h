// BatchNorm backward, element-wise (shared by norm.hip's k_bn_dx4 and the fused
// bf16 conv backward kernels of conv_bf16.hip, so both form bit-identical values).
#pragma once
#include "common.h"

namespace vt {

// BatchNorm backward applied to an operand while it is staged (the bf16 conv
// backward kernels read the block's output gradient dy and its pre-BN conv output
// x instead of a materialised BN input gradient): with p = [mean | rstd | gamma |
// beta | dgamma | dbeta] (6 x C, the column sums of this backward) and invM = 1/M,
//   dx = gamma rstd (dz - dbeta/M - xhat dgamma/M),  xhat = (x - mean) rstd,
//   dz = dy act'(xhat gamma + beta)
// — one definition for both paths (bit-identical values).
__device__ __forceinline__ float bn_actd(float z, int act) {
#pragma clang fp contract(off)   // the same rounding in every kernel that inlines it
    switch (act) {
        case 1: return z > 0.f ? 1.f : 0.f;
        case 2: {
            const float cdf = 0.5f * (1.f + erff(z * 0.70710678118654752f));
            const float pdf = 0.39894228040143268f * expf(-0.5f * z * z);
            return cdf + z * pdf;
        }
        case 3: {
            const float t = tanhf(z);
            return 1.f - t * t;
        }
        default: return 1.f;
    }
}
// the same with the six parameters of channel c already in registers
__device__ __forceinline__ float bn_bwd_val_r(float dy, float x, float mean, float rstd, float gam, float bet,
                                              float dgam, float dbet, int act, float invM) {
#pragma clang fp contract(off)
    const float h = (x - mean) * rstd;
    const float dz = dy * bn_actd(h * gam + bet, act);
    return gam * rstd * (dz - dbet * invM - h * dgam * invM);
}
__device__ __forceinline__ float bn_bwd_val(float dy, float x, const float* p, int C, int c, int act, float invM) {
    return bn_bwd_val_r(dy, x, p[c], p[C + c], p[2 * C + c], p[3 * C + c], p[4 * C + c], p[5 * C + c], act, invM);
}

// BatchNorm + activation forward as a per-channel affine map, act(x scale + shift) with
// scale = rstd gamma and shift = beta - mean scale (ATen's batch_norm_elemt form): k_bn_apply4
// and the conv kernels that apply the previous block's BatchNorm while staging their window (a
// conv stack's inner block outputs are not materialised, round 5) — one definition, identical
// values, one fma per element
__device__ __forceinline__ float2 bn_affine(float mean, float rstd, float gam, float bet) {
#pragma clang fp contract(off)
    const float sc = rstd * gam;
    return make_float2(sc, fmaf(-mean, sc, bet));
}
__device__ __forceinline__ float bn_fwd_val(float x, float sc, float sh, int act) {
    const float z = fmaf(x, sc, sh);
    switch (act) {
        case 1: return z > 0.f ? z : 0.f;
        case 2: return 0.5f * z * (1.f + erff(z * 0.70710678118654752f));
        case 3: return tanhf(z);
        default: return z;
    }
}

// The previous block's BatchNorm of a staged input (nullptr mean: none): the per-channel
// affine map staged into LDS as [2][cs] floats (scale | shift); channels cs > C are padding
struct BnIn {
    const float *mean, *rstd, *gamma, *beta;
    int act;   // 1 (ReLU): the only activation the staging applies
};
__device__ __forceinline__ void stage_bn_in(const BnIn& bi, int C, float* ip, int cs) {
    for (int c = threadIdx.x; c < cs; c += blockDim.x) {
        const float2 a = c < C ? bn_affine(bi.mean[c], bi.rstd[c], bi.gamma[c], bi.beta[c]) : make_float2(0.f, 0.f);
        ip[c] = a.x;
        ip[cs + c] = a.y;
    }
}
// the fold's inner blocks are ReLU blocks (the stacks' tanh block is always their last, whose
// output is materialised): ReLU only in the staging, so the kernels carry no tanh / erf code
__device__ __forceinline__ float bn_relu_val(float x, float sc, float sh) { return bn_fwd_val(x, sc, sh, 1); }
__device__ __forceinline__ float bn_relu_at(const float* ip, int cs, int c, float x) {
    return bn_relu_val(x, ip[c], ip[cs + c]);
}
// NC (4 or 8) consecutive channels cb .. cb + NC - 1 (cb + NC <= cs, cb % 4 == 0): 16-byte LDS reads
template <int NC>
__device__ __forceinline__ void bn_in_n(const float* ip, int cs, int cb, float (&sc)[NC], float (&sh)[NC]) {
    static_assert(NC % 4 == 0, "bn_in_n: 4-channel groups");
#pragma unroll
    for (int q = 0; q < NC / 4; ++q) {
        const float4 s = *reinterpret_cast<const float4*>(ip + cb + 4 * q);
        const float4 h = *reinterpret_cast<const float4*>(ip + cs + cb + 4 * q);
        sc[4 * q] = s.x; sc[4 * q + 1] = s.y; sc[4 * q + 2] = s.z; sc[4 * q + 3] = s.w;
        sh[4 * q] = h.x; sh[4 * q + 1] = h.y; sh[4 * q + 2] = h.z; sh[4 * q + 3] = h.w;
    }
}

}  // namespace vt
