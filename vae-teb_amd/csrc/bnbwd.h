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

// BatchNorm + activation forward, act(fma((x - mean) rstd, gamma, beta)) — the expression the
// apply kernel computed before round 5 (its contraction made explicit): k_bn_apply4 and the conv
// kernels that apply the previous block's BatchNorm while staging their window (a conv stack's
// inner block outputs are not materialised, round 5) — one definition, identical values.  (A
// precomputed scale / shift, one fma per element, moved the bf16 step's losses by more than the
// reference's own autocast spread at S = 256: test_s256_bf16_step_within_reference_autocast_spread.)
__device__ __forceinline__ float bn_fwd_val(float x, float mean, float rstd, float gam, float bet, int act) {
    const float z = fmaf((x - mean) * rstd, gam, bet);
    switch (act) {
        case 1: return z > 0.f ? z : 0.f;
        case 2: return 0.5f * z * (1.f + erff(z * 0.70710678118654752f));
        case 3: return tanhf(z);
        default: return z;
    }
}

// The previous block's BatchNorm of a staged input (nullptr mean: none): per-channel parameters
// staged into LDS interleaved, [cs][4] floats (mean, rstd, gamma, beta); channels >= C padding
struct BnIn {
    const float *mean, *rstd, *gamma, *beta;
    int act;   // 1 (ReLU): the only activation the staging applies
};
__device__ __forceinline__ void stage_bn_in(const BnIn& bi, int C, float* ip, int cs) {
    for (int c = threadIdx.x; c < cs; c += blockDim.x) {
        const bool ok = c < C;
        *reinterpret_cast<float4*>(ip + 4 * c) = ok ? make_float4(bi.mean[c], bi.rstd[c], bi.gamma[c], bi.beta[c])
                                                    : make_float4(0.f, 0.f, 0.f, 0.f);
    }
}
// the fold's inner blocks are ReLU blocks (the stacks' tanh block is always their last, whose
// output is materialised): ReLU only in the staging, so the kernels carry no tanh / erf code;
// a channel's four parameters are one 16-byte LDS read, taken where the element is formed
__device__ __forceinline__ float bn_relu_at(const float* ip, int cs, int c, float x) {
    (void)cs;
    const float4 q = *reinterpret_cast<const float4*>(ip + 4 * c);
    return bn_fwd_val(x, q.x, q.y, q.z, q.w, 1);
}

}  // namespace vt
