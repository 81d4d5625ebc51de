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

}  // namespace vt
