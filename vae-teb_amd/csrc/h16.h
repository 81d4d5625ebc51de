// 16-bit MFMA operand formats (round 6).  The kernels that multiply 16-bit operands with
// fp32 accumulation (decoder heads, conv blocks, ResidualMLP stacks) are templates over the
// operand type H:
//   __bf16    (default) fp32's exponent range, 8 significant bits: no loss scaling needed;
//   _Float16  the reference's own autocast width (Lightning precision="16-mixed",
//             torch.amp.autocast('cuda'): ref/model/graph_model.py:510,670,709-726), 11
//             significant bits, range +-65504: trained with a dynamic loss scale
//             (vt_grad_norm_clip_scaled / vt_loss_scale_*, optim.hip), as GradScaler does.
// Both run v_mfma_f32_16x16x32_{bf16,f16} at the same rate on gfx950.  The format is a
// library-wide setting (vt_set_h16_format), read by the host dispatchers at launch time, so
// every C-ABI signature stays the same; a captured step keeps the kernels it was captured with.
#pragma once
#include "common.h"

namespace vt {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <typename H> struct HVec;
template <> struct HVec<__bf16> {
    typedef bf16x8 v8;
    typedef bf16x4 v4;
};
template <> struct HVec<_Float16> {
    typedef f16x8 v8;
    typedef f16x4 v4;
};
template <typename H> using hv8 = typename HVec<H>::v8;
template <typename H> using hv4 = typename HVec<H>::v4;

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(f16x8 a, f16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// the library-wide operand format: 0 bf16, 1 fp16 (vt_set_h16_format, abi.cpp)
int h16_format();

// run a launch statement with H bound to the current format's element type
#define VT_H16(...)                          \
    do {                                     \
        if (::vt::h16_format()) {            \
            typedef _Float16 H;              \
            __VA_ARGS__;                     \
        } else {                             \
            typedef __bf16 H;                \
            __VA_ARGS__;                     \
        }                                    \
    } while (0)

}  // namespace vt
