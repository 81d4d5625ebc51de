// Column-range copies of row-major fp32 matrices: the concatenation along the last axis in the
// encoders (ref/model/vae_teb_model.py: torch.cat([a, b], dim=-1) before cross_modal_fusion and the
// conditional encoder's MLP) and its backward split.  ATen's strided copy of a column slice into a
// contiguous tensor (the cat's gradient handed to a LayerNorm / LSTM backward that needs
// contiguous rows) ran at ~0.1 TB/s — 46 us for one 256 x 256 x 16 half on the critical chain; this
// moves 16-B pieces when the column range allows (one row's columns per thread group).
#include <algorithm>

#include "common.h"

namespace vt {
namespace {

// dst[r * ld_dst + dc0 + c] = src[r * ld_src + sc0 + c], c < ncols; V floats per thread piece
template <int V>
__global__ __launch_bounds__(256) void k_copy_cols(const float* __restrict__ src, int64_t rows, int ld_src, int sc0,
                                                   int ncols, float* __restrict__ dst, int ld_dst, int dc0) {
    const int per_row = ncols / V;
    const int64_t n = rows * per_row;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / per_row;
        const int c = (int)(i - r * per_row) * V;
        const float* s = src + r * ld_src + sc0 + c;
        float* d = dst + r * ld_dst + dc0 + c;
        if constexpr (V == 4) *(float4*)d = *(const float4*)s;
        else *d = *s;
    }
}

}  // namespace
}  // namespace vt

using namespace vt;

extern "C" int vt_copy_cols(const float* src, int64_t rows, int ld_src, int src_col0, int ncols, float* dst, int ld_dst,
                            int dst_col0, void* stream) {
    VT_CHECK_ARG(src && dst && rows > 0 && ncols > 0 && src_col0 >= 0 && dst_col0 >= 0 && src_col0 + ncols <= ld_src &&
                     dst_col0 + ncols <= ld_dst,
                 "vt_copy_cols: shape");
    const bool v4 = ncols % 4 == 0 && src_col0 % 4 == 0 && dst_col0 % 4 == 0 && ld_src % 4 == 0 && ld_dst % 4 == 0 &&
                    ((uintptr_t)src & 15u) == 0 && ((uintptr_t)dst & 15u) == 0;
    const int64_t n = rows * (v4 ? ncols / 4 : ncols);
    const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
    if (v4)
        hipLaunchKernelGGL(k_copy_cols<4>, dim3(grid), dim3(256), 0, S(stream), src, rows, ld_src, src_col0, ncols, dst,
                           ld_dst, dst_col0);
    else
        hipLaunchKernelGGL(k_copy_cols<1>, dim3(grid), dim3(256), 0, S(stream), src, rows, ld_src, src_col0, ncols, dst,
                           ld_dst, dst_col0);
    VT_LAUNCH_CHECK("vt_copy_cols");
    return VT_OK;
}
