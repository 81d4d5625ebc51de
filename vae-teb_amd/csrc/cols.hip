// Glue kernels of the step that were ATen launches on the critical chain.
//
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
    const unsigned per_row = (unsigned)(ncols / V);
    const unsigned n = (unsigned)(rows * per_row);   // < 2^31 (checked on the host): 32-bit index math
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const unsigned r = i / per_row;
        const int c = (int)(i - r * per_row) * V;
        const float* s = src + (int64_t)r * ld_src + sc0 + c;
        float* d = dst + (int64_t)r * ld_dst + dc0 + c;
        if constexpr (V == 4) *(float4*)d = *(const float4*)s;
        else *d = *s;
    }
}

// torch.clamp's backward (autograd: where((x >= lo) & (x <= hi), g, 0), four ATen launches): one pass
// (V = 4: float4 pieces, n a multiple of 4 and the pointers 16-B aligned)
template <int V>
__global__ __launch_bounds__(256) void k_clamp_bwd(const float* __restrict__ g, const float* __restrict__ x, int64_t n,
                                                   float lo, float hi, float* __restrict__ gx) {
    auto one = [&](float v, float gv) { return (v >= lo && v <= hi) ? gv : 0.f; };
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / V; i += (int64_t)gridDim.x * blockDim.x) {
        if constexpr (V == 4) {
            const float4 v = ((const float4*)x)[i], gv = ((const float4*)g)[i];
            ((float4*)gx)[i] = make_float4(one(v.x, gv.x), one(v.y, gv.y), one(v.z, gv.z), one(v.w, gv.w));
        } else {
            gx[i] = one(x[i], g[i]);
        }
    }
}

// zero up to ZR_MAX ranges [a, b) of one buffer in one launch (the gradient buffer's non-first-writer
// ranges at the step start: one Fill launch each before)
constexpr int ZR_MAX = 16;
struct ZeroRanges {
    int n;
    int64_t a[ZR_MAX], len[ZR_MAX];
};
__global__ __launch_bounds__(256) void k_zero_ranges(float* __restrict__ base, ZeroRanges zr, int64_t total) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t j = i;
        int r = 0;
        while (r + 1 < zr.n && j >= zr.len[r]) j -= zr.len[r++];
        base[zr.a[r] + j] = 0.f;
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
    VT_CHECK_ARG(n < (1ll << 31), "vt_copy_cols: %lld pieces (at most 2^31 - 1)", (long long)n);
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

extern "C" int vt_clamp_bwd(const float* g, const float* x, int64_t n, float lo, float hi, float* gx, void* stream) {
    VT_CHECK_ARG(g && x && gx && n > 0, "vt_clamp_bwd: shape");
    const bool v4 = n % 4 == 0 && (((uintptr_t)g | (uintptr_t)x | (uintptr_t)gx) & 15u) == 0;
    const int64_t pieces = v4 ? n / 4 : n;
    const unsigned grid = (unsigned)std::min<int64_t>((pieces + 255) / 256, 8192);
    if (v4)
        hipLaunchKernelGGL(k_clamp_bwd<4>, dim3(grid), dim3(256), 0, S(stream), g, x, n, lo, hi, gx);
    else
        hipLaunchKernelGGL(k_clamp_bwd<1>, dim3(grid), dim3(256), 0, S(stream), g, x, n, lo, hi, gx);
    VT_LAUNCH_CHECK("vt_clamp_bwd");
    return VT_OK;
}

extern "C" int vt_zero_ranges(float* base, int n, const int64_t* starts, const int64_t* ends, void* stream) {
    VT_CHECK_ARG(base && n >= 1 && n <= ZR_MAX && starts && ends, "vt_zero_ranges: 1 <= n <= %d ranges", ZR_MAX);
    ZeroRanges zr{};
    zr.n = n;
    int64_t total = 0;
    for (int r = 0; r < n; ++r) {
        VT_CHECK_ARG(ends[r] >= starts[r] && starts[r] >= 0, "vt_zero_ranges: range %d", r);
        zr.a[r] = starts[r];
        zr.len[r] = ends[r] - starts[r];
        total += zr.len[r];
    }
    if (total == 0) return VT_OK;
    const unsigned grid = (unsigned)std::min<int64_t>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(k_zero_ranges, dim3(grid), dim3(256), 0, S(stream), base, zr, total);
    VT_LAUNCH_CHECK("vt_zero_ranges");
    return VT_OK;
}
