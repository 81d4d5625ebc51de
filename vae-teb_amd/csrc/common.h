// Shared helpers for the VAE-TEB gfx950 kernels (C-ABI in include/vaeteb.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/vaeteb.h"

namespace vt {

// Error channel for the C ABI: every entry point returns VT_OK or a negative
// code; the message of the last failure on this thread is kept for
// vt_last_error().  No C++ exception crosses the ABI.
void set_error(const char* fmt, ...);
// host stub of the gradient-bucket marker kernel (optim.hip), recognised by the executor
const void* bucket_marker_kernel();

#define VT_CHECK_ARG(cond, ...)                  \
    do {                                         \
        if (!(cond)) {                           \
            ::vt::set_error(__VA_ARGS__);        \
            return VT_ERR_ARG;                   \
        }                                        \
    } while (0)

#define VT_LAUNCH_CHECK(name)                                                     \
    do {                                                                          \
        hipError_t e_ = hipGetLastError();                                        \
        if (e_ != hipSuccess) {                                                   \
            ::vt::set_error("%s: %s", name, hipGetErrorString(e_));               \
            return VT_ERR_HIP;                                                    \
        }                                                                         \
    } while (0)

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cconj(float2 a) { return make_float2(a.x, -a.y); }
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Block-wide sum for blockDim.x <= 1024; `red` must hold >= 16 floats.
__device__ __forceinline__ float block_sum(float v, float* red) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    float t = 0.f;
    for (int i = 0; i < nw; ++i) t += red[i];
    return t;
}

// Reflect index (torch 'reflect', edge not repeated), extended periodically
// with period 2(n-1): equals the iterated reflection of
// ref/hdf5_dataset/kymatio_phase_scattering.py:174-205 for any pad size, and
// kymatio's single F.pad reflect (torch_backend.py:50-78) when pad < n.
__device__ __forceinline__ int reflect_idx(int i, int n) {
    if (n == 1) return 0;
    const int p = 2 * (n - 1);
    i %= p;
    if (i < 0) i += p;
    return i < n ? i : p - i;
}

// Source index of padded position i (relative to the signal start) for the
// front-end border modes of ref/hdf5_dataset/kymatio_phase_scattering.py:162-172:
// 0 reflect (iterated), 1 constant zero (returns -1), 2 circular.
__device__ __forceinline__ int pad_src(int i, int n, int mode) {
    if (mode == 0) return reflect_idx(i, n);
    if (mode == 1) return (i < 0 || i >= n) ? -1 : i;
    i %= n;
    return i < 0 ? i + n : i;
}

}  // namespace vt
