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

// n consecutive arrival counters of a VT_ARRIVE_POOL (round-robin; n <= ARRIVE_POOL / 8).  Launches
// enqueued on a capturing stream draw from the upper half of the pool, all others from the lower
// half: counters baked into a captured step are never handed to an eager launch, however many
// eager launches wrap their half, so an eager kernel on another stream cannot share a counter with
// a replay running beside it.  (Two captures share the upper half: their graphs are replayed one
// at a time.)
unsigned arrive_slots(unsigned n, hipStream_t st);
// host shadow of a VT_ARRIVE_POOL, registered at load time for vt_arrive_reset
int register_arrive_pool(const void* sym, size_t bytes);

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cconj(float2 a) { return make_float2(a.x, -a.y); }
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }

// ------------------------------------------------------- last-arriving workgroup
// Cross-workgroup reductions finished inside the producing kernel instead of a separate
// finaliser launch (round 5): every workgroup writes its partial with agent-coherent stores
// (st_agent: the store reaches the device's coherence point past this XCD's L2), waits for
// them, and arrives on a counter (a vector-memory atomic); the workgroup that arrives last —
// whichever it is — reads the partials with agent-coherent loads (ld_agent) and combines them
// in a FIXED order (by index, never by arrival), so the result is deterministic.  No
// agent-scope fence: on gfx950 that writes back the whole L2 of the XCD, and in the step's
// concurrent streams the write-backs slowed every kernel sharing the L2 (measured: 7.80 ->
// 8.71 ms/step with fences in the split sums).  The counters live in a per-translation-unit
// pool of zero-initialised device words (VT_ARRIVE_POOL); the last arrival resets its counter,
// so a counter is zero again whenever its kernel has finished (graph replays reuse the same
// slots).  Host side: arrive_slots() hands out disjoint runs round-robin, so kernels that may
// run concurrently on different streams never share one; vt_arrive_reset zeroes every pool
// after a failed launch.
// INVARIANT: every cross-workgroup partial a finaliser reads is written with st_agent and read
// with ld_agent (sc1: past the XCD's L2).  There is no release / acquire fence, so a plain load
// or store of a partial (another XCD's L2 may hold a stale line) would silently break the
// reduction: k_sum_splits_grp, bn_fold_finalize / k_col_partial4 and k_mfma_gemm keep to it.
constexpr unsigned ARRIVE_POOL = 1u << 16;
#define VT_ARRIVE_POOL(name)                                 \
    static __device__ unsigned name[::vt::ARRIVE_POOL];      \
    [[maybe_unused]] static const int name##_registered =    \
        ::vt::register_arrive_pool((const void*)&name, sizeof(unsigned) * ::vt::ARRIVE_POOL)

// agent-coherent (sc1) buffer accesses of a partial-result array: a descriptor over the array
// (uniform base) and per-lane byte offsets
__device__ __forceinline__ __amdgpu_buffer_rsrc_t agent_rsrc(const void* p, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0,
                                             (int)(bytes < 0x7ffffff0 ? bytes : 0x7ffffff0), 0x00020000);
}
constexpr int CPOL_SC1 = 16;
__device__ __forceinline__ void st_agent(__amdgpu_buffer_rsrc_t r, unsigned off, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, (int)off, 0, CPOL_SC1);
}
__device__ __forceinline__ float ld_agent(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, CPOL_SC1));
}

__device__ __forceinline__ void st_agent(__amdgpu_buffer_rsrc_t r, unsigned off, double v) {
    typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), r, (int)off, 0, CPOL_SC1);
}
__device__ __forceinline__ double ld_agent_d(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, CPOL_SC1));
}

// true in every thread of the workgroup that arrives last of `total` on *ctr; the caller's
// partial stores (st_agent) are complete before the arrival
__device__ __forceinline__ bool last_arrival(unsigned* ctr, unsigned total) {
    __shared__ unsigned s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this thread's partial stores have landed
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned old = atomicAdd(ctr, 1u);
        const bool last = old == total - 1;
        if (last) atomicExch(ctr, 0u);   // every arrival is in: ready for the next launch
        s_last = last ? 1u : 0u;
    }
    __syncthreads();
    return s_last != 0u;
}

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
