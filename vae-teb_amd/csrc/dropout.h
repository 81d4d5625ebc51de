// Dropout masks shared by the classifier's kernels (cls.hip: Dropout / Dropout1d, attention
// probabilities) and the BatchNorm apply with a fused Dropout1d (norm.hip): one counter-based
// hash per (seed, element index), so a mask is a pure function of its index.
#pragma once
#include <stdint.h>

#include <hip/hip_runtime.h>

namespace vt {

__device__ __forceinline__ uint32_t mix_hash(uint64_t seed, uint64_t idx) {
    uint64_t z = seed + 0x9E3779B97F4A7C15ull * (idx + 1ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (uint32_t)(z >> 32);
}

__device__ __forceinline__ uint32_t drop_threshold(float p) {
    const double t = (double)p * 4294967296.0;
    return t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
}

// Device-side seed offset (the seed_offset argument of the dropout / attention calls): added to every dropout seed, advanced
// once per training step on the device (vt_dropout_seed_advance), so a captured step replayed
// by the native executor draws new masks each replay (its host seeds are frozen at capture).
__device__ __forceinline__ uint64_t eff_seed(uint64_t seed, const uint64_t* __restrict__ soff) {
    return soff ? seed + soff[0] : seed;
}

// the seed offset is read only when something is dropped (p > 0): a caller without one, or an
// eval / p = 0 call, passes nothing the kernels would dereference
static inline const uint64_t* seed_off(const void* off, float p) {
    return p > 0.f ? reinterpret_cast<const uint64_t*>(off) : nullptr;
}

}  // namespace vt
