// Packed-fp32 complex arithmetic and register DFTs for the front-end's
// training-geometry transforms (gfx950).
//
// A complex value lives in an even-aligned VGPR pair (re, im) and every
// complex add / multiply is a VOP3P v_pk_{add,mul,fma}_f32: one instruction
// moves both components, and the op_sel / neg modifiers do the swaps and sign
// flips of multiplications by -i and of the cross terms of a product, so a
// complex product is 2 packed instructions, a multiply-add by -i 1.  The
// compiler's own vectorisation of float2 code forms each product from 4-5
// packed instructions plus v_mov_b32 shuffles (75 of 268 VALU instructions
// of a radix-16 pass + twiddles; 151 with these helpers).
#pragma once
#include "common.h"

namespace vt {

typedef float c2 __attribute__((ext_vector_type(2)));  // (re, im)

__device__ __forceinline__ c2 C2(float2 a) { return c2{a.x, a.y}; }
__device__ __forceinline__ float2 F2(c2 a) { return make_float2(a.x, a.y); }

// a + (-i) b = (a.re + b.im, a.im - b.re)
__device__ __forceinline__ c2 add_mi(c2 a, c2 b) {
    c2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// a - (-i) b = (a.re - b.im, a.im + b.re)
__device__ __forceinline__ c2 sub_mi(c2 a, c2 b) {
    c2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// (-i) b
__device__ __forceinline__ c2 mul_mi(c2 b) {
    c2 r;
    asm("v_pk_add_f32 %0, 0, %1 op_sel:[0,1] op_sel_hi:[0,0] neg_hi:[0,1]" : "=v"(r) : "v"(b));
    return r;
}
// a * w
__device__ __forceinline__ c2 pmul(c2 a, c2 w) {
    c2 t, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(t) : "v"(a), "v"(w));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(r) : "v"(a), "v"(w), "v"(t));
    return r;
}
// a * conj(w)
__device__ __forceinline__ c2 pmulc(c2 a, c2 w) {
    c2 t, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0]" : "=v"(t) : "v"(a), "v"(w));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] neg_hi:[0,1,0]" : "=v"(r) : "v"(a), "v"(w), "v"(t));
    return r;
}
// acc + a * w
__device__ __forceinline__ c2 pmac(c2 acc, c2 a, c2 w) {
    c2 t, r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(t) : "v"(a), "v"(w), "v"(acc));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]" : "=v"(r) : "v"(a), "v"(w), "v"(t));
    return r;
}

// forward DFT-4 in place: X[k] = sum_n x[n] (-i)^{nk}
__device__ __forceinline__ void pdft4(c2& x0, c2& x1, c2& x2, c2& x3) {
    const c2 s02 = x0 + x2, d02 = x0 - x2, s13 = x1 + x3, d13 = x1 - x3;
    x0 = s02 + s13;
    x2 = s02 - s13;
    x1 = add_mi(d02, d13);
    x3 = sub_mi(d02, d13);
}

constexpr float kC16 = 0.92387953251128674f, kS16 = 0.38268343236508977f, kR2 = 0.70710678118654752f;

// forward DFT-8 in place, natural order (2 x DFT-4 + W_8 butterflies)
__device__ __forceinline__ void pdft8(c2 v[8]) {
    c2 e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6], o0 = v[1], o1 = v[3], o2 = v[5], o3 = v[7];
    pdft4(e0, e1, e2, e3);
    pdft4(o0, o1, o2, o3);
    const c2 w1 = pmul(o1, c2{kR2, -kR2}), w3 = pmul(o3, c2{-kR2, -kR2});
    v[0] = e0 + o0;
    v[4] = e0 - o0;
    v[1] = e1 + w1;
    v[5] = e1 - w1;
    v[2] = add_mi(e2, o2);
    v[6] = sub_mi(e2, o2);
    v[3] = e3 + w3;
    v[7] = e3 - w3;
}

// forward DFT-16 in registers, natural order in and out (4 x 4, twiddles W_16)
__device__ __forceinline__ void pdft16(c2 v[16]) {
#pragma unroll
    for (int n0 = 0; n0 < 4; ++n0) pdft4(v[n0], v[n0 + 4], v[n0 + 8], v[n0 + 12]);  // a[n0][k1] at v[n0 + 4 k1]
    v[5] = pmul(v[5], c2{kC16, -kS16});
    v[9] = pmul(v[9], c2{kR2, -kR2});
    v[13] = pmul(v[13], c2{kS16, -kC16});
    v[6] = pmul(v[6], c2{kR2, -kR2});
    v[10] = mul_mi(v[10]);
    v[14] = pmul(v[14], c2{-kR2, -kR2});
    v[7] = pmul(v[7], c2{kS16, -kC16});
    v[11] = pmul(v[11], c2{-kR2, -kR2});
    v[15] = pmul(v[15], c2{-kC16, kS16});
    c2 o[16];
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) {
        c2 a0 = v[4 * k1], a1 = v[4 * k1 + 1], a2 = v[4 * k1 + 2], a3 = v[4 * k1 + 3];
        pdft4(a0, a1, a2, a3);  // over n0 -> k0
        o[k1] = a0;
        o[k1 + 4] = a1;
        o[k1 + 8] = a2;
        o[k1 + 12] = a3;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = o[i];
}

// W_32^n = exp(-2 pi i n / 32), n < 32
constexpr float kW32Re[32] = {1.f, 0.980785251f, 0.923879504f, 0.831469595f, 0.707106769f, 0.555570245f,
                              0.382683426f, 0.195090324f, 0.f, -0.195090324f, -0.382683426f, -0.555570245f,
                              -0.707106769f, -0.831469595f, -0.923879504f, -0.980785251f, -1.f, -0.980785251f,
                              -0.923879504f, -0.831469595f, -0.707106769f, -0.555570245f, -0.382683426f,
                              -0.195090324f, 0.f, 0.195090324f, 0.382683426f, 0.555570245f, 0.707106769f,
                              0.831469595f, 0.923879504f, 0.980785251f};
__device__ __forceinline__ c2 w32(int n) { return c2{kW32Re[n & 31], kW32Re[(n + 8) & 31]}; }

// forward DFT-32 in registers, natural order (2 x DFT-16 + W_32 butterflies)
__device__ __forceinline__ void pdft32(c2 v[32]) {
    c2 e[16], o[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        e[i] = v[2 * i];
        o[i] = v[2 * i + 1];
    }
    pdft16(e);
    pdft16(o);
    v[0] = e[0] + o[0];
    v[16] = e[0] - o[0];
    v[8] = add_mi(e[8], o[8]);
    v[24] = sub_mi(e[8], o[8]);
#pragma unroll
    for (int k = 1; k < 16; ++k) {
        if (k == 8) continue;
        const c2 w = pmul(o[k], w32(k));
        v[k] = e[k] + w;
        v[k + 16] = e[k] - w;
    }
}

// Twiddle tables of the 8192 = 16 x 16 x 32 decomposition and of the 512-point
// transform (8 x 8 x 8), one fp64-accurate table per device, laid out so that
// each pass reads them coalesced (lane-contiguous):
//   T1[k2 - 1][n1]  = W_8192^{n1 k2}   k2 1..15, n1 < 512   (pass 1)
//   T2[kb - 1][n1a] = W_512^{n1a kb}   kb 1..15, n1a < 32   (pass 2)
//   TA[q - 1][l]    = W_512^{l q}      q 1..7,   l < 64     (512-point, pass A)
//   TB[r - 1][l0]   = W_64^{l0 r}      r 1..7,   l0 < 8     (512-point, pass B)
static constexpr int TW8K_T1 = 0, TW8K_T2 = 15 * 512, TW8K_TA = TW8K_T2 + 15 * 32, TW8K_TB = TW8K_TA + 7 * 64,
                     TW8K_N = TW8K_TB + 7 * 8;

// forward 512-point DFT by ONE wave (8 x 8 x 8, three register passes), in place
// in z (natural index i at position i + (i >> 3)); returns in r[j] the output
// k = (lane >> 3) + 8 (lane & 7) + 64 j.  Only lanes of the calling wave touch z:
// the passes are ordered by wave-scope fences, no workgroup barrier.
__device__ __forceinline__ int z512_pos(int i) { return i + (i >> 3); }
// the lane's twiddles of wave_fft512 (passes A and B), loadable ahead of the call
__device__ __forceinline__ void fft512_twiddles(const float2* __restrict__ tab, c2 w[7], c2 wb[7]) {
    const int l = threadIdx.x & 63, l0 = l & 7;
#pragma unroll
    for (int j = 0; j < 7; ++j) {
        w[j] = C2(tab[TW8K_TA + 64 * j + l]);
        wb[j] = C2(tab[TW8K_TB + 8 * j + l0]);
    }
}
__device__ __forceinline__ void wave_fft512(float2* z, const c2 w[7], const c2 wb[7], c2 r[8]) {
    const int l = threadIdx.x & 63, q = l >> 3, l0 = l & 7;
    c2 u[8];
    // A: n = l + 64 j -> y[l][q'] = W_512^{l q'} DFT8_j
#pragma unroll
    for (int j = 0; j < 8; ++j) u[j] = C2(z[z512_pos(l + 64 * j)]);
    pdft8(u);
#pragma unroll
    for (int j = 1; j < 8; ++j) u[j] = pmul(u[j], w[j - 1]);
#pragma unroll
    for (int j = 0; j < 8; ++j) z[z512_pos(l + 64 * j)] = F2(u[j]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // B: lane (q, l0), l = l0 + 8 l1 -> W_64^{l0 r0} DFT8_{l1}
#pragma unroll
    for (int j = 0; j < 8; ++j) u[j] = C2(z[z512_pos(l0 + 8 * j + 64 * q)]);
    pdft8(u);
#pragma unroll
    for (int j = 1; j < 8; ++j) u[j] = pmul(u[j], wb[j - 1]);
#pragma unroll
    for (int j = 0; j < 8; ++j) z[z512_pos(l0 + 8 * j + 64 * q)] = F2(u[j]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // C: lane (q, r0) -> DFT8 over l0 -> r1
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = C2(z[z512_pos(j + 8 * l0 + 64 * q)]);
    pdft8(r);
}
__device__ __forceinline__ void wave_fft512(float2* z, const float2* __restrict__ tab, c2 r[8]) {
    c2 w[7], wb[7];
    fft512_twiddles(tab, w, wb);
    wave_fft512(z, w, wb, r);
}

}  // namespace vt
