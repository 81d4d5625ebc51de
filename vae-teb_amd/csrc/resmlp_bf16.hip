// Whole-ResidualMLP kernels on bf16 MFMA (ref/model/vae_teb_model.py:336-403),
// the 16-bit-autocast counterpart of resmlp.hip (the reference trains under
// fp16 autocast, ref/model/graph_model.py:510,709-711: Linear in 16-bit, LayerNorm
// in fp32).  Linear layers multiply bf16 operands with fp32 accumulation
// (v_mfma_f32_16x16x32_bf16); LayerNorm, activations, the saved state and every
// reduction stay fp32.
//
// Orientation.  Every activation tile is kept TRANSPOSED: a wave owns 16 rows,
// lane (g = lane>>4, r = lane&15) holds row r, features 16t + 4g + i (i < 4) in
// a[t][i] — exactly the accumulator (D) layout of Z^T = W H^T.  So the D tile of
// one layer is, after a pairwise bf16 conversion, the B operand of the next
// (k-step s of 32 features = {a[2s][0..3], a[2s+1][0..3]}, no lane movement);
// the A operand (weights) is staged in LDS with the matching permutation of its
// k index inside each 32-block:  image[n][32s + 8g + j] = W[n][32s + 16(j>>2) + 4g + (j&3)].
// LayerNorm statistics of a row are a register sum + two cross-group shuffles.
//
// k_mlpb_fwd  1 workgroup per CU (8 waves), every layer's weight image resident
//             in LDS (staged once), waves independent over 16-row tiles.  Saves
//             xhat feature-major (xh[f][row], 64-B row segments) and rstd.
// k_mlpb_bwd  layer-major over a 256-row block per workgroup (wave w owns rows
//             128u + 16w + r, u = 0, 1): per GEMM, LayerNorm backward in
//             registers -> dZ; dZ^T and H^T (recomputed from xhat) go to LDS
//             images, dW|db = dZ^T H over the block on MFMA (rows as the
//             contraction); dH_prev = W^T dZ with dZ as the B operand.  One
//             dW|db + gamma|beta partial per workgroup.
// k_mlpb_sum  fixed-order sum of the partials into the parameter gradients.
// No atomics: bitwise reproducible run to run.
#include <math.h>
#include <string.h>

#include <memory>
#include <mutex>
#include <unordered_map>
#include <vector>

#include <stdlib.h>

#include "h16.h"

namespace vt {
namespace {


constexpr int MAXL = VT_MLP_MAX_LAYERS;
constexpr int MAXG = MAXL + 1;   // layers + skip projection
constexpr int BT = 512;          // threads per workgroup (8 waves)
constexpr int NW = BT / 64;
constexpr int IMR = 128;         // backward rows per workgroup and tile-per-wave (8 waves x 16)

struct BG {                      // one GEMM: z = h W^T + b, W [N][K]
    int K, N;
    int fo, fs;                  // forward image (bf16 offset, row stride): rows pad16(N), cols pad32(K)
    int bw, bs;                  // backward image W^T: LDS offset (bf16), row stride: rows pad16(K), cols pad32(N)
    int po;                      // fp32 params in LDS: bias[pad16 N], gamma, beta
    int wo;                      // dW|db partial offset (floats), N x (K + 1)
    int gbw;                     // W^T image offset (bf16) in the global image's backward region
    // split backward (k_mlpb_bwdx + k_mlpb_dw): dZ rows (bf16) of this GEMM at dz16 + zo, row stride
    // zs = pad16(N); the bias-gradient partial at xdb of a k_mlpb_bwdx workgroup's partial; the dW
    // partial (N x K) at dwo of a k_mlpb_dw row chunk's partial
    int64_t zo;
    int zs, xdb, dwo;
    const float* W;
    const float* b;
};
struct BL {                      // LayerNorm (+ act) after GEMM l
    int ln, act, xo, ri, lpo, bpo;   // xo: saved-xhat region (x Rp floats); bpo: backward LDS params
    int xlpo;                        // split backward: gamma | beta partial offset (k_mlpb_bwdx)
    const float* g;
    const float* be;
};
struct BDesc {
    int L, d0, skip, nG;
    float eps;
    int fimg;                    // forward: bytes of all weight images (params follow)
    int fbytes;                  // forward LDS bytes
    int pin;                     // LDS float offset of the input LN gamma / beta (pad16 d0 each)
    int bwimg;                   // backward: bf16 elements of the largest W^T image
    int bhrows;                  // backward: rows of the H image (max pad16(K))
    int bres;                    // backward: every W^T image resident in LDS (else one at a time, at offset 0)
    int bzrows;                  // backward: rows of the dZ image (max pad16(N))
    int bprm;                    // backward: floats of LN parameters in LDS
    int bbytes;                  // backward LDS bytes
    int P;                       // partial floats per workgroup
    int lpo0;                    // LN partial offset of the input LN
    int bpin;                    // backward LDS float offset of the input LN gamma / beta
    int gbo, gpo;                // global image: byte offsets of the W^T region and of the backward params
    char* gimg;                  // global image (k_mlpb_prep): [forward LDS image | W^T images | backward params]
    int xP, xlpo0;               // split backward: k_mlpb_bwdx partial floats per workgroup, input-LN offset
    int xbytes;                  // ... k_mlpb_bwdx LDS bytes (every W^T image resident), 0: no split plan
    int dP;                      // ... k_mlpb_dw partial floats per row chunk (every GEMM's N x K)
    const float* g0;
    const float* be0;
    BG G[MAXG];
    BL l[MAXL];
};

__device__ __forceinline__ int p16(int n) { return (n + 15) & ~15; }
__device__ __forceinline__ int p32(int n) { return (n + 31) & ~31; }

__device__ __forceinline__ float bact(float z, int act) {
    switch (act) {
        case 1: return z > 0.f ? z : 0.f;
        case 2: return 0.5f * z * (1.f + erff(z * 0.70710678118654752f));
        case 3: return tanhf(z);
        default: return z;
    }
}

__device__ __forceinline__ float bact_d(float z, int act) {
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

// k position p (0..31) of a 32-block -> feature offset inside the block
__device__ __forceinline__ int kperm(int p) {
    const int g = p >> 3, j = p & 7;
    return 16 * (j >> 2) + 4 * g + (j & 3);
}

// act over a whole tile (one uniform switch, not one per element)
template <int NT>
__device__ __forceinline__ void act_tile(f32x4 (&z)[NT], int act) {
    switch (act) {
        case 1:
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i) z[t][i] = fmaxf(z[t][i], 0.f);
            break;
        case 2:
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i) z[t][i] = bact(z[t][i], 2);
            break;
        case 3:
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i) z[t][i] = tanhf(z[t][i]);
            break;
        default:
            break;
    }
}

// act'(z) over a whole tile
template <int NT>
__device__ __forceinline__ void actd_tile(f32x4 (&z)[NT], int act) {
    switch (act) {
        case 1:
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i) z[t][i] = z[t][i] > 0.f ? 1.f : 0.f;
            break;
        case 2:
        case 3:
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i) z[t][i] = bact_d(z[t][i], act);
            break;
        default:
#pragma unroll
            for (int t = 0; t < NT; ++t) z[t] = f32x4{1.f, 1.f, 1.f, 1.f};
            break;
    }
}

// B fragments of a transposed activation tile (k-step s = features 32s..32s+31)
template <int NT, typename H>
__device__ __forceinline__ void frags(const f32x4 (&a)[NT], hv8<H> (&b)[(NT + 1) / 2]) {
#pragma unroll
    for (int s = 0; s < (NT + 1) / 2; ++s) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            b[s][j] = (H)a[2 * s][j];
            b[s][4 + j] = (2 * s + 1 < NT) ? (H)a[2 * s + 1][j] : (H)0.f;
        }
    }
}

// acc[t] = sum_s (image rows 16t..16t+15) x b[s];  nt output tiles, ks k-steps (runtime, <= template bounds)
template <int NT, int KS, typename H>
__device__ __forceinline__ void tile_gemm(const H* img, int stride, int nt, int ks, const hv8<H> (&b)[KS],
                                          f32x4 (&acc)[NT]) {
    const int lane = threadIdx.x & 63;
    const H* p = img + (lane & 15) * stride + 8 * (lane >> 4);
    const int step = 16 * stride;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        f32x4 c = f32x4{0.f, 0.f, 0.f, 0.f};
        if (t < nt) {
#pragma unroll
            for (int s = 0; s < KS; ++s)
                if (s < ks) c = mfma16(*(const hv8<H>*)(p + 32 * s), b[s], c);
        }
        acc[t] = c;
        p += step;
        __builtin_amdgcn_sched_barrier(0);   // bound the fragment loads in flight (registers)
    }
}

// Global memory through raw buffer descriptors: an access past num_records
// returns 0 / is dropped by the hardware, so rows past R and masked lanes need
// no branches (OOB: an offset past any buffer here, < 2 GiB each).
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr unsigned OOB = 0x80000000u;

__device__ __forceinline__ rsrc_t brs(const void* p, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0,
                                             (int)(bytes < 0x7ffffff0 ? bytes : 0x7ffffff0), 0x00020000);
}
__device__ __forceinline__ float bld(rsrc_t r, unsigned off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}
__device__ __forceinline__ void bst(rsrc_t r, unsigned off, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, (int)off, 0, 0);
}
__device__ __forceinline__ f32x4 bld4(rsrc_t r, unsigned off) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}
__device__ __forceinline__ void bst4(rsrc_t r, unsigned off, f32x4 v) {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (int)off, 0, 0);
}

// row-major [R][C] tile (any C) -> transposed layout (0 past C and for rows >= R).
// Element masks only in the one partial 16-feature tile (uniform branches on
// full / partial / empty tiles: per-element masks of every tile, hoisted out of
// the layer loop, exhaust the scalar registers).
template <int NT>
__device__ __forceinline__ void load_rows(f32x4 (&a)[NT], const float* src, int C, int64_t R, int64_t row) {
    const int g4 = (threadIdx.x & 63) >> 4;
    const rsrc_t r = brs(src, R * C * 4);
    const unsigned base = row < R ? (unsigned)((row * C + 4 * g4) * 4) : OOB;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
        if (16 * t < C) {
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = bld(r, base + 4 * (16 * t + i));
            if (16 * t + 16 > C) {
                const int lim = C - 16 * t - 4 * g4;   // valid elements of this lane's quad
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] = i < lim ? v[i] : 0.f;
            }
        }
        a[t] = v;
    }
}

template <int NT>
__device__ __forceinline__ void store_rows(float* dst, const f32x4 (&a)[NT], int C, int64_t R, int64_t row) {
    const int g4 = (threadIdx.x & 63) >> 4;
    const rsrc_t r = brs(dst, R * C * 4);
    const unsigned base = row < R ? (unsigned)((row * C + 4 * g4) * 4) : OOB;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        if (16 * t + 16 <= C) {
#pragma unroll
            for (int i = 0; i < 4; ++i) bst(r, base + 4 * (16 * t + i), a[t][i]);
        } else if (16 * t < C) {
#pragma unroll
            for (int i = 0; i < 4; ++i) bst(r, 16 * t + 4 * g4 + i < C ? base + 4 * (16 * t + i) : OOB, a[t][i]);
        }
    }
}

// Saved LayerNorm state xhat: fp16, row-major [Rp][pad16(C)] per LN layer (4 halves = 8 bytes per
// lane and tile), rows past R read 0.  xhat is normalised (|xhat| <= sqrt(C) <= 12), so fp16 keeps
// 11 significant bits over its whole range: the backward's LayerNorm gradient and its recomputed
// GEMM input (rounded to bf16 anyway) see it at the precision the reference's autocast gives the
// LayerNorm input (the 16-bit Linear output), at half the bytes of fp32 (round 5).
typedef _Float16 h16x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
// the region of LN layer xo (feature offset, x Rp rows) in the saved-state buffer
__device__ __forceinline__ const _Float16* xh_region(const float* xh, int64_t xo, int64_t Rp) {
    return reinterpret_cast<const _Float16*>(xh) + xo * Rp;
}
// raw halves (2 VGPRs per tile, converted where used: a prefetch stays in flight across barriers)
template <int NT>
__device__ __forceinline__ void load_sv(u32x2 (&a)[NT], const _Float16* src, int C, int64_t Rp, int64_t row,
                                        bool rok) {
    const int g4 = (threadIdx.x & 63) >> 4;
    const int nt = (C + 15) >> 4;
    const rsrc_t r = brs(src, Rp * 32 * nt);
    const unsigned base = rok ? (unsigned)((row * 16 * nt + 4 * g4) * 2) : OOB;
#pragma unroll
    for (int t = 0; t < NT; ++t)
        a[t] = t < nt ? __builtin_amdgcn_raw_buffer_load_b64(r, (int)(base + 32 * t), 0, 0) : u32x2{0u, 0u};
}
__device__ __forceinline__ f32x4 sv_f32(u32x2 v) {
    const h16x4 h = __builtin_bit_cast(h16x4, v);
    return f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
}
template <int NT>
__device__ __forceinline__ void sv_f32(const u32x2 (&a)[NT], f32x4 (&o)[NT]) {
#pragma unroll
    for (int t = 0; t < NT; ++t) o[t] = sv_f32(a[t]);
}

__device__ __forceinline__ float sum_groups(float v) {  // over the 4 lane groups (same row)
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    return v;
}

// LayerNorm (+ act) of a transposed tile, fp32: saves xhat (row-major, rows
// padded to 16 features; 0 in the padding) and rstd; z is 0 past C on entry;
// leaves h (0 past C).
template <int NT>
__device__ __forceinline__ void ln_fwd(f32x4 (&z)[NT], int C, const float* gl, const float* bl, int act, float eps,
                                       _Float16* xh, float* rs, int64_t Rp, int64_t row, bool rok) {
    const int lane = threadIdx.x & 63, g4 = lane >> 4;
    const int nt = (C + 15) >> 4;
    const float invC = 1.f / (float)C;
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t)
        if (t < nt) s += (z[t][0] + z[t][1]) + (z[t][2] + z[t][3]);
    const float mean = sum_groups(s) * invC;
    float v = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        if (t < nt) {
            z[t] -= mean;
            if (16 * t + 16 > C) {   // the partial tile: 0 past C
                const int lim = C - 16 * t - 4 * g4;
#pragma unroll
                for (int i = 0; i < 4; ++i) z[t][i] = i < lim ? z[t][i] : 0.f;
            }
            v += (z[t][0] * z[t][0] + z[t][1] * z[t][1]) + (z[t][2] * z[t][2] + z[t][3] * z[t][3]);
        }
    }
    const float rstd = rsqrtf(sum_groups(v) * invC + eps);
    bst(brs(rs, Rp * 4), (rok && g4 == 0) ? (unsigned)(row * 4) : OOB, rstd);
    const rsrc_t rx = brs(xh, Rp * 32 * nt);     // fp16 saved state (load_sv)
    const unsigned bx = rok ? (unsigned)((row * 16 * nt + 4 * g4) * 2) : OOB;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        if (t < nt) {
            z[t] *= rstd;                               // xhat (0 past C)
            const h16x4 hv = {(_Float16)z[t][0], (_Float16)z[t][1], (_Float16)z[t][2], (_Float16)z[t][3]};
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, hv), rx, (int)(bx + 32 * t), 0, 0);
            const f32x4 gv = *(const f32x4*)(gl + 16 * t + 4 * g4);
            const f32x4 bv = *(const f32x4*)(bl + 16 * t + 4 * g4);
            z[t] = z[t] * gv + bv;                      // gamma / beta are 0 past C
        }
    }
    act_tile<NT>(z, act);
}

// ------------------------------------------------------------ global images
// k_mlpb_prep builds, once per forward call (the optimizer rewrites the master
// weights every step), the stack's bf16 weight images and staged parameters in
// the exact LDS layouts: [0, fbytes) the forward LDS image (W images, bias |
// gamma | beta, input LN), then the W^T images (at G.gbw) and the backward LN
// parameters.  One element per thread, a segment per blockIdx.y.  The forward /
// backward workgroups then copy them to LDS with LDS-DMA (global_load_lds, no
// VGPR round trip), instead of every workgroup re-gathering and converting the
// fp32 weights (18 us of a 92 us backward workgroup, tools/mlpb_phases.py).
template <typename H>
__device__ __forceinline__ void mlpb_prep_seg(const BDesc& d, int seg, int e) {
    H* fimg = reinterpret_cast<H*>(d.gimg);
    float* fprm = reinterpret_cast<float*>(d.gimg + d.fimg);
    H* bimg = reinterpret_cast<H*>(d.gimg + d.gbo);
    float* bprm = reinterpret_cast<float*>(d.gimg + d.gpo);
    if (seg < d.nG) {                                  // forward image of GEMM seg: [pad16 N][fs]
        const BG& G = d.G[seg];
        if (e >= p16(G.N) * G.fs) return;
        const int n = e / G.fs, q = e - n * G.fs;
        const int k = (q & ~31) + kperm(q & 31);
        fimg[G.fo + e] = (H)((n < G.N && q < p32(G.K) && k < G.K) ? G.W[(int64_t)n * G.K + k] : 0.f);
    } else if (seg == d.nG) {                          // forward params
        const int d0p = p16(d.d0);
        if (e < d.pin) {
            int g = 0;
            while (g + 1 < d.nG && e >= d.G[g + 1].po) ++g;
            const BG& G = d.G[g];
            const int Np = p16(G.N), c = e - G.po, w = c >= 2 * Np ? 2 : (c >= Np ? 1 : 0), f = c - w * Np;
            const bool lnl = g < d.L && d.l[g].ln;
            const float* src = w == 0 ? G.b : (lnl ? (w == 1 ? d.l[g].g : d.l[g].be) : nullptr);
            fprm[e] = (src && f < G.N) ? src[f] : 0.f;
        } else if (e < d.pin + 2 * d0p) {
            const int c = e - d.pin, w = c >= d0p, f = c - w * d0p;
            fprm[e] = f < d.d0 ? (w == 0 ? d.g0 : d.be0)[f] : 0.f;
        }
    } else if (seg <= 2 * d.nG) {                      // W^T image: [pad16 K][bs], img[k][p] = W[perm p][k]
        const BG& G = d.G[seg - d.nG - 1];
        if (e >= p16(G.K) * G.bs) return;
        const int k = e / G.bs, q = e - k * G.bs;
        const int n = (q & ~31) + kperm(q & 31);
        bimg[G.gbw + e] = (H)((q < p32(G.N) && n < G.N && k < G.K) ? G.W[(int64_t)n * G.K + k] : 0.f);
    } else {                                           // backward LN params (+ the input LN)
        if (e >= d.bprm) return;
        if (e >= d.bpin) {
            const int d0p = p16(d.d0), c = e - d.bpin, w = c >= d0p, f = c - w * d0p;
            bprm[e] = f < d.d0 ? (w == 0 ? d.g0 : d.be0)[f] : 0.f;
            return;
        }
        int l = -1;
        for (int i = 0; i < d.L; ++i)
            if (d.l[i].ln && e >= d.l[i].bpo) l = i;
        const int Np = p16(d.G[l].N), c = e - d.l[l].bpo, w = c >= Np, f = c - w * Np;
        bprm[e] = f < d.G[l].N ? (w == 0 ? d.l[l].g : d.l[l].be)[f] : 0.f;
    }
}

template <typename H>
__global__ __launch_bounds__(256) void k_mlpb_prep(const BDesc* __restrict__ dp) {
    mlpb_prep_seg<H>(*dp, blockIdx.y, blockIdx.x * 256 + threadIdx.x);
}

// Every stack of a model in ONE launch (round 6, VERDICT r05 item 5: the 14 k_mlpb_prep launches of
// a step were each ~6.7 us of latency on the forward's chain): blockIdx.y walks the stacks' segment
// ranges (prefix y0), each block then does k_mlpb_prep's work for its (stack, segment) — the same
// element mapping, the same images.
constexpr int PREP_BATCH = 32;
struct PrepBatch {
    int n;
    const BDesc* d[PREP_BATCH];
    int y0[PREP_BATCH + 1];
    int x[PREP_BATCH];
};
template <typename H>
__device__ __forceinline__ void mlpb_prep_seg(const BDesc& d, int seg, int e);
template <typename H>
__global__ __launch_bounds__(256) void k_mlpb_prep_batch(PrepBatch pb) {
    int s = 0;
    while (s + 1 < pb.n && (int)blockIdx.y >= pb.y0[s + 1]) ++s;
    if ((int)blockIdx.x >= pb.x[s]) return;
    mlpb_prep_seg<H>(*pb.d[s], (int)blockIdx.y - pb.y0[s], blockIdx.x * 256 + threadIdx.x);
}

// bytes [0, nbytes) of global src -> LDS dst (16-B aligned, nbytes a multiple of 16)
// by LDS-DMA: each wave moves 1 KB per instruction (lane l -> dst + 16 l); the caller
// waits (vmcnt) and synchronises
__device__ __forceinline__ void lds_copy(char* dst, const char* src, int nbytes) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int c = 1024 * wv; c < nbytes; c += 1024 * NW) {
        if (c + 16 * lane < nbytes)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + c + 16 * lane),
                                             (__attribute__((address_space(3))) void*)(dst + c), 16, 0, 0);
    }
}
__device__ __forceinline__ void lds_copy_wait() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

// ------------------------------------------------------------------ forward
// the weight images are built from the fp32 master weights at every launch
// (the optimizer rewrites them each step); loads in batches of SB per thread,
// all in flight before the first conversion

template <typename H>
__device__ void stage_fwd(const BDesc& d, H* img, float* prm) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int g = 0; g < d.nG; ++g) {
        const BG& G = d.G[g];
        const int Np = p16(G.N), Kp = p32(G.K);
        const float* __restrict__ W = G.W;
        H* dst = img + G.fo;
        // wave w: rows n = w, w + 8, ... (two per pass); lane: columns p = lane + 64 j
        for (int n0 = wv; n0 < Np; n0 += 2 * NW) {
            float v[2][3];
#pragma unroll
            for (int r = 0; r < 2; ++r)
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    const int n = n0 + NW * r, p = lane + 64 * j;
                    const int k = (p & ~31) + kperm(p & 31);
                    v[r][j] = (n < G.N && p < Kp && k < G.K) ? W[(int64_t)n * G.K + k] : 0.f;
                }
#pragma unroll
            for (int r = 0; r < 2; ++r)
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    const int n = n0 + NW * r, p = lane + 64 * j;
                    if (n < Np && p < Kp) dst[n * G.fs + p] = (H)v[r][j];
                }
        }
        const bool lnl = g < d.L && d.l[g].ln;
        for (int c = threadIdx.x; c < 3 * Np; c += BT) {
            const int w = c >= 2 * Np ? 2 : (c >= Np ? 1 : 0), f = c - w * Np;
            const float* src = w == 0 ? G.b : (lnl ? (w == 1 ? d.l[g].g : d.l[g].be) : nullptr);
            prm[G.po + c] = (src && f < G.N) ? src[f] : 0.f;
        }
    }
    const int d0p = p16(d.d0);
    for (int c = threadIdx.x; c < 2 * d0p; c += BT) {
        const int w = c >= d0p, f = c - w * d0p;
        prm[d.pin + c] = f < d.d0 ? (w == 0 ? d.g0 : d.be0)[f] : 0.f;
    }
}

// ID: identity skip (out += x0); otherwise skip 0 / 2 (projection of x0 at the end)
template <int NT, bool ID, typename H>
__global__ __launch_bounds__(BT, 1) void k_mlpb_fwd(const BDesc* __restrict__ dp, const float* __restrict__ X, int64_t R,
                                                    float* __restrict__ out, float* __restrict__ xh,
                                                    float* __restrict__ rs, int64_t Rp) {
    const BDesc& d = *dp;   // device-resident (uniform scalar loads; a by-value descriptor indexed
                            // by layer is copied to scratch)
    constexpr int KS = (NT + 1) / 2;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const H* img = reinterpret_cast<const H*>(smem);
    float* prm = reinterpret_cast<float*>(smem + d.fimg);
    if (d.gimg) {
        lds_copy(smem, d.gimg, d.fbytes);
        lds_copy_wait();
    } else {
        stage_fwd<H>(d, reinterpret_cast<H*>(smem), prm);
        __syncthreads();
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g4 = lane >> 4, lr = lane & 15;
    const int L = d.L, d0 = d.d0, DL = d.G[L - 1].N;
    const int64_t ntiles = (R + 15) / 16;
    for (int64_t tile = (int64_t)blockIdx.x * NW + wv; tile < ntiles; tile += (int64_t)gridDim.x * NW) {
        const int64_t row = tile * 16 + lr;
        const bool rok = row < R;
        f32x4 a[NT];
        load_rows<NT>(a, X, d0, R, row);
        _Float16* xh16 = reinterpret_cast<_Float16*>(xh);
        ln_fwd<NT>(a, d0, prm + d.pin, prm + d.pin + p16(d0), 0, d.eps, xh16, rs, Rp, row, rok);
        f32x4 x0[ID ? NT : 1];
        if constexpr (ID) {
#pragma unroll
            for (int t = 0; t < NT; ++t) x0[t] = a[t];
        }
        hv8<H> bx[KS], b[KS];
        frags<NT, H>(a, bx);
#pragma unroll
        for (int s = 0; s < KS; ++s) b[s] = bx[s];
        for (int l = 0; l < L; ++l) {
            const int K = d.G[l].K, N = d.G[l].N, fo = d.G[l].fo, fs = d.G[l].fs, po = d.G[l].po;
            tile_gemm<NT, KS, H>(img + fo, fs, (N + 15) >> 4, (K + 31) >> 5, b, a);
#pragma unroll
            for (int t = 0; t < NT; ++t) a[t] += *(const f32x4*)(prm + po + 16 * t + 4 * g4);   // bias (0 past N)
            if (d.l[l].ln)
                ln_fwd<NT>(a, N, prm + po + p16(N), prm + po + 2 * p16(N), d.l[l].act, d.eps,
                           xh16 + (int64_t)d.l[l].xo * Rp, rs + (int64_t)d.l[l].ri * Rp, Rp, row, rok);
            if (l < L - 1) frags<NT, H>(a, b);
        }
        if constexpr (ID) {
#pragma unroll
            for (int t = 0; t < NT; ++t) a[t] += x0[t];
        } else if (d.skip == 2) {
            const BG& G = d.G[L];
            f32x4 sk[NT];
            tile_gemm<NT, KS, H>(img + G.fo, G.fs, (G.N + 15) >> 4, (G.K + 31) >> 5, bx, sk);
#pragma unroll
            for (int t = 0; t < NT; ++t) a[t] += sk[t] + *(const f32x4*)(prm + G.po + 16 * t + 4 * g4);
        }
        store_rows<NT>(out, a, DL, R, row);
    }
}

// ----------------------------------------------------------------- backward
// W^T image of GEMM G: img[k][32s + 8g + j] = W[32s + kperm(8g + j)][k]
// (column p = n-position of the permuted image per wave, lanes over k: coalesced W rows)
template <typename H>
__device__ void stage_wt(const BG& G, H* img) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int Kp = p16(G.K), Np = p32(G.N);
    const float* __restrict__ W = G.W;
    for (int p0 = wv; p0 < Np; p0 += 2 * NW) {
        float v[2][3];
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int p = p0 + NW * r, k = lane + 64 * j;
                const int n = (p & ~31) + kperm(p & 31);
                v[r][j] = (p < Np && n < G.N && k < G.K) ? W[(int64_t)n * G.K + k] : 0.f;
            }
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int p = p0 + NW * r, k = lane + 64 * j;
                if (p < Np && k < Kp) img[G.bw + k * G.bs + p] = (H)v[r][j];
            }
    }
}

// lane l of a 16-lane row receives lane l ^ M's value (M = 1, 2, 4, 8) by DPP: the
// same value as __shfl_xor(v, M) (ds_bpermute through the LDS crossbar) without an
// LDS round trip.  M = 4 writes the two bank pairs of the row in two moves.
template <int M>
__device__ __forceinline__ float xshfl(float v) {
    const int x = __builtin_bit_cast(int, v);
    int r;
    if constexpr (M == 1) {
        r = __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false);    // quad_perm [1,0,3,2]
    } else if constexpr (M == 2) {
        r = __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false);    // quad_perm [2,3,0,1]
    } else if constexpr (M == 4) {
        r = __builtin_amdgcn_update_dpp(x, x, 0x104, 0xF, 0x5, false);   // row_shl:4 into banks 0, 2
        r = __builtin_amdgcn_update_dpp(r, x, 0x114, 0xF, 0xA, false);   // row_shr:4 into banks 1, 3
    } else {
        static_assert(M == 8, "xshfl: M in {1, 2, 4, 8}");
        r = __builtin_amdgcn_update_dpp(0, x, 0x128, 0xF, 0xF, false);   // row_ror:8
    }
    return __builtin_bit_cast(float, r);
}

// LayerNorm(+act) backward of a transposed tile (fp32): dh -> dz in place
// (xv = xhat, 0 past C and for invalid rows; rstd 0 for invalid rows); adds the
// tile's gamma / beta column sums (over its 16 rows) to la[t]: lane (g, r)
// accumulates value v = r >> 1 of feature block 16t + 4g: v < 4 -> dgamma of
// feature 16t + 4g + v, else dbeta of feature 16t + 4g + v - 4.
template <int NT>
__device__ __forceinline__ void ln_bwd(f32x4 (&dh)[NT], const f32x4 (&xv)[NT], float rstd, int C, const float* gl,
                                       const float* bl, int act, float (&la)[NT]) {
    const int lane = threadIdx.x & 63, g4 = lane >> 4, lr = lane & 15;
    const int nt = (C + 15) >> 4;
    const float invC = 1.f / (float)C;
    if (act) {
        f32x4 pre[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t)
            pre[t] = xv[t] * *(const f32x4*)(gl + 16 * t + 4 * g4) + *(const f32x4*)(bl + 16 * t + 4 * g4);
        actd_tile<NT>(pre, act);
#pragma unroll
        for (int t = 0; t < NT; ++t) dh[t] *= pre[t];   // du (dh is 0 past C)
    }
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        if (t >= nt) continue;
        const f32x4 gv = *(const f32x4*)(gl + 16 * t + 4 * g4);
        float pq[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float du = dh[t][i];
            pq[i] = du * xv[t][i];
            pq[4 + i] = du;
            const float gd = du * gv[i];
            dh[t][i] = gd;
            s1 += gd;
            s2 += gd * xv[t][i];
        }
        // reduce-scatter of the 8 column values over the 16 rows of the group
        float q4[4], q2[2];
        const bool h8 = lr & 8, h4 = lr & 4, h2 = lr & 2;
#pragma unroll
        for (int i = 0; i < 4; ++i) q4[i] = (h8 ? pq[4 + i] : pq[i]) + xshfl<8>(h8 ? pq[i] : pq[4 + i]);
#pragma unroll
        for (int i = 0; i < 2; ++i) q2[i] = (h4 ? q4[2 + i] : q4[i]) + __shfl_xor(h4 ? q4[i] : q4[2 + i], 4);
        float q = (h2 ? q2[1] : q2[0]) + xshfl<2>(h2 ? q2[0] : q2[1]);
        q += xshfl<1>(q);
        la[t] += q;
    }
    const float m1 = sum_groups(s1) * invC, m2 = sum_groups(s2) * invC;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        if (t >= nt) {
            dh[t] = f32x4{0.f, 0.f, 0.f, 0.f};
            continue;
        }
        dh[t] = rstd * (dh[t] - m1 - xv[t] * m2);
        if (16 * t + 16 > C) {
            const int lim = C - 16 * t - 4 * g4;
#pragma unroll
            for (int i = 0; i < 4; ++i) dh[t][i] = i < lim ? dh[t][i] : 0.f;
        }
    }
}

// transposed tile -> bf16 image rows [f][col0 + r] (row stride S) for the tiles covering C
template <int NT, int S, typename H>
__device__ __forceinline__ void put_img(H* im, const f32x4 (&a)[NT], int C, int col0) {
    const int lane = threadIdx.x & 63, g4 = lane >> 4, lr = lane & 15;
    const int nt = (C + 15) >> 4;
    H* p = im + 4 * g4 * S + col0 + lr;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        if (t >= nt) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i) p[(16 * t + i) * S] = (H)a[t][i];
    }
}

// column sums of a transposed tile over its 16 rows (fp32), added to lb[t]:
// after the reduce-scatter lane (g, r) holds feature 16t + 4g + (r >> 2)
template <int NT>
__device__ __forceinline__ void colsum(const f32x4 (&z)[NT], int C, float (&lb)[NT]) {
    const int lr = threadIdx.x & 15;
    const int nt = (C + 15) >> 4;
    const bool h8 = lr & 8, h4 = lr & 4;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        if (t >= nt) continue;
        float w[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) w[i] = (h8 ? z[t][2 + i] : z[t][i]) + xshfl<8>(h8 ? z[t][i] : z[t][2 + i]);
        float q = (h4 ? w[1] : w[0]) + __shfl_xor(h4 ? w[0] : w[1], 4);
        q += xshfl<2>(q);
        q += xshfl<1>(q);
        lb[t] += q;
    }
}

// workgroup partials of the column sums, fixed-order sum over the waves:
// LayerNorm gamma | beta (la, if ln) -> dln[0 .. 2C); bias (lb, if db) -> db[f * dbs].
// flush_cols = flush_write (each wave's column sums into red), a barrier, flush_sum (the fixed-order
// sum over the waves into the partial); k_mlpb_bwd runs flush_sum of a layer step after the NEXT
// step's opening barrier instead of behind a barrier of its own (the same sums, one barrier less
// per layer step; red is next written after that step's image barrier)
template <int NT>
__device__ __forceinline__ void flush_write(float* red, const float (&la)[NT], const float (&lb)[NT], int C, bool ln,
                                            bool db) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g4 = lane >> 4, lr = lane & 15;
    const int nt = (C + 15) >> 4;
    float* rw = red + wv * (48 * NT);
    if (ln && !(lr & 1)) {
        const int v = lr >> 1;
#pragma unroll
        for (int t = 0; t < NT; ++t)
            if (t < nt) rw[t * 32 + (v >> 2) * 16 + 4 * g4 + (v & 3)] = la[t];
    }
    if (db && !(lr & 3)) {
#pragma unroll
        for (int t = 0; t < NT; ++t)
            if (t < nt) rw[32 * NT + t * 16 + 4 * g4 + (lr >> 2)] = lb[t];
    }
}
template <int NT>
__device__ __forceinline__ void flush_sum(const float* red, int C, bool ln, float* __restrict__ dln,
                                          float* __restrict__ db, int dbs) {
    const int nt = (C + 15) >> 4;
    if (ln) {
        for (int idx = threadIdx.x; idx < nt * 32; idx += BT) {
            const int t = idx >> 5, which = (idx >> 4) & 1, f = 16 * t + (idx & 15);
            float s = 0.f;
#pragma unroll
            for (int w = 0; w < NW; ++w) s += red[w * (48 * NT) + idx];
            if (f < C) dln[which * C + f] = s;
        }
    }
    if (db) {
        for (int f = threadIdx.x; f < C; f += BT) {
            float s = 0.f;
#pragma unroll
            for (int w = 0; w < NW; ++w) s += red[w * (48 * NT) + 32 * NT + f];
            db[(int64_t)f * dbs] = s;
        }
    }
}
template <int NT>
__device__ __forceinline__ void flush_cols(float* red, const float (&la)[NT], const float (&lb)[NT], int C, bool ln,
                                           float* __restrict__ dln, float* __restrict__ db, int dbs) {
    flush_write<NT>(red, la, lb, C, ln, db != nullptr);
    __syncthreads();
    flush_sum<NT>(red, C, ln, dln, db, dbs);
}

// dW partial of one GEMM over images of ROWS rows (row stride S) -> dst[n * K1 + k]
// (k < K): wave (wn = w >> 2, wk = w & 3) owns output tiles tn = wn + 2a,
// tk = wk + 4c, one tn at a time (TKS accumulators live)
template <int TNS, int TKS, int ROWS, int S, typename H>
__device__ __forceinline__ void dw_img(const H* zi, const H* hi, int N, int K, float* __restrict__ dst) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, wn = wv >> 2, wk = wv & 3;
    const int g4 = lane >> 4, lr = lane & 15, K1 = K + 1;
    const int ntn = (N + 15) >> 4, ntk = (K + 15) >> 4;
    const int off = lr * S + 8 * g4;
    for (int a = 0; a < TNS; ++a) {
        const int tn = wn + 2 * a;
        if (tn >= ntn) break;
        f32x4 acc[TKS];
#pragma unroll
        for (int c = 0; c < TKS; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
        for (int s = 0; s < ROWS / 32; ++s) {
            const hv8<H> af = *(const hv8<H>*)(zi + 16 * tn * S + off + 32 * s);
#pragma unroll
            for (int c = 0; c < TKS; ++c) {
                const int tk = wk + 4 * c;
                if (tk < ntk) acc[c] = mfma16(af, *(const hv8<H>*)(hi + 16 * tk * S + off + 32 * s), acc[c]);
            }
        }
#pragma unroll
        for (int c = 0; c < TKS; ++c) {
            const int k = 16 * (wk + 4 * c) + lr;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int n = 16 * tn + 4 * g4 + i;
                if (n < N && k < K) dst[n * K1 + k] = acc[c][i];
            }
        }
    }
}

// TPW: 16-row tiles per wave; the workgroup's block is 128 TPW rows, all of it in
// one dZ / H image (row stride IS).  Per GEMM step (layer l, last to first, then the
// skip projection) with ONE global round trip, overlapped with the LayerNorm
// backward: the raw xhat of the step's H source (layer l-1's LN output) is loaded
// at the step start, used for H, and carried to the next step as its LN input.
// stamps (diagnostic, vt_resmlp_bf16_set_stamps; nullptr normally): wave 0's wall clock at
// the start, after the staging, per step after the first barrier, the dZ pass, the H pass, the
// image barrier, the GEMM + dW and the flush, and at the end (255): 256 entries per workgroup
#define MB_STAMP(k)                                                                          \
    do {                                                                                     \
        if (stamps && threadIdx.x == 0) stamps[(int64_t)blockIdx.x * 256 + (k)] = wall_clock64(); \
    } while (0)
template <int NT, int TPW, int OCC = 1, typename H = __bf16>
__global__ __launch_bounds__(BT, 2 * OCC) void k_mlpb_bwd(const BDesc* __restrict__ dp, const float* __restrict__ dout,
                                                    const float* __restrict__ xh, const float* __restrict__ rs,
                                                    int64_t R, int64_t Rp, float* __restrict__ dx,
                                                    float* __restrict__ part, unsigned long long* __restrict__ stamps) {
    const BDesc& d = *dp;
    constexpr int KS = (NT + 1) / 2;
    constexpr int TNS = (NT + 1) / 2;          // dW output tiles per wave along n
    constexpr int TKS = (NT + 3) / 4;          // ... along k
    constexpr int ROWS = IMR * TPW;            // rows per workgroup (one image)
    constexpr int IS = ROWS + 16;              // image row stride: == 16 mod 32 -> conflict-free fragments
    extern __shared__ __attribute__((aligned(16))) char smem[];
    H* wimg = reinterpret_cast<H*>(smem);
    H* zimg = wimg + d.bwimg;
    H* himg = zimg + d.bzrows * IS;
    float* prm = reinterpret_cast<float*>(himg + d.bhrows * IS);   // [LN params per LN layer][input LN]
    float* red = prm + d.bprm;                                     // [NW][48 NT]
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g4 = lane >> 4;
    const int L = d.L, d0 = d.d0, DL = d.G[L - 1].N;
    const int64_t rbase = (int64_t)blockIdx.x * ROWS + 16 * wv + (lane & 15);
    float* pb = part + (int64_t)blockIdx.x * d.P;
    MB_STAMP(0);

    if (d.gimg) {   // W^T images (if resident) and LN parameters from the global image
        if (d.bres) lds_copy(reinterpret_cast<char*>(wimg), d.gimg + d.gbo, 2 * d.bwimg);
        lds_copy(reinterpret_cast<char*>(prm), d.gimg + d.gpo, 4 * d.bprm);
        lds_copy_wait();
    } else {
    if (d.bres)
        for (int g = 0; g < d.nG; ++g) stage_wt<H>(d.G[g], wimg);
    // gamma / beta of every LayerNorm (+ the input LN), staged once; layer l's at prm + l.bpo
    for (int l = 0; l <= L; ++l) {
        const bool inl = l == L;
        if (!inl && !d.l[l].ln) continue;
        const int C = inl ? d0 : d.G[l].N, Np = p16(C), o = inl ? d.bpin : d.l[l].bpo;
        const float* g = inl ? d.g0 : d.l[l].g;
        const float* be = inl ? d.be0 : d.l[l].be;
        for (int c = threadIdx.x; c < 2 * Np; c += BT) {
            const int w = c >= Np, f = c - w * Np;
            prm[o + c] = f < C ? (w == 0 ? g : be)[f] : 0.f;
        }
    }
    }
    const float* prm_in = prm + d.bpin;
    MB_STAMP(1);

    f32x4 dh[TPW][NT];                         // output gradient
    u32x2 xc[TPW][NT];                         // fp16 xhat of the current layer
    float rsc[TPW];                            // rstd of the current layer's LayerNorm (prefetched with xc)
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
        const int64_t row = rbase + IMR * u;
        load_rows<NT>(dh[u], dout, DL, R, row);
        rsc[u] = 0.f;
        if (d.l[L - 1].ln) {
            load_sv<NT>(xc[u], xh_region(xh, d.l[L - 1].xo, Rp), DL, Rp, row, row < R);
            rsc[u] = bld(brs(rs + (int64_t)d.l[L - 1].ri * Rp, Rp * 4), row < R ? (unsigned)(row * 4) : OOB);
        }
    }

    const int nsteps = L + (d.skip == 2 ? 1 : 0);
    // the previous layer step's column-sum flush, summed after this step's opening barrier
    int fC = 0, fdbs = 0;
    bool fln = false, fpend = false;
    float *fdln = nullptr, *fdb = nullptr;
    for (int step = 0; step < nsteps; ++step) {
        const bool skp = step == L;
        const int l = skp ? -1 : L - 1 - step;
        const BG& G = d.G[skp ? L : l];
        const int N = G.N, K = G.K, bs = G.bs;
        const bool ln = !skp && d.l[l].ln;
        const int hsrc = skp ? -1 : l - 1;    // H = output of layer hsrc (-1: x0, the input LN output)
        const float* gH = hsrc >= 0 ? prm + d.l[hsrc].bpo : prm_in;
        const int CH = hsrc >= 0 ? d.G[hsrc].N : d0, actH = hsrc >= 0 ? d.l[hsrc].act : 0;
        const _Float16* xH = xh_region(xh, hsrc >= 0 ? d.l[hsrc].xo : 0, Rp);
        const rsrc_t rH = brs(rs + (hsrc >= 0 ? (int64_t)d.l[hsrc].ri * Rp : 0), Rp * 4);   // its rstd
        // the H source rows: in flight during the LayerNorm backward below (the
        // widest stacks load them after it, for registers)
        constexpr bool PF = NT <= 6;
        u32x2 xn[TPW][NT];
        float rsn[TPW];
#pragma unroll
        for (int u = 0; u < TPW; ++u) {
            const int64_t row = rbase + IMR * u;
            rsn[u] = bld(rH, row < R ? (unsigned)(row * 4) : OOB);
        }
        if constexpr (PF) {
#pragma unroll
            for (int u = 0; u < TPW; ++u) {
                const int64_t row = rbase + IMR * u;
                load_sv<NT>(xn[u], xH, CH, Rp, row, row < R);
            }
        }
        __syncthreads();                      // previous step done with the W^T / dZ / H images and red
        if (fpend) flush_sum<NT>(red, fC, fln, fdln, fdb, fdbs);   // before this step's image barrier
        MB_STAMP(2 + 6 * step);
        if (!d.bres) {
            if (d.gimg)
                lds_copy(reinterpret_cast<char*>(wimg), d.gimg + d.gbo + 2 * G.gbw, 2 * ((p16(K) * G.bs + 7) & ~7));
            else
                stage_wt<H>(G, wimg);
        }
        float la[NT], lb[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) la[t] = lb[t] = 0.f;
        hv8<H> b[TPW][KS];
#pragma unroll
        for (int u = 0; u < TPW; ++u) {
            const int64_t row = rbase + IMR * u;
            f32x4 dz[NT];
            if (skp) {
                load_rows<NT>(dz, dout, DL, R, row);
            } else {
#pragma unroll
                for (int t = 0; t < NT; ++t) dz[t] = dh[u][t];
                if (ln) {
                    const float* gl = prm + d.l[l].bpo;
                    f32x4 xf[NT];
                    sv_f32<NT>(xc[u], xf);
                    ln_bwd<NT>(dz, xf, rsc[u], N, gl, gl + p16(N), d.l[l].act, la);
                }
            }
            if (step == 1 && u == 0) MB_STAMP(240);   // diagnostic sub-phases of step 1, first tile
            colsum<NT>(dz, N, lb);            // the bias gradient: fp32 sum of dZ (not of its bf16 image)
            if (step == 1 && u == 0) MB_STAMP(241);
            put_img<NT, IS, H>(zimg, dz, N, 128 * u + 16 * wv);
            if (step == 1 && u == 0) MB_STAMP(242);
            frags<NT, H>(dz, b[u]);
            if (step == 1 && u == 0) MB_STAMP(243);
        }
        MB_STAMP(3 + 6 * step);
        if constexpr (!PF) {
#pragma unroll
            for (int u = 0; u < TPW; ++u) {
                const int64_t row = rbase + IMR * u;
                load_sv<NT>(xn[u], xH, CH, Rp, row, row < R);
            }
        }
#pragma unroll
        for (int u = 0; u < TPW; ++u) {
            // H = act(xhat_hsrc * gamma + beta) (0 for rows past R)
            const bool rok = rbase + IMR * u < R;
            f32x4 hv[NT];
#pragma unroll
            for (int t = 0; t < NT; ++t)
                hv[t] = sv_f32(xn[u][t]) * *(const f32x4*)(gH + 16 * t + 4 * g4) +
                        *(const f32x4*)(gH + p16(CH) + 16 * t + 4 * g4);
            act_tile<NT>(hv, actH);
            if (!rok) {
#pragma unroll
                for (int t = 0; t < NT; ++t) hv[t] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
            put_img<NT, IS, H>(himg, hv, K, 128 * u + 16 * wv);
#pragma unroll
            for (int t = 0; t < NT; ++t) xc[u][t] = xn[u][t];   // the next step's LN input
            rsc[u] = rsn[u];
        }
        MB_STAMP(4 + 6 * step);
        if (!d.bres && d.gimg) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this step's W^T image
        __syncthreads();   // images (W^T, dZ, H) complete
        MB_STAMP(5 + 6 * step);
        // dH_prev = W^T dz (dz as the B operand; the W^T image rows = K features)
#pragma unroll
        for (int u = 0; u < TPW; ++u) {
            f32x4 nh[NT];
            tile_gemm<NT, KS, H>(wimg + G.bw, bs, (K + 15) >> 4, (N + 31) >> 5, b[u], nh);
            if (skp) {
#pragma unroll
                for (int t = 0; t < NT; ++t) dh[u][t] += nh[t];
            } else {
#pragma unroll
                for (int t = 0; t < NT; ++t) dh[u][t] = nh[t];
            }
        }
        // dW over the block's rows -> this workgroup's partial (db: column K, from the column sums)
        dw_img<TNS, TKS, ROWS, IS, H>(zimg, himg, N, K, pb + G.wo);
        MB_STAMP(6 + 6 * step);
        flush_write<NT>(red, la, lb, N, ln, true);
        fC = N, fln = ln, fdln = ln ? pb + d.l[l].lpo : nullptr, fdb = pb + G.wo + K, fdbs = K + 1, fpend = true;
        MB_STAMP(7 + 6 * step);
    }
    if (fpend) {
        __syncthreads();
        flush_sum<NT>(red, fC, fln, fdln, fdb, fdbs);   // red is next written after the final barrier below
    }
    // identity skip: d x0 += dout
    if (d.skip == 1) {
#pragma unroll
        for (int u = 0; u < TPW; ++u) {
            const int64_t row = rbase + IMR * u;
            f32x4 t2[NT];
            load_rows<NT>(t2, dout, DL, R, row);
#pragma unroll
            for (int t = 0; t < NT; ++t) dh[u][t] += t2[t];
        }
    }
    // input LayerNorm backward -> dx (xc holds the input LN's xhat: the last step's H source)
    float la[NT], lb[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) la[t] = lb[t] = 0.f;
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
        const int64_t row = rbase + IMR * u;
        f32x4 xf[NT];
        sv_f32<NT>(xc[u], xf);
        ln_bwd<NT>(dh[u], xf, rsc[u], d0, prm_in, prm_in + p16(d0), 0, la);   // rsc: the input LN's rstd
        store_rows<NT>(dx, dh[u], d0, R, row);
    }
    __syncthreads();
    flush_cols<NT>(red, la, lb, d0, true, pb + d.lpo0, nullptr, 0);
    MB_STAMP(255);
}
#undef MB_STAMP

// ----------------------------------------------------------- split backward
// The same backward in two kernels, so the weight gradients leave the data-gradient chain
// (tools/mlpb_phases.py, round 5: of a 64-wide step's ~10.5 us, the H image, its barrier and the
// dW MFMAs took ~3.5 us on the chain the encoders' backward waits for):
//   k_mlpb_bwdx  per GEMM step: LayerNorm backward in registers -> dZ; dZ stored as bf16 rows
//                (dz16) for k_mlpb_dw; dH = W^T dZ; bias / gamma / beta column sums of the fp32 dZ
//                (as k_mlpb_bwd).  Every W^T image resident, no dZ / H images: one barrier per
//                step (the column-sum flush, double-buffered).
//   k_mlpb_dw    per (row chunk, GEMM): dW partial = dZ^T H over the chunk, H = act(xhat gamma +
//                beta) of the GEMM's input recomputed from the saved xhat, both staged as bf16
//                row images and read as MFMA fragments with ds_read_b64_tr_b16 (rows as the
//                contraction); fixed-order sum of the chunk partials afterwards.
// dW = sum over rows of bf16(dZ) bf16(H) with fp32 accumulation, as k_mlpb_bwd (another row
// grouping: other rounding, same precision).
// (the second launch bound is waves per SIMD: two 512-thread workgroups per CU for the narrow
// stacks with 128-row blocks, whose W^T images fit 80 KB; one otherwise)
template <int NT, int TPW, typename H = __bf16>
__global__ __launch_bounds__(BT, (NT <= 4 && TPW == 1) ? 4 : 2) void k_mlpb_bwdx(const BDesc* __restrict__ dp, const float* __restrict__ dout,
                                                     const float* __restrict__ xh, const float* __restrict__ rs,
                                                     int64_t R, int64_t Rp, float* __restrict__ dx,
                                                     float* __restrict__ part, H* __restrict__ dz16) {
    const BDesc& d = *dp;
    constexpr int KS = (NT + 1) / 2;
    constexpr int ROWS = IMR * TPW;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // every W^T image at its global-image offset G.gbw, then the LN parameters
    H* wimg = reinterpret_cast<H*>(smem);
    float* prm = reinterpret_cast<float*>(smem + (d.gpo - d.gbo));   // [LN params per LN layer][input LN]
    float* red = prm + d.bprm;                                         // [2][NW][48 NT]: flushes double-buffered
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g4 = lane >> 4;
    const int L = d.L, d0 = d.d0, DL = d.G[L - 1].N;
    const int64_t rbase = (int64_t)blockIdx.x * ROWS + 16 * wv + (lane & 15);
    float* pb = part + (int64_t)blockIdx.x * d.xP;

    lds_copy(reinterpret_cast<char*>(wimg), d.gimg + d.gbo, d.gpo - d.gbo);
    lds_copy(reinterpret_cast<char*>(prm), d.gimg + d.gpo, 4 * d.bprm);
    lds_copy_wait();
    const float* prm_in = prm + d.bpin;

    f32x4 dh[TPW][NT];
    u32x2 xc[TPW][NT];
    float rsc[TPW];
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
        const int64_t row = rbase + IMR * u;
        load_rows<NT>(dh[u], dout, DL, R, row);
        rsc[u] = 0.f;
        if (d.l[L - 1].ln) {
            load_sv<NT>(xc[u], xh_region(xh, d.l[L - 1].xo, Rp), DL, Rp, row, row < R);
            rsc[u] = bld(brs(rs + (int64_t)d.l[L - 1].ri * Rp, Rp * 4), row < R ? (unsigned)(row * 4) : OOB);
        }
    }

    const int nsteps = L + (d.skip == 2 ? 1 : 0);
    for (int step = 0; step < nsteps; ++step) {
        const bool skp = step == L;
        const int l = skp ? -1 : L - 1 - step;
        const BG& G = d.G[skp ? L : l];
        const int N = G.N, K = G.K, bs = G.bs;
        const bool ln = !skp && d.l[l].ln;
        const int hsrc = skp ? -1 : l - 1;
        const int CH = hsrc >= 0 ? d.G[hsrc].N : d0;
        const _Float16* xH = xh_region(xh, hsrc >= 0 ? d.l[hsrc].xo : 0, Rp);
        const rsrc_t rH = brs(rs + (hsrc >= 0 ? (int64_t)d.l[hsrc].ri * Rp : 0), Rp * 4);
        float la[NT], lb[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) la[t] = lb[t] = 0.f;
        const int ntz = (N + 15) >> 4;
        H* zrow = dz16 + G.zo;
#pragma unroll
        for (int u = 0; u < TPW; ++u) {
            const int64_t row = rbase + IMR * u;
            f32x4 dz[NT];
            if (skp) {
                load_rows<NT>(dz, dout, DL, R, row);
            } else {
#pragma unroll
                for (int t = 0; t < NT; ++t) dz[t] = dh[u][t];
                if (ln) {
                    const float* gl = prm + d.l[l].bpo;
                    f32x4 xf[NT];
                    sv_f32<NT>(xc[u], xf);
                    ln_bwd<NT>(dz, xf, rsc[u], N, gl, gl + p16(N), d.l[l].act, la);
                }
            }
            // the next step's LayerNorm input (this GEMM's input's xhat) into the registers just
            // consumed: in flight during this step's GEMM and flush
            rsc[u] = bld(rH, row < R ? (unsigned)(row * 4) : OOB);
            load_sv<NT>(xc[u], xH, CH, Rp, row, row < R);
            colsum<NT>(dz, N, lb);
            // dZ row (bf16, 0 past N and for rows past R) for the weight-gradient kernel
            
            H* zp = zrow + row * G.zs + 4 * g4;
#pragma unroll
            for (int t = 0; t < NT; ++t)
                if (t < ntz)
                    *(hv4<H>*)(zp + 16 * t) = hv4<H>{(H)dz[t][0], (H)dz[t][1], (H)dz[t][2],
                                                      (H)dz[t][3]};
            hv8<H> b[KS];
            frags<NT, H>(dz, b);
            f32x4 nh[NT];
            tile_gemm<NT, KS, H>(wimg + G.gbw, bs, (K + 15) >> 4, (N + 31) >> 5, b, nh);
            if (skp) {
#pragma unroll
                for (int t = 0; t < NT; ++t) dh[u][t] += nh[t];
            } else {
#pragma unroll
                for (int t = 0; t < NT; ++t) dh[u][t] = nh[t];
            }
        }
        flush_cols<NT>(red + (step & 1) * (NW * 48 * NT), la, lb, N, ln, ln ? pb + d.l[l].xlpo : nullptr,
                       pb + G.xdb, 1);
    }
    if (d.skip == 1) {
#pragma unroll
        for (int u = 0; u < TPW; ++u) {
            const int64_t row = rbase + IMR * u;
            f32x4 t2[NT];
            load_rows<NT>(t2, dout, DL, R, row);
#pragma unroll
            for (int t = 0; t < NT; ++t) dh[u][t] += t2[t];
        }
    }
    float la[NT], lb[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) la[t] = lb[t] = 0.f;
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
        const int64_t row = rbase + IMR * u;
        f32x4 xf[NT];
        sv_f32<NT>(xc[u], xf);
        ln_bwd<NT>(dh[u], xf, rsc[u], d0, prm_in, prm_in + p16(d0), 0, la);
        store_rows<NT>(dx, dh[u], d0, R, row);
    }
    flush_cols<NT>(red + (nsteps & 1) * (NW * 48 * NT), la, lb, d0, true, pb + d.xlpo0, nullptr, 0);
}

// weight gradient of one GEMM over a chunk of rows: images of 64 rows (bf16 [r][col], row
// stride DZS plus 64 every 8 rows: the transposed fragment reads of mfma.hip's k_mfma_dw)
constexpr int DWROWS = 64, DZS = 160;
constexpr int DZIMG = DWROWS * DZS + (DWROWS / 8) * 64;
__device__ __forceinline__ int dz_pos(int r, int c) { return r * DZS + (r >> 3) * 64 + c; }

// 16 columns col0.. x 32 rows row0.. of a [r][col] image as an MFMA operand (rows = the
// contraction): lane 4q + p of 16-lane group g reads rows row0 + 8g + q (+4), columns col0 + 4p ..
template <typename H>
__device__ __forceinline__ hv8<H> dz_frag(const H* img, int row0, int col0) {
    typedef short v4i16 __attribute__((ext_vector_type(4)));
    typedef short v8i16 __attribute__((ext_vector_type(8)));
    const int lane = threadIdx.x & 63, g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const H* a0 = img + dz_pos(row0 + 8 * g + q, col0 + 4 * p);
    const H* a1 = img + dz_pos(row0 + 8 * g + q + 4, col0 + 4 * p);
    const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)a0);
    const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)a1);
    const v8i16 r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(hv8<H>, r);
}

// grid (row chunks, GEMMs), 256 threads; MT >= output tiles per wave (4 waves share the
// ceil(N/16) x ceil(K/16) tiles round-robin).  part: [chunk][dP], this GEMM's N x K at G.dwo.
template <int MT, typename H = __bf16>
__global__ __launch_bounds__(256) void k_mlpb_dw(const BDesc* __restrict__ dp, const H* __restrict__ dz16,
                                                 const float* __restrict__ xh, int64_t R, int64_t Rp, int chunk_rows,
                                                 float* __restrict__ part) {
    const BDesc& d = *dp;
    __shared__ __attribute__((aligned(16))) H zimg[DZIMG];
    __shared__ __attribute__((aligned(16))) H himg[DZIMG];
    const int gi = blockIdx.y;
    const BG& G = d.G[gi];
    const int N = G.N, K = G.K;
    const bool skp = gi == d.L;
    const int hsrc = skp ? -1 : gi - 1;   // this GEMM's input: layer hsrc's output, or x0 (input LN)
    const float* gam = hsrc >= 0 ? d.l[hsrc].g : d.g0;
    const float* bet = hsrc >= 0 ? d.l[hsrc].be : d.be0;
    const int actH = hsrc >= 0 ? d.l[hsrc].act : 0;
    const int kp = p16(K);                // saved-xhat row stride (floats)
    const _Float16* xH = xh_region(xh, hsrc >= 0 ? d.l[hsrc].xo : 0, Rp);
    const H* zsrc = dz16 + G.zo;
    const int zs = G.zs;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, lr = lane & 15, lc = lane >> 4;
    const int ntn = (N + 15) >> 4, ntk = (K + 15) >> 4, ntiles = ntn * ntk;
    f32x4 acc[MT];
#pragma unroll
    for (int j = 0; j < MT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int64_t Rz = (R + DWROWS - 1) / DWROWS * DWROWS;   // rows past it are all 0: skipped
    const int64_t r0 = (int64_t)blockIdx.x * chunk_rows;
    const int64_t r1 = r0 + chunk_rows < Rz ? r0 + chunk_rows : Rz;
    
    for (int64_t rb = r0; rb < r1; rb += DWROWS) {
        // dZ rows: 16-B pieces (8 bf16), zs / 8 per row; rows past R are 0 (k_mlpb_bwdx writes
        // the rows of its blocks only, not up to the padded Rp)
        const int zq = zs >> 3;
        for (int e = tid; e < DWROWS * zq; e += 256) {
            const int r = e / zq, q = e - r * zq;
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (rb + r < R) v = *(const uint4*)(zsrc + (rb + r) * zs + 8 * q);
            *(uint4*)(zimg + dz_pos(r, 8 * q)) = v;
        }
        // H rows: act(xhat gamma + beta), 0 past K and for rows past R
        const int hq = kp >> 2;
        for (int e = tid; e < DWROWS * hq; e += 256) {
            const int r = e / hq, q = e - r * hq;
            const int64_t row = rb + r;
            h16x4 v = {(_Float16)0.f, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f};
            if (row < R) v = *(const h16x4*)(xH + row * kp + 4 * q);
            float h[4] = {(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int k = 4 * q + i;
                h[i] = (row < R && k < K) ? bact(fmaf(h[i], gam[k], bet[k]), actH) : 0.f;
            }
            *(hv4<H>*)(himg + dz_pos(r, 4 * q)) = hv4<H>{(H)h[0], (H)h[1], (H)h[2], (H)h[3]};
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < DWROWS / 32; ++s) {
#pragma unroll
            for (int j = 0; j < MT; ++j) {
                const int tile = w + 4 * j;
                if (tile < ntiles) {
                    const int tn = tile / ntk, tk = tile - tn * ntk;
                    acc[j] = mfma16(dz_frag<H>(zimg, 32 * s, 16 * tn), dz_frag<H>(himg, 32 * s, 16 * tk), acc[j]);
                }
            }
        }
        __syncthreads();
    }
    // D: col (k) = lane & 15, row (n) = 4 (lane >> 4) + rr
    float* pd = part + (int64_t)blockIdx.x * d.dP + G.dwo;
#pragma unroll
    for (int j = 0; j < MT; ++j) {
        const int tile = w + 4 * j;
        if (tile >= ntiles) continue;
        const int tn = tile / ntk, tk = tile - tn * ntk;
        const int k = 16 * tk + lr;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int n = 16 * tn + 4 * lc + rr;
            if (n < N && k < K) pd[n * K + k] = acc[j][rr];
        }
    }
}

// ---------------------------------------------------------------- final sum
// one segment per dW|db slab (E = N (K + 1), K1 = K + 1) or gamma|beta pair
// (E = 2N, K1 = 0), summed over the nblk workgroup partials in fixed order
struct SumSeg {
    int E, N, K1, src;
    float* da;
    float* db;
};
constexpr int MAXSEG = MAXG + MAXL + 1;
struct SumArgs {
    int nseg, P;
    SumSeg s[MAXSEG];
};

__global__ __launch_bounds__(256) void k_mlpb_sum(SumArgs sa, const float* __restrict__ part, int nblk, int accumulate) {
    // 64 outputs per workgroup; wave w sums partials w, w + 4, w + 8, ... in sequence
    // (coalesced 256-byte rows, up to 64 loads in flight), then (w0 + w1) + (w2 + w3)
    __shared__ float red[4][64];
    const SumSeg& sg = sa.s[blockIdx.y];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int E = sg.E, P = sa.P;
    if ((int64_t)blockIdx.x * 64 >= E) return;
    const float* src = part + sg.src;
    const int i = blockIdx.x * 64 + lane;
    float a = 0.f;
    if (i < E) {
        const float* q = src + i;
        int b = w;
        // 64 loads in flight while 64 partials remain for this wave (one batch at 256 blocks), then
        // 16, then one at a time: the same sequence of b, so the same sums as 16 at a time
        for (; b + 4 * 63 < nblk; b += 256) {
            float v[64];
#pragma unroll
            for (int m = 0; m < 64; ++m) v[m] = q[(int64_t)(b + 4 * m) * P];
#pragma unroll
            for (int m = 0; m < 64; ++m) a += v[m];
        }
        for (; b + 60 < nblk; b += 64) {
            float v[16];
#pragma unroll
            for (int m = 0; m < 16; ++m) v[m] = q[(int64_t)(b + 4 * m) * P];
#pragma unroll
            for (int m = 0; m < 16; ++m) a += v[m];
        }
        for (; b < nblk; b += 4) a += q[(int64_t)b * P];
    }
    red[w][lane] = a;
    __syncthreads();
    if (w != 0 || i >= E) return;
    const float t = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    float* dst;
    if (sg.K1 < 0) {                     // a plain vector (split backward: dW N x K, or a bias)
        dst = sg.da ? sg.da + i : nullptr;
    } else if (sg.K1) {
        const int n = i / sg.K1, k = i - n * sg.K1;
        dst = k < sg.K1 - 1 ? (sg.da ? sg.da + (int64_t)n * (sg.K1 - 1) + k : nullptr) : (sg.db ? sg.db + n : nullptr);
    } else {
        dst = i < sg.N ? (sg.da ? sg.da + i : nullptr) : (sg.db ? sg.db + (i - sg.N) : nullptr);
    }
    if (dst) *dst = accumulate ? *dst + t : t;
}

// ---------------------------------------------------------------- host side
inline int h16(int n) { return (n + 15) & ~15; }
inline int h32(int n) { return (n + 31) & ~31; }

struct BPlan {
    BDesc d;
    int nt, tpw;
    int xtpw, mt;                // split backward: k_mlpb_bwdx tiles per wave; k_mlpb_dw tiles per wave bound
    int64_t xnblk, dz_elems;     // ... k_mlpb_bwdx workgroups; bf16 elements of the dZ rows
    int dw_rows, dw_chunks;      // ... k_mlpb_dw rows per chunk and chunks
    int occ;                     // backward workgroups per CU the launch is built for (1, or 2: 128-row blocks)
    int64_t Rp, xh_floats, rs_floats, nblk;
    int gbytes;                  // global image bytes
    int prep_x, prep_y;          // k_mlpb_prep grid
};

int make_bplan(BPlan& p, int n_layers, const int* dims, const int* layer_ln, const int* layer_act, int skip, float eps,
               const float* const* params, int64_t R, const char* who) {
    VT_CHECK_ARG(n_layers >= 1 && n_layers <= MAXL, "%s: n_layers %d not in [1, %d]", who, n_layers, MAXL);
    VT_CHECK_ARG(skip >= 0 && skip <= 2, "%s: skip %d", who, skip);
    VT_CHECK_ARG(R >= 1, "%s: rows %lld", who, (long long)R);
    BDesc& d = p.d;
    d = BDesc{};
    d.L = n_layers;
    d.d0 = dims[0];
    d.skip = skip;
    d.eps = eps;
    d.nG = n_layers + (skip == 2 ? 1 : 0);
    int wmax = dims[0], n_ln = 0, xo = h16(dims[0]), lnp = 0;
    for (int l = 0; l < n_layers; ++l) {
        const int K = dims[l], N = dims[l + 1];
        VT_CHECK_ARG(K >= 1 && N >= 1 && K <= VT_MLP_MAX_WIDTH && N <= VT_MLP_MAX_WIDTH,
                     "%s: layer %d width %d -> %d outside [1, %d]", who, l, K, N, VT_MLP_MAX_WIDTH);
        VT_CHECK_ARG(layer_ln[l] || l == n_layers - 1, "%s: hidden layer %d without LayerNorm", who, l);
        VT_CHECK_ARG(layer_ln[l] || layer_act[l] == 0, "%s: activation without LayerNorm (layer %d)", who, l);
        VT_CHECK_ARG(layer_act[l] >= 0 && layer_act[l] <= 3, "%s: act %d", who, layer_act[l]);
        BL& ly = d.l[l];
        ly.ln = layer_ln[l] ? 1 : 0;
        ly.act = layer_act[l];
        ly.g = params[4 + 4 * l];
        ly.be = params[5 + 4 * l];
        BG& G = d.G[l];
        G.K = K;
        G.N = N;
        G.W = params[2 + 4 * l];
        G.b = params[3 + 4 * l];
        VT_CHECK_ARG(G.W && (!ly.ln || (ly.g && ly.be)), "%s: missing parameter of layer %d", who, l);
        wmax = N > wmax ? N : wmax;
        if (ly.ln) {
            ly.xo = xo;
            ly.ri = 1 + n_ln;
            ++n_ln;
            xo += h16(N);
        } else {
            ly.xo = ly.ri = -1;
        }
    }
    d.g0 = params[0];
    d.be0 = params[1];
    VT_CHECK_ARG(d.g0 && d.be0, "%s: missing input LayerNorm parameters", who);
    VT_CHECK_ARG(skip != 1 || dims[0] == dims[n_layers], "%s: identity skip needs in == out width", who);
    if (skip == 2) {
        BG& G = d.G[n_layers];
        G.K = dims[0];
        G.N = dims[n_layers];
        G.W = params[2 + 4 * n_layers];
        G.b = params[3 + 4 * n_layers];
        VT_CHECK_ARG(G.W, "%s: projection skip without weight", who);
    }
    // forward LDS: images, then [bias, gamma, beta] per GEMM, then the input LN
    int off = 0, po = 0, bw = 0, bwtot = 0, bh = 0, bz = 0;
    for (int g = 0; g < d.nG; ++g) {
        BG& G = d.G[g];
        G.fo = off;
        G.fs = h32(G.K) + 16;
        off += h16(G.N) * G.fs;
        off = (off + 7) & ~7;                 // 16-B aligned images
        G.po = po;
        po += 3 * h16(G.N);
        G.bs = h32(G.N) + 16;
        const int e = (h16(G.K) * G.bs + 7) & ~7;
        G.bw = G.gbw = bwtot;
        bwtot += e;
        bw = e > bw ? e : bw;
        bh = h16(G.K) > bh ? h16(G.K) : bh;
        bz = h16(G.N) > bz ? h16(G.N) : bz;
    }
    d.fimg = 2 * off;
    d.pin = po;
    d.fbytes = (d.fimg + 4 * (po + 2 * h16(dims[0])) + 15) & ~15;   // 16-B multiple: copied by LDS-DMA
    const int ntw = (wmax + 15) / 16;
    p.nt = ntw <= 2 ? 2 : ntw <= 4 ? 4 : ntw <= 6 ? 6 : 9;
    d.bhrows = bh;
    d.bzrows = bz;
    int bprm = 0;
    for (int l = 0; l < n_layers; ++l) {
        d.l[l].bpo = d.l[l].ln ? bprm : -1;
        if (d.l[l].ln) bprm += 2 * h16(d.G[l].N);
    }
    d.bpin = bprm;
    bprm += 2 * h16(dims[0]);
    d.bprm = bprm;
    static int tpw_env = -1;  // VAETEB_MLPB_TPW: 1 / 2 force the backward block (tuning experiments)
    if (tpw_env < 0) {
        const char* e = getenv("VAETEB_MLPB_TPW");
        tpw_env = e && (e[0] == '1' || e[0] == '2') ? e[0] - '0' : 0;
    }
    // VAETEB_MLPB_OCC=2 (tuning option, off by default): two 128-row workgroups per CU
    // (<= 128 VGPRs and <= 80 KB of LDS each, W^T images streamed per GEMM when they do not
    // fit beside the images) instead of one 256-row workgroup, for widths <= 32 (isolated
    // kernel span 213 -> 174 us on the 33-GEMM stacks, but the replayed step 8.19-8.22 vs
    // 8.16-8.18 ms: DESIGN.md §9); =3 also at width 64, where the 128-VGPR cap spills
    // (74 -> 104 us)
    static int occ_env = -1;
    if (occ_env < 0) {
        const char* e = getenv("VAETEB_MLPB_OCC");
        occ_env = e && (e[0] == '2' || e[0] == '3') ? e[0] - '0' : 1;
    }
    const bool occ2 = !tpw_env && (occ_env == 3 ? p.nt <= 4 : occ_env == 2 && p.nt == 2);
    for (int occ = occ2 ? 2 : 1;; --occ) {
        const int cap = 160 * 1024 / occ;
        p.occ = occ;
        p.tpw = occ == 2 ? 1 : p.nt >= 6 ? 1 : (tpw_env ? tpw_env : 2);
        const int ims = IMR * p.tpw + 16;
        const int rest = 2 * (bz + bh) * ims + 4 * (bprm + NW * 48 * p.nt);
        d.bres = 2 * bwtot + rest <= cap;  // all W^T images resident when they fit
        for (int g = 0, o = 0; g < d.nG; ++g) {
            d.G[g].bw = d.bres ? o : 0;
            o += (h16(d.G[g].K) * d.G[g].bs + 7) & ~7;
        }
        d.bwimg = d.bres ? bwtot : bw;
        d.bbytes = 2 * d.bwimg + rest;
        if (d.bbytes <= cap || occ == 1) break;
    }
    // global image (k_mlpb_prep): forward LDS image | W^T images | backward params
    d.gbo = (d.fbytes + 15) & ~15;
    d.gpo = d.gbo + ((2 * bwtot + 15) & ~15);
    p.gbytes = d.gpo + ((4 * bprm + 15) & ~15);
    // partials: dW|db of every GEMM, then gamma|beta of every LN and the input LN
    int P = 0;
    for (int g = 0; g < d.nG; ++g) {
        d.G[g].wo = P;
        P += d.G[g].N * (d.G[g].K + 1);
    }
    for (int l = 0; l < n_layers; ++l) {
        d.l[l].lpo = d.l[l].ln ? P : -1;
        if (d.l[l].ln) P += 2 * d.G[l].N;
    }
    d.lpo0 = P;
    P += 2 * dims[0];
    d.P = P;
    (void)lnp;
    const int blk = IMR * p.tpw;
    p.Rp = (R + 2 * IMR - 1) / (2 * IMR) * (2 * IMR);   // the saved state is padded for either block size
    p.nblk = (R + blk - 1) / blk;
    p.xh_floats = ((int64_t)xo * p.Rp + 1) / 2;   // fp16 saved state
    p.rs_floats = (int64_t)(1 + n_ln) * p.Rp;
    // split backward (k_mlpb_bwdx + k_mlpb_dw)
    int xP = 0;
    for (int g = 0; g < d.nG; ++g) {
        d.G[g].xdb = xP;
        xP += d.G[g].N;
    }
    for (int l = 0; l < n_layers; ++l) {
        d.l[l].xlpo = d.l[l].ln ? xP : -1;
        if (d.l[l].ln) xP += 2 * d.G[l].N;
    }
    d.xlpo0 = xP;
    xP += 2 * dims[0];
    d.xP = xP;
    int dP = 0;
    int64_t zo = 0;
    for (int g = 0; g < d.nG; ++g) {
        BG& G = d.G[g];
        G.dwo = dP;
        dP += G.N * G.K;
        G.zs = h16(G.N);
        G.zo = zo;
        zo += (int64_t)G.zs * p.Rp;
    }
    d.dP = dP;
    p.dz_elems = zo;
    const int xbytes = (d.gpo - d.gbo) + 4 * (bprm + 2 * NW * 48 * p.nt);
    d.xbytes = xbytes <= 160 * 1024 ? xbytes : 0;
    // 128-row blocks, two workgroups per CU, when they fit 80 KB; else 256-row blocks (one per CU);
    // the wide stacks keep 128 rows (their registers)
    p.xtpw = (xbytes <= 80 * 1024 || p.nt >= 6) ? 1 : 2;
    p.xnblk = (R + IMR * p.xtpw - 1) / (IMR * p.xtpw);
    p.mt = p.nt == 2 ? 1 : p.nt == 4 ? 4 : p.nt == 6 ? 9 : 21;
    p.dw_rows = 1024;
    p.dw_chunks = (int)((p.Rp + p.dw_rows - 1) / p.dw_rows);
    VT_CHECK_ARG(d.fbytes <= 160 * 1024, "%s: weights need %d bytes of LDS (> 160 KiB)", who, d.fbytes);
    VT_CHECK_ARG(d.bbytes <= 160 * 1024, "%s: backward needs %d bytes of LDS (> 160 KiB)", who, d.bbytes);
    return VT_OK;
}

unsigned long long* g_mlpb_stamps = nullptr;  // diagnostic (vt_resmlp_bf16_set_stamps)

int n_fwd_blocks(int64_t R) {
    static int ncu = 0;
    if (!ncu) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount,
                                                                      dev) != hipSuccess || ncu <= 0)
            ncu = 256;
    }
    const int64_t tiles = (R + 15) / 16, need = (tiles + NW - 1) / NW;
    return (int)(need < ncu ? need : ncu);
}

// Device copies of the descriptors, keyed by content: a plan's descriptor is
// uploaded once (stream-ordered copy from pinned host memory, so it is also
// valid under hipGraph capture) and reused by every later launch.
const BDesc* device_desc(const BDesc& d, hipStream_t st) {
    struct Entry {
        BDesc* host;
        BDesc* dev;
    };
    static std::unordered_map<uint64_t, std::vector<Entry>> cache;
    static std::mutex mu;
    const unsigned char* b = reinterpret_cast<const unsigned char*>(&d);
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < sizeof(BDesc); ++i) h = (h ^ b[i]) * 1099511628211ull;
    std::lock_guard<std::mutex> lk(mu);
    auto& v = cache[h];
    for (const Entry& e : v)
        if (!memcmp(e.host, &d, sizeof(BDesc))) return e.dev;
    Entry e{nullptr, nullptr};
    if (hipHostMalloc(reinterpret_cast<void**>(&e.host), sizeof(BDesc), 0) != hipSuccess) return nullptr;
    if (hipMalloc(reinterpret_cast<void**>(&e.dev), sizeof(BDesc)) != hipSuccess) return nullptr;
    memcpy(e.host, &d, sizeof(BDesc));
    if (hipMemcpyAsync(e.dev, e.host, sizeof(BDesc), hipMemcpyHostToDevice, st) != hipSuccess) return nullptr;
    v.push_back(e);
    return e.dev;
}

// every kernel may use the whole LDS: set once per instantiation
template <typename Kern>
void set_lds(Kern k, int) {
    static bool done = false;
    if (!done) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        done = true;
    }
}

// Plans (host descriptor + device copy) cached by their arguments: the training
// step calls every stack with the same widths, parameter pointers and rows.
struct PlanEntry {
    std::vector<int64_t> key;
    BPlan plan;
    const BDesc* dev;
};

int get_plan(const BPlan*& out, const BDesc*& dev, int n_layers, const int* dims, const int* layer_ln,
             const int* layer_act, int skip, float eps, const float* const* params, int64_t R, hipStream_t st,
             const char* who) {
    static std::unordered_map<uint64_t, std::vector<PlanEntry>> cache;
    static std::mutex mu;
    VT_CHECK_ARG(n_layers >= 1 && n_layers <= MAXL, "%s: n_layers %d not in [1, %d]", who, n_layers, MAXL);
    std::vector<int64_t> key;
    key.reserve(8 + 3 * n_layers + 4 * n_layers + 4);
    key.push_back(n_layers);
    key.push_back(skip);
    key.push_back(R);
    key.push_back(__builtin_bit_cast(int, eps));
    for (int i = 0; i <= n_layers; ++i) key.push_back(dims[i]);
    for (int i = 0; i < n_layers; ++i) key.push_back(layer_ln[i] * 16 + layer_act[i]);
    for (int i = 0; i < 4 * n_layers + 4; ++i) key.push_back(reinterpret_cast<int64_t>(params[i]));
    uint64_t h = 1469598103934665603ull;
    for (int64_t v : key) h = (h ^ (uint64_t)v) * 1099511628211ull;
    std::lock_guard<std::mutex> lk(mu);
    auto& bucket = cache[h];
    for (const PlanEntry& e : bucket)
        if (e.key == key) {
            out = &e.plan;
            dev = e.dev;
            return VT_OK;
        }
    PlanEntry e;
    const int rc = make_bplan(e.plan, n_layers, dims, layer_ln, layer_act, skip, eps, params, R, who);
    if (rc) return rc;
    {
        BPlan& p = e.plan;
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        VT_CHECK_ARG(hipStreamIsCapturing(st, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone,
                     "%s: new stack shape under stream capture (run one eager step first)", who);
        VT_CHECK_ARG(hipMalloc(reinterpret_cast<void**>(&p.d.gimg), p.gbytes) == hipSuccess,
                     "%s: global image allocation (%d bytes)", who, p.gbytes);
        int emax = p.d.pin + 2 * h16(dims[0]);
        emax = p.d.bprm > emax ? p.d.bprm : emax;
        for (int g = 0; g < p.d.nG; ++g) {
            const BG& G = p.d.G[g];
            emax = h16(G.N) * G.fs > emax ? h16(G.N) * G.fs : emax;
            emax = h16(G.K) * G.bs > emax ? h16(G.K) * G.bs : emax;
        }
        p.prep_x = (emax + 255) / 256;
        p.prep_y = 2 * p.d.nG + 2;
    }
    e.dev = device_desc(e.plan.d, st);
    VT_CHECK_ARG(e.dev, "%s: descriptor upload failed", who);
    e.key = std::move(key);
    bucket.push_back(std::move(e));
    out = &bucket.back().plan;
    dev = bucket.back().dev;
    return VT_OK;
}

}  // namespace
}  // namespace vt

using namespace vt;

extern "C" {

int vt_resmlp_bf16_sizes(int n_layers, const int* dims, const int* layer_ln, const int* layer_act, int skip,
                         int64_t rows, int64_t* sizes) {
    const float* dummy[4 * MAXL + 4];
    for (int i = 0; i < 4 * MAXL + 4; ++i) dummy[i] = reinterpret_cast<const float*>(16);
    BPlan p;
    const int rc = make_bplan(p, n_layers, dims, layer_ln, layer_act, skip, 1e-5f, dummy, rows, "vt_resmlp_bf16_sizes");
    if (rc) return rc;
    sizes[0] = p.xh_floats;
    sizes[1] = p.rs_floats;
    sizes[2] = p.nblk * p.d.P;
    return VT_OK;
}

int vt_resmlp_bf16_plan(int n_layers, const int* dims, const int* layer_ln, const int* layer_act, int skip, float eps,
                        const float* const* params, int64_t rows, int64_t* handle, void* stream) {
    const BPlan* pp;
    const BDesc* ddev;
    const int rc = get_plan(pp, ddev, n_layers, dims, layer_ln, layer_act, skip, eps, params, rows, S(stream),
                            "vt_resmlp_bf16_plan");
    if (rc) return rc;
    VT_CHECK_ARG(handle, "vt_resmlp_bf16_plan: null handle");
    // a stable copy per cached plan (the plan cache's vectors may move their entries); the image
    // buffer it points at is the plan's own
    static std::unordered_map<const BPlan*, std::unique_ptr<BPlan>> handles;
    static std::mutex mu;
    std::lock_guard<std::mutex> lk(mu);
    auto& h = handles[pp];
    if (!h) h.reset(new BPlan(*pp));
    *handle = reinterpret_cast<int64_t>(h.get());
    return VT_OK;
}

int vt_resmlp_bf16_prep_batch(int n, const int64_t* handles, void* stream) {
    VT_CHECK_ARG(n >= 1 && n <= PREP_BATCH && handles, "vt_resmlp_bf16_prep_batch: 1..%d plans", PREP_BATCH);
    PrepBatch pb{};
    pb.n = n;
    int xmax = 0;
    for (int i = 0; i < n; ++i) {
        const BPlan* p = reinterpret_cast<const BPlan*>(handles[i]);
        VT_CHECK_ARG(p && p->d.gimg, "vt_resmlp_bf16_prep_batch: plan %d", i);
        pb.d[i] = device_desc(p->d, S(stream));
        VT_CHECK_ARG(pb.d[i], "vt_resmlp_bf16_prep_batch: descriptor upload failed");
        pb.y0[i + 1] = pb.y0[i] + p->prep_y;
        pb.x[i] = p->prep_x;
        xmax = p->prep_x > xmax ? p->prep_x : xmax;
    }
    VT_H16(hipLaunchKernelGGL(k_mlpb_prep_batch<H>, dim3((unsigned)xmax, (unsigned)pb.y0[n]), dim3(256), 0, S(stream),
                              pb));
    VT_LAUNCH_CHECK("vt_resmlp_bf16_prep_batch");
    return VT_OK;
}

static int resmlp_fwd(int n_layers, const int* dims, const int* layer_ln, const int* layer_act, int skip, float eps,
                      const float* const* params, const float* x, int64_t rows, float* out, float* xhat, float* rstd,
                      hipStream_t st, bool prep, const char* who) {
    const BPlan* pp;
    const BDesc* ddev;
    const int rc = get_plan(pp, ddev, n_layers, dims, layer_ln, layer_act, skip, eps, params, rows, st, who);
    if (rc) return rc;
    const BPlan& p = *pp;
    VT_CHECK_ARG(x && out && xhat && rstd, "%s: null buffer", who);
    // the weight images of this step (read again by the backward of this forward); prepared already
    // (vt_resmlp_bf16_prep_batch, in the current format) when prep is false
    if (prep)
        VT_H16(hipLaunchKernelGGL(k_mlpb_prep<H>, dim3((unsigned)p.prep_x, (unsigned)p.prep_y), dim3(256), 0, st,
                                  ddev));
    const dim3 grid((unsigned)n_fwd_blocks(rows));
    const bool id = skip == 1;
    switch (p.nt * 2 + (id ? 1 : 0)) {
#define VT_MBF(NTV, IDV)                                                                                   \
    case NTV * 2 + IDV:                                                                                    \
        VT_H16(set_lds(k_mlpb_fwd<NTV, IDV, H>, p.d.fbytes);                                              \
               hipLaunchKernelGGL((k_mlpb_fwd<NTV, IDV, H>), grid, dim3(BT), p.d.fbytes, st, ddev, x, rows, out, \
                                  xhat, rstd, p.Rp));                                                       \
        break;
        VT_MBF(2, 0) VT_MBF(2, 1) VT_MBF(4, 0) VT_MBF(4, 1) VT_MBF(6, 0) VT_MBF(6, 1) VT_MBF(9, 0)
        default: VT_MBF(9, 1)
#undef VT_MBF
    }
    VT_LAUNCH_CHECK(who);
    return VT_OK;
}

int vt_resmlp_bf16_fwd(int n_layers, const int* dims, const int* layer_ln, const int* layer_act, int skip, float eps,
                       const float* const* params, const float* x, int64_t rows, float* out, float* xhat, float* rstd,
                       void* stream) {
    return resmlp_fwd(n_layers, dims, layer_ln, layer_act, skip, eps, params, x, rows, out, xhat, rstd, S(stream), true,
                      "vt_resmlp_bf16_fwd");
}

int vt_resmlp_bf16_fwd_prepped(int n_layers, const int* dims, const int* layer_ln, const int* layer_act, int skip,
                               float eps, const float* const* params, const float* x, int64_t rows, float* out,
                               float* xhat, float* rstd, void* stream) {
    return resmlp_fwd(n_layers, dims, layer_ln, layer_act, skip, eps, params, x, rows, out, xhat, rstd, S(stream),
                      false, "vt_resmlp_bf16_fwd_prepped");
}

int vt_resmlp_bf16_bwd(int n_layers, const int* dims, const int* layer_ln, const int* layer_act, int skip, float eps,
                       const float* const* params, const float* dout, const float* xhat, const float* rstd,
                       int64_t rows, float* dx, float* const* grads, int accumulate, float* ws, int64_t ws_floats,
                       void* stream) {
    hipStream_t st = S(stream);
    const BPlan* pp;
    const BDesc* ddev;
    const int rc = get_plan(pp, ddev, n_layers, dims, layer_ln, layer_act, skip, eps, params, rows, st,
                            "vt_resmlp_bf16_bwd");
    if (rc) return rc;
    const BPlan& p = *pp;
    VT_CHECK_ARG(dout && xhat && rstd && dx && grads, "vt_resmlp_bf16_bwd: null buffer");
    VT_CHECK_ARG(ws && ws_floats >= p.nblk * p.d.P, "vt_resmlp_bf16_bwd: workspace %lld floats < %lld",
                 (long long)ws_floats, (long long)(p.nblk * p.d.P));
    SumArgs sa{};
    sa.P = p.d.P;
    int emax = 0;
    auto add = [&](int E, int N, int K1, int src, float* da, float* db) {
        if (!da && !db) return;
        sa.s[sa.nseg++] = SumSeg{E, N, K1, src, da, db};
        emax = E > emax ? E : emax;
    };
    for (int q = 0; q < p.d.nG; ++q) {
        const int gi = q < n_layers ? 2 + 4 * q : 2 + 4 * n_layers;
        add(p.d.G[q].N * (p.d.G[q].K + 1), p.d.G[q].N, p.d.G[q].K + 1, p.d.G[q].wo, grads[gi], grads[gi + 1]);
    }
    for (int l = 0; l < n_layers; ++l)
        if (p.d.l[l].ln) add(2 * p.d.G[l].N, p.d.G[l].N, 0, p.d.l[l].lpo, grads[4 + 4 * l], grads[5 + 4 * l]);
    add(2 * dims[0], dims[0], 0, p.d.lpo0, grads[0], grads[1]);
    const dim3 grid((unsigned)p.nblk);
#define VT_MBB(NTV, TPWV, OCCV)                                                                                  \
    if (p.nt == NTV && p.tpw == TPWV && p.occ == OCCV) {                                                           \
        VT_H16(set_lds(k_mlpb_bwd<NTV, TPWV, OCCV, H>, p.d.bbytes);                                                \
               hipLaunchKernelGGL((k_mlpb_bwd<NTV, TPWV, OCCV, H>), grid, dim3(BT), p.d.bbytes, st, ddev, dout, xhat,  \
                                  rstd, rows, p.Rp, dx, ws, g_mlpb_stamps));                                         \
    }
    VT_MBB(2, 2, 1) VT_MBB(4, 2, 1) VT_MBB(2, 1, 1) VT_MBB(4, 1, 1) VT_MBB(6, 1, 1) VT_MBB(9, 1, 1)
    VT_MBB(2, 1, 2) VT_MBB(4, 1, 2)
#undef VT_MBB
    if (sa.nseg) {
        const dim3 gs((unsigned)((emax + 63) / 64), (unsigned)sa.nseg);
        hipLaunchKernelGGL(k_mlpb_sum, gs, dim3(256), 0, st, sa, ws, (int)p.nblk, accumulate);
    }
    VT_LAUNCH_CHECK("vt_resmlp_bf16_bwd");
    return VT_OK;
}

int vt_resmlp_bf16_split_sizes(int n_layers, const int* dims, const int* layer_ln, const int* layer_act, int skip,
                               int64_t rows, int64_t* sizes) {
    const float* dummy[4 * MAXL + 4];
    for (int i = 0; i < 4 * MAXL + 4; ++i) dummy[i] = reinterpret_cast<const float*>(16);
    BPlan p;
    const int rc = make_bplan(p, n_layers, dims, layer_ln, layer_act, skip, 1e-5f, dummy, rows,
                              "vt_resmlp_bf16_split_sizes");
    if (rc) return rc;
    sizes[0] = p.dz_elems;
    sizes[1] = p.xnblk * p.d.xP;
    sizes[2] = (int64_t)p.dw_chunks * p.d.dP;
    sizes[3] = p.d.xbytes > 0 ? 1 : 0;
    return VT_OK;
}

static void sum_launch(const SumArgs& sa, int emax, const float* part, int nblk, int accumulate, hipStream_t st) {
    if (!sa.nseg) return;
    const dim3 gs((unsigned)((emax + 63) / 64), (unsigned)sa.nseg);
    hipLaunchKernelGGL(k_mlpb_sum, gs, dim3(256), 0, st, sa, part, nblk, accumulate);
}

int vt_resmlp_bf16_bwd_data(int n_layers, const int* dims, const int* layer_ln, const int* layer_act, int skip,
                            float eps, const float* const* params, const float* dout, const float* xhat,
                            const float* rstd, int64_t rows, float* dx, float* const* grads, int accumulate,
                            void* dz16, float* ws, int64_t ws_floats, void* stream) {
    hipStream_t st = S(stream);
    const BPlan* pp;
    const BDesc* ddev;
    const int rc = get_plan(pp, ddev, n_layers, dims, layer_ln, layer_act, skip, eps, params, rows, st,
                            "vt_resmlp_bf16_bwd_data");
    if (rc) return rc;
    const BPlan& p = *pp;
    VT_CHECK_ARG(p.d.xbytes > 0, "vt_resmlp_bf16_bwd_data: the W^T images do not fit in LDS (use vt_resmlp_bf16_bwd)");
    VT_CHECK_ARG(!h16_format(), "vt_resmlp_bf16_bwd_data: the split backward has no fp16 form (use vt_resmlp_bf16_bwd)");
    VT_CHECK_ARG(dout && xhat && rstd && dx && grads && dz16, "vt_resmlp_bf16_bwd_data: null buffer");
    VT_CHECK_ARG(ws && ws_floats >= p.xnblk * p.d.xP, "vt_resmlp_bf16_bwd_data: workspace %lld floats < %lld",
                 (long long)ws_floats, (long long)(p.xnblk * p.d.xP));
    SumArgs sa{};
    sa.P = p.d.xP;
    int emax = 0;
    auto add = [&](int E, int N, int K1, int src, float* da, float* db) {
        if (!da && !db) return;
        sa.s[sa.nseg++] = SumSeg{E, N, K1, src, da, db};
        emax = E > emax ? E : emax;
    };
    for (int q = 0; q < p.d.nG; ++q) {   // biases
        const int gi = q < n_layers ? 2 + 4 * q : 2 + 4 * n_layers;
        add(p.d.G[q].N, p.d.G[q].N, -1, p.d.G[q].xdb, grads[gi + 1], nullptr);
    }
    for (int l = 0; l < n_layers; ++l)
        if (p.d.l[l].ln) add(2 * p.d.G[l].N, p.d.G[l].N, 0, p.d.l[l].xlpo, grads[4 + 4 * l], grads[5 + 4 * l]);
    add(2 * dims[0], dims[0], 0, p.d.xlpo0, grads[0], grads[1]);
    const dim3 grid((unsigned)p.xnblk);
    __bf16* z = reinterpret_cast<__bf16*>(dz16);
#define VT_MBX(NTV, TPWV)                                                                                       \
    if (p.nt == NTV && p.xtpw == TPWV) {                                                                          \
        set_lds(k_mlpb_bwdx<NTV, TPWV, __bf16>, p.d.xbytes);                                                              \
        hipLaunchKernelGGL((k_mlpb_bwdx<NTV, TPWV, __bf16>), grid, dim3(BT), p.d.xbytes, st, ddev, dout, xhat, rstd, rows, \
                           p.Rp, dx, ws, z);                                                                      \
    }
    VT_MBX(2, 1) VT_MBX(2, 2) VT_MBX(4, 1) VT_MBX(4, 2) VT_MBX(6, 1) VT_MBX(9, 1)
#undef VT_MBX
    sum_launch(sa, emax, ws, (int)p.xnblk, accumulate, st);
    VT_LAUNCH_CHECK("vt_resmlp_bf16_bwd_data");
    return VT_OK;
}

int vt_resmlp_bf16_bwd_weight(int n_layers, const int* dims, const int* layer_ln, const int* layer_act, int skip,
                              float eps, const float* const* params, const float* xhat, const void* dz16,
                              int64_t rows, float* const* grads, int accumulate, float* ws, int64_t ws_floats,
                              void* stream) {
    hipStream_t st = S(stream);
    const BPlan* pp;
    const BDesc* ddev;
    const int rc = get_plan(pp, ddev, n_layers, dims, layer_ln, layer_act, skip, eps, params, rows, st,
                            "vt_resmlp_bf16_bwd_weight");
    if (rc) return rc;
    const BPlan& p = *pp;
    VT_CHECK_ARG(p.d.xbytes > 0, "vt_resmlp_bf16_bwd_weight: no split plan for this stack");
    VT_CHECK_ARG(!h16_format(), "vt_resmlp_bf16_bwd_weight: the split backward has no fp16 form");
    VT_CHECK_ARG(xhat && dz16 && grads, "vt_resmlp_bf16_bwd_weight: null buffer");
    VT_CHECK_ARG(ws && ws_floats >= (int64_t)p.dw_chunks * p.d.dP,
                 "vt_resmlp_bf16_bwd_weight: workspace %lld floats < %lld", (long long)ws_floats,
                 (long long)p.dw_chunks * p.d.dP);
    SumArgs sa{};
    sa.P = p.d.dP;
    int emax = 0;
    for (int q = 0; q < p.d.nG; ++q) {
        const int gi = q < n_layers ? 2 + 4 * q : 2 + 4 * n_layers;
        if (!grads[gi]) continue;
        const int E = p.d.G[q].N * p.d.G[q].K;
        sa.s[sa.nseg++] = SumSeg{E, p.d.G[q].N, -1, p.d.G[q].dwo, grads[gi], nullptr};
        emax = E > emax ? E : emax;
    }
    const dim3 grid((unsigned)p.dw_chunks, (unsigned)p.d.nG);
    const __bf16* z = reinterpret_cast<const __bf16*>(dz16);
    switch (p.mt) {
        case 1: hipLaunchKernelGGL((k_mlpb_dw<1, __bf16>), grid, dim3(256), 0, st, ddev, z, xhat, rows, p.Rp, p.dw_rows, ws); break;
        case 4: hipLaunchKernelGGL((k_mlpb_dw<4, __bf16>), grid, dim3(256), 0, st, ddev, z, xhat, rows, p.Rp, p.dw_rows, ws); break;
        case 9: hipLaunchKernelGGL((k_mlpb_dw<9, __bf16>), grid, dim3(256), 0, st, ddev, z, xhat, rows, p.Rp, p.dw_rows, ws); break;
        default: hipLaunchKernelGGL((k_mlpb_dw<21, __bf16>), grid, dim3(256), 0, st, ddev, z, xhat, rows, p.Rp, p.dw_rows, ws); break;
    }
    sum_launch(sa, emax, ws, p.dw_chunks, accumulate, st);
    VT_LAUNCH_CHECK("vt_resmlp_bf16_bwd_weight");
    return VT_OK;
}

// Diagnostic: while buf != NULL, backward launches stamp their phase boundaries
// (128 uint64 per workgroup, k_mlpb_bwd's MB_STAMP points) into buf.
int vt_resmlp_bf16_set_stamps(void* buf) {
    g_mlpb_stamps = (unsigned long long*)buf;
    return VT_OK;
}

}  // extern "C"
