// Flat-buffer optimiser step: gradient L2 norm + clip coefficient + AdamW
// (SURVEY.md §8(a) a18).  All parameters, gradients and Adam moments live in
// single contiguous fp32 buffers (per-parameter tensors are views), so the
// step is three launches over one stream of memory instead of ~550 small ones.
//   clip_grad_norm_  : coef = min(max_norm / (||g|| + 1e-6), 1)
//                      (torch.nn.utils.clip_grad_norm_, as called at
//                       ref/model/graph_model.py:724 and Lightning's
//                       gradient_clip_val=0.5, ref/model/graph_model.py:511)
//   AdamW            : torch.optim.AdamW single-tensor update order, with the
//                      hyper-parameters of ref/model/graph_model.py:654-660.
//   dynamic loss scale (fp16 operands, round 6): torch.amp.GradScaler's unscale_ + inf check
//                      + step skip + update (ref/model/graph_model.py:670,718-726), on device
//                      state, no host sync (vt_grad_norm_clip_scaled, vt_adamw_step_dev*_skip).
#include <math.h>
#include <stdlib.h>

#include "h16.h"

namespace vt {

static constexpr int OPT_THREADS = 256;
static constexpr int NORM_BLOCKS = 1024;

// Sum of squares in double: each thread squares in fp32 (exact products of fp32 values need
// 48 bits; the fp32 rounding of one square is 6e-8 relative) and accumulates in double, the
// workgroup and the final reduction in double — an fp32 running sum over ~260 positive squares
// per thread and a 256-way fp32 tree drifted by ~4e-5 of the 67.8 M-parameter norm (the B = 256
// fp32 step vs the fp64 oracle: tests/test_gpu_parity_s256.py), 16x the reference's own fp32
// clip_grad_norm_ error.
__global__ __launch_bounds__(OPT_THREADS) void k_sumsq(const float* __restrict__ g, int64_t n,
                                                       double* __restrict__ partial) {
    __shared__ double red[OPT_THREADS];
    double a = 0.0;
    const int64_t n4 = n >> 2;
    const float4* g4 = reinterpret_cast<const float4*>(g);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 v = g4[i];
        a += (double)(v.x * v.x) + (double)(v.y * v.y) + (double)(v.z * v.z) + (double)(v.w * v.w);
    }
    for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        a += (double)(g[i] * g[i]);
    red[threadIdx.x] = a;
    __syncthreads();
    for (int o = OPT_THREADS / 2; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

// out[0] = ||pre_scale * g||, out[1] = pre_scale * clip_coef (the factor the
// optimiser applies to the raw gradient buffer).
__global__ void k_norm_finalize(const double* __restrict__ partial, int count, float pre_scale, float max_norm,
                                float* __restrict__ out) {
    __shared__ double red[256];
    double a = 0.0;
    for (int i = threadIdx.x; i < count; i += blockDim.x) a += partial[i];
    red[threadIdx.x] = a;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const float norm = (float)sqrt(red[0]) * pre_scale;
        float coef = 1.0f;
        if (max_norm > 0.f) {
            coef = max_norm / (norm + 1e-6f);
            coef = coef > 1.0f ? 1.0f : coef;
        }
        out[0] = norm;
        out[1] = pre_scale * coef;
    }
}

// GradScaler over the flat gradient buffer, which holds scale * (the gradients): the backward
// ran on loss * scale.  sc = {scale, growth tracker, found_inf of this step, skipped steps}.
//   found_inf = the squared norm is not finite (an inf / NaN anywhere in the buffer: its sum of
//               squares is then inf / NaN — GradScaler's _amp_foreach_non_finite_check_and_unscale_);
//   out[0]   = the pre-clip norm of the UNSCALED gradients, pre_scale * ||g|| / scale (inf if found);
//   out[1]   = the factor AdamW applies to the raw buffer: pre_scale * clip_coef / scale (0 if found);
//   out[2]   = found_inf (AdamW and its step counter skip the step: GradScaler.step);
// then the scale update of GradScaler.update (torch's _amp_update_scale_): found -> scale *=
// backoff, tracker = 0; else tracker + 1 == interval -> scale *= growth, tracker = 0.  The norm
// and coefficient use the OLD scale (the one the backward ran with).
__global__ void k_norm_finalize_scaled(const double* __restrict__ partial, int count, float pre_scale, float max_norm,
                                       float* __restrict__ out, float* __restrict__ sc, float growth, float backoff,
                                       int interval) {
    __shared__ double red[256];
    double a = 0.0;
    for (int i = threadIdx.x; i < count; i += blockDim.x) a += partial[i];
    red[threadIdx.x] = a;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const float scale = sc[0];
        const float inv = (float)(1.0 / (double)scale);   // GradScaler: scale.double().reciprocal().float()
        const bool found = !isfinite(red[0]);
        if (found) {
            out[0] = INFINITY;
            out[1] = 0.f;
            out[2] = 1.f;
            sc[0] = scale * backoff;
            sc[1] = 0.f;
            sc[3] += 1.f;
        } else {
            const float norm = (float)sqrt(red[0]) * inv * pre_scale;
            float coef = 1.0f;
            if (max_norm > 0.f) {
                coef = max_norm / (norm + 1e-6f);
                coef = coef > 1.0f ? 1.0f : coef;
            }
            out[0] = norm;
            out[1] = pre_scale * inv * coef;
            out[2] = 0.f;
            const float t = sc[1] + 1.f;
            if (t >= (float)interval) {
                sc[0] = scale * growth;
                sc[1] = 0.f;
            } else {
                sc[1] = t;
            }
        }
        sc[2] = out[2];
    }
}

// One element of the torch.optim.AdamW single-tensor update, shared by the
// scalar and the float4 kernels.  Contraction is off (every multiply and add
// rounded, as torch's separate lerp_ / mul_ / addcmul_ / addcdiv_ ops), so the
// compiler's fma choices cannot differ between the two: the same bits.
struct AdamwK {
    float gs, decay, w1, w2, beta2, eps, step_size, bc2_sqrt;
};
__device__ __forceinline__ void adamw_elem(const AdamwK& k, float& p, float g, float& m, float& v) {
#pragma clang fp contract(off)
    const float gi = g * k.gs;
    const float pi = p * k.decay;
    const float mi = m + k.w1 * (gi - m);                 // exp_avg.lerp_(grad, 1-beta1)
    const float vi = v * k.beta2 + k.w2 * gi * gi;        // exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2)
    const float denom = sqrtf(vi) / k.bc2_sqrt + k.eps;
    p = pi - k.step_size * (mi / denom);                  // param.addcdiv_(m, denom, -step_size)
    m = mi;
    v = vi;
}

__device__ __forceinline__ AdamwK adamw_consts(float lr, float beta1, float beta2, float eps, float wd,
                                               float step_size, float bc2_sqrt, const float* gscale,
                                               const float* coef) {
    AdamwK k;
    k.gs = gscale ? gscale[0] : 1.0f;
    if (coef) {  // device-side step (graph-capturable): coef = {lr / bc1, sqrt(bc2)}
        step_size = coef[0];
        bc2_sqrt = coef[1];
    }
    k.decay = 1.0f - lr * wd;
    k.w1 = 1.0f - beta1;
    k.w2 = 1.0f - beta2;
    k.beta2 = beta2;
    k.eps = eps;
    k.step_size = step_size;
    k.bc2_sqrt = bc2_sqrt;
    return k;
}

__global__ __launch_bounds__(OPT_THREADS) void k_adamw(float* __restrict__ p, const float* __restrict__ g,
                                                       float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                       float lr, float beta1, float beta2, float eps, float wd,
                                                       float step_size, float bc2_sqrt,
                                                       const float* __restrict__ gscale,
                                                       const float* __restrict__ coef,
                                                       const float* __restrict__ skip) {
    if (skip && skip[0] != 0.f) return;   // GradScaler.step: an overflowing step is skipped
    const AdamwK k = adamw_consts(lr, beta1, beta2, eps, wd, step_size, bc2_sqrt, gscale, coef);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        adamw_elem(k, p[i], g[i], m[i], v[i]);
}

// The same update over 16-byte vectors (all four buffers 16-byte aligned):
// 2 float4 of each stream in flight per thread and iteration (8 x 16 B loads
// issued before the first use), the < 4 tail elements by the first threads.
typedef float f32x4n __attribute__((ext_vector_type(4)));

// Ranges of the flat buffers the float4 kernel leaves out (in float4 units, sorted, disjoint):
// the 2-D weights k_adamw_tile16 updates (with their bf16 shadows).  Index c of the complement
// maps to the flat float4 index c + the lengths of the ranges starting at or before it.
constexpr int ADAMW_MAX_SKIP = 8;
struct AdamwSkip {
    int n;
    int64_t start4[ADAMW_MAX_SKIP], len4[ADAMW_MAX_SKIP];
};
__device__ __forceinline__ int64_t skip_map(const AdamwSkip& sk, int64_t c) {
    for (int r = 0; r < sk.n; ++r)
        if (c >= sk.start4[r]) c += sk.len4[r];
    return c;
}

// U float4 of each stream in flight per thread and iteration; NT: the gradient read and the
// three write-backs as non-temporal accesses (streamed once per step)
template <int U, bool NT>
__global__ __launch_bounds__(OPT_THREADS) void k_adamw4(float* __restrict__ p, const float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                        float lr, float beta1, float beta2, float eps, float wd,
                                                        float step_size, float bc2_sqrt,
                                                        const float* __restrict__ gscale,
                                                        const float* __restrict__ coef, AdamwSkip sk,
                                                        const float* __restrict__ skip) {
    if (skip && skip[0] != 0.f) return;
    const AdamwK k = adamw_consts(lr, beta1, beta2, eps, wd, step_size, bc2_sqrt, gscale, coef);
    float4* p4 = reinterpret_cast<float4*>(p);
    const float4* g4 = reinterpret_cast<const float4*>(g);
    float4* m4 = reinterpret_cast<float4*>(m);
    float4* v4 = reinterpret_cast<float4*>(v);
    int64_t skipped = 0;
    for (int r = 0; r < sk.n; ++r) skipped += sk.len4[r];
    const int64_t n4 = (n >> 2) - skipped, stride = (int64_t)gridDim.x * blockDim.x;
    auto upd = [&](float4& pp, const float4& gg, float4& mm, float4& vv) {
        adamw_elem(k, pp.x, gg.x, mm.x, vv.x);
        adamw_elem(k, pp.y, gg.y, mm.y, vv.y);
        adamw_elem(k, pp.z, gg.z, mm.z, vv.z);
        adamw_elem(k, pp.w, gg.w, mm.w, vv.w);
    };
    auto ldg = [&](int64_t j) -> float4 {
        if constexpr (NT) {
            const f32x4n x = __builtin_nontemporal_load(reinterpret_cast<const f32x4n*>(g4 + j));
            return make_float4(x[0], x[1], x[2], x[3]);
        } else {
            return g4[j];
        }
    };
    auto st4 = [&](float4* a, int64_t j, const float4& x) {
        if constexpr (NT) __builtin_nontemporal_store(f32x4n{x.x, x.y, x.z, x.w}, reinterpret_cast<f32x4n*>(a + j));
        else a[j] = x;
    };
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < n4; i += U * stride) {
        float4 pa[U], ga[U], ma[U], va[U];
        int64_t f[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            f[u] = skip_map(sk, i + u * stride);
            pa[u] = p4[f[u]];
            ga[u] = ldg(f[u]);
            ma[u] = m4[f[u]];
            va[u] = v4[f[u]];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            upd(pa[u], ga[u], ma[u], va[u]);
            st4(p4, f[u], pa[u]);
            st4(m4, f[u], ma[u]);
            st4(v4, f[u], va[u]);
        }
    }
    for (; i < n4; i += stride) {
        const int64_t f = skip_map(sk, i);
        float4 pa = p4[f];
        const float4 ga = ldg(f);
        float4 ma = m4[f], va = v4[f];
        upd(pa, ga, ma, va);
        st4(p4, f, pa); st4(m4, f, ma); st4(v4, f, va);
    }
    const int64_t t = ((n >> 2) << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) adamw_elem(k, p[t], g[t], m[t], v[t]);
}

// AdamW over 2-D weights W [N][K] (N, K multiples of 64; each 64-float aligned in the flat
// buffers) as 64 x 64 tiles, writing the 16-bit shadows the MFMA GEMMs read (H: bf16 or fp16,
// h16.h) — W16 [N][K] and the transposed W16t [K][N] (round to nearest even, as k_bf16_shadow)
// — from the updated values:
// the forward then needs no shadow pass.  The same element function as the flat kernels (the
// same bits); gradient reads and fp32 write-backs non-temporal, the shadows cached (read by the
// next forward).  Up to 4 weights per launch, workgroup b -> (weight, tile) by prefix sums.
struct TileHeads {
    int n;
    int64_t off[4];
    int N[4], K[4];
    int prefix[5];
    void* w16[4];
    void* w16t[4];
};
template <typename H>
__global__ __launch_bounds__(256) void k_adamw_tile16(float* __restrict__ p, const float* __restrict__ g,
                                                      float* __restrict__ m, float* __restrict__ v, float lr,
                                                      float beta1, float beta2, float eps, float wd, float step_size,
                                                      float bc2_sqrt, const float* __restrict__ gscale,
                                                      const float* __restrict__ coef, TileHeads th,
                                                      const float* __restrict__ skip) {
    if (skip && skip[0] != 0.f) return;
    __shared__ float tile[64][65];
    const AdamwK k = adamw_consts(lr, beta1, beta2, eps, wd, step_size, bc2_sqrt, gscale, coef);
    int h = 0;
    while (h + 1 < th.n && (int)blockIdx.x >= th.prefix[h + 1]) ++h;
    const int t = (int)blockIdx.x - th.prefix[h], K = th.K[h], N = th.N[h], tk = K >> 6;
    const int64_t n0 = (int64_t)(t / tk) * 64, k0 = (int64_t)(t % tk) * 64;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;   // float4 column, row within 16
    const int64_t base = th.off[h] + n0 * K + k0 + 4 * tx;
    float4 pa[4], ga[4], ma[4], va[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int64_t e = base + (int64_t)(ty + 16 * j) * K;
        pa[j] = *reinterpret_cast<const float4*>(p + e);
        const f32x4n x = __builtin_nontemporal_load(reinterpret_cast<const f32x4n*>(g + e));
        ga[j] = make_float4(x[0], x[1], x[2], x[3]);
        ma[j] = *reinterpret_cast<const float4*>(m + e);
        va[j] = *reinterpret_cast<const float4*>(v + e);
    }
    H* const w16 = reinterpret_cast<H*>(th.w16[h]);
    H* const w16t = reinterpret_cast<H*>(th.w16t[h]);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        adamw_elem(k, pa[j].x, ga[j].x, ma[j].x, va[j].x);
        adamw_elem(k, pa[j].y, ga[j].y, ma[j].y, va[j].y);
        adamw_elem(k, pa[j].z, ga[j].z, ma[j].z, va[j].z);
        adamw_elem(k, pa[j].w, ga[j].w, ma[j].w, va[j].w);
        const int r = ty + 16 * j;
        const int64_t e = base + (int64_t)r * K;
        __builtin_nontemporal_store(f32x4n{pa[j].x, pa[j].y, pa[j].z, pa[j].w}, reinterpret_cast<f32x4n*>(p + e));
        __builtin_nontemporal_store(f32x4n{ma[j].x, ma[j].y, ma[j].z, ma[j].w}, reinterpret_cast<f32x4n*>(m + e));
        __builtin_nontemporal_store(f32x4n{va[j].x, va[j].y, va[j].z, va[j].w}, reinterpret_cast<f32x4n*>(v + e));
        *reinterpret_cast<hv4<H>*>(w16 + (n0 + r) * K + k0 + 4 * tx) =
            hv4<H>{(H)pa[j].x, (H)pa[j].y, (H)pa[j].z, (H)pa[j].w};
        tile[r][4 * tx] = pa[j].x;
        tile[r][4 * tx + 1] = pa[j].y;
        tile[r][4 * tx + 2] = pa[j].z;
        tile[r][4 * tx + 3] = pa[j].w;
    }
    __syncthreads();
    // W16t row k0 + i, columns n0 + 4 tx .. +3: W[n0 + 4 tx + q][k0 + i]
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int i = ty + 16 * j;
        *reinterpret_cast<hv4<H>*>(w16t + (k0 + i) * N + n0 + 4 * tx) =
            hv4<H>{(H)tile[4 * tx][i], (H)tile[4 * tx + 1][i], (H)tile[4 * tx + 2][i], (H)tile[4 * tx + 3][i]};
    }
}

static inline bool aligned16(const void* a) { return ((uintptr_t)a & 15u) == 0; }

// step += 1; coef = {lr / (1 - b1^step), sqrt(1 - b2^step)} in fp64 (as the host path); a skipped
// step (GradScaler) leaves the step counter as it is, as torch's optimizer.step never ran
__global__ void k_adamw_coef(int* step, float lr, float beta1, float beta2, float* coef, const float* skip) {
    if (skip && skip[0] != 0.f) return;
    const int s = step[0] + 1;
    step[0] = s;
    const double bc1 = 1.0 - pow((double)beta1, (double)s);
    const double bc2 = 1.0 - pow((double)beta2, (double)s);
    coef[0] = (float)((double)lr / bc1);
    coef[1] = (float)sqrt(bc2);
}

// bf16 shadow of the parameters for the MFMA GEMM operands (round-to-nearest-even).
__global__ void k_cast_bf16(const float* __restrict__ src, uint16_t* __restrict__ dst, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t u = __float_as_uint(src[i]);
        dst[i] = (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
    }
}

__global__ void k_bf16_to_f32(const uint16_t* __restrict__ src, float* __restrict__ dst, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = __uint_as_float((uint32_t)src[i] << 16);
}

static inline int grid_for(int64_t n, int cap) {
    int64_t b = (n + OPT_THREADS - 1) / OPT_THREADS;
    return (int)(b < 1 ? 1 : (b > cap ? cap : b));
}

static int g_adamw_vec = -1;  // -1: from VAETEB_ADAMW_SCALAR (unset: vector kernel when aligned)

static void adamw_launch(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2,
                         float eps, float wd, float step_size, float bc2_sqrt, const float* gscale, const float* coef,
                         hipStream_t st, const AdamwSkip* skip = nullptr, const float* skipf = nullptr) {
    AdamwSkip sk{};
    if (skip) sk = *skip;
    int64_t skipped4 = 0;
    for (int r = 0; r < sk.n; ++r) skipped4 += sk.len4[r];
    if (g_adamw_vec < 0) {
        const char* e = getenv("VAETEB_ADAMW_SCALAR");
        g_adamw_vec = (e && e[0] == '1') ? 0 : 1;
    }
    // skipped ranges need the vector kernel (the caller checked the alignment)
    if ((g_adamw_vec || sk.n > 0) && aligned16(p) && aligned16(g) && aligned16(m) && aligned16(v)) {
        // U float4 per thread and iteration, at most cap x 256 threads (default 4, non-temporal, 2048:
        // 8 per CU; same-box step 8.72-8.75 vs 8.78-9.0 ms with 2 and cached accesses)
        static const int U = getenv("VAETEB_ADAMW_U") ? atoi(getenv("VAETEB_ADAMW_U")) : 4;
        static const int cap = getenv("VAETEB_ADAMW_GRID") ? atoi(getenv("VAETEB_ADAMW_GRID")) : 2048;
        static const bool nt = !(getenv("VAETEB_ADAMW_NT") && getenv("VAETEB_ADAMW_NT")[0] == '0');
        const dim3 grid(grid_for((n / 4 - skipped4 + 1) / (U == 4 ? 4 : 2), cap > 0 ? cap : 2048));
#define VT_ADAMW4(UU, NN)                                                                                          \
    hipLaunchKernelGGL((k_adamw4<UU, NN>), grid, dim3(OPT_THREADS), 0, st, p, g, m, v, n, lr, beta1, beta2, eps, wd, \
                       step_size, bc2_sqrt, gscale, coef, sk, skipf)
        if (U == 4) {
            if (nt) VT_ADAMW4(4, true); else VT_ADAMW4(4, false);
        } else {
            if (nt) VT_ADAMW4(2, true); else VT_ADAMW4(2, false);
        }
#undef VT_ADAMW4
    } else {
        hipLaunchKernelGGL(k_adamw, dim3(grid_for(n, 8192)), dim3(OPT_THREADS), 0, st, p, g, m, v, n, lr, beta1,
                           beta2, eps, wd, step_size, bc2_sqrt, gscale, coef, skipf);
    }
}

}  // namespace vt

using namespace vt;

extern "C" {

int vt_grad_norm_workspace_floats(void) { return 2 * NORM_BLOCKS; }   // NORM_BLOCKS doubles

int vt_grad_norm_clip(const float* g, int64_t n, float pre_scale, float max_norm, float* out2, float* ws,
                      void* stream) {
    VT_CHECK_ARG(n > 0, "vt_grad_norm_clip: empty");
    const int blocks = grid_for(n / 4 + 1, NORM_BLOCKS);
    double* wd = reinterpret_cast<double*>(ws);
    hipLaunchKernelGGL(k_sumsq, dim3(blocks), dim3(OPT_THREADS), 0, S(stream), g, n, wd);
    hipLaunchKernelGGL(k_norm_finalize, dim3(1), dim3(256), 0, S(stream), wd, blocks, pre_scale, max_norm, out2);
    VT_LAUNCH_CHECK("vt_grad_norm_clip");
    return VT_OK;
}

int vt_grad_norm_clip_scaled(const float* g, int64_t n, float pre_scale, float max_norm, float* out3, float* ws,
                             float* scaler, float growth_factor, float backoff_factor, int growth_interval,
                             void* stream) {
    VT_CHECK_ARG(n > 0 && out3 && scaler && growth_interval > 0 && growth_factor >= 1.f && backoff_factor > 0.f &&
                     backoff_factor <= 1.f,
                 "vt_grad_norm_clip_scaled: args");
    const int blocks = grid_for(n / 4 + 1, NORM_BLOCKS);
    double* wd = reinterpret_cast<double*>(ws);
    hipLaunchKernelGGL(k_sumsq, dim3(blocks), dim3(OPT_THREADS), 0, S(stream), g, n, wd);
    hipLaunchKernelGGL(k_norm_finalize_scaled, dim3(1), dim3(256), 0, S(stream), wd, blocks, pre_scale, max_norm, out3,
                       scaler, growth_factor, backoff_factor, growth_interval);
    VT_LAUNCH_CHECK("vt_grad_norm_clip_scaled");
    return VT_OK;
}

int vt_adamw_step(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2,
                  float eps, float weight_decay, int step, const float* gscale, void* stream) {
    VT_CHECK_ARG(n > 0 && step >= 1, "vt_adamw_step: n=%lld step=%d", (long long)n, step);
    const double bc1 = 1.0 - pow((double)beta1, (double)step);
    const double bc2 = 1.0 - pow((double)beta2, (double)step);
    adamw_launch(p, g, m, v, n, lr, beta1, beta2, eps, weight_decay, (float)((double)lr / bc1), (float)sqrt(bc2),
                 gscale, nullptr, S(stream), nullptr, nullptr);
    VT_LAUNCH_CHECK("vt_adamw_step");
    return VT_OK;
}

int vt_adamw_step_dev_skip(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
                           float beta2, float eps, float weight_decay, int* step, float* coef, const float* gscale,
                           const float* skip, void* stream) {
    VT_CHECK_ARG(n > 0 && step && coef, "vt_adamw_step_dev: args");
    hipLaunchKernelGGL(k_adamw_coef, dim3(1), dim3(1), 0, S(stream), step, lr, beta1, beta2, coef, skip);
    adamw_launch(p, g, m, v, n, lr, beta1, beta2, eps, weight_decay, 0.f, 1.f, gscale, coef, S(stream), nullptr, skip);
    VT_LAUNCH_CHECK("vt_adamw_step_dev");
    return VT_OK;
}

int vt_adamw_step_dev(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2,
                      float eps, float weight_decay, int* step, float* coef, const float* gscale, void* stream) {
    return vt_adamw_step_dev_skip(p, g, m, v, n, lr, beta1, beta2, eps, weight_decay, step, coef, gscale, nullptr,
                                  stream);
}

int vt_adamw_step_dev_shadow_skip(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
                                  float beta2, float eps, float weight_decay, int* step, float* coef,
                                  const float* gscale, int n_tiled, const int64_t* tiled_off, const int* tiled_N,
                                  const int* tiled_K, const int64_t* tiled_w16, const int64_t* tiled_w16t,
                                  const float* skip, void* stream) {
    VT_CHECK_ARG(n > 0 && step && coef && n_tiled >= 0 && n_tiled <= 4, "vt_adamw_step_dev_shadow: args (<= 4 tiled)");
    VT_CHECK_ARG(aligned16(p) && aligned16(g) && aligned16(m) && aligned16(v),
                 "vt_adamw_step_dev_shadow: buffers must be 16-byte aligned");
    AdamwSkip sk{};
    TileHeads th{};
    th.n = n_tiled;
    th.prefix[0] = 0;
    int64_t prev_end = -1;
    for (int h = 0; h < n_tiled; ++h) {
        const int64_t o = tiled_off[h];
        const int N = tiled_N[h], K = tiled_K[h];
        VT_CHECK_ARG(o % 64 == 0 && N > 0 && K > 0 && N % 64 == 0 && K % 64 == 0 && o + (int64_t)N * K <= n &&
                         o >= prev_end && tiled_w16[h] && tiled_w16t[h],
                     "vt_adamw_step_dev_shadow: tiled weight %d (offset %lld a multiple of 64, N %d / K %d multiples "
                     "of 64, sorted, disjoint)", h, (long long)o, N, K);
        prev_end = o + (int64_t)N * K;
        sk.start4[h] = o / 4;
        sk.len4[h] = (int64_t)N * K / 4;
        th.off[h] = o;
        th.N[h] = N;
        th.K[h] = K;
        th.prefix[h + 1] = th.prefix[h] + (N / 64) * (K / 64);
        th.w16[h] = reinterpret_cast<void*>(tiled_w16[h]);
        th.w16t[h] = reinterpret_cast<void*>(tiled_w16t[h]);
    }
    sk.n = n_tiled;
    hipStream_t st = S(stream);
    hipLaunchKernelGGL(k_adamw_coef, dim3(1), dim3(1), 0, st, step, lr, beta1, beta2, coef, skip);
    if (n_tiled > 0)
        VT_H16(hipLaunchKernelGGL(k_adamw_tile16<H>, dim3((unsigned)th.prefix[n_tiled]), dim3(256), 0, st, p, g, m, v, lr,
                                  beta1, beta2, eps, weight_decay, 0.f, 1.f, gscale, coef, th, skip));
    adamw_launch(p, g, m, v, n, lr, beta1, beta2, eps, weight_decay, 0.f, 1.f, gscale, coef, st, &sk, skip);
    VT_LAUNCH_CHECK("vt_adamw_step_dev_shadow");
    return VT_OK;
}

int vt_adamw_step_dev_shadow(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
                             float beta2, float eps, float weight_decay, int* step, float* coef, const float* gscale,
                             int n_tiled, const int64_t* tiled_off, const int* tiled_N, const int* tiled_K,
                             const int64_t* tiled_w16, const int64_t* tiled_w16t, void* stream) {
    return vt_adamw_step_dev_shadow_skip(p, g, m, v, n, lr, beta1, beta2, eps, weight_decay, step, coef, gscale, n_tiled,
                                         tiled_off, tiled_N, tiled_K, tiled_w16, tiled_w16t, nullptr, stream);
}

int vt_adamw_set_vector(int on) {
    g_adamw_vec = on ? 1 : 0;
    return VT_OK;
}

int vt_cast_bf16(const float* src, void* dst, int64_t n, void* stream) {
    VT_CHECK_ARG(n > 0, "vt_cast_bf16: empty");
    hipLaunchKernelGGL(k_cast_bf16, dim3(grid_for(n, 8192)), dim3(OPT_THREADS), 0, S(stream), src, (uint16_t*)dst, n);
    VT_LAUNCH_CHECK("vt_cast_bf16");
    return VT_OK;
}

int vt_cast_bf16_to_f32(const void* src, float* dst, int64_t n, void* stream) {
    VT_CHECK_ARG(n > 0, "vt_cast_bf16_to_f32: empty");
    hipLaunchKernelGGL(k_bf16_to_f32, dim3(grid_for(n, 8192)), dim3(OPT_THREADS), 0, S(stream), (const uint16_t*)src,
                       dst, n);
    VT_LAUNCH_CHECK("vt_cast_bf16_to_f32");
    return VT_OK;
}

}  // extern "C"

// ------------------------------------------------------------ bucket markers
// A no-op kernel captured into the step where a gradient bucket becomes complete
// (vaeteb.train.GradBuckets under Trainer.capture with several ranks): the native
// executor recognises it by its function pointer, does not launch it, and splits
// its launch list there so the bucket's all-reduce is issued mid-backward
// (csrc/stepgraph.cpp, vt_stepgraph_markers / vt_stepgraph_launch_range).
__global__ void k_bucket_mark(int bucket) { (void)bucket; }

namespace vt {
const void* bucket_marker_kernel() { return reinterpret_cast<const void*>(&k_bucket_mark); }
}  // namespace vt

extern "C" int vt_bucket_marker(int bucket, void* stream) {
    VT_CHECK_ARG(bucket >= 0, "vt_bucket_marker: bucket %d", bucket);
    hipLaunchKernelGGL(k_bucket_mark, dim3(1), dim3(1), 0, S(stream), bucket);
    VT_LAUNCH_CHECK("vt_bucket_marker");
    return VT_OK;
}
