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
#include <math.h>

#include "common.h"

namespace vt {

static constexpr int OPT_THREADS = 256;
static constexpr int NORM_BLOCKS = 1024;

__global__ __launch_bounds__(OPT_THREADS) void k_sumsq(const float* __restrict__ g, int64_t n,
                                                       float* __restrict__ partial) {
    __shared__ float red[16];
    float a = 0.f;
    const int64_t n4 = n >> 2;
    const float4* g4 = reinterpret_cast<const float4*>(g);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 v = g4[i];
        a += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        a += g[i] * g[i];
    const float t = block_sum(a, red);
    if (threadIdx.x == 0) partial[blockIdx.x] = t;
}

// out[0] = ||pre_scale * g||, out[1] = pre_scale * clip_coef (the factor the
// optimiser applies to the raw gradient buffer).
__global__ void k_norm_finalize(const float* __restrict__ partial, int count, float pre_scale, float max_norm,
                                float* __restrict__ out) {
    __shared__ double red[256];
    double a = 0.0;
    for (int i = threadIdx.x; i < count; i += blockDim.x) a += (double)partial[i];
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

__global__ __launch_bounds__(OPT_THREADS) void k_adamw(float* __restrict__ p, const float* __restrict__ g,
                                                       float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                       float lr, float beta1, float beta2, float eps, float wd,
                                                       float step_size, float bc2_sqrt,
                                                       const float* __restrict__ gscale,
                                                       const float* __restrict__ coef) {
    const float gs = gscale ? gscale[0] : 1.0f;
    if (coef) {  // device-side step (graph-capturable): coef = {lr / bc1, sqrt(bc2)}
        step_size = coef[0];
        bc2_sqrt = coef[1];
    }
    const float decay = 1.0f - lr * wd;
    const float w1 = 1.0f - beta1, w2 = 1.0f - beta2;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float gi = g[i] * gs;
        float pi = p[i] * decay;
        const float mi = m[i] + w1 * (gi - m[i]);          // exp_avg.lerp_(grad, 1-beta1)
        const float vi = v[i] * beta2 + w2 * gi * gi;      // exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2)
        const float denom = sqrtf(vi) / bc2_sqrt + eps;
        pi = pi - step_size * (mi / denom);                // param.addcdiv_(m, denom, -step_size)
        p[i] = pi;
        m[i] = mi;
        v[i] = vi;
    }
}

// step += 1; coef = {lr / (1 - b1^step), sqrt(1 - b2^step)} in fp64 (as the host path)
__global__ void k_adamw_coef(int* step, float lr, float beta1, float beta2, float* coef) {
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

static inline int grid_for(int64_t n, int cap) {
    int64_t b = (n + OPT_THREADS - 1) / OPT_THREADS;
    return (int)(b < 1 ? 1 : (b > cap ? cap : b));
}

}  // namespace vt

using namespace vt;

extern "C" {

int vt_grad_norm_workspace_floats(void) { return NORM_BLOCKS; }

int vt_grad_norm_clip(const float* g, int64_t n, float pre_scale, float max_norm, float* out2, float* ws,
                      void* stream) {
    VT_CHECK_ARG(n > 0, "vt_grad_norm_clip: empty");
    const int blocks = grid_for(n / 4 + 1, NORM_BLOCKS);
    hipLaunchKernelGGL(k_sumsq, dim3(blocks), dim3(OPT_THREADS), 0, S(stream), g, n, ws);
    hipLaunchKernelGGL(k_norm_finalize, dim3(1), dim3(256), 0, S(stream), ws, blocks, pre_scale, max_norm, out2);
    VT_LAUNCH_CHECK("vt_grad_norm_clip");
    return VT_OK;
}

int vt_adamw_step(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2,
                  float eps, float weight_decay, int step, const float* gscale, void* stream) {
    VT_CHECK_ARG(n > 0 && step >= 1, "vt_adamw_step: n=%lld step=%d", (long long)n, step);
    const double bc1 = 1.0 - pow((double)beta1, (double)step);
    const double bc2 = 1.0 - pow((double)beta2, (double)step);
    hipLaunchKernelGGL(k_adamw, dim3(grid_for(n, 8192)), dim3(OPT_THREADS), 0, S(stream), p, g, m, v, n, lr, beta1,
                       beta2, eps, weight_decay, (float)((double)lr / bc1), (float)sqrt(bc2), gscale, nullptr);
    VT_LAUNCH_CHECK("vt_adamw_step");
    return VT_OK;
}

int vt_adamw_step_dev(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2,
                      float eps, float weight_decay, int* step, float* coef, const float* gscale, void* stream) {
    VT_CHECK_ARG(n > 0 && step && coef, "vt_adamw_step_dev: args");
    hipLaunchKernelGGL(k_adamw_coef, dim3(1), dim3(1), 0, S(stream), step, lr, beta1, beta2, coef);
    hipLaunchKernelGGL(k_adamw, dim3(grid_for(n, 8192)), dim3(OPT_THREADS), 0, S(stream), p, g, m, v, n, lr, beta1,
                       beta2, eps, weight_decay, 0.f, 1.f, gscale, coef);
    VT_LAUNCH_CHECK("vt_adamw_step_dev");
    return VT_OK;
}

int vt_cast_bf16(const float* src, void* dst, int64_t n, void* stream) {
    VT_CHECK_ARG(n > 0, "vt_cast_bf16: empty");
    hipLaunchKernelGGL(k_cast_bf16, dim3(grid_for(n, 8192)), dim3(OPT_THREADS), 0, S(stream), src, (uint16_t*)dst, n);
    VT_LAUNCH_CHECK("vt_cast_bf16");
    return VT_OK;
}

}  // extern "C"
