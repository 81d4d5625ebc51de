// Fused ELBO kernels.
//
// Kernel A (latent): mu_post = mu_c + mu_y, z = mu_post + eps*exp(0.5*lv_q),
//   KL = mean_rows sum_D 0.5*(lv_p - lv_q - 1 + (e^lv_q + (mu_post-mu_p)^2)/e^lv_p)
//   ref/model/vae_teb_model.py:1046-1082 (reparameterize, _kld_loss), :1115 (residual)
// Kernel B (output): NLL = mean 0.5*(lv + (y-mu)^2/e^lv)   (:964-973, no log 2pi)
//   MSE = mean (lin - cat(y_st, y_ph))^2                      (:956-962)
//   computed together with their unit-upstream gradients (the loss leaves).
// Reductions: wave64 shuffles -> LDS -> one partial per block; a fixed-order
// finaliser sums the partials in double, so results are run-to-run identical.
#include "common.h"

namespace vt {

static constexpr int ELBO_THREADS = 256;
static constexpr int ELBO_MAX_BLOCKS = 1024;

static inline int elbo_blocks(int64_t n) {
    int64_t b = (n + ELBO_THREADS - 1) / ELBO_THREADS;
    return (int)(b < 1 ? 1 : (b > ELBO_MAX_BLOCKS ? ELBO_MAX_BLOCKS : b));
}

__global__ __launch_bounds__(ELBO_THREADS) void k_latent_fwd(const float* __restrict__ mu_c,
                                                             const float* __restrict__ lv_q,
                                                             const float* __restrict__ mu_y,
                                                             const float* __restrict__ lv_p,
                                                             const float* __restrict__ eps, int64_t n,
                                                             float* __restrict__ z, float* __restrict__ mu_post,
                                                             float* __restrict__ partial) {
    __shared__ float red[16];
    float acc = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float mq = mu_c[i] + mu_y[i];
        const float lq = lv_q[i], lp = lv_p[i];
        mu_post[i] = mq;
        z[i] = mq + eps[i] * expf(0.5f * lq);
        const float dm = mq - mu_y[i];
        acc += 0.5f * (lp - lq - 1.f + (expf(lq) + dm * dm) / expf(lp));
    }
    const float t = block_sum(acc, red);
    if (threadIdx.x == 0) partial[blockIdx.x] = t;
}

// g_kl: device scalar dL/dKL.  g_z / g_mu_post may be null (no upstream).
__global__ __launch_bounds__(ELBO_THREADS) void k_latent_bwd(
    const float* __restrict__ mu_c, const float* __restrict__ lv_q, const float* __restrict__ mu_y,
    const float* __restrict__ lv_p, const float* __restrict__ eps, int64_t n, float inv_rows,
    const float* __restrict__ g_z, const float* __restrict__ g_mu_post, const float* __restrict__ g_kl,
    float* __restrict__ g_mu_c, float* __restrict__ g_lv_q, float* __restrict__ g_mu_y, float* __restrict__ g_lv_p) {
    const float gk = g_kl ? g_kl[0] * inv_rows : 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float mq = mu_c[i] + mu_y[i];
        const float lq = lv_q[i], lp = lv_p[i];
        const float dm = mq - mu_y[i];
        const float ip = expf(-lp);
        const float eq = expf(lq);
        const float gz = g_z ? g_z[i] : 0.f;
        const float gmp = g_mu_post ? g_mu_post[i] : 0.f;
        // d/dmu_post: from z (gz), from the KL (dm * ip), plus direct upstream
        const float g_mq = gz + gmp + gk * dm * ip;
        g_mu_c[i] = g_mq;
        // mu_prior is mu_y itself and mu_post - mu_prior = mu_c: the KL does not depend
        // on mu_y, so its two terms (via mu_post and via mu_prior) cancel exactly.  Written
        // as gz + gmp instead of g_mq - gk*dm*ip: at beta = 1 the rounding residue of that
        // cancellation (~ulp of the KL term) swamps the decoder's gradient into the
        // 33-layer target mu_layer (the reference's fp32 autograd carries such a residue;
        // tests compare against the fp64 oracle with the reference's own error as the bound)
        g_mu_y[i] = gz + gmp;
        g_lv_q[i] = gz * 0.5f * eps[i] * expf(0.5f * lq) + gk * 0.5f * (eq * ip - 1.f);
        g_lv_p[i] = gk * 0.5f * (1.f - (eq + dm * dm) * ip);
    }
}

// NLL + MSE with gradients for unit upstream.
__global__ __launch_bounds__(ELBO_THREADS) void k_output_fwd(
    const float* __restrict__ mu, const float* __restrict__ lv, const float* __restrict__ y, int64_t n_nll,
    const float* __restrict__ lin, const float* __restrict__ t_st, const float* __restrict__ t_ph, int64_t n_rows,
    int c_st, int c_ph, float* __restrict__ g_mu, float* __restrict__ g_lv, float* __restrict__ g_lin,
    float* __restrict__ partial_nll, float* __restrict__ partial_mse) {
    __shared__ float red[16];
    const float inv_nll = 1.0f / (float)n_nll;
    float a = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_nll; i += (int64_t)gridDim.x * blockDim.x) {
        const float l = lv[i], d = y[i] - mu[i];
        const float iv = expf(-l);
        a += 0.5f * (l + d * d * iv);
        g_mu[i] = -d * iv * inv_nll;
        g_lv[i] = 0.5f * (1.f - d * d * iv) * inv_nll;
    }
    float t = block_sum(a, red);
    if (threadIdx.x == 0) partial_nll[blockIdx.x] = t;
    if (lin == nullptr) return;
    const int C = c_st + c_ph;
    const int64_t n_mse = n_rows * C;
    const float inv_mse = 1.0f / (float)n_mse;
    float b = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_mse; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / C;
        const int c = (int)(i - r * C);
        const float tg = c < c_st ? t_st[r * c_st + c] : t_ph[r * c_ph + (c - c_st)];
        const float d = lin[i] - tg;
        b += d * d;
        g_lin[i] = 2.f * d * inv_mse;
    }
    t = block_sum(b, red);
    if (threadIdx.x == 0) partial_mse[blockIdx.x] = t;
}

__global__ void k_scale_by_scalar(float* __restrict__ x, int64_t n, const float* __restrict__ s) {
    const float v = s[0];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        x[i] *= v;
}

// Small fixed-order finaliser used by the C entry points: sums `count`
// partials (double accumulation) and multiplies by `scale`.
__global__ void k_sum_partials(const float* __restrict__ partials, int count, float scale, float* __restrict__ out) {
    __shared__ double red[256];
    double a = 0.0;
    for (int i = threadIdx.x; i < count; i += blockDim.x) a += (double)partials[i];
    red[threadIdx.x] = a;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[0] = (float)(red[0] * (double)scale);
}

}  // namespace vt

using namespace vt;

extern "C" {

int vt_elbo_workspace_floats(void) { return 2 * ELBO_MAX_BLOCKS; }

int vt_elbo_latent_fwd(const float* mu_c, const float* lv_q, const float* mu_y, const float* lv_p, const float* eps,
                       int64_t rows, int D, float* z, float* mu_post, float* kl, float* ws, void* stream) {
    VT_CHECK_ARG(rows > 0 && D > 0, "vt_elbo_latent_fwd: shape");
    const int64_t n = rows * D;
    const int g = elbo_blocks(n);
    hipLaunchKernelGGL(k_latent_fwd, dim3(g), dim3(ELBO_THREADS), 0, S(stream), mu_c, lv_q, mu_y, lv_p, eps, n, z,
                       mu_post, ws);
    hipLaunchKernelGGL(k_sum_partials, dim3(1), dim3(256), 0, S(stream), ws, g, (float)(1.0 / (double)rows), kl);
    VT_LAUNCH_CHECK("vt_elbo_latent_fwd");
    return VT_OK;
}

int vt_elbo_latent_bwd(const float* mu_c, const float* lv_q, const float* mu_y, const float* lv_p, const float* eps,
                       int64_t rows, int D, const float* g_z, const float* g_mu_post, const float* g_kl,
                       float* g_mu_c, float* g_lv_q, float* g_mu_y, float* g_lv_p, void* stream) {
    VT_CHECK_ARG(rows > 0 && D > 0, "vt_elbo_latent_bwd: shape");
    const int64_t n = rows * D;
    hipLaunchKernelGGL(k_latent_bwd, dim3(elbo_blocks(n)), dim3(ELBO_THREADS), 0, S(stream), mu_c, lv_q, mu_y, lv_p,
                       eps, n, (float)(1.0 / (double)rows), g_z, g_mu_post, g_kl, g_mu_c, g_lv_q, g_mu_y, g_lv_p);
    VT_LAUNCH_CHECK("vt_elbo_latent_bwd");
    return VT_OK;
}

int vt_elbo_output_fwd(const float* mu, const float* lv, const float* y, int64_t n_nll, const float* lin,
                       const float* t_st, const float* t_ph, int64_t rows, int c_st, int c_ph, float* g_mu,
                       float* g_lv, float* g_lin, float* nll, float* mse, float* ws, void* stream) {
    VT_CHECK_ARG(n_nll > 0, "vt_elbo_output_fwd: empty");
    VT_CHECK_ARG(lin == nullptr || (rows > 0 && c_st > 0 && c_ph > 0 && t_st && t_ph && g_lin),
                 "vt_elbo_output_fwd: mse operands");
    const int64_t n = n_nll > rows * (c_st + c_ph) ? n_nll : rows * (c_st + c_ph);
    const int g = elbo_blocks(n);
    hipLaunchKernelGGL(k_output_fwd, dim3(g), dim3(ELBO_THREADS), 0, S(stream), mu, lv, y, n_nll, lin, t_st, t_ph,
                       rows, c_st, c_ph, g_mu, g_lv, g_lin, ws, ws + ELBO_MAX_BLOCKS);
    hipLaunchKernelGGL(k_sum_partials, dim3(1), dim3(256), 0, S(stream), ws, g, (float)(1.0 / (double)n_nll), nll);
    if (lin)
        hipLaunchKernelGGL(k_sum_partials, dim3(1), dim3(256), 0, S(stream), ws + ELBO_MAX_BLOCKS, g,
                           (float)(1.0 / (double)(rows * (c_st + c_ph))), mse);
    VT_LAUNCH_CHECK("vt_elbo_output_fwd");
    return VT_OK;
}

int vt_scale_by_device_scalar(float* x, int64_t n, const float* s, void* stream) {
    VT_CHECK_ARG(n >= 0, "vt_scale_by_device_scalar: n");
    if (n == 0) return VT_OK;
    hipLaunchKernelGGL(k_scale_by_scalar, dim3(elbo_blocks(n)), dim3(ELBO_THREADS), 0, S(stream), x, n, s);
    VT_LAUNCH_CHECK("vt_scale_by_device_scalar");
    return VT_OK;
}

}  // extern "C"
