/*
 * vaeteb.h — C ABI of the MI355X (gfx950) VAE-TEB training-step library
 * (libvaeteb.so, built from vae-teb_amd/csrc/).
 *
 * Conventions
 *  - Plain C: pointers, int / int64_t sizes, `void* stream` (a hipStream_t;
 *    NULL = default stream).  No torch or C++ types cross the boundary.
 *  - The caller owns every buffer (device memory) and every table; nothing
 *    here allocates or frees caller memory.  Workspaces are passed in.
 *  - Complex data is interleaved float2 {re, im} — the layout of a torch
 *    complex64 tensor and of kymatio's "trailing dim 2" convention
 *    (ref/kymatio/kymatio/backend/torch_backend.py:129-135).
 *  - Every call is stream-ordered, asynchronous, re-entrant and host-sync free
 *    (capturable in a hipGraph).  Return 0 (VT_OK) or a negative code; the
 *    message of the last failure on the calling thread is vt_last_error().
 *
 * Each entry point names the reference interface it replaces (file:line,
 * paths relative to the reference repository root).
 */
#ifndef VAETEB_H
#define VAETEB_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VT_OK 0
#define VT_ERR_ARG (-1)    /* bad argument / shape  -> Python ValueError     */
#define VT_ERR_LAYOUT (-2) /* non-contiguous input  -> RuntimeError        */
#define VT_ERR_HIP (-3)    /* HIP runtime error     -> RuntimeError        */

#define VT_FFT_MAX_LDS 8192 /* longest FFT held in one workgroup's LDS     */

const char* vt_last_error(void);
/* Stream `to` waits for the work enqueued on stream `from` so far (pooled event
 * record + wait; hipGraph-capturable).  Host-side helper for the model's side-stream
 * forks and joins (torch.cuda.Stream.wait_stream without a Python Event).        */
int vt_stream_fork(void* from, void* to);
/* The same in two halves: mark = record a pooled event on `stream` (its slot in
 * *slot), wait_mark = `stream` waits for a marked point.                          */
int vt_stream_mark(void* stream, int* slot);
int vt_stream_wait_mark(void* stream, int slot);
int vt_abi_version(void);
/* Zero every last-arriving-workgroup counter pool of the library (the in-kernel finalisers of
 * the split sums, BatchNorm column sums and head GEMMs, csrc/common.h last_arrival), stream
 * ordered.  A finished kernel leaves its counters at 0; after a failed or aborted launch a
 * counter may not be, and the next kernel using it would elect the wrong last workgroup —
 * call this (with nothing else in flight) to recover.  No reference counterpart (library
 * hygiene).                                                                                 */
int vt_arrive_reset(void* stream);
/* Diagnostic: the hipGraph capture state of `stream` as text (status, capture id, node counts
 * by type, the stream's current dependency nodes, kernel nodes with an empty grid) into buf[len]
 * (tools/capture_probe.py).  No reference counterpart.                                        */
int vt_capture_info(void* stream, char* buf, int len);
/* The 16-bit MFMA operand format of the decoder heads (vt_mfma_*), the bf16 conv blocks
 * (vt_conv1d_*_bf16*, vt_conv1d_*16*, vt_batchnorm_bwd_x16) and the bf16 ResidualMLP stacks
 * (vt_resmlp_bf16_*), and of the weight shadows they read (vt_mfma_weight_shadow,
 * vt_conv1d_bf16_shadow*, vt_adamw_step_dev_shadow): 0 = bf16 (default), 1 = fp16, the
 * reference's autocast width (ref/model/graph_model.py:510 precision="16-mixed",
 * :709-711 torch.amp.autocast('cuda')), trained with the dynamic loss scale below.  Read at
 * launch time by every such entry point (library-wide: set it before a forward / capture;
 * a captured step keeps the format it was captured with; shadow buffers written in one format
 * must not be read in the other).  Returns the previous format.                            */
int vt_set_h16_format(int fp16);
int vt_get_h16_format(void);

/* ------------------------------------------------------------------ front-end
 * Twiddle tables `tw`: float2[n], tw[k] = exp(-2*pi*i*k/n) computed in fp64 on
 * the host; an FFT of length n/stride reads it with that stride.            */

/* Pad (to n_pad, pad_left on the left; pad_mode 0 reflect, 1 constant zero,
 * 2 circular) + forward FFT of each row.
 * replaces: kymatio pad+rfft  ref/kymatio/kymatio/scattering1d/core/scattering1d.py:288-290,
 *           _pad_signal + fft ref/hdf5_dataset/kymatio_phase_scattering.py:162-205,222-223 */
int vt_fe_spectrum(const float* x, int64_t rows, int N, int n_pad, int pad_left, int pad_mode, const void* tw,
                   void* xhat, void* stream);

/* S0: phi-lowpass + 2^log2T decimation of the padded signal, as a short
 * correlation with h0 = ifft(phi_0) (even, radius taps each side).
 * out[row*out_row_stride + m] = sum_d x_pad[step*(m+start)-d] * h0[|d|], m < S.
 * replaces: scattering1d.py:295-303 (S_0 = unpad(irfft(subsample(U_0_hat*phi))))      */
int vt_fe_lowpass(const float* x, int64_t rows, int64_t x_row_stride, int N, int n_pad, int pad_left,
                  const float* h0, int radius, int step, int start, int S, float* out, int64_t out_row_stride,
                  void* stream);

/* One workgroup per (sample b, item): xhat[b,chan] * psi[filter] -> inverse FFT
 * in LDS -> analytic[b, slot, 0:N] = result[pad_left:pad_left+N] (if slot>=0; in the
 * polar form when vt_fe_set_analytic_polar(1) on the 8192-point geometry)
 * and s1[b, s1_channel, :] = lowpass(|result[::2^k1]|) (if s1_channel>=0).
 * items: int[n_items][5] = {chan, filter, slot, s1_channel, k1}.
 * replaces: first-order loop scattering1d.py:306-333 and
 *           _apply_filters kymatio_phase_scattering.py:220-231                           */
int vt_fe_wavelet(const void* xhat, int64_t B, int C, int n_pad, const float* psi, int n_items, const int* items,
                  const void* tw, int N, int pad_left, void* analytic, int n_slots, const float* h0, int radius,
                  int step, int start, int S, float* s1, int s1_channels, void* stream);

/* One workgroup per (sample b, pair p): c = |a_i| e^{i power*arg(a_i)} conj(a_j),
 * pad to n_pad (pad_mode as vt_fe_spectrum), FFT, multiply bins [0, n_pad/dec)
 * by phi0 (real), inverse FFT of length n_pad/dec, out[b,p,m] = Re(.)[start+m],
 * m < S.  dec == 0: no low-pass, out[b,p,i] = Re(c[i]), S == N
 * (cross_phase_low_pass=False).
 * replaces: _compute_phase_correlation        kymatio_phase_scattering.py:275-301,
 *           _compute_cross_channel_phase_correlation :303-360, _apply_phi_filter :233-273 */
int vt_fe_pairs(const void* analytic, int64_t B, int n_slots, int N, int n_pad, int pad_left, int n_pairs,
                const int* slot_i, const int* slot_j, const float* power, const void* tw, const float* phi0, int dec,
                int start, int S, int pad_mode, float* out, void* stream);

/* Product staging of vt_fe_pairs on the training geometry (N 4096, n_pad 8192, dec 16):
 * 0 = the product is formed once per sample into LDS (default), 1 = each thread forms
 * its padded column straight from HBM/L2 (faster alone, slower when the phase and cross
 * launches run concurrently).  Initial value from VAETEB_PAIRS_DIRECT; returns the
 * previous setting (not an error code).  Not thread-safe: set before launching. */
/* pair kernel form on the training geometry: grid > 0 = the persistent kernel with that many
 * workgroups (a multiple of 8), -1 = persistent with 2 per CU, 0 = one workgroup per item (the
 * default: measured faster in the step); returns the previous grid (same bits either way) */
int vt_fe_set_pairs_persist(int grid);
int vt_fe_set_pairs_direct(int on);
/* pair kernel form on the training geometry: 1 = half-image k_fe_pairs8k_h at three workgroups per CU
 * (default), 2 = the same at four (64 VGPRs), 3 = three per CU with the four-lane pass 3, 0 = the
 * full-image k_fe_pairs8k of rounds 2-5; initial value from VAETEB_PAIRS_HALF; returns the previous
 * setting */
int vt_fe_set_pairs_half(int on);
/* Storage form of the analytic slots on the 8192-point geometry (n_pad 8192,
 * pad_left + N <= 8192), shared by vt_fe_wavelet (writes) and vt_fe_pairs (reads):
 * 1 = polar {arg(a) / 2 pi, |a|} (the pair product becomes |a_i| |a_j|
 * e^{2 pi i (power arg_i - arg_j)}, no per-pair arctangent: pair kernel 0.837 -> 0.785 ms),
 * 0 = complex {re, im} (every other geometry is always complex).  Default 1;
 * VAETEB_ANALYTIC_POLAR=0 sets 0 initially; returns the previous setting.  Not thread-safe.  */
int vt_fe_set_analytic_polar(int on);

/* Diagnostic (tools/pairs_phases.py): while buf != NULL, training-geometry vt_fe_pairs
 * launches stamp wave 0's wall clock (100 MHz) at each phase boundary into
 * buf[(b * n_pairs + pair) * 8 + phase] (uint64).  NULL turns it off. */
int vt_fe_set_pairs_stamps(void* buf);

/* Per-channel transform (kind 0 none, 1 log(max(x,0)+log_eps), 2 asinh) and
 * z-score (x-mean)/(std+1e-8); in[b, c, s] (batch stride in_C*S) -> out[b, s, out_off + c]
 * (row width out_C).
 * replaces: normalize_tensor_data ref/hdf5_dataset/hdf5_dataset.py:18-137 + the
 *           (C,S)->(S,C) transpose :758-759                                              */
int vt_fe_normalize(const float* in, int64_t B, int C, int in_C, int S, const int* kind, const float* mean, const float* stdv,
                    float log_eps, float* out, int out_C, int out_off, void* stream);
/* The same on the steps [s0, s0 + S_len) of input rows of in_S steps: the dataset's
 * trim of trim_minutes at each end (ref/hdf5_dataset/hdf5_dataset.py:359-364, :733-741;
 * 2 minutes = 30 decimated steps of a 5760-point window -> 300) fused into the pass.    */
int vt_fe_normalize_window(const float* in, int64_t B, int C, int in_C, int in_S, int s0, int S_len,
                           const int* kind, const float* mean, const float* stdv, float log_eps, float* out,
                           int out_C, int out_off, void* stream);
/* dst[r][dst_col0 + c] = src[r][src_col0 + c] for c < ncols, r < rows (row strides ld_src / ld_dst
 * floats): the encoders' last-axis concatenation and its backward split (ref/model/vae_teb_model.py
 * torch.cat([a, b], dim=-1) before cross_modal_fusion / the conditional encoder's MLP).            */
int vt_copy_cols(const float* src, int64_t rows, int ld_src, int src_col0, int ncols, float* dst, int ld_dst,
                 int dst_col0, void* stream);
/* torch.clamp(x, lo, hi)'s backward in one pass: gx = (lo <= x <= hi) ? g : 0 (the target encoder's logvar
 * clamp, ref/model/vae_teb_model.py:568).                                                   */
int vt_clamp_bwd(const float* g, const float* x, int64_t n, float lo, float hi, float* gx, void* stream);
/* zero the ranges [starts[r], ends[r]) of base (1 <= n <= 16) in one launch                    */
int vt_zero_ranges(float* base, int n, const int64_t* starts, const int64_t* ends, void* stream);
/* fhr / up: (x-mean)/(std+1e-8)  (hdf5_dataset.py:78-80)                                */
int vt_normalize_raw(const float* x, int64_t rows, int64_t row_stride, int N, float mean, float stdv, float* out,
                     void* stream);

/* kymatio backend-plugin primitives (TorchBackend1D, ref/kymatio/kymatio/scattering1d/
 * backend/torch_backend.py:17-174 and ref/kymatio/kymatio/backend/torch_backend.py:99-219) */
int vt_fft(const void* in, void* out, int64_t rows, int n, int inverse, const void* tw, int tw_stride,
           void* stream);                                                   /* fft / ifft (1/n)   */
/* n > VT_FFT_MAX_LDS (pow2, <= 2^21): four-step FFT through HBM, n = 256 x n/256 (column
 * pass with twiddles, then row pass); ws: rows * n complex64, distinct from in / out;
 * tw = W_n^k, k < n.  Same contract as vt_fft otherwise (torch.fft / pocketfft in the
 * reference's torch backend, torch_backend.py:106-121).                                  */
int vt_fft_large(const void* in, void* out, void* ws, int64_t rows, int n, int inverse, const void* tw,
                 void* stream);
int vt_cdgmm(const void* A, const void* B, int b_is_real, void* C, int64_t rows, int n, void* stream);
/* Batched Scattering1D cascade (scatter.hip; the per-filter loop of
 * ref/kymatio/kymatio/scattering1d/core/scattering1d.py:197-399 regrouped by level):
 * filter_sub: out[b,p,m] = mean_c A[b, a_idx[p], m + c n/k] * pool[f_off[p] + m + c n/k]
 *             (cdgmm + subsample_fourier; A (B, a_rows, n) c64, out (B, P, n/k) c64);
 * mod_spec:   filter_sub fused with ifft -> modulus -> rfft of each row (n/k <= VT_FFT_MAX_LDS,
 *             tw = W_{n/k}^j table);
 * lowpass:    out[b, ch[p], t] = real(ifft(subsample(U[b,p] . phi, k)))[i0 + t], t < i1 - i0
 *             (cdgmm + subsample_fourier + irfft + unpad into the (B, out_C, i1-i0) output);
 *             tw = W_{n/k}^j table;
 * modulus_cplx: out = (|in|, 0) complex (modulus + rfft's zero imaginary part).            */
int vt_scat_filter_sub(const void* A, int B, int64_t a_rows, int n, const int* a_idx, const float* pool,
                       const int64_t* f_off, int P, int k, void* out, void* stream);
int vt_scat_mod_spec(const void* A, int B, int64_t a_rows, int n, const int* a_idx, const float* pool,
                     const int64_t* f_off, int P, int k, const void* tw, void* out, void* stream);
int vt_scat_lowpass(const void* U, int B, int P, int n, const float* phi, int k, int i0, int i1, const int* ch,
                    int out_C, const void* tw, float* out, void* stream);
int vt_modulus_cplx(const void* in, void* out, int64_t count, void* stream);
int vt_modulus(const void* in, float* out, int64_t count, void* stream);
int vt_modulus_bwd(const void* in, const float* mod, const float* grad, void* grad_in, int64_t count, void* stream);
int vt_subsample_fourier(const void* in, void* out, int64_t rows, int n, int k, void* stream);
int vt_pad_reflect(const float* in, float* out, int64_t rows, int N, int pad_left, int pad_right, void* stream);


/* ---------------------------------------------------------------------- ELBO
 * Workspace `ws`: float[vt_elbo_workspace_floats()], device.  Scalars (kl,
 * nll, mse, g_kl) are single device floats, so no host sync is needed.       */
int vt_elbo_workspace_floats(void);

/* mu_post = mu_c + mu_y; z = mu_post + eps*exp(0.5*lv_q);
 * kl = mean_rows sum_D 0.5*(lv_p - lv_q - 1 + (exp(lv_q) + (mu_post-mu_y)^2)/exp(lv_p)).
 * replaces: SeqVaeTeb.reparameterize ref/model/vae_teb_model.py:1046-1050,
 *           _kld_loss :1052-1082 and the residual mu_post += mu_y :1115          */
int vt_elbo_latent_fwd(const float* mu_c, const float* lv_q, const float* mu_y, const float* lv_p, const float* eps,
                       int64_t rows, int D, float* z, float* mu_post, float* kl, float* ws, void* stream);
/* Gradients of the above given dL/dz (nullable), dL/dmu_post (nullable) and the
 * device scalar dL/dkl (nullable).                                               */
int vt_elbo_latent_bwd(const float* mu_c, const float* lv_q, const float* mu_y, const float* lv_p, const float* eps,
                       int64_t rows, int D, const float* g_z, const float* g_mu_post, const float* g_kl,
                       float* g_mu_c, float* g_lv_q, float* g_mu_y, float* g_lv_p, void* stream);
/* nll = mean 0.5*(lv + (y-mu)^2/exp(lv)) over n_nll; mse = mean (lin - [t_st|t_ph])^2
 * over rows x (c_st+c_ph) (skipped when lin == NULL); writes the unit-upstream
 * gradients g_mu, g_lv, g_lin.
 * replaces: Decoder.compute_loss ref/model/vae_teb_model.py:932-979              */
int vt_elbo_output_fwd(const float* mu, const float* lv, const float* y, int64_t n_nll, const float* lin,
                       const float* t_st, const float* t_ph, int64_t rows, int c_st, int c_ph, float* g_mu,
                       float* g_lv, float* g_lin, float* nll, float* mse, float* ws, void* stream);
/* x *= s[0] (s a device scalar): applies an upstream loss gradient.             */
int vt_scale_by_device_scalar(float* x, int64_t n, const float* s, void* stream);

/* ----------------------------------------------------------------- optimiser
 * Flat fp32 buffers: every parameter / gradient / moment is a view of one
 * contiguous allocation.                                                        */
int vt_grad_norm_workspace_floats(void);
/* out2[0] = ||pre_scale*g||_2; out2[1] = pre_scale * min(max_norm/(out2[0]+1e-6), 1)
 * (max_norm <= 0: no clipping).  replaces: clip_grad_norm_ ref/model/graph_model.py:724 */
int vt_grad_norm_clip(const float* g, int64_t n, float pre_scale, float max_norm, float* out2, float* ws,
                      void* stream);
/* The same over a buffer that holds scale * gradients (the backward ran on loss * scale:
 * the fp16 operand format, vt_set_h16_format), with the dynamic loss scale on the device,
 * scaler = float[4] {scale, growth tracker, found_inf, skipped-step count}: found_inf = the
 * squared norm is not finite; out3[0] = pre_scale * ||g|| / scale (inf if found), out3[1] =
 * pre_scale * clip_coef / scale (0 if found), out3[2] = found_inf; then scale *= backoff_factor
 * and tracker = 0 if found, else tracker + 1 == growth_interval -> scale *= growth_factor.
 * replaces: torch.amp.GradScaler('cuda') scale / unscale_ / update around clip_grad_norm_
 *           (ref/model/graph_model.py:670, 718-726), GradScaler defaults 2.0 / 0.5 / 2000   */
int vt_grad_norm_clip_scaled(const float* g, int64_t n, float pre_scale, float max_norm, float* out3, float* ws,
                             float* scaler, float growth_factor, float backoff_factor, int growth_interval,
                             void* stream);
/* torch.optim.AdamW (decoupled decay) with g <- g*gscale[0] (nullable).
 * replaces: torch.optim.AdamW configured at ref/model/graph_model.py:654-660,
 *           ref/model/pytorch_lightning_modules.py:540-546                       */
int vt_adamw_step(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2,
                  float eps, float weight_decay, int step, const float* gscale, void* stream);
/* Same update with the step counter on the device (int[1], incremented in
 * place; coef: float[2] scratch) — no host scalar changes between steps, so a
 * whole training step can be captured once in a hipGraph and replayed.          */
int vt_adamw_step_dev(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2,
                      float eps, float weight_decay, int* step, float* coef, const float* gscale, void* stream);
/* vt_adamw_step_dev + the bf16 shadows of up to 4 2-D weights written by the update itself:
 * tiled weight h is W [N_h][K_h] at float offset off_h of the flat buffers (off_h a multiple of
 * 64, N_h and K_h multiples of 64, sorted and disjoint; buffers 16-byte aligned); it is updated
 * as 64 x 64 tiles that also write W16 [N][K] and W16t [K][N] in bf16 (round to nearest even:
 * the vt_mfma_weight_shadow images) at the device addresses tiled_w16[h] / tiled_w16t[h]
 * (host arrays of addresses); everything else as vt_adamw_step_dev.  The same element update
 * (bits) as vt_adamw_step_dev.  The MFMA heads' forward then needs no shadow pass.
 * replaces: torch.optim.AdamW.step (ref/model/graph_model.py:654-660, :726) + the 16-bit weight
 *           casts of autocast in the next forward (:709-711)                                    */
int vt_adamw_step_dev_shadow(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
                             float beta2, float eps, float weight_decay, int* step, float* coef, const float* gscale,
                             int n_tiled, const int64_t* tiled_off, const int* tiled_N, const int* tiled_K,
                             const int64_t* tiled_w16, const int64_t* tiled_w16t, void* stream);
/* vt_adamw_step_dev / vt_adamw_step_dev_shadow skipped on the device when skip[0] != 0 (the
 * found_inf of vt_grad_norm_clip_scaled, out3 + 2): no parameter, moment, shadow or step-counter
 * change, as GradScaler.step skips optimizer.step (ref/model/graph_model.py:725).  The shadows
 * are written in the current 16-bit format (vt_set_h16_format).                           */
int vt_adamw_step_dev_skip(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
                           float beta2, float eps, float weight_decay, int* step, float* coef, const float* gscale,
                           const float* skip, void* stream);
int vt_adamw_step_dev_shadow_skip(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
                                  float beta2, float eps, float weight_decay, int* step, float* coef,
                                  const float* gscale, int n_tiled, const int64_t* tiled_off, const int* tiled_N,
                                  const int* tiled_K, const int64_t* tiled_w16, const int64_t* tiled_w16t,
                                  const float* skip, void* stream);
/* Tuning switch: 1 (default) = the float4 AdamW kernel when p, g, m, v are all
 * 16-byte aligned, 0 = the scalar kernel.  Same per-element expression: the
 * two give the same bits (tested).  Env override: VAETEB_ADAMW_SCALAR=1.         */
int vt_adamw_set_vector(int on);
/* bf16 (RNE) shadow copy of fp32 data, for MFMA operands.                         */
int vt_cast_bf16(const float* src, void* dst, int64_t n, void* stream);
/* dst = float(src) for bf16 src (exact).  With vt_cast_bf16: the optional bf16 gradient
 * all-reduce of the data-parallel step (vaeteb.train.GradBuckets(reduce_dtype=bfloat16)). */
int vt_cast_bf16_to_f32(const void* src, float* dst, int64_t n, void* stream);

/* --------------------------------------------------------------- dense layers
 * fp32 tiled GEMM engine (gemm.hip).  Activations are row-major (rows, C);
 * rows = B*S.  `ws` is caller scratch for split-K partials (ws_floats floats). */
int vt_gemm_splits_hint(int64_t M, int N, int64_t K);
/* Y[R,N] = X[R,K] W[N,K]^T + b   — nn.Linear inside ResidualMLP
 * (ref/model/vae_teb_model.py:336-403) and the LSTM input projections.        */
int vt_linear_fwd(const float* X, int64_t R, int K, const float* W, int N, const float* bias, float* Y, void* stream);
/* dX (+)= dY W                                                                   */
int vt_linear_bwd_data(const float* dY, int64_t R, int N, const float* W, int K, float* dX, int accumulate,
                       void* stream);
/* dW (+)= dY^T X and, if db != NULL, db (+)= column sums of dY (fused as a
 * ones-column of X); split-K over R with a fixed-order reduction.              */
int vt_linear_bwd_weight(const float* dY, int64_t R, int N, const float* X, int K, float* dW, float* db,
                         int accumulate, float* ws, int64_t ws_floats, void* stream);
/* Y = act(LayerNorm(X W^T + b; gamma, beta, eps)), N <= 256, also xhat and
 * rstd (saved for vt_layernorm_bwd) — a ResidualMLP hidden layer
 * Linear -> LayerNorm -> act (ref/model/vae_teb_model.py:336-403) in one pass:
 * the LN statistics are taken in the GEMM epilogue.  act as vt_act_fwd.        */
int vt_linear_ln_fwd(const float* X, int64_t R, int K, const float* W, int N, const float* bias, const float* gamma,
                     const float* beta, int act, float eps, float* Y, float* xhat, float* rstd, void* stream);
/* out[N] (+)= column sums of X[R,N]                                             */
int vt_colsum(const float* X, int64_t R, int N, float* out, int accumulate, float* ws, int64_t ws_floats,
              void* stream);

/* ------------------------------------------------------- whole ResidualMLP
 * One ResidualMLP (ref/model/vae_teb_model.py:336-403) per launch sequence:
 *   x0 = LN_in(x); h_0 = x0; h_l = act_l(LN_l(h_{l-1} W_l^T + b_l)) for the
 *   layers with layer_ln[l] (every hidden layer; the last one too when
 *   final_activation), else h_L = h_{L-1} W_L^T + b_L (act must be 0);
 *   out = h_L + skip, skip 0 none, 1 identity (dims[0] == dims[L]),
 *   2 projection Linear(dims[0] -> dims[L]) of x0 (use_skip_connection, :398-403).
 * dims[0..L]: widths (<= VT_MLP_MAX_WIDTH); L <= VT_MLP_MAX_LAYERS; act as vt_act_fwd.
 * params (4L+4 device pointers): [g_in, b_in, (W_l [N][K], b_l, g_l, beta_l) x L,
 *   Ws, bs]; g_l/beta_l NULL for a layer without LN, Ws/bs NULL unless skip == 2.
 * The forward saves xhat (sizes[0] floats) and rstd (sizes[1]) of every LN;
 * the backward takes dout, writes dx (overwrite) and the parameter gradients
 * `grads` (same layout as params, NULL entries skipped; accumulate: += else =)
 * and needs sizes[2] floats of workspace.                                       */
#define VT_MLP_MAX_LAYERS 34
#define VT_MLP_MAX_WIDTH 144
int vt_resmlp_sizes(int n_layers, const int* dims, const int* layer_ln, const int* layer_act, int skip,
                    int64_t rows, int64_t* sizes);
int vt_resmlp_fwd(int n_layers, const int* dims, const int* layer_ln, const int* layer_act, int skip, float eps,
                  const float* const* params, const float* x, int64_t rows, float* out, float* xhat, float* rstd,
                  void* stream);
int vt_resmlp_bwd(int n_layers, const int* dims, const int* layer_ln, const int* layer_act, int skip, float eps,
                  const float* const* params, const float* dout, const float* xhat, const float* rstd, int64_t rows,
                  float* dx, float* const* grads, int accumulate, float* ws, int64_t ws_floats, void* stream);

/* ------------------------------------------- whole ResidualMLP, bf16 MFMA
 * The same ResidualMLP (ref/model/vae_teb_model.py:336-403, same arguments and
 * parameter / gradient layout as vt_resmlp_*) with every Linear on bf16 MFMA
 * (v_mfma_f32_16x16x32_bf16, fp32 accumulation) — the reference trains under
 * fp16 autocast (ref/model/graph_model.py:510, :709-711; bf16 here): Linear in 16 bit,
 * LayerNorm, activations, the saved state and every reduction in fp32.  The
 * saved xhat / rstd (sizes[0], sizes[1] floats) use this family's own layout
 * (pass them only to vt_resmlp_bf16_bwd); the backward needs sizes[2] floats of
 * workspace.  Widths <= VT_MLP_MAX_WIDTH, the weights must fit the LDS budget
 * (VT_ERR_ARG otherwise).                                                       */
int vt_resmlp_bf16_sizes(int n_layers, const int* dims, const int* layer_ln, const int* layer_act, int skip,
                         int64_t rows, int64_t* sizes);
int vt_resmlp_bf16_fwd(int n_layers, const int* dims, const int* layer_ln, const int* layer_act, int skip, float eps,
                       const float* const* params, const float* x, int64_t rows, float* out, float* xhat, float* rstd,
                       void* stream);
int vt_resmlp_bf16_bwd(int n_layers, const int* dims, const int* layer_ln, const int* layer_act, int skip, float eps,
                       const float* const* params, const float* dout, const float* xhat, const float* rstd,
                       int64_t rows, float* dx, float* const* grads, int accumulate, float* ws, int64_t ws_floats,
                       void* stream);
/* The forward's weight images (the 16-bit W / W^T images and staged LayerNorm parameters every
 * launch of a stack copies into LDS, rebuilt from the fp32 master weights each step) for SEVERAL
 * stacks in one launch (round 6): vt_resmlp_bf16_plan returns a stack's plan handle (its
 * arguments as vt_resmlp_bf16_fwd; cached, valid for the library's lifetime),
 * vt_resmlp_bf16_prep_batch builds the images of up to 32 plans in the current 16-bit format,
 * and vt_resmlp_bf16_fwd_prepped is vt_resmlp_bf16_fwd without its own image pass (the caller
 * prepared that plan's images after the weights last changed, same stream order).  The same
 * images and results as vt_resmlp_bf16_fwd.  replaces: the per-Linear weight casts of autocast
 * (ref/model/graph_model.py:709-711), once per step for the whole model.                      */
int vt_resmlp_bf16_plan(int n_layers, const int* dims, const int* layer_ln, const int* layer_act, int skip, float eps,
                        const float* const* params, int64_t rows, int64_t* handle, void* stream);
int vt_resmlp_bf16_prep_batch(int n, const int64_t* handles, void* stream);
int vt_resmlp_bf16_fwd_prepped(int n_layers, const int* dims, const int* layer_ln, const int* layer_act, int skip,
                               float eps, const float* const* params, const float* x, int64_t rows, float* out,
                               float* xhat, float* rstd, void* stream);
/* The same backward split in two (round 5), so the weight gradients leave the data-gradient
 * chain (ref/model/vae_teb_model.py:336-403 backward, the reference's autograd of Linear /
 * LayerNorm under fp16 autocast):
 *   vt_resmlp_bf16_bwd_data   dx, the LayerNorm gamma / beta and bias gradients (grads as in
 *                             vt_resmlp_bf16_bwd; the weight entries are not touched), and every
 *                             GEMM's dZ as bf16 rows in dz16 (sizes[0] bf16 elements);
 *                             workspace sizes[1] floats;
 *   vt_resmlp_bf16_bwd_weight the weight gradients from dz16 and the saved xhat, on any stream
 *                             ordered after bwd_data (e.g. a side stream); workspace sizes[2].
 * vt_resmlp_bf16_split_sizes: sizes[0..2] as above, sizes[3] = 1 when the stack's W^T images fit
 * the LDS budget of the split kernel (else use vt_resmlp_bf16_bwd).                        */
int vt_resmlp_bf16_split_sizes(int n_layers, const int* dims, const int* layer_ln, const int* layer_act, int skip,
                               int64_t rows, int64_t* sizes);
int vt_resmlp_bf16_bwd_data(int n_layers, const int* dims, const int* layer_ln, const int* layer_act, int skip,
                            float eps, const float* const* params, const float* dout, const float* xhat,
                            const float* rstd, int64_t rows, float* dx, float* const* grads, int accumulate,
                            void* dz16, float* ws, int64_t ws_floats, void* stream);
int vt_resmlp_bf16_bwd_weight(int n_layers, const int* dims, const int* layer_ln, const int* layer_act, int skip,
                              float eps, const float* const* params, const float* xhat, const void* dz16,
                              int64_t rows, float* const* grads, int accumulate, float* ws, int64_t ws_floats,
                              void* stream);
/* Diagnostic (tools/mlpb_phases.py): while buf != NULL, vt_resmlp_bf16_bwd launches stamp
 * wave 0's wall clock at the kernel's phase boundaries, 256 uint64 per workgroup. */
int vt_resmlp_bf16_set_stamps(void* buf);

/* ------------------------------------------------------- bf16 MFMA (heads)
 * The decoder's R x R output heads (Decoder.output_mu / output_logvar,
 * ref/model/vae_teb_model.py:882-897,926-927, R = 16*S; the reference runs
 * them in fp16 autocast, ref/model/graph_model.py:510,710; bf16 here) as bf16 MFMA GEMMs
 * (v_mfma_f32_16x16x32_bf16, fp32 accumulation).  Same meaning as vt_linear_*;
 * the weight operand is a bf16 shadow of the fp32 master weight W [N][K]:
 * W16 = bf16(W) [N][K] for the forward, W16t = bf16(W)^T [K][N] for the input
 * gradient, both written by vt_mfma_weight_shadow (once per optimizer step).
 * K and N must be multiples of 64 (vt_mfma_supported), any R.  ws: caller
 * scratch of at least vt_mfma_workspace_floats(R, K, N) floats.                */
int vt_mfma_supported(int K, int N);
int vt_mfma_workspace_floats(int64_t R, int K, int N, int64_t* floats);
int vt_mfma_weight_shadow(const float* W, int N, int K, void* W16, void* W16t, void* stream);
int vt_mfma_linear_fwd(const float* X, int64_t R, int K, const void* W16, int N, const float* bias, float* Y,
                       float* ws, int64_t ws_floats, void* stream);
int vt_mfma_linear_bwd_data(const float* dY, int64_t R, int N, const void* W16t, int K, float* dX, int accumulate,
                            float* ws, int64_t ws_floats, void* stream);
int vt_mfma_linear_bwd_weight(const float* dY, int64_t R, int N, const float* X, int K, float* dW, float* db,
                              int accumulate, float* ws, int64_t ws_floats, void* stream);

/* ------------------------------------------------------------------ 1-D conv
 * Conv1d(bias=False) over (B, L, C) activations as an implicit GEMM whose
 * operand load performs the padding / upsampling.
 * mode 0: CausalMultiChannelConvBlock  (ref/model/vae_teb_model.py:128-212)
 * mode 1: MultiChannelConvBlock, reflect pad (K-1)/2, replicate if L <= pad,
 *         up = 1: F.interpolate(x2, linear, align_corners=False) first (:214-253) */
int vt_conv1d_out_len(int L_in, int K, int mode, int up);
int vt_conv1d_fwd(const float* X, int B, int L_in, int Cin, const float* W, int Cout, int K, int mode, int up,
                  float* Y, void* stream);
/* gpad: scratch of B*(L_out+K-1)*Cin floats                                       */
int vt_conv1d_bwd_data(const float* dY, int B, int L_in, int Cin, const float* W, int Cout, int K, int mode, int up,
                       float* dX, int accumulate, float* gpad, void* stream);
int vt_conv1d_bwd_weight(const float* dY, const float* X, int B, int L_in, int Cin, int Cout, int K, int mode, int up,
                         float* dW, int accumulate, float* ws, int64_t ws_floats, void* stream);
/* Conv1d(bias=False) -> train-mode BatchNorm1d -> act in three launches: the
 * conv kernel also writes per-tile (sum, sum of squared deviations) of its
 * outputs, one finalize combines them (Chan, double) into mean / rstd and the
 * running statistics, one pass applies BN + act.  conv_out (B, L_out, Cout) is
 * kept for the backward; ws: vt_conv1d_bn_workspace_floats floats.
 * replaces: CausalMultiChannelConvBlock / MultiChannelConvBlock forward
 *           (ref/model/vae_teb_model.py:128-212, :214-253)                        */
int vt_conv1d_bn_workspace_floats(int B, int L_in, int Cin, int Cout, int K, int mode, int up, int64_t* floats);
int vt_conv1d_bn_fwd(const float* X, int B, int L_in, int Cin, const float* W, int Cout, int K, int mode, int up,
                     const float* gamma, const float* beta, int act, float eps, float momentum, float* conv_out,
                     float* Y, float* mean, float* rstd, float* run_mean, float* run_var, float* ws,
                     int64_t ws_floats, void* stream);
/* bf16-MFMA variants (conv_bf16.hip) — the reference trains in fp16 (bf16 here) under
 * autocast (ref/model/graph_model.py:510, :709-711): bf16 operands, fp32
 * accumulation, fp32 activations and BatchNorm.  Weights come from a bf16
 * shadow refreshed from the fp32 master weight W [Cout][Cin][K] once per
 * step: w16 [Cout][K][ceil32(Cin)] (forward), w16t [Cin][K][ceil32(Cout)]
 * = W[co][ci][K-1-k] (backward-data), zero-padded.                             */
int vt_conv1d_bf16_shadow(const float* W, int Cout, int Cin, int K, void* w16, void* w16t, void* stream);
/* the same shadows of n <= 24 conv weights in one launch (host arrays; device addresses as int64):
 * issued by the trainer after its optimizer step, so the next forward needs no shadow launches */
int vt_conv1d_bf16_shadow_batch(int n, const int64_t* W, const int* Cout, const int* Cin, const int* K,
                                const int64_t* w16, const int64_t* w16t, void* stream);
/* Operand-window staging of the bf16 conv kernels (A/B; bit-identical results):
 * 0 octets per lane, 2 lanes along channels (coalesced row segments), 1 (default) lanes
 * along channels for the fused-BN backward-data kernels with K >= 7, octets elsewhere. */
int vt_conv_bf16_set_staging(int mode);
/* Kernel selection of the bf16 conv forward / weight gradient (A/B; bit-identical results):
 * bit 0 = the flat-staged forward of conv_fwd16.hip (source rows copied with float4 loads,
 * the whole bf16 window formed in LDS, next chunk's taps prefetched) for K <= 5, bit 1 = the
 * flat-staged, prefetching weight gradient (k_cdw16) for K >= 7 — where each measured faster —
 * bit 2 = both at every K, bit 3 = the weight gradient in 256-row chunks for dY <= 32 channels
 * (default 11); 0 = k_conv_bf16 / k_conv_dw_bf16 everywhere.                              */
int vt_conv_bf16_set_kernels(int flags);
int vt_conv1d_bn_fwd_bf16(const float* X, int B, int L_in, int Cin, const void* w16, int Cout, int K, int mode,
                          int up, const float* gamma, const float* beta, int act, float eps, float momentum,
                          float* conv_out, float* Y, float* mean, float* rstd, float* run_mean, float* run_var,
                          float* ws, int64_t ws_floats, void* stream);
/* The same block when its input is the PREVIOUS block's pre-BN conv output X: that block's
 * BatchNorm + ReLU (in_act must be 1: the stacks' inner blocks), max(0, X scale + shift) with
 * scale = in_rstd in_gamma, shift = in_beta - in_mean scale, applied to each source sample as
 * the window is staged, before padding / the x2
 * interpolation — the values vt_batchnorm_apply would have written, so a conv stack's inner
 * block outputs are never materialised (round 5).  Y nullable: no BatchNorm apply of this
 * block's own output either (the next block of the stack stages it from conv_out).
 * replaces: ConvBlock -> ConvBlock in a Sequential (ref/model/vae_teb_model.py:175-212,
 *           :230-253, the BatchNorm1d + activation output feeding the next Conv1d)         */
int vt_conv1d_bn_fwd_bf16_in(const float* X, const float* in_mean, const float* in_rstd, const float* in_gamma,
                             const float* in_beta, int in_act, int B, int L_in, int Cin, const void* w16, int Cout,
                             int K, int mode, int up, const float* gamma, const float* beta, int act, float eps,
                             float momentum, float* conv_out, float* Y, float* mean, float* rstd, float* run_mean,
                             float* run_var, float* ws, int64_t ws_floats, void* stream);
int vt_conv1d_fwd_bf16(const float* X, int B, int L_in, int Cin, const void* w16, int Cout, int K, int mode, int up,
                       float* Y, void* stream);
int vt_conv1d_bwd_gpad_bf16(const float* dY, int B, int L_in, int Cin, const void* w16t, int Cout, int K, int mode,
                            int up, float* gpad, void* stream);
/* dW (+)= sum_rows dY^T xpad on bf16 MFMA (transposed LDS reads), fixed-order
 * split reduction; channels <= 128; ws as vt_conv1d_direct_bwd_weight.          */
int vt_conv1d_bwd_weight_bf16(const float* dY, const float* X, int B, int L_in, int Cin, int Cout, int K, int mode,
                              int up, float* dW, int accumulate, float* ws, int64_t ws_floats, void* stream);
/* Fused BatchNorm backward: as vt_conv1d_bwd_gpad_bf16 on the BN input gradient
 * gamma rstd (dz - dbeta/M - xhat dgamma/M), dz = dY act'(xhat gamma + beta),
 * xhat = (Xc - mean) rstd, formed while the operand is staged from the block output
 * gradient dY (B, L_out, Cout), the pre-BN conv output Xc and bnp (vt_batchnorm_bwd_coef):
 * the same values as vt_batchnorm_bwd's dx, never written in fp32.  dxbn16 (nullable):
 * receives that gradient in bf16, rows of ceil8(Cout) (padding 0) — the operand of
 * vt_conv1d_bwd_weight_bf16_dy16, which then equals vt_conv1d_bwd_weight_bf16 on dx.
 * replaces: the BatchNorm1d backward feeding the conv input / weight gradients
 *           (ref/model/vae_teb_model.py:175, :230 under autograd)                       */
int vt_conv1d_bwd_gpad_bf16_bn(const float* dY, const float* Xc, const float* bnp, int act, int64_t M, int B,
                               int L_in, int Cin, const void* w16t, int Cout, int K, int mode, int up, float* gpad,
                               void* dxbn16, void* stream);
/* The same backward-data conv writing dX directly (no gpad + vt_conv1d_fold pass)
 * for the geometries whose fold is a crop: no upsample; causal, or reflect with
 * L_in > pad, whose 2 pad mirrored rows per sample go through edge [B][2 pad][Cin]
 * and are added back by a small second kernel (the fold's order: same bits).     */
int vt_conv1d_bwd_dx_bf16_bn(const float* dY, const float* Xc, const float* bnp, int act, int64_t M, int B, int L_in,
                             int Cin, const void* w16t, int Cout, int K, int mode, int up, float* dX, float* edge,
                             void* dxbn16, void* stream);
int vt_conv1d_bwd_weight_bf16_dy16(const void* dY16, const float* X, int B, int L_in, int Cin, int Cout, int K,
                                   int mode, int up, float* dW, int accumulate, float* ws, int64_t ws_floats,
                                   void* stream);
/* The same with the bf16 rows of dY16 dys elements apart (a multiple of 8, >= ceil8(Cout);
 * the rows of vt_batchnorm_bwd_x16 are ceil32(Cout)).                              */
int vt_conv1d_bwd_weight_bf16_dy16s(const void* dY16, int dys, const float* X, int B, int L_in, int Cin, int Cout,
                                    int K, int mode, int up, float* dW, int accumulate, float* ws, int64_t ws_floats,
                                    void* stream);
/* The weight gradient of a block fed by the previous block's pre-BN output X (as
 * vt_conv1d_bn_fwd_bf16_in: its BatchNorm + activation applied while the window is staged)
 * from dY16 (bf16 rows dys apart, as vt_conv1d_bwd_weight_bf16_dy16s); dY unused (NULL).   */
int vt_conv1d_bwd_weight_bf16_in(const float* dY, const void* dY16, int dys, const float* X, const float* in_mean,
                                 const float* in_rstd, const float* in_gamma, const float* in_beta, int in_act, int B,
                                 int L_in, int Cin, int Cout, int K, int mode, int up, float* dW, int accumulate,
                                 float* ws, int64_t ws_floats, void* stream);
/* Conv-block backward in two launches on a bf16 operand (conv_bwd16.hip):
 * vt_batchnorm_bwd_x16: the BatchNorm input gradient of vt_conv1d_bwd_gpad_bf16_bn (the
 *   same bits) written once, in bf16, rows of ceil32(C) channels (padding 0), from dY, the
 *   pre-BN conv output Xc and bnp (vt_batchnorm_bwd_coef); M rows.
 * vt_conv1d_bwd_dx16: dX (B, L_in, Cin) of the conv (W as in vt_conv1d_bwd_gpad_bf16: w16t
 *   from vt_conv1d_bf16_shadow) from that operand (B, L_out, ceil32(Cout)) — the padded
 *   gradient and vt_conv1d_fold in one launch (x2 upsample: the fold applied in LDS;
 *   reflect without upsample: mirror rows through edge [B][2 pad][Cin]).  Geometries:
 *   causal without upsample, reflect with L_in*(1+up) > pad.  Bit-identical to
 *   vt_conv1d_bwd_gpad_bf16_bn + vt_conv1d_fold.
 * replaces: the BatchNorm1d + Conv1d (+ F.interpolate x2) backward of the conv blocks
 *           (ref/model/vae_teb_model.py:170-176, :225-232 under autograd)             */
int vt_batchnorm_bwd_x16(const float* dY, const float* Xc, const float* bnp, int act, int64_t M, int C, void* d16,
                         void* stream);
int vt_conv1d_bwd_dx16(const void* d16, int B, int L_in, int Cin, const void* w16t, int Cout, int K, int mode, int up,
                       float* dX, float* edge, void* stream);
/* Direct (LDS-windowed) conv kernels used on the training path (conv.hip), K <= 11:
 * forward; bwd-data as a full correlation into gpad (B, L_out+K-1, Cin) + fold;
 * bwd-weight with fixed-order split reduction.                                   */
int vt_conv1d_direct_fwd(const float* X, int B, int L_in, int Cin, const float* W, int Cout, int K, int mode, int up,
                         float* Y, void* stream);
int vt_conv1d_direct_bwd_gpad(const float* dY, int B, int L_in, int Cin, const float* W, int Cout, int K, int mode,
                              int up, float* gpad, void* stream);
int vt_conv1d_fold(const float* gpad, int B, int L_in, int Cin, int Cout, int K, int mode, int up, float* dX,
                   int accumulate, void* stream);
int vt_conv1d_direct_bwd_weight(const float* dY, const float* X, int B, int L_in, int Cin, int Cout, int K, int mode,
                                int up, float* dW, int accumulate, float* ws, int64_t ws_floats, void* stream);

/* -------------------------------------------------------- norms / activations
 * act: 0 none, 1 ReLU, 2 GELU (erf), 3 tanh.                                    */
/* y = act(LayerNorm(x)*gamma + beta); saves xhat (nullable) and rstd (nullable).
 * replaces: nn.LayerNorm (+ the following activation) in ResidualMLP and the
 *           encoders' fused/lstm norms (ref/model/vae_teb_model.py:342-403, :460-464) */
int vt_layernorm_fwd(const float* x, int64_t R, int C, const float* gamma, const float* beta, int act, float eps,
                     float* y, float* xhat, float* rstd, void* stream);
int vt_layernorm_bwd(const float* dy, const float* xhat, const float* rstd, int64_t R, int C, const float* gamma,
                     const float* beta, int act, float* dx, float* dgamma, float* dbeta, int accumulate_params,
                     float* ws, int64_t ws_floats, void* stream);
/* Train-mode BatchNorm1d (batch stats over M = B*L rows, momentum semantics of
 * torch, running stats updated in place) + activation.
 * replaces: nn.BatchNorm1d(C, momentum=0.9) + ReLU/tanh (vae_teb_model.py:175, :230) */
int vt_batchnorm_fwd(const float* x, int64_t M, int C, const float* gamma, const float* beta, int act, float eps,
                     float momentum, float* y, float* mean, float* rstd, float* run_mean, float* run_var, float* ws,
                     int64_t ws_floats, void* stream);
int vt_batchnorm_bwd(const float* dy, const float* x, int64_t M, int C, const float* mean, const float* rstd,
                     const float* gamma, const float* beta, int act, float* dx, float* dgamma, float* dbeta,
                     int accumulate_params, float* ws, int64_t ws_floats, void* stream);
/* vt_batchnorm_fwd / vt_batchnorm_bwd with the Dropout1d that follows the BatchNorm fused in:
 * the forward writes y = vt_dropout_apply(BN(x)) (same mask index b C + c over L-row samples,
 * same hash and scale: the values of the two calls), the backward reads dy through the mask
 * (the values of vt_dropout_apply on dy followed by vt_batchnorm_bwd).  L = 0: element-wise.
 * replaces: BatchNorm1d + ReLU + Dropout1d of FHRInception / FHRResidual
 *           (ref/model/inception_time.py:89-117, :152-170) in one pass each way */
int vt_batchnorm_fwd_dropout(const float* x, int64_t M, int C, const float* gamma, const float* beta, int act,
                             float eps, float momentum, float* y, float* mean, float* rstd, float* run_mean,
                             float* run_var, int L, float p, int64_t seed, const void* seed_offset, float* ws,
                             int64_t ws_floats, void* stream);
int vt_batchnorm_bwd_dropout(const float* dy, const float* x, int64_t M, int C, const float* mean, const float* rstd,
                             const float* gamma, const float* beta, int act, int L, float p, int64_t seed,
                             const void* seed_offset, float* dx, float* dgamma, float* dbeta, int accumulate_params,
                             float* ws, int64_t ws_floats, void* stream);
/* The column-sum half of vt_batchnorm_bwd (dgamma / dbeta (+)= their sums) with no dx:
 * bnp = [mean | rstd | gamma | beta | dgamma_now | dbeta_now] (6 x C floats) for the bf16
 * conv backward kernels that form dx while staging their operand (*_bf16_bn below). */
int vt_batchnorm_bwd_coef(const float* dy, const float* x, int64_t M, int C, const float* mean, const float* rstd,
                          const float* gamma, const float* beta, int act, float* dgamma, float* dbeta,
                          int accumulate_params, float* bnp, float* ws, int64_t ws_floats, void* stream);
/* Eval-mode BatchNorm1d (running statistics) + activation, elementwise on (M, C).
 * replaces: model.eval() BatchNorm in ref/model/vae_teb_model.py:175,:230 and
 *           ref/model/inception_time.py:77,:139 (validation, frozen VAE, predict) */
int vt_batchnorm_eval(const float* x, int64_t M, int C, const float* run_mean, const float* run_var, float eps,
                      const float* gamma, const float* beta, int act, float* y, void* stream);
/* Synchronised train-mode BatchNorm, split at its cross-rank exchange points (the
 * caller all-reduces `sums` (SUM) between the launches; no host synchronisation).
 * replaces: torch.nn.SyncBatchNorm, which Lightning's sync_batchnorm=True substitutes for
 *           the 17 BatchNorm1d on more than one GPU (ref/model/graph_model.py:517).
 * vt_syncbn_sums: sums = [S0 | S1] (2 x C doubles) + the local row count at [2C];
 *   which 0: S0 = sum x;  which 1: S0 = sum (x - mean)^2;  which 2 (backward, dy given):
 *   S0 = sum dz, S1 = sum dz xhat, dz = dy act'(xhat gamma + beta).  ws: as vt_batchnorm_fwd.
 * vt_syncbn_stats (on the all-reduced sums): which 0: mean;  which 1: rstd + running
 *   statistics (unbiased with the global count);  which 2 (on the LOCAL sums, before the
 *   all-reduce): dbeta / dgamma (+)= S0 / S1 (this rank's parameter gradients).
 * vt_batchnorm_apply: y = act((x - mean) rstd gamma + beta).
 * vt_syncbn_bwd_dx: dx from the all-reduced backward sums; ws: 2 x C floats.           */
int vt_syncbn_sums(const float* x, const float* dy, int64_t M, int C, int which, const float* mean,
                   const float* rstd, const float* gamma, const float* beta, int act, double* sums, float* ws,
                   int64_t ws_floats, void* stream);
int vt_syncbn_stats(const double* sums, int C, int which, float eps, float momentum, float* mean, float* rstd,
                    float* run_mean, float* run_var, float* dgamma, float* dbeta, int accumulate, void* stream);
int vt_batchnorm_apply(const float* x, int64_t M, int C, const float* mean, const float* rstd, const float* gamma,
                       const float* beta, int act, float* y, void* stream);
int vt_syncbn_bwd_dx(const float* dy, const float* x, int64_t M, int C, const float* mean, const float* rstd,
                     const float* gamma, const float* beta, int act, const double* sums, float* dx, float* ws,
                     void* stream);
int vt_act_fwd(const float* x, int64_t n, int act, float* y, void* stream);
int vt_act_bwd(const float* dy, const float* x, int64_t n, int act, float* dx, void* stream);

/* ----------------------------------------------------------------------- LSTM
 * One layer's recurrence (hidden 64).  gin = X W_ih^T + b_ih for all t (from
 * vt_linear_fwd); b_hh is added here.  Outputs h, h_{t-1}, c and the
 * post-activation gates (saved for the backward).
 * replaces: nn.LSTM(in, 64, num_layers=4, batch_first=True)
 *           (ref/model/vae_teb_model.py:474-480, :647-653)                          */
int vt_lstm_layer_fwd(const float* gin, const float* w_hh, const float* b_hh, int B, int S, int hidden, float* out_h,
                      float* out_hprev, float* out_c, float* gates, void* stream);
/* dgates = d(loss)/d(gate pre-activations) given d(loss)/d(h_t) of this layer.     */
int vt_lstm_layer_bwd(const float* dh_out, const float* gates, const float* cst, const float* w_hh, int B, int S,
                      int hidden, float* dgates, void* stream);
/* The same layer with its input projection inside the recurrence kernel (input
 * size In <= 64, exact-fp32 MFMA): x [B, S, In] -> h, h_{t-1}, c, gates; the
 * results are bitwise those of vt_linear_fwd + vt_lstm_layer_fwd.
 * replaces: one layer of nn.LSTM (ref/model/vae_teb_model.py:474-480, :647-653),
 *           input GEMM and recurrence together                                     */
int vt_lstm_layer_fwd_x(const float* x, int In, const float* w_ih, const float* b_ih, const float* w_hh,
                        const float* b_hh, int B, int S, int hidden, float* out_h, float* out_hprev, float* out_c,
                        float* gates, void* stream);
/* Backward with dx = dgates W_ih inside (dx may be null; dgates may be null when
 * no weight gradient is wanted); bitwise vt_lstm_layer_bwd + vt_linear_bwd_data.  */
int vt_lstm_layer_bwd_x(const float* dh_out, const float* gates, const float* cst, const float* w_hh,
                        const float* w_ih, int In, int B, int S, int hidden, float* dgates, float* dx, void* stream);
/* The same layer at the reference's 16-bit autocast width (its LSTM runs with fp16
 * operands under torch.amp, ref/model/graph_model.py:510, :709-711): 4 samples per
 * workgroup, the recurrent matvec and the input projection on
 * v_mfma_f32_16x16x32_f16 (h, x, W rounded to f16; fp32 accumulation, cell state,
 * activations and outputs).  In % 4 == 0, In <= 64.  Same outputs as
 * vt_lstm_layer_fwd_x, except: gates are [B, S, hidden, 4] (each unit's i, f, g~, o
 * contiguous; consumed by vt_lstm16_layer_bwd only) and out_hprev may be null
 * (vt_lstm16_layer_bwd_weight reads h_{t-1} from h).
 * replaces: one layer of nn.LSTM under torch.amp.autocast (vae_teb_model.py:474-480,
 *           :647-653; graph_model.py:709-711)                                       */
int vt_lstm16_layer_fwd(const float* x, int In, const float* w_ih, const float* b_ih, const float* w_hh,
                        const float* b_hh, int B, int S, int hidden, float* out_h, float* out_hprev, float* out_c,
                        float* gates, void* stream);
/* Its backward: dh_rec = dg_{t+1} W_hh and dx = dgates W_ih on bf16 MFMA (bf16
 * keeps fp32's exponent range, so no loss scale is needed where the reference uses
 * GradScaler); cell derivatives and dgates fp32.  dgates / dx may be null.          */
int vt_lstm16_layer_bwd(const float* dh_out, const float* gates, const float* cst, const float* w_hh,
                        const float* w_ih, int In, int B, int S, int hidden, float* dgates, float* dx, void* stream);
/* Two stacked layers (l with input size In, l + 1 with input size hidden) in one launch:
 * layer l + 1 runs one 16-step chunk behind layer l in the same workgroup (8 waves, the
 * chunk's h handed over in LDS), S + 16 steps instead of 2 S.  Outputs are exactly two
 * vt_lstm16_layer_fwd calls' (out_hprev omitted), bit for bit.  In % 4 == 0, In <= 64;
 * layer l's input is staged in LDS: seq <= 416 (VAETEB_L16_PAIR_NS=4: <= 208).
 * replaces: two layers of nn.LSTM(num_layers=4) under torch.amp.autocast
 *           (vae_teb_model.py:474-480, :647-653)                                   */
int vt_lstm16_pair_fwd(const float* x, int In, const float* w_ih0, const float* b_ih0, const float* w_hh0,
                       const float* b_hh0, const float* w_ih1, const float* b_ih1, const float* w_hh1,
                       const float* b_hh1, int B, int seq, int hidden, float* h0, float* c0, float* gates0, float* h1,
                       float* c1, float* gates1, void* stream);
/* Its backward: layer l + 1 (dh_out at its outputs, its forward's gates1 / c1) and layer l
 * one chunk behind it, layer l + 1's dX handed to layer l in LDS.  dgates1 / dgates0 and
 * dx (layer l's input gradient [B, S, In0], may be null) are exactly two
 * vt_lstm16_layer_bwd calls', bit for bit.                                          */
int vt_lstm16_pair_bwd(const float* dh_out, const float* gates1, const float* c1, const float* w_hh1,
                       const float* w_ih1, const float* gates0, const float* c0, const float* w_hh0,
                       const float* w_ih0, int In0, int B, int seq, int hidden, float* dgates1, float* dgates0,
                       float* dx, void* stream);
/* All four layers of nn.LSTM(num_layers=4) in ONE launch (round 6): the two layer pairs of
 * vt_lstm16_pair_fwd run concurrently, pair 1 (layers 2, 3) consuming layer 1's h chunk by
 * chunk as pair 0 publishes it (a per-chunk flag; agent-coherent stores / loads) — S + 4
 * chunks of steps instead of 2 (S + 1 chunk).  params: the 16 pointers [w_ih, w_hh, b_ih,
 * b_hh] of layers 0..3; outs: the 12 pointers [h, c, gates] of layers 0..3.  Outputs are
 * exactly two vt_lstm16_pair_fwd calls', bit for bit (which it runs instead when the
 * workgroups per pair are not a multiple of 8, or VAETEB_L16_CHAIN=0).
 * replaces: nn.LSTM(in, 64, 4 layers) under torch.amp.autocast (vae_teb_model.py:474-480,
 *           :647-653)                                                                   */
int vt_lstm16_quad_fwd(const float* x, int In, const float* const* params, int B, int seq, int hidden,
                       float* const* outs, void* stream);
/* Its backward in one launch: layers 3, 2 (dh_out at layer 3's outputs) publish layer 2's dX —
 * the gradient at layer 1's outputs, written to dmid [B, S, hidden] — chunk by chunk to layers
 * 1, 0 running concurrently.  w: [w_ih, w_hh] x 4 layers; gc: [gates, c] x 4 layers (the
 * forward's); dg: the 4 layers' dgates [B, S, 4 hidden]; dx: layer 0's input gradient [B, S,
 * In0] (may be null).  Exactly two vt_lstm16_pair_bwd calls', bit for bit.                */
int vt_lstm16_quad_bwd(const float* dh_out, const float* const* w, const float* const* gc, int In0, int B, int seq,
                       int hidden, float* const* dg, float* dmid, float* dx, void* stream);
/* Timeouts of the chained launches' bounded waits since the last reset (0 unless a producer
 * workgroup could not run; host-synchronous diagnostic).                                  */
int vt_lstm16_chain_errors(int* count, int reset);
/* All of a layer's parameter gradients in one pass over dgates [B*S, 4H]:
 * dw_ih (+)= dgates^T x, dw_hh (+)= dgates^T h_{t-1}, db_ih and db_hh (may be
 * null) (+)= column sums of dgates.  In + hidden + 1 <= 144; ws: at least
 * min(256, B*S/256) * 4H * (In + hidden + 1) floats.                              */
int vt_lstm_layer_bwd_weight(const float* dgates, const float* x, int In, const float* hprev, int B, int S,
                             int hidden, float* dw_ih, float* dw_hh, float* db_ih, float* db_hh, int accumulate,
                             float* ws, int64_t ws_floats, void* stream);
/* The same with h_{t-1} read from the layer's outputs h [B, S, hidden] (row t - 1 of each
 * sample, zero at t = 0): the 16-bit forward need not write h_{t-1} (out_hprev = null).  */
int vt_lstm16_layer_bwd_weight(const float* dgates, const float* x, int In, const float* h, int B, int S,
                               int hidden, float* dw_ih, float* dw_hh, float* db_ih, float* db_hh, int accumulate,
                               float* ws, int64_t ws_floats, void* stream);

/* ---------------------------------------------------------- classifier (c4)
 * FHRInceptionTimeClassifier (ref/model/inception_time.py:185-333) on
 * (B, L, C) activations; every X / Y below is a row-major (B*L, ld) matrix
 * whose first / [col, col+C) columns are the operand (concatenations are
 * column slices of one buffer, no copies).                                     */
/* Zero-padded Conv1d(bias=False), output length L:
 *   Y[b,t,o] (+)= sum_{i,k} W[o][i][k] X[b, t+k-pad_left, i]
 * Cin, Cout multiples of 16, Cout <= 128, K in {1, 5, 15, 40}.  conv_long
 * (K 40, padding 20) yields L+1 positions in the reference, which then fails to
 * concatenate; the first L are kept (the documented crop).
 * replaces: FHRInception bottleneck1/conv_short/conv_medium/conv_long/bottleneck2,
 *           FHRResidual.bottleneck (ref/model/inception_time.py:21-71, :131-138) */
int vt_zconv_fwd(const float* X, int ldx, int B, int L, int Cin, const float* W, int Cout, int K, int pad_left,
                 float* Y, int ldy, int accumulate, void* stream);
/* dX (+)= conv of dY with the transposed, flipped taps (pad K-1-pad_left)      */
int vt_zconv_bwd_data(const float* dY, int ldy, int B, int L, int Cin, const float* W, int Cout, int K, int pad_left,
                      float* dX, int ldx, int accumulate, void* stream);
/* dW (+)= sum_{b,t} dY[b,t,o] X[b,t+k-pad_left,i]: per-workgroup slabs summed in
 * fixed order; ws >= vt_zconv_bwd_weight_ws_floats(...) floats.                */
/* The same convolution (forward / backward-data) on bf16 MFMA: operands rounded to bf16 as
 * they are staged, fp32 accumulation (the reference's 16-bit autocast; the fp32 entry points
 * above are the exact parity path).  X / dY 16-byte aligned with a row stride that is a
 * multiple of 4 floats.                                                                  */
int vt_zconv16_ws_floats(int Cin, int Cout, int K, int64_t* floats);   /* ws of the two below: the bf16 tap image */
int vt_zconv16_fwd(const float* X, int ldx, int B, int L, int Cin, const float* W, int Cout, int K, int pad_left,
                   float* Y, int ldy, int accumulate, float* ws, int64_t ws_floats, void* stream);
int vt_zconv16_bwd_data(const float* dY, int ldy, int B, int L, int Cin, const float* W, int Cout, int K, int pad_left,
                        float* dX, int ldx, int accumulate, float* ws, int64_t ws_floats, void* stream);
/* The tap images of up to 8 weights W[h] [Cout][Cin][K] in one launch (flip = 0: for
 * vt_zconv16_fwd_t; 1: the flipped, transposed taps of vt_zconv16_bwd_data_t), each into T[h]
 * (16-B aligned, vt_zconv16_taps_elems(Cin, Cout, K) bf16 elements for the forward image,
 * (Cout, Cin, K) for the flipped one) — then the convolutions read them without converting. */
int vt_zconv16_taps_elems(int Cin, int Cout, int K, int64_t* elems);
int vt_zconv16_taps(int n, const int64_t* W, const int* Cin, const int* Cout, const int* K, int flip,
                    const int64_t* T, void* stream);
int vt_zconv16_fwd_t(const float* X, int ldx, int B, int L, int Cin, const void* T, int Cout, int K, int pad_left,
                     float* Y, int ldy, int accumulate, void* stream);
int vt_zconv16_bwd_data_t(const float* dY, int ldy, int B, int L, int Cin, const void* T, int Cout, int K,
                          int pad_left, float* dX, int ldx, int accumulate, void* stream);
/* ... and the weight gradient on bf16 MFMA (transposed LDS reads of the bf16 dY / window row
 * images), fp32 accumulation and fixed-order slab sum; ws as vt_zconv_bwd_weight.      */
int vt_zconv16_bwd_weight(const float* dY, int ldy, const float* X, int ldx, int B, int L, int Cin, int Cout, int K,
                          int pad_left, float* dW, int accumulate, float* ws, int64_t ws_floats, void* stream);
int vt_zconv_bwd_weight_ws_floats(int B, int Cin, int Cout, int K, int64_t* floats);
int vt_zconv_bwd_weight(const float* dY, int ldy, const float* X, int ldx, int B, int L, int Cin, int Cout, int K,
                        int pad_left, float* dW, int accumulate, float* ws, int64_t ws_floats, void* stream);
/* MaxPool1d(kernel 3, stride 1, padding 1) over t (first maximum wins, as
 * torch's CPU kernel), and its backward (dX (+)= routed dY).
 * replaces: FHRInception.max_pool (ref/model/inception_time.py:60-64)           */
int vt_maxpool3_fwd(const float* X, int B, int L, int C, float* Y, void* stream);
int vt_maxpool3_bwd(const float* dY, const float* X, int B, int L, int C, float* dX, int accumulate, void* stream);
/* Y = act(A + Bm) elementwise (act as vt_act_fwd; backward: vt_act_bwd on Y).
 * replaces: y + residual -> relu (ref/model/inception_time.py:165-167),
 *           y_seq + attn_out (:310)                                            */
int vt_add_act_fwd(const float* A, const float* Bm, int64_t n, int act, float* Y, void* stream);
/* FHRResidual's tail fused with its Dropout1d (ref/model/inception_time.py:152-170):
 * vt_add_act_dropout_fwd: S_out = act(A + Bm) (saved), Y = Dropout1d(S_out) over L-row samples
 *   of C channels (L = 0: element-wise) — the values of vt_add_act_fwd + vt_dropout_apply;
 * vt_act_dropout_bwd: dX = Dropout1d(dY) act'(S) — the values of vt_dropout_apply +
 *   vt_act_bwd.  act: 0 none, 1 ReLU.                                                      */
int vt_add_act_dropout_fwd(const float* A, const float* Bm, int64_t n, int C, int act, int L, float p, int64_t seed,
                           const void* seed_offset, float* S_out, float* Y, void* stream);
int vt_act_dropout_bwd(const float* dY, const float* S_in, int64_t n, int C, int act, int L, float p, int64_t seed,
                       const void* seed_offset, float* dX, void* stream);
/* Dropout with a stateless counter hash: keep element i iff hash(seed, m(i)) >=
 * p * 2^32, kept values scaled by 1/(1-p); m(i) = i (nn.Dropout) or, with
 * L > 0 on (B, L, C) data, the (sample, channel) pair (nn.Dropout1d drops whole
 * channels).  The same call with the same seed is the backward (in place ok).
 * replaces: nn.Dropout / nn.Dropout1d in ref/model/inception_time.py:78,139,209,247,251 */
int vt_dropout_apply(const float* X, int64_t n, int C, int L, float p, int64_t seed, const void* seed_offset, float* Y,
                     void* stream);
/* seed_offset (vt_dropout_apply, vt_attn_fwd / _bwd): a device uint64 the caller owns, added to
 * the host seed (nullptr: none; read only when p > 0), and its per-step advance: a captured step
 * (host seeds frozen at capture) replayed by the native executor then draws new masks every
 * replay; the forward and the backward of a step pass the same offset (it advances once, at the
 * step's start).  Passed per call: no process-wide state, so two models never share an offset. */
int vt_dropout_seed_advance(void* offset, void* stream);
/* Mean over t of (B, L, C) -> (B, C); backward dX (+)= dY / L broadcast.
 * replaces: AdaptiveAvgPool1d(1) + squeeze (ref/model/inception_time.py:243,320-321) */
int vt_time_mean_fwd(const float* X, int B, int L, int C, float* Y, void* stream);
int vt_time_mean_bwd(const float* dY, int B, int L, int C, float* dX, int accumulate, void* stream);
/* Multi-head self-attention core on packed in-projections qkv (B*S, 3E),
 * E = H*32 (head dim 32), S a multiple of 16, S <= 256:
 *   O_h = dropout(softmax(Q_h K_h^T * scale)) V_h   -> out (B*S, E);  lse (B, H, S)
 * Backward writes dqkv (B*S, 3E) completely.  Attention-weight dropout uses the
 * vt_dropout_apply hash over (b, h, query, key).
 * replaces: nn.MultiheadAttention(128, 4, dropout, batch_first=True) core
 *           (ref/model/inception_time.py:236-242, :306-309)                     */
int vt_attn_fwd(const float* qkv, int B, int S, int H, float scale, float p, int64_t seed, const void* seed_offset,
                float* out, float* lse, void* stream);
int vt_attn_bwd(const float* qkv, const float* out, const float* dout, const float* lse, int B, int S, int H,
                float scale, float p, int64_t seed, const void* seed_offset, float* dqkv, void* stream);
/* nn.CrossEntropyLoss (mean) over logits (B, C), int64 labels: loss[0] and the
 * softmax probabilities; backward dlogits = g[0] * (probs - onehot) / B with
 * g a device scalar (the upstream gradient).
 * replaces: SeqVaeTebClassifier.classification_criterion (ref/model/vae_teb_model.py:1332,1488) */
int vt_cross_entropy_fwd(const float* logits, const int64_t* labels, int B, int C, float* loss, float* probs,
                         void* stream);
int vt_cross_entropy_bwd(const float* probs, const int64_t* labels, int B, int C, const float* g, float* dlogits,
                         void* stream);

/* ---- native step executor (csrc/stepgraph.cpp) ----------------------------------------
 * Runs a captured training step (a hipGraph_t, e.g. torch.cuda.CUDAGraph(keep_graph=True)
 * .raw_cuda_graph()) as a multi-stream launch list: nodes in capture order, assigned to
 * n_streams caller-provided streams, cross-stream dependencies as event waits.  The graph (its node storage and memory pool) must outlive the handle.
 * Supported nodes: kernel, 1-D memcpy / memset, empty.  In-graph RNG offsets are NOT
 * advanced (draw random inputs outside the graph).
 * replaces: the per-op Python dispatch of the eager step (ref/model/graph_model.py:692-760
 *           training_step / Lightning's optimizer loop) and ROCm's hipGraphLaunch        */
int vt_stepgraph_build(void* graph, int n_streams, void** handle);
/* enqueue one step: streams[0..n_streams) are distinct hipStream_t; the step forks
 * from streams[0] and joins back into it (stream-ordered there) */
int vt_stepgraph_launch(void* handle, void* const* streams);
int vt_stepgraph_info(void* handle, int* n_kernel, int* n_memcpy, int* n_memset, int* n_waits);
int vt_stepgraph_destroy(void* handle);
/* Data-parallel replay with the gradient all-reduce overlapped (the reference's DDP
 * reducer launches bucket all-reduces from the backward: ref/model/graph_model.py:644,
 * Lightning DDPStrategy :470-471).  vt_bucket_marker enqueues a no-op marker kernel; a step
 * captured with one marker per gradient bucket, each on a "comm" stream that has joined
 * every stream that wrote the bucket, builds an executor whose markers are not launched but
 * run on an extra stream streams[n_streams] (only their event waits): the launch list can
 * then be enqueued in ranges, and after the range that ends with a bucket's marker the
 * caller issues that bucket's collective on the comm stream (it waits only for the
 * bucket's writers, not for the rest of the backward).
 * vt_stepgraph_markers: n_ops (the length of the launch list), and for the first `cap`
 *   markers in launch order the op index just past it (ends[i]) and its bucket id.
 * vt_stepgraph_launch_range: ops [begin, end); flags bit 0 = fork every stream from
 *   streams[0] first, bit 1 = join every stream into streams[0] after.  A full step is
 *   ranges covering [0, n_ops) in order, the first with bit 0, the last with bit 1.
 *   streams has n_streams + 1 entries when the graph holds markers.                      */
int vt_bucket_marker(int bucket, void* stream);
int vt_stepgraph_markers(void* handle, int* n_ops, int* n_markers, int* ends, int* buckets, int cap);
int vt_stepgraph_launch_range(void* handle, void* const* streams, int begin, int end, int flags);

#ifdef __cplusplus
}
#endif
#endif /* VAETEB_H */
