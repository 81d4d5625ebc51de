// Whole-ResidualMLP kernels (ref/model/vae_teb_model.py:336-403):
//
//   x0 = LN_in(x);  h_0 = x0;  h_l = act_l(LN_l(h_{l-1} W_l^T + b_l))  (last
//   layer: plain Linear unless final_activation);  out = h_L + skip(x0)
//   with skip = none | identity | Linear(x0).
//
// The encoders hold 14 of these stacks (up to 33 layers, widths <= 130) over
// rows = B*S = 65,536.  Per layer the work is tiny (a 32-wide layer is 8 MB of
// activations), so a launch per layer op is latency- and launch-bound; here
// one launch runs the whole stack:
//
//  k_mlp_fwd   a wave owns 16 rows for the whole stack: its activation tile
//              lives in LDS between layers (D layout of the fp32 MFMA
//              v_mfma_f32_16x16x4_f32 written back as the next layer's A
//              operand), the layer weights are staged in 32-row chunks shared
//              by the 4 waves of the workgroup, LayerNorm + activation run in
//              the accumulator layout (16-lane shuffles).  Saves xhat / rstd of
//              every LayerNorm for the backward (h is recomputed from them).
//  k_mlp_bwd   the chain backward per 16-row wave tile, layers in reverse:
//              act' and LayerNorm backward in registers, dX = dZ W on MFMA,
//              and each layer's weight gradient dZ^T h_{l-1} over the
//              workgroup's 64 rows (h_{l-1} recomputed from the prefetched
//              xhat as act(xhat*g+b), the bias as a ones column), written with
//              the gamma/beta column partials as per-workgroup partials.
//  k_mlp_sum   every partial (dW, db, gamma, beta of every layer) summed over
//              the workgroups in fixed order into the parameter gradients
//              (accumulate or overwrite).
//
// No atomics anywhere: results are bitwise reproducible run to run.
#include <math.h>

#include "common.h"

namespace vt {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int MAXL = VT_MLP_MAX_LAYERS;
constexpr int KC = 32;          // reduction rows of W staged per step
constexpr int FWD_THREADS = 256;  // 4 waves x 16 rows

struct MlpLayer {
    int K, N, ln, act;
    const float* W;
    const float* b;
    const float* g;
    const float* be;
    // precomputed on the host (no running offsets in the kernels):
    int xo;   // xhat region of this LayerNorm: xh + R * xo   (-1 without LN)
    int ri;   // rstd row: rs + R * ri                        (-1 without LN)
    int po;   // gamma/beta partials at part[blk * P + po]     (-1 without LN)
    int dzo;  // dZ region: dz + R * dzo
    int wo;   // dW/db slab: part2 + C * wo (N * (K + 1) floats per chunk)
    int pad_;
};

struct MlpDesc {
    int L, d0, skip, pad_;
    float eps;
    int pad2_;
    const float* g0;
    const float* be0;
    const float* Ws;
    const float* bs;
    MlpLayer l[MAXL];
};

struct MlpGrads {
    float* dg0;
    float* dbe0;
    float* dWs;
    float* dbs;
    float* dW[MAXL];
    float* db[MAXL];
    float* dg[MAXL];
    float* dbe[MAXL];
};

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops,
// not for its global loads / stores (a __syncthreads() would also drain
// vmcnt, i.e. wait for the prefetched weights and the xhat / dZ stores of
// the previous layer at every barrier).  Global data written here is only
// read by later launches.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}

// sum over the 16 lanes of a DPP row (lanes with equal lane >> 4), on VALU DPP
// moves: quad xor 1, quad xor 2, half-row mirror, row mirror.  Every lane of the
// row ends with the same bits (each step adds commuted operand pairs).
__device__ __forceinline__ float sum16(float v) {
    v += dppf<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dppf<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dppf<0x141>(v);  // row_half_mirror
    v += dppf<0x140>(v);  // row_mirror
    return v;
}

__device__ __forceinline__ float mact(float z, int act) {
    switch (act) {
        case 1: return z > 0.f ? z : 0.f;
        case 2: return 0.5f * z * (1.f + erff(z * 0.70710678118654752f));
        case 3: return tanhf(z);
        default: return z;
    }
}

__device__ __forceinline__ float mact_d(float z, int act) {
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

// minimum workgroups per CU requested from the register allocator (4 waves
// each): the narrow stacks are latency-bound and gain from a second / third
// resident workgroup; the wide ones (NT >= 6) need their registers
#ifndef VT_MLP_FWD_OCC
#define VT_MLP_FWD_OCC(nt) ((nt) <= 2 ? 4 : ((nt) <= 4 ? 3 : 1))
#endif
#ifndef VT_MLP_BWD_OCC
#define VT_MLP_BWD_OCC(nt) ((nt) <= 4 ? 2 : 1)
#endif

template <int NT>
struct Cfg {
    static constexpr int W16 = 16 * NT;
    static constexpr int BS = W16 + ((NT & 1) ? 0 : 16);               // == 16 mod 32
    static constexpr int AS = W16 + (((18 - W16) % 32) + 32) % 32;     // == 18 mod 32
    static constexpr int TILE = 16 * AS;                               // one wave's 16-row tile
    static constexpr int BFL = KC * BS;                                // staged W chunk
    static constexpr int SU = (KC * W16 + FWD_THREADS - 1) / FWD_THREADS;  // staging loads per thread
    static constexpr int HS = 16 * (NT + 1) + (((NT + 1) & 1) ? 0 : 16);  // h_{l-1} tile (+ ones column), == 16 mod 32
    static constexpr int HTILE = 16 * HS;
};

// Weight chunks are staged through registers: w_load issues the global loads
// of KC reduction rows of W (one layer ahead of their use, so their latency
// overlaps the MFMAs and epilogue of the current layer) and w_store writes
// them to the shared B operand Bs[k][n].  trans: W is [Nout][Kr] (B = W^T,
// forward), else W is [Kr][Nout] (B = W, input gradient).
template <int NT>
__device__ __forceinline__ void w_load(float (&v)[Cfg<NT>::SU], const float* __restrict__ W, int Kr, int Nout,
                                       bool trans, int k0) {
    const int tid = threadIdx.x;
    constexpr int wcols = 16 * NT, tot = KC * wcols;
    const int kc = Kr - k0 < KC ? Kr - k0 : KC;
#pragma unroll
    for (int u = 0; u < Cfg<NT>::SU; ++u) {
        const int i = tid + FWD_THREADS * u;
        int k, n;
        if (trans) { n = i >> 5; k = i & 31; }
        else { k = i / wcols; n = i - k * wcols; }
        float x = 0.f;
        if (i < tot && k < kc && n < Nout) x = trans ? W[(int64_t)n * Kr + k0 + k] : W[(int64_t)(k0 + k) * Nout + n];
        v[u] = x;
    }
}

template <int NT>
__device__ __forceinline__ void w_store(const float (&v)[Cfg<NT>::SU], float* Bs, int Nout, bool trans) {
    const int tid = threadIdx.x;
    constexpr int wcols = 16 * NT, tot = KC * wcols;
    (void)Nout;
#pragma unroll
    for (int u = 0; u < Cfg<NT>::SU; ++u) {
        const int i = tid + FWD_THREADS * u;
        if (i < tot) {
            int k, n;
            if (trans) { n = i >> 5; k = i & 31; }
            else { k = i / wcols; n = i - k * wcols; }
            Bs[k * Cfg<NT>::BS + n] = v[u];
        }
    }
}

// acc[n] += A[16 rows][k0 : k0+kc] * Bs[0:kc][16n + .], A = this wave's tile Tw
template <int NT>
__device__ __forceinline__ void mfma_chunk(const float* Tw, const float* Bs, int k0, int kc, int,
                                           f32x4 (&acc)[NT]) {
    using C = Cfg<NT>;
    const int lane = threadIdx.x & 63, lr = lane & 15, lc = lane >> 4;
    const int steps = (kc + 3) >> 2;
    const float* ap = Tw + lr * C::AS + k0 + lc;
    const float* bp = Bs + lc * C::BS + lr;
    for (int s = 0; s < steps; ++s) {
        const float a = ap[4 * s];
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[n] = mfma4(a, bp[4 * s * C::BS + 16 * n], acc[n]);
    }
}

// per-lane column vector of the accumulator layout: o[n] = p[16n + lr] (0 past N or if p is null)
template <int NT>
__device__ __forceinline__ void col_load(float (&o)[NT], const float* __restrict__ p, int N) {
    const int lr = threadIdx.x & 15;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
        const int col = 16 * n + lr;
        o[n] = (p && col < N) ? p[col] : 0.f;
    }
}

// bias / gamma / beta of one layer staged through LDS PB[3][VT_MLP_MAX_WIDTH]
// (PV registers per thread, loaded one layer ahead)
constexpr int PV = (3 * VT_MLP_MAX_WIDTH + FWD_THREADS - 1) / FWD_THREADS;
__device__ __forceinline__ void p_load(float (&pv)[PV], const float* __restrict__ b, const float* __restrict__ g,
                                       const float* __restrict__ be, int N) {
#pragma unroll
    for (int u = 0; u < PV; ++u) {
        const int i = threadIdx.x + FWD_THREADS * u;
        const int which = i / VT_MLP_MAX_WIDTH, c = i - which * VT_MLP_MAX_WIDTH;
        const float* p = which == 0 ? b : which == 1 ? g : be;
        pv[u] = (which < 3 && p && c < N) ? p[c] : 0.f;
    }
}
__device__ __forceinline__ void p_store(const float (&pv)[PV], float* PB, int N) {
#pragma unroll
    for (int u = 0; u < PV; ++u) {
        const int i = threadIdx.x + FWD_THREADS * u;
        if (i < 3 * VT_MLP_MAX_WIDTH) PB[i] = pv[u];
    }
}

// 16-row wave tile of a row-major [R][N] array in the accumulator layout.
// Loads are branch-free (row / column clamped into the array, value selected);
// stores take a uniform fast path when the tile is complete (16 rows, N % 16 == 0).
template <int NT>
__device__ __forceinline__ void tile_load(float (&z)[NT][4], const float* __restrict__ src, int N, int64_t rbase,
                                          int64_t R) {
    const int lane = threadIdx.x & 63, lr = lane & 15, lc = lane >> 4;
    const int64_t last = R - 1 - rbase;  // last valid row of the tile (relative)
    const float* base = src + (rbase < R ? rbase : R - 1) * (int64_t)N;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int rr = 4 * lc + r;
        const bool rok = rr <= last;
        const int ro = rok ? rr : 0;
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            const int col = 16 * n + lr;
            const bool ok = rok && col < N;
            const float x = base[ro * N + (col < N ? col : N - 1)];
            z[n][r] = ok ? x : 0.f;
        }
    }
}

template <int NT>
__device__ __forceinline__ void tile_store(float* __restrict__ dst, const float (&z)[NT][4], int N, int64_t rbase,
                                           int64_t R) {
    const int lane = threadIdx.x & 63, lr = lane & 15, lc = lane >> 4;
    if (rbase >= R) return;
    float* base = dst + rbase * (int64_t)N;
    const int64_t last = R - 1 - rbase;
    const int nt = (N + 15) >> 4;
    if (last >= 15 && N == 16 * nt) {
#pragma unroll
        for (int n = 0; n < NT; ++n)
            if (n < nt)
#pragma unroll
                for (int r = 0; r < 4; ++r) base[(4 * lc + r) * N + 16 * n + lr] = z[n][r];
    } else {
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int rr = 4 * lc + r, col = 16 * n + lr;
                if (rr <= last && col < N) base[rr * N + col] = z[n][r];
            }
    }
}

// rstd of the tile rows (lanes with lr == 0 store)
__device__ __forceinline__ void rows_store(float* __restrict__ dst, const float (&v)[4], int64_t rbase, int64_t R) {
    const int lane = threadIdx.x & 63, lr = lane & 15, lc = lane >> 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int64_t row = rbase + 4 * lc + r;
        if (lr == 0 && row < R) dst[row] = v[r];
    }
}

__device__ __forceinline__ void rows_load(float (&v)[4], const float* __restrict__ src, int64_t rbase, int64_t R) {
    const int lane = threadIdx.x & 63, lc = lane >> 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int64_t row = rbase + 4 * lc + r;
        const float x = src[row < R ? row : R - 1];
        v[r] = row < R ? x : 0.f;
    }
}

// Row-wise LayerNorm (+ affine + act) of a 16-row wave tile held in the
// accumulator layout z[n][r] = (row 4*lc + r, col 16n + lr).  Saves xhat and
// rstd for rows < R, leaves h in z (0 for col >= N).
template <int NT>
__device__ __forceinline__ void ln_tile(float (&z)[NT][4], int N, const float (&gc)[NT], const float (&bc)[NT],
                                        int act, float eps, int64_t rbase, int64_t R, float* __restrict__ xh,
                                        float* __restrict__ rs) {
    const int lane = threadIdx.x & 63, lr = lane & 15;
    const float invN = 1.f / (float)N;
    float rsv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        float s = 0.f;
#pragma unroll
        for (int n = 0; n < NT; ++n) s += z[n][r];   // z is 0 past N
        const float mean = sum16(s) * invN;
        float v = 0.f;
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            const float d = (16 * n + lr < N) ? z[n][r] - mean : 0.f;
            z[n][r] = d;
            v += d * d;
        }
        const float rstd = rsqrtf(sum16(v) * invN + eps);
        rsv[r] = rstd;
#pragma unroll
        for (int n = 0; n < NT; ++n) z[n][r] *= rstd;   // xhat
    }
    tile_store<NT>(xh, z, N, rbase, R);
    rows_store(rs, rsv, rbase, R);
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) z[n][r] = (16 * n + lr < N) ? mact(z[n][r] * gc[n] + bc[n], act) : 0.f;
}

template <int NT>
__device__ __forceinline__ void store_tile(float* Tw, const float (&z)[NT][4], int ncols) {
    using C = Cfg<NT>;
    const int lane = threadIdx.x & 63, lr = lane & 15, lc = lane >> 4;
    (void)ncols;  // z is 0 past the valid columns: the whole 16*NT-wide tile is written
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) Tw[(4 * lc + r) * C::AS + 16 * n + lr] = z[n][r];
}

// ------------------------------------------------------------------ forward
// GEMM sequence: layers 0..L-1 (A = the activation tile T), then the skip
// projection (A = the x0 tile) when skip == 2.
template <int NT>
__global__ __launch_bounds__(FWD_THREADS, VT_MLP_FWD_OCC(NT)) void k_mlp_fwd(MlpDesc d, const float* __restrict__ X, int64_t R,
                                                         float* __restrict__ out, float* __restrict__ xh,
                                                         float* __restrict__ rs) {
    using C = Cfg<NT>;
    extern __shared__ float sm[];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lr = lane & 15, lc = lane >> 4;
    float* Bs = sm;
    float* T = sm + C::BFL + wv * C::TILE;
    float* X0 = sm + C::BFL + (4 + wv) * C::TILE;  // only when d.skip
    const int L = d.L, d0 = d.d0, DL = d.l[L - 1].N;
    const int nV = L + (d.skip == 2 ? 1 : 0);
    const int64_t rbase = (int64_t)blockIdx.x * 64 + 16 * wv;
    float* PB = sm + C::BFL + 8 * C::TILE;  // [3][144]: bias, gamma, beta of the current GEMM
    // first weight chunk + first layer's bias / LN parameters in flight with the input rows
    float v[C::SU], pv[PV];
    w_load<NT>(v, d.l[0].W, d.l[0].K, d.l[0].N, true, 0);
    p_load(pv, d.l[0].b, d.l[0].g, d.l[0].be, d.l[0].N);
    float z[NT][4];
    {
        float gi[NT], bi[NT];
        col_load<NT>(gi, d.g0, d0);
        col_load<NT>(bi, d.be0, d0);
        tile_load<NT>(z, X, d0, rbase, R);
        for (int i = lane; i < C::TILE; i += 64) {
            T[i] = 0.f;
            if (d.skip) X0[i] = 0.f;
        }
        ln_tile<NT>(z, d0, gi, bi, 0, d.eps, rbase, R, xh, rs);
    }
    store_tile<NT>(T, z, d0);
    if (d.skip) store_tile<NT>(X0, z, d0);
    for (int vl = 0; vl < nV; ++vl) {
        const bool sk = vl == L;
        const float* W = sk ? d.Ws : d.l[vl].W;
        const int Kr = sk ? d0 : d.l[vl].K, N = sk ? DL : d.l[vl].N;
        const int nt = (N + 15) >> 4;
        f32x4 acc[NT];
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
        const float* A = sk ? X0 : T;
        for (int k0 = 0; k0 < Kr; k0 += KC) {
            lds_barrier();  // readers of the previous chunk / parameters are done; A tiles are visible
            w_store<NT>(v, Bs, N, true);
            if (k0 == 0) p_store(pv, PB, N);
            lds_barrier();
            if (k0 + KC < Kr) {
                w_load<NT>(v, W, Kr, N, true, k0 + KC);
            } else if (vl + 1 < nV) {  // next layer's first chunk and parameters
                const bool sk2 = vl + 1 == L;
                const int N2 = sk2 ? DL : d.l[vl + 1].N;
                w_load<NT>(v, sk2 ? d.Ws : d.l[vl + 1].W, sk2 ? d0 : d.l[vl + 1].K, N2, true, 0);
                p_load(pv, sk2 ? d.bs : d.l[vl + 1].b, sk2 ? nullptr : d.l[vl + 1].g,
                       sk2 ? nullptr : d.l[vl + 1].be, N2);
            }
            mfma_chunk<NT>(A, Bs, k0, Kr - k0 < KC ? Kr - k0 : KC, nt, acc);
        }
        float cb[NT];
#pragma unroll
        for (int n = 0; n < NT; ++n) cb[n] = PB[16 * n + lr];
        if (!sk) {
#pragma unroll
            for (int n = 0; n < NT; ++n)
#pragma unroll
                for (int r = 0; r < 4; ++r) z[n][r] = (16 * n + lr < N) ? acc[n][r] + cb[n] : 0.f;
            if (d.l[vl].ln) {
                float cg[NT], cbe[NT];
#pragma unroll
                for (int n = 0; n < NT; ++n) {
                    cg[n] = PB[VT_MLP_MAX_WIDTH + 16 * n + lr];
                    cbe[n] = PB[2 * VT_MLP_MAX_WIDTH + 16 * n + lr];
                }
                ln_tile<NT>(z, N, cg, cbe, d.l[vl].act, d.eps, rbase, R, xh + R * d.l[vl].xo,
                            rs + R * d.l[vl].ri);
            }
            if (vl < L - 1) store_tile<NT>(T, z, N);  // the A operand of the next layer
        } else {
#pragma unroll
            for (int n = 0; n < NT; ++n)
#pragma unroll
                for (int r = 0; r < 4; ++r) z[n][r] += acc[n][r] + cb[n];
        }
    }
    if (d.skip == 1) {
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
            for (int r = 0; r < 4; ++r) z[n][r] += X0[(4 * lc + r) * C::AS + 16 * n + lr];
    }
    tile_store<NT>(out, z, DL, rbase, R);
}

// ----------------------------------------------------------------- backward
// partial layout per workgroup (P floats): [dgamma0, dbeta0 (2*d0)] then, for
// each LayerNorm layer in order, [dgamma_l, dbeta_l (2*N_l)].
// LayerNorm(+act) backward of a wave tile: g (dL/dh) -> dL/dz in place, with
// xhat / rstd / gamma / beta already in registers (prefetched).
template <int NT>
__device__ __forceinline__ void ln_bwd_tile(float (&g)[NT][4], int N, const float (&gc)[NT], const float (&bc)[NT],
                                            int act, const float (&hv)[NT][4], const float (&rsv)[4],
                                            float* red /* [2][16*NT] for this wave */) {
    const int lane = threadIdx.x & 63, lr = lane & 15, lc = lane >> 4;
    const float invN = 1.f / (float)N;
    float dgc[NT], dbc[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) dgc[n] = dbc[n] = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            const float h = hv[n][r];
            const float du = (16 * n + lr < N) ? g[n][r] * mact_d(h * gc[n] + bc[n], act) : 0.f;
            dgc[n] += du * h;
            dbc[n] += du;
            const float gv = du * gc[n];
            g[n][r] = gv;
            s1 += gv;
            s2 += gv * h;
        }
        const float m1 = sum16(s1) * invN, m2 = sum16(s2) * invN;
#pragma unroll
        for (int n = 0; n < NT; ++n) g[n][r] = (16 * n + lr < N) ? rsv[r] * (g[n][r] - m1 - hv[n][r] * m2) : 0.f;
    }
    // column partials of this wave's 16 rows: lanes l, l^16, l^32, l^48 hold the same column
#pragma unroll
    for (int n = 0; n < NT; ++n) {
        float a = dgc[n], b = dbc[n];
        a += __shfl_xor(a, 16);
        a += __shfl_xor(a, 32);
        b += __shfl_xor(b, 16);
        b += __shfl_xor(b, 32);
        if (lc == 0) {
            red[16 * n + lr] = a;
            red[16 * NT + 16 * n + lr] = b;
        }
    }
}

// after a barrier: workgroup partial = fixed-order sum of the 4 waves' partials
template <int NT>
__device__ __forceinline__ void flush_red(const float* red, int N, float* __restrict__ dst) {
    for (int i = threadIdx.x; i < 2 * N; i += FWD_THREADS) {
        const int which = i >= N, c = i - which * N;
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) t += red[w * 32 * NT + which * 16 * NT + c];
        dst[i] = t;
    }
}

// Partial dW (+ db as the ones column) of one layer over the workgroup's 64
// rows: dst[n * K1 + k] = sum_rows dZ[row][n] * H[row][k].  dZ rows are the
// 4 waves' T tiles, H rows their h_{l-1} tiles (both contiguous in LDS); the
// waves own (16 x 16) output tile pairs, two at a time.
template <int NT>
__device__ __forceinline__ void wg_dw(const float* Tall, const float* Hall, int N, int K1, float* __restrict__ dst) {
    using C = Cfg<NT>;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, lr = lane & 15, lc = lane >> 4;
    const int ntn = (N + 15) >> 4, ntk = (K1 + 15) >> 4, pairs = ntn * ntk;
    for (int p0 = wv; p0 < pairs; p0 += 8) {
        const int p1 = p0 + 4;
        const bool two = p1 < pairs;
        const int tn0 = p0 / ntk, tk0 = p0 - tn0 * ntk;
        const int tn1 = two ? p1 / ntk : tn0, tk1 = two ? p1 - tn1 * ntk : tk0;
        const float* a0 = Tall + lc * C::AS + 16 * tn0 + lr;
        const float* b0 = Hall + lc * C::HS + 16 * tk0 + lr;
        const float* a1 = Tall + lc * C::AS + 16 * tn1 + lr;
        const float* b1 = Hall + lc * C::HS + 16 * tk1 + lr;
        f32x4 c0 = f32x4{0.f, 0.f, 0.f, 0.f}, c1 = c0;
#pragma unroll 4
        for (int s4 = 0; s4 < 16; ++s4) {
            c0 = mfma4(a0[4 * s4 * C::AS], b0[4 * s4 * C::HS], c0);
            if (two) c1 = mfma4(a1[4 * s4 * C::AS], b1[4 * s4 * C::HS], c1);
        }
        const int k0c = 16 * tk0 + lr, k1c = 16 * tk1 + lr;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int n0 = 16 * tn0 + 4 * lc + r, n1 = 16 * tn1 + 4 * lc + r;
            if (n0 < N && k0c < K1) dst[n0 * K1 + k0c] = c0[r];
            if (two && n1 < N && k1c < K1) dst[n1 * K1 + k1c] = c1[r];
        }
    }
}

// this wave's h tile for the weight gradient: act(xhat * g + b) on the valid
// columns, 1 in column K (the bias), 0 beyond
template <int NT>
__device__ __forceinline__ void store_h(float* Hw, const float (&xn)[NT][4], const float (&gn)[NT],
                                        const float (&bn)[NT], int act, int K) {
    using C = Cfg<NT>;
    const int lane = threadIdx.x & 63, lr = lane & 15, lc = lane >> 4;
#pragma unroll
    for (int n = 0; n <= NT; ++n) {
        const int col = 16 * n + lr;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float h = col == K ? 1.f : 0.f;
            if (n < NT && col < K) h = mact(xn[n][r] * gn[n] + bn[n], act);
            Hw[(4 * lc + r) * C::HS + col] = h;
        }
    }
}

// GEMM sequence: the skip projection (skip == 2, A = dout), then layers
// L-1..0 (A = dZ_l).  While a layer's GEMM runs, the next weight chunk and
// the next LayerNorm's xhat / rstd / gamma / beta are already loading; that
// xhat (-> h_{l-1}) then gives the layer's weight gradient dZ_l^T h_{l-1}
// over the workgroup's rows, written as a per-workgroup partial.
// Partial layout per workgroup (P floats): [dgamma0, dbeta0 (2*d0)], then for
// each LayerNorm layer [dgamma_l, dbeta_l (2*N_l)] (ly.po); then at PL + ly.wo
// each layer's [N][K+1] dW|db, and the skip projection's [DL][d0+1] last.
template <int NT>
__global__ __launch_bounds__(FWD_THREADS, VT_MLP_BWD_OCC(NT)) void k_mlp_bwd(MlpDesc d, const float* __restrict__ dout,
                                                         const float* __restrict__ xh, const float* __restrict__ rs,
                                                         int64_t R, float* __restrict__ dx,
                                                         float* __restrict__ part, int P, int PL, int wskip) {
    using C = Cfg<NT>;
    extern __shared__ float sm[];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lr = lane & 15, lc = lane >> 4;
    float* Bs = sm;
    float* Tall = sm + C::BFL;
    float* T = Tall + wv * C::TILE;
    float* G0 = sm + C::BFL + (4 + wv) * C::TILE;       // skip gradient (d.skip)
    float* Hall = sm + C::BFL + 8 * C::TILE;            // [4 waves][16][HS]
    float* H = Hall + wv * C::HTILE;
    float* red = Hall + 4 * C::HTILE;                   // [4 waves][2][16*NT]
    float* redw = red + wv * 32 * NT;
    const int64_t rbase = (int64_t)blockIdx.x * 64 + 16 * wv;
    const int L = d.L, d0 = d.d0, DL = d.l[L - 1].N;
    float* pb = part + (int64_t)blockIdx.x * P;
    float xn[NT][4], rn[4], gn[NT], bn[NT];  // the next LayerNorm's saved state (prefetched)
#define VT_LN_PREFETCH(q)                                                                      \
    do {                                                                                       \
        const int q_ = (q);                                                                    \
        const int Nq = q_ >= 0 ? d.l[q_].N : d0;                                               \
        tile_load<NT>(xn, xh + (q_ >= 0 ? R * d.l[q_].xo : 0), Nq, rbase, R);                  \
        rows_load(rn, rs + (q_ >= 0 ? R * d.l[q_].ri : 0), rbase, R);                          \
        col_load<NT>(gn, q_ >= 0 ? d.l[q_].g : d.g0, Nq);                                      \
        col_load<NT>(bn, q_ >= 0 ? d.l[q_].be : d.be0, Nq);                                    \
    } while (0)

    float v[C::SU];
    if (d.skip == 2) w_load<NT>(v, d.Ws, DL, d0, false, 0);
    else w_load<NT>(v, d.l[L - 1].W, d.l[L - 1].N, d.l[L - 1].K, false, 0);
    float g[NT][4];
    tile_load<NT>(g, dout, DL, rbase, R);
    if (d.skip != 2 && d.l[L - 1].ln) VT_LN_PREFETCH(L - 1);
    for (int i = lane; i < C::TILE; i += 64) {
        T[i] = 0.f;
        G0[i] = 0.f;
    }
    if (d.skip == 1) {
        store_tile<NT>(G0, g, DL);
    } else if (d.skip == 2) {
        store_tile<NT>(T, g, DL);
        f32x4 acc[NT];
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int k0 = 0; k0 < DL; k0 += KC) {
            lds_barrier();
            w_store<NT>(v, Bs, d0, false);
            lds_barrier();
            if (k0 + KC < DL) {
                w_load<NT>(v, d.Ws, DL, d0, false, k0 + KC);
            } else {
                w_load<NT>(v, d.l[L - 1].W, d.l[L - 1].N, d.l[L - 1].K, false, 0);
                if (d.l[L - 1].ln) VT_LN_PREFETCH(L - 1);
            }
            mfma_chunk<NT>(T, Bs, k0, DL - k0 < KC ? DL - k0 : KC, 0, acc);  // d x0 += dout Ws
        }
        float t[NT][4];
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
            for (int r = 0; r < 4; ++r) t[n][r] = acc[n][r];
        store_tile<NT>(G0, t, d0);
    }
    for (int l = L - 1; l >= 0; --l) {
        const MlpLayer& ly = d.l[l];
        const int N = ly.N, K = ly.K;
        if (ly.ln) ln_bwd_tile<NT>(g, N, gn, bn, ly.act, xn, rn, redw);
        lds_barrier();  // the previous layer's weight-gradient MFMAs are done with the T tiles
        store_tile<NT>(T, g, N);
        lds_barrier();
        if (ly.ln) flush_red<NT>(red, N, pb + ly.po);
        f32x4 acc[NT];
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int k0 = 0; k0 < N; k0 += KC) {
            lds_barrier();
            w_store<NT>(v, Bs, K, false);
            lds_barrier();
            if (k0 + KC < N) {
                w_load<NT>(v, ly.W, N, K, false, k0 + KC);
            } else {
                if (l >= 1) w_load<NT>(v, d.l[l - 1].W, d.l[l - 1].N, d.l[l - 1].K, false, 0);
                VT_LN_PREFETCH(l - 1);  // layer l-1 (a hidden layer: always normalised) or the input LN
            }
            mfma_chunk<NT>(T, Bs, k0, N - k0 < KC ? N - k0 : KC, 0, acc);  // dh_{l-1} = dZ W
        }
        // weight gradient of layer l: dZ_l (T tiles) ^T h_{l-1} (from the prefetched xhat)
        store_h<NT>(H, xn, gn, bn, l >= 1 ? d.l[l - 1].act : 0, K);
        lds_barrier();
        wg_dw<NT>(Tall, Hall, N, K + 1, pb + PL + ly.wo);
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
            for (int r = 0; r < 4; ++r) g[n][r] = acc[n][r];
    }
#undef VT_LN_PREFETCH
    if (d.skip == 2) {  // dWs = dout^T x0 (H still holds x0)
        float t[NT][4];
        tile_load<NT>(t, dout, DL, rbase, R);
        lds_barrier();
        store_tile<NT>(T, t, DL);
        lds_barrier();
        wg_dw<NT>(Tall, Hall, DL, d0 + 1, pb + PL + wskip);
    }
    if (d.skip) {
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
            for (int r = 0; r < 4; ++r) g[n][r] += G0[(4 * lc + r) * C::AS + 16 * n + lr];
    }
    ln_bwd_tile<NT>(g, d0, gn, bn, 0, xn, rn, redw);
    tile_store<NT>(dx, g, d0, rbase, R);
    lds_barrier();
    flush_red<NT>(red, d0, pb);
}

// ---------------------------------------------------------------- final sum
// segment s < nG: the dW|db partials of layer s (s == L: the skip projection);
// s >= nG: the gamma/beta partials of LayerNorm s - nG (layer s - nG < L, or
// the input norm when == L); summed over the nblk chain workgroups in fixed
// order (16 outputs x 16 partial lanes per block, then a fixed tree).
__global__ __launch_bounds__(256) void k_mlp_sum(MlpDesc d, MlpGrads gr, int nG, const float* __restrict__ part,
                                                 int nblk, int P, int PL, int wskip, int accumulate) {
    __shared__ float red[16][17];
    const int s = blockIdx.y;
    const int o = threadIdx.x & 15, sl = threadIdx.x >> 4;
    const float* src;
    int E, N = 0, K1 = 0;
    float *da, *dbp;
    const bool dwseg = s < nG;
    if (dwseg) {
        if (s < d.L) {
            N = d.l[s].N;
            K1 = d.l[s].K + 1;
            da = gr.dW[s];
            dbp = gr.db[s];
            src = part + PL + d.l[s].wo;
        } else {
            N = d.l[d.L - 1].N;
            K1 = d.d0 + 1;
            da = gr.dWs;
            dbp = gr.dbs;
            src = part + PL + wskip;
        }
        E = N * K1;
    } else {
        const int q = s - nG;
        if (q < d.L) {
            if (!d.l[q].ln) return;
            N = d.l[q].N;
            da = gr.dg[q];
            dbp = gr.dbe[q];
            src = part + d.l[q].po;
        } else {
            N = d.d0;
            da = gr.dg0;
            dbp = gr.dbe0;
            src = part;
        }
        E = 2 * N;
    }
    if ((int64_t)blockIdx.x * 16 >= E) return;
    const int i = blockIdx.x * 16 + o;
    // 4 interleaved accumulators, 4 loads in flight per thread (a single
    // dependent chain of nblk/16 loads was latency-bound)
    float a4[4] = {0.f, 0.f, 0.f, 0.f};
    if (i < E) {
        int b = sl;
        for (; b + 48 < nblk; b += 64)
#pragma unroll
            for (int u = 0; u < 4; ++u) a4[u] += src[(int64_t)(b + 16 * u) * P + i];
        for (int u = 0; b < nblk; b += 16, ++u) a4[u & 3] += src[(int64_t)b * P + i];
    }
    const float a = (a4[0] + a4[1]) + (a4[2] + a4[3]);
    red[sl][o] = a;
    __syncthreads();
    if (sl != 0 || i >= E) return;
    float t8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) t8[j] = red[2 * j][o] + red[2 * j + 1][o];
#pragma unroll
    for (int j = 0; j < 4; ++j) t8[j] = t8[2 * j] + t8[2 * j + 1];
    const float t = (t8[0] + t8[1]) + (t8[2] + t8[3]);
    float* dst;
    if (dwseg) {
        const int n = i / K1, k = i - n * K1;
        const int K = K1 - 1;
        dst = k < K ? (da ? da + (int64_t)n * K + k : nullptr) : (dbp ? dbp + n : nullptr);
    } else {
        dst = i < N ? (da ? da + i : nullptr) : (dbp ? dbp + (i - N) : nullptr);
    }
    if (dst) *dst = accumulate ? *dst + t : t;
}

// ---------------------------------------------------------------- host side
struct Plan {
    MlpDesc d;
    int nt;
    int64_t xh_floats, rs_floats, P, PL, wskip, nblk;
};

int make_plan(Plan& p, int n_layers, const int* dims, const int* layer_ln, const int* layer_act, int skip, float eps,
              const float* const* params, int64_t R, const char* who) {
    VT_CHECK_ARG(n_layers >= 1 && n_layers <= MAXL, "%s: n_layers %d not in [1, %d]", who, n_layers, MAXL);
    VT_CHECK_ARG(skip >= 0 && skip <= 2, "%s: skip %d", who, skip);
    VT_CHECK_ARG(R >= 1, "%s: rows %lld", who, (long long)R);
    MlpDesc& d = p.d;
    d = MlpDesc{};
    d.L = n_layers;
    d.d0 = dims[0];
    d.skip = skip;
    d.eps = eps;
    int wmax = dims[0];
    int n_ln = 0;
    int64_t sum_ln = 0, sum_n = 0, sum_nk = 0;
    for (int l = 0; l < n_layers; ++l) {
        const int K = dims[l], N = dims[l + 1];
        VT_CHECK_ARG(K >= 1 && N >= 1 && K <= VT_MLP_MAX_WIDTH && N <= VT_MLP_MAX_WIDTH,
                     "%s: layer %d width %d -> %d outside [1, %d]", who, l, K, N, VT_MLP_MAX_WIDTH);
        VT_CHECK_ARG(layer_ln[l] || l == n_layers - 1, "%s: hidden layer %d without LayerNorm", who, l);
        VT_CHECK_ARG(layer_ln[l] || layer_act[l] == 0, "%s: activation without LayerNorm (layer %d)", who, l);
        VT_CHECK_ARG(layer_act[l] >= 0 && layer_act[l] <= 3, "%s: act %d", who, layer_act[l]);
        MlpLayer& ly = d.l[l];
        ly.K = K;
        ly.N = N;
        ly.ln = layer_ln[l] ? 1 : 0;
        ly.act = layer_act[l];
        ly.W = params[2 + 4 * l];
        ly.b = params[3 + 4 * l];
        ly.g = params[4 + 4 * l];
        ly.be = params[5 + 4 * l];
        VT_CHECK_ARG(ly.W && (!ly.ln || (ly.g && ly.be)), "%s: missing parameter of layer %d", who, l);
        wmax = N > wmax ? N : wmax;
        ly.dzo = (int)sum_n;
        ly.wo = (int)sum_nk;
        sum_n += N;
        sum_nk += (int64_t)N * (K + 1);
        if (ly.ln) {
            ly.xo = (int)(dims[0] + sum_ln);
            ly.ri = 1 + n_ln;
            ly.po = (int)(2 * (dims[0] + sum_ln));
            ++n_ln;
            sum_ln += N;
        } else {
            ly.xo = ly.ri = ly.po = -1;
        }
    }
    d.g0 = params[0];
    d.be0 = params[1];
    d.Ws = params[2 + 4 * n_layers];
    d.bs = params[3 + 4 * n_layers];
    VT_CHECK_ARG(d.g0 && d.be0, "%s: missing input LayerNorm parameters", who);
    VT_CHECK_ARG(skip != 1 || dims[0] == dims[n_layers], "%s: identity skip needs in == out width", who);
    VT_CHECK_ARG(skip != 2 || d.Ws, "%s: projection skip without weight", who);
    const int ntw = (wmax + 15) / 16;
    p.nt = ntw <= 2 ? 2 : ntw <= 4 ? 4 : ntw <= 6 ? 6 : 9;
    p.xh_floats = R * (dims[0] + sum_ln);
    p.rs_floats = R * (1 + n_ln);
    p.PL = 2 * (dims[0] + sum_ln);
    p.wskip = sum_nk;
    if (skip == 2) sum_nk += (int64_t)dims[n_layers] * (dims[0] + 1);
    p.P = p.PL + sum_nk;
    p.nblk = (R + 63) / 64;
    VT_CHECK_ARG(p.xh_floats < (int64_t)1 << 31 && p.nblk * p.P < ((int64_t)1 << 40), "%s: too many rows", who);
    return VT_OK;
}

template <int NT>
size_t fwd_lds(int) {
    return sizeof(float) * (Cfg<NT>::BFL + 8 * Cfg<NT>::TILE + 3 * VT_MLP_MAX_WIDTH);
}
template <int NT>
size_t bwd_lds() {
    return sizeof(float) * (Cfg<NT>::BFL + 8 * Cfg<NT>::TILE + 4 * Cfg<NT>::HTILE + 4 * 32 * NT);
}

}  // namespace
}  // namespace vt

using namespace vt;

extern "C" {

int vt_resmlp_sizes(int n_layers, const int* dims, const int* layer_ln, const int* layer_act, int skip,
                    int64_t rows, int64_t* sizes) {
    // params are not needed for the sizes: validate with dummy non-null pointers
    const float* dummy[4 * MAXL + 4];
    for (int i = 0; i < 4 * MAXL + 4; ++i) dummy[i] = reinterpret_cast<const float*>(16);
    Plan p;
    const int rc = make_plan(p, n_layers, dims, layer_ln, layer_act, skip, 1e-5f, dummy, rows, "vt_resmlp_sizes");
    if (rc) return rc;
    sizes[0] = p.xh_floats;
    sizes[1] = p.rs_floats;
    sizes[2] = p.nblk * p.P;
    return VT_OK;
}

int vt_resmlp_fwd(int n_layers, const int* dims, const int* layer_ln, const int* layer_act, int skip, float eps,
                  const float* const* params, const float* x, int64_t rows, float* out, float* xhat, float* rstd,
                  void* stream) {
    Plan p;
    const int rc = make_plan(p, n_layers, dims, layer_ln, layer_act, skip, eps, params, rows, "vt_resmlp_fwd");
    if (rc) return rc;
    VT_CHECK_ARG(x && out && xhat && rstd, "vt_resmlp_fwd: null buffer");
    const dim3 grid((unsigned)p.nblk);
    hipStream_t st = S(stream);
    switch (p.nt) {
        case 2: hipLaunchKernelGGL(k_mlp_fwd<2>, grid, dim3(FWD_THREADS), fwd_lds<2>(skip), st, p.d, x, rows, out, xhat, rstd); break;
        case 4: hipLaunchKernelGGL(k_mlp_fwd<4>, grid, dim3(FWD_THREADS), fwd_lds<4>(skip), st, p.d, x, rows, out, xhat, rstd); break;
        case 6: hipLaunchKernelGGL(k_mlp_fwd<6>, grid, dim3(FWD_THREADS), fwd_lds<6>(skip), st, p.d, x, rows, out, xhat, rstd); break;
        default: hipLaunchKernelGGL(k_mlp_fwd<9>, grid, dim3(FWD_THREADS), fwd_lds<9>(skip), st, p.d, x, rows, out, xhat, rstd); break;
    }
    VT_LAUNCH_CHECK("vt_resmlp_fwd");
    return VT_OK;
}

int vt_resmlp_bwd(int n_layers, const int* dims, const int* layer_ln, const int* layer_act, int skip, float eps,
                  const float* const* params, const float* dout, const float* xhat, const float* rstd, int64_t rows,
                  float* dx, float* const* grads, int accumulate, float* ws, int64_t ws_floats, void* stream) {
    Plan p;
    const int rc = make_plan(p, n_layers, dims, layer_ln, layer_act, skip, eps, params, rows, "vt_resmlp_bwd");
    if (rc) return rc;
    VT_CHECK_ARG(dout && xhat && rstd && dx && grads, "vt_resmlp_bwd: null buffer");
    VT_CHECK_ARG(ws && ws_floats >= p.nblk * p.P, "vt_resmlp_bwd: workspace %lld floats < %lld",
                 (long long)ws_floats, (long long)(p.nblk * p.P));
    MlpGrads g{};
    g.dg0 = grads[0];
    g.dbe0 = grads[1];
    for (int l = 0; l < n_layers; ++l) {
        g.dW[l] = grads[2 + 4 * l];
        g.db[l] = grads[3 + 4 * l];
        g.dg[l] = grads[4 + 4 * l];
        g.dbe[l] = grads[5 + 4 * l];
    }
    g.dWs = grads[2 + 4 * n_layers];
    g.dbs = grads[3 + 4 * n_layers];
    hipStream_t st = S(stream);
    const dim3 grid((unsigned)p.nblk);
    const int P = (int)p.P, PL = (int)p.PL, wskip = (int)p.wskip;
    const int nG = n_layers + (skip == 2 ? 1 : 0);
    switch (p.nt) {
#define VT_MLPB(NTV)                                                                                               \
    case NTV:                                                                                                      \
        hipLaunchKernelGGL(k_mlp_bwd<NTV>, grid, dim3(FWD_THREADS), bwd_lds<NTV>(), st, p.d, dout, xhat, rstd,     \
                           rows, dx, ws, P, PL, wskip);                                                            \
        break;
        VT_MLPB(2) VT_MLPB(4) VT_MLPB(6)
        default: VT_MLPB(9)
#undef VT_MLPB
    }
    int emax = 2 * p.d.d0;
    for (int l = 0; l < n_layers; ++l) {
        const int e = p.d.l[l].N * (p.d.l[l].K + 1);
        emax = e > emax ? e : emax;
    }
    if (skip == 2) emax = dims[n_layers] * (dims[0] + 1) > emax ? dims[n_layers] * (dims[0] + 1) : emax;
    const dim3 gs((unsigned)((emax + 15) / 16), (unsigned)(nG + n_layers + 1));
    hipLaunchKernelGGL(k_mlp_sum, gs, dim3(256), 0, st, p.d, g, nG, ws, (int)p.nblk, P, PL, wskip, accumulate);
    VT_LAUNCH_CHECK("vt_resmlp_bwd");
    return VT_OK;
}

}  // extern "C"
