// bf16 MFMA GEMM for the decoder's dense R x R output heads
// (Decoder.output_mu / output_logvar, ref/model/vae_teb_model.py:882-897,926-927
// with R = 16*S): Y = X W^T + b, dX = dY W, dW = dY^T X — the only true GEMMs of the
// step (every other layer is <= 130 wide and stays on the fp32 kernels).
//
// One kernel, C[M,N] = sum_k A[m,k] B[n,k] with A and B bf16, K-contiguous:
//   * v_mfma_f32_16x16x32_bf16, fp32 accumulation;
//   * block tile 256(M) x 64(N) x 64(K), 8 waves stacked in M, each wave
//     32 x 64 = 2 x 4 MFMA tiles;
//   * operands reach LDS by LDS-DMA (global_load_lds_dwordx4, no VGPR staging):
//     3 LDS stages, tiles t+1 and t+2 in flight while tile t is multiplied,
//     counted vmcnt + raw s_barrier (the M = 256 shape is load-latency bound);
//     rows are 128 B, 16-B chunks XOR-swizzled on the SOURCE address so the
//     ds_read_b128 fragment reads are bank-conflict free;
//   * split-K so that tiles x splits ~ the 256 CUs; the split partials are combined by the
//     workgroup of the tile that arrives last (common.h last_arrival), in the fixed split order
//     (((p0 + p1) + p2) + ...) + bias, then + C — the order of the separate reduce pass this
//     replaced (k_mfma_reduce4, 8 launches / 68 us per step in round 5), so the same bits.
// Operand images: the weight side is a bf16 shadow of the fp32 master weights
// (W for the forward, W^T for the input gradient) refreshed by
// vt_mfma_weight_shadow; the activation side (X, dY, X^T, dY^T) is converted by
// small prep kernels into zero-padded images, so the main loop has no predicates.
#include "h16.h"

namespace vt {

constexpr int QM = 256, QN = 64, QK = 64, QT = 512;
constexpr int ROWB = QK * 2;                      // 128 B per operand row in LDS
constexpr int A_BYTES = QM * ROWB;                // 32 KB per A stage (the activations: L2-resident)
constexpr int B_BYTES = QN * ROWB;                // 8 KB per B stage (the weights: streamed from HBM)
// A (shared by every workgroup of the launch, L2 hits) two tiles ahead; B (each weight tile read
// by the launch's only M-tile, i.e. once: HBM misses, ~3 us under load) NB - 1 tiles ahead.  With
// both operands two tiles ahead the loop ran at the HBM-miss latency / 2 per tile (~1.6 us).
constexpr int NA = 3, NB = 8;
constexpr int GEMM_LDS = NA * A_BYTES + NB * B_BYTES;   // 160 KB

// 16-B chunk position of chunk c in LDS row r (involution)
__device__ __forceinline__ int swz(int r, int c) { return c ^ ((r >> 1) & 7); }

__device__ __forceinline__ void glds16(const void* src, char* lds) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

VT_ARRIVE_POOL(g_arrive_gemm);

// b128 agent-coherent (sc1) accesses of the split partials
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_agent4(__amdgpu_buffer_rsrc_t r, unsigned off, f32x4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (int)off, 0, CPOL_SC1);
}
__device__ __forceinline__ f32x4 ld_agent4(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, CPOL_SC1));
}

// common.h last_arrival with its flag in the kernel's (by then unused) dynamic LDS: the
// operand stages take all 160 KB, so a static __shared__ word would not fit beside them
__device__ __forceinline__ bool last_arrival_in(unsigned* ctr, unsigned total, unsigned* flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();   // every wave is past its last LDS read of the stages
    if (threadIdx.x == 0) {
        const unsigned old = atomicAdd(ctr, 1u);
        const bool last = old == total - 1;
        if (last) atomicExch(ctr, 0u);
        *flag = last ? 1u : 0u;
    }
    __syncthreads();
    return *flag != 0u;
}

// grid (N/64, Mpad/256, splits); K = reduction length of ONE split (multiple of 64).  splits > 1:
// part holds tiles x splits slabs of 512 x 32 floats (a thread's 32 accumulators as 8 float4,
// wave-contiguous), slot0 the tiles' arrival counters
template <typename H>
__global__ __launch_bounds__(QT) void k_mfma_gemm(const H* __restrict__ A, int64_t lda,
                                                  const H* __restrict__ B, int64_t ldb, int M, int N, int K,
                                                  float* __restrict__ C, int64_t ldc, const float* __restrict__ bias,
                                                  int accumulate, float* __restrict__ part, unsigned slot0) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* sa = smem;                     // NA stages of A
    char* sb = smem + NA * A_BYTES;      // NB stages of B
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int n0 = blockIdx.x * QN, m0 = blockIdx.y * QM;
    const int64_t kbeg = (int64_t)blockIdx.z * K;
    const int T = K / QK;

    // LDS-DMA of one k-tile: lane l writes LDS byte (base + 16 l) = row l>>3, position l&7
    const int rsub = lane >> 3, pos = lane & 7;
    auto kof = [&](int t) { return kbeg + (int64_t)(t < T ? t : T - 1) * QK; };  // past the end: re-read, unused
    auto issue_a = [&](int t) {          // 4 DMAs per wave
        const int64_t k0 = kof(t);
        char* st = sa + (t % NA) * A_BYTES;
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // A rows 32w + 8i .. +7
            const int r = 32 * w + 8 * i + rsub;
            glds16(A + (int64_t)(m0 + r) * lda + k0 + 8 * swz(r, pos), st + (32 * w + 8 * i) * ROWB);
        }
    };
    auto issue_b = [&](int t) {          // 1 DMA per wave
        const int64_t k0 = kof(t);
        const int r = 8 * w + rsub;  // B rows 8w .. 8w+7
        glds16(B + (int64_t)(n0 + r) * ldb + k0 + 8 * swz(r, pos), sb + (t % NB) * B_BYTES + 8 * w * ROWB);
    };

    f32x4 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int lr = lane & 15, lc = lane >> 4;
    auto compute = [&](int t) {
        const char* ta = sa + (t % NA) * A_BYTES;
        const char* tb = sb + (t % NB) * B_BYTES;
#pragma unroll
        for (int h = 0; h < 2; ++h) {  // k 0..31, 32..63: chunks 4h + lc
            const int c = 4 * h + lc;
            hv8<H> af[2], bfr[4];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int r = 32 * w + 16 * i + lr;
                af[i] = *(const hv8<H>*)(ta + r * ROWB + 16 * swz(r, c));
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int r = 16 * j + lr;
                bfr[j] = *(const hv8<H>*)(tb + r * ROWB + 16 * swz(r, c));
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
        }
    };

    // prologue: B tiles 0 .. NB-2, then A tiles 0, 1.  Loop t issues A(t+2), B(t+NB-1) after its
    // barrier, so the DMAs younger than A(t) when tile t is needed are: t = 0: A(1) (4);
    // t = 1: A(2), B(NB) (5); t >= 2: B(t+NB-3), A(t+1), B(t+NB-2) (6).  B(t) is older than A(t).
#pragma unroll
    for (int t = 0; t < NB - 1; ++t) issue_b(t);
    issue_a(0);
    issue_a(1);
    for (int t = 0; t < T; ++t) {
        if (t == 0) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else if (t == 1) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // tile t complete for all waves; all waves done with tile t-1
        issue_a(t + 2);                // overwrites A stage (t-1) % NA, B stage (t-1) % NB: both consumed
        issue_b(t + NB - 1);
        compute(t);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the re-read DMAs before the block exits

    if (part) {
        // this split's partial, then the tile's last arrival sums the splits in index order
        const int splits = gridDim.z, z = blockIdx.z;
        const unsigned tile = blockIdx.y * gridDim.x + blockIdx.x;
        const int64_t slab = (int64_t)QT * 32 * 4;                    // bytes per (tile, split)
        const __amdgpu_buffer_rsrc_t pr = agent_rsrc(part + (int64_t)tile * splits * QT * 32, splits * slab);
#pragma unroll
        for (int g = 0; g < 8; ++g) st_agent4(pr, (unsigned)(z * slab + (g * QT + tid) * 16), acc[g >> 2][g & 3]);
        if (!last_arrival_in(&g_arrive_gemm[slot0 + tile], (unsigned)splits, (unsigned*)smem)) return;
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            f32x4 s = z == 0 ? acc[g >> 2][g & 3] : ld_agent4(pr, (unsigned)((g * QT + tid) * 16));
            for (int p = 1; p < splits; ++p)
                s += p == z ? acc[g >> 2][g & 3] : ld_agent4(pr, (unsigned)(p * slab + (g * QT + tid) * 16));
            acc[g >> 2][g & 3] = s;
        }
    }
    // C/D layout of 16x16x32: col = lane & 15, row = 4 * (lane >> 4) + r
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int col = n0 + 16 * j + lr;
            const float bcol = bias ? bias[col] : 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = m0 + 32 * w + 16 * i + 4 * lc + r;
                if (row >= M) continue;
                float o = acc[i][j][r] + bcol;
                if (accumulate) o = C[(int64_t)row * ldc + col] + o;
                C[(int64_t)row * ldc + col] = o;
            }
        }
}

// out[m][k] = H(X[m][k]) for m < M, k < K; zero in the padding (Mpad x Kpad)
template <typename H>
__global__ void k_bf16_rows(const float* __restrict__ X, int64_t M, int K, H* __restrict__ out, int64_t Mpad,
                            int Kpad) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = Mpad * Kpad;
    if (i >= total) return;
    const int64_t m = i / Kpad;
    const int k = (int)(i - m * Kpad);
    out[i] = (m < M && k < K) ? (H)X[m * K + k] : (H)0.f;
}

// out[c][r] = H(X[r][c]) (X is R x Cn row-major); zero padded to Cpad x Rpad
template <typename H>
__global__ __launch_bounds__(256) void k_bf16_transpose(const float* __restrict__ X, int64_t R, int Cn,
                                                        H* __restrict__ out, int64_t Cpad, int64_t Rpad) {
    __shared__ float tile[64][65];
    const int64_t r0 = (int64_t)blockIdx.x * 64, c0 = (int64_t)blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int i = ty; i < 64; i += 4) {
        const int64_t r = r0 + i, c = c0 + tx;
        tile[i][tx] = (r < R && c < Cn) ? X[r * Cn + c] : 0.f;
    }
    __syncthreads();
    for (int i = ty; i < 64; i += 4) {
        const int64_t c = c0 + i, r = r0 + tx;
        if (c < Cpad && r < Rpad) out[c * Rpad + r] = (H)tile[tx][i];
    }
}

// W fp32 [N][K] -> W16 = H(W) [N][K] and W16t = H(W)^T [K][N]  (N, K multiples of 64)
template <typename H>
__global__ __launch_bounds__(256) void k_bf16_shadow(const float* __restrict__ W, int N, int K,
                                                     H* __restrict__ W16, H* __restrict__ W16t) {
    __shared__ float tile[64][65];
    const int64_t n0 = (int64_t)blockIdx.y * 64, k0 = (int64_t)blockIdx.x * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int i = ty; i < 64; i += 4) {
        const float v = W[(n0 + i) * K + k0 + tx];
        tile[i][tx] = v;
        W16[(n0 + i) * K + k0 + tx] = (H)v;
    }
    __syncthreads();
    for (int i = ty; i < 64; i += 4) W16t[(k0 + i) * N + n0 + tx] = (H)tile[tx][i];
}

// ------------------------------------------------------------ weight gradient
// dW[n][k] (+)= sum_r dY[r][n] X[r][k] with the batch rows r as the (short)
// reduction (R = 256 for the heads): a 128 x 128 tile per workgroup of 4
// waves (2 x 2, 64 x 64 each), 64-row chunks of dY and X staged from fp32 to
// bf16 row-major images in LDS (the next chunk prefetched into registers while
// the current one is multiplied) and read as MFMA fragments with the gfx950
// transposed read ds_read_b64_tr_b16 (r contiguous per fragment) — no
// transposed bf16 copies in HBM, no split-K slabs.  39 KB of LDS and 256
// threads: it runs beside the decoder's backward on the other stream instead of
// waiting for a whole CU.
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef short v8i16 __attribute__((ext_vector_type(8)));
constexpr int DWT = 128, DWC = 64;              // tile edge, rows per chunk
constexpr int DWS = DWT + 16;                   // bf16 row stride (72 dwords == 8 mod 64 banks)
constexpr int DWIMG = DWC * DWS + (DWC / 8) * 64;  // + 32 dwords every 8 rows: rows 8 apart -> banks +32

__device__ __forceinline__ int dw_pos(int r, int c) { return r * DWS + (r >> 3) * 64 + c; }

// 16 x 32 fragment (16 columns col0.., 32 rows row0..) of a [r][col] image, r the reduction:
// lane 4q + p of 16-lane group g reads rows row0 + 8g + q (+4), columns col0 + 4p .. +3
template <typename H>
__device__ __forceinline__ hv8<H> dw_frag(const H* img, int row0, int col0) {
    const int lane = threadIdx.x & 63, g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const H* a0 = img + dw_pos(row0 + 8 * g + q, col0 + 4 * p);
    const H* a1 = img + dw_pos(row0 + 8 * g + q + 4, col0 + 4 * p);
    const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)a0);
    const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)a1);
    const v8i16 r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(hv8<H>, r);
}

template <typename H>
__global__ __launch_bounds__(256) void k_mfma_dw(const float* __restrict__ dY, int64_t R, int N,
                                                 const float* __restrict__ X, int K, float* __restrict__ dW,
                                                 int accumulate) {
    __shared__ __attribute__((aligned(16))) H img[2][DWIMG];  // [0] dY chunk, [1] X chunk
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
    const int n0 = blockIdx.y * DWT, k0 = blockIdx.x * DWT;
    // staging: chunk rows r0 .. r0 + 63, 32 float4 per row per operand; thread -> (row, quad) pairs
    float4 pf[2][8];
    auto load = [&](int64_t r0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int e = tid + 256 * i, row = e >> 5, q4 = e & 31;
            const bool ok = r0 + row < R;
            pf[0][i] = ok ? *(const float4*)(dY + (r0 + row) * N + n0 + 4 * q4) : make_float4(0.f, 0.f, 0.f, 0.f);
            pf[1][i] = ok ? *(const float4*)(X + (r0 + row) * K + k0 + 4 * q4) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto store = [&]() {
#pragma unroll
        for (int o = 0; o < 2; ++o)
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int e = tid + 256 * i, row = e >> 5, q4 = e & 31;
                const hv4<H> v = {(H)pf[o][i].x, (H)pf[o][i].y, (H)pf[o][i].z, (H)pf[o][i].w};
                *(hv4<H>*)(img[o] + dw_pos(row, 4 * q4)) = v;
            }
    };
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    load(0);
    for (int64_t r0 = 0; r0 < R; r0 += DWC) {
        store();
        __syncthreads();
        if (r0 + DWC < R) load(r0 + DWC);
#pragma unroll
        for (int s = 0; s < DWC / 32; ++s) {
            hv8<H> a[4], b[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = dw_frag(img[0], 32 * s, 64 * wm + 16 * i);
#pragma unroll
            for (int j = 0; j < 4; ++j) b[j] = dw_frag(img[1], 32 * s, 64 * wn + 16 * j);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = mfma16(a[i], b[j], acc[i][j]);
        }
        __syncthreads();
    }
    // D: col (k) = lane & 15, row (n) = 4 * (lane >> 4) + rr.  Accumulating: every
    // old value is loaded before the first store (one round trip, not 64: the compiler
    // cannot prove the 64 addresses distinct for a runtime K, so an interleaved
    // load / store sequence would serialise)
    const int lr = lane & 15, lc = lane >> 4;
    float* c0 = dW + (int64_t)(n0 + 64 * wm + 4 * lc) * K + k0 + 64 * wn + lr;
    if (accumulate) {
        f32x4 old[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) old[i][j][rr] = c0[(int64_t)(16 * i + rr) * K + 16 * j];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] += old[i][j];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) c0[(int64_t)(16 * i + rr) * K + 16 * j] = acc[i][j][rr];
}

static inline int64_t up_to(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

// largest divisor s of the k-tile count with tiles * s <= ~1.25 x CU count
static int mfma_splits(int64_t tiles, int64_t ktiles) {
    int best = 1;
    for (int64_t d = 1; d <= ktiles && d <= 64; ++d)
        if (ktiles % d == 0 && tiles * d <= 320) best = (int)d;
    return best;
}

struct MfmaPlan {
    int64_t Mpad, Kpad, a_floats, part_floats;
    int splits;
};

static MfmaPlan plan(int64_t M, int N, int64_t K) {
    MfmaPlan p;
    p.Mpad = up_to(M, QM);
    p.Kpad = up_to(K, QK);
    p.a_floats = up_to(p.Mpad * p.Kpad / 2, 64);
    p.splits = mfma_splits((p.Mpad / QM) * (N / QN), p.Kpad / QK);
    p.part_floats = p.splits > 1 ? (int64_t)p.splits * p.Mpad * N : 0;   // tiles x splits x 512 x 32
    return p;
}

template <typename H>
static int run(const char* who, const H* A, const H* B, int64_t ldb, int64_t M, int N, const MfmaPlan& p,
               float* C, const float* bias, int accumulate, float* part, hipStream_t st) {
    static bool attr = false;
    if (!attr) {   // 160 KB of dynamic LDS (above the 64 KB default cap)
        if (hipFuncSetAttribute((const void*)k_mfma_gemm<H>, hipFuncAttributeMaxDynamicSharedMemorySize, GEMM_LDS) !=
            hipSuccess) {
            set_error("%s: cannot allow %d B of LDS for k_mfma_gemm", who, GEMM_LDS);
            return VT_ERR_HIP;
        }
        attr = true;
    }
    const int kper = (int)(p.Kpad / p.splits);
    dim3 grid(N / QN, (unsigned)(p.Mpad / QM), p.splits);
    const unsigned tiles = grid.x * grid.y;
    hipLaunchKernelGGL(k_mfma_gemm<H>, grid, dim3(QT), GEMM_LDS, st, A, p.Kpad, B, ldb, (int)M, N, kper, C, (int64_t)N,
                       bias, accumulate, p.splits > 1 ? part : nullptr, p.splits > 1 ? arrive_slots(tiles, st) : 0u);
    VT_LAUNCH_CHECK(who);
    return VT_OK;
}

}  // namespace vt

using namespace vt;

extern "C" {

int vt_mfma_supported(int K, int N) { return (K > 0 && N > 0 && K % QK == 0 && N % QN == 0) ? 1 : 0; }

int vt_mfma_workspace_floats(int64_t R, int K, int N, int64_t* floats) {
    VT_CHECK_ARG(R > 0 && K > 0 && N > 0 && floats, "vt_mfma_workspace_floats: shape");
    MfmaPlan f = plan(R, N, K), d = plan(R, K, N), w = plan(N, K, R);
    const int64_t wf = w.a_floats + up_to((int64_t)K * w.Kpad / 2, 64) + w.part_floats + N;
    int64_t m = f.a_floats + f.part_floats;
    if (d.a_floats + d.part_floats > m) m = d.a_floats + d.part_floats;
    if (wf > m) m = wf;
    *floats = m;
    return VT_OK;
}

int vt_mfma_weight_shadow(const float* W, int N, int K, void* W16, void* W16t, void* stream) {
    VT_CHECK_ARG(vt_mfma_supported(K, N) && W && W16 && W16t, "vt_mfma_weight_shadow: K and N must be multiples of 64");
    VT_H16(hipLaunchKernelGGL(k_bf16_shadow<H>, dim3(K / 64, N / 64), dim3(256), 0, S(stream), W, N, K, (H*)W16,
                              (H*)W16t));
    VT_LAUNCH_CHECK("vt_mfma_weight_shadow");
    return VT_OK;
}

// Y[R,N] = X[R,K] W[N,K]^T + b     (W16 = bf16 shadow of W, [N][K])
int vt_mfma_linear_fwd(const float* X, int64_t R, int K, const void* W16, int N, const float* bias, float* Y,
                       float* ws, int64_t ws_floats, void* stream) {
    VT_CHECK_ARG(R > 0 && vt_mfma_supported(K, N), "vt_mfma_linear_fwd: K and N must be positive multiples of 64");
    MfmaPlan p = plan(R, N, K);
    VT_CHECK_ARG(p.a_floats + p.part_floats <= ws_floats, "vt_mfma_linear_fwd: workspace too small");
    const int64_t tot = p.Mpad * p.Kpad;
    int rc = VT_OK;
    VT_H16(H* A = (H*)ws;
           hipLaunchKernelGGL(k_bf16_rows<H>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, S(stream), X, R, K, A,
                              p.Mpad, (int)p.Kpad);
           rc = run("vt_mfma_linear_fwd", (const H*)A, (const H*)W16, K, R, N, p, Y, bias, 0, ws + p.a_floats,
                    S(stream)));
    return rc;
}

// dX[R,K] (+)= dY[R,N] W[N,K]      (W16t = bf16 shadow of W^T, [K][N])
int vt_mfma_linear_bwd_data(const float* dY, int64_t R, int N, const void* W16t, int K, float* dX, int accumulate,
                            float* ws, int64_t ws_floats, void* stream) {
    VT_CHECK_ARG(R > 0 && vt_mfma_supported(N, K), "vt_mfma_linear_bwd_data: K and N must be positive multiples of 64");
    MfmaPlan p = plan(R, K, N);  // C = dX (M=R, cols=K), reduction over N
    VT_CHECK_ARG(p.a_floats + p.part_floats <= ws_floats, "vt_mfma_linear_bwd_data: workspace too small");
    const int64_t tot = p.Mpad * p.Kpad;
    int rc = VT_OK;
    VT_H16(H* A = (H*)ws;
           hipLaunchKernelGGL(k_bf16_rows<H>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, S(stream), dY, R, N, A,
                              p.Mpad, (int)p.Kpad);
           rc = run("vt_mfma_linear_bwd_data", (const H*)A, (const H*)W16t, N, R, K, p, dX, nullptr, accumulate,
                    ws + p.a_floats, S(stream)));
    return rc;
}

// dW[N,K] (+)= dY[R,N]^T X[R,K];  db (+)= column sums of dY (if db != NULL)
int vt_mfma_linear_bwd_weight(const float* dY, int64_t R, int N, const float* X, int K, float* dW, float* db,
                              int accumulate, float* ws, int64_t ws_floats, void* stream) {
    VT_CHECK_ARG(R > 0 && vt_mfma_supported(K, N), "vt_mfma_linear_bwd_weight: K and N must be positive multiples of 64");
    if (N % DWT == 0 && K % DWT == 0) {
        // direct: fp32 operands staged and transposed in LDS, no split (k_mfma_dw)
        VT_H16(hipLaunchKernelGGL(k_mfma_dw<H>, dim3(K / DWT, N / DWT), dim3(256), 0, S(stream), dY, R, N, X, K, dW,
                                  accumulate));
        VT_LAUNCH_CHECK("vt_mfma_linear_bwd_weight");
        return db ? vt_colsum(dY, R, N, db, accumulate, ws, ws_floats, stream) : VT_OK;
    }
    MfmaPlan p = plan(N, K, R);  // C = dW (M=N, cols=K), reduction over R
    const int64_t b_floats = up_to((int64_t)K * p.Kpad / 2, 64);
    VT_CHECK_ARG(p.a_floats + b_floats + p.part_floats + N <= ws_floats, "vt_mfma_linear_bwd_weight: workspace too small");
    float* part = ws + p.a_floats + b_floats;
    int rc = VT_OK;
    VT_H16(H* A = (H*)ws;                   // dY^T  [Npad][Rpad]
           H* Bt = (H*)(ws + p.a_floats);   // X^T   [K][Rpad]
           hipLaunchKernelGGL(k_bf16_transpose<H>, dim3((unsigned)(p.Kpad / 64), (unsigned)(p.Mpad / 64)), dim3(256), 0,
                              S(stream), dY, R, N, A, p.Mpad, p.Kpad);
           hipLaunchKernelGGL(k_bf16_transpose<H>, dim3((unsigned)(p.Kpad / 64), (unsigned)(K / 64)), dim3(256), 0,
                              S(stream), X, R, K, Bt, (int64_t)K, p.Kpad);
           rc = run("vt_mfma_linear_bwd_weight", (const H*)A, (const H*)Bt, p.Kpad, N, K, p, dW, nullptr, accumulate,
                    part, S(stream)));
    if (rc || !db) return rc;
    return vt_colsum(dY, R, N, db, accumulate, part, ws_floats - p.a_floats - b_floats, stream);
}

}  // extern "C"
