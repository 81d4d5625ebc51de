// LSTM parameter gradients on bf16 MFMA for the 16-bit recurrences (SURVEY.md §8(a) a12;
// ref/model/vae_teb_model.py:474-480, :647-653: nn.LSTM's weight_ih / weight_hh / biases
// under the reference's 16-mixed autocast, where cuDNN forms them from 16-bit gate
// gradients and inputs with fp32 accumulation — graph_model.py:510, :709-711).
//
//   [dW_ih | dW_hh | db] = bf16(dG)^T bf16([x | h_{t-1} | 1])   (fp32 accumulation)
//
// over the B*S rows of a layer (dG [rows][4H] fp32 from vt_lstm16_layer_bwd, x [rows][In],
// h [rows][H] read one row back within each sample, zero at t = 0).  The exact-fp32 path
// (mlp.hip k_sk_dw, v_mfma_f32_16x16x4_f32) is MFMA-bound at fp32's 157 TF: 4.8 GFLOP per
// In = 64 layer, >= 30 us.  Here the rows are the MFMA reduction (v_mfma_f32_16x16x32_bf16,
// 32 rows per k-step): a workgroup of 8 waves streams its row range in 64-row chunks, the
// next chunk's fp32 rows loaded into registers during the current chunk's MFMAs and
// converted to bf16 as they are stored (dG [64][4H], [x | h_{t-1}] [64][16 NTK] row-major),
// operand fragments read with the gfx950 transposed LDS read (ds_read_b64_tr_b16, rows
// contiguous per fragment).  Each wave owns two whole 16-row tiles of dW (its A fragments read
// once per k-step for all NTK column tiles).  Per-workgroup partial slabs, summed in fixed
// order by mlp.hip's k_sk_sum (the fp32 path's reduction and output layout).
#include <stdlib.h>

#include "common.h"
#include "skinny.h"

namespace vt {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef short v8i16 __attribute__((ext_vector_type(8)));

constexpr int G = 256;       // 4 H gate rows (H = 64)
constexpr int CR = 64;       // rows per chunk (2 MFMA k-steps)
constexpr int DS = G + 8;    // bf16 row stride of the dG image (16 B mod 128 B: conflict-free transposed reads)
constexpr int NTH = 512;     // 8 waves
constexpr int UG = CR * G / 4 / NTH;   // dG float4 per thread and chunk (8)

__device__ __forceinline__ bf16x8 tr_frag(const __bf16* img, int row0, int col0, int stride) {
    // lane 4q+p of each 16-lane group: row (row0 + 8 g + q), columns col0 + 4p .. +3; rows
    // +0..3 and +4..7 of the group's 8-row block (conv_bf16.hip tr_frag)
    const int lane = threadIdx.x & 63, g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const __bf16* a0 = img + (row0 + 8 * g + q) * stride + col0 + 4 * p;
    const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)a0);
    const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) v4i16*)(a0 + 4 * stride));
    const v8i16 r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, r);
}

__device__ __forceinline__ bf16x4 cvt4(float4 v) {
    return bf16x4{(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
}

// part[blk][n][k'] (k' < K1 = In + H + 1) = sum over the workgroup's rows of
// bf16(dG[r][n]) bf16(X1[r][k']), X1 = [x | h_{t-1} | 1]
template <int NTK>
__global__ __launch_bounds__(NTH) void k_sk_dw16(const float* __restrict__ dG, const float* __restrict__ x, int In,
                                                 const float* __restrict__ h, int S, int64_t R,
                                                 int64_t rows_per_block, float* __restrict__ part) {
    constexpr int XS = 16 * NTK + 8;   // bf16 row stride of the [x | h_{t-1} | 1] image
    __shared__ __attribute__((aligned(16))) __bf16 gs[CR * DS];
    __shared__ __attribute__((aligned(16))) __bf16 xs[CR * XS];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int K1 = In + 64 + 1;
    const int ix4 = In / 4;                 // float4 per x row
    const int xitems = CR * (ix4 + 16);     // x and h_{t-1} float4 of a chunk
    const int UX = (CR * (16 + 16) + NTH - 1) / NTH;   // (In <= 64) <= 4 per thread
    const int64_t rb = (int64_t)blockIdx.x * rows_per_block;
    const int64_t re = rb + rows_per_block < R ? rb + rows_per_block : R;
    // the ones column and the zero padding of the X1 image are the same for every chunk
    for (int i = tid; i < CR * (16 * NTK - In - 64); i += NTH) {
        const int t = i / (16 * NTK - In - 64), c = In + 64 + (i - t * (16 * NTK - In - 64));
        xs[t * XS + c] = (__bf16)(c == K1 - 1 ? 1.f : 0.f);
    }
    float4 vg[UG], vx[4];
    auto load = [&](int64_t c0) {
        const int n = re - c0 < CR ? (int)(re - c0) : CR;
#pragma unroll
        for (int u = 0; u < UG; ++u) {
            const int i = tid + NTH * u;            // float4 index within the chunk's [64][256]
            const int t = i >> 6;
            vg[u] = t < n ? *reinterpret_cast<const float4*>(dG + (c0 + t) * G + 4 * (i & 63))
                          : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = tid + NTH * u;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (u < UX && i < xitems) {
                const int t = i / (ix4 + 16), j = i - t * (ix4 + 16);
                const int64_t r = c0 + t;
                if (t < n) {
                    if (j < ix4) {
                        v = *reinterpret_cast<const float4*>(x + r * In + 4 * j);
                    } else if (r % S != 0) {   // h_{t-1}: the previous row of the same sample
                        v = *reinterpret_cast<const float4*>(h + (r - 1) * 64 + 4 * (j - ix4));
                    }
                }
            }
            vx[u] = v;
        }
    };
    // two whole 16-row dW tiles per wave: tn = 2 wv, 2 wv + 1
    f32x4 acc[2][NTK];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int k = 0; k < NTK; ++k) acc[a][k] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (rb < re) load(rb);
    for (int64_t c0 = rb; c0 < re; c0 += CR) {
        // registers -> bf16 images (rows past the range are zero in dG: no contribution)
#pragma unroll
        for (int u = 0; u < UG; ++u) {
            const int i = tid + NTH * u;
            *reinterpret_cast<bf16x4*>(gs + (i >> 6) * DS + 4 * (i & 63)) = cvt4(vg[u]);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = tid + NTH * u;
            if (u < UX && i < xitems) {
                const int t = i / (ix4 + 16), j = i - t * (ix4 + 16);
                const int c = j < ix4 ? 4 * j : In + 4 * (j - ix4);
                *reinterpret_cast<bf16x4*>(xs + t * XS + c) = cvt4(vx[u]);
            }
        }
        __syncthreads();
        if (c0 + CR < re) load(c0 + CR);   // in flight during the MFMAs
#pragma unroll
        for (int s = 0; s < CR / 32; ++s) {
            bf16x8 b[NTK];
#pragma unroll
            for (int k = 0; k < NTK; ++k) b[k] = tr_frag(xs, 32 * s, 16 * k, XS);
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                const bf16x8 af = tr_frag(gs, 32 * s, 16 * (2 * wv + a), DS);
#pragma unroll
                for (int k = 0; k < NTK; ++k)
                    acc[a][k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, b[k], acc[a][k], 0, 0, 0);
            }
        }
        __syncthreads();
    }
    // D: col (k') = 16 k + (lane & 15), row (n) = 16 tn + 4 (lane >> 4) + r
    float* pb = part + (int64_t)blockIdx.x * G * K1;
    const int lr = lane & 15, lc = lane >> 4;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int k = 0; k < NTK; ++k) {
            const int kk = 16 * k + lr;
            if (kk >= K1) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) pb[(16 * (2 * wv + a) + 4 * lc + r) * K1 + kk] = acc[a][k][r];
        }
}

}  // namespace

// bf16 LSTM parameter gradients (see above); In % 4 == 0, In <= 64, H = 64, 16-byte aligned
// operands; blocks of >= 256 rows, at most 128 workgroups (partials 128 x 256 x K1 floats).
int sk_lstm16_dw(const float* dG, const float* x, int In, const float* h, int S, int64_t R, float* dW_ih,
                 float* dW_hh, float* db_ih, float* db_hh, int accumulate, float* ws, int64_t ws_floats,
                 hipStream_t st) {
    const int K1 = In + 64 + 1, NTK = (K1 + 15) / 16;
    if (In % 4 != 0 || In > 64 || NTK < 5 || NTK > 9 || (((uintptr_t)dG | (uintptr_t)x | (uintptr_t)h) & 15))
        return VT_ERR_ARG;
    static const int cap = getenv("VAETEB_L16DW_BLOCKS") ? atoi(getenv("VAETEB_L16DW_BLOCKS")) : 128;
    int64_t blocks = (R + 255) / 256;
    if (blocks > cap) blocks = cap > 0 ? cap : 128;
    if (blocks * G * K1 > ws_floats) blocks = ws_floats / ((int64_t)G * K1);
    if (blocks < 1) return VT_ERR_ARG;
    int64_t rpb = (R + blocks - 1) / blocks;
    blocks = (R + rpb - 1) / rpb;
    const dim3 grid((unsigned)blocks);
    switch (NTK) {
        case 5: hipLaunchKernelGGL(k_sk_dw16<5>, grid, dim3(NTH), 0, st, dG, x, In, h, S, R, rpb, ws); break;
        case 6: hipLaunchKernelGGL(k_sk_dw16<6>, grid, dim3(NTH), 0, st, dG, x, In, h, S, R, rpb, ws); break;
        case 7: hipLaunchKernelGGL(k_sk_dw16<7>, grid, dim3(NTH), 0, st, dG, x, In, h, S, R, rpb, ws); break;
        case 8: hipLaunchKernelGGL(k_sk_dw16<8>, grid, dim3(NTH), 0, st, dG, x, In, h, S, R, rpb, ws); break;
        default: hipLaunchKernelGGL(k_sk_dw16<9>, grid, dim3(NTH), 0, st, dG, x, In, h, S, R, rpb, ws); break;
    }
    sk_sum_launch(ws, (int)blocks, G, In, 64, K1, dW_ih, dW_hh, db_ih, db_hh, accumulate, st);
    return VT_OK;
}

}  // namespace vt
