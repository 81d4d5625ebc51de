// Per-step latency floor of a 4-wave recurrence on gfx950 (diagnostic, not product code):
// cycles per iteration (s_memtime) of
//   0: s_barrier alone
//   1: ds_write_b16 -> lgkmcnt(0) -> s_barrier -> ds_read_b128 x2 -> use
//   2: 1 + 8 MFMAs 16x16x32 f16 (4 chains of 2) on the read data
//   3: 2 + a dependent chain of 5 exp/rcp activations (the LSTM cell)
//   4: 3 with 2 waves per SIMD (512 threads, two independent 4-wave groups)
// Build: hipcc --offload-arch=gfx950 -O3 step_latency.hip -o step_latency
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void probe(unsigned long long* out, float* sink, int iters) {
    __shared__ __attribute__((aligned(16))) _Float16 hs[2][4][72];
    const int j = threadIdx.x, lane = j & 63, ln = lane & 15, lg = lane >> 4, w = (j >> 6) & 3;
    for (int i = j; i < 2 * 4 * 72; i += blockDim.x) (&hs[0][0][0])[i] = (_Float16)0.01f;
    __syncthreads();
    f16x8 b[4][2];
    for (int g = 0; g < 4; ++g)
        for (int k = 0; k < 2; ++k)
            for (int e = 0; e < 8; ++e) b[g][k][e] = (_Float16)(0.001f * (g + k + e));
    float c = 0.1f, acc = 0.f;
    unsigned long long t0 = 0;
    for (int it = 0; it < iters; ++it) {
        if (it == 16) t0 = __builtin_amdgcn_s_memtime();
        float hn = c;
        if constexpr (MODE >= 1) {
            const _Float16* hp = &hs[it & 1][ln >> 2][8 * lg];
            const f16x8 a0 = *(const f16x8*)hp, a1 = *(const f16x8*)(hp + 32);
            if constexpr (MODE >= 2) {
                f32x4 p[4];
                for (int g = 0; g < 4; ++g) {
                    p[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b[g][0], f32x4{c, c, c, c}, 0, 0, 0);
                    p[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b[g][1], p[g], 0, 0, 0);
                }
                if constexpr (MODE >= 3) {
                    const float gi = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(p[0][0]));
                    const float gf = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(p[1][0]));
                    const float gg = fmaf(2.f, __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(p[2][0])), -1.f);
                    const float go = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(p[3][0]));
                    c = fmaf(gf, c, gi * gg);
                    hn = go * fmaf(2.f, __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-2.88539f * c)), -1.f);
                } else {
                    hn = p[0][0] + p[1][0] + p[2][0] + p[3][0];
                }
            } else {
                hn = (float)a0[0] + (float)a1[1];
            }
            hs[(it + 1) & 1][lg][16 * w + ln] = (_Float16)hn;
        }
        acc += hn;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (blockIdx.x == 0 && j == 0) out[0] = t1 - t0;
    sink[blockIdx.x * blockDim.x + j] = acc;
}

template <int MODE>
void run(int threads, const char* name) {
    unsigned long long* d;
    float* s;
    hipMalloc(&d, 8);
    hipMalloc(&s, 1 << 20);
    const int iters = 4096 + 16;
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(probe<MODE>, dim3(1), dim3(threads), 0, 0, d, s, iters);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(probe<MODE>, dim3(1), dim3(threads), 0, 0, d, s, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long cyc;
    hipMemcpy(&cyc, d, 8, hipMemcpyDeviceToHost);
    printf("%-52s %7.1f cycles/iter  %6.1f ns/iter (events)\n", name, (double)cyc / 4096, ms * 1e6 / iters);
    hipFree(d);
    hipFree(s);
}

int main() {
    run<0>(256, "0 barrier only (4 waves)");
    run<1>(256, "1 + ds_write/lgkm/ds_read x2");
    run<2>(256, "2 + 8 MFMA 16x16x32 f16 (4 chains of 2)");
    run<3>(256, "3 + cell activations (5 exp/rcp)");
    run<3>(512, "4 = 3 with 8 waves (2 per SIMD)");
    run<3>(64, "5 = 3 with 1 wave");
    return 0;
}
