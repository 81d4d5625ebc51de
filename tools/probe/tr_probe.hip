// Probe of ds_read_b64_tr_b16 lane semantics: LDS holds value 100*row + col
// (row-major, stride 24 bf16); each lane addresses row (lane>>2)&3, cols 4*(lane&3).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short v4i16 __attribute__((ext_vector_type(4)));
__global__ void k(int* out) {
    __shared__ __attribute__((aligned(16))) short img[16 * 24];
    const int lane = threadIdx.x;
    for (int i = lane; i < 16 * 24; i += 64) img[i] = (short)(100 * (i / 24) + (i % 24));
    __syncthreads();
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    short* a = img + (4 * g + q) * 24 + 4 * p;
    v4i16 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)a);
    for (int j = 0; j < 4; ++j) out[lane * 4 + j] = r[j];
}
int main() {
    int* d; hipMalloc(&d, 256 * 4);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    int h[256]; hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; ++l) printf("lane %2d: %4d %4d %4d %4d\n", l, h[4*l], h[4*l+1], h[4*l+2], h[4*l+3]);
    return 0;
}
