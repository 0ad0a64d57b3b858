// Probe: LDS layout written by global_load_lds with size 1 (dev tool).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const unsigned char* src, unsigned char* out) {
    extern __shared__ unsigned char sm[];
    for (int i = threadIdx.x; i < 1024; i += 64) sm[i] = 0xEE;
    __syncthreads();
    __builtin_amdgcn_global_load_lds(src + threadIdx.x, sm + 64, 1, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 512; i += 64) out[i] = sm[i];
}
int main() {
    unsigned char h[64], *d, *o, ho[512];
    for (int i = 0; i < 64; ++i) h[i] = (unsigned char)(i + 1);
    hipMalloc(&d, 64); hipMalloc(&o, 512);
    hipMemcpy(d, h, 64, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 1024, 0, d, o);
    hipMemcpy(ho, o, 512, hipMemcpyDeviceToHost);
    for (int i = 60; i < 340; ++i) printf("%d:%d ", i, ho[i]);
    printf("\n");
    return 0;
}
