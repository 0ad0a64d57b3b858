// Dev probe: round-trip latency of global_load_lds_dword vs global_load_dword
// under full occupancy (16 one-wave workgroups per CU), random 256-B rows of a
// 256 MiB buffer.  Prints mean ticks per load round trip.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ __launch_bounds__(64) void probe(const unsigned char* buf, size_t rows, int mode, unsigned long long* out) {
    extern __shared__ unsigned char sm[];
    unsigned long long acc = 0;
    unsigned x = blockIdx.x * 2654435761u + 12345u;
    unsigned sink = 0;
    for (int it = 0; it < 64; ++it) {
        x = x * 1664525u + 1013904223u;
        const size_t row = x % rows;
        const unsigned char* src = buf + row * 256 + 4 * threadIdx.x;
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        if (mode == 0) {
            __builtin_amdgcn_global_load_lds(src, sm, 4, 0, 0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            unsigned v = *reinterpret_cast<const unsigned*>(src);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            asm volatile("" : "+v"(v));
            sink += v;
        }
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        acc += t1 - t0;
    }
    if (threadIdx.x == 0) atomicAdd(out, acc);
    if (sink == 0xdeadbeef) out[1] = sink;
}
int main() {
    const size_t rows = (256u << 20) / 256;
    unsigned char* buf;
    unsigned long long* out;
    hipMalloc(&buf, rows * 256);
    hipMemset(buf, 1, rows * 256);
    hipMalloc(&out, 16);
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    for (int occ : {1, 4, 16}) {
        for (int mode = 0; mode < 2; ++mode) {
            hipMemset(out, 0, 16);
            const int grid = ncu * occ;
            hipLaunchKernelGGL(probe, dim3(grid), dim3(64), 1024, 0, buf, rows, mode, out);
            hipDeviceSynchronize();
            unsigned long long h = 0;
            hipMemcpy(&h, out, 8, hipMemcpyDeviceToHost);
            printf("waves/CU=%2d %s: %.0f ticks per round trip\n", occ, mode == 0 ? "global_load_lds" : "global_load    ",
                   (double)h / (grid * 64.0));
        }
    }
    return 0;
}
