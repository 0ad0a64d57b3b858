// Microbenchmark: issue cost of f64 vs f32 VALU ops on gfx950 (cycles per wave
// instruction, 8 independent chains per lane, 1..8 waves per SIMD).
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/f64_rates tools/dev/f64_rates.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int OP, typename T>
__global__ void k(T* out, long long* cyc, int iters, T a, T b) {
    T x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = a + (T)(threadIdx.x + i);
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (OP == 0) x[i] = x[i] + b;
            if constexpr (OP == 1) x[i] = x[i] * b;
            if constexpr (OP == 2) x[i] = fmin(x[i], b + x[(i + 1) & 7]);
            if constexpr (OP == 3) x[i] = (x[i] <= b) ? x[i] : b;  // cmp + select
            if constexpr (OP == 4) x[i] = fmax(x[i], b);
        }
        asm volatile("" ::: "memory");
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    T s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP, typename T>
void run(const char* name) {
    const int iters = 4096;
    for (int wps : {1, 2, 4, 8}) {
        const int blocks = 256 * 4 * wps;  // one-wave blocks: wps waves per SIMD
        T* out;
        long long* cyc;
        hipMalloc(&out, sizeof(T) * blocks * 64);
        hipMalloc(&cyc, sizeof(long long) * blocks);
        hipLaunchKernelGGL((k<OP, T>), dim3(blocks), dim3(64), 0, 0, out, cyc, iters, (T)1.5, (T)0.75);
        hipDeviceSynchronize();
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0);
        hipLaunchKernelGGL((k<OP, T>), dim3(blocks), dim3(64), 0, 0, out, cyc, iters, (T)1.5, (T)0.75);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        std::vector<long long> c(blocks);
        hipMemcpy(c.data(), cyc, sizeof(long long) * blocks, hipMemcpyDeviceToHost);
        double avg = 0;
        for (auto v : c) avg += v;
        avg /= blocks;
        // per SIMD: wps waves x iters x 8 ops; cycles from wall clock at 2.4 GHz-ish and s_memtime
        const double ops_per_simd = (double)wps * iters * 8;
        printf("%-10s %s waves/SIMD=%d  wall %.3f ms  -> %.2f cyc/op (memtime/wave %.2f cyc/op-per-wave)\n", name,
               sizeof(T) == 8 ? "f64" : "f32", wps, ms, ms * 1e-3 * 2.4e9 / ops_per_simd, avg / (iters * 8.0));
        hipFree(out);
        hipFree(cyc);
    }
}

int main() {
    run<0, double>("add");
    run<0, float>("add");
    run<1, double>("mul");
    run<2, double>("min");
    run<2, float>("min");
    run<3, double>("cmp+sel");
    run<3, float>("cmp+sel");
    run<4, double>("max");
    return 0;
}
