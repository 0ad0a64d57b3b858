// Dev: LDS-array cycles and bank conflicts of the LDS atomics bp_ms_lds64_kernel
// issues (ds_min_u64, ds_min_rtn_u64, ds_xor_b32) and of ds_read_b64, per lane
// address pattern.  Build: hipcc --offload-arch=gfx950 -O3 lds_atomic_probe.hip -o
// /tmp/lds_atomic_probe; run under rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE
// SQ_LDS_BANK_CONFLICT (one dispatch per (op, pattern), kernel names carry both).
#include <hip/hip_runtime.h>

#include <cstdio>

// slot (u64 element, or u32 word for OP 2) of lane l
__device__ __forceinline__ int pat(int p, int l) {
    switch (p) {
        case 0: return l;                            // consecutive
        case 1: return (l & 15) + 32 * (l >> 4);     // 16-lane runs, runs 32 apart
        case 2: return (l & 31) + 64 * (l >> 5);     // 32-lane runs, runs 64 apart
        case 3: return 16 * l;                       // 128-B stride
        case 4: return 32 * l;                       // 256-B stride: one bank
        case 5: return (l & 7) + 32 * (l >> 3);      // 8-lane runs, runs 32 apart
        default: return (l * 67) & 1023;             // the kernel's column stride
    }
}

template <int OP, int P>
__global__ __launch_bounds__(1024) void probe(unsigned long long* out, int iters) {
    __shared__ unsigned long long s[2048 + 64];
    for (int i = threadIdx.x; i < 2048 + 64; i += 1024) s[i] = ~0ull;
    __syncthreads();
    const int l = threadIdx.x & 63;
    int slot = pat(P, l);
    unsigned long long acc = 0, v = threadIdx.x;
    for (int i = 0; i < iters; ++i) {
        asm volatile("" : "+v"(slot));
        if (OP == 0) {
            atomicMin(&s[slot], v + i);
        } else if (OP == 1) {
            acc += atomicMin(&s[slot], v + i);
        } else if (OP == 2) {
            atomicXor(reinterpret_cast<unsigned*>(s) + slot, 1u << (i & 31));
        } else {
            acc += *reinterpret_cast<volatile unsigned long long*>(&s[slot]);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = acc + s[l];
}

template <int OP, int P>
static float run(unsigned long long* d, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL((probe<OP, P>), dim3(256), dim3(1024), 0, 0, d, iters);
    hipEventRecord(a);
    hipLaunchKernelGGL((probe<OP, P>), dim3(256), dim3(1024), 0, 0, d, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

template <int OP>
static void ops(unsigned long long* d, int iters, const char* name) {
    const float t[7] = {run<OP, 0>(d, iters), run<OP, 1>(d, iters), run<OP, 2>(d, iters), run<OP, 3>(d, iters),
                        run<OP, 4>(d, iters), run<OP, 5>(d, iters), run<OP, 6>(d, iters)};
    // cycles per wave-instruction per CU at 2.4 GHz: 16 waves x iters instructions
    printf("%-14s", name);
    for (float ms : t) printf(" %7.2f", ms * 1e-3 * 2.4e9 / (16.0 * iters));
    printf("   (clk per wave-instr; patterns: consec, 16runs, 32runs, 128B, 256B, 8runs, x67)\n");
}

int main() {
    unsigned long long* d;
    hipMalloc(&d, 256 * 8);
    const int iters = 4000;
    ops<0>(d, iters, "ds_min_u64");
    ops<1>(d, iters, "ds_min_rtn_u64");
    ops<2>(d, iters, "ds_xor_b32");
    ops<3>(d, iters, "ds_read_b64");
    hipFree(d);
    return 0;
}
