// Dev: CPU stand-ins for the HIP device builtins the hypergraph-product kernel
// uses (tools/dev/hgp_cpu_emu.cpp): one std::thread per GPU thread, barriers by
// std::barrier.  Only for debugging the kernel's logic.
#pragma once
#include <atomic>
#include <barrier>
#include <cmath>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>
#define __global__
#define __device__
#define __forceinline__ inline
#define __launch_bounds__(...)
#define __shared__ static
struct double2 { double x, y; };
inline double2 make_double2(double a, double b) { return {a, b}; }
struct Dim { unsigned x; };
inline thread_local Dim threadIdx{0};
inline std::barrier<>* emu_bar = nullptr;
inline std::atomic<int> emu_or{0};
inline std::barrier<>* emu_bar2 = nullptr;
inline void __syncthreads() { emu_bar->arrive_and_wait(); }
inline int __syncthreads_or(int p) {
    if (p) emu_or.fetch_or(1);
    emu_bar->arrive_and_wait();
    const int r = emu_or.load();
    emu_bar2->arrive_and_wait();
    if (threadIdx.x == 0) emu_or.store(0);
    emu_bar->arrive_and_wait();
    return r;
}
inline long long __double_as_longlong(double d) { long long v; std::memcpy(&v, &d, 8); return v; }
inline double __longlong_as_double(long long v) { double d; std::memcpy(&d, &v, 8); return d; }
inline unsigned long long atomicAdd(unsigned long long* p, unsigned long long v) { return __atomic_fetch_add(p, v, __ATOMIC_SEQ_CST); }
inline unsigned atomicOr(unsigned* p, unsigned v) { return __atomic_fetch_or(p, v, __ATOMIC_SEQ_CST); }
inline void emu_run(int threads, std::function<void()> f) {
    std::barrier<> b(threads), b2(threads);
    emu_bar = &b;
    emu_bar2 = &b2;
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t) ts.emplace_back([&, t] { threadIdx.x = t; f(); });
    for (auto& t : ts) t.join();
}
inline unsigned __builtin_amdgcn_bitop3_b32(unsigned a, unsigned b, unsigned c, unsigned t) {
    unsigned r = 0;
    for (int i = 0; i < 32; ++i) {
        const unsigned idx = (((a >> i) & 1u) << 2) | (((b >> i) & 1u) << 1) | ((c >> i) & 1u);
        r |= ((t >> idx) & 1u) << i;
    }
    return r;
}
#define asm(...) asm_unsupported
