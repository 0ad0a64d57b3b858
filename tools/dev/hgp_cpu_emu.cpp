// Dev: run the generated hypergraph-product kernel (qdec_hgp_kernel.hip after
// its prologue) on the CPU, one std::thread per GPU thread, to debug its
// logic without a device.  Build: g++ -std=c++20 -O1 -pthread
//   -include tools/dev/hgp_cpu_shim.h tools/dev/hgp_cpu_emu.cpp
// (the generated source is written by qd_graph_hgp_source).  Input on stdin:
// B m n, then the priors (n doubles), then B*m syndrome bytes (0/1); output:
// per shot its iterations and hard decision.
#include <cstdio>
#include <thread>
#include <vector>

#include HGP_SRC  // the generated kernel source

int main(int argc, char** argv) {
    long long B;
    int m, n, max_iter;
    if (scanf("%lld %d %d %d", &B, &m, &n, &max_iter) != 4) return 1;
    std::vector<double> prior(n);
    for (auto& p : prior) scanf("%lf", &p);
    std::vector<unsigned char> syn(B * m);
    for (auto& s : syn) { int v; scanf("%d", &v); s = (unsigned char)v; }
    std::vector<unsigned char> x(B * n, 0), st(B, 0);
    std::vector<int> it(B, 0);
    unsigned long long counter = 0;
    HgArgs a{syn.data(), prior.data(), x.data(), it.data(), st.data(), &counter, B, max_iter, 0.0};
    emu_run(HG_THREADS, [&] { hgp_bp_ms_f64(a); });
    for (long long b = 0; b < B; ++b) {
        printf("%d %d ", it[b], st[b]);
        for (int j = 0; j < n; ++j) putchar('0' + x[b * n + j]);
        putchar('\n');
    }
    return 0;
}
