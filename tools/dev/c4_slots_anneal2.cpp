// Dev prototype: anneal bp_ms_lds64_kernel's check -> state-slot permutation
// against the measured gfx950 banking (tools/dev/lds_atomic_probe.hip):
//   m1 / m2 reads      2 x 32-lane groups, key slot % 32          (x2 per edge)
//   m1 / m2 atomics    4 x 16-lane groups, key slot % 16          (x2 per edge)
//   parw / hdw words   2 x 32-lane groups, key (slot >> 5) % 32   (x1.5)
// Objective: the max-per-bank cycles themselves (the sum over groups of the
// most lanes on one bank, weighted), updated incrementally per swap.
// Input: tools/dev/c4_bank_model2.py's instructions (64 lane checks each, -1 idle).
// Usage: c4_slots_anneal2 groups.txt iters [T0 T1 seed]
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

struct Group {
    int mod, shift;
    double w;
    std::vector<int> cnt;
};

int main(int argc, char** argv) {
    FILE* f = fopen(argv[1], "r");
    const long iters = argc > 2 ? atol(argv[2]) : 20000000L;
    const double T0 = argc > 3 ? atof(argv[3]) : 2.0, T1 = argc > 4 ? atof(argv[4]) : 0.05;
    const unsigned seed = argc > 5 ? (unsigned)atoi(argv[5]) : 1u;
    int m, ni;
    if (fscanf(f, "%d %d", &m, &ni) != 2) return 1;
    std::vector<Group> G;
    std::vector<std::vector<int>> occ(m);  // group ids per check (with multiplicity)
    for (int t = 0; t < ni; ++t) {
        int lanes[64];
        for (int l = 0; l < 64; ++l)
            if (fscanf(f, "%d", &lanes[l]) != 1) return 1;
        auto add = [&](int lo, int len, int mod, int shift, double w) {
            Group g{mod, shift, w, std::vector<int>(mod, 0)};
            const int id = (int)G.size();
            bool any = false;
            for (int l = lo; l < lo + len; ++l)
                if (lanes[l] >= 0) occ[lanes[l]].push_back(id), any = true;
            if (any) G.push_back(g);
            else return;
        };
        for (int h = 0; h < 2; ++h) add(32 * h, 32, 32, 0, 2.0);   // reads m1, m2
        for (int q = 0; q < 4; ++q) add(16 * q, 16, 16, 0, 2.0);   // atomics m1, m2
        for (int h = 0; h < 2; ++h) add(32 * h, 32, 32, 5, 1.5);   // words
    }
    std::vector<int> slot(m);
    for (int i = 0; i < m; ++i) slot[i] = i;
    auto key = [&](const Group& g, int s) { return (s >> g.shift) % g.mod; };
    for (int i = 0; i < m; ++i)
        for (int id : occ[i]) G[id].cnt[key(G[id], slot[i])]++;
    std::vector<int> gmax(G.size());
    double cost = 0, base = 0;
    for (size_t id = 0; id < G.size(); ++id) {
        gmax[id] = *std::max_element(G[id].cnt.begin(), G[id].cnt.end());
        cost += G[id].w * gmax[id];
        base += G[id].w;
    }
    printf("groups %zu start cost %.0f ideal %.0f\n", G.size(), cost, base);
    std::mt19937_64 rng(seed);
    std::uniform_real_distribution<double> uni(0.0, 1.0);
    std::vector<int> touched;
    std::vector<int> mark(G.size(), 0);
    int stamp = 0;
    // squared-load tie-break keeps the walk moving on plateaus of the max model
    auto sq_delta = [&](int i, int from, int to) {
        double d = 0;
        for (int id : occ[i]) {
            Group& g = G[id];
            const int a = key(g, from), b = key(g, to);
            if (a == b) continue;
            d += g.w * (2.0 * (g.cnt[b] - g.cnt[a]) + 2.0) * 0.02;
        }
        return d;
    };
    for (long it = 0; it < iters; ++it) {
        const int i = (int)(rng() % (uint64_t)m), j = (int)(rng() % (uint64_t)m);
        const int si = slot[i], sj = slot[j];
        if (i == j) continue;
        ++stamp;
        touched.clear();
        for (int id : occ[i])
            if (mark[id] != stamp) mark[id] = stamp, touched.push_back(id);
        for (int id : occ[j])
            if (mark[id] != stamp) mark[id] = stamp, touched.push_back(id);
        const double sq = sq_delta(i, si, sj) + sq_delta(j, sj, si);
        for (int id : occ[i]) G[id].cnt[key(G[id], si)]--, G[id].cnt[key(G[id], sj)]++;
        for (int id : occ[j]) G[id].cnt[key(G[id], sj)]--, G[id].cnt[key(G[id], si)]++;
        double d = 0;
        std::vector<int> nm(touched.size());
        for (size_t t = 0; t < touched.size(); ++t) {
            const int id = touched[t];
            nm[t] = *std::max_element(G[id].cnt.begin(), G[id].cnt.end());
            d += G[id].w * (nm[t] - gmax[id]);
        }
        const double temp = T0 * std::pow(T1 / T0, (double)it / (double)iters);
        const double dd = d + sq;
        if (dd <= 0 || uni(rng) < std::exp(-dd / temp)) {
            slot[i] = sj;
            slot[j] = si;
            for (size_t t = 0; t < touched.size(); ++t) gmax[touched[t]] = nm[t];
            cost += d;
        } else {
            for (int id : occ[i]) G[id].cnt[key(G[id], sj)]--, G[id].cnt[key(G[id], si)]++;
            for (int id : occ[j]) G[id].cnt[key(G[id], si)]--, G[id].cnt[key(G[id], sj)]++;
        }
        if (it % (iters / 10) == 0) printf("it %ld cost %.0f temp %.3f\n", it, cost, temp);
    }
    printf("final cost %.0f ideal %.0f conflict share %.3f\n", cost, base, 1 - base / cost);
    return 0;
}
