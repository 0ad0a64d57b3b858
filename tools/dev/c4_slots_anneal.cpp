// Dev prototype: anneal a check -> state-slot permutation for bp_ms_lds64_kernel
// (tools/dev/c4_bank_model.py writes the halves).  Objective per 32-lane half:
// sum over banks of cnt^2 for x = slot % 32 (u64 state ops) and y = (slot >> 5) % 32
// (bit-word ops); reported: the max-per-bank model of c4_bank_model.py.
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>
#include <cmath>
#include <algorithm>
int main(int argc, char** argv) {
    FILE* f = fopen(argv[1], "r");
    int m, nh;
    if (fscanf(f, "%d %d", &m, &nh) != 2) return 1;
    std::vector<std::vector<int>> halves(nh);
    std::vector<std::vector<int>> occ(m);
    for (int h = 0; h < nh; ++h) {
        int c;
        if (fscanf(f, "%d", &c) != 1) return 1;
        halves[h].resize(c);
        for (int t = 0; t < c; ++t) { if (fscanf(f, "%d", &halves[h][t]) != 1) return 1; occ[halves[h][t]].push_back(h); }
    }
    const double WX = 5.0, WY = 1.5;
    std::vector<int> slot(m);
    for (int i = 0; i < m; ++i) slot[i] = i;
    std::vector<int> cx((size_t)nh * 32, 0), cy((size_t)nh * 32, 0);
    auto X = [&](int s) { return s & 31; };
    auto Y = [&](int s) { return (s >> 5) & 31; };
    for (int h = 0; h < nh; ++h) for (int i : halves[h]) { cx[h * 32 + X(slot[i])]++; cy[h * 32 + Y(slot[i])]++; }
    auto maxcost = [&]() {
        double c = 0;
        for (int h = 0; h < nh; ++h) {
            int mx = 0, my = 0;
            for (int b = 0; b < 32; ++b) { mx = std::max(mx, cx[h * 32 + b]); my = std::max(my, cy[h * 32 + b]); }
            c += 3.0 * mx + 2.0 * mx + 1.0 * my + 0.5 * my;
        }
        return c;
    };
    printf("identity max-model %.1f ideal %.1f\n", maxcost(), nh * 6.5);
    std::mt19937_64 rng(1);
    const long iters = argc > 2 ? atol(argv[2]) : 20000000;
    double T = argc > 3 ? atof(argv[3]) : 2.0;
    // delta of moving check i from slot a to slot b (counts of other checks fixed)
    auto apply = [&](int i, int s_old, int s_new, int sign_dummy) {
        for (int h : occ[i]) { cx[h * 32 + X(s_old)]--; cy[h * 32 + Y(s_old)]--; cx[h * 32 + X(s_new)]++; cy[h * 32 + Y(s_new)]++; }
    };
    auto local = [&](int i, int s) {  // sum of squares contribution of check i's bins (after placement)
        double c = 0;
        for (int h : occ[i]) { int a = cx[h * 32 + X(s)], b = cy[h * 32 + Y(s)]; c += WX * (2 * a - 1) + WY * (2 * b - 1); }
        return c;
    };
    for (long it = 0; it < iters; ++it) {
        int i = rng() % m, j = rng() % m;
        if (i == j) continue;
        int si = slot[i], sj = slot[j];
        if (X(si) == X(sj) && Y(si) == Y(sj)) continue;
        double before = local(i, si) + local(j, sj);
        apply(i, si, sj, 0); apply(j, sj, si, 0);
        double after = local(i, sj) + local(j, si);
        double d = after - before;
        if (d <= 0 || std::generate_canonical<double, 53>(rng) < std::exp(-d / T)) { slot[i] = sj; slot[j] = si; }
        else { apply(j, si, sj, 0); apply(i, sj, si, 0); }
        if (it % 1000000 == 0) { T *= 0.8; }
    }
    printf("annealed max-model %.1f\n", maxcost());
    return 0;
}
