// Dev: joint simulated annealing of the f64 min-sum wave kernel's LDS layout
// (variable lane slots, check state slots, v2c row positions) under the bank
// model of tools/dev/ms_conflicts.py (MI355X_MICROARCH.md §LDS):
//   scatter  ds_write_b64, 4 groups of 16 contiguous lanes, class = element % 16
//   gather   ds_read_b128, 4 hardware lane groups, class = state slot % 16
//   state    ds_write_b128, 8 groups of 8 contiguous lanes, class = slot % 8
// Input (stdin): m n, then m lines "deg c0 c1 ..." (CSR rows, ascending).
// Output: the modelled array cycles of the degree-order layout after the
// sequential anneal (ms_layout's) and of the joint anneal.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

static const int kDC = 4, DRS = 10, NCL = 16;
int m, n, m_pad, n_pad, RVn, D3P;
std::vector<std::vector<int>> rows, cols;  // rows: columns ascending; cols: rows ascending
std::vector<int> cdeg;

static int rgroup(int l) {
    const int q = l % 32, h = (l / 32) * 2;
    return h + ((q < 4 || (q >= 12 && q < 16) || (q >= 20 && q < 28)) ? 0 : 1);
}

struct Layout {
    std::vector<int> var_of_slot, slot_of;  // [n_pad], [n]
    std::vector<std::vector<int>> pos;      // pos[i][t]: position of row i's t-th edge
    std::vector<int> sst;                   // [m_pad]
};

// cost pieces
long scatter_cost(const Layout& L, int gi) {  // instruction gi = rv * kDC + k
    const int rv = gi / kDC, k = gi % kDC;
    if (rv < D3P && k == 3) return 0;
    int load[4][NCL] = {{0}};
    bool pad[4] = {false, false, false, false};
    for (int l = 0; l < 64; ++l) {
        const int j = L.var_of_slot[rv * 64 + l];
        if (j < 0 || k >= cdeg[j]) { pad[l / 16] = true; continue; }
        const int i = cols[j][k];
        int t = (int)(std::lower_bound(rows[i].begin(), rows[i].end(), j) - rows[i].begin());
        load[l / 16][(i * DRS + L.pos[i][t]) % NCL]++;
    }
    // pads write one dummy element, in the class least loaded over the pad groups
    int bestb = 0, bestc = 1 << 30;
    for (int b = 0; b < NCL; ++b) {
        int c = 0;
        for (int h = 0; h < 4; ++h) if (pad[h]) c = std::max(c, load[h][b]);
        if (c < bestc) { bestc = c; bestb = b; }
    }
    long s = 0;
    for (int h = 0; h < 4; ++h) {
        if (pad[h]) load[h][bestb]++;
        int mx = 0;
        for (int b = 0; b < NCL; ++b) mx = std::max(mx, load[h][b]);
        s += mx;
    }
    return std::max(4L, s);
}

long gather_cost(const Layout& L, int gi) {
    const int rv = gi / kDC, k = gi % kDC;
    if (rv < D3P && k == 3) return 0;
    std::vector<int> seen[4];
    bool pad[4] = {false, false, false, false};
    for (int l = 0; l < 64; ++l) {
        const int j = L.var_of_slot[rv * 64 + l];
        if (j < 0 || k >= cdeg[j]) { pad[rgroup(l)] = true; continue; }
        const int i = cols[j][k];
        auto& v = seen[rgroup(l)];
        if (std::find(v.begin(), v.end(), i) == v.end()) v.push_back(i);
    }
    long s = 0;
    for (int h = 0; h < 4; ++h) {
        int cnt[NCL] = {0}, mx = 0;
        for (int i : seen[h]) mx = std::max(mx, ++cnt[L.sst[i] % NCL]);
        if (pad[h]) mx = std::max(mx, ++cnt[m_pad % NCL]);
        s += mx;
    }
    return s;
}

long state_cost(const Layout& L) {
    long s = 0;
    for (int w = 0; w < m_pad / 8; ++w) {
        int cnt[8] = {0}, mx = 0;
        for (int t = 0; t < 8; ++t) mx = std::max(mx, ++cnt[L.sst[w * 8 + t] % 8]);
        s += mx;
    }
    return s;
}

long total(const Layout& L, long* sc, long* gc, long* wc) {
    long a = 0, b = 0;
    for (int gi = 0; gi < RVn * kDC; ++gi) { a += scatter_cost(L, gi); b += gather_cost(L, gi); }
    const long c = state_cost(L);
    if (sc) *sc = a;
    if (gc) *gc = b;
    if (wc) *wc = c;
    return a + b + c;
}

bool slot_ok(const Layout& L, int s, int j) {  // variable j (or pad -1) may sit in slot s
    if (j < 0) return true;
    return !(s / 64 < D3P && cdeg[j] > 3);
}

int main(int argc, char** argv) {
    const long iters = argc > 1 ? atol(argv[1]) : 2000000;
    const unsigned seed = argc > 2 ? (unsigned)atoi(argv[2]) : 1u;
    if (scanf("%d %d", &m, &n) != 2) return 1;
    rows.resize(m);
    cols.resize(n);
    for (int i = 0; i < m; ++i) {
        int d;
        if (scanf("%d", &d) != 1) return 1;
        rows[i].resize(d);
        for (int t = 0; t < d; ++t) { if (scanf("%d", &rows[i][t]) != 1) return 1; cols[rows[i][t]].push_back(i); }
    }
    m_pad = (m + 63) / 64 * 64;
    n_pad = (n + 63) / 64 * 64;
    RVn = n_pad / 64;
    cdeg.resize(n);
    for (int j = 0; j < n; ++j) cdeg[j] = (int)cols[j].size();
    Layout L;
    std::vector<int> order(n);
    for (int j = 0; j < n; ++j) order[j] = j;
    std::stable_sort(order.begin(), order.end(), [](int x, int y) { return cdeg[x] < cdeg[y]; });
    L.var_of_slot.assign(n_pad, -1);
    L.slot_of.assign(n, 0);
    for (int s = 0; s < n; ++s) { L.var_of_slot[s] = order[s]; L.slot_of[order[s]] = s; }
    D3P = 0;
    for (int r = 0; r < RVn; ++r) {
        bool ok = true;
        for (int l = 0; l < 64; ++l) { const int j = L.var_of_slot[r * 64 + l]; if (j >= 0 && cdeg[j] > 3) ok = false; }
        if (!ok) break;
        D3P = r + 1;
    }
    D3P &= ~1;
    L.pos.resize(m);
    for (int i = 0; i < m; ++i) { L.pos[i].resize(rows[i].size()); for (size_t t = 0; t < rows[i].size(); ++t) L.pos[i][t] = (int)t; }
    L.sst.resize(m_pad);
    for (int i = 0; i < m_pad; ++i) L.sst[i] = i;
    long sc, gc, wc;
    long cur = total(L, &sc, &gc, &wc);
    printf("identity layout: total %ld (scatter %ld gather %ld state %ld) + rows 32, D3P %d\n", cur, sc, gc, wc, D3P);
    std::mt19937 rng(seed);
    auto ur = [&]() { return (double)(rng() & 0xFFFFFF) / 16777216.0; };
    long best = cur;
    Layout bestL = L;
    for (long it = 0; it < iters; ++it) {
        const double T = 1.5 * std::pow(0.005, (double)it / iters);
        const int mv = (int)(rng() % 3);
        if (mv == 0) {  // swap two variable slots
            const int s1 = (int)(rng() % n_pad), s2 = (int)(rng() % n_pad);
            const int j1 = L.var_of_slot[s1], j2 = L.var_of_slot[s2];
            if (s1 == s2 || (j1 < 0 && j2 < 0) || !slot_ok(L, s1, j2) || !slot_ok(L, s2, j1)) continue;
            const int r1 = s1 / 64, r2 = s2 / 64;
            long old = 0;
            for (int k = 0; k < kDC; ++k) {
                old += scatter_cost(L, r1 * kDC + k) + gather_cost(L, r1 * kDC + k);
                if (r2 != r1) old += scatter_cost(L, r2 * kDC + k) + gather_cost(L, r2 * kDC + k);
            }
            std::swap(L.var_of_slot[s1], L.var_of_slot[s2]);
            long nw = 0;
            for (int k = 0; k < kDC; ++k) {
                nw += scatter_cost(L, r1 * kDC + k) + gather_cost(L, r1 * kDC + k);
                if (r2 != r1) nw += scatter_cost(L, r2 * kDC + k) + gather_cost(L, r2 * kDC + k);
            }
            const long d = nw - old;
            if (d <= 0 || ur() < std::exp(-d / T)) {
                cur += d;
                if (L.var_of_slot[s1] >= 0) L.slot_of[L.var_of_slot[s1]] = s1;
                if (L.var_of_slot[s2] >= 0) L.slot_of[L.var_of_slot[s2]] = s2;
            } else std::swap(L.var_of_slot[s1], L.var_of_slot[s2]);
        } else if (mv == 1) {  // swap two state slots
            const int c1 = (int)(rng() % m_pad), c2 = (int)(rng() % m_pad);
            if (c1 == c2) continue;
            auto gs = [&]() {
                long a = state_cost(L);
                for (int gi = 0; gi < RVn * kDC; ++gi) a += gather_cost(L, gi);
                return a;
            };
            const long old = gs();
            std::swap(L.sst[c1], L.sst[c2]);
            const long nw = gs();
            const long d = nw - old;
            if (d <= 0 || ur() < std::exp(-d / T)) cur += d;
            else std::swap(L.sst[c1], L.sst[c2]);
        } else {  // swap two row positions
            const int i = (int)(rng() % m);
            const int d0 = (int)rows[i].size();
            if (d0 < 2) continue;
            const int t1 = (int)(rng() % d0), t2 = (int)(rng() % d0);
            if (t1 == t2) continue;
            const int g1 = L.slot_of[rows[i][t1]] / 64 * kDC +
                           (int)(std::find(cols[rows[i][t1]].begin(), cols[rows[i][t1]].end(), i) - cols[rows[i][t1]].begin());
            const int g2 = L.slot_of[rows[i][t2]] / 64 * kDC +
                           (int)(std::find(cols[rows[i][t2]].begin(), cols[rows[i][t2]].end(), i) - cols[rows[i][t2]].begin());
            const long old = scatter_cost(L, g1) + (g2 != g1 ? scatter_cost(L, g2) : 0);
            std::swap(L.pos[i][t1], L.pos[i][t2]);
            const long nw = scatter_cost(L, g1) + (g2 != g1 ? scatter_cost(L, g2) : 0);
            const long d = nw - old;
            if (d <= 0 || ur() < std::exp(-d / T)) cur += d;
            else std::swap(L.pos[i][t1], L.pos[i][t2]);
        }
        if (cur < best) { best = cur; bestL = L; }
    }
    total(bestL, &sc, &gc, &wc);
    printf("joint anneal (%ld moves, seed %u): total %ld (scatter %ld gather %ld state %ld) + rows 32\n", iters, seed,
           best, sc, gc, wc);
    return 0;
}
