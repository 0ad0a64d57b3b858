// qdec_osd.cpp -- ordered-statistics decoding (OSD-0 / OSD-E / OSD-CS) for shots
// BP did not converge on (ldpc v1 bposd_decoder, used by the reference at
// python/qldpc/misc/_experiment.py:23,37,77,96).
//
// Host-side stage of the hybrid pipeline: the GPU returns the BP soft output
// (log-probability ratios) for the failing shots, this stage post-processes them
// on the host cores (std::thread over shots).  Per shot:
//   1. order columns by ascending log-probability ratio (stable: ties by index);
//   2. Gauss-Jordan eliminate [H_ordered | I_m] over GF(2), bit-packed rows,
//      pivots taken greedily in that column order (first row holding a 1);
//   3. OSD-0: pivot bits = transformed syndrome, other bits 0;
//   4. OSD-E(lambda): every assignment of the first lambda non-pivot columns;
//      OSD-CS(lambda): every single non-pivot column, plus every pair among the
//      first lambda non-pivot columns.  For a candidate set g of non-pivot columns
//      the pivot part is T s ^ xor_{j in g} T H_j (T = the elimination transform);
//      keep the candidate of least Hamming weight (strictly less replaces).
// The spec is this build's restatement of ldpc v1's published OSD; ldpc itself is
// absent, so parity against it is unpinned.  The checker is
// oracle/osd_py.py (an independent dense numpy implementation).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/qdec.h"

namespace {

thread_local std::string g_osd_error;

struct Osd {
    int m, n, method, order;
    const int32_t* row_ptr;
    const int32_t* col_idx;
};

inline int popcount_words(const uint64_t* a, int W) {
    int c = 0;
    for (int w = 0; w < W; ++w) c += __builtin_popcountll(a[w]);
    return c;
}

// Decode one shot.  llr: BP log-probability ratios (n); syn: m bytes.
void osd_one(const Osd& P, const uint8_t* syn, const double* llr, uint8_t* out0, uint8_t* outw,
             std::vector<uint64_t>& mat, std::vector<int>& order_buf) {
    const int m = P.m, n = P.n;
    // augmented row: n column bits (in sorted order) + m transform bits + 1 syndrome bit
    const int bits = n + m + 1;
    const int W = (bits + 63) / 64;
    mat.assign((size_t)m * W, 0);
    std::vector<int>& cols = order_buf;
    cols.resize(n);
    std::iota(cols.begin(), cols.end(), 0);
    std::stable_sort(cols.begin(), cols.end(), [&](int a, int b) { return llr[a] < llr[b]; });
    std::vector<int> pos(n);
    for (int k = 0; k < n; ++k) pos[cols[k]] = k;
    for (int i = 0; i < m; ++i) {
        uint64_t* r = &mat[(size_t)i * W];
        for (int e = P.row_ptr[i]; e < P.row_ptr[i + 1]; ++e) {
            const int k = pos[P.col_idx[e]];
            r[k >> 6] ^= 1ull << (k & 63);
        }
        const int tb = n + i;
        r[tb >> 6] |= 1ull << (tb & 63);
        if (syn[i] & 1) r[(n + m) >> 6] |= 1ull << ((n + m) & 63);
    }
    // Gauss-Jordan in sorted column order
    std::vector<int> pivcol;  // sorted-position of pivot for row index r
    pivcol.reserve(m);
    int rank = 0;
    for (int k = 0; k < n && rank < m; ++k) {
        const int w = k >> 6;
        const uint64_t bit = 1ull << (k & 63);
        int piv = -1;
        for (int i = rank; i < m; ++i)
            if (mat[(size_t)i * W + w] & bit) { piv = i; break; }
        if (piv < 0) continue;
        if (piv != rank)
            std::swap_ranges(mat.begin() + (size_t)piv * W, mat.begin() + (size_t)(piv + 1) * W,
                             mat.begin() + (size_t)rank * W);
        const uint64_t* pr = &mat[(size_t)rank * W];
        for (int i = 0; i < m; ++i) {
            if (i == rank) continue;
            uint64_t* r = &mat[(size_t)i * W];
            if (r[w] & bit)
                for (int t = 0; t < W; ++t) r[t] ^= pr[t];
        }
        pivcol.push_back(k);
        ++rank;
    }
    // solution vectors are kept over pivot rows: bit r = value of pivot column pivcol[r]
    const int RW = (rank + 63) / 64;
    auto sbit = [&](int r) -> int { return (int)((mat[(size_t)r * W + ((n + m) >> 6)] >> ((n + m) & 63)) & 1); };
    std::vector<uint64_t> x0(std::max(RW, 1), 0);
    for (int r = 0; r < rank; ++r)
        if (sbit(r)) x0[r >> 6] |= 1ull << (r & 63);
    // non-pivot columns in sorted order
    std::vector<int> nonpiv;
    nonpiv.reserve(n - rank);
    {
        size_t p = 0;
        for (int k = 0; k < n; ++k) {
            if (p < pivcol.size() && pivcol[p] == k) { ++p; continue; }
            nonpiv.push_back(k);
        }
    }
    // transformed column of non-pivot k: bit r = mat[r][k] (the reduced matrix)
    auto tcol = [&](int k, std::vector<uint64_t>& dst) {
        dst.assign(std::max(RW, 1), 0);
        for (int r = 0; r < rank; ++r)
            if ((mat[(size_t)r * W + (k >> 6)] >> (k & 63)) & 1) dst[r >> 6] |= 1ull << (r & 63);
    };
    auto emit = [&](const std::vector<uint64_t>& xp, const std::vector<int>& g, uint8_t* out) {
        std::memset(out, 0, (size_t)n);
        for (int r = 0; r < rank; ++r)
            if ((xp[r >> 6] >> (r & 63)) & 1) out[cols[pivcol[r]]] = 1;
        for (int k : g) out[cols[k]] ^= 1;
    };
    emit(x0, {}, out0);
    if (P.method == 0 || P.order < 0) {
        std::memcpy(outw, out0, (size_t)n);
        return;
    }
    int best_w = popcount_words(x0.data(), RW);
    std::vector<uint64_t> best = x0;
    std::vector<int> best_g;
    const int kn = (int)nonpiv.size();
    const int lam = std::min(P.order, kn);
    std::vector<std::vector<uint64_t>> tc(kn);
    // columns needed: all non-pivots for CS weight-1; first lam for pairs / OSD-E
    const int need = (P.method == 2) ? kn : lam;
    for (int t = 0; t < need; ++t) tcol(nonpiv[t], tc[t]);
    std::vector<uint64_t> cand(std::max(RW, 1));
    auto consider = [&](const std::vector<int>& gidx) {
        cand = x0;
        for (int t : gidx)
            for (int w = 0; w < RW; ++w) cand[w] ^= tc[t][w];
        const int wgt = popcount_words(cand.data(), RW) + (int)gidx.size();
        if (wgt < best_w) {
            best_w = wgt;
            best = cand;
            best_g.clear();
            for (int t : gidx) best_g.push_back(nonpiv[t]);
        }
    };
    if (P.method == 1) {  // OSD-E: all 2^lam assignments (ascending bitmask)
        for (long s = 1; s < (1L << lam); ++s) {
            std::vector<int> gidx;
            for (int t = 0; t < lam; ++t)
                if ((s >> t) & 1) gidx.push_back(t);
            consider(gidx);
        }
    } else {  // OSD-CS: singles over every non-pivot column, then pairs among the first lam
        for (int t = 0; t < kn; ++t) consider({t});
        for (int a = 0; a < lam; ++a)
            for (int b = a + 1; b < lam; ++b) consider({a, b});
    }
    emit(best, best_g, outw);
}

}  // namespace

extern "C" int qd_osd_batch(int32_t m, int32_t n, const int32_t* row_ptr, const int32_t* col_idx, int32_t method,
                            int32_t order, int64_t B, const uint8_t* syn, const double* llr, uint8_t* osd0_out,
                            uint8_t* osdw_out, int32_t nthreads) {
    try {
        if (m <= 0 || n <= 0 || !row_ptr || !col_idx || B < 0) throw std::invalid_argument("invalid OSD graph");
        if (method < 0 || method > 2) throw std::invalid_argument("osd method must be 0 (osd0), 1 (osd_e), 2 (osd_cs)");
        if (method == 1 && order > 20) throw std::invalid_argument("osd_e order above 20 is not supported");
        if (B == 0) return 0;
        if (!syn || !llr || !osd0_out || !osdw_out) throw std::invalid_argument("null OSD buffers");
        Osd P{m, n, method, order, row_ptr, col_idx};
        int T = nthreads > 0 ? nthreads : (int)std::max(1u, std::thread::hardware_concurrency());
        if (T > B) T = (int)B;
        std::vector<std::thread> pool;
        for (int t = 0; t < T; ++t) {
            pool.emplace_back([&, t] {
                std::vector<uint64_t> mat;
                std::vector<int> ord;
                for (int64_t b = t; b < B; b += T)
                    osd_one(P, syn + b * m, llr + b * n, osd0_out + b * n, osdw_out + b * n, mat, ord);
            });
        }
        for (auto& th : pool) th.join();
        return 0;
    } catch (const std::exception& e) {
        g_osd_error = e.what();
        return -80;
    }
}

extern "C" const char* qd_osd_last_error(void) { return g_osd_error.c_str(); }
