// GF(2) elimination on bit-packed rows, on the host cores.
//
// Offline code-construction support, not part of the decode hot path: the
// logical operators of a CSS code (ker Hx / row Hz and ker Hz / row Hx) that the
// fused failure check consumes.  The reference computes them with galois
// (python/qldpc/homological_product_code.py:6-60: null_space, column_space,
// row_reduce), which is absent here and, like the numpy restatement in
// exp_ldpc_amd/gf2.py, too slow for the 10^4..5*10^4-qubit codes of BASELINE
// configs 4 and 5.
//
// Layout: row-major uint64 words, bit j of a row at word j/64, bit j%64
// (exp_ldpc_amd/gf2.py pack_rows).
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/qdec.h"

namespace {

inline bool bit(const uint64_t* row, int64_t col) { return (row[col >> 6] >> (col & 63)) & 1u; }

// Sense-reversing spin barrier for the fixed worker team of one elimination.
struct SpinBarrier {
    explicit SpinBarrier(int n) : n_(n) {}
    void wait() {
        const int gen = gen_.load(std::memory_order_acquire);
        if (count_.fetch_add(1, std::memory_order_acq_rel) + 1 == n_) {
            count_.store(0, std::memory_order_relaxed);
            gen_.fetch_add(1, std::memory_order_acq_rel);
        } else {
            while (gen_.load(std::memory_order_acquire) == gen) std::this_thread::yield();
        }
    }
    int n_;
    std::atomic<int> count_{0};
    std::atomic<int> gen_{0};
};

}  // namespace

extern "C" int64_t qd_gf2_rref(uint64_t* rows, int64_t nrows, int64_t words, int64_t ncols, int64_t* pivots,
                               int32_t nthreads) {
    if (!rows || nrows < 0 || words <= 0 || ncols < 0 || ncols > words * 64) return -1;
    int T = nthreads > 0 ? nthreads : (int)std::max(1u, std::thread::hardware_concurrency());
    // below ~1M words of work per pivot, threads only add barrier latency
    if (nrows * words < (int64_t)1 << 16) T = 1;
    T = (int)std::min<int64_t>(T, std::max<int64_t>(1, nrows / 64));
    std::vector<uint64_t> tmp(words);
    int64_t rank = 0;
    std::atomic<int64_t> piv_row{-1};
    SpinBarrier bar(T);
    auto worker = [&](int tid) {
        int64_t r = 0;  // local copy of rank
        for (int64_t col = 0; col < ncols && r < nrows; ++col) {
            if (tid == 0) {
                int64_t p = -1;
                for (int64_t i = r; i < nrows; ++i)
                    if (bit(rows + i * words, col)) { p = i; break; }
                if (p >= 0 && p != r) {
                    std::memcpy(tmp.data(), rows + p * words, words * 8);
                    std::memcpy(rows + p * words, rows + r * words, words * 8);
                    std::memcpy(rows + r * words, tmp.data(), words * 8);
                }
                piv_row.store(p, std::memory_order_release);
            }
            bar.wait();
            if (piv_row.load(std::memory_order_acquire) < 0) {
                bar.wait();
                continue;
            }
            // Rows at or below the pivot are zero left of col, so the XOR starts
            // at col's word; rows above may have bits anywhere right of their own
            // pivots, but the pivot row is zero left of col too.
            const uint64_t* prow = rows + r * words;
            const int64_t w0 = col >> 6;
            for (int64_t i = tid; i < nrows; i += T) {
                if (i == r) continue;
                uint64_t* x = rows + i * words;
                if (bit(x, col))
                    for (int64_t w = w0; w < words; ++w) x[w] ^= prow[w];
            }
            if (tid == 0 && pivots) pivots[r] = col;
            ++r;
            bar.wait();
        }
        if (tid == 0) rank = r;
    };
    if (T == 1) {
        worker(0);
    } else {
        std::vector<std::thread> pool;
        for (int t = 1; t < T; ++t) pool.emplace_back(worker, t);
        worker(0);
        for (auto& th : pool) th.join();
    }
    return rank;
}

// Reduce candidate rows against an echelon basis whose row b has its lowest set
// bit at basis_lead[b]; candidates that stay nonzero are accepted (flag 1), in
// order, and join the basis.  Returns the number accepted.  This extends a basis
// of span(basis) to one of span(basis + candidates), as the reference does with
// its augmented row reduction (homological_product_code.py:15-21).
extern "C" int64_t qd_gf2_extend_basis(const uint64_t* basis, int64_t nbasis, const int64_t* basis_lead,
                                       const uint64_t* cand, int64_t ncand, int64_t words, int64_t ncols,
                                       uint8_t* accepted, int64_t max_accept) {
    if (words <= 0 || ncols > words * 64 || (nbasis && (!basis || !basis_lead)) || (ncand && !cand) || !accepted)
        return -1;
    std::vector<int64_t> lead_row(ncols, -1);
    std::vector<uint64_t> store((size_t)(nbasis + ncand) * words);
    if (nbasis) std::memcpy(store.data(), basis, (size_t)nbasis * words * 8);
    for (int64_t b = 0; b < nbasis; ++b) {
        if (basis_lead[b] < 0 || basis_lead[b] >= ncols) return -2;
        lead_row[basis_lead[b]] = b;
    }
    int64_t n = nbasis, acc = 0;
    std::vector<uint64_t> v(words);
    for (int64_t c = 0; c < ncand; ++c) {
        accepted[c] = 0;
        if (max_accept >= 0 && acc >= max_accept) continue;
        std::memcpy(v.data(), cand + c * words, words * 8);
        int64_t lead = -1;
        for (int64_t w = 0; w < words && lead < 0;) {
            if (!v[w]) { ++w; continue; }
            int64_t col = w * 64 + __builtin_ctzll(v[w]);
            int64_t b = lead_row[col];
            if (b < 0) { lead = col; break; }
            const uint64_t* row = store.data() + b * words;
            for (int64_t u = w; u < words; ++u) v[u] ^= row[u];
        }
        if (lead >= 0) {
            std::memcpy(store.data() + n * words, v.data(), words * 8);
            lead_row[lead] = n++;
            accepted[c] = 1;
            ++acc;
        }
    }
    return acc;
}
