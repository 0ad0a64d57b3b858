// qdec_osd.hip -- ordered-statistics decoding on the GPU for the shots BP did not
// converge on (the OSD stage of ldpc v1 bposd_decoder; reference call sites
// python/qldpc/misc/_experiment.py:23, 37, 77, 96 -- osd_cs order 7 is the
// p_sweep default, _experiment.py:218-219).
//
// Same spec as the host stage (qdec_osd.cpp, checked by oracle/osd_py.py), so the
// outputs are bit-identical:
//   1. columns in ascending order of the BP log-probability ratio, ties by index
//      (stable sort);
//   2. Gauss-Jordan over GF(2) in that column order, the pivot of a column being
//      the first row at or below the current rank that holds a 1 (rows swapped);
//   3. OSD-0: pivot bits = the transformed syndrome, everything else 0;
//   4. OSD-E(lambda): every assignment of the first lambda non-pivot columns;
//      OSD-CS(lambda): every single non-pivot column, then every pair among the
//      first lambda; the candidate of least Hamming weight wins, an earlier
//      candidate keeping a tie.
//
// One wave64 per shot (persistent over the batch).  Row i of the augmented
// matrix [H_sorted | s] lives in registers of lane i % 64, slot i / 64 (RS <= 6
// slots: m <= 384, i.e. spacetime graphs up to R = 2; W <= 16 64-bit words:
// n < 1024), so a pivot step is: a ballot per slot to find the pivot, two
// readlanes per word to broadcast the pivot row, and one masked XOR per word and
// slot -- no LDS traffic inside the elimination.  The sort is a bitonic network
// in LDS on (order-preserving key, column) pairs.  Candidate scoring reads the
// reduced matrix back from LDS: a transformed column is RS ballots, its weight
// RS scalar popcounts.  The fused fold + logical check reuses finalize_shot.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "qdec_device.h"
#include "qdec_internal.h"

namespace qdec {

constexpr int kOsdMaxLam = 64;  // pair / exhaustive search width kept in LDS

// LDS layout of one wave (byte offsets); identical on host and device.
struct OsdLayout {
    int ns, o_key, o_idx, o_pos, o_isp, o_piv, o_npv, o_red, o_tcl, o_out, total;
    __host__ __device__ OsdLayout(int n, int m, int RS, int W) {
        ns = 64;
        while (ns < n) ns <<= 1;
        int o = 0;
        auto take = [&](int bytes) {
            const int at = o;
            o += (bytes + 15) / 16 * 16;
            return at;
        };
        o_key = take(8 * ns);
        o_red = take(8 * RS * 64 * W);
        o_tcl = take(8 * kOsdMaxLam * RS);
        o_idx = take(2 * ns);
        o_pos = take(2 * n);
        o_piv = take(2 * (m > 0 ? m : 1));
        o_npv = take(2 * n);
        o_isp = take(n);
        o_out = take(n);
        total = o;
        (void)RS;
    }
};

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

// Ascending doubles -> ascending unsigned keys (-0.0 folded onto +0.0, as the
// host's `<` comparison treats them as equal).
__device__ __forceinline__ uint64_t order_key(double v) {
    uint64_t b = (uint64_t)__double_as_longlong(v);
    if (b == 0x8000000000000000ull) b = 0;
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

// Calls f(std::integral_constant<int, I>) for I = B .. E-1 (compile-time indices).
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// Bit k of a W-word register row.  Written as masked arithmetic over every word:
// an `if (w == k >> 6)` select chain is folded back by the compiler into a
// dynamically indexed array, which demotes the whole row to scratch memory.
template <int W>
__device__ __forceinline__ void flip_bit(uint64_t (&r)[W], int k) {
    const uint64_t bit = 1ull << (k & 63);
#pragma unroll
    for (int w = 0; w < W; ++w) r[w] ^= bit & (0ull - (uint64_t)((unsigned)(k - 64 * w) < 64u));
}

template <int W>
__device__ __forceinline__ int get_bit(const uint64_t (&r)[W], int k) {
    uint64_t v = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) v |= r[w] & (0ull - (uint64_t)((unsigned)(k - 64 * w) < 64u));
    return (int)((v >> (k & 63)) & 1);
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, d);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), d);
        const uint64_t o = ((uint64_t)hi << 32) | lo;
        v = o < v ? o : v;
    }
    return v;
}

template <int RS, int W>
__global__ __launch_bounds__(64) void osd_wave_kernel(DevGraph g, OsdArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x;
    const int m = g.m, n = g.n;
    const OsdLayout L(n, m, RS, W);
    uint64_t* skey = reinterpret_cast<uint64_t*>(smem + L.o_key);
    uint64_t* red = reinterpret_cast<uint64_t*>(smem + L.o_red);
    uint64_t* tcl = reinterpret_cast<uint64_t*>(smem + L.o_tcl);
    uint16_t* sidx = reinterpret_cast<uint16_t*>(smem + L.o_idx);  // sorted position -> column
    uint16_t* pos = reinterpret_cast<uint16_t*>(smem + L.o_pos);   // column -> sorted position
    uint16_t* pivc = reinterpret_cast<uint16_t*>(smem + L.o_piv);  // rank row -> pivot position
    uint16_t* npv = reinterpret_cast<uint16_t*>(smem + L.o_npv);   // non-pivot positions, ascending
    uint8_t* isp = smem + L.o_isp;
    uint8_t* outb = smem + L.o_out;
    const int NS = L.ns;
    const int32_t* rp = g.row_ptr;
    const int32_t* ci = g.col_idx;

    for (int64_t shot = blockIdx.x; shot < a.B; shot += gridDim.x) {
        if (a.status && (a.status[shot] & 1)) continue;  // BP converged: nothing to do
        // ---- 1. stable sort of the columns by log-probability ratio
        for (int k = lane; k < NS; k += 64) {
            uint64_t key = ~0ull;
            uint16_t idx = 0xffff;
            if (k < n) {
                const double v = a.llr_f32 ? (double)static_cast<const float*>(a.llr)[shot * n + k]
                                           : static_cast<const double*>(a.llr)[shot * n + k];
                key = order_key(v);
                idx = (uint16_t)k;
            }
            skey[k] = key;
            sidx[k] = idx;
        }
        __syncthreads();
        for (int size = 2; size <= NS; size <<= 1) {
            for (int stride = size >> 1; stride > 0; stride >>= 1) {
                for (int t = lane; t < NS / 2; t += 64) {
                    const int i = 2 * t - (t & (stride - 1));
                    const int j = i + stride;
                    const uint64_t ki = skey[i], kj = skey[j];
                    const uint16_t ii = sidx[i], ij = sidx[j];
                    const bool gt = ki > kj || (ki == kj && ii > ij);
                    if (gt == ((i & size) == 0)) {
                        skey[i] = kj;
                        skey[j] = ki;
                        sidx[i] = ij;
                        sidx[j] = ii;
                    }
                }
                __syncthreads();
            }
        }
        for (int k = lane; k < n; k += 64) {
            pos[sidx[k]] = (uint16_t)k;
            isp[k] = 0;
        }
        __syncthreads();

        // ---- 2. augmented rows [H_sorted | s] into registers
        uint64_t row[RS][W];
#pragma unroll
        for (int s = 0; s < RS; ++s) {
#pragma unroll
            for (int w = 0; w < W; ++w) row[s][w] = 0;
            const int i = s * 64 + lane;
            if (i < m) {
                int sb = a.syn ? (a.syn[shot * m + i] & 1) : 0;
                for (int e = rp[i]; e < rp[i + 1]; ++e) {
                    const int j = ci[e];
                    flip_bit<W>(row[s], pos[j]);
                    if (a.syn_flags && j < g.n_data) {
                        if ((a.syn_flags & 1) && a.base) sb ^= a.base[shot * g.n_data + j] & 1;
                        if ((a.syn_flags & 2) && a.readout) sb ^= a.readout[shot * g.n_data + j] & 1;
                    }
                }
                if (sb) flip_bit<W>(row[s], n);
            }
        }

        // ---- 3. Gauss-Jordan in sorted column order.  The word index is a
        // compile-time constant in every instantiation of `step` (static_for), so
        // row[][] stays in registers (a runtime word index would demote it to
        // scratch memory).
        int rank = 0;
        static_for<0, W>([&](auto wwc) {
            constexpr int ww = decltype(wwc)::value;
            for (int b = 0; b < 64; ++b) {
                const int k = ww * 64 + b;
                if (k >= n || rank >= m) return;
                int piv = -1;
#pragma unroll
                for (int s = 0; s < RS; ++s) {
                    const int i = s * 64 + lane;
                    const uint64_t bal = __ballot(((row[s][ww] >> b) & 1) && i >= rank && i < m);
                    if (piv < 0 && bal) piv = s * 64 + __builtin_ctzll(bal);
                }
                if (piv < 0) continue;
                const int pl = piv & 63, ps = piv >> 6;
                uint64_t P[W];
#pragma unroll
                for (int w = 0; w < W; ++w) P[w] = 0;
#pragma unroll
                for (int s = 0; s < RS; ++s)
                    if (s == ps)
#pragma unroll
                        for (int w = ww; w < W; ++w) P[w] = readlane64(row[s][w], pl);
                if (piv != rank) {  // swap rows piv and rank (words left of ww are zero in both)
                    const int rl = rank & 63, rsl = rank >> 6;
                    uint64_t Q[W];
#pragma unroll
                    for (int w = 0; w < W; ++w) Q[w] = 0;
#pragma unroll
                    for (int s = 0; s < RS; ++s)
                        if (s == rsl)
#pragma unroll
                            for (int w = ww; w < W; ++w) Q[w] = readlane64(row[s][w], rl);
#pragma unroll
                    for (int s = 0; s < RS; ++s)
#pragma unroll
                        for (int w = ww; w < W; ++w) {
                            if (s == rsl && lane == rl) row[s][w] = P[w];
                            if (s == ps && lane == pl) row[s][w] = Q[w];
                        }
                }
#pragma unroll
                for (int s = 0; s < RS; ++s) {
                    const int i = s * 64 + lane;
                    const uint64_t hit = (((row[s][ww] >> b) & 1) && i != rank) ? ~0ull : 0ull;
#pragma unroll
                    for (int w = ww; w < W; ++w) row[s][w] ^= P[w] & hit;
                }
                if (lane == 0) {
                    pivc[rank] = (uint16_t)k;
                    isp[k] = 1;
                }
                ++rank;
            }
        });

        // ---- 4. reduced rows to LDS, transformed syndrome, non-pivot columns
        uint64_t x0[RS];
#pragma unroll
        for (int s = 0; s < RS; ++s) {
            const int i = s * 64 + lane;
#pragma unroll
            for (int w = 0; w < W; ++w) red[(size_t)i * W + w] = row[s][w];
            x0[s] = __ballot(i < rank && get_bit<W>(row[s], n));
        }
        __syncthreads();
        int kn = 0;
        for (int base = 0; base < n; base += 64) {
            const int k = base + lane;
            const bool f = k < n && !isp[k];
            const uint64_t bal = __ballot(f);
            if (f) npv[kn + __popcll(bal & ((1ull << lane) - 1ull))] = (uint16_t)k;
            kn += __popcll(bal);
        }
        __syncthreads();
        auto tcol = [&](int k, uint64_t (&tc)[RS]) {
            const int w = k >> 6, b = k & 63;
#pragma unroll
            for (int s = 0; s < RS; ++s) {
                const int i = s * 64 + lane;
                tc[s] = __ballot(i < rank && ((red[(size_t)i * W + w] >> b) & 1));
            }
        };
        const int lam = a.order < 0 ? 0 : (a.order < kn ? a.order : kn);
        const int lam_s = lam < kOsdMaxLam ? lam : kOsdMaxLam;
        for (int t = 0; t < lam_s; ++t) {
            uint64_t tc[RS];
            tcol(npv[t], tc);
            if (lane == 0)
#pragma unroll
                for (int s = 0; s < RS; ++s) tcl[t * RS + s] = tc[s];
        }
        __syncthreads();

        // ---- 5. candidate search (kind 0: OSD-0, 1: single, 2: pair, 3: OSD-E mask)
        int best_w = 0;
#pragma unroll
        for (int s = 0; s < RS; ++s) best_w += __popcll(x0[s]);
        int kind = 0, ca = -1, cb = -1;
        uint32_t cmask = 0;
        if (a.method == 2) {
            for (int t = 0; t < kn; ++t) {
                uint64_t tc[RS];
                tcol(npv[t], tc);
                int wgt = 1;
#pragma unroll
                for (int s = 0; s < RS; ++s) wgt += __popcll(x0[s] ^ tc[s]);
                if (wgt < best_w) {
                    best_w = wgt;
                    kind = 1;
                    ca = t;
                }
            }
            for (int u = 0; u < lam_s; ++u)
                for (int v = u + 1; v < lam_s; ++v) {
                    int wgt = 2;
#pragma unroll
                    for (int s = 0; s < RS; ++s) wgt += __popcll(x0[s] ^ tcl[u * RS + s] ^ tcl[v * RS + s]);
                    if (wgt < best_w) {
                        best_w = wgt;
                        kind = 2;
                        ca = u;
                        cb = v;
                    }
                }
        } else if (a.method == 1 && lam_s > 0) {
            uint64_t bestkey = ~0ull;
            const uint32_t lim = 1u << lam_s;
            for (uint32_t sm = 1 + lane; sm < lim; sm += 64) {
                uint64_t c[RS];
#pragma unroll
                for (int s = 0; s < RS; ++s) c[s] = x0[s];
                for (int t = 0; t < lam_s; ++t)
                    if ((sm >> t) & 1)
#pragma unroll
                        for (int s = 0; s < RS; ++s) c[s] ^= tcl[t * RS + s];
                int wgt = __popc(sm);
#pragma unroll
                for (int s = 0; s < RS; ++s) wgt += __popcll(c[s]);
                const uint64_t key = ((uint64_t)wgt << 32) | sm;
                bestkey = key < bestkey ? key : bestkey;
            }
            bestkey = wave_min_u64(bestkey);
            if ((int)(bestkey >> 32) < best_w) {
                best_w = (int)(bestkey >> 32);
                kind = 3;
                cmask = (uint32_t)bestkey;
            }
        }

        // ---- 6. outputs: osd0, then the best candidate (+ fused fold / failure check)
        auto emit = [&](const uint64_t (&xp)[RS], int kd) {
            for (int j = lane; j < n; j += 64) outb[j] = 0;
            __syncthreads();
#pragma unroll
            for (int s = 0; s < RS; ++s) {
                const int i = s * 64 + lane;
                if (i < rank && ((xp[s] >> lane) & 1)) outb[sidx[pivc[i]]] = 1;
            }
            __syncthreads();
            if (lane == 0) {
                if (kd == 1) outb[sidx[npv[ca]]] ^= 1;
                if (kd == 2) {
                    outb[sidx[npv[ca]]] ^= 1;
                    outb[sidx[npv[cb]]] ^= 1;
                }
                if (kd == 3)
                    for (int t = 0; t < lam_s; ++t)
                        if ((cmask >> t) & 1) outb[sidx[npv[t]]] ^= 1;
            }
            __syncthreads();
        };
        if (a.osd0_out) {
            emit(x0, 0);
            for (int j = lane; j < n; j += 64) a.osd0_out[shot * n + j] = outb[j];
        }
        uint64_t xp[RS];
#pragma unroll
        for (int s = 0; s < RS; ++s) xp[s] = x0[s];
        if (kind == 1) {
            uint64_t tc[RS];
            tcol(npv[ca], tc);
#pragma unroll
            for (int s = 0; s < RS; ++s) xp[s] ^= tc[s];
        } else if (kind == 2) {
#pragma unroll
            for (int s = 0; s < RS; ++s) xp[s] ^= tcl[ca * RS + s] ^ tcl[cb * RS + s];
        } else if (kind == 3) {
            for (int t = 0; t < lam_s; ++t)
                if ((cmask >> t) & 1)
#pragma unroll
                    for (int s = 0; s < RS; ++s) xp[s] ^= tcl[t * RS + s];
        }
        emit(xp, kind);
        DecodeArgs fa{};
        fa.B = a.B;
        fa.base = a.base;
        fa.readout = a.readout;
        fa.x_out = a.osdw_out;
        fa.corr_out = a.corr_out;
        fa.fail = a.fail;
        finalize_shot(g, fa, shot, outb, false, false, 0, lane);
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Workgroup variant for graphs beyond the register kernel (m > 384 or n >= 1024,
// e.g. the R = 3 spacetime matrix 432 x 1224 of the reference's default bposd
// mode): one 256-thread workgroup per BP-failed shot, the augmented rows
// [H_sorted | s] in LDS as W 64-bit words each.  Same spec and tie rules as
// osd_wave_kernel / the host stage (steps 1-6 above); the elimination walks the
// sorted columns with the whole workgroup: block-wide first-row pivot search
// (LDS atomic min), row swap, then the rows holding the pivot bit (flags taken
// before any write) XOR the pivot row, over (row, word) pairs.  Candidate
// weights are computed thread-parallel and the winner is the minimum of
// (weight, position in the host's candidate order).
constexpr int kOsdBlock = 256;

struct OsdBlockLayout {
    int ns, W, RW, o_rows, o_key, o_idx, o_pos, o_piv, o_npv, o_isp, o_out, o_hit, o_x0, o_tcl, o_ctl, total;
    __host__ __device__ OsdBlockLayout(int n, int m) {
        ns = 64;
        while (ns < n) ns <<= 1;
        W = (n + 1 + 63) / 64;
        RW = (m + 63) / 64;
        int o = 0;
        auto take = [&](int bytes) {
            const int at = o;
            o += (bytes + 15) / 16 * 16;
            return at;
        };
        o_rows = take(8 * m * W);
        o_key = take(8 * ns);
        o_x0 = take(8 * RW);
        o_tcl = take(8 * kOsdMaxLam * RW);
        o_ctl = take(64);
        o_idx = take(2 * ns);
        o_pos = take(2 * n);
        o_piv = take(2 * (m > 0 ? m : 1));
        o_npv = take(2 * n);
        o_isp = take(n);
        o_out = take(n);
        o_hit = take(m);
        total = o;
    }
};

__global__ __launch_bounds__(kOsdBlock) void osd_block_kernel(DevGraph g, OsdArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int m = g.m, n = g.n;
    const OsdBlockLayout L(n, m);
    const int W = L.W, RW = L.RW, NS = L.ns;
    uint64_t* A = reinterpret_cast<uint64_t*>(smem + L.o_rows);       // [m][W]
    uint64_t* skey = reinterpret_cast<uint64_t*>(smem + L.o_key);
    uint64_t* x0 = reinterpret_cast<uint64_t*>(smem + L.o_x0);        // [RW] transformed syndrome over pivot rows
    uint64_t* tcl = reinterpret_cast<uint64_t*>(smem + L.o_tcl);      // [lam][RW] transformed columns
    unsigned long long* ctl = reinterpret_cast<unsigned long long*>(smem + L.o_ctl);  // [0] pivot, [1] best key
    uint16_t* sidx = reinterpret_cast<uint16_t*>(smem + L.o_idx);
    uint16_t* pos = reinterpret_cast<uint16_t*>(smem + L.o_pos);
    uint16_t* pivc = reinterpret_cast<uint16_t*>(smem + L.o_piv);
    uint16_t* npv = reinterpret_cast<uint16_t*>(smem + L.o_npv);
    uint8_t* isp = smem + L.o_isp;
    uint8_t* outb = smem + L.o_out;
    uint8_t* hit = smem + L.o_hit;
    const int32_t* rp = g.row_ptr;
    const int32_t* ci = g.col_idx;
    auto bit = [&](int i, int k) -> int { return (int)((A[(size_t)i * W + (k >> 6)] >> (k & 63)) & 1); };

    for (int64_t shot = blockIdx.x; shot < a.B; shot += gridDim.x) {
        if (a.status && (a.status[shot] & 1)) continue;  // uniform over the workgroup
        // ---- 1. stable sort of the columns by log-probability ratio
        for (int k = tid; k < NS; k += kOsdBlock) {
            uint64_t key = ~0ull;
            uint16_t idx = 0xffff;
            if (k < n) {
                const double v = a.llr_f32 ? (double)static_cast<const float*>(a.llr)[shot * n + k]
                                           : static_cast<const double*>(a.llr)[shot * n + k];
                key = order_key(v);
                idx = (uint16_t)k;
            }
            skey[k] = key;
            sidx[k] = idx;
        }
        __syncthreads();
        for (int size = 2; size <= NS; size <<= 1) {
            for (int stride = size >> 1; stride > 0; stride >>= 1) {
                for (int t = tid; t < NS / 2; t += kOsdBlock) {
                    const int i = 2 * t - (t & (stride - 1));
                    const int j = i + stride;
                    const uint64_t ki = skey[i], kj = skey[j];
                    const uint16_t ii = sidx[i], ij = sidx[j];
                    const bool gt = ki > kj || (ki == kj && ii > ij);
                    if (gt == ((i & size) == 0)) {
                        skey[i] = kj;
                        skey[j] = ki;
                        sidx[i] = ij;
                        sidx[j] = ii;
                    }
                }
                __syncthreads();
            }
        }
        for (int k = tid; k < n; k += kOsdBlock) {
            pos[sidx[k]] = (uint16_t)k;
            isp[k] = 0;
        }
        for (int e = tid; e < m * W; e += kOsdBlock) A[e] = 0;
        __syncthreads();

        // ---- 2. augmented rows [H_sorted | s] (one thread per row)
        for (int i = tid; i < m; i += kOsdBlock) {
            uint64_t* r = A + (size_t)i * W;
            int sb = a.syn ? (a.syn[shot * m + i] & 1) : 0;
            for (int e = rp[i]; e < rp[i + 1]; ++e) {
                const int j = ci[e];
                const int k = pos[j];
                r[k >> 6] ^= 1ull << (k & 63);
                if (a.syn_flags && j < g.n_data) {
                    if ((a.syn_flags & 1) && a.base) sb ^= a.base[shot * g.n_data + j] & 1;
                    if ((a.syn_flags & 2) && a.readout) sb ^= a.readout[shot * g.n_data + j] & 1;
                }
            }
            if (sb) r[n >> 6] ^= 1ull << (n & 63);
        }
        __syncthreads();

        // ---- 3. Gauss-Jordan in sorted column order
        int rank = 0;
        for (int k = 0; k < n && rank < m; ++k) {
            if (tid == 0) ctl[0] = ~0ull;
            __syncthreads();
            unsigned long long cand = ~0ull;
            for (int i = rank + tid; i < m; i += kOsdBlock)
                if (bit(i, k)) {
                    cand = (unsigned long long)i;
                    break;
                }
            if (cand != ~0ull) atomicMin(&ctl[0], cand);
            __syncthreads();
            const unsigned long long pv = ctl[0];
            if (pv == ~0ull) continue;  // uniform
            const int piv = (int)pv, ww = k >> 6;
            if (piv != rank)
                for (int w = ww + tid; w < W; w += kOsdBlock) {
                    const uint64_t t = A[(size_t)piv * W + w];
                    A[(size_t)piv * W + w] = A[(size_t)rank * W + w];
                    A[(size_t)rank * W + w] = t;
                }
            for (int i = tid; i < m; i += kOsdBlock) hit[i] = (uint8_t)(i != rank && i != piv && bit(i, k));
            __syncthreads();
            if (tid == 0) hit[piv] = (uint8_t)(piv != rank && bit(piv, k));  // the swapped-out row
            __syncthreads();
            const int nw = W - ww;
            for (int e = tid; e < m * nw; e += kOsdBlock) {
                const int i = e / nw, w = ww + e % nw;
                if (hit[i]) A[(size_t)i * W + w] ^= A[(size_t)rank * W + w];
            }
            if (tid == 0) {
                pivc[rank] = (uint16_t)k;
                isp[k] = 1;
            }
            ++rank;
            __syncthreads();
        }

        // ---- 4. transformed syndrome, non-pivot columns, the first lam transformed columns
        for (int w = tid; w < RW; w += kOsdBlock) {
            uint64_t v = 0;
            for (int b = 0; b < 64; ++b) {
                const int i = w * 64 + b;
                if (i < rank && bit(i, n)) v |= 1ull << b;
            }
            x0[w] = v;
        }
        if (wave == 0) {
            int kn = 0;
            for (int base = 0; base < n; base += 64) {
                const int k = base + lane;
                const bool f = k < n && !isp[k];
                const uint64_t bal = __ballot(f);
                if (f) npv[kn + __popcll(bal & ((1ull << lane) - 1ull))] = (uint16_t)k;
                kn += __popcll(bal);
            }
            if (lane == 0) ctl[2] = (unsigned long long)kn;
        }
        __syncthreads();
        const int kn = (int)ctl[2];
        const int lam = a.order < 0 ? 0 : (a.order < kn ? a.order : kn);
        const int lam_s = lam < kOsdMaxLam ? lam : kOsdMaxLam;
        for (int e = tid; e < lam_s * RW; e += kOsdBlock) {
            const int t = e / RW, w = e % RW, k = npv[t];
            uint64_t v = 0;
            for (int b = 0; b < 64; ++b) {
                const int i = w * 64 + b;
                if (i < rank && bit(i, k)) v |= 1ull << b;
            }
            tcl[t * RW + w] = v;
        }
        int w0 = 0;
        for (int w = 0; w < RW; ++w) w0 += __popcll(x0[w]);
        if (tid == 0) ctl[1] = ((unsigned long long)w0 << 32);  // OSD-0: weight, order 0
        __syncthreads();

        // ---- 5. candidates: key = weight << 32 | position in the host's order
        // (1 + t: single t, 1 + kn + pair index, or the OSD-E mask)
        unsigned long long best = ~0ull;
        if (a.method == 2) {
            for (int t = tid; t < kn; t += kOsdBlock) {
                const int k = npv[t];
                int wgt = 1;
                for (int w = 0; w < RW; ++w) {
                    uint64_t v = 0;
                    for (int b = 0; b < 64; ++b) {
                        const int i = w * 64 + b;
                        if (i < rank && bit(i, k)) v |= 1ull << b;
                    }
                    wgt += __popcll(x0[w] ^ v);
                }
                const unsigned long long key = ((unsigned long long)wgt << 32) | (unsigned long long)(1 + t);
                best = key < best ? key : best;
            }
            const int np = lam_s * (lam_s - 1) / 2;
            for (int q = tid; q < np; q += kOsdBlock) {
                int u = 0, rem = q;  // q -> (u, v), u < v, lexicographic
                while (rem >= lam_s - 1 - u) {
                    rem -= lam_s - 1 - u;
                    ++u;
                }
                const int v = u + 1 + rem;
                int wgt = 2;
                for (int w = 0; w < RW; ++w) wgt += __popcll(x0[w] ^ tcl[u * RW + w] ^ tcl[v * RW + w]);
                const unsigned long long key = ((unsigned long long)wgt << 32) | (unsigned long long)(1 + kn + q);
                best = key < best ? key : best;
            }
        } else if (a.method == 1 && lam_s > 0) {
            const uint32_t lim = 1u << lam_s;
            for (uint32_t sm = 1 + tid; sm < lim; sm += kOsdBlock) {
                int wgt = __popc(sm);
                for (int w = 0; w < RW; ++w) {
                    uint64_t c = x0[w];
                    for (int t = 0; t < lam_s; ++t)
                        if ((sm >> t) & 1) c ^= tcl[t * RW + w];
                    wgt += __popcll(c);
                }
                const unsigned long long key = ((unsigned long long)wgt << 32) | sm;
                best = key < best ? key : best;
            }
        }
        // OSD-0 keeps a tie (strict improvement): its key has the lowest position
        if (best != ~0ull) atomicMin(&ctl[1], best);
        __syncthreads();
        const unsigned long long bk = ctl[1];
        const int bpos = (int)(bk & 0xffffffffu);
        int kind = 0, ca = -1, cb = -1;
        uint32_t cmask = 0;
        if (bpos != 0) {
            if (a.method == 2) {
                if (bpos <= kn) {
                    kind = 1;
                    ca = bpos - 1;
                } else {
                    int q = bpos - 1 - kn, u = 0;
                    while (q >= lam_s - 1 - u) {
                        q -= lam_s - 1 - u;
                        ++u;
                    }
                    kind = 2;
                    ca = u;
                    cb = u + 1 + q;
                }
            } else {
                kind = 3;
                cmask = (uint32_t)bpos;
            }
        }

        // ---- 6. outputs (osd0, then the chosen candidate + fused fold / failure check)
        auto emit = [&](int kd) {
            for (int j = tid; j < n; j += kOsdBlock) outb[j] = 0;
            __syncthreads();
            for (int i = tid; i < rank; i += kOsdBlock) {
                int xb = (int)((x0[i >> 6] >> (i & 63)) & 1);
                if (kd == 1) xb ^= bit(i, npv[ca]);
                if (kd == 2) xb ^= (int)(((tcl[ca * RW + (i >> 6)] ^ tcl[cb * RW + (i >> 6)]) >> (i & 63)) & 1);
                if (kd == 3)
                    for (int t = 0; t < lam_s; ++t)
                        if ((cmask >> t) & 1) xb ^= (int)((tcl[t * RW + (i >> 6)] >> (i & 63)) & 1);
                if (xb) outb[sidx[pivc[i]]] = 1;
            }
            __syncthreads();
            if (tid == 0) {
                if (kd == 1) outb[sidx[npv[ca]]] ^= 1;
                if (kd == 2) {
                    outb[sidx[npv[ca]]] ^= 1;
                    outb[sidx[npv[cb]]] ^= 1;
                }
                if (kd == 3)
                    for (int t = 0; t < lam_s; ++t)
                        if ((cmask >> t) & 1) outb[sidx[npv[t]]] ^= 1;
            }
            __syncthreads();
        };
        if (a.osd0_out) {
            emit(0);
            for (int j = tid; j < n; j += kOsdBlock) a.osd0_out[shot * n + j] = outb[j];
            __syncthreads();
        }
        emit(kind);
        if (wave == 0) {
            DecodeArgs fa{};
            fa.B = a.B;
            fa.base = a.base;
            fa.readout = a.readout;
            fa.x_out = a.osdw_out;
            fa.corr_out = a.corr_out;
            fa.fail = a.fail;
            finalize_shot(g, fa, shot, outb, false, false, 0, lane);
        }
        __syncthreads();
    }
}

namespace {
template <int RS, int W>
int launch_osd_shape(const DevGraph& g, const OsdArgs& a, int num_cus, hipStream_t stream) {
    const OsdLayout L(g.n, g.m, RS, W);
    int per_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, osd_wave_kernel<RS, W>, 64, L.total);
    if (e != hipSuccess) return (int)e;
    if (per_cu <= 0) return (int)hipErrorInvalidConfiguration;
    long long grid = (long long)num_cus * per_cu;
    if (grid > a.B) grid = a.B;
    if (grid <= 0) return 0;
    hipLaunchKernelGGL((osd_wave_kernel<RS, W>), dim3((unsigned)grid), dim3(64), L.total, stream, g, a);
    return (int)hipGetLastError();
}
}  // namespace

#define QDEC_OSD_SHAPES(X) X(2, 4) X(2, 6) X(2, 9) X(2, 16) X(4, 6) X(4, 9) X(4, 12) X(4, 16) X(6, 14) X(6, 16)

static int osd_row_slots(int m) { return m <= 128 ? 2 : (m <= 256 ? 4 : 6); }

static bool osd_wave_supports(const DevGraph& g) {
    if (g.m <= 0 || g.m > 384 || g.n + 1 > 1024) return false;
    const int rs = osd_row_slots(g.m);
    const int need = (g.n + 1 + 63) / 64;
#define QDEC_OSD_FITS(R, V) if (rs == R && need <= V) return true;
    QDEC_OSD_SHAPES(QDEC_OSD_FITS)
#undef QDEC_OSD_FITS
    return false;
}

// the workgroup variant: its LDS image within one CU's 160 KiB, 16-bit indices
static bool osd_block_supports(const DevGraph& g) {
    if (g.m <= 0 || g.n <= 0 || g.n >= 65535 || g.m >= 65535) return false;
    return OsdBlockLayout(g.n, g.m).total <= 160 * 1024 && g.k <= 256;
}

bool osd_kernel_supports(const DevGraph& g) { return osd_wave_supports(g) || osd_block_supports(g); }

int launch_osd(const DevGraph& g, const OsdArgs& a, int num_cus, hipStream_t stream) {
    if (a.B <= 0) return 0;
    if (!osd_wave_supports(g)) {
        if (!osd_block_supports(g)) return (int)hipErrorNotSupported;
        const OsdBlockLayout L(g.n, g.m);
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&osd_block_kernel),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, L.total);
        if (e != hipSuccess) return (int)e;
        int per_cu = 0;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, osd_block_kernel, kOsdBlock, L.total);
        if (e != hipSuccess) return (int)e;
        if (per_cu <= 0) return (int)hipErrorInvalidConfiguration;
        long long grid = (long long)num_cus * per_cu;
        if (grid > a.B) grid = a.B;
        hipLaunchKernelGGL(osd_block_kernel, dim3((unsigned)grid), dim3(kOsdBlock), L.total, stream, g, a);
        return (int)hipGetLastError();
    }
    const int rs = osd_row_slots(g.m);
    const int need = (g.n + 1 + 63) / 64;
#define QDEC_OSD_LAUNCH(R, V) \
    if (rs == R && need <= V) return launch_osd_shape<R, V>(g, a, num_cus, stream);
    QDEC_OSD_SHAPES(QDEC_OSD_LAUNCH)
#undef QDEC_OSD_LAUNCH
    return (int)hipErrorNotSupported;
}

}  // namespace qdec
