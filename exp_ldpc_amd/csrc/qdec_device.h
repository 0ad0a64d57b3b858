// qdec_device.h -- device helpers shared by the wave kernels (qdec_bp.hip) and
// the workgroup kernels (qdec_bp_block.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "qdec_internal.h"

namespace qdec {

// Development-only phase timers (build with -DQDEC_STAMPS: `python -m
// exp_ldpc_amd.build --stamps`): per-wave s_memtime deltas accumulated into a
// device array, read with qd_dev_read_stamps.
#ifdef QDEC_STAMPS
static __device__ unsigned long long qdec_stamps[64];
#define QDEC_STAMP_DECL                                                   \
    unsigned long long qdec_acc_[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}; \
    unsigned long long qdec_st_prev_ = __builtin_amdgcn_s_memtime();
#define QDEC_STAMP(k)                                                  \
    do {                                                               \
        const unsigned long long qdec_n_ = __builtin_amdgcn_s_memtime(); \
        qdec_acc_[k] += qdec_n_ - qdec_st_prev_;                       \
        qdec_st_prev_ = qdec_n_;                                       \
    } while (0)
#define QDEC_COUNT(k, v) qdec_acc_[k] += (unsigned long long)(v)
#define QDEC_FLUSH_AT(off)                                                    \
    do {                                                                      \
        if ((threadIdx.x & 63) == 0)                                          \
            for (int qdec_k_ = 0; qdec_k_ < 16; ++qdec_k_) atomicAdd(&qdec_stamps[(off) + qdec_k_], qdec_acc_[qdec_k_]); \
    } while (0)
#else
#define QDEC_STAMP_DECL
#define QDEC_STAMP(k) \
    do {              \
    } while (0)
#define QDEC_COUNT(k, v) \
    do {                 \
    } while (0)
#define QDEC_FLUSH_AT(off) \
    do {                   \
    } while (0)
#endif

// Parity of popc(X & M) over NW 64-bit words, X wave-uniform (ballot words).
// Two 32-bit accumulators, each step acc = (M & X) ^ acc as one v_bitop3_b32
// (table 0x6c = (src0 & src2) ^ src1); written as the builtin so the xor chain
// is not reassociated into and/and/xor triples.
template <int NW>
__device__ __forceinline__ int masked_parity(const uint64_t (&M)[NW], const uint64_t (&X)[NW]) {
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        lo = __builtin_amdgcn_bitop3_b32((uint32_t)M[w], lo, (uint32_t)X[w], 0x6c);
        hi = __builtin_amdgcn_bitop3_b32((uint32_t)(M[w] >> 32), hi, (uint32_t)(X[w] >> 32), 0x6c);
    }
    return __builtin_popcount(lo ^ hi) & 1;
}

// Orders this wave's LDS accesses across lanes.  A wave's LDS operations
// execute in issue order, so for a one-wave workgroup (or a wave working on its
// own LDS region) it is enough to keep the compiler from moving them; unlike
// __syncthreads() this does not wait for outstanding LDS operations to drain.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <typename T>
struct Big;
template <>
struct Big<float> {
    static constexpr float v = 1e30f;  // fp32 stand-in for ldpc's 1e308 "no minimum yet"
};
template <>
struct Big<double> {
    static constexpr double v = 1e308;
};

// 16-byte LDS vector loads of D consecutive elements (16-B aligned).
template <typename T, int D>
__device__ __forceinline__ void lds_load(const T* p, T (&v)[D]) {
    static_assert((D * sizeof(T)) % 16 == 0, "row must be a multiple of 16 bytes");
    using V = __attribute__((ext_vector_type(16 / sizeof(T)))) T;
    constexpr int per = 16 / sizeof(T);
#pragma unroll
    for (int c = 0; c < D / per; ++c) {
        V x = *reinterpret_cast<const V*>(p + c * per);
#pragma unroll
        for (int e = 0; e < per; ++e) v[c * per + e] = x[e];
    }
}

// The first N elements of a 16-B aligned row: 16-byte loads, then one 8-byte
// load for an odd f64 tail (a degree-7 f64 row: 3 x ds_read_b128 + ds_read_b64,
// 14 LDS cycles instead of the 16 of four b128 loads).  Elements >= N of v are
// left unset.
template <typename T, int N, int D>
__device__ __forceinline__ void lds_load_first(const T* p, T (&v)[D]) {
    static_assert(N <= D && sizeof(T) == 8, "f64 rows");
    using V = __attribute__((ext_vector_type(2))) T;
#pragma unroll
    for (int c = 0; c < N / 2; ++c) {
        V x = *reinterpret_cast<const V*>(p + 2 * c);
        v[2 * c] = x[0];
        v[2 * c + 1] = x[1];
    }
    if constexpr (N % 2) v[N - 1] = p[N - 1];
}

__device__ __forceinline__ long long wave_max_i64(long long v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        int lo = __shfl_xor((int)(unsigned)(v & 0xffffffffll), off);
        int hi = __shfl_xor((int)(v >> 32), off);
        long long o = ((long long)hi << 32) | (unsigned)lo;
        v = o > v ? o : v;
    }
    return v;
}

__device__ __forceinline__ int wave_sum_i32(int v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// median of three with lo <= hi: clamp(a, lo, hi) = min(hi, max(lo, a))
__device__ __forceinline__ float med3(float a, float lo, float hi) { return __builtin_amdgcn_fmed3f(a, lo, hi); }
__device__ __forceinline__ double med3(double a, double lo, double hi) { return fmin(hi, fmax(lo, a)); }

template <typename T>
__device__ __forceinline__ T alpha_at(int it, double ms_scaling) {
    return ms_scaling == 0.0 ? (T)(1.0 - ldexp(1.0, -it)) : (T)ms_scaling;
}

// 840/size for SSF subset sizes 1..8 (index 0 unused); read with uniform indices
// (scalar loads).
static __constant__ int kInvSize[9] = {0, 840, 420, 280, 210, 168, 140, 120, 105};


// Best small-set-flip key of one generator: all subsets t of its <= 8 qubits,
// key32 = (gain * 840/|t|) << 8 | (255 - t), where gain = popc(sl) -
// popc(sl ^ M_t), M_t = xor of the qubits' local-check masks qm.  Subsets using
// qubits beyond the generator's weight have zero masks (same gain, larger |t|),
// so they never win; t = 0 scores 0 and is never selected (a flip needs a
// positive score).  5 VALU ops per subset; nhi = 2^(wmax-4) blocks of 16.
__device__ __forceinline__ int gen_best_key(uint32_t sl, const uint32_t (&qm)[kGenW], int nhi) {
    const int base = __builtin_popcount(sl);
    uint32_t lo[16];
    lo[0] = 0;
#pragma unroll
    for (int l = 1; l < 16; ++l) lo[l] = lo[l & (l - 1)] ^ qm[__builtin_ctz(l)];
    int best32 = INT_MIN;
#pragma unroll 1
    for (int hi = 0; hi < nhi; ++hi) {
        uint32_t mh = 0;
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) mh ^= ((hi >> bb) & 1) ? qm[4 + bb] : 0u;
        const uint32_t sh = sl ^ mh;
        const int hs = __builtin_popcount(hi);
        int ih[5];  // 840/size for size = hs + popc(l)
#pragma unroll
        for (int d = 0; d < 5; ++d) ih[d] = kInvSize[hs + d];  // uniform scalar loads
#pragma unroll
        for (int l = 0; l < 16; ++l) {
            const int d = __builtin_popcount(l);
            // full-rate 24-bit multiply (|base - cnt| <= 32, ih <= 840)
            const int score = __mul24(base - (int)__builtin_popcount(sh ^ lo[l]), ih[d]);
            const int t = hi * 16 + l;
            const int key = (int)(((unsigned)score << 8) | (unsigned)(255 - t));
            best32 = key > best32 ? key : best32;
        }
    }
    return best32;
}

// Wave-wide max of an int with DPP row shifts and row broadcasts (VALU only, no
// LDS round trips): inclusive max-scan within each 16-lane row, then rows 0-1
// and 2-3 via row_bcast:15, then all four via row_bcast:31; lane 63 holds the
// result.  All 64 lanes must be active.
__device__ __forceinline__ int wave_max_i32(int v) {
#define QDEC_DPP_MAX(ctrl, rm, bm) v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, ctrl, rm, bm, false))
    QDEC_DPP_MAX(0x111, 0xf, 0xf);  // row_shr:1
    QDEC_DPP_MAX(0x112, 0xf, 0xf);  // row_shr:2
    QDEC_DPP_MAX(0x114, 0xf, 0xf);  // row_shr:4
    QDEC_DPP_MAX(0x118, 0xf, 0xf);  // row_shr:8
    QDEC_DPP_MAX(0x142, 0xa, 0xf);  // row_bcast:15 -> rows 1, 3
    QDEC_DPP_MAX(0x143, 0xc, 0xf);  // row_bcast:31 -> rows 2, 3
#undef QDEC_DPP_MAX
    return __builtin_amdgcn_readlane(v, 63);
}

// XOR over lanes 0..7 of v (other lanes must pass 0), result in every lane.
__device__ __forceinline__ int wave_xor_masked(int v) {
    v ^= __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v ^= __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v ^= __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);  // row_shr:4
    return __builtin_amdgcn_readlane(v, 7);
}

// Best small-set-flip SCORE of one generator (the subset itself is recovered
// afterwards, for the winning generator only; ssf_pick_subset).  For every
// subset size d the minimum residual weight popc(sl ^ M_t) over |t| = d is kept
// (3 VALU per subset: xor, popcount, min), then score = max_d (popc(sl) -
// min_d) * 840/d.  Subsets are visited in Gray-code order, so each one's
// residual is the previous one's with one qubit mask XORed in (no table of
// subset masks in registers), and the first 2^w of them are exactly the
// subsets of the first w qubits.  Subsets using qubits beyond the generator's
// weight have zero masks and a larger |t| than the same subset without them,
// so they never raise the maximum of a positive score.  nhi = 2^(wmax-4)
// blocks of 16.
__device__ __forceinline__ int gen_best_score(uint32_t sl, const uint32_t (&qm)[kGenW], int nhi) {
    const int base = __builtin_popcount(sl);
    uint32_t mn[kGenW + 1];
#pragma unroll
    for (int d = 0; d <= kGenW; ++d) mn[d] = 64u;
    uint32_t r = sl;  // residual of the current Gray-code subset
#pragma unroll
    for (int blk = 0; blk < 16; ++blk) {
        if (blk < nhi) {  // uniform
#pragma unroll
            for (int l = 0; l < 16; ++l) {
                const int t = blk * 16 + l;
                if (t == 0) continue;  // empty set
                r ^= qm[__builtin_ctz(t)];
                const int d = __builtin_popcount(t ^ (t >> 1));
                mn[d] = min(mn[d], (uint32_t)__builtin_popcount(r));
            }
        }
    }
    int best = INT_MIN;
#pragma unroll
    for (int d = 1; d <= kGenW; ++d) best = max(best, (base - (int)mn[d]) * (840 / d));
    return best;
}

// A 1/S share of a generator's subsets (S = 2 or 4), for listing steps with
// <= 64/S generators: the S lanes l + (64/S) q, q < S, score the same generator,
// lane q taking the subsets whose top log2(S) qubits (the generator's last ones)
// are the bits of q, the others in Gray-code order over the first qubits.
// Per-size minima are then combined by lane-xor shuffles and lane q = 0 gets
// the same score as gen_best_score (the minima are over the same subsets).
// tq = masks of those top qubits (tq[0] the highest), part = nhi / S >= 1
// blocks of 16 per lane.
template <int S>
__device__ __forceinline__ int gen_best_score_split(uint32_t sl, const uint32_t (&qm)[kGenW], int part,
                                                    const uint32_t (&tq)[2], int q) {
    static_assert(S == 2 || S == 4, "split");
    const int base = __builtin_popcount(sl);
    uint32_t mn[kGenW + 1];
#pragma unroll
    for (int d = 0; d <= kGenW; ++d) mn[d] = 64u;
    // q's bit 0 selects the highest qubit, bit 1 (S = 4) the next one
    const uint32_t extra = ((q & 1) ? tq[0] : 0u) ^ ((S == 4 && (q & 2)) ? tq[1] : 0u);
    uint32_t r = sl ^ extra;  // residual of the current subset (top qubits of q included)
    if (q) mn[0] = (uint32_t)__builtin_popcount(r);  // the top qubits alone (the empty set on q = 0)
#pragma unroll
    for (int blk = 0; blk < 8; ++blk) {
        if (blk < part) {  // uniform
#pragma unroll
            for (int l = 0; l < 16; ++l) {
                const int t = blk * 16 + l;
                if (t == 0) continue;
                // dd = subset size without the top qubits; lane q's size is dd + popc(q)
                r ^= qm[__builtin_ctz(t)];
                const int dd = __builtin_popcount(t ^ (t >> 1));
                mn[dd] = min(mn[dd], (uint32_t)__builtin_popcount(r));
            }
        }
    }
    // lane q holds sizes dd + popc(q) at index dd; lane 0 folds in its partners
    uint32_t o1[kGenW + 1], o2[kGenW + 1], o3[kGenW + 1];
    constexpr int w = 64 / S;
#pragma unroll
    for (int d = 0; d <= kGenW; ++d) o1[d] = (uint32_t)__shfl_xor((int)mn[d], w);  // q ^ 1
    if constexpr (S == 4) {
#pragma unroll
        for (int d = 0; d <= kGenW; ++d) {
            o2[d] = (uint32_t)__shfl_xor((int)mn[d], 2 * w);      // q ^ 2
            o3[d] = (uint32_t)__shfl_xor((int)mn[d], 3 * w);      // q ^ 3
        }
    }
    int best = INT_MIN;
#pragma unroll
    for (int d = 1; d <= kGenW; ++d) {
        uint32_t m = min(mn[d], o1[d - 1]);
        if constexpr (S == 4) {
            m = min(m, o2[d - 1]);
            if (d >= 2) m = min(m, o3[d - 2]);
        }
        best = max(best, (base - (int)m) * (840 / d));
    }
    return best;
}

// (score, -g, -t) packed so that a signed max picks the spec's winner.
__device__ __forceinline__ long long gen_key64(int best32, int gi) {
    return ((long long)(best32 >> 8) << 32) | ((long long)(0xFFFFFF - gi) << 8) | (long long)(best32 & 255);
}

constexpr int kMaxLogicalRounds = 4;  // k <= 256 logicals in the fused check

// Final per-shot outputs from the hard decision in LDS: x_out, corr = base ^
// fold(x), fail = any_r parity(lz[r] & (readout ^ corr)), status, ssf_steps.
__device__ inline void finalize_shot(const DevGraph& g, const DecodeArgs& a, int64_t shot, const uint8_t* xh,
                              bool conv, bool satisfied, int steps, int lane) {
    const int n = g.n;
    if (a.x_out)
        for (int j = lane; j < n; j += 64) a.x_out[shot * n + j] = xh[j];
    const bool want_fail = a.fail && a.readout && g.k > 0;
    int lpar[kMaxLogicalRounds] = {0, 0, 0, 0};
    if (a.corr_out || want_fail) {
        for (int w0 = 0; w0 < g.lz_words; ++w0) {
            const int q = w0 * 64 + lane;
            int cb = 0;
            if (q < g.n_data) {
                cb = a.base ? (a.base[shot * g.n_data + q] & 1) : 0;
                for (int t = 0; t < g.fold_blocks; ++t) cb ^= xh[t * g.n_data + q];
                if (a.corr_out) a.corr_out[shot * g.n_data + q] = (uint8_t)cb;
            }
            if (want_fail) {
                const int v = (q < g.n_data) ? ((a.readout[shot * g.n_data + q] ^ cb) & 1) : 0;
                const unsigned long long word = __ballot(v);
#pragma unroll
                for (int rr = 0; rr < kMaxLogicalRounds; ++rr) {
                    const int r = rr * 64 + lane;
                    if (r < g.k) lpar[rr] ^= __popcll(g.lz[(size_t)r * g.lz_words + w0] & word) & 1;
                }
            }
        }
    }
    int any_fail = 0;
    if (want_fail) {
        int f = 0;
#pragma unroll
        for (int rr = 0; rr < kMaxLogicalRounds; ++rr) f |= lpar[rr];
        any_fail = __ballot(f) != 0ull;
    }
    if (lane == 0) {
        if (a.status) a.status[shot] = (uint8_t)((conv ? 1 : 0) | (satisfied ? 2 : 0));
        if (a.ssf_steps) a.ssf_steps[shot] = steps;
        if (a.fail) a.fail[shot] = (uint8_t)any_fail;
    }
}

// ---------------------------------------------------------------- shot I/O staging
// Per-wave LDS staging of shot inputs with LDS-DMA loads (global_load_lds: no
// VGPR destination, completes while the wave decodes).  At the start of shot s
// the wave stages the syndrome row and the readout row of shot s+1 (one
// persistent-loop step ahead), so no HBM round trip sits on a shot's critical
// path.  Rows are fetched as whole dwords (64 lanes x 4 B per instruction) from
// the dword-aligned address at or below the row start; `shift` is the row's
// byte offset inside the staged bytes.  The readout is double buffered (shot s
// reads its buffer at the end while s+1's lands).  Every stage issues the same
// number of loads (lanes past the row re-read its last dword, so a stage
// fetches the row's lines only; past the batch end it re-reads shot 0; lanes past the buffer
// read its last whole dword), so consumers wait with a counted vmcnt: vector
// memory operations retire in issue order and the kStaged most recent ones are
// the next shot's.  The final 1-3 bytes of a buffer whose length is not a
// multiple of 4 are not covered by a whole dword; the shot that needs them
// patches them in with byte loads (patch_tail).
// The wave kernels (one shot per wave: bp_ms_wave_kernel, ssf_wave_kernel)
// keep the dense logical table in LDS: for their graphs (n <= 576, so at most
// 9 words per logical) it is at most 41.5 KB, and C2's is 288 B.  Every word
// is read through an LDS-typed pointer: a generic (flat) load would wait for
// every vector-memory operation of the wave, i.e. for the next shot's LDS-DMA
// stage, serialising the stage with the shot (SSF launch at p = 0.032: 8.1 k of
// 18.7 k ticks per shot), and a global fallback path costs the f64 BP kernel 12
// VGPRs, past the 168 that fit three waves per SIMD.
__host__ __device__ inline bool lz_in_lds(const DevGraph& g) { return g.k > 0 && g.lz != nullptr; }

using lds_u64 = __attribute__((address_space(3))) const uint64_t;
__device__ __forceinline__ uint64_t lz_word(const uint64_t* lz_lds, size_t idx) {
    // volatile: keeps the loop-invariant rows from being hoisted into
    // registers across the shot loop
    return ((const volatile lds_u64*)lz_lds)[idx];
}
// Parity of popc(Lz[r] & R) for logical row r < g.k.
template <int NW>
__device__ __forceinline__ int lz_row_parity(const DevGraph& g, const uint64_t* lz_lds, int r, const uint64_t (&R)[NW]) {
    const size_t base = (size_t)r * g.lz_words;
    int par = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i)
        if (i < g.lz_words) par += __popcll(lz_word(lz_lds, base + i) & R[i]);
    return par & 1;
}

template <int RC, int NW>
struct ShotIo {
    static constexpr int NS = (64 * RC + 3 + 255) / 256;  // syndrome glds per stage
    static constexpr int NR = (64 * NW + 3 + 255) / 256;  // readout glds per stage
    static constexpr int kStaged = NS + NR;
    // one shot staged ahead: one syndrome and two readout buffers
    static constexpr int kSynBufs = 1, kRdBufs = 2;
    // vmcnt at the loop top (this shot's syndrome landed: its readout loads are
    // younger) and before the readout is read (the next shot's stage is
    // younger); stores and counter atomics in between only make either wait
    // stricter
    static constexpr int kWaitSyn = NR;
    static constexpr int kWaitRd = kStaged;
    __host__ __device__ static size_t bytes(const DevGraph& g) {
        size_t b = 256 * (size_t)(NS * kSynBufs + NR * kRdBufs);
        if (lz_in_lds(g)) b += ((size_t)g.k * g.lz_words * 8 + 15) / 16 * 16;
        return b;
    }
    uint8_t* syn;        // [kSynBufs][NS*256]  staged syndrome rows
    uint8_t* rd;         // [kRdBufs][NR*256]   staged readout rows
    const uint64_t* lz;  // the LDS copy of the logicals (read with lz_word / lz_row_parity)
    // byte offsets of a staged shot's rows inside their buffers; the kernel
    // rotates them with the shot indices (a per-buffer array selected by a
    // loop-carried index would live in scratch)
    struct Shift {
        int s = 0, r = 0;
    };

    __device__ ShotIo(const DevGraph& g, unsigned char* base) {
        syn = base;
        rd = base + 256 * NS * kSynBufs;
        lz = reinterpret_cast<const uint64_t*>(base + 256 * (NS * kSynBufs + NR * kRdBufs));
    }
    __device__ void init(const DevGraph& g, int lane) {
        if (lz_in_lds(g)) {
            uint64_t* l = const_cast<uint64_t*>(lz);
            for (int e = lane; e < g.k * g.lz_words; e += 64) l[e] = g.lz[e];
        }
    }
    // N glds of whole dwords covering row `row` of a [B][len] byte buffer into
    // dst: a uniform base address plus 32-bit lane offsets, clamped to the
    // buffer's last whole dword.
    template <int N>
    __device__ static int stage_row(const uint8_t* buf, int64_t B, int len, int64_t row, uint8_t* dst, int lane,
                                    const uint8_t* dummy) {
        const int64_t total_dw = B * (int64_t)len / 4;  // whole dwords inside the buffer
        if (!buf || len <= 0 || total_dw <= 0) {
#pragma unroll
            for (int c = 0; c < N; ++c) __builtin_amdgcn_global_load_lds(dummy, dst + 256 * c, 4, 0, 0);
            return 0;
        }
        const int64_t start = row * len;
        const int64_t dw0 = start >> 2;
        const uint8_t* base = buf + 4 * dw0;
        int64_t lim64 = total_dw - 1 - dw0;  // last loadable dword, relative (>= 0)
        // lanes past the row re-read the row's last dword (same line, coalesced
        // in the instruction) instead of fetching the following rows' bytes
        const int64_t row_last = ((start + len - 1) >> 2) - dw0;
        lim64 = row_last < lim64 ? row_last : lim64;
        const int lim = lim64 > 0x3fffffff ? 0x3fffffff : (int)lim64;
#pragma unroll
        for (int c = 0; c < N; ++c) {
            const int rel = min(64 * c + lane, lim);
            __builtin_amdgcn_global_load_lds(base + 4 * rel, dst + 256 * c, 4, 0, 0);
        }
        return (int)(start & 3);
    }
    // exactly kStaged LDS-DMA loads: syndrome and readout rows of `shot` (shot 0
    // past B) into syndrome buffer sb and readout buffer rb
    __device__ Shift stage(const DevGraph& g, const DecodeArgs& a, int64_t shot, int sb, int rb, int lane) const {
        if (shot >= a.B) shot = 0;
        const uint8_t* dummy = reinterpret_cast<const uint8_t*>(g.col_idx);
        Shift sh;
        sh.s = stage_row<NS>(a.syn, a.B, g.m, shot, syn_area(sb), lane, dummy);
        sh.r = stage_row<NR>(a.readout, a.B, g.n_data, shot, rd_area(rb), lane, dummy);
        return sh;
    }
    // bytes [total_dw*4, B*len) of the last row (only when B*len % 4 != 0), after the row's wait
    __device__ static void patch_tail(const uint8_t* buf, int64_t B, int len, int64_t row, uint8_t* dst, int shift,
                                      int lane) {
        if (!buf || len <= 0 || row != B - 1) return;
        const int64_t total = B * (int64_t)len, covered = total / 4 * 4;
        const int64_t start = row * len;
        const int64_t q = covered + lane;
        if (q < total && q >= start) dst[shift + (q - start)] = buf[q];
    }
    __device__ uint8_t* syn_area(int sb) const { return syn + 256 * NS * sb; }
    __device__ uint8_t* rd_area(int rb) const { return rd + 256 * NR * rb; }
};

// Waits until at most N of this wave's vector-memory operations (LDS-DMA loads
// included) are outstanding, and orders that before the following LDS reads.
template <int N>
__device__ __forceinline__ void wait_vmem() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
    wave_lds_sync();
}
// Waits for this wave's LDS reads to return (before an LDS-DMA overwrites them).
__device__ __forceinline__ void wait_lds() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// finalize_shot with the readout taken from the LDS staging buffer `rdl`
// (columns w*64 + lane) and the logicals from `lzs` (LDS or global).
__device__ inline void finalize_shot_io(const DevGraph& g, const DecodeArgs& a, int64_t shot, const uint8_t* xh,
                                        bool conv, bool satisfied, int steps, int lane, const uint8_t* rdl,
                                        const uint64_t* lzs) {
    const int n = g.n;
    if (a.x_out)
        for (int j = lane; j < n; j += 64) a.x_out[shot * n + j] = xh[j];
    const bool want_fail = a.fail && a.readout && g.k > 0;
    int lpar[kMaxLogicalRounds] = {0, 0, 0, 0};
    if (a.corr_out || want_fail) {
        for (int w0 = 0; w0 < g.lz_words; ++w0) {
            const int q = w0 * 64 + lane;
            int cb = 0;
            if (q < g.n_data) {
                cb = a.base ? (a.base[shot * g.n_data + q] & 1) : 0;
                for (int t = 0; t < g.fold_blocks; ++t) cb ^= xh[t * g.n_data + q];
                if (a.corr_out) a.corr_out[shot * g.n_data + q] = (uint8_t)cb;
            }
            if (want_fail) {
                const int v = (q < g.n_data) ? ((rdl[q] ^ cb) & 1) : 0;
                const unsigned long long word = __ballot(v);
#pragma unroll
                for (int rr = 0; rr < kMaxLogicalRounds; ++rr) {
                    const int r = rr * 64 + lane;
                    if (r < g.k) lpar[rr] ^= __popcll(lz_word(lzs, (size_t)r * g.lz_words + w0) & word) & 1;
                }
            }
        }
    }
    int any_fail = 0;
    if (want_fail) {
        int f = 0;
#pragma unroll
        for (int rr = 0; rr < kMaxLogicalRounds; ++rr) f |= lpar[rr];
        any_fail = __ballot(f) != 0ull;
    }
    if (lane == 0) {
        if (a.status) a.status[shot] = (uint8_t)((conv ? 1 : 0) | (satisfied ? 2 : 0));
        if (a.ssf_steps) a.ssf_steps[shot] = steps;
        if (a.fail) a.fail[shot] = (uint8_t)any_fail;
    }
}

// Fused failure check from the hard decision held as ballot words
// (X[w] bit l = column 64 w + l), for graphs without a spacetime fold:
// corr = base ^ x, fail = any_r parity(lz_r . (readout ^ corr)).  Readout from
// the LDS staging area, logicals from `lzs`.
template <int NW, bool WITH_BASE>
__device__ inline int fail_from_words(const DevGraph& g, const DecodeArgs& a, int64_t shot, int lane,
                                      const uint64_t (&X)[NW], const uint8_t* rdl, const uint64_t* lzs) {
    uint64_t R[NW];
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        R[w] = 0;
        if (w < g.lz_words) {
            const int q = w * 64 + lane;
            int v = 0;
            if (q < g.n_data) {
                v = (int)rdl[q];
                if (WITH_BASE && a.base) v ^= a.base[shot * g.n_data + q];
            }
            R[w] = __ballot(v & 1) ^ X[w];  // columns >= n_data: lz bits are zero
        }
    }
    int f = 0;
#pragma unroll
    for (int rr = 0; rr < kMaxLogicalRounds; ++rr) {
        const int r = rr * 64 + lane;
        if (r < g.k) {
            f |= lz_row_parity<NW>(g, lzs, r, R);
        }
    }
    return __ballot(f) != 0ull;
}

// ---------------------------------------------------------------- packed SSF queue
// Entry of one non-converged shot (u64 words): shot index, hard decision by
// column (XW words), residual syndrome by check (RW words), readout by column
// (XW words; zero when there is no fused failure check), so the SSF kernel
// never touches the shot's rows in HBM.  Lanes 0..QW-1 store one word each.
template <int XW, int RW>
struct QEntry {
    static constexpr int QW = 1 + 2 * XW + RW;
    static_assert(QW <= 32, "queue entry");
};

template <int XW, int RW>
__device__ inline void queue_push_packed(const DecodeArgs& a, int64_t shot, const uint64_t (&xw)[XW],
                                         const uint64_t (&rw)[RW], const uint64_t (&dw)[XW], int lane) {
    constexpr int QW = QEntry<XW, RW>::QW;
    int slot = 0;
    if (lane == 0) slot = atomicAdd(a.q_count, 1);
    slot = __shfl(slot, 0);
    // uniform words into lanes 0..QW-1: 32-bit selects (two registers in total)
    uint32_t lo = (uint32_t)shot, hi = (uint32_t)((uint64_t)shot >> 32);
#pragma unroll
    for (int w = 0; w < XW; ++w) {
        lo = lane == 1 + w ? (uint32_t)xw[w] : lo;
        hi = lane == 1 + w ? (uint32_t)(xw[w] >> 32) : hi;
        lo = lane == 1 + XW + RW + w ? (uint32_t)dw[w] : lo;
        hi = lane == 1 + XW + RW + w ? (uint32_t)(dw[w] >> 32) : hi;
    }
#pragma unroll
    for (int w = 0; w < RW; ++w) {
        lo = lane == 1 + XW + w ? (uint32_t)rw[w] : lo;
        hi = lane == 1 + XW + w ? (uint32_t)(rw[w] >> 32) : hi;
    }
    if (lane < QW) a.q_w[(int64_t)slot * QW + lane] = ((uint64_t)hi << 32) | lo;
}

}  // namespace qdec
