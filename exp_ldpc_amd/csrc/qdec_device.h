// qdec_device.h -- device helpers shared by the wave kernels (qdec_bp.hip) and
// the workgroup kernels (qdec_bp_block.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "qdec_internal.h"

namespace qdec {

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
// min_d) * 840/d.  Subsets using qubits beyond the generator's weight have zero
// masks and a larger |t| than the same subset without them, so they never
// raise the maximum of a positive score.  nhi = 2^(wmax-4) blocks of 16.
__device__ __forceinline__ int gen_best_score(uint32_t sl, const uint32_t (&qm)[kGenW], int nhi) {
    const int base = __builtin_popcount(sl);
    uint32_t lo[16];
    lo[0] = 0;
#pragma unroll
    for (int l = 1; l < 16; ++l) lo[l] = lo[l & (l - 1)] ^ qm[__builtin_ctz(l)];
    uint32_t mn[kGenW + 1];
#pragma unroll
    for (int d = 0; d <= kGenW; ++d) mn[d] = 64u;
#pragma unroll
    for (int hi = 0; hi < 16; ++hi) {
        if (hi < nhi) {  // uniform
            uint32_t mh = 0;
#pragma unroll
            for (int bb = 0; bb < 4; ++bb)
                if ((hi >> bb) & 1) mh ^= qm[4 + bb];
            const uint32_t sh = sl ^ mh;
#pragma unroll
            for (int l = 0; l < 16; ++l) {
                if (hi == 0 && l == 0) continue;  // empty set
                const int d = __builtin_popcount(hi) + __builtin_popcount(l);
                mn[d] = min(mn[d], (uint32_t)__builtin_popcount(sh ^ lo[l]));
            }
        }
    }
    int best = INT_MIN;
#pragma unroll
    for (int d = 1; d <= kGenW; ++d) best = max(best, (base - (int)mn[d]) * (840 / d));
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

}  // namespace qdec
