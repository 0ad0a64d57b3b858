// qdec_bp_ms.h -- min-sum BP wave kernel with compressed check-node state
// (included by qdec_bp.hip).
//
// Same arithmetic as bp_wave_kernel<T, MIN_SUM> (ldpc v1 min-sum-log, bit-exact
// against the oracle), with less LDS traffic.  The check pass does not scatter
// c2v messages.  It only writes a per-check state (m1, m2, parity); m2's sign
// bit carries the parity.  The variable lane rebuilds each incoming message
// from that state and from the v2c message it sent last iteration, which it
// keeps in registers:
//     c = alpha * ((|v| == m1) ? m2 : m1),  negated iff parity ^ (v <= 0).
// This is the same selection the check pass of bp_wave_kernel makes, on the
// same operands.  Per iteration and wave, the LDS traffic is:
//   check pass  RC x (ds_read_b128 x2 row + ds_write_b64 state)
//   var pass    RV x 4 x (ds_read_b64 state gather + ds_write_b32 v2c scatter)
// The syndrome test needs no LDS at all.  Hard decisions are ballots
// (X[w] = 64 lane slots per word), and check i's parity is
// popc(X & smask_i) mod 2 with per-lane slot masks.  The host (qdec_abi.cpp
// ms_layout) places variables in lane slots by ascending degree, so the
// leading all-degree-3 rounds (D3R) run a 3-edge variable pass.  It also picks
// v2c row positions so each scatter instruction has at most 2-way bank
// conflicts, which ds_write_b32 absorbs for free.  Shot inputs are staged
// through LDS one shot ahead (ShotIo).
#pragma once

namespace qdec {

template <typename T>
struct FBits;
template <>
struct FBits<float> {
    using U = uint32_t;
    __device__ static U to(float x) { return __float_as_uint(x); }
    __device__ static float from(U u) { return __uint_as_float(u); }
};
template <>
struct FBits<double> {
    using U = unsigned long long;
    __device__ static U to(double x) { return (U)__double_as_longlong(x); }
    __device__ static double from(U u) { return __longlong_as_double((long long)u); }
};

// f64 min/max on the VALU without the IEEE canonicalisation of the operands
// (finite, non-NaN inputs only): max(a, |b|), min(a, |b|), min(a, b).
__device__ __forceinline__ double max_abs_f64(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double min_abs_f64(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double min_f64(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

__device__ __forceinline__ double max_f64(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double min_abs2_f64(double a, double b) {
    double r;
    asm("v_min_f64 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double max_abs2_f64(double a, double b) {
    double r;
    asm("v_max_f64 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// Sign-bit tests for f64 messages (LEAN launches only; the others keep the
// compares).  ldpc's sign test `v <= 0` equals v's sign bit for every v but +0.
// The check pass takes its row parity as the XOR of the high dwords (no f64
// compares) and the variable pass flips a message's sign by the sign bit of the
// v2c message it sent.  Both differ from the compares only through zero
// entries, and a zero entry makes the row's m1 zero, so a row with m1 == 0
// (rare; a divergent branch) takes the parity from the compares and gives m2
// (the magnitude its zero entries select) the sign that makes the variable
// side's sign bit test exact: the parity, flipped when the zeros are +0.  A
// row holding both +0 and -0 has m2 = 0, where only the sign of a zero message
// is left open, which changes no `<= 0` test, no magnitude and no hard
// decision (only the sign of an exactly-zero posterior, which LEAN launches do
// not output).
__device__ __forceinline__ uint32_t f64_hi(double x) { return (uint32_t)((unsigned long long)__double_as_longlong(x) >> 32); }
// x with its sign bit XORed with bit 31 of m: one v_bitop3_b32 on the high
// dword (table 0x6c = (src0 & src2) ^ src1)
__device__ __forceinline__ double f64_xor_sign(double x, uint32_t m) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(x);
    const uint32_t hi = __builtin_amdgcn_bitop3_b32(m, (uint32_t)(b >> 32), 0x80000000u, 0x6c);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | (uint32_t)b));
}

// The zero-row fix-up of the sign-bit check pass (a call: its registers stay
// out of the BP loop's allocation).  `row`: the check's v2c row, `par`: its
// syndrome bit, `sp`: its (m1, m2) state slot, written with the sign-bit parity.
// m1's sign becomes the parity by ldpc's compares; m2 (the magnitude the row's
// zero entries select) gets the parity flipped when those zeros are +0, so that
// the variable side's sign-bit test gives parity ^ (v <= 0) for them too.
using lds_f64 = __attribute__((address_space(3))) double;
template <int DRC>
__device__ __noinline__ void ms_zero_row_fix(lds_f64* row, bool par, lds_f64* sp) {
    bool pz = false;
#pragma unroll 1
    for (int j = 0; j < DRC; ++j) {
        const double w = row[j];
        par ^= w <= 0.0;
        pz |= __double_as_longlong(w) == 0ll;  // +0
    }
    const uint32_t hx = par ? 0x80000000u : 0u;
    const uint32_t h2 = pz ? hx ^ 0x80000000u : hx;
    sp[0] = f64_xor_sign(fabs(sp[0]), hx);
    sp[1] = f64_xor_sign(fabs(sp[1]), h2);
}

// (smallest, second smallest) of |v[B]| .. |v[E-1]|, counted with multiplicity
// (ldpc's leave-one-out minima need exactly these two).  Leaves are pairs
// (min, max) or a single value (hi = none); merge(A, B) = (min(A.lo, B.lo),
// min(max(A.lo, B.lo), min(A.hi, B.hi))).
struct Top2 {
    double lo, hi;
    bool has_hi;
};
template <int B, int E>
__device__ __forceinline__ Top2 top2_tree(const double* v) {
    static_assert(E > B, "empty range");
    if constexpr (E - B == 1) {
        return Top2{fabs(v[B]), 0.0, false};
    } else if constexpr (E - B == 2) {
        return Top2{min_abs2_f64(v[B], v[B + 1]), max_abs2_f64(v[B], v[B + 1]), true};
    } else {
        constexpr int M = B + ((E - B) / 2 + 1) / 2 * 2;  // left part: an even count of leaves' values
        const Top2 a = top2_tree<B, M>(v);
        const Top2 b = top2_tree<M, E>(v);
        Top2 r;
        r.lo = min_f64(a.lo, b.lo);
        double h = max_f64(a.lo, b.lo);
        if (a.has_hi && b.has_hi)
            h = min_f64(h, min_f64(a.hi, b.hi));
        else if (a.has_hi)
            h = min_f64(h, a.hi);
        else if (b.has_hi)
            h = min_f64(h, b.hi);
        r.hi = h;
        r.has_hi = true;
        return r;
    }
}

// LDS carve-up (elements of T, then bytes)
template <typename T>
struct MsLds {
    static constexpr int DRS = lds_stride<T, kDR>();
    // v2c rows: the m checks plus one all-Big row (index m) that every pad check
    // lane reads; then the 64 dummy elements pad edges scatter into
    __host__ __device__ static int rows(const DevGraph& g) { return g.m + 1; }
    __host__ __device__ static size_t v2c_elems(int nrows) { return ((size_t)nrows * DRS + 64 + 1) / 2 * 2; }
    __host__ __device__ static size_t state_elems(int m_pad) {
        return ((size_t)2 * (m_pad + 1) * sizeof(T) + 15) / 16 * 16 / sizeof(T);
    }
    __host__ __device__ static size_t core_bytes(const DevGraph& g) {
        return ((v2c_elems(rows(g)) + state_elems(g.m_pad)) * sizeof(T) + (size_t)g.n_pad + 64 + 15) / 16 * 16;
    }
    template <int RC, int RV>
    __host__ __device__ static size_t bytes(const DevGraph& g) {
        return core_bytes(g) + ShotIo<RC, RV>::bytes(g);
    }
};

// alpha_t = 1 - 2^-t (ms_scaling == 0) built from bits on the scalar unit:
// 1 - 2^-t is 1.0 minus 2^(P-t) units in the last place below 1.0 (P = 24 for
// float, 53 for double), and rounds to 1.0 for t > P, exactly as
// (T)(1.0 - ldexp(1.0, -t)) does.
template <typename T>
__device__ __forceinline__ T alpha_bits(int it, double ms_scaling) {
    if (ms_scaling != 0.0) return (T)ms_scaling;
    if constexpr (sizeof(T) == 4) {
        const uint32_t u = 0x3F800000u - (it <= 24 ? (1u << (24 - it)) : 0u);
        return __uint_as_float(u);
    } else {
        const unsigned long long u = 0x3FF0000000000000ull - (it <= 53 ? (1ull << (53 - it)) : 0ull);
        return __longlong_as_double((long long)u);
    }
}

// Shot order of a persistent wave (guided scheduling): the first ~80 % of the
// batch by a static stride (no atomics), the rest handed out in chunks of kChunk
// shots from a counter (a.wave_ctr, zeroed by the launcher), so waves that drew
// cheap shots or sit on a less loaded SIMD take more of the tail.  The counter
// result for the following chunk is requested when a chunk is started and read
// kChunk shots later (its latency hidden by a shot's work).  Every shot < B is
// produced exactly once; indices >= B end the wave's loop.  Without a counter
// the whole sequence is the static stride (no request is ever issued).
struct ShotSeq {
    int64_t t = 0, rounds0 = 0, base = 0, grid = 1, blk = 0;
    int left = 0, kChunk = 4;
    unsigned long long pend = 0;  // lane 0: prefetched chunk id
    unsigned long long* ctr = nullptr;
    bool have = false;
// BP counter chunk (diagnostic define): 8 / 16 trade fewer atomics at low p
// (p = 0.001: 0.51 -> 0.45 / 0.47 ms per 2^18 shots) for coarser tail balance
// at high p (p = 0.1: 7.04 -> 7.08 / 7.50 ms); the sweep's sum is flat at 8
    static constexpr int kBpChunk = 4;
    __device__ ShotSeq(const DecodeArgs& a, int lane)
        : ShotSeq(a.B, a.wave_ctr, blockIdx.x, gridDim.x, lane, kBpChunk) {}
    // `total` items over `nw` persistent waves, this one being wave `wid`
    __device__ ShotSeq(int64_t total, unsigned long long* counter, int64_t wid, int64_t nw, int lane, int chunk = 4) {
        kChunk = chunk;
        grid = nw;
        blk = wid;
        ctr = counter;
        rounds0 = ctr ? (total * 4 / 5) / grid : (total + grid - 1) / grid + 1;
        if (ctr && rounds0 == 0) request(lane);
    }
    __device__ void request(int lane) {
        if (lane == 0) pend = atomicAdd(ctr, 1ull);
        have = true;
    }
    __device__ int64_t next(int lane) {
        if (t < rounds0 || !ctr) {  // no counter: the static stride throughout
            const int64_t s = blk + t * grid;
            if (++t == rounds0 && ctr) request(lane);
            return s;
        }
        if (left == 0) {
            const unsigned long long c = __builtin_amdgcn_readfirstlane((unsigned)pend) |
                                         ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(pend >> 32)) << 32);
            base = rounds0 * grid + (int64_t)c * kChunk;
            left = kChunk;
            request(lane);
        }
        return base + (kChunk - left--);
    }
};

// The per-wave part shared by the min-sum wave kernels: this lane's slot and
// state tables, and BP iterations on the wave's LDS rows.  D3R: leading
// variable rounds whose slots all have degree <= 3.  LEAN: the kernel writes no
// llr (Q is not kept) and may use the sign-bit check pass.
template <typename T, int RC, int RV, int DRC, bool LEAN, int D3R>
struct MsCore {
    static_assert(DRC <= kDR, "compute width exceeds the LDS row");
    static_assert(D3R <= RV, "degree rounds");
    using V2 = __attribute__((ext_vector_type(2))) T;
    static constexpr int DRS = MsLds<T>::DRS;
    // the variable pass runs rounds in pairs (2p, 2p+1) on packed fp32 pairs;
    // an odd last round pairs with itself.  D3P: leading 3-edge rounds, whole pairs.
    static constexpr int NP = (RV + 1) / 2;
    static constexpr int D3P = D3R & ~1;
    static constexpr int PREC = sizeof(T) == 4 ? 1 : 0;
    static constexpr bool SB = sizeof(T) == 8 && LEAN;

    uint32_t etab[RV][kDC];      // v2c element | state index << 16 (edges k < kd(rv))
    V2 L[NP];                    // priors of rounds (2p, 2p+1)
    uint32_t vsl[(RV + 1) / 2];  // columns of this lane's slots, u16 pairs
    int sslot[RC];               // where this lane's checks write their state (host-placed)
    uint64_t smask[RC][RV];      // slots of this lane's checks' columns, per 64-slot word

    __device__ __forceinline__ void load(const DevGraph& g, int lane) {
        const T* prior = reinterpret_cast<const T*>(g.ms_prior[PREC]);
#pragma unroll
        for (int rv = 0; rv < RV; ++rv) {
            const int sl = rv * 64 + lane;
            if (rv % 2 == 0) L[rv / 2].x = L[rv / 2].y = prior[sl];
            else L[rv / 2].y = prior[sl];
#pragma unroll
            for (int k = 0; k < kDC; ++k) etab[rv][k] = (rv < D3P && k == 3) ? 0u : g.ms_etab[PREC][k * g.n_pad + sl];
            if (rv % 2 == 0) vsl[rv / 2] = g.ms_vslot[sl];
            else vsl[rv / 2] |= (uint32_t)g.ms_vslot[sl] << 16;
        }
#pragma unroll
        for (int rc = 0; rc < RC; ++rc) sslot[rc] = g.ms_sslot[PREC][rc * 64 + lane];
#pragma unroll
        for (int rc = 0; rc < RC; ++rc)
#pragma unroll
            for (int w = 0; w < RV; ++w) smask[rc][w] = g.ms_smask[(size_t)w * g.m_pad + rc * 64 + lane];
    }
    __device__ __forceinline__ int col_of(int rv) const { return (int)((vsl[rv / 2] >> (16 * (rv % 2))) & 0xffffu); }

    // one-time LDS init: unused row positions hold Big forever (never the
    // minimum, positive sign), state m_pad is the zero state of pad edges
    __device__ __forceinline__ static void init_lds(const DevGraph& g, T* v2c, T* st, uint8_t* xh, int lane) {
        for (int e = lane; e < (int)MsLds<T>::v2c_elems(MsLds<T>::rows(g)); e += 64) v2c[e] = Big<T>::v;
        for (int e = lane; e < (int)MsLds<T>::state_elems(g.m_pad); e += 64) st[e] = (T)0;
        for (int e = lane; e < g.n_pad + 64; e += 64) xh[e] = 0;
    }

    // initial messages: v2c = prior
    __device__ __forceinline__ void write_priors(T* v2c) const {
#pragma unroll
        for (int rv = 0; rv < RV; ++rv)
#pragma unroll
            for (int k = 0; k < kDC; ++k)
                if (!(rv < D3P && k == 3)) v2c[etab[rv][k] & 0xffff] = (rv % 2 == 0) ? L[rv / 2].x : L[rv / 2].y;
    }

    // BP iterations it, it + 1, .. max_iter on rows holding the priors
    // (write_priors, then a wave_lds_sync).  Returns true when the syndrome is
    // met (`it` = that iteration); X: hard decisions by slot (ballot words),
    // pres: the residual syndrome bit of this lane's checks, Q: posteriors (!LEAN).
    __device__ __forceinline__ bool iterate(const DecodeArgs& a, T* v2c, T* st, int m, int lane, const bool (&sbit)[RC],
                                            T (&Q)[RV], uint64_t (&X)[RV], bool (&pres)[RC], int& it) const {
        V2 vp[NP][kDC];  // v2c messages this lane sent last iteration, round pairs
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
            for (int k = 0; k < kDC; ++k) vp[p][k] = L[p];
        for (; it <= a.max_iter; ++it) {
            const T alpha = alpha_bits<T>(it, a.ms_scaling);
            // ---- check pass: state (m1, m2) with the parity in both signs ----
            uint32_t zrows = 0;  // rows holding a zero entry (sign-bit parity inexact)
#pragma unroll
            for (int rc = 0; rc < RC; ++rc) {
                const int i = min(rc * 64 + lane, m);  // pad check lanes share the Big row m
                T v[kDR];
                // odd f64 rows load only their DRC slots (r03i A/B: -0.5% BP kernel time)
                if constexpr (sizeof(T) == 8 && DRC % 2 == 1) lds_load_first<T, DRC>(v2c + i * DRS, v);
                else lds_load<T, kDR>(v2c + i * DRS, v);
                T m1 = Big<T>::v, m2 = Big<T>::v;
                bool par = sbit[rc];
                if constexpr (sizeof(T) == 4) {
#pragma unroll
                    for (int k = 0; k < DRC; ++k) {
                        const T av = fabs(v[k]);
                        m2 = med3(av, m1, m2);
                        m1 = med3(av, m1, -Big<T>::v);  // true median = min(|v|, m1): one VALU, abs modifier
                    }
                } else {
                    // f64: (minimum, second minimum) of |v| by a merge tree instead of a
                    // sequential chain (17 instead of 21 f64 ops for 7 values, depth 5
                    // instead of 14); the same two values, so bit-identical
                    const Top2 t = top2_tree<0, DRC>(v);
                    m1 = t.lo;
                    m2 = t.hi;
                }
                V2 s2;
                if constexpr (SB) {
                    // sign-canonical row: the parity is the XOR of the sign bits
                    uint32_t hx = par ? 0x80000000u : 0u;
                    int k = 0;
#pragma unroll
                    for (; k + 1 < DRC; k += 2) hx = __builtin_amdgcn_bitop3_b32(hx, f64_hi(v[k]), f64_hi(v[k + 1]), 0x96);
                    if (k < DRC) hx ^= f64_hi(v[k]);
                    // m1, m2 >= +0: the XOR of the parity bit sets their sign bit
                    s2.x = f64_xor_sign(m1, hx);
                    s2.y = f64_xor_sign(m2, hx);
                    if (m1 == (T)0) zrows |= 1u << rc;  // a zero entry: fixed below
                } else {
#pragma unroll
                    for (int k = 0; k < DRC; ++k)
                        par ^= v[k] <= (T)0;  // ldpc: bit_to_check <= 0 flips the sign (s_xor of compare masks)
                    // both minima carry the parity in their sign bit (they are >= +0)
                    s2.x = par ? -m1 : m1;
                    s2.y = par ? -m2 : m2;
                }
                *reinterpret_cast<V2*>(st + 2 * sslot[rc]) = s2;
            }
            if constexpr (SB) {
                if (__ballot(zrows != 0u)) {  // rare (wave-uniform): rows with a zero entry, parity by the compares
                    asm volatile("" ::: "memory");  // re-read the row and the state just written
#pragma unroll
                    for (int rc = 0; rc < RC; ++rc)
                        if ((zrows >> rc) & 1u)
                            ms_zero_row_fix<DRC>((lds_f64*)(v2c + min(rc * 64 + lane, m) * DRS), sbit[rc],
                                                 (lds_f64*)(st + 2 * sslot[rc]));
                }
            }
            wave_lds_sync();

            // ---- variable pass, rounds in pairs (the next pair's states are
            // gathered while this pair sums) ----
            auto gather = [&](int p, V2 (&sa)[kDC], V2 (&sb)[kDC]) {
                const int r0 = 2 * p, r1 = 2 * p + 1 < RV ? 2 * p + 1 : 2 * p;
#pragma unroll
                for (int k = 0; k < kDC; ++k)
                    if (!(r1 < D3P && k == 3)) {
                        sa[k] = *reinterpret_cast<const V2*>(st + 2 * (etab[r0][k] >> 16));
                        if (r1 != r0) sb[k] = *reinterpret_cast<const V2*>(st + 2 * (etab[r1][k] >> 16));
                    }
            };
            V2 sa[kDC], sb[kDC];
            gather(0, sa, sb);
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                const int r0 = 2 * p, r1 = 2 * p + 1 < RV ? 2 * p + 1 : 2 * p;
                const int KD = r1 < D3P ? 3 : kDC;
                // |c| = alpha * ((|v| == m1) ? m2 : m1), sign = parity ^ (v <= 0);
                // the state's signs carry the parity, so one select picks both
                V2 y[kDC];
#pragma unroll
                for (int k = 0; k < kDC; ++k) {
                    if (k < KD) {
                        y[k].x = (fabs(vp[p][k].x) == fabs(sa[k].x)) ? sa[k].y : sa[k].x;
                        const V2 sbk = r1 != r0 ? sb[k] : sa[k];
                        y[k].y = (fabs(vp[p][k].y) == fabs(sbk.x)) ? sbk.y : sbk.x;
                    }
                }
                if (p + 1 < NP) gather(p + 1 < NP ? p + 1 : p, sa, sb);
                V2 c[kDC];
#pragma unroll
                for (int k = 0; k < kDC; ++k) {
                    if (k < KD) {
                        const V2 yk = y[k] * alpha;
                        if constexpr (SB) {
                            c[k].x = f64_xor_sign(yk.x, f64_hi(vp[p][k].x));
                            c[k].y = f64_xor_sign(yk.y, f64_hi(vp[p][k].y));
                        } else {
                            c[k].x = (vp[p][k].x <= (T)0) ? -yk.x : yk.x;
                            c[k].y = (vp[p][k].y <= (T)0) ? -yk.y : yk.y;
                        }
                    }
                }
                V2 pre[kDC];
                V2 acc = L[p];
#pragma unroll
                for (int k = 0; k < kDC; ++k) {
                    if (k < KD) {
                        pre[k] = acc;
                        acc += c[k];
                    }
                }
                if constexpr (!LEAN) {
                    Q[r0] = acc.x;
                    Q[r1] = acc.y;
                }
                X[r0] = __ballot(acc.x <= (T)0);
                if (r1 != r0) X[r1] = __ballot(acc.y <= (T)0);
                // ldpc: out_k = pre_k + (sum of the later c); the last one adds an
                // empty sum (+0), which can only turn -0 into +0: both are <= 0 and
                // have |v| = 0, so the message is used identically either way
                V2 suf;
#pragma unroll
                for (int k = kDC - 1; k >= 0; --k) {
                    if (k < KD) {
                        const V2 out = (k == KD - 1) ? pre[k] : pre[k] + suf;
                        suf = (k == KD - 1) ? c[k] : suf + c[k];
                        vp[p][k] = out;
                        v2c[etab[r0][k] & 0xffff] = out.x;  // pads -> dummy element
                        if (r1 != r0) v2c[etab[r1][k] & 0xffff] = out.y;
                    }
                }
            }

            // ---- syndrome test (registers only) ----
            int bad = 0;
#pragma unroll
            for (int rc = 0; rc < RC; ++rc) {
                pres[rc] = sbit[rc] != (masked_parity<RV>(smask[rc], X) != 0);
                bad |= pres[rc];
            }
            wave_lds_sync();  // v2c scatter complete before the next check pass
            if (__ballot(bad) == 0ull) return true;
        }
        return false;
    }
};

// LEAN: the throughput configuration (no x / corr / llr outputs, no base, no
// syndrome flags, no spacetime fold): the per-shot epilogue is the ballot-word
// failure check only, which keeps the kernel's scalar state small.
// D3R: leading variable rounds whose slots all have degree <= 3.
// f64: launched at 2 waves per SIMD (launch_bp_wave caps the grid; measured
// faster than 3), so the register budget is 256; f32: 4 waves (<= 128 VGPRs).
// OCC: waves per SIMD the registers are budgeted for (0 = the default above).
// The f64 LEAN kernel also comes as OCC = 3 (<= 168 VGPRs, a few dwords of the
// per-shot epilogue spilled), launched when a handle asks for more than 8 f64
// waves per CU (qd_graph_set_wave_occupancy: the bench's concurrent points).
template <typename T, int RC, int RV, int DRC, bool DEFER, bool LEAN, int D3R, int OCC = 0>
__global__ __launch_bounds__(64, OCC > 0 ? OCC : (sizeof(T) == 4 ? 4 : 2)) void bp_ms_wave_kernel(DevGraph g, DecodeArgs a) {
    using Io = ShotIo<RC, RV>;
    using Core = MsCore<T, RC, RV, DRC, LEAN, D3R>;
    constexpr int PREC = Core::PREC;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T* v2c = reinterpret_cast<T*>(smem);
    T* st = v2c + MsLds<T>::v2c_elems(MsLds<T>::rows(g));
    uint8_t* xh = reinterpret_cast<uint8_t*>(st + MsLds<T>::state_elems(g.m_pad));
    Io io(g, smem + MsLds<T>::core_bytes(g));

    const int lane = threadIdx.x;
    const int m = g.m, n = g.n;
    Core core;
    core.load(g, lane);
    // zero syndrome + every prior > 0: iteration 1 converges with x = 0 (all
    // messages are >= 0, so every posterior is >= its prior > 0), and the LEAN
    // outputs (iterations 1, converged, failure from the readout alone) need
    // nothing else
    const bool zero_ok = LEAN && ((g.ms_allpos >> PREC) & 1);

    Core::init_lds(g, v2c, st, xh, lane);
    io.init(g, lane);
    ShotSeq seq(a, lane);
    int64_t shot = seq.next(lane);
    typename Io::Shift sh = io.stage(g, a, shot, 0, 0, lane);  // row offsets of `shot`'s stage
    int64_t nxt = seq.next(lane);
    wave_lds_sync();

    int sb = 0, buf = 0;  // syndrome / readout staging buffers of `shot`
    QDEC_STAMP_DECL
#ifdef QDEC_STAMPS
    const unsigned long long qdec_t0 = __builtin_amdgcn_s_memtime(), qdec_r0 = __builtin_amdgcn_s_memrealtime();
#endif
    for (; shot < a.B;) {
        // ---- syndrome (staged one shot ahead: at least the NR readout loads of
        // the same stage are younger); then stage the next shot ----
        QDEC_STAMP(5);
        wait_vmem<Io::kWaitSyn>();
        Io::patch_tail(a.syn, a.B, m, shot, io.syn_area(sb), sh.s, lane);
        wave_lds_sync();
        QDEC_STAMP(0);
        bool sbit[RC];  // lane masks: parity work stays on the scalar unit
        const uint8_t* srow = io.syn_area(sb) + sh.s;
#pragma unroll
        for (int rc = 0; rc < RC; ++rc) {
            const int i = rc * 64 + lane;
            sbit[rc] = (i < m && a.syn) ? (srow[i] & 1) != 0 : false;
        }
        wait_lds();
        const int64_t nn = seq.next(lane);  // any counter request is older than the stage
        const typename Io::Shift shn = io.stage(g, a, nxt, 0, buf ^ 1, lane);
        if (!LEAN && a.syn_flags) {
            const bool use_b = (a.syn_flags & 1) && a.base;
            const bool use_r = (a.syn_flags & 2) && a.readout;
            uint64_t Xf[RV];
#pragma unroll
            for (int w = 0; w < RV; ++w) {
                const int q = core.col_of(w);
                int v = 0;
                if (q < g.n_data) {
                    if (use_b) v ^= a.base[shot * g.n_data + q];
                    if (use_r) v ^= a.readout[shot * g.n_data + q];
                }
                Xf[w] = __ballot(v & 1);
            }
#pragma unroll
            for (int rc = 0; rc < RC; ++rc) {
                uint64_t acc = 0;
#pragma unroll
                for (int w = 0; w < RV; ++w) acc ^= core.smask[rc][w] & Xf[w];
                sbit[rc] ^= (__popcll(acc) & 1) != 0;
            }
        }

        // ---- initial messages: v2c = prior, unless the shot is skipped ----
        bool skip = false;
        if (zero_ok) {
            bool any = false;
#pragma unroll
            for (int rc = 0; rc < RC; ++rc) any |= sbit[rc];
            skip = __ballot(any) == 0ull;
        }
        if (!skip) core.write_priors(v2c);
        wave_lds_sync();

        QDEC_STAMP(1);
        T Q[RV];
        uint64_t X[RV];
        bool pres[RC];
        int it = 1;
        bool conv = false;
        if (skip) {
            conv = true;
#pragma unroll
            for (int rv = 0; rv < RV; ++rv) X[rv] = 0ull;
#pragma unroll
            for (int rc = 0; rc < RC; ++rc) pres[rc] = false;
        }
        if (!skip) conv = core.iterate(a, v2c, st, m, lane, sbit, Q, X, pres, it);
        const int iters = conv ? it : a.max_iter;
        QDEC_STAMP(2);
        QDEC_COUNT(8, iters);
        QDEC_COUNT(9, 1);
        // this shot's readout: wait before any store of this shot, so the
        // kWaitRd most recent vector-memory operations are the later shots' stages
        const bool need_rd = a.readout && a.fail && g.k > 0;  // the SSF queue carries it too
        if (need_rd) {
            wait_vmem<Io::kWaitRd>();
            Io::patch_tail(a.readout, a.B, g.n_data, shot, io.rd_area(buf), sh.r, lane);
        }
        if (lane == 0 && a.iters) a.iters[shot] = iters;
        // hard decision by column (slot order -> xh[column])
#pragma unroll
        for (int rv = 0; rv < RV; ++rv) xh[core.col_of(rv)] = (uint8_t)((X[rv] >> lane) & 1);
        if (!LEAN && a.llr_out) {
            T* lo = reinterpret_cast<T*>(a.llr_out);
#pragma unroll
            for (int rv = 0; rv < RV; ++rv) {
                const int j = core.col_of(rv);
                if (j < n) lo[shot * n + j] = Q[rv];
            }
        }
        wave_lds_sync();
        QDEC_STAMP(3);
        if (DEFER && !conv) {
            if (LEAN || a.q_packed) {  // LEAN launches always use the packed queue
                uint64_t xw[RV], rw[RC], dw[RV];
                const uint8_t* rrow = io.rd_area(buf) + sh.r;
#pragma unroll
                for (int w = 0; w < RV; ++w) {
                    const int q = w * 64 + lane;
                    xw[w] = __ballot(xh[q] & 1);
                    dw[w] = need_rd ? __ballot(q < g.n_data && (rrow[q] & 1)) : 0ull;
                }
#pragma unroll
                for (int rc = 0; rc < RC; ++rc) rw[rc] = __ballot(pres[rc]);
                queue_push_packed<RV, RC>(a, shot, xw, rw, dw, lane);
            } else {
                int slot = 0;
                if (lane == 0) slot = atomicAdd(a.q_count, 1);
                slot = __shfl(slot, 0);
                for (int j = lane; j < n; j += 64) a.q_x[(int64_t)slot * n + j] = xh[j];
#pragma unroll
                for (int rc = 0; rc < RC; ++rc) {
                    const int i = rc * 64 + lane;
                    if (i < m) a.q_r[(int64_t)slot * m + i] = (uint8_t)pres[rc];
                }
                if (lane == 0) a.q_idx[slot] = shot;
            }
        } else if (LEAN || (g.fold_blocks == 1 && !a.corr_out)) {
            if (!LEAN && a.x_out)
                for (int j = lane; j < n; j += 64) a.x_out[shot * n + j] = xh[j];
            int any_fail = 0;
            if (a.fail && a.readout && g.k > 0) {
                uint64_t Xc[RV];  // hard decision by column
#pragma unroll
                for (int w = 0; w < RV; ++w) Xc[w] = __ballot(xh[w * 64 + lane] & 1);
                any_fail = fail_from_words<RV, !LEAN>(g, a, shot, lane, Xc, io.rd_area(buf) + sh.r, io.lz);
            }
            if (lane == 0) {
                if (a.status) a.status[shot] = (uint8_t)(conv ? 3 : 0);
                if (a.ssf_steps) a.ssf_steps[shot] = 0;
                if (a.fail) a.fail[shot] = (uint8_t)any_fail;
            }
        } else {
            finalize_shot_io(g, a, shot, xh, conv, conv, 0, lane, io.rd_area(buf) + sh.r, io.lz);
        }
        wave_lds_sync();
        QDEC_STAMP(4);
        shot = nxt;
        nxt = nn;
        sh = shn;
        buf ^= 1;
    }
#ifdef QDEC_STAMPS
    QDEC_COUNT(10, __builtin_amdgcn_s_memtime() - qdec_t0);
    QDEC_COUNT(11, __builtin_amdgcn_s_memrealtime() - qdec_r0);
    QDEC_COUNT(12, 1);
#endif
    QDEC_FLUSH_AT(0);
}

// ---------------------------------------------------------------- compact shot list
// Lean min-sum launches on wave graphs run in two passes.  ms_triage_kernel
// streams every shot's syndrome and readout rows once (coalesced tiles of 64
// shots), packs the syndrome into bit words and reduces the readout to its
// logical parities (bit r = parity of Lz[r] . readout).  A shot with an
// all-zero syndrome under all-positive priors converges in iteration 1 with
// x = 0 (every message >= 0, so every posterior >= its prior > 0: the same
// shortcut the one-pass kernel takes), so its outputs are written right there
// (iterations 1, status 3, no SSF steps, failure = any readout parity).  Every
// other shot is appended to a compact list: shot index, syndrome words,
// readout-parity words.  bp_ms_cmp_kernel then decodes only the listed shots,
// reading each as one entry from registers (no row staging, no readout): its
// failure check is the parity of Lz (in lane-slot order, ms_lzs) against the
// ballot words of the hard decision, XOR the readout parities, and a
// BP-failed shot enters the SSF queue with the parities in place of the
// readout words (q_rpar), which the SSF kernel's check uses the same way.
template <int RC>
struct CmpEntry {
    static constexpr int EW = 1 + RC + kMaxLogicalRounds;  // shot, syndrome words, readout-parity words
    static constexpr int kPer = 4;                          // entries per chunk (one u64 load per lane)
    static_assert(kPer * EW <= 64, "chunk");
};

// bits 24..27 of (d & 0x01010101) * 0x01020408 are bit 0 of d's four bytes
__device__ __forceinline__ uint32_t byte_bits4(uint32_t d) { return ((d & 0x01010101u) * 0x01020408u) >> 24; }

// One tile of a shot-major byte buffer, as the 16-B chunks covering bytes
// [start, start + len) of a buffer of `total` bytes (image chunk 0 = the chunk
// at or below `start`; `shift` = the byte offset of `start` inside the image).
// The LDS image keeps only bit 0 of every byte (16 bits per chunk, 1/8 of the
// bytes), so a tile pair needs ~3 KB of LDS instead of ~21 KB and more tiles
// are in flight per CU.
using u32x4 = __attribute__((ext_vector_type(4))) uint32_t;
// bit 0 of 16 bytes as a 16-bit word (byte t -> bit t)
__device__ __forceinline__ uint32_t chunk_bits16(u32x4 v) {
    return byte_bits4(v.x) | (byte_bits4(v.y) << 4) | (byte_bits4(v.z) << 8) | (byte_bits4(v.w) << 12);
}
struct TileSrc {
    const uint8_t* buf;
    int64_t total, c0;  // c0: first 16-B chunk
    int nch, shift;
    void* img;          // u16 bits per chunk
    __device__ TileSrc(const uint8_t* b, int64_t tot, int64_t start, int64_t len, void* dst) : buf(b), total(tot), img(dst) {
        c0 = start >> 4;
        nch = (int)(((start + len + 15) >> 4) - c0);
        shift = (int)(start & 15);
    }
    __device__ __forceinline__ void put(int c, u32x4 v) const { static_cast<uint16_t*>(img)[c] = (uint16_t)chunk_bits16(v); }
    // chunk c of the image from its bytes (the buffer's last partial chunk)
    __device__ u32x4 bytes(int c) const {
        uint32_t w[4] = {0u, 0u, 0u, 0u};
        for (int t = 0; t < 16; ++t) {
            const int64_t q = 16 * (c0 + c) + t;
            if (q < total) w[t / 4] |= (uint32_t)buf[q] << (8 * (t % 4));
        }
        return u32x4{w[0], w[1], w[2], w[3]};
    }
};

// Copy a tile into its LDS image: U 16-B loads per lane per round (64 U
// chunks), all issued before any LDS store.  Every load is unconditional, from
// a chunk index clamped into the buffer's whole 16-B chunks (no exec-masked
// loads, so the compiler keeps them all in flight); chunks past the buffer's
// last whole 16 B are assembled from byte loads.  The buffer must be 16-B
// aligned (the launcher checks; torch allocations are).
template <int U>
__device__ __forceinline__ void tile_to_lds(const TileSrc& T, int lane) {
    const int64_t whole = T.total >> 4;
    const u32x4* src = reinterpret_cast<const u32x4*>(T.buf);
    for (int r0 = 0; r0 < T.nch; r0 += 64 * U) {
        u32x4 v[U];
        if (whole > 0) {  // uniform
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t gi = min(T.c0 + r0 + u * 64 + lane, whole - 1);
                v[u] = __builtin_nontemporal_load(src + gi);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int c = r0 + u * 64 + lane;
            if (c < T.nch) T.put(c, T.c0 + c < whole ? v[u] : T.bytes(c));
        }
    }
}

// Two tiles (syndrome and readout) into their LDS images with every load of a
// round issued before any LDS store, so the second tile's HBM latency overlaps
// the first's: UA / UB 16-B loads per lane per round (the bench shape does
// both tiles in one round).  Same clamping and tail handling as tile_to_lds.
template <int UA, int UB>
__device__ __forceinline__ void tile_pair_to_lds(const TileSrc& A, const TileSrc& B, int lane) {
    const int64_t wa = A.total >> 4, wb = B.total >> 4;
    const u32x4* sa = reinterpret_cast<const u32x4*>(A.buf);
    const u32x4* sb = reinterpret_cast<const u32x4*>(B.buf);
    for (int ra = 0, rb = 0; ra < A.nch || rb < B.nch; ra += 64 * UA, rb += 64 * UB) {
        u32x4 va[UA], vb[UB];
        if (wa > 0 && ra < A.nch) {  // uniform
#pragma unroll
            for (int u = 0; u < UA; ++u) va[u] = __builtin_nontemporal_load(sa + min(A.c0 + ra + u * 64 + lane, wa - 1));
        }
        if (wb > 0 && rb < B.nch) {  // uniform
#pragma unroll
            for (int u = 0; u < UB; ++u) vb[u] = __builtin_nontemporal_load(sb + min(B.c0 + rb + u * 64 + lane, wb - 1));
        }
#pragma unroll
        for (int u = 0; u < UA; ++u) {
            const int c = ra + u * 64 + lane;
            if (c < A.nch) A.put(c, A.c0 + c < wa ? va[u] : A.bytes(c));
        }
#pragma unroll
        for (int u = 0; u < UB; ++u) {
            const int c = rb + u * 64 + lane;
            if (c < B.nch) B.put(c, B.c0 + c < wb ? vb[u] : B.bytes(c));
        }
    }
}

// Iteration 1 in the triage (DecodeArgs::it1_lut), bit-sliced over the tile's
// 64 shots: the syndrome is transposed to one word per check (bit s = shot s),
// each column's decision word is its 16-bit table (it1_tables, qdec_abi.cpp)
// applied to its <= 4 checks' words, and a shot whose decision meets its
// syndrome has converged in iteration 1 -- the BP kernel would report exactly
// that (iterations 1, status 3, failure = parity of Lz x against the readout).
// LDS (over the tile images, dead by then): check words [RC*64 + 1] (the last
// one zero: pad check id), decision words [RV*64 + 1] (the last zero: pad
// column id), logical parities [256].
template <int RC, int RV>
struct TriageIt1 {
    static constexpr size_t bytes = 8 * (size_t)(RC * 64 + 1 + RV * 64 + 1 + 64 * kMaxLogicalRounds) + 16;
};

constexpr int kHeavyW = 6;  // listed shots of larger syndrome weight go to the heavy list
constexpr int kT1GateW = 12;  // iteration-1 tile gate: syndrome weight bound ...
constexpr int kT1GateN = 8;   // ... and shots of the tile within it
constexpr int kTriageUB = 16;  // readout-tile loads per lane per round
// 64 x 64 bit transpose across the wave: lane r holds row r (bit c = entry
// (r, c)), and gets back column r (bit c = entry (c, r)).  Six block-swap
// stages, each one exchange with lane ^ j: the off-diagonal j x j blocks of
// every 2j x 2j block trade places.
__device__ __forceinline__ uint64_t wave_transpose64(uint64_t v, int lane) {
    const uint64_t keep[6] = {0x00000000FFFFFFFFull, 0x0000FFFF0000FFFFull, 0x00FF00FF00FF00FFull,
                              0x0F0F0F0F0F0F0F0Full, 0x3333333333333333ull, 0x5555555555555555ull};
#pragma unroll
    for (int st = 0; st < 6; ++st) {
        const int j = 32 >> st;
        const uint64_t k0 = keep[st];  // columns c with (c & j) == 0
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, j);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), j);
        const uint64_t w = ((uint64_t)hi << 32) | lo;
        v = (lane & j) ? ((v & ~k0) | ((w >> j) & k0)) : ((v & k0) | ((w & k0) << j));
    }
    return v;
}

// f(w0..w3) of a 16-entry truth table, bit-sliced: OR over the patterns p with
// table bit p of the minterm (w_k or ~w_k by bit k of p)
__device__ __forceinline__ uint64_t lut4_words(uint32_t lut, uint64_t w0, uint64_t w1, uint64_t w2, uint64_t w3) {
    const uint64_t A[4] = {~w0 & ~w1, w0 & ~w1, ~w0 & w1, w0 & w1};
    const uint64_t C[4] = {~w2 & ~w3, w2 & ~w3, ~w2 & w3, w2 & w3};
    uint64_t f = 0ull;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        uint64_t gsel = 0ull;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            // all-ones / zero from table bit q + 4r
            const int64_t msk = -(int64_t)((lut >> (q + 4 * r)) & 1u);
            gsel |= A[q] & (uint64_t)msk;
        }
        f |= gsel & C[r];
    }
    return f;
}

// The same from a bit image: bit `off` onwards, `len` bits;
// reads up to three dwords past the row's last bit (the image has spares).
template <int NW>
__device__ __forceinline__ void row_bits_b(const uint32_t* img, int off, int len, uint64_t (&w)[NW]) {
    const int q = off >> 5;
    const uint32_t sh = (uint32_t)(off & 31);
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        w[i] = 0ull;
        if (64 * i < len) {  // uniform
            const uint32_t d0 = img[q + 2 * i], d1 = img[q + 2 * i + 1], d2 = img[q + 2 * i + 2];
            uint64_t v = (uint64_t)__builtin_amdgcn_alignbit(d1, d0, sh) |
                         ((uint64_t)__builtin_amdgcn_alignbit(d2, d1, sh) << 32);
            if (64 * i + 64 > len) v &= (1ull << (len - 64 * i)) - 1ull;
            w[i] = v;
        }
    }
}

// LDS bytes of a triage tile image of `len` bytes (plus the spares the row
// readers run past its end)
__host__ __device__ inline size_t triage_img_bytes(int64_t len) {
    const int64_t nch = (len + 15) / 16 + 2;
    return (size_t)((2 * (nch + 8) + 15) / 16 * 16);
}

// One wave per tile of 64 shots (lane l = shot 64 * blockIdx.x + l).  PK:
// bit-packed input rows (QD_INPUT_PACKED; a.in_packed), read as u64 words, no
// tile images (its own instantiation: the byte path's 16-B tile loads keep ~100
// VGPRs in flight, which the packed path does not need).
template <int RC, int NWD, bool PK = false>
__global__ __launch_bounds__(64, 1) void ms_triage_kernel(DevGraph g, DecodeArgs a) {
    using Ent = CmpEntry<RC>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x;
    const int m = g.m, nd = g.n_data;
    const int64_t s0 = (int64_t)blockIdx.x * 64;
    const int ns = (int)min((int64_t)64, a.B - s0);
    const bool want_fail = a.fail && a.readout && g.k > 0;
    // the launch's counters that run behind this pass (compact-kernel chunk
    // counter, SSF slot counter, SSF queue length) are zeroed here, saving a
    // memset launch each (the previous decode on the handle has finished with
    // them: the workspace chain orders decodes)
    if (blockIdx.x == 0 && lane == 0) {
        if (a.wave_ctr) a.wave_ctr[0] = a.wave_ctr[1] = 0ull;
        if (a.q_count) *a.q_count = 0;
    }
    // the handle's other list-counter set, for its next two-pass decode (the
    // decode that last used it has finished: the workspace chain orders them)
    if (blockIdx.x == 0 && a.cmp_count_next)
        for (int s = lane; s < kCmpLists * kCmpSegs; s += 64) a.cmp_count_next[16 * s] = 0ull;
    // LDS: the logicals (k x lz_words u64, read as broadcasts), then the
    // syndrome and readout tiles as 16-B chunk images (one spare chunk each:
    // row_bits reads one dword past a row)
    uint64_t* lz_lds = reinterpret_cast<uint64_t*>(smem);
    const int nlz = want_fail ? g.k * g.lz_words : 0;
    constexpr bool pk = PK;  // bit-packed input rows: no tile images
    unsigned char* syn_img = smem + ((size_t)nlz * 8 + 15) / 16 * 16;
    unsigned char* rd_img = syn_img + (pk ? 0 : triage_img_bytes(64 * (int64_t)m));
    // iteration-1 words: past the images
    unsigned char* it1_base = rd_img + (pk ? 0 : triage_img_bytes(64 * (int64_t)nd));
    for (int e = lane; e < nlz; e += 64) lz_lds[e] = g.lz[e];
    // iteration-1 tables (TriageIt1), loaded ahead of the tiles
    uint64_t it_ids[NWD], it_cv[RC][2];
    uint32_t it_lut[NWD];
    if (a.it1_lut) {
#pragma unroll
        for (int rv = 0; rv < NWD; ++rv) {
            it_ids[rv] = g.it1_vchk[rv * 64 + lane];
            it_lut[rv] = a.it1_lut[rv * 64 + lane];
        }
#pragma unroll
        for (int rc = 0; rc < RC; ++rc) {
            it_cv[rc][0] = g.it1_cvar[2 * (rc * 64 + lane)];
            it_cv[rc][1] = g.it1_cvar[2 * (rc * 64 + lane) + 1];
        }
    }
    const bool live = lane < ns;
    const int64_t shot = s0 + lane;
    uint64_t sw[RC];
    uint64_t rw[NWD];
    if constexpr (PK) {
        // one row of u64 words per shot (RC = ceil(m / 64), NWD = ceil(n_data / 64)
        // on wave graphs): lane-strided loads, padding bits cleared
        const uint64_t* sp = reinterpret_cast<const uint64_t*>(a.syn) + min(shot, a.B - 1) * RC;
#pragma unroll
        for (int rc = 0; rc < RC; ++rc) {
            uint64_t v = __builtin_nontemporal_load(sp + rc);
            if (64 * rc + 64 > m) v &= (m - 64 * rc >= 64) ? ~0ull : ((1ull << (m - 64 * rc)) - 1ull);
            sw[rc] = live ? v : 0ull;
        }
        if (want_fail) {
            const int rdw = (nd + 63) / 64;
            const uint64_t* rq = reinterpret_cast<const uint64_t*>(a.readout) + min(shot, a.B - 1) * rdw;
#pragma unroll
            for (int w = 0; w < NWD; ++w) {
                uint64_t v = w < rdw ? __builtin_nontemporal_load(rq + w) : 0ull;
                if (64 * w + 64 > nd) v &= (nd - 64 * w >= 64) ? ~0ull : (nd > 64 * w ? (1ull << (nd - 64 * w)) - 1ull : 0ull);
                rw[w] = v;
            }
        }
        __syncthreads();  // the logicals' LDS copy (above) before its reads
    } else {
        const TileSrc ts(a.syn, a.B * (int64_t)m, s0 * m, (int64_t)ns * m, syn_img);
        const TileSrc tr(want_fail ? a.readout : a.syn, want_fail ? a.B * (int64_t)nd : 0, s0 * nd,
                         want_fail ? (int64_t)ns * nd : 0, rd_img);
        if (want_fail)
            tile_pair_to_lds<(4 * RC < 8 ? 4 * RC : 8), (4 * NWD < kTriageUB ? 4 * NWD : kTriageUB)>(ts, tr, lane);
        else tile_to_lds<8>(ts, lane);
        __syncthreads();
        row_bits_b<RC>(reinterpret_cast<const uint32_t*>(syn_img), ts.shift + lane * m, m, sw);
        if (want_fail) row_bits_b<NWD>(reinterpret_cast<const uint32_t*>(rd_img), tr.shift + lane * nd, nd, rw);
    }
    uint64_t rp[kMaxLogicalRounds] = {0ull, 0ull, 0ull, 0ull};
    if (want_fail) {
        for (int r = 0; r < g.k; ++r) {  // uniform rows of the dense logical table (LDS broadcasts)
            int par = 0;
#pragma unroll
            for (int w = 0; w < NWD; ++w)
                if (w < g.lz_words) par += __popcll(lz_word(lz_lds, (size_t)r * g.lz_words + w) & rw[w]);
#pragma unroll
            for (int rr = 0; rr < kMaxLogicalRounds; ++rr)
                if (rr == (r >> 6)) rp[rr] |= (uint64_t)(par & 1) << (r & 63);
        }
    }
    bool trivial;
    uint8_t fbit;
    // iteration 1 pays only where shots converge in it: tiles with >= 8 shots of
    // syndrome weight <= 12 (about three isolated errors); others just list
    int wt = 0;
#pragma unroll
    for (int rc = 0; rc < RC; ++rc) wt += __popcll(sw[rc]);
    const bool it1 = a.it1_lut && __popcll(__ballot(live && wt <= kT1GateW)) >= kT1GateN;
    if (it1) {  // uniform: iteration 1 here (TriageIt1)
        wave_lds_sync();
        uint64_t* synT = reinterpret_cast<uint64_t*>(it1_base);
        uint64_t* xT = synT + RC * 64 + 1;
        uint64_t* lzp = xT + NWD * 64 + 1;
        // transpose: lane t gets the word of check rc * 64 + t
#pragma unroll
        for (int rc = 0; rc < RC; ++rc) {
            const uint64_t mine = wave_transpose64(live ? sw[rc] : 0ull, lane);
            synT[rc * 64 + lane] = mine;  // checks >= m: zero words
        }
        if (lane == 0) {
            synT[RC * 64] = 0ull;
            xT[NWD * 64] = 0ull;
        }
        wave_lds_sync();
        // decision words, one column per lane
#pragma unroll
        for (int rv = 0; rv < NWD; ++rv) {
            const uint64_t ids = it_ids[rv];
            xT[rv * 64 + lane] = lut4_words(it_lut[rv], synT[ids & 0xffff], synT[(ids >> 16) & 0xffff],
                                            synT[(ids >> 32) & 0xffff], synT[ids >> 48]);
        }
        wave_lds_sync();
        // residual syndrome words, one check per lane, OR-reduced over the wave
        uint64_t bad = 0ull;
#pragma unroll
        for (int rc = 0; rc < RC; ++rc) {
            const uint64_t c0 = it_cv[rc][0], c1 = it_cv[rc][1];
            uint64_t par = synT[rc * 64 + lane];
#pragma unroll
            for (int t = 0; t < 4; ++t) par ^= xT[(c0 >> (16 * t)) & 0xffff] ^ xT[(c1 >> (16 * t)) & 0xffff];
            bad |= par;
        }
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)bad, off);
            const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(bad >> 32), off);
            bad |= ((uint64_t)hi << 32) | lo;
        }
        trivial = live && !((bad >> lane) & 1ull);
        int f = 0;
        if (want_fail && __ballot(trivial)) {
            // parity words of the logicals (one logical per lane: the set bits of
            // its row of the dense table), then each shot's bits
            for (int r = lane; r < g.k; r += 64) {
                uint64_t p = 0ull;
                for (int w = 0; w < g.lz_words; ++w)
                    for (uint64_t bits = lz_word(lz_lds, (size_t)r * g.lz_words + w); bits; bits &= bits - 1ull)
                        p ^= xT[w * 64 + __builtin_ctzll(bits)];
                lzp[r] = p;
            }
            wave_lds_sync();
#pragma unroll
            for (int rr = 0; rr < kMaxLogicalRounds; ++rr) {
                const int nr = min(64, g.k - rr * 64);
                for (int t = 0; t < nr; ++t) f |= (int)(((lzp[rr * 64 + t] >> lane) ^ (rp[rr] >> t)) & 1ull);
            }
        }
        fbit = (uint8_t)f;
    } else {
        uint64_t any = 0ull;
#pragma unroll
        for (int rc = 0; rc < RC; ++rc) any |= sw[rc];
        trivial = live && any == 0ull && a.cmp_zero_ok;
        fbit = (uint8_t)((rp[0] | rp[1] | rp[2] | rp[3]) != 0ull);
    }
    if (live && trivial) {
        if (a.iters) a.iters[shot] = 1;
        if (a.status) a.status[shot] = 3;
        if (a.ssf_steps) a.ssf_steps[shot] = 0;
        if (a.fail) a.fail[shot] = want_fail ? fbit : (uint8_t)0;
    }
    const bool listed = live && !trivial;
    const unsigned long long bal = __ballot(listed);
    if (bal == 0ull) return;
    // segment blockIdx % kCmpSegs: 64 counters on their own lines, so the
    // per-tile atomics do not serialise on one address.  Shots of syndrome
    // weight > kHeavyW go to the heavy list (segments kCmpSegs..), which the BP
    // kernel hands out first: the long decodes start at the launch's beginning
    // instead of setting its end (longest-processing-time-first)
    const bool heavy = listed && wt > kHeavyW;
    const unsigned long long balh = __ballot(heavy), ball = bal & ~balh;
    const int seg = (int)(blockIdx.x % kCmpSegs);
    unsigned long long bh = 0, bl = 0;
    if (lane == 0) {
        if (balh) bh = atomicAdd(a.cmp_count + 16 * (kCmpSegs + seg), (unsigned long long)__popcll(balh));
        if (ball) bl = atomicAdd(a.cmp_count + 16 * seg, (unsigned long long)__popcll(ball));
    }
    bh = __shfl(bh, 0);
    bl = __shfl(bl, 0);
    if (listed) {
        const unsigned long long mb = heavy ? balh : ball;
        const uint64_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mb, 0u));
        const int sg = heavy ? kCmpSegs + seg : seg;
        uint64_t* e = a.cmp + ((uint64_t)sg * a.cmp_cap + (heavy ? bh : bl) + rank) * Ent::EW;
        e[0] = (uint64_t)shot;
#pragma unroll
        for (int rc = 0; rc < RC; ++rc) e[1 + rc] = sw[rc];
#pragma unroll
        for (int rr = 0; rr < kMaxLogicalRounds; ++rr) e[1 + RC + rr] = rp[rr];
    }
}

// lane l's copy of v from lane l - off (lanes below off: their own value)
__device__ __forceinline__ uint64_t readlane64_up(uint64_t v, int off, int lane) {
    const int src = lane >= off ? lane - off : lane;
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}

// v_readlane of a 64-bit value (lane uniform)
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

// Small-set-flip of one BP-failed shot inside the compact BP kernel (FUSE > 0,
// QD_OPT_SSF_FUSE): the table-driven spec of ssf_lut_kernel (qdec_bp.hip), with
// the same tables (s_lut, s_off, s_lcw, s_tog), the same key, the same step
// order and the same flip application, so the same outputs; the tables are read
// through the cache hierarchy instead of a workgroup's LDS copy, and the shot
// never goes through the HBM queue or a second launch.  RG: generators per lane
// (n_gen <= 64 * RG).  xb: the wave's hard decision by column as LDS bit words
// (updated in place); flog: the wave's step log; R: residual words by check.
// Returns the steps taken; sw_out = the residual weight left.
template <int RG, int RW>
__device__ __forceinline__ int ssf_fused(const DevGraph& g, int max_steps, uint32_t* xb, uint16_t* flog,
                                      const uint64_t* Rin, int lane, int* sw_out) {
    const uint32_t* __restrict__ lut = g.s_lut;
    const uint32_t* __restrict__ tog = g.s_tog;
    // this lane's generators' table offsets (the winner's local-check ids are read
    // per step at a wave-uniform address instead of being held in registers)
    uint32_t off[RG];
#pragma unroll
    for (int rg = 0; rg < RG; ++rg) off[rg] = g.s_off[rg * 64 + lane];
    // first local syndromes: the toggle rows of the violated checks, 8 rows per
    // round (independent loads; row m_pad is all zero)
    const uint32_t zrow = (uint32_t)g.m_pad;
    uint32_t sl = 0;
    int sw = 0;
#pragma unroll
    for (int w = 0; w < RW; ++w) {
        uint64_t bits = Rin[w];
        sw += __popcll(bits);
        while (bits) {
            uint32_t t = 0;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                uint32_t c = zrow;
                if (bits) {
                    c = (uint32_t)(w * 64 + __builtin_ctzll(bits));
                    bits &= bits - 1;
                }
                t ^= tog[c * 64 + lane];
            }
            sl ^= t;
        }
    }
    int steps = 0;
    while (sw > 0 && (max_steps <= 0 || steps < max_steps)) {
        // every generator's best (rank, -g, t); wave max
        uint32_t e[RG];
        int kv = 0;
#pragma unroll
        for (int rg = 0; rg < RG; ++rg) {
            const uint32_t s = rg ? (sl >> 16) : (sl & 0xffffu);
            e[rg] = lut[off[rg] + s];
            const uint32_t rank = e[rg] >> 24;
            const int key = rank ? (int)((rank << 15) | ((uint32_t)(127 - (rg * 64 + lane)) << 8) | (e[rg] & 0xffu)) : 0;
            kv = max(kv, key);
        }
        const int best = wave_max_i32(kv);
        if (best == 0) break;  // no positive gain left
        const int gsel = 127 - ((best >> 8) & 127);
        const int tsel = best & 255;
        const int owner = gsel & 63;
        const bool hi = RG == 2 && gsel >= 64;
        const uint32_t esel = (uint32_t)__builtin_amdgcn_readlane((int)(hi ? e[RG - 1] : e[0]), owner);
        const uint32_t slg = ((uint32_t)__builtin_amdgcn_readlane((int)sl, owner) >> (hi ? 16 : 0)) & 0xffffu;
        const uint32_t fm = (esel >> 8) & 0xffffu;
        sw -= __builtin_popcount(slg) - __builtin_popcount(slg ^ fm);
        ++steps;
        // toggle the flipped checks' local-syndrome bits (all loads issued first)
        uint32_t tr[kLutLC];
#pragma unroll
        for (int w = 0; w < kLutLCW; ++w) {
            const uint32_t nib = (fm >> (4 * w)) & 0xfu;
            const uint32_t word = nib ? g.s_lcw[w * g.g_pad + gsel] : 0u;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                tr[4 * w + b] = 0u;
                if ((nib >> b) & 1u) tr[4 * w + b] = tog[((word >> (8 * b)) & 0xffu) * 64 + lane];
            }
        }
        uint32_t tg = 0;
#pragma unroll
        for (int b = 0; b < kLutLC; ++b) tg ^= tr[b];
        sl ^= tg;
        if (lane == 0) flog[steps - 1] = (uint16_t)(gsel | (tsel << 8));
    }
    wave_lds_sync();
    // x ^= 1_F of every logged step (a qubit flipped twice cancels, in any order)
    for (int b0 = 0; b0 < steps; b0 += 64) {
        if (b0 + lane < steps) {
            const uint32_t e = flog[b0 + lane];
            const int gg = (int)(e & 0xffu);
#pragma unroll
            for (int k = 0; k < kGenW; ++k)
                if ((e >> (8 + k)) & 1u) {
                    const uint32_t q = g.g_q[k * g.g_pad + gg];
                    atomicXor(&xb[q >> 5], 1u << (q & 31));
                }
        }
    }
    wave_lds_sync();
    *sw_out = sw;
    return steps;
}

// The compact-list BP kernel (see above): the lean bp_ms_wave_kernel's BP
// (MsCore) on the listed shots only.  Entries come in chunks of up to
// CmpEntry::kPer (one u64 per lane, the next chunk loaded while this one
// decodes; a list shorter than kPer entries per wave is cut finer); chunks are
// handed out by ShotSeq (static stride, then a counter for the tail).
// FUSE (with DEFER): 0 = BP-failed shots go to the SSF queue; 1 / 2 = SSF runs
// here (ssf_fused with RG = FUSE generators per lane).
template <typename T, int RC, int RV, int DRC, bool DEFER, int D3R, int OCC = 0, int FUSE = 0>
__global__ __launch_bounds__(64, OCC > 0 ? OCC : (sizeof(T) == 4 ? 4 : 2)) void bp_ms_cmp_kernel(DevGraph g, DecodeArgs a) {
    using Core = MsCore<T, RC, RV, DRC, true, D3R>;
    using Ent = CmpEntry<RC>;
    constexpr int EW = Ent::EW, KP = Ent::kPer;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T* v2c = reinterpret_cast<T*>(smem);
    T* st = v2c + MsLds<T>::v2c_elems(MsLds<T>::rows(g));
    uint8_t* xh = reinterpret_cast<uint8_t*>(st + MsLds<T>::state_elems(g.m_pad));
    uint64_t* lzs = reinterpret_cast<uint64_t*>(smem + MsLds<T>::core_bytes(g));  // [k][RV] slot-order logicals

    const int lane = threadIdx.x;
    const int m = g.m;
    if constexpr (sizeof(T) == 8 && OCC == 0) {
        // f64 at 2 waves per SIMD (the one-pass kernel's placement): the kernel
        // needs ~160 VGPRs, which would let a CU put 3 waves on one SIMD and 1 on
        // another; claiming v175 makes the allocation 176, so at most 2 per SIMD
        asm volatile("" ::: "v175");
    }
    Core core;
    core.load(g, lane);
    Core::init_lds(g, v2c, st, xh, lane);
    const bool want_fail = a.fail && a.readout && g.k > 0;
    if (want_fail)
        for (int e = lane; e < g.k * RV; e += 64) lzs[e] = g.ms_lzs[e];
    wave_lds_sync();

    // chunks of KP entries inside the segments, the heavy list first: virtual
    // segment v < 64 is heavy segment v (physical kCmpSegs + v), v >= 64 light
    // segment v - 64; lane s holds heavy and light segment s's entry counts;
    // seg_end = inclusive prefix of the virtual segments' chunk counts
    static_assert(kCmpSegs == 64, "one lane per segment");
    const int64_t hcount = (int64_t)__builtin_nontemporal_load(a.cmp_count + 16 * (kCmpSegs + lane));
    const int64_t lcount = (int64_t)__builtin_nontemporal_load(a.cmp_count + 16 * lane);
    // entries per chunk: KP, fewer when the list is short (below KP entries per
    // wave the decode is latency-bound: spread the shots over more waves)
    auto wave_prefix = [&](int64_t v) {
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int64_t o = (int64_t)readlane64_up((uint64_t)v, off, lane);
            v += lane >= off ? o : 0;
        }
        return v;
    };
    const int64_t tot = (int64_t)readlane64((uint64_t)wave_prefix(hcount + lcount), 63);
    const int kp = (int)min((int64_t)KP, max((int64_t)1, (tot + gridDim.x - 1) / gridDim.x));
    const int64_t hend = wave_prefix((hcount + kp - 1) / kp);
    const int64_t hch = (int64_t)readlane64((uint64_t)hend, 63);
    const int64_t lend = hch + wave_prefix((lcount + kp - 1) / kp);
    const int64_t nch = (int64_t)readlane64((uint64_t)lend, 63);
    // kept in LDS (read once per chunk), not in registers across the BP loop
    int64_t* seg_end = reinterpret_cast<int64_t*>(lzs + (size_t)g.k * RV);  // [128] chunk prefix
    int64_t* seg_cnt = seg_end + 2 * kCmpSegs;                             // [128] entries
    seg_end[lane] = hend;
    seg_end[kCmpSegs + lane] = lend;
    seg_cnt[lane] = hcount;
    seg_cnt[kCmpSegs + lane] = lcount;
    wave_lds_sync();
    // the chunk counter only pays when the tail is long (>= 16 chunks per wave)
    unsigned long long* ctr = a.wave_ctr && nch >= 16 * (int64_t)gridDim.x ? a.wave_ctr : nullptr;
    ShotSeq seq(nch, ctr, blockIdx.x, gridDim.x, lane, 1);
    int ne_n = 0;  // entries in the chunk load_chunk loaded last
    auto load_chunk = [&](int64_t c) -> uint64_t {
        ne_n = 0;
        if (c >= nch) return 0ull;
        // the virtual segment holding chunk c, then its physical segment
        const int v = __popcll(__ballot(seg_end[lane] <= c)) + __popcll(__ballot(seg_end[kCmpSegs + lane] <= c));
        const int64_t c_in = c - (v ? seg_end[v - 1] : 0);
        const int64_t cnt = seg_cnt[v];
        ne_n = (int)min((int64_t)kp, cnt - c_in * kp);
        const int ps = v < kCmpSegs ? kCmpSegs + v : v - kCmpSegs;
        const int64_t e = ((int64_t)ps * a.cmp_cap + c_in * kp) * EW + lane;
        return lane < ne_n * EW ? __builtin_nontemporal_load(a.cmp + e) : 0ull;
    };
    // one flat loop over this wave's entries (chunk c, entry q of it; the next
    // chunk cn is in flight in entn)
    QDEC_STAMP_DECL
#ifdef QDEC_STAMPS
    const unsigned long long qdec_t0 = __builtin_amdgcn_s_memtime();
#endif
    int64_t c = seq.next(lane);
    uint64_t ent = load_chunk(c);
    int ne = ne_n;
    int64_t cn = c < nch ? seq.next(lane) : nch;
    uint64_t entn = load_chunk(cn);
    int q = 0;
    QDEC_STAMP(4);  // prologue
    while (c < nch) {
        {
            const int64_t shot = (int64_t)readlane64(ent, q * EW);
            bool sbit[RC];
#pragma unroll
            for (int rc = 0; rc < RC; ++rc) sbit[rc] = (readlane64(ent, q * EW + 1 + rc) >> lane) & 1;
            uint64_t rpar[kMaxLogicalRounds];
#pragma unroll
            for (int rr = 0; rr < kMaxLogicalRounds; ++rr) rpar[rr] = readlane64(ent, q * EW + 1 + RC + rr);
            core.write_priors(v2c);
            wave_lds_sync();
            QDEC_STAMP(0);  // entry + initial messages
            T Q[RV];
            uint64_t X[RV];
            bool pres[RC];
            int it = 1;
            const bool conv = core.iterate(a, v2c, st, m, lane, sbit, Q, X, pres, it);
            const int iters = conv ? it : a.max_iter;
            QDEC_STAMP(1);  // BP iterations
            QDEC_COUNT(8, iters);
            QDEC_COUNT(9, 1);
            if (lane == 0 && a.iters) a.iters[shot] = iters;
            if (DEFER && FUSE && !conv) {
                // SSF right here: hard decision by column as LDS bit words, residual
                // by check, then the table-driven flips (ssf_fused)
                uint64_t* xb = reinterpret_cast<uint64_t*>(seg_cnt + 2 * kCmpSegs);  // [RV] (kernel LDS tail)
                uint16_t* flog = reinterpret_cast<uint16_t*>(xb + RV);                // [m_pad]
#pragma unroll
                for (int rv = 0; rv < RV; ++rv) xh[core.col_of(rv)] = (uint8_t)((X[rv] >> lane) & 1);
                wave_lds_sync();
                uint64_t rw[RC];
#pragma unroll
                for (int w = 0; w < RV; ++w) {
                    const uint64_t xw = __ballot(xh[w * 64 + lane] & 1);
                    if (lane == 0) xb[w] = xw;
                }
#pragma unroll
                for (int rc = 0; rc < RC; ++rc) rw[rc] = __ballot(pres[rc]);
                wave_lds_sync();
                int sw = 0;
                const int steps = ssf_fused<(FUSE > 0 ? FUSE : 1), RC>(g, a.ssf_max_steps,
                                                                       reinterpret_cast<uint32_t*>(xb), flog, rw,
                                                                       lane, &sw);
                int f = 0;
                if (want_fail) {  // Lz (by column, the graph's dense table) x against the readout parities
#pragma unroll
                    for (int rr = 0; rr < kMaxLogicalRounds; ++rr) {
                        const int r = rr * 64 + lane;
                        if (r < g.k) {
                            int par = (int)((rpar[rr] >> lane) & 1);
                            for (int w = 0; w < g.lz_words && w < RV; ++w)
                                par += __popcll(g.lz[(size_t)r * g.lz_words + w] & xb[w]);
                            f |= par & 1;
                        }
                    }
                }
                const int any_fail = __ballot(f) != 0ull;
                if (lane == 0) {
                    if (a.status) a.status[shot] = (uint8_t)(sw == 0 ? 2 : 0);
                    if (a.ssf_steps) a.ssf_steps[shot] = steps;
                    if (a.fail) a.fail[shot] = (uint8_t)any_fail;
                }
                wave_lds_sync();
            } else if (DEFER && !conv) {
                // hard decision by column for the SSF queue (slot order -> xh[column])
#pragma unroll
                for (int rv = 0; rv < RV; ++rv) xh[core.col_of(rv)] = (uint8_t)((X[rv] >> lane) & 1);
                wave_lds_sync();
                uint64_t xw[RV], rw[RC], dw[RV];
#pragma unroll
                for (int w = 0; w < RV; ++w) {
                    xw[w] = __ballot(xh[w * 64 + lane] & 1);
                    dw[w] = w < kMaxLogicalRounds ? rpar[w < kMaxLogicalRounds ? w : 0] : 0ull;
                }
#pragma unroll
                for (int rc = 0; rc < RC; ++rc) rw[rc] = __ballot(pres[rc]);
                queue_push_packed<RV, RC>(a, shot, xw, rw, dw, lane);
                wave_lds_sync();
            } else {
                int f = 0;
                if (want_fail) {  // parity of Lz x (slot order) against the readout's
#pragma unroll
                    for (int rr = 0; rr < kMaxLogicalRounds; ++rr) {
                        const int r = rr * 64 + lane;
                        if (r < g.k) {
                            int par = (int)((rpar[rr] >> lane) & 1);
#pragma unroll
                            for (int w = 0; w < RV; ++w) par += __popcll(lz_word(lzs, (size_t)r * RV + w) & X[w]);
                            f |= par & 1;
                        }
                    }
                }
                const int any_fail = __ballot(f) != 0ull;
                if (lane == 0) {
                    if (a.status) a.status[shot] = (uint8_t)(conv ? 3 : 0);
                    if (a.ssf_steps) a.ssf_steps[shot] = 0;
                    if (a.fail) a.fail[shot] = (uint8_t)any_fail;
                }
            }
        }
        QDEC_STAMP(2);  // failure check, outputs / SSF queue
        if (++q == ne) {  // next chunk
            q = 0;
            c = cn;
            ent = entn;
            ne = ne_n;
            cn = c < nch ? seq.next(lane) : nch;
            entn = load_chunk(cn);
            QDEC_STAMP(3);  // chunk hand-off
        }
    }
#ifdef QDEC_STAMPS
    QDEC_COUNT(10, __builtin_amdgcn_s_memtime() - qdec_t0);
    QDEC_COUNT(12, 1);
#endif
    QDEC_FLUSH_AT(32);
}

}  // namespace qdec
