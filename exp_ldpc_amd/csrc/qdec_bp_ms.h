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
// (X[w] = 64 columns per word), and check i's parity is
// popc(X & smask_i) mod 2 with per-lane column masks.  The host picks v2c row
// positions (qdec_abi.cpp ms_layout) so each scatter instruction has at most
// 2-way bank conflicts, which ds_write_b32 absorbs for free.
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

// LDS carve-up (elements of T, then bytes)
template <typename T>
struct MsLds {
    static constexpr int DRS = lds_stride<T, kDR>();
    __host__ __device__ static size_t v2c_elems(int m_pad) { return ((size_t)m_pad * DRS + 64 + 1) / 2 * 2; }
    __host__ __device__ static size_t state_elems(int m_pad) {
        return ((size_t)2 * (m_pad + 1) * sizeof(T) + 15) / 16 * 16 / sizeof(T);
    }
    __host__ __device__ static size_t bytes(int m_pad, int n_pad) {
        return ((v2c_elems(m_pad) + state_elems(m_pad)) * sizeof(T) + (size_t)n_pad + 64 + 15) / 16 * 16;
    }
};

template <typename T, int RC, int RV, int DRC, bool DEFER>
__global__ __launch_bounds__(64, 4) void bp_ms_wave_kernel(DevGraph g, DecodeArgs a) {
    static_assert(DRC <= kDR, "compute width exceeds the LDS row");
    using U = typename FBits<T>::U;
    using V2 = __attribute__((ext_vector_type(2))) T;
    constexpr int DRS = MsLds<T>::DRS;
    constexpr int PREC = sizeof(T) == 4 ? 1 : 0;
    constexpr U kSign = (U)1 << (8 * sizeof(T) - 1);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T* v2c = reinterpret_cast<T*>(smem);
    T* st = v2c + MsLds<T>::v2c_elems(g.m_pad);
    uint8_t* xh = reinterpret_cast<uint8_t*>(st + MsLds<T>::state_elems(g.m_pad));

    const int lane = threadIdx.x;
    const int m = g.m, n = g.n;
    const T* prior = reinterpret_cast<const T*>(g.prior[1][PREC]);

    uint32_t etab[RV][kDC];  // v2c element | state index << 16
    T L[RV];
#pragma unroll
    for (int rv = 0; rv < RV; ++rv) {
        const int j = rv * 64 + lane;
        L[rv] = prior[j];
#pragma unroll
        for (int k = 0; k < kDC; ++k) etab[rv][k] = g.ms_etab[PREC][k * g.n_pad + j];
    }
    uint64_t smask[RC][RV];
#pragma unroll
    for (int rc = 0; rc < RC; ++rc)
#pragma unroll
        for (int w = 0; w < RV; ++w) smask[rc][w] = g.ms_smask[(size_t)w * g.m_pad + rc * 64 + lane];

    // one-time LDS init: unused row positions hold Big forever (never the
    // minimum, positive sign), state m_pad is the zero state of pad edges
    for (int e = lane; e < (int)MsLds<T>::v2c_elems(g.m_pad); e += 64) v2c[e] = Big<T>::v;
    for (int e = lane; e < (int)MsLds<T>::state_elems(g.m_pad); e += 64) st[e] = (T)0;
    for (int e = lane; e < g.n_pad + 64; e += 64) xh[e] = 0;
    __syncthreads();

    for (int64_t shot = blockIdx.x; shot < a.B; shot += gridDim.x) {
        // ---- syndrome ----
        int sbit[RC];
#pragma unroll
        for (int rc = 0; rc < RC; ++rc) {
            const int i = rc * 64 + lane;
            sbit[rc] = (i < m && a.syn) ? (a.syn[shot * m + i] & 1) : 0;
        }
        if (a.syn_flags) {
            const bool use_b = (a.syn_flags & 1) && a.base;
            const bool use_r = (a.syn_flags & 2) && a.readout;
            uint64_t Xf[RV];
#pragma unroll
            for (int w = 0; w < RV; ++w) {
                const int q = w * 64 + lane;
                int v = 0;
                if (q < g.n_data) {
                    if (use_b) v ^= a.base[shot * g.n_data + q];
                    if (use_r) v ^= a.readout[shot * g.n_data + q];
                }
                Xf[w] = __ballot(v & 1);
            }
#pragma unroll
            for (int rc = 0; rc < RC; ++rc) {
                int c = 0;
#pragma unroll
                for (int w = 0; w < RV; ++w) c += __popcll(smask[rc][w] & Xf[w]);
                sbit[rc] ^= c & 1;
            }
        }

        // ---- initial messages: v2c = prior ----
        T vp[RV][kDC];
#pragma unroll
        for (int rv = 0; rv < RV; ++rv)
#pragma unroll
            for (int k = 0; k < kDC; ++k) {
                vp[rv][k] = L[rv];
                v2c[etab[rv][k] & 0xffff] = L[rv];
            }
        __syncthreads();

        T Q[RV];
        uint64_t X[RV];
        int pres[RC];
        int it = 1;
        bool conv = false;
        for (; it <= a.max_iter; ++it) {
            const T alpha = alpha_at<T>(it, a.ms_scaling);
            // ---- check pass: state (m1, m2 | parity) ----
#pragma unroll
            for (int rc = 0; rc < RC; ++rc) {
                const int i = rc * 64 + lane;
                T v[kDR];
                lds_load<T, kDR>(v2c + i * DRS, v);
                T m1 = Big<T>::v, m2 = Big<T>::v;
                int par = sbit[rc];
#pragma unroll
                for (int k = 0; k < DRC; ++k) {
                    const T av = fabs(v[k]);
                    m2 = med3(av, m1, m2);
                    if constexpr (sizeof(T) == 4)
                        m1 = med3(av, m1, -Big<T>::v);  // true median = min(|v|, m1): one VALU, abs modifier
                    else
                        m1 = fmin(m1, av);
                    par ^= v[k] <= (T)0;  // ldpc: bit_to_check <= 0 flips the sign
                }
                V2 s2;
                s2.x = m1;
                s2.y = FBits<T>::from(FBits<T>::to(m2) | (par ? kSign : (U)0));
                *reinterpret_cast<V2*>(st + 2 * i) = s2;
            }
            __syncthreads();

            // ---- variable pass ----
#pragma unroll
            for (int rv = 0; rv < RV; ++rv) {
                T c[kDC];
#pragma unroll
                for (int k = 0; k < kDC; ++k) {
                    const V2 s2 = *reinterpret_cast<const V2*>(st + 2 * (etab[rv][k] >> 16));
                    const U mb = FBits<T>::to(s2.y);
                    const T m2 = FBits<T>::from(mb & ~kSign);
                    const T v = vp[rv][k];
                    const T y = ((fabs(v) == s2.x) ? m2 : s2.x) * alpha;
                    const bool neg = ((mb & kSign) != 0) ^ (v <= (T)0);
                    c[k] = neg ? -y : y;
                }
                T pre[kDC];
                T acc = L[rv];
#pragma unroll
                for (int k = 0; k < kDC; ++k) {
                    pre[k] = acc;
                    acc += c[k];
                }
                Q[rv] = acc;
                X[rv] = __ballot(acc <= (T)0);
                T suf = (T)0;
#pragma unroll
                for (int k = kDC - 1; k >= 0; --k) {
                    const T out = pre[k] + suf;
                    suf += c[k];
                    vp[rv][k] = out;
                    v2c[etab[rv][k] & 0xffff] = out;  // pads -> dummy element
                }
            }

            // ---- syndrome test (registers only) ----
            int bad = 0;
#pragma unroll
            for (int rc = 0; rc < RC; ++rc) {
                uint64_t acc = 0;  // xor of the masked words: (X & M) ^ acc is one v_bitop3 per dword
#pragma unroll
                for (int w = 0; w < RV; ++w) acc ^= smask[rc][w] & X[w];
                pres[rc] = (sbit[rc] ^ __popcll(acc)) & 1;
                bad |= pres[rc];
            }
            __syncthreads();  // v2c scatter complete before the next check pass
            if (__ballot(bad) == 0ull) {
                conv = true;
                break;
            }
        }
        const int iters = conv ? it : a.max_iter;
        if (lane == 0 && a.iters) a.iters[shot] = iters;
#pragma unroll
        for (int rv = 0; rv < RV; ++rv) {
            const int j = rv * 64 + lane;
            if (j < n) xh[j] = (uint8_t)((X[rv] >> lane) & 1);
        }
        if (a.llr_out) {
            T* lo = reinterpret_cast<T*>(a.llr_out);
#pragma unroll
            for (int rv = 0; rv < RV; ++rv) {
                const int j = rv * 64 + lane;
                if (j < n) lo[shot * n + j] = Q[rv];
            }
        }
        __syncthreads();
        if (DEFER && !conv) {
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
        } else {
            finalize_shot(g, a, shot, xh, conv, conv, 0, lane);
        }
        __syncthreads();
    }
}

}  // namespace qdec
