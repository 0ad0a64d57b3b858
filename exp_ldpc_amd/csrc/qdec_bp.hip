// qdec_bp.hip -- BP (+ small-set-flip) syndrome decoding on gfx950.
//
// One wave64 decodes one shot at a time (workgroup = one wave; the grid is
// persistent and walks the shot range).  Everything a shot touches lives in that
// wave's LDS slice:
//   v2c  [m_pad][DRS]  variable->check messages, check-major, 16-B aligned rows
//   c2v  [n_pad][DCS]  check->variable messages, variable-major
//   xh   [n_pad+64]    hard decisions (u8; pad bytes stay 0)
//   sres [m_pad]       residual syndrome for SSF
// A lane owns checks i = lane + 64*rc and variables j = lane + 64*rv.  The check
// pass reads its check's v2c row with ds_read_b128 (conflict-free strides,
// qdec_internal.h lds_stride) and scatters c2v with ds_write_b32 through a slot
// table held in registers; the variable pass does the mirror image.  Slot tables,
// degrees and priors are loaded once per wave.
//
// Arithmetic is the ldpc v1 bp_decoder restated operation for operation (see
// oracle/bp_impl.inc, the CPU copy of the same loops): min-sum in the log domain
// with alpha_t = 1 - 2^-t (ms_scaling_factor = 0) or a constant, product-sum in
// the probability-ratio domain; row leave-one-out products/minima, column
// prefix + suffix sums.  Built with -ffp-contract=off so every multiply and add is
// separately rounded: results are bit-identical to the CPU oracle at the same
// precision.  Min over a row uses min1/min2 (exactly the leave-one-out minimum).
//
// Small-set-flip (build-defined spec): for each generator g (lane
// owned), all subsets F of its <= 8 qubits are scored as
//   key = (gain(F) * 840/|F|, -g, -F)      gain(F) = |s| - |s xor H 1_F|
// with the syndrome restricted to the generator's <= 32 local checks as a bitmask
// (popcount of xor with a per-subset mask).  A wave max picks the flip.
#include <hip/hip_runtime.h>

#include "qdec_internal.h"

namespace qdec {

template <typename T>
struct Big;
template <>
struct Big<float> {
    static constexpr float v = 1e30f;   // fp32 stand-in for ldpc's 1e308 "no minimum yet"
};
template <>
struct Big<double> {
    static constexpr double v = 1e308;
};

__constant__ int kInvSize[9] = {0, 840, 420, 280, 210, 168, 140, 120, 105};

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

template <typename T>
__device__ __forceinline__ T alpha_at(int it, double ms_scaling) {
    return ms_scaling == 0.0 ? (T)(1.0 - ldexp(1.0, -it)) : (T)ms_scaling;
}

// Logical check: fail = any_r parity(lz[r] & (readout ^ corr)).  corr bits are
// produced chunk by chunk (64 qubits) and ballot-ed into a wave-uniform word.
constexpr int kMaxLogicalRounds = 4;  // k <= 256 in the wave kernels

template <typename T, int METHOD, int RC, int RV>
__global__ __launch_bounds__(64) void bp_wave_kernel(DevGraph g, DecodeArgs a) {
    constexpr int DRS = lds_stride<T, kDR>();
    constexpr int DCS = lds_stride<T, kDC>();
    constexpr int PREC = sizeof(T) == 4 ? 1 : 0;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T* v2c = reinterpret_cast<T*>(smem);
    T* c2v = v2c + g.m_pad * DRS;
    uint8_t* xh = reinterpret_cast<uint8_t*>(c2v + g.n_pad * DCS);
    uint8_t* sres = xh + g.n_pad + 64;

    const int lane = threadIdx.x;
    const SlotTables st = g.slots[PREC];
    const T* prior = reinterpret_cast<const T*>(g.prior[METHOD][PREC]);
    const int m = g.m, n = g.n;

    // ---- per-lane graph tables (registers) ----
    int degR[RC];
    uint32_t rtab[RC][kDR];  // col | cslot << 16
    int degC[RV];
    uint32_t ctab[RV][kDC / 2];  // rslot pairs
    T L[RV];
#pragma unroll
    for (int rc = 0; rc < RC; ++rc) {
        const int i = rc * 64 + lane;
        const bool on = rc * 64 < m;
        degR[rc] = on ? g.r_deg[i] : 0;
#pragma unroll
        for (int k = 0; k < kDR; ++k)
            rtab[rc][k] = on ? ((uint32_t)g.r_col[k * g.m_pad + i] | ((uint32_t)st.r_cslot[k * g.m_pad + i] << 16))
                             : (uint32_t)g.n_pad;
    }
#pragma unroll
    for (int rv = 0; rv < RV; ++rv) {
        const int j = rv * 64 + lane;
        const bool on = rv * 64 < n;
        degC[rv] = on ? g.c_deg[j] : 0;
        L[rv] = on ? prior[j] : (T)0;
#pragma unroll
        for (int k = 0; k < kDC / 2; ++k)
            ctab[rv][k] = on ? ((uint32_t)st.c_rslot[(2 * k) * g.n_pad + j] |
                                ((uint32_t)st.c_rslot[(2 * k + 1) * g.n_pad + j] << 16))
                             : 0u;
    }

    // ---- one-time LDS init: pads hold neutral messages forever ----
    const T vneutral = METHOD == 1 ? Big<T>::v : (T)0;  // MS: |v| never the min; PS: factor 1
    const T cneutral = METHOD == 1 ? (T)0 : (T)1;       // MS: +0 in sums; PS: x1 in products
    for (int e = lane; e < g.m_pad * DRS; e += 64) v2c[e] = vneutral;
    for (int e = lane; e < g.n_pad * DCS; e += 64) c2v[e] = cneutral;
    for (int e = lane; e < g.n_pad + 64; e += 64) xh[e] = 0;
    for (int e = lane; e < g.m_pad; e += 64) sres[e] = 0;
    __syncthreads();

    for (int64_t shot = blockIdx.x; shot < a.B; shot += gridDim.x) {
        // ---- syndrome ----
        int sbit[RC];
#pragma unroll
        for (int rc = 0; rc < RC; ++rc) {
            const int i = rc * 64 + lane;
            sbit[rc] = (rc * 64 < m && i < m && a.syn) ? (a.syn[shot * m + i] & 1) : 0;
        }
        if (a.syn_flags) {
            const bool use_b = (a.syn_flags & 1) && a.base;
            const bool use_r = (a.syn_flags & 2) && a.readout;
            for (int q = lane; q < g.n_pad; q += 64) {
                uint8_t v = 0;
                if (q < g.n_data) {
                    if (use_b) v ^= a.base[shot * g.n_data + q];
                    if (use_r) v ^= a.readout[shot * g.n_data + q];
                }
                xh[q] = v & 1;
            }
            __syncthreads();
#pragma unroll
            for (int rc = 0; rc < RC; ++rc) {
                if (rc * 64 >= m) continue;
                int p = 0;
#pragma unroll
                for (int k = 0; k < kDR; ++k)
                    if (k < degR[rc]) p ^= xh[rtab[rc][k] & 0xffff];
                sbit[rc] ^= p;
            }
            __syncthreads();
        }

        // ---- initial messages ----
#pragma unroll
        for (int rv = 0; rv < RV; ++rv) {
#pragma unroll
            for (int k = 0; k < kDC; ++k) {
                if (k < degC[rv]) {
                    const uint32_t s = (ctab[rv][k >> 1] >> ((k & 1) * 16)) & 0xffff;
                    v2c[s] = L[rv];
                }
            }
        }
        __syncthreads();

        T Q[RV];
        int pres[RC];
        int it = 1;
        bool conv = false;
        for (; it <= a.max_iter; ++it) {
            // ---- check -> variable ----
            const T alpha = alpha_at<T>(it, a.ms_scaling);
#pragma unroll
            for (int rc = 0; rc < RC; ++rc) {
                if (rc * 64 >= m) continue;
                const int i = rc * 64 + lane;
                T v[kDR];
                lds_load<T, kDR>(v2c + i * DRS, v);
                if constexpr (METHOD == 1) {
                    T min1 = Big<T>::v, min2 = Big<T>::v;
                    int idx = 0, par = sbit[rc];
#pragma unroll
                    for (int k = 0; k < kDR; ++k) {
                        const T av = fabs(v[k]);
                        if (av < min1) {
                            min2 = min1;
                            min1 = av;
                            idx = k;
                        } else if (av < min2) {
                            min2 = av;
                        }
                        par ^= (v[k] <= (T)0) ? 1 : 0;
                    }
#pragma unroll
                    for (int k = 0; k < kDR; ++k) {
                        if (k < degR[rc]) {
                            const T mag = (k == idx) ? min2 : min1;
                            const int pk = par ^ ((v[k] <= (T)0) ? 1 : 0);
                            c2v[rtab[rc][k] >> 16] = mag * (pk ? -alpha : alpha);
                        }
                    }
                } else {
                    T t[kDR], fw[kDR];
                    T f = sbit[rc] ? (T)-1 : (T)1;
#pragma unroll
                    for (int k = 0; k < kDR; ++k) {
                        t[k] = (T)2 / ((T)1 + v[k]) - (T)1;
                        fw[k] = f;
                        f *= t[k];
                    }
                    T b = (T)1;
#pragma unroll
                    for (int k = kDR - 1; k >= 0; --k) {
                        T c = fw[k] * b;
                        c = ((T)1 - c) / ((T)1 + c);
                        b *= t[k];
                        if (k < degR[rc]) c2v[rtab[rc][k] >> 16] = c;
                    }
                }
            }
            __syncthreads();

            // ---- variable -> check, hard decision ----
#pragma unroll
            for (int rv = 0; rv < RV; ++rv) {
                if (rv * 64 >= n) continue;
                const int j = rv * 64 + lane;
                T c[kDC];
                lds_load<T, kDC>(c2v + j * DCS, c);
                T pre[kDC];
                int xb;
                if constexpr (METHOD == 1) {
                    T acc = L[rv];
#pragma unroll
                    for (int k = 0; k < kDC; ++k) {
                        pre[k] = acc;
                        acc += c[k];
                    }
                    Q[rv] = acc;
                    xb = acc <= (T)0;
                    T suf = (T)0;
#pragma unroll
                    for (int k = kDC - 1; k >= 0; --k) {
                        const T out = pre[k] + suf;
                        suf += c[k];
                        if (k < degC[rv]) v2c[(ctab[rv][k >> 1] >> ((k & 1) * 16)) & 0xffff] = out;
                    }
                } else {
                    T acc = L[rv];
#pragma unroll
                    for (int k = 0; k < kDC; ++k) {
                        pre[k] = acc;
                        acc *= c[k];
                        if (isnan(acc)) acc = (T)1;
                    }
                    Q[rv] = acc;
                    xb = acc >= (T)1;
                    T suf = (T)1;
#pragma unroll
                    for (int k = kDC - 1; k >= 0; --k) {
                        const T out = pre[k] * suf;
                        suf *= c[k];
                        if (isnan(suf)) suf = (T)1;
                        if (k < degC[rv]) v2c[(ctab[rv][k >> 1] >> ((k & 1) * 16)) & 0xffff] = out;
                    }
                }
                if (j < n) xh[j] = (uint8_t)xb;
            }
            __syncthreads();

            // ---- syndrome test ----
            int bad = 0;
#pragma unroll
            for (int rc = 0; rc < RC; ++rc) {
                int p = sbit[rc];
                if (rc * 64 < m) {
#pragma unroll
                    for (int k = 0; k < kDR; ++k)
                        if (k < degR[rc]) p ^= xh[rtab[rc][k] & 0xffff];
                }
                pres[rc] = p;
                bad |= p;
            }
            if (__ballot(bad) == 0ull) {
                conv = true;
                break;
            }
        }
        const int iters = conv ? it : a.max_iter;

        // ---- small-set-flip on the residual syndrome ----
        int steps = 0;
        bool satisfied = conv;
        if (a.ssf && !conv && g.n_gen > 0) {
            int w_local = 0;
#pragma unroll
            for (int rc = 0; rc < RC; ++rc) {
                const int i = rc * 64 + lane;
                if (rc * 64 < m && i < m) sres[i] = (uint8_t)pres[rc];
                w_local += pres[rc];
            }
            int sw = wave_sum_i32(w_local);
            __syncthreads();
            const int nhi = g.g_wmax > 4 ? (1 << (g.g_wmax - 4)) : 1;
            while (sw > 0 && (a.ssf_max_steps <= 0 || steps < a.ssf_max_steps)) {
                long long best = LLONG_MIN;
                for (int g0 = 0; g0 < g.n_gen; g0 += 64) {
                    const int gi = g0 + lane;
                    if (gi >= g.n_gen) continue;
                    const int w = g.g_w[gi];
                    const int nlc = g.g_nlc[gi];
                    uint32_t sl = 0;
                    for (int c = 0; c < nlc; ++c) sl |= (uint32_t)sres[g.g_lc[c * g.g_pad + gi]] << c;
                    uint32_t qm[kGenW];
#pragma unroll
                    for (int k = 0; k < kGenW; ++k) qm[k] = k < w ? g.g_qmask[k * g.g_pad + gi] : 0u;
                    uint32_t lo[16];
                    lo[0] = 0;
#pragma unroll
                    for (int l = 1; l < 16; ++l) {
                        const int b = __builtin_ctz(l);
                        lo[l] = lo[l & (l - 1)] ^ qm[b];
                    }
                    const int base = __builtin_popcount(sl);
                    const int tlim = 1 << w;
                    int best32 = INT_MIN;
                    for (int hi = 0; hi < nhi; ++hi) {
                        const uint32_t mh = ((hi & 1) ? qm[4] : 0u) ^ ((hi & 2) ? qm[5] : 0u) ^
                                            ((hi & 4) ? qm[6] : 0u) ^ ((hi & 8) ? qm[7] : 0u);
                        const uint32_t sh = sl ^ mh;
                        const int hs = __builtin_popcount(hi);
#pragma unroll
                        for (int l = 0; l < 16; ++l) {
                            const int t = hi * 16 + l;
                            const int size = hs + __builtin_popcount(l);
                            const int score = (base - __builtin_popcount(sh ^ lo[l])) * kInvSize[size];
                            const int key = score * 256 + (255 - t);
                            if (t > 0 && t < tlim) best32 = key > best32 ? key : best32;
                        }
                    }
                    const long long key64 = ((long long)(best32 >> 8) << 32) |
                                            ((long long)(0xFFFFFF - gi) << 8) | (long long)(best32 & 255);
                    best = key64 > best ? key64 : best;
                }
                best = wave_max_i64(best);
                const int score = (int)(best >> 32);
                if (score <= 0) break;
                const int gsel = 0xFFFFFF - (int)((best >> 8) & 0xFFFFFF);
                const int tsel = 255 - (int)(best & 255);
                const int size = __builtin_popcount(tsel);
                const int gain = score * size / kSsfScale;
                const int w = g.g_w[gsel];
                uint32_t mask = 0;
                for (int k = 0; k < w; ++k)
                    if ((tsel >> k) & 1) mask ^= g.g_qmask[k * g.g_pad + gsel];
                const int nlc = g.g_nlc[gsel];
                if (lane < nlc && ((mask >> lane) & 1)) sres[g.g_lc[lane * g.g_pad + gsel]] ^= 1;
                if (lane < w && ((tsel >> lane) & 1)) xh[g.g_q[lane * g.g_pad + gsel]] ^= 1;
                __syncthreads();
                sw -= gain;
                ++steps;
            }
            satisfied = (sw == 0);
            // leave sres clean for the next shot
            for (int e = lane; e < g.m_pad; e += 64) sres[e] = 0;
            __syncthreads();
        }

        // ---- outputs ----
        if (a.x_out)
            for (int j = lane; j < n; j += 64) a.x_out[shot * n + j] = xh[j];
        if (a.llr_out) {
            T* lo = reinterpret_cast<T*>(a.llr_out);
#pragma unroll
            for (int rv = 0; rv < RV; ++rv) {
                const int j = rv * 64 + lane;
                if (rv * 64 < n && j < n) {
                    if constexpr (METHOD == 1) lo[shot * n + j] = Q[rv];
                    else lo[shot * n + j] = (T)log((double)((T)1 / Q[rv]));
                }
            }
        }
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
            if (a.iters) a.iters[shot] = iters;
            if (a.status) a.status[shot] = (uint8_t)((conv ? 1 : 0) | (satisfied ? 2 : 0));
            if (a.ssf_steps) a.ssf_steps[shot] = steps;
            if (a.fail) a.fail[shot] = (uint8_t)any_fail;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------- launcher
template <typename T>
static size_t wave_lds_bytes(const DevGraph& g) {
    constexpr int DRS = lds_stride<T, kDR>();
    constexpr int DCS = lds_stride<T, kDC>();
    return (size_t)g.m_pad * DRS * sizeof(T) + (size_t)g.n_pad * DCS * sizeof(T) + (size_t)g.n_pad + 64 +
           (size_t)g.m_pad;
}

template <typename T, int METHOD, int RC, int RV>
static int launch_wave(const DevGraph& g, const DecodeArgs& a, int num_cus, hipStream_t stream) {
    auto kern = bp_wave_kernel<T, METHOD, RC, RV>;
    const size_t lds = (wave_lds_bytes<T>(g) + 15) / 16 * 16;
    int per_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64, lds);
    if (e != hipSuccess) return (int)e;
    if (per_cu <= 0) return (int)hipErrorInvalidConfiguration;
    long long grid = (long long)num_cus * per_cu;
    if (grid > a.B) grid = a.B;
    if (grid <= 0) return 0;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64), lds, stream, g, a);
    return (int)hipGetLastError();
}

template <typename T, int METHOD>
static int dispatch_shape(const DevGraph& g, const DecodeArgs& a, int num_cus, hipStream_t stream) {
    const int rc = g.m_pad / 64, rv = g.n_pad / 64;
    if (rc <= 2 && rv <= 4) return launch_wave<T, METHOD, 2, 4>(g, a, num_cus, stream);
    if (rc <= 4 && rv <= 9) return launch_wave<T, METHOD, 4, 9>(g, a, num_cus, stream);
    return (int)hipErrorNotSupported;
}

bool wave_kernel_supports(const DevGraph& g) {
    return g.max_rdeg <= kDR && g.max_cdeg <= kDC && g.m_pad / 64 <= 4 && g.n_pad / 64 <= 9 && g.k <= 256;
}

int launch_decode(const DevGraph& g, int method, int precision, const DecodeArgs& a, int num_cus,
                  hipStream_t stream) {
    if (a.B <= 0) return 0;
    if (!wave_kernel_supports(g)) return (int)hipErrorNotSupported;
    if (precision == 1)
        return method == 1 ? dispatch_shape<float, 1>(g, a, num_cus, stream)
                           : dispatch_shape<float, 0>(g, a, num_cus, stream);
    return method == 1 ? dispatch_shape<double, 1>(g, a, num_cus, stream)
                       : dispatch_shape<double, 0>(g, a, num_cus, stream);
}

// ---------------------------------------------------------------- flag counter
__global__ void count_flags_kernel(const uint8_t* __restrict__ f, int64_t B, uint8_t mask,
                                   unsigned long long* out) {
    long long local = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < B; i += (int64_t)gridDim.x * blockDim.x)
        local += (f[i] & mask) ? 1 : 0;
    local = wave_sum_i32((int)local);
    if ((threadIdx.x & 63) == 0 && local) atomicAdd(out, (unsigned long long)local);
}

int launch_count_flags(const uint8_t* flags, int64_t B, uint8_t mask, int64_t* out, hipStream_t stream) {
    if (B <= 0) return 0;
    long long blocks = (B + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(count_flags_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, flags, B, mask,
                       reinterpret_cast<unsigned long long*>(out));
    return (int)hipGetLastError();
}

}  // namespace qdec
