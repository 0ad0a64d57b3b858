// qdec_bp_block.hip -- BP + SSF for graphs outside the wave kernels' shapes
// (multi-round spacetime matrices with R >= 2, codes with n > 576, degrees > 8/4).
//
// One 256-thread workgroup decodes one shot at a time (persistent grid).  Graph
// tables are read from global memory (CSR row_ptr/col_idx, CSC col_ptr/col_edge;
// L1/L2 resident, shared by every workgroup).  Messages are indexed by CSR edge
// id: v2c[E], c2v[E] live in LDS when 2*E*sizeof(T) fits, otherwise in a
// per-workgroup slice of an HBM scratch buffer (the HBM-bound regime of the 10k
// and 50k qubit configurations).  The loops are ldpc v1's, operation for
// operation (same arithmetic as the wave kernels and oracle/bp_impl.inc):
//   check pass: thread per check, forward/backward along the row
//   variable pass: thread per variable, prefix then suffix along the column
// Small-set-flip runs in ssf_block_kernel on the same HBM work queue as the wave
// path, with generators spread over the workgroup's threads.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "qdec_device.h"

namespace qdec {

constexpr int kBlock = 256;

// Every block kernel starts its dynamic LDS with a 64-byte control area (no
// static __shared__, so the dynamic base stays 16-byte aligned):
//   [0, 32) long long red64[4]   [32, 48) int red32[4]   [48, 52) int slot
//   [56, 64) long long next shot (dynamic shot counter)
constexpr int kCtrl = 64;

// block-wide sum / max through the control area (all threads must call)
__device__ long long block_max_i64(long long v, long long* red) {
    v = wave_max_i64(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    long long r = red[0];
    for (int i = 1; i < kBlock / 64; ++i) r = red[i] > r ? red[i] : r;
    __syncthreads();
    return r;
}

__device__ int block_sum_i32(int v, int* red) {
    v = wave_sum_i32(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    int r = 0;
    for (int i = 0; i < kBlock / 64; ++i) r += red[i];
    __syncthreads();
    return r;
}

// dst[0..len) = src[0..len) (byte arrays, thread-strided), eight loads per
// thread issued before the stores; returns this thread's sum of the bytes
__device__ __forceinline__ int copy_bytes8(const uint8_t* src, uint8_t* dst, int len, int tid) {
    int sum = 0;
    for (int j0 = tid; j0 < len; j0 += 8 * kBlock) {
        uint8_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = j0 + u * kBlock < len ? src[j0 + u * kBlock] : (uint8_t)0;
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (j0 + u * kBlock < len) {
                dst[j0 + u * kBlock] = v[u];
                sum += v[u];
            }
    }
    return sum;
}

// Outputs of one shot from its hard decision xh (LDS): x_out, corr = base ^
// fold(xh), fail = any_r parity(lz[r] & (readout ^ corr)) (per-thread word parities
// xor-reduced into LDS), status, ssf_steps.
__device__ void finalize_block(const DevGraph& g, const DecodeArgs& a, int64_t shot, const uint8_t* xh, bool conv,
                               bool satisfied, int steps, int* lpar /* LDS [k] */,
                               const uint8_t* rd_lds = nullptr /* LDS copy of the shot's readout, or null */) {
    const int tid = threadIdx.x;
    auto rd = [&](int q) -> uint8_t { return rd_lds ? rd_lds[q] : a.readout[shot * g.n_data + q]; };
    if (a.x_out)
        for (int j = tid; j < g.n; j += kBlock) a.x_out[shot * g.n + j] = xh[j];
    const bool want_fail = a.fail && a.readout && g.k > 0;
    if (want_fail)
        for (int r = tid; r < g.k; r += kBlock) lpar[r] = 0;
    __syncthreads();
    // by qubit (DevGraph::lz_t): lpar holds lz_tw parity words; each residual one
    // XORs its qubit's words in
    const bool cols = want_fail && g.lz_t;
    const bool walk = want_fail && !cols && g.lz_sparse;
    if (cols) {
        uint32_t* lw = reinterpret_cast<uint32_t*>(lpar);  // lz_tw <= k words, zeroed above
        const int nd = g.n_data, tw = g.lz_tw;
        for (int q0 = tid; q0 < nd; q0 += 8 * kBlock) {
            uint8_t rv[8], bv[8];  // eight qubits per round, their loads first
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int q = q0 + u * kBlock;
                rv[u] = q < nd ? rd(q) : (uint8_t)0;
                bv[u] = (q < nd && a.base) ? a.base[shot * nd + q] : (uint8_t)0;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int q = q0 + u * kBlock;
                if (q >= nd) break;
                int cb = bv[u] & 1;
                for (int t = 0; t < g.fold_blocks; ++t) cb ^= xh[t * nd + q];
                if (a.corr_out) a.corr_out[shot * nd + q] = (uint8_t)cb;
                if ((rv[u] ^ cb) & 1)
                    for (int t = 0; t < tw; ++t) {
                        const uint32_t v = g.lz_t[(size_t)q * tw + t];
                        if (v) atomicXor(&lw[t], v);
                    }
            }
        }
    }
    if (walk) {  // sparse logicals: each thread tests whole logicals on their supports
        for (int r = tid; r < g.k; r += kBlock) {
            int par = 0;
            for (int t = g.lz_ptr[r]; t < g.lz_ptr[r + 1]; ++t) {
                const int q = g.lz_idx[t];
                int cb = rd(q) ^ (a.base ? a.base[shot * g.n_data + q] : 0);
                for (int b = 0; b < g.fold_blocks; ++b) cb ^= xh[b * g.n_data + q];
                par ^= cb & 1;
            }
            lpar[r] = par;
        }
    }
    if (a.corr_out && !cols && (!want_fail || walk)) {
        for (int q = tid; q < g.n_data; q += kBlock) {
            int cb = a.base ? (a.base[shot * g.n_data + q] & 1) : 0;
            for (int t = 0; t < g.fold_blocks; ++t) cb ^= xh[t * g.n_data + q];
            a.corr_out[shot * g.n_data + q] = (uint8_t)cb;
        }
    } else if (want_fail && !cols && !walk) {
        // dense logicals, kBlock words at a time: wave w builds words
        // base + 64 w + i (i < 64) by ballots over coalesced byte reads and lane
        // i keeps word i; then per logical r each lane ANDs its word with the
        // row's (a coalesced load across the lanes), the wave folds the parities
        // with one ballot, and one LDS XOR per wave and row accumulates them
        const int lane = tid & 63, wv = tid >> 6;
        for (int wbase = 0; wbase < g.lz_words; wbase += kBlock) {
            unsigned long long mine = 0ull;
            for (int i0 = 0; i0 < 64; i0 += 8) {
                if (wbase + wv * 64 + i0 >= g.lz_words) break;  // uniform
                // eight words per round: their readout / base bytes loaded first
                uint8_t rv[8], bv[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int q = (wbase + wv * 64 + i0 + u) * 64 + lane;
                    const bool in = q < g.n_data && wbase + wv * 64 + i0 + u < g.lz_words;
                    rv[u] = in ? rd(q) : (uint8_t)0;
                    bv[u] = (in && a.base) ? a.base[shot * g.n_data + q] : (uint8_t)0;
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int w0 = wbase + wv * 64 + i0 + u;
                    if (w0 >= g.lz_words) break;  // uniform
                    const int q = w0 * 64 + lane;
                    int v = 0;
                    if (q < g.n_data) {
                        int cb = bv[u] & 1;
                        for (int t = 0; t < g.fold_blocks; ++t) cb ^= xh[t * g.n_data + q];
                        if (a.corr_out) a.corr_out[shot * g.n_data + q] = (uint8_t)cb;
                        v = (rv[u] ^ cb) & 1;
                    }
                    const unsigned long long word = __ballot(v);
                    mine = lane == i0 + u ? word : mine;
                }
            }
            const int w0 = wbase + tid;
            const bool have = w0 < g.lz_words;
            for (int r = 0; r < g.k; ++r) {
                const int x = have ? (__popcll(g.lz[(size_t)r * g.lz_words + w0] & mine) & 1) : 0;
                if (__popcll(__ballot(x)) & 1) {  // uniform per wave
                    if (lane == 0) atomicXor(&lpar[r], 1);
                }
            }
        }
    }
    __syncthreads();
    int f = 0;
    if (want_fail)
        for (int r = tid; r < g.k; r += kBlock) f |= lpar[r] != 0;
    f = __syncthreads_or(f) ? 1 : 0;
    if (tid == 0) {
        if (a.status) a.status[shot] = (uint8_t)((conv ? 1 : 0) | (satisfied ? 2 : 0));
        if (a.ssf_steps) a.ssf_steps[shot] = steps;
        if (a.fail) a.fail[shot] = (uint8_t)(want_fail ? f : 0);
    }
    __syncthreads();
}

// control area + xh + one or two m_pad byte arrays + logical parities
__host__ __device__ inline size_t block_small_lds(const DevGraph& g) {
    return kCtrl + (size_t)g.n_pad + 2 * (size_t)g.m_pad + 4 * (size_t)(g.k > 0 ? g.k : 1);
}

// Bytes of one workgroup's HBM scratch slice: the messages and/or the per-shot
// byte arrays that do not fit the LDS budget (placement bits as in bp_block_kernel).
__host__ __device__ inline size_t block_slice_bytes(const DevGraph& g, size_t tsz, int placement) {
    size_t b = 0;
    if (!(placement & 1)) b += ((size_t)2 * g.E * tsz + 15) / 16 * 16;
    if (!(placement & 2)) b += (block_small_lds(g) + 255) / 256 * 256;
    return (b + 255) / 256 * 256;
}

// DRM / DCM > 0 (row degree <= DRM, column degree <= DCM; both methods): the row and
// column loops are unrolled to that width with every load of a row (column)
// issued before any use, and the column pass keeps its prefix sums in registers
// (one scattered read and one scattered write per edge instead of five).  Same
// operations in the same order as the generic loops.
template <typename T, int METHOD, bool DEFER, int DRM = 0, int DCM = 0>
__global__ __launch_bounds__(kBlock) void bp_block_kernel(DevGraph g, DecodeArgs a, T* gscratch, int placement) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int E = g.E, m = g.m, n = g.n, tid = threadIdx.x;
    constexpr int PREC = sizeof(T) == 4 ? 1 : 0;
    int* slot_s = reinterpret_cast<int*>(smem + 48);
    // placement bit 0: messages in LDS, bit 1: per-shot byte arrays in LDS;
    // whatever is not in LDS lives in this workgroup's HBM scratch slice
    const size_t msg_bytes = ((size_t)2 * E * sizeof(T) + 15) / 16 * 16;
    unsigned char* slice = reinterpret_cast<unsigned char*>(gscratch) +
                           (size_t)blockIdx.x * block_slice_bytes(g, sizeof(T), placement);
    unsigned char* p = (placement & 2) ? smem + kCtrl : slice + ((placement & 1) ? 0 : msg_bytes);
    T* v2c;
    if (placement & 1) {
        v2c = reinterpret_cast<T*>(p);
        p += msg_bytes;
    } else {
        v2c = reinterpret_cast<T*>(slice);
    }
    T* c2v = v2c + E;
    uint8_t* xh = p;                      // [n_pad]
    uint8_t* sb = xh + g.n_pad;           // [m_pad] syndrome bits
    int* lpar = reinterpret_cast<int*>(sb + g.m_pad);  // [k]
    uint8_t* rs = reinterpret_cast<uint8_t*>(lpar + (g.k > 0 ? g.k : 1));  // [m_pad] last residual
    const T* prior = reinterpret_cast<const T*>(g.prior[METHOD][PREC]);
    const int32_t* rp = g.row_ptr;
    const int32_t* ci = g.col_idx;
    const int32_t* cp = g.col_ptr;
    const int32_t* ce = g.col_edge;
    // the unrolled instantiations store c2v in CSC (column) order, so the
    // column pass reads it sequentially and only the row pass's writes scatter
    const int32_t* ecs = g.edge_csc;
    constexpr bool kCsc = DRM > 0;
    // unrolled min-sum with messages in HBM: v2c in CSC order and c2v in CSR
    // order instead, so both passes write contiguously and only their reads
    // scatter.  A scattered 4-byte HBM write costs a partial-sector write-back
    // (C5: ~30 B of HBM writes per message write, 155 MB per shot); a
    // scattered read costs a sector fetch without the write-back.
    const bool vcsc = METHOD == 1 && DRM > 0 && !(placement & 1);
    // placement 0 (byte arrays in HBM): the unrolled instantiation also keeps the
    // hard decision as bits in LDS ([n_pad/64] words, one ballot per wave), so the
    // syndrome test gathers bits from LDS instead of bytes from HBM
    uint64_t* xbits = reinterpret_cast<uint64_t*>(smem + kCtrl);
    const bool xb = DRM > 0 && placement == 0;

    // next shot: from the launcher's counter (dynamic, a.work_ctr) or by stride
    long long* next_s = reinterpret_cast<long long*>(smem + 56);
    auto next_shot = [&](int64_t cur) -> int64_t {
        if (!a.work_ctr) return cur < 0 ? (int64_t)blockIdx.x : cur + gridDim.x;
        if (tid == 0) *next_s = (long long)atomicAdd(a.work_ctr, 1ull);
        __syncthreads();
        const int64_t s = *next_s;
        __syncthreads();  // every thread has read it before the next overwrite
        return s;
    };
    for (int64_t shot = next_shot(-1); shot < a.B; shot = next_shot(shot)) {
        for (int i = tid; i < m; i += kBlock) {
            int s = a.syn ? (a.syn[shot * m + i] & 1) : 0;
            if (a.syn_flags) {
                for (int e = rp[i]; e < rp[i + 1]; ++e) {
                    const int j = ci[e];
                    if (j >= g.n_data) continue;
                    if ((a.syn_flags & 1) && a.base) s ^= a.base[shot * g.n_data + j] & 1;
                    if ((a.syn_flags & 2) && a.readout) s ^= a.readout[shot * g.n_data + j] & 1;
                }
            }
            sb[i] = (uint8_t)s;
        }
        if (vcsc) {
            for (int j = tid; j < n; j += kBlock) {
                const T pj = prior[j];
                for (int t = cp[j]; t < cp[j + 1]; ++t) v2c[t] = pj;  // CSC order
            }
        } else {
            for (int e = tid; e < E; e += kBlock) v2c[e] = prior[ci[e]];  // CSR order: coalesced
        }
        __syncthreads();
        int it = 1;
        bool conv = false;
        for (; it <= a.max_iter; ++it) {
            const T alpha = alpha_at<T>(it, a.ms_scaling);
            for (int i = tid; i < m; i += kBlock) {
                const int e0 = rp[i], e1 = rp[i + 1];
                if constexpr (METHOD == 1 && DRM > 0) {
                    const int d = e1 - e0;
                    T v[DRM];
#pragma unroll
                    for (int t = 0; t < DRM; ++t)
                        if (t < d) v[t] = v2c[vcsc ? ecs[e0 + t] : e0 + t];
                    T m1 = Big<T>::v, m2 = Big<T>::v;
                    int par = sb[i];
#pragma unroll
                    for (int t = 0; t < DRM; ++t)
                        if (t < d) {
                            const T av = fabs(v[t]);
                            m2 = med3(av, m1, m2);
                            m1 = fmin(m1, av);
                            par ^= v[t] <= (T)0;
                        }
                    const T m1a = m1 * alpha, m2a = m2 * alpha;
#pragma unroll
                    for (int t = 0; t < DRM; ++t)
                        if (t < d) {
                            const T y = (fabs(v[t]) == m1) ? m2a : m1a;
                            c2v[vcsc ? e0 + t : ecs[e0 + t]] = (par ^ (v[t] <= (T)0)) ? -y : y;
                        }
                } else if constexpr (METHOD == 1) {
                    T m1 = Big<T>::v, m2 = Big<T>::v;
                    int par = sb[i];
                    for (int e = e0; e < e1; ++e) {
                        const T v = v2c[e];
                        const T av = fabs(v);
                        m2 = med3(av, m1, m2);
                        m1 = fmin(m1, av);
                        par ^= v <= (T)0;
                    }
                    const T m1a = m1 * alpha, m2a = m2 * alpha;
                    for (int e = e0; e < e1; ++e) {
                        const T v = v2c[e];
                        const T y = (fabs(v) == m1) ? m2a : m1a;
                        c2v[e] = (par ^ (v <= (T)0)) ? -y : y;
                    }
                } else if constexpr (DRM > 0) {
                    // product-sum, unrolled: forward products, then backward
                    const int d = e1 - e0;
                    T v[DRM], r[DRM], fw[DRM];
#pragma unroll
                    for (int t = 0; t < DRM; ++t)
                        if (t < d) v[t] = v2c[e0 + t];
                    T f = sb[i] ? (T)-1 : (T)1;
#pragma unroll
                    for (int t = 0; t < DRM; ++t)
                        if (t < d) {
                            fw[t] = f;
                            r[t] = (T)2 / ((T)1 + v[t]) - (T)1;
                            f *= r[t];
                        }
                    T b = (T)1;
#pragma unroll
                    for (int t = DRM - 1; t >= 0; --t)
                        if (t < d) {
                            const T c = fw[t] * b;
                            c2v[ecs[e0 + t]] = ((T)1 - c) / ((T)1 + c);
                            b *= r[t];
                        }
                } else {
                    T f = sb[i] ? (T)-1 : (T)1;
                    for (int e = e0; e < e1; ++e) {
                        c2v[e] = f;
                        f *= (T)2 / ((T)1 + v2c[e]) - (T)1;
                    }
                    T b = (T)1;
                    for (int e = e1 - 1; e >= e0; --e) {
                        T c = c2v[e] * b;
                        c2v[e] = ((T)1 - c) / ((T)1 + c);
                        b *= (T)2 / ((T)1 + v2c[e]) - (T)1;
                    }
                }
            }
            __syncthreads();
            for (int j = tid; j < n; j += kBlock) {
                const int t0 = cp[j], t1 = cp[j + 1];
                T acc = prior[j];
                if constexpr (METHOD == 1 && DCM > 0) {
                    const int d = t1 - t0;
                    int ev[DCM];
                    T c[DCM], pre[DCM];
#pragma unroll
                    for (int t = 0; t < DCM; ++t)
                        if (t < d) ev[t] = ce[t0 + t];
#pragma unroll
                    for (int t = 0; t < DCM; ++t)
                        if (t < d) c[t] = c2v[vcsc ? ev[t] : t0 + t];  // CSC order: contiguous
#pragma unroll
                    for (int t = 0; t < DCM; ++t)
                        if (t < d) {
                            pre[t] = acc;
                            acc += c[t];
                        }
                    xh[j] = acc <= (T)0;
                    if (xb) {
                        const uint64_t w = __ballot(acc <= (T)0);
                        if ((tid & 63) == 0) xbits[j >> 6] = w;
                    }
                    T suf = (T)0;
#pragma unroll
                    for (int t = DCM - 1; t >= 0; --t)
                        if (t < d) {
                            v2c[vcsc ? t0 + t : ev[t]] = pre[t] + suf;
                            suf += c[t];
                        }
                } else if constexpr (METHOD == 1) {
                    for (int t = t0; t < t1; ++t) {
                        const int e = ce[t];
                        v2c[e] = acc;
                        acc += c2v[e];
                    }
                    xh[j] = acc <= (T)0;
                    T suf = (T)0;
                    for (int t = t1 - 1; t >= t0; --t) {
                        const int e = ce[t];
                        v2c[e] = v2c[e] + suf;
                        suf += c2v[e];
                    }
                } else if constexpr (DCM > 0) {
                    // product-sum, unrolled (NaN guards as in the generic loop)
                    const int d = t1 - t0;
                    int ev[DCM];
                    T c[DCM], pre[DCM];
#pragma unroll
                    for (int t = 0; t < DCM; ++t)
                        if (t < d) ev[t] = ce[t0 + t];
#pragma unroll
                    for (int t = 0; t < DCM; ++t)
                        if (t < d) c[t] = c2v[t0 + t];  // CSC order: contiguous
#pragma unroll
                    for (int t = 0; t < DCM; ++t)
                        if (t < d) {
                            pre[t] = acc;
                            acc *= c[t];
                            if (isnan(acc)) acc = (T)1;
                        }
                    xh[j] = acc >= (T)1;
                    if (xb) {
                        const uint64_t w = __ballot(acc >= (T)1);
                        if ((tid & 63) == 0) xbits[j >> 6] = w;
                    }
                    T suf = (T)1;
#pragma unroll
                    for (int t = DCM - 1; t >= 0; --t)
                        if (t < d) {
                            v2c[ev[t]] = pre[t] * suf;
                            suf *= c[t];
                            if (isnan(suf)) suf = (T)1;
                        }
                } else {
                    for (int t = t0; t < t1; ++t) {
                        const int e = ce[t];
                        v2c[e] = acc;
                        acc *= c2v[e];
                        if (isnan(acc)) acc = (T)1;
                    }
                    xh[j] = acc >= (T)1;
                    T suf = (T)1;
                    for (int t = t1 - 1; t >= t0; --t) {
                        const int e = ce[t];
                        v2c[e] = v2c[e] * suf;
                        suf *= c2v[e];
                        if (isnan(suf)) suf = (T)1;
                    }
                }
            }
            __syncthreads();
            int bad = 0;
            for (int i = tid; i < m; i += kBlock) {
                int par = sb[i];
                if constexpr (DRM > 0) {
                    const int e0 = rp[i], d = rp[i + 1] - e0;
                    int cc[DRM];
#pragma unroll
                    for (int t = 0; t < DRM; ++t)
                        if (t < d) cc[t] = ci[e0 + t];
#pragma unroll
                    for (int t = 0; t < DRM; ++t)
                        if (t < d) par ^= xb ? (int)((xbits[cc[t] >> 6] >> (cc[t] & 63)) & 1ull) : (int)xh[cc[t]];
                } else {
                    for (int e = rp[i]; e < rp[i + 1]; ++e) par ^= xh[ci[e]];
                }
                rs[i] = (uint8_t)par;
                bad |= par;
            }
            if (!__syncthreads_or(bad)) {
                conv = true;
                break;
            }
        }
        const int iters = conv ? it : a.max_iter;
        if (tid == 0 && a.iters) a.iters[shot] = iters;
        if (a.llr_out) {  // soft output of the last iteration, same summation order
            T* lo = reinterpret_cast<T*>(a.llr_out);
            for (int j = tid; j < n; j += kBlock) {
                T acc = prior[j];
                for (int t = cp[j]; t < cp[j + 1]; ++t) {
                    if constexpr (METHOD == 1) {
                        acc += c2v[(kCsc && !vcsc) ? t : ce[t]];
                    } else {
                        acc *= c2v[kCsc ? t : ce[t]];
                        if (isnan(acc)) acc = (T)1;
                    }
                }
                if constexpr (METHOD == 1) lo[shot * n + j] = acc;
                else lo[shot * n + j] = (T)log((double)((T)1 / acc));
            }
        }
        if (DEFER && !conv) {
            if (tid == 0) *slot_s = atomicAdd(a.q_count, 1);
            __syncthreads();
            const int slot = *slot_s;
            for (int j = tid; j < n; j += kBlock) a.q_x[(int64_t)slot * n + j] = xh[j];
            for (int i = tid; i < m; i += kBlock) a.q_r[(int64_t)slot * m + i] = rs[i];
            if (tid == 0) a.q_idx[slot] = shot;
            __syncthreads();
        } else {
            finalize_block(g, a, shot, xh, conv, conv, 0, lpar);
        }
    }
}

// Small-set-flip for queued shots, one workgroup per shot; generator gi is
// scanned by thread gi % 256.  Same keys as ssf_wave_kernel.
// gstate: when non-null, the shot state (xh, sres, lpar) of workgroup b lives at
// gstate + b * block_state_stride(g) in HBM instead of LDS (graphs whose state
// exceeds the LDS budget, e.g. the 1.2*10^5-column spacetime graph of config 5).
__host__ __device__ inline size_t block_state_stride(const DevGraph& g) {
    return (block_small_lds(g) + 255) / 256 * 256;
}

__global__ __launch_bounds__(kBlock) void ssf_block_kernel(DevGraph g, DecodeArgs a, unsigned char* gstate) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    long long* redl = reinterpret_cast<long long*>(smem);
    int* redi = reinterpret_cast<int*>(smem + 32);
    uint8_t* xh = gstate ? gstate + (size_t)blockIdx.x * block_state_stride(g) : smem + kCtrl;  // [n_pad]
    uint8_t* sres = xh + g.n_pad;     // [m_pad]
    int* lpar = reinterpret_cast<int*>(sres + g.m_pad);  // [k]
    const int tid = threadIdx.x, m = g.m, n = g.n;
    const int count = *a.q_count;
    const int nhi = g.g_wmax > 4 ? (1 << (g.g_wmax - 4)) : 1;
    for (int slot = blockIdx.x; slot < count; slot += gridDim.x) {
        // queue entries of the shot-lane kernel carry its BP-converged bit in bit 62
        const int64_t qv = a.q_idx[slot];
        const int64_t shot = qv & ((1ll << 62) - 1);
        const bool bp_conv = (qv >> 62) & 1;
        // the queued hard decision and residual, eight loads in flight per
        // thread before any LDS store (a loop of single byte loads waited for
        // each one: ~40 HBM round trips per shot at n = 10^4)
        copy_bytes8(a.q_x + (int64_t)slot * n, xh, n, tid);
        int wl = copy_bytes8(a.q_r + (int64_t)slot * m, sres, m, tid);
        int sw = block_sum_i32(wl, redi);  // includes a barrier: LDS fills visible
        int steps = 0;
        while (a.ssf && sw > 0 && (a.ssf_max_steps <= 0 || steps < a.ssf_max_steps)) {
            long long best = LLONG_MIN;
            for (int gi = tid; gi < g.n_gen; gi += kBlock) {
                const int nlc = g.g_nlc[gi];
                uint32_t sl = 0;
                for (int c = 0; c < nlc; ++c) sl |= (uint32_t)sres[g.g_lc[c * g.g_pad + gi]] << c;
                if (sl == 0) continue;
                uint32_t qm[kGenW];
#pragma unroll
                for (int k = 0; k < kGenW; ++k) qm[k] = g.g_qmask[k * g.g_pad + gi];
                best = max(best, gen_key64(gen_best_key(sl, qm, nhi), gi));
            }
            best = block_max_i64(best, redl);
            const int score = (int)(best >> 32);
            if (best == LLONG_MIN || score <= 0) break;
            const int gsel = 0xFFFFFF - (int)((best >> 8) & 0xFFFFFF);
            const int tsel = 255 - (int)(best & 255);
            const int gain = score * __builtin_popcount(tsel) / kSsfScale;
            const int w = g.g_w[gsel];
            uint32_t mask = 0;
            for (int k = 0; k < w; ++k)
                if ((tsel >> k) & 1) mask ^= g.g_qmask[k * g.g_pad + gsel];
            if (tid < g.g_nlc[gsel] && ((mask >> tid) & 1)) sres[g.g_lc[tid * g.g_pad + gsel]] ^= 1;
            if (tid < w && ((tsel >> tid) & 1)) xh[g.g_q[tid * g.g_pad + gsel]] ^= 1;
            __syncthreads();
            sw -= gain;
            ++steps;
        }
        finalize_block(g, a, shot, xh, bp_conv, sw == 0, steps, lpar);
    }
}

// Incremental small-set-flip for queued shots (same spec and keys as
// ssf_block_kernel, one workgroup per shot): every generator's local syndrome
// and best key are cached in LDS, and a step only re-scores the generators
// whose local syndrome it changed (found through the check -> generator inverse
// table g_iptr / g_ient), instead of re-gathering and re-scoring all of them.
// Key (int32): score << 13 | (8191 - g), so a signed max picks the highest
// score, then the lowest g; the lowest subset reaching that score is found
// afterwards by wave 0 (as in ssf_wave_kernel).
//   LDS: ctrl | key[g_pad] i32 | slg[g_pad] u32 | dlist[g_pad] u16 | dbits
//        [g_pad/32] | xh[n_pad] | sres[m_pad] | lpar[k]
__host__ __device__ inline size_t ssf_inc_lds(const DevGraph& g) {
    const size_t gp = (size_t)g.g_pad;
    return kCtrl + gp * 4 + gp * 4 + (gp * 2 + 15) / 16 * 16 + ((gp + 31) / 32 * 4 + 15) / 16 * 16 +
           ((size_t)g.n_pad + 15) / 16 * 16 + ((size_t)g.m_pad + 15) / 16 * 16 +
           (4 * (size_t)(g.k > 0 ? g.k : 1) + 15) / 16 * 16 + ((size_t)g.n_data + 15) / 16 * 16;
}

__global__ __launch_bounds__(kBlock) void ssf_inc_block_kernel(DevGraph g, DecodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    long long* redl = reinterpret_cast<long long*>(smem);
    int* redi = reinterpret_cast<int*>(smem + 32);
    int* ctl = reinterpret_cast<int*>(smem + 48);  // [0] dirty count, [1] chosen subset
    const size_t gp = (size_t)g.g_pad;
    int* key = reinterpret_cast<int*>(smem + kCtrl);
    uint32_t* slg = reinterpret_cast<uint32_t*>(key + gp);
    uint16_t* dlist = reinterpret_cast<uint16_t*>(slg + gp);
    uint32_t* dbits = reinterpret_cast<uint32_t*>(reinterpret_cast<unsigned char*>(dlist) + (gp * 2 + 15) / 16 * 16);
    uint8_t* xh = reinterpret_cast<uint8_t*>(dbits) + ((gp + 31) / 32 * 4 + 15) / 16 * 16;
    uint8_t* sres = xh + ((size_t)g.n_pad + 15) / 16 * 16;
    int* lpar = reinterpret_cast<int*>(sres + ((size_t)g.m_pad + 15) / 16 * 16);
    uint8_t* rdl = reinterpret_cast<uint8_t*>(lpar) + (4 * (size_t)(g.k > 0 ? g.k : 1) + 15) / 16 * 16;
    const int tid = threadIdx.x, m = g.m, n = g.n, ng = g.n_gen, nd = g.n_data;
    const int count = *a.q_count;
    // whole rows by 16-B loads, every load of a shot issued before the first LDS
    // store, when the rows allow (16-B multiples at 16-B aligned bases, <= kRowU
    // loads per thread): the byte rounds of copy_bytes8 (8 bytes of a thread's
    // share per HBM round trip) made the rows' loads ~8 dependent round trips
    // per shot at n = 10^4.  The readout row goes to LDS too (finalize_block).
    constexpr int kRowU = 3;
    const bool want_rd = a.fail && a.readout && g.k > 0;
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    const bool vec = ((n | m | (want_rd ? nd : 0)) & 15) == 0 && al16(a.q_x) && al16(a.q_r) &&
                     (!want_rd || al16(a.readout)) && n <= 16 * kRowU * kBlock && m <= 16 * kRowU * kBlock &&
                     nd <= 16 * kRowU * kBlock;
    const int nhi = g.g_wmax > 4 ? (1 << (g.g_wmax - 4)) : 1;
    for (int w = tid; w < (int)((gp + 31) / 32); w += kBlock) dbits[w] = 0u;
    if (tid == 0) ctl[0] = 0;
    // table scoring (DevGraph::s_lut, ssf_lut_tables): a generator's best
    // (score, subset) is one lookup on its local syndrome; the key then carries
    // the score's rank, which orders like the score
    const bool lut = g.s_lut && g.opt_ssf == kSsfAuto;
    auto rescore = [&](int gi) {
        const uint32_t sl = slg[gi];
        if (sl == 0u) {
            key[gi] = INT_MIN;
            return;
        }
        if (lut) {
            const uint32_t r = g.s_lut[g.s_off[gi] + sl] >> 24;
            key[gi] = r ? (int)((r << 13) | (uint32_t)(8191 - gi)) : INT_MIN;
            return;
        }
        uint32_t qm[kGenW];
#pragma unroll
        for (int k = 0; k < kGenW; ++k) qm[k] = g.g_qmask[k * gp + gi];
        key[gi] = (int)((unsigned)gen_best_score(sl, qm, nhi) << 13) | (8191 - gi);
    };
    for (int slot = blockIdx.x; slot < count; slot += gridDim.x) {
        const int64_t qv = a.q_idx[slot];
        const int64_t shot = qv & ((1ll << 62) - 1);
        const bool bp_conv = (qv >> 62) & 1;
        // the queued hard decision and residual, eight loads in flight per
        // thread before any LDS store (a loop of single byte loads waited for
        // each one: ~40 HBM round trips per shot at n = 10^4)
        int wl = 0;
        if (vec) {
            uint4 vx[kRowU], vr[kRowU], vd[kRowU];
            const uint4 z = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
            for (int u = 0; u < kRowU; ++u) {
                const int j = (u * kBlock + tid) * 16;
                vx[u] = j < n ? *reinterpret_cast<const uint4*>(a.q_x + (int64_t)slot * n + j) : z;
                vr[u] = j < m ? *reinterpret_cast<const uint4*>(a.q_r + (int64_t)slot * m + j) : z;
                vd[u] = (want_rd && j < nd) ? *reinterpret_cast<const uint4*>(a.readout + shot * nd + j) : z;
            }
#pragma unroll
            for (int u = 0; u < kRowU; ++u) {
                const int j = (u * kBlock + tid) * 16;
                if (j < n) *reinterpret_cast<uint4*>(xh + j) = vx[u];
                if (j < m) {
                    *reinterpret_cast<uint4*>(sres + j) = vr[u];
                    // bytes are 0 / 1: the bit count is the byte sum
                    wl += __builtin_popcount(vr[u].x) + __builtin_popcount(vr[u].y) + __builtin_popcount(vr[u].z) +
                          __builtin_popcount(vr[u].w);
                }
                if (want_rd && j < nd) *reinterpret_cast<uint4*>(rdl + j) = vd[u];
            }
        } else {
            copy_bytes8(a.q_x + (int64_t)slot * n, xh, n, tid);
            wl = copy_bytes8(a.q_r + (int64_t)slot * m, sres, m, tid);
        }
        int sw = block_sum_i32(wl, redi);  // includes a barrier: LDS fills visible
        int steps = 0;
        if (a.ssf && sw > 0) {
            for (int gi = tid; gi < ng; gi += kBlock) {
                const int nlc = g.g_nlc[gi];
                uint32_t sl = 0;
                for (int c = 0; c < nlc; ++c) sl |= (uint32_t)sres[g.g_lc[c * gp + gi]] << c;
                slg[gi] = sl;
                rescore(gi);
            }
            __syncthreads();
            while (sw > 0 && (a.ssf_max_steps <= 0 || steps < a.ssf_max_steps)) {
                long long best = LLONG_MIN;
                for (int gi = tid; gi < ng; gi += kBlock) best = max(best, (long long)key[gi]);
                best = block_max_i64(best, redl);
                const int kv = (int)best;
                const int score = kv >> 13;
                if (best == LLONG_MIN || kv == INT_MIN || score <= 0) break;
                const int gsel = 8191 - (kv & 8191);
                const int w = g.g_w[gsel];
                if (lut) {  // the table entry names the subset and the local checks it toggles
                    if (tid == 0) {
                        const uint32_t sl = slg[gsel];
                        const uint32_t e = g.s_lut[g.s_off[gsel] + sl];
                        ctl[1] = (int)(e & 0xffu);
                        ctl[2] = __builtin_popcount(sl) - __builtin_popcount(sl ^ ((e >> 8) & 0xffffu));  // gain
                    }
                } else if (tid < 64) {  // wave 0: the lowest subset reaching the score
                    const uint32_t sl = slg[gsel];
                    const int base = __builtin_popcount(sl);
                    uint32_t qs[kGenW];
#pragma unroll
                    for (int k = 0; k < kGenW; ++k) qs[k] = g.g_qmask[k * gp + gsel];
                    int tsel = -1;
                    for (int t0 = 0; t0 < 16 * nhi; t0 += 64) {
                        const int t = t0 + tid;
                        uint32_t mt = 0;
#pragma unroll
                        for (int k = 0; k < kGenW; ++k) mt ^= ((t >> k) & 1) ? qs[k] : 0u;
                        const int gain = base - __builtin_popcount(sl ^ mt);
                        const bool hit = t > 0 && t < 16 * nhi && gain * kSsfScale == score * __builtin_popcount(t);
                        const unsigned long long hb = __ballot(hit);
                        if (hb) {
                            tsel = t0 + __builtin_ctzll(hb);
                            break;
                        }
                    }
                    if (tid == 0) ctl[1] = tsel;
                }
                __syncthreads();
                const int tsel = ctl[1];
                if (tsel <= 0) break;  // unreachable: the best score is some subset's score
                uint32_t mask = 0;
                for (int k = 0; k < w; ++k)
                    if ((tsel >> k) & 1) mask ^= g.g_qmask[k * gp + gsel];
                // (read before any thread's flip below changes slg: set by tid 0
                // before the barrier)
                const int gain = lut ? ctl[2] : score * __builtin_popcount(tsel) / kSsfScale;
                // flip: residual, hard decision, and every generator's local syndrome
                // bit of each flipped check (those generators are queued for re-scoring)
                if (tid < g.g_nlc[gsel] && ((mask >> tid) & 1)) {
                    const int c = g.g_lc[tid * gp + gsel];
                    sres[c] ^= 1;
                    for (int e = g.g_iptr[c]; e < g.g_iptr[c + 1]; ++e) {
                        const uint32_t ent = g.g_ient[e];
                        const int g2 = (int)(ent & 0xffffu);
                        atomicXor(&slg[g2], 1u << (ent >> 16));
                        const uint32_t bit = 1u << (g2 & 31);
                        if (!(atomicOr(&dbits[g2 >> 5], bit) & bit)) dlist[atomicAdd(&ctl[0], 1)] = (uint16_t)g2;
                    }
                }
                if (tid < w && ((tsel >> tid) & 1)) xh[g.g_q[tid * gp + gsel]] ^= 1;
                __syncthreads();
                const int nd = ctl[0];
                for (int d = tid; d < nd; d += kBlock) {
                    const int g2 = dlist[d];
                    dbits[g2 >> 5] = 0u;  // whole word: every generator in it is being re-scored or clean
                    rescore(g2);
                }
                __syncthreads();
                if (tid == 0) ctl[0] = 0;
                sw -= gain;
                ++steps;
            }
        }
        finalize_block(g, a, shot, xh, bp_conv, sw == 0, steps, lpar, vec && want_rd ? rdl : nullptr);
    }
}

// ---------------------------------------------------------------- slot-group BP
// BP for graphs whose messages do not fit LDS (configs 4 and 5: 10^4 to 1.3*10^5
// columns), laid out so every HBM access of the message loops is a whole
// cache line.  A workgroup of grp_waves<T>() waves decodes a group of 64 shot slots
// together: lane l of every wave works on slot l.  The group owns a scratch
// block in HBM:
//   v2c [E][64] T   messages by CSR edge, slot-minor: a wave reading edge e of
//                   its 64 slots reads one contiguous 256-B (fp32) / 512-B run
//   c2v [E][64] T   by CSC position (the column pass reads it sequentially)
//   sw  [m]  u64    syndrome bit of check i for every slot (bit l = slot l)
//   xw  [n]  u64    hard decision of column j for every slot (one ballot)
//   pw  [m]  u64    parity of check i under the hard decision (residual words)
//   rw  [n_data] u64  residual readout ^ corr of slots being finalised
// Per iteration: check pass (waves split the checks, UC checks per step with
// all their loads issued first), barrier, column pass (waves split the
// columns), barrier, syndrome test (lanes split the checks: each lane xors the
// 64-slot hard-decision words of its row, so one pass tests all 64 slots),
// barrier.  Slots whose shot converged or reached max_iter are finalised
// (or queued for SSF) and refilled at once from a group-aggregated atomic
// counter, so a slot's work is its own shot's iteration count.  Refilling
// writes no messages: a slot's first check pass reads its columns' priors
// instead of v2c (the same values ldpc initialises the messages to), and its
// syndrome bits go into sw in one coalesced sweep per refill batch.
// Outputs of a finished slot come from the words: corr = base ^ xor of the
// fold blocks' words, fail = any logical's parity over its CSR support of the
// residual words (64 slots per gather), x as bytes; BP-unconverged shots go
// to the SSF queue (bytes, as the other BP kernels write it) when SSF is on.
// Arithmetic is bp_block_kernel's unrolled loops, operation for operation
// (min-sum: med3/fmin row minimum and ldpc's column prefix/suffix sums;
// product-sum: ldpc's forward/backward products and NaN guards), with alpha_t
// of the slot's own iteration.  HBM traffic per shot-iteration: the 16*E-byte
// message model (fp32; 32*E fp64) plus O(m + n) bytes of words.
// Waves per group: 4 for f32 (a 4-wave group fits 3 waves per SIMD, i.e. three
// groups per CU: +30 % on config 5 against 8-wave groups), 8 for f64 (register
// bound at 2 waves per SIMD either way; 8-wave groups finish and refill slots
// with twice the threads: config 4 f64 at p = 0.005, 2.9 iterations per shot,
// 604 k vs 401 k shots/s).
template <typename T>
constexpr int grp_waves() {
    return sizeof(T) == 4 ? 4 : 8;
}
// Checks / columns per wave step: every load of a step is issued before any is
// used, so a wave keeps UC * DR (check pass) or UV * (column degree) loads of
// whole 64-slot lines in flight; the column pass has few edges per column, so
// it takes more columns per step.
template <typename T, int DR>
constexpr int grp_uc() {
    return sizeof(T) == 4 ? 4 : (DR <= 8 ? 4 : 2);
}
template <typename T, int DC>
constexpr int grp_uv() {
    return sizeof(T) == 4 ? (DC <= 4 ? 16 : 8) : (DC <= 4 ? 8 : 4);
}
constexpr int kLzTGrp = 16;           // logical-parity words per slot in the group kernel (k <= 512)
constexpr int kFinPerCu = 8;          // SSF/finalize workgroups per CU when their state is in HBM
constexpr size_t kGrpHeader = 256;    // scratch header: the shot counter

struct GroupLayout {  // byte offsets inside one group's scratch block
    size_t v2c, c2v, sw, xw, pw, rw, total;
};

__host__ __device__ inline size_t grp_round(size_t b) { return (b + 255) / 256 * 256; }

__host__ __device__ inline GroupLayout group_layout(const DevGraph& g, size_t tsz) {
    GroupLayout L;
    L.v2c = 0;
    L.c2v = L.v2c + grp_round(((size_t)g.E + kEdgePad) * 64 * tsz);
    L.sw = L.c2v + grp_round(((size_t)g.E + kEdgePad) * 64 * tsz);
    L.xw = L.sw + grp_round((size_t)g.m * 8);
    L.pw = L.xw + grp_round((size_t)g.n * 8);
    L.rw = L.pw + grp_round((size_t)g.m * 8);
    L.total = L.rw + grp_round((size_t)g.n_data * 8);
    return L;
}

__device__ __forceinline__ int64_t readlane64(int64_t v, int l) {
    const int lo = __builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const int hi = __builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

template <typename T, int METHOD, int DR, int DC>
__global__ __launch_bounds__(64 * grp_waves<T>()) void bp_group_kernel(DevGraph g, DecodeArgs a, unsigned char* scratch,
                                                               size_t group_bytes,
                                                               const int32_t* __restrict__ rp,
                                                               const int32_t* __restrict__ ci,
                                                               const int32_t* __restrict__ cp,
                                                               const int32_t* __restrict__ ce,
                                                               const int32_t* __restrict__ ecs,
                                                               const T* __restrict__ prior,
                                                               const T* __restrict__ ep) {
    constexpr int kGrpWaves = grp_waves<T>(), kGrpThreads = 64 * kGrpWaves;
    __shared__ unsigned long long s_bad, s_fail;
    __shared__ long long s_base;
    __shared__ int s_qbase;
    // per slot the logical-parity words of its residual (DevGraph::lz_t)
    __shared__ uint32_t s_lp[64 * kLzTGrp];
    // wave index as a scalar: the graph index loads of the passes are scalar loads
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), tid = threadIdx.x;
    const int m = g.m, n = g.n, nd = g.n_data;
    const GroupLayout L = group_layout(g, sizeof(T));
    unsigned long long* counter = reinterpret_cast<unsigned long long*>(scratch);
    unsigned char* blk = scratch + kGrpHeader + (size_t)blockIdx.x * group_bytes;
    T* v2c = reinterpret_cast<T*>(blk + L.v2c) + lane;
    T* c2v = reinterpret_cast<T*>(blk + L.c2v) + lane;
    uint64_t* sw = reinterpret_cast<uint64_t*>(blk + L.sw);
    uint64_t* xw = reinterpret_cast<uint64_t*>(blk + L.xw);
    uint64_t* pw = reinterpret_cast<uint64_t*>(blk + L.pw);
    uint64_t* rw = reinterpret_cast<uint64_t*>(blk + L.rw);
    const uint64_t below = (1ull << lane) - 1ull;
    const bool want_fail = a.fail && a.readout && g.k > 0;
    const bool lzcols = want_fail && g.lz_t && g.lz_tw <= kLzTGrp;
    for (int i = tid; i < 64 * kLzTGrp; i += kGrpThreads) s_lp[i] = 0u;  // (the refill's barrier orders it)
    int64_t shot = -1;  // slot `lane`'s shot: identical in every wave (all decisions are group-uniform)
    int it = 0;
    uint64_t need = ~0ull;  // slots to refill (uniform)
    for (;;) {
        if (need) {
            if (tid == 0) s_base = (long long)atomicAdd(counter, (unsigned long long)__popcll(need));
            __syncthreads();
            const long long b0 = s_base;
            if ((need >> lane) & 1) {
                const long long s2 = b0 + __popcll(need & below);
                shot = s2 < a.B ? s2 : -1;
                it = 0;
            }
            const uint64_t live = __ballot(((need >> lane) & 1) && shot >= 0);
            // syndrome words: the refilled slots' bits are replaced in one sweep
            // (per slot l a coalesced read of its shot's syndrome row)
            for (int i = tid; i < m; i += kGrpThreads) {
                uint64_t w = sw[i] & ~need;
                // four slots per round: their loads issued before any is used
                for (uint64_t rem = live; rem;) {
                    int ls[4];
                    uint8_t bv[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        ls[u] = rem ? __builtin_ctzll(rem) : -1;
                        rem &= rem - 1;
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        bv[u] = ls[u] >= 0 ? a.syn[(b0 + __popcll(need & ((1ull << ls[u]) - 1ull))) * m + i] : 0;
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (ls[u] >= 0) w |= (uint64_t)(bv[u] & 1) << ls[u];
                }
                sw[i] = w;
            }
        }
        const bool active = shot >= 0;
        if (!__syncthreads_or(active)) break;
        // every thread read the previous iteration's s_bad before this barrier;
        // the next atomics come two barriers later
        if (tid == 0) s_bad = 0;
        ++it;
        const T alpha = alpha_at<T>(it, a.ms_scaling);
        const bool fresh = it == 1;  // first pass of this slot's shot: v2c = priors
        // Every lane runs the passes, idle slots on garbage, so control flow is
        // wave-uniform: scalar branches, no exec masking.
        constexpr int UC = grp_uc<T, DR>(), UV = grp_uv<T, DC>();
        // Loads first, for the whole step (scalar-guarded by the row / column
        // degree, 32-bit offsets), then the arithmetic with pad positions masked
        // by selects (Big for the row minimum, the neutral factor 1 for the
        // products), so no load waits behind another's use.
        for (int i0 = wv * UC; i0 < m; i0 += kGrpWaves * UC) {  // check pass
            int e0[UC], d[UC], par[UC];
            T mv[UC][DR], pv[UC][DR];
#pragma unroll
            for (int u = 0; u < UC; ++u) {
                const int i = i0 + u;
                const int ii = i < m ? i : m - 1;
                e0[u] = rp[ii];
                d[u] = i < m ? rp[ii + 1] - e0[u] : 0;
            }
#pragma unroll
            for (int u = 0; u < UC; ++u)
#pragma unroll
                for (int t = 0; t < DR; ++t)
                    if (t < d[u]) mv[u][t] = v2c[(uint32_t)(e0[u] + t) * 64u];
#pragma unroll
            for (int u = 0; u < UC; ++u) {
                const int ii = i0 + u < m ? i0 + u : m - 1;
                // sw is written by this kernel: a volatile (vector) load, never the scalar cache
                par[u] = (int)((*(volatile const uint64_t*)&sw[ii] >> lane) & 1ull);
#pragma unroll
                for (int t = 0; t < DR; ++t) pv[u][t] = ep[e0[u] + t];  // padded array: unguarded
            }
#pragma unroll
            for (int u = 0; u < UC; ++u) {
                T v[DR];
#pragma unroll
                for (int t = 0; t < DR; ++t) v[t] = fresh ? pv[u][t] : mv[u][t];
                if constexpr (METHOD == 1) {
                    T m1 = Big<T>::v, m2 = Big<T>::v;
                    int pu = par[u];
#pragma unroll
                    for (int t = 0; t < DR; ++t) {
                        const bool on = t < d[u];
                        const T av = on ? fabs(v[t]) : Big<T>::v;  // Big changes neither minimum
                        m2 = med3(av, m1, m2);
                        m1 = fmin(m1, av);
                        pu ^= on && v[t] <= (T)0;
                    }
                    const T m1a = m1 * alpha, m2a = m2 * alpha;
#pragma unroll
                    for (int t = 0; t < DR; ++t)
                        if (t < d[u]) {
                            const T y = (fabs(v[t]) == m1) ? m2a : m1a;
                            c2v[(uint32_t)ecs[e0[u] + t] * 64u] = (pu ^ (v[t] <= (T)0)) ? -y : y;
                        }
                } else {
                    T r[DR], fw[DR];
                    T f = par[u] ? (T)-1 : (T)1;
#pragma unroll
                    for (int t = 0; t < DR; ++t) {
                        fw[t] = f;
                        r[t] = t < d[u] ? (T)2 / ((T)1 + v[t]) - (T)1 : (T)1;  // pads: the neutral factor
                        f *= r[t];
                    }
                    T b = (T)1;
#pragma unroll
                    for (int t = DR - 1; t >= 0; --t) {
                        if (t < d[u]) {
                            const T c = fw[t] * b;
                            c2v[(uint32_t)ecs[e0[u] + t] * 64u] = ((T)1 - c) / ((T)1 + c);
                        }
                        b *= r[t];
                    }
                }
            }
        }
        __syncthreads();
        for (int j0 = wv * UV; j0 < n; j0 += kGrpWaves * UV) {  // column pass
            int t0[UV], d[UV];
            T c[UV][DC];
#pragma unroll
            for (int u = 0; u < UV; ++u) {
                const int j = j0 + u;
                const int jj = j < n ? j : n - 1;
                t0[u] = cp[jj];
                d[u] = j < n ? cp[jj + 1] - t0[u] : 0;
            }
#pragma unroll
            for (int u = 0; u < UV; ++u)
#pragma unroll
                for (int t = 0; t < DC; ++t)
                    if (t < d[u]) c[u][t] = c2v[(uint32_t)(t0[u] + t) * 64u];  // CSC order: contiguous
#pragma unroll
            for (int u = 0; u < UV; ++u) {
                const int j = j0 + u;
                if (j >= n) break;
                T pre[DC];
                T acc = prior[j];
                bool hard;
                if constexpr (METHOD == 1) {
#pragma unroll
                    for (int t = 0; t < DC; ++t) {
                        pre[t] = acc;
                        acc = t < d[u] ? acc + c[u][t] : acc;
                    }
                    hard = acc <= (T)0;
                } else {
#pragma unroll
                    for (int t = 0; t < DC; ++t) {
                        pre[t] = acc;
                        T x = acc * c[u][t];
                        if (isnan(x)) x = (T)1;
                        acc = t < d[u] ? x : acc;
                    }
                    hard = acc >= (T)1;
                }
                const uint64_t hw = __ballot(hard);
                if (lane == 0) xw[j] = hw;
                if (a.llr_out && active) {
                    T* lo = reinterpret_cast<T*>(a.llr_out);
                    if constexpr (METHOD == 1) lo[shot * n + j] = acc;
                    else lo[shot * n + j] = (T)log((double)((T)1 / acc));
                }
                if constexpr (METHOD == 1) {
                    T suf = (T)0;
#pragma unroll
                    for (int t = DC - 1; t >= 0; --t)
                        if (t < d[u]) {
                            v2c[(uint32_t)ce[t0[u] + t] * 64u] = pre[t] + suf;
                            suf += c[u][t];
                        }
                } else {
                    T suf = (T)1;
#pragma unroll
                    for (int t = DC - 1; t >= 0; --t)
                        if (t < d[u]) {
                            v2c[(uint32_t)ce[t0[u] + t] * 64u] = pre[t] * suf;
                            suf *= c[u][t];
                            if (isnan(suf)) suf = (T)1;
                        }
                }
            }
        }
        __syncthreads();
        {  // syndrome test: lane-parallel over checks, 64 slots per word
            uint64_t bad = 0;
            for (int i = tid; i < m; i += kGrpThreads) {
                const int e0 = rp[i], d = rp[i + 1] - e0;
                uint64_t p = sw[i];
                int cc[DR];
#pragma unroll
                for (int t = 0; t < DR; ++t)
                    if (t < d) cc[t] = ci[e0 + t];
#pragma unroll
                for (int t = 0; t < DR; ++t)
                    if (t < d) p ^= xw[cc[t]];
                pw[i] = p;
                bad |= p;
            }
            if (bad) atomicOr(&s_bad, (unsigned long long)bad);
        }
        __syncthreads();
        const uint64_t anybad = s_bad;
        const bool conv = active && !((anybad >> lane) & 1ull);
        const bool done = conv || (active && it >= a.max_iter);
        const uint64_t D = __ballot(done);
        need = D;
        if (!D) continue;
        const uint64_t C = __ballot(conv);
        const uint64_t Q = a.ssf ? (D & ~C) : 0ull;  // BP-unconverged shots -> the SSF queue
        const uint64_t F = D & ~Q;                   // finalised here
        if (wv == 0 && done && a.iters) a.iters[shot] = it;
        if (Q) {
            if (tid == 0) s_qbase = atomicAdd(a.q_count, __popcll(Q));
            __syncthreads();
            const int qb = s_qbase;
            if (wv == 0 && ((Q >> lane) & 1)) a.q_idx[qb + __popcll(Q & below)] = shot;
            for (int j = tid; j < n; j += kGrpThreads) {
                const uint64_t w = xw[j];
                int r = 0;
                for (uint64_t rem = Q; rem; rem &= rem - 1, ++r)
                    a.q_x[(int64_t)(qb + r) * n + j] = (uint8_t)((w >> __builtin_ctzll(rem)) & 1ull);
            }
            for (int i = tid; i < m; i += kGrpThreads) {
                const uint64_t w = pw[i];
                int r = 0;
                for (uint64_t rem = Q; rem; rem &= rem - 1, ++r)
                    a.q_r[(int64_t)(qb + r) * m + i] = (uint8_t)((w >> __builtin_ctzll(rem)) & 1ull);
            }
        }
        if (F) {
            if (a.x_out)
                for (int j = tid; j < n; j += kGrpThreads) {
                    const uint64_t w = xw[j];
                    for (uint64_t rem = F; rem; rem &= rem - 1) {
                        const int l = __builtin_ctzll(rem);
                        a.x_out[readlane64(shot, l) * n + j] = (uint8_t)((w >> l) & 1ull);
                    }
                }
            if (a.corr_out || want_fail) {
                for (int q = tid; q < nd; q += kGrpThreads) {
                    uint64_t cw = 0;
                    for (int b = 0; b < g.fold_blocks; ++b) cw ^= xw[b * nd + q];
                    uint64_t rword = 0;
                    // four finishing slots per round, loads first
                    for (uint64_t rem = F; rem;) {
                        int ls[4];
                        int64_t sls[4];
                        uint8_t bb[4], rb[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            ls[u] = rem ? __builtin_ctzll(rem) : -1;
                            rem &= rem - 1;
                            sls[u] = ls[u] >= 0 ? readlane64(shot, ls[u]) : 0;
                        }
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            bb[u] = (ls[u] >= 0 && a.base) ? a.base[sls[u] * nd + q] : 0;
                            rb[u] = (ls[u] >= 0 && want_fail) ? a.readout[sls[u] * nd + q] : 0;
                        }
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            if (ls[u] < 0) continue;
                            const int cb = (int)((cw >> ls[u]) & 1ull) ^ (bb[u] & 1);
                            if (a.corr_out) a.corr_out[sls[u] * nd + q] = (uint8_t)cb;
                            if (want_fail) rword |= (uint64_t)((rb[u] ^ cb) & 1) << ls[u];
                        }
                    }
                    if (lzcols) {  // the residual's ones XOR their qubit's parity words into their slots'
                        if (rword)
                            for (int t = 0; t < g.lz_tw; ++t) {
                                const uint32_t v = g.lz_t[(size_t)q * g.lz_tw + t];
                                if (v)
                                    for (uint64_t rem = rword; rem; rem &= rem - 1)
                                        atomicXor(&s_lp[__builtin_ctzll(rem) * kLzTGrp + t], v);
                            }
                    } else if (want_fail) {
                        rw[q] = rword;
                    }
                }
            }
            if (lzcols) {
                __syncthreads();  // parity words complete
                if (wv == 0) {
                    uint32_t o = 0;
                    for (int t = 0; t < g.lz_tw; ++t) {
                        o |= s_lp[lane * kLzTGrp + t];
                        s_lp[lane * kLzTGrp + t] = 0u;
                    }
                    const uint64_t fb = __ballot(o != 0u);
                    if (lane == 0) s_fail = fb & F;
                }
                __syncthreads();
            } else if (want_fail) {
                if (tid == 0) s_fail = 0;
                __syncthreads();  // rw complete
                uint64_t fm = 0;
                for (int r = tid; r < g.k; r += kGrpThreads) {
                    uint64_t p = 0;
                    const int t1 = g.lz_ptr[r + 1];
                    int t = g.lz_ptr[r];
                    for (; t + 4 <= t1; t += 4) {  // four supports per round, loads first
                        int q4[4];
                        uint64_t v4[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) q4[u] = g.lz_idx[t + u];
#pragma unroll
                        for (int u = 0; u < 4; ++u) v4[u] = rw[q4[u]];
                        p ^= v4[0] ^ v4[1] ^ v4[2] ^ v4[3];
                    }
                    for (; t < t1; ++t) p ^= rw[g.lz_idx[t]];
                    fm |= p;
                }
                if (fm & F) atomicOr(&s_fail, (unsigned long long)(fm & F));
                __syncthreads();
            }
            if (wv == 0 && ((F >> lane) & 1)) {
                if (a.status) a.status[shot] = (uint8_t)(conv ? 3 : 0);
                if (a.ssf_steps) a.ssf_steps[shot] = 0;
                if (a.fail) a.fail[shot] = (uint8_t)(want_fail ? ((s_fail >> lane) & 1ull) : 0);
            }
        }
        __syncthreads();  // every read of s_fail and of the words before the refill
    }
}

// ---------------------------------------------------------------- LDS-resident min-sum BP
// Min-sum BP (fp32) for graphs whose messages spill the small-graph LDS budget
// but whose edge slots alone fit one CU's 160 KB LDS (config 4: m = 4800 rows of
// kMlDRS = 8 floats = 150 KB).  One 1024-thread workgroup per CU decodes one
// shot at a time with every message on chip:
//   rows   [m][kMlDRS] f32: one slot per edge at (row, position); it holds the
//          edge's v2c message between the variable pass and the check pass and
//          its c2v message between the check pass and the variable pass
//   pbuf   two bit arrays of m bits: parity of the hard decision per check,
//          built by the variable pass with LDS xor atomics (only ones touch it)
// Thread t owns checks t + 1024 c and variables t + 1024 r.  Per iteration (2
// barriers):
//   A  check pass: syndrome test of the previous iteration's hard decision
//      (parity bits vs syndrome); each owned row reads its v2c slots (two
//      16-B halves), takes m1 / m2 (minimum and second minimum of |v|, counted
//      with multiplicity), the argmin position and the parity, and writes every
//      slot's c2v: alpha * (m2 at the argmin, m1 elsewhere) with sign parity ^
//      (own v2c <= 0) -- ldpc's leave-one-out minimum and sign, bit for bit
//      (when the minimum is tied m2 = m1, so the argmin's choice is immaterial)
//   B  barrier-or: all checks satisfied -> converged at it - 1
//   C  variable pass: read the c2v slots, prefix / suffix sums (ldpc's order),
//      hard decision, parity xors, and the new v2c written back into the same
//      slots at once (a slot is read and written by its own variable only)
//   D  barrier
// Finished shots go to the SSF queue in the byte format of the other BP kernels (hard
// decision, residual, converged bit); ssf_inc_block_kernel runs SSF and finalises.
// Pad edges (k >= the column's degree, variables j >= n) point at dummy rows
// past row m (element m * kMlDRS + lane, so no two lanes of a wave write the
// same address): they read garbage that the sums mask out and write into them,
// so the loops have no per-edge branches; only real edges xor parity.
constexpr int kMlThreads = 1024;
constexpr int kMlNch = 5;  // check rounds per thread: 32 B of rows per check in 160 KB

constexpr int kMlDummyRows = 64 / kMlDRS;  // pad edges of lane l use element m * kMlDRS + l

__host__ __device__ inline size_t ml_pbuf_words(const DevGraph& g) {
    return ((size_t)g.m + kMlDummyRows + 31) / 32 + 3 & ~(size_t)3;
}
__host__ __device__ inline size_t ml_lds_bytes(const DevGraph& g) {
    return kCtrl + ((size_t)g.m + kMlDummyRows) * kMlDRS * 4 + 2 * 4 * ml_pbuf_words(g) + 2 * 4 * (kMlThreads / 64);
}

// Step A of bp_ms_lds_kernel on row i, in place (v2c slots in, c2v slots out);
// also ml_init_check_kernel's iteration 1 on the image in HBM.
__device__ __forceinline__ void ml_check_row(float* rows, int i, int deg, uint32_t sbit, float alpha) {
    // the row's halves in swizzled order (so = 4 * bit 4 of the row): the 16-B
    // reads of a 16-lane group (banks a/4 mod 64) and the 16-B writes of an
    // 8-lane group (banks a/4 mod 32) then land in distinct 4-bank slots; loaded
    // element u sits at row position u ^ so
    const int so = ((i >> 4) & 1) << 2;
    float v[kMlDRS];
    {
        const float4 h0 = *reinterpret_cast<const float4*>(rows + (size_t)i * kMlDRS + so);
        const float4 h1 = *reinterpret_cast<const float4*>(rows + (size_t)i * kMlDRS + (so ^ 4));
        v[0] = h0.x, v[1] = h0.y, v[2] = h0.z, v[3] = h0.w;
        v[4] = h1.x, v[5] = h1.y, v[6] = h1.z, v[7] = h1.w;
    }
    // sign test by bits: bit 31 of bits(v) - 1 is (v <= 0) for every v but -0,
    // and a v2c message is never -0 (the prior is not, and a sum is -0 only when
    // both terms are)
    float m1 = Big<float>::v, m2 = Big<float>::v;
    int au = 0;  // element index of the argmin
    uint32_t sx = sbit << 31;
    uint32_t sg[kMlDRS];
#pragma unroll
    for (int u = 0; u < kMlDRS; ++u) {
        const float vt = (u ^ so) < deg ? v[u] : Big<float>::v;
        const float av = fabsf(vt);
        au = av < m1 ? u : au;
        m2 = med3(av, m1, m2);
        m1 = med3(av, m1, -Big<float>::v);
        sg[u] = (uint32_t)__float_as_int(vt) - 1u;
        sx ^= sg[u];
    }
    // c2v of every position, in place of its v2c: alpha times the leave-one-out
    // minimum (m2 at the argmin, m1 elsewhere), sign = syndrome ^ the other
    // edges' signs = bit 31 of sx ^ sg[u]
    const float y1 = m1 * alpha, y2 = m2 * alpha;
    float o[kMlDRS];
#pragma unroll
    for (int u = 0; u < kMlDRS; ++u) {
        const float y = u == au ? y2 : y1;
        o[u] = __uint_as_float(__float_as_uint(y) ^ ((sg[u] ^ sx) & 0x80000000u));
    }
    *reinterpret_cast<float4*>(rows + (size_t)i * kMlDRS + so) = make_float4(o[0], o[1], o[2], o[3]);
    *reinterpret_cast<float4*>(rows + (size_t)i * kMlDRS + (so ^ 4)) = make_float4(o[4], o[5], o[6], o[7]);
}

// Iteration 1's c2v rows depend on the priors and, through one sign per row, on
// the syndrome: the image (rows of `ml_lds_bytes`' layout, m x kMlDRS f32 in
// HBM, syndrome bit 0) is built once per launch -- the priors scattered to the
// edge slots, then step A on every row -- and each shot copies it, flipping
// every sign of the rows whose syndrome bit is 1 (step A's sx carries that bit
// into all of a row's signs).  The image's unused row positions are never read
// (step A masks positions >= the degree, and pad edges use the dummy rows).
__host__ __device__ inline size_t ml_image_bytes(const DevGraph& g) { return (size_t)g.m * kMlDRS * 4; }

__global__ __launch_bounds__(256) void ml_init_scatter_kernel(DevGraph g, const uint16_t* __restrict__ etab,
                                                             const float* __restrict__ prior, float* __restrict__ img) {
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= g.n) return;
    const float L = prior[j];
#pragma unroll
    for (int k = 0; k < kMlDC; ++k) {
        const uint32_t e = etab[(size_t)k * g.n + j];
        if (e != 0xffffu) img[e] = L;
    }
}

__global__ __launch_bounds__(256) void ml_init_check_kernel(DevGraph g, float* __restrict__ img, double ms_scaling) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= g.m) return;
    ml_check_row(img, i, g.row_ptr[i + 1] - g.row_ptr[i], 0u, alpha_at<float>(1, ms_scaling));
}

template <int VPT>
__global__ __launch_bounds__(kMlThreads) void bp_ms_lds_kernel(DevGraph g, DecodeArgs a,
                                                              const uint16_t* __restrict__ etab,
                                                              const float* __restrict__ prior,
                                                              const float* __restrict__ img) {
    static_assert(VPT * 3 <= 64 && VPT <= 32, "degree and decision bits");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    long long* next = reinterpret_cast<long long*>(smem + 56);
    float* rows = reinterpret_cast<float*>(smem + kCtrl);
    const int tid = threadIdx.x;
    const int m = g.m, n = g.n;
    const int npw = (m + kMlDummyRows + 31) / 32;
    const uint32_t pbw = (uint32_t)ml_pbuf_words(g);
    uint32_t* pb0 = reinterpret_cast<uint32_t*>(rows + ((size_t)m + kMlDummyRows) * kMlDRS);
    int* flags = reinterpret_cast<int*>(pb0 + 2 * pbw);  // [2][16]
    const uint32_t pad0 = (uint32_t)m * kMlDRS;        // first dummy element
    const uint32_t pad = pad0 + (uint32_t)(tid & 63);  // this lane's (distinct banks, no same-address writes)
    const int ncr = (m - tid + kMlThreads - 1) / kMlThreads;  // checks of this thread (<= 32)
    if (blockIdx.x == 0 && tid == 0) *a.q_count = (int32_t)a.B;

    // per-variable constants: prior, degree, LDS element of each edge (u16 pairs)
    float L[VPT];
    uint32_t ep[VPT][kMlDC / 2];
#pragma unroll
    for (int r = 0; r < VPT; ++r) {
        const int j = r * kMlThreads + tid;
        L[r] = j < n ? prior[j] : 0.0f;
#pragma unroll
        for (int h = 0; h < kMlDC / 2; ++h) {
            uint32_t e0 = pad, e1 = pad;
            if (j < n) {
                e0 = etab[(size_t)(2 * h) * n + j];
                e1 = etab[(size_t)(2 * h + 1) * n + j];
                e0 = e0 == 0xffffu ? pad : e0;
                e1 = e1 == 0xffffu ? pad : e1;
            }
            ep[r][h] = e0 | (e1 << 16);
        }
    }
    auto edge = [&](int r, int k) -> uint32_t { return (ep[r][k >> 1] >> (16 * (k & 1))) & 0xffffu; };
    // Keeps the compiler from hoisting the per-edge addresses, positions and
    // parity masks derived from ep out of the iteration loop (5 live values per
    // edge instead of half a register): they are re-derived where used.
    auto opaque_edges = [&]() {
#pragma unroll
        for (int r = 0; r < VPT; ++r)
#pragma unroll
            for (int h = 0; h < kMlDC / 2; ++h) asm volatile("" : "+v"(ep[r][h]));
    };
    uint64_t djs = 0;  // 3 bits per owned variable: its degree (real edges come first)
#pragma unroll
    for (int r = 0; r < VPT; ++r) {
        int dj = 0;
#pragma unroll
        for (int k = 0; k < kMlDC; ++k) dj += edge(r, k) < pad0;
        djs |= (uint64_t)dj << (3 * r);
    }
    uint32_t rdeg = 0;  // 4 bits per owned check (degrees <= 8), checks c < 8
    for (int c = 0; c < ncr && c < 8; ++c) {
        const int i = c * kMlThreads + tid;
        rdeg |= (uint32_t)(g.row_ptr[i + 1] - g.row_ptr[i]) << (4 * c);
    }

    // The next shot's index is fetched under this shot's syndrome loads and
    // stored behind the barrier below (every thread has read this one by then);
    // the barriers of the shot's iterations order it before the next read.  The
    // syndrome loads of a thread are issued together (kMlNch, clamped, masked),
    // and the barrier orders LDS only, so the last shot's queue stores stay in
    // flight (a __syncthreads would wait for them).
    if (tid == 0) *next = (long long)atomicAdd(a.wave_ctr, 1ull);
    __syncthreads();
    for (;;) {
        const long long sl = *next;  // uniform: held in SGPRs
        const int64_t shot = (int64_t)((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)sl) |
                                       ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(sl >> 32)) << 32));
        if (shot >= a.B) break;
        long long shot_next = 0;
        if (tid == 0) {
            int z = 0;  // opaque offset: keeps the atomic optimiser (which waits at once) off
            asm volatile("" : "+v"(z));
            shot_next = (long long)atomicAdd(a.wave_ctr + z, 1ull);
        }
        int to = tid;
        asm volatile("" : "+v"(to));  // per-shot addresses re-derived, not hoisted and spilled
        uint32_t sb = 0;  // syndrome bits of the owned checks
#pragma unroll
        for (int c = 0; c < kMlNch; ++c) {
            const int i = c * kMlThreads + to;
            sb |= (uint32_t)(a.syn[shot * m + min(i, m - 1)] & (i < m ? 1u : 0u)) << c;
        }
        // iteration 1's c2v rows: the image, signs flipped where the syndrome bit
        // is 1; the parity bits of iteration 1 cleared
#pragma unroll
        for (int c = 0; c < kMlNch; ++c) {
            const int i = c * kMlThreads + to;
            if (i < m) {
                const uint32_t f = ((sb >> c) & 1u) << 31;
                const uint4 h0 = *reinterpret_cast<const uint4*>(img + (size_t)i * kMlDRS);
                const uint4 h1 = *reinterpret_cast<const uint4*>(img + (size_t)i * kMlDRS + 4);
                *reinterpret_cast<uint4*>(rows + (size_t)i * kMlDRS) = make_uint4(h0.x ^ f, h0.y ^ f, h0.z ^ f, h0.w ^ f);
                *reinterpret_cast<uint4*>(rows + (size_t)i * kMlDRS + 4) = make_uint4(h1.x ^ f, h1.y ^ f, h1.z ^ f, h1.w ^ f);
            }
        }
        for (int w = to; w < npw; w += kMlThreads) pb0[pbw + w] = 0u;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        if (tid == 0) *next = shot_next;

        uint32_t xb = 0, bad = 0;  // hard decisions (bit r), failing owned checks (bit c)
        bool conv = false;
        int it = 1;
        for (;; ++it) {
            // ---- A: test of iteration it - 1, then the c2v messages of iteration it
            // (iteration 1's came from the image)
            uint32_t* pcur = pb0 + (it & 1) * pbw;
            if (it > 1) {
                const uint32_t* pprev = pb0 + ((it - 1) & 1) * pbw;
                const bool work = it <= a.max_iter;
                const float alpha = alpha_at<float>(it, a.ms_scaling);
                bad = 0;
                for (int c = 0; c < ncr; ++c) {
                    const int i = c * kMlThreads + tid;
                    bad |= (((pprev[i >> 5] >> (i & 31)) ^ (sb >> c)) & 1u) << c;
                    if (work) {
                        const int deg = c < 8 ? (int)((rdeg >> (4 * c)) & 15u) : (g.row_ptr[i + 1] - g.row_ptr[i]);
                        ml_check_row(rows, i, deg, (sb >> c) & 1u, alpha);
                    }
                }
                if (work)
                    for (int w = tid; w < npw; w += kMlThreads) pcur[w] = 0u;
                // block-wide "any check failing": one flag per wave, double-buffered by
                // iteration parity so one barrier suffices
                int* fl = flags + (it & 1) * (kMlThreads / 64);
                const unsigned long long wb = __ballot(bad != 0u);
                if ((tid & 63) == 0) fl[tid >> 6] = wb != 0ull;
                __syncthreads();
                int any_bad = 0;
#pragma unroll
                for (int w = 0; w < kMlThreads / 64; ++w) any_bad |= fl[w];
                if (!any_bad) {
                    conv = true;
                    break;
                }
                if (!work) break;
            }
            // ---- C: variable pass.  Each edge's slot is read and rewritten by its
            // own variable only (c2v in, new v2c out), so no barrier separates them
            opaque_edges();
            xb = 0;
            // software-pipelined by one variable: the next variable's slots are
            // read before this one's arithmetic (distinct slots, so the order
            // against this variable's writes is immaterial)
            float cn[kMlDC];
#pragma unroll
            for (int k = 0; k < kMlDC; ++k) cn[k] = rows[edge(0, k)];
#pragma unroll
            for (int r = 0; r < VPT; ++r) {
                const int dj = (int)((djs >> (3 * r)) & 7u);  // degree: real edges come first
                float c[kMlDC];
#pragma unroll
                for (int k = 0; k < kMlDC; ++k) c[k] = cn[k];
                if (r + 1 < VPT)
#pragma unroll
                    for (int k = 0; k < kMlDC; ++k) cn[k] = rows[edge(r + 1, k)];
                // ldpc's order: prefix sums from the prior, then each outgoing
                // message = prefix + (sum of the later edges, accumulated from the end)
                float pre[kMlDC];
                float acc = L[r];
#pragma unroll
                for (int k = 0; k < kMlDC; ++k) {
                    pre[k] = acc;
                    acc = k < dj ? acc + c[k] : acc;
                }
                const bool x = acc <= 0.0f;
                xb |= (uint32_t)x << r;
                float suf = 0.0f;
                bool started = false;
#pragma unroll
                for (int k = kMlDC - 1; k >= 0; --k) {
                    const float o = started ? pre[k] + suf : pre[k];
                    suf = started ? suf + c[k] : c[k];
                    started = started || k < dj;
                    rows[edge(r, k)] = o;
                }
                if (x) {
#pragma unroll
                    for (int k = 0; k < kMlDC; ++k) {
                        const uint32_t i = edge(r, k) / kMlDRS;
                        if (k < dj) atomicXor(&pcur[i >> 5], 1u << (i & 31));
                    }
                }
                // two variables' reads in flight at most (otherwise the
                // scheduler hoists all of them and spills)
                __builtin_amdgcn_sched_barrier(0);
            }
            __syncthreads();
        }
        // ---- queue the shot: hard decision, residual syndrome, converged bit
#pragma unroll
        for (int r = 0; r < VPT; ++r) {
            const int j = r * kMlThreads + tid;
            if (j < n) a.q_x[shot * n + j] = (uint8_t)((xb >> r) & 1);
        }
        for (int c = 0; c < ncr; ++c) a.q_r[shot * m + c * kMlThreads + tid] = (uint8_t)((bad >> c) & 1);
        if (tid == 0) {
            a.q_idx[shot] = shot | ((int64_t)(conv ? 1 : 0) << 62);
            if (a.iters) a.iters[shot] = conv ? it - 1 : a.max_iter;
        }
    }
}

// ---------------------------------------------------------------- LDS-resident min-sum BP, f64
// bp_ms_lds_kernel's one-shot-per-CU scheme at ldpc's precision.  The f64 edge
// slots of config 4 (33,600 x 8 B) do not fit the 160 KB LDS, so no message is
// kept there: each variable thread keeps the v2c messages it sent last
// iteration in registers, and the check side is reduced to its min-sum state,
// built by LDS atomics on the IEEE bit patterns (|v| >= +0 orders like an
// unsigned integer, so ds_min_u64 is the exact minimum):
//   m1[b][i], m2[b][i]  u64 bits (two arrays): minimum and second minimum of
//             |v| over the row, with multiplicity (a repeated minimum gives m2 = m1)
//   parw[b]   per check: syndrome ^ parity of (v <= 0) over the row
//   hdw[b]    per check: parity of the hard decision (the syndrome test)
// Both minima come from ONE pass of the messages: each message x does
//   old = ds_min_rtn_u64(m1, x);  ds_min_u64(m2, max(old, x)).
// The updates of m1 are atomic, so they have a total order; with a1 <= a2 <= ...
// the row's sorted values, min over the messages of max(old, x) is a2:
//   >= a2: a message x >= a2 gives max >= a2; a minimum message x = a1 whose old
//          is >= a2 too unless an equal minimum came first (then a2 = a1);
//   <= a2: of the messages holding a1 and a2, the later one sees old <= the
//          other's value, and its max is a2.
// so m2 is the second minimum with multiplicity (kBig for a row of one edge),
// the two-pass construction's value bit for bit, without the second pass over
// the messages and its barrier.
// Buffers alternate by iteration parity b = it & 1.  Per iteration (2 barriers):
//   D  variable pass: c2v of edge (i, v) = alpha * (|v| == m1 ? m2 : m1) with
//      sign parw ^ (v <= 0) -- ldpc's leave-one-out minimum and sign, the same
//      selection as MsCore's and the f32 kernel's -- then ldpc's prefix / suffix
//      sums, the hard decision (xor into hdw[b]), and the new v2c messages'
//      atomics into buffer b ^ 1 (the two minima above, xor of the sign parity)
//   B  syndrome test of hdw[b] (a flag per wave); buffer b reset for iteration
//      it + 2 (every read of it is behind the barrier)
// A v2c message is never -0 (see bp_ms_lds_kernel), so (bits(v) - 1) >> 63 is
// ldpc's (v <= 0).  Finished shots are queued like bp_ms_lds_kernel's.
constexpr int kM64Threads = 1024;
constexpr int kM64Nch = 5;  // check rounds per thread: 32 B of state per check in 160 KB

__host__ __device__ inline size_t m64_words(const DevGraph& g) { return ((size_t)g.m + 31) / 32; }
__host__ __device__ inline size_t m64_lds_bytes(const DevGraph& g) {
    return kCtrl + (size_t)2 * g.m * 16 + 5 * 4 * m64_words(g) + 2 * 4 * (kM64Threads / 64);
}

__device__ __forceinline__ unsigned long long dbits(double x) { return (unsigned long long)__double_as_longlong(x); }

// Iteration 1's check states depend on the priors only (every v2c message of
// column j is its prior): m64_init_kernel builds them once per launch in slot
// order -- m1[m], m2[m] (u64 bits, the row's minimum and second minimum of
// |prior| with multiplicity), then par[W] (u32 words: parity of (prior <= 0) over
// the row) -- and every shot copies them into LDS instead of running the
// message atomics.  The values are those of the atomics (same multiset).
__host__ __device__ inline size_t m64_image_bytes(const DevGraph& g) {
    return (size_t)g.m * 16 + 4 * ((m64_words(g) + 1) / 2 * 2);
}

__global__ __launch_bounds__(256) void m64_init_kernel(DevGraph g, const double* __restrict__ prior,
                                                      const uint16_t* __restrict__ cslot,
                                                      unsigned long long* __restrict__ img) {
    const int s = blockIdx.x * 256 + threadIdx.x, lane = threadIdx.x & 63;
    const unsigned long long kBig = dbits(Big<double>::v);
    unsigned long long m1 = kBig, m2 = kBig;
    uint32_t par = 0;
    if (s < g.m) {
        const int i = cslot[s];
        for (int e = g.row_ptr[i]; e < g.row_ptr[i + 1]; ++e) {
            const unsigned long long pb = dbits(prior[g.col_idx[e]]);
            const unsigned long long x = pb & 0x7fffffffffffffffull;
            par ^= (uint32_t)((pb - 1ull) >> 63);  // (prior <= 0); a prior is never -0
            if (x < m1) {
                m2 = m1;
                m1 = x;
            } else if (x < m2) {
                m2 = x;
            }
        }
        img[s] = m1;
        img[(size_t)g.m + s] = m2;
    }
    const unsigned long long bw = __ballot(par != 0u);
    const int w0 = (s - lane) >> 5;
    uint32_t* pw = reinterpret_cast<uint32_t*>(img + (size_t)2 * g.m);
    if (lane < 2 && w0 + lane < (int)m64_words(g)) pw[w0 + lane] = (uint32_t)(bw >> (32 * lane));
}

// The check states live at host-placed slots (DevGraph::m64_etab / m64_check,
// m64_layout in qdec_abi.cpp: a wave's state accesses spread over the LDS
// banks); every array below is indexed by slot, and the syndrome input and the
// residual output go through cslot (slot -> check).
// D3R: the variable rounds r < D3R hold columns of degree <= 3 only (host:
// DevGraph::m64_d3r), so their messages take 3 registers instead of kMlDC.
template <int VPT, int D3R>
__global__ __launch_bounds__(kM64Threads) void bp_ms_lds64_kernel(DevGraph g, DecodeArgs a,
                                                                 const uint16_t* __restrict__ etab,
                                                                 const double* __restrict__ prior,
                                                                 const uint16_t* __restrict__ cslot,
                                                                 const unsigned long long* __restrict__ img) {
    static_assert(VPT * 3 <= 32 && VPT <= 32 && D3R <= VPT, "degree and decision bits");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    long long* next = reinterpret_cast<long long*>(smem + 56);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int m = g.m, n = g.n;
    const int W = (int)m64_words(g);
    unsigned long long* st = reinterpret_cast<unsigned long long*>(smem + kCtrl);  // m1 [2][m], then m2 [2][m]
    uint32_t* synw = reinterpret_cast<uint32_t*>(smem + kCtrl + (size_t)2 * m * 16);
    uint32_t* parw = synw + W;     // [2][W]
    uint32_t* hdw = parw + 2 * W;  // [2][W]
    int* flags = reinterpret_cast<int*>(hdw + 2 * W);  // [2][16]
    // variable slot of this thread: tid * 67 mod 1024, so the 64 lanes of a wave own
    // columns 67 apart instead of 64 neighbours (neighbouring columns of a
    // hypergraph product share checks, and lanes of one wave hitting one check's
    // state serialise its atomics)
    const int tq = (tid * 67) & (kM64Threads - 1);
    const int ncr = tid < m ? (m - tid + kM64Threads - 1) / kM64Threads : 0;  // checks of this thread
    const unsigned long long kBig = dbits(Big<double>::v);
    constexpr unsigned long long kAbs = 0x7fffffffffffffffull;
    if (blockIdx.x == 0 && tid == 0) *a.q_count = (int32_t)a.B;

    // per-variable constants: degree, check of each edge (u16 pairs); the priors
    // are re-read from global memory (L1) where used, to leave the registers to
    // the messages
    uint32_t ep[VPT][kMlDC / 2];
    uint32_t djs = 0;  // 3 bits per owned variable: its degree (real edges come first)
    // prior of round r's column (a pad slot, j >= n, reads column n - 1: its value
    // only reaches the pad's unused hard decision); tqv is an opaque copy of tq
    // taken per pass, so the column offsets are re-derived where used instead of
    // being held (spilled) across the loop
    auto prior_of = [&](const double* pr, int tqv, int r) -> double {
        return pr[min(r * kM64Threads + tqv, n - 1)];
    };
    auto opaque_tq = [&]() {
        int t = tq;
        asm volatile("" : "+v"(t));
        return t;
    };
    // the same for tid: the per-shot addresses (syndrome, image, queue) are
    // re-derived each shot instead of being hoisted out of the shot loop and spilled
    auto opaque_tid = [&]() {
        int t = tid;
        asm volatile("" : "+v"(t));
        return t;
    };
    // barrier ordering LDS only: global stores (the queue) stay in flight
    auto lds_barrier = []() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    };
#pragma unroll
    for (int r = 0; r < VPT; ++r) {
        const int j = r * kM64Threads + tq;
        int dj = 0;
#pragma unroll
        for (int h = 0; h < kMlDC / 2; ++h) {
            uint32_t e0 = 0xffffu, e1 = 0xffffu;
            if (j < n) {
                e0 = etab[(size_t)(2 * h) * n + j];
                e1 = etab[(size_t)(2 * h + 1) * n + j];
            }
            dj += (e0 != 0xffffu) + (e1 != 0xffffu);
            e0 = e0 == 0xffffu ? 0u : e0;  // state slots (m64_etab)
            e1 = e1 == 0xffffu ? 0u : e1;
            ep[r][h] = e0 | (e1 << 16);
        }
        djs |= (uint32_t)dj << (3 * r);
        __builtin_amdgcn_sched_barrier(0);  // one variable's loads at a time (registers)
    }
    auto chk = [&](int r, int k) -> int { return (int)((ep[r][k >> 1] >> (16 * (k & 1))) & 0xffffu); };
    auto deg = [&](int r) -> int { return (int)((djs >> (3 * r)) & 7u); };
    auto dmax = [](int r) -> int { return r < D3R ? kMlDC - 1 : kMlDC; };  // compile time once unrolled
    // keeps the per-edge addresses from being hoisted out of the loops (as in
    // bp_ms_lds_kernel): they are re-derived from ep where used
    auto opaque_edges = [&]() {
#pragma unroll
        for (int r = 0; r < VPT; ++r)
#pragma unroll
            for (int h = 0; h < kMlDC / 2; ++h) asm volatile("" : "+v"(ep[r][h]));
        asm volatile("" : "+v"(djs));
    };
    // ldpc's (v <= 0) for a v2c message (never -0)
    auto neg = [](double v) -> uint32_t { return (uint32_t)((dbits(v) - 1ull) >> 63); };
    // one new message (magnitude bits x) into the minima of check slot i, buffer nb
    auto put_min = [&](int nb, int i, unsigned long long x) {
        const unsigned long long old = atomicMin(st + (size_t)nb * m + i, x);
        atomicMin(st + (size_t)(2 + nb) * m + i, old > x ? old : x);
    };

    QDEC_STAMP_DECL
    if (tid == 0) *next = (long long)atomicAdd(a.wave_ctr, 1ull);
    __syncthreads();
    for (;;) {
        const long long sl = *next;  // uniform: held in SGPRs
        const int64_t shot = (int64_t)((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)sl) |
                                       ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(sl >> 32)) << 32));
        if (shot >= a.B) break;
        QDEC_STAMP(4);
        QDEC_COUNT(8, 1);
        // the next shot's index, fetched under this shot's syndrome loads (stored
        // behind the barrier below, after every thread has read this one)
        // (an opaque offset keeps the atomic optimiser, which would wait for the
        // result right away, off this single-lane add)
        long long shot_next = 0;
        if (tid == 0) {
            int z = 0;
            asm volatile("" : "+v"(z));
            shot_next = (long long)atomicAdd(a.wave_ctr + z, 1ull);
        }
        const int to = opaque_tid();
        // ---- S: syndrome words (ballots of 64 consecutive slots); buffer 0 reset,
        // buffer 1 = iteration 1's states (img).  The kM64Nch syndrome loads of a
        // thread and its image loads are issued together (clamped index, masked).
        uint32_t sv[kM64Nch], ip[kM64Nch];
        unsigned long long i1[kM64Nch], i2[kM64Nch];
        const uint32_t* ipar = reinterpret_cast<const uint32_t*>(img + (size_t)2 * m);
        const int ln = to & 63, wbase = to & ~63;
#pragma unroll
        for (int c = 0; c < kM64Nch; ++c) {
            const int i = c * kM64Threads + to, ic = min(i, m - 1);
            sv[c] = a.syn[shot * m + cslot[ic]] & (i < m ? 1u : 0u);
            i1[c] = img[ic];
            i2[c] = img[(size_t)m + ic];
            ip[c] = ipar[min(((c * kM64Threads + wbase) >> 5) + (ln & 1), W - 1)];
        }
#pragma unroll
        for (int c = 0; c < kM64Nch; ++c) {
            const int i = c * kM64Threads + to;
            if (i < m) {
                st[i] = kBig;
                st[(size_t)m + i] = i1[c];
                st[(size_t)2 * m + i] = kBig;
                st[(size_t)3 * m + i] = i2[c];
            }
            const unsigned long long bw = __ballot(sv[c] != 0u);
            const int w0 = (c * kM64Threads + wbase) >> 5;
            if (ln < 2 && w0 + ln < W) {
                const uint32_t word = (uint32_t)(bw >> (32 * ln));
                synw[w0 + ln] = word;
                parw[w0 + ln] = word;
                parw[W + w0 + ln] = word ^ ip[c];
            }
        }
        for (int w = to; w < W; w += kM64Threads) hdw[w] = hdw[W + w] = 0u;
        lds_barrier();
        QDEC_STAMP(0);
        if (tid == 0) *next = shot_next;
        double v[VPT][kMlDC];
        {
            const int tq0 = opaque_tq();
#pragma unroll
            for (int r = 0; r < VPT; ++r) {
                const double Lr = prior_of(prior, tq0, r);
#pragma unroll
                for (int k = 0; k < kMlDC; ++k) v[r][k] = Lr;
            }
        }

        uint32_t xb = 0, bad = 0;  // hard decisions (bit r), failing owned checks (bit c)
        bool conv = false;
        int it = 1;
        for (;; ++it) {
            const int b = it & 1, nb = b ^ 1;
            const double alpha = alpha_at<double>(it, a.ms_scaling);
            // ---- D: c2v from buffer b, sums, hard decision, new v2c -> buffer nb
            xb = 0;
            opaque_edges();
            int pz = 0;
            asm volatile("" : "+s"(pz));  // the prior loads stay in the loop (global, not flat)
            const double* pr = prior + pz;
            const int tqv = opaque_tq();
#pragma unroll
            for (int r = 0; r < VPT; ++r) {
                const int dj = deg(r);
                const double Lr = prior_of(pr, tqv, r);
                double c[kMlDC];
#pragma unroll
                for (int k = 0; k < kMlDC; ++k) {
                    c[k] = 0.0;
                    if (k < dmax(r) && k < dj) {
                        const int i = chk(r, k);
                        const unsigned long long* s = st + (size_t)b * m + i;
                        const unsigned long long m1 = s[0], m2 = s[2 * (size_t)m];
                        const uint32_t pw = parw[b * W + (i >> 5)];
                        const unsigned long long vb = dbits(v[r][k]);
                        const double y = __longlong_as_double((long long)((vb & kAbs) == m1 ? m2 : m1)) * alpha;
                        const uint32_t sg = ((pw >> (i & 31)) ^ (uint32_t)((vb - 1ull) >> 63)) & 1u;
                        c[k] = __longlong_as_double((long long)(dbits(y) ^ ((unsigned long long)sg << 63)));
                    }
                    __builtin_amdgcn_sched_barrier(0);  // one edge's state in flight (registers; issuing a
                                                        // column's reads together measured the same, profiles/r06ab,
                                                        // profiles/r06c4/ab_edge_batch)
                }
                // ldpc's order: prefix sums from the prior, then each outgoing
                // message = prefix + (sum of the later edges, accumulated from the end)
                double pre[kMlDC];
                double acc = Lr;
#pragma unroll
                for (int k = 0; k < kMlDC; ++k) {
                    pre[k] = acc;
                    acc = (k < dmax(r) && k < dj) ? acc + c[k] : acc;
                }
                const bool x = acc <= 0.0;
                xb |= (uint32_t)x << r;
                double suf = 0.0;
                bool started = false;
#pragma unroll
                for (int k = kMlDC - 1; k >= 0; --k) {
                    if (k >= dmax(r)) continue;
                    const double o = started ? pre[k] + suf : pre[k];
                    suf = started ? suf + c[k] : c[k];
                    started = started || k < dj;
                    if (k < dj) {
                        v[r][k] = o;
                        const int i = chk(r, k);
                        put_min(nb, i, dbits(o) & kAbs);  // (every ds_min_rtn of the column first, then
                                                          // the m2 updates: spills, 11 % slower, r06c4)
                        if (neg(o)) atomicXor(&parw[nb * W + (i >> 5)], 1u << (i & 31));
                        if (x) atomicXor(&hdw[b * W + (i >> 5)], 1u << (i & 31));
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            __syncthreads();
            QDEC_STAMP(1);
            QDEC_COUNT(9, 1);
            // ---- B: syndrome test of iteration it; reset of buffer b
            bad = 0;
            for (int c = 0; c < ncr; ++c) {
                const int i = c * kM64Threads + tid;
                bad |= (((hdw[b * W + (i >> 5)] ^ synw[i >> 5]) >> (i & 31)) & 1u) << c;
            }
            const unsigned long long wb = __ballot(bad != 0u);
            if (lane == 0) flags[b * (kM64Threads / 64) + wv] = wb != 0ull;
            for (int i = tid; i < m; i += kM64Threads) {
                st[(size_t)b * m + i] = kBig;
                st[(size_t)(2 + b) * m + i] = kBig;
            }
            for (int w = tid; w < W; w += kM64Threads) {
                parw[b * W + w] = synw[w];
                hdw[nb * W + w] = 0u;
            }
            __syncthreads();
            int any_bad = 0;
#pragma unroll
            for (int w = 0; w < kM64Threads / 64; ++w) any_bad |= flags[b * (kM64Threads / 64) + w];
            QDEC_STAMP(2);
            if (!any_bad) {
                conv = true;
                break;
            }
            if (it >= a.max_iter) break;
        }
        // ---- queue the shot: hard decision, residual syndrome, converged bit.
        // The bytes are staged in LDS (the state arrays are free after the last
        // B barrier) in column / check order and leave as whole lines: written
        // directly, the lanes' columns 67 apart and the slot-ordered checks put
        // every lane of a store in its own line.
        {
            uint8_t* sx = reinterpret_cast<uint8_t*>(st);  // [n] hard decisions
            uint8_t* sr = sx + ((n + 15) & ~15);            // [m] residual syndrome
            const int tqs = opaque_tq(), tt = opaque_tid();
            int ck[kM64Nch];
#pragma unroll
            for (int c = 0; c < kM64Nch; ++c) ck[c] = cslot[min(c * kM64Threads + tt, m - 1)];
#pragma unroll
            for (int r = 0; r < VPT; ++r) {
                const int j = r * kM64Threads + tqs;
                if (j < n) sx[j] = (uint8_t)((xb >> r) & 1);
            }
#pragma unroll
            for (int c = 0; c < kM64Nch; ++c)
                if (c * kM64Threads + tt < m) sr[ck[c]] = (uint8_t)((bad >> c) & 1);
            lds_barrier();
            auto copy_row = [&](uint8_t* dst, const uint8_t* src, int len) {
                if ((((uintptr_t)dst | (uintptr_t)len) & 3) == 0) {
                    for (int w = tt; w < len / 4; w += kM64Threads)
                        reinterpret_cast<uint32_t*>(dst)[w] = reinterpret_cast<const uint32_t*>(src)[w];
                } else {
                    for (int j = tt; j < len; j += kM64Threads) dst[j] = src[j];
                }
            };
            copy_row(a.q_x + shot * n, sx, n);
            copy_row(a.q_r + shot * m, sr, m);
            if (tid == 0) {
                a.q_idx[shot] = shot | ((int64_t)(conv ? 1 : 0) << 62);
                if (a.iters) a.iters[shot] = conv ? it : a.max_iter;
            }
            lds_barrier();  // the staged bytes are read before the next shot's S phase writes
        }
        QDEC_STAMP(3);
    }
    QDEC_FLUSH_AT(16);
}

#ifdef QDEC_STAMPS
// this translation unit's phase timers (qdec_stamps is per file): slots 16.. of
// bp_ms_lds64_kernel (tools/dev/stamps_c4.py)
extern "C" __attribute__((visibility("default"))) int qd_dev_read_stamps_block(unsigned long long* out, int n,
                                                                              int reset) {
    unsigned long long h[64] = {0};
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(qdec_stamps), sizeof(h)) != hipSuccess) return -1;
    for (int i = 0; i < n && i < 64; ++i) out[i] = h[i];
    if (reset) {
        unsigned long long z[64] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(qdec_stamps), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

// ---------------------------------------------------------------- launcher
template <typename K, typename P>
static int launch_block(K kern, size_t lds, int64_t work, int num_cus, hipStream_t stream, int cap_per_cu,
                        const DevGraph& g, const DecodeArgs& a, P* extra0, int extra1) {
    int per_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kBlock, lds);
    if (e != hipSuccess) return (int)e;
    if (per_cu <= 0) return (int)hipErrorInvalidConfiguration;
    if (cap_per_cu > 0 && per_cu > cap_per_cu) per_cu = cap_per_cu;
    long long grid = (long long)num_cus * per_cu;
    if (grid > work) grid = work;
    if (grid <= 0) return 0;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kBlock), lds, stream, g, a, extra0, extra1);
    return (int)hipGetLastError();
}

template <typename K>
static int launch_block2(K kern, size_t lds, int64_t work, int num_cus, hipStream_t stream, const DevGraph& g,
                         const DecodeArgs& a, unsigned char* gstate = nullptr, int max_per_cu = 0) {
    int per_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kBlock, lds);
    if (e != hipSuccess) return (int)e;
    if (per_cu <= 0) return (int)hipErrorInvalidConfiguration;
    if (max_per_cu > 0 && per_cu > max_per_cu) per_cu = max_per_cu;
    long long grid = (long long)num_cus * per_cu;
    if (grid > work) grid = work;
    if (grid <= 0) return 0;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kBlock), lds, stream, g, a, gstate);
    return (int)hipGetLastError();
}

// SSF + finalize of queued shots whose state fits LDS: the incremental kernel
// when the inverse table exists (QD_OPT_SSF_INC = 0 selects the re-scanning one).
static int launch_ssf_fin(const DevGraph& g, const DecodeArgs& a, int num_cus, hipStream_t stream) {
    const size_t lds = ssf_inc_lds(g);
    if (a.ssf && g.g_iptr && g.n_gen <= 8192 && lds <= 160 * 1024 && g.opt_ssf_inc) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&ssf_inc_block_kernel),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return (int)e;
        int per_cu = 0;
        hipError_t e2 = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ssf_inc_block_kernel, kBlock, lds);
        if (e2 != hipSuccess) return (int)e2;
        if (per_cu <= 0) return (int)hipErrorInvalidConfiguration;
        const long long grid = std::min<long long>((long long)num_cus * per_cu, a.B);
        if (grid <= 0) return 0;
        hipLaunchKernelGGL(ssf_inc_block_kernel, dim3((unsigned)grid), dim3(kBlock), lds, stream, g, a);
        return (int)hipGetLastError();
    }
    return launch_block2(ssf_block_kernel, (block_small_lds(g) + 15) / 16 * 16, a.B, num_cus, stream, g, a);
}

constexpr size_t kLdsMsgLimit = 64 * 1024;  // messages in LDS up to this (2 workgroups per CU)

// Where the BP workgroup keeps its state: messages in LDS when everything fits
// kLdsMsgLimit, else in HBM; the per-shot byte arrays stay in LDS up to
// kLdsMsgLimit (n ~ 6*10^4), beyond that (e.g. the 1.2*10^5-column spacetime
// graph of config 5) they move to the HBM slice as well.
inline int block_placement(const DevGraph& g, size_t tsz) {
    const size_t msg = ((size_t)2 * g.E * tsz + 15) / 16 * 16;
    const size_t small = (block_small_lds(g) + 15) / 16 * 16;
    if (msg + small <= kLdsMsgLimit) return 3;
    return small <= kLdsMsgLimit ? 2 : 0;
}

template <typename T, int METHOD>
static int launch_block_typed(const DevGraph& g, const DecodeArgs& a0, int num_cus, hipStream_t stream, void* scratch,
                              size_t scratch_bytes) {
    const size_t msg = ((size_t)2 * g.E * sizeof(T) + 15) / 16 * 16;
    const size_t small = (block_small_lds(g) + 15) / 16 * 16;
    const int placement = block_placement(g, sizeof(T));
    // placement 0: control area + the hard-decision bits of the unrolled kernel
    const size_t lds = (placement & 2) ? small + ((placement & 1) ? msg : 0) : kCtrl + (size_t)g.n_pad / 8;
    int cap = 0;
    T* gs = nullptr;
    DecodeArgs a = a0;
    // placement 0 with SSF: the SSF/finalize workgroups keep their shot state in
    // HBM too, in the scratch tail (kFinPerCu workgroups per CU)
    const bool fin_hbm = a0.ssf && placement == 0;
    const size_t fin_bytes = fin_hbm ? (size_t)num_cus * kFinPerCu * block_state_stride(g) : 0;
    if (placement != 3) {
        // scratch = header (dynamic shot counter) + per-workgroup slices in HBM
        const size_t per_wg = block_slice_bytes(g, sizeof(T), placement);
        if (!scratch || per_wg == 0 || scratch_bytes <= kGrpHeader + fin_bytes) return (int)hipErrorInvalidValue;
        const long long max_wg = (long long)((scratch_bytes - kGrpHeader - fin_bytes) / per_wg);
        // the grid is num_cus * cap workgroups, each owning one slice: at least
        // one slice per CU (block_scratch_bytes sizes 4 per CU)
        if (max_wg < num_cus) return (int)hipErrorOutOfMemory;
        cap = (int)(max_wg / num_cus);
        // Resident workgroups per CU.  With the shot state in HBM too (placement
        // 0, the C5 spacetime graph: 3.3 MB of slices per shot) the scattered
        // message accesses of more resident shots only add HBM traffic: on C5 at
        // p = 0.005, 4 / 3 / 2 / 1 per CU ran 18.0 / 20.8 / 26.3 / 19.2 k shots/s
        // (scattered writes), 23.9 / 27.1 / 29.3 k (contiguous writes, vcsc), so
        // placement 0 runs 2.  QD_OPT_BLOCK_WG overrides.
        if (placement == 0) cap = std::min(cap, 2);
        if (g.opt_block_wg > 0) cap = std::min((int)(max_wg / num_cus), g.opt_block_wg);
        a.work_ctr = static_cast<unsigned long long*>(scratch);
        gs = reinterpret_cast<T*>(static_cast<unsigned char*>(scratch) + kGrpHeader);
        const hipError_t e0 = hipMemsetAsync(a.work_ctr, 0, sizeof(unsigned long long), stream);
        if (e0 != hipSuccess) return (int)e0;
    }
    // graphs with row degree <= 16 and column degree <= 8: unrolled loops
    const bool unr = g.max_rdeg <= 16 && g.max_cdeg <= 8;
    constexpr int UR = 16, UC = 8;
    if (!a.ssf) {
        record_ev(a, 0, stream);
        const int rc = unr ? launch_block(bp_block_kernel<T, METHOD, false, UR, UC>, lds, a.B, num_cus, stream, cap, g, a,
                                          gs, placement)
                           : launch_block(bp_block_kernel<T, METHOD, false>, lds, a.B, num_cus, stream, cap, g, a, gs,
                                          placement);
        record_ev(a, 1, stream);
        record_ev(a, 2, stream);
        return rc;
    }
    if (!a.q_count || !a.q_idx || !a.q_x || !a.q_r) return (int)hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(a.q_count, 0, sizeof(int32_t), stream);
    if (e != hipSuccess) return (int)e;
    record_ev(a, 0, stream);
    int rc = unr ? launch_block(bp_block_kernel<T, METHOD, true, UR, UC>, lds, a.B, num_cus, stream, cap, g, a, gs,
                                placement)
                 : launch_block(bp_block_kernel<T, METHOD, true>, lds, a.B, num_cus, stream, cap, g, a, gs, placement);
    record_ev(a, 1, stream);
    if (rc != 0) return rc;
    rc = fin_hbm ? launch_block2(ssf_block_kernel, kCtrl, a.B, num_cus, stream, g, a,
                                 static_cast<unsigned char*>(scratch) + (scratch_bytes - fin_bytes), kFinPerCu)
                 : launch_ssf_fin(g, a, num_cus, stream);
    record_ev(a, 2, stream);
    return rc;
}

// ---------------------------------------------------------------- LDS-resident launch
// QD_OPT_LDS_KERNEL = 0 disables bp_ms_lds_kernel / bp_ms_lds64_kernel, 1 forces
// them on any graph they can hold (also those whose messages fit the small-graph
// LDS budget); by default they take the min-sum graphs whose messages would go
// to HBM (f32: edge slots <= 160 KB; f64: n <= 10240 and the check states <= 160 KB).
bool lds_kernel_applies(const DevGraph& g, int method, int precision, const DecodeArgs& a) {
    if (method != 1 || !g.ml_etab || (precision == 0 && (!g.m64_etab || !g.m64_check))) return false;
    if (!a.syn || a.syn_flags || a.llr_out || !a.wave_ctr) return false;
    if (precision == 0) {  // bp_ms_lds64_kernel (automatic: graphs whose messages would go to HBM)
        if (g.n > 10 * kM64Threads || g.m <= 0 || g.m > kM64Nch * kM64Threads || a.max_iter < 1) return false;
        if (m64_lds_bytes(g) > 160 * 1024 || block_placement(g, 8) == 0) return false;
        if (g.opt_lds_kernel == 0) return false;
        return g.opt_lds_kernel == 1 || block_placement(g, 8) != 3;
    }
    if (precision != 1) return false;
    if (g.n > 16 * kMlThreads || g.m <= 0 || g.m > kMlNch * kMlThreads || a.max_iter < 1 ||
        ml_lds_bytes(g) > 160 * 1024)
        return false;
    if (block_placement(g, 4) == 0) return false;  // the SSF/finalize state would not fit LDS
    if (g.opt_lds_kernel == 0) return false;
    if (g.opt_lds_kernel == 1) return true;
    return block_placement(g, 4) != 3;
}

template <int VPT>
static int launch_lds_typed(const DevGraph& g, const DecodeArgs& a, int num_cus, hipStream_t stream, float* img,
                            size_t img_bytes) {
    const size_t lds = ml_lds_bytes(g);
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&bp_ms_lds_kernel<VPT>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
    int per_cu = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, bp_ms_lds_kernel<VPT>, kMlThreads, lds);
    if (e != hipSuccess) return (int)e;
    if (per_cu <= 0) return (int)hipErrorInvalidConfiguration;
    if (!img || img_bytes < ml_image_bytes(g)) return (int)hipErrorInvalidValue;
    const long long grid = std::min<long long>((long long)num_cus * per_cu, a.B);
    e = hipMemsetAsync(a.wave_ctr, 0, sizeof(unsigned long long), stream);  // shot counter
    if (e != hipSuccess) return (int)e;
    const float* prior = reinterpret_cast<const float*>(g.prior[1][1]);
    hipLaunchKernelGGL(ml_init_scatter_kernel, dim3((unsigned)((g.n + 255) / 256)), dim3(256), 0, stream, g, g.ml_etab,
                       prior, img);
    hipLaunchKernelGGL(ml_init_check_kernel, dim3((unsigned)((g.m + 255) / 256)), dim3(256), 0, stream, g, img,
                       a.ms_scaling);
    record_ev(a, 0, stream);
    QDEC_NOTE_BP("qdec::bp_ms_lds_kernel", VPT);
    hipLaunchKernelGGL((bp_ms_lds_kernel<VPT>), dim3((unsigned)grid), dim3(kMlThreads), lds, stream, g, a, g.ml_etab,
                       prior, img);
    const hipError_t le = hipGetLastError();
    record_ev(a, 1, stream);
    if (le != hipSuccess) return (int)le;
    const bool fin_hbm = block_placement(g, 4) == 0;
    const int rc = fin_hbm ? (int)hipErrorNotSupported
                           : launch_ssf_fin(g, a, num_cus, stream);
    record_ev(a, 2, stream);
    return rc;
}

template <int VPT, int D3R>
static int launch_lds64_typed(const DevGraph& g, const DecodeArgs& a, int num_cus, hipStream_t stream,
                              unsigned long long* img, size_t img_bytes) {
    const size_t lds = m64_lds_bytes(g);
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&bp_ms_lds64_kernel<VPT, D3R>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
    int per_cu = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, bp_ms_lds64_kernel<VPT, D3R>, kM64Threads, lds);
    if (e != hipSuccess) return (int)e;
    if (per_cu <= 0) return (int)hipErrorInvalidConfiguration;
    const long long grid = std::min<long long>((long long)num_cus * per_cu, a.B);
    e = hipMemsetAsync(a.wave_ctr, 0, sizeof(unsigned long long), stream);  // shot counter
    if (e != hipSuccess) return (int)e;
    if (!img || img_bytes < m64_image_bytes(g)) return (int)hipErrorInvalidValue;
    const double* prior = reinterpret_cast<const double*>(g.prior[1][0]);
    hipLaunchKernelGGL(m64_init_kernel, dim3((unsigned)((g.m + 255) / 256)), dim3(256), 0, stream, g, prior,
                       g.m64_check, img);
    record_ev(a, 0, stream);
    QDEC_NOTE_BP("qdec::bp_ms_lds64_kernel", VPT, D3R);
    hipLaunchKernelGGL((bp_ms_lds64_kernel<VPT, D3R>), dim3((unsigned)grid), dim3(kM64Threads), lds, stream, g, a,
                       g.m64_etab, prior, g.m64_check, img);
    const hipError_t le = hipGetLastError();
    record_ev(a, 1, stream);
    if (le != hipSuccess) return (int)le;
    const int rc = launch_ssf_fin(g, a, num_cus, stream);
    record_ev(a, 2, stream);
    return rc;
}

static int launch_lds(const DevGraph& g, int precision, const DecodeArgs& a, int num_cus, hipStream_t stream,
                      void* scratch, size_t scratch_bytes) {
    unsigned long long* img = reinterpret_cast<unsigned long long*>(scratch);  // f64: iteration 1's states
    if (!a.q_count || !a.q_idx || !a.q_x || !a.q_r) return (int)hipErrorInvalidValue;
    if (precision == 0) {
        // the largest instantiated D3R <= the graph's (leading rounds of degree <= 3)
        const int vpt = (g.n + kM64Threads - 1) / kM64Threads, d3r = g.m64_d3r;
        if (vpt <= 4) return launch_lds64_typed<4, 0>(g, a, num_cus, stream, img, scratch_bytes);
        if (vpt <= 8)
            return d3r >= 4 ? launch_lds64_typed<8, 4>(g, a, num_cus, stream, img, scratch_bytes)
                            : launch_lds64_typed<8, 0>(g, a, num_cus, stream, img, scratch_bytes);
        if (d3r >= 6) return launch_lds64_typed<10, 6>(g, a, num_cus, stream, img, scratch_bytes);
        if (d3r >= 3) return launch_lds64_typed<10, 3>(g, a, num_cus, stream, img, scratch_bytes);
        return launch_lds64_typed<10, 0>(g, a, num_cus, stream, img, scratch_bytes);
    }
    float* fimg = reinterpret_cast<float*>(scratch);  // f32: iteration 1's c2v rows
    const int vpt = (g.n + kMlThreads - 1) / kMlThreads;
    if (vpt <= 4) return launch_lds_typed<4>(g, a, num_cus, stream, fimg, scratch_bytes);
    if (vpt <= 8) return launch_lds_typed<8>(g, a, num_cus, stream, fimg, scratch_bytes);
    if (vpt <= 10) return launch_lds_typed<10>(g, a, num_cus, stream, fimg, scratch_bytes);
    if (vpt <= 12) return launch_lds_typed<12>(g, a, num_cus, stream, fimg, scratch_bytes);
    return launch_lds_typed<16>(g, a, num_cus, stream, fimg, scratch_bytes);
}

// ---------------------------------------------------------------- slot-group launch
// HBM budget of one handle's group scratch: QD_OPT_GROUP_MB when set, else
// a quarter of the device memory free right now (a bpssf_hybrid pipeline holds
// two such handles; the batch cap in group_count keeps small decodes small)
static size_t group_scratch_budget(const DevGraph& g) {
    if (g.opt_group_mb > 0) return (size_t)std::max(64, g.opt_group_mb) << 20;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess || free_b == 0) return (size_t)4 << 30;
    return std::max<size_t>(free_b / 4, (size_t)64 << 20);
}

template <typename T, int METHOD, int DR, int DC>
static int group_occupancy() {
    static const int per_cu = [] {
        int v = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, bp_group_kernel<T, METHOD, DR, DC>, 64 * grp_waves<T>(),
                                                         0) != hipSuccess)
            v = 1;
        return std::max(v, 1);
    }();
    return per_cu;
}

// resident slot groups per CU of the instantiation launch_group_shape picks
static int group_per_cu(const DevGraph& g, int method, size_t tsz) {
    const bool r8 = g.max_rdeg <= 8, c4 = g.max_cdeg <= 4;
#define QDEC_GOCC(T, M)                                                          \
    return r8 ? (c4 ? group_occupancy<T, M, 8, 4>() : group_occupancy<T, M, 8, 8>()) \
              : (c4 ? group_occupancy<T, M, 16, 4>() : group_occupancy<T, M, 16, 8>())
    if (tsz == 4) {
        if (method == 1) QDEC_GOCC(float, 1);
        QDEC_GOCC(float, 0);
    }
    if (method == 1) QDEC_GOCC(double, 1);
    QDEC_GOCC(double, 0);
#undef QDEC_GOCC
}

// Groups in flight: as many as the kernel's occupancy keeps resident, capped by
// the scratch budget and by the batch (every slot should see >= 2 shots, so the
// tail of a launch stays short and small test batches stay small).  The
// scratch is sized from exactly this count (block_scratch_bytes).
static int64_t group_count(const DevGraph& g, int method, size_t tsz, int num_cus, int64_t B) {
    const size_t per = group_layout(g, tsz).total;
    int64_t c = std::min<int64_t>((int64_t)num_cus * group_per_cu(g, method, tsz),
                                  (int64_t)(group_scratch_budget(g) / per));
    c = std::min<int64_t>(c, (B + 127) / 128);
    return std::max<int64_t>(c, 1);
}

// The slot-group kernel takes min-sum and product-sum graphs whose messages do
// not fit the small-graph LDS budget (row degree <= 16, column degree <= 8, the
// syndrome given directly).  QD_OPT_GROUP_KERNEL = 0 disables it (workgroup kernel
// with HBM message slices), =1 forces it on any graph within those degrees.
// For fp32 min-sum graphs the LDS-resident kernel (bp_ms_lds_kernel) keeps
// precedence unless the group kernel is forced.
bool group_kernel_applies(const DevGraph& g, int method, int precision, const DecodeArgs& a) {
    if (g.max_rdeg > 16 || g.max_cdeg > 8 || !a.syn || a.syn_flags) return false;
    (void)method;
    if (g.opt_group_kernel == 0) return false;
    if (g.opt_group_kernel == 1) return true;
    return block_placement(g, precision == 1 ? 4 : 8) != 3;
}

template <typename T, int METHOD, int DR, int DC>
static int launch_group_typed(const DevGraph& g, const DecodeArgs& a, int num_cus, hipStream_t stream, void* scratch,
                              size_t scratch_bytes) {
    const size_t gb = group_layout(g, sizeof(T)).total;
    // tail of the scratch: HBM shot state of the SSF/finalize workgroups when it
    // does not fit LDS (kFinPerCu workgroups per CU)
    const bool fin_hbm = a.ssf && block_placement(g, sizeof(T)) == 0;
    const size_t fin_bytes = fin_hbm ? (size_t)num_cus * kFinPerCu * block_state_stride(g) : 0;
    if (!scratch || scratch_bytes < fin_bytes + kGrpHeader + gb) return (int)hipErrorOutOfMemory;
    unsigned char* base = static_cast<unsigned char*>(scratch);
    unsigned char* fin_state = fin_hbm ? base + (scratch_bytes - fin_bytes) : nullptr;
    const int64_t max_groups = (int64_t)((scratch_bytes - fin_bytes - kGrpHeader) / gb);
    int per_cu = 0;
    constexpr int kGrpThreads = 64 * grp_waves<T>();
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, bp_group_kernel<T, METHOD, DR, DC>,
                                                                kGrpThreads, 0);
    if (e != hipSuccess) return (int)e;
    if (per_cu <= 0) return (int)hipErrorInvalidConfiguration;
    int64_t grid = std::min<int64_t>((int64_t)num_cus * per_cu, max_groups);
    grid = std::min<int64_t>(grid, group_count(g, METHOD, sizeof(T), num_cus, a.B));
    if (grid <= 0) return (int)hipErrorOutOfMemory;
    e = hipMemsetAsync(base, 0, sizeof(unsigned long long), stream);  // shot counter
    if (e != hipSuccess) return (int)e;
    if (a.ssf) {
        if (!a.q_count || !a.q_idx || !a.q_x || !a.q_r) return (int)hipErrorInvalidValue;
        e = hipMemsetAsync(a.q_count, 0, sizeof(int32_t), stream);
        if (e != hipSuccess) return (int)e;
    }
    record_ev(a, 0, stream);
    QDEC_NOTE_BP("qdec::bp_group_kernel", tname<T>(), METHOD, DR, DC);
    hipLaunchKernelGGL((bp_group_kernel<T, METHOD, DR, DC>), dim3((unsigned)grid), dim3(kGrpThreads), 0, stream, g, a,
                       base, gb, g.row_ptr, g.col_idx, g.col_ptr, g.col_edge, g.edge_csc,
                       reinterpret_cast<const T*>(g.prior[METHOD][sizeof(T) == 4 ? 1 : 0]),
                       reinterpret_cast<const T*>(g.eprior[METHOD][sizeof(T) == 4 ? 1 : 0]));
    const hipError_t le = hipGetLastError();
    record_ev(a, 1, stream);
    if (le != hipSuccess) return (int)le;
    int rc = 0;
    if (a.ssf)
        rc = fin_hbm ? launch_block2(ssf_block_kernel, kCtrl, a.B, num_cus, stream, g, a, fin_state, kFinPerCu)
                     : launch_ssf_fin(g, a, num_cus, stream);
    record_ev(a, 2, stream);
    return rc;
}

template <typename T, int METHOD>
static int launch_group_shape(const DevGraph& g, const DecodeArgs& a, int num_cus, hipStream_t stream, void* scratch,
                              size_t scratch_bytes) {
    const bool r8 = g.max_rdeg <= 8, c4 = g.max_cdeg <= 4;
    if (r8) return c4 ? launch_group_typed<T, METHOD, 8, 4>(g, a, num_cus, stream, scratch, scratch_bytes)
                      : launch_group_typed<T, METHOD, 8, 8>(g, a, num_cus, stream, scratch, scratch_bytes);
    return c4 ? launch_group_typed<T, METHOD, 16, 4>(g, a, num_cus, stream, scratch, scratch_bytes)
              : launch_group_typed<T, METHOD, 16, 8>(g, a, num_cus, stream, scratch, scratch_bytes);
}

size_t block_scratch_bytes(const DevGraph& g, int method, int precision, int num_cus, const DecodeArgs& a) {
    const size_t tsz = precision == 1 ? 4 : 8;
    if (group_kernel_applies(g, method, precision, a) && !(lds_kernel_applies(g, method, precision, a) && g.opt_group_kernel != 1)) {
        const size_t fin = (a.ssf && block_placement(g, tsz) == 0) ? (size_t)num_cus * kFinPerCu * block_state_stride(g)
                                                                  : 0;
        return kGrpHeader + (size_t)group_count(g, method, tsz, num_cus, a.B) * group_layout(g, tsz).total + fin;
    }
    // LDS-resident kernels: iteration 1's image (f64: check states, m64_init_kernel;
    // f32: c2v rows, ml_init_*_kernel)
    if (lds_kernel_applies(g, method, precision, a)) return precision == 0 ? m64_image_bytes(g) : ml_image_bytes(g);
    const int placement = block_placement(g, tsz);
    if (placement == 3) return 0;
    // shot-counter header + up to 4 workgroup slices per CU (+ the SSF/finalize
    // shot state when it lives in HBM)
    const size_t fin = (a.ssf && placement == 0) ? (size_t)num_cus * kFinPerCu * block_state_stride(g) : 0;
    return kGrpHeader + (size_t)num_cus * 4 * block_slice_bytes(g, tsz, placement) + fin;
}

// The smallest scratch a launch can run with (one slot group, or one workgroup
// slice per CU); block_scratch_bytes' figure may be cut down to it when the
// allocation fails (fewer groups / slices in flight, same results).
size_t block_scratch_floor(const DevGraph& g, int method, int precision, int num_cus, const DecodeArgs& a) {
    const size_t full = block_scratch_bytes(g, method, precision, num_cus, a);
    if (full == 0) return 0;
    const size_t tsz = precision == 1 ? 4 : 8;
    const size_t fin = (a.ssf && block_placement(g, tsz) == 0) ? (size_t)num_cus * kFinPerCu * block_state_stride(g) : 0;
    if (group_kernel_applies(g, method, precision, a) && !(lds_kernel_applies(g, method, precision, a) && g.opt_group_kernel != 1))
        return std::min(full, kGrpHeader + group_layout(g, tsz).total + fin);
    return full;  // workgroup slices: the launch needs its per-CU slices
}

int launch_decode_block(const DevGraph& g, int method, int precision, const DecodeArgs& a, int num_cus,
                        hipStream_t stream, void* scratch, size_t scratch_bytes) {
    if (a.B <= 0) return 0;
    if (a.ssf && g.n_gen <= 0) return (int)hipErrorInvalidValue;
    const bool lds = lds_kernel_applies(g, method, precision, a);
    if (group_kernel_applies(g, method, precision, a) && !(lds && g.opt_group_kernel != 1)) {
        if (precision == 1)
            return method == 1 ? launch_group_shape<float, 1>(g, a, num_cus, stream, scratch, scratch_bytes)
                               : launch_group_shape<float, 0>(g, a, num_cus, stream, scratch, scratch_bytes);
        return method == 1 ? launch_group_shape<double, 1>(g, a, num_cus, stream, scratch, scratch_bytes)
                           : launch_group_shape<double, 0>(g, a, num_cus, stream, scratch, scratch_bytes);
    }
    if (lds) return launch_lds(g, precision, a, num_cus, stream, scratch, scratch_bytes);
    if (precision == 1)
        return method == 1 ? launch_block_typed<float, 1>(g, a, num_cus, stream, scratch, scratch_bytes)
                           : launch_block_typed<float, 0>(g, a, num_cus, stream, scratch, scratch_bytes);
    return method == 1 ? launch_block_typed<double, 1>(g, a, num_cus, stream, scratch, scratch_bytes)
                       : launch_block_typed<double, 0>(g, a, num_cus, stream, scratch, scratch_bytes);
}

int launch_ssf_block(const DevGraph& g, const DecodeArgs& a, int num_cus, hipStream_t stream) {
    return launch_ssf_fin(g, a, num_cus, stream);
}

}  // namespace qdec
