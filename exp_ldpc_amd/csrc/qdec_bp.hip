// qdec_bp.hip -- BP + small-set-flip syndrome decoding on gfx950.
//
// Two kernels per decode call:
//
// 1. bp_wave_kernel: one wave64 decodes one shot at a time (workgroup = one
//    wave; persistent grid walking the shot range).  Everything a shot touches
//    lives in that wave's LDS slice:
//      v2c  [m_pad][DRS]+64  variable->check messages, check-major, 16-B rows
//      c2v  [n_pad][DCS]+64  check->variable messages, variable-major
//      xh   [n_pad+64]       hard decisions (u8; the last 64 bytes stay 0)
//    The trailing 64 elements of v2c/c2v are per-lane dummy slots: pad edges of a
//    low-degree check/variable write there, so every scatter is unconditional and
//    the passes are branch-free.  A lane owns checks i = lane + 64*rc and
//    variables j = lane + 64*rv; the graph is padded to exactly RC*64 checks and
//    RV*64 variables (QDEC_WAVE_SHAPES).  The check pass reads its row with
//    ds_read_b128 (conflict-free strides, lds_stride) and scatters c2v through a
//    slot table held in registers; the variable pass does the mirror image.
//    With SSF requested, shots BP did not converge on are appended (hard
//    decision + residual syndrome) to an HBM work queue instead of finalised.
// 2. ssf_wave_kernel: one wave per queued shot runs small-set-flip and
//    finalises it.  Only failing shots are touched (compacted), and the BP
//    kernel's register budget does not carry the SSF scan.
//
// Arithmetic is the ldpc v1 bp_decoder restated (oracle/bp_impl.inc is the CPU
// copy of the same loops): min-sum in the log domain with alpha_t = 1 - 2^-t
// (ms_scaling_factor = 0) or a constant; product-sum in the probability-ratio
// domain; column prefix + suffix sums in ldpc's order.  Built with
// -ffp-contract=off so every multiply and add is rounded separately: results are
// bit-identical to the CPU oracle at the same precision.
//
// Small-set-flip (build-defined spec): for each generator g (lane
// owned), every subset F of its <= 8 qubits is scored as
//   key = (gain(F) * 840/|F|, -g, -F)      gain(F) = |s| - |s xor H 1_F|
// with the syndrome restricted to the generator's <= 32 local checks as a bitmask
// (popcount of xor with a per-subset mask: 5 VALU ops per subset).  A wave max
// picks the flip.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdlib>

#include "qdec_device.h"
#include "qdec_bp_ms.h"

namespace qdec {

// ============================================================== BP kernel
template <typename T, int METHOD, int RC, int RV, int DRC, bool DEFER>
__global__ __launch_bounds__(64) void bp_wave_kernel(DevGraph g, DecodeArgs a) {
    static_assert(DRC <= kDR, "compute width exceeds the LDS row");
    constexpr int DRS = lds_stride<T, kDR>();
    constexpr int DCS = lds_stride<T, kDC>();
    constexpr int PREC = sizeof(T) == 4 ? 1 : 0;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T* v2c = reinterpret_cast<T*>(smem);
    T* c2v = v2c + g.m_pad * DRS + 64;
    uint8_t* xh = reinterpret_cast<uint8_t*>(c2v + g.n_pad * DCS + 64);

    const int lane = threadIdx.x;
    const SlotTables st = g.slots[PREC];
    const T* prior = reinterpret_cast<const T*>(g.prior[METHOD][PREC]);
    const int m = g.m, n = g.n;

    // ---- per-lane graph tables (registers); pad edges -> dummy slots / zero bytes
    uint32_t rtab[RC][DRC];      // col | cslot << 16 (slots >= DRC are pads: never used)
    uint32_t ctab[RV][kDC / 2];  // rslot pairs
    T L[RV];
#pragma unroll
    for (int rc = 0; rc < RC; ++rc) {
        const int i = rc * 64 + lane;
#pragma unroll
        for (int k = 0; k < DRC; ++k)
            rtab[rc][k] = (uint32_t)g.r_col[k * g.m_pad + i] | ((uint32_t)st.r_cslot[k * g.m_pad + i] << 16);
    }
#pragma unroll
    for (int rv = 0; rv < RV; ++rv) {
        const int j = rv * 64 + lane;
        L[rv] = prior[j];
#pragma unroll
        for (int k = 0; k < kDC / 2; ++k)
            ctab[rv][k] = (uint32_t)st.c_rslot[(2 * k) * g.n_pad + j] |
                          ((uint32_t)st.c_rslot[(2 * k + 1) * g.n_pad + j] << 16);
    }

    // ---- one-time LDS init: pads hold neutral messages forever ----
    const T vneutral = METHOD == 1 ? Big<T>::v : (T)0;  // MS: |v| never the min; PS: factor 1
    const T cneutral = METHOD == 1 ? (T)0 : (T)1;       // MS: +0 in sums; PS: x1 in products
    for (int e = lane; e < g.m_pad * DRS + 64; e += 64) v2c[e] = vneutral;
    for (int e = lane; e < g.n_pad * DCS + 64; e += 64) c2v[e] = cneutral;
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
                int p = 0;
#pragma unroll
                for (int k = 0; k < DRC; ++k) p ^= xh[rtab[rc][k] & 0xffff];
                sbit[rc] ^= p;
            }
            __syncthreads();
        }

        // ---- initial messages ----
#pragma unroll
        for (int rv = 0; rv < RV; ++rv) {
#pragma unroll
            for (int k = 0; k < kDC; ++k) v2c[(ctab[rv][k >> 1] >> ((k & 1) * 16)) & 0xffff] = L[rv];
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
                const int i = rc * 64 + lane;
                T v[kDR];
                lds_load<T, kDR>(v2c + i * DRS, v);
                if constexpr (METHOD == 1) {
                    // ldpc's forward/backward leave-one-out minimum equals
                    //   |c2v_k| = (|v_k| == m1) ? m2 : m1
                    // with m1 <= m2 the two smallest |v| (ties: m2 = m1).  min/med3
                    // give exactly that for NaN-free messages (priors in (0,1)).
                    T m1 = Big<T>::v, m2 = Big<T>::v;
                    bool par = sbit[rc] != 0;
                    bool sk[DRC];
#pragma unroll
                    for (int k = 0; k < DRC; ++k) {
                        const T av = fabs(v[k]);
                        m2 = med3(av, m1, m2);
                        m1 = fmin(m1, av);
                        sk[k] = v[k] <= (T)0;  // ldpc: bit_to_check <= 0 flips the sign
                        par ^= sk[k];
                    }
                    const T m1a = m1 * alpha, m2a = m2 * alpha;  // |c| * alpha, sign applied after
#pragma unroll
                    for (int k = 0; k < DRC; ++k) {
                        const T y = (fabs(v[k]) == m1) ? m2a : m1a;
                        c2v[rtab[rc][k] >> 16] = (par ^ sk[k]) ? -y : y;
                    }
                } else {
                    T t[DRC], fw[DRC];
                    T f = sbit[rc] ? (T)-1 : (T)1;
#pragma unroll
                    for (int k = 0; k < DRC; ++k) {
                        t[k] = (T)2 / ((T)1 + v[k]) - (T)1;
                        fw[k] = f;
                        f *= t[k];
                    }
                    T b = (T)1;
#pragma unroll
                    for (int k = DRC - 1; k >= 0; --k) {
                        T c = fw[k] * b;
                        c = ((T)1 - c) / ((T)1 + c);
                        b *= t[k];
                        c2v[rtab[rc][k] >> 16] = c;
                    }
                }
            }
            __syncthreads();

            // ---- variable -> check, hard decision ----
#pragma unroll
            for (int rv = 0; rv < RV; ++rv) {
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
                        v2c[(ctab[rv][k >> 1] >> ((k & 1) * 16)) & 0xffff] = out;  // pads -> dummy
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
                        v2c[(ctab[rv][k >> 1] >> ((k & 1) * 16)) & 0xffff] = out;
                    }
                }
                xh[j] = (uint8_t)xb;  // j in [n, n_pad): never read as data
            }
            __syncthreads();

            // ---- syndrome test ----
            int bad = 0;
#pragma unroll
            for (int rc = 0; rc < RC; ++rc) {
                int p = sbit[rc];
#pragma unroll
                for (int k = 0; k < DRC; ++k) p ^= xh[rtab[rc][k] & 0xffff];  // pads -> zero bytes
                pres[rc] = p;
                bad |= p;
            }
            if (__ballot(bad) == 0ull) {
                conv = true;
                break;
            }
        }
        const int iters = conv ? it : a.max_iter;
        if (lane == 0 && a.iters) a.iters[shot] = iters;
        if (a.llr_out) {
            T* lo = reinterpret_cast<T*>(a.llr_out);
#pragma unroll
            for (int rv = 0; rv < RV; ++rv) {
                const int j = rv * 64 + lane;
                if (j < n) {
                    if constexpr (METHOD == 1) lo[shot * n + j] = Q[rv];
                    else lo[shot * n + j] = (T)log((double)((T)1 / Q[rv]));
                }
            }
        }
        if (DEFER && !conv) {
            // hand the shot to the SSF kernel: hard decision + residual syndrome
            if (a.q_packed) {
                uint64_t xw[RV], rw[RC], dw[RV];
                const bool with_rd = a.readout && a.fail && g.k > 0;
#pragma unroll
                for (int w = 0; w < RV; ++w) {
                    const int q = w * 64 + lane;
                    xw[w] = __ballot(q < n && (xh[q] & 1));
                    dw[w] = with_rd ? __ballot(q < g.n_data && (a.readout[shot * g.n_data + q] & 1)) : 0ull;
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
        } else {
            finalize_shot(g, a, shot, xh, conv, conv, 0, lane);
        }
        __syncthreads();
    }
}

// ============================================================== SSF kernel
// Four waves per workgroup share the generator tables in LDS; each wave
// decodes its own queued shots independently (no cross-wave sync after the
// table fill).  Incremental greedy: a generator's best score only changes when
// its local syndrome changes, so every step
//   1. lane l gathers the local syndromes (<= 32 bits) of generators l + 64 rg
//      and compares them with the previous step's; changed generators with a
//      non-zero local syndrome are compacted into a list (others score <= 0),
//   2. the list is scored in chunks of 64 lanes (gen_best_score: 3 VALU per
//      subset), each generator's key cached in LDS,
//   3. a DPP wave max over the cached (score, -g) keys picks the generator, and
//      the lowest subset reaching that score is found lane-parallel
//      (spec: ties -> lowest g, then lowest subset bitmask),
//   4. the flip updates the residual (u32 per check in LDS) and hard decision.
// Key (int32): score << 15 | (127 - g) << 8; |score| <= 32*840 < 2^15, g < 128.
constexpr int kSsfWaves = 4;  // waves per workgroup sharing the generator tables
// Registers are budgeted for 5 waves per SIMD (<= 96 VGPRs, ~40 dwords of the
// shot setup / finalisation spilled): with the u8 residual five 4-wave
// workgroups fit a CU's LDS.  Measured against 4 per SIMD with a u32 residual,
// interleaved: isolated SSF sum 6.57-6.59 vs 6.76-6.78 ms, headline 87.7-89.2 vs
// 85.8-86.5 M shots/s (the smaller LDS footprint also co-resides better with the
// concurrent BP kernels).
constexpr int kSsfOcc = 5;  // minimum waves per SIMD the SSF kernel is compiled for
using SsfRes = uint8_t;     // residual bit per check

template <int RG>
struct SsfLds {
    static constexpr int GP = 64 * RG;
    static constexpr int kStage = 3;  // packed queue entries staged per wave (two slots ahead)
    __host__ __device__ static size_t table_bytes() { return (size_t)GP * 4 * (kGenW + kGenLC / 4 + kGenW / 2); }
    __host__ __device__ static size_t lz_bytes(const DevGraph& g) {
        return lz_in_lds(g) ? ((size_t)g.k * g.lz_words * 8 + 15) / 16 * 16 : 0;
    }
    __host__ __device__ static size_t inv_bytes(const DevGraph& g) {
        return g.g_inv ? ((size_t)g.m_pad * g.g_invd * 2 + 15) / 16 * 16 : 0;
    }
    __host__ __device__ static size_t shared_bytes(const DevGraph& g) { return table_bytes() + lz_bytes(g) + inv_bytes(g); }
    // residual, cached keys, listed local syndromes, current local syndromes,
    // flipped-check list, listed generators, hard decision, staged queue entries
    __host__ __device__ static size_t res_bytes(const DevGraph& g) {
        return (((size_t)g.m_pad + 64) * sizeof(SsfRes) + 15) / 16 * 16;
    }
    __host__ __device__ static size_t wave_bytes(const DevGraph& g) {
        return res_bytes(g) + ((size_t)GP * 4 * 3 + kGenLC * 4 + GP + (size_t)g.n_pad + 64 + 15) / 16 * 16 +
               256 * kStage;
    }
};

// XW/RW: words of the packed queue entries (hard decision by column, residual
// by check) written by the wave BP kernels (queue_push_packed).
template <int RG, int XW, int RW>
__global__ __launch_bounds__(64 * kSsfWaves, kSsfOcc) void ssf_wave_kernel(DevGraph g, DecodeArgs a) {
    constexpr int GP = SsfLds<RG>::GP;
    constexpr int QW = QEntry<XW, RW>::QW;
    static_assert(2 * QW <= 64, "entry staging");
    constexpr int NLW = kGenLC / 4;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    // shared: qubit local-check masks, packed u8 local-check ids, packed u16 qubit ids
    uint32_t* qmt = reinterpret_cast<uint32_t*>(smem);  // [kGenW][GP]
    uint32_t* lct = qmt + kGenW * GP;                   // [NLW][GP]   (pad id m_pad -> zero residual)
    uint32_t* qt = lct + NLW * GP;                      // [kGenW/2][GP]
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint64_t* lzs_lds = reinterpret_cast<uint64_t*>(smem + SsfLds<RG>::table_bytes());
    const uint64_t* lzs = lzs_lds;  // LDS copy when lz_in_lds (lz_word / lz_row_parity)
    uint16_t* invt = reinterpret_cast<uint16_t*>(smem + SsfLds<RG>::table_bytes() + SsfLds<RG>::lz_bytes(g));
    const bool inc = g.g_inv != nullptr;  // incremental local syndromes
    unsigned char* wbase = smem + SsfLds<RG>::shared_bytes(g) + (size_t)wave * SsfLds<RG>::wave_bytes(g);
    SsfRes* sres = reinterpret_cast<SsfRes*>(wbase);          // [m_pad + 64] residual (pads stay 0)
    int* key = reinterpret_cast<int*>(wbase + SsfLds<RG>::res_bytes(g));  // [GP] cached best keys
    uint32_t* slt = reinterpret_cast<uint32_t*>(key + GP);    // [GP] local syndromes of listed gens
    uint32_t* slc = slt + GP;                                 // [GP] current local syndromes (inc)
    uint32_t* clist = slc + GP;                               // [kGenLC] checks flipped by a step (inc)
    uint8_t* list = reinterpret_cast<uint8_t*>(clist + kGenLC);  // [GP] listed generators
    uint8_t* xh = list + GP;                                  // [n_pad + 64]
    uint8_t* ent = wbase + SsfLds<RG>::wave_bytes(g) - 256 * SsfLds<RG>::kStage;  // [kStage][256] queue entries
    const int m = g.m, n = g.n;

    for (int e = threadIdx.x; e < GP; e += 64 * kSsfWaves) {
#pragma unroll
        for (int k = 0; k < kGenW; ++k) qmt[k * GP + e] = g.g_qmask[k * g.g_pad + e];
#pragma unroll
        for (int wq = 0; wq < NLW; ++wq) lct[wq * GP + e] = g.g_lc8[wq * g.g_pad + e];
#pragma unroll
        for (int k = 0; k < kGenW / 2; ++k)
            qt[k * GP + e] = (uint32_t)g.g_q[(2 * k) * g.g_pad + e] | ((uint32_t)g.g_q[(2 * k + 1) * g.g_pad + e] << 16);
    }
    if (lz_in_lds(g))
        for (int e = threadIdx.x; e < g.k * g.lz_words; e += 64 * kSsfWaves) lzs_lds[e] = g.lz[e];
    if (inc)
        for (int e = threadIdx.x; e < g.m_pad * g.g_invd; e += 64 * kSsfWaves) invt[e] = g.g_inv[e];
    for (int e = lane; e < g.m_pad + 64; e += 64) sres[e] = 0;
    for (int e = lane; e < g.n_pad + 64; e += 64) xh[e] = 0;
    __syncthreads();

    const int count = *a.q_count;
    // entry of queue slot `sl` into staging buffer `b` (one LDS-DMA load; past
    // the queue end it re-reads entry 0, so every stage issues exactly one)
    auto stage_entry = [&](int sl, int b) {
        const int64_t e = sl < count ? sl : 0;
        const uint8_t* src = reinterpret_cast<const uint8_t*>(a.q_w + e * QW) + 4 * min(lane, 2 * QW - 1);
        __builtin_amdgcn_global_load_lds(src, ent + 256 * b, 4, 0, 0);
    };
    const int stride = gridDim.x * kSsfWaves;
    const bool lean_fin = !a.x_out && !a.corr_out && !a.base && g.fold_blocks == 1;
    const bool want_fail = a.fail && a.readout && g.k > 0;
    const int nhi = g.g_wmax > 4 ? (1 << (g.g_wmax - 4)) : 1;
    // the split scorer enumerates hi < 8 per lane (generators of up to 8 qubits
    // have nhi <= 16, half <= 8); QD_SSF_SCAN_NOSPLIT disables it
    const bool split_ok = nhi <= 16 && !a.ssf_nosplit;
    const int nlcw = (g.g_nlcmax + 3) / 4;
    QDEC_STAMP_DECL
    // queue slots in guided order (ShotSeq: static stride, then counter chunks;
    // a shot's SSF cost varies with its step count, so a static split leaves a
    // tail of waves still working); the counter is zeroed with q_count.
    // Queues of < 16 slots per wave stay static: there the counter's
    // same-address atomics cost more than the tail they would balance
    // (measured: p = 0.018, 8.5 slots per wave, 0.14 -> 0.21 ms per launch).
    unsigned long long* sctr = a.wave_ctr && count >= 16 * stride ? a.wave_ctr + 1 : nullptr;
    ShotSeq seq(count, sctr, (int64_t)blockIdx.x * kSsfWaves + wave, stride, lane);
    int64_t slot = seq.next(lane);
    int64_t slot1 = seq.next(lane);
    stage_entry((int)min(slot, (int64_t)count), 0);
    stage_entry((int)min(slot1, (int64_t)count), 1);
    int sb = 0;
    for (; slot < count; sb = sb == 2 ? 0 : sb + 1) {
        QDEC_STAMP(12);
        // entry staged two slots ahead; the next slot's stage is younger (a
        // counter request issued between them is older and is waited for too)
        wait_vmem<1>();
        const uint64_t* ew = reinterpret_cast<const uint64_t*>(ent + 256 * sb);
        const int64_t shot = (int64_t)ew[0];
        uint64_t X[XW], R[RW];
#pragma unroll
        for (int w = 0; w < XW; ++w) X[w] = ew[1 + w];
#pragma unroll
        for (int w = 0; w < RW; ++w) R[w] = ew[1 + XW + w];
        wait_lds();
        const int64_t slot2 = seq.next(lane);
        stage_entry((int)min(slot2, (int64_t)count), sb == 0 ? 2 : sb - 1);
#pragma unroll
        for (int w = 0; w < XW; ++w) {
            const int j = w * 64 + lane;
            xh[j] = j < n ? (uint8_t)((X[w] >> lane) & 1) : (uint8_t)0;
        }
        int sw = 0;
#pragma unroll
        for (int w = 0; w < RW; ++w) {
            const int i = w * 64 + lane;
            sres[i] = i < m ? (SsfRes)((R[w] >> lane) & 1) : (SsfRes)0;
            sw += __popcll(R[w]);
        }
        wave_lds_sync();
        uint32_t slo[RG];
        int steps = 0;
        bool first = true;
        while (sw > 0 && (a.ssf_max_steps <= 0 || steps < a.ssf_max_steps)) {
            // ---- 1. local syndromes (gathered from the residual on the first
            // step, afterwards kept current by step 4); compact the changed,
            // non-zero ones ----
            int nl = 0;
#pragma unroll
            for (int rg = 0; rg < RG; ++rg) {
                const int gi = rg * 64 + lane;
                uint32_t sl = 0;
                if (!inc || first) {
#pragma unroll
                    for (int wq = 0; wq < NLW; ++wq) {
                        if (wq < nlcw) {
                            const uint32_t pk = lct[wq * GP + gi];
#pragma unroll
                            for (int bb = 0; bb < 4; ++bb) sl |= (uint32_t)sres[(pk >> (8 * bb)) & 0xff] << (wq * 4 + bb);
                        }
                    }
                    if (inc) slc[gi] = sl;
                } else {
                    sl = slc[gi];
                }
                const bool changed = first || sl != slo[rg];
                slo[rg] = sl;
                const bool need = changed && sl != 0u;
                if (changed && !need) key[gi] = INT_MIN;
                const unsigned long long bal = __ballot(need);
                if (need) {
                    const int pos = nl + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                    list[pos] = (uint8_t)gi;
                    slt[pos] = sl;
                }
                nl += __popcll(bal);
            }
            first = false;
            wave_lds_sync();
            QDEC_STAMP(0);
            QDEC_COUNT(5, nl);
            // ---- 2. score the listed generators (<= 32 listed and >= 5 qubits:
            // two lanes per generator, each half of its subsets) ----
            if (nl <= 32 && nhi >= 2 && split_ok) {
                const bool four = nl <= 16 && nhi >= 4;
                const int sw = four ? 16 : 32;
                const int idx = lane & (sw - 1);
                const int q = lane / sw;
                uint32_t sl = 0, qm[kGenW];
                int gg = 0;
                if (idx < nl) {
                    gg = list[idx];
                    sl = slt[idx];
                }
#pragma unroll
                for (int k = 0; k < kGenW; ++k) qm[k] = idx < nl ? qmt[k * GP + gg] : 0u;
                uint32_t tq[2] = {0u, 0u};  // the generator's last two qubit masks (wmax-1, wmax-2)
#pragma unroll
                for (int k = 0; k < kGenW; ++k) {
                    if (k == g.g_wmax - 1) tq[0] = qm[k];
                    if (k == g.g_wmax - 2) tq[1] = qm[k];
                }
                const int sc = four ? gen_best_score_split<4>(sl, qm, nhi / 4, tq, q)
                                    : gen_best_score_split<2>(sl, qm, nhi / 2, tq, q);
                if (q == 0 && idx < nl) key[gg] = (int)(((unsigned)sc << 15) | ((unsigned)(127 - gg) << 8));
            } else
            for (int c0 = 0; c0 < nl; c0 += 64) {
                const int idx = c0 + lane;
                if (idx < nl) {
                    const int gg = list[idx];
                    const uint32_t sl = slt[idx];
                    uint32_t qm[kGenW];
#pragma unroll
                    for (int k = 0; k < kGenW; ++k) qm[k] = qmt[k * GP + gg];
                    const int sc = gen_best_score(sl, qm, nhi);
                    key[gg] = (int)(((unsigned)sc << 15) | ((unsigned)(127 - gg) << 8));
                }
            }
            wave_lds_sync();
            QDEC_STAMP(1);
            // ---- 3. pick (score, -g), then the lowest subset reaching the score ----
            int kv = INT_MIN;
#pragma unroll
            for (int rg = 0; rg < RG; ++rg) kv = max(kv, key[rg * 64 + lane]);
            const int best = wave_max_i32(kv);
            const int score = best >> 15;
            if (score <= 0) break;
            const int gsel = 127 - ((best >> 8) & 127);
            const int owner = gsel & 63, rsel = gsel >> 6;
            uint32_t slg = 0;
#pragma unroll
            for (int rg = 0; rg < RG; ++rg)
                if (rg == rsel) slg = (uint32_t)__builtin_amdgcn_readlane((int)slo[rg], owner);
            const int base = __builtin_popcount(slg);
            // lane k < kGenW holds qubit k's mask of the chosen generator
            const uint32_t qk = lane < kGenW ? qmt[lane * GP + gsel] : 0u;
            int tsel = -1;
            uint32_t qs[kGenW];  // the chosen generator's qubit masks, broadcast once
#pragma unroll
            for (int k = 0; k < kGenW; ++k) qs[k] = (uint32_t)__builtin_amdgcn_readlane((int)qk, k);
            for (int t0 = 0; t0 < 16 * nhi; t0 += 64) {
                const int t = t0 + lane;
                uint32_t mt = 0;
#pragma unroll
                for (int k = 0; k < kGenW; ++k) mt ^= ((t >> k) & 1) ? qs[k] : 0u;
                const int gain = base - __builtin_popcount(slg ^ mt);
                const bool hit = t > 0 && t < 16 * nhi && gain * kSsfScale == score * __builtin_popcount(t);
                const unsigned long long hb = __ballot(hit);
                if (hb) {
                    tsel = t0 + __builtin_ctzll(hb);
                    break;
                }
            }
            if (tsel < 0) break;  // unreachable: the best score is some subset's score
            QDEC_STAMP(2);
            // ---- 4. apply the flip ----
            const uint32_t fm = (uint32_t)wave_xor_masked(lane < kGenW && ((tsel >> lane) & 1) ? qk : 0u);
            const int gain = score * __builtin_popcount(tsel) / kSsfScale;
            if (lane < kGenLC && ((fm >> lane) & 1)) {
                const uint32_t wv = lct[(lane >> 2) * GP + gsel];
                const uint32_t c = (wv >> (8 * (lane & 3))) & 0xff;
                sres[c] ^= (SsfRes)1;
                clist[__builtin_popcount(fm & ((1u << lane) - 1u))] = c;
            }
            if (inc) {
                // every generator with a flipped check as local check `bit`
                // toggles that bit: (check, entry) pairs spread over the lanes
                wave_lds_sync();
                const int npair = __builtin_popcount(fm) << g.g_invl;
                for (int pr = lane; pr < npair; pr += 64) {
                    const uint32_t e = invt[(clist[pr >> g.g_invl] << g.g_invl) + (pr & (g.g_invd - 1))];
                    if (e != 0xffffu) atomicXor(&slc[e & 0xff], 1u << (e >> 8));
                }
            }
            if (lane < kGenW && ((tsel >> lane) & 1)) {
                const uint32_t qv = qt[(lane >> 1) * GP + gsel];
                xh[(qv >> (16 * (lane & 1))) & 0xffff] ^= 1;
            }
            wave_lds_sync();
            sw -= gain;
            ++steps;
            QDEC_STAMP(3);
            QDEC_COUNT(6, 1);
        }
        QDEC_STAMP(13);
        if (lean_fin) {
            int any_fail = 0;
            if (want_fail) {  // readout words came with the queue entry
                // the readout words are re-read from this slot's staging buffer
                // (restaged only by the next slot), not held across the steps
                // (q_rpar: the entry holds the readout's logical parities, bit r
                // of word r / 64, instead of the readout words)
                const bool rpar = a.q_rpar != 0;
                uint64_t Rd[XW];
#pragma unroll
                for (int w = 0; w < XW; ++w) Rd[w] = __ballot(xh[w * 64 + lane] & 1) ^ (rpar ? 0ull : ew[1 + XW + RW + w]);
                QDEC_STAMP(8);
                int f = 0;
#pragma unroll
                for (int rr = 0; rr < kMaxLogicalRounds; ++rr) {
                    const int r = rr * 64 + lane;
                    if (r < g.k)
                        f |= lz_row_parity<XW>(g, lzs, r, Rd) ^
                             (rpar && rr < XW ? (int)((ew[1 + XW + RW + (rr < XW ? rr : 0)] >> lane) & 1) : 0);
                }
                any_fail = __ballot(f) != 0ull;
                QDEC_STAMP(9);
            }
            if (lane == 0) {
                if (a.status) a.status[shot] = (uint8_t)(sw == 0 ? 2 : 0);
                if (a.ssf_steps) a.ssf_steps[shot] = steps;
                if (a.fail) a.fail[shot] = (uint8_t)any_fail;
            }
        } else {
            finalize_shot(g, a, shot, xh, false, sw == 0, steps, lane);
        }
        QDEC_STAMP(14);
        QDEC_COUNT(7, 1);
        wave_lds_sync();
        slot = slot1;
        slot1 = slot2;
    }
    QDEC_FLUSH_AT(16);
}

// ============================================================== SSF, table-driven
// ssf_lut_kernel: the same spec as ssf_wave_kernel with the per-generator subset
// search replaced by one LDS table lookup (DevGraph::s_lut, built by
// ssf_lut_tables in qdec_abi.cpp): the best (score, subset) of a generator is a
// function of its <= 16-bit local syndrome.  One wave per queued shot; lane l
// owns generators l and 64 + l, whose local syndromes it keeps in registers
// (one u32: generator l in the low half-word).  A step is
//   1. two table reads -> key (rank, -g, t) per generator, a DPP wave max;
//   2. the winner's entry and local syndrome from its owner lane (readlane);
//   3. for every check the flip toggles, one coalesced read of that check's
//      toggle row (s_tog: the local-syndrome bits of every lane's generators),
//      XORed into the registers; lanes k < 8 toggle the hard-decision byte of
//      the winner's qubit k when it is in the subset (qubit ids from an LDS
//      table; nothing waits for these writes until the shot's end).
// Two dependent LDS round trips per step and no LDS writes, against the scanning
// kernel's gather / list / score / pick / apply chain.  The shot's first local
// syndromes are the toggle rows of its residual's violated checks.
constexpr int kLutWaves = 16;  // waves per workgroup sharing the tables
constexpr int kLutOcc = 8;     // waves per SIMD the table-driven kernel is compiled for (lean build)

struct SsfLutLds {
    static constexpr int kStage = 3;  // packed queue entries staged per wave (two slots ahead)
    __host__ __device__ static size_t lut_bytes(const DevGraph& g) { return ((size_t)g.s_lut_n * 4 + 15) / 16 * 16; }
    // toggle rows [m_pad + 1][64] (the last one zero)
    __host__ __device__ static size_t tog_bytes(const DevGraph& g) { return ((size_t)g.m_pad + 1) * 64 * 4; }
    __host__ __device__ static size_t lz_bytes(const DevGraph& g) {
        return lz_in_lds(g) ? ((size_t)g.k * g.lz_words * 8 + 15) / 16 * 16 : 0;
    }
    static constexpr size_t qt_bytes = (size_t)(kGenW / 2) * 128 * 4;  // qubit id pairs [kGenW/2][128]
    __host__ __device__ static size_t shared_bytes(const DevGraph& g) {
        return lut_bytes(g) + tog_bytes(g) + qt_bytes + lz_bytes(g);
    }
    // staged queue entries, hard decision as bit words (u32 [n_pad / 32]), the
    // step log (u16 [m_pad]: a shot takes at most m steps), hard decision bytes
    // (non-lean finalisation)
    __host__ __device__ static size_t wave_bytes(const DevGraph& g) {
        return 256 * kStage + (size_t)g.n_pad / 8 + ((size_t)g.m_pad * 2 + 15) / 16 * 16 +
               ((size_t)g.n_pad + 64 + 15) / 16 * 16;
    }
};

// LEAN: outputs are status, SSF steps and the failure flag only (the bench's and
// p_sweep's call); otherwise finalize_shot writes x / corr (its registers would
// push the lean build past 64 VGPRs, 8 waves per SIMD).
template <int RG, int XW, int RW, bool LEAN>
__global__ __launch_bounds__(64 * kLutWaves, LEAN ? kLutOcc : 4) void ssf_lut_kernel(DevGraph g, DecodeArgs a) {
    static_assert(RG == 1 || RG == 2, "two generators per lane at most (16-bit halves of one word)");
    static_assert(XW <= 32, "hard-decision bits per lane");
    constexpr int QW = QEntry<XW, RW>::QW;
    static_assert(2 * QW <= 64, "entry staging");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t* lut = reinterpret_cast<uint32_t*>(smem);
    uint32_t* tog = reinterpret_cast<uint32_t*>(smem + SsfLutLds::lut_bytes(g));
    uint32_t* qt = reinterpret_cast<uint32_t*>(smem + SsfLutLds::lut_bytes(g) + SsfLutLds::tog_bytes(g));
    uint64_t* lzs = reinterpret_cast<uint64_t*>(smem + SsfLutLds::lut_bytes(g) + SsfLutLds::tog_bytes(g) +
                                                SsfLutLds::qt_bytes);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    unsigned char* wbase = smem + SsfLutLds::shared_bytes(g) + (size_t)wave * SsfLutLds::wave_bytes(g);
    uint8_t* ent = wbase;                                  // [kStage][256] queue entries
    uint32_t* xb = reinterpret_cast<uint32_t*>(wbase + 256 * SsfLutLds::kStage);  // [n_pad / 32] hard decision bits
    uint16_t* flog = reinterpret_cast<uint16_t*>(xb + g.n_pad / 32);                 // [m_pad] (g, t) of every step
    uint8_t* xh = reinterpret_cast<uint8_t*>(flog) + ((size_t)g.m_pad * 2 + 15) / 16 * 16;  // [n_pad + 64] bytes

    {   // tables -> LDS, 16-B copies (every size is a multiple of 16 B)
        const uint4* src = reinterpret_cast<const uint4*>(g.s_lut);
        uint4* dst = reinterpret_cast<uint4*>(lut);
        const int nl = (int)(SsfLutLds::lut_bytes(g) / 16);
        for (int e = threadIdx.x; e < nl; e += 64 * kLutWaves) dst[e] = src[e];
        src = reinterpret_cast<const uint4*>(g.s_tog);
        dst = reinterpret_cast<uint4*>(tog);
        const int nt = (int)(SsfLutLds::tog_bytes(g) / 16);
        for (int e = threadIdx.x; e < nt; e += 64 * kLutWaves) dst[e] = src[e];
    }
    if (lz_in_lds(g))
        for (int e = threadIdx.x; e < g.k * g.lz_words; e += 64 * kLutWaves) lzs[e] = g.lz[e];
    for (int e = threadIdx.x; e < 64 * RG; e += 64 * kLutWaves)
#pragma unroll
        for (int k = 0; k < kGenW / 2; ++k)
            qt[k * 128 + e] = (uint32_t)g.g_q[(2 * k) * g.g_pad + e] | ((uint32_t)g.g_q[(2 * k + 1) * g.g_pad + e] << 16);
    for (int e = lane; e < g.n_pad + 64; e += 64) xh[e] = 0;
    // this lane's generators: table offsets, canonical local checks
    uint32_t off[RG], lcw[RG][kLutLCW];
#pragma unroll
    for (int rg = 0; rg < RG; ++rg) {
        const int gi = rg * 64 + lane;
        off[rg] = g.s_off[gi];
#pragma unroll
        for (int w = 0; w < kLutLCW; ++w) lcw[rg][w] = g.s_lcw[w * g.g_pad + gi];
    }
    __syncthreads();

    const int count = *a.q_count;
    auto stage_entry = [&](int sl, int b) {  // as ssf_wave_kernel: one LDS-DMA load per stage
        const int64_t e = sl < count ? sl : 0;
        const uint8_t* src = reinterpret_cast<const uint8_t*>(a.q_w + e * QW) + 4 * min(lane, 2 * QW - 1);
        __builtin_amdgcn_global_load_lds(src, ent + 256 * b, 4, 0, 0);
    };
    const int stride = gridDim.x * kLutWaves;
    const bool lean_fin = LEAN;
    const bool want_fail = a.fail && a.readout && g.k > 0;
    const bool rpar = a.q_rpar != 0;
    unsigned long long* sctr = a.wave_ctr && count >= 16 * stride ? a.wave_ctr + 1 : nullptr;
    ShotSeq seq(count, sctr, (int64_t)blockIdx.x * kLutWaves + wave, stride, lane);
    int64_t slot = seq.next(lane);
    int64_t slot1 = seq.next(lane);
    stage_entry((int)min(slot, (int64_t)count), 0);
    stage_entry((int)min(slot1, (int64_t)count), 1);
    int sb = 0;
    for (; slot < count; sb = sb == 2 ? 0 : sb + 1) {
        wait_vmem<1>();
        const uint64_t* ew = reinterpret_cast<const uint64_t*>(ent + 256 * sb);
        const int64_t shot = (int64_t)ew[0];
        if (lane < 2 * XW) xb[lane] = reinterpret_cast<const uint32_t*>(ew + 1)[lane];
        uint64_t R[RW];  // residual words (uniform)
#pragma unroll
        for (int w = 0; w < RW; ++w) {
            const uint64_t v = ew[1 + XW + w];
            R[w] = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v) |
                   ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32)) << 32);
        }
        wait_lds();
        const int64_t slot2 = seq.next(lane);
        stage_entry((int)min(slot2, (int64_t)count), sb == 0 ? 2 : sb - 1);
        // first local syndromes: the toggle rows of the violated checks, 8 rows
        // per round (independent LDS reads, one wait; row m_pad is all zero)
        const uint32_t zrow = (uint32_t)g.m_pad;
        uint32_t sl = 0;
        int sw = 0;
#pragma unroll
        for (int w = 0; w < RW; ++w) {
            uint64_t bits = R[w];
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
        while (sw > 0 && (a.ssf_max_steps <= 0 || steps < a.ssf_max_steps)) {
            // ---- 1. every generator's best (rank, -g, t); wave max ----
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
            // ---- 2. the winner's toggled checks and gain (owner lane) ----
            const uint32_t esel = (uint32_t)__builtin_amdgcn_readlane((int)(hi ? e[RG - 1] : e[0]), owner);
            const uint32_t slg = ((uint32_t)__builtin_amdgcn_readlane((int)sl, owner) >> (hi ? 16 : 0)) & 0xffffu;
            const uint32_t fm = (esel >> 8) & 0xffffu;
            sw -= __builtin_popcount(slg) - __builtin_popcount(slg ^ fm);
            ++steps;
            // ---- 3. toggle the flipped checks' local-syndrome bits: one read
            // of a toggle row per flipped check, each behind a uniform branch and
            // all issued before the first XOR (one LDS round trip); flip the qubits ----
            uint32_t tr[kLutLC];
#pragma unroll
            for (int w = 0; w < kLutLCW; ++w) {
                const uint32_t nib = (fm >> (4 * w)) & 0xfu;
                const uint32_t word =
                    nib ? (uint32_t)__builtin_amdgcn_readlane((int)(hi ? lcw[RG - 1][w] : lcw[0][w]), owner) : 0u;
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
            // the flip itself is logged (steps <= m: every step lowers |s|) and
            // applied to the hard decision once, after the last step
            if (lane == 0) flog[steps - 1] = (uint16_t)(gsel | (tsel << 8));
        }
        wave_lds_sync();
        // x ^= 1_F of every logged step: lane s takes step s, its qubits' bits by
        // LDS atomic XOR (a qubit flipped twice cancels, in any order)
        for (int b0 = 0; b0 < steps; b0 += 64) {
            if (b0 + lane < steps) {
                const uint32_t e = flog[b0 + lane];
                const int gg = (int)(e & 0xffu);
#pragma unroll
                for (int k = 0; k < kGenW; ++k)
                    if ((e >> (8 + k)) & 1u) {
                        const uint32_t q = (qt[(k >> 1) * 128 + gg] >> (16 * (k & 1))) & 0xffffu;
                        atomicXor(&xb[q >> 5], 1u << (q & 31));
                    }
            }
        }
        wave_lds_sync();
        if (lean_fin) {
            uint64_t X[XW];
#pragma unroll
            for (int w = 0; w < XW; ++w) X[w] = (uint64_t)xb[2 * w] | ((uint64_t)xb[2 * w + 1] << 32);
            int any_fail = 0;
            if (want_fail) {  // the entry carries the readout words or (q_rpar) its logical parities
                uint64_t Rd[XW];
#pragma unroll
                for (int w = 0; w < XW; ++w) Rd[w] = X[w] ^ (rpar ? 0ull : ew[1 + XW + RW + w]);
                int f = 0;
#pragma unroll
                for (int rr = 0; rr < kMaxLogicalRounds; ++rr) {
                    const int r = rr * 64 + lane;
                    if (r < g.k)
                        f |= lz_row_parity<XW>(g, lzs, r, Rd) ^
                             (rpar && rr < XW ? (int)((ew[1 + XW + RW + (rr < XW ? rr : 0)] >> lane) & 1) : 0);
                }
                any_fail = __ballot(f) != 0ull;
            }
            if (lane == 0) {
                if (a.status) a.status[shot] = (uint8_t)(sw == 0 ? 2 : 0);
                if (a.ssf_steps) a.ssf_steps[shot] = steps;
                if (a.fail) a.fail[shot] = (uint8_t)any_fail;
            }
        } else if constexpr (!LEAN) {
#pragma unroll
            for (int w = 0; w < XW; ++w) xh[w * 64 + lane] = (uint8_t)((xb[2 * w + (lane >> 5)] >> (lane & 31)) & 1u);
            wave_lds_sync();
            finalize_shot(g, a, shot, xh, false, sw == 0, steps, lane);
        }
        wave_lds_sync();
        slot = slot1;
        slot1 = slot2;
    }
}

// ---------------------------------------------------------------- launcher
LaunchNames& last_launch_names() {
    static thread_local LaunchNames n;
    return n;
}

template <typename T>
static size_t wave_lds_bytes(const DevGraph& g) {
    constexpr int DRS = lds_stride<T, kDR>();
    constexpr int DCS = lds_stride<T, kDC>();
    return ((size_t)g.m_pad * DRS + 64) * sizeof(T) + ((size_t)g.n_pad * DCS + 64) * sizeof(T) +
           (size_t)g.n_pad + 64;
}

template <int RG, int XW, int RW>
static int launch_ssf_wave(const DevGraph& g, const DecodeArgs& a, int num_cus, hipStream_t stream) {
    // the fused failure check reads the dense logical table's LDS copy (as launch_bp_wave)
    if (a.fail && g.k > 0 && !g.lz) return (int)hipErrorInvalidValue;
    const size_t lds = SsfLds<RG>::shared_bytes(g) + kSsfWaves * SsfLds<RG>::wave_bytes(g);
    if (lds > 64 * 1024) {
        const hipError_t ea = hipFuncSetAttribute(reinterpret_cast<const void*>(ssf_wave_kernel<RG, XW, RW>),
                                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (ea != hipSuccess) return (int)ea;
    }
    int per_cu = 0;
    hipError_t e =
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ssf_wave_kernel<RG, XW, RW>, 64 * kSsfWaves, lds);
    if (e != hipSuccess) return (int)e;
    if (per_cu <= 0) return (int)hipErrorInvalidConfiguration;
    long long grid = (long long)num_cus * per_cu;
    const long long need = (a.B + kSsfWaves - 1) / kSsfWaves;  // queue length <= B
    if (grid > need) grid = need;
    if (grid <= 0) return 0;
    QDEC_NOTE_SSF("qdec::ssf_wave_kernel", RG, XW, RW);
    hipLaunchKernelGGL((ssf_wave_kernel<RG, XW, RW>), dim3((unsigned)grid), dim3(64 * kSsfWaves), lds, stream, g, a);
    return (int)hipGetLastError();
}

template <int RG, int XW, int RW, bool LEAN>
static int launch_ssf_lut_t(const DevGraph& g, const DecodeArgs& a, int num_cus, hipStream_t stream) {
    const size_t lds = SsfLutLds::shared_bytes(g) + kLutWaves * SsfLutLds::wave_bytes(g);
    if (lds > 160 * 1024) return (int)hipErrorInvalidConfiguration;
    if (lds > 64 * 1024) {
        const hipError_t ea = hipFuncSetAttribute(reinterpret_cast<const void*>(ssf_lut_kernel<RG, XW, RW, LEAN>),
                                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (ea != hipSuccess) return (int)ea;
    }
    int per_cu = 0;
    hipError_t e =
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ssf_lut_kernel<RG, XW, RW, LEAN>, 64 * kLutWaves, lds);
    if (e != hipSuccess) return (int)e;
    if (per_cu <= 0) return (int)hipErrorInvalidConfiguration;
    long long grid = (long long)num_cus * per_cu;
    const long long need = (a.B + kLutWaves - 1) / kLutWaves;  // queue length <= B
    if (grid > need) grid = need;
    if (grid <= 0) return 0;
    QDEC_NOTE_SSF("qdec::ssf_lut_kernel", RG, XW, RW, LEAN);
    hipLaunchKernelGGL((ssf_lut_kernel<RG, XW, RW, LEAN>), dim3((unsigned)grid), dim3(64 * kLutWaves), lds, stream, g,
                       a);
    return (int)hipGetLastError();
}

template <int RG, int XW, int RW>
static int launch_ssf_lut(const DevGraph& g, const DecodeArgs& a, int num_cus, hipStream_t stream) {
    if (a.fail && g.k > 0 && !g.lz) return (int)hipErrorInvalidValue;
    const bool lean = !a.x_out && !a.corr_out && !a.base && g.fold_blocks == 1;
    return lean ? launch_ssf_lut_t<RG, XW, RW, true>(g, a, num_cus, stream)
                : launch_ssf_lut_t<RG, XW, RW, false>(g, a, num_cus, stream);
}

template <typename K>
static int launch_persistent(K kern, size_t lds, int64_t work, int num_cus, hipStream_t stream, const DevGraph& g,
                             const DecodeArgs& a, int block = 64, int max_per_cu = 0) {
    if (lds > 64 * 1024) {  // e.g. a large LDS copy of the logicals (lz_in_lds)
        const hipError_t ea = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (ea != hipSuccess) return (int)ea;
    }
    int per_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, block, lds);
    if (e != hipSuccess) return (int)e;
    if (per_cu <= 0) return (int)hipErrorInvalidConfiguration;
    if (max_per_cu > 0 && per_cu > max_per_cu) per_cu = max_per_cu;
    // one-wave blocks: a multiple of 4 per CU puts the same number of waves on
    // every SIMD (11 f64 waves would sit 3/3/3/2 and run slower than 8)
    if (block == 64 && per_cu > 4) per_cu &= ~3;
    long long grid = (long long)num_cus * per_cu;
    if (grid > work) grid = work;
    if (grid <= 0) return 0;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(block), lds, stream, g, a);
    return (int)hipGetLastError();
}

// BP kernel of a wave shape: min-sum uses the compressed-state kernel, product-sum
// the message-array kernel.
// Lean launches: no x / corr / llr outputs, no base, no syndrome flags, no fold.
static bool lean_launch(const DevGraph& g, const DecodeArgs& a, bool defer) {
    return !a.x_out && !a.corr_out && !a.llr_out && !a.base && !a.syn_flags && g.fold_blocks == 1 &&
           (!defer || a.q_packed);
}

// The two-pass compact path (ms_triage_kernel + bp_ms_cmp_kernel) serves lean
// min-sum launches whose graph has the slot-order logicals (or no fused check);
// QDEC_COMPACT=0 keeps the one-pass kernel (A/B, parity tests run both).
static bool compact_launch(const DevGraph& g, const DecodeArgs& a, bool defer) {
    // the triage reads 16-B chunks of byte rows (16-B aligned syndrome / readout
    // buffers only) or u64 words of packed rows (8-B aligned, checked by the ABI);
    // its list counters take u64 atomics (natural alignment), entries 16-B stores
    const uintptr_t al = a.in_packed ? 7 : 15;
    if ((reinterpret_cast<uintptr_t>(a.syn) & al) || (a.readout && (reinterpret_cast<uintptr_t>(a.readout) & al)))
        return false;
    if ((reinterpret_cast<uintptr_t>(a.cmp_count) & 127) || (reinterpret_cast<uintptr_t>(a.cmp) & 15)) return false;
    const bool want_fail = a.fail && a.readout && g.k > 0;
    return g.opt_compact && a.cmp && a.cmp_count && a.syn && lean_launch(g, a, defer) && (!want_fail || g.ms_lzs);
}

template <int RC, int RV>
static int launch_triage(const DevGraph& g, const DecodeArgs& a, hipStream_t stream) {
    const bool want_fail = a.fail && a.readout && g.k > 0;
    // the tile loads are 16-B vector loads (packed rows: u64 loads)
    const uintptr_t al = a.in_packed ? 7 : 15;
    if ((reinterpret_cast<uintptr_t>(a.syn) & al) || (want_fail && (reinterpret_cast<uintptr_t>(a.readout) & al)))
        return (int)hipErrorInvalidValue;
    if (a.it1_lut && (!g.it1_vchk || !g.it1_cvar || g.m_pad != 64 * RC || g.n_pad != 64 * RV))
        return (int)hipErrorInvalidValue;
    // the logicals, the tile images, the iteration-1 words (byte images: over
    // the images; the kernel's layout, ms_triage_kernel)
    const size_t tiles =
        a.in_packed ? 0 : triage_img_bytes(64 * (int64_t)g.m) + triage_img_bytes(64 * (int64_t)g.n_data);
    const size_t it1 = a.it1_lut ? TriageIt1<RC, RV>::bytes : 0;
    const size_t lds = ((want_fail ? (size_t)g.k * g.lz_words * 8 : 0) + 15) / 16 * 16 +
                       tiles + it1;
    const void* fn = a.in_packed ? reinterpret_cast<const void*>(ms_triage_kernel<RC, RV, true>)
                                 : reinterpret_cast<const void*>(ms_triage_kernel<RC, RV, false>);
    if (lds > 64 * 1024) {  // large logical tables (k <= 256, lz_words <= 9)
        const hipError_t ea = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (ea != hipSuccess) return (int)ea;
    }
    const dim3 grid((unsigned)((a.B + 63) / 64));
    if (a.in_packed) {
        QDEC_NOTE_PRE("qdec::ms_triage_kernel", RC, RV, true);
        hipLaunchKernelGGL((ms_triage_kernel<RC, RV, true>), grid, dim3(64), lds, stream, g, a);
    } else {
        QDEC_NOTE_PRE("qdec::ms_triage_kernel", RC, RV, false);
        hipLaunchKernelGGL((ms_triage_kernel<RC, RV, false>), grid, dim3(64), lds, stream, g, a);
    }
    return (int)hipGetLastError();
}

template <typename T, int METHOD, int RC, int RV, int DRC, bool DEFER, int FUSE = 0>
static int launch_bp_wave(const DevGraph& g, const DecodeArgs& a, int num_cus, hipStream_t stream) {
    if constexpr (METHOD == 1) {
        // the fused failure check reads the dense logical table's LDS copy
        // (lz_in_lds); wave-kernel graphs always have one (n <= 576)
        if (a.fail && g.k > 0 && !g.lz) return (int)hipErrorInvalidValue;
        const size_t lds = MsLds<T>::template bytes<RC, RV>(g);
        const bool two_pass = a.q_rpar || (!DEFER && compact_launch(g, a, DEFER));
        if (a.wave_ctr && !two_pass) {  // ShotSeq's chunk counter (two passes: the triage zeroes it)
            const hipError_t e = hipMemsetAsync(a.wave_ctr, 0, sizeof(unsigned long long), stream);
            if (e != hipSuccess) return (int)e;
        }
        const bool lean = lean_launch(g, a, DEFER);
        // f64: 2 waves per SIMD measured faster than 3 for a lone decode at every
        // p (n = 225: 7.1 vs 9.3 ms per 2^18 shots at p = 0.1); concurrent
        // decodes may ask for more (qd_graph_set_wave_occupancy)
        const int cap = g.wave_occ > 0 ? g.wave_occ : (sizeof(T) == 8 ? 8 : 0);
        if (two_pass) {  // triage, then the listed shots
            DecodeArgs b = a;
            b.cmp_zero_ok = (g.ms_allpos >> (sizeof(T) == 4 ? 1 : 0)) & 1;
            // iteration 1 in the triage: the tables assume alpha_1 = 0.5 (the
            // default schedule); QD_OPT_TRIAGE_IT1 = 0 leaves it to the BP kernel
            b.it1_lut = (a.ms_scaling == 0.0 && a.max_iter >= 1 && g.opt_triage_it1)
                            ? g.it1_lut[sizeof(T) == 4 ? 1 : 0]
                            : nullptr;
            if (!b.cmp_count_next) {  // double-buffered counters arrive zeroed (the previous triage)
                const hipError_t e = hipMemsetAsync(b.cmp_count, 0, (size_t)kCmpLists * kCmpSegs * 128, stream);
                if (e != hipSuccess) return (int)e;
            }
            int rc = launch_triage<RC, RV>(g, b, stream);
            if (rc != 0) return rc;
            if (b.ev) (void)hipEventRecord(b.ev[3], stream);  // end of the pre-pass
            size_t clds = MsLds<T>::core_bytes(g) + ((size_t)g.k * RV * 8 + 15) / 16 * 16 +
                          2 * kCmpLists * kCmpSegs * 8;
            if (FUSE) clds += ((size_t)RV * 8 + (size_t)g.m_pad * 2 + 15) / 16 * 16;  // fused SSF: xb, flog
            // a capped grid (f64: 8 waves per CU) must also be placed evenly: the
            // dispatcher stacks up to the kernel's own occupancy on a CU (11 for
            // the 159-VGPR f64 kernel) while others sit idle, so the LDS request is
            // padded to 1/cap of the CU
            if (cap > 0) clds = std::max(clds, (size_t)(160 * 1024 / cap) / 16 * 16);
            // degree-3 rounds: the (2, 4, 7) shape instantiates D3R = 2 (n = 225 HGP: 144 degree-3 columns)
            if constexpr (RC == 2 && RV == 4 && DRC == 7) {
                if (g.ms_d3r >= 2) {
                    if constexpr (sizeof(T) == 8) {
                        if (cap > 8) {  // 3 waves per SIMD
                            QDEC_NOTE_BP("qdec::bp_ms_cmp_kernel", tname<T>(), RC, RV, DRC, DEFER, 2, 3, FUSE);
                            return launch_persistent(bp_ms_cmp_kernel<T, RC, RV, DRC, DEFER, 2, 3, FUSE>, clds, b.B,
                                                     num_cus, stream, g, b, 64, cap);
                        }
                    }
                    QDEC_NOTE_BP("qdec::bp_ms_cmp_kernel", tname<T>(), RC, RV, DRC, DEFER, 2, 0, FUSE);
                    return launch_persistent(bp_ms_cmp_kernel<T, RC, RV, DRC, DEFER, 2, 0, FUSE>, clds, b.B, num_cus,
                                             stream, g, b, 64, cap);
                }
            }
            QDEC_NOTE_BP("qdec::bp_ms_cmp_kernel", tname<T>(), RC, RV, DRC, DEFER, 0, 0, FUSE);
            return launch_persistent(bp_ms_cmp_kernel<T, RC, RV, DRC, DEFER, 0, 0, FUSE>, clds, b.B, num_cus, stream,
                                     g, b, 64, cap);
        }
        // degree-3 rounds: the (2, 4, 7) shape (n = 225 HGP: 144 degree-3 columns) instantiates D3R = 2
        if constexpr (RC == 2 && RV == 4 && DRC == 7) {
            if (g.ms_d3r >= 2) {
                if constexpr (sizeof(T) == 8) {
                    if (lean && cap > 8) {  // 3 waves per SIMD: the 168-VGPR build
                        QDEC_NOTE_BP("qdec::bp_ms_wave_kernel", tname<T>(), RC, RV, DRC, DEFER, true, 2, 3);
                        return launch_persistent(bp_ms_wave_kernel<T, RC, RV, DRC, DEFER, true, 2, 3>, lds, a.B,
                                                 num_cus, stream, g, a, 64, cap);
                    }
                }
                if (lean) {
                    QDEC_NOTE_BP("qdec::bp_ms_wave_kernel", tname<T>(), RC, RV, DRC, DEFER, true, 2, 0);
                    return launch_persistent(bp_ms_wave_kernel<T, RC, RV, DRC, DEFER, true, 2>, lds, a.B, num_cus,
                                             stream, g, a, 64, cap);
                }
                QDEC_NOTE_BP("qdec::bp_ms_wave_kernel", tname<T>(), RC, RV, DRC, DEFER, false, 2, 0);
                return launch_persistent(bp_ms_wave_kernel<T, RC, RV, DRC, DEFER, false, 2>, lds, a.B, num_cus,
                                         stream, g, a, 64, cap);
            }
        }
        if (lean) {
            QDEC_NOTE_BP("qdec::bp_ms_wave_kernel", tname<T>(), RC, RV, DRC, DEFER, true, 0, 0);
            return launch_persistent(bp_ms_wave_kernel<T, RC, RV, DRC, DEFER, true, 0>, lds, a.B, num_cus, stream, g, a,
                                     64, cap);
        }
        QDEC_NOTE_BP("qdec::bp_ms_wave_kernel", tname<T>(), RC, RV, DRC, DEFER, false, 0, 0);
        return launch_persistent(bp_ms_wave_kernel<T, RC, RV, DRC, DEFER, false, 0>, lds, a.B, num_cus, stream, g, a,
                                 64, cap);
    } else {
        const size_t lds = (wave_lds_bytes<T>(g) + 15) / 16 * 16;
        QDEC_NOTE_BP("qdec::bp_wave_kernel", tname<T>(), METHOD, RC, RV, DRC, DEFER);
        return launch_persistent(bp_wave_kernel<T, METHOD, RC, RV, DRC, DEFER>, lds, a.B, num_cus, stream, g, a);
    }
}

template <typename T, int METHOD, int RC, int RV, int DRC>
static int launch_wave(const DevGraph& g, const DecodeArgs& a0, int num_cus, hipStream_t stream) {
    DecodeArgs a = a0;
    // the wave SSF kernel reads the packed queue (register-owned generators, u8 local-check ids)
    const bool ssf_wave = g.n_gen <= 128 && g.g_lc8;
    a.q_packed = a.ssf && ssf_wave ? 1 : 0;
    a.q_w = reinterpret_cast<uint64_t*>(a.q_x);
    // compact path with SSF: the queue entries carry readout parities
    // (the entry's readout area holds RV words: up to 64 RV logicals)
    a.q_rpar = (METHOD == 1 && a.ssf && ssf_wave && g.k <= 64 * RV && compact_launch(g, a, true)) ? 1 : 0;
    if (!a.ssf) {
        record_ev(a, 0, stream);
        const int rc = launch_bp_wave<T, METHOD, RC, RV, DRC, false>(g, a, num_cus, stream);
        record_ev(a, 1, stream);
        record_ev(a, 2, stream);
        return rc;
    }
    if (!a.q_count || !a.q_idx || !a.q_x || !a.q_r) return (int)hipErrorInvalidValue;
    if constexpr (METHOD == 1) {
        // fused SSF: the compact BP kernel runs the table-driven SSF itself
        // (QD_OPT_SSF_FUSE; same tables and spec as ssf_lut_kernel)
        if (a.q_rpar && g.opt_ssf_fuse && g.s_lut && g.s_tog && g.opt_ssf == kSsfAuto && g.n_gen <= 128) {
            record_ev(a, 0, stream);
            const int rc = g.n_gen <= 64 ? launch_bp_wave<T, METHOD, RC, RV, DRC, true, 1>(g, a, num_cus, stream)
                                         : launch_bp_wave<T, METHOD, RC, RV, DRC, true, 2>(g, a, num_cus, stream);
            record_ev(a, 1, stream);
            record_ev(a, 2, stream);
            return rc;
        }
    }
    if (!a.q_rpar) {  // the compact path's triage zeroes both counters itself (one launch fewer each)
        hipError_t e = hipMemsetAsync(a.q_count, 0, sizeof(int32_t), stream);
        if (e == hipSuccess && a.wave_ctr)  // the SSF kernel's slot counter (ShotSeq)
            e = hipMemsetAsync(a.wave_ctr + 1, 0, sizeof(unsigned long long), stream);
        if (e != hipSuccess) return (int)e;
    }
    record_ev(a, 0, stream);
    int rc = launch_bp_wave<T, METHOD, RC, RV, DRC, true>(g, a, num_cus, stream);
    record_ev(a, 1, stream);
    if (rc != 0) return rc;
    if (ssf_wave) {
        hipStream_t ss = stream;
        if (a.ssf_stream && a.ssf_stream != stream && a.ssf_ev) {  // SSF behind an event on its own stream
            hipError_t e2 = hipEventRecord(a.ssf_ev, stream);
            if (e2 == hipSuccess) e2 = hipStreamWaitEvent(a.ssf_stream, a.ssf_ev, 0);
            if (e2 != hipSuccess) return (int)e2;
            ss = a.ssf_stream;
        }
        if (g.s_lut && g.s_tog && g.opt_ssf == kSsfAuto) {
            rc = g.n_gen <= 64 ? launch_ssf_lut<1, RV, RC>(g, a, num_cus, ss)
                               : launch_ssf_lut<2, RV, RC>(g, a, num_cus, ss);
        } else {
            DevGraph gs = g;  // QD_SSF_SCAN_GATHER: no incremental local syndromes
            if (g.opt_ssf == kSsfScanGather) gs.g_inv = nullptr;
            rc = g.n_gen <= 64 ? launch_ssf_wave<1, RV, RC>(gs, a, num_cus, ss)
                               : launch_ssf_wave<2, RV, RC>(gs, a, num_cus, ss);
        }
        record_ev(a, 2, ss);
        return rc;
    }
    rc = launch_ssf_block(g, a, num_cus, stream);
    record_ev(a, 2, stream);
    return rc;
}

template <typename T, int METHOD>
static int dispatch_shape(const DevGraph& g, const DecodeArgs& a, int num_cus, hipStream_t stream) {
    const int rc = g.m_pad / 64, rv = g.n_pad / 64;
#define QDEC_SHAPE(R, V, D) \
    if (rc == R && rv == V && g.shape_drc == D) return launch_wave<T, METHOD, R, V, D>(g, a, num_cus, stream);
    QDEC_WAVE_SHAPES(QDEC_SHAPE)
#undef QDEC_SHAPE
    return (int)hipErrorNotSupported;
}

bool wave_kernel_supports(const DevGraph& g) {
    bool shape = false;
#define QDEC_SHAPE(R, V, D) shape |= (g.m_pad == 64 * R && g.n_pad == 64 * V && g.shape_drc == D);
    QDEC_WAVE_SHAPES(QDEC_SHAPE)
#undef QDEC_SHAPE
    return shape && g.max_rdeg <= kDR && g.max_cdeg <= kDC && g.k <= 256;
}

// ---------------------------------------------------------------- packed inputs
// Bit-packed rows (QD_INPUT_PACKED) expanded to one byte per bit: dst[r][c] =
// bit c of src row r (words of `words` u64 per row).  Grid-stride over 4-byte
// groups of the output (coalesced stores; the source words are re-read from
// L1/L2 by neighbouring threads).
__global__ void unpack_rows_kernel(const uint64_t* __restrict__ src, int64_t rows, int cols, int words,
                                   uint8_t* __restrict__ dst) {
    const int64_t total = rows * cols;
    for (int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; e < total;
         e += (int64_t)gridDim.x * blockDim.x * 4) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int64_t q = e + t;
            if (q < total) {
                const int64_t r = q / cols;
                const int c = (int)(q - r * cols);
                dst[q] = (uint8_t)((src[r * words + (c >> 6)] >> (c & 63)) & 1ull);
            }
        }
    }
}

static int launch_unpack_rows(const uint8_t* src, int64_t rows, int cols, uint8_t* dst, int num_cus,
                              hipStream_t stream) {
    if (rows <= 0 || cols <= 0) return 0;
    const int64_t groups = (rows * cols + 3) / 4;
    const long long blocks = std::min<long long>((groups + 255) / 256, (long long)num_cus * 16);
    hipLaunchKernelGGL(unpack_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, stream,
                       reinterpret_cast<const uint64_t*>(src), rows, cols, (cols + 63) / 64, dst);
    return (int)hipGetLastError();
}

// A packed decode the triage can read directly: a lean min-sum launch on a wave
// graph that takes the two-pass path (launch_wave / launch_bp_wave's choice).
static bool packed_two_pass(const DevGraph& g, int method, const DecodeArgs& a0) {
    if (method != 1 || !g.wave || !wave_kernel_supports(g)) return false;
    DecodeArgs a = a0;
    const bool ssf_wave = g.n_gen <= 128 && g.g_lc8;
    a.q_packed = a.ssf && ssf_wave ? 1 : 0;
    if (a.ssf) return ssf_wave && g.k <= g.n_pad && compact_launch(g, a, true);
    return compact_launch(g, a, false);
}

int launch_decode(const DevGraph& g, int method, int precision, const DecodeArgs& a0, int num_cus,
                  hipStream_t stream, void* scratch, size_t scratch_bytes) {
    last_launch_names() = LaunchNames{};
    if (a0.B <= 0) return 0;
    DecodeArgs a = a0;
    if (a.in_packed && !packed_two_pass(g, method, a)) {
        // every other path reads byte rows: expand the inputs first
        if (!a.unpack_buf) return (int)hipErrorInvalidValue;
        uint8_t* u = a.unpack_buf;
        int rc = 0;
        if (a.syn) {
            rc = launch_unpack_rows(a.syn, a.B, g.m, u, num_cus, stream);
            a.syn = u;
            u += (size_t)a.B * g.m;
        }
        if (rc == 0 && a.base) {
            rc = launch_unpack_rows(a.base, a.B, g.n_data, u, num_cus, stream);
            a.base = u;
            u += (size_t)a.B * g.n_data;
        }
        if (rc == 0 && a.readout) {
            rc = launch_unpack_rows(a.readout, a.B, g.n_data, u, num_cus, stream);
            a.readout = u;
        }
        if (rc != 0) return rc;
        a.in_packed = 0;
    }
    if (!g.wave || !wave_kernel_supports(g))
        return launch_decode_block(g, method, precision, a, num_cus, stream, scratch, scratch_bytes);
    if (precision == 1)
        return method == 1 ? dispatch_shape<float, 1>(g, a, num_cus, stream)
                           : dispatch_shape<float, 0>(g, a, num_cus, stream);
    return method == 1 ? dispatch_shape<double, 1>(g, a, num_cus, stream)
                       : dispatch_shape<double, 0>(g, a, num_cus, stream);
}

#ifdef QDEC_STAMPS
extern "C" __attribute__((visibility("default"))) int qd_dev_read_stamps(unsigned long long* out, int n, int reset) {
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
