// qdec_sample.hip -- on-device sampler for the storage experiment.
//
// Restates what Stim samples from the reference's storage circuit
// (storage_sim.py:110-199) under depolarizing_noise(p, pm) (noise_model.py:117-123):
// DEPOLARIZE1(p) on every data qubit at the start of every timestep that contains
// a measurement, MRX(pm)/MZ(pm) record flips.  Only the X/Y part of DEPOLARIZE1
// (probability 2p/3) changes Z-basis records; the random X-stabilizer component
// of the readout is invisible to Hz and Lz and is not generated.  Per shot:
//   round t:  cum ^= Da(t); s_t = Hz cum ^ M_t; cum ^= Db(t); if t >= 1: cum ^= Dc(t)
//   (Dc = the DEPOLARIZE1 the rewriter places inside the REPEAT body before '}')
//   readout = cum ^ F   (R = 0: readout = D ^ F)
//   syn = [s_0, s_1^s_0, ..., Hz readout ^ s_{R-1}]   (spacetime_code.py:98-119)
// Bernoulli(p) bits are u32 < floor(p 2^32) from Philox4x32-10 with key
// (seed, stream_id) and counter (word, event, shot_lo, shot_hi); word w covers
// elements 4w..4w+3.  Event ids: R = 0: D=0, F=1; R >= 1: Da=4t, M=4t+1, Db=4t+2,
// Dc=4t+3, F=4R.  Identical to oracle/qdec_oracle.c qdo_sample_storage.
#include <hip/hip_runtime.h>

#include "qdec_internal.h"

namespace qdec {

__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, c[0]);
        const uint32_t lo0 = 0xD2511F53u * c[0];
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c[2]);
        const uint32_t lo1 = 0xCD9E8D57u * c[2];
        const uint32_t n0 = hi1 ^ c[1] ^ k0;
        const uint32_t n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0;
        c[1] = lo1;
        c[2] = n2;
        c[3] = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

// dst[e] ^= Bernoulli(thr) for e < count, event `ev`; lanes split the words.
__device__ __forceinline__ void bern_xor(uint8_t* dst, int count, uint32_t thr, uint32_t ev, int64_t shot,
                                         uint32_t k0, uint32_t k1, int lane) {
    if (thr == 0) return;
    const int words = (count + 3) / 4;
    for (int w = lane; w < words; w += 64) {
        uint32_t c[4] = {(uint32_t)w, ev, (uint32_t)shot, (uint32_t)((uint64_t)shot >> 32)};
        philox4x32_10(c, k0, k1);
#pragma unroll
        for (int l = 0; l < 4; ++l)
            if (4 * w + l < count) dst[4 * w + l] ^= (uint8_t)(c[l] < thr);
    }
}

__device__ __forceinline__ int row_parity(const DevGraph& g, const uint8_t* v, int i) {
    int p = 0;
    for (int e = g.row_ptr[i]; e < g.row_ptr[i + 1]; ++e) p ^= v[g.col_idx[e]];
    return p;
}

// OR a 64-bit ballot (bits of elements pos .. pos + 63) into a packed row held
// in LDS (one wave per block: lane 0 writes; the row has a spare word)
__device__ __forceinline__ void put_bits(uint64_t* w, int64_t pos, uint64_t mask, int lane) {
    if (lane == 0 && mask) {
        const int sh = (int)(pos & 63);
        w[pos >> 6] |= mask << sh;
        if (sh) w[(pos >> 6) + 1] |= mask >> (64 - sh);
    }
}

// PACKED: rows written as u64 words (bit j of word w = element 64 w + j; the
// layout of qd_sample_storage_packed_device), assembled in LDS by ballots.
template <bool PACKED>
__global__ __launch_bounds__(64) void sample_storage_kernel(DevGraph g, int rounds, uint32_t td, uint32_t tm,
                                                            uint32_t seed, uint32_t sid, int64_t shot0, int64_t B,
                                                            uint8_t* __restrict__ syn,
                                                            uint8_t* __restrict__ readout) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x;
    const int m = g.m, n = g.n;
    const int64_t syn_len = (int64_t)(rounds + 1) * m;
    const int sw_words = (int)((syn_len + 63) / 64), rw_words = (n + 63) / 64;
    uint64_t* synw = reinterpret_cast<uint64_t*>(smem);  // PACKED: [sw_words + 1], [rw_words + 1]
    uint64_t* rdw = synw + (PACKED ? sw_words + 1 : 0);
    uint8_t* cum = reinterpret_cast<uint8_t*>(rdw + (PACKED ? rw_words + 1 : 0));  // [n_pad]
    uint8_t* prev = cum + g.n_pad;    // [m_pad]
    uint8_t* cur = prev + g.m_pad;    // [m_pad]

    for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
        const int64_t shot = shot0 + b;
        for (int e = lane; e < g.n_pad; e += 64) cum[e] = 0;
        for (int e = lane; e < g.m_pad; e += 64) prev[e] = 0;
        if constexpr (PACKED) {
            for (int e = lane; e <= sw_words; e += 64) synw[e] = 0ull;
            for (int e = lane; e <= rw_words; e += 64) rdw[e] = 0ull;
        }
        __syncthreads();
        uint8_t* out = syn + b * syn_len;
        for (int t = 0; t < rounds; ++t) {
            bern_xor(cum, n, td, 4u * t + 0u, shot, seed, sid, lane);
            __syncthreads();
            for (int i = lane; i < m; i += 64) cur[i] = (uint8_t)row_parity(g, cum, i);
            __syncthreads();
            bern_xor(cur, m, tm, 4u * t + 1u, shot, seed, sid, lane);
            bern_xor(cum, n, td, 4u * t + 2u, shot, seed, sid, lane);
            __syncthreads();
            if (t >= 1) bern_xor(cum, n, td, 4u * t + 3u, shot, seed, sid, lane);
            if constexpr (PACKED) {
                for (int i0 = 0; i0 < m; i0 += 64) {
                    const int i = i0 + lane;
                    const bool bit = i < m && ((cur[i] ^ prev[i]) & 1);
                    if (i < m) prev[i] = cur[i];
                    put_bits(synw, (int64_t)t * m + i0, __ballot(bit), lane);
                }
            } else {
                for (int i = lane; i < m; i += 64) {
                    out[(int64_t)t * m + i] = cur[i] ^ prev[i];
                    prev[i] = cur[i];
                }
            }
            __syncthreads();
        }
        if (rounds == 0) {
            bern_xor(cum, n, td, 0u, shot, seed, sid, lane);
            __syncthreads();
        }
        bern_xor(cum, n, tm, rounds == 0 ? 1u : 4u * (uint32_t)rounds, shot, seed, sid, lane);
        __syncthreads();
        if constexpr (PACKED) {
            for (int j0 = 0; j0 < n; j0 += 64) {
                const int j = j0 + lane;
                put_bits(rdw, j0, __ballot(j < n && (cum[j] & 1)), lane);
            }
            for (int i0 = 0; i0 < m; i0 += 64) {
                const int i = i0 + lane;
                const bool bit = i < m && ((row_parity(g, cum, i) ^ prev[i]) & 1);
                put_bits(synw, (int64_t)rounds * m + i0, __ballot(bit), lane);
            }
            __syncthreads();
            uint64_t* so = reinterpret_cast<uint64_t*>(syn) + b * sw_words;
            uint64_t* ro = reinterpret_cast<uint64_t*>(readout) + b * rw_words;
            for (int e = lane; e < sw_words; e += 64) so[e] = synw[e];
            for (int e = lane; e < rw_words; e += 64) ro[e] = rdw[e];
        } else {
            for (int j = lane; j < n; j += 64) readout[b * n + j] = cum[j];
            for (int i = lane; i < m; i += 64) out[(int64_t)rounds * m + i] = (uint8_t)row_parity(g, cum, i) ^ prev[i];
        }
        __syncthreads();
    }
}

int launch_sample_storage(const DevGraph& g, int rounds, uint32_t thr_data, uint32_t thr_meas, uint32_t seed,
                          uint32_t stream_id, int64_t shot0, int64_t B, uint8_t* syn, uint8_t* readout,
                          int num_cus, hipStream_t stream, bool packed) {
    if (B <= 0) return 0;
    size_t lds = (size_t)g.n_pad + 2 * (size_t)g.m_pad;
    if (packed) lds += 8 * ((((int64_t)(rounds + 1) * g.m + 63) / 64 + 1) + ((int64_t)g.n + 63) / 64 + 1);
    const void* fn = packed ? reinterpret_cast<const void*>(sample_storage_kernel<true>)
                            : reinterpret_cast<const void*>(sample_storage_kernel<false>);
    if (lds > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return (int)e;
    }
    long long grid = (long long)num_cus * 16;
    if (grid > B) grid = B;
    if (packed)
        hipLaunchKernelGGL(sample_storage_kernel<true>, dim3((unsigned)grid), dim3(64), lds, stream, g, rounds,
                           thr_data, thr_meas, seed, stream_id, shot0, B, syn, readout);
    else
        hipLaunchKernelGGL(sample_storage_kernel<false>, dim3((unsigned)grid), dim3(64), lds, stream, g, rounds,
                           thr_data, thr_meas, seed, stream_id, shot0, B, syn, readout);
    return (int)hipGetLastError();
}

}  // namespace qdec
