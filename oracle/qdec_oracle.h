/*
 * qdec_oracle.h -- CPU restatement of the decoding hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the HIP
 * product library (include/qdec.h) and the timed CPU baseline in bench.py.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * Nothing in exp_ldpc_amd/ links or calls it.
 *
 * What it restates:
 *   - BP exactly as the third-party `ldpc` package v1 runs it (quantumgizmos/ldpc,
 *     rev 7909a97d, labelled 1.9.0, pinned at reference overlays/python/ldpc/
 *     default.nix:14-22; called from reference python/qldpc/misc/_experiment.py:
 *     23,37,77,96,110,137 / .decode at :51,59,82,117,125,149).  `ldpc` is NOT in
 *     this image, so the loops below are a restatement of its published
 *     bp_decoder min-sum-log and product-sum (probability-ratio) routines, operation
 *     for operation: forward/backward leave-one-out sweeps along each row, prefix/
 *     suffix sums along each column, syndrome test after every iteration.
 *     -> BP parity against ldpc itself is UNPINNED (no ldpc fixture exists).
 *   - Small-set-flip: absent from the reference; specified by this
 *     build (DESIGN.md "SSF spec") and restated here by brute force.
 *   - final_correction fold (reference spacetime_code.py:81-84), logical check
 *     (reference misc/_experiment.py:209), storage-experiment sampler (noise of
 *     noise_model.py:117-123 on the circuit of storage_sim.py:110-199).
 */
#ifndef QDEC_ORACLE_H
#define QDEC_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { QDO_PRODUCT_SUM = 0, QDO_MIN_SUM = 1 };
enum { QDO_F64 = 0, QDO_F32 = 1 };
enum { QDO_SYN_ADD_BASE = 1, QDO_SYN_ADD_READOUT = 2 };
enum { QDO_ST_BP_CONVERGED = 1, QDO_ST_SATISFIED = 2 };
enum { QDO_SSF_BRUTE = 0, QDO_SSF_FAST = 1 };

/* Decode B shots (OpenMP over shots, nthreads <= 0 -> all cores).
 * See DESIGN.md "Decode contract" for the meaning of every argument; it is the
 * same contract as qd_decode_batch in include/qdec.h. llr_out is double for both
 * precisions (fp32 values are widened exactly).  ssf_impl: QDO_SSF_BRUTE (the
 * checker: literal subset enumeration) or QDO_SSF_FAST (same spec with bitmasks;
 * the timed baseline). */
int qdo_decode_batch(int32_t m, int32_t n, const int32_t* row_ptr, const int32_t* col_idx,
                     const double* channel_probs, int32_t method, int32_t precision,
                     int32_t max_iter, double ms_scaling,
                     int32_t ssf, int32_t ssf_max_steps,
                     int32_t n_gen, const int32_t* gen_ptr, const int32_t* gen_idx,
                     int32_t n_data, int32_t fold_blocks,
                     int32_t k, const uint8_t* lz,
                     int64_t B, const uint8_t* syn, const uint8_t* base, const uint8_t* readout,
                     int32_t syn_flags,
                     uint8_t* x_out, uint8_t* corr_out, double* llr_out,
                     int32_t* iters, uint8_t* status, int32_t* ssf_steps, uint8_t* fail,
                     int32_t ssf_impl, int32_t nthreads);

/* Storage-experiment sampler (DESIGN.md "Sampler"): Philox4x32-10, key =
 * {seed, stream}, counter = {word, event, shot_lo, shot_hi}.  Writes the
 * difference (spacetime) syndrome syn[B][(R+1)*m] and readout[B][n]. */
int qdo_sample_storage(int32_t m, int32_t n, const int32_t* row_ptr, const int32_t* col_idx,
                       int32_t rounds, double p_data, double p_meas,
                       uint32_t seed, uint32_t stream, int64_t shot0, int64_t B,
                       uint8_t* syn, uint8_t* readout, int32_t nthreads);

/* OSD of B shots from their BP soft output (oracle/osd_impl.inc; same spec as
 * oracle/osd_py.py and the product's qd_osd_batch): method 0 osd0, 1 osd_e,
 * 2 osd_cs; llr[B][n] double; osd0 / osdw [B][n] (either may be NULL).
 * OpenMP over shots. */
int qdo_osd_batch(int32_t m, int32_t n, const int32_t* row_ptr, const int32_t* col_idx, int64_t B,
                  const uint8_t* syn, const double* llr, int32_t method, int32_t order, uint8_t* osd0,
                  uint8_t* osdw, int32_t nthreads);

/* Raw Philox4x32-10 block (exposed for known-answer tests). */
void qdo_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

/* Bernoulli threshold used by the sampler: floor(p * 2^32), clamped. */
uint32_t qdo_threshold(double p);

#ifdef __cplusplus
}
#endif
#endif
