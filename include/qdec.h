/*
 * qdec.h -- C ABI of libqdec_hip.so, the MI355X (gfx950) BP + small-set-flip
 * syndrome decoder.
 *
 * This is the drop-in boundary for the reference's decoding hot path.  In the
 * reference (qldpc/exp_ldpc @ 2025-02-21) that boundary is the third-party
 * `ldpc` v1 decoder-object API, called only from python/qldpc/misc/_experiment.py:
 *   - construction  bposd_decoder(H, error_rate=.., **opts)     _experiment.py:23-27, 96-100
 *                   bposd_decoder(H, channel_probs=.., **opts)  _experiment.py:37-40
 *                   bposd_decoder(H, channel_prior=.., **opts)  _experiment.py:77
 *                   bp_decoder(H, channel_probs=.., **opts)     _experiment.py:110-113, 137-140
 *   - decode        .decode(syndrome) -> ndarray[n]             _experiment.py:51, 59, 82, 117, 125, 149
 *   - per-shot logical check  any(GF2(Lz) @ GF2(readout))       _experiment.py:209
 * Each entry point below names the reference interface it replaces.  The Python
 * binding (exp_ldpc_amd/_abi.py, ctypes) and the ldpc-v1-compatible classes are
 * described in INTEGRATION.md.
 *
 * Conventions: plain pointers and sizes; no C++ exceptions cross the ABI; status
 * 0 = OK, negative = error (message via qd_last_error(), thread-local).  The
 * library owns device copies of the graph; the caller owns every buffer it
 * passes.  A handle is used from one host thread at a time; one handle per
 * device for multi-GPU.  Device-buffer decodes on one handle may be enqueued on
 * different streams: the handle's SSF queue and message scratch are shared, so
 * the library chains such calls with an event (a call waits for the previous
 * call's kernels) and frees a grown buffer only after its last use completed.
 * Calls on one handle therefore never run concurrently; use one handle per
 * stream for concurrent decodes.
 */
#ifndef QDEC_H
#define QDEC_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QDEC_ABI_VERSION 1

typedef struct qd_graph qd_graph;

enum qd_method { QD_PRODUCT_SUM = 0, QD_MIN_SUM = 1 };      /* ldpc bp_method 'ps' / 'ms','msl' */
enum qd_precision { QD_F64 = 0, QD_F32 = 1 };               /* message arithmetic */
/* syn_flags bits.  QD_INPUT_PACKED: the decode's syn / base / readout inputs are
 * bit-packed rows of little-endian u64 words instead of one byte per bit:
 * syn [B][ceil(m/64)], base / readout [B][ceil(n_data/64)], bit j of word w =
 * element 64 w + j, padding bits ignored, 8-B aligned.  Byte for byte this is
 * Stim's sample(bit_packed=True) layout (the reference sampler,
 * _experiment.py:196-197) with each row zero-padded to a multiple of 8 bytes.
 * Outputs keep their layouts. */
enum qd_syn_flags { QD_SYN_ADD_BASE = 1, QD_SYN_ADD_READOUT = 2, QD_INPUT_PACKED = 16 };
enum qd_status_bits { QD_ST_BP_CONVERGED = 1, QD_ST_SATISFIED = 2 };

typedef struct qd_params {
    int32_t max_iter;      /* <= 0 -> n (ldpc v1: max_iter=0 means n) */
    int32_t method;        /* enum qd_method */
    int32_t precision;     /* enum qd_precision */
    int32_t ssf;           /* 1: small-set-flip on shots BP did not converge (needs flip sets) */
    int32_t ssf_max_steps; /* <= 0: unbounded (terminates: |residual| strictly decreases) */
    int32_t syn_flags;     /* enum qd_syn_flags: syndrome ^= H[:, :n_data] (base ^ readout) */
    double ms_scaling;     /* 0 -> alpha_t = 1 - 2^-t (ldpc ms_scaling_factor=0) */
} qd_params;

/* Version / device discovery. */
int qd_abi_version(void);
int qd_device_count(void);
const char* qd_last_error(void);

/* Replaces the ldpc constructor's copy of H into mod2sparse (_experiment.py:23,
 * 37, 77, 96, 110, 137).  H is m x n CSR with column indices sorted within each
 * row (row_ptr[m+1], col_idx[row_ptr[m]]).  Columns t*n_data + q (t <
 * fold_blocks) fold onto data qubit q (SpacetimeCode.final_correction,
 * spacetime_code.py:81-84); fold_blocks = 1, n_data = n for a plain code.  The
 * graph is uploaded to `device` (HIP ordinal). */
int qd_graph_create(int32_t m, int32_t n, const int32_t* row_ptr, const int32_t* col_idx,
                    int32_t n_data, int32_t fold_blocks, int32_t device, qd_graph** out);
int qd_graph_destroy(qd_graph* g);

/* Host-only graph: the same validation and host tables as qd_graph_create
 * (kernel layouts and anneals, flip-set and logical tables, priors) with no
 * device and no HIP call; the tables are kept in host memory.  For CPU tests
 * and sanitizer runs (tools/sanitize.sh); decode calls on it fail.
 * qd_graph_table_digest returns an FNV-1a digest and the byte count of every
 * table built so far.  No reference counterpart. */
int qd_graph_create_host(int32_t m, int32_t n, const int32_t* row_ptr, const int32_t* col_idx, int32_t n_data,
                         int32_t fold_blocks, qd_graph** out);
int qd_graph_table_digest(const qd_graph* g, uint64_t* digest, int64_t* bytes);

/* Flip sets for small-set-flip: generator rows (CSR over H's columns; for the
 * storage experiment the X-check rows of Hx).  Each generator must have <= 8
 * qubits whose checks in H number <= 32.  No reference counterpart (SSF is
 * absent from the reference). */
int qd_graph_set_flipsets(qd_graph* g, int32_t n_gen, const int32_t* gen_ptr, const int32_t* gen_idx);

/* Logical operators for the fused failure check, dense 0/1 k x n_data (the `LZ`
 * rows of the qecc file; replaces GF2(logicals.z) @ GF2(readout) at
 * _experiment.py:209). */
int qd_graph_set_logicals(qd_graph* g, int32_t k, const uint8_t* lz);

/* The same logicals as a CSR over data qubits (row r = the support of logical r,
 * lz_ptr[k+1], lz_idx[nnz] in [0, n_data), duplicates cancel mod 2).  For codes
 * with many sparse logicals (the PSL(2,16) Cayley-graph LP code of config 5:
 * k = 4080 of weight 3, n = 53,040) where the dense k x n_data form is hundreds
 * of MB; the workgroup kernels then test each logical on its support only. */
int qd_graph_set_logicals_csr(qd_graph* g, int32_t k, const int32_t* lz_ptr, const int32_t* lz_idx);

/* Per-column error probabilities (ldpc `error_rate` broadcast / `channel_probs`;
 * reference call sites _experiment.py:23-27, 37-40, 74-77, 106-113).  Converted
 * on the host to the ldpc initial messages log((1-p)/p) (min-sum) and p/(1-p)
 * (product-sum) in both precisions. */
int qd_graph_set_priors(qd_graph* g, const double* channel_probs);

/* Batched replacement of B calls to .decode(syndrome) (_experiment.py:82, 117,
 * 125, ...), plus the fused fold and logical check.  Host buffers; synchronous.
 *   syn       uint8 [B][m]       syndrome bits (nullable when syn_flags set)
 *   base      uint8 [B][n_data]  xor-ed into corr_out (and into the syndrome with
 *                                QD_SYN_ADD_BASE); nullable
 *   readout   uint8 [B][n_data]  data readout for the failure flag (and the
 *                                syndrome with QD_SYN_ADD_READOUT); nullable
 * outputs (each nullable):
 *   x_out     uint8 [B][n]       decoding (BP hard decision, SSF applied) = ldpc .decode() result
 *   corr_out  uint8 [B][n_data]  base ^ fold(x_out)
 *   llr_out   [B][n] float (QD_F32) or double (QD_F64): ldpc .log_prob_ratios
 *   iters     int32 [B]          ldpc .iter
 *   status    uint8 [B]          QD_ST_BP_CONVERGED (= ldpc .converge) | QD_ST_SATISFIED
 *   ssf_steps int32 [B]          flips applied by SSF
 *   fail      uint8 [B]          any(Lz (readout ^ corr_out)) mod 2 (needs logicals+readout) */
int qd_decode_batch(qd_graph* g, const qd_params* prm, int64_t B,
                    const uint8_t* syn, const uint8_t* base, const uint8_t* readout,
                    uint8_t* x_out, uint8_t* corr_out, void* llr_out,
                    int32_t* iters, uint8_t* status, int32_t* ssf_steps, uint8_t* fail);

/* Same contract on device-resident buffers (HBM), enqueued on `stream`
 * (hipStream_t; NULL = default stream); returns after the launch. */
int qd_decode_batch_device(qd_graph* g, const qd_params* prm, int64_t B,
                           const uint8_t* syn, const uint8_t* base, const uint8_t* readout,
                           uint8_t* x_out, uint8_t* corr_out, void* llr_out,
                           int32_t* iters, uint8_t* status, int32_t* ssf_steps, uint8_t* fail,
                           void* stream);

/* Replaces Stim's compile_sampler().sample(B) + StorageSim slicing +
 * _spacetime_syndrome (_experiment.py:196-207, storage_sim.py:187-196,
 * spacetime_code.py:98-119) for the storage experiment under
 * depolarizing_noise(p_data, pm=p_meas) (noise_model.py:117-123).  The graph must
 * be a plain code (fold_blocks = 1): H = Hz.  Writes, on device:
 *   syn     uint8 [B][(rounds+1)*m]  spacetime (difference) syndrome
 *   readout uint8 [B][n]             transversal Z readout
 * Philox4x32-10 keyed (seed, stream_id), counter (word, event, shot): results
 * do not depend on how shots are split across calls or devices. */
int qd_sample_storage_device(qd_graph* g, int32_t rounds, double p_data, double p_meas,
                             uint32_t seed, uint32_t stream_id, int64_t shot0, int64_t B,
                             uint8_t* syn, uint8_t* readout, void* stream);
/* The same shots, written bit-packed (the QD_INPUT_PACKED layout):
 *   syn     uint64 [B][ceil((rounds+1)*m/64)]   readout uint64 [B][ceil(n/64)]
 * 8-B aligned buffers.  With rounds = 0 the rows feed qd_decode_batch_device
 * with QD_INPUT_PACKED directly (42 B per shot at n = 225 instead of 333). */
int qd_sample_storage_packed_device(qd_graph* g, int32_t rounds, double p_data, double p_meas,
                                    uint32_t seed, uint32_t stream_id, int64_t shot0, int64_t B,
                                    uint64_t* syn, uint64_t* readout, void* stream);

/* Ordered-statistics decoding of shots BP did not converge on (the OSD stage of
 * ldpc v1 bposd_decoder; reference _experiment.py:23-27, 37-40, 77, 96-100).  Host
 * buffers; runs on the host cores (nthreads <= 0: all).  method: 0 = osd0,
 * 1 = osd_e, 2 = osd_cs; order = osd_order.  llr = BP log-probability ratios
 * (qd_decode_batch llr_out widened to double).  Outputs osd0 and the best
 * higher-order solution (ldpc .osd0_decoding / .osdw_decoding), uint8 [B][n]. */
int qd_osd_batch(int32_t m, int32_t n, const int32_t* row_ptr, const int32_t* col_idx, int32_t method,
                 int32_t order, int64_t B, const uint8_t* syn, const double* llr, uint8_t* osd0_out,
                 uint8_t* osdw_out, int32_t nthreads);
const char* qd_osd_last_error(void);

/* The same OSD on the GPU, on device-resident buffers, enqueued on `stream`
 * (hipStream_t).  Graph = the BP graph handle (H, fold and logicals).  Shots with
 * status bit QD_ST_BP_CONVERGED set are skipped (status nullable: all shots).
 * llr: [B][n] float (QD_F32) or double (QD_F64), the BP .log_prob_ratios; the
 * syndrome is syn (^ H[:, :n_data] base/readout per syn_flags, as in
 * qd_decode_batch).  Outputs for processed shots (each nullable): osd0_out,
 * osdw_out [B][n] (ldpc .osd0_decoding / .osdw_decoding), corr_out = base ^
 * fold(osdw), fail = any(Lz (readout ^ corr_out)).  Bit-identical to
 * qd_osd_batch.  Needs m <= 384 and n < 1024 (qd_osd_device_supported). */
int qd_osd_device_supported(const qd_graph* g);
int qd_osd_batch_device(qd_graph* g, int32_t method, int32_t order, int64_t B, const uint8_t* syn, int32_t syn_flags,
                        const void* llr, int32_t llr_precision, const uint8_t* status, const uint8_t* base,
                        const uint8_t* readout, uint8_t* osd0_out, uint8_t* osdw_out, uint8_t* corr_out, uint8_t* fail,
                        void* stream);

/* Kernel timing for measurement: with capacity > 0, the next `capacity` decode
 * calls record HIP events on their launch stream immediately before the BP kernel,
 * after it and after the SSF kernel.  qd_graph_read_timing returns the per-call
 * BP and SSF kernel durations (ms) and resets the ring.  No reference
 * counterpart (the reference only reports whole-sweep walltime,
 * misc/p_sweep.py:26-33). */
int qd_graph_set_timing(qd_graph* g, int32_t capacity);

/* Route the SSF kernel of later qd_decode_batch_device calls (wave-kernel graphs)
 * to `ssf_stream` (hipStream_t; NULL = the decode's own stream, the default):
 * it runs behind an event recorded after the BP kernel on the decode stream.
 * Outputs the SSF stage writes (status, ssf_steps, fail, x/corr of BP-failed
 * shots) are complete when `ssf_stream` has passed that point; the caller
 * synchronises with it.  Split decodes alternate between two SSF queues (and
 * their control words), so a decode waits for the SSF kernel of the decode two
 * back on this handle, not the previous one: the handle's next triage and BP
 * run while this SSF kernel is still on `ssf_stream`.  Replaces nothing in the
 * reference (its decode is one synchronous call per shot). */
int qd_graph_set_ssf_stream(qd_graph* g, void* ssf_stream);

/* Occupancy of the wave BP kernels (one wave per shot, persistent grid) in waves
 * per CU: 0 = the default (f64: 8, measured fastest for a lone decode; f32: the
 * hardware maximum), N > 0 = N, bounded by what the kernel's LDS and registers
 * allow and rounded down to a multiple of 4 (equal waves per SIMD).  For
 * several decodes running concurrently on different streams: the bench's
 * 9-stream sweep measured 82-83 M shots/s at 12 f64 waves per CU against 80 M
 * at 8, while a lone f64 decode at 12 is slower (p = 0.1: 9.3 vs 7.1 ms per 2^18
 * shots).  A request above 8 f64 waves per CU launches the kernel's build for
 * 3 waves per SIMD (the f64 LEAN kernel otherwise needs 172 VGPRs, which fit
 * only 2).  Results are identical at every setting.  No reference counterpart. */
int qd_graph_set_wave_occupancy(qd_graph* g, int32_t waves_per_cu);
int qd_graph_read_timing(qd_graph* g, float* bp_ms, float* ssf_ms, int32_t max_calls, int32_t* n_calls);
/* The same ring split finer: per recorded call the BP stage's pre-pass (the
 * lean launches' shot triage; 0 when none ran), the BP kernel alone, the SSF
 * kernel (ms), and `listed` = the number of shots the triage left to the BP
 * kernel (-1 when the call did not run the two-pass path).  Resets the ring
 * like qd_graph_read_timing.  Any output may be NULL.  No reference
 * counterpart. */
int qd_graph_read_timing_detail(qd_graph* g, float* pre_ms, float* bp_ms, float* ssf_ms, int64_t* listed,
                                int32_t max_calls, int32_t* n_calls);

/* Names of the BP and SSF kernels the last decode call on `g` launched, and of
 * the pass run before the BP kernel inside the BP timing (the lean launches'
 * shot triage), as rocprofv3 spells them (template arguments included; "" when
 * a stage did not run or has no recorded name), NUL-terminated and truncated to
 * the buffer lengths.  Lets a measurement match a rocprof / PMC entry to the
 * exact instantiation it timed.  No reference counterpart. */
int qd_graph_last_kernels(qd_graph* g, char* bp, int32_t bp_len, char* ssf, int32_t ssf_len, char* pre,
                          int32_t pre_len);

/* Kernel choices of one handle, for A/B measurements and for tests that keep
 * every kernel path covered.  Results are identical under every setting (each
 * path is parity-tested against the oracle).  Returns -2 for an unknown option
 * or an out-of-range value.  No reference counterpart: ldpc has one decoder
 * implementation.
 *   QD_OPT_COMPACT       1 (default): lean min-sum decodes on wave graphs run the
 *                        shot triage + compact-list kernel; 0: the one-pass kernel.
 *   QD_OPT_TRIAGE_IT1    1 (default): the triage runs min-sum iteration 1
 *                        bit-sliced (default alpha schedule, positive priors); 0: off.
 *   QD_OPT_SSF           SSF kernels: QD_SSF_AUTO (default: the table-driven
 *                        wave kernel, or table scoring in the workgroup kernel,
 *                        when the graph's tables qualify, else the scanning
 *                        kernels), QD_SSF_SCAN (scanning kernel / subset search,
 *                        incremental local syndromes), QD_SSF_SCAN_GATHER (scanning
 *                        kernel, local syndromes re-gathered every step),
 *                        QD_SSF_SCAN_NOSPLIT (scanning, one lane per generator).
 *   QD_OPT_LDS_KERNEL    -1 (default) automatic, 0 never, 1 forced: the
 *                        LDS-resident min-sum workgroup kernels (f32: every
 *                        message in LDS; f64: v2c in registers, check states
 *                        by LDS atomics).
 *   QD_OPT_GROUP_KERNEL  -1 (default) automatic, 0 never, 1 forced: the slot-group
 *                        HBM-streaming kernel.
 *   QD_OPT_SSF_INC       1 (default): incremental workgroup SSF; 0: re-scanning.
 *   QD_OPT_BLOCK_WG      0 (default) automatic, N > 0: workgroups per CU of the
 *                        HBM-slice workgroup BP kernel.
 *   QD_OPT_GROUP_MB      0 (default): a quarter of the free HBM, N > 0: N MiB for
 *                        the slot-group kernel's message scratch.
 *   QD_OPT_SSF_FUSE      0 (default): BP-failed shots of two-pass min-sum decodes
 *                        are queued for ssf_lut_kernel; 1: the compact BP kernel
 *                        runs the same table-driven SSF itself right after a
 *                        shot's BP fails (no queue, no second launch; its tables
 *                        come through the caches, not LDS: measured slower). */
#define QD_OPT_COMPACT 1
#define QD_OPT_TRIAGE_IT1 2
#define QD_OPT_SSF 3
#define QD_OPT_LDS_KERNEL 4
#define QD_OPT_GROUP_KERNEL 5
#define QD_OPT_SSF_INC 6
#define QD_OPT_BLOCK_WG 7
#define QD_OPT_GROUP_MB 8
#define QD_OPT_SSF_FUSE 9
#define QD_SSF_AUTO 0
#define QD_SSF_SCAN 1
#define QD_SSF_SCAN_GATHER 2
#define QD_SSF_SCAN_NOSPLIT 3
int qd_graph_set_option(qd_graph* g, int32_t option, int32_t value);
int qd_graph_get_option(const qd_graph* g, int32_t option, int32_t* value);

/* Which table-driven SSF the handle's graph qualifies for: 1 when the wave
 * kernel's tables were built (ssf_lut_kernel: QD_SSF_AUTO then runs it), 2 when
 * only the score tables were (graphs beyond the wave shapes: the workgroup SSF
 * kernel scores generators by table lookup), 0 otherwise.  *lut_bytes
 * (nullable) = bytes of the score tables.  No reference counterpart. */
int qd_graph_ssf_tables(const qd_graph* g, int32_t* has_lut, int64_t* lut_bytes);
/* Copies of the table-driven SSF kernel's tables, for host-only graphs
 * (qd_graph_create_host; tests emulate the kernel's steps on them): lut
 * [lut_bytes / 4], off [g_pad], lcw [4][g_pad], tog [m_pad + 1][64] (u32 each; the
 * layouts of DevGraph::s_lut / s_off / s_lcw / s_tog in qdec_internal.h);
 * *g_pad and *m_pad receive the strides.  Any output may be NULL. */
/* Host-side layout of the handle's queue scratch for a batch of B shots (the
 * workspace attach_queue allocates; tests check its alignment and capacities
 * on host-only graphs): out[8] = total bytes, offsets of the shot-index array,
 * the hard-decision / packed-entry region, the residual region, the compact
 * lists' 2 x 64 segment counters (light, then heavy) and their entries, the
 * entries per segment, the
 * bytes per entry.  No reference counterpart. */
int qd_graph_queue_layout(const qd_graph* g, int64_t B, int64_t* out);

/* Copies of the triage's iteration-1 tables (host-only graphs): lut[n_pad]
 * (bit b = column j's hard decision after min-sum iteration 1 under syndrome
 * pattern b of its checks, in the kernels' precision and summation order) and
 * vchk[n_pad] (the checks of column j's edges, 4 x u16, pad = m).  Fails when
 * the precision has no tables (a prior <= 0).  No reference counterpart. */
int qd_graph_it1_tables_copy(const qd_graph* g, int32_t precision, uint16_t* lut, uint64_t* vchk, int32_t* n_pad);
/* Host-only graphs: the f64 LDS-resident kernel's check-state slots (m64_layout):
 * etab uint16 [4][n] (slot of edge k of column j, 0xffff pad), check_of_slot
 * uint16 [m].  -38 when the graph has none.  For tests. */
int qd_graph_lds64_slots_copy(const qd_graph* g, uint16_t* etab, uint16_t* check_of_slot);

int qd_graph_ssf_tables_copy(const qd_graph* g, uint32_t* lut, uint32_t* off, uint32_t* lcw, uint32_t* tog,
                             int32_t* g_pad, int32_t* m_pad);

/* Hypergraph-product kernel (qdec_hgp.cpp, qdec_hgp_kernel.hip).  When H =
 * [I_a0 (x) B | A (x) I_b0] (the Z checks of hgp.py homological_product, e.g.
 * biregular_hgp, reference python/qldpc/hypergraph_product_code.py:7-35), the
 * library generates an f64 min-sum BP kernel with B's and A's Tanner graphs as
 * compile-time tables and compiles it with hipRTC.  qd_graph_hgp_info: 1 and
 * out8 = {a0, a1, b0, b1, shot slots per workgroup, left waves, right waves,
 * workgroups per CU (0 before the first decode)} for such a graph, 0 otherwise.
 * qd_graph_hgp_source: the generated source (its length; copied into buf).
 * qd_graph_hgp_compile: compile only (no device needed).  No reference
 * counterpart (the reference decodes with ldpc's generic BpDecoder). */
int qd_graph_hgp_info(qd_graph* g, int32_t* out8);
/* Re-plan with `slots` shot slots per workgroup (0: the library's choice);
 * -95 when no workgroup shape holds `slots` (the previous plan stays). */
int qd_graph_hgp_set_slots(qd_graph* g, int32_t slots);
int64_t qd_graph_hgp_source(qd_graph* g, char* buf, int64_t cap);
int qd_graph_hgp_compile(qd_graph* g);
/* (Development builds with -DQDEC_DEV_HOOKS also export
 * qd_graph_hgp_replace_source(g, src), which recompiles an edited kernel
 * source; the product library does not.) */
/* BP only (f64 min-sum, ldpc v1 semantics as qd_decode_batch_device with
 * method QD_MIN_SUM, precision QD_F64, no SSF): device buffers syn [B][m],
 * x_out [B][n] (or null), iters [B], status [B] (bit 0: converged). */
int qd_graph_hgp_decode_bp(qd_graph* g, int64_t B, const uint8_t* syn, uint8_t* x_out, int32_t* iters,
                           uint8_t* status, int32_t max_iter, double ms_scaling, void* stream);

/* Device-side sum of a uint8 flag array (failure / status counts) into *out
 * (device int64, accumulated: caller zeroes it).  `mask` selects bits. */
int qd_count_flags_device(const uint8_t* flags, int64_t B, uint8_t mask, int64_t* out, void* stream);

/* GF(2) elimination on bit-packed rows (uint64 words, bit j at word j/64), host
 * cores.  Offline code-construction support for the logical operators the fused
 * failure check consumes; replaces galois row_reduce / null_space /
 * column_space in the reference's get_logicals
 * (python/qldpc/homological_product_code.py:6-60).
 * qd_gf2_rref: in-place reduced row echelon form over columns [0, ncols); the
 * first `rank` rows are the pivot rows, pivots[r] = their pivot columns
 * (nullable).  Returns rank, or < 0 on bad arguments.
 * qd_gf2_extend_basis: reduce each candidate row against an echelon basis (row b
 * has its lowest set bit at basis_lead[b]) plus the candidates accepted so far;
 * accepted[c] = 1 for candidates outside that span (at most max_accept when >= 0).
 * Returns the number accepted (homological_product_code.py:15-21). */
int64_t qd_gf2_rref(uint64_t* rows, int64_t nrows, int64_t words, int64_t ncols, int64_t* pivots, int32_t nthreads);
int64_t qd_gf2_extend_basis(const uint64_t* basis, int64_t nbasis, const int64_t* basis_lead, const uint64_t* cand,
                            int64_t ncand, int64_t words, int64_t ncols, uint8_t* accepted, int64_t max_accept);

#ifdef __cplusplus
}
#endif
#endif
