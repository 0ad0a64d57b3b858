// qdec_internal.h -- device-side graph description shared by the host ABI
// (qdec_abi.cpp) and the kernels (qdec_bp.hip, qdec_sample.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace qdec {

constexpr int kWave = 64;        // CDNA wavefront
constexpr int kDR = 8;           // max check degree of the wave kernels
constexpr int kDC = 4;           // max variable degree of the wave kernels
constexpr int kMlDRS = 8;        // LDS-resident min-sum kernel: row stride (elements), max check degree
constexpr int kMlDC = 4;         // LDS-resident min-sum kernel: max variable degree
constexpr int kGenW = 8;         // max flip-set generator weight (255 subsets)
constexpr int kGenLC = 32;       // max local checks per generator (u32 masks)
constexpr int kSsfScale = 840;   // lcm(1..8): gain/|F| compared as gain*(840/|F|)
constexpr int kLutLC = 16;       // table-driven SSF: max local checks per generator (16-bit local syndromes)
constexpr int kLutLCW = kLutLC / 4;  // words of u8 local-check ids per generator
constexpr int kEdgePad = 16;     // index / prior arrays padded past E (>= the largest row / column width)
constexpr int kCmpSegs = 64;     // segments (and counters) of each compact shot list
constexpr int kCmpLists = 2;     // the light list (segments 0..63) and the heavy list (64..127)
// entries a compact-list segment must hold for a batch of B shots (64-shot tiles)
inline int64_t cmp_seg_cap(int64_t B) { return ((B + 63) / 64 + kCmpSegs - 1) / kCmpSegs * 64; }

// Wave-kernel shapes (check rounds RC, variable rounds RV, check-node compute
// width D <= kDR): a graph is padded to the first shape that holds it (RC*64 >= m,
// RV*64 >= n, D >= max check degree), and the kernel is instantiated for exactly
// that shape so no per-round guard is needed.  (2, 4, 7) is the n = 225 HGP code.
#define QDEC_WAVE_SHAPES(X) X(1, 2, 8) X(2, 3, 6) X(2, 3, 8) X(2, 4, 7) X(2, 4, 8) X(2, 6, 8) X(4, 9, 8)
inline bool pick_wave_shape(int m, int n, int max_rdeg, int* rc, int* rv, int* drc) {
    const int need_c = (m + 63) / 64, need_v = (n + 63) / 64;
#define QDEC_PICK(R, V, D) \
    if (need_c <= R && need_v <= V && max_rdeg <= D) { *rc = R; *rv = V; *drc = D; return true; }
    QDEC_WAVE_SHAPES(QDEC_PICK)
#undef QDEC_PICK
    return false;
}

// LDS stride, in elements, of a per-lane block of D values of type T, chosen so a
// wave reading its 64 blocks with 16-byte ds_read_b128 is bank-conflict free:
// dword stride a multiple of 4 with an odd quotient (16 lanes cover 64 banks).
template <typename T, int D>
constexpr int lds_stride() {
    int dw = (int)((D * sizeof(T) + 3) / 4);
    dw = (dw + 3) / 4 * 4;
    if ((dw / 4) % 2 == 0) dw += 4;
    return dw * 4 / (int)sizeof(T);
}

// Slot tables depend on the element stride, i.e. on the precision.
struct SlotTables {
    const uint16_t* r_cslot;  // [kDR][m_pad]  c2v element written by check i, edge k
    const uint16_t* c_rslot;  // [kDC][n_pad]  v2c element written by variable j, edge k
};

struct DevGraph {
    int m, n, m_pad, n_pad;       // pads: multiples of 64
    int E;                        // edges (nnz of H)
    int wave;                     // 1: a wave-kernel shape holds this graph
    int n_data, fold_blocks;
    int max_rdeg, max_cdeg;
    int shape_drc;                // check-node compute width of the chosen wave shape
    const uint8_t* r_deg;         // [m_pad]
    const uint16_t* r_col;        // [kDR][m_pad]  column of edge k of check i (pad -> n_pad)
    const uint8_t* c_deg;         // [n_pad]
    SlotTables slots[2];          // [QD_F64], [QD_F32]
    const void* prior[2][2];      // [method][precision] initial message per column, [n_pad]
    // the same by CSR edge (the prior of edge e's column), [E + kEdgePad]
    // (slot-group kernel: one load per edge, no column-index chain)
    const void* eprior[2][2];
    // CSR / CSC copies (sampler; workgroup kernels)
    const int32_t* row_ptr;
    const int32_t* col_idx;
    const int32_t* col_ptr;       // [n+1]
    const int32_t* col_edge;      // [E] CSR edge ids of column j, ascending row
    const int32_t* edge_csc;      // [E] CSC position (col_ptr[col] + rank in column) of CSR edge e
    // col_idx, col_edge and edge_csc carry kEdgePad zero entries past E, so a
    // kernel may load a whole row's (column's) worth of indices unguarded
    // min-sum wave kernel with compressed check state (qdec_bp_ms.h).  Variables
    // sit in lane slots sorted by degree (ms_vslot); slot edge k scatters its v2c
    // message to element (etab & 0xffff) and gathers check state (etab >> 16);
    // pads -> a dummy element / the zero state m_pad.
    // Row positions inside a check's v2c row and the state slot of each check
    // are chosen on the host (per precision) to cut the LDS bank conflicts of
    // the scatter and of the state gather (ms_layout in qdec_abi.cpp).
    const uint32_t* ms_etab[2];   // [kDC][n_pad], per precision (element strides differ)
    const uint16_t* ms_sslot[2];  // [m_pad] state slot written by check lane i, per precision
    const uint64_t* ms_smask;     // [n_pad/64][m_pad] slots of check i's columns inside 64-slot word w
    const uint16_t* ms_vslot;     // [n_pad] column held by lane slot s (pads: n_pad + s % 64)
    const void* ms_prior[2];      // [precision][n_pad] min-sum priors in slot order
    int ms_d3r;                   // leading 64-slot rounds whose variables all have degree <= 3
    int ms_allpos;                // bit p: every prior LLR of precision p is > 0
    // iteration 1 of min-sum inside the triage (ms_triage_kernel, qdec_bp_ms.h):
    // the checks of column j's edges in edge order (4 x u16, pad -> m), the
    // columns of check i's row (8 x u16 over two words, pad -> n), and per
    // precision each column's hard decision after iteration 1 as a 16-bit table
    // over its checks' syndrome bits (nullptr unless every prior of that
    // precision is > 0; it1_tables in qdec_abi.cpp)
    const uint64_t* it1_vchk;     // [n_pad]
    const uint64_t* it1_cvar;     // [m_pad][2]
    const uint16_t* it1_lut[2];   // [precision][n_pad]
    int wave_occ;                 // qd_graph_set_wave_occupancy (0: default)
    // LDS-resident min-sum workgroup kernel (qdec_bp_block.hip, bp_ms_lds_kernel):
    // [kMlDC][n] LDS element of edge k of column j (row * kMlDRS + CSR position),
    // pad 0xffff; nullptr when the graph's degrees exceed kMlDRS / kMlDC
    const uint16_t* ml_etab;
    // bp_ms_lds64_kernel: check states live at host-placed slots (m64_layout,
    // qdec_abi.cpp): [kMlDC][n] state slot of edge k of column j (pad 0xffff),
    // and [m] the check held by each slot
    const uint16_t* m64_etab;
    const uint16_t* m64_check;
    int m64_d3r;                  // leading variable rounds (1024 columns each) of degree <= 3
    // flip sets (SSF)
    int n_gen, g_pad, g_wmax;
    const uint8_t* g_w;           // [g_pad]
    const uint16_t* g_q;          // [kGenW][g_pad]   qubit (column) k of generator g
    const uint8_t* g_nlc;         // [g_pad]
    const uint16_t* g_lc;         // [kGenLC][g_pad]  local check c of generator g
    const uint32_t* g_lc8;        // [kGenLC/4][g_pad] the same ids packed 4 per word (pad -> m_pad)
    int g_nlcmax;
    // inverse of the local-check lists, for the wave SSF kernel's incremental
    // local syndromes: [m_pad][g_invd] u16 entries g | (bit << 8) (generator g has
    // check i as local check `bit`), pad 0xffff; g_invd a power of two (log2:
    // g_invl).  nullptr when unavailable (the kernel re-gathers every step).
    const uint16_t* g_inv;
    int g_invd, g_invl;
    const uint32_t* g_qmask;      // [kGenW][g_pad]   local-check mask of qubit k
    // every generator's local checks inverted, CSR by check: entries of check i
    // are g_ient[g_iptr[i] .. g_iptr[i+1]), each g | (local bit << 16)
    // (ssf_inc_block_kernel; nullptr when n_gen >= 65536)
    const int32_t* g_iptr;
    const uint32_t* g_ient;
    // table-driven SSF (ssf_lut_kernel, qdec_bp.hip; built by ssf_lut_tables in
    // qdec_abi.cpp, nullptr when the graph does not qualify).  A generator's
    // local checks are put in a canonical order (by the set of its qubits that
    // touch them), so generators with the same local structure share one table
    // over their <= 16-bit local syndrome sl: s_lut[s_off[g] + sl] = rank << 24 |
    // M_t << 8 | t, t the spec's best subset (lowest bitmask among the best
    // gain/|t|), M_t the local checks it toggles, rank the position of its score
    // among all positive scores (0: no positive gain).  s_lcw: the canonical local
    // checks as u8 ids, 4 per word ([kLutLCW][g_pad], pad 0xff); s_tog: per check
    // c and lane l the local-syndrome bits that toggle when c flips, generator l
    // in the low half-word, generator 64 + l in the high one ([m_pad + 1][64],
    // row m_pad all zero).
    const uint32_t* s_lut;
    int s_lut_n;
    const uint32_t* s_off;
    const uint32_t* s_lcw;
    const uint32_t* s_tog;
    // logicals (fused failure check)
    int k, lz_words;
    const uint64_t* lz;           // [k][lz_words]    bit q%64 of word q/64 (nullptr when too large)
    const uint64_t* ms_lzs;       // wave graphs: [k][n_pad/64] the same by min-sum lane slot (ms_vslot order)
    // the same logicals as CSR supports over data qubits (always set with k > 0);
    // lz_sparse: the workgroup finalize tests logicals on their supports (nnz small
    // against k * lz_words) instead of by dense words
    const int32_t* lz_ptr;        // [k+1]
    const int32_t* lz_idx;        // [nnz]
    int lz_sparse;
    // the same logicals by qubit: word t of qubit q holds bit r % 32 of logical
    // r = 32 t + (r % 32) (nullptr when n_data * lz_tw words exceed 64 MB).  The
    // workgroup finalizes test a residual through it: only the residual's ones
    // read their qubit's lz_tw words, so a decoded shot (residual zero or a
    // stabilizer) costs a few words instead of k * lz_words
    const uint32_t* lz_t;         // [n_data][lz_tw]
    int lz_tw;
    // per-handle kernel choices (qd_graph_set_option, QD_OPT_* in include/qdec.h;
    // defaults from default_options): the launchers read these, never the
    // environment
    int opt_compact;       // 1: two-pass lean min-sum decodes (triage + compact list); 0: one-pass kernel
    int opt_triage_it1;    // 1: min-sum iteration 1 inside the triage; 0: left to the BP kernel
    int opt_ssf;           // QD_SSF_*: table-driven, scanning (incremental / re-gathered / unsplit scorer)
    int opt_lds_kernel;    // -1: automatic; 0: never; 1: forced (bp_ms_lds_kernel)
    int opt_group_kernel;  // -1: automatic; 0: never; 1: forced (bp_group_kernel)
    int opt_ssf_inc;       // 1: incremental workgroup SSF (ssf_inc_block_kernel); 0: the re-scanning one
    int opt_block_wg;      // > 0: workgroups per CU of the HBM-slice workgroup kernels (0: automatic)
    int opt_group_mb;      // > 0: HBM budget of the slot-group scratch in MiB (0: a quarter of free HBM)
    int opt_ssf_fuse;      // 1: two-pass SSF decodes run SSF inside the compact BP kernel (no queue, no
                           // second launch); 0 (default): queue + ssf_lut_kernel
};

// SSF kernel choice of wave graphs (DevGraph::opt_ssf)
enum { kSsfAuto = 0, kSsfScan = 1, kSsfScanGather = 2, kSsfScanNoSplit = 3 };
inline void default_options(DevGraph& g) {
    g.opt_compact = 1;
    g.opt_triage_it1 = 1;
    g.opt_ssf = kSsfAuto;
    g.opt_lds_kernel = -1;
    g.opt_group_kernel = -1;
    g.opt_ssf_inc = 1;
    g.opt_block_wg = 0;
    g.opt_group_mb = 0;
    g.opt_ssf_fuse = 0;  // measured: 2x the separate SSF kernel's time at p = 0.1 (profiles/r06c)
}

struct DecodeArgs {
    int64_t B;
    int max_iter, ssf, ssf_max_steps, syn_flags;
    double ms_scaling;
    const uint8_t* syn;
    const uint8_t* base;
    const uint8_t* readout;
    uint8_t* x_out;
    uint8_t* corr_out;
    void* llr_out;
    int32_t* iters;
    uint8_t* status;
    int32_t* ssf_steps;
    uint8_t* fail;
    // SSF work queue (device scratch owned by the graph handle)
    int32_t* q_count;  // [1]
    int64_t* q_idx;    // [B]   shot of queue slot
    uint8_t* q_x;      // [B][n] BP hard decision
    uint8_t* q_r;      // [B][m] residual syndrome
    // packed queue (wave kernels, q_packed = 1): entry s = q_w[s*(1+XW+RW) ..]:
    // shot index, hard decision by column (XW = n_pad/64 words), residual by
    // check (RW = m_pad/64 words); replaces q_idx/q_x/q_r
    int q_packed;
    uint64_t* q_w;
    // workgroup BP kernel with HBM message slices: shot counter handing out
    // shots dynamically (a straggler does not hold up a fixed stride of shots);
    // nullptr -> static stride.  Set by the launcher.
    unsigned long long* work_ctr;
    // min-sum wave kernel: counter of the dynamically scheduled shot chunks
    // (ShotSeq, qdec_bp_ms.h); zeroed by the launcher; nullptr -> static stride
    unsigned long long* wave_ctr;
    // SSF on a second stream (qd_graph_set_ssf_stream, wave kernels only): the
    // SSF kernel waits for ssf_ev (recorded after the BP kernel) on ssf_stream,
    // so a later BP launch on the BP stream can overlap it; nullptr -> same stream
    hipStream_t ssf_stream;
    hipEvent_t ssf_ev;
    // SSF wave kernel: 1 disables the two-lanes-per-generator scoring of short
    // listing steps (QDEC_SSF_NOSPLIT=1; parity tests run both ways)
    int ssf_nosplit;
    // optional timing (host side only): events recorded on the launch stream
    // before the BP kernel, after it, after the SSF kernel, and after the BP
    // stage's pre-pass (record_ev)
    hipEvent_t* ev;    // [4] or nullptr
    // compact shot list of lean min-sum wave launches (ms_triage_kernel ->
    // bp_ms_cmp_kernel), in kCmpLists x kCmpSegs segments: triage tile t appends
    // to segment t % kCmpSegs (light shots) and kCmpSegs + t % kCmpSegs (heavy
    // ones, decoded first), whose entries [cmp_cap][CmpEntry::EW] u64 start at
    // cmp + s * cmp_cap * EW, counted at cmp_count[s * 16] (one 128-B line per
    // counter; zeroed by the launcher).  nullptr -> no compact path
    uint64_t* cmp;
    unsigned long long* cmp_count;
    // the other counter set of the handle (double-buffered): the triage zeroes
    // it for the handle's next two-pass decode, so no decode needs a memset
    // launch (nullptr: the launcher memsets cmp_count itself)
    unsigned long long* cmp_count_next;
    int64_t cmp_cap;
    int cmp_zero_ok;  // every prior of the launch's precision > 0: zero syndromes finish in the triage
    // the triage runs iteration 1 itself (g.it1_lut of the launch's precision;
    // set by the launcher when the schedule's alpha_1 is 0.5): shots whose
    // iteration-1 decision meets the syndrome finish there
    const uint16_t* it1_lut;
    // packed SSF queue entries carry the readout's logical parities (bit r of
    // the dw area = parity of Lz[r] . readout) instead of the readout words
    int q_rpar;
    // QD_INPUT_PACKED: syn / base / readout are bit-packed rows of u64 words
    // (syn [B][ceil(m/64)], base / readout [B][ceil(n_data/64)]; bit j of word
    // w = element 64 w + j).  The two-pass path's triage reads them directly;
    // every other path first expands them into unpack_buf (library-owned,
    // B * (m + 2 n_data) bytes) with unpack_rows_kernel.
    int in_packed;
    uint8_t* unpack_buf;
};

// Arguments of the GPU OSD stage (qdec_osd.hip).  Shots whose status has bit 0
// (BP converged) set are skipped; outputs of other shots are left untouched.
struct OsdArgs {
    int64_t B;
    int method, order, syn_flags, llr_f32;
    const uint8_t* syn;      // [B][m] (nullable with syn_flags)
    const void* llr;         // [B][n] float or double: BP log-probability ratios
    const uint8_t* status;   // [B] nullable: every shot is post-processed
    const uint8_t* base;     // [B][n_data] nullable
    const uint8_t* readout;  // [B][n_data] nullable
    uint8_t* osd0_out;       // [B][n] nullable
    uint8_t* osdw_out;       // [B][n] nullable
    uint8_t* corr_out;       // [B][n_data] nullable: base ^ fold(osdw)
    uint8_t* fail;           // [B] nullable: any(Lz (readout ^ corr))
};
bool osd_kernel_supports(const DevGraph& g);
int launch_osd(const DevGraph& g, const OsdArgs& a, int num_cus, hipStream_t stream);

// ev[3] marks the end of a pre-pass inside the BP timing (the shot triage):
// recorded with ev[0] and again after the pre-pass when one runs
inline void record_ev(const DecodeArgs& a, int i, hipStream_t s) {
    if (!a.ev) return;
    (void)hipEventRecord(a.ev[i], s);
    if (i == 0) (void)hipEventRecord(a.ev[3], s);
}

// Names of the BP and SSF kernels the calling host thread's last launch_decode
// enqueued, spelled as rocprofv3 prints them (template arguments included; ""
// when none / not recorded).  Host only; read by qd_graph_last_kernels.
struct LaunchNames {
    const char* bp = "";
    const char* ssf = "";
    const char* pre = "";  // a pass before the BP kernel (ms_triage_kernel), inside the BP timing
};
LaunchNames& last_launch_names();

// rocprofv3's spelling of a kernel instantiation: base<arg, arg, ...>
inline std::string targ(bool b) { return b ? "true" : "false"; }
inline std::string targ(int v) { return std::to_string(v); }
inline std::string targ(const char* s) { return s; }
template <typename T>
inline const char* tname() { return sizeof(T) == 8 ? "double" : "float"; }
template <typename... A>
inline std::string kernel_name(const char* base, A... args) {
    std::string s = std::string(base) + "<";
    bool first = true;
    ((s += (first ? std::string() : std::string(", ")) + targ(args), first = false), ...);
    return s + ">";
}
// record the instantiation (one string per call site and instantiation)
#define QDEC_NOTE_BP(...)                                           \
    do {                                                            \
        static const std::string qdec_kn_ = kernel_name(__VA_ARGS__); \
        last_launch_names().bp = qdec_kn_.c_str();                  \
    } while (0)
#define QDEC_NOTE_PRE(...)                                          \
    do {                                                            \
        static const std::string qdec_kn_ = kernel_name(__VA_ARGS__); \
        last_launch_names().pre = qdec_kn_.c_str();                 \
    } while (0)
#define QDEC_NOTE_SSF(...)                                          \
    do {                                                            \
        static const std::string qdec_kn_ = kernel_name(__VA_ARGS__); \
        last_launch_names().ssf = qdec_kn_.c_str();                 \
    } while (0)


// Launchers (qdec_bp.hip / qdec_sample.hip).  Return hipError_t as int.
int launch_decode(const DevGraph& g, int method, int precision, const DecodeArgs& a,
                  int num_cus, hipStream_t stream, void* scratch, size_t scratch_bytes);
int launch_decode_block(const DevGraph& g, int method, int precision, const DecodeArgs& a, int num_cus,
                        hipStream_t stream, void* scratch, size_t scratch_bytes);
int launch_ssf_block(const DevGraph& g, const DecodeArgs& a, int num_cus, hipStream_t stream);
size_t block_scratch_bytes(const DevGraph& g, int method, int precision, int num_cus, const DecodeArgs& a);
size_t block_scratch_floor(const DevGraph& g, int method, int precision, int num_cus, const DecodeArgs& a);
bool group_kernel_applies(const DevGraph& g, int method, int precision, const DecodeArgs& a);
bool lds_kernel_applies(const DevGraph& g, int method, int precision, const DecodeArgs& a);
int launch_sample_storage(const DevGraph& g, int rounds, uint32_t thr_data, uint32_t thr_meas,
                          uint32_t seed, uint32_t stream_id, int64_t shot0, int64_t B,
                          uint8_t* syn, uint8_t* readout, int num_cus, hipStream_t stream, bool packed = false);
int launch_count_flags(const uint8_t* flags, int64_t B, uint8_t mask, int64_t* out, hipStream_t stream);

// ---------------------------------------------------------------- HGP kernel
// Hypergraph-product codes get their own f64 min-sum BP kernel, generated and
// compiled per code with hipRTC (qdec_hgp.cpp, qdec_hgp_kernel.hip).
struct HgpPlan;
struct HgpBpArgs {  // the kernel's HgArgs, field for field
    const uint8_t* syn;           // [B][m]
    const double* prior;          // [n] min-sum prior per column
    uint8_t* x_out;               // [B][n] or null
    int32_t* iters;               // [B] or null
    uint8_t* status;              // [B] or null (bit 0: BP converged)
    unsigned long long* counter;  // shot counter (zeroed by hgp_launch_bp)
    int64_t B;
    int32_t max_iter;
    double ms_scaling;
};
// nullptr unless H = [I_a0 (x) B | A (x) I_b0] within the kernel's limits
// slots: shot slots per workgroup (0: the plan's choice)
HgpPlan* hgp_plan_create(int m, int n, const std::vector<int32_t>& rp, const std::vector<int32_t>& ci, int slots = 0);
void hgp_plan_destroy(HgpPlan* P);
const std::string& hgp_plan_source(const HgpPlan* P);
void hgp_plan_replace_source(HgpPlan* P, const std::string& src);  // development
int hgp_plan_compile(HgpPlan* P, const char* arch, std::string* log);  // hipRTC (no device needed)
int hgp_plan_load(HgpPlan* P, int num_cus, const char* arch);           // compile + load on the current device
std::string hgp_target_arch(int device);  // hipRTC target of `device` (< 0: the build's QDEC_ARCH)
int hgp_launch_bp(HgpPlan* P, const HgpBpArgs& a, hipStream_t stream);
void hgp_plan_info(const HgpPlan* P, int* out8);  // a0 a1 b0 b1 S WL WR per_cu

}  // namespace qdec
