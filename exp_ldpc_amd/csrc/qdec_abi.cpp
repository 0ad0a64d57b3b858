// qdec_abi.cpp -- extern "C" entry points of libqdec_hip.so (include/qdec.h).
//
// Host-side graph preparation: CSR -> per-lane slot tables for the wave
// kernels, flip-set tables for SSF, bit-packed logicals, priors in both
// precisions; device upload; launches.  No C++ exception crosses the ABI.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <mutex>
#include <random>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/qdec.h"
#include "qdec_internal.h"

using namespace qdec;

namespace {

thread_local std::string g_last_error;

struct Fail : std::runtime_error {
    int code;
    Fail(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw Fail(-100 - (int)e, std::string(what) + ": " + hipGetErrorString(e));
}

template <typename F>
int guarded(F&& f) {
    try {
        f();
        return 0;
    } catch (const Fail& e) {
        g_last_error = e.what();
        return e.code;
    } catch (const std::exception& e) {
        g_last_error = e.what();
        return -99;
    } catch (...) {
        g_last_error = "unknown error";
        return -99;
    }
}

// A device allocation list owned by the graph.  A host-only arena
// (qd_graph_create_host: table builds without a GPU, for tests and sanitizer
// runs) keeps host copies instead and makes no HIP call.
struct DevArena {
    std::vector<void*> ptrs;
    bool host = false;
    std::vector<std::vector<uint8_t>> kept;  // host-only: the uploaded bytes, in order
    template <typename T>
    const T* upload(const std::vector<T>& h) {
        const size_t bytes = std::max<size_t>(h.size() * sizeof(T), 16);
        if (host) {
            kept.emplace_back(bytes, 0);
            if (!h.empty()) std::memcpy(kept.back().data(), h.data(), h.size() * sizeof(T));
            return reinterpret_cast<const T*>(kept.back().data());
        }
        void* d = nullptr;
        hip_check(hipMalloc(&d, bytes), "hipMalloc");
        ptrs.push_back(d);
        if (!h.empty()) hip_check(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice), "hipMemcpy H2D");
        return static_cast<const T*>(d);
    }
    void release() {
        for (void* p : ptrs) (void)hipFree(p);
        ptrs.clear();
        kept.clear();
    }
};

}  // namespace

struct qd_graph {
    int device = 0;
    int num_cus = 0;
    hipStream_t stream = nullptr;
    DevGraph dg{};
    bool has_priors = false;
    // host copies needed to rebuild tables
    std::vector<int32_t> row_ptr, col_idx;
    std::vector<int32_t> col_ptr, col_rows;  // CSC (row ids, ascending)
    DevArena arena;                          // graph tables
    DevArena flip_arena, lz_arena, prior_arena;
    // workspace for the host-buffer API (grow only)
    void* ws = nullptr;
    size_t ws_bytes = 0;
    // SSF work queue scratch (grow only): count | idx[B] | x[B][n] | r[B][m]
    void* qws = nullptr;
    int64_t q_cap = 0;
    // HBM message scratch for the workgroup kernels on graphs too large for LDS
    void* mws = nullptr;
    size_t mws_bytes = 0;
    // QD_INPUT_PACKED decodes off the two-pass path: the inputs expanded to
    // byte rows (grow only; DecodeArgs::unpack_buf)
    void* ubuf = nullptr;
    size_t ubuf_bytes = 0;
    // compact-list segment counters, two sets (DecodeArgs::cmp_count_next):
    // two-pass decodes alternate between them, each triage zeroing the other
    void* cmpc = nullptr;
    int cmp_par = 0;
    size_t mws_failed = 0;  // smallest scratch size whose allocation failed (0: none)
    uint64_t mws_capped_calls = 0;  // calls served the reduced scratch since the failure
    // kernel timing ring (qd_graph_set_timing): 3 events per decode call
    // [0..3] around the launch's kernels (record_ev), [4] behind the copy of
    // the compact-list counters (note_listed): kTimingEvents per call
    std::vector<hipEvent_t> tev;
    int t_cap = 0, t_count = 0;
    // per timed call: compact-list length of a two-pass launch (summed segment
    // counters, copied into pinned memory behind the launch), -1 otherwise
    uint64_t* t_listed = nullptr;  // [t_cap][kCmpLists * kCmpSegs], hipHostMalloc
    std::vector<int> t_cmp;
    // min-sum wave kernel: variable (column) held by each lane slot, -1 for pads
    std::vector<int> ms_var_of_slot;
    // workspace chain: every device-buffer decode records ws_ev on its stream after
    // its launches; a decode on another stream waits for it first, so the queue and
    // message scratch of one handle are never used by two streams at once, and a
    // grow path frees a buffer only after ws_ev (the last use) has completed
    hipEvent_t ws_ev = nullptr;
    bool ws_ev_live = false;
    // 256-B control block: [0] shot-chunk counter of the min-sum wave kernel
    void* ctl = nullptr;
    // qd_graph_set_ssf_stream: SSF kernels of device-buffer decodes go to this
    // stream behind ssf_ev (nullptr: the decode's own stream)
    hipStream_t ssf_stream = nullptr;
    hipEvent_t ssf_ev = nullptr;
    // split-SSF decodes alternate between two SSF queues (queue 1: qws2, the
    // SSF region of the layout; control words ctl + 32 * q), so a decode waits
    // for the SSF kernel of the decode two back on this handle, not the last
    // one: ssf_done[q] is recorded on the SSF stream behind the kernel that
    // used queue q
    void* qws2 = nullptr;
    int64_t q2_cap = 0;
    int q_buf = 0;
    hipEvent_t ssf_done[2] = {nullptr, nullptr};
    bool ssf_done_live[2] = {false, false};
    hipStream_t ws_last = nullptr;
    // kernels the last decode on this handle launched (qd_graph_last_kernels)
    std::string last_bp, last_ssf, last_pre;
    // qd_graph_create_host: tables only, no device, no stream; decodes refuse it
    bool host_only = false;
    // hypergraph-product kernel (qd_graph_hgp_*): plan once per graph
    HgpPlan* hgp = nullptr;
    bool hgp_tried = false;
};

namespace {

constexpr int kTimingEvents = 5;
constexpr size_t kCtlBytes = 512;  // control words: queue q's at ctl + 32 q (u64), the HGP counter at 16

template <typename T>
int drs() { return lds_stride<T, kDR>(); }
template <typename T>
int dcs() { return lds_stride<T, kDC>(); }

void set_device(qd_graph* g) {
    if (!g->host_only) hip_check(hipSetDevice(g->device), "hipSetDevice");
}

// Workspace chain (see qd_graph::ws_ev).
void ws_acquire(qd_graph* G, hipStream_t s) {
    if (G->ws_ev_live && G->ws_last != s) hip_check(hipStreamWaitEvent(s, G->ws_ev, 0), "hipStreamWaitEvent");
}
void ws_release(qd_graph* G, hipStream_t s) {
    if (!G->ws_ev) hip_check(hipEventCreateWithFlags(&G->ws_ev, hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventRecord(G->ws_ev, s), "hipEventRecord");
    G->ws_ev_live = true;
    G->ws_last = s;
}
void ws_drain(qd_graph* G) {
    if (G->ws_ev_live) hip_check(hipEventSynchronize(G->ws_ev), "hipEventSynchronize");
    for (int q = 0; q < 2; ++q)
        if (G->ssf_done_live[q]) hip_check(hipEventSynchronize(G->ssf_done[q]), "hipEventSynchronize");
}

// Layout of the compressed-state min-sum kernel (qdec_bp_ms.h).  Variable
// lane j = rv*64 + l scatters its k-th v2c message to element i*DRS + pos of
// check i's row.  One ds_write_b32 per (rv, k) serves 2 x 32 lanes, bank =
// dword % 32.  It costs max(4, L0 + L1) cycles, where L_h is the worst bank
// load in half h.  The check pass takes min/sign over the whole row, which is
// independent of the row order, so edge positions inside a row are free.  A
// seeded hill climb over position swaps drives every instruction to <= 2-way
// conflicts (tie-break: sum of squared loads).  Pad lanes of an instruction all
// write one dummy element, placed in the least-loaded bank.
// Check-state slots of bp_ms_lds64_kernel (f64, one shot per CU; qdec_bp_block.hip).
// Its variable thread t owns columns r * 1024 + (67 t mod 1024); per (wave,
// round r, edge k) one LDS instruction of 64 lanes reads or atomically updates
// the state of each lane's k-th check.  The banking gfx950 applies
// (tools/dev/lds_atomic_probe.hip): the u64 m1 / m2 reads (ds_read_b64) in two
// 32-lane halves, key slot mod 32; the u64 atomics (ds_min(_rtn)_u64) in four
// 16-lane quarters, key slot mod 16; the bit words (parw / hdw: word = slot >> 5)
// in halves, key word mod 32.  With checks in their natural order a group's
// lanes land on ~3-4 lanes per bank.  A seeded anneal over slot swaps spreads
// every group over its banks (objective: sum of squared lanes per bank, all
// three keys; tools/dev/c4_bank_model2.py's max-per-bank cycles on C4: 23,102
// natural -> 16,086, conflict-free 7,600; an anneal of the max model itself,
// tools/dev/c4_slots_anneal2.cpp, stops at the same 16.2k).  The kernel then works in
// slot space; m64_check maps a slot back to its check for the syndrome input and
// the residual output.  Cached per process like ms_layout.
void m64_layout(qd_graph* G, int m, int n, const std::vector<int32_t>& rp, const std::vector<int32_t>& ci,
                const std::vector<int>& edge_cpos) {
    DevGraph& g = G->dg;
    struct Entry {
        std::vector<int32_t> rp, ci;
        std::vector<uint16_t> et, chk;
        int d3r;
    };
    static std::mutex mu;
    static std::vector<Entry> cache;
    {
        std::lock_guard<std::mutex> lk(mu);
        for (const auto& c : cache)
            if (c.rp == rp && c.ci == ci) {
                g.m64_etab = G->arena.upload(c.et);
                g.m64_check = G->arena.upload(c.chk);
                g.m64_d3r = c.d3r;
                return;
            }
    }
    constexpr int T = 1024;  // kM64Threads
    const int E = rp[m];
    // k-th check of every column (edge_cpos order, as ml_etab)
    std::vector<int> colchk((size_t)kMlDC * n, -1);
    for (int i = 0; i < m; ++i)
        for (int e = rp[i]; e < rp[i + 1]; ++e)
            if (edge_cpos[e] < kMlDC) colchk[(size_t)edge_cpos[e] * n + ci[e]] = i;
    // the lane groups of one instruction: 32-lane halves (ds_read_b64 of m1 / m2,
    // key slot mod 32; b32 words, key (slot >> 5) mod 32) and 16-lane quarters
    // (ds_min(_rtn)_u64 on m1 / m2, key slot mod 16) -- the banking measured by
    // tools/dev/lds_atomic_probe.hip; occurrences of each check in both
    std::vector<std::vector<int>> halves, quarters;
    const int rounds = (n + T - 1) / T;
    for (int w = 0; w < T / 64; ++w)
        for (int r = 0; r < rounds; ++r)
            for (int k = 0; k < kMlDC; ++k)
                for (int q = 0; q < 4; ++q) {
                    std::vector<int> qq;
                    for (int l = 16 * q; l < 16 * q + 16; ++l) {
                        const int j = r * T + ((64 * w + l) * 67) % T;
                        if (j < n && colchk[(size_t)k * n + j] >= 0) qq.push_back(colchk[(size_t)k * n + j]);
                    }
                    if (q & 1) {  // the half: this quarter and the one before it
                        std::vector<int> hh(quarters.back());
                        hh.insert(hh.end(), qq.begin(), qq.end());
                        if (!hh.empty()) halves.push_back(std::move(hh));
                    }
                    quarters.push_back(std::move(qq));
                }
    const int nh = (int)halves.size(), nq = (int)quarters.size();
    std::vector<std::vector<int>> occ(m), occq(m);
    for (int h = 0; h < nh; ++h)
        for (int i : halves[h]) occ[i].push_back(h);
    for (int q = 0; q < nq; ++q)
        for (int i : quarters[q]) occq[i].push_back(q);
    std::vector<int> slot(m);
    for (int i = 0; i < m; ++i) slot[i] = i;
    std::vector<int> cx((size_t)nh * 32, 0), cy((size_t)nh * 32, 0), cz((size_t)nq * 16, 0);
    auto X = [](int s) { return s & 31; };
    auto Y = [](int s) { return (s >> 5) & 31; };
    auto Z = [](int s) { return s & 15; };
    for (int h = 0; h < nh; ++h)
        for (int i : halves[h]) ++cx[(size_t)h * 32 + X(slot[i])], ++cy[(size_t)h * 32 + Y(slot[i])];
    for (int q = 0; q < nq; ++q)
        for (int i : quarters[q]) ++cz[(size_t)q * 16 + Z(slot[i])];
    // per edge: two u64 reads (halves), two u64 atomics (quarters), one b32 read
    // and the occasional b32 xor (halves)
    const double WX = 2.0, WZ = 2.0, WY = 1.5;
    auto move = [&](int i, int from, int to) {
        for (int h : occ[i]) {
            --cx[(size_t)h * 32 + X(from)], --cy[(size_t)h * 32 + Y(from)];
            ++cx[(size_t)h * 32 + X(to)], ++cy[(size_t)h * 32 + Y(to)];
        }
        for (int q : occq[i]) --cz[(size_t)q * 16 + Z(from)], ++cz[(size_t)q * 16 + Z(to)];
    };
    auto local = [&](int i, int s) {  // check i's share of the squared loads at slot s
        double c = 0;
        for (int h : occ[i]) c += WX * (2 * cx[(size_t)h * 32 + X(s)] - 1) + WY * (2 * cy[(size_t)h * 32 + Y(s)] - 1);
        for (int q : occq[i]) c += WZ * (2 * cz[(size_t)q * 16 + Z(s)] - 1);
        return c;
    };
    std::mt19937_64 rng(20250221);
    std::uniform_real_distribution<double> uni(0.0, 1.0);
    const long iters = m > 1 ? std::min<long>(6000000L, 1500L * E) : 0;
    const double T0 = 1.0, T1 = 0.01;
    for (long it = 0; it < iters; ++it) {
        const int i = (int)(rng() % (uint64_t)m), j = (int)(rng() % (uint64_t)m);
        const int si = slot[i], sj = slot[j];
        if (i == j || (X(si) == X(sj) && Y(si) == Y(sj))) continue;
        const double before = local(i, si) + local(j, sj);
        move(i, si, sj);
        move(j, sj, si);
        const double d = local(i, sj) + local(j, si) - before;
        const double temp = T0 * std::pow(T1 / T0, (double)it / (double)iters);
        if (d <= 0 || uni(rng) < std::exp(-d / temp)) {
            slot[i] = sj;
            slot[j] = si;
        } else {
            move(j, si, sj);
            move(i, sj, si);
        }
    }
    // leading rounds whose columns all have degree <= 3 (the kernel's D3R)
    int d3r = 0;
    while (d3r < rounds) {
        bool ok = true;
        for (int j = d3r * T; j < std::min(n, (d3r + 1) * T) && ok; ++j) ok = colchk[(size_t)(kMlDC - 1) * n + j] < 0;
        if (!ok) break;
        ++d3r;
    }
    Entry e{rp, ci, std::vector<uint16_t>((size_t)kMlDC * n, 0xffff), std::vector<uint16_t>(m), d3r};
    for (size_t t = 0; t < colchk.size(); ++t)
        if (colchk[t] >= 0) e.et[t] = (uint16_t)slot[colchk[t]];
    for (int i = 0; i < m; ++i) e.chk[slot[i]] = (uint16_t)i;
    g.m64_etab = G->arena.upload(e.et);
    g.m64_check = G->arena.upload(e.chk);
    g.m64_d3r = d3r;
    std::lock_guard<std::mutex> lk(mu);
    if (cache.size() >= 8) cache.erase(cache.begin());
    cache.push_back(std::move(e));
}

void ms_layout(qd_graph* G, int m, int n, const std::vector<int>& edge_cpos) {
    DevGraph& g = G->dg;
    const auto& rp = G->row_ptr;
    const auto& ci = G->col_idx;
    const int E = rp[m];
    const int drc = g.shape_drc;
    const int RVn = g.n_pad / 64;
    // Lane slots of the variables: ascending column degree (stable), so the
    // leading 64-variable rounds whose variables all have degree <= 3 run a
    // 3-edge variable pass (ms_d3r).  Each variable's arithmetic is unchanged.
    std::vector<int> order(n);
    for (int j = 0; j < n; ++j) order[j] = j;
    auto cdeg = [&](int j) { return G->col_ptr[j + 1] - G->col_ptr[j]; };
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return cdeg(x) < cdeg(y); });
    std::vector<int> slot_of(n);
    G->ms_var_of_slot.assign(g.n_pad, -1);
    for (int s2 = 0; s2 < n; ++s2) {
        slot_of[order[s2]] = s2;
        G->ms_var_of_slot[s2] = order[s2];
    }
    g.ms_d3r = 0;
    for (int r = 0; r < RVn; ++r) {
        bool ok = true;
        for (int l = 0; l < 64; ++l) {
            const int j = G->ms_var_of_slot[r * 64 + l];
            if (j >= 0 && cdeg(j) > 3) ok = false;
        }
        if (!ok) break;
        g.ms_d3r = r + 1;
    }
    const int D3P = g.ms_d3r & ~1;  // leading 3-edge round pairs: no k = 3 instruction
    std::vector<int> row_of(E);
    for (int i = 0; i < m; ++i)
        for (int e = rp[i]; e < rp[i + 1]; ++e) row_of[e] = i;
    const int NG = RVn * kDC;
    auto has_pad = [&](int gi, int l) {
        const int j = G->ms_var_of_slot[(gi / kDC) * 64 + l];
        return j < 0 || gi % kDC >= cdeg(j);
    };
    const int DRS[2] = {drs<double>(), drs<float>()};
    // The placement below is a deterministic function of the graph; it is cached
    // per process (several handles on one graph, e.g. one per sweep point).
    struct LayoutCache {
        std::vector<int32_t> rp, ci;
        int m_pad, n_pad;
        std::vector<uint32_t> etab[2];
        std::vector<uint16_t> ss16[2];
    };
    static std::mutex cache_mu;
    static std::vector<LayoutCache> cache;
    {
        std::lock_guard<std::mutex> lk(cache_mu);
        for (const auto& c : cache)
            if (c.m_pad == g.m_pad && c.n_pad == g.n_pad && c.rp == rp && c.ci == ci) {
                for (int p = 0; p < 2; ++p) {
                    g.ms_sslot[p] = G->arena.upload(c.ss16[p]);
                    g.ms_etab[p] = G->arena.upload(c.etab[p]);
                }
                goto tables_done;
            }
    }
    {
    LayoutCache entry{rp, ci, g.m_pad, g.n_pad, {}, {}};
    std::mt19937 rng(12345);
    for (int p = 0; p < 2; ++p) {
        // ---- v2c scatter: one ds_write per (rv, k).  f32 (ds_write_b32): 2 lane
        // groups of 32, class = dword % 32, cost max(4, L0 + L1).  f64
        // (ds_write_b64): 4 groups of 16 contiguous lanes, class = element % 16,
        // cost max(6, sum of L).  Row positions are free (min/sign over the row).
        // f64: the transfer of a ds_write_b64 takes 6 cycles but every array
        // cycle beyond 4 is a bank-conflict cycle the CU's other waves wait
        // for (PMC: the array is the busiest unit), so the floor is 4
        const int ngl = p == 1 ? 2 : 4, ncl = p == 1 ? 32 : 16, floor_c = 4;
        const int lanes_per = 64 / ngl;
        std::vector<int> grp(E), lg(E), pos(E);
        for (int i = 0; i < m; ++i)
            for (int e = rp[i], t = 0; e < rp[i + 1]; ++e, ++t) {
                const int sl = slot_of[ci[e]];
                grp[e] = (sl / 64) * kDC + edge_cpos[e];
                lg[e] = (sl % 64) / lanes_per;
                pos[e] = t;
            }
        std::vector<int> load((size_t)NG * ngl * ncl, 0);
        auto cls = [&](int e) { return (row_of[e] * DRS[p] + pos[e]) % ncl; };
        for (int e = 0; e < E; ++e) load[((size_t)grp[e] * ngl + lg[e]) * ncl + cls(e)]++;
        auto gcost = [&](int gi) {
            int sum = 0, sq = 0;
            for (int h = 0; h < ngl; ++h) {
                int mx = 0;
                for (int b = 0; b < ncl; ++b) {
                    const int v = load[((size_t)gi * ngl + h) * ncl + b];
                    mx = std::max(mx, v);
                    sq += v * v;
                }
                sum += mx;
            }
            return (long)std::max(floor_c, sum) * 100000 + sq;
        };
        for (int iter = 0; iter < 40 * E; ++iter) {
            const int i = (int)(rng() % (unsigned)m);
            const int deg = rp[i + 1] - rp[i];
            if (deg < 1) continue;
            const int e1 = rp[i] + (int)(rng() % (unsigned)deg);
            const int p2 = (int)(rng() % (unsigned)drc);
            int e2 = -1;
            for (int e = rp[i]; e < rp[i + 1]; ++e)
                if (pos[e] == p2) e2 = e;
            if (e2 == e1) continue;
            const int g1 = grp[e1], g2 = e2 >= 0 ? grp[e2] : -1;
            const long before = gcost(g1) + (g2 >= 0 && g2 != g1 ? gcost(g2) : 0);
            auto move = [&](int e, int newpos) {
                load[((size_t)grp[e] * ngl + lg[e]) * ncl + cls(e)]--;
                pos[e] = newpos;
                load[((size_t)grp[e] * ngl + lg[e]) * ncl + cls(e)]++;
            };
            const int p1 = pos[e1];
            move(e1, p2);
            if (e2 >= 0) move(e2, p1);
            const long after = gcost(g1) + (g2 >= 0 && g2 != g1 ? gcost(g2) : 0);
            if (after > before) {  // undo
                if (e2 >= 0) move(e2, p2);
                move(e1, p1);
            }
        }
        // pad lanes of an instruction write one dummy element past the rows, in
        // the class least loaded over the lane groups that hold pads
        const int dstart = (m + 1) * DRS[p];  // past the m rows and the shared Big row (MsLds::rows)
        std::vector<int> dummy(NG, dstart);
        for (int gi = 0; gi < NG; ++gi) {
            std::vector<bool> pads(ngl, false);
            for (int l = 0; l < 64; ++l)
                if (has_pad(gi, l)) pads[l / lanes_per] = true;
            int bestb = 0, bestc = 1 << 30;
            for (int b = 0; b < ncl; ++b) {
                int c = 0;
                for (int h = 0; h < ngl; ++h)
                    if (pads[h]) c = std::max(c, load[((size_t)gi * ngl + h) * ncl + b]);
                if (c < bestc) { bestc = c; bestb = b; }
            }
            dummy[gi] = dstart + ((bestb - dstart % ncl) % ncl + ncl) % ncl;
        }
        // ---- check state (m1, m2): check i's state lives at slot sst[i] in
        // [0, m_pad); slot m_pad is the zero state read by pad lanes.  Variable
        // lanes gather it once per (rv, k): f32 ds_read_b64 (2 groups of 32 lanes,
        // class = slot % 32), f64 ds_read_b128 (4 groups of 16 lanes in the
        // hardware's grouping, class = slot % 16).  Only distinct slots in one
        // class of one group conflict; the anneal below minimises the sum over
        // instructions and groups of the worst class load.
        // every check lane, pads included, writes its state once per iteration:
        // f64 ds_write_b128 (8 groups of 8 contiguous lanes, class = slot % 8),
        // f32 ds_write_b64 (4 groups of 16, class = slot % 16); the anneal adds
        // the worst class load of each group (round 2 placed only the gathers:
        // modelled 37 state-write array cycles per iteration for f64, ideal 16)
        std::vector<int> sst(g.m_pad);
        for (int i = 0; i < g.m_pad; ++i) sst[i] = i;
        {
            const int rcl = p == 1 ? 32 : 16;
            auto rgroup = [&](int l) -> int {
                if (p == 1) return l / 32;
                const int q = l % 32, h = (l / 32) * 2;  // {0-3,12-15,20-27} / {4-11,16-19,28-31}
                return h + ((q < 4 || (q >= 12 && q < 16) || (q >= 20 && q < 28)) ? 0 : 1);
            };
            const int nrg = p == 1 ? 2 : 4;
            std::vector<std::vector<int>> mem;  // distinct checks per (instruction, group)
            std::vector<char> gpad;
            for (int gi = 0; gi < NG; ++gi) {
                if (gi / kDC < D3P && gi % kDC == 3) continue;
                std::vector<std::vector<int>> gm(nrg);
                std::vector<char> gp(nrg, 0);
                for (int l = 0; l < 64; ++l) {
                    const int j = G->ms_var_of_slot[(gi / kDC) * 64 + l];
                    if (j < 0 || gi % kDC >= cdeg(j)) { gp[rgroup(l)] = 1; continue; }
                    const int i = G->col_rows[G->col_ptr[j] + gi % kDC];
                    auto& v = gm[rgroup(l)];
                    if (std::find(v.begin(), v.end(), i) == v.end()) v.push_back(i);
                }
                for (int h = 0; h < nrg; ++h) {
                    mem.push_back(gm[h]);
                    gpad.push_back(gp[h]);
                }
            }
            const int NGR = (int)mem.size();
            std::vector<std::vector<int>> app(m);
            for (int q = 0; q < NGR; ++q)
                for (int i : mem[q]) app[i].push_back(q);
            auto qcost = [&](int q) {
                int cnt[32] = {0};
                int mx = 0;
                for (int i : mem[q]) mx = std::max(mx, ++cnt[sst[i] % rcl]);
                if (gpad[q]) mx = std::max(mx, ++cnt[g.m_pad % rcl]);
                return mx;
            };
            const int wl = p == 1 ? 16 : 8;  // state-write group width = classes
            const int NW = g.m_pad / wl;
            auto wcost = [&](int w) {
                int cnt[16] = {0};
                int mx = 0;
                for (int t = 0; t < wl; ++t) mx = std::max(mx, ++cnt[sst[w * wl + t] % wl]);
                return mx;
            };
            std::vector<int> qc(NGR), wc(NW);
            long cur = 0;
            for (int q = 0; q < NGR; ++q) cur += (qc[q] = qcost(q));
            for (int w = 0; w < NW; ++w) cur += (wc[w] = wcost(w));
            std::vector<int> occ(g.m_pad, -1);
            for (int i = 0; i < g.m_pad; ++i) occ[sst[i]] = i;
            std::vector<int> best = sst;
            long bestc = cur;
            const int iters = 60000;
            std::vector<int> aff;
            std::vector<int> newc;
            const int nmov = g.m_pad;
            for (int it = 0; it < iters; ++it) {
                const double T = 0.6 * (1.0 - (double)it / iters) + 0.02;
                const int c1 = (int)(rng() % (unsigned)nmov);
                const int s2 = (int)(rng() % (unsigned)g.m_pad);
                const int c2 = occ[s2];
                if (c2 == c1) continue;
                aff = app[c1 < m ? c1 : 0];
                if (c1 >= m) aff.clear();
                if (c2 >= 0 && c2 < m) aff.insert(aff.end(), app[c2].begin(), app[c2].end());
                std::sort(aff.begin(), aff.end());
                aff.erase(std::unique(aff.begin(), aff.end()), aff.end());
                const int w1 = NW ? c1 / wl : -1, w2 = NW && c2 >= 0 && c2 / wl != w1 ? c2 / wl : -1;
                long old = 0;
                for (int q : aff) old += qc[q];
                if (w1 >= 0) old += wc[w1];
                if (w2 >= 0) old += wc[w2];
                const int s1 = sst[c1];
                sst[c1] = s2;
                if (c2 >= 0) sst[c2] = s1;
                newc.resize(aff.size());
                long nw = 0;
                for (size_t t = 0; t < aff.size(); ++t) nw += (newc[t] = qcost(aff[t]));
                const int nw1 = w1 >= 0 ? wcost(w1) : 0, nw2 = w2 >= 0 ? wcost(w2) : 0;
                nw += nw1 + nw2;
                const long d = nw - old;
                const double u = (double)(rng() & 0xFFFFFF) / 16777216.0;
                if (d <= 0 || u < std::exp(-(double)d / T)) {
                    occ[s2] = c1;
                    occ[s1] = c2;
                    for (size_t t = 0; t < aff.size(); ++t) qc[aff[t]] = newc[t];
                    if (w1 >= 0) wc[w1] = nw1;
                    if (w2 >= 0) wc[w2] = nw2;
                    cur += d;
                    if (cur < bestc) { bestc = cur; best = sst; }
                } else {
                    sst[c1] = s1;
                    if (c2 >= 0) sst[c2] = s2;
                }
            }
            sst = best;
        }
        // pad check lanes write zeros into their own slots (min-sum of an empty
        // row never reaches them: their rows hold Big)
        std::vector<uint16_t> ss16(g.m_pad, (uint16_t)g.m_pad);
        for (int i = 0; i < g.m_pad; ++i) ss16[i] = (uint16_t)sst[i];
        g.ms_sslot[p] = G->arena.upload(ss16);
        std::vector<uint32_t> etab((size_t)kDC * g.n_pad);
        for (int gi = 0; gi < NG; ++gi) {
            const int rv = gi / kDC, k = gi % kDC;
            for (int l = 0; l < 64; ++l)
                etab[(size_t)k * g.n_pad + rv * 64 + l] = (uint32_t)dummy[gi] | ((uint32_t)g.m_pad << 16);
        }
        for (int i = 0; i < m; ++i)
            for (int e = rp[i]; e < rp[i + 1]; ++e)
                etab[(size_t)edge_cpos[e] * g.n_pad + slot_of[ci[e]]] =
                    (uint32_t)(i * DRS[p] + pos[e]) | ((uint32_t)sst[i] << 16);
        g.ms_etab[p] = G->arena.upload(etab);
        entry.etab[p] = std::move(etab);
        entry.ss16[p] = std::move(ss16);
    }
    std::lock_guard<std::mutex> lk(cache_mu);
    if (cache.size() >= 16) cache.erase(cache.begin());
    cache.push_back(std::move(entry));
    }
tables_done:
    // column of each slot (pads: a per-lane dummy past n_pad in the kernel's xh)
    std::vector<uint16_t> vsl(g.n_pad);
    for (int s2 = 0; s2 < g.n_pad; ++s2)
        vsl[s2] = (uint16_t)(G->ms_var_of_slot[s2] >= 0 ? G->ms_var_of_slot[s2] : g.n_pad + s2 % 64);
    g.ms_vslot = G->arena.upload(vsl);
    const int W = g.n_pad / 64;
    std::vector<uint64_t> smask((size_t)W * g.m_pad, 0);
    for (int i = 0; i < m; ++i)
        for (int e = rp[i]; e < rp[i + 1]; ++e) {
            const int sl = slot_of[ci[e]];
            smask[(size_t)(sl / 64) * g.m_pad + i] ^= 1ull << (sl % 64);
        }
    g.ms_smask = G->arena.upload(smask);
}

// Iteration 1 of lean min-sum as a table per column, for ms_triage_kernel.
// With every prior L > 0 nothing in the first check pass depends on signs but
// the syndrome: check i sends column j the message (s_i ? -1 : 1) * alpha_1 *
// (L_j == m1_i ? m2_i : m1_i), m1 / m2 the two smallest priors on row i (Big
// where the row has fewer: the kernels' unused row positions), alpha_1 = 1 -
// 2^-1 = 0.5 (exact).  So column j's decision after iteration 1 (posterior
// L_j + sum of the messages <= 0) is a function of its <= 4 checks' syndrome
// bits.  It is evaluated here in the kernels' precision and summation order
// (MsCore::iterate: edges by ascending row, acc += c_k), so the table is the
// kernel's decision bit for bit; bit b = the decision under pattern b (bit k =
// the syndrome bit of edge k's check).
template <typename T>
static std::vector<uint16_t> it1_lut(const qd_graph* G, const std::vector<T>& L, T big) {
    const DevGraph& g = G->dg;
    std::vector<T> m1(g.m, big), m2(g.m, big);
    for (int i = 0; i < g.m; ++i)
        for (int e = G->row_ptr[i]; e < G->row_ptr[i + 1]; ++e) {
            const T av = std::fabs(L[G->col_idx[e]]);  // the med3 chain / top-2 tree of the check pass
            if (av < m1[i]) {
                m2[i] = m1[i];
                m1[i] = av;
            } else if (av < m2[i]) {
                m2[i] = av;
            }
        }
    std::vector<uint16_t> lut(g.n_pad, 0);
    for (int j = 0; j < g.n; ++j) {
        const int t0 = G->col_ptr[j], deg = G->col_ptr[j + 1] - t0;
        T y[kDC];
        for (int k = 0; k < deg; ++k) {
            const int i = G->col_rows[t0 + k];
            y[k] = (L[j] == m1[i] ? m2[i] : m1[i]) * (T)0.5;
        }
        uint32_t bits = 0;
        for (int b = 0; b < (1 << deg); ++b) {
            T acc = L[j];
            for (int k = 0; k < deg; ++k) acc = acc + (((b >> k) & 1) ? -y[k] : y[k]);
            if (acc <= (T)0) bits |= 1u << b;
        }
        lut[j] = (uint16_t)bits;
    }
    return lut;
}

// The precision-independent part: checks of each column, columns of each row.
static void it1_tables(qd_graph* G, bool pos64, const std::vector<double>& L64, bool pos32,
                       const std::vector<float>& L32) {
    DevGraph& g = G->dg;
    g.it1_vchk = nullptr;
    g.it1_cvar = nullptr;
    g.it1_lut[QD_F64] = g.it1_lut[QD_F32] = nullptr;
    if (!g.wave || g.max_cdeg > kDC || g.max_rdeg > kDR || g.m > 0xfffe || g.n > 0xfffe) return;
    std::vector<uint64_t> vchk(g.n_pad, 0), cvar(2 * (size_t)g.m_pad, 0);
    for (int j = 0; j < g.n_pad; ++j) {
        uint64_t w = 0;
        for (int k = 0; k < kDC; ++k) {
            const int t = j < g.n ? G->col_ptr[j] + k : 0;
            const int i = (j < g.n && t < G->col_ptr[j + 1]) ? G->col_rows[t] : g.m;
            w |= (uint64_t)i << (16 * k);
        }
        vchk[j] = w;
    }
    for (int i = 0; i < g.m_pad; ++i)
        for (int t = 0; t < kDR; ++t) {
            const int e = i < g.m ? G->row_ptr[i] + t : 0;
            const int j = (i < g.m && e < G->row_ptr[i + 1]) ? G->col_idx[e] : g.n;
            cvar[2 * (size_t)i + t / 4] |= (uint64_t)j << (16 * (t % 4));
        }
    g.it1_vchk = G->prior_arena.upload(vchk);
    g.it1_cvar = G->prior_arena.upload(cvar);
    if (pos64) g.it1_lut[QD_F64] = G->prior_arena.upload(it1_lut<double>(G, L64, 1e308));
    if (pos32) g.it1_lut[QD_F32] = G->prior_arena.upload(it1_lut<float>(G, L32, 1e30f));
}

// Row positions of the edges for the LDS-resident min-sum kernel
// (bp_ms_lds_kernel): edge e of row i sits at LDS element i * kMlDRS + pos[e].
// The check pass is independent of the order inside a row, so positions are
// free; the variable pass scatters with one ds_write_b32 per (variable round
// r, wave w, edge k): 2 x 32 lanes, bank = element % 32, cost max(4, L0 + L1)
// with L_h the worst bank load of half h (pad lanes write element m * kMlDRS +
// lane).  A seeded hill climb over position swaps inside rows lowers the sum
// over instructions (tie-break: sum of squared loads).  Cached per graph.
std::vector<int> ml_positions(int m, int n, const std::vector<int32_t>& rp, const std::vector<int32_t>& ci,
                              const std::vector<int>& edge_cpos) {
    struct Entry {
        std::vector<int32_t> rp, ci;
        std::vector<int> pos;
    };
    static std::mutex mu;
    static std::vector<Entry> cache;
    {
        std::lock_guard<std::mutex> lk(mu);
        for (const auto& c : cache)
            if (c.rp == rp && c.ci == ci) return c.pos;
    }
    const int E = rp[m];
    constexpr int NT = 1024, NB = 32;
    std::vector<int> pos(E), row(E), grp(E), half(E);
    const int rounds = (n + NT - 1) / NT;
    const int NG = rounds * (NT / 64) * kMlDC;
    std::vector<int> load((size_t)NG * 2 * NB, 0);
    for (int i = 0; i < m; ++i)
        for (int e = rp[i]; e < rp[i + 1]; ++e) {
            const int j = ci[e];
            pos[e] = e - rp[i];
            row[e] = i;
            grp[e] = ((j / NT) * (NT / 64) + (j % NT) / 64) * kMlDC + edge_cpos[e];
            half[e] = (j % 64) / 32;
        }
    auto bank = [&](int e) { return (row[e] * kMlDRS + pos[e]) % NB; };
    for (int e = 0; e < E; ++e) load[((size_t)grp[e] * 2 + half[e]) * NB + bank(e)]++;
    // pad lanes: variables without a k-th edge, slots past n
    std::vector<int> cdeg(n, 0);
    for (int e = 0; e < E; ++e) cdeg[ci[e]]++;
    for (int s = 0; s < rounds * NT; ++s)
        for (int k = 0; k < kMlDC; ++k)
            if (s >= n || k >= cdeg[s]) {
                const int gi = ((s / NT) * (NT / 64) + (s % NT) / 64) * kMlDC + k;
                load[((size_t)gi * 2 + (s % 64) / 32) * NB + (m * kMlDRS + s % 64) % NB]++;
            }
    auto gcost = [&](int gi) {
        int sum = 0, sq = 0;
        for (int h = 0; h < 2; ++h) {
            int mx = 0;
            for (int b = 0; b < NB; ++b) {
                const int v = load[((size_t)gi * 2 + h) * NB + b];
                mx = std::max(mx, v);
                sq += v * v;
            }
            sum += mx;
        }
        return (long)std::max(4, sum) * 100000 + sq;
    };
    std::mt19937 rng(2024);
    std::vector<int> at(kMlDRS);
    for (long it = 0; it < 40L * E; ++it) {
        const int i = (int)(rng() % (unsigned)m);
        const int deg = rp[i + 1] - rp[i];
        if (deg < 2) continue;
        const int e1 = rp[i] + (int)(rng() % (unsigned)deg);
        const int p2 = (int)(rng() % (unsigned)deg);
        int e2 = -1;
        for (int e = rp[i]; e < rp[i + 1]; ++e)
            if (pos[e] == p2) e2 = e;
        if (e2 == e1 || e2 < 0) continue;
        const int g1 = grp[e1], g2 = grp[e2];
        const long before = gcost(g1) + (g2 != g1 ? gcost(g2) : 0);
        auto move = [&](int e, int np) {
            load[((size_t)grp[e] * 2 + half[e]) * NB + bank(e)]--;
            pos[e] = np;
            load[((size_t)grp[e] * 2 + half[e]) * NB + bank(e)]++;
        };
        const int p1 = pos[e1];
        move(e1, p2);
        move(e2, p1);
        const long after = gcost(g1) + (g2 != g1 ? gcost(g2) : 0);
        if (after > before) {
            move(e2, p2);
            move(e1, p1);
        }
    }
    std::lock_guard<std::mutex> lk(mu);
    if (cache.size() >= 8) cache.erase(cache.begin());
    cache.push_back(Entry{rp, ci, pos});
    return pos;
}

void build_tables(qd_graph* G, int m, int n) {
    DevGraph& g = G->dg;
    g.m = m;
    g.n = n;
    const auto& rp = G->row_ptr;
    const auto& ci = G->col_idx;
    const int E = rp[m];
    // CSC with ascending rows; position of each edge inside its column list
    G->col_ptr.assign(n + 1, 0);
    for (int e = 0; e < E; ++e) G->col_ptr[ci[e] + 1]++;
    for (int j = 0; j < n; ++j) G->col_ptr[j + 1] += G->col_ptr[j];
    G->col_rows.assign(std::max(E, 1), 0);
    std::vector<int> fill(G->col_ptr.begin(), G->col_ptr.end() - 1);
    std::vector<int> edge_cpos(std::max(E, 1), 0);
    for (int i = 0; i < m; ++i)
        for (int e = rp[i]; e < rp[i + 1]; ++e) {
            const int j = ci[e];
            edge_cpos[e] = fill[j] - G->col_ptr[j];
            G->col_rows[fill[j]++] = i;
        }
    g.max_rdeg = 0;
    for (int i = 0; i < m; ++i) g.max_rdeg = std::max(g.max_rdeg, rp[i + 1] - rp[i]);
    g.max_cdeg = 0;
    for (int j = 0; j < n; ++j) g.max_cdeg = std::max(g.max_cdeg, G->col_ptr[j + 1] - G->col_ptr[j]);
    g.E = E;
    // CSC edge lists for the workgroup kernels
    std::vector<int32_t> col_edge(std::max(E, 1), 0);
    {
        std::vector<int> f2(G->col_ptr.begin(), G->col_ptr.end() - 1);
        for (int i = 0; i < m; ++i)
            for (int e = rp[i]; e < rp[i + 1]; ++e) col_edge[f2[ci[e]]++] = e;
    }
    std::vector<int32_t> edge_csc(std::max(E, 1), 0);
    for (int e = 0; e < E; ++e) edge_csc[e] = G->col_ptr[ci[e]] + edge_cpos[e];
    // edge arrays padded by kEdgePad zeros (unguarded whole-row index loads)
    col_edge.resize((size_t)E + kEdgePad, 0);
    edge_csc.resize((size_t)E + kEdgePad, 0);
    std::vector<int32_t> ci_pad(G->col_idx);
    ci_pad.resize((size_t)E + kEdgePad, 0);
    g.col_ptr = G->arena.upload(G->col_ptr);
    g.col_edge = G->arena.upload(col_edge);
    g.edge_csc = G->arena.upload(edge_csc);
    g.row_ptr = G->arena.upload(G->row_ptr);
    g.col_idx = G->arena.upload(ci_pad);
    int rc = 0, rv = 0, drc = 0;
    g.wave = (g.max_rdeg <= kDR && g.max_cdeg <= kDC && pick_wave_shape(m, n, g.max_rdeg, &rc, &rv, &drc)) ? 1 : 0;
    if (!g.wave) {  // workgroup kernels: plain 64-padding, no wave tables
        g.m_pad = (m + 63) / 64 * 64;
        g.n_pad = (n + 63) / 64 * 64;
        g.shape_drc = 0;
        // LDS-resident min-sum kernel (bp_ms_lds_kernel): edge k of column j (CSC
        // order) lives at LDS element row * kMlDRS + position in the CSR row
        g.ml_etab = nullptr;
        g.m64_etab = nullptr;
        g.m64_check = nullptr;
        g.m64_d3r = 0;
        if (g.max_rdeg <= kMlDRS && g.max_cdeg <= kMlDC && (size_t)m * kMlDRS + 64 < 0xffff) {
            const std::vector<int> pos = ml_positions(m, n, rp, ci, edge_cpos);
            std::vector<uint16_t> et((size_t)kMlDC * n, 0xffff);
            for (int i = 0; i < m; ++i)
                for (int e = rp[i]; e < rp[i + 1]; ++e)
                    et[(size_t)edge_cpos[e] * n + ci[e]] = (uint16_t)(i * kMlDRS + pos[e]);
            g.ml_etab = G->arena.upload(et);
            m64_layout(G, m, n, rp, ci, edge_cpos);
        }
        return;
    }
    g.m_pad = rc * 64;
    g.n_pad = rv * 64;
    g.shape_drc = drc;
    std::vector<uint8_t> r_deg(g.m_pad, 0), c_deg(g.n_pad, 0);
    // Pad edges (k >= degree, or padding rows/columns) point at per-lane dummies:
    // column n_pad + lane (a zero byte of xh) and message slot <array end> + lane.
    std::vector<uint16_t> r_col((size_t)kDR * g.m_pad);
    for (size_t t = 0; t < r_col.size(); ++t) r_col[t] = (uint16_t)(g.n_pad + (t % g.m_pad) % 64);
    std::vector<uint16_t> r_cslot[2], c_rslot[2];
    const int DRS[2] = {drs<double>(), drs<float>()};
    const int DCS[2] = {dcs<double>(), dcs<float>()};
    for (int p = 0; p < 2; ++p) {
        if ((size_t)g.m_pad * DRS[p] + 64 > 65535 || (size_t)g.n_pad * DCS[p] + 64 > 65535)
            throw Fail(-21, "graph too large for 16-bit LDS slots");
        r_cslot[p].resize((size_t)kDR * g.m_pad);
        for (size_t t = 0; t < r_cslot[p].size(); ++t)
            r_cslot[p][t] = (uint16_t)(g.n_pad * DCS[p] + (t % g.m_pad) % 64);
        c_rslot[p].resize((size_t)kDC * g.n_pad);
        for (size_t t = 0; t < c_rslot[p].size(); ++t)
            c_rslot[p][t] = (uint16_t)(g.m_pad * DRS[p] + (t % g.n_pad) % 64);
    }
    for (int i = 0; i < m; ++i) {
        r_deg[i] = (uint8_t)(rp[i + 1] - rp[i]);
        for (int e = rp[i], k = 0; e < rp[i + 1]; ++e, ++k) {
            const int j = ci[e];
            r_col[(size_t)k * g.m_pad + i] = (uint16_t)j;
            for (int p = 0; p < 2; ++p) {
                r_cslot[p][(size_t)k * g.m_pad + i] = (uint16_t)(j * DCS[p] + edge_cpos[e]);
            }
        }
    }
    for (int j = 0; j < n; ++j) {
        c_deg[j] = (uint8_t)(G->col_ptr[j + 1] - G->col_ptr[j]);
        for (int t = G->col_ptr[j], k = 0; t < G->col_ptr[j + 1]; ++t, ++k) {
            const int i = G->col_rows[t];
            // position of this edge inside row i
            int kr = 0;
            for (int e = rp[i]; e < rp[i + 1]; ++e, ++kr)
                if (ci[e] == j) break;
            for (int p = 0; p < 2; ++p) c_rslot[p][(size_t)k * g.n_pad + j] = (uint16_t)(i * DRS[p] + kr);
        }
    }
    g.r_deg = G->arena.upload(r_deg);
    g.r_col = G->arena.upload(r_col);
    g.c_deg = G->arena.upload(c_deg);
    for (int p = 0; p < 2; ++p) {
        g.slots[p].r_cslot = G->arena.upload(r_cslot[p]);
        g.slots[p].c_rslot = G->arena.upload(c_rslot[p]);
    }
    ms_layout(G, m, n, edge_cpos);
}

// Attach the SSF queue scratch (capacity >= B shots) to the launch arguments.
// Words of a compact-list entry (wave graphs; qdec_bp_ms.h CmpEntry): shot,
// syndrome words, readout logical-parity words.
size_t cmp_entry_bytes(const DevGraph& g) { return 8 * (1 + (size_t)g.m_pad / 64 + 4); }

// Byte layout of the queue scratch for a capacity of `cap` shots: the queue
// count (256 B), idx[cap] u64, then the byte-format x[cap][n] | r[cap][m] region
// (the packed format of the wave kernels reuses it for [cap][1 + 2 n_pad/64 +
// m_pad/64] u64 entries), and for wave graphs the compact shot list:
// kCmpSegs counters on their own 128-B lines (the triage's u64 atomics need
// natural alignment, so the region starts on a 256-B boundary), then the
// segments of cmp_seg_cap(cap) entries.
struct QueueLayout {
    size_t bytes, idx, x, r, cmp_count, cmp;
    int64_t cmp_cap;
};
QueueLayout queue_layout(const DevGraph& g, int64_t cap) {
    QueueLayout L{};
    const size_t packed = 8 * (1 + 2 * (size_t)g.n_pad / 64 + (size_t)g.m_pad / 64);
    const size_t xr = std::max((size_t)g.n + (size_t)g.m, packed);
    L.idx = 256;
    L.x = 256 + (size_t)cap * 8;
    L.r = L.x + (size_t)cap * g.n;
    const size_t cbase = 256 + ((size_t)cap * (8 + xr) + 255) / 256 * 256 + 256;
    L.cmp_count = g.wave ? cbase : 0;
    L.cmp = g.wave ? cbase + (size_t)kCmpLists * kCmpSegs * 128 : 0;
    L.cmp_cap = g.wave ? cmp_seg_cap(cap) : 0;
    L.bytes = cbase +
              (g.wave ? (size_t)kCmpLists * kCmpSegs * (128 + (size_t)L.cmp_cap * cmp_entry_bytes(g)) : 0) + 256;
    return L;
}

// Attach the SSF queue scratch (capacity >= B shots) and, for wave graphs, the
// compact shot list of lean launches to the launch arguments.
void attach_queue(qd_graph* G, DecodeArgs& a, int method, int precision) {
    const DevGraph& g = G->dg;
    const bool cmp = g.wave && method == QD_MIN_SUM && !G->ms_var_of_slot.empty();
    if (a.B <= 0 || (!a.ssf && !cmp && !lds_kernel_applies(G->dg, method, precision, a)))
        return;
    if (a.B > G->q_cap) {
        ws_drain(G);  // launches still in flight may use the old queue
        if (G->qws) hip_check(hipFree(G->qws), "hipFree queue");
        G->qws = nullptr;
        G->q_cap = 0;
        hip_check(hipMalloc(&G->qws, queue_layout(g, a.B).bytes), "hipMalloc queue");
        G->q_cap = a.B;
    }
    const QueueLayout L = queue_layout(g, G->q_cap);
    auto* base = static_cast<uint8_t*>(G->qws);
    a.q_count = reinterpret_cast<int32_t*>(base);
    a.q_idx = reinterpret_cast<int64_t*>(base + L.idx);
    a.q_x = base + L.x;
    a.q_r = base + L.r;
    a.q_w = reinterpret_cast<uint64_t*>(a.q_x);
    if (g.wave) {
        a.cmp_count = reinterpret_cast<unsigned long long*>(base + L.cmp_count);
        a.cmp = reinterpret_cast<uint64_t*>(base + L.cmp);
        a.cmp_cap = L.cmp_cap;
        // double-buffered counters (zeroed once here, then by each triage for
        // the next decode): no memset launch per decode
        const size_t set = (size_t)kCmpLists * kCmpSegs * 128;
        if (!G->cmpc) {
            hip_check(hipMalloc(&G->cmpc, 2 * set), "hipMalloc list counters");
            hip_check(hipMemset(G->cmpc, 0, 2 * set), "hipMemset list counters");
            G->cmp_par = 0;
        }
        auto* c = static_cast<uint8_t*>(G->cmpc);
        a.cmp_count = reinterpret_cast<unsigned long long*>(c + (size_t)G->cmp_par * set);
        a.cmp_count_next = reinterpret_cast<unsigned long long*>(c + (size_t)(G->cmp_par ^ 1) * set);
    }
}

// The second SSF queue of split-SSF decodes (the SSF region of the layout:
// count, index, entries; the compact lists stay in the first buffer, which only
// the BP stage uses)
void attach_queue2(qd_graph* G, DecodeArgs& a) {
    if (!a.q_count) return;  // no queue for this launch
    const DevGraph& g = G->dg;
    if (G->q2_cap < G->q_cap) {
        ws_drain(G);
        if (G->qws2) hip_check(hipFree(G->qws2), "hipFree queue 2");
        G->qws2 = nullptr;
        G->q2_cap = 0;
        const QueueLayout L = queue_layout(g, G->q_cap);
        hip_check(hipMalloc(&G->qws2, g.wave ? L.cmp_count : L.bytes), "hipMalloc queue 2");
        G->q2_cap = G->q_cap;
    }
    const QueueLayout L = queue_layout(g, G->q2_cap);
    auto* base = static_cast<uint8_t*>(G->qws2);
    a.q_count = reinterpret_cast<int32_t*>(base);
    a.q_idx = reinterpret_cast<int64_t*>(base + L.idx);
    a.q_x = base + L.x;
    a.q_r = base + L.r;
    a.q_w = reinterpret_cast<uint64_t*>(a.q_x);
}

// after a launch: a two-pass decode (its triage ran) used one counter set and
// zeroed the other, so the next one takes the other set
void flip_counters(qd_graph* G, const DecodeArgs& a) {
    if (a.cmp_count_next && !G->last_pre.empty()) G->cmp_par ^= 1;
}

void* message_scratch(qd_graph* G, int method, int precision, const DecodeArgs& a, size_t* bytes) {
    size_t need = block_scratch_bytes(G->dg, method, precision, G->num_cus, a);
    *bytes = need;
    if (need == 0) return nullptr;
    const size_t floor = block_scratch_floor(G->dg, method, precision, G->num_cus, a);
    // capped after an allocation failure: a request at or above the size that
    // failed keeps the reduced scratch (the launch sizes its grid from the bytes
    // it gets) instead of draining and failing the same allocation every call
    // (every 64th such call retries the full size: the memory may be free again)
    if (need > G->mws_bytes && G->mws && G->mws_failed && need >= G->mws_failed && G->mws_bytes >= floor &&
        ++G->mws_capped_calls % 64 != 0) {
        *bytes = G->mws_bytes;
        return G->mws;
    }
    const size_t want = need;
    if (need > G->mws_bytes) {
        ws_drain(G);  // launches still in flight may use the old scratch
        if (G->mws) hip_check(hipFree(G->mws), "hipFree scratch");
        G->mws = nullptr;
        G->mws_bytes = 0;
        // on an allocation failure, halve the slot groups in flight down to one
        // (the launch sizes its grid from the bytes it gets; results do not change)
        for (;;) {
            const hipError_t e = hipMalloc(&G->mws, need);
            if (e == hipSuccess) {
                if (need == want) G->mws_failed = 0;  // the full size fits again: no longer capped
                break;
            }
            (void)hipGetLastError();  // clear the sticky error before any launch checks it
            G->mws = nullptr;
            if (e != hipErrorOutOfMemory || need <= floor)
                hip_check(e, "hipMalloc message scratch");
            G->mws_failed = G->mws_failed ? std::min(G->mws_failed, need) : need;
            need = std::max(floor, floor + (need - floor) / 2);
        }
        G->mws_bytes = need;
        *bytes = need;
    }
    return G->mws;
}

// byte rows for a packed decode that does not take the two-pass path (every
// input the call passes: syn [B][m], base and readout [B][n_data])
void attach_unpack(qd_graph* G, DecodeArgs& a) {
    if (!a.in_packed) return;
    const size_t need = (size_t)a.B * ((size_t)G->dg.m + 2 * (size_t)G->dg.n_data) + 256;
    if (need > G->ubuf_bytes) {
        ws_drain(G);  // launches in flight may still read the old buffer
        if (G->ubuf) hip_check(hipFree(G->ubuf), "hipFree unpack buffer");
        G->ubuf = nullptr;
        G->ubuf_bytes = 0;
        hip_check(hipMalloc(&G->ubuf, need), "hipMalloc unpack buffer");
        G->ubuf_bytes = need;
    }
    a.unpack_buf = static_cast<uint8_t*>(G->ubuf);
}

void note_kernels(qd_graph* G) {
    const LaunchNames& n = last_launch_names();
    G->last_bp = n.bp ? n.bp : "";
    G->last_ssf = n.ssf ? n.ssf : "";
    G->last_pre = n.pre ? n.pre : "";
}

void attach_timing(qd_graph* G, DecodeArgs& a) {
    a.ev = nullptr;
    if (G->t_cap > 0 && G->t_count < G->t_cap) a.ev = &G->tev[(size_t)kTimingEvents * G->t_count++];
}

// after a timed launch: the compact list's length (the triage's segment
// counters, one per 128-B line) into the call's pinned slot, on the BP stream,
// with the call's event [4] behind the copy (read_timing_detail waits on it).
// A split SSF stream waits for that event too, so the workspace chain, which
// continues on the SSF stream, covers the copy: the next decode's triage never
// resets the counters while the copy still reads them.
void note_listed(qd_graph* G, const DecodeArgs& a, hipStream_t s, hipStream_t chain) {
    if (!a.ev || !G->t_listed) return;
    const size_t slot = (size_t)(a.ev - G->tev.data()) / kTimingEvents;
    const bool cmp = !G->last_pre.empty() && a.cmp_count;
    G->t_cmp[slot] = cmp ? 1 : 0;
    if (cmp)
        hip_check(hipMemcpy2DAsync(G->t_listed + slot * kCmpLists * kCmpSegs, 8, a.cmp_count, 128, 8,
                                   kCmpLists * kCmpSegs,
                                   hipMemcpyDeviceToHost, s),
                  "hipMemcpy2DAsync list counters");
    hip_check(hipEventRecord(a.ev[4], s), "hipEventRecord");
    if (chain != s) hip_check(hipStreamWaitEvent(chain, a.ev[4], 0), "hipStreamWaitEvent");
}

void free_timing(qd_graph* G) {
    ws_drain(G);  // list-counter copies into t_listed may still be in flight
    for (hipEvent_t e : G->tev) (void)hipEventDestroy(e);
    G->tev.clear();
    if (G->t_listed) (void)hipHostFree(G->t_listed);
    G->t_listed = nullptr;
    G->t_cmp.clear();
    G->t_cap = G->t_count = 0;
}

void check_graph(const qd_graph* g) {
    if (!g) throw Fail(-1, "null graph handle");
}

void check_params(const qd_graph* g, const qd_params* p) {
    if (g->host_only) throw Fail(-16, "host-only graph (qd_graph_create_host): no device to decode on");
    if (!p) throw Fail(-2, "null params");
    if (p->method != QD_MIN_SUM && p->method != QD_PRODUCT_SUM) throw Fail(-3, "unknown BP method");
    if (p->precision != QD_F32 && p->precision != QD_F64) throw Fail(-4, "unknown precision");
    if (!g->has_priors) throw Fail(-5, "priors not set (qd_graph_set_priors)");
    if (p->ssf && g->dg.n_gen <= 0) throw Fail(-6, "SSF requested but the graph has no flip sets");
}

DecodeArgs make_args(const qd_graph* g, const qd_params* p, int64_t B, const uint8_t* syn, const uint8_t* base,
                     const uint8_t* readout, uint8_t* x_out, uint8_t* corr_out, void* llr_out, int32_t* iters,
                     uint8_t* status, int32_t* ssf_steps, uint8_t* fail) {
    DecodeArgs a{};
    a.B = B;
    a.max_iter = p->max_iter > 0 ? p->max_iter : g->dg.n;
    a.ssf = p->ssf ? 1 : 0;
    a.ssf_max_steps = p->ssf_max_steps;
    a.syn_flags = p->syn_flags & 3;
    a.in_packed = (p->syn_flags & QD_INPUT_PACKED) ? 1 : 0;
    if (a.in_packed && (((uintptr_t)syn | (uintptr_t)base | (uintptr_t)readout) & 7))
        throw Fail(-9, "QD_INPUT_PACKED rows must be 8-B aligned");
    a.ms_scaling = p->ms_scaling;
    a.syn = syn;
    a.base = base;
    a.readout = readout;
    a.x_out = x_out;
    a.corr_out = corr_out;
    a.llr_out = llr_out;
    a.iters = iters;
    a.status = status;
    a.ssf_steps = ssf_steps;
    a.fail = fail;
    if (!syn && !(a.syn_flags && (base || readout))) throw Fail(-7, "no syndrome source");
    if (!g->ctl) hip_check(hipMalloc(&const_cast<qd_graph*>(g)->ctl, kCtlBytes), "hipMalloc control block");
    a.wave_ctr = static_cast<unsigned long long*>(g->ctl);
    a.ssf_nosplit = g->dg.opt_ssf == kSsfScanNoSplit ? 1 : 0;
    return a;
}

}  // namespace

extern "C" {

int qd_abi_version(void) { return QDEC_ABI_VERSION; }

const char* qd_last_error(void) { return g_last_error.c_str(); }

int qd_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int qd_graph_create(int32_t m, int32_t n, const int32_t* row_ptr, const int32_t* col_idx, int32_t n_data,
                    int32_t fold_blocks, int32_t device, qd_graph** out) {
    return guarded([&] {
        if (!out) throw Fail(-1, "null output handle");
        *out = nullptr;
        if (m <= 0 || n <= 0 || !row_ptr || !col_idx) throw Fail(-10, "invalid graph shape or null arrays");
        if (n_data <= 0 || fold_blocks <= 0 || (int64_t)n_data * fold_blocks > n)
            throw Fail(-11, "invalid fold (n_data * fold_blocks must be <= n)");
        if (row_ptr[0] != 0) throw Fail(-12, "row_ptr[0] must be 0");
        for (int i = 0; i < m; ++i) {
            if (row_ptr[i + 1] < row_ptr[i]) throw Fail(-12, "row_ptr not monotone");
            for (int e = row_ptr[i]; e < row_ptr[i + 1]; ++e) {
                if (col_idx[e] < 0 || col_idx[e] >= n) throw Fail(-13, "column index out of range");
                if (e > row_ptr[i] && col_idx[e] <= col_idx[e - 1])
                    throw Fail(-14, "column indices must be strictly ascending within a row");
            }
        }
        int ndev = 0;
        hip_check(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
        if (device < 0 || device >= ndev) throw Fail(-15, "device ordinal out of range");
        auto* G = new qd_graph();
        try {
            G->device = device;
            set_device(G);
            hipDeviceProp_t prop;
            hip_check(hipGetDeviceProperties(&prop, device), "hipGetDeviceProperties");
            G->num_cus = prop.multiProcessorCount;
            hip_check(hipStreamCreateWithFlags(&G->stream, hipStreamNonBlocking), "hipStreamCreate");
            G->row_ptr.assign(row_ptr, row_ptr + m + 1);
            G->col_idx.assign(col_idx, col_idx + row_ptr[m]);
            G->dg.n_data = n_data;
            G->dg.fold_blocks = fold_blocks;
            build_tables(G, m, n);
            G->dg.lz_words = (n_data + 63) / 64;
            G->dg.k = 0;
            G->dg.lz = nullptr;
            G->dg.lz_ptr = G->dg.lz_idx = nullptr;
            G->dg.lz_sparse = 0;
            G->dg.lz_t = nullptr;
            G->dg.lz_tw = 0;
            G->dg.n_gen = 0;
            G->dg.g_inv = nullptr;
            G->dg.g_invd = G->dg.g_invl = 0;
            default_options(G->dg);
        } catch (...) {
            G->arena.release();
            if (G->stream) (void)hipStreamDestroy(G->stream);
            delete G;
            throw;
        }
        *out = G;
    });
}

int qd_graph_create_host(int32_t m, int32_t n, const int32_t* row_ptr, const int32_t* col_idx, int32_t n_data,
                         int32_t fold_blocks, qd_graph** out) {
    return guarded([&] {
        if (!out) throw Fail(-1, "null output handle");
        *out = nullptr;
        if (m <= 0 || n <= 0 || !row_ptr || !col_idx) throw Fail(-10, "invalid graph shape or null arrays");
        if (n_data <= 0 || fold_blocks <= 0 || (int64_t)n_data * fold_blocks > n)
            throw Fail(-11, "invalid fold (n_data * fold_blocks must be <= n)");
        if (row_ptr[0] != 0) throw Fail(-12, "row_ptr[0] must be 0");
        for (int i = 0; i < m; ++i) {
            if (row_ptr[i + 1] < row_ptr[i]) throw Fail(-12, "row_ptr not monotone");
            for (int e = row_ptr[i]; e < row_ptr[i + 1]; ++e) {
                if (col_idx[e] < 0 || col_idx[e] >= n) throw Fail(-13, "column index out of range");
                if (e > row_ptr[i] && col_idx[e] <= col_idx[e - 1])
                    throw Fail(-14, "column indices must be strictly ascending within a row");
            }
        }
        auto* G = new qd_graph();
        G->host_only = true;
        for (DevArena* a : {&G->arena, &G->flip_arena, &G->lz_arena, &G->prior_arena}) a->host = true;
        G->num_cus = 256;
        try {
            G->row_ptr.assign(row_ptr, row_ptr + m + 1);
            G->col_idx.assign(col_idx, col_idx + row_ptr[m]);
            G->dg.n_data = n_data;
            G->dg.fold_blocks = fold_blocks;
            build_tables(G, m, n);
            G->dg.lz_words = (n_data + 63) / 64;
            G->dg.k = 0;
            G->dg.lz = nullptr;
            G->dg.lz_ptr = G->dg.lz_idx = nullptr;
            G->dg.lz_sparse = 0;
            G->dg.lz_t = nullptr;
            G->dg.lz_tw = 0;
            G->dg.n_gen = 0;
            G->dg.g_inv = nullptr;
            G->dg.g_invd = G->dg.g_invl = 0;
            default_options(G->dg);
        } catch (...) {
            delete G;
            throw;
        }
        *out = G;
    });
}

int qd_graph_table_digest(const qd_graph* G, uint64_t* digest, int64_t* bytes) {
    return guarded([&] {
        check_graph(G);
        if (!G->host_only) throw Fail(-16, "table digests are kept for host-only graphs (qd_graph_create_host)");
        uint64_t h = 1469598103934665603ull;  // FNV-1a over every table, in upload order
        int64_t total = 0;
        for (const DevArena* a : {&G->arena, &G->flip_arena, &G->lz_arena, &G->prior_arena})
            for (const auto& v : a->kept) {
                for (uint8_t b : v) h = (h ^ b) * 1099511628211ull;
                total += (int64_t)v.size();
            }
        if (digest) *digest = h;
        if (bytes) *bytes = total;
    });
}

static HgpPlan* hgp_plan_of(qd_graph* G) {
    if (!G->hgp_tried) {
        G->hgp = hgp_plan_create(G->dg.m, G->dg.n, G->row_ptr, G->col_idx);
        G->hgp_tried = true;
    }
    return G->hgp;
}

int qd_graph_hgp_set_slots(qd_graph* G, int32_t slots) {
    return guarded([&] {
        check_graph(G);
        if (slots < 0 || slots > 64) throw Fail(-95, "slots out of range");
        if (!G->host_only) set_device(G);
        if (G->stream) hip_check(hipStreamSynchronize(G->stream), "hipStreamSynchronize");
        ws_drain(G);  // an HGP launch on another stream may still use the plan's module
        HgpPlan* P = hgp_plan_create(G->dg.m, G->dg.n, G->row_ptr, G->col_idx, slots);
        if (!P && slots > 0 && hgp_plan_of(G))  // a hypergraph product, but no feasible plan with `slots`
            throw Fail(-95, "no feasible HGP plan with this many slots per workgroup");
        hgp_plan_destroy(G->hgp);
        G->hgp = P;
        G->hgp_tried = true;
    });
}

int qd_graph_hgp_info(qd_graph* G, int32_t* out8) {
    int rc = 0;
    const int e = guarded([&] {
        check_graph(G);
        HgpPlan* P = hgp_plan_of(G);
        rc = P ? 1 : 0;
        if (P && out8) hgp_plan_info(P, out8);
    });
    return e ? e : rc;
}

int64_t qd_graph_hgp_source(qd_graph* G, char* buf, int64_t cap) {
    int64_t len = 0;
    const int e = guarded([&] {
        check_graph(G);
        HgpPlan* P = hgp_plan_of(G);
        if (!P) throw Fail(-90, "not a hypergraph-product check matrix");
        const std::string& s = hgp_plan_source(P);
        len = (int64_t)s.size();
        if (buf && cap > 0) {
            const size_t k = std::min<size_t>(s.size(), (size_t)cap - 1);
            std::memcpy(buf, s.data(), k);
            buf[k] = 0;
        }
    });
    return e ? e : len;
}

#ifdef QDEC_DEV_HOOKS
// development build only (python -m exp_ldpc_amd.build --tag dev -DQDEC_DEV_HOOKS):
// compile an edited kernel source at run time (tools/gpu/hgp_debug.py)
int qd_graph_hgp_replace_source(qd_graph* G, const char* src) {
    return guarded([&] {
        check_graph(G);
        HgpPlan* P = hgp_plan_of(G);
        if (!P || !src) throw Fail(-90, "not a hypergraph-product check matrix");
        if (G->stream) hip_check(hipStreamSynchronize(G->stream), "hipStreamSynchronize");
        hgp_plan_replace_source(P, src);
    });
}
#endif

int qd_graph_hgp_compile(qd_graph* G) {
    return guarded([&] {
        check_graph(G);
        HgpPlan* P = hgp_plan_of(G);
        if (!P) throw Fail(-90, "not a hypergraph-product check matrix");
        std::string log;
        if (hgp_plan_compile(P, hgp_target_arch(G->host_only ? -1 : G->device).c_str(), &log) != 0)
            throw Fail(-91, "HGP kernel compile failed: " + log);
    });
}

int qd_graph_hgp_decode_bp(qd_graph* G, int64_t B, const uint8_t* syn, uint8_t* x_out, int32_t* iters,
                           uint8_t* status, int32_t max_iter, double ms_scaling, void* stream) {
    return guarded([&] {
        check_graph(G);
        if (G->host_only) throw Fail(-2, "host-only graph handle");
        set_device(G);
        HgpPlan* P = hgp_plan_of(G);
        if (!P) throw Fail(-90, "not a hypergraph-product check matrix");
        if (!G->has_priors) throw Fail(-51, "priors not set");
        if (B < 0 || (B > 0 && !syn) || max_iter < 1) throw Fail(-92, "invalid HGP decode arguments");
        if (hgp_plan_load(P, G->num_cus, hgp_target_arch(G->device).c_str()) != 0)
            throw Fail(-93, "HGP kernel load failed");
        if (!G->ctl) hip_check(hipMalloc(&G->ctl, kCtlBytes), "hipMalloc control block");
        if (B == 0) return;
        HgpBpArgs a{};
        a.syn = syn;
        a.prior = static_cast<const double*>(G->dg.prior[QD_MIN_SUM][QD_F64]);
        a.x_out = x_out;
        a.iters = iters;
        a.status = status;
        // its own shot counter on its own 128-B line (words 0 / 1 are the BP and
        // SSF kernels' counters), and inside the workspace chain like every decode
        a.counter = static_cast<unsigned long long*>(G->ctl) + 16;
        a.B = B;
        a.max_iter = max_iter;
        a.ms_scaling = ms_scaling;
        hipStream_t st = stream ? static_cast<hipStream_t>(stream) : G->stream;
        ws_acquire(G, st);
        if (hgp_launch_bp(P, a, st) != 0) throw Fail(-94, "HGP kernel launch failed");
        hip_check(hipGetLastError(), "HGP kernel");
        ws_release(G, st);
    });
}

int qd_graph_destroy(qd_graph* g) {
    return guarded([&] {
        if (!g) return;
        if (g->host_only) {
            for (DevArena* a : {&g->arena, &g->flip_arena, &g->lz_arena, &g->prior_arena}) a->release();
            hgp_plan_destroy(g->hgp);
            delete g;
            return;
        }
        (void)hipSetDevice(g->device);
        if (g->stream) (void)hipStreamSynchronize(g->stream);
        if (g->ws_ev_live) (void)hipEventSynchronize(g->ws_ev);
        for (int q = 0; q < 2; ++q)
            if (g->ssf_done[q]) {
                if (g->ssf_done_live[q]) (void)hipEventSynchronize(g->ssf_done[q]);
                (void)hipEventDestroy(g->ssf_done[q]);
                g->ssf_done[q] = nullptr;
                g->ssf_done_live[q] = false;
            }
        if (g->qws2) (void)hipFree(g->qws2);
        if (g->ws_ev) (void)hipEventDestroy(g->ws_ev);
        g->ws_ev = nullptr;
        g->ws_ev_live = false;  // drained above (free_timing's drain is a no-op)
        if (g->ssf_ev) (void)hipEventDestroy(g->ssf_ev);
        g->arena.release();
        g->flip_arena.release();
        g->lz_arena.release();
        g->prior_arena.release();
        if (g->ws) (void)hipFree(g->ws);
        if (g->qws) (void)hipFree(g->qws);
        if (g->mws) (void)hipFree(g->mws);
        if (g->ubuf) (void)hipFree(g->ubuf);
        if (g->cmpc) (void)hipFree(g->cmpc);
        if (g->ctl) (void)hipFree(g->ctl);
        hgp_plan_destroy(g->hgp);
        free_timing(g);
        if (g->stream) (void)hipStreamDestroy(g->stream);
        delete g;
    });
}

// Tables of the table-driven SSF kernel (ssf_lut_kernel, qdec_bp.hip; the s_*
// fields of DevGraph).  Inside one generator the spec's choice depends only on
// its local syndrome sl (the residual restricted to the checks its qubits
// touch): the best score max_t gain(t) * 840 / |t| over the non-empty subsets t,
// gain(t) = popc(sl) - popc(sl ^ M_t), and the lowest t reaching it (the
// oracle's strict-improvement scan in ascending t, oracle/qdec_oracle.c
// ssf_run).  One table over sl therefore replaces the per-step subset search,
// and generators whose qubits meet their local checks in the same pattern share
// it: local checks are ordered by signature (the bitmask of the generator's
// qubit positions touching them, ties by check id), which makes the masks M_t
// of two such generators identical (every generator of a hypergraph product
// code has the same 4 x 3 pattern).  Qualifies with <= 128 generators, m_pad <=
// 255 (u8 check ids), <= kLutLC local checks per generator, <= 255 distinct
// positive scores and tables within kLutBudget bytes of LDS; otherwise the s_*
// pointers stay null and the scanning kernel (ssf_wave_kernel) runs.
constexpr size_t kLutBudget = 96 * 1024;
static void ssf_lut_tables(qd_graph* G, int n_gen, const int32_t* gen_ptr, const int32_t* gen_idx, int gp) {
    DevGraph& g = G->dg;
    g.s_lut = g.s_off = g.s_lcw = g.s_tog = nullptr;
    g.s_lut_n = 0;
    // the wave kernel's per-lane tables (u8 check ids, toggle rows by lane);
    // the workgroup SSF kernel reads only the score tables and offsets
    const bool lanes = n_gen <= 128 && g.m_pad <= 255;
    if (n_gen >= 8192) return;
    std::vector<std::vector<uint32_t>> shapes;  // (w, nlc, M_0 .. M_{w-1}) in first-seen order
    std::vector<int> shape_off;
    std::vector<uint32_t> off(gp, 0);
    std::vector<uint32_t> lcw((size_t)kLutLCW * gp, 0xffffffffu);
    std::vector<uint32_t> tog(lanes ? ((size_t)g.m_pad + 1) * 64 : 0, 0);  // row m_pad: zero (unflipped bits)
    int total = 0;
    for (int gi = 0; gi < n_gen; ++gi) {
        const int a = gen_ptr[gi], w = gen_ptr[gi + 1] - a;
        std::vector<std::pair<int, uint32_t>> sig;  // (check, signature)
        for (int k = 0; k < w; ++k) {
            const int q = gen_idx[a + k];
            for (int t = G->col_ptr[q]; t < G->col_ptr[q + 1]; ++t) {
                const int c = G->col_rows[t];
                auto it = std::find_if(sig.begin(), sig.end(), [c](const auto& e) { return e.first == c; });
                if (it == sig.end()) sig.push_back({c, 1u << k});
                else it->second ^= 1u << k;
            }
        }
        if ((int)sig.size() > kLutLC) return;
        std::sort(sig.begin(), sig.end(), [](const auto& x, const auto& y) {
            return x.second != y.second ? x.second < y.second : x.first < y.first;
        });
        const int nlc = (int)sig.size();
        std::vector<uint32_t> key = {(uint32_t)w, (uint32_t)nlc};
        for (int k = 0; k < w; ++k) {
            uint32_t mk = 0;
            for (int b = 0; b < nlc; ++b)
                if ((sig[b].second >> k) & 1) mk |= 1u << b;
            key.push_back(mk);
        }
        const auto it = std::find(shapes.begin(), shapes.end(), key);
        int o;
        if (it == shapes.end()) {
            o = total;
            shapes.push_back(key);
            shape_off.push_back(o);
            total += 1 << nlc;
        } else {
            o = shape_off[it - shapes.begin()];
        }
        off[gi] = (uint32_t)o;
        if (lanes)
            for (int b = 0; b < nlc; ++b) {
                const int c = sig[b].first;
                uint32_t& word = lcw[(size_t)(b / 4) * gp + gi];
                word = (word & ~(0xffu << (8 * (b % 4)))) | ((uint32_t)c << (8 * (b % 4)));
                tog[(size_t)c * 64 + (gi & 63)] |= (1u << b) << (16 * (gi >> 6));
            }
    }
    if ((size_t)total * 4 > kLutBudget) return;
    const bool lane_tabs = lanes && (size_t)total * 4 + ((size_t)g.m_pad + 1) * 256 <= kLutBudget;
    // best (score, t) of every local syndrome of every shape; scores -> ranks
    std::vector<int> score(total, 0);
    std::vector<uint32_t> lut(total, 0);
    for (size_t s = 0; s < shapes.size(); ++s) {
        const int w = (int)shapes[s][0], nlc = (int)shapes[s][1], o = shape_off[s];
        std::vector<uint32_t> Mt((size_t)1 << w, 0);
        for (int t = 1; t < (1 << w); ++t) Mt[t] = Mt[t & (t - 1)] ^ shapes[s][2 + __builtin_ctz(t)];
        for (int sl = 0; sl < (1 << nlc); ++sl) {
            const int base = __builtin_popcount(sl);
            int best = 0, bt = 0;
            for (int t = 1; t < (1 << w); ++t) {
                const int gain = base - __builtin_popcount((uint32_t)sl ^ Mt[t]);
                if (gain <= 0) continue;
                const int sc = gain * kSsfScale / __builtin_popcount(t);
                if (sc > best) {  // strict: ties keep the lowest t
                    best = sc;
                    bt = t;
                }
            }
            score[o + sl] = best;
            lut[o + sl] = bt ? (Mt[bt] << 8 | (uint32_t)bt) : 0u;
        }
    }
    std::vector<int> ranks(score.begin(), score.end());
    std::sort(ranks.begin(), ranks.end());
    ranks.erase(std::unique(ranks.begin(), ranks.end()), ranks.end());
    if (!ranks.empty() && ranks[0] == 0) ranks.erase(ranks.begin());
    if (ranks.size() > 255) return;
    for (int e = 0; e < total; ++e)
        if (score[e] > 0)
            lut[e] |= (uint32_t)(std::lower_bound(ranks.begin(), ranks.end(), score[e]) - ranks.begin() + 1) << 24;
    g.s_lut = G->flip_arena.upload(lut);
    g.s_lut_n = total;
    g.s_off = G->flip_arena.upload(off);
    if (lane_tabs) {
        g.s_lcw = G->flip_arena.upload(lcw);
        g.s_tog = G->flip_arena.upload(tog);
    }
}

int qd_graph_set_flipsets(qd_graph* G, int32_t n_gen, const int32_t* gen_ptr, const int32_t* gen_idx) {
    return guarded([&] {
        check_graph(G);
        set_device(G);
        if (n_gen <= 0 || !gen_ptr || !gen_idx) throw Fail(-30, "invalid flip sets");
        DevGraph& g = G->dg;
        const int gp = std::max(g.m_pad, (n_gen + 63) / 64 * 64);
        const bool pack8 = g.m_pad <= 255;  // u8 local-check ids for the wave SSF kernel
        std::vector<uint8_t> w(gp, 0), nlc(gp, 0);
        std::vector<uint16_t> q((size_t)kGenW * gp, 0), lc((size_t)kGenLC * gp, 0);
        std::vector<uint32_t> qm((size_t)kGenW * gp, 0);
        std::vector<uint32_t> lc8((size_t)(kGenLC / 4) * gp, 0);
        for (int gi = 0; gi < gp; ++gi)
            for (int c = 0; c < kGenLC; ++c) lc8[(size_t)(c / 4) * gp + gi] |= (uint32_t)g.m_pad << (8 * (c % 4));
        int wmax = 0, nlcmax = 0;
        std::vector<std::vector<uint16_t>> inv(g.m_pad);  // check -> (generator, local bit)
        std::vector<std::vector<uint32_t>> inv_all(g.m);  // the same for every generator (block SSF)
        for (int gi = 0; gi < n_gen; ++gi) {
            const int a = gen_ptr[gi], b = gen_ptr[gi + 1];
            if (b < a) throw Fail(-31, "gen_ptr not monotone");
            const int wg = b - a;
            if (wg > kGenW) throw Fail(-32, "flip-set generator weight exceeds 8");
            // local checks in the canonical order of ssf_lut_tables: by signature
            // (the bitmask of this generator's qubit positions touching the
            // check), ties by check id.  The spec does not depend on the order
            // (it is internal to the local-syndrome words), and with it every
            // kernel's local syndrome indexes the shared score tables directly.
            std::vector<std::pair<uint32_t, int>> sig;  // (signature, check)
            for (int k = 0; k < wg; ++k) {
                const int qq = gen_idx[a + k];
                if (qq < 0 || qq >= g.n) throw Fail(-33, "flip-set qubit out of range");
                if (k > 0 && qq <= gen_idx[a + k - 1]) throw Fail(-34, "flip-set qubits must be strictly ascending");
                for (int t = G->col_ptr[qq]; t < G->col_ptr[qq + 1]; ++t) {
                    const int c = G->col_rows[t];
                    auto it = std::find_if(sig.begin(), sig.end(), [c](const auto& e) { return e.second == c; });
                    if (it == sig.end()) sig.push_back({1u << k, c});
                    else it->first ^= 1u << k;
                }
            }
            std::sort(sig.begin(), sig.end());
            std::vector<int> checks;
            for (const auto& e : sig) checks.push_back(e.second);
            if ((int)checks.size() > kGenLC) throw Fail(-35, "flip-set generator touches more than 32 checks");
            w[gi] = (uint8_t)wg;
            nlc[gi] = (uint8_t)checks.size();
            wmax = std::max(wmax, wg);
            nlcmax = std::max(nlcmax, (int)checks.size());
            for (size_t c = 0; c < checks.size(); ++c) {
                lc[c * gp + gi] = (uint16_t)checks[c];
                if (gi < 256) inv[checks[c]].push_back((uint16_t)(gi | (c << 8)));
                inv_all[checks[c]].push_back((uint32_t)gi | ((uint32_t)c << 16));
                uint32_t& word = lc8[(c / 4) * gp + gi];
                word = (word & ~(0xffu << (8 * (c % 4)))) | ((uint32_t)checks[c] << (8 * (c % 4)));
            }
            for (int k = 0; k < wg; ++k) {
                q[(size_t)k * gp + gi] = (uint16_t)gen_idx[a + k];
                uint32_t mask = 0;
                for (size_t c = 0; c < sig.size(); ++c)
                    if ((sig[c].first >> k) & 1u) mask |= 1u << c;
                qm[(size_t)k * gp + gi] = mask;
            }
        }
        size_t invmax = 1;
        for (const auto& v : inv) invmax = std::max(invmax, v.size());
        int invl = 0;
        while ((size_t)1 << invl < invmax) ++invl;
        const int invd = 1 << invl;
        std::vector<uint16_t> invt;
        // graphs whose table would be too wide get none: the scanning wave SSF
        // kernel then re-gathers the local syndromes every step (QD_SSF_SCAN_GATHER
        // takes that path on any graph)
        if (pack8 && n_gen <= 128 && invd <= 64) {
            invt.assign((size_t)g.m_pad * invd, 0xffff);
            for (int i = 0; i < g.m_pad; ++i)
                for (size_t t = 0; t < inv[i].size(); ++t) invt[(size_t)i * invd + t] = inv[i][t];
        }
        G->flip_arena.release();
        g.g_lc8 = nullptr;
        g.g_inv = invt.empty() ? nullptr : G->flip_arena.upload(invt);
        g.g_invd = invt.empty() ? 0 : invd;
        g.g_invl = invt.empty() ? 0 : invl;
        g.g_w = G->flip_arena.upload(w);
        g.g_nlc = G->flip_arena.upload(nlc);
        g.g_q = G->flip_arena.upload(q);
        g.g_lc = G->flip_arena.upload(lc);
        g.g_qmask = G->flip_arena.upload(qm);
        if (pack8) g.g_lc8 = G->flip_arena.upload(lc8);
        g.g_nlcmax = nlcmax;
        ssf_lut_tables(G, n_gen, gen_ptr, gen_idx, gp);
        g.g_iptr = nullptr;
        g.g_ient = nullptr;
        if (n_gen < 65536) {
            std::vector<int32_t> iptr(g.m + 1, 0);
            std::vector<uint32_t> ient;
            for (int i = 0; i < g.m; ++i) {
                ient.insert(ient.end(), inv_all[i].begin(), inv_all[i].end());
                iptr[i + 1] = (int32_t)ient.size();
            }
            g.g_iptr = G->flip_arena.upload(iptr);
            g.g_ient = G->flip_arena.upload(ient);
        }
        g.n_gen = n_gen;
        g.g_pad = gp;
        g.g_wmax = wmax;
    });
}

// Upload logicals given as CSR supports: the CSR itself (duplicates cancelled,
// sorted) and, when it stays below 256 MB, the dense bit-packed table the wave
// kernels and the OSD finalize read.  lz_sparse picks the workgroup finalize's
// support walk when the supports are small against the dense words.
static void upload_logicals(qd_graph* G, int32_t k, std::vector<int32_t> ptr, std::vector<int32_t> idx) {
    DevGraph& g = G->dg;
    const int W = g.lz_words;
    G->lz_arena.release();
    g.lz = nullptr;
    g.lz_ptr = g.lz_idx = nullptr;
    g.ms_lzs = nullptr;
    g.lz_t = nullptr;
    g.lz_tw = 0;
    g.k = 0;
    g.lz_sparse = 0;
    if (k == 0) return;
    // canonical supports: sorted, pairs cancel
    std::vector<int32_t> cptr(1, 0), cidx;
    cidx.reserve(idx.size());
    for (int r = 0; r < k; ++r) {
        std::vector<int32_t> row(idx.begin() + ptr[r], idx.begin() + ptr[r + 1]);
        std::sort(row.begin(), row.end());
        for (size_t t = 0; t < row.size();) {
            size_t u = t;
            while (u < row.size() && row[u] == row[t]) ++u;
            if ((u - t) & 1) cidx.push_back(row[t]);
            t = u;
        }
        cptr.push_back((int32_t)cidx.size());
    }
    if ((size_t)k * W * 8 <= ((size_t)256 << 20)) {
        std::vector<uint64_t> packed((size_t)k * W, 0);
        for (int r = 0; r < k; ++r)
            for (int t = cptr[r]; t < cptr[r + 1]; ++t) packed[(size_t)r * W + cidx[t] / 64] |= 1ull << (cidx[t] % 64);
        g.lz = G->lz_arena.upload(packed);
    }
    g.lz_ptr = G->lz_arena.upload(cptr);
    g.lz_idx = G->lz_arena.upload(cidx);
    const int tw = (k + 31) / 32;
    if ((size_t)g.n_data * tw * 4 <= ((size_t)64 << 20)) {
        std::vector<uint32_t> tr((size_t)g.n_data * tw, 0u);
        for (int r = 0; r < k; ++r)
            for (int t = cptr[r]; t < cptr[r + 1]; ++t) tr[(size_t)cidx[t] * tw + r / 32] |= 1u << (r % 32);
        g.lz_t = G->lz_arena.upload(tr);
        g.lz_tw = tw;
    }
    // wave graphs: the same logicals in the min-sum kernel's lane-slot order
    // ([k][n_pad/64] words, bit s%64 of word s/64 = the column of slot s), so the
    // compact-list kernel tests its ballot words without a column permutation
    g.ms_lzs = nullptr;
    if (!G->ms_var_of_slot.empty() && k <= 256) {
        const int RVn = g.n_pad / 64;
        std::vector<int> col_bit(g.n_data, -1);
        for (int sl = 0; sl < g.n_pad; ++sl) {
            const int j = G->ms_var_of_slot[sl];
            if (j >= 0 && j < g.n_data) col_bit[j] = sl;
        }
        std::vector<uint64_t> lzs((size_t)k * RVn, 0);
        for (int r = 0; r < k; ++r)
            for (int t = cptr[r]; t < cptr[r + 1]; ++t) {
                const int sl = col_bit[cidx[t]];
                if (sl >= 0) lzs[(size_t)r * RVn + sl / 64] |= 1ull << (sl % 64);
            }
        g.ms_lzs = G->lz_arena.upload(lzs);
    }
    // a support walk costs ~ one gather per entry, the dense test one word per
    // (logical, word): walk when that is clearly cheaper, or when there is no table
    g.lz_sparse = (!g.lz || cidx.size() <= (size_t)k * W / 4) ? 1 : 0;
    g.k = k;
}

int qd_graph_set_logicals(qd_graph* G, int32_t k, const uint8_t* lz) {
    return guarded([&] {
        check_graph(G);
        set_device(G);
        DevGraph& g = G->dg;
        if (k < 0 || (k > 0 && !lz)) throw Fail(-40, "invalid logicals");
        if (k > 65536) throw Fail(-41, "more than 65536 logicals not supported");
        std::vector<int32_t> ptr(1, 0), idx;
        for (int r = 0; r < k; ++r) {
            for (int q = 0; q < g.n_data; ++q)
                if (lz[(size_t)r * g.n_data + q] & 1) idx.push_back(q);
            ptr.push_back((int32_t)idx.size());
        }
        upload_logicals(G, k, std::move(ptr), std::move(idx));
    });
}

int qd_graph_set_logicals_csr(qd_graph* G, int32_t k, const int32_t* lz_ptr, const int32_t* lz_idx) {
    return guarded([&] {
        check_graph(G);
        set_device(G);
        const DevGraph& g = G->dg;
        if (k < 0 || (k > 0 && (!lz_ptr || (!lz_idx && lz_ptr[k] > 0)))) throw Fail(-40, "invalid logicals");
        if (k > 65536) throw Fail(-41, "more than 65536 logicals not supported");
        std::vector<int32_t> ptr(lz_ptr, lz_ptr + (k > 0 ? k + 1 : 0)), idx;
        if (k > 0) {
            if (ptr[0] != 0) throw Fail(-42, "logicals CSR must start at 0");
            for (int r = 0; r < k; ++r)
                if (ptr[r + 1] < ptr[r]) throw Fail(-42, "logicals CSR pointers must be non-decreasing");
            idx.assign(lz_idx, lz_idx + ptr[k]);
            for (int32_t q : idx)
                if (q < 0 || q >= g.n_data) throw Fail(-43, "logical support index out of range");
        }
        upload_logicals(G, k, std::move(ptr), std::move(idx));
    });
}

int qd_graph_set_priors(qd_graph* G, const double* probs) {
    return guarded([&] {
        check_graph(G);
        set_device(G);
        if (!probs) throw Fail(-50, "null channel_probs");
        DevGraph& g = G->dg;
        std::vector<double> ms64(g.n_pad, 0.0), ps64(g.n_pad, 0.0);
        std::vector<float> ms32(g.n_pad, 0.0f), ps32(g.n_pad, 0.0f);
        for (int j = 0; j < g.n; ++j) {
            const double p = probs[j];
            // open interval: keeps every BP message finite (and NaN-free), the
            // precondition of the kernels' min/med3 check-node formulation
            if (!(p > 0.0 && p < 1.0)) throw Fail(-51, "channel probability outside (0, 1)");
            ms64[j] = std::log((1 - p) / p);   // ldpc v1: log((1-p)/p)
            ps64[j] = p / (1 - p);             // ldpc v1: p/(1-p)
            ms32[j] = (float)ms64[j];
            ps32[j] = (float)ps64[j];
        }
        G->prior_arena.release();
        g.prior[QD_MIN_SUM][QD_F64] = G->prior_arena.upload(ms64);
        g.prior[QD_MIN_SUM][QD_F32] = G->prior_arena.upload(ms32);
        if (!G->ms_var_of_slot.empty()) {  // min-sum wave kernel: lane-slot order
            std::vector<double> s64(g.n_pad, 0.0);
            std::vector<float> s32(g.n_pad, 0.0f);
            for (int s2 = 0; s2 < g.n_pad; ++s2) {
                const int j = G->ms_var_of_slot[s2];
                if (j >= 0) {
                    s64[s2] = ms64[j];
                    s32[s2] = ms32[j];
                }
            }
            g.ms_prior[QD_F64] = G->prior_arena.upload(s64);
            g.ms_prior[QD_F32] = G->prior_arena.upload(s32);
            // all priors > 0: the wave kernel's zero-syndrome shortcut applies
            bool pos64 = true, pos32 = true;
            for (int j = 0; j < g.n; ++j) {
                pos64 = pos64 && ms64[j] > 0.0;
                pos32 = pos32 && ms32[j] > 0.0f;
            }
            g.ms_allpos = (pos64 ? 1 << QD_F64 : 0) | (pos32 ? 1 << QD_F32 : 0);
            it1_tables(G, pos64, ms64, pos32, ms32);
        }
        g.prior[QD_PRODUCT_SUM][QD_F64] = G->prior_arena.upload(ps64);
        g.prior[QD_PRODUCT_SUM][QD_F32] = G->prior_arena.upload(ps32);
        {  // by CSR edge, padded (slot-group kernel)
            const size_t ne = (size_t)g.E + kEdgePad;
            std::vector<double> ems64(ne, 0.0), eps64(ne, 0.0);
            std::vector<float> ems32(ne, 0.0f), eps32(ne, 0.0f);
            for (int e = 0; e < g.E; ++e) {
                const int j = G->col_idx[e];
                ems64[e] = ms64[j], eps64[e] = ps64[j], ems32[e] = ms32[j], eps32[e] = ps32[j];
            }
            g.eprior[QD_MIN_SUM][QD_F64] = G->prior_arena.upload(ems64);
            g.eprior[QD_MIN_SUM][QD_F32] = G->prior_arena.upload(ems32);
            g.eprior[QD_PRODUCT_SUM][QD_F64] = G->prior_arena.upload(eps64);
            g.eprior[QD_PRODUCT_SUM][QD_F32] = G->prior_arena.upload(eps32);
        }
        G->has_priors = true;
    });
}

int qd_decode_batch_device(qd_graph* G, const qd_params* p, int64_t B, const uint8_t* syn, const uint8_t* base,
                           const uint8_t* readout, uint8_t* x_out, uint8_t* corr_out, void* llr_out, int32_t* iters,
                           uint8_t* status, int32_t* ssf_steps, uint8_t* fail, void* stream) {
    return guarded([&] {
        check_graph(G);
        check_params(G, p);
        if (B < 0) throw Fail(-8, "negative batch");
        if (B == 0) return;  // nothing to enqueue
        set_device(G);
        DecodeArgs a = make_args(G, p, B, syn, base, readout, x_out, corr_out, llr_out, iters, status, ssf_steps, fail);
        attach_queue(G, a, p->method, p->precision);
        attach_unpack(G, a);
        attach_timing(G, a);
        size_t sb = 0;
        void* scr = message_scratch(G, p->method, p->precision, a, &sb);
        const hipStream_t s = (hipStream_t)stream;
        const bool split = G->ssf_stream && G->ssf_stream != s && a.ssf;
        const int qb = split ? G->q_buf : 0;
        if (split) {
            a.ssf_stream = G->ssf_stream;
            a.ssf_ev = G->ssf_ev;
            if (qb == 1) attach_queue2(G, a);
            a.wave_ctr = static_cast<unsigned long long*>(G->ctl) + 32 * qb;
        }
        ws_acquire(G, s);
        // the SSF kernel that last used this decode's queue (split decodes: two
        // back on this handle) must have finished before the queue is reset
        if (G->ssf_done_live[qb]) hip_check(hipStreamWaitEvent(s, G->ssf_done[qb], 0), "hipStreamWaitEvent");
        const int rc = launch_decode(G->dg, p->method, p->precision, a, G->num_cus, s, scr, sb);
        note_kernels(G);
        flip_counters(G, a);  // also after a failed BP launch: its triage zeroed the other set
        if (rc != 0) throw Fail(-101, std::string("decode launch failed: ") + hipGetErrorString((hipError_t)rc));
        note_listed(G, a, s, s);
        if (split) {  // the SSF kernel runs on its own stream behind this decode's BP
            if (!G->ssf_done[qb])
                hip_check(hipEventCreateWithFlags(&G->ssf_done[qb], hipEventDisableTiming), "hipEventCreate");
            hip_check(hipEventRecord(G->ssf_done[qb], G->ssf_stream), "hipEventRecord");
            G->ssf_done_live[qb] = true;
            G->q_buf ^= 1;
        }
        // the workspace chain (message scratch, compact lists, counters) ends with
        // the BP stage; the SSF queues are ordered by ssf_done
        ws_release(G, s);
    });
}

int qd_decode_batch(qd_graph* G, const qd_params* p, int64_t B, const uint8_t* syn, const uint8_t* base,
                    const uint8_t* readout, uint8_t* x_out, uint8_t* corr_out, void* llr_out, int32_t* iters,
                    uint8_t* status, int32_t* ssf_steps, uint8_t* fail) {
    return guarded([&] {
        check_graph(G);
        check_params(G, p);
        if (B < 0) throw Fail(-8, "negative batch");
        if (B == 0) return;
        set_device(G);
        const DevGraph& g = G->dg;
        const size_t tsz = p->precision == QD_F32 ? 4 : 8;
        // input row bytes: one byte per bit, or whole u64 words (QD_INPUT_PACKED)
        const bool pk = (p->syn_flags & QD_INPUT_PACKED) != 0;
        const size_t syn_row = pk ? ((size_t)g.m + 63) / 64 * 8 : (size_t)g.m;
        const size_t dat_row = pk ? ((size_t)g.n_data + 63) / 64 * 8 : (size_t)g.n_data;
        // workspace layout (each region 256-B aligned)
        struct Reg { size_t off, bytes; };
        size_t off = 0;
        auto reg = [&](size_t bytes, bool on) {
            Reg r{off, on ? bytes : 0};
            if (on) off += (bytes + 255) / 256 * 256;
            return r;
        };
        const Reg r_syn = reg((size_t)B * syn_row, syn != nullptr);
        const Reg r_base = reg((size_t)B * dat_row, base != nullptr);
        const Reg r_rd = reg((size_t)B * dat_row, readout != nullptr);
        const Reg r_x = reg((size_t)B * g.n, x_out != nullptr);
        const Reg r_corr = reg((size_t)B * g.n_data, corr_out != nullptr);
        const Reg r_llr = reg((size_t)B * g.n * tsz, llr_out != nullptr);
        const Reg r_it = reg((size_t)B * 4, iters != nullptr);
        const Reg r_st = reg((size_t)B, status != nullptr);
        const Reg r_ss = reg((size_t)B * 4, ssf_steps != nullptr);
        const Reg r_fl = reg((size_t)B, fail != nullptr);
        if (off > G->ws_bytes) {
            if (G->ws) hip_check(hipFree(G->ws), "hipFree");
            G->ws = nullptr;
            G->ws_bytes = 0;
            hip_check(hipMalloc(&G->ws, off), "hipMalloc workspace");
            G->ws_bytes = off;
        }
        auto* w = static_cast<uint8_t*>(G->ws);
        auto dptr = [&](const Reg& r) -> void* { return r.bytes ? (void*)(w + r.off) : nullptr; };
        hipStream_t s = G->stream;
        if (syn) hip_check(hipMemcpyAsync(dptr(r_syn), syn, r_syn.bytes, hipMemcpyHostToDevice, s), "H2D syn");
        if (base) hip_check(hipMemcpyAsync(dptr(r_base), base, r_base.bytes, hipMemcpyHostToDevice, s), "H2D base");
        if (readout) hip_check(hipMemcpyAsync(dptr(r_rd), readout, r_rd.bytes, hipMemcpyHostToDevice, s), "H2D readout");
        DecodeArgs a = make_args(G, p, B, (const uint8_t*)dptr(r_syn), (const uint8_t*)dptr(r_base),
                                 (const uint8_t*)dptr(r_rd), (uint8_t*)dptr(r_x), (uint8_t*)dptr(r_corr), dptr(r_llr),
                                 (int32_t*)dptr(r_it), (uint8_t*)dptr(r_st), (int32_t*)dptr(r_ss), (uint8_t*)dptr(r_fl));
        attach_queue(G, a, p->method, p->precision);
        attach_unpack(G, a);
        attach_timing(G, a);
        size_t sb = 0;
        void* scr = message_scratch(G, p->method, p->precision, a, &sb);
        ws_acquire(G, s);
        const int rc = launch_decode(g, p->method, p->precision, a, G->num_cus, s, scr, sb);
        note_kernels(G);
        flip_counters(G, a);  // also after a failed BP launch: its triage zeroed the other set
        if (rc != 0) throw Fail(-101, std::string("decode launch failed: ") + hipGetErrorString((hipError_t)rc));
        note_listed(G, a, s, s);
        ws_release(G, s);
        auto d2h = [&](void* h, const Reg& r, const char* what) {
            if (h) hip_check(hipMemcpyAsync(h, dptr(r), r.bytes, hipMemcpyDeviceToHost, s), what);
        };
        d2h(x_out, r_x, "D2H x");
        d2h(corr_out, r_corr, "D2H corr");
        d2h(llr_out, r_llr, "D2H llr");
        d2h(iters, r_it, "D2H iters");
        d2h(status, r_st, "D2H status");
        d2h(ssf_steps, r_ss, "D2H ssf_steps");
        d2h(fail, r_fl, "D2H fail");
        hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
    });
}

static int sample_storage(qd_graph* G, int32_t rounds, double p_data, double p_meas, uint32_t seed,
                          uint32_t stream_id, int64_t shot0, int64_t B, uint8_t* syn, uint8_t* readout,
                          void* stream, bool packed) {
    return guarded([&] {
        check_graph(G);
        if (rounds < 0 || B < 0) throw Fail(-60, "invalid sampler arguments");
        if (B == 0) return;
        if (!syn || !readout) throw Fail(-60, "invalid sampler arguments");
        if (packed && (((uintptr_t)syn | (uintptr_t)readout) & 7)) throw Fail(-60, "packed rows must be 8-B aligned");
        if (G->dg.fold_blocks != 1 || G->dg.n_data != G->dg.n) throw Fail(-61, "sampler needs a plain code graph (H = Hz)");
        auto thr = [](double p) -> uint32_t {
            if (!(p > 0)) return 0u;
            const double v = std::floor(p * 4294967296.0);
            return v >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)v;
        };
        set_device(G);
        const int rc = launch_sample_storage(G->dg, rounds, thr(2.0 * p_data / 3.0), thr(p_meas), seed, stream_id,
                                             shot0, B, syn, readout, G->num_cus, (hipStream_t)stream, packed);
        if (rc != 0) throw Fail(-102, std::string("sampler launch failed: ") + hipGetErrorString((hipError_t)rc));
    });
}

int qd_sample_storage_device(qd_graph* G, int32_t rounds, double p_data, double p_meas, uint32_t seed,
                             uint32_t stream_id, int64_t shot0, int64_t B, uint8_t* syn, uint8_t* readout,
                             void* stream) {
    return sample_storage(G, rounds, p_data, p_meas, seed, stream_id, shot0, B, syn, readout, stream, false);
}

int qd_sample_storage_packed_device(qd_graph* G, int32_t rounds, double p_data, double p_meas, uint32_t seed,
                                    uint32_t stream_id, int64_t shot0, int64_t B, uint64_t* syn, uint64_t* readout,
                                    void* stream) {
    return sample_storage(G, rounds, p_data, p_meas, seed, stream_id, shot0, B, reinterpret_cast<uint8_t*>(syn),
                          reinterpret_cast<uint8_t*>(readout), stream, true);
}

int qd_osd_device_supported(const qd_graph* G) {
    if (!G) return 0;
    return osd_kernel_supports(G->dg) ? 1 : 0;
}

int qd_osd_batch_device(qd_graph* G, int32_t method, int32_t order, int64_t B, const uint8_t* syn, int32_t syn_flags,
                        const void* llr, int32_t llr_precision, const uint8_t* status, const uint8_t* base,
                        const uint8_t* readout, uint8_t* osd0_out, uint8_t* osdw_out, uint8_t* corr_out, uint8_t* fail,
                        void* stream) {
    return guarded([&] {
        check_graph(G);
        if (method < 0 || method > 2) throw Fail(-80, "osd method must be 0 (osd0), 1 (osd_e), 2 (osd_cs)");
        if (method == 1 && order > 20) throw Fail(-81, "osd_e order above 20 is not supported");
        if (method == 2 && order > 64) throw Fail(-82, "osd_cs order above 64 is not supported on the device");
        if (B < 0) throw Fail(-8, "negative batch");
        if (B == 0) return;
        if (!llr || (!syn && !syn_flags)) throw Fail(-83, "null OSD inputs");
        if (llr_precision != QD_F32 && llr_precision != QD_F64) throw Fail(-84, "invalid llr precision");
        if (!osd_kernel_supports(G->dg)) throw Fail(-85, "graph too large for the device OSD (LDS image above 160 KiB)");
        if (fail && G->dg.k > 256) throw Fail(-86, "fused failure check after OSD supports <= 256 logicals");
        if (B == 0) return;
        set_device(G);
        OsdArgs a{};
        a.B = B;
        a.method = method;
        a.order = order;
        a.syn_flags = syn_flags;
        a.llr_f32 = llr_precision == QD_F32 ? 1 : 0;
        a.syn = syn;
        a.llr = llr;
        a.status = status;
        a.base = base;
        a.readout = readout;
        a.osd0_out = osd0_out;
        a.osdw_out = osdw_out;
        a.corr_out = corr_out;
        a.fail = fail;
        const int rc = launch_osd(G->dg, a, G->num_cus, (hipStream_t)stream);
        if (rc != 0) throw Fail(-104, std::string("osd launch failed: ") + hipGetErrorString((hipError_t)rc));
    });
}

int qd_graph_set_ssf_stream(qd_graph* G, void* ssf_stream) {
    return guarded([&] {
        check_graph(G);
        set_device(G);
        if (ssf_stream && !G->ssf_ev)
            hip_check(hipEventCreateWithFlags(&G->ssf_ev, hipEventDisableTiming), "hipEventCreate");
        G->ssf_stream = (hipStream_t)ssf_stream;
    });
}

int qd_graph_set_wave_occupancy(qd_graph* G, int32_t waves_per_cu) {
    return guarded([&] {
        check_graph(G);
        if (waves_per_cu < 0 || waves_per_cu > 64) throw Fail(-62, "waves_per_cu outside [0, 64]");
        G->dg.wave_occ = waves_per_cu;
    });
}

int qd_graph_set_timing(qd_graph* G, int32_t capacity) {
    return guarded([&] {
        check_graph(G);
        set_device(G);
        if (capacity < 0) throw Fail(-90, "negative timing capacity");
        free_timing(G);
        G->tev.resize((size_t)kTimingEvents * capacity);
        for (auto& e : G->tev) hip_check(hipEventCreate(&e), "hipEventCreate");
        if (capacity > 0) {
            void* h = nullptr;
            hip_check(hipHostMalloc(&h, (size_t)capacity * kCmpLists * kCmpSegs * 8, hipHostMallocDefault),
                      "hipHostMalloc");
            G->t_listed = static_cast<uint64_t*>(h);
            G->t_cmp.assign(capacity, 0);
        }
        G->t_cap = capacity;
        G->t_count = 0;
    });
}

int qd_graph_read_timing(qd_graph* G, float* bp_ms, float* ssf_ms, int32_t max_calls, int32_t* n_calls) {
    return guarded([&] {
        check_graph(G);
        set_device(G);
        if (!n_calls) throw Fail(-91, "null n_calls");
        const int n = std::min(G->t_count, std::max(0, max_calls));
        for (int i = 0; i < n; ++i) {
            hipEvent_t* e = &G->tev[(size_t)kTimingEvents * i];
            hip_check(hipEventSynchronize(e[2]), "hipEventSynchronize");
            float t0 = 0, t1 = 0;
            hip_check(hipEventElapsedTime(&t0, e[0], e[1]), "hipEventElapsedTime");
            hip_check(hipEventElapsedTime(&t1, e[1], e[2]), "hipEventElapsedTime");
            if (bp_ms) bp_ms[i] = t0;
            if (ssf_ms) ssf_ms[i] = t1;
        }
        *n_calls = n;
        G->t_count = 0;
    });
}

int qd_graph_read_timing_detail(qd_graph* G, float* pre_ms, float* bp_ms, float* ssf_ms, int64_t* listed,
                                int32_t max_calls, int32_t* n_calls) {
    return guarded([&] {
        check_graph(G);
        set_device(G);
        if (!n_calls) throw Fail(-91, "null n_calls");
        const int n = std::min(G->t_count, std::max(0, max_calls));
        for (int i = 0; i < n; ++i) {
            hipEvent_t* e = &G->tev[(size_t)kTimingEvents * i];
            hip_check(hipEventSynchronize(e[2]), "hipEventSynchronize");
            hip_check(hipEventSynchronize(e[1]), "hipEventSynchronize");
            if (G->t_cmp[i]) hip_check(hipEventSynchronize(e[4]), "hipEventSynchronize");
            float t0 = 0, t1 = 0, t2 = 0;
            hip_check(hipEventElapsedTime(&t0, e[0], e[3]), "hipEventElapsedTime");
            hip_check(hipEventElapsedTime(&t1, e[3], e[1]), "hipEventElapsedTime");
            hip_check(hipEventElapsedTime(&t2, e[1], e[2]), "hipEventElapsedTime");
            if (pre_ms) pre_ms[i] = t0;
            if (bp_ms) bp_ms[i] = t1;
            if (ssf_ms) ssf_ms[i] = t2;
            if (listed) {
                int64_t c = -1;
                if (G->t_cmp[i]) {
                    c = 0;
                    for (int k = 0; k < kCmpLists * kCmpSegs; ++k)
                        c += (int64_t)G->t_listed[((size_t)i * kCmpLists) * kCmpSegs + k];
                }
                listed[i] = c;
            }
        }
        *n_calls = n;
        G->t_count = 0;
    });
}

int qd_graph_last_kernels(qd_graph* G, char* bp, int32_t bp_len, char* ssf, int32_t ssf_len, char* pre,
                          int32_t pre_len) {
    return guarded([&] {
        check_graph(G);
        auto put = [](const std::string& v, char* out, int32_t len) {
            if (!out || len <= 0) return;
            const size_t k = std::min(v.size(), (size_t)len - 1);
            std::memcpy(out, v.data(), k);
            out[k] = '\0';
        };
        put(G->last_bp, bp, bp_len);
        put(G->last_ssf, ssf, ssf_len);
        put(G->last_pre, pre, pre_len);
    });
}

int qd_graph_set_option(qd_graph* G, int32_t option, int32_t value) {
    return guarded([&] {
        check_graph(G);
        DevGraph& g = G->dg;
        auto in = [&](int lo, int hi) {
            if (value < lo || value > hi) throw Fail(-2, "option value out of range");
        };
        switch (option) {
            case QD_OPT_COMPACT: in(0, 1); g.opt_compact = value; break;
            case QD_OPT_TRIAGE_IT1: in(0, 1); g.opt_triage_it1 = value; break;
            case QD_OPT_SSF: in(QD_SSF_AUTO, QD_SSF_SCAN_NOSPLIT); g.opt_ssf = value; break;
            case QD_OPT_LDS_KERNEL: in(-1, 1); g.opt_lds_kernel = value; break;
            case QD_OPT_GROUP_KERNEL: in(-1, 1); g.opt_group_kernel = value; break;
            case QD_OPT_SSF_INC: in(0, 1); g.opt_ssf_inc = value; break;
            case QD_OPT_BLOCK_WG: in(0, 64); g.opt_block_wg = value; break;
            case QD_OPT_GROUP_MB: in(0, 1 << 22); g.opt_group_mb = value; break;
            case QD_OPT_SSF_FUSE: in(0, 1); g.opt_ssf_fuse = value; break;
            default: throw Fail(-2, "unknown option");
        }
    });
}

int qd_graph_get_option(const qd_graph* G, int32_t option, int32_t* value) {
    return guarded([&] {
        check_graph(G);
        if (!value) throw Fail(-1, "null output");
        const DevGraph& g = G->dg;
        switch (option) {
            case QD_OPT_COMPACT: *value = g.opt_compact; break;
            case QD_OPT_TRIAGE_IT1: *value = g.opt_triage_it1; break;
            case QD_OPT_SSF: *value = g.opt_ssf; break;
            case QD_OPT_LDS_KERNEL: *value = g.opt_lds_kernel; break;
            case QD_OPT_GROUP_KERNEL: *value = g.opt_group_kernel; break;
            case QD_OPT_SSF_INC: *value = g.opt_ssf_inc; break;
            case QD_OPT_BLOCK_WG: *value = g.opt_block_wg; break;
            case QD_OPT_GROUP_MB: *value = g.opt_group_mb; break;
            case QD_OPT_SSF_FUSE: *value = g.opt_ssf_fuse; break;
            default: throw Fail(-2, "unknown option");
        }
    });
}

int qd_graph_ssf_tables(const qd_graph* G, int32_t* has_lut, int64_t* lut_bytes) {
    return guarded([&] {
        check_graph(G);
        if (has_lut) *has_lut = G->dg.s_lut ? (G->dg.s_tog ? 1 : 2) : 0;
        if (lut_bytes) *lut_bytes = G->dg.s_lut ? (int64_t)G->dg.s_lut_n * 4 : 0;
    });
}

int qd_graph_ssf_tables_copy(const qd_graph* G, uint32_t* lut, uint32_t* off, uint32_t* lcw, uint32_t* tog,
                             int32_t* g_pad, int32_t* m_pad) {
    return guarded([&] {
        check_graph(G);
        if (!G->host_only) throw Fail(-16, "table copies are kept for host-only graphs (qd_graph_create_host)");
        const DevGraph& g = G->dg;
        if (!g.s_lut || !g.s_tog) throw Fail(-36, "the graph has no table-driven wave SSF tables");
        if (g_pad) *g_pad = g.g_pad;
        if (m_pad) *m_pad = g.m_pad;
        auto put = [](uint32_t* dst, const uint32_t* src, size_t n) {
            if (dst) std::memcpy(dst, src, n * 4);
        };
        put(lut, g.s_lut, (size_t)g.s_lut_n);
        put(off, g.s_off, (size_t)g.g_pad);
        put(lcw, g.s_lcw, (size_t)kLutLCW * g.g_pad);
        put(tog, g.s_tog, ((size_t)g.m_pad + 1) * 64);
    });
}

int qd_graph_queue_layout(const qd_graph* G, int64_t B, int64_t* out) {
    return guarded([&] {
        check_graph(G);
        if (B <= 0 || !out) throw Fail(-8, "invalid batch or null output");
        const QueueLayout L = queue_layout(G->dg, B);
        const int64_t v[8] = {(int64_t)L.bytes, (int64_t)L.idx, (int64_t)L.x, (int64_t)L.r, (int64_t)L.cmp_count,
                              (int64_t)L.cmp, L.cmp_cap, (int64_t)cmp_entry_bytes(G->dg)};
        std::memcpy(out, v, sizeof(v));
    });
}

int qd_graph_it1_tables_copy(const qd_graph* G, int32_t precision, uint16_t* lut, uint64_t* vchk, int32_t* n_pad) {
    return guarded([&] {
        check_graph(G);
        if (!G->host_only) throw Fail(-16, "table copies are kept for host-only graphs (qd_graph_create_host)");
        if (precision != QD_F64 && precision != QD_F32) throw Fail(-4, "invalid precision");
        const DevGraph& g = G->dg;
        if (n_pad) *n_pad = g.n_pad;
        if (!g.it1_lut[precision] || !g.it1_vchk) throw Fail(-37, "no iteration-1 tables for this precision");
        if (lut) std::memcpy(lut, g.it1_lut[precision], (size_t)g.n_pad * 2);
        if (vchk) std::memcpy(vchk, g.it1_vchk, (size_t)g.n_pad * 8);
    });
}

int qd_graph_lds64_slots_copy(const qd_graph* G, uint16_t* etab, uint16_t* check_of_slot) {
    return guarded([&] {
        check_graph(G);
        if (!G->host_only) throw Fail(-16, "table copies are kept for host-only graphs (qd_graph_create_host)");
        const DevGraph& g = G->dg;
        if (!g.m64_etab || !g.m64_check) throw Fail(-38, "no f64 LDS-kernel slot tables for this graph");
        if (etab) std::memcpy(etab, g.m64_etab, (size_t)kMlDC * g.n * 2);
        if (check_of_slot) std::memcpy(check_of_slot, g.m64_check, (size_t)g.m * 2);
    });
}

int qd_count_flags_device(const uint8_t* flags, int64_t B, uint8_t mask, int64_t* out, void* stream) {
    return guarded([&] {
        if (B < 0 || (B > 0 && (!flags || !out))) throw Fail(-70, "invalid count arguments");
        const int rc = launch_count_flags(flags, B, mask, out, (hipStream_t)stream);
        if (rc != 0) throw Fail(-103, std::string("count launch failed: ") + hipGetErrorString((hipError_t)rc));
    });
}

}  // extern "C"
