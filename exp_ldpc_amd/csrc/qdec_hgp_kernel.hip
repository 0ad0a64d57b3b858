// qdec_hgp_kernel.hip -- f64 min-sum BP for hypergraph-product codes, one
// kernel per code, compiled at graph set-up by hipRTC (qdec_hgp.cpp) after a
// generated prologue that fixes the code's factors as compile-time tables.
//
// A hypergraph-product Z check matrix is H = [I_a0 (x) B | A (x) I_b0] (hgp.py
// homological_product: A is a0 x a1, B is b0 x b1).  Check (x, y) = x*b0 + y
// meets the left qubits (x, z) = x*b1 + z with B[y, z] = 1 and the right qubits
// (w, y) = a0*b1 + w*b0 + y with A[x, w] = 1.  So the left qubits of "column"
// x and the left halves of checks (x, .) form one copy of B's Tanner graph,
// and the right qubits of "row" y with the right halves of checks (., y) one
// copy of A's.  A left lane owns copy x of one shot, a right lane copy y: all
// of its v2c messages live in registers (indexed by the compile-time edge
// lists below), and the only cross-lane traffic per iteration is the two
// halves' partial check states (min-sum: (m1, m2) with the half's parity, 16 B
// per check and side) through LDS -- against 32 B per edge + 16 B per check for
// the generic wave kernel.
//
// Arithmetic, operation for operation as ldpc v1 min-sum (and MsCore, the
// generic f64 wave kernel, qdec_bp_ms.h):
//   check: c2v_k = alpha_it * (|v_k| == m1 ? m2 : m1), sign = syndrome ^ XOR of
//          (v <= 0) over the other edges; (m1, m2) = the two smallest |v| with
//          multiplicity, merged from the halves (min / max are exact, so the
//          split changes no value)
//   variable: prefix sums from the prior in ascending check order, each
//          outgoing message = prefix + (sum of the later c2v, accumulated
//          from the end); hard decision acc <= 0
//   sign tests by sign bits with MsCore's zero rule (qdec_bp_ms.h:76-118): a
//   half holding a zero entry (its m1 == 0, rare, a divergent branch) takes its
//   parity from compares, and flags a +0 in its m2's sign so the merged m2
//   carries parity ^ (+0 present).
// Iteration pipeline of a workgroup (S shot slots, every slot at its own
// iteration, refilled from a counter when its shot ends), 2 barriers per step:
//   A  left lanes test the previous step's hard decision (their own check
//      parities, the right lanes' through XR, the syndrome); every lane writes
//      its partial states of its current v2c messages
//   |  barrier
//   B  a slot whose decision satisfied the syndrome (or reached max_iter) ends:
//      outputs, refill; the others merge the other side's partials, update
//      messages and decision, and write their decision's check parities
//   |  barrier
// Generated prologue (qdec_hgp.cpp):
//   HG_A0 HG_A1 HG_B0 HG_B1 HG_S HG_WL HG_WR, constexpr edge tables kBrp/kBce/
//   kBcp (B by rows, B's edges by column in ascending row), kBer (row of each
//   edge), kArp/kAce/kAcp/kAer, the row masks kBrm / kArm (bit q: the row
//   touches qubit q), kBE / kAE (edge counts).

#ifndef HG_A0
#error "qdec_hgp_kernel.hip needs the generated prologue"
#endif

typedef unsigned char u8;
typedef unsigned int u32;
typedef unsigned long long u64;
typedef long long i64;

#define HG_THREADS (64 * (HG_WL + HG_WR))
constexpr double kBig = 1e308;

__device__ __forceinline__ u32 hi32(double x) { return (u32)((u64)__double_as_longlong(x) >> 32); }
// x with its sign bit XORed with bit 31 of m: one v_bitop3_b32 on the high dword
// (table 0x6c = (src0 & src2) ^ src1)
__device__ __forceinline__ double xor_sign(double x, u32 m) {
    const u64 b = (u64)__double_as_longlong(x);
    const u32 h = __builtin_amdgcn_bitop3_b32(m, (u32)(b >> 32), 0x80000000u, 0x6c);
    return __longlong_as_double((i64)(((u64)h << 32) | (u32)b));
}
// a magnitude (sign bit clear) given bit 31 of m as its sign: (src0 & src2) | src1
__device__ __forceinline__ double with_sign(double mag, u32 m) {
    const u64 b = (u64)__double_as_longlong(mag);
    const u32 h = __builtin_amdgcn_bitop3_b32(m, (u32)(b >> 32), 0x80000000u, 0xec);
    return __longlong_as_double((i64)(((u64)h << 32) | (u32)b));
}
__device__ __forceinline__ double alpha_at(int it, double ms_scaling) {
    if (ms_scaling != 0.0) return ms_scaling;
    const u64 u = 0x3FF0000000000000ull - (it <= 53 ? (1ull << (53 - it)) : 0ull);
    return __longlong_as_double((i64)u);
}

// f64 min / max on the VALU without the IEEE canonicalisation of the operands
// (the messages are finite, never NaN), with |x| source modifiers
__device__ __forceinline__ double vmin_aa(double a, double b) {
    double r;
    asm("v_min_f64 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double vmax_aa(double a, double b) {
    double r;
    asm("v_max_f64 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double vmin(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double vmax(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// compile-time loops: f(IC<I>{}) for I in [B, E) (the edge tables are then
// constant expressions, so every register index below is static)
template <int V>
struct IC {
    static constexpr int value = V;
};
template <int B, int E, typename F>
__device__ __forceinline__ void sfor(F&& f) {
    if constexpr (B < E) {
        f(IC<B>{});
        sfor<B + 1, E>(f);
    }
}

// (smallest, second smallest) of |v[B]| .. |v[E-1]| with multiplicity, by a
// merge tree (the two values are unique, so the tree's shape changes nothing):
// leaves are pairs (min, max) or a single value (hi = none)
struct Top2 {
    double lo, hi;
    bool has_hi;
};
template <int B, int E>
__device__ __forceinline__ Top2 top2(const double* v) {
    if constexpr (E - B == 1) {
        return Top2{fabs(v[B]), 0.0, false};
    } else if constexpr (E - B == 2) {
        return Top2{vmin_aa(v[B], v[B + 1]), vmax_aa(v[B], v[B + 1]), true};
    } else {
        constexpr int M = B + ((E - B) / 2 + 1) / 2 * 2;
        const Top2 a = top2<B, M>(v), b = top2<M, E>(v);
        Top2 r;
        r.lo = vmin(a.lo, b.lo);
        double h = vmax(a.lo, b.lo);
        if (a.has_hi && b.has_hi) h = vmin(h, vmin(a.hi, b.hi));
        else if (a.has_hi) h = vmin(h, a.hi);
        else if (b.has_hi) h = vmin(h, b.hi);
        r.hi = h;
        r.has_hi = true;
        return r;
    }
}

// one side (left: copy of B, right: copy of A) of a lane's shot
template <int SIDE>
struct Side;
template <>
struct Side<0> {  // left lane x: checks y < b0 (rows of B), qubits z < b1
    static constexpr int NC = HG_B0, NQ = HG_B1, E = kBE;
    __device__ static constexpr int rp(int c) { return kBrp[c]; }
    __device__ static constexpr int cp(int q) { return kBcp[q]; }
    __device__ static constexpr int ce(int t) { return kBce[t]; }
    __device__ static constexpr u64 rm(int c) { return kBrm[c]; }
    __device__ static constexpr int row(int e) { return kBer[e]; }
};
template <>
struct Side<1> {  // right lane y: checks x < a0 (rows of A), qubits w < a1
    static constexpr int NC = HG_A0, NQ = HG_A1, E = kAE;
    __device__ static constexpr int rp(int c) { return kArp[c]; }
    __device__ static constexpr int cp(int q) { return kAcp[q]; }
    __device__ static constexpr int ce(int t) { return kAce[t]; }
    __device__ static constexpr u64 rm(int c) { return kArm[c]; }
    __device__ static constexpr int row(int e) { return kAer[e]; }
};

struct HgArgs {
    const u8* syn;          // [B][m]
    const double* prior;    // [n] min-sum prior per column
    u8* x_out;              // [B][n] or null
    int* iters;             // [B] or null
    u8* status;             // [B] or null (bit 0: BP converged)
    u64* counter;           // shot counter (zeroed by the launcher)
    i64 B;
    int max_iter;
    double ms_scaling;
};

struct HgLds {
    double2 pl[HG_S * HG_A0 * HG_B0];  // left halves' partial states, check (s, x, y)
    double2 pr[HG_S * HG_A0 * HG_B0];  // right halves'
    u32 xr[HG_S * HG_B0];              // right lane (s, y): parity of its decision per check x (bit x)
    u32 bad[2][HG_S];                  // by step parity: some check of slot s unsatisfied
    i64 shot[HG_S];                    // slot s's shot (>= B: slot idle)
};

template <int SIDE>
__device__ __forceinline__ void hg_lane(const HgArgs& a, HgLds& L, int s, int ix, bool idle) {
    using S_ = Side<SIDE>;
    constexpr int NC = S_::NC, NQ = S_::NQ, E = S_::E;
    const int m = HG_A0 * HG_B0, n = HG_A0 * HG_B1 + HG_A1 * HG_B0;
    // column of qubit q of this copy, and the check of local check c
    auto col = [&](int q) { return SIDE == 0 ? ix * HG_B1 + q : HG_A0 * HG_B1 + q * HG_B0 + ix; };
    auto chk = [&](int c) { return SIDE == 0 ? ix * HG_B0 + c : c * HG_B0 + ix; };
    // LDS index of check c's partial: (s, x, y)
    auto pidx = [&](int c) { return (s * HG_A0 + (SIDE == 0 ? ix : c)) * HG_B0 + (SIDE == 0 ? c : ix); };
    double2* mine = SIDE == 0 ? L.pl : L.pr;
    const double2* other = SIDE == 0 ? L.pr : L.pl;

    double pri[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) pri[q] = idle ? 0.0 : a.prior[col(q)];
    double v[E];       // v2c messages, by edge (rows of this copy's matrix)
    u32 sb = 0;        // syndrome bits of the own checks (left lanes only use them)
    u32 xm = 0;        // hard decision of the own qubits (bit q)
    int it = 0;
    i64 shot = idle ? a.B : L.shot[s];
    bool live = shot < a.B;
    auto start = [&]() {
        sfor<0, NQ>([&](auto qi) {
            constexpr int q = decltype(qi)::value;
#pragma unroll
            for (int t = S_::cp(q); t < S_::cp(q + 1); ++t) v[S_::ce(t)] = pri[q];
        });
        sb = 0;
        if (SIDE == 0)
#pragma unroll
            for (int c = 0; c < NC; ++c) sb |= (u32)(a.syn[shot * m + chk(c)] & 1) << c;
        it = 0;
        xm = 0;
    };
    if (live) start();
    int step = 0;
    for (;;) {
        // ---- A: test of the previous decision; partial states of v
        const int sp = step & 1;
        if (SIDE == 0 && ix == 0 && !idle) L.bad[sp ^ 1][s] = 0u;  // set next step (readers done: last step's B)
        if (live) {
            if (SIDE == 0 && it > 0) {
                u32 badc = 0;
#pragma unroll
                for (int c = 0; c < NC; ++c) {
                    const u32 own = (u32)__builtin_popcountll(S_::rm(c) & (u64)xm) & 1u;
                    const u32 oth = (L.xr[s * HG_B0 + c] >> ix) & 1u;
                    badc |= (own ^ oth ^ (sb >> c)) & 1u;
                }
                if (badc) atomicOr(&L.bad[sp][s], 1u);
            }
            sfor<0, NC>([&](auto ci) {
                constexpr int c = decltype(ci)::value;
                constexpr int e0 = S_::rp(c), e1 = S_::rp(c + 1);
                double m1 = kBig, m2 = kBig;
                if constexpr (e1 > e0) {
                    const Top2 t = top2<e0, e1>(v);
                    m1 = t.lo;
                    if (t.has_hi) m2 = t.hi;
                }
                u32 hx = (SIDE == 0 && ((sb >> c) & 1u)) ? 0x80000000u : 0u;
#pragma unroll
                for (int e = e0; e < e1; ++e) hx ^= hi32(v[e]);
                u32 hz = 0;  // bit 31: the half holds a +0 entry
                if (m1 == 0.0) {  // rare: parity by ldpc's compares, +0 flag
                    u32 par = (SIDE == 0) ? ((sb >> c) & 1u) : 0u;
#pragma unroll
                    for (int e = e0; e < e1; ++e) {
                        par ^= v[e] <= 0.0 ? 1u : 0u;
                        hz |= __double_as_longlong(v[e]) == 0ll ? 0x80000000u : 0u;
                    }
                    hx = par << 31;
                }
                mine[pidx(c)] = make_double2(with_sign(m1, hx), with_sign(m2, hz));
            });
        }
        __syncthreads();
        // ---- B: end of a shot, or one iteration
        bool fin = false;
        if (live) {
            const bool conv = it > 0 && L.bad[sp][s] == 0u;
            if (conv || it == a.max_iter) {
                fin = true;
                if (a.x_out)
#pragma unroll
                    for (int q = 0; q < NQ; ++q) a.x_out[shot * n + col(q)] = (u8)((xm >> q) & 1u);
                if (SIDE == 0 && ix == 0) {
                    if (a.iters) a.iters[shot] = conv ? it : a.max_iter;
                    if (a.status) a.status[shot] = conv ? 1 : 0;
                    L.shot[s] = (i64)atomicAdd(a.counter, 1ull);
                }
            } else {
                ++it;
                const double alpha = alpha_at(it, a.ms_scaling);
                // full states of the own checks: s1 = M1 with the parity's sign, s2 = M2
                // with parity ^ (+0 present) (M1, M2: the smaller two of both halves)
                double s1[NC], s2[NC];
                sfor<0, NC>([&](auto ci) {
                    constexpr int c = decltype(ci)::value;
                    const double2 pm = mine[pidx(c)];
                    const double2 po = other[pidx(c)];
                    const double M1 = vmin_aa(pm.x, po.x);
                    const double M2 = vmin(vmax_aa(pm.x, po.x), vmin_aa(pm.y, po.y));
                    const u32 par = hi32(pm.x) ^ hi32(po.x);
                    const u32 pz = hi32(pm.y) | hi32(po.y);
                    s1[c] = with_sign(M1, par);
                    s2[c] = with_sign(M2, par ^ pz);
                });
                // per qubit: c2v of its edges (alpha * (|v| == M1 ? M2 : M1), sign by
                // the state ^ v's sign bit), then ldpc's sums in ascending check
                // order; each edge's v is read before it is replaced
                xm = 0;
                sfor<0, NQ>([&](auto qi) {
                    constexpr int q = decltype(qi)::value;
                    constexpr int t0 = S_::cp(q), K = S_::cp(q + 1) - t0;
                    double c[K > 0 ? K : 1], pre[K > 0 ? K : 1];
                    double acc = pri[q];
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const int e = S_::ce(t0 + k), r = S_::row(e);
                        const double y = fabs(v[e]) == fabs(s1[r]) ? s2[r] : s1[r];
                        c[k] = xor_sign(y * alpha, hi32(v[e]));
                        pre[k] = acc;
                        acc += c[k];
                    }
                    xm |= (acc <= 0.0 ? 1u : 0u) << q;
                    double suf = 0.0;
#pragma unroll
                    for (int k = K - 1; k >= 0; --k) {
                        const double out = (k == K - 1) ? pre[k] : pre[k] + suf;
                        suf = (k == K - 1) ? c[k] : suf + c[k];
                        v[S_::ce(t0 + k)] = out;
                    }
                });
                if (SIDE == 1) {  // the decision's parity per own check, for the left lanes' test
                    u32 xp = 0;
#pragma unroll
                    for (int c = 0; c < NC; ++c) xp |= ((u32)__builtin_popcountll(S_::rm(c) & (u64)xm) & 1u) << c;  // (masks: constexpr)
                    L.xr[s * HG_B0 + ix] = xp;
                }
            }
        }
        const bool any = __syncthreads_or(live ? 1 : 0);
        if (!any) break;
        if (fin) {  // the slot's next shot (written by its leader before the barrier)
            shot = L.shot[s];
            live = shot < a.B;
            if (live) start();
        }
        ++step;
    }
}

extern "C" __global__ __launch_bounds__(HG_THREADS) void hgp_bp_ms_f64(HgArgs a) {
    __shared__ HgLds L;
    const int tid = threadIdx.x;
    if (tid < HG_S) L.shot[tid] = (i64)atomicAdd(a.counter, 1ull);
    if (tid < 2 * HG_S) (&L.bad[0][0])[tid] = 0u;
    __syncthreads();
    const int LW = 64 * HG_WL;
    // every wave runs one side's code (waves < HG_WL left); lanes past the S
    // slots run it idle, so every wave meets the same barriers
    if (tid < LW) {
        const int s = tid / HG_A0, x = tid % HG_A0;
        hg_lane<0>(a, L, s < HG_S ? s : 0, x, s >= HG_S);
    } else {
        const int r = tid - LW;
        const int s = r / HG_B0, y = r % HG_B0;
        hg_lane<1>(a, L, s < HG_S ? s : 0, y, s >= HG_S);
    }
}
