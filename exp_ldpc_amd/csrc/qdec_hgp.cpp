// qdec_hgp.cpp -- host side of the hypergraph-product BP kernel
// (qdec_hgp_kernel.hip): recognise H = [I_a0 (x) B | A (x) I_b0] (hgp.py
// homological_product's Z checks), generate the kernel's compile-time tables,
// compile it for the device with hipRTC, launch it.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include "qdec_internal.h"

namespace qdec {

static const char* kHgpKernelSrc =
#include "qdec_hgp_src.inc"
    ;

struct HgpPlan {
    int a0 = 0, a1 = 0, b0 = 0, b1 = 0;
    std::vector<std::vector<int>> A, B;  // rows: sorted column lists
    int S = 0, WL = 0, WR = 0;           // shot slots per workgroup, left / right waves
    std::string src;
    std::vector<char> code;  // gfx950 code object (hipRTC)
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;
    int per_cu = 0, grid = 0;
};

namespace {

bool rows_equal(const std::vector<int32_t>& rp, const std::vector<int32_t>& ci, int i, const std::vector<int>& want) {
    if (rp[i + 1] - rp[i] != (int)want.size()) return false;
    std::vector<int> got(ci.begin() + rp[i], ci.begin() + rp[i + 1]);
    std::sort(got.begin(), got.end());
    return got == want;
}

// H = [I_a0 (x) B | A (x) I_b0] with B b0 x b1, A a0 x a1: m = a0 b0, n = a0 b1 + a1 b0
bool factor(int m, int n, const std::vector<int32_t>& rp, const std::vector<int32_t>& ci, HgpPlan* P) {
    for (int a0 = 2; a0 <= m / 2; ++a0) {
        if (m % a0) continue;
        const int b0 = m / a0;
        for (int b1 = 1; a0 * b1 < n; ++b1) {
            const int rem = n - a0 * b1;
            if (rem % b0) continue;
            const int a1 = rem / b0;
            // B from the checks (0, y): their columns below b1; A from the checks (x, 0)
            std::vector<std::vector<int>> B(b0), A(a0);
            bool ok = true;
            for (int y = 0; y < b0 && ok; ++y)
                for (int e = rp[y]; e < rp[y + 1]; ++e) {
                    const int c = ci[e];
                    if (c < b1) B[y].push_back(c);
                    else if (c < a0 * b1) ok = false;
                }
            for (int x = 0; x < a0 && ok; ++x)
                for (int e = rp[x * b0]; e < rp[x * b0 + 1]; ++e) {
                    const int c = ci[e];
                    if (c < a0 * b1) continue;
                    const int r = c - a0 * b1;
                    if (r % b0 != 0) ok = false;
                    else A[x].push_back(r / b0);
                }
            if (!ok) continue;
            for (auto& r : B) std::sort(r.begin(), r.end());
            for (auto& r : A) std::sort(r.begin(), r.end());
            for (int x = 0; x < a0 && ok; ++x)
                for (int y = 0; y < b0 && ok; ++y) {
                    std::vector<int> want;
                    for (int z : B[y]) want.push_back(x * b1 + z);
                    for (int w : A[x]) want.push_back(a0 * b1 + w * b0 + y);
                    ok = rows_equal(rp, ci, x * b0 + y, want);
                }
            if (!ok) continue;
            P->a0 = a0, P->a1 = a1, P->b0 = b0, P->b1 = b1;
            P->A = std::move(A);
            P->B = std::move(B);
            return true;
        }
    }
    return false;
}

// edge tables of one factor M (rows x cols): rows' edges in row order; per column
// its edges in ascending row order; the row of each edge; row masks over columns
void emit_tables(std::ostringstream& o, const char* X, const std::vector<std::vector<int>>& M, int cols) {
    std::vector<int> rp(1, 0), ec, er;
    for (size_t r = 0; r < M.size(); ++r) {
        for (int c : M[r]) ec.push_back(c), er.push_back((int)r);
        rp.push_back((int)ec.size());
    }
    std::vector<int> cp(cols + 1, 0), ce;
    for (int c : ec) cp[c + 1]++;
    for (int c = 0; c < cols; ++c) cp[c + 1] += cp[c];
    ce.assign(ec.size(), 0);
    std::vector<int> f(cp.begin(), cp.end() - 1);
    for (size_t e = 0; e < ec.size(); ++e) ce[f[ec[e]]++] = (int)e;  // rows ascending: edges are in row order
    auto arr = [&](const char* name, const std::vector<int>& v) {
        o << "__device__ constexpr int k" << X << name << "[" << std::max<size_t>(v.size(), 1) << "] = {";
        for (size_t i = 0; i < v.size(); ++i) o << (i ? "," : "") << v[i];
        if (v.empty()) o << "0";
        o << "};\n";
    };
    o << "constexpr int k" << X << "E = " << ec.size() << ";\n";
    arr("rp", rp);
    arr("cp", cp);
    arr("ce", ce);
    arr("er", er);
    o << "__device__ constexpr unsigned long long k" << X << "rm[" << std::max<size_t>(M.size(), 1) << "] = {";
    for (size_t r = 0; r < M.size(); ++r) {
        unsigned long long mk = 0;
        for (int c : M[r]) mk |= 1ull << c;
        o << (r ? "," : "") << mk << "ull";
    }
    if (M.empty()) o << "0ull";
    o << "};\n";
}

}  // namespace

HgpPlan* hgp_plan_create(int m, int n, const std::vector<int32_t>& rp, const std::vector<int32_t>& ci, int slots) {
    HgpPlan* P = new HgpPlan;
    if (!factor(m, n, rp, ci, P)) {
        delete P;
        return nullptr;
    }
    // register budget: a copy's v2c messages (<= 48 edges) and decision / parity
    // masks in 32 bits (<= 32 qubits and checks per copy)
    const size_t eA = [&] { size_t s = 0; for (auto& r : P->A) s += r.size(); return s; }();
    const size_t eB = [&] { size_t s = 0; for (auto& r : P->B) s += r.size(); return s; }();
    if (eA > 48 || eB > 48 || P->a1 > 32 || P->b1 > 32 || P->a0 > 32 || P->b0 > 32) {
        delete P;
        return nullptr;
    }
    // slots per workgroup: the most lanes used per CU, at most 16 waves per
    // workgroup and 8 per CU (a lane's messages and check states take up to
    // 256 VGPRs: 2 waves per SIMD), the partial states in LDS
    int bestS = 0, bestW = 0;
    double best = 0;
    for (int S = 1; S <= 64; ++S) {
        const int WL = (S * P->a0 + 63) / 64, WR = (S * P->b0 + 63) / 64, W = WL + WR;
        if (W > 8) break;
        const size_t lds = (size_t)2 * S * m * 16 + (size_t)S * (P->b0 * 4 + 8 + 16) + 64;
        if (lds > 64 * 1024) break;
        const int per_cu = std::min(8 / W, (int)(160 * 1024 / lds));
        if (per_cu < 1) continue;
        const double used = (double)per_cu * S * (P->a0 + P->b0);
        if (slots > 0 ? S == slots : used > best * 1.0001) best = used, bestS = S, bestW = WL;
    }
    if (bestS == 0) {  // `slots` (or every S) fits no workgroup: no plan
        delete P;
        return nullptr;
    }
    P->S = bestS;
    P->WL = bestW;
    P->WR = (bestS * P->b0 + 63) / 64;
    std::ostringstream o;
    o << "// generated by qdec_hgp.cpp: H = [I_" << P->a0 << " (x) B | A (x) I_" << P->b0 << "]\n";
    o << "#define HG_A0 " << P->a0 << "\n#define HG_A1 " << P->a1 << "\n#define HG_B0 " << P->b0 << "\n#define HG_B1 "
      << P->b1 << "\n#define HG_S " << P->S << "\n#define HG_WL " << P->WL << "\n#define HG_WR " << P->WR << "\n";
    emit_tables(o, "B", P->B, P->b1);
    emit_tables(o, "A", P->A, P->a1);
    P->src = o.str() + kHgpKernelSrc;
    return P;
}

void hgp_plan_destroy(HgpPlan* P) {
    if (!P) return;
    if (P->mod) (void)hipModuleUnload(P->mod);
    delete P;
}

const std::string& hgp_plan_source(const HgpPlan* P) { return P->src; }

// development: run an edited source (QDEC_DEV_HOOKS builds, kernel debugging)
void hgp_plan_replace_source(HgpPlan* P, const std::string& src) {
    if (P->mod) (void)hipModuleUnload(P->mod);
    P->mod = nullptr;
    P->fn = nullptr;
    P->code.clear();
    P->src = src;
}

// hipRTC, with the library's numerics flags (build.py: no contraction, fp32
// denormals kept); code objects cached per source text (process-wide)
int hgp_plan_compile(HgpPlan* P, const char* arch, std::string* log) {
    static std::mutex mu;
    static std::vector<std::pair<std::string, std::vector<char>>> cache;
    const std::string key = std::string(arch) + "\n" + P->src;
    {
        std::lock_guard<std::mutex> lk(mu);
        for (auto& c : cache)
            if (c.first == key) {
                P->code = c.second;
                return 0;
            }
    }
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, P->src.c_str(), "qdec_hgp_kernel.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
        return -1;
    const std::string a = std::string("--offload-arch=") + arch;
    const char* opts[] = {a.c_str(), "-O3", "-std=c++17", "-ffp-contract=off", "-fno-gpu-flush-denormals-to-zero"};
    const hiprtcResult r = hiprtcCompileProgram(prog, 5, opts);
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    if (log && ls > 1) {
        log->resize(ls);
        hiprtcGetProgramLog(prog, &(*log)[0]);
    }
    if (r != HIPRTC_SUCCESS) {
        hiprtcDestroyProgram(&prog);
        return -2;
    }
    size_t cs = 0;
    hiprtcGetCodeSize(prog, &cs);
    P->code.resize(cs);
    hiprtcGetCode(prog, P->code.data());
    hiprtcDestroyProgram(&prog);
    std::lock_guard<std::mutex> lk(mu);
    if (cache.size() >= 8) cache.erase(cache.begin());
    cache.emplace_back(key, P->code);
    return 0;
}

// compile (if needed) and load on the current device
int hgp_plan_load(HgpPlan* P, int num_cus, const char* arch) {
    if (P->fn) return 0;
    if (P->code.empty()) {
        std::string log;
        if (int rc = hgp_plan_compile(P, arch, &log)) {
            std::fprintf(stderr, "qdec: HGP kernel compile failed (%d):\n%s\n", rc, log.c_str());
            return rc;
        }
    }
    if (hipModuleLoadData(&P->mod, P->code.data()) != hipSuccess) return -3;
    if (hipModuleGetFunction(&P->fn, P->mod, "hgp_bp_ms_f64") != hipSuccess) return -4;
    int per_cu = 0;
    const int threads = 64 * (P->WL + P->WR);
    if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, P->fn, threads, 0) != hipSuccess || per_cu < 1)
        return -5;
    P->per_cu = per_cu;
    P->grid = num_cus * per_cu;
    return 0;
}

int hgp_launch_bp(HgpPlan* P, const HgpBpArgs& args, hipStream_t stream) {
    if (!P->fn) return -6;
    HgpBpArgs a = args;
    void* params[] = {&a};
    if (hipMemsetAsync(a.counter, 0, 8, stream) != hipSuccess) return -7;
    const int threads = 64 * (P->WL + P->WR);
    const long long need = (a.B + P->S - 1) / P->S;
    const unsigned grid = (unsigned)std::max<long long>(1, std::min<long long>(P->grid, need));
    if (hipModuleLaunchKernel(P->fn, grid, 1, 1, threads, 1, 1, 0, stream, params, nullptr) != hipSuccess) return -8;
    return 0;
}

// the hipRTC target: the device's own gfx name without its feature suffix
// (gcnArchName "gfx950:sramecc+:xnack-" -> "gfx950"); device < 0 (host-only
// handles) or no device: the architecture the library itself was built for
std::string hgp_target_arch(int device) {
    if (device >= 0) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.gcnArchName[0]) {
            std::string a(prop.gcnArchName);
            return a.substr(0, a.find(':'));
        }
        (void)hipGetLastError();
    }
    return QDEC_ARCH;
}

void hgp_plan_info(const HgpPlan* P, int* out8) {
    out8[0] = P->a0, out8[1] = P->a1, out8[2] = P->b0, out8[3] = P->b1;
    out8[4] = P->S, out8[5] = P->WL, out8[6] = P->WR, out8[7] = P->per_cu;
}

}  // namespace qdec
