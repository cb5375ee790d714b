// Autotuned hipBLASLt GEMM for the projection GEMMs (host code only; the kernels are hipBLASLt's
// Tensile/asm kernels for gfx950).
//
// torch.mm asks hipBLASLt's heuristic for ONE algorithm and runs it. For the XL weight-gradient
// shapes (dYᵀ·X, fp32 output, K = 12288 tokens) that first pick is a 128x128 macro-tile grid without
// split-K that leaves the chip a third idle on the 1600x1600 o-proj dW (0.47 PF in situ,
// profiles/r1_xl_step_breakdown_serial.txt). PyTorch's TunableOp does not cover the fp32-output
// GEMM. Here we take the heuristic's top-N candidates for the exact problem (shape, transposes,
// leading dimensions, output dtype), time each once on the current stream with HIP events, and
// cache the fastest per problem key. Later calls (and HIP-graph captures) reuse the cached
// algorithm; a capture that meets an untuned key uses the heuristic's first pick instead of timing.
//
// Row-major -> column-major: hipBLASLt is column-major. A row-major out[M][N] (row stride ldo) is the
// column-major matrix outᵀ (N x M, ld ldo), and outᵀ = op(b)ᵀ·op(a)ᵀ, so hipBLASLt's A is our b and its
// B is our a, each with the transpose flag that turns its row-major storage into the needed operand.
//
//   out = op(a) · op(b);  op(a): M x K (a stored K x M when a_t),  op(b): K x N (b stored N x K when b_t)
//
// Only beta = 0 (overwrite) -- the weight gradients are written straight into their DDP bucket slot.
//
// flags & kNoStreamK: only non-stream-K solutions. hipBLASLt's default picks for the projection
// GEMMs are stream-K Tensile kernels ("SK3" in the kernel name): a grid of at most one workgroup
// per CU (124 KB of LDS each), where a workgroup that owns a split tile spins on a workspace flag
// that the NEXT-indexed workgroup sets when its partial sum is written (label_SK_Fixup in the
// disassembly, profiles/r2_streamk_hang.md). That is only deadlock-free while the whole grid is
// co-resident. Two such GEMMs on two streams need ~2x256 slots of a 256-slot chip: each kernel's
// resident workgroups wait for its own undispatched successors and neither can finish -- the
// round-1 hang of the 2.7b step with weight-gradient GEMMs on a side stream. GEMMs that may run
// concurrently with another GEMM therefore use data-parallel (SK0) solutions.

#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <ATen/hip/HIPContextLight.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt-ext.hpp>
#include <hipblaslt/hipblaslt.h>
#include <torch/library.h>

#include "cs336/tensile_names.h"

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

namespace {

using cs336::macro_tile_area;
using cs336::stream_k_mode;

#define LT_CHECK(expr)                                                                          \
  do {                                                                                          \
    hipblasStatus_t _s = (expr);                                                                \
    TORCH_CHECK(_s == HIPBLAS_STATUS_SUCCESS, "hipBLASLt error ", int(_s), " at " #expr);       \
  } while (0)

constexpr int64_t kNoStreamK = 1;

struct Key {
  int64_t m, n, k, lda, ldb, ldo;
  bool a_t, b_t;
  int out;  // hipDataType of the output
  int dev;
  int64_t flags;
  bool operator==(const Key& o) const {
    return m == o.m && n == o.n && k == o.k && lda == o.lda && ldb == o.ldb && ldo == o.ldo && a_t == o.a_t &&
           b_t == o.b_t && out == o.out && dev == o.dev && flags == o.flags;
  }
};

struct KeyHash {
  size_t operator()(const Key& k) const {
    size_t h = 1469598103934665603ull;
    for (int64_t v : {k.m, k.n, k.k, k.lda, k.ldb, k.ldo, int64_t(k.a_t), int64_t(k.b_t), int64_t(k.out), int64_t(k.dev),
                      k.flags})
      h = (h ^ size_t(v)) * 1099511628211ull;
    return h;
  }
};

// Descriptors are cheap but not free (~µs); keep one set per problem alongside the chosen algorithm.
struct Plan {
  hipblasLtMatmulDesc_t op = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lo = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  size_t ws = 0;
  bool tuned = false;
  float best_us = 0.f, first_us = 0.f;
  int n_cand = 0, best_idx = 0;
  std::string kernel;  // Tensile kernel name of the chosen algorithm
};

std::string kernel_name(hipblasLtHandle_t h, hipblasLtMatmulAlgo_t& algo) {
  try {
    return hipblaslt_ext::getKernelNameFromAlgo(h, algo);
  } catch (...) {
    return std::string();
  }
}

std::mutex g_mu;
std::unordered_map<Key, Plan, KeyHash> g_plans;

// Committed picks (cs336_systems/tuning/gemm_table_mi355x.json "lt_pins"): problem -> index into the
// heuristic's candidate list + that candidate's kernel name. A pinned problem takes its candidate
// without timing (same kernel on every rank and box); a stale pin (name mismatch: another hipBLASLt)
// is ignored. g_no_timing (multi-rank jobs): an unpinned problem takes the heuristic's first choice
// instead of timing candidates inside a DDP backward, beside in-flight all-reduces.
struct PinKey {
  int64_t m, n, k;
  bool a_t, b_t;
  int out;
  bool operator==(const PinKey& o) const {
    return m == o.m && n == o.n && k == o.k && a_t == o.a_t && b_t == o.b_t && out == o.out;
  }
};
struct PinHash {
  size_t operator()(const PinKey& k) const {
    return std::hash<int64_t>()(k.m * 1000003 + k.n * 10007 + k.k) ^ (size_t(k.a_t) << 1) ^ (size_t(k.b_t) << 2) ^
           (size_t(k.out) << 3);
  }
};
std::unordered_map<PinKey, std::pair<int, std::string>, PinHash> g_pins;
bool g_no_timing = false;

int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return v && *v ? std::atoi(v) : dflt;
}

Plan make_plan(const Key& k) {
  Plan p;
  const hipDataType in_t = HIP_R_16BF, out_t = hipDataType(k.out);
  LT_CHECK(hipblasLtMatmulDescCreate(&p.op, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  // hipBLASLt A = our b, B = our a (see header comment).
  hipblasOperation_t ta = k.b_t ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  hipblasOperation_t tb = k.a_t ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  LT_CHECK(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  LT_CHECK(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  // Stored (column-major) shapes: A' = b is (N x K) when !b_t else (K x N); B' = a is (K x M) when !a_t else (M x K).
  LT_CHECK(hipblasLtMatrixLayoutCreate(&p.la, in_t, k.b_t ? k.k : k.n, k.b_t ? k.n : k.k, k.ldb));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&p.lb, in_t, k.a_t ? k.m : k.k, k.a_t ? k.k : k.m, k.lda));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&p.lo, out_t, k.n, k.m, k.ldo));
  return p;
}

hipblasStatus_t launch(hipblasLtHandle_t h, Plan& p, const hipblasLtMatmulAlgo_t* algo, const void* a, const void* b,
                       void* out, void* ws, size_t ws_bytes, hipStream_t s) {
  const float alpha = 1.f, beta = 0.f;
  return hipblasLtMatmul(h, p.op, &alpha, b, p.la, a, p.lb, &beta, out, p.lo, out, p.lo, algo, ws, ws_bytes, s);
}

void run(hipblasLtHandle_t h, Plan& p, const hipblasLtMatmulAlgo_t* algo, const void* a, const void* b, void* out,
         void* ws, size_t ws_bytes, hipStream_t s) {
  LT_CHECK(launch(h, p, algo, a, b, out, ws, ws_bytes, s));
}

// The heuristic's top candidates for the big projection GEMMs are all stream-K; enumerate every
// solution of the problem type instead and keep the supported data-parallel ones, largest macro
// tiles first (these GEMMs are large), at most CS336_LT_DP_CANDIDATES of them for timing.
void all_data_parallel(hipblasLtHandle_t h, Plan& p, const Key& k, size_t ws_bytes,
                       std::vector<hipblasLtMatmulHeuristicResult_t>& res, std::vector<std::string>& names) {
  std::vector<hipblasLtMatmulHeuristicResult_t> cands;
  const hipblasOperation_t ta = k.b_t ? HIPBLAS_OP_T : HIPBLAS_OP_N, tb = k.a_t ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  LT_CHECK(hipblaslt_ext::getAllAlgos(h, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, ta, tb, HIP_R_16BF, HIP_R_16BF,
                                      hipDataType(k.out), hipDataType(k.out), HIPBLAS_COMPUTE_32F, cands));
  const float alpha = 1.f, beta = 0.f;
  std::vector<std::tuple<int64_t, size_t>> keep;  // (tile area, index)
  std::vector<std::string> cn(cands.size());
  for (size_t i = 0; i < cands.size(); ++i) {
    cn[i] = kernel_name(h, cands[i].algo);
    if (cn[i].empty() || stream_k_mode(cn[i]) != 0) continue;
    size_t ws = 0;
    if (hipblaslt_ext::matmulIsAlgoSupported(h, p.op, &alpha, p.la, p.lb, &beta, p.lo, p.lo, cands[i].algo, ws) !=
            HIPBLAS_STATUS_SUCCESS ||
        ws > ws_bytes)
      continue;
    cands[i].workspaceSize = ws;
    cands[i].state = HIPBLAS_STATUS_SUCCESS;
    keep.emplace_back(macro_tile_area(cn[i]), i);
  }
  std::stable_sort(keep.begin(), keep.end(), [](const auto& x, const auto& y) { return std::get<0>(x) > std::get<0>(y); });
  if (env_int("CS336_LT_VERBOSE", 0)) {
    int n_sk = 0, n_unnamed = 0;
    for (const auto& nm : cn) n_unnamed += nm.empty(), n_sk += !nm.empty() && stream_k_mode(nm) != 0;
    std::fprintf(stderr, "[lt] %ldx%ldx%ld all-algos: %zu total, %d stream-K, %d unnamed, %zu data-parallel supported\n",
                 long(k.m), long(k.n), long(k.k), cands.size(), n_sk, n_unnamed, keep.size());
    for (size_t i = 0; i < cands.size() && i < 6; ++i) std::fprintf(stderr, "[lt]   e.g. %s\n", cn[i].c_str());
  }
  const size_t cap = size_t(std::max(1, env_int("CS336_LT_DP_CANDIDATES", 96)));
  for (size_t j = 0; j < keep.size() && j < cap; ++j) {
    res.push_back(cands[std::get<1>(keep[j])]);
    names.push_back(cn[std::get<1>(keep[j])]);
  }
}

void tune(hipblasLtHandle_t h, Plan& p, const Key& k, const void* a, const void* b, void* out, void* ws, size_t ws_bytes,
          hipStream_t s, bool capturing) {
  const bool really_capturing = capturing;
  hipblasLtMatmulPreference_t pref;
  LT_CHECK(hipblasLtMatmulPreferenceCreate(&pref));
  uint64_t wsb = ws_bytes;
  LT_CHECK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)));
  const bool no_sk = (k.flags & kNoStreamK) != 0;
  // (stream-K candidates are dropped below when no_sk: ask for more so data-parallel ones remain)
  const int want = no_sk ? std::max(64, env_int("CS336_LT_CANDIDATES", 48))
                         : (capturing ? 1 : std::max(1, env_int("CS336_LT_CANDIDATES", 48)));
  std::vector<hipblasLtMatmulHeuristicResult_t> all(want);
  int got_all = 0;
  LT_CHECK(hipblasLtMatmulAlgoGetHeuristic(h, p.op, p.la, p.lb, p.lo, p.lo, pref, want, all.data(), &got_all));
  hipblasLtMatmulPreferenceDestroy(pref);
  std::vector<hipblasLtMatmulHeuristicResult_t> res;
  std::vector<std::string> names;
  for (int i = 0; i < got_all; ++i) {
    std::string nm = kernel_name(h, all[i].algo);
    if (no_sk && (nm.empty() || stream_k_mode(nm) != 0)) continue;
    res.push_back(all[i]);
    names.push_back(std::move(nm));
  }
  if (no_sk && res.empty()) all_data_parallel(h, p, k, ws_bytes, res, names);
  const int got = int(res.size());
  TORCH_CHECK(got > 0, "hipBLASLt: no ", no_sk ? "data-parallel (non-stream-K) " : "", "algorithm for ", k.m, "x",
              k.n, "x", k.k, " among ", got_all, " candidates");
  p.n_cand = got;
  if (!no_sk) {
    auto pin = g_pins.find(PinKey{k.m, k.n, k.k, k.a_t, k.b_t, k.out});
    if (pin != g_pins.end() && pin->second.first < got && names[pin->second.first] == pin->second.second &&
        res[pin->second.first].workspaceSize <= ws_bytes) {
      const int i = pin->second.first;
      p.algo = res[i].algo;
      p.ws = res[i].workspaceSize;
      p.kernel = names[i];
      p.best_idx = i;
      p.tuned = true;
      return;
    }
    if (g_no_timing) capturing = true;  // heuristic first choice, marked tuned below
  }
  if (capturing || got == 1) {
    // Cannot time inside a capture: use the heuristic's first choice, retune on the next eager call.
    p.algo = res[0].algo;
    p.ws = res[0].workspaceSize;
    p.kernel = names[0];
    p.tuned = !really_capturing;
    return;
  }
  const int reps = std::max(1, env_int("CS336_LT_REPS", 5));
  const bool verbose = env_int("CS336_LT_VERBOSE", 0) != 0;
  hipEvent_t e0, e1;
  TORCH_CHECK(hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess);
  float best = 1e30f;
  int best_i = 0;
  p.first_us = 0.f;
  for (int i = 0; i < got; ++i) {
    if (res[i].state != HIPBLAS_STATUS_SUCCESS || res[i].workspaceSize > ws_bytes) continue;
    const hipblasLtMatmulAlgo_t* al = &res[i].algo;
    // warm (code object load, clocks); a candidate the library refuses at launch is skipped
    if (launch(h, p, al, a, b, out, ws, ws_bytes, s) != HIPBLAS_STATUS_SUCCESS) continue;
    TORCH_CHECK(hipEventRecord(e0, s) == hipSuccess);
    for (int r = 0; r < reps; ++r) run(h, p, al, a, b, out, ws, ws_bytes, s);
    TORCH_CHECK(hipEventRecord(e1, s) == hipSuccess && hipEventSynchronize(e1) == hipSuccess);
    float ms = 0.f;
    TORCH_CHECK(hipEventElapsedTime(&ms, e0, e1) == hipSuccess);
    const float us = 1000.f * ms / reps;
    if (p.first_us == 0.f) p.first_us = us;
    if (verbose)
      std::fprintf(stderr, "[lt] %ldx%ldx%ld a_t=%d b_t=%d out=%d cand %2d: %8.1f us  %6.1f TF  ws %zu  waves %.2f\n",
                   long(k.m), long(k.n), long(k.k), int(k.a_t), int(k.b_t), k.out, i, us,
                   2.0 * k.m * k.n * k.k / (us * 1e6), res[i].workspaceSize, res[i].wavesCount);
    if (us < best) best = us, best_i = i;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  p.algo = res[best_i].algo;
  p.ws = res[best_i].workspaceSize;
  p.kernel = names[best_i];
  p.best_us = best;
  p.best_idx = best_i;
  p.tuned = true;
  if (verbose)
    std::fprintf(stderr, "[lt] %ldx%ldx%ld -> cand %d (%.1f us, heuristic first %.1f us)\n", long(k.m), long(k.n),
                 long(k.k), best_i, best, p.first_us);
}

Plan* plan_for(const at::Tensor& a, const at::Tensor& b, bool a_t, bool b_t, const at::Tensor& out, int64_t flags,
               bool* empty);

void lt_gemm_out_ex(const at::Tensor& a, const at::Tensor& b, bool a_t, bool b_t, at::Tensor& out, int64_t flags) {
  bool empty = false;
  Plan* p = plan_for(a, b, a_t, b_t, out, flags, &empty);
  if (empty) return;
  hipblasLtHandle_t h = at::cuda::getCurrentCUDABlasLtHandle();
  run(h, *p, &p->algo, a.data_ptr(), b.data_ptr(), out.data_ptr(), at::cuda::getCUDABlasLtWorkspace(),
      at::cuda::getCUDABlasLtWorkspaceSize(), at::hip::getCurrentHIPStream());
}

void lt_gemm_out(const at::Tensor& a, const at::Tensor& b, bool a_t, bool b_t, at::Tensor& out) {
  lt_gemm_out_ex(a, b, a_t, b_t, out, 0);
}

// Kernel name of the plan the op would run for this problem (tunes it first if needed).
std::string lt_gemm_kernel(const at::Tensor& a, const at::Tensor& b, bool a_t, bool b_t, at::Tensor& out,
                           int64_t flags) {
  bool empty = false;
  Plan* p = plan_for(a, b, a_t, b_t, out, flags, &empty);
  return empty ? std::string() : p->kernel;
}

Plan* plan_for(const at::Tensor& a, const at::Tensor& b, bool a_t, bool b_t, const at::Tensor& out, int64_t flags,
               bool* empty) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && out.is_cuda(), "lt_gemm_out: CUDA tensors expected");
  TORCH_CHECK(a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16, "lt_gemm_out: bf16 operands");
  TORCH_CHECK(out.scalar_type() == at::kFloat || out.scalar_type() == at::kBFloat16, "lt_gemm_out: fp32/bf16 out");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && out.dim() == 2, "lt_gemm_out: 2-D tensors");
  TORCH_CHECK(a.stride(1) == 1 && b.stride(1) == 1 && out.stride(1) == 1, "lt_gemm_out: row-major (unit inner stride)");
  const int64_t M = a_t ? a.size(1) : a.size(0), K = a_t ? a.size(0) : a.size(1);
  const int64_t N = b_t ? b.size(0) : b.size(1), Kb = b_t ? b.size(1) : b.size(0);
  TORCH_CHECK(K == Kb && out.size(0) == M && out.size(1) == N, "lt_gemm_out: shape mismatch");
  if (M == 0 || N == 0) {
    *empty = true;
    return nullptr;
  }
  if (K == 0) {
    const_cast<at::Tensor&>(out).zero_();
    *empty = true;
    return nullptr;
  }
  const Key key{M, N, K, a.stride(0), b.stride(0), out.stride(0), a_t, b_t,
                int(out.scalar_type() == at::kFloat ? HIP_R_32F : HIP_R_16BF), a.get_device(), flags};
  hipStream_t s = at::hip::getCurrentHIPStream();
  hipblasLtHandle_t h = at::cuda::getCurrentCUDABlasLtHandle();
  void* ws = at::cuda::getCUDABlasLtWorkspace();
  const size_t ws_bytes = at::cuda::getCUDABlasLtWorkspaceSize();
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  TORCH_CHECK(hipStreamIsCapturing(s, &cs) == hipSuccess);
  const bool capturing = cs != hipStreamCaptureStatusNone;
  Plan* p;
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_plans.find(key);
    if (it == g_plans.end()) it = g_plans.emplace(key, make_plan(key)).first;
    p = &it->second;
    if (!p->tuned) tune(h, *p, key, a.data_ptr(), b.data_ptr(), out.data_ptr(), ws, ws_bytes, s, capturing);
  }
  return p;
}

at::Tensor lt_gemm_ex(const at::Tensor& a, const at::Tensor& b, bool a_t, bool b_t, at::ScalarType out_dtype,
                      int64_t flags) {
  const int64_t M = a_t ? a.size(1) : a.size(0), N = b_t ? b.size(0) : b.size(1);
  at::Tensor out = at::empty({M, N}, a.options().dtype(out_dtype));
  lt_gemm_out_ex(a, b, a_t, b_t, out, flags);
  return out;
}

at::Tensor lt_gemm(const at::Tensor& a, const at::Tensor& b, bool a_t, bool b_t, at::ScalarType out_dtype) {
  return lt_gemm_ex(a, b, a_t, b_t, out_dtype, 0);
}

// [m, n, k, a_t, b_t, out_dtype_code, n_candidates, best_index, best_ns, heuristic_first_ns] per tuned problem.
std::vector<int64_t> lt_gemm_table() {
  std::lock_guard<std::mutex> g(g_mu);
  std::vector<int64_t> t;
  for (auto& kv : g_plans) {
    const Key& k = kv.first;
    const Plan& p = kv.second;
    if (!p.tuned) continue;
    for (int64_t v : {k.m, k.n, k.k, int64_t(k.a_t), int64_t(k.b_t), int64_t(k.out), int64_t(p.n_cand),
                      int64_t(p.best_idx), int64_t(p.best_us * 1000.f), int64_t(p.first_us * 1000.f)})
      t.push_back(v);
  }
  return t;
}

void lt_gemm_pin(int64_t m, int64_t n, int64_t k, bool a_t, bool b_t, int64_t out_code, int64_t idx,
                 const std::string& kernel) {
  std::lock_guard<std::mutex> g(g_mu);
  g_pins[PinKey{m, n, k, a_t, b_t, int(out_code)}] = {int(idx), kernel};
}

void lt_gemm_set_no_timing(bool v) {
  std::lock_guard<std::mutex> g(g_mu);
  g_no_timing = v;
}

// "m,n,k,a_t,b_t,out,best_idx,kernel" per tuned problem (the pin list scripts/gemm_table.py commits)
std::vector<std::string> lt_gemm_picks() {
  std::lock_guard<std::mutex> g(g_mu);
  std::vector<std::string> r;
  for (auto& kv : g_plans) {
    const Key& k = kv.first;
    const Plan& p = kv.second;
    if (!p.tuned || (k.flags & kNoStreamK)) continue;
    r.push_back(std::to_string(k.m) + "," + std::to_string(k.n) + "," + std::to_string(k.k) + "," +
                std::to_string(int(k.a_t)) + "," + std::to_string(int(k.b_t)) + "," + std::to_string(k.out) + "," +
                std::to_string(p.best_idx) + "," + p.kernel);
  }
  return r;
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(cs336, m) {
  m.def("lt_gemm_pin(int m, int n, int k, bool a_t, bool b_t, int out_code, int idx, str kernel) -> ()", &lt_gemm_pin);
  m.def("lt_gemm_set_no_timing(bool v) -> ()", &lt_gemm_set_no_timing);
  m.def("lt_gemm_picks() -> str[]", &lt_gemm_picks);
  m.def("lt_gemm(Tensor a, Tensor b, bool a_t, bool b_t, ScalarType out_dtype) -> Tensor");
  m.def("lt_gemm_out(Tensor a, Tensor b, bool a_t, bool b_t, Tensor(a!) out) -> ()");
  m.def("lt_gemm_table() -> int[]", &lt_gemm_table);
  // flags: 1 = data-parallel (non-stream-K) solutions only (safe beside another GEMM on another stream)
  m.def("lt_gemm_ex(Tensor a, Tensor b, bool a_t, bool b_t, ScalarType out_dtype, int flags) -> Tensor");
  m.def("lt_gemm_out_ex(Tensor a, Tensor b, bool a_t, bool b_t, Tensor(a!) out, int flags) -> ()");
  m.def("lt_gemm_kernel(Tensor a, Tensor b, bool a_t, bool b_t, Tensor out, int flags) -> str");
  m.def("tensile_stream_k_mode(str kernel_name) -> int", [](const std::string& n) { return int64_t(stream_k_mode(n)); });
}

TORCH_LIBRARY_IMPL(cs336, CUDA, m) {
  m.impl("lt_gemm", &lt_gemm);
  m.impl("lt_gemm_out", &lt_gemm_out);
  m.impl("lt_gemm_ex", &lt_gemm_ex);
  m.impl("lt_gemm_out_ex", &lt_gemm_out_ex);
  m.impl("lt_gemm_kernel", &lt_gemm_kernel);
}
