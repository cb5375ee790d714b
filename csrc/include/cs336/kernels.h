// Host-side launchers of the cs336 HIP kernels. These take raw device pointers + a HIP stream and
// have no PyTorch dependency; csrc/bindings.cpp adapts them to torch.ops.cs336.*.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace cs336 {

// ---- RMSNorm (csrc/ops/rmsnorm.hip) ----
void rmsnorm_fwd(const void* x, DType xt, const void* w, DType wt, void* y, DType yt, float* rstd, int64_t M,
                 int64_t H, float eps, hipStream_t s);
// dx (dtype xt); dw (fp32, H) via a (rows x H) fp32 workspace of per-workgroup partials
void rmsnorm_bwd(const void* dy, DType dyt, const void* x, DType xt, const void* w, DType wt, const float* rstd,
                 void* dx, float* dw, float* workspace, int64_t M, int64_t H, hipStream_t s);
int rmsnorm_bwd_workspace_rows(int64_t M, int64_t H);
// fused pre-norm residual: sum = x + r (dtype xt), y = rmsnorm(sum) * w; xt/rt/yt in {F32, BF16}
void add_rmsnorm_fwd(const void* x, DType xt, const void* r, DType rt, const float* w, void* y, DType yt, void* sum,
                     float* rstd, int64_t M, int64_t H, float eps, hipStream_t s);
// dx = rmsnorm_bwd(dy) + dres (dtype xt, dres same dtype); dx_bf16 (optional) = bf16 copy of dx
// rmsnorm_bwd_add that also writes the bf16 result transposed (dxt: H x M, ld M); M % rows == 0
int rmsnorm_bwd_add_t_rows(int64_t H);
int rmsnorm_bwd_add_t_workspace_rows(int64_t M, int64_t H);
void rmsnorm_bwd_add_t(const void* dy, DType dyt, const void* x, DType xt, const float* w, const float* rstd,
                       const void* dres, void* dx, void* dx_bf16, void* dxt, float* dw, float* workspace, int64_t M,
                       int64_t H, hipStream_t s);
void rmsnorm_bwd_add(const void* dy, DType dyt, const void* x, DType xt, const float* w, const float* rstd,
                     const void* dres, void* dx, void* dx_bf16, float* dw, float* workspace, int64_t M, int64_t H,
                     hipStream_t s);

// ---- 2-byte transpose (csrc/ops/transpose.hip): out[c][r] = in[r][c]; R, C multiples of 8,
// 16-B aligned rows
void transpose16(const void* in, int64_t ld_in, void* out, int64_t ld_out, int R, int C, hipStream_t s);
// fp32 [R][C] -> bf16 w [R][C] and its transpose wt [C][R] in one pass (R, C multiples of 8, 16-B rows)
void cast_transpose_bf16(const float* in, int64_t ld_in, void* w, int64_t ld_w, void* wt, int64_t ld_t, int R, int C,
                         hipStream_t s);

// ---- diagnostics (csrc/ops/occupy.hip): n_workgroups x 256 threads, each holding lds_bytes of LDS,
// spin for `ms` of wall-clock time, then atomically increment *done
void occupy(int n_workgroups, int lds_bytes, double ms, int* done, hipStream_t s);
// the same, moving `total_bytes` (half read from src, half written to dst, both nbytes long, cycled)
// paced over `ms` -- the per-rank HBM traffic of a ring all-reduce (scripts/comm_emulation.py)
void occupy_bytes(int n_workgroups, int lds_bytes, double ms, const void* src, void* dst, int64_t nbytes,
                  int64_t total_bytes, int* done, hipStream_t s);
// co-residency probe: n_workgroups that each wait (up to deadline_ms) until all of them have arrived;
// state[0] arrivals (reset per launch), state[1] += workgroups that timed out, state[2] = max wait
// in 100 MHz ticks
void cohort(int n_workgroups, int lds_bytes, double deadline_ms, int* state, hipStream_t s);

// ---- bf16 MFMA GEMM (csrc/gemm/gemm.hip) ----
// C[M][N] = Σ_k A(m,k) B(k,n); A(m,k) = a[m·lda+k] (K-major) or a[k·lda+m]; B(k,n) = b[n·ldb+k]
// (K-major) or b[k·ldb+n]. out_mode 0: bf16 C, 1: fp32 C, 2: fp32 C += . splits > 1: fp32 slabs
// at c + s·split_stride (out_mode 1), summed by splitk_reduce.
struct GemmArgs {
  const bf16_t* a;
  const bf16_t* b;
  void* c;
  int64_t lda, ldb, ldc, split_stride;
  int M, N, K;
};
namespace gemm {
bool tile_supported(int bm, int bn);
bool gemm_bf16(const GemmArgs& p, int bm, int bn, bool a_kmajor, bool b_kmajor, int out_mode, int splits,
               hipStream_t s);
void splitk_reduce(const float* slabs, float* out, int64_t M, int64_t N, int nsplit, int64_t ld_out, bool accumulate,
                   hipStream_t s);
}  // namespace gemm

// ---- RoPE (csrc/ops/rope.hip) ----
// x: (B,H,N,D) strided (elements), out: contiguous (B,N,H,D); cos/sin: (ctx, D/2) fp32;
// pos: (B,N) int64 or nullptr (position = n).
struct RopeArgs {
  const void* x;
  int64_t x_sb, x_sh, x_sn;
  void* out;
  int64_t o_sb, o_sh, o_sn;
};
void rope(const RopeArgs& a, DType t, const float* cos_, const float* sin_, const int64_t* pos, int B, int H, int N,
          int D, bool inverse, hipStream_t s);

// ---- SwiGLU gate (csrc/ops/swiglu.hip) ----
// (M, F) elementwise; a/b/da/db rows at stride ld (elements), h/dh contiguous. M == 1 allows any F.
void silu_mul_fwd(const void* a, const void* b, void* h, DType t, int64_t M, int64_t F, int64_t ld, hipStream_t s);
void silu_mul_bwd(const void* dh, const void* a, const void* b, void* da, void* db, DType t, int64_t M, int64_t F,
                  int64_t ld, hipStream_t s);

// ---- token-embedding backward (csrc/ops/embedding.hip) ----
// gw[v][:] = sum of g[perm[i]][:] over the run of sorted_ids equal to v (in order); gw fp32 (V, D),
// every row written; g (n_tok, D) row-major; sorted_ids / perm from a stable sort of the ids; D % 4 == 0
void embedding_bwd(const void* g, DType gt, const int64_t* sorted_ids, const int64_t* perm, float* gw, int64_t n_tok,
                   int64_t V, int64_t D, hipStream_t s);

// ---- cross entropy (csrc/ops/xent.hip) ----
void xent_fwd(const void* z, DType t, const int64_t* tgt, float* loss, float* lse, int64_t M, int64_t V,
              hipStream_t s);
void xent_bwd(const float* g, const void* z, DType t, const int64_t* tgt, const float* lse, void* dz, float mult,
              int64_t M, int64_t V, hipStream_t s);

// ---- multi-tensor ops (csrc/ops/multi_tensor.hip) ----
struct TensorTable {
  // device arrays, n entries each
  const int64_t* ptrs;        // [n * nptr] pointers as int64
  const int64_t* chunk_base;  // [n + 1] prefix sum of chunks per tensor
  const int64_t* numel;       // [n]
  int n;
  int64_t total_chunks;
};
constexpr int64_t kMTChunk = 32768;  // elements per workgroup chunk

// scalars are rounded to fp32 from double exactly like the reference's Python-float * fp32-tensor ops
// table pointers per tensor: p, g, m, v (+ bf16 shadow when shadow == true)
// alpha_dev: when non-null, the step size lr·sqrt(1-b2^t)/(1-b1^t) is read from device memory (written
// by adamw_device_step) instead of alpha_t, so a HIP graph can replay the update on later steps
void adamw_step(const TensorTable& tt, DType grad_t, bool shadow, float beta1, float beta2, float one_minus_beta1,
                float one_minus_beta2, float eps, float lr_wd, float alpha_t, const float* alpha_dev, hipStream_t s);
// 2-D weights, also writing the transposed bf16 shadow: per tensor 6 pointers (p, g, m, v, shadow,
// Wᵀ at its first element) and dims (R, C, ldt); tiles of 256 rows x 64 columns; R, C multiples of 8,
// every pointer 16-B aligned, ldt a multiple of 8 (host checks)
void adamw_step_t(const int64_t* ptrs, const int64_t* tile_base, const int64_t* dims, int n, int64_t total_tiles,
                  DType grad_t, float beta1, float beta2, float one_minus_beta1, float one_minus_beta2, float eps,
                  float lr_wd, float alpha_t, const float* alpha_dev, hipStream_t s);
// Device-side step counter of a captured optimizer step: t += 1, alpha = lr·sqrt(1-b2^t)/(1-b1^t)
// (double math, rounded to fp32 as the host computes alpha_t)
void adamw_device_step(int64_t* t, float* alpha, double lr, double beta1, double beta2, hipStream_t s);
// table pointers per tensor: fp32 src, bf16 dst
void multi_tensor_cast_bf16(const TensorTable& tt, hipStream_t s);
void multi_tensor_sumsq(const TensorTable& tt, DType t, float* partials, hipStream_t s);
void finalize_l2norm(const float* partials, int64_t n, float* out, hipStream_t s);
void multi_tensor_scale(const TensorTable& tt, DType t, const float* scale, hipStream_t s);

// ---- FlashAttention-2 (csrc/flash_attn/) ----
struct AttnParams {
  const void* q;
  const void* k;
  const void* v;
  void* o;
  float* lse;  // (B, H, Nq) contiguous
  // element strides for batch, head, seq (last dim contiguous)
  int64_t q_sb, q_sh, q_sn;
  int64_t k_sb, k_sh, k_sn;
  int64_t v_sb, v_sh, v_sn;
  int64_t o_sb, o_sh, o_sn;
  int B, H, Nq, Nk, D;
  float scale;
  bool causal;
  // optional fused RoPE on q and k (self-attention, Nq == Nk): cos/sin (ctx, D/2) fp32, positions
  // (B, N) int64 or nullptr (= index). q/k are the UN-rotated projections; dq/dk come out un-rotated.
  const float* rope_cos = nullptr;
  const float* rope_sin = nullptr;
  const int64_t* rope_pos = nullptr;
  // backward only: q/k are ALREADY rotated (the model's separate RoPE pass); dq/dk are still
  // returned w.r.t. the un-rotated inputs (inverse rotation fused into their store)
  int rope_out_only = 0;
  // block dispatch order under the causal mask: 0 = per-(batch, head) interleaved, 1 = heaviest tile
  // level first within each XCD's heads (longest-processing-time order, see tile_order in fa_common.h)
  int order = 1;
  int lpt_group = 1 << 20;  // heads per level-major group (sized by the host to the L2, fill_attn)
  // tile staging by buffer_load ... lds (16-bit, no RoPE-on-load) instead of through VGPRs: bit 0 the
  // forward's K/V tiles, bit 1 the backward's K/V (dQ) and Q/dO (dK/dV) tiles (CS336_FA_DMA, fill_attn)
  int dma = 1;
  // optional transposed copy of O for the output projection's weight gradient: element (b, h, n, d)
  // also goes to ot[(h * D + d) * ot_ld + b * Nq + n] (token-contiguous rows, ot_ld = B * Nq)
  void* ot = nullptr;
  int64_t ot_ld = 0;
  // forward split over the keys (low parallelism: few heads x few query blocks): kv_splits > 1
  // workgroups per query block, each over one contiguous range of key tiles, write a normalized fp32
  // partial O (opart [split][B·H][Nq][D]) and its natural-log LSE (lpart [split][B·H][Nq]); a merge
  // kernel combines them into o and lse (flash_attn_fwd)
  int kv_splits = 1;
  float* opart = nullptr;
  float* lpart = nullptr;
};

struct AttnBwdParams {
  AttnParams f;  // q,k,v,o,lse + strides (o is read)
  const void* dout;
  int64_t do_sb, do_sh, do_sn;
  void* dq;
  void* dk;
  void* dv;
  int64_t dq_sb, dq_sh, dq_sn;
  int64_t dk_sb, dk_sh, dk_sn;
  int64_t dv_sb, dv_sh, dv_sn;
  // (B, H, Nq) workspaces written by the dQ kernel for the dK/dV kernel: the row constants
  // -delta (delta = rowsum(dO * O)) and -lse / scale, loaded as the initial dP and S accumulators
  float* delta;
  float* lrow;
  // fp32 (B, H, Nq, 64) dQ partial sums of the fused head-sequential backward (fa_bwd_fused.hip)
  float* dq_acc = nullptr;
  // two-kernel form at low parallelism (flash_attn_bwd_splits): the dQ kernel split over key ranges
  // (ksplit) and the dK/dV kernel over query ranges (qsplit); each split writes unscaled fp32
  // partials ([split][B·H][N][D] slabs) that a reduce kernel sums, scales, rotates back and casts
  int ksplit = 1, qsplit = 1;
  float* dq_part = nullptr;
  float* dk_part = nullptr;
  float* dv_part = nullptr;
};

void flash_attn_fwd(const AttnParams& p, DType t, hipStream_t s);
// key splits the forward uses for p (1 = none) and the fp32 workspace they need (floats)
int flash_attn_fwd_splits(const AttnParams& p);
size_t flash_attn_fwd_split_workspace(const AttnParams& p, int splits);
void flash_attn_bwd(const AttnBwdParams& p, DType t, hipStream_t s);
// (ksplit, qsplit) the two-kernel backward uses for p at low parallelism, and their fp32 workspace
void flash_attn_bwd_splits(const AttnBwdParams& p, int& ksplit, int& qsplit);
size_t flash_attn_bwd_split_workspace(const AttnBwdParams& p, int ksplit, int qsplit);
// one-kernel backward, one workgroup per (batch, head): 16-bit, d 64, Nq == Nk, N % 64 == 0, N <= 1024
bool flash_attn_bwd_fused_ok(const AttnBwdParams& p, DType t);
void flash_attn_bwd_fused(const AttnBwdParams& p, DType t, hipStream_t s);
// one-kernel backward, one workgroup per 256-key block, dQ by fp32 atomics (fa_bwd_kp.hip): 16-bit,
// d 64 / 80, Nq == Nk, N % 64 == 0; ws = flash_attn_bwd_kp_workspace(p) floats
bool flash_attn_bwd_kp_ok(const AttnBwdParams& p, DType t);
size_t flash_attn_bwd_kp_workspace(const AttnBwdParams& p);
void flash_attn_bwd_kp(const AttnBwdParams& p, DType t, float* ws, hipStream_t s);
// one-kernel backward, one 4-wave workgroup per (batch, head) over 128-key blocks, two workgroups per
// CU (fa_bwd_hs.hip): 16-bit, d 64, Nq == Nk, N % 128 == 0; ws = flash_attn_bwd_hs_workspace(p) floats
bool flash_attn_bwd_hs_ok(const AttnBwdParams& p, DType t);
size_t flash_attn_bwd_hs_workspace(const AttnBwdParams& p);
// rope_dq = false (with RoPE): only dK is rotated back in the kernel; the caller rotates dQ
void flash_attn_bwd_hs(const AttnBwdParams& p, DType t, float* ws, hipStream_t s, bool rope_dq = true);

}  // namespace cs336
