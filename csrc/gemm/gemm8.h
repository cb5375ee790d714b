// Host interface of the NT projection GEMM with fused SwiGLU epilogues (csrc/gemm/gemm8.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cs336 {
namespace gemm8 {

// C = A · Bᵀ, A [M][K] and B [N][K] bf16 K-major (row strides lda, ldb), bf16 out.
// epi 0: C [M][N].
// epi 1 (W1|W3 forward): B = [W1; W3] (2·half rows), N = 2·half; writes y = C = [a|b] (ldc) and
//        h = silu(a)·b [M][half] (ldh).
// epi 2 (W2 input gradient): N = half; dh = A·Bᵀ is not stored; reads y = [a|b] (ldy) and writes
//        C = [da|db] [M][2·half] (ldc).
// epi 3 (QKV forward + RoPE): C [M][N] with columns < rope_cols rotated in interleaved pairs by
//        the fp32 (ctx, rdh/2) cos/sin tables at position rpos[row] (or row % rseq when rpos is null).
// Requires M % 256 == 0, K % 64 == 0, N % (64·fn) == 0 (epi 1: half % (32·fn) == 0), 16-B aligned
// rows; fn = 5 (BN 320) or 4 (BN 256), 0 = pick.
struct Args {
  const uint16_t* a;
  const uint16_t* b;
  uint16_t* c;
  uint16_t* h;
  const uint16_t* y;
  int64_t lda, ldb, ldc, ldh, ldy;
  int M, N, K;
  int half;
  // epi 3
  const float* rcos;
  const float* rsin;
  const int64_t* rpos;
  int rseq, rope_cols, rdh;
  // diagnostic builds only (-DCS336_G8_STAMP, scripts/gemm8_stamps.py): per workgroup 8 uint64 --
  // s_memtime at start / after the prologue / after the main loop / after the epilogue's stores
  // retired, s_memrealtime at start and end, HW_ID, XCC_ID. Ignored by the shipped build.
  uint64_t* stamps = nullptr;
};
int pick_fn(int N, int epi, int half);
// diagnostic: later launches with at most `blocks` workgroups write 8 stamps per workgroup into buf
// (builds with -DCS336_G8_STAMP; returns false in other builds). blocks 0 = off.
bool set_stamp_buffer(uint64_t* buf, int64_t blocks);
bool launch(const Args& p, int epi, int fn, hipStream_t s);

// Weight gradient with both operands MN-major (csrc/gemm/gemm8w.hip): C[m][n] = Σ_t A[t][m]·B[t][n],
// A [K][lda] (m < M), B [K][ldb] (n < N), fp32 out. trans_out: C[m][n] stored at c[n·ldc + m].
// splits > 1: split s writes its partial to c + s·slab_stride (dense slabs, reduced by the caller).
// accumulate: c += (splits == 1 only). Requires K % 64 == 0, N % (64·fn) == 0 (fn 5 or 4), M % 4 == 0;
// M is padded to the 256-row tile (rows >= M are computed and dropped).
struct WArgs {
  const uint16_t* a;
  const uint16_t* b;
  float* c;
  int64_t lda, ldb, ldc, slab_stride;
  int64_t a_elems, b_elems;  // storage extent of a / b from their base pointers (bounds for the DMA)
  int M, N, K;
  int splits;
  int trans_out, accumulate;
};
bool launch_w(const WArgs& p, int fn, hipStream_t s);

}  // namespace gemm8
}  // namespace cs336
