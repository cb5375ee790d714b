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
};
int pick_fn(int N, int epi, int half);
bool launch(const Args& p, int epi, int fn, hipStream_t s);

}  // namespace gemm8
}  // namespace cs336
