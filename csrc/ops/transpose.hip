// 2-byte matrix transpose (bf16/f16) for MI355X: out[c][r] = in[r][c].
//
// Used to give the input-gradient GEMM a K-major copy of each projection weight (Wᵀ), the layout
// hipBLASLt runs 1.15-1.4x faster (models/fused.py). 64×64 tiles through LDS: every global access
// is a 16-byte chunk of a row (coalesced both ways); the LDS image is padded by one 16-B chunk per
// row so the column gather spreads over the banks. Memory-bound: 2 B read + 2 B written per element.
#include "cs336/kernels.h"

namespace cs336 {
namespace {

constexpr int kT = 64;        // tile edge
constexpr int kLd = kT + 8;   // padded LDS row (elements): 144 B, keeps 16-B row alignment

__global__ __launch_bounds__(256) void transpose16_kernel(const uint16_t* __restrict__ in, int64_t ld_in,
                                                          uint16_t* __restrict__ out, int64_t ld_out, int R, int C) {
  __shared__ __attribute__((aligned(16))) uint16_t t[kT * kLd];
  const int r0 = blockIdx.y * kT, c0 = blockIdx.x * kT, tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = tid + 256 * k, r = q >> 3, ch = q & 7;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r0 + r < R && c0 + 8 * ch < C) v = *reinterpret_cast<const uint4*>(in + (int64_t)(r0 + r) * ld_in + c0 + 8 * ch);
    *reinterpret_cast<uint4*>(t + r * kLd + 8 * ch) = v;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = tid + 256 * k, c = q >> 3, ch = q & 7;
    if (c0 + c >= C || r0 + 8 * ch >= R) continue;
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w[j] = (uint32_t)t[(8 * ch + 2 * j) * kLd + c] | ((uint32_t)t[(8 * ch + 2 * j + 1) * kLd + c] << 16);
    *reinterpret_cast<uint4*>(out + (int64_t)(c0 + c) * ld_out + r0 + 8 * ch) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

}  // namespace

void transpose16(const void* in, int64_t ld_in, void* out, int64_t ld_out, int R, int C, hipStream_t s) {
  const dim3 grid((unsigned)((C + kT - 1) / kT), (unsigned)((R + kT - 1) / kT)), block(256);
  hipLaunchKernelGGL(transpose16_kernel, grid, block, 0, s, (const uint16_t*)in, ld_in, (uint16_t*)out, ld_out, R, C);
}

}  // namespace cs336
