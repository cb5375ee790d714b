// 2-byte matrix transpose (bf16/f16) for MI355X: out[c][r] = in[r][c].
//
// Used to give the input-gradient GEMM a K-major copy of each projection weight (Wᵀ), the layout
// hipBLASLt runs 1.15-1.4x faster, and the W1|W3 weight-gradient GEMM a token-contiguous Xᵀ
// (models/fused.py). Memory-bound: 2 B read + 2 B written per element.
//
// Register transpose, no LDS: each thread loads an 8×8 block as eight 16-byte row chunks, transposes
// it in VGPRs (16-bit lane packing, v_perm/v_and_or) and stores eight 16-byte column chunks. Lanes are
// laid out chunk-fastest (ch = tid & 7, row group rr = tid >> 3), so within one wave every load
// instruction reads eight 128-byte row runs and every store writes eight 128-byte output-row runs.
// A workgroup covers 256 rows × 64 columns (32 KB), 4x the bytes in flight of the previous 64×64
// LDS tile, and drops its eight 2-byte LDS gathers per stored chunk.
#include <cstdlib>
#include <string>

#include "cs336/kernels.h"

namespace cs336 {
namespace {

constexpr int kRows = 256;  // rows per workgroup (32 row groups of 8)
constexpr int kCols = 64;   // columns per workgroup (8 chunks of 8)

__device__ __forceinline__ uint32_t lo_pair(uint32_t a, uint32_t b) { return (a & 0xffffu) | (b << 16); }
__device__ __forceinline__ uint32_t hi_pair(uint32_t a, uint32_t b) { return (a >> 16) | (b & 0xffff0000u); }

__global__ __launch_bounds__(256) void transpose16_kernel(const uint16_t* __restrict__ in, int64_t ld_in,
                                                          uint16_t* __restrict__ out, int64_t ld_out, int R, int C) {
  const int tid = threadIdx.x, ch = tid & 7, rr = tid >> 3;
  const int r = blockIdx.y * kRows + 8 * rr;  // first of this thread's 8 input rows
  const int c = blockIdx.x * kCols + 8 * ch;  // first of its 8 input columns
  if (r >= R || c >= C) return;               // R, C are multiples of 8 (host check)
  uint32_t v[8][4];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint4 x = *reinterpret_cast<const uint4*>(in + (int64_t)(r + j) * ld_in + c);
    v[j][0] = x.x; v[j][1] = x.y; v[j][2] = x.z; v[j][3] = x.w;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {  // output row c + k = input column c + k; element k sits in dword k/2
    const int d = k >> 1;
    uint32_t w[4];
#pragma unroll
    for (int p = 0; p < 4; ++p)
      w[p] = (k & 1) ? hi_pair(v[2 * p][d], v[2 * p + 1][d]) : lo_pair(v[2 * p][d], v[2 * p + 1][d]);
    *reinterpret_cast<uint4*>(out + (int64_t)(c + k) * ld_out + r) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// fp32 -> bf16 cast that also writes the transpose: w[r][c] = bf16(in[r][c]), wt[c][r] = the same.
// Same 8x8-per-thread register transpose as above; 4 B read + 4 B written per element (a cast and a
// separate 16-bit transpose move 10). The compiled model's projections use it for their bf16
// compute weight and the K-major Wᵀ their input gradient reads when no bf16 shadows are attached
// (models/compiled.py).
__global__ __launch_bounds__(256) void cast_t_kernel(const float* __restrict__ in, int64_t ld_in,
                                                     uint16_t* __restrict__ w, int64_t ld_w,
                                                     uint16_t* __restrict__ wt, int64_t ld_t, int R, int C) {
  const int tid = threadIdx.x, ch = tid & 7, rr = tid >> 3;
  const int r = blockIdx.y * kRows + 8 * rr;
  const int c = blockIdx.x * kCols + 8 * ch;
  if (r >= R || c >= C) return;  // R, C multiples of 8 (host check)
  uint32_t v[8][4];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float4 a = *reinterpret_cast<const float4*>(in + (int64_t)(r + j) * ld_in + c);
    const float4 b = *reinterpret_cast<const float4*>(in + (int64_t)(r + j) * ld_in + c + 4);
    v[j][0] = (uint32_t)f32_to_bf16(a.x) | ((uint32_t)f32_to_bf16(a.y) << 16);
    v[j][1] = (uint32_t)f32_to_bf16(a.z) | ((uint32_t)f32_to_bf16(a.w) << 16);
    v[j][2] = (uint32_t)f32_to_bf16(b.x) | ((uint32_t)f32_to_bf16(b.y) << 16);
    v[j][3] = (uint32_t)f32_to_bf16(b.z) | ((uint32_t)f32_to_bf16(b.w) << 16);
    *reinterpret_cast<uint4*>(w + (int64_t)(r + j) * ld_w + c) = make_uint4(v[j][0], v[j][1], v[j][2], v[j][3]);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int d = k >> 1;
    uint32_t o[4];
#pragma unroll
    for (int p = 0; p < 4; ++p)
      o[p] = (k & 1) ? hi_pair(v[2 * p][d], v[2 * p + 1][d]) : lo_pair(v[2 * p][d], v[2 * p + 1][d]);
    *reinterpret_cast<uint4*>(wt + (int64_t)(c + k) * ld_t + r) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

}  // namespace

void cast_transpose_bf16(const float* in, int64_t ld_in, void* w, int64_t ld_w, void* wt, int64_t ld_t, int R, int C,
                         hipStream_t s) {
  const dim3 grid((unsigned)((C + kCols - 1) / kCols), (unsigned)((R + kRows - 1) / kRows)), block(256);
  hipLaunchKernelGGL(cast_t_kernel, grid, block, 0, s, in, ld_in, (uint16_t*)w, ld_w, (uint16_t*)wt, ld_t, R, C);
}

// (the round-1 64x64 LDS-tile version, CS336_TRANSPOSE=lds, was retired in round 5:
// profiles/r1_transpose_reg_vs_lds.md)
void transpose16(const void* in, int64_t ld_in, void* out, int64_t ld_out, int R, int C, hipStream_t s) {
  const dim3 grid((unsigned)((C + kCols - 1) / kCols), (unsigned)((R + kRows - 1) / kRows)), block(256);
  hipLaunchKernelGGL(transpose16_kernel, grid, block, 0, s, (const uint16_t*)in, ld_in, (uint16_t*)out, ld_out, R, C);
}

}  // namespace cs336
