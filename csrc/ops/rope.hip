// Rotary position embedding (interleaved pairs) for MI355X.
//
// Semantics: reference cs336-basics/cs336_basics/model.py:121-147. x and out are (B,H,N,D) views
// with arbitrary batch/head/seq strides and a contiguous last dim: x is typically a slice of the
// fused QKV projection output, out either fresh (B,N,H,D) memory (forward: exactly the layout the
// flash-attention kernels read) or a slice of the fused dQKV gradient (backward), so neither
// direction ever makes a transpose or split/cat copy. Each thread rotates 2 pairs (4 elements:
// 16 B fp32 / 8 B bf16 per access), reading cos/sin from the fp32 (ctx, D/2) cache (no on-device
// trig: Appendix B, element-wise). inverse=true applies R(-theta) (the backward).
#include "cs336/kernels.h"

namespace cs336 {
namespace {

template <typename T>
__global__ __launch_bounds__(256) void rope_kernel(const RopeArgs a, const float* __restrict__ cs,
                                                   const float* __restrict__ sn_, const int64_t* __restrict__ pos,
                                                   int H, int N, int D, float sgn, int64_t total) {
  typedef typename Elem<T>::storage S;
  const S* __restrict__ x = (const S*)a.x;
  S* __restrict__ out = (S*)a.out;
  const int D4 = D >> 2;
  const int half = D >> 1;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    // idx enumerates (b, n, h, d4): consecutive threads walk a token's heads -> coalesced rows
    const int d4 = (int)(idx % D4);
    int64_t r = idx / D4;
    const int h = (int)(r % H);
    r /= H;
    const int n = (int)(r % N);
    const int64_t b = r / N;
    const int64_t p = pos ? pos[b * N + n] : (int64_t)n;
    const float4 v = load4<T>(x + b * a.x_sb + h * a.x_sh + n * a.x_sn + 4 * d4);
    const float2 c = *reinterpret_cast<const float2*>(cs + p * half + 2 * d4);
    const float2 s = *reinterpret_cast<const float2*>(sn_ + p * half + 2 * d4);
    const float s0 = sgn * s.x, s1 = sgn * s.y;
    float4 o;
    o.x = c.x * v.x - s0 * v.y;
    o.y = s0 * v.x + c.x * v.y;
    o.z = c.y * v.z - s1 * v.w;
    o.w = s1 * v.z + c.y * v.w;
    store4<T>(out + b * a.o_sb + h * a.o_sh + n * a.o_sn + 4 * d4, o);
  }
}

}  // namespace

void rope(const RopeArgs& a, DType t, const float* cos_, const float* sin_, const int64_t* pos, int B, int H, int N,
          int D, bool inverse, hipStream_t s) {
  const int64_t total = (int64_t)B * N * H * (D / 4);
  const int grid = stream_grid(total, 256);
  const float sgn = inverse ? -1.f : 1.f;
  switch (t) {
    case DType::F32:
      hipLaunchKernelGGL(rope_kernel<float>, dim3(grid), dim3(256), 0, s, a, cos_, sin_, pos, H, N, D, sgn, total);
      break;
    case DType::BF16:
      hipLaunchKernelGGL(rope_kernel<BF16>, dim3(grid), dim3(256), 0, s, a, cos_, sin_, pos, H, N, D, sgn, total);
      break;
    case DType::F16:
      hipLaunchKernelGGL(rope_kernel<F16>, dim3(grid), dim3(256), 0, s, a, cos_, sin_, pos, H, N, D, sgn, total);
      break;
  }
}

}  // namespace cs336
