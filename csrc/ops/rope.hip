// Rotary position embedding (interleaved pairs) for MI355X.
//
// Semantics: reference cs336-basics/cs336_basics/model.py:121-147. x is a (B,H,N,D) view with
// arbitrary batch/head/seq strides and a contiguous last dim (typically the transposed view of a
// (B,N,H,D) projection output); the result is written in (B,N,H,D) memory order, i.e. exactly
// the layout the flash-attention kernels and the output projection want, so attention needs no
// transpose copies. Each thread rotates 2 pairs (4 elements: one 16 B fp32 or 8 B bf16 access),
// reading cos/sin from the fp32 (ctx, D/2) cache (no on-device trig: Appendix B, element-wise).
// inverse=true applies R(-theta) (the backward).
#include "cs336/kernels.h"

namespace cs336 {
namespace {

template <typename T>
__global__ __launch_bounds__(256) void rope_kernel(const typename Elem<T>::storage* __restrict__ x, int64_t sb,
                                                   int64_t sh, int64_t sn, typename Elem<T>::storage* __restrict__ out,
                                                   const float* __restrict__ cs, const float* __restrict__ sn_,
                                                   const int64_t* __restrict__ pos, int B, int H, int N, int D,
                                                   float sgn, int64_t total) {
  const int D4 = D >> 2;
  const int half = D >> 1;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    // idx enumerates (b, n, h, d4) in output (BNHD) order -> coalesced stores
    const int d4 = (int)(idx % D4);
    int64_t r = idx / D4;
    const int h = (int)(r % H);
    r /= H;
    const int n = (int)(r % N);
    const int b = (int)(r / N);
    const int64_t p = pos ? pos[(int64_t)b * N + n] : (int64_t)n;
    const float4 v = load4<T>(x + b * sb + h * sh + n * sn + 4 * d4);
    const float2 c = *reinterpret_cast<const float2*>(cs + p * half + 2 * d4);
    const float2 s = *reinterpret_cast<const float2*>(sn_ + p * half + 2 * d4);
    const float s0 = sgn * s.x, s1 = sgn * s.y;
    float4 o;
    o.x = c.x * v.x - s0 * v.y;
    o.y = s0 * v.x + c.x * v.y;
    o.z = c.y * v.z - s1 * v.w;
    o.w = s1 * v.z + c.y * v.w;
    store4<T>(out + idx * 4, o);
  }
}

}  // namespace

void rope(const void* x, DType t, int64_t sb, int64_t sh, int64_t sn, void* out, const float* cos_, const float* sin_,
          const int64_t* pos, int B, int H, int N, int D, bool inverse, hipStream_t s) {
  const int64_t total = (int64_t)B * N * H * (D / 4);
  const int grid = stream_grid(total, 256);
  const float sgn = inverse ? -1.f : 1.f;
  switch (t) {
    case DType::F32:
      hipLaunchKernelGGL(rope_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)x, sb, sh, sn, (float*)out,
                         cos_, sin_, pos, B, H, N, D, sgn, total);
      break;
    case DType::BF16:
      hipLaunchKernelGGL(rope_kernel<BF16>, dim3(grid), dim3(256), 0, s, (const bf16_t*)x, sb, sh, sn, (bf16_t*)out,
                         cos_, sin_, pos, B, H, N, D, sgn, total);
      break;
    case DType::F16:
      hipLaunchKernelGGL(rope_kernel<F16>, dim3(grid), dim3(256), 0, s, (const f16_t*)x, sb, sh, sn, (f16_t*)out,
                         cos_, sin_, pos, B, H, N, D, sgn, total);
      break;
  }
}

}  // namespace cs336
