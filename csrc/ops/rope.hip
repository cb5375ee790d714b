// Rotary position embedding (interleaved pairs) for MI355X.
//
// Semantics: reference cs336-basics/cs336_basics/model.py:121-147. x and out are (B,H,N,D) views
// with arbitrary batch/head/seq strides and a contiguous last dim: x is typically a slice of the
// fused QKV projection output, out either fresh (B,N,H,D) memory (forward: exactly the layout the
// flash-attention kernels read) or a slice of the fused dQKV gradient (backward), so neither
// direction ever makes a transpose or split/cat copy. inverse=true applies R(-theta) (the backward).
//
// Mapping: one thread per (token, head, 8-element group), flat over the grid with 32-bit index math
// (64-bit div/mod per element once cost more than the memory traffic), so every thread moves 16 B
// (bf16) / 32 B (fp32) per access and no lane idles (a block per token left 22-44 % of the lanes
// idle at 25/50 heads x 8 groups). No on-device trig: cos/sin come from the fp32 (ctx, D/2) cache
// (Appendix B, element-wise).
#include "cs336/kernels.h"

namespace cs336 {
namespace {

template <typename T>
__global__ __launch_bounds__(256) void rope_kernel(const RopeArgs a, const float* __restrict__ cs,
                                                   const float* __restrict__ sn_, const int64_t* __restrict__ pos,
                                                   int H, int N, int D8, int total, float sgn) {
  typedef typename Elem<T>::storage S;
  const S* __restrict__ x = (const S*)a.x;
  S* __restrict__ out = (S*)a.out;
  const int half = 4 * D8, HD = H * D8;
  const int i = blockIdx.x * 256 + threadIdx.x;  // flat (token, head, 8-element group): no idle lanes
  if (i >= total) return;
  const int t = i / HD, hd = i - t * HD;
  const int h = hd / D8, d8 = hd - h * D8;  // any D % 8 == 0 (e.g. d_head 80 of the 2.7b model)
  const int b = t / N, n = t - b * N;
  const int64_t p = pos ? pos[t] : (int64_t)n;
  const S* xp = x + b * a.x_sb + h * a.x_sh + n * a.x_sn + 8 * d8;
  S* op = out + b * a.o_sb + h * a.o_sh + n * a.o_sn + 8 * d8;
  const float4 c = *reinterpret_cast<const float4*>(cs + p * half + 4 * d8);
  const float4 s = *reinterpret_cast<const float4*>(sn_ + p * half + 4 * d8);
  const float4 v0 = load4<T>(xp), v1 = load4<T>(xp + 4);
  float4 o0, o1;
  o0.x = c.x * v0.x - sgn * s.x * v0.y;
  o0.y = sgn * s.x * v0.x + c.x * v0.y;
  o0.z = c.y * v0.z - sgn * s.y * v0.w;
  o0.w = sgn * s.y * v0.z + c.y * v0.w;
  o1.x = c.z * v1.x - sgn * s.z * v1.y;
  o1.y = sgn * s.z * v1.x + c.z * v1.y;
  o1.z = c.w * v1.z - sgn * s.w * v1.w;
  o1.w = sgn * s.w * v1.z + c.w * v1.w;
  store4<T>(op, o0);
  store4<T>(op + 4, o1);
}

}  // namespace

void rope(const RopeArgs& a, DType t, const float* cos_, const float* sin_, const int64_t* pos, int B, int H, int N,
          int D, bool inverse, hipStream_t s) {
  // D % 8 == 0 (head dims 8 .. 256); the binding checks it
  const int D8 = D / 8;
  const int64_t total64 = (int64_t)B * N * H * D8;
  const int total = (int)total64;  // < 2^31 for every model shape (checked by the binding)
  const dim3 grid((unsigned)((total64 + 255) / 256)), block(256);
  const float sgn = inverse ? -1.f : 1.f;
  switch (t) {
    case DType::F32:
      hipLaunchKernelGGL(rope_kernel<float>, grid, block, 0, s, a, cos_, sin_, pos, H, N, D8, total, sgn);
      break;
    case DType::BF16:
      hipLaunchKernelGGL(rope_kernel<BF16>, grid, block, 0, s, a, cos_, sin_, pos, H, N, D8, total, sgn);
      break;
    case DType::F16:
      hipLaunchKernelGGL(rope_kernel<F16>, grid, block, 0, s, a, cos_, sin_, pos, H, N, D8, total, sgn);
      break;
  }
}

}  // namespace cs336
