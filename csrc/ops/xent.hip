// Fused cross-entropy over logits for MI355X.
//
// Semantics: reference cs336-basics/cs336_basics/nn_utils.py:9-17 — loss_r = logsumexp(z_r) - z_r[t_r],
// mean over rows (the mean is a trivial torch reduction over the (M,) fp32 losses).
// Forward: one 256-thread workgroup per row; each lane keeps an online (max, sum-exp) over its
// strided slice of the vocab (one read of the logits, 8 B per lane per access), then a
// wave-shuffle + LDS merge of the (m, s) pairs. Backward: dz = (exp(z - lse) - onehot(t)) * g * mult,
// with the upstream scalar g read from device memory (no host sync), written in the logits dtype.
#include "cs336/kernels.h"

namespace cs336 {
namespace {

__device__ __forceinline__ void merge_ms(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  if (mn == -INFINITY) return;
  s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
  m = mn;
}

template <typename T>
__global__ __launch_bounds__(256) void xent_fwd_kernel(const typename Elem<T>::storage* __restrict__ z,
                                                       const int64_t* __restrict__ tgt, float* __restrict__ loss,
                                                       float* __restrict__ lse, int64_t V) {
  __shared__ float sm[4], ss[4];
  const int64_t row = blockIdx.x;
  const auto* zr = z + row * V;
  float m = -INFINITY, s = 0.f;
  const bool vec = (V % 4 == 0);
  if (vec) {
    const int64_t V4 = V / 4;
    for (int64_t i = threadIdx.x; i < V4; i += 256) {
      const float4 v = load4<T>(zr + 4 * i);
      const float vm = fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w));
      if (vm > m) {
        s *= __expf(m - vm);
        m = vm;
      }
      s += __expf(v.x - m) + __expf(v.y - m) + __expf(v.z - m) + __expf(v.w - m);
    }
  } else {
    for (int64_t i = threadIdx.x; i < V; i += 256) {
      const float v = Elem<T>::to_f(zr[i]);
      if (v > m) {
        s *= __expf(m - v);
        m = v;
      }
      s += __expf(v - m);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, kWave), s2 = __shfl_xor(s, o, kWave);
    merge_ms(m, s, m2, s2);
  }
  const int w = threadIdx.x / kWave;
  if ((threadIdx.x % kWave) == 0) {
    sm[w] = m;
    ss[w] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M_ = sm[0], S_ = ss[0];
    for (int i = 1; i < 4; ++i) merge_ms(M_, S_, sm[i], ss[i]);
    const float l = M_ + __logf(S_);
    lse[row] = l;
    loss[row] = l - Elem<T>::to_f(zr[tgt[row]]);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void xent_bwd_kernel(const float* __restrict__ g, const typename Elem<T>::storage* __restrict__ z,
                                                       const int64_t* __restrict__ tgt, const float* __restrict__ lse,
                                                       typename Elem<T>::storage* __restrict__ dz, float mult, int64_t V) {
  const int64_t row = blockIdx.x;
  const auto* zr = z + row * V;
  auto* dr = dz + row * V;
  const float l = lse[row];
  const float sc = g[0] * mult;
  const int64_t t = tgt[row];
  if (V % 4 == 0) {
    const int64_t V4 = V / 4;
    for (int64_t i = threadIdx.x; i < V4; i += 256) {
      const float4 v = load4<T>(zr + 4 * i);
      float4 o;
      o.x = (__expf(v.x - l) - (4 * i + 0 == t ? 1.f : 0.f)) * sc;
      o.y = (__expf(v.y - l) - (4 * i + 1 == t ? 1.f : 0.f)) * sc;
      o.z = (__expf(v.z - l) - (4 * i + 2 == t ? 1.f : 0.f)) * sc;
      o.w = (__expf(v.w - l) - (4 * i + 3 == t ? 1.f : 0.f)) * sc;
      store4<T>(dr + 4 * i, o);
    }
  } else {
    for (int64_t i = threadIdx.x; i < V; i += 256) {
      const float v = Elem<T>::to_f(zr[i]);
      dr[i] = Elem<T>::from_f((__expf(v - l) - (i == t ? 1.f : 0.f)) * sc);
    }
  }
}

}  // namespace

void xent_fwd(const void* z, DType t, const int64_t* tgt, float* loss, float* lse, int64_t M, int64_t V, hipStream_t s) {
  if (M == 0) return;
  switch (t) {
    case DType::F32: hipLaunchKernelGGL(xent_fwd_kernel<float>, dim3(M), dim3(256), 0, s, (const float*)z, tgt, loss, lse, V); break;
    case DType::BF16: hipLaunchKernelGGL(xent_fwd_kernel<BF16>, dim3(M), dim3(256), 0, s, (const bf16_t*)z, tgt, loss, lse, V); break;
    case DType::F16: hipLaunchKernelGGL(xent_fwd_kernel<F16>, dim3(M), dim3(256), 0, s, (const f16_t*)z, tgt, loss, lse, V); break;
  }
}

void xent_bwd(const float* g, const void* z, DType t, const int64_t* tgt, const float* lse, void* dz, float mult,
              int64_t M, int64_t V, hipStream_t s) {
  if (M == 0) return;
  switch (t) {
    case DType::F32: hipLaunchKernelGGL(xent_bwd_kernel<float>, dim3(M), dim3(256), 0, s, g, (const float*)z, tgt, lse, (float*)dz, mult, V); break;
    case DType::BF16: hipLaunchKernelGGL(xent_bwd_kernel<BF16>, dim3(M), dim3(256), 0, s, g, (const bf16_t*)z, tgt, lse, (bf16_t*)dz, mult, V); break;
    case DType::F16: hipLaunchKernelGGL(xent_bwd_kernel<F16>, dim3(M), dim3(256), 0, s, g, (const f16_t*)z, tgt, lse, (f16_t*)dz, mult, V); break;
  }
}

}  // namespace cs336
