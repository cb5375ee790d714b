// Multi-tensor kernels for MI355X: fused AdamW, global L2 norm, in-place scale.
//
// One launch covers a whole list of tensors. The host passes a small device table (per tensor:
// its pointers, numel and the prefix sum of its 32 Ki-element chunks); workgroup b finds its
// tensor with a binary search over the prefix sums and streams its chunk with 16-byte vector
// accesses (scalar fallback when a tensor view is not 16-byte aligned). The AdamW step is
// HBM-bound at 28 B/param (read p, g, m, v; write p, m, v) versus ~9 eager kernels per tensor
// in the reference's Python loop (cs336-basics/cs336_basics/optimizer.py:50-86).
#include "cs336/kernels.h"

namespace cs336 {
namespace {

__device__ __forceinline__ int find_tensor(const int64_t* __restrict__ base, int n, int64_t chunk) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (base[mid] <= chunk) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// ---- AdamW ------------------------------------------------------------------------------------
// Exactly the reference update order, with FP contraction disabled so every product/sum rounds
// like the separate eager kernels do:
//   m = b1*m + (1-b1)*g;  v = b2*v + (1-b2)*g*g;  p -= (alpha_t*m) / (sqrt(v)+eps);  p -= (lr*wd)*p
#pragma clang fp contract(off)
__device__ __forceinline__ void adamw_elem(float& p, float g, float& m, float& v, float b1, float omb1, float b2,
                                           float omb2, float eps, float alpha_t, float lr_wd) {
  m = b1 * m + omb1 * g;
  v = b2 * v + omb2 * (g * g);
  p = p - (alpha_t * m) / (sqrtf(v) + eps);
  p = p - lr_wd * p;
}

// SHADOW: also write the bf16 copy of the updated fp32 master weight (the compute weights the
// model's GEMMs read), in the same pass: +2 B/param instead of a separate 6 B/param cast pass.
template <typename TG, bool SHADOW>
__global__ __launch_bounds__(256) void adamw_kernel(const int64_t* __restrict__ ptrs,
                                                    const int64_t* __restrict__ chunk_base,
                                                    const int64_t* __restrict__ numel, int n, float b1, float b2,
                                                    float omb1, float omb2, float eps, float lr_wd,
                                                    float alpha_h, const float* __restrict__ alpha_dev) {
  constexpr int NP = SHADOW ? 5 : 4;
  const float alpha_t = alpha_dev ? *alpha_dev : alpha_h;
  const int64_t chunk = blockIdx.x;
  const int t = find_tensor(chunk_base, n, chunk);
  float* p = reinterpret_cast<float*>(ptrs[NP * t + 0]);
  const auto* g = reinterpret_cast<const typename Elem<TG>::storage*>(ptrs[NP * t + 1]);
  float* m = reinterpret_cast<float*>(ptrs[NP * t + 2]);
  float* v = reinterpret_cast<float*>(ptrs[NP * t + 3]);
  bf16_t* sh = SHADOW ? reinterpret_cast<bf16_t*>(ptrs[NP * t + 4]) : nullptr;
  const int64_t N = numel[t];
  const int64_t start = (chunk - chunk_base[t]) * kMTChunk;
  const int64_t end = start + kMTChunk < N ? start + kMTChunk : N;
  const uintptr_t align = (uintptr_t)p | (uintptr_t)m | (uintptr_t)v | (uintptr_t)g;
  const int gal = sizeof(typename Elem<TG>::storage) == 4 ? 15 : 7;
  const bool shal = !SHADOW || (((uintptr_t)sh) & 7) == 0;
  if ((align & 15) == 0 && (((uintptr_t)g) & gal) == 0 && (start & 3) == 0 && shal) {
    const int64_t end4 = start + ((end - start) & ~(int64_t)3);
    for (int64_t i = start + 4 * threadIdx.x; i < end4; i += 4 * 256) {
      float4 pv = *reinterpret_cast<float4*>(p + i);
      float4 mv = *reinterpret_cast<float4*>(m + i);
      float4 vv = *reinterpret_cast<float4*>(v + i);
      const float4 gv = load4<TG>(g + i);
      adamw_elem(pv.x, gv.x, mv.x, vv.x, b1, omb1, b2, omb2, eps, alpha_t, lr_wd);
      adamw_elem(pv.y, gv.y, mv.y, vv.y, b1, omb1, b2, omb2, eps, alpha_t, lr_wd);
      adamw_elem(pv.z, gv.z, mv.z, vv.z, b1, omb1, b2, omb2, eps, alpha_t, lr_wd);
      adamw_elem(pv.w, gv.w, mv.w, vv.w, b1, omb1, b2, omb2, eps, alpha_t, lr_wd);
      *reinterpret_cast<float4*>(p + i) = pv;
      *reinterpret_cast<float4*>(m + i) = mv;
      *reinterpret_cast<float4*>(v + i) = vv;
      if (SHADOW) store4<BF16>(sh + i, pv);
    }
    for (int64_t i = end4 + threadIdx.x; i < end; i += 256) {
      float pp = p[i], mm = m[i], vv = v[i];
      adamw_elem(pp, Elem<TG>::to_f(g[i]), mm, vv, b1, omb1, b2, omb2, eps, alpha_t, lr_wd);
      p[i] = pp;
      m[i] = mm;
      v[i] = vv;
      if (SHADOW) sh[i] = f32_to_bf16(pp);
    }
  } else {
    for (int64_t i = start + threadIdx.x; i < end; i += 256) {
      float pp = p[i], mm = m[i], vv = v[i];
      adamw_elem(pp, Elem<TG>::to_f(g[i]), mm, vv, b1, omb1, b2, omb2, eps, alpha_t, lr_wd);
      p[i] = pp;
      m[i] = mm;
      v[i] = vv;
      if (SHADOW) sh[i] = f32_to_bf16(pp);
    }
  }
}

// ---- AdamW + transposed bf16 shadow --------------------------------------------------------------
// For 2-D weights (R x C, row-major) the update also writes Wᵀ in bf16 (C x R view with row stride
// ldt), the K-major operand of the input-gradient GEMM (models/fused.py), so the forward needs no
// per-call transpose of every weight. One workgroup = 256 rows x 64 columns; each thread updates an
// 8 x 8 block row by row (8 x 32-B row segments per tensor: a wave's loads cover 8 rows x 256 B),
// keeps the 8 x 8 bf16 results packed in 32 VGPRs, and writes them transposed as eight 16-B column
// chunks (a wave's stores cover 8 output rows x 128 B). Same update arithmetic as adamw_kernel.
__device__ __forceinline__ uint32_t lo_pair(uint32_t a, uint32_t b) { return (a & 0xffffu) | (b << 16); }
__device__ __forceinline__ uint32_t hi_pair(uint32_t a, uint32_t b) { return (a >> 16) | (b & 0xffff0000u); }

template <typename TG>
__global__ __launch_bounds__(256) void adamw_t_kernel(const int64_t* __restrict__ ptrs,
                                                      const int64_t* __restrict__ tile_base,
                                                      const int64_t* __restrict__ dims, int n, float b1, float b2,
                                                      float omb1, float omb2, float eps, float lr_wd, float alpha_h,
                                                      const float* __restrict__ alpha_dev) {
  const int64_t tile = blockIdx.x;
  const float alpha_t = alpha_dev ? *alpha_dev : alpha_h;
  const int t = find_tensor(tile_base, n, tile);
  float* p = reinterpret_cast<float*>(ptrs[6 * t + 0]);
  const auto* g = reinterpret_cast<const typename Elem<TG>::storage*>(ptrs[6 * t + 1]);
  float* m = reinterpret_cast<float*>(ptrs[6 * t + 2]);
  float* v = reinterpret_cast<float*>(ptrs[6 * t + 3]);
  bf16_t* sh = reinterpret_cast<bf16_t*>(ptrs[6 * t + 4]);
  bf16_t* wt = reinterpret_cast<bf16_t*>(ptrs[6 * t + 5]);
  const int64_t R = dims[3 * t], C = dims[3 * t + 1], ldt = dims[3 * t + 2];
  const int64_t ctiles = (C + 63) >> 6;
  const int64_t local = tile - tile_base[t];
  const int ch = threadIdx.x & 7, rr = threadIdx.x >> 3;
  const int64_t r = (local / ctiles) * 256 + 8 * rr;  // first of this thread's 8 rows
  const int64_t c = (local % ctiles) * 64 + 8 * ch;   // first of its 8 columns
  if (r >= R || c >= C) return;                       // R, C multiples of 8 (host check)
  uint32_t w[8][4];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int64_t i = (r + j) * C + c;
    float4 p0 = *reinterpret_cast<float4*>(p + i), p1 = *reinterpret_cast<float4*>(p + i + 4);
    float4 m0 = *reinterpret_cast<float4*>(m + i), m1 = *reinterpret_cast<float4*>(m + i + 4);
    float4 v0 = *reinterpret_cast<float4*>(v + i), v1 = *reinterpret_cast<float4*>(v + i + 4);
    const float4 g0 = load4<TG>(g + i), g1 = load4<TG>(g + i + 4);
    adamw_elem(p0.x, g0.x, m0.x, v0.x, b1, omb1, b2, omb2, eps, alpha_t, lr_wd);
    adamw_elem(p0.y, g0.y, m0.y, v0.y, b1, omb1, b2, omb2, eps, alpha_t, lr_wd);
    adamw_elem(p0.z, g0.z, m0.z, v0.z, b1, omb1, b2, omb2, eps, alpha_t, lr_wd);
    adamw_elem(p0.w, g0.w, m0.w, v0.w, b1, omb1, b2, omb2, eps, alpha_t, lr_wd);
    adamw_elem(p1.x, g1.x, m1.x, v1.x, b1, omb1, b2, omb2, eps, alpha_t, lr_wd);
    adamw_elem(p1.y, g1.y, m1.y, v1.y, b1, omb1, b2, omb2, eps, alpha_t, lr_wd);
    adamw_elem(p1.z, g1.z, m1.z, v1.z, b1, omb1, b2, omb2, eps, alpha_t, lr_wd);
    adamw_elem(p1.w, g1.w, m1.w, v1.w, b1, omb1, b2, omb2, eps, alpha_t, lr_wd);
    *reinterpret_cast<float4*>(p + i) = p0;
    *reinterpret_cast<float4*>(p + i + 4) = p1;
    *reinterpret_cast<float4*>(m + i) = m0;
    *reinterpret_cast<float4*>(m + i + 4) = m1;
    *reinterpret_cast<float4*>(v + i) = v0;
    *reinterpret_cast<float4*>(v + i + 4) = v1;
    w[j][0] = (uint32_t)f32_to_bf16(p0.x) | ((uint32_t)f32_to_bf16(p0.y) << 16);
    w[j][1] = (uint32_t)f32_to_bf16(p0.z) | ((uint32_t)f32_to_bf16(p0.w) << 16);
    w[j][2] = (uint32_t)f32_to_bf16(p1.x) | ((uint32_t)f32_to_bf16(p1.y) << 16);
    w[j][3] = (uint32_t)f32_to_bf16(p1.z) | ((uint32_t)f32_to_bf16(p1.w) << 16);
    *reinterpret_cast<uint4*>(sh + i) = make_uint4(w[j][0], w[j][1], w[j][2], w[j][3]);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {  // Wᵀ row c + k holds column c + k of the block; element k sits in dword k/2
    const int d = k >> 1;
    uint32_t o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = (k & 1) ? hi_pair(w[2 * q][d], w[2 * q + 1][d]) : lo_pair(w[2 * q][d], w[2 * q + 1][d]);
    *reinterpret_cast<uint4*>(wt + (c + k) * ldt + r) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}
#pragma clang fp contract(on)

// ---- sum of squares (per-chunk partials, deterministic) ----------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void sumsq_kernel(const int64_t* __restrict__ ptrs,
                                                    const int64_t* __restrict__ chunk_base,
                                                    const int64_t* __restrict__ numel, int n,
                                                    float* __restrict__ partials) {
  __shared__ float red[4];
  const int64_t chunk = blockIdx.x;
  const int t = find_tensor(chunk_base, n, chunk);
  const auto* x = reinterpret_cast<const typename Elem<T>::storage*>(ptrs[t]);
  const int64_t N = numel[t];
  const int64_t start = (chunk - chunk_base[t]) * kMTChunk;
  const int64_t end = start + kMTChunk < N ? start + kMTChunk : N;
  float acc = 0.f;
  const int al = sizeof(typename Elem<T>::storage) == 4 ? 15 : 7;
  if ((((uintptr_t)x) & al) == 0) {
    const int64_t end4 = start + ((end - start) & ~(int64_t)3);
    for (int64_t i = start + 4 * threadIdx.x; i < end4; i += 4 * 256) {
      const float4 v = load4<T>(x + i);
      acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    for (int64_t i = end4 + threadIdx.x; i < end; i += 256) {
      const float v = Elem<T>::to_f(x[i]);
      acc += v * v;
    }
  } else {
    for (int64_t i = start + threadIdx.x; i < end; i += 256) {
      const float v = Elem<T>::to_f(x[i]);
      acc += v * v;
    }
  }
  acc = block_sum<256>(acc, red);
  if (threadIdx.x == 0) partials[chunk] = acc;
}

__global__ __launch_bounds__(1024) void finalize_l2_kernel(const float* __restrict__ partials, int64_t n,
                                                           float* __restrict__ out) {
  __shared__ float red[16];
  float acc = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += 1024) acc += partials[i];
  acc = block_sum<1024>(acc, red);
  if (threadIdx.x == 0) out[0] = sqrtf(acc);
}

template <typename T>
__global__ __launch_bounds__(256) void scale_kernel(const int64_t* __restrict__ ptrs,
                                                    const int64_t* __restrict__ chunk_base,
                                                    const int64_t* __restrict__ numel, int n,
                                                    const float* __restrict__ scale) {
  const int64_t chunk = blockIdx.x;
  const int t = find_tensor(chunk_base, n, chunk);
  auto* x = reinterpret_cast<typename Elem<T>::storage*>(ptrs[t]);
  const int64_t N = numel[t];
  const int64_t start = (chunk - chunk_base[t]) * kMTChunk;
  const int64_t end = start + kMTChunk < N ? start + kMTChunk : N;
  const float c = scale[0];
  for (int64_t i = start + threadIdx.x; i < end; i += 256) x[i] = Elem<T>::from_f(Elem<T>::to_f(x[i]) * c);
}

}  // namespace

void adamw_step(const TensorTable& tt, DType grad_t, bool shadow, float beta1, float beta2, float one_minus_beta1,
                float one_minus_beta2, float eps, float lr_wd, float alpha_t, const float* alpha_dev, hipStream_t s) {
  if (tt.total_chunks == 0) return;
  const dim3 grid((unsigned)tt.total_chunks), block(256);
  auto go = [&](auto tg, auto sh) {
    using TG = decltype(tg);
    constexpr bool SH = decltype(sh)::value;
    hipLaunchKernelGGL((adamw_kernel<TG, SH>), grid, block, 0, s, tt.ptrs, tt.chunk_base, tt.numel, tt.n, beta1,
                       beta2, one_minus_beta1, one_minus_beta2, eps, lr_wd, alpha_t, alpha_dev);
  };
  auto by_shadow = [&](auto tg) {
    if (shadow) go(tg, std::true_type{});
    else go(tg, std::false_type{});
  };
  switch (grad_t) {
    case DType::F32: by_shadow(float{}); break;
    case DType::BF16: by_shadow(BF16{}); break;
    case DType::F16: by_shadow(F16{}); break;
  }
}

void adamw_step_t(const int64_t* ptrs, const int64_t* tile_base, const int64_t* dims, int n, int64_t total_tiles,
                  DType grad_t, float beta1, float beta2, float one_minus_beta1, float one_minus_beta2, float eps,
                  float lr_wd, float alpha_t, const float* alpha_dev, hipStream_t s) {
  if (total_tiles == 0) return;
  const dim3 grid((unsigned)total_tiles), block(256);
  auto go = [&](auto tg) {
    using TG = decltype(tg);
    hipLaunchKernelGGL((adamw_t_kernel<TG>), grid, block, 0, s, ptrs, tile_base, dims, n, beta1, beta2,
                       one_minus_beta1, one_minus_beta2, eps, lr_wd, alpha_t, alpha_dev);
  };
  switch (grad_t) {
    case DType::F32: go(float{}); break;
    case DType::BF16: go(BF16{}); break;
    case DType::F16: go(F16{}); break;
  }
}

// One thread: the step counter of a HIP-graph-captured optimizer step and its bias-corrected step
// size, in double as the host evaluates it (bindings.cpp adamw_step), rounded once to fp32.
__global__ __launch_bounds__(64) void adamw_device_step_kernel(int64_t* t, float* alpha, double lr, double b1,
                                                               double b2) {
  if (threadIdx.x != 0) return;
  const int64_t s = *t + 1;
  *t = s;
  *alpha = (float)(lr * (sqrt(1.0 - pow(b2, (double)s)) / (1.0 - pow(b1, (double)s))));
}

void adamw_device_step(int64_t* t, float* alpha, double lr, double beta1, double beta2, hipStream_t s) {
  hipLaunchKernelGGL(adamw_device_step_kernel, dim3(1), dim3(64), 0, s, t, alpha, lr, beta1, beta2);
}

// bf16 copy of fp32 tensors (initial sync of the compute-weight shadows)
__global__ __launch_bounds__(256) void cast_bf16_kernel(const int64_t* __restrict__ ptrs,
                                                        const int64_t* __restrict__ chunk_base,
                                                        const int64_t* __restrict__ numel, int n) {
  const int64_t chunk = blockIdx.x;
  const int t = find_tensor(chunk_base, n, chunk);
  const float* x = reinterpret_cast<const float*>(ptrs[2 * t]);
  bf16_t* y = reinterpret_cast<bf16_t*>(ptrs[2 * t + 1]);
  const int64_t N = numel[t];
  const int64_t start = (chunk - chunk_base[t]) * kMTChunk;
  const int64_t end = start + kMTChunk < N ? start + kMTChunk : N;
  for (int64_t i = start + threadIdx.x; i < end; i += 256) y[i] = f32_to_bf16(x[i]);
}

void multi_tensor_cast_bf16(const TensorTable& tt, hipStream_t s) {
  if (tt.total_chunks == 0) return;
  hipLaunchKernelGGL(cast_bf16_kernel, dim3((unsigned)tt.total_chunks), dim3(256), 0, s, tt.ptrs, tt.chunk_base,
                     tt.numel, tt.n);
}

void multi_tensor_sumsq(const TensorTable& tt, DType t, float* partials, hipStream_t s) {
  if (tt.total_chunks == 0) return;
  const dim3 grid((unsigned)tt.total_chunks), block(256);
  switch (t) {
    case DType::F32: hipLaunchKernelGGL(sumsq_kernel<float>, grid, block, 0, s, tt.ptrs, tt.chunk_base, tt.numel, tt.n, partials); break;
    case DType::BF16: hipLaunchKernelGGL(sumsq_kernel<BF16>, grid, block, 0, s, tt.ptrs, tt.chunk_base, tt.numel, tt.n, partials); break;
    case DType::F16: hipLaunchKernelGGL(sumsq_kernel<F16>, grid, block, 0, s, tt.ptrs, tt.chunk_base, tt.numel, tt.n, partials); break;
  }
}

void finalize_l2norm(const float* partials, int64_t n, float* out, hipStream_t s) {
  hipLaunchKernelGGL(finalize_l2_kernel, dim3(1), dim3(1024), 0, s, partials, n, out);
}

void multi_tensor_scale(const TensorTable& tt, DType t, const float* scale, hipStream_t s) {
  if (tt.total_chunks == 0) return;
  const dim3 grid((unsigned)tt.total_chunks), block(256);
  switch (t) {
    case DType::F32: hipLaunchKernelGGL(scale_kernel<float>, grid, block, 0, s, tt.ptrs, tt.chunk_base, tt.numel, tt.n, scale); break;
    case DType::BF16: hipLaunchKernelGGL(scale_kernel<BF16>, grid, block, 0, s, tt.ptrs, tt.chunk_base, tt.numel, tt.n, scale); break;
    case DType::F16: hipLaunchKernelGGL(scale_kernel<F16>, grid, block, 0, s, tt.ptrs, tt.chunk_base, tt.numel, tt.n, scale); break;
  }
}

}  // namespace cs336
