// SwiGLU gate h = silu(a) * b and its backward, for MI355X.
//
// Semantics: reference cs336-basics/cs336_basics/model.py:396-397, 526-527 (silu(x)=x*sigmoid(x)).
// Memory-bound: every lane moves 16 B per access (4 fp32 / 8 bf16 elements; Guideline 13),
// grid-stride over (M rows x F columns). a and b may be row-strided views: the fused W1|W3
// projection produces one (M, 2F) tensor whose column halves are a and b, so the gate reads it in
// place, and the backward writes da | db straight into the two halves of one (M, 2F) gradient —
// the fused GEMM's dY — with no split/cat copies. The backward is a single pass over (dh, a, b).
#include "cs336/kernels.h"

namespace cs336 {
namespace {

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

__device__ __forceinline__ void silu_mul_grad(float dh, float a, float b, float& da, float& db) {
  const float s = sigmoidf_(a);
  const float sa = a * s;
  db = dh * sa;
  da = dh * b * (s + sa * (1.f - s));
}

// element (r, c) of a/b/da/db at r*ld + c; h/dh contiguous (M, F).
// Every lane moves 16 B per access: VW = 4 fp32 or 8 16-bit elements (Guideline 13; the 8-B
// accesses of the first version ran these kernels at 83-90 % of the HBM roofline). Index math is
// 32-bit (the host keeps M*F/VW < 2^31): a 64-bit division per vector was a VALU cost of its own.
template <typename T>
struct Vec {
  static constexpr int VW = 16 / sizeof(typename Elem<T>::storage);
  float v[VW];
  __device__ __forceinline__ void load(const typename Elem<T>::storage* p) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    if constexpr (VW == 4) {
      v[0] = __uint_as_float(u.x); v[1] = __uint_as_float(u.y); v[2] = __uint_as_float(u.z); v[3] = __uint_as_float(u.w);
    } else {
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[2 * k] = Elem<T>::to_f((typename Elem<T>::storage)(w[k] & 0xffff));
        v[2 * k + 1] = Elem<T>::to_f((typename Elem<T>::storage)(w[k] >> 16));
      }
    }
  }
  __device__ __forceinline__ void store(typename Elem<T>::storage* p) const {
    uint4 u;
    if constexpr (VW == 4) {
      u = make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3]));
    } else {
      uint32_t w[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        w[k] = (uint32_t)Elem<T>::from_f(v[2 * k]) | ((uint32_t)Elem<T>::from_f(v[2 * k + 1]) << 16);
      u = make_uint4(w[0], w[1], w[2], w[3]);
    }
    *reinterpret_cast<uint4*>(p) = u;
  }
};

template <typename T>
__global__ __launch_bounds__(256) void silu_mul_fwd_kernel(const typename Elem<T>::storage* __restrict__ a,
                                                           const typename Elem<T>::storage* __restrict__ b,
                                                           typename Elem<T>::storage* __restrict__ h, int M,
                                                           int F, int ld) {
  constexpr int VW = Vec<T>::VW;
  const uint32_t Fv = (uint32_t)F / VW, n = (uint32_t)M * Fv;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t r = i / Fv, c = VW * (i - r * Fv);
    Vec<T> av, bv, o;
    av.load(a + (size_t)r * ld + c);
    bv.load(b + (size_t)r * ld + c);
#pragma unroll
    for (int k = 0; k < VW; ++k) o.v[k] = av.v[k] * sigmoidf_(av.v[k]) * bv.v[k];
    o.store(h + (size_t)r * F + c);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void silu_mul_bwd_kernel(const typename Elem<T>::storage* __restrict__ dh,
                                                           const typename Elem<T>::storage* __restrict__ a,
                                                           const typename Elem<T>::storage* __restrict__ b,
                                                           typename Elem<T>::storage* __restrict__ da,
                                                           typename Elem<T>::storage* __restrict__ db, int M,
                                                           int F, int ld) {
  constexpr int VW = Vec<T>::VW;
  const uint32_t Fv = (uint32_t)F / VW, n = (uint32_t)M * Fv;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t r = i / Fv, c = VW * (i - r * Fv);
    Vec<T> g, av, bv, oa, ob;
    g.load(dh + (size_t)r * F + c);
    av.load(a + (size_t)r * ld + c);
    bv.load(b + (size_t)r * ld + c);
#pragma unroll
    for (int k = 0; k < VW; ++k) silu_mul_grad(g.v[k], av.v[k], bv.v[k], oa.v[k], ob.v[k]);
    oa.store(da + (size_t)r * ld + c);
    ob.store(db + (size_t)r * ld + c);
  }
}

// 4-wide fallback (8-B accesses for 16-bit types) for views the 16-B kernels cannot take
template <typename T>
__global__ __launch_bounds__(256) void silu_mul_fwd4_kernel(const typename Elem<T>::storage* __restrict__ a,
                                                            const typename Elem<T>::storage* __restrict__ b,
                                                            typename Elem<T>::storage* __restrict__ h, int64_t M,
                                                            int64_t F, int64_t ld) {
  const int64_t F4 = F >> 2, n4 = M * F4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / F4, c = 4 * (i - r * F4);
    const float4 av = load4<T>(a + r * ld + c), bv = load4<T>(b + r * ld + c);
    float4 o;
    o.x = av.x * sigmoidf_(av.x) * bv.x;
    o.y = av.y * sigmoidf_(av.y) * bv.y;
    o.z = av.z * sigmoidf_(av.z) * bv.z;
    o.w = av.w * sigmoidf_(av.w) * bv.w;
    store4<T>(h + r * F + c, o);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void silu_mul_bwd4_kernel(const typename Elem<T>::storage* __restrict__ dh,
                                                            const typename Elem<T>::storage* __restrict__ a,
                                                            const typename Elem<T>::storage* __restrict__ b,
                                                            typename Elem<T>::storage* __restrict__ da,
                                                            typename Elem<T>::storage* __restrict__ db, int64_t M,
                                                            int64_t F, int64_t ld) {
  const int64_t F4 = F >> 2, n4 = M * F4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / F4, c = 4 * (i - r * F4);
    const float4 g = load4<T>(dh + r * F + c), av = load4<T>(a + r * ld + c), bv = load4<T>(b + r * ld + c);
    float4 oa, ob;
    silu_mul_grad(g.x, av.x, bv.x, oa.x, ob.x);
    silu_mul_grad(g.y, av.y, bv.y, oa.y, ob.y);
    silu_mul_grad(g.z, av.z, bv.z, oa.z, ob.z);
    silu_mul_grad(g.w, av.w, bv.w, oa.w, ob.w);
    store4<T>(da + r * ld + c, oa);
    store4<T>(db + r * ld + c, ob);
  }
}

// scalar tail for flat (M = 1) calls whose length is not a multiple of 4
template <typename T>
__global__ void silu_mul_tail(const typename Elem<T>::storage* a, const typename Elem<T>::storage* b,
                              typename Elem<T>::storage* h, int64_t start, int64_t n) {
  const int64_t i = start + threadIdx.x;
  if (i < n) {
    const float av = Elem<T>::to_f(a[i]);
    h[i] = Elem<T>::from_f(av * sigmoidf_(av) * Elem<T>::to_f(b[i]));
  }
}
template <typename T>
__global__ void silu_mul_bwd_tail(const typename Elem<T>::storage* dh, const typename Elem<T>::storage* a,
                                  const typename Elem<T>::storage* b, typename Elem<T>::storage* da,
                                  typename Elem<T>::storage* db, int64_t start, int64_t n) {
  const int64_t i = start + threadIdx.x;
  if (i < n) {
    float x, y;
    silu_mul_grad(Elem<T>::to_f(dh[i]), Elem<T>::to_f(a[i]), Elem<T>::to_f(b[i]), x, y);
    da[i] = Elem<T>::from_f(x);
    db[i] = Elem<T>::from_f(y);
  }
}

template <typename T>
void fwd_impl(const void* a, const void* b, void* h, int64_t M, int64_t F, int64_t ld, hipStream_t s) {
  typedef typename Elem<T>::storage S;
  constexpr int VW = Vec<T>::VW;
  if (M == 1) ld = F;
  // 16-B vectors need F, ld and the bases to be multiples of VW elements; else the scalar kernel
  const bool vec = F % VW == 0 && ld % VW == 0 && (reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) |
                                                   reinterpret_cast<uintptr_t>(h)) % 16 == 0 &&
                   M * (F / VW) < ((int64_t)1 << 31);
  if (vec) {
    hipLaunchKernelGGL(silu_mul_fwd_kernel<T>, dim3(stream_grid(M * (F / VW), 256)), dim3(256), 0, s, (const S*)a,
                       (const S*)b, (S*)h, (int)M, (int)F, (int)ld);
    return;
  }
  const int64_t Fv = F & ~(int64_t)3;  // tail only possible when M == 1
  if (Fv)
    hipLaunchKernelGGL(silu_mul_fwd4_kernel<T>, dim3(stream_grid(M * (Fv / 4), 256)), dim3(256), 0, s, (const S*)a,
                       (const S*)b, (S*)h, M, Fv, ld);
  if (F != Fv) hipLaunchKernelGGL(silu_mul_tail<T>, dim3(1), dim3(64), 0, s, (const S*)a, (const S*)b, (S*)h, Fv, F);
}
template <typename T>
void bwd_impl(const void* dh, const void* a, const void* b, void* da, void* db, int64_t M, int64_t F, int64_t ld,
              hipStream_t s) {
  typedef typename Elem<T>::storage S;
  constexpr int VW = Vec<T>::VW;
  if (M == 1) ld = F;
  const bool vec = F % VW == 0 && ld % VW == 0 &&
                   (reinterpret_cast<uintptr_t>(dh) | reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) |
                    reinterpret_cast<uintptr_t>(da) | reinterpret_cast<uintptr_t>(db)) % 16 == 0 &&
                   M * (F / VW) < ((int64_t)1 << 31);
  if (vec) {
    hipLaunchKernelGGL(silu_mul_bwd_kernel<T>, dim3(stream_grid(M * (F / VW), 256)), dim3(256), 0, s, (const S*)dh,
                       (const S*)a, (const S*)b, (S*)da, (S*)db, (int)M, (int)F, (int)ld);
    return;
  }
  const int64_t Fv = F & ~(int64_t)3;
  if (Fv)
    hipLaunchKernelGGL(silu_mul_bwd4_kernel<T>, dim3(stream_grid(M * (Fv / 4), 256)), dim3(256), 0, s, (const S*)dh,
                       (const S*)a, (const S*)b, (S*)da, (S*)db, M, Fv, ld);
  if (F != Fv)
    hipLaunchKernelGGL(silu_mul_bwd_tail<T>, dim3(1), dim3(64), 0, s, (const S*)dh, (const S*)a, (const S*)b, (S*)da,
                       (S*)db, Fv, F);
}

}  // namespace

void silu_mul_fwd(const void* a, const void* b, void* h, DType t, int64_t M, int64_t F, int64_t ld, hipStream_t s) {
  if (t == DType::F32) fwd_impl<float>(a, b, h, M, F, ld, s);
  else if (t == DType::BF16) fwd_impl<BF16>(a, b, h, M, F, ld, s);
  else fwd_impl<F16>(a, b, h, M, F, ld, s);
}

void silu_mul_bwd(const void* dh, const void* a, const void* b, void* da, void* db, DType t, int64_t M, int64_t F,
                  int64_t ld, hipStream_t s) {
  if (t == DType::F32) bwd_impl<float>(dh, a, b, da, db, M, F, ld, s);
  else if (t == DType::BF16) bwd_impl<BF16>(dh, a, b, da, db, M, F, ld, s);
  else bwd_impl<F16>(dh, a, b, da, db, M, F, ld, s);
}

}  // namespace cs336
