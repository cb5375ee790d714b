// Shared device helpers for the cs336 MI355X (gfx950 / CDNA4) kernels.
//
// Conventions: wave64 everywhere (never 32), fp32 accumulation, 16-bit storage as raw bits with
// conversions through clang's native __bf16 / _Float16 types (hipcc -O3 lowers the f32->bf16
// cast to v_cvt_pk_bf16_f32, which keeps NaNs NaN), 8-16 byte vector memory accesses per lane.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <type_traits>

namespace cs336 {

enum class DType : int { F32 = 0, F16 = 1, BF16 = 2 };

constexpr int kWave = 64;

// ------------------------------------------------------------------------------------------
// scalar conversions
// ------------------------------------------------------------------------------------------
typedef uint16_t bf16_t;  // raw bits
typedef uint16_t f16_t;   // raw bits

__device__ __forceinline__ float bf16_to_f32(bf16_t b) { return __uint_as_float(((uint32_t)b) << 16); }
__device__ __forceinline__ bf16_t f32_to_bf16(float f) {
  __bf16 h = (__bf16)f;
  return __builtin_bit_cast(bf16_t, h);
}
__device__ __forceinline__ float f16_to_f32(f16_t b) { return (float)__builtin_bit_cast(_Float16, b); }
__device__ __forceinline__ f16_t f32_to_f16(float f) { return __builtin_bit_cast(f16_t, (_Float16)f); }

// Element-type traits: T is the storage type (float, or a tag for 16-bit types).
struct BF16 {};
struct F16 {};

template <typename T> struct Elem;
template <> struct Elem<float> {
  typedef float storage;
  static __device__ __forceinline__ float to_f(float x) { return x; }
  static __device__ __forceinline__ float from_f(float x) { return x; }
};
template <> struct Elem<BF16> {
  typedef bf16_t storage;
  static __device__ __forceinline__ float to_f(bf16_t x) { return bf16_to_f32(x); }
  static __device__ __forceinline__ bf16_t from_f(float x) { return f32_to_bf16(x); }
};
template <> struct Elem<F16> {
  typedef f16_t storage;
  static __device__ __forceinline__ float to_f(f16_t x) { return f16_to_f32(x); }
  static __device__ __forceinline__ f16_t from_f(float x) { return f32_to_f16(x); }
};

// ------------------------------------------------------------------------------------------
// 4-wide vector load/store of any element type as float4 (16 B for f32, 8 B for 16-bit)
// ------------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ float4 load4(const typename Elem<T>::storage* p) {
  if constexpr (sizeof(typename Elem<T>::storage) == 4) {
    return *reinterpret_cast<const float4*>(p);
  } else {
    uint2 u = *reinterpret_cast<const uint2*>(p);
    typedef typename Elem<T>::storage S;
    S s0 = (S)(u.x & 0xffff), s1 = (S)(u.x >> 16), s2 = (S)(u.y & 0xffff), s3 = (S)(u.y >> 16);
    return make_float4(Elem<T>::to_f(s0), Elem<T>::to_f(s1), Elem<T>::to_f(s2), Elem<T>::to_f(s3));
  }
}

template <typename T>
__device__ __forceinline__ void store4(typename Elem<T>::storage* p, float4 v) {
  if constexpr (sizeof(typename Elem<T>::storage) == 4) {
    *reinterpret_cast<float4*>(p) = v;
  } else {
    uint32_t a = (uint32_t)Elem<T>::from_f(v.x) | ((uint32_t)Elem<T>::from_f(v.y) << 16);
    uint32_t b = (uint32_t)Elem<T>::from_f(v.z) | ((uint32_t)Elem<T>::from_f(v.w) << 16);
    *reinterpret_cast<uint2*>(p) = make_uint2(a, b);
  }
}

// Non-temporal forms (the `nt` cache-policy bit: the line is streamed, not kept for reuse) for tensors
// touched once now and next only after other work has cycled the caches -- the fp32 residual stream
// and its gradient (csrc/ops/rmsnorm.hip), so that the bf16 operands the next GEMM reads stay cached.
typedef __attribute__((ext_vector_type(4))) float cs336_f32x4_t;
typedef __attribute__((ext_vector_type(2))) unsigned int cs336_u32x2_t;
template <typename T>
__device__ __forceinline__ float4 load4_nt(const typename Elem<T>::storage* p) {
  if constexpr (sizeof(typename Elem<T>::storage) == 4) {
    const cs336_f32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const cs336_f32x4_t*>(p));
    return make_float4(v[0], v[1], v[2], v[3]);
  } else {
    const cs336_u32x2_t u = __builtin_nontemporal_load(reinterpret_cast<const cs336_u32x2_t*>(p));
    typedef typename Elem<T>::storage S;
    S s0 = (S)(u[0] & 0xffff), s1 = (S)(u[0] >> 16), s2 = (S)(u[1] & 0xffff), s3 = (S)(u[1] >> 16);
    return make_float4(Elem<T>::to_f(s0), Elem<T>::to_f(s1), Elem<T>::to_f(s2), Elem<T>::to_f(s3));
  }
}
template <typename T>
__device__ __forceinline__ void store4_nt(typename Elem<T>::storage* p, float4 v) {
  if constexpr (sizeof(typename Elem<T>::storage) == 4) {
    cs336_f32x4_t w;
    w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
    __builtin_nontemporal_store(w, reinterpret_cast<cs336_f32x4_t*>(p));
  } else {
    cs336_u32x2_t w;
    w[0] = (uint32_t)Elem<T>::from_f(v.x) | ((uint32_t)Elem<T>::from_f(v.y) << 16);
    w[1] = (uint32_t)Elem<T>::from_f(v.z) | ((uint32_t)Elem<T>::from_f(v.w) << 16);
    __builtin_nontemporal_store(w, reinterpret_cast<cs336_u32x2_t*>(p));
  }
}

// ------------------------------------------------------------------------------------------
// wave64 / block reductions
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Block-wide sum for blockDim.x = NT (multiple of 64). `red` must hold NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x / kWave, l = threadIdx.x % kWave;
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / kWave; ++i) t += red[i];
  __syncthreads();
  return t;
}
template <int NT>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x / kWave, l = threadIdx.x % kWave;
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / kWave; ++i) t = fmaxf(t, red[i]);
  __syncthreads();
  return t;
}

// Grid size for a memory-bound streaming kernel: enough blocks to fill 256 CUs several times
// over, capped (grid-stride loops cover the rest) — cdna_hip_programming.md Guideline 11.
inline int stream_grid(int64_t work_items, int block) {
  int64_t g = (work_items + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

#define CS336_HIP_CHECK(expr)                                                     \
  do {                                                                            \
    hipError_t _e = (expr);                                                       \
    if (_e != hipSuccess) {                                                       \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(_e), __FILE__, \
              __LINE__);                                                          \
      abort();                                                                    \
    }                                                                             \
  } while (0)

}  // namespace cs336
