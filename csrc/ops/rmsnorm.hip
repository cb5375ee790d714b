// RMSNorm forward/backward for MI355X (gfx950).
//
// Semantics: reference cs336-basics/cs336_basics/model.py:101-107 — y = w * (x * rsqrt(mean(x^2)+eps))
// computed in fp32, stored in the requested output dtype (bf16 under autocast: the next op is a
// bf16 GEMM, so the separate cast kernel of the eager path disappears).
//
// Layout: one wave64 per row, 4 rows per 256-thread workgroup. The row is read ONCE into
// registers (NV float4 per lane, NV chosen at dispatch from H), reduced with wave shuffles, and
// written from registers: 1 read + 1 write of the activation, which is the HBM floor.
// Backward: each wave walks a strided set of rows, producing dx per row and accumulating its dw
// partial in registers; partials (one per wave) go to a workspace that a column-tiled kernel
// reduces (deterministic, no float atomics).
#include <cstdlib>

#include "cs336/kernels.h"

namespace cs336 {
namespace {

// ADD: s = x + r is formed in fp32, stored (dtype TX: the residual stream) and normalized, so the
// residual add of a pre-norm block and the next RMSNorm read the stream once instead of twice.
template <typename TX, typename TW, typename TY, int NV, bool ADD = false, typename TR = TX>
__global__ __launch_bounds__(256) void rmsnorm_fwd_kernel(const typename Elem<TX>::storage* __restrict__ x,
                                                          const typename Elem<TW>::storage* __restrict__ w,
                                                          typename Elem<TY>::storage* __restrict__ y,
                                                          float* __restrict__ rstd, int64_t M, int H, float eps,
                                                          const typename Elem<TR>::storage* __restrict__ res = nullptr,
                                                          typename Elem<TX>::storage* __restrict__ s = nullptr) {
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int64_t row = (int64_t)blockIdx.x * 4 + wave;
  if (row >= M) return;
  const int H4 = H >> 2;
  const auto* xr = x + row * H;
  float4 v[NV];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int i = lane + kWave * k;
    if (i < H4) {
      // ADD (pre-norm residual): the stream x comes from a sublayer ago and s is read next a sublayer
      // from now (and in the backward): both stream past the caches (nt), which keeps the bf16 branch
      // output r (just written by a GEMM) and y (read next by a GEMM) cached
      v[k] = ADD ? load4_nt<TX>(xr + 4 * i) : load4<TX>(xr + 4 * i);
      if constexpr (ADD) {
        const float4 rv = load4<TR>(res + row * H + 4 * i);
        v[k].x += rv.x; v[k].y += rv.y; v[k].z += rv.z; v[k].w += rv.w;
        store4_nt<TX>(s + row * H + 4 * i, v[k]);
        // normalize what was stored (rounded to TX), like the unfused add -> rmsnorm
        if constexpr (!std::is_same<TX, float>::value) {
          v[k].x = Elem<TX>::to_f(Elem<TX>::from_f(v[k].x));
          v[k].y = Elem<TX>::to_f(Elem<TX>::from_f(v[k].y));
          v[k].z = Elem<TX>::to_f(Elem<TX>::from_f(v[k].z));
          v[k].w = Elem<TX>::to_f(Elem<TX>::from_f(v[k].w));
        }
      }
      ss += v[k].x * v[k].x + v[k].y * v[k].y + v[k].z * v[k].z + v[k].w * v[k].w;
    } else {
      v[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / (float)H + eps);
  if (lane == 0) rstd[row] = r;
  auto* yr = y + row * H;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int i = lane + kWave * k;
    if (i < H4) {
      const float4 wv = load4<TW>(w + 4 * i);
      float4 o;
      o.x = wv.x * (v[k].x * r);
      o.y = wv.y * (v[k].y * r);
      o.z = wv.z * (v[k].z * r);
      o.w = wv.w * (v[k].w * r);
      store4<TY>(yr + 4 * i, o);
    }
  }
}

// ADD: dx += dres (the gradient that reaches the residual stream from later layers) and, if dx2 is
// given, a bf16 copy of the sum for the branch whose output was bf16 (the o/w2 projection GEMM).
template <typename TDY, typename TX, typename TW, int NV, bool ADD = false>
__global__ __launch_bounds__(256) void rmsnorm_bwd_kernel(const typename Elem<TDY>::storage* __restrict__ dy,
                                                          const typename Elem<TX>::storage* __restrict__ x,
                                                          const typename Elem<TW>::storage* __restrict__ w,
                                                          const float* __restrict__ rstd,
                                                          typename Elem<TX>::storage* __restrict__ dx,
                                                          float* __restrict__ ws, int64_t M, int H,
                                                          const typename Elem<TX>::storage* __restrict__ dres = nullptr,
                                                          bf16_t* __restrict__ dx2 = nullptr) {
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int H4 = H >> 2;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t gw = (int64_t)blockIdx.x * 4 + wave;
  float4 wv[NV], dwp[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int i = lane + kWave * k;
    wv[k] = i < H4 ? load4<TW>(w + 4 * i) : make_float4(0.f, 0.f, 0.f, 0.f);
    dwp[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const float invH = 1.f / (float)H;
  for (int64_t row = gw; row < M; row += nw) {
    const auto* xr = x + row * H;
    const auto* dyr = dy + row * H;
    const float r = rstd[row];
    float4 xv[NV], gv[NV];
    // ADD: the residual gradient is loaded with x and dy, before the row reduction, so its latency
    // hides under the reduction instead of stalling the output pass
    float4 dv[ADD ? NV : 1];
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int i = lane + kWave * k;
      if (i < H4) {
        // ADD: the saved stream x and the residual gradient dres (a sublayer old) stream past the
        // caches; dy (just written by a GEMM) is read normally
        xv[k] = ADD ? load4_nt<TX>(xr + 4 * i) : load4<TX>(xr + 4 * i);
        gv[k] = load4<TDY>(dyr + 4 * i);
        if constexpr (ADD) dv[k] = load4_nt<TX>(dres + row * H + 4 * i);
      } else {
        xv[k] = gv[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (ADD) dv[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int k = 0; k < NV; ++k)
      dot += wv[k].x * gv[k].x * xv[k].x + wv[k].y * gv[k].y * xv[k].y + wv[k].z * gv[k].z * xv[k].z +
             wv[k].w * gv[k].w * xv[k].w;
    dot = wave_sum(dot);
    const float c = r * r * r * invH * dot;
    auto* dxr = dx + row * H;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int i = lane + kWave * k;
      if (i < H4) {
        float4 o;
        o.x = r * wv[k].x * gv[k].x - c * xv[k].x;
        o.y = r * wv[k].y * gv[k].y - c * xv[k].y;
        o.z = r * wv[k].z * gv[k].z - c * xv[k].z;
        o.w = r * wv[k].w * gv[k].w - c * xv[k].w;
        if constexpr (ADD) {
          o.x += dv[k].x; o.y += dv[k].y; o.z += dv[k].z; o.w += dv[k].w;
          if (dx2) store4<BF16>(dx2 + row * H + 4 * i, o);
        }
        if constexpr (ADD) store4_nt<TX>(dxr + 4 * i, o);  // (read next a sublayer from now)
        else store4<TX>(dxr + 4 * i, o);
        dwp[k].x += gv[k].x * xv[k].x * r;
        dwp[k].y += gv[k].y * xv[k].y * r;
        dwp[k].z += gv[k].z * xv[k].z * r;
        dwp[k].w += gv[k].w * xv[k].w * r;
      }
    }
  }
  // fold the 4 waves' dw partials through LDS (one partial row per workgroup, in wave order so the
  // result is deterministic), then workgroup partials are reduced by colsum_kernel
  extern __shared__ __attribute__((aligned(16))) float red[];  // H floats
  for (int wv_ = 0; wv_ < 4; ++wv_) {
    if (wave == wv_) {
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int i = lane + kWave * k;
        if (i < H4) {
          float4* rp = reinterpret_cast<float4*>(red + 4 * i);
          if (wv_ == 0) {
            *rp = dwp[k];
          } else {
            float4 a = *rp;
            a.x += dwp[k].x; a.y += dwp[k].y; a.z += dwp[k].z; a.w += dwp[k].w;
            *rp = a;
          }
        }
      }
    }
    __syncthreads();
  }
  float* wr = ws + (int64_t)blockIdx.x * H;
  for (int i = threadIdx.x; i < H4; i += 256) reinterpret_cast<float4*>(wr)[i] = reinterpret_cast<float4*>(red)[i];
}

// Fused-residual backward that also writes the bf16 residual gradient TRANSPOSED, dxT[h][m]
// (ld = M), for the narrow projections' weight-gradient GEMMs dW = dYᵀ·X (models/fused.py
// `_dy_transposed`): their dY is this gradient, and a token-contiguous dYᵀ is the layout hipBLASLt
// runs fastest. Workgroup = 16 consecutive rows (4 per wave); the bf16 rows are staged in LDS as
// [h][16 rows] (pitch 18 halves: 2-4-way write conflicts instead of 16) and leave as one 32-B
// piece per h, so two neighbouring workgroups fill a 64-B segment of a dxT row. Same math and dw
// partials (one row per workgroup) as rmsnorm_bwd_kernel<..., ADD=true>. M % 16 == 0 (host).
// R = 16 rows per workgroup while the staged tile fits 64 KB of LDS (H <= 1820), else 8.
template <typename TDY, typename TX, int NV, int R>
__global__ __launch_bounds__(256) void rmsnorm_bwd_add_t_kernel(const typename Elem<TDY>::storage* __restrict__ dy,
                                                                const typename Elem<TX>::storage* __restrict__ x,
                                                                const float* __restrict__ w,
                                                                const float* __restrict__ rstd,
                                                                typename Elem<TX>::storage* __restrict__ dx,
                                                                float* __restrict__ ws, int64_t M, int H,
                                                                const typename Elem<TX>::storage* __restrict__ dres,
                                                                bf16_t* __restrict__ dx2, bf16_t* __restrict__ dxt) {
  constexpr int kTRows = R, kTPitch = R + 2;  // rows per workgroup, LDS halves per h
  extern __shared__ __attribute__((aligned(16))) char lds[];  // H * kTPitch halves, reused for dw
  uint16_t* tile = reinterpret_cast<uint16_t*>(lds);
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int H4 = H >> 2;
  const int64_t row0 = (int64_t)blockIdx.x * kTRows;
  float4 wv[NV], dwp[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int i = lane + kWave * k;
    wv[k] = i < H4 ? load4<float>(w + 4 * i) : make_float4(0.f, 0.f, 0.f, 0.f);
    dwp[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const float invH = 1.f / (float)H;
  for (int rr = 0; rr < kTRows / 4; ++rr) {
    const int lr = wave * (kTRows / 4) + rr;  // row within the workgroup
    const int64_t row = row0 + lr;
    const float r = rstd[row];
    float4 xv[NV], gv[NV], dv[NV];
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int i = lane + kWave * k;
      if (i < H4) {
        xv[k] = load4<TX>(x + row * H + 4 * i);
        gv[k] = load4<TDY>(dy + row * H + 4 * i);
        dv[k] = load4<TX>(dres + row * H + 4 * i);
      } else {
        xv[k] = gv[k] = dv[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int k = 0; k < NV; ++k)
      dot += wv[k].x * gv[k].x * xv[k].x + wv[k].y * gv[k].y * xv[k].y + wv[k].z * gv[k].z * xv[k].z +
             wv[k].w * gv[k].w * xv[k].w;
    dot = wave_sum(dot);
    const float c = r * r * r * invH * dot;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int i = lane + kWave * k;
      if (i < H4) {
        float4 o;
        o.x = r * wv[k].x * gv[k].x - c * xv[k].x + dv[k].x;
        o.y = r * wv[k].y * gv[k].y - c * xv[k].y + dv[k].y;
        o.z = r * wv[k].z * gv[k].z - c * xv[k].z + dv[k].z;
        o.w = r * wv[k].w * gv[k].w - c * xv[k].w + dv[k].w;
        store4<TX>(dx + row * H + 4 * i, o);
        if (dx2) store4<BF16>(dx2 + row * H + 4 * i, o);
        uint16_t* tp = tile + (4 * i) * kTPitch + lr;
        tp[0] = __builtin_bit_cast(uint16_t, (__bf16)o.x);
        tp[kTPitch] = __builtin_bit_cast(uint16_t, (__bf16)o.y);
        tp[2 * kTPitch] = __builtin_bit_cast(uint16_t, (__bf16)o.z);
        tp[3 * kTPitch] = __builtin_bit_cast(uint16_t, (__bf16)o.w);
        dwp[k].x += gv[k].x * xv[k].x * r;
        dwp[k].y += gv[k].y * xv[k].y * r;
        dwp[k].z += gv[k].z * xv[k].z * r;
        dwp[k].w += gv[k].w * xv[k].w * r;
      }
    }
  }
  __syncthreads();
  // transposed store: thread -> (h, part): 8 rows of column h as one 16-B store
  constexpr int PARTS = kTRows / 8;
  for (int q = threadIdx.x; q < PARTS * H; q += 256) {
    const int h = q / PARTS, half = q % PARTS;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(tile + h * kTPitch + 8 * half);
    const uint4 v = make_uint4(src[0], src[1], src[2], src[3]);
    *reinterpret_cast<uint4*>(dxt + (int64_t)h * M + row0 + 8 * half) = v;
  }
  __syncthreads();
  // dw partials: fold the 4 waves through LDS (wave order: deterministic), one row per workgroup
  float* red = reinterpret_cast<float*>(lds);
  for (int wv_ = 0; wv_ < 4; ++wv_) {
    if (wave == wv_) {
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int i = lane + kWave * k;
        if (i < H4) {
          float4* rp = reinterpret_cast<float4*>(red + 4 * i);
          if (wv_ == 0) {
            *rp = dwp[k];
          } else {
            float4 a = *rp;
            a.x += dwp[k].x; a.y += dwp[k].y; a.z += dwp[k].z; a.w += dwp[k].w;
            *rp = a;
          }
        }
      }
    }
    __syncthreads();
  }
  float* wr = ws + (int64_t)blockIdx.x * H;
  for (int i = threadIdx.x; i < H4; i += 256) reinterpret_cast<float4*>(wr)[i] = reinterpret_cast<float4*>(red)[i];
}

// out[s][j] = sum over the partial rows p of split s of ws[p][j] (H % 4 == 0). Block = 64 float4
// columns x 8 row slices; the slices are folded through LDS in a fixed order (deterministic).
// grid (ceil(H/256), splits)
__global__ __launch_bounds__(512) void colsum_kernel(const float* __restrict__ ws, float* __restrict__ out, int P,
                                                     int H) {
  __shared__ float4 red[8][64];
  const int H4 = H >> 2;
  const int c4 = blockIdx.x * 64 + (threadIdx.x & 63), slice = threadIdx.x >> 6;
  const int S = gridDim.y, s = blockIdx.y;
  const int per = (P + S - 1) / S;
  const int p0 = s * per, p1 = min(P, p0 + per);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c4 < H4) {
    const float4* w4 = reinterpret_cast<const float4*>(ws);
#pragma unroll 4
    for (int p = p0 + slice; p < p1; p += 8) {
      const float4 v = w4[(int64_t)p * H4 + c4];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  red[slice][threadIdx.x & 63] = acc;
  __syncthreads();
  if (slice == 0 && c4 < H4) {
#pragma unroll
    for (int k = 1; k < 8; ++k) {
      const float4 v = red[k][threadIdx.x];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    reinterpret_cast<float4*>(out + (int64_t)s * H)[c4] = acc;
  }
}

template <int NV, typename F>
void dispatch_nv(int H, F&& f) {
  (void)NV;
  const int per_lane = (H / 4 + kWave - 1) / kWave;
  // 10 and 12 (d_model 2560 / 3072): rounding them up to 16 left the backward at one wave per SIMD
  // (256 VGPRs + AGPRs) and 66 % of the HBM rate in the 2.7b step (profiles/r4_2p7b_roofline_b24.md)
  if (per_lane <= 2) f(std::integral_constant<int, 2>{});
  else if (per_lane <= 4) f(std::integral_constant<int, 4>{});
  else if (per_lane <= 8) f(std::integral_constant<int, 8>{});
#ifndef CS336_RMS_NV16  // A/B probe: the round-3 rounding (10 and 12 -> 16)
  else if (per_lane <= 10) f(std::integral_constant<int, 10>{});
  else if (per_lane <= 12) f(std::integral_constant<int, 12>{});
#endif
  else if (per_lane <= 16) f(std::integral_constant<int, 16>{});
  else f(std::integral_constant<int, 32>{});
}

template <typename F>
void dispatch_type(DType t, F&& f) {
  switch (t) {
    case DType::F32: f(float{}); break;
    case DType::BF16: f(BF16{}); break;
    case DType::F16: f(F16{}); break;
  }
}

}  // namespace

void rmsnorm_fwd(const void* x, DType xt, const void* w, DType wt, void* y, DType yt, float* rstd, int64_t M,
                 int64_t H, float eps, hipStream_t s) {
  const dim3 grid((unsigned)((M + 3) / 4)), block(256);
  dispatch_nv<0>((int)H, [&](auto nv) {
    constexpr int NV = decltype(nv)::value;
    dispatch_type(xt, [&](auto tx) {
      using TX = decltype(tx);
      dispatch_type(wt, [&](auto tw) {
        using TW = decltype(tw);
        dispatch_type(yt, [&](auto ty) {
          using TY = decltype(ty);
          hipLaunchKernelGGL((rmsnorm_fwd_kernel<TX, TW, TY, NV>), grid, block, 0, s,
                             (const typename Elem<TX>::storage*)x, (const typename Elem<TW>::storage*)w,
                             (typename Elem<TY>::storage*)y, rstd, M, (int)H, eps);
        });
      });
    });
  });
}

// ~3 rows per wave: 1024 workgroups of 4 waves = 16 waves/CU (the occupancy the ~130-VGPR row loop
// allows) in one round for the XL rows (M = 12288), capped so the partial-row workspace stays small.
static int bwd_blocks(int64_t M) {
  int64_t nb = (M + 11) / 12;
  return (int)(nb < 1024 ? (nb > 0 ? nb : 1) : 1024);
}
constexpr int kColSplits = 16;

int rmsnorm_bwd_workspace_rows(int64_t M, int64_t H) {
  (void)H;
  return bwd_blocks(M) + kColSplits;  // rows of H floats: workgroup partials + split sums
}

void rmsnorm_bwd(const void* dy, DType dyt, const void* x, DType xt, const void* w, DType wt, const float* rstd,
                 void* dx, float* dw, float* workspace, int64_t M, int64_t H, hipStream_t s) {
  const int nb = bwd_blocks(M);
  const size_t lds = (size_t)H * sizeof(float);
  dispatch_nv<0>((int)H, [&](auto nv) {
    constexpr int NV = decltype(nv)::value;
    dispatch_type(dyt, [&](auto tdy) {
      using TDY = decltype(tdy);
      dispatch_type(xt, [&](auto tx) {
        using TX = decltype(tx);
        dispatch_type(wt, [&](auto tw) {
          using TW = decltype(tw);
          hipLaunchKernelGGL((rmsnorm_bwd_kernel<TDY, TX, TW, NV>), dim3(nb), dim3(256), lds, s,
                             (const typename Elem<TDY>::storage*)dy, (const typename Elem<TX>::storage*)x,
                             (const typename Elem<TW>::storage*)w, rstd, (typename Elem<TX>::storage*)dx, workspace,
                             M, (int)H);
        });
      });
    });
  });
  float* split = workspace + (int64_t)nb * H;
  const unsigned ct = (unsigned)((H / 4 + 63) / 64);
  hipLaunchKernelGGL(colsum_kernel, dim3(ct, kColSplits), dim3(512), 0, s, workspace, split, nb, (int)H);
  hipLaunchKernelGGL(colsum_kernel, dim3(ct, 1), dim3(512), 0, s, split, dw, kColSplits, (int)H);
}

// Fused residual variants: fp32 weights only (master weights), stream/branch dtypes fp32 or bf16.
template <typename F>
void dispatch_f32_bf16(DType t, F&& f) {
  if (t == DType::F32) f(float{});
  else f(BF16{});
}

void add_rmsnorm_fwd(const void* x, DType xt, const void* r, DType rt, const float* w, void* y, DType yt, void* sum,
                     float* rstd, int64_t M, int64_t H, float eps, hipStream_t s) {
  const dim3 grid((unsigned)((M + 3) / 4)), block(256);
  dispatch_nv<0>((int)H, [&](auto nv) {
    constexpr int NV = decltype(nv)::value;
    dispatch_f32_bf16(xt, [&](auto tx) {
      using TX = decltype(tx);
      dispatch_f32_bf16(rt, [&](auto tr) {
        using TR = decltype(tr);
        dispatch_f32_bf16(yt, [&](auto ty) {
          using TY = decltype(ty);
          hipLaunchKernelGGL((rmsnorm_fwd_kernel<TX, float, TY, NV, true, TR>), grid, block, 0, s,
                             (const typename Elem<TX>::storage*)x, w, (typename Elem<TY>::storage*)y, rstd, M, (int)H,
                             eps, (const typename Elem<TR>::storage*)r, (typename Elem<TX>::storage*)sum);
        });
      });
    });
  });
}

void rmsnorm_bwd_add(const void* dy, DType dyt, const void* x, DType xt, const float* w, const float* rstd,
                     const void* dres, void* dx, void* dx_bf16, float* dw, float* workspace, int64_t M, int64_t H,
                     hipStream_t s) {
  const int nb = bwd_blocks(M);
  const size_t lds = (size_t)H * sizeof(float);
  dispatch_nv<0>((int)H, [&](auto nv) {
    constexpr int NV = decltype(nv)::value;
    dispatch_f32_bf16(dyt, [&](auto tdy) {
      using TDY = decltype(tdy);
      dispatch_f32_bf16(xt, [&](auto tx) {
        using TX = decltype(tx);
        hipLaunchKernelGGL((rmsnorm_bwd_kernel<TDY, TX, float, NV, true>), dim3(nb), dim3(256), lds, s,
                           (const typename Elem<TDY>::storage*)dy, (const typename Elem<TX>::storage*)x, w, rstd,
                           (typename Elem<TX>::storage*)dx, workspace, M, (int)H,
                           (const typename Elem<TX>::storage*)dres, (bf16_t*)dx_bf16);
      });
    });
  });
  float* split = workspace + (int64_t)nb * H;
  const unsigned ct = (unsigned)((H / 4 + 63) / 64);
  hipLaunchKernelGGL(colsum_kernel, dim3(ct, kColSplits), dim3(512), 0, s, workspace, split, nb, (int)H);
  hipLaunchKernelGGL(colsum_kernel, dim3(ct, 1), dim3(512), 0, s, split, dw, kColSplits, (int)H);
}

}  // namespace cs336

namespace cs336 {

int rmsnorm_bwd_add_t_rows(int64_t H) {
  return H * 18 * 2 <= 65536 ? 16 : 8;
}

int rmsnorm_bwd_add_t_workspace_rows(int64_t M, int64_t H) {
  return (int)(M / rmsnorm_bwd_add_t_rows(H)) + kColSplits;
}

void rmsnorm_bwd_add_t(const void* dy, DType dyt, const void* x, DType xt, const float* w, const float* rstd,
                       const void* dres, void* dx, void* dx_bf16, void* dxt, float* dw, float* workspace, int64_t M,
                       int64_t H, hipStream_t s) {
  const int R = rmsnorm_bwd_add_t_rows(H);
  const int nb = (int)(M / R);
  const size_t tile = (size_t)H * (R + 2) * 2, red = (size_t)H * sizeof(float);
  const size_t lds = tile > red ? tile : red;
  dispatch_nv<0>((int)H, [&](auto nv) {
    constexpr int NV = decltype(nv)::value;
    dispatch_f32_bf16(dyt, [&](auto tdy) {
      using TDY = decltype(tdy);
      dispatch_f32_bf16(xt, [&](auto tx) {
        using TX = decltype(tx);
        auto go = [&](auto rr) {
          constexpr int RR = decltype(rr)::value;
          hipLaunchKernelGGL((rmsnorm_bwd_add_t_kernel<TDY, TX, NV, RR>), dim3(nb), dim3(256), lds, s,
                             (const typename Elem<TDY>::storage*)dy, (const typename Elem<TX>::storage*)x, w, rstd,
                             (typename Elem<TX>::storage*)dx, workspace, M, (int)H,
                             (const typename Elem<TX>::storage*)dres, (bf16_t*)dx_bf16, (bf16_t*)dxt);
        };
        if (R == 16) go(std::integral_constant<int, 16>{});
        else go(std::integral_constant<int, 8>{});
      });
    });
  });
  float* split = workspace + (int64_t)nb * H;
  const unsigned ct = (unsigned)((H / 4 + 63) / 64);
  hipLaunchKernelGGL(colsum_kernel, dim3(ct, kColSplits), dim3(512), 0, s, workspace, split, nb, (int)H);
  hipLaunchKernelGGL(colsum_kernel, dim3(ct, 1), dim3(512), 0, s, split, dw, kColSplits, (int)H);
}

}  // namespace cs336
