// Shared building blocks of the CDNA4 FlashAttention-2 kernels (fa_fwd.hip, fa_bwd.hip).
//
// MFMA shapes: 16-bit inputs use v_mfma_f32_32x32x16_{bf16,f16}; fp32 inputs use the exact
// f32-in/f32-acc v_mfma_f32_32x32x2_f32 (no TF32-like shortcut exists on gfx950, and the
// 1e-2-tolerance fp32 tests deserve exact products).
//
// "Key on the register, query on the lane": every score tile is computed *transposed*
// (S^T = K Q^T, C[key][q]), so a lane owns one query row and its running max / sum / rescale are
// lane-local (one cross-half exchange per tile for the max). The S^T accumulator is then directly
// the B operand of the next MFMA (O^T += V^T P^T), see cdna_hip_programming.md §3 "An accumulator
// tile as the next MFMA's operand": registers 8s..8s+7 packed to bf16 are k-step s, whose k order
// is key = 16s + 8(j>>2) + 4h + (j&3); the V^T operand is gathered in exactly that key order with
// ds_read_b64_tr_b16 hardware-transposed LDS reads.
//
// LDS images: one XOR swizzle on 16-byte chunks (function of the row length) makes BOTH the
// row-fragment reads (ds_read_b128, 16 lanes on 16 different rows) and the transposed reads
// (ds_read_b64_tr_b16, a 32-lane half on 4 rows x 64 B) bank-conflict free, so a K (or Q/dO)
// tile staged once serves row-wise and column-wise consumers (T2 + T10 of the guide).
#pragma once

#include "cs336/common.h"
#include "cs336/kernels.h"

namespace cs336 {
namespace fa {

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
constexpr float kNegBig = -1e30f;
// Online-softmax rescale threshold in log2 units (guide T13): the running max is only raised
// (and O, l rescaled) when some row's tile max exceeds it by more than this, so P <= 2^8.
constexpr float kRescaleThr = 8.f;

// raw v_exp_f32 (2^x); exp2f() adds a denormal-range fixup sequence we do not need here
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// ---- lane halves: v_permlane32_swap (guide T12 / T21) ------------------------------------------
// lane i's value combined with lane i ^ 32's by one half swap, instead of a ds_bpermute round trip
// (__shfl_xor(x, 32)); both operations are commutative, so every lane gets the same bits as before
__device__ __forceinline__ float xhalf_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xhalf_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// wave index as a provably wave-uniform (SGPR) value, so per-wave tile skips / mask decisions
// compile to scalar branches instead of predicated vector code
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// ---- padded head dims ------------------------------------------------------------------------
// d_head 80 (the 2.7b model) runs as 96 = 3 x 32 inside the kernels: d 80..95 are zero in the LDS
// images and fragments (zeros add nothing to S, dP or the d-sums) and never loaded or stored, so
// there is no host-side padding copy and 20 % (not 60 %) extra MFMA work.
template <int D>
struct PadD {
  static constexpr int value = D % 32 == 0 ? D : (D + 31) / 32 * 32;
};

// ---- swizzle: physical 16-B chunk = chunk ^ swz(row) --------------------------------------
template <int RB>
__host__ __device__ __forceinline__ int swz(int r) {
  if constexpr (RB == 64) {
    return (r >> 2) & 3;
  } else if constexpr (RB == 192) {
    // 12-chunk rows (d_head 80 stored padded to 96): row r starts at slot 12r mod 16, so rows with the
    // same r mod 4 share a slot pair; XOR-ing the chunk's low 2 bits with (r>>2)&3 spreads every
    // ds_read_b128 lane group and every ds_read_b64_tr_b16 half over distinct banks (checked by
    // enumeration of both access patterns); chunk groups of 4 stay inside the 12-chunk row
    return (r >> 2) & 3;
  } else if constexpr (RB == 128) {
    const int g = (r >> 1) & 7;
    return g ^ ((g & 1) << 2);
  } else {
    return ((r & 3) << 2) | ((r >> 2) & 3);
  }
}
template <int RB>
__host__ __device__ __forceinline__ int lds_off(int r, int chunk) {
  return r * RB + ((chunk ^ swz<RB>(r)) << 4);
}

// ---- 16-bit MFMA traits ------------------------------------------------------------------
template <typename T> struct Mma16;
template <> struct Mma16<BF16> {
  typedef bf16x8 frag;
  static __device__ __forceinline__ f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ frag pack(float x0, float x1, float x2, float x3, float x4, float x5, float x6,
                                              float x7) {
    frag f;
    f[0] = (__bf16)x0; f[1] = (__bf16)x1; f[2] = (__bf16)x2; f[3] = (__bf16)x3;
    f[4] = (__bf16)x4; f[5] = (__bf16)x5; f[6] = (__bf16)x6; f[7] = (__bf16)x7;
    return f;
  }
};
template <> struct Mma16<F16> {
  typedef f16x8 frag;
  static __device__ __forceinline__ f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ frag pack(float x0, float x1, float x2, float x3, float x4, float x5, float x6,
                                              float x7) {
    frag f;
    f[0] = (_Float16)x0; f[1] = (_Float16)x1; f[2] = (_Float16)x2; f[3] = (_Float16)x3;
    f[4] = (_Float16)x4; f[5] = (_Float16)x5; f[6] = (_Float16)x6; f[7] = (_Float16)x7;
    return f;
  }
};

template <typename T>
__device__ __forceinline__ typename Mma16<T>::frag as_frag(uint4 u) {
  return __builtin_bit_cast(typename Mma16<T>::frag, u);
}

// pack accumulator registers 8s..8s+7 of a 32x32 tile into the bf16/f16 operand of k-step s
template <typename T>
__device__ __forceinline__ typename Mma16<T>::frag pack_acc(const f32x16& a, int s) {
  return Mma16<T>::pack(a[8 * s + 0], a[8 * s + 1], a[8 * s + 2], a[8 * s + 3], a[8 * s + 4], a[8 * s + 5],
                        a[8 * s + 6], a[8 * s + 7]);
}

__device__ __forceinline__ f32x16 mma_f32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// Row fragment (A operand of a 32x32x16 MFMA over a [row][d] LDS image): lane reads row
// `row0 + (lane&31)`, 8 elements starting at d = 16*ks + 8*(lane>>5).
template <typename T, int RB>
__device__ __forceinline__ typename Mma16<T>::frag lds_row_frag(const char* img, int row0, int ks, int lane) {
  const int r = row0 + (lane & 31);
  const int chunk = 2 * ks + (lane >> 5);
  return as_frag<T>(*reinterpret_cast<const uint4*>(img + lds_off<RB>(r, chunk)));
}

// Transposed fragment (A operand = image^T): lane (d = dt*32 + (lane&31), half h) gets the 8
// elements image[row0 + 16s + 8(j>>2) + 4h + (j&3)][d], j = 0..7, via two ds_read_b64_tr_b16.
template <typename T, int RB>
__device__ __forceinline__ typename Mma16<T>::frag lds_tr_frag(const char* img, int row0, int s, int dt, int lane) {
  const int i = lane & 15, gq = (lane >> 4) & 1, h = lane >> 5;
  const int chunk = dt * 4 + gq * 2 + ((i & 3) >> 1);
  const int within = (i & 1) * 8;
  const int ra = row0 + 16 * s + 4 * h + (i >> 2);
  const int rb = ra + 8;
  const lds_s16x4* pa = (const lds_s16x4*)(img + lds_off<RB>(ra, chunk) + within);
  const lds_s16x4* pb = (const lds_s16x4*)(img + lds_off<RB>(rb, chunk) + within);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)pa);
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)pb);
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return __builtin_bit_cast(typename Mma16<T>::frag, v);
}

// f32 images: 4 consecutive floats of row r starting at element e (e % 4 == 0)
template <int RB>
__device__ __forceinline__ float4 lds_f4(const char* img, int r, int e) {
  return *reinterpret_cast<const float4*>(img + lds_off<RB>(r, e >> 2));
}
template <int RB>
__device__ __forceinline__ float lds_f1(const char* img, int r, int e) {
  return *reinterpret_cast<const float*>(img + lds_off<RB>(r, e >> 2) + ((e & 3) << 2));
}

// ---- fused RoPE (interleaved pairs) on 16-byte chunks ---------------------------------------
// Rotation R(pos) of the pairs (d0, d0+1), ... of one chunk, computed in fp32 from the (ctx, D/2)
// cos/sin cache (L2-resident); sgn = -1 applies R^T (the backward's inverse rotation).
struct Rope {
  const float* cs;
  const float* sn;
  int half;
};

template <typename T>
__device__ __forceinline__ uint4 rope_chunk(uint4 u, const Rope& r, int64_t pos, int d0, float sgn) {
  typedef typename Elem<T>::storage S;
  if constexpr (sizeof(S) == 4) {
    const float2 c = *reinterpret_cast<const float2*>(r.cs + pos * r.half + (d0 >> 1));
    const float2 s = *reinterpret_cast<const float2*>(r.sn + pos * r.half + (d0 >> 1));
    float4 v = __builtin_bit_cast(float4, u);
    const float s0 = sgn * s.x, s1 = sgn * s.y;
    float4 o;
    o.x = c.x * v.x - s0 * v.y;
    o.y = s0 * v.x + c.x * v.y;
    o.z = c.y * v.z - s1 * v.w;
    o.w = s1 * v.z + c.y * v.w;
    return __builtin_bit_cast(uint4, o);
  } else {
    const float4 c = *reinterpret_cast<const float4*>(r.cs + pos * r.half + (d0 >> 1));
    const float4 s = *reinterpret_cast<const float4*>(r.sn + pos * r.half + (d0 >> 1));
    const float cc[4] = {c.x, c.y, c.z, c.w};
    const float ss[4] = {sgn * s.x, sgn * s.y, sgn * s.z, sgn * s.w};
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float a = Elem<T>::to_f((S)(w[i] & 0xffff)), b = Elem<T>::to_f((S)(w[i] >> 16));
      const float x = cc[i] * a - ss[i] * b, y = ss[i] * a + cc[i] * b;
      w[i] = (uint32_t)Elem<T>::from_f(x) | ((uint32_t)Elem<T>::from_f(y) << 16);
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// Split form for software-pipelined staging: fetch the coefficients together with the tile's
// global loads (no use of the loaded data yet), rotate when the registers are written to LDS.
struct RopeCoef {
  float4 c, s;
};
template <typename T>
__device__ __forceinline__ RopeCoef rope_coef(const Rope& r, int64_t pos, int d0) {
  RopeCoef k;
  if constexpr (sizeof(typename Elem<T>::storage) == 4) {
    const float2 c = *reinterpret_cast<const float2*>(r.cs + pos * r.half + (d0 >> 1));
    const float2 s = *reinterpret_cast<const float2*>(r.sn + pos * r.half + (d0 >> 1));
    k.c = make_float4(c.x, c.y, 0.f, 0.f);
    k.s = make_float4(s.x, s.y, 0.f, 0.f);
  } else {
    k.c = *reinterpret_cast<const float4*>(r.cs + pos * r.half + (d0 >> 1));
    k.s = *reinterpret_cast<const float4*>(r.sn + pos * r.half + (d0 >> 1));
  }
  return k;
}
template <typename T>
__device__ __forceinline__ uint4 rope_apply(uint4 u, const RopeCoef& k) {
  typedef typename Elem<T>::storage S;
  if constexpr (sizeof(S) == 4) {
    float4 v = __builtin_bit_cast(float4, u);
    float4 o;
    o.x = k.c.x * v.x - k.s.x * v.y;
    o.y = k.s.x * v.x + k.c.x * v.y;
    o.z = k.c.y * v.z - k.s.y * v.w;
    o.w = k.s.y * v.z + k.c.y * v.w;
    return __builtin_bit_cast(uint4, o);
  } else {
    const float cc[4] = {k.c.x, k.c.y, k.c.z, k.c.w};
    const float ss[4] = {k.s.x, k.s.y, k.s.z, k.s.w};
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float a = Elem<T>::to_f((S)(w[i] & 0xffff)), b = Elem<T>::to_f((S)(w[i] >> 16));
      const float x = cc[i] * a - ss[i] * b, y = ss[i] * a + cc[i] * b;
      w[i] = (uint32_t)Elem<T>::from_f(x) | ((uint32_t)Elem<T>::from_f(y) << 16);
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// inverse rotation of 4 consecutive fp32 accumulator values (d0 % 4 == 0) before the dQ/dK store
__device__ __forceinline__ void rope_inv4(float& v0, float& v1, float& v2, float& v3, const Rope& r, int64_t pos,
                                          int d0) {
  const float2 c = *reinterpret_cast<const float2*>(r.cs + pos * r.half + (d0 >> 1));
  const float2 s = *reinterpret_cast<const float2*>(r.sn + pos * r.half + (d0 >> 1));
  const float a0 = c.x * v0 + s.x * v1, a1 = -s.x * v0 + c.x * v1;
  const float b0 = c.y * v2 + s.y * v3, b1 = -s.y * v2 + c.y * v3;
  v0 = a0; v1 = a1; v2 = b0; v3 = b1;
}

// ---- direct-to-LDS tile staging (buffer_load ... lds) ------------------------------------------
// One ROWS x RB tile of a strided [row][d] operand (K, V, Q or dO of one head) goes global -> LDS
// without VGPRs: each wave-instruction moves 64 lanes x 16 B into 1 KB of consecutive LDS, so the
// image's XOR swizzle is applied to each lane's GLOBAL source chunk (slot q = row r, physical chunk
// pc holds logical chunk pc ^ swz(r)) and undone by the usual lds_off reads. Rows past the tile's
// valid count and the zero padding chunks of d_head 80 (chunk >= CREAL) read out of the buffer
// descriptor's range; the kernel zero-fills its LDS ring once at entry, so such slots hold zeros or
// finite stale rows, which the masks turn into exact zeros (P = 0 for keys >= Nk / queries >= Nq).
// One LDS-DMA wave instruction (buffer_load_dwordx4 ... lds: 64 lanes x 16 B into 1 KB of LDS at
// the wave-uniform address lds_addr) in inline asm. Issued through the builtin, the load is a pending
// LDS write that hipcc's waitcnt pass cannot disambiguate from the kernel's LDS reads, so it put
// s_waitcnt vmcnt(0) in front of the first read after every issue -- draining the prefetch ring at
// each tile. Every DMA of these kernels goes through here (M0 is written by no other code in them);
// its data is waited for by the explicit counted wait_vmcnt + dma_barrier before any read.
__device__ __forceinline__ void dma16(const __amdgpu_buffer_rsrc_t& rs, uint32_t lds_addr, uint32_t voff, uint32_t soff) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %2, %3 offen lds"
               :
               : "v"(voff), "s"(lds_addr), "s"(rs), "s"(soff)
               : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const void*)p;
}

template <int ROWS, int RB, int CREAL, int ES>
struct TileDma {
  static constexpr int CPR = RB / 16;
  static constexpr int PER_WAVE = ROWS * CPR / 256;  // 4 waves x 64 lanes per round
  static_assert(ROWS * CPR % 256 == 0, "DMA rounds must be whole");
  uint32_t voff[PER_WAVE];  // per-lane byte offsets from the tile's first row (0x80000000: padding)

  __device__ __forceinline__ void init(int wave, int lane, int64_t ld) {
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) {
      const int q = (i * 4 + wave) * 64 + lane;
      const int r = q / CPR, pc = q % CPR, c = pc ^ swz<RB>(r);
      voff[i] = c < CREAL ? (uint32_t)(((int64_t)r * ld + c * (16 / ES)) * ES) : 0x80000000u;
    }
  }
  // rows_valid rows from `tile` are loaded; (wave-uniform arguments)
  __device__ __forceinline__ void issue(const void* tile, int rows_valid, int64_t ld, char* img, int wave) const {
    const uint32_t bytes = rows_valid > 0 ? (uint32_t)((int64_t)(rows_valid - 1) * ld * ES + CREAL * 16) : 0u;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)tile, (short)0, (int)bytes, 0x00020000);
    const uint32_t base = lds_addr(img);
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) dma16(rsrc, base + 1024 * (i * 4 + wave), voff[i], 0);
  }
};

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  // A full drain is also stated to the compiler (vmcnt 0; expcnt / lgkmcnt left at their maxima),
  // which cannot see the inline-asm wait above: otherwise operands it loaded earlier (the V / K / Q
  // fragments kept in registers) count as pending forever after, and it re-inserts vmcnt(0) in
  // front of their MFMAs inside the tile loop -- a drain of the LDS-DMA prefetch (invisible to it)
  // at every tile. At runtime this adds nothing: the counter is already 0.
  if constexpr (N == 0) __builtin_amdgcn_s_waitcnt(0x0F70);
}

// Workgroup barrier that keeps LDS-DMA in flight: __syncthreads()'s fence makes hipcc emit
// s_waitcnt vmcnt(0) in front of the s_barrier, and an LDS-DMA is a pending write on the VM counter,
// so it drained the whole prefetch ring at every tile (the counted wait_vmcnt before it did nothing).
// Here: this wave's LDS reads/writes retired (lgkmcnt(0): the WAR/RAW for other waves), then a raw
// s_barrier the compiler cannot move anything across.
__device__ __forceinline__ void dma_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// zero a block of LDS (all 256 threads; bytes % 4096 == 0)
__device__ __forceinline__ void lds_zero(char* p, int bytes) {
  for (int o = threadIdx.x * 16; o < bytes; o += 256 * 16) *reinterpret_cast<uint4*>(p + o) = make_uint4(0, 0, 0, 0);
}

// key (or row) index held by accumulator register `reg` of lane-half h in a 32x32 tile
__host__ __device__ __forceinline__ int acc_row(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

// Staging position of query row r (0..63) of a backward tile so that lane-half h of 32-row group t
// finds its 16 accumulator rows (acc_row(reg, h)) at 32t + 16h + reg: one 64-B read per lane loads
// a row-constant accumulator (fa_bwd.hip dK/dV kernel).
__host__ __device__ __forceinline__ int row_perm(int r) {
  return (r & ~31) | (((r >> 2) & 1) << 4) | (((r >> 3) & 3) << 2) | (r & 3);
}
// LDS-DMA form of the same staging: 16 lanes move 16 B each; lane c (LDS chunk c = positions
// 4c..4c+3) reads source chunk row_perm_src_chunk(c) (rows 4 src .. 4 src + 3)
__host__ __device__ __forceinline__ int row_perm_src_chunk(int c) { return 8 * (c >> 3) + 2 * (c & 3) + ((c >> 2) & 1); }

// Bijective XCD-aware remap of a 1-D block id: blocks that share a (batch, head) — and hence the
// same K/V (or Q/dO) stream — become contiguous in the remapped order, i.e. share one XCD's L2
// (guide T1, bijective variant for totals not divisible by 8).
__host__ __device__ __forceinline__ int xcd_remap(int bid, int total) {
  const int xcd = bid & 7, q = total >> 3, r = total & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// (batch*head, tile level) of block `bid` for a grid of nbh*nt blocks. order 0: xcd_remap, levels of
// one head adjacent. order 1 (causal LPT): callers map level 0 to the heaviest tile under the causal
// mask. Heads are taken in groups of `grp`; inside a group every head's level-0 tile is dispatched
// before any level-1 tile, ..., so the short tiles fill the tail of the grid instead of a long one
// starting last (the light tiles of one group run next to the heavy ones of the next). The host sizes
// `grp` so that the group's K/V fit one XCD's 4 MB L2 (fill_attn): at N 16384 that is one head, i.e.
// the per-head order, which measured 20 % faster there than level-major over all heads. With
// nbh % 8 == 0 each XCD (bid & 7) keeps a contiguous range of heads, grouped inside the range;
// otherwise the groups (of 8*grp heads) run over the whole grid. order 2 forces the whole-grid form.
// Measurements: profiles/r1_fa_lpt_order.md.
__host__ __device__ __forceinline__ void grouped_levels(int j, int nh, int nt, int grp, int& hd, int& lvl) {
  const int g = grp < nh ? grp : nh;
  const int gi = j / (g * nt), h0 = gi * g;
  const int gs = nh - h0 < g ? nh - h0 : g;  // the last group may be short
  const int r = j - gi * g * nt;
  lvl = r / gs;
  hd = h0 + r % gs;
}

__host__ __device__ __forceinline__ void tile_order(int bid, int nbh, int nt, int order, int grp, int& bh, int& lvl) {
  if (order == 1 && (nbh & 7) == 0) {
    const int per = nbh >> 3;
    int hd;
    grouped_levels(bid >> 3, per, nt, grp, hd, lvl);
    bh = (bid & 7) * per + hd;
  } else if (order != 0) {
    grouped_levels(bid, nbh, nt, 8 * grp, bh, lvl);
  } else {
    const int rid = xcd_remap(bid, nbh * nt);
    bh = rid / nt;
    lvl = rid % nt;
  }
}

}  // namespace fa
}  // namespace cs336
