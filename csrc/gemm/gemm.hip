// cs336-build: agpr-accumulators
//
// bf16 MFMA GEMM for MI355X (gfx950) with fp32 accumulate, for the Transformer's projection
// GEMMs in all three training orientations:
//
//   forward      Y  = X · Wᵀ    A = X   [M][K]  (K-major)   B = W  [N][K] (K-major)
//   input grad   dX = dY · W    A = dY  [M][N]  (K-major)   B = W  [N][K] (MN-major)
//   weight grad  dW = dYᵀ · X   A = dYᵀ [M][N]  (MN-major)  B = X  [M][K] (MN-major)
//
// C[m][n] = Σ_k A(m,k)·B(k,n), with A(m,k) = a[m·lda + k] (K-major) or a[k·lda + m] (MN-major), and
// B(k,n) = b[n·ldb + k] (K-major) or b[k·ldb + n] (MN-major). Output bf16, fp32, or fp32 += (grad
// accumulation); split-K writes fp32 slabs reduced by splitk_reduce.
//
// Design (cdna_hip_programming.md §5):
// * tile BM×BN×64 with BM, BN ∈ {160, 192, 256}: the model's d_model = 1600 = 10·160 and
//   d_ff = 6400 = 25·256, so every projection GEMM of the XL/2.7b models tiles exactly and the grid
//   fills ~2 waves of 256 CUs (256² tiles leave 1600-wide outputs at 1.3 waves with a 25 %-used
//   edge tile). Waves WGM×WGN (8 waves = 2 per SIMD where the per-wave tile allows), each owning a
//   (BM/WGM)×(BN/WGN) block of v_mfma_f32_16x16x32_bf16 accumulators (kept in AGPRs);
// * both operands go global → LDS with global_load_lds_dwordx4 (no VGPR staging) into a 3-stage
//   ring (≤ 160 KiB LDS), one raw s_barrier per k-tile and a COUNTED vmcnt, so the next k-tile's
//   loads stay in flight across the barrier while the current one is multiplied;
// * K-major images are [rows][64] with the 16-B chunk XOR-swizzled by (row>>1)&7 (conflict-free
//   ds_read_b128 for the 16x16x32 fragment's lane groups); MN-major images are [64][rows] and give
//   the k-strided fragments with ds_read_b64_tr_b16, their 32-B slots XOR-swizzled per row so the
//   8 rows a 32-lane group touches land on distinct banks. glds writes lane-linear, so the swizzle
//   is applied to the per-lane GLOBAL source address and undone on the LDS read;
// * XCD-aware bijective block remap, then grouped tile order (8 tile-rows per group) so the tiles
//   co-resident on one XCD share A row-panels and B column-panels in that XCD's L2.
#include "cs336/kernels.h"

namespace cs336 {
namespace gemm {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int kBK = 64;

// Build switches (A/B variants via CS336_BUILD_VARIANT): vectorised LDS-staged epilogue, and
// s_setprio(1) around each MFMA cluster (cdna_hip_programming.md §5.5 T5).
#ifndef CS336_GEMM_EPI
#define CS336_GEMM_EPI 1
#endif
#ifndef CS336_GEMM_PRIO
#define CS336_GEMM_PRIO 0
#endif
constexpr int kGroupM = 8;

__device__ __forceinline__ int xcd_remap(int bid, int total) {
  const int xcd = bid & 7, q = total >> 3, r = total & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// ---- swizzles ---------------------------------------------------------------------------------
// K-major image: row r (128 B = 8 chunks of 8 bf16); physical chunk = logical ^ ((r>>1)&7)
__device__ __forceinline__ int kswz(int r) { return (r >> 1) & 7; }

// MN-major image: row r = k (S = 2·R bytes, R/16 slots of 32 B); physical slot = logical ^ mswz(r).
// A tr-read 32-lane group touches rows {0..3, 8..11} (+4 for the second read) of a k32 block,
// 32 B each: the XOR spreads those 8 rows over the 8 32-B bank slots of a 256-B bank row.
// (Measured: leaving 160-wide images unswizzled — a 2-way conflict between rows r and r+8 — in
// exchange for cheaper addressing was slower.)
template <int S>
__device__ __forceinline__ int mswz(int r) {
  if constexpr (S % 256 == 0) return (r & 3) | (((r >> 3) & 1) << 2);
  else if constexpr (S % 256 == 64) return (r >> 3) & 1;
  else if constexpr (S % 256 == 128) return ((r >> 1) & 1) | (((r >> 3) & 1) << 1);
  else if constexpr (S % 256 == 192) return (r >> 3) & 1;
  else return 0;
}

// ---- operand staging: per-thread element offsets of its 16-B chunks within one k-tile ----------
// K-major (R rows × 64 k): chunk q → row q>>3, physical chunk q&7 holding logical (q&7)^kswz(row)
// MN-major (64 k × R cols): chunk q → byte 16q of the [64][R] image
// The 8R chunks are dealt in rounds of NT (one per thread); a partial last round is issued by the
// first (HIGH=false) or last (HIGH=true) kRemW waves, so per-wave load counts stay wave-uniform.
template <int R, bool KMAJ, int NT, bool HIGH>
struct Stager {
  static constexpr int kChunks = R * kBK * 2 / 16;
  static constexpr int kFull = kChunks / NT;
  static constexpr int kRemW = (kChunks % NT) / 64;
  static constexpr int kPer = kFull + (kRemW ? 1 : 0);
  static_assert(kChunks % 64 == 0, "chunks must fill whole waves");
  uint32_t off[kPer];           // BYTE offset from the tile origin (row0 / col0 at k-tile 0)
  __amdgpu_buffer_rsrc_t rsrc;  // buffer descriptor based at the tile origin (wave-uniform)
  __device__ __forceinline__ static bool has_extra(int wave) {
    return kRemW && (HIGH ? wave >= NT / 64 - kRemW : wave < kRemW);
  }
  __device__ __forceinline__ static int chunk(int i, int wave, int lane) {
    // rounds 0..kFull-1: all waves; round kFull: the kRemW extra waves, packed from chunk kFull·NT
    if (i < kFull) return i * NT + wave * 64 + lane;
    const int w = HIGH ? wave - (NT / 64 - kRemW) : wave;
    return kFull * NT + w * 64 + lane;
  }
  __device__ __forceinline__ void init(const bf16_t* origin, int wave, int lane, int64_t ld) {
    // buffer_load ... lds: 32-bit per-lane VGPR offset + per-k-tile SGPR offset, no 64-bit address
    // math per load (the host guarantees every operand spans < 2 GiB)
    rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)origin, (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int q = chunk(i, wave, lane);
      if constexpr (KMAJ) {
        const int r = q >> 3, lc = (q & 7) ^ kswz(r);
        off[i] = 2u * (uint32_t)(r * ld + lc * 8);
      } else {
        constexpr int S = 2 * R;
        const int byte = 16 * q, r = byte / S, cb = byte % S;
        const int ls = (cb >> 5) ^ mswz<S>(r);
        off[i] = 2u * (uint32_t)(r * ld + ls * 16 + ((cb >> 4) & 1) * 8);
      }
    }
  }
  __device__ __forceinline__ void glds(uint32_t voff, uint32_t soff, char* dst) const {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)dst, 16, voff, soff, 0, 0);
  }
  // issue this wave's loads for one k-tile; soff = byte offset of the k-tile from the origin
  __device__ __forceinline__ void issue(uint32_t soff, char* img, int wave) const {
#pragma unroll
    for (int i = 0; i < kFull; ++i) glds(off[i], soff, img + 16 * (i * NT + wave * 64));
    if constexpr (kRemW > 0) {
      if (has_extra(wave)) {
        const int w = HIGH ? wave - (NT / 64 - kRemW) : wave;
        glds(off[kFull], soff, img + 16 * (kFull * NT + w * 64));
      }
    }
  }
};

// ---- fragments for v_mfma_f32_16x16x32_bf16: lane l holds (row/col l&15, k = 8(l>>4) + j) -----
__device__ __forceinline__ bf16x8 frag_k(const char* img, int row0, int ks, int lane) {
  const int r = row0 + (lane & 15);
  const int pc = (ks * 4 + (lane >> 4)) ^ kswz(r);
  return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(img + r * 128 + pc * 16));
}

template <int S>
__device__ __forceinline__ bf16x8 frag_mn(const char* img, int col0, int ks, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const int ra = ks * 32 + 8 * g + (i >> 2), rb = ra + 4;
  const int slot = col0 >> 4, within = 8 * (i & 3);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + ra * S + 32 * (slot ^ mswz<S>(ra)) + within));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + rb * S + 32 * (slot ^ mswz<S>(rb)) + within));
  s16x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return __builtin_bit_cast(bf16x8, v);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }

// round-to-nearest-even via v_cvt_pk_bf16_f32 (keeps NaN a NaN, unlike the integer trick)
__device__ __forceinline__ uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }

// ABL (ablation builds for profiling only): 1 = no global loads after the prologue (MFMA + LDS
// reads on stale tiles), 2 = no LDS fragment reads after the first k-tile (MFMA + glds).
template <int BM, int BN, int WGM, int WGN, bool AK, bool BKM, int OUT, int ABL = 0>
__global__ __launch_bounds__(WGM* WGN * 64, 1) void gemm_kernel(const GemmArgs p) {
  constexpr int NW = WGM * WGN, NT = NW * 64;
  constexpr int WTM = BM / WGM, WTN = BN / WGN, FM = WTM / 16, FN = WTN / 16;
  static_assert(WTM % 16 == 0 && WTN % 16 == 0, "per-wave tile must be a multiple of 16");
  constexpr int A_BYTES = BM * kBK * 2, B_BYTES = BN * kBK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int SA = 2 * BM, SB = 2 * BN;  // MN-major row bytes
  constexpr int NS = 3 * STAGE <= 160 * 1024 ? 3 : 2;  // ring depth
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE];
  using SAt = Stager<BM, AK, NT, false>;
  using SBt = Stager<BN, BKM, NT, true>;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;

  // tile coordinates: XCD remap, then grouped order
  const int tiles_n = p.N / BN, tiles_m = p.M / BM;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int per_group = kGroupM * tiles_n;
  const int first_m = (bid / per_group) * kGroupM;
  const int gsz = min(tiles_m - first_m, kGroupM);
  const int tm = first_m + (bid % per_group) % gsz, tn = (bid % per_group) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  // k-tile range of this split
  const int nkt_all = p.K / kBK, split = blockIdx.y, nsplit = gridDim.y;
  const int kt0 = (int)((int64_t)nkt_all * split / nsplit), kt1 = (int)((int64_t)nkt_all * (split + 1) / nsplit);
  const int nkt = kt1 - kt0;

  SAt sa;
  SBt sb;
  sa.init(p.a + (AK ? (int64_t)m0 * p.lda : (int64_t)m0), wave, lane, p.lda);
  sb.init(p.b + (BKM ? (int64_t)n0 * p.ldb : (int64_t)n0), wave, lane, p.ldb);
  const uint32_t a_step = AK ? 2 * kBK : 2u * kBK * (uint32_t)p.lda;  // bytes per k-tile
  const uint32_t b_step = BKM ? 2 * kBK : 2u * kBK * (uint32_t)p.ldb;
  // this wave's glds per k-tile: 0, 1 or 2 extra beyond the full rounds (wave-uniform)
  const int extra = (SAt::has_extra(wave) ? 1 : 0) + (SBt::has_extra(wave) ? 1 : 0);
  constexpr int LF = SAt::kFull + SBt::kFull;

  auto stage = [&](int kt, int slot) {
    char* img = smem + slot * STAGE;
    sa.issue((uint32_t)(kt0 + kt) * a_step, img, wave);
    sb.issue((uint32_t)(kt0 + kt) * b_step, img + A_BYTES, wave);
  };
  // own loads of the oldest outstanding tile retired, one younger tile may stay in flight
  auto wait_one_in_flight = [&]() {
    if (extra == 0) wait_vm<LF>();
    else if (extra == 1) wait_vm<LF + 1>();
    else wait_vm<LF + 2>();
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto read = [&](int kt, int ks, bf16x8 (&fa)[FM], bf16x8 (&fb)[FN]) {
    if (ABL == 2 && kt > 0) return;
    const char* ia = smem + (kt % NS) * STAGE;
    const char* ib = ia + A_BYTES;
#pragma unroll
    for (int i = 0; i < FM; ++i)
      fa[i] = AK ? frag_k(ia, wm * WTM + 16 * i, ks, lane) : frag_mn<SA>(ia, wm * WTM + 16 * i, ks, lane);
#pragma unroll
    for (int j = 0; j < FN; ++j)
      fb[j] = BKM ? frag_k(ib, wn * WTN + 16 * j, ks, lane) : frag_mn<SB>(ib, wn * WTN + 16 * j, ks, lane);
  };
  auto mma = [&](const bf16x8 (&fa)[FM], const bf16x8 (&fb)[FN]) {
    if constexpr (CS336_GEMM_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    if constexpr (CS336_GEMM_PRIO) __builtin_amdgcn_s_setprio(0);
  };
  // the wait that retires tile t (loads of t+1 may stay in flight) + the barrier that publishes it
  auto land = [&](int t) {
    if (NS == 3 && t + 1 < nkt) wait_one_in_flight();
    else wait_vm<0>();
    // this wave's reads of the slot about to be restaged have returned (WAR across the barrier)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    barrier();
  };

  // Software pipeline over half k-tiles (k32 steps): the fragment reads of the next half are in
  // flight while the MFMAs of the current half run, including across the per-tile barrier:
  //   read(kt,1) | mma(kt,0) | land(kt+1), restage | read(kt+1,0) | mma(kt,1)
  // Restaging tile kt's slot with tile kt+NS right after land(kt+1) is safe: every wave retired its
  // reads of tile kt (lgkmcnt(0)) before that barrier.
  bf16x8 fa0[FM], fb0[FN], fa1[FM], fb1[FN];
#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < nkt) stage(t, t);
  if (nkt > 0) {
    land(0);
    if (NS - 1 < nkt) stage(NS - 1, NS - 1);
    read(0, 0, fa0, fb0);
  }
  // ds_read instructions per half step (tr-read fragments take two)
  constexpr int NR = (AK ? 1 : 2) * FM + (BKM ? 1 : 2) * FN;
  // interleave the next half's fragment reads into this half's MFMA stream: 1 MFMA, 1 read, ...
  auto interleave = [&]() {
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
    }
    __builtin_amdgcn_sched_group_barrier(0x008, FM * FN - NR > 0 ? FM * FN - NR : 0, 0);
  };
  // K-major operands only (ds_read_b128 fragments): the next half's reads ride in this half's
  // MFMA stream. With tr-read (MN-major) fragments the doubled address/fragment registers spill
  // at the 256-VGPR budget of 2 waves/SIMD, so those variants read-then-multiply per half and
  // rely on the SIMD's other wave for overlap.
  constexpr bool PIPE = AK && BKM;
  for (int kt = 0; kt < nkt; ++kt) {
    if constexpr (PIPE) {
      mma(fa0, fb0);
      read(kt, 1, fa1, fb1);
      interleave();
      if (kt + 1 < nkt) {
        land(kt + 1);
        if (ABL != 1 && kt + NS < nkt) stage(kt + NS, (kt + NS) % NS);
        mma(fa1, fb1);
        read(kt + 1, 0, fa0, fb0);
        interleave();
      } else {
        mma(fa1, fb1);
      }
    } else {
      if (kt > 0) {
        land(kt);
        if (ABL != 1 && kt + NS - 1 < nkt) stage(kt + NS - 1, (kt + NS - 1) % NS);
        read(kt, 0, fa0, fb0);
      }
      mma(fa0, fb0);
      read(kt, 1, fa0, fb0);
      mma(fa0, fb0);
    }
  }

  // epilogue: lane holds C[4(l>>4)+r][l&15] of each 16x16 block
  const int rbase = m0 + wm * WTM + 4 * (lane >> 4), cbase = n0 + wn * WTN + (lane & 15);
  constexpr int ES = OUT == 0 ? 2 : 4;  // output element bytes
  float* cf = reinterpret_cast<float*>(p.c) + (OUT == 0 ? 0 : (int64_t)split * p.split_stride);
  uint16_t* ch = reinterpret_cast<uint16_t*>(p.c);
  const bool vec_ok = CS336_GEMM_EPI && ((p.ldc * ES) % 16 == 0) && ((reinterpret_cast<uintptr_t>(p.c) & 15) == 0) &&
                      ((p.split_stride * ES) % 16 == 0);
  if (vec_ok) {
    // Through LDS, one 16-row block of the wave's tile at a time: the accumulators go to a private
    // [16][WTN] scratch row-major, then come back as 16-B row chunks, so each global store
    // instruction writes whole 16-B pieces of contiguous rows (the per-lane layout above would
    // store 2-4 B per lane at a row stride: FM·FN·4 store instructions instead of ~FM·WTN/64).
    constexpr int RB = WTN * ES, CPR = RB / 16, NCH = 16 * CPR;  // row bytes, chunks per row / block
    static_assert(RB % 16 == 0, "wave tile row must be whole 16-B chunks");
    static_assert(NW * 16 * RB <= NS * STAGE, "epilogue scratch exceeds the LDS ring");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    barrier();  // every wave's last fragment reads of the ring are done
    char* scr = smem + wave * 16 * RB;
    const int r0 = m0 + wm * WTM, c0 = n0 + wn * WTN;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          char* d = scr + (4 * (lane >> 4) + r) * RB + (16 * j + (lane & 15)) * ES;
          if constexpr (OUT == 0) *reinterpret_cast<uint16_t*>(d) = f2bf(acc[i][j][r]);
          else *reinterpret_cast<float*>(d) = acc[i][j][r];
        }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int q0 = 0; q0 < NCH; q0 += 64) {
        const int q = q0 + lane;
        if (NCH % 64 == 0 || q < NCH) {
          const int rr = q / CPR, cc = q % CPR;
          const uint4 v = *reinterpret_cast<const uint4*>(scr + rr * RB + cc * 16);
          const int64_t row = r0 + 16 * i + rr;
          if constexpr (OUT == 0) {
            *reinterpret_cast<uint4*>(ch + row * p.ldc + c0 + cc * 8) = v;
          } else {
            float4* dst = reinterpret_cast<float4*>(cf + row * p.ldc + c0 + cc * 4);
            float4 f = __builtin_bit_cast(float4, v);
            if constexpr (OUT == 2) {
              const float4 o = *dst;
              f.x += o.x; f.y += o.y; f.z += o.z; f.w += o.w;
            }
            *dst = f;
          }
        }
      }
      __builtin_amdgcn_wave_barrier();  // reads of this block done before the next block's writes
    }
    return;
  }
  if constexpr (OUT == 0) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) ch[(int64_t)(rbase + 16 * i + r) * p.ldc + cbase + 16 * j] = f2bf(acc[i][j][r]);
  } else {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float* dst = cf + (int64_t)(rbase + 16 * i + r) * p.ldc + cbase + 16 * j;
          if constexpr (OUT == 2) *dst += acc[i][j][r];
          else *dst = acc[i][j][r];
        }
  }
}

// out[m][n] (+)= Σ_s slab[s][m][n]; slabs are dense [M][N] fp32 (ld = N)
template <bool ACC>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ slabs, float* __restrict__ out,
                                                            int64_t MN, int nsplit, int64_t ld_out, int N) {
  const int64_t i4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i4 >= MN) return;
  float4 s = *reinterpret_cast<const float4*>(slabs + i4);
  for (int k = 1; k < nsplit; ++k) {
    const float4 t = *reinterpret_cast<const float4*>(slabs + (int64_t)k * MN + i4);
    s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
  }
  const int64_t m = i4 / N, n = i4 % N;
  float4* dst = reinterpret_cast<float4*>(out + m * ld_out + n);
  if (ACC) {
    const float4 o = *dst;
    s.x += o.x; s.y += o.y; s.z += o.z; s.w += o.w;
  }
  *dst = s;
}

template <int BM, int BN, int WGM, int WGN>
bool launch_tile(const GemmArgs& p, bool ak, bool bk, int out, int splits, hipStream_t st) {
  const dim3 grid((unsigned)((p.M / BM) * (p.N / BN)), (unsigned)splits), block(WGM * WGN * 64);
#define CS336_GEMM_LAUNCH(AK, BKM, OUT)                                                          \
  do {                                                                                           \
    hipLaunchKernelGGL((gemm_kernel<BM, BN, WGM, WGN, AK, BKM, OUT>), grid, block, 0, st, p); \
    return true;                                                                                 \
  } while (0)
  if (ak && bk) {
    if (out == 0) CS336_GEMM_LAUNCH(true, true, 0);
    if (out == 1) CS336_GEMM_LAUNCH(true, true, 1);
    CS336_GEMM_LAUNCH(true, true, 2);
  }
  if (ak && !bk) {
    if (out == 0) CS336_GEMM_LAUNCH(true, false, 0);
    if (out == 1) CS336_GEMM_LAUNCH(true, false, 1);
    CS336_GEMM_LAUNCH(true, false, 2);
  }
  if (!ak && !bk) {
    if (out == 0) CS336_GEMM_LAUNCH(false, false, 0);
    if (out == 1) CS336_GEMM_LAUNCH(false, false, 1);
    CS336_GEMM_LAUNCH(false, false, 2);
  }
#undef CS336_GEMM_LAUNCH
  return false;
}

}  // namespace

bool tile_supported(int bm, int bn) {
  return (bm == 256 && bn == 160) || (bm == 160 && bn == 256) || (bm == 192 && bn == 160) || (bm == 160 && bn == 160);
}

// wave layouts: 8 waves (2 per SIMD) when both per-wave dims stay multiples of 16, else 4
bool gemm_bf16(const GemmArgs& p, int bm, int bn, bool a_kmajor, bool b_kmajor, int out_mode, int splits,
               hipStream_t s) {
  if (!a_kmajor && b_kmajor) return false;  // (MN, K) orientation is not used by the model
  switch (bm * 1000 + bn) {
    case 256160: return launch_tile<256, 160, 4, 2>(p, a_kmajor, b_kmajor, out_mode, splits, s);
    case 160256: return launch_tile<160, 256, 2, 4>(p, a_kmajor, b_kmajor, out_mode, splits, s);
    case 192160: return launch_tile<192, 160, 4, 2>(p, a_kmajor, b_kmajor, out_mode, splits, s);
    case 160160: return launch_tile<160, 160, 2, 2>(p, a_kmajor, b_kmajor, out_mode, splits, s);
    default: return false;
  }
}

void splitk_reduce(const float* slabs, float* out, int64_t M, int64_t N, int nsplit, int64_t ld_out, bool accumulate,
                   hipStream_t s) {
  const int64_t MN = M * N;
  const unsigned blocks = (unsigned)((MN / 4 + 255) / 256);
  if (accumulate)
    hipLaunchKernelGGL(splitk_reduce_kernel<true>, dim3(blocks), dim3(256), 0, s, slabs, out, MN, nsplit, ld_out, (int)N);
  else
    hipLaunchKernelGGL(splitk_reduce_kernel<false>, dim3(blocks), dim3(256), 0, s, slabs, out, MN, nsplit, ld_out, (int)N);
}

}  // namespace gemm
}  // namespace cs336
