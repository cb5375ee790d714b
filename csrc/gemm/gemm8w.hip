// cs336-build: agpr-accumulators
//
// "gemm8w": the weight-gradient GEMMs of the Transformer step, dW = dYᵀ·X, straight from the
// token-major activations (no dYᵀ / Xᵀ transposes):
//
//   C[m][n] = Σ_t A[t][m] · B[t][n]     A = dY [tokens][N_out], B = X [tokens][K_in], fp32 out
//
// (or the transposed roles, C stored transposed, when that tiles the shape better). Both operands are
// "MN-major": the contraction index t is the row of the stored matrix. Structure follows gemm8
// (csrc/gemm/gemm8.hip: 256 × 64·FN tile, BK 64, 8 waves 2 × 4, second wave group one barrier
// behind, two LDS-DMA stages, one counted vmcnt per K-tile), with what MN-major operands change:
//
// * LDS images are [64 t][R] (R = 256 or 320 columns, rows of 512 / 640 B) and every 16x16x32
//   fragment is two ds_read_b64_tr_b16 (the transposed LDS read: lane i of a 16-lane group gets
//   column i of 4 rows). The 32-B slots of each row are XOR-swizzled by the row so the 8 rows a
//   32-lane half reads land on 8 different bank slots (conflict-free for both row lengths); as
//   always with LDS-DMA, the swizzle is applied to the per-lane global source address;
// * a K-tile runs as 4 phases split along K -- (k 0-31, rows 0-63), (k 0-31, rows 64-127),
//   (k 32-63, rows 0-63), (k 32-63, rows 64-127) -- because a DMA granule holds whole t-rows: the
//   t-rows 0-31 of a stage are free after phase 2 and restaged with the K-tile after next there, the
//   t-rows 32-63 at the next K-tile's phase 1; each half is waited for (counted vmcnt) only one phase
//   before its first read -- the first half at phase 3 of the previous K-tile, the second half at
//   phase 1 of its own -- so both have five phases in flight (the round-5 form retired the whole
//   next K-tile at phase 3: its second half had three);
// * fp32 accumulators leave straight from registers, 16 B per lane (4 consecutive output columns, or
//   4 consecutive output rows when the result is stored transposed), into the DDP bucket or a
//   split-K slab; rows beyond M (the last, padded row tile) are computed and dropped.
#include "cs336/kernels.h"
#include "gemm8.h"

namespace cs336 {
namespace gemm8 {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int BM = 256, BK = 64, NT = 512;
constexpr int kGroupM = 8;

__device__ __forceinline__ int xcd_remap(int bid, int total) {
  const int xcd = bid & 7, q = total >> 3, r = total & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}
__device__ __forceinline__ void sbarrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
template <int N>
__device__ __forceinline__ void vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// 32-B slot swizzle of an MN-major image row t (S = row bytes): the 8 rows {0..3, 8..11} (+4) a
// 32-lane half of a transposed fragment read touches map to 8 distinct slots of a 256-B bank row
template <int S>
__device__ __forceinline__ int swz(int t) {
  static_assert(S % 256 == 0 || S % 256 == 128, "row bytes");
  if constexpr (S % 256 == 0) return (t & 3) | (((t >> 3) & 1) << 2);
  else return ((t >> 1) & 1) | (((t >> 3) & 1) << 1);  // rows alternate 128-B bank halves already
}

template <int FN>
struct WGeo {
  static constexpr int BN = 64 * FN, WTN = 16 * FN;
  static constexpr int SA = 2 * BM, SB = 2 * BN;          // image row bytes
  static constexpr int A_BYTES = BK * SA, B_BYTES = BK * SB, STAGE = A_BYTES + B_BYTES;
  static constexpr int GA = (32 * SA / 1024) / 8;         // A granules per wave per K-half (2)
  static constexpr int GB_T = 32 * SB / 1024;             // B granules per K-half (16 or 20)
  static constexpr int GB_HI = (GB_T + 7) / 8, GB_LO = GB_T / 8;  // 3/2 (FN 5) or 2/2 (FN 4)
};

template <int FN, int TRANS>
__global__ __launch_bounds__(NT, 2) void gemm8w_kernel(const WArgs p) {
  using G = WGeo<FN>;
  constexpr int BN = G::BN, WTN = G::WTN, SA = G::SA, SB = G::SB, STAGE = G::STAGE;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  const int tiles_n = p.N / BN, tiles_m = (p.M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int per_group = kGroupM * tiles_n;
  const int first_m = (bid / per_group) * kGroupM;
  const int gsz = min(tiles_m - first_m, kGroupM);
  const int tm = first_m + (bid % per_group) % gsz, tn = (bid % per_group) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  const int nkt_all = p.K / BK, split = blockIdx.y, nsplit = gridDim.y;
  const int kt0 = (int)((int64_t)nkt_all * split / nsplit), kt1 = (int)((int64_t)nkt_all * (split + 1) / nsplit);
  const int nkt = kt1 - kt0;

  // buffer descriptors based at (first row of this split, first column of this tile); the record
  // count ends at the tensor's last element, so the padded columns of the last row tile read zeros
  // instead of faulting at the very end
  const int64_t a_off = (int64_t)kt0 * BK * p.lda + m0, b_off = (int64_t)kt0 * BK * p.ldb + n0;
  auto rec = [](int64_t elems) -> uint32_t {
    const int64_t bytes = elems > 0 ? 2 * elems : 0;
    return (uint32_t)(bytes < 0x7fffffff ? bytes : 0x7fffffff);
  };
  const uint32_t a_rec = rec(p.a_elems - a_off), b_rec = rec(p.b_elems - b_off);
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)(p.a + a_off), (short)0, a_rec, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)(p.b + b_off), (short)0, b_rec, 0x00020000);

  // ---- DMA granules: per K-half h (t-rows 32h..32h+31) A: 2 per wave; B: FN 5 -> 3 for the wave
  // group with wr == h, 2 for the other (20 in all), FN 4 -> 2 ---------------------------------
  uint32_t va[2][G::GA], la[2][G::GA];
  uint32_t vb[2][G::GB_HI], lb[2][G::GB_HI];
  auto src_off = [&](int S, int64_t ld, int byte) -> uint32_t {  // image byte -> global byte offset
    const int t = byte / S, cb = byte % S, ps = cb >> 5, hb = (cb >> 4) & 1;
    const int ls = ps ^ (S == SA ? swz<SA>(t) : swz<SB>(t));
    return 2u * (uint32_t)(t * ld + ls * 16 + hb * 8);
  };
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int i = 0; i < G::GA; ++i) {
      const int g = wave + 8 * i;
      const int byte = h * 32 * SA + g * 1024;
      la[h][i] = (uint32_t)byte;
      va[h][i] = src_off(SA, p.lda, byte + lane * 16);
    }
#pragma unroll
    for (int i = 0; i < G::GB_HI; ++i) {
      int g;
      if constexpr (G::GB_HI == G::GB_LO) g = wave + 8 * i;
      else g = (wr == h) ? (wc + 4 * i) : (12 + wc + 4 * i);  // 3-group: 0..11, 2-group: 12..19
      const int byte = h * 32 * SB + g * 1024;
      lb[h][i] = (uint32_t)(G::A_BYTES + byte);
      vb[h][i] = src_off(SB, p.ldb, byte + lane * 16);
    }
  }
  const int nb_h0 = (G::GB_HI == G::GB_LO || wr == 0) ? G::GB_HI : G::GB_LO;  // B granules in half 0
  const int nb_h1 = (G::GB_HI == G::GB_LO || wr == 1) ? G::GB_HI : G::GB_LO;
  // LDS-DMA in inline asm (M0 = the wave-uniform LDS address; nothing else in this kernel writes
  // M0): issued through the builtin, the DMA is a pending LDS write the compiler cannot tell from the
  // transposed fragment reads, so it would need asm reads (below) whose results it must then copy
  // into the MFMA operand registers -- 4 v_mov per MFMA, measured 1.4x the VALU and 1.37x the wave
  // cycles of gemm8 on the same FLOPs (profiles/r3_gemm8w_pmc.md)
  const uint32_t lds_base = (uint32_t)(uintptr_t)(lds_ptr_t)smem;
  auto glds = [&](const __amdgpu_buffer_rsrc_t& rs, uint32_t vo, uint32_t so, uint32_t lds_off) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %2, %3 offen lds"
                 :
                 : "v"(vo), "s"(lds_base + lds_off), "s"(rs), "s"(so)
                 : "memory");
  };
#define CS336_G8W_ISSUE(H, KT, ST)                                                                          \
  do {                                                                                                     \
    const uint32_t base_ = (uint32_t)((ST) * STAGE);                                                       \
    const uint32_t soa_ = (uint32_t)(KT) * BK * 2u * (uint32_t)p.lda, sob_ = (uint32_t)(KT) * BK * 2u * (uint32_t)p.ldb; \
    _Pragma("unroll") for (int i_ = 0; i_ < G::GA; ++i_)                                                   \
      glds(ra, va[H][i_], soa_, base_ + la[H][i_]); \
    const int nb_ = (H) == 0 ? nb_h0 : nb_h1;                                                              \
    _Pragma("unroll") for (int i_ = 0; i_ < G::GB_HI; ++i_) if (i_ < nb_)                                  \
      glds(rb, vb[H][i_], sob_, base_ + lb[H][i_]); \
  } while (0)
  // outstanding DMA of one K-half issue (this wave): n0 = GA + nb_h0, n1 = GA + nb_h1 (n0 + n1 does
  // not depend on the wave)
  const bool big0 = G::GB_HI != G::GB_LO && wr == 0;  // this wave issues 3 B granules in half 0
  constexpr int N01 = 2 * G::GA + G::GB_HI + G::GB_LO;  // both halves of one K-tile

  // ---- transposed fragment reads ------------------------------------------------------------
  const int g4 = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  // Each fragment = two ds_read_b64_tr_b16 (builtin) joined into one 128-bit MFMA operand; the
  // phase's explicit lgkmcnt(0) before its barrier retires them (WAR against the DMA restaging)
  auto tr = [&](uint32_t img, int S, int c0, int t) -> s16x4 {
    const int s = c0 >> 4, f = S == SA ? swz<SA>(t) : swz<SB>(t);
    const uint32_t off = img + (uint32_t)(t * S + ((s ^ f) << 5) + 8 * pp);
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(smem + off));
  };
  auto frag = [&](uint32_t img, int S, int c0, int ks) -> bf16x8 {
    const int t0 = 32 * ks + 8 * g4 + q;
    const s16x4 lo = tr(img, S, c0, t0), hi = tr(img, S, c0, t0 + 4);
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };

  f32x4 acc[8][FN];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa[4], fb[FN];
  const int arow = wr * 128, bcol = wc * WTN;
  auto wait_a = [&]() { lgkm0(); };
  auto wait_ab = [&]() { lgkm0(); };

  auto mma = [&](int i0) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        if constexpr (TRANS)  // lane: C[m = 4(l>>4)+r][n = l&15] -> 4 consecutive m (stored along a row of Cᵀ)
          acc[i0 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i0 + i][j], 0, 0, 0);
        else  // lane: C[m = l&15][n = 4(l>>4)+r] -> 4 consecutive n
          acc[i0 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i0 + i][j], 0, 0, 0);
      }
    __builtin_amdgcn_s_setprio(0);
  };

  // ---- prologue: K-tile 0 whole, K-tile 1's first half; only K-tile 0's first half is waited
  // for here (its second half at phase 1) ---------------------------------------------------------
  if (nkt > 0) {
    CS336_G8W_ISSUE(0, 0, 0);
    CS336_G8W_ISSUE(1, 0, 0);
    if (nkt > 1) {
      CS336_G8W_ISSUE(0, 1, 1);
      vmcnt<N01>();  // younger: K-tile 0's second half, K-tile 1's first half
    } else {
      if (big0) vmcnt<G::GA + G::GB_LO>();  // younger: K-tile 0's second half (n1)
      else vmcnt<G::GA + G::GB_HI>();
    }
  }
  sbarrier();
  if (wr == 1) sbarrier();

  for (int t = 0; t < nkt; ++t) {
    const uint32_t st = (uint32_t)((t & 1) * STAGE);
    // P0: k 0-31, rows 0-63 (+ all column tiles); restage K-tile t+1's second half
    if (t + 1 < nkt) CS336_G8W_ISSUE(1, t + 1, (t + 1) & 1);
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = frag(st, SA, arow + 16 * i, 0);
#pragma unroll
    for (int j = 0; j < FN; ++j) fb[j] = frag(st + G::A_BYTES, SB, bcol + 16 * j, 0);
    wait_ab();
    sbarrier();
    mma(0);
    sbarrier();
    // P1: k 0-31, rows 64-127; retire this K-tile's second half (read from P2 on): issued at the
    // previous K-tile's P0, it has had five phases in flight
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = frag(st, SA, arow + 64 + 16 * i, 0);
    if (t + 1 < nkt) vmcnt<N01>();  // younger: K-tile t+1's two halves
    else vmcnt<0>();
    wait_a();
    sbarrier();
    mma(4);
    sbarrier();
    // P2: k 32-63, rows 0-63; restage this stage's first half with K-tile t+2
    if (t + 2 < nkt) CS336_G8W_ISSUE(0, t + 2, t & 1);
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = frag(st, SA, arow + 16 * i, 1);
#pragma unroll
    for (int j = 0; j < FN; ++j) fb[j] = frag(st + G::A_BYTES, SB, bcol + 16 * j, 1);
    wait_ab();
    sbarrier();
    mma(0);
    sbarrier();
    // P3: k 32-63, rows 64-127; retire K-tile t+1's first half (read at its P0); its second half and
    // K-tile t+2's first half stay in flight
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = frag(st, SA, arow + 64 + 16 * i, 1);
    if (t + 1 < nkt) {
      if (t + 2 < nkt) {
        vmcnt<N01>();  // younger: K-tile t+1's second half (P0), K-tile t+2's first half (P2)
      } else if (big0) {
        vmcnt<G::GA + G::GB_LO>();  // younger: K-tile t+1's second half (n1)
      } else {
        vmcnt<G::GA + G::GB_HI>();
      }
    }
    wait_a();
    sbarrier();
    mma(4);
    sbarrier();
  }
#undef CS336_G8W_ISSUE
  if (wr == 0) sbarrier();

  // ---- epilogue: fp32 straight from the accumulators, 16 B per lane ----------------------------
  float* c = p.c + (int64_t)split * p.slab_stride;
  const int lr = lane & 15, lq = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const f32x4 v = acc[i][j];
      if constexpr (TRANS) {
        // C[m .. m+3][n] -> Cᵀ row n, columns m .. m+3
        const int m = m0 + arow + 16 * i + lq, n = n0 + bcol + 16 * j + lr;
        if (m < p.M) {
          float4* d = reinterpret_cast<float4*>(c + (int64_t)n * p.ldc + m);
          float4 w = make_float4(v[0], v[1], v[2], v[3]);
          if (p.accumulate) {
            const float4 o = *d;
            w.x += o.x; w.y += o.y; w.z += o.z; w.w += o.w;
          }
          *d = w;
        }
      } else {
        const int m = m0 + arow + 16 * i + lr, n = n0 + bcol + 16 * j + lq;
        if (m < p.M) {
          float4* d = reinterpret_cast<float4*>(c + (int64_t)m * p.ldc + n);
          float4 w = make_float4(v[0], v[1], v[2], v[3]);
          if (p.accumulate) {
            const float4 o = *d;
            w.x += o.x; w.y += o.y; w.z += o.z; w.w += o.w;
          }
          *d = w;
        }
      }
    }
}

template <int FN, int TRANS>
void launch_wt(const WArgs& p, hipStream_t s) {
  const dim3 grid((unsigned)(((p.M + BM - 1) / BM) * (p.N / (64 * FN))), (unsigned)p.splits), block(NT);
  hipLaunchKernelGGL((gemm8w_kernel<FN, TRANS>), grid, block, 0, s, p);
}

}  // namespace

bool launch_w(const WArgs& p, int fn, hipStream_t s) {
  if (p.K % BK || p.K < BK || p.M <= 0 || p.M % 4 || p.splits < 1 || p.splits > 64) return false;
  if (fn == 0) fn = p.N % 320 == 0 ? 5 : (p.N % 256 == 0 ? 4 : 0);
  if ((fn != 4 && fn != 5) || p.N % (64 * fn)) return false;
  if (p.splits > 1 && p.accumulate) return false;
  if (fn == 5) {
    if (p.trans_out) launch_wt<5, 1>(p, s);
    else launch_wt<5, 0>(p, s);
  } else {
    if (p.trans_out) launch_wt<4, 1>(p, s);
    else launch_wt<4, 0>(p, s);
  }
  return true;
}

}  // namespace gemm8
}  // namespace cs336
