// cs336-build: agpr-accumulators
//
// "gemm8": the projection GEMMs of the Transformer step in NT form, C = A · Bᵀ with both operands
// K-major (forward X·Wᵀ; input gradient dY·W read through the Wᵀ shadow the fused AdamW writes),
// with the SwiGLU gate fused into the epilogues:
//
//   EPI 0  C = A·Bᵀ (bf16)
//   EPI 1  W1|W3 forward: the tile's columns are W1 rows j0.. and the W3 rows half+j0.. , so one tile
//          holds a and b of the same hidden units; writes y = [a|b] (saved for backward) AND
//          h = silu(a)·b (the W2 input) -- no separate SwiGLU pass over the 2·d_ff activation
//   EPI 2  W2 input gradient: dh = dY·W2 is never stored; the epilogue reads the saved a, b and writes
//          da = dh·b·silu'(a), db = dh·silu(a) into [da|db] (the W1|W3 output gradient)
//   EPI 3  QKV forward with RoPE: C = A·Bᵀ (bf16) with the interleaved-pair rotation applied to the
//          columns below rope_cols (q|k heads) in the store -- no separate RoPE pass over q|k. The
//          rotation reads the bf16-rounded product, as the separate pass did (same rounding points).
//
// Tails (EPI 0 only): N % 8 == 0 with a partial last column tile, K % 8 == 0 with a partial last
// k-tile -- the vocabulary head's forward (N = 10000) and input gradient (K = 10000), so no hipBLASLt
// kernel is left in the step. Out-of-range B rows and K chunks are loaded as zeros by the buffer
// range check; partial-tile stores are masked per 8-column piece.
//
// Structure (cdna_hip_programming.md §5 "256² 8-phase template", re-derived for these shapes):
// * tile 256 × BN (BN = 64·FN: 256 or 320 -- every N of the XL/2.7b projections is a multiple of
//   320 or 256, d_model 1600 = 5·320), BK = 64, 512 threads = 8 waves as 2 (M) × 4 (N), each wave
//   128 × 16·FN of v_mfma_f32_16x16x32_bf16 accumulators (AGPRs);
// * two LDS stages (one K-tile each, ≤ 144 KiB) filled by LDS-DMA (buffer_load … lds, 16 B/lane),
//   K-major images with the 16-B chunk XOR-swizzled by (row>>1)&7 (conflict-free ds_read_b128 for
//   the 16x16x32 fragment lane groups; the swizzle goes on the per-lane global source address);
// * each K-tile runs as 4 phases = the wave's 4 output quadrants (rows 0-63 / 64-127 × the first
//   FB0 / last FN-FB0 column tiles). Phase = {ds_read its fragments; issue a slice of the K-tile
//   after next; lgkmcnt(0); s_barrier; MFMA cluster; s_barrier}. The second wave group (waves 4-7,
//   the partner of waves 0-3 on every SIMD) runs one barrier behind, so on each SIMD one wave
//   multiplies while the other reads LDS / issues DMA;
// * the K-tile after next is restaged into the stage just read as soon as the quadrant reads of its
//   region retired (A rows 0-63 + first col tiles in phase 1, last col tiles in phase 2, A rows 64-127
//   in phase 3), and one counted vmcnt per K-tile (phase 3) retires the next K-tile; DMA stays in
//   flight across the raw s_barriers (never __syncthreads(), which would drain it);
// * XCD-aware bijective block remap + grouped tile order (8 tile-rows) for L2 reuse.
#include "cs336/kernels.h"
#include "gemm8.h"

namespace cs336 {
namespace gemm8 {


namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int v4u32;
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

// sigmoid with the hardware reciprocal (v_exp_f32 + v_rcp_f32): the epilogues run outside the MFMA
// stream, so every VALU instruction there is on the tile's critical path
__device__ __forceinline__ float sigmoid_f(float a) { return __builtin_amdgcn_rcpf(1.f + __expf(-a)); }

// Geometry of one instantiation.
template <int FN>
struct Geo {
  static constexpr int BN = 64 * FN;           // tile columns
  static constexpr int WTN = 16 * FN;          // per-wave columns
  static constexpr int FB0 = (FN + 1) / 2;     // column tiles of the first column quadrant
  static constexpr int B0C = 16 * FB0;         // its width
  static constexpr int A_BYTES = BM * 128;     // [256 rows][64 k] bf16
  static constexpr int B_BYTES = BN * 128;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  // DMA granules (8 image rows = 1 KiB = one wave instruction) per wave, per restage slice
  static constexpr int G_A0 = 16 / 8;                 // A rows {0..63, 128..191}: 16 granules
  static constexpr int G_B0 = (4 * B0C / 8) / 8;      // B rows wc·WTN + [0, B0C)
  static constexpr int G_B1 = (4 * (WTN - B0C) / 8) / 8;
  static constexpr int G_A1 = 16 / 8;
  static constexpr int G_P1 = G_A0 + G_B0, G_P2 = G_B1, G_P3 = G_A1;
  static constexpr int G_ALL = G_P1 + G_P2 + G_P3;
  static_assert((4 * B0C / 8) % 8 == 0 && (4 * (WTN - B0C) / 8) % 8 == 0, "B granules must split over 8 waves");
};

// TAIL: bit 0 = partial last column tile (N % BN), bit 1 = partial last k-tile (K % 64)
template <int FN, int EPI, int TAIL>
__global__ __launch_bounds__(NT, 2) void gemm8_kernel(const Args p) {
  static_assert(!TAIL || EPI == 0, "tails: plain C = A·Bᵀ only");
  constexpr bool NTAIL = TAIL & 1, KTAIL = TAIL & 2;
  using G = Geo<FN>;
  constexpr int BN = G::BN, WTN = G::WTN, FB0 = G::FB0, B0C = G::B0C, STAGE = G::STAGE;
  // the main loop's two stages, or (epilogue) the whole bf16 tile image
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE > BM * BN * 2 ? 2 * STAGE : BM * BN * 2];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
#ifdef CS336_G8_STAMP
  const uint64_t st_t0 = __builtin_amdgcn_s_memtime(), st_r0 = __builtin_amdgcn_s_memrealtime();
  uint64_t st_t1 = 0, st_t2 = 0;
#endif

  // ---- tile coordinates -------------------------------------------------------------------
  // EPI 1: N = 2·half, BN/2 units of each half per tile. EPI 0 also takes an N tail (N % BN != 0,
  // N % 8 == 0: the vocabulary head, 10000 = 31·320 + 80): B rows >= N read zeros, stores masked
  const int tiles_n = NTAIL ? (p.N + BN - 1) / BN : p.N / BN;
  const int tiles_m = p.M / BM;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int per_group = kGroupM * tiles_n;
  const int first_m = (bid / per_group) * kGroupM;
  const int gsz = min(tiles_m - first_m, kGroupM);
  const int tm = first_m + (bid % per_group) % gsz, tn = (bid % per_group) / gsz;
  const int m0 = tm * BM;
  // EPI 1: tile column c < BN/2 is W1 row j0 + c, else W3 row half + j0 + c - BN/2
  const int n0 = tn * (EPI == 1 ? BN / 2 : BN);

  // ---- DMA setup: per wave G_ALL granules; slot order P1 (A0 then B0), P2 (B1), P3 (A1) ------
  // The record counts end at each operand's last element (host: both extents < 2 GiB), so B rows
  // past N (EPI 0 N tail) and the lanes of a K tail pointed at kOOB read zeros (raw-buffer range check)
  // (the tail bookkeeping lives in its own instantiation: in the full-tile kernel one more live
  // register spilled the FN 5 main loop)
  const int nkt = KTAIL ? (p.K + BK - 1) / BK : p.K / BK;  // (KTAIL: the last k-tile is partial)
  constexpr uint32_t kOOB = 0x7ffffff0u;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.a + (int64_t)m0 * p.lda), (short)0, (uint32_t)(((BM - 1) * p.lda + p.K) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.b, (short)0, (uint32_t)(((int64_t)(p.N - 1) * p.ldb + p.K) * 2), 0x00020000);
  uint32_t voff[G::G_ALL];   // per-lane byte offset at k-tile 0
  uint32_t ldso[G::G_ALL];   // wave-uniform LDS byte offset within a stage
  {
    int s = 0;
    auto a_gran = [&](int row0) {  // A image rows row0..row0+7
      const int r = row0 + (lane >> 3), lc = (lane & 7) ^ ((r >> 1) & 7);
      voff[s] = 2u * (uint32_t)(r * p.lda + lc * 8);
      ldso[s] = (uint32_t)(row0 * 128);
      ++s;
    };
    auto b_gran = [&](int row0) {  // B image rows row0..row0+7 (tile-local column index)
      const int r = row0 + (lane >> 3), lc = (lane & 7) ^ ((r >> 1) & 7);
      int grow;
      if constexpr (EPI == 1) grow = r < BN / 2 ? n0 + r : p.half + n0 + (r - BN / 2);
      else grow = n0 + r;
      voff[s] = 2u * (uint32_t)((int64_t)grow * p.ldb + lc * 8);
      ldso[s] = (uint32_t)(G::A_BYTES + row0 * 128);
      ++s;
    };
#pragma unroll
    for (int i = 0; i < G::G_A0; ++i) {  // A0 rows: granule g -> rows 8g (g < 8) or 128 + 8(g-8)
      const int g = wave + 8 * i;
      a_gran(g < 8 ? 8 * g : 128 + 8 * (g - 8));
    }
#pragma unroll
    for (int i = 0; i < G::G_B0; ++i) {
      const int g = wave + 8 * i, per = B0C / 8;
      b_gran((g / per) * WTN + (g % per) * 8);
    }
#pragma unroll
    for (int i = 0; i < G::G_B1; ++i) {
      const int g = wave + 8 * i, per = (WTN - B0C) / 8;
      b_gran((g / per) * WTN + B0C + (g % per) * 8);
    }
#pragma unroll
    for (int i = 0; i < G::G_A1; ++i) {
      const int g = wave + 8 * i;
      a_gran(g < 8 ? 64 + 8 * g : 192 + 8 * (g - 8));
    }
  }
  auto glds = [&](const __amdgpu_buffer_rsrc_t& rs, uint32_t vo, uint32_t so, uint32_t lds_off) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(smem + lds_off), 16, vo, so, 0, 0);
  };
  // image row0 of granule i (slot order, as laid out above): the K-tail mask re-derives a lane's
  // source chunk from it and the lane id instead of keeping a mask register live through the loop
  auto gran_row = [&](int i) -> int {
    if (i < G::G_A0) {
      const int g = wave + 8 * i;
      return g < 8 ? 8 * g : 128 + 8 * (g - 8);
    } else if (i < G::G_P1) {
      const int g = wave + 8 * (i - G::G_A0), per = B0C / 8;
      return (g / per) * WTN + (g % per) * 8;
    } else if (i < G::G_P1 + G::G_P2) {
      const int g = wave + 8 * (i - G::G_P1), per = (WTN - B0C) / 8;
      return (g / per) * WTN + B0C + (g % per) * 8;
    }
    const int g = wave + 8 * (i - G::G_P1 - G::G_P2);
    return g < 8 ? 64 + 8 * g : 192 + 8 * (g - 8);
  };
  // issue slice `part` (1: A0+B0, 2: B1, 3: A1; 0: all) of k-tile kt into stage st; `masked`: the
  // partial last k-tile (lanes whose chunk lies at or past K read out of range = zeros)
  auto issue_v = [&](int part, int kt, int st, bool masked) {
    const uint32_t so = (uint32_t)kt * (BK * 2), base = (uint32_t)(st * STAGE);
    auto vo = [&](int i) -> uint32_t {
      if (!masked) return voff[i];
      const int ln = __lane_id(), r = gran_row(i) + (ln >> 3), lc = (ln & 7) ^ ((r >> 1) & 7);
      return kt * BK + lc * 8 >= p.K ? kOOB : voff[i];
    };
    if (part == 0 || part == 1) {
#pragma unroll
      for (int i = 0; i < G::G_A0; ++i) glds(ra, vo(i), so, base + ldso[i]);
#pragma unroll
      for (int i = G::G_A0; i < G::G_P1; ++i) glds(rb, vo(i), so, base + ldso[i]);
    }
    if (part == 0 || part == 2) {
#pragma unroll
      for (int i = G::G_P1; i < G::G_P1 + G::G_P2; ++i) glds(rb, vo(i), so, base + ldso[i]);
    }
    if (part == 0 || part == 3) {
#pragma unroll
      for (int i = G::G_P1 + G::G_P2; i < G::G_ALL; ++i) glds(ra, vo(i), so, base + ldso[i]);
    }
  };
  auto issue = [&](int part, int kt, int st) {
    if (KTAIL && kt == nkt - 1) issue_v(part, kt, st, true);
    else issue_v(part, kt, st, false);
  };

  // ---- fragment reads: lane row (l&15), 16-B chunk 4·ks + (l>>4) XOR ((l&15)>>1) -----------
  const int x = (lane & 15) >> 1, q4 = lane >> 4;
  const uint32_t lo0 = (uint32_t)((lane & 15) * 128 + ((q4 ^ x) * 16));
  const uint32_t lo1 = (uint32_t)((lane & 15) * 128 + (((4 + q4) ^ x) * 16));
  auto frag = [&](uint32_t img_off, int row0, int ks) -> bf16x8 {
    const char* ptr = smem + img_off + row0 * 128 + (ks ? lo1 : lo0);
    return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(ptr));
  };

  f32x4 acc[8][FN];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 fa[4][2], fb0[FB0][2], fb1[FN - FB0 > 0 ? FN - FB0 : 1][2];
  const int arow = wr * 128, bcol = wc * WTN;

  auto mma = [&](int i0, const bf16x8 (&a)[4][2], auto& bq, int j0, int nj) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < nj; ++j)
          // B fragment as the MFMA's A operand: D = (A·Bᵀ)ᵀ per 16x16 block, so lane l holds
          // C[m = l&15][n = 4(l>>4) + r] -- four consecutive output columns (one 8/16-B LDS write)
          acc[i0 + i][j0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[j][ks], a[i][ks], acc[i0 + i][j0 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // ---- prologue: k-tiles 0 and 1 -------------------------------------------------------------
  issue(0, 0, 0);
  if (nkt > 1) {
    issue(0, 1, 1);
    vmcnt<G::G_ALL>();
  } else {
    vmcnt<0>();
  }
  sbarrier();
#ifdef CS336_G8_STAMP
  st_t1 = __builtin_amdgcn_s_memtime();
#endif
  if (wr == 1) sbarrier();  // second wave group one barrier behind (SIMD partners offset)

  for (int t = 0; t < nkt; ++t) {
    const uint32_t st = (uint32_t)((t & 1) * STAGE);
    const bool pre = t + 2 < nkt;  // the k-tile after next exists: restage this stage with it
    // P0: quadrant (rows 0-63, first col tiles)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) fa[i][ks] = frag(st, arow + 16 * i, ks);
#pragma unroll
    for (int j = 0; j < FB0; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) fb0[j][ks] = frag(st + G::A_BYTES, bcol + 16 * j, ks);
    lgkm0();
    sbarrier();
    mma(0, fa, fb0, 0, FB0);
    sbarrier();
    // P1: quadrant (rows 0-63, last col tiles); restage A rows 0-63 / B first cols with t+2
    if constexpr (FN - FB0 > 0) {
#pragma unroll
      for (int j = 0; j < FN - FB0; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) fb1[j][ks] = frag(st + G::A_BYTES, bcol + B0C + 16 * j, ks);
    }
    if (pre) issue(1, t + 2, t & 1);
    lgkm0();
    sbarrier();
    if constexpr (FN - FB0 > 0) mma(0, fa, fb1, FB0, FN - FB0);
    sbarrier();
    // P2: quadrant (rows 64-127, last col tiles); restage B last cols
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) fa[i][ks] = frag(st, arow + 64 + 16 * i, ks);
    if (pre) issue(2, t + 2, t & 1);
    lgkm0();
    sbarrier();
    if constexpr (FN - FB0 > 0) mma(4, fa, fb1, FB0, FN - FB0);
    sbarrier();
    // P3: quadrant (rows 64-127, first col tiles); retire k-tile t+1, restage A rows 64-127
    if (t + 1 < nkt) {
      if (pre) vmcnt<G::G_P1 + G::G_P2>();
      else vmcnt<0>();
    }
    if (pre) issue(3, t + 2, t & 1);
    sbarrier();
    mma(4, fa, fb0, 0, FB0);
    sbarrier();
  }
  if (wr == 0) sbarrier();  // balance the wave-group offset
  lgkm0();
  sbarrier();
#ifdef CS336_G8_STAMP
  st_t2 = __builtin_amdgcn_s_memtime();
#endif

  // ---- epilogue ----------------------------------------------------------------------------
  // cache policy of the epilogue's streams: the SwiGLU outputs (EPI 1 y and h, EPI 2 da|db) and the
  // EPI 2 a/b inputs are touched once here, so they go out / come in nontemporal (aux bit 1 = nt):
  // -7 % on W1|W3 forward and -6 % on the W2 input gradient from nt stores, a further -7 % on the
  // latter from nt a/b loads (49152 tokens, same box; profiles/r5_gemm8_epilogue.md). Plain EPI 0
  // stores stay default-policy (their consumer usually reads them next; nt measured neutral there)
  constexpr int ST_AUX = EPI == 0 ? 0 : 2, LD_AUX = 2;
  // Lane l holds C[m = l&15][n = 4(l>>4) + r] of each 16x16 block (operand-swapped MFMA).
  const int m_l = lane & 15, n_l = 4 * (lane >> 4);
  if constexpr (EPI != 3) {
    // Whole-tile epilogue (EPI 0/1/2): every wave dumps its blocks as bf16 into one [256][BN] image
    // that fills the LDS (160 KiB at BN 320), then the workgroup streams it out row-major: each
    // wave instruction covers whole 640-B (320-B) row runs instead of the 160-B pieces of a per-wave
    // scratch. EPI 2 issues ALL of the thread's a/b loads (20 + 20 x 16 B) as soon as the
    // accumulators are dumped: the round-3/4 form kept one 32-row piece in flight and was
    // latency-bound (ablation: the a/b loads were 0.22 of 1.14 ms, profiles/r5_gemm8_epilogue.md).
    // EPI 2 rounds dh to bf16 before the SwiGLU backward, as the unfused path (bf16 GEMM output) does.
    // Image chunks (16 B = 8 columns) are XOR-swizzled by the row: conflict-free 8-B dump writes
    // (16 rows per lane group) and 16-B row-major reads.
    constexpr int RB = BN * 2, CH = BN / 8;
    auto img = [&](int row, int ch) -> uint32_t {
      const int x = FN == 5 ? ((row >> 1) & 7) : (row & 15);
      return (uint32_t)(row * RB + ((ch ^ x) << 4));
    };
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const f32x4 v = acc[i][j];
        const int row = arow + 16 * i + m_l, col = bcol + 16 * j + n_l;
        const uint32_t lo = (uint32_t)f32_to_bf16(v[0]) | ((uint32_t)f32_to_bf16(v[1]) << 16);
        const uint32_t hi = (uint32_t)f32_to_bf16(v[2]) | ((uint32_t)f32_to_bf16(v[3]) << 16);
        *reinterpret_cast<uint2*>(smem + img(row, col >> 3) + ((col >> 2) & 1) * 8) = make_uint2(lo, hi);
      }
    // output (and EPI 2 input) descriptors based at the tile's first row; 32-bit offsets within it
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.c + (int64_t)m0 * p.ldc), (short)0, 0x7fffffffu, 0x00020000);
    if constexpr (EPI == 2) {
      constexpr int PT = BM * CH / NT;  // 20 (BN 320) or 16 chunks per thread
      static_assert(BM * CH % NT == 0, "chunks must split over the workgroup");
      const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(p.y + (int64_t)m0 * p.ldy), (short)0, 0x7fffffffu, 0x00020000);
      uint4 av[PT], bv[PT];
#pragma unroll
      for (int i = 0; i < PT; ++i) {
        const int q = tid + NT * i, row = q / CH, ch = q % CH;
        const uint32_t off = 2u * (uint32_t)(row * p.ldy + n0 + 8 * ch);
        av[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(ry, off, 0, LD_AUX));
        bv[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(ry, off + 2u * (uint32_t)p.half, 0, LD_AUX));
      }
      lgkm0();
      sbarrier();  // image complete
#pragma unroll
      for (int i = 0; i < PT; ++i) {
        const int q = tid + NT * i, row = q / CH, ch = q % CH;
        const uint4 dv = *reinterpret_cast<const uint4*>(smem + img(row, ch));
        const bf16_t* de = reinterpret_cast<const bf16_t*>(&dv);
        const bf16_t* ae = reinterpret_cast<const bf16_t*>(&av[i]);
        const bf16_t* be = reinterpret_cast<const bf16_t*>(&bv[i]);
        uint4 dav, dbv;
        bf16_t* da = reinterpret_cast<bf16_t*>(&dav);
        bf16_t* db = reinterpret_cast<bf16_t*>(&dbv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float a = bf16_to_f32(ae[e]), b = bf16_to_f32(be[e]), dh = bf16_to_f32(de[e]);
          const float sg = sigmoid_f(a), gb = dh * sg;
          da[e] = f32_to_bf16(gb * b * (1.f + a * (1.f - sg)));
          db[e] = f32_to_bf16(gb * a);
        }
        const uint32_t off = 2u * (uint32_t)(row * p.ldc + n0 + 8 * ch);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, dav), rc, off, 0, ST_AUX);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, dbv), rc, off + 2u * (uint32_t)p.half, 0, ST_AUX);
      }
    } else if constexpr (EPI == 1) {
      // tile columns [0, BN/2) are a = W1 units n0.., [BN/2, BN) b = W3 units: one thread takes a
      // unit chunk pair, stores both halves of y and h = silu(a)·b
      constexpr int HU = CH / 2, PT = BM * HU / NT;  // 10 (BN 320) or 8 pairs per thread
      static_assert(BM * HU % NT == 0, "pairs must split over the workgroup");
      const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(p.h + (int64_t)m0 * p.ldh), (short)0, 0x7fffffffu, 0x00020000);
      lgkm0();
      sbarrier();  // image complete
#pragma unroll
      for (int i = 0; i < PT; ++i) {
        const int q = tid + NT * i, row = q / HU, u = q % HU;
        const uint4 va = *reinterpret_cast<const uint4*>(smem + img(row, u));
        const uint4 vb = *reinterpret_cast<const uint4*>(smem + img(row, u + HU));
        const uint32_t off = 2u * (uint32_t)(row * p.ldc + n0 + 8 * u);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, va), rc, off, 0, ST_AUX);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, vb), rc, off + 2u * (uint32_t)p.half, 0, ST_AUX);
        const bf16_t* ae = reinterpret_cast<const bf16_t*>(&va);
        const bf16_t* be = reinterpret_cast<const bf16_t*>(&vb);
        uint4 hv;
        bf16_t* he = reinterpret_cast<bf16_t*>(&hv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float a = bf16_to_f32(ae[e]);
          he[e] = f32_to_bf16(a * sigmoid_f(a) * bf16_to_f32(be[e]));
        }
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, hv), rh, 2u * (uint32_t)(row * p.ldh + n0 + 8 * u), 0, ST_AUX);
      }
    } else {
      constexpr int PT = BM * CH / NT;
      lgkm0();
      sbarrier();  // image complete
#pragma unroll
      for (int i = 0; i < PT; ++i) {
        const int q = tid + NT * i, row = q / CH, ch = q % CH;
        const uint4 v = *reinterpret_cast<const uint4*>(smem + img(row, ch));
        const int col = n0 + 8 * ch;
        if (!NTAIL || col < p.N)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, v), rc, 2u * (uint32_t)(row * p.ldc + col), 0, ST_AUX);
      }
    }
  } else {
    // EPI 3 (QKV + RoPE): per-wave scratch in 32-row pieces (40 KiB in all), the tile rows' RoPE
    // cos/sin staged in the LDS behind it, so the store loop reads no global memory (a global load
    // there waits for every earlier store: vmcnt retires in issue order)
    constexpr int CPR = WTN / 8;  // 8-column units per scratch row
    constexpr int PR = 32, UNITS = PR * CPR, PER = UNITS / 64;
    static_assert(UNITS % 64 == 0, "epilogue units must fill the wave");
    char* scr = smem + wave * (PR * WTN * 2);
    constexpr int TOFF = 8 * PR * WTN * 2;  // table: cos [256][np], then sin [256][np] (fp32)
    const int np = p.rdh >> 1;
    const bool rot = n0 < p.rope_cols;  // tile-uniform (host: rope_cols % BN == 0)
    static_assert(TOFF + 2 * 256 * 48 * 4 <= 2 * STAGE, "cos/sin table of d_head <= 96 behind the scratch");
    if (rot) {
      // two threads per tile row, each half of the row's np/4 float4 of cos and of sin: every load
      // issued before any is waited for (d_head <= 96: at most 6 float4 per thread and table)
      constexpr int MAXQ = 6;
      float* tc = reinterpret_cast<float*>(smem + TOFF);
      float* ts = tc + 256 * np;
      const int r = tid >> 1, q4n = np >> 2, hq = (q4n + 1) >> 1;
      const int qb = (tid & 1) * hq;
      const int row = m0 + r;
      const int64_t pos = p.rpos ? p.rpos[row] : (int64_t)(row % p.rseq);
      // indices past this thread's share are clamped to the row's last float4: a duplicate load
      // and an identical rewrite, never a branch (keeps the arrays in registers)
      float4 cb[MAXQ], sb[MAXQ];
#pragma unroll
      for (int q = 0; q < MAXQ; ++q) {
        const int i4 = min(qb + q, q4n - 1);
        cb[q] = *reinterpret_cast<const float4*>(p.rcos + pos * np + 4 * i4);
        sb[q] = *reinterpret_cast<const float4*>(p.rsin + pos * np + 4 * i4);
      }
#pragma unroll
      for (int q = 0; q < MAXQ; ++q) {
        const int i4 = min(qb + q, q4n - 1);
        *reinterpret_cast<float4*>(tc + r * np + 4 * i4) = cb[q];
        *reinterpret_cast<float4*>(ts + r * np + 4 * i4) = sb[q];
      }
      __syncthreads();
    }
#pragma unroll
    for (int piece = 0; piece < 128 / PR; ++piece) {
#pragma unroll
      for (int ib = 0; ib < PR / 16; ++ib)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const f32x4 v = acc[piece * (PR / 16) + ib][j];
          const uint32_t lo = (uint32_t)f32_to_bf16(v[0]) | ((uint32_t)f32_to_bf16(v[1]) << 16);
          const uint32_t hi = (uint32_t)f32_to_bf16(v[2]) | ((uint32_t)f32_to_bf16(v[3]) << 16);
          *reinterpret_cast<uint2*>(scr + ((16 * ib + m_l) * WTN + 16 * j + n_l) * 2) = make_uint2(lo, hi);
        }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int q = lane + 64 * u, rr = q / CPR, cc = q % CPR;
        const uint4 v = *reinterpret_cast<const uint4*>(scr + (rr * WTN + cc * 8) * 2);
        const int64_t row = (int64_t)m0 + arow + PR * piece + rr;
        const int col = n0 + bcol + cc * 8;
        uint4 o = v;
        if (rot) {  // q|k: rotate pairs (2i, 2i+1), i = (col mod d_head) / 2 + 0..3
          const int i0 = (col % p.rdh) >> 1, tr = arow + PR * piece + rr;
          const float* tc = reinterpret_cast<const float*>(smem + TOFF);
          const float4 c4 = *reinterpret_cast<const float4*>(tc + tr * np + i0);
          const float4 s4 = *reinterpret_cast<const float4*>(tc + 256 * np + tr * np + i0);
          const float cv[4] = {c4.x, c4.y, c4.z, c4.w}, sv[4] = {s4.x, s4.y, s4.z, s4.w};
          const uint32_t w[4] = {v.x, v.y, v.z, v.w};
          uint32_t r[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float x0 = bf16_to_f32((bf16_t)(w[e] & 0xffff)), x1 = bf16_to_f32((bf16_t)(w[e] >> 16));
            r[e] = (uint32_t)f32_to_bf16(cv[e] * x0 - sv[e] * x1) |
                   ((uint32_t)f32_to_bf16(sv[e] * x0 + cv[e] * x1) << 16);
          }
          o = make_uint4(r[0], r[1], r[2], r[3]);
        }
        *reinterpret_cast<uint4*>(p.c + row * p.ldc + col) = o;
      }
      lgkm0();
      __builtin_amdgcn_wave_barrier();
    }
  }
#ifdef CS336_G8_STAMP
  vmcnt<0>();
  __syncthreads();
  if (tid == 0 && p.stamps) {
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    uint64_t* o = p.stamps + 8 * (int64_t)blockIdx.x;
    const uint64_t t3 = __builtin_amdgcn_s_memtime(), r3 = __builtin_amdgcn_s_memrealtime();
    o[0] = st_t0; o[1] = st_t1; o[2] = st_t2; o[3] = t3; o[4] = st_r0; o[5] = r3; o[6] = hw; o[7] = xcc;
  }
#endif
}

uint64_t* g_stamps = nullptr;  // diagnostic stamp buffer (set_stamp_buffer), null in normal runs
int64_t g_stamp_blocks = 0;

template <int FN, int EPI>
void launch_t(const Args& p_in, hipStream_t s) {
  Args p = p_in;
  constexpr int BN = 64 * FN;
  const int tail = EPI == 0 ? (p.N % BN != 0 ? 1 : 0) | (p.K % BK != 0 ? 2 : 0) : 0;
  const int tiles_n = (tail & 1) ? (p.N + BN - 1) / BN : p.N / BN;
  const dim3 grid((unsigned)((p.M / BM) * tiles_n)), block(NT);
  if (g_stamps && (int64_t)grid.x <= g_stamp_blocks) p.stamps = g_stamps;
  if constexpr (EPI == 0) {
    if (tail == 1) {
      hipLaunchKernelGGL((gemm8_kernel<FN, 0, 1>), grid, block, 0, s, p);
      return;
    }
    if (tail == 2) {
      hipLaunchKernelGGL((gemm8_kernel<FN, 0, 2>), grid, block, 0, s, p);
      return;
    }
    if (tail == 3) {
      hipLaunchKernelGGL((gemm8_kernel<FN, 0, 3>), grid, block, 0, s, p);
      return;
    }
  }
  hipLaunchKernelGGL((gemm8_kernel<FN, EPI, 0>), grid, block, 0, s, p);
}

}  // namespace

bool set_stamp_buffer(uint64_t* buf, int64_t blocks) {
  g_stamps = blocks > 0 ? buf : nullptr;
  g_stamp_blocks = blocks > 0 ? blocks : 0;
#ifdef CS336_G8_STAMP
  return true;
#else
  return false;  // this build writes no stamps
#endif
}

// Tile width for an output of N columns (EPI 1: N = 2·half): 320 if it divides, else 256, else 0.
int pick_fn(int N, int epi, int half) {
  if (epi == 1) {  // a tile holds BN/2 hidden units of each of W1, W3
    if (half % 160 == 0) return 5;
    if (half % 128 == 0) return 4;
    return 0;
  }
  if (N % 320 == 0) return 5;
  if (N % 256 == 0) return 4;
  if (epi == 0 && N % 8 == 0 && N > 0) {  // N tail: the width that pads fewer columns (ties: 320)
    const int p5 = (N + 319) / 320 * 320, p4 = (N + 255) / 256 * 256;
    return p4 < p5 ? 4 : 5;
  }
  return 0;
}

bool launch(const Args& p, int epi, int fn, hipStream_t s) {
  if (p.M % BM || p.M <= 0 || p.N <= 0 || p.K <= 0) return false;
  // K tail (K % 8 == 0) and N tail (N % 8 == 0): plain C = A·Bᵀ only
  if (epi == 0 ? (p.K % 8 || p.N % 8) : (p.K % BK != 0)) return false;
  if (fn == 0) fn = pick_fn(p.N, epi, p.half);
  if (fn != 4 && fn != 5) return false;
  if (epi != 0 && p.N % (64 * fn)) return false;
  // one DMA descriptor per operand with 32-bit offsets: both extents below 2 GiB
  const int64_t lim = (int64_t)0x7fffffff - (1 << 20);
  if (((int64_t)(BM - 1) * p.lda + p.K) * 2 >= lim || ((int64_t)(p.N - 1) * p.ldb + p.K) * 2 >= lim) return false;
  // the EPI 0-2 epilogue streams (C, h, y) go through per-tile buffer descriptors with 32-bit byte
  // offsets from the tile's first row: one tile's row range must stay below 2 GiB (EPI 3 stores
  // through 64-bit pointers)
  if (epi != 3) {
    const int64_t c_cols = epi == 2 ? (int64_t)p.N + p.half : (int64_t)p.N;  // EPI 2: [da|db]
    if (((int64_t)(BM - 1) * p.ldc + c_cols) * 2 >= lim) return false;
    if (epi == 1 && ((int64_t)(BM - 1) * p.ldh + p.half) * 2 >= lim) return false;
    if (epi == 2 && ((int64_t)(BM - 1) * p.ldy + p.N + p.half) * 2 >= lim) return false;
  }
#define CS336_G8(F, E)        \
  do {                        \
    launch_t<F, E>(p, s);     \
    return true;              \
  } while (0)
  if (fn == 5) {
    if (epi == 0) CS336_G8(5, 0);
    if (epi == 1) CS336_G8(5, 1);
    if (epi == 2) CS336_G8(5, 2);
    if (epi == 3) CS336_G8(5, 3);
  } else {
    if (epi == 0) CS336_G8(4, 0);
    if (epi == 1) CS336_G8(4, 1);
    if (epi == 2) CS336_G8(4, 2);
    if (epi == 3) CS336_G8(4, 3);
  }
#undef CS336_G8
  return false;
}

}  // namespace gemm8
}  // namespace cs336
