// FlashAttention-2 backward, key-block parallel: ONE main kernel with the five MFMA products per
// tile pair (S, dP, dVᵀ, dKᵀ, dQ), one workgroup per 256-key block, dQ summed across key blocks
// (slabs or fp32 atomics, below). For the shapes the head-sequential kernels (fa_bwd_hs.hip /
// fa_bwd_fused.hip: d 64, N <= 1024, B·H >= 512) do not serve: d_head 80 (the 2.7b model) and long
// d 64 sequences (the reference's FA benchmark at N 4096, B·H 64: 16 key blocks x 64 heads = 1024
// workgroups; the leaderboard's N 16384).
// cs336-build: no-slp
//
// Parity: reference cs336_systems/flash_attention.py:270-289 (recompute backward, there over the
// full N x N matrices; handout Algorithm 2). fa_bwd.hip's two-kernel form computes S and dP in both
// kernels (7 GEMM-equivalents per tile pair); this one computes them once.
//
// The dQ sum across key blocks: up to 4 key blocks (N <= 1024, the 2.7b step) each block writes its
// dQ contribution with plain stores into its own fp32 slab (slab kb holds rows kbase.. under the
// causal mask, every row otherwise) and the convert launch sums the slabs in key-block order --
// deterministic, and 4.5 % faster than atomics there. Longer sequences use no-return
// global_atomic_add_f32 into one zeroed accumulator (16 per tile and wave, one accumulator register
// each = two 128-B row segments, the full-rate shape; not bitwise reproducible): the convert would
// read nkb / 2 slabs per row.
//
// Launches: (1) prep: per query row -lse·log2(e) and -delta (delta = rowsum(dO·O)) in the row order
// the accumulators want (row_perm) (+ the atomic accumulator zeroed); (2) the main kernel;
// (3) dQ = scale · (sum of the slabs | acc) cast to the output dtype (inverse RoPE folded in when q
// was rotated).
//
// Main kernel structure: WV = 8 waves (two per SIMD, <= 256 registers each; the default) or 4
// (one per SIMD, up to 512 registers), wave w owns 32 keys (8 waves) or 64 keys as two 32-key groups
// (4 waves) of the block (key on the MFMA lane), keeping dKᵀ / dVᵀ of its keys and V (B operand of
// dP) in registers; K lives in one LDS image read by rows (S) and by
// columns (dQ). The workgroup sweeps 64-row query slices (Q, dO and the slice's row constants staged
// by LDS-DMA in a 3-slot ring, two slices ahead); per 32-query tile and group:
//   S = Q Kᵀ, dP = dO Vᵀ - delta (row constant as the accumulator's start), P = exp2(S c - L),
//   dS = P dP, dVᵀ += dOᵀ P, dKᵀ += Qᵀ dS (accumulators as B operands, dOᵀ / Qᵀ by transposed LDS
//   reads of the same slot images), dSᵀ -> LDS;
// barrier; each wave forms its dQ tile(s) (32 q x 32 d) = dS K over the active keys (both operands
// transposed reads) and issues their stores / atomics at the start of the next slice, so a slice's DMA
// wait stays a compile-time count (stores and DMA share vmcnt, which retires in issue order). Waves 0-3
// stage the slices (TileDma's 4 x 64-lane rounds); with 8 waves, waves 4-7 issue no DMA.
// Causal: key block 0 (the heaviest) of every head is dispatched first; the slices start at the
// block's diagonal and only diagonal tiles are masked.
#include "fa_common.h"

namespace cs336 {
namespace fa {

namespace {
constexpr int KP_KB = 256;  // keys per workgroup
constexpr int KP_BQ = 64;   // query slice
constexpr int64_t KP_SLAB_LIMIT = (int64_t)4 << 30;  // bytes of dQ slabs before the atomic fallback

// waves per workgroup: 4 (one per SIMD, 64 keys = two 32-key groups each) or 8 (two per SIMD, one group
// each: a second wave on every SIMD covers the first one's LDS and barrier latencies): 8 by default,
// 1.15-1.45x the 4-wave form at every measured shape (profiles/r6_fa_kp_waves.md; the d 80 non-causal
// build spills 13-15 registers and still wins); CS336_FA_KP_WAVES=4 selects the 4-wave form.
inline int kp_waves(const AttnBwdParams&) {
  const char* e = getenv("CS336_FA_KP_WAVES");
  return (e && *e && atoi(e) == 4) ? 4 : 8;
}

inline int kp_nkb(const AttnBwdParams& bp) { return (bp.f.Nq + KP_KB - 1) / KP_KB; }
// slabs up to 4 key blocks (N <= 1024): B 32 H 32 N 1024 d 80 causal 1.11 vs 1.16 ms with atomics;
// at N 4096 (16 blocks; the convert then reads 8.5 slabs per row) atomics win, 0.70 vs 0.80 ms
// (profiles/r6_fa_kp_waves.md). CS336_FA_KP_SLAB=0|1 forces one (slabs only within KP_SLAB_LIMIT).
inline bool kp_slabs(const AttnBwdParams& bp) {
  const char* e = getenv("CS336_FA_KP_SLAB");
  const bool want = (e && *e) ? atoi(e) != 0 : kp_nkb(bp) <= 4;
  return want && (int64_t)kp_nkb(bp) * bp.f.B * bp.f.H * bp.f.Nq * bp.f.D * 4 <= KP_SLAB_LIMIT;
}

template <int D, int WV>
struct KpGeo {
  static constexpr int GPW = 8 / WV;            // 32-key groups per wave
  static constexpr int DP = PadD<D>::value;     // compute width (80 -> 96: d >= D zero in the images)
  static constexpr int RB = DP * 2;             // Q / dO / K image row bytes
  static constexpr int CPR = RB / 16;
  static constexpr int CREAL = D * 2 / 16;      // 16-B chunks with data
  static constexpr int NDT = DP / 32, NKS = DP / 16;
  static constexpr int NKR = (D + 15) / 16;     // k-steps of S / dP over the real d (d 80: 5 of 6)
  static constexpr int TILE = KP_BQ * RB;       // one slice image
  static constexpr int SLOT = 2 * TILE + 1024;  // Q | dO | row constants (512 B used)
  static constexpr int NS = 3;
  static constexpr int OFF_K = NS * SLOT;
  static constexpr int OFF_DS = OFF_K + KP_KB * RB;  // dSᵀ [key][64 q], 128-B rows
  static constexpr int LDS = OFF_DS + KP_KB * 128;
  static constexpr int NQT = 2 * NDT;                // dQ tiles (32 q x 32 d) per slice
  static constexpr int SLICE_DMA = 2 * (KP_BQ * CPR / 256);  // Q + dO wave-instructions per wave
  static_assert(LDS <= 160 * 1024, "LDS budget");
  // dQ tiles of wave w (w, w + WV, ... < NQT) and the vmcnt a slice's wait may leave in flight: this
  // wave's dQ stores of the previous slice (issued after that slice's DMA) + the next slice's DMA
  // (waves 0-3 stage the slices: TileDma's 4 x 64-lane rounds)
  static constexpr int tiles(int w) { return (w < NQT ? 1 : 0) + (w + WV < NQT ? 1 : 0) + (w + 2 * WV < NQT ? 1 : 0); }
  static constexpr int inflight(int w) { return 16 * tiles(w) + SLICE_DMA + (w == 0 ? 1 : 0); }
  static_assert(inflight(0) <= 63, "vmcnt range");
};

// transposed-fragment offsets (ds_read_b64_tr_b16 pair, see lds_tr_frag) of column tile c (32
// elements) in an image with R-byte rows, for a row base that is a multiple of 16 rows
template <int R>
__device__ __forceinline__ void tr_offsets(int lane, int c, uint32_t& oa, uint32_t& ob) {
  const int hh = lane >> 5, ti = lane & 15;
  const int tra = 4 * hh + (ti >> 2), tcl = ((lane >> 4) & 1) * 2 + ((ti & 3) >> 1);
  const int ch = (c << 2) | tcl;
  oa = (uint32_t)(tra * R + ((ch ^ swz<R>(tra)) << 4) + (ti & 1) * 8);
  ob = (uint32_t)((tra + 8) * R + ((ch ^ swz<R>(tra + 8)) << 4) + (ti & 1) * 8);
}
}  // namespace

// ---- (1) row constants + zeroed dQ accumulator ------------------------------------------------
// block = (head, 64-row slice); 4 threads per row, each over 16-B chunks c, c+4, ... of d
template <typename T, int D, bool SLAB>
__global__ __launch_bounds__(256) void fa_bwd_kp_prep(const AttnBwdParams bp, float* __restrict__ rowc,
                                                      float* __restrict__ acc) {
  typedef typename Elem<T>::storage S;
  const int N = bp.f.Nq, nqs = N / KP_BQ;
  const int bh = blockIdx.x / nqs, s = blockIdx.x % nqs;
  const int b = bh / bp.f.H, h = bh % bp.f.H;
  const int tid = threadIdx.x, r = tid >> 2, k = tid & 3, row = s * KP_BQ + r;
  const S* o = (const S*)bp.f.o + b * bp.f.o_sb + h * bp.f.o_sh + (int64_t)row * bp.f.o_sn;
  const S* g = (const S*)bp.dout + b * bp.do_sb + h * bp.do_sh + (int64_t)row * bp.do_sn;
  float dsum = 0.f;
#pragma unroll
  for (int c = k; c < D / 8; c += 4) {
    const uint4 uo = *reinterpret_cast<const uint4*>(o + 8 * c);
    const uint4 ug = *reinterpret_cast<const uint4*>(g + 8 * c);
    const uint32_t wo[4] = {uo.x, uo.y, uo.z, uo.w}, wg[4] = {ug.x, ug.y, ug.z, ug.w};
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      dsum = fmaf(Elem<T>::to_f((S)(wo[w] & 0xffff)), Elem<T>::to_f((S)(wg[w] & 0xffff)), dsum);
      dsum = fmaf(Elem<T>::to_f((S)(wo[w] >> 16)), Elem<T>::to_f((S)(wg[w] >> 16)), dsum);
    }
  }
  dsum += __shfl_xor(dsum, 1, 64);
  dsum += __shfl_xor(dsum, 2, 64);
  float* rc = rowc + ((int64_t)bh * nqs + s) * 128;
  if (k == 0) {
    rc[row_perm(r)] = -bp.f.lse[(int64_t)bh * N + row] * kLog2e;
    rc[64 + row_perm(r)] = -dsum;
  }
  if constexpr (!SLAB) {
    float4* z = reinterpret_cast<float4*>(acc + ((int64_t)bh * N + s * KP_BQ) * D);
    for (int i = tid; i < KP_BQ * D / 4; i += 256) z[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// ---- (2) main kernel ---------------------------------------------------------------------------
template <typename T, int D, bool CAUSAL, bool ROPE, bool SLAB, int WV>
__global__ __launch_bounds__(64 * WV, 1) void fa_bwd_kp_kernel(const AttnBwdParams bp, const float* __restrict__ rowc,
                                                               float* __restrict__ acc) {
  using G = KpGeo<D, WV>;
  constexpr int GPW = G::GPW;
  typedef typename Elem<T>::storage S;
  typedef typename Mma16<T>::frag F;
  constexpr int DP = G::DP, RB = G::RB, NDT = G::NDT, NKS = G::NKS, NKR = G::NKR, CREAL = G::CREAL;
  __shared__ __attribute__((aligned(1024))) char smem[G::LDS];

  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  const int l32 = lane & 31, hh = lane >> 5;
  const int BH = bp.f.B * bp.f.H;
  // key block 0 (all queries attend to it: the heaviest under the causal mask) of every head first
  const int kb = blockIdx.x / BH, bh = blockIdx.x % BH;
  const int b = bh / bp.f.H, h = bh % bp.f.H;
  const int N = bp.f.Nq, nqs = N / KP_BQ;
  const int kbase = kb * KP_KB;
  const S* Qp = (const S*)bp.f.q + b * bp.f.q_sb + h * bp.f.q_sh;
  const S* Kp = (const S*)bp.f.k + b * bp.f.k_sb + h * bp.f.k_sh;
  const S* Vp = (const S*)bp.f.v + b * bp.f.v_sb + h * bp.f.v_sh;
  const S* dOp = (const S*)bp.dout + b * bp.do_sb + h * bp.do_sh;
  const float sc = bp.f.scale, c2 = bp.f.scale * kLog2e;

  if constexpr (DP != D) {
    // d 80 runs as 96: the pad columns of every image must read as zeros (the DMA never writes them);
    // all of LDS is zeroed before any wave issues a DMA into it
    for (int o = tid * 16; o < G::LDS; o += 64 * WV * 16) *reinterpret_cast<uint4*>(smem + o) = make_uint4(0, 0, 0, 0);
    __syncthreads();
  }

  // ---- per-lane LDS offsets (row bases are multiples of 16 rows: the swizzle is the lane's) ----
  uint32_t roff[NKS];  // row fragments: row l32, chunk 2ks + hh
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) roff[ks] = (uint32_t)(l32 * RB + (((2 * ks + hh) ^ swz<RB>(l32)) << 4));
  uint32_t toa[NDT], tob[NDT];  // transposed fragments of d column tile dt (Q, dO, K images)
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) tr_offsets<RB>(lane, dt, toa[dt], tob[dt]);
  uint32_t dsa[2], dsb[2];  // transposed fragments of query column tile qq (dSᵀ image)
#pragma unroll
  for (int qq = 0; qq < 2; ++qq) tr_offsets<128>(lane, qq, dsa[qq], dsb[qq]);
  auto rowf = [&](const char* img, int ks) -> F { return as_frag<T>(*reinterpret_cast<const uint4*>(img + roff[ks])); };
  auto trf2 = [&](const char* img, uint32_t oa, uint32_t ob) -> F {
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + oa));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + ob));
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    s16x8 v;
    v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
    v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
    return __builtin_bit_cast(F, v);
  };

  // ---- LDS-DMA staging --------------------------------------------------------------------------
  TileDma<KP_BQ, RB, CREAL, 2> dq_, dd_;  // Q / dO slices (waves 0-3)
  const bool stager = WV == 4 || wave < 4;
  dq_.init(wave & 3, lane, bp.f.q_sn);
  dd_.init(wave & 3, lane, bp.do_sn);
  const int64_t nrc = (int64_t)nqs * 512;  // this head's row constants: 512 B per slice
  const __amdgpu_buffer_rsrc_t rrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(rowc + (int64_t)bh * nqs * 128), (short)0, (int)nrc, 0x00020000);
  const uint32_t vrc = lane < 32 ? (uint32_t)(lane * 16) : 0x80000000u;  // lanes 32-63: out of range
  auto issue_slot = [&](int s, int slot) {
    if (!stager) return;
    char* base = smem + slot * G::SLOT;
    dq_.issue(Qp + (int64_t)s * KP_BQ * bp.f.q_sn, KP_BQ, bp.f.q_sn, base, wave);
    dd_.issue(dOp + (int64_t)s * KP_BQ * bp.do_sn, KP_BQ, bp.do_sn, base + G::TILE, wave);
    if (wave == 0) dma16(rrc, lds_addr(base + 2 * G::TILE), vrc, (uint32_t)(s * 512));
  };
  char* const Kimg = smem + G::OFF_K;
  char* const dsimg = smem + G::OFF_DS;
  {
    TileDma<KP_KB, RB, CREAL, 2> dk_;
    if (stager) {
      dk_.init(wave, lane, bp.f.k_sn);
      dk_.issue(Kp + (int64_t)kbase * bp.f.k_sn, min(KP_KB, N - kbase), bp.f.k_sn, Kimg, wave);
    }
  }
  const int s0 = CAUSAL ? kbase / KP_BQ : 0;
  if (s0 < nqs) issue_slot(s0, 0);
  if (s0 + 1 < nqs) issue_slot(s0 + 1, 1);

  // ---- per-wave state: keys kw + 32g + l32, g < GPW ------------------------------------------------
  const int kw = kbase + 32 * GPW * wave;
  uint4 vf[GPW][NKR];  // V as the B operand of dP (key on the lane), d = 16ks + 8hh .. +7
#pragma unroll
  for (int g = 0; g < GPW; ++g) {
    const int key = min(kw + 32 * g + l32, N - 1);  // keys >= N: whole skipped groups (N % 64 == 0)
#pragma unroll
    for (int ks = 0; ks < NKR; ++ks) {
      const int d = 16 * ks + 8 * hh;
      vf[g][ks] = (DP == D || d < D) ? *reinterpret_cast<const uint4*>(Vp + (int64_t)key * bp.f.v_sn + d)
                                     : make_uint4(0, 0, 0, 0);
    }
  }
  f32x16 dk[GPW][NDT], dv[GPW][NDT];
#pragma unroll
  for (int g = 0; g < GPW; ++g)
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      dk[g][dt] = zero16();
      dv[g][dt] = zero16();
    }
  // pending dQ tiles of the previous slice (atomics issued after the next slice's wait)
  constexpr int MT = G::tiles(0);
  f32x16 dqp[MT];
  int dq_row0 = -1;  // first query row of the pending slice (-1: none)
  float* const accb = acc + ((SLAB ? (int64_t)kb * BH : 0) + bh) * N * D;  // this block's slab | the accumulator
  auto flush_dq = [&]() {
    if (dq_row0 < 0) return;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int tq = wave + WV * i;
      if (tq >= G::NQT) break;
      const int qq = tq / NDT, dt = tq % NDT, d = 32 * dt + l32;
      float* p = accb + (int64_t)(dq_row0 + 32 * qq + 4 * hh) * D + d;
      if (DP == D || d < D) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float* pr = p + (int64_t)((r & 3) + 8 * (r >> 2)) * D;
          if constexpr (SLAB) *pr = dqp[i][r];
          else unsafeAtomicAdd(pr, dqp[i][r]);
        }
      }
    }
  };

  wait_vmcnt<0>();
  dma_barrier();

  // ---- the sweep over query slices -----------------------------------------------------------------
  for (int s = s0, it = 0; s < nqs; ++s, ++it) {
    const int slot = it % G::NS;
    const char* Qs = smem + slot * G::SLOT;
    const char* dOs = Qs + G::TILE;
    const float* Ls = reinterpret_cast<const float*>(Qs + 2 * G::TILE);  // -lse·log2e, row_perm order
    const float* Ds = Ls + 64;                                           // -delta
    const int q0 = s * KP_BQ;
    // A: this slice landed (this wave may keep its previous atomics and the next slice's DMA in flight)
    if (wave == 0) wait_vmcnt<G::inflight(0)>();
    else if (wave == 1) wait_vmcnt<G::inflight(1)>();
    else if (wave == 2) wait_vmcnt<G::inflight(2)>();
    else if (wave == 3) wait_vmcnt<G::inflight(3)>();  // (waves 4-7 stage nothing)
    dma_barrier();
    // B: the previous slice's dQ atomics, then the slice two ahead (ring slot of the previous slice)
    flush_dq();
    if (s + 2 < nqs) issue_slot(s + 2, (it + 2) % G::NS);

    // C: S, dP, P, dS, dVᵀ, dKᵀ per 32-query tile and 32-key group; dSᵀ into LDS
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int qt0 = q0 + 32 * t;
      bool act[GPW], any = false;
#pragma unroll
      for (int g = 0; g < GPW; ++g) {
        const int key0 = kw + 32 * g;
        act[g] = key0 < N && (!CAUSAL || key0 <= qt0 + 31);
        any = any || act[g];
      }
      if (!any) continue;
      const char* Qt = Qs + 32 * t * RB;
      const char* dOt = dOs + 32 * t * RB;
      f32x16 sa[GPW], dp[GPW];
      {
        F qa[NKR], oa[NKR];
#pragma unroll
        for (int ks = 0; ks < NKR; ++ks) {
          qa[ks] = rowf(Qt, ks);
          oa[ks] = rowf(dOt, ks);
        }
#pragma unroll
        for (int g = 0; g < GPW; ++g) {
          if (!act[g]) continue;
          const char* Kg = Kimg + (32 * (GPW * wave + g)) * RB;
          dp[g] = *reinterpret_cast<const f32x16*>(Ds + 32 * t + 16 * hh);
          sa[g] = zero16();
#pragma unroll
          for (int ks = 0; ks < NKR; ++ks) {
            sa[g] = Mma16<T>::mma(qa[ks], rowf(Kg, ks), sa[g]);
            dp[g] = Mma16<T>::mma(oa[ks], as_frag<T>(vf[g][ks]), dp[g]);
          }
        }
      }
      F pf[GPW][2], sf[GPW][2];
#pragma unroll
      for (int g = 0; g < GPW; ++g) {
        if (!act[g]) continue;
        const int key0 = kw + 32 * g;
        const bool diag = CAUSAL && key0 + 31 > qt0;
        const int kq = key0 + l32 - qt0 - 4 * hh;  // key - (query of register 0 of this half)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const float4 L4 = *reinterpret_cast<const float4*>(Ls + 32 * t + 16 * hh + 4 * g4);
          const float Lv[4] = {L4.x, L4.y, L4.z, L4.w};
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int r = 4 * g4 + u;
            float pv = fexp2(fmaf(sa[g][r], c2, Lv[u]));
            if (diag && kq > 8 * g4 + u) pv = 0.f;
            sa[g][r] = pv;
            dp[g][r] = pv * dp[g][r];
          }
        }
        pf[g][0] = pack_acc<T>(sa[g], 0);
        pf[g][1] = pack_acc<T>(sa[g], 1);
        sf[g][0] = pack_acc<T>(dp[g], 0);
        sf[g][1] = pack_acc<T>(dp[g], 1);
        // dSᵀ rows (block-local key 32 (GPW w + g) + l32): query halves 16s2 + 4hh + 0..3 and + 8
        char* drow = dsimg + (32 * (GPW * wave + g) + l32) * 128 + 8 * hh;
        const int swl = swz<128>(l32);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const uint4 w = __builtin_bit_cast(uint4, sf[g][s2]);
          const int ch = 4 * t + 2 * s2;
          *reinterpret_cast<uint2*>(drow + ((ch ^ swl) << 4)) = make_uint2(w.x, w.y);
          *reinterpret_cast<uint2*>(drow + (((ch + 1) ^ swl) << 4)) = make_uint2(w.z, w.w);
        }
      }
      // dVᵀ += dOᵀ P, dKᵀ += Qᵀ dS, one d tile at a time (its transposed fragments serve both groups)
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        F ot[2], qt[2];
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          ot[s2] = trf2(dOt + 16 * s2 * RB, toa[dt], tob[dt]);
          qt[s2] = trf2(Qt + 16 * s2 * RB, toa[dt], tob[dt]);
        }
#pragma unroll
        for (int g = 0; g < GPW; ++g) {
          if (!act[g]) continue;
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            dv[g][dt] = Mma16<T>::mma(ot[s2], pf[g][s2], dv[g][dt]);
            dk[g][dt] = Mma16<T>::mma(qt[s2], sf[g][s2], dk[g][dt]);
          }
        }
      }
    }
    dma_barrier();  // D: every wave's dSᵀ written

    // E: dQ tiles (32 q x 32 d) = dS K over the keys active for their query tile; atomics next slice
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int tq = wave + WV * i;
      if (tq >= G::NQT) break;
      const int qq = tq / NDT, dt = tq % NDT;
      const int ng = CAUSAL ? min(8, (q0 + 32 * qq + 32 - kbase) / 32) : 8;
      const int nv = min(ng, (N - kbase) / 32);
      f32x16 a = zero16();
#pragma unroll
      for (int gg = 0; gg < 8; ++gg) {
        if (gg >= nv) break;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int r0 = 32 * gg + 16 * s2;
          a = Mma16<T>::mma(trf2(dsimg + r0 * 128, dsa[qq], dsb[qq]), trf2(Kimg + r0 * RB, toa[dt], tob[dt]), a);
        }
      }
      dqp[i] = a;
    }
    dq_row0 = q0;
  }
  flush_dq();

  // ---- dK (x scale), dV of this wave's keys: lane = key, registers = d 32dt + 8g4 + 4hh + 0..3 ----
  const Rope rope{bp.f.rope_cos, bp.f.rope_sin, D / 2};
#pragma unroll
  for (int g = 0; g < GPW; ++g) {
    const int key = kw + 32 * g + l32;
    if (key >= N) continue;
    S* rk = (S*)bp.dk + b * bp.dk_sb + h * bp.dk_sh + (int64_t)key * bp.dk_sn;
    S* rv = (S*)bp.dv + b * bp.dv_sb + h * bp.dv_sh + (int64_t)key * bp.dv_sn;
    const int64_t pos = ROPE ? (bp.f.rope_pos ? bp.f.rope_pos[(int64_t)b * N + key] : key) : 0;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = 32 * dt + 8 * g4 + 4 * hh;
        if (DP != D && d >= D) continue;
        float k0 = dk[g][dt][4 * g4] * sc, k1 = dk[g][dt][4 * g4 + 1] * sc, k2 = dk[g][dt][4 * g4 + 2] * sc,
              k3 = dk[g][dt][4 * g4 + 3] * sc;
        if constexpr (ROPE) rope_inv4(k0, k1, k2, k3, rope, pos, d);
        store4<T>(rk + d, make_float4(k0, k1, k2, k3));
        store4<T>(rv + d, make_float4(dv[g][dt][4 * g4], dv[g][dt][4 * g4 + 1], dv[g][dt][4 * g4 + 2],
                                      dv[g][dt][4 * g4 + 3]));
      }
  }
}

// ---- (3) dQ = scale · (slabs summed in key-block order | acc) (inverse RoPE when q was rotated), cast
// to the output dtype ---------------------------------------------------------------------------------
template <typename T, int D, bool ROPE, bool SLAB>
__global__ __launch_bounds__(256) void fa_bwd_kp_dq(const AttnBwdParams bp, const float* __restrict__ acc) {
  typedef typename Elem<T>::storage S;
  constexpr int Q4 = D / 4;
  const int N = bp.f.Nq;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)bp.f.B * bp.f.H * N * Q4;
  if (gid >= total) return;
  const int64_t row = gid / Q4;
  const int d = 4 * (int)(gid % Q4);
  const int bh = (int)(row / N), n = (int)(row % N);
  const int b = bh / bp.f.H, h = bh % bp.f.H;
  float4 a = *reinterpret_cast<const float4*>(acc + row * D + d);
  if constexpr (SLAB) {
    // slab kb holds this row when the row is not masked out of key block kb entirely
    const int nkb = (N + KP_KB - 1) / KP_KB, kbn = bp.f.causal ? n / KP_KB + 1 : nkb;
    const int64_t slab = total * 4;  // B·H·N·D floats
    for (int kb = 1; kb < kbn; ++kb) {
      const float4 x = *reinterpret_cast<const float4*>(acc + kb * slab + row * D + d);
      a.x += x.x;
      a.y += x.y;
      a.z += x.z;
      a.w += x.w;
    }
  }
  const float sc = bp.f.scale;
  float v0 = a.x * sc, v1 = a.y * sc, v2 = a.z * sc, v3 = a.w * sc;
  if constexpr (ROPE) {
    const Rope rope{bp.f.rope_cos, bp.f.rope_sin, D / 2};
    const int64_t pos = bp.f.rope_pos ? bp.f.rope_pos[(int64_t)b * N + n] : n;
    rope_inv4(v0, v1, v2, v3, rope, pos, d);
  }
  store4<T>((S*)bp.dq + b * bp.dq_sb + h * bp.dq_sh + (int64_t)n * bp.dq_sn + d, make_float4(v0, v1, v2, v3));
}

template <typename T, int D, bool ROPE, bool SLAB>
void launch_kp(const AttnBwdParams& bp, float* rowc, float* acc, hipStream_t s) {
  const int BH = bp.f.B * bp.f.H, N = bp.f.Nq;
  hipLaunchKernelGGL((fa_bwd_kp_prep<T, D, SLAB>), dim3((unsigned)(BH * (N / KP_BQ))), dim3(256), 0, s, bp, rowc, acc);
  const dim3 grid((unsigned)(BH * kp_nkb(bp)));
  if (kp_waves(bp) == 8) {
    if (bp.f.causal) hipLaunchKernelGGL((fa_bwd_kp_kernel<T, D, true, ROPE, SLAB, 8>), grid, dim3(512), 0, s, bp, rowc, acc);
    else hipLaunchKernelGGL((fa_bwd_kp_kernel<T, D, false, ROPE, SLAB, 8>), grid, dim3(512), 0, s, bp, rowc, acc);
  } else {
    if (bp.f.causal) hipLaunchKernelGGL((fa_bwd_kp_kernel<T, D, true, ROPE, SLAB, 4>), grid, dim3(256), 0, s, bp, rowc, acc);
    else hipLaunchKernelGGL((fa_bwd_kp_kernel<T, D, false, ROPE, SLAB, 4>), grid, dim3(256), 0, s, bp, rowc, acc);
  }
  const int64_t quads = (int64_t)BH * N * (D / 4);
  hipLaunchKernelGGL((fa_bwd_kp_dq<T, D, ROPE, SLAB>), dim3((unsigned)((quads + 255) / 256)), dim3(256), 0, s, bp, acc);
}

template <typename T, int D, bool ROPE>
void launch_kp(const AttnBwdParams& bp, float* rowc, float* acc, hipStream_t s) {
  if (kp_slabs(bp)) launch_kp<T, D, ROPE, true>(bp, rowc, acc, s);
  else launch_kp<T, D, ROPE, false>(bp, rowc, acc, s);
}

template <typename T>
void dispatch_kp(const AttnBwdParams& bp, float* rowc, float* acc, hipStream_t s) {
  const bool rope = bp.f.rope_cos != nullptr;
  if (bp.f.D == 64) {
    if (rope) launch_kp<T, 64, true>(bp, rowc, acc, s);
    else launch_kp<T, 64, false>(bp, rowc, acc, s);
  } else {
    if (rope) launch_kp<T, 80, true>(bp, rowc, acc, s);
    else launch_kp<T, 80, false>(bp, rowc, acc, s);
  }
}

}  // namespace fa

// 16-bit, d 64 or 80, self-attention with N % 64 == 0; RoPE only in the rope_out_only form (q, k
// already rotated, dq / dk returned w.r.t. the un-rotated inputs); lse contiguous (B, H, N). The DMA
// offsets are 32-bit: a 256-row K block and a 64-row slice must stay below 2 GiB (host-checked).
bool flash_attn_bwd_kp_ok(const AttnBwdParams& bp, DType t) {
  const AttnParams& p = bp.f;
  if (t == DType::F32 || (p.D != 64 && p.D != 80) || p.Nq != p.Nk || p.Nq <= 0 || p.Nq % 64) return false;
  if (p.rope_cos != nullptr && !p.rope_out_only) return false;
  const int64_t lim = (int64_t)1 << 30;
  for (int64_t st : {p.q_sn, p.k_sn, p.v_sn, bp.do_sn})
    if (st <= 0 || st * 256 * 2 >= lim) return false;
  return (int64_t)p.B * p.H * (p.Nq / 64) < (int64_t)1 << 31;
}

size_t flash_attn_bwd_kp_workspace(const AttnBwdParams& bp) {
  const size_t rows = (size_t)bp.f.B * bp.f.H * bp.f.Nq;
  const size_t nacc = fa::kp_slabs(bp) ? (size_t)fa::kp_nkb(bp) : 1;
  return rows * 2 + nacc * rows * (size_t)bp.f.D;  // floats: row constants + dQ slabs | accumulator
}

void flash_attn_bwd_kp(const AttnBwdParams& bp, DType t, float* ws, hipStream_t s) {
  if (bp.f.B * bp.f.H == 0) return;
  float* rowc = ws;
  float* acc = ws + (size_t)bp.f.B * bp.f.H * bp.f.Nq * 2;
  if (t == DType::BF16) fa::dispatch_kp<BF16>(bp, rowc, acc, s);
  else fa::dispatch_kp<F16>(bp, rowc, acc, s);
}

}  // namespace cs336
