// FlashAttention-2 backward for MI355X (gfx950 / CDNA4).
// cs336-build: no-slp
//
// Parity: reference cs336_systems/flash_attention.py:270-289 (torch.compile of a recompute
// backward that materializes the full N x N S/P/dP/dS — O(N^2) memory) and the handout's
// Algorithm 2. Here the backward is O(N) memory, atomics-free and deterministic, as two kernels:
//
//  1. fa_bwd_dq   (query-block stationary, like the forward): recomputes S^T = K Q^T and
//     dP^T = V dO^T per 64-key tile with the query on the MFMA lane, so P = exp2(S*c - L2[q]) and
//     dS = P (dP - delta[q]) use lane-local row constants; dQ^T += K^T dS^T reuses dS^T straight
//     from the accumulator as the B operand and gathers K^T with transposed LDS reads of the same
//     swizzled K image the S^T product reads row-wise. It also computes delta = rowsum(dO * O)
//     for its rows (written for kernel 2), so no separate preprocessing launch exists.
//  2. fa_bwd_dkdv (key-block stationary): per 64-query tile S = Q K^T and dP = dO V^T with the
//     KEY on the lane (cdna_hip_programming.md App. B "Attention backward": their accumulators
//     are then the B operands of dV^T += dO^T P and dK^T += Q^T dS), Q and dO staged once in
//     dual-use LDS images (row reads for S/dP, ds_read_b64_tr_b16 for the dO^T/Q^T operands);
//     the per-query L and delta are staged with the tile and read as float4 per 4 rows.
// Causal: kernel 1 stops at the diagonal, kernel 2 starts at it; only diagonal tiles are masked.
#include "fa_common.h"

#include <algorithm>

namespace cs336 {
namespace fa {

// ============================================================================================
// dQ (+ delta) kernel
// ============================================================================================
template <typename T, int D, bool CAUSAL, int ROPE, bool DMA>
__global__ __launch_bounds__(256) void fa_bwd_dq_kernel(const AttnBwdParams bp) {
  typedef typename Elem<T>::storage S;
  const AttnParams p = bp.f;  // by value: a reference would spill the kernarg struct to scratch
  constexpr bool F32 = std::is_same<T, float>::value;
  constexpr int ES = sizeof(S);
  constexpr int DP = PadD<D>::value;  // compute width (80 -> 96; d >= D is zero, never loaded/stored)
  constexpr int RB = DP * ES, CPR = RB / 16, EPC = 16 / ES, CREAL = D * ES / 16;
  // -delta as the dP accumulators' initial value (+1-2 % at d64/d128); at the padded d80 the extra
  // live row constants cost more than the saved subtraction (-17 %), so it keeps the explicit form
  constexpr bool DINIT = DP == D;
  // D=128 streams 32-key tiles: halves the S^T/dP^T/staging registers so the kernel fits 256
  // VGPRs without spilling (64-key tiles spilled at occupancy 1)
  constexpr int BM = 128, BN = DP == 128 ? 32 : 64;
  constexpr int NT = BN / 32;
  constexpr int TILE = BN * RB;
  constexpr int LPT = BN * CPR / 256;
  static_assert(BN * CPR % 256 == 0, "staging rounds must be whole");
  constexpr int NDT = DP / 32;
  // no register prefetch of the next tile at fp32 d128: it fits (no scratch) but measured 2-10 %
  // slower on every fp32 d128 shape (profiles/r4_fa_fp32_prefetch.md)
  constexpr bool PREFETCH = !(F32 && D == 128);
  static_assert(!DMA || (!F32 && ROPE != 1), "LDS-DMA staging: 16-bit, no RoPE-on-load");
  constexpr int NS = DMA ? 3 : 2;  // K/V ring depth
  // VGPR-staged loop unrolled by two (compile-time slots, immediate LDS offsets): 5.3 instead of 7.6
  // VALU per MFMA at d64 (+6 % backward); at d80/d128 the extra live registers cost more (-10-16 %)
  constexpr bool UNROLL2 = DP <= 64;
  // LDS-DMA loop unrolled by its ring depth at every d (no staging registers to add): d128 causal
  // backward 492 -> 531 TF (profiles/r2_fa_bwd_valu.md)
  constexpr bool DUNROLL = true;

  __shared__ __attribute__((aligned(1024))) char smem[NS * 2 * TILE];

  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  const int l32 = lane & 31, hh = lane >> 5;
  const int nqb = (p.Nq + BM - 1) / BM;
  // key splits (low parallelism, bp.ksplit > 1): consecutive blocks are the splits of one query block
  const int nsplit = bp.ksplit, sp = (int)(blockIdx.x % (unsigned)nsplit);
  int bh, qb;
  tile_order((int)(blockIdx.x / (unsigned)nsplit), p.B * p.H, nqb, CAUSAL ? p.order : 0, p.lpt_group, bh, qb);
  if (CAUSAL) qb = nqb - 1 - qb;
  const int b = bh / p.H, h = bh % p.H;
  const int q0 = qb * BM;
  const int qw0 = q0 + wave * 32;
  const int qrow = qw0 + l32;
  const bool valid_q = qrow < p.Nq;

  const S* Qp = (const S*)p.q + b * p.q_sb + h * p.q_sh;
  const S* Kp = (const S*)p.k + b * p.k_sb + h * p.k_sh;
  const S* Vp = (const S*)p.v + b * p.v_sb + h * p.v_sh;
  const S* Op = (const S*)p.o + b * p.o_sb + h * p.o_sh;
  const S* dOp = (const S*)bp.dout + b * bp.do_sb + h * bp.do_sh;
  S* dQp = (S*)bp.dq + b * bp.dq_sb + h * bp.dq_sh;
  const int64_t row_lin = ((int64_t)b * p.H + h) * p.Nq + qrow;

  const Rope rope{p.rope_cos, p.rope_sin, D / 2};
  const int64_t* rpos = p.rope_pos ? p.rope_pos + (int64_t)b * p.Nq : nullptr;
  const int64_t qpos = rpos && valid_q ? rpos[qrow] : qrow;
  constexpr int NQF = F32 ? DP / 8 : DP / 16;
  uint4 qf[NQF], dof[NQF];
  float delta = 0.f;
#pragma unroll
  for (int i = 0; i < NQF; ++i) {
    const int e = F32 ? (hh * (DP / 2) + 4 * i) : (16 * i + 8 * hh);
    if (valid_q && (DP == D || e < D)) {
      qf[i] = *reinterpret_cast<const uint4*>(Qp + (int64_t)qrow * p.q_sn + e);
      if (ROPE == 1) qf[i] = rope_chunk<T>(qf[i], rope, qpos, e, 1.f);
      dof[i] = *reinterpret_cast<const uint4*>(dOp + (int64_t)qrow * bp.do_sn + e);
      // delta partial over this lane's half of d
#pragma unroll
      for (int k = 0; k < EPC; k += 4) {
        const float4 a = load4<T>(dOp + (int64_t)qrow * bp.do_sn + e + k);
        const float4 c = load4<T>(Op + (int64_t)qrow * p.o_sn + e + k);
        delta += a.x * c.x + a.y * c.y + a.z * c.z + a.w * c.w;
      }
    } else {
      qf[i] = dof[i] = make_uint4(0, 0, 0, 0);
    }
  }
  delta += __shfl_xor(delta, 32, 64);
  const float lse2 = valid_q ? p.lse[row_lin] * kLog2e : INFINITY;
  // row constants of the dK/dV kernel, pre-transformed so they load straight into its accumulators
  if (valid_q && hh == 0 && sp == 0) {
    bp.delta[row_lin] = -delta;
    bp.lrow[row_lin] = -lse2;
  }

  const int kv_end = CAUSAL ? min(p.Nk, q0 + BM) : p.Nk;
  // this block's key tiles [jt0, jt0 + ntiles) (all unless split); tile indices j are relative to jt0
  const int ntiles_all = (kv_end + BN - 1) / BN;
  const int jt0 = (int)((int64_t)ntiles_all * sp / nsplit);
  const int ntiles = (int)((int64_t)ntiles_all * (sp + 1) / nsplit) - jt0;

  uint4 kst[LPT], vst[LPT];
  RopeCoef kst_rc[ROPE == 1 ? LPT : 1];  // rotation applied at LDS-write time (keeps the prefetch async)
  auto gload = [&](int j) {
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int c = tid + 256 * i;
      const int r = c / CPR, ch = c % CPR;
      const int key = (jt0 + j) * BN + r;
      if (ROPE == 1) kst_rc[i] = rope_coef<T>(rope, key < p.Nk ? (rpos ? rpos[key] : key) : 0, ch < CREAL ? ch * EPC : 0);
      if (key < p.Nk && (CREAL == CPR || ch < CREAL)) {
        kst[i] = *reinterpret_cast<const uint4*>(Kp + (int64_t)key * p.k_sn + ch * EPC);
        vst[i] = *reinterpret_cast<const uint4*>(Vp + (int64_t)key * p.v_sn + ch * EPC);
      } else {
        kst[i] = make_uint4(0, 0, 0, 0);
        vst[i] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto swrite = [&](int buf) {
    char* Ks = smem + buf * 2 * TILE;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int c = tid + 256 * i;
      const int off = lds_off<RB>(c / CPR, c % CPR);
      *reinterpret_cast<uint4*>(Ks + off) = ROPE == 1 ? rope_apply<T>(kst[i], kst_rc[i]) : kst[i];
      *reinterpret_cast<uint4*>(Ks + TILE + off) = vst[i];
    }
  };

  f32x16 dq[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i) dq[i] = zero16();
  const float c2 = p.scale * kLog2e;

  // one K/V tile: S^T, dP^T, dS^T, dQ^T += K^T dS^T (Ks: the tile's K image, V after it)
  auto tile = [&](int j, const char* Ks) __attribute__((always_inline)) {
    const int kt0 = (jt0 + j) * BN;
    const bool active = !CAUSAL || kt0 <= qw0 + 31;
    if (active) {
      const char* Vs = Ks + TILE;
      f32x16 s[NT], dp[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        s[t] = zero16();
        // row constant as the initial accumulator: dP' = dO V^T - delta[q] leaves the chain ready
        // for dS = P dP' (one VALU op per element fewer; the query is on the lane)
#pragma unroll
        for (int r = 0; r < 16; ++r) dp[t][r] = DINIT ? -delta : 0.f;
        if constexpr (F32) {
#pragma unroll
          for (int i = 0; i < DP / 8; ++i) {
            const float4 kv = lds_f4<RB>(Ks, 32 * t + l32, hh * (DP / 2) + 4 * i);
            const float4 vv = lds_f4<RB>(Vs, 32 * t + l32, hh * (DP / 2) + 4 * i);
            const float4 qv = __builtin_bit_cast(float4, qf[i]);
            const float4 gv = __builtin_bit_cast(float4, dof[i]);
            s[t] = mma_f32(kv.x, qv.x, s[t]);
            s[t] = mma_f32(kv.y, qv.y, s[t]);
            s[t] = mma_f32(kv.z, qv.z, s[t]);
            s[t] = mma_f32(kv.w, qv.w, s[t]);
            dp[t] = mma_f32(vv.x, gv.x, dp[t]);
            dp[t] = mma_f32(vv.y, gv.y, dp[t]);
            dp[t] = mma_f32(vv.z, gv.z, dp[t]);
            dp[t] = mma_f32(vv.w, gv.w, dp[t]);
          }
        } else {
#pragma unroll
          for (int ks = 0; ks < DP / 16; ++ks) {
            s[t] = Mma16<T>::mma(lds_row_frag<T, RB>(Ks, 32 * t, ks, lane), as_frag<T>(qf[ks]), s[t]);
            dp[t] = Mma16<T>::mma(lds_row_frag<T, RB>(Vs, 32 * t, ks, lane), as_frag<T>(dof[ks]), dp[t]);
          }
        }
      }
      const bool need_mask = (kt0 + BN > p.Nk) || (CAUSAL && kt0 + BN - 1 > qw0);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float pv = fexp2(fmaf(s[t][r], c2, -lse2));
          if (need_mask) {
            const int key = kt0 + 32 * t + acc_row(r, hh);
            if (key >= p.Nk || (CAUSAL && key > qrow)) pv = 0.f;
          }
          s[t][r] = DINIT ? pv * dp[t][r] : pv * (dp[t][r] - delta);  // dS^T
        }
      if constexpr (F32) {
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
          for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r)
              dq[dt] = mma_f32(lds_f1<RB>(Ks, 32 * t + acc_row(r, hh), dt * 32 + l32), s[t][r], dq[dt]);
      } else {
        typename Mma16<T>::frag pf[NT][2];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          pf[t][0] = pack_acc<T>(s[t], 0);
          pf[t][1] = pack_acc<T>(s[t], 1);
        }
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
          for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)
              dq[dt] = Mma16<T>::mma(lds_tr_frag<T, RB>(Ks, 32 * t, s2, dt, lane), pf[t][s2], dq[dt]);
      }
    }
  };

  if constexpr (DMA) {
    using Dma = TileDma<BN, RB, CREAL, ES>;
    Dma kd, vd;
    kd.init(wave, lane, p.k_sn);
    vd.init(wave, lane, p.v_sn);
    if (D != DP || p.Nk % BN != 0) {  // some slots are read out of range: start from zeros
      lds_zero(smem, NS * 2 * TILE);
      __syncthreads();
    }
    auto issue = [&](int j) {
      char* Ks = smem + (j % NS) * 2 * TILE;
      const int rows = min(BN, p.Nk - (jt0 + j) * BN);
      kd.issue(Kp + (int64_t)(jt0 + j) * BN * p.k_sn, rows, p.k_sn, Ks, wave);
      vd.issue(Vp + (int64_t)(jt0 + j) * BN * p.v_sn, rows, p.v_sn, Ks + TILE, wave);
    };
#pragma unroll
    for (int t = 0; t < NS - 1; ++t)
      if (t < ntiles) issue(t);
    // the resident Q / dO fragments retired, stated to the compiler (see the dK/dV kernel's prologue)
    __builtin_amdgcn_s_waitcnt(0x0F70);
    auto dstep = [&](int j, auto slot) __attribute__((always_inline)) {
      if (NS == 3 && j + 1 < ntiles) wait_vmcnt<2 * Dma::PER_WAVE>();
      else wait_vmcnt<0>();
      dma_barrier();
      if (j + NS - 1 < ntiles) issue(j + NS - 1);
      const int B = slot;  // integral_constant (unrolled loop) or runtime slot
      tile(j, smem + B * 2 * TILE);
    };
    int j = 0;
    if constexpr (DUNROLL && NS == 3) {  // unrolled by the ring depth: compile-time slots
      for (; j + 2 < ntiles; j += 3) {
        dstep(j, std::integral_constant<int, 0>{});
        dstep(j + 1, std::integral_constant<int, 1>{});
        dstep(j + 2, std::integral_constant<int, 2>{});
      }
    }
    for (; j < ntiles; ++j) dstep(j, j % NS);
  } else {
    if (ntiles > 0) {
      gload(0);
      swrite(0);
    }
    __syncthreads();
    // unrolled by two with compile-time slots: the slots' LDS addresses become immediates
    auto step = [&](int j, auto slot) __attribute__((always_inline)) {
      const int B = slot;  // integral_constant (unrolled loop) or runtime slot
      if (PREFETCH && j + 1 < ntiles) gload(j + 1);
      tile(j, smem + B * 2 * TILE);
      if (j + 1 < ntiles) {
        if (PREFETCH) {
          swrite(B ^ 1);
        } else {
          __syncthreads();
          gload(j + 1);
          swrite(0);
        }
      }
      __syncthreads();
    };
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, PREFETCH ? 1 : 0>;
    int j = 0;
    if constexpr (UNROLL2) {
      for (; j + 1 < ntiles; j += 2) {
        step(j, S0{});
        step(j + 1, S1{});
      }
    }
    for (; j < ntiles; ++j) step(j, PREFETCH ? (j & 1) : 0);
  }

  if (nsplit > 1) {  // unscaled fp32 partial of this key range (summed by fa_bwd_reduce_kernel)
    if (valid_q) {
      float* prow = bp.dq_part + (((int64_t)sp * p.B * p.H + bh) * p.Nq + qrow) * D;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int d = dt * 32 + 8 * g + 4 * hh;
          if (DP != D && d >= D) continue;
          *reinterpret_cast<float4*>(prow + d) = make_float4(dq[dt][4 * g], dq[dt][4 * g + 1], dq[dt][4 * g + 2], dq[dt][4 * g + 3]);
        }
    }
    return;
  }
  if (valid_q) {
    S* row = dQp + (int64_t)qrow * bp.dq_sn;
    const float sc = p.scale;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = dt * 32 + 8 * g + 4 * hh;
        if (DP != D && d >= D) continue;
        float v0 = dq[dt][4 * g] * sc, v1 = dq[dt][4 * g + 1] * sc, v2 = dq[dt][4 * g + 2] * sc,
              v3 = dq[dt][4 * g + 3] * sc;
        if (ROPE != 0) rope_inv4(v0, v1, v2, v3, rope, qpos, d);  // dQ w.r.t. the un-rotated q
        store4<T>(row + d, make_float4(v0, v1, v2, v3));
      }
  }
}

// ============================================================================================
// dK / dV kernel
// ============================================================================================
// Occupancy hint: 16-bit D=64 asks for two workgroups per CU explicitly (same occupancy as without
// the hint, but the register schedule it produces measured 2-5 % faster at N=512 and 4096); at D=128
// the hint spills the resident K/V fragments (1153 -> 1461 us at N=4096), so D=128 runs one per CU.
template <typename T, int D>
constexpr int dkdv_min_waves() {
  return (D == 64 && !std::is_same<T, float>::value) ? 2 : 1;
}

template <typename T, int D, bool CAUSAL, int ROPE, bool DMA>
__global__ __launch_bounds__(256, (dkdv_min_waves<T, D>())) void fa_bwd_dkdv_kernel(const AttnBwdParams bp) {
  typedef typename Elem<T>::storage S;
  const AttnParams p = bp.f;  // by value: a reference would spill the kernarg struct to scratch
  constexpr bool F32 = std::is_same<T, float>::value;
  constexpr int ES = sizeof(S);
  constexpr int DP = PadD<D>::value;  // compute width (80 -> 96; d >= D is zero, never loaded/stored)
  constexpr int RB = DP * ES, CPR = RB / 16, EPC = 16 / ES, CREAL = D * ES / 16;
  // -delta as the dP accumulators' initial value (+1-2 % at d64/d128); at the padded d80 the extra
  // live row constants cost more than the saved subtraction (-17 %), so it keeps the explicit form
  // (16-bit only: with the fp32 MFMA chains the accumulator-initialising loads crash hipcc's
  // AGPR-copy rewrite in the d128 instances)
  constexpr bool DINIT = DP == D && !F32;
  // 64-query tiles; at D=128 (one workgroup per CU anyway) part of the state lives in AGPRs
  // rather than halving the tile: 1153 -> 1046 us at N=4096 (fp32 keeps 32-query tiles)
  constexpr int BK = 128, BQ = (D == 128 && std::is_same<T, float>::value) ? 32 : 64;
  constexpr int NT = BQ / 32;
  constexpr int TILE = BQ * RB;
  constexpr int BUF = 2 * TILE + 2 * BQ * 4;  // Q, dO images + L2, delta rows
  constexpr int LPT = BQ * CPR / 256;
  static_assert(BQ * CPR % 256 == 0, "staging rounds must be whole");
  constexpr int NDT = DP / 32;
  constexpr bool PREFETCH = !(F32 && D == 128);  // see fa_bwd_dq_kernel
  static_assert(!DMA || (!F32 && ROPE != 1), "LDS-DMA staging: 16-bit, no RoPE-on-load");
  // LDS-DMA slot: Q, dO images, then L and delta in 1 KB regions (one wave-instruction each)
  constexpr int BUFD = 2 * TILE + 2048;
  constexpr int NS = DMA ? (DP <= 96 ? 3 : 2) : (PREFETCH ? 2 : 1);
  constexpr int SLOT = DMA ? BUFD : BUF;
  constexpr bool UNROLL2 = DP <= 64;  // see fa_bwd_dq_kernel
  // LDS-DMA loop unrolled by its ring depth at every d (no staging registers to add): d128 causal
  // backward 492 -> 531 TF (profiles/r2_fa_bwd_valu.md)
  constexpr bool DUNROLL = true;

  __shared__ __attribute__((aligned(1024))) char smem[NS * SLOT];

  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  const int l32 = lane & 31, hh = lane >> 5;
  const int nkb = (p.Nk + BK - 1) / BK;
  // query splits (low parallelism, bp.qsplit > 1): consecutive blocks are the splits of one key block
  const int nsplit = bp.qsplit, sp = (int)(blockIdx.x % (unsigned)nsplit);
  int bh, kb;  // ascending kb = heaviest first under the causal mask
  tile_order((int)(blockIdx.x / (unsigned)nsplit), p.B * p.H, nkb, CAUSAL ? p.order : 0, p.lpt_group, bh, kb);
  const int b = bh / p.H, h = bh % p.H;
  const int k0 = kb * BK;
  const int kw0 = k0 + wave * 32;
  const int krow = kw0 + l32;
  const bool valid_k = krow < p.Nk;

  const S* Qp = (const S*)p.q + b * p.q_sb + h * p.q_sh;
  const S* Kp = (const S*)p.k + b * p.k_sb + h * p.k_sh;
  const S* Vp = (const S*)p.v + b * p.v_sb + h * p.v_sh;
  const S* dOp = (const S*)bp.dout + b * bp.do_sb + h * bp.do_sh;
  // per-query row constants written by the dQ kernel: -lse log2(e) and -delta (dP accumulator start)
  const float* Lp = bp.lrow + ((int64_t)b * p.H + h) * p.Nq;
  const float* Dp = bp.delta + ((int64_t)b * p.H + h) * p.Nq;
  S* dKp = (S*)bp.dk + b * bp.dk_sb + h * bp.dk_sh;
  S* dVp = (S*)bp.dv + b * bp.dv_sb + h * bp.dv_sh;

  // K, V fragments (B operands), resident
  const Rope rope{p.rope_cos, p.rope_sin, D / 2};
  const int64_t* rpos = p.rope_pos ? p.rope_pos + (int64_t)b * p.Nq : nullptr;
  const int64_t kpos = rpos && valid_k ? rpos[krow] : krow;
  constexpr int NKF = F32 ? DP / 8 : DP / 16;
  uint4 kf[NKF], vf[NKF];
#pragma unroll
  for (int i = 0; i < NKF; ++i) {
    const int e = F32 ? (hh * (DP / 2) + 4 * i) : (16 * i + 8 * hh);
    if (valid_k && (DP == D || e < D)) {
      kf[i] = *reinterpret_cast<const uint4*>(Kp + (int64_t)krow * p.k_sn + e);
      if (ROPE == 1) kf[i] = rope_chunk<T>(kf[i], rope, kpos, e, 1.f);
      vf[i] = *reinterpret_cast<const uint4*>(Vp + (int64_t)krow * p.v_sn + e);
    } else {
      kf[i] = vf[i] = make_uint4(0, 0, 0, 0);
    }
  }

  // this block's query tiles [qt_begin, qt_end): the key block's range, or one split of it
  const int qt_first = CAUSAL ? (k0 / BQ) : 0;
  const int qt_last = (p.Nq + BQ - 1) / BQ;
  const int qt_begin = qt_first + (int)((int64_t)(qt_last - qt_first) * sp / nsplit);
  const int qt_end = qt_first + (int)((int64_t)(qt_last - qt_first) * (sp + 1) / nsplit);

  uint4 qst[LPT], dst[LPT];
  RopeCoef qst_rc[ROPE == 1 ? LPT : 1];  // rotation applied at LDS-write time (keeps the prefetch async)
  float lst = 0.f, dlt = 0.f;
  auto gload = [&](int it) {
    const int qbase = it * BQ;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int c = tid + 256 * i;
      const int r = c / CPR, ch = c % CPR;
      const int q = qbase + r;
      if (ROPE == 1) qst_rc[i] = rope_coef<T>(rope, q < p.Nq ? (rpos ? rpos[q] : q) : 0, ch < CREAL ? ch * EPC : 0);
      if (q < p.Nq && (CREAL == CPR || ch < CREAL)) {
        qst[i] = *reinterpret_cast<const uint4*>(Qp + (int64_t)q * p.q_sn + ch * EPC);
        dst[i] = *reinterpret_cast<const uint4*>(dOp + (int64_t)q * bp.do_sn + ch * EPC);
      } else {
        qst[i] = make_uint4(0, 0, 0, 0);
        dst[i] = make_uint4(0, 0, 0, 0);
      }
    }
    if (tid < BQ) {
      const int q = qbase + tid;
      lst = q < p.Nq ? Lp[q] : -INFINITY;  // P = exp2(c2 S - lse log2 e) = 0 past Nq
      dlt = q < p.Nq ? Dp[q] : 0.f;
    }
  };
  auto swrite = [&](int buf) {
    char* base = smem + buf * BUF;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int c = tid + 256 * i;
      const int off = lds_off<RB>(c / CPR, c % CPR);
      *reinterpret_cast<uint4*>(base + off) = ROPE == 1 ? rope_apply<T>(qst[i], qst_rc[i]) : qst[i];
      *reinterpret_cast<uint4*>(base + TILE + off) = dst[i];
    }
    if (tid < BQ) {
      const int pos = DINIT ? row_perm(tid) : tid;
      reinterpret_cast<float*>(base + 2 * TILE)[pos] = lst;
      reinterpret_cast<float*>(base + 2 * TILE + BQ * 4)[pos] = dlt;
    }
  };

  f32x16 dk[NDT], dv[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i) {
    dk[i] = zero16();
    dv[i] = zero16();
  }
  const float c2 = p.scale * kLog2e;

  // one query tile: S, dP, P, dS, dV^T += dO^T P, dK^T += Q^T dS (Qs: the slot's Q image, dO after it).
  // The row constant -delta starts the dP accumulators (DINIT; loaded from the staged rows straight
  // into them) and -lse log2(e) is pre-scaled, so P = exp2(fma(S, c2, L')) and dS = P dP' need no
  // further VALU op; the
  // causal/Nq mask is a separate instantiation taken only on diagonal (or ragged) tiles, so the bulk
  // of the tiles carries no compare/select per element.
  auto tile = [&](int it, const char* Qs, auto mask_tag) __attribute__((always_inline)) {
    constexpr bool MASK = decltype(mask_tag)::value;
    const int qt0 = it * BQ;
    if (CAUSAL && qt0 + BQ - 1 < kw0) return;  // whole tile above this wave's keys
    const char* dOs = Qs + TILE;
    const float* Ls = reinterpret_cast<const float*>(Qs + 2 * TILE);
    const float* Ds = DMA ? Ls + 256 : Ls + BQ;
    f32x16 s[NT], dp[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if constexpr (DINIT) {
        // the rows are staged in accumulator order (row_perm): one 64-B read lands in the
        // registers the dP chain accumulates into
#ifndef CS336_DINIT_F4
        dp[t] = *reinterpret_cast<const f32x16*>(Ds + 32 * t + 16 * hh);
#else
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 D4 = *reinterpret_cast<const float4*>(Ds + 32 * t + 16 * hh + 4 * g);
          dp[t][4 * g] = D4.x; dp[t][4 * g + 1] = D4.y; dp[t][4 * g + 2] = D4.z; dp[t][4 * g + 3] = D4.w;
        }
#endif
      } else {
        dp[t] = zero16();
      }
      s[t] = zero16();
      if constexpr (F32) {
#pragma unroll
        for (int i = 0; i < DP / 8; ++i) {
          const float4 qv = lds_f4<RB>(Qs, 32 * t + l32, hh * (DP / 2) + 4 * i);
          const float4 gv = lds_f4<RB>(dOs, 32 * t + l32, hh * (DP / 2) + 4 * i);
          const float4 kv = __builtin_bit_cast(float4, kf[i]);
          const float4 vv = __builtin_bit_cast(float4, vf[i]);
          s[t] = mma_f32(qv.x, kv.x, s[t]);
          s[t] = mma_f32(qv.y, kv.y, s[t]);
          s[t] = mma_f32(qv.z, kv.z, s[t]);
          s[t] = mma_f32(qv.w, kv.w, s[t]);
          dp[t] = mma_f32(gv.x, vv.x, dp[t]);
          dp[t] = mma_f32(gv.y, vv.y, dp[t]);
          dp[t] = mma_f32(gv.z, vv.z, dp[t]);
          dp[t] = mma_f32(gv.w, vv.w, dp[t]);
        }
      } else {
#pragma unroll
        for (int ks = 0; ks < DP / 16; ++ks) {
          s[t] = Mma16<T>::mma(lds_row_frag<T, RB>(Qs, 32 * t, ks, lane), as_frag<T>(kf[ks]), s[t]);
          dp[t] = Mma16<T>::mma(lds_row_frag<T, RB>(dOs, 32 * t, ks, lane), as_frag<T>(vf[ks]), dp[t]);
        }
      }
    }
    // P = exp2(c2 S - lse log2 e); dS = P (dP - delta); rows (q) are in registers
    {
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int qr = 32 * t + 8 * g + 4 * hh;  // query row of register 4g (+u)
          const int lpos = DINIT ? 32 * t + 16 * hh + 4 * g : qr;  // its staging position
          const float4 L4 = *reinterpret_cast<const float4*>(Ls + lpos);
          const float Lv[4] = {L4.x, L4.y, L4.z, L4.w};
          float Dv[4] = {0.f, 0.f, 0.f, 0.f};
          if constexpr (!DINIT) {
            const float4 D4 = *reinterpret_cast<const float4*>(Ds + qr);
            Dv[0] = D4.x; Dv[1] = D4.y; Dv[2] = D4.z; Dv[3] = D4.w;
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int r = 4 * g + u;
            float pv = fexp2(fmaf(s[t][r], c2, Lv[u]));
            if constexpr (MASK) {
              if ((CAUSAL && krow > qt0 + qr + u) || (DMA && qt0 + qr + u >= p.Nq)) pv = 0.f;
            }
            s[t][r] = pv;
            dp[t][r] = DINIT ? pv * dp[t][r] : pv * (dp[t][r] + Dv[u]);
          }
        }
    }
    if constexpr (F32) {
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int qr = 32 * t + acc_row(r, hh);
            dv[dt] = mma_f32(lds_f1<RB>(dOs, qr, dt * 32 + l32), s[t][r], dv[dt]);
            dk[dt] = mma_f32(lds_f1<RB>(Qs, qr, dt * 32 + l32), dp[t][r], dk[dt]);
          }
    } else {
      typename Mma16<T>::frag pf[NT][2], sf[NT][2];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        pf[t][0] = pack_acc<T>(s[t], 0);
        pf[t][1] = pack_acc<T>(s[t], 1);
        sf[t][0] = pack_acc<T>(dp[t], 0);
        sf[t][1] = pack_acc<T>(dp[t], 1);
      }
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            dv[dt] = Mma16<T>::mma(lds_tr_frag<T, RB>(dOs, 32 * t, s2, dt, lane), pf[t][s2], dv[dt]);
            dk[dt] = Mma16<T>::mma(lds_tr_frag<T, RB>(Qs, 32 * t, s2, dt, lane), sf[t][s2], dk[dt]);
          }
    }
  };

  // Tiles that need the causal mask for some wave (the diagonal ones, qt0 < k0 + BK - 1) and, with
  // LDS-DMA staging, a ragged last tile (rows past Nq are not -inf-padded there) run a masked
  // instantiation of the tile; the bulk runs without the per-element compare/select.
  const int mask_end = CAUSAL ? min(qt_end, max(qt_begin, (k0 + BK - 2) / BQ + 1)) : qt_begin;
  const int ragged = (DMA && p.Nq % BQ != 0 && qt_end == qt_last && qt_end > qt_begin) ? 1 : 0;
  if constexpr (DMA) {
    using Dma = TileDma<BQ, RB, CREAL, ES>;
    Dma qd, dd;
    qd.init(wave, lane, p.q_sn);
    dd.init(wave, lane, bp.do_sn);
    // L / delta: 64 floats = 16 lanes of 16 B; LDS chunk c holds source rows 4 row_perm^-1 chunk
    // (accumulator order, see row_perm) when the tile reads them as whole accumulators
    const int lsrc = DINIT ? row_perm_src_chunk(lane) : lane;
    const uint32_t row_off = lane < 16 ? 16u * lsrc : 0x80000000u;
    if (D != DP || p.Nq % BQ != 0) {  // some slots are read out of range: start from zeros
      lds_zero(smem, NS * SLOT);
      __syncthreads();
    }
    auto issue = [&](int it) {
      char* base = smem + ((it - qt_begin) % NS) * SLOT;
      const int rows = min(BQ, p.Nq - it * BQ);
      qd.issue(Qp + (int64_t)it * BQ * p.q_sn, rows, p.q_sn, base, wave);
      dd.issue(dOp + (int64_t)it * BQ * bp.do_sn, rows, bp.do_sn, base + TILE, wave);
      // every wave loads the same L / delta rows (identical bytes): uniform vmcnt accounting
      const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc((void*)(Lp + it * BQ), (short)0, rows * 4, 0x00020000);
      const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)(Dp + it * BQ), (short)0, rows * 4, 0x00020000);
      dma16(rl, lds_addr(base + 2 * TILE), row_off, 0);
      dma16(rd, lds_addr(base + 2 * TILE + 1024), row_off, 0);
    };
    constexpr int PER_TILE = 2 * Dma::PER_WAVE + 2;
#pragma unroll
    for (int t = 0; t < NS - 1; ++t)
      if (qt_begin + t < qt_end) issue(qt_begin + t);
    // The resident K / V fragments (loaded above) retired, stated to the compiler: it cannot see the
    // inline-asm DMA or the counted asm waits, so without this it keeps them pending and puts
    // vmcnt(0/1) in front of their first MFMA in EVERY tile -- a drain of the prefetch ring per tile.
    // Costs one wait for the prologue's DMA, which the first tile waits for anyway.
    __builtin_amdgcn_s_waitcnt(0x0F70);
    auto dstep = [&](int it, auto slot, auto mask_tag) __attribute__((always_inline)) {
      if (NS == 3 && it + 1 < qt_end) wait_vmcnt<PER_TILE>();
      else wait_vmcnt<0>();
      dma_barrier();
      if (it + NS - 1 < qt_end) issue(it + NS - 1);
      const int B = slot;  // integral_constant (unrolled loop) or runtime slot
      tile(it, smem + B * SLOT, mask_tag);
    };
    auto run = [&](int lo, int hi, auto mask_tag) __attribute__((always_inline)) {
      int it = lo;
      if constexpr (DUNROLL && NS == 3) {  // unrolled by the ring depth: compile-time slots
        while (it < hi && (it - qt_begin) % 3 != 0) {
          dstep(it, (it - qt_begin) % 3, mask_tag);
          ++it;
        }
        for (; it + 2 < hi; it += 3) {
          dstep(it, std::integral_constant<int, 0>{}, mask_tag);
          dstep(it + 1, std::integral_constant<int, 1>{}, mask_tag);
          dstep(it + 2, std::integral_constant<int, 2>{}, mask_tag);
        }
      } else if constexpr (DUNROLL && NS == 2) {
        if (it < hi && ((it - qt_begin) & 1)) {
          dstep(it, 1, mask_tag);
          ++it;
        }
        for (; it + 1 < hi; it += 2) {
          dstep(it, std::integral_constant<int, 0>{}, mask_tag);
          dstep(it + 1, std::integral_constant<int, 1>{}, mask_tag);
        }
      }
      for (; it < hi; ++it) dstep(it, (it - qt_begin) % NS, mask_tag);
    };
    if constexpr (CAUSAL) run(qt_begin, mask_end, std::true_type{});
    run(mask_end, qt_end - ragged, std::false_type{});
    run(max(mask_end, qt_end - ragged), qt_end, std::true_type{});
  } else {
    if (qt_begin < qt_end) {
      gload(qt_begin);
      swrite(0);
    }
    __syncthreads();
    // one iteration with a compile-time slot (B): the slot's LDS addresses become immediates
    auto step = [&](int it, auto slot, auto mask_tag) __attribute__((always_inline)) {
      const int B = slot;  // integral_constant (unrolled loop) or runtime slot
      if (PREFETCH && it + 1 < qt_end) gload(it + 1);
      tile(it, smem + B * BUF, mask_tag);
      if (it + 1 < qt_end) {
        if (PREFETCH) {
          swrite(B ^ 1);
        } else {
          __syncthreads();
          gload(it + 1);
          swrite(0);
        }
      }
      __syncthreads();
    };
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, PREFETCH ? 1 : 0>;
    auto run = [&](int lo, int hi, auto mask_tag) __attribute__((always_inline)) {
      int it = lo;
      if constexpr (UNROLL2) {
        if (PREFETCH && it < hi && ((it - qt_begin) & 1)) step(it++, S1{}, mask_tag);  // even slot next
        for (; it + 1 < hi; it += 2) {  // unrolled by two: slot 0, slot 1
          step(it, S0{}, mask_tag);
          step(it + 1, S1{}, mask_tag);
        }
      }
      for (; it < hi; ++it) step(it, PREFETCH ? ((it - qt_begin) & 1) : 0, mask_tag);
    };
    if constexpr (CAUSAL) run(qt_begin, mask_end, std::true_type{});
    run(mask_end, qt_end, std::false_type{});
  }

  if (nsplit > 1) {  // unscaled fp32 partials of this query range (summed by fa_bwd_reduce_kernel)
    if (valid_k) {
      const int64_t prow = (((int64_t)sp * p.B * p.H + bh) * p.Nk + krow) * D;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int d = dt * 32 + 8 * g + 4 * hh;
          if (DP != D && d >= D) continue;
          *reinterpret_cast<float4*>(bp.dk_part + prow + d) =
              make_float4(dk[dt][4 * g], dk[dt][4 * g + 1], dk[dt][4 * g + 2], dk[dt][4 * g + 3]);
          *reinterpret_cast<float4*>(bp.dv_part + prow + d) =
              make_float4(dv[dt][4 * g], dv[dt][4 * g + 1], dv[dt][4 * g + 2], dv[dt][4 * g + 3]);
        }
    }
    return;
  }
  if (valid_k) {
    S* krow_dk = dKp + (int64_t)krow * bp.dk_sn;
    S* krow_dv = dVp + (int64_t)krow * bp.dv_sn;
    const float sc = p.scale;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = dt * 32 + 8 * g + 4 * hh;
        if (DP != D && d >= D) continue;
        float v0 = dk[dt][4 * g] * sc, v1 = dk[dt][4 * g + 1] * sc, v2 = dk[dt][4 * g + 2] * sc,
              v3 = dk[dt][4 * g + 3] * sc;
        if (ROPE != 0) rope_inv4(v0, v1, v2, v3, rope, kpos, d);  // dK w.r.t. the un-rotated k
        store4<T>(krow_dk + d, make_float4(v0, v1, v2, v3));
        store4<T>(krow_dv + d, make_float4(dv[dt][4 * g], dv[dt][4 * g + 1], dv[dt][4 * g + 2], dv[dt][4 * g + 3]));
      }
  }
}

// Explicit instantiation of the LDS-DMA variants (hipcc referenced some implicit ones from the launch
// chain without emitting their host stubs; see fa_fwd.hip)
#define CS336_FA_BWD_DMA(T, D)                                                                  \
  template __global__ void fa_bwd_dq_kernel<T, D, false, false, true>(const AttnBwdParams);   \
  template __global__ void fa_bwd_dq_kernel<T, D, true, false, true>(const AttnBwdParams);    \
  template __global__ void fa_bwd_dkdv_kernel<T, D, false, false, true>(const AttnBwdParams); \
  template __global__ void fa_bwd_dkdv_kernel<T, D, true, false, true>(const AttnBwdParams);
CS336_FA_BWD_DMA(BF16, 32)
CS336_FA_BWD_DMA(BF16, 64)
CS336_FA_BWD_DMA(BF16, 80)
CS336_FA_BWD_DMA(BF16, 128)
CS336_FA_BWD_DMA(F16, 32)
CS336_FA_BWD_DMA(F16, 64)
CS336_FA_BWD_DMA(F16, 80)
CS336_FA_BWD_DMA(F16, 128)
#undef CS336_FA_BWD_DMA

// One split-partial reduction: `ns` unscaled fp32 partials ([split][B·H][N][D]) -> out (B, H, N, D
// strided) = scale · sum, rotated back by RoPE when rcos (dQ/dK w.r.t. the un-rotated q/k)
struct SplitSum {
  const float* part;
  int ns, N;
  void* out;
  int64_t sb, sh, sn;
  float scale;
  const float* rcos;
  const float* rsin;
  const int64_t* rpos;
  int64_t units;  // B·H·N·D/4 (0: nothing to reduce)
};

// dQ, dK and dV split sums in ONE launch (three launches cost ~4 us each at the B 1 H 1 sizes the
// split serves); one thread per 4 d, partials summed in split order. An in-launch form (the dK/dV
// kernel summing dQ, its last-arriving split summing dK/dV) measured 1.3-2.7x slower: one workgroup
// at 1-2 waves per SIMD reads a key block's slabs serially (scripts/experiments.md)
template <typename T, int D>
__global__ __launch_bounds__(256) void fa_bwd_reduce_kernel(const SplitSum s0, const SplitSum s1, const SplitSum s2, int H) {
  typedef typename Elem<T>::storage S;
  constexpr int Q4 = D / 4;
  int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  SplitSum a = s0;  // (a copy, not a pointer into the kernel arguments: that would go to scratch)
  if (gid >= s0.units) {
    gid -= s0.units;
    a = s1;
    if (gid >= s1.units) {
      gid -= s1.units;
      a = s2;
      if (gid >= s2.units) return;
    }
  }
  const int64_t rows = a.units / Q4;
  const int64_t row = gid / Q4;
  const int d = 4 * (int)(gid % Q4);
  float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;
  for (int s = 0; s < a.ns; ++s) {
    const float4 x = *reinterpret_cast<const float4*>(a.part + (s * rows + row) * D + d);
    v0 += x.x; v1 += x.y; v2 += x.z; v3 += x.w;
  }
  v0 *= a.scale; v1 *= a.scale; v2 *= a.scale; v3 *= a.scale;
  const int bh = (int)(row / a.N), n = (int)(row % a.N), b = bh / H, h = bh % H;
  if (a.rcos != nullptr) {
    const Rope rope{a.rcos, a.rsin, D / 2};
    rope_inv4(v0, v1, v2, v3, rope, a.rpos ? a.rpos[(int64_t)b * a.N + n] : n, d);
  }
  store4<T>((S*)a.out + b * a.sb + h * a.sh + (int64_t)n * a.sn + d, make_float4(v0, v1, v2, v3));
}

template <typename T, int D, bool C, int R, bool DMA>
void launch_bwd_v(const AttnBwdParams& bp, hipStream_t s, dim3 gq, dim3 gk, dim3 block) {
  // (a two-stream form -- dK/dV beside dQ after a delta prep kernel -- measured slower:
  // profiles/r4_fa_conc.md; removed in round 5)
  hipLaunchKernelGGL((fa_bwd_dq_kernel<T, D, C, R, DMA>), gq, block, 0, s, bp);
  hipLaunchKernelGGL((fa_bwd_dkdv_kernel<T, D, C, R, DMA>), gk, block, 0, s, bp);
  const AttnParams& p = bp.f;
  if (bp.ksplit == 1 && bp.qsplit == 1) return;
  const float* rc = R != 0 ? p.rope_cos : nullptr;
  const int64_t q4 = bp.ksplit > 1 ? (int64_t)p.B * p.H * p.Nq * (D / 4) : 0;
  const int64_t k4 = bp.qsplit > 1 ? (int64_t)p.B * p.H * p.Nk * (D / 4) : 0;
  const SplitSum sq{bp.dq_part, bp.ksplit, p.Nq, bp.dq, bp.dq_sb, bp.dq_sh, bp.dq_sn, p.scale, rc, p.rope_sin, p.rope_pos, q4};
  const SplitSum sk{bp.dk_part, bp.qsplit, p.Nk, bp.dk, bp.dk_sb, bp.dk_sh, bp.dk_sn, p.scale, rc, p.rope_sin, p.rope_pos, k4};
  const SplitSum sv{bp.dv_part, bp.qsplit, p.Nk, bp.dv, bp.dv_sb, bp.dv_sh, bp.dv_sn, 1.f, nullptr, nullptr, nullptr, k4};
  hipLaunchKernelGGL((fa_bwd_reduce_kernel<T, D>), dim3((unsigned)((q4 + 2 * k4 + 255) / 256)), block, 0, s, sq, sk, sv, p.H);
}

template <typename T, int D, bool C>
void launch_bwd_c(const AttnBwdParams& bp, hipStream_t s, dim3 gq, dim3 gk, dim3 block) {
  if (bp.f.rope_cos != nullptr && bp.f.rope_out_only) {
    // q/k were rotated by the forward's RoPE pass: only dQ/dK are rotated back, at their store
    launch_bwd_v<T, D, C, 2, false>(bp, s, gq, gk, block);
  } else if (bp.f.rope_cos != nullptr) {
    launch_bwd_v<T, D, C, 1, false>(bp, s, gq, gk, block);
  } else if constexpr (!std::is_same<T, float>::value) {
    if (bp.f.dma & 2) launch_bwd_v<T, D, C, 0, true>(bp, s, gq, gk, block);
    else launch_bwd_v<T, D, C, false, false>(bp, s, gq, gk, block);
  } else {
    launch_bwd_v<T, D, C, false, false>(bp, s, gq, gk, block);
  }
}

template <typename T, int D>
void launch_bwd(const AttnBwdParams& bp, hipStream_t s) {
  const AttnParams& p = bp.f;
  const int nqb = (p.Nq + 127) / 128;
  const int nkb = (p.Nk + 127) / 128;
  const dim3 gq((unsigned)(nqb * p.B * p.H * bp.ksplit)), gk((unsigned)(nkb * p.B * p.H * bp.qsplit)), block(256);
  if (p.causal) launch_bwd_c<T, D, true>(bp, s, gq, gk, block);
  else launch_bwd_c<T, D, false>(bp, s, gq, gk, block);
}

template <typename T>
void launch_bwd_d(const AttnBwdParams& bp, hipStream_t s) {
  switch (bp.f.D) {
    case 16:  // computed as 32 inside the kernel (d 16..31 zero in LDS, never loaded or stored): no host padding copies
      if constexpr (std::is_same<T, float>::value) {
        fprintf(stderr, "fa_bwd: head dim 16 is 16-bit only\n");
        abort();
      } else {
        launch_bwd<T, 16>(bp, s);
      }
      break;
    case 32: launch_bwd<T, 32>(bp, s); break;
    case 64: launch_bwd<T, 64>(bp, s); break;
    case 80:
      if constexpr (std::is_same<T, float>::value) {
        fprintf(stderr, "fa_bwd: head dim 80 is 16-bit only\n");
        abort();
      } else {
        launch_bwd<T, 80>(bp, s);
      }
      break;
    case 128: launch_bwd<T, 128>(bp, s); break;
    default: fprintf(stderr, "fa_bwd: unsupported head dim %d\n", bp.f.D); abort();
  }
}

}  // namespace fa

// Low parallelism (the reference sweep's B 1, H 1: N/128 query blocks and key blocks on 256 CUs):
// split the dQ kernel's keys and the dK/dV kernel's queries until each kernel has ~512 workgroups,
// each split keeping at least 4 tiles of its loop.
void flash_attn_bwd_splits(const AttnBwdParams& bp, int& ksplit, int& qsplit) {
  const AttnParams& p = bp.f;
  ksplit = qsplit = 1;
  if (p.B * p.H == 0 || p.D % 4) return;
  const int64_t bh = (int64_t)p.B * p.H;
  const int64_t nqb = (p.Nq + 127) / 128, nkb = (p.Nk + 127) / 128;
  if (nqb * bh < 256) ksplit = (int)std::max<int64_t>(1, std::min<int64_t>({(512 + nqb * bh - 1) / (nqb * bh), (p.Nk / 32) / 4, 16}));
  if (nkb * bh < 256) qsplit = (int)std::max<int64_t>(1, std::min<int64_t>({(512 + nkb * bh - 1) / (nkb * bh), (p.Nq / 32) / 4, 16}));
}

size_t flash_attn_bwd_split_workspace(const AttnBwdParams& bp, int ksplit, int qsplit) {
  const AttnParams& p = bp.f;
  const size_t bh = (size_t)p.B * p.H;
  return (ksplit > 1 ? ksplit * bh * p.Nq * p.D : 0) + (qsplit > 1 ? 2 * qsplit * bh * p.Nk * p.D : 0);
}

void flash_attn_bwd(const AttnBwdParams& bp, DType t, hipStream_t s) {
  if (bp.f.B * bp.f.H == 0 || bp.f.Nq == 0 || bp.f.Nk == 0) return;
  switch (t) {
    case DType::BF16: fa::launch_bwd_d<BF16>(bp, s); break;
    case DType::F16: fa::launch_bwd_d<F16>(bp, s); break;
    case DType::F32: fa::launch_bwd_d<float>(bp, s); break;
  }
}

}  // namespace cs336
