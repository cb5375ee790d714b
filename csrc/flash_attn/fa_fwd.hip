// FlashAttention-2 forward for MI355X (gfx950 / CDNA4).
//
// Parity: reference cs336_systems/flash_attention.py:137-266 (Triton kernel, 16x16 tiles) and the
// handout's Algorithm 1. Design here is CDNA4-first:
//   * workgroup = 4 waves = 128 query rows (32 per wave, one query row per MFMA lane column);
//     grid = (query blocks) x (batch*heads), 1-D with an XCD-aware remap so one head's blocks
//     share an L2, causal blocks dispatched heaviest-first;
//   * K/V tiles of 64 keys are staged global -> registers -> swizzled LDS, double-buffered with
//     the next tile's global loads issued before the current tile's MFMAs (T14 split);
//   * S^T = K Q^T on v_mfma_f32_32x32x16_{bf16,f16} (exact v_mfma_f32_32x32x2_f32 for fp32),
//     online softmax in registers with exp2 and the scale folded into one FMA, P^T packed from the
//     accumulator straight into the PV MFMA's B operand, V^T gathered by ds_read_b64_tr_b16;
//   * causal: tiles above the diagonal are never loaded (kv_end = q0 + 128), waves skip tiles
//     entirely above their rows, and only tiles straddling the diagonal pay the mask.
// Output O keeps the input dtype and is written through arbitrary (batch, head, seq) strides;
// LSE (natural log, fp32, (B,H,Nq)) is the single extra tensor the backward needs.
#include "fa_common.h"

#include <algorithm>

namespace cs336 {
namespace fa {

// 16-bit variants ask for two workgroups per CU (<= 256 VGPRs): without the hint the LDS-DMA variant
// at d 128 took 260 registers, ran one workgroup per CU and lost 37 % (causal, N 4096)
// The pipelined variant (DMA 2) holds two S^T tiles: one workgroup per CU except at d 64 without
// the causal mask, where two still fit 256 VGPRs (measured spills otherwise: 72-148 B/lane).
template <typename T, int D, bool CAUSAL = false, int DMA = 0>
constexpr int fwd_min_waves() {
#ifdef CS336_FA_FWD_WAVES64
  if (D <= 64 && !std::is_same<T, float>::value) return CS336_FA_FWD_WAVES64;
#endif
  if (DMA == 2) return (D <= 64 && !CAUSAL) ? 2 : 1;
  // d <= 64 causal with VGPR staging: three workgroups per CU (168 VGPRs, no spill): +11-12 % at
  // N 512 and 4096 (profiles/r2_fa_fwd_waves.md); the other d-64 variants would spill at 168
  if (D <= 64 && CAUSAL && DMA == 0 && !std::is_same<T, float>::value) return 3;
  return std::is_same<T, float>::value ? 1 : 2;
}

// the PV loop's prefetched V^T fragment type (16-bit only; a placeholder for fp32)
template <typename T, bool ON>
struct VFrag {
  typedef int type;
};
template <typename T>
struct VFrag<T, true> {
  typedef typename Mma16<T>::frag type;
};

// DMA: 0 = VGPR staging, 1 = LDS-DMA ring of K|V tiles, 2 = LDS-DMA into separate K and V rings
// with the next tile's S^T MFMAs issued inside the current tile's softmax (software pipeline)
template <typename T, int D, bool CAUSAL, bool ROPE, int DMA>
__global__ __launch_bounds__(256, (fwd_min_waves<T, D, CAUSAL, DMA>())) void fa_fwd_kernel(const AttnParams p) {
  typedef typename Elem<T>::storage S;
  constexpr bool F32 = std::is_same<T, float>::value;
  constexpr int ES = sizeof(S);
  constexpr int DP = PadD<D>::value;  // compute width (80 -> 96; d >= D is zero, never loaded/stored)
  constexpr int RB = DP * ES;      // bytes per LDS row
  constexpr int CPR = RB / 16;     // 16-byte chunks per row
  constexpr int CREAL = D * ES / 16;  // chunks that hold real data
  constexpr int EPC = 16 / ES;     // elements per chunk
  constexpr int BM = 128, BN = 64;
  constexpr int TILE = BN * RB;
  constexpr int LPT = BN * CPR / 256;  // 16-B staging loads per thread per tile
  static_assert(BN * CPR % 256 == 0, "staging rounds must be whole");
  constexpr int NDT = DP / 32;         // 32-wide d tiles of O^T
  constexpr bool PREFETCH = !(F32 && D == 128);
  static_assert(!DMA || (!F32 && !ROPE), "LDS-DMA staging: 16-bit, no RoPE-on-load");
  // LDS-DMA ring depth: 3 K/V stages (two tiles in flight) up to 96-wide rows, 2 at d 128
  // (DMA 2: NS slots in each of the K and V rings, the same bytes)
  constexpr int NS = DMA ? (DP <= 96 ? 3 : 2) : 2;

  __shared__ __attribute__((aligned(1024))) char smem[NS * 2 * TILE];

  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  const int l32 = lane & 31, hh = lane >> 5;

  const int nqb = (p.Nq + BM - 1) / BM;
  // split-KV (p.kv_splits > 1, low parallelism): consecutive blocks are the key splits of one query block
  const int nsplit = p.kv_splits, sp = (int)(blockIdx.x % (unsigned)nsplit);
  int bh, qb;
  tile_order((int)(blockIdx.x / (unsigned)nsplit), p.B * p.H, nqb, CAUSAL ? p.order : 0, p.lpt_group, bh, qb);
  if (CAUSAL) qb = nqb - 1 - qb;
  const int b = bh / p.H, h = bh % p.H;
  const int q0 = qb * BM;

  const S* Qp = (const S*)p.q + b * p.q_sb + h * p.q_sh;
  const S* Kp = (const S*)p.k + b * p.k_sb + h * p.k_sh;
  const S* Vp = (const S*)p.v + b * p.v_sb + h * p.v_sh;
  S* Op = (S*)p.o + b * p.o_sb + h * p.o_sh;

  const int qw0 = q0 + wave * 32;
  const int qrow = qw0 + l32;
  const bool valid_q = qrow < p.Nq;

  // ---- Q fragments (B operand), resident for the whole kernel -------------------------------
  constexpr int NQF = F32 ? DP / 8 : DP / 16;  // uint4 per lane
  // 16-bit S = K Qᵀ reduces over the real d only: the 16-wide k-steps past D hold the zero pad
  // (d 80: 5 of the 6 steps of the padded 96, d 16: 1 of 2)
  constexpr int NKR = (D + 15) / 16;
  const Rope rope{p.rope_cos, p.rope_sin, D / 2};
  const int64_t* rpos = p.rope_pos ? p.rope_pos + (int64_t)b * p.Nq : nullptr;
  uint4 qf[NQF];
#pragma unroll
  for (int i = 0; i < NQF; ++i) {
    // 16-bit: chunk 2*ks + hh  |  f32: d = hh*D/2 + 4*i .. +3
    const int e = F32 ? (hh * (DP / 2) + 4 * i) : (16 * i + 8 * hh);
    const bool in = valid_q && e < D;
    qf[i] = in ? *reinterpret_cast<const uint4*>(Qp + (int64_t)qrow * p.q_sn + e) : make_uint4(0, 0, 0, 0);
    if (ROPE && in) qf[i] = rope_chunk<T>(qf[i], rope, rpos ? rpos[qrow] : qrow, e, 1.f);
  }

  const int kv_end = CAUSAL ? min(p.Nk, q0 + BM) : p.Nk;
  // this block's key tiles: [jt0, jt0 + ntiles) of the query block's range (all of it unless split);
  // tile indices j below are relative to jt0
  const int ntiles_all = (kv_end + BN - 1) / BN;
  const int jt0 = (int)((int64_t)ntiles_all * sp / nsplit);
  const int ntiles = (int)((int64_t)ntiles_all * (sp + 1) / nsplit) - jt0;

  uint4 kst[LPT], vst[LPT];
  RopeCoef kst_rc[ROPE ? LPT : 1];  // rotation applied at LDS-write time (keeps the prefetch async)
  auto gload = [&](int j) {
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int c = tid + 256 * i;
      const int r = c / CPR, ch = c % CPR;
      const int key = (jt0 + j) * BN + r;
      if (ROPE) kst_rc[i] = rope_coef<T>(rope, key < p.Nk ? (rpos ? rpos[key] : key) : 0, ch < CREAL ? ch * EPC : 0);
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
      const int r = c / CPR, ch = c % CPR;
      const int off = lds_off<RB>(r, ch);
      *reinterpret_cast<uint4*>(Ks + off) = ROPE ? rope_apply<T>(kst[i], kst_rc[i]) : kst[i];
      *reinterpret_cast<uint4*>(Ks + TILE + off) = vst[i];
    }
  };

  float m = kNegBig, l = 0.f;
  f32x16 o[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i) o[i] = zero16();
  const float c2 = p.scale * kLog2e;

  // one K/V tile's work, in two parts so the pipelined loop can put the NEXT tile's S^T MFMAs
  // between this tile's softmax VALU work: s_tile = S^T = K Q^T (Ks: the tile's K image);
  // finish = mask, online softmax, O^T += V^T P^T (Vs: the tile's V image), with `mid` issued after
  // the rescale branch, in the same basic block as the exp2 loop and the PV MFMAs
  auto active = [&](int j) { return !CAUSAL || (jt0 + j) * BN <= qw0 + 31; };
  auto s_tile = [&](const char* Ks, f32x16 (&s)[2]) {
    // ---- S^T = K Q^T ----
    if constexpr (!F32 && DP <= 64) {
      // every K fragment of the tile read before the first MFMA (<= 32 VGPRs): the MFMA chain then
      // waits on one LDS round trip instead of one per fragment
      typename Mma16<T>::frag kf[2][NKR];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int ks = 0; ks < NKR; ++ks) kf[t][ks] = lds_row_frag<T, RB>(Ks, 32 * t, ks, lane);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        s[t] = zero16();
#pragma unroll
        for (int ks = 0; ks < NKR; ++ks) s[t] = Mma16<T>::mma(kf[t][ks], as_frag<T>(qf[ks]), s[t]);
      }
      return;
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      s[t] = zero16();
      if constexpr (F32) {
#pragma unroll
        for (int i = 0; i < DP / 8; ++i) {
          const float4 kv = lds_f4<RB>(Ks, 32 * t + l32, hh * (DP / 2) + 4 * i);
          const float4 qv = __builtin_bit_cast(float4, qf[i]);
          s[t] = mma_f32(kv.x, qv.x, s[t]);
          s[t] = mma_f32(kv.y, qv.y, s[t]);
          s[t] = mma_f32(kv.z, qv.z, s[t]);
          s[t] = mma_f32(kv.w, qv.w, s[t]);
        }
      } else {
#pragma unroll
        for (int ks = 0; ks < NKR; ++ks)
          s[t] = Mma16<T>::mma(lds_row_frag<T, RB>(Ks, 32 * t, ks, lane), as_frag<T>(qf[ks]), s[t]);
      }
    }
  };
  auto finish = [&](int j, const char* Vs, f32x16 (&s)[2], auto&& mid) {
    const int kt0 = (jt0 + j) * BN;
    // ---- mask (bounds / causal diagonal) ----
    const bool need_mask = (kt0 + BN > p.Nk) || (CAUSAL && kt0 + BN - 1 > qw0);
    if (need_mask) {
      // key = kt0 + 32t + acc_row(r, hh) is masked iff it exceeds min(Nk - 1, qrow): one compare of
      // a constant against a per-lane limit per element
      const int lim = (CAUSAL ? min(p.Nk - 1, qrow) : p.Nk - 1) - kt0 - 4 * hh;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (32 * t + acc_row(r, 0) > lim) s[t][r] = -INFINITY;
    }
    // ---- online softmax (query on the lane), deferred rescale (T13) ----
    float mx = s[0][0];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[t][r]);
    mx = xhalf_max(mx);
    const float mt = mx * c2;
    if (__ballot(mt > m + kRescaleThr) != 0) {  // wave-uniform
      const float m_new = fmaxf(m, mt);
      const float alpha = fexp2(m - m_new);
      l *= alpha;
      m = m_new;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
    }
    mid();
    // 16-bit causal LDS-DMA kernel, d <= 64: the tile's V^T fragments (<= 32 VGPRs) are requested
    // before the exp2 loop, so their LDS round trip runs under it instead of in front of every PV
    // MFMA: +9 % at N 4096 d 64 (707 -> 771 TF), +1.5 % at the XL step's N 512 (profiles/r5_fa_fwd.md).
    // Not without the mask: there the extra registers (163 -> 187) cost a wave per SIMD (-4 %)
    constexpr bool VPRE = !F32 && DP <= 64 && DMA == 1 && CAUSAL;
    typename VFrag<T, VPRE>::type vf[VPRE ? NDT : 1][2][2];
    if constexpr (VPRE) {
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) vf[dt][t][s2] = lds_tr_frag<T, RB>(Vs, 32 * t, s2, dt, lane);
      __builtin_amdgcn_sched_barrier(0);  // keep the reads here (the scheduler sinks them to their MFMAs)
    }
    float rs = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float pv = fexp2(fmaf(s[t][r], c2, -m));
        s[t][r] = pv;
        rs += pv;
      }
    l += rs;
    // ---- O^T += V^T P^T ----
    if constexpr (F32) {
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            o[dt] = mma_f32(lds_f1<RB>(Vs, 32 * t + acc_row(r, hh), dt * 32 + l32), s[t][r], o[dt]);
    } else {
      typename Mma16<T>::frag pf[2][2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        pf[t][0] = pack_acc<T>(s[t], 0);
        pf[t][1] = pack_acc<T>(s[t], 1);
      }
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2)
            if constexpr (VPRE) o[dt] = Mma16<T>::mma(vf[dt][t][s2], pf[t][s2], o[dt]);
            else o[dt] = Mma16<T>::mma(lds_tr_frag<T, RB>(Vs, 32 * t, s2, dt, lane), pf[t][s2], o[dt]);
    }
  };
  auto tile = [&](int j, const char* Ks) __attribute__((always_inline)) {
    if (active(j)) {
      f32x16 s[2];
      s_tile(Ks, s);
      finish(j, Ks + TILE, s, [] {});
    }
  };

  if constexpr (DMA == 2) {
    // Separate K and V rings of NS slots each (K ring at smem, V ring after it). Iteration j needs
    // K(j+1) (for the next S^T) and V(j) (for this PV); it then refills the slots freed by the
    // previous iteration: V(j+NS-1) and K(j+NS). Groups past the last tile are still issued (an
    // empty buffer range: the loads return zeros) so every wait below is one static count: after
    // K(j+1) and V(j), exactly 2*NS-4 younger groups of this wave are in flight.
    using Dma = TileDma<BN, RB, CREAL, ES>;
    constexpr int PW = Dma::PER_WAVE;
    Dma kd, vd;
    kd.init(wave, lane, p.k_sn);
    vd.init(wave, lane, p.v_sn);
    char* Kr = smem;
    char* Vr = smem + NS * TILE;
    if (D != DP || p.Nk % BN != 0) {
      lds_zero(smem, NS * 2 * TILE);
      __syncthreads();
    }
    auto issue_k = [&](int j) {
      const int rows = min(BN, p.Nk - (jt0 + j) * BN);
      kd.issue(Kp + (int64_t)(jt0 + j) * BN * p.k_sn, rows, p.k_sn, Kr + (j % NS) * TILE, wave);
    };
    auto issue_v = [&](int j) {
      const int rows = min(BN, p.Nk - (jt0 + j) * BN);
      vd.issue(Vp + (int64_t)(jt0 + j) * BN * p.v_sn, rows, p.v_sn, Vr + (j % NS) * TILE, wave);
    };
    // prologue: K(0), V(0), K(1), V(1), ..., K(NS-2), V(NS-2), K(NS-1)
#pragma unroll
    for (int t = 0; t < NS - 1; ++t) {
      issue_k(t);
      issue_v(t);
    }
    issue_k(NS - 1);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // resident Q retired, stated to the compiler (see above)
    wait_vmcnt<(2 * NS - 2) * PW>();  // K(0) landed
    dma_barrier();
    f32x16 sa[2], sb[2];
    if (active(0)) s_tile(Kr, sa);
    // one iteration: publish K(j+1), V(j); refill; finish tile j with S^T(j+1) inside its softmax
    auto body = [&](int j, f32x16 (&cur)[2], f32x16 (&nxt)[2]) {
      wait_vmcnt<(2 * NS - 4) * PW>();
      dma_barrier();
      issue_v(j + NS - 1);
      issue_k(j + NS);
      if (active(j)) finish(j, Vr + (j % NS) * TILE, cur, [&] { s_tile(Kr + ((j + 1) % NS) * TILE, nxt); });
    };
    auto last = [&](int j, f32x16 (&cur)[2]) {
      wait_vmcnt<0>();  // V(j) (and the trailing empty groups)
      dma_barrier();
      if (active(j)) finish(j, Vr + (j % NS) * TILE, cur, [] {});
    };
    int j = 0;
    for (; j + 2 < ntiles; j += 2) {  // unrolled by two: sa/sb swap roles with static names
      body(j, sa, sb);
      body(j + 1, sb, sa);
    }
    if (j + 1 < ntiles) {
      body(j, sa, sb);
      last(j + 1, sb);
    } else if (j < ntiles) {
      last(j, sa);
    }
  } else if constexpr (DMA) {
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
    // the resident Q fragments retired, stated to the compiler, which cannot see the inline-asm DMA
    // or the counted asm waits (else it re-waits vmcnt(0) before their MFMAs in every tile)
    __builtin_amdgcn_s_waitcnt(0x0F70);
    auto step = [&](int j, auto slot) __attribute__((always_inline)) {
      // this wave's pieces of tile j have landed once only the younger tiles' DMAs are in flight;
      // the barrier then publishes every wave's pieces and retires all reads of tile j-1's slot
      if (NS == 3 && j + 1 < ntiles) wait_vmcnt<2 * Dma::PER_WAVE>();
      else wait_vmcnt<0>();
      dma_barrier();
      if (j + NS - 1 < ntiles) issue(j + NS - 1);
      const int B = slot;  // integral_constant (unrolled loop) or runtime slot
      tile(j, smem + B * 2 * TILE);
    };
    int j = 0;
#ifndef CS336_FA_FWD_NO_UNROLL
    // unrolled by the ring depth with compile-time slots: the slots' LDS addresses become immediates
    if constexpr (NS == 3) {
      for (; j + 2 < ntiles; j += 3) {
        step(j, std::integral_constant<int, 0>{});
        step(j + 1, std::integral_constant<int, 1>{});
        step(j + 2, std::integral_constant<int, 2>{});
      }
    } else if constexpr (NS == 2) {
      for (; j + 1 < ntiles; j += 2) {
        step(j, std::integral_constant<int, 0>{});
        step(j + 1, std::integral_constant<int, 1>{});
      }
    }
#endif
    for (; j < ntiles; ++j) step(j, j % NS);
  } else {
    if (ntiles > 0) {
      gload(0);
      swrite(0);
    }
    __syncthreads();
    for (int j = 0; j < ntiles; ++j) {
      const int buf = PREFETCH ? (j & 1) : 0;
      if (PREFETCH && j + 1 < ntiles) gload(j + 1);
      tile(j, smem + buf * 2 * TILE);
      if (j + 1 < ntiles) {
        if (PREFETCH) {
          swrite(buf ^ 1);
        } else {
          __syncthreads();
          gload(j + 1);
          swrite(0);
        }
      }
      __syncthreads();
    }
  }

  // ---- epilogue ----
  // (an empty key split of the DMA-2 ring issued its prologue and never reached the draining `last`)
  if constexpr (DMA == 2) wait_vmcnt<0>();
  l = xhalf_sum(l);
  const float inv = l > 0.f ? 1.f / l : 0.f;
  if (nsplit > 1) {
    // split-KV partial: normalized fp32 O of this key range and its natural-log LSE (merge kernel)
    if (valid_q) {
      const int64_t prow = ((int64_t)sp * p.B * p.H + bh) * p.Nq + qrow;
      float* orow = p.opart + prow * D;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int d = dt * 32 + 8 * g + 4 * hh;
          if (DP == D || d < D)
            *reinterpret_cast<float4*>(orow + d) =
                make_float4(o[dt][4 * g] * inv, o[dt][4 * g + 1] * inv, o[dt][4 * g + 2] * inv, o[dt][4 * g + 3] * inv);
        }
      if (hh == 0) p.lpart[prow] = l > 0.f ? (m + __log2f(l)) * kLn2 : -INFINITY;
    }
    return;
  }
  if (valid_q) {
    S* orow = Op + (int64_t)qrow * p.o_sn;
    // 16-bit O with 16-B aligned rows (T21): lane half hh holds d 8g+4hh .. +3 of its row per register
    // group g; one v_permlane32_swap per dword pairs groups (g, g+1), after which lanes 0-31 hold d
    // 8g .. 8g+7 and lanes 32-63 d 8g+8 .. 8g+15 of the same row: one 16-B store where there were two
    // 8-B stores (the per-block store tail is issue-bound)
    bool wide = false;
    if constexpr (!F32) wide = ((p.o_sn | p.o_sb | p.o_sh) & 7) == 0 && ((uintptr_t)p.o & 15) == 0;
    if constexpr (!F32) if (wide) {
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int g = 0; g < 4; g += 2) {
          uint32_t c[4];
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            const int r0 = 4 * g + 2 * k;
            const uint32_t lo = (uint32_t)Elem<T>::from_f(o[dt][r0] * inv) | ((uint32_t)Elem<T>::from_f(o[dt][r0 + 1] * inv) << 16);
            const uint32_t hi = (uint32_t)Elem<T>::from_f(o[dt][r0 + 4] * inv) | ((uint32_t)Elem<T>::from_f(o[dt][r0 + 5] * inv) << 16);
            const auto sw = __builtin_amdgcn_permlane32_swap(lo, hi, false, false);
            c[k] = sw[0];
            c[2 + k] = sw[1];
          }
          const int d = dt * 32 + 8 * g + 8 * hh;
          if (DP == D || d < D) *reinterpret_cast<uint4*>(orow + d) = make_uint4(c[0], c[1], c[2], c[3]);
        }
    }
    if (!wide) {
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int d = dt * 32 + 8 * g + 4 * hh;
          if (DP == D || d < D)
            store4<T>(orow + d, make_float4(o[dt][4 * g] * inv, o[dt][4 * g + 1] * inv, o[dt][4 * g + 2] * inv,
                                            o[dt][4 * g + 3] * inv));
        }
    }

    if (hh == 0) p.lse[((int64_t)b * p.H + h) * p.Nq + qrow] = l > 0.f ? (m + __log2f(l)) * kLn2 : -INFINITY;
  }
  if constexpr (!F32) {
    if (p.ot != nullptr) {
      // Oᵀ (d-major, queries contiguous) through an LDS transpose: each lane parks its 16-bit outputs at
      // [d][q] (32 lanes = 32 consecutive queries = 64 B per d), then every d row of the block's 128
      // queries leaves as 16-B stores (256 B per row)
      constexpr int LDT = BM + 8;  // padded row (elements)
      static_assert(DP * LDT * 2 <= NS * 2 * TILE, "Oᵀ staging must fit the K/V ring");
      S* t = reinterpret_cast<S*>(smem);
      __syncthreads();  // every wave is done with the K/V ring
      const int ql = wave * 32 + l32;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int d = dt * 32 + 8 * (r >> 2) + 4 * hh + (r & 3);
          t[d * LDT + ql] = Elem<T>::from_f(o[dt][r] * inv);
        }
      __syncthreads();
      S* ot = (S*)p.ot + (int64_t)h * D * p.ot_ld + (int64_t)b * p.Nq + q0;
      const int nq = min(BM, p.Nq - q0);
      if ((p.Nq & 7) == 0 && (p.ot_ld & 7) == 0) {
        for (int c = tid; c < D * (BM / 8); c += 256) {
          const int d = c / (BM / 8), q8 = 8 * (c % (BM / 8));
          if (q8 < nq) *reinterpret_cast<uint4*>(ot + (int64_t)d * p.ot_ld + q8) = *reinterpret_cast<const uint4*>(t + d * LDT + q8);
        }
      } else {
        for (int c = tid; c < D * BM; c += 256) {
          const int d = c / BM, q = c % BM;
          if (q < nq) ot[(int64_t)d * p.ot_ld + q] = t[d * LDT + q];
        }
      }
    }
  }
}

// Explicit instantiation of the LDS-DMA variants: hipcc (ROCm 7.2) referenced some of them from the
// launch chain below without emitting their host stubs (undefined __device_stub__ at load time).
#define CS336_FA_FWD_DMA(T, D)                                                  \
  template __global__ void fa_fwd_kernel<T, D, false, false, 1>(const AttnParams); \
  template __global__ void fa_fwd_kernel<T, D, true, false, 1>(const AttnParams);  \
  template __global__ void fa_fwd_kernel<T, D, false, false, 2>(const AttnParams); \
  template __global__ void fa_fwd_kernel<T, D, true, false, 2>(const AttnParams);
CS336_FA_FWD_DMA(BF16, 32)
CS336_FA_FWD_DMA(BF16, 64)
CS336_FA_FWD_DMA(BF16, 80)
CS336_FA_FWD_DMA(BF16, 128)
CS336_FA_FWD_DMA(F16, 32)
CS336_FA_FWD_DMA(F16, 64)
CS336_FA_FWD_DMA(F16, 80)
CS336_FA_FWD_DMA(F16, 128)
#undef CS336_FA_FWD_DMA

template <typename T, int D, bool C>
void launch_fwd_c(const AttnParams& p, hipStream_t s, dim3 grid, dim3 block) {
  if (p.rope_cos != nullptr) {
    hipLaunchKernelGGL((fa_fwd_kernel<T, D, C, true, 0>), grid, block, 0, s, p);
  } else if constexpr (!std::is_same<T, float>::value) {
    if (p.dma & 4) hipLaunchKernelGGL((fa_fwd_kernel<T, D, C, false, 2>), grid, block, 0, s, p);
    else if (p.dma & 1) hipLaunchKernelGGL((fa_fwd_kernel<T, D, C, false, 1>), grid, block, 0, s, p);
    else hipLaunchKernelGGL((fa_fwd_kernel<T, D, C, false, 0>), grid, block, 0, s, p);
  } else {
    hipLaunchKernelGGL((fa_fwd_kernel<T, D, C, false, 0>), grid, block, 0, s, p);
  }
}

// merge of the split-KV partials: lse = log Σ exp(lse_s), O = Σ exp(lse_s - lse) · O_s; one thread per
// 4 consecutive d of a row
template <typename T, int D>
__global__ __launch_bounds__(256) void fa_fwd_merge_kernel(const AttnParams p) {
  typedef typename Elem<T>::storage S;
  constexpr int Q4 = (D + 3) / 4;
  const int64_t rows = (int64_t)p.B * p.H * p.Nq;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= rows * Q4) return;
  const int64_t row = gid / Q4;
  const int d = 4 * (int)(gid % Q4);
  const int bh = (int)(row / p.Nq), n = (int)(row % p.Nq);
  const int b = bh / p.H, h = bh % p.H;
  float mx = -INFINITY;
  for (int sp = 0; sp < p.kv_splits; ++sp) mx = fmaxf(mx, p.lpart[sp * rows + row]);
  float den = 0.f, a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (mx > -INFINITY) {
    for (int sp = 0; sp < p.kv_splits; ++sp) {
      const float w = __expf(p.lpart[sp * rows + row] - mx);
      const float4 v = *reinterpret_cast<const float4*>(p.opart + (sp * rows + row) * D + d);
      den += w;
      a0 = fmaf(w, v.x, a0);
      a1 = fmaf(w, v.y, a1);
      a2 = fmaf(w, v.z, a2);
      a3 = fmaf(w, v.w, a3);
    }
  }
  const float inv = den > 0.f ? 1.f / den : 0.f;
  S* orow = (S*)p.o + b * p.o_sb + h * p.o_sh + (int64_t)n * p.o_sn;
  store4<T>(orow + d, make_float4(a0 * inv, a1 * inv, a2 * inv, a3 * inv));
  if (d == 0) p.lse[row] = den > 0.f ? mx + __logf(den) : -INFINITY;
}

template <typename T, int D>
void launch_fwd(const AttnParams& p, hipStream_t s) {
  const int nqb = (p.Nq + 127) / 128;
  const dim3 grid((unsigned)(nqb * p.B * p.H * p.kv_splits)), block(256);
  if (p.causal) launch_fwd_c<T, D, true>(p, s, grid, block);
  else launch_fwd_c<T, D, false>(p, s, grid, block);
  if (p.kv_splits > 1) {
    const int64_t quads = (int64_t)p.B * p.H * p.Nq * ((D + 3) / 4);
    hipLaunchKernelGGL((fa_fwd_merge_kernel<T, D>), dim3((unsigned)((quads + 255) / 256)), block, 0, s, p);
  }
}

template <typename T>
void launch_fwd_d(const AttnParams& p, hipStream_t s) {
  switch (p.D) {
    case 16:  // computed as 32 inside the kernel (d 16..31 zero in LDS, never loaded or stored): no host padding copies
      if constexpr (std::is_same<T, float>::value) {
        fprintf(stderr, "fa_fwd: head dim 16 is 16-bit only\n");
        abort();
      } else {
        launch_fwd<T, 16>(p, s);
      }
      break;
    case 32: launch_fwd<T, 32>(p, s); break;
    case 64: launch_fwd<T, 64>(p, s); break;
    case 80:
      if constexpr (std::is_same<T, float>::value) {
        fprintf(stderr, "fa_fwd: head dim 80 is 16-bit only\n");
        abort();
      } else {
        launch_fwd<T, 80>(p, s);
      }
      break;
    case 128: launch_fwd<T, 128>(p, s); break;
    default: fprintf(stderr, "fa_fwd: unsupported head dim %d\n", p.D); abort();
  }
}

}  // namespace fa

// Split the keys when the (query block, head) workgroups cannot fill the chip (the reference sweep's
// B 1, H 1): enough splits for ~2 workgroups per CU, each split at least 4 key tiles (256 keys).
int flash_attn_fwd_splits(const AttnParams& p) {
  if (p.ot != nullptr || p.D % 4 || p.B * p.H == 0) return 1;
  const int64_t wgs = (int64_t)((p.Nq + 127) / 128) * p.B * p.H;
  const int tiles = (p.Nk + 63) / 64;
  if (wgs >= 256 || tiles < 8) return 1;
  int sp = (int)std::min<int64_t>((512 + wgs - 1) / wgs, tiles / 4);
  return std::max(1, std::min(sp, 16));
}

size_t flash_attn_fwd_split_workspace(const AttnParams& p, int splits) {
  const size_t rows = (size_t)splits * p.B * p.H * p.Nq;
  return rows * (size_t)p.D + rows;
}

void flash_attn_fwd(const AttnParams& p, DType t, hipStream_t s) {
  if (p.B * p.H == 0 || p.Nq == 0) return;
  switch (t) {
    case DType::BF16: fa::launch_fwd_d<BF16>(p, s); break;
    case DType::F16: fa::launch_fwd_d<F16>(p, s); break;
    case DType::F32: fa::launch_fwd_d<float>(p, s); break;
  }
}

}  // namespace cs336
