// FlashAttention-2 forward, persistent multi-item form for the many-heads / short-sequence regime
// (GPT-2-XL training step: B·H = 2,448-2,550 heads of N = 512, d 64).
//
// Parity: reference cs336_systems/flash_attention.py:137-266 (Triton forward, one program per query
// tile) and the handout's Algorithm 1; same math, outputs and LSE as fa_fwd.hip.
//
// Why: fa_fwd.hip runs one 128-query block per workgroup. At N 512 a block walks 2-8 key tiles, and
// the per-block fixed cost -- the Q load's HBM round trip, the first K/V tiles' DMA latency, the
// epilogue -- is worth ~8 tiles of work (fit of the round-5 A/B: 367 TF at N 512 vs 771 TF at N 4096,
// same kernel), so the forward ran at 15 % of the matrix cores and 48 % of its HBM roofline.
// Here a fixed grid of workgroups (as many as fit the CUs at once) walks a static list of
// (batch·head, query block) items, and ONE LDS-DMA stream carries everything a workgroup reads:
// for each item its Q block (128 rows, one ring slot) followed by its K/V tiles (64 keys, K | V in
// one slot). The ring keeps two slots in flight across item boundaries, so the next item's Q and
// first K/V tiles land while the current item's last tiles compute, and there is no per-item
// launch, descriptor setup or cold start. The epilogue stores go out through buffer stores whose
// count is the same for every wave (out-of-range lanes are dropped by the descriptor), so the
// ring's counted vmcnt waits stay exact with stores in flight.
//
// Item order: workgroup g serves XCD g % 8 (the dispatcher's round-robin) and only heads bh ≡ g
// (mod 8), so a head's query blocks share one L2; inside an XCD the heads form groups whose K/V
// fit the 4 MB L2, each group's items are taken level-major (heaviest causal block first), and a
// workgroup's rank is rotated by one group per round so that every workgroup sees every level.
#include "fa_common.h"

#include <algorithm>

namespace cs336 {
namespace fa {

namespace {

typedef __attribute__((ext_vector_type(4))) unsigned int v4u32;

template <int D>
constexpr int multi_min_wgs() {
  return PadD<D>::value <= 64 ? 3 : 2;  // 48 KiB of LDS and <= 168 VGPRs at d <= 64
}

struct MultiItems {
  int x, r, Gx;       // XCD, rank inside the XCD, workgroups of the XCD
  int nbh, nqb, nhx;  // heads, query blocks per head, heads of this XCD
  int g;              // heads per group
  int n;              // items of this XCD
  // item k of this workgroup's walk (k = 0, 1, ...): false past the end
  __device__ __forceinline__ bool get(int k, int& bh, int& lvl) const {
    const int t = k * Gx + (r + k * g) % Gx;
    if (t >= n) return false;
    const int gsz = g * nqb, gi = t / gsz, w = t - gi * gsz;
    const int gs = min(g, nhx - gi * g);
    lvl = w / gs;
    bh = x + 8 * (gi * g + (w - lvl * gs));
    return true;
  }
};

}  // namespace

template <typename T, int D, bool CAUSAL>
__global__ __launch_bounds__(256, (multi_min_wgs<D>())) void fa_fwd_multi_kernel(const AttnParams p, int group) {
  typedef typename Elem<T>::storage S;
  typedef typename Mma16<T>::frag F;
  constexpr int ES = 2;
  constexpr int DP = PadD<D>::value;
  constexpr int RB = DP * ES;
  constexpr int CREAL = D * ES / 16;
  constexpr int BM = 128, BN = 64;
  constexpr int TILE = BN * RB;   // one K (or V) tile
  constexpr int SLOT = BM * RB;   // = a Q block = K tile | V tile
  constexpr int NDT = DP / 32;
  constexpr int NS = DP <= 64 ? 3 : 2;
  using QDma = TileDma<BM, RB, CREAL, ES>;
  using KDma = TileDma<BN, RB, CREAL, ES>;
  constexpr int PER = QDma::PER_WAVE;  // wave-instructions per slot (Q: 128 rows; K + V: 2 x 64)
  static_assert(PER == 2 * KDma::PER_WAVE, "a Q slot and a K|V slot take the same DMA count");
  constexpr int NST = 2 * NDT + 1;  // epilogue stores per wave: O (16-B pairs) + LSE
  // (the V-fragment prefetch of fa_fwd.hip spills here: the Q ring offsets and the item cursors take
  // the registers it needs; 158 VGPRs without it)
  constexpr bool VPRE = false;

  __shared__ __attribute__((aligned(1024))) char smem[NS * SLOT];

  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  const int l32 = lane & 31, hh = lane >> 5;

  MultiItems it;
  it.x = (int)(blockIdx.x & 7u);
  it.r = (int)(blockIdx.x >> 3);
  it.Gx = (int)(gridDim.x >> 3);
  it.nbh = p.B * p.H;
  it.nqb = (p.Nq + BM - 1) / BM;
  it.nhx = (it.nbh - it.x + 7) / 8;
  it.g = group;
  it.n = it.nhx * it.nqb;

  auto qblock = [&](int lvl) { return CAUSAL ? it.nqb - 1 - lvl : lvl; };
  auto ntiles_of = [&](int qb) {
    const int kv_end = CAUSAL ? min(p.Nk, qb * BM + BM) : p.Nk;
    return (kv_end + BN - 1) / BN;
  };

  QDma qd;
  KDma kd, vd;
  qd.init(wave, lane, p.q_sn);
  kd.init(wave, lane, p.k_sn);
  vd.init(wave, lane, p.v_sn);

  // ---- the stream: per item, part -1 = its Q block, parts 0 .. ntiles-1 = its K/V tiles ----------
  int ik = 0, ipart = -1, ibh = 0, iqb = 0, intl = 0;  // issue cursor
  bool ivalid;
  {
    int lvl;
    ivalid = it.get(0, ibh, lvl);
    if (ivalid) {
      iqb = qblock(lvl);
      intl = ntiles_of(iqb);
    }
  }
  auto issue_next = [&](char* slot) {
    if (!ivalid) {  // past the last item: an empty group keeps every wait count static
      qd.issue(p.q, 0, p.q_sn, slot, wave);
      return;
    }
    const int b = ibh / p.H, h = ibh % p.H;
    if (ipart < 0) {
      const int q0 = iqb * BM;
      qd.issue((const S*)p.q + b * p.q_sb + h * p.q_sh + (int64_t)q0 * p.q_sn, min(BM, p.Nq - q0), p.q_sn, slot, wave);
    } else {
      const int k0 = ipart * BN, rows = min(BN, p.Nk - k0);
      kd.issue((const S*)p.k + b * p.k_sb + h * p.k_sh + (int64_t)k0 * p.k_sn, rows, p.k_sn, slot, wave);
      vd.issue((const S*)p.v + b * p.v_sb + h * p.v_sh + (int64_t)k0 * p.v_sn, rows, p.v_sn, slot + TILE, wave);
    }
    if (++ipart == intl) {
      ipart = -1;
      int lvl;
      ivalid = it.get(++ik, ibh, lvl);
      if (ivalid) {
        iqb = qblock(lvl);
        intl = ntiles_of(iqb);
      }
    }
  };

  // zero the ring once: rows a DMA leaves untouched (d 80..95, tails past Nq / Nk) stay finite
  lds_zero(smem, NS * SLOT);
  __syncthreads();
#pragma unroll
  for (int u = 0; u < NS - 1; ++u) issue_next(smem + u * SLOT);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // (nothing the compiler issued is outstanding: see wait_vmcnt)

  const float c2 = p.scale * kLog2e;
  uint4 qf[DP / 16];
  float m = kNegBig, l = 0.f;
  f32x16 o[NDT];
  int cbh = 0, cqb = 0, cntl = 0, cpart = -1, ck = 0;  // consume cursor
  {
    int lvl;
    if (!it.get(0, cbh, lvl)) {
      wait_vmcnt<0>();
      return;
    }
    cqb = qblock(lvl);
    cntl = ntiles_of(cqb);
  }
  // epilogues of the last two steps: slot u's DMA was issued at step u-NS+1, before that step's
  // consume, so the stores of steps u-NS+1 .. u-1 are younger than it (at most one of them: two
  // epilogues are at least two steps apart, a Q step between them)
  bool epi1 = false, epi2 = false;
  // one step of the stream; SL = the step's ring slot (compile time: the loop below is unrolled by the
  // ring depth, so every slot address is an immediate)
  auto step = [&](auto sl) __attribute__((always_inline)) -> bool {
    constexpr int SL = decltype(sl)::value;
    // slot u landed: younger are the slots u+1 .. u+NS-2 and those stores
    if constexpr (NS == 3) {
      if (epi1 || epi2) wait_vmcnt<PER + NST>();
      else wait_vmcnt<PER>();
    } else {
      if (epi1) wait_vmcnt<NST>();
      else wait_vmcnt<0>();
    }
    dma_barrier();
    issue_next(smem + ((SL + NS - 1) % NS) * SLOT);
    epi2 = epi1;
    epi1 = false;
    const char* slot = smem + SL * SLOT;
    const int q0 = cqb * BM, qw0 = q0 + wave * 32, qrow = qw0 + l32;
    if (cpart < 0) {
      // ---- new item: Q fragments from the ring, fresh softmax state ----
#pragma unroll
      for (int ks = 0; ks < DP / 16; ++ks) qf[ks] = __builtin_bit_cast(uint4, lds_row_frag<T, RB>(slot, wave * 32, ks, lane));
      m = kNegBig;
      l = 0.f;
#pragma unroll
      for (int i = 0; i < NDT; ++i) o[i] = zero16();
    } else if (!CAUSAL || cpart * BN <= qw0 + 31) {
      // ---- one K/V tile: S^T = K Q^T, mask, online softmax, O^T += V^T P^T (as fa_fwd.hip) ----
      const int kt0 = cpart * BN;
      const char* Ks = slot;
      const char* Vs = slot + TILE;
      f32x16 s[2];
      if constexpr (DP <= 64) {
        F kf[2][DP / 16];
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int ks = 0; ks < DP / 16; ++ks) kf[t][ks] = lds_row_frag<T, RB>(Ks, 32 * t, ks, lane);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          s[t] = zero16();
#pragma unroll
          for (int ks = 0; ks < DP / 16; ++ks) s[t] = Mma16<T>::mma(kf[t][ks], as_frag<T>(qf[ks]), s[t]);
        }
      } else {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          s[t] = zero16();
#pragma unroll
          for (int ks = 0; ks < DP / 16; ++ks)
            s[t] = Mma16<T>::mma(lds_row_frag<T, RB>(Ks, 32 * t, ks, lane), as_frag<T>(qf[ks]), s[t]);
        }
      }
      if ((kt0 + BN > p.Nk) || (CAUSAL && kt0 + BN - 1 > qw0)) {
        const int lim = (CAUSAL ? min(p.Nk - 1, qrow) : p.Nk - 1) - kt0 - 4 * hh;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (32 * t + acc_row(r, 0) > lim) s[t][r] = -INFINITY;
      }
      float mx = s[0][0];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[t][r]);
      mx = xhalf_max(mx);
      const float mt = mx * c2;
      if (__ballot(mt > m + kRescaleThr) != 0) {  // wave-uniform (T13)
        const float m_new = fmaxf(m, mt);
        const float alpha = fexp2(m - m_new);
        l *= alpha;
        m = m_new;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
      }
      F vf[VPRE ? NDT : 1][2][2];
      if constexpr (VPRE) {
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) vf[dt][t][s2] = lds_tr_frag<T, RB>(Vs, 32 * t, s2, dt, lane);
        __builtin_amdgcn_sched_barrier(0);
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
      F pf[2][2];
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
          for (int s2 = 0; s2 < 2; ++s2) {
            if constexpr (VPRE) o[dt] = Mma16<T>::mma(vf[dt][t][s2], pf[t][s2], o[dt]);
            else o[dt] = Mma16<T>::mma(lds_tr_frag<T, RB>(Vs, 32 * t, s2, dt, lane), pf[t][s2], o[dt]);
          }
    }
    if (cpart == cntl - 1) {
      // ---- epilogue: O (16-B pairs, guide T21) and LSE through buffer stores; every wave issues
      // exactly NST of them (rows >= Nq and d >= D fall outside the descriptor and are dropped) ----
      const int b = cbh / p.H, h = cbh % p.H;
      const float lt = xhalf_sum(l);
      const float inv = lt > 0.f ? 1.f / lt : 0.f;
      const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
          (void*)((S*)p.o + b * p.o_sb + h * p.o_sh), (short)0, (int)((int64_t)p.Nq * p.o_sn * ES), 0x00020000);
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
          const uint32_t voff = (DP == D || d < D) ? (uint32_t)(((int64_t)qrow * p.o_sn + d) * ES) : 0x80000000u;
          v4u32 cv;
          cv[0] = c[0];
          cv[1] = c[1];
          cv[2] = c[2];
          cv[3] = c[3];
          __builtin_amdgcn_raw_buffer_store_b128(cv, ro, voff, 0, 0);
        }
      const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(p.lse + (int64_t)cbh * p.Nq), (short)0, p.Nq * 4, 0x00020000);
      const float lse = lt > 0.f ? (m + __log2f(lt)) * kLn2 : -INFINITY;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(lse), rl, hh == 0 ? (uint32_t)qrow * 4u : 0x80000000u, 0, 0);
      epi1 = true;
      // next item (or the end of this workgroup's walk)
      int lvl;
      if (!it.get(++ck, cbh, lvl)) return false;
      cqb = qblock(lvl);
      cntl = ntiles_of(cqb);
      cpart = -1;
    } else {
      ++cpart;
    }
    return true;
  };
  for (;;) {
    if (!step(std::integral_constant<int, 0>{})) break;
    if (!step(std::integral_constant<int, 1>{})) break;
    if constexpr (NS == 3)
      if (!step(std::integral_constant<int, 2>{})) break;
  }
  // the trailing (empty) DMA groups and the last stores retire before the workgroup's LDS is freed
  wait_vmcnt<0>();
}

template <typename T, int D>
void launch_multi(const AttnParams& p, hipStream_t s, int grid, int group) {
  if (p.causal) hipLaunchKernelGGL((fa_fwd_multi_kernel<T, D, true>), dim3((unsigned)grid), dim3(256), 0, s, p, group);
  else hipLaunchKernelGGL((fa_fwd_multi_kernel<T, D, false>), dim3((unsigned)grid), dim3(256), 0, s, p, group);
}

}  // namespace fa

namespace {
int cu_count_cached() {
  static const int n = [] {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    return cus;
  }();
  return n;
}
}  // namespace

// The persistent multi-item forward takes 16-bit causal or full attention at d 64 without RoPE-on-load,
// split-KV or the Oᵀ copy, when the items outnumber the resident workgroups several times (else the
// one-block-per-workgroup kernel has nothing to amortize). Opt-in (CS336_FA_FWD_MULTI=1) until it
// beats that kernel at the step's shapes (profiles/r5_fa_fwd.md).
bool flash_attn_fwd_multi(const AttnParams& p, DType t, hipStream_t s) {
  const char* e = std::getenv("CS336_FA_FWD_MULTI");  // per call (cheap next to a launch): tests switch it
  const int env = e && *e ? std::atoi(e) : -1;
  if (env != 1 || t == DType::F32 || p.rope_cos != nullptr || p.ot != nullptr || p.kv_splits > 1) return false;
  if (p.D != 64) return false;
  const int64_t nbh = (int64_t)p.B * p.H, nqb = (p.Nq + 127) / 128, items = nbh * nqb;
  const int wgs = 3;  // fa::multi_min_wgs<64>()
  int grid = cu_count_cached() * wgs;
  grid -= grid % 8;
  if (grid < 8 || items < 4 * (int64_t)grid || nbh < 8) return false;
  // 32-bit buffer offsets: one head's rows of q / k / v / o
  const int64_t rows = std::max<int64_t>(p.Nq, p.Nk);
  const int64_t ld = std::max({p.q_sn, p.k_sn, p.v_sn, p.o_sn});
  if (rows * ld * 2 >= (int64_t(1) << 31)) return false;
  // heads per group: the group's K/V fit one XCD's 4 MB L2 and its items fill about one round of
  // the XCD's workgroups
  const int gx = grid / 8;
  const int64_t kv_head = 2 * (int64_t)p.Nk * p.D * 2;
  const int group = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t(4) << 20) / kv_head, std::max<int64_t>(1, gx / nqb)));
  switch (t) {
    case DType::BF16: fa::launch_multi<BF16, 64>(p, s, grid, group); break;
    case DType::F16: fa::launch_multi<F16, 64>(p, s, grid, group); break;
    default: return false;
  }
  return true;
}

}  // namespace cs336
