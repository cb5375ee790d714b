// FlashAttention-2 backward, head-sequential with TWO workgroups per CU: one kernel, five MFMA
// products per tile pair (S, dP, dVᵀ, dKᵀ, dQᵀ), one 4-wave workgroup per (batch, head) walking the
// head's 128-key blocks in order, for the many-heads / short-sequence regime of the training step
// (GPT-2-XL: B·H = 2400 heads of N = 512, d 64 at per-GPU batch 96).
// cs336-build: no-slp
//
// Parity: reference cs336_systems/flash_attention.py:270-289 (a torch.compile'd recompute backward
// over the full N x N matrices; handout Algorithm 2).
//
// Why another head-sequential form: fa_bwd_fused.hip (8 waves, 256-key blocks) needs 152 KiB of LDS,
// so one workgroup holds a CU and its waves wait 50-55 % of their cycles -- on its own barriers
// and on the prologue / key-block-switch memory round trips that nothing else on the CU covers
// (profiles/r3_fa_bwd_fused_ab.md). Here a workgroup is 4 waves (one per SIMD, <= 256 registers)
// over a 128-key block and needs 66 KiB, so two independent workgroups share every CU: while one
// waits on a barrier or a memory round trip, the other's MFMAs run on the same SIMDs.
//
// Layout per workgroup (78 KiB of LDS; two fit a CU's 160 KiB):
//   2 slots x {Q slice image 8 KiB | dO slice image 8 KiB | row constants 1 KiB}   (LDS-DMA)
//   K block image 16 KiB (LDS-DMA, once per key block) | dSᵀ image 16 KiB
//   O slice image 8 KiB | -delta of the whole head 4 KiB (N <= 1024)
// delta = rowsum(dO·O) is computed here during the first key block (every slice passes once), from
// the dO image the item staged anyway and an O image staged one item ahead; the slot's row constants
// are then the slice's raw lse. For N > 1024 (or CS336_FA_HS_DELTA=0) a prep kernel writes both row
// constants instead (one pass over O and dO, as fa_bwd_kp.hip) and the kernel needs 66 KiB.
//
// Wave w owns keys 32w .. 32w+31 of the block (key on the MFMA lane), keeps their dKᵀ / dVᵀ (fp32)
// and V (the B operand of dP) in registers, and per 64-query slice, one 32-query tile at a time:
//   S = Q Kᵀ, dP = dO Vᵀ - delta (row constant as the accumulator's start), P = exp2(S c - L),
//   dS = P dP, dVᵀ += dOᵀ P, dKᵀ += Qᵀ dS, dSᵀ -> LDS;
// barrier; wave w then forms the dQᵀ tile (d 32(w&1).., queries 32(w>>1)..) = Kᵀ dSᵀ over the block's
// active keys. The dQ sum across key blocks runs through fp32 partials in global memory, loaded and
// stored by the same lanes (L2-resident, no atomics, deterministic); the slice's last contributing
// key block writes dQ (x scale, inverse RoPE folded in when q was rotated).
//
// Memory ordering (vmcnt counts LDS-DMA, loads and stores in issue order): item j issues, in order,
// its dQ partial loads (key blocks > 0), its 4 dQ stores, then the DMA of item j + 2 into the slot it
// just finished reading. The compiler's own wait for the partial loads (it cannot see the DMA) also
// retires item j + 1's DMA, issued an item earlier; without partial loads the next item waits for
// everything but this item's stores and DMA (4 + its DMA count). A key-block switch drains to 0.
#include "fa_common.h"

namespace cs336 {
namespace fa {

namespace {
constexpr int HS_D = 64;
constexpr int HS_RB = HS_D * 2;              // 128-B image rows
constexpr int HS_BQ = 64;                    // query slice
constexpr int HS_KB = 128;                   // keys per block: 4 waves x 32
constexpr int HS_TILE = HS_BQ * HS_RB;       // 8 KiB
constexpr int HS_SLOT = 2 * HS_TILE + 1024;  // Q | dO | row constants (512 B used)
constexpr int HS_NS = 2;
constexpr int HS_OFF_K = HS_NS * HS_SLOT;
constexpr int HS_OFF_DS = HS_OFF_K + HS_KB * HS_RB;
constexpr int HS_LDS = HS_OFF_DS + HS_KB * 128;  // dSᵀ [key][64 q], 128-B rows
static_assert(HS_LDS <= 80 * 1024, "two workgroups per CU");
// in-kernel delta (IND): + an O slice image (single, restaged one item ahead) + -delta of the whole
// head (fp32, row_perm order per slice), N <= HS_MAXN
constexpr int HS_MAXN = 1024;
constexpr int HS_OFF_O = HS_LDS;
constexpr int HS_OFF_DH = HS_OFF_O + HS_TILE;
constexpr int HS_LDS_IND = HS_OFF_DH + HS_MAXN * 4;
static_assert(HS_LDS_IND <= 80 * 1024, "two workgroups per CU");
constexpr int HS_SLICE_DMA = 2 * (HS_BQ * (HS_RB / 16) / 256);  // Q + dO wave-instructions per wave

// CS336_FA_HS_DELTA=0: row constants from the prep kernel instead of the in-kernel delta
inline bool hs_in_kernel_delta() {
  const char* e = getenv("CS336_FA_HS_DELTA");
  return !(e && *e && atoi(e) == 0);
}

// wait until at most n of this wave's vector memory operations are outstanding (n wave-uniform;
// the counts that occur: 4 + {0, 4, 5})
__device__ __forceinline__ void wait_vm_upto(int n) {
  if (n >= 9) wait_vmcnt<9>();
  else if (n >= 8) wait_vmcnt<8>();
  else if (n >= 4) wait_vmcnt<4>();
  else wait_vmcnt<0>();
}
}  // namespace

// ---- (1) row constants -----------------------------------------------------------------------
// block = (head, 64-row slice); 4 threads per row, 16 d each
template <typename T>
__global__ __launch_bounds__(256) void fa_bwd_hs_prep(const AttnBwdParams bp, float* __restrict__ rowc) {
  typedef typename Elem<T>::storage S;
  const int N = bp.f.Nq, nqs = N / HS_BQ;
  const int bh = blockIdx.x / nqs, s = blockIdx.x % nqs;
  const int b = bh / bp.f.H, h = bh % bp.f.H;
  const int tid = threadIdx.x, r = tid >> 2, k = tid & 3, row = s * HS_BQ + r;
  const S* o = (const S*)bp.f.o + b * bp.f.o_sb + h * bp.f.o_sh + (int64_t)row * bp.f.o_sn + 16 * k;
  const S* g = (const S*)bp.dout + b * bp.do_sb + h * bp.do_sh + (int64_t)row * bp.do_sn + 16 * k;
  const uint4 uo[2] = {*reinterpret_cast<const uint4*>(o), *reinterpret_cast<const uint4*>(o + 8)};
  const uint4 ug[2] = {*reinterpret_cast<const uint4*>(g), *reinterpret_cast<const uint4*>(g + 8)};
  float dsum = 0.f;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const uint32_t wo[4] = {uo[c].x, uo[c].y, uo[c].z, uo[c].w}, wg[4] = {ug[c].x, ug[c].y, ug[c].z, ug[c].w};
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      dsum = fmaf(Elem<T>::to_f((S)(wo[w] & 0xffff)), Elem<T>::to_f((S)(wg[w] & 0xffff)), dsum);
      dsum = fmaf(Elem<T>::to_f((S)(wo[w] >> 16)), Elem<T>::to_f((S)(wg[w] >> 16)), dsum);
    }
  }
  dsum += __shfl_xor(dsum, 1, 64);
  dsum += __shfl_xor(dsum, 2, 64);
  if (k == 0) {
    float* rc = rowc + ((int64_t)bh * nqs + s) * 128;
    rc[row_perm(r)] = -bp.f.lse[(int64_t)bh * N + row] * kLog2e;
    rc[64 + row_perm(r)] = -dsum;
  }
}

// ---- (2) main kernel -------------------------------------------------------------------------
// ROPE: 0 = none, 1 = inverse rotation in the dQ and dK stores, 2 = in the dK stores only (the caller
// rotates dQ back in a separate pass). IND: delta = rowsum(dO·O) computed here during the first key
// block's pass (O slices staged by LDS-DMA one item ahead, -delta of the head kept in LDS) and the
// row's lse staged raw with each slice -- no prep kernel, no second read of dO; else the row
// constants come from fa_bwd_hs_prep (rowc).
template <typename T, bool CAUSAL, int ROPE, bool IND>
__global__ __launch_bounds__(256, 2) void fa_bwd_hs_kernel(const AttnBwdParams bp, const float* __restrict__ rowc,
                                                           float* __restrict__ part_all) {
  typedef typename Elem<T>::storage S;
  typedef typename Mma16<T>::frag F;
  __shared__ __attribute__((aligned(1024))) char smem[IND ? HS_LDS_IND : HS_LDS];

  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  const int l32 = lane & 31, hh = lane >> 5;
  const int bh = blockIdx.x, b = bh / bp.f.H, h = bh % bp.f.H;
  const int N = bp.f.Nq;  // == Nk, N % 128 == 0 (host-checked)
  const int nqs = N / HS_BQ, nkb = N / HS_KB;
  const int q_sn = (int)bp.f.q_sn, k_sn = (int)bp.f.k_sn, v_sn = (int)bp.f.v_sn, do_sn = (int)bp.do_sn;
  const S* Qp = (const S*)bp.f.q + b * bp.f.q_sb + h * bp.f.q_sh;
  const S* Kp = (const S*)bp.f.k + b * bp.f.k_sb + h * bp.f.k_sh;
  const S* Vp = (const S*)bp.f.v + b * bp.f.v_sb + h * bp.f.v_sh;
  const S* dOp = (const S*)bp.dout + b * bp.do_sb + h * bp.do_sh;
  const float sc = bp.f.scale, c2 = bp.f.scale * kLog2e;
  char* const Kimg = smem + HS_OFF_K;
  char* const dsimg = smem + HS_OFF_DS;

  // ---- per-lane LDS offsets (row bases are multiples of 16 rows: the swizzle is the lane's) ----
  const int swl = swz<HS_RB>(l32);
  uint32_t roff[4];  // row fragments: row l32, chunk 2ks + hh
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) roff[ks] = (uint32_t)(l32 * HS_RB + (((2 * ks + hh) ^ swl) << 4));
  uint32_t toa[2], tob[2];  // transposed fragments of 32-column tile c of a 128-B-row image
  {
    const int ti = lane & 15, tra = 4 * hh + (ti >> 2), tcl = ((lane >> 4) & 1) * 2 + ((ti & 3) >> 1);
    const int swa = swz<HS_RB>(tra), swb = swz<HS_RB>(tra + 8);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      toa[c] = (uint32_t)(tra * HS_RB + ((((c << 2) | tcl) ^ swa) << 4) + (ti & 1) * 8);
      tob[c] = (uint32_t)((tra + 8) * HS_RB + ((((c << 2) | tcl) ^ swb) << 4) + (ti & 1) * 8);
    }
  }
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

  // ---- LDS-DMA staging ---------------------------------------------------------------------------
  TileDma<HS_BQ, HS_RB, 8, 2> dq_, dd_;
  dq_.init(wave, lane, q_sn);
  dd_.init(wave, lane, do_sn);
  TileDma<HS_KB, HS_RB, 8, 2> dk_;
  dk_.init(wave, lane, k_sn);
  // row constants of a slice: IND -- the slice's 64 raw lse values (256 B) in row_perm order, lane c < 16
  // moving source rows 4 row_perm_src_chunk(c) .. +3; else 512 B of the prep kernel's rowc
  const __amdgpu_buffer_rsrc_t rrc =
      IND ? __builtin_amdgcn_make_buffer_rsrc((void*)(bp.f.lse + (int64_t)bh * N), (short)0, N * 4, 0x00020000)
          : __builtin_amdgcn_make_buffer_rsrc((void*)(rowc + (int64_t)bh * nqs * 128), (short)0, nqs * 512, 0x00020000);
  const uint32_t vrc = IND ? (lane < 16 ? (uint32_t)(row_perm_src_chunk(lane) * 16) : 0x80000000u)
                           : (lane < 32 ? (uint32_t)(lane * 16) : 0x80000000u);  // other lanes: out of range
  auto issue_slot = [&](int s, int slot) {
    char* base = smem + slot * HS_SLOT;
    dq_.issue(Qp + (int64_t)s * HS_BQ * q_sn, HS_BQ, q_sn, base, wave);
    dd_.issue(dOp + (int64_t)s * HS_BQ * do_sn, HS_BQ, do_sn, base + HS_TILE, wave);
    if (wave == 0) dma16(rrc, lds_addr(base + 2 * HS_TILE), vrc, (uint32_t)(s * (IND ? 256 : 512)));
  };
  // IND: O slice image (single buffer) and the head's -delta
  TileDma<HS_BQ, HS_RB, 8, 2> do_;
  if constexpr (IND) do_.init(wave, lane, bp.f.o_sn);
  const S* Op = (const S*)bp.f.o + b * bp.f.o_sb + h * bp.f.o_sh;
  char* const Oimg = smem + HS_OFF_O;
  float* const Dh = reinterpret_cast<float*>(smem + HS_OFF_DH);
  auto issue_o = [&](int s) { do_.issue(Op + (int64_t)s * HS_BQ * bp.f.o_sn, HS_BQ, bp.f.o_sn, Oimg, wave); };
  // -delta of slice s from the landed dO (slot image) and O images: thread = (row tid>>2, 16 d of
  // quarter tid&3 = chunks 2k, 2k+1)
  auto delta_slice = [&](int s, const char* dOs) {
    const int r = tid >> 2, k = tid & 3;
    float acc = 0.f;
#pragma unroll
    for (int c = 2 * k; c < 2 * k + 2; ++c) {
      const uint4 ug = *reinterpret_cast<const uint4*>(dOs + lds_off<HS_RB>(r, c));
      const uint4 uo = *reinterpret_cast<const uint4*>(Oimg + lds_off<HS_RB>(r, c));
      const uint32_t wg[4] = {ug.x, ug.y, ug.z, ug.w}, wo[4] = {uo.x, uo.y, uo.z, uo.w};
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        acc = fmaf(Elem<T>::to_f((S)(wg[w] & 0xffff)), Elem<T>::to_f((S)(wo[w] & 0xffff)), acc);
        acc = fmaf(Elem<T>::to_f((S)(wg[w] >> 16)), Elem<T>::to_f((S)(wo[w] >> 16)), acc);
      }
    }
    acc += __shfl_xor(acc, 1, 64);
    acc += __shfl_xor(acc, 2, 64);
    if (k == 0) Dh[s * HS_BQ + row_perm(r)] = -acc;
  };
  auto sbeg = [&](int kb) { return CAUSAL ? kb * (HS_KB / HS_BQ) : 0; };
  auto advance = [&](int& kb, int& s) {
    if (++s >= nqs) {
      ++kb;
      s = sbeg(kb);
    }
  };

  // ---- per-wave state: keys kbase + 32 wave + l32 ------------------------------------------------
  uint4 vf[4];          // V B fragments (key on the lane): d = 16i + 8hh .. +7
  f32x16 dk[2], dv[2];  // dKᵀ, dVᵀ per d tile: lane = key, registers = d
  auto load_v = [&](int kb) {
    const int key = kb * HS_KB + 32 * wave + l32;
#pragma unroll
    for (int i = 0; i < 4; ++i) vf[i] = *reinterpret_cast<const uint4*>(Vp + key * v_sn + 16 * i + 8 * hh);
  };
  auto zero_kv = [&]() {
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      dk[dt] = zero16();
      dv[dt] = zero16();
    }
  };
  const Rope rope{bp.f.rope_cos, bp.f.rope_sin, HS_D / 2};
  auto store_kv = [&](int kb) {
    const int key = kb * HS_KB + 32 * wave + l32;
    S* rk = (S*)bp.dk + b * bp.dk_sb + h * bp.dk_sh + (int64_t)key * bp.dk_sn;
    S* rv = (S*)bp.dv + b * bp.dv_sb + h * bp.dv_sh + (int64_t)key * bp.dv_sn;
    const int64_t pos = ROPE != 0 ? (bp.f.rope_pos ? bp.f.rope_pos[(int64_t)b * N + key] : key) : 0;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = 32 * dt + 8 * g4 + 4 * hh;
        float k0 = dk[dt][4 * g4] * sc, k1 = dk[dt][4 * g4 + 1] * sc, k2 = dk[dt][4 * g4 + 2] * sc,
              k3 = dk[dt][4 * g4 + 3] * sc;
        if constexpr (ROPE != 0) rope_inv4(k0, k1, k2, k3, rope, pos, d);
        store4<T>(rk + d, make_float4(k0, k1, k2, k3));
        store4<T>(rv + d, make_float4(dv[dt][4 * g4], dv[dt][4 * g4 + 1], dv[dt][4 * g4 + 2], dv[dt][4 * g4 + 3]));
      }
  };

  // dQᵀ tile of this wave: d rows 32 dqt.., queries 32 qqt..
  const int dqt = wave & 1, qqt = wave >> 1;
  float* const part = part_all + (int64_t)bh * N * HS_D + 32 * dqt + 4 * hh;  // + q * 64: fp32 partials
  S* const dQp = (S*)bp.dq + b * bp.dq_sb + h * bp.dq_sh;

  // ---- prologue: K image 0, slices of items 0 and 1, V of block 0 -----------------------------------
  dk_.issue(Kp, HS_KB, k_sn, Kimg, wave);
  if constexpr (IND) issue_o(0);
  {
    int kb1 = 0, s1 = sbeg(0);
    issue_slot(s1, 0);
    advance(kb1, s1);
    if (kb1 < nkb) issue_slot(s1, 1);
  }
  load_v(0);
  zero_kv();
  wait_vmcnt<0>();
  dma_barrier();

  // ---- the walk ------------------------------------------------------------------------------------
  int it = 0, nwait = 63;  // nwait: vector memory ops the next item may leave in flight
  for (int kb = 0; kb < nkb; ++kb) {
    const int kbase = kb * HS_KB;
    const int k0g = kbase + 32 * wave;
    for (int s = sbeg(kb); s < nqs; ++s, ++it) {
      const int slot = it & 1;
      const char* Qs = smem + slot * HS_SLOT;
      const char* dOs = Qs + HS_TILE;
      const float* Ls = reinterpret_cast<const float*>(Qs + 2 * HS_TILE);  // -lse·log2e (IND: lse), row_perm order
      const float* Ds = IND ? Dh + s * HS_BQ : Ls + 64;                    // -delta
      const int q0 = s * HS_BQ;
      // A: this item's slice landed in every wave's share; the previous item's dSᵀ / K reads retired
      wait_vm_upto(nwait);
      dma_barrier();
      if (IND && kb == 0) {
        // the slice's -delta (first key block: every slice passes once), then the next O slice into
        // the freed O image
        delta_slice(s, dOs);
        dma_barrier();
        if (s + 1 < nqs) issue_o(s + 1);
      }
      // B: this tile's dQ partial sums from the earlier key blocks (L2)
      const int kb_last = CAUSAL ? min((q0 + HS_BQ - 1) / HS_KB, nkb - 1) : nkb - 1;
      const bool first = kb == 0, last = kb == kb_last;
      const int qrow = q0 + 32 * qqt + l32;
      float4 pp[4];
      if (!first) {
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) pp[g4] = *reinterpret_cast<const float4*>(part + qrow * HS_D + 8 * g4);
      }

      // C: S, dP, P, dS, dVᵀ, dKᵀ of this wave's group; dSᵀ into LDS
      if (!CAUSAL || k0g <= q0 + HS_BQ - 1) {
        const char* Kg = Kimg + 32 * wave * HS_RB;
        F kfr[4];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) kfr[ks] = rowf(Kg, ks);
        const int kq = k0g + l32 - q0 - 4 * hh;  // key - (query of register 0 of this half)
        char* drow = dsimg + (32 * wave + l32) * 128 + 8 * hh;
#pragma nounroll
        for (int t = 0; t < 2; ++t) {
          const char* Qt = Qs + 32 * t * HS_RB;
          const char* dOt = dOs + 32 * t * HS_RB;
          F qa[4], oa[4];
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) {
            qa[ks] = rowf(Qt, ks);
            oa[ks] = rowf(dOt, ks);
          }
          f32x16 dp = *reinterpret_cast<const f32x16*>(Ds + 32 * t + 16 * hh);
          f32x16 sa = zero16();
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) {
            sa = Mma16<T>::mma(qa[ks], kfr[ks], sa);
            dp = Mma16<T>::mma(oa[ks], as_frag<T>(vf[ks]), dp);
          }
          // P = exp2(S c - L), dS = P dP; the causal compare runs on every tile (off the diagonal it is never
          // true): specializing the diagonal tiles measured 1 % slower (profiles/r4_fa_bwd_hs.md)
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {
            const float4 L4 = *reinterpret_cast<const float4*>(Ls + 32 * t + 16 * hh + 4 * g4);
            const float lm = IND ? -kLog2e : 1.f;
            const float Lv[4] = {lm * L4.x, lm * L4.y, lm * L4.z, lm * L4.w};
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int r = 4 * g4 + u;
              float pv = fexp2(fmaf(sa[r], c2, Lv[u]));
              if (CAUSAL && kq > 32 * t + 8 * g4 + u) pv = 0.f;
              sa[r] = pv;
              dp[r] = pv * dp[r];
            }
          }
          F pf[2], sf[2];
          pf[0] = pack_acc<T>(sa, 0);
          pf[1] = pack_acc<T>(sa, 1);
          sf[0] = pack_acc<T>(dp, 0);
          sf[1] = pack_acc<T>(dp, 1);
#pragma unroll
          for (int dt = 0; dt < 2; ++dt) {
            F ot[2], qt[2];
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
              ot[s2] = trf2(dOt + 16 * s2 * HS_RB, toa[dt], tob[dt]);
              qt[s2] = trf2(Qt + 16 * s2 * HS_RB, toa[dt], tob[dt]);
            }
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
              dv[dt] = Mma16<T>::mma(ot[s2], pf[s2], dv[dt]);
              dk[dt] = Mma16<T>::mma(qt[s2], sf[s2], dk[dt]);
            }
          }
          // dSᵀ row (block-local key 32 wave + l32): query halves 32t + 16s2 + 4hh + 0..3 and + 8
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            const uint4 w = __builtin_bit_cast(uint4, sf[s2]);
            const int ch = 4 * t + 2 * s2;
            *reinterpret_cast<uint2*>(drow + ((ch ^ swl) << 4)) = make_uint2(w.x, w.y);
            *reinterpret_cast<uint2*>(drow + (((ch + 1) ^ swl) << 4)) = make_uint2(w.z, w.w);
          }
        }
      }
      dma_barrier();  // D: dSᵀ of every group written, every wave done with this slot
      // E: dQᵀ tile = Kᵀ dSᵀ over the active groups (+ the earlier blocks' partial sums)
      {
        const int ng = CAUSAL ? min(4, (q0 + HS_BQ - kbase) / 32) : 4;  // active groups: 0 .. ng-1
        f32x16 dq = zero16();
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
          if (gg >= ng) break;
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            const int ro = (32 * gg + 16 * s2) * HS_RB;
            dq = Mma16<T>::mma(trf2(Kimg + ro, toa[dqt], tob[dqt]), trf2(dsimg + ro, toa[qqt], tob[qqt]), dq);
          }
        }
        // F: store (lane = query row qrow, registers 4g4..4g4+3 = d 32dqt + 8g4 + 4hh + 0..3)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          float v0 = dq[4 * g4], v1 = dq[4 * g4 + 1], v2 = dq[4 * g4 + 2], v3 = dq[4 * g4 + 3];
          if (!first) {
            v0 += pp[g4].x;
            v1 += pp[g4].y;
            v2 += pp[g4].z;
            v3 += pp[g4].w;
          }
          if (last) {
            const int d = 32 * dqt + 8 * g4 + 4 * hh;
            v0 *= sc;
            v1 *= sc;
            v2 *= sc;
            v3 *= sc;
            if constexpr (ROPE == 1) {  // R(pos)ᵀ on the pairs (d, d+1), (d+2, d+3)
              const int64_t pos = bp.f.rope_pos ? bp.f.rope_pos[(int64_t)b * N + qrow] : qrow;
              rope_inv4(v0, v1, v2, v3, rope, pos, d);
            }
            store4<T>(dQp + (int64_t)qrow * bp.dq_sn + d, make_float4(v0, v1, v2, v3));
          } else {
            *reinterpret_cast<float4*>(part + qrow * HS_D + 8 * g4) = make_float4(v0, v1, v2, v3);
          }
        }
      }
      // G: the slice two items ahead into this item's (now free) slot
      int ndma = 0;
      {
        int kb2 = kb, s2 = s;
        advance(kb2, s2);
        advance(kb2, s2);
        if (kb2 < nkb) {
          issue_slot(s2, slot);
          ndma = HS_SLICE_DMA + (wave == 0 ? 1 : 0);
        }
      }
      nwait = 4 + ndma;
    }
    // H: the next block's K image and V in flight first, then this block's dK, dV stores (the wait
    // for their RoPE coefficient loads also covers those), then drain
    if (kb + 1 < nkb) {
      dma_barrier();  // every wave done reading the K image
      dk_.issue(Kp + (int64_t)(kb + 1) * HS_KB * k_sn, HS_KB, k_sn, Kimg, wave);
      load_v(kb + 1);
    }
    store_kv(kb);
    if (kb + 1 < nkb) {
      zero_kv();
      wait_vmcnt<0>();
      dma_barrier();
      nwait = 63;
    }
  }
}

template <typename T, bool C, int R>
void launch_hs(const AttnBwdParams& bp, float* rowc, float* part, hipStream_t s) {
  const int BH = bp.f.B * bp.f.H, N = bp.f.Nq;
  // (the in-store RoPE option keeps the prep kernel: with both it needs more than 256 registers)
  if constexpr (R != 1) {
    if (N <= HS_MAXN && hs_in_kernel_delta()) {
      hipLaunchKernelGGL((fa_bwd_hs_kernel<T, C, R, true>), dim3((unsigned)BH), dim3(256), 0, s, bp, rowc, part);
      return;
    }
  }
  hipLaunchKernelGGL((fa_bwd_hs_prep<T>), dim3((unsigned)(BH * (N / HS_BQ))), dim3(256), 0, s, bp, rowc);
  hipLaunchKernelGGL((fa_bwd_hs_kernel<T, C, R, false>), dim3((unsigned)BH), dim3(256), 0, s, bp, rowc, part);
}

template <typename T>
void dispatch_hs(const AttnBwdParams& bp, float* rowc, float* part, bool rope_dq, hipStream_t s) {
  const int rope = bp.f.rope_cos == nullptr ? 0 : (rope_dq ? 1 : 2);
  if (bp.f.causal) {
    if (rope == 1) launch_hs<T, true, 1>(bp, rowc, part, s);
    else if (rope == 2) launch_hs<T, true, 2>(bp, rowc, part, s);
    else launch_hs<T, true, 0>(bp, rowc, part, s);
  } else {
    if (rope == 1) launch_hs<T, false, 1>(bp, rowc, part, s);
    else if (rope == 2) launch_hs<T, false, 2>(bp, rowc, part, s);
    else launch_hs<T, false, 0>(bp, rowc, part, s);
  }
}

}  // namespace fa

// 16-bit, d 64, self-attention with N % 128 == 0; RoPE only in the rope_out_only form (q, k already
// rotated, dq / dk returned w.r.t. the un-rotated inputs); lse contiguous (B, H, N) (the binding
// checks it). Row strides are kept in 32-bit registers and a head's rows addressed with 32-bit
// offsets: each stride must fit int32 and N rows of it stay below 2 GiB.
bool flash_attn_bwd_hs_ok(const AttnBwdParams& bp, DType t) {
  const AttnParams& p = bp.f;
  if (t == DType::F32 || p.D != 64 || p.Nq != p.Nk || p.Nq <= 0 || p.Nq % fa::HS_KB) return false;
  if (p.rope_cos != nullptr && !p.rope_out_only) return false;
  for (int64_t st : {p.q_sn, p.k_sn, p.v_sn, p.o_sn, bp.do_sn, bp.dq_sn, bp.dk_sn, bp.dv_sn})
    if (st <= 0 || st > INT32_MAX || (int64_t)p.Nq * st * 2 >= ((int64_t)1 << 31)) return false;
  return (int64_t)p.B * p.H * p.Nq * fa::HS_D < ((int64_t)1 << 40);
}

size_t flash_attn_bwd_hs_workspace(const AttnBwdParams& bp) {
  const size_t rows = (size_t)bp.f.B * bp.f.H * bp.f.Nq;
  return rows * 2 + (bp.f.Nq > fa::HS_KB ? rows * fa::HS_D : 4);  // floats: row constants + dQ partials
}

void flash_attn_bwd_hs(const AttnBwdParams& bp, DType t, float* ws, hipStream_t s, bool rope_dq) {
  if (bp.f.B * bp.f.H == 0) return;
  float* rowc = ws;
  float* part = ws + (size_t)bp.f.B * bp.f.H * bp.f.Nq * 2;
  if (t == DType::BF16) fa::dispatch_hs<BF16>(bp, rowc, part, rope_dq, s);
  else fa::dispatch_hs<F16>(bp, rowc, part, rope_dq, s);
}

}  // namespace cs336
