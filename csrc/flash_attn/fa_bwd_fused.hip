// FlashAttention-2 backward, fused: ONE kernel, five MFMA products per tile (S, dP, dV, dK, dQ),
// head-sequential, for the many-heads / short-sequence regime of the training step (GPT-2-XL:
// B·H = 1200 heads of N = 512, d 64).
// cs336-build: no-slp
//
// Parity: reference cs336_systems/flash_attention.py:270-289 (a torch.compile'd recompute backward
// over the full N x N matrices). fa_bwd.hip is the general two-kernel form (dQ kernel + dK/dV kernel,
// 7 GEMM-equivalents per tile pair: S and dP are recomputed by both); this one computes them once.
//
// Why head-sequential: the dQ sum runs across key blocks. With one workgroup per key block it needs
// float atomics (≈1.3 TB/s chip-wide, MI355X_MICROARCH.md "Global float atomics"): at N = 512 that
// floor alone (1.5 x the fp32 dQ bytes) is ~180 us per XL layer. Here ONE workgroup owns a whole
// (batch, head) and walks its key blocks in order, so a query slice's dQ is summed in registers
// within a key block and across key blocks through plain fp32 stores/loads of the same lanes (L2
// resident, no atomics, deterministic); the last contributing key block writes dQ (bf16). RoPE, if any, is undone by one
// pass over d(q|k) after this kernel (csrc/bindings.cpp fa_bwd_run): measured faster than a rotating
// store here. With B·H >> 256 CUs the grid still fills the chip (XL: 1200 workgroups, ~4.7 per CU).
//
// Structure (cdna_hip_programming.md "Attention backward"): 8 waves, two per SIMD (≤ 256 registers
// each); key block = 256 keys; wave w owns the 32-key group g = w (w < 4) or 11 - w, so the two
// waves of a SIMD hold groups g and 7 - g (balanced work under the causal mask); each keeps dKᵀ/dVᵀ
// (2 x 32x32 fp32 tiles) and V (MFMA B fragments, key on the lane) in registers and reads K from the
// block's LDS image. The workgroup sweeps 64-row query slices staged by LDS-DMA (3-slot ring,
// prefetched across key-block boundaries), one 32-query tile at a time per wave:
//   S = Q Kᵀ, dP = dO Vᵀ - delta (row constant as the accumulator's start), P = exp2(S c - L),
//   dS = P dP, dVᵀ += dOᵀ P, dKᵀ += Qᵀ dS (accumulators as B operands, Q/dO transposed LDS reads),
//   dSᵀ -> LDS (8-B writes), barrier, then waves 0-3 each form one 32 d x 32 q tile of dQᵀ = Kᵀ dSᵀ
//   over the block's active key groups (both operands transposed reads of the K and dSᵀ images),
//   while waves 4-7 compute the next slice's delta during the first key block.
// delta = rowsum(dO·O) is computed in the first key block's pass (registers prefetched one slice
// ahead) and kept with -lse·log2(e) for the whole head in LDS (N ≤ 1024).
#include "fa_common.h"

namespace cs336 {
namespace fa {

namespace {
constexpr int FD = 64;            // head dim
constexpr int FRB = FD * 2;       // 128-B image rows
constexpr int FBQ = 64;           // query slice
constexpr int FKB = 256;          // keys per block: 4 waves x 2 groups x 32
constexpr int FTILE = FBQ * FRB;  // 8 KiB
constexpr int FSLOT = 2 * FTILE;  // Q, dO images
constexpr int FNS = 3;            // ring depth (slices)
constexpr int FKIMG = FKB * FRB;  // 32 KiB
constexpr int FMAXN = 1024;
// LDS: slice ring 48 KiB | K images 2 x 32 KiB | dSᵀ image 32 KiB | L, delta of the head 2 x 4 KiB
constexpr int OFF_K = FNS * FSLOT;
constexpr int OFF_DS = OFF_K + 2 * FKIMG;
constexpr int OFF_L = OFF_DS + FKB * FRB;
constexpr int OFF_D = OFF_L + FMAXN * 4;
constexpr int FLDS = OFF_D + FMAXN * 4;
static_assert(FLDS <= 160 * 1024, "LDS budget");
}  // namespace

template <typename T, bool CAUSAL>
__global__ __launch_bounds__(512, 1) void fa_bwd_fused_kernel(const AttnBwdParams bp) {
  typedef typename Elem<T>::storage S;
  typedef typename Mma16<T>::frag F;
  __shared__ __attribute__((aligned(1024))) char smem[FLDS];

  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  const int l32 = lane & 31, hh = lane >> 5;
  const int bh = blockIdx.x, b = bh / bp.f.H, h = bh % bp.f.H;
  const int N = bp.f.Nq;  // == Nk, N % 64 == 0, N <= FMAXN (host-checked)
  const int nqs = N / FBQ, nkb = (N + FKB - 1) / FKB;
  // row strides in elements, 32-bit (host-checked): fewer scalar registers than the int64 params
  const int q_sn = (int)bp.f.q_sn, k_sn = (int)bp.f.k_sn, v_sn = (int)bp.f.v_sn, o_sn = (int)bp.f.o_sn;
  const int do_sn = (int)bp.do_sn, dq_sn = (int)bp.dq_sn, dk_sn = (int)bp.dk_sn, dv_sn = (int)bp.dv_sn;
  const S* Qp = (const S*)bp.f.q + b * bp.f.q_sb + h * bp.f.q_sh;
  const S* Kp = (const S*)bp.f.k + b * bp.f.k_sb + h * bp.f.k_sh;
  const S* Vp = (const S*)bp.f.v + b * bp.f.v_sb + h * bp.f.v_sh;
  const S* Op = (const S*)bp.f.o + b * bp.f.o_sb + h * bp.f.o_sh;
  const S* dOp = (const S*)bp.dout + b * bp.do_sb + h * bp.do_sh;
  const float sc = bp.f.scale, c2 = bp.f.scale * kLog2e;

  float* Lh = reinterpret_cast<float*>(smem + OFF_L);  // -lse·log2(e), row_perm order per slice
  float* Dh = reinterpret_cast<float*>(smem + OFF_D);  // -delta, same order
  char* dsimg = smem + OFF_DS;                         // dSᵀ [key][query] of the current slice

  // ---- per-lane LDS offsets. Every fragment's row base is a multiple of 16 rows, so the XOR
  // swizzle of its rows depends on the lane only and the base is an immediate offset:
  // row fragments (A/B operand with the image row on the lane): rows 32t + l32, chunk 2ks + hh
  const int swl = swz<FRB>(l32);
  uint32_t roff[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) roff[ks] = l32 * FRB + (((2 * ks + hh) ^ swl) << 4);
  // transposed fragments (ds_read_b64_tr_b16, see lds_tr_frag): rows 16s + tra (+8), column tile dt
  const int ti = lane & 15, tra = 4 * hh + (ti >> 2), tcl = ((lane >> 4) & 1) * 2 + ((ti & 3) >> 1);
  const int swa = swz<FRB>(tra), swb = swz<FRB>(tra + 8);
  uint32_t toa[2], tob[2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    toa[dt] = tra * FRB + ((((dt << 2) | tcl) ^ swa) << 4) + (ti & 1) * 8;
    tob[dt] = (tra + 8) * FRB + ((((dt << 2) | tcl) ^ swb) << 4) + (ti & 1) * 8;
  }
  auto rowf = [&](const char* img, int ks) -> F {
    return as_frag<T>(*reinterpret_cast<const uint4*>(img + roff[ks]));
  };
  auto trf2 = [&](const char* img, uint32_t oa, uint32_t ob) -> F {
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + oa));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + ob));
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    s16x8 v;
    v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
    v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
    return __builtin_bit_cast(F, v);
  };
  auto trf = [&](const char* img, int dt) -> F { return trf2(img, toa[dt], tob[dt]); };

  // ---- LDS-DMA: wave-instruction i of a tile moves rows 64i + 8 wave + (lane>>3), physical chunk
  // lane&7 (source chunk XOR-swizzled; the swizzle of those rows is independent of i): one lane
  // offset per operand, the row group in the scalar offset
  const int dr = 8 * wave + (lane >> 3), dcs = ((lane & 7) ^ swz<FRB>(dr)) * 8;
  const uint32_t vq = (uint32_t)((dr * q_sn + dcs) * 2), vd = (uint32_t)((dr * do_sn + dcs) * 2),
                 vk = (uint32_t)((dr * k_sn + dcs) * 2);
  const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc((void*)Qp, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)dOp, (short)0, 0x7fffffff, 0x00020000);
  auto issue_slot = [&](int s, int slot) {  // one wave-instruction each of the slice's Q and dO
    char* base = smem + slot * FSLOT + 1024 * wave;
    dma16(rq, lds_addr(base), vq, (uint32_t)(s * FBQ * q_sn * 2));
    dma16(rd, lds_addr(base + FTILE), vd, (uint32_t)(s * FBQ * do_sn * 2));
  };
  auto issue_k = [&](int kb) {  // rows past N read out of the descriptor's range (never used)
    const int rows = min(FKB, N - kb * FKB);
    const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(Kp + (int64_t)kb * FKB * k_sn), (short)0, ((rows - 1) * k_sn + FD) * 2, 0x00020000);
    char* base = smem + OFF_K + (kb & 1) * FKIMG + 1024 * wave;
#pragma unroll
    for (int i = 0; i < 4; ++i) dma16(rk, lds_addr(base + 8192 * i), vk, (uint32_t)(64 * i * k_sn * 2));
  };
  auto sbeg = [&](int kb) { return CAUSAL ? kb * (FKB / FBQ) : 0; };
  auto advance = [&](int& kb, int& s) {
    if (++s >= nqs) {
      ++kb;
      s = sbeg(kb);
    }
  };

  // delta = rowsum(dO·O) of one slice, by waves 4-7 while waves 0-3 run the dQ product: thread
  // (row (tid-256)>>2, 16 d of quarter tid&3)
  auto prep = [&](int s) {
    const int pt = tid & 255, row = s * FBQ + (pt >> 2), e = 16 * (pt & 3);
    uint4 pd[2], po[2];
    pd[0] = *reinterpret_cast<const uint4*>(dOp + row * do_sn + e);
    pd[1] = *reinterpret_cast<const uint4*>(dOp + row * do_sn + e + 8);
    po[0] = *reinterpret_cast<const uint4*>(Op + row * o_sn + e);
    po[1] = *reinterpret_cast<const uint4*>(Op + row * o_sn + e + 8);
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const uint32_t a[4] = {pd[i].x, pd[i].y, pd[i].z, pd[i].w};
      const uint32_t c[4] = {po[i].x, po[i].y, po[i].z, po[i].w};
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        acc = fmaf(Elem<T>::to_f((S)(a[w] & 0xffff)), Elem<T>::to_f((S)(c[w] & 0xffff)), acc);
        acc = fmaf(Elem<T>::to_f((S)(a[w] >> 16)), Elem<T>::to_f((S)(c[w] >> 16)), acc);
      }
    }
    acc += __shfl_xor(acc, 1, 64);
    acc += __shfl_xor(acc, 2, 64);
    if ((pt & 3) == 0) Dh[s * FBQ + row_perm(pt >> 2)] = -acc;
  };

  // ---- per-wave state: one 32-key group of the current key block. SIMD partners (waves w, w+4)
  // hold groups g and 7 - g, so the causal work per SIMD is balanced
  const int g = wave < 4 ? wave : 11 - wave;
  uint4 vf[4];             // V B fragments (key on the lane): d = 16i + 8hh .. +7
  f32x16 dk[2], dv[2];     // dKᵀ, dVᵀ per d tile: lane = key, registers = d
  // V from global, rows clamped: keys past N only occur as whole inactive groups (N % 32 == 0),
  // never multiplied (a zeroing branch here crashed hipcc 7.2's machine copy propagation)
  auto load_v = [&](int kb) {
    const int key = min(kb * FKB + 32 * g + l32, N - 1);
#pragma unroll
    for (int i = 0; i < 4; ++i) vf[i] = *reinterpret_cast<const uint4*>(Vp + key * v_sn + 16 * i + 8 * hh);
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      dk[dt] = zero16();
      dv[dt] = zero16();
    }
  };
  auto store_kv = [&](int kb) {
    const int key = kb * FKB + 32 * g + l32;
    if (key >= N) return;
    S* rk = (S*)bp.dk + b * bp.dk_sb + h * bp.dk_sh + key * dk_sn;
    S* rv = (S*)bp.dv + b * bp.dv_sb + h * bp.dv_sh + key * dv_sn;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = 32 * dt + 8 * g4 + 4 * hh;
        store4<T>(rk + d, make_float4(dk[dt][4 * g4] * sc, dk[dt][4 * g4 + 1] * sc, dk[dt][4 * g4 + 2] * sc,
                                      dk[dt][4 * g4 + 3] * sc));
        store4<T>(rv + d, make_float4(dv[dt][4 * g4], dv[dt][4 * g4 + 1], dv[dt][4 * g4 + 2], dv[dt][4 * g4 + 3]));
      }
  };

  // ---- dQ (waves 0-3): tile d rows 32 dqt.., queries 32 qqt.. ---------------------------------
  const bool dqw = wave < 4;
  const int dqt = wave & 1, qqt = (wave >> 1) & 1;
  const uint32_t kqa = dqt ? toa[1] : toa[0], kqb = dqt ? tob[1] : tob[0];
  const uint32_t dsa = qqt ? toa[1] : toa[0], dsb = qqt ? tob[1] : tob[0];
  float* part = bp.dq_acc + (int64_t)bh * N * FD + 32 * dqt + 4 * hh;  // + q * 64: fp32 partial sums

  // ---- prologue: L of the head, K image 0, slices of items 0 and 1, V of block 0, delta slice 0 ---
  for (int r0 = 4 * tid; r0 < N; r0 += 2048) {
    const float4 l = *reinterpret_cast<const float4*>(bp.f.lse + (int64_t)bh * N + r0);
    *reinterpret_cast<float4*>(Lh + (r0 & ~63) + row_perm(r0 & 63)) =
        make_float4(-l.x * kLog2e, -l.y * kLog2e, -l.z * kLog2e, -l.w * kLog2e);
  }
  issue_k(0);
  {
    int kb1 = 0, s1 = 0;
    issue_slot(0, 0);
    advance(kb1, s1);
    if (kb1 < nkb) issue_slot(s1, 1);
  }
  load_v(0);
  if (wave >= 4) prep(0);
  wait_vmcnt<0>();
  dma_barrier();

  // ---- the walk --------------------------------------------------------------------------------
  int it = 0;
  for (int kb = 0; kb < nkb; ++kb) {
    const int kbase = kb * FKB;
    const char* Kimg = smem + OFF_K + (kb & 1) * FKIMG;
    const int k0g = kbase + 32 * g;
    for (int s = sbeg(kb); s < nqs; ++s, ++it) {
      const int slot = it % FNS;
      const char* Qs = smem + slot * FSLOT;
      const char* dOs = Qs + FTILE;
      const int q0 = s * FBQ;
      // A: this item's slice landed. dQ waves: every item in flight after it issued >= 8 later
      // vector memory operations (two items' dQ stores); the other waves wait for all of theirs
      // (their newest, the next slice's DMA, was issued an item ago). The prologue and the
      // key-block switch drain to 0. The barrier also orders the previous item's dSᵀ reads.
      if (dqw) {
        if (it >= 2) wait_vmcnt<8>();
      } else {
        wait_vmcnt<0>();
      }
      dma_barrier();
      // B: the slice two items ahead
      {
        int kb2 = kb, s2 = s;
        advance(kb2, s2);
        advance(kb2, s2);
        if (kb2 < nkb) issue_slot(s2, (it + 2) % FNS);
      }
      // C: the next key block's K image, behind the whole block
      if (s == sbeg(kb) && kb + 1 < nkb) issue_k(kb + 1);
      // D: this wave's dQ partial sums from the earlier key blocks (L2), loaded here so their latency
      // runs under the S/dP work instead of in front of the dQ product
      const int kb_last = CAUSAL ? min((q0 + FBQ - 1) / FKB, nkb - 1) : nkb - 1;
      const bool first = kb == 0, last = kb == kb_last;
      const int qrow = q0 + 32 * qqt + l32;
      float4 pp[4];
      if (dqw && !first) {
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) pp[g4] = *reinterpret_cast<const float4*>(part + qrow * FD + 8 * g4);
      }
      const bool do_prep = first && s + 1 < nqs;  // next slice's delta (first key block only)

      // F: S, dP, P, dS, dVᵀ, dKᵀ of this wave's group; dSᵀ into LDS
      if (k0g < N && (!CAUSAL || k0g <= q0 + FBQ - 1)) {
        const bool diag = CAUSAL && k0g + 31 > q0;
        const char* Kg = Kimg + 32 * g * FRB;
        F kfr[4];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) kfr[ks] = rowf(Kg, ks);
        const int kq = k0g + l32 - q0 - 4 * hh;  // key - (query of register 0 of this half)
        char* drow = dsimg + (32 * g + l32) * FRB + 8 * hh;
        const float* Ls = Lh + q0;
        const float* Ds = Dh + q0;
        // one 32-query tile at a time: S, dP (32 x 32 each), P, dS, then dVᵀ/dKᵀ over its queries
        // (a loop, not unrolled: the registers of one tile leave room to keep fragment reads in flight)
#pragma nounroll
        for (int t = 0; t < 2; ++t) {
          // all eight row fragments of the tile first, then the 8 MFMAs (the counted lgkmcnt waits
          // then overlap the reads with the chain instead of one read latency per MFMA)
          const char* Qt = Qs + 32 * t * FRB;
          const char* dOt = dOs + 32 * t * FRB;
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
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {
            const float4 L4 = *reinterpret_cast<const float4*>(Ls + 32 * t + 16 * hh + 4 * g4);
            const float Lv[4] = {L4.x, L4.y, L4.z, L4.w};
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int r = 4 * g4 + u;
              float pv = fexp2(fmaf(sa[r], c2, Lv[u]));
              if (diag && kq > 32 * t + 8 * g4 + u) pv = 0.f;
              sa[r] = pv;
              dp[r] = pv * dp[r];
            }
          }
          F pf[2], sf[2];
          pf[0] = pack_acc<T>(sa, 0);
          pf[1] = pack_acc<T>(sa, 1);
          sf[0] = pack_acc<T>(dp, 0);
          sf[1] = pack_acc<T>(dp, 1);
          F ot[2][2], qt[2][2];  // dOᵀ, Qᵀ fragments [s2][dt]
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int dt = 0; dt < 2; ++dt) ot[s2][dt] = trf(dOt + 16 * s2 * FRB, dt);
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int dt = 0; dt < 2; ++dt) qt[s2][dt] = trf(Qt + 16 * s2 * FRB, dt);
          #pragma unroll
          for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int dt = 0; dt < 2; ++dt) dv[dt] = Mma16<T>::mma(ot[s2][dt], pf[s2], dv[dt]);
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int dt = 0; dt < 2; ++dt) dk[dt] = Mma16<T>::mma(qt[s2][dt], sf[s2], dk[dt]);
          // dSᵀ row (block-local key 32g + l32, swizzle swl): the fragment's two 4-query halves are
          // q = 32t + 16s2 + 4hh + 0..3 and the same + 8 (pack_acc order), one 8-B write each
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            const uint4 w = __builtin_bit_cast(uint4, sf[s2]);
            const int ch = 4 * t + 2 * s2;
            *reinterpret_cast<uint2*>(drow + ((ch ^ swl) << 4)) = make_uint2(w.x, w.y);
            *reinterpret_cast<uint2*>(drow + (((ch + 1) ^ swl) << 4)) = make_uint2(w.z, w.w);
          }
        }
      }
      dma_barrier();  // dSᵀ of every group written

      // G: dQᵀ tile = Kᵀ dSᵀ over the active groups (+ the earlier blocks' partial sum), waves 0-3
      // (splitting it over all eight waves with a partial-tile hand-off through LDS, or reading all
      // fragments ahead of the MFMAs, measured slower: profiles/r3_fa_bwd_fused_ab.md)
      if (dqw) {
        const int ng = CAUSAL ? min(8, (q0 + FBQ - kbase) / 32) : 8;  // active groups: 0 .. ng-1
        const int nv = min(ng, (N - kbase) / 32);
        f32x16 dq = zero16();
#pragma unroll
        for (int gg = 0; gg < 8; ++gg) {
          if (gg >= nv) break;
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            const int ro = (32 * gg + 16 * s2) * FRB;
            dq = Mma16<T>::mma(trf2(Kimg + ro, kqa, kqb), trf2(dsimg + ro, dsa, dsb), dq);
          }
        }
        // H: store (lane = query row qrow, registers 4g4..4g4+3 = d 32dqt + 8g4 + 4hh + 0..3)
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
            S* dQp = (S*)bp.dq + b * bp.dq_sb + h * bp.dq_sh;
            store4<T>(dQp + qrow * dq_sn + d, make_float4(v0 * sc, v1 * sc, v2 * sc, v3 * sc));
          } else {
            *reinterpret_cast<float4*>(part + qrow * FD + 8 * g4) = make_float4(v0, v1, v2, v3);
          }
        }
      } else if (do_prep) {
        prep(s + 1);  // I: the next slice's delta (published by the next item's barrier)
      }
    }
    // J: this key block's dK, dV; switch to the next block (drain: its K image, the ring)
    store_kv(kb);
    if (kb + 1 < nkb) {
      load_v(kb + 1);
      wait_vmcnt<0>();
      dma_barrier();
    }
  }
}

template <typename T, bool C>
void launch_fused_c(const AttnBwdParams& bp, hipStream_t s) {
  const dim3 grid((unsigned)(bp.f.B * bp.f.H)), block(512);
  hipLaunchKernelGGL((fa_bwd_fused_kernel<T, C>), grid, block, 0, s, bp);
}

}  // namespace fa

bool flash_attn_bwd_fused_ok(const AttnBwdParams& bp, DType t) {
  const AttnParams& p = bp.f;
  if (!(t != DType::F32 && p.D == 64 && p.Nq == p.Nk && p.Nq % 64 == 0 && p.Nq > 0 && p.Nq <= fa::FMAXN &&
        p.rope_cos == nullptr && bp.dq_acc != nullptr))
    return false;
  // the kernel keeps row strides in 32-bit registers and addresses a head's rows with 32-bit DMA
  // offsets (s·64·stride·2 B): every row stride must fit int32 and N rows of it stay below 2 GiB
  // (lse (B, H, N) contiguity is checked by the binding)
  for (int64_t st : {p.q_sn, p.k_sn, p.v_sn, p.o_sn, bp.do_sn, bp.dq_sn, bp.dk_sn, bp.dv_sn})
    if (st <= 0 || st > INT32_MAX || (int64_t)p.Nq * st * 2 >= ((int64_t)1 << 31)) return false;
  return true;
}

void flash_attn_bwd_fused(const AttnBwdParams& bp, DType t, hipStream_t s) {
  if (bp.f.B * bp.f.H == 0) return;
  if (t == DType::BF16) {
    if (bp.f.causal) fa::launch_fused_c<BF16, true>(bp, s);
    else fa::launch_fused_c<BF16, false>(bp, s);
  } else {
    if (bp.f.causal) fa::launch_fused_c<F16, true>(bp, s);
    else fa::launch_fused_c<F16, false>(bp, s);
  }
}

}  // namespace cs336
