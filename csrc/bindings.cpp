// torch.ops.cs336.* registration for the MI355X HIP kernels.
//
// Pure TORCH_LIBRARY (no Python headers): the shared library is loaded with
// torch.ops.load_library, and every op gets a fake impl in cs336_systems/ops/_fake.py so
// torch.compile can trace through the autograd Functions. Kernels run on the current HIP stream
// of the tensors' device; nothing here synchronizes the host.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <c10/core/DeviceGuard.h>
#include <torch/library.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "cs336/kernels.h"
#include "../gemm/gemm8.h"

namespace {

using cs336::DType;

DType to_dtype(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return DType::F32;
    case at::kBFloat16: return DType::BF16;
    case at::kHalf: return DType::F16;
    default: TORCH_CHECK(false, "cs336: unsupported dtype ", t.scalar_type());
  }
  return DType::F32;
}

hipStream_t stream() { return at::hip::getCurrentHIPStream(); }

void check_cuda(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "cs336: ", name, " must be a GPU tensor");
}

// ------------------------------------------------------------------------------------------
// FlashAttention
// ------------------------------------------------------------------------------------------
void check_bhnd(const at::Tensor& t, const char* name) {
  check_cuda(t, name);
  TORCH_CHECK(t.dim() == 4, "cs336: ", name, " must be (B, H, N, D)");
  TORCH_CHECK(t.stride(3) == 1, "cs336: ", name, " must have a contiguous last dim");
  const int D = (int)t.size(3);
  TORCH_CHECK(D == 32 || D == 64 || D == 128 || ((D == 80 || D == 16) && t.element_size() == 2),
              "cs336: head dim must be 32, 64, 128, or 16 / 80 for 16-bit inputs (got ", D, ")");
  const int64_t es = t.element_size();
  TORCH_CHECK((reinterpret_cast<uintptr_t>(t.data_ptr()) % 16) == 0, "cs336: ", name, " must be 16-byte aligned");
  TORCH_CHECK((t.stride(2) * es) % 16 == 0 && (t.stride(1) * es) % 16 == 0 && (t.stride(0) * es) % 16 == 0,
              "cs336: ", name, " strides must be multiples of 16 bytes");
}

// (B,H,N,D) view of freshly allocated (B,N,H,D) memory
at::Tensor empty_bnhd_like(const at::Tensor& q) {
  return at::empty({q.size(0), q.size(2), q.size(1), q.size(3)}, q.options()).permute({0, 2, 1, 3});
}

void fill_attn(cs336::AttnParams& p, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
               const at::Tensor& o, const at::Tensor& lse, bool causal, double scale) {
  p.q = q.data_ptr();
  p.k = k.data_ptr();
  p.v = v.data_ptr();
  p.o = o.data_ptr();
  p.lse = lse.data_ptr<float>();
  p.q_sb = q.stride(0); p.q_sh = q.stride(1); p.q_sn = q.stride(2);
  p.k_sb = k.stride(0); p.k_sh = k.stride(1); p.k_sn = k.stride(2);
  p.v_sb = v.stride(0); p.v_sh = v.stride(1); p.v_sn = v.stride(2);
  p.o_sb = o.stride(0); p.o_sh = o.stride(1); p.o_sn = o.stride(2);
  p.B = (int)q.size(0);
  p.H = (int)q.size(1);
  p.Nq = (int)q.size(2);
  p.Nk = (int)k.size(2);
  p.D = (int)q.size(3);
  p.scale = (float)scale;
  p.causal = causal;
  // CS336_FA_ORDER=0 restores the per-head interleaved block order (A/B switch for tile_order)
  static const int order = [] {
    const char* e = std::getenv("CS336_FA_ORDER");
    return e ? std::atoi(e) : 1;
  }();
  p.order = order;
  // heads whose K+V fit one XCD's 4 MB L2 form one level-major group (tile_order, fa_common.h)
  const int64_t kv_head = 2 * (int64_t)p.Nk * p.D * (int64_t)q.element_size();
  p.lpt_group = (int)std::max<int64_t>(1, std::min<int64_t>(1 << 20, (int64_t(4) << 20) / std::max<int64_t>(kv_head, 1)));
  // LDS-DMA staging (fa_common.h TileDma), measured per kernel (scripts/fa_ab.py): with the DMA
  // loop unrolled by its ring depth the forward gains everywhere except causal at short N (d64 causal
  // N 4096 +7.5 %, d80 causal N 1024 +5 %, d64 causal N 512 -1.3 %, profiles/r2_fa_bwd_valu.md); the
  // backward kernels lose 2-7 % (their time is not in the tile loads). CS336_FA_DMA: unset = that
  // choice, 0 = never, 1 = every forward, 2 = forward and backward.
  const int dma_env = [] {  // read per call (cheap next to a launch): tests switch it in-process
    const char* e = std::getenv("CS336_FA_DMA");
    return e && *e ? std::atoi(e) : -1;
  }();
  // 4: the forward's pipelined variant (separate K/V rings, next S^T inside this tile's softmax)
  // backward (bit 2): with the dQ / dK-dV DMA loops unrolled by their ring depth LDS-DMA staging
  // wins at Nk >= 1024 (d 64 +5 %, d 128 +5-10 %, d 80 even); it loses 2 % at the XL step's N 512
  // (profiles/r2_fa_bwd_valu.md)
  // (since the resident-fragment wait hint, profiles/r3_fa_vmcnt_hint.md, the LDS-DMA forward also
  // wins at the XL step's causal N 512: 0.1306-0.1313 vs 0.1343-0.1357 ms, so it is every forward)
  if (dma_env < 0) p.dma = 1 | (p.Nk >= 1024 ? 2 : 0);
  else if (dma_env == 4) p.dma = 1 | 4;
  else p.dma = dma_env == 0 ? 0 : (dma_env == 1 ? 1 : 3);
}

using OptT = std::optional<at::Tensor>;

// fused RoPE: q/k are the un-rotated projections; cos/sin (ctx, D/2) fp32, pos (B, N) int64 or None
void set_rope(cs336::AttnParams& p, const at::Tensor& q, const at::Tensor& k, const OptT& cos, const OptT& sin,
              const OptT& pos) {
  if (!cos.has_value() || !cos->defined()) return;
  TORCH_CHECK(sin.has_value() && sin->defined(), "cs336: rope needs cos and sin");
  TORCH_CHECK(cos->scalar_type() == at::kFloat && cos->is_contiguous() && sin->is_contiguous() &&
                  cos->size(1) * 2 == q.size(3),
              "cs336: rope cache must be contiguous fp32 (ctx, D/2)");
  TORCH_CHECK(q.size(2) == k.size(2), "cs336: fused rope is for self-attention (Nq == Nk)");
  if (pos.has_value() && pos->defined()) {
    TORCH_CHECK(pos->scalar_type() == at::kLong && pos->is_contiguous() && pos->numel() == q.size(0) * q.size(2),
                "cs336: rope positions must be contiguous int64 (B, N)");
    p.rope_pos = pos->data_ptr<int64_t>();
  } else {
    TORCH_CHECK(q.size(2) <= cos->size(0), "cs336: sequence longer than the RoPE cache");
  }
  p.rope_cos = cos->data_ptr<float>();
  p.rope_sin = sin->data_ptr<float>();
}

std::tuple<at::Tensor, at::Tensor> fa_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, bool causal,
                                          double scale, const OptT& rope_cos, const OptT& rope_sin,
                                          const OptT& rope_pos) {
  check_bhnd(q, "q");
  check_bhnd(k, "k");
  check_bhnd(v, "v");
  TORCH_CHECK(q.scalar_type() == k.scalar_type() && q.scalar_type() == v.scalar_type(), "cs336: q/k/v dtype mismatch");
  TORCH_CHECK(k.sizes() == v.sizes(), "cs336: k/v shape mismatch");
  TORCH_CHECK(q.size(0) == k.size(0) && q.size(1) == k.size(1) && q.size(3) == k.size(3), "cs336: q/k shape mismatch");
  c10::DeviceGuard g(q.device());
  at::Tensor o = empty_bnhd_like(q);
  at::Tensor lse = at::empty({q.size(0), q.size(1), q.size(2)}, q.options().dtype(at::kFloat));
  cs336::AttnParams p;
  fill_attn(p, q, k, v, o, lse, causal, scale);
  set_rope(p, q, k, rope_cos, rope_sin, rope_pos);
  // split-KV when the query blocks cannot fill the chip (CS336_FA_SPLITS=n forces n, 1 = off)
  const int force_splits = [] {  // read per call (cheap next to a launch): tests switch it in-process
    const char* e = std::getenv("CS336_FA_SPLITS");
    return e && *e ? std::atoi(e) : 0;
  }();
  const int splits = force_splits > 0 ? force_splits : cs336::flash_attn_fwd_splits(p);
  at::Tensor ws;
  if (splits > 1) {
    ws = at::empty({(int64_t)cs336::flash_attn_fwd_split_workspace(p, splits)}, q.options().dtype(at::kFloat));
    p.kv_splits = splits;
    p.opart = ws.data_ptr<float>();
    p.lpart = p.opart + (int64_t)splits * p.B * p.H * p.Nq * p.D;
  }
  cs336::flash_attn_fwd(p, to_dtype(q), stream());
  return {o, lse};
}

// forward that also writes Oᵀ as a (H*D, B*Nq) token-contiguous matrix (no RoPE-on-load)
std::tuple<at::Tensor, at::Tensor, at::Tensor> fa_fwd_ot(const at::Tensor& q, const at::Tensor& k,
                                                         const at::Tensor& v, bool causal, double scale) {
  check_bhnd(q, "q");
  check_bhnd(k, "k");
  check_bhnd(v, "v");
  TORCH_CHECK(q.scalar_type() == k.scalar_type() && q.scalar_type() == v.scalar_type(), "cs336: q/k/v dtype mismatch");
  TORCH_CHECK(q.element_size() == 2, "cs336: fa_fwd_ot is 16-bit only");
  TORCH_CHECK(k.sizes() == v.sizes(), "cs336: k/v shape mismatch");
  TORCH_CHECK(q.size(0) == k.size(0) && q.size(1) == k.size(1) && q.size(3) == k.size(3), "cs336: q/k shape mismatch");
  c10::DeviceGuard g(q.device());
  at::Tensor o = empty_bnhd_like(q);
  at::Tensor lse = at::empty({q.size(0), q.size(1), q.size(2)}, q.options().dtype(at::kFloat));
  at::Tensor ot = at::empty({q.size(1) * q.size(3), q.size(0) * q.size(2)}, q.options());
  cs336::AttnParams p;
  fill_attn(p, q, k, v, o, lse, causal, scale);
  p.ot = ot.data_ptr();
  p.ot_ld = ot.size(1);
  cs336::flash_attn_fwd(p, to_dtype(q), stream());
  return {o, lse, ot};
}

void rope_into(const at::Tensor& x, const at::Tensor& cos, const at::Tensor& sin, const std::optional<at::Tensor>& pos,
               bool inverse, const at::Tensor& out);
void fa_bwd_run(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                const at::Tensor& out, const at::Tensor& lse, bool causal, double scale, const at::Tensor& dq,
                const at::Tensor& dk, const at::Tensor& dv, const OptT& rope_cos, const OptT& rope_sin,
                const OptT& rope_pos, bool rope_out_only = false);

void check_bwd_inputs(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                      const at::Tensor& out, const at::Tensor& lse) {
  check_bhnd(q, "q");
  check_bhnd(k, "k");
  check_bhnd(v, "v");
  check_bhnd(out, "out");
  check_bhnd(dout, "dout");
  TORCH_CHECK(lse.is_contiguous() && lse.scalar_type() == at::kFloat, "cs336: lse must be contiguous fp32");
  TORCH_CHECK(dout.scalar_type() == q.scalar_type() && out.scalar_type() == q.scalar_type(), "cs336: dtype mismatch");
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> fa_bwd(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k,
                                                      const at::Tensor& v, const at::Tensor& out,
                                                      const at::Tensor& lse, bool causal, double scale,
                                                      const OptT& rope_cos, const OptT& rope_sin,
                                                      const OptT& rope_pos) {
  check_bwd_inputs(dout, q, k, v, out, lse);
  c10::DeviceGuard g(q.device());
  at::Tensor dq = empty_bnhd_like(q);
  at::Tensor dk = empty_bnhd_like(k);
  at::Tensor dv = empty_bnhd_like(v);
  fa_bwd_run(dout, q, k, v, out, lse, causal, scale, dq, dk, dv, rope_cos, rope_sin, rope_pos);
  return {dq, dk, dv};
}

// backward writing dq/dk/dv into caller-provided (B,H,N,D) strided views (e.g. the three slices of
// one fused dQKV buffer that feeds the fused QKV-projection GEMM)
void fa_bwd_into(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                 const at::Tensor& out, const at::Tensor& lse, bool causal, double scale, const at::Tensor& dq,
                 const at::Tensor& dk, const at::Tensor& dv, const OptT& rope_cos, const OptT& rope_sin,
                 const OptT& rope_pos, bool rope_out_only) {
  check_bwd_inputs(dout, q, k, v, out, lse);
  check_bhnd(dq, "dq");
  check_bhnd(dk, "dk");
  check_bhnd(dv, "dv");
  TORCH_CHECK(dq.sizes() == q.sizes() && dk.sizes() == k.sizes() && dv.sizes() == v.sizes(), "cs336: grad shapes");
  TORCH_CHECK(dq.scalar_type() == q.scalar_type() && dk.scalar_type() == q.scalar_type() &&
                  dv.scalar_type() == q.scalar_type(),
              "cs336: dtype mismatch");
  c10::DeviceGuard g(q.device());
  fa_bwd_run(dout, q, k, v, out, lse, causal, scale, dq, dk, dv, rope_cos, rope_sin, rope_pos, rope_out_only);
}

void fa_bwd_run(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                const at::Tensor& out, const at::Tensor& lse, bool causal, double scale, const at::Tensor& dq,
                const at::Tensor& dk, const at::Tensor& dv, const OptT& rope_cos, const OptT& rope_sin,
                const OptT& rope_pos, bool rope_out_only) {
  cs336::AttnBwdParams bp;
  fill_attn(bp.f, q, k, v, out, lse, causal, scale);
  set_rope(bp.f, q, k, rope_cos, rope_sin, rope_pos);
  bp.f.rope_out_only = rope_out_only && bp.f.rope_cos != nullptr;
  bp.dout = dout.data_ptr();
  bp.do_sb = dout.stride(0); bp.do_sh = dout.stride(1); bp.do_sn = dout.stride(2);
  bp.dq = dq.data_ptr();
  bp.dk = dk.data_ptr();
  bp.dv = dv.data_ptr();
  bp.dq_sb = dq.stride(0); bp.dq_sh = dq.stride(1); bp.dq_sn = dq.stride(2);
  bp.dk_sb = dk.stride(0); bp.dk_sh = dk.stride(1); bp.dk_sn = dk.stride(2);
  bp.dv_sb = dv.stride(0); bp.dv_sh = dv.stride(1); bp.dv_sn = dv.stride(2);
  // CS336_FA_BWD selects the backward:
  //   unset: a head-sequential kernel where it applies and the (batch, head) workgroups fill the chip
  //          (B·H >= 512): fa_bwd_hs.hip (d 64, N <= 1024, N % 128 == 0), else fa_bwd_fused.hip
  //          (d 64, N <= 1024: the N % 128 == 64 shapes, 1.37x the two-kernel form,
  //          profiles/r5_fa_bwd_forms.md); else at d 80 and long-N d 64 the key-block-parallel fused
  //          kernel (fa_bwd_kp.hip, dQ by slabs / fp32 atomics), else the two-kernel form (split over keys /
  //          queries at low parallelism);
  //   1: head-sequential wherever it applies (then as unset); 2: key-block parallel wherever it
  //   applies; 0: the two-kernel form (dQ kernel + dK/dV kernel: deterministic, any shape);
  //   3: the two-workgroups-per-CU head-sequential kernel (fa_bwd_hs.hip) where it applies.
  const int mode = [] {
    const char* e = std::getenv("CS336_FA_BWD");
    return e && *e ? std::atoi(e) : -1;
  }();
  const int64_t nbh = q.size(0) * q.size(1);
  // inverse RoPE of d(q|k) as one in-place pass after a kernel that returned them w.r.t. the rotated
  // inputs (dq and dk adjacent head blocks of one buffer -- the fused dQKV layout -- take one launch)
  auto rope_after_pass = [&]() {
    const int64_t es = dq.element_size();
    if (dk.strides() == dq.strides() &&
        static_cast<const char*>(dk.data_ptr()) == static_cast<const char*>(dq.data_ptr()) + dq.size(1) * dq.stride(1) * es) {
      const at::Tensor dqk = dq.as_strided({dq.size(0), 2 * dq.size(1), dq.size(2), dq.size(3)}, dq.strides());
      rope_into(dqk, *rope_cos, *rope_sin, rope_pos, true, dqk);
    } else {
      rope_into(dq, *rope_cos, *rope_sin, rope_pos, true, dq);
      rope_into(dk, *rope_cos, *rope_sin, rope_pos, true, dk);
    }
  };
  // head-sequential with two 4-wave workgroups per CU (fa_bwd_hs.hip): mode 3, and by default for
  // the training step's regime (B·H >= 512, N <= 1024), where it beat the 8-wave fused kernel in the
  // XL step by 2.5-4.3 ms/step on two boxes (profiles/r4_fa_bwd_hs.md). The inverse RoPE runs as the
  // separate pass after it (1.7-3.5 ms/step faster than in its stores). CS336_FA_HS_ROPE: 0 (default)
  // both dQ and dK by the pass, 1 both in the kernel's stores, 2 dK in the kernel (at the key-block
  // switch, where it drains anyway) and dQ by the pass
  if (mode == 3 || (mode < 0 && nbh >= 512 && q.size(2) <= 1024)) {
    const char* re = std::getenv("CS336_FA_HS_ROPE");
    const int hr = re && *re ? std::atoi(re) : 0;
    const bool rope = bp.f.rope_out_only;
    cs336::AttnBwdParams hb = bp;
    if (rope && hr == 0) {
      hb.f.rope_cos = hb.f.rope_sin = nullptr;
      hb.f.rope_pos = nullptr;
      hb.f.rope_out_only = false;
    }
    if (cs336::flash_attn_bwd_hs_ok(hb, to_dtype(q))) {
      at::Tensor ws = at::empty({(int64_t)cs336::flash_attn_bwd_hs_workspace(hb)}, q.options().dtype(at::kFloat));
      cs336::flash_attn_bwd_hs(hb, to_dtype(q), ws.data_ptr<float>(), stream(), hr != 2);
      if (rope && hr == 0) rope_after_pass();
      if (rope && hr == 2) rope_into(dq, *rope_cos, *rope_sin, rope_pos, true, dq);
      return;
    }
  }
  at::Tensor dq_acc;
  if (mode != 0 && mode != 2 && (mode == 1 || nbh >= 512)) {
    // partial sums exist only for rows with more than one 256-key block
    dq_acc = at::empty({q.size(2) > 256 ? nbh * q.size(2) * 64 : 4}, q.options().dtype(at::kFloat));
    bp.dq_acc = dq_acc.data_ptr<float>();
    // RoPE (dQ/dK w.r.t. the un-rotated q, k) as one in-place inverse pass over d(q|k) after the fused
    // kernel: a rotating store inside it measured slower (0.430 vs 0.373 ms at the XL shape in the
    // step's fused-QKV layout, scripts/fa_step_layout.py; profiles/r3_qkv_rope_ab.md)
    const bool rope_after = bp.f.rope_out_only;
    cs336::AttnBwdParams fb = bp;
    if (rope_after) {
      fb.f.rope_cos = fb.f.rope_sin = nullptr;
      fb.f.rope_pos = nullptr;
      fb.f.rope_out_only = false;
    }
    if (cs336::flash_attn_bwd_fused_ok(fb, to_dtype(q))) {
      cs336::flash_attn_bwd_fused(fb, to_dtype(q), stream());
      if (rope_after) rope_after_pass();
      return;
    }
    bp.dq_acc = nullptr;
  }
  // key-block parallel: forced by mode 2; by default at d 80 (the 2.7b model: B 32 H 32 N 1024 causal
  // 1.11 vs 1.35 ms for the two-kernel form, N 4096 617 vs 445 TF) and at d 64 for N >= 2048 with at
  // least 512 key-block workgroups (N 2048 causal even, full 679 vs 654-674 TF; N 4096 causal even,
  // full 744 vs 701; B 1 H 16 N 8192 684-687 vs 652 causal, 755-760 vs 726 full; N 16384 causal 753 vs
  // 719 TF); the 8-wave form, profiles/r6_fa_kp_waves.md. Below that (few heads: the two-kernel form
  // splits keys / queries) and at N <= 1024 (head-sequential forms) it is not the default.
  const bool kp_default = q.size(3) == 80 ||
      (q.size(3) == 64 && q.size(2) >= 2048 && q.size(0) * q.size(1) * ((q.size(2) + 255) / 256) >= 512);
  if ((mode == 2 || (mode < 0 && kp_default)) && cs336::flash_attn_bwd_kp_ok(bp, to_dtype(q))) {
    at::Tensor ws = at::empty({(int64_t)cs336::flash_attn_bwd_kp_workspace(bp)}, q.options().dtype(at::kFloat));
    cs336::flash_attn_bwd_kp(bp, to_dtype(q), ws.data_ptr<float>(), stream());
    return;
  }
  at::Tensor delta = at::empty({2, q.size(0), q.size(1), q.size(2)}, q.options().dtype(at::kFloat));
  bp.delta = delta.data_ptr<float>();
  bp.lrow = bp.delta + q.size(0) * q.size(1) * q.size(2);
  // low parallelism: split the dQ kernel over keys and the dK/dV kernel over queries (fp32 partial
  // slabs + reduce); CS336_FA_BWD_SPLITS=1 turns it off
  int ks = 1, qs = 1;
  const char* se = std::getenv("CS336_FA_BWD_SPLITS");
  if (!(se && *se && std::atoi(se) == 1)) cs336::flash_attn_bwd_splits(bp, ks, qs);
  at::Tensor parts;
  if (ks > 1 || qs > 1) {
    parts = at::empty({(int64_t)cs336::flash_attn_bwd_split_workspace(bp, ks, qs)}, q.options().dtype(at::kFloat));
    float* w = parts.data_ptr<float>();
    bp.ksplit = ks;
    bp.qsplit = qs;
    if (ks > 1) {
      bp.dq_part = w;
      w += (int64_t)ks * q.size(0) * q.size(1) * q.size(2) * q.size(3);
    }
    if (qs > 1) {
      const int64_t n = (int64_t)qs * k.size(0) * k.size(1) * k.size(2) * k.size(3);
      bp.dk_part = w;
      bp.dv_part = w + n;
    }
  }
  cs336::flash_attn_bwd(bp, to_dtype(q), stream());
}

// ------------------------------------------------------------------------------------------
// RMSNorm
// ------------------------------------------------------------------------------------------
std::tuple<at::Tensor, at::Tensor> rmsnorm_fwd(const at::Tensor& x, const at::Tensor& w, double eps,
                                               std::optional<at::ScalarType> out_dtype) {
  check_cuda(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous(), "cs336: rmsnorm x must be contiguous (M, H)");
  TORCH_CHECK(w.is_contiguous() && w.numel() == x.size(1), "cs336: rmsnorm weight shape");
  TORCH_CHECK(x.size(1) % 4 == 0 && x.size(1) <= 8192, "cs336: rmsnorm hidden size must be a multiple of 4, <= 8192");
  c10::DeviceGuard g(x.device());
  at::Tensor y = at::empty_like(x, x.options().dtype(out_dtype.value_or(x.scalar_type())));
  at::Tensor rstd = at::empty({x.size(0)}, x.options().dtype(at::kFloat));
  if (x.size(0) == 0) return {y, rstd};
  cs336::rmsnorm_fwd(x.data_ptr(), to_dtype(x), w.data_ptr(), to_dtype(w), y.data_ptr(), to_dtype(y),
                     rstd.data_ptr<float>(), x.size(0), x.size(1), (float)eps, stream());
  return {y, rstd};
}

// dw_out: an fp32 (H) contiguous tensor the column reduction writes dw into (a DDP bucket view:
// parallel/ddp.py), else a fresh tensor
std::tuple<at::Tensor, at::Tensor> rmsnorm_bwd_impl(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w,
                                                    const at::Tensor& rstd, const at::Tensor* dw_out) {
  check_cuda(dy, "dy");
  TORCH_CHECK(dy.is_contiguous() && x.is_contiguous() && dy.sizes() == x.sizes(), "cs336: rmsnorm_bwd shapes");
  TORCH_CHECK(x.size(1) % 4 == 0, "cs336: rmsnorm_bwd needs a hidden size divisible by 4");
  c10::DeviceGuard g(x.device());
  at::Tensor dx = at::empty_like(x);
  at::Tensor dw = dw_out ? *dw_out : at::empty({x.size(1)}, x.options().dtype(at::kFloat));
  if (x.size(0) == 0) return {dx, dw.zero_()};
  const int rows = cs336::rmsnorm_bwd_workspace_rows(x.size(0), x.size(1));
  at::Tensor ws = at::empty({(int64_t)rows, x.size(1)}, x.options().dtype(at::kFloat));
  cs336::rmsnorm_bwd(dy.data_ptr(), to_dtype(dy), x.data_ptr(), to_dtype(x), w.data_ptr(), to_dtype(w),
                     rstd.data_ptr<float>(), dx.data_ptr(), dw.data_ptr<float>(), ws.data_ptr<float>(), x.size(0),
                     x.size(1), stream());
  return {dx, dw};
}

void check_dw_out(const at::Tensor& dw, const at::Tensor& x) {
  TORCH_CHECK(dw.is_cuda() && dw.scalar_type() == at::kFloat && dw.is_contiguous() && dw.numel() == x.size(1) &&
                  dw.device() == x.device(),
              "cs336: dw_out must be a contiguous fp32 (H) tensor on the input's device");
}

std::tuple<at::Tensor, at::Tensor> rmsnorm_bwd(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w,
                                               const at::Tensor& rstd) {
  return rmsnorm_bwd_impl(dy, x, w, rstd, nullptr);
}

at::Tensor rmsnorm_bwd_into(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w, const at::Tensor& rstd,
                            at::Tensor& dw_out) {
  check_dw_out(dw_out, x);
  return std::get<0>(rmsnorm_bwd_impl(dy, x, w, rstd, &dw_out));
}

// ------------------------------------------------------------------------------------------
// bf16 MFMA GEMM: C = op(a) @ op(b), op = transpose if trans_*; (trans_a, trans_b) in
// {(F,T): X·Wᵀ, (F,F): dY·W, (T,F): dYᵀ·X}. Tile/split auto-chosen unless given (bm, bn, splits > 0).
// ------------------------------------------------------------------------------------------
struct TileChoice {
  int bm = 0, bn = 0, splits = 1;
};

TileChoice choose_tile(int64_t M, int64_t N, int64_t K, bool fp32_out) {
  static const int cand[][2] = {{256, 160}, {160, 256}, {192, 160}, {160, 160}};
  TileChoice best;
  double best_score = -1.0;
  const int64_t kt = K / 64;
  for (const auto& c : cand) {
    if (M % c[0] || N % c[1]) continue;
    const int64_t tiles = (M / c[0]) * (N / c[1]);
    const double intensity = (double)c[0] * c[1] / (c[0] + c[1]) / (256.0 * 160.0 / 416.0);
    for (int s : {1, 2, 3, 4, 5, 6, 8}) {
      if (s > 1 && (!fp32_out || kt / s < 16)) break;
      const int64_t wg = tiles * s;
      const double util = (double)wg / (double)(((wg + 255) / 256) * 256);
      const double score = util * intensity * (s > 1 ? 0.93 : 1.0);
      if (score > best_score + 1e-9) {
        best_score = score;
        best = {c[0], c[1], s};
      }
    }
  }
  return best;
}

bool gemm_supported(const at::Tensor& a, const at::Tensor& b, bool trans_a, bool trans_b) {
  if (!a.is_cuda() || !b.is_cuda() || a.dim() != 2 || b.dim() != 2) return false;
  if (a.scalar_type() != at::kBFloat16 || b.scalar_type() != at::kBFloat16) return false;
  if (trans_a && trans_b) return false;
  if (a.stride(1) != 1 || b.stride(1) != 1 || a.stride(0) % 8 || b.stride(0) % 8) return false;
  if (reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 || reinterpret_cast<uintptr_t>(b.data_ptr()) % 16) return false;
  const int64_t M = trans_a ? a.size(1) : a.size(0), K = trans_a ? a.size(0) : a.size(1);
  const int64_t N = trans_b ? b.size(0) : b.size(1), Kb = trans_b ? b.size(1) : b.size(0);
  if (K != Kb || K % 64 || K == 0) return false;
  if (M > INT32_MAX || N > INT32_MAX || K > INT32_MAX) return false;
  return choose_tile(M, N, K, true).bm != 0;
}

at::Tensor gemm(const at::Tensor& a, const at::Tensor& b, bool trans_a, bool trans_b, std::optional<at::ScalarType> out_dtype,
                const std::optional<at::Tensor>& out, bool accumulate, int64_t bm, int64_t bn, int64_t splits) {
  TORCH_CHECK(gemm_supported(a, b, trans_a, trans_b), "cs336: gemm shape/layout/dtype not supported (see gemm_supported)");
  const int64_t M = trans_a ? a.size(1) : a.size(0), K = trans_a ? a.size(0) : a.size(1);
  const int64_t N = trans_b ? b.size(0) : b.size(1);
  c10::DeviceGuard g(a.device());
  at::Tensor c;
  if (out.has_value() && out->defined()) {
    c = *out;
    TORCH_CHECK(c.dim() == 2 && c.size(0) == M && c.size(1) == N && c.stride(1) == 1, "cs336: gemm out must be (M, N) with unit column stride");
    TORCH_CHECK(c.scalar_type() == at::kFloat || (c.scalar_type() == at::kBFloat16 && !accumulate), "cs336: gemm out dtype");
  } else {
    TORCH_CHECK(!accumulate, "cs336: gemm accumulate needs out");
    c = at::empty({M, N}, a.options().dtype(out_dtype.value_or(at::kBFloat16)));
  }
  const bool f32 = c.scalar_type() == at::kFloat;
  TileChoice t = choose_tile(M, N, K, f32);
  if (bm > 0 && bn > 0) {
    TORCH_CHECK(cs336::gemm::tile_supported((int)bm, (int)bn) && M % bm == 0 && N % bn == 0, "cs336: gemm tile");
    t.bm = (int)bm;
    t.bn = (int)bn;
    t.splits = 1;
  }
  if (splits > 0) t.splits = f32 ? (int)splits : 1;
  // the split-K reduction stores float4: needs a 16-B aligned output with ld % 4 == 0
  if (t.splits > 1 && (reinterpret_cast<uintptr_t>(c.data_ptr()) % 16 || c.stride(0) % 4 || N % 4)) t.splits = 1;
  cs336::GemmArgs p;
  p.a = reinterpret_cast<const cs336::bf16_t*>(a.data_ptr());
  p.b = reinterpret_cast<const cs336::bf16_t*>(b.data_ptr());
  p.lda = a.stride(0);
  p.ldb = b.stride(0);
  p.M = (int)M;
  p.N = (int)N;
  p.K = (int)K;
  if (t.splits > 1) {
    at::Tensor slabs = at::empty({t.splits, M, N}, a.options().dtype(at::kFloat));
    p.c = slabs.data_ptr();
    p.ldc = N;
    p.split_stride = M * N;
    TORCH_CHECK(cs336::gemm::gemm_bf16(p, t.bm, t.bn, !trans_a, trans_b, 1, t.splits, stream()), "cs336: gemm launch");
    cs336::gemm::splitk_reduce(slabs.data_ptr<float>(), c.data_ptr<float>(), M, N, t.splits, c.stride(0), accumulate, stream());
  } else {
    p.c = c.data_ptr();
    p.ldc = c.stride(0);
    p.split_stride = 0;
    const int mode = f32 ? (accumulate ? 2 : 1) : 0;
    TORCH_CHECK(cs336::gemm::gemm_bf16(p, t.bm, t.bn, !trans_a, trans_b, mode, 1, stream()), "cs336: gemm launch");
  }
  return c;
}

at::Tensor gemm_new(const at::Tensor& a, const at::Tensor& b, bool trans_a, bool trans_b, at::ScalarType out_dtype,
                    int64_t bm, int64_t bn, int64_t splits) {
  return gemm(a, b, trans_a, trans_b, out_dtype, std::nullopt, false, bm, bn, splits);
}

void gemm_out(const at::Tensor& a, const at::Tensor& b, bool trans_a, bool trans_b, const at::Tensor& out,
              bool accumulate, int64_t bm, int64_t bn, int64_t splits) {
  gemm(a, b, trans_a, trans_b, std::nullopt, out, accumulate, bm, bn, splits);
}

bool gemm_ok(const at::Tensor& a, const at::Tensor& b, bool trans_a, bool trans_b) {
  return gemm_supported(a, b, trans_a, trans_b);
}

std::vector<int64_t> gemm_plan(int64_t M, int64_t N, int64_t K, bool fp32_out) {
  const TileChoice t = choose_tile(M, N, K, fp32_out);
  return {t.bm, t.bn, t.splits};
}

// out = x.t().contiguous() for a 2-D 16-bit tensor with unit column stride
at::Tensor transpose2d(const at::Tensor& x) {
  check_cuda(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.element_size() == 2, "cs336: transpose2d needs a 2-D 16-bit row-major tensor");
  TORCH_CHECK(x.size(0) % 8 == 0 && x.size(1) % 8 == 0 && x.stride(0) % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "cs336: transpose2d needs dims and row stride multiples of 8 and a 16-B aligned base");
  c10::DeviceGuard g(x.device());
  at::Tensor out = at::empty({x.size(1), x.size(0)}, x.options());
  if (x.numel() == 0) return out;
  cs336::transpose16(x.data_ptr(), x.stride(0), out.data_ptr(), out.stride(0), (int)x.size(0), (int)x.size(1), stream());
  return out;
}

// out = x.T into an existing (possibly column-block) view: out (C, R) with unit column stride
// (bf16 w, bf16 wᵀ) of an fp32 2-D weight in one pass (csrc/ops/transpose.hip cast_t_kernel)
std::tuple<at::Tensor, at::Tensor> cast_transpose_bf16(const at::Tensor& x) {
  check_cuda(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.scalar_type() == at::kFloat,
              "cs336: cast_transpose_bf16 needs a 2-D fp32 row-major tensor");
  const int64_t R = x.size(0), C = x.size(1);
  TORCH_CHECK(R % 8 == 0 && C % 8 == 0 && x.stride(0) % 4 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 &&
                  R < INT32_MAX && C < INT32_MAX,
              "cs336: cast_transpose_bf16 needs dims multiples of 8 and 16-B aligned rows");
  c10::DeviceGuard g(x.device());
  at::Tensor w = at::empty({R, C}, x.options().dtype(at::kBFloat16));
  at::Tensor wt = at::empty({C, R}, x.options().dtype(at::kBFloat16));
  if (R > 0 && C > 0)
    cs336::cast_transpose_bf16(x.data_ptr<float>(), x.stride(0), w.data_ptr(), C, wt.data_ptr(), R, (int)R, (int)C,
                               stream());
  return {w, wt};
}

void transpose2d_into(const at::Tensor& x, at::Tensor& out) {
  check_cuda(x, "x");
  check_cuda(out, "out");
  TORCH_CHECK(x.dim() == 2 && out.dim() == 2 && x.stride(1) == 1 && out.stride(1) == 1 && x.element_size() == 2 &&
                  out.scalar_type() == x.scalar_type(),
              "cs336: transpose2d_into needs 2-D 16-bit row-major tensors of one dtype");
  TORCH_CHECK(out.size(0) == x.size(1) && out.size(1) == x.size(0), "cs336: transpose2d_into shape");
  TORCH_CHECK(x.size(0) % 8 == 0 && x.size(1) % 8 == 0 && x.stride(0) % 8 == 0 && out.stride(0) % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
              "cs336: transpose2d_into needs dims/strides multiples of 8 and 16-B aligned bases");
  c10::DeviceGuard g(x.device());
  if (x.numel() == 0) return;
  cs336::transpose16(x.data_ptr(), x.stride(0), out.data_ptr(), out.stride(0), (int)x.size(0), (int)x.size(1), stream());
}

static bool f32_or_bf16(const at::Tensor& t) {
  return t.scalar_type() == at::kFloat || t.scalar_type() == at::kBFloat16;
}

// s = x + r; y = rmsnorm(s) * w  (pre-norm residual add fused with the next norm)
std::tuple<at::Tensor, at::Tensor, at::Tensor> add_rmsnorm_fwd(const at::Tensor& x, const at::Tensor& r,
                                                               const at::Tensor& w, double eps,
                                                               std::optional<at::ScalarType> out_dtype) {
  check_cuda(x, "x");
  check_cuda(r, "r");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && r.is_contiguous() && r.sizes() == x.sizes(),
              "cs336: add_rmsnorm x, r must be contiguous (M, H) of the same shape");
  TORCH_CHECK(w.scalar_type() == at::kFloat && w.is_contiguous() && w.numel() == x.size(1),
              "cs336: add_rmsnorm weight must be fp32 (H)");
  TORCH_CHECK(f32_or_bf16(x) && f32_or_bf16(r), "cs336: add_rmsnorm x, r must be fp32 or bf16");
  TORCH_CHECK(x.size(1) % 4 == 0 && x.size(1) <= 8192, "cs336: rmsnorm hidden size must be a multiple of 4, <= 8192");
  c10::DeviceGuard g(x.device());
  at::Tensor y = at::empty_like(x, x.options().dtype(out_dtype.value_or(x.scalar_type())));
  TORCH_CHECK(f32_or_bf16(y), "cs336: add_rmsnorm out dtype must be fp32 or bf16");
  at::Tensor s = at::empty_like(x);
  at::Tensor rstd = at::empty({x.size(0)}, x.options().dtype(at::kFloat));
  if (x.size(0) == 0) return {s, y, rstd};
  cs336::add_rmsnorm_fwd(x.data_ptr(), to_dtype(x), r.data_ptr(), to_dtype(r), w.data_ptr<float>(), y.data_ptr(),
                         to_dtype(y), s.data_ptr(), rstd.data_ptr<float>(), x.size(0), x.size(1), (float)eps, stream());
  return {s, y, rstd};
}

// dx = rmsnorm_bwd(dy; s) + dres; dx_bf16 = bf16(dx) when emit_bf16 (else an empty tensor)
std::tuple<at::Tensor, at::Tensor, at::Tensor> rmsnorm_bwd_add_impl(const at::Tensor& dy, const at::Tensor& x,
                                                                    const at::Tensor& w, const at::Tensor& rstd,
                                                                    const at::Tensor& dres, bool emit_bf16,
                                                                    const at::Tensor* dw_out) {
  check_cuda(dy, "dy");
  TORCH_CHECK(dy.is_contiguous() && x.is_contiguous() && dy.sizes() == x.sizes(), "cs336: rmsnorm_bwd_add shapes");
  TORCH_CHECK(x.size(1) % 4 == 0, "cs336: rmsnorm_bwd_add needs a hidden size divisible by 4");
  TORCH_CHECK(dres.is_contiguous() && dres.sizes() == x.sizes() && dres.scalar_type() == x.scalar_type(),
              "cs336: rmsnorm_bwd_add dres must match x");
  TORCH_CHECK(w.scalar_type() == at::kFloat && w.is_contiguous() && w.numel() == x.size(1),
              "cs336: rmsnorm_bwd_add weight must be fp32 (H)");
  TORCH_CHECK(f32_or_bf16(dy) && f32_or_bf16(x), "cs336: rmsnorm_bwd_add dtypes must be fp32 or bf16");
  c10::DeviceGuard g(x.device());
  at::Tensor dx = at::empty_like(x);
  at::Tensor dx2 = emit_bf16 ? at::empty_like(x, x.options().dtype(at::kBFloat16)) : at::empty({0}, x.options().dtype(at::kBFloat16));
  at::Tensor dw = dw_out ? *dw_out : at::empty({x.size(1)}, x.options().dtype(at::kFloat));
  if (x.size(0) == 0) return {dx, dx2, dw.zero_()};
  const int rows = cs336::rmsnorm_bwd_workspace_rows(x.size(0), x.size(1));
  at::Tensor ws = at::empty({(int64_t)rows, x.size(1)}, x.options().dtype(at::kFloat));
  cs336::rmsnorm_bwd_add(dy.data_ptr(), to_dtype(dy), x.data_ptr(), to_dtype(x), w.data_ptr<float>(),
                         rstd.data_ptr<float>(), dres.data_ptr(), dx.data_ptr(), emit_bf16 ? dx2.data_ptr() : nullptr,
                         dw.data_ptr<float>(), ws.data_ptr<float>(), x.size(0), x.size(1), stream());
  return {dx, dx2, dw};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> rmsnorm_bwd_add(const at::Tensor& dy, const at::Tensor& x,
                                                               const at::Tensor& w, const at::Tensor& rstd,
                                                               const at::Tensor& dres, bool emit_bf16) {
  return rmsnorm_bwd_add_impl(dy, x, w, rstd, dres, emit_bf16, nullptr);
}

std::tuple<at::Tensor, at::Tensor> rmsnorm_bwd_add_into(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w,
                                                        const at::Tensor& rstd, const at::Tensor& dres, bool emit_bf16,
                                                        at::Tensor& dw_out) {
  check_dw_out(dw_out, x);
  auto r = rmsnorm_bwd_add_impl(dy, x, w, rstd, dres, emit_bf16, &dw_out);
  return {std::get<0>(r), std::get<1>(r)};
}

// also returns the bf16 result transposed, (H, M) row-major, for the dW = dYᵀ·X GEMMs
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> rmsnorm_bwd_add_t_impl(
    const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w, const at::Tensor& rstd, const at::Tensor& dres,
    bool emit_bf16, const at::Tensor* dw_out) {
  check_cuda(dy, "dy");
  TORCH_CHECK(dy.is_contiguous() && x.is_contiguous() && dy.sizes() == x.sizes() && x.dim() == 2,
              "cs336: rmsnorm_bwd_add_t shapes");
  const int64_t M = x.size(0), H = x.size(1);
  TORCH_CHECK(H % 8 == 0 && H <= 8192, "cs336: rmsnorm_bwd_add_t needs a hidden size divisible by 8, <= 8192");
  TORCH_CHECK(M % cs336::rmsnorm_bwd_add_t_rows(H) == 0, "cs336: rmsnorm_bwd_add_t needs rows divisible by ",
              cs336::rmsnorm_bwd_add_t_rows(H));
  TORCH_CHECK(dres.is_contiguous() && dres.sizes() == x.sizes() && dres.scalar_type() == x.scalar_type(),
              "cs336: rmsnorm_bwd_add_t dres must match x");
  TORCH_CHECK(w.scalar_type() == at::kFloat && w.is_contiguous() && w.numel() == H,
              "cs336: rmsnorm_bwd_add_t weight must be fp32 (H)");
  TORCH_CHECK(f32_or_bf16(dy) && f32_or_bf16(x), "cs336: rmsnorm_bwd_add_t dtypes must be fp32 or bf16");
  c10::DeviceGuard g(x.device());
  at::Tensor dx = at::empty_like(x);
  at::Tensor dx2 = emit_bf16 ? at::empty_like(x, x.options().dtype(at::kBFloat16)) : at::empty({0}, x.options().dtype(at::kBFloat16));
  at::Tensor dxt = at::empty({H, M}, x.options().dtype(at::kBFloat16));
  at::Tensor dw = dw_out ? *dw_out : at::empty({H}, x.options().dtype(at::kFloat));
  if (M == 0) return {dx, dx2, dxt, dw.zero_()};
  at::Tensor ws = at::empty({(int64_t)cs336::rmsnorm_bwd_add_t_workspace_rows(M, H), H}, x.options().dtype(at::kFloat));
  cs336::rmsnorm_bwd_add_t(dy.data_ptr(), to_dtype(dy), x.data_ptr(), to_dtype(x), w.data_ptr<float>(),
                           rstd.data_ptr<float>(), dres.data_ptr(), dx.data_ptr(), emit_bf16 ? dx2.data_ptr() : nullptr,
                           dxt.data_ptr(), dw.data_ptr<float>(), ws.data_ptr<float>(), M, H, stream());
  return {dx, dx2, dxt, dw};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> rmsnorm_bwd_add_t(const at::Tensor& dy, const at::Tensor& x,
                                                                             const at::Tensor& w, const at::Tensor& rstd,
                                                                             const at::Tensor& dres, bool emit_bf16) {
  return rmsnorm_bwd_add_t_impl(dy, x, w, rstd, dres, emit_bf16, nullptr);
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> rmsnorm_bwd_add_t_into(const at::Tensor& dy, const at::Tensor& x,
                                                                      const at::Tensor& w, const at::Tensor& rstd,
                                                                      const at::Tensor& dres, bool emit_bf16,
                                                                      at::Tensor& dw_out) {
  check_dw_out(dw_out, x);
  auto r = rmsnorm_bwd_add_t_impl(dy, x, w, rstd, dres, emit_bf16, &dw_out);
  return {std::get<0>(r), std::get<1>(r), std::get<2>(r)};
}

// ------------------------------------------------------------------------------------------
// RoPE
// ------------------------------------------------------------------------------------------
void rope_into(const at::Tensor& x, const at::Tensor& cos, const at::Tensor& sin, const std::optional<at::Tensor>& pos,
               bool inverse, const at::Tensor& out);

at::Tensor rope(const at::Tensor& x, const at::Tensor& cos, const at::Tensor& sin, const std::optional<at::Tensor>& pos,
                bool inverse) {
  check_cuda(x, "x");
  TORCH_CHECK(x.dim() == 4, "cs336: rope x must be (B,H,N,D)");
  c10::DeviceGuard g(x.device());
  at::Tensor out = empty_bnhd_like(x);
  rope_into(x, cos, sin, pos, inverse, out);
  return out;
}

// writes into a caller-provided (B,H,N,D) strided view (e.g. a slice of a fused dQKV buffer)
void rope_into(const at::Tensor& x, const at::Tensor& cos, const at::Tensor& sin, const std::optional<at::Tensor>& pos,
               bool inverse, const at::Tensor& out) {
  check_cuda(x, "x");
  TORCH_CHECK(x.dim() == 4 && x.stride(3) == 1, "cs336: rope x must be (B,H,N,D) with contiguous D");
  TORCH_CHECK(out.dim() == 4 && out.stride(3) == 1 && out.sizes() == x.sizes() && out.dtype() == x.dtype(),
              "cs336: rope out must match x with contiguous D");
  const int64_t D = x.size(3);
  TORCH_CHECK(D >= 8 && D <= 256 && D % 8 == 0, "cs336: rope head dim must be a multiple of 8 in [8, 256]");
  TORCH_CHECK(x.size(0) * x.size(1) * x.size(2) * (D / 8) < ((int64_t)1 << 31), "cs336: rope tensor too large for 32-bit indexing");
  // 16-B vector accesses: every stride and base 16-B aligned
  const int64_t es = x.element_size();
  for (const at::Tensor* t : {&x, &out}) {
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0 && (t->stride(0) * es) % 16 == 0 &&
                    (t->stride(1) * es) % 16 == 0 && (t->stride(2) * es) % 16 == 0,
                "cs336: rope tensors must be 16-byte aligned with 16-byte aligned strides");
  }
  TORCH_CHECK(cos.scalar_type() == at::kFloat && cos.is_contiguous() && sin.is_contiguous(), "cs336: rope cache");
  TORCH_CHECK(cos.size(1) * 2 == x.size(3), "cs336: rope cache width");
  c10::DeviceGuard g(x.device());
  const int64_t* pp = nullptr;
  if (pos.has_value() && pos->defined()) {
    TORCH_CHECK(pos->scalar_type() == at::kLong && pos->is_contiguous() && pos->numel() == x.size(0) * x.size(2),
                "cs336: rope positions must be contiguous int64 (B, N)");
    pp = pos->data_ptr<int64_t>();
  } else {
    TORCH_CHECK(x.size(2) <= cos.size(0), "cs336: sequence longer than the RoPE cache");
  }
  if (x.numel() == 0) return;
  cs336::RopeArgs ra{x.data_ptr(), x.stride(0), x.stride(1), x.stride(2), out.data_ptr(), out.stride(0), out.stride(1),
                     out.stride(2)};
  cs336::rope(ra, to_dtype(x), cos.data_ptr<float>(), sin.data_ptr<float>(), pp, (int)x.size(0), (int)x.size(1),
              (int)x.size(2), (int)x.size(3), inverse, stream());
}

// ------------------------------------------------------------------------------------------
// SwiGLU gate
// ------------------------------------------------------------------------------------------
at::Tensor silu_mul_fwd(const at::Tensor& a, const at::Tensor& b) {
  check_cuda(a, "a");
  TORCH_CHECK(a.is_contiguous() && b.is_contiguous() && a.sizes() == b.sizes() && a.dtype() == b.dtype(),
              "cs336: silu_mul operands");
  c10::DeviceGuard g(a.device());
  at::Tensor h = at::empty_like(a);
  cs336::silu_mul_fwd(a.data_ptr(), b.data_ptr(), h.data_ptr(), to_dtype(a), 1, a.numel(), a.numel(), stream());
  return h;
}

std::tuple<at::Tensor, at::Tensor> silu_mul_bwd(const at::Tensor& dh, const at::Tensor& a, const at::Tensor& b) {
  check_cuda(a, "a");
  TORCH_CHECK(dh.is_contiguous() && dh.sizes() == a.sizes() && dh.dtype() == a.dtype(), "cs336: silu_mul_bwd dh");
  c10::DeviceGuard g(a.device());
  at::Tensor da = at::empty_like(a), db = at::empty_like(b);
  cs336::silu_mul_bwd(dh.data_ptr(), a.data_ptr(), b.data_ptr(), da.data_ptr(), db.data_ptr(), to_dtype(a), 1,
                      a.numel(), a.numel(), stream());
  return {da, db};
}

// fused layout: y = [a | b] of shape (..., 2F) (output of the fused W1|W3 GEMM) -> h (..., F)
at::Tensor swiglu_fused_fwd(const at::Tensor& y) {
  check_cuda(y, "y");
  TORCH_CHECK(y.is_contiguous() && y.size(-1) % 8 == 0, "cs336: swiglu_fused y must be contiguous (..., 2F), F%4==0");
  c10::DeviceGuard g(y.device());
  const int64_t F = y.size(-1) / 2, M = y.numel() / y.size(-1);
  auto sizes = y.sizes().vec();
  sizes.back() = F;
  at::Tensor h = at::empty(sizes, y.options());
  const int64_t es = y.element_size();
  cs336::silu_mul_fwd(y.data_ptr(), (char*)y.data_ptr() + F * es, h.data_ptr(), to_dtype(y), M, F, 2 * F, stream());
  return h;
}

at::Tensor swiglu_fused_bwd(const at::Tensor& dh, const at::Tensor& y) {
  check_cuda(y, "y");
  TORCH_CHECK(dh.is_contiguous() && dh.dtype() == y.dtype() && dh.numel() * 2 == y.numel(), "cs336: swiglu_fused_bwd");
  c10::DeviceGuard g(y.device());
  const int64_t F = y.size(-1) / 2, M = y.numel() / y.size(-1);
  at::Tensor dy = at::empty_like(y);
  const int64_t es = y.element_size();
  cs336::silu_mul_bwd(dh.data_ptr(), y.data_ptr(), (char*)y.data_ptr() + F * es, dy.data_ptr(),
                      (char*)dy.data_ptr() + F * es, to_dtype(y), M, F, 2 * F, stream());
  return dy;
}

// ------------------------------------------------------------------------------------------
// cross entropy
// ------------------------------------------------------------------------------------------
std::tuple<at::Tensor, at::Tensor> xent_fwd(const at::Tensor& z, const at::Tensor& t) {
  check_cuda(z, "logits");
  TORCH_CHECK(z.dim() == 2 && z.is_contiguous(), "cs336: logits must be contiguous (M, V)");
  TORCH_CHECK(t.scalar_type() == at::kLong && t.is_contiguous() && t.numel() == z.size(0), "cs336: targets");
  c10::DeviceGuard g(z.device());
  at::Tensor loss = at::empty({z.size(0)}, z.options().dtype(at::kFloat));
  at::Tensor lse = at::empty({z.size(0)}, z.options().dtype(at::kFloat));
  cs336::xent_fwd(z.data_ptr(), to_dtype(z), t.data_ptr<int64_t>(), loss.data_ptr<float>(), lse.data_ptr<float>(),
                  z.size(0), z.size(1), stream());
  return {loss, lse};
}

at::Tensor xent_bwd(const at::Tensor& gs, const at::Tensor& z, const at::Tensor& t, const at::Tensor& lse,
                    double mult) {
  check_cuda(z, "logits");
  TORCH_CHECK(gs.scalar_type() == at::kFloat && gs.numel() == 1, "cs336: xent_bwd grad must be a fp32 scalar");
  c10::DeviceGuard g(z.device());
  at::Tensor dz = at::empty_like(z);
  cs336::xent_bwd(gs.data_ptr<float>(), z.data_ptr(), to_dtype(z), t.data_ptr<int64_t>(), lse.data_ptr<float>(),
                  dz.data_ptr(), (float)mult, z.size(0), z.size(1), stream());
  return dz;
}

// ------------------------------------------------------------------------------------------
// multi-tensor
// ------------------------------------------------------------------------------------------
// Device copy of a multi-tensor launch's pointer / size table, reused while the table repeats: the
// optimizer's parameter, state and shadow pointers are fixed and the caching allocator gives the
// gradients the same addresses step after step, so steady-state steps issue no host-to-device blit
// per launch (with the update overlapped with the backward, each blit waited for a CU beside the
// one-workgroup-per-CU GEMMs: profiles/r5_2p7b_roofline_b32_ovl.md). Keyed by the exact contents,
// the device and the stream; a copy is only reused on the stream that enqueued it (ordered after
// the copy), and it stays allocated while cached. Step time: XL 573.6-574.3 -> 574.0-574.5 ms,
// 2.7b 607.2 / 608.1 -> 606.9 / 605.9 ms (profiles/r5_table_cache_ab.log): within noise, 56-88
// fewer blit kernels per step.
// HIP-graph capture: a captured launch bakes the table's device address into the graph, and a
// table first built inside the capture is filled by a captured copy that re-reads its host bytes at
// every replay. Tables used by a capture therefore move to a second map that is never evicted, and
// the host bytes of one built during the capture live in a pinned arena of this file's own
// (hipHostMalloc'd outside any capture, never freed): PyTorch's caching host allocator cannot serve
// there (it queries the events of its freed blocks, and one recorded in the capturing stream fails).
struct CaptureArena {
  char* base = nullptr;
  size_t used = 0, cap = 0;
  void reserve() {  // outside a capture: a fresh 4 MiB block once the current one is 3/4 used
    if (base && used + (cap >> 2) <= cap) return;
    void* p = nullptr;
    TORCH_CHECK(hipHostMalloc(&p, 4u << 20, hipHostMallocDefault) == hipSuccess, "cs336: hipHostMalloc (table arena)");
    base = static_cast<char*>(p);  // the previous block stays allocated: captured copies read it
    used = 0;
    cap = 4u << 20;
  }
  const void* put(const std::vector<int64_t>& h) {
    const size_t bytes = (h.size() * sizeof(int64_t) + 255) & ~(size_t)255;
    TORCH_CHECK(base && used + bytes <= cap, "cs336: table arena exhausted inside a HIP-graph capture");
    char* dst = base + used;
    std::memcpy(dst, h.data(), h.size() * sizeof(int64_t));
    used += bytes;
    return dst;
  }
};

at::Tensor device_table(const std::vector<int64_t>& h, c10::Device device) {
  static std::mutex mu;
  // leaked on purpose: tensors freed by a static destructor at exit would reach a torn-down allocator
  static auto& cache = *new std::unordered_map<std::string, at::Tensor>();
  static auto& captured = *new std::unordered_map<std::string, at::Tensor>();
  static auto& arena = *new CaptureArena();
  const hipStream_t st = stream();
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  TORCH_CHECK(hipStreamIsCapturing(st, &cs) == hipSuccess, "cs336: hipStreamIsCapturing failed");
  const bool capturing = cs != hipStreamCaptureStatusNone;
  std::string key(sizeof(st) + sizeof(int) + h.size() * sizeof(int64_t), '\0');
  const int di = device.index();
  std::memcpy(&key[0], &st, sizeof(st));
  std::memcpy(&key[sizeof(st)], &di, sizeof(int));
  std::memcpy(&key[sizeof(st) + sizeof(int)], h.data(), h.size() * sizeof(int64_t));
  std::lock_guard<std::mutex> lock(mu);
  auto pit = captured.find(key);
  if (pit != captured.end()) return pit->second;
  auto it = cache.find(key);
  if (it != cache.end()) {
    if (!capturing) return it->second;
    at::Tensor dev = it->second;  // filled before the capture: pin it for the graph's lifetime
    cache.erase(it);
    captured.emplace(std::move(key), dev);
    return dev;
  }
  if (capturing) {
    const void* src = arena.put(h);
    at::Tensor dev = at::empty({(int64_t)h.size()}, at::TensorOptions().dtype(at::kLong).device(device));
    TORCH_CHECK(hipMemcpyAsync(dev.data_ptr(), src, h.size() * sizeof(int64_t), hipMemcpyHostToDevice, st) == hipSuccess,
                "cs336: captured table copy");
    captured.emplace(std::move(key), dev);
    return dev;
  }
  arena.reserve();  // ready before any capture starts
  at::Tensor host = at::empty({(int64_t)h.size()}, at::TensorOptions().dtype(at::kLong).pinned_memory(true));
  std::memcpy(host.data_ptr<int64_t>(), h.data(), h.size() * sizeof(int64_t));
  at::Tensor dev = host.to(device, /*non_blocking=*/true);
  if (cache.size() >= 4096) cache.clear();  // a workload whose tables never repeat: bounded
  cache.emplace(std::move(key), dev);
  return dev;
}

struct HostTable {
  at::Tensor dev;  // keeps the device copy alive until the ops that use it are enqueued
  cs336::TensorTable tt;
};

HostTable build_table(const std::vector<std::vector<at::Tensor>>& lists) {
  const int n = (int)lists[0].size();
  const int nptr = (int)lists.size();
  for (const auto& l : lists) TORCH_CHECK((int)l.size() == n, "cs336: tensor lists must have equal length");
  const int64_t len = (int64_t)n * nptr + (n + 1) + n;
  std::vector<int64_t> hv((size_t)len);
  int64_t* h = hv.data();
  int64_t chunks = 0;
  for (int i = 0; i < n; ++i) {
    const at::Tensor& t0 = lists[0][i];
    for (int k = 0; k < nptr; ++k) {
      const at::Tensor& t = lists[k][i];
      TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "cs336: multi-tensor inputs must be contiguous GPU tensors");
      TORCH_CHECK(t.numel() == t0.numel(), "cs336: multi-tensor numel mismatch");
      h[(int64_t)i * nptr + k] = reinterpret_cast<int64_t>(t.data_ptr());
    }
    h[(int64_t)n * nptr + i] = chunks;
    chunks += (t0.numel() + cs336::kMTChunk - 1) / cs336::kMTChunk;
    h[(int64_t)n * nptr + (n + 1) + i] = t0.numel();
  }
  h[(int64_t)n * nptr + n] = chunks;
  HostTable ht;
  ht.dev = device_table(hv, lists[0][0].device());
  const int64_t* d = ht.dev.data_ptr<int64_t>();
  ht.tt.ptrs = d;
  ht.tt.chunk_base = d + (int64_t)n * nptr;
  ht.tt.numel = d + (int64_t)n * nptr + (n + 1);
  ht.tt.n = n;
  ht.tt.total_chunks = chunks;
  return ht;
}

void check_same_dtype(const std::vector<at::Tensor>& ts, at::ScalarType st, const char* name) {
  for (const auto& t : ts) TORCH_CHECK(t.scalar_type() == st, "cs336: ", name, " dtype mismatch");
}

// ------------------------------------------------------------------------------------------
// token embedding backward (deterministic, graph-safe): gw = Σ rows of g per token id
// ------------------------------------------------------------------------------------------
void embedding_bwd_into(const at::Tensor& g, const at::Tensor& sorted_ids, const at::Tensor& perm, at::Tensor& out) {
  check_cuda(g, "g");
  TORCH_CHECK(g.dim() == 2 && g.is_contiguous() && g.size(1) % 4 == 0, "cs336: embedding_bwd g must be contiguous (T, D), D % 4 == 0");
  TORCH_CHECK(g.scalar_type() == at::kFloat || g.scalar_type() == at::kBFloat16 || g.scalar_type() == at::kHalf,
              "cs336: embedding_bwd g dtype");
  TORCH_CHECK(sorted_ids.scalar_type() == at::kLong && perm.scalar_type() == at::kLong && sorted_ids.is_contiguous() &&
                  perm.is_contiguous() && sorted_ids.numel() == g.size(0) && perm.numel() == g.size(0),
              "cs336: embedding_bwd sorted ids / perm must be contiguous int64 of T entries");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.dim() == 2 && out.is_contiguous() &&
                  out.size(1) == g.size(1) && out.device() == g.device(),
              "cs336: embedding_bwd out must be a contiguous fp32 (V, D) tensor");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(g.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
              "cs336: embedding_bwd needs 16-B aligned g / out");
  c10::DeviceGuard dg(g.device());
  cs336::embedding_bwd(g.data_ptr(), to_dtype(g), sorted_ids.data_ptr<int64_t>(), perm.data_ptr<int64_t>(),
                       out.data_ptr<float>(), g.size(0), out.size(0), g.size(1), stream());
}

at::Tensor embedding_bwd(const at::Tensor& g, const at::Tensor& sorted_ids, const at::Tensor& perm, int64_t vocab) {
  at::Tensor out = at::empty({vocab, g.size(1)}, g.options().dtype(at::kFloat));
  embedding_bwd_into(g, sorted_ids, perm, out);
  return out;
}

// the device-resident step size of a graph-captured update (adamw_device_step), or null
const float* alpha_ptr(const std::optional<at::Tensor>& alpha_dev, const at::Tensor& like) {
  if (!alpha_dev.has_value()) return nullptr;
  const at::Tensor& a = *alpha_dev;
  TORCH_CHECK(a.is_cuda() && a.device() == like.device() && a.scalar_type() == at::kFloat && a.numel() == 1,
              "cs336: alpha_dev must be a one-element fp32 tensor on the parameters' device");
  return a.data_ptr<float>();
}

// t += 1; alpha = lr·sqrt(1-b2^t)/(1-b1^t) on the device (the bias correction of a HIP-graph-replayed
// optimizer step, ops/adamw.py FusedAdamW.enable_device_step)
void adamw_device_step(at::Tensor& t, at::Tensor& alpha, double lr, double beta1, double beta2) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kLong && t.numel() == 1, "cs336: t must be a one-element int64 GPU tensor");
  TORCH_CHECK(alpha.is_cuda() && alpha.scalar_type() == at::kFloat && alpha.numel() == 1 && alpha.device() == t.device(),
              "cs336: alpha must be a one-element fp32 tensor on t's device");
  c10::DeviceGuard g(t.device());
  cs336::adamw_device_step(t.data_ptr<int64_t>(), alpha.data_ptr<float>(), lr, beta1, beta2, stream());
}

void adamw_step(std::vector<at::Tensor> params, std::vector<at::Tensor> grads, std::vector<at::Tensor> exp_avg,
                std::vector<at::Tensor> exp_avg_sq, std::vector<at::Tensor> shadows, double lr, double beta1,
                double beta2, double eps, double weight_decay, int64_t step,
                const std::optional<at::Tensor>& alpha_dev) {
  if (params.empty()) return;
  check_same_dtype(params, at::kFloat, "params (fp32 master weights)");
  check_same_dtype(exp_avg, at::kFloat, "exp_avg");
  check_same_dtype(exp_avg_sq, at::kFloat, "exp_avg_sq");
  const at::ScalarType gt = grads[0].scalar_type();
  check_same_dtype(grads, gt, "grads");
  const bool shadow = !shadows.empty();
  if (shadow) check_same_dtype(shadows, at::kBFloat16, "bf16 shadows");
  c10::DeviceGuard g(params[0].device());
  HostTable ht = shadow ? build_table({params, grads, exp_avg, exp_avg_sq, shadows})
                        : build_table({params, grads, exp_avg, exp_avg_sq});
  // alpha * (sqrt(1 - b2^t) / (1 - b1^t)) in double, as the reference evaluates it in Python
  const double alpha_t = lr * (std::sqrt(1.0 - std::pow(beta2, (double)step)) / (1.0 - std::pow(beta1, (double)step)));
  cs336::adamw_step(ht.tt, to_dtype(grads[0]), shadow, (float)beta1, (float)beta2, (float)(1.0 - beta1),
                    (float)(1.0 - beta2), (float)eps, (float)(lr * weight_decay), (float)alpha_t,
                    alpha_ptr(alpha_dev, params[0]), stream());
}

// AdamW over 2-D weights that also writes each weight's transposed bf16 shadow (Wᵀ, a (C, R) view
// with unit column stride whose row stride may exceed R: a column block of a grouped Wᵀ)
void adamw_step_t(std::vector<at::Tensor> params, std::vector<at::Tensor> grads, std::vector<at::Tensor> exp_avg,
                  std::vector<at::Tensor> exp_avg_sq, std::vector<at::Tensor> shadows, std::vector<at::Tensor> wts,
                  double lr, double beta1, double beta2, double eps, double weight_decay, int64_t step,
                  const std::optional<at::Tensor>& alpha_dev) {
  const int n = (int)params.size();
  if (n == 0) return;
  TORCH_CHECK((int)grads.size() == n && (int)exp_avg.size() == n && (int)exp_avg_sq.size() == n &&
                  (int)shadows.size() == n && (int)wts.size() == n,
              "cs336: adamw_step_t list lengths differ");
  check_same_dtype(params, at::kFloat, "params (fp32 master weights)");
  check_same_dtype(exp_avg, at::kFloat, "exp_avg");
  check_same_dtype(exp_avg_sq, at::kFloat, "exp_avg_sq");
  check_same_dtype(shadows, at::kBFloat16, "bf16 shadows");
  check_same_dtype(wts, at::kBFloat16, "transposed bf16 shadows");
  const at::ScalarType gt = grads[0].scalar_type();
  check_same_dtype(grads, gt, "grads");
  const int64_t len = (int64_t)n * 6 + (n + 1) + (int64_t)n * 3;
  std::vector<int64_t> hv((size_t)len);
  int64_t* h = hv.data();
  int64_t tiles = 0;
  auto aligned = [](const at::Tensor& t) { return (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0; };
  for (int i = 0; i < n; ++i) {
    const at::Tensor &p = params[i], &g = grads[i], &m = exp_avg[i], &v = exp_avg_sq[i], &s = shadows[i], &w = wts[i];
    TORCH_CHECK(p.dim() == 2 && p.is_cuda() && p.is_contiguous() && g.is_contiguous() && m.is_contiguous() &&
                    v.is_contiguous() && s.is_contiguous(),
                "cs336: adamw_step_t needs contiguous 2-D GPU tensors");
    const int64_t R = p.size(0), C = p.size(1);
    TORCH_CHECK(g.sizes() == p.sizes() && m.sizes() == p.sizes() && v.sizes() == p.sizes() && s.sizes() == p.sizes(),
                "cs336: adamw_step_t shape mismatch");
    TORCH_CHECK(w.dim() == 2 && w.size(0) == C && w.size(1) == R && w.stride(1) == 1 && w.stride(0) % 8 == 0,
                "cs336: Wᵀ must be a (C, R) view with unit column stride and a row stride multiple of 8");
    TORCH_CHECK(R % 8 == 0 && C % 8 == 0, "cs336: adamw_step_t needs R, C multiples of 8");
    TORCH_CHECK(aligned(p) && aligned(g) && aligned(m) && aligned(v) && aligned(s) && aligned(w),
                "cs336: adamw_step_t pointers must be 16-byte aligned");
    const at::Tensor* ts[6] = {&p, &g, &m, &v, &s, &w};
    for (int k = 0; k < 6; ++k) h[(int64_t)i * 6 + k] = reinterpret_cast<int64_t>(ts[k]->data_ptr());
    h[(int64_t)n * 6 + i] = tiles;
    tiles += ((R + 255) / 256) * ((C + 63) / 64);
    int64_t* d = h + (int64_t)n * 6 + (n + 1) + 3 * i;
    d[0] = R;
    d[1] = C;
    d[2] = w.stride(0);
  }
  h[(int64_t)n * 6 + n] = tiles;
  c10::DeviceGuard guard(params[0].device());
  at::Tensor dev = device_table(hv, params[0].device());
  const int64_t* dptr = dev.data_ptr<int64_t>();
  const double alpha_t = lr * (std::sqrt(1.0 - std::pow(beta2, (double)step)) / (1.0 - std::pow(beta1, (double)step)));
  cs336::adamw_step_t(dptr, dptr + (int64_t)n * 6, dptr + (int64_t)n * 6 + (n + 1), n, tiles, to_dtype(grads[0]),
                      (float)beta1, (float)beta2, (float)(1.0 - beta1), (float)(1.0 - beta2), (float)eps,
                      (float)(lr * weight_decay), (float)alpha_t, alpha_ptr(alpha_dev, params[0]), stream());
}

void multi_tensor_cast_bf16(std::vector<at::Tensor> src, std::vector<at::Tensor> dst) {
  if (src.empty()) return;
  check_same_dtype(src, at::kFloat, "src");
  check_same_dtype(dst, at::kBFloat16, "dst");
  c10::DeviceGuard g(src[0].device());
  HostTable ht = build_table({src, dst});
  cs336::multi_tensor_cast_bf16(ht.tt, stream());
}

at::Tensor multi_tensor_l2norm(std::vector<at::Tensor> tensors) {
  TORCH_CHECK(!tensors.empty(), "cs336: empty tensor list");
  const at::ScalarType st = tensors[0].scalar_type();
  check_same_dtype(tensors, st, "tensors");
  c10::DeviceGuard g(tensors[0].device());
  HostTable ht = build_table({tensors});
  at::Tensor partials = at::empty({std::max<int64_t>(ht.tt.total_chunks, 1)}, tensors[0].options().dtype(at::kFloat));
  at::Tensor out = at::zeros({}, tensors[0].options().dtype(at::kFloat));
  cs336::multi_tensor_sumsq(ht.tt, to_dtype(tensors[0]), partials.data_ptr<float>(), stream());
  cs336::finalize_l2norm(partials.data_ptr<float>(), ht.tt.total_chunks, out.data_ptr<float>(), stream());
  return out;
}

void multi_tensor_scale_(std::vector<at::Tensor> tensors, const at::Tensor& scale) {
  if (tensors.empty()) return;
  const at::ScalarType st = tensors[0].scalar_type();
  check_same_dtype(tensors, st, "tensors");
  TORCH_CHECK(scale.scalar_type() == at::kFloat && scale.numel() == 1 && scale.is_cuda(), "cs336: scale");
  c10::DeviceGuard g(tensors[0].device());
  HostTable ht = build_table({tensors});
  cs336::multi_tensor_scale(ht.tt, to_dtype(tensors[0]), scale.data_ptr<float>(), stream());
}

}  // namespace

// CU-occupying spin kernel (RCCL stand-in for concurrency tests), on the current stream
void occupy(int64_t n_workgroups, int64_t lds_bytes, double ms, at::Tensor& counter) {
  check_cuda(counter, "counter");
  TORCH_CHECK(counter.scalar_type() == at::kInt && counter.numel() >= 1, "cs336: occupy counter must be int32");
  TORCH_CHECK(n_workgroups > 0 && n_workgroups <= 65536 && lds_bytes >= 4 && lds_bytes <= 160 * 1024 && ms >= 0 &&
                  ms <= 10000,
              "cs336: occupy arguments out of range");
  cs336::occupy((int)n_workgroups, (int)lds_bytes, ms, counter.data_ptr<int>(), stream());
}

// byte-moving occupant (csrc/ops/occupy.hip): src read / dst written, same byte size, 16 KiB multiples
void occupy_bytes(int64_t n_workgroups, int64_t lds_bytes, double ms, const at::Tensor& src, at::Tensor& dst,
                  int64_t total_bytes, at::Tensor& counter) {
  check_cuda(src, "src");
  TORCH_CHECK(counter.scalar_type() == at::kInt && counter.numel() >= 1, "cs336: occupy counter must be int32");
  const int64_t nb = src.numel() * src.element_size();
  TORCH_CHECK(src.is_contiguous() && dst.is_contiguous() && dst.numel() * dst.element_size() >= nb && nb >= 16384,
              "cs336: occupy_bytes needs contiguous src/dst of >= 16 KiB, dst at least src's size");
  TORCH_CHECK(n_workgroups > 0 && n_workgroups <= 4096 && lds_bytes >= 4 && lds_bytes <= 65536 && ms > 0 && ms < 10000 &&
                  total_bytes >= 0,
              "cs336: occupy_bytes arguments out of range");
  c10::DeviceGuard g(src.device());
  cs336::occupy_bytes((int)n_workgroups, (int)lds_bytes, ms, src.data_ptr(), dst.data_ptr(), nb & ~(int64_t)16383,
                      total_bytes, counter.data_ptr<int>(), stream());
}

// co-residency probe (csrc/ops/occupy.hip), on the current stream; state: int32[3]
void cohort(int64_t n_workgroups, int64_t lds_bytes, double deadline_ms, at::Tensor& state) {
  check_cuda(state, "state");
  TORCH_CHECK(state.scalar_type() == at::kInt && state.numel() >= 3 && state.is_contiguous(),
              "cs336: cohort state must be a contiguous int32[3]");
  TORCH_CHECK(n_workgroups > 0 && n_workgroups <= 4096 && lds_bytes >= 4 && lds_bytes <= 160 * 1024 &&
                  deadline_ms > 0 && deadline_ms <= 2000,
              "cs336: cohort arguments out of range");
  cs336::cohort((int)n_workgroups, (int)lds_bytes, deadline_ms, state.data_ptr<int>(), stream());
}

// NT projection GEMM with fused SwiGLU epilogues (csrc/gemm/gemm8.hip), on the current stream.
//   epi 0: c = a @ b.T                      a (M,K), b (N,K), c (M,N)
//   epi 1: y = c = a @ [w1; w3].T, h = silu(y[:, :half]) * y[:, half:]     b (2·half, K)
//   epi 2: dh = a @ b.T (not stored); c = [dh·b·silu'(a) | dh·silu(a)] from y = [a|b]   b (half, K)
bool gemm8_check(const at::Tensor& t, int64_t rows, int64_t cols, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.dim() == 2 && t.stride(1) == 1, "cs336: gemm8 ",
              what, " must be a row-major bf16 CUDA matrix");
  TORCH_CHECK(t.size(0) == rows && t.size(1) == cols, "cs336: gemm8 ", what, " shape ", t.sizes(), " expected (", rows,
              ", ", cols, ")");
  TORCH_CHECK(t.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "cs336: gemm8 ", what,
              " rows must be 16-B aligned");
  return true;
}

// epi 3: `half` carries rope_cols, which must cover whole column tiles (the rotation is decided per
// tile); the binding also needs d_head <= 96 (the tile rows' cos/sin fit the LDS behind the scratch)
// epi 0 also takes N and K tails (multiples of 8: the vocabulary head, 10000 = 31·320 + 80)
bool gemm8_ok(int64_t M, int64_t N, int64_t K, int64_t epi, int64_t half) {
  if (M <= 0 || N <= 0 || K <= 0 || M >= (1 << 30) || N >= (1 << 30) || K >= (1 << 30)) return false;
  const int fn = cs336::gemm8::pick_fn((int)N, (int)epi, (int)half);
  if (fn == 0 || M % 256) return false;
  if (epi == 0) return N % 8 == 0 && K % 8 == 0;
  return K % 64 == 0 && N % (64 * fn) == 0 && (epi != 3 || half % (64 * fn) == 0);
}

// gemm8 / gemm8w address each operand through one buffer descriptor with 32-bit byte offsets
constexpr int64_t kDmaLimit = (int64_t(1) << 31) - (int64_t(1) << 20);
bool gemm8_extents_ok(const at::Tensor& a, const at::Tensor& b) {
  const int64_t K = a.size(1);
  return (255 * a.stride(0) + K) * 2 < kDmaLimit && ((b.size(0) - 1) * b.stride(0) + K) * 2 < kDmaLimit;
}

void gemm8(const at::Tensor& a, const at::Tensor& b, at::Tensor& c, int64_t epi, int64_t fn, const OptT& h,
           const OptT& y, int64_t half) {
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  gemm8_check(a, M, K, "a");
  gemm8_check(b, N, K, "b");
  TORCH_CHECK(epi >= 0 && epi <= 2, "cs336: gemm8 epi");
  TORCH_CHECK(gemm8_ok(M, N, K, epi, half), "cs336: gemm8 does not take M=", M, " N=", N, " K=", K, " epi=", epi);
  TORCH_CHECK(gemm8_extents_ok(a, b), "cs336: gemm8 operand extent exceeds the 2 GiB DMA range");
  cs336::gemm8::Args p{};
  p.a = reinterpret_cast<const uint16_t*>(a.data_ptr());
  p.b = reinterpret_cast<const uint16_t*>(b.data_ptr());
  p.lda = a.stride(0);
  p.ldb = b.stride(0);
  p.M = (int)M;
  p.N = (int)N;
  p.K = (int)K;
  p.half = (int)half;
  if (epi == 0) {
    gemm8_check(c, M, N, "c");
  } else if (epi == 1) {
    TORCH_CHECK(N == 2 * half, "cs336: gemm8 epi 1 needs b = [w1; w3] with 2·half rows");
    gemm8_check(c, M, N, "y");
    TORCH_CHECK(h.has_value() && h->defined(), "cs336: gemm8 epi 1 needs h");
    gemm8_check(*h, M, half, "h");
    p.h = reinterpret_cast<uint16_t*>(h->data_ptr());
    p.ldh = h->stride(0);
  } else {
    TORCH_CHECK(N == half, "cs336: gemm8 epi 2 needs b with half rows");
    gemm8_check(c, M, 2 * half, "c = [da|db]");
    TORCH_CHECK(y.has_value() && y->defined(), "cs336: gemm8 epi 2 needs y");
    gemm8_check(*y, M, 2 * half, "y");
    p.y = reinterpret_cast<const uint16_t*>(y->data_ptr());
    p.ldy = y->stride(0);
  }
  p.c = reinterpret_cast<uint16_t*>(c.data_ptr());
  p.ldc = c.stride(0);
  c10::DeviceGuard g(a.device());
  TORCH_CHECK(cs336::gemm8::launch(p, (int)epi, (int)fn, stream()), "cs336: gemm8 launch (fn ", fn, ")");
}

// diagnostic stamp buffer of gemm8 (CS336_G8_STAMP builds, scripts/gemm8_stamps.py): uint64 (blocks, 8)
// or None = off; returns whether this build writes stamps
bool gemm8_stamps(const std::optional<at::Tensor>& buf) {
  if (!buf.has_value()) return cs336::gemm8::set_stamp_buffer(nullptr, 0);
  const at::Tensor& b = *buf;
  TORCH_CHECK(b.is_cuda() && b.scalar_type() == at::kLong && b.is_contiguous() && b.dim() == 2 && b.size(1) == 8,
              "cs336: gemm8 stamp buffer must be a contiguous int64 (blocks, 8) GPU tensor");
  return cs336::gemm8::set_stamp_buffer(reinterpret_cast<uint64_t*>(b.data_ptr<int64_t>()), b.size(0));
}

// QKV projection forward with RoPE in the store (gemm8 epi 3): c = a @ b.T with columns < rope_cols
// rotated (interleaved pairs, d_head dhead) at position pos[row] (pos: int64 per row, or None: row % seq).
void gemm8_rope(const at::Tensor& a, const at::Tensor& b, at::Tensor& c, const at::Tensor& cos, const at::Tensor& sin,
                const OptT& pos, int64_t seq, int64_t rope_cols, int64_t dhead) {
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  gemm8_check(a, M, K, "a");
  gemm8_check(b, N, K, "b");
  gemm8_check(c, M, N, "c");
  TORCH_CHECK(gemm8_ok(M, N, K, 3, rope_cols), "cs336: gemm8_rope does not take M=", M, " N=", N, " K=", K,
              " rope_cols=", rope_cols);
  TORCH_CHECK(gemm8_extents_ok(a, b), "cs336: gemm8_rope operand extent exceeds the 2 GiB DMA range");
  TORCH_CHECK(dhead % 8 == 0 && dhead > 0 && dhead <= 96 && rope_cols % dhead == 0 && rope_cols <= N && seq > 0,
              "cs336: gemm8_rope needs d_head % 8 == 0, d_head <= 96 and whole rotated heads");
  TORCH_CHECK(cos.is_cuda() && sin.is_cuda() && cos.scalar_type() == at::kFloat && sin.scalar_type() == at::kFloat &&
                  cos.is_contiguous() && sin.is_contiguous() && cos.dim() == 2 && cos.size(1) == dhead / 2 &&
                  sin.sizes() == cos.sizes(),
              "cs336: gemm8_rope cos/sin must be contiguous fp32 (ctx, d_head/2)");
  const int64_t* pp = nullptr;
  if (pos.has_value() && pos->defined()) {
    TORCH_CHECK(pos->is_cuda() && pos->scalar_type() == at::kLong && pos->is_contiguous() && pos->numel() == M,
                "cs336: gemm8_rope pos must be contiguous int64 with one entry per row");
    pp = pos->data_ptr<int64_t>();
  } else {
    TORCH_CHECK(seq <= cos.size(0), "cs336: gemm8_rope seq ", seq, " exceeds the RoPE cache ", cos.size(0));
  }
  cs336::gemm8::Args p{};
  p.a = reinterpret_cast<const uint16_t*>(a.data_ptr());
  p.b = reinterpret_cast<const uint16_t*>(b.data_ptr());
  p.c = reinterpret_cast<uint16_t*>(c.data_ptr());
  p.lda = a.stride(0);
  p.ldb = b.stride(0);
  p.ldc = c.stride(0);
  p.M = (int)M;
  p.N = (int)N;
  p.K = (int)K;
  p.rcos = cos.data_ptr<float>();
  p.rsin = sin.data_ptr<float>();
  p.rpos = pp;
  p.rseq = (int)seq;
  p.rope_cols = (int)rope_cols;
  p.rdh = (int)dhead;
  c10::DeviceGuard g(a.device());
  TORCH_CHECK(cs336::gemm8::launch(p, 3, 0, stream()), "cs336: gemm8_rope launch");
}

// Weight gradient straight from token-major operands (csrc/gemm/gemm8w.hip):
//   out[m][n] (+)= Σ_t a[t][m]·b[t][n]    (trans_out: out[n][m])
// a (K, M) and b (K, N) bf16 with unit column stride; out fp32 (M, N) or (N, M) with unit column
// stride; splits > 1: out is (splits, rows, cols) dense slabs, one partial per split.
void gemm8w(const at::Tensor& a, const at::Tensor& b, at::Tensor& out, int64_t splits, bool trans_out,
            bool accumulate, int64_t fn) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16 &&
                  a.dim() == 2 && b.dim() == 2 && a.stride(1) == 1 && b.stride(1) == 1,
              "cs336: gemm8w needs row-major bf16 CUDA operands");
  const int64_t K = a.size(0), M = a.size(1), N = b.size(1);
  TORCH_CHECK(b.size(0) == K, "cs336: gemm8w contraction mismatch");
  TORCH_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(b.data_ptr()) % 16 == 0 && M % 8 == 0 && N % 8 == 0,
              "cs336: gemm8w needs 16-B aligned rows");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat, "cs336: gemm8w out must be fp32 CUDA");
  const int64_t rows = trans_out ? N : M, cols = trans_out ? M : N;
  if (splits > 1) {
    TORCH_CHECK(out.dim() == 3 && out.size(0) == splits && out.size(1) == rows && out.size(2) == cols &&
                    out.is_contiguous() && !accumulate,
                "cs336: gemm8w split-K out must be contiguous (splits, rows, cols) slabs");
  } else {
    TORCH_CHECK(out.dim() == 2 && out.size(0) == rows && out.size(1) == cols && out.stride(1) == 1 &&
                    out.stride(0) % 4 == 0 && reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
                "cs336: gemm8w out shape/alignment");
  }
  // The kernel addresses one split's token rows through a buffer descriptor with 32-bit byte offsets:
  // each launch's per-split extent must stay below 2 GiB (a 50304-vocabulary head at
  // 49152 tokens is 4.9 GB of dY). splits == 1 is cut into token chunks here, each chunk after the
  // first accumulating into `out`; with split-K slabs the caller must pick enough splits.
  TORCH_CHECK(K % 64 == 0 && K > 0, "cs336: gemm8w needs K % 64 == 0");
  const int64_t ld = std::max(a.stride(0), b.stride(0)), wide = std::max(M, N);
  auto extent = [&](int64_t rows) { return rows * ld * 2 + wide * 2; };
  const int64_t nkt = K / 64, per_split = (nkt + splits - 1) / splits * 64;
  TORCH_CHECK(splits == 1 || extent(per_split) < kDmaLimit, "cs336: gemm8w split of ", per_split,
              " token rows exceeds the 2 GiB DMA range; use more splits (", splits, " given)");
  const int64_t chunk = std::max<int64_t>(64, std::min(K, (kDmaLimit - wide * 2) / (ld * 2) / 64 * 64));
  TORCH_CHECK(splits > 1 || extent(chunk) < kDmaLimit, "cs336: gemm8w rows too wide for the DMA range");
  c10::DeviceGuard g(a.device());
  for (int64_t k0 = 0; k0 < K; k0 += (splits > 1 ? K : chunk)) {
    const int64_t kc = splits > 1 ? K : std::min(chunk, K - k0);
    cs336::gemm8::WArgs p{};
    p.a = reinterpret_cast<const uint16_t*>(a.data_ptr()) + k0 * a.stride(0);
    p.b = reinterpret_cast<const uint16_t*>(b.data_ptr()) + k0 * b.stride(0);
    p.c = out.data_ptr<float>();
    p.lda = a.stride(0);
    p.ldb = b.stride(0);
    p.ldc = splits > 1 ? cols : out.stride(0);
    p.slab_stride = splits > 1 ? rows * cols : 0;
    p.a_elems = (kc - 1) * a.stride(0) + M;
    p.b_elems = (kc - 1) * b.stride(0) + N;
    p.M = (int)M;
    p.N = (int)N;
    p.K = (int)kc;
    p.splits = (int)splits;
    p.trans_out = trans_out ? 1 : 0;
    p.accumulate = (accumulate || k0 > 0) ? 1 : 0;
    TORCH_CHECK(cs336::gemm8::launch_w(p, (int)fn, stream()), "cs336: gemm8w does not take M=", M, " N=", N,
                " K=", kc, " splits=", splits);
  }
}

// Sum of split-K fp32 slabs (splits, M, N) into out (M, N; unit column stride, 16-B aligned rows),
// optionally added to it: one float4 per thread walking the splits (csrc/gemm/gemm.hip). Replaces
// torch.sum(slabs, 0), whose generic dim-0 reduction ran at ~40 % of HBM for the weight gradients'
// slabs (profiles/r5_2p7b_roofline_b32.md: 75.6 us per 2560 x 2560 call).
void splitk_sum(const at::Tensor& slabs, at::Tensor& out, bool accumulate) {
  TORCH_CHECK(slabs.is_cuda() && slabs.scalar_type() == at::kFloat && slabs.dim() == 3 && slabs.is_contiguous(),
              "cs336: splitk_sum slabs must be contiguous fp32 (splits, M, N)");
  const int64_t M = slabs.size(1), N = slabs.size(2);
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.dim() == 2 && out.size(0) == M &&
                  out.size(1) == N && out.stride(1) == 1 && out.stride(0) % 4 == 0 && N % 4 == 0 &&
                  reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
              "cs336: splitk_sum out must be fp32 (M, N) with 16-B aligned rows");
  if (M * N == 0 || slabs.size(0) == 0) return;
  c10::DeviceGuard g(slabs.device());
  cs336::gemm::splitk_reduce(slabs.data_ptr<float>(), out.data_ptr<float>(), M, N, (int)slabs.size(0), out.stride(0),
                             accumulate, stream());
}

TORCH_LIBRARY(cs336, m) {
  m.def(
      "fa_fwd(Tensor q, Tensor k, Tensor v, bool causal, float scale, Tensor? rope_cos=None, Tensor? rope_sin=None, "
      "Tensor? rope_pos=None) -> (Tensor, Tensor)");
  m.def(
      "fa_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor out, Tensor lse, bool causal, float scale, "
      "Tensor? rope_cos=None, Tensor? rope_sin=None, Tensor? rope_pos=None) -> "
      "(Tensor, Tensor, Tensor)");
  m.def("rmsnorm_fwd(Tensor x, Tensor weight, float eps, ScalarType? out_dtype) -> (Tensor, Tensor)");
  m.def("rmsnorm_bwd(Tensor dy, Tensor x, Tensor weight, Tensor rstd) -> (Tensor, Tensor)");
  m.def("rmsnorm_bwd_into(Tensor dy, Tensor x, Tensor weight, Tensor rstd, Tensor(a!) dw_out) -> Tensor");
  m.def("add_rmsnorm_fwd(Tensor x, Tensor r, Tensor weight, float eps, ScalarType? out_dtype) -> (Tensor, Tensor, Tensor)");
  m.def("transpose2d(Tensor x) -> Tensor");
  m.def("transpose2d_into(Tensor x, Tensor(a!) out) -> ()");
  m.def("gemm(Tensor a, Tensor b, bool trans_a, bool trans_b, ScalarType out_dtype, int bm=0, int bn=0, int splits=0) -> Tensor");
  m.def("gemm_out(Tensor a, Tensor b, bool trans_a, bool trans_b, Tensor(a!) out, bool accumulate=False, int bm=0, int bn=0, int splits=0) -> ()");
  m.def("gemm_ok(Tensor a, Tensor b, bool trans_a, bool trans_b) -> bool", &gemm_ok);
  m.def("gemm_plan(int M, int N, int K, bool fp32_out) -> int[]", &gemm_plan);
  m.def("rmsnorm_bwd_add(Tensor dy, Tensor x, Tensor weight, Tensor rstd, Tensor dres, bool emit_bf16) -> (Tensor, Tensor, Tensor)");
  m.def("rmsnorm_bwd_add_t(Tensor dy, Tensor x, Tensor weight, Tensor rstd, Tensor dres, bool emit_bf16) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("rmsnorm_bwd_add_into(Tensor dy, Tensor x, Tensor weight, Tensor rstd, Tensor dres, bool emit_bf16, Tensor(a!) dw_out) -> (Tensor, Tensor)");
  m.def("rmsnorm_bwd_add_t_into(Tensor dy, Tensor x, Tensor weight, Tensor rstd, Tensor dres, bool emit_bf16, Tensor(a!) dw_out) -> (Tensor, Tensor, Tensor)");
  m.def("rope(Tensor x, Tensor cos, Tensor sin, Tensor? pos, bool inverse) -> Tensor");
  m.def(
      "fa_bwd_into(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor out, Tensor lse, bool causal, float scale, "
      "Tensor(a!) dq, Tensor(b!) dk, Tensor(c!) dv, Tensor? rope_cos=None, Tensor? rope_sin=None, Tensor? rope_pos=None, "
      "bool rope_out_only=False) -> ()");
  m.def("rope_into(Tensor x, Tensor cos, Tensor sin, Tensor? pos, bool inverse, Tensor(a!) out) -> ()");
  m.def("swiglu_fused_fwd(Tensor y) -> Tensor");
  m.def("swiglu_fused_bwd(Tensor dh, Tensor y) -> Tensor");
  m.def("multi_tensor_cast_bf16(Tensor[] src, Tensor(a!)[] dst) -> ()");
  m.def("silu_mul_fwd(Tensor a, Tensor b) -> Tensor");
  m.def("silu_mul_bwd(Tensor dh, Tensor a, Tensor b) -> (Tensor, Tensor)");
  m.def("xent_fwd(Tensor logits, Tensor targets) -> (Tensor, Tensor)");
  m.def("xent_bwd(Tensor g, Tensor logits, Tensor targets, Tensor lse, float mult) -> Tensor");
  m.def(
      "adamw_step(Tensor(a!)[] params, Tensor[] grads, Tensor(b!)[] exp_avg, Tensor(c!)[] exp_avg_sq, "
      "Tensor(d!)[] shadows, float lr, float beta1, float beta2, float eps, float weight_decay, int step, "
      "Tensor? alpha_dev=None) -> ()");
  m.def("adamw_device_step(Tensor(a!) t, Tensor(b!) alpha, float lr, float beta1, float beta2) -> ()");
  m.def("embedding_bwd(Tensor g, Tensor sorted_ids, Tensor perm, int vocab) -> Tensor");
  m.def("cast_transpose_bf16(Tensor x) -> (Tensor, Tensor)");
  m.def("gemm8_stamps(Tensor? buf) -> bool", &gemm8_stamps);
  m.def("embedding_bwd_into(Tensor g, Tensor sorted_ids, Tensor perm, Tensor(a!) out) -> ()");
  m.def("multi_tensor_l2norm(Tensor[] tensors) -> Tensor");
  m.def("fa_fwd_ot(Tensor q, Tensor k, Tensor v, bool causal, float scale) -> (Tensor, Tensor, Tensor)");
  m.def(
      "adamw_step_t(Tensor(a!)[] params, Tensor[] grads, Tensor(b!)[] exp_avg, Tensor(c!)[] exp_avg_sq, "
      "Tensor(d!)[] shadows, Tensor(e!)[] wts, float lr, float beta1, float beta2, float eps, float weight_decay, "
      "int step, Tensor? alpha_dev=None) -> ()");
  m.def("occupy(int n_workgroups, int lds_bytes, float ms, Tensor(a!) counter) -> ()");
  m.def("occupy_bytes(int n_workgroups, int lds_bytes, float ms, Tensor src, Tensor(a!) dst, int total_bytes, Tensor(b!) counter) -> ()");
  m.def("cohort(int n_workgroups, int lds_bytes, float deadline_ms, Tensor(a!) state) -> ()");
  m.def("gemm8(Tensor a, Tensor b, Tensor(a!) c, int epi, int fn, Tensor(b!)? h, Tensor? y, int half) -> ()");
  m.def("gemm8_ok(int M, int N, int K, int epi, int half) -> bool", &gemm8_ok);
  m.def("gemm8_rope(Tensor a, Tensor b, Tensor(a!) c, Tensor cos, Tensor sin, Tensor? pos, int seq, int rope_cols, int dhead) -> ()");
  m.def("gemm8w(Tensor a, Tensor b, Tensor(a!) out, int splits, bool trans_out, bool accumulate, int fn) -> ()");
  m.def("splitk_sum(Tensor slabs, Tensor(a!) out, bool accumulate) -> ()");
  m.def("multi_tensor_scale_(Tensor(a!)[] tensors, Tensor scale) -> ()");
}

TORCH_LIBRARY_IMPL(cs336, CUDA, m) {
  m.impl("fa_fwd", &fa_fwd);
  m.impl("fa_fwd_ot", &fa_fwd_ot);
  m.impl("fa_bwd", &fa_bwd);
  m.impl("rmsnorm_fwd", &rmsnorm_fwd);
  m.impl("rmsnorm_bwd", &rmsnorm_bwd);
  m.impl("rmsnorm_bwd_into", &rmsnorm_bwd_into);
  m.impl("transpose2d", &transpose2d);
  m.impl("transpose2d_into", &transpose2d_into);
  m.impl("gemm", &gemm_new);
  m.impl("gemm_out", &gemm_out);
  m.impl("add_rmsnorm_fwd", &add_rmsnorm_fwd);
  m.impl("rmsnorm_bwd_add", &rmsnorm_bwd_add);
  m.impl("rmsnorm_bwd_add_t", &rmsnorm_bwd_add_t);
  m.impl("rmsnorm_bwd_add_into", &rmsnorm_bwd_add_into);
  m.impl("rmsnorm_bwd_add_t_into", &rmsnorm_bwd_add_t_into);
  m.impl("rope", &rope);
  m.impl("fa_bwd_into", &fa_bwd_into);
  m.impl("rope_into", &rope_into);
  m.impl("swiglu_fused_fwd", &swiglu_fused_fwd);
  m.impl("swiglu_fused_bwd", &swiglu_fused_bwd);
  m.impl("multi_tensor_cast_bf16", &multi_tensor_cast_bf16);
  m.impl("silu_mul_fwd", &silu_mul_fwd);
  m.impl("silu_mul_bwd", &silu_mul_bwd);
  m.impl("xent_fwd", &xent_fwd);
  m.impl("xent_bwd", &xent_bwd);
  m.impl("adamw_step", &adamw_step);
  m.impl("adamw_step_t", &adamw_step_t);
  m.impl("adamw_device_step", &adamw_device_step);
  m.impl("embedding_bwd", &embedding_bwd);
  m.impl("cast_transpose_bf16", &cast_transpose_bf16);
  m.impl("embedding_bwd_into", &embedding_bwd_into);
  m.impl("multi_tensor_l2norm", &multi_tensor_l2norm);
  m.impl("occupy", &occupy);
  m.impl("occupy_bytes", &occupy_bytes);
  m.impl("cohort", &cohort);
  m.impl("gemm8", &gemm8);
  m.impl("gemm8_rope", &gemm8_rope);
  m.impl("gemm8w", &gemm8w);
  m.impl("splitk_sum", &splitk_sum);
  m.impl("multi_tensor_scale_", &multi_tensor_scale_);
}
