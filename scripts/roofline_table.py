"""Achieved throughput of every hot kernel of one training step vs the MI355X roofline, from a
rocprofv3 kernel trace of ``bench.py`` (default: XL, ctx 512, batch 24, bf16).

    python scripts/roofline_table.py <run>_kernel_trace.csv [--d 1600 --ff 6400 --layers 48 --heads 25 --batch 24 --ctx 512]

Bytes per element follow the kernels' actual dtypes (fp32 residual stream, bf16 activations, fp32
master weights/optimizer state, bf16 shadows), counting each tensor once per read or write. Peaks:
2.5 PF/s dense bf16 MFMA (spec) and 6.3 TB/s (the measured float4-copy HBM rate of
MI355X_MICROARCH.md; 8 TB/s spec). A kernel whose operands were written just before it (e.g. RoPE on
the QKV GEMM's 157 MB output) can be served partly from the 256 MB Infinity Cache (MALL); such a row
cannot be priced against HBM alone, and is labelled "MALL-assisted" if its byte rate exceeds the HBM
roofline instead of reporting a percentage above 100.
"""

import argparse
import csv
import re
from collections import defaultdict

PEAK_TF, PEAK_TBS = 2500.0, 6.3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--d", type=int, default=1600)
    ap.add_argument("--ff", type=int, default=6400)
    ap.add_argument("--layers", type=int, default=48)
    ap.add_argument("--heads", type=int, default=25)
    ap.add_argument("--batch", type=int, default=96)  # bench.py default per-GPU batch
    ap.add_argument("--ctx", type=int, default=512)
    ap.add_argument("--vocab", type=int, default=10000)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    starts = [s for s, _, n in iv if "vectorized_gather_kernel" in n]
    lo, hi = starts[-2], starts[-1]
    step = [x for x in iv if lo <= x[0] < hi]
    t = defaultdict(float)
    n = defaultdict(int)
    xf = [s for s, _, k in step if "xent_fwd" in k][0]
    for s, e, k in step:
        if is_gemm(k):
            key = "GEMM fwd" if s < xf else "GEMM bwd (dX + dW)"
        elif "fa_fwd" in k:
            key = "FA fwd"
        elif "fa_bwd" in k:
            key = "FA bwd (dq + dkdv)"
        else:
            m = re.search(r"(\w+_kernel)\b", k)
            key = m.group(1) if m else k.split("(")[0][:40]
        t[key] += (e - s) / 1e6
        n[key] += 1
    M, d, f, L, H, N, B, V = a.batch * a.ctx, a.d, a.ff, a.layers, a.heads, a.ctx, a.batch, a.vocab
    P = L * (4 * d * d + 3 * d * f + 2 * d) + 2 * V * d + d
    gemm_fwd = 2 * M * L * (4 * d * d + 3 * d * f) + 2 * M * d * V
    attn_fwd = 4 * B * H * N * N * (d // H) / 2
    work = {  # kernel -> (kind, amount): FLOPs or bytes for the whole step
        "GEMM fwd": ("F", gemm_fwd),
        "GEMM bwd (dX + dW)": ("F", 2 * gemm_fwd),
        # attention: FLOPs AND bytes (q, k, v read + o written; the backward reads q, k, v, o, dO and
        # writes dq, dk, dv, all bf16, + fp32 row constants): at N 512-1024 the byte time is the larger
        "FA fwd": ("FB", (L * attn_fwd, L * (4 * M * d * 2 + M * H * 4))),
        "FA bwd (dq + dkdv)": ("FB", (L * 2.5 * attn_fwd, L * (8 * M * d * 2 + 2 * M * H * 4))),
        "rmsnorm_fwd_kernel": ("B", 2 * L * M * d * 12),  # x f32 + r bf16 in, s f32 + y bf16 out
        "rmsnorm_bwd_kernel": ("B", 2 * L * M * d * 16),  # dy bf16, x f32, dres f32 in; dx f32 + bf16 out
        "silu_mul_fwd_kernel": ("B", L * M * f * 6),
        "silu_mul_bwd_kernel": ("B", L * M * f * 10),
        "rope_kernel": ("B", L * M * 2 * d * 2 * 2),  # q|k bf16 read + write (d each)
        "adamw_kernel": ("B", P * 30),  # p,g,m,v in; p,m,v + bf16 shadow out
        # the 2-D weights' update (all but the 2L + 1 norm vectors): + the bf16 Wᵀ shadow
        "adamw_t_kernel": ("B", (P - (2 * L + 1) * d) * 32),
        "transpose16_kernel": ("B", None),
    }
    total = sum(t.values())
    print(f"step window {(hi - lo) / 1e6:.1f} ms, kernel time {total:.1f} ms\n")
    print("| kernel | calls | ms/step | achieved | roofline | % of roofline |")
    print("|---|---|---|---|---|---|")
    for k, ms in sorted(t.items(), key=lambda x: -x[1]):
        if ms < 0.3:
            continue
        kind, amt = work.get(k, (None, None))
        if kind == "FB":
            fl, by = amt
            tf, tb = fl / (ms * 1e-3) / 1e12, by / (ms * 1e-3) / 1e12
            bound = max(fl / PEAK_TF, by / PEAK_TBS) / 1e12 * 1e3  # ms at the binding roof
            which = "HBM" if by / PEAK_TBS > fl / PEAK_TF else "MFMA"
            print(f"| {k} | {n[k]} | {ms:.1f} | {tf:.0f} TFLOP/s, {tb:.2f} TB/s | {bound:.1f} ms ({which}-bound) | "
                  f"{100 * bound / ms:.0f} % |")
        elif kind == "F":
            ach = amt / (ms * 1e-3) / 1e12
            print(f"| {k} | {n[k]} | {ms:.1f} | {ach:.0f} TFLOP/s | {PEAK_TF:.0f} TFLOP/s dense bf16 | {100 * ach / PEAK_TF:.0f} % |")
        elif kind == "B" and amt:
            ach = amt / (ms * 1e-3) / 1e12
            pct = f"{100 * ach / PEAK_TBS:.0f} %" if ach <= PEAK_TBS else "MALL-assisted (above the HBM roofline)"
            print(f"| {k} | {n[k]} | {ms:.1f} | {ach:.2f} TB/s | {PEAK_TBS} TB/s HBM | {pct} |")
        else:
            print(f"| {k} | {n[k]} | {ms:.1f} | | | |")
    gemm_roles(step, xf, M, d, f, L, V)


def is_gemm(k: str) -> bool:
    """hipBLASLt/Tensile kernels and the cs336 GEMMs (gemm8 NT with fused epilogues, older gemm)."""
    return (k.startswith("Cijk") or k.startswith("Custom_Cijk") or "gemm8_kernel" in k or "gemm8w_kernel" in k
            or "gemm_kernel<" in k)


def gemm_roles(step, xf, M, d, f, L, V):
    """Per-projection GEMM times, labelled by the step's fixed launch order: forward = L x (qkv, o,
    w13, w2) + lm head; backward = lm head (dX, dW), then per layer in reverse w2, w13, o, qkv, each
    dX then dW. Only printed when the GEMM counts match that order (no side-stream reordering)."""
    g = [(s, e, k) for s, e, k in step if is_gemm(k)]
    fwd = [x for x in g if x[0] < xf]
    bwd = [x for x in g if x[0] >= xf]
    if len(fwd) != 4 * L + 1 or len(bwd) != 8 * L + 2:
        # (gemm8w runs in the step's own order inside the backward, counted with it here)
        print(f"\n(GEMM order not recognised: {len(fwd)} fwd / {len(bwd)} bwd GEMMs)")
        return
    flops = {"qkv": 2 * M * d * 3 * d, "o": 2 * M * d * d, "w13": 2 * M * d * 2 * f, "w2": 2 * M * f * d, "lm": 2 * M * d * V}
    t = defaultdict(float)
    names = {}
    for i, (s, e, k) in enumerate(fwd[:-1]):
        role = ("qkv", "o", "w13", "w2")[i % 4] + " fwd"
        t[role] += (e - s) / 1e6
        names[role] = k
    t["lm fwd"] += (fwd[-1][1] - fwd[-1][0]) / 1e6
    names["lm fwd"] = fwd[-1][2]
    # fused SwiGLU FFN (gemm8 epilogue 2 in the step): per layer w2 dW, w2 dX(+gate bwd), then the rest
    # (kernel names carry the template args: gemm8_kernel<FN, EPI[, TAIL]>, demangled or not)
    fused = any(re.search(r"gemm8_kernel(<\d, 2[,>]|ILi\dELi2E)", k) for _, _, k in bwd)
    order = (["w2 dW", "w2 dX", "w13 dX", "w13 dW", "o dX", "o dW", "qkv dX", "qkv dW"] if fused else
             ["w2 dX", "w2 dW", "w13 dX", "w13 dW", "o dX", "o dW", "qkv dX", "qkv dW"])
    # the lm-head weight gradient may be a gemm8w kernel too: then the first backward GEMM is lm dW
    lm_order = ("dX", "dW")
    if bwd and "gemm8w" in bwd[0][2] and len(bwd) > 1 and "gemm8w" not in bwd[1][2]:
        lm_order = ("dW", "dX")
    for j, (s, e, k) in enumerate(bwd):
        if j < 2:
            role = "lm " + lm_order[j]
        else:
            role = order[(j - 2) % 8]
        t[role] += (e - s) / 1e6
        names[role] = k
    print("\n| GEMM | ms/step | us/call | TFLOP/s | kernel (last call) |")
    print("|---|---|---|---|---|")
    for role, ms in sorted(t.items(), key=lambda x: -x[1]):
        proj = role.split()[0]
        calls = 1 if proj == "lm" else L
        tf = flops[proj] * calls / (ms * 1e-3) / 1e12
        tile = re.search(r"MT\d+x\d+x\d+", names[role])
        sk = "SK" if "_SK" in names[role] else ""
        print(f"| {role} | {ms:.2f} | {1000 * ms / calls:.1f} | {tf:.0f} | {tile.group(0) if tile else names[role][:30]} {sk} |")


if __name__ == "__main__":
    main()
