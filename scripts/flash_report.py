"""Tables and plots for the FlashAttention-2 sweep (reference ``flashattentioncode.py:69-258``: a
latency table for fwd / bwd / fwd+bwd per (seq, d, dtype) and three plots), from the JSON rows of
``python -m cs336_systems.bench.flash --sweep --json sweep.json``.

    python scripts/flash_report.py sweep.json --out profiles/r3_flash_sweep

writes ``<out>.md`` (markdown table: HIP FA2 vs ROCm SDPA vs materializing PyTorch, ms and TFLOP/s)
and ``<out>_{fwd,bwd,fwd_bwd}.png`` (latency vs sequence length, one panel per head dim and dtype).
"""

import argparse
import json
from collections import defaultdict

IMPL_NAMES = {"hip_fa2": "HIP FA2", "torch_sdpa": "ROCm SDPA", "torch_naive": "PyTorch (materializing)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("sweep")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    rows = json.load(open(a.sweep))
    table = defaultdict(dict)  # (dtype, d, causal, N) -> impl -> row
    for r in rows:
        key = (r.get("dtype"), r.get("d"), r.get("causal"), r.get("N"))
        table[key][r["impl"]] = r
    impls = [i for i in IMPL_NAMES if any(i in v for v in table.values())]
    lines = ["# FlashAttention-2 sweep (B = 1, H = 1; do_bench with L2 + Infinity Cache flushed per call)", "",
             "ms per call (TFLOP/s in parentheses; fwd = 4·N²·d (x½ causal), bwd = 2.5x fwd). `OOM` / `-`: did not run.", ""]
    hdr = "| dtype | d | causal | N | " + " | ".join(f"{IMPL_NAMES[i]} {m}" for m in ("fwd", "bwd", "fwd+bwd") for i in impls) + " |"
    lines += [hdr, "|" + "---|" * (4 + 3 * len(impls))]
    for key in sorted(table, key=lambda k: (k[0], k[1], not k[2], k[3])):
        dt, d, c, n = key
        cells = []
        for m in ("fwd", "bwd", "fwd_bwd"):
            for i in impls:
                r = table[key].get(i)
                if r is None or f"{m}_ms" not in r:
                    cells.append(r.get("error", "-") if r else "-")
                else:
                    cells.append(f"{r[m + '_ms']:.3f} ({r[m + '_tflops']:.0f})")
        lines.append(f"| {dt} | {d} | {'yes' if c else 'no'} | {n} | " + " | ".join(cells) + " |")
    with open(a.out + ".md", "w") as f:
        f.write("\n".join(lines) + "\n")
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:
        print("matplotlib not available: table only")
        return
    panels = sorted({(k[0], k[1]) for k in table})
    for m, title in (("fwd", "forward"), ("bwd", "backward"), ("fwd_bwd", "forward + backward")):
        cols = 4
        nrows = (len(panels) + cols - 1) // cols
        fig, axes = plt.subplots(nrows, cols, figsize=(4.2 * cols, 3.4 * nrows), squeeze=False)
        for ax, (dt, d) in zip(axes.flat, panels):
            for i in impls:
                pts = sorted((k[3], table[k][i][m + "_ms"]) for k in table
                             if k[0] == dt and k[1] == d and k[2] and i in table[k] and m + "_ms" in table[k][i])
                if pts:
                    ax.plot([p[0] for p in pts], [p[1] for p in pts], marker="o", ms=3, label=IMPL_NAMES[i])
            ax.set_xscale("log", base=2)
            ax.set_yscale("log")
            ax.set_title(f"{dt}, d={d}, causal")
            ax.set_xlabel("sequence length")
            ax.set_ylabel("ms")
            ax.grid(True, which="both", alpha=0.3)
        for ax in list(axes.flat)[len(panels):]:
            ax.axis("off")
        axes.flat[0].legend(fontsize=8)
        fig.suptitle(f"FlashAttention-2 {title} latency on 1x MI355X (B=1, H=1)")
        fig.tight_layout()
        fig.savefig(f"{a.out}_{m}.png", dpi=110)
        plt.close(fig)
    print(f"wrote {a.out}.md and {a.out}_{{fwd,bwd,fwd_bwd}}.png")


if __name__ == "__main__":
    main()
