"""Same-box A/B of build variants, env switches or arguments (one process per arm, rounds interleaved
so box drift hits every arm alike). Replaces the per-experiment ``*_ab.sh`` scripts.

    python scripts/ab.py bench  "base:" "norope:CS336_QKV_ROPE=0"            # bench.py ms/step
    python scripts/ab.py bench  "b24::--batch 24" "b48::--batch 48"          # arguments per arm
    python scripts/ab.py fa     "base:CS336_LIB=cs336_systems/_native/variants/base/libcs336_hip.so" "new:"
    python scripts/ab.py flash  "two:CS336_FA_BWD=0" "fused:CS336_FA_BWD=1" --args "--seq 512 --batch 48 --heads 25 --d 64 --causal 1"
    python scripts/ab.py gemm   "default:" "prio:CS336_LIB=cs336_systems/_native/variants/prio/libcs336_hip.so"

An arm is ``label:ENV=V,ENV2=V2:extra args`` (env and args optional). ``--rounds`` (2), ``--steps``
(bench: 10), ``--timeout`` per process (s). Every process runs under its own time limit; a crash-like
exit (timeout, abort, segfault) stops the whole A/B so nothing else touches a sick GPU. Raw output
goes to ``gpurun_out/ab_<kind>_<label>_<round>.*``."""

from __future__ import annotations

import argparse
import json
import os
import shlex
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "gpurun_out")


def parse_arm(spec: str) -> tuple[str, dict, list[str]]:
    label, _, rest = spec.partition(":")
    envs, _, args = rest.partition(":")
    env = dict(kv.split("=", 1) for kv in envs.split(",") if kv)
    return label, env, shlex.split(args)


def command(kind: str, a: argparse.Namespace, extra: list[str], outfile: str) -> list[str]:
    py = sys.executable
    if kind == "bench":
        return [py, "bench.py", "--steps", str(a.steps), "--warmup", "3", *shlex.split(a.args), *extra]
    if kind == "fa":
        return [py, "scripts/fa_ab.py", *shlex.split(a.args), *extra]
    if kind == "flash":
        return [py, "-m", "cs336_systems.bench.flash", "--impls", "hip_fa2", "--no-compile", "--json", outfile,
                *shlex.split(a.args), *extra]
    if kind == "gemm":
        return [py, "scripts/gemm_vs_blas.py", "--json", outfile, *shlex.split(a.args), *extra]
    raise SystemExit(f"unknown kind {kind}")


def summarize(kind: str, log: str, outfile: str) -> list[str]:
    if kind == "bench":
        for line in open(log):
            if line.startswith("{") and '"ms_per_step"' in line:
                d = json.loads(line)
                return [f"ms_per_step={d['ms_per_step']} tok/s={d['value']}"]
        return ["(no JSON line)"]
    if kind == "fa":
        rows = [json.loads(x) for x in open(log) if x.startswith("{")]
        return [f"B{r['B']} H{r['H']} N{r['N']} d{r['D']} causal={int(r['causal'])} fwd {r['fwd_tflops']} TF bwd "
                f"{r['bwd_tflops']} TF" for r in rows]
    rows = json.load(open(outfile))
    if kind == "flash":
        return [f"{r.get('impl')} B{r.get('B')} H{r.get('H')} N{r.get('N')} d{r.get('d')} causal={r.get('causal')} "
                f"fwd {r.get('fwd_ms')} ms bwd {r.get('bwd_ms')} ms ({r.get('bwd_tflops')} TF)" for r in rows]
    return [f"{r['shape']} {r['case']} blas={r['blas_tflops']} cs336={r.get('cs336_tflops')} err={r.get('max_rel_err')}"
            for r in rows]


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("kind", choices=["bench", "fa", "flash", "gemm"])
    ap.add_argument("arms", nargs="+")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=int(os.environ.get("AB_STEPS", 10)))
    ap.add_argument("--args", default="", help="arguments for every arm's command")
    ap.add_argument("--timeout", type=int, default=240)
    a = ap.parse_args()
    os.makedirs(OUT, exist_ok=True)
    for rnd in range(1, a.rounds + 1):
        for spec in a.arms:
            label, env, extra = parse_arm(spec)
            base = os.path.join(OUT, f"ab_{a.kind}_{label}_{rnd}")
            cmd = command(a.kind, a, extra, base + ".json")
            with open(base + ".log", "w") as log:
                try:
                    rc = subprocess.run(cmd, cwd=REPO, env={**os.environ, **env}, stdout=log, stderr=subprocess.STDOUT,
                                        timeout=a.timeout).returncode
                except subprocess.TimeoutExpired:
                    rc = 124
            if rc != 0:
                print(f"round {rnd} {label}: exit {rc}; see {base}.log", flush=True)
                os.system(f"tail -n 15 {shlex.quote(base + '.log')}")
                return rc if rc > 0 else 128 - rc
            for line in summarize(a.kind, base + ".log", base + ".json"):
                print(f"round {rnd} {label:10s} {line}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
